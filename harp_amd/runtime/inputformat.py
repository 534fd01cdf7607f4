"""Input splitting (Harp ``MultiFileInputFormat`` / ``SingleFileInputFormat``).

Reference: harp-daal-interface fileformat/MultiFileInputFormat.java:46-125 — the file
list is shuffled, each of the M mappers gets floor(F/M) files and the remainder is
spread one per mapper; one split = a list of paths; MultiFileRecordReader yields
(key, path). SingleFileInputFormat gives each file its own split.
"""
from __future__ import annotations

import glob
import os
import random
from typing import List, Sequence


def list_input_files(path_or_glob: str | Sequence[str]) -> List[str]:
    if isinstance(path_or_glob, (list, tuple)):
        out: List[str] = []
        for p in path_or_glob:
            out += list_input_files(p)
        return out
    p = str(path_or_glob)
    if os.path.isdir(p):
        return sorted(os.path.join(p, f) for f in os.listdir(p) if not f.startswith((".", "_")))
    return sorted(glob.glob(p)) or ([p] if os.path.exists(p) else [])


def multi_file_splits(files: Sequence[str], num_mappers: int, seed: int | None = None) -> List[List[str]]:
    files = list(files)
    rng = random.Random(seed)
    rng.shuffle(files)
    per, rem = divmod(len(files), num_mappers)
    splits: List[List[str]] = []
    pos = 0
    for m in range(num_mappers):
        n = per + (1 if m < rem else 0)
        splits.append(files[pos:pos + n])
        pos += n
    return splits


def single_file_splits(files: Sequence[str]) -> List[List[str]]:
    return [[f] for f in files]
