"""Every ctypes registration (ops._lib._SIGNATURES) declares as many arguments as the
exported C launcher in csrc/*.hip takes: a mismatch passes garbage to a kernel launch."""
import glob
import importlib
import os
import pkgutil
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_registered_argtypes_match_exports():
    import harp_amd.models
    import harp_amd.ops
    from harp_amd.ops import _lib

    for mod in pkgutil.iter_modules(harp_amd.ops.__path__):
        importlib.import_module("harp_amd.ops." + mod.name)
    for mod in pkgutil.iter_modules(harp_amd.models.__path__):
        importlib.import_module("harp_amd.models." + mod.name)
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "csrc", "*.hip")))
    bad = []
    for name, args in _lib._SIGNATURES.items():
        m = re.search(r"HARP_EXPORT\s+\w+\s+" + name + r"\(([^)]*)\)", src, re.S)
        assert m, f"{name} is registered but not exported by csrc/*.hip"
        n = len([a for a in m.group(1).split(",") if a.strip()])
        if n != len(args):
            bad.append((name, n, len(args)))
    assert not bad, bad
