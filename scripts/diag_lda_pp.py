"""Diagnostic: LDA push-pull final log-likelihood by comm layout (dense / sparse / local)
and seed, plus an exact count-rebuild check of the server table against (word, z)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from harp_amd.models.lda import LDAConfig, LDAPushPullMapper, synthetic_corpus  # noqa: E402
from harp_amd.parallel.comm import Communicator  # noqa: E402
from harp_amd.runtime.mapper import KeyValReader  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    toks = synthetic_corpus(3000, 4000, 20, 50, seed=2)
    n = toks[0].numel()
    rows = []
    for mode, ls in (("off", False), ("on", False), ("off", True)):
        for seed in range(4):
            for rep in range(2 if seed == 0 else 1):
                cfg = LDAConfig(num_topics=64, alpha=0.1, beta=0.01, iterations=12, print_interval=6, block_words=512,
                                sparse_comm=mode, local_server=ls, seed=seed)
                m = LDAPushPullMapper(Communicator(device=dev), cfg, 3000, 4000, toks)
                t0 = time.time()
                m.run(KeyValReader([]))
                ll = [v for _, v in m.result["loglik"]]
                ok = m.check_counts() if hasattr(m, "check_counts") else None
                rows.append((m.comm_mode, seed, rep, ll[0] / n, ll[-1] / n, ok, time.time() - t0))
                print(rows[-1], flush=True)


if __name__ == "__main__":
    main()
