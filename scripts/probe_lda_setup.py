"""Profile of the LDA push-pull setup (init_model) on P gloo ranks (GPU buffers with host
staging when a GPU is present): python scripts/probe_lda_setup.py P"""
import os, sys, time
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import torch, torch.distributed as dist
import torch.multiprocessing as mp

def run(rank, P, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    dist.init_process_group('gloo', rank=rank, world_size=P)
    from harp_amd.parallel.comm import Communicator
    from harp_amd.models.lda import LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader
    import cProfile, pstats
    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')
    comm = Communicator(None, dev)
    t0 = time.perf_counter()
    toks = synthetic_corpus(int(2e5), int(2e5), 1000, 100, seed=3, device=dev)
    t1 = time.perf_counter()
    cfg = LDAConfig(num_topics=1000, alpha=0.05, beta=0.01, iterations=2, local_server=False)
    m = LDAPushPullMapper(comm, cfg, int(2e5), int(2e5), toks)
    pr = cProfile.Profile(); pr.enable()
    m.init_model(KeyValReader([]))
    pr.disable()
    t2 = time.perf_counter()
    if rank == 0:
        print(f"corpus {t1-t0:.2f}s init {t2-t1:.2f}s", flush=True)
        pstats.Stats(pr).sort_stats('cumulative').print_stats(30)
    dist.destroy_process_group()

if __name__ == '__main__':
    P = int(sys.argv[1]); mp.spawn(run, args=(P, 29733), nprocs=P)
