set -o pipefail
out=gpurun_out/r6_owner_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for o in on off; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_$o -o run -- python3 scripts/bench_lda.py --topics 10000 --strategy push_pull --local-server off --iters 2 --owner-slots $o > $out/k10k_$o.log 2>&1 || { tail -5 $out/k10k_$o.log; exit 1; }
  python3 scripts/rocpd_summary.py $out/p_$o/run_results.db --out $out/k10k_kernels_$o.json --top 15 > /dev/null && rm -rf $out/p_$o
done
