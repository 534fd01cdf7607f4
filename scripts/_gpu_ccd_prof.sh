set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_ccd
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ccd -o ccd -- python3 $R/scripts/bench_ccd.py --iters 1 > $R/gpurun_out/prof_ccd/run.log 2>&1
