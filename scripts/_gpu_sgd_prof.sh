set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/sgd_prof
mkdir -p $O
run() {  # name, rocprof args..., -- , bench args
  local n=$1; shift
  timeout -k 10 300 "$@" > $O/$n.log 2>&1 || return 1
  python3 $R/scripts/pmc_summary.py $O/$n --match mf_ || return 1
}
run kt rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/scripts/bench_sgd.py --layout xcd --epochs 2 --warmup 1 || exit 1
run ktflat rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktflat -o run -- python3 $R/scripts/bench_sgd.py --layout flat --epochs 2 --warmup 1 || exit 1
run pmc1 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc1 -o run -- python3 $R/scripts/bench_sgd.py --layout xcd --epochs 1 --warmup 0 || exit 1
run pmc2 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- python3 $R/scripts/bench_sgd.py --layout xcd --epochs 1 --warmup 0 || exit 1
run pmc3 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc3 -o run -- python3 $R/scripts/bench_sgd.py --layout flat --epochs 1 --warmup 0 || exit 1
du -sh $O
