#!/bin/bash
# LDA sampler kernels, where does the time go: full size (sparse doc-span sampler, push-pull
# with pull / push running) and the 8-GPU rank share (dense fused-rows sampler): kernel stats
# and two SQ counter passes each
set -o pipefail
O=gpurun_out/round5_lda_pmc
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
FULL="--docs 1e6 --strategy push_pull --local-server off --iters 3"
SHARE="--docs 125000 --strategy push_pull --local-server off --iters 5"




for C in "share:$SHARE" "full:$FULL"; do
  N=${C%%:*}; A=${C#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$N -o run -- python3 scripts/bench_lda.py $A > $O/kt_$N.log 2>&1 || { echo "kt $N failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcA_$N -o run -- python3 scripts/bench_lda.py $A > $O/pmcA_$N.log 2>&1 || { echo "pmcA $N failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_WR --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcB_$N -o run -- python3 scripts/bench_lda.py $A > $O/pmcB_$N.log 2>&1 || { echo "pmcB $N failed"; exit 1; }
done
for D in $O/kt_* $O/pmcA_* $O/pmcB_*; do
  [ -d "$D" ] && python3 scripts/pmc_summary.py "$D" --match lda_cgs > /dev/null 2>&1
done
echo done
