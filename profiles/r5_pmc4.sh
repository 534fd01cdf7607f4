#!/bin/bash
# LDA dense sampler after the round-5 VALU / chunk-start trims at full size and at the 8-GPU share: SQ counters
set -o pipefail
O=gpurun_out/round5_pmc4
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for C in "share:--docs 125000 --strategy push_pull --local-server off --iters 3" "full:--docs 1000000 --strategy push_pull --local-server off --iters 2"; do
  N=${C%%:*}; A=${C#*:}
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcA_$N -o run -- python3 scripts/bench_lda.py $A > $O/pmcA_$N.log 2>&1 || { echo "pmcA $N failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcB_$N -o run -- python3 scripts/bench_lda.py $A > $O/pmcB_$N.log 2>&1 || { echo "pmcB $N failed"; exit 1; }
done
for D in $O/pmcA_* $O/pmcB_*; do
  python3 scripts/pmc_summary.py "$D" --match lda_cgs > /dev/null 2>&1
done
echo done
