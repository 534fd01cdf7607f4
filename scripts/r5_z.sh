#!/bin/bash
# LDA sparse sampler at K = 10,000 (rotation, full size): kernel stats + two SQ counter passes
set -o pipefail
O=gpurun_out/round5_z
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
A="--docs 1000000 --topics 10000 --iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/bench_lda.py $A > $O/kt.log 2>&1 || { echo "kt failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcA -o run -- python3 scripts/bench_lda.py $A > $O/pmcA.log 2>&1 || { echo "pmcA failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM --kernel-include-regex "lda_cgs" --output-format csv -d $O/pmcB -o run -- python3 scripts/bench_lda.py $A > $O/pmcB.log 2>&1 || { echo "pmcB failed"; exit 1; }
for D in $O/kt $O/pmcA $O/pmcB; do
  python3 scripts/pmc_summary.py "$D" --match lda_cgs > /dev/null 2>&1
done
echo done
