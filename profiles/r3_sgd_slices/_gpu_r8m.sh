#!/bin/bash
# round-3: PMC after the LDA doc-list prefetch (same counters as r8h) and of the MF-SGD XCD
# kernel at one slice per rank (L2 hit rate, wave waits)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r8m
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "lda_cgs" --output-format csv -d /tmp/pa -o pmc -- python3 $R/scripts/bench_lda.py --iters 1 --warmup 0 --strategy push_pull > $O/lda.log 2>&1
echo "lda rc=$?"
find /tmp/pa -name "*counter_collection.csv" -exec cp {} $O/pmc_lda.csv \;
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex "mf_sgd" --output-format csv -d /tmp/pb -o pmc -- python3 $R/scripts/bench_sgd.py --epochs 1 --warmup 0 > $O/sgd.log 2>&1
echo "sgd rc=$?"
find /tmp/pb -name "*counter_collection.csv" -exec cp {} $O/pmc_sgd.csv \;
ls -la $O
