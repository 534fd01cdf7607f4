#!/bin/bash
# round-3: PMC of the LDA sparse sampler (1M docs x 1M vocab x 1000 topics, push-pull, 1 GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r8h
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "lda_cgs" --output-format csv -d /tmp/pa -o pmc -- python3 $R/scripts/bench_lda.py --iters 1 --warmup 0 --strategy push_pull > $O/a.log 2>&1
echo "a rc=$?"
find /tmp/pa -name "*counter_collection.csv" -exec cp {} $O/pmc_a.csv \;
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS FETCH_SIZE --kernel-include-regex "lda_cgs" --output-format csv -d /tmp/pb -o pmc -- python3 $R/scripts/bench_lda.py --iters 1 --warmup 0 --strategy push_pull > $O/b.log 2>&1
echo "b rc=$?"
find /tmp/pb -name "*counter_collection.csv" -exec cp {} $O/pmc_b.csv \;
ls -la $O
