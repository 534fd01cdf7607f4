set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_lda
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_lda/a -o pmc -- python3 $R/scripts/bench_lda.py --iters 1 --warmup 0 > $R/gpurun_out/pmc_lda/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d $R/gpurun_out/pmc_lda/b -o pmc -- python3 $R/scripts/bench_lda.py --iters 1 --warmup 0 > $R/gpurun_out/pmc_lda/b.log 2>&1
