set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_syrk
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_syrk/a -o pmc -- python3 $R/scripts/bench_pca.py --n 2e7 --steps 1 --warmup 0 > $R/gpurun_out/pmc_syrk/a.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_syrk/c -o pmc -- python3 $R/scripts/bench_pca.py --n 2e7 --steps 1 --warmup 0 > $R/gpurun_out/pmc_syrk/c.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_syrk/b -o pmc -- python3 $R/scripts/bench_pca.py --n 2e7 --steps 1 --warmup 0 > $R/gpurun_out/pmc_syrk/b.log 2>&1
