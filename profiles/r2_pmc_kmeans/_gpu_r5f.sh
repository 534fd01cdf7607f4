#!/bin/bash
# PMC of the spill-fixed K-means assign (variant 14, KS=7): MFMA busy, VALU/MFMA mix, LDS
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5f
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/r5f/a -o pmc -- python3 $R/scripts/kmeans_one.py --variant 14 --reps 2 > $R/gpurun_out/r5f/a.log 2>&1 || { tail -20 $R/gpurun_out/r5f/a.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $R/gpurun_out/r5f/b -o pmc -- python3 $R/scripts/kmeans_one.py --variant 14 --reps 2 > $R/gpurun_out/r5f/b.log 2>&1 || { tail -20 $R/gpurun_out/r5f/b.log; exit 1; }
cd $R && python scripts/pmc_summary.py gpurun_out/r5f/a --match kmeans_assign && python scripts/pmc_summary.py gpurun_out/r5f/b --match kmeans_assign
