set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
for v in 14; do
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc/v$v -o pmc -- python3 $R/scripts/kmeans_one.py --variant $v --reps 2 > $R/gpurun_out/pmc/v$v.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $R/gpurun_out/pmc/v${v}b -o pmc -- python3 $R/scripts/kmeans_one.py --variant $v --reps 2 > $R/gpurun_out/pmc/v${v}b.log 2>&1 || exit 1
done
