#!/bin/bash
# round-3: MF-SGD flow kernel (claim-then-wait) A/B at the 8-GPU share incl. fewer blocks,
# S=1 vs S=2 slices; SYRK PMC (clock, MFMA busy) for the full kernel vs MFMA+LDS only
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6f
mkdir -p $O
for cfg in "0 128 16" "1 128 16" "1 32 16" "1 64 16" "0 128 8" "1 128 8"; do
  set -- $cfg
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 12560063 --slices $3 --epochs 10 --variant $1 --blocks-per-xcd $2 --chunk 0 > $O/sgd_v$1_b$2_s$3.log 2>&1 || { echo "sgd $cfg failed"; tail -5 $O/sgd_v$1_b$2_s$3.log; exit 1; }
  echo "sgd v=$1 bpx=$2 slices=$3: $(grep '^{' $O/sgd_v$1_b$2_s$3.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["value"]/1e9,2), "e9/s rmse", round(r["train_rmse"],5))')"
done
timeout -k 10 200 python -u -m pytest tests/test_sgd_flow_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest_flow.log 2>&1
rc=$?; echo "flow pytest rc=$rc"; tail -2 $O/pytest_flow.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
for m in 0 1; do
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA --kernel-trace --output-format csv -d /tmp/pmc_m$m -o pmc -- python3 $R/scripts/syrk_diag.py --modes $m --reps 1 > $O/pmc_m$m.log 2>&1 || { echo "pmc m$m failed"; tail -5 $O/pmc_m$m.log; exit 1; }
  for f in $(find /tmp/pmc_m$m -name "*.csv"); do cp $f $O/pmc_m${m}_$(basename $f); done
done
ls $O
