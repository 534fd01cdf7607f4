#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7g
mkdir -p $O
timeout -k 10 120 python scripts/probe_gmm.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep '^{' $O/probe.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof7g -o run -- python $GRAFT_REPO_ROOT/scripts/probe_gmm.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find /tmp/prof7g -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r7g/kernel_stats.csv")))
for r in rows[:12]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PY
