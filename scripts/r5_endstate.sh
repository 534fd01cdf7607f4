#!/bin/bash
# round-5 end state: kernel trace + stats of the default bench (short), then the bench itself
set -o pipefail
O=gpurun_out/round5_end
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 2 > $O/kt_bench.json 2> $O/kt_bench.err || { echo "kt failed"; tail -20 $O/kt_bench.err; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/round5_end/kt/run_kernel_stats.csv")))
with open("gpurun_out/round5_end/kernel_summary.txt", "w") as f:
    for r in rows[:40]:
        f.write(f'{float(r["TotalDurationNs"])/1e6:10.3f} ms  {int(r["Calls"]):7d} calls  {float(r["AverageNs"])/1e3:10.2f} us avg  {r["Name"][:150]}\n')
print(open("gpurun_out/round5_end/kernel_summary.txt").read()[:3000])
PY
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cut -c 1-300 $O/bench.json
