#!/bin/bash
# LDA rotation at P = 1: one vs two word slices, and a kernel trace of the two-slice run
set -o pipefail
O=gpurun_out/round5_jj
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for S in 1 2; do
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --iters 5 --slices $S > $O/rot_s$S.log 2>&1 || { echo rot failed; tail $O/rot_s$S.log; exit 1; }
  tail -1 $O/rot_s$S.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot S=$S', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/bench_lda.py --docs 1000000 --iters 3 > $O/kt.log 2>&1 || { echo kt failed; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/round5_jj/kt/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us  {r["Name"][:110]}')
PY
