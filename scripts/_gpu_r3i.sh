#!/bin/bash
# round-2 validation after the ring-stride rotation change: GPU suite + 1-GPU bench
set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3i/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3i/gpu_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r3i/bench.log 2>&1 || { tail -20 gpurun_out/r3i/bench.log; exit 1; }
grep '^{' gpurun_out/r3i/bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read().splitlines()[-1]); print(r['value'], r['phase_ms_per_iter'], r['sgd'].get('updates_per_sec'), r['sgd'].get('s_per_epoch'))"
