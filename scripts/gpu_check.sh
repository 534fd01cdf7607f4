#!/bin/bash
# One GPU session: build, GPU tests, 1-GPU bench. Stops at the first crash/timeout
# (exit codes 124/134/137/139 or negative) so nothing else runs on a faulted GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if fatal $rc; then echo "stopping after fatal pytest exit"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
