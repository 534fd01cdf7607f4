#!/bin/bash
# end-of-round state: GPU suite, smoke, the driver's bench command, and a kernel-stats profile of it
mkdir -p gpurun_out/r4e2
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r4e2/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e2/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4e2/bench.json 2> gpurun_out/r4e2/bench.err || exit $?
echo "bench ok"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e2/prof -o run -- python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4e2/prof_bench.json 2> gpurun_out/r4e2/prof.err
rc=$?; echo "prof rc=$rc"
# the trace database of a whole bench run is too large to bring back: keep its summary
for db in $(find gpurun_out/r4e2/prof -name "*.db"); do python3 scripts/rocpd_summary.py "$db" --top 40 --out gpurun_out/r4e2/kernels.json > gpurun_out/r4e2/kernel_summary.txt 2>&1; done
rm -rf gpurun_out/r4e2/prof
