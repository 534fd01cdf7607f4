#!/bin/bash
# full GPU suite, smoke, and the driver's bench command
mkdir -p gpurun_out/r4v
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4v/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4v/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4v/bench.json 2> gpurun_out/r4v/bench.err
echo "bench rc=$?"
