#!/bin/bash
# eig crossover to rocSOLVER: tests + native-vs-rocSOLVER timings around the threshold
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eig_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for n in 1200 1536 1792; do
  echo "n=$n" >> gpurun_out/r4c/cross.log
  HARP_EIG_NATIVE_MAX=4096 timeout -k 10 120 python -u scripts/prof_eigh.py $n >> gpurun_out/r4c/cross.log 2>&1 || exit $?
done
echo done
