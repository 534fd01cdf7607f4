#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7b
timeout -k 10 300 python scripts/probe_sgd_launch.py > gpurun_out/r7b/probe.log 2>&1; rc=$?
cat gpurun_out/r7b/probe.log | grep '^{'; exit $rc
