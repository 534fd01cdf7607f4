#!/bin/bash
# L2 behaviour of the fused reduction: TCC hits / misses per pass at n = 1000 and 1536
mkdir -p gpurun_out/r4k2
export TMPDIR=/tmp
for n in 1000 1536; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "sytrd_fused" -d gpurun_out/r4k2/pmc_tcc_$n -o run -- python3 scripts/probe_eig_phases.py $n > gpurun_out/r4k2/pmc_tcc_$n.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "sytrd_fused" -d gpurun_out/r4k2/pmc_sq -o run -- python3 scripts/probe_eig_phases.py 1000 > gpurun_out/r4k2/pmc_sq.log 2>&1
echo "rc=$?"
