#!/bin/bash
# MF-CCD at the full clueweb2 8-GPU share (2.0e9 ratings, rank 120) and a kernel-stats
# profile of LDA-CGS at the clueweb1 half share (K = 10,000) (profiles/r4_published), and
# LDA-CVB on the reference's dataset-1 when the box has the reference checkout (profiles/r4_ldacvb).
set -o pipefail
out=gpurun_out/r4pubp
mkdir -p $out
export TMPDIR=/tmp
(while sleep 45; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 420 python -u scripts/bench_ccd.py --users 9520495 --items 999933 --ratings 2e9 --rank 120 \
  --iters 2 > $out/ccd_r120_full_share.log 2>&1
rc=$?; echo "ccd rc=$rc" >> $out/status.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 scripts/bench_lda.py --docs 4.76e6 \
  --vocab 999933 --topics 10000 --len 392 --iters 2 --warmup 1 --strategy rotation > $out/lda_prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $out/status.txt
for db in $(find $out/prof -name "*.db"); do
  python3 scripts/rocpd_summary.py "$db" --top 25 --out $out/lda_kernels.json > $out/lda_kernel_summary.txt 2>&1
done
rm -rf $out/prof
[ $rc -eq 0 ] || exit $rc
# contrib LDA-CVB on the reference's own dataset-1 (744 docs, 89,907 terms), K = 50, 5 iterations
# a copy of the reference's datasets/tutorial/lda-cvb/sample-sparse-1k (git-ignored data/)
d=data/lda-cvb-1k
if [ -d $d ]; then
  for init in uniform random; do
    timeout -k 10 300 python -m harp_amd.cli ldacvb $d $d/sample-sparse-1k-metadata $out/cvb_$init 89907 50 744 1 5 1 1 \
      --init $init > $out/cvb_$init.log 2>&1 || exit $?
  done
fi
