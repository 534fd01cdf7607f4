# One-wave D&C merge kernel (csrc/tridiag_dc.hip dc_wave_merge_kernel): eig tests, eigh timings
# for merge-size thresholds 64 .. 8 and without it (HARP_DC_WAVE_MERGE=0), per-level kernel trace (scripts/dc_level_summary.py).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_dc_wave.sh gpurun_out/r6_dcwave'
set -o pipefail
out=${1:-gpurun_out/r6_dcwave}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_eig_gpu.py tests/test_coop_contention_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
for m in 64 32 16 8 0; do HARP_DC_WAVE_MERGE=$m timeout -k 10 200 python scripts/bench_eigh.py 1000 > "$out/bench_$m.json" 2> "$out/bench_$m.err" || { tail -5 "$out/bench_$m.err"; exit 1; }; done
for f in 64 32 16 8 0; do python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[1], r['dc_ms'], r['eigh_ll_ms'], r['dc_wave_phase_cycles'], r['dc_wave_secular_max_iters'])" "$out/bench_$f.json"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/prof" -o run -- python3 scripts/bench_eigh.py 1000 > "$out/prof.log" 2>&1 || { tail -5 "$out/prof.log"; exit 1; }
python scripts/dc_level_summary.py "$out/prof/run_results.db" > "$out/dc_levels.txt" && cat "$out/dc_levels.txt"
python scripts/eigh_timeline.py "$out/prof/run_results.db" > "$out/eigh_timeline.txt" && tail -50 "$out/eigh_timeline.txt"
rm -rf "$out/prof"
