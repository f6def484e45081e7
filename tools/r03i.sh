# full-rate band-pass: big-block staging with every load in flight (default) vs 8-load groups
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_next_rows.py tests/test_gpu_lowpass.py -m gpu -x -q -k "full_rate or fullrate or band or sosfiltfilt" --timeout 120 --timeout-method thread > gpurun_out/r03i_tests.log 2>&1 || { tail -30 gpurun_out/r03i_tests.log; exit 1; }
tail -1 gpurun_out/r03i_tests.log
for e in "" "LFD_FR_STAGE_OLD=1" ""; do
  echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'rel', d['relrms_vs_oracle_3ch'])" || exit 1
done
