# full-rate segmented scan: 8 channels x 64 segments per workgroup (2,000 ch) vs 16 x 32
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "full_rate or bandpass or env or fullrate" > gpurun_out/r04s_pytest.log 2>&1 || { tail -30 gpurun_out/r04s_pytest.log; exit 1; }
tail -1 gpurun_out/r04s_pytest.log
for e in "" "LFD_FR_SEG_CW=16" "" "LFD_FR_SEG_CW=16"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/r04s_fr.txt 2>&1 || { tail -20 gpurun_out/r04s_fr.txt; exit 1; }
  tail -1 gpurun_out/r04s_fr.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'pipe', round(d['pipeline_hbm_frac'],3), 'rel', d['relrms_vs_oracle_3ch'])"
done
