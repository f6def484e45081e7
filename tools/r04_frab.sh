# full-rate output pass A/B (diag knobs): 16x16x4 vs 4x4x4_4b steps (LFD_FR_M4)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04e}
for e in "" "LFD_FR_M4=1" "" "LFD_FR_M4=1" "" "LFD_FR_M4=1"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/${tag}_fr.txt 2>&1 || { tail -20 gpurun_out/${tag}_fr.txt; exit 1; }
  tail -1 gpurun_out/${tag}_fr.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'rel', d['relrms_vs_oracle_3ch'])"
done
