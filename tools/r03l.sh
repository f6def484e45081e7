# narrow shard (1,250 channels): K1 unit order A/B (LFD_K1_BAND)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_K1_BAND=1" "LFD_K1_BAND=4" "LFD_K1_BAND=16" > gpurun_out/r03l_band_1250.txt 2>&1 || { tail -20 gpurun_out/r03l_band_1250.txt; exit 1; }
grep -v amdgpu gpurun_out/r03l_band_1250.txt
