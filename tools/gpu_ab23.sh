set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 3 "" "LFD_K1_BAND=8" "LFD_K1_BAND=32" "LFD_K1_BAND=79" "LFD_RUN_PF=2 LFD_RUN_MINW=0" > gpurun_out/ab_band1250.log 2>&1 || { tail -20 gpurun_out/ab_band1250.log; exit 1; }
grep median gpurun_out/ab_band1250.log
