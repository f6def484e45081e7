set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_plan.py --reps 3 "" "LFD_RUN_MODE=5" "LFD_NO_RUNS=1 LFD_MF_MODE=3" > gpurun_out/ab_k1lds.log 2>&1 || { tail -20 gpurun_out/ab_k1lds.log; exit 1; }
grep median gpurun_out/ab_k1lds.log
