set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
timeout -k 10 200 python tools/ab_roll_env.py 1 "LFD_ROLL_MINW=3" "LFD_ROLL_MINW=4" "LFD_ROLL_MINW=4 LFD_ROLL_PF=2" > gpurun_out/roll6.log 2>&1 || { tail -20 gpurun_out/roll6.log; exit 1; }
grep "S=1" gpurun_out/roll6.log
timeout -k 10 400 python tools/ab_plan.py --reps 5 "" "LFD_RUN_MINW=0 LFD_RUN_PF=2" > gpurun_out/ab_k1def.log 2>&1 || { tail -20 gpurun_out/ab_k1def.log; exit 1; }
grep median gpurun_out/ab_k1def.log
