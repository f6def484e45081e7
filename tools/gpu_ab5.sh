set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 400 python tools/ab_plan.py --reps 5 "" "LFD_RUN_MINW=4 LFD_RUN_PF=1" "LFD_RUN_M4=1 LFD_RUN_PF=1" "LFD_RUN_M4=1 LFD_RUN_MINW=4 LFD_RUN_PF=1" "LFD_RUN_PF=1" > gpurun_out/ab_k1m4_$i.log 2>&1 || { tail -20 gpurun_out/ab_k1m4_$i.log; exit 1; }
grep median gpurun_out/ab_k1m4_$i.log
done
