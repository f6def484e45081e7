set -o pipefail
mkdir -p gpurun_out
for c in 1250 5000 10000; do
timeout -k 10 300 python tools/ab_plan.py --replan --ch $c --reps 3 "" "LFD_RUN_UNIT=8" "LFD_RUN_UNIT=16" "LFD_RUN_UNIT=24" > gpurun_out/ab_unit$c.log 2>&1 || { tail -20 gpurun_out/ab_unit$c.log; exit 1; }
echo "ch=$c"; grep median gpurun_out/ab_unit$c.log
done
