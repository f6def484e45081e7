set -o pipefail
mkdir -p gpurun_out
for c in 2500 5000; do
timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 3 "" "LFD_SCAN_DEFER=0" > gpurun_out/ab_defer$c.log 2>&1 || { tail -20 gpurun_out/ab_defer$c.log; exit 1; }
echo "ch=$c"; grep median gpurun_out/ab_defer$c.log
done
