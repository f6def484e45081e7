set -o pipefail
mkdir -p gpurun_out
for c in 160 320 640 1250; do
timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 2 "" > gpurun_out/ab_small$c.log 2>&1 || { tail -20 gpurun_out/ab_small$c.log; exit 1; }
echo "ch=$c $(grep median gpurun_out/ab_small$c.log)"
done
