set -o pipefail
mkdir -p gpurun_out
for c in 1250 2500 5000; do
timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 3 "" > gpurun_out/ab_ch$c.log 2>&1 || { tail -20 gpurun_out/ab_ch$c.log; exit 1; }
echo "ch=$c $(grep median gpurun_out/ab_ch$c.log)"
done
