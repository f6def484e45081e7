set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -1 gpurun_out/t14.log
for c in 1250 10000; do
timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 2 "" > gpurun_out/ab_sc$c.log 2>&1 || { tail -20 gpurun_out/ab_sc$c.log; exit 1; }
echo "ch=$c $(grep median gpurun_out/ab_sc$c.log)"
done
