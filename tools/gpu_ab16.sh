set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1 || { tail -30 gpurun_out/t16.log; exit 1; }
tail -1 gpurun_out/t16.log
for c in 1250 10000; do
timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 3 "" "LFD_SCAN_DEFER=0" > gpurun_out/ab_defer$c.log 2>&1 || { tail -20 gpurun_out/ab_defer$c.log; exit 1; }
echo "ch=$c"; grep -v amdgpu.ids gpurun_out/ab_defer$c.log
done
