set -o pipefail
mkdir -p gpurun_out
for d in 0 8 2 4 1 15; do
LFD_SCAN_DIAG=$d timeout -k 10 200 python tools/ab_plan.py --ch 1250 --reps 2 "" > gpurun_out/ab_scan1250_$d.log 2>&1 || { tail -20 gpurun_out/ab_scan1250_$d.log; exit 1; }
echo "diag=$d $(grep median gpurun_out/ab_scan1250_$d.log)"
done
