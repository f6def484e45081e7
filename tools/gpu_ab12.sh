set -o pipefail
mkdir -p gpurun_out
for c in 5000 10000; do for pad in 0 64 1024 3072; do
timeout -k 10 300 python tools/ab_plan.py --ch $c --pad $pad --reps 2 "" > gpurun_out/ab_pad${c}_$pad.log 2>&1 || { tail -20 gpurun_out/ab_pad${c}_$pad.log; exit 1; }
echo "ch=$c pad=$pad $(grep median gpurun_out/ab_pad${c}_$pad.log)"
done; done
