# round-5: K1 timing modes on cfg3 (what a producer/consumer split could win)
set -o pipefail
O=gpurun_out/r05k1
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 600 python tools/ab_plan.py --ch 10000 --reps 3 --steps 5 "" "LFD_RUN_MODE=4" "LFD_RUN_MODE=1" > $O/modes.txt 2>&1
echo "exit $?"; grep -E "K1|bit" $O/modes.txt
