# round-5: cfg3 full-width scan variants (in-chain default vs deferred / segmented / fused)
set -o pipefail
O=gpurun_out/r05sc
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 600 python tools/ab_plan.py --ch 10000 --reps 3 --steps 5 "" "LFD_SCAN_DEFER=2" "LFD_SCAN_DEFER=3" "LFD_SCAN_DEFER=4" > $O/scan10k.txt 2>&1
echo "exit $?"; grep -E "K1|bit" $O/scan10k.txt
