# round-5: rolling S = 1 (k_rolling_scan_tc) span / cap A/B
set -o pipefail
O=gpurun_out/r05z3
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 400 python tools/roll_ab.py 1000 1 "" "LFD_ROLL_SEG=16384" "LFD_ROLL_SEG=8192" "LFD_ROLL_CAP=4096" "LFD_ROLL_CAP=16384" "LFD_ROLL_MINW=4" > $O/roll_ab1.txt 2>&1
echo "exit $?"; grep -E "W=|bit" $O/roll_ab1.txt
