# round-5: rolling units sized to 3 rounds (S = 250), S = 1 span A/B
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 400 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEG=32768" > $O/roll_ab250.txt 2>&1
echo "exit $?"; grep -E "W=|bit" $O/roll_ab250.txt
timeout -k 10 400 python tools/roll_ab.py 1000 1 "" "LFD_ROLL_SEG=65536" "LFD_ROLL_SEG=131072" "LFD_ROLL_SEG=300000" "LFD_ROLL_SEG=131072 LFD_ROLL_CAP=0" > $O/roll_ab1.txt 2>&1
echo "exit $?"; grep -E "W=|bit" $O/roll_ab1.txt
