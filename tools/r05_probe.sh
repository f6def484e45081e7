# round-5: rolling segment sums with coalesced tile loads A/B
set -o pipefail
O=gpurun_out/r05co
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 300 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEG_CO=1" "LFD_ROLL_SEG_CO=1 LFD_ROLL_SEG_DIAG=2" "LFD_ROLL_SEG_DIAG=2" > $O/roll250.txt 2>&1; grep -E "W=|bit" $O/roll250.txt
timeout -k 10 300 python tools/roll_ab.py 1000 200 "" "LFD_ROLL_SEG_CO=1" > $O/roll200.txt 2>&1; grep -E "W=|bit" $O/roll200.txt
LFD_ROLL_SEG_CO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -x -q --timeout 200 --timeout-method thread -k "rolling" > $O/pytest.log 2>&1
echo "pytest CO exit $?"; tail -2 $O/pytest.log
