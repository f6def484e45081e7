# round-5: FIR 16-B staging in production: parity tests + timing
set -o pipefail
O=gpurun_out/r05f5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fir or decimate" > $O/pytest.log 2>&1
echo "pytest exit $?"; tail -2 $O/pytest.log
timeout -k 10 300 python tools/fir_ab.py 10 "" > $O/fir.txt 2>&1; grep -E "q=" $O/fir.txt
