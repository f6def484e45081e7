# FIR decimation on the matrix cores: parity tests, then timing vs the VALU kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_next_rows.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 || { tail -40 gpurun_out/r03f_tests.log; exit 1; }
tail -3 gpurun_out/r03f_tests.log
timeout -k 10 200 python tools/fir_bench.py > gpurun_out/r03f_fir.txt 2>&1 || { tail -20 gpurun_out/r03f_fir.txt; exit 1; }
LFD_FIR_VALU=1 timeout -k 10 200 python tools/fir_bench.py >> gpurun_out/r03f_fir.txt 2>&1 || { tail -20 gpurun_out/r03f_fir.txt; exit 1; }
cat gpurun_out/r03f_fir.txt
