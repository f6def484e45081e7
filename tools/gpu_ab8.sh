set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_next_rows.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1 || { tail -30 gpurun_out/t8.log; exit 1; }
tail -1 gpurun_out/t8.log
timeout -k 10 200 python tools/fir_bench.py > gpurun_out/fir.log 2>&1 || { tail -20 gpurun_out/fir.log; exit 1; }
cat gpurun_out/fir.log
