# lattice (composite) plans: parity at 3 kHz, then the low-pass / drop-in / stream GPU suites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -x -v -k lattice --timeout 200 --timeout-method thread > gpurun_out/r03k_lattice.log 2>&1 || { tail -40 gpurun_out/r03k_lattice.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r03k_lattice.log | tail -4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03k_suite.log 2>&1 || { tail -40 gpurun_out/r03k_suite.log; exit 1; }
tail -1 gpurun_out/r03k_suite.log
