# the whole GPU suite (each step time-limited; stop on failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" > gpurun_out/r03_suite.log 2>&1 || { tail -40 gpurun_out/r03_suite.log; exit 1; }
tail -2 gpurun_out/r03_suite.log
