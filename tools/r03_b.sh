# full GPU suite, then the time-major K1 floor at higher occupancy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || { tail -40 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_MODE=3" "LFD_TM_MODE=3 LFD_TM_DIAG_LDS=1" "LFD_TM_MODE=3 LFD_TM_DIAG_LDS=1 LFD_TM_PF=2" "LFD_TM_MODE=4 LFD_TM_DIAG_LDS=1" > gpurun_out/r03b_tm_diag.txt 2>&1 || { tail -20 gpurun_out/r03b_tm_diag.txt; exit 1; }
tail -5 gpurun_out/r03b_tm_diag.txt
