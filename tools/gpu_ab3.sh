set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
timeout -k 10 200 python tools/ab_plan.py --off-ns 1900000 --reps 2 "" > gpurun_out/ab_off.log 2>&1 || { tail -20 gpurun_out/ab_off.log; exit 1; }
cat gpurun_out/ab_off.log
LFD_NO_HSKIP=1 timeout -k 10 200 python tools/ab_plan.py --off-ns 1900000 --reps 2 "" > gpurun_out/ab_off0.log 2>&1 || { tail -20 gpurun_out/ab_off0.log; exit 1; }
cat gpurun_out/ab_off0.log
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/ubench_mfma64b tools/ubench_mfma64b.hip > gpurun_out/hipcc.log 2>&1
timeout -k 5 60 /tmp/ubench_mfma64b > gpurun_out/ub64b.txt 2>&1; cat gpurun_out/ub64b.txt
