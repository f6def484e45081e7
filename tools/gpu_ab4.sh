set -o pipefail
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/ubench_mfma64b tools/ubench_mfma64b.hip > gpurun_out/hipcc.log 2>&1 || { tail gpurun_out/hipcc.log; exit 1; }
timeout -k 5 60 /tmp/ubench_mfma64b > gpurun_out/ub64b.txt 2>&1; cat gpurun_out/ub64b.txt
timeout -k 10 300 python tools/ab_plan.py --reps 3 "" "LFD_RUN_PF=1" "LFD_RUN_MODE=4 LFD_RUN_NT=512" "LFD_NO_RUNS=1" "LFD_NO_RUNS=1 LFD_MF_MODE=3" "LFD_NO_RUNS=1 LFD_MF_MODE=1" > gpurun_out/ab_k1diag.log 2>&1 || { tail -20 gpurun_out/ab_k1diag.log; exit 1; }
cat gpurun_out/ab_k1diag.log
