set -o pipefail
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_mfma64b tools/ubench_mfma64b.hip 2>/dev/null
timeout -k 5 60 /tmp/ubench_mfma64b > gpurun_out/ub64b.txt 2>&1; cat gpurun_out/ub64b.txt
timeout -k 10 300 python tools/ab_plan.py --tm --reps 4 "LFD_TM_X2=1" "LFD_TM_X2=0" > gpurun_out/ab_tm.log 2>&1 || { tail -20 gpurun_out/ab_tm.log; exit 1; }
cat gpurun_out/ab_tm.log
