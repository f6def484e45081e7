set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --tm --reps 4 "" "LFD_TM_M4=1" "LFD_TM_M4=1 LFD_TM_PF=1" > gpurun_out/ab_tm4.log 2>&1 || { tail -20 gpurun_out/ab_tm4.log; exit 1; }
cat gpurun_out/ab_tm4.log | grep -v amdgpu.ids
