set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_NT=768 LFD_TM_PF=1" "LFD_TM_NT=768 LFD_TM_PF=1 LFD_TM_X2=0" > gpurun_out/ab_tm768.log 2>&1 || { tail -20 gpurun_out/ab_tm768.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_tm768.log
