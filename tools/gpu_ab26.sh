set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_BUF=1" "LFD_TM_BUF=1 LFD_TM_PF=1" > gpurun_out/ab_tmbuf.log 2>&1 || { tail -20 gpurun_out/ab_tmbuf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_tmbuf.log
