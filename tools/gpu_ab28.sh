set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --reps 4 "" "LFD_RUN_BUF=1" "LFD_RUN_BUF=1 LFD_RUN_PF=2" > gpurun_out/ab_k1buf.log 2>&1 || { tail -20 gpurun_out/ab_k1buf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_k1buf.log
