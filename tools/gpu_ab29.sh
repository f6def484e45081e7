set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rolling" > gpurun_out/t29.log 2>&1 || { tail -30 gpurun_out/t29.log; exit 1; }
tail -1 gpurun_out/t29.log
timeout -k 10 200 python tools/ab_roll_env.py 1 "LFD_ROLL_DPP=1" "LFD_ROLL_DPP=0" > gpurun_out/roll29.log 2>&1 || { tail -20 gpurun_out/roll29.log; exit 1; }
grep -v amdgpu.ids gpurun_out/roll29.log
timeout -k 10 200 python tools/ab_roll_env.py 250 "LFD_ROLL_DPP=1" "LFD_ROLL_DPP=0" > gpurun_out/roll29b.log 2>&1 || { tail -20 gpurun_out/roll29b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/roll29b.log
