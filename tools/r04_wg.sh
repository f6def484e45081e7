# workgroup-size A/B (same registers / occupancy, smaller groups): time-major K1 and channel-major K1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --tm --reps 5 "" "LFD_TM_W=2" "LFD_TM_W=21" > gpurun_out/r04q_ab_tm_w.txt 2>&1 || { tail -20 gpurun_out/r04q_ab_tm_w.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04q_ab_tm_w.txt | tail -5
timeout -k 10 400 python tools/ab_plan.py --reps 5 "" "LFD_K1_WG=256" "LFD_K1_WG=2561" > gpurun_out/r04q_ab_cm_wg.txt 2>&1 || { tail -20 gpurun_out/r04q_ab_cm_wg.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04q_ab_cm_wg.txt | tail -5
timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 5 "" "LFD_K1_WG=256" > gpurun_out/r04q_ab_cm_wg_1250.txt 2>&1 || { tail -20 gpurun_out/r04q_ab_cm_wg_1250.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04q_ab_cm_wg_1250.txt | tail -3
