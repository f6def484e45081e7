set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --reps 4 "" "LFD_RUN_SEPI=1" "LFD_RUN_SEPI=1 LFD_RUN_MINW=0 LFD_RUN_PF=2" > gpurun_out/r03d_cm_sepi.txt 2>&1 || { tail -20 gpurun_out/r03d_cm_sepi.txt; exit 1; }
cat gpurun_out/r03d_cm_sepi.txt
timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_RUN_SEPI=1" "LFD_RUN_SEPI=1 LFD_RUN_MINW=0 LFD_RUN_PF=2" > gpurun_out/r03d_cm_sepi_1250.txt 2>&1 || { tail -20 gpurun_out/r03d_cm_sepi_1250.txt; exit 1; }
cat gpurun_out/r03d_cm_sepi_1250.txt
timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 3 --replan "" "LFD_RUN_UNIT=8" "LFD_RUN_UNIT=16" "LFD_RUN_TAIL=0" "LFD_RUN_TAIL=4" > gpurun_out/r03d_narrow_units.txt 2>&1 || { tail -20 gpurun_out/r03d_narrow_units.txt; exit 1; }
cat gpurun_out/r03d_narrow_units.txt
