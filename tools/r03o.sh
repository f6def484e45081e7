# narrow shard scan: phase breakdown (LFD_SCAN_DIAG, separate processes) and deferred workgroup size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/probe_scan.py narrow > gpurun_out/r03o_scan_phases.txt 2>&1 || { tail -20 gpurun_out/r03o_scan_phases.txt; exit 1; }
timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_SCAN_DEFER_THREADS=64" "LFD_SCAN_DEFER_THREADS=128" >> gpurun_out/r03o_scan_phases.txt 2>&1 || { tail -20 gpurun_out/r03o_scan_phases.txt; exit 1; }
grep -v amdgpu gpurun_out/r03o_scan_phases.txt
