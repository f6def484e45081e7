# narrow shard: deferred scan ring depth / batched stores (A/B, outputs compared bit for bit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_SCAN_DEEP=1" "LFD_SCAN_DEEP=2" "LFD_SCAN_DEEP=3" > gpurun_out/r03n_scan_deep.txt 2>&1 || { tail -20 gpurun_out/r03n_scan_deep.txt; exit 1; }
timeout -k 10 400 python tools/ab_plan.py --fs 1000 --dt 10 --P 120 --B 6 --ch 2000 --reps 3 "" "LFD_SCAN_DEEP=1" "LFD_SCAN_DEEP=2" >> gpurun_out/r03n_scan_deep.txt 2>&1 || { tail -20 gpurun_out/r03n_scan_deep.txt; exit 1; }
grep -v amdgpu gpurun_out/r03n_scan_deep.txt
