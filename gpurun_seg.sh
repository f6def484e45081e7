set -o pipefail
mkdir -p gpurun_out
for c in 1250 2500; do
  timeout -k 10 240 python tools/ab_plan.py --ch $c --reps 4 "" "LFD_SCAN_DEFER=3" > gpurun_out/r04x_ab_$c.txt 2>&1 || { tail -20 gpurun_out/r04x_ab_$c.txt; exit 1; }
  grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04x_ab_$c.txt | tail -3
done
timeout -k 10 300 python tools/ab_plan.py --fs 1000 --dt 10 --P 120 --B 6 --ch 2000 --reps 3 "" "LFD_SCAN_DEFER=3" > gpurun_out/r04x_ab_dt10_2000.txt 2>&1 || { tail -20 gpurun_out/r04x_ab_dt10_2000.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04x_ab_dt10_2000.txt | tail -3
