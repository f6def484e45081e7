# FIR matrix-core kernel: next-tile load placement / priority variants
set -o pipefail
mkdir -p gpurun_out
for e in "" "LFD_FIR_DIAG=4" "LFD_FIR_DIAG=8" "LFD_FIR_DIAG=12" ""; do
  echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py 2>&1 | grep -v amdgpu.ids | grep "q= 10" || exit 1
done
# time-major K1: 4x4x4 MFMA steps with the streaming epilogue
timeout -k 10 300 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_M4=1" > gpurun_out/r03h_tm_m4.txt 2>&1 || { tail -20 gpurun_out/r03h_tm_m4.txt; exit 1; }
cat gpurun_out/r03h_tm_m4.txt
