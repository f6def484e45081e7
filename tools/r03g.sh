# FIR matrix-core kernel: timing breakdown (staging only / MFMA only) and strip length
set -o pipefail
mkdir -p gpurun_out
for e in "" "LFD_FIR_DIAG=1" "LFD_FIR_DIAG=2" "LFD_FIR_STRIP=2" "LFD_FIR_STRIP=32"; do
  echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
