# FIR matrix-core kernel: workgroup stagger A/B (about a third of a tile per step)
set -o pipefail
for e in "" "LFD_FIR_DIAG=16" "LFD_FIR_DIAG=48" "" "LFD_FIR_DIAG=16" "LFD_FIR_DIAG=48"; do
  echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py 2>&1 | grep "q= 10\|q=  5" || exit 1
done
