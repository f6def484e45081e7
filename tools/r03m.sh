# FIR matrix-core kernel: conversions hoisted ahead of the MFMAs (A/B)
set -o pipefail
for e in "" "LFD_FIR_DIAG=64" "" "LFD_FIR_DIAG=64" "LFD_FIR_DIAG=72"; do
  echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py 2>&1 | grep "q= 10\|q=  5" || exit 1
done
