# round-5: fused scan phase stamps (diag LFD_FU_TIMES)
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
for c in 1250 10000; do
  echo "== $c"; timeout -k 10 300 python tools/ab_plan.py --ch $c --reps 1 --steps 2 "LFD_SCAN_DEFER=4 LFD_FU_TIMES=1" 2>&1 | grep -E "K1|k_scan" || exit 1
done > $O/fu_times.txt
echo "exit $?"
