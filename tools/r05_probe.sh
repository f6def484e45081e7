# round-5: narrow-shard K1 by allocation (fresh process each), then the fused scan
# phase stamps with parts removed, then the rolling S = 250 diag split
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
for m in torch pool pool64 vmm1 vmm4 vmmone big8 torch pool pool64 vmm1 vmm4 vmmone; do
  timeout -k 10 120 python tools/r05_alloc_first.py $m 1250 2>&1 | grep -E "K1|vmm|Error|error" || exit 1
done > $O/alloc.txt 2>&1
echo "exit $?"
cat $O/alloc.txt
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
for spec in "" "LFD_FU_DIAG=1" "LFD_FU_DIAG=2" "LFD_FU_DIAG=3" "LFD_SCAN_DIAG=4" "LFD_SCAN_DIAG=5"; do
  echo "== $spec"
  timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 3 --steps 5 "LFD_SCAN_DEFER=4 $spec" 2>&1 | grep -E "K1|k_scan" | tail -8 || exit 1
  timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 1 --steps 2 "LFD_SCAN_DEFER=4 LFD_FU_TIMES=1 $spec" 2>&1 | grep -E "k_scan" | tail -5 || exit 1
done > $O/fu_parts.txt 2>&1
echo "exit $?"
cat $O/fu_parts.txt
echo "== rolling"
timeout -k 10 300 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEG_DIAG=1" "LFD_ROLL_SEG_DIAG=2" > $O/roll_parts.txt 2>&1
echo "exit $?"
cat $O/roll_parts.txt
