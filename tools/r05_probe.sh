# round-5: non-temporal output stores A/B (FIR, rolling S = 1, full-rate)
set -o pipefail
O=gpurun_out/r05nt
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
timeout -k 10 300 python tools/fir_ab.py 10 "" "LFD_NT_STORES=1" "" "LFD_NT_STORES=1" > $O/fir.txt 2>&1; grep -E "q=|bit" $O/fir.txt
timeout -k 10 300 python tools/roll_ab.py 1000 1 "" "LFD_NT_STORES=1" > $O/roll.txt 2>&1; grep -E "W=|bit" $O/roll.txt
for v in 0 1 0 1; do
  LFD_NT_STORES=$v timeout -k 10 200 python tools/fr_bench.py 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('NT=$v', round(d['ms'],3), {k.split(' ')[0]: round(v,3) for k,v in d['kernels_ms'].items()}, d['relrms_vs_oracle_3ch'])" || exit 1
done
