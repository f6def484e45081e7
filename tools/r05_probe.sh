# round-5: K1 unit mapping — workgroup shares a channel group (LFD_K1_WGCG) vs
# channel-group-fastest waves; allocation-size probe; TLB counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
for c in 1250 2500 10000; do
  echo "== $c"; timeout -k 10 300 python tools/ab_plan.py --ch $c --reps 4 "" "LFD_K1_WGCG=1" 2>&1 | grep -E "K1|bit" || exit 1
done > $O/ab_wgcg.txt
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
run() { name=$1; shift; timeout -s KILL 150 rocprofv3 --kernel-trace -f csv -d $O/$name -o $name --kernel-include-regex "k_block_runs" --pmc $C -- python3 tools/ab_plan.py --reps 1 --steps 2 "$@" > $O/$name.log 2>&1; }
run wgcg1250 --ch 1250 "LFD_K1_WGCG=1" &&
run wgcg10k --ch 10000 "LFD_K1_WGCG=1" &&
unset LFDAS_LIB && timeout -k 10 400 python tools/r05_alloc_probe.py 1250 > $O/alloc.txt 2>&1
echo "exit $?"
