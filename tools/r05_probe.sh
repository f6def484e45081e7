# round-5: K1 translation misses / read latency by placement (narrow shard own
# allocation vs inside a wide one vs the full width)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n
mkdir -p $O
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
run() { name=$1; shift; timeout -s KILL 150 rocprofv3 --kernel-trace -f csv -d $O/$name -o $name --kernel-include-regex "k_block_runs" --pmc $C -- python3 tools/ab_plan.py --reps 1 --steps 2 "$@" "" > $O/$name.log 2>&1; }
run own --ch 1250 &&
run in10k --ch 1250 --alloc-ch 10000 &&
run mid10k --ch 1250 --alloc-ch 10000 --alloc-off 5000 &&
run full --ch 10000
echo "exit $?"
