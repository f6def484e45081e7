# narrow-shard scan: kernel trace of the 1,250- and 2,500-channel plans, default (deep ring, trimmed constants) vs the 4 / 2 ring
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "scan or defer or lattice or shard or dist or stream or parity" > gpurun_out/r04m_pytest.log 2>&1 || { tail -30 gpurun_out/r04m_pytest.log; exit 1; }
tail -1 gpurun_out/r04m_pytest.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for e in "" "LFD_SCAN_DEEP=0"; do
for c in 1250 2500; do
  export LFDAS_LIB=$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so
  d=gpurun_out/r04m_trace_${c}_${e:-default}
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $d -o tr -- python3 tools/scan_one.py $c > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  echo "== $c ${e:-default}"
  python3 - "$d" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/tr_kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "chunk_scan" in n or "run_outputs" in n or "runs_mfma" in n:
        d[n[:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    v = sorted(v)[1:] if len(v) > 2 else v
    print(f"  {n:50s} {sum(v)/len(v):9.1f} us  (n={len(v)})")
PY
done
done
