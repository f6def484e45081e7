set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_ord; mkdir -p $OUT
for o in 0 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LFD_FR_ORDER=$o timeout -k 10 90 rocprofv3 --kernel-trace -f csv -d $OUT/o${o}_$c -o p --kernel-include-regex "fullrate_out_mb|block_functionals_mfma|fullrate_scan_seg" --pmc $c -- python3 tools/fr_one.py 2 > $OUT/o${o}_$c.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob, collections
for o in (0, 2):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = collections.defaultdict(list)
        for f in glob.glob(f"gpurun_out/pmc_ord/o{o}_{c}/*counter_collection.csv") + glob.glob(f"gpurun_out/pmc_ord/o{o}_{c}/*/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                v[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
        for k, xs in v.items():
            print(o, c, k, len(xs), sum(xs) / len(xs))
PY
