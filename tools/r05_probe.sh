# round-5: pipelined executes (test + bench), narrow-shard K1 by allocation,
# fused scan phase stamps with parts removed, rolling S = 250 diag split
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -x -q --timeout 200 --timeout-method thread -k "pipeline or fused" > $O/pytest_pipe.log 2>&1
echo "pytest exit $?"; tail -3 $O/pytest_pipe.log
timeout -k 10 600 python bench.py --no-cpu --no-rolling --no-stream > $O/bench.json 2> $O/bench.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r05t/bench.json"))
print("headline", d["ms_per_step"], d["ms_per_step_serial"], d["roofline"]["kernel_ms"], d["roofline"]["scan_kernel_ms"])
for k, v in d["secondary"]["shard_widths_1gpu"].items():
    print(k, {a: round(b, 4) if isinstance(b, float) else b for a, b in v.items()})
for k, v in d["secondary"].items():
    if isinstance(v, dict) and "ms_per_step_serial" in v:
        print(k, round(v["ms_per_step"], 3), round(v["ms_per_step_serial"], 3))
PY
for m in torch pool pool64 vmm1 vmm4 vmmone big8 torch pool pool64 vmm1 vmm4 vmmone; do
  timeout -k 10 120 python tools/r05_alloc_first.py $m 1250 2>&1 | grep -E "K1|vmm|Error|error" || exit 1
done > $O/alloc.txt 2>&1
echo "exit $?"
cat $O/alloc.txt
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
for spec in "" "LFD_FU_DIAG=1" "LFD_FU_DIAG=2" "LFD_SCAN_DIAG=4"; do
  echo "== $spec"
  timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 3 --steps 5 "LFD_SCAN_DEFER=4 $spec" 2>&1 | grep -E "K1|k_scan" | tail -3 || exit 1
  timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 1 --steps 2 "LFD_SCAN_DEFER=4 LFD_FU_TIMES=1 $spec" 2>&1 | grep -E "k_scan" | tail -5 || exit 1
done > $O/fu_parts.txt 2>&1
echo "exit $?"
cat $O/fu_parts.txt
timeout -k 10 300 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEG_DIAG=1" "LFD_ROLL_SEG_DIAG=2" > $O/roll_parts.txt 2>&1
echo "exit $?"
cat $O/roll_parts.txt
