# A/B an environment switch on the bench's K1 time: ab_env.sh "NAME=VAL" ...
set -e -o pipefail
mkdir -p gpurun_out
for kv in "$@"; do
  env $kv timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --no-rolling > gpurun_out/bench_ab.log 2>&1
  echo "$kv $(tail -1 gpurun_out/bench_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["kernel_ms"],2), "ms", round(r["frac"],3), "scan", round(r["scan_kernel_ms"],2), "step", round(d["ms_per_step"],2))')"
done
