# A/B liblfdas variants (build/variants/lib_<name>.so) on the bench's K1 time
set -e -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  LFDAS_LIB=$PWD/build/variants/lib_$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --no-rolling --no-stream > gpurun_out/bench_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["kernel_ms"],2), "ms", round(r["frac"],3), "scan", round(r["scan_kernel_ms"],2))')"
done
