set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
for v in lds nolds; do
  if [ $v = nolds ]; then export LFD_K1_NOLDS=1; else unset LFD_K1_NOLDS; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --no-rolling > gpurun_out/bench_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["kernel_ms"],2), "ms", round(r["frac"],3), "scan", round(r["scan_kernel_ms"],2), "step", round(d["ms_per_step"],2))')"
done
