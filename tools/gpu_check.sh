# GPU parity tests then a short bench (each step time-limited; stop on failure)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-rolling "$@" > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("K1", round(r["kernel_ms"],2), "ms frac", round(r["frac"],3), "scan", round(r["scan_kernel_ms"],2), "step", round(d["ms_per_step"],2), "value %.3e" % d["value"])'
