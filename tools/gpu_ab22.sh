set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t22.log 2>&1 || { tail -30 gpurun_out/t22.log; exit 1; }
tail -1 gpurun_out/t22.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu --no-rolling --no-stream > gpurun_out/b22.json 2> gpurun_out/b22.err || { tail -20 gpurun_out/b22.err; exit 1; }
tail -1 gpurun_out/b22.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['scan_kernel_ms']); print({k:(round(v['ms_per_step'],3), round(v['kernel_ms'],3), round(v['scan_kernel_ms'],3), round(v['projected_efficiency'],3)) for k,v in d['secondary']['shard_widths_1gpu'].items()})"
