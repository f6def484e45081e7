set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t35.log 2>&1 || { tail -30 gpurun_out/t35.log; exit 1; }
tail -1 gpurun_out/t35.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu --no-rolling --no-stream > gpurun_out/b35.json 2> gpurun_out/b35.err || { tail -20 gpurun_out/b35.err; exit 1; }
tail -1 gpurun_out/b35.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('head', round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['scan_kernel_ms'],3)); print({k:(round(v.get('ms_per_step',0),3), round(v['roofline']['kernel_ms'],3) if 'roofline' in v and 'kernel_ms' in v['roofline'] else None, round(v['roofline']['scan_kernel_ms'],3) if 'roofline' in v and 'scan_kernel_ms' in v['roofline'] else None) for k,v in d['secondary'].items() if 'roofline' in v})"
