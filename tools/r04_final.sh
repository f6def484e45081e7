# round-4 end check, as the driver runs it: GPU suite, smoke, default bench line
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04z}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 700 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -1 gpurun_out/${tag}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=d['secondary']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3), 'cpu', d.get('cpu_baseline')); print({k: (round(v['roofline']['frac'],3), round(v.get('ms_per_step') or 0, 3)) for k, v in s.items() if isinstance(v, dict) and 'roofline' in v}); print(s.get('shard_widths_1gpu'))"
