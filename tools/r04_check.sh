# round-4 tree check: GPU suite, smoke, the N = 2 one-device rehearsal
# (strong-scaling headline + the sharded cfg5 stream) and a default bench line
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --no-rolling --no-extra > gpurun_out/${tag}_rehearsal.json 2> gpurun_out/${tag}_rehearsal.err || { tail -20 gpurun_out/${tag}_rehearsal.err; exit 1; }
tail -1 gpurun_out/${tag}_rehearsal.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['secondary']; print('rehearsal', d['n_gpus'], d['ranks_seen'], d['scaling'], d['config']['channels'], d['config']['channels_rank0'], {k: (v.get('value'), v.get('check', {}).get('pass')) for k, v in s.items() if isinstance(v, dict)})"
timeout -k 10 500 python bench.py --no-cpu > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -1 gpurun_out/${tag}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=d['secondary']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3)); print({k: round(v['roofline']['frac'],3) for k, v in s.items() if isinstance(v, dict) and 'roofline' in v}); print(s.get('shard_widths_1gpu'))"
