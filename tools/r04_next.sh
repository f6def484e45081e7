# round 4: GPU suite, full-rate A/B, the N = 2 one-device rehearsal (strong
# scaling headline + sharded cfg5 stream) and the default bench line (no CPU legs)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.log
for e in "" "LFD_FULLRATE_BIGBLOCK=1"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/${tag}_fr_${e:-default}.txt 2>&1 || { tail -20 gpurun_out/${tag}_fr_${e:-default}.txt; exit 1; }
  tail -1 gpurun_out/${tag}_fr_${e:-default}.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'pipe', round(d['pipeline_hbm_frac'],3), 'rel', d['relrms_vs_oracle_3ch'])"
done
timeout -k 10 400 python bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --no-rolling --no-extra > gpurun_out/${tag}_rehearsal.json 2> gpurun_out/${tag}_rehearsal.err || { tail -20 gpurun_out/${tag}_rehearsal.err; exit 1; }
tail -1 gpurun_out/${tag}_rehearsal.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['secondary']; print('rehearsal', d['n_gpus'], d['ranks_seen'], d['scaling'], d['config']['channels'], d['config']['channels_rank0'], {k: (v.get('value'), v.get('check', {}).get('pass')) for k, v in s.items() if isinstance(v, dict)})"
timeout -k 10 500 python bench.py --no-cpu > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
tail -1 gpurun_out/${tag}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=d['secondary']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3)); print({k: round(v['roofline']['frac'],3) for k, v in s.items() if isinstance(v, dict) and 'roofline' in v}); print(s.get('shard_widths_1gpu'))"
