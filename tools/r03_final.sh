# final tree check: GPU suite, smoke, default bench line (what the driver runs at round end)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03d_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03d_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || { tail -20 gpurun_out/r03d_smoke.log; exit 1; }
tail -1 gpurun_out/r03d_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || { tail -20 gpurun_out/r03d_bench.err; exit 1; }
tail -1 gpurun_out/r03d_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; s=d['secondary']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3), 'dt10', round(s['lowpass_1khz_dt10']['roofline']['scan_kernel_ms'],3), 'lattice', round(s['lowpass_3khz_lattice']['ms_per_step'],2))"
timeout -k 10 300 python bench.py --gpus 2 --one-device --steps 2 --warmup 1 --no-cpu --no-rolling --no-extra --no-stream > gpurun_out/r03d_rehearsal.json 2> gpurun_out/r03d_rehearsal.err || { tail -20 gpurun_out/r03d_rehearsal.err; exit 1; }
tail -1 gpurun_out/r03d_rehearsal.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal n_gpus', d['n_gpus'], 'ranks_seen', d['ranks_seen'], 'scaling', d['scaling'], list(d['secondary']))"
