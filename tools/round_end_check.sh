# GPU tests, smoke and the default bench line (what the driver runs at round end)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || { tail -30 gpurun_out/rc_tests.log; exit 1; }
tail -1 gpurun_out/rc_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc_smoke.log 2>&1 || { tail -20 gpurun_out/rc_smoke.log; exit 1; }
tail -2 gpurun_out/rc_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err || { tail -20 gpurun_out/rc_bench.err; exit 1; }
tail -1 gpurun_out/rc_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3)); print('cpu', d['cpu_baseline'])"
