set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -1 gpurun_out/t18.log
for c in 1250 2500 5000 10000; do
timeout -k 10 300 python bench.py --channels $c --steps 10 --warmup 2 --no-cpu --no-rolling --no-stream --no-extra > gpurun_out/bench_ch$c.json 2> gpurun_out/bench_ch$c.err || { tail -20 gpurun_out/bench_ch$c.err; exit 1; }
tail -1 gpurun_out/bench_ch$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ch', $c, 'K1', round(r['kernel_ms'],3), 'scan', round(r['scan_kernel_ms'],3), 'step', round(d['ms_per_step'],3), 'value %.3e' % d['value'])"
done
