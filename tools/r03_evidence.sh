# Round-3 evidence: GPU suite, smoke, default bench line, rocprofv3 trace + PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03b_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03b_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03b_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.log 2>&1 || { tail -20 gpurun_out/r03b_smoke.log; exit 1; }
tail -2 gpurun_out/r03b_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { tail -20 gpurun_out/r03b_bench.err; exit 1; }
tail -1 gpurun_out/r03b_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', round(d['ms_per_step'],3), 'K1', round(r['kernel_ms'],3), 'frac', round(r['frac'],3))"
bash tools/profile.sh r03b || exit 1
python3 tools/trace_summary.py gpurun_out/prof_r03b gpurun_out/prof_r03b/kernel_stats.txt || true
echo evidence done
