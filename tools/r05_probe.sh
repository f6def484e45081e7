# round-5 final: GPU suite, smoke, default bench
set -o pipefail
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest exit $?"; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke exit $?"; tail -3 $O/smoke.log
timeout -k 10 1000 python bench.py > $O/bench.json 2> $O/bench.err
echo "bench exit $?"
python tools/bench_summary.py $O/bench.json
