# full GPU suite on the current tree, then the N > 1 launcher checks (each step time-limited; stop on failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e_suite.log 2>&1 || { tail -40 gpurun_out/r03e_suite.log; exit 1; }
tail -2 gpurun_out/r03e_suite.log
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > gpurun_out/r03e_gpus2.out 2> gpurun_out/r03e_gpus2.err; echo "bench --gpus 2 exit $? (want 2)"; tail -3 gpurun_out/r03e_gpus2.err
timeout -k 10 300 python bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --no-rolling --no-extra > gpurun_out/r03e_rehearsal.json 2> gpurun_out/r03e_rehearsal.err || { tail -30 gpurun_out/r03e_rehearsal.err; exit 1; }
tail -c 1500 gpurun_out/r03e_rehearsal.json
timeout -k 10 300 python bench.py > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err || { tail -30 gpurun_out/r03e_bench.err; exit 1; }
tail -c 3000 gpurun_out/r03e_bench.json
