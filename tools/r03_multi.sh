# Round 3: the multi-GPU path on a 1-GPU box (each step time-limited; stop on failure)
set -o pipefail
mkdir -p gpurun_out
T="--timeout 150 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dropin.py -x -v $T > gpurun_out/r03_dist.log 2>&1 || { tail -40 gpurun_out/r03_dist.log; exit 1; }
tail -3 gpurun_out/r03_dist.log
# an N > 1 request on a 1-GPU node: must fail clearly, no JSON line
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > gpurun_out/r03_gpus2.out 2> gpurun_out/r03_gpus2.err; echo "bench --gpus 2 exit $? (want 2)"; cat gpurun_out/r03_gpus2.err
# rehearsal of the N = 2 bench path: both ranks on cuda:0 over gloo
timeout -k 10 400 python bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --no-rolling --no-extra > gpurun_out/r03_rehearsal.json 2> gpurun_out/r03_rehearsal.err || { tail -30 gpurun_out/r03_rehearsal.err; exit 1; }
tail -1 gpurun_out/r03_rehearsal.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'ranks_seen', d['ranks_seen'], 'value %.3e' % d['value']); print(json.dumps(d['secondary'].get('out_of_core_cfg5_sharded'))[:600]); print(json.dumps(d['secondary'].get('allgather_outputs')))"
# time-major K1: production vs loads-only floor (MODE 3) vs no epilogue (MODE 4), one allocation
timeout -k 10 300 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_MODE=3" "LFD_TM_MODE=4" > gpurun_out/r03_tm_diag.txt 2>&1 || { tail -20 gpurun_out/r03_tm_diag.txt; exit 1; }
tail -4 gpurun_out/r03_tm_diag.txt
# rolling mean: the new segment-sum kernel vs the running-sum scan (cfg2, S = 250 / 200)
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -x -q -k rolling --timeout 120 --timeout-method thread > gpurun_out/r03_roll_tests.log 2>&1 || { tail -30 gpurun_out/r03_roll_tests.log; exit 1; }
tail -1 gpurun_out/r03_roll_tests.log
timeout -k 10 200 python tools/roll_ab.py > gpurun_out/r03_roll_ab.txt 2>&1 || { tail -20 gpurun_out/r03_roll_ab.txt; exit 1; }
cat gpurun_out/r03_roll_ab.txt
