# round 4: GPU suite, full-rate medium/big-block A/B, lattice one-pass vs per-phase
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.log
for e in "" "LFD_FULLRATE_BIGBLOCK=1"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/${tag}_fr_${e:-default}.txt 2>&1 || { tail -20 gpurun_out/${tag}_fr_${e:-default}.txt; exit 1; }
  tail -1 gpurun_out/${tag}_fr_${e:-default}.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'pipe', round(d['pipeline_hbm_frac'],3), 'rel', d['relrms_vs_oracle_3ch'])"
done
echo "== lattice"; timeout -k 10 200 python tools/lattice_bench.py > gpurun_out/${tag}_lattice.txt 2>&1 || { tail -20 gpurun_out/${tag}_lattice.txt; exit 1; }
cat gpurun_out/${tag}_lattice.txt
for c in 1250 2500; do
  echo "== narrow shard $c"; timeout -k 10 240 python tools/ab_plan.py --ch $c --replan --reps 3 "" "LFD_RUN_UNIT=8" "LFD_RUN_TAIL=0" "LFD_RUN_UNIT=8 LFD_RUN_TAIL=4" > gpurun_out/${tag}_ab_narrow_$c.txt 2>&1 || { tail -20 gpurun_out/${tag}_ab_narrow_$c.txt; exit 1; }
  tail -6 gpurun_out/${tag}_ab_narrow_$c.txt
done
