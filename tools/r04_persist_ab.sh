# round 4: GPU suite with the persistent run-mode K1, then the persistent vs
# one-unit-per-wave A/B at the shard widths (diag library, one allocation each)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.log
for ch in 1250 2500 5000 10000; do
  timeout -k 10 300 python tools/ab_plan.py --ch $ch --reps 4 --steps 5 "" "LFD_K1_PERSIST=0" > gpurun_out/${tag}_ab_persist_${ch}.txt 2>&1 || { tail -20 gpurun_out/${tag}_ab_persist_${ch}.txt; exit 1; }
  tail -2 gpurun_out/${tag}_ab_persist_${ch}.txt
done
for e in "" "LFD_FULLRATE_BIGBLOCK=1"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/${tag}_fr_${e:-default}.txt 2>&1 || { tail -20 gpurun_out/${tag}_fr_${e:-default}.txt; exit 1; }
  tail -6 gpurun_out/${tag}_fr_${e:-default}.txt
done
