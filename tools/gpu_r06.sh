# Round-6 GPU check: pytest -m gpu (gate values logged), smoke, bench.
#   bash tools/gpu_r06.sh TAG [measure]   ("measure": gates held to 1e-4 only)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${1:-r06}
export LFD_GATE_LOG=$PWD/gpurun_out/gates_${T}.jsonl
[ "$2" = measure ] && export LFD_GATE_MEASURE=1
rm -f "$LFD_GATE_LOG"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail 15 > gpurun_out/${T}_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${T}_gpu.log
unset LFD_GATE_MEASURE LFD_GATE_LOG
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc2=$?; echo "smoke+bench rc=$rc2"; tail -2 gpurun_out/${T}_smoke.log; tail -c 1500 gpurun_out/${T}_bench.json; exit $rc2
