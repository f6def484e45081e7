# round-5: GPU suite after removing the rejected kernel variants; FIR / full-rate / tm timings
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest exit $?"; tail -3 $O/pytest_gpu.log
timeout -k 10 300 python tools/fir_ab.py 10 "" > $O/fir.txt 2>&1; grep "q=" $O/fir.txt
timeout -k 10 300 python tools/fr_bench.py 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k.split(' ')[0]: round(v,3) for k,v in d['kernels_ms'].items()})"
