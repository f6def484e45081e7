# round-5: rolling segment-sum output batches test
set -o pipefail
O=gpurun_out/r05rb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowpass.py -x -q --timeout 200 --timeout-method thread -k "rolling" > $O/pytest.log 2>&1
echo "pytest exit $?"; tail -3 $O/pytest.log
