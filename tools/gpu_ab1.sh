set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "time_major or lfproc_parity or rolling" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 200 python tools/tm_bench.py > gpurun_out/tm.log 2>&1 || { tail -20 gpurun_out/tm.log; exit 1; }
grep TM gpurun_out/tm.log
timeout -k 10 200 python tools/ab_roll_env.py 1 "LFD_ROLL_PF=1" "LFD_ROLL_PF=2" "LFD_ROLL_PF=3" "LFD_ROLL_PF=2 LFD_ROLL_SEG=65536" > gpurun_out/roll.log 2>&1 || { tail -20 gpurun_out/roll.log; exit 1; }
cat gpurun_out/roll.log
timeout -k 5 60 ./tools/ubench_mfma64b > gpurun_out/ub64b.txt 2>&1; cat gpurun_out/ub64b.txt
