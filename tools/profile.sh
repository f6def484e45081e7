#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box).
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats of the bench config (durations agree with bench.py)
# 2) PMC passes, each its own run with --kernel-trace only:
#    FETCH_SIZE / WRITE_SIZE of the full-size K1, and the same counters on
#    tools/ubench_hbm_pattern (known byte counts) to calibrate their units
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o trace -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --no-rolling --no-stream "$@" > $OUT/bench_traced.log 2>&1
FULL="--steps 2 --warmup 0 --no-cpu --no-rolling --no-stream --no-extra"
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_fetch -o fetch --pmc FETCH_SIZE \
    --kernel-include-regex k_block_ -- python3 bench.py $FULL "$@" > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_write -o write --pmc WRITE_SIZE \
    --kernel-include-regex k_block_ -- python3 bench.py $FULL "$@" > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/calib_fetch -o cf --pmc FETCH_SIZE \
    -- ./tools/ubench_hbm_pattern > $OUT/calib_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/calib_write -o cw --pmc WRITE_SIZE \
    -- ./tools/ubench_hbm_pattern > $OUT/calib_write.log 2>&1
# the rolling-mean kernels (cfg2, W = S = 1000 and S = 1)
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/roll_fetch -o rf --pmc FETCH_SIZE \
    --kernel-include-regex k_rolling -- python3 tools/roll_only.py > $OUT/roll_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/roll_write -o rw --pmc WRITE_SIZE \
    --kernel-include-regex k_rolling -- python3 tools/roll_only.py > $OUT/roll_write.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
echo done
