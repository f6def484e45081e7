#!/bin/bash
# Collect the rocprofv3 evidence for bench.py's dominant kernel on the GPU box.
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats of the full bench config (timing agrees with bench.py)
# 2) PMC passes (separate runs, no tracing domains besides kernel-trace)
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o trace -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --no-rolling "$@" > $OUT/bench_traced.log 2>&1
SMALL="--channels 2000 --steps 2 --warmup 0 --no-cpu --no-rolling"
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_sq -o sq \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
    -- python3 bench.py $SMALL > $OUT/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_fetch -o fetch --pmc FETCH_SIZE \
    -- python3 bench.py $SMALL > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_write -o write --pmc WRITE_SIZE \
    -- python3 bench.py $SMALL > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/pmc_tcc -o tcc --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    -- python3 bench.py $SMALL > $OUT/pmc_tcc.log 2>&1 || true
echo done
