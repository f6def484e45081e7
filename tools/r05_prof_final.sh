#!/bin/bash
# rocprofv3 kernel-trace statistics of the kernels changed in round 5, with
# the product library where the tool allows it (profiles/r05f_kernel_stats.txt):
# the headline bench (K1 + scan), the full-rate band-pass line and the FIR line.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof_r05f
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/head -o head -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu --no-rolling --no-stream --no-extra > $OUT/head.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fr -o fr -- \
    python3 tools/fr_bench.py > $OUT/fr.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fir -o fir -- \
    python3 tools/fir_bench.py > $OUT/fir.log 2>&1
echo done
