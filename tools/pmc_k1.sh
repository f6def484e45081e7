# Focused PMC passes on the block-functional kernel (small config)
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-k1}; shift || true
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
ARGS="--channels 2000 --steps 2 --warmup 0 --no-cpu --no-rolling"
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/$name -o $name --kernel-include-regex block_functionals --pmc "$@" -- python3 bench.py $ARGS > $OUT/$name.log 2>&1; }
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM
run tc1 TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
