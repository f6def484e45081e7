# PMC passes on the full-rate kernels (2,000 x 600,000 band-pass, tools/fr_one.py)
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-fr}; shift || true
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/$name -o $name --kernel-include-regex "fullrate|block_functionals_mfma" --pmc "$@" -- python3 tools/fr_one.py 2 > $OUT/$name.log 2>&1; }
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM
run sq3 SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
