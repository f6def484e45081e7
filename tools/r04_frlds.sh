# full-rate output pass with the conflict-free LDS layout: parity, timing, LDS PMC
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04f}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "full_rate or bandpass or env" > gpurun_out/${tag}_pytest_fr.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_fr.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest_fr.log
for i in 1 2; do
  timeout -k 10 120 python tools/fr_bench.py > gpurun_out/${tag}_fr.txt 2>&1 || { tail -20 gpurun_out/${tag}_fr.txt; exit 1; }
  tail -1 gpurun_out/${tag}_fr.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'pipe', round(d['pipeline_hbm_frac'],3), 'rel', d['relrms_vs_oracle_3ch'])"
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/pmc_${tag}/sq2 -o sq2 --kernel-include-regex "fullrate|block_functionals_mfma" --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -- python3 tools/fr_one.py 2 > gpurun_out/pmc_${tag}_sq2.log 2>&1 || { tail -20 gpurun_out/pmc_${tag}_sq2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_${tag} > gpurun_out/pmc_${tag}/summary.txt
grep -E "out_mb|functionals|scan_seg" gpurun_out/pmc_${tag}/summary.txt
