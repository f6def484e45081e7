# time-major K1 with 256-thread groups (GPU suite, in-process A/B against the 512-thread groups) and the full-rate functionals with round-filling units (vs 32 blocks per wave)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04r_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04r_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04r_pytest_gpu.log
timeout -k 10 400 python tools/ab_plan.py --tm --reps 5 "" "LFD_TM_W=512" > gpurun_out/r04r_ab_tm.txt 2>&1 || { tail -20 gpurun_out/r04r_ab_tm.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04r_ab_tm.txt | tail -3
timeout -k 10 300 python tools/ab_plan.py --tm --ch 1250 --reps 5 "" "LFD_TM_W=512" > gpurun_out/r04r_ab_tm_1250.txt 2>&1 || { tail -20 gpurun_out/r04r_ab_tm_1250.txt; exit 1; }
grep -v "amdgpu.ids\|lfdas: loaded" gpurun_out/r04r_ab_tm_1250.txt | tail -3
for e in "" "LFD_MF_BPW=32" "" "LFD_MF_BPW=32"; do
  echo "== fullrate $e"; env $e timeout -k 10 120 python tools/fr_bench.py > gpurun_out/r04r_fr.txt 2>&1 || { tail -20 gpurun_out/r04r_fr.txt; exit 1; }
  tail -1 gpurun_out/r04r_fr.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'pipe', round(d['pipeline_hbm_frac'],3), 'rel', d['relrms_vs_oracle_3ch'])"
done
