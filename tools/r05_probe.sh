# round-5: full-rate output pass: wave stagger A/B (separate processes)
set -o pipefail
O=gpurun_out/r05fr
mkdir -p $O
for v in 0; do
  echo "== LFD_FR_STAGGER=$v"
  LFD_FR_TIMES=1 timeout -k 10 200 python tools/fr_bench.py 2>&1 | grep -v amdgpu.ids | tee -a $O/times.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms'],3), {k.split(' ')[0]: round(v,3) for k,v in d['kernels_ms'].items()}, d['relrms_vs_oracle_3ch'])" || exit 1
done > $O/stagger.txt 2>&1
echo "exit $?"; cat $O/stagger.txt
grep k_fullrate_out $O/times.txt | sort | uniq -c | head -5
