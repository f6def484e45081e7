# A/B of the MFMA block-functional kernel variants (env knobs of lfd_kernels.hip).
# SPECS="tag:VAR=v,VAR2=v tag2:..."  (default: production / loads only / nt loads)
set -e -o pipefail
mkdir -p gpurun_out/ab_mf
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --no-rolling --no-stream > gpurun_out/ab_mf/$tag.log 2>&1
  printf "%-14s " $tag
  tail -1 gpurun_out/ab_mf/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("K1", round(r["kernel_ms"],3), "ms frac", round(r["frac"],3))'
}
for spec in ${SPECS:-base:LFD_MF_MODE=0 ldonly:LFD_MF_MODE=1 nt:LFD_MF_MODE=2}; do
  run ${spec%%:*} $(echo ${spec#*:} | tr ',' ' ')
done
