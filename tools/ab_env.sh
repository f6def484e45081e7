# A/B of env-knob variants of the current library (plus optional variant libs)
#   SPECS="tag:VAR=v,VAR2=v tag2:..."  LIBS="name ..." (build/variants/lib_<name>.so)
set -e -o pipefail
mkdir -p gpurun_out/ab
one() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-rolling --no-stream > gpurun_out/ab/$tag.log 2>&1
  printf "%-12s " $tag
  tail -1 gpurun_out/ab/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("K1", round(r["kernel_ms"],3), "scan", round(r["scan_kernel_ms"],3), "step", round(d["ms_per_step"],3))'
}
for rep in 1 2 3; do
  for l in $LIBS; do one lib_$l LFDAS_LIB=$PWD/build/variants/lib_$l.so; done
  for spec in $SPECS; do one ${spec%%:*} $(echo ${spec#*:} | tr ',' ' '); done
done
