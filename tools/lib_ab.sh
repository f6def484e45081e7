#!/bin/bash
# A/B of two builds of the diagnostic library on one box, alternating runs in
# separate processes: tools/lib_ab.sh OLD_LIB NEW_LIB ROUNDS -- python SCRIPT ARGS...
# (each run's JSON / text output tagged with the library it used)
old=$1; new=$2; rounds=$3; shift 4
for r in $(seq 1 "$rounds"); do
  for tag in old new; do
    lib=$old; [ "$tag" = new ] && lib=$new
    out=$(LFDAS_LIB=$lib timeout -k 10 200 "$@" 2>&1 | grep -v "amdgpu.ids\|lfdas: loaded") || exit 1
    echo "[$tag r$r] $out"
  done
done
