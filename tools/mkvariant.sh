# Build liblfdas variants for tools/ab_libs.sh:
#   tools/mkvariant.sh <name> [git-rev]   (no rev: the working tree)
set -e
name=$1; rev=$2
out=build/variants/lib_$name.so
mkdir -p build/variants
if [ -n "$rev" ]; then
  d=$(mktemp -d); git archive "$rev" low-freq-real-time_amd/csrc include | tar -x -C "$d"
  src=$d/low-freq-real-time_amd/csrc
else
  src=low-freq-real-time_amd/csrc
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $EXTRA \
  $src/lfd_kernels.hip $src/lfd_capi.cpp $src/lfd_stream.cpp -o $out
echo "$out"
