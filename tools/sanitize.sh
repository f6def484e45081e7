#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of liblfdas's
# host code: lfd_capi.cpp (plan geometry, x87 constants),
# lfd_stream.cpp (arena / schedule bookkeeping), linked with the kernels'
# object (its launchers uninstrumented: build/liblfdas/lfd_kernels.o from
# __graft_entry__.build(), else compiled here) into
# tests/capi/host_sanitize.cpp; plus
# lfd_h5.cpp with its round-trip driver when libhdf5 is present.  Host only:
# `-Xarch_host -fsanitize=...` (no GPU sanitizer), CPU container.
#   bash tools/sanitize.sh [outdir]   -> <outdir>/host_sanitize [, <outdir>/h5_sanitize]
set -e -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/build/sanitize}"
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all
     -fno-gpu-sanitize -fno-omit-frame-pointer -g -O1 -std=c++17 -fPIC)
CS="$ROOT/low-freq-real-time_amd/csrc"
pids=()
KO="$ROOT/build/liblfdas/lfd_kernels.o"
if [ ! -f "$KO" ] || [ "$KO" -ot "$CS/lfd_kernels.hip" ]; then
  KO="$OUT/lfd_kernels.o"
  "$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$CS/lfd_kernels.hip" -o "$KO" & pids+=($!)
fi
"$HIPCC" --offload-arch=gfx950 "${SAN[@]}" -c "$CS/lfd_capi.cpp" -o "$OUT/lfd_capi.o" & pids+=($!)
"$HIPCC" --offload-arch=gfx950 "${SAN[@]}" -c "$CS/lfd_stream.cpp" -o "$OUT/lfd_stream.o" & pids+=($!)
"$HIPCC" --offload-arch=gfx950 "${SAN[@]}" -c "$ROOT/tests/capi/host_sanitize.cpp" -o "$OUT/host_sanitize.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch=gfx950 -fsanitize=address,undefined -fno-gpu-sanitize "$KO" "$OUT"/lfd_capi.o \
    "$OUT"/lfd_stream.o "$OUT"/host_sanitize.o -o "$OUT/host_sanitize"
if [ -f /opt/conda/include/hdf5.h ]; then
  g++ -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1 -std=c++17 -static-libstdc++ \
      -I/opt/conda/include "$CS/lfd_h5.cpp" "$ROOT/tests/capi/h5_sanitize.cpp" -L/opt/conda/lib -lhdf5 \
      -Wl,-rpath,/opt/conda/lib -o "$OUT/h5_sanitize"
fi
echo "built $OUT"
