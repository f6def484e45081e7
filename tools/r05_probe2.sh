# round-5: rolling S = 1 with 16 positions per lane per step (LFD_RS_E=16 build) vs 8, separate processes
set -o pipefail
O=gpurun_out/r05rs
mkdir -p $O
for lib in liblfdas_diag.so liblfdas_diag_rs16.so liblfdas_diag.so liblfdas_diag_rs16.so; do
  echo "== $lib"
  LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/$lib" timeout -k 10 300 python tools/roll_ab.py 1000 1 "" 2>&1 | grep -E "W=" || exit 1
done > $O/rs.txt 2>&1
echo "exit $?"; cat $O/rs.txt
