set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/ubench_tm > gpurun_out/r03c_ubench_tm.txt 2>&1 || { cat gpurun_out/r03c_ubench_tm.txt; exit 1; }
cat gpurun_out/r03c_ubench_tm.txt
