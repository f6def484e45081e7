# round-5: PMC passes on the full-rate kernels and the FIR decimation (after this round's changes)
set -o pipefail
bash tools/pmc_fullrate.sh r05fr > /dev/null 2>&1 && echo fr-ok
bash tools/pmc_kernel.sh r05fir k_fir_decimate tools/fir_one.py > /dev/null 2>&1 && echo fir-ok
cat gpurun_out/pmc_r05fr/summary.txt | grep -E "k_fullrate_out_mb" | head -30
cat gpurun_out/pmc_r05fir/summary.txt | head -30
