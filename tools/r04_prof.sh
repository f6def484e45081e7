# round 4 profiles: PMC of the full-rate kernels and of the lattice one-pass
# line (each counter group its own rocprofv3 run, --kernel-trace only)
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_fullrate.sh r04fr > gpurun_out/r04_pmc_fullrate.log 2>&1 || { tail -30 gpurun_out/r04_pmc_fullrate.log; exit 1; }
cat gpurun_out/pmc_r04fr/summary.txt
bash tools/pmc_kernel.sh r04lat "k_block_runs_mfma|k_chunk_scan|k_run_outputs|k_blend_grid" tools/lattice_one.py 2 > gpurun_out/r04_pmc_lattice.log 2>&1 || { tail -30 gpurun_out/r04_pmc_lattice.log; exit 1; }
cat gpurun_out/pmc_r04lat/summary.txt
