# lattice one-pass with the fused output kernel: parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "lattice or 3khz or stream" > gpurun_out/r04n_pytest.log 2>&1 || { tail -30 gpurun_out/r04n_pytest.log; exit 1; }
tail -1 gpurun_out/r04n_pytest.log
timeout -k 10 200 python tools/lattice_bench.py > gpurun_out/r04n_lattice.txt 2>&1 || { tail -20 gpurun_out/r04n_lattice.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04n_lattice.txt
