# GPU-box recipes behind the A/B and profile records in profiles/ (each step
# time-limited; run one at a time through gpurun):  bash tools/recipes.sh <name>
#
# Every A/B knob (LFD_*) exists only in the diagnostic build liblfdas_diag.so
# (-DLFD_DIAG, made by __graft_entry__.build()); the product liblfdas.so reads
# no environment variable.  The recipes therefore load the diagnostic library.
# In-process A/Bs compare knobs on ONE input allocation (tools/ab_plan.py),
# because K1's speed depends on the physical placement of a fresh 72 GB
# tensor, and NaN-fill the output before every compared execute.
set -o pipefail
mkdir -p gpurun_out
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
case "$1" in
  # ---- round 2
  k1)      # K1 launch configuration (profiles/r02_ab_k1_minw.txt, r02_ab_k1_diag.txt)
    timeout -k 10 400 python tools/ab_plan.py --reps 5 "" "LFD_RUN_MINW=0 LFD_RUN_PF=2" "LFD_RUN_M4=1" \
        "LFD_RUN_BUF=1" "LFD_NO_RUNS=1 LFD_MF_MODE=3" ;;
  units)   # K1 unit size at a 1,250-channel shard, one-run tail units (plan-time knobs: --replan)
    timeout -k 10 300 python tools/ab_plan.py --replan --ch 1250 --reps 3 "" "LFD_RUN_UNIT=8" "LFD_RUN_UNIT=32" &&
    timeout -k 10 300 python tools/ab_plan.py --replan --reps 4 "" "LFD_RUN_TAIL=0" ;;
  scan)    # deferred-output scan by width (DESIGN §2 k_chunk_scan)
    for c in 1250 2500 5000 10000; do
      timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 3 "" "LFD_SCAN_DEFER=0" "LFD_SCAN_DEFER=1" || exit 1
    done ;;
  offgrid) # head skip (plan-time knob: separate processes)
    timeout -k 10 200 python tools/ab_plan.py --off-ns 1900000 --reps 2 "" &&
    LFD_NO_HSKIP=1 timeout -k 10 200 python tools/ab_plan.py --off-ns 1900000 --reps 2 "" ;;
  tm_r02)  # time-major K1 loads / MFMA shape (profiles/r02_ab_tm.txt)
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_BUF=0" "LFD_TM_X2=0" "LFD_TM_M4=1" \
        "LFD_TM_NT=768 LFD_TM_PF=1" ;;
  rolling_r02) # rolling-mean scan kernel (profiles/r02_ab_roll_ring.txt)
    for S in 1 250; do
      timeout -k 10 200 python tools/roll_ab.py 1000 $S "" "LFD_ROLL_RING=0" "LFD_ROLL_DPP=0" || exit 1
    done ;;
  mfma)    # fp64 MFMA issue rates and the 4x4x4 operand layout
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/ub tools/ubench_mfma64b.hip &&
    timeout -k 5 60 /tmp/ub &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/c4 tools/check_mfma4x4.hip &&
    timeout -k 5 30 /tmp/c4 ;;
  # ---- round 3
  tm)       # time-major K1: streaming epilogue, diagnostics, 4x4x4 steps
            # (profiles/r03_ab_tm_sepi.txt, r03_tm_diag.txt, r03_ab_tm_m4.txt)
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_SEPI=0" "LFD_TM_MODE=3" \
        "LFD_TM_MODE=4 LFD_TM_DIAG_LDS=1" "LFD_TM_M4=1" ;;
  tm_ubench) # bare time-major access shapes (profiles/r03_ubench_tm.txt)
    timeout -k 10 300 ./tools/ubench_tm ;;
  narrow)   # 1,250-channel shard: units, drain, unit order, scan rings / workgroup size
            # (profiles/r03_ab_narrow_units.txt, r03_ab_narrow_band.txt, r03_ab_scan_deep.txt)
    timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 3 --replan "" "LFD_RUN_UNIT=8" "LFD_RUN_TAIL=0" &&
    timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_K1_BAND=1" "LFD_K1_BAND=16" \
        "LFD_SCAN_DEEP=1" "LFD_SCAN_DEFER_THREADS=64" &&
    timeout -k 10 400 python tools/probe_scan.py narrow ;;
  longscan) # deep scan rings on long run chains (dt = 10 s at 1 kHz)
    timeout -k 10 400 python tools/ab_plan.py --fs 1000 --dt 10 --P 120 --B 6 --ch 2000 --reps 3 "" "LFD_SCAN_DEEP=0" ;;
  rolling)  # segment-sum rolling mean vs the running-sum scan (profiles/r03_ab_roll_segsum.txt)
    timeout -k 10 200 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEGSUM=0" ;;
  fir)      # FIR decimation: matrix-core kernel vs VALU kernel, breakdown and variants
            # (profiles/r03_ab_fir.txt)
    for e in "" "LFD_FIR_VALU=1" "LFD_FIR_DIAG=1" "LFD_FIR_DIAG=2" "LFD_FIR_DIAG=4" "LFD_FIR_DIAG=8" \
             "LFD_FIR_DIAG=16" "LFD_FIR_DB=1" "LFD_FIR_STRIP=2"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py || exit 1
    done ;;
  fir_pmc)  # PMC of the matrix-core FIR kernel (profiles/r03_pmc_fir_mfma.txt)
    bash tools/pmc_kernel.sh fir fir_decimate_mfma tools/fir_one.py 10 ;;
  fullrate) # full-rate band-pass staging A/B and PMC (profiles/r03_pmc_fullrate.txt)
    for e in "" "LFD_FR_STAGE_OLD=1"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py || exit 1
    done &&
    bash tools/pmc_kernel.sh fr fullrate tools/fr_one.py 2 ;;
  lattice)  # lattice plan vs the per-chunk general path at 3 kHz
    timeout -k 10 300 python tools/lattice_bench.py ;;
  multi)    # N > 1 launcher on a 1-GPU box: refusal, then the one-device rehearsal
    timeout -k 10 120 python bench.py --gpus 2 --steps 1; echo "bench --gpus 2 exit $? (want 2)"
    timeout -k 10 300 python bench.py --gpus 2 --one-device --steps 2 --warmup 1 --no-cpu --no-rolling \
        --no-extra --no-stream ;;
  # ---- round 4
  persist)  # persistent run-mode K1 (units pulled from a counter) vs one unit per wave, by shard width
    for ch in 1250 2500 5000 10000; do
      timeout -k 10 300 python tools/ab_plan.py --ch $ch --reps 4 --steps 5 "" "LFD_K1_PERSIST=0" || exit 1
    done ;;
  *) echo "recipes: k1 units scan offgrid tm_r02 rolling_r02 mfma tm tm_ubench narrow longscan rolling fir fir_pmc"
     echo "         fullrate lattice multi persist"; exit 2 ;;
esac
