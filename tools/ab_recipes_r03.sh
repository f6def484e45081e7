# GPU-box recipes behind the round-3 records in profiles/ (each step is
# time-limited; run one at a time through gpurun):  bash tools/ab_recipes_r03.sh <name>
# In-process A/Bs compare env knobs on ONE input allocation (tools/ab_plan.py).
set -o pipefail
mkdir -p gpurun_out
case "$1" in
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
    timeout -k 10 200 python tools/roll_ab.py ;;
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
  *) echo "recipes: tm tm_ubench narrow longscan rolling fir fir_pmc fullrate lattice multi"; exit 2 ;;
esac
