# GPU-box recipes behind the A/B and profile records in profiles/ (each step
# time-limited; run one at a time through gpurun):  bash tools/recipes.sh <name>
#
# Every A/B knob (LFD_*) exists only in the diagnostic build liblfdas_diag.so
# (-DLFD_DIAG, made by __graft_entry__.build()); the product liblfdas.so reads
# no environment variable.  The recipes therefore load the diagnostic library.
# In-process A/Bs compare knobs on ONE input allocation (tools/ab_plan.py),
# because K1's speed depends on the physical placement of a fresh 72 GB
# tensor, and NaN-fill the output before every compared execute.
# Round 5 deleted the kernel variants those records rejected (K1 4x4x4 /
# buffer-load / streaming-epilogue / persistent / band orders; time-major
# swap / one-tile / 4x4x4 / 768-thread / depth-3; full-rate direct stores,
# 34-float layout, 4x4x4, early-KAZ; FIR double buffer; rolling staged loads,
# depth 2-3, 4 waves per SIMD; functionals 4x4x4 and depth 1): their knobs in
# the recipes below are now no-ops and the records in profiles/ are the
# history.  The timing-only modes (LFD_RUN_MODE, LFD_TM_MODE, LFD_MF_MODE,
# LFD_FIR_DIAG 1 / 2, LFD_SCAN_DIAG, LFD_FU_*, LFD_FR_TIMES) remain.
set -o pipefail
mkdir -p gpurun_out
export LFDAS_LIB="$PWD/low-freq-real-time_amd/lfdas/liblfdas_diag.so"
case "$1" in
  # ---- round 2
  k1)      # K1 launch configuration (profiles/archive_r01_r03.md (r02_ab_k1_minw.txt), r02_ab_k1_diag.txt)
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
  tm_r02)  # time-major K1 loads / MFMA shape (profiles/archive_r01_r03.md (r02_ab_tm.txt))
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_BUF=0" "LFD_TM_X2=0" "LFD_TM_M4=1" \
        "LFD_TM_NT=768 LFD_TM_PF=1" ;;
  rolling_r02) # rolling-mean scan kernel (profiles/archive_r01_r03.md (r02_ab_roll_ring.txt))
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
            # (profiles/archive_r01_r03.md (r03_ab_tm_sepi.txt), r03_tm_diag.txt, r03_ab_tm_m4.txt)
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_SEPI=0" "LFD_TM_MODE=3" \
        "LFD_TM_MODE=4 LFD_TM_DIAG_LDS=1" "LFD_TM_M4=1" ;;
  tm_ubench) # bare time-major access shapes (profiles/archive_r01_r03.md (r03_ubench_tm.txt))
    timeout -k 10 300 ./tools/ubench_tm ;;
  narrow)   # 1,250-channel shard: units, drain, unit order, scan rings / workgroup size
            # (profiles/archive_r01_r03.md (r03_ab_narrow_units.txt), r03_ab_narrow_band.txt, r03_ab_scan_deep.txt)
    timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 3 --replan "" "LFD_RUN_UNIT=8" "LFD_RUN_TAIL=0" &&
    timeout -k 10 400 python tools/ab_plan.py --ch 1250 --reps 4 "" "LFD_K1_BAND=1" "LFD_K1_BAND=16" \
        "LFD_SCAN_DEEP=1" "LFD_SCAN_DEFER_THREADS=64" &&
    timeout -k 10 400 python tools/probe_scan.py narrow ;;
  longscan) # deep scan rings on long run chains (dt = 10 s at 1 kHz)
    timeout -k 10 400 python tools/ab_plan.py --fs 1000 --dt 10 --P 120 --B 6 --ch 2000 --reps 3 "" "LFD_SCAN_DEEP=0" ;;
  rolling)  # segment-sum rolling mean vs the running-sum scan (profiles/archive_r01_r03.md (r03_ab_roll_segsum.txt))
    timeout -k 10 200 python tools/roll_ab.py 1000 250 "" "LFD_ROLL_SEGSUM=0" ;;
  fir)      # FIR decimation: matrix-core kernel vs VALU kernel, breakdown and variants
            # (profiles/archive_r01_r03.md (r03_ab_fir.txt))
    for e in "" "LFD_FIR_VALU=1" "LFD_FIR_DIAG=1" "LFD_FIR_DIAG=2" "LFD_FIR_DIAG=4" "LFD_FIR_DIAG=8" \
             "LFD_FIR_DIAG=16" "LFD_FIR_DB=1" "LFD_FIR_STRIP=2"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fir_bench.py || exit 1
    done ;;
  fir_pmc)  # PMC of the matrix-core FIR kernel (profiles/archive_r01_r03.md (r03_pmc_fir_mfma.txt))
    bash tools/pmc_kernel.sh fir fir_decimate_mfma tools/fir_one.py 10 ;;
  fullrate) # full-rate band-pass staging A/B and PMC (profiles/archive_r01_r03.md (r03_pmc_fullrate.txt))
    for e in "" "LFD_FR_STAGE_OLD=1"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py || exit 1
    done &&
    bash tools/pmc_kernel.sh fr fullrate tools/fr_one.py 2 ;;
  lattice)  # lattice plan: one pass vs the per-phase sub-plans at 3 kHz
            # (profiles/r04d_lattice_onepass_vs_phases.txt, r04n_lattice_fused_outputs.txt)
    timeout -k 10 300 python tools/lattice_bench.py ;;
  multi)    # N > 1 launcher on a 1-GPU box: refusal, then the one-device rehearsal
    timeout -k 10 120 python bench.py --gpus 2 --steps 1; echo "bench --gpus 2 exit $? (want 2)"
    timeout -k 10 300 python bench.py --gpus 2 --one-device --steps 2 --warmup 1 --no-cpu --no-rolling \
        --no-extra --no-stream ;;
  # ---- round 4
  persist)  # persistent run-mode K1 (static unit assignment) vs one unit per wave, by shard width
            # (profiles/r04_ab_k1_persist_*.txt)
    for ch in 1250 2500 5000 10000; do
      timeout -k 10 300 python tools/ab_plan.py --ch $ch --reps 4 --steps 5 "" "LFD_K1_PERSIST=1" || exit 1
    done ;;
  narrow_units) # K1 unit size / tail rounds at 1,250 and 2,500 channels (profiles/r04d_ab_narrow_units.txt)
    for c in 1250 2500; do
      timeout -k 10 240 python tools/ab_plan.py --ch $c --replan --reps 3 "" "LFD_RUN_UNIT=8" "LFD_RUN_TAIL=0" \
          "LFD_RUN_UNIT=8 LFD_RUN_TAIL=4" || exit 1
    done ;;
  scan_trace) # narrow-shard scan phases (diag) and kernel times, deep vs 4 / 2 ring
              # (profiles/r04l_scan_deep.txt)
    timeout -k 10 350 python tools/probe_scan.py narrow || exit 1
    cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
    for e in "" "LFD_SCAN_DEEP=0"; do
      for c in 1250 2500; do
        d=gpurun_out/scan_trace_${c}_${e:-default}
        env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $d -o tr -- python3 tools/scan_one.py $c \
            > $d.log 2>&1 || exit 1
        echo "== $c ${e:-default}"; grep -h "chunk_scan\|run_outputs\|runs_mfma" $d/*/tr_kernel_stats.csv $d/tr_kernel_stats.csv 2>/dev/null
      done
    done ;;
  seg_scan) # segmented run chains vs the unsegmented deferred scan (profiles/r04y_ab_seg_scan.txt)
    timeout -k 10 300 python tools/ab_plan.py --fs 1000 --dt 10 --P 120 --B 6 --ch 2000 --reps 4 "" "LFD_SCAN_DEFER=2" &&
    timeout -k 10 300 python tools/ab_plan.py --fs 3000 --dt 1 --seconds 1800 --P 600 --B 7 --ch 2000 --reps 4 "" \
        "LFD_SCAN_DEFER=2" &&
    for c in 1250 2500; do
      timeout -k 10 240 python tools/ab_plan.py --ch $c --reps 4 "" "LFD_SCAN_DEFER=3" || exit 1
    done ;;
  fr_mb)    # full-rate: medium-block path vs the big-block path (profiles/r04d_fr_ab_mfma_output_vs_bigblock.txt)
    for e in "" "LFD_FULLRATE_BIGBLOCK=1"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py || exit 1
    done ;;
  fr_out)   # full-rate output pass variants: direct stores, LDS layouts, 4x4x4 steps
            # (profiles/r04e_fr_ab_direct_stores.txt, r04h_fr_ab_lds_layout.txt, r04t_fr_ab_mfma4x4.txt)
    for e in "" "LFD_FR_OUT_DIRECT=1" "LFD_FR_LAYOUT=0" "LFD_FR_LAYOUT=2" "LFD_FR_M4=1" \
             "LFD_MF_BPW=32" "LFD_FR_SEG_CW=8"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py || exit 1
    done ;;
  fr_pmc)   # PMC of the medium-block full-rate kernels (profiles/r04_pmc_fullrate.txt)
    bash tools/pmc_fullrate.sh r04fr ;;
  lattice_pmc) # PMC of the lattice one-pass line (profiles/r04_pmc_lattice.txt)
    bash tools/pmc_kernel.sh r04lat "k_block_runs_mfma|k_chunk_scan|k_lat_outputs|k_blend_grid" tools/lattice_one.py 2 ;;
  tm_wg)    # time-major K1 workgroup size / waves per SIMD (profiles/r04q_ab_tm_w.txt)
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 5 "" "LFD_TM_W=512" "LFD_TM_W=21" "LFD_TM_W=3" ;;
  cm_wg)    # channel-major K1 with 256-thread groups (profiles/r04q_ab_cm_wg.txt)
    timeout -k 10 400 python tools/ab_plan.py --reps 5 "" "LFD_K1_WG=256" "LFD_K1_WG=2561" &&
    timeout -k 10 300 python tools/ab_plan.py --ch 1250 --reps 5 "" "LFD_K1_WG=256" ;;
  fir_strip) # FIR tiles per workgroup (profiles: DESIGN §9)
    for e in "" "LFD_FIR_STRIP=4" "LFD_FIR_STRIP=6" "LFD_FIR_STRIP=12" "LFD_FIR_STRIP=16" "LFD_FIR_STRIP=30"; do
      echo "${e:-default}"; env $e timeout -k 10 120 python tools/fir_bench.py | grep "q= 10" || exit 1
    done ;;
  odd_strides) # rows of any stride on the MFMA kernels (profiles/r04ag_ab_odd_strides.txt)
    for n in 599553 599800 600000 600063; do
      timeout -k 10 120 python tools/fr_bench.py $n || exit 1
    done &&
    for p in 1 0 2; do echo "== pad $p"; timeout -k 10 200 python tools/ab_plan.py --pad $p --reps 3 "" || exit 1; done ;;
  fr_scan_edges) # full-rate scan edge walks: LDS windows vs global (profiles/r04ah_fr_scan_lds_edges.txt)
    for e in "" "LFD_FR_TAIL_GLOBAL=1"; do
      echo "== $e"; env $e timeout -k 10 120 python tools/fr_bench.py 600000 || exit 1
    done ;;
  fir_xcd)  # FIR strip length and the XCD remap (diag bit 128) (profiles/r04am_fir_xcd.txt)
    for r in 1 2 3; do
      for e in "" "LFD_FIR_DIAG=128" "LFD_FIR_STRIP=16" "LFD_FIR_STRIP=4 LFD_FIR_DIAG=128" "LFD_FIR_STRIP=30 LFD_FIR_DIAG=128"; do
        echo "${e:-default} $(env $e timeout -k 10 120 python tools/fir_bench.py 2>/dev/null | grep "q= 10")" || exit 1
      done
    done ;;
  final)    # the driver's round-end steps: GPU suite, smoke, default bench line (product library)
    unset LFDAS_LIB
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
        > gpurun_out/final_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/final_pytest_gpu.log; exit 1; }
    tail -1 gpurun_out/final_pytest_gpu.log
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
    timeout -k 10 700 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
    tail -1 gpurun_out/final_bench.json ;;
  # ---- round 5 (lib_ab: old / new diagnostic libraries alternated in separate
  # processes; the old one built from the previous commit into tools/ab/old/lib)
  dp_pipe)  # fp64 MFMA vs VALU issue on one SIMD (profiles/r05_dp_pipe.txt)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/ubench_dp_pipe tools/ubench_dp_pipe.hip &&
    timeout -k 10 120 ./tools/ubench_dp_pipe ;;
  fr_lib_ab) # full-rate output pass, old vs new library (profiles/r05_fr_dpp_boundctrl.txt)
    ./tools/lib_ab.sh "$PWD/tools/ab/old/lib/liblfdas_diag.so" "$LFDAS_LIB" 3 -- python -u tools/fr_bench.py ;;
  fu_tailmap) # fused scan right-edge map and register budget (profiles/r05_scan_tailmap.txt)
    timeout -k 10 300 python -u tools/ab_plan.py --ch 1250 --reps 5 --replan "" "LFD_FU_TAILMAP=0" ;;
  mf_modes) # full-rate functionals diag modes (profiles/r05_mf_modes.txt)
    for m in 0 1 3 6; do LFD_MF_MODE=$m timeout -k 10 100 python -u tools/fr_bench.py || exit 1; done ;;
  copy_ceiling) # read + write ceiling for rolling S = 1 (profiles/r05_copy_ceiling.txt)
    timeout -k 10 120 python -u tools/copy_ceiling.py ;;
  rehearsal) # N = 2 on one device: strong-scaling headline + sharded cfg5 stream
    unset LFDAS_LIB
    timeout -k 10 400 python bench.py --gpus 2 --one-device --steps 3 --warmup 1 --no-cpu --no-rolling --no-extra ;;
  *) echo "recipes: k1 units scan offgrid tm_r02 rolling_r02 mfma tm tm_ubench narrow longscan rolling fir fir_pmc"
     echo "         fullrate lattice multi persist narrow_units scan_trace fr_mb fr_out fr_pmc lattice_pmc tm_wg"
     echo "         cm_wg fir_strip final rehearsal seg_scan odd_strides fr_scan_edges fir_xcd"
     echo "         dp_pipe fr_lib_ab fu_tailmap mf_modes copy_ceiling"; exit 2 ;;
esac
