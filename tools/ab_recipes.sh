# GPU-box recipes behind the round-2 A/B records in profiles/ (each step is
# time-limited; run one at a time through gpurun).  In-process A/Bs compare
# env knobs on ONE input allocation (tools/ab_plan.py), because K1's speed
# depends on the physical placement of a fresh 72 GB tensor.
set -o pipefail
mkdir -p gpurun_out
case "$1" in
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
  tm)      # time-major K1 loads / MFMA shape (profiles/r02_ab_tm.txt)
    timeout -k 10 400 python tools/ab_plan.py --tm --reps 3 "" "LFD_TM_BUF=0" "LFD_TM_X2=0" "LFD_TM_M4=1" \
        "LFD_TM_NT=768 LFD_TM_PF=1" ;;
  rolling) # rolling-mean scan kernel (profiles/r02_ab_roll_ring.txt)
    for S in 1 250; do
      timeout -k 10 200 python tools/ab_roll_env.py $S "" "LFD_ROLL_RING=0" "LFD_ROLL_DPP=0" || exit 1
    done ;;
  mfma)    # fp64 MFMA issue rates and the 4x4x4 operand layout
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/ub tools/ubench_mfma64b.hip &&
    timeout -k 5 60 /tmp/ub &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/c4 tools/check_mfma4x4.hip &&
    timeout -k 5 30 /tmp/c4 ;;
  *) echo "usage: bash tools/ab_recipes.sh k1|units|scan|offgrid|tm|rolling|mfma"; exit 2 ;;
esac
