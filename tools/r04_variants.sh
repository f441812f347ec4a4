#!/bin/bash
# The round-4 variant comparisons (profiles/r04_*.jsonl), one named step each, run through gpurun:
#   bash tools/r04_variants.sh jit_forms jit_rows ...
# Study libraries are built first on the CPU: tools/study_build.sh <name> (patches under tools/study/).
# Each step: tools/variant_bench.py <scene> name=lib[:debug option=value,...] (two alternating rounds, bit-identity
# against the first variant checked), output under gpurun_out/r04v/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04v; mkdir -p $O
V=sail_amd/lib/variants
vb() {  # vb <out> <timeout> <scene> <specs...>
  local out=$1 t=$2; shift 2
  VARIANT_ROUNDS=2 timeout -k 10 $t python -u tools/variant_bench.py "$@" > $O/$out.jsonl 2>&1 || { tail $O/$out.jsonl; exit 3; }
  cut -c1-160 $O/$out.jsonl
}
for step in "$@"; do
  echo "== $step"
  case $step in
    jit_forms)   # run-time kernels for the plugin set: all-plugin form vs room form; room-set and pre-cull scenes
      for sc in ALL AREA BILERP AREA0; do vb forms_$sc 300 $sc jit=main:9=1 jitroom=main:9=9; done
      vb forms_C3 300 C3 base=main:9=0 jit=main:9=5
      vb forms_C4 400 C4 base=main:9=0 jit=main:9=3 ;;
    jit_rows)    # compiled for the scene's rows too (bit 16)
      for sc in C1 C3 UI ALL AREA BILERP; do vb rows_$sc 300 $sc sets=main:9=11 rows=main:9=27; done ;;
    occupancy)   # launch bounds of the run-time forms (study builds jit_cw7 jit_cw6 jit_c512w6 jit_rw8 jit_rw6 jit_c2w7 jit_c3w6 jit_c3w8)
      vb occ_C4 500 C4 base=main cw7=$V/libsail_hip_jit_cw7.so cw6=$V/libsail_hip_jit_cw6.so c512w6=$V/libsail_hip_jit_c512w6.so
      vb occ_C1 400 C1 base=main c2w7=$V/libsail_hip_jit_c2w7.so c2room=$V/libsail_hip_jit_c2room.so
      vb occ_C3 400 C3 base=main c3w6=$V/libsail_hip_jit_c3w6.so c3w8=$V/libsail_hip_jit_c3w8.so ;;
    rounds)      # sample-group residency rounds (SAIL_DEBUG_GROUP_ROUNDS 7, _CULL_GROUP_ROUNDS 8)
      for sc in C1 C3; do vb rounds_$sc 400 $sc r36=main r18=main:7=18 r72=main:7=72; done
      vb rounds_C4 500 C4 r64=main r32=main:8=32 r128=main:8=128 ;;
    launch)      # samples per launch, whole-config bench lines
      for r in 1 2; do for cfg in C2 C3 C4; do for l in 32 64; do
        timeout -k 10 300 python bench.py --config $cfg --launch-spp $l --no-cpu-baseline --steps 1 --warmup 1 > $O/launch_${cfg}_${l}_$r.json 2> $O/launch.err || { tail $O/launch.err; exit 5; }
      done; done; done ;;
    live_state)  # fewer live VGPRs across the sample loop (study builds segs_scalar, acc_lds)
      for sc in C1 C3 UI ALL; do vb live_$sc 400 $sc base=main segs=$V/libsail_hip_segs_scalar.so acc=$V/libsail_hip_acc_lds.so; done
      vb live_C4 500 C4 base=main segs=$V/libsail_hip_segs_scalar.so ;;
    cull_stash)  # the pre-cull sweep without throughput / pixel in VGPRs (study build cull_stash)
      vb stash_C4 500 C4 base=main stash=$V/libsail_hip_cull_stash.so ;;
    skip_sort1)  # no path sort at the first bounce (study build skip_sort1)
      for sc in C1 C3 UI; do vb skip1_$sc 400 $sc base=main skip1=$V/libsail_hip_skip_sort1.so; done
      vb skip1_C4 500 C4 base=main skip1=$V/libsail_hip_skip_sort1.so ;;
    cull_unroll) # the pre-cull mask build unrolled by 4 rows (study build cull_unroll)
      vb unroll_C4 500 C4 base=main unroll=$V/libsail_hip_cull_unroll.so ;;
    cull_unroll8) # eight rows per step instead of four (study build cull_unroll8)
      vb unroll8_C4 500 C4 base=main unroll8=$V/libsail_hip_cull_unroll8.so ;;
    cull_ldsfit) # LDS scene tables unconditional: ds_read instead of flat loads (study build cull_ldsfit; C4 fits)
      vb ldsfit_C4 500 C4 base=main ldsfit=$V/libsail_hip_cull_ldsfit.so ;;
    flat_lds)    # typed LDS scene tables in the flat kernels (study build flat_lds; C1, C3, UI fit)
      for sc in C1 C3 UI; do vb flatlds_$sc 400 $sc base=main flatlds=$V/libsail_hip_flat_lds.so; done ;;
    cornell_tp)  # the Cornell form with only texParams in LDS (study build cornell_tp_lds)
      vb cornelltp_C1 400 C1 base=main tplds=$V/libsail_hip_cornell_tp_lds.so ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "variants ok"
