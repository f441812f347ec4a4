#!/bin/bash
# The round-5 variant comparisons (profiles/r05_*.jsonl), one named step each, run through gpurun:
#   bash tools/r05_variants.sh ns ...
# Each step: tools/variant_bench.py <scene> name=lib[:debug option=value,...] (two alternating rounds, bit-identity
# against the first variant checked), output under gpurun_out/r05v/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05v; mkdir -p $O
V=sail_amd/lib/variants
vb() {  # vb <out> <timeout> <scene> <specs...>
  local out=$1 t=$2; shift 2
  VARIANT_ROUNDS=${VARIANT_ROUNDS:-2} timeout -k 10 $t python -u tools/variant_bench.py "$@" > $O/$out.jsonl 2>&1 || { tail $O/$out.jsonl; exit 3; }
  cut -c1-170 $O/$out.jsonl
}
for step in "$@"; do
  echo "== $step"
  case $step in
    ns)  # samples of each pixel in flight per workgroup of the run-time kernels (SAIL_DEBUG_JIT_NS 11)
      for sc in C1 C3; do vb ns_$sc 400 $sc ns1=main:11=1 ns4=main:11=4 ns16=main:11=16; done
      VARIANT_SPP=64 vb ns_C4 600 C4 ns1=main:11=1 ns4=main:11=4 ns16=main:11=16 ;;
    ns_groups)  # the same with sample groups off (no stage at all)
      for sc in C1 C3; do vb nsg_$sc 400 $sc ns1g1=main:11=1,4=1 ns4g1=main:11=4,4=1 ns16g1=main:11=16,4=1; done ;;
    nt)  # threads per workgroup of the run-time kernels (SAIL_DEBUG_JIT_NT 12): the path sort's pool and barrier width
      vb nt_C1 400 C1 nt256=main nt128=main:12=128 nt512=main:12=512
      vb nt_C3 500 C3 nt256ns4=main:11=4 nt128ns4=main:12=128,11=4 nt512ns4=main:12=512,11=4 nt128=main:12=128
      VARIANT_SPP=64 vb nt_C4 600 C4 nt1024ns4=main:11=4 nt512ns4=main:12=512,11=4 nt512=main:12=512 ;;
    nt_c1)  # wider sort pools for the Cornell form, with samples in flight
      vb nt2_C1 500 C1 nt512=main:12=512 nt1024=main:12=1024 nt512ns4=main:12=512,11=4 nt1024ns4=main:12=1024,11=4 nt1024ns16=main:12=1024,11=16 ;;
    nt_c1b)  # the Cornell form at 512 threads with 1 / 4 / 16 samples in flight (16: no sample stage)
      vb nt3_C1 500 C1 nt512=main:12=512 nt512ns16=main:12=512,11=16 nt256ns16=main:11=16 nt256=main:12=256,11=1 ;;
    shdefer)  # the room form's shadow rays traced inside the next sort vs inside the shading (study build room_nodefer)
      for sc in C3 UI AREA; do vb shdefer_$sc 400 $sc defer=main nodefer=$V/libsail_hip_room_nodefer.so; done ;;
    launder)  # per-lane pixel values recomputed per sample step (working tree) vs kept from the start (HEAD build) vs
              # recomputed at the step's start only (study launder_start_only)
      for sc in C1 C3; do vb launder_$sc 400 $sc cur=main head=$V/libsail_hip_head.so start=$V/libsail_hip_launder_start_only.so; done
      VARIANT_SPP=64 vb launder_C4 600 C4 cur=main head=$V/libsail_hip_head.so start=$V/libsail_hip_launder_start_only.so ;;
    cornell)  # the Cornell form's sort: two barriers (study cornell_twobar), sorted first bounce (cornell_sort1); and
              # 128-sample launches
      vb cornell_C1 500 C1 cur=main twobar=$V/libsail_hip_cornell_twobar.so sort1=$V/libsail_hip_cornell_sort1.so
      VARIANT_LAUNCH=128 vb cornell_C1_l128 300 C1 cur128=main ;;
    groups)  # sample groups at the new workgroup shapes (SAIL_DEBUG_SAMPLE_GROUPS 4; default: sized by residency rounds)
      vb groups_C3 500 C3 auto=main g1=main:4=1 g4=main:4=4
      VARIANT_SPP=64 vb groups_C4 700 C4 auto=main g1=main:4=1 g4=main:4=4 ;;
    recheck)  # samples in flight / workgroup width of the room and pre-cull forms after the shadow-record rework
      vb recheck_C3 600 C3 ns4=main ns16=main:11=16 nt512ns4=main:12=512,11=4 nt512ns16=main:12=512,11=16 nt128ns4=main:12=128,11=4
      VARIANT_SPP=64 vb recheck_C4 700 C4 ns4=main ns1=main:11=1 ns16=main:11=16 nt512ns4=main:12=512,11=4 ;;
    sched)  # the run-time kernels under other LLVM machine-scheduler strategies (studies sched_*)
      for sc in C1 C3; do vb sched_$sc 500 $sc cur=main ilp=$V/libsail_hip_sched_ilp.so memclause=$V/libsail_hip_sched_memclause.so iterilp=$V/libsail_hip_sched_iterilp.so; done
      VARIANT_SPP=64 vb sched_C4 700 C4 cur=main ilp=$V/libsail_hip_sched_ilp.so memclause=$V/libsail_hip_sched_memclause.so iterilp=$V/libsail_hip_sched_iterilp.so ;;
    acclds)  # the Cornell form's running accumulator in LDS (working tree) against the HEAD build
      vb acclds_C1 400 C1 cur=main head=$V/libsail_hip_head.so
      vb acclds_C1b 400 C1 cur=main head=$V/libsail_hip_head.so ;;
    launch)  # samples per launch at 1,024 spp (working tree): fewer, longer-lived waves per frame
      for L in 64 128 256 1024; do VARIANT_SPP=1024 VARIANT_LAUNCH=$L vb launch_C1_$L 400 C1 cur=main; done
      for L in 64 256; do VARIANT_SPP=256 VARIANT_LAUNCH=$L vb launch_C3_$L 400 C3 cur=main; done ;;
    acclds_room)  # the room form's running accumulator in LDS (study acclds_room)
      for sc in C3 UI; do vb acclds_room_$sc 400 $sc cur=main room=$V/libsail_hip_acclds_room.so; done ;;
    twobar2)  # the Cornell form's two-barrier sort re-measured at whole-frame launches (study cornell_twobar)
      VARIANT_SPP=1024 VARIANT_LAUNCH=1024 vb twobar2_C1 500 C1 cur=main twobar=$V/libsail_hip_cornell_twobar.so ;;
    roomwaves)  # the room form's occupancy with 4 samples in flight (studies room_w8, room_w6)
      vb roomwaves_C3 500 C3 cur=main w8=$V/libsail_hip_room_w8.so w6=$V/libsail_hip_room_w6.so ;;
    sorthalf)  # the Cornell form sorting every other bounce (studies cornell_sort_even / _odd)
      VARIANT_SPP=1024 VARIANT_LAUNCH=1024 vb sorthalf_C1 500 C1 cur=main even=$V/libsail_hip_cornell_sort_even.so odd=$V/libsail_hip_cornell_sort_odd.so ;;
    boxface)  # the room form's first box row (Cube too) sorted by face (study room_box_face_key)
      for sc in C3 UI AREA; do vb boxface_$sc 400 $sc cur=main box=$V/libsail_hip_room_box_face_key.so; done ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "variants ok"
