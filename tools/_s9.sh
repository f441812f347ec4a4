set -o pipefail
O=gpurun_out/s9; mkdir -p $O
V=sail_amd/lib/variants
VARIANT_ROUNDS=2 timeout -k 10 500 python -u tools/variant_bench.py C4 base=main cw7=$V/libsail_hip_jit_cw7.so cw6=$V/libsail_hip_jit_cw6.so c512w6=$V/libsail_hip_jit_c512w6.so > $O/var_c4_occ.jsonl 2>&1 || { tail $O/var_c4_occ.jsonl; exit 3; }
cut -c1-150 $O/var_c4_occ.jsonl
for sc in ALL AREA; do
  VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py $sc base=main rw8=$V/libsail_hip_jit_rw8.so rw6=$V/libsail_hip_jit_rw6.so > $O/var_occ_$sc.jsonl 2>&1 || { tail $O/var_occ_$sc.jsonl; exit 4; }
  cut -c1-150 $O/var_occ_$sc.jsonl
done
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py C1 base=main c1_struct=$V/libsail_hip_c1_struct.so > $O/var_c1_struct.jsonl 2>&1 || { tail $O/var_c1_struct.jsonl; exit 6; }
cut -c1-150 $O/var_c1_struct.jsonl
for r in 1 2; do for cfg in C2 C3; do for l in 32 64; do
  timeout -k 10 300 python bench.py --config $cfg --launch-spp $l --no-cpu-baseline --steps 3 --warmup 1 > $O/launch_${cfg}_${l}_${r}.json 2> $O/launch.err || { tail $O/launch.err; exit 5; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $O/launch_${cfg}_${l}_${r}.json $cfg $l | tee -a $O/launch.txt
done; done; done
OUT=s9 bash tools/session.sh scale phases
