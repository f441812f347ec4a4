set -o pipefail
O=gpurun_out/s5; mkdir -p $O
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py ALL base=main kset_all=sail_amd/lib/variants/libsail_hip_kset_all.so > $O/var_all.jsonl 2>&1 || { tail $O/var_all.jsonl; exit 2; }
VARIANT_ROUNDS=2 timeout -k 10 300 python -u tools/variant_bench.py AREA base=main kset_area=sail_amd/lib/variants/libsail_hip_kset_area.so > $O/var_area.jsonl 2>&1 || { tail $O/var_area.jsonl; exit 3; }
VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py C3 base=main room_sh7=sail_amd/lib/variants/libsail_hip_room_sh7.so room_sh6=sail_amd/lib/variants/libsail_hip_room_sh6.so room_w6=sail_amd/lib/variants/libsail_hip_room_w6.so > $O/var_c3.jsonl 2>&1 || { tail $O/var_c3.jsonl; exit 4; }
cut -c1-170 $O/var_all.jsonl $O/var_area.jsonl $O/var_c3.jsonl
