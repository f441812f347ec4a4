set -o pipefail
O=gpurun_out/s14; mkdir -p $O
V=sail_amd/lib/variants
VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py C1 base=main c2w7=$V/libsail_hip_jit_c2w7.so c2room=$V/libsail_hip_jit_c2room.so > $O/var_c1.jsonl 2>&1 || { tail $O/var_c1.jsonl; exit 3; }
cut -c1-150 $O/var_c1.jsonl
VARIANT_ROUNDS=2 timeout -k 10 400 python -u tools/variant_bench.py C3 base=main c3w6=$V/libsail_hip_jit_c3w6.so c3w8=$V/libsail_hip_jit_c3w8.so > $O/var_c3.jsonl 2>&1 || { tail $O/var_c3.jsonl; exit 4; }
cut -c1-150 $O/var_c3.jsonl
