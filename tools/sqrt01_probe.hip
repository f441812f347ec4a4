// sqrt01_probe.hip — exhaustive GPU check of sail_math.h sqrt01 and sqrtg (v_sqrt_f32 + two-neighbour residual correction,
// no scaling / class fix-ups) against the compiler's IEEE sqrtf lowering on its whole domain: both zeros, every f32
// in [2^-96, 1] and every NaN bit pattern (and, reported apart, the excluded (0, 2^-96)). Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -Isail_amd/csrc tools/sqrt01_probe.hip -o sail_amd/build/sqrt01_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "sail_math.h"

__global__ void probe(uint64_t base, uint64_t end, unsigned long long* bad, unsigned long long* tested, uint32_t* firstBad) {
  // bad[0]: mismatches on the domain, bad[1]: mismatches on the excluded (0, 2^-96)
  const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= end) return;
  const uint32_t bits = (uint32_t)i;
  const float x = __uint_as_float(bits);
  if (!((x >= 0.0f && x <= 1.0f) || x != x)) return;
  const bool excluded = x > 0.0f && x < 0x1p-96f;  // never an argument (sail_math.h sqrt01)
  const float want = __builtin_sqrtf(x), got = sm::sqrt01(x);
  const bool same = (__float_as_uint(got) == __float_as_uint(want)) || (got != got && want != want);
  if (!same) { atomicAdd(&bad[excluded ? 1 : 0], 1ull); if (!excluded) *firstBad = bits; }
  if ((threadIdx.x & 63) == 0) atomicAdd(tested, 1ull);
}
// sail_math.h sqrtg (the general square root) against the IEEE lowering on EVERY f32 bit pattern: bad[2] counts
// mismatches of the correction core on its fast domain (>= 2^-96, +inf, +-0, NaN), bad[3] of sqrtg overall
__global__ void probeAll(uint64_t base, uint64_t end, unsigned long long* bad, uint32_t* firstBad) {
  const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= end) return;
  const uint32_t bits = (uint32_t)i;
  const float x = __uint_as_float(bits);
  const float want = __builtin_sqrtf(x);
  const bool fast = !(x < 0x1p-96f && x != 0.0f);
  if (fast) {
    const float core = sm::sqrt01(x);
    if (!((__float_as_uint(core) == __float_as_uint(want)) || (core != core && want != want))) {
      atomicAdd(&bad[2], 1ull); firstBad[1] = bits;
    }
  }
  const float got = sm::sqrtg(x);
  if (!((__float_as_uint(got) == __float_as_uint(want)) || (got != got && want != want))) {
    atomicAdd(&bad[3], 1ull); firstBad[2] = bits;
  }
}

int main() {
  unsigned long long *dBad, *dTested; uint32_t* dFirst;
  if (hipMalloc(&dBad, 32) != hipSuccess || hipMalloc(&dTested, 8) != hipSuccess || hipMalloc(&dFirst, 12) != hipSuccess) return 1;
  (void)hipMemset(dBad, 0, 32); (void)hipMemset(dTested, 0, 8); (void)hipMemset(dFirst, 0, 12);
  const uint64_t chunk = 1ull << 28;
  for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
    hipLaunchKernelGGL(probe, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, base + chunk, dBad, dTested, dFirst);
    hipLaunchKernelGGL(probeAll, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, base + chunk, dBad, dFirst);
  }
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  unsigned long long bad[4], tested; uint32_t first[3];
  (void)hipMemcpy(bad, dBad, 32, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&tested, dTested, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(first, dFirst, 12, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"sqrt01 vs IEEE sqrtf on {+-0} u [2^-96, 1] u NaN\", \"mismatches\": %llu, \"witness_bits\": \"0x%08x\", "
         "\"mismatches_excluded_0_to_2^-96\": %llu, \"waves_tested\": %llu, "
         "\"core_mismatches_on_fast_domain_all_2^32\": %llu, \"core_witness\": \"0x%08x\", "
         "\"sqrtg_mismatches_all_2^32\": %llu, \"sqrtg_witness\": \"0x%08x\"}\n",
         bad[0], first[0], bad[1], tested, bad[2], first[1], bad[3], first[2]);
  return (bad[0] | bad[2] | bad[3]) != 0;
}
