// sqrt_probe.hip — exhaustive GPU check of short correctly-rounded f32 sqrt sequences against the compiler's
// IEEE sqrtf lowering (all 2^32 inputs; NaN == NaN). Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
// tools/sqrt_probe.hip -o sail_amd/build/sqrt_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define NV 3
__device__ __forceinline__ float sq_v(int v, float x) {
  const bool inRange = x >= 0x1p-96f && x < 0x1p127f;  // positive normal range without the compiler's scaling
  if (!inRange) return __builtin_sqrtf(x);
  const float s = __builtin_amdgcn_sqrtf(x);
  if (v == 0) return s;  // bare hardware square root
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
  if (v == 1) {  // both-neighbour residual correction (the compiler's sequence without scaling / class fixups)
    float r = s;
    if (__builtin_fmaf(-sdn, s, x) <= 0.0f) r = sdn;
    if (__builtin_fmaf(-sup, s, x) > 0.0f) r = sup;
    return r;
  }
  // v == 2: one residual, one direction choice: e = x - s*s decides between s and the neighbour on e's side
  const float e = __builtin_fmaf(-s, s, x);
  const float h = e > 0.0f ? sup : sdn;  // candidate neighbour
  const float m = 0.5f * (s + h);        // not exact: only a probe
  return (__builtin_fabsf(__builtin_fmaf(-h, h, x)) < __builtin_fabsf(e)) ? h : (m == m ? s : s);
}

__global__ void probe(uint64_t base, unsigned long long* bad, uint32_t* firstBad) {
  const uint32_t bits = (uint32_t)(base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  const float x = __uint_as_float(bits);
  const float want = __builtin_sqrtf(x);
  for (int v = 0; v < NV; v++) {
    const float got = sq_v(v, x);
    const bool same = (__float_as_uint(got) == __float_as_uint(want)) || (got != got && want != want);
    if (!same) { atomicAdd(&bad[v], 1ull); firstBad[v] = bits; }
  }
}

int main() {
  unsigned long long* dBad; uint32_t* dFirst;
  if (hipMalloc(&dBad, NV * sizeof(unsigned long long)) != hipSuccess) return 1;
  if (hipMalloc(&dFirst, NV * sizeof(uint32_t)) != hipSuccess) return 1;
  (void)hipMemset(dBad, 0, NV * sizeof(unsigned long long));
  (void)hipMemset(dFirst, 0, NV * sizeof(uint32_t));
  const uint64_t chunk = 1ull << 28;
  for (uint64_t base = 0; base < (1ull << 32); base += chunk)
    hipLaunchKernelGGL(probe, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, dBad, dFirst);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  unsigned long long bad[NV]; uint32_t first[NV];
  (void)hipMemcpy(bad, dBad, sizeof bad, hipMemcpyDeviceToHost);
  (void)hipMemcpy(first, dFirst, sizeof first, hipMemcpyDeviceToHost);
  const char* names[NV] = {"bare v_sqrt_f32", "two-neighbour residual", "one-residual probe"};
  for (int v = 0; v < NV; v++)
    printf("{\"variant\": \"%s\", \"mismatches\": %llu, \"witness_bits\": \"0x%08x\"}\n", names[v], bad[v], first[v]);
  return 0;
}
