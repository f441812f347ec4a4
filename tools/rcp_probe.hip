// rcp_probe.hip — exhaustive GPU check of fast correctly-rounded f32 reciprocal sequences.
//
// The math spec defines GLSL division a / b as a * RN(1/b) (sail_math.h: fdiv). This probe runs every f32 bit
// pattern b through candidate device sequences for RN(1/b) and counts the ones whose result differs (bitwise;
// NaN == NaN) from the IEEE divide 1.0f / b. Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
// tools/rcp_probe.hip -o sail_amd/build/rcp_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define NV 5
__device__ __forceinline__ float rcp_v(int v, float b) {
  const float ab = fabsf(b);
  const bool inRange = ab >= 0x1p-126f && ab <= 0x1p126f;
  if (v == 0) {  // one f32 Newton step from the hardware reciprocal
    if (!inRange) return 1.0f / b;
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
  }
  if (v == 1) {  // two f32 Newton steps
    if (!inRange) return 1.0f / b;
    float y = __builtin_amdgcn_rcpf(b);
    float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    e = __builtin_fmaf(-b, y, 1.0f);
    return __builtin_fmaf(e, y, y);
  }
  if (v == 2) {  // f32 Newton step, then the residual-corrected rounding of Markstein's reciprocal
    if (!inRange) return 1.0f / b;
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    const float y1 = __builtin_fmaf(e, y0, y0);
    const float e1 = __builtin_fmaf(-b, y1, 1.0f);
    return __builtin_fmaf(e1, y1, y1);
  }
  if (v == 4) return __builtin_amdgcn_rcpf(b);  // control: the bare hardware reciprocal (must mismatch)
  // v == 3: f64 reciprocal (hardware f32 seed + two f64 Newton steps) rounded once to f32
  if (!(ab >= 0x1p-120f && ab <= 0x1p120f)) return 1.0f / b;
  const double bd = (double)b;
  double r = (double)__builtin_amdgcn_rcpf(b);
  double e = __builtin_fma(-bd, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-bd, r, 1.0);
  return (float)__builtin_fma(r, e, r);
}

__global__ void probe(uint64_t base, unsigned long long* bad, uint32_t* firstBad) {
  const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t bits = (uint32_t)i;
  const float b = __uint_as_float(bits);
  const float want = 1.0f / b;
  for (int v = 0; v < NV; v++) {
    const float got = rcp_v(v, b);
    const bool same = (__float_as_uint(got) == __float_as_uint(want)) || (got != got && want != want);
    if (!same) {
      atomicAdd(&bad[v], 1ull);
      firstBad[v] = bits;  // any one witness
    }
  }
}

int main() {
  unsigned long long* dBad; uint32_t* dFirst;
  hipMalloc(&dBad, NV * sizeof(unsigned long long));
  hipMalloc(&dFirst, NV * sizeof(uint32_t));
  hipMemset(dBad, 0, NV * sizeof(unsigned long long));
  hipMemset(dFirst, 0, NV * sizeof(uint32_t));
  const uint64_t chunk = 1ull << 28;
  for (uint64_t base = 0; base < (1ull << 32); base += chunk)
    hipLaunchKernelGGL(probe, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, dBad, dFirst);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  unsigned long long bad[NV]; uint32_t first[NV];
  hipMemcpy(bad, dBad, sizeof bad, hipMemcpyDeviceToHost);
  hipMemcpy(first, dFirst, sizeof first, hipMemcpyDeviceToHost);
  const char* names[NV] = {"rcp+1 f32 Newton", "rcp+2 f32 Newton", "rcp+Newton+residual", "f64 2-Newton rounded", "control: bare v_rcp_f32"};
  for (int v = 0; v < NV; v++)
    printf("{\"variant\": \"%s\", \"mismatches\": %llu, \"witness_bits\": \"0x%08x\"}\n", names[v], bad[v], first[v]);
  return 0;
}
