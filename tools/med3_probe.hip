// med3_probe.hip — exhaustive GPU check that v_med3_f32(x, 0, 1), and a multiply's output clamp modifier, equal the
// build's GLSL clamp(x, 0, 1) (sail_math.h clamp_ = v_max_f32 then v_min_f32: a NaN operand yields the other,
// -0 < +0) for every f32 bit pattern. Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -Isail_amd/csrc tools/med3_probe.hip -o sail_amd/build/med3_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// the instructions themselves (inline asm), so that no compiler canonicalisation decides the comparison
__device__ __forceinline__ float maxmin01(float x) {  // what clamp_ lowers to in the trace kernels
  float t, r;
  __asm__ volatile("v_max_f32 %0, 0, %1" : "=v"(t) : "v"(x));
  __asm__ volatile("v_min_f32 %0, 1.0, %1" : "=v"(r) : "v"(t));
  return r;
}
__device__ __forceinline__ float med3_01(float x) {
  float r;
  __asm__ volatile("v_med3_f32 %0, %1, 0, 1.0" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ float maxminpm1(float x) {
  float t, r;
  __asm__ volatile("v_max_f32 %0, -1.0, %1" : "=v"(t) : "v"(x));
  __asm__ volatile("v_min_f32 %0, 1.0, %1" : "=v"(r) : "v"(t));
  return r;
}
__device__ __forceinline__ float med3_pm1(float x) {
  float r;
  __asm__ volatile("v_med3_f32 %0, %1, -1.0, 1.0" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ float mulclamp(float x, float y) {  // x * y with the output clamp modifier
  float r;
  __asm__ volatile("v_mul_f32_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ float mul(float x, float y) {
  float r;
  __asm__ volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

__global__ void probe(uint64_t base, unsigned long long* bad, uint32_t* firstBad, float scale) {
  const uint32_t bits = (uint32_t)(base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  const float x = __uint_as_float(bits);
  const float want0 = maxmin01(x), got0 = med3_01(x);
  const float want1 = maxmin01(mul(x, scale)), got1 = mulclamp(x, scale);
  if (__float_as_uint(got0) != __float_as_uint(want0)) { atomicAdd(&bad[0], 1ull); firstBad[0] = bits; }
  if (__float_as_uint(got1) != __float_as_uint(want1)) { atomicAdd(&bad[1], 1ull); firstBad[1] = bits; }
  if (__float_as_uint(med3_pm1(x)) != __float_as_uint(maxminpm1(x))) { atomicAdd(&bad[2], 1ull); firstBad[2] = bits; }
}

int main(int argc, char** argv) {
  unsigned long long* dBad; uint32_t* dFirst;
  if (hipMalloc(&dBad, 24) != hipSuccess || hipMalloc(&dFirst, 12) != hipSuccess) return 1;
  (void)hipMemset(dBad, 0, 24); (void)hipMemset(dFirst, 0, 12);
  const float scale = argc > 5 ? 2.0f : 1.0f;
  const uint64_t chunk = 1ull << 28;
  for (uint64_t base = 0; base < (1ull << 32); base += chunk)
    hipLaunchKernelGGL(probe, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, dBad, dFirst, scale);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  unsigned long long bad[3]; uint32_t first[3];
  (void)hipMemcpy(bad, dBad, 24, hipMemcpyDeviceToHost);
  (void)hipMemcpy(first, dFirst, 12, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"v_med3_f32(x,0,1) and v_mul_f32 clamp vs v_max_f32 + v_min_f32, all 2^32 x\", \"mismatches_median\": %llu, \"witness_median\": \"0x%08x\", "
         "\"mismatches_folded_into_multiply\": %llu, \"witness_folded\": \"0x%08x\", \"mismatches_median_minus1_1\": %llu, \"witness_pm1\": \"0x%08x\"}\n",
         bad[0], first[0], bad[1], first[1], bad[2], first[2]);
  return (bad[0] || bad[1] || bad[2]) ? 1 : 0;
}
