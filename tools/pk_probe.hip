// pk_probe.hip — issue-rate probe of packed f32 VALU on gfx950: the same number of f32 FMAs / multiplies / adds
// as plain v_fma_f32 / v_mul_f32 / v_add_f32 or as packed v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (inline asm,
// 8 independent chains per lane, 8 waves per SIMD), timed with HIP events. Settles whether packing the trace
// kernels' f32 arithmetic could double its issue rate ("No SLP vectorisation"). Build:
//   hipcc -O3 --offload-arch=gfx950 tools/pk_probe.hip -o sail_amd/build/pk_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

#define PLAIN(op, x, b, c) __asm__ volatile(op " %0, %1, %2" : "+v"(x) : "v"(b), "v"(c))
#define PLAIN3(op, x, b, c) __asm__ volatile(op " %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c))

// clk[0..1]: shader-clock cycles (s_memtime) and 100 MHz ticks (s_memrealtime) spent by workgroup 0's first wave:
// their ratio is the engine clock the chip actually ran at under this load
template <int MODE>
__global__ void __launch_bounds__(256) probe(float* out, int iters, unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const float s = (float)threadIdx.x * 1e-3f;
  f2 p[8];
  float q[16];
  for (int j = 0; j < 8; j++) { p[j] = f2{s + j, s - j}; q[2 * j] = s + j; q[2 * j + 1] = s - j; }
  const f2 b2 = {1.0000001f, 0.9999999f}, c2 = {1e-9f, 2e-9f};
  const float b = 1.0000001f, c = 1e-9f;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (MODE == 0) { PLAIN3("v_fma_f32", q[2 * j], b, c); PLAIN3("v_fma_f32", q[2 * j + 1], b, c); }
      if (MODE == 1) __asm__ volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[j]) : "v"(b2), "v"(c2));
      if (MODE == 2) { PLAIN("v_mul_f32", q[2 * j], q[2 * j], b); PLAIN("v_mul_f32", q[2 * j + 1], q[2 * j + 1], b); }
      if (MODE == 3) __asm__ volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[j]) : "v"(b2));
      if (MODE == 4) { PLAIN("v_add_f32", q[2 * j], q[2 * j], c); PLAIN("v_add_f32", q[2 * j + 1], q[2 * j + 1], c); }
      if (MODE == 5) __asm__ volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[j]) : "v"(c2));
    }
  }
  float acc = 0.0f;
  for (int j = 0; j < 8; j++) acc += p[j].x + p[j].y + q[2 * j] + q[2 * j + 1];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main() {
  const int blocks = 256 * 4 * 8 / 4 * 4;  // 8 waves per SIMD on 256 CUs, 4 rounds
  const int iters = 4096;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipMalloc(&clk, 2 * sizeof(unsigned long long));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[6] = {"v_fma_f32 x2", "v_pk_fma_f32", "v_mul_f32 x2", "v_pk_mul_f32", "v_add_f32 x2", "v_pk_add_f32"};
  void (*ks[6])(float*, int, unsigned long long*) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>};
  double ms[6], ghz[6];
  for (int m = 0; m < 6; m++) {
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, 16, clk);  // warm-up
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t; hipEventElapsedTime(&t, e0, e1);
    ms[m] = t;
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    ghz[m] = (double)h[0] / (double)h[1] * 0.1;  // s_memrealtime ticks at 100 MHz
  }
  // f32 operations per launch: blocks * 256 lanes * iters * 16 (either as 16 plain or 8 packed instructions)
  const double ops = (double)blocks * 256 * iters * 16;
  printf("{\"probe\": \"packed vs plain f32 VALU issue, 8 independent chains per lane, %d workgroups of 256\"", blocks);
  for (int m = 0; m < 6; m++)
    printf(", \"%s_ms\": %.3f, \"%s_Gop_per_s\": %.1f, \"%s_clock_GHz\": %.3f, \"%s_wave_instr_per_SIMD_cycle\": %.3f", names[m], ms[m],
           names[m], ops / ms[m] / 1e6, names[m], ghz[m], names[m],
           ops / 64.0 / ((m & 1) ? 2.0 : 1.0) / 1024.0 / (ms[m] * 1e-3 * ghz[m] * 1e9));
  printf(", \"pk_fma_speedup\": %.3f, \"pk_mul_speedup\": %.3f, \"pk_add_speedup\": %.3f}\n", ms[0] / ms[1], ms[2] / ms[3], ms[4] / ms[5]);
  hipFree(out);
  return 0;
}
