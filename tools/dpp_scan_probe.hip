// Probe: the wave64 inclusive prefix sum by DPP (row_shr 1/2/4/8 within rows of 16, then row_bcast 15 / 31 across
// rows) that the trace kernels' path sort can use (SAIL_SCAN_DPP), checked against a serial scan on the host over
// many random waves. Prints one JSON line; exit status 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../sail_amd/csrc/sail_scan.h"

__global__ void scanKernel(const int* in, int* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int v = i < n ? in[i] : 0;
  const int r = waveScanIncl(v);
  if (i < n) out[i] = r;
}

int main() {
  const int waves = 1 << 16, n = waves * 64;
  std::vector<int> in(n), out(n);
  srand(7);
  for (int i = 0; i < n; i++) in[i] = (i % 5 == 0) ? 0 : (rand() % 2000) - ((i % 7 == 0) ? 1000 : 0);
  int *dIn, *dOut;
  if (hipMalloc(&dIn, n * sizeof(int)) || hipMalloc(&dOut, n * sizeof(int))) return 2;
  hipMemcpy(dIn, in.data(), n * sizeof(int), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(scanKernel, dim3(n / 256), dim3(256), 0, 0, dIn, dOut, n);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipMemcpy(out.data(), dOut, n * sizeof(int), hipMemcpyDeviceToHost);
  long bad = 0;
  for (int w = 0; w < waves; w++) {
    int acc = 0;
    for (int l = 0; l < 64; l++) { acc += in[w * 64 + l]; if (out[w * 64 + l] != acc) bad++; }
  }
  printf("{\"probe\": \"dpp_wave_scan\", \"waves\": %d, \"mismatches\": %ld}\n", waves, bad);
  hipFree(dIn); hipFree(dOut);
  return bad ? 1 : 0;
}
