// Wave64 inclusive prefix sum by DPP on gfx9-family lanes: Hillis-Steele within each row of 16 lanes (row_shr 1, 2,
// 4, 8; lanes shifted in from outside the row read 0), then the row totals across rows (row_bcast 15 adds lane 15 to
// row 1 and lane 47 to row 3; row_bcast 31 adds lane 31 to rows 2 and 3). Six VALU, no LDS round trips
// (tools/dpp_scan_probe.hip checks it against a serial scan on the GPU).
#pragma once
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#endif
__device__ __forceinline__ int waveScanIncl(int x) {
  int v = x;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31 -> rows 2, 3
  return v;
}
