// sail_jit.h — what one run-time compiled trace kernel pair is specialised to (sail_jit.cpp, used by sail_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

constexpr int kSailJitMaxRows = 8;  // scenes of at most this many rows can be compiled for their rows (flat path)
constexpr int kSailJitMaxFlatTp = 32;  // flat forms copy texParams tables of at most this many rows into LDS
struct SailJitSpec {
  uint32_t ks = 0, km = 0, kt = 0, kl = 0;  // plugin masks: shapes, materials, textures, lights
  int mode = 0;                             // sail_jit_mode (include/sail_hip.h): 0 flat, 1 pre-cull, 2 room family
  int waves = 6;                            // launch bounds: waves per SIMD
  int rows = 0;                             // > 0: the scene's row count, with each row's shape id in types
  int ldsFit = 0;                           // pre-cull: the scene's tables fit the LDS copies (SAIL_CULL_LDS_*)
  int tn = 0;                               // flat forms with rows: the texParams row count (LDS copies), 0 = none
  int types[kSailJitMaxRows] = {};
};
// the kernel pair for `spec` on `device` (the current device), compiled and loaded on first use
int sail_jit_kernels(int device, const SailJitSpec& spec, hipFunction_t* plain, hipFunction_t* grouped, std::string* err);
// host only: the code object for `arch`, compiled by the same path (sail_jit_compile)
int sail_jit_code(const char* arch, const SailJitSpec& spec, void* code, size_t* bytes, std::string* err);
