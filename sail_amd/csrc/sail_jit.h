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
  int ns = 1;                               // samples of each pixel in flight per workgroup (1, 4, 16: traceTileCompact)
  int nt = 0;                               // threads per workgroup (128 .. 1,024); 0 = the form's own (1,024 pre-cull, 256)
  int types[kSailJitMaxRows] = {};
};
bool sailJitSpecEqual(const SailJitSpec& a, const SailJitSpec& b);
int sailJitThreads(const SailJitSpec& s);  // threads per workgroup of the spec's kernels

// A loaded kernel pair and where its code object came from.
struct SailJitKernel {
  hipFunction_t plain = nullptr, grouped = nullptr;
  uint64_t buildId = 0;     // FNV-1a 64 of the code object, its compilation-unit id masked (sail_jit.cpp codeId)
  double compileMs = 0.0;   // hipRTC time of the code object (0 when it came from a disk cache)
  int fromCache = 0;        // 1: the user's on-disk cache, 2: the cache shipped next to the library
};
// The kernel pair for `spec` on `device` (made current). The code object is built on a background thread at the first
// request (disk caches first, then hipRTC), outside every lock the launch path takes. Returns 0 with the loaded pair;
// 1 while the code object is still being built and wait_ms allows no more waiting (wait_ms < 0: wait until it is done);
// -1 with a message when it cannot be built or loaded (the caller then runs the precompiled kernel, same results).
int sail_jit_kernels(int device, const SailJitSpec& spec, int wait_ms, SailJitKernel* out, std::string* err);
// A context's claim on the kernel of `spec` on `device` (delta +1 when it adopts the spec, -1 when it drops it): a queued
// build of a spec no context holds any more is skipped by the build worker, so the scene's current kernel never waits
// behind builds of specs that a newer scene, partition or switch replaced.
void sail_jit_hold(int device, const SailJitSpec& spec, int delta);
// host only: the code object for `arch`, built by the same path (sail_jit_compile, sail_jit_prebuild); blocks
int sail_jit_code(const char* arch, const SailJitSpec& spec, void* code, size_t* bytes, std::string* err);
// the on-disk code-object cache directory: nullptr = the default ($XDG_CACHE_HOME or $HOME/.cache, /sail_amd/jit),
// "" = none (sail_set_jit_cache); `dir` of sail_jit_code / prebuild when it is not null
void sail_jit_set_cache_dir(const char* dir);
int sail_jit_code_to_dir(const char* arch, const SailJitSpec& spec, const char* dir, std::string* err);
// FNV-1a 64 of the library image plus a precompiled kernel's name: the build identity of a precompiled kernel
uint64_t sail_precompiled_build_id(const char* kernel);
