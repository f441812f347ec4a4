// sail_jit.cpp — per-plugin-set trace kernels compiled at run time with hipRTC.
//
// The reference compiles one GLSL program per scene: Scene.tracerConfig() lists the plugins the scene uses
// (src/scene/scene.js:70-112), Generator.generate assembles exactly those functions (src/shader/generator.js:107-123)
// and Shader.combinefs links the result (src/core/shader.js:58-76). This build precompiles kernels for two plugin sets
// (the Cornell box, rooms of boxes / spheres / rectangles) and the all-plugin one; other scenes can get a kernel
// compiled for exactly their plugin set here, from the same sail_trace.hip (embedded in the library at build time,
// sail_jit_src.cpp), with the product's floating-point flags. Measured (profiles/r04_jit_vs_generic.jsonl): ALL +4.1 %,
// AREA +6.1 %, BILERP +4.6 % over the all-plugin kernel, bit-identical. Code objects are cached per process and plugin
// set, modules per device.
//
// The compiler is the ROCm toolchain's own hipRTC (and the comgr it loads), opened in a link namespace of its own
// (dlmopen): a process that loaded another HIP runtime first -- PyTorch ships hipRTC and comgr of an older ROCm under
// the same sonames -- would otherwise compile with that one, and the kernels would differ from the precompiled ones
// (tests/test_jit_compile.py checks instruction identity after importing torch).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "sail_jit.h"

extern const char* const sail_jit_src_names[];
extern const char* const sail_jit_src_texts[];
extern const int sail_jit_src_count;

namespace {

struct Key {
  SailJitSpec s;
  bool operator<(const Key& o) const {
    const auto t = [](const SailJitSpec& x) {
      return std::tie(x.ks, x.km, x.kt, x.kl, x.mode, x.waves, x.rows, x.ldsFit, x.tn, x.types[0], x.types[1], x.types[2],
                      x.types[3], x.types[4], x.types[5], x.types[6], x.types[7]);
    };
    return t(s) < t(o.s);
  }
};
std::mutex g_jitMutex;
std::map<std::pair<std::string, Key>, std::vector<char>> g_code;  // (arch, spec) -> code object
struct Loaded { hipModule_t mod; hipFunction_t plain, grouped; };
std::map<std::pair<int, Key>, Loaded> g_loaded;                  // (device, spec) -> module

// hipRTC entry points from the toolchain's library (SAIL_HIPRTC, else $ROCM_PATH or /opt/rocm, lib/libhiprtc.so.7)
struct Rtc {
  decltype(&hiprtcCreateProgram) create;
  decltype(&hiprtcCompileProgram) compile;
  decltype(&hiprtcGetProgramLogSize) logSize;
  decltype(&hiprtcGetProgramLog) log;
  decltype(&hiprtcGetCodeSize) codeSize;
  decltype(&hiprtcGetCode) code;
  decltype(&hiprtcDestroyProgram) destroy;
  decltype(&hiprtcGetErrorString) errStr;
};
const Rtc* rtc(std::string& err) {  // under g_jitMutex
  static Rtc r;
  static bool tried = false, ok = false;
  static std::string why;
  if (!tried) {
    tried = true;
    std::string path;
    if (const char* e = getenv("SAIL_HIPRTC")) path = e;
    else path = std::string(getenv("ROCM_PATH") ? getenv("ROCM_PATH") : "/opt/rocm") + "/lib/libhiprtc.so.7";
    void* h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* d = dlerror();
      why = "dlmopen " + path + ": " + (d ? d : "?");
    } else {
      r.create = (decltype(r.create))dlsym(h, "hiprtcCreateProgram");
      r.compile = (decltype(r.compile))dlsym(h, "hiprtcCompileProgram");
      r.logSize = (decltype(r.logSize))dlsym(h, "hiprtcGetProgramLogSize");
      r.log = (decltype(r.log))dlsym(h, "hiprtcGetProgramLog");
      r.codeSize = (decltype(r.codeSize))dlsym(h, "hiprtcGetCodeSize");
      r.code = (decltype(r.code))dlsym(h, "hiprtcGetCode");
      r.destroy = (decltype(r.destroy))dlsym(h, "hiprtcDestroyProgram");
      r.errStr = (decltype(r.errStr))dlsym(h, "hiprtcGetErrorString");
      ok = r.create && r.compile && r.logSize && r.log && r.codeSize && r.code && r.destroy && r.errStr;
      if (!ok) why = path + ": missing hipRTC entry points";
    }
  }
  if (!ok) { err = why; return nullptr; }
  return &r;
}

// the same floating-point contract as sail_amd/build.sh: no contraction, no fast math, no SLP packing
int compile(const std::string& arch, const Key& k, std::vector<char>& code, std::string& err) {
  const SailJitSpec& sp = k.s;
  std::string types;
  for (int i = 0; i < sp.rows; i++) types += (i ? ", " : "") + std::to_string(sp.types[i]);
  char defs[768];
  snprintf(defs, sizeof defs,
           "#define SAIL_JIT 1\n#define SAIL_JIT_WAVES %d\n#define SAIL_JIT_CULL %d\n#define SAIL_JIT_FAM %d\n"
           "#define SAIL_JIT_KS 0x%xu\n#define SAIL_JIT_KM 0x%xu\n#define SAIL_JIT_KT 0x%xu\n#define SAIL_JIT_KL 0x%xu\n"
           "#define SAIL_JIT_NT %d\n#define SAIL_JIT_N %d\n#define SAIL_JIT_TYPES %s\n#define SAIL_JIT_LDSFIT %d\n"
           "#define SAIL_JIT_TN %d\n#include \"sail_trace.hip\"\n",
           sp.waves, sp.mode == 1, sp.mode == 2, sp.ks, sp.km, sp.kt, sp.kl, sp.mode == 1 ? 1024 : 256, sp.rows,
           sp.rows ? types.c_str() : "0", sp.ldsFit, sp.tn);
  const Rtc* R = rtc(err);
  if (!R) return -1;
  hiprtcProgram prog;
  hiprtcResult r = R->create(&prog, defs, "sail_jit.hip", sail_jit_src_count, sail_jit_src_texts, sail_jit_src_names);
  if (r != HIPRTC_SUCCESS) { err = R->errStr(r); return -1; }
  const std::string archOpt = "--offload-arch=" + arch;
  const char* opts[] = {archOpt.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                        "-mllvm", "-vectorize-slp=false"};
  r = R->compile(prog, (int)(sizeof opts / sizeof opts[0]), opts);
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    R->logSize(prog, &n);
    std::string log(n, '\0');
    if (n) R->log(prog, &log[0]);
    err = std::string(R->errStr(r)) + ": " + log.substr(0, 2000);
    R->destroy(&prog);
    return -1;
  }
  size_t n = 0;
  R->codeSize(prog, &n);
  code.resize(n);
  R->code(prog, code.data());
  R->destroy(&prog);
  return n ? 0 : -1;
}

bool validSpec(const SailJitSpec& sp, std::string* err) {
  bool ok = sp.mode >= 0 && sp.mode <= 2 && sp.waves >= 1 && sp.waves <= 8 && sp.rows >= 0 && sp.rows <= kSailJitMaxRows &&
            !(sp.mode == 1 && sp.rows) &&  // the pre-cull kernels sweep candidates, not rows
            (sp.ldsFit == 0 || (sp.ldsFit == 1 && sp.mode == 1)) &&
            (sp.tn == 0 || (sp.tn >= 1 && sp.tn <= kSailJitMaxFlatTp && sp.mode != 1 && sp.rows > 0));
  for (int i = 0; ok && i < sp.rows; i++) ok = sp.types[i] >= 1 && sp.types[i] <= 9 && ((sp.ks >> sp.types[i]) & 1u);
  if (!ok) *err = "invalid kernel specialisation";
  return ok;
}
}  // namespace

// The trace kernel pair (ungrouped, _grouped) for `spec` on `device` (the current device), compiled on first use.
// Returns 0 and the functions, or -1 with a message (the caller then runs the precompiled kernel).
int sail_jit_kernels(int device, const SailJitSpec& spec, hipFunction_t* plain, hipFunction_t* grouped, std::string* err) {
  if (!validSpec(spec, err)) return -1;
  const Key k{spec};
  std::lock_guard<std::mutex> lock(g_jitMutex);
  auto it = g_loaded.find({device, k});
  if (it == g_loaded.end()) {
    if (hipSetDevice(device) != hipSuccess) { *err = "hipSetDevice"; return -1; }  // the module loads on this device
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { *err = "hipGetDeviceProperties"; return -1; }
    std::string arch = prop.gcnArchName;
    const size_t colon = arch.find(':');  // "gfx950:sramecc+:xnack-": the features follow the device
    if (colon != std::string::npos) arch = arch.substr(0, colon);
    auto& code = g_code[{arch, k}];
    if (code.empty() && compile(arch, k, code, *err)) { g_code.erase({arch, k}); return -1; }
    Loaded L{};
    if (hipModuleLoadData(&L.mod, code.data()) != hipSuccess) { *err = "hipModuleLoadData"; return -1; }
    const char* fn = spec.mode == 1 ? "sail_trace_kernel_cull_jit" : "sail_trace_kernel_jit";
    if (hipModuleGetFunction(&L.plain, L.mod, fn) != hipSuccess ||
        hipModuleGetFunction(&L.grouped, L.mod, (std::string(fn) + "_grouped").c_str()) != hipSuccess) {
      (void)hipModuleUnload(L.mod);
      *err = "hipModuleGetFunction";
      return -1;
    }
    it = g_loaded.emplace(std::make_pair(device, k), L).first;
  }
  *plain = it->second.plain;
  *grouped = it->second.grouped;
  return 0;
}

// Host-only: the code object of `spec`'s kernel pair for `arch`, compiled (not loaded) by the same path
// (include/sail_hip.h sail_jit_compile). *bytes = its size; copied into `code` when `code` is not null and the
// buffer (*bytes on entry) is large enough.
int sail_jit_code(const char* arch, const SailJitSpec& spec, void* code, size_t* bytes, std::string* err) {
  if (!validSpec(spec, err)) return -1;
  const Key k{spec};
  std::lock_guard<std::mutex> lock(g_jitMutex);
  auto& c = g_code[{arch, k}];
  if (c.empty() && compile(arch, k, c, *err)) { g_code.erase({arch, k}); return -1; }
  const size_t have = *bytes;
  *bytes = c.size();
  if (code) {
    if (have < c.size()) { *err = "buffer too small"; return -1; }
    std::copy(c.begin(), c.end(), static_cast<char*>(code));
  }
  return 0;
}
