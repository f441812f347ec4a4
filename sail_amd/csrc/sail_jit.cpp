// sail_jit.cpp — per-plugin-set trace kernels compiled at run time with hipRTC.
//
// The reference compiles one GLSL program per scene: Scene.tracerConfig() lists the plugins the scene uses
// (src/scene/scene.js:70-112), Generator.generate assembles exactly those functions (src/shader/generator.js:107-123)
// and Shader.combinefs links the result (src/core/shader.js:58-76), inside Renderer.update (src/core/renderer.js:45-52),
// in milliseconds. This build precompiles kernels for two plugin sets (the Cornell box, rooms of boxes / spheres /
// rectangles) and the all-plugin one; a scene gets a kernel compiled for exactly its plugin set (and rows) here, from the
// same sail_trace.hip (embedded in the library at build time, sail_jit_src.cpp), with the product's floating-point flags.
//
// A hipRTC compile takes seconds, so it never runs on the caller's thread: the first request for a spec starts a
// background build, and until its module is loaded the context launches the precompiled kernel of the scene's set (the
// frames are bit-identical either way; tests/test_gpu_parity.py renders across the swap). Code objects are kept
//  * per process, per (arch, spec); modules per (device, spec);
//  * on disk, keyed by (arch, spec, the embedded sources' hash, the compile flags, the compiler's version): the user's
//    cache ($XDG_CACHE_HOME or $HOME/.cache, sail_amd/jit; sail_set_jit_cache) and a read-only cache shipped next to the
//    library (sail_amd/lib/jit, filled at build time for the frozen scenes by sail_jit_prebuild).
//
// The compiler is the ROCm toolchain's own hipRTC (and the comgr it loads), opened in a link namespace of its own
// (dlmopen): a process that loaded another HIP runtime first -- PyTorch ships hipRTC and comgr of an older ROCm under
// the same sonames -- would otherwise compile with that one, and the kernels would differ from the precompiled ones
// (tests/test_jit_compile.py checks instruction identity after importing torch). A code object produced by another
// compiler than the one this library was built with is refused (sameCompiler; the precompiled kernels serve).
#include <ctype.h>
#include <dlfcn.h>
#include <pthread.h>
#include <errno.h>
#include <hip/hip_runtime.h>
#include <hip/hip_version.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "sail_jit.h"

extern const char* const sail_jit_src_names[];
extern const char* const sail_jit_src_texts[];
extern const int sail_jit_src_count;
extern const int sail_trace_phase_timing;  // sail_trace.hip: 1 in the phase-timing build (libsail_hip_phase.so)

int sailJitThreads(const SailJitSpec& s) { return s.nt ? s.nt : (s.mode == 1 ? 1024 : 256); }
bool sailJitSpecEqual(const SailJitSpec& a, const SailJitSpec& b) {
  const auto t = [](const SailJitSpec& x) {
    return std::tie(x.ks, x.km, x.kt, x.kl, x.mode, x.waves, x.rows, x.ldsFit, x.tn, x.ns, x.nt, x.types[0], x.types[1], x.types[2],
                    x.types[3], x.types[4], x.types[5], x.types[6], x.types[7]);
  };
  return t(a) == t(b);
}

namespace {

struct Key {
  SailJitSpec s;
  bool operator<(const Key& o) const {
    const auto t = [](const SailJitSpec& x) {
      return std::tie(x.ks, x.km, x.kt, x.kl, x.mode, x.waves, x.rows, x.ldsFit, x.tn, x.ns, x.nt, x.types[0], x.types[1], x.types[2],
                      x.types[3], x.types[4], x.types[5], x.types[6], x.types[7]);
    };
    return t(s) < t(o.s);
  }
};

uint64_t fnv(const void* p, size_t n, uint64_t h = 14695981039346656037ull) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}
uint64_t fnvStr(const std::string& s, uint64_t h) { return fnv(s.data(), s.size() + 1, h); }  // with the terminator
std::string hex16(uint64_t v) {
  char b[17];
  snprintf(b, sizeof b, "%016llx", (unsigned long long)v);
  return b;
}

// the embedded kernel sources (names and texts), hashed once
uint64_t sourceHash() {
  static const uint64_t h = [] {
    uint64_t x = fnv("sail-jit-src", 12);
    for (int i = 0; i < sail_jit_src_count; i++) { x = fnvStr(sail_jit_src_names[i], x); x = fnvStr(sail_jit_src_texts[i], x); }
    return x;
  }();
  return h;
}

// the same floating-point contract as sail_amd/build.sh: no contraction, no fast math, no SLP packing
const char* const kOpts[] = {"-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-mllvm", "-vectorize-slp=false"};

std::string defsFor(const SailJitSpec& sp) {
  std::string types;
  for (int i = 0; i < sp.rows; i++) types += (i ? ", " : "") + std::to_string(sp.types[i]);
  char defs[768];
  snprintf(defs, sizeof defs,
           "#define SAIL_JIT 1\n#define SAIL_JIT_WAVES %d\n#define SAIL_JIT_CULL %d\n#define SAIL_JIT_FAM %d\n"
           "#define SAIL_JIT_KS 0x%xu\n#define SAIL_JIT_KM 0x%xu\n#define SAIL_JIT_KT 0x%xu\n#define SAIL_JIT_KL 0x%xu\n"
           "#define SAIL_JIT_NT %d\n#define SAIL_JIT_N %d\n#define SAIL_JIT_TYPES %s\n#define SAIL_JIT_LDSFIT %d\n"
           "#define SAIL_JIT_TN %d\n#define SAIL_JIT_NS %d\n#include \"sail_trace.hip\"\n",
           sp.waves, sp.mode == 1, sp.mode == 2, sp.ks, sp.km, sp.kt, sp.kl, sailJitThreads(sp), sp.rows,
           sp.rows ? types.c_str() : "0", sp.ldsFit, sp.tn, sp.ns);
  // the phase-timing build compiles its run-time kernels instrumented as well (their own g_sailPhase)
  return sail_trace_phase_timing ? std::string("#define SAIL_PHASE_TIMING 1\n") + defs : std::string(defs);
}

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
  decltype(&hiprtcVersion) version;
  int major = 0, minor = 0;
};

void waitInFlight();  // atexit: waits for the build that is running, drops the queued ones (below)

const Rtc* rtc(std::string& err) {
  static Rtc r;
  static std::string why;
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] {
    std::string path;
    if (const char* e = getenv("SAIL_HIPRTC")) path = e;
    else path = std::string(getenv("ROCM_PATH") ? getenv("ROCM_PATH") : "/opt/rocm") + "/lib/libhiprtc.so.7";
    void* h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* d = dlerror();
      why = "dlmopen " + path + ": " + (d ? d : "?");
      return;
    }
    atexit(waitInFlight);
    r.create = (decltype(r.create))dlsym(h, "hiprtcCreateProgram");
    r.compile = (decltype(r.compile))dlsym(h, "hiprtcCompileProgram");
    r.logSize = (decltype(r.logSize))dlsym(h, "hiprtcGetProgramLogSize");
    r.log = (decltype(r.log))dlsym(h, "hiprtcGetProgramLog");
    r.codeSize = (decltype(r.codeSize))dlsym(h, "hiprtcGetCodeSize");
    r.code = (decltype(r.code))dlsym(h, "hiprtcGetCode");
    r.destroy = (decltype(r.destroy))dlsym(h, "hiprtcDestroyProgram");
    r.errStr = (decltype(r.errStr))dlsym(h, "hiprtcGetErrorString");
    r.version = (decltype(r.version))dlsym(h, "hiprtcVersion");
    if (!(r.create && r.compile && r.logSize && r.log && r.codeSize && r.code && r.destroy && r.errStr && r.version)) {
      why = path + ": missing hipRTC entry points";
      return;
    }
    if (r.version(&r.major, &r.minor) != HIPRTC_SUCCESS) { why = path + ": hiprtcVersion failed"; return; }
    ok = true;
  });
  if (!ok) { err = why; return nullptr; }
  return &r;
}

// ---- on-disk code-object caches -------------------------------------------------------------------------------------
std::mutex g_cacheMutex;
bool g_cacheDirSet = false;
std::string g_cacheDir;
std::string userCacheDir() {
  std::lock_guard<std::mutex> lk(g_cacheMutex);
  if (g_cacheDirSet) return g_cacheDir;
  if (const char* x = getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/sail_amd/jit";
  if (const char* h = getenv("HOME"); h && *h) return std::string(h) + "/.cache/sail_amd/jit";
  return "";
}
// the read-only cache shipped beside the library: <dir of libsail_hip.so>/jit
std::string shippedCacheDir() {
  static const std::string d = [] {
    Dl_info info;
    if (!dladdr(reinterpret_cast<void*>(&sourceHash), &info) || !info.dli_fname) return std::string();
    std::string p = info.dli_fname;
    const size_t s = p.rfind('/');
    return s == std::string::npos ? std::string("jit") : p.substr(0, s) + "/jit";
  }();
  return d;
}
void mkdirs(const std::string& dir) {
  for (size_t i = 1; i <= dir.size(); i++)
    if (i == dir.size() || dir[i] == '/') (void)mkdir(dir.substr(0, i).c_str(), 0755);
}
// (arch, spec, flags, embedded sources, the compiler that built this library -- which is the only producer a code
// object may come from, sameCompiler): no hipRTC is needed to look a code object up
uint64_t cacheKey(const std::string& arch, const Key& k) {
  uint64_t h = fnvStr("sailjit-v2", 14695981039346656037ull);
  h = fnvStr(arch, h);
  h = fnvStr(defsFor(k.s), h);
  for (const char* o : kOpts) h = fnvStr(o, h);
  h = fnvStr(hex16(sourceHash()), h);
  h = fnvStr(__clang_version__, h);
  return h;
}
constexpr char kMagic[8] = {'S', 'A', 'I', 'L', 'J', 'I', 'T', '1'};
bool cacheRead(const std::string& dir, uint64_t key, std::vector<char>& code) {
  if (dir.empty()) return false;
  FILE* f = fopen((dir + "/" + hex16(key) + ".co").c_str(), "rb");
  if (!f) return false;
  char magic[8];
  uint64_t hdr[3];  // key, payload size, payload hash
  bool ok = fread(magic, 1, 8, f) == 8 && fread(hdr, 8, 3, f) == 3 && std::equal(magic, magic + 8, kMagic) &&
            hdr[0] == key && hdr[1] > 0 && hdr[1] < (64u << 20);
  if (ok) {
    code.resize(hdr[1]);
    ok = fread(code.data(), 1, code.size(), f) == code.size() && fnv(code.data(), code.size()) == hdr[2];
  }
  fclose(f);
  if (!ok) code.clear();
  return ok;
}
void cacheWrite(const std::string& dir, uint64_t key, const std::vector<char>& code) {
  if (dir.empty() || code.empty()) return;
  mkdirs(dir);
  const std::string fin = dir + "/" + hex16(key) + ".co";
  const std::string tmp = fin + "." + std::to_string((long)getpid()) + "." +
                          std::to_string((unsigned long long)std::hash<std::thread::id>()(std::this_thread::get_id())) + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t hdr[3] = {key, (uint64_t)code.size(), fnv(code.data(), code.size())};
  const bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(hdr, 8, 3, f) == 3 && fwrite(code.data(), 1, code.size(), f) == code.size();
  if (fclose(f) == 0 && ok && rename(tmp.c_str(), fin.c_str()) == 0) return;  // atomic: readers see all of it or none
  (void)unlink(tmp.c_str());
}

// The compiler that produced a code object, from its .comment section ("AMD clang version <__clang_version__>"). The
// run-time kernels must come from the compiler that built this library's precompiled kernels -- their results equal the
// precompiled kernels' only as long as the code generator is the same -- so any other producer is refused (the
// precompiled kernels then serve). hiprtcVersion() is an API version (9.0 for ROCm 7.2 and its predecessors alike) and
// cannot tell compilers apart.
std::string producerOf(const std::vector<char>& code) {
  static const char tag[] = "AMD clang version ";
  const auto it = std::search(code.begin(), code.end(), tag, tag + sizeof tag - 1);
  if (it == code.end()) return "";
  const auto end = std::find(it, code.end(), '\0');
  return std::string(it + (sizeof tag - 1), end);
}
bool sameCompiler(const std::vector<char>& code, std::string& err) {
  const std::string prod = producerOf(code), mine = __clang_version__;
  // __clang_version__ may carry a trailing space
  const std::string m = mine.substr(0, mine.find_last_not_of(' ') + 1);
  if (!m.empty() && prod.compare(0, m.size(), m) == 0) return true;
  err = "the code object was produced by clang '" + prod + "', this library's kernels by '" + m + "'";
  return false;
}

// one hipRTC compile at a time (the compiler's thread safety is not relied on). On the heap: a fork child replaces it
// (forkChild), since the parent's build worker may hold it at the fork and does not exist in the child.
std::mutex* g_compileMutex = new std::mutex;
int compile(const Rtc& R, const std::string& arch, const Key& k, std::vector<char>& code, std::string& err) {
  std::lock_guard<std::mutex> lk(*g_compileMutex);
  const std::string defs = defsFor(k.s);
  hiprtcProgram prog;
  hiprtcResult r = R.create(&prog, defs.c_str(), "sail_jit.hip", sail_jit_src_count, sail_jit_src_texts, sail_jit_src_names);
  if (r != HIPRTC_SUCCESS) { err = R.errStr(r); return -1; }
  const std::string archOpt = "--offload-arch=" + arch;
  std::vector<const char*> opts{archOpt.c_str()};
  for (const char* o : kOpts) opts.push_back(o);
  r = R.compile(prog, (int)opts.size(), opts.data());
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    R.logSize(prog, &n);
    std::string log(n, '\0');
    if (n) R.log(prog, &log[0]);
    err = std::string(R.errStr(r)) + ": " + log.substr(0, 2000);
    R.destroy(&prog);
    return -1;
  }
  size_t n = 0;
  R.codeSize(prog, &n);
  code.resize(n);
  R.code(prog, code.data());
  R.destroy(&prog);
  if (!n) { err = "hipRTC returned an empty code object"; return -1; }
  return 0;
}

bool validSpec(const SailJitSpec& sp, std::string* err) {
  bool ok = sp.mode >= 0 && sp.mode <= 2 && sp.waves >= 1 && sp.waves <= 8 && sp.rows >= 0 && sp.rows <= kSailJitMaxRows &&
            !(sp.mode == 1 && sp.rows) &&  // the pre-cull kernels sweep candidates, not rows
            (sp.ldsFit == 0 || (sp.ldsFit == 1 && sp.mode == 1)) &&
            (sp.tn == 0 || (sp.tn >= 1 && sp.tn <= kSailJitMaxFlatTp && sp.mode != 1 && sp.rows > 0)) &&
            (sp.ns == 1 || sp.ns == 4 || sp.ns == 16) &&
            (sp.nt == 0 || sp.nt == 128 || sp.nt == 256 || sp.nt == 512 || sp.nt == 1024) && sailJitThreads(sp) / sp.ns >= 16;
  for (int i = 0; ok && i < sp.rows; i++) ok = sp.types[i] >= 1 && sp.types[i] <= 9 && ((sp.ks >> sp.types[i]) & 1u);
  if (!ok) *err = "invalid kernel specialisation";
  return ok;
}

// ---- code objects: one entry per (arch, spec), built once on a background thread ------------------------------------
struct Entry {
  std::mutex m;
  std::condition_variable cv;
  int state = 0;  // 0 building, 1 ready, 2 failed
  std::vector<char> code;
  std::string err;
  uint64_t id = 0;
  double compileMs = 0.0;
  int fromCache = 0;
  bool pinned = false;  // a host-only request waits for it: built even when no context holds the spec (g_mapMutex)
};
std::mutex g_mapMutex;
std::map<std::pair<std::string, Key>, std::shared_ptr<Entry>> g_code;
// Contexts' claims on specs (sail_jit_hold), under g_mapMutex: the build worker skips a queued build of a context's spec
// that no context holds any more (refreshJit replaced it), so a scene's current kernel does not wait behind stale builds.
std::map<std::pair<std::string, Key>, int> g_holds;

// The build identity of a code object: FNV-1a 64 over the sections that hold what runs -- the instructions (.text), the
// kernel descriptors (.rodata), the code-object metadata (.note: registers, LDS, launch bounds) and any initialised
// data -- each with its name. The symbol, string and hash tables are left out: they carry the compilation-unit id the
// compiler derives from the source text (`__hip_cuid_<hex>`), so an edit that changes no instruction (a comment, code
// compiled out of this kernel) keeps the id, and any change to what runs changes it. Not an ELF: the whole image.
uint64_t codeId(const std::vector<char>& code) {
  const unsigned char* b = reinterpret_cast<const unsigned char*>(code.data());
  const size_t n = code.size();
  auto u16 = [&](size_t o) { return o + 2 <= n ? (uint64_t)b[o] | (uint64_t)b[o + 1] << 8 : 0; };
  auto u32 = [&](size_t o) { return o + 4 <= n ? u16(o) | u16(o + 2) << 16 : 0; };
  auto u64 = [&](size_t o) { return o + 8 <= n ? u32(o) | u32(o + 4) << 32 : 0; };
  if (n < 64 || memcmp(b, "\177ELF", 4) != 0 || b[4] != 2) return fnv(code.data(), n);  // ELF64 only
  const uint64_t shoff = u64(0x28), shentsize = u16(0x3a), shnum = u16(0x3c), shstrndx = u16(0x3e);
  if (shentsize < 64 || shstrndx >= shnum || shoff + shnum * shentsize > n) return fnv(code.data(), n);
  const uint64_t strOff = u64(shoff + shstrndx * shentsize + 0x18), strSize = u64(shoff + shstrndx * shentsize + 0x20);
  if (strOff + strSize > n) return fnv(code.data(), n);
  uint64_t h = fnv("sail-code", 9);
  for (uint64_t k = 0; k < shnum; k++) {
    const size_t e = shoff + k * shentsize;
    const uint64_t nameOff = u32(e), type = u32(e + 4), off = u64(e + 0x18), size = u64(e + 0x20);
    if (nameOff >= strSize) continue;
    const char* name = reinterpret_cast<const char*>(b + strOff + nameOff);
    const size_t nameLen = strnlen(name, strSize - nameOff);
    const std::string nm(name, nameLen);
    if (nm != ".text" && nm != ".rodata" && nm != ".note" && nm != ".data") continue;
    h = fnvStr(nm, h);
    if (type != 8 /* SHT_NOBITS */ && off + size <= n) h = fnv(b + off, size, h);
  }
  return h;
}
void finish(Entry& e, std::vector<char>& code, const std::string& err, double ms, int from) {
  {
    std::lock_guard<std::mutex> lk(e.m);
    if (!code.empty()) {
      e.id = codeId(code);
      e.code.swap(code);
      e.compileMs = ms;
      e.fromCache = from;
      e.state = 1;
    } else {
      e.err = err.empty() ? "code object build failed" : err;
      e.state = 2;
    }
  }
  e.cv.notify_all();
}
// A code object from the disk caches (the shipped one first), checked: 2 shipped, 1 user, 0 none
int cacheLookup(uint64_t key, std::vector<char>& code) {
  std::string err;
  if (cacheRead(shippedCacheDir(), key, code) && sameCompiler(code, err)) return 2;
  if (cacheRead(userCacheDir(), key, code) && sameCompiler(code, err)) return 1;
  code.clear();
  return 0;
}
// the background build: hipRTC, then the user cache (and extraDir: sail_jit_code_to_dir)
void buildEntry(const std::shared_ptr<Entry>& e, const std::string& arch, const Key& k, const std::string& extraDir) {
  std::vector<char> code;
  std::string err;
  double ms = 0.0;
  const uint64_t key = cacheKey(arch, k);
  if (const Rtc* R = rtc(err)) {
    const auto t0 = std::chrono::steady_clock::now();
    if (compile(*R, arch, k, code, err) == 0 && sameCompiler(code, err)) {
      ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      err.clear();
      cacheWrite(userCacheDir(), key, code);
      if (!extraDir.empty()) cacheWrite(extraDir, key, code);
    } else {
      code.clear();
    }
  }
  finish(*e, code, err, ms, 0);
}

struct BuildJob { std::shared_ptr<Entry> e; std::string arch; Key k; std::string extraDir; };

// Whether a queued job is still wanted when the worker reaches it: a host-only request (pinned: sail_jit_code, prebuild)
// always is; a context's only while some context holds its spec. An unwanted entry leaves the map (a later request for
// the spec starts afresh) and fails with a message no caller sees: nobody holds it, so nobody waits on it.
bool stillWanted(const BuildJob& j) {
  std::lock_guard<std::mutex> lk(g_mapMutex);
  if (j.e->pinned) return true;
  const auto h = g_holds.find({j.arch, j.k});
  if (h != g_holds.end() && h->second > 0) return true;
  const auto it = g_code.find({j.arch, j.k});
  if (it != g_code.end() && it->second == j.e) g_code.erase(it);
  return false;
}

// One build worker for the process, fed by a queue: every compile runs on that same thread, one at a time. (A thread
// per build crashed hipRTC: the second pre-cull-form compile of a process, on a new thread after the first one's had
// exited, faulted inside the compiler -- reproduced on the CPU, whatever the stack limit. One long-lived thread is how
// the synchronous round-4 path used it: always from one thread.) Its stack is large and explicit (256 MB of address
// space, committed as used): the compiler recurses deeply on the big kernels, and under an "unlimited" stack limit
// glibc would give a new thread only 2 MB.
// `running` counts the job the worker has taken (0 or 1): at exit (waitInFlight) the process waits for that compile
// alone -- exiting inside the compiler would run its static destructors under it -- and drops the queued ones.
// The queue outlives static destruction (never freed): the worker still waits on its condition variable while the
// process exits, and destroying a condition variable that has a waiter blocks. A fork child gets a fresh queue
// (forkChild): the parent's worker thread does not exist there.
struct BuildQueue {
  std::mutex m;
  std::condition_variable cv, idle;
  std::vector<BuildJob*> jobs;
  bool workerUp = false;
  bool exiting = false;
  int running = 0;
};
BuildQueue* g_queue = new BuildQueue;
void dropJob(BuildJob* j, const char* why) {
  std::vector<char> none;
  finish(*j->e, none, why, 0.0, 0);
  delete j;
}
void* buildWorker(void* arg) {
  BuildQueue& q = *static_cast<BuildQueue*>(arg);
  for (;;) {
    BuildJob* j;
    {
      std::unique_lock<std::mutex> lk(q.m);
      q.cv.wait(lk, [&] { return !q.jobs.empty() || q.exiting; });
      if (q.exiting) { q.idle.notify_all(); return nullptr; }
      j = q.jobs.front();
      q.jobs.erase(q.jobs.begin());
      q.running++;
    }
    if (stillWanted(*j)) {
      buildEntry(j->e, j->arch, j->k, j->extraDir);
      delete j;
    } else {
      dropJob(j, "build dropped: no context holds this kernel any more");
    }
    {
      std::lock_guard<std::mutex> lk(q.m);
      q.running--;
    }
    q.idle.notify_all();
  }
}
// fork: the child has no build worker, and the parent's may hold the queue, map or compile locks at the fork. The prepare
// handler takes the queue and map locks (the fork happens between jobs' bookkeeping, not inside it); the child gets a
// fresh queue and compile lock, and forgets the entries still being built in the parent (their jobs ran there), so a
// request in the child builds them afresh. (A compile the parent's worker was running inside hipRTC at the fork may
// leave the compiler's own state inconsistent in the child; its next compile then fails and the precompiled kernels
// serve.)
void forkPrepare() { g_queue->m.lock(); g_mapMutex.lock(); }
void forkParent() { g_mapMutex.unlock(); g_queue->m.unlock(); }
void forkChild() {
  g_queue = new BuildQueue;  // the parent's (locked, with its jobs) is abandoned
  g_compileMutex = new std::mutex;
  for (auto it = g_code.begin(); it != g_code.end();) {
    std::lock_guard<std::mutex> lk(it->second->m);
    if (it->second->state == 0) it = g_code.erase(it);
    else ++it;
  }
  g_mapMutex.unlock();
}
bool enqueue(BuildJob* job) {
  static std::once_flag atforkOnce;
  std::call_once(atforkOnce, [] { pthread_atfork(forkPrepare, forkParent, forkChild); });
  BuildQueue& q = *g_queue;
  std::lock_guard<std::mutex> lk(q.m);
  if (q.exiting) return false;
  if (!q.workerUp) {
    pthread_attr_t attr;
    pthread_t tid;
    if (pthread_attr_init(&attr) != 0) return false;
    const bool ok = pthread_attr_setstacksize(&attr, (size_t)256 << 20) == 0 &&
                    pthread_attr_setdetachstate(&attr, PTHREAD_CREATE_DETACHED) == 0 &&
                    pthread_create(&tid, &attr, buildWorker, &q) == 0;
    pthread_attr_destroy(&attr);
    if (!ok) return false;
    q.workerUp = true;
  }
  q.jobs.push_back(job);
  q.cv.notify_one();
  return true;
}

// The entry of (arch, spec). At the first request a code object in a disk cache is read here, on the caller's thread
// (a file read: the warm path of Renderer.update stays in milliseconds), outside the map lock -- other contexts' launches
// look their kernels up under it; a concurrent request for the same spec finds the entry pending and waits on it --
// otherwise its build is queued for the background worker. pinned: a host-only caller that waits for the build.
std::shared_ptr<Entry> request(const std::string& arch, const Key& k, bool pinned, const std::string& extraDir = std::string()) {
  std::shared_ptr<Entry> e;
  {
    std::lock_guard<std::mutex> lk(g_mapMutex);
    auto& slot = g_code[{arch, k}];
    if (slot) {  // built, being built, or failed (a failed spec is not retried in this process)
      if (pinned) slot->pinned = true;
      return slot;
    }
    slot = std::make_shared<Entry>();
    slot->pinned = pinned;
    e = slot;
  }
  std::vector<char> code;
  const uint64_t key = cacheKey(arch, k);
  if (getenv("SAIL_JIT_DEFS"))  // tooling (tools/isa.sh): the source prefix of this spec, to rebuild it with hipcc
    fprintf(stderr, "sail_jit %s %s\n%s", arch.c_str(), hex16(key).c_str(), defsFor(k.s).c_str());
  if (const int from = cacheLookup(key, code)) {
    if (!extraDir.empty()) cacheWrite(extraDir, key, code);
    finish(*e, code, "", 0.0, from);
    return e;
  }
  auto* job = new BuildJob{e, arch, k, extraDir};
  if (!enqueue(job)) {  // no worker thread (or the process is exiting): build here
    buildEntry(job->e, job->arch, job->k, job->extraDir);
    delete job;
  }
  return e;
}
// atexit (registered once the compiler library is loaded: handlers run in reverse order, so this one runs before that
// library's destructors): wait for the compile the worker is running, drop the queued ones (their entries fail)
void waitInFlight() {
  BuildQueue& q = *g_queue;
  std::vector<BuildJob*> dropped;
  {
    std::unique_lock<std::mutex> lk(q.m);
    q.exiting = true;
    dropped.swap(q.jobs);
    q.cv.notify_all();
    q.idle.wait(lk, [&] { return q.running == 0; });
  }
  for (BuildJob* j : dropped) dropJob(j, "build dropped: the process is exiting");
}
// wait_ms < 0: until the build is done
int await(Entry& e, int wait_ms) {
  std::unique_lock<std::mutex> lk(e.m);
  if (e.state == 0 && wait_ms != 0) {
    if (wait_ms < 0) e.cv.wait(lk, [&] { return e.state != 0; });
    else e.cv.wait_for(lk, std::chrono::milliseconds(wait_ms), [&] { return e.state != 0; });
  }
  return e.state;
}

struct Loaded { hipModule_t mod; SailJitKernel k; };
std::mutex g_loadMutex;
std::map<std::pair<int, Key>, Loaded> g_loaded;  // (device, spec) -> module
std::mutex g_archMutex;
std::map<int, std::string> g_arch;  // device -> "gfx950"
int deviceArch(int device, std::string& arch, std::string* err) {
  std::lock_guard<std::mutex> lk(g_archMutex);
  auto it = g_arch.find(device);
  if (it == g_arch.end()) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { *err = "hipGetDeviceProperties"; return -1; }
    std::string a = prop.gcnArchName;
    const size_t colon = a.find(':');  // "gfx950:sramecc+:xnack-": the features follow the device
    if (colon != std::string::npos) a = a.substr(0, colon);
    it = g_arch.emplace(device, a).first;
  }
  arch = it->second;
  return 0;
}
}  // namespace

int sail_jit_kernels(int device, const SailJitSpec& spec, int wait_ms, SailJitKernel* out, std::string* err) {
  if (!validSpec(spec, err)) return -1;
  const Key k{spec};
  {
    std::lock_guard<std::mutex> lk(g_loadMutex);
    auto it = g_loaded.find({device, k});
    if (it != g_loaded.end()) { *out = it->second.k; return 0; }
  }
  std::string arch;
  if (deviceArch(device, arch, err)) return -1;
  std::shared_ptr<Entry> e = request(arch, k, false);
  const int st = await(*e, wait_ms);
  if (st == 0) return 1;
  if (st == 2) { *err = e->err; return -1; }
  std::lock_guard<std::mutex> lk(g_loadMutex);
  auto it = g_loaded.find({device, k});
  if (it == g_loaded.end()) {
    if (hipSetDevice(device) != hipSuccess) { *err = "hipSetDevice"; return -1; }  // the module loads on this device
    Loaded L{};
    if (hipModuleLoadData(&L.mod, e->code.data()) != hipSuccess) { *err = "hipModuleLoadData"; return -1; }
    const char* fn = spec.mode == 1 ? "sail_trace_kernel_cull_jit" : "sail_trace_kernel_jit";
    if (hipModuleGetFunction(&L.k.plain, L.mod, fn) != hipSuccess ||
        hipModuleGetFunction(&L.k.grouped, L.mod, (std::string(fn) + "_grouped").c_str()) != hipSuccess) {
      (void)hipModuleUnload(L.mod);
      *err = "hipModuleGetFunction";
      return -1;
    }
    L.k.buildId = e->id;
    L.k.compileMs = e->compileMs;
    L.k.fromCache = e->fromCache;
    it = g_loaded.emplace(std::make_pair(device, k), L).first;
  }
  *out = it->second.k;
  return 0;
}

// Host-only: the code object of `spec`'s kernel pair for `arch`, built (not loaded) by the same path
// (include/sail_hip.h sail_jit_compile). *bytes = its size; copied into `code` when `code` is not null and the
// buffer (*bytes on entry) is large enough.
int sail_jit_code(const char* arch, const SailJitSpec& spec, void* code, size_t* bytes, std::string* err) {
  if (!validSpec(spec, err)) return -1;
  std::shared_ptr<Entry> e = request(arch, Key{spec}, true);
  if (await(*e, -1) != 1) { *err = e->err; return -1; }
  const size_t have = *bytes;
  *bytes = e->code.size();
  if (code) {
    if (have < e->code.size()) { *err = "buffer too small"; return -1; }
    std::copy(e->code.begin(), e->code.end(), static_cast<char*>(code));
  }
  return 0;
}

int sail_jit_code_to_dir(const char* arch, const SailJitSpec& spec, const char* dir, std::string* err) {
  if (!validSpec(spec, err)) return -1;
  std::shared_ptr<Entry> e = request(arch, Key{spec}, true, dir && *dir ? std::string(dir) : std::string());
  if (await(*e, -1) != 1) { *err = e->err; return -1; }
  if (dir && *dir) {  // an entry made earlier in this process wrote only the user cache: write this directory too
    std::vector<char> have;
    const uint64_t key = cacheKey(arch, Key{spec});
    if (!cacheRead(dir, key, have)) cacheWrite(dir, key, e->code);
  }
  return 0;
}

void sail_jit_hold(int device, const SailJitSpec& spec, int delta) {
  std::string arch, err;
  if (deviceArch(device, arch, &err)) return;
  std::lock_guard<std::mutex> lk(g_mapMutex);
  const auto key = std::make_pair(arch, Key{spec});
  int& h = g_holds[key];
  h += delta;
  if (h <= 0) g_holds.erase(key);
}

void sail_jit_set_cache_dir(const char* dir) {
  std::lock_guard<std::mutex> lk(g_cacheMutex);
  g_cacheDirSet = dir != nullptr;
  g_cacheDir = dir ? dir : "";
}

uint64_t sail_precompiled_build_id(const char* kernel) {
  static const uint64_t lib = [] {
    Dl_info info;
    uint64_t h = fnv("sail-lib", 8);
    if (!dladdr(reinterpret_cast<void*>(&sourceHash), &info) || !info.dli_fname) return h;
    FILE* f = fopen(info.dli_fname, "rb");
    if (!f) return h;
    std::vector<char> buf(1 << 16);
    size_t n;
    while ((n = fread(buf.data(), 1, buf.size(), f)) > 0) h = fnv(buf.data(), n, h);
    fclose(f);
    return h;
  }();
  return fnvStr(kernel, lib);
}

// The phase-timing build: the per-phase sums of every loaded run-time module, added to out (reset: zeroed)
int sail_jit_phase_read(unsigned long long out[12], int reset) {
  std::lock_guard<std::mutex> lk(g_loadMutex);
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  int rc = 0;
  for (auto& kv : g_loaded) {
    hipDeviceptr_t p = nullptr;
    size_t bytes = 0;
    if (hipSetDevice(kv.first.first) != hipSuccess) { rc = -1; break; }
    if (hipModuleGetGlobal(&p, &bytes, kv.second.mod, "g_sailPhase") != hipSuccess || bytes < 12 * sizeof(unsigned long long))
      continue;  // not instrumented
    unsigned long long v[12];
    if (hipMemcpyDtoH(v, p, sizeof v) != hipSuccess) { rc = -1; break; }
    for (int q = 0; q < 12; q++) out[q] += v[q];
    if (reset && hipMemsetD8(p, 0, sizeof v) != hipSuccess) { rc = -1; break; }
  }
  (void)hipSetDevice(cur);  // the caller's current device
  return rc;
}
