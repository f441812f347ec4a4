// sail_capi.cpp — libsail_hip.so: context, scene decode, launches, readback, filter, RCCL reduce.
// The C ABI is declared (with the reference interface each entry replaces) in include/sail_hip.h.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <math.h>
#include <algorithm>
#include <cmath>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../include/sail_hip.h"
#include "sail_device.h"

// launch wrappers defined next to the kernels (sail_trace.hip)
hipError_t sail_launch_trace(const SailTraceArgs& A, int blocks, hipStream_t s);
// sail_jit.cpp: the trace kernel pair compiled at run time for exactly one plugin set (on the current device)
#include "sail_jit.h"
hipError_t sail_launch_filter(const SailFilterArgs& A, hipStream_t s);
hipError_t sail_launch_accum(const SailTraceArgs& A, int blocks, hipStream_t s);
hipError_t sail_launch_math(int fn, const float* x, const float* y, float* out, int count);
hipError_t sail_launch_sum(const SailSumArgs& A, hipStream_t s);
hipError_t sail_launch_negzero_unowned(float4* a, float4* b, int W, int H, int rank, int world, hipStream_t s);
hipError_t sail_launch_wavefront(const SailTraceArgs& A, const SailWfState& S, hipStream_t s);
hipError_t sail_launch_pick(const SailPrim* prims, int n, const float* rays, int count, int32_t* index, float* t,
                            hipStream_t s);

namespace {

thread_local std::string g_create_error;

// ---- RCCL, bound at run time (the process may already hold torch's copy under the same soname) ----
typedef struct { char internal[128]; } nccl_uid_t;
typedef void* nccl_comm_t;
struct Rccl {
  bool tried = false, ok = false;
  int (*getUniqueId)(nccl_uid_t*) = nullptr;
  int (*commInitRank)(nccl_comm_t*, int, nccl_uid_t, int) = nullptr;
  int (*reduce)(const void*, void*, size_t, int, int, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*commDestroy)(nccl_comm_t) = nullptr;
  int (*commInitAll)(nccl_comm_t*, int, const int*) = nullptr;   // single-process multi-device communicator
  int (*groupStart)() = nullptr;
  int (*groupEnd)() = nullptr;
  int (*commGetAsyncError)(nccl_comm_t, int*) = nullptr;
  const char* (*errStr)(int) = nullptr;
  bool load() {
    if (tried) return ok;
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    getUniqueId = (int (*)(nccl_uid_t*))dlsym(h, "ncclGetUniqueId");
    commInitRank = (int (*)(nccl_comm_t*, int, nccl_uid_t, int))dlsym(h, "ncclCommInitRank");
    reduce = (int (*)(const void*, void*, size_t, int, int, int, nccl_comm_t, hipStream_t))dlsym(h, "ncclReduce");
    commDestroy = (int (*)(nccl_comm_t))dlsym(h, "ncclCommDestroy");
    errStr = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
    commInitAll = (int (*)(nccl_comm_t*, int, const int*))dlsym(h, "ncclCommInitAll");
    groupStart = (int (*)())dlsym(h, "ncclGroupStart");
    groupEnd = (int (*)())dlsym(h, "ncclGroupEnd");
    commGetAsyncError = (int (*)(nccl_comm_t, int*))dlsym(h, "ncclCommGetAsyncError");
    ok = getUniqueId && commInitRank && reduce && commDestroy && commInitAll && groupStart && groupEnd &&
         commGetAsyncError;
    return ok;
  }
};
Rccl g_rccl;
constexpr int kNcclFloat32 = 7, kNcclSum = 0;

// GLSL division on the host, for the shader expressions evaluated here once per scene or per sample: the math
// spec's a * RN(1/b) (sail_math.h fdiv, oracle/ref_math.h div_s); host f32 arithmetic is IEEE (no contraction)
float gdiv(float a, float b) { return a * (1.0f / b); }

// ---- the reference's texture addressing (texhelper.glsl, NEAREST + CLAMP_TO_EDGE) ----------------------
int texel(float c, int size) {
  if (c != c) return 0;  // NaN row coordinate (n = 1 / ln = 1: 0/0) addresses texel 0
  const float s = floorf(c * (float)size);
  if (!(s >= 0.0f)) return 0;
  if (s >= (float)(size - 1)) return size - 1;
  return (int)s;
}
int to_int(float x) {
  if (x != x) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}
struct TexView {
  const float* d; int w, h;
  float at(float cx, float cy) const {
    if (h <= 0) return 0.0f;
    return d[texel(cy, h) * w + texel(cx, w)];
  }
  float readFloat(float x, float y, float width) const { return at(gdiv(x, width), y); }
  void readVec3(float x, float y, float width, float* out) const {
    float px = gdiv(x, width);
    out[0] = at(px, y); px += gdiv(1.0f, width);
    out[1] = at(px, y); px += gdiv(1.0f, width);
    out[2] = at(px, y);
  }
};

}  // namespace

// union of the primitives' finite bounds and its diagonal (sceneBox)
struct SceneBox { double lo[3], hi[3]; double diag; };

struct sail_ctx {
  int device = 0, W = 0, H = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  float4* accum = nullptr;
  float4* aovN = nullptr;
  float4* aovP = nullptr;
  float4* filterOut = nullptr;    // display-filter outputs, allocated on first use
  uint8_t* filterOut8 = nullptr;
  unsigned long long* segCounter = nullptr;
  SailPrim* prims = nullptr;
  float* tp = nullptr;
  float* lt = nullptr;
  int32_t* lightObjRow = nullptr;
  SailSample* samples = nullptr;
  int samplesCap = 0;
  int samplesPos = 0;  // ring position: each launch sequence reads its own slice of the sample buffer
  SailSample* samplesPinned = nullptr;  // pinned host mirror of the ring (asynchronous uploads)
  std::vector<SailSample> hostSamples;
  std::vector<float> objectsRows;
  std::vector<float> tpRows;  // host copy of texParams (category words of updated objects)
  int n = 0, tn = 0, ln = 0;
  sail_plugins plugins{};
  bool haveScene = false;
  int shadowAnyHit = 0;
  std::vector<unsigned long long> typeMasksHost;  // staging for the per-chunk type masks (async copy source)
  int cullMinPrims = 8;  // scenes with at least this many primitives use the padded-box pre-cull
  int lastGroups = 1;         // the last trace launch: sample groups (sail_kernel_name)
  bool lastWavefront = false;
  int flatGroupRounds = 36;  // sample groups: residency rounds queued per launch (flat kernels, SAIL_DEBUG_GROUP_ROUNDS)
  int cullGroupRounds = 64;  // the same for the pre-cull kernel's 1,024-thread workgroups
  int cullFma = 1;       // SAIL_CULL_FMA=0: always the plain pre-cull form (tests)
  double primExtent = INFINITY;  // largest |padded bound| coordinate (inf: some primitive is unbounded)
  SceneBox scene{};              // union of the primitives' finite bounds (padPrimBounds)
  int forceGeneric = 0;  // SAIL_FORCE_GENERIC=1: always launch the all-plugin kernel (tests)
  int forceGroups = 0;   // SAIL_SAMPLE_GROUPS=g: fixed sample-group count (tests); 0 = by occupancy
  int wavefront = 0;     // SAIL_DEBUG_WAVEFRONT: the pre-cull path by the wavefront split (study)
  int jit = 27;  // SAIL_DEBUG_JIT bits: which scenes get a run-time kernel (jitKernels; instrumented in the phase build)
  // The scene's run-time kernel (refreshJit): its spec, and whether it is still being built, loaded or failed. Until it
  // is loaded the precompiled kernel of the scene's set serves (same results); a launch waits up to jitWait ms for it
  // (SAIL_DEBUG_JIT_WAIT; -1 until it is built).
  bool jitHave = false;
  SailJitSpec jitSpec;
  int jitMode = 0;
  int jitState = SAIL_KERNEL_JIT_NONE;
  SailJitKernel jitK;
  std::string jitError;  // why the scene's run-time kernel failed (sail_get_kernel_info)
  int jitWait = 0;
  int jitNt = 0;  // SAIL_DEBUG_JIT_NT: threads per workgroup of the run-time kernels (0: the form's own)
  int jitNs = 0;  // SAIL_DEBUG_JIT_NS: samples in flight of the run-time kernels (0: the form's default, jitNsFor)
  bool lastJit = false;  // the last trace launch ran a run-time compiled kernel (sail_kernel_name)
  int lastJitMode = 0;
  uint64_t lastBuildId = 0;  // the run-time kernel's build identity (sail_get_kernel_info)
  std::vector<int> primTypes;  // decoded shape id of each row (run-time kernels compiled for the scene's rows)
  float4* wf = nullptr;  // its path state: 11 float4 arrays of wfSlots
  size_t wfSlots = 0;
  int numCUs = 256;
  float* stage = nullptr;    // sample-group staging, allocated on first use
  size_t stageBytes = 0;
  int accumMode = SAIL_ACCUM_SUM;
  int rank = 0, world = 1, partMode = SAIL_PART_TILES;
  // samples per launch (sail_set_launch_samples); 0 = by form (launchSamples): 64 measured C2 +0.7 %, C3 +0.5 %, C4/C5
  // +-0.2 % over 32 (profiles/r04_launch_spp*)
  int launchSpp = 0;
  uint64_t k = 0;  // global sample index of the next sample (the reference's sampleCount)
  uint64_t samplesThisRank = 0;
  uint64_t nominalSegments = 0;
  std::vector<hipEvent_t> evPool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double kernelMs = 0.0, lastLaunchMs = 0.0;
  double lastFilterMs = 0.0;  // device time of the last display-filter pass
  uint32_t launches = 0;
  nccl_comm_t comm = nullptr;
  int commRanks = 0, commRank = 0;
  // Reduced frame (root of sail_reduce / device 0 of a multi-device context): the sum of every rank's
  // cumulative accumulator, recomputed from scratch by each reduce, so render -> reduce -> render -> reduce
  // never counts a sample twice. While `reduced` is set, readback / read_accum / filter show this frame.
  float4* frame = nullptr;
  float4* frameN = nullptr;  // reduced AOVs (SAIL_FLAG_AOV)
  float4* frameP = nullptr;
  bool reduced = false;
  // Multi-device context (sail_create_multi): one sub-context per device, each rendering its share of the
  // partition on its own stream; `dirty` = rendered since the last reduce. Devices are all distinct (grouped
  // RCCL reduce over a ncclCommInitAll communicator) or all the same one (`groupLocal`: summed by a kernel).
  std::vector<sail_ctx*> subs;
  // A checkpoint loaded part by part (sail_load_accum part >= 0): the parts still missing (bit i = device i) and the
  // checkpoint's k. Until every part is in, the frame mixes old and loaded accumulators, so rendering, reading, saving
  // and reducing are refused.
  uint64_t loadMissing = 0;
  uint64_t loadK = 0;
  std::vector<nccl_comm_t> groupComms;
  bool groupLocal = false;
  bool dirty = false;
  // One-sample frames of sail_render waiting to be launched together (sail_render / flushQueued): their records
  // (global sample index already counted in k), the bounce count and eye they were queued with
  std::vector<SailSample> queued;
  int queuedBounces = 0;
  float eyeCache[3] = {0.0f, 0.0f, 0.0f};
  std::string err;
};

namespace {

int fail(sail_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf; else g_create_error = buf;
  return code;
}
// a multi-device context's call failed in one of its sub-contexts: carry that context's message up
int relay(sail_ctx* c, int rc, const sail_ctx* sub) {
  if (rc != SAIL_OK && sub && c != sub) c->err = sub->err;
  return rc;
}
// a part-wise checkpoint load still missing parts (sail_load_accum): refuse whatever would see the half-loaded frame
int loadIncomplete(sail_ctx* c, const char* what) {
  if (!c->loadMissing) return SAIL_OK;
  return fail(c, SAIL_E_STATE, "%s: checkpoint parts not loaded yet (mask 0x%llx of %d devices); load every part or reset",
              what, (unsigned long long)c->loadMissing, (int)c->subs.size());
}
#define HIPCHK(ctx, call)                                                                       \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return fail((ctx), SAIL_E_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

// the smallest precompiled plugin-set kernel that covers the scene (sail_device.h SAIL_KSET_*)
int kernelSetFor(const sail_ctx* c) {
  if (c->forceGeneric || c->n >= c->cullMinPrims) return SAIL_KSET_GENERIC;
  const sail_plugins& p = c->plugins;
  const bool lightsOk = c->ln == 0 || (p.light_mask & ~SAIL_KSET_CORNELL_LIGHTS) == 0;
  if ((p.shape_mask & ~SAIL_KSET_CORNELL_SHAPES) == 0 && (p.material_mask & ~SAIL_KSET_CORNELL_MATS) == 0 &&
      (p.texture_mask & ~SAIL_KSET_CORNELL_TEX) == 0 && lightsOk && SAIL_KSET_CORNELL_LIGHTS == 0 && c->ln == 0)
    return SAIL_KSET_CORNELL;
  if ((p.shape_mask & ~SAIL_KSET_ROOM_SHAPES) == 0) return SAIL_KSET_ROOM;
  return SAIL_KSET_GENERIC;
}

// the sample-group stage's cap (12 B per owned pixel per staged sample): 8 GiB
constexpr size_t kStageCapBytes = (size_t)8 << 30;
// Launch bounds of a run-time kernel by form and by the precompiled family its plugin set falls in: the precompiled
// kernels' own (6 waves all-plugin, 8 Cornell, 7 room, 8 pre-cull), except that a flat scene outside the Cornell and room
// sets compiled in the room form runs at 8 waves (its smaller kernel spills less: ALL +3.6 %, AREA +3.8 % over 7,
// profiles/r04_jit_occupancy.jsonl).
int jitWaves(int mode, int kernelSet) {
  if (mode == SAIL_JIT_MODE_CULL) return 8;
  if (mode == SAIL_JIT_MODE_ROOM) return kernelSet == SAIL_KSET_ROOM ? 7 : 8;
  return kernelSet == SAIL_KSET_CORNELL ? 8 : 6;
}
// Workgroup shape of a run-time kernel by form (profiles/r05_ns_*.jsonl, r05_nt*_C1.jsonl; 1080p / 4K, 64-sample
// launches, bit-identical): the Cornell form at 512 threads holding 16 samples of 32 pixels (C1 98.6 Gseg/s against 97.5-98.1
// at 256 threads x 1 sample with 8 staged sample groups: no stage and no sail_accum_kernel at full frame; 512 x 1 sample,
// staged, 98.8-99.0); the room and pre-cull forms at their 256 / 1,024 threads holding 4 samples (C3 +1.2 %, C4 +0.8 %;
// 16 samples C3 -0.4 %, C4 -1.3 %; C3 at 128 / 512 threads -9 % / -4 %, C4 at 512 -62 %: its LDS tables then
// leave room for too few workgroups).
// The Cornell form's 16 samples in flight pay while the context's share of the frame queues enough workgroups: with a
// small share (a rank of 8 or more, one eighth of 1080p) it holds 1 sample and the launch is split into staged sample
// groups instead (C2 per GPU at N = 8: 95.4 Gseg/s against 92.1 with 16 samples and no groups, 91.4 with both; at
// N = 4 95.2 against 94.9; profiles/r05_scale_ns_c2.jsonl, tools/scale_groups.sh).
int ownedTiles(const sail_ctx* c, int* tilesX, int* tilesY);
bool cornellShareLarge(const sail_ctx* c) {
  int tx, ty;
  const int owned = ownedTiles(c, &tx, &ty);
  // residency rounds of 512-thread workgroups at 8 waves per SIMD (4,096 / 32 pixels = 128 workgroups per tile)
  const double rounds = (double)owned * 128.0 / ((double)c->numCUs * 4.0);
  return rounds >= 12.0;
}
int jitNsFor(const sail_ctx* c, int mode, int kernelSet) {
  if (mode == SAIL_JIT_MODE_FLAT && kernelSet == SAIL_KSET_CORNELL) return cornellShareLarge(c) ? 16 : 1;
  if (mode == SAIL_JIT_MODE_ROOM || mode == SAIL_JIT_MODE_CULL) return 4;
  return 1;
}
int jitNtFor(int mode, int kernelSet) {
  return (mode == SAIL_JIT_MODE_FLAT && kernelSet == SAIL_KSET_CORNELL) ? 512 : 0;
}
// The run-time kernel spec of the context's scene under its switches, or false when none applies.
// SAIL_DEBUG_JIT bits (include/sail_hip.h): 1 flat scenes outside the Cornell and room sets, 2 pre-cull scenes, 4 room-set
// scenes, 8 the flat scenes of bit 1 in the room form, 16 flat scenes compiled for their rows as well (any flat scene).
bool jitSpecFor(const sail_ctx* c, SailJitSpec* out, int* mode) {
  if (!c->jit || !c->haveScene || c->forceGeneric) return false;
  const int set = kernelSetFor(c);
  const bool rows = (c->jit & 16) && c->n >= 1 && c->n <= kSailJitMaxRows && c->n < c->cullMinPrims &&
                    (int)c->primTypes.size() == c->n;
  int m;
  if (set == SAIL_KSET_GENERIC && c->n >= c->cullMinPrims) {
    if (!(c->jit & 2)) return false;
    m = SAIL_JIT_MODE_CULL;
  } else if (set == SAIL_KSET_GENERIC) {
    if (!(c->jit & 1) && !rows) return false;
    m = (c->jit & 8) ? SAIL_JIT_MODE_ROOM : SAIL_JIT_MODE_FLAT;
  } else if (set == SAIL_KSET_ROOM) {
    if (!(c->jit & 4) && !rows) return false;
    m = SAIL_JIT_MODE_ROOM;
  } else {
    if (!rows) return false;  // the Cornell kernel's set is the Cornell box's own
    m = SAIL_JIT_MODE_FLAT;
  }
  const sail_plugins& p = c->plugins;
  SailJitSpec spec;
  spec.ks = p.shape_mask; spec.km = p.material_mask; spec.kt = p.texture_mask; spec.kl = p.light_mask;
  spec.mode = m;
  spec.waves = jitWaves(m, set);
  spec.ldsFit = (m == SAIL_JIT_MODE_CULL && c->n <= SAIL_CULL_LDS_ROWS && c->tn <= SAIL_CULL_LDS_TP) ? 1 : 0;
  spec.ns = c->jitNs ? c->jitNs : jitNsFor(c, m, set);
  spec.nt = c->jitNt ? c->jitNt : jitNtFor(m, set);
  if (sailJitThreads(spec) / spec.ns < 16) spec.ns = 4;  // at least 16 pixels per workgroup
  if (rows && m != SAIL_JIT_MODE_CULL) {
    spec.rows = c->n;
    for (int i = 0; i < c->n; i++) spec.types[i] = c->primTypes[i];
    for (int i = 0; i < c->n; i++)
      if (spec.types[i] < 1 || !((spec.ks >> spec.types[i]) & 1u)) spec.rows = 0;  // a row no compiled shape hits
    if (!spec.rows) for (int& t : spec.types) t = 0;
    // the room form copies both tables into LDS (C3 +2.8 %, UI +2.2 %; the Cornell form measured -0.5 %)
    if (spec.rows && m == SAIL_JIT_MODE_ROOM && c->tn >= 1 && c->tn <= kSailJitMaxFlatTp) spec.tn = c->tn;
  }
  *out = spec;
  *mode = m;
  return true;
}
// Re-derive the scene's run-time kernel after anything it depends on changed (scene, rows, switches). A new spec starts
// its background build now (Tracer.update links the scene's program, tracer.js:42-90), so the caller never waits for it.
void refreshJit(sail_ctx* c) {
  // a multi-device context renders through its sub-contexts, which derive their own kernels (its own plugins and rows
  // are not kept: a spec derived here would be a useless build)
  if (!c->subs.empty()) return;
  SailJitSpec spec;
  int mode = 0;
  const bool have = jitSpecFor(c, &spec, &mode);
  if (have == c->jitHave && (!have || sailJitSpecEqual(spec, c->jitSpec))) return;
  // hold the new spec before dropping the old one: a build both share is never skipped in between
  if (have) sail_jit_hold(c->device, spec, +1);
  if (c->jitHave) sail_jit_hold(c->device, c->jitSpec, -1);
  c->jitHave = have;
  c->jitSpec = spec;
  c->jitMode = mode;
  c->jitK = SailJitKernel{};
  c->jitError.clear();
  c->jitState = have ? SAIL_KERNEL_JIT_PENDING : SAIL_KERNEL_JIT_NONE;
  if (!have) return;
  std::string err;
  const int r = sail_jit_kernels(c->device, spec, 0, &c->jitK, &err);  // starts the build; loads it if it is cached
  if (r == 0) c->jitState = SAIL_KERNEL_JIT_READY;
  else if (r < 0) { c->jitState = SAIL_KERNEL_JIT_FAILED; c->jitError = err; }
}
// The run-time compiled kernel of the scene's plugin set (sail_jit.cpp), waiting up to wait_ms for its build; false when
// none applies, it is still being built or it failed (the precompiled kernel of the scene's set then runs, with the same
// results). *mode: SAIL_JIT_MODE_*.
bool jitKernels(sail_ctx* c, int wait_ms, SailJitKernel* k, int* mode) {
  if (!c->jitHave || c->jitState == SAIL_KERNEL_JIT_FAILED) return false;
  if (c->jitState != SAIL_KERNEL_JIT_READY) {
    std::string err;
    const int r = sail_jit_kernels(c->device, c->jitSpec, wait_ms, &c->jitK, &err);
    if (r == 1) return false;
    if (r < 0) { c->jitState = SAIL_KERNEL_JIT_FAILED; c->jitError = err; return false; }
    c->jitState = SAIL_KERNEL_JIT_READY;
  }
  *k = c->jitK;
  *mode = c->jitMode;
  return true;
}
// Samples per launch when the host has not fixed them: the Cornell form holding 16 samples in flight runs a whole
// 1,024-sample frame in one launch (its waves live 16 times longer, so their per-wave start -- the spill stores of the
// loop-invariant registers among it -- is paid 16 times less often: C1 Gseg/s at 64 / 128 / 256 / 1,024 samples per
// launch 97.26 / 97.73 / 97.99 / 98.36, profiles/r05_launch_*.jsonl); everything else 64 (sample groups stage a launch's
// samples, which a larger launch would push past the stage's cap).
int launchSamples(const sail_ctx* c) {
  if (c->launchSpp > 0) return c->launchSpp;
  return (c->jitHave && c->jitState != SAIL_KERNEL_JIT_FAILED && c->jitSpec.ns >= 16) ? 1024 : 64;
}
int ownedTiles(const sail_ctx* c, int* tilesX, int* tilesY) {
  const int tx = (c->W + 63) / 64, ty = (c->H + 63) / 64;
  *tilesX = tx; *tilesY = ty;
  if (c->partMode == SAIL_PART_SAMPLES) return tx * ty;
  const int total = tx * ty;
  return c->rank < total ? (total - c->rank + c->world - 1) / c->world : 0;
}
long long ownedPixels(const sail_ctx* c) {
  int tx, ty;
  const int owned = ownedTiles(c, &tx, &ty);
  long long px = 0;
  const int w = (c->partMode == SAIL_PART_SAMPLES) ? 1 : c->world, r = (c->partMode == SAIL_PART_SAMPLES) ? 0 : c->rank;
  for (int j = 0; j < owned; j++) {
    const int t = r + j * w;
    const int x0 = (t % tx) * 64, y0 = (t / tx) * 64;
    const int cw = (c->W - x0) < 64 ? (c->W - x0) : 64, ch = (c->H - y0) < 64 ? (c->H - y0) : 64;
    px += (long long)cw * ch;
  }
  return px;
}

int collectEvents(sail_ctx* c) {
  for (auto& pr : c->pending) {
    HIPCHK(c, hipEventSynchronize(pr.second));
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, pr.first, pr.second));
    c->kernelMs += ms;
    c->lastLaunchMs = ms;
    c->evPool.push_back(pr.first);
    c->evPool.push_back(pr.second);
  }
  c->pending.clear();
  return SAIL_OK;
}
int getEvent(sail_ctx* c, hipEvent_t* ev) {
  if (!c->evPool.empty()) { *ev = c->evPool.back(); c->evPool.pop_back(); return SAIL_OK; }
  HIPCHK(c, hipEventCreate(ev));
  return SAIL_OK;
}

// corner directions of vstrace.glsl:4-6 for one jittered inverse matrix (column-major, f32)
void cornerDirs(const float* M, const float* eye, float out[4][3]) {
  static const float cx[4] = {-1.0f, -1.0f, 1.0f, 1.0f}, cy[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
  for (int c = 0; c < 4; c++) {
    float q[4];
    for (int r = 0; r < 4; r++) q[r] = M[0 * 4 + r] * cx[c] + M[1 * 4 + r] * cy[c] + M[2 * 4 + r] * 0.0f + M[3 * 4 + r] * 1.0f;
    const float w[3] = {gdiv(q[0], q[3]) - eye[0], gdiv(q[1], q[3]) - eye[1], gdiv(q[2], q[3]) - eye[2]};
    const float len = sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    out[c][0] = gdiv(w[0], len); out[c][1] = gdiv(w[1], len); out[c][2] = gdiv(w[2], len);
  }
}

int resetAccum(sail_ctx* c) {
  c->reduced = false;
  c->queued.clear();  // queued one-sample frames belong to the accumulation being discarded
  const size_t bytes = (size_t)c->W * c->H * sizeof(float4);
  HIPCHK(c, hipMemsetAsync(c->accum, 0, bytes, c->stream));
  if (c->aovN) HIPCHK(c, hipMemsetAsync(c->aovN, 0, bytes, c->stream));
  if (c->aovP) HIPCHK(c, hipMemsetAsync(c->aovP, 0, bytes, c->stream));
  if ((c->aovN || c->aovP) && c->partMode == SAIL_PART_TILES && c->world > 1)
    HIPCHK(c, sail_launch_negzero_unowned(c->aovN, c->aovP, c->W, c->H, c->rank, c->world, c->stream));
  if (c->segCounter) HIPCHK(c, hipMemsetAsync(c->segCounter, 0, SAIL_SEG_SLOTS * sizeof(unsigned long long), c->stream));
  int rc = collectEvents(c);
  if (rc) return rc;
  c->k = 0;
  c->samplesThisRank = 0;
  c->nominalSegments = 0;
  c->kernelMs = 0.0;
  c->lastLaunchMs = 0.0;
  c->launches = 0;
  return SAIL_OK;
}

// Decode the objects rows into SailPrim records with the reference's addressing rules
// (shader.shape.js:34 row = float(i)/float(n-1); parseX readFloat/readVec3 columns; matIndex/texIndex as
// readFloat(...)/float(tn-1) normalised rows; cornellbox.glsl:17 material from slot 7).
// Rectangle frame (rectangle.glsl:32-44), the same f32 operations in the same order as the per-ray GLSL,
// evaluated once per scene: a[6..8] normal, a[9..11] ss, a[12..14] ts, a[15] maxX, a[16] maxY and
// a[17] the area-light pdf 1/(|x||y|) of sampleGeometry (shader.shape.js:53-67). Host f32 arithmetic is
// IEEE (SSE, no contraction), so the values are bit-identical to the kernel's own evaluation.
struct F3 { float x, y, z; };
F3 f3cross(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float f3dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
F3 f3div(F3 a, float s) { return {gdiv(a.x, s), gdiv(a.y, s), gdiv(a.z, s)}; }
void rectFrameHost(SailPrim& p) {
  const F3 dpdu{p.a[3] - p.a[0], 0.0f, 0.0f}, dpdv{0.0f, p.a[4] - p.a[1], p.a[5] - p.a[2]};
  const F3 cr = f3cross(dpdu, dpdv);
  const F3 normal = f3div(cr, sqrtf(f3dot(cr, cr)));
  const float maxX = sqrtf(f3dot(dpdu, dpdu)), maxY = sqrtf(f3dot(dpdv, dpdv));
  const F3 ss = f3div(dpdu, maxX);
  const F3 ts = f3cross(normal, ss);
  const float f[12] = {normal.x, normal.y, normal.z, ss.x, ss.y, ss.z, ts.x, ts.y, ts.z, maxX, maxY,
                       gdiv(1.0f, maxX * maxY)};
  memcpy(&p.a[6], f, sizeof f);
}

// GLSL min/max as v_min_f32/v_max_f32 evaluate them (a NaN operand yields the other; -0 < +0)
float hwmin(float a, float b) { if (a != a) return b; if (b != b) return a; if (a < b) return a; if (b < a) return b; return signbit(a) ? a : b; }
float hwmax(float a, float b) { if (a != a) return b; if (b != b) return a; if (a > b) return a; if (b > a) return b; return signbit(a) ? b : a; }
// Per-scene quadric constants, each the exact f32 expression the GLSL evaluates per ray:
//   cone (cone.glsl:58-59)            a[5] = (rad / h)^2
//   hyperboloid (hyperboloid.glsl:13-24)  a[11] = max(r1, r2), a[12] = min(p1.z, p2.z), a[13] = max(p1.z, p2.z)
//   paraboloid (paraboloid.glsl:60)   a[6] = zMax / (rad * rad)
void quadricHost(SailPrim& p) {
  if (p.type == SAIL_CONE) { float k = gdiv(p.a[4], p.a[3]); p.a[5] = k * k; }
  if (p.type == SAIL_HYPERBOLOID) {
    const float r1 = sqrtf(p.a[3] * p.a[3] + p.a[4] * p.a[4]), r2 = sqrtf(p.a[6] * p.a[6] + p.a[7] * p.a[7]);
    p.a[11] = hwmax(r1, r2); p.a[12] = hwmin(p.a[5], p.a[8]); p.a[13] = hwmax(p.a[5], p.a[8]);
  }
  if (p.type == SAIL_PARABOLOID) p.a[6] = gdiv(hwmax(p.a[3], p.a[4]), p.a[5] * p.a[5]);
}

// Conservative world-space bounds of what each primitive's intersection can return, padded, in a[18..23]
// (min xyz, max xyz; +-inf when the shape has no finite bound). The trace kernel uses them for a cheap f32
// pre-cull before the exact per-primitive test: a primitive whose padded box the ray misses, or enters
// beyond the closest distance so far, cannot change the sweep's result (n = 67).
// Local frames: OBJECT_SPACE maps world (x, y, z) -> local (-z, x, y), so the local z axis is world y.
struct PrimBox { double lo[3], hi[3]; };
PrimBox primBoundsRaw(const SailPrim& p) {
  const double inf = INFINITY;
  PrimBox b{{-inf, -inf, -inf}, {inf, inf, inf}};
  double* lo = b.lo;
  double* hi = b.hi;
  const float* a = p.a;
  auto box = [&](double x0, double y0, double z0, double x1, double y1, double z1) {
    lo[0] = fmin(x0, x1); lo[1] = fmin(y0, y1); lo[2] = fmin(z0, z1);
    hi[0] = fmax(x0, x1); hi[1] = fmax(y0, y1); hi[2] = fmax(z0, z1);
  };
  switch (p.type) {
    case SAIL_CUBE: case SAIL_CORNELLBOX: box(a[0], a[1], a[2], a[3], a[4], a[5]); break;
    case SAIL_RECTANGLE: {  // corners mn + {0, maxX} ss + {0, maxY} ts (rectangle.glsl:32-63)
      const double ss[3] = {a[9], a[10], a[11]}, ts[3] = {a[12], a[13], a[14]}, mx = a[15], my = a[16];
      for (int k = 0; k < 3; k++) {
        const double c0 = a[k], c1 = a[k] + mx * ss[k], c2 = a[k] + my * ts[k], c3 = a[k] + mx * ss[k] + my * ts[k];
        lo[k] = fmin(fmin(c0, c1), fmin(c2, c3));
        hi[k] = fmax(fmax(c0, c1), fmax(c2, c3));
      }
      break;
    }
    case SAIL_SPHERE: { const double r = fabs(a[3]); box(a[0] - r, a[1] - r, a[2] - r, a[0] + r, a[1] + r, a[2] + r); break; }
    case SAIL_CONE: case SAIL_CYLINDER: {  // radius <= rad for local z in [-EPS, h]
      const double r = fabs(a[4]);
      box(a[0] - r, a[1], a[2] - r, a[0] + r, a[1] + a[3], a[2] + r);
      break;
    }
    case SAIL_DISK: { const double r = fabs(a[3]); box(a[0] - r, a[1], a[2] - r, a[0] + r, a[1], a[2] + r); break; }
    case SAIL_HYPERBOLOID: {  // ah (x^2 + y^2) - ch z^2 = 1 for z in [zMin, zMax] (a[12], a[13])
      const double ah = a[9], ch = a[10], z0 = a[12], z1 = a[13];
      double r2 = -1.0;
      if (ah > 0.0 && z0 <= z1) {
        const double zs[3] = {z0, z1, (z0 < 0.0 && z1 > 0.0) ? 0.0 : z0};
        for (double z : zs) r2 = fmax(r2, (1.0 + ch * z * z) / ah);
      }
      if (r2 >= 0.0 && std::isfinite(r2)) {
        const double r = sqrt(r2);
        box(a[0] - r, a[1] + z0, a[2] - r, a[0] + r, a[1] + z1, a[2] + r);
      }
      break;
    }
    case SAIL_PARABOLOID: {  // k (x^2 + y^2) = z, k = zMax / rad^2 (a[6]); z in [min(z0,z1), max(z0,z1)]
      const double k = a[6], z0 = fmin(a[3], a[4]), z1 = fmax(a[3], a[4]);
      if (k > 0.0 && std::isfinite(k) && z1 >= 0.0) {
        const double r = sqrt(z1 / k);
        box(a[0] - r, a[1] + z0, a[2] - r, a[0] + r, a[1] + z1, a[2] + r);
      }
      break;
    }
    default: break;
  }
  for (int k = 0; k < 3; k++)
    if (!std::isfinite(lo[k]) || !std::isfinite(hi[k])) { lo[k] = -inf; hi[k] = inf; }
  return b;
}

// Union of the primitives' finite bounds: every hit point, hence every bounce / shadow ray origin, lies in it.
SceneBox sceneBox(const std::vector<PrimBox>& raw) {
  SceneBox s{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}, 0.0};
  bool any = false;
  for (const PrimBox& b : raw) {
    if (!std::isfinite(b.lo[0]) || !std::isfinite(b.lo[1]) || !std::isfinite(b.lo[2])) continue;
    any = true;
    for (int k = 0; k < 3; k++) { s.lo[k] = fmin(s.lo[k], b.lo[k]); s.hi[k] = fmax(s.hi[k], b.hi[k]); }
  }
  if (!any) { for (int k = 0; k < 3; k++) s.lo[k] = s.hi[k] = 0.0; }
  s.diag = sqrt((s.hi[0] - s.lo[0]) * (s.hi[0] - s.lo[0]) + (s.hi[1] - s.lo[1]) * (s.hi[1] - s.lo[1]) +
                (s.hi[2] - s.lo[2]) * (s.hi[2] - s.lo[2]));
  return s;
}

// Padding of each primitive's bounds into a[18..23]. The exact f32 tests (the reference's GLSL) can report a hit
// slightly outside the true surface, the more so the farther the ray origin: a slab / plane distance is off by
// about L 2^-23 at range L, and a quadric's discriminant b^2 - 4ac loses about 20 L^2 2^-24 to cancellation,
// which moves its hit band by that over the local radius (and by its square root near a cone apex or where the
// radius is unknown). Origins here are hit points inside the scene box, or the eye when it lies within one
// scene diagonal D of the box (sail_launch: cullPrimary), so L = 2D bounds every origin-to-primitive distance.
// Padding = 1e-3 + 1e-4 |bound| + 2^-20 L, plus 1.2e-6 L^2 / r for quadrics (+ 1.1e-3 L for cones,
// hyperboloids and paraboloids). Measured by the far-origin tests (tests/test_gpu_fullsize.py).
void padPrimBounds(std::vector<SailPrim>& prims, const std::vector<PrimBox>& raw, const SceneBox& sb) {
  const double L = 2.0 * sb.diag, kQ = 20.0 / 16777216.0;
  for (size_t i = 0; i < prims.size(); i++) {
    SailPrim& p = prims[i];
    const PrimBox& b = raw[i];
    double extra = L / 1048576.0;
    double r = -1.0;  // local radius of a quadric (its smallest), -1: not a quadric
    bool apex = false;
    switch (p.type) {
      case SAIL_SPHERE: r = fabs(p.a[3]); break;
      case SAIL_CYLINDER: r = fabs(p.a[4]); break;
      case SAIL_CONE: r = fabs(p.a[4]); apex = true; break;
      case SAIL_HYPERBOLOID: case SAIL_PARABOLOID:
        r = 0.5 * fmin(b.hi[0] - b.lo[0], b.hi[2] - b.lo[2]); apex = true; break;
      default: break;
    }
    if (r >= 0.0) {
      extra += (r > 0.0 && std::isfinite(r)) ? kQ * L * L / r : INFINITY;
      if (apex) extra += sqrt(kQ) * L;
    }
    for (int k = 0; k < 3; k++) {
      double lo = b.lo[k], hi = b.hi[k];
      if (std::isfinite(lo) && std::isfinite(hi) && std::isfinite(extra)) {
        const double pad = 1e-3 + 1e-4 * fmax(fabs(lo), fabs(hi)) + extra;
        lo -= pad; hi += pad;
      } else {
        lo = -INFINITY; hi = INFINITY;
      }
      p.a[18 + k] = (float)lo; p.a[21 + k] = (float)hi;
    }
  }
}

// Largest padded-bound coordinate of the scene, inf when a primitive has no finite bound. Every ray origin
// is the eye or a hit point inside some padded box, so |origin| <= max(extent, |eye|) (see cullFmaOk).
double primExtent(const std::vector<SailPrim>& prims) {
  double m = 0.0;
  for (const SailPrim& p : prims)
    for (int k = 18; k < 24; k++) m = fmax(m, std::isfinite(p.a[k]) ? fabs((double)p.a[k]) : INFINITY);
  return m;
}

// The fused pre-cull form (sail_trace.hip padHitF) tests each slab plane as fma(a, R, -RN(o R)): the plane
// lands within |o| 2^-24 of where the plain (a - o) R puts it, so the test stays conservative while that is
// far inside the 1e-3 padding. |o| < 4096 keeps it under 2.5e-4; it also keeps o R finite with R <= 1e30.
bool cullFmaOk(const sail_ctx* c) {
  const double e = fmax(fmax(fabs(c->eyeCache[0]), fabs(c->eyeCache[1])), fabs(c->eyeCache[2]));
  return c->cullFma && fmax(c->primExtent, e) < 4096.0;
}

// Primary rays may use the pre-cull only when the eye lies within one scene diagonal of the scene box: the
// padding (padPrimBounds) covers origin-to-primitive distances up to two diagonals.
int eyeNearScene(const sail_ctx* c) {
  double d2 = 0.0;
  for (int k = 0; k < 3; k++) {
    const double e = c->eyeCache[k];
    const double g = e < c->scene.lo[k] ? c->scene.lo[k] - e : (e > c->scene.hi[k] ? e - c->scene.hi[k] : 0.0);
    d2 += g * g;
  }
  return d2 == d2 && sqrt(d2) <= c->scene.diag;
}

// the category words the kernel tests (material.glsl / texture dispatch: int(readFloat(row, 0))), clamped to
// [-1, 32] (every test is == c, < 0 or >= 32 against categories in [0, 31]) and packed in SailPrim.cats
void fillCats(std::vector<SailPrim>& prims, const float* texparams, int tn) {
  auto cat = [&](int row) {
    const int v = (tn > 0 && row >= 0 && row < tn) ? to_int(texparams[(size_t)row * 16]) : 0;
    return v < -1 ? -1 : (v > 32 ? 32 : v);
  };
  for (SailPrim& p : prims)
    p.cats = (int32_t)(((uint32_t)(uint16_t)(int16_t)cat(p.matRow)) | ((uint32_t)(uint16_t)(int16_t)cat(p.texRow) << 16));
}

void decodePrims(const float* objects, int n, int tn, uint32_t shapeMask, std::vector<SailPrim>& out, int* anyHitOk,
                 SceneBox* sbOut) {
  std::vector<PrimBox> raw((size_t)n);
  TexView o{objects, 18, n};
  const float L = 17.0f;
  out.assign((size_t)n, SailPrim{});
  *anyHitOk = 1;
  auto row = [&](float v) { return texel(gdiv(v, (float)(tn - 1)), tn); };
  for (int i = 0; i < n; i++) {
    const float rc = gdiv((float)i, (float)(n - 1));
    SailPrim& p = out[i];
    memset(&p, 0, sizeof p);
    const int cat = to_int(o.at(0.0f, rc));
    if (cat < 1 || cat > 9 || !((shapeMask >> cat) & 1u)) { p.type = 0; continue; }
    p.type = cat;
    float v3[3];
    switch (cat) {
      case SAIL_CUBE: case SAIL_RECTANGLE:
        o.readVec3(1.0f, rc, L, &p.a[0]); o.readVec3(4.0f, rc, L, &p.a[3]);
        p.rev = to_int(o.readFloat(7.0f, rc, L)) == 1;
        p.matRow = row(o.readFloat(8.0f, rc, L)); p.texRow = row(o.readFloat(9.0f, rc, L));
        o.readVec3(10.0f, rc, L, v3);
        if (cat == SAIL_RECTANGLE) rectFrameHost(p);
        break;
      case SAIL_SPHERE:
        o.readVec3(1.0f, rc, L, &p.a[0]); p.a[3] = o.readFloat(4.0f, rc, L);
        p.rev = to_int(o.readFloat(5.0f, rc, L)) == 1;
        p.matRow = row(o.readFloat(6.0f, rc, L)); p.texRow = row(o.readFloat(7.0f, rc, L));
        o.readVec3(8.0f, rc, L, v3);
        break;
      case SAIL_CONE: case SAIL_CYLINDER: case SAIL_DISK:  // p3, (h r) or (r innerR)
        o.readVec3(1.0f, rc, L, &p.a[0]); p.a[3] = o.readFloat(4.0f, rc, L); p.a[4] = o.readFloat(5.0f, rc, L);
        p.rev = to_int(o.readFloat(6.0f, rc, L)) == 1;
        p.matRow = row(o.readFloat(7.0f, rc, L)); p.texRow = row(o.readFloat(8.0f, rc, L));
        o.readVec3(9.0f, rc, L, v3);
        break;
      case SAIL_HYPERBOLOID:
        o.readVec3(1.0f, rc, L, &p.a[0]); o.readVec3(4.0f, rc, L, &p.a[3]); o.readVec3(7.0f, rc, L, &p.a[6]);
        p.a[9] = o.readFloat(10.0f, rc, L); p.a[10] = o.readFloat(11.0f, rc, L);
        p.rev = to_int(o.readFloat(12.0f, rc, L)) == 1;
        p.matRow = row(o.readFloat(13.0f, rc, L)); p.texRow = row(o.readFloat(14.0f, rc, L));
        o.readVec3(15.0f, rc, L, v3);
        break;
      case SAIL_PARABOLOID:
        o.readVec3(1.0f, rc, L, &p.a[0]);
        p.a[3] = o.readFloat(4.0f, rc, L); p.a[4] = o.readFloat(5.0f, rc, L); p.a[5] = o.readFloat(6.0f, rc, L);
        p.rev = to_int(o.readFloat(7.0f, rc, L)) == 1;
        p.matRow = row(o.readFloat(8.0f, rc, L)); p.texRow = row(o.readFloat(9.0f, rc, L));
        o.readVec3(10.0f, rc, L, v3);
        break;
      case SAIL_CORNELLBOX:
        o.readVec3(1.0f, rc, L, &p.a[0]); o.readVec3(4.0f, rc, L, &p.a[3]);
        p.rev = 0;
        p.matRow = row(o.readFloat(7.0f, rc, L));  // slot 7 = reverseNormal (cornellbox.glsl:17)
        p.texRow = 0;
        v3[0] = v3[1] = v3[2] = 0.0f;
        break;
      default: break;
    }
    p.em[0] = v3[0]; p.em[1] = v3[1]; p.em[2] = v3[2];
    quadricHost(p);
    raw[i] = primBoundsRaw(p);
    // only slabs return t > EPSILON strictly; anything else may tie or undercut EPSILON, so shadow
    // rays must then find the true closest distance (shader.light.js:24-31)
    if (cat != SAIL_CUBE && cat != SAIL_CORNELLBOX) *anyHitOk = 0;
  }
  const SceneBox sb = sceneBox(raw);
  padPrimBounds(out, raw, sb);
  if (sbOut) *sbOut = sb;
}

int ensureSamples(sail_ctx* c, int count) {
  if (count <= c->samplesCap) return SAIL_OK;
  c->samplesPos = 0;
  if (c->samples) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->samples)); c->samples = nullptr; }
  int cap = 4096;  // 256 KB: thousands of one-sample frames before the ring wraps
  while (cap < count) cap *= 2;
  if (c->samplesPinned) { (void)hipHostFree(c->samplesPinned); c->samplesPinned = nullptr; }
  if (hipMalloc(&c->samples, sizeof(SailSample) * cap) != hipSuccess) return fail(c, SAIL_E_OOM, "sample buffer");
  if (hipHostMalloc(&c->samplesPinned, sizeof(SailSample) * cap) != hipSuccess) c->samplesPinned = nullptr;
  c->samplesCap = cap;
  return SAIL_OK;
}

int launchTrace(sail_ctx* c, const SailSample* hs, int count, int maxBounces) {
  int tx, ty;
  const int owned = ownedTiles(c, &tx, &ty);
  if (count <= 0 || owned <= 0) return SAIL_OK;
  int rc = ensureSamples(c, count);
  if (rc) return rc;
  // The upload is ordered with its launches on the context stream. Each call takes the next slice of a ring
  // of sample records, so the host never waits for launches still reading earlier slices (one-sample frames
  // from Renderer.render() queue back to back); only a wrap of the ring waits for the stream.
  if (c->samplesPos + count > c->samplesCap) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->samplesPos = 0;
  }
  SailSample* dev = c->samples + c->samplesPos;
  const SailSample* src = hs;
  if (c->samplesPinned) {  // staged in the pinned mirror: the copy is a true async DMA (pageable ones wait)
    memcpy(c->samplesPinned + c->samplesPos, hs, sizeof(SailSample) * count);
    src = c->samplesPinned + c->samplesPos;
  }
  c->samplesPos += count;
  HIPCHK(c, hipMemcpyAsync(dev, src, sizeof(SailSample) * count, hipMemcpyHostToDevice, c->stream));
  const long long px = ownedPixels(c);
  // The stage holds 12 B per owned pixel per staged sample. It is capped (kStageCapBytes): a launch that would need
  // more runs one workgroup per block (no stage).
  const long long stageStride = (long long)owned * 4096;
  const int stageSpp = (int)std::max<long long>(1, (long long)(kStageCapBytes / ((size_t)stageStride * 12)));
  const int L = launchSamples(c);
  for (int s0 = 0; s0 < count; s0 += L) {
    const int nspp = (count - s0) < L ? (count - s0) : L;
    SailTraceArgs A;
    memset(&A, 0, sizeof A);
    A.prims = c->prims; A.typeMasks = reinterpret_cast<const unsigned long long*>(c->prims + c->n);
    A.texparams = c->tp; A.lights = c->lt; A.lightObjRow = c->lightObjRow;
    A.samples = dev + s0;
    A.accum = c->accum; A.aovN = c->aovN; A.aovP = c->aovP; A.segCounter = c->segCounter;
    A.W = c->W; A.H = c->H; A.n = c->n; A.tn = c->tn; A.ln = c->ln;
    A.matMask = c->plugins.material_mask; A.texMask = c->plugins.texture_mask; A.lightMask = c->plugins.light_mask;
    A.maxBounces = maxBounces; A.spp = nspp; A.accumMode = c->accumMode;
    A.tilesX = tx; A.tilesY = ty;
    A.world = (c->partMode == SAIL_PART_SAMPLES) ? 1 : c->world;
    A.rank = (c->partMode == SAIL_PART_SAMPLES) ? 0 : c->rank;
    A.ownedTiles = owned;
    A.shadowAnyHit = c->shadowAnyHit;
    A.cullPrims = c->n >= c->cullMinPrims ? (cullFmaOk(c) ? 2 : 1) : 0;
    A.cullPrimary = eyeNearScene(c);
    A.kernelSet = kernelSetFor(c);
    memcpy(A.eye, c->eyeCache, sizeof A.eye);
    // Sample groups: a rank's share of a small frame is too few workgroups to fill the device (1/8 of 1080p
    // = 1,016 workgroups = 4 waves per SIMD); split the launch's samples over G workgroups per block so
    // that about 4 rounds of 7-wave-per-SIMD residency are queued, and add the staged samples in order.
    const bool wavefront = c->wavefront && A.kernelSet == SAIL_KSET_GENERIC && A.cullPrims;
    SailJitKernel jk;
    int jmode = 0;
    const bool jit = !wavefront && jitKernels(c, c->jitWait, &jk, &jmode);
    // samples of each pixel in flight per workgroup (the run-time kernels' spec; the precompiled kernels hold one):
    // NS times the workgroups of one sample in flight, each NS times shorter
    const int ns = jit ? c->jitSpec.ns : 1;
    int G = 1;
    if (c->forceGroups > 0) {
      G = c->forceGroups;
    } else if (A.kernelSet == SAIL_KSET_GENERIC && A.cullPrims) {
      // The pre-cull kernel's workgroups are 1,024 threads, two per CU at 8 waves per SIMD. Its per-workgroup cost
      // varies with the primitives a 16x64 strip sees, so a grid of few rounds ends in a long tail (1/8 of C4: 1,020
      // workgroups = 2 rounds, 0.92 of the one-GPU rate per GPU): below 6 rounds, split the samples so that about 8
      // rounds are queued (the grouped kernel is 1,024 threads too; measured 0.95 at N = 8 with 4 groups).
      // Round 3: more groups pay at any frame size (a shorter tail per launch); C4 at N = 1: G = 1 / 2 / 4 9.96 / 10.06
      // / 10.12 Gseg/s (gpurun_out/r03o), so about SAIL_CULL_GROUP_ROUNDS rounds are queued.
      const double rounds = (double)owned * 4.0 * ns / (double)(c->numCUs * 2);
      if (rounds < (double)c->cullGroupRounds) G = (int)ceil((double)c->cullGroupRounds / rounds);
    } else {
      // Round 3: splitting pays at full frame size too (shorter launch tails): C2 at N = 1 with G = 1 / 2 / 4 / 8 / 16
      // 89.3 / 89.7 / 90.9 / 91.6 / 91.4 Gseg/s, C5 87.0 / 89.3 / 90.9 / 91.6 / 91.9, C3 29.2 / 28.6 / 29.2 / 29.5 / 29.4;
      // at N = 8 (C2) G = 8 / 16 / 32 85 / 87 / 88 (gpurun_out/r03o). About 36 rounds of 7-wave residency are queued.
      const long long waves = (long long)owned * 16 * 4 * ns;
      const long long target = (long long)c->numCUs * 4 * 7 * c->flatGroupRounds;
      G = (int)((target + waves - 1) / waves);
      // the Cornell form holds 16 samples in flight only while its share queues enough workgroups (jitNsFor), and then
      // runs unsplit: staged groups lost 2-3 % per GPU at N = 4 and 8 (profiles/r05_scale_groups_c2.jsonl)
      if (ns >= 16) G = 1;
    }
    if (G > nspp) G = nspp;
    if (G < 1) G = 1;
    if (nspp > stageSpp) G = 1;  // the stage would pass its cap
    A.groupSpp = (nspp + G - 1) / G;
    // whole steps of the workgroup's samples in flight: a group of 11 samples at 4 in flight would idle a quarter of
    // the lanes in its last step (C4 per GPU at N = 2 and 4: 12.6 Gseg/s against 13.4, profiles/r05_scale_groups_c4.jsonl)
    if (ns > 1 && A.groupSpp < nspp && c->forceGroups <= 0) A.groupSpp = ((A.groupSpp + ns - 1) / ns) * ns;
    A.sampleGroups = (nspp + A.groupSpp - 1) / A.groupSpp;
    A.groupHome = (jit ? jmode == SAIL_JIT_MODE_ROOM : SAIL_GROUP_HOME_FOR(A.kernelSet)) ? 1 : 0;
    A.stageStride = stageStride;
    const bool staged = A.sampleGroups > 1;
    if (staged) {  // sized for this launch's samples (it grows to the largest launch seen)
      const size_t need = (size_t)A.stageStride * (size_t)nspp * 3 * sizeof(float);
      if (need > c->stageBytes) {
        if (c->stage) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->stage)); c->stage = nullptr; }
        c->stageBytes = 0;
        if (hipMalloc(&c->stage, need) != hipSuccess) { c->stage = nullptr; return fail(c, SAIL_E_OOM, "sample-group stage"); }
        c->stageBytes = need;
      }
      A.stage = c->stage;
    }
    SailWfState WS;
    memset(&WS, 0, sizeof WS);
    if (wavefront) {
      A.sampleGroups = 1; A.groupSpp = nspp; A.stage = nullptr;
      const size_t slots = (size_t)owned * 4096;
      if (slots > c->wfSlots) {
        if (c->wf) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->wf)); c->wf = nullptr; }
        c->wfSlots = 0;
        if (hipMalloc(&c->wf, slots * 11 * sizeof(float4)) != hipSuccess) { c->wf = nullptr; return fail(c, SAIL_E_OOM, "wavefront state"); }
        c->wfSlots = slots;
      }
      float4* b = c->wf;
      WS.o = b; WS.d = b + c->wfSlots; WS.f = b + 2 * c->wfSlots; WS.e = b + 3 * c->wfSlots; WS.s = b + 4 * c->wfSlots;
      for (int i = 0; i < 6; i++) WS.sp[i] = b + (5 + i) * c->wfSlots;
    }
    hipEvent_t e0, e1;
    if ((rc = getEvent(c, &e0)) || (rc = getEvent(c, &e1))) return rc;
    HIPCHK(c, hipEventRecord(e0, c->stream));
    if (wavefront) {
      HIPCHK(c, sail_launch_wavefront(A, WS, c->stream));
    } else {
      if (jit) {
        void* args[] = {&A};
        const unsigned nt = (unsigned)sailJitThreads(c->jitSpec);
        const unsigned px = nt / (unsigned)ns;                            // pixels per workgroup
        HIPCHK(c, hipModuleLaunchKernel(A.sampleGroups > 1 ? jk.grouped : jk.plain,
                                        (unsigned)owned * (4096u / px) * (unsigned)A.sampleGroups, 1, 1, nt, 1, 1, 0,
                                        c->stream, args, nullptr));
        c->lastJit = true;
        c->lastJitMode = jmode;
        c->lastBuildId = jk.buildId;
      } else {
        HIPCHK(c, sail_launch_trace(A, owned * 16 * A.sampleGroups, c->stream));
        c->lastJit = false;
      }
      if (staged) HIPCHK(c, sail_launch_accum(A, owned * 16, c->stream));
    }
    HIPCHK(c, hipEventRecord(e1, c->stream));
    c->pending.emplace_back(e0, e1);
    c->lastGroups = A.sampleGroups;
    c->lastWavefront = wavefront;
    c->launches++;
    c->nominalSegments += (uint64_t)px * (uint64_t)nspp * (uint64_t)maxBounces;
  }
  return SAIL_OK;
}

// Launch the queued one-sample frames of sail_render as one launch sequence (launchTrace splits it into launches of
// launchSpp samples). Their sample index and counts were taken when they were queued.
int flushQueued(sail_ctx* c) {
  if (c->queued.empty()) return SAIL_OK;
  std::vector<SailSample> q;
  q.swap(c->queued);
  HIPCHK(c, hipSetDevice(c->device));
  return launchTrace(c, q.data(), (int)q.size(), c->queuedBounces);
}

// ---- reduced frame (sail_reduce, multi-device contexts) -----------------------------------------------------------
int ensureFrame(sail_ctx* c) {
  const size_t bytes = (size_t)c->W * c->H * sizeof(float4);
  float4** bufs[3] = {&c->frame, c->aovN ? &c->frameN : nullptr, c->aovP ? &c->frameP : nullptr};
  for (float4** b : bufs) {
    if (!b || *b) continue;
    if (hipMalloc(b, bytes) != hipSuccess) { *b = nullptr; return fail(c, SAIL_E_OOM, "reduced frame"); }
  }
  return SAIL_OK;
}
// the buffers readback / filter show: the last reduced frame while it is current, else this rank's own
const float4* shownAccum(const sail_ctx* c) { return c->reduced ? c->frame : c->accum; }
const float4* shownAovN(const sail_ctx* c) { return c->reduced && c->frameN ? c->frameN : c->aovN; }
const float4* shownAovP(const sail_ctx* c) { return c->reduced && c->frameP ? c->frameP : c->aovP; }

// asynchronous RCCL errors (ncclCommGetAsyncError): a failed collective surfaces here, not at enqueue time
int commCheck(sail_ctx* c, nccl_comm_t comm) {
  if (!comm || !g_rccl.commGetAsyncError) return SAIL_OK;
  int ae = 0;
  const int r = g_rccl.commGetAsyncError(comm, &ae);
  constexpr int kNcclInProgress = 7;  // non-blocking communicators only; this library creates blocking ones
  if (r != 0 || (ae != 0 && ae != kNcclInProgress)) {
    const int code = r ? r : ae;
    return fail(c, SAIL_E_RCCL, "RCCL communicator error %d: %s", code, g_rccl.errStr ? g_rccl.errStr(code) : "?");
  }
  return SAIL_OK;
}
int groupCommCheck(sail_ctx* g) {
  for (nccl_comm_t cm : g->groupComms) if (int rc = commCheck(g, cm)) return rc;
  return SAIL_OK;
}

// The reduce plan of rank `rank` of `world` (sail_plan_reduce): the one place sail_reduce and groupReduce take their
// choices from. A sample partition shows the AOVs of the rank (device) that rendered the frame's last sample, as on one
// GPU (sample k is rendered by rank k % world; k = the context's sample count); every other rank sends -0 maps.
sail_reduce_plan planReduce(int W, int H, int rank, int world, int mode, uint64_t k, int root) {
  sail_reduce_plan p;
  memset(&p, 0, sizeof p);
  const bool tiles = mode == SAIL_PART_TILES;
  const int tx = (W + 63) / 64, ty = (H + 63) / 64, total = tx * ty;
  p.receives = rank == root;
  p.tiles = tiles ? (rank < total ? (total - rank + world - 1) / world : 0) : total;
  p.aov_owner = tiles ? -1 : (k > 0 ? (int)((k - 1) % (uint64_t)world) : 0);
  p.send_own_aovs = tiles || rank == p.aov_owner;
  if (tiles || world <= 1) p.samples = k;
  else p.samples = k > (uint64_t)rank ? (k - 1 - (uint64_t)rank) / (uint64_t)world + 1 : 0;
  return p;
}
// one step of a part-wise checkpoint load (sail_plan_load_part): SAIL_OK or SAIL_E_INVALID, state unchanged on error
int planLoadPart(uint64_t* missing, uint64_t* k, int parts, int part, uint64_t kPart) {
  if (parts < 1 || parts > 64 || part < -1 || part >= parts) return SAIL_E_INVALID;
  if (part == -1) { *missing = 0; *k = kPart; return SAIL_OK; }
  const uint64_t all = parts >= 64 ? ~0ull : (1ull << parts) - 1ull;
  uint64_t m = *missing, kk = *k;
  if (!m) { m = all; kk = kPart; }
  else if (kPart != kk) return SAIL_E_INVALID;
  *missing = m & ~(1ull << part);
  *k = kk;
  return SAIL_OK;
}
// -0 in every component: the additive identity that keeps each AOV bit (x + -0 == x for +-0 and NaN too)
hipError_t fillNegZero(float4* p, size_t np, hipStream_t s) {
  return hipMemsetD32Async((hipDeviceptr_t)p, (int)0x80000000u, np * 4, s);
}

// Multi-device context: device 0's frame = the sum of every device's cumulative accumulator (and, for tile
// partitions, of the AOV maps: -0 outside each device's tiles, so the sum is exact). Recomputed from scratch
// whenever something was rendered since the last one, so progressive frames never count a sample twice.
// Sample partitions show the AOVs of the device that rendered the last sample: in the RCCL reduce every other
// device contributes a -0 map, so the reduced maps are that device's bits (the tile reduce's rule).
int groupReduce(sail_ctx* g) {
  const int nd = (int)g->subs.size();
  sail_ctx* r = g->subs[0];
  for (sail_ctx* s : g->subs) if (int rc = flushQueued(s)) return relay(g, rc, s);
  if ((nd == 1 && g->groupComms.empty()) || !g->dirty) return SAIL_OK;
  HIPCHK(g, hipSetDevice(r->device));
  if (int rc = ensureFrame(r)) return relay(g, rc, r);
  const bool tiles = g->partMode == SAIL_PART_TILES;
  const size_t np = (size_t)g->W * g->H, bytes = np * sizeof(float4);
  // every device's share of the exchange (sail_plan_reduce: device i = rank i of nd, root 0)
  std::vector<sail_reduce_plan> plan((size_t)nd);
  for (int i = 0; i < nd; i++) plan[i] = planReduce(g->W, g->H, i, nd, g->partMode, r->k, 0);
  const int owner = tiles ? 0 : plan[0].aov_owner;
  if (g->groupLocal) {  // every "device" is the same GPU: wait for the others' streams, sum in rank order
    for (sail_ctx* s : g->subs) HIPCHK(g, hipStreamSynchronize(s->stream));
    auto sum = [&](float4* dst, float4* sail_ctx::*src) -> hipError_t {
      SailSumArgs A;
      memset(&A, 0, sizeof A);
      A.dst = dst; A.n = (long long)np; A.nsrc = nd;
      for (int i = 0; i < nd; i++) A.src[i] = g->subs[i]->*src;
      return sail_launch_sum(A, r->stream);
    };
    const sail_ctx* o = g->subs[owner];
    HIPCHK(g, sum(r->frame, &sail_ctx::accum));
    if (r->aovN) HIPCHK(g, tiles ? sum(r->frameN, &sail_ctx::aovN) : hipMemcpyAsync(r->frameN, o->aovN, bytes, hipMemcpyDeviceToDevice, r->stream));
    if (r->aovP) HIPCHK(g, tiles ? sum(r->frameP, &sail_ctx::aovP) : hipMemcpyAsync(r->frameP, o->aovP, bytes, hipMemcpyDeviceToDevice, r->stream));
    HIPCHK(g, hipStreamSynchronize(r->stream));  // the other devices' next renders may overwrite their inputs
  } else {  // one grouped RCCL reduce into device 0 over the ncclCommInitAll communicator
    const bool aov = r->aovN || r->aovP;
    if (!tiles && aov) {  // every device but the owner sends a -0 map (its frameN / frameP, device 0's in place)
      for (int i = 0; i < nd; i++) {
        sail_ctx* s = g->subs[i];
        HIPCHK(g, hipSetDevice(s->device));
        if (int rc = ensureFrame(s)) return relay(g, rc, s);
        if (!plan[i].send_own_aovs) {
          if (s->frameN) HIPCHK(g, fillNegZero(s->frameN, np, s->stream));
          if (s->frameP) HIPCHK(g, fillNegZero(s->frameP, np, s->stream));
        }
      }
    }
    int e = g_rccl.groupStart();
    for (int i = 0; i < nd && e == 0; i++) {
      sail_ctx* s = g->subs[i];
      if (hipSetDevice(s->device) != hipSuccess) { e = -1; break; }
      e = g_rccl.reduce(s->accum, i == 0 ? r->frame : s->accum, np * 4, kNcclFloat32, kNcclSum, 0, g->groupComms[i], s->stream);
      const bool own = plan[i].send_own_aovs != 0;  // the send buffer of this device's AOV maps
      if (e == 0 && s->aovN)
        e = g_rccl.reduce(own ? s->aovN : s->frameN, i == 0 ? r->frameN : (own ? s->aovN : s->frameN), np * 4,
                          kNcclFloat32, kNcclSum, 0, g->groupComms[i], s->stream);
      if (e == 0 && s->aovP)
        e = g_rccl.reduce(own ? s->aovP : s->frameP, i == 0 ? r->frameP : (own ? s->aovP : s->frameP), np * 4,
                          kNcclFloat32, kNcclSum, 0, g->groupComms[i], s->stream);
    }
    const int e2 = g_rccl.groupEnd();
    if (e || e2) return fail(g, SAIL_E_RCCL, "grouped ncclReduce: %s", g_rccl.errStr ? g_rccl.errStr(e ? e : e2) : "?");
    HIPCHK(g, hipSetDevice(r->device));
    if (int rc = groupCommCheck(g)) return rc;
  }
  r->reduced = true;
  g->dirty = false;
  return SAIL_OK;
}

// Host copy of a whole-frame accumulator keeping only what partition (rank, world, mode) holds: its own tiles, or
// (sample partition) everything on rank 0 and nothing elsewhere (sail_load_accum part -1, sail_plan_keep)
void keepPart(int W, int H, int rank, int world, int mode, const float* sums, float* out) {
  const size_t np = (size_t)W * H;
  if (world <= 1 || (mode == SAIL_PART_SAMPLES && rank == 0)) {
    if (out != sums) memmove(out, sums, np * 4 * sizeof(float));
    return;
  }
  if (mode == SAIL_PART_SAMPLES) { memset(out, 0, np * 4 * sizeof(float)); return; }
  const int tx = (W + 63) / 64;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const size_t i = ((size_t)y * W + x) * 4;
      if (((y >> 6) * tx + (x >> 6)) % world != rank) memset(out + i, 0, 4 * sizeof(float));
      else if (out != sums) memcpy(out + i, sums + i, 4 * sizeof(float));
    }
}

}  // namespace

extern "C" {

int sail_abi_version(void) { return SAIL_ABI_VERSION; }

int sail_filter_ms(sail_ctx* c, double* ms) {
  if (!c || !ms) return SAIL_E_INVALID;
  if (!c->subs.empty()) return sail_filter_ms(c->subs[0], ms);
  *ms = c->lastFilterMs;
  return SAIL_OK;
}

int sail_kernel_name(sail_ctx* c, char* name, int len) {
  if (!c || !name || len <= 0) return SAIL_E_INVALID;
  if (!c->subs.empty()) return relay(c, sail_kernel_name(c->subs[0], name, len), c->subs[0]);
  if (!c->haveScene) return fail(c, SAIL_E_STATE, "sail_kernel_name: no scene");
  const int set = kernelSetFor(c);
  const char* k = set == SAIL_KSET_CORNELL ? "sail_trace_kernel_cornell"
                  : set == SAIL_KSET_ROOM ? "sail_trace_kernel_room"
                  : (c->n >= c->cullMinPrims ? "sail_trace_kernel_cull" : "sail_trace_kernel");
  // the last launch's form: sample groups run the _grouped kernel followed by sail_accum_kernel
  if (c->lastWavefront) k = "sail_wf_*";
  else if (c->lastJit) k = c->lastJitMode == SAIL_JIT_MODE_CULL ? "sail_trace_kernel_cull_jit" : "sail_trace_kernel_jit";
  snprintf(name, (size_t)len, "%s%s", k, (!c->lastWavefront && c->lastGroups > 1) ? "_grouped" : "");
  return SAIL_OK;
}

int sail_get_kernel_info(sail_ctx* c, sail_kernel_info* out) {
  if (!c || !out) return SAIL_E_INVALID;
  if (!c->subs.empty()) return relay(c, sail_get_kernel_info(c->subs[0], out), c->subs[0]);
  memset(out, 0, sizeof *out);
  if (int rc = sail_kernel_name(c, out->name, (int)sizeof out->name)) return rc;
  out->build_id = c->lastJit ? c->lastBuildId : sail_precompiled_build_id(out->name);
  if (c->jitState == SAIL_KERNEL_JIT_PENDING) {  // poll the background build (loads the module when it is done)
    SailJitKernel k;
    int m;
    (void)jitKernels(c, 0, &k, &m);
  }
  out->jit_state = c->jitState;
  out->jit_build_id = c->jitState == SAIL_KERNEL_JIT_READY ? c->jitK.buildId : 0;
  out->jit_compile_ms = c->jitK.compileMs;
  out->jit_from_cache = c->jitK.fromCache;
  snprintf(out->jit_error, sizeof out->jit_error, "%s", c->jitError.c_str());
  return SAIL_OK;
}

int sail_kernel_ready(sail_ctx* c, int timeout_ms, int* ready) {
  if (!c || !ready || timeout_ms < -1) return SAIL_E_INVALID;
  *ready = 0;
  if (!c->subs.empty()) {
    int all = 1;
    for (sail_ctx* s : c->subs) {
      int r = 0;
      if (int rc = sail_kernel_ready(s, timeout_ms, &r)) return relay(c, rc, s);
      all &= r;
    }
    *ready = all;
    return SAIL_OK;
  }
  if (!c->haveScene) return fail(c, SAIL_E_STATE, "sail_kernel_ready: no scene");
  SailJitKernel k;
  int m;
  *ready = jitKernels(c, timeout_ms, &k, &m) ? 1 : 0;
  return SAIL_OK;
}

int sail_set_jit_cache(const char* dir) {
  sail_jit_set_cache_dir(dir);
  return SAIL_OK;
}

int sail_device_count(int* count) {
  if (!count) return SAIL_E_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return SAIL_OK;
}

int sail_device_info(int device, int* compute_units, int* clock_khz) {
  if (!compute_units || !clock_khz) return SAIL_E_INVALID;
  int cus = 0, khz = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, device) != hipSuccess)
    return SAIL_E_HIP;
  *compute_units = cus;
  *clock_khz = khz;
  return SAIL_OK;
}

const char* sail_last_error(const sail_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int sail_create(sail_ctx** out, int width, int height, int device, uint32_t flags) {
  if (!out || width <= 0 || height <= 0 || width > 32768 || height > 32768)
    return fail(nullptr, SAIL_E_INVALID, "sail_create: bad arguments %dx%d", width, height);
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(nullptr, SAIL_E_NODEVICE, "no HIP device");
  if (device < 0) { if (hipGetDevice(&device) != hipSuccess) device = 0; }
  if (device >= ndev) return fail(nullptr, SAIL_E_INVALID, "device %d out of range (%d devices)", device, ndev);
  sail_ctx* c = new sail_ctx();
  c->device = device; c->W = width; c->H = height; c->flags = flags;
  auto bail = [&](int code, const char* what) {
    g_create_error = std::string("sail_create: ") + what;
    sail_destroy(c);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(SAIL_E_HIP, "hipSetDevice");
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) c->numCUs = cus;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(SAIL_E_HIP, "stream");
  const size_t bytes = (size_t)width * height * sizeof(float4);
  if (hipMalloc(&c->accum, bytes) != hipSuccess) return bail(SAIL_E_OOM, "accumulator");
  if (flags & SAIL_FLAG_AOV) {
    if (hipMalloc(&c->aovN, bytes) != hipSuccess || hipMalloc(&c->aovP, bytes) != hipSuccess) return bail(SAIL_E_OOM, "aov");
  }
  if (flags & SAIL_FLAG_SEGMENT_COUNT) {
    if (hipMalloc(&c->segCounter, SAIL_SEG_SLOTS * sizeof(unsigned long long)) != hipSuccess) return bail(SAIL_E_OOM, "counter");
  }
  if (resetAccum(c) != SAIL_OK) return bail(SAIL_E_HIP, c->err.c_str());
  if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(SAIL_E_HIP, "sync");
  *out = c;
  return SAIL_OK;
}

void sail_destroy(sail_ctx* c) {
  if (!c) return;
  if (!c->subs.empty()) {
    for (sail_ctx* s : c->subs) if (s) { (void)hipSetDevice(s->device); (void)hipStreamSynchronize(s->stream); }
    for (nccl_comm_t cm : c->groupComms) if (cm && g_rccl.commDestroy) g_rccl.commDestroy(cm);
    for (sail_ctx* s : c->subs) sail_destroy(s);
    delete c;
    return;
  }
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->jitHave) sail_jit_hold(c->device, c->jitSpec, -1);  // its queued build, if any, is no longer needed
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm && g_rccl.commDestroy) g_rccl.commDestroy(c->comm);
  for (auto& pr : c->pending) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  for (auto e : c->evPool) (void)hipEventDestroy(e);
  void* bufs[] = {c->accum, c->frame, c->frameN, c->frameP, c->aovN, c->aovP, c->filterOut, c->filterOut8, c->stage, c->segCounter, c->prims, c->tp, c->lt, c->lightObjRow, c->samples, c->wf};
  for (void* b : bufs) if (b) (void)hipFree(b);
  if (c->samplesPinned) (void)hipHostFree(c->samplesPinned);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int sail_create_multi(sail_ctx** out, int width, int height, const int* devices, int n_devices, uint32_t flags) {
  if (!out || n_devices < 1 || n_devices > 64)
    return fail(nullptr, SAIL_E_INVALID, "sail_create_multi: bad arguments (%d devices)", n_devices);
  *out = nullptr;
  std::vector<int> dev((size_t)n_devices);
  for (int i = 0; i < n_devices; i++) dev[i] = devices ? devices[i] : i;
  for (int i = 0; i < n_devices; i++)  // a negative ordinal is the current device (sail_create's rule), resolved first
    if (dev[i] < 0 && hipGetDevice(&dev[i]) != hipSuccess) return fail(nullptr, SAIL_E_HIP, "sail_create_multi: hipGetDevice");
  bool allSame = true, allDistinct = true;
  for (int i = 0; i < n_devices; i++)
    for (int j = 0; j < n_devices; j++) {
      if (dev[i] != dev[j]) allSame = false;
      if (i != j && dev[i] == dev[j]) allDistinct = false;
    }
  if (!allSame && !allDistinct)
    return fail(nullptr, SAIL_E_INVALID, "sail_create_multi: devices must be all distinct or all the same one");
  sail_ctx* g = new sail_ctx();
  g->W = width; g->H = height; g->flags = flags; g->device = dev[0];
  g->world = n_devices;
  g->groupLocal = n_devices > 1 && allSame;
  for (int i = 0; i < n_devices; i++) {
    sail_ctx* s = nullptr;
    int rc = sail_create(&s, width, height, dev[i], flags);
    if (rc == SAIL_OK) g->subs.push_back(s);
    if (rc == SAIL_OK) rc = sail_set_partition(s, i, n_devices, SAIL_PART_TILES);
    if (rc != SAIL_OK) {
      const std::string msg = s ? s->err : g_create_error;
      sail_destroy(g);
      return fail(nullptr, rc, "sail_create_multi: device %d: %s", dev[i], msg.c_str());
    }
  }
  if (n_devices > 1 && allDistinct) {
    if (!g_rccl.load()) { sail_destroy(g); return fail(nullptr, SAIL_E_RCCL, "sail_create_multi: librccl not loadable"); }
    g->groupComms.assign((size_t)n_devices, nullptr);
    const int r = g_rccl.commInitAll(g->groupComms.data(), n_devices, dev.data());
    if (r) {
      g->groupComms.clear();
      sail_destroy(g);
      return fail(nullptr, SAIL_E_RCCL, "ncclCommInitAll: %s", g_rccl.errStr ? g_rccl.errStr(r) : "?");
    }
  }
  *out = g;
  return SAIL_OK;
}

int sail_set_debug(sail_ctx* c, int option, int value) {
  if (!c) return SAIL_E_INVALID;
  if (option == SAIL_DEBUG_FORCE_RCCL) {  // the multi-device context's own communicator, not its devices'
    if (c->subs.empty() || c->groupLocal)
      return fail(c, SAIL_E_INVALID, "SAIL_DEBUG_FORCE_RCCL needs a multi-device context of distinct devices");
    for (sail_ctx* s : c->subs) if (int rc = flushQueued(s)) return relay(c, rc, s);
    const int nd = (int)c->subs.size();
    if (value && c->groupComms.empty()) {
      if (!g_rccl.load()) return fail(c, SAIL_E_RCCL, "librccl not loadable");
      std::vector<int> dev((size_t)nd);
      for (int i = 0; i < nd; i++) dev[i] = c->subs[i]->device;
      c->groupComms.assign((size_t)nd, nullptr);
      const int r = g_rccl.commInitAll(c->groupComms.data(), nd, dev.data());
      if (r) {
        c->groupComms.clear();
        return fail(c, SAIL_E_RCCL, "ncclCommInitAll: %s", g_rccl.errStr ? g_rccl.errStr(r) : "?");
      }
    } else if (!value && nd == 1 && !c->groupComms.empty()) {
      for (sail_ctx* s : c->subs) { (void)hipSetDevice(s->device); (void)hipStreamSynchronize(s->stream); }
      for (nccl_comm_t cm : c->groupComms) if (cm) g_rccl.commDestroy(cm);
      c->groupComms.clear();
    }
    c->dirty = true;
    return SAIL_OK;
  }
  for (sail_ctx* s : c->subs) if (int rc = sail_set_debug(s, option, value)) return relay(c, rc, s);
  if (int rc = flushQueued(c)) return rc;  // queued samples launch with the settings they were queued under
  switch (option) {
    case SAIL_DEBUG_CULL_MIN_PRIMS: c->cullMinPrims = value; break;
    case SAIL_DEBUG_FORCE_GENERIC: c->forceGeneric = value; break;
    case SAIL_DEBUG_CULL_FMA: c->cullFma = value; break;
    case SAIL_DEBUG_SAMPLE_GROUPS: c->forceGroups = value; break;
    case SAIL_DEBUG_WAVEFRONT: c->wavefront = value; break;
    case SAIL_DEBUG_JIT: c->jit = value; break;
    case SAIL_DEBUG_JIT_NT:
      if (value != 0 && value != 128 && value != 256 && value != 512 && value != 1024)
        return fail(c, SAIL_E_INVALID, "sail_set_debug: threads per workgroup must be 0 (default), 128, 256, 512 or 1024");
      c->jitNt = value;
      break;
    case SAIL_DEBUG_JIT_NS:
      if (value != 0 && value != 1 && value != 4 && value != 16)
        return fail(c, SAIL_E_INVALID, "sail_set_debug: samples in flight must be 0 (default), 1, 4 or 16");
      c->jitNs = value;
      break;
    case SAIL_DEBUG_JIT_WAIT:
      if (value < -1) return fail(c, SAIL_E_INVALID, "sail_set_debug: jit wait must be >= -1");
      c->jitWait = value;
      break;
    case SAIL_DEBUG_GROUP_ROUNDS:
      if (value <= 0) return fail(c, SAIL_E_INVALID, "sail_set_debug: group rounds must be > 0");
      c->flatGroupRounds = value;
      break;
    case SAIL_DEBUG_CULL_GROUP_ROUNDS:
      if (value <= 0) return fail(c, SAIL_E_INVALID, "sail_set_debug: group rounds must be > 0");
      c->cullGroupRounds = value;
      break;
    default: return fail(c, SAIL_E_INVALID, "sail_set_debug: unknown option %d", option);
  }
  refreshJit(c);  // the switches decide which run-time kernel (if any) the scene gets
  return SAIL_OK;
}

// The primitive buffer holds the decoded rows followed by the candidate sweep's per-type masks: for each chunk
// of 64 rows, 16 words whose bit j says row 64*chunk + j has shape type t (SailTraceArgs.typeMasks).
static size_t primBytes(int n) {
  const size_t chunks = (size_t)(n + 63) / 64;
  return sizeof(SailPrim) * (size_t)(n > 0 ? n : 1) + chunks * 16 * sizeof(unsigned long long);
}
static int uploadPrims(sail_ctx* c, const std::vector<SailPrim>& prims) {
  const int n = (int)prims.size();
  if (n <= 0) return SAIL_OK;
  const size_t chunks = (size_t)(n + 63) / 64;
  c->typeMasksHost.assign(chunks * 16, 0ull);
  for (int i = 0; i < n; i++)
    if (prims[i].type >= 0 && prims[i].type < 16) c->typeMasksHost[(size_t)(i / 64) * 16 + prims[i].type] |= 1ull << (i % 64);
  HIPCHK(c, hipMemcpyAsync(c->prims, prims.data(), sizeof(SailPrim) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->prims + n, c->typeMasksHost.data(), chunks * 16 * sizeof(unsigned long long),
                           hipMemcpyHostToDevice, c->stream));
  return SAIL_OK;
}

int sail_set_scene(sail_ctx* c, const float* objects, int n, const float* texparams, int tn, const float* lights,
                   int ln, const sail_plugins* plugins) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    for (sail_ctx* s : c->subs)
      if (int rc = sail_set_scene(s, objects, n, texparams, tn, lights, ln, plugins)) return relay(c, rc, s);
    c->haveScene = true; c->n = n; c->tn = tn; c->ln = ln; c->dirty = false;
    c->loadMissing = 0;  // every device's accumulation restarted: a half-loaded checkpoint is abandoned
    return SAIL_OK;
  }
  if (n < 0 || tn < 0 || ln < 0 || (n > 0 && !objects) || (tn > 0 && !texparams) || (ln > 0 && !lights) || !plugins)
    return fail(c, SAIL_E_INVALID, "sail_set_scene: bad arguments (n=%d tn=%d ln=%d)", n, tn, ln);
  if (n > 0 && tn < 1) return fail(c, SAIL_E_INVALID, "sail_set_scene: objects need texParams rows");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->plugins = *plugins;
  c->lastGroups = 1;
  c->lastWavefront = false;
  c->lastJit = false;
  std::vector<SailPrim> prims;
  decodePrims(objects, n, tn, plugins->shape_mask, prims, &c->shadowAnyHit, &c->scene);
  fillCats(prims, texparams, tn);
  c->primExtent = primExtent(prims);
  c->primTypes.clear();
  for (const SailPrim& q : prims) c->primTypes.push_back(q.type);
  // per light row: the geometry row an AreaLight samples (area.glsl:8 + shader.shape.js:56)
  std::vector<int32_t> lrow((size_t)(ln > 0 ? ln : 1), 0);
  TexView lv{lights, 18, ln};
  for (int r = 0; r < ln; r++) {
    const float rc = (ln == 1) ? NAN : gdiv((float)r, (float)(ln - 1));
    const int gi = to_int(lv.readFloat(1.0f, rc, 17.0f));
    lrow[r] = (n > 0) ? texel(gdiv((float)gi, (float)(n - 1)), n) : 0;
  }
  void* old[] = {c->prims, c->tp, c->lt, c->lightObjRow};
  for (void* b : old) if (b) HIPCHK(c, hipFree(b));
  c->prims = nullptr; c->tp = nullptr; c->lt = nullptr; c->lightObjRow = nullptr;
  const size_t pb = primBytes(n), tb = sizeof(float) * 16 * (size_t)(tn > 0 ? tn : 1),
               lb = sizeof(float) * 18 * (size_t)(ln > 0 ? ln : 1), rb = sizeof(int32_t) * lrow.size();
  if (hipMalloc(&c->prims, pb) != hipSuccess || hipMalloc(&c->tp, tb) != hipSuccess || hipMalloc(&c->lt, lb) != hipSuccess ||
      hipMalloc(&c->lightObjRow, rb) != hipSuccess)
    return fail(c, SAIL_E_OOM, "scene buffers");
  HIPCHK(c, hipMemsetAsync(c->tp, 0, tb, c->stream));
  HIPCHK(c, hipMemsetAsync(c->lt, 0, lb, c->stream));
  if (int rc = uploadPrims(c, prims)) return rc;
  if (tn > 0) HIPCHK(c, hipMemcpyAsync(c->tp, texparams, sizeof(float) * 16 * tn, hipMemcpyHostToDevice, c->stream));
  if (ln > 0) HIPCHK(c, hipMemcpyAsync(c->lt, lights, sizeof(float) * 18 * ln, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->lightObjRow, lrow.data(), rb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->objectsRows.assign(objects, objects + (size_t)n * 18);
  c->tpRows.assign(texparams, texparams + (size_t)tn * 16);
  c->n = n; c->tn = tn; c->ln = ln;
  c->haveScene = true;
  // Tracer.update links the scene's program (tracer.js:42-90): the plugin set's kernel starts building now, in the
  // background; the precompiled kernel of the set serves until it is loaded
  refreshJit(c);
  return resetAccum(c);
}

int sail_update_objects(sail_ctx* c, const float* objects, int n) {
  if (c && !c->subs.empty()) {
    for (sail_ctx* s : c->subs) if (int rc = sail_update_objects(s, objects, n)) return relay(c, rc, s);
    c->dirty = false;
    c->loadMissing = 0;
    return SAIL_OK;
  }
  if (!c || !c->haveScene) return c ? fail(c, SAIL_E_STATE, "sail_update_objects before sail_set_scene") : SAIL_E_INVALID;
  if (n != c->n || !objects) return fail(c, SAIL_E_INVALID, "sail_update_objects: n must stay %d", c->n);
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<SailPrim> prims;
  decodePrims(objects, n, c->tn, c->plugins.shape_mask, prims, &c->shadowAnyHit, &c->scene);
  fillCats(prims, c->tpRows.data(), c->tn);
  c->primExtent = primExtent(prims);
  c->primTypes.clear();
  for (const SailPrim& q : prims) c->primTypes.push_back(q.type);  // a kernel compiled for the rows follows them
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (int rc = uploadPrims(c, prims)) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->objectsRows.assign(objects, objects + (size_t)n * 18);
  refreshJit(c);  // a drag keeps the kernel; a changed shape type starts the new rows' kernel building
  return resetAccum(c);
}

int sail_set_accum_mode(sail_ctx* c, int mode) {
  if (!c) return SAIL_E_INVALID;
  if (mode < SAIL_ACCUM_SUM || mode > SAIL_ACCUM_COMPAT8) return fail(c, SAIL_E_INVALID, "accum mode %d", mode);
  if (!c->subs.empty()) {
    for (sail_ctx* s : c->subs) if (int rc = sail_set_accum_mode(s, mode)) return relay(c, rc, s);
    c->accumMode = mode; c->dirty = false;
    c->loadMissing = 0;
    return SAIL_OK;
  }
  if (mode != SAIL_ACCUM_SUM && c->partMode == SAIL_PART_SAMPLES && c->world > 1)
    return fail(c, SAIL_E_INVALID, "running-mean accumulation cannot be split by samples");
  HIPCHK(c, hipSetDevice(c->device));
  c->accumMode = mode;
  return resetAccum(c);
}

int sail_set_partition(sail_ctx* c, int rank, int world, int mode) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {  // the devices of one context split the frame among themselves: only the mode is chosen
    if (rank != 0 || world != 1 || (mode != SAIL_PART_TILES && mode != SAIL_PART_SAMPLES))
      return fail(c, SAIL_E_INVALID, "multi-device context: partition must be (0, 1, mode), got (%d, %d, %d)", rank, world, mode);
    const int nd = (int)c->subs.size();
    for (int i = 0; i < nd; i++) if (int rc = sail_set_partition(c->subs[i], i, nd, mode)) return relay(c, rc, c->subs[i]);
    c->partMode = mode; c->dirty = false;
    c->loadMissing = 0;
    return SAIL_OK;
  }
  if (world < 1 || rank < 0 || rank >= world || (mode != SAIL_PART_TILES && mode != SAIL_PART_SAMPLES))
    return fail(c, SAIL_E_INVALID, "partition rank=%d world=%d mode=%d", rank, world, mode);
  if (mode == SAIL_PART_SAMPLES && world > 1 && c->accumMode != SAIL_ACCUM_SUM)
    return fail(c, SAIL_E_INVALID, "sample partition needs SAIL_ACCUM_SUM");
  HIPCHK(c, hipSetDevice(c->device));
  c->rank = rank; c->world = world; c->partMode = mode;
  refreshJit(c);  // the Cornell form's samples in flight follow the share of the frame (jitNsFor)
  return resetAccum(c);
}

int sail_set_launch_samples(sail_ctx* c, int spp) {
  if (!c) return SAIL_E_INVALID;
  if (spp < 0 || spp > 1 << 20) return fail(c, SAIL_E_INVALID, "launch samples %d", spp);  // 0: by form
  for (sail_ctx* s : c->subs) if (int rc = sail_set_launch_samples(s, spp)) return relay(c, rc, s);
  if (int rc = flushQueued(c)) return rc;
  c->launchSpp = spp;
  return SAIL_OK;
}

int sail_render_schedule(sail_ctx* c, const float* inv, const float* seeds, const float eye[3], int spp, int maxBounces) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    // every device queues its share on its own stream; the host does not wait
    if (int rc = loadIncomplete(c, "sail_render_schedule")) return rc;
    for (sail_ctx* s : c->subs)
      if (int rc = sail_render_schedule(s, inv, seeds, eye, spp, maxBounces)) return relay(c, rc, s);
    c->dirty = true;
    return SAIL_OK;
  }
  if (!c->haveScene) return fail(c, SAIL_E_STATE, "sail_render before sail_set_scene");
  if (spp < 0 || (spp > 0 && (!inv || !seeds)) || !eye || maxBounces < 0 || maxBounces > 1024)
    return fail(c, SAIL_E_INVALID, "sail_render_schedule: bad arguments (spp=%d bounces=%d)", spp, maxBounces);
  if (int rc = flushQueued(c)) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  memcpy(c->eyeCache, eye, sizeof(float) * 3);
  c->hostSamples.clear();
  for (int s = 0; s < spp; s++) {
    const uint64_t k = c->k + (uint64_t)s;
    if (c->partMode == SAIL_PART_SAMPLES && c->world > 1 && (int)(k % (uint64_t)c->world) != c->rank) continue;
    SailSample S;
    memset(&S, 0, sizeof S);
    cornerDirs(inv + 16 * s, eye, S.d);
    S.seed = seeds[s];
    S.mixw = (float)((double)k / (double)(k + 1));  // tracer.js:97, f64 then uniform1f
    c->hostSamples.push_back(S);
  }
  const int rc = launchTrace(c, c->hostSamples.data(), (int)c->hostSamples.size(), maxBounces);
  if (rc) return rc;
  c->reduced = false;  // the frame of the last sail_reduce is stale now: reduce again to refresh it
  c->samplesThisRank += c->hostSamples.size();
  c->k += (uint64_t)spp;
  return SAIL_OK;
}

// One progressive sample (Renderer.render): queued, and launched with the samples queued after it once launchSpp of
// them are waiting or anything observes or changes the context (flushQueued). The sample's record is built now,
// from the sample index it is given now, exactly as sail_render_schedule builds it.
int sail_render(sail_ctx* c, const float inv[16], const float eye[3], float seed, int maxBounces) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    if (int rc = loadIncomplete(c, "sail_render")) return rc;
    for (sail_ctx* s : c->subs) if (int rc = sail_render(s, inv, eye, seed, maxBounces)) return relay(c, rc, s);
    c->dirty = true;
    return SAIL_OK;
  }
  if (!c->haveScene) return fail(c, SAIL_E_STATE, "sail_render before sail_set_scene");
  if (!inv || !eye || maxBounces < 0 || maxBounces > 1024)
    return fail(c, SAIL_E_INVALID, "sail_render: bad arguments (bounces=%d)", maxBounces);
  // a launch has one eye (its pre-cull decisions) and one bounce count
  if (!c->queued.empty() && (maxBounces != c->queuedBounces || memcmp(eye, c->eyeCache, sizeof(float) * 3) != 0))
    if (int rc = flushQueued(c)) return rc;
  memcpy(c->eyeCache, eye, sizeof(float) * 3);
  c->queuedBounces = maxBounces;
  const uint64_t k = c->k;
  if (!(c->partMode == SAIL_PART_SAMPLES && c->world > 1 && (int)(k % (uint64_t)c->world) != c->rank)) {
    SailSample S;
    memset(&S, 0, sizeof S);
    cornerDirs(inv, eye, S.d);
    S.seed = seed;
    S.mixw = (float)((double)k / (double)(k + 1));  // tracer.js:97, f64 then uniform1f
    c->queued.push_back(S);
    c->samplesThisRank++;
  }
  c->k++;
  c->reduced = false;
  // one-sample frames launch 64 at a time unless the host fixed the launch size: the host keeps queueing the next
  // frames while a launch runs (a whole 1,024-frame queue launched at once left the GPU idle meanwhile: the JS host's
  // render() per frame at 85,391 against 91,161 Msamples/s, profiles/r05_bench_js_host*.json)
  if ((int)c->queued.size() >= (c->launchSpp > 0 ? c->launchSpp : 64)) return flushQueued(c);
  return SAIL_OK;
}

int sail_reset(sail_ctx* c) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    for (sail_ctx* s : c->subs) if (int rc = sail_reset(s)) return relay(c, rc, s);
    c->dirty = false;
    c->loadMissing = 0;
    return SAIL_OK;
  }
  HIPCHK(c, hipSetDevice(c->device));
  return resetAccum(c);
}

int sail_sync(sail_ctx* c) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    for (sail_ctx* s : c->subs) if (int rc = sail_sync(s)) return relay(c, rc, s);
    return groupCommCheck(c);
  }
  if (int rc = flushQueued(c)) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (int rc = commCheck(c, c->comm)) return rc;
  return collectEvents(c);
}

int sail_read_accum(sail_ctx* c, float* rgba) {
  if (!c || !rgba) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    if (int rc = loadIncomplete(c, "sail_read_accum")) return rc;
    if (int rc = groupReduce(c)) return rc;
    return relay(c, sail_read_accum(c->subs[0], rgba), c->subs[0]);
  }
  int rc = sail_sync(c);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy(rgba, shownAccum(c), (size_t)c->W * c->H * sizeof(float4), hipMemcpyDeviceToHost));
  return SAIL_OK;
}

int sail_readback(sail_ctx* c, float* rgba, float* normal, float* position) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    if (int rc = loadIncomplete(c, "sail_readback")) return rc;
    if (int rc = groupReduce(c)) return rc;
    return relay(c, sail_readback(c->subs[0], rgba, normal, position), c->subs[0]);
  }
  int rc = sail_sync(c);
  if (rc) return rc;
  const size_t np = (size_t)c->W * c->H, bytes = np * sizeof(float4);
  if (rgba) {
    HIPCHK(c, hipMemcpy(rgba, shownAccum(c), bytes, hipMemcpyDeviceToHost));
    if (c->accumMode == SAIL_ACCUM_SUM) {
      for (size_t i = 0; i < np; i++) {
        const float cnt = rgba[4 * i + 3];
        if (cnt > 0.0f) { rgba[4 * i] /= cnt; rgba[4 * i + 1] /= cnt; rgba[4 * i + 2] /= cnt; }
        rgba[4 * i + 3] = 1.0f;
      }
    }
  }
  if (normal) {
    if (!c->aovN) return fail(c, SAIL_E_STATE, "AOVs not enabled (SAIL_FLAG_AOV)");
    HIPCHK(c, hipMemcpy(normal, shownAovN(c), bytes, hipMemcpyDeviceToHost));
  }
  if (position) {
    if (!c->aovP) return fail(c, SAIL_E_STATE, "AOVs not enabled (SAIL_FLAG_AOV)");
    HIPCHK(c, hipMemcpy(position, shownAovP(c), bytes, hipMemcpyDeviceToHost));
  }
  return SAIL_OK;
}

int sail_filter(sail_ctx* c, int kind, const float* weights16, float rx, float ry, float gammaC, float* out, uint8_t* out8) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    // the display pass runs on device 0 over the reduced frame
    if (int rc = loadIncomplete(c, "sail_filter")) return rc;
    if (int rc = groupReduce(c)) return rc;
    return relay(c, sail_filter(c->subs[0], kind, weights16, rx, ry, gammaC, out, out8), c->subs[0]);
  }
  if (kind < SAIL_FILTER_COLOR || kind > SAIL_FILTER_POSITION || (kind == SAIL_FILTER_WINDOW && !weights16))
    return fail(c, SAIL_E_INVALID, "sail_filter: kind %d", kind);
  if (kind >= SAIL_FILTER_WAVELET && !c->aovN)
    return fail(c, SAIL_E_STATE, "sail_filter: kind %d reads the AOVs (create with SAIL_FLAG_AOV)", kind);
  HIPCHK(c, hipSetDevice(c->device));
  int rc = sail_sync(c);
  if (rc) return rc;
  const size_t np = (size_t)c->W * c->H;
  if (out && !c->filterOut && hipMalloc(&c->filterOut, np * sizeof(float4)) != hipSuccess) {
    c->filterOut = nullptr;
    return fail(c, SAIL_E_OOM, "filter output");
  }
  if (out8 && !c->filterOut8 && hipMalloc(&c->filterOut8, np * 4) != hipSuccess) {
    c->filterOut8 = nullptr;
    return fail(c, SAIL_E_OOM, "filter output");
  }
  float4* dOut = out ? c->filterOut : nullptr;
  uint8_t* dOut8 = out8 ? c->filterOut8 : nullptr;
  SailFilterArgs A;
  memset(&A, 0, sizeof A);
  A.accum = shownAccum(c); A.aovN = shownAovN(c); A.aovP = shownAovP(c);
  A.out = dOut; A.out8 = dOut8; A.W = c->W; A.H = c->H; A.kind = kind; A.accumMode = c->accumMode;
  if (weights16) memcpy(A.weights, weights16, sizeof A.weights);
  A.rx = rx; A.ry = ry; A.gammaC = gammaC;
  // window taps reach 0.875 r pixels (offsets (j + 0.5) r / 4, j < 4) + the bilinear footprint + rounding
  if (kind == SAIL_FILTER_WINDOW) {
    const float r = fmaxf(fabsf(rx), fabsf(ry));
    const int h = (r == r) ? (int)ceilf(0.875f * r) + 2 : 99;
    A.halo = h <= 8 ? h : 0;
  }
  hipEvent_t f0 = nullptr, f1 = nullptr;
  int rcE = getEvent(c, &f0);
  if (rcE == SAIL_OK) rcE = getEvent(c, &f1);
  if (rcE != SAIL_OK) return rcE;
  hipError_t e = hipEventRecord(f0, c->stream);
  if (e == hipSuccess) e = sail_launch_filter(A, c->stream);
  if (e == hipSuccess) e = hipEventRecord(f1, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) {
    float ms = 0.0f;
    e = hipEventElapsedTime(&ms, f0, f1);
    c->lastFilterMs = ms;
  }
  c->evPool.push_back(f0);
  c->evPool.push_back(f1);
  if (e == hipSuccess && out) e = hipMemcpy(out, dOut, np * sizeof(float4), hipMemcpyDeviceToHost);
  if (e == hipSuccess && out8) e = hipMemcpy(out8, dOut8, np * 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(c, SAIL_E_HIP, "sail_filter: %s", hipGetErrorString(e));
  return SAIL_OK;
}

int sail_pick(sail_ctx* c, const float* rays, int count, int32_t* index, float* t) {
  if (!c || count < 0 || (count > 0 && (!rays || !index || !t))) return SAIL_E_INVALID;
  if (!c->subs.empty()) return relay(c, sail_pick(c->subs[0], rays, count, index, t), c->subs[0]);
  if (!c->haveScene) return fail(c, SAIL_E_STATE, "sail_pick: no scene (call sail_set_scene first)");
  if (count == 0) return SAIL_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = sail_sync(c);
  if (rc) return rc;
  float* dRays = nullptr;
  void* dOut = nullptr;
  if (hipMalloc(&dRays, (size_t)count * 6 * sizeof(float)) != hipSuccess) return fail(c, SAIL_E_OOM, "pick rays");
  if (hipMalloc(&dOut, (size_t)count * 8) != hipSuccess) { (void)hipFree(dRays); return fail(c, SAIL_E_OOM, "pick out"); }
  int32_t* dIdx = (int32_t*)dOut;
  float* dT = (float*)((char*)dOut + (size_t)count * 4);
  hipError_t e = hipMemcpyAsync(dRays, rays, (size_t)count * 6 * sizeof(float), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = sail_launch_pick(c->prims, c->n, dRays, count, dIdx, dT, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(index, dIdx, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(t, dT, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(dRays);
  (void)hipFree(dOut);
  if (e != hipSuccess) return fail(c, SAIL_E_HIP, "sail_pick: %s", hipGetErrorString(e));
  return SAIL_OK;
}

int sail_get_stats(sail_ctx* c, sail_stats* s) {
  if (!c || !s) return SAIL_E_INVALID;
  if (!c->subs.empty()) {  // samples per pixel of the frame; work summed; time = the slowest device's
    memset(s, 0, sizeof *s);
    for (sail_ctx* d : c->subs) {
      sail_stats q;
      if (int rc = sail_get_stats(d, &q)) return relay(c, rc, d);
      s->samples = c->partMode == SAIL_PART_SAMPLES ? s->samples + q.samples : q.samples;
      s->segments += q.segments;
      s->nominal_segments += q.nominal_segments;
      s->kernel_ms = fmax(s->kernel_ms, q.kernel_ms);
      s->last_launch_ms = fmax(s->last_launch_ms, q.last_launch_ms);
      s->launches = q.launches > s->launches ? q.launches : s->launches;
    }
    return SAIL_OK;
  }
  int rc = sail_sync(c);
  if (rc) return rc;
  memset(s, 0, sizeof *s);
  s->samples = c->samplesThisRank;
  s->nominal_segments = c->nominalSegments;
  s->kernel_ms = c->kernelMs;
  s->last_launch_ms = c->lastLaunchMs;
  s->launches = c->launches;
  if (c->segCounter) {
    unsigned long long v[SAIL_SEG_SLOTS];
    HIPCHK(c, hipMemcpy(v, c->segCounter, sizeof v, hipMemcpyDeviceToHost));
    s->segments = 0;
    for (int i = 0; i < SAIL_SEG_SLOTS; i++) s->segments += v[i];
  }
  return SAIL_OK;
}

int sail_accum_device_ptr(sail_ctx* c, void** ptr, size_t* bytes) {
  if (!c || !ptr || !bytes) return SAIL_E_INVALID;
  if (!c->subs.empty()) return relay(c, sail_accum_device_ptr(c->subs[0], ptr, bytes), c->subs[0]);
  if (int rc = flushQueued(c)) return rc;  // the sums the caller's collective will read are queued on this stream
  *ptr = c->accum;
  *bytes = (size_t)c->W * c->H * sizeof(float4);
  return SAIL_OK;
}

int sail_comm_unique_id(char id[128]) {
  if (!id) return SAIL_E_INVALID;
  if (!g_rccl.load()) return fail(nullptr, SAIL_E_RCCL, "librccl not loadable");
  nccl_uid_t u;
  const int r = g_rccl.getUniqueId(&u);
  if (r) return fail(nullptr, SAIL_E_RCCL, "ncclGetUniqueId: %d", r);
  memcpy(id, u.internal, 128);
  return SAIL_OK;
}

int sail_comm_init(sail_ctx* c, const char id[128], int nranks, int rank) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return SAIL_E_INVALID;
  if (!c->subs.empty()) return fail(c, SAIL_E_STATE, "a multi-device context reduces over its own communicator");
  if (!g_rccl.load()) return fail(c, SAIL_E_RCCL, "librccl not loadable");
  HIPCHK(c, hipSetDevice(c->device));
  if (c->comm) {  // a second init replaces the communicator
    HIPCHK(c, hipStreamSynchronize(c->stream));
    g_rccl.commDestroy(c->comm);
    c->comm = nullptr;
    c->commRanks = 0; c->commRank = 0;
  }
  nccl_uid_t u;
  memcpy(u.internal, id, 128);
  const int r = g_rccl.commInitRank(&c->comm, nranks, u, rank);
  if (r) return fail(c, SAIL_E_RCCL, "ncclCommInitRank: %s", g_rccl.errStr ? g_rccl.errStr(r) : "?");
  c->commRanks = nranks; c->commRank = rank;
  return SAIL_OK;
}

int sail_reduce(sail_ctx* c, int root) {
  if (!c) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    if (root != 0) return fail(c, SAIL_E_INVALID, "multi-device context: the frame is reduced into device 0");
    if (int rc = loadIncomplete(c, "sail_reduce")) return rc;
    c->dirty = true;  // reduce now even if nothing was rendered since the last one
    return groupReduce(c);
  }
  if (!c->comm) return fail(c, SAIL_E_STATE, "sail_reduce before sail_comm_init");
  if (root < 0 || root >= c->commRanks) return fail(c, SAIL_E_INVALID, "sail_reduce: root %d of %d ranks", root, c->commRanks);
  if (int rc = flushQueued(c)) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const bool isRoot = c->commRank == root;
  const bool aov = c->aovN || c->aovP;
  // a sample split shows the AOVs of the rank that rendered the last sample: the others send -0 maps
  const bool own = planReduce(c->W, c->H, c->rank, c->world, c->partMode, c->k, root).send_own_aovs != 0;
  if (isRoot || (aov && !own)) { if (int rc = ensureFrame(c)) return rc; }
  const size_t np = (size_t)c->W * c->H, count = np * 4;
  if (aov && !own) {
    if (c->frameN) HIPCHK(c, fillNegZero(c->frameN, np, c->stream));
    if (c->frameP) HIPCHK(c, fillNegZero(c->frameP, np, c->stream));
  }
  // out of place into root's frame: every reduce sums the ranks' cumulative accumulators afresh
  float4* sendN = own ? c->aovN : c->frameN;
  float4* sendP = own ? c->aovP : c->frameP;
  int r = g_rccl.groupStart();
  if (r == 0) r = g_rccl.reduce(c->accum, isRoot ? c->frame : c->accum, count, kNcclFloat32, kNcclSum, root, c->comm, c->stream);
  if (r == 0 && c->aovN) r = g_rccl.reduce(sendN, isRoot ? c->frameN : sendN, count, kNcclFloat32, kNcclSum, root, c->comm, c->stream);
  if (r == 0 && c->aovP) r = g_rccl.reduce(sendP, isRoot ? c->frameP : sendP, count, kNcclFloat32, kNcclSum, root, c->comm, c->stream);
  const int r2 = g_rccl.groupEnd();
  if (r || r2) return fail(c, SAIL_E_RCCL, "ncclReduce: %s", g_rccl.errStr ? g_rccl.errStr(r ? r : r2) : "?");
  if (int rc = commCheck(c, c->comm)) return rc;
  c->reduced = isRoot;
  return SAIL_OK;
}

// ---- checkpoint / resume --------------------------------------------------------------------------------------------
int sail_accum_parts(sail_ctx* c, int* parts) {
  if (!c || !parts) return SAIL_E_INVALID;
  *parts = c->subs.empty() ? 1 : (int)c->subs.size();
  return SAIL_OK;
}

int sail_save_accum(sail_ctx* c, int part, float* sums, uint64_t* k) {
  if (!c || !sums || !k) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    if (int rc = loadIncomplete(c, "sail_save_accum")) return rc;
    if (part < 0 || part >= (int)c->subs.size()) return fail(c, SAIL_E_INVALID, "sail_save_accum: part %d of %d", part, (int)c->subs.size());
    return relay(c, sail_save_accum(c->subs[part], 0, sums, k), c->subs[part]);
  }
  if (part != 0) return fail(c, SAIL_E_INVALID, "sail_save_accum: part %d of 1", part);
  if (int rc = sail_sync(c)) return rc;
  HIPCHK(c, hipMemcpy(sums, c->accum, (size_t)c->W * c->H * sizeof(float4), hipMemcpyDeviceToHost));
  *k = c->k;
  return SAIL_OK;
}

int sail_load_accum(sail_ctx* c, int part, const float* sums, uint64_t k) {
  if (!c || !sums || k > (1ull << 53)) return SAIL_E_INVALID;
  if (!c->subs.empty()) {
    const int nd = (int)c->subs.size();
    if (part < -1 || part >= nd) return fail(c, SAIL_E_INVALID, "sail_load_accum: part %d of %d", part, nd);
    // one part of a checkpoint: the others must follow with the same k before the frame is used (sail_plan_load_part)
    uint64_t missing = c->loadMissing, loadK = c->loadK;
    if (planLoadPart(&missing, &loadK, nd, part, k) != SAIL_OK)
      return fail(c, SAIL_E_INVALID, "sail_load_accum: part %d has k %llu, the checkpoint being loaded %llu", part,
                  (unsigned long long)k, (unsigned long long)c->loadK);
    for (int i = 0; i < nd; i++) {  // part -1: each device keeps its share of the frame; else one part, every k
      if (part == -1 || part == i) {
        if (int rc = sail_load_accum(c->subs[i], part == -1 ? -1 : 0, sums, k)) return relay(c, rc, c->subs[i]);
      } else {
        c->subs[i]->k = k;
      }
    }
    c->loadMissing = missing;
    c->loadK = loadK;
    c->dirty = true;
    return SAIL_OK;
  }
  if (part != 0 && part != -1) return fail(c, SAIL_E_INVALID, "sail_load_accum: part %d of 1", part);
  if (part == -1 && c->world > 1 && c->partMode == SAIL_PART_SAMPLES && c->accumMode != SAIL_ACCUM_SUM)
    return fail(c, SAIL_E_INVALID, "sail_load_accum: a running mean cannot be split by samples");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = resetAccum(c)) return rc;  // queued samples, stats and AOVs restart; the accumulator is replaced
  std::vector<float> mine;
  const float* src = sums;
  if (part == -1 && c->world > 1) {
    mine.resize((size_t)c->W * c->H * 4);
    keepPart(c->W, c->H, c->rank, c->world, c->partMode, sums, mine.data());
    src = mine.data();
  }
  HIPCHK(c, hipMemcpyAsync(c->accum, src, (size_t)c->W * c->H * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->k = k;
  // this rank's samples among 0 .. k-1 (every one, or those k' = rank mod world of a sample split)
  c->samplesThisRank = planReduce(c->W, c->H, c->rank, c->world, c->partMode, k, 0).samples;
  return SAIL_OK;
}

int sail_jit_compile(const sail_plugins* plugins, int mode, const int32_t* row_types, int rows, void* code,
                     size_t* bytes) {
  if (!plugins || !bytes || mode < SAIL_JIT_MODE_FLAT || mode > SAIL_JIT_MODE_ROOM || rows < 0 ||
      rows > kSailJitMaxRows || (rows > 0 && !row_types))
    return SAIL_E_INVALID;
  // the plugin set's precompiled family, as kernelSetFor decides it for a flat scene of these masks
  const sail_plugins& p = *plugins;
  int set = SAIL_KSET_GENERIC;
  if ((p.shape_mask & ~SAIL_KSET_CORNELL_SHAPES) == 0 && (p.material_mask & ~SAIL_KSET_CORNELL_MATS) == 0 &&
      (p.texture_mask & ~SAIL_KSET_CORNELL_TEX) == 0 && p.light_mask == 0)
    set = SAIL_KSET_CORNELL;
  else if ((p.shape_mask & ~SAIL_KSET_ROOM_SHAPES) == 0)
    set = SAIL_KSET_ROOM;
  SailJitSpec spec;
  spec.ks = p.shape_mask; spec.km = p.material_mask; spec.kt = p.texture_mask; spec.kl = p.light_mask;
  spec.mode = mode;
  spec.waves = jitWaves(mode, mode == SAIL_JIT_MODE_CULL ? SAIL_KSET_GENERIC : set);
  spec.rows = rows;
  for (int i = 0; i < rows; i++) spec.types[i] = row_types[i];
  std::string err;
  if (sail_jit_code("gfx950", spec, code, bytes, &err))
    return fail(nullptr, SAIL_E_INVALID, "sail_jit_compile: %s", err.c_str());
  return SAIL_OK;
}

int sail_jit_prebuild(const float* objects, int n, const float* texparams, int tn, const float* lights, int ln,
                      const sail_plugins* plugins, const char* arch, const char* dir, int* built) {
  if (n < 0 || tn < 0 || ln < 0 || (n > 0 && !objects) || (tn > 0 && !texparams) || (ln > 0 && !lights) || !plugins ||
      !arch || (n > 0 && tn < 1))
    return fail(nullptr, SAIL_E_INVALID, "sail_jit_prebuild: bad arguments");
  (void)lights;
  // the spec a context with the product's defaults derives for this scene (jitSpecFor), without a device
  sail_ctx t;
  t.plugins = *plugins;
  t.n = n; t.tn = tn; t.ln = ln;
  t.haveScene = true;
  std::vector<SailPrim> prims;
  int anyHit = 0;
  decodePrims(objects, n, tn, plugins->shape_mask, prims, &anyHit, nullptr);
  for (const SailPrim& q : prims) t.primTypes.push_back(q.type);
  SailJitSpec spec;
  int mode = 0;
  if (built) *built = 0;
  if (!jitSpecFor(&t, &spec, &mode)) return SAIL_OK;  // the scene gets no run-time kernel
  std::string err;
  // the Cornell form in both shapes: 16 samples in flight (a large share of the frame) and 1 (a rank of 8, jitNsFor)
  const bool cornell = mode == SAIL_JIT_MODE_FLAT && kernelSetFor(&t) == SAIL_KSET_CORNELL;
  for (int ns : {16, 1}) {
    if (cornell) spec.ns = ns;
    if (sail_jit_code_to_dir(arch, spec, dir, &err)) return fail(nullptr, SAIL_E_INVALID, "sail_jit_prebuild: %s", err.c_str());
    if (!cornell) break;
  }
  if (built) *built = 1;
  return SAIL_OK;
}

int sail_prim_bounds(const float* objects, int n, int tn, float* out) {
  if (n < 0 || (n > 0 && (!objects || !out))) return SAIL_E_INVALID;
  std::vector<SailPrim> prims;
  int anyHit = 0;
  decodePrims(objects, n, tn, ~0u, prims, &anyHit, nullptr);
  for (int i = 0; i < n; i++) {
    const SailPrim& p = prims[(size_t)i];
    for (int k = 0; k < 3; k++) {
      out[6 * i + k] = p.type ? p.a[18 + k] : INFINITY;
      out[6 * i + 3 + k] = p.type ? p.a[21 + k] : -INFINITY;
    }
  }
  return SAIL_OK;
}

int sail_partition_tiles(int width, int height, int rank, int world, int* out, int capacity) {
  if (width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world || capacity < 0) return SAIL_E_INVALID;
  const int tx = (width + 63) / 64, ty = (height + 63) / 64;
  int count = 0;
  for (int t = rank; t < tx * ty; t += world) {
    if (out && count < capacity) {
      const int x0 = (t % tx) * 64, y0 = (t / tx) * 64;
      out[4 * count + 0] = x0;
      out[4 * count + 1] = y0;
      out[4 * count + 2] = (width - x0) < 64 ? (width - x0) : 64;
      out[4 * count + 3] = (height - y0) < 64 ? (height - y0) : 64;
    }
    count++;
  }
  return count;
}

int sail_plan_reduce(int width, int height, int rank, int world, int mode, uint64_t k, int root, sail_reduce_plan* out) {
  if (width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world || root < 0 || root >= world || !out ||
      (mode != SAIL_PART_TILES && mode != SAIL_PART_SAMPLES))
    return fail(nullptr, SAIL_E_INVALID, "sail_plan_reduce: bad arguments");
  *out = planReduce(width, height, rank, world, mode, k, root);
  return SAIL_OK;
}

int sail_plan_keep(int width, int height, int rank, int world, int mode, const float* sums, float* out) {
  if (width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world || !sums || !out ||
      (mode != SAIL_PART_TILES && mode != SAIL_PART_SAMPLES))
    return fail(nullptr, SAIL_E_INVALID, "sail_plan_keep: bad arguments");
  keepPart(width, height, rank, world, mode, sums, out);
  return SAIL_OK;
}

int sail_plan_load_part(uint64_t* missing, uint64_t* k, int parts, int part, uint64_t k_part) {
  if (!missing || !k) return fail(nullptr, SAIL_E_INVALID, "sail_plan_load_part: bad arguments");
  if (int rc = planLoadPart(missing, k, parts, part, k_part))
    return fail(nullptr, rc, "sail_plan_load_part: part %d of %d (index %llu, checkpoint %llu)", part, parts,
                (unsigned long long)k_part, (unsigned long long)*k);
  return SAIL_OK;
}

int sail_math_probe(int fn, const float* x, const float* y, float* out, int count) {
  if (!x || !y || !out || count < 0) return SAIL_E_INVALID;
  if (count == 0) return SAIL_OK;
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  const size_t b = sizeof(float) * count;
  if (hipMalloc(&dx, b) != hipSuccess || hipMalloc(&dy, b) != hipSuccess || hipMalloc(&dout, b) != hipSuccess) {
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    return fail(nullptr, SAIL_E_OOM, "math probe buffers");
  }
  hipError_t e = hipMemcpy(dx, x, b, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dy, y, b, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    e = sail_launch_math(fn, dx, dy, dout, count);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dout, b, hipMemcpyDeviceToHost);
  (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dout);
  if (e != hipSuccess) return fail(nullptr, SAIL_E_HIP, "math probe: %s", hipGetErrorString(e));
  return SAIL_OK;
}

}  // extern "C"
