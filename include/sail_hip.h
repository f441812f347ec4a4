/* sail_hip.h — C ABI of libsail_hip.so, the MI355X drop-in for Sail's per-frame GPU work.
 *
 * Sail drives its hot path through WebGL: Renderer.update(scene) -> Tracer.update uploads the scene
 * rows as R32F textures and links a generated trace program (src/core/tracer.js:42-90,
 * src/core/shader.js:58-76); Renderer.render(scene) -> Tracer.render sets the per-frame uniforms and
 * calls gl.drawArrays (src/core/tracer.js:92-101, src/core/webgl.js:51-93), then RenderShader.render
 * runs the display filter (src/core/renderer.js:54-72). Each entry point below names the reference
 * interface it replaces. Plain C types only; the caller owns every host pointer (valid for the call);
 * the library owns all device memory; no global state; a context is used from one thread.
 * Every function returns SAIL_OK (0) or a negative SAIL_E_* code; sail_last_error() gives text.
 * The JS host binds these through the N-API addon in sail_amd/js/native.
 */
#ifndef SAIL_HIP_H
#define SAIL_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAIL_ABI_VERSION 4

enum sail_status {
  SAIL_OK = 0,
  SAIL_E_INVALID = -1,   /* bad argument / shape mismatch */
  SAIL_E_HIP = -2,       /* HIP runtime error */
  SAIL_E_OOM = -3,       /* device allocation failed */
  SAIL_E_STATE = -4,     /* call out of order (e.g. render before set_scene) */
  SAIL_E_RCCL = -5,      /* collective failed or RCCL unavailable */
  SAIL_E_NODEVICE = -6   /* no HIP device */
};

/* sail_create flags */
enum sail_flags {
  SAIL_FLAG_AOV = 1u << 0,          /* keep the normal/position outputs (fstrace.glsl:15-16) */
  SAIL_FLAG_SEGMENT_COUNT = 1u << 1 /* exact in-kernel segment counter (sail_stats.segments) */
};
/* accumulation modes (sail_set_accum_mode) */
enum sail_accum_mode {
  SAIL_ACCUM_SUM = 0,    /* float4 sum + count; mean = sum / count (default, order-independent) */
  SAIL_ACCUM_MIX = 1,    /* the reference's running mean mix(e, prev, k/(k+1)) (fstrace.glsl:14) */
  SAIL_ACCUM_COMPAT8 = 2 /* MIX with the per-frame UNORM8 store of a WebGL2 RGB8 frame texture */
};
/* multi-GPU partition of one frame (sail_set_partition) */
enum sail_partition { SAIL_PART_TILES = 0, SAIL_PART_SAMPLES = 1 };
/* display filters (Scene.filter, src/shader/filter/shader.filter.js:18-30) */
enum sail_filter_kind {
  SAIL_FILTER_COLOR = 0, SAIL_FILTER_GAMMA = 1, SAIL_FILTER_TONEMAPPING = 2, SAIL_FILTER_WINDOW = 3,
  SAIL_FILTER_WAVELET = 4,  /* wavelet.glsl: a-trous over colour + position AOV (needs SAIL_FLAG_AOV) */
  SAIL_FILTER_NORMAL = 5,   /* normal.glsl: the normal AOV (needs SAIL_FLAG_AOV) */
  SAIL_FILTER_POSITION = 6  /* position.glsl: the position AOV (needs SAIL_FLAG_AOV) */
};

/* compiled plugin set (Scene.tracerConfig(), src/scene/scene.js:70-112), as bit masks over category ids:
 * shape bit = shape id (define.glsl:18-26), material bit = material id (:32-35), texture bit = texture id
 * (:38-44; UniformColor is always available), light bit = light id (:28-30). */
typedef struct sail_plugins {
  uint32_t shape_mask, material_mask, texture_mask, light_mask;
} sail_plugins;

typedef struct sail_stats {
  uint64_t samples;          /* samples accumulated since the last reset (this rank) */
  uint64_t segments;         /* exact segments traced (needs SAIL_FLAG_SEGMENT_COUNT) */
  uint64_t nominal_segments; /* pixels * samples * max_bounces of the launches since reset */
  double kernel_ms;          /* sum of trace-kernel durations (HIP events) since reset */
  double last_launch_ms;     /* duration of the most recent trace launch */
  uint32_t launches;         /* trace launches since reset */
} sail_stats;

typedef struct sail_ctx sail_ctx;

/* new Sail.Renderer(canvas) (src/core/renderer.js:9-39): one device, a W x H float accumulator.
 * device < 0 uses the current device. */
int sail_create(sail_ctx** out, int width, int height, int device, uint32_t flags);
/* new Sail.Renderer({devices: N}): ONE context over n_devices GPUs of this process (devices = NULL: 0..n-1).
 * The reference renders on one WebGL context (src/core/renderer.js:9-39, tracer.js:92-101); here the frame's
 * 64x64 tiles (or, after sail_set_partition(ctx, 0, 1, SAIL_PART_SAMPLES), its samples) are dealt across the
 * devices, each renders its share on its own stream, and readback / read_accum / filter first sum the devices'
 * accumulators into device 0 with one grouped RCCL reduce over a ncclCommInitAll communicator (progressive:
 * the sum is recomputed from the cumulative accumulators whenever something was rendered since). Every other
 * entry point fans out. Devices must be all distinct (RCCL over xGMI) or all the same one (the partition runs on
 * one GPU and a kernel sums it: the emulation the parity tests use). sail_comm_init is refused on it. */
int sail_create_multi(sail_ctx** out, int width, int height, const int* devices, int n_devices, uint32_t flags);
void sail_destroy(sail_ctx* ctx);
const char* sail_last_error(const sail_ctx* ctx); /* ctx may be NULL: last creation error */
int sail_device_count(int* count);
/* Device facts for reports (bench.py's roofline): compute units and peak engine clock in kHz. No reference
 * counterpart (WebGL exposes neither). */
int sail_device_info(int device, int* compute_units, int* clock_khz);

/* Tracer.update(scene) (src/core/tracer.js:42-90): the objects / texParams / lights rows exactly as
 * gen() serialises them (18 / 16 / 18 floats per row, Appendix A of SURVEY.md). Copied. */
int sail_set_scene(sail_ctx* ctx, const float* objects, int n, const float* texparams, int tn,
                   const float* lights, int ln, const sail_plugins* plugins);
/* Tracer.updateObjects(scene) (src/core/tracer.js:25-40): new object rows, same n; resets accumulation */
int sail_update_objects(sail_ctx* ctx, const float* objects, int n);

int sail_set_accum_mode(sail_ctx* ctx, int mode);        /* resets accumulation */
int sail_set_partition(sail_ctx* ctx, int rank, int world, int mode);
int sail_set_launch_samples(sail_ctx* ctx, int spp_per_launch); /* samples per kernel launch; 0 (default) = by kernel form: 1024 for the Cornell form with 16 samples in flight, else 64 */
/* Test / study switches (no reference counterpart; none changes a result, which the parity suite checks).
 * The product's defaults are the values in brackets. */
enum sail_debug_option {
  SAIL_DEBUG_CULL_MIN_PRIMS = 1, /* scenes with >= value primitives use the padded-box pre-cull kernel [8] */
  SAIL_DEBUG_FORCE_GENERIC = 2,  /* 1: always launch the all-plugin kernel [0] */
  SAIL_DEBUG_CULL_FMA = 3,       /* 0: the plain pre-cull slab form instead of the fused one [1] */
  SAIL_DEBUG_SAMPLE_GROUPS = 4,  /* > 0: fixed sample-group count per 16x16 block [0 = sized by occupancy] */
  /* multi-device contexts of distinct devices only: 1 builds the ncclCommInitAll communicator now even for ONE
   * device, so the grouped RCCL reduce (the path of N distinct GPUs) runs on a one-GPU machine [0: a one-device
   * context needs no reduce]. Refused (SAIL_E_INVALID) on a context whose devices are all the same GPU. */
  SAIL_DEBUG_FORCE_RCCL = 5,
  /* 1: scenes on the pre-cull path are traced by the wavefront split (one sample at a time, path state in HBM, sweep /
   * shade / shadow kernels per bounce) instead of the megakernel; same results [0] */
  SAIL_DEBUG_WAVEFRONT = 6,
  /* > 0: residency rounds of workgroups queued per launch when sizing the sample groups, flat kernels [36] and the
   * pre-cull kernel [64] (SAIL_DEBUG_SAMPLE_GROUPS overrides both) */
  SAIL_DEBUG_GROUP_ROUNDS = 7,
  SAIL_DEBUG_CULL_GROUP_ROUNDS = 8,
  /* which scenes run a kernel compiled by hipRTC for exactly their plugin set at sail_set_scene (the reference's
   * per-scene program, src/scene/scene.js:70-112), a sum of bits: 1 flat-path scenes (fewer than
   * SAIL_DEBUG_CULL_MIN_PRIMS primitives) that the precompiled Cornell and room kernels do not cover, 8 those as a
   * room-family kernel (SAIL_JIT_MODE_ROOM) instead of a plain one, 4 scenes of the room kernel's set, 2 pre-cull-path
   * scenes, 16 every flat-path scene of at most 8 primitives compiled for its rows too (their count and shape types).
   * 0: the precompiled kernels only. Same results [27 = 1 + 2 + 8 + 16; measured in profiles/r04_jit_*.jsonl] */
  SAIL_DEBUG_JIT = 9,
  /* how long (ms) a launch waits for the scene's run-time kernel while it is still being built in the background; -1:
   * until it is built. Meanwhile the precompiled kernel of the scene's set renders, with the same results [0: never
   * wait, so Renderer.update / render stay interactive; the Python binding used by the tests and bench.py sets -1] */
  SAIL_DEBUG_JIT_WAIT = 10,
  /* samples of each pixel in flight per workgroup of the run-time kernels: 1, 4 or 16 (the workgroup's lanes hold
   * 256 / value pixels, 1,024 / value in the pre-cull form, each with `value` samples); 0 = the form's default */
  SAIL_DEBUG_JIT_NS = 11,
  /* threads per workgroup of the run-time kernels: 128, 256, 512 or 1024 (the path sort's pool); 0 = the form's own
   * [0: 256 flat, 1,024 pre-cull] */
  SAIL_DEBUG_JIT_NT = 12
};
int sail_set_debug(sail_ctx* ctx, int option, int value);

/* Tracer.render(mvp, eye, k) (src/core/tracer.js:92-101) = one progressive sample with the caller's
 * jittered inverse matrix (16 f32, column-major as uniformMatrix4fv uploads it, webgl.js:103) and seed.
 * One-sample frames are queued and launched together (up to sail_set_launch_samples of them per launch) when
 * nothing observes the frame in between: every entry point that reads, filters, reduces, counts or changes the
 * context launches the queue first, and a change of eye or bounce count launches it before the new sample is
 * queued. The frame is bit-identical to one launch per call (samples are accumulated in the same order); a
 * launch error of a queued sample is reported by the call that launches it. */
int sail_render(sail_ctx* ctx, const float inv_mvp[16], const float eye[3], float time_seed, int max_bounces);
/* spp samples in one call: inv_mvp = spp x 16 floats, seeds = spp floats (a deterministic schedule). */
int sail_render_schedule(sail_ctx* ctx, const float* inv_mvp, const float* seeds, const float eye[3],
                         int spp, int max_bounces);
/* Renderer.render with scene.moving: sampleCount = 0 (src/core/renderer.js:57-60) */
int sail_reset(sail_ctx* ctx);
int sail_sync(sail_ctx* ctx);

/* mean image (W*H*4 f32, row 0 = bottom, like glReadPixels), optional AOVs (W*H*4 each) */
int sail_readback(sail_ctx* ctx, float* rgba, float* normal, float* position);
/* raw accumulator (SUM: rgb sums + count in .w; MIX: running mean) */
int sail_read_accum(sail_ctx* ctx, float* rgba);
/* RenderShader.render (src/core/renderer.js:63) -> pixelFilter (src/shader/filter/<kind>.glsl):
 * out_rgba = W*H*4 f32 (may be NULL), out_rgba8 = W*H*4 UNORM8 canvas pixels (may be NULL).
 * weights16 = the 16-entry window table (window filters), radius (rx, ry) in pixels, gamma_c for GAMMA. */
/* Pickup.pick (src/core/pickup.js:46-66) on the GPU: for each of `count` rays (origin xyz, direction xyz;
 * f32, 6 per ray) the trace kernel's own primitive sweep returns the first object row with the smallest
 * distance (-1 on a miss) and that distance (1e5 = MAX_DISTANCE on a miss). Replaces the reference's f64 CPU
 * picker (geometry.js intersect(), whose Rectangle test has the wrong plane) with the shader's intersection. */
int sail_pick(sail_ctx* ctx, const float* rays, int count, int32_t* index, float* t);
int sail_filter(sail_ctx* ctx, int kind, const float* weights16, float rx, float ry, float gamma_c,
                float* out_rgba, uint8_t* out_rgba8);
int sail_get_stats(sail_ctx* ctx, sail_stats* out);

/* ---- checkpoint / resume of a progressive render (no reference counterpart: the reference restarts its
 * accumulation on every camera or object change, src/core/renderer.js:57-60, src/scene/scene.js:65-68) ----
 * A context's accumulation is `parts` raw accumulators (1 for sail_create, one per device for sail_create_multi),
 * each W*H*4 f32 in sail_read_accum's layout, plus the global sample index k of the next sample. Saving every part
 * and loading them into a fresh context with the same size, scene, partition and accumulation mode continues the
 * render bit for bit: render k -> save -> new context -> load -> render k more == the 2k-sample frame. */
int sail_accum_parts(sail_ctx* ctx, int* parts);
/* copy accumulator `part` (this rank's own, never the reduced frame) and the sample index k */
int sail_save_accum(sail_ctx* ctx, int part, float* sums, uint64_t* k);
/* replace accumulator `part` by `sums` and set the sample index to k (every part of the context). part = -1 loads a
 * whole-frame accumulator (sail_read_accum of a reduced frame): on a multi-device context each device keeps its own
 * tiles of it (tile partition) or device 0 takes all of it (sample partition: equal to the uninterrupted render to
 * summation order only; load the parts for bit-exactness). The AOVs restart with the next sample. On a multi-device
 * context a part-wise load must be followed by every other part with the same k: until then rendering, reading,
 * filtering, saving and reducing fail with SAIL_E_STATE (sail_reset abandons the half-loaded checkpoint), and a part
 * with a different k fails with SAIL_E_INVALID. The caller checks the sums' size: W*H*4 floats. */
int sail_load_accum(sail_ctx* ctx, int part, const float* sums, uint64_t k);

/* ---- run-time compiled plugin-set kernels (Scene.tracerConfig -> Generator.generate, src/scene/scene.js:70-112,
 * src/shader/generator.js:107-123: the reference builds one program per scene plugin set) ----
 * Host only, no device needed: compile (hipRTC, gfx950) the trace kernel pair for exactly this plugin set in one of the
 * kernel forms below, from the kernel sources embedded in the library, with the product's floating-point flags.
 * *bytes = the code object's size; with code != NULL and *bytes large enough on entry it is copied there. The
 * contexts do the same at sail_set_scene (SAIL_DEBUG_JIT) and load the result on their device. */
enum sail_jit_mode {
  SAIL_JIT_MODE_FLAT = 0, /* flat path, the all-plugin kernel's form (6 waves per SIMD, three-barrier sort) */
  SAIL_JIT_MODE_CULL = 1, /* pre-cull path (1,024-thread workgroups) */
  SAIL_JIT_MODE_ROOM = 2  /* flat path, the room kernel's form (7 waves, two-barrier sort, first sample group at home) */
};
/* rows > 0 (at most 8, flat forms only): compile for a scene of exactly these rows, row_types[i] = the shape id of row i
 * (SAIL_CUBE ..., each in plugins->shape_mask): the primitive sweeps become straight-line code over the rows */
int sail_jit_compile(const sail_plugins* plugins, int mode, const int32_t* row_types, int rows, void* code,
                     size_t* bytes);
/* The reference links a scene's program inside Renderer.update in milliseconds (src/core/renderer.js:45-52 ->
 * tracer.js:42-90 -> webgl.js:165-192); a hipRTC compile takes seconds, so sail_set_scene / sail_update_objects only
 * START the build of the scene's run-time kernel, on a background thread, and return; launches use the precompiled
 * kernel of the scene's plugin set until the module is loaded (bit-identical frames). Code objects are cached on disk,
 * keyed by (arch, spec, kernel-source hash, compile flags, compiler version): a read-only cache beside the library
 * (<lib dir>/jit, filled by sail_jit_prebuild at build time) and the user's cache. A code object produced by another
 * compiler than the one that built the library is refused (the precompiled kernels serve). */
enum sail_kernel_jit_state {
  SAIL_KERNEL_JIT_NONE = 0,     /* the scene gets no run-time kernel (switches, or a precompiled kernel is exact) */
  SAIL_KERNEL_JIT_PENDING = 1,  /* being built in the background */
  SAIL_KERNEL_JIT_READY = 2,    /* loaded: launches use it */
  SAIL_KERNEL_JIT_FAILED = 3    /* could not be built or loaded (jit_error): the precompiled kernel serves */
};
typedef struct sail_kernel_info {
  char name[64];          /* the kernel the last launch ran (sail_kernel_name) */
  uint64_t build_id;      /* its build identity: FNV-1a 64 of the code object with the compiler's source-derived
                           * compilation-unit id masked (run-time kernels), or of the library image and the kernel's name
                           * (precompiled): profiles are matched to kernels by it */
  int jit_state;          /* sail_kernel_jit_state of the scene's run-time kernel */
  int jit_from_cache;     /* its code object came from 0: hipRTC in this process, 1: the user's disk cache, 2: the
                           * cache shipped beside the library */
  double jit_compile_ms;  /* hipRTC time of that code object (0 from a cache) */
  uint64_t jit_build_id;  /* the run-time kernel's build identity once READY */
  char jit_error[256];    /* why it FAILED */
} sail_kernel_info;
int sail_get_kernel_info(sail_ctx* ctx, sail_kernel_info* out);
/* *ready = 1 when the scene's run-time kernel is loaded (the next launch uses it), after waiting up to timeout_ms for
 * its build (-1: until done); 0 while it is still building, when none applies, or when it failed */
int sail_kernel_ready(sail_ctx* ctx, int timeout_ms, int* ready);
/* process-wide user cache directory of run-time code objects: NULL = default ($XDG_CACHE_HOME or $HOME/.cache, then
 * sail_amd/jit), "" = no user cache */
int sail_set_jit_cache(const char* dir);
/* Host only (no device): build the run-time kernel a context with the default switches derives for this scene (the rows
 * of sail_set_scene) for `arch`, into the cache directory `dir` (the shipped cache when dir is <lib dir>/jit). *built
 * (may be NULL) = 1 when the scene gets a run-time kernel, 0 when it does not. */
int sail_jit_prebuild(const float* objects, int n, const float* texparams, int tn, const float* lights, int ln,
                      const sail_plugins* plugins, const char* arch, const char* dir, int* built);

/* ---- host math of the reference, so every host language gets identical uniforms ---- */
/* Camera(eye, center, up) + makePerspective(fovy, aspect, near, far) (src/scene/camera.js:6-57):
 * P*MV (scene.mat, src/scene/scene.js:40-42) as 16 doubles, row-major */
int sail_camera(const double eye[3], const double center[3], const double up[3], double fovy, double aspect,
                double znear, double zfar, double mvp_rowmajor[16]);
/* inverse(Translation(jx/W, jy/H, 0) * mvp) flattened column-major in f32 (tracer.js:94-96, matrix.js:501-527) */
int sail_jitter_inverse(const double mvp_rowmajor[16], double jx, double jy, int width, int height, float inv_colmajor[16]);
/* The frozen deterministic schedule: sample k uses time_seed = 0.001*round(1000*(k+1)/60)
 * and jitter from xorshift32(0x5A11 + k). Fills spp x 16 matrices and spp seeds for k = k0 .. k0+spp-1. */
int sail_schedule(const double mvp_rowmajor[16], int width, int height, int k0, int spp, float* inv_colmajor, float* seeds);

/* Object3D.boundbox() (src/scene/geometry.js; the picker's pre-test, pickup.js:55-56), answered by the bounds the
 * trace kernels' pre-cull tests: for each of the n object rows (18 floats, Appendix A wire format; tn = the
 * texParams row count the rows index), 6 floats min.xyz, max.xyz of the padded box, +-inf where a primitive has no
 * finite bound; a row whose category is not a shape gets an empty box (+inf, -inf). Host-only (no device). */
int sail_prim_bounds(const float* objects, int n, int tn, float* out_minmax);

/* ---- multi-GPU (one process per GPU): image tiles / sample split + RCCL sum-reduce of the accumulators ---- */
int sail_comm_unique_id(char id[128]);
/* a second call replaces the communicator */
int sail_comm_init(sail_ctx* ctx, const char id[128], int nranks, int rank);
/* Sum of every rank's float4 accumulator (and, with SAIL_FLAG_AOV on a tile partition, of the AOV maps) into a
 * separate frame on `root`; collective: every rank calls it, all created with the same flags. The ranks'
 * accumulators are left as they are, so render -> reduce -> render -> reduce is progressive: each reduce sums
 * the cumulative accumulators afresh. On root, readback / read_accum / filter show that frame until the next
 * sail_render* or sail_reset (then this rank's own accumulator again). With a sample partition the AOVs shown are
 * those of the rank that rendered the frame's last sample, as on one GPU. Asynchronous RCCL errors are reported
 * here and by sail_sync (ncclCommGetAsyncError). On a multi-device context it reduces into device 0 (root 0). */
int sail_reduce(sail_ctx* ctx, int root);
/* this rank's own accumulator (device 0's on a multi-device context), never the reduced frame: since ABI v2 the
 * reduce is out of place, so after sail_reduce the pointer still holds rank-local sums */
int sail_accum_device_ptr(sail_ctx* ctx, void** ptr, size_t* bytes);
/* the 64x64 tiles rank `rank` of `world` owns in a W x H frame (tile t -> rank t % world), as
 * (x0, y0, w, h) quadruples; returns the tile count (or a negative error); out may be NULL to count */
int sail_partition_tiles(int width, int height, int rank, int world, int* out_xywh, int capacity);
/* Host only (no device): the bookkeeping both reduces follow -- sail_reduce (one process per GPU) and a multi-device
 * context's grouped reduce -- for rank `rank` of `world` under partition `mode` once k samples (global indices
 * 0 .. k-1) are rendered, the frame reduced into `root`. Both derive their choices from this function, so a host
 * language, or a test over gloo (tests/test_partition_gloo.py), plans the same exchange without a device. */
typedef struct sail_reduce_plan {
  int receives;       /* 1: this rank is `root`, where the reduced frame lands */
  int tiles;          /* 64x64 tiles this rank renders: tiles t = rank (mod world), or every tile (sample partition) */
  int aov_owner;      /* the rank whose AOV maps the frame shows: the one that rendered sample k-1 (sample partition; 0
                       * before any sample), or -1 for a tile partition (every rank owns its own tiles' maps) */
  int send_own_aovs;  /* 1: this rank reduces its own AOV maps; 0: it sends -0 maps, the additive identity that keeps
                       * every bit of the owner's maps (x + -0 == x for +-0 and NaN too) */
  uint64_t samples;   /* how many of the samples 0 .. k-1 this rank rendered: k for a tile partition, those with index
                       * = rank (mod world) for a sample partition */
} sail_reduce_plan;
int sail_plan_reduce(int width, int height, int rank, int world, int mode, uint64_t k, int root, sail_reduce_plan* out);
/* Host only: what rank `rank` keeps of a whole-frame accumulator when it resumes from it (sail_load_accum part -1):
 * its own tiles and zeros elsewhere, or for a sample partition all of it on rank 0 and zeros on the others. sums and
 * out hold W*H*4 floats (they may be the same buffer). */
int sail_plan_keep(int width, int height, int rank, int world, int mode, const float* sums, float* out);
/* Host only: one step of a part-wise checkpoint load over `parts` parts (sail_load_accum on a multi-device context).
 * *missing = bit mask of the parts still to load (0: no load in progress), *k = the checkpoint's sample index. Loading
 * part `part` saved at index k_part: the first part of a checkpoint sets *missing to every part and *k = k_part, then
 * clears its own bit; a later part with another index fails with SAIL_E_INVALID and leaves the state unchanged; part -1
 * (a whole frame) clears *missing. A frame is usable again once *missing is 0. */
int sail_plan_load_part(uint64_t* missing, uint64_t* k, int parts, int part, uint64_t k_part);

/* ---- diagnostics ---- */
/* evaluate the build's f32 math spec on the device (fn: 0 sin 1 cos 2 tan 3 atan2(y,x) 4 acos 5 pow(x,y)
 * 6 atan 7 sqrt 8 x/y); for the CPU/GPU bit-parity test */
int sail_math_probe(int fn, const float* x, const float* y, float* out, int count);
int sail_abi_version(void);
/* the trace kernel the context's current scene launches (a plugin-set specialisation, like the reference's
 * per-scene generated program): writes its name (e.g. "sail_trace_kernel_cornell") into name[len]; after a launch
 * that split its samples into groups, the "_grouped" form it ran (followed by sail_accum_kernel) */
int sail_kernel_name(sail_ctx* ctx, char* name, int len);
/* device time of the last sail_filter pass (HIP events around the kernel), for the stencil's roofline */
int sail_filter_ms(sail_ctx* ctx, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* SAIL_HIP_H */
