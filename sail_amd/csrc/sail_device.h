// sail_device.h — device-side data layout shared by the trace/filter kernels and the host library.
// All structs are POD, 16-byte aligned, and identical on host and device.
#pragma once
#if defined(__HIPCC_RTC__)  // hipRTC (sail_jit.cpp) has the fixed-width types in its runtime header's namespace
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#else
#include <stdint.h>
#endif

// Shape / material / texture / light category ids (src/shader/const/define.glsl:18-44)
enum {
  SAIL_CUBE = 1, SAIL_SPHERE = 2, SAIL_RECTANGLE = 3, SAIL_CONE = 4, SAIL_CYLINDER = 5, SAIL_DISK = 6,
  SAIL_HYPERBOLOID = 7, SAIL_PARABOLOID = 8, SAIL_CORNELLBOX = 9
};
enum { SAIL_AREA = 0, SAIL_POINT = 1, SAIL_SPOT = 2 };
enum { SAIL_MATTE = 1, SAIL_MIRROR = 2, SAIL_METAL = 3, SAIL_GLASS = 4 };
enum {
  SAIL_TEX_UNIFORM = 0, SAIL_TEX_CHECKERBOARD = 5, SAIL_TEX_CHECKERBOARD2 = 7, SAIL_TEX_BILERP = 8,
  SAIL_TEX_MIXF = 9, SAIL_TEX_SCALE = 10, SAIL_TEX_UVF = 11
};

// One decoded primitive: the row of the `objects` texture (tracer.js:45-52, webgl.js:137) resolved once on
// the host with the reference's texture-addressing rules (texhelper.glsl) into integer rows and typed
// parameters. 128 B, read by the primitive loop with a wave-uniform index (scalar loads).
struct __attribute__((aligned(16))) SailPrim {
  int32_t type;     // shape id, 0 when the shape's plugin is not compiled in (never hit)
  int32_t rev;      // reverseNormal (readBool: int(v) == 1)
  int32_t matRow;   // texParams row of the material (Cornellbox: slot 7 quirk resolved here)
  int32_t texRow;   // texParams row of the texture
  float em[3];      // emission (Cornellbox: forced BLACK, cornellbox.glsl:19)
  int32_t cats;     // int() of the material / texture category words (texParams[row][0]) clamped to [-1, 32]:
                    // low / high 16 bits (host-evaluated; every category test reads the same answer)
  float a[24];      // shape parameters in row order, per-scene constants, a[18..23] padded bounds (sail_capi.cpp)
};

// Per-sample uniforms (the reference's per-frame `matrix` + `timeSinceStart` + `textureWeight`,
// tracer.js:92-101) pre-reduced on the host to the 4 normalised corner directions the vertex
// shader produces (vstrace.glsl:4-6).
struct __attribute__((aligned(16))) SailSample {
  float d[4][3];    // corner directions v0=(-1,-1) v1=(-1,1) v2=(1,-1) v3=(1,1)
  float seed;       // timeSinceStart
  float mixw;       // f32(k/(k+1))
  float pad[2];
};

struct SailTraceArgs {
  const SailPrim* prims;
  const unsigned long long* typeMasks;  // per 64-row chunk: 16 words, bit j of word t = row 64*chunk+j has type t
  const float* texparams;   // tn x 16
  const float* lights;      // ln x 18
  const int32_t* lightObjRow;  // per light row: decoded object row of the area-light geometry
  const SailSample* samples;
  float4* accum;            // W x H, row 0 = bottom
  float4* aovN;             // optional
  float4* aovP;             // optional
  unsigned long long* segCounter;  // optional exact segment counter: SAIL_SEG_SLOTS partial sums
  float eye[3];
  int W, H;
  int n, tn, ln;
  uint32_t matMask, texMask, lightMask;
  int maxBounces;
  int spp;                  // samples in this launch
  int accumMode;            // 0 sum, 1 mix, 2 compat8
  int tilesX, tilesY;       // 64x64 partition tiles of the frame
  int world, rank;          // tile partition: global tile t belongs to rank t % world
  int ownedTiles;           // tiles of this rank
  int shadowAnyHit;         // 1 when no primitive can return d <= EPSILON (any-hit shadow rays are exact)
  int cullPrims;            // padded-box f32 pre-cull (SailPrim.a[18..23]) before each exact primitive test:
                            // 1 plain slab form, 2 fused form (host-checked scene extent, sail_capi.cpp cullFmaOk)
  int cullPrimary;          // 1: primary rays use the pre-cull too (the eye is near the scene: eyeNearScene)
  int kernelSet;            // SAIL_KSET_*: the precompiled plugin-set kernel to launch
  // sample groups: sampleGroups workgroups share each 16x16 block, group g renders samples [g*groupSpp,
  // (g+1)*groupSpp); group 0 adds its samples to the accumulator itself, the others stage theirs, and
  // sail_accum_kernel then adds the staged ones in sample order, so the sums are bit-identical to one workgroup
  // doing all samples
  int sampleGroups, groupSpp;
  int groupHome;            // 1: group 0 accumulated its samples itself (SAIL_GROUP_HOME_FOR), the stage starts at groupSpp
  float* stage;             // three f32 planes per sample: stage[(3k + c) * stageStride + slot]
  long long stageStride;    // slots per sample = ownedTiles * 4096
};

// Wavefront split of the pre-cull path (study switch SAIL_DEBUG_WAVEFRONT): the path state of one sample of every
// owned pixel in HBM, one float4 array per field, slot = owned tile * 4096 + local y * 64 + local x
struct SailWfState {
  float4* o;     // ray origin, w = 1 while the path is alive
  float4* d;     // ray direction
  float4* f;     // throughput
  float4* e;     // radiance
  float4* s;     // sweep result: t, winning row (int bits)
  float4* sp[6]; // a deferred shadow test: hit (w = 1 when pending), toLight, contribution, f, emission, throughput
};

// Precompiled plugin-set kernels (bit masks over the ids above). A scene whose plugin masks are subsets of a
// set's masks may use that set's kernel; everything else runs the generic one.
enum { SAIL_KSET_GENERIC = 0, SAIL_KSET_CORNELL = 1, SAIL_KSET_ROOM = 2 };
// Group home: with sample groups, the room kernel's first group adds its samples to the accumulator itself and the
// other groups stage theirs (C3 +1 %); in the other kernels the extra path costs more registers than the staged
// samples it saves (C2 -1.4 %, C4 -0.6 %), so every group stages. Shared by the kernel (traceTileCompact kHome) and the
// host (which tells sail_accum_kernel where the staged samples start).
#define SAIL_GROUP_HOME_FOR(kernelSet) ((kernelSet) == SAIL_KSET_ROOM)
// the exact segment counter is kept as this many partial sums (spread atomics), added on readback
#define SAIL_SEG_SLOTS 64
// the pre-cull kernels' per-workgroup LDS copies of the scene tables (rows of SailPrim, texParams rows of 16 floats)
#define SAIL_CULL_LDS_ROWS 72
#define SAIL_CULL_LDS_TP 136
#define SAIL_KSET_CORNELL_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_CORNELLBOX))
#define SAIL_KSET_CORNELL_MATS ((1u << SAIL_MATTE) | (1u << SAIL_MIRROR))
#define SAIL_KSET_CORNELL_TEX 0u
#define SAIL_KSET_CORNELL_LIGHTS 0u
// rooms of boxes, spheres and rectangle lights (C3 materials demo, the UI demo): no quadrics or disks
#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE) | (1u << SAIL_CORNELLBOX))
#define SAIL_KSET_ROOM_MATS 0xffffffffu
#define SAIL_KSET_ROOM_TEX 0xffffffffu
#define SAIL_KSET_ROOM_LIGHTS 0xffffffffu

struct SailFilterArgs {
  const float4* accum;
  const float4* aovN;       // normalMap (kinds 4-5)
  const float4* aovP;       // positionMap (kinds 4, 6)
  float4* out;
  uint8_t* out8;
  int W, H;
  int kind;                 // 0 color, 1 gamma, 2 tonemapping, 3 window, 4 wavelet, 5 normal, 6 position
  int accumMode;            // SUM: every texel is divided by its own count (.w)
  float weights[16];
  float rx, ry, gammaC;
  int halo;                 // window filters: LDS tile halo in pixels (0: taps read global memory)
};

// multi-device frame reduction on one GPU (sail_sum_kernel): dst = the sum of src[0..nsrc) in rank order
#define SAIL_SUM_MAX_SRC 64
struct SailSumArgs {
  const float4* src[SAIL_SUM_MAX_SRC];
  float4* dst;
  long long n;              // float4 elements
  int nsrc;
};
