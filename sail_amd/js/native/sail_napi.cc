// sail_napi.cc — Node-API binding of libsail_hip.so (include/sail_hip.h) for the JavaScript host.
// Built against the Node headers of this image (/usr/include/node, N-API 8); links libsail_hip.so with
// an $ORIGIN rpath. Every failing C call becomes a thrown JS Error carrying sail_last_error().
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../../include/sail_hip.h"

namespace {

struct Handle {
  sail_ctx* ctx;
  int W, H;
};

#define NAPI_OK(call)                                              \
  do {                                                             \
    if ((call) != napi_ok) {                                       \
      napi_throw_error(env, nullptr, "N-API call failed: " #call); \
      return nullptr;                                              \
    }                                                              \
  } while (0)

napi_value throwSail(napi_env env, const char* what, int rc, const sail_ctx* c) {
  std::string msg = std::string(what) + " failed (" + std::to_string(rc) + "): " + sail_last_error(c);
  napi_throw_error(env, nullptr, msg.c_str());
  return nullptr;
}

bool args(napi_env env, napi_callback_info info, size_t n, napi_value* out) {
  size_t argc = n;
  if (napi_get_cb_info(env, info, &argc, out, nullptr, nullptr) != napi_ok) return false;
  if (argc < n) {
    napi_throw_type_error(env, nullptr, "not enough arguments");
    return false;
  }
  return true;
}
bool getInt(napi_env env, napi_value v, int* out) {
  if (napi_get_value_int32(env, v, out) != napi_ok) { napi_throw_type_error(env, nullptr, "expected a number"); return false; }
  return true;
}
bool getDouble(napi_env env, napi_value v, double* out) {
  if (napi_get_value_double(env, v, out) != napi_ok) { napi_throw_type_error(env, nullptr, "expected a number"); return false; }
  return true;
}
// typed-array view (nullptr for null/undefined when allowed)
template <typename T>
bool getArray(napi_env env, napi_value v, napi_typedarray_type want, T** data, size_t* len, bool nullable = false) {
  napi_valuetype vt;
  napi_typeof(env, v, &vt);
  if (nullable && (vt == napi_null || vt == napi_undefined)) { *data = nullptr; *len = 0; return true; }
  bool is = false;
  napi_is_typedarray(env, v, &is);
  if (!is) { napi_throw_type_error(env, nullptr, "expected a typed array"); return false; }
  napi_typedarray_type t;
  void* p = nullptr;
  napi_value ab;
  size_t off = 0;
  napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off);
  if (t != want) { napi_throw_type_error(env, nullptr, "typed array has the wrong element type"); return false; }
  *data = static_cast<T*>(p);
  return true;
}
bool getHandle(napi_env env, napi_value v, Handle** h) {
  void* p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p || !static_cast<Handle*>(p)->ctx) {
    napi_throw_error(env, nullptr, "invalid or destroyed renderer context");
    return false;
  }
  *h = static_cast<Handle*>(p);
  return true;
}
napi_value makeF32(napi_env env, const float* src, size_t n) {
  void* data = nullptr;
  napi_value ab, arr;
  napi_create_arraybuffer(env, n * sizeof(float), &data, &ab);
  if (src) memcpy(data, src, n * sizeof(float));
  napi_create_typedarray(env, napi_float32_array, n, ab, 0, &arr);
  return arr;
}
napi_value makeTyped(napi_env env, napi_typedarray_type t, size_t n, size_t elem, void** data) {
  napi_value ab, arr;
  napi_create_arraybuffer(env, n * elem, data, &ab);
  napi_create_typedarray(env, t, n, ab, 0, &arr);
  return arr;
}
napi_value num(napi_env env, double v) { napi_value r; napi_create_double(env, v, &r); return r; }
napi_value undef(napi_env env) { napi_value r; napi_get_undefined(env, &r); return r; }

void finalizeHandle(napi_env, void* data, void*) {
  Handle* h = static_cast<Handle*>(data);
  if (h->ctx) sail_destroy(h->ctx);
  delete h;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
  int n = 0;
  sail_device_count(&n);
  return num(env, n);
}
napi_value AbiVersion(napi_env env, napi_callback_info) { return num(env, sail_abi_version()); }

napi_value Create(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!args(env, info, 4, a)) return nullptr;
  int w, h, dev, flags;
  if (!getInt(env, a[0], &w) || !getInt(env, a[1], &h) || !getInt(env, a[2], &dev) || !getInt(env, a[3], &flags)) return nullptr;
  sail_ctx* c = nullptr;
  const int rc = sail_create(&c, w, h, dev, (uint32_t)flags);
  if (rc) return throwSail(env, "sail_create", rc, nullptr);
  Handle* hd = new Handle{c, w, h};
  napi_value ext;
  NAPI_OK(napi_create_external(env, hd, finalizeHandle, nullptr, &ext));
  return ext;
}
// (W, H, Int32Array devices, flags): one context over several GPUs (sail_create_multi)
napi_value CreateMulti(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!args(env, info, 4, a)) return nullptr;
  int w, h, flags;
  int32_t* dev;
  size_t nd;
  if (!getInt(env, a[0], &w) || !getInt(env, a[1], &h) || !getArray(env, a[2], napi_int32_array, &dev, &nd) ||
      !getInt(env, a[3], &flags))
    return nullptr;
  sail_ctx* c = nullptr;
  const int rc = sail_create_multi(&c, w, h, dev, (int)nd, (uint32_t)flags);
  if (rc) return throwSail(env, "sail_create_multi", rc, nullptr);
  Handle* hd = new Handle{c, w, h};
  napi_value ext;
  NAPI_OK(napi_create_external(env, hd, finalizeHandle, nullptr, &ext));
  return ext;
}
napi_value Destroy(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  void* p = nullptr;
  if (napi_get_value_external(env, a[0], &p) == napi_ok && p) {
    Handle* h = static_cast<Handle*>(p);
    if (h->ctx) { sail_destroy(h->ctx); h->ctx = nullptr; }
  }
  return undef(env);
}
napi_value SetScene(napi_env env, napi_callback_info info) {
  napi_value a[8];
  if (!args(env, info, 8, a)) return nullptr;
  Handle* h;
  float *o, *t, *l;
  size_t no, nt, nl;
  int n, tn, ln;
  if (!getHandle(env, a[0], &h) || !getArray(env, a[1], napi_float32_array, &o, &no) || !getInt(env, a[2], &n) ||
      !getArray(env, a[3], napi_float32_array, &t, &nt) || !getInt(env, a[4], &tn) ||
      !getArray(env, a[5], napi_float32_array, &l, &nl) || !getInt(env, a[6], &ln))
    return nullptr;
  if (no < (size_t)n * 18 || nt < (size_t)tn * 16 || nl < (size_t)ln * 18) {
    napi_throw_range_error(env, nullptr, "scene rows shorter than n/tn/ln");
    return nullptr;
  }
  uint32_t m[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < 4; i++) {
    napi_value e;
    NAPI_OK(napi_get_element(env, a[7], i, &e));
    NAPI_OK(napi_get_value_uint32(env, e, &m[i]));
  }
  sail_plugins pl{m[0], m[1], m[2], m[3]};
  const int rc = sail_set_scene(h->ctx, o, n, t, tn, l, ln, &pl);
  if (rc) return throwSail(env, "sail_set_scene", rc, h->ctx);
  return undef(env);
}
napi_value UpdateObjects(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!args(env, info, 3, a)) return nullptr;
  Handle* h;
  float* o;
  size_t no;
  int n;
  if (!getHandle(env, a[0], &h) || !getArray(env, a[1], napi_float32_array, &o, &no) || !getInt(env, a[2], &n)) return nullptr;
  if (no < (size_t)n * 18) { napi_throw_range_error(env, nullptr, "object rows shorter than n"); return nullptr; }
  const int rc = sail_update_objects(h->ctx, o, n);
  if (rc) return throwSail(env, "sail_update_objects", rc, h->ctx);
  return undef(env);
}
napi_value IntSetter(napi_env env, napi_callback_info info, int nargs, const char* name,
                     int (*fn3)(sail_ctx*, int, int, int), int (*fn1)(sail_ctx*, int)) {
  napi_value a[4];
  if (!args(env, info, nargs + 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  int v[3] = {0, 0, 0};
  for (int i = 0; i < nargs; i++) if (!getInt(env, a[1 + i], &v[i])) return nullptr;
  const int rc = fn3 ? fn3(h->ctx, v[0], v[1], v[2]) : fn1(h->ctx, v[0]);
  if (rc) return throwSail(env, name, rc, h->ctx);
  return undef(env);
}
napi_value SetAccumMode(napi_env env, napi_callback_info info) { return IntSetter(env, info, 1, "sail_set_accum_mode", nullptr, sail_set_accum_mode); }
napi_value SetLaunchSamples(napi_env env, napi_callback_info info) { return IntSetter(env, info, 1, "sail_set_launch_samples", nullptr, sail_set_launch_samples); }
napi_value SetPartition(napi_env env, napi_callback_info info) { return IntSetter(env, info, 3, "sail_set_partition", sail_set_partition, nullptr); }
int setDebug3(sail_ctx* c, int opt, int val, int) { return sail_set_debug(c, opt, val); }
napi_value SetDebug(napi_env env, napi_callback_info info) { return IntSetter(env, info, 2, "sail_set_debug", setDebug3, nullptr); }
int reduce3(sail_ctx* c, int root, int, int) { return sail_reduce(c, root); }
napi_value Reduce(napi_env env, napi_callback_info info) { return IntSetter(env, info, 1, "sail_reduce", reduce3, nullptr); }

napi_value Render(napi_env env, napi_callback_info info) {
  napi_value a[5];
  if (!args(env, info, 5, a)) return nullptr;
  Handle* h;
  float *inv, *eye;
  size_t ni, ne;
  double seed;
  int b;
  if (!getHandle(env, a[0], &h) || !getArray(env, a[1], napi_float32_array, &inv, &ni) ||
      !getArray(env, a[2], napi_float32_array, &eye, &ne) || !getDouble(env, a[3], &seed) || !getInt(env, a[4], &b))
    return nullptr;
  if (ni < 16 || ne < 3) { napi_throw_range_error(env, nullptr, "inv_mvp needs 16 and eye 3 floats"); return nullptr; }
  const int rc = sail_render(h->ctx, inv, eye, (float)seed, b);
  if (rc) return throwSail(env, "sail_render", rc, h->ctx);
  return undef(env);
}
napi_value RenderSchedule(napi_env env, napi_callback_info info) {
  napi_value a[5];
  if (!args(env, info, 5, a)) return nullptr;
  Handle* h;
  float *inv, *seeds, *eye;
  size_t ni, ns, ne;
  int b;
  if (!getHandle(env, a[0], &h) || !getArray(env, a[1], napi_float32_array, &inv, &ni) ||
      !getArray(env, a[2], napi_float32_array, &seeds, &ns) || !getArray(env, a[3], napi_float32_array, &eye, &ne) ||
      !getInt(env, a[4], &b))
    return nullptr;
  if (ni < ns * 16 || ne < 3) { napi_throw_range_error(env, nullptr, "schedule arrays too short"); return nullptr; }
  const int rc = sail_render_schedule(h->ctx, inv, seeds, eye, (int)ns, b);
  if (rc) return throwSail(env, "sail_render_schedule", rc, h->ctx);
  return undef(env);
}
napi_value Simple(napi_env env, napi_callback_info info, int (*fn)(sail_ctx*), const char* name) {
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  const int rc = fn(h->ctx);
  if (rc) return throwSail(env, name, rc, h->ctx);
  return undef(env);
}
napi_value Reset(napi_env env, napi_callback_info info) { return Simple(env, info, sail_reset, "sail_reset"); }
napi_value Sync(napi_env env, napi_callback_info info) { return Simple(env, info, sail_sync, "sail_sync"); }

napi_value Readback(napi_env env, napi_callback_info info) {  // (ctx, wantAov) -> {rgba, normal?, position?}
  napi_value a[2];
  if (!args(env, info, 2, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  bool aov = false;
  napi_get_value_bool(env, a[1], &aov);
  const size_t np = (size_t)h->W * h->H * 4;
  void *pr = nullptr, *pn = nullptr, *pp = nullptr;
  napi_value rgba = makeTyped(env, napi_float32_array, np, 4, &pr);
  napi_value out;
  NAPI_OK(napi_create_object(env, &out));
  NAPI_OK(napi_set_named_property(env, out, "rgba", rgba));
  if (aov) {
    napi_value nn = makeTyped(env, napi_float32_array, np, 4, &pn), ppv = makeTyped(env, napi_float32_array, np, 4, &pp);
    NAPI_OK(napi_set_named_property(env, out, "normal", nn));
    NAPI_OK(napi_set_named_property(env, out, "position", ppv));
  }
  const int rc = sail_readback(h->ctx, (float*)pr, (float*)pn, (float*)pp);
  if (rc) return throwSail(env, "sail_readback", rc, h->ctx);
  return out;
}
napi_value ReadAccum(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  void* p = nullptr;
  napi_value arr = makeTyped(env, napi_float32_array, (size_t)h->W * h->H * 4, 4, &p);
  const int rc = sail_read_accum(h->ctx, (float*)p);
  if (rc) return throwSail(env, "sail_read_accum", rc, h->ctx);
  return arr;
}
// checkpoint / resume (sail_accum_parts, sail_save_accum, sail_load_accum)
napi_value SaveAccum(napi_env env, napi_callback_info info) {  // (ctx) -> {k, parts: [Float32Array]}
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  int parts = 0;
  int rc = sail_accum_parts(h->ctx, &parts);
  if (rc) return throwSail(env, "sail_accum_parts", rc, h->ctx);
  napi_value list, out;
  NAPI_OK(napi_create_array_with_length(env, (size_t)parts, &list));
  uint64_t k = 0;
  for (int i = 0; i < parts; i++) {
    void* p = nullptr;
    napi_value arr = makeTyped(env, napi_float32_array, (size_t)h->W * h->H * 4, 4, &p);
    rc = sail_save_accum(h->ctx, i, (float*)p, &k);
    if (rc) return throwSail(env, "sail_save_accum", rc, h->ctx);
    napi_set_element(env, list, (uint32_t)i, arr);
  }
  NAPI_OK(napi_create_object(env, &out));
  napi_set_named_property(env, out, "k", num(env, (double)k));
  napi_set_named_property(env, out, "parts", list);
  return out;
}
napi_value LoadAccum(napi_env env, napi_callback_info info) {  // (ctx, part, Float32Array sums, k)
  napi_value a[4];
  if (!args(env, info, 4, a)) return nullptr;
  Handle* h;
  int part;
  float* sums;
  size_t n;
  double k;
  if (!getHandle(env, a[0], &h) || !getInt(env, a[1], &part) || !getArray(env, a[2], napi_float32_array, &sums, &n) ||
      !getDouble(env, a[3], &k))
    return nullptr;
  if (n != (size_t)h->W * h->H * 4) { napi_throw_range_error(env, nullptr, "accumulator has the wrong size"); return nullptr; }
  if (!(k >= 0.0 && k <= 9007199254740992.0) || k != (double)(uint64_t)k) {
    napi_throw_range_error(env, nullptr, "sample index must be a non-negative integer");
    return nullptr;
  }
  const int rc = sail_load_accum(h->ctx, part, sums, (uint64_t)k);
  if (rc) return throwSail(env, "sail_load_accum", rc, h->ctx);
  return undef(env);
}
napi_value Filter(napi_env env, napi_callback_info info) {  // (ctx, kind, weights|null, rx, ry, gamma) -> {rgba, rgba8}
  napi_value a[6];
  if (!args(env, info, 6, a)) return nullptr;
  Handle* h;
  int kind;
  float* w;
  size_t nw;
  double rx, ry, g;
  if (!getHandle(env, a[0], &h) || !getInt(env, a[1], &kind) || !getArray(env, a[2], napi_float32_array, &w, &nw, true) ||
      !getDouble(env, a[3], &rx) || !getDouble(env, a[4], &ry) || !getDouble(env, a[5], &g))
    return nullptr;
  if (w && nw < 16) { napi_throw_range_error(env, nullptr, "window weights need 16 floats"); return nullptr; }
  const size_t np = (size_t)h->W * h->H * 4;
  void *pf = nullptr, *p8 = nullptr;
  napi_value f = makeTyped(env, napi_float32_array, np, 4, &pf), u8 = makeTyped(env, napi_uint8_array, np, 1, &p8);
  const int rc = sail_filter(h->ctx, kind, w, (float)rx, (float)ry, (float)g, (float*)pf, (uint8_t*)p8);
  if (rc) return throwSail(env, "sail_filter", rc, h->ctx);
  napi_value out;
  NAPI_OK(napi_create_object(env, &out));
  NAPI_OK(napi_set_named_property(env, out, "rgba", f));
  NAPI_OK(napi_set_named_property(env, out, "rgba8", u8));
  return out;
}
napi_value Pick(napi_env env, napi_callback_info info) {  // (ctx, Float32Array rays[6*count]) -> {index, t}
  napi_value a[2];
  if (!args(env, info, 2, a)) return nullptr;
  Handle* h;
  float* rays;
  size_t nr;
  if (!getHandle(env, a[0], &h) || !getArray(env, a[1], napi_float32_array, &rays, &nr)) return nullptr;
  if (nr % 6) { napi_throw_range_error(env, nullptr, "rays need 6 floats each"); return nullptr; }
  const size_t count = nr / 6;
  void *pi = nullptr, *pt = nullptr;
  napi_value idx = makeTyped(env, napi_int32_array, count, 4, &pi), t = makeTyped(env, napi_float32_array, count, 4, &pt);
  const int rc = sail_pick(h->ctx, rays, (int)count, (int32_t*)pi, (float*)pt);
  if (rc) return throwSail(env, "sail_pick", rc, h->ctx);
  napi_value out;
  NAPI_OK(napi_create_object(env, &out));
  NAPI_OK(napi_set_named_property(env, out, "index", idx));
  NAPI_OK(napi_set_named_property(env, out, "t", t));
  return out;
}
napi_value Stats(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  sail_stats s;
  const int rc = sail_get_stats(h->ctx, &s);
  if (rc) return throwSail(env, "sail_get_stats", rc, h->ctx);
  napi_value out;
  NAPI_OK(napi_create_object(env, &out));
  napi_set_named_property(env, out, "samples", num(env, (double)s.samples));
  napi_set_named_property(env, out, "segments", num(env, (double)s.segments));
  napi_set_named_property(env, out, "nominalSegments", num(env, (double)s.nominal_segments));
  napi_set_named_property(env, out, "kernelMs", num(env, s.kernel_ms));
  napi_set_named_property(env, out, "lastLaunchMs", num(env, s.last_launch_ms));
  napi_set_named_property(env, out, "launches", num(env, s.launches));
  return out;
}
// (ctx, timeoutMs) -> whether the scene's run-time kernel is loaded (sail_kernel_ready; -1 waits for its build)
napi_value KernelReady(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!args(env, info, 2, a)) return nullptr;
  Handle* h;
  int ms = 0;
  if (!getHandle(env, a[0], &h) || !getInt(env, a[1], &ms)) return nullptr;
  int ready = 0;
  const int rc = sail_kernel_ready(h->ctx, ms, &ready);
  if (rc) return throwSail(env, "sail_kernel_ready", rc, h->ctx);
  napi_value out;
  NAPI_OK(napi_get_boolean(env, ready != 0, &out));
  return out;
}
// (ctx) -> {name, buildId, jitState, jitFromCache, jitCompileMs, jitError} (sail_get_kernel_info)
napi_value KernelInfo(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!args(env, info, 1, a)) return nullptr;
  Handle* h;
  if (!getHandle(env, a[0], &h)) return nullptr;
  sail_kernel_info k;
  const int rc = sail_get_kernel_info(h->ctx, &k);
  if (rc) return throwSail(env, "sail_get_kernel_info", rc, h->ctx);
  char id[17];
  snprintf(id, sizeof id, "%016llx", (unsigned long long)k.build_id);
  napi_value out, v;
  NAPI_OK(napi_create_object(env, &out));
  NAPI_OK(napi_create_string_utf8(env, k.name, NAPI_AUTO_LENGTH, &v));
  napi_set_named_property(env, out, "name", v);
  NAPI_OK(napi_create_string_utf8(env, id, NAPI_AUTO_LENGTH, &v));
  napi_set_named_property(env, out, "buildId", v);
  static const char* const states[] = {"none", "pending", "ready", "failed"};
  NAPI_OK(napi_create_string_utf8(env, states[k.jit_state & 3], NAPI_AUTO_LENGTH, &v));
  napi_set_named_property(env, out, "jitState", v);
  napi_set_named_property(env, out, "jitFromCache", num(env, k.jit_from_cache));
  napi_set_named_property(env, out, "jitCompileMs", num(env, k.jit_compile_ms));
  NAPI_OK(napi_create_string_utf8(env, k.jit_error, NAPI_AUTO_LENGTH, &v));
  napi_set_named_property(env, out, "jitError", v);
  return out;
}
bool getVec(napi_env env, napi_value v, double* out, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    if (napi_get_element(env, v, i, &e) != napi_ok || napi_get_value_double(env, e, &out[i]) != napi_ok) {
      napi_throw_type_error(env, nullptr, "expected an array of numbers");
      return false;
    }
  }
  return true;
}
napi_value Camera(napi_env env, napi_callback_info info) {  // (eye, center, up, fovy, aspect, near, far) -> Float64Array(16)
  napi_value a[7];
  if (!args(env, info, 7, a)) return nullptr;
  double e[3], c[3], u[3], fovy, asp, zn, zf;
  if (!getVec(env, a[0], e, 3) || !getVec(env, a[1], c, 3) || !getVec(env, a[2], u, 3) || !getDouble(env, a[3], &fovy) ||
      !getDouble(env, a[4], &asp) || !getDouble(env, a[5], &zn) || !getDouble(env, a[6], &zf))
    return nullptr;
  void* p = nullptr;
  napi_value arr = makeTyped(env, napi_float64_array, 16, 8, &p);
  const int rc = sail_camera(e, c, u, fovy, asp, zn, zf, (double*)p);
  if (rc) return throwSail(env, "sail_camera", rc, nullptr);
  return arr;
}
napi_value JitterInverse(napi_env env, napi_callback_info info) {  // (mvp f64[16] row-major, jx, jy, W, H)
  napi_value a[5];
  if (!args(env, info, 5, a)) return nullptr;
  double* m;
  size_t nm;
  double jx, jy;
  int w, hh;
  if (!getArray(env, a[0], napi_float64_array, &m, &nm) || !getDouble(env, a[1], &jx) || !getDouble(env, a[2], &jy) ||
      !getInt(env, a[3], &w) || !getInt(env, a[4], &hh))
    return nullptr;
  if (nm < 16) { napi_throw_range_error(env, nullptr, "mvp needs 16 doubles"); return nullptr; }
  void* p = nullptr;
  napi_value arr = makeTyped(env, napi_float32_array, 16, 4, &p);
  const int rc = sail_jitter_inverse(m, jx, jy, w, hh, (float*)p);
  if (rc) return throwSail(env, "sail_jitter_inverse", rc, nullptr);
  return arr;
}
napi_value Schedule(napi_env env, napi_callback_info info) {  // (mvp, W, H, k0, spp) -> {inv, seeds}
  napi_value a[5];
  if (!args(env, info, 5, a)) return nullptr;
  double* m;
  size_t nm;
  int w, hh, k0, spp;
  if (!getArray(env, a[0], napi_float64_array, &m, &nm) || !getInt(env, a[1], &w) || !getInt(env, a[2], &hh) ||
      !getInt(env, a[3], &k0) || !getInt(env, a[4], &spp))
    return nullptr;
  if (nm < 16 || spp < 0) { napi_throw_range_error(env, nullptr, "bad schedule arguments"); return nullptr; }
  void *pi = nullptr, *ps = nullptr;
  napi_value inv = makeTyped(env, napi_float32_array, (size_t)spp * 16, 4, &pi);
  napi_value seeds = makeTyped(env, napi_float32_array, (size_t)spp, 4, &ps);
  const int rc = sail_schedule(m, w, hh, k0, spp, (float*)pi, (float*)ps);
  if (rc) return throwSail(env, "sail_schedule", rc, nullptr);
  napi_value out;
  NAPI_OK(napi_create_object(env, &out));
  NAPI_OK(napi_set_named_property(env, out, "inv", inv));
  NAPI_OK(napi_set_named_property(env, out, "seeds", seeds));
  return out;
}
napi_value PartitionTiles(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!args(env, info, 4, a)) return nullptr;
  int w, hh, r, wo;
  if (!getInt(env, a[0], &w) || !getInt(env, a[1], &hh) || !getInt(env, a[2], &r) || !getInt(env, a[3], &wo)) return nullptr;
  const int n = sail_partition_tiles(w, hh, r, wo, nullptr, 0);
  if (n < 0) return throwSail(env, "sail_partition_tiles", n, nullptr);
  void* p = nullptr;
  napi_value arr = makeTyped(env, napi_int32_array, (size_t)n * 4, 4, &p);
  sail_partition_tiles(w, hh, r, wo, (int*)p, n);
  return arr;
}
napi_value MathProbe(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!args(env, info, 3, a)) return nullptr;
  int fn;
  float *x, *y;
  size_t nx, ny;
  if (!getInt(env, a[0], &fn) || !getArray(env, a[1], napi_float32_array, &x, &nx) ||
      !getArray(env, a[2], napi_float32_array, &y, &ny))
    return nullptr;
  if (ny < nx) { napi_throw_range_error(env, nullptr, "y shorter than x"); return nullptr; }
  void* p = nullptr;
  napi_value arr = makeTyped(env, napi_float32_array, nx, 4, &p);
  const int rc = sail_math_probe(fn, x, y, (float*)p, (int)nx);
  if (rc) return throwSail(env, "sail_math_probe", rc, nullptr);
  return arr;
}

napi_value Init(napi_env env, napi_value exports) {
  const napi_property_descriptor props[] = {
      {"deviceCount", 0, DeviceCount, 0, 0, 0, napi_enumerable, 0},
      {"abiVersion", 0, AbiVersion, 0, 0, 0, napi_enumerable, 0},
      {"create", 0, Create, 0, 0, 0, napi_enumerable, 0},
      {"createMulti", 0, CreateMulti, 0, 0, 0, napi_enumerable, 0},
      {"setDebug", 0, SetDebug, 0, 0, 0, napi_enumerable, 0},
      {"reduce", 0, Reduce, 0, 0, 0, napi_enumerable, 0},
      {"destroy", 0, Destroy, 0, 0, 0, napi_enumerable, 0},
      {"setScene", 0, SetScene, 0, 0, 0, napi_enumerable, 0},
      {"updateObjects", 0, UpdateObjects, 0, 0, 0, napi_enumerable, 0},
      {"setAccumMode", 0, SetAccumMode, 0, 0, 0, napi_enumerable, 0},
      {"setPartition", 0, SetPartition, 0, 0, 0, napi_enumerable, 0},
      {"setLaunchSamples", 0, SetLaunchSamples, 0, 0, 0, napi_enumerable, 0},
      {"render", 0, Render, 0, 0, 0, napi_enumerable, 0},
      {"renderSchedule", 0, RenderSchedule, 0, 0, 0, napi_enumerable, 0},
      {"reset", 0, Reset, 0, 0, 0, napi_enumerable, 0},
      {"sync", 0, Sync, 0, 0, 0, napi_enumerable, 0},
      {"readback", 0, Readback, 0, 0, 0, napi_enumerable, 0},
      {"readAccum", 0, ReadAccum, 0, 0, 0, napi_enumerable, 0},
      {"saveAccum", 0, SaveAccum, 0, 0, 0, napi_enumerable, 0},
      {"loadAccum", 0, LoadAccum, 0, 0, 0, napi_enumerable, 0},
      {"filter", 0, Filter, 0, 0, 0, napi_enumerable, 0},
      {"stats", 0, Stats, 0, 0, 0, napi_enumerable, 0},
      {"kernelReady", 0, KernelReady, 0, 0, 0, napi_enumerable, 0},
      {"kernelInfo", 0, KernelInfo, 0, 0, 0, napi_enumerable, 0},
      {"pick", 0, Pick, 0, 0, 0, napi_enumerable, 0},
      {"camera", 0, Camera, 0, 0, 0, napi_enumerable, 0},
      {"jitterInverse", 0, JitterInverse, 0, 0, 0, napi_enumerable, 0},
      {"schedule", 0, Schedule, 0, 0, 0, napi_enumerable, 0},
      {"partitionTiles", 0, PartitionTiles, 0, 0, 0, napi_enumerable, 0},
      {"mathProbe", 0, MathProbe, 0, 0, 0, napi_enumerable, 0},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
