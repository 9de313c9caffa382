// rt0_node.cc -- N-API binding of include/rt0.h for the reference's JS host.
//
// The reference's GlslViewport (index.js) talks to WebGL2; js/glsl_viewport.js
// keeps that class surface and calls these functions instead.  Every rt0 error
// code becomes a thrown JS Error carrying rt0_last_error(), mirroring how the
// reference throws shader compile/link errors as strings (index.js:606, 622).
// Built with: g++ -shared -fPIC -I/usr/include/node rt0_node.cc -lrt0 (Makefile).
#include <node_api.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt0.h"

#define NAPI_OK(env, call)                                   \
  do {                                                       \
    if ((call) != napi_ok) {                                 \
      napi_throw_error((env), nullptr, "N-API call failed"); \
      return nullptr;                                        \
    }                                                        \
  } while (0)

static napi_value throw_rt0(napi_env env, int rc, const char *msg) {
  std::string m = std::string("rt0 error ") + std::to_string(rc) + ": " + (msg ? msg : "");
  napi_throw_error(env, nullptr, m.c_str());
  return nullptr;
}

static bool get_args(napi_env env, napi_callback_info info, size_t n, napi_value *argv) {
  size_t argc = n;
  if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
  for (size_t i = argc; i < n; i++) napi_get_undefined(env, &argv[i]);
  return true;
}

static std::string get_string(napi_env env, napi_value v) {
  size_t len = 0;
  if (napi_get_value_string_utf8(env, v, nullptr, 0, &len) != napi_ok) return std::string();
  std::string s(len, '\0');
  napi_get_value_string_utf8(env, v, &s[0], len + 1, &len);
  return s;
}

static std::vector<std::string> get_string_array(napi_env env, napi_value v) {
  std::vector<std::string> out;
  bool is_arr = false;
  napi_is_array(env, v, &is_arr);
  if (!is_arr) return out;
  uint32_t n = 0;
  napi_get_array_length(env, v, &n);
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    napi_get_element(env, v, i, &e);
    out.push_back(get_string(env, e));
  }
  return out;
}

static std::vector<const char *> c_strs(const std::vector<std::string> &v) {
  std::vector<const char *> p;
  for (auto &s : v) p.push_back(s.c_str());
  return p;
}

static bool get_floats(napi_env env, napi_value v, float *out, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    double d;
    if (napi_get_element(env, v, i, &e) != napi_ok || napi_get_value_double(env, e, &d) != napi_ok) return false;
    out[i] = (float)d;
  }
  return true;
}

static rt0_ctx *get_ctx(napi_env env, napi_value v) {
  void *p = nullptr;
  if (napi_get_value_external(env, v, &p) != napi_ok) return nullptr;
  return (rt0_ctx *)p;
}

static void finalize_ctx(napi_env, void *data, void *) { rt0_destroy((rt0_ctx *)data); }

static napi_value num(napi_env env, double d) {
  napi_value v;
  napi_create_double(env, d, &v);
  return v;
}

static void set(napi_env env, napi_value obj, const char *k, napi_value v) { napi_set_named_property(env, obj, k, v); }

static napi_value config_object(napi_env env, const rt0_config &c) {
  napi_value o;
  napi_create_object(env, &o);
  set(env, o, "defines", num(env, c.defines));
  set(env, o, "MAX_BOUNCES", num(env, c.max_bounces));
  set(env, o, "MAX_DIFF_BOUNCES", num(env, c.max_diff_bounces));
  set(env, o, "MAX_SPEC_BOUNCES", num(env, c.max_spec_bounces));
  set(env, o, "MAX_TRANS_BOUNCES", num(env, c.max_trans_bounces));
  set(env, o, "MAX_SCATTERING_EVENTS", num(env, c.max_scattering_events));
  set(env, o, "MARCHING_STEPS", num(env, c.marching_steps));
  set(env, o, "FUDGE_FACTOR", num(env, c.fudge_factor));
  set(env, o, "sample_lights", num(env, c.sample_lights));
  set(env, o, "use_mis", num(env, c.use_mis));
  set(env, o, "use_restir", num(env, c.use_restir));
  set(env, o, "LIGHT_PATH_LENGTH", num(env, c.light_path_length));
  set(env, o, "RESTIR_SAMPLES", num(env, c.restir_samples));
  set(env, o, "RENDER_MODE", num(env, c.render_mode));
  return o;
}

// parseConfig(defines: string[], constants: string[]) -> object
static napi_value ParseConfig(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  auto d = get_string_array(env, argv[0]), k = get_string_array(env, argv[1]);
  auto dp = c_strs(d), kp = c_strs(k);
  rt0_config c;
  int rc = rt0_parse_config(dp.data(), (int)dp.size(), kp.data(), (int)kp.size(), &c);
  if (rc != RT0_OK) return throw_rt0(env, rc, "cannot parse defines/constants");
  return config_object(env, c);
}

// parseScene(scene: string, sdf_meshes: string[]) -> {meshes, nMeshes, nSdfs, lightIndex}
static napi_value ParseScene(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  std::string scene = get_string(env, argv[0]);
  auto s = get_string_array(env, argv[1]);
  auto sp = c_strs(s);
  std::vector<rt0_mesh> m(256);
  std::vector<int32_t> l(256);
  int ne = 0, ns = 0, nm = 0, nl = 0;
  int rc = rt0_parse_scene_glsl(scene.c_str(), sp.data(), (int)sp.size(), m.data(), 256, &ne, &ns, &nm, l.data(), 256,
                                &nl);
  if (rc != RT0_OK) return throw_rt0(env, rc, "cannot parse scene");
  napi_value o, arr, li;
  napi_create_object(env, &o);
  napi_create_array_with_length(env, ne + ns + nm, &arr);
  for (int i = 0; i < ne + ns + nm; i++) {
    napi_value e;
    napi_create_object(env, &e);
    set(env, e, "type", num(env, m[i].type));
    set(env, e, "matType", num(env, m[i].mat_type));
    set(env, e, "sdfKind", num(env, m[i].sdf_kind));
    napi_value pos, jk;
    napi_create_array_with_length(env, 3, &pos);
    napi_create_array_with_length(env, 4, &jk);
    for (int j = 0; j < 3; j++) napi_set_element(env, pos, j, num(env, m[i].pos[j]));
    for (int j = 0; j < 4; j++) napi_set_element(env, jk, j, num(env, m[i].joker[j]));
    set(env, e, "pos", pos);
    set(env, e, "joker", jk);
    napi_set_element(env, arr, i, e);
  }
  napi_create_array_with_length(env, nl, &li);
  for (int i = 0; i < nl; i++) napi_set_element(env, li, i, num(env, l[i]));
  set(env, o, "meshes", arr);
  set(env, o, "nMeshes", num(env, ne));
  set(env, o, "nSdfs", num(env, ns));
  set(env, o, "nModels", num(env, nm));
  set(env, o, "lightIndex", li);
  return o;
}

// create(width, height, device) -> handle
static napi_value Create(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return nullptr;
  int32_t w = 0, h = 0, dev = 0;
  napi_get_value_int32(env, argv[0], &w);
  napi_get_value_int32(env, argv[1], &h);
  napi_get_value_int32(env, argv[2], &dev);
  rt0_ctx *c = nullptr;
  int rc = rt0_create(w, h, dev, &c);
  if (rc != RT0_OK) return throw_rt0(env, rc, "rt0_create failed (no HIP device?)");
  napi_value ext;
  NAPI_OK(env, napi_create_external(env, c, finalize_ctx, nullptr, &ext));
  return ext;
}

#define CTX_OR_THROW(v)                                      \
  rt0_ctx *c = get_ctx(env, (v));                            \
  if (!c) {                                                  \
    napi_throw_type_error(env, nullptr, "bad rt0 handle");   \
    return nullptr;                                          \
  }
#define RC_OR_THROW(expr)                                    \
  do {                                                       \
    int rc_ = (expr);                                        \
    if (rc_ != RT0_OK) return throw_rt0(env, rc_, rt0_last_error(c)); \
  } while (0)

static napi_value SetConfig(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  auto d = get_string_array(env, argv[1]), k = get_string_array(env, argv[2]);
  auto dp = c_strs(d), kp = c_strs(k);
  rt0_config cfg;
  int rc = rt0_parse_config(dp.data(), (int)dp.size(), kp.data(), (int)kp.size(), &cfg);
  if (rc != RT0_OK) return throw_rt0(env, rc, "cannot parse defines/constants");
  RC_OR_THROW(rt0_set_config(c, &cfg));
  return nullptr;
}

static napi_value SetScene(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  std::string scene = get_string(env, argv[1]);
  auto s = get_string_array(env, argv[2]);
  auto sp = c_strs(s);
  RC_OR_THROW(rt0_set_scene_glsl(c, scene.c_str(), sp.data(), (int)sp.size()));
  return nullptr;
}

static napi_value SetCamera(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  float p[3], l[3], q[3];
  if (!get_floats(env, argv[1], p, 3) || !get_floats(env, argv[2], l, 3) || !get_floats(env, argv[3], q, 3)) {
    napi_throw_type_error(env, nullptr, "camera vectors must be arrays of 3 numbers");
    return nullptr;
  }
  RC_OR_THROW(rt0_set_camera(c, p, l, q));
  return nullptr;
}

static napi_value Render(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  uint32_t first = 1;
  int32_t n = 1;
  double t = 0;
  napi_get_value_uint32(env, argv[1], &first);
  napi_get_value_int32(env, argv[2], &n);
  napi_get_value_double(env, argv[3], &t);
  RC_OR_THROW(rt0_render(c, first, n, (float)t));
  return nullptr;
}

static napi_value SetViewport(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t v[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) napi_get_value_int32(env, argv[1 + i], &v[i]);
  RC_OR_THROW(rt0_set_viewport(c, v[0], v[1], v[2], v[3]));
  return nullptr;
}

static napi_value SetTemporalFrames(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t n = 5;
  napi_get_value_int32(env, argv[1], &n);
  RC_OR_THROW(rt0_set_temporal_frames(c, n));
  return nullptr;
}

static napi_value SetExecutorCompat(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  bool on = false;
  napi_get_value_bool(env, argv[1], &on);
  RC_OR_THROW(rt0_set_executor_compat(c, on ? 1 : 0));
  return nullptr;
}

static napi_value SetTextureFilter(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t mode = 1;
  napi_get_value_int32(env, argv[1], &mode);
  RC_OR_THROW(rt0_set_texture_filter(c, mode));
  return nullptr;
}

static napi_value ReadAccum(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int w = 0, h = 0;
  rt0_get_size(c, &w, &h);
  size_t bytes = (size_t)w * h * 4 * sizeof(float);
  void *data = nullptr;
  napi_value ab, ta;
  NAPI_OK(env, napi_create_arraybuffer(env, bytes, &data, &ab));
  RC_OR_THROW(rt0_read_accum(c, (float *)data));
  NAPI_OK(env, napi_create_typedarray(env, napi_float32_array, (size_t)w * h * 4, ab, 0, &ta));
  return ta;
}

static napi_value Tonemap(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  double cont = 1.0;
  napi_get_value_double(env, argv[1], &cont);
  int w = 0, h = 0;
  rt0_get_size(c, &w, &h);
  void *data = nullptr;
  napi_value ab, ta;
  NAPI_OK(env, napi_create_arraybuffer(env, (size_t)w * h * 4, &data, &ab));
  RC_OR_THROW(rt0_tonemap(c, (float)cont, (uint8_t *)data));
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, (size_t)w * h * 4, ab, 0, &ta));
  return ta;
}

static napi_value Clear(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  RC_OR_THROW(rt0_clear(c));
  return nullptr;
}

static napi_value Resize(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t w = 0, h = 0;
  napi_get_value_int32(env, argv[1], &w);
  napi_get_value_int32(env, argv[2], &h);
  RC_OR_THROW(rt0_resize(c, w, h));
  return nullptr;
}

// setTexture(h, unit, width, height, rgba8: Uint8Array | null) -- loadTexture
// (index.js:699-728) for u_tex0..3 (unit 0..3) and u_rnd_tex (unit 4)
static napi_value SetTexture(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t unit = 0, w = 0, h = 0;
  napi_get_value_int32(env, argv[1], &unit);
  napi_get_value_int32(env, argv[2], &w);
  napi_get_value_int32(env, argv[3], &h);
  const uint8_t *px = nullptr;
  bool is_ta = false;
  napi_is_typedarray(env, argv[4], &is_ta);
  if (is_ta) {
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void *data = nullptr;
    napi_value ab;
    NAPI_OK(env, napi_get_typedarray_info(env, argv[4], &tt, &len, &data, &ab, &off));
    if (tt != napi_uint8_array && tt != napi_uint8_clamped_array) return throw_rt0(env, RT0_E_ARG, "texture must be a Uint8Array");
    if (len != (size_t)w * h * 4) return throw_rt0(env, RT0_E_ARG, "texture length != width*height*4");
    px = (const uint8_t *)data;
  }
  RC_OR_THROW(rt0_set_texture(c, unit, w, h, px));
  return nullptr;
}

// setCubemap(h, size, faces: Uint8Array[6] (RGB8, reference order -X -Y -Z
// +X +Y +Z) | null) -- load_cubemap, index.js:298-331
static napi_value SetCubemap(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t size = 0;
  napi_get_value_int32(env, argv[1], &size);
  bool is_arr = false;
  napi_is_array(env, argv[2], &is_arr);
  if (!is_arr) {
    RC_OR_THROW(rt0_set_cubemap(c, 0, nullptr));
    return nullptr;
  }
  const uint8_t *faces[6];
  for (uint32_t i = 0; i < 6; i++) {
    napi_value e;
    bool is_ta = false;
    if (napi_get_element(env, argv[2], i, &e) != napi_ok) return throw_rt0(env, RT0_E_ARG, "six faces expected");
    napi_is_typedarray(env, e, &is_ta);
    if (!is_ta) return throw_rt0(env, RT0_E_ARG, "cubemap face must be a Uint8Array");
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void *data = nullptr;
    napi_value ab;
    NAPI_OK(env, napi_get_typedarray_info(env, e, &tt, &len, &data, &ab, &off));
    if (len != (size_t)size * size * 3) return throw_rt0(env, RT0_E_ARG, "cubemap face length != size*size*3");
    faces[i] = (const uint8_t *)data;
  }
  RC_OR_THROW(rt0_set_cubemap(c, size, faces));
  return nullptr;
}

// setModel(h, k, positions: Float32Array (3/vertex), indices: Int32Array (3/triangle))
static napi_value SetModel(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t k = 0;
  napi_get_value_int32(env, argv[1], &k);
  void *pd = nullptr, *id = nullptr;
  size_t pl = 0, il = 0, off = 0;
  napi_typedarray_type pt, it;
  napi_value ab;
  bool ta = false;
  napi_is_typedarray(env, argv[2], &ta);
  if (!ta) return throw_rt0(env, RT0_E_ARG, "positions must be a Float32Array");
  NAPI_OK(env, napi_get_typedarray_info(env, argv[2], &pt, &pl, &pd, &ab, &off));
  napi_is_typedarray(env, argv[3], &ta);
  if (!ta) return throw_rt0(env, RT0_E_ARG, "indices must be an Int32Array");
  NAPI_OK(env, napi_get_typedarray_info(env, argv[3], &it, &il, &id, &ab, &off));
  if (pt != napi_float32_array || it != napi_int32_array || pl % 3 || il % 3)
    return throw_rt0(env, RT0_E_ARG, "positions: Float32Array of xyz, indices: Int32Array of triangles");
  RC_OR_THROW(rt0_set_model(c, k, (const float *)pd, (int)(pl / 3), (const int32_t *)id, (int)(il / 3)));
  return nullptr;
}

// readObj(path) -> {positions: Float32Array, indices: Int32Array}
static napi_value ReadObj(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  std::string path = get_string(env, argv[0]);
  float *pos = nullptr;
  int32_t *idx = nullptr;
  int nv = 0, nt = 0;
  int rc = rt0_obj_read(path.c_str(), &pos, &nv, &idx, &nt);
  if (rc != RT0_OK) return throw_rt0(env, rc, ("cannot read OBJ " + path).c_str());
  void *a = nullptr, *b = nullptr;
  napi_value ab1, ab2, ta1, ta2, o;
  napi_create_arraybuffer(env, (size_t)nv * 12, &a, &ab1);
  napi_create_arraybuffer(env, (size_t)nt * 12, &b, &ab2);
  memcpy(a, pos, (size_t)nv * 12);
  memcpy(b, idx, (size_t)nt * 12);
  rt0_free(pos);
  rt0_free(idx);
  napi_create_typedarray(env, napi_float32_array, (size_t)nv * 3, ab1, 0, &ta1);
  napi_create_typedarray(env, napi_int32_array, (size_t)nt * 3, ab2, 0, &ta2);
  napi_create_object(env, &o);
  set(env, o, "positions", ta1);
  set(env, o, "indices", ta2);
  return o;
}

// readPng(path) / readImage(path) -> {width, height, data: Uint8Array (RGBA8,
// first row = top)}; PNG or baseline JPEG
static napi_value ReadPng(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  std::string path = get_string(env, argv[0]);
  int w = 0, h = 0;
  uint8_t *px = nullptr;
  // PNG or baseline JPEG by signature (textures are PNG, cubemap faces JPEG)
  unsigned char sig[2] = {0, 0};
  if (FILE *f = fopen(path.c_str(), "rb")) {
    if (fread(sig, 1, 2, f) != 2) sig[0] = 0;
    fclose(f);
  }
  int rc = (sig[0] == 0xFF && sig[1] == 0xD8) ? rt0_jpeg_read(path.c_str(), &w, &h, &px)
                                               : rt0_png_read(path.c_str(), &w, &h, &px);
  if (rc != RT0_OK) return throw_rt0(env, rc, ("cannot read image " + path).c_str());
  void *data = nullptr;
  napi_value ab, ta, o;
  size_t n = (size_t)w * h * 4;
  if (napi_create_arraybuffer(env, n, &data, &ab) != napi_ok) {
    rt0_free(px);
    return throw_rt0(env, RT0_E_ARG, "out of memory");
  }
  memcpy(data, px, n);
  rt0_free(px);
  NAPI_OK(env, napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta));
  napi_create_object(env, &o);
  set(env, o, "width", num(env, w));
  set(env, o, "height", num(env, h));
  set(env, o, "data", ta);
  return o;
}

static napi_value LastKernelMs(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  float ms = 0;
  int n = 0;
  RC_OR_THROW(rt0_last_kernel_ms(c, &ms, &n));
  return num(env, ms);
}

// setWavefront(h, mode): rt0_set_wavefront (0 off, 1 SDF scenes, 2 also ReSTIR model scenes)
static napi_value SetWavefront(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  int32_t mode = 1;
  napi_get_value_int32(env, argv[1], &mode);
  RC_OR_THROW(rt0_set_wavefront(c, mode));
  return nullptr;
}

// lastRenderPath(h): which kernels the last render ran (rt0_last_render_path)
static napi_value LastRenderPath(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return nullptr;
  CTX_OR_THROW(argv[0]);
  static const char *names[] = {"", "aot", "pass", "deferred", "wavefront"};
  const int k = rt0_last_render_path(c);
  napi_value v;
  napi_create_string_utf8(env, k >= 0 && k <= 4 ? names[k] : "", NAPI_AUTO_LENGTH, &v);
  return v;
}

static napi_value Version(napi_env env, napi_callback_info) {
  napi_value v;
  napi_create_string_utf8(env, rt0_version(), NAPI_AUTO_LENGTH, &v);
  return v;
}

static napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"version", nullptr, Version, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"parseConfig", nullptr, ParseConfig, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"parseScene", nullptr, ParseScene, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"create", nullptr, Create, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setConfig", nullptr, SetConfig, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setScene", nullptr, SetScene, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setCamera", nullptr, SetCamera, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"render", nullptr, Render, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setTemporalFrames", nullptr, SetTemporalFrames, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setExecutorCompat", nullptr, SetExecutorCompat, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setTextureFilter", nullptr, SetTextureFilter, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setViewport", nullptr, SetViewport, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"readAccum", nullptr, ReadAccum, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"tonemap", nullptr, Tonemap, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"clear", nullptr, Clear, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"resize", nullptr, Resize, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"lastKernelMs", nullptr, LastKernelMs, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setWavefront", nullptr, SetWavefront, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"lastRenderPath", nullptr, LastRenderPath, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setTexture", nullptr, SetTexture, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"readPng", nullptr, ReadPng, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"readImage", nullptr, ReadPng, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setCubemap", nullptr, SetCubemap, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setModel", nullptr, SetModel, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"readObj", nullptr, ReadObj, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
