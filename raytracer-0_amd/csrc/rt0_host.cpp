// rt0_host.cpp -- the C ABI of include/rt0.h over HIP.
//
// Replaces GlslViewport's GL plumbing (index.js:4-1105): device buffers instead
// of textures, kernel launches instead of gl.drawArrays, pointer rotation for
// the ReSTIR swap chain (index.js:795-820) and the accumulator ping-pong.
// Product code: there is no CPU fallback -- without a HIP device every render
// entry point fails with RT0_E_HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include "../../include/rt0.h"
#include "rt0_device.h"
#include "rt0_internal.h"
#include "rt0_jit.h"

extern "C" hipError_t rt0_launch_pass(int variant, const LaunchParams *p, dim3 grid, hipStream_t stream);
extern "C" hipError_t rt0_launch_tonemap(const float4 *acc, uchar4 *out, int n, float cont, int mode,
                                         hipStream_t stream);
extern "C" hipError_t rt0_launch_sum(const LaunchParams *p, dim3 grid, hipStream_t stream);
extern "C" hipError_t rt0_bvh_build(int n, const float *d_v, const int32_t *d_model, float3 lo, float3 hi,
                                    BvhNode *d_nodes, TriDev *d_tris, int *depth_out,
                                    hipStream_t s);

// A pass launch with fewer than kTargetWaves waves (16 per SIMD of the 1024
// SIMDs) is frame-chunked up to kChunkWaves (measured on one 1/2/4/8-way band
// shard of the 1024^2 bench image: 0.96 / 0.95 / 0.91 of linear for 2 / 4 / 8
// shards, against 0.89 / 0.78 / 0.61 unchunked).
static const long kTargetWaves = 16384;
static const long kChunkWaves = 65536;
// BVH nodes ordered breadth-first at the top of the tree (whole levels, at
// most this many): the scene-specialised kernels stage the first RT0_TREELET
// of them in LDS (rt0_jit.cpp: 64 x 64 B = 4 KiB per workgroup, six levels of
// a full tree -- with the 12 KiB traversal stack the pass kernel still holds
// 8 workgroups per CU in 160 KiB); the order itself serves any capacity up to
// seven levels
static const int kTreeletNodes = 128;
// pass-wave record regions per light-sampling wave (JitKey::nee_regions)
static long nee_regions_per_wave() { return 2L; }
// deferred ReSTIR keys without the walk kernel: rt0_jit_nee completes its
// pixels' samples (rt0_integrator.h RT0_FUSED_RESOLVE), no resolve launch;
// RT0_FUSED_RESOLVE=0 keeps rt0_jit_resolve (read when the module is built:
// a test compares the two bit for bit)
static bool fused_resolve() {
  const char *e = getenv("RT0_FUSED_RESOLVE");
  return !e || atoi(e) != 0;
}

enum { R_OUT_MAIN = 0, R_OUT_AUX, R_BACK_MAIN, R_BACK_AUX, R_H1, R_H1A, R_H2, R_H2A, R_COUNT };
// The reservoir textures are four interleaved pair buffers (rt0_integrator.h
// RT0_RES_STRIDE): d_restir[2k] = a pair's base = its main plane (texel i at
// float4 2i), d_restir[2k + 1] = base + 1 float4 = its aux plane.  The swap
// chain moves main and aux pointers together, so every pair stays a pair.
static float4 *pair_aux(float4 *base) { return base + 1; }

struct rt0_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int W = 0, H = 0;
  rt0_config cfg{};
  bool has_scene = false;
  std::vector<rt0_mesh> meshes;
  int n_meshes = 0, n_sdfs = 0, n_models = 0;
  std::vector<int32_t> lights;
  // triangle models (rt0_set_model), object space; instanced by the scene's
  // TRIANGLE entries (pos = translation, joker.x = scale) into one world-space LBVH
  struct Model {
    std::vector<float> pos;
    std::vector<int32_t> tri;
  };
  std::vector<Model> models;
  bool bvh_dirty = false;
  BvhNode *d_bvh = nullptr;
  TriDev *d_tris = nullptr;
  int n_tris = 0, bvh_depth = 0;
  int treelet = 0;  // leading BVH nodes staged in LDS (bvh_treelet_order; 0: LBVH build)
  SceneDev *d_scene = nullptr;
  float cam_pos[3] = {0.f, 0.f, 2.8f}, cam_look[3] = {0.f, 0.f, -1.f}, cam_params[3] = {50.f, 0.f, 3.5f};
  float4 *d_accum = nullptr;
  float4 *ext_accum = nullptr;  // caller-owned accumulator (rt0_set_accum_buffer)
  bool compact = false;         // ext_accum holds only this shard's bands (rt0_set_accum_buffer_compact)
  int compact_rows = 0;         // owned_rows() when the compact buffer was set (its row capacity)
  float4 *acc() const { return ext_accum ? ext_accum : d_accum; }
  // rows of this shard's bands: the band-compressed grid height
  int owned_rows() const {
    const int total = (H + band - 1) / band;
    return (total / n_shards + (shard < total % n_shards ? 1 : 0)) * band;
  }
  // rows the accumulator buffer holds
  int accum_rows() const { return compact ? owned_rows() : H; }
  float4 *d_restir[R_COUNT] = {};
  uchar4 *d_tonemap = nullptr;
  unsigned long long *d_counters = nullptr;
  bool counting = false;
  int temporal_frames = 5;
  int vp[4] = {0, 0, 0, 0};  // gl.viewport (x, y, w, h); w or h <= 0 = whole canvas  // GlslViewport.temporalFrames (index.js:236) -> u_temporalFrames
  uint64_t counters[RT0_N_COUNTERS] = {};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0.f;
  int last_launches = 0;
  int last_path = 0;  // RT0_PATH_* of the last render
  int shard = 0, n_shards = 1, band = 16;
  int halo = 0;                  // rows of exchanged reservoir halo (sharded ReSTIR)
  bool ext_restir = false;       // reservoir planes owned by the caller (rt0_set_restir_buffers)
  uint32_t *d_halo_miss = nullptr;
  float4 *d_samples = nullptr;   // per-frame samples of frame-chunked launches
  size_t samples_bytes = 0;
  int max_frames_per_launch = 64;
  uint32_t *d_tex[RT0_TEX_UNITS] = {};  // asset textures (rt0_set_texture)
  int tex_w[RT0_TEX_UNITS] = {}, tex_h[RT0_TEX_UNITS] = {};
  uint32_t *d_cube = nullptr;  // cubemap faces, GL order (rt0_set_cubemap)
  int cube_size = 0;
  SceneDev host_scene;   // what d_scene holds (also the JIT's scene data)
  bool use_jit = true;   // scene-specialised kernels (rt0_jit.cpp); RT0_JIT=0 disables
  bool exec_compat = false;  // rt0_set_executor_compat: F_EXEC_GHOST
  int tex_filter = RT0_TEX_FILTER_FIXED16;  // rt0_set_texture_filter: F_TEX_FIXED
  // executor compatibility, rule 11 (Integrator::light_q): per-pixel light-loop
  // records of a frame's recording launch, and the accumulator it writes to
  uint2 *d_quad = nullptr;
  float4 *d_quad_acc = nullptr;
  size_t quad_pixels = 0;
  // the scene-specialised kernel of the current (scene, config): looked up once
  // per change instead of regenerating and hashing its source on every render
  rt0h::JitFns jit;
  bool jit_dirty = true;
  // deferred ReSTIR light sampling (RT0_DEFER_NEE, default on): the calls one
  // pass appends (NeeRec), their results (one float4 plane per call index),
  // the paths' own radiance + hero wavelength, and the calls per pixel
  bool defer_nee = true;
  NeeRec *d_nee_rec = nullptr;
  uint32_t *d_nee_count = nullptr;  // records per pass wave
  float4 *d_nee_out = nullptr, *d_nee_partial = nullptr;
  WalkJob *d_walk_jobs = nullptr;  // RT0_NEE_WALK buffers (LaunchParams::walk_*)
  uint32_t *d_walk_count = nullptr, *d_walk_res = nullptr;
  size_t walk_jobs_n = 0, walk_res_n = 0, walk_waves_n = 0;
  int32_t *d_nee_n = nullptr;
  size_t nee_slots = 0;  // records d_nee_rec holds (pass waves x 64 x calls per lane)
  size_t nee_waves = 0;  // entries of d_nee_count
  size_t nee_pixels = 0;
  size_t nee_planes = 0;  // float4 planes of the image d_nee_out holds (one per call index)
  // wavefront SDF rounds (rt0_integrator.h wf_shade_body; LaunchParams::wf_*):
  // one allocation carved into the path state, two march lists, the march
  // answers, the shadow list and its answers, sized for wf_bytes
  void *d_wf = nullptr;
  size_t wf_bytes = 0;
  int wavefront = 1;  // rt0_set_wavefront mode (RT0_WAVEFRONT=<mode> at rt0_create)
  hipStream_t wf_streams[3] = {};  // the wavefront halves' extra streams (wf_render)
  hipEvent_t wf_fork = nullptr, wf_join[3] = {};
  std::string jit_err;
  std::string err;
};

static int fail(rt0_ctx *c, int code, const std::string &msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(c, expr)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail((c), RT0_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void free_buffers(rt0_ctx *c) {
  if (c->d_accum) (void)hipFree(c->d_accum);
  for (int i = 0; i < R_COUNT; i += 2)  // (the pair bases)
    if (c->d_restir[i] && !c->ext_restir) (void)hipFree(c->d_restir[i]);
  for (auto &p : c->d_restir) p = nullptr;
  c->ext_restir = false;
  if (c->d_tonemap) (void)hipFree(c->d_tonemap);
  c->d_accum = nullptr;
  c->d_tonemap = nullptr;
}

static int alloc_buffers(rt0_ctx *c, int w, int h) {
  size_t n = (size_t)w * h;
  HIPCHK(c, hipMalloc(&c->d_accum, n * sizeof(float4)));
  for (int i = 0; i < R_COUNT; i += 2) {
    HIPCHK(c, hipMalloc(&c->d_restir[i], 2 * n * sizeof(float4)));
    c->d_restir[i + 1] = pair_aux(c->d_restir[i]);
  }
  HIPCHK(c, hipMalloc(&c->d_tonemap, n * sizeof(uchar4)));
  c->W = w;
  c->H = h;
  return RT0_OK;
}

static int clear_buffers(rt0_ctx *c) {
  size_t n = (size_t)c->W * c->H * sizeof(float4);
  HIPCHK(c, hipMemsetAsync(c->acc(), 0, (size_t)c->W * c->accum_rows() * sizeof(float4), c->stream));
  for (int i = 0; i < R_COUNT; i += 2) HIPCHK(c, hipMemsetAsync(c->d_restir[i], 0, 2 * n, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT0_OK;
}

// Diagnostics: RT0_SEGV_TRACE=1 prints the native stack of a segmentation
// fault to stderr (then the previous handler -- e.g. Python's faulthandler --
// runs).  Installed at the first rt0_create.
static struct sigaction g_prev_segv;
static void put_hex(char *buf, int *len, uintptr_t v) {  // async-signal-safe formatting
  char t[2 + 2 * sizeof v];
  int n = 0;
  do {
    t[n++] = "0123456789abcdef"[v & 15];
    v >>= 4;
  } while (v);
  buf[(*len)++] = '0';
  buf[(*len)++] = 'x';
  while (n) buf[(*len)++] = t[--n];
}
static void segv_trace(int sig, siginfo_t *si, void *) {
  char msg[96];
  int len = 0;
  static const char head[] = "rt0: SIGSEGV at address ";
  memcpy(msg, head, sizeof head - 1);
  len = sizeof head - 1;
  put_hex(msg, &len, (uintptr_t)(si ? si->si_addr : nullptr));
  static const char tail[] = "; native stack:\n";
  memcpy(msg + len, tail, sizeof tail - 1);
  len += sizeof tail - 1;
  (void)!write(2, msg, (size_t)len);
  void *frames[64];
  const int n = backtrace(frames, 64);  // libgcc preloaded at install: no allocation here
  backtrace_symbols_fd(frames, n, 2);
  // the fault repeats into the previous handler; an ignored or default
  // disposition would re-execute the faulting instruction forever or be lost
  if (!(g_prev_segv.sa_flags & SA_SIGINFO) &&
      (g_prev_segv.sa_handler == SIG_IGN || g_prev_segv.sa_handler == SIG_DFL)) {
    signal(sig, SIG_DFL);
    raise(sig);
    return;
  }
  sigaction(SIGSEGV, &g_prev_segv, nullptr);
}
static void install_segv_trace() {
  static bool done = false;
  if (done || !getenv("RT0_SEGV_TRACE")) return;
  done = true;
  void *warm[2];
  (void)backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
  // an alternate stack (this thread's), so that a stack overflow can be reported too
  static char altstack[1 << 16];
  stack_t ss;
  memset(&ss, 0, sizeof ss);
  ss.ss_sp = altstack;
  ss.ss_size = sizeof altstack;
  sigaltstack(&ss, nullptr);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}

extern "C" {

const char *rt0_version(void) { return "rt0-mi355x 0.1 (gfx950)"; }

int rt0_create(int width, int height, int device, rt0_ctx **out) {
  if (!out || width <= 0 || height <= 0) return RT0_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT0_E_HIP;
  if (device < 0 || device >= ndev) return RT0_E_ARG;
  install_segv_trace();
  rt0_ctx *c = new rt0_ctx();
  c->device = device;
  if (const char *e = getenv("RT0_JIT")) c->use_jit = atoi(e) != 0;
  if (const char *e = getenv("RT0_DEFER_NEE")) c->defer_nee = atoi(e) != 0;
  if (const char *e = getenv("RT0_WAVEFRONT")) c->wavefront = std::max(0, std::min(2, atoi(e)));
  rt0h::default_config(c->cfg);
  int rc;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipMalloc(&c->d_scene, sizeof(SceneDev)) != hipSuccess ||
      hipMalloc(&c->d_counters, RT0_N_COUNTERS * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&c->d_halo_miss, sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->d_halo_miss, 0, sizeof(uint32_t)) != hipSuccess) {
    rt0_destroy(c);
    return RT0_E_HIP;
  }
  if ((rc = alloc_buffers(c, width, height)) != RT0_OK || (rc = clear_buffers(c)) != RT0_OK) {
    rt0_destroy(c);
    return rc;
  }
  *out = c;
  return RT0_OK;
}

void rt0_destroy(rt0_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_buffers(c);
  if (c->d_scene) (void)hipFree(c->d_scene);
  if (c->d_counters) (void)hipFree(c->d_counters);
  if (c->d_halo_miss) (void)hipFree(c->d_halo_miss);
  if (c->d_samples) (void)hipFree(c->d_samples);
  for (void *q : {(void *)c->d_walk_jobs, (void *)c->d_walk_count, (void *)c->d_walk_res})
    if (q) (void)hipFree(q);
  for (void *q : {(void *)c->d_nee_rec, (void *)c->d_nee_count, (void *)c->d_nee_out, (void *)c->d_nee_partial,
                  (void *)c->d_nee_n, c->d_wf, (void *)c->d_quad, (void *)c->d_quad_acc})
    if (q) (void)hipFree(q);
  for (auto &t : c->d_tex)
    if (t) (void)hipFree(t);
  if (c->d_cube) (void)hipFree(c->d_cube);
  if (c->d_bvh) (void)hipFree(c->d_bvh);
  if (c->d_tris) (void)hipFree(c->d_tris);
  for (auto &s : c->wf_streams)
    if (s) (void)hipStreamDestroy(s);
  if (c->wf_fork) (void)hipEventDestroy(c->wf_fork);
  for (auto &e : c->wf_join)
    if (e) (void)hipEventDestroy(e);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char *rt0_last_error(const rt0_ctx *c) { return c ? c->err.c_str() : "null context"; }

int rt0_parse_config(const char *const *defines, int nd, const char *const *constants, int nc, rt0_config *out) {
  if (!out || nd < 0 || nc < 0) return RT0_E_ARG;
  std::string err;
  return rt0h::parse_config(defines, nd, constants, nc, *out, err);
}

int rt0_set_config(rt0_ctx *c, const rt0_config *cfg) {
  if (!c || !cfg) return RT0_E_ARG;
  if (cfg->render_mode != 0 && cfg->render_mode != 1) return fail(c, RT0_E_ARG, "RENDER_MODE must be 0 or 1");
  if (cfg->max_bounces < 0 || cfg->marching_steps < 0) return fail(c, RT0_E_ARG, "negative loop bound");
  c->cfg = *cfg;
  c->jit_dirty = true;
  return RT0_OK;
}

int rt0_get_config(const rt0_ctx *c, rt0_config *out) {
  if (!c || !out) return RT0_E_ARG;
  *out = c->cfg;
  return RT0_OK;
}

static int upload_scene(rt0_ctx *c) {
  SceneDev s = rt0h::make_scene_dev(c->meshes.data(), c->n_meshes, c->n_sdfs, c->n_models, c->lights.data(),
                                    (int)c->lights.size());
  HIPCHK(c, hipSetDevice(c->device));
  c->host_scene = s;
  c->jit_dirty = true;
  HIPCHK(c, hipMemcpyAsync(c->d_scene, &s, sizeof s, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->has_scene = true;
  c->bvh_dirty = true;  // the TRIANGLE entries' transforms / materials may have changed
  return RT0_OK;
}

static int validate_and_store(rt0_ctx *c, const rt0_mesh *m, int ne, int ns, int nm, const int32_t *li, int nl) {
  if (ne < 0 || ns < 0 || nm < 0 || nl < 0) return fail(c, RT0_E_ARG, "negative count");
  if (ne + ns + nm > RT0_MAX_MESH) return fail(c, RT0_E_UNSUPPORTED, "too many meshes");
  if (nl > RT0_MAX_LIGHTS) return fail(c, RT0_E_UNSUPPORTED, "too many lights");
  if (ne + ns + nm == 0) return fail(c, RT0_E_ARG, "empty scene");  // meshes[hit.index] needs meshes[0]
  for (int i = 0; i < ne + ns + nm; i++) {
    if (m[i].tex_type < -1 || m[i].tex_type > 9) return fail(c, RT0_E_ARG, "bad texture type");
    bool sdf = m[i].type == 3, tri = m[i].type == 5;
    if (i >= ne + ns ? !tri : (i >= ne ? !sdf : (sdf || tri)))
      return fail(c, RT0_E_ARG, "meshes must be n_meshes Euclidean, then n_sdfs SDF, then n_models TRIANGLE entries");
    if (!sdf && !tri && (m[i].type < 0 || m[i].type > 2)) return fail(c, RT0_E_UNSUPPORTED, "unsupported mesh type");
    if (sdf && (m[i].sdf_kind < 0 || m[i].sdf_kind > 6)) return fail(c, RT0_E_ARG, "bad sdf_kind");
    if (m[i].mat_type < -1 || m[i].mat_type > 6) return fail(c, RT0_E_ARG, "bad material type");
  }
  for (int i = 0; i < nl; i++)
    if (li[i] >= ne + ns + nm) return fail(c, RT0_E_ARG, "light_index out of range");
  c->meshes.assign(m, m + ne + ns + nm);
  c->n_meshes = ne;
  c->n_sdfs = ns;
  c->n_models = nm;
  c->lights.assign(li, li + nl);
  return upload_scene(c);
}

int rt0_set_scene(rt0_ctx *c, const rt0_mesh *meshes, int n_meshes, int n_sdfs, int n_models,
                  const int32_t *light_index, int n_lights) {
  if (!c || (!meshes && n_meshes + n_sdfs + n_models > 0) || (!light_index && n_lights > 0)) return RT0_E_ARG;
  return validate_and_store(c, meshes, n_meshes, n_sdfs, n_models, light_index, n_lights);
}

int rt0_set_scene_glsl(rt0_ctx *c, const char *scene_text, const char *const *sdf_meshes, int n_sdf) {
  if (!c) return RT0_E_ARG;
  std::vector<rt0_mesh> m;
  std::vector<int32_t> l;
  int ne = 0, ns = 0, nm = 0;
  std::string err;
  int rc = rt0h::parse_scene_glsl(scene_text, sdf_meshes, n_sdf, m, ne, ns, nm, l, err);
  if (rc != RT0_OK) return fail(c, rc, err);
  return validate_and_store(c, m.data(), ne, ns, nm, l.data(), (int)l.size());
}

int rt0_parse_scene_glsl(const char *scene_text, const char *const *sdf_meshes, int n_sdf, rt0_mesh *meshes,
                         int max_meshes, int *n_meshes, int *n_sdfs, int *n_models, int32_t *light_index,
                         int max_lights, int *n_lights) {
  std::vector<rt0_mesh> m;
  std::vector<int32_t> l;
  int ne = 0, ns = 0, nm = 0;
  std::string err;
  int rc = rt0h::parse_scene_glsl(scene_text, sdf_meshes, n_sdf, m, ne, ns, nm, l, err);
  if (rc != RT0_OK) return rc;
  if ((int)m.size() > max_meshes || (int)l.size() > max_lights) return RT0_E_ARG;
  for (size_t i = 0; i < m.size(); i++) meshes[i] = m[i];
  for (size_t i = 0; i < l.size(); i++) light_index[i] = l[i];
  if (n_meshes) *n_meshes = ne;
  if (n_sdfs) *n_sdfs = ns;
  if (n_models) *n_models = nm;
  if (n_lights) *n_lights = (int)l.size();
  return RT0_OK;
}

int rt0_get_scene(const rt0_ctx *c, rt0_mesh *meshes, int max_meshes, int *n_meshes, int *n_sdfs, int *n_models,
                  int32_t *light_index, int max_lights, int *n_lights) {
  if (!c) return RT0_E_ARG;
  if (!c->has_scene) return RT0_E_STATE;
  int n = c->n_meshes + c->n_sdfs + c->n_models;
  if (n_meshes) *n_meshes = c->n_meshes;
  if (n_sdfs) *n_sdfs = c->n_sdfs;
  if (n_models) *n_models = c->n_models;
  if (n_lights) *n_lights = (int)c->lights.size();
  if (meshes)
    for (int i = 0; i < n && i < max_meshes; i++) meshes[i] = c->meshes[i];
  if (light_index)
    for (int i = 0; i < (int)c->lights.size() && i < max_lights; i++) light_index[i] = c->lights[i];
  return RT0_OK;
}

int rt0_set_texture(rt0_ctx *c, int unit, int w, int h, const uint8_t *rgba8) {
  if (!c || unit < 0 || unit >= RT0_TEX_UNITS) return RT0_E_ARG;
  if (rgba8 && (w <= 0 || h <= 0 || (long long)w * h > (1ll << 28)))
    return fail(c, RT0_E_ARG, "texture size out of range");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // a running pass may read the old texels
  if (c->d_tex[unit]) HIPCHK(c, hipFree(c->d_tex[unit]));
  c->d_tex[unit] = nullptr;
  c->tex_w[unit] = c->tex_h[unit] = 0;
  if (!rgba8) return RT0_OK;
  const size_t n = (size_t)w * h * 4;
  HIPCHK(c, hipMalloc(&c->d_tex[unit], n));
  HIPCHK(c, hipMemcpyAsync(c->d_tex[unit], rgba8, n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->tex_w[unit] = w;
  c->tex_h[unit] = h;
  return RT0_OK;
}

int rt0_set_cubemap(rt0_ctx *c, int size, const uint8_t *const faces[6]) {
  if (!c) return RT0_E_ARG;
  if (faces && (size <= 0 || size > 16384)) return fail(c, RT0_E_ARG, "cubemap face size out of range");
  if (faces)
    for (int i = 0; i < 6; i++)
      if (!faces[i]) return fail(c, RT0_E_ARG, "cubemap face is NULL");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->d_cube) HIPCHK(c, hipFree(c->d_cube));
  c->d_cube = nullptr;
  c->cube_size = 0;
  if (!faces) return RT0_OK;
  // reference order (-X, -Y, -Z, +X, +Y, +Z; index.js:301-302) -> GL order
  // (+X, -X, +Y, -Y, +Z, -Z); RGB8 -> RGBA8 so a texel is one aligned dword
  static const int gl_of_ref[6] = {1, 3, 5, 0, 2, 4};
  const size_t n = (size_t)size * size;
  std::vector<uint32_t> host(n * 6);
  for (int i = 0; i < 6; i++) {
    uint32_t *dst = host.data() + n * gl_of_ref[i];
    const uint8_t *src = faces[i];
    for (size_t k = 0; k < n; k++)
      dst[k] = (uint32_t)src[3 * k] | ((uint32_t)src[3 * k + 1] << 8) | ((uint32_t)src[3 * k + 2] << 16) | 0xff000000u;
  }
  HIPCHK(c, hipMalloc(&c->d_cube, host.size() * 4));
  HIPCHK(c, hipMemcpyAsync(c->d_cube, host.data(), host.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->cube_size = size;
  return RT0_OK;
}

int rt0_set_model(rt0_ctx *c, int model, const float *positions, int n_vertices, const int32_t *indices,
                  int n_triangles) {
  if (!c || model < 0 || model >= RT0_MAX_MESH || n_vertices < 0 || n_triangles < 0) return RT0_E_ARG;
  if ((n_vertices && !positions) || (n_triangles && !indices)) return RT0_E_ARG;
  for (long k = 0; k < 3L * n_triangles; k++)
    if (indices[k] < 0 || indices[k] >= n_vertices) return fail(c, RT0_E_ARG, "triangle index out of range");
  if ((int)c->models.size() <= model) c->models.resize(model + 1);
  c->models[model].pos.assign(positions, positions + 3L * n_vertices);
  c->models[model].tri.assign(indices, indices + 3L * n_triangles);
  c->bvh_dirty = true;
  return RT0_OK;
}

// World-space triangles of every TRIANGLE entry (instance k uses model k) ->
// one BVH: the binned-SAH tree built on the host (rt0_bvh_sah.cpp, default) or
// the device LBVH (rt0_bvh.hip; RT0_BVH_BUILD=lbvh).  Runs at the first render
// after a scene/model change.
// (A 4-wide collapse of the SAH tree was measured slower on C5 -- 9.66 vs
// 8.32 ms per pass, profiles/r05/c5_bvh4 -- and removed: scripts/ab_r5_bvh4.patch.)
static bool bvh_builder_sah() {
  static const bool sah = !(getenv("RT0_BVH_BUILD") && std::string(getenv("RT0_BVH_BUILD")) == "lbvh");
  return sah;
}
static int build_bvh(rt0_ctx *c) {
  c->bvh_dirty = false;
  std::vector<float> v;
  std::vector<int32_t> owner;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = 0; k < c->n_models; k++) {
    const rt0_mesh &m = c->meshes[c->n_meshes + c->n_sdfs + k];
    if (m.joker[0] == 0.0f || k >= (int)c->models.size()) continue;  // skipped like intersection()'s joker.x == 0
    const auto &M = c->models[k];
    const int32_t tag = k | ((m.mat_opts & 8u) ? RT0_TRI_CULL_BIT : 0);
    for (size_t t = 0; t + 2 < M.tri.size(); t += 3) {
      for (int j = 0; j < 3; j++) {
        const float *p = &M.pos[3 * (size_t)M.tri[t + j]];
        for (int a = 0; a < 3; a++) {
          const float w = m.pos[a] + m.joker[0] * p[a];
          v.push_back(w);
          lo[a] = std::min(lo[a], w);
          hi[a] = std::max(hi[a], w);
        }
      }
      owner.push_back(tag);
    }
  }
  const int n = (int)owner.size();
  if (c->d_bvh) HIPCHK(c, hipFree(c->d_bvh));
  if (c->d_tris) HIPCHK(c, hipFree(c->d_tris));
  c->d_bvh = nullptr;
  c->d_tris = nullptr;
  c->n_tris = 0;
  c->bvh_depth = 0;
  c->treelet = 0;
  if (n == 0) return RT0_OK;
  HIPCHK(c, hipMalloc(&c->d_bvh, (size_t)std::max(1, n - 1) * sizeof(BvhNode)));
  HIPCHK(c, hipMalloc(&c->d_tris, (size_t)n * sizeof(TriDev)));
  int depth = 0;
  if (bvh_builder_sah()) {
    std::vector<BvhNode> nodes;
    std::vector<TriDev> tris;
    depth = rt0h::bvh_build_sah(n, v.data(), owner.data(), nodes, tris);
    c->treelet = rt0h::bvh_treelet_order(nodes, kTreeletNodes);
    HIPCHK(c, hipMemcpy(c->d_bvh, nodes.data(), nodes.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_tris, tris.data(), tris.size() * sizeof(TriDev), hipMemcpyHostToDevice));
  } else {
    float *d_v = nullptr;
    int32_t *d_owner = nullptr;
    HIPCHK(c, hipMalloc(&d_v, v.size() * sizeof(float)));
    HIPCHK(c, hipMalloc(&d_owner, owner.size() * sizeof(int32_t)));
    HIPCHK(c, hipMemcpyAsync(d_v, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d_owner, owner.data(), owner.size() * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    hipError_t e = rt0_bvh_build(n, d_v, d_owner, make_float3(lo[0], lo[1], lo[2]), make_float3(hi[0], hi[1], hi[2]),
                                 c->d_bvh, c->d_tris, &depth, c->stream);
    (void)hipFree(d_v);
    (void)hipFree(d_owner);
    if (e != hipSuccess) return fail(c, RT0_E_HIP, std::string("BVH build: ") + hipGetErrorString(e));
  }
  if (depth >= RT0_BVH_STACK)
    return fail(c, RT0_E_UNSUPPORTED, "BVH depth " + std::to_string(depth) + " exceeds the traversal stack");
  c->n_tris = n;
  c->bvh_depth = depth;
  c->jit_dirty = true;  // the scene-specialised kernel's traversal stack follows the depth
  return RT0_OK;
}

int rt0_model_info(rt0_ctx *c, int *n_triangles, int *bvh_depth) {
  if (!c) return RT0_E_ARG;
  if (c->has_scene && c->bvh_dirty) {
    HIPCHK(c, hipSetDevice(c->device));
    int rc = build_bvh(c);
    if (rc != RT0_OK) return rc;
  }
  if (n_triangles) *n_triangles = c->n_tris;
  if (bvh_depth) *bvh_depth = c->bvh_depth;
  return RT0_OK;
}

int rt0_set_camera(rt0_ctx *c, const float pos[3], const float lookat[3], const float params[3]) {
  if (!c || !pos || !lookat || !params) return RT0_E_ARG;
  memcpy(c->cam_pos, pos, sizeof c->cam_pos);
  memcpy(c->cam_look, lookat, sizeof c->cam_look);
  memcpy(c->cam_params, params, sizeof c->cam_params);
  return RT0_OK;
}

int rt0_set_shard(rt0_ctx *c, int shard, int n_shards, int band_rows) {
  if (!c || n_shards < 1 || shard < 0 || shard >= n_shards || band_rows < 1) return RT0_E_ARG;
  if (band_rows % 16) return fail(c, RT0_E_ARG, "band_rows must be a multiple of 16");
  if ((c->n_shards > 1) != (n_shards > 1)) c->jit_dirty = true;  // the halo check is compiled in or out
  c->shard = shard;
  c->n_shards = n_shards;
  c->band = band_rows;
  return RT0_OK;
}

// getAnimatedPosition (raytracer.glsl:263-298) for every scene entry at
// u_time = time_ms: uniform over the image, so it is evaluated once per launch
// here (fp32, the shader's operation order) instead of per lane.
static void animated_positions(const rt0_ctx *c, float time_ms, float4 *out) {
  const SceneDev &s = c->host_scene;
  const float t = time_ms * 0.001f;
  for (int i = 0; i < s.n_total && i < RT0_MAX_MESH; i++) {
    const GeomRec &g = s.geom[i];
    float x = g.px, y = g.py, z = g.pz;
    if (i >= 6 && i <= 14) {
      const float radius = 0.6f;
      const float speed = 1.0f + (float)(i - 6) * 0.2f;
      const float phase = (float)(i - 6) * 0.7f;
      const float a = t * speed + phase;
      x = g.px + (cosf(a) * radius) * 0.3f;
      z = g.pz + (sinf(a) * radius) * 0.3f;
      y = g.py + sinf((t * speed) * 2.0f + phase) * 0.1f;
    }
    if (i >= s.n_meshes && s.n_sdfs > 0) {  // SDF entries rotate about y
      const float ang = t * 0.5f;
      const float ca = cosf(ang), sa = sinf(ang);
      const float rx = x * ca - z * sa, rz = x * sa + z * ca;
      x = rx;
      z = rz;
      y = y + sinf(t * 1.5f) * 0.05f;
    }
    out[i] = make_float4(x, y, z, 0.f);
  }
}

static void fill_params(rt0_ctx *c, LaunchParams &p) {
  memset(&p, 0, sizeof p);
  const rt0_config &g = c->cfg;
  p.width = c->W;
  p.height = c->H;
  p.res_x = (float)c->W;
  p.res_y = (float)c->H;
  p.aspect = p.res_x / p.res_y;
  p.cam_px = c->cam_pos[0];
  p.cam_py = c->cam_pos[1];
  p.cam_pz = c->cam_pos[2];
  // camera basis, raytracer.glsl:2127-2133 (float, same operation order)
  float lx = c->cam_look[0], ly = c->cam_look[1], lz = c->cam_look[2];
  float il = 1.0f / sqrtf(lx * lx + ly * ly + lz * lz);
  float wx = lx * il, wy = ly * il, wz = lz * il;
  float cx = wy * 0.0f - 1.0f * wz, cy = wz * 0.0f - 0.0f * wx, cz = wx * 1.0f - 0.0f * wy;  // cross(w, (0,1,0))
  float ic = 1.0f / sqrtf(cx * cx + cy * cy + cz * cz);
  float ux = cx * ic, uy = cy * ic, uz = cz * ic;
  p.ux = ux;
  p.uy = uy;
  p.uz = uz;
  p.vx = uy * wz - wy * uz;
  p.vy = uz * wx - wz * ux;
  p.vz = ux * wy - wx * uy;
  p.wx = wx;
  p.wy = wy;
  p.wz = wz;
  float theta = c->cam_params[0] * 0.01745329f;
  p.uVLen = tanf(theta * 0.5f);
  p.uULen = p.aspect * p.uVLen;
  p.aperture = c->cam_params[1];
  p.focal = c->cam_params[2];
  p.flags = rt0h::flags_from_config(g) | (c->exec_compat ? F_EXEC_GHOST : 0u) |
            (c->tex_filter == RT0_TEX_FILTER_FIXED16 ? F_TEX_FIXED : 0u);
  p.max_bounces = g.max_bounces;
  p.max_diff = g.max_diff_bounces;
  p.max_spec = g.max_spec_bounces;
  p.max_trans = g.max_trans_bounces;
  p.max_scatter = g.max_scattering_events;
  p.marching_steps = g.marching_steps;
  p.fudge = g.fudge_factor;
  p.restir_samples = g.restir_samples;
  p.shard = c->shard;
  p.n_shards = c->n_shards;
  p.band = c->band;
  int total_bands = (c->H + c->band - 1) / c->band;
  int owned = total_bands / c->n_shards + (c->shard < total_bands % c->n_shards ? 1 : 0);
  p.n_band_rows = owned * c->band;
  p.vp_x0 = 0;
  p.vp_y0 = 0;
  p.vp_x1 = c->W;
  p.vp_y1 = p.n_band_rows;
  if (c->vp[2] > 0 && c->vp[3] > 0) {  // clipped to the canvas like gl.viewport's scissor-free draw
    p.vp_x0 = std::max(0, std::min(c->W, c->vp[0]));
    p.vp_y0 = std::max(0, std::min(c->H, c->vp[1]));
    p.vp_x1 = std::max(p.vp_x0, std::min(c->W, c->vp[0] + c->vp[2]));
    p.vp_y1 = std::max(p.vp_y0, std::min(c->H, c->vp[1] + c->vp[3]));
  }
  p.scene = c->d_scene;
  for (int u = 0; u < RT0_TEX_UNITS; u++) {
    p.tex_img[u] = c->d_tex[u];
    p.tex_w[u] = c->tex_w[u];
    p.tex_h[u] = c->tex_h[u];
  }
  p.cube = c->d_cube;
  p.cube_size = c->cube_size;
  p.bvh = c->d_bvh;
  p.tris = c->d_tris;
  p.n_tris = c->n_tris;
  p.treelet = c->treelet;
  p.accum = c->acc();
  p.compact = c->compact ? 1 : 0;
  p.counters = c->d_counters;
  p.ema_alpha = 1.0f / (float)c->temporal_frames;  // raytracer.glsl:2164
  p.halo_rows = 0;
  p.band_inv = 1.0f / (float)c->band;
  p.shards_inv = 1.0f / (float)c->n_shards;
  p.shard_next = (c->shard + 1) % c->n_shards;
  p.shard_prev = (c->shard + c->n_shards - 1) % c->n_shards;
  if (c->n_shards > 1 && (long)c->band * c->n_shards >= c->H) {  // one contiguous block per shard
    const int lo = c->shard * c->band, hi = std::min(c->H, lo + c->band);
    p.valid_lo = std::max(0, lo - c->halo);
    p.valid_hi = std::min(c->H, hi + c->halo);
    p.halo_miss = c->d_halo_miss;
  } else if (c->n_shards > 1) {  // several bands per shard, dealt round-robin
    p.valid_lo = 0;
    p.valid_hi = c->H;
    p.halo_rows = c->halo;  // >= 1 (render_impl)
    p.halo_miss = c->d_halo_miss;
  } else {
    p.valid_lo = 0;
    p.valid_hi = c->H;
    p.halo_miss = nullptr;
  }
}

static int choose_variant(const rt0_ctx *c) {
  const rt0_config &g = c->cfg;
  if (c->counting) return 4;
  if (g.defines & RT0_USE_RESTIR) return 3;
  if (g.defines & (RT0_USE_VOLUMETRICS | RT0_USE_SPECTRAL)) return 2;
  if (c->n_sdfs > 0) return 1;
  return 0;
}

// Wavefront SDF rounds (rt0_integrator.h wf_shade_body) serve the
// scene-specialised renders of SDF scenes without ReSTIR or triangle models,
// whose light-sampling shadow rays are decided by quadric lights: no SDF
// entry is a light or is sampled as one (direct_light's WfShadow), at most 32
// light slots (one bit each in the path state), 1..127 bounces (the state's
// 7-bit counters) -- and the deferred ReSTIR passes of scenes with triangle
// models whose light sampling has the occlusion-walk kernel (`restir_walk`:
// render_impl's want_walk; wf_restir_shade_body).  rt0_set_wavefront(0)
// keeps the pass kernel.
// Executor compatibility with two or more lights and no ReSTIR: rule 11's
// quad-shared light index (Integrator::light_q) -- each frame is a recording
// launch and the frame's launch proper, on the pass kernel.
static bool quad_lights_mode(const rt0_ctx *c) {
  return c->exec_compat && !c->counting && !(c->cfg.defines & RT0_USE_RESTIR) && c->cfg.sample_lights &&
         c->host_scene.n_lights >= 2;
}

static bool wf_eligible(const rt0_ctx *c, bool restir_walk) {
  const SceneDev &s = c->host_scene;
  const rt0_config &g = c->cfg;
  if (!c->wavefront || !c->use_jit || c->counting || g.max_bounces < 1 || g.max_bounces > 127) return false;
  if (quad_lights_mode(c)) return false;  // (the wavefront state holds no light-loop records)
  if (g.defines & RT0_USE_RESTIR) return restir_walk && c->wavefront >= 2;
  if (s.n_sdfs <= 0 || s.n_models > 0 || s.n_lights > 32) return false;
  for (int i = s.n_meshes; i < s.n_meshes + s.n_sdfs; i++)
    if (s.mat[i].type == 0 /* LIGHT */) return false;
  for (int i = 0; i < s.n_lights; i++)
    if (s.light_index[i] >= s.n_meshes) return false;
  return true;
}

// One launch of frames [p.frame0, p.frame0 + p.nframes) as wavefront rounds:
// frame chunks of as many frames as wf_bytes holds, each MAX_BOUNCES + 2
// rounds of the shade and march kernels; the samples land in p.samples and
// rt0_sum_kernel adds them in frame order (the caller launches it).
// ReSTIR (one pass, p.nframes = 1): MAX_BOUNCES + 1 rounds of the shade and
// closest-hit walk kernels over 64-slot regions (one per pass wave); the
// caller then launches the deferred-pass kernels (nee, walk, resolve).
static int wf_render(rt0_ctx *c, LaunchParams &p, dim3 grid) {
  const bool restir = (c->cfg.defines & RT0_USE_RESTIR) != 0;
  const uint32_t L = restir ? 0u : (uint32_t)std::max(1, c->host_scene.n_lights);
  const bool extra = (p.flags & F_MIS) || ((p.flags & F_SPECTRAL) && (c->cfg.defines & RT0_USE_SPECTRAL));
  // bytes per slot: state (per slot for ReSTIR; two list-ordered copies for
  // SDF rounds), two march-list entries, the answer + id, L shadow entries + answers
  const size_t per_slot = (extra ? 48 : 32) * (restir ? 1 : 2) + 2 * 32 + 16 + 4 + (size_t)L * (48 + 16);
  const size_t budget = getenv("RT0_WF_BYTES") ? (size_t)atoll(getenv("RT0_WF_BYTES")) : (size_t)8 << 30;
  const size_t apad = (size_t)grid.x * grid.y * 256;
  // The slots of a frame chunk run as K independent halves on K HIP streams
  // (RT0_WF_STREAMS, default 2): every round ends when its slowest march does
  // (a long march's ~0.2 ms at the end of a nearly empty round), and the other
  // half's kernels fill that tail.
  const int K = std::max(1, std::min(4, getenv("RT0_WF_STREAMS") ? atoi(getenv("RT0_WF_STREAMS")) : 2));
  // slots per region (one shade wave; the march kernel's unit of work): 512,
  // halved down to 128 while a half has fewer than 4 regions per march wave
  // the device holds (an 8-way shard of C4: 8 192 regions of 512 slots for
  // ~8 000 waves left each wave one region and its tail)
  uint32_t kR = 512;
  if (restir) {
    kR = 64;  // the deferred calls' regions are the pass waves'
  } else {
    const size_t waves = (size_t)std::max(1, c->jit.wf_march_blocks) * 4;
    while (kR > 128 && apad * (size_t)p.nframes / K / kR < 4 * waves) kR /= 2;
  }
  // A chunk holds as many whole frames as the budget does; a frame that does
  // not fit (e.g. 4096^2 with 32 lights: ~36 GB) runs as slot chunks of whole
  // regions, so RT0_WF_BYTES bounds the allocation (a slot's frame and pixel
  // follow from its global index, wf_slot0 + slot: any cut is valid)
  const size_t fit = budget / per_slot, unit = (size_t)K * kR;
  const int fc = (int)std::max<size_t>(1, std::min<size_t>((size_t)p.nframes, fit / apad));
  const size_t S = fit >= apad ? apad * (size_t)fc : std::max(unit, fit / unit * unit);  // slots of a chunk
  const size_t Sk = ((S + K - 1) / K + kR - 1) / kR * kR;  // slots of one half (whole regions)
  if (Sk * std::max(1u, L) >= (1ull << 32)) return fail(c, RT0_E_UNSUPPORTED, "wavefront render: too many path slots");
  const size_t NR = Sk / kR, cap = NR * kR;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_state = al(cap * (extra ? 3 : 2) * 16), b_list = al(cap * 32), b_res = al(cap * 16),
               b_id = al(cap * 4), b_sh = al(cap * L * 48), b_shres = al(cap * L * 16), b_cnt = al((NR + 4) * 4);
  const size_t b_ws = restir ? b_state : 0, b_sl = restir ? 0 : b_state;  // per slot (ReSTIR) / list order (SDF)
  const size_t one = b_ws + 2 * b_sl + 2 * b_list + b_res + b_id + b_sh + b_shres + 7 * b_cnt + 512 + 2048;
  if ((size_t)K * one > c->wf_bytes) {
    if (c->d_wf) HIPCHK(c, hipFree(c->d_wf));
    c->d_wf = nullptr;
    c->wf_bytes = 0;
    HIPCHK(c, hipMalloc(&c->d_wf, (size_t)K * one));
    c->wf_bytes = (size_t)K * one;
  }
  for (int k = 0; k < K - 1; k++)
    if (!c->wf_streams[k]) HIPCHK(c, hipStreamCreateWithFlags(&c->wf_streams[k], hipStreamNonBlocking));
  if (!c->wf_fork) HIPCHK(c, hipEventCreateWithFlags(&c->wf_fork, hipEventDisableTiming));
  for (int k = 0; k < 3; k++)
    if (!c->wf_join[k]) HIPCHK(c, hipEventCreateWithFlags(&c->wf_join[k], hipEventDisableTiming));
  hipStream_t st[4] = {c->stream, c->wf_streams[0], c->wf_streams[1], c->wf_streams[2]};
  LaunchParams q[4];
  float4 *lists[4][2], *sts[4][2];
  uint32_t *cnts[4][2];
  for (int k = 0; k < K; k++) {
    LaunchParams &u = q[k];
    u = p;
    char *m = (char *)c->d_wf + (size_t)k * one;
    auto take = [&](size_t b) {
      char *r = m;
      m += b;
      return r;
    };
    u.wf_state = (float4 *)take(b_ws);
    sts[k][0] = (float4 *)take(b_sl);
    sts[k][1] = (float4 *)take(b_sl);
    u.wf_cap = (uint32_t)cap;
    lists[k][0] = (float4 *)take(b_list);
    lists[k][1] = (float4 *)take(b_list);
    u.wf_res = (float4 *)take(b_res);
    u.wf_res_id = (float *)take(b_id);
    u.wf_sh = (float4 *)take(b_sh);
    u.wf_shres = (float4 *)take(b_shres);
    cnts[k][0] = (uint32_t *)take(b_cnt);
    cnts[k][1] = (uint32_t *)take(b_cnt);
    u.wf_sh_cnt = (uint32_t *)take(b_cnt);
    u.wf_ctr = (uint32_t *)take(512);          // 8 range counters, 64 B apart
    u.wf_plan = (uint32_t *)take(4 * b_cnt);   // uint4 per region
    u.wf_plan_bn = (uint32_t *)take(1024);     // per plan block (<= 256)
    u.wf_plan_bj = (uint32_t *)take(1024);
    u.wf_R = (int32_t)kR;
    u.wf_L = (int32_t)L;
    u.wf_apad = (uint32_t)apad;
    u.wf_gx = grid.x;
  }
  // persistent march waves: what the device holds at once, at most one per region
  const unsigned march_blocks = (unsigned)std::min<size_t>((size_t)c->jit.wf_march_blocks, (NR + 3) / 4);
  const int rounds = p.max_bounces + (restir ? 1 : 2);
  auto launch = [&](void *fn, const LaunchParams &u, unsigned blocks, hipStream_t s) {
    return rt0h::jit_launch(fn, &u, blocks, 1, 1, s) == RT0_OK ? hipSuccess : hipErrorLaunchFailure;
  };
  HIPCHK(c, hipEventRecord(c->wf_fork, c->stream));
  for (int k = 1; k < K; k++) HIPCHK(c, hipStreamWaitEvent(st[k], c->wf_fork, 0));
  for (size_t ck = 0, nck = (size_t)p.nframes * apad; ck < nck;) {
    const int f0 = (int)(ck / apad);  // the chunk's first frame
    const size_t s0 = ck - (size_t)f0 * apad, in_frames = apad * (size_t)std::min(fc, p.nframes - f0) - s0;
    const size_t Sc = std::min(S, in_frames);  // this chunk's slots
    ck += Sc;
    int live = 0;
    for (int k = 0; k < K; k++) {
      LaunchParams &u = q[k];
      u.wf_f0 = f0;
      u.wf_slot0 = (uint32_t)(s0 + std::min(Sc, (size_t)k * Sk));
      u.wf_slots = (uint32_t)(std::min(Sc, (size_t)(k + 1) * Sk) - std::min(Sc, (size_t)k * Sk));
      u.wf_nregions = (int32_t)((u.wf_slots + kR - 1) / kR);
      // plan blocks of >= 256 regions, at most 256 of them (wf_plan_prefix)
      u.wf_plan_span = std::max(256, (u.wf_nregions + 255) / 256);
      u.wf_plan_blocks = std::max(1, (u.wf_nregions + u.wf_plan_span - 1) / u.wf_plan_span);
      if (u.wf_slots > 0) live = k + 1;
    }
    for (int r = 0; r < rounds; r++) {
      for (int k = 0; k < live; k++) {
        LaunchParams &u = q[k];
        u.wf_round = r;
        u.wf_in = lists[k][r & 1];
        u.wf_in_cnt = cnts[k][r & 1];
        u.wf_out = lists[k][(r + 1) & 1];
        u.wf_out_cnt = cnts[k][(r + 1) & 1];
        u.wf_sin = sts[k][r & 1];
        u.wf_sout = sts[k][(r + 1) & 1];
        HIPCHK(c, launch(c->jit.wf_shade, u, (unsigned)((u.wf_nregions + 3) / 4), st[k]));
      }
      if (r + 1 == rounds) break;  // (the last round only finishes samples: nothing to march)
      for (int k = 0; k < live; k++) {
        HIPCHK(c, launch(c->jit.wf_plan, q[k], (unsigned)q[k].wf_plan_blocks, st[k]));
        HIPCHK(c, launch(c->jit.wf_march, q[k], std::max(1u, march_blocks), st[k]));
      }
    }
  }
  for (int k = 1; k < K; k++) {
    HIPCHK(c, hipEventRecord(c->wf_join[k - 1], st[k]));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->wf_join[k - 1], 0));
  }
  return RT0_OK;
}

// A deferred ReSTIR pass as two row halves, each running pass -> nee -> walk
// -> resolve on its own HIP stream.  Within a pass the halves are
// independent -- every kernel reads the previous passes' reservoirs (rin) and
// writes per pixel (accumulator, reservoirs, nee_out planes) or into its own
// record / walk-job ranges -- so one half's kernels fill the other's tails;
// the next pass starts after both (its spatial taps cross the seam).
// RT0_RESTIR_SPLIT: 0 never, 1 two halves, K (<= 4) K row parts; default:
// three parts for scenes with triangle models (C5: 2 parts 2 084-2 088, 3
// parts 2 135-2 138, 4 parts 2 017 Msamples/s)
// (the walk kernel's long glass walks leave tails: C5 2 089 vs 2 046
// Msamples/s), not the quadric-only ones (C3 5 240 vs 5 975: its ~0.1 ms
// kernels lose more to the halves' smaller grids than the tails cost).
// (RT0_RESTIR_SPLIT = K >= 2: K row parts on K streams, at most 4)
static int restir_split_parts(const rt0_ctx *c) {
  const char *e = getenv("RT0_RESTIR_SPLIT");  // (read per render: tests switch it)
  const int v = e ? atoi(e) : -1;
  return v < 0 ? (c->jit.walk != nullptr ? 3 : 1) : std::max(1, std::min(4, v == 1 ? 2 : v));
}
static int restir_split_pass(rt0_ctx *c, const LaunchParams &p, dim3 grid, int K) {
  K = std::max(2, std::min(K, std::min(4, (int)grid.y)));
  for (int k = 0; k < K - 1; k++) {
    if (!c->wf_streams[k]) HIPCHK(c, hipStreamCreateWithFlags(&c->wf_streams[k], hipStreamNonBlocking));
    if (!c->wf_join[k]) HIPCHK(c, hipEventCreateWithFlags(&c->wf_join[k], hipEventDisableTiming));
  }
  if (!c->wf_fork) HIPCHK(c, hipEventCreateWithFlags(&c->wf_fork, hipEventDisableTiming));
  const hipStream_t st[4] = {c->stream, c->wf_streams[0], c->wf_streams[1], c->wf_streams[2]};
  const long R = nee_regions_per_wave();
  size_t wave0 = 0, nee_wave0 = 0;       // the half's first pass wave / light-sampling wave
  HIPCHK(c, hipEventRecord(c->wf_fork, c->stream));
  for (int h = 1; h < K; h++) HIPCHK(c, hipStreamWaitEvent(st[h], c->wf_fork, 0));
  unsigned y0 = 0;  // the part's first tile row
  for (int h = 0; h < K; h++) {
    LaunchParams u = p;
    const unsigned y1 = (unsigned)(((size_t)grid.y * (h + 1)) / K);  // tile rows [y0, y1)
    const dim3 g(grid.x, y1 - y0);
    u.vp_y0 = p.vp_y0 + (int)y0 * 16;
    u.vp_y1 = h == K - 1 ? p.vp_y1 : p.vp_y0 + (int)y1 * 16;
    y0 = y1;
    const size_t waves = (size_t)g.x * g.y * 4, nee_waves = (waves + R - 1) / R;
    u.nee_regions = (int32_t)waves;
    u.nee_rec = p.nee_rec + wave0 * (size_t)p.nee_cap;
    u.nee_count = p.nee_count + wave0;
    if (c->jit.walk) {
      u.walk_jobs = p.walk_jobs + nee_wave0 * 2 * (size_t)R * (size_t)p.nee_cap;
      u.walk_count = p.walk_count + nee_wave0;
      u.walk_res = p.walk_res + 2 * wave0 * (size_t)p.nee_cap;
      u.walk_waves = (int32_t)nee_waves;
    }
    HIPCHK(c, hipMemsetAsync(u.nee_count, 0, waves * sizeof(uint32_t), st[h]));
    auto go = [&](void *fn, unsigned gx, unsigned gy) {
      return rt0h::jit_launch(fn, &u, gx, gy, 1, st[h]) == RT0_OK ? hipSuccess : hipErrorLaunchFailure;
    };
    HIPCHK(c, go(c->jit.pass, g.x, g.y));
    HIPCHK(c, go(c->jit.nee, (unsigned)((nee_waves + 3) / 4), 1));
    if (c->jit.walk) HIPCHK(c, go(c->jit.walk, (unsigned)((nee_waves + 3) / 4), 1));
    if (c->jit.resolve) HIPCHK(c, go(c->jit.resolve, g.x, g.y));  // (null: rt0_jit_nee resolved)
    wave0 += waves;
    nee_wave0 += nee_waves;
  }
  for (int h = 1; h < K; h++) {
    HIPCHK(c, hipEventRecord(c->wf_join[h - 1], st[h]));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->wf_join[h - 1], 0));
  }
  return RT0_OK;
}

static int render_impl(rt0_ctx *c, uint32_t first, int n, float time_ms, bool sync) {
  if (!c || n < 0) return RT0_E_ARG;
  if (!c->has_scene) return fail(c, RT0_E_STATE, "rt0_render before rt0_set_scene*");
  const bool restir = (c->cfg.defines & RT0_USE_RESTIR) != 0;
  // ReSTIR reads neighbouring pixels of the previous passes' reservoirs: a
  // shard owns one contiguous row block or several round-robin bands, whose
  // halo rows the caller exchanges between passes (rt0_device_restir;
  // rt0/shard.py); a halo reaches into the neighbouring bands only
  if (restir && c->n_shards > 1 && (long)c->band * c->n_shards < c->H && c->halo > c->band)
    return fail(c, RT0_E_UNSUPPORTED, "ReSTIR sharding over round-robin bands needs halo <= band_rows (" +
                                          std::to_string(c->halo) + " > " + std::to_string(c->band) + ")");
  // the kernel's round-robin halo check (row_local) treats halo_rows rows of
  // each neighbouring band as local: with no exchanged rows a bilinear tap into
  // a neighbour's edge row would go uncounted
  if (restir && c->n_shards > 1 && (long)c->band * c->n_shards < c->H && c->halo < 1)
    return fail(c, RT0_E_ARG, "ReSTIR sharding over round-robin bands needs halo >= 1 (rt0_set_halo)");
  if (restir && c->n_shards > 1 && n > 1)
    return fail(c, RT0_E_ARG, "sharded ReSTIR renders one pass per call (halo exchange between passes)");
  // a band-packed caller buffer holds exactly the rows of the shard it was set
  // for: a later rt0_set_shard / ReSTIR config would index past its end
  if (c->compact && restir)
    return fail(c, RT0_E_UNSUPPORTED, "band-packed accumulator (rt0_set_accum_buffer_compact) with ReSTIR on");
  if (c->compact && c->owned_rows() != c->compact_rows)
    return fail(c, RT0_E_STATE, "the shard changed after rt0_set_accum_buffer_compact (buffer holds " +
                                    std::to_string(c->compact_rows) + " rows, shard owns " +
                                    std::to_string(c->owned_rows()) + "): set the buffer again");
  HIPCHK(c, hipSetDevice(c->device));
  if (c->bvh_dirty) {
    int rc = build_bvh(c);
    if (rc != RT0_OK) return rc;
  }
  LaunchParams p;
  fill_params(c, p);
  if (p.flags & F_ANIM) animated_positions(c, time_ms, p.apos);
  if (p.n_band_rows == 0 || n == 0) {
    c->last_ms = 0.f;
    c->last_launches = 0;
    return RT0_OK;
  }
  const int variant = choose_variant(c);
  if (c->n_shards > 1 && c->vp[2] > 0 && c->vp[3] > 0)
    return fail(c, RT0_E_UNSUPPORTED, "a viewport (tile rendering) and pixel sharding do not combine");
  if (p.vp_x1 <= p.vp_x0 || p.vp_y1 <= p.vp_y0) {  // empty viewport: nothing to draw
    c->last_ms = 0.f;
    c->last_launches = 0;
    return RT0_OK;
  }
  dim3 grid((p.vp_x1 - p.vp_x0 + 15) / 16, (p.vp_y1 - p.vp_y0 + 15) / 16);
  // scene-specialised kernel (compiled once per scene/config, cached); the
  // counting instance is always the ahead-of-time one
  void *jit_fn = nullptr;
  // ReSTIR light sampling in its own kernel over the pass's appended calls
  // (rt0_integrator.h nee_body): scene-specialised kernels only; the executor
  // ghost (F_EXEC_GHOST) keeps the inline calls
  // (NeeRec packs the call index in 8 bits: deeper paths keep the inline calls)
  const bool defer = restir && c->use_jit && !c->counting && !c->exec_compat && c->defer_nee && p.max_bounces > 0 &&
                     p.max_bounces <= RT0_NEE_MAX_BOUNCES;
  // the occlusion-walk kernel (rt0_integrator.h walk_body) for scenes with
  // triangle models: quadric-only shadow geometry (no SDFs, no textured
  // lights) and RENDER_MODE 0 (Integrator::restir_split), and a grid whose
  // records fit the result tag's 29-bit slot field.  Re-evaluated every render:
  // a viewport or image size change alone can flip it.
  const bool want_walk = defer && c->host_scene.n_models > 0 && c->n_tris > 0 &&
                         c->host_scene.n_sdfs == 0 && !c->host_scene.any_tex && c->cfg.render_mode == 0 &&
                         (size_t)grid.x * grid.y * 4 * 64 * (size_t)p.max_bounces < (1u << 29) - 1u;
  const bool want_wf = wf_eligible(c, want_walk);
  if (!want_wf && c->d_wf) {  // a scene or config the rounds no longer serve: release their state
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->d_wf));
    c->d_wf = nullptr;
    c->wf_bytes = 0;
  }
  if (c->use_jit && !c->counting) {
    if (c->jit_dirty || !(c->jit.pass || c->jit.wf_shade) || (defer != (c->jit.nee != nullptr)) ||
        (defer && want_walk != (c->jit.walk != nullptr)) || want_wf != (c->jit.wf_shade != nullptr)) {
      rt0h::JitKey key = rt0h::make_jit_key(c->cfg, c->n_sdfs);
      if (c->exec_compat) key.flags |= F_EXEC_GHOST;
      key.halo_check = c->n_shards > 1 ? 1 : 0;
      key.bvh_stack = (c->host_scene.n_models > 0 && c->n_tris > 0) ? c->bvh_depth + 1 : 0;
      key.defer = defer ? 1 : 0;
      {  // 16-bit traversal stack entries + high bits in a 64-bit register (rt0_integrator.h BvhStack)
        const int entries = key.bvh_stack > 0 ? rt0h::jit_stack_entries(key) : 0;
        const char *e16 = getenv("RT0_BVH_STACK16");
        key.stack16 = entries > 0 && entries <= 32 && (!e16 || atoi(e16) != 0) &&
                             (long long)c->n_tris - 1 < (1ll << (16 + 64 / entries))
                         ? 1
                         : 0;
      }
      key.nee_regions = (int)nee_regions_per_wave();
      key.walk = want_walk ? 1 : 0;
      key.fused = defer && !want_walk && fused_resolve() ? 1 : 0;
      key.wf = want_wf ? 1 : 0;
      int rc = rt0h::jit_get(c->host_scene, key, c->device, &c->jit, c->jit_err);
      if (rc != RT0_OK) return fail(c, rc, c->jit_err);
      c->jit_dirty = false;
    }
    jit_fn = c->jit.pass;
  }
  // the module's kernels are the wavefront rounds (no pass kernel) for an eligible SDF scene
  const bool wf_run = c->use_jit && !c->counting && c->jit.wf_shade != nullptr;
  const size_t pass_waves = (size_t)grid.x * grid.y * 4;
  if (defer) {
    // a region of 64 lanes x max_bounces records per pass wave: a path makes
    // at most one light-sampling call per bounce (rt0_integrator.h step)
    // (nee_out holds max_bounces planes of the whole image: a config with more
    // bounces needs more planes even when a smaller viewport or shard needs
    // fewer record slots)
    const size_t pixels = (size_t)c->W * c->H, slots = pass_waves * 64 * (size_t)p.max_bounces;
    if (slots > c->nee_slots || pass_waves > c->nee_waves || pixels != c->nee_pixels ||
        (size_t)p.max_bounces > c->nee_planes) {
      for (void **q : {(void **)&c->d_nee_rec, (void **)&c->d_nee_count, (void **)&c->d_nee_out,
                       (void **)&c->d_nee_partial, (void **)&c->d_nee_n}) {
        if (*q) HIPCHK(c, hipFree(*q));
        *q = nullptr;
      }
      c->nee_slots = c->nee_waves = c->nee_pixels = c->nee_planes = 0;
      HIPCHK(c, hipMalloc(&c->d_nee_rec, slots * sizeof(NeeRec)));
      HIPCHK(c, hipMalloc(&c->d_nee_count, pass_waves * sizeof(uint32_t)));
      HIPCHK(c, hipMalloc(&c->d_nee_out, pixels * (size_t)p.max_bounces * sizeof(float4)));
      HIPCHK(c, hipMalloc(&c->d_nee_partial, pixels * sizeof(float4)));
      HIPCHK(c, hipMalloc(&c->d_nee_n, pixels * sizeof(int32_t)));
      c->nee_slots = slots;
      c->nee_waves = pass_waves;
      c->nee_pixels = pixels;
      c->nee_planes = (size_t)p.max_bounces;
    }
    p.defer = 1;
    p.nee_cap = 64 * p.max_bounces;
    p.nee_regions = (int32_t)pass_waves;
    p.nee_rec = c->d_nee_rec;
    p.nee_count = c->d_nee_count;
    p.nee_out = c->d_nee_out;
    p.nee_partial = c->d_nee_partial;
    p.nee_n = c->d_nee_n;
    if (c->jit.walk) {
      // per light-sampling wave: up to two rays per record of its regions
      // (+3: the up to 4 parts of a split pass round their wave counts up apart)
      // p.walk_waves is the exact count (the walk kernel's guard): the padding
      // waves of the unsplit launch must not read counts no nee wave wrote
      const size_t exact = (pass_waves + nee_regions_per_wave() - 1) / nee_regions_per_wave();
      const size_t waves = exact + 3;
      const size_t jobs = waves * 2 * (size_t)nee_regions_per_wave() * (size_t)p.nee_cap;
      if (jobs > c->walk_jobs_n || 2 * slots > c->walk_res_n || waves > c->walk_waves_n) {
        for (void **q : {(void **)&c->d_walk_jobs, (void **)&c->d_walk_count, (void **)&c->d_walk_res}) {
          if (*q) HIPCHK(c, hipFree(*q));
          *q = nullptr;
        }
        c->walk_jobs_n = c->walk_res_n = c->walk_waves_n = 0;
        HIPCHK(c, hipMalloc(&c->d_walk_jobs, jobs * sizeof(WalkJob)));
        HIPCHK(c, hipMalloc(&c->d_walk_count, waves * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc(&c->d_walk_res, 2 * slots * sizeof(uint32_t)));
        c->walk_jobs_n = jobs;
        c->walk_res_n = 2 * slots;
        c->walk_waves_n = waves;
      }
      p.walk_jobs = c->d_walk_jobs;
      p.walk_count = c->d_walk_count;
      p.walk_res = c->d_walk_res;
      p.walk_waves = (int32_t)exact;
    }
  }
  auto launch = [&](const LaunchParams &lp, unsigned gz, dim3 g) -> hipError_t {
    if (jit_fn) return rt0h::jit_launch(jit_fn, &lp, g.x, g.y, gz, c->stream) == RT0_OK ? hipSuccess : hipErrorLaunchFailure;
    return rt0_launch_pass(variant, &lp, dim3(g.x, g.y, gz), c->stream);
  };
  if (c->counting) HIPCHK(c, hipMemsetAsync(c->d_counters, 0, RT0_N_COUNTERS * sizeof(unsigned long long), c->stream));
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  int launches = 0;
  // two row halves per deferred ReSTIR pass (not with the wavefront rounds,
  // which split their own work)
  const int split_parts = restir && defer && !wf_run ? restir_split_parts(c) : 1;
  const bool split = split_parts > 1 && grid.y >= 2;
  if (restir) {
    for (int k = 0; k < n; k++) {
      p.frame0 = first + (uint32_t)k;
      p.nframes = 1;
      p.rin[0] = c->d_restir[R_BACK_MAIN];
      p.rin[1] = c->d_restir[R_BACK_AUX];
      p.rin[2] = c->d_restir[R_H1];
      p.rin[3] = c->d_restir[R_H1A];
      p.rin[4] = c->d_restir[R_H2];
      p.rin[5] = c->d_restir[R_H2A];
      p.rout_main = c->d_restir[R_OUT_MAIN];
      p.rout_aux = c->d_restir[R_OUT_AUX];
      if (defer && split) {
        // the pass as two row halves on two streams (restir_split_enabled)
        int rc = restir_split_pass(c, p, grid, split_parts);
        if (rc != RT0_OK) return rc;
        launches++;
      } else if (defer) {
        // waves wholly outside the viewport write no count
        HIPCHK(c, hipMemsetAsync(c->d_nee_count, 0, pass_waves * sizeof(uint32_t), c->stream));
        if (wf_run) {  // the pass's paths as wavefront rounds (shade + closest-hit walk)
          int rc = wf_render(c, p, grid);
          if (rc != RT0_OK) return rc;
        } else {
          HIPCHK(c, launch(p, 1, grid));
        }
        // one light-sampling wave per RT0_NEE_REGIONS pass waves' regions
        const unsigned nee_waves = (unsigned)((pass_waves + nee_regions_per_wave() - 1) / nee_regions_per_wave());
        HIPCHK(c, rt0h::jit_launch(c->jit.nee, &p, (nee_waves + 3) / 4, 1, 1, c->stream) == RT0_OK
                      ? hipSuccess
                      : hipErrorLaunchFailure);
        if (c->jit.walk)  // the calls' triangle occlusion queries (resolve completes the calls)
          HIPCHK(c, rt0h::jit_launch(c->jit.walk, &p, (nee_waves + 3) / 4, 1, 1, c->stream) == RT0_OK
                        ? hipSuccess
                        : hipErrorLaunchFailure);
        if (c->jit.resolve)  // (null: rt0_jit_nee completed the samples)
          HIPCHK(c, rt0h::jit_launch(c->jit.resolve, &p, grid.x, grid.y, 1, c->stream) == RT0_OK
                        ? hipSuccess
                        : hipErrorLaunchFailure);
        launches++;  // one pass (rt0_last_kernel_ms)
      } else {
        HIPCHK(c, launch(p, 1, grid));
        launches++;
      }
      // swapReSTIRBuffers, index.js:795-820
      float4 **R = c->d_restir;
      float4 *o2 = R[R_H2], *o2a = R[R_H2A];
      R[R_H2] = R[R_H1];
      R[R_H2A] = R[R_H1A];
      R[R_H1] = R[R_BACK_MAIN];
      R[R_H1A] = R[R_BACK_AUX];
      R[R_BACK_MAIN] = o2;
      R[R_BACK_AUX] = o2a;
      float4 *tm = R[R_OUT_MAIN], *ta = R[R_OUT_AUX];
      R[R_OUT_MAIN] = R[R_BACK_MAIN];
      R[R_OUT_AUX] = R[R_BACK_AUX];
      R[R_BACK_MAIN] = tm;
      R[R_BACK_AUX] = ta;
    }
  } else {
    // the counting instance also carries the ReSTIR plumbing: give it valid planes
    for (int i = 0; i < 6; i++) p.rin[i] = c->d_restir[R_BACK_MAIN + i];
    p.rout_main = c->d_restir[R_OUT_MAIN];
    p.rout_aux = c->d_restir[R_OUT_AUX];
    // Few pixels per device (e.g. one 8-way shard of 1024^2 = 2048 waves for
    // 1024 SIMDs): split the passes of a launch into chunks over grid.z so the
    // device holds ~16 waves per SIMD; samples go to a scratch buffer and
    // rt0_sum_kernel adds them in frame order (bit-identical accumulation).
    const long waves = (long)grid.x * grid.y * 4;
    const long target = kChunkWaves, min_waves = kTargetWaves;
    const int want = (c->counting || waves >= min_waves)
                         ? 1
                         : (int)std::min<long>(c->max_frames_per_launch, (target + waves - 1) / waves);
    if (quad_lights_mode(c)) {
      // rule 11: per frame, a launch that records every pixel's light-loop
      // bounces (its samples go to a scratch accumulator; the rectangle grown
      // to whole 2x2 quads), then the frame, each lane reading its quad's
      // first lane's record
      const size_t pixels = (size_t)c->W * c->H;
      if (pixels != c->quad_pixels) {
        for (void **q : {(void **)&c->d_quad, (void **)&c->d_quad_acc}) {
          if (*q) HIPCHK(c, hipFree(*q));
          *q = nullptr;
        }
        c->quad_pixels = 0;
        HIPCHK(c, hipMalloc(&c->d_quad, pixels * sizeof(uint2)));
        HIPCHK(c, hipMalloc(&c->d_quad_acc, pixels * sizeof(float4)));
        c->quad_pixels = pixels;
      }
      LaunchParams rec = p;
      rec.vp_x0 &= ~1;
      rec.vp_y0 &= ~1;
      rec.accum = c->d_quad_acc;
      rec.compact = 0;
      rec.quad_masks = c->d_quad;
      rec.quad_mode = 1;
      const dim3 rgrid((rec.vp_x1 - rec.vp_x0 + 15) / 16, (rec.vp_y1 - rec.vp_y0 + 15) / 16);
      p.quad_masks = c->d_quad;
      p.quad_mode = 2;
      p.nframes = rec.nframes = 1;
      p.frame_chunk = rec.frame_chunk = 1;
      p.samples = rec.samples = nullptr;
      for (int k = 0; k < n; ++k) {
        p.frame0 = rec.frame0 = first + (uint32_t)k;
        HIPCHK(c, launch(rec, 1, rgrid));
        HIPCHK(c, launch(p, 1, grid));
        launches++;
      }
      n = 0;  // (done: the loop below has nothing left)
    }
    for (int k = 0; k < n; k += c->max_frames_per_launch) {
      p.frame0 = first + (uint32_t)k;
      p.nframes = (n - k) < c->max_frames_per_launch ? (n - k) : c->max_frames_per_launch;
      int chunks = std::min(want, p.nframes);
      if (wf_run) {  // wavefront rounds: samples out, rt0_sum_kernel accumulates
        const size_t need = (size_t)p.nframes * (p.vp_x1 - p.vp_x0) * (p.vp_y1 - p.vp_y0) * sizeof(float4);
        if (need > c->samples_bytes) {
          if (c->d_samples) HIPCHK(c, hipFree(c->d_samples));
          c->d_samples = nullptr;
          c->samples_bytes = 0;
          HIPCHK(c, hipMalloc(&c->d_samples, need));
          c->samples_bytes = need;
        }
        p.samples = c->d_samples;
        p.frame_chunk = p.nframes;
        int rc = wf_render(c, p, grid);
        if (rc != RT0_OK) return rc;
        HIPCHK(c, rt0_launch_sum(&p, grid, c->stream));
        launches++;
        continue;
      }
      if (chunks > 1) {
        p.frame_chunk = (p.nframes + chunks - 1) / chunks;
        chunks = (p.nframes + p.frame_chunk - 1) / p.frame_chunk;
        // one plane per frame over the launch rectangle (sample_plane in rt0_integrator.h)
        const size_t need = (size_t)p.nframes * (p.vp_x1 - p.vp_x0) * (p.vp_y1 - p.vp_y0) * sizeof(float4);
        if (need > c->samples_bytes) {
          if (c->d_samples) HIPCHK(c, hipFree(c->d_samples));
          c->d_samples = nullptr;
          c->samples_bytes = 0;
          HIPCHK(c, hipMalloc(&c->d_samples, need));
          c->samples_bytes = need;
        }
        p.samples = c->d_samples;
        HIPCHK(c, launch(p, (unsigned)chunks, grid));
        HIPCHK(c, rt0_launch_sum(&p, grid, c->stream));
        launches++;  // pass + rt0_sum_kernel: one launch (rt0_last_kernel_ms)
      } else {
        p.frame_chunk = p.nframes;
        p.samples = nullptr;
        HIPCHK(c, launch(p, 1, grid));
        launches++;
      }
    }
  }
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  c->last_launches = launches;
  c->last_path = wf_run ? RT0_PATH_WAVEFRONT : defer ? RT0_PATH_DEFERRED : jit_fn ? RT0_PATH_PASS : RT0_PATH_AOT;
  if (sync) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    if (c->counting) {
      unsigned long long h[RT0_N_COUNTERS];
      HIPCHK(c, hipMemcpy(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost));
      for (int i = 0; i < RT0_N_COUNTERS; i++) c->counters[i] = h[i];
    }
  }
  return RT0_OK;
}

int rt0_render(rt0_ctx *c, uint32_t first, int n, float time_ms) { return render_impl(c, first, n, time_ms, true); }

int rt0_render_async(rt0_ctx *c, uint32_t first, int n, float time_ms) {
  return render_impl(c, first, n, time_ms, false);
}

int rt0_set_viewport(rt0_ctx *c, int x, int y, int w, int h) {
  if (!c) return RT0_E_ARG;
  c->vp[0] = x;
  c->vp[1] = y;
  c->vp[2] = w;
  c->vp[3] = h;
  return RT0_OK;
}

int rt0_set_temporal_frames(rt0_ctx *c, int n) {
  if (!c || n <= 0) return RT0_E_ARG;
  c->temporal_frames = n;
  return RT0_OK;
}

int rt0_sync(rt0_ctx *c) {
  if (!c) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->last_launches) HIPCHK(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
  if (c->counting) {
    unsigned long long h[RT0_N_COUNTERS];
    HIPCHK(c, hipMemcpy(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost));
    for (int i = 0; i < RT0_N_COUNTERS; i++) c->counters[i] = h[i];
  }
  return RT0_OK;
}

int rt0_read_accum(rt0_ctx *c, float *out) {
  if (!c || !out) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, c->acc(), (size_t)c->W * c->accum_rows() * sizeof(float4), hipMemcpyDeviceToHost));
  return RT0_OK;
}

int rt0_write_accum(rt0_ctx *c, const float *in) {
  if (!c || !in) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->acc(), in, (size_t)c->W * c->accum_rows() * sizeof(float4), hipMemcpyHostToDevice));
  return RT0_OK;
}

int rt0_clear(rt0_ctx *c) {
  if (!c) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  return clear_buffers(c);
}

int rt0_resize(rt0_ctx *c, int w, int h) {
  if (!c || w <= 0 || h <= 0) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  free_buffers(c);
  c->ext_accum = nullptr;  // a caller buffer has the old size
  c->compact = false;
  int rc = alloc_buffers(c, w, h);
  if (rc != RT0_OK) return rc;
  return clear_buffers(c);
}

int rt0_get_size(const rt0_ctx *c, int *w, int *h) {
  if (!c) return RT0_E_ARG;
  if (w) *w = c->W;
  if (h) *h = c->H;
  return RT0_OK;
}

int rt0_tonemap(rt0_ctx *c, float contribution, uint8_t *out) { return rt0_tonemap_ex(c, contribution, 0, out); }

int rt0_tonemap_ex(rt0_ctx *c, float contribution, int mode, uint8_t *out) {
  if (!c || !out || mode < 0 || mode > 2) return RT0_E_ARG;
  // a band-packed shard buffer is not an image (rows in band order, H/N of
  // them): gather it first (rt0/shard.py: BandGather) and tonemap the image
  if (c->compact)
    return fail(c, RT0_E_UNSUPPORTED, "rt0_tonemap on a band-packed accumulator (rt0_set_accum_buffer_compact)");
  HIPCHK(c, hipSetDevice(c->device));
  int n = c->W * c->H;
  HIPCHK(c, rt0_launch_tonemap(c->acc(), c->d_tonemap, n, contribution, mode, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, c->d_tonemap, (size_t)n * sizeof(uchar4), hipMemcpyDeviceToHost));
  return RT0_OK;
}

int rt0_read_restir(rt0_ctx *c, int which, float *main_out, float *aux_out) {
  if (!c || which < 0 || which > 2) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // after the swap, the last pass's output sits in restir_buffer_back (index.js:817-819)
  const int mi = which == 0 ? R_BACK_MAIN : which == 1 ? R_H1 : R_H2;
  const size_t n = (size_t)c->W * c->H;
  std::vector<float4> pair(2 * n);  // the interleaved pair, split on the host
  HIPCHK(c, hipMemcpy(pair.data(), c->d_restir[mi], 2 * n * sizeof(float4), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++) {
    if (main_out) memcpy(main_out + 4 * i, &pair[2 * i], sizeof(float4));
    if (aux_out) memcpy(aux_out + 4 * i, &pair[2 * i + 1], sizeof(float4));
  }
  return RT0_OK;
}

int rt0_write_restir_inputs(rt0_ctx *c, const float *sm, const float *sa, const float *h1m, const float *h1a,
                            const float *h2m, const float *h2a) {
  if (!c) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t n = (size_t)c->W * c->H;
  const float *src[6] = {sm, sa, h1m, h1a, h2m, h2a};
  const int dst[6] = {R_BACK_MAIN, R_BACK_AUX, R_H1, R_H1A, R_H2, R_H2A};
  std::vector<float4> pair(2 * n);  // interleaved on the host (zeros where a plane is NULL)
  for (int k = 0; k < 6; k += 2) {
    for (size_t i = 0; i < n; i++) {
      pair[2 * i] = src[k] ? make_float4(src[k][4 * i], src[k][4 * i + 1], src[k][4 * i + 2], src[k][4 * i + 3])
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      pair[2 * i + 1] = src[k + 1] ? make_float4(src[k + 1][4 * i], src[k + 1][4 * i + 1], src[k + 1][4 * i + 2],
                                                 src[k + 1][4 * i + 3])
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    HIPCHK(c, hipMemcpy(c->d_restir[dst[k]], pair.data(), 2 * n * sizeof(float4), hipMemcpyHostToDevice));
  }
  return RT0_OK;
}

int rt0_device_accum(rt0_ctx *c, void **dptr, void **stream) {
  if (!c) return RT0_E_ARG;
  if (dptr) *dptr = c->acc();
  if (stream) *stream = c->stream;
  return RT0_OK;
}

int rt0_set_jit(rt0_ctx *c, int enable) {
  if (!c) return RT0_E_ARG;
  c->use_jit = enable != 0;
  return RT0_OK;
}

int rt0_set_wavefront(rt0_ctx *c, int enable) {
  if (!c) return RT0_E_ARG;
  c->wavefront = std::max(0, std::min(2, enable));  // the next render picks the matching JIT module
  return RT0_OK;
}

int rt0_set_defer_light_sampling(rt0_ctx *c, int enable) {
  if (!c) return RT0_E_ARG;
  c->defer_nee = enable != 0;  // the next render picks the matching JIT module
  return RT0_OK;
}

int rt0_set_executor_compat(rt0_ctx *c, int enable) {
  if (!c) return RT0_E_ARG;
  if (c->exec_compat != (enable != 0)) c->jit_dirty = true;
  c->exec_compat = enable != 0;
  return RT0_OK;
}

int rt0_set_texture_filter(rt0_ctx *c, int mode) {
  if (!c || (mode != RT0_TEX_FILTER_FLOAT && mode != RT0_TEX_FILTER_FIXED16)) return RT0_E_ARG;
  c->tex_filter = mode;
  return RT0_OK;
}

int rt0_set_accum_buffer(rt0_ctx *c, void *dptr) {
  if (!c) return RT0_E_ARG;
  c->ext_accum = (float4 *)dptr;
  c->compact = false;
  return RT0_OK;
}

int rt0_set_accum_buffer_compact(rt0_ctx *c, void *dptr, int *rows) {
  if (!c || !dptr) return RT0_E_ARG;
  if (c->cfg.defines & RT0_USE_RESTIR)
    return fail(c, RT0_E_UNSUPPORTED, "ReSTIR shards keep a full-size accumulator (contiguous row blocks)");
  c->ext_accum = (float4 *)dptr;
  c->compact = true;
  c->compact_rows = c->owned_rows();
  if (rows) *rows = c->compact_rows;
  return RT0_OK;
}

int rt0_set_restir_buffers(rt0_ctx *c, void *const planes[8]) {
  if (!c) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t bytes = (size_t)c->W * c->H * 2 * sizeof(float4);  // one pair buffer
  if (planes) {
    for (int i = 0; i < R_COUNT; i += 2) {
      if (!planes[i] || !planes[i + 1]) return fail(c, RT0_E_ARG, "rt0_set_restir_buffers: null plane");
      if ((char *)planes[i + 1] != (char *)planes[i] + 16)
        return fail(c, RT0_E_ARG, "rt0_set_restir_buffers: planes[2k+1] must be planes[2k] + 16 bytes "
                                  "(interleaved main/aux pairs, W*H*8 floats each)");
    }
    if (!c->ext_restir)
      for (int i = 0; i < R_COUNT; i += 2) (void)hipFree(c->d_restir[i]);
    for (int i = 0; i < R_COUNT; i++) c->d_restir[i] = (float4 *)planes[i];
    c->ext_restir = true;
  } else if (c->ext_restir) {  // back to planes owned by the context
    for (int i = 0; i < R_COUNT; i += 2) {
      HIPCHK(c, hipMalloc(&c->d_restir[i], bytes));
      c->d_restir[i + 1] = pair_aux(c->d_restir[i]);
    }
    c->ext_restir = false;
  }
  for (int i = 0; i < R_COUNT; i += 2) HIPCHK(c, hipMemsetAsync(c->d_restir[i], 0, bytes, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT0_OK;
}

int rt0_device_restir(rt0_ctx *c, int which, void **main_out, void **aux_out) {
  if (!c || which < 0 || which > 2) return RT0_E_ARG;
  static const int M[3] = {R_BACK_MAIN, R_H1, R_H2}, A[3] = {R_BACK_AUX, R_H1A, R_H2A};
  if (main_out) *main_out = c->d_restir[M[which]];
  if (aux_out) *aux_out = c->d_restir[A[which]];
  return RT0_OK;
}

int rt0_set_halo(rt0_ctx *c, int rows) {
  if (!c || rows < 0) return RT0_E_ARG;
  c->halo = rows;
  return RT0_OK;
}

int rt0_read_halo_misses(rt0_ctx *c, uint32_t *misses, int reset) {
  if (!c || !misses) return RT0_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(misses, c->d_halo_miss, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (reset) HIPCHK(c, hipMemset(c->d_halo_miss, 0, sizeof(uint32_t)));
  return RT0_OK;
}

int rt0_set_counting(rt0_ctx *c, int enable) {
  if (!c) return RT0_E_ARG;
  c->counting = enable != 0;
  return RT0_OK;
}

int rt0_read_counters(rt0_ctx *c, uint64_t out[5]) {
  if (!c || !out) return RT0_E_ARG;
  for (int i = 0; i < 5; i++) out[i] = c->counters[i];
  return RT0_OK;
}

int rt0_read_counters_n(rt0_ctx *c, uint64_t *out, int n) {
  if (!c || !out || n < 0) return RT0_E_ARG;
  for (int i = 0; i < n && i < RT0_N_COUNTERS; i++) out[i] = c->counters[i];
  for (int i = RT0_N_COUNTERS; i < n; i++) out[i] = 0;
  return RT0_N_COUNTERS;
}

int rt0_scratch_bytes(const rt0_ctx *c, size_t *bytes) {
  if (!c || !bytes) return RT0_E_ARG;
  // per-frame samples + the wavefront rounds' state + the deferred ReSTIR
  // records, results and walk jobs
  *bytes = c->samples_bytes + c->wf_bytes + c->nee_slots * sizeof(NeeRec) + c->nee_waves * sizeof(uint32_t) +
           c->nee_pixels * (c->nee_planes + 1) * sizeof(float4) + c->nee_pixels * sizeof(int32_t) +
           c->walk_jobs_n * sizeof(WalkJob) + (c->walk_waves_n + c->walk_res_n) * sizeof(uint32_t) +
           c->quad_pixels * (sizeof(uint2) + sizeof(float4));
  return RT0_OK;
}

int rt0_last_render_path(const rt0_ctx *c) { return c ? c->last_path : RT0_E_ARG; }

int rt0_last_kernel_ms(const rt0_ctx *c, float *ms, int *launches) {
  if (!c) return RT0_E_ARG;
  if (ms) *ms = c->last_ms;
  if (launches) *launches = c->last_launches;
  return RT0_OK;
}

}  // extern "C"
