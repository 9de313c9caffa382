// rt0_integrator.h -- raytracer-0's per-pixel integrator for gfx950 (device code).
//
// Included by rt0_kernels.hip (ahead-of-time instances over a scene in HBM) and
// embedded verbatim into librt0.so for the scene-specialising JIT (rt0_jit.cpp):
// like the reference, which recompiles its shader whenever the scene or the
// flags change (index.html:1167-1196), the JIT bakes the scene and the
// constants in as compile-time data so that the mesh loop unrolls and every
// type dispatch / flag test folds away.
//
// Semantics follow shaders/pathtracing/raytracer.glsl line by line (cited per
// function).  Geometry and shading may be FMA-contracted (ulp-level); every
// expression that feeds the RNG or the ReSTIR packing is evaluated in the
// reference's operation order with contraction off (NC(...) helpers), so the
// RNG stream is bit-identical to the reference; hash() reproduces the
// reference executor's uint->float.  Deviation: powerHeuristic's max(0, 0/0)
// is 0 (IEEE maxNum), not NaN.
#pragma once
#ifndef RT0_JIT
#include <hip/hip_runtime.h>
#include "rt0_device.h"
#endif

#define DEV __device__ __forceinline__

namespace rt0 {

constexpr float EPSILON = 0.001f;
constexpr float INF_T = 1e4f;
constexpr float F_INF = __builtin_huge_valf();  // (hipRTC has no INFINITY macro)
constexpr float PI_F = 3.14159265f;
constexpr float ONE_OVER_PI = 0.31830989f;
constexpr float TWO_PI = 6.28318531f;
constexpr float FOUR_PI = 12.5663706f;
constexpr float VOL_SIGMA_T = 0.15f;
constexpr float VOL_SIGMA_S = 0.13f;
constexpr float VOL_G = 0.5f;

enum { T_SPHERE = 0, T_PLANE = 1, T_BOX = 2, T_SDF = 3, T_TRIANGLE = 5 };
enum { M_LIGHT = 0, M_DIR_LIGHT = 1, M_DIFF = 2, M_SPEC = 3, M_REFR_FRESNEL = 4, M_REFR_SCHLICK = 5, M_COAT = 6 };

// ------------------------------------------------------------------ math
struct v3 {
  float x, y, z;
};
DEV v3 mk(float x, float y, float z) { return v3{x, y, z}; }
DEV v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV v3 operator*(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
DEV float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
DEV float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
DEV float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
DEV float fdiv(float a, float b) { return a * frcp(b); }
DEV float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
DEV float step_(float e, float x) { return x < e ? 0.0f : 1.0f; }
DEV float mixf(float x, float y, float a) { return a * (y - x) + x; }
DEV v3 normalize(v3 a) { return a * frsq(dot(a, a)); }
DEV float length(v3 a) { return fsqrt(dot(a, a)); }
DEV v3 vmaxs(v3 a, float s) { return mk(fmaxf(a.x, s), fmaxf(a.y, s), fmaxf(a.z, s)); }
DEV float vmaxc(v3 a) { return fmaxf(a.x, fmaxf(a.y, a.z)); }
DEV v3 vabs(v3 a) { return mk(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
DEV v3 reflect(v3 i, v3 n) { return i - n * (2.0f * dot(n, i)); }
DEV v3 refract(v3 i, v3 n, float eta) {
  float d = dot(n, i);
  float k = 1.0f - eta * eta * (1.0f - d * d);
  if (k < 0.0f) return mk(0.f, 0.f, 0.f);
  return i * eta - n * (eta * d + fsqrt(k));
}
DEV float fsin(float x) { return __sinf(x); }
DEV float fcos(float x) { return __cosf(x); }
// sin/cos(2*pi*t) for t in [0, 1): v_sin/v_cos take revolutions, so the
// reference's angle = 2*pi*t (and __sinf's x * 1/(2*pi)) is two multiplies the
// hardware undoes; the argument differs from sin(fl(2*pi*t)) by an ulp
DEV float fsin_rev(float t) { return __builtin_amdgcn_sinf(t); }
DEV float fcos_rev(float t) { return __builtin_amdgcn_cosf(t); }
DEV float fexp(float x) { return __expf(x); }
DEV float flog(float x) { return __logf(x); }

// ----------------------------------------------- non-contracted arithmetic
// Every helper below is evaluated exactly as the reference writes it (no FMA):
// the RNG seeds feed a bit-level hash, so one fused a*b+c changes the whole
// random stream.  The library and the JIT compile with
// -ffp-contract=fast-honor-pragmas, under which the backend keeps every
// product of a `#pragma clang fp contract(off)` block unfused (checked on the
// gfx950 ISA; plain `fast` ignores the pragma in the backend).  Round 1 also
// hid each such product behind an empty asm; that cost a v_mov + s_nop each
// (5.66 vs 5.80 ms per 64-spp C2 launch) and was dropped in round 2.
// The sharded-ReSTIR halo check of every reservoir tap (row_local).  The
// scene-specialised kernels of unsharded renders are compiled without it
// (rt0_jit.cpp): its integer divisions cost the one-device C3 kernel 0.643 vs
// 0.614 ms per pass even behind the null test of P.halo_miss.
#ifndef RT0_HALO_CHECK
#define RT0_HALO_CHECK 1
#endif
// Deferred light sampling for ReSTIR scenes (NeeRec, rt0_device.h): the
// scene-specialised kernels of ReSTIR scenes are compiled with 1 (rt0_jit.cpp)
#ifndef RT0_DEFER_NEE
#define RT0_DEFER_NEE 0
#endif
#ifndef RT0_NEE_REGIONS  // pass-wave record regions per light-sampling wave
#define RT0_NEE_REGIONS 2
#endif
// ReSTIR reservoir taps fetched per batch (temporal levels together, spatial
// taps RT0_TAP_BATCH at a time); 1 = one tap at a time.  The scene-specialised
// kernels of ReSTIR scenes without models use 2 (rt0_jit.cpp)
#ifndef RT0_TAP_BATCH
#define RT0_TAP_BATCH 1
#endif
#ifndef RT0_NEE_WALK  // light-sampling calls' triangle occlusion queries in rt0_jit_walk (models scenes)
#define RT0_NEE_WALK 0
#endif
#ifndef RT0_WALK_ROOT_TEST  // light-sampling kernel drops walk jobs that miss the root's child boxes
#define RT0_WALK_ROOT_TEST 1
#endif
#ifndef RT0_WALK_SPEC  // rt0_jit_walk postpones leaf tests until half the busy lanes hold one
#define RT0_WALK_SPEC 1
#endif
// ReSTIR reservoir textures (index.js:149-163) as interleaved pairs: texel i
// of a main plane at float4 2i of its pair buffer, the aux plane's at 2i + 1
// (rt0_host.cpp alloc_buffers), so a bilinear tap's main and aux texels share
// 32-B segments instead of touching two planes' lines
#define RT0_RES_STRIDE 2
#ifndef RT0_TREELET  // BVH nodes (top levels) each traversing kernel stages in LDS (bvh_fetch); 0 = none
#define RT0_TREELET 0
#endif
#ifndef RT0_BVH_STACK16  // BVH traversal stacks as 16-bit LDS entries + high bits in a register
#define RT0_BVH_STACK16 0
#endif
// Wavefront SDF renders (rt0_jit_wf_shade / rt0_jit_wf_march, see
// wf_shade_body): the scene-specialised modules of SDF scenes without ReSTIR
// are compiled with 1 (rt0_jit.cpp JitKey::wf)
#ifndef RT0_WAVEFRONT
#define RT0_WAVEFRONT 0
#endif
#ifndef RT0_WF_REFILL  // free lanes that trigger a march-kernel refill (wf_march_body)
#define RT0_WF_REFILL 1
#endif
#ifndef RT0_WF_WALK_REFILL  // free lanes that trigger a walk-kernel refill (wf_walk_body)
#define RT0_WF_WALK_REFILL 16
#endif
#ifndef RT0_WF_INLINE_NODES  // BVH nodes the ReSTIR shade kernel walks before parking a ray (intersect)
#define RT0_WF_INLINE_NODES 1
#endif
#ifndef RT0_WF_UNIT  // entries a march wave takes per device-counter grab, about (wf_march_body)
#define RT0_WF_UNIT 256
#endif
DEV float nc_fract(float x) {
#pragma clang fp contract(off)
  return x - floorf(x);
}
// a + b*c, unfused
DEV float nc_addmul(float a, float b, float c) {
#pragma clang fp contract(off)
  return a + (b * c);
}
// ((s + a*f) + b) + c*d  (raytracer.glsl:1810, 1956, 1972, 2003, 2024, 2046)
DEV float nc_seed4(float s, float a, float f, float b, float c, float d) {
#pragma clang fp contract(off)
  return ((s + (a * f)) + b) + (c * d);
}
// (s + a*f) + c*d  (raytracer.glsl:1909/1943)
DEV float nc_seed3(float s, float a, float f, float c, float d) {
#pragma clang fp contract(off)
  return (s + (a * f)) + (c * d);
}

// ------------------------------------------------------------------- RNG
// raytracer.glsl:302-306.  The last line converts m = (n >> 22) ^ n to float
// the way the reference executor does (the conversion the golden fixtures
// were produced with): float(m - 2^31) + 2^31 above 2^31, two roundings; times
// 2^-32.  Evaluated as fma(float(m mod 2^31), 2^-32, m >= 2^31 ? 0.5 : 0):
// the product is exact (a power of two), so the fma's one rounding is that
// `+ 2^31` scaled by 2^-32 -- the same bits, without a second conversion,
// compare and select
// (5 instead of 7 VALU instructions per call; tests/test_kernel_identities.py)
DEV float hash(float seed) {
#pragma clang fp contract(off)
  uint32_t n = __float_as_uint(seed) * 747796405u + 2891336453u;
  n = ((n >> ((n >> 28u) + 4u)) ^ n) * 277803737u;
  const uint32_t m = (n >> 22u) ^ n;
  const float lo = (float)(int32_t)(m & 0x7fffffffu);
  const float hi = __int_as_float((int32_t)m >> 31 & 0x3f000000);
  return __builtin_fmaf(lo, 2.3283064365386963e-10f, hi);
}
// raytracer.glsl:308-312
DEV void hash2(float sx, float sy, float &ox, float &oy) {
#pragma clang fp contract(off)
  float x = (sx * 0.1031f), y = (sy * 0.1030f);
  x = x - floorf(x);
  y = y - floorf(y);
  float d = (x * (y + 19.19f)) + (y * (x + 19.19f));
  x += d;
  y += d;
  float a = ((x + y) * x), b = ((x + y) * y);
  ox = a - floorf(a);
  oy = b - floorf(b);
}

// ------------------------------------------------------- scene policies
// DynScene: the scene lives in HBM (SceneDev) and is read with wave-uniform
// indices (scalar loads).  A JIT scene (generated by rt0_jit.cpp) provides the
// same interface as compile-time constants with kStatic = true.
struct DynScene {
  static constexpr bool kStatic = false;
  static constexpr int kMeshes = 0, kSdfs = 0, kLights = 0;
  static constexpr bool kMayHaveModels = true;  // runtime check of n_models()
  const SceneDev *__restrict__ S;
  DEV int n_meshes() const { return S->n_meshes; }
  DEV int n_sdfs() const { return S->n_sdfs; }
  DEV int n_models() const { return S->n_models; }
  DEV int n_lights() const { return S->n_lights; }
  DEV GeomRec geom(int i) const { return S->geom[i]; }
  DEV MatRec mat(int i) const { return S->mat[i]; }
  DEV float j3(int i) const { return S->j3[i]; }
  DEV int sdf_kind(int i) const { return S->sdf_kind[i]; }
  DEV int light(int i) const { return S->light_index[i]; }
  DEV bool any_tex() const { return S->any_tex != 0; }
  DEV TexRec tex(int i) const { return S->tex[i]; }
};

// DynCfg: defines/constants as wave-uniform kernel arguments.  A JIT config
// provides the same accessors as constexpr.
struct DynCfg {
  uint32_t fl;
  int mb, md, ms, mt, msc, mst, rs;
  float fud;
  DEV explicit DynCfg(const LaunchParams &P)
      : fl(P.flags), mb(P.max_bounces), md(P.max_diff), ms(P.max_spec), mt(P.max_trans), msc(P.max_scatter),
        mst(P.marching_steps), rs(P.restir_samples), fud(P.fudge) {}
  DEV uint32_t flags() const { return fl; }
  DEV int max_bounces() const { return mb; }
  DEV int max_diff() const { return md; }
  DEV int max_spec() const { return ms; }
  DEV int max_trans() const { return mt; }
  DEV int max_scatter() const { return msc; }
  DEV int marching_steps() const { return mst; }
  DEV int restir_samples() const { return rs; }
  DEV float fudge() const { return fud; }
};

template <int I, int N, class F>
DEV void static_for(F &&f) {
  if constexpr (I < N) {
    f(I);
    static_for<I + 1, N>(f);
  }
}
// loop over meshes [0, n_meshes): fully unrolled with constant indices for a
// static (JIT) scene, a uniform runtime loop otherwise
template <class Scene, class F>
DEV void for_meshes(const Scene &sc, F &&f) {
  if constexpr (Scene::kStatic) static_for<0, Scene::kMeshes>(f);
  else
    for (int i = 0; i < sc.n_meshes(); ++i) f(i);
}
template <class Scene, class F>
DEV void for_lights(const Scene &sc, F &&f) {
  if constexpr (Scene::kStatic) static_for<0, Scene::kLights>(f);
  else
    for (int i = 0; i < sc.n_lights(); ++i) f(i);
}
template <class Scene, class F>
DEV void for_sdfs(const Scene &sc, F &&f) {
  if constexpr (Scene::kStatic) static_for<0, Scene::kSdfs>(f);
  else
    for (int i = 0; i < sc.n_sdfs(); ++i) f(i);
}

// --------------------------------------------------------------- geometry
struct Hit {
  v3 n, pos;
  int index;
  int type;  // -1 miss, else T_* (the uv/texel parser's dispatch, raytracer.glsl:1049-1078)
};

// A sphere-tracing march (iSDF, raytracer.glsl:979-984) handed out of
// intersection() to the kernel's one march loop (SUSP kernels, see
// Integrator::march_pending): the ray, the closest quadric distance it must
// beat, and the loop state (t, step count, last map() id).  Marched in slices
// of RT0_MARCH_BUDGET steps; `done` hands (t, id) back to intersection(),
// which the caller repeats with the same ray -- the same sequence of map()
// evaluations as the reference's uninterrupted loop.
#ifndef RT0_MARCH_BUDGET
#define RT0_MARCH_BUDGET 12  // 8 in rounds 2-3; 12 measured +1% on C4 in round 4
#endif

struct March {
  v3 o, d;
  float tmin, t, id;
  int i;
  bool active, done;
  v3 n;  // RT0_WAVEFRONT: calcNormal at the hit, evaluated by the march kernel
};

// o + d*t as every march step and normal probe evaluates it: one fused
// multiply-add per axis, written out so that every kernel (the pass kernel's
// march, the wavefront march kernel) rounds it the same way
DEV v3 ray_at(v3 o, v3 d, float t) {
  return v3{__builtin_fmaf(d.x, t, o.x), __builtin_fmaf(d.y, t, o.y), __builtin_fmaf(d.z, t, o.z)};
}

// SDF primitives, raytracer.glsl:496-528, 642-698
DEV float sdBox(v3 p, v3 b) {
  v3 d = vabs(p) - b;
  v3 m = mk(fmaxf(d.x, 0.f), fmaxf(d.y, 0.f), fmaxf(d.z, 0.f));
  return length(m) + fminf(fmaxf(d.x, fmaxf(d.y, d.z)), 0.0f);
}
DEV float sdCone(v3 p, v3 c) {
  float qx = fsqrt(p.x * p.x + p.z * p.z), qy = p.y;
  float d1 = -qy - c.z;
  float d2 = fmaxf(qx * c.x + qy * c.y, qy);
  float a = fmaxf(d1, 0.f), b = fmaxf(d2, 0.f);
  return fsqrt(a * a + b * b) + fminf(fmaxf(d1, d2), 0.f);
}
DEV float gmod(float x, float y) { return x - y * floorf(x * frcp(y)); }
DEV float menger(v3 p, v3 scale) {
  float d = sdBox(p, scale);
  float s = 1.0f;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    v3 ps = p * s;
    v3 a = mk(gmod(ps.x, 2.0f) - 1.0f, gmod(ps.y, 2.0f) - 1.0f, gmod(ps.z, 2.0f) - 1.0f);
    s *= 3.0f;
    v3 r = mk(fabsf(1.0f - 3.0f * fabsf(a.x)), fabsf(1.0f - 3.0f * fabsf(a.y)), fabsf(1.0f - 3.0f * fabsf(a.z)));
    float da = fmaxf(r.x, r.y), db = fmaxf(r.y, r.z), dc = fmaxf(r.z, r.x);
    float c = (fminf(da, fminf(db, dc)) - 1.0f) / s;
    d = fmaxf(c, d);
  }
  return d;
}
DEV float mandelbulb(v3 p) {
  v3 w = p;
  float m = dot(w, w);
  float dz = 1.0f;
  for (int i = 0; i < 3; ++i) {
    float m2 = m * m, m4 = m2 * m2;
    const float dzn = 8.0f * fsqrt(m4 * m2 * m) * dz + 1.0f;
    float x = w.x, x2 = x * x, x4 = x2 * x2;
    float y = w.y, y2 = y * y, y4 = y2 * y2;
    float z = w.z, z2 = z * z, z4 = z2 * z2;
    float k3 = x2 + z2;
    float k2 = frsq(k3 * k3 * k3 * k3 * k3 * k3 * k3);
    float k1 = x4 + y4 + z4 - 6.0f * y2 * z2 - 6.0f * x2 * y2 + 2.0f * z2 * x2;
    float k4 = x2 - y2 + z2;
    v3 wn;
    wn.x = p.x + 64.0f * x * y * z * (x2 - z2) * k4 * (x4 - 6.0f * x2 * z2 + z4) * k1 * k2;
    wn.y = p.y + -16.0f * y2 * k3 * k4 * k4 + k1 * k1;
    wn.z = p.z + -8.0f * y * k4 * (x4 * x4 - 28.0f * x4 * x2 * z2 + 70.0f * x4 * z4 - 28.0f * x2 * z2 * z4 + z4 * z4) * k1 * k2;
    const float mn = dot(wn, wn);
    dz = dzn;
    w = wn;
    m = mn;
    if (m > 4.0f) break;  // a branch: the select form took 124.8 vs 80.8 ms per C4 step
  }
  return fdiv(0.25f * flog(m) * fsqrt(m), dz);
}

// Index of the axis a unit plane normal lies on (n = +-e_axis), else -1.
DEV int axis_of(v3 n) {
  if (n.y == 0.f && n.z == 0.f && fabsf(n.x) == 1.f) return 0;
  if (n.x == 0.f && n.z == 0.f && fabsf(n.y) == 1.f) return 1;
  if (n.x == 0.f && n.y == 0.f && fabsf(n.z) == 1.f) return 2;
  return -1;
}


// --------------------------------------------------- triangles + BVH
// iTriangle (the reference's commented-out Moller-Trumbore, raytracer.glsl:
// 864-892) over the BVH of all TRIANGLE models (rt0_bvh_sah.cpp / rt0_bvh.hip).
// t must lie in (EPSILON, tmin) as there.  Deviation: the
// parallel-ray test compares the determinant a = d . (e1 x e0) with
// T.eps = EPSILON*|e0|*|e1| instead of the absolute EPSILON -- a scales with
// the triangle's area, and with the absolute threshold every triangle of the
// C5 model (edges ~0.015, |a| <= 1.9e-4) was rejected at every angle.
// |a| < eps rejects (a < eps with back-face culling, opts[3]).
DEV bool tri_test(const TriDev &T, v3 o, v3 d, float tmin, float &t) {
  const v3 e0 = mk(T.e0x, T.e0y, T.e0z), e1 = mk(T.e1x, T.e1y, T.e1z);
  const v3 h = mk(d.y * e1.z - d.z * e1.y, d.z * e1.x - d.x * e1.z, d.x * e1.y - d.y * e1.x);
  const float a = dot(e0, h);
  if (T.cull ? a < T.eps : (a > -T.eps && a < T.eps)) return false;
  const float f = 1.0f / a;
  const v3 s = o - mk(T.v0x, T.v0y, T.v0z);
  const float u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return false;
  const v3 q = mk(s.y * e0.z - s.z * e0.y, s.z * e0.x - s.x * e0.z, s.x * e0.y - s.y * e0.x);
  const float v = f * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  t = f * dot(e1, q);
  return t > EPSILON && t < tmin;
}
// slab test of a child box: entry distance, or +inf when the ray misses it or
// enters beyond tmin
DEV float box_enter(float x0, float y0, float z0, float x1, float y1, float z1, v3 o, v3 inv, float tmin) {
  const float tx0 = (x0 - o.x) * inv.x, tx1 = (x1 - o.x) * inv.x;
  const float ty0 = (y0 - o.y) * inv.y, ty1 = (y1 - o.y) * inv.y;
  const float tz0 = (z0 - o.z) * inv.z, tz1 = (z1 - o.z) * inv.z;
  const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
  return (tn <= tf && tn < tmin) ? tn : F_INF;
}
// The BVH's top levels in LDS (RT0_TREELET nodes of capacity; the
// scene-specialised modules of scenes with triangle models): the host numbers
// every node of the top levels breadth-first first (rt0_bvh_sah.cpp
// bvh_treelet_order: P.treelet of them, the rest in pre-order), every kernel
// that walks the tree copies them to LDS at its start (treelet_load), and a
// walk's first dependent node loads -- the same few nodes for every ray --
// are LDS reads instead of L2 round trips.  Same nodes, same order: the same
// hits bit for bit.
DEV float4 *treelet_lds() {
  __shared__ float4 t[4 * (RT0_TREELET > 0 ? RT0_TREELET : 1)];
  return t;
}
// (every thread of the block, before any leaves: one barrier)
DEV void treelet_load(const LaunchParams &P) {
#if RT0_TREELET > 0
  const int n = 4 * min(P.treelet, RT0_TREELET);
  float4 *t = treelet_lds();
  const float4 *__restrict__ g = reinterpret_cast<const float4 *>(P.bvh);
  for (int i = (int)threadIdx.x; i < n; i += (int)blockDim.x) t[i] = g[i];
  __syncthreads();
#else
  (void)P;
#endif
}
// node `node` of the tree: both child boxes (a, b, c) and the links (lk.x, lk.y)
DEV void bvh_fetch(const LaunchParams &P, const float4 *__restrict__ nodes, int node, float4 &a, float4 &b,
                   float4 &c, int4 &lk) {
#if RT0_TREELET > 0
  if (node < min(P.treelet, RT0_TREELET)) {  // (the host may order more levels than this module holds)
    const float4 *t = treelet_lds() + 4 * node;
    a = t[0];
    b = t[1];
    c = t[2];
    lk = reinterpret_cast<const int4 *>(t)[3];
    return;
  }
#endif
  a = nodes[4 * node];
  b = nodes[4 * node + 1];
  c = nodes[4 * node + 2];
  lk = reinterpret_cast<const int4 *>(nodes)[4 * node + 3];
}
// whether a ray (1/d = inv) enters neither child box of the BVH's root
// before tmax: then every walk of it ends at its first node with no triangle
// test (bvh_closest, walk_body), so it needs none
DEV bool bvh_root_miss(const LaunchParams &P, v3 o, v3 inv, float tmax) {
  const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(P.bvh);
  const float4 a = nodes[0], b = nodes[1], c = nodes[2];
  return box_enter(a.x, a.y, a.z, b.x, b.y, b.z, o, inv, tmax) == F_INF &&
         box_enter(a.w, b.w, c.x, c.y, c.z, c.w, o, inv, tmax) == F_INF;
}
// The per-lane traversal stacks: ONE LDS array for every traversal of the
// kernel (closest-hit and occlusion instances alike -- a __shared__ array
// declared inside the template would be one array per instance); stride =
// block size, so the 64 lanes of a wave hit 64 different banks.
// RT0_BVH_STACK16 (scene-specialised kernels whose every node index fits
// 16 + 64 / RT0_BVH_STACK bits, selected by the host): 16-bit LDS entries
// (the index's low half) and the high bits of every entry in one 64-bit
// register -- 2 B of LDS per entry instead of 4, so the stack no longer caps
// the waves per CU.  Pushed entries are inner nodes (>= 0).
struct BvhStack {
#if RT0_BVH_STACK16
  static constexpr int HB = 64 / RT0_BVH_STACK;
  static constexpr uint64_t HM = (1ull << HB) - 1ull;
  uint16_t *s;
  uint64_t hb = 0;
  DEV BvhStack() {
    __shared__ uint16_t stk_base[RT0_BVH_STACK * 256];
    s = stk_base + threadIdx.x;
  }
  DEV void put(int sp, int v) {
    s[256 * sp] = (uint16_t)v;
    hb = (hb & ~(HM << (HB * sp))) | ((uint64_t)((uint32_t)v >> 16) << (HB * sp));
  }
  DEV int get(int sp) const { return (int)((uint32_t)s[256 * sp] | ((uint32_t)((hb >> (HB * sp)) & HM) << 16)); }
#else
  int32_t *s;
  DEV BvhStack() {
    __shared__ int32_t stk_base[RT0_BVH_STACK * 256];
    s = stk_base + threadIdx.x;
  }
  DEV void put(int sp, int v) { s[256 * sp] = v; }
  DEV int get(int sp) const { return s[256 * sp]; }
#endif
};
// the record counter of this wave's deferred light-sampling region
DEV uint32_t *nee_wave_counter() {
  __shared__ uint32_t cnt[4];
  return cnt + (threadIdx.x >> 6);
}
// the wavefront shade kernel's append counters of this wave's region:
// k = 0 the round's march list, 1 its shadow list
DEV uint32_t *wf_wave_counter(int k) {
  __shared__ uint32_t cnt[8];
  return cnt + 4 * k + (threadIdx.x >> 6);
}
// append `n` entries for the active lanes of a (possibly divergent) call
// site: one LDS add by the first active lane; returns this lane's position
DEV uint32_t wave_append(uint32_t *ctr) {
  const unsigned long long act = __ballot(1);
  const int lane = (int)(threadIdx.x & 63u);
  const int leader = __ffsll((long long)act) - 1;
  const uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(act));
  return (uint32_t)__shfl((int)base, leader) + rank;
}
// closest triangle hit along (o, d) before tmin: depth-first, nearer child
// first, the far child on the per-lane LDS stack.  Returns the leaf-order
// triangle index or -1; tmin is updated.  ANY: stop at the first hit before
// tmin (an occlusion query: whether some triangle lies in (EPSILON, tmin)).
// Leaves hold one triangle and are tested in place, left before right; the
// first leaf test of every lane runs in one block whichever side it is on
// (8.36-8.39 vs 8.57-8.59 ms at 1024^2).
// budget (the wavefront ReSTIR shade kernel): stop after that many nodes,
// *complete = false if the walk had not finished.
template <bool ANY = false>
DEV int bvh_closest(const LaunchParams &P, v3 o, v3 d, v3 inv, float &tmin, unsigned long long *cnt = nullptr,
                    int budget = 0x7fffffff, bool *complete = nullptr) {
  BvhStack stk;
  int sp = 0, node = 0, best = -1;
  const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(P.bvh);
  const TriDev *__restrict__ tris = P.tris;
  // a ray visits each of the n-1 nodes at most once: the cap only guarantees
  // that every wave exits even on a corrupt tree
  for (int guard = 2 * P.n_tris + 8; guard > 0; --guard) {
    if (complete && budget-- <= 0) {
      *complete = false;
      break;
    }
    float4 a, b, c;
    int4 lk;
    bvh_fetch(P, nodes, node, a, b, c, lk);
    float tl = box_enter(a.x, a.y, a.z, b.x, b.y, b.z, o, inv, tmin);
    float tr = box_enter(a.w, b.w, c.x, c.y, c.z, c.w, o, inv, tmin);
    const int cl = lk.x, cr = lk.y;
    if (cnt) ++cnt[0];  // counting instance: nodes visited (two child boxes each)
    int l0 = -1, l1 = -1;
    if (tl != F_INF && cl < 0) {
      l0 = ~cl;
      tl = F_INF;
    }
    if (tr != F_INF && cr < 0) {
      if (l0 < 0) l0 = ~cr;
      else l1 = ~cr;
      tr = F_INF;
    }
    if (l0 >= 0) {
      float t;
      if (cnt) cnt[1] += 1 + (l1 >= 0);  // triangle tests
      if (tri_test(tris[l0], o, d, tmin, t)) {
        tmin = t;
        best = l0;
      }
      if (l1 >= 0 && tri_test(tris[l1], o, d, tmin, t)) {
        tmin = t;
        best = l1;
      }
      if (ANY && best >= 0) break;
    }
    if (tl != F_INF && tr != F_INF) {
      const bool lfirst = tl <= tr;
      stk.put(sp, lfirst ? cr : cl);
      sp = min(sp + 1, RT0_BVH_STACK - 1);  // the build guarantees depth < RT0_BVH_STACK
      node = lfirst ? cl : cr;
    } else if (tl != F_INF) {
      node = cl;
    } else if (tr != F_INF) {
      node = cr;
    } else {
      if (sp == 0) break;
      node = stk.get(--sp);
    }
  }
  return best;
}

// getAnimatedPosition(meshes[i].pos, i, u_time) (raytracer.glsl:263-298),
// precomputed per launch (LaunchParams::apos); only read under F_ANIM.
DEV v3 anim_pos(const LaunchParams &P, int i) {
  const float4 a = P.apos[i];
  return mk(a.x, a.y, a.z);
}

template <class Scene>
struct Geometry {
  // map(), raytracer.glsl:700-712 + the #sdf_meshes statements of index.html:702-717
  static DEV float map(const Scene &sc, v3 p, float &id, unsigned long long &nmap) {
    ++nmap;
    float rx = 0.f, ry = 0.f;
    const int ne = sc.n_meshes();
    for_sdfs(sc, [&](int i) {
      const GeomRec g = sc.geom(ne + i);
      v3 q = p - mk(g.px, g.py, g.pz);
      v3 j = mk(g.j0, g.j1, g.j2);
      float d;
      switch (sc.sdf_kind(ne + i)) {
        case 0: d = sdBox(q, j); break;
        case 1: {
          v3 dd = vabs(q) - j;
          d = length(mk(fmaxf(dd.x, 0.f), fmaxf(dd.y, 0.f), fmaxf(dd.z, 0.f))) - sc.j3(ne + i);
          break;
        }
        case 2: d = length(q) - g.j0; break;
        case 3: {
          v3 qa = vabs(q);
          d = fmaxf(qa.z - g.j1, fmaxf(qa.x * 0.866025f + q.y * 0.5f, -q.y) - g.j0 * 0.5f);
          break;
        }
        case 4: d = sdCone(q, j); break;
        case 5: d = menger(q, j); break;
        default: d = mandelbulb(q); break;
      }
      if (i == 0) {
        rx = d;
        ry = 0.f;
      } else {
        float a = (rx < d) ? 1.0f : 0.0f;
        rx = mixf(d, rx, a);
        ry = mixf((float)i, ry, a);
      }
    });
    id = ry;
    return rx;
  }
  // raytracer.glsl:714-722
  static DEV v3 calcNormal(const Scene &sc, v3 pos, unsigned long long &nmap) {
    float id;
    v3 a = mk(1.f, -1.f, -1.f) * map(sc, pos + mk(EPSILON, -EPSILON, -EPSILON), id, nmap);
    v3 b = mk(-1.f, -1.f, 1.f) * map(sc, pos + mk(-EPSILON, -EPSILON, EPSILON), id, nmap);
    v3 c = mk(-1.f, 1.f, -1.f) * map(sc, pos + mk(-EPSILON, EPSILON, -EPSILON), id, nmap);
    v3 d = mk(1.f, 1.f, 1.f) * map(sc, pos + mk(EPSILON, EPSILON, EPSILON), id, nmap);
    return normalize(((a + b) + c) + d);
  }

  // One candidate of intersection()'s mesh loop (raytracer.glsl:1009-1044):
  // mesh i's hit distance if it is valid and beats `bound` (the running tmin),
  // as iSphere (818-833, centre animated in RENDER_MODE 1, 819), iPlane
  // (812-815) or iBox (836-851) decide it; returns the mesh type, -1 = no hit.
  // Branch-free (v_cndmask selects): a lane never waits on another lane's
  // taken branch inside the mesh loop.  m = 1/d (iBox's, hoisted), mo = m*o.
  template <class Cfg>
  static DEV int prim(const LaunchParams &P, const Scene &sc, const Cfg &C, int i, v3 o, v3 d, v3 m, v3 mo,
                      float bound, float &t) {
    const GeomRec g = sc.geom(i);
    t = bound;
    if (g.j0 == 0.0f) return -1;  // raytracer.glsl:1009
    const v3 gp = mk(g.px, g.py, g.pz);
    if (g.type == T_SPHERE) {
      v3 oc = o - ((C.flags() & F_ANIM) ? anim_pos(P, i) : gp);
      float b = dot(oc, d);
      float c = dot(oc, oc) - g.d0;
      float disc = b * b - c;
      float sd = fsqrt(fmaxf(disc, 0.0f));
      float t0 = -b - sd, t1 = -b + sd;
      bool ok0 = (t0 > EPSILON && t0 < bound);
      bool ok1 = (t1 > EPSILON && t1 < bound);
      t = ok0 ? t0 : t1;
      return disc >= 0.0f && (ok0 || ok1) ? (int)T_SPHERE : -1;
    } else if (g.type == T_PLANE) {
      int ax = -1;
      if constexpr (Scene::kStatic) ax = axis_of(gp);  // folds: the normal is compile-time data
      if (ax >= 0) {
        // axis-aligned normal s*e_ax: dot(n, v) == s*v[ax] exactly for finite v,
        // and 1/(s*d[ax]) == s*m[ax] (v_rcp is sign-symmetric) -- same bits,
        // without the zero terms and a second reciprocal
        const float s = ax == 0 ? gp.x : (ax == 1 ? gp.y : gp.z);
        const float oa = ax == 0 ? o.x : (ax == 1 ? o.y : o.z);
        const float ma = ax == 0 ? m.x : (ax == 1 ? m.y : m.z);
        t = (g.d0 - s * oa) * (s * ma);
      } else {
        t = fdiv(g.d0 - dot(gp, o), dot(gp, d));
      }
      return (t > EPSILON && t < bound) ? (int)T_PLANE : -1;
    } else if (g.type == T_BOX) {
      // iBox's m*(centre - o) as m*centre - m*o: one FMA per axis (ulp-level,
      // like the other contracted geometry); the box normal (853-856) depends
      // only on the winner and its t, so intersect() evaluates it once after the loop
      v3 nv = mk(__builtin_fmaf(m.x, gp.x, -mo.x), __builtin_fmaf(m.y, gp.y, -mo.y), __builtin_fmaf(m.z, gp.z, -mo.z));
      v3 k = vabs(m) * g.d0;
      v3 t1 = nv - k, t2 = nv + k;
      float tN = fmaxf(fmaxf(t1.x, t1.y), t1.z);
      float tF = fminf(fminf(t2.x, t2.y), t2.z);
      t = (tN > 0.0f) ? tN : tF;
      return !(tN > tF || tF < 0.0f) && !(t < EPSILON || t >= bound) ? (int)T_BOX : -1;
    }
    return -1;
  }

  // intersection() as calcDirectLighting's shadow ray reads it (raytracer.glsl:
  // 1189-1196): only "is the closest hit a LIGHT, and which one" -- for
  // scene-specialised quadric scenes.  The closest hit of intersection() is the
  // lowest-index mesh of least valid t (strict < in index order), so it is a
  // light iff the closest light (tL, iL) beats every other mesh: non-light i
  // occludes iff t_i < tL, or t_i == tL and i < iL.  The light tests run
  // first; the occluder tests are then independent of one another (no running
  // tmin chain, no index/type bookkeeping).  A ray that hits nothing has
  // hit.index = 0 (HIT_MISS, 105): lit iff mesh 0 is a light.  Returns the
  // light's mesh or -1; tl = the closest hit's t.
  template <class Cfg>
  static DEV int shadow_light(const LaunchParams &P, const Scene &sc, const Cfg &C, v3 o, v3 d, float &tl,
                              unsigned long long *nbvh = nullptr) {
    const v3 m = mk(frcp(d.x), frcp(d.y), frcp(d.z));
    int il = shadow_light_q<Cfg>(P, sc, C, o, d, m, tl);
    if constexpr (Scene::kMayHaveModels) {
      // triangles come after the quadrics (strict <): one before tL is the
      // closest hit, and no model is a light -- an occlusion query suffices
      if (il >= 0 && sc.n_models() > 0 && P.n_tris > 0) {
        float tt = tl;
        if (bvh_closest<true>(P, o, d, m, tt, nbvh) >= 0) il = -1;
      }
    }
    return il;
  }
  // shadow_light's quadric part (m = 1/d): the light mesh the ray reaches
  // through the quadrics, or -1; tl = its t
  template <class Cfg>
  static DEV int shadow_light_q(const LaunchParams &P, const Scene &sc, const Cfg &C, v3 o, v3 d, v3 m, float &tl) {
    const v3 mo = m * o;
    float tL = INF_T;
    int iL = -1;
    for_meshes(sc, [&](int i) {
      if (sc.mat(i).type != M_LIGHT) return;
      float t;
      const bool ok = prim<Cfg>(P, sc, C, i, o, d, m, mo, tL, t) >= 0;
      tL = ok ? t : tL;
      iL = ok ? i : iL;
    });
    // the next float above tL: a bound that also admits t == tL
    const float tL_up = __int_as_float(__float_as_int(tL) + 1);
    bool occ = false;
    for_meshes(sc, [&](int i) {
      if (sc.mat(i).type == M_LIGHT) return;
      float t;
      occ |= prim<Cfg>(P, sc, C, i, o, d, m, mo, i < iL ? tL_up : tL, t) >= 0;
    });
    tl = tL;
    return occ ? -1 : (iL >= 0 ? iL : (sc.mat(0).type == M_LIGHT ? 0 : -1));
  }
  // isVisible() (raytracer.glsl:1539-1557) in the same spirit: the closest
  // quadric (t_q, i_q), then one occlusion query of the triangles up to
  // min(t_q, dist - 2*EPSILON): a triangle there is the closest hit and hides
  // `to`; otherwise the quadric decides (a light is transparent to the test).
  template <class Cfg>
  static DEV bool visible_fast(const LaunchParams &P, const Scene &sc, const Cfg &C, v3 o, v3 d, float lim,
                               unsigned long long *nbvh = nullptr) {
    const v3 m = mk(frcp(d.x), frcp(d.y), frcp(d.z));
    float tt;
    const bool vq = visible_q<Cfg>(P, sc, C, o, d, m, lim, tt);
    if constexpr (Scene::kMayHaveModels) {
      if (sc.n_models() > 0 && P.n_tris > 0) {
        if (bvh_closest<true>(P, o, d, m, tt, nbvh) >= 0) return false;
      }
    }
    return vq;
  }
  // visible_fast's quadric part: what the quadrics decide, and tt = the
  // bound of the triangle occlusion query, min(t_q, lim)
  template <class Cfg>
  static DEV bool visible_q(const LaunchParams &P, const Scene &sc, const Cfg &C, v3 o, v3 d, v3 m, float lim,
                            float &tt) {
    const v3 mo = m * o;
    float tq = INF_T;
    bool lq = sc.mat(0).type == M_LIGHT;  // the closest quadric is a light (mesh 0 on a miss)
    for_meshes(sc, [&](int i) {
      float t;
      const bool ok = prim<Cfg>(P, sc, C, i, o, d, m, mo, tq, t) >= 0;
      tq = ok ? t : tq;
      lq = ok ? sc.mat(i).type == M_LIGHT : lq;  // (a constant per mesh: no per-lane table read)
    });
    tt = fminf(tq, lim);
    if (tq < lim) return lq;
    return true;
  }

  // intersection(), raytracer.glsl:997-1082.  Returns tmin (INF_T = miss,
  // hit.index = 0 as HIT_MISS).  uv/texel parsing is omitted: only NULL_TEX
  // materials are accepted, so they never reach an output.
  // With a March slot (ms != null) the SDF march is not run here: the first
  // call records the ray in *ms and returns -1 (pending); once the kernel's
  // march loop has finished it (ms->done), the same call with the same ray
  // recomputes the quadric tests (deterministic) and completes the hit.
  template <bool SDF, class Cfg>
  // gt: the LDS copy of the geometry table (scene-specialised kernels; the
  // winner's normal reads it at a per-lane index), null otherwise
  static DEV float intersect(const LaunchParams &P, const Scene &sc, const Cfg &C, v3 o, v3 d, Hit &hit,
                             unsigned long long &nmap, March *ms = nullptr, unsigned long long *nbvh = nullptr,
                             const GeomRec *gt = nullptr) {
    auto geom_of = [&](int i) -> GeomRec {
      if constexpr (Scene::kStatic) return gt[i];
      else return sc.geom(i);
    };
    hit.n = mk(0.f, 0.f, 0.f);
    hit.index = 0;
    int type = -1;
    float tmin = INF_T;
    const v3 m = mk(frcp(d.x), frcp(d.y), frcp(d.z));  // iBox's 1/r.d, hoisted (837)
    // iBox's m*(centre - o) as m*centre - m*o: m*o once per ray, one FMA per
    // axis and box (ulp-level, like the other contracted geometry)
    const v3 mo = m * o;
    // Each candidate test is branch-free (v_cndmask selects): a lane never
    // waits on another lane's taken branch inside the mesh loop.  The box
    // normal of iBox (853-856) depends only on the winning box and its t, so
    // it is evaluated once after the loop for the winner.
    for_meshes(sc, [&](int i) {
      float t;
      const int ty = prim<Cfg>(P, sc, C, i, o, d, m, mo, tmin, t);
      const bool ok = ty >= 0;
      tmin = ok ? t : tmin;
      type = ok ? ty : type;
      hit.index = ok ? i : hit.index;
    });
    if constexpr (Scene::kMayHaveModels) {  // TRIANGLE models (after the quadrics, before the SDF march)
      if (sc.n_models() > 0 && P.n_tris > 0) {
        int ti;
        if (RT0_WAVEFRONT != 0 && !SDF && ms) {
          // wavefront ReSTIR rounds: the closest-hit walk kernel (wf_walk_body)
          // answers the ray -- the first call parks it with the quadrics' bound,
          // the same call after the walk recomputes the quadrics (deterministic)
          // and takes the walk's (t, triangle)
          if (!ms->done) {
            // the walk's first RT0_WF_INLINE_NODES nodes here: a ray that misses
            // the model's root boxes (most of them) or ends that soon is
            // answered in place; the others are walked again from the root
            float tb = tmin;
            bool complete = true;
            ti = bvh_closest(P, o, d, m, tb, nbvh, RT0_WF_INLINE_NODES, &complete);
            if (!complete) {
              *ms = March{o, d, tmin, 0.f, 0.f, 0, true, false, mk(0.f, 0.f, 0.f)};
              return -1.0f;
            }
            tmin = tb;
          } else {
            ms->done = false;
            ti = __float_as_int(ms->id);
            if (ti >= 0) tmin = ms->t;
          }
        } else {
          ti = bvh_closest(P, o, d, m, tmin, nbvh);
        }
        if (ti >= 0) {
          const TriDev T = P.tris[ti];
          const v3 e0 = mk(T.e0x, T.e0y, T.e0z), e1 = mk(T.e1x, T.e1y, T.e1z);
          hit.n = normalize(mk(e0.y * e1.z - e0.z * e1.y, e0.z * e1.x - e0.x * e1.z, e0.x * e1.y - e0.y * e1.x));
          hit.index = sc.n_meshes() + sc.n_sdfs() + T.model;
          type = T_TRIANGLE;
        }
      }
    }
    if (type == T_BOX) {  // iBox's normal for the winning box, 853-856
      const GeomRec g = geom_of(hit.index);
      v3 hp = (o + d * tmin) - mk(g.px, g.py, g.pz);
      v3 dd = vabs(hp) - mk(g.d0, g.d0, g.d0);
      v3 s = mk(sgn(hp.x), sgn(hp.y), sgn(hp.z));
      v3 st = mk(step_(dd.y, dd.x) * step_(dd.z, dd.x), step_(dd.z, dd.y) * step_(dd.x, dd.y),
                 step_(dd.x, dd.z) * step_(dd.y, dd.z));
      hit.n = normalize(s * st);
    }
    if constexpr (SDF) {
      if (sc.n_sdfs() > 0) {  // iSDF, 974-993
        float t = EPSILON * 4.0f;
        float id = 0.f;
        bool have_n = false;  // the wavefront march kernel's normal
        if (ms) {
          if (ms->active) return -1.0f;  // still being marched
          if (!ms->done) {
            *ms = March{o, d, tmin, t, id, 0, true, false, mk(0.f, 0.f, 0.f)};
            return -1.0f;
          }
          t = ms->t;
          id = ms->id;
          ms->done = false;
          have_n = RT0_WAVEFRONT != 0;
        } else {
          for (int i = 0; i < C.marching_steps(); ++i) {
            float dist = map(sc, ray_at(o, d, t), id, nmap);
            float h = fabsf(dist);
            if (h < EPSILON || t > tmin) break;
            t = __builtin_fmaf(h, C.fudge(), t);  // (written out: every march kernel rounds it alike)
          }
        }
        if (!(t > tmin)) {
          hit.n = have_n ? ms->n : calcNormal(sc, ray_at(o, d, t), nmap);
          hit.index = sc.n_meshes() + (int)id;
          tmin = t;
          type = T_SDF;
        }
      }
    }
    hit.type = type;
    if (type >= 0) {
      hit.pos = d * tmin + o;
      if (type == T_SPHERE) {  // 1060
        const GeomRec g = geom_of(hit.index);
        hit.n = normalize(hit.pos - ((C.flags() & F_ANIM) ? anim_pos(P, hit.index) : mk(g.px, g.py, g.pz)));
      } else if (type == T_PLANE) {
        const GeomRec g = geom_of(hit.index);
        hit.n = normalize(mk(g.px, g.py, g.pz));
      }
    } else {
      hit.pos = mk(0.f, 0.f, 0.f);
    }
    return tmin;
  }
};

// ------------------------------------------------------------ sampling
// raytracer.glsl:1092-1107
DEV void calc_binormals(v3 n, v3 &ox, v3 &oz) {
  float sig = n.z < 0.0f ? -1.0f : 1.0f;
  if (fabsf(n.z) > 0.99999f) {
    ox = mk(1.f, 0.f, 0.f);
    oz = mk(0.f, sig, 0.f);
    return;
  }
  float a = frcp(sig - n.z);
  float b = n.x * n.y * a;
  ox = mk(1.0f + sig * n.x * n.x * a, sig * b, -sig * n.x);
  oz = mk(b, sig + n.y * n.y * a, -n.y);
}
DEV v3 frame_dir(v3 w, v3 u, v3 v, float rx, float ry) {  // rx: the angle in revolutions
  float om = fsqrt(1.0f - ry * ry);
  return normalize((u * (fcos_rev(rx) * om) + v * (fsin_rev(rx) * om)) + w * ry);
}
// getSampleBiased(w, 1.0, seed), 1109-1120: pow(r.y, 1/2) == sqrt(r.y)
DEV v3 sample_cosine(v3 w, float seed) {
  v3 u, v;
  calc_binormals(w, u, v);
  float rx, ry;
  hash2(seed, seed, rx, ry);
  return frame_dir(w, u, v, rx, fsqrt(ry));
}
// getConeSample, 1122-1133
DEV v3 sample_cone(v3 w, float extent, float seed) {
  v3 u, v;
  calc_binormals(w, u, v);
  float rx, ry;
  hash2(seed, seed, rx, ry);
  return frame_dir(w, u, v, rx, 1.0f - ry * extent);
}
// randomSphereDirection, 1143-1147
DEV v3 random_sphere_dir(float seed) {
  float rx, ry;
  hash2(seed, seed, rx, ry);
  float sy = fsin_rev(ry), cy = fcos_rev(ry), sx = fsin_rev(rx);  // angles 2*pi*r
  return mk(sx * sy, sx * cy, fcos_rev(rx));
}
// sampleHG, 1157-1171
DEV v3 sample_hg(v3 w, float seed) {
  float ux, uy;
  hash2(seed, seed + 1.789f, ux, uy);
  constexpr float g = VOL_G;
  float sqr = (1.0f - g * g) / (1.0f - g + 2.0f * g * ux);
  float cos_theta = (1.0f + g * g - sqr * sqr) / (2.0f * g);
  float sin_theta = fsqrt(fmaxf(0.0f, 1.0f - cos_theta * cos_theta));
  v3 t, b;  // phi = 2*pi*uy
  calc_binormals(w, t, b);
  return normalize((t * (fcos_rev(uy) * sin_theta) + b * (fsin_rev(uy) * sin_theta)) + w * cos_theta);
}

// powerHeuristic / cosineHemispherePdf / lightSamplingPdf, 1233-1262
DEV float power_heuristic(float f, float g) {
  float denom = f * f + g * g;
  return fmaxf(0.0f, fdiv(f * f, denom));  // maxNum: 0/0 -> 0 (documented deviation)
}
DEV float cos_pdf(v3 wi, v3 n) { return fmaxf(0.0f, dot(wi, n)) * ONE_OVER_PI; }
DEV float light_pdf(const GeomRec &g, const MatRec &mt, v3 x) {
  if (mt.type != M_LIGHT) return 0.0f;
  if (g.type == T_SPHERE) {
    v3 d = mk(g.px, g.py, g.pz) - x;
    float d2 = dot(d, d);
    float r2 = g.d0;
    if (d2 <= r2) return 0.0f;
    float ctm = fsqrt(fmaxf(0.0f, 1.0f - fdiv(r2, d2)));
    float denom = 1.0f - ctm;
    if (denom < 1e-6f) return 0.0f;
    return frcp(TWO_PI * denom);
  }
  return 1.0f / FOUR_PI;
}

DEV float spectral_ior(float lambda, float A) {
  float lu = lambda * 0.001f;
  return A + fdiv(0.04f, lu * lu);
}
DEV float pow5(float x) {
  float a = fabsf(x), a2 = a * a;
  return a2 * a2 * a;
}
DEV float schlick(v3 rd, v3 n, float nc, float nt) {
  float q = fdiv(nc - nt, nc + nt);
  float R0 = q * q;
  return R0 + (1.0f - R0) * pow5(1.0f + dot(n, rd));
}
DEV float fresnel(v3 rd, v3 n, float nc, float nt, v3 refr) {
  float cosI = dot(rd, n), cosT = dot(n, refr);
  float rs = fdiv(nc * cosI - nt * cosT, nc * cosI + nt * cosT);
  float rp = fdiv(nc * cosT - nt * cosI, nc * cosT + nt * cosI);
  return (rs * rs + rp * rp) * 0.5f;
}

// CIE fit, raytracer.glsl:324-353
DEV v3 wavelength_to_rgb(float l) {
  float t1 = (l - 442.0f) * (l < 442.0f ? 0.0624f : 0.0374f);
  float t2 = (l - 599.8f) * (l < 599.8f ? 0.0264f : 0.0323f);
  float t3 = (l - 501.1f) * (l < 501.1f ? 0.0490f : 0.0382f);
  float X = 0.362f * fexp(-0.5f * t1 * t1) + 1.056f * fexp(-0.5f * t2 * t2) - 0.065f * fexp(-0.5f * t3 * t3);
  float y1 = (l - 568.8f) * (l < 568.8f ? 0.0213f : 0.0247f);
  float y2 = (l - 530.9f) * (l < 530.9f ? 0.0613f : 0.0322f);
  float Y = 0.821f * fexp(-0.5f * y1 * y1) + 0.286f * fexp(-0.5f * y2 * y2);
  float z1 = (l - 437.0f) * (l < 437.0f ? 0.0845f : 0.0278f);
  float z2 = (l - 459.0f) * (l < 459.0f ? 0.0385f : 0.0725f);
  float Z = 1.217f * fexp(-0.5f * z1 * z1) + 0.681f * fexp(-0.5f * z2 * z2);
  v3 rgb = mk(3.2404542f * X - 1.5371385f * Y - 0.4985314f * Z, -0.9692660f * X + 1.8760108f * Y + 0.0415560f * Z,
              0.0556434f * X - 0.2040259f * Y + 1.0572252f * Z);
  return mk(fmaxf(0.0f, rgb.x) / 0.378f, fmaxf(0.0f, rgb.y) / 0.298f, fmaxf(0.0f, rgb.z) / 0.285f);
}


// --------------------------------------------------------------- textures
// raytracer.glsl:363-433 (noise), 726-772 (getTexel), 1049-1078 (uv parser).
// The texel is evaluated lazily -- only where the reference reads
// hit.texel (shading 2071/2077, light hits in calcDirectLighting 1203/1215) --
// which is the same value: it depends only on the hit's mesh, position,
// normal and uv.
struct T4 {
  float r, g, b, a;
};
DEV T4 t4s(float x) { return T4{x, x, x, x}; }
// GLSL mod(x, y) = x - y*floor(x/y) (correctly rounded division)
DEV float glsl_mod(float x, float y) { return x - y * floorf(x / y); }
DEV float smoothstep_(float e0, float e1, float x) {
  float t = fminf(fmaxf((x - e0) / (e1 - e0), 0.0f), 1.0f);
  return t * t * (3.0f - 2.0f * t);
}
// GL_LINEAR + GL_REPEAT fetch at level 0 of an RGBA8 asset texture
// (GlslViewport.loadTexture, index.js:703-708); unbound unit = (0,0,0,1).
// F_TEX_FIXED (rt0_set_texture_filter, the default): SwiftShader 4.1's
// fixed-point GL_LINEAR + GL_REPEAT fetch -- GLSL leaves the filter's
// precision to the implementation, and GPU texture units filter in fixed
// point too -- measured by the known-answer shaders of
// oracle/gen/tex_kat.py (tests/golden/tex_filter_kat.npz; restated as
// tex_fetch_ss in oracle/rt0_oracle.c): the coordinate as a 16-bit fraction
// (trunc(u * 65536) & 0xFFFF), the half texel taken off in that unit
// (32768 / w), times w a 16.16 texel position (texel s >> 16, weight
// s & 0xFFFF); texels widened to v * 257, tap weights (wx * wy) >> 16, taps
// (t * w) >> 16 summed, read back times 1 / 65535.
DEV int ss_coord(float u, int w, int &i0, int &i1) {
  const float x = u * 65536.0f;
  const int q = fabsf(x) < 2147483520.0f ? (int)x : (int)0x80000000;  // (cvttps2dq: out of range -> INT_MIN)
  const int s = ((q & 0xFFFF) - 32768 / w) * w;
  int i = (s >> 16) % w;  // (arithmetic shift: floor)
  i += i < 0 ? w : 0;
  i0 = i;
  i1 = i + 1 == w ? 0 : i + 1;
  return s & 0xFFFF;
}
DEV T4 tex_rgba8_ss(const uint32_t *__restrict__ img, int w, int h, float u, float v) {
  int x0, x1, y0, y1;
  const uint32_t fu = (uint32_t)ss_coord(u, w, x0, x1), fv = (uint32_t)ss_coord(v, h, y0, y1);
  const uint32_t w00 = ((65535u - fu) * (65535u - fv)) >> 16, w10 = (fu * (65535u - fv)) >> 16;
  const uint32_t w01 = ((65535u - fu) * fv) >> 16, w11 = (fu * fv) >> 16;
  const uint32_t q00 = img[y0 * w + x0], q10 = img[y0 * w + x1], q01 = img[y1 * w + x0], q11 = img[y1 * w + x1];
  float r[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    auto t = [&](uint32_t q) { return ((q >> (8 * c)) & 255u) * 257u; };
    const uint32_t n = ((t(q00) * w00) >> 16) + ((t(q10) * w10) >> 16) + ((t(q01) * w01) >> 16) + ((t(q11) * w11) >> 16);
    r[c] = (float)n * (1.0f / 65535.0f);
  }
  return T4{r[0], r[1], r[2], r[3]};
}
DEV T4 tex_rgba8(const LaunchParams &P, int unit, float u, float v) {
  const uint32_t *__restrict__ img = P.tex_img[unit];
  if (img == nullptr) return T4{0.f, 0.f, 0.f, 1.f};
  const int w = P.tex_w[unit], h = P.tex_h[unit];
  if (P.flags & F_TEX_FIXED) return tex_rgba8_ss(img, w, h, u, v);
  const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
  const float fx = floorf(x), fy = floorf(y);
  const float a = x - fx, b = y - fy;
  int x0 = (int)fx % w, y0 = (int)fy % h;
  x0 += x0 < 0 ? w : 0;
  y0 += y0 < 0 ? h : 0;
  const int x1 = x0 + 1 == w ? 0 : x0 + 1, y1 = y0 + 1 == h ? 0 : y0 + 1;
  const uint32_t q00 = img[y0 * w + x0], q10 = img[y0 * w + x1], q01 = img[y1 * w + x0], q11 = img[y1 * w + x1];
  float r[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float t00 = (float)((q00 >> (8 * c)) & 255u), t10 = (float)((q10 >> (8 * c)) & 255u);
    const float t01 = (float)((q01 >> (8 * c)) & 255u), t11 = (float)((q11 >> (8 * c)) & 255u);
    const float top = t00 + a * (t10 - t00), bot = t01 + a * (t11 - t01);
    r[c] = (top + b * (bot - top)) / 255.0f;  // unorm8, correctly rounded like the restatement
  }
  return T4{r[0], r[1], r[2], r[3]};
}
// value_noise, 393-401 (the .yx swizzle: mix(G, R, f.z))
DEV float value_noise(const LaunchParams &P, v3 x) {
  const v3 p = mk(floorf(x.x), floorf(x.y), floorf(x.z));
  v3 f = x - p;
  f = mk(f.x * f.x * (3.0f - 2.0f * f.x), f.y * f.y * (3.0f - 2.0f * f.y), f.z * f.z * (3.0f - 2.0f * f.z));
  const float ux = (p.x + 37.0f * p.z) + f.x, uy = (p.y + 17.0f * p.z) + f.y;
  const T4 t = tex_rgba8(P, 4, (ux + 0.5f) * (1.0f / 256.0f), (uy + 0.5f) * (1.0f / 256.0f));
  return mixf(t.g, t.r, f.z);
}
// voronoi, 404-431
DEV v3 voronoi(const LaunchParams &P, v3 x) {
  const v3 p = mk(floorf(x.x), floorf(x.y), floorf(x.z));
  const v3 f = x - p;
  float id = 0.0f, r0 = 100.0f, r1 = 100.0f;
  for (int k = -1; k <= 1; ++k)
    for (int j = -1; j <= 1; ++j)
      for (int i = -1; i <= 1; ++i) {
        const v3 b = mk((float)i, (float)j, (float)k);
        const v3 hx = p + b;
        const T4 t = tex_rgba8(P, 4, ((hx.x + 3.0f * hx.z) + 0.5f) * (1.0f / 256.0f),
                               ((hx.y + 1.0f * hx.z) + 0.5f) * (1.0f / 256.0f));
        const v3 r = (b - f) + mk(t.r, t.g, t.b);
        const float d = dot(r, r);
        if (d < r0) {
          id = dot(p + b, mk(1.0f, 57.0f, 113.0f));
          r1 = r0;
          r0 = d;
        } else if (d < r1) {
          r1 = d;
        }
      }
  return mk(sqrtf(r0), sqrtf(r1), fabsf(id));
}
// gradient_hash / gradient_noise, 363-387 (sin of large arguments times
// 43758.5: executor-dependent in the last bits; no reference material uses it)
DEV v3 gradient_hash(v3 p) {
  const v3 q = mk(dot(p, mk(127.1f, 311.7f, 74.7f)), dot(p, mk(269.5f, 183.3f, 246.1f)),
                  dot(p, mk(113.5f, 271.9f, 124.6f)));
  const float sx = sinf(q.x) * 43758.5453f, sy = sinf(q.y) * 43758.5453f, sz = sinf(q.z) * 43758.5453f;
  return mk(-1.0f + 2.0f * (sx - floorf(sx)), -1.0f + 2.0f * (sy - floorf(sy)), -1.0f + 2.0f * (sz - floorf(sz)));
}
DEV float gradient_noise(v3 p) {
  const v3 i = mk(floorf(p.x), floorf(p.y), floorf(p.z));
  const v3 f = p - i;
  const v3 u = mk(f.x * f.x * (3.0f - 2.0f * f.x), f.y * f.y * (3.0f - 2.0f * f.y), f.z * f.z * (3.0f - 2.0f * f.z));
  float c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const v3 o = mk((float)(k & 1), (float)((k >> 1) & 1), (float)(k >> 2));
    c[k] = dot(gradient_hash(i + o), f - o);
  }
  const float x00 = mixf(c[0], c[1], u.x), x10 = mixf(c[2], c[3], u.x);
  const float x01 = mixf(c[4], c[5], u.x), x11 = mixf(c[6], c[7], u.x);
  return mixf(mixf(x00, x10, u.y), mixf(x01, x11, u.y), u.z);
}
// getTexel, 726-772
DEV T4 get_texel(const LaunchParams &P, const TexRec &t, v3 pos, float u, float v) {
  if (t.type >= 0 && t.type <= 3) return tex_rgba8(P, t.type, u, v);
  if (t.type == 7) return t4s(glsl_mod(floorf(t.p0 * u) + floorf(t.p1 * v), t.p2));  // CHECK
  if (t.type == 8) {                                                                 // RIPPLE
    const float du = u - t.p0, dv = v - t.p1;
    return t4s(glsl_mod(ceilf(sqrtf(du * du + dv * dv) * t.p2), t.p3));
  }
  const v3 sp = mk(t.p0, t.p1, t.p2) * pos;
  if (t.type == 4) {  // VORONOI
    const v3 r = voronoi(P, sp);
    return T4{r.x, r.y, r.z, 0.0f};
  }
  if (t.type == 5) return t4s(smoothstep_(-0.7f, 0.7f, gradient_noise(sp)));  // GRADIENT_NOISE
  if (t.type == 6) return t4s(value_noise(P, sp));                             // VALUE_NOISE
  if (t.type == 9) {                                                           // METAL
    const v3 m = mk(-1.2f, 1.99f, -1.6f);
    v3 q = sp;
    float f = 0.5f * value_noise(P, q);
    q = (m * q) * 2.01f;
    f += 0.25f * value_noise(P, q);
    q = (m * q) * 2.02f;
    f += 0.125f * value_noise(P, q);
    return t4s(f);
  }
  return t4s(0.0f);
}
// texture(u_cubemap, d) (raytracer.glsl:1895, 2060): GL ES 3.0 cube face
// selection (major axis, table 3.21) and GL_LINEAR with seamless filtering
// (always on in ES 3.0): a footprint texel beyond the face edge is fetched
// from the adjacent face (its centre mapped back to a direction and
// re-projected) -- what the reference executor does.  Faces in
// GL order +X -X +Y -Y +Z -Z; unbound = (0,0,0,1).
DEV int cube_face(v3 d, float &s, float &t) {
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  int face;
  float sc, tc, ma;
  if (ax >= ay && ax >= az) {
    face = d.x >= 0.f ? 0 : 1;
    sc = d.x >= 0.f ? -d.z : d.z;
    tc = -d.y;
    ma = ax;
  } else if (ay >= az) {
    face = d.y >= 0.f ? 2 : 3;
    sc = d.x;
    tc = d.y >= 0.f ? d.z : -d.z;
    ma = ay;
  } else {
    face = d.z >= 0.f ? 4 : 5;
    sc = d.z >= 0.f ? d.x : -d.x;
    tc = -d.y;
    ma = az;
  }
  s = 0.5f * (sc / ma + 1.0f);
  t = 0.5f * (tc / ma + 1.0f);
  return face;
}
DEV uint32_t cube_texel(const LaunchParams &P, int face, int i, int j) {
  const int n = P.cube_size;
  if (i < 0 || i >= n || j < 0 || j >= n) {  // seamless: the neighbouring face's texel
    const float scn = 2.0f * ((float)i + 0.5f) / (float)n - 1.0f, tcn = 2.0f * ((float)j + 0.5f) / (float)n - 1.0f;
    v3 d;
    switch (face) {  // the face table inverted (major-axis component 1)
      case 0: d = mk(1.f, -tcn, -scn); break;
      case 1: d = mk(-1.f, -tcn, scn); break;
      case 2: d = mk(scn, 1.f, tcn); break;
      case 3: d = mk(scn, -1.f, -tcn); break;
      case 4: d = mk(scn, -tcn, 1.f); break;
      default: d = mk(-scn, -tcn, -1.f); break;
    }
    float s, t;
    face = cube_face(d, s, t);
    i = min(max((int)floorf(s * (float)n), 0), n - 1);
    j = min(max((int)floorf(t * (float)n), 0), n - 1);
  }
  return P.cube[((size_t)face * n + j) * n + i];
}
DEV T4 cube_sample(const LaunchParams &P, v3 d) {
  if (P.cube == nullptr) return T4{0.f, 0.f, 0.f, 1.f};
  float s, t;
  const int face = cube_face(d, s, t), n = P.cube_size;
  const float x = s * (float)n - 0.5f, y = t * (float)n - 0.5f;
  const float fx = floorf(x), fy = floorf(y);
  const float a = x - fx, b = y - fy;
  const int x0 = (int)fx, y0 = (int)fy;
  uint32_t q00, q10, q01, q11;
  // a footprint over a cube corner: the texel beyond both edges belongs to no
  // face; like the reference executor (the cubemap KAT) it is the
  // average of the three texels that meet there (bit 0..3: which tap)
  int corner = -1;
  if (x0 >= 0 && y0 >= 0 && x0 + 1 < n && y0 + 1 < n) {  // footprint inside the face (the common case)
    const uint32_t *__restrict__ img = P.cube + ((size_t)face * n + y0) * n + x0;
    q00 = img[0];
    q10 = img[1];
    q01 = img[n];
    q11 = img[n + 1];
  } else {
    q00 = cube_texel(P, face, x0, y0);
    q10 = cube_texel(P, face, x0 + 1, y0);
    q01 = cube_texel(P, face, x0, y0 + 1);
    q11 = cube_texel(P, face, x0 + 1, y0 + 1);
    const bool ox0 = x0 < 0 || x0 >= n, ox1 = x0 + 1 < 0 || x0 + 1 >= n;
    const bool oy0 = y0 < 0 || y0 >= n, oy1 = y0 + 1 < 0 || y0 + 1 >= n;
    corner = ox0 && oy0 ? 0 : ox1 && oy0 ? 1 : ox0 && oy1 ? 2 : ox1 && oy1 ? 3 : -1;
  }
  float r[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float t00 = (float)((q00 >> (8 * c)) & 255u), t10 = (float)((q10 >> (8 * c)) & 255u);
    float t01 = (float)((q01 >> (8 * c)) & 255u), t11 = (float)((q11 >> (8 * c)) & 255u);
    if (corner == 0) t00 = (t10 + t01 + t11) / 3.0f;
    else if (corner == 1) t10 = (t00 + t11 + t01) / 3.0f;
    else if (corner == 2) t01 = (t11 + t00 + t10) / 3.0f;
    else if (corner == 3) t11 = (t01 + t10 + t00) / 3.0f;
    const float top = t00 + a * (t10 - t00), bot = t01 + a * (t11 - t01);
    r[c] = (top + b * (bot - top)) / 255.0f;
  }
  return T4{r[0], r[1], r[2], 1.0f};
}
// hit.uv (1051-1076) + getTexel for a hit on a textured mesh (type >= 0)
DEV T4 hit_texel(const LaunchParams &P, const TexRec &t, const Hit &h) {
  float u = -1.0f, v = -1.0f;
  if (h.type == T_SPHERE) {  // cartesianToSpherical of the WORLD position (467-471)
    const float rho = sqrtf(dot(h.pos, h.pos));
    u = asinf(h.pos.y / rho) / PI_F;
    v = atan2f(h.pos.z, h.pos.x) / TWO_PI;
  }
  if (u < 0.0f) {
    const v3 a = vabs(h.n);
    if (a.x > a.y && a.x > a.z) {
      u = -h.pos.z;
      v = -h.pos.y;
    } else if (a.y > a.x && a.y > a.z) {
      u = h.pos.x;
      v = h.pos.z;
    } else {
      u = h.pos.x;
      v = -h.pos.y;
    }
  }
  return get_texel(P, t, h.pos, u, v);
}

// ---------------------------------------------------------------- ReSTIR
// raytracer.glsl:1264-1802.
struct Res {
  v3 pos, col;
  float ws, M, W, age;
  int idx;
};
DEV Res empty_res() { return Res{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), 0.f, 0.f, 0.f, 0.f, -1}; }
DEV bool finite_(float x) { return __builtin_isfinite(x); }
// packReservoirAux alpha, 1425-1430 (unfused, as the next pass decodes it with fract)
DEV float pack_alpha(float age, float M, int idx, int nlights) {
#pragma clang fp contract(off)
  float na = fminf(fmaxf(age / 30.0f, 0.0f), 1.0f);
  float nM = fminf(fmaxf(M / 100.0f, 0.0f), 1.0f);
  float nli = (float)(idx + 1) / (float)(nlights > 1 ? nlights : 1);
  return ((na * 0.33f) + (nM * 0.33f)) + (nli * 0.34f);
}
// unpackReservoirEnhanced alpha decode, 1448-1457 (unfused)
DEV void unpack_alpha(float pa, int nlights, float &age, float &M, int &idx) {
#pragma clang fp contract(off)
  float nli = (pa * 2.94f);
  nli = nli - floorf(nli);
  float temp = pa - (nli * 0.34f);
  float nM = (temp * 3.03f);
  nM = nM - floorf(nM);
  float nage = (temp - (nM * 0.33f)) * 3.03f;
  age = nage * 30.0f;
  M = nM * 100.0f;
  int len1 = nlights > 1 ? nlights : 1;
  idx = (int)(nli * (float)len1) - 1;
}

// LDS copies of a scene-specialised kernel's geometry and material tables,
// written by the workgroup's first threads before one barrier, for the
// lookups at a per-lane index (the hit mesh's material each bounce, a
// light-sampling record's material, the light a shadow ray reached): the
// constant tables are read with a dependent per-lane global load there.
// Loops over the meshes keep reading the constant tables (compile-time
// indices fold to immediates).  All null for the ahead-of-time kernels.
struct SceneTables {
  const GeomRec *g;
  const MatRec *m, *ms;
};
template <class Scene>
DEV SceneTables scene_tables(const Scene &sc) {
  if constexpr (Scene::kStatic) {
    constexpr int n = Scene::kMeshes + Scene::kSdfs + Scene::kModels;
    __shared__ GeomRec g[n > 0 ? n : 1];
    __shared__ MatRec m[n > 0 ? n : 1], ms[n > 0 ? n : 1];
    for (int k = (int)threadIdx.x; k < n; k += (int)blockDim.x) {
      g[k] = sc.geom(k);
      m[k] = sc.mat(k);
      ms[k] = sc.mat_shade(k);
    }
    __syncthreads();
    return SceneTables{g, m, ms};
  }
  (void)sc;
  return SceneTables{nullptr, nullptr, nullptr};
}

// ----------------------------------------------------------- integrator
template <class Scene, class Cfg, bool RESTIR, bool VOL, bool SDF, bool SPECTRAL, bool COUNT>
struct Integrator {
  using G = Geometry<Scene>;
  const LaunchParams &P;
  Scene sc;
  Cfg C;
  float fcx, fcy;  // gl_FragCoord
  float stx, sty;  // 2 * gl_FragCoord / resolution - 1 (set_pixel)
  uint32_t frame;
  float hero;
  int diff_b, spec_b, scat_ev;
  unsigned long long n_isect, n_iter, n_nee, n_map;
  // counting instance only: ReSTIR calls / candidates / temporal taps /
  // spatial taps, BVH nodes / triangle tests (rt0_read_counters_n [5..10])
  unsigned long long n_restir = 0, n_cand = 0, n_ttap = 0, n_stap = 0, n_bvh[2] = {0, 0};
  Res fin;  // g_final_reservoir (raytracer.glsl:1616)
  // deferred light sampling (P.defer): this sample's image pixel and the
  // number of sampleLightsReSTIR calls it has deferred so far
  int32_t nee_pix = 0, nee_k = 0;
  uint32_t nee_wave = 0;  // the pass grid's wave index: the region defer_nee appends to
  // F_EXEC_GHOST: brdf()'s parameter registers as the lane's last live call
  // left them (see ghost_brdf)
  v3 gr_x, gr_nl, gr_rd;
  float gr_bounce;
  int gr_mat;
  bool gr_have, gr_spec;
  // F_EXEC_GHOST + P.quad_mode (rule 11, light_q): this sample's pixel, the
  // bounces at which its path ran brdf()'s light loop / a ghost call's, and
  // its quad's first lane's (q0_on: this lane reads them)
  int q_px = 0, q_py = 0;
  uint32_t q_own = 0, q_gown = 0, q0_m = 0, q0_g = 0;
  bool q0_on = false;
  // the light-sampling kernel's LDS copy of the ReSTIR candidates' light data
  // (candidate_table), or null: read from the scene tables
  const float4 *cand_lds = nullptr;
  // LDS copies of the scene tables for lookups at a per-lane index (the hit
  // mesh, a record's material, the lit light; scene_tables): every
  // scene-specialised Integrator gets them (pass_body, nee_body)
  const GeomRec *g_lds = nullptr;
  const MatRec *m_lds = nullptr, *ms_lds = nullptr;
  // wavefront shade kernel (WF): this sample's path slot and region, and the
  // light-sampling calls this bounce handed to the march kernel (one bit per
  // light slot; wf_kind 1 = brdf()'s surface loop, 2 = the in-scatter loop)
  uint32_t wf_slot = 0, wf_region = 0, wf_bits = 0;
  int wf_kind = 0;
  DEV GeomRec geom_at(int i) const {
    if constexpr (Scene::kStatic) return g_lds[i];
    else return sc.geom(i);
  }
  DEV MatRec mat_at(int i) const {
    if constexpr (Scene::kStatic) return m_lds[i];
    else return sc.mat(i);
  }
  // light_index[k] at a per-lane k: from the candidate table when the kernel has one
  DEV int light_at(int k) const { return cand_lds ? __float_as_int(cand_lds[2 * k + 1].z) : sc.light(k); }
  DEV MatRec mat_shade_at(int i) const {
    if constexpr (Scene::kStatic) return ms_lds[i];
    else return sc.mat_shade(i);
  }
  template <class T>
  DEV void use_tables(const T &t) {
    g_lds = t.g;
    m_lds = t.m;
    ms_lds = t.ms;
  }

  DEV Integrator(const LaunchParams &p, Scene s, Cfg c)
      : P(p), sc(s), C(c), n_isect(0), n_iter(0), n_nee(0), n_map(0) {}

  DEV bool flag(uint32_t f) const { return (C.flags() & f) != 0; }
  // Shadow rays of sphere lights through G::shadow_light: scene-specialised
  // scenes of quadrics only (no SDF march, no triangle models, no textured
  // light colour to evaluate at the hit).
  DEV bool fast_shadow() const {
    if constexpr (Scene::kStatic) return Scene::kSdfs == 0 && !Scene::any_tex();
    else return sc.n_sdfs() == 0 && !sc.any_tex();
  }
  // material of a shadow ray's light: folds to the one light mesh of a
  // single-light scene, a per-lane record otherwise
  DEV MatRec light_mat(int il) const {
    int n = 0, only = 0;
    if constexpr (Scene::kStatic)
      static_for<0, Scene::kMeshes>([&](int i) {
        if (sc.mat(i).type == M_LIGHT) {
          ++n;
          only = i;
        }
      });
    return n == 1 ? sc.mat(only) : mat_at(il);
  }
  // a light/sphere position as the reference reads it where it calls
  // getAnimatedPosition (RENDER_MODE 1); the static position otherwise
  DEV v3 lpos(int i, const GeomRec &g) const { return flag(F_ANIM) ? anim_pos(P, i) : mk(g.px, g.py, g.pz); }

  DEV float isect(v3 o, v3 d, Hit &h, March *ms = nullptr) {
    if (COUNT) ++n_isect;
    return G::template intersect<SDF>(P, sc, C, o, d, h, n_map, ms, COUNT ? n_bvh : nullptr, g_lds);
  }

  // mix(mesh.mat.c, hit.texel.rgb, hit.texel.a) of a shadow ray's light hit
  // (raytracer.glsl:1203, 1215); hit.texel is HIT_MISS's zero on a miss
  DEV v3 light_color(const Hit &h, const MatRec &m) {
    v3 c = mk(m.cr, m.cg, m.cb);
    if (sc.any_tex() && h.type >= 0) {
      const TexRec tr = sc.tex(h.index);
      if (tr.type >= 0) {
        const T4 tx = hit_texel(P, tr, h);
        c = mk(mixf(c.x, tx.r, tx.a), mixf(c.y, tx.g, tx.a), mixf(c.z, tx.b, tx.a));
      }
    }
    return c;
  }

  // calcDirectLighting, raytracer.glsl:1174-1230
  // ms/susp: resumable shadow-ray march (SUSP kernels); *susp = true when it
  // was suspended (the call is repeated with the same arguments later)
  // What the MIS weight of a sphere light's sample reuses from the sampling
  // (brdf(), 1956-1962): lightSamplingPdf's d², r² and cos θmax are the
  // same expressions as calcDirectLighting's (1185-1187) when the light does
  // not move (RENDER_MODE 0): max(0, 1 - r²/d²) and 1 - clamp(r²/d², 0, 1)
  // agree wherever lightSamplingPdf reaches its sqrt (d² > r²)
  struct LightGeo {
    bool sphere;
    float d2, r2, cam;
    v3 ld;  // normalize(light - x)
  };
  // calcDirectLighting's contribution of a sphere light's sample whose shadow
  // ray reached light mesh il at t (1198-1205; il < 0: blocked)
  DEV v3 sphere_light_lit(int il, float t, float cos_a_max, v3 sr, v3 nl) {
    if (il < 0) return mk(0.f, 0.f, 0.f);
    const MatRec mh = light_mat(il);
    float weight = 2.0f * (1.0f - cos_a_max);
    float T_fog = 1.0f;
    if (VOL && flag(F_VOL)) T_fog = fexp(-VOL_SIGMA_T * t);
    v3 c = vmaxs(mk(mh.cr, mh.cg, mh.cb), 0.001f);
    return (((c * mk(mh.er, mh.eg, mh.eb)) * weight) * fmaxf(0.001f, dot(sr, nl))) * T_fog;
  }
  // The shadow ray of a wavefront shade kernel's light-sampling call
  // (RT0_WAVEFRONT): direct_light evaluates the call with the ray's closest
  // QUADRIC hit and returns the contribution that gives; the ray, that hit's
  // t (the SDF march's bound) and whether a march that stops exactly at INF_T
  // still lights it (a directional light) go to the march kernel, which keeps
  // the contribution only if the march finds no SDF surface before the bound
  // (wf_march_body).  Exact because no SDF of these scenes is a light
  // (rt0_host.cpp wf_eligible): a winning SDF surface is never lit, and when
  // the quadric hit gives nothing the SDF cannot give anything either.
  struct WfShadow {
    v3 o, d;
    float tq;
    bool dirl;
  };
  // the closest quadric hit only (intersection()'s mesh loop, no SDF march)
  DEV float isect_q(v3 o, v3 d, Hit &h) {
    return G::template intersect<false>(P, sc, C, o, d, h, n_map, nullptr, nullptr, g_lds);
  }
  // (dyn: li is a per-lane index -- ReSTIR's chosen light -- read from the
  // LDS tables; otherwise a loop constant that folds)
  DEV v3 direct_light(int li, v3 x, v3 nl, float seed, March *ms = nullptr, bool *susp = nullptr,
                      LightGeo *geo = nullptr, bool dyn = false, WfShadow *wj = nullptr) {
    if (COUNT) ++n_nee;
    const GeomRec g = dyn ? geom_at(li) : sc.geom(li);
    const MatRec lm = dyn ? mat_at(li) : sc.mat(li);
    Hit hit;
    v3 dl = mk(0.f, 0.f, 0.f);
    if (lm.type == M_LIGHT) {
      if (g.type == T_SPHERE) {
        v3 sw = lpos(li, g) - x;  // 1185
        float d2 = dot(sw, sw);
        float cos_a_max = fsqrt(1.0f - fminf(fmaxf(fdiv(g.d0, d2), 0.0f), 1.0f));
        const v3 lw = normalize(sw);
        if (geo) *geo = LightGeo{true, d2, g.d0, cos_a_max, lw};
        v3 sr = sample_cone(lw, 1.0f - cos_a_max, seed + 23.1656f);
        if (fast_shadow()) {
          float t;
          if (COUNT) ++n_isect;
          const int il = G::template shadow_light<Cfg>(P, sc, C, x + nl * EPSILON, sr, t, COUNT ? n_bvh : nullptr);
          return sphere_light_lit(il, t, cos_a_max, sr, nl);
        }
        const v3 so = x + nl * EPSILON;
        float t;
        if (wj) {
          t = isect_q(so, sr, hit);
          *wj = WfShadow{so, sr, t, false};
        } else {
          t = isect(so, sr, hit, ms);
        }
        if (ms && t < 0.0f) {
          *susp = true;
          return dl;
        }
        const MatRec mh = mat_at(hit.index);
        if (mh.type == M_LIGHT) {
          float weight = 2.0f * (1.0f - cos_a_max);
          float T_fog = 1.0f;
          if (VOL && flag(F_VOL)) T_fog = fexp(-VOL_SIGMA_T * t);
          v3 c = vmaxs(light_color(hit, mh), 0.001f);
          dl = (((c * mk(mh.er, mh.eg, mh.eb)) * weight) * fmaxf(0.001f, dot(sr, nl))) * T_fog;
        }
      } else if (SDF && g.type == T_SDF) {
        v3 ld = lpos(li, g) + random_sphere_dir(seed + 78.2358f) * mk(g.j0, g.j1, g.j2);  // 1207
        v3 sr = normalize(ld - x);
        if (isect(x + nl * EPSILON, sr, hit, ms) < 0.0f && ms) {
          *susp = true;
          return dl;
        }
        const MatRec mh = mat_at(hit.index);
        if (mh.type == M_LIGHT) {
          v3 c = vmaxs(light_color(hit, mh), 0.001f);
          dl = (c * mk(mh.er, mh.eg, mh.eb)) * fmaxf(0.001f, dot(sr, nl));
        }
      }
    } else if (lm.type == M_DIR_LIGHT) {
      v3 ld = mk(g.px, g.py, g.pz);
      const v3 so = x + nl * EPSILON;
      float t;
      if (wj) {
        t = isect_q(so, ld, hit);
        *wj = WfShadow{so, ld, t, true};
      } else {
        t = isect(so, ld, hit, ms);
      }
      if (ms && t < 0.0f) {
        *susp = true;
        return dl;
      }
      if (t == INF_T) dl = (mk(lm.cr, lm.cg, lm.cb) * mk(lm.er, lm.eg, lm.eb)) * fmaxf(0.001f, dot(ld, nl));
    }
    return dl;
  }

  // --------------------------------------------------------- ReSTIR parts
  DEV bool valid_res(const Res &r) {
    if (!finite_(r.M) || !finite_(r.ws) || !finite_(r.W) || !finite_(r.age)) return false;
    if (r.M <= 0.0f || r.M > 200.0f) return false;
    if (r.ws <= 0.0f || r.ws > 1000.0f) return false;
    if (r.W < 0.0f || r.W > 20.0f) return false;
    if (r.age < 0.0f || r.age > 35.0f) return false;
    float lc = dot(r.col, r.col);
    if (lc < 0.000001f || lc > 10000.0f) return false;
    if (r.idx >= sc.n_lights() && r.idx != -1) return false;
    if (dot(r.pos, r.pos) < EPSILON * EPSILON && r.idx >= 0) return false;
    return true;
  }
  DEV float target_fn(v3 lp, v3 lc, v3 hp, v3 hn, const MatRec &mat) {
    v3 lv = lp - hp;
    float dist_sq = dot(lv, lv);
    if (dist_sq < EPSILON * EPSILON) return 0.0f;
    v3 ld = normalize(lv);
    float ct = fmaxf(0.0f, dot(hn, ld));
    if (ct <= 0.0f) return 0.0f;
    const v3 lum = mk(0.2126f, 0.7152f, 0.0722f);
    float llum = dot(lc, lum);
    if (llum <= 0.0f) return 0.0f;
    float slum = dot(mk(mat.cr, mat.cg, mat.cb), lum);
    float nnt = fdiv(mat.nt - 1.0f, mat.nt + 1.0f);
    float R0 = nnt * nnt;
    float is_refr = (mat.type == M_REFR_FRESNEL || mat.type == M_REFR_SCHLICK) ? 1.0f : 0.0f;
    float is_coat = (mat.type == M_COAT) ? 1.0f : 0.0f;
    float base = mixf(slum, R0, is_refr);
    float bw = mixf(base, (1.0f - R0) * slum, is_coat) * ONE_OVER_PI;
    float safe = fmaxf(dist_sq, 1e-4f);
    return fdiv(llum * bw * ct, safe);
  }
  DEV bool visible(v3 from, v3 to) {
    v3 sd = to - from;
    float dist = length(sd);
    if (dist < EPSILON * 10.0f) return true;
    sd = normalize(sd);
    if (fast_shadow()) {
      if (COUNT) ++n_isect;
      return G::template visible_fast<Cfg>(P, sc, C, from + (sd * EPSILON) * 2.0f, sd, dist - EPSILON * 2.0f,
                                           COUNT ? n_bvh : nullptr);
    }
    Hit h;
    float t = isect(from + (sd * EPSILON) * 2.0f, sd, h);
    if (t < dist - EPSILON * 2.0f) {
      if (h.index >= 0 && h.index < sc.n_meshes() + sc.n_sdfs()) return sc.mat(h.index).type == M_LIGHT;
      return false;
    }
    return true;
  }
  // Sharded ReSTIR: does this shard hold reservoir row y (an own band, or
  // within halo_rows of one: the rows the exchange brings in)?
  // The band b = y / band and its owner b % n_shards by float reciprocals
  // (quot_small, exact far above any image height; tests/
  // test_kernel_identities.py): the integer divisions they replace cost ~30
  // VALU instructions each, four per row, two rows per reservoir tap.
  DEV bool row_local(int y) const {
    if (P.halo_rows <= 0) return y >= P.valid_lo && y < P.valid_hi;
    const int b = quot_small(y, P.band_inv), off = y - __mul24(b, P.band);
    const int r = b - __mul24(quot_small(b, P.shards_inv), P.n_shards);  // b % n_shards
    const bool own = r == P.shard;
    const bool below = b > 0 && r == P.shard_next && off < P.halo_rows;  // band b-1 is ours
    const bool above = __mul24(b + 1, P.band) < P.height && r == P.shard_prev && off >= P.band - P.halo_rows;
    return own || below || above;
  }
  // floor(a / d) for 0 <= a < 2^21 from inv = fl(1/d): (a + 0.5) / d lies at
  // least 0.5/d from an integer, and the two roundings move it by at most
  // (a + 0.5)/d * 2^-23 < 0.5/d
  DEV static int quot_small(int a, float inv) { return (int)(((float)a + 0.5f) * inv); }
  // GL LINEAR + CLAMP_TO_EDGE fetch of an RGBA32F plane (index.js:660-664)
  DEV float4 tex2d(const float4 *__restrict__ t, float u, float v) {
#pragma clang fp contract(off)
    float x = (u * P.res_x) - 0.5f, y = (v * P.res_y) - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float a = x - fx0, b = y - fy0;
    int x0 = (int)fx0, y0 = (int)fy0;
    int x1 = min(max(x0 + 1, 0), P.width - 1), y1 = min(max(y0 + 1, 0), P.height - 1);
    x0 = min(max(x0, 0), P.width - 1);
    y0 = min(max(y0, 0), P.height - 1);
    if (RT0_HALO_CHECK && P.halo_miss && !(row_local(y0) && row_local(y1))) atomicAdd(P.halo_miss, 1u);
    const size_t S = RT0_RES_STRIDE;
    float4 t00 = t[S * ((size_t)y0 * P.width + x0)], t10 = t[S * ((size_t)y0 * P.width + x1)];
    float4 t01 = t[S * ((size_t)y1 * P.width + x0)], t11 = t[S * ((size_t)y1 * P.width + x1)];
    return bil_lerp(t00, t10, t01, t11, a, b);
  }
  DEV static float4 bil_lerp(float4 t00, float4 t10, float4 t01, float4 t11, float a, float b) {
#pragma clang fp contract(off)
    float4 r;
    float top, bot;
    top = t00.x + (a * (t10.x - t00.x)); bot = t01.x + (a * (t11.x - t01.x)); r.x = top + (b * (bot - top));
    top = t00.y + (a * (t10.y - t00.y)); bot = t01.y + (a * (t11.y - t01.y)); r.y = top + (b * (bot - top));
    top = t00.z + (a * (t10.z - t00.z)); bot = t01.z + (a * (t11.z - t01.z)); r.z = top + (b * (bot - top));
    top = t00.w + (a * (t10.w - t00.w)); bot = t01.w + (a * (t11.w - t01.w)); r.w = top + (b * (bot - top));
    return r;
  }
  // tex2d split in two so that several taps' loads can be issued before any
  // of them is consumed (RT0_TAP_BATCH): the texel addresses and weights of a
  // tap (the same arithmetic as tex2d; `count` = the tap is really fetched,
  // for the sharded-ReSTIR halo check), then the lerp of the loaded texels
  struct Bil {
    uint32_t i00, i10, i01, i11;
    float a, b;
  };
  DEV Bil bil_at(float u, float v, bool count) {
#pragma clang fp contract(off)
    float x = (u * P.res_x) - 0.5f, y = (v * P.res_y) - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    Bil r;
    r.a = x - fx0;
    r.b = y - fy0;
    int x0 = (int)fx0, y0 = (int)fy0;
    int x1 = min(max(x0 + 1, 0), P.width - 1), y1 = min(max(y0 + 1, 0), P.height - 1);
    x0 = min(max(x0, 0), P.width - 1);
    y0 = min(max(y0, 0), P.height - 1);
    if (RT0_HALO_CHECK && count && P.halo_miss && !(row_local(y0) && row_local(y1))) atomicAdd(P.halo_miss, 1u);
    r.i00 = (uint32_t)(y0 * P.width + x0);
    r.i10 = (uint32_t)(y0 * P.width + x1);
    r.i01 = (uint32_t)(y1 * P.width + x0);
    r.i11 = (uint32_t)(y1 * P.width + x1);
    return r;
  }
  // the bilinear main/aux reservoir pair of a tap
  DEV static void bil_fetch2(const float4 *__restrict__ tm, const float4 *__restrict__ ta, const Bil &q, float4 &m,
                             float4 &a) {
    constexpr size_t S = RT0_RES_STRIDE;
    const float4 m00 = tm[S * q.i00], m10 = tm[S * q.i10], m01 = tm[S * q.i01], m11 = tm[S * q.i11];
    const float4 a00 = ta[S * q.i00], a10 = ta[S * q.i10], a01 = ta[S * q.i01], a11 = ta[S * q.i11];
    m = bil_lerp(m00, m10, m01, m11, q.a, q.b);
    a = bil_lerp(a00, a10, a01, a11, q.a, q.b);
  }
  DEV Res unpack(float4 m, float4 a) {
    Res r = empty_res();
    if (m.w > 0.0f) {
      r.pos = mk(m.x, m.y, m.z);
      r.W = m.w;
      r.col = mk(a.x, a.y, a.z);
      unpack_alpha(a.w, sc.n_lights(), r.age, r.M, r.idx);
      r.idx = min(max(r.idx, -1), sc.n_lights() - 1);
      r.M = fmaxf(1.0f, r.M);
      r.ws = r.W * r.M;
    }
    return r;
  }
  DEV void combine(Res &t, const Res &s, v3 hp, v3 hn, const MatRec &mat, float rnd) {
    if (!valid_res(s)) return;
    float tw = target_fn(s.pos, s.col, hp, hn, mat);
    if (tw <= 0.0f) return;
    float sc_ = fminf(fmaxf(tw * fmaxf(s.W, 0.0f) * fmaxf(s.M, 1.0f), 0.0f), 200.0f);
    t.ws += sc_;
    t.M += s.M;
    if (t.M > 40.0f) {
      float inv = fdiv(40.0f, t.M);
      t.ws *= inv;
      t.M = 40.0f;
    }
    if (t.ws > 0.0f) {
      float p = fdiv(sc_, t.ws);
      if (rnd < p) {
        t.pos = s.pos;
        t.col = s.col;
        t.idx = s.idx;
        t.age = fminf(s.age + 0.25f, 30.0f);
      }
    }
  }
  // isVisible() as a ghost call executes it (F_EXEC_GHOST): intersection()'s
  // mesh loop and iSDF's march do not run, so no quadric is hit and iSDF
  // reports its initial t = 4*EPSILON on the first SDF (index NUM_MESHES)
  DEV bool ghost_visible(v3 from, v3 to) {
    float dist = length(to - from);
    if (dist < EPSILON * 10.0f) return true;
    if (sc.n_sdfs() > 0 && EPSILON * 4.0f < dist - EPSILON * 2.0f) return sc.mat(sc.n_meshes()).type == M_LIGHT;
    return true;
  }
  // sampleLightsReSTIR, raytracer.glsl:1619-1801.  GHOST: the call as the
  // reference executor runs it for a lane that already left the bounce loop
  // (ghost_brdf): loops that are not unrolled (candidates, spatial taps,
  // the mesh loop of the visibility ray) do not run; the 2-level temporal loop
  // (unrolled) does; only g_final_reservoir is kept.
  template <bool GHOST = false>
  DEV v3 restir(v3 hp, v3 hn, const MatRec &mat, float sx, float sy) {
    if (!flag(F_RESTIR)) return mk(0.f, 0.f, 0.f);
    const int nl = sc.n_lights();
    if (nl == 0 || sc.light(0) < 0) return mk(0.f, 0.f, 0.f);
    if (COUNT && !GHOST) ++n_restir;
    return restir_finalize<GHOST>(restir_reservoir<GHOST>(hp, hn, mat, sx, sy), hp, hn, mat, sx);
  }
  // sampleLightsReSTIR up to finalizeReservoir (1625-1760): the initial RIS
  // reservoir, the two temporal levels and the spatial taps combined
  template <bool GHOST = false>
  DEV Res restir_reservoir(v3 hp, v3 hn, const MatRec &mat, float sx, float sy) {
    const int nl = sc.n_lights();
    const float scx = fcx / P.res_x, scy = fcy / P.res_y;
    Res init = empty_res();
    int eff = GHOST ? 0 : min(C.restir_samples(), max(4, nl));
    for (int i = 0; i < eff; i++) {
      float rvx, rvy;
      hash2(nc_addmul(sx, (float)i, 0.1f), nc_addmul(sy, (float)i, 0.2f), rvx, rvy);
      int ai = min(max((int)(rvx * (float)nl), 0), nl - 1);
      int li;
      v3 lp, lc;
      if (cand_lds) {  // the same values, one LDS round trip instead of two dependent global ones
        const float4 a = cand_lds[2 * ai], b = cand_lds[2 * ai + 1];
        li = __float_as_int(b.z);
        if (li < 0) continue;
        lp = mk(a.x, a.y, a.z);
        lc = mk(a.w, b.x, b.y);
      } else {
        li = sc.light(ai);
        if (li < 0 || li >= sc.n_meshes() + sc.n_sdfs()) continue;
        const GeomRec lg = sc.geom(li);
        const MatRec lmt = sc.mat(li);
        lp = lpos(li, lg);  // 1645
        lc = mk(lmt.cr, lmt.cg, lmt.cb) * mk(lmt.er, lmt.eg, lmt.eb);
      }
      if (COUNT) ++n_cand;
      float tv = target_fn(lp, lc, hp, hn, mat);
      if (tv > 0.0f) {  // updateReservoir, 1305-1326
        init.ws += tv;
        init.M += 1.0f;
        if (init.M > 60.0f) {
          init.ws *= 0.95f;
          init.M *= 0.95f;
        }
        if (init.ws > 0.0f) {
          if (rvy < fdiv(tv, init.ws)) {
            init.pos = lp;
            init.col = lc;
            init.idx = li;
          }
        }
      }
    }
    Res tr = init;
    if (frame > 2u) {
#if RT0_TAP_BATCH > 1
      // both history levels' texels are fetched before either is combined
      // (the same taps and arithmetic; only the loads move up)
      bool hin[2];
      float4 hm[2], ha[2];
      {
        Bil hq[2];
#pragma unroll
        for (int lvl = 0; lvl < 2; lvl++) {  // sampleTemporalHistory, 1485-1523
          v3 m3 = hp - mk(P.cam_px, P.cam_py, P.cam_pz);
          float ms = 0.001f * (float)(lvl + 1);
          float hjx, hjy;
          hash2(nc_addmul(scx, (float)((uint32_t)lvl + frame), 0.1f),
                nc_addmul(scy, (float)((uint32_t)lvl + frame), 0.1f), hjx, hjy);
          float px = (scx + m3.x * ms) + (hjx - 0.5f) * 0.002f;
          float py = (scy + m3.y * ms) + (hjy - 0.5f) * 0.002f;
          hin[lvl] = !(px < 0.01f || px > 0.99f || py < 0.01f || py > 0.99f);
          if (COUNT && !GHOST && hin[lvl]) ++n_ttap;
          hq[lvl] = bil_at(px, py, hin[lvl]);
        }
        bil_fetch2(P.rin[2], P.rin[3], hq[0], hm[0], ha[0]);
        bil_fetch2(P.rin[4], P.rin[5], hq[1], hm[1], ha[1]);
      }
#endif
      for (int lvl = 0; lvl < 2; lvl++) {
        Res h = empty_res();
#if RT0_TAP_BATCH > 1
        if (hin[lvl]) {
          h = unpack(lvl == 0 ? hm[0] : hm[1], lvl == 0 ? ha[0] : ha[1]);
          if (valid_res(h)) h.age += (float)(lvl + 1);
        }
#else
        {  // sampleTemporalHistory, 1485-1523
          v3 m3 = hp - mk(P.cam_px, P.cam_py, P.cam_pz);
          float ms = 0.001f * (float)(lvl + 1);
          float hjx, hjy;
          hash2(nc_addmul(scx, (float)((uint32_t)lvl + frame), 0.1f), nc_addmul(scy, (float)((uint32_t)lvl + frame), 0.1f),
                hjx, hjy);
          float px = (scx + m3.x * ms) + (hjx - 0.5f) * 0.002f;
          float py = (scy + m3.y * ms) + (hjy - 0.5f) * 0.002f;
          if (!(px < 0.01f || px > 0.99f || py < 0.01f || py > 0.99f)) {
            if (COUNT && !GHOST) ++n_ttap;
            float4 md = tex2d(P.rin[lvl == 0 ? 2 : 4], px, py);
            float4 ad = tex2d(P.rin[lvl == 0 ? 3 : 5], px, py);
            h = unpack(md, ad);
            if (valid_res(h)) h.age += (float)(lvl + 1);
          }
        }
#endif
        if (valid_res(h) && h.M > 0.0f && h.age < 30.0f) {
          if (flag(F_ANIM) && h.idx >= 0 && h.idx < nl) {  // history follows the moving light, 1669-1676
            const int act = sc.light(h.idx);
            if (act >= 0 && act < sc.n_meshes() + sc.n_sdfs()) {
              const MatRec am = sc.mat(act);
              h.pos = lpos(act, sc.geom(act));
              h.col = mk(am.cr, am.cg, am.cb) * mk(am.er, am.eg, am.eb);
            }
          }
          h.age += (float)(lvl + 1);
          float ta = lvl == 1 ? 0.95f * 0.80f : 0.95f;
          if (flag(F_ANIM)) ta *= 0.85f;  // 1688-1690
          h.M *= ta;
          h.ws *= ta;
          float trand = hash(nc_addmul(sx + 789.123f, (float)lvl, 456.789f));
          combine(tr, h, hp, hn, mat, trand);
        }
      }
      if (tr.M > 100.0f) {
        tr.M = fminf(tr.M, 80.0f);
        tr.ws *= 0.9f;
      }
    }
    Res fr = tr;
    int ns = nl > 10 ? 4 : 8;
    if (frame < 10u) ns = max(2, ns / 2);
    if (GHOST) ns = 0;
    const float PX[8] = {-0.4706f, 0.8090f, -0.2628f, 0.6882f, -0.9511f, 0.1625f, 0.5000f, -0.6882f};
    const float PY[8] = {0.4706f, 0.2628f, -0.8090f, -0.5000f, -0.1625f, 0.9511f, -0.6882f, 0.5000f};
#if RT0_TAP_BATCH > 1
    // RT0_TAP_BATCH taps at a time: their texel loads are issued together
    // before the first of them is combined, so a lane waits for one memory
    // round trip per batch instead of one per tap.  Same taps, same order,
    // same arithmetic (out-of-range taps load clamped texels and drop them).
    for (int i0 = 0; i0 < ns; i0 += RT0_TAP_BATCH) {
      float tsx[RT0_TAP_BATCH], tsy[RT0_TAP_BATCH];
      bool tin[RT0_TAP_BATCH];
      float4 tm[RT0_TAP_BATCH], ta[RT0_TAP_BATCH];
      {
        Bil tq[RT0_TAP_BATCH];
#pragma unroll
        for (int j = 0; j < RT0_TAP_BATCH; ++j) {
          const int i = i0 + j, ic = min(i, 7);
          hash2(nc_addmul(sx, (float)i, 0.3f), nc_addmul(sy, (float)i, 0.4f), tsx[j], tsy[j]);
          float nx = scx + (PX[ic] * 16.0f) / P.res_x, ny = scy + (PY[ic] * 16.0f) / P.res_y;
          tin[j] = i < ns && !(nx < 0.0f || nx > 1.0f || ny < 0.0f || ny > 1.0f);
          if (COUNT && tin[j]) ++n_stap;
          tq[j] = bil_at(nx, ny, tin[j]);
        }
#pragma unroll
        for (int j = 0; j < RT0_TAP_BATCH; ++j) bil_fetch2(P.rin[0], P.rin[1], tq[j], tm[j], ta[j]);
      }
#pragma unroll
      for (int j = 0; j < RT0_TAP_BATCH; ++j) {
        if (i0 + j >= ns) break;
        Res nb = empty_res();
        if (tin[j]) nb = unpack(tm[j], ta[j]);
        if (nb.M > 0.0f) {
          if (nb.idx >= 0) {
            v3 ldf = nb.pos - hp;
            if (dot(ldf, ldf) > 225.0f) continue;
          }
          if (nb.age > (flag(F_ANIM) ? 2.0f : 30.0f * 0.8f) || tsx[j] < 0.03f) continue;  // 1743
          combine(fr, nb, hp, hn, mat, tsy[j]);
        }
      }
    }
#else
    for (int i = 0; i < ns; i++) {
      float srx, sry;
      hash2(nc_addmul(sx, (float)i, 0.3f), nc_addmul(sy, (float)i, 0.4f), srx, sry);
      float nx = scx + (PX[i] * 16.0f) / P.res_x, ny = scy + (PY[i] * 16.0f) / P.res_y;
      Res nb = empty_res();
      if (!(nx < 0.0f || nx > 1.0f || ny < 0.0f || ny > 1.0f)) {
        if (COUNT) ++n_stap;
        nb = unpack(tex2d(P.rin[0], nx, ny), tex2d(P.rin[1], nx, ny));
      }
      if (nb.M > 0.0f) {
        if (nb.idx >= 0) {
          v3 ldf = nb.pos - hp;
          if (dot(ldf, ldf) > 225.0f) continue;
        }
        if (nb.age > (flag(F_ANIM) ? 2.0f : 30.0f * 0.8f) || srx < 0.03f) continue;  // 1743
        combine(fr, nb, hp, hn, mat, sry);
      }
    }
#endif
    return fr;
  }
  // finalizeReservoir's W of a visible reservoir with target tp > 0 (1541-1568)
  DEV float restir_weight(const Res &fr, float tp) {
    float cM = fminf(fmaxf(fr.M, 1.0f), 40.0f);
    float raw = fr.ws / (tp * cM);
    float bc = 1.0f;
    if (fr.age > 0.0f) {
      float na = fminf(fmaxf(fr.age / 30.0f, 0.0f), 1.0f);
      bc *= mixf(0.85f, 1.0f, 1.0f - na * 0.3f);
    }
    if (cM > 16.0f) bc *= fsqrt(16.0f / cM);
    float W = fminf(fmaxf(bc * raw, 0.0f), 12.0f);
    return finite_(W) ? W : 0.0f;
  }
  // the light's shading weight of a reservoir (1778-1780)
  DEV static float restir_ew(const Res &fr) {
    float ew = fminf(fmaxf(fr.W, 0.0f), 8.0f);
    if (fr.M > 30.0f) ew *= fsqrt(30.0f / fr.M);
    return ew;
  }

  // RT0_NEE_WALK (light-sampling kernels of scenes with triangle models):
  // sampleLightsReSTIR with its two triangle occlusion queries -- the
  // visibility ray of finalizeReservoir (isVisible, 1539-1557) and the shadow
  // ray of the picked light (calcDirectLighting, 1185-1205) -- handed to
  // rt0_jit_walk, which walks them on dense lanes; rt0_jit_resolve completes the
  // call from their answers.  Everything else runs here, as in restir(): the
  // reservoir, the quadric part of both rays (a quadric that decides alone
  // leaves no walk), W, and the light's contribution as it is if the shadow
  // ray passes.  The shadow ray is cast before visibility is known (it is a
  // function of the hit point, the light and the seed only); its answer is
  // used only where restir() would cast it (visible, W > 0).
  struct Split {
    bool done;     // finished here: c and fin are final
    v3 c;          // done: the call's result
    WalkJob j[2];  // [0] visibility, [1] shadow ray
    bool has[2];
    float W;  // W if visible
    v3 f;     // the result if visible and the shadow ray passes
  };
  DEV Split restir_split(v3 hp, v3 hn, const MatRec &mat, float sx, float sy) {
    Split o;
    o.done = true;
    o.c = mk(0.f, 0.f, 0.f);
    o.has[0] = o.has[1] = false;
    if (!flag(F_RESTIR)) return o;
    const int nl = sc.n_lights();
    if (nl == 0 || sc.light(0) < 0) return o;
    Res fr = restir_reservoir<false>(hp, hn, mat, sx, sy);
    // the host selects RT0_NEE_WALK only for such scenes (and a BVH with
    // triangles), so in a walk module this folds away
    if (!fast_shadow() || flag(F_ANIM) || sc.n_models() <= 0) {
      o.c = restir_finalize<false>(fr, hp, hn, mat, sx);
      return o;
    }
    const float tp = (fr.ws > 0.0f && fr.M > 0.0f) ? target_fn(fr.pos, fr.col, hp, hn, mat) : 0.0f;
    if (!(tp > 0.0f)) {  // W = 0 without a ray
      fr.W = 0.0f;
      fr.age = fminf(fr.age, 30.0f);
      fin = fr;
      return o;
    }
    // visible(hp, fr.pos)
    v3 sd = fr.pos - hp;
    const float dist = length(sd);
    if (!(dist < EPSILON * 10.0f)) {
      sd = normalize(sd);
      const v3 o1 = hp + (sd * EPSILON) * 2.0f;
      const v3 m1 = mk(frcp(sd.x), frcp(sd.y), frcp(sd.z));
      float t1;
      if (!G::template visible_q<Cfg>(P, sc, C, o1, sd, m1, dist - EPSILON * 2.0f, t1)) {
        fr.W = 0.0f;  // a quadric hides the light
        fr.age = fminf(fr.age, 30.0f);
        fin = fr;
        return o;
      }
      o.has[0] = true;
      o.j[0] = WalkJob{o1.x, o1.y, o1.z, t1, sd.x, sd.y, sd.z, 0u};
    }
    fr.W = restir_weight(fr, tp);
    v3 f = mk(0.f, 0.f, 0.f);
    if (fr.W > 0.0f && fr.idx >= 0 && fr.idx < nl) {
      const int act = light_at(fr.idx);
      if (act >= 0 && act < sc.n_meshes() + sc.n_sdfs()) {
        // direct_light(act, hp, hn, sx + 456.789f), 1174-1230, up to its triangle query
        const GeomRec g = geom_at(act);
        const MatRec lm = mat_at(act);
        const float ew = restir_ew(fr);
        const v3 o2 = hp + hn * EPSILON;
        if (lm.type == M_LIGHT && g.type == T_SPHERE) {  // 1185-1205
          const v3 sw = mk(g.px, g.py, g.pz) - hp;
          const float d2 = dot(sw, sw);
          const float cos_a_max = fsqrt(1.0f - fminf(fmaxf(fdiv(g.d0, d2), 0.0f), 1.0f));
          const v3 sr = sample_cone(normalize(sw), 1.0f - cos_a_max, (sx + 456.789f) + 23.1656f);
          float t2;
          const int il = G::template shadow_light_q<Cfg>(P, sc, C, o2, sr, mk(frcp(sr.x), frcp(sr.y), frcp(sr.z)), t2);
          f = sphere_light_lit(il, t2, cos_a_max, sr, hn) * ew;
          if (il >= 0) o.j[1] = WalkJob{o2.x, o2.y, o2.z, t2, sr.x, sr.y, sr.z, 1u};
        } else if (lm.type == M_DIR_LIGHT) {  // 1224-1229: lit iff intersection() misses everything
          const v3 ld = mk(g.px, g.py, g.pz);
          float tq;
          (void)G::template visible_q<Cfg>(P, sc, C, o2, ld, mk(frcp(ld.x), frcp(ld.y), frcp(ld.z)), INF_T, tq);
          if (tq == INF_T) {
            f = ((mk(lm.cr, lm.cg, lm.cb) * mk(lm.er, lm.eg, lm.eb)) * fmaxf(0.001f, dot(ld, hn))) * ew;
            o.j[1] = WalkJob{o2.x, o2.y, o2.z, INF_T, ld.x, ld.y, ld.z, 1u};
          }
        }  // other light meshes contribute nothing (direct_light's own cases)
        if (!finite_(f.x) || !finite_(f.y) || !finite_(f.z)) f = mk(0.f, 0.f, 0.f);
        // a shadow ray matters only for a non-zero contribution
        o.has[1] = f.x != 0.0f || f.y != 0.0f || f.z != 0.0f;
        if (!o.has[1]) f = mk(0.f, 0.f, 0.f);
      }
    }
    fr.age = fminf(fr.age, 30.0f);
    fin = fr;  // W as if visible; rt0_jit_resolve zeroes it when the visibility ray is blocked
    if (!o.has[0] && !o.has[1]) {  // nothing left to walk
      o.c = f;
      return o;
    }
    o.done = false;
    o.W = fr.W;
    o.f = f;
    return o;
  }

  // finalizeReservoir (1525-1576) and the light's shading (1762-1800)
  template <bool GHOST = false>
  DEV v3 restir_finalize(Res fr, v3 hp, v3 hn, const MatRec &mat, float sx) {
    const int nl = sc.n_lights();
    if (fr.ws <= 0.0f || fr.M <= 0.0f) {
      fr.W = 0.0f;
    } else {
      float tp = target_fn(fr.pos, fr.col, hp, hn, mat);
      if (tp <= 0.0f || !(GHOST ? ghost_visible(hp, fr.pos) : visible(hp, fr.pos))) {
        fr.W = 0.0f;
      } else {
        fr.W = restir_weight(fr, tp);
      }
    }
    fr.age = fminf(fr.age, 30.0f);
    fin = fr;
    if (GHOST) return mk(0.f, 0.f, 0.f);
    if (fr.W > 0.0f && fr.idx >= 0 && fr.idx < nl) {
      int act = light_at(fr.idx);
      if (act >= 0 && act < sc.n_meshes() + sc.n_sdfs()) {
        // RENDER_MODE 1 re-checks visibility of the light's current position
        // (1767-1776); g_final_reservoir was stored before that update
        if (flag(F_ANIM) && !visible(hp, lpos(act, sc.geom(act)))) return mk(0.f, 0.f, 0.f);
        v3 lc = direct_light(act, hp, hn, sx + 456.789f, nullptr, nullptr, nullptr, true);
        v3 fc = lc * restir_ew(fr);
        if (!finite_(fc.x) || !finite_(fc.y) || !finite_(fc.z)) return mk(0.f, 0.f, 0.f);
        return fc;
      }
    }
    return mk(0.f, 0.f, 0.f);
  }

  // Does sample_lights() route this call to sampleLightsReSTIR (raytracer.
  // glsl:1900-1946)?  use_restir without use_mis, or use_mis with more than 8
  // lights; never in the counting instance (its event counts stay inline)
  DEV bool restir_routed() const {
    if constexpr (!RESTIR || COUNT) return false;
    if (!flag(F_RESTIR) || !flag(F_RESTIR_DEF)) return false;
    return !flag(F_MIS) || sc.n_lights() > 8;
  }
  // RT0_DEFER_NEE: append the call as a NeeRec to the wave's region (one LDS
  // add per wave: the active lanes take consecutive slots) instead of running
  // it; rt0_jit_nee runs it
  // with the same arguments and rt0_jit_resolve adds result * mask to the
  // sample.  The seeds are the ones sample_lights() passes (1909/1943).
  DEV void defer_nee(v3 x, v3 nl, int mi, float seed, float bounce, v3 mask) {
    (void)seed;  // the light-sampling kernel recomputes it from the pixel (restir_seeds)
    const unsigned long long act = __ballot(1);
    const int lane = (int)(threadIdx.x & 63u);
    const int leader = __ffsll((long long)act) - 1;
    const int rank = __popcll(act & ((1ull << lane) - 1ull));
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(nee_wave_counter(), (uint32_t)__popcll(act));
    base = __shfl(base, leader);
    const uint32_t i = base + (uint32_t)rank;
    if (i < (uint32_t)P.nee_cap) {  // nee_cap = 64 lanes x max_bounces calls: never exceeded
      NeeRec r;
      r.x = x.x;
      r.y = x.y;
      r.z = x.z;
      r.nx = nl.x;
      r.ny = nl.y;
      r.nz = nl.z;
      r.mr = mask.x;
      r.mg = mask.y;
      r.mb = mask.z;
      r.pix = nee_pix;
      r.mkb = (uint32_t)mi | ((uint32_t)nee_k << 8) | ((uint32_t)bounce << 16);
      r.pad = 0;
      P.nee_rec[(size_t)nee_wave * (uint32_t)P.nee_cap + i] = r;
    }
    ++nee_k;
  }

  // Non-specular light sampling dispatch, raytracer.glsl:1899-1976
  DEV v3 sample_lights(v3 x, v3 nl, const MatRec &mat, float seed, float bounce) {
    const float fr = (float)frame;
    v3 acc = mk(0.f, 0.f, 0.f);
    const int nlights = sc.n_lights();
    if (flag(F_RESTIR) && flag(F_MIS)) {
      if (RESTIR && flag(F_RESTIR_DEF)) {
        if (nlights > 8) {
          acc = restir(x, nl, mat, nc_seed3(seed, 8652.1f, fr, bounce, 7895.13f),
                       nc_seed3(seed, 1234.567f, fr, bounce, 9876.54f));
        } else {
          const float base = nc_seed4(seed, 8652.1f, fr, 5681.123f, bounce, 7895.13f);
          for_lights(sc, [&](int i) {
            int idx = sc.light(i);
            if (idx < 0) return;
            const GeomRec lg = sc.geom(idx);
            const MatRec lmt = sc.mat(idx);
            if (lmt.type != M_LIGHT) return;
            v3 lv = mk(lg.px, lg.py, lg.pz) - x;
            v3 ld = normalize(lv);
            float dsq = dot(lv, lv);
            float ct = fmaxf(0.0f, dot(nl, ld));
            float imp = ct * dot(mk(lmt.er, lmt.eg, lmt.eb), mk(0.2126f, 0.7152f, 0.0722f)) * frsq(dsq + 1.0f);
            if (imp < 0.001f) return;
            v3 ls = direct_light(idx, x, nl, nc_addmul(base, (float)i, 123.456f));
            if (dot(ls, ls) < 0.001f * 0.001f) return;
            acc = acc + ls * power_heuristic(light_pdf(lg, lmt, x), cos_pdf(ld, nl));
          });
        }
      }
    } else if (flag(F_RESTIR)) {
      if (RESTIR && flag(F_RESTIR_DEF))
        acc = restir(x, nl, mat, nc_seed3(seed, 8652.1f, fr, bounce, 7895.13f),
                     nc_seed3(seed, 1234.567f, fr, bounce, 9876.54f));
    } else if (flag(F_MIS) && nlights > 0) {
      const float base = nc_seed4(seed, 8652.1f, fr, 5681.123f, bounce, 7895.13f);
      for_lights(sc, [&](int i) {
        int idx = light_q(i, bounce);
        if (idx < 0) return;
        const GeomRec lg = sc.geom(idx);
        const MatRec lmt = sc.mat(idx);
        if (lmt.type != M_LIGHT) return;
        LightGeo geo{false, 0.f, 0.f, 0.f, mk(0.f, 0.f, 0.f)};
        v3 ls = direct_light(idx, x, nl, nc_addmul(base, (float)i, 123.456f), nullptr, nullptr, &geo);
        if (dot(ls, ls) > 0.000001f) {
          if (geo.sphere && !flag(F_ANIM)) {  // the sampling's own d², cos θmax and direction
            float lp = 0.0f;
            if (geo.d2 > geo.r2 && 1.0f - geo.cam >= 1e-6f) lp = frcp(TWO_PI * (1.0f - geo.cam));
            acc = acc + ls * power_heuristic(lp, cos_pdf(geo.ld, nl));
          } else {
            v3 ld = normalize(lpos(idx, lg) - x);  // 1959 (lightSamplingPdf keeps light.pos)
            acc = acc + ls * power_heuristic(light_pdf(lg, lmt, x), cos_pdf(ld, nl));
          }
        }
      });
    } else {
      const float s = nc_seed4(seed, 8652.1f, fr, 5681.123f, bounce, 7895.13f);
      for_lights(sc, [&](int i) {
        int idx = light_q(i, bounce);
        if (idx >= 0) acc = acc + direct_light(idx, x, nl, s);
      });
    }
    return acc;
  }

  // F_EXEC_GHOST: the reference executor (SwiftShader 4.1, the oracle) still
  // calls brdf() (raytracer.glsl:2094) for a lane in the iteration in which
  // it executed `break` (2049, 2057, 2065, 2089), with its parameter
  // registers as the lane's previous call left them, and does not mask the
  // global g_final_reservoir that call's sampleLightsReSTIR stores (1757).
  // Pinned by oracle/gen/mask_kat.py; the same model in the restatement
  // matches the reference's reservoir outputs on >= 99.7% of pixels through 6
  // chained passes (tests/test_oracle_golden.py).  Repeats the previous
  // call's material branch (COAT's Schlick pick on the post-call ray) and,
  // when that leaves the bounce diffuse and routes light sampling through
  // ReSTIR, the ghost ReSTIR call.
  DEV void ghost_brdf(float seed) {
    if (!gr_have) return;
    const MatRec mt = sc.mat(gr_mat);
    bool spec = gr_spec;
    if (mt.type == M_DIFF) {
      spec = false;
    } else if (mt.type == M_SPEC || mt.type == M_REFR_FRESNEL || mt.type == M_REFR_SCHLICK) {
      spec = true;
    } else if (mt.type == M_COAT) {
      float nt_eff = fabsf(mt.nt);
      if constexpr (SPECTRAL) {
        if (flag(F_SPECTRAL) && mt.nt < 0.0f) nt_eff = spectral_ior(hero, fabsf(mt.nt));
      }
      spec = hash(seed) < schlick(gr_rd, gr_nl, 1.00029f, nt_eff);
    }
    if (spec || !flag(F_SAMPLE_LIGHTS) || !flag(F_RESTIR_DEF)) return;
    if (flag(F_RESTIR) && flag(F_MIS)) {
      if (sc.n_lights() <= 8) return;
    } else if (!flag(F_RESTIR)) {
      return;
    }
    const float fr = (float)frame;
    restir<true>(gr_x, gr_nl, mt, nc_seed3(seed, 8652.1f, fr, gr_bounce, 7895.13f),
                 nc_seed3(seed, 1234.567f, fr, gr_bounce, 9876.54f));
  }
  DEV bool ghost_on() const { return RESTIR && (C.flags() & F_EXEC_GHOST) != 0; }

  // ---- executor compatibility, rule 11 (mask_kat.py QUAD LIGHTS; the
  // restatement's quad_light_index, oracle/rt0_oracle.c): in brdf()'s light
  // loops (raytracer.glsl:1955-1974) the reference executor reads the
  // loop-indexed light_index[i] at the index register of the 2x2 quad's FIRST
  // lane.  That register holds i when the first lane runs the same loop in
  // the same bounce-loop iteration -- live, or as the ghost brdf() call of
  // the iteration it breaks in (the plain loop unrolled, rule 5; not counted
  // under the medium) -- and a stale value otherwise: mesh 0 (the loop's end,
  // one past the array, reads 0), or with the medium's `continue` before the
  // breaks (USE_VOLUMETRICS) element 0 before the first lane's first run.
  // The first lane's record comes from a preceding launch of the same frame
  // (P.quad_mode 1, rt0_host.cpp render_impl).  Quadric-only modules without
  // ReSTIR; compiled out unless F_EXEC_GHOST.
  DEV bool quad_rec() const { return !RESTIR && (C.flags() & F_EXEC_GHOST) != 0 && P.quad_mode != 0; }
  DEV int light_q(int i, float bounce) {
    const int li = sc.light(i);
    if (!quad_rec()) return li;
    const int d = (int)bounce;
    if (d >= 32) return li;  // (32 bounces of record)
    if (i == 0) q_own |= 1u << d;
    if (!q0_on || sc.n_lights() < 2) return li;
    const uint32_t m = q0_m | (flag(F_VOL) ? 0u : q0_g);
    if ((m >> d) & 1u) return li;
    if (flag(F_VOL) && (m & ((1u << d) - 1u)) == 0u) return sc.light(0);
    return 0;
  }
  // the ghost brdf() of a `break` iteration (see ghost_brdf): its material
  // branch on the last live call's registers; a non-specular outcome runs the
  // plain light loop (unrolled: constant trip count <= 4)
  DEV void quad_ghost(float seed, int depth) {
    if (!gr_have || depth >= 32) return;
    const MatRec mt = sc.mat(gr_mat);
    bool spec = gr_spec;
    if (mt.type == M_DIFF) {
      spec = false;
    } else if (mt.type == M_SPEC || mt.type == M_REFR_FRESNEL || mt.type == M_REFR_SCHLICK) {
      spec = true;
    } else if (mt.type == M_COAT) {
      float nt_eff = fabsf(mt.nt);
      if constexpr (SPECTRAL) {
        if (flag(F_SPECTRAL) && mt.nt < 0.0f) nt_eff = spectral_ior(hero, fabsf(mt.nt));
      }
      spec = hash(seed) < schlick(gr_rd, gr_nl, 1.00029f, nt_eff);
    }
    if (!spec && flag(F_SAMPLE_LIGHTS) && !flag(F_RESTIR) && !(flag(F_MIS) && sc.n_lights() > 0) &&
        sc.n_lights() <= 4)
      q_gown |= 1u << depth;
  }
  DEV void quad_begin() {
    if (!quad_rec()) return;
    q_own = q_gown = 0u;
    gr_have = false;
    q0_on = P.quad_mode == 2 && ((q_px | q_py) & 1) != 0;
    if (q0_on) {
      const uint2 m = P.quad_masks[(size_t)(q_py & ~1) * P.width + (q_px & ~1)];
      q0_m = m.x;
      q0_g = m.y;
    }
  }
  DEV void quad_store() const {
    if (quad_rec() && P.quad_mode == 1) P.quad_masks[(size_t)q_py * P.width + q_px] = make_uint2(q_own, q_gown);
  }

  // ---- wavefront SDF renders (WF): light sampling as march jobs
  // One shadow ray of light slot l whose answer matters: appended to this
  // wave's region of the round's shadow list through the wave's LDS counter
  // (any subset of lanes may append: one LDS add per call site).  c = the
  // contribution if the march finds no SDF surface before tq (WfShadow).
  DEV void wf_emit_shadow(int l, v3 o, v3 d, float tq, v3 c, bool dirl) {
    const uint32_t i = wave_append(wf_wave_counter(1));  // < wf_R * wf_L: one job per light per slot
    float4 *e = P.wf_sh + 3 * ((size_t)wf_region * (uint32_t)P.wf_R * (uint32_t)P.wf_L + i);
    e[0] = make_float4(o.x, o.y, o.z, tq);
    e[1] = make_float4(d.x, d.y, d.z, __uint_as_float((uint32_t)l * P.wf_slots + wf_slot));
    e[2] = make_float4(c.x, c.y, c.z, dirl ? 1.0f : 0.0f);
    wf_bits |= 1u << l;
  }
  // brdf()'s non-specular light sampling (raytracer.glsl:1899-1976, plain or
  // MIS; ReSTIR is not in these modules): sample_lights' calls, each with
  // its quadric answer, the surviving ones as march jobs
  DEV void wf_nee_surface(v3 x, v3 nl, float seed, float bounce) {
    if (flag(F_RESTIR)) return;  // (sample_lights: use_restir without USE_RESTIR adds nothing)
    const float fr = (float)frame;
    const float base = nc_seed4(seed, 8652.1f, fr, 5681.123f, bounce, 7895.13f);
    wf_kind = 1;
    for_lights(sc, [&](int i) {
      const int idx = sc.light(i);
      if (idx < 0) return;
      WfShadow wj{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), -1.0f, false};
      if (flag(F_MIS)) {
        const GeomRec lg = sc.geom(idx);
        const MatRec lmt = sc.mat(idx);
        if (lmt.type != M_LIGHT) return;
        LightGeo geo{false, 0.f, 0.f, 0.f, mk(0.f, 0.f, 0.f)};
        const v3 ls = direct_light(idx, x, nl, nc_addmul(base, (float)i, 123.456f), nullptr, nullptr, &geo, false, &wj);
        if (!(dot(ls, ls) > 0.000001f) || wj.tq < 0.0f) return;
        float w;
        if (geo.sphere && !flag(F_ANIM)) {  // (sample_lights' reuse of the sampling's d², cos θmax, direction)
          float lp = 0.0f;
          if (geo.d2 > geo.r2 && 1.0f - geo.cam >= 1e-6f) lp = frcp(TWO_PI * (1.0f - geo.cam));
          w = power_heuristic(lp, cos_pdf(geo.ld, nl));
        } else {
          const v3 ld = normalize(lpos(idx, lg) - x);
          w = power_heuristic(light_pdf(lg, lmt, x), cos_pdf(ld, nl));
        }
        wf_emit_shadow(i, wj.o, wj.d, wj.tq, ls * w, wj.dirl);
      } else {
        const v3 dl = direct_light(idx, x, nl, base, nullptr, nullptr, nullptr, false, &wj);
        if ((dl.x != 0.0f || dl.y != 0.0f || dl.z != 0.0f) && wj.tq >= 0.0f) wf_emit_shadow(i, wj.o, wj.d, wj.tq, dl, wj.dirl);
      }
    });
  }
  // the in-scatter light loop of a volume event (raytracer.glsl:2011-2044):
  // each light's term with its quadric answer, the lit ones as march jobs
  DEV void wf_nee_volume(v3 sp, v3 rd, v3 mask, float seed, int depth) {
    wf_kind = 2;
    for_lights(sc, [&](int li) {
      const int lidx = sc.light(li);
      if (lidx < 0) return;
      const GeomRec lg = sc.geom(lidx);
      const MatRec lmt = sc.mat(lidx);
      if (lmt.type != M_LIGHT || lg.type != T_SPHERE) return;
      v3 dlc = mk(lg.px, lg.py, lg.pz) - sp;
      float dc = length(dlc);
      float cam = fsqrt(1.0f - fminf(fmaxf(fdiv(lg.d0, dc * dc), 0.0f), 1.0f));
      float idc = frcp(dc);
      v3 dir = sample_cone(mk(dlc.x * idc, dlc.y * idc, dlc.z * idc), 1.0f - cam,
                           nc_addmul(nc_addmul(seed + 2341.7f, (float)li, 917.3f), (float)depth, 199.1f));
      Hit sh;
      const v3 so = sp + dir * (EPSILON * 20.0f);
      float ts = isect_q(so, dir, sh);
      if (sh.index != lidx) return;  // an SDF surface would only hide it
      float omega = 2.0f * (1.0f - cam);
      float ct = dot(rd, dir);
      constexpr float g2 = VOL_G * VOL_G;
      float den = 1.0f + g2 - 2.0f * VOL_G * ct;
      float phase = fdiv(1.0f - g2, FOUR_PI * den * fsqrt(den));
      float Tf = fexp(-VOL_SIGMA_T * ts);
      const v3 c = ((((mask * mk(lmt.cr, lmt.cg, lmt.cb)) * mk(lmt.er, lmt.eg, lmt.eb)) * phase) * Tf) * (PI_F * omega);
      wf_emit_shadow(li, so, dir, ts, c, false);
    });
  }

  // radiance() + brdf(), raytracer.glsl:1986-2105 and 1804-1980, as a step
  // function: one iteration of the bounce loop per call, so that a lane whose
  // path ended can start its next sample while the rest of its wave is still
  // bouncing (path regeneration in pass_body).  The path state is what the
  // shader keeps across iterations.
  //
  // SUSP kernels (SDF scenes, path regeneration, no ReSTIR): a sphere-tracing
  // march runs at most RT0_MARCH_BUDGET steps per call.  A lane whose march is
  // unfinished returns from step() and resumes it at its next call, while the
  // other lanes of its wave go on with their own bounces and samples -- so one
  // long march no longer holds 63 finished lanes idle.  A bounce is two
  // phases: 0 = its ray (and the shading that follows), 1 = its light
  // sampling (one shadow ray per light), each resumable; every lane still
  // performs exactly the operations of the uninterrupted loop, in order.
  // WF (RT0_WAVEFRONT modules): the same bounce step in the wavefront shade
  // kernel -- a pending march parks the path (wf_shade_body) instead of
  // suspending it, and the light-sampling calls' shadow rays become march
  // jobs (wf_nee_surface / wf_nee_volume)
  static constexpr bool WF = RT0_WAVEFRONT != 0 && SDF && !RESTIR && !COUNT;
  static constexpr bool SUSP = SDF && !RESTIR && !COUNT && !WF;
  // WFB (RT0_WAVEFRONT modules of ReSTIR scenes with triangle models): the
  // bounce step in the wavefront ReSTIR shade kernel -- a closest-hit query of
  // the triangles parks the path for the walk kernel (wf_restir_shade_body)
  static constexpr bool WFB = RT0_WAVEFRONT != 0 && RESTIR && !SDF && !COUNT && Scene::kMayHaveModels;
  struct NeeCtx {
    v3 x, n, acc;  // surface: hit point, nl, sum over lights; volume: scatter point, incoming rd
    float seed;    // surface: the light-sampling seed base; volume: the path seed
    int li;        // next light of the loop
    bool vol, end;  // in-scatter NEE; the path ends after this bounce
  };
  struct Path {
    v3 ro, rd, acc, mask, prev_nl;
    float seed;
    int depth;
    bool spec;
    int phase;  // SUSP only
    March ms;
    NeeCtx nc;
  };
  DEV March *march_slot(Path &ps) {
    if constexpr (WFB) return (sc.n_models() > 0 && P.n_tris > 0) ? &ps.ms : nullptr;
    if constexpr (!SUSP && !WF) return nullptr;
    // with triangle models the resumed call would walk the BVH again: no budget
    if constexpr (Scene::kMayHaveModels)
      if (sc.n_models() > 0 && P.n_tris > 0) return nullptr;
    return &ps.ms;
  }
  // The kernel's one sphere-tracing loop (SUSP): up to RT0_MARCH_BUDGET steps
  // of the lane's pending march, at a single program point for every lane of
  // the wave whatever ray (camera, bounce, shadow) it belongs to.  The steps
  // are iSDF's (raytracer.glsl:979-984) verbatim.
  DEV void march_pending(Path &ps) {
    March &m = ps.ms;
    if (!m.active) return;
    const int cap = C.marching_steps();
    float t = m.t, id = m.id;
    int i = m.i;
    const int lim = min(cap, i + RT0_MARCH_BUDGET);
    bool stop = i >= cap;
    for (; i < lim; ++i) {
      float dist = G::map(sc, ray_at(m.o, m.d, t), id, n_map);
      float h = fabsf(dist);
      if (h < EPSILON || t > m.tmin) {
        stop = true;
        break;
      }
      t = __builtin_fmaf(h, C.fudge(), t);
    }
    if (i >= cap) stop = true;
    m.t = t;
    m.id = id;
    m.i = i;
    if (stop) {
      m.active = false;
      m.done = true;
    }
  }
  // phase 1 of a SUSP bounce: the light-sampling loop of brdf() (1899-1976,
  // plain or MIS NEE) or of the in-scatter event (2011-2044), resumable per
  // light.  false = suspended.
  DEV bool nee_phase(Path &ps) {
    NeeCtx &nc = ps.nc;
    March *mq = march_slot(ps);
    bool susp = false;
    if (VOL && nc.vol) {
      const v3 sp = nc.x, rd = nc.n;
      const float seed = ps.seed;
      const int depth = ps.depth;
      for_lights(sc, [&](int li) {
        if (susp || li < nc.li) return;
        int lidx = sc.light(li);
        if (lidx < 0) return;
        const GeomRec lg = sc.geom(lidx);
        const MatRec lmt = sc.mat(lidx);
        if (lmt.type != M_LIGHT || lg.type != T_SPHERE) return;
        v3 dlc = mk(lg.px, lg.py, lg.pz) - sp;
        float dc = length(dlc);
        float cam = fsqrt(1.0f - fminf(fmaxf(fdiv(lg.d0, dc * dc), 0.0f), 1.0f));
        float idc = frcp(dc);
        v3 dir = sample_cone(mk(dlc.x * idc, dlc.y * idc, dlc.z * idc), 1.0f - cam,
                             nc_addmul(nc_addmul(seed + 2341.7f, (float)li, 917.3f), (float)depth, 199.1f));
        Hit sh;
        float ts = isect(sp + dir * (EPSILON * 20.0f), dir, sh, mq);
        if (mq && ts < 0.0f) {
          nc.li = li;
          susp = true;
          return;
        }
        if (sh.index != lidx) return;
        float omega = 2.0f * (1.0f - cam);
        float ct = dot(rd, dir);
        constexpr float g2 = VOL_G * VOL_G;
        float den = 1.0f + g2 - 2.0f * VOL_G * ct;
        float phase = fdiv(1.0f - g2, FOUR_PI * den * fsqrt(den));
        float Tf = fexp(-VOL_SIGMA_T * ts);
        ps.acc = ps.acc + ((((ps.mask * mk(lmt.cr, lmt.cg, lmt.cb)) * mk(lmt.er, lmt.eg, lmt.eb)) * phase) * Tf) *
                              (PI_F * omega);
      });
      return !susp;
    }
    // sample_lights() without ReSTIR: use_restir routes nothing here
    if (!flag(F_RESTIR)) {
      if (flag(F_MIS) && sc.n_lights() > 0) {
        for_lights(sc, [&](int i) {
          if (susp || i < nc.li) return;
          int idx = light_q(i, (float)ps.depth);
          if (idx < 0) return;
          const GeomRec lg = sc.geom(idx);
          const MatRec lmt = sc.mat(idx);
          if (lmt.type != M_LIGHT) return;
          v3 ls = direct_light(idx, nc.x, nc.n, nc_addmul(nc.seed, (float)i, 123.456f), mq, &susp);
          if (susp) {
            nc.li = i;
            return;
          }
          if (dot(ls, ls) > 0.000001f) {
            v3 ld = normalize(lpos(idx, lg) - nc.x);  // 1959
            nc.acc = nc.acc + ls * power_heuristic(light_pdf(lg, lmt, nc.x), cos_pdf(ld, nc.n));
          }
        });
      } else {
        for_lights(sc, [&](int i) {
          if (susp || i < nc.li) return;
          int idx = light_q(i, (float)ps.depth);
          if (idx < 0) return;
          v3 dl = direct_light(idx, nc.x, nc.n, nc.seed, mq, &susp);
          if (susp) {
            nc.li = i;
            return;
          }
          nc.acc = nc.acc + dl;
        });
      }
    }
    if (susp) return false;
    ps.acc = ps.acc + nc.acc * ps.mask;
    return true;
  }
  // false = the path ended (a `break` of the reference loop, or depth reached MAX_BOUNCES)
  DEV bool step(Path &ps) {
    if constexpr (SUSP) {
      if (ps.phase == 1) {  // resume this bounce's light sampling
        if (!nee_phase(ps)) return true;
        ps.phase = 0;
        return ps.nc.end ? false : ++ps.depth < C.max_bounces();
      }
    }
    v3 &ro = ps.ro, &rd = ps.rd, &acc = ps.acc, &mask = ps.mask, &prev_nl = ps.prev_nl;
    bool &spec = ps.spec;
    const float seed = ps.seed;
    const int depth = ps.depth;
    const float fr = (float)frame;
    {
    if (COUNT) ++n_iter;
    Hit hit;
    float t = isect(ro, rd, hit, march_slot(ps));
    if ((SUSP || WF || WFB) && t < 0.0f) return true;  // march (or walk) pending: step() repeats this bounce once it is done
    if constexpr (VOL) {
      if (flag(F_VOL)) {
        float sd = -flog(fmaxf(hash(nc_addmul(seed + 4729.3f, (float)depth, 991.1f)), 1e-6f)) / VOL_SIGMA_T;
        if (sd < fminf(INF_T, t)) {
          v3 sp = ro + rd * sd;
          mask = mask * (VOL_SIGMA_S / VOL_SIGMA_T);
          if constexpr (WF) {  // the in-scatter light loop's shadow rays become march jobs
            const v3 rd_in = rd;
            rd = sample_hg(rd, nc_addmul(seed + 8293.7f, (float)depth, 773.3f));
            ro = sp;
            spec = false;
            ++scat_ev;
            const bool stop = scat_ev >= C.max_scatter() || vmaxc(mask) < 0.01f;
            if (flag(F_SAMPLE_LIGHTS)) wf_nee_volume(sp, rd_in, mask, seed, depth);
            return stop ? false : ++ps.depth < C.max_bounces();
          }
          if constexpr (SUSP) {  // the in-scatter NEE becomes phase 1 (it reads sp, the incoming rd and mask)
            const v3 rd_in = rd;
            rd = sample_hg(rd, nc_addmul(seed + 8293.7f, (float)depth, 773.3f));
            ro = sp;
            spec = false;
            ++scat_ev;
            const bool stop = scat_ev >= C.max_scatter() || vmaxc(mask) < 0.01f;
            if (flag(F_SAMPLE_LIGHTS)) {
              ps.nc = NeeCtx{sp, rd_in, mk(0.f, 0.f, 0.f), seed, 0, true, stop};
              ps.phase = 1;
              if (!nee_phase(ps)) return true;
              ps.phase = 0;
            }
            return stop ? false : ++ps.depth < C.max_bounces();
          }
          if (flag(F_SAMPLE_LIGHTS)) {
            for_lights(sc, [&](int li) {
              int lidx = sc.light(li);
              if (lidx < 0) return;
              const GeomRec lg = sc.geom(lidx);
              const MatRec lmt = sc.mat(lidx);
              if (lmt.type != M_LIGHT || lg.type != T_SPHERE) return;
              v3 dlc = mk(lg.px, lg.py, lg.pz) - sp;
              float dc = length(dlc);
              float cam = fsqrt(1.0f - fminf(fmaxf(fdiv(lg.d0, dc * dc), 0.0f), 1.0f));
              float idc = frcp(dc);
              v3 dir = sample_cone(mk(dlc.x * idc, dlc.y * idc, dlc.z * idc), 1.0f - cam,
                                   nc_addmul(nc_addmul(seed + 2341.7f, (float)li, 917.3f), (float)depth, 199.1f));
              if (COUNT) ++n_nee;
              Hit sh;
              float ts = isect(sp + dir * (EPSILON * 20.0f), dir, sh);
              if (sh.index != lidx) return;
              float omega = 2.0f * (1.0f - cam);
              float ct = dot(rd, dir);
              constexpr float g2 = VOL_G * VOL_G;
              float den = 1.0f + g2 - 2.0f * VOL_G * ct;
              float phase = fdiv(1.0f - g2, FOUR_PI * den * fsqrt(den));
              float Tf = fexp(-VOL_SIGMA_T * ts);
              acc = acc + ((((mask * mk(lmt.cr, lmt.cg, lmt.cb)) * mk(lmt.er, lmt.eg, lmt.eb)) * phase) * Tf) *
                              (PI_F * omega);
            });
          }
          rd = sample_hg(rd, nc_addmul(seed + 8293.7f, (float)depth, 773.3f));
          ro = sp;
          spec = false;
          ++scat_ev;
          if (scat_ev >= C.max_scatter() || vmaxc(mask) < 0.01f) {
            if (ghost_on()) ghost_brdf(seed);
            else if (quad_rec()) quad_ghost(seed, depth);
            return false;
          }
          return ++ps.depth < C.max_bounces();
        }
      }
    }
    if (t == INF_T) {
      if (ghost_on()) ghost_brdf(seed);  // 2057 and 2065 both `break`
      else if (quad_rec()) quad_ghost(seed, depth);
      if (!spec && flag(F_SAMPLE_LIGHTS)) return false;
      if (flag(F_CUBEMAP)) {  // 2059-2060 (USE_CUBEMAP wins over the procedural sky)
        const T4 cm = cube_sample(P, rd);
        acc = acc + mask * mk(cm.r, cm.g, cm.b);
      } else if (flag(F_SKY)) {
        float k = fminf(fmaxf(rd.y * 0.6f + 0.5f, 0.3f), 1.0f);
        v3 sky = mk(0.5f + 0.5f * fcos(TWO_PI * (0.525f + 0.9f * k)), 0.5f + 0.5f * fcos(TWO_PI * (0.408f + 0.97f * k)),
                    0.5f + 0.5f * fcos(TWO_PI * (0.409f + 0.8f * k)));
        acc = acc + mask * sky;
      }
      return false;
    }
    const GeomRec g = geom_at(hit.index);
    const MatRec mt = mat_at(hit.index);
    v3 c = mk(mt.cr, mt.cg, mt.cb), e = mk(mt.er, mt.eg, mt.eb);
    // scene-specialised scenes without textures read c and e with their
    // max(., 0.001) clamps applied at compile time (JitScene::mat_shade); the
    // light sampling below still gets the material as the shader passes it
    bool pre = false;
    if constexpr (Scene::kStatic) {
      if constexpr (!Scene::any_tex()) {
        const MatRec ms = mat_shade_at(hit.index);
        c = mk(ms.cr, ms.cg, ms.cb);
        e = mk(ms.er, ms.eg, ms.eb);
        pre = true;
      }
    }
    if (sc.any_tex()) {  // raytracer.glsl:2071, 2077
      const TexRec tr = sc.tex(hit.index);
      if (tr.type >= 0 && (tr.opts & 3u)) {
        const T4 tx = hit_texel(P, tr, hit);
        if (tr.opts & 1u) {
          const float a = tx.a;
          c = mk(mixf(c.x, tx.r * tr.cmr, a), mixf(c.y, tx.g * tr.cmg, a), mixf(c.z, tx.b * tr.cmb, a));
        }
        if (tr.opts & 2u) {
          const float a = tx.a;
          e = mk(mixf(e.x, tx.r * tr.emr, a), mixf(e.y, tx.g * tr.emg, a), mixf(e.z, tx.b * tr.emb, a));
        }
      }
    }
    if (!pre) c = vmaxs(c, 0.001f);
    float inside = -sgn(dot(rd, hit.n));
    if (!pre) e = vmaxs(e, 0.001f);
    if (mt.type == M_LIGHT) {
      mask = mask * c;
      float w = 1.0f;
      if (flag(F_MIS) && !spec && flag(F_SAMPLE_LIGHTS) && depth > 0) {
        v3 ld = normalize(hit.pos - ro);
        w = power_heuristic(cos_pdf(ld, prev_nl), light_pdf(g, mt, ro));
      }
      acc = acc + (mask * e) * w;
      if (ghost_on()) ghost_brdf(seed);
      else if (quad_rec()) quad_ghost(seed, depth);
      return false;
    }
    prev_nl = hit.n * inside;

    // ---- brdf(), 1804-1980
    const v3 x = hit.pos;
    const v3 nl = hit.n * inside;
    const float bounce = (float)depth;
    v3 rdir;
    {
      float s = nc_seed4(seed, 7.1f, fr, 5681.123f, bounce, 92.13f);
      rdir = flag(F_BIASED) ? sample_cosine(nl, s) : sample_cone(nl, 1.0f, s);
    }
    const float ncr = 1.00029f;
    float nt_eff = fabsf(mt.nt);
    if constexpr (SPECTRAL) {
      if (flag(F_SPECTRAL) && mt.nt < 0.0f) nt_eff = spectral_ior(hero, fabsf(mt.nt));
    }
    const int mtype = mt.type;
    if (mtype == M_DIFF) {
      ro = x + nl * EPSILON;
      rd = rdir;
      mask = mask * c;
      ++diff_b;
      spec = false;
    } else if (mtype == M_SPEC) {
      ro = x + nl * EPSILON;
      rd = normalize(e * rdir + reflect(rd, nl));
      mask = mask * c;
      ++spec_b;
      spec = true;
    } else if (mtype == M_REFR_FRESNEL || mtype == M_REFR_SCHLICK) {
      float nnt = inside < 0.0f ? fdiv(nt_eff, ncr) : fdiv(ncr, nt_eff);
      v3 tdir = refract(rd, nl, nnt);
      // total internal reflection: length(tdir) == 0 (raytracer.glsl:1844) as dot(tdir, tdir) == 0
      // -- sqrt(x) == 0 exactly when x == 0 (f32 denormals preserved), one
      // v_sqrt_f32 less per refraction
      if (dot(tdir, tdir) == 0.0f) {
        ro = x + nl * EPSILON;
        rd = normalize(e * rdir + reflect(rd, nl));
        ++spec_b;
        spec = true;
      } else {
        tdir = normalize(e * rdir + tdir);
        float Re = mtype == M_REFR_FRESNEL ? fresnel(rd, nl, ncr, nt_eff, tdir) : schlick(rd, nl, ncr, nt_eff);
        if (hash(seed) < Re) {
          ro = x + nl * EPSILON;
          rd = normalize(e * rdir + reflect(rd, nl));
          ++spec_b;
        } else {
          ro = x - nl * EPSILON;
          mask = mask * c;
          rd = tdir;
          ++scat_ev;
        }
        spec = true;
      }
    } else if (mtype == M_COAT) {
      ro = x + nl * EPSILON;
      if (hash(seed) < schlick(rd, nl, ncr, nt_eff)) {
        rd = normalize(e * rdir + reflect(rd, nl));
        ++spec_b;
        spec = true;
      } else {
        rd = rdir;
        mask = mask * c;
        ++diff_b;
        spec = false;
      }
    }
    if (quad_rec()) {  // brdf()'s registers for a later ghost call (quad_ghost)
      gr_have = true;
      gr_nl = nl;
      gr_rd = rd;
      gr_spec = spec;
      gr_mat = hit.index;
    }
    if (!spec && flag(F_CUBEMAP)) {  // environment NEE, 1887-1897
      const float s = nc_addmul(seed, bounce, 965.325f);
      const v3 sr = flag(F_BIASED) ? sample_cosine(nl, s) : sample_cone(nl, 1.0f, s);
      Hit eh;
      if (isect(x + nl * EPSILON, sr, eh) == INF_T) {
        const T4 cm = cube_sample(P, sr);
        acc = acc + mask * mk(cm.r, cm.g, cm.b);
      }
    }
    if constexpr (WF) {  // light sampling's shadow rays become march jobs; the end tests do not depend on them
      const bool end = vmaxc(mask) < 0.01f || diff_b >= C.max_diff() || spec_b >= C.max_spec() || 0 >= C.max_trans() ||
                       scat_ev >= C.max_scatter();
      if (!spec && flag(F_SAMPLE_LIGHTS)) wf_nee_surface(x, nl, seed, bounce);
      return end ? false : ++ps.depth < C.max_bounces();
    }
    if constexpr (SUSP) {  // light sampling becomes phase 1; the end tests below do not depend on it
      const bool end = vmaxc(mask) < 0.01f || diff_b >= C.max_diff() || spec_b >= C.max_spec() || 0 >= C.max_trans() ||
                       scat_ev >= C.max_scatter();
      if (!spec && flag(F_SAMPLE_LIGHTS)) {
        ps.nc = NeeCtx{x, nl, mk(0.f, 0.f, 0.f), nc_seed4(seed, 8652.1f, fr, 5681.123f, bounce, 7895.13f), 0, false, end};
        ps.phase = 1;
        if (!nee_phase(ps)) return true;
        ps.phase = 0;
      }
      return end ? false : ++ps.depth < C.max_bounces();
    }
    if (!spec && flag(F_SAMPLE_LIGHTS)) {
      if constexpr (RT0_DEFER_NEE && RESTIR && !COUNT) {
        if (restir_routed()) defer_nee(x, nl, hit.index, seed, bounce, mask);
        else acc = acc + sample_lights(x, nl, mt, seed, bounce) * mask;
      } else {
        acc = acc + sample_lights(x, nl, mt, seed, bounce) * mask;
      }
    }
    // ---- end brdf
    if (ghost_on()) {
      gr_have = true;
      gr_x = x;
      gr_nl = nl;
      gr_rd = rd;
      gr_spec = spec;
      gr_bounce = bounce;
      gr_mat = hit.index;
    }

    if (vmaxc(mask) < 0.01f) return false;
    if (diff_b >= C.max_diff() || spec_b >= C.max_spec() || 0 >= C.max_trans() || scat_ev >= C.max_scatter()) return false;
    }
    return ++ps.depth < C.max_bounces();
  }

  DEV v3 radiance(v3 ro, v3 rd, float seed) {
    Path ps{ro, rd, mk(0.f, 0.f, 0.f), mk(1.f, 1.f, 1.f), mk(0.f, 1.f, 0.f), seed, 0, true};
    if (C.max_bounces() > 0)
      while (step(ps)) {
        if constexpr (SUSP) march_pending(ps);
      }
    return ps.acc;
  }

  // main() up to radiance(), raytracer.glsl:2111-2150: seed, hero wavelength
  // and the camera ray of pixel (px, py) at `frame`
  // the pixel's seed for `frame`, raytracer.glsl:2120 (fcx, fcy set)
  DEV float pixel_seed() const {
#pragma clang fp contract(off)
    return hash(((fcx * 12.9898f) + (fcy * 78.233f)) + (1113.1f * (float)frame));
  }
  // a deferred sampleLightsReSTIR call's two seeds (1909/1943), as defer_nee's
  // path computed them: from the pixel's seed, the pass and the bounce
  DEV void restir_seeds(int bounce, float &sx, float &sy) const {
    const float seed = pixel_seed(), fr = (float)frame, b = (float)bounce;
    sx = nc_seed3(seed, 8652.1f, fr, b, 7895.13f);
    sy = nc_seed3(seed, 1234.567f, fr, b, 9876.54f);
  }
  // the pixel's gl_FragCoord and the camera offset that depends on it alone
  // (once per pixel: path regeneration starts its samples with begin_sample)
  DEV void set_pixel(int px, int py) {
    q_px = px;
    q_py = py;
    fcx = (float)px + 0.5f;
    fcy = (float)py + 0.5f;
    stx = 2.0f * fcx / P.res_x - 1.0f;
    sty = 2.0f * fcy / P.res_y - 1.0f;
  }
  DEV void begin(Path &ps, int px, int py) {
    set_pixel(px, py);
    begin_sample(ps);
  }
  // main()'s camera ray of this pixel and `frame` (raytracer.glsl:2118-2150)
  DEV void begin_sample(Path &ps) {
    diff_b = spec_b = scat_ev = 0;
    const float seed = pixel_seed();
    hero = 550.0f;
    if constexpr (SPECTRAL) {
      if (flag(F_SPECTRAL)) hero = nc_addmul(380.0f, hash(seed + 4821.73f), 340.0f);
    }
    const v3 u = mk(P.ux, P.uy, P.uz), v = mk(P.vx, P.vy, P.vz), w = mk(P.wx, P.wy, P.wz);
    const float ax = hash(seed + 13.271f), ay = hash(seed + 63.216f);
    const float flx = step_(0.5f, ax), fly = step_(0.5f, ay);
    const float hx = mixf(ax, 1.0f - ax, flx), hy = mixf(ay, 1.0f - ay, fly);
    const float sx = fsqrt(2.0f * hx), sy = fsqrt(2.0f * hy);
    // x * (1/(res/2)): the reciprocal is per launch (hoisted), the division it
    // replaces was a ~10-instruction correctly rounded expansion per sample
    // (ulp-level, like the contracted geometry; 5.59 vs 5.80 ms per C2 launch)
    const float dx = mixf(sx - 1.0f, 1.0f - sx, flx) * (1.0f / (P.res_x * 0.5f)) + stx;
    const float dy = mixf(sy - 1.0f, 1.0f - sy, fly) * (1.0f / (P.res_y * 0.5f)) + sty;
    const v3 fp = normalize(((u * dx) * P.uULen + (v * dy) * P.uVLen) + w) * P.focal;
    v3 ro = mk(P.cam_px, P.cam_py, P.cam_pz), rd;
    if (P.aperture != 0.0f) {
      const float ang = hash(seed + 496.4562f);  // revolutions
      const float rad = hash(seed + 249.1686f) * P.aperture;
      const v3 ap = (u * fcos_rev(ang) + v * fsin_rev(ang)) * rad;
      ro = ro + ap;
      rd = normalize(fp - ap);
    } else {
      rd = normalize(fp);  // aperture 0: randomAperturePos == 0 exactly
    }
    if (RESTIR) {
      fin = empty_res();
      gr_have = false;
      nee_k = 0;
    }
    quad_begin();
    ps = Path{ro, rd, mk(0.f, 0.f, 0.f), mk(1.f, 1.f, 1.f), mk(0.f, 1.f, 0.f), seed, 0, true};
  }
  // main() after radiance(): the spectral weighting (2152-2155)
  DEV v3 finish(const Path &ps) {
    v3 col = ps.acc;
    if constexpr (SPECTRAL) {
      if (flag(F_SPECTRAL)) col = col * wavelength_to_rgb(hero);
    }
    return col;
  }
  // main(), raytracer.glsl:2111-2180: one sample of pixel (px, py) at `frame`
  DEV v3 sample(int px, int py) {
    Path ps;
    begin(ps, px, py);
    if (C.max_bounces() > 0)
      while (step(ps)) {
        if constexpr (SUSP) march_pending(ps);
      }
    return finish(ps);
  }
};

// Row-band sharding: launch row `r` of the band-compressed grid maps to image
// row (r/band * n_shards + shard) * band + r % band.
DEV int image_row(const LaunchParams &P, int r) {
  const int b = r / P.band;
  return (b * P.n_shards + P.shard) * P.band + (r - b * P.band);
}

// accumulator update of one sample: prev + sample (raytracer.glsl:2168) or, in
// RENDER_MODE 1, mix(previousFrame, currentFrame, 1/u_temporalFrames) (2159-2165)
template <class It>
DEV void accumulate(const It &it, const LaunchParams &P, float4 &a, v3 s) {
  if (it.flag(F_ANIM)) {
    a.x = mixf(a.x, s.x, P.ema_alpha);
    a.y = mixf(a.y, s.y, P.ema_alpha);
    a.z = mixf(a.z, s.z, P.ema_alpha);
  } else {
#pragma clang fp contract(off)
    a.x += (s.x);
    a.y += (s.y);
    a.z += (s.z);
  }
}

// Frame-chunked scratch: one plane per frame covering only the launch's
// rectangle (viewport x band rows), indexed relative to its corner.
DEV size_t sample_plane(const LaunchParams &P) { return (size_t)(P.vp_x1 - P.vp_x0) * (P.vp_y1 - P.vp_y0); }
DEV size_t sample_index(const LaunchParams &P, int px, int r) {
  return (size_t)(r - P.vp_y0) * (P.vp_x1 - P.vp_x0) + (px - P.vp_x0);
}

// The pass kernel body: 16x16 pixel tile per 256-thread workgroup (four 8x8
// wave tiles); each lane accumulates its pixel's passes in registers.
// (XCD-aware tile orders -- whole bands or interleaved runs of tiles per XCD
// -- were measured and lost or tied, DESIGN 4.7: blockIdx maps straight to
// the tile.)

// Path regeneration: the lane runs its pixel's passes back to back as ONE
// loop of bounce steps; when its path ends it accumulates the sample and
// starts the next pass at once instead of idling until the longest path of
// its wave has finished.  Each pixel's samples are still produced and summed
// in pass order, so the result is bit-identical to the plain loop.
template <class It, class Cfg>
DEV void regen_pixel(const LaunchParams &P, It &it, const Cfg &cfg, int px, int py, size_t apix) {
  float4 a = P.accum[apix];
  if (P.nframes > 0) {
    typename It::Path ps;
    int f = 0;
    it.frame = P.frame0;
    it.begin(ps, px, py);
    bool alive = cfg.max_bounces() > 0;
    while (true) {
      // a lane whose march is still pending skips step() (its bounce resumes once it is done)
      if (alive && !(It::SUSP && ps.ms.active)) alive = it.step(ps);
      if (!alive) {
        accumulate(it, P, a, it.finish(ps));
        it.quad_store();  // (rule 11's recording launch: one frame)
        if (++f >= P.nframes) break;
        it.frame = P.frame0 + (uint32_t)f;
        it.begin_sample(ps);  // same pixel: set_pixel's values stand
        alive = cfg.max_bounces() > 0;
      }
      if constexpr (It::SUSP) it.march_pending(ps);
    }
  }
  P.accum[apix] = a;
}

template <class Scene, class Cfg, bool RESTIR, bool VOL, bool SDF, bool SPECTRAL, bool COUNT>
DEV void pass_body(const LaunchParams &P, Scene sc, Cfg cfg) {
  treelet_load(P);
  // (a wavefront module parks pending marches for its march kernel: its SDF
  // paths cannot run here)
  static_assert(!Integrator<Scene, Cfg, RESTIR, VOL, SDF, SPECTRAL, COUNT>::WF &&
                    !Integrator<Scene, Cfg, RESTIR, VOL, SDF, SPECTRAL, COUNT>::WFB,
                "RT0_WAVEFRONT modules render through wf_shade_body / wf_restir_shade_body");
  const SceneTables tabs = scene_tables(sc);  // (before any thread leaves: one barrier)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lx = (lane & 7) + ((wave & 1) << 3);
  const int ly = (lane >> 3) + ((wave >> 1) << 3);
  const int px = P.vp_x0 + (int)blockIdx.x * 16 + lx;
  const int r = P.vp_y0 + (int)blockIdx.y * 16 + ly;
  if (px >= P.vp_x1 || r >= P.vp_y1) return;
  const int py = image_row(P, r);
  if (py >= P.height) return;
  Integrator<Scene, Cfg, RESTIR, VOL, SDF, SPECTRAL, COUNT> it(P, sc, cfg);
  it.use_tables(tabs);
  const size_t pix = (size_t)py * P.width + px;                        // image pixel (ReSTIR planes)
  const size_t apix = P.compact ? (size_t)r * P.width + px : pix;      // accumulator pixel
  if (!RESTIR && P.samples) {  // frame-chunked: samples out, rt0_sum_kernel accumulates
    const int f0 = (int)blockIdx.z * P.frame_chunk;
    const int f1 = min(P.nframes, f0 + P.frame_chunk);
    const size_t plane = sample_plane(P), lp = sample_index(P, px, r);
    for (int f = f0; f < f1; ++f) {
      it.frame = P.frame0 + (uint32_t)f;
      v3 s = it.sample(px, py);
      P.samples[(size_t)f * plane + lp] = make_float4(s.x, s.y, s.z, 0.f);
    }
  } else if constexpr (!RESTIR && !COUNT) {
    regen_pixel(P, it, cfg, px, py, apix);
  } else if constexpr (RT0_DEFER_NEE && RESTIR && !COUNT) {
    // the path without its deferred sampleLightsReSTIR calls; rt0_jit_resolve
    // completes the sample and accumulates it
    it.frame = P.frame0;
    it.nee_pix = (int32_t)pix;
    it.nee_wave = (blockIdx.y * gridDim.x + blockIdx.x) * 4u + (uint32_t)wave;
    volatile uint32_t *wc = nee_wave_counter();
    *wc = 0u;  // every active lane stores the same 0 before the wave's first append
    typename decltype(it)::Path ps;
    it.begin(ps, px, py);
    if (cfg.max_bounces() > 0)
      while (it.step(ps)) {
      }
    // the wave has reconverged: every append is in the counter
    const uint32_t total = *wc;
    if (lane == __ffsll((long long)__ballot(1)) - 1) P.nee_count[it.nee_wave] = total;
    P.nee_partial[pix] = make_float4(ps.acc.x, ps.acc.y, ps.acc.z, it.hero);
    P.nee_n[pix] = it.nee_k;
    if (it.nee_k > 0) return;  // g_final_reservoir is the last deferred call's: rt0_jit_nee writes it
  } else {
    float4 a = P.accum[apix];
    for (int f = 0; f < P.nframes; ++f) {
      it.frame = P.frame0 + (uint32_t)f;
      accumulate(it, P, a, it.sample(px, py));
    }
    P.accum[apix] = a;
  }
  if constexpr (RESTIR) {
    if (P.rout_main == nullptr || P.rout_aux == nullptr) return;
    if (it.flag(F_RESTIR_DEF)) {
      const Res &q = it.fin;
      P.rout_main[RT0_RES_STRIDE * (size_t)pix] = make_float4(q.pos.x, q.pos.y, q.pos.z, q.W);
      P.rout_aux[RT0_RES_STRIDE * (size_t)pix] = make_float4(q.col.x, q.col.y, q.col.z, pack_alpha(q.age, q.M, q.idx, sc.n_lights()));
    } else {
      P.rout_main[RT0_RES_STRIDE * (size_t)pix] = make_float4(0.f, 0.f, 0.f, 0.f);
      P.rout_aux[RT0_RES_STRIDE * (size_t)pix] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if constexpr (COUNT) {
    atomicAdd(&P.counters[0], it.n_isect);
    atomicAdd(&P.counters[1], it.n_iter);
    atomicAdd(&P.counters[2], it.n_nee);
    atomicAdd(&P.counters[3], it.n_map);
    atomicAdd(&P.counters[4], (unsigned long long)P.nframes);
    atomicAdd(&P.counters[5], it.n_restir);
    atomicAdd(&P.counters[6], it.n_cand);
    atomicAdd(&P.counters[7], it.n_ttap);
    atomicAdd(&P.counters[8], it.n_stap);
    atomicAdd(&P.counters[9], it.n_bvh[0]);
    atomicAdd(&P.counters[10], it.n_bvh[1]);
  }
}

// The deferred sampleLightsReSTIR calls of one pass (rt0_jit_nee): each wave
// takes one pass wave's region 64 records at a time, so the candidates,
// reservoir taps and visibility rays run on full waves whatever the paths'
// lengths.  Same arguments, same arithmetic as the inline call;
// the last call of a pixel writes its reservoir MRTs (g_final_reservoir,
// raytracer.glsl:2171-2174).
// The ReSTIR candidates' light data in LDS (scene-specialised, non-animated
// scenes): per light slot k, (pos, c*e, the mesh index or -1 if the slot is
// skipped) in two float4s, written by the workgroup's first threads before
// its one barrier.  A candidate's light is picked per lane at random, so the
// scene-table reads are two dependent per-lane loads (light_index[k], then
// the mesh's geometry and material) for each of the up to 16 candidates of a
// call; from LDS it is one short round trip (raytracer.glsl:1633-1650).
// Returns null where the tables are read as before.
template <class Scene, class Cfg>
DEV const float4 *candidate_table(const Scene &sc, const Cfg &cfg) {
  if constexpr (Scene::kStatic && Scene::kLights > 0) {
    if constexpr ((Cfg::flags() & F_ANIM) == 0u) {
      __shared__ float4 cand[2 * Scene::kLights];
      for (int k = (int)threadIdx.x; k < Scene::kLights; k += (int)blockDim.x) {
        const int li = sc.light(k);
        const bool ok = li >= 0 && li < sc.n_meshes() + sc.n_sdfs();
        const GeomRec lg = sc.geom(ok ? li : 0);
        const MatRec lmt = sc.mat(ok ? li : 0);
        const v3 lc = mk(lmt.cr, lmt.cg, lmt.cb) * mk(lmt.er, lmt.eg, lmt.eb);
        cand[2 * k] = make_float4(lg.px, lg.py, lg.pz, lc.x);
        cand[2 * k + 1] = make_float4(lc.y, lc.z, __int_as_float(ok ? li : -1), 0.f);
      }
      __syncthreads();
      return cand;
    }
  }
  (void)sc;
  (void)cfg;
  return nullptr;
}

#ifndef RT0_FUSED_RESOLVE  // rt0_jit_nee completes its pixels' samples (no rt0_jit_resolve; no walk kernel)
#define RT0_FUSED_RESOLVE 0
#endif
template <class Cfg, bool SPECTRAL>
DEV void resolve_pixel(const LaunchParams &P, const Cfg &cfg, int px, int r);

template <class Scene, class Cfg, bool VOL, bool SDF, bool SPECTRAL>
DEV void nee_body(const LaunchParams &P, Scene sc, Cfg cfg) {
  treelet_load(P);
  // one wave per RT0_NEE_REGIONS consecutive regions: their records form one
  // list, so a region's tail chunk does not idle most of a wave (C5 averages
  // ~68 records per region: one region per wave ran a 64-record chunk and a
  // 4-record chunk).  Measured 1 / 2 / 4 / 8 regions: C3 5326 / 5491 / 4627 /
  // 3320, C5 1467 / 1558 / 1513 / 1403 Msamples/s (profiles/r03/defer/)
  const float4 *cand = candidate_table(sc, cfg);
  const SceneTables tabs = scene_tables(sc);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4u + (threadIdx.x >> 6))) *
                      RT0_NEE_REGIONS;
  if (r0 >= (uint32_t)P.nee_regions) return;
  uint32_t cnt[RT0_NEE_REGIONS], total = 0;
#pragma unroll
  for (int q = 0; q < RT0_NEE_REGIONS; ++q) {
    cnt[q] = r0 + q < (uint32_t)P.nee_regions ? min(P.nee_count[r0 + q], (uint32_t)P.nee_cap) : 0u;
    total += cnt[q];
  }
  const size_t plane = (size_t)P.width * P.height;
  using It = Integrator<Scene, Cfg, true, VOL, SDF, SPECTRAL, false>;
  // list position i -> the record's slot in its pass wave's region
  auto slot_of = [&](uint32_t i) -> size_t {
    uint32_t q = 0, off = i;
#pragma unroll
    for (int k = 0; k < RT0_NEE_REGIONS - 1; ++k)
      if (q == (uint32_t)k && off >= cnt[k]) {
        off -= cnt[k];
        q = k + 1;
      }
    return (size_t)(r0 + q) * (uint32_t)P.nee_cap + off;
  };
  auto setup = [&](It &it, const NeeRec &r) {
    it.cand_lds = cand;
    it.use_tables(tabs);
    it.frame = P.frame0;
    const int py = r.pix / P.width, px = r.pix - py * P.width;
    it.fcx = (float)px + 0.5f;
    it.fcy = (float)py + 0.5f;
    it.fin = empty_res();
    it.gr_have = false;
  };
  // the call's result x mask; the pixel's last call writes g_final_reservoir
  auto store = [&](const NeeRec &r, v3 c, const Res &q) {
    P.nee_out[(size_t)r.k() * plane + r.pix] = make_float4(c.x * r.mr, c.y * r.mg, c.z * r.mb, 0.f);
    if (r.k() == P.nee_n[r.pix] - 1 && P.rout_main != nullptr && P.rout_aux != nullptr) {
      P.rout_main[RT0_RES_STRIDE * (size_t)r.pix] = make_float4(q.pos.x, q.pos.y, q.pos.z, q.W);
      P.rout_aux[RT0_RES_STRIDE * (size_t)r.pix] = make_float4(q.col.x, q.col.y, q.col.z, pack_alpha(q.age, q.M, q.idx, sc.n_lights()));
    }
  };
#if RT0_NEE_WALK
  // the calls' triangle occlusion queries become this wave's walk jobs,
  // appended densely in record order (wave-wide ballots, no atomics)
  WalkJob *wj = P.walk_jobs + (size_t)(r0 / RT0_NEE_REGIONS) * (2u * RT0_NEE_REGIONS * (uint32_t)P.nee_cap);
  uint32_t njob = 0;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (uint32_t base = 0; base < total; base += 64u) {  // wave-uniform trip count
    const uint32_t i = base + lane;
    bool has0 = false, has1 = false;
    WalkJob j0, j1;
    if (i < total) {
      const size_t slot = slot_of(i);
      const NeeRec r = P.nee_rec[slot];
      It it(P, sc, cfg);
      setup(it, r);
      float sx, sy;
      it.restir_seeds(r.bounce(), sx, sy);
      const auto sp = it.restir_split(mk(r.x, r.y, r.z), mk(r.nx, r.ny, r.nz), it.mat_at(r.mat()), sx, sy);
      if (sp.done) {
        store(r, sp.c, it.fin);
      } else {
        // the result as it is if both rays pass, tagged for rt0_jit_resolve; the
        // pixel's last call writes the reservoir MRTs with W as if visible
        // (resolve zeroes W when the visibility ray is blocked).  A ray that
        // misses the model's root boxes is answered here (not occluded).
        bool w0 = sp.has[0], w1 = sp.has[1];
        if constexpr (RT0_WALK_ROOT_TEST) {
          auto miss = [&](const WalkJob &j) {
            return bvh_root_miss(P, mk(j.ox, j.oy, j.oz), mk(frcp(j.dx), frcp(j.dy), frcp(j.dz)), j.tmax);
          };
          w0 = w0 && !miss(sp.j[0]);
          w1 = w1 && !miss(sp.j[1]);
        }
        const int tag = (w0 || w1) ? (int)(((uint32_t)slot + 1u) << 2) | (w0 ? 1 : 0) | (w1 ? 2 : 0) : 0;
        P.nee_out[(size_t)r.k() * plane + r.pix] =
            make_float4(sp.f.x * r.mr, sp.f.y * r.mg, sp.f.z * r.mb, __int_as_float(tag));
        if (r.k() == P.nee_n[r.pix] - 1 && P.rout_main != nullptr && P.rout_aux != nullptr) {
          const Res &q = it.fin;
          P.rout_main[RT0_RES_STRIDE * (size_t)r.pix] = make_float4(q.pos.x, q.pos.y, q.pos.z, sp.W);
          P.rout_aux[RT0_RES_STRIDE * (size_t)r.pix] = make_float4(q.col.x, q.col.y, q.col.z, pack_alpha(q.age, q.M, q.idx, sc.n_lights()));
        }
        has0 = w0;
        has1 = w1;
        j0 = sp.j[0];
        j1 = sp.j[1];
        j0.slot2 = 2u * (uint32_t)slot;
        j1.slot2 = 2u * (uint32_t)slot + 1u;
      }
    }
    const uint64_t b0 = __ballot(has0), b1 = __ballot(has1);
    const uint32_t n0 = (uint32_t)__popcll(b0);
    if (has0) wj[njob + (uint32_t)__popcll(b0 & lt)] = j0;
    if (has1) wj[njob + n0 + (uint32_t)__popcll(b1 & lt)] = j1;
    njob += n0 + (uint32_t)__popcll(b1);
  }
  if (lane == 0) P.walk_count[r0 / RT0_NEE_REGIONS] = njob;
#else
  for (uint32_t i = threadIdx.x & 63u; i < total; i += 64u) {
    const NeeRec r = P.nee_rec[slot_of(i)];
    It it(P, sc, cfg);
    setup(it, r);
    float sx, sy;
    it.restir_seeds(r.bounce(), sx, sy);
    const v3 c = it.restir(mk(r.x, r.y, r.z), mk(r.nx, r.ny, r.nz), it.mat_at(r.mat()), sx, sy);
    store(r, c, it.fin);
  }
#if RT0_FUSED_RESOLVE
  // Every call of this wave's regions is stored, and a region holds every
  // call of its pass wave's 64 pixels: the wave completes those pixels'
  // samples itself (resolve_pixel, rt0_jit_resolve's arithmetic) instead of a
  // resolve launch.  The stores were this wave's own (one L1): a
  // workgroup-scope fence orders them before the loads.
  __threadfence_block();
  const int lane = (int)(threadIdx.x & 63u), gx = (P.vp_x1 - P.vp_x0 + 15) / 16;
#pragma unroll
  for (int q = 0; q < RT0_NEE_REGIONS; ++q) {
    const uint32_t rg = r0 + (uint32_t)q;  // pass wave (blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave
    if (rg >= (uint32_t)P.nee_regions) break;
    const int b = (int)(rg >> 2), wv = (int)(rg & 3u), bx = b % gx, by = b / gx;
    resolve_pixel<Cfg, SPECTRAL>(P, cfg, P.vp_x0 + bx * 16 + (lane & 7) + ((wv & 1) << 3),
                                 P.vp_y0 + by * 16 + (lane >> 3) + ((wv >> 1) << 3));
  }
#endif
#endif
}

#if RT0_NEE_WALK
// rt0_jit_walk: the triangle occlusion queries of one light-sampling wave's
// calls (WalkJobs, bvh_closest<true>'s walk), with lanes that stay busy: a
// lane whose ray is answered takes the wave's next job (an LDS counter), so
// the wave walks on full lanes until its list runs dry instead of waiting for
// its longest ray every 64 jobs.  One node (two child boxes) per iteration.
// RT0_WALK_SPEC: walk_body with the leaf tests postponed (speculative
// while-while traversal, Aila & Laine 2009): a lane whose node visit finds
// leaf triangles keeps them pending and the wave tests pending leaves only
// once half its busy lanes hold some (or every busy lane does), so the
// triangle tests run on many lanes at once instead of splitting every
// iteration into node lanes and leaf lanes.  An occlusion answer is a set
// property (some triangle in (EPSILON, tmax)): the visiting order does not
// change it.
DEV void walk_body_spec(const LaunchParams &P) {
  treelet_load(P);
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4u + (threadIdx.x >> 6)));
  if (w >= (uint32_t)P.walk_waves) return;
  const uint32_t n = P.walk_count[w];
  const WalkJob *__restrict__ jobs = P.walk_jobs + (size_t)w * (2u * RT0_NEE_REGIONS * (uint32_t)P.nee_cap);
  uint32_t *ctr = nee_wave_counter();
  *(volatile uint32_t *)ctr = 64u;  // every lane stores the same value: jobs 0..63 go by lane index
  const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(P.bvh);
  const TriDev *__restrict__ tris = P.tris;
  BvhStack stk;
  uint32_t j = threadIdx.x & 63u;
  bool have = false;
  v3 o = mk(0.f, 0.f, 0.f), d = o, inv = o;
  float tmax = 0.f;
  uint32_t slot2 = 0;
  int node = 0, sp = 0, guard = 0, pa = -1, pb = -1;  // node -1: traversal over; pa/pb: pending leaves
  auto load = [&]() {
    have = j < n;
    if (have) {
      const WalkJob jb = jobs[j];
      o = mk(jb.ox, jb.oy, jb.oz);
      d = mk(jb.dx, jb.dy, jb.dz);
      inv = mk(frcp(d.x), frcp(d.y), frcp(d.z));
      tmax = jb.tmax;
      slot2 = jb.slot2;
      node = 0;
      sp = 0;
      guard = 0;  // (stale stack entries are never read: sp restarts at 0)
      pa = pb = -1;
    }
  };
  load();
  while (__ballot(have) != 0ull) {
    // node phase: lanes without pending leaves visit their next node
    if (have && pa < 0 && node >= 0) {
      float4 a, b, c;
      int4 lk;
      bvh_fetch(P, nodes, node, a, b, c, lk);
      float tl = box_enter(a.x, a.y, a.z, b.x, b.y, b.z, o, inv, tmax);
      float tr = box_enter(a.w, b.w, c.x, c.y, c.z, c.w, o, inv, tmax);
      const int cl = lk.x, cr = lk.y;
      if (tl != F_INF && cl < 0) {
        pa = ~cl;
        tl = F_INF;
      }
      if (tr != F_INF && cr < 0) {
        if (pa < 0) pa = ~cr;
        else pb = ~cr;
        tr = F_INF;
      }
      if (tl != F_INF && tr != F_INF) {
        const bool lfirst = tl <= tr;
        stk.put(sp, lfirst ? cr : cl);
        sp = min(sp + 1, RT0_BVH_STACK - 1);  // the build guarantees depth < RT0_BVH_STACK
        node = lfirst ? cl : cr;
      } else if (tl != F_INF) {
        node = cl;
      } else if (tr != F_INF) {
        node = cr;
      } else if (sp == 0) {
        node = -1;
      } else {
        node = stk.get(--sp);
      }
      // a ray visits each node at most once: the cap only guarantees that
      // every wave drains even on a corrupt tree
      if (++guard > 2 * P.n_tris + 8) node = -1;
    }
    // leaf phase: once half the busy lanes hold leaves, or no busy lane can
    // visit a node without testing its leaves first
    const uint64_t busy = __ballot(have), lf = __ballot(have && pa >= 0),
                   stuck = __ballot(have && (pa >= 0 || node < 0));
    bool occ = false;
    if ((2 * __popcll(lf) >= __popcll(busy) || stuck == busy) && have && pa >= 0) {
      float t;
      occ = tri_test(tris[pa], o, d, tmax, t) || (pb >= 0 && tri_test(tris[pb], o, d, tmax, t));
      pa = pb = -1;
    }
    if (have && (occ || (pa < 0 && node < 0))) {
      P.walk_res[slot2] = occ ? 1u : 0u;
      j = atomicAdd(ctr, 1u);
      load();
    }
  }
}

DEV void walk_body(const LaunchParams &P) {
#if RT0_WALK_SPEC
  walk_body_spec(P);
#else
  treelet_load(P);
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4u + (threadIdx.x >> 6)));
  if (w >= (uint32_t)P.walk_waves) return;
  const uint32_t n = P.walk_count[w];
  const WalkJob *__restrict__ jobs = P.walk_jobs + (size_t)w * (2u * RT0_NEE_REGIONS * (uint32_t)P.nee_cap);
  uint32_t *ctr = nee_wave_counter();
  *(volatile uint32_t *)ctr = 64u;  // every lane stores the same value: jobs 0..63 go by lane index
  const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(P.bvh);
  const TriDev *__restrict__ tris = P.tris;
  BvhStack stk;
  uint32_t j = threadIdx.x & 63u;
  bool have = j < n;
  v3 o = mk(0.f, 0.f, 0.f), d = o, inv = o;
  float tmax = 0.f;
  uint32_t slot2 = 0;
  int node = 0, sp = 0, guard = 0;
  if (have) {
    const WalkJob jb = jobs[j];
    o = mk(jb.ox, jb.oy, jb.oz);
    d = mk(jb.dx, jb.dy, jb.dz);
    inv = mk(frcp(d.x), frcp(d.y), frcp(d.z));
    tmax = jb.tmax;
    slot2 = jb.slot2;
  }
  while (__ballot(have) != 0ull) {
    if (have) {
      bool done = false, occ = false;
      float4 a, b, c;
      int4 lk;
      bvh_fetch(P, nodes, node, a, b, c, lk);
      float tl = box_enter(a.x, a.y, a.z, b.x, b.y, b.z, o, inv, tmax);
      float tr = box_enter(a.w, b.w, c.x, c.y, c.z, c.w, o, inv, tmax);
      const int cl = lk.x, cr = lk.y;
      int l0 = -1, l1 = -1;
      if (tl != F_INF && cl < 0) {
        l0 = ~cl;
        tl = F_INF;
      }
      if (tr != F_INF && cr < 0) {
        if (l0 < 0) l0 = ~cr;
        else l1 = ~cr;
        tr = F_INF;
      }
      if (l0 >= 0) {
        float t;
        occ = tri_test(tris[l0], o, d, tmax, t) || (l1 >= 0 && tri_test(tris[l1], o, d, tmax, t));
      }
      if (occ) {
        done = true;
      } else if (tl != F_INF && tr != F_INF) {
        const bool lfirst = tl <= tr;
        stk.put(sp, lfirst ? cr : cl);
        sp = min(sp + 1, RT0_BVH_STACK - 1);  // the build guarantees depth < RT0_BVH_STACK
        node = lfirst ? cl : cr;
      } else if (tl != F_INF) {
        node = cl;
      } else if (tr != F_INF) {
        node = cr;
      } else if (sp == 0) {
        done = true;
      } else {
        node = stk.get(--sp);
      }
      // a ray visits each node at most once: the cap only guarantees that
      // every wave drains even on a corrupt tree
      if (++guard > 2 * P.n_tris + 8) done = true;
      if (done) {
        P.walk_res[slot2] = occ ? 1u : 0u;
        j = atomicAdd(ctr, 1u);
        have = j < n;
        if (have) {
          const WalkJob jb = jobs[j];
          o = mk(jb.ox, jb.oy, jb.oz);
          d = mk(jb.dx, jb.dy, jb.dz);
          inv = mk(frcp(d.x), frcp(d.y), frcp(d.z));
          tmax = jb.tmax;
          slot2 = jb.slot2;
          node = 0;
          sp = 0;
          guard = 0;  // (stale stack entries are never read: sp restarts at 0)
        }
      }
    }
  }
#endif
}

#endif

// Completes the samples of a deferred pass (rt0_jit_resolve): the path's own
// radiance plus its light-sampling results in call order, main()'s spectral
// weighting (2152-2155), then the accumulator (2157-2169).  Same tile grid as
// pass_body.
// (one pixel: launch column px, launch row r)
template <class Cfg, bool SPECTRAL>
DEV void resolve_pixel(const LaunchParams &P, const Cfg &cfg, int px, int r) {
  if (px >= P.vp_x1 || r >= P.vp_y1) return;
  const int py = image_row(P, r);
  if (py >= P.height) return;
  const size_t pix = (size_t)py * P.width + px;
  const size_t apix = P.compact ? (size_t)r * P.width + px : pix;
  const size_t plane = (size_t)P.width * P.height;
  const float4 part = P.nee_partial[pix];
  const int n = P.nee_n[pix];
  v3 col = mk(part.x, part.y, part.z);
  // every call's result is loaded before the first is added: the loads are
  // independent, so a pixel waits one round trip for its calls instead of n
  // (the kernel waited on memory 93% of its cycles, loading them one by one)
  constexpr int K = Cfg::max_bounces() < 16 ? Cfg::max_bounces() : 16;
  float4 res[K > 0 ? K : 1];
#pragma unroll
  for (int k = 0; k < K; ++k) res[k] = k < n ? P.nee_out[(size_t)k * plane + pix] : make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](int k, float4 o) {
#if RT0_NEE_WALK
    if (const uint32_t tag = (uint32_t)__float_as_int(o.w)) {
      // a call rt0_jit_nee left to the walks: its result counts if both rays
      // passed; a blocked visibility ray makes the last call's W 0
      // (finalizeReservoir, 1541-1545)
      const size_t slot2 = 2u * (size_t)((tag >> 2) - 1u);
      const bool vis = !(tag & 1u) || P.walk_res[slot2] == 0u;
      if (!(vis && (!(tag & 2u) || P.walk_res[slot2 + 1] == 0u))) o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!vis && k == n - 1 && P.rout_main != nullptr) P.rout_main[RT0_RES_STRIDE * (size_t)pix].w = 0.0f;
    }
#endif
    col = col + mk(o.x, o.y, o.z);
  };
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k < n) add(k, res[k]);  // (constant indices: the results stay in registers)
  for (int k = K; k < n; ++k) add(k, P.nee_out[(size_t)k * plane + pix]);
  if constexpr (SPECTRAL) {
    if (cfg.flags() & F_SPECTRAL) col = col * wavelength_to_rgb(part.w);
  }
  float4 a = P.accum[apix];
  if (cfg.flags() & F_ANIM) {
    a.x = mixf(a.x, col.x, P.ema_alpha);
    a.y = mixf(a.y, col.y, P.ema_alpha);
    a.z = mixf(a.z, col.z, P.ema_alpha);
  } else {
#pragma clang fp contract(off)
    a.x += col.x;
    a.y += col.y;
    a.z += col.z;
  }
  P.accum[apix] = a;
}
template <class Scene, class Cfg, bool SPECTRAL>
DEV void resolve_body(const LaunchParams &P, Scene, Cfg cfg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  resolve_pixel<Cfg, SPECTRAL>(P, cfg, P.vp_x0 + (int)blockIdx.x * 16 + (lane & 7) + ((wave & 1) << 3),
                               P.vp_y0 + (int)blockIdx.y * 16 + (lane >> 3) + ((wave >> 1) << 3));
}

// Frame-chunked launches: accumulator += samples of frames 0..nframes-1 in
// order -- the same sequential fp32 sum as the in-register loop above.
DEV void sum_body(const LaunchParams &P) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int px = P.vp_x0 + blockIdx.x * 16 + (lane & 7) + ((wave & 1) << 3);
  const int r = P.vp_y0 + blockIdx.y * 16 + (lane >> 3) + ((wave >> 1) << 3);
  if (px >= P.vp_x1 || r >= P.vp_y1) return;
  const int py = image_row(P, r);
  if (py >= P.height) return;
  const size_t pix = P.compact ? (size_t)r * P.width + px : (size_t)py * P.width + px;
  const size_t plane = sample_plane(P), lp = sample_index(P, px, r);
  float4 a = P.accum[pix];
  for (int f = 0; f < P.nframes; ++f) {
    const float4 s = P.samples[(size_t)f * plane + lp];
    if (P.flags & F_ANIM) {
      a.x = mixf(a.x, s.x, P.ema_alpha);
      a.y = mixf(a.y, s.y, P.ema_alpha);
      a.z = mixf(a.z, s.z, P.ema_alpha);
    } else {
      a.x += s.x;
      a.y += s.y;
      a.z += s.z;
    }
  }
  P.accum[pix] = a;
}

// ================================================== wavefront SDF renders
// SDF scenes without ReSTIR (C4: the Mandelbulb in a medium) spend ~93% of
// their FLOP in map() (raytracer.glsl:700-712), 17.7 calls per march
// (iSDF, 974-993, plus calcNormal's 4, 714-722).  In the pass kernel the
// marches run at a quarter of the lanes: a wave's lanes march rays of
// different lengths, or shade, at the same time.  Here a pass is split into
// rounds of two kernels over path slots (one slot = one pixel and frame of
// the launch, so a launch's frames run side by side):
//   rt0_jit_wf_shade: per slot, the bounce step of the pass kernel
//     (Integrator::step) up to the next pending march: it consumes the
//     previous round's march answers, adds the light-sampling results the
//     march kernel returned, shades, and parks the path (its state in
//     wf_state, its next ray as an entry of the region's march list, its
//     light-sampling shadow rays as entries of the shadow list);
//   rt0_jit_wf_march: persistent waves take regions off a device counter
//     (one atomic per kRegionGroup regions) and march their entries with
//     lanes that never wait for each other -- a lane whose march (or normal)
//     is done takes the queue's next entry (ballot + prefix count), and every
//     lane evaluates map() at one program point per loop trip, be it a
//     sphere-tracing step or one of calcNormal's four probes.
// A path takes one round per bounce, so a launch is MAX_BOUNCES + 2 rounds.
// Every map() evaluation, the march's bound and stop tests and calcNormal's
// sum are the pass kernel's (bit-identical steps); the light-sampling sums
// are formed in call order in the next round (wf_apply_nee).  Samples go to
// the frame-chunk planes and rt0_sum_kernel adds them in frame order.
//
// Path state, wf_state[k * wf_slots + slot]:
//   k = 0: acc.xyz, mask.x;  1: mask.yz, packed bounce counters, light bits;
//   2 (MIS or spectral): the previous bounce's normal, hero wavelength.
// packed = depth | spec << 7 | diff_b << 8 | spec_b << 15 | scat_ev << 22 |
//          kind << 29 (7-bit counters: MAX_BOUNCES <= 127, rt0_host.cpp)
template <class Cfg, bool SPECTRAL>
DEV constexpr bool wf_extra_state() {
  return (Cfg::flags() & F_MIS) != 0u || (SPECTRAL && (Cfg::flags() & F_SPECTRAL) != 0u);
}

template <class Scene, class Cfg, bool VOL, bool SPECTRAL>
DEV void wf_shade_body(const LaunchParams &P, Scene sc, Cfg cfg) {
  const SceneTables tabs = scene_tables(sc);  // (one barrier, before any wave leaves)
  if (blockIdx.x == 0 && threadIdx.x < 8) P.wf_ctr[16 * threadIdx.x] = 0u;  // the march kernel's range counters
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (w >= (uint32_t)P.wf_nregions) return;
  using It = Integrator<Scene, Cfg, false, VOL, true, SPECTRAL, false>;
  constexpr bool kExtra = wf_extra_state<Cfg, SPECTRAL>();
  const uint32_t R = (uint32_t)P.wf_R, S = P.wf_slots;
  *(volatile uint32_t *)wf_wave_counter(0) = 0u;  // (every lane stores the same 0)
  *(volatile uint32_t *)wf_wave_counter(1) = 0u;
  const uint32_t n = P.wf_round == 0 ? R : P.wf_in_cnt[w];
  const size_t rbase = (size_t)w * R;
  for (uint32_t b = 0; b < n; b += 64u) {
    const uint32_t e = b + lane;
    if (e >= n) continue;
    uint32_t slot;
    v3 ro = mk(0.f, 0.f, 0.f), rd = ro;
    bool marched = false;
    if (P.wf_round == 0) {
      slot = (uint32_t)rbase + e;
      if (slot >= S) continue;
    } else {
      const float4 j0 = P.wf_in[2 * (rbase + e)], j1 = P.wf_in[2 * (rbase + e) + 1];
      slot = __float_as_uint(j1.w);
      ro = mk(j0.x, j0.y, j0.z);
      rd = mk(j1.x, j1.y, j1.z);
      marched = j0.w >= 0.0f;
    }
    // the slot's frame and pixel (pass_body's tile order within a frame)
    const uint32_t gs = P.wf_slot0 + slot, f = gs / P.wf_apad, loc = gs - f * P.wf_apad;
    const uint32_t tile = loc >> 8, tx = tile % P.wf_gx, ty = tile / P.wf_gx, wv = (loc >> 6) & 3u, ln = loc & 63u;
    const int px = P.vp_x0 + (int)(tx * 16u + (ln & 7u) + ((wv & 1u) << 3));
    const int r = P.vp_y0 + (int)(ty * 16u + (ln >> 3) + ((wv >> 1) << 3));
    if (px >= P.vp_x1 || r >= P.vp_y1) continue;
    const int py = image_row(P, r);
    if (py >= P.height) continue;
    It it(P, sc, cfg);
    it.use_tables(tabs);
    it.set_pixel(px, py);
    it.frame = P.frame0 + (uint32_t)P.wf_f0 + f;
    it.wf_slot = slot;
    it.wf_region = w;
    typename It::Path ps;
    bool alive = true;
    if (P.wf_round == 0) {
      it.begin_sample(ps);
      ps.phase = 0;
      ps.ms.active = ps.ms.done = false;
    } else {
      // (the state in list order: the same index as the entry)
      const size_t cap = P.wf_cap, ei = rbase + e;
      const float4 s0 = P.wf_sin[ei], s1 = P.wf_sin[cap + ei];
      const uint32_t pk = __float_as_uint(s1.z), bits = __float_as_uint(s1.w);
      ps.ro = ro;
      ps.rd = rd;
      ps.acc = mk(s0.x, s0.y, s0.z);
      ps.mask = mk(s0.w, s1.x, s1.y);
      ps.prev_nl = mk(0.f, 1.f, 0.f);
      if constexpr (kExtra) {
        const float4 s2 = P.wf_sin[2 * cap + ei];
        ps.prev_nl = mk(s2.x, s2.y, s2.z);
        it.hero = s2.w;
      } else {
        it.hero = 550.0f;
      }
      ps.seed = it.pixel_seed();
      ps.depth = (int)(pk & 127u);
      ps.spec = ((pk >> 7) & 1u) != 0u;
      ps.phase = 0;
      it.diff_b = (int)((pk >> 8) & 127u);
      it.spec_b = (int)((pk >> 15) & 127u);
      it.scat_ev = (int)((pk >> 22) & 127u);
      // the previous bounce's light sampling, in call order (sample_lights:
      // sum then x mask; the in-scatter loop: each term in turn)
      if (bits) {
        const int kind = (int)(pk >> 29);
        v3 sum = mk(0.f, 0.f, 0.f);
        for_lights(sc, [&](int l) {
          if (!(bits & (1u << l))) return;
          const float4 q = P.wf_shres[(size_t)l * S + slot];
          if (kind == 2) ps.acc = ps.acc + mk(q.x, q.y, q.z);
          else sum = sum + mk(q.x, q.y, q.z);
        });
        if (kind == 1) ps.acc = ps.acc + sum * ps.mask;
      }
      ps.ms.active = false;
      ps.ms.done = marched;
      if (marched) {
        const float4 q = P.wf_res[rbase + e];
        ps.ms.t = q.x;
        ps.ms.n = mk(q.y, q.z, q.w);
        ps.ms.id = Scene::kSdfs > 1 ? P.wf_res_id[rbase + e] : 0.0f;
      }
      alive = marched;
    }
    // the bounce this march answers, then the next bounce up to its march
    if (alive) {
      alive = it.step(ps);
      if (alive && !ps.ms.active) alive = it.step(ps);
    }
    const bool pending = alive && ps.ms.active;
    if (pending || it.wf_bits) {
      const uint32_t pk = (uint32_t)ps.depth | (ps.spec ? 1u << 7 : 0u) | ((uint32_t)it.diff_b << 8) |
                          ((uint32_t)it.spec_b << 15) | ((uint32_t)it.scat_ev << 22) | ((uint32_t)it.wf_kind << 29);
      // the next round's entry: the march (bound < 0: none, only light sampling
      // to add), and beside it in list order the path's state
      const uint32_t o = wave_append(wf_wave_counter(0));
      const size_t cap = P.wf_cap, oi = rbase + o;
      P.wf_sout[oi] = make_float4(ps.acc.x, ps.acc.y, ps.acc.z, ps.mask.x);
      P.wf_sout[cap + oi] = make_float4(ps.mask.y, ps.mask.z, __uint_as_float(pk), __uint_as_float(it.wf_bits));
      if constexpr (kExtra) P.wf_sout[2 * cap + oi] = make_float4(ps.prev_nl.x, ps.prev_nl.y, ps.prev_nl.z, it.hero);
      const March &m = ps.ms;
      P.wf_out[2 * (rbase + o)] = pending ? make_float4(m.o.x, m.o.y, m.o.z, m.tmin) : make_float4(0.f, 0.f, 0.f, -1.0f);
      P.wf_out[2 * (rbase + o) + 1] = make_float4(m.d.x, m.d.y, m.d.z, __uint_as_float(slot));
    } else {
      const v3 col = it.finish(ps);
      P.samples[(size_t)(P.wf_f0 + (int)f) * sample_plane(P) + sample_index(P, px, r)] = make_float4(col.x, col.y, col.z, 0.f);
    }
  }
  // (the wave has reconverged: every append is counted)
  if (lane == 0) {
    P.wf_out_cnt[w] = *(volatile uint32_t *)wf_wave_counter(0);
    P.wf_sh_cnt[w] = *(volatile uint32_t *)wf_wave_counter(1);
  }
}

// ============================================= wavefront ReSTIR model renders
// ReSTIR scenes with triangle models (C5: a glass icosphere of 81 920
// triangles under 10 lights) spent half their pass kernel in the inline
// closest-hit walk at a third of the lanes busy: one lane's ray walks a deep
// subtree while its neighbours' rays missed the model or finished.  Here the
// pass kernel's paths run as rounds of
//   rt0_jit_wf_shade (wf_restir_shade_body): per path slot, the bounce step of
//     the pass kernel (Integrator::step, RESTIR, deferred sampleLightsReSTIR
//     calls appended to the pass wave's NeeRec region as before) up to the
//     next closest-hit query of the triangles, whose ray (bounded by the
//     quadrics' closest t) is parked as an entry of the region's list;
//   rt0_jit_wf_plan + rt0_jit_wf_walk (wf_walk_body): the entries walked
//     through the BVH by persistent waves whose lanes refill as they finish.
// One region = one pass wave (64 slots, pass_body's pixel order), so the
// deferred-call regions, rt0_jit_nee, rt0_jit_walk and rt0_jit_resolve run
// unchanged after the last round.  Every walk is bvh_closest's (same node
// order, same tests, strict t < tmin) and the quadric part of intersection()
// is recomputed on resume, so the samples are bit-identical to the pass
// kernel's.  Path state, wf_state[k * wf_slots + slot]: k = 0 acc.xyz,
// mask.x; 1: mask.yz, packed bounce counters (wf_shade_body's layout), the
// deferred calls so far; 2 (MIS or spectral): previous normal, hero.
template <class Scene, class Cfg, bool VOL, bool SPECTRAL>
DEV void wf_restir_shade_body(const LaunchParams &P, Scene sc, Cfg cfg) {
  treelet_load(P);
  const SceneTables tabs = scene_tables(sc);  // (one barrier, before any wave leaves)
  if (blockIdx.x == 0 && threadIdx.x < 8) P.wf_ctr[16 * threadIdx.x] = 0u;  // the walk kernel's range counters
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (w >= (uint32_t)P.wf_nregions) return;
  using It = Integrator<Scene, Cfg, true, VOL, false, SPECTRAL, false>;
  static_assert(It::WFB, "wavefront ReSTIR shading needs a module of triangle models (RT0_WAVEFRONT)");
  constexpr bool kExtra = wf_extra_state<Cfg, SPECTRAL>();
  const uint32_t S = P.wf_slots;
  const uint32_t nw = (P.wf_slot0 >> 6) + w;  // the pass wave (wf_slot0: whole waves)
  *(volatile uint32_t *)wf_wave_counter(0) = 0u;  // (every lane stores the same value)
  *(volatile uint32_t *)nee_wave_counter() = P.wf_round == 0 ? 0u : P.nee_count[nw];
  const uint32_t n = P.wf_round == 0 ? 64u : P.wf_in_cnt[w];
  const size_t rbase = (size_t)w * 64u;
  if (lane < n) do {
    uint32_t slot;
    v3 ro = mk(0.f, 0.f, 0.f), rd = ro;
    bool walked = false;
    if (P.wf_round == 0) {
      slot = (uint32_t)rbase + lane;
      if (slot >= S) break;
    } else {
      const float4 j0 = P.wf_in[2 * (rbase + lane)], j1 = P.wf_in[2 * (rbase + lane) + 1];
      slot = __float_as_uint(j1.w);
      ro = mk(j0.x, j0.y, j0.z);
      rd = mk(j1.x, j1.y, j1.z);
      walked = j0.w >= 0.0f;
    }
    const uint32_t loc = P.wf_slot0 + slot;  // pass_body's tile order (one frame)
    const uint32_t tile = loc >> 8, tx = tile % P.wf_gx, ty = tile / P.wf_gx, wv = (loc >> 6) & 3u, ln = loc & 63u;
    const int px = P.vp_x0 + (int)(tx * 16u + (ln & 7u) + ((wv & 1u) << 3));
    const int r = P.vp_y0 + (int)(ty * 16u + (ln >> 3) + ((wv >> 1) << 3));
    if (px >= P.vp_x1 || r >= P.vp_y1) break;
    const int py = image_row(P, r);
    if (py >= P.height) break;
    const size_t pix = (size_t)py * P.width + px;
    It it(P, sc, cfg);
    it.use_tables(tabs);
    it.set_pixel(px, py);
    it.frame = P.frame0;
    it.nee_pix = (int32_t)pix;
    it.nee_wave = nw;
    typename It::Path ps;
    bool alive = true;
    if (P.wf_round == 0) {
      it.begin_sample(ps);
      ps.ms.active = ps.ms.done = false;
    } else {
      const float4 s0 = P.wf_state[slot], s1 = P.wf_state[(size_t)S + slot];
      const uint32_t pk = __float_as_uint(s1.z);
      ps.ro = ro;
      ps.rd = rd;
      ps.acc = mk(s0.x, s0.y, s0.z);
      ps.mask = mk(s0.w, s1.x, s1.y);
      ps.prev_nl = mk(0.f, 1.f, 0.f);
      if constexpr (kExtra) {
        const float4 s2 = P.wf_state[2 * (size_t)S + slot];
        ps.prev_nl = mk(s2.x, s2.y, s2.z);
        it.hero = s2.w;
      } else {
        it.hero = 550.0f;
      }
      ps.seed = it.pixel_seed();
      ps.depth = (int)(pk & 127u);
      ps.spec = ((pk >> 7) & 1u) != 0u;
      it.diff_b = (int)((pk >> 8) & 127u);
      it.spec_b = (int)((pk >> 15) & 127u);
      it.scat_ev = (int)((pk >> 22) & 127u);
      it.nee_k = (int32_t)__float_as_uint(s1.w);
      it.fin = empty_res();  // (only the deferred calls touch g_final_reservoir)
      it.gr_have = false;
      ps.ms.active = false;
      ps.ms.done = walked;
      if (walked) {
        const float4 q = P.wf_res[rbase + lane];
        ps.ms.t = q.x;
        ps.ms.id = q.y;  // the triangle (int bits) or -1
      }
      alive = walked;
    }
    // the bounce this walk answers, then the next bounces up to the next walk
    while (alive && !ps.ms.active) alive = it.step(ps);
    if (alive) {
      const uint32_t pk = (uint32_t)ps.depth | (ps.spec ? 1u << 7 : 0u) | ((uint32_t)it.diff_b << 8) |
                          ((uint32_t)it.spec_b << 15) | ((uint32_t)it.scat_ev << 22);
      P.wf_state[slot] = make_float4(ps.acc.x, ps.acc.y, ps.acc.z, ps.mask.x);
      P.wf_state[(size_t)S + slot] = make_float4(ps.mask.y, ps.mask.z, __uint_as_float(pk), __uint_as_float((uint32_t)it.nee_k));
      if constexpr (kExtra) P.wf_state[2 * (size_t)S + slot] = make_float4(ps.prev_nl.x, ps.prev_nl.y, ps.prev_nl.z, it.hero);
      const uint32_t o = wave_append(wf_wave_counter(0));
      const March &m = ps.ms;
      P.wf_out[2 * (rbase + o)] = make_float4(m.o.x, m.o.y, m.o.z, m.tmin);
      P.wf_out[2 * (rbase + o) + 1] = make_float4(m.d.x, m.d.y, m.d.z, __uint_as_float(slot));
    } else {
      // pass_body's deferred-pass ending: the path's own radiance and its
      // number of deferred calls for rt0_jit_resolve; without deferred calls
      // the reservoir MRTs here (rt0_jit_nee writes them otherwise)
      P.nee_partial[pix] = make_float4(ps.acc.x, ps.acc.y, ps.acc.z, it.hero);
      P.nee_n[pix] = it.nee_k;
      if (it.nee_k == 0 && P.rout_main != nullptr && P.rout_aux != nullptr) {
        if (it.flag(F_RESTIR_DEF)) {
          const Res q = empty_res();
          P.rout_main[RT0_RES_STRIDE * (size_t)pix] = make_float4(q.pos.x, q.pos.y, q.pos.z, q.W);
          P.rout_aux[RT0_RES_STRIDE * (size_t)pix] = make_float4(q.col.x, q.col.y, q.col.z, pack_alpha(q.age, q.M, q.idx, sc.n_lights()));
        } else {
          P.rout_main[RT0_RES_STRIDE * (size_t)pix] = make_float4(0.f, 0.f, 0.f, 0.f);
          P.rout_aux[RT0_RES_STRIDE * (size_t)pix] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  } while (false);
  // (the wave has reconverged: every append is counted)
  if (lane == 0) {
    P.wf_out_cnt[w] = *(volatile uint32_t *)wf_wave_counter(0);
    P.wf_sh_cnt[w] = 0u;
    P.nee_count[nw] = *(volatile uint32_t *)nee_wave_counter();
  }
}

// The round's plan (rt0_jit_wf_plan): the regions whose march or shadow list
// is not empty, as (region, march entries, all entries), so that the march
// kernel's grabs skip the empty regions of the late rounds and take several
// sparse regions at once (kRegionGroup), each region opened with one load.
// Plan block b (wf_plan_blocks workgroups of 256 threads) lists the non-empty
// regions of [b * span, (b + 1) * span) at plan[b * span ...] and their count
// and entries in wf_plan_bn[b] / wf_plan_bj[b]; each march workgroup scans
// those totals once (wf_plan_prefix) -- no device-wide prefix pass.
DEV void wf_plan_body(const LaunchParams &P) {
  __shared__ uint32_t wn[4], wj[4];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t NR = (uint32_t)P.wf_nregions, span = (uint32_t)P.wf_plan_span, b = blockIdx.x;
  const uint32_t lo = min(b * span, NR), hi = min(lo + span, NR);
  uint32_t at = 0, nj = 0;  // (block-uniform)
  uint4 *plan = reinterpret_cast<uint4 *>(P.wf_plan) + (size_t)b * span;
  for (uint32_t r0 = lo; r0 < hi; r0 += 256u) {
    const uint32_t r = r0 + threadIdx.x;
    uint32_t ca = 0, cb = 0;
    if (r < hi) {
      ca = P.wf_out_cnt[r];
      cb = P.wf_sh_cnt[r];
    }
    const bool ne = (ca | cb) != 0u;
    const uint64_t m = __ballot(ne);
    uint32_t j = ca + cb;  // this wave's entries: a butterfly sum
    for (int o = 32; o > 0; o >>= 1) j += (uint32_t)__shfl_xor((int)j, o);
    if (lane == 0) {
      wn[w] = (uint32_t)__popcll(m);
      wj[w] = j;
    }
    __syncthreads();
    uint32_t before = 0, total = 0, jt = 0;
    for (uint32_t k = 0; k < 4; ++k) {
      before += k < w ? wn[k] : 0u;
      total += wn[k];
      jt += wj[k];
    }
    if (ne) plan[at + before + (uint32_t)__popcll(m & lt)] = make_uint4(r, ca, ca + cb, 0u);
    at += total;
    nj += jt;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    P.wf_plan_bn[b] = at;
    P.wf_plan_bj[b] = nj;
  }
}

// A march workgroup's view of the plan: the exclusive prefix of the plan
// blocks' counts in LDS (wf_plan_blocks <= 256), the plan's length and the
// round's entries
struct WfPlan {
  const uint32_t *pre;
  uint32_t np, tj;
};
DEV WfPlan wf_plan_prefix(const LaunchParams &P) {
  __shared__ uint32_t pre[257], tot[2];
  const uint32_t B = (uint32_t)P.wf_plan_blocks, t = threadIdx.x;
  if (t < 64) {  // one wave: 4 blocks per lane, a shuffle scan of the lanes' sums
    uint32_t n[4], j = 0, s = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t bb = 4 * t + k;
      n[k] = bb < B ? P.wf_plan_bn[bb] : 0u;
      j += bb < B ? P.wf_plan_bj[bb] : 0u;
      s += n[k];
    }
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)inc, o);
      if ((int)t >= o) inc += x;
    }
    uint32_t e = inc - s;
    for (int k = 0; k < 4; ++k) {
      pre[4 * t + k] = e;
      e += n[k];
    }
    for (int o = 32; o > 0; o >>= 1) j += (uint32_t)__shfl_xor((int)j, o);
    if (t == 63) {
      pre[256] = inc;
      tot[0] = inc;
      tot[1] = j;
    }
  }
  __syncthreads();
  return WfPlan{pre, tot[0], tot[1]};
}

// A march / walk wave's queue over the round's plan (wf_plan_body: the
// regions with any entry, in order), split into kParts ranges with a counter
// each (64 B apart): a wave grabs G plan entries from the range of its XCD
// (the dispatcher deals workgroups round-robin over the 8 XCDs), then from
// the others once its own is taken; G covers ~RT0_WF_UNIT entries at the
// round's mean entries per region (1 region in the first rounds, tens once
// most paths ended).  A device-scope atomic on one address serialises at
// ~0.1 us: one counter over every region made the late rounds (a few paths
// left in a few regions) cost ~0.5-1 ms each in grabs alone.  Wave-uniform.
struct WfQueue {
  static constexpr uint32_t kParts = 8;
  const LaunchParams &P;
  WfPlan pl;
  uint32_t lane, NR, NP, PB, PS, G;
  uint32_t reg, pos, pos_end, q, nc, nall, part, tried;
  DEV WfQueue(const LaunchParams &p, const WfPlan &plan)
      : P(p), pl(plan), lane(threadIdx.x & 63u), NR((uint32_t)p.wf_nregions), NP(plan.np),
        PB((uint32_t)p.wf_plan_blocks), PS((uint32_t)p.wf_plan_span),
        G(max(1u, (uint32_t)(((uint64_t)RT0_WF_UNIT * plan.np + plan.tj - 1) / max(plan.tj, 1u)))), reg(NR), pos(0),
        pos_end(0), q(0), nc(0), nall(0), part(blockIdx.x % kParts), tried(0) {}
  // a wave beyond this round's number of grabs leaves at once: in the late
  // rounds (a few hundred grabs) the whole grid probing every range cost
  // ~0.5 ms per round in serialised read-modify-writes
  DEV bool surplus() const { return blockIdx.x * 4u + (threadIdx.x >> 6) >= (NP + G - 1) / G; }
  DEV uint32_t part_lo(uint32_t k) const { return (uint32_t)(((uint64_t)NP * k) / kParts); }
  DEV void grab() {
    while (tried < kParts) {
      const uint32_t lo = part_lo(part), hi = part_lo(part + 1);
      uint32_t g = 0;
      if (lane == 0) {
        uint32_t *ctr = P.wf_ctr + 16 * part;
        // (a plain look first: a taken range costs no read-modify-write)
        g = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lo + g * G < hi) g = atomicAdd(ctr, 1u);
      }
      g = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)g, 0));
      const uint32_t p0 = lo + g * G;
      if (p0 < hi) {
        pos = p0;
        pos_end = min(p0 + G, hi);
        return;
      }
      part = (part + 1) % kParts;
      ++tried;
    }
    pos = pos_end = NP;  // the whole plan is taken
  }
  DEV void open() {
    q = 0;
    nc = nall = 0;
    reg = NR;
    if (pos < NP) {
      uint32_t lo = 0, hi = PB;  // the plan block holding entry pos: pre[lo] <= pos < pre[lo + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pl.pre[mid] <= pos) lo = mid;
        else hi = mid;
      }
      const uint4 e = reinterpret_cast<const uint4 *>(P.wf_plan)[(size_t)lo * PS + (pos - pl.pre[lo])];
      reg = e.x;
      nc = e.y;
      nall = e.z;
    }
  }
  DEV void start() {
    grab();
    open();
  }
  DEV void next_region() {
    if (++pos >= pos_end) grab();
    open();
  }
  DEV bool dry() const { return reg >= NR; }
  // hand up to popcount(fr) entries of the queue to the lanes of fr (ballot
  // + prefix count; across regions): take(j) runs on each lane that gets
  // entry j of region reg, and may leave the lane free again (an entry with
  // nothing to do), which then takes the next one
  template <class Busy, class Take>
  DEV void refill(uint64_t fr, Busy busy, Take take) {
    const uint64_t lt = (1ull << lane) - 1ull;
    while (fr != 0ull && !dry()) {
      if (q >= nall) {
        next_region();
        continue;
      }
      const uint32_t n = min((uint32_t)__popcll(fr), nall - q);
      const uint32_t rank = (uint32_t)__popcll(fr & lt);
      if (!busy() && rank < n) take(q + rank);
      q += n;
      fr = __ballot(!busy());
    }
  }
};

// The march kernel: persistent waves over the round's march and shadow lists.
// A lane holds one entry: a closest-hit march (then, on a hit, calcNormal's
// four probes) or a shadow march.  Each loop trip every busy lane evaluates
// map() once; a lane that is done writes its answer and is refilled from the
// wave's queue (WfQueue) before the next trip, once RT0_WF_REFILL lanes are
// free.
template <class Scene, class Cfg>
DEV void wf_march_body(const LaunchParams &P, Scene sc, Cfg cfg) {
  using G = Geometry<Scene>;
  const uint32_t R = (uint32_t)P.wf_R, RL = R * (uint32_t)P.wf_L;
  const int cap = cfg.marching_steps();
  const float fud = cfg.fudge();
  const WfPlan pl = wf_plan_prefix(P);  // (one barrier, before any wave leaves)
  WfQueue Q(P, pl);
  if (Q.surplus()) return;
  Q.start();
  bool busy = false, shadow = false, dirl = false;
  v3 o = mk(0.f, 0.f, 0.f), d = o, c = o, na = o;
  float tmin = 0.f, t = 0.f, id = 0.f;
  int i = 0, ph = 4;  // ph 4: sphere tracing; 0..3: calcNormal's probe ph
  uint32_t idx = 0;
  // a march has stopped (iSDF's loop exit): a closest-hit march that found
  // the surface goes on to its normal, every other entry is answered
  auto stopped = [&]() {
    const bool hit = !(t > tmin);
    if (!shadow && hit) {
      ph = 0;
      return;
    }
    if (shadow) {
      const bool lit = !hit || (dirl && t == INF_T);
      P.wf_shres[idx] = lit ? make_float4(c.x, c.y, c.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      P.wf_res[idx] = make_float4(t, 0.f, 0.f, 0.f);
    }
    busy = false;
  };
  // entry j of region Q.reg: its march entries, then its shadow entries
  auto take = [&](uint32_t j) {
    float4 a, b, e = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < Q.nc) {
      const size_t k = (size_t)Q.reg * R + j;
      a = P.wf_out[2 * k];
      b = P.wf_out[2 * k + 1];
      idx = (uint32_t)k;
      shadow = false;
    } else {
      const size_t k = 3 * ((size_t)Q.reg * RL + (j - Q.nc));
      a = P.wf_sh[k];
      b = P.wf_sh[k + 1];
      e = P.wf_sh[k + 2];
      idx = __float_as_uint(b.w);
      shadow = true;
    }
    o = mk(a.x, a.y, a.z);
    tmin = a.w;
    d = mk(b.x, b.y, b.z);
    c = mk(e.x, e.y, e.z);
    dirl = shadow && e.w != 0.0f;
    busy = shadow || tmin >= 0.0f;  // (a march entry without a march: only its light sampling goes on)
    t = EPSILON * 4.0f;
    id = 0.0f;
    i = 0;
    ph = 4;
    if (busy && cap <= 0) stopped();  // (MARCHING_STEPS 0: no step at all)
  };
  while (true) {
    const uint64_t fr = __ballot(!busy);
    // refill once RT0_WF_REFILL lanes are free (or all are): each refill's
    // loads are a round trip the wave waits for
    if (__popcll(fr) >= RT0_WF_REFILL || __ballot(busy) == 0ull) Q.refill(fr, [&]() { return busy; }, take);
    if (__ballot(busy) == 0ull) break;  // the queue is dry and every lane answered
    if (busy) {
      const v3 hp = ray_at(o, d, t);
      // calcNormal's probe ph: pos + (s.x, s.y, s.z) * EPSILON, times the same signs
      const float sx = (ph == 0 || ph == 3) ? 1.0f : -1.0f, sy = ph >= 2 ? 1.0f : -1.0f,
                  sz = (ph == 1 || ph == 3) ? 1.0f : -1.0f;
      const v3 p = ph < 4 ? mk(hp.x + sx * EPSILON, hp.y + sy * EPSILON, hp.z + sz * EPSILON) : hp;
      float idm;
      unsigned long long nm = 0;
      const float dist = G::map(sc, p, idm, nm);
      if (ph == 4) {
        id = idm;
        const float h = fabsf(dist);
        bool stop = h < EPSILON || t > tmin;
        if (!stop) {
          t = __builtin_fmaf(h, fud, t);
          stop = ++i >= cap;
        }
        if (stop) stopped();
      } else {
        const v3 sv = mk(sx, sy, sz) * dist;
        na = ph == 0 ? sv : na + sv;
        if (++ph == 4) {
          const v3 n = normalize(na);
          P.wf_res[idx] = make_float4(t, n.x, n.y, n.z);
          if constexpr (Scene::kSdfs > 1) P.wf_res_id[idx] = id;
          busy = false;
        }
      }
    }
  }
}

// The closest-hit walk kernel of wavefront ReSTIR passes over triangle models
// (rt0_jit_wf_walk): each march-list entry is a camera or bounce ray whose
// quadric part the shade kernel has done (the bound is the closest quadric's
// t); a lane walks it through the BVH as bvh_closest does -- nearer child
// first, the far one on the lane's LDS stack, leaves tested in place left
// before right, strict t < tmin -- one node per loop trip, and on answering
// (t, triangle) takes the queue's next entry, so the lanes keep walking
// whatever the rays' lengths.
#if RT0_BVH_STACK16 || defined(RT0_BVH_STACK)
DEV void wf_walk_body(const LaunchParams &P) {
  treelet_load(P);
  const uint32_t R = (uint32_t)P.wf_R;
  const WfPlan pl = wf_plan_prefix(P);  // (one barrier, before any wave leaves)
  WfQueue Q(P, pl);
  if (Q.surplus()) return;
  Q.start();
  const float4 *__restrict__ nodes = reinterpret_cast<const float4 *>(P.bvh);
  const TriDev *__restrict__ tris = P.tris;
  BvhStack stk;
  bool busy = false;
  v3 o = mk(0.f, 0.f, 0.f), d = o, inv = o;
  float tmin = 0.f;
  int node = 0, sp = 0, guard = 0, best = -1;
  uint32_t idx = 0;
  auto take = [&](uint32_t j) {
    const size_t k = (size_t)Q.reg * R + j;
    const float4 a = P.wf_out[2 * k], b = P.wf_out[2 * k + 1];
    o = mk(a.x, a.y, a.z);
    tmin = a.w;
    d = mk(b.x, b.y, b.z);
    inv = mk(frcp(d.x), frcp(d.y), frcp(d.z));
    idx = (uint32_t)k;
    busy = tmin >= 0.0f;  // (an entry without a walk: only its light sampling goes on)
    node = 0;
    sp = 0;
    guard = 0;
    best = -1;
  };
  while (true) {
    const uint64_t fr = __ballot(!busy);
    // (a walk trip is one node: refills wait for RT0_WF_WALK_REFILL free lanes)
    if (__popcll(fr) >= RT0_WF_WALK_REFILL || __ballot(busy) == 0ull) Q.refill(fr, [&]() { return busy; }, take);
    if (__ballot(busy) == 0ull) break;  // the queue is dry and every lane answered
    if (busy) {
      bool done = false;
      float4 a, b, c;
      int4 lk;
      bvh_fetch(P, nodes, node, a, b, c, lk);
      float tl = box_enter(a.x, a.y, a.z, b.x, b.y, b.z, o, inv, tmin);
      float tr = box_enter(a.w, b.w, c.x, c.y, c.z, c.w, o, inv, tmin);
      const int cl = lk.x, cr = lk.y;
      int l0 = -1, l1 = -1;
      if (tl != F_INF && cl < 0) {
        l0 = ~cl;
        tl = F_INF;
      }
      if (tr != F_INF && cr < 0) {
        if (l0 < 0) l0 = ~cr;
        else l1 = ~cr;
        tr = F_INF;
      }
      if (l0 >= 0) {
        float t;
        if (tri_test(tris[l0], o, d, tmin, t)) {
          tmin = t;
          best = l0;
        }
        if (l1 >= 0 && tri_test(tris[l1], o, d, tmin, t)) {
          tmin = t;
          best = l1;
        }
      }
      if (tl != F_INF && tr != F_INF) {
        const bool lfirst = tl <= tr;
        stk.put(sp, lfirst ? cr : cl);
        sp = min(sp + 1, RT0_BVH_STACK - 1);  // the build guarantees depth < RT0_BVH_STACK
        node = lfirst ? cl : cr;
      } else if (tl != F_INF) {
        node = cl;
      } else if (tr != F_INF) {
        node = cr;
      } else if (sp == 0) {
        done = true;
      } else {
        node = stk.get(--sp);
      }
      // a ray visits each node at most once: the cap only guarantees that
      // every wave drains even on a corrupt tree
      if (++guard > 2 * P.n_tris + 8) done = true;
      if (done) {
        P.wf_res[idx] = make_float4(tmin, __int_as_float(best), 0.f, 0.f);
        busy = false;
      }
    }
  }
}
#endif

}  // namespace rt0
