/*
 * rt0_oracle.c -- CPU restatement of raytracer-0's per-pixel integrator.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity CHECKER for the HIP path and the
 * `cpu_baseline` of bench.py ("kind": "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it; the product library never links it.
 *
 * It restates shaders/pathtracing/raytracer.glsl (the reference's whole hot
 * path) in plain C, scalar fp32, one fragment at a time, following the
 * reference's evaluation order.  Each function cites the GLSL line range it
 * follows.  Float semantics follow the oracle that pins it -- the reference
 * shader executed by SwiftShader 4.1 (tests/golden, oracle/gen):
 *   - no FMA contraction (built with -ffp-contract=off);
 *   - uint->float conversion with SwiftShader's double rounding above 2^31
 *     (u2f below) -- this is what makes the RNG stream bit-exact;
 *   - max(a,b) = a > b ? a : b and min(a,b) = a < b ? a : b (SSE semantics:
 *     the second operand wins when either is NaN; max(0.0, NaN) = NaN, which
 *     is the reference's NaN hazard in powerHeuristic, raytracer.glsl:1237);
 *   - pow(x,y) = pow(|x|, y) (SwiftShader evaluates exp2(y*log2|x|));
 *   - mix(x,y,a) = a*(y-x) + x.
 * Transcendentals come from glibc and differ from SwiftShader's by ulps, so
 * radiance parity is within tolerance while the RNG stream is bit-exact.
 *
 * Parity pinned: tests/test_oracle_golden.py checks this file against every
 * golden fixture generated from the reference (tests/golden/manifest.json).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#pragma STDC FP_CONTRACT OFF

#define OR_MAX_MESH 256
#define OR_MAX_LIGHTS 256

/* ------------------------------------------------------------ GLSL helpers */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float gmax(float a, float b) { return a > b ? a : b; }
static inline float gmin(float a, float b) { return a < b ? a : b; }
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
static inline float fract(float x) { return x - floorf(x); }
static inline float gsign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
static inline float step(float e, float x) { return x < e ? 0.0f : 1.0f; }
static inline float mixf(float x, float y, float a) { return a * (y - x) + x; }
static inline v3 mix3(v3 x, v3 y, float a) { return V(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a)); }
static inline float gpow(float x, float y) { return powf(fabsf(x), y); }
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline float isqrt(float x) { return 1.0f / sqrtf(x); }
static inline v3 normalize(v3 a) { return muls(a, isqrt(dot3(a, a))); }
static inline v3 vabs(v3 a) { return V(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline v3 vmax3s(v3 a, float s) { return V(gmax(a.x, s), gmax(a.y, s), gmax(a.z, s)); }
static inline float vmaxc(v3 a) { return gmax(a.x, gmax(a.y, a.z)); }
static inline v3 cross(v3 a, v3 b) {
  return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline v3 reflect(v3 i, v3 n) { return sub(i, muls(n, 2.0f * dot3(n, i))); }
static inline v3 refract(v3 i, v3 n, float eta) {
  float d = dot3(n, i);
  float k = 1.0f - eta * eta * (1.0f - d * d);
  if (k < 0.0f) return V(0, 0, 0);
  return sub(muls(i, eta), muls(n, eta * d + sqrtf(k)));
}

/* uint -> float as SwiftShader converts it (double rounding above 2^31). */
static inline float u2f(uint32_t m) {
  if (m < 0x80000000u) return (float)(int32_t)m;
  return (float)(int32_t)(m - 0x80000000u) + 2147483648.0f;
}
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* raytracer.glsl:302-306 */
float or_hash(float seed) {
  uint32_t n = fbits(seed) * 747796405u + 2891336453u;
  n = ((n >> ((n >> 28u) + 4u)) ^ n) * 277803737u;
  return u2f((n >> 22u) ^ n) * (1.0f / 4294967296.0f);
}
/* raytracer.glsl:308-312 */
static inline v2 hash2(float sx, float sy) {
  float x = fract(sx * 0.1031f), y = fract(sy * 0.1030f);
  float d = x * (y + 19.19f) + y * (x + 19.19f);
  x += d;
  y += d;
  v2 r = {fract((x + y) * x), fract((x + y) * y)};
  return r;
}
void or_hash2(float sx, float sy, float *out) { v2 r = hash2(sx, sy); out[0] = r.x; out[1] = r.y; }

/* ----------------------------------------------------------- scene model */
enum { T_SPHERE = 0, T_PLANE = 1, T_BOX = 2, T_SDF = 3, T_GRID_SDF = 4, T_TRIANGLE = 5 };
enum { M_LIGHT = 0, M_DIR_LIGHT = 1, M_DIFF = 2, M_SPEC = 3, M_REFR_FRESNEL = 4, M_REFR_SCHLICK = 5, M_COAT = 6 };
enum { TEX_NULL = -1 };

typedef struct {
  v3 c, e;
  float nt;
  int t;
  int tex_t;
  v3 tex_c_mask, tex_e_mask;
  float tex_params[4];
  int opts[4];
} Material;

typedef struct {
  Material mat;
  int t;
  v3 pos;
  float joker[4];
} Mesh;

/* Material table, raytracer.glsl:165-224 (textures: 129-141). */
typedef struct { const char *name; float c[3], e[3], nt; int t, tex; int o0, o1; } MatDef;
#define IOR_GLASS 1.53f
#define IOR_SAPPHIRE 1.77f
#define IOR_WATER 1.33f
#define IOR_COAT 1.4f
enum { TX_NONE = -1, TX_1 = 1, TX_CHECK = 7, TX_METAL = 9 };
static const MatDef MATS[] = {
    {"NULL_MAT", {0, 0, 0}, {0, 0, 0}, 0, -1, TX_NONE, 0, 0},
    {"MAT_REFR_CLEAR", {1.f, 0.5f, 0.f}, {0, 0, 0}, IOR_GLASS, M_REFR_FRESNEL, TX_NONE, 0, 0},
    {"MAT_REFR_CLEAR_2", {1, 1, 1}, {0, 0, 0}, IOR_GLASS, M_REFR_SCHLICK, TX_NONE, 0, 0},
    {"MAT_REFR_SAPPHIRE", {1, 1, 1}, {0, 0, 0}, IOR_SAPPHIRE, M_REFR_FRESNEL, TX_NONE, 0, 0},
    {"MAT_REFR_WATER", {0.25f, 0.64f, 0.88f}, {0, 0, 0}, IOR_WATER, M_REFR_FRESNEL, TX_NONE, 0, 0},
    {"MAT_REFR_TEST", {1, 1, 1}, {0, 0, 0}, IOR_GLASS, M_REFR_FRESNEL, TX_1, 1, 0},
    {"MAT_LIGHT_4", {1, 1, 1}, {4, 4, 4}, 0, M_LIGHT, TX_NONE, 0, 0},
    {"MAT_LIGHT_CANDLE_4", {1.0f, 0.57647058823f, 0.16078431372f}, {4, 4, 4}, 0, M_LIGHT, TX_NONE, 0, 0},
    {"MAT_LIGHT_HALOGEN_4", {1.0f, 0.94509803921f, 0.87843137254f}, {4, 4, 4}, 0, M_LIGHT, TX_NONE, 0, 0},
    {"MAT_LIGHT_DEMO", {1, 1, 1}, {10, 10, 10}, 0, M_LIGHT, TX_NONE, 0, 0},
    {"MAT_LIGHT_4_TEX", {1, 1, 1}, {1, 1, 1}, 0, M_LIGHT, TX_1, 1, 0},
    {"MAT_CLEAR_SKY", {0.25098039215f, 0.61176470588f, 1.0f}, {1, 1, 1}, 0, M_DIR_LIGHT, TX_NONE, 0, 0},
    {"MAT_OVERCAST_SKY", {0.78823529411f, 0.8862745098f, 1.0f}, {1, 1, 1}, 0, M_DIR_LIGHT, TX_NONE, 0, 0},
    {"MAT_DIRECT_SUNLIGHT", {1, 1, 1}, {1, 1, 1}, 0, M_DIR_LIGHT, TX_NONE, 0, 0},
    {"MAT_MIRROR", {1, 1, 1}, {0, 0, 0}, 0, M_SPEC, TX_NONE, 0, 0},
    {"MAT_METAL", {0.6f, 0.6f, 0.6f}, {0, 0, 0}, 0, M_SPEC, TX_METAL, 0, 1},
    {"MAT_BLACK", {0, 0, 0}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_WHITE", {1, 1, 1}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_RED", {1, 0, 0}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_GREEN", {0, 1, 0}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_BLUE", {0, 0, 1}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_CORNELL_WHITE", {1, 1, 1}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_CORNELL_RED", {0.7f, 0.12f, 0.05f}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_CORNELL_GREEN", {0.2f, 0.4f, 0.36f}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_YELLOW", {1, 1, 0}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_PURPLE", {0.50196078431f, 0, 0.50196078431f}, {0, 0, 0}, 0, M_DIFF, TX_NONE, 0, 0},
    {"MAT_CHECK_WHITE", {0, 0, 0}, {0, 0, 0}, 0, M_DIFF, TX_CHECK, 1, 0},
    {"MAT_COAT_NAVY", {0, 0, 0.50196078431f}, {1, 1, 1}, IOR_COAT, M_COAT, TX_NONE, 0, 0},
    {"MAT_COAT_PURPLE", {0.50196078431f, 0, 0.50196078431f}, {0, 0, 0}, IOR_COAT, M_COAT, TX_NONE, 0, 0},
    {"MAT_COAT_WAX", {0.9333f, 0.6666f, 0.6f}, {0.005f, 0.005f, 0.005f}, IOR_COAT, M_COAT, TX_NONE, 0, 0},
    {"MAT_TEST", {1, 1, 1}, {0, 0, 0}, 0, M_DIFF, TX_1, 1, 0},
    {"MAT_SPECTRAL_FLINT", {1, 1, 1}, {0, 0, 0}, -1.7167f, M_REFR_FRESNEL, TX_NONE, 0, 0},
    {"MAT_SPECTRAL_DIAMOND", {1, 1, 1}, {0, 0, 0}, -2.3991f, M_REFR_FRESNEL, TX_NONE, 0, 0},
};

typedef struct {
  int w, h;
  int n_meshes, n_sdfs, n_models, n_total;
  Mesh meshes[OR_MAX_MESH];
  int sdf_kind[OR_MAX_MESH];
  int n_lights;
  int light_index[OR_MAX_LIGHTS];
  int u_sphere, u_plane, u_box;
  /* defines (index.js:11-19) */
  int use_cubemap, use_sky, use_biased, use_restir_def, use_spectral, use_vol;
  /* constants (index.js:21-35) */
  int max_bounces, max_diff, max_spec, max_trans, max_scatter, marching_steps;
  float fudge;
  int sample_lights, use_mis, use_restir, restir_samples, render_mode;
  /* uniforms u_time (ms) and u_temporalFrames, read by RENDER_MODE 1 only */
  float time_ms;
  int temporal_frames;
  /* 1 = model SwiftShader 4.1's masked-execution quirk (see radiance()) */
  int ghost;
  int scatter0_exit; /* SWIFTSHADER_SCATTER0_EXIT: the executor's first-iteration `continue` (see radiance) */
  int scatter_exit;  /* SWIFTSHADER_SCATTER_EXIT: the executor retires the lane at every scatter `continue` */
  int ss_tex;        /* SWIFTSHADER_TEX_FILTER: the executor's fixed-point RGBA8 bilinear filter (tex_fetch_ss) */
  int ss_quad_lights; /* SWIFTSHADER_QUAD_LIGHTS: light_index[i] in brdf's light loops read at the quad's first lane's index (rule 7) */
  int dbg_paths;     /* RT0_DEBUG_PATHS: non-ReSTIR reservoir outputs carry per-sample path statistics */
  int dbg_events;    /* RT0_DEBUG_EVENTS: ... carry the first-event record (instrument_events) */
  /* camera uniforms (index.js:421-423) */
  v3 cam_pos, cam_look, cam_params;
  /* asset textures (index.js:256-296): 0..3 u_tex0..3, 4 u_rnd_tex; RGBA8 */
  const unsigned char *tex_img[5];
  int tex_w[5], tex_h[5];
  /* world-space triangles of the TRIANGLE models (9 floats each) and their
   * owner model (bit 30: back-face culling); brute force, no BVH: the oracle
   * for the product's LBVH closest hit */
  const float *tri_v;
  const int *tri_model;
  int n_tris;
  /* u_cubemap: 6 RGB8 faces in the reference's order -X -Y -Z +X +Y +Z */
  const unsigned char *cube[6];
  int cube_size;
  char err[256];
} Oracle;

/* Per-fragment state: the shader's mutable globals (raytracer.glsl:435-439, 1616). */
typedef struct {
  const Oracle *o;
  unsigned frame;
  float fcx, fcy; /* gl_FragCoord.xy */
  int diff_b, spec_b, trans_b, scat_ev;
  int last_depth, first_scat; /* RT0_DEBUG_PATHS */
  /* RT0_DEBUG_PATHS: bounce-loop iterations, depth history (base 16, six
   * iterations per float: dbg_hist[(i-1)/6]) and loop-exit events (base 8,
   * eight per float: dbg_ev[(i-1)/8]) -- every field an integer < 2^24, exact
   * in fp32 (make_golden.py instrument_paths writes the same) */
  float dbg_pit, dbg_hist[3], dbg_ev[2];
  /* RT0_DEBUG_EVENTS (make_golden.py instrument_events): the first
   * intersection's t and texel, the ray direction after the first bounce,
   * the second intersection's t, the first miss's environment sample */
  float ev_t0, ev_f0, ev_t1, ev_dec, ev_env;
  v3 ev_rd1;
  int q0_iters;                /* SWIFTSHADER_QUAD_LIGHTS: bounce-loop iterations of the quad's first lane (-1: this is it) */
  unsigned nee_mask;           /* bounces at which this lane ran brdf's light loop (bit d) */
  unsigned q0_nee_mask;        /* the quad's first lane's nee_mask */
  unsigned nee_gmask, q0_nee_gmask; /* the same for ghost calls' runs */
  int cur_depth;               /* radiance()'s bounce-loop iteration (a ghost brdf's light loop marks it) */
  float hero;
  /* ReSTIR */
  const float *tex[6]; /* restir_buffer, restir_aux, h1, h1a, h2, h2a */
  float fr_pos[3], fr_col[3], fr_ws, fr_M, fr_W, fr_age;
  int fr_idx;
  /* event counters for the algorithmic-FLOP formula */
  uint64_t n_isect, n_iter, n_nee, n_map;
} Frag;

typedef struct {
  v3 n, pos;
  int index;
  v2 uv;      /* raytracer.glsl:102 */
  float texel[4];
} Hit;

/* ------------------------------------------------------------- SDFs */
/* raytracer.glsl:496-528, 642-698 */
static float sdBox(v3 p, v3 b) {
  v3 d = sub(vabs(p), b);
  v3 m = V(gmax(d.x, 0.f), gmax(d.y, 0.f), gmax(d.z, 0.f));
  return length3(m) + gmin(gmax(d.x, gmax(d.y, d.z)), 0.0f);
}
static float sdSphere(v3 p, float s) { return length3(p) - s; }
static float sdCone(v3 p, v3 c) {
  float qx = sqrtf(p.x * p.x + p.z * p.z), qy = p.y;
  float d1 = -qy - c.z;
  float d2 = gmax(qx * c.x + qy * c.y, qy);
  float a = gmax(d1, 0.f), b = gmax(d2, 0.f);
  return sqrtf(a * a + b * b) + gmin(gmax(d1, d2), 0.f);
}
static float sdTriPrism(v3 p, float hx, float hy) {
  v3 q = vabs(p);
  return gmax(q.z - hy, gmax(q.x * 0.866025f + p.y * 0.5f, -p.y) - hx * 0.5f);
}
static float udRoundBox(v3 p, v3 b, float r) {
  v3 d = sub(vabs(p), b);
  return length3(V(gmax(d.x, 0.f), gmax(d.y, 0.f), gmax(d.z, 0.f))) - r;
}
static inline float gmod(float x, float y) { return x - y * floorf(x / y); }
static float MengerSponge(v3 p, v3 scale) {
  float d = sdBox(p, scale);
  float s = 1.0f;
  for (int m = 0; m < 4; ++m) {
    v3 ps = muls(p, s);
    v3 a = V(gmod(ps.x, 2.0f) - 1.0f, gmod(ps.y, 2.0f) - 1.0f, gmod(ps.z, 2.0f) - 1.0f);
    s *= 3.0f;
    v3 r = V(fabsf(1.0f - 3.0f * fabsf(a.x)), fabsf(1.0f - 3.0f * fabsf(a.y)), fabsf(1.0f - 3.0f * fabsf(a.z)));
    float da = gmax(r.x, r.y), db = gmax(r.y, r.z), dc = gmax(r.z, r.x);
    float c = (gmin(da, gmin(db, dc)) - 1.0f) / s;
    d = gmax(c, d);
  }
  return d;
}
static float Mandelbulb(v3 p) {
  v3 w = p;
  float m = dot3(w, w);
  float dz = 1.0f;
  for (int i = 0; i < 3; ++i) {
    float m2 = m * m, m4 = m2 * m2;
    dz = 8.0f * sqrtf(m4 * m2 * m) * dz + 1.0f;
    float x = w.x, x2 = x * x, x4 = x2 * x2;
    float y = w.y, y2 = y * y, y4 = y2 * y2;
    float z = w.z, z2 = z * z, z4 = z2 * z2;
    float k3 = x2 + z2;
    float k2 = isqrt(k3 * k3 * k3 * k3 * k3 * k3 * k3);
    float k1 = x4 + y4 + z4 - 6.0f * y2 * z2 - 6.0f * x2 * y2 + 2.0f * z2 * x2;
    float k4 = x2 - y2 + z2;
    w.x = p.x + 64.0f * x * y * z * (x2 - z2) * k4 * (x4 - 6.0f * x2 * z2 + z4) * k1 * k2;
    w.y = p.y + -16.0f * y2 * k3 * k4 * k4 + k1 * k1;
    w.z = p.z + -8.0f * y * k4 * (x4 * x4 - 28.0f * x4 * x2 * z2 + 70.0f * x4 * z4 - 28.0f * x2 * z2 * z4 + z4 * z4) * k1 * k2;
    m = dot3(w, w);
    if (m > 4.0f) break;
  }
  return 0.25f * logf(m) * sqrtf(m) / dz;
}

/* map(), raytracer.glsl:700-712 with the #sdf_meshes statements of index.html:702-717 */
static v2 map(Frag *F, v3 p) {
  const Oracle *o = F->o;
  F->n_map++;
  v2 res = {0, 0};
  for (int i = 0; i < o->n_sdfs; i++) {
    const Mesh *m = &o->meshes[o->n_meshes + i];
    v3 q = sub(p, m->pos);
    v3 j = V(m->joker[0], m->joker[1], m->joker[2]);
    float d;
    switch (o->sdf_kind[i]) {
      case 0: d = sdBox(q, j); break;
      case 1: d = udRoundBox(q, j, m->joker[3]); break;
      case 2: d = sdSphere(q, m->joker[0]); break;
      case 3: d = sdTriPrism(q, m->joker[0], m->joker[1]); break;
      case 4: d = sdCone(q, j); break;
      case 5: d = MengerSponge(q, j); break;
      default: d = Mandelbulb(q); break;
    }
    v2 s = {d, (float)i};
    if (i == 0) res = s;
    else {
      float a = (res.x < s.x) ? 1.0f : 0.0f;
      res.x = mixf(s.x, res.x, a);
      res.y = mixf(s.y, res.y, a);
    }
  }
  return res;
}

/* raytracer.glsl:714-722 */
static v3 calcNormal(Frag *F, v3 pos) {
  const float E = 0.001f;
  v3 a = muls(V(1, -1, -1), map(F, add(pos, muls(V(1, -1, -1), E))).x);
  v3 b = muls(V(-1, -1, 1), map(F, add(pos, muls(V(-1, -1, 1), E))).x);
  v3 c = muls(V(-1, 1, -1), map(F, add(pos, muls(V(-1, 1, -1), E))).x);
  v3 d = muls(V(1, 1, 1), map(F, add(pos, muls(V(1, 1, 1), E))).x);
  return normalize(add(add(add(a, b), c), d));
}

/* ------------------------------------------------------ intersections */
#define EPSILON 0.001f
#define INF_T 1e4f
#define PI_F 3.14159265f
#define ONE_OVER_PI 0.31830989f
#define TWO_PI 6.28318531f
#define FOUR_PI 12.5663706f
#define RAD 0.01745329f

/* raytracer.glsl:812-815 */
/* getAnimatedPosition, raytracer.glsl:263-298 (identity unless RENDER_MODE 1) */
static v3 anim_pos(const Oracle *o, v3 base, int idx) {
  if (o->render_mode != 1) return base;
  v3 p = base;
  float t = o->time_ms * 0.001f;
  if (idx >= 6 && idx <= 14) {
    float radius = 0.6f;
    float speed = 1.0f + (float)(idx - 6) * 0.2f;
    float phase = (float)(idx - 6) * 0.7f;
    p.x = base.x + cosf(t * speed + phase) * radius * 0.3f;
    p.z = base.z + sinf(t * speed + phase) * radius * 0.3f;
    p.y = base.y + sinf(t * speed * 2.0f + phase) * 0.1f;
  }
  if (idx >= o->n_meshes && o->n_sdfs > 0) {
    float angle = t * 0.5f;
    float ca = cosf(angle), sa = sinf(angle);
    v3 r = V(p.x * ca - p.z * sa, p.y, p.x * sa + p.z * ca);
    r.y += sinf(t * 1.5f) * 0.05f;
    return r;
  }
  return p;
}
static int iPlane(const Mesh *pl, v3 o, v3 d, float tmin, float *t) {
  *t = (-pl->joker[0] - dot3(pl->pos, o)) / dot3(pl->pos, d);
  return (*t > EPSILON) && (*t < tmin);
}
/* raytracer.glsl:818-833 */
static int iSphere(const Oracle *op, const Mesh *s, v3 o, v3 d, float tmin, float *t, int idx) {
  v3 oc = sub(o, anim_pos(op, s->pos, idx));
  float b = dot3(oc, d);
  float c = dot3(oc, oc) - s->joker[0] * s->joker[0];
  float disc = b * b - c;
  if (disc < 0.0f) return 0;
  float sd = sqrtf(disc);
  *t = -b - sd;
  if (*t > EPSILON && *t < tmin) return 1;
  *t = -b + sd;
  return (*t > EPSILON && *t < tmin);
}
/* raytracer.glsl:836-859.  The out-normal is written only on a hit (an
 * unassigned GLSL out parameter leaves the caller's value untouched under the
 * oracle's SwiftShader). */
static int iBox(const Mesh *bx, v3 o, v3 d, float tmin, float *t, v3 *n) {
  v3 m = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  v3 nv = mul(m, sub(bx->pos, o));
  v3 k = muls(muls(vabs(m), bx->joker[0]), 0.5f);
  v3 t1 = sub(nv, k), t2 = add(nv, k);
  float tN = gmax(gmax(t1.x, t1.y), t1.z);
  float tF = gmin(gmin(t2.x, t2.y), t2.z);
  if (tN > tF || tF < 0.0f) return 0;
  *t = (tN > 0.0f) ? tN : tF;
  if (*t < EPSILON || *t >= tmin) return 0;
  v3 hp = sub(add(o, muls(d, *t)), bx->pos);
  float half = bx->joker[0] * 0.5f;
  v3 dd = sub(vabs(hp), V(half, half, half));
  v3 s = V(gsign(hp.x), gsign(hp.y), gsign(hp.z));
  v3 st = V(step(dd.y, dd.x) * step(dd.z, dd.x), step(dd.z, dd.y) * step(dd.x, dd.y),
            step(dd.x, dd.z) * step(dd.y, dd.z));
  *n = normalize(mul(s, st));
  return 1;
}
/* raytracer.glsl:974-993 */
static int iSDF(Frag *F, v3 o, v3 d, float tmin, float *t, v3 *n, int *index) {
  const Oracle *op = F->o;
  *t = EPSILON * 4.0f;
  v2 res = {0, 0};
  for (int i = 0; i < op->marching_steps; ++i) {
    res = map(F, add(o, muls(d, *t)));
    float h = fabsf(res.x);
    if (h < EPSILON || *t > tmin) break;
    *t += h * op->fudge;
  }
  if (*t > tmin) return 0;
  *n = calcNormal(F, add(o, muls(d, *t)));
  *index = op->n_meshes + (int)res.y;
  return 1;
}


/* -------------------------------------------------------------- textures */
/* GL texture() on an RGBA8 asset: GL_LINEAR, GL_REPEAT, level 0
 * (GlslViewport.loadTexture, index.js:703-708); unbound = (0,0,0,1). */
/* SwiftShader 4.1's GL_LINEAR + GL_REPEAT fetch of an RGBA8 texture, as the
 * known-answer shaders of oracle/gen/tex_kat.py measure it (tests/golden/
 * tex_filter_kat.npz; bit-exact on power-of-two sizes, every asset of the
 * reference is one): the coordinate becomes a 16-bit fixed-point fraction
 * (trunc(u * 65536) & 0xFFFF -- REPEAT wraps there), the half-texel offset
 * is taken off in that unit (floor(32768 / w)), and times w it is a 16.16
 * texel position: texel x >> 16 and weight f = x & 0xFFFF.  Texels widen to
 * 16 bits (v * 257); each of the four taps weighs ((wx * wy) >> 16) with
 * wx = 65535 - f or f (likewise wy), contributes (t * w) >> 16, and the sum
 * is read back as sum * (1 / 65535).  Against exact bilinear this loses 1-3 units
 * of 1/65535 and quantises the sub-texel position to w / 65536 texels (64
 * steps per texel at w = 1024). */
static int ss_coord(float u, int w, int *i0, int *i1) {
  float x = u * 65536.0f;
  int q = (fabsf(x) < 2147483520.0f) ? (int)x : (int)0x80000000; /* cvttps2dq (out of range: 0x80000000) */
  int s = ((q & 0xFFFF) - 32768 / w) * w, i = s >> 16; /* arithmetic shift: floor */
  *i0 = ((i % w) + w) % w;
  *i1 = (*i0 + 1) % w;
  return s & 0xFFFF;
}
void tex_fetch_ss(const unsigned char *img, int w, int h, float u, float v, float out[4]) {
  int x0, x1, y0, y1;
  unsigned fu = (unsigned)ss_coord(u, w, &x0, &x1), fv = (unsigned)ss_coord(v, h, &y0, &y1);
  unsigned w00 = ((65535u - fu) * (65535u - fv)) >> 16, w10 = (fu * (65535u - fv)) >> 16;
  unsigned w01 = ((65535u - fu) * fv) >> 16, w11 = (fu * fv) >> 16;
  for (int c = 0; c < 4; c++) {
    unsigned t00 = img[((size_t)y0 * w + x0) * 4 + c] * 257u, t10 = img[((size_t)y0 * w + x1) * 4 + c] * 257u;
    unsigned t01 = img[((size_t)y1 * w + x0) * 4 + c] * 257u, t11 = img[((size_t)y1 * w + x1) * 4 + c] * 257u;
    unsigned n = ((t00 * w00) >> 16) + ((t10 * w10) >> 16) + ((t01 * w01) >> 16) + ((t11 * w11) >> 16);
    out[c] = (float)n * (1.0f / 65535.0f); /* (the readback multiplies by the reciprocal) */
  }
}
static void tex_fetch(const Oracle *o, int unit, float u, float v, float out[4]) {
  const unsigned char *img = o->tex_img[unit];
  if (!img) { out[0] = out[1] = out[2] = 0.0f; out[3] = 1.0f; return; }
  int w = o->tex_w[unit], h = o->tex_h[unit];
  if (o->ss_tex) {
    tex_fetch_ss(img, w, h, u, v, out);
    return;
  }
  float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
  float fx = floorf(x), fy = floorf(y);
  float a = x - fx, b = y - fy;
#ifdef OR_TEX_WEIGHT_BITS /* experiment: quantised sub-texel weights */
  a = floorf(a * (float)(1 << OR_TEX_WEIGHT_BITS)) / (float)(1 << OR_TEX_WEIGHT_BITS);
  b = floorf(b * (float)(1 << OR_TEX_WEIGHT_BITS)) / (float)(1 << OR_TEX_WEIGHT_BITS);
#endif
  int x0 = ((int)fx % w + w) % w, y0 = ((int)fy % h + h) % h;
  int x1 = (x0 + 1) % w, y1 = (y0 + 1) % h;
  for (int c = 0; c < 4; c++) {
    float t00 = img[((size_t)y0 * w + x0) * 4 + c], t10 = img[((size_t)y0 * w + x1) * 4 + c];
    float t01 = img[((size_t)y1 * w + x0) * 4 + c], t11 = img[((size_t)y1 * w + x1) * 4 + c];
    float top = t00 + a * (t10 - t00), bot = t01 + a * (t11 - t01);
    out[c] = (top + b * (bot - top)) / 255.0f;
  }
}
static float glsl_mod(float x, float y) { return x - y * floorf(x / y); }
/* raytracer.glsl:393-401 */
static float value_noise(const Oracle *o, v3 x) {
  v3 p = V(floorf(x.x), floorf(x.y), floorf(x.z));
  v3 f = sub(x, p);
  f = V(f.x * f.x * (3.0f - 2.0f * f.x), f.y * f.y * (3.0f - 2.0f * f.y), f.z * f.z * (3.0f - 2.0f * f.z));
  float ux = (p.x + 37.0f * p.z) + f.x, uy = (p.y + 17.0f * p.z) + f.y;
  float t[4];
  tex_fetch(o, 4, (ux + 0.5f) / 256.0f, (uy + 0.5f) / 256.0f, t);
  return mixf(t[1], t[0], f.z); /* .yx */
}
/* raytracer.glsl:404-431 */
static v3 voronoi(const Oracle *o, v3 x) {
  v3 p = V(floorf(x.x), floorf(x.y), floorf(x.z));
  v3 f = sub(x, p);
  float id = 0.0f, r0 = 100.0f, r1 = 100.0f;
  for (int k = -1; k <= 1; ++k)
    for (int j = -1; j <= 1; ++j)
      for (int i = -1; i <= 1; ++i) {
        v3 b = V((float)i, (float)j, (float)k);
        v3 hx = add(p, b);
        float t[4];
        tex_fetch(o, 4, ((hx.x + 3.0f * hx.z) + 0.5f) / 256.0f, ((hx.y + 1.0f * hx.z) + 0.5f) / 256.0f, t);
        v3 r = add(sub(b, f), V(t[0], t[1], t[2]));
        float d = dot3(r, r);
        if (d < r0) { id = dot3(add(p, b), V(1.0f, 57.0f, 113.0f)); r1 = r0; r0 = d; }
        else if (d < r1) r1 = d;
      }
  return V(sqrtf(r0), sqrtf(r1), fabsf(id));
}
/* raytracer.glsl:363-387 */
static v3 gradient_hash(v3 p) {
  v3 q = V(dot3(p, V(127.1f, 311.7f, 74.7f)), dot3(p, V(269.5f, 183.3f, 246.1f)), dot3(p, V(113.5f, 271.9f, 124.6f)));
  return V(-1.0f + 2.0f * fract(sinf(q.x) * 43758.5453f), -1.0f + 2.0f * fract(sinf(q.y) * 43758.5453f),
           -1.0f + 2.0f * fract(sinf(q.z) * 43758.5453f));
}
static float gradient_noise(v3 p) {
  v3 i = V(floorf(p.x), floorf(p.y), floorf(p.z));
  v3 f = sub(p, i);
  v3 u = V(f.x * f.x * (3.0f - 2.0f * f.x), f.y * f.y * (3.0f - 2.0f * f.y), f.z * f.z * (3.0f - 2.0f * f.z));
  float c[8];
  for (int k = 0; k < 8; k++) {
    v3 of = V((float)(k & 1), (float)((k >> 1) & 1), (float)(k >> 2));
    c[k] = dot3(gradient_hash(add(i, of)), sub(f, of));
  }
  return mixf(mixf(mixf(c[0], c[1], u.x), mixf(c[2], c[3], u.x), u.y),
              mixf(mixf(c[4], c[5], u.x), mixf(c[6], c[7], u.x), u.y), u.z);
}
/* getTexel, raytracer.glsl:726-772 */
static void getTexel(const Oracle *o, const Material *mat, const Hit *hit, float out[4]) {
  int t = mat->tex_t;
  const float *P = mat->tex_params;
  if (t >= 0 && t <= 3) { tex_fetch(o, t, hit->uv.x, hit->uv.y, out); return; }
  if (t == 7) {
    float x = glsl_mod(floorf(P[0] * hit->uv.x) + floorf(P[1] * hit->uv.y), P[2]);
    out[0] = out[1] = out[2] = out[3] = x;
    return;
  }
  if (t == 8) {
    float du = hit->uv.x - P[0], dv = hit->uv.y - P[1];
    float x = glsl_mod(ceilf(sqrtf(du * du + dv * dv) * P[2]), P[3]);
    out[0] = out[1] = out[2] = out[3] = x;
    return;
  }
  v3 sp = mul(V(P[0], P[1], P[2]), hit->pos);
  float x = 0.0f;
  if (t == 4) {
    v3 r = voronoi(o, sp);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = 0.0f;
    return;
  } else if (t == 5) {
    float f = gradient_noise(sp);
    float q = gclamp((f + 0.7f) / 1.4f, 0.0f, 1.0f);
    x = q * q * (3.0f - 2.0f * q);
  } else if (t == 6) {
    x = value_noise(o, sp);
  } else if (t == 9) {
    v3 m = V(-1.2f, 1.99f, -1.6f), q = sp;
    float f = 0.5f * value_noise(o, q);
    q = muls(mul(m, q), 2.01f);
    f += 0.25f * value_noise(o, q);
    q = muls(mul(m, q), 2.02f);
    f += 0.125f * value_noise(o, q);
    x = f;
  }
  out[0] = out[1] = out[2] = out[3] = x;
}

/* texture(u_cubemap, d): GLES 3.0 cube face selection (major axis, table
 * 3.21) and GL_LINEAR with seamless filtering (always on in ES 3.0, 3.8.10):
 * a footprint texel beyond the face edge is fetched from the adjacent face
 * (the texel centre mapped back to a direction and re-projected).  Measured:
 * SwiftShader 4.1 does the same (cube_spheres: 99.2% -> 100% of pixels when
 * edge clamping is replaced by this).  Unbound cubemap = (0,0,0,1). */
static int cube_face(v3 d, float *s, float *t) { /* face in the reference order -X -Y -Z +X +Y +Z */
  float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z), sc, tc, ma;
  int face;
  if (ax >= ay && ax >= az) { face = d.x >= 0 ? 3 : 0; sc = d.x >= 0 ? -d.z : d.z; tc = -d.y; ma = ax; }
  else if (ay >= az) { face = d.y >= 0 ? 4 : 1; sc = d.x; tc = d.y >= 0 ? d.z : -d.z; ma = ay; }
  else { face = d.z >= 0 ? 5 : 2; sc = d.z >= 0 ? d.x : -d.x; tc = -d.y; ma = az; }
  *s = 0.5f * (sc / ma + 1.0f);
  *t = 0.5f * (tc / ma + 1.0f);
  return face;
}
static const unsigned char *cube_texel(const Oracle *o, int face, int i, int j) {
  int n = o->cube_size;
  if (i < 0 || i >= n || j < 0 || j >= n) {
    float scn = 2.0f * ((float)i + 0.5f) / (float)n - 1.0f, tcn = 2.0f * ((float)j + 0.5f) / (float)n - 1.0f;
    v3 d;
    switch (face) { /* the face table inverted: a direction with major-axis component 1 */
      case 3: d = V(1, -tcn, -scn); break;
      case 0: d = V(-1, -tcn, scn); break;
      case 4: d = V(scn, 1, tcn); break;
      case 1: d = V(scn, -1, -tcn); break;
      case 5: d = V(scn, -tcn, 1); break;
      default: d = V(-scn, -tcn, -1); break;
    }
    float s, t;
    face = cube_face(d, &s, &t);
    i = (int)floorf(s * n);
    j = (int)floorf(t * n);
    i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
  }
  return o->cube[face] + ((size_t)j * n + i) * 3;
}
static v3 cube_sample(const Oracle *o, v3 d) {
  if (!o->cube[0]) return V(0, 0, 0);
  float s, t;
  int face = cube_face(d, &s, &t), n = o->cube_size;
  float x = s * (float)n - 0.5f, y = t * (float)n - 0.5f;
  float fx = floorf(x), fy = floorf(y), a = x - fx, b = y - fy;
  int x0 = (int)fx, y0 = (int)fy;
  const unsigned char *q00 = cube_texel(o, face, x0, y0), *q10 = cube_texel(o, face, x0 + 1, y0);
  const unsigned char *q01 = cube_texel(o, face, x0, y0 + 1), *q11 = cube_texel(o, face, x0 + 1, y0 + 1);
  /* a footprint over a cube corner: the texel beyond both edges is the average
   * of the three that meet there (the executor's rule, measured by a cubemap
   * KAT: 0 of 4 096 corner-region samples off by more than 2.4e-4) */
  int ox0 = x0 < 0 || x0 >= n, ox1 = x0 + 1 < 0 || x0 + 1 >= n, oy0 = y0 < 0 || y0 >= n, oy1 = y0 + 1 < 0 || y0 + 1 >= n;
  int corner = ox0 && oy0 ? 0 : ox1 && oy0 ? 1 : ox0 && oy1 ? 2 : ox1 && oy1 ? 3 : -1;
  float r[3];
  for (int c = 0; c < 3; c++) {
    float t00 = q00[c], t10 = q10[c], t01 = q01[c], t11 = q11[c];
    if (corner == 0) t00 = (t10 + t01 + t11) / 3.0f;
    else if (corner == 1) t10 = (t00 + t11 + t01) / 3.0f;
    else if (corner == 2) t01 = (t11 + t00 + t10) / 3.0f;
    else if (corner == 3) t11 = (t01 + t10 + t00) / 3.0f;
    float top = t00 + a * (t10 - t00), bot = t01 + a * (t11 - t01);
    r[c] = (top + b * (bot - top)) / 255.0f;
  }
  return V(r[0], r[1], r[2]);
}

/* test probe (tests/test_oracle_golden.py): cube_sample on six RGB8 faces of
 * size n (order -X -Y -Z +X +Y +Z) for direction d */
void or_cube_probe(const unsigned char *const *faces, int n, const float *d, float *out) {
  Oracle o;
  memset(&o, 0, sizeof o);
  for (int i = 0; i < 6; i++) o.cube[i] = faces[i];
  o.cube_size = n;
  v3 c = cube_sample(&o, V(d[0], d[1], d[2]));
  out[0] = c.x;
  out[1] = c.y;
  out[2] = c.z;
}

/* iTriangle, the reference's commented-out Moller-Trumbore (raytracer.glsl:
 * 864-892), evaluated as written (no FMA: -ffp-contract=off), except for the
 * parallel-ray threshold: EPSILON * |e0| * |e1| instead of the absolute
 * EPSILON (the determinant scales with the triangle's area; with the absolute
 * test the C5 model's ~0.015-edge triangles are rejected at every angle).
 * The product computes the same threshold per triangle (TriDev.eps). */
static int iTriangle(const float *v, int cull, v3 o, v3 d, float tmin, float *t) {
  v3 v1 = V(v[0], v[1], v[2]), e0 = sub(V(v[3], v[4], v[5]), v1), e1 = sub(V(v[6], v[7], v[8]), v1);
  v3 h = cross(d, e1);
  float a = dot3(e0, h);
  float eps = EPSILON * sqrtf(e0.x * e0.x + e0.y * e0.y + e0.z * e0.z) * sqrtf(e1.x * e1.x + e1.y * e1.y + e1.z * e1.z);
  if (cull && a < eps) return 0;
  if (!cull && a > -eps && a < eps) return 0;
  float f = 1.0f / a;
  v3 s = sub(o, v1);
  float u = f * dot3(s, h);
  if (u < 0.0f || u > 1.0f) return 0;
  v3 q = cross(s, e0);
  float vv = f * dot3(d, q);
  if (vv < 0.0f || u + vv > 1.0f) return 0;
  *t = f * dot3(e1, q);
  return *t > EPSILON && *t < tmin;
}

/* intersection(), raytracer.glsl:997-1082 (texture/uv parsing omitted: every
 * supported material has NULL_TEX, so hit.uv / hit.texel never reach the output). */
static float intersection(Frag *F, v3 o, v3 d, Hit *hit) {
  const Oracle *op = F->o;
  F->n_isect++;
  hit->n = V(0, 0, 0);
  hit->pos = V(0, 0, 0);
  hit->index = 0;
  hit->uv = (v2){-1.0f, -1.0f};
  hit->texel[0] = hit->texel[1] = hit->texel[2] = hit->texel[3] = 0.0f;
  int type = -1;
  float tt = INF_T, tmin = INF_T;
  if (op->n_meshes > 0) {
    for (int i = 0; i < op->n_meshes; ++i) {
      const Mesh *m = &op->meshes[i];
      if (m->joker[0] == 0.0f) continue;
      if (m->t == T_SPHERE) {
        if (iSphere(op, m, o, d, tmin, &tt, i)) { tmin = tt; type = T_SPHERE; hit->index = i; }
      } else if (m->t == T_PLANE) {
        if (iPlane(m, o, d, tmin, &tt)) { tmin = tt; type = T_PLANE; hit->index = i; }
      } else if (m->t == T_BOX) {
        if (iBox(m, o, d, tmin, &tt, &hit->n)) { tmin = tt; type = T_BOX; hit->index = i; }
      }
    }
  }
  if (op->n_models > 0) { /* every triangle, lowest index wins ties (strict <) */
    int best = -1;
    for (int i = 0; i < op->n_tris; ++i)
      if (iTriangle(op->tri_v + 9 * (size_t)i, (op->tri_model[i] >> 30) & 1, o, d, tmin, &tt)) { tmin = tt; best = i; }
    if (best >= 0) {
      const float *v = op->tri_v + 9 * (size_t)best;
      v3 v1 = V(v[0], v[1], v[2]);
      hit->n = normalize(cross(sub(V(v[3], v[4], v[5]), v1), sub(V(v[6], v[7], v[8]), v1)));
      hit->index = op->n_meshes + op->n_sdfs + (op->tri_model[best] & 0x3fffffff);
      type = T_TRIANGLE;
    }
  }
  if (op->n_sdfs > 0) {
    if (iSDF(F, o, d, tmin, &tt, &hit->n, &hit->index)) { tmin = tt; type = T_SDF; }
  }
  if (type + 1) {
    hit->pos = add(muls(d, tmin), o);
    if (type == T_SPHERE) {
      /* cartesianToSpherical of the world position (467-471, 1057-1059) */
      float rho = sqrtf(hit->pos.x * hit->pos.x + hit->pos.y * hit->pos.y + hit->pos.z * hit->pos.z);
      hit->uv = (v2){asinf(hit->pos.y / rho) / PI_F, atan2f(hit->pos.z, hit->pos.x) / TWO_PI};
      hit->n = normalize(sub(hit->pos, anim_pos(op, op->meshes[hit->index].pos, hit->index)));
    } else if (type == T_PLANE) hit->n = normalize(op->meshes[hit->index].pos);
    if (hit->uv.x < 0.0f) { /* 1069-1076 */
      v3 nl = vabs(hit->n);
      if (nl.x > nl.y && nl.x > nl.z) hit->uv = (v2){-hit->pos.z, -hit->pos.y};
      else if (nl.y > nl.x && nl.y > nl.z) hit->uv = (v2){hit->pos.x, hit->pos.z};
      else hit->uv = (v2){hit->pos.x, -hit->pos.y};
    }
    if (op->meshes[hit->index].mat.tex_t != TEX_NULL) getTexel(op, &op->meshes[hit->index].mat, hit, hit->texel);
  }
  return tmin;
}

/* ---------------------------------------------------------- sampling */
/* raytracer.glsl:1092-1107 */
static void calc_binormals(v3 n, v3 *ox, v3 *oz) {
  float sig = n.z < 0.0f ? -1.0f : 1.0f;
  if (fabsf(n.z) > 0.99999f) {
    *ox = V(1, 0, 0);
    *oz = V(0, sig, 0);
    return;
  }
  float a = 1.0f / (sig - n.z);
  float b = n.x * n.y * a;
  *ox = V(1.0f + sig * n.x * n.x * a, sig * b, -sig * n.x);
  *oz = V(b, sig + n.y * n.y * a, -n.y);
}
static v3 frame_dir(v3 w, v3 u, v3 v, float rx, float ry) {
  float om = sqrtf(1.0f - ry * ry);
  return normalize(add(add(muls(u, cosf(rx) * om), muls(v, sinf(rx) * om)), muls(w, ry)));
}
/* raytracer.glsl:1109-1120 */
static v3 getSampleBiased(v3 w, float power, float seed) {
  v3 u, v;
  calc_binormals(w, &u, &v);
  v2 r = hash2(seed, seed);
  float rx = r.x * TWO_PI;
  float ry = gpow(r.y, 1.0f / (power + 1.0f));
  return frame_dir(w, u, v, rx, ry);
}
/* raytracer.glsl:1122-1133 */
static v3 getConeSample(v3 w, float extent, float seed) {
  v3 u, v;
  calc_binormals(w, &u, &v);
  v2 r = hash2(seed, seed);
  float rx = r.x * TWO_PI;
  float ry = 1.0f - r.y * extent;
  return frame_dir(w, u, v, rx, ry);
}
/* raytracer.glsl:1135-1141 */
static v3 getRandomDirection(const Oracle *o, v3 n, float seed) {
  return o->use_biased ? getSampleBiased(n, 1.0f, seed) : getConeSample(n, 1.0f, seed);
}
/* raytracer.glsl:1143-1147 */
static v3 randomSphereDirection(float seed) {
  v2 r = hash2(seed, seed);
  float rx = r.x * TWO_PI, ry = r.y * TWO_PI;
  float sy = sinf(ry), cy = cosf(ry);
  return V(sinf(rx) * sy, sinf(rx) * cy, cosf(rx));
}
/* raytracer.glsl:1157-1171 */
#define VOL_SIGMA_T 0.15f
#define VOL_SIGMA_S 0.13f
#define VOL_G 0.5f
static v3 sampleHG(v3 w, float g, float seed) {
  v2 uv = hash2(seed, seed + 1.789f);
  float cos_theta;
  if (fabsf(g) < 0.001f) cos_theta = 1.0f - 2.0f * uv.x;
  else {
    float sqr = (1.0f - g * g) / (1.0f - g + 2.0f * g * uv.x);
    cos_theta = (1.0f + g * g - sqr * sqr) / (2.0f * g);
  }
  float sin_theta = sqrtf(gmax(0.0f, 1.0f - cos_theta * cos_theta));
  float phi = TWO_PI * uv.y;
  v3 t, b;
  calc_binormals(w, &t, &b);
  return normalize(add(add(muls(t, cosf(phi) * sin_theta), muls(b, sinf(phi) * sin_theta)), muls(w, cos_theta)));
}

/* ------------------------------------------------------ light sampling */
/* raytracer.glsl:1174-1230 */
static v3 calcDirectLighting(Frag *F, const Mesh *light, v3 x, v3 nl, float seed) {
  const Oracle *o = F->o;
  Hit hit;
  v3 dl = V(0, 0, 0);
  const int li = (int)(light - o->meshes); /* lightIndex (the light's scene entry) */
  F->n_nee++;
  if (light->mat.t == M_LIGHT) {
    if (light->t == T_SPHERE) {
      v3 sw = sub(anim_pos(o, light->pos, li), x);
      float r2 = light->joker[0] * light->joker[0];
      float d2 = dot3(sw, sw);
      float cos_a_max = sqrtf(1.0f - gclamp(r2 / d2, 0.0f, 1.0f));
      v3 sr = getConeSample(normalize(sw), 1.0f - cos_a_max, seed + 23.1656f);
      float t = intersection(F, add(x, muls(nl, EPSILON)), sr, &hit);
      const Mesh *mh = &o->meshes[hit.index];
      if (mh->mat.t == M_LIGHT) {
        float weight = 2.0f * (1.0f - cos_a_max);
        float T_fog = o->use_vol ? expf(-VOL_SIGMA_T * t) : 1.0f;
        v3 c = vmax3s(mix3(mh->mat.c, V(hit.texel[0], hit.texel[1], hit.texel[2]), hit.texel[3]), 0.001f);
        dl = add(dl, muls(muls(muls(mul(c, mh->mat.e), weight), gmax(0.001f, dot3(sr, nl))), T_fog));
      }
    } else if (light->t == T_SDF) {
      v3 ld = add(anim_pos(o, light->pos, li), mul(randomSphereDirection(seed + 78.2358f), V(light->joker[0], light->joker[1], light->joker[2])));
      v3 sr = normalize(sub(ld, x));
      intersection(F, add(x, muls(nl, EPSILON)), sr, &hit);
      const Mesh *mh = &o->meshes[hit.index];
      if (mh->mat.t == M_LIGHT) {
        v3 c = vmax3s(mix3(mh->mat.c, V(hit.texel[0], hit.texel[1], hit.texel[2]), hit.texel[3]), 0.001f);
        dl = add(dl, muls(mul(c, mh->mat.e), gmax(0.001f, dot3(sr, nl))));
      }
    }
  } else if (light->mat.t == M_DIR_LIGHT) {
    float t = intersection(F, add(x, muls(nl, EPSILON)), light->pos, &hit);
    if (t == INF_T) dl = add(dl, muls(mul(light->mat.c, light->mat.e), gmax(0.001f, dot3(light->pos, nl))));
  }
  return dl;
}
/* raytracer.glsl:1233-1262 */
static float powerHeuristic(float nf, float fPdf, float ng, float gPdf) {
  float f = nf * fPdf, g = ng * gPdf;
  float denom = f * f + g * g;
  return gmax(0.0f, (f * f) / denom);
}
static float cosineHemispherePdf(v3 wi, v3 n) { return gmax(0.0f, dot3(wi, n)) * ONE_OVER_PI; }
static float lightSamplingPdf(const Mesh *light, v3 x) {
  if (light->mat.t != M_LIGHT) return 0.0f;
  if (light->t == T_SPHERE) {
    v3 d = sub(light->pos, x);
    float d2 = dot3(d, d), r2 = light->joker[0] * light->joker[0];
    if (d2 <= r2) return 0.0f;
    float ctm = sqrtf(gmax(0.0f, 1.0f - r2 / d2));
    float denom = 1.0f - ctm;
    if (denom < 1e-6f) return 0.0f;
    return 1.0f / (TWO_PI * denom);
  }
  return 1.0f / FOUR_PI;
}

/* -------------------------------------------------------------- ReSTIR */
/* raytracer.glsl:1264-1802.  A reservoir is {pos, color, ws, M, W, age, idx}. */
typedef struct { v3 pos, col; float ws, M, W, age; int idx; } Res;
static const Res EMPTY_RES = {{0, 0, 0}, {0, 0, 0}, 0, 0, 0, 0, -1};
static const float POISSON[8][2] = {{-0.4706f, 0.4706f}, {0.8090f, 0.2628f}, {-0.2628f, -0.8090f},
                                    {0.6882f, -0.5000f}, {-0.9511f, -0.1625f}, {0.1625f, 0.9511f},
                                    {0.5000f, -0.6882f}, {-0.6882f, 0.5000f}};

static void updateReservoir(Res *r, v3 pos, v3 col, int idx, float weight, float rnd) {
  if (weight <= 0.0f) return;
  r->ws += weight;
  r->M += 1.0f;
  if (r->M > 60.0f) { r->ws *= 0.95f; r->M *= 0.95f; }
  if (r->ws > 0.0f) {
    float p = weight / r->ws;
    if (rnd < p) { r->pos = pos; r->col = col; r->idx = idx; }
  }
}
static int is_finite_f(float x) { return !isnan(x) && !isinf(x); }
static int isValidReservoir(const Oracle *o, const Res *r) {
  if (!is_finite_f(r->M) || !is_finite_f(r->ws) || !is_finite_f(r->W) || !is_finite_f(r->age)) return 0;
  if (r->M <= 0.0f || r->M > 200.0f) return 0;
  if (r->ws <= 0.0f || r->ws > 1000.0f) return 0;
  if (r->W < 0.0f || r->W > 20.0f) return 0;
  if (r->age < 0.0f || r->age > 35.0f) return 0;
  float lc = dot3(r->col, r->col);
  if (lc < 0.000001f || lc > 10000.0f) return 0;
  if (r->idx >= o->n_lights && r->idx != -1) return 0;
  if (dot3(r->pos, r->pos) < EPSILON * EPSILON && r->idx >= 0) return 0;
  return 1;
}
static float evaluateTargetFunction(v3 lp, v3 lc, v3 hp, v3 hn, const Material *mat) {
  v3 lv = sub(lp, hp);
  float dist_sq = dot3(lv, lv);
  if (dist_sq < EPSILON * EPSILON) return 0.0f;
  v3 ld = normalize(lv);
  float ct = gmax(0.0f, dot3(hn, ld));
  if (ct <= 0.0f) return 0.0f;
  v3 lum = V(0.2126f, 0.7152f, 0.0722f);
  float llum = dot3(lc, lum);
  if (llum <= 0.0f) return 0.0f;
  float slum = dot3(mat->c, lum);
  float nnt = (mat->nt - 1.0f) / (mat->nt + 1.0f);
  float R0 = nnt * nnt;
  float is_refr = (mat->t == M_REFR_FRESNEL || mat->t == M_REFR_SCHLICK) ? 1.0f : 0.0f;
  float is_coat = (mat->t == M_COAT) ? 1.0f : 0.0f;
  float base = mixf(slum, R0, is_refr);
  float bw = mixf(base, (1.0f - R0) * slum, is_coat) * ONE_OVER_PI;
  float safe = gmax(dist_sq, 1e-4f);
  return llum * bw * ct / safe;
}
static int isVisible(Frag *F, v3 from, v3 to) {
  v3 sd = sub(to, from);
  float dist = length3(sd);
  if (dist < EPSILON * 10.0f) return 1;
  sd = normalize(sd);
  Hit h;
  float t = intersection(F, add(from, muls(muls(sd, EPSILON), 2.0f)), sd, &h);
  if (t < dist - EPSILON * 2.0f) {
    if (h.index >= 0 && h.index < F->o->n_meshes + F->o->n_sdfs) return F->o->meshes[h.index].mat.t == M_LIGHT;
    return 0;
  }
  return 1;
}
/* GL bilinear fetch, LINEAR + CLAMP_TO_EDGE, level 0 (index.js:660-664). */
static void tex_bilinear(const Oracle *o, const float *tex, float u, float v, float out[4]) {
  if (!tex) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }
  float x = u * (float)o->w - 0.5f, y = v * (float)o->h - 0.5f;
  float fx0 = floorf(x), fy0 = floorf(y);
  float a = x - fx0, b = y - fy0;
  int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
  if (x0 < 0) x0 = 0; if (x0 > o->w - 1) x0 = o->w - 1;
  if (x1 < 0) x1 = 0; if (x1 > o->w - 1) x1 = o->w - 1;
  if (y0 < 0) y0 = 0; if (y0 > o->h - 1) y0 = o->h - 1;
  if (y1 < 0) y1 = 0; if (y1 > o->h - 1) y1 = o->h - 1;
  for (int c = 0; c < 4; c++) {
    float t00 = tex[((size_t)y0 * o->w + x0) * 4 + c], t10 = tex[((size_t)y0 * o->w + x1) * 4 + c];
    float t01 = tex[((size_t)y1 * o->w + x0) * 4 + c], t11 = tex[((size_t)y1 * o->w + x1) * 4 + c];
    float top = t00 + a * (t10 - t00), bot = t01 + a * (t11 - t01);
    out[c] = top + b * (bot - top);
  }
}
static Res unpackReservoir(const Oracle *o, const float m[4], const float a[4]) {
  Res r = EMPTY_RES;
  if (m[3] > 0.0f) {
    r.pos = V(m[0], m[1], m[2]);
    r.W = m[3];
    r.col = V(a[0], a[1], a[2]);
    float pa = a[3];
    float nli = fract(pa * 2.94f);
    float temp = pa - nli * 0.34f;
    float nM = fract(temp * 3.03f);
    float nage = (temp - nM * 0.33f) * 3.03f;
    r.age = nage * 30.0f;
    r.M = nM * 100.0f;
    int len1 = o->n_lights > 1 ? o->n_lights : 1;
    r.idx = (int)(nli * (float)len1) - 1;
    if (r.idx < -1) r.idx = -1;
    if (r.idx > o->n_lights - 1) r.idx = o->n_lights - 1;
    r.M = gmax(1.0f, r.M);
    r.ws = r.W * r.M;
  }
  return r;
}
static void combineReservoirs(const Oracle *o, Res *t, const Res *s, v3 hp, v3 hn, const Material *mat, float rnd) {
  if (!isValidReservoir(o, s)) return;
  float tw = evaluateTargetFunction(s->pos, s->col, hp, hn, mat);
  if (tw <= 0.0f) return;
  float sc = gclamp(tw * gmax(s->W, 0.0f) * gmax(s->M, 1.0f), 0.0f, 200.0f);
  t->ws += sc;
  t->M += s->M;
  if (t->M > 40.0f) {
    float inv = 40.0f / t->M;
    t->ws *= inv;
    t->M = 40.0f;
  }
  if (t->ws > 0.0f) {
    float p = sc / t->ws;
    if (rnd < p) {
      t->pos = s->pos;
      t->col = s->col;
      t->idx = s->idx;
      t->age = gmin(s->age + 0.25f, 30.0f);
    }
  }
}
/* isVisible() as the ghost call of ghost_brdf() executes it: intersection()'s
 * mesh loop (a `continue` loop) and iSDF's march do not run, so no quadric is
 * hit; iSDF then reports a hit at its initial t = 4*EPSILON on the SDF of its
 * never-updated `res` register (the lane's last live map() result: the first
 * SDF, index NUM_MESHES, in every fixture scene with SDFs). */
static int ghost_isVisible(Frag *F, v3 from, v3 to) {
  const Oracle *o = F->o;
  float dist = length3(sub(to, from));
  if (dist < EPSILON * 10.0f) return 1;
  if (o->n_sdfs > 0 && EPSILON * 4.0f < dist - EPSILON * 2.0f) return o->meshes[o->n_meshes].mat.t == M_LIGHT;
  return 1;
}
static v3 sampleLightsReSTIR(Frag *F, v3 hp, v3 hn, const Material *mat, float sx, float sy, int ghost) {
  const Oracle *o = F->o;
  if (!o->use_restir) return V(0, 0, 0);
  if (o->n_lights == 0 || o->light_index[0] < 0) return V(0, 0, 0);
  float scx = F->fcx / (float)o->w, scy = F->fcy / (float)o->h;
  Res init = EMPTY_RES;
  int maxl = o->n_lights > 4 ? o->n_lights : 4;
  int eff = o->restir_samples < maxl ? o->restir_samples : maxl;
  for (int i = 0; i < eff && !ghost; i++) { /* a ghost call skips every non-unrolled loop */
    v2 rv = hash2(sx + (float)i * 0.1f, sy + (float)i * 0.2f);
    int ai = (int)(rv.x * (float)o->n_lights);
    if (ai < 0) ai = 0;
    if (ai > o->n_lights - 1) ai = o->n_lights - 1;
    int li = o->light_index[ai];
    if (li < 0 || li >= o->n_meshes + o->n_sdfs) continue;
    v3 lp = anim_pos(o, o->meshes[li].pos, li);
    v3 lc = mul(o->meshes[li].mat.c, o->meshes[li].mat.e);
    float tv = evaluateTargetFunction(lp, lc, hp, hn, mat);
    if (tv > 0.0f) updateReservoir(&init, lp, lc, li, tv, rv.y);
  }
  Res tr = init;
  if (F->frame > 2u) {
    for (int lvl = 0; lvl < 2; lvl++) {
      /* sampleTemporalHistory, raytracer.glsl:1485-1523 */
      Res h = EMPTY_RES;
      {
        v3 m3 = sub(hp, o->cam_pos);
        float ms = 0.001f * (float)(lvl + 1);
        float mvx = m3.x * ms, mvy = m3.y * ms;
        float js = (float)((unsigned)lvl + F->frame) * 0.1f;
        v2 hj = hash2(scx + js, scy + js);
        float jx = (hj.x - 0.5f) * 0.002f, jy = (hj.y - 0.5f) * 0.002f;
        float px = scx + mvx + jx, py = scy + mvy + jy;
        if (!(px < 0.01f || px > 0.99f || py < 0.01f || py > 0.99f)) {
          float md[4], ad[4];
          tex_bilinear(o, F->tex[lvl == 0 ? 2 : 4], px, py, md);
          tex_bilinear(o, F->tex[lvl == 0 ? 3 : 5], px, py, ad);
          h = unpackReservoir(o, md, ad);
          if (isValidReservoir(o, &h)) h.age += (float)(lvl + 1);
        }
      }
      if (isValidReservoir(o, &h) && h.M > 0.0f && h.age < 30.0f) {
        if (o->render_mode == 1 && h.idx >= 0 && h.idx < o->n_lights) { /* 1669-1676 */
          int act = o->light_index[h.idx];
          if (act >= 0 && act < o->n_meshes + o->n_sdfs) {
            h.pos = anim_pos(o, o->meshes[act].pos, act);
            h.col = mul(o->meshes[act].mat.c, o->meshes[act].mat.e);
          }
        }
        h.age += (float)(lvl + 1);
        float ta = 0.95f;
        if (lvl == 1) ta *= 0.80f;
        if (o->render_mode == 1) ta *= 0.85f;
        h.M *= ta;
        h.ws *= ta;
        float trand = or_hash(sx + 789.123f + (float)lvl * 456.789f);
        combineReservoirs(o, &tr, &h, hp, hn, mat, trand);
      }
    }
    if (tr.M > 100.0f) {
      tr.M = gmin(tr.M, 80.0f);
      tr.ws *= 0.9f;
    }
  }
  Res fr = tr;
  int ns = 8;
  if (o->n_lights > 10) ns = 4;
  if (F->frame < 10u) ns = (ns / 2 > 2) ? ns / 2 : 2;
  for (int i = 0; i < ns && !ghost; i++) {
    v2 sr = hash2(sx + (float)i * 0.3f, sy + (float)i * 0.4f);
    float ox = POISSON[i][0] * 16.0f / (float)o->w, oy = POISSON[i][1] * 16.0f / (float)o->h;
    float nx = scx + ox, ny = scy + oy;
    Res nb = EMPTY_RES;
    if (!(nx < 0.0f || nx > 1.0f || ny < 0.0f || ny > 1.0f)) {
      float md[4], ad[4];
      tex_bilinear(o, F->tex[0], nx, ny, md);
      tex_bilinear(o, F->tex[1], nx, ny, ad);
      nb = unpackReservoir(o, md, ad);
    }
    if (nb.M > 0.0f) {
      if (nb.idx >= 0) {
        v3 ldf = sub(nb.pos, hp);
        if (dot3(ldf, ldf) > 225.0f) continue;
      }
      float thr = o->render_mode == 1 ? 2.0f : 30.0f * 0.8f;
      if (nb.age > thr || sr.x < 0.03f) continue;
      combineReservoirs(o, &fr, &nb, hp, hn, mat, sr.y);
    }
  }
  /* finalizeReservoir, raytracer.glsl:1525-1576 */
  if (fr.ws <= 0.0f || fr.M <= 0.0f) fr.W = 0.0f;
  else {
    float tp = evaluateTargetFunction(fr.pos, fr.col, hp, hn, mat);
    if (tp <= 0.0f) fr.W = 0.0f;
    else if (!(ghost ? ghost_isVisible(F, hp, fr.pos) : isVisible(F, hp, fr.pos))) fr.W = 0.0f;
    else {
      float cM = gclamp(fr.M, 1.0f, 40.0f);
      float raw = fr.ws / (tp * cM);
      float bc = 1.0f;
      if (fr.age > 0.0f) {
        float na = gclamp(fr.age / 30.0f, 0.0f, 1.0f);
        bc *= mixf(0.85f, 1.0f, 1.0f - na * 0.3f);
      }
      if (cM > 16.0f) bc *= sqrtf(16.0f / cM);
      fr.W = bc * raw;
      fr.W = gclamp(fr.W, 0.0f, 12.0f);
      if (!is_finite_f(fr.W)) fr.W = 0.0f;
    }
  }
  fr.age = gmin(fr.age, 30.0f);
  F->fr_pos[0] = fr.pos.x; F->fr_pos[1] = fr.pos.y; F->fr_pos[2] = fr.pos.z;
  F->fr_col[0] = fr.col.x; F->fr_col[1] = fr.col.y; F->fr_col[2] = fr.col.z;
  F->fr_ws = fr.ws; F->fr_M = fr.M; F->fr_W = fr.W; F->fr_age = fr.age; F->fr_idx = fr.idx;
  if (ghost) return V(0, 0, 0); /* only g_final_reservoir survives a ghost call */
  if (fr.W > 0.0f && fr.idx >= 0 && fr.idx < o->n_lights) {
    int ai = fr.idx;
    int act = o->light_index[ai];
    if (act >= 0 && act < o->n_meshes + o->n_sdfs) {
      /* RENDER_MODE 1: current light position must be visible (1767-1776) */
      if (o->render_mode == 1 && !isVisible(F, hp, anim_pos(o, o->meshes[act].pos, act))) return V(0, 0, 0);
      v3 lc = calcDirectLighting(F, &o->meshes[act], hp, hn, sx + 456.789f);
      float ew = gclamp(fr.W, 0.0f, 8.0f);
      if (fr.M > 30.0f) ew *= sqrtf(30.0f / fr.M);
      v3 fc = muls(lc, ew);
      if (!is_finite_f(fc.x) || !is_finite_f(fc.y) || !is_finite_f(fc.z)) return V(0, 0, 0);
      return fc;
    }
  }
  return V(0, 0, 0);
}

/* ------------------------------------------------------------- brdf */
static inline float schlick(v3 rd, v3 n, float nc, float nt) {
  float R0 = gpow((nc - nt) / (nc + nt), 2.0f);
  return R0 + (1.0f - R0) * gpow(1.0f + dot3(n, rd), 5.0f);
}
static inline float fresnel(v3 rd, v3 n, float nc, float nt, v3 refr) {
  float cosI = dot3(rd, n), cosT = dot3(n, refr);
  float Rs = gpow((nc * cosI - nt * cosT) / (nc * cosI + nt * cosT), 2.0f);
  float Rp = gpow((nc * cosT - nt * cosI) / (nc * cosT + nt * cosI), 2.0f);
  return (Rs + Rp) * 0.5f;
}
static inline float spectralIOR(float lambda, float A) {
  float lu = lambda * 0.001f;
  return A + 0.04f / (lu * lu);
}

/* brdf(), raytracer.glsl:1804-1980 */
/* SWIFTSHADER_QUAD_LIGHTS (mask_kat.py rule 11, brdf's light loop,
 * raytracer.glsl:1955-1974): the executor reads the loop-indexed
 * light_index[i] at the index register of the quad's first lane.  It holds
 * i when that lane runs the same loop in the same bounce-loop iteration --
 * live, or as the ghost call of the iteration it breaks in (rule 1; the
 * plain loop is unrolled, rule 5) -- and is stale otherwise (KATs
 * quad_lights_*: every pixel).  The stale value depends on the loop's code
 * shape (the KATs give the end index or 0): without a `continue` before the
 * breaks it reads as mesh 0 (the end index, one past the array, reads 0);
 * with the medium's scatter `continue` (USE_VOLUMETRICS) as mesh 0 after a
 * run of the loop and as element 0 before any, and the ghost run does not
 * refresh it -- those two choices fitted on spectral_vol_2l, the rest held
 * out. */
static int quad_light_index(Frag *F, int i, float bounce) {
  const Oracle *o = F->o;
  const int d = (int)bounce;
  if (i == 0) F->nee_mask |= 1u << d;
  if (!o->ss_quad_lights || o->n_lights < 2 || F->q0_iters < 0) return o->light_index[i];
  const unsigned m = F->q0_nee_mask | (o->use_vol ? 0u : F->q0_nee_gmask);
  if (m & (1u << d)) return o->light_index[i];
  if (o->use_vol && !(m & ((1u << d) - 1u))) return o->light_index[0];
  return 0;
}
static void brdf(Frag *F, const Hit *hit, v3 f, v3 e, float inside, v3 *ro, v3 *rd, v3 *mask, v3 *acc,
                 int *spec, float seed, float bounce) {
  const Oracle *o = F->o;
  v3 x = hit->pos;
  v3 nl = muls(hit->n, inside);
  float fr = (float)F->frame;
  v3 rdir = getRandomDirection(o, nl, seed + 7.1f * fr + 5681.123f + bounce * 92.13f);
  v3 rough = mul(e, rdir);
  float nc = 1.00029f;
  const Material *mat = &o->meshes[hit->index].mat;
  float nt = mat->nt;
  int mt = mat->t;
  float nt_eff = (o->use_spectral && nt < 0.0f) ? spectralIOR(F->hero, fabsf(nt)) : fabsf(nt);

  if (mt == M_DIFF) {
    *ro = add(x, muls(nl, EPSILON));
    *rd = rdir;
    *mask = mul(*mask, f);
    ++F->diff_b;
    *spec = 0;
  } else if (mt == M_SPEC) {
    *ro = add(x, muls(nl, EPSILON));
    *rd = normalize(add(rough, reflect(*rd, nl)));
    *mask = mul(*mask, f);
    ++F->spec_b;
    *spec = 1;
  } else if (mt == M_REFR_FRESNEL || mt == M_REFR_SCHLICK) {
    float nnt = inside < 0.0f ? nt_eff / nc : nc / nt_eff;
    v3 tdir = refract(*rd, nl, nnt);
    *ro = x;
    if (length3(tdir) == 0.0f) {
      *ro = add(*ro, muls(nl, EPSILON));
      *rd = normalize(add(rough, reflect(*rd, nl)));
      ++F->spec_b;
      *spec = 1;
      return;
    }
    tdir = normalize(add(rough, tdir));
    float Re = mixf(schlick(*rd, nl, nc, nt_eff), fresnel(*rd, nl, nc, nt_eff, tdir), mt == M_REFR_FRESNEL ? 1.0f : 0.0f);
    if (or_hash(seed) < Re) {
      *ro = add(*ro, muls(nl, EPSILON));
      *rd = normalize(add(rough, reflect(*rd, nl)));
      ++F->spec_b;
    } else {
      *ro = sub(*ro, muls(nl, EPSILON));
      *mask = mul(*mask, f);
      *rd = tdir;
      ++F->scat_ev;
    }
    *spec = 1;
  } else if (mt == M_COAT) {
    *ro = add(x, muls(nl, EPSILON));
    if (or_hash(seed) < schlick(*rd, nl, nc, nt_eff)) {
      *rd = normalize(add(rough, reflect(*rd, nl)));
      ++F->spec_b;
      *spec = 1;
    } else {
      *rd = rdir;
      *mask = mul(*mask, f);
      ++F->diff_b;
      *spec = 0;
    }
  }

  if (!*spec && o->use_cubemap) { /* environment NEE, raytracer.glsl:1887-1897 */
    Hit eh;
    v3 sr = getRandomDirection(o, nl, seed + bounce * 965.325f);
    float te = intersection(F, add(x, muls(nl, EPSILON)), sr, &eh);
    if (te == INF_T) *acc = add(*acc, mul(*mask, cube_sample(o, sr)));
  }
  if (!*spec && o->sample_lights) {
    float base = seed + 8652.1f * fr;
    if (o->use_restir && o->use_mis) {
      if (o->use_restir_def) {
        v3 tot = V(0, 0, 0);
        if (o->n_lights > 8) {
          float sx = seed + 8652.1f * fr + bounce * 7895.13f;
          float sy = seed + 1234.567f * fr + bounce * 9876.54f;
          tot = sampleLightsReSTIR(F, x, nl, mat, sx, sy, 0);
        } else {
          for (int i = 0; i < o->n_lights; ++i) {
            int idx = o->light_index[i];
            if (idx < 0) continue;
            const Mesh *L = &o->meshes[idx];
            if (L->mat.t != M_LIGHT) continue;
            v3 lv = sub(L->pos, x);
            v3 ld = normalize(lv);
            float dsq = dot3(lv, lv);
            float ct = gmax(0.0f, dot3(nl, ld));
            float imp = ct * dot3(L->mat.e, V(0.2126f, 0.7152f, 0.0722f)) * isqrt(dsq + 1.0f);
            if (imp < 0.001f) continue;
            v3 ls = calcDirectLighting(F, L, x, nl, base + 5681.123f + bounce * 7895.13f + (float)i * 123.456f);
            if (dot3(ls, ls) < 0.001f * 0.001f) continue;
            float lp = lightSamplingPdf(L, x);
            float bp = cosineHemispherePdf(ld, nl);
            tot = add(tot, muls(ls, powerHeuristic(1.0f, lp, 1.0f, bp)));
          }
        }
        *acc = add(*acc, mul(tot, *mask));
      }
    } else if (o->use_restir) {
      if (o->use_restir_def) {
        float sx = seed + 8652.1f * fr + bounce * 7895.13f;
        float sy = seed + 1234.567f * fr + bounce * 9876.54f;
        v3 rc = sampleLightsReSTIR(F, x, nl, mat, sx, sy, 0);
        *acc = add(*acc, mul(rc, *mask));
      }
    } else if (o->use_mis && o->n_lights > 0) {
      v3 mc = V(0, 0, 0);
      for (int i = 0; i < o->n_lights; ++i) {
        int idx = quad_light_index(F, i, bounce);
        if (idx < 0) continue;
        const Mesh *L = &o->meshes[idx];
        if (L->mat.t != M_LIGHT) continue;
        v3 ls = calcDirectLighting(F, L, x, nl, base + 5681.123f + bounce * 7895.13f + (float)i * 123.456f);
        if (dot3(ls, ls) > 0.000001f) {
          v3 ld = normalize(sub(anim_pos(o, L->pos, (int)(L - o->meshes)), x)); /* 1959 */
          float lp = lightSamplingPdf(L, x);
          float bp = cosineHemispherePdf(ld, nl);
          mc = add(mc, muls(ls, powerHeuristic(1.0f, lp, 1.0f, bp)));
        }
      }
      *acc = add(*acc, mul(mc, *mask));
    } else {
      for (int i = 0; i < o->n_lights; ++i) {
        int idx = quad_light_index(F, i, bounce);
        if (idx >= 0) {
          v3 ls = calcDirectLighting(F, &o->meshes[idx], x, nl, base + 5681.123f + bounce * 7895.13f);
          *acc = add(*acc, mul(ls, *mask));
        }
      }
    }
  }
}

/* SwiftShader 4.1's execution of `break` in radiance()'s bounce loop, as pinned
 * by the known-answer shaders of oracle/gen/mask_kat.py (tests/golden/
 * mask_kat.json) and by instrumented copies of the reference shader:
 *  - after a lane executes `break`, the rest of that iteration still CALLS the
 *    functions that follow (here brdf(), raytracer.glsl:2094) for the lane:
 *    code inside a callee is not masked by the caller's break mask, so a global
 *    it writes changes (g_final_reservoir, raytracer.glsl:1757);
 *  - the callee sees its parameter registers as the lane's PREVIOUS call left
 *    them: `in` arguments of that call, `inout` ones (r, mask, acc,
 *    bounceIsSpecular) at their values after it -- the caller's copies into the
 *    parameters are masked;
 *  - loops inside the callee do not run for the lane (their masks start from
 *    the caller's break mask), `if` blocks and straight-line code do.
 * So the "ghost" brdf() repeats the previous call's material branch (with the
 * post-call ray for COAT's Schlick pick) and, when that branch leaves the bounce
 * non-specular and routes light sampling through sampleLightsReSTIR, the ghost
 * sampleLightsReSTIR skips its candidate/temporal/spatial loops and stores an
 * EMPTY reservoir (finalizeReservoir sets W = 0) as g_final_reservoir.  With
 * no previous call the registers hold another fragment's values, but then
 * g_final_reservoir is still EMPTY and stays EMPTY either way.  `continue`
 * (the volumetric scatter, 2050) does not produce a ghost (mask_kat.json).
 * Only enabled for fixture parity (SWIFTSHADER_GHOST). */
typedef struct {
  int have;      /* a live brdf() call happened in this fragment */
  Hit hit;       /* its `in` arguments */
  v3 e;
  float inside, bounce;
  v3 rd;         /* `inout` r.d and bounceIsSpecular after it */
  int spec;
} BrdfRegs;

static void ghost_brdf(Frag *F, const BrdfRegs *g, float seed) {
  const Oracle *o = F->o;
  if (!g->have) return;
  int spec = g->spec;
  const Material *mat = &o->meshes[g->hit.index].mat;
  if (mat->t == M_DIFF) spec = 0;
  else if (mat->t == M_SPEC || mat->t == M_REFR_FRESNEL || mat->t == M_REFR_SCHLICK) spec = 1;
  else if (mat->t == M_COAT) {
    v3 nl = muls(g->hit.n, g->inside);
    float nt = mat->nt;
    float nt_eff = (o->use_spectral && nt < 0.0f) ? spectralIOR(F->hero, fabsf(nt)) : fabsf(nt);
    spec = or_hash(seed) < schlick(g->rd, nl, 1.00029f, nt_eff);
  }
  /* the plain light loop (constant trip count <= 4, no break/continue:
   * unrolled, rule 5) runs in the ghost call too (SWIFTSHADER_QUAD_LIGHTS) */
  if (!spec && o->sample_lights && !o->use_restir && !(o->use_mis && o->n_lights > 0) && o->n_lights <= 4)
    F->nee_gmask |= 1u << F->cur_depth;
  if (spec || !o->sample_lights || !o->use_restir_def) return;
  if (o->use_restir && o->use_mis) {
    if (o->n_lights <= 8) return;
  } else if (!o->use_restir) {
    return;
  }
  /* ghost sampleLightsReSTIR on the previous call's x, nl, material and seed */
  float fr = (float)F->frame;
  float sx = seed + 8652.1f * fr + g->bounce * 7895.13f;
  float sy = seed + 1234.567f * fr + g->bounce * 9876.54f;
  sampleLightsReSTIR(F, g->hit.pos, muls(g->hit.n, g->inside), mat, sx, sy, 1);
}

/* Diagnostics: RT0_ORACLE_TRACE="x,y" prints every bounce of that pixel's
 * paths (ray, closest hit) to stderr, e.g. to see how close a decision that
 * flips under ulp-level differences sits to its threshold. */
static int trace_pixel(const Frag *F) {
  static int tx = -2, ty = -2;
  if (tx == -2) {
    const char *e = getenv("RT0_ORACLE_TRACE");
    tx = ty = -1;
    if (e) sscanf(e, "%d,%d", &tx, &ty);
  }
  return tx >= 0 && F->fcx == (float)tx + 0.5f && F->fcy == (float)ty + 0.5f;
}

/* RT0_DEBUG_PATHS: the exit event of the current bounce-loop iteration */
static inline void dbg_event(Frag *F, float e) {
  float *v = &F->dbg_ev[F->dbg_pit <= 8.0f ? 0 : 1];
  *v = *v * 8.0f + e;
}

/* radiance(), raytracer.glsl:1986-2105 */
static v3 radiance(Frag *F, v3 ro, v3 rd, float seed) {
  const Oracle *o = F->o;
  v3 acc = V(0, 0, 0), mask = V(1, 1, 1);
  int spec = 1;
  v3 prev_nl = V(0, 1, 0);
  BrdfRegs regs; /* SWIFTSHADER_GHOST: brdf()'s parameter registers */
  regs.have = 0;
  for (int depth = 0; depth < o->max_bounces; ++depth) {
    F->cur_depth = depth;
    F->n_iter++;
    F->last_depth = depth;
    F->dbg_pit += 1.0f;
    {
      float *h = &F->dbg_hist[F->dbg_pit <= 6.0f ? 0 : F->dbg_pit <= 12.0f ? 1 : 2];
      *h = *h * 16.0f + (float)depth;
    }
    Hit hit;
    float t = intersection(F, ro, rd, &hit);
    if (depth == 0) {
      F->ev_t0 = t;
      F->ev_f0 = hit.texel[0];
    } else if (depth == 1) {
      F->ev_t1 = t;
    }
    if (depth < 6) /* 1 the first SDF, 2 another hit, 3 a miss; two bits per bounce */
      F->ev_dec += (t == INF_T ? 3.0f : hit.index == o->n_meshes ? 1.0f : 2.0f) * (float)(1 << (2 * depth));
    if (trace_pixel(F))
      fprintf(stderr, "frame %d depth %d ro (%.9g %.9g %.9g) rd (%.9g %.9g %.9g) t %.9g index %d spec %d\n", F->frame,
              depth, ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, t, t == INF_T ? -1 : hit.index, spec);
    if (o->use_vol) {
      float sd = -logf(gmax(or_hash(seed + 4729.3f + (float)depth * 991.1f), 1e-6f)) / VOL_SIGMA_T;
      float tb = gmin(INF_T, t);
      if (sd < tb) {
        v3 sp = add(ro, muls(rd, sd));
        mask = muls(mask, VOL_SIGMA_S / VOL_SIGMA_T);
        if (o->sample_lights) {
          for (int li = 0; li < o->n_lights; ++li) {
            int lidx = o->light_index[li];
            if (lidx < 0) continue;
            const Mesh *lm = &o->meshes[lidx];
            if (lm->mat.t != M_LIGHT || lm->t != T_SPHERE) continue;
            v3 dlc = sub(lm->pos, sp);
            float dc = length3(dlc);
            float r2 = lm->joker[0] * lm->joker[0];
            float cam = sqrtf(1.0f - gclamp(r2 / (dc * dc), 0.0f, 1.0f));
            v3 dir = getConeSample(divs(dlc, dc), 1.0f - cam, seed + 2341.7f + (float)li * 917.3f + (float)depth * 199.1f);
            Hit sh;
            F->n_nee++;
            float ts = intersection(F, add(sp, muls(dir, EPSILON * 20.0f)), dir, &sh);
            if (sh.index != lidx) continue;
            float omega = 2.0f * (1.0f - cam);
            float ct = dot3(rd, dir);
            float g2 = VOL_G * VOL_G;
            float den = 1.0f + g2 - 2.0f * VOL_G * ct;
            float phase = (1.0f - g2) / (FOUR_PI * den * sqrtf(den));
            float Tf = expf(-VOL_SIGMA_T * ts);
            acc = add(acc, muls(muls(muls(mul(mul(mask, lm->mat.c), lm->mat.e), phase), Tf), PI_F * omega));
          }
        }
        rd = sampleHG(rd, VOL_G, seed + 8293.7f + (float)depth * 773.3f);
        ro = sp;
        spec = 0;
        ++F->scat_ev;
        if (F->first_scat < 0) F->first_scat = depth;
        int stop = (F->scat_ev >= o->max_scatter || vmaxc(mask) < 0.01f);
        if (o->ghost) ghost_brdf(F, &regs, seed);
        if (stop) { dbg_event(F, 6.0f); break; }
        /* SWIFTSHADER_SCATTER0_EXIT: the reference executor (SwiftShader 4.1)
         * leaves the bounce loop at this `continue` (raytracer.glsl:2050) when
         * it is executed in the loop's first iteration: the loop body has
         * `break`s after it (2057, 2065, 2089, 2101) and the executor's
         * continue mask then also retires the lane.  Pinned by
         * oracle/gen/mask_kat.py case continue_then_break (a lane that
         * continues at iteration 0 ends with one iteration's contribution;
         * at later iterations the same continue is honoured). */
        if (o->scatter0_exit && depth == 0) break;
        if (o->scatter_exit) break;
        dbg_event(F, 1.0f);
        continue;
      }
    }
    if (t == INF_T) {
      if (!spec && o->sample_lights) {
        if (o->ghost) ghost_brdf(F, &regs, seed);
        dbg_event(F, 2.0f);
        break;
      }
      if (o->use_cubemap) {
        const v3 env = cube_sample(o, rd);
        acc = add(acc, mul(mask, env));
        if (F->ev_env < 0.0f) F->ev_env = env.x;
      } else if (o->use_sky) {
        float k = gclamp(rd.y * 0.6f + 0.5f, 0.3f, 1.0f);
        v3 sky = V(0.5f + 0.5f * cosf(TWO_PI * (0.525f + 0.9f * k)), 0.5f + 0.5f * cosf(TWO_PI * (0.408f + 0.97f * k)),
                   0.5f + 0.5f * cosf(TWO_PI * (0.409f + 0.8f * k)));
        acc = add(acc, mul(mask, sky));
        if (F->ev_env < 0.0f) F->ev_env = sky.x;
      }
      if (o->ghost) ghost_brdf(F, &regs, seed);
      dbg_event(F, 2.0f);
      break;
    }
    const Mesh *mesh = &o->meshes[hit.index];
    v3 trgb = V(hit.texel[0], hit.texel[1], hit.texel[2]);
    v3 c = vmax3s(mix3(mesh->mat.c, mul(trgb, mesh->mat.tex_c_mask), (float)mesh->mat.opts[0] * hit.texel[3]), 0.001f);
    float inside = -gsign(dot3(rd, hit.n));
    v3 e = vmax3s(mix3(mesh->mat.e, mul(trgb, mesh->mat.tex_e_mask), (float)mesh->mat.opts[1] * hit.texel[3]), 0.001f);
    if (mesh->mat.t == M_LIGHT) {
      mask = mul(mask, c);
      float w = 1.0f;
      if (o->use_mis && !spec && o->sample_lights && depth > 0) {
        v3 ld = normalize(sub(hit.pos, ro));
        float lp = lightSamplingPdf(mesh, ro);
        float bp = cosineHemispherePdf(ld, prev_nl);
        w = powerHeuristic(1.0f, bp, 1.0f, lp);
      }
      acc = add(acc, muls(mul(mask, e), w));
      if (o->ghost) ghost_brdf(F, &regs, seed);
      dbg_event(F, 3.0f);
      break;
    }
    prev_nl = muls(hit.n, inside);
    const v3 acc0 = acc;
    brdf(F, &hit, c, e, inside, &ro, &rd, &mask, &acc, &spec, seed, (float)depth);
    if (depth == 0) F->ev_rd1 = rd;
    if (depth < 6 && (acc.x != acc0.x || acc.y != acc0.y || acc.z != acc0.z))  /* brdf() added radiance */
      F->ev_dec += (float)(4096 << depth);
    if (o->ghost) {
      regs.have = 1; regs.hit = hit; regs.e = e; regs.inside = inside; regs.bounce = (float)depth;
      regs.rd = rd; regs.spec = spec;
    }
    if (vmaxc(mask) < 0.01f) {
      dbg_event(F, 4.0f);
      break;
    }
    if (F->diff_b >= o->max_diff || F->spec_b >= o->max_spec || F->trans_b >= o->max_trans ||
        F->scat_ev >= o->max_scatter) {
      dbg_event(F, 5.0f);
      break;
    }
    dbg_event(F, 7.0f);
  }
  return acc;
}

/* CIE fit, raytracer.glsl:324-353 */
static float cmf_x(float l) {
  float t1 = (l - 442.0f) * (l < 442.0f ? 0.0624f : 0.0374f);
  float t2 = (l - 599.8f) * (l < 599.8f ? 0.0264f : 0.0323f);
  float t3 = (l - 501.1f) * (l < 501.1f ? 0.0490f : 0.0382f);
  return 0.362f * expf(-0.5f * t1 * t1) + 1.056f * expf(-0.5f * t2 * t2) - 0.065f * expf(-0.5f * t3 * t3);
}
static float cmf_y(float l) {
  float t1 = (l - 568.8f) * (l < 568.8f ? 0.0213f : 0.0247f);
  float t2 = (l - 530.9f) * (l < 530.9f ? 0.0613f : 0.0322f);
  return 0.821f * expf(-0.5f * t1 * t1) + 0.286f * expf(-0.5f * t2 * t2);
}
static float cmf_z(float l) {
  float t1 = (l - 437.0f) * (l < 437.0f ? 0.0845f : 0.0278f);
  float t2 = (l - 459.0f) * (l < 459.0f ? 0.0385f : 0.0725f);
  return 1.217f * expf(-0.5f * t1 * t1) + 0.681f * expf(-0.5f * t2 * t2);
}
static v3 wavelengthToRGB(float l) {
  float X = cmf_x(l), Y = cmf_y(l), Z = cmf_z(l);
  v3 rgb = V(3.2404542f * X - 1.5371385f * Y - 0.4985314f * Z, -0.9692660f * X + 1.8760108f * Y + 0.0415560f * Z,
             0.0556434f * X - 0.2040259f * Y + 1.0572252f * Z);
  return V(gmax(0.0f, rgb.x) / 0.378f, gmax(0.0f, rgb.y) / 0.298f, gmax(0.0f, rgb.z) / 0.285f);
}

/* main(), raytracer.glsl:2111-2180 -- one sample for the fragment at (px, py). */
static v3 shade_pixel(Frag *F, int px, int py) {
  const Oracle *o = F->o;
  float rx = (float)o->w, ry = (float)o->h;
  float fcx = (float)px + 0.5f, fcy = (float)py + 0.5f;
  F->fcx = fcx;
  F->fcy = fcy;
  F->diff_b = F->spec_b = F->trans_b = F->scat_ev = 0;
  F->last_depth = -1;
  F->first_scat = -1;
  F->dbg_pit = 0.0f;
  F->ev_t0 = F->ev_f0 = F->ev_t1 = F->ev_env = -1.0f;
  F->ev_dec = 0.0f;
  F->ev_rd1 = V(0, 0, 0);
  F->dbg_hist[0] = F->dbg_hist[1] = F->dbg_hist[2] = 0.0f;
  F->dbg_ev[0] = F->dbg_ev[1] = 0.0f;
  F->hero = 550.0f;
  float stx = 2.0f * fcx / rx - 1.0f, sty = 2.0f * fcy / ry - 1.0f;
  float aspect = rx / ry;
  float seed = or_hash(fcx * 12.9898f + fcy * 78.233f + 1113.1f * (float)F->frame);
  if (o->use_spectral) F->hero = or_hash(seed + 4821.73f) * 340.0f + 380.0f;
  float theta = o->cam_params.x * RAD;
  float uVLen = tanf(theta * 0.5f);
  float uULen = aspect * uVLen;
  v3 w = normalize(o->cam_look);
  v3 u = normalize(cross(w, V(0, 1, 0)));
  v3 v = cross(u, w);
  float ax = or_hash(seed + 13.271f), ay = or_hash(seed + 63.216f);
  float flx = step(0.5f, ax), fly = step(0.5f, ay);
  float hx = mixf(ax, 1.0f - ax, flx), hy = mixf(ay, 1.0f - ay, fly);
  float sx = sqrtf(2.0f * hx), sy = sqrtf(2.0f * hy);
  float dx = mixf(sx - 1.0f, 1.0f - sx, flx) / (rx * 0.5f) + stx;
  float dy = mixf(sy - 1.0f, 1.0f - sy, fly) / (ry * 0.5f) + sty;
  v3 fp = muls(normalize(add(add(muls(muls(u, dx), uULen), muls(muls(v, dy), uVLen)), w)), o->cam_params.z);
  float ang = or_hash(seed + 496.4562f) * TWO_PI;
  float rad = or_hash(seed + 249.1686f) * o->cam_params.y;
  v3 ap = muls(add(muls(u, cosf(ang)), muls(v, sinf(ang))), rad);
  v3 ro = add(o->cam_pos, ap);
  v3 rd = normalize(sub(fp, ap));
  v3 col = radiance(F, ro, rd, seed);
  if (o->use_spectral) col = mul(col, wavelengthToRGB(F->hero));
  return col;
}

/* ============================================================ C ABI (test-only) */
static int lookup_material(const char *name, Material *m) {
  for (size_t i = 0; i < sizeof MATS / sizeof MATS[0]; i++) {
    if (!strcmp(MATS[i].name, name)) {
      const MatDef *d = &MATS[i];
      m->c = V(d->c[0], d->c[1], d->c[2]);
      m->e = V(d->e[0], d->e[1], d->e[2]);
      m->nt = d->nt;
      m->t = d->t;
      m->tex_t = d->tex;
      /* TEX_1 (135), TEX_CHECK (140), TEX_METAL (141); NULL_TEX (131) */
      m->tex_c_mask = V(1, 1, 1);
      m->tex_e_mask = V(1, 1, 1);
      memset(m->tex_params, 0, sizeof m->tex_params);
      if (d->tex == TX_1) m->tex_params[3] = 1.0f;
      if (d->tex == TX_CHECK) {
        m->tex_e_mask = V(0, 0, 0);
        m->tex_params[0] = 5.0f; m->tex_params[1] = 5.0f; m->tex_params[2] = 2.0f;
      }
      if (d->tex == TX_METAL) {
        m->tex_c_mask = V(0.7f, 0.25f, 0.055f);
        m->tex_e_mask = V(0.6f, 0.2f, 0.6f);
        m->tex_params[0] = 16.0f; m->tex_params[1] = 10.0f; m->tex_params[2] = 16.0f;
      }
      m->opts[0] = d->o0;
      m->opts[1] = d->o1;
      m->opts[2] = m->opts[3] = 0;
      return 0;
    }
  }
  return -1;
}

/* parse "vecN(a, b, ...)" with GLSL scalar-broadcast semantics */
static int parse_vec(const char **sp, int n, float *out) {
  const char *s = *sp;
  while (isspace((unsigned char)*s) || *s == ',') s++;
  if (strncmp(s, "vec", 3)) return -1;
  s += 4;
  while (isspace((unsigned char)*s)) s++;
  if (*s != '(') return -1;
  s++;
  int k = 0;
  float vals[4] = {0, 0, 0, 0};
  while (*s && *s != ')') {
    char *end;
    float v = strtof(s, &end);
    if (end == s) return -1;
    if (k < 4) vals[k++] = v;
    s = end;
    while (isspace((unsigned char)*s) || *s == ',') s++;
  }
  if (*s != ')') return -1;
  s++;
  for (int i = 0; i < n; i++) out[i] = (k == 1) ? vals[0] : vals[i];
  *sp = s;
  return 0;
}

void *or_create(void) {
  Oracle *o = (Oracle *)calloc(1, sizeof(Oracle));
  /* GlslViewport defaults, index.js:11-35, 89-95 */
  o->w = o->h = 64;
  o->use_sky = 1;
  o->use_biased = 1;
  o->max_bounces = 12; o->max_diff = 4; o->max_spec = 4; o->max_trans = 12; o->max_scatter = 12;
  o->marching_steps = 128; o->fudge = 0.9f;
  o->sample_lights = 1; o->use_mis = 0; o->use_restir = 0; o->restir_samples = 16; o->render_mode = 0;
  o->time_ms = 0.0f; o->temporal_frames = 5;
  o->cam_pos = V(0, 0, 2.8f); o->cam_look = V(0, 0, -1); o->cam_params = V(50, 0, 3.5f);
  return o;
}
void or_destroy(void *h) { free(h); }
const char *or_error(void *h) { return ((Oracle *)h)->err; }

/* Scene text in the reference's textarea grammar (index.html:624-653), one
 * mesh per line; light_index collects lines whose material contains MAT_LIGHT
 * (index.html:632-634, [-1] if none). */
int or_set_scene_lines(void *h, const char *text, const int *sdf_kinds, int n_kinds) {
  Oracle *o = (Oracle *)h;
  Mesh tmp[OR_MAX_MESH];
  int types[OR_MAX_MESH], n = 0, nl = 0, lights[OR_MAX_LIGHTS];
  const char *s = text;
  while (*s) {
    const char *eol = strchr(s, '\n');
    size_t len = eol ? (size_t)(eol - s) : strlen(s);
    char line[512];
    if (len >= sizeof line) { snprintf(o->err, sizeof o->err, "line too long"); return -1; }
    memcpy(line, s, len);
    line[len] = 0;
    s += len + (eol ? 1 : 0);
    char *p = line;
    while (isspace((unsigned char)*p)) p++;
    if (!*p) continue;
    if (n >= OR_MAX_MESH) { snprintf(o->err, sizeof o->err, "too many meshes"); return -1; }
    char mat[64], typ[32];
    int k = 0;
    while (*p && *p != ',' && !isspace((unsigned char)*p) && k < 63) mat[k++] = *p++;
    mat[k] = 0;
    while (*p && (*p == ',' || isspace((unsigned char)*p))) p++;
    k = 0;
    while (*p && *p != ',' && !isspace((unsigned char)*p) && k < 31) typ[k++] = *p++;
    typ[k] = 0;
    Mesh *m = &tmp[n];
    memset(m, 0, sizeof *m);
    if (lookup_material(mat, &m->mat)) { snprintf(o->err, sizeof o->err, "unknown material %s", mat); return -1; }
    if (strstr(mat, "MAT_LIGHT")) lights[nl++] = n;
    if (!strcmp(typ, "SPHERE")) m->t = T_SPHERE;
    else if (!strcmp(typ, "PLANE")) m->t = T_PLANE;
    else if (!strcmp(typ, "BOX")) m->t = T_BOX;
    else if (!strcmp(typ, "SDF")) m->t = T_SDF;
    else if (!strcmp(typ, "TRIANGLE")) m->t = T_TRIANGLE;
    else { snprintf(o->err, sizeof o->err, "unsupported mesh type %s", typ); return -1; }
    float pos[3], jk[4];
    const char *q = p;
    if (parse_vec(&q, 3, pos) || parse_vec(&q, 4, jk)) { snprintf(o->err, sizeof o->err, "bad vectors"); return -1; }
    m->pos = V(pos[0], pos[1], pos[2]);
    memcpy(m->joker, jk, sizeof jk);
    types[n] = m->t;
    n++;
  }
  /* the reference orders meshes as written; SDFs must follow the Euclidean
   * meshes for meshes[NUM_MESHES + i] to address them (index.html:702-717) */
  int ne = 0, ns = 0, nm = 0;
  for (int i = 0; i < n; i++) {
    if (types[i] == T_TRIANGLE) nm++;
    else if (types[i] == T_SDF) {
      if (nm) { snprintf(o->err, sizeof o->err, "TRIANGLE models must follow SDF meshes"); return -1; }
      ns++;
    } else {
      if (ns || nm) { snprintf(o->err, sizeof o->err, "SDF meshes must follow Euclidean meshes"); return -1; }
      ne++;
    }
  }
  o->n_meshes = ne;
  o->n_sdfs = ns;
  o->n_models = nm;
  o->n_total = n;
  memcpy(o->meshes, tmp, sizeof(Mesh) * n);
  for (int i = 0; i < ns; i++) o->sdf_kind[i] = (i < n_kinds) ? sdf_kinds[i] : 0;
  if (nl == 0) lights[nl++] = -1;
  o->n_lights = nl;
  memcpy(o->light_index, lights, sizeof(int) * nl);
  return 0;
}

int or_set_define(void *h, const char *name, int on) {
  Oracle *o = (Oracle *)h;
  if (!strcmp(name, "USE_CUBEMAP")) o->use_cubemap = on;
  else if (!strcmp(name, "USE_PROCEDURAL_SKY")) o->use_sky = on;
  else if (!strcmp(name, "USE_BIASED_SAMPLING")) o->use_biased = on;
  else if (!strcmp(name, "USE_BIDIRECTIONAL")) { /* no #ifdef in the shader */ }
  else if (!strcmp(name, "USE_RESTIR")) o->use_restir_def = on;
  else if (!strcmp(name, "USE_SPECTRAL")) o->use_spectral = on;
  else if (!strcmp(name, "USE_VOLUMETRICS")) o->use_vol = on;
  else { snprintf(o->err, sizeof o->err, "unknown define %s", name); return -1; }
  return 0;
}

int or_set_constant(void *h, const char *name, double v) {
  Oracle *o = (Oracle *)h;
  int iv = (int)v;
  if (!strcmp(name, "MAX_BOUNCES")) o->max_bounces = iv;
  else if (!strcmp(name, "MAX_DIFF_BOUNCES")) o->max_diff = iv;
  else if (!strcmp(name, "MAX_SPEC_BOUNCES")) o->max_spec = iv;
  else if (!strcmp(name, "MAX_TRANS_BOUNCES")) o->max_trans = iv;
  else if (!strcmp(name, "MAX_SCATTERING_EVENTS")) o->max_scatter = iv;
  else if (!strcmp(name, "MARCHING_STEPS")) o->marching_steps = iv;
  else if (!strcmp(name, "FUDGE_FACTOR")) o->fudge = (float)v;
  else if (!strcmp(name, "sample_lights")) o->sample_lights = iv;
  else if (!strcmp(name, "use_mis")) o->use_mis = iv;
  else if (!strcmp(name, "use_restir")) o->use_restir = iv;
  else if (!strcmp(name, "RESTIR_SAMPLES")) o->restir_samples = iv;
  else if (!strcmp(name, "LIGHT_PATH_LENGTH")) { /* unused by the shader */ }
  else if (!strcmp(name, "SWIFTSHADER_GHOST")) o->ghost = iv;
  else if (!strcmp(name, "SWIFTSHADER_SCATTER0_EXIT")) o->scatter0_exit = iv;
  else if (!strcmp(name, "SWIFTSHADER_SCATTER_EXIT")) o->scatter_exit = iv;
  else if (!strcmp(name, "SWIFTSHADER_TEX_FILTER")) o->ss_tex = iv;
  else if (!strcmp(name, "SWIFTSHADER_QUAD_LIGHTS")) o->ss_quad_lights = iv;
  else if (!strcmp(name, "RT0_DEBUG_PATHS")) o->dbg_paths = iv;
  else if (!strcmp(name, "RT0_DEBUG_EVENTS")) o->dbg_events = iv;
  else if (!strcmp(name, "RENDER_MODE")) {
    o->render_mode = iv;
    if (iv != 0 && iv != 1) { snprintf(o->err, sizeof o->err, "RENDER_MODE must be 0 or 1"); return -1; }
  } else { snprintf(o->err, sizeof o->err, "unknown constant %s", name); return -1; }
  return 0;
}

void or_set_camera(void *h, const float *pos, const float *look, const float *params) {
  Oracle *o = (Oracle *)h;
  o->cam_pos = V(pos[0], pos[1], pos[2]);
  o->cam_look = V(look[0], look[1], look[2]);
  o->cam_params = V(params[0], params[1], params[2]);
}
/* loadTexture (index.js:699-728): unit 0..3 = u_tex0..3, 4 = u_rnd_tex; the
 * caller keeps the RGBA8 buffer alive while rendering (NULL = unbound). */
int or_set_texture(void *h, int unit, int w, int hh, const unsigned char *rgba8) {
  Oracle *o = (Oracle *)h;
  if (unit < 0 || unit > 4) return -1;
  o->tex_img[unit] = rgba8;
  o->tex_w[unit] = w;
  o->tex_h[unit] = hh;
  return 0;
}
/* world-space triangles (caller keeps the arrays alive); model ids may carry
 * bit 30 = back-face culling */
int or_set_triangles(void *h, const float *v9, const int *model, int n) {
  Oracle *o = (Oracle *)h;
  o->tri_v = v9;
  o->tri_model = model;
  o->n_tris = n;
  return 0;
}
/* load_cubemap (index.js:298-331): 6 RGB8 faces, reference order; NULL unbinds */
int or_set_cubemap(void *h, int size, const unsigned char *const *faces) {
  Oracle *o = (Oracle *)h;
  for (int i = 0; i < 6; i++) o->cube[i] = faces ? faces[i] : NULL;
  o->cube_size = faces ? size : 0;
  return 0;
}
/* u_time (ms) and u_temporalFrames for RENDER_MODE 1 */
void or_set_time(void *h, float time_ms, int temporal_frames) {
  ((Oracle *)h)->time_ms = time_ms;
  ((Oracle *)h)->temporal_frames = temporal_frames > 0 ? temporal_frames : 5;
}
void or_set_resolution(void *h, int w, int hh) { ((Oracle *)h)->w = w; ((Oracle *)h)->h = hh; }

/* One pass: out[y][x] = that pass's sample (rgb, a = 0) for rows [row0,row1).
 * restir_in: 6 RGBA32F W*H textures (buffer, aux, hist1, hist1_aux, hist2,
 * hist2_aux) or NULL; restir_out_main/aux receive the packed reservoirs
 * (raytracer.glsl:1418-1433, 2171-2179).  counters (4 x u64, may be NULL):
 * intersections, loop iterations, NEE calls, map() calls. */
int or_render_frame(void *h, unsigned frame, float *out, const float *const *restir_in, float *restir_main,
                    float *restir_aux, int row0, int row1, int nthreads, uint64_t *counters) {
  Oracle *o = (Oracle *)h;
  uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  if (row0 < 0) row0 = 0;
  if (row1 > o->h) row1 = o->h;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : c0, c1, c2, c3)
#endif
  for (int y = row0; y < row1; y++) {
    Frag F;
    memset(&F, 0, sizeof F);
    F.o = o;
    F.frame = frame;
    for (int k = 0; k < 6; k++) F.tex[k] = restir_in ? restir_in[k] : NULL;
    for (int x = 0; x < o->w; x++) {
      F.fr_W = 0; F.fr_M = 0; F.fr_ws = 0; F.fr_age = 0; F.fr_idx = -1;
      memset(F.fr_pos, 0, sizeof F.fr_pos);
      memset(F.fr_col, 0, sizeof F.fr_col);
      F.q0_iters = -1;
      F.nee_mask = F.nee_gmask = 0;
      if (o->ss_quad_lights && ((x | y) & 1)) {  /* the quad's first lane's path, rendered aside */
        Frag Q = F;
        const uint64_t q0 = Q.n_iter;
        Q.nee_mask = Q.nee_gmask = 0;
        (void)shade_pixel(&Q, x & ~1, y & ~1);
        F.q0_iters = (int)(Q.n_iter - q0);
        F.q0_nee_mask = Q.nee_mask;
        F.q0_nee_gmask = Q.nee_gmask;
      }
      const uint64_t it0 = F.n_iter;
      v3 col = shade_pixel(&F, x, y);
      size_t p = ((size_t)y * o->w + x) * 4;
      out[p] = col.x; out[p + 1] = col.y; out[p + 2] = col.z; out[p + 3] = 0.0f;
      if (o->dbg_events && !o->use_restir_def && restir_main && restir_aux) {
        restir_main[p] = F.ev_t0; restir_main[p + 1] = F.ev_f0;
        restir_main[p + 2] = F.ev_rd1.x; restir_main[p + 3] = F.ev_rd1.y;
        restir_aux[p] = F.ev_rd1.z; restir_aux[p + 1] = F.ev_t1;
        restir_aux[p + 2] = F.ev_dec; restir_aux[p + 3] = F.ev_env;
        continue;
      }
      if (o->dbg_paths && !o->use_restir_def && restir_main && restir_aux) {
        (void)it0;
        restir_main[p] = F.dbg_pit; restir_main[p + 1] = F.dbg_hist[0];
        restir_main[p + 2] = F.dbg_hist[1]; restir_main[p + 3] = F.dbg_hist[2];
        restir_aux[p] = F.dbg_ev[0]; restir_aux[p + 1] = F.dbg_ev[1];
        restir_aux[p + 2] = (float)F.scat_ev + 256.0f * (float)F.diff_b;
        restir_aux[p + 3] = (float)F.trans_b + 256.0f * (float)F.spec_b;
        continue;
      }
      if (restir_main) {
        int have = o->use_restir_def;
        restir_main[p] = have ? F.fr_pos[0] : 0; restir_main[p + 1] = have ? F.fr_pos[1] : 0;
        restir_main[p + 2] = have ? F.fr_pos[2] : 0; restir_main[p + 3] = have ? F.fr_W : 0;
      }
      if (restir_aux) {
        int have = o->use_restir_def;
        float na = gclamp(F.fr_age / 30.0f, 0.0f, 1.0f);
        float nM = gclamp(F.fr_M / 100.0f, 0.0f, 1.0f);
        int len1 = o->n_lights > 1 ? o->n_lights : 1;
        float nli = (float)(F.fr_idx + 1) / (float)len1;
        restir_aux[p] = have ? F.fr_col[0] : 0; restir_aux[p + 1] = have ? F.fr_col[1] : 0;
        restir_aux[p + 2] = have ? F.fr_col[2] : 0;
        restir_aux[p + 3] = have ? na * 0.33f + nM * 0.33f + nli * 0.34f : 0;
      }
    }
    c0 += F.n_isect; c1 += F.n_iter; c2 += F.n_nee; c3 += F.n_map;
  }
  if (counters) { counters[0] += c0; counters[1] += c1; counters[2] += c2; counters[3] += c3; }
  return 0;
}

/* Progressive accumulation over passes first..first+n-1 (raytracer.glsl:2168,
 * no ReSTIR): acc[y][x].rgb = acc + sample, sequential fp32 sums. */
int or_render_accum(void *h, unsigned first, int n, float *acc, int row0, int row1, int nthreads, uint64_t *counters) {
  Oracle *o = (Oracle *)h;
  if (o->use_restir_def && o->use_restir) { snprintf(o->err, sizeof o->err, "use or_render_frame for ReSTIR"); return -1; }
  size_t npx = (size_t)o->w * o->h * 4;
  float *tmp = (float *)malloc(npx * sizeof(float));
  for (int f = 0; f < n; f++) {
    or_render_frame(h, first + f, tmp, NULL, NULL, NULL, row0, row1, nthreads, counters);
    for (int y = row0 < 0 ? 0 : row0; y < (row1 > o->h ? o->h : row1); y++)
      for (int x = 0; x < o->w; x++) {
        size_t p = ((size_t)y * o->w + x) * 4;
        if (o->render_mode == 1) { /* mix(previousFrame, currentFrame, 1/u_temporalFrames), 2159-2165 */
          float a = 1.0f / (float)o->temporal_frames;
          for (int k = 0; k < 3; k++) acc[p + k] = mixf(acc[p + k], tmp[p + k], a);
        } else {
          acc[p] += tmp[p]; acc[p + 1] += tmp[p + 1]; acc[p + 2] += tmp[p + 2];
        }
      }
  }
  free(tmp);
  return 0;
}

/* Seed of raytracer.glsl:2120 for the fragment centre (fx, fy). */
float or_pixel_seed(float fx, float fy, unsigned frame) {
  return or_hash(fx * 12.9898f + fy * 78.233f + 1113.1f * (float)frame);
}
