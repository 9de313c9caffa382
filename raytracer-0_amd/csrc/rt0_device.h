// rt0_device.h -- data layout shared by the host library and the gfx950 kernels.
//
// HBM layout (one context):
//   SceneDev  (one struct, ~9 KiB): geometry records, material records,
//             light_index, sdf kinds.  Read with wave-uniform indices only, so
//             the compiler emits scalar (s_load) fetches: the scene never
//             occupies VGPRs or vector-memory bandwidth.
//   accum     W*H float4 (RGBA32F), row 0 = bottom row.
//   ReSTIR    8 W*H float4 planes: out main/aux, spatial-in main/aux,
//             history1 main/aux, history2 main/aux (index.js:125-221 swap chain
//             kept as pointer rotation on the host).
#pragma once
#include <stdint.h>

#define RT0_MAX_MESH 128
#define RT0_MAX_LIGHTS 128

// Geometry half of raytracer.glsl's `Mesh` (239-244), 32 B.  Derived fields
// are exact rewrites of the reference's per-test arithmetic:
//   SPHERE: r2 = joker.x*joker.x (iSphere, 821)
//   PLANE : negd = -joker.x (iPlane, 813)
//   BOX   : half = joker.x*0.5 (a power-of-two scale: (|m|*jx)*0.5 == |m|*(jx*0.5))
struct GeomRec {
  float px, py, pz;
  float j0;      // joker.x (0 => skipped, raytracer.glsl:1009)
  int32_t type;  // 0 SPHERE 1 PLANE 2 BOX 3 SDF
  float d0;      // r2 / negd / half
  float j1, j2;  // joker.y, joker.z
};

// Material half, 32 B.  c/e are the raw material colours; the integrator
// applies max(.,0.001) where the reference does (raytracer.glsl:2071, 2077).
struct MatRec {
  float cr, cg, cb;
  int32_t type;  // 0 LIGHT 1 DIR_LIGHT 2 DIFF 3 SPEC 4 REFR_FRESNEL 5 REFR_SCHLICK 6 COAT
  float er, eg, eb;
  float nt;
};

// Material texture, raytracer.glsl:124-128 (`Texture`) + Material.opts (161),
// 48 B.  type -1 = NULL_TEX; opts bit 0 = colour texture, bit 1 = emission.
struct TexRec {
  float cmr, cmg, cmb;
  int32_t type;
  float emr, emg, emb;
  uint32_t opts;
  float p0, p1, p2, p3;
};

// Asset texture units (index.js:149-163): 0..3 = u_tex0..3, 4 = u_rnd_tex.
#define RT0_TEX_UNITS 5

// Triangle models (TRIANGLE scene entries, raytracer.glsl:236; the
// reference's commented-out iTriangle, 864-892).  One LBVH over the triangles
// of all models, built on the device (rt0_bvh.hip) in world space:
//   TriDev  48 B: v0 + model index, e0 = v1 - v0, e1 = v2 - v0 (the three
//           Moller-Trumbore operands) + the determinant threshold, stored in
//           leaf order;
//   BvhNode 64 B: both children's boxes + child links (>= 0 internal node,
//           < 0 leaf ~triangle), so one node fetch tests two boxes.
struct TriDev {
  float v0x, v0y, v0z;
  int32_t model;  // owner model k (scene entry n_meshes + n_sdfs + k)
  float e0x, e0y, e0z;
  int32_t cull;   // Material.opts[3]: back-face culling (iTriangle, 869-872)
  float e1x, e1y, e1z;
  float eps;      // EPSILON * |e0| * |e1|: iTriangle's parallel-ray threshold, scale-invariant
};
#define RT0_TRI_CULL_BIT (1 << 30)  // set in the build's model ids for culling models
struct BvhNode {
  float lx0, ly0, lz0, rx0;
  float lx1, ly1, lz1, ry0;
  float rz0, rx1, ry1, rz1;
  int32_t left, right, pad0, pad1;
};
#ifndef RT0_BVH_STACK
#define RT0_BVH_STACK 48  // traversal stack entries per lane (LDS); the build checks the bound
#endif

// Deferred light sampling (ReSTIR scenes, scene-specialised kernels): the
// pass kernel appends one NeeRec per sampleLightsReSTIR call instead of
// running it (its result only adds to the path's radiance; the path's next
// direction does not depend on it), rt0_jit_nee evaluates the records densely
// -- every lane has one -- and rt0_jit_resolve adds them to the pixel's
// sample in bounce order.  60 B.  Each wave of the pass kernel owns a region
// of nee_cap records (64 lanes x max_bounces calls) that it fills in call
// order through an LDS counter -- no device-wide atomic, whose single address
// serialises every wave of the chip -- and the NEE kernel gives each region to
// one wave, so a wave's records are one 8x8 tile's calls (coherent taps).
struct NeeRec {
  float x, y, z;     // the shading point (hit.pos)
  float nx, ny, nz;  // nl
  float mr, mg, mb;  // the path's mask at the call
  int32_t pix;       // image pixel (y * W + x)
  uint32_t mkb;      // the hit mesh (material) | the call's index along the path << 8 | the bounce << 16
  uint32_t pad;
  // sampleLightsReSTIR's two seeds (raytracer.glsl:1909/1943) are recomputed
  // from the pixel, the pass and the bounce (Integrator::restir_seeds)
  __host__ __device__ int mat() const { return (int)(mkb & 0xffu); }
  __host__ __device__ int k() const { return (int)((mkb >> 8) & 0xffu); }
  __host__ __device__ int bounce() const { return (int)(mkb >> 16); }
};
static_assert(sizeof(NeeRec) == 48, "NeeRec is 12 words: three 16-B loads");
// the packed fields' ranges: mat < RT0_MAX_MESH fits 8 bits; a path makes at
// most one deferred call per bounce, so k < max_bounces and bounce <
// max_bounces -- deferral is used only while max_bounces fits the 8-bit k
// (rt0_host.cpp, rt0_jit_compile); deeper configs keep the inline calls
#define RT0_NEE_MAX_BOUNCES 255
static_assert(RT0_MAX_MESH <= 256, "NeeRec::mat is 8 bits");
static_assert(RT0_NEE_MAX_BOUNCES <= 255 && RT0_NEE_MAX_BOUNCES < 65536, "NeeRec::k is 8 bits, bounce 16");

// RT0_NEE_WALK (scenes with triangle models): a light-sampling call's
// triangle occlusion queries go to rt0_jit_walk as WalkJobs, 32 B: the ray
// and its bound, and `slot2` = 2 * the call's record slot + which ray (0 =
// visibility, 1 = shadow ray); the answer (1 = occluded) goes to
// walk_res[slot2].  The call's result plane entry then holds its result as it
// is if both rays pass, and w = a tag ((slot + 1) << 2 | 1 if the visibility
// ray was walked | 2 if the shadow ray was) as int bits, which
// rt0_jit_resolve reads (a finished call's w is 0.0f).
struct WalkJob {
  float ox, oy, oz, tmax;
  float dx, dy, dz;
  uint32_t slot2;
};
static_assert(sizeof(WalkJob) == 32, "WalkJob is 32 B");

struct SceneDev {
  int32_t n_meshes, n_sdfs, n_lights, n_total;
  int32_t n_models;  // TRIANGLE entries: geom/mat[n_meshes + n_sdfs + k]
  int32_t any_tex;  // some mesh has tex.type != NULL (texel code runs at all)
  GeomRec geom[RT0_MAX_MESH];
  MatRec mat[RT0_MAX_MESH];
  TexRec tex[RT0_MAX_MESH];
  float j3[RT0_MAX_MESH];  // joker.w (udRoundBox radius)
  int32_t sdf_kind[RT0_MAX_MESH];
  int32_t light_index[RT0_MAX_LIGHTS];
};

// Feature flags resolved on the host (runtime, wave-uniform).
enum : uint32_t {
  F_SKY = 1u << 0,
  F_BIASED = 1u << 1,
  F_SAMPLE_LIGHTS = 1u << 2,
  F_MIS = 1u << 3,
  F_RESTIR = 1u << 4,      // use_restir constant
  F_RESTIR_DEF = 1u << 5,  // #define USE_RESTIR
  F_SPECTRAL = 1u << 6,
  F_VOL = 1u << 7,
  F_CUBEMAP = 1u << 8,  // #define USE_CUBEMAP
  F_ANIM = 1u << 9,     // RENDER_MODE 1 (animated: getAnimatedPosition + EMA accumulator)
  // Reference-executor compatibility (rt0_set_executor_compat): reproduce how
  // the oracle's GLES executor stores g_final_reservoir after a `break` of the
  // bounce loop (oracle/gen/mask_kat.py).  Off = GLSL semantics.
  F_EXEC_GHOST = 1u << 10,
  // RGBA8 asset / noise textures through the fixed-point bilinear filter the
  // reference's executor uses (rt0_set_texture_filter, default on)
  F_TEX_FIXED = 1u << 11,
};

struct LaunchParams {
  int32_t width, height;
  uint32_t frame0;
  int32_t nframes;
  float res_x, res_y, aspect;
  float cam_px, cam_py, cam_pz;
  float ux, uy, uz, vx, vy, vz, wx, wy, wz;
  float uULen, uVLen, aperture, focal;
  uint32_t flags;
  int32_t max_bounces, max_diff, max_spec, max_trans, max_scatter, marching_steps;
  float fudge;
  int32_t restir_samples;
  int32_t shard, n_shards, band;  // row-band sharding
  int32_t n_band_rows;            // rows covered by this launch's grid (host-computed)
  // gl.viewport rectangle of the pass (tile rendering, index.js:761-792):
  // columns [vp_x0, vp_x1) x band rows [vp_y0, vp_y1); the whole canvas by default
  int32_t vp_x0, vp_y0, vp_x1, vp_y1;
  const SceneDev *scene;
  float4 *accum;
  int32_t compact;  // accum holds only this shard's bands: row r of the band-compressed grid
  const float4 *rin[6];  // spatial main/aux, history1 main/aux, history2 main/aux
  float4 *rout_main, *rout_aux;
  unsigned long long *counters;  // RT0_N_COUNTERS x u64 (counting instance only)
  // Sharded ReSTIR: rows [valid_lo, valid_hi) of the input reservoir planes hold
  // data (own block + exchanged halo); a bilinear fetch outside them bumps
  // *halo_miss (null when the whole image is local).
  int32_t valid_lo, valid_hi;
  // halo_rows > 0: the shard owns the row bands b with b % n_shards == shard
  // (several per shard when band * n_shards < height) and holds `halo_rows`
  // exchanged rows on either side of each; a fetch elsewhere bumps *halo_miss
  int32_t halo_rows;
  uint32_t *halo_miss;
  // the same check without integer division (row_local): 1/band and
  // 1/n_shards as floats, and the shards that own the bands next to ours
  float band_inv, shards_inv;
  int32_t shard_next, shard_prev;  // (shard + 1) % n_shards, (shard - 1) mod n_shards
  // Frame-chunked launch (few pixels per device, e.g. 8-way sharding): grid.z
  // = chunk index, each lane renders frames [z*frame_chunk, +frame_chunk) of
  // its pixel into samples[frame][launch pixel]; rt0_sum_kernel then adds them
  // to the accumulator in frame order (the same sequential sum).  samples ==
  // null: one chunk, accumulated in registers.
  int32_t frame_chunk;
  float4 *samples;
  // Executor compatibility, rule 11 (oracle/gen/mask_kat.py QUAD LIGHTS;
  // Integrator::light_q): per image pixel the bounces at which its path ran
  // brdf()'s light loop (x) and a ghost call's unrolled loop (y).  quad_mode 1:
  // this launch records them (its samples are discarded); 2: every lane
  // reads its 2x2 quad's first lane's record; 0: neither.
  uint2 *quad_masks;
  int32_t quad_mode;
  // BVH nodes [0, treelet) are the tree's top levels, staged in LDS by the
  // scene-specialised kernels that walk it (rt0_integrator.h bvh_fetch)
  int32_t treelet;
  // Asset textures: RGBA8 texels (R in the low byte), row 0 = t 0; null =
  // unbound unit.
  const uint32_t *tex_img[RT0_TEX_UNITS];
  int32_t tex_w[RT0_TEX_UNITS], tex_h[RT0_TEX_UNITS];
  // Cubemap (u_cubemap): 6 faces of cube_size^2 RGBA8 texels in GL face
  // order +X -X +Y -Y +Z -Z, row 0 = t 0; null = unbound.
  const uint32_t *cube;
  int32_t cube_size;
  // Triangle models: LBVH nodes (root 0) and triangles in leaf order; n_tris 0 = none.
  const BvhNode *bvh;
  const TriDev *tris;
  int32_t n_tris;
  // RENDER_MODE 1 (F_ANIM): the accumulator is an EMA with weight ema_alpha =
  // 1/u_temporalFrames (raytracer.glsl:2159-2165), and apos[i] is
  // getAnimatedPosition(meshes[i].pos, i, u_time) (263-298), evaluated once
  // per launch on the host (it is uniform over the image).  Unused otherwise.
  float ema_alpha;
  // deferred light sampling (NeeRec): defer != 0 routes sampleLightsReSTIR
  // calls into its region nee_rec[wave * nee_cap ...], nee_count[wave] = the
  // records the wave wrote (wave = (blockIdx.y * gridDim.x + blockIdx.x) * 4
  // + threadIdx.x / 64 of the pass grid); results go to
  // nee_out[k * width * height + pix]; nee_partial[pix] = (the path's radiance
  // without them, hero wavelength), nee_n[pix] = its number of calls
  int32_t defer, nee_cap, nee_regions;  // nee_regions = pass waves (entries of nee_count)
  NeeRec *nee_rec;
  uint32_t *nee_count;
  float4 *nee_out, *nee_partial;
  int32_t *nee_n;
  // RT0_NEE_WALK: walk_jobs[w * walk_cap ...] = light-sampling wave w's
  // jobs (walk_count[w] of them, walk_cap = 2 * RT0_NEE_REGIONS * nee_cap),
  // walk_res[2 * record slot + ray]; walk_waves = light-sampling waves
  WalkJob *walk_jobs;
  uint32_t *walk_count, *walk_res;
  int32_t walk_waves;
  // Wavefront SDF renders (RT0_WAVEFRONT modules: rt0_jit_wf_shade +
  // rt0_jit_wf_march, rt0_integrator.h "wavefront SDF renders").  A launch's
  // samples are `wf_slots` path slots (frame-major, then the pass grid's tile
  // order, wf_apad slots per frame, frames [wf_f0, wf_f0 + wf_slots /
  // wf_apad) of the launch); region w = slots [w * wf_R, (w + 1) * wf_R) is
  // one shade wave's.  Per round: the shade kernel reads region w of the
  // previous round's march list (wf_in: 2 float4 per entry = ray + bound,
  // direction + slot; wf_in_cnt[w] entries) and its results (wf_res, same
  // index), and writes region w of this round's march list (wf_out,
  // wf_out_cnt) and shadow list (wf_sh: 3 float4 per entry, capacity wf_R *
  // wf_L per region, wf_sh_cnt); the march kernel takes regions off
  // wf_ctr[16 * k] (one counter per eighth of the regions) and answers them
  // (wf_res; wf_shres[light * wf_slots + slot]).
  // Path state between rounds: SDF rounds keep it in list order, beside the
  // march list: wf_sin[k * wf_cap + entry] is the state of region entry
  // `entry` of wf_in, and the shade kernel writes wf_sout[k * wf_cap + o] for
  // the entry o it appends to wf_out (coalesced, like the lists; the two
  // swap every round); ReSTIR rounds keep wf_state[k * wf_slots + slot].
  int32_t wf_round, wf_R, wf_L, wf_nregions, wf_f0;
  uint32_t wf_apad, wf_slots, wf_gx;
  uint32_t wf_slot0;  // the launch's first slot of this part (a wavefront half on its own stream)
  uint32_t *wf_ctr;
  // the round's non-empty regions (wf_plan_body): plan block b's at
  // wf_plan[4 * (b * wf_plan_span ...)], their number and entries per block
  uint32_t *wf_plan, *wf_plan_bn, *wf_plan_bj;
  int32_t wf_plan_blocks, wf_plan_span;
  float4 *wf_state;
  float4 *wf_sin, *wf_sout;
  uint32_t wf_cap;  // entries per state component (the half's regions x wf_R)
  float4 *wf_in, *wf_out;
  uint32_t *wf_in_cnt, *wf_out_cnt, *wf_sh_cnt;
  float4 *wf_res;
  float *wf_res_id;
  float4 *wf_sh, *wf_shres;
  float4 apos[RT0_MAX_MESH];
};
