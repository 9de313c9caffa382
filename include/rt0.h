/*
 * rt0.h -- C ABI of the MI355X (gfx950) path-tracing backend for raytracer-0.
 *
 * Drop-in boundary.  The reference drives its integrator through WebGL2
 * (index.js `class GlslViewport`): compile-time strings spliced into the shader
 * by parseShader (tools.js:22-61), per-pass uniforms and one gl.drawArrays per
 * pass (index.js:986-1105).  This header replaces that GL boundary with plain
 * C entry points; a GlslViewport-compatible host class (JS over N-API, or
 * Python over ctypes) calls them.  Every function returns RT0_OK (0) or a
 * negative RT0_E* code; rt0_last_error() gives the message.  Handles are not
 * reentrant; calls are synchronous unless stated.
 *
 * Pixel layout everywhere: RGBA32F, row-major, row 0 = bottom row
 * (gl_FragCoord.y = 0.5), exactly what glReadPixels returns in the reference.
 */
#ifndef RT0_H
#define RT0_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT0_OK 0
#define RT0_E_ARG (-1)     /* bad argument / parse error */
#define RT0_E_HIP (-2)     /* HIP runtime failure */
#define RT0_E_UNSUPPORTED (-3) /* feature outside the supported set */
#define RT0_E_STATE (-4)   /* call order (e.g. render before set_scene) */

/* defines[] flags, index.js:11-19 (same order) */
#define RT0_USE_CUBEMAP (1u << 0)
#define RT0_USE_PROCEDURAL_SKY (1u << 1)
#define RT0_USE_BIASED_SAMPLING (1u << 2)
#define RT0_USE_BIDIRECTIONAL (1u << 3)
#define RT0_USE_RESTIR (1u << 4)
#define RT0_USE_SPECTRAL (1u << 5)
#define RT0_USE_VOLUMETRICS (1u << 6)

/* constants[], index.js:21-35 (same order and meaning) */
typedef struct rt0_config {
  uint32_t defines;            /* RT0_USE_* bits */
  int32_t max_bounces;         /* MAX_BOUNCES */
  int32_t max_diff_bounces;    /* MAX_DIFF_BOUNCES */
  int32_t max_spec_bounces;    /* MAX_SPEC_BOUNCES */
  int32_t max_trans_bounces;   /* MAX_TRANS_BOUNCES */
  int32_t max_scattering_events; /* MAX_SCATTERING_EVENTS */
  int32_t marching_steps;      /* MARCHING_STEPS */
  float fudge_factor;          /* FUDGE_FACTOR */
  int32_t sample_lights;       /* sample_lights */
  int32_t use_mis;             /* use_mis */
  int32_t use_restir;          /* use_restir */
  int32_t light_path_length;   /* LIGHT_PATH_LENGTH (unused by the integrator) */
  int32_t restir_samples;      /* RESTIR_SAMPLES */
  int32_t render_mode;         /* RENDER_MODE: 0 progressive sum, 1 animated (EMA + getAnimatedPosition) */
} rt0_config;

/* Mesh record = the reference's `Mesh` struct (raytracer.glsl:239-244) with its
 * `Material` (157-163) flattened.  type: 0 SPHERE 1 PLANE 2 BOX 3 SDF.
 * mat_type: 0 LIGHT 1 DIR_LIGHT 2 DIFF 3 SPEC 4 REFR_FRESNEL 5 REFR_SCHLICK 6 COAT.
 * type 5 TRIANGLE (raytracer.glsl:236): an instance of triangle model k
 *   (k-th TRIANGLE entry; geometry from rt0_set_model) translated by pos and
 *   scaled by joker.x (0 = skipped, like every mesh with joker.x == 0).
 * tex_type: the material's `Texture.t` (raytracer.glsl:112-121): -1 NULL_TEX,
 *   0..3 TEXTURE0..3 (image units, rt0_set_texture), 4 VORONOI, 5 GRADIENT_NOISE,
 *   6 VALUE_NOISE, 7 CHECK, 8 RIPPLE, 9 METAL (4/6/9 read the noise texture).
 * tex_c_mask / tex_e_mask / tex_params: the rest of that `Texture` (124-128).
 * mat_opts: Material.opts (161) as bits -- 1 colour texture, 2 emission /
 *   glossiness texture, 4 bump (unused by the reference), 8 backface flag.
 * sdf_kind (type == SDF only): the index.html:702-717 selector value
 * (0 sdBox 1 udRoundBox 2 sdSphere 3 sdTriPrism 4 sdCone 5 MengerSponge 6 Mandelbulb). */
typedef struct rt0_mesh {
  float c[3];
  float e[3];
  float nt;
  int32_t mat_type;
  int32_t tex_type;
  int32_t type;
  float pos[3];
  float joker[4];
  int32_t sdf_kind;
  float tex_c_mask[3];
  float tex_e_mask[3];
  float tex_params[4];
  uint32_t mat_opts;
} rt0_mesh;

typedef struct rt0_ctx rt0_ctx;

/* Replaces `new GlslViewport(canvas, opts)` (index.js:4-382): allocates the
 * accumulator + ReSTIR buffers for a width x height canvas on `device`, with
 * GlslViewport's default defines/constants/camera (index.js:11-35, 89-95). */
int rt0_create(int width, int height, int device, rt0_ctx **out);
void rt0_destroy(rt0_ctx *ctx);
const char *rt0_last_error(const rt0_ctx *ctx);

/* Parses GlslViewport's `defines` / `constants` string arrays (index.js:11-35,
 * the text parseShader splices at `#constants`) into *out. */
int rt0_parse_config(const char *const *defines, int n_defines, const char *const *constants,
                     int n_constants, rt0_config *out);
/* Replaces the recompile after a defines/constants change (index.html:1167-1196). */
int rt0_set_config(rt0_ctx *ctx, const rt0_config *cfg);
int rt0_get_config(const rt0_ctx *ctx, rt0_config *out);

/* Replaces `#scene` + `#sdf_meshes` substitution (tools.js:48-55): parses
 * GlslViewport.scene (the GLSL `Mesh[]` / `light_index[]` text of index.js:54-85
 * or index.html:657-676) and the sdf_meshes statements (index.html:702-717). */
int rt0_set_scene_glsl(rt0_ctx *ctx, const char *scene_text, const char *const *sdf_meshes, int n_sdf);
/* Same from already-flattened records; meshes[0..n_meshes) are Euclidean,
 * then n_sdfs SDFs, then n_models TRIANGLE instances (the reference's
 * meshes[NUM_MESHES + NUM_SDFS + NUM_MODELS], index.html:669); light_index as
 * in the GLSL scene. */
int rt0_set_scene(rt0_ctx *ctx, const rt0_mesh *meshes, int n_meshes, int n_sdfs, int n_models,
                  const int32_t *light_index, int n_lights);
/* Pure parser (no device needed): scene text + sdf statements -> records.
 * Fails with RT0_E_ARG if max_meshes / max_lights are too small. */
int rt0_parse_scene_glsl(const char *scene_text, const char *const *sdf_meshes, int n_sdf, rt0_mesh *meshes,
                         int max_meshes, int *n_meshes, int *n_sdfs, int *n_models, int32_t *light_index,
                         int max_lights, int *n_lights);
int rt0_get_scene(const rt0_ctx *ctx, rt0_mesh *meshes, int max_meshes, int *n_meshes, int *n_sdfs, int *n_models,
                  int32_t *light_index, int max_lights, int *n_lights);

/* Triangle model k for the k-th TRIANGLE scene entry (replaces the
 * reference's unshipped mesh.js/bvh.js path; its iTriangle is the commented
 * Moller-Trumbore of raytracer.glsl:864-892): positions = n_vertices x 3
 * floats (object space), indices = n_triangles x 3 vertex indices.  Copied.
 * The next render builds one BVH over all instances in world space: a
 * binned-SAH tree on the host (rt0_bvh_sah.cpp, the default), or with
 * RT0_BVH_BUILD=lbvh in the environment the device LBVH of rt0_bvh.hip
 * (Morton codes + radix sort + Karras hierarchy + refit).  Traversal is part
 * of intersection() (after the quadrics, before the SDF march).  rt0_model_info builds now if needed and reports the triangle count
 * and tree depth (RT0_E_UNSUPPORTED if deeper than the traversal stack). */
int rt0_set_model(rt0_ctx *ctx, int model, const float *positions, int n_vertices, const int32_t *indices,
                  int n_triangles);
int rt0_model_info(rt0_ctx *ctx, int *n_triangles, int *bvh_depth);
/* Wavefront OBJ (v / f records; polygons fan-triangulated; v/vt/vn and
 * negative indices accepted) -> malloc'd positions / indices (rt0_free). */
int rt0_obj_read(const char *path, float **positions, int *n_vertices, int32_t **indices, int *n_triangles);

/* Asset textures, replacing GlslViewport.loadTexture (index.js:699-728) for
 * the image textures opts.textures[0..3] (units u_tex0..3, index.js:276-296)
 * and the RGBA noise image rgba_noise256.png (u_rnd_tex, index.js:258-273):
 * unit 0..3 = TEXTURE0..3, RT0_TEX_NOISE = the noise texture.  rgba8: w*h RGBA
 * bytes, first row = the image's top row (WebGL's upload without FLIP_Y puts
 * it at t = 0); sampled GL_LINEAR with GL_REPEAT at level 0 like the
 * reference, by the filter rt0_set_texture_filter selects.  rgba8 = NULL unbinds the unit (an unbound unit samples
 * (0,0,0,1), the GL value of an incomplete texture).  Copied to the device;
 * the caller keeps ownership. */
#define RT0_TEX_NOISE 4
int rt0_set_texture(rt0_ctx *ctx, int unit, int w, int h, const uint8_t *rgba8);

/* The environment cubemap (u_cubemap, used with USE_CUBEMAP), replacing the
 * load_cubemap promise of index.js:298-331: six size x size RGB8 faces in the
 * reference's upload order -X, -Y, -Z, +X, +Y, +Z (index.js:301-302; the
 * page passes left, bottom, back, right, top, front, index.html:267-270),
 * each first row = the image's top row (t = 0).  Sampled GL_LINEAR on the
 * selected face with its edges clamped.  faces = NULL unbinds (samples
 * (0,0,0,1)).  Copied; the caller keeps ownership. */
int rt0_set_cubemap(rt0_ctx *ctx, int size, const uint8_t *const faces[6]);

/* Uniforms u_camPos, u_camLookAt (a direction), u_camParams = (fov deg,
 * aperture, focal length) (index.js:421-423). */
int rt0_set_camera(rt0_ctx *ctx, const float pos[3], const float lookat[3], const float params[3]);

/* Replaces n_passes consecutive GlslViewport.render() calls (index.js:986-1105)
 * with u_frame = first_frame .. first_frame+n_passes-1: each pass adds one
 * sample per pixel to the accumulator (raytracer.glsl:2168) and, with ReSTIR,
 * rotates the reservoir swap chain (index.js:795-820).  Synchronous.
 * time_ms is u_time (index.js:1011), read only by RENDER_MODE 1: every pass of
 * the call sees the scene at that time (getAnimatedPosition,
 * raytracer.glsl:263-298) and the accumulator becomes the running average
 * mix(prev, sample, 1/temporal_frames) (2159-2165). */
int rt0_render(rt0_ctx *ctx, uint32_t first_frame, int n_passes, float time_ms);
/* Asynchronous variant on the context's stream; rt0_sync() waits. */
int rt0_render_async(rt0_ctx *ctx, uint32_t first_frame, int n_passes, float time_ms);
int rt0_sync(rt0_ctx *ctx);
/* gl.viewport of the passes (tile rendering: index.js:379, updateTile
 * 761-792): only pixels x in [x, x+w), y in [y, y+h) (row 0 = bottom) are
 * rendered, the rest of the accumulator is left untouched; clipped to the
 * canvas.  w or h <= 0 restores the whole canvas.  Not with rt0_set_shard. */
int rt0_set_viewport(rt0_ctx *ctx, int x, int y, int w, int h);
/* u_temporalFrames (GlslViewport.temporalFrames, index.js:236; default 5):
 * the RENDER_MODE 1 running-average length. */
int rt0_set_temporal_frames(rt0_ctx *ctx, int n);

/* Host copy of the accumulator (W*H*4 floats). */
int rt0_read_accum(rt0_ctx *ctx, float *rgba_out);
/* Host copy into / out of the accumulator (resume from a checkpoint). */
int rt0_write_accum(rt0_ctx *ctx, const float *rgba_in);
/* Replaces clear() (index.js:822-880): zero accumulator + all reservoirs. */
int rt0_clear(rt0_ctx *ctx);
/* Replaces resize() (index.js:471-493); contents are cleared. */
int rt0_resize(rt0_ctx *ctx, int width, int height);
int rt0_get_size(const rt0_ctx *ctx, int *width, int *height);

/* Display epilogue, tonemapper.glsl:28-33: rgba8 = 255*pow(acc*cont, 1/2.2),
 * alpha 255, cont = 1/passes (index.js:1089).  RT0_E_UNSUPPORTED on a
 * band-packed accumulator (rt0_set_accum_buffer_compact). */
int rt0_tonemap(rt0_ctx *ctx, float contribution, uint8_t *rgba8_out);
/* Same with a curve: RT0_TONEMAP_GAMMA (= rt0_tonemap), RT0_TONEMAP_ACES
 * (tonemapper.glsl's unused ACESFilm, 17-26, at its exposure 1.5) or
 * RT0_TONEMAP_REINHARD (x/(1+x), the README:22 claim) -- the last two are
 * not used by the reference (parity unpinned); gamma 1/2.2 follows both. */
#define RT0_TONEMAP_GAMMA 0
#define RT0_TONEMAP_ACES 1
#define RT0_TONEMAP_REINHARD 2
int rt0_tonemap_ex(rt0_ctx *ctx, float contribution, int mode, uint8_t *rgba8_out);

/* Image files: PNG for texture assets and the display canvas, PFM
 * for the HDR accumulator.  Host-only, no context needed.
 *   rt0_png_decode / rt0_png_read: 8-bit gray / RGB / palette / gray+alpha /
 *     RGBA, non-interlaced -> RGBA8, row 0 = the file's first row; the buffer
 *     is malloc'd, release it with rt0_free.
 *   rt0_png_write: RGBA8; flip_y = 1 writes row h-1 first (accumulator /
 *     canvas rows are bottom-up, PNG rows top-down).
 *   rt0_pfm_write: RGB float32 of a W*H*4 buffer times `scale` (1/passes),
 *     rows bottom-up as PFM stores them. */
int rt0_png_decode(const uint8_t *data, size_t size, int *w, int *h, uint8_t **rgba_out);
int rt0_png_read(const char *path, int *w, int *h, uint8_t **rgba_out);
int rt0_png_write(const char *path, int w, int h, const uint8_t *rgba, int flip_y);
int rt0_pfm_write(const char *path, int w, int h, const float *rgba, float scale);
/* Baseline JPEG (SOF0, 8-bit, 1 or 3 components, sampling factors 1..2,
 * restart markers; JFIF YCbCr) -> RGBA8, the format of the reference's
 * cubemap faces (the .jpg files under cubemaps/, loaded at index.js:298-331).
 * Progressive / arithmetic / 12-bit files return RT0_E_UNSUPPORTED. */
int rt0_jpeg_decode(const uint8_t *data, size_t size, int *w, int *h, uint8_t **rgba_out);
int rt0_jpeg_read(const char *path, int *w, int *h, uint8_t **rgba_out);
void rt0_free(void *p);

/* ReSTIR reservoir MRTs (raytracer.glsl:2171-2179).  which: 0 = current output
 * (restir_buffer/aux of the last pass), 1 = history1, 2 = history2.  main/aux:
 * W*H*4 floats each (planes, de-interleaved from the device pairs). */
int rt0_read_restir(rt0_ctx *ctx, int which, float *main_out, float *aux_out);
/* Set the six ReSTIR inputs the NEXT pass reads (spatial = restir_buffer_back,
 * history1, history2; main+aux each); any pointer may be NULL = zeros. */
int rt0_write_restir_inputs(rt0_ctx *ctx, const float *spatial_main, const float *spatial_aux,
                            const float *h1_main, const float *h1_aux, const float *h2_main,
                            const float *h2_aux);

/* Pixel sharding for multi-GPU: this context renders only rows
 * r with (r / band) % n_shards == shard.  Its accumulator stays full-size;
 * rows it does not own are left untouched. */
int rt0_set_shard(rt0_ctx *ctx, int shard, int n_shards, int band_rows);

/* Device pointer of the accumulator (W*H*4 f32, hipMalloc'd, owned by ctx) and
 * the HIP stream used for kernels, for zero-copy collectives by the caller. */
int rt0_device_accum(rt0_ctx *ctx, void **dptr, void **stream);
/* Use a caller-owned device buffer (W*H*4 f32 on the ctx's device, e.g. a
 * torch tensor that RCCL gathers) as the accumulator; NULL restores the
 * context's own buffer.  Contents are not cleared. */
int rt0_set_accum_buffer(rt0_ctx *ctx, void *dptr);
/* Same with a band-packed layout for multi-GPU sharding (rt0_set_shard): the
 * buffer holds only this shard's bands, in band order ((*rows) x W x 4 f32,
 * *rows = owned bands x band_rows), so it is the send buffer of the gather
 * as it stands.  Not for ReSTIR (RT0_E_UNSUPPORTED).  rt0_read_accum /
 * rt0_write_accum / rt0_clear then cover these rows; rt0_tonemap* return
 * RT0_E_UNSUPPORTED (gather the bands into an image first), and rt0_render
 * returns RT0_E_STATE once rt0_set_shard changed the rows this shard owns
 * (set the buffer again). */
int rt0_set_accum_buffer_compact(rt0_ctx *ctx, void *dptr, int *rows);

/* Sharded ReSTIR: the reservoir textures of index.js:149-163
 * (units 7-12) and their swap chain (swapReSTIRBuffers, index.js:795-820).
 * A shard renders its row bands of rt0_set_shard -- one contiguous row block
 * when band_rows * n_shards >= height, or several bands dealt round-robin
 * (what bench.py runs: rt0/shard.py interleaved_band), then halo <= band_rows
 * -- one pass per rt0_render call; between passes the caller copies `rows`
 * halo rows of the newest reservoir planes across every band boundary between
 * two shards (rt0/shard.py RestirShard does it over RCCL).
 *   The reservoir textures live as four interleaved main/aux PAIRS: texel i
 *   of a pair is its main RGBA32F then its aux RGBA32F (32 B), so a
 *   bilinear tap reads one 32-B segment per texel instead of one line in each
 *   of two planes (rt0_integrator.h RT0_RES_STRIDE).
 *   rt0_set_restir_buffers: caller-owned device memory (e.g. torch tensors
 *     the collective reads/writes) for the 4 pairs, W*H*8 f32 each, given as
 *     8 plane pointers: planes[2k] = pair k's base (its main plane),
 *     planes[2k+1] = that base + 16 bytes (its aux plane) -- RT0_E_ARG
 *     otherwise; NULL returns to context-owned pairs.  All pairs are cleared.
 *   rt0_device_restir: device pointers of the reservoir planes a following
 *     pass reads: which = 0 newest output (spatial input), 1 / 2 the
 *     temporal history levels; aux = main + 16 bytes (one pair; a row range
 *     of the pair, W*32 B per row, is what a halo exchange moves).
 *   rt0_set_halo: rows of exchanged halo (valid rows around the own block).
 *   rt0_read_halo_misses: bilinear fetches that fell outside own block + halo
 *     since the last reset (non-zero = the halo was too small: the result
 *     differs from the unsharded render). */
int rt0_set_restir_buffers(rt0_ctx *ctx, void *const planes[8]);
int rt0_device_restir(rt0_ctx *ctx, int which, void **main_out, void **aux_out);
int rt0_set_halo(rt0_ctx *ctx, int rows);
int rt0_read_halo_misses(rt0_ctx *ctx, uint32_t *misses, int reset);

/* Scene-specialised kernels (default on; env RT0_JIT=0 turns the default off):
 * like the reference recompiling its shader per scene (index.html:1167), the
 * integrator is compiled by hipRTC with the scene and the constants baked in,
 * once per (scene, config), cached per process.  0 = ahead-of-time kernels
 * that read the scene from HBM. */
int rt0_set_jit(rt0_ctx *ctx, int enable);
/* Reference-executor compatibility for the ReSTIR reservoir outputs (MRT1/2,
 * raytracer.glsl:2171-2174).  The golden vectors come from the reference
 * shader run on SwiftShader 4.1, which after a lane's `break` out of
 * radiance()'s bounce loop still runs that iteration's brdf() call
 * (raytracer.glsl:2094) and lets it overwrite the global g_final_reservoir
 * (1757) -- a GLES execution artefact, pinned by oracle/gen/mask_kat.py.
 * 1 = reproduce it (the reservoir chain then matches the reference executor
 * pass after pass); 0 (default) = GLSL semantics.  Radiance of a pass is the
 * same either way; only the reservoirs the next passes read differ.
 * (The texture filter is its own switch, rt0_set_texture_filter.) */
int rt0_set_executor_compat(rt0_ctx *ctx, int enable);
/* GL_LINEAR filtering of the RGBA8 asset textures (u_tex0..3) and the noise
 * texture (u_rnd_tex), getTexel and value_noise / voronoi (raytracer.glsl:
 * 393-433, 726-772) on the textures of loadTexture (index.js:699-728).  GLSL
 * leaves the filter's precision to the implementation; GPU texture units,
 * like the reference's executor, filter in fixed point.
 *   RT0_TEX_FILTER_FIXED16 (default): the reference executor's filter -- the
 *     coordinate as a 16-bit fraction, a 16.16 texel position, texels widened
 *     to 16 bits, 16-bit tap weights (oracle/gen/tex_kat.py known-answer
 *     shaders; bit-exact on power-of-two textures, every reference asset);
 *   RT0_TEX_FILTER_FLOAT: exact fp32 bilinear.
 * The cubemap is filtered in fp32 either way (the executor does too). */
#define RT0_TEX_FILTER_FLOAT 0
#define RT0_TEX_FILTER_FIXED16 1
int rt0_set_texture_filter(rt0_ctx *ctx, int mode);
/* Deferred ReSTIR light sampling (scene-specialised kernels): a pass runs its
 * paths with every sampleLightsReSTIR call (raytracer.glsl:1619-1801)
 * appended to a per-wave list, evaluates the list in a second kernel with
 * every lane busy, and completes the samples in a last one (resolve).  In
 * scenes with triangle models (RENDER_MODE 0, no SDFs, no textured lights)
 * a third kernel between them answers the calls' triangle occlusion queries
 * (the visibility and shadow rays) on dense lanes: four dispatches per pass.
 * Without that kernel the light-sampling kernel completes its pixels'
 * samples itself (two dispatches per pass; RT0_FUSED_RESOLVE=0 in the
 * environment when the module is built keeps the third: bit-identical).
 * Same arguments and arithmetic as the inline calls, but NOT bitwise equal:
 * FMA placement can differ, and a sample's fp32 additions run in another
 * order (the path's own radiance first, then the light-sampling results in
 * call order, instead of interleaved per bounce).  tests/test_gpu_defer.py
 * holds samples within 1e-5 and reservoirs within 1e-4 relative of the
 * inline calls, >= 98% of each bit-identical.
 * 1 (default; RT0_DEFER_NEE=0 in the environment at rt0_create turns it
 * off) or 0 = inline calls.  Executor compatibility always runs them inline.
 * Replaces nothing in the reference: the GL pipeline has no such choice. */
int rt0_set_defer_light_sampling(rt0_ctx *ctx, int enable);
/* Wavefront rounds.  mode 1 (default): SDF scenes (scene-specialised
 * kernels, no ReSTIR, no triangle models, no SDF light): a pass runs as
 * MAX_BOUNCES + 2 rounds of a shade kernel (each path's bounce up to its next
 * SDF march) and a march kernel (every pending sphere trace, normal and shadow
 * march on lanes that refill as they finish), the launch's passes side by
 * side; samples are added in pass order (rt0_integrator.h wf_shade_body).
 * The same map() steps as the pass kernel; light-sampling sums are formed in
 * call order one round later, so FMA placement can differ at the last bit
 * (tests/test_gpu_wavefront.py).  mode 2: also the deferred ReSTIR passes of
 * scenes with triangle models -- shade rounds and a closest-hit walk kernel
 * (wf_restir_shade_body, wf_walk_body); the same walks and hits, measured
 * slower than the pass kernel on BASELINE config 5, hence not
 * the default.  0 = the pass kernel.  RT0_WAVEFRONT=<mode> in the environment
 * sets the default at rt0_create.  Replaces nothing in the reference. */
int rt0_set_wavefront(rt0_ctx *ctx, int mode);
/* Compile the scene-specialised kernel for (scene, config) without a device
 * (hipRTC only): checks the generated code builds; *code_size receives the
 * code-object size.  err (may be NULL) receives the compiler log. */
int rt0_jit_compile(const char *scene_text, const char *const *sdf_meshes, int n_sdf, const rt0_config *cfg,
                    size_t *code_size, char *err, size_t err_len);

/* Event counters of the last rt0_render call when enabled: [0] intersection()
 * calls, [1] radiance-loop iterations, [2] light-sampling (NEE) calls,
 * [3] map() evaluations, [4] samples.  Counting uses a separate kernel
 * instance; it never runs in a timed render unless enabled. */
int rt0_set_counting(rt0_ctx *ctx, int enable);
int rt0_read_counters(rt0_ctx *ctx, uint64_t out[5]);
/* All event counters (the first five as above), for the FLOP model of the
 * ReSTIR and triangle-model workloads: [5] sampleLightsReSTIR calls,
 * [6] ReSTIR candidates evaluated (raytracer.glsl:1635-1654), [7] temporal
 * history taps read (1485-1523), [8] spatial taps read (1725-1748), [9] BVH
 * nodes visited, [10] triangle tests.  Copies min(n, RT0_N_COUNTERS) values
 * (zero-fills the rest); returns RT0_N_COUNTERS. */
#define RT0_N_COUNTERS 11
int rt0_read_counters_n(rt0_ctx *ctx, uint64_t *out, int n);

/* Wall time of the kernels of the last rt0_render (HIP events on the
 * context's stream), milliseconds, and the number of kernel launches (a
 * ReSTIR pass with deferred light sampling -- three dependent dispatches on the
 * stream: path, light sampling, resolve -- counts as one, and so does a
 * frame-chunked launch: the pass kernel and the frame-order sum after it). */
int rt0_last_kernel_ms(const rt0_ctx *ctx, float *ms, int *launches);
/* Which kernels the last rt0_render ran: RT0_PATH_* (0 before any render). */
#define RT0_PATH_AOT 1        /* the ahead-of-time pass kernels (rt0_set_jit(0), counting) */
#define RT0_PATH_PASS 2       /* the scene-specialised pass kernel */
#define RT0_PATH_DEFERRED 3   /* ReSTIR: pass + light sampling (+ walk) + resolve */
#define RT0_PATH_WAVEFRONT 4  /* wavefront shade + march / walk rounds (rt0_set_wavefront) */
int rt0_last_render_path(const rt0_ctx *ctx);
/* Bytes of device scratch the context holds beyond the accumulator and the
 * reservoir planes: per-frame sample planes of frame-chunked launches (over
 * the launch rectangle), the wavefront rounds' path state (bounded by
 * RT0_WF_BYTES, default 8 GiB: a frame that does not fit runs as slot chunks;
 * released when a render no longer takes the wavefront path), and the
 * deferred ReSTIR records, result planes and walk jobs.  Grows on demand. */
int rt0_scratch_bytes(const rt0_ctx *ctx, size_t *bytes);

/* Library version string. */
const char *rt0_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT0_H */
