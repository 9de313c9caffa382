'use strict';
/*
 * glsl_viewport.js -- GlslViewport on the MI355X rt0 backend.
 *
 * Same constructor, fields and methods the reference's page script uses on its
 * `sandbox` object (index.js:3-1105, index.html:259-1387): defines, constants,
 * animatedConstants, scene, sdf_meshes, camera, passes, max_passes, render(),
 * clear(), resize(v), setAnimatedMode(b), updateFrontTarget().  The shader
 * pipeline is replaced by the rt0 C ABI (include/rt0.h) through the N-API
 * addon rt0.node: a change of defines/constants/scene is picked up at the next
 * render() (the reference needs recompile(), index.html:1167-1196).
 * Backends: opts.backend = 'hip' (default) renders through librt0 on an
 * MI355X -- without a HIP device the constructor throws, there is no silent
 * fallback; opts.backend = 'cpu' renders with the JS integrator on the host
 * (cpu_backend.js; BASELINE configs[0], the reference's "JS CPU fallback").
 */
const path = require('path');

let _addon = null;
function addonModule() {  // loaded on first use: the CPU backend needs no librt0
  if (!_addon) _addon = require(path.join(__dirname, 'rt0.node'));
  return _addon;
}

// The HIP backend: the N-API addon's calls on one librt0 context
class AddonBackend {
  constructor(width, height, device) {
    this.kind = 'hip';
    this.a = addonModule();
    this.h = this.a.create(width, height, device);
  }
  setExecutorCompat(on) { this.a.setExecutorCompat(this.h, on); }
  setTextureFilter(mode) { this.a.setTextureFilter(this.h, mode); }
  setCubemap(size, faces) { this.a.setCubemap(this.h, size, faces); }
  setTexture(unit, w, h, data) { this.a.setTexture(this.h, unit, w, h, data); }
  setConfig(defines, constants) { this.a.setConfig(this.h, defines, constants); }
  setScene(scene, sdf) { this.a.setScene(this.h, scene, sdf); }
  setCamera(pos, look, params) { this.a.setCamera(this.h, pos, look, params); }
  setViewport(x, y, w, h) { this.a.setViewport(this.h, x, y, w, h); }
  setTemporalFrames(n) { this.a.setTemporalFrames(this.h, n); }
  render(first, n, t) { this.a.render(this.h, first, n, t); }
  clear() { this.a.clear(this.h); }
  resize(w, h) { this.a.resize(this.h, w, h); }
  readAccum() { return this.a.readAccum(this.h); }
  tonemap(cont) { return this.a.tonemap(this.h, cont); }
  lastKernelMs() { return this.a.lastKernelMs(this.h); }
  setWavefront(mode) { this.a.setWavefront(this.h, mode); }
  lastRenderPath() { return this.a.lastRenderPath(this.h); }
}

function readImage(p) { return addonModule().readImage(p); }

// vector.js:2-95, the part the camera uses
class Vector3 {
  constructor(x, y, z) {
    this.x = x === undefined ? 0.0 : x;
    this.y = y === undefined ? 0.0 : y;
    this.z = z === undefined ? 0.0 : z;
  }
  toArray() { return [this.x, this.y, this.z]; }
}

// index.html:610-676: scene textarea lines -> the GLSL text spliced at #scene
function sceneFromLines(lines) {
  let nMeshes = 0, nSdfs = 0, nModels = 0;
  let uSphere = false, uPlane = false, uBox = false;
  const lights = [], text = [];
  lines.forEach((line, i) => {
    const fields = line.split(',');
    const mat = fields[0].trim(), type = fields[1].trim();
    if (mat.lastIndexOf('MAT_LIGHT') >= 0) lights.push(i);
    text.push('Mesh(' + line + ')' + (i !== lines.length - 1 ? ',' : ''));
    if (type === 'SDF' || type === 'GRID_SDF') nSdfs++;
    else if (type === 'PLANE' || type === 'SPHERE' || type === 'BOX') {
      uSphere = uSphere || type === 'SPHERE';
      uPlane = uPlane || type === 'PLANE';
      uBox = uBox || type === 'BOX';
      nMeshes++;
    } else if (type === 'TRIANGLE') nModels++;
    else throw new Error("There's no such thing as " + type);
  });
  if (lights.length === 0) lights.push(-1);
  return {
    nSdfs,
    scene: 'const bool U_EUCLIDEAN = ' + (nMeshes > 0) + ';\nconst bool U_SPHERE = ' + uSphere +
      ';\nconst bool U_PLANE = ' + uPlane + ';\nconst bool U_BOX = ' + uBox + ';\nconst bool U_SDF = ' +
      (nSdfs > 0) + ';\n\nconst lowp int NUM_MESHES = ' + nMeshes + ';\nconst lowp int NUM_SDFS   = ' + nSdfs +
      ';\nconst lowp int NUM_MODELS = ' + nModels + ';\n\nconst Mesh meshes[NUM_MESHES + NUM_SDFS + NUM_MODELS] = ' +
      'Mesh[](\n' + text.join('\n') + '\n);\n\nconst lowp int light_index[' + lights.length + '] = int[](\n' +
      lights.join(', ') + '\n);',
  };
}

// index.html:702-717: SDF selector value -> #sdf_meshes statement
const SDF_PRIMS = ['sdBox', 'udRoundBox', 'sdSphere', 'sdTriPrism', 'sdCone', 'MengerSponge', 'Mandelbulb'];
function sdfStatement(i, kind) {
  const m = 'meshes[NUM_MESHES + ' + i + ']';
  const args = [
    `p-${m}.pos, ${m}.joker.xyz`, `p-${m}.pos, ${m}.joker.xyz, ${m}.joker.w`, `p-${m}.pos, ${m}.joker.x`,
    `p-${m}.pos, ${m}.joker.xy`, `p-${m}.pos, ${m}.joker.xyz`, `p-${m}.pos, ${m}.joker.xyz`, `p-${m}.pos`,
  ][kind];
  return `sdf_meshes[${i}] = vec2(${SDF_PRIMS[kind]}(${args}), ${i.toFixed(4)});`;
}

const STATIC_CONSTANTS = [
  'const lowp int MAX_BOUNCES = 12;', 'const lowp int MAX_DIFF_BOUNCES = 4;', 'const lowp int MAX_SPEC_BOUNCES = 4;',
  'const lowp int MAX_TRANS_BOUNCES = 12;', 'const lowp int MAX_SCATTERING_EVENTS = 12;',
  'const mediump int MARCHING_STEPS = 128;', 'const lowp float FUDGE_FACTOR = 0.9;', 'const bool sample_lights = true;',
  'const bool use_mis = false;', 'const bool use_restir = false;', 'const lowp int LIGHT_PATH_LENGTH = 2;',
  'const lowp int RESTIR_SAMPLES = 16;', 'const lowp int RENDER_MODE = 0;',
];
const ANIMATED_CONSTANTS = [
  'const lowp int MAX_BOUNCES = 6;', 'const lowp int MAX_DIFF_BOUNCES = 2;', 'const lowp int MAX_SPEC_BOUNCES = 2;',
  'const lowp int MAX_TRANS_BOUNCES = 4;', 'const lowp int MAX_SCATTERING_EVENTS = 4;',
  'const mediump int MARCHING_STEPS = 64;', 'const lowp float FUDGE_FACTOR = 0.9;', 'const bool sample_lights = true;',
  'const bool use_mis = false;', 'const bool use_restir = true;', 'const lowp int LIGHT_PATH_LENGTH = 1;',
  'const lowp int RESTIR_SAMPLES = 8;', 'const lowp int RENDER_MODE = 1;',
];
// index.js:54-85 default scene (Cornell box), textarea grammar
const CORNELL_LINES = [
  'MAT_CORNELL_WHITE, PLANE,  vec3( 0.0, 1.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_WHITE, PLANE,  vec3( 0.0,-1.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_WHITE, PLANE,  vec3( 0.0, 0.0, 1.0), vec4(2.5, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_RED,   PLANE,  vec3( 1.0, 0.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_GREEN, PLANE,  vec3(-1.0, 0.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)',
  'MAT_LIGHT_4,       SPHERE, vec3( 0.0, 1.4,-1.2), vec4(0.3, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_WHITE, BOX,    vec3( 0.5,-1.0,-1.8), vec4(1.0, 0.0, 0.0, 0.0)',
  'MAT_CORNELL_WHITE, BOX,    vec3(-0.45,-1.15,-1.3), vec4(0.7, 0.0, 0.0, 0.0)',
];

class GlslViewport {
  constructor(canvas, opts) {
    opts = opts || {};
    this.canvas = canvas || {};
    this.canvas.width = opts.width || 600;
    this.canvas.height = opts.height || 600;
    this.tile_rendering = opts.tile_rendering || false;
    this.device = opts.device || 0;
    this.defines = ['//#define USE_CUBEMAP', '#define USE_PROCEDURAL_SKY', '#define USE_BIASED_SAMPLING',
      '//#define USE_BIDIRECTIONAL', '//#define USE_RESTIR', '//#define USE_SPECTRAL', '//#define USE_VOLUMETRICS'];
    this.constants = STATIC_CONSTANTS.slice();
    this.animatedConstants = ANIMATED_CONSTANTS.slice();
    this.scene = sceneFromLines(CORNELL_LINES).scene;
    this.sdf_meshes = [];
    this.camera = {
      origin: new Vector3(0.0, 0.0, 2.8), lookat: new Vector3(0.0, 0.0, -1.0), fov: 50.0, aperture: 0.0,
      focalLength: 3.5,
    };
    this.passes = 0;
    this.max_passes = opts.max_passes || Infinity;
    this.paused = opts.paused || false;
    this.animatedScene = false;
    this.temporalFrames = 5;
    this.loadTime = Date.now();
    // tile rendering (index.js:97-103, 379): 32x32 viewports visited by updateTile()
    this.tile = [0, 0];
    this.tile_size = [32, 32];
    this.total_tiles = [Math.ceil(this.canvas.width / 32) - 1, Math.ceil(this.canvas.height / 32) - 1];
    this.viewport = this.tile_rendering ? [0, 0, 32, 32] : [0, 0, this.canvas.width, this.canvas.height];
    const backend = opts.backend || 'hip';
    if (backend === 'cpu') {
      const { CpuBackend } = require(path.join(__dirname, 'cpu_backend.js'));
      this._b = new CpuBackend(this.canvas.width, this.canvas.height);
    } else if (backend === 'hip') {
      this._b = new AddonBackend(this.canvas.width, this.canvas.height, this.device);
    } else {
      throw new Error("opts.backend must be 'hip' or 'cpu'");
    }
    this.backend = this._b.kind;
    // opts.executorCompat: ReSTIR reservoirs as the reference's GLES executor
    // stores them (rt0_set_executor_compat); default GLSL semantics
    if (opts.executorCompat) this._b.setExecutorCompat(true);
    // opts.textureFilter: 1 the executor's fixed-point filter (the HIP
    // backend's default), 0 exact fp32 bilinear (rt0_set_texture_filter)
    if (opts.textureFilter !== undefined) {
      if (!this._b.setTextureFilter) throw new Error('opts.textureFilter: not supported by the ' + this.backend + ' backend');
      this._b.setTextureFilter(opts.textureFilter);
    }
    this._compiled = null;
    this.images = {};
    // index.js:256-296: the RGBA noise image (u_rnd_tex) and opts.textures[0..3]
    // (u_tex0..3), each loaded like loadTexture does (REPEAT, LINEAR).  Paths or
    // {width, height, data} objects; the reference's asset paths are relative
    // to its page, so the caller names them (opts.rndTexture for the noise).
    if (opts.rndTexture) this.loadTexture({ name: 'rnd_tex' }, opts.rndTexture);
    (opts.textures || []).forEach((t, i) => this.loadTexture({ name: 'tex' + i }, t));
    // index.js:298-331: opts.cubemap = six faces (left, bottom, back, right,
    // top, front = -X -Y -Z +X +Y +Z), paths or {width, height, data} (RGB or RGBA)
    if (opts.cubemap) this.loadCubemap(opts.cubemap);
  }

  loadCubemap(faces) {
    if (!faces) {
      this._b.setCubemap(0, null);
      return;
    }
    const rgb = faces.map((f) => {
      const img = typeof f === 'string' ? readImage(f) : f;
      const n = img.width * img.height;
      if (img.data.length === n * 3) return { img, data: img.data };
      const d = new Uint8Array(n * 3);
      for (let k = 0; k < n; k++) {
        d[3 * k] = img.data[4 * k]; d[3 * k + 1] = img.data[4 * k + 1]; d[3 * k + 2] = img.data[4 * k + 2];
      }
      return { img, data: d };
    });
    const size = rgb[0].img.width;
    if (rgb.length !== 6 || rgb.some((f) => f.img.width !== size || f.img.height !== size))
      throw new Error('cubemap: six square faces of one size expected');
    this._b.setCubemap(size, rgb.map((f) => f.data));
    rgb.forEach((f, i) => { this.images['cubemap_img' + i] = f.img; });
  }

  // index.js:699-728 (assets only: the framebuffer textures live in librt0)
  loadTexture(opts, img) {
    const name = (opts && opts.name) || 'tex0';
    const unit = name === 'rnd_tex' ? 4 : Number(name.replace('tex', ''));
    if (!(unit >= 0 && unit <= 4)) throw new Error('unknown texture unit ' + name);
    if (typeof img === 'string') img = readImage(img);
    if (img === null) {
      this._b.setTexture(unit, 0, 0, null);
      return;
    }
    this._b.setTexture(unit, img.width, img.height, img.data);
    this.images[name === 'rnd_tex' ? 'rnd_img' : 'img' + unit] = img;
  }

  // index.js:384-440 (uniform upload); here also the "recompile" of scene/flags
  updateFrontTarget() {
    const key = JSON.stringify([this.defines, this.constants, this.scene, this.sdf_meshes]);
    if (key !== this._compiled) {
      this._b.setConfig(this.defines, this.constants);
      this._b.setScene(this.scene, this.sdf_meshes);
      this._compiled = key;
    }
    const c = this.camera;
    this._b.setCamera([c.origin.x, c.origin.y, c.origin.z], [c.lookat.x, c.lookat.y, c.lookat.z],
      [c.fov, c.aperture, c.focalLength]);
  }

  // index.js:986-1105: one pass, u_frame = ++passes (n > 1 batches passes).
  // Animated mode (index.js:990-1005): the pass counter cycles
  // (passes > 2*temporalFrames -> temporalFrames) and the accumulator is the
  // RENDER_MODE 1 running average over u_temporalFrames.
  render(n, timeMs) {
    n = n || 1;
    this.updateFrontTarget();
    const t = timeMs === undefined ? Date.now() - this.loadTime : timeMs;
    const vp = this.tile_rendering ? this.viewport : [0, 0, this.canvas.width, this.canvas.height];
    this._b.setViewport(vp[0], vp[1], vp[2], vp[3]);
    if (!this.animatedScene) {
      this._b.render(this.passes + 1, n, t);
      this.passes += n;
      return;
    }
    this._b.setTemporalFrames(this.temporalFrames);
    for (let k = 0; k < n; k++) {
      if (this.passes > this.temporalFrames * 2) this.passes = this.temporalFrames;
      this._b.render(++this.passes, 1, t);
    }
  }

  // index.js:822-880
  clear() { this._b.clear(); }

  // index.js:471-493
  resize(v) {
    const size = { 0: 256, 1: 512, 2: 1024, 3: 2048, 4: 4096, 5: 8192 }[v] || v;
    this.canvas.width = this.canvas.height = size;
    this._b.resize(size, size);
    this.passes = 0;
    this.total_tiles = [Math.ceil(size / this.tile_size[0]) - 1, Math.ceil(size / this.tile_size[1]) - 1];
  }

  // index.js:761-792: the next 32x32 viewport (row-major, bottom-up); passes
  // restart at 0 and the viewer pauses after the last tile.  As in the
  // reference, the edge tile's extent goes through tileMax, which IS
  // tile_size, so it persists for the tiles that follow.
  updateTile() {
    const tileMax = this.tile_size;
    this.passes = 0;
    if (this.tile[0] < this.total_tiles[0]) {
      this.tile[0]++;
      if (this.tile[0] === this.total_tiles[0] - 1)
        tileMax[0] = Math.abs(this.canvas.width - this.total_tiles[0] * this.tile_size[0]);
    } else {
      this.tile[0] = 0;
      if (this.tile[1] < this.total_tiles[1]) {
        this.tile[1]++;
        if (this.tile[1] === this.total_tiles[1] - 1)
          tileMax[1] = Math.abs(this.canvas.height - this.total_tiles[1] * this.tile_size[1]);
      } else {
        this.paused = true;
        this.tile[1] = 0;
      }
    }
    this.viewport = [this.tile[0] * this.tile_size[0], this.tile[1] * this.tile_size[1], tileMax[0], tileMax[1]];
  }

  // index.js:911-927: force USE_RESTIR, use_restir and sample_lights on (next render())
  toggleReSTIR() {
    this.defines[4] = '#define USE_RESTIR';
    this.constants[9] = 'const bool use_restir = true;';
    this.constants[7] = 'const bool sample_lights = true;';
  }

  // index.js:930-938 (the reference reports ReSTIR as active exactly in animated mode)
  getReSTIRDebugInfo() {
    return { isReSTIREnabled: this.animatedScene, temporalFrames: this.temporalFrames, passes: this.passes,
      animatedMode: this.animatedScene, debugViewActive: false };
  }

  // index.js:940-983
  setAnimatedMode(isAnimated) {
    this.animatedScene = !!isAnimated;
    this.constants = isAnimated ? this.animatedConstants.slice() : STATIC_CONSTANTS.slice();
    this.defines[4] = isAnimated ? '#define USE_RESTIR' : '//#define USE_RESTIR';
    this.clear();
  }

  accumulator() { return this._b.readAccum(); }

  // display pass (tonemapper.glsl:28-33) with u_cont = 1/passes, 1 when animated (index.js:1080-1090)
  image() { return this._b.tonemap(this.animatedScene ? 1.0 : 1.0 / Math.max(1, this.passes)); }

  lastKernelMs() { return this._b.lastKernelMs(); }
  // rt0_set_wavefront: 0 off, 1 SDF scenes (the default), 2 also ReSTIR scenes with models
  setWavefront(mode) { this._b.setWavefront(mode); }
  // which kernels the last render ran: 'pass', 'deferred', 'wavefront' ('cpu' on the CPU backend)
  renderPath() { return this._b.lastRenderPath(); }
}

module.exports = { GlslViewport, Vector3, sceneFromLines, sdfStatement, STATIC_CONSTANTS, ANIMATED_CONSTANTS,
  CORNELL_LINES, get addon() { return addonModule(); } };
