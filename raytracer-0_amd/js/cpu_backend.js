'use strict';
/*
 * cpu_backend.js -- GlslViewport's CPU backend (opts.backend = 'cpu'): the JS
 * integrator of rt0_cpu.js behind the same calls the N-API backend makes into
 * librt0 (glsl_viewport.js AddonBackend), so the reference's page sequence --
 * new GlslViewport, updateFrontTarget, render() per frame (index.html:
 * 1218-1242 -> index.js:986-1105) -- renders on the host cores.  This is
 * BASELINE configs[0], "JS CPU integrator path (no GPU)".
 *
 * The state arrives as the reference keeps it: `defines` and `constants` as
 * GLSL lines (tools.js:45-46 splices them at #constants), `scene` as the GLSL
 * text sceneFromLines builds (index.html:610-676) and `sdf_meshes` as the
 * #sdf_meshes statements (index.html:702-717); they are parsed back into the
 * integrator's config here.  Passes accumulate as the shader's
 * `prev + sample` chain (raytracer.glsl:2168) in fp32, rows bottom-up like the
 * GL framebuffer, ReSTIR configs run index.js's swap chain (795-820).
 * Asset textures, the cubemap, animated mode and the executor-compat switch
 * belong to the HIP backend: asking for them here throws.
 */
const { CpuRenderer } = require('./rt0_cpu.js');

const f = Math.fround;
const SDF_PRIMS = ['sdBox', 'udRoundBox', 'sdSphere', 'sdTriPrism', 'sdCone', 'MengerSponge', 'Mandelbulb'];

// '#define USE_X' lines on, '//#define USE_X' off (tools.js:45)
function parseDefines(lines) {
  const on = {};
  for (const s of lines) {
    const m = /^\s*(\/\/)?\s*#define\s+(\w+)/.exec(s);
    if (m) on[m[2]] = !m[1];
  }
  return on;
}

// 'const lowp int MAX_BOUNCES = 12;' -> {MAX_BOUNCES: 12}
function parseConstants(lines) {
  const c = {};
  for (const s of lines) {
    const m = /const\s+(?:(?:lowp|mediump|highp)\s+)?(int|float|bool)\s+(\w+)\s*=\s*([^;]+);/.exec(s);
    if (!m) throw new Error('cannot parse constant: ' + s);
    const v = m[3].trim();
    c[m[2]] = m[1] === 'bool' ? v === 'true' : Number(v);
  }
  return c;
}

// the Mesh(...) entries of the #scene text -> textarea lines "MAT, TYPE, vec3(..), vec4(..)"
function sceneLines(text) {
  const lines = [];
  let i = 0;
  for (;;) {
    i = text.indexOf('Mesh(', i);
    if (i < 0) break;
    let depth = 0, j = i + 4;
    for (; j < text.length; j++) {
      if (text[j] === '(') depth++;
      else if (text[j] === ')' && --depth === 0) break;
    }
    lines.push(text.slice(i + 5, j).trim());
    i = j;
  }
  return lines;
}

// #sdf_meshes statements -> the primitive kind of each SDF entry
function sdfKinds(statements) {
  const kinds = [];
  for (const s of statements) {
    const m = /sdf_meshes\[(\d+)\]\s*=\s*vec2\(\s*(\w+)\s*\(/.exec(s);
    if (!m) throw new Error('cannot parse #sdf_meshes statement: ' + s);
    const k = SDF_PRIMS.indexOf(m[2]);
    if (k < 0) throw new Error('unknown SDF primitive ' + m[2]);
    kinds[Number(m[1])] = k;
  }
  return kinds;
}

class CpuBackend {
  constructor(width, height) {
    this.kind = 'cpu';
    this.resize(width, height);
    this.defines = {};
    this.constants = {};
    this.lines = [];
    this.kinds = [];
    this.camera = { origin: [0, 0, 2.8], lookat: [0, 0, -1], fov: 50, aperture: 0, focalLength: 3.5 };
    this.vp = [0, 0, 0, 0];
    this._r = null;
    this._ms = 0;
  }

  resize(w, h) {
    this.w = w;
    this.h = h;
    this.accum = new Float32Array(w * h * 4);
    this.planes = Array.from({ length: 8 }, () => new Float32Array(w * h * 4));
    this._r = null;
  }

  clear() {
    this.accum.fill(0);
    this.planes.forEach((p) => p.fill(0));
  }

  setConfig(defines, constants) {
    this.defines = parseDefines(defines);
    this.constants = parseConstants(constants);
    this._r = null;
  }

  setScene(scene, sdf) {
    this.lines = sceneLines(scene);
    this.kinds = sdfKinds(sdf || []);
    this._r = null;
  }

  setCamera(pos, look, params) {
    this.camera = { origin: pos.slice(), lookat: look.slice(), fov: params[0], aperture: params[1],
      focalLength: params[2] };
    this._r = null;
  }

  setViewport(x, y, w, h) { this.vp = [x, y, w, h]; }

  setTemporalFrames() {}

  setTexture(unit, w, h, data) {
    if (data) throw new Error('asset textures are outside the JS CPU integrator (use the HIP backend)');
  }

  setCubemap(size, faces) {
    if (faces) throw new Error('the cubemap is outside the JS CPU integrator (use the HIP backend)');
  }

  setExecutorCompat(on) {
    if (on) throw new Error('executor compatibility is outside the JS CPU integrator (GLSL semantics only)');
  }

  renderer() {
    if (!this._r) {
      const cfg = { defines: this.defines, constants: this.constants, scene_lines: this.lines, sdf_kinds: this.kinds,
        camera: this.camera };
      this._r = new CpuRenderer(cfg, null, null, this.w, this.h);
    }
    return this._r;
  }

  // n passes u_frame = first .. first + n - 1 over the viewport rectangle
  render(first, n) {
    const t0 = process.hrtime.bigint();
    const r = this.renderer();
    let [x0, y0, vw, vh] = this.vp;
    if (!(vw > 0 && vh > 0)) [x0, y0, vw, vh] = [0, 0, this.w, this.h];
    const x1 = Math.min(this.w, x0 + vw), y1 = Math.min(this.h, y0 + vh);
    x0 = Math.max(0, x0);
    y0 = Math.max(0, y0);
    const A = this.accum;
    if (r.restirDef) {
      // one pass at a time: this pass reads the reservoirs the previous ones wrote
      const sample = new Float32Array(this.w * this.h * 4);
      for (let k = 0; k < n; k++) {
        const P = this.planes;  // [out main, out aux, back, back aux, hist1, hist1 aux, hist2, hist2 aux]
        r.tex = [P[2], P[3], P[4], P[5], P[6], P[7]];
        r.x0 = x0;
        r.x1 = x1;
        r.renderPass(first + k, y0, y1, sample, P[0], P[1]);
        for (let y = y0; y < y1; y++)
          for (let x = x0; x < x1; x++) {
            const p = (y * this.w + x) * 4;
            A[p] = f(A[p] + sample[p]);
            A[p + 1] = f(A[p + 1] + sample[p + 1]);
            A[p + 2] = f(A[p + 2] + sample[p + 2]);
          }
        // swapReSTIRBuffers (index.js:795-820): outputs become the newest history
        this.planes = [P[6], P[7], P[0], P[1], P[2], P[3], P[4], P[5]];
      }
    } else {
      for (let y = y0; y < y1; y++)
        for (let x = x0; x < x1; x++) {
          const p = (y * this.w + x) * 4;
          for (let k = 0; k < n; k++) {
            const s = r.sample(x, y, first + k);
            A[p] = f(A[p] + s.x);
            A[p + 1] = f(A[p + 1] + s.y);
            A[p + 2] = f(A[p + 2] + s.z);
          }
        }
    }
    this._ms = Number(process.hrtime.bigint() - t0) / 1e6;
  }

  readAccum() { return new Float32Array(this.accum); }

  // tonemapper.glsl:28-33: pow(acc * u_cont, 1/2.2) to an RGBA8 canvas, rows bottom-up
  tonemap(cont) {
    const out = new Uint8Array(this.w * this.h * 4);
    for (let i = 0; i < this.w * this.h; i++) {
      for (let c = 0; c < 3; c++) {
        const v = Math.min(Math.max(Math.pow(Math.max(this.accum[4 * i + c] * cont, 0), 1 / 2.2), 0), 1);
        out[4 * i + c] = Math.floor(v * 255 + 0.5);
      }
      out[4 * i + 3] = 255;
    }
    return out;
  }

  lastKernelMs() { return this._ms; }

  setWavefront() {}  // (a HIP-backend scheduling choice: the JS integrator has one path)

  lastRenderPath() { return 'cpu'; }
}

module.exports = { CpuBackend, parseDefines, parseConstants, sceneLines, sdfKinds };
