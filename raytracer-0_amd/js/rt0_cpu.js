'use strict';
// rt0_cpu.js -- the raytracer-0 integrator in JavaScript for the CPU: the
// product's CPU backend of GlslViewport (glsl_viewport.js, opts.backend =
// 'cpu'; BASELINE configs[0], "JS CPU integrator path (no GPU)") and the
// integrator bench.py times as `cpu_baseline` (SURVEY 8d).  It is chosen
// explicitly, never as a silent fallback: without a HIP device the GPU
// backend throws.  Checked against the reference's golden fixtures and the C
// restatement (oracle/rt0_oracle.c, the checker) by tests/test_cpu_js.py; it
// imports nothing from oracle/.
//
// It follows shaders/pathtracing/raytracer.glsl (line numbers cited per
// function) in fp32: every operation is rounded with Math.fround, and the RNG
// reproduces the reference executor's uint->float conversion, so frame k of a
// pixel draws the same random numbers as the reference.  Scope: planes,
// spheres, boxes, SDFs (every #sdf_meshes kind, sphere-traced with
// calcNormal), every untextured material, sky, plain NEE, MIS, SDF lights,
// homogeneous volumetrics (free-flight sampling, in-scatter NEE, HG phase, fog
// transmittance), ReSTIR in RENDER_MODE 0 (sampleLightsReSTIR with its
// candidates, two-level temporal history, spatial taps, finalize, MRT packing:
// renderPass() takes the six reservoir input planes and writes the two MRTs,
// the caller runs index.js's swap chain), spectral rendering (the hero
// wavelength, Cauchy IOR of the MAT_SPECTRAL_* materials and the CIE fit,
// 322-359, 1819-1824, 2153-2155) and TRIANGLE models (setTriangles: the
// commented-out Moller-Trumbore iTriangle of 864-892 over every triangle, as
// the C restatement runs it -- the reference has no triangle path at all),
// under GLSL semantics.  Animated-mode, cubemap and texture configs are
// rejected ("outside the JS CPU integrator"; the HIP backend renders them).
const f = Math.fround;

// ------------------------------------------------------------------ RNG
const _fb = new Float32Array(1);
const _ub = new Uint32Array(_fb.buffer);
const TWO_M32 = f(1.0 / 4294967296.0);
function u2f(m) {  // SwiftShader: double rounding above 2^31
  return m < 0x80000000 ? f(m) : f(f(m - 0x80000000) + 2147483648.0);
}
// raytracer.glsl:302-306
function hash(seed) {
  _fb[0] = seed;
  let n = (Math.imul(_ub[0], 747796405) + 2891336453) >>> 0;
  n = Math.imul(((n >>> ((n >>> 28) + 4)) ^ n) >>> 0, 277803737) >>> 0;
  return f(u2f(((n >>> 22) ^ n) >>> 0) * TWO_M32);
}
const K1031 = f(0.1031), K1030 = f(0.1030), K1919 = f(19.19);
function fract(x) { return f(x - Math.floor(x)); }
// raytracer.glsl:308-312 (returns [x, y])
function hash2(sx, sy) {
  let x = fract(f(sx * K1031)), y = fract(f(sy * K1030));
  const d = f(f(x * f(y + K1919)) + f(y * f(x + K1919)));
  x = f(x + d);
  y = f(y + d);
  return [fract(f(f(x + y) * x)), fract(f(f(x + y) * y))];
}

// ----------------------------------------------------------------- math
function V(x, y, z) { return { x, y, z }; }
function add(a, b) { return V(f(a.x + b.x), f(a.y + b.y), f(a.z + b.z)); }
function sub(a, b) { return V(f(a.x - b.x), f(a.y - b.y), f(a.z - b.z)); }
function mul(a, b) { return V(f(a.x * b.x), f(a.y * b.y), f(a.z * b.z)); }
function muls(a, s) { return V(f(a.x * s), f(a.y * s), f(a.z * s)); }
function dot(a, b) { return f(f(f(a.x * b.x) + f(a.y * b.y)) + f(a.z * b.z)); }
function isqrt(x) { return f(1.0 / f(Math.sqrt(x))); }
function normalize(a) { return muls(a, isqrt(dot(a, a))); }
function length(a) { return f(Math.sqrt(dot(a, a))); }
function gmax(a, b) { return a > b ? a : b; }
function gmin(a, b) { return a < b ? a : b; }
function clamp(x, lo, hi) { return gmin(gmax(x, lo), hi); }
function sgn(x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }
function step(e, x) { return x < e ? 0 : 1; }
function mixf(x, y, a) { return f(f(a * f(y - x)) + x); }
function vmaxs(a, s) { return V(gmax(a.x, s), gmax(a.y, s), gmax(a.z, s)); }
function vmaxc(a) { return gmax(a.x, gmax(a.y, a.z)); }
function vabs(a) { return V(Math.abs(a.x), Math.abs(a.y), Math.abs(a.z)); }
function cross(a, b) {
  return V(f(f(a.y * b.z) - f(a.z * b.y)), f(f(a.z * b.x) - f(a.x * b.z)), f(f(a.x * b.y) - f(a.y * b.x)));
}
function reflect(i, n) { return sub(i, muls(n, f(2 * dot(n, i)))); }
function refract(i, n, eta) {
  const d = dot(n, i);
  const k = f(1 - f(f(eta * eta) * f(1 - f(d * d))));
  if (k < 0) return V(0, 0, 0);
  return sub(muls(i, eta), muls(n, f(f(eta * d) + f(Math.sqrt(k)))));
}
function gpow(x, y) { return f(Math.pow(Math.abs(x), y)); }
const fsin = (x) => f(Math.sin(x)), fcos = (x) => f(Math.cos(x));

const EPS = f(0.001), INF_T = f(1e4), TWO_PI = f(6.28318531), ONE_OVER_PI = f(0.31830989), FOUR_PI = f(12.5663706);
const RAD = f(0.01745329);

const PI_F = f(3.14159265), VOL_SIGMA_T = f(0.15), VOL_SIGMA_S = f(0.13), VOL_G = f(0.5);

// ------------------------------------------------ SDF primitives (496-576, 642-698)
function sdBox(p, b) {
  const d = sub(vabs(p), b);
  return f(length(V(gmax(d.x, 0), gmax(d.y, 0), gmax(d.z, 0))) + gmin(gmax(d.x, gmax(d.y, d.z)), 0));
}
function sdCone(p, c) {
  const qx = f(Math.sqrt(f(f(p.x * p.x) + f(p.z * p.z)))), qy = p.y;
  const d1 = f(-qy - c.z), d2 = gmax(f(f(qx * c.x) + f(qy * c.y)), qy);
  const a = gmax(d1, 0), b = gmax(d2, 0);
  return f(f(Math.sqrt(f(f(a * a) + f(b * b)))) + gmin(gmax(d1, d2), 0));
}
function gmod(x, y) { return f(x - f(y * Math.floor(f(x / y)))); }
function menger(p, scale) {
  let d = sdBox(p, scale), s = 1;
  for (let m = 0; m < 4; m++) {
    const ps = muls(p, s);
    const a = V(f(gmod(ps.x, 2) - 1), f(gmod(ps.y, 2) - 1), f(gmod(ps.z, 2) - 1));
    s = f(s * 3);
    const r = V(Math.abs(f(1 - f(3 * Math.abs(a.x)))), Math.abs(f(1 - f(3 * Math.abs(a.y)))), Math.abs(f(1 - f(3 * Math.abs(a.z)))));
    const da = gmax(r.x, r.y), db = gmax(r.y, r.z), dc = gmax(r.z, r.x);
    d = gmax(f(f(gmin(da, gmin(db, dc)) - 1) / s), d);
  }
  return d;
}
function mul5(a, b, c, d, e) { return f(f(f(f(a * b) * c) * d) * e); }
function mandelbulb(p) {
  let w = p, m = dot(w, w), dz = 1;
  for (let i = 0; i < 3; i++) {
    const m2 = f(m * m), m4 = f(m2 * m2);
    dz = f(f(f(8 * f(Math.sqrt(f(f(m4 * m2) * m)))) * dz) + 1);
    const x = w.x, x2 = f(x * x), x4 = f(x2 * x2);
    const y = w.y, y2 = f(y * y), y4 = f(y2 * y2);
    const z = w.z, z2 = f(z * z), z4 = f(z2 * z2);
    const k3 = f(x2 + z2);
    const k2 = isqrt(f(f(f(mul5(k3, k3, k3, k3, k3) * k3) * k3)));
    const k1 = f(f(f(f(f(x4 + y4) + z4) - f(f(6 * y2) * z2)) - f(f(6 * x2) * y2)) + f(f(2 * z2) * x2));
    const k4 = f(f(x2 - y2) + z2);
    const pxz = f(f(x4 - f(f(6 * x2) * z2)) + z4);
    const wx = f(p.x + f(f(f(f(mul5(64, x, y, z, f(x2 - z2)) * k4) * pxz) * k1) * k2));
    const wy = f(f(p.y + mul5(-16, y2, k3, k4, k4)) + f(k1 * k1));
    const poly = f(f(f(f(f(x4 * x4) - f(f(f(28 * x4) * x2) * z2)) + f(f(70 * x4) * z4)) - f(f(f(28 * x2) * z2) * z4)) + f(z4 * z4));
    const wz = f(p.z + f(f(f(f(f(f(-8 * y) * k4) * poly) * k1) * k2)));
    w = V(wx, wy, wz);
    m = dot(w, w);
    if (m > 4) break;
  }
  return f(f(f(f(0.25 * f(Math.log(m))) * f(Math.sqrt(m)))) / dz);
}
// randomSphereDirection (1143-1147), sampleHG (1157-1171)
function randomSphereDirection(seed) {
  const r = hash2(seed, seed), rx = f(r[0] * TWO_PI), ry = f(r[1] * TWO_PI);
  const sy = fsin(ry), cy = fcos(ry);
  return V(f(fsin(rx) * sy), f(fsin(rx) * cy), fcos(rx));
}
function sampleHG(w, seed) {
  const uv = hash2(seed, f(seed + f(1.789))), g = VOL_G;
  const sqr = f(f(1 - f(g * g)) / f(f(1 - g) + f(f(2 * g) * uv[0])));
  const cosT = f(f(f(1 + f(g * g)) - f(sqr * sqr)) / f(2 * g));
  const sinT = f(Math.sqrt(gmax(0, f(1 - f(cosT * cosT)))));
  const phi = f(TWO_PI * uv[1]);
  const [t, b] = CpuRenderer.binormals(w);
  return normalize(add(add(muls(t, f(fcos(phi) * sinT)), muls(b, f(fsin(phi) * sinT))), muls(w, cosT)));
}

// ------------------------------------------------------- scene grammar
const T_SPHERE = 0, T_PLANE = 1, T_BOX = 2, T_SDF = 3, T_TRIANGLE = 5;
const M_LIGHT = 0, M_DIR_LIGHT = 1, M_DIFF = 2, M_SPEC = 3, M_REFR_FRESNEL = 4, M_REFR_SCHLICK = 5, M_COAT = 6;
// Material table, raytracer.glsl:165-224 ([c, e, nt, type]; textured ones omitted)
const MATS = {
  MAT_REFR_CLEAR: [[1, 0.5, 0], [0, 0, 0], 1.53, M_REFR_FRESNEL],
  MAT_REFR_CLEAR_2: [[1, 1, 1], [0, 0, 0], 1.53, M_REFR_SCHLICK],
  MAT_REFR_SAPPHIRE: [[1, 1, 1], [0, 0, 0], 1.77, M_REFR_FRESNEL],
  MAT_REFR_WATER: [[0.25, 0.64, 0.88], [0, 0, 0], 1.33, M_REFR_FRESNEL],
  MAT_LIGHT_4: [[1, 1, 1], [4, 4, 4], 0, M_LIGHT],
  MAT_LIGHT_CANDLE_4: [[1.0, 0.57647058823, 0.16078431372], [4, 4, 4], 0, M_LIGHT],
  MAT_LIGHT_HALOGEN_4: [[1.0, 0.94509803921, 0.87843137254], [4, 4, 4], 0, M_LIGHT],
  MAT_LIGHT_DEMO: [[1, 1, 1], [10, 10, 10], 0, M_LIGHT],
  MAT_CLEAR_SKY: [[0.25098039215, 0.61176470588, 1.0], [1, 1, 1], 0, M_DIR_LIGHT],
  MAT_OVERCAST_SKY: [[0.78823529411, 0.8862745098, 1.0], [1, 1, 1], 0, M_DIR_LIGHT],
  MAT_DIRECT_SUNLIGHT: [[1, 1, 1], [1, 1, 1], 0, M_DIR_LIGHT],
  MAT_MIRROR: [[1, 1, 1], [0, 0, 0], 0, M_SPEC],
  MAT_BLACK: [[0, 0, 0], [0, 0, 0], 0, M_DIFF],
  MAT_WHITE: [[1, 1, 1], [0, 0, 0], 0, M_DIFF],
  MAT_RED: [[1, 0, 0], [0, 0, 0], 0, M_DIFF],
  MAT_GREEN: [[0, 1, 0], [0, 0, 0], 0, M_DIFF],
  MAT_BLUE: [[0, 0, 1], [0, 0, 0], 0, M_DIFF],
  MAT_CORNELL_WHITE: [[1, 1, 1], [0, 0, 0], 0, M_DIFF],
  MAT_CORNELL_RED: [[0.7, 0.12, 0.05], [0, 0, 0], 0, M_DIFF],
  MAT_CORNELL_GREEN: [[0.2, 0.4, 0.36], [0, 0, 0], 0, M_DIFF],
  MAT_YELLOW: [[1, 1, 0], [0, 0, 0], 0, M_DIFF],
  MAT_PURPLE: [[0.50196078431, 0, 0.50196078431], [0, 0, 0], 0, M_DIFF],
  MAT_COAT_NAVY: [[0, 0, 0.50196078431], [1, 1, 1], 1.4, M_COAT],
  MAT_COAT_PURPLE: [[0.50196078431, 0, 0.50196078431], [0, 0, 0], 1.4, M_COAT],
  MAT_COAT_WAX: [[0.9333, 0.6666, 0.6], [0.005, 0.005, 0.005], 1.4, M_COAT],
  // spectral materials: nt < 0 = Cauchy A (220-224), dispersive under USE_SPECTRAL
  MAT_SPECTRAL_FLINT: [[1, 1, 1], [0, 0, 0], -1.7167, M_REFR_FRESNEL],
  MAT_SPECTRAL_DIAMOND: [[1, 1, 1], [0, 0, 0], -2.3991, M_REFR_FRESNEL],
};
const TYPES = { SPHERE: T_SPHERE, PLANE: T_PLANE, BOX: T_BOX, SDF: T_SDF, TRIANGLE: T_TRIANGLE };

// spectral rendering: Cauchy IOR (357) and the CIE 1931 fit -> sRGB (324-353)
function spectralIOR(lambda, A) {
  const lu = f(lambda * f(0.001));
  return f(A + f(f(0.04) / f(lu * lu)));
}
const fexp = (x) => f(Math.exp(x));
function lobe(l, c, lo, hi) { const t = f(f(l - c) * (l < c ? lo : hi)); return fexp(f(f(-0.5 * t) * t)); }
function cmfX(l) {
  return f(f(f(f(0.362) * lobe(l, f(442.0), f(0.0624), f(0.0374))) + f(f(1.056) * lobe(l, f(599.8), f(0.0264), f(0.0323))))
    - f(f(0.065) * lobe(l, f(501.1), f(0.0490), f(0.0382))));
}
function cmfY(l) {
  return f(f(f(0.821) * lobe(l, f(568.8), f(0.0213), f(0.0247))) + f(f(0.286) * lobe(l, f(530.9), f(0.0613), f(0.0322))));
}
function cmfZ(l) {
  return f(f(f(1.217) * lobe(l, f(437.0), f(0.0845), f(0.0278))) + f(f(0.681) * lobe(l, f(459.0), f(0.0385), f(0.0725))));
}
function wavelengthToRGB(l) {
  const X = cmfX(l), Y = cmfY(l), Z = cmfZ(l);
  const r = f(f(f(f(3.2404542) * X) - f(f(1.5371385) * Y)) - f(f(0.4985314) * Z));
  const g = f(f(f(f(-0.9692660) * X) + f(f(1.8760108) * Y)) + f(f(0.0415560) * Z));
  const b = f(f(f(f(0.0556434) * X) - f(f(0.2040259) * Y)) + f(f(1.0572252) * Z));
  return V(f(gmax(0, r) / f(0.378)), f(gmax(0, g) / f(0.298)), f(gmax(0, b) / f(0.285)));
}

// parse "vecN(a, b, ...)" with GLSL scalar broadcast
function parseVec(s, n) {
  const m = /vec\d\s*\(([^)]*)\)/.exec(s);
  if (!m) throw new Error('bad vector: ' + s);
  const v = m[1].split(',').map((t) => f(parseFloat(t)));
  return { vals: Array.from({ length: n }, (_, i) => (v.length === 1 ? v[0] : v[i])), rest: s.slice(m.index + m[0].length) };
}

// Scene textarea grammar (index.html:624-653): "MAT, TYPE, vec3(pos), vec4(joker)"
function parseScene(lines) {
  const meshes = [], lights = [];
  lines.forEach((line, i) => {
    const parts = line.split(',');
    const mat = parts[0].trim(), type = parts[1].trim();
    if (!(mat in MATS)) throw new Error('unsupported material for the JS CPU integrator: ' + mat);
    if (!(type in TYPES)) throw new Error('unsupported mesh type for the JS CPU integrator: ' + type);
    if (mat.indexOf('MAT_LIGHT') >= 0) lights.push(i);
    const rest = parts.slice(2).join(',');
    const p = parseVec(rest, 3), j = parseVec(p.rest, 4);
    const d = MATS[mat];
    meshes.push({
      t: TYPES[type], pos: V(...p.vals), joker: j.vals,
      c: V(f(d[0][0]), f(d[0][1]), f(d[0][2])), e: V(f(d[1][0]), f(d[1][1]), f(d[1][2])), nt: f(d[2]), mt: d[3],
    });
  });
  if (lights.length === 0) lights.push(-1);
  // meshes[NUM_MESHES + i] addresses SDF i: the SDF lines follow the quadrics,
  // and the TRIANGLE entries (model instances) follow the SDFs
  const rank = (t) => (t === T_SDF ? 1 : t === T_TRIANGLE ? 2 : 0);
  for (let i = 1; i < meshes.length; i++)
    if (rank(meshes[i].t) < rank(meshes[i - 1].t)) throw new Error('SDF meshes must follow the quadrics, TRIANGLE entries the SDFs');
  const nMeshes = meshes.filter((m) => rank(m.t) === 0).length;
  const nSdf = meshes.filter((m) => m.t === T_SDF).length;
  return { meshes, lights, nMeshes, nSdf };
}

// ------------------------------------------------- ReSTIR (1264-1801)
function EMPTY_RES() { return { pos: V(0, 0, 0), col: V(0, 0, 0), ws: 0, M: 0, W: 0, age: 0, idx: -1 }; }
const POISSON = [[-0.4706, 0.4706], [0.8090, 0.2628], [-0.2628, -0.8090], [0.6882, -0.5000],
  [-0.9511, -0.1625], [0.1625, 0.9511], [0.5000, -0.6882], [-0.6882, 0.5000]].map((p) => [f(p[0]), f(p[1])]);
const LUM = V(f(0.2126), f(0.7152), f(0.0722));
const finite = (x) => Number.isFinite(x);
// updateReservoir, 1305-1326
function updateReservoir(r, pos, col, idx, weight, rnd) {
  if (weight <= 0) return;
  r.ws = f(r.ws + weight);
  r.M = f(r.M + 1);
  if (r.M > 60) { r.ws = f(r.ws * f(0.95)); r.M = f(r.M * f(0.95)); }
  if (r.ws > 0) {
    const p = f(weight / r.ws);
    if (rnd < p) { r.pos = pos; r.col = col; r.idx = idx; }
  }
}
// evaluateTargetFunction, 1361-1387
function targetFn(lp, lc, hp, hn, m) {
  const lv = sub(lp, hp), distSq = dot(lv, lv);
  if (distSq < f(EPS * EPS)) return 0;
  const ld = normalize(lv), ct = gmax(0, dot(hn, ld));
  if (ct <= 0) return 0;
  const llum = dot(lc, LUM);
  if (llum <= 0) return 0;
  const slum = dot(m.c, LUM);
  const nnt = f(f(m.nt - 1) / f(m.nt + 1)), R0 = f(nnt * nnt);
  const isRefr = (m.mt === M_REFR_FRESNEL || m.mt === M_REFR_SCHLICK) ? 1 : 0, isCoat = m.mt === M_COAT ? 1 : 0;
  const base = mixf(slum, R0, isRefr);
  const bw = f(mixf(base, f(f(1 - R0) * slum), isCoat) * ONE_OVER_PI);
  return f(f(f(llum * bw) * ct) / gmax(distSq, f(1e-4)));
}

// ---------------------------------------------------------- renderer
class CpuRenderer {
  // cfg: a tests/golden/configs.json entry; cornell: cfgs.cornell_lines; camera default
  constructor(cfg, cornellLines, defaultCamera, width, height) {
    const defs = Object.assign({ USE_PROCEDURAL_SKY: true, USE_BIASED_SAMPLING: true }, cfg.defines || {});
    if (defs.USE_CUBEMAP) throw new Error('USE_CUBEMAP is outside the JS CPU integrator');
    this.spectral = !!defs.USE_SPECTRAL;
    this.hero = f(550);
    const c = Object.assign({
      MAX_BOUNCES: 12, MAX_DIFF_BOUNCES: 4, MAX_SPEC_BOUNCES: 4, MAX_TRANS_BOUNCES: 12, MAX_SCATTERING_EVENTS: 12,
      sample_lights: true, use_mis: false, use_restir: false, MARCHING_STEPS: 128, FUDGE_FACTOR: 0.9,
      RESTIR_SAMPLES: 16, RENDER_MODE: 0,
    }, cfg.constants || {});
    if (c.RENDER_MODE !== 0) throw new Error('RENDER_MODE 1 is outside the JS CPU integrator');
    this.restir = !!c.use_restir;
    this.restirDef = !!defs.USE_RESTIR;
    this.restirSamples = c.RESTIR_SAMPLES;
    this.tex = [null, null, null, null, null, null];  // reservoir inputs: back, back aux, hist1, hist1 aux, hist2, hist2 aux
    this.fr = EMPTY_RES();  // g_final_reservoir of the current fragment
    this.sky = !!defs.USE_PROCEDURAL_SKY;
    this.biased = !!defs.USE_BIASED_SAMPLING;
    this.maxB = c.MAX_BOUNCES; this.maxD = c.MAX_DIFF_BOUNCES; this.maxS = c.MAX_SPEC_BOUNCES;
    this.maxT = c.MAX_TRANS_BOUNCES; this.maxSc = c.MAX_SCATTERING_EVENTS;
    this.sampleLights = !!c.sample_lights; this.mis = !!c.use_mis;
    const sc = parseScene(cfg.scene_lines || cornellLines);
    this.meshes = sc.meshes; this.lights = sc.lights;
    this.nMeshes = sc.nMeshes; this.nSdf = sc.nSdf;
    this.nModels = sc.meshes.length - sc.nMeshes - sc.nSdf;
    this.nTris = 0;  // setTriangles
    this.sdfKinds = Array.from({ length: this.nSdf }, (_, i) => ((cfg.sdf_kinds || [])[i] || 0));
    this.vol = !!defs.USE_VOLUMETRICS;
    this.marchSteps = c.MARCHING_STEPS; this.fudge = f(c.FUDGE_FACTOR);
    this.w = width; this.h = height;
    const cam = cfg.camera || defaultCamera;
    this.camPos = V(f(cam.origin[0]), f(cam.origin[1]), f(cam.origin[2]));
    this.camLook = V(f(cam.lookat[0]), f(cam.lookat[1]), f(cam.lookat[2]));
    this.camParams = V(f(cam.fov), f(cam.aperture), f(cam.focalLength));
    this.nIsect = 0;
    this.nMap = 0;
  }

  // World-space triangles of the TRIANGLE entries: v9 = n x 9 floats (three
  // vertices), model = owner entry k | (back-face culling, opts[3]) << 30 --
  // the same soup the C restatement takes (or_set_triangles).
  setTriangles(v9, model) {
    const n = model.length;
    this.nTris = n;
    this.tri = new Float32Array(n * 13);  // v1, e0, e1, eps, cull
    this.triModel = Int32Array.from(model);
    for (let i = 0; i < n; i++) {
      const q = 9 * i, v1 = V(f(v9[q]), f(v9[q + 1]), f(v9[q + 2]));
      const e0 = sub(V(f(v9[q + 3]), f(v9[q + 4]), f(v9[q + 5])), v1), e1 = sub(V(f(v9[q + 6]), f(v9[q + 7]), f(v9[q + 8])), v1);
      const eps = f(f(EPS * f(Math.sqrt(dot(e0, e0)))) * f(Math.sqrt(dot(e1, e1))));
      this.tri.set([v1.x, v1.y, v1.z, e0.x, e0.y, e0.z, e1.x, e1.y, e1.z, eps, (model[i] >> 30) & 1], 13 * i);
    }
  }
  // iTriangle (864-892, Moller-Trumbore) with the restatement's size-relative
  // parallel-ray threshold (oracle/rt0_oracle.c iTriangle): t in (EPS, tmin) or -1
  triHit(i, o, d, tmin) {
    const T = this.tri, b = 13 * i;
    const e0x = T[b + 3], e0y = T[b + 4], e0z = T[b + 5], e1x = T[b + 6], e1y = T[b + 7], e1z = T[b + 8];
    const hx = f(f(d.y * e1z) - f(d.z * e1y)), hy = f(f(d.z * e1x) - f(d.x * e1z)), hz = f(f(d.x * e1y) - f(d.y * e1x));
    const a = f(f(f(e0x * hx) + f(e0y * hy)) + f(e0z * hz));
    const eps = T[b + 9];
    if (T[b + 10] ? a < eps : (a > -eps && a < eps)) return -1;
    const fa = f(1 / a);
    const sx = f(o.x - T[b]), sy = f(o.y - T[b + 1]), sz = f(o.z - T[b + 2]);
    const u = f(fa * f(f(f(sx * hx) + f(sy * hy)) + f(sz * hz)));
    if (u < 0 || u > 1) return -1;
    const qx = f(f(sy * e0z) - f(sz * e0y)), qy = f(f(sz * e0x) - f(sx * e0z)), qz = f(f(sx * e0y) - f(sy * e0x));
    const v = f(fa * f(f(f(d.x * qx) + f(d.y * qy)) + f(d.z * qz)));
    if (v < 0 || f(u + v) > 1) return -1;
    const t = f(fa * f(f(f(e1x * qx) + f(e1y * qy)) + f(e1z * qz)));
    return t > EPS && t < tmin ? t : -1;
  }

  // map(), raytracer.glsl:700-712 (+ the #sdf_meshes statements, index.html:702-717) -> [d, id]
  map(p) {
    this.nMap++;
    let rx = 0, ry = 0;
    for (let i = 0; i < this.nSdf; i++) {
      const m = this.meshes[this.nMeshes + i];
      const q = sub(p, m.pos), j = V(m.joker[0], m.joker[1], m.joker[2]);
      let d;
      switch (this.sdfKinds[i]) {
        case 0: d = sdBox(q, j); break;
        case 1: { const dd = sub(vabs(q), j); d = f(length(V(gmax(dd.x, 0), gmax(dd.y, 0), gmax(dd.z, 0))) - m.joker[3]); break; }
        case 2: d = f(length(q) - m.joker[0]); break;
        case 3: {
          const qa = vabs(q);
          d = gmax(f(qa.z - m.joker[1]), f(gmax(f(f(qa.x * f(0.866025)) + f(q.y * 0.5)), -q.y) - f(m.joker[0] * 0.5)));
          break;
        }
        case 4: d = sdCone(q, j); break;
        case 5: d = menger(q, j); break;
        default: d = mandelbulb(q); break;
      }
      if (i === 0) { rx = d; ry = 0; } else {
        const a = rx < d ? 1 : 0;
        rx = mixf(d, rx, a); ry = mixf(f(i), ry, a);
      }
    }
    return [rx, ry];
  }
  // 714-722
  calcNormal(p) {
    const E = EPS;
    const a = muls(V(1, -1, -1), this.map(add(p, V(E, -E, -E)))[0]);
    const b = muls(V(-1, -1, 1), this.map(add(p, V(-E, -E, E)))[0]);
    const c = muls(V(-1, 1, -1), this.map(add(p, V(-E, E, -E)))[0]);
    const d = muls(V(1, 1, 1), this.map(add(p, V(E, E, E)))[0]);
    return normalize(add(add(add(a, b), c), d));
  }

  // intersection(), raytracer.glsl:997-1082 -> {t, n, pos, index}
  intersect(o, d) {
    this.nIsect++;
    let tmin = INF_T, type = -1, index = 0, n = V(0, 0, 0);
    const ms = this.meshes;
    for (let i = 0; i < this.nMeshes; i++) {
      const m = ms[i];
      if (m.joker[0] === 0) continue;
      if (m.t === T_SPHERE) {  // 818-833
        const oc = sub(o, m.pos), b = dot(oc, d);
        const c = f(dot(oc, oc) - f(m.joker[0] * m.joker[0]));
        const disc = f(f(b * b) - c);
        if (disc < 0) continue;
        const sd = f(Math.sqrt(disc));
        let t = f(-b - sd);
        if (!(t > EPS && t < tmin)) { t = f(-b + sd); if (!(t > EPS && t < tmin)) continue; }
        tmin = t; type = T_SPHERE; index = i;
      } else if (m.t === T_PLANE) {  // 812-815
        const t = f(f(-m.joker[0] - dot(m.pos, o)) / dot(m.pos, d));
        if (t > EPS && t < tmin) { tmin = t; type = T_PLANE; index = i; }
      } else {  // iBox 836-859
        const mv = V(f(1 / d.x), f(1 / d.y), f(1 / d.z));
        const nv = mul(mv, sub(m.pos, o));
        const k = muls(muls(vabs(mv), m.joker[0]), 0.5);
        const t1 = sub(nv, k), t2 = add(nv, k);
        const tN = gmax(gmax(t1.x, t1.y), t1.z), tF = gmin(gmin(t2.x, t2.y), t2.z);
        if (tN > tF || tF < 0) continue;
        const t = tN > 0 ? tN : tF;
        if (t < EPS || t >= tmin) continue;
        const hp = sub(add(o, muls(d, t)), m.pos);
        const half = f(m.joker[0] * 0.5);
        const dd = sub(vabs(hp), V(half, half, half));
        const s = V(sgn(hp.x), sgn(hp.y), sgn(hp.z));
        const st = V(step(dd.y, dd.x) * step(dd.z, dd.x), step(dd.z, dd.y) * step(dd.x, dd.y),
          step(dd.x, dd.z) * step(dd.y, dd.z));
        n = normalize(mul(s, st));
        tmin = t; type = T_BOX; index = i;
      }
    }
    if (this.nModels > 0) {  // every triangle, lowest index wins ties (strict <)
      if (this.nTris === 0) throw new Error('TRIANGLE entries without setTriangles');
      let best = -1;
      for (let i = 0; i < this.nTris; i++) {
        const t = this.triHit(i, o, d, tmin);
        if (t >= 0) { tmin = t; best = i; }
      }
      if (best >= 0) {
        const T = this.tri, b = 13 * best;
        n = normalize(cross(V(T[b + 3], T[b + 4], T[b + 5]), V(T[b + 6], T[b + 7], T[b + 8])));
        index = this.nMeshes + this.nSdf + (this.triModel[best] & 0x3fffffff);
        type = T_TRIANGLE;
      }
    }
    if (this.nSdf > 0) {  // iSDF, 974-993
      let t = f(EPS * 4), res = [0, 0];
      for (let i = 0; i < this.marchSteps; i++) {
        res = this.map(add(o, muls(d, t)));
        const h = Math.abs(res[0]);
        if (h < EPS || t > tmin) break;
        t = f(t + f(h * this.fudge));
      }
      if (!(t > tmin)) {
        n = this.calcNormal(add(o, muls(d, t)));
        index = this.nMeshes + Math.trunc(res[1]);
        tmin = t; type = T_SDF;
      }
    }
    let pos = V(0, 0, 0);
    if (type >= 0) {
      pos = add(muls(d, tmin), o);
      if (type === T_SPHERE) n = normalize(sub(pos, ms[index].pos));
      else if (type === T_PLANE) n = normalize(ms[index].pos);
    }
    return { t: tmin, n, pos, index };
  }

  // 1092-1107
  static binormals(n) {
    const sig = n.z < 0 ? -1 : 1;
    if (Math.abs(n.z) > f(0.99999)) return [V(1, 0, 0), V(0, sig, 0)];
    const a = f(1 / f(sig - n.z)), b = f(f(n.x * n.y) * a);
    return [V(f(1 + f(f(f(sig * n.x) * n.x) * a)), f(sig * b), f(-sig * n.x)), V(b, f(sig + f(f(n.y * n.y) * a)), -n.y)];
  }
  static frameDir(w, u, v, rx, ry) {
    const om = f(Math.sqrt(f(1 - f(ry * ry))));
    return normalize(add(add(muls(u, f(fcos(rx) * om)), muls(v, f(fsin(rx) * om))), muls(w, ry)));
  }
  // getSampleBiased (1109-1120) / getConeSample (1122-1133)
  static coneSample(w, extent, seed) {
    const [u, v] = CpuRenderer.binormals(w);
    const r = hash2(seed, seed);
    return CpuRenderer.frameDir(w, u, v, f(r[0] * TWO_PI), f(1 - f(r[1] * extent)));
  }
  randomDirection(n, seed) {
    if (!this.biased) return CpuRenderer.coneSample(n, 1, seed);
    const [u, v] = CpuRenderer.binormals(n);
    const r = hash2(seed, seed);
    return CpuRenderer.frameDir(n, u, v, f(r[0] * TWO_PI), gpow(r[1], f(1 / 2)));
  }

  // calcDirectLighting, 1174-1230
  directLight(li, x, nl, seed) {
    const L = this.meshes[li];
    if (L.mt === M_LIGHT) {
      if (L.t === T_SDF) {  // 1205-1216
        const ld = add(L.pos, mul(randomSphereDirection(f(seed + f(78.2358))), V(L.joker[0], L.joker[1], L.joker[2])));
        const sr = normalize(sub(ld, x));
        const hit = this.intersect(add(x, muls(nl, EPS)), sr);
        const mh = this.meshes[hit.index];
        if (mh.mt !== M_LIGHT) return V(0, 0, 0);
        return muls(mul(vmaxs(mh.c, f(0.001)), mh.e), gmax(f(0.001), dot(sr, nl)));
      }
      if (L.t !== T_SPHERE) return V(0, 0, 0);
      const sw = sub(L.pos, x);
      const r2 = f(L.joker[0] * L.joker[0]), d2 = dot(sw, sw);
      const cosA = f(Math.sqrt(f(1 - clamp(f(r2 / d2), 0, 1))));
      const sr = CpuRenderer.coneSample(normalize(sw), f(1 - cosA), f(seed + f(23.1656)));
      const hit = this.intersect(add(x, muls(nl, EPS)), sr);
      const mh = this.meshes[hit.index];
      if (mh.mt !== M_LIGHT) return V(0, 0, 0);
      const weight = f(2 * f(1 - cosA));
      const fog = this.vol ? f(Math.exp(f(-VOL_SIGMA_T * hit.t))) : 1;
      return muls(muls(muls(mul(vmaxs(mh.c, f(0.001)), mh.e), weight), gmax(f(0.001), dot(sr, nl))), fog);
    }
    if (L.mt === M_DIR_LIGHT) {
      const hit = this.intersect(add(x, muls(nl, EPS)), L.pos);
      if (hit.t === INF_T) return muls(mul(L.c, L.e), gmax(f(0.001), dot(L.pos, nl)));
    }
    return V(0, 0, 0);
  }
  // 1233-1262
  static power(f1, g1) {
    const denom = f(f(f1 * f1) + f(g1 * g1));
    const r = f(f(f1 * f1) / denom);
    return r > 0 ? r : 0;  // max(0, 0/0) -> 0 (IEEE maxNum; DESIGN.md deviation)
  }
  static cosPdf(wi, n) { return f(gmax(0, dot(wi, n)) * ONE_OVER_PI); }
  static lightPdf(L, x) {
    if (L.mt !== M_LIGHT) return 0;
    if (L.t === T_SPHERE) {
      const d = sub(L.pos, x);
      const d2 = dot(d, d), r2 = f(L.joker[0] * L.joker[0]);
      if (d2 <= r2) return 0;
      const ctm = f(Math.sqrt(gmax(0, f(1 - f(r2 / d2)))));
      const denom = f(1 - ctm);
      if (denom < f(1e-6)) return 0;
      return f(1 / f(TWO_PI * denom));
    }
    return f(1 / FOUR_PI);
  }

  // isValidReservoir, 1389-1416
  validRes(r) {
    if (!finite(r.M) || !finite(r.ws) || !finite(r.W) || !finite(r.age)) return false;
    if (r.M <= 0 || r.M > 200) return false;
    if (r.ws <= 0 || r.ws > 1000) return false;
    if (r.W < 0 || r.W > 20) return false;
    if (r.age < 0 || r.age > 35) return false;
    const lc = dot(r.col, r.col);
    if (lc < f(0.000001) || lc > 10000) return false;
    if (r.idx >= this.lights.length && r.idx !== -1) return false;
    if (dot(r.pos, r.pos) < f(EPS * EPS) && r.idx >= 0) return false;
    return true;
  }
  // isVisible, 1539-1557
  visible(from, to) {
    let sd = sub(to, from);
    const dist = length(sd);
    if (dist < f(EPS * 10)) return true;
    sd = normalize(sd);
    const h = this.intersect(add(from, muls(muls(sd, EPS), 2)), sd);
    if (h.t < f(dist - f(EPS * 2))) {
      if (h.index >= 0 && h.index < this.meshes.length) return this.meshes[h.index].mt === M_LIGHT;
      return false;
    }
    return true;
  }
  // texture(sampler, uv) of an RGBA32F plane: GL LINEAR + CLAMP_TO_EDGE, level 0
  bilinear(tex, u, v) {
    if (!tex) return [0, 0, 0, 0];
    const W = this.w, H = this.h;
    const x = f(f(u * W) - 0.5), y = f(f(v * H) - 0.5);
    const fx0 = Math.floor(x), fy0 = Math.floor(y), a = f(x - fx0), b = f(y - fy0);
    const cl = (i, n) => (i < 0 ? 0 : (i > n - 1 ? n - 1 : i));
    const x0 = cl(fx0, W), x1 = cl(fx0 + 1, W), y0 = cl(fy0, H), y1 = cl(fy0 + 1, H);
    const out = [0, 0, 0, 0];
    for (let c = 0; c < 4; c++) {
      const t00 = tex[(y0 * W + x0) * 4 + c], t10 = tex[(y0 * W + x1) * 4 + c];
      const t01 = tex[(y1 * W + x0) * 4 + c], t11 = tex[(y1 * W + x1) * 4 + c];
      const top = f(t00 + f(a * f(t10 - t00))), bot = f(t01 + f(a * f(t11 - t01)));
      out[c] = f(top + f(b * f(bot - top)));
    }
    return out;
  }
  // unpackReservoir, 1437-1468
  unpack(m, a) {
    const r = EMPTY_RES();
    if (m[3] > 0) {
      r.pos = V(m[0], m[1], m[2]);
      r.W = m[3];
      r.col = V(a[0], a[1], a[2]);
      const pa = a[3];
      const nli = fract(f(pa * f(2.94)));
      const temp = f(pa - f(nli * f(0.34)));
      const nM = fract(f(temp * f(3.03)));
      const nage = f(f(temp - f(nM * f(0.33))) * f(3.03));
      r.age = f(nage * 30);
      r.M = f(nM * 100);
      const len1 = this.lights.length > 1 ? this.lights.length : 1;
      r.idx = Math.trunc(f(nli * len1)) - 1;
      if (r.idx < -1) r.idx = -1;
      if (r.idx > this.lights.length - 1) r.idx = this.lights.length - 1;
      r.M = gmax(1, r.M);
      r.ws = f(r.W * r.M);
    }
    return r;
  }
  // combineReservoirs, 1579-1611
  combine(t, s, hp, hn, m, rnd) {
    if (!this.validRes(s)) return;
    const tw = targetFn(s.pos, s.col, hp, hn, m);
    if (tw <= 0) return;
    const sc = clamp(f(f(tw * gmax(s.W, 0)) * gmax(s.M, 1)), 0, 200);
    t.ws = f(t.ws + sc);
    t.M = f(t.M + s.M);
    if (t.M > 40) {
      const inv = f(40 / t.M);
      t.ws = f(t.ws * inv);
      t.M = 40;
    }
    if (t.ws > 0) {
      const p = f(sc / t.ws);
      if (rnd < p) { t.pos = s.pos; t.col = s.col; t.idx = s.idx; t.age = gmin(f(s.age + f(0.25)), 30); }
    }
  }
  // sampleLightsReSTIR, 1619-1801 (RENDER_MODE 0); sets this.fr (g_final_reservoir)
  restirLight(hp, hn, m, sx, sy, frame) {
    if (!this.restir) return V(0, 0, 0);
    const nl = this.lights.length;
    if (nl === 0 || this.lights[0] < 0) return V(0, 0, 0);
    const scx = f(this.fcx / this.w), scy = f(this.fcy / this.h);
    const init = EMPTY_RES();
    const eff = Math.min(this.restirSamples, Math.max(nl, 4));
    for (let i = 0; i < eff; i++) {
      const rv = hash2(f(sx + f(f(i) * f(0.1))), f(sy + f(f(i) * f(0.2))));
      let ai = Math.trunc(f(rv[0] * nl));
      ai = ai < 0 ? 0 : (ai > nl - 1 ? nl - 1 : ai);
      const li = this.lights[ai];
      if (li < 0 || li >= this.meshes.length) continue;
      const L = this.meshes[li];
      const tv = targetFn(L.pos, mul(L.c, L.e), hp, hn, m);
      if (tv > 0) updateReservoir(init, L.pos, mul(L.c, L.e), li, tv, rv[1]);
    }
    const tr = Object.assign({}, init);
    if (frame > 2) {
      for (let lvl = 0; lvl < 2; lvl++) {  // sampleTemporalHistory, 1485-1523
        let h = EMPTY_RES();
        const m3 = sub(hp, this.camPos);
        const ms = f(f(0.001) * (lvl + 1));
        const mvx = f(m3.x * ms), mvy = f(m3.y * ms);
        const js = f(f(lvl + frame) * f(0.1));
        const hj = hash2(f(scx + js), f(scy + js));
        const jx = f(f(hj[0] - 0.5) * f(0.002)), jy = f(f(hj[1] - 0.5) * f(0.002));
        const px = f(f(scx + mvx) + jx), py = f(f(scy + mvy) + jy);
        if (!(px < f(0.01) || px > f(0.99) || py < f(0.01) || py > f(0.99))) {
          h = this.unpack(this.bilinear(this.tex[lvl === 0 ? 2 : 4], px, py),
            this.bilinear(this.tex[lvl === 0 ? 3 : 5], px, py));
          if (this.validRes(h)) h.age = f(h.age + (lvl + 1));
        }
        if (this.validRes(h) && h.M > 0 && h.age < 30) {
          h.age = f(h.age + (lvl + 1));
          let ta = f(0.95);
          if (lvl === 1) ta = f(ta * f(0.80));
          h.M = f(h.M * ta);
          h.ws = f(h.ws * ta);
          const trand = hash(f(f(sx + f(789.123)) + f(f(lvl) * f(456.789))));
          this.combine(tr, h, hp, hn, m, trand);
        }
      }
      if (tr.M > 100) { tr.M = gmin(tr.M, 80); tr.ws = f(tr.ws * f(0.9)); }
    }
    const fr = Object.assign({}, tr);
    let ns = 8;
    if (nl > 10) ns = 4;
    if (frame < 10) ns = Math.max(Math.trunc(ns / 2), 2);
    for (let i = 0; i < ns; i++) {
      const sr = hash2(f(sx + f(f(i) * f(0.3))), f(sy + f(f(i) * f(0.4))));
      const ox = f(f(POISSON[i][0] * 16) / this.w), oy = f(f(POISSON[i][1] * 16) / this.h);
      const nx = f(scx + ox), ny = f(scy + oy);
      let nb = EMPTY_RES();
      if (!(nx < 0 || nx > 1 || ny < 0 || ny > 1)) nb = this.unpack(this.bilinear(this.tex[0], nx, ny), this.bilinear(this.tex[1], nx, ny));
      if (nb.M > 0) {
        if (nb.idx >= 0) {
          const ldf = sub(nb.pos, hp);
          if (dot(ldf, ldf) > 225) continue;
        }
        if (nb.age > 24 || sr[0] < f(0.03)) continue;
        this.combine(fr, nb, hp, hn, m, sr[1]);
      }
    }
    // finalizeReservoir, 1525-1576
    if (fr.ws <= 0 || fr.M <= 0) fr.W = 0;
    else {
      const tp = targetFn(fr.pos, fr.col, hp, hn, m);
      if (tp <= 0 || !this.visible(hp, fr.pos)) fr.W = 0;
      else {
        const cM = clamp(fr.M, 1, 40);
        const raw = f(fr.ws / f(tp * cM));
        let bc = 1;
        if (fr.age > 0) {
          const na = clamp(f(fr.age / 30), 0, 1);
          bc = f(bc * mixf(f(0.85), 1, f(1 - f(na * f(0.3)))));
        }
        if (cM > 16) bc = f(bc * f(Math.sqrt(f(16 / cM))));
        fr.W = clamp(f(bc * raw), 0, 12);
        if (!finite(fr.W)) fr.W = 0;
      }
    }
    fr.age = gmin(fr.age, 30);
    this.fr = fr;
    if (fr.W > 0 && fr.idx >= 0 && fr.idx < nl) {
      const act = this.lights[fr.idx];
      if (act >= 0 && act < this.meshes.length) {
        const lc = this.directLight(act, hp, hn, f(sx + f(456.789)));
        let ew = clamp(fr.W, 0, 8);
        if (fr.M > 30) ew = f(ew * f(Math.sqrt(f(30 / fr.M))));
        const fc = muls(lc, ew);
        if (!finite(fc.x) || !finite(fc.y) || !finite(fc.z)) return V(0, 0, 0);
        return fc;
      }
    }
    return V(0, 0, 0);
  }

  // radiance() + brdf(), 1986-2105 and 1804-1980
  radiance(ro, rd, seed, frame) {
    let acc = V(0, 0, 0), mask = V(1, 1, 1), spec = true, prevNl = V(0, 1, 0);
    let diffB = 0, specB = 0, scat = 0;
    const fr = f(frame);
    for (let depth = 0; depth < this.maxB; depth++) {
      const hit = this.intersect(ro, rd);
      if (this.vol) {
        const sd = f(f(-f(Math.log(gmax(hash(f(f(seed + f(4729.3)) + f(f(depth) * f(991.1)))), f(1e-6))))) / VOL_SIGMA_T);
        if (sd < gmin(INF_T, hit.t)) {
          const sp = add(ro, muls(rd, sd));
          mask = muls(mask, f(VOL_SIGMA_S / VOL_SIGMA_T));
          if (this.sampleLights) {
            for (let li = 0; li < this.lights.length; li++) {
              const lidx = this.lights[li];
              if (lidx < 0) continue;
              const L = this.meshes[lidx];
              if (L.mt !== M_LIGHT || L.t !== T_SPHERE) continue;
              const dlc = sub(L.pos, sp), dc = length(dlc);
              const r2 = f(L.joker[0] * L.joker[0]);
              const cam = f(Math.sqrt(f(1 - clamp(f(r2 / f(dc * dc)), 0, 1))));
              const s2 = f(f(f(seed + f(2341.7)) + f(f(li) * f(917.3))) + f(f(depth) * f(199.1)));
              const dir = CpuRenderer.coneSample(V(f(dlc.x / dc), f(dlc.y / dc), f(dlc.z / dc)), f(1 - cam), s2);
              const sh = this.intersect(add(sp, muls(dir, f(EPS * 20))), dir);
              if (sh.index !== lidx) continue;
              const omega = f(2 * f(1 - cam)), ct = dot(rd, dir);
              const g2 = f(VOL_G * VOL_G), den = f(f(1 + g2) - f(f(2 * VOL_G) * ct));
              const phase = f(f(1 - g2) / f(f(FOUR_PI * den) * f(Math.sqrt(den))));
              const Tf = f(Math.exp(f(-VOL_SIGMA_T * sh.t)));
              acc = add(acc, muls(muls(muls(mul(mul(mask, L.c), L.e), phase), Tf), f(PI_F * omega)));
            }
          }
          rd = sampleHG(rd, f(f(seed + f(8293.7)) + f(f(depth) * f(773.3))));
          ro = sp; spec = false; scat++;
          if (scat >= this.maxSc || vmaxc(mask) < f(0.01)) break;
          continue;
        }
      }
      if (hit.t === INF_T) {
        if (!spec && this.sampleLights) break;
        if (this.sky) {
          const k = clamp(f(f(rd.y * f(0.6)) + 0.5), f(0.3), 1);
          const sky = V(f(0.5 + f(0.5 * fcos(f(TWO_PI * f(f(0.525) + f(f(0.9) * k)))))),
            f(0.5 + f(0.5 * fcos(f(TWO_PI * f(f(0.408) + f(f(0.97) * k)))))),
            f(0.5 + f(0.5 * fcos(f(TWO_PI * f(f(0.409) + f(f(0.8) * k)))))));
          acc = add(acc, mul(mask, sky));
        }
        break;
      }
      const m = this.meshes[hit.index];
      const c = vmaxs(m.c, f(0.001)), e = vmaxs(m.e, f(0.001));
      const inside = -sgn(dot(rd, hit.n));
      if (m.mt === M_LIGHT) {
        mask = mul(mask, c);
        let w = 1;
        if (this.mis && !spec && this.sampleLights && depth > 0) {
          const ld = normalize(sub(hit.pos, ro));
          w = CpuRenderer.power(CpuRenderer.cosPdf(ld, prevNl), CpuRenderer.lightPdf(m, ro));
        }
        acc = add(acc, muls(mul(mask, e), w));
        break;
      }
      prevNl = muls(hit.n, inside);
      const x = hit.pos, nl = prevNl, bounce = f(depth);
      const rdir = this.randomDirection(nl, f(f(f(seed + f(f(7.1) * fr)) + f(5681.123)) + f(bounce * f(92.13))));
      const rough = mul(e, rdir);
      const nc = f(1.00029), mt = m.mt;
      // USE_SPECTRAL: a negative IOR is Cauchy's A at the hero wavelength (1819-1824)
      const nt = this.spectral && m.nt < 0 ? spectralIOR(this.hero, Math.abs(m.nt)) : Math.abs(m.nt);
      if (mt === M_DIFF) {
        ro = add(x, muls(nl, EPS)); rd = rdir; mask = mul(mask, c); diffB++; spec = false;
      } else if (mt === M_SPEC) {
        ro = add(x, muls(nl, EPS)); rd = normalize(add(rough, reflect(rd, nl))); mask = mul(mask, c); specB++; spec = true;
      } else if (mt === M_REFR_FRESNEL || mt === M_REFR_SCHLICK) {
        const nnt = inside < 0 ? f(nt / nc) : f(nc / nt);
        let tdir = refract(rd, nl, nnt);
        if (length(tdir) === 0) {
          ro = add(x, muls(nl, EPS)); rd = normalize(add(rough, reflect(rd, nl))); specB++; spec = true;
        } else {
          tdir = normalize(add(rough, tdir));
          let Re;
          if (mt === M_REFR_FRESNEL) {
            const cosI = dot(rd, nl), cosT = dot(nl, tdir);
            const rs = f(f(f(nc * cosI) - f(nt * cosT)) / f(f(nc * cosI) + f(nt * cosT)));
            const rp = f(f(f(nc * cosT) - f(nt * cosI)) / f(f(nc * cosT) + f(nt * cosI)));
            Re = f(f(f(rs * rs) + f(rp * rp)) * 0.5);
          } else {
            const q = f(f(nc - nt) / f(nc + nt)), R0 = f(q * q);
            Re = f(R0 + f(f(1 - R0) * gpow(f(1 + dot(nl, rd)), 5)));
          }
          if (hash(seed) < Re) {
            ro = add(x, muls(nl, EPS)); rd = normalize(add(rough, reflect(rd, nl))); specB++;
          } else {
            ro = sub(x, muls(nl, EPS)); mask = mul(mask, c); rd = tdir; scat++;
          }
          spec = true;
        }
      } else if (mt === M_COAT) {
        ro = add(x, muls(nl, EPS));
        const q = f(f(nc - nt) / f(nc + nt)), R0 = f(q * q);
        const Re = f(R0 + f(f(1 - R0) * gpow(f(1 + dot(nl, rd)), 5)));
        if (hash(seed) < Re) { rd = normalize(add(rough, reflect(rd, nl))); specB++; spec = true; } else {
          rd = rdir; mask = mul(mask, c); diffB++; spec = false;
        }
      }
      if (!spec && this.sampleLights && this.restir) {  // 1900-1946: ReSTIR routes
        if (this.restirDef) {
          const sx = f(f(seed + f(f(8652.1) * fr)) + f(bounce * f(7895.13)));
          const sy = f(f(seed + f(f(1234.567) * fr)) + f(bounce * f(9876.54)));
          let tot = V(0, 0, 0);
          if (!this.mis || this.lights.length > 8) {
            tot = this.restirLight(x, nl, m, sx, sy, frame);
          } else {  // use_mis with <= 8 lights: importance-culled MIS over the lights
            const base = f(f(f(seed + f(f(8652.1) * fr)) + f(5681.123)) + f(bounce * f(7895.13)));
            for (let i = 0; i < this.lights.length; i++) {
              const idx = this.lights[i];
              if (idx < 0) continue;
              const L = this.meshes[idx];
              if (L.mt !== M_LIGHT) continue;
              const lv = sub(L.pos, x), ld = normalize(lv), dsq = dot(lv, lv);
              const ct = gmax(0, dot(nl, ld));
              const imp = f(f(ct * dot(L.e, LUM)) * isqrt(f(dsq + 1)));
              if (imp < f(0.001)) continue;
              const ls = this.directLight(idx, x, nl, f(base + f(f(i) * f(123.456))));
              if (dot(ls, ls) < f(f(0.001) * f(0.001))) continue;
              tot = add(tot, muls(ls, CpuRenderer.power(CpuRenderer.lightPdf(L, x), CpuRenderer.cosPdf(ld, nl))));
            }
          }
          acc = add(acc, mul(tot, mask));
        }
      } else if (!spec && this.sampleLights) {  // 1899-1976
        const base = f(f(f(seed + f(f(8652.1) * fr)) + f(5681.123)) + f(bounce * f(7895.13)));
        let lc = V(0, 0, 0);
        for (let i = 0; i < this.lights.length; i++) {
          const idx = this.lights[i];
          if (idx < 0) continue;
          if (this.mis) {
            const L = this.meshes[idx];
            if (L.mt !== M_LIGHT) continue;
            const ls = this.directLight(idx, x, nl, f(base + f(f(i) * f(123.456))));
            if (dot(ls, ls) > f(0.000001)) {
              const ld = normalize(sub(L.pos, x));
              lc = add(lc, muls(ls, CpuRenderer.power(CpuRenderer.lightPdf(L, x), CpuRenderer.cosPdf(ld, nl))));
            }
          } else {
            acc = add(acc, mul(this.directLight(idx, x, nl, base), mask));
          }
        }
        if (this.mis) acc = add(acc, mul(lc, mask));
      }
      if (vmaxc(mask) < f(0.01)) break;
      if (diffB >= this.maxD || specB >= this.maxS || 0 >= this.maxT || scat >= this.maxSc) break;
    }
    return acc;
  }

  // main(), 2111-2180: one sample of pixel (px, py) (py counted from the bottom)
  sample(px, py, frame) {
    const rx = f(this.w), ry = f(this.h);
    const fcx = f(px + 0.5), fcy = f(py + 0.5);
    this.fcx = fcx;
    this.fcy = fcy;
    this.fr = EMPTY_RES();
    const stx = f(f(f(2 * fcx) / rx) - 1), sty = f(f(f(2 * fcy) / ry) - 1);
    const seed = hash(f(f(f(fcx * f(12.9898)) + f(fcy * f(78.233))) + f(f(1113.1) * f(frame))));
    this.hero = this.spectral ? f(f(hash(f(seed + f(4821.73))) * 340) + 380) : f(550);  // 2123
    const uVLen = f(Math.tan(f(f(this.camParams.x * RAD) * 0.5)));
    const uULen = f(f(rx / ry) * uVLen);
    const w = normalize(this.camLook);
    const u = normalize(cross(w, V(0, 1, 0)));
    const v = cross(u, w);
    const ax = hash(f(seed + f(13.271))), ay = hash(f(seed + f(63.216)));
    const flx = step(0.5, ax), fly = step(0.5, ay);
    const hx = mixf(ax, f(1 - ax), flx), hy = mixf(ay, f(1 - ay), fly);
    const sx = f(Math.sqrt(f(2 * hx))), sy = f(Math.sqrt(f(2 * hy)));
    const dx = f(f(mixf(f(sx - 1), f(1 - sx), flx) / f(rx * 0.5)) + stx);
    const dy = f(f(mixf(f(sy - 1), f(1 - sy), fly) / f(ry * 0.5)) + sty);
    const fp = muls(normalize(add(add(muls(muls(u, dx), uULen), muls(muls(v, dy), uVLen)), w)), this.camParams.z);
    const ang = f(hash(f(seed + f(496.4562))) * TWO_PI);
    const rad = f(hash(f(seed + f(249.1686))) * this.camParams.y);
    const ap = muls(add(muls(u, fcos(ang)), muls(v, fsin(ang))), rad);
    const col = this.radiance(add(this.camPos, ap), normalize(sub(fp, ap)), seed, frame);
    return this.spectral ? mul(col, wavelengthToRGB(this.hero)) : col;  // 2152-2155
  }

  // One ReSTIR pass over rows [y0, y1): sample[y][x] = that pass's sample
  // (rgb, a = 0); main/aux = the packed g_final_reservoir MRTs (1418-1433,
  // 2171-2179).  this.tex holds the six reservoir input planes (W*H RGBA
  // Float32Arrays, rows bottom-up, or null for zeros).
  renderPass(frame, y0, y1, sample, main, aux) {
    const len1 = this.lights.length > 1 ? this.lights.length : 1;
    const x0 = this.x0 || 0, x1 = this.x1 || this.w;  // column span (bench samples of costly scenes)
    for (let y = y0; y < y1; y++) {
      for (let x = x0; x < x1; x++) {
        const s = this.sample(x, y, frame), p = (y * this.w + x) * 4, r = this.fr, have = this.restirDef;
        sample[p] = s.x; sample[p + 1] = s.y; sample[p + 2] = s.z; sample[p + 3] = 0;
        main[p] = have ? r.pos.x : 0; main[p + 1] = have ? r.pos.y : 0; main[p + 2] = have ? r.pos.z : 0;
        main[p + 3] = have ? r.W : 0;
        const na = clamp(f(r.age / 30), 0, 1), nM = clamp(f(r.M / 100), 0, 1), nli = f((r.idx + 1) / len1);
        aux[p] = have ? r.col.x : 0; aux[p + 1] = have ? r.col.y : 0; aux[p + 2] = have ? r.col.z : 0;
        aux[p + 3] = have ? f(f(f(na * f(0.33)) + f(nM * f(0.33))) + f(nli * f(0.34))) : 0;
      }
    }
  }

  // rows [y0, y1) of passes frame0..frame0+n-1 accumulated: Float32Array RGBA
  render(frame0, n, y0, y1) {
    const out = new Float32Array((y1 - y0) * this.w * 4);
    for (let y = y0; y < y1; y++) {
      for (let x = 0; x < this.w; x++) {
        const o = ((y - y0) * this.w + x) * 4;
        for (let k = 0; k < n; k++) {
          const s = this.sample(x, y, frame0 + k);
          out[o] = f(out[o] + s.x);
          out[o + 1] = f(out[o + 1] + s.y);
          out[o + 2] = f(out[o + 2] + s.z);
        }
      }
    }
    return out;
  }
}

module.exports = { CpuRenderer, hash, hash2, parseScene, wavelengthToRGB, spectralIOR };
