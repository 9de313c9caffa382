'use strict';
/*
 * make_shader.js -- expand the REFERENCE ray-tracing shader for one oracle config.
 *
 * TEST INFRASTRUCTURE ONLY (golden-vector generation in this container).
 * It loads the reference's own tools.js / vector.js / index.js into a Node `vm`
 * context, lets `new GlslViewport(fakeCanvas)` populate its defaults (the
 * constructor returns early when getContext() yields null, index.js:106-110),
 * applies the config's defines/constants/scene/sdf_meshes overrides, and calls
 * the reference's parseShader (tools.js:22-61) on
 * shaders/pathtracing/raytracer.glsl.  The expanded text is written OUTSIDE of
 * version control (oracle/_gen/, git- and gpurun-ignored).
 *
 * Textual edits applied to the expanded text (every fixture):
 *   1. `const Mesh meshes[` -> `Mesh meshes[` (required: SwiftShader 4.1 rejects
 *      dynamic indexing into const struct arrays; semantically neutral).
 *   2. the `out` parameters of iBox (`out vec3 n`, raytracer.glsl:836) and iSDF
 *      (`out vec3 n, out int index`, 974) become `inout`.  This is a REAL
 *      modification of the reference, not a neutral one: GLSL leaves an `out`
 *      parameter the callee does not assign undefined, and iBox/iSDF return
 *      false without assigning them while intersection() passes hit.n /
 *      hit.index (1028, 1041) and relies on them keeping their values
 *      (HIT_MISS, 998).  SwiftShader copies out a stale register there, which
 *      turns every SDF miss into hit.index = NUM_MESHES and renders scenes that
 *      mix quadrics with SDFs black.  `inout` pins the undefined value to "the
 *      caller's value unchanged", the only reading under which the reference
 *      renders its own scenes (DESIGN.md 2).
 *   3. the volumetric in-scatter light loop's `if (c) continue;` statements are
 *      rewritten as the equivalent `if (!(c)) { ... }` (SwiftShader 4.1 does not
 *      finish the loop as written; see the edit below).  GLSL semantics unchanged.
 *   4. with --nanfix only: powerHeuristic's `max(0.0, (f*f)/denom)` becomes
 *      `denom > 0.0 ? (f*f)/denom : 0.0`, i.e. IEEE-maxNum semantics for the 0/0
 *      case (raytracer.glsl:1233-1238).  Every non-NaN pixel is unchanged.
 *      No committed fixture uses it (manifest.json: unpatched powerHeuristic).
 * With --kat, the reference main() is renamed and a known-answer main() that
 * writes the RNG stream (seed schedule of raytracer.glsl:2120, 2135, 2143,
 * 1810, 1972/1190) into the three MRTs is appended.
 *
 * usage: node make_shader.js <configs.json> <config-name> <out.frag> [--nanfix] [--kat]
 */
const fs = require('fs');
const path = require('path');
const vm = require('vm');

const REF = process.env.RT0_REFERENCE || '/root/reference';

function loadReference() {
  const quiet = () => {};
  const fakeCanvas = { getContext: () => null };
  const ctx = {
    console: { log: quiet, error: quiet, info: quiet, warn: quiet, clear: quiet },
    window: { devicePixelRatio: 1 },
    performance: { now: () => 0 },
    document: { createElement: () => fakeCanvas, dispatchEvent: quiet },
  };
  ctx.XMLHttpRequest = class {
    open(method, url) { this.url = url; }
    overrideMimeType() {}
    send() {
      this.responseText = fs.readFileSync(path.join(REF, this.url), 'utf8');
      this.readyState = 4;
      this.status = 200;
      if (this.onreadystatechange) this.onreadystatechange();
    }
  };
  vm.createContext(ctx);
  for (const f of ['tools.js', 'vector.js', 'index.js']) {
    vm.runInContext(fs.readFileSync(path.join(REF, f), 'utf8'), ctx, { filename: f });
  }
  return ctx;
}

// index.html:610-676 -- textarea lines -> GLSL scene text (restated: the page
// script is inline HTML with jQuery and cannot be loaded headlessly).
function sceneFromLines(lines) {
  let NUM_MESHES = 0, NUM_SDFS = 0, NUM_MODELS = 0;
  let U_SPHERE = false, U_PLANE = false, U_BOX = false;
  const light_indices = [];
  const text = [];
  for (let i = 0; i < lines.length; i++) {
    const fields = lines[i].split(',');
    const mat = fields[0].trim();
    if (mat.lastIndexOf('MAT_LIGHT') >= 0) light_indices.push(i);
    const type = fields[1].trim();
    text[i] = 'Mesh(' + lines[i] + ')';
    if (i != lines.length - 1) text[i] += ',';
    if (type == 'SDF' || type == 'GRID_SDF') NUM_SDFS++;
    else if (type == 'PLANE' || type == 'SPHERE' || type == 'BOX') {
      U_SPHERE = U_SPHERE || type == 'SPHERE';
      U_PLANE = U_PLANE || type == 'PLANE';
      U_BOX = U_BOX || type == 'BOX';
      NUM_MESHES++;
    } else if (type == 'TRIANGLE') NUM_MODELS++;
    else throw new Error("There's no such thing as " + type);
  }
  if (light_indices.length == 0) light_indices.push(-1);
  const scene = `//--------------------- EUCLIDEAN/QUADRIC PARAMS --------------------------------

const bool U_EUCLIDEAN = ` + (NUM_MESHES > 0) + `;
const bool U_SPHERE = ` + Boolean(U_SPHERE) + `;
const bool U_PLANE = ` + Boolean(U_PLANE) + `;
const bool U_BOX = ` + Boolean(U_BOX) + `;
const bool U_SDF = ` + (NUM_SDFS > 0) + `;

const lowp int NUM_MESHES = ` + NUM_MESHES + `;
const lowp int NUM_SDFS   = ` + NUM_SDFS + `;
const lowp int NUM_MODELS = ` + NUM_MODELS + `;

const Mesh meshes[NUM_MESHES + NUM_SDFS + NUM_MODELS] = Mesh[](
` + text.join('\n') + `
);

// light index
const lowp int light_index[` + light_indices.length + `] = int[](
` + light_indices.join(', ') + `
);`;
  return { scene, NUM_SDFS };
}

// index.html:702-717 -- SDF selector value -> map() statement.
function sdfStatement(i, kind) {
  const m = 'meshes[NUM_MESHES + ' + i + ']';
  const id = i.toFixed(4);
  switch (kind) {
    case 0: return `sdf_meshes[${i}] = vec2(sdBox(p-${m}.pos, ${m}.joker.xyz), ${id});`;
    case 1: return `sdf_meshes[${i}] = vec2(udRoundBox(p-${m}.pos, ${m}.joker.xyz, ${m}.joker.w), ${id});`;
    case 2: return `sdf_meshes[${i}] = vec2(sdSphere(p-${m}.pos, ${m}.joker.x), ${id});`;
    case 3: return `sdf_meshes[${i}] = vec2(sdTriPrism(p-${m}.pos, ${m}.joker.xy), ${id});`;
    case 4: return `sdf_meshes[${i}] = vec2(sdCone(p-${m}.pos, ${m}.joker.xyz), ${id});`;
    case 5: return `sdf_meshes[${i}] = vec2(MengerSponge(p-${m}.pos, ${m}.joker.xyz), ${id});`;
    case 6: return `sdf_meshes[${i}] = vec2(Mandelbulb(p-${m}.pos), ${id});`;
    default: throw new Error('unsupported sdf kind ' + kind);
  }
}

const DEFINE_NAMES = ['USE_CUBEMAP', 'USE_PROCEDURAL_SKY', 'USE_BIASED_SAMPLING',
  'USE_BIDIRECTIONAL', 'USE_RESTIR', 'USE_SPECTRAL', 'USE_VOLUMETRICS'];

function applyConfig(vp, cfg) {
  for (const [name, on] of Object.entries(cfg.defines || {})) {
    const k = DEFINE_NAMES.indexOf(name);
    if (k < 0) throw new Error('unknown define ' + name);
    vp.defines[k] = (on ? '' : '//') + '#define ' + name;
  }
  for (const [name, val] of Object.entries(cfg.constants || {})) {
    const k = vp.constants.findIndex((s) => new RegExp('\\b' + name + '\\s*=').test(s));
    if (k < 0) throw new Error('unknown constant ' + name);
    vp.constants[k] = vp.constants[k].replace(/=\s*[^;]+;/, '= ' + String(val) + ';');
  }
  if (cfg.scene_lines) {
    const { scene, NUM_SDFS } = sceneFromLines(cfg.scene_lines);
    vp.scene = scene;
    const kinds = cfg.sdf_kinds || [];
    vp.sdf_meshes = [];
    for (let i = 0; i < NUM_SDFS; i++) vp.sdf_meshes.push(sdfStatement(i, kinds[i] || 0));
  }
}

const KAT_MAIN = `
void main(void){
  float seed = hash(dot( gl_FragCoord.xy, vec2(12.9898, 78.233) ) + 1113.1*float(u_frame));
  FragColor = vec4(seed, hash(seed+13.271), hash(seed+63.216), hash(seed+496.4562));
  vec2 b0 = hash2(vec2(seed + 7.1*float(u_frame) + 5681.123 + 0.0*92.13));
  vec2 b3 = hash2(vec2(seed + 7.1*float(u_frame) + 5681.123 + 3.0*92.13));
  ReSTIRData = vec4(b0, b3);
  vec2 n1 = hash2(vec2(seed + 8652.1*float(u_frame) + 5681.123 + 1.0*7895.13 + 23.1656));
  ReSTIRAux = vec4(n1, hash(seed+249.1686), dot( gl_FragCoord.xy, vec2(12.9898, 78.233) ) + 1113.1*float(u_frame));
}
`;

function main() {
  const args = process.argv.slice(2);
  const [cfgFile, name, out] = args;
  const nanfix = args.includes('--nanfix');
  const kat = args.includes('--kat');
  const cfgs = JSON.parse(fs.readFileSync(cfgFile, 'utf8'));
  const cfg = cfgs.configs.find((c) => c.name === name);
  if (!cfg) throw new Error('no config ' + name);

  const ctx = loadReference();
  ctx.__cfg = cfg;
  const vp = vm.runInContext('new GlslViewport({ getContext() { return null; } }, {})', ctx);
  applyConfig(vp, cfg);
  ctx.__vp = vp;
  let src = vm.runInContext("parseShader('shaders/pathtracing/raytracer.glsl', __vp)", ctx);

  const n1 = src.split('const Mesh meshes[').length - 1;
  if (n1 !== 1) throw new Error('expected exactly one `const Mesh meshes[`, found ' + n1);
  src = src.replace('const Mesh meshes[', 'Mesh meshes[');
  // 2. iBox / iSDF leave their `out` normal (and iSDF its `out` index) unassigned
  //    on a miss (raytracer.glsl:836-859, 974-993).  GLSL makes such values
  //    undefined; SwiftShader copies out a stale register, which after the first
  //    SDF hit turns every later SDF miss into hit.index = NUM_MESHES (black
  //    images for every scene mixing quadrics and SDFs).  Declaring them `inout`
  //    pins the undefined value to "caller's value unchanged" -- the behaviour
  //    intersection() relies on (it pre-sets hit = HIT_MISS, 998) and the one the
  //    Cornell fixtures already exhibit.
  const patches = [
    ['bool iBox(const Mesh box, in Ray r, in float tmin, out float t, out vec3 n){',
     'bool iBox(const Mesh box, in Ray r, in float tmin, out float t, inout vec3 n){'],
    ['bool iSDF(in Ray r, in float tmin, out float t, out vec3 n, out int index){',
     'bool iSDF(in Ray r, in float tmin, out float t, inout vec3 n, inout int index){'],
  ];
  for (const [from, to] of patches) {
    if (src.split(from).length !== 2) throw new Error('patch target not found: ' + from);
    src = src.replace(from, to);
  }
  // 3. the in-scatter light loop of the volumetric branch (raytracer.glsl:
  //    2011-2044) skips lights with `if (...) continue;` three times.  SwiftShader
  //    4.1 does not finish that loop: an 8x8 render with it ran > 20 min (killed),
  //    the same shader with each `if (c) continue; rest` written as the
  //    equivalent `if (!(c)) { rest }` renders in 1.9 s, as does one without the
  //    loop.  GLSL semantics are unchanged; USE_VOLUMETRICS scenes only (the block
  //    is preprocessed out everywhere else).
  {
    const head = 'for (int li = 0; li < num_lights; ++li) {';
    const tail = 'acc += mask * lm.mat.c * lm.mat.e * phase * T_fog * (PI * omega);';
    if (src.split(head).length !== 2 || src.split(tail).length !== 2) throw new Error('volumetric light loop not found');
    const i = src.indexOf(head), j = src.indexOf(tail, i) + tail.length;
    let body = src.slice(i, j), n = 0;
    for (const cond of ['light_idx < 0', 'lm.mat.t != LIGHT || lm.t != SPHERE', 'sh.index != light_idx']) {
      const from = 'if (' + cond + ') continue;';
      if (body.split(from).length !== 2) throw new Error('volumetric loop pattern not found: ' + from);
      body = body.replace(from, 'if (!(' + cond + ')) {');
      n++;
    }
    src = src.slice(0, i) + body + ' ' + '}'.repeat(n) + src.slice(j);
  }
  if (nanfix) {
    const needle = 'return max(0.0, (f * f) / denom);';
    if (src.split(needle).length !== 2) throw new Error('powerHeuristic pattern not found');
    src = src.replace(needle, 'return denom > 0.0 ? (f * f) / denom : 0.0;');
  }
  if (kat) {
    if (src.split('void main(void){').length !== 2) throw new Error('main() not found');
    src = src.replace('void main(void){', 'void main_reference(void){') + KAT_MAIN;
  }
  fs.mkdirSync(path.dirname(out), { recursive: true });
  fs.writeFileSync(out, src);
  // echo the effective host-side state so the fixture sidecar records it
  process.stdout.write(JSON.stringify({
    defines: vp.defines, constants: vp.constants, scene: vp.scene,
    sdf_meshes: vp.sdf_meshes,
    camera: {
      origin: [vp.camera.origin.x, vp.camera.origin.y, vp.camera.origin.z],
      lookat: [vp.camera.lookat.x, vp.camera.lookat.y, vp.camera.lookat.z],
      fov: vp.camera.fov, aperture: vp.camera.aperture, focalLength: vp.camera.focalLength,
    },
  }));
}

main();
