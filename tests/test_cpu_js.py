"""The JS CPU integrator (raytracer-0_amd/js/rt0_cpu.js) -- GlslViewport's CPU
backend (opts.backend = 'cpu', BASELINE configs[0]) and the reported CPU
baseline of bench.py, SURVEY 8d -- renders what the reference renders: checked against
the golden fixtures (the reference shader under SwiftShader) and the C oracle
on the configs it covers (quadrics, SDFs, volumetrics, ReSTIR).  CPU only."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "oracle", "js", "cpu_bench.js")
CONFIGS = os.path.join(REPO, "tests", "golden", "configs.json")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is missing")


def js_image(name, w, h, frame0, n, tmp_path, threads=4, extra=()):
    out = tmp_path / ("%s.f32" % name)
    r = subprocess.run([NODE, BENCH, CONFIGS, name, str(w), str(h), str(threads), "image", str(frame0), str(n),
                        str(out)] + list(extra), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return np.fromfile(str(out), np.float32).reshape(h, w, 4)


def match(a, b):
    return ((np.abs(a[..., :3] - b[..., :3]) <= 1e-3 * np.maximum(1.0, np.abs(b[..., :3]))).all(-1)).mean()


@pytest.mark.parametrize("name", ["c1_cornell_cos", "c2_cornell_mis_refcaps", "c2_cornell_mis_8", "cornell_nee_plain",
                                  "thinlens_glass", "menger_coat", "sdf_cone", "sdf_triprism", "mis_demo_sdfbox"])
def test_js_integrator_matches_reference_fixtures(name, cfgs, tmp_path):
    gold = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))["samples"]
    F, H, W = gold.shape[:3]
    for k in (1, F):
        got = js_image(name, W, H, k, 1, tmp_path)
        # SDF scenes: every path grazes many edges (the oracle's own allowance, test_oracle_golden.BAD_FRAC)
        assert match(got, gold[k - 1]) >= (0.98 if name == "menger_coat" else 0.99), (name, k)


def test_js_integrator_matches_c_oracle_accumulated(cfgs, tmp_path):
    cfg = [c for c in cfgs["configs"] if c["name"] == "c2_cornell_mis_8"][0]
    o = O.Oracle(cfg, cfgs, width=48, height=40)
    ref = sum(o.frame(k)[0] for k in (1, 2, 3))
    got = js_image("c2_cornell_mis_8", 48, 40, 1, 3, tmp_path)
    assert match(got, ref) >= 0.99
    assert abs(got[..., :3].mean() - ref[..., :3].mean()) <= 1e-3 * ref[..., :3].mean()


@pytest.mark.parametrize("name", ["c4_mandelbulb_vol", "vol_cornell_2"])
def test_js_integrator_matches_c_oracle_sdf_volumetrics(name, cfgs, tmp_path):
    """C4's feature set (Mandelbulb SDF, homogeneous medium, in-scatter NEE):
    the JS baseline against the C restatement, single-sample frames."""
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    o = O.Oracle(cfg, cfgs, width=24, height=24)
    for k in (1, 2):
        ref = o.frame(k)[0]
        got = js_image(name, 24, 24, k, 1, tmp_path)
        assert match(got, ref) >= 0.99, (name, k)


def test_js_bench_mode_reports_throughput():
    r = subprocess.run([NODE, BENCH, CONFIGS, "c1_cornell_cos", "256", "256", "2", "bench", "0", "8", "0.5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["samples"] > 0 and d["msamples_s"] > 0 and d["threads"] == 2


def test_js_integrator_rejects_features_outside_its_scope(tmp_path):
    for name in ("anim_restir_demo",):  # RENDER_MODE 1
        r = subprocess.run([NODE, BENCH, CONFIGS, name, "16", "16", "1", "image", "1", "1",
                            str(tmp_path / "x.f32")], capture_output=True, text=True, timeout=120)
        assert r.returncode != 0 and "outside the JS CPU integrator" in r.stderr, name


def js_restir_chain(name, w, h, n, tmp_path, constants=None, threads=4, extra=()):
    out = tmp_path / ("%s_restir.f32" % name)
    cmd = [NODE, BENCH, CONFIGS, name, str(w), str(h), str(threads), "restir-image", str(n), str(out)] + list(extra)
    if constants:
        cmd += ["--constants", json.dumps(constants)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return np.fromfile(str(out), np.float32).reshape(n, 3, h, w, 4)


def res_match(a, b):
    return ((np.abs(a - b) <= 1e-3 * np.maximum(1.0, np.abs(b))).all(-1)).mean()


@pytest.mark.parametrize("name,constants", [("c3_outdoor_restir", None), ("restir_mis_demo", None),
                                            ("c3_outdoor_restir", {"use_mis": True})])
def test_js_restir_chain_matches_c_oracle(name, constants, cfgs, tmp_path):
    """ReSTIR in the JS baseline (sampleLightsReSTIR, raytracer.glsl:1619-1801,
    and index.js's swap chain, 795-820), GLSL semantics: six chained passes
    against the C restatement's chain -- samples and both reservoir MRTs per
    pass -- and pass 1 (no history yet) against the reference's own fixture.
    With use_mis and <= 8 lights the call routes to the importance-culled MIS
    loop instead (1900-1946): the third case."""
    cfg = dict([c for c in cfgs["configs"] if c["name"] == name][0])
    if constants:
        cfg["constants"] = dict(cfg.get("constants", {}), **constants)
    n = 6
    J = js_restir_chain(name, 64, 64, n, tmp_path, constants)
    S, M, A = O.Oracle(cfg, cfgs, width=64, height=64).frames_restir(n, cfg)
    for k in range(n):
        assert match(J[k, 0], S[k]) >= 0.995, (name, k + 1, "sample")
        assert res_match(J[k, 1], M[k]) >= 0.995 and res_match(J[k, 2], A[k]) >= 0.995, (name, k + 1, "reservoirs")
    assert abs(J[:, 0, ..., :3].mean() - S[..., :3].mean()) <= 1e-3 * S[..., :3].mean()
    if not constants:
        gold = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))["samples"]
        assert match(J[0, 0], gold[0]) >= 0.99


def test_js_restir_bench_mode_reports_throughput():
    r = subprocess.run([NODE, BENCH, CONFIGS, "c3_outdoor_restir", "192", "108", "2", "restir-bench", "40", "48", "0.5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["samples"] > 0 and d["msamples_s"] > 0 and d["threads"] == 2 and d["passes"] >= 1


def test_js_spectral_matches_reference_fixture(cfgs, tmp_path):
    """USE_SPECTRAL (hero wavelength, Cauchy IOR of MAT_SPECTRAL_FLINT, the CIE
    fit; raytracer.glsl:322-359, 1819-1824, 2153-2155) against the reference's
    own spectral Cornell fixture, first and last pass."""
    gold = np.load(os.path.join(REPO, "tests", "golden", "spectral_cornell.npz"))["samples"]
    F, H, W = gold.shape[:3]
    for k in (1, F):
        got = js_image("spectral_cornell", W, H, k, 1, tmp_path)
        assert match(got, gold[k - 1]) >= 0.99, k


def test_js_spectral_restir_chain_matches_c_oracle(cfgs, tmp_path):
    """C5 without the model (spectral + ReSTIR/MIS with 10 lights): the JS
    chain against the C restatement's, samples and reservoirs, and pass 1
    against the reference's fixture."""
    name = "c5_spectral_sphere"
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    n = 4
    J = js_restir_chain(name, 48, 48, n, tmp_path)
    S, M, A = O.Oracle(cfg, cfgs, width=48, height=48).frames_restir(n, cfg)
    for k in range(n):
        assert match(J[k, 0], S[k]) >= 0.995, (k + 1, "sample")
        assert res_match(J[k, 1], M[k]) >= 0.995 and res_match(J[k, 2], A[k]) >= 0.995, (k + 1, "reservoirs")
    gold = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))["samples"]
    assert match(js_restir_chain(name, 64, 64, 1, tmp_path)[0, 0], gold[0]) >= 0.99


def test_js_triangle_models_match_c_oracle(cfgs, tmp_path):
    """C5 itself (the 81,920-triangle model instanced by a TRIANGLE entry,
    spectral + ReSTIR/MIS): the JS integrator's brute-force iTriangle
    (raytracer.glsl:864-892, commented out in the reference: parity unpinned)
    against the C restatement's, two chained passes at 20x16."""
    import test_models as T
    cfg = [c for c in cfgs["configs"] if c["name"] == "c5_spectral_models"][0]
    v, own = T.world_soup(cfg, cfgs)
    tris = tmp_path / "c5.tris"
    O.write_tris(str(tris), v, own)
    n, w, h = 2, 20, 16
    J = js_restir_chain("c5_spectral_models", w, h, n, tmp_path, threads=8, extra=["--tris", str(tris)])
    o = O.Oracle(cfg, cfgs, width=w, height=h)
    o.set_triangles(v, own)
    S, M, A = o.frames_restir(n, cfg)
    for k in range(n):
        assert match(J[k, 0], S[k]) >= 0.99, (k + 1, "sample")
        assert res_match(J[k, 1], M[k]) >= 0.99, (k + 1, "reservoirs")
    # the model is in the picture: some pixels see it (hit index = the TRIANGLE entry)
    assert S[..., :3].mean() > 0 and abs(J[:, 0, ..., :3].mean() - S[..., :3].mean()) <= 2e-3 * S[..., :3].mean()



VIEWPORT_JS = os.path.join(REPO, "raytracer-0_amd", "js", "glsl_viewport.js")


def run_viewport_cpu(src, tmp_path):
    script = tmp_path / "page.js"
    script.write_text(src)
    r = subprocess.run([NODE, str(script)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_viewport_cpu_backend_renders_c1_like_the_page(cfgs, tmp_path):
    """BASELINE configs[0] through the product surface: GlslViewport with
    opts.backend = 'cpu' (the JS integrator, no GPU) driven the way the
    reference's page drives it -- the C1 constants set on `sandbox`, then
    RenderLoop's one render() per frame until max_passes (index.html:1218-1242
    -> index.js:986-1105) -- against the reference's own C1 fixture (the
    accumulated passes) and the C restatement."""
    gold = np.load(os.path.join(REPO, "tests", "golden", "c1_cornell_cos.npz"))["samples"]
    F, H, W = gold.shape[:3]
    out = tmp_path / "acc.f32"
    src = """
const fs = require('fs');
const v = require(%r);
const sandbox = new v.GlslViewport(null, {width: %d, height: %d, backend: 'cpu', max_passes: %d});
if (sandbox.backend !== 'cpu') throw new Error('backend ' + sandbox.backend);
sandbox.constants[0] = 'const lowp int MAX_BOUNCES = 4;';
sandbox.constants[7] = 'const bool sample_lights = false;';
sandbox.constants[8] = 'const bool use_mis = false;';
while (sandbox.passes < sandbox.max_passes) sandbox.render();   // RenderLoop
fs.writeFileSync(%r, Buffer.from(sandbox.accumulator().buffer));
const img = sandbox.image();
console.log(JSON.stringify({passes: sandbox.passes, px: img.length, ms: sandbox.lastKernelMs()}));
""" % (VIEWPORT_JS, W, H, F, str(out))
    info = json.loads(run_viewport_cpu(src, tmp_path).strip().splitlines()[-1])
    assert info["passes"] == F and info["px"] == W * H * 4
    got = np.fromfile(str(out), np.float32).reshape(H, W, 4)
    ref = np.zeros_like(gold[0])
    for k in range(F):
        ref[..., :3] = ref[..., :3] + gold[k][..., :3]
    assert match(got, ref) >= 0.99
    cfg = [c for c in cfgs["configs"] if c["name"] == "c1_cornell_cos"][0]
    o = O.Oracle(cfg, cfgs, width=W, height=H)
    oref = sum(o.frame(k)[0] for k in range(1, F + 1))
    assert match(got, oref) >= 0.999


def test_viewport_cpu_backend_scene_text_and_restir(cfgs, tmp_path):
    """The CPU backend parses the reference's GLSL-side state back (scene
    text from sceneFromLines, #sdf_meshes statements, define/constant lines):
    an SDF scene and a ReSTIR scene (index.js's swap chain) render what the
    JS integrator renders from the same config directly."""
    import rt0
    for name, n in (("sdf_cone", 2), ("c3_outdoor_restir", 3)):
        cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
        scene, sdf = rt0.scene_strings(cfg, cfgs)
        defines, consts = rt0.config_strings(cfg)
        cam = cfg.get("camera") or cfgs["default_camera"]
        out = tmp_path / ("%s.f32" % name)
        src = """
const fs = require('fs');
const v = require(%r);
const vp = new v.GlslViewport(null, {width: 32, height: 24, backend: 'cpu'});
vp.defines = %s; vp.constants = %s; vp.scene = %s; vp.sdf_meshes = %s;
const c = %s;
vp.camera.origin = new v.Vector3(...c.origin); vp.camera.lookat = new v.Vector3(...c.lookat);
vp.camera.fov = c.fov; vp.camera.aperture = c.aperture; vp.camera.focalLength = c.focalLength;
for (let k = 0; k < %d; k++) vp.render();
fs.writeFileSync(%r, Buffer.from(vp.accumulator().buffer));
""" % (VIEWPORT_JS, json.dumps(defines), json.dumps(consts), json.dumps(scene), json.dumps(sdf), json.dumps(cam),
       n, str(out))
        run_viewport_cpu(src, tmp_path)
        got = np.fromfile(str(out), np.float32).reshape(24, 32, 4)
        if name == "c3_outdoor_restir":
            ref = js_restir_chain(name, 32, 24, n, tmp_path)[:, 0].sum(0)
        else:
            ref = js_image(name, 32, 24, 1, n, tmp_path)
        assert np.array_equal(got[..., :3], ref[..., :3]), name


def test_viewport_backend_is_explicit(tmp_path):
    """No silent fallback: an unknown backend is refused, and the CPU backend
    refuses what only the HIP backend renders (textures, cubemap)."""
    src = """
const v = require(%r);
let msg = [];
try { new v.GlslViewport(null, {width: 8, height: 8, backend: 'webgl'}); } catch (e) { msg.push(e.message); }
const vp = new v.GlslViewport(null, {width: 8, height: 8, backend: 'cpu'});
try { vp.loadTexture({name: 'tex0'}, {width: 1, height: 1, data: new Uint8Array(4)}); } catch (e) { msg.push(e.message); }
try { vp.loadCubemap([1,2,3,4,5,6].map(() => ({width: 1, height: 1, data: new Uint8Array(3)}))); } catch (e) { msg.push(e.message); }
console.log(JSON.stringify(msg));
""" % VIEWPORT_JS
    msg = json.loads(run_viewport_cpu(src, tmp_path).strip().splitlines()[-1])
    assert len(msg) == 3 and "backend" in msg[0] and "outside the JS CPU integrator" in msg[1] + msg[2]
