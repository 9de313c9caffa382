"""Parity of the HIP path (librt0.so through the C ABI) with the reference.

* against the golden fixtures (the reference shader run by SwiftShader):
  every config, single-sample passes 1..F, same tolerance as the oracle;
* ReSTIR: conditional parity -- the reference's own reservoir buffers of passes
  k-1..k-3 are uploaded through rt0_write_restir_inputs, pass k's radiance
  must match -- and the product's own unconditional 6-pass chain against the
  reference's (rt0_set_executor_compat: the executor's reservoir stores);
* against the CPU restatement at sizes the fixtures do not cover (128^2 bench
  scene, 12-bounce volumetric C4 scene).
All calls go through include/rt0.h; nothing here can fall back to the CPU.
"""
import os

import numpy as np
import pytest

import oracle as O
import rt0
from textures import cubemap_for, textures_for

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REL_TOL = 1e-3
# fraction of pixels allowed to differ (discrete flips from ulp-level
# differences between gfx950 transcendentals and the reference executor's, and
# from FMA contraction outside the RNG; ray-marched SDF scenes amplify them)
BAD_FRAC = {"default": 0.01, "c4_mandelbulb_vol": 0.03, "spectral_vol_1l": 0.03, "menger_coat": 0.03,
            # C4 at 12 bounces: compared on the lanes whose executor path
            # record equals GLSL semantics (the fixture's `conformant` mask,
            # oracle/gen/make_golden.py instrument_paths)
            "c4_mandelbulb_deep": 0.03, "c4_mandelbulb_deep_novol": 0.03,
            "mis_demo_sdfbox": 0.02, "restir_mis_demo": 0.02, "c3_outdoor_restir": 0.01,
            # glossy METAL reflections grazing the slab's front edge: the SDF
            # marches' decisions and calcNormal's normal, chaotic under
            # ulp-level changes (each departing pixel's first divergent event:
            # test_oracle_golden.test_metal_departures_attributed)
            "tex_sdf_metal": 0.05, "cube_sdf_metal": 0.08,
            # the reference's own assets (real rgba_noise256.png, tex0-3.png,
            # Tropical Beach cubemap) with the executor's texture filter (the
            # default, rt0_set_texture_filter): tests/test_oracle_golden.py BAD_FRAC
            "page_scene0_slabfirst": 0.07, "page_scene1": 0.01, "tex_check_assets": 0.002}
# mean radiance vs the fixture (default 5e-3); cube_sdf_metal: SwiftShader's
# image of this SDF-only scene depends on the order of its SDF statements
# (tests/test_oracle_golden.py MEAN_TOL)
MEAN_TOL = {"cube_sdf_metal": 0.025,
            # 8x8 per-frame volumetric fixtures: one flip onto the light moves the mean by up to 0.03
            "c4_mandelbulb_vol": 0.1, "vol_cornell_2": 0.02, "spectral_vol_1l": 0.05,
            "c4_mandelbulb_deep": 0.01, "c4_mandelbulb_deep_novol": 0.01}


def cfg_by_name(cfgs, name):
    return [c for c in cfgs["configs"] if c["name"] == name][0]


def pixel_match(got, ref):
    nan = np.isnan(ref).any(-1)
    d = np.abs(got - ref)
    ok = (d <= REL_TOL * np.maximum(1.0, np.abs(ref))).all(-1) | nan
    return ok, nan


def configure(r, cfg, cfgs):
    """rt0.configure + the config's asset textures (oracle/textures.py stand-ins)."""
    rt0.configure(r, cfg, cfgs)
    for unit, img in textures_for(cfg).items():
        r.set_texture(unit, img)
    faces = cubemap_for(cfg)
    if faces is not None:
        r.set_cubemap(faces)


def make(cfgs, name, w, h):
    r = rt0.Renderer(w, h)
    configure(r, cfg_by_name(cfgs, name), cfgs)
    return r


def single(r, k):
    r.clear()
    r.render(k, 1)
    return r.read_accum()


def have(name):
    return os.path.exists(os.path.join(GOLD, name + ".npz"))


NON_RESTIR = ["c1_cornell_cos", "c2_cornell_mis_refcaps", "c2_cornell_mis_8", "cornell_nee_plain",
              "mis_demo_sdfbox", "menger_coat", "thinlens_glass", "c4_mandelbulb_vol", "spectral_vol_1l",
              "tex_sdf_metal", "tex_light_sphere", "tex_check_test", "cube_spheres", "cube_sdf_metal",
              "sdf_triprism", "sdf_cone", "spectral_cornell", "vol_cornell_2",
              "page_scene0_slabfirst", "tex_check_assets", "page_scene1", "cube_spheres_assets",
              "c4_mandelbulb_deep", "c4_mandelbulb_deep_novol"]


@pytest.mark.parametrize("name", NON_RESTIR)
def test_gpu_matches_reference_fixture(name, cfgs, gpu_required):
    if not have(name):
        pytest.skip("fixture not generated")
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"]
    F, H, W = gold.shape[:3]
    # u_frame of each pass (per-frame fixtures skip passes the executor did not finish)
    frames = G["frames"] if "frames" in G else range(1, F + 1)
    r = make(cfgs, name, W, H)
    got = np.stack([single(r, int(k)) for k in frames])
    # tiled fixtures: the pixels whose tile the executor finished, stable
    # under two thread counts (oracle/gen/make_golden.py run_tiled); with path
    # records, those whose bounce loop ran as GLSL says (`conformant`)
    valid = G["conformant"] if "conformant" in G else G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    ok, nan = pixel_match(got[..., :3], gold[..., :3])
    bad = 1.0 - ok[valid].mean()
    assert bad <= BAD_FRAC.get(name, BAD_FRAC["default"]), "%s: %.4f of pixels differ" % (name, bad)
    assert not np.isnan(got).any()
    m = ~nan & valid
    g, s = gold[..., :3][m], got[..., :3][m]
    assert abs(s.mean() - g.mean()) <= MEAN_TOL.get(name, 5e-3) * max(1.0, abs(g.mean()))


@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "c5_spectral_sphere"])
def test_gpu_restir_conditional_parity(name, cfgs, gpu_required):
    if not have(name):
        pytest.skip("fixture not generated")
    G = np.load(os.path.join(GOLD, name + ".npz"))
    F, H, W = G["samples"].shape[:3]
    r = make(cfgs, name, W, H)

    def out(k, key):
        return G[key][k - 1] if k >= 1 else None

    for k in range(1, F + 1):
        r.clear()
        r.write_restir_inputs(out(k - 1, "restir_main"), out(k - 1, "restir_aux"), out(k - 2, "restir_main"),
                              out(k - 2, "restir_aux"), out(k - 3, "restir_main"), out(k - 3, "restir_aux"))
        r.render(k, 1)
        ok, _ = pixel_match(r.read_accum()[..., :3], G["samples"][k - 1][..., :3])
        assert 1.0 - ok.mean() <= BAD_FRAC.get(name, BAD_FRAC["default"]), (name, k, 1.0 - ok.mean())


# SURVEY 8c on the unconditional chain: per pass <= 1% of pixels outside the
# tolerance (discrete flips: a shadow ray grazing an edge under gfx950's
# transcendentals); relative L2 of the mean over the passes <= 1e-3 on the
# pixels that match in every pass, and <= 5e-3 including the flips (one
# flipped light pixel of 4096 at pass 1 -- the same in the conditional test,
# which uploads the reference's reservoirs -- gives 2.6e-3 on c3).  The nearly
# black restir_mis_demo (mean radiance 6e-5, where a few ulp-level flips of
# ~1e-4 dominate any relative norm) bounds the RMS of that mean instead.
CHAIN_REL_L2 = {"c3_outdoor_restir": 1e-3, "anim_restir_demo": 1e-3, "c5_spectral_sphere": 1e-3}


def chain_l2_ok(name, got, gold, ok_all):
    m, g = got.mean(0), gold.mean(0)
    if name not in CHAIN_REL_L2:
        return np.sqrt(np.mean((m - g) ** 2)) <= 1e-3, "rms"
    st = ok_all[..., None]
    stable = np.linalg.norm((m - g) * st) / max(np.linalg.norm(g * st), 1e-30)
    full = np.linalg.norm(m - g) / np.linalg.norm(g)
    return stable <= CHAIN_REL_L2[name] and full <= 5e-3, (stable, full)


@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "anim_restir_demo", "c5_spectral_sphere"])
def test_gpu_restir_chain_matches_reference(name, cfgs, gpu_required):
    """The product's own multi-pass ReSTIR (its swap chain of index.js:795-820,
    nothing uploaded) against the reference's chained passes, with the
    reservoir stores of the reference executor (rt0_set_executor_compat)."""
    if not have(name):
        pytest.skip("fixture not generated")
    cfg = cfg_by_name(cfgs, name)
    G = np.load(os.path.join(GOLD, name + ".npz"))
    F, H, W = G["samples"].shape[:3]
    r = make(cfgs, name, W, H)
    r.set_executor_compat(True)
    r.set_temporal_frames(cfg.get("temporal_frames", 5))
    zero = np.zeros((H, W, 4), np.float32)
    got = []
    ok_all = np.ones((H, W), bool)
    for k in range(1, F + 1):
        r.write_accum(zero)  # single-sample pass (u_bufferA = 0), reservoirs chain on
        r.render(k, 1, O.pass_time(cfg, k) if cfg.get("time_ms") else 0.0)
        s = r.read_accum()
        got.append(s)
        ok, _ = pixel_match(s[..., :3], G["samples"][k - 1][..., :3])
        ok_all &= ok
        assert 1.0 - ok.mean() <= 0.01, (name, k, 1.0 - ok.mean())
        m, a = r.read_restir(0)
        okr = pixel_match(m, G["restir_main"][k - 1])[0] & pixel_match(a, G["restir_aux"][k - 1])[0]
        assert 1.0 - okr.mean() <= 0.01, (name, k, "reservoirs", 1.0 - okr.mean())
    good, l2 = chain_l2_ok(name, np.stack(got)[..., :3], G["samples"][..., :3], ok_all)
    assert good, (name, l2)


@pytest.mark.parametrize("name", ["page_scene0_slabfirst", "page_scene1", "tex_check_assets", "tex_check_test"])
def test_gpu_texture_filter_fixed_vs_float(name, cfgs, gpu_required):
    """The asset textures through the executor's fixed-point bilinear filter
    (rt0_integrator.h tex_rgba8_ss, pinned by tests/golden/tex_filter_kat.npz;
    the default, rt0_set_texture_filter) hold the restatement's bounds against
    the reference's own fixtures (test_oracle_golden.TEX_FILTER_BAD); exact
    fp32 bilinear (TEX_FILTER_FLOAT) is measurably worse."""
    from test_oracle_golden import TEX_FILTER_BAD
    if not have(name):
        pytest.skip("fixture not generated")
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"]
    frames = G["frames"] if "frames" in G else range(1, gold.shape[0] + 1)
    valid = G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    bad = []
    for mode in (rt0.TEX_FILTER_FIXED16, rt0.TEX_FILTER_FLOAT):
        r = make(cfgs, name, gold.shape[2], gold.shape[1])
        r.set_texture_filter(mode)
        got = np.stack([single(r, int(k)) for k in frames])
        ok, _ = pixel_match(got[..., :3], gold[..., :3])
        bad.append(1.0 - ok[valid].mean())
    print("%s: %.4f of pixels differ (fixed-point filter), %.4f (fp32)" % (name, bad[0], bad[1]))
    fixed_bound, float_worse = TEX_FILTER_BAD[name]
    assert bad[0] <= max(fixed_bound, BAD_FRAC.get(name, 0.0)), (name, bad)
    assert bad[1] - bad[0] >= 0.5 * float_worse, (name, bad)


def test_gpu_page_scene0(cfgs, gpu_required):
    """The reference page's default scene (index.html:752-790) end to end on
    its real assets.  GLSL semantics make the order of its two SDF statements
    matter only at the ulp level (map()'s mix() rounds differently; under the
    high-frequency cubemap and METAL glossiness that moves ~10% of pixels in
    the restatement too, with the same mean); the reference executor's image
    depends on it for real (oracle/gen/mask_kat.py rule 7: 5% mean shift).  So
    the product's page-order render must agree in mean with its slab-first
    render and with the reference's slab-first fixture (the per-pixel test of
    that fixture is test_gpu_matches_reference_fixture)."""
    if not (have("page_scene0") and have("page_scene0_slabfirst")):
        pytest.skip("fixture not generated")
    a = make(cfgs, "page_scene0", 64, 64)
    b = make(cfgs, "page_scene0_slabfirst", 64, 64)
    ia = np.stack([single(a, k) for k in (1, 2, 3, 4)])[..., :3]
    ib = np.stack([single(b, k) for k in (1, 2, 3, 4)])[..., :3]
    ok, _ = pixel_match(ia, ib)
    assert ok.mean() >= 0.85, ok.mean()
    assert abs(ia.mean() - ib.mean()) <= 2e-3 * max(1.0, ib.mean())
    g = np.load(os.path.join(GOLD, "page_scene0_slabfirst.npz"))["samples"][..., :3]
    assert abs(ia.mean() - g.mean()) <= 5e-3 * max(1.0, g.mean())


def test_gpu_restir_chain_matches_oracle_chain(cfgs, gpu_required):
    """GLSL semantics (executor compat off, the default): the product's
    unconditional chain against the restatement's, both without the executor
    artefact."""
    name = "c3_outdoor_restir"
    cfg = cfg_by_name(cfgs, name)
    o = O.Oracle(cfg, cfgs, width=64, height=64)
    s_ref, m_ref, a_ref = o.frames_restir(4)
    r = make(cfgs, name, 64, 64)
    zero = np.zeros((64, 64, 4), np.float32)
    for k in range(1, 5):
        r.write_accum(zero)
        r.render(k, 1)
        ok, _ = pixel_match(r.read_accum()[..., :3], s_ref[k - 1][..., :3])
        assert 1.0 - ok.mean() <= 0.03, (k, 1.0 - ok.mean())
        m, a = r.read_restir(0)
        okm, _ = pixel_match(m, m_ref[k - 1])
        assert okm.mean() >= 0.95, (k, okm.mean())


@pytest.mark.parametrize("name,size,frames", [("c2_cornell_mis_8", 128, 2), ("cornell_nee_plain", 96, 1),
                                              ("c4_mandelbulb_vol", 48, 1), ("tex_check_test", 96, 2),
                                              ("tex_light_sphere", 96, 1), ("cube_spheres", 96, 2),
                                              ("spectral_vol", 64, 2), ("c2_cornell_mis_8", (120, 68), 2),
                                              ("c3_outdoor_restir", (150, 83), 1)])
def test_gpu_matches_oracle_beyond_fixtures(name, size, frames, cfgs, gpu_required):
    """Sizes beyond the fixtures' 8x8 / 64x64, against the restatement.  The
    non-power-of-two and non-square cases pin the camera: the kernel scales
    the tent-filter offset by a per-launch 1/(res/2) where raytracer.glsl:2138
    (and the restatement) divide -- equal for power-of-two sizes, an ulp apart
    otherwise (deviations)."""
    cfg = cfg_by_name(cfgs, name)
    over = {"MAX_BOUNCES": 12} if name == "c4_mandelbulb_vol" else {}
    w, h = size if isinstance(size, tuple) else (size, size)
    o = O.Oracle(cfg, cfgs, width=w, height=h, overrides=over)
    r = rt0.Renderer(w, h)
    cfg2 = dict(cfg)
    cfg2["constants"] = dict(cfg["constants"], **over)
    configure(r, cfg2, cfgs)
    for k in range(1, frames + 1):
        ref = o.frame(k)[0]
        got = single(r, k)
        ok, _ = pixel_match(got[..., :3], ref[..., :3])
        assert 1.0 - ok.mean() <= 0.02, (name, k, 1.0 - ok.mean())


def test_gpu_accumulation_is_sequential_sum(cfgs, gpu_required):
    """In-kernel multi-pass accumulation == the reference's per-pass
    `prev + sample` chain (raytracer.glsl:2168), bit for bit."""
    r = make(cfgs, "c2_cornell_mis_8", 64, 64)
    samples = [single(r, k) for k in range(1, 6)]
    ref = np.zeros_like(samples[0])
    for s in samples:
        ref[..., :3] = ref[..., :3] + s[..., :3]
    r.clear()
    r.render(1, 5)
    acc = r.read_accum()
    assert np.array_equal(acc[..., :3], ref[..., :3])
    # resumable: passes 1..2 then 3..5 == 1..5
    r.clear()
    r.render(1, 2)
    r.render(3, 3)
    assert np.array_equal(r.read_accum(), acc)


@pytest.mark.parametrize("name", ["c2_cornell_mis_8", "c3_outdoor_restir", "spectral_vol", "mis_demo_sdfbox",
                                  "tex_check_test", "tex_sdf_metal", "cube_spheres"])
def test_jit_matches_aot(name, cfgs, gpu_required):
    """Scene-specialised kernels == ahead-of-time kernels (same arithmetic up
    to FMA placement, so compare with the parity tolerance)."""
    cfg = cfg_by_name(cfgs, name)
    out = []
    for jit in (True, False):
        r = rt0.Renderer(64, 64)
        r.set_jit(jit)
        configure(r, cfg, cfgs)
        r.render(1, 2)
        out.append(r.read_accum())
    ok, _ = pixel_match(out[0][..., :3], out[1][..., :3])
    assert ok.mean() >= 0.97, ok.mean()


@pytest.mark.parametrize("name", ["spectral_vol_2l", "spectral_2l_novol"])
def test_gpu_two_light_quad_first_lanes(name, cfgs, gpu_required):
    """Two lights: the executor reads brdf's light_index[i] at the 2x2 quad's
    first lane's index (tests/test_oracle_golden.py QUAD_LIGHTS); the product
    computes GLSL semantics, so it is held to the reference on the first lanes
    at the default bound and to GLSL semantics (the restatement) on all."""
    if not have(name):
        pytest.skip("fixture not generated")
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    F, H, W = gold.shape[:3]
    frames = G["frames"] if "frames" in G else range(1, F + 1)
    r = make(cfgs, name, W, H)
    got = np.stack([single(r, int(k)) for k in frames])[..., :3]
    valid = G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    ok, _ = pixel_match(got, gold)
    # the medium's discrete flips on 16x16 fixtures: spectral_vol_1l's bound
    bound = BAD_FRAC["spectral_vol_1l"] if "vol" in name else BAD_FRAC["default"]
    first = valid[:, 0::2, 0::2]
    assert 1.0 - ok[:, 0::2, 0::2][first].mean() <= bound
    o = O.Oracle(cfg_by_name(cfgs, name), cfgs, width=W, height=H)
    want = np.stack([o.frame(int(k))[0] for k in frames])[..., :3]
    ok, _ = pixel_match(got, want)
    assert 1.0 - ok.mean() <= bound


@pytest.mark.parametrize("name,bound", [("spectral_2l_novol", 0.01), ("spectral_vol_2l", 0.04)])
def test_gpu_two_light_executor_quad_lights(name, bound, cfgs, gpu_required):
    """Rule 11 in the product (rt0_set_executor_compat; Integrator::light_q):
    each frame is a recording launch (every pixel's light-loop bounces) and
    the frame proper, whose lanes read brdf's light_index[i] as the reference
    executor does, at their 2x2 quad's first lane's index.  Against the
    reference on ALL lanes (first lanes and the other three), and against the
    restatement's model of the same rule (SWIFTSHADER_QUAD_LIGHTS)."""
    if not have(name):
        pytest.skip("fixture not generated")
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    F, H, W = gold.shape[:3]
    frames = G["frames"] if "frames" in G else range(1, F + 1)
    r = make(cfgs, name, W, H)
    r.set_executor_compat(True)
    got = np.stack([single(r, int(k)) for k in frames])[..., :3]
    assert r.last_render_path() == "pass"
    valid = G["conformant"] if "conformant" in G else G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    ok, _ = pixel_match(got, gold)
    bad = 1.0 - ok[valid].mean()
    per_lane = [1.0 - ok[:, ly::2, lx::2][valid[:, ly::2, lx::2]].mean() for ly in (0, 1) for lx in (0, 1)]
    print("%s: %.4f of valid samples differ under compat; per quad lane %s" % (name, bad, per_lane))
    assert bad <= bound, (name, bad, per_lane)
    o = O.Oracle(cfg_by_name(cfgs, name), cfgs, width=W, height=H,
                 overrides={"SWIFTSHADER_GHOST": 1, "SWIFTSHADER_QUAD_LIGHTS": 1})
    want = np.stack([o.frame(int(k))[0] for k in frames])[..., :3]
    ok, _ = pixel_match(got, want)
    assert 1.0 - ok.mean() <= bound, (name, 1.0 - ok.mean())
    # without compat: GLSL semantics, the non-first lanes depart
    r.set_executor_compat(False)
    plain = np.stack([single(r, int(k)) for k in frames])[..., :3]
    okp, _ = pixel_match(plain, gold)
    assert 1.0 - okp[valid].mean() > bad


def test_gpu_quad_lights_tile_and_resume(cfgs, gpu_required):
    """Rule 11's recording launch covers whole 2x2 quads of a tile whose
    corner is odd, and a multi-pass call equals its passes one by one."""
    name = "spectral_2l_novol"
    cfg = cfg_by_name(cfgs, name)
    full = make(cfgs, name, 32, 32)
    full.set_executor_compat(True)
    full.render(1, 3)
    ref = full.read_accum()
    one = make(cfgs, name, 32, 32)
    one.set_executor_compat(True)
    for k in (1, 2, 3):
        one.render(k, 1)
    assert np.array_equal(one.read_accum(), ref)
    t = make(cfgs, name, 32, 32)
    t.set_executor_compat(True)
    t.set_viewport(5, 7, 20, 14)
    t.render(1, 3)
    got = t.read_accum()
    assert np.array_equal(got[7:21, 5:25], ref[7:21, 5:25])
    assert cfg["name"] == name
