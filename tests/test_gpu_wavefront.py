"""Wavefront rounds (rt0_set_wavefront; rt0_integrator.h wf_shade_body /
wf_march_body for SDF scenes, wf_restir_shade_body / wf_walk_body for ReSTIR
scenes with triangle models) against the pass kernel they replace, and their
own exact properties.

The march kernel runs every map() evaluation, bound test and calcNormal sum
of the pass kernel's march (the same arithmetic at one program point); the
light-sampling sums are formed one round later in call order, so FMA
placement differs at the last bit: compared at the parity tolerance.  Frame order of the accumulation, shards,
viewports and frame chunks are exact (bitwise).
"""
import os

import numpy as np
import pytest

import rt0
from test_gpu_parity import cfg_by_name, configure, have, pixel_match

pytestmark = pytest.mark.gpu

# SDF scenes of the parity set the wavefront path serves (quadric lights
# only): the Mandelbulb + medium (C4) at 3 and 12 bounces, MIS, textures,
# cubemap, Menger, prism, cone, the reference's default page scene
WF_SCENES = ["c4_mandelbulb_vol", "c4_mandelbulb_deep", "c4_mandelbulb_deep_novol", "mis_demo_sdfbox",
             "menger_coat", "tex_sdf_metal", "cube_sdf_metal", "sdf_triprism", "sdf_cone",
             "page_scene0_slabfirst"]


def render(cfgs, name, wf, w=64, h=64, frames=(1, 3), env=None, sample_lights=None, scratch=None):
    r = rt0.Renderer(w, h)
    configure(r, cfg_by_name(cfgs, name), cfgs)
    if sample_lights is not None:
        c = r.get_config()
        c.sample_lights = sample_lights
        r.set_config(c)
    r.set_wavefront(wf)
    r.render(*frames)
    if scratch is not None:
        scratch.append(r.samples_bytes())
    return r.read_accum(), r.last_render_path()


@pytest.mark.parametrize("name", WF_SCENES)
def test_wavefront_matches_pass_kernel(name, cfgs, gpu_required):
    a, pa = render(cfgs, name, True)
    b, pb = render(cfgs, name, False)
    assert pa == "wavefront" and pb == "pass", (pa, pb)
    assert np.isfinite(a).all()
    ok, _ = pixel_match(a[..., :3], b[..., :3])
    same = (a[..., :3] == b[..., :3]).all(-1)
    # ray-marched scenes amplify a last-bit difference into a different path
    # now and then (the parity tests' SDF allowance); most samples are equal
    assert ok.mean() >= 0.97, (name, ok.mean(), same.mean())
    # (bit-identical: 19-100% of pixels; the in-scatter and surface
    # light-sampling terms are rounded before the path adds them, where the
    # pass kernel fuses the last product into the add)
    assert abs(a[..., :3].mean() - b[..., :3].mean()) <= 0.01 * max(1.0, abs(b[..., :3].mean())), name


def test_wavefront_not_used_where_ineligible(cfgs, gpu_required):
    """An SDF light (direct_light's SDF branch), ReSTIR and quadric-only
    scenes keep their kernels."""
    for name, want in (("anim_mis_sdflight", "pass"), ("c2_cornell_mis_8", "pass"),
                       ("c3_outdoor_restir", "deferred")):
        _, p = render(cfgs, name, True, 32, 32, (1, 1))
        assert p == want, (name, p)


def test_wavefront_accumulation_exact(cfgs, gpu_required):
    """Several passes per launch run side by side as path slots; their samples
    are still added in pass order: 1..5 at once == 1..2 then 3..5 == five
    single-pass renders summed in order, bit for bit."""
    name = "c4_mandelbulb_vol"
    r = rt0.Renderer(48, 48)
    configure(r, cfg_by_name(cfgs, name), cfgs)
    singles = []
    for k in range(1, 6):
        r.clear()
        r.render(k, 1)
        singles.append(r.read_accum())
    ref = np.zeros_like(singles[0])
    for s in singles:
        ref[..., :3] = ref[..., :3] + s[..., :3]
    r.clear()
    r.render(1, 5)
    acc = r.read_accum()
    assert r.last_render_path() == "wavefront"
    assert np.array_equal(acc[..., :3], ref[..., :3])
    r.clear()
    r.render(1, 2)
    r.render(3, 3)
    assert np.array_equal(r.read_accum(), acc)


def test_wavefront_frame_chunks_exact(cfgs, gpu_required, monkeypatch):
    """A launch whose path slots exceed the device budget (RT0_WF_BYTES) runs
    its passes in frame chunks: the same bits as one chunk."""
    name = "c4_mandelbulb_deep"
    a, _ = render(cfgs, name, True, 64, 64, (1, 4))
    monkeypatch.setenv("RT0_WF_BYTES", str(64 * 64 * 400))  # ~1 frame per chunk
    b, _ = render(cfgs, name, True, 64, 64, (1, 4))
    assert np.array_equal(a, b)


def test_wavefront_slot_chunks_bound_memory(cfgs, gpu_required, monkeypatch):
    """A frame whose path slots exceed RT0_WF_BYTES (e.g. 4096^2 with 32
    lights) runs as chunks of whole regions within the frame instead of
    allocating the frame: the same bits, and the context's scratch stays
    within the budget (rt0_scratch_bytes counts the rounds' state)."""
    name = "c4_mandelbulb_deep"
    a, _ = render(cfgs, name, True, 96, 96, (1, 3))
    budget = 96 * 96 * 200 // 3  # about a third of one frame's slots
    monkeypatch.setenv("RT0_WF_BYTES", str(budget))
    sc = []
    b, p = render(cfgs, name, True, 96, 96, (1, 3), scratch=sc)
    assert p == "wavefront"
    assert np.array_equal(a, b)
    # state of K halves of a chunk + 3 frames of samples, nothing frame-sized besides
    assert sc[0] <= 2 * budget + 3 * 96 * 96 * 16, sc


def test_wavefront_state_released_on_pass_kernel(cfgs, gpu_required):
    """A context that leaves the wavefront path frees the rounds' state."""
    r = rt0.Renderer(64, 64)
    configure(r, cfg_by_name(cfgs, "sdf_cone"), cfgs)
    r.render(1, 2)
    with_wf = r.samples_bytes()
    r.set_wavefront(0)
    r.render(3, 1)
    assert r.last_render_path() == "pass"
    assert r.samples_bytes() < with_wf - 64 * 64 * 100, (with_wf, r.samples_bytes())


@pytest.mark.parametrize("name", ["c4_mandelbulb_deep_novol", "c4_mandelbulb_vol", "menger_coat", "sdf_cone",
                                  "mis_demo_sdfbox"])
def test_wavefront_bitwise_without_light_sampling(name, cfgs, gpu_required):
    """With sample_lights = 0 nothing is summed in another order (no NEE
    terms): every sample is the march answers (t, calcNormal's normal, the
    SDF id) fed through the same bounce code, so the wavefront image must
    equal the pass kernel's bit for bit -- the march kernel's map() steps,
    bound tests and normal probes are the pass kernel's."""
    a, pa = render(cfgs, name, True, sample_lights=0)
    b, pb = render(cfgs, name, False, sample_lights=0)
    assert pa == "wavefront" and pb == "pass", (pa, pb)
    assert np.isfinite(a).all() and a[..., :3].any()
    same = (a[..., :3] == b[..., :3]).all(-1)
    assert same.all(), (name, same.mean(), np.argwhere(~same)[:5].tolist())


def test_wavefront_shards_and_viewport_exact(cfgs, gpu_required):
    """Row-band shards and a viewport rectangle render exactly the whole
    image's pixels (slots map to pixels whatever the launch covers)."""
    name = "mis_demo_sdfbox"
    cfg = cfg_by_name(cfgs, name)
    W = H = 96
    whole, _ = render(cfgs, name, True, W, H, (1, 2))
    parts = np.zeros_like(whole)
    for s in range(3):
        r = rt0.Renderer(W, H)
        configure(r, cfg, cfgs)
        r.set_shard(s, 3, 16)
        r.render(1, 2)
        assert r.last_render_path() == "wavefront"
        p = r.read_accum()
        rows = np.array([(y // 16) % 3 == s for y in range(H)])
        assert not p[~rows].any()
        parts[rows] = p[rows]
    assert np.array_equal(parts, whole)
    r = rt0.Renderer(W, H)
    configure(r, cfg, cfgs)
    r.set_viewport(13, 21, 40, 33)
    r.render(1, 2)
    got = r.read_accum()
    inside = np.zeros((H, W), bool)
    inside[21:54, 13:53] = True
    assert np.array_equal(got[inside], whole[inside])
    assert not got[~inside].any()


@pytest.mark.parametrize("name", ["c4_mandelbulb_vol", "c4_mandelbulb_deep", "sdf_cone"])
def test_wavefront_matches_reference_fixture(name, cfgs, gpu_required):
    """The wavefront path against the reference's own images (the golden
    fixtures), at the GPU parity tolerances, per single-sample pass."""
    from test_gpu_parity import BAD_FRAC, GOLD
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    frames = G["frames"] if "frames" in G else range(1, gold.shape[0] + 1)
    valid = G["conformant"] if "conformant" in G else G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    r = rt0.Renderer(gold.shape[2], gold.shape[1])
    configure(r, cfg_by_name(cfgs, name), cfgs)
    got = []
    for k in frames:
        r.clear()
        r.render(int(k), 1)
        assert r.last_render_path() == "wavefront"
        got.append(r.read_accum()[..., :3])
    ok, _ = pixel_match(np.stack(got), gold)
    bad = 1.0 - ok[valid].mean()
    assert bad <= BAD_FRAC.get(name, BAD_FRAC["default"]), (name, bad)


def restir_chain(cfgs, wf, n=6, size=64, viewport=None, shard=None):
    import test_models as T
    cfg = T.cfg_by_name(cfgs, "c5_spectral_models")
    r = T.make(cfg, cfgs, size, size)
    r.set_wavefront(2 if wf else 0)  # (mode 2: ReSTIR scenes with models too)
    if viewport:
        r.set_viewport(*viewport)
    if shard:
        r.set_shard(*shard)
        r.set_halo(4)
    S, M, A = [], [], []
    for k in range(1, n + 1):
        r.render(k, 1)
        S.append(r.read_accum())
        m, a = r.read_restir(0)
        M.append(m)
        A.append(a)
    return np.stack(S), np.stack(M), np.stack(A), r.last_render_path()


def test_wavefront_restir_models_match_pass_kernel(cfgs, gpu_required):
    """ReSTIR with triangle models (BASELINE config 5 at 64x64): the pass's
    paths as shade rounds + closest-hit walk rounds against the deferred pass
    kernel, over a 6-pass chain (each pass reads the reservoirs the previous
    ones wrote).  Every walk is bvh_closest's and the quadric tests are
    recomputed on resume: the same hits, the same deferred calls; only the
    compiler's FMA contraction can differ between the two kernels -- held to
    test_gpu_defer's bar (1e-5 / 1e-4 relative, >= 98% bit-identical)."""
    from test_gpu_defer import close_and_mostly_identical
    s1, m1, a1, p1 = restir_chain(cfgs, True)
    s0, m0, a0, p0 = restir_chain(cfgs, False)
    assert p1 == "wavefront" and p0 == "deferred", (p1, p0)
    assert np.isfinite(s1).all()
    print("bit-identical samples %.4f reservoirs %.4f" % ((s0[..., :3] == s1[..., :3]).all(-1).mean(),
                                                          (m0 == m1).all(-1).mean()))
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(a0, a1, "reservoir aux")
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    assert s1[..., :3].mean() > 0.0


def test_wavefront_restir_models_viewport_and_shards(cfgs, gpu_required):
    """A tile and a contiguous row-block shard of the model scene through the
    wavefront rounds: only their pixels are drawn, and they match the
    deferred pass kernel's render of the same tile / shard (slots map to
    pass waves whatever the launch covers)."""
    from test_gpu_defer import close_and_mostly_identical
    vp = (8, 16, 40, 24)
    s1, m1, _, p1 = restir_chain(cfgs, True, n=3, viewport=vp)
    s0, m0, _, _ = restir_chain(cfgs, False, n=3, viewport=vp)
    assert p1 == "wavefront"
    inside = np.zeros(s1.shape[1:3], bool)
    inside[vp[1]:vp[1] + vp[3], vp[0]:vp[0] + vp[2]] = True
    assert not s1[:, ~inside, :3].any()
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    # one pass per call of a sharded ReSTIR render: shard 1 of 2 (rows 32..63)
    s1, m1, _, p1 = restir_chain(cfgs, True, n=1, shard=(1, 2, 32))
    s0, m0, _, _ = restir_chain(cfgs, False, n=1, shard=(1, 2, 32))
    assert p1 == "wavefront"
    assert not s1[0][:32, :, :3].any() and s1[0][32:, :, :3].any()
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
