"""Wavefront SDF rounds (rt0_set_wavefront; rt0_integrator.h wf_shade_body /
wf_march_body) against the pass kernel they replace, and their own exact
properties.

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


def render(cfgs, name, wf, w=64, h=64, frames=(1, 3), env=None):
    r = rt0.Renderer(w, h)
    configure(r, cfg_by_name(cfgs, name), cfgs)
    r.set_wavefront(wf)
    r.render(*frames)
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
