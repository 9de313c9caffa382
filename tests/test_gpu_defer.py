"""Deferred ReSTIR light sampling (rt0_integrator.h pool of NeeRec regions,
rt0_jit_nee, rt0_jit_resolve) against the inline calls.

Every sampleLightsReSTIR call runs with the same arguments and the same
source in the deferred kernels as inline.  What can differ is FMA placement
(the compiler contracts a product into an add only when the product has one
use, which depends on the surrounding kernel) and the order of a sample's
final additions (the path's own radiance first, then the light-sampling
results in call order, instead of interleaved).  Measured on the GPU: 98.7-
99.7% of samples bit-identical, the rest within 4.8e-7; reservoir MRTs
(g_final_reservoir, raytracer.glsl:2171-2174) identical except 0-56 of 4096
pixels per pass, by <= 1.5e-5 relative.  The test holds them to that: every
reservoir within 1e-4 and every sample within 1e-5 relative (the parity
tolerance is 1e-3), >= 98% of each bit-identical.
rt0_set_defer_light_sampling switches between the two per context.
"""
import os

import numpy as np
import pytest

import rt0
from test_gpu_parity import cfg_by_name, configure, have

import oracle as O


def chain(cfgs, name, defer, n=6, size=64, viewport=None):
    r = rt0.Renderer(size, size)
    r.set_defer_light_sampling(defer == "1")
    cfg = cfg_by_name(cfgs, name)
    configure(r, cfg, cfgs)
    r.set_temporal_frames(cfg.get("temporal_frames", 5))
    if viewport:
        r.set_viewport(*viewport)
    S, M, A = [], [], []
    for k in range(1, n + 1):
        r.render(k, 1, O.pass_time(cfg, k) if cfg.get("time_ms") else 0.0)
        S.append(r.read_accum())
        m, a = r.read_restir(0)
        M.append(m)
        A.append(a)
    return np.stack(S), np.stack(M), np.stack(A)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "c5_spectral_sphere", "anim_restir_demo"])
def test_deferred_matches_inline(name, cfgs, gpu_required):
    if not have(name):
        pytest.skip("fixture not generated")
    s0, m0, a0 = chain(cfgs, name, "0")
    s1, m1, a1 = chain(cfgs, name, "1")
    if os.environ.get("RT0_TEST_DUMP"):
        np.savez_compressed(os.path.join(os.environ["RT0_TEST_DUMP"], name + "_defer.npz"),
                            s0=s0, m0=m0, a0=a0, s1=s1, m1=m1, a1=a1)
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(a0, a1, "reservoir aux")
    assert np.isfinite(s1).all()
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    assert s1[..., :3].mean() > 0.0


def close_and_mostly_identical(x, y, what, rel=None):
    rel = rel or (1e-5 if what == "samples" else 1e-4)
    d = np.abs(x - y)
    assert (d <= rel * np.maximum(1.0, np.abs(x))).all(), (what, float(d.max()))
    same = (x == y).all(-1).mean()
    assert same >= 0.98, (what, same)


@pytest.mark.gpu
def test_deferred_viewport_matches_inline(cfgs, gpu_required):
    """A tile (gl.viewport rectangle, index.js:761-792) with deferral: only
    the rectangle's pixels get records, and they resolve like the inline
    render of the same rectangle."""
    vp = (8, 16, 40, 24)
    s0, m0, a0 = chain(cfgs, "c3_outdoor_restir", "0", n=3, viewport=vp)
    s1, m1, a1 = chain(cfgs, "c3_outdoor_restir", "1", n=3, viewport=vp)
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(a0, a1, "reservoir aux")
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    outside = np.ones(s1.shape[1:3], bool)
    outside[vp[1]:vp[1] + vp[3], vp[0]:vp[0] + vp[2]] = False
    assert not s1[:, outside, :3].any()


@pytest.mark.gpu
def test_deferred_walks_match_inline_models(cfgs, gpu_required):
    """A scene with triangle models (BASELINE config 5 at 64x64: 10 sphere
    lights, the 81,920-triangle model): deferred light sampling hands each
    call's two triangle occlusion queries (the visibility ray and the picked
    light's shadow ray) to rt0_jit_walk, whose lanes take the next query as
    soon as theirs is answered, and rt0_jit_resolve completes the calls
    through the tagged result entries (rt0_integrator.h restir_split,
    walk_body, resolve_body).  Against the
    inline calls of the same 6-pass chain: same answers, so the same
    tolerance as above."""
    import test_models as T
    cfg = T.cfg_by_name(cfgs, "c5_spectral_models")
    out = []
    for defer in (False, True):
        r = T.make(cfg, cfgs, 64, 64)
        r.set_defer_light_sampling(defer)
        S, M, A = [], [], []
        for k in range(1, 7):
            r.render(k, 1)
            S.append(r.read_accum())
            m, a = r.read_restir(0)
            M.append(m)
            A.append(a)
        out.append((np.stack(S), np.stack(M), np.stack(A)))
    (s0, m0, a0), (s1, m1, a1) = out
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(a0, a1, "reservoir aux")
    assert np.isfinite(s1).all()
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    # some calls were answered by the walks: the model occludes lights
    assert (m1[..., 3] == 0).any() and (m1[..., 3] > 0).any()


@pytest.mark.gpu
def test_deferred_walks_viewport_models(cfgs, gpu_required):
    """The walk path on a tile (gl.viewport rectangle) of the model scene:
    only the rectangle's calls queue walks, and they resolve like the inline
    render of the same rectangle."""
    import test_models as T
    cfg = T.cfg_by_name(cfgs, "c5_spectral_models")
    vp = (8, 16, 40, 24)
    out = []
    for defer in (False, True):
        r = T.make(cfg, cfgs, 64, 64)
        r.set_defer_light_sampling(defer)
        r.set_viewport(*vp)
        S, M = [], []
        for k in range(1, 4):
            r.render(k, 1)
            S.append(r.read_accum())
            M.append(r.read_restir(0)[0])
        out.append((np.stack(S), np.stack(M)))
    (s0, m0), (s1, m1) = out
    close_and_mostly_identical(m0, m1, "reservoir main")
    close_and_mostly_identical(s0[..., :3], s1[..., :3], "samples")
    outside = np.ones(s1.shape[1:3], bool)
    outside[vp[1]:vp[1] + vp[3], vp[0]:vp[0] + vp[2]] = False
    assert not s1[:, outside, :3].any()


@pytest.mark.gpu
def test_deferred_buffers_follow_bounce_count(cfgs, gpu_required):
    """One context renders the whole image at MAX_BOUNCES 2, then a 16x16
    tile at MAX_BOUNCES 12: fewer record slots but more result planes (one
    per call index, nee_out).  The tile must equal a fresh context's render
    of it -- the buffers are re-sized for the plane count, not only for the
    slot count (an out-of-bounds write before)."""
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    vp = (24, 24, 16, 16)

    def bounces(r, n):
        c = r.get_config()
        c.max_bounces = n
        r.set_config(c)

    r = rt0.Renderer(64, 64)
    configure(r, cfg, cfgs)
    bounces(r, 2)
    r.render(1, 1)
    bounces(r, 12)
    r.set_viewport(*vp)
    r.clear()
    for k in (1, 2):
        r.render(k, 1)
    got = r.read_accum()
    f = rt0.Renderer(64, 64)
    configure(f, cfg, cfgs)
    bounces(f, 12)
    f.set_viewport(*vp)
    for k in (1, 2):
        f.render(k, 1)
    want = f.read_accum()
    assert np.isfinite(got).all()
    assert np.array_equal(got, want)
    assert got[vp[1]:vp[1] + 16, vp[0]:vp[0] + 16, :3].any()


@pytest.mark.gpu
def test_deferral_off_beyond_packed_call_index(cfgs, gpu_required):
    """NeeRec packs a call's index along its path in 8 bits (rt0_device.h):
    with MAX_BOUNCES above RT0_NEE_MAX_BOUNCES (255) the host keeps the inline
    calls, so asking for deferral renders the same bits as not asking."""
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    out = []
    for defer in (True, False):
        r = rt0.Renderer(32, 32)
        configure(r, cfg, cfgs)
        c = r.get_config()
        c.max_bounces = 300
        r.set_config(c)
        r.set_defer_light_sampling(defer)
        for k in (1, 2):
            r.render(k, 1)
        out.append(r.read_accum())
    assert np.isfinite(out[0]).all()
    assert np.array_equal(out[0], out[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name,size,viewport", [("c5_spectral_models", (64, 80), None),
                                                ("c3_outdoor_restir", (64, 48), None),
                                                ("c3_outdoor_restir", (64, 64), (8, 5, 40, 50))])
def test_split_pass_is_bit_identical(name, size, viewport, cfgs, monkeypatch, gpu_required):
    """A deferred ReSTIR pass as two row halves on two streams
    (rt0_host.cpp restir_split_pass; default for scenes with models) gives
    the unsplit pass's samples and reservoirs bit for bit: the halves only
    change which wave holds a record.  An odd number of 16-row tile rows, and
    a viewport whose rows are not a multiple of 16."""
    import test_models as T
    cfg = T.cfg_by_name(cfgs, name)
    out = []
    for split in ("0", "1", "3"):
        monkeypatch.setenv("RT0_RESTIR_SPLIT", split)
        if name == "c3_outdoor_restir":
            r = rt0.Renderer(*size)
            configure(r, cfg, cfgs)
        else:
            r = T.make(cfg, cfgs, *size)
        if viewport:
            r.set_viewport(*viewport)
        S, M, A = [], [], []
        for k in range(1, 5):
            r.render(k, 1)
            S.append(r.read_accum())
            m, a = r.read_restir(0)
            M.append(m)
            A.append(a)
        out.append((np.stack(S), np.stack(M), np.stack(A)))
        r.close()
    for o in out[1:]:
        for x, y in zip(out[0], o):
            assert np.array_equal(x, y)
    assert out[1][0][..., :3].mean() > 0.0


@pytest.mark.gpu
def test_split_then_unsplit_on_one_context(cfgs, monkeypatch, gpu_required):
    """One context renders split passes (4 row parts: the walk buffers padded
    for the parts' rounded wave counts), is resized smaller, renders unsplit
    passes, then a 16-row tile (grid.y == 1, never split).  The unsplit walk launch rounds its wave
    count up to whole workgroups; its padding waves must stop at the exact
    light-sampling wave count and not walk the counts an earlier split pass
    left in the padded entries.  Each stage equals a fresh context's render."""
    import test_models as T
    cfg = T.cfg_by_name(cfgs, "c5_spectral_models")
    vp = (0, 24, 80, 16)

    def run(r, split, frames, viewport=None):
        monkeypatch.setenv("RT0_RESTIR_SPLIT", split)
        if viewport:
            r.set_viewport(*viewport)
            r.clear()
        for k in frames:
            r.render(k, 1)
        return r.read_accum(), r.read_restir(0)[0]

    # 80x96: 60 light-sampling waves, all walk counts written by the split
    # passes; 80x80 then has 50, and its unsplit walk launch 52 waves
    r = T.make(cfg, cfgs, 80, 96)
    run(r, "4", (1, 2))
    r.resize(80, 80)
    got = run(r, "0", (1, 2, 3))
    got_tile = run(r, "0", (1, 2), vp)
    f = T.make(cfg, cfgs, 80, 80)
    want = run(f, "0", (1, 2, 3))
    f.close()
    f = T.make(cfg, cfgs, 80, 80)
    want_tile = run(f, "0", (1, 2), vp)
    for x, y in zip(got + got_tile, want + want_tile):
        assert np.array_equal(x, y)
    assert want_tile[0][24:40, :, :3].any()


@pytest.mark.gpu
@pytest.mark.parametrize("streams", ["1", "3", "4"])
def test_wavefront_stream_count_is_bit_identical(streams, cfgs, monkeypatch, gpu_required):
    """The wavefront rounds' slot halves on 1, 3 or 4 streams (RT0_WF_STREAMS;
    default 2) only change which half holds a slot: the same bits."""
    def go():
        r = rt0.Renderer(80, 64)
        configure(r, cfg_by_name(cfgs, "c4_mandelbulb_vol"), cfgs)
        r.render(1, 3)
        assert r.last_render_path() == "wavefront"
        return r.read_accum()
    monkeypatch.setenv("RT0_WF_STREAMS", "2")
    a = go()
    monkeypatch.setenv("RT0_WF_STREAMS", streams)
    assert np.array_equal(a, go())


@pytest.mark.gpu
@pytest.mark.parametrize("name,size,viewport,split", [
    ("c3_outdoor_restir", 72, None, None),            # ragged tiles
    ("c3_outdoor_restir", 64, (8, 16, 40, 24), None),  # a tile
    ("c3_outdoor_restir", 64, None, "3"),              # three row parts
    ("restir_mis_demo", 64, None, None),
    ("c5_spectral_sphere", 64, None, None),            # spectral weighting
    ("anim_restir_demo", 64, None, None),              # RENDER_MODE 1 (EMA)
])
def test_fused_resolve_is_bit_identical(name, size, viewport, split, cfgs, monkeypatch, gpu_required):
    """rt0_jit_nee completing its own pixels' samples (RT0_FUSED_RESOLVE, the
    default for deferred passes without the occlusion-walk kernel) runs
    rt0_jit_resolve's arithmetic (resolve_pixel) on the same stored calls,
    right after them in the same wave: a 4-pass chain equals the one with the
    resolve launch bit for bit -- samples and reservoirs."""
    if not have(name):
        pytest.skip("fixture not generated")
    if split:
        monkeypatch.setenv("RT0_RESTIR_SPLIT", split)
    monkeypatch.setenv("RT0_FUSED_RESOLVE", "0")
    ref = chain(cfgs, name, "1", n=4, size=size, viewport=viewport)
    monkeypatch.setenv("RT0_FUSED_RESOLVE", "1")
    got = chain(cfgs, name, "1", n=4, size=size, viewport=viewport)
    for what, a, b in zip(("samples", "reservoir main", "reservoir aux"), ref, got):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), what
    assert got[0][..., :3].mean() > 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("name,size", [("c5_spectral_models", (64, 80)), ("c3_outdoor_restir", (72, 64)),
                                       ("restir_mis_demo", (64, 64))])
def test_tap_batch_is_bit_identical(name, size, cfgs, monkeypatch, gpu_required):
    """The light-sampling kernel issues the loads of RT0_TAP_BATCH reservoir
    taps before it lerps any (rt0_integrator.h bil_at / Bil; 2 by default,
    also beside the walk kernel since round 6): the same texels, weights and
    arithmetic as one tap at a time, so a 4-pass chain matches
    RT0_TAP_BATCH=1 bit for bit -- samples and reservoirs."""
    import test_models as T
    if name != "c5_spectral_models" and not have(name):
        pytest.skip("fixture not generated")
    cfg = T.cfg_by_name(cfgs, name)
    out = []
    for extra in ("-DRT0_TAP_BATCH=1", None):
        if extra:
            monkeypatch.setenv("RT0_JIT_EXTRA", extra)
        else:
            monkeypatch.delenv("RT0_JIT_EXTRA", raising=False)
        if name == "c5_spectral_models":
            r = T.make(cfg, cfgs, *size)
        else:
            r = rt0.Renderer(*size)
            configure(r, cfg, cfgs)
            r.set_temporal_frames(cfg.get("temporal_frames", 5))
        S, M, A = [], [], []
        for k in range(1, 5):
            r.render(k, 1)
            S.append(r.read_accum())
            m, a = r.read_restir(0)
            M.append(m)
            A.append(a)
        out.append((np.stack(S), np.stack(M), np.stack(A)))
        r.close()
    for what, a, b in zip(("samples", "reservoir main", "reservoir aux"), out[0], out[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), what
    assert out[1][0][..., :3].mean() > 0.0
