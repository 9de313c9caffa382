"""Size-independent properties of the HIP path at BASELINE sizes (1024^2),
where the CPU oracle would take minutes: determinism, shard/whole identity,
accumulation chaining, finiteness, tonemap epilogue, API state errors."""
import numpy as np
import pytest

import rt0

pytestmark = pytest.mark.gpu


def cfg_by_name(cfgs, name):
    return [c for c in cfgs["configs"] if c["name"] == name][0]


def test_determinism_and_sharding_bitwise(cfgs, gpu_required):
    cfg = cfg_by_name(cfgs, "c2_cornell_mis_8")
    r = rt0.Renderer(1024, 1024)
    rt0.configure(r, cfg, cfgs)
    r.render(1, 2)
    a = r.read_accum()
    r.clear()
    r.render(1, 2)
    assert np.array_equal(a, r.read_accum())
    assert np.isfinite(a).all() and a[..., :3].mean() > 0.01
    # 4 shards of 16-row bands, each rendering only its bands, summed == whole
    parts = np.zeros_like(a)
    for s in range(4):
        rs = rt0.Renderer(1024, 1024)
        rt0.configure(rs, cfg, cfgs)
        rs.set_shard(s, 4, 16)
        rs.render(1, 2)
        p = rs.read_accum()
        rows = np.array([(y // 16) % 4 == s for y in range(1024)])
        assert not p[~rows].any()
        parts[rows] = p[rows]
        rs.close()
    assert np.array_equal(parts, a)


def test_band_packed_shards_bitwise(cfgs, gpu_required):
    """bench.py's multi-GPU layout: each shard renders into a band-packed torch
    buffer (rt0_set_accum_buffer_compact); BandGather's reorder of those
    buffers == the single-GPU image, bit for bit (8 shards: the 1024^2 / 8
    frame-chunked launches included)."""
    import torch
    import rt0.shard as shard
    cfg = cfg_by_name(cfgs, "c2_cornell_mis_8")
    H = W = 256
    r = rt0.Renderer(W, H)
    rt0.configure(r, cfg, cfgs)
    r.render(1, 3)
    a = r.read_accum()
    for world in (3, 8):
        nb = H // 16
        max_owned = (nb + world - 1) // world
        img = np.zeros_like(a)
        for s in range(world):
            rs = rt0.Renderer(W, H)
            rt0.configure(rs, cfg, cfgs)
            rs.set_shard(s, world, 16)
            buf = torch.zeros((max_owned * 16, W, 4), dtype=torch.float32, device="cuda:0")
            rows = rs.set_accum_buffer_compact(buf.data_ptr())
            own = shard.owned_bands(s, world, nb)
            assert rows == len(own) * 16
            rs.render(1, 3)
            torch.cuda.synchronize()
            got = buf.cpu().numpy()
            assert np.array_equal(rs.read_accum()[:rows], got[:rows])  # read_accum covers the packed rows
            for j, b in enumerate(own):
                img[b * 16:(b + 1) * 16] = got[j * 16:(j + 1) * 16]
            assert not got[rows:].any()  # padding rows untouched
            rs.close()
        assert np.array_equal(img, a), world


def test_band_packed_buffer_guards(cfgs, gpu_required):
    """A band-packed buffer is not an image and holds exactly one shard's
    rows: tonemap refuses it, and a later set_shard that changes the owned
    rows makes render fail instead of writing past the buffer."""
    import torch
    cfg = cfg_by_name(cfgs, "c2_cornell_mis_8")
    W = H = 64
    r = rt0.Renderer(W, H)
    rt0.configure(r, cfg, cfgs)
    r.set_shard(0, 2, 16)
    buf = torch.zeros((32, W, 4), dtype=torch.float32, device="cuda:0")
    assert r.set_accum_buffer_compact(buf.data_ptr()) == 32
    r.render(1, 1)
    with pytest.raises(rt0.Rt0Error) as e:
        r.tonemap(1.0)
    assert e.value.code == -3
    r.set_shard(0, 1, 16)  # now owns all 64 rows: the 32-row buffer is too small
    with pytest.raises(rt0.Rt0Error) as e:
        r.render(2, 1)
    assert e.value.code == -4
    r.set_shard(0, 2, 16)  # back to the rows the buffer was set for
    r.render(2, 1)
    r.set_accum_buffer(None)  # the context's own full-size buffer again
    r.set_shard(0, 1, 16)
    r.render(1, 1)
    assert r.tonemap(1.0).shape == (H, W, 4)


def test_chunked_viewport_scratch_is_tile_sized(cfgs, gpu_required):
    """Tile rendering with several passes frame-chunks its launches (a 32x32
    tile is ~16 waves): the per-frame scratch covers the tile, not the
    canvas, and the tile equals the same rectangle of a whole-canvas render."""
    cfg = cfg_by_name(cfgs, "c2_cornell_mis_8")
    W = H = 256
    full = rt0.Renderer(W, H)
    rt0.configure(full, cfg, cfgs)
    full.render(1, 8)
    ref = full.read_accum()
    r = rt0.Renderer(W, H)
    rt0.configure(r, cfg, cfgs)
    r.set_viewport(96, 64, 32, 32)
    r.render(1, 8)
    _, launches = r.last_kernel_ms()
    # the chunked pass and its ordered sum count as one launch of the pass
    # (rt0_host.cpp render_impl); the scratch shows that the pass was chunked
    assert launches == 1
    assert r.samples_bytes() == 8 * 32 * 32 * 16
    got = r.read_accum()
    assert np.array_equal(got[64:96, 96:128], ref[64:96, 96:128])
    mask = np.ones((H, W), bool)
    mask[64:96, 96:128] = False
    assert not got[mask].any()


def test_odd_sizes_and_edges(cfgs, gpu_required):
    cfg = cfg_by_name(cfgs, "c1_cornell_cos")
    for w, h in ((1, 1), (17, 5), (130, 67)):
        r = rt0.Renderer(w, h)
        rt0.configure(r, cfg, cfgs)
        r.render(1, 3)
        a = r.read_accum()
        assert a.shape == (h, w, 4) and np.isfinite(a).all()
    r.render(1, 0)  # zero passes is a no-op
    assert np.array_equal(r.read_accum(), a)


def test_tonemap_epilogue(cfgs, gpu_required):
    r = rt0.Renderer(32, 32)
    rt0.configure(r, cfg_by_name(cfgs, "c2_cornell_mis_8"), cfgs)
    r.render(1, 4)
    acc = r.read_accum()
    img = r.tonemap(0.25)
    ref = np.clip(np.power(np.maximum(acc[..., :3] * 0.25, 0), 1 / 2.2), 0, 1) * 255
    assert img.dtype == np.uint8 and (img[..., 3] == 255).all()
    assert np.abs(img[..., :3].astype(np.float32) - ref).max() <= 1.0


def test_state_errors(cfgs, gpu_required):
    r = rt0.Renderer(16, 16)
    with pytest.raises(rt0.Rt0Error) as e:
        r.render(1, 1)
    assert e.value.code == -4
    cfg = rt0.parse_config([], ["const lowp int RENDER_MODE = 2;"])  # the shader knows modes 0 and 1
    with pytest.raises(rt0.Rt0Error) as e:
        r.set_config(cfg)
    assert e.value.code == -1
    with pytest.raises(ValueError):  # six square RGB faces
        r.set_cubemap([np.zeros((4, 4, 3), np.uint8)] * 5)
    with pytest.raises(ValueError):
        r.set_cubemap([np.zeros((4, 3, 3), np.uint8)] * 6)


def test_glslviewport_drives_backend(cfgs, gpu_required):
    vp = rt0.GlslViewport(None, {"width": 64, "height": 64})
    vp.constants[0] = "const lowp int MAX_BOUNCES = 8;"
    vp.constants[8] = "const bool use_mis = true;"
    for _ in range(3):
        vp.render()
    assert vp.passes == 3
    a = vp.accumulator()
    r = rt0.Renderer(64, 64)
    rt0.configure(r, cfg_by_name(cfgs, "c2_cornell_mis_refcaps"), cfgs)
    r.render(1, 3)
    assert np.array_equal(a, r.read_accum())
    vp.resize(0)
    assert vp.width == 256 and vp.passes == 0


def test_counters_feed_flop_model(cfgs, gpu_required):
    r = rt0.Renderer(64, 64)
    rt0.configure(r, cfg_by_name(cfgs, "c2_cornell_mis_8"), cfgs)
    r.set_counting(True)
    r.render(1, 2)
    c = r.counters()
    assert c["samples"] == 64 * 64 * 2
    assert 5 < c["isect"] / c["samples"] < 30 and 2 < c["iter"] / c["samples"] <= 8
    counted = r.read_accum()
    r.set_counting(False)
    r.clear()
    r.render(1, 2)
    # the counting instance renders the same paths; FMA placement may differ
    # from the uncounted kernels, so compare with the parity tolerance
    plain = r.read_accum()
    ok = (np.abs(counted - plain) <= 1e-3 * np.maximum(1.0, np.abs(plain))).all(-1)
    assert ok.mean() >= 0.99, ok.mean()


def _restir_shards(cfgs, cfg, W, H, world, halo, band=None):
    import torch
    import rt0.shard as shard
    band = band or shard.block_band(H, world)
    out = []
    for rank in range(world):
        r = rt0.Renderer(W, H)
        rt0.configure(r, cfg, cfgs)
        pairs = torch.zeros((4, H, W, 2, 4), dtype=torch.float32, device="cuda:0")  # interleaved main/aux
        r.set_restir_buffers([pairs[k, :, :, j].data_ptr() for k in range(4) for j in range(2)])
        r.set_shard(rank, world, band)
        r.set_halo(halo)
        out.append((r, pairs, {pairs[k, :, :, 0].data_ptr(): k for k in range(4)}))
    torch.cuda.synchronize()
    return out, band


@pytest.mark.parametrize("world,halo", [(3, 24), (4, 24)])
def test_sharded_restir_matches_whole_image(cfgs, gpu_required, world, halo):
    """ReSTIR over contiguous row blocks + per-pass halo exchange of the newest
    reservoir planes (the SURVEY 8e exchange step) == the unsharded render, bit
    for bit, including the temporal passes (u_frame > 2)."""
    import torch
    import rt0.shard as shard
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    W, H, F = 48, 96, 5
    whole = rt0.Renderer(W, H)
    rt0.configure(whole, cfg, cfgs)
    for k in range(1, F + 1):
        whole.render(k, 1)
    ref = whole.read_accum()
    ref_main, ref_aux = whole.read_restir(0)
    shards, band = _restir_shards(cfgs, cfg, W, H, world, halo)

    def newest(s):
        r, pairs, by_ptr = s
        m, _ = r.device_restir(0)
        return [pairs[by_ptr[m]]]

    for k in range(1, F + 1):
        for r, _, _ in shards:
            r.render(k, 1)
        shard.exchange_halo_local([newest(s) for s in shards], band, halo)
        torch.cuda.synchronize()  # torch's copies before librt0's next launch (its own stream)
    img = np.zeros_like(ref)
    main = np.zeros_like(ref_main)
    for rank, (r, _, _) in enumerate(shards):
        lo, hi = shard.block_rows(rank, band, H)
        img[lo:hi] = r.read_accum()[lo:hi]
        main[lo:hi] = r.read_restir(0)[0][lo:hi]
        assert r.halo_misses() == 0
    assert np.array_equal(img, ref)
    assert np.array_equal(main, ref_main)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_restir_round_robin_bands_match_whole_image(cfgs, gpu_required, world):
    """ReSTIR over several round-robin row bands per shard (the bench's
    load-balanced split, shard.interleaved_band) + the per-boundary halo
    exchange == the unsharded render, bit for bit, through temporal passes."""
    import torch
    import rt0.shard as shard
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    W, H, F, halo, band = 48, 192, 5, 24, 48
    whole = rt0.Renderer(W, H)
    rt0.configure(whole, cfg, cfgs)
    for k in range(1, F + 1):
        whole.render(k, 1)
    ref = whole.read_accum()
    ref_main, ref_aux = whole.read_restir(0)
    shards, band = _restir_shards(cfgs, cfg, W, H, world, halo, band)

    def newest(s):
        r, pairs, by_ptr = s
        m, _ = r.device_restir(0)
        return [pairs[by_ptr[m]]]

    for k in range(1, F + 1):
        for r, _, _ in shards:
            r.render(k, 1)
        shard.exchange_halo_local([newest(s) for s in shards], band, halo)
        torch.cuda.synchronize()
    img = np.zeros_like(ref)
    main, aux = np.zeros_like(ref_main), np.zeros_like(ref_aux)
    for rank, (r, _, _) in enumerate(shards):
        own = shard.owned_band_rows(rank, world, band, H)
        assert len(own) >= 1 and (world == 3 or len(own) == 2)
        acc, (m, a) = r.read_accum(), r.read_restir(0)
        for lo, hi in own:
            img[lo:hi], main[lo:hi], aux[lo:hi] = acc[lo:hi], m[lo:hi], a[lo:hi]
        assert r.halo_misses() == 0
    assert np.array_equal(img, ref)
    assert np.array_equal(main, ref_main)
    assert np.array_equal(aux, ref_aux)


def test_round_robin_restir_reports_a_too_small_halo(cfgs, gpu_required):
    """The kernel's halo check over round-robin bands: a 2-row halo is too
    small for the ~16 px spatial taps, and every shard reports misses."""
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    shards, band = _restir_shards(cfgs, cfg, 48, 192, 2, 2, band=48)
    for k in range(1, 3):
        for r, _, _ in shards:
            r.render(k, 1)
    assert all(r.halo_misses() > 0 for r, _, _ in shards)


def test_sharded_restir_reports_a_too_small_halo(cfgs, gpu_required):
    import rt0.shard as shard
    cfg = cfg_by_name(cfgs, "c3_outdoor_restir")
    shards, band = _restir_shards(cfgs, cfg, 48, 96, 3, 2)
    for k in range(1, 3):
        for r, _, _ in shards:
            r.render(k, 1)
    assert shards[1][0].halo_misses() > 0  # the middle block reads 16 px away
    with pytest.raises(rt0.Rt0Error):
        shards[0][0].render(3, 2)  # sharded ReSTIR: one pass per call


def test_tonemap_curves_and_image_files(cfgs, gpu_required, tmp_path):
    """Display epilogue variants + PNG/PFM output of a rendered image."""
    PIL = pytest.importorskip("PIL.Image")
    r = rt0.Renderer(32, 24)
    rt0.configure(r, cfg_by_name(cfgs, "c2_cornell_mis_8"), cfgs)
    r.render(1, 4)
    acc = r.read_accum()
    x = np.maximum(acc[..., :3] * 0.25, 0)
    for mode, curve in ((rt0.TONEMAP_GAMMA, x), (rt0.TONEMAP_REINHARD, x / (1 + x)),
                        (rt0.TONEMAP_ACES, (1.5 * x * (2.51 * 1.5 * x + 0.03)) / (1.5 * x * (2.43 * 1.5 * x + 0.59) + 0.14))):
        img = r.tonemap(0.25, mode)
        ref = np.clip(np.power(np.maximum(curve, 0), 1 / 2.2), 0, 1) * 255
        assert np.abs(img[..., :3].astype(np.float32) - ref).max() <= 1.0, mode
    r.save_png(tmp_path / "c.png", 4)
    assert np.array_equal(np.asarray(PIL.open(tmp_path / "c.png").convert("RGBA")), r.tonemap(0.25)[::-1])
    r.save_pfm(tmp_path / "c.pfm", 4)
    raw = open(tmp_path / "c.pfm", "rb").read()
    assert raw.startswith(b"PF\n32 24\n-1.0\n") and len(raw) == len(b"PF\n32 24\n-1.0\n") + 32 * 24 * 12


def test_texture_api(cfgs, gpu_required):
    """rt0_set_texture argument checks; re-binding a unit takes effect at the
    next render; an unbound unit samples (0,0,0,1) (GL incomplete texture)."""
    from textures import textures_for
    cfg = [c for c in cfgs["configs"] if c["name"] == "tex_light_sphere"][0]
    r = rt0.Renderer(32, 32)
    rt0.configure(r, cfg, cfgs)
    with pytest.raises(rt0.Rt0Error):
        r.set_texture(5, np.zeros((4, 4, 4), np.uint8))
    with pytest.raises(ValueError):
        r.set_texture(0, np.zeros((4, 4, 3), np.uint8))
    r.render(1, 1)
    unbound = r.read_accum()
    tex = textures_for(cfg)
    r.set_texture(1, tex[1])
    r.clear()
    r.render(1, 1)
    bound = r.read_accum()
    assert not np.array_equal(bound, unbound)
    # an all-(0,0,0,255) texture is what an unbound unit samples
    r.set_texture(1, np.tile(np.array([0, 0, 0, 255], np.uint8), (8, 8, 1)))
    r.clear()
    r.render(1, 1)
    assert np.array_equal(r.read_accum(), unbound)


def test_viewport_renders_only_its_rectangle(cfgs, gpu_required):
    """rt0_set_viewport (gl.viewport of tile rendering, index.js:379, 761-792):
    pixels inside the rectangle equal the whole-canvas render bit for bit, the
    rest stays zero; rectangles are clipped to the canvas."""
    cfg = cfg_by_name(cfgs, "c2_cornell_mis_8")
    W, H = 96, 80
    r = rt0.Renderer(W, H)
    rt0.configure(r, cfg, cfgs)
    r.render(1, 3)
    full = r.read_accum()
    for x, y, w, h in ((0, 0, 32, 32), (32, 16, 40, 24), (70, 60, 64, 64), (5, 3, 1, 1)):
        r.clear()
        r.set_viewport(x, y, w, h)
        r.render(1, 3)
        got = r.read_accum()
        inside = np.zeros((H, W), bool)
        inside[y:min(H, y + h), x:min(W, x + w)] = True
        assert np.array_equal(got[inside], full[inside]), (x, y, w, h)
        assert not got[~inside].any()
    r.set_viewport(0, 0, 0, 0)  # whole canvas again
    r.clear()
    r.render(1, 3)
    assert np.array_equal(r.read_accum(), full)


def test_glslviewport_tile_rendering(cfgs, gpu_required):
    """tile_rendering: render() draws the current 32x32 tile, updateTile()
    walks the tiles (passes restart), and after every tile had its passes the
    accumulator is the whole-canvas image."""
    vp = rt0.GlslViewport(None, {"width": 64, "height": 64, "tile_rendering": True})
    vp.constants[0] = "const lowp int MAX_BOUNCES = 8;"
    vp.constants[8] = "const bool use_mis = true;"
    seen = []
    while not vp.paused:
        vp.render(2)
        seen.append(tuple(vp.viewport))
        vp.updateTile()
    assert seen == [(0, 0, 32, 32), (32, 0, 32, 32), (0, 32, 32, 32), (32, 32, 32, 32)]
    r = rt0.Renderer(64, 64)
    rt0.configure(r, cfg_by_name(cfgs, "c2_cornell_mis_refcaps"), cfgs)
    r.render(1, 2)
    assert np.array_equal(vp.accumulator(), r.read_accum())


def test_glslviewport_toggle_restir(cfgs, gpu_required):
    """toggleReSTIR() (index.js:911-927) switches the next render() to the
    ReSTIR path; getReSTIRDebugInfo() reports as the reference does."""
    vp = rt0.GlslViewport(None, {"width": 32, "height": 32})
    vp.render()
    before = vp.accumulator()
    vp.toggleReSTIR()
    assert vp.defines[4] == "#define USE_RESTIR" and "true" in vp.constants[9]
    vp.clear()
    vp.passes = 0
    vp.render(3)
    after = vp.accumulator()
    assert np.isfinite(after).all() and not np.array_equal(after, before)
    info = vp.getReSTIRDebugInfo()
    assert info["passes"] == 3 and info["isReSTIREnabled"] is False and info["temporalFrames"] == 5


@pytest.mark.parametrize("var,val,name,want", [("RT0_JIT", "0", "c2_cornell_mis_8", "aot"),
                                               ("RT0_DEFER_NEE", "0", "c3_outdoor_restir", "pass"),
                                               ("RT0_WAVEFRONT", "0", "sdf_cone", "pass"),
                                               ("RT0_SEGV_TRACE", "1", "c1_cornell_cos", "pass")])
def test_environment_switches_at_create(cfgs, monkeypatch, gpu_required, var, val, name, want):
    """The environment switches include/rt0.h documents, read at rt0_create:
    RT0_JIT=0 (ahead-of-time kernels), RT0_DEFER_NEE=0 (inline ReSTIR light
    sampling), RT0_WAVEFRONT=0 (the pass kernel for SDF scenes) and
    RT0_SEGV_TRACE=1 (a native stack on SIGSEGV; chains to the previous
    handler) -- each changes which kernels run, never the image beyond the
    documented tolerances."""
    cfg = cfg_by_name(cfgs, name)

    def go():
        r = rt0.Renderer(32, 32)
        rt0.configure(r, cfg, cfgs)
        r.render(1, 2)
        return r.read_accum(), r.last_render_path()
    base, bp = go()
    monkeypatch.setenv(var, val)
    got, gp = go()
    assert gp == want, (var, gp)
    assert np.isfinite(got).all() and got[..., :3].any()
    ok = (np.abs(got - base) <= 1e-3 * np.maximum(1.0, np.abs(base))).all(-1)
    assert ok.mean() >= 0.97, (var, bp, gp, ok.mean())
