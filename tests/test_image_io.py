"""Image assets either side of the path: librt0's PNG
decoder (texture units, index.js:257-300 / 699-728) and PNG / PFM writers
(display canvas, HDR accumulator), checked against PIL on synthetic images.
Host-only: runs on CPU."""
import io

import numpy as np
import pytest

import rt0

PIL = pytest.importorskip("PIL.Image")


def _png(img, **kw):
    b = io.BytesIO()
    img.save(b, format="PNG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("mode", ["RGBA", "RGB", "L", "LA", "P"])
def test_png_decode_matches_pil(mode):
    rng = np.random.default_rng(7)
    rgba = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    img = PIL.fromarray(rgba, "RGBA").convert(mode)
    data = _png(img, optimize=(mode == "P"))
    got = rt0.png_decode(data)
    ref = np.asarray(PIL.open(io.BytesIO(data)).convert("RGBA"))
    assert got.shape == (37, 53, 4) and np.array_equal(got, ref)


def test_png_decode_every_filter_type():
    # a gradient + noise image makes PIL's encoder pick all five filters
    y, x = np.mgrid[0:64, 0:64]
    rgba = np.stack([x * 4, y * 4, (x * y) % 256, 255 - x], -1).astype(np.uint8)
    rgba[::7] = np.random.default_rng(1).integers(0, 256, rgba[::7].shape, dtype=np.uint8)
    data = _png(PIL.fromarray(rgba, "RGBA"), optimize=True)
    assert np.array_equal(rt0.png_decode(data), rgba)


def test_png_decode_rejects_bad_input():
    good = _png(PIL.fromarray(np.zeros((4, 4, 4), np.uint8), "RGBA"))
    bad = bytearray(good)
    bad[40] ^= 0xFF  # inside IDAT: CRC mismatch
    with pytest.raises(rt0.Rt0Error):
        rt0.png_decode(bytes(bad))
    with pytest.raises(rt0.Rt0Error):
        rt0.png_decode(b"not a png at all")
    sixteen = _png(PIL.fromarray(np.zeros((4, 4), np.uint16)))
    with pytest.raises(rt0.Rt0Error) as e:
        rt0.png_decode(sixteen)
    assert e.value.code == -3  # RT0_E_UNSUPPORTED


def test_png_write_roundtrip_and_flip(tmp_path):
    rgba = np.random.default_rng(3).integers(0, 256, (20, 30, 4), dtype=np.uint8)
    p = tmp_path / "a.png"
    rt0.png_write(p, rgba)
    assert np.array_equal(np.asarray(PIL.open(p).convert("RGBA")), rgba)
    assert np.array_equal(rt0.png_read(p), rgba)
    rt0.png_write(p, rgba, flip_y=True)  # accumulator rows are bottom-up
    assert np.array_equal(np.asarray(PIL.open(p).convert("RGBA")), rgba[::-1])


def test_pfm_write(tmp_path):
    acc = np.random.default_rng(5).random((6, 9, 4), dtype=np.float32) * 10
    p = tmp_path / "a.pfm"
    rt0.pfm_write(p, acc, 0.25)
    raw = open(p, "rb").read()
    head = b"PF\n9 6\n-1.0\n"
    assert raw.startswith(head)
    data = np.frombuffer(raw[len(head):], "<f4").reshape(6, 9, 3)
    assert np.array_equal(data, (acc[..., :3] * np.float32(0.25)).astype(np.float32))


def test_jpeg_decode_matches_libjpeg():
    """Baseline JPEG (the reference's cubemap format) decodes within 3 levels of
    libjpeg (Pillow), for 4:4:4, 4:2:2 and 4:2:0 chroma and a restart interval."""
    PIL = pytest.importorskip("PIL.Image")
    import io
    y, x = np.mgrid[0:70, 0:93]
    img = np.stack([(x * 2.7) % 256, (y * 3.1) % 256, ((x + y) * 1.3) % 256], -1)
    img = (img * 0.8 + (np.arange(70 * 93 * 3).reshape(70, 93, 3) * 7919 % 50)).clip(0, 255).astype(np.uint8)
    for sub, extra in [(0, {}), (1, {}), (2, {}), (2, {"restart_marker_blocks": 3})]:
        b = io.BytesIO()
        try:
            PIL.fromarray(img).save(b, "JPEG", quality=90, subsampling=sub, **extra)
        except TypeError:
            continue
        data = b.getvalue()
        ref = np.asarray(PIL.open(io.BytesIO(data)).convert("RGB")).astype(int)
        got = rt0.jpeg_decode(data)
        assert got.shape == (70, 93, 4) and (got[..., 3] == 255).all()
        assert np.abs(got[..., :3].astype(int) - ref).max() <= 3, sub


def test_jpeg_rejects_non_baseline(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    import io
    b = io.BytesIO()
    PIL.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, "JPEG", progressive=True)
    with pytest.raises(rt0.Rt0Error) as e:
        rt0.jpeg_decode(b.getvalue())
    assert e.value.code == -3
    with pytest.raises(rt0.Rt0Error):
        rt0.jpeg_decode(b"\x00\x01garbage")
