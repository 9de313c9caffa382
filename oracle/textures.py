"""Asset textures for the texture fixtures: the reference's own files, and
deterministic synthetic stand-ins.

TEST INFRASTRUCTURE ONLY (imported by oracle/gen/make_golden.py and tests/).
The reference samples four image textures (textures/tex0-3.png, index.html:262)
and an RGBA noise image (textures/rgba_noise/rgba_noise256.png, index.js:258-273).
Those assets are not shipped; the fixtures use stand-ins of the same kind,
generated here by integer hashing only (bit-identical on every machine and
numpy version), so that the SwiftShader run of the reference shader, the C
restatement and the GPU see the same texels:

* noise256: 256x256 RGBA8; R, B, A are hash noise and G is R shifted by
  (37, 17) texels -- G(x, y) = R(x - 37, y - 17) -- the layout value_noise()
  relies on (raytracer.glsl:397-399 reads .yx at uv + (37, 17)*z), so the
  noise is continuous across integer z like with the reference asset.
* image(w, h, seed): RGBA8 with smooth colour gradients, a hash-noise term and
  an alpha channel that varies over the image (MAT_LIGHT_4_TEX / MAT_TEST mix
  by texel.a, raytracer.glsl:1203, 2071).
"""
import os

import numpy as np

# The reference's asset files, copied unchanged as test inputs
# (tests/golden/assets/: textures/rgba_noise/rgba_noise256.png,
# textures/tex0-3.png, cubemaps/Tropical Beach/*.jpg).  Decoded with Pillow --
# PNG is lossless, and Pillow's libjpeg is the decoder family browsers use for
# the reference's JPEG faces; the same pixels go to the reference executor
# (oracle/gen/glrun.c), the restatement and the GPU, so the fixtures test the
# integrator, not the decoders (rt0's own PNG/JPEG decoders are checked
# against Pillow in tests/test_image_io.py).
ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "assets")
# index.html:267-270: left, bottom, back, right, top, front = -X -Y -Z +X +Y +Z
CUBE_FACES = ("left", "bottom", "back", "right", "top", "front")


def asset_rgba(name):
    """RGBA8 [h, w, 4] of an asset file; RGB images get alpha 255 (what
    texImage2D(RGBA) of an opaque image holds)."""
    from PIL import Image
    im = Image.open(os.path.join(ASSETS, name))
    return np.asarray(im.convert("RGBA"), np.uint8).copy()


def asset_cube():
    from PIL import Image
    return [np.asarray(Image.open(os.path.join(ASSETS, "tropical_beach", f + ".jpg")).convert("RGB"), np.uint8).copy()
            for f in CUBE_FACES]


def _hash32(x):
    """lowbias32 integer hash, uint32 -> uint32 (numpy, wrap-around)."""
    x = np.asarray(x, np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def _noise_plane(w, h, salt):
    y, x = np.mgrid[0:h, 0:w].astype(np.uint32)
    return (_hash32(x + np.uint32(w) * y + np.uint32((salt * 0x9E3779B9) & 0xFFFFFFFF)) >> np.uint32(24)).astype(np.uint8)


def noise256():
    n = 256
    r = _noise_plane(n, n, 1)
    g = np.roll(np.roll(r, 17, axis=0), 37, axis=1)  # g[y, x] = r[y - 17, x - 37]
    b = _noise_plane(n, n, 2)
    a = _noise_plane(n, n, 3)
    return np.stack([r, g, b, a], axis=-1)


def image(w, h, seed):
    y, x = np.mgrid[0:h, 0:w].astype(np.int64)
    nz = _noise_plane(w, h, 100 + seed).astype(np.int64)
    r = (x * 255) // max(1, w - 1)
    g = (y * 255) // max(1, h - 1)
    b = ((x + y + 64 * seed) * 3) % 256
    a = 64 + ((x * 7 + y * 3 + 17 * seed) % 192)
    px = np.stack([(r * 3 + nz) // 4, (g * 3 + nz) // 4, (b * 3 + nz) // 4, a], axis=-1)
    return px.astype(np.uint8)


def cube_faces(n=64):
    """Six smooth RGB8 n x n faces (reference upload order -X -Y -Z +X +Y +Z):
    per-face gradients with a distinct blue level, so the sky a ray sees
    depends on the face and the position on it."""
    y, x = np.mgrid[0:n, 0:n].astype(np.int64)
    faces = []
    for i in range(6):
        r = (x * 255) // (n - 1) if i % 2 == 0 else 255 - (x * 255) // (n - 1)
        g = (y * 200) // (n - 1) + 20 * (i // 2)
        b = np.full_like(x, 30 + 40 * i)
        faces.append(np.stack([r, g, b], axis=-1).astype(np.uint8))
    return faces


def cubemap_for(cfg):
    """Cube faces for a configs.json entry: "cubemap": true -> the synthetic
    faces, "asset" -> the reference's Tropical Beach faces, else None."""
    c = cfg.get("cubemap")
    if c == "asset":
        return asset_cube()
    return cube_faces(64) if c else None


def textures_for(cfg):
    """{unit: uint8 [h, w, 4]} for a configs.json entry's "textures" list
    ("noise" -> unit 4 = u_rnd_tex; "imageN" -> unit N = u_texN; the
    reference's files: "asset:noise" -> unit 4, "asset:texN" -> unit N)."""
    out = {}
    for name in cfg.get("textures", []):
        if name == "asset:noise":
            out[4] = asset_rgba("rgba_noise256.png")
        elif name.startswith("asset:tex"):
            k = int(name[9:])
            out[k] = asset_rgba("tex%d.png" % k)
        elif name == "noise":
            out[4] = noise256()
        elif name.startswith("image"):
            k = int(name[5:])
            out[k] = image(64 + 32 * k, 64 + 16 * k, k)
        else:
            raise KeyError(name)
    return out
