#!/usr/bin/env python3
"""tex_kat.py -- known-answer shaders that measure how the oracle's executor
(SwiftShader 4.1, run by oracle/gen/glrun.c) filters an RGBA8 texture with
GL_LINEAR + GL_REPEAT, the state of the reference's asset textures
(GlslViewport.loadTexture, index.js:703-708; glrun.c --tex).

TEST INFRASTRUCTURE ONLY (build container; needs the kaleido SwiftShader
bundle).  The shaders are minimal GLSL ES 3.00 programs, not reference text:
each fragment samples one texture at a coordinate computed from its
gl_FragCoord and writes the texel to FragColor and the coordinate to
ReSTIRData, so the fixture holds the exact float32 (u, v) the executor used.

Output: tests/golden/tex_filter_kat.npz -- per case k: tex_k (H x W x 4
uint8), uv_k (4096 x 2 float32), n_k (4096 x 4 uint16: the sample x 65535,
which the executor's readback makes an integer); and a cubemap case --
cube_faces (6 x 16 x 16 x 3, order -X -Y -Z +X +Y +Z), cube_dir_* / cube_rgb_*
(4 096 directions each, spread over the sphere and next to a face edge and
its corners) -- for the seamless filter's corner rule.  tests/test_oracle_golden.py
checks the restatement's tex_fetch_ss (oracle/rt0_oracle.c) against it.

usage: python3 oracle/gen/tex_kat.py
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
GLRUN = os.path.join(REPO, "oracle", "_ref", "glrun")

HEAD = """#version 300 es
precision highp float;
precision highp int;
uniform vec2 u_resolution;
uniform uint u_frame;
uniform sampler2D u_bufferA;
uniform sampler2D u_tex0;
layout(location = 0) out vec4 FragColor;
layout(location = 1) out vec4 ReSTIRData;
layout(location = 2) out vec4 ReSTIRAux;
void main() {
  ivec2 p = ivec2(gl_FragCoord.xy);
  float i = float(p.y * 64 + p.x);
  vec2 uv = %s;
  FragColor = texture(u_tex0, uv);
  ReSTIRData = vec4(uv, 0.0, 0.0);
  ReSTIRAux = vec4(0.0);
}
"""


def textures():
    rng = np.random.default_rng(2026)
    out = []
    # 2x1 pairs: constants, ramps both ways, small steps
    for pairs in ([(255, 255), (0, 0), (1, 1), (128, 128)], [(0, 1), (1, 0), (254, 255), (100, 200)],
                  [(0, 255), (255, 0), (10, 250), (128, 129)], [(2, 2), (127, 127), (64, 64), (0, 17)]):
        t = np.array([[[a for a, _ in pairs], [b for _, b in pairs]]], np.uint8)
        out.append(("pairs", t, "vec2(i / 4096.0, 0.5)"))
    # the same pairs vertically (1x2), and off the 1/4096 grid
    out.append(("vertical", out[2][1].transpose(1, 0, 2).copy(), "vec2(0.5, i / 4096.0)"))
    out.append(("offgrid", out[2][1], "vec2(i / 4096.0 + 1.0 / 28672.0, 0.5)"))
    # 2x2: one-hot texels on a grid of sub-texel positions, random texels off it
    oh = np.zeros((2, 2, 4), np.uint8)
    oh[0, 0, 0] = oh[0, 1, 1] = oh[1, 0, 2] = oh[1, 1, 3] = 255
    out.append(("onehot", oh, "(vec2(p) / 64.0 + 0.5) / 2.0"))
    out.append(("rand2x2", rng.integers(0, 256, (2, 2, 4), dtype=np.uint8),
                "vec2((float(p.x) + 0.37) / 64.0, (float(p.y) + 0.61) / 64.0)"))
    # wrapped coordinates on larger power-of-two sizes (the assets are 256^2 and 512^2)
    out.append(("w64", rng.integers(0, 256, (1, 64, 4), dtype=np.uint8), "vec2(-2.3 + i * 0.00123457, 0.37)"))
    out.append(("w8x4", rng.integers(0, 256, (4, 8, 4), dtype=np.uint8),
                "vec2(-2.3 + i * 0.00123457, 1.7 - i * 0.000731)"))
    # (the assets' widths; few rows keep the fixture small)
    out.append(("w256", rng.integers(0, 256, (4, 256, 4), dtype=np.uint8),
                "vec2(-1.37 + i * 0.000913, 2.11 - i * 0.001093)"))
    out.append(("w512", rng.integers(0, 256, (8, 512, 4), dtype=np.uint8),
                "vec2(3.7 - i * 0.00171, -0.43 + i * 0.000377)"))
    # a non-power-of-two size (none of the reference's assets)
    out.append(("npot53x37", rng.integers(0, 256, (37, 53, 4), dtype=np.uint8),
                "vec2((1.7 - i * 0.000731) * 3.1, (-2.3 + i * 0.00123457) * 0.77)"))
    return out


def run(tex, expr, d):
    frag = os.path.join(d, "k.frag")
    with open(frag, "w") as f:
        f.write(HEAD % expr)
    tf = os.path.join(d, "t.rgba8")
    tex.tofile(tf)
    prefix = os.path.join(d, "o")
    subprocess.run([GLRUN, "--frag", frag, "--w", "64", "--h", "64", "--frames", "1", "--single", "--restir-out",
                    "--out", prefix, "--tex", "1", str(tex.shape[1]), str(tex.shape[0]), tf],
                   check=True, capture_output=True, text=True, timeout=300)
    c = np.fromfile(prefix + "_f1_c.bin", np.float32).reshape(-1, 4).astype(np.float64) * 65535.0
    n = np.round(c)
    assert np.abs(c - n).max() < 0.01, "readback is not k / 65535"
    uv = np.fromfile(prefix + "_f1_r.bin", np.float32).reshape(-1, 4)[:, :2].copy()
    return n.astype(np.uint16), uv


CUBE = """#version 300 es
precision highp float;
precision highp int;
uniform vec2 u_resolution;
uniform uint u_frame;
uniform sampler2D u_bufferA;
uniform samplerCube u_cubemap;
layout(location = 0) out vec4 FragColor;
layout(location = 1) out vec4 ReSTIRData;
layout(location = 2) out vec4 ReSTIRAux;
void main() {
  ivec2 p = ivec2(gl_FragCoord.xy);
  float i = float(p.y * 64 + p.x);
  vec3 d;
  if (%s) {  // directions spread over the sphere
    float z = 1.0 - 2.0 * (i + 0.5) / 4096.0;
    float r = sqrt(max(0.0, 1.0 - z * z));
    float a = i * 2.399963;
    d = vec3(r * cos(a), z, r * sin(a));
  } else {  // next to the +Z / +X edge and its two corners
    float a = -1.0 + 2.0 * (float(p.x) + 0.5) / 64.0;
    float b = 0.9 + 0.1 * (float(p.y) + 0.5) / 64.0;
    d = vec3(b, a, 1.0);
  }
  FragColor = texture(u_cubemap, d);
  ReSTIRData = vec4(d, 0.0);
  ReSTIRAux = vec4(0.0);
}
"""


def run_cube(faces, spread, d):
    """The cubemap (RGB8, GL_LINEAR, seamless as GLES3 filters it; glrun.c
    --cube) at 4 096 directions: (RGB, the direction)."""
    frag = os.path.join(d, "c.frag")
    with open(frag, "w") as f:
        f.write(CUBE % ("true" if spread else "false"))
    cf = os.path.join(d, "cube.rgb8")
    faces.tofile(cf)
    prefix = os.path.join(d, "q")
    subprocess.run([GLRUN, "--frag", frag, "--w", "64", "--h", "64", "--frames", "1", "--single", "--restir-out",
                    "--out", prefix, "--cube", str(faces.shape[1]), cf], check=True, capture_output=True, text=True,
                   timeout=300)
    c = np.fromfile(prefix + "_f1_c.bin", np.float32).reshape(-1, 4)[:, :3].copy()
    dirs = np.fromfile(prefix + "_f1_r.bin", np.float32).reshape(-1, 4)[:, :3].copy()
    return c, dirs


def main():
    arrays, names = {}, []
    with tempfile.TemporaryDirectory() as d:
        for k, (name, tex, expr) in enumerate(textures()):
            n, uv = run(tex, expr, d)
            arrays["tex_%d" % k], arrays["uv_%d" % k], arrays["n_%d" % k] = tex, uv, n
            names.append(name)
            print(name, tex.shape, n[:2].tolist())
        faces = np.random.default_rng(7).integers(0, 256, (6, 16, 16, 3), dtype=np.uint8)
        arrays["cube_faces"] = faces
        for tag, spread in (("spread", True), ("edge", False)):
            arrays["cube_rgb_" + tag], arrays["cube_dir_" + tag] = run_cube(faces, spread, d)
    arrays["names"] = np.array(names)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "tex_filter_kat.npz"), **arrays)


if __name__ == "__main__":
    main()
