#!/usr/bin/env python3
"""make_golden.py -- generate tests/golden/*.npz from the REFERENCE shader.

TEST INFRASTRUCTURE ONLY; runs in the build container (needs /root/reference,
node and the SwiftShader libraries bundled with kaleido).  Nothing here runs on
the GPU box.

For every config of tests/golden/configs.json:
  1. node make_shader.js expands raytracer.glsl with the reference's own
     parseShader / GlslViewport defaults (oracle/_gen/<name>.frag, ignored by git);
  2. glrun (oracle/gen/glrun.c, built to oracle/_ref/glrun) renders `frames`
     passes at 64x64 with the accumulator input bound to zero (--single), so each
     output is exactly one sample per pixel of pass k (u_frame = k);
  3. the RGBA32F outputs are stored as <name>.npz: samples[F,H,W,4] (row 0 =
     bottom row, gl_FragCoord.y = 0.5), and for ReSTIR configs the two reservoir
     MRTs restir_main/restir_aux[F,H,W,4].
A known-answer shader (make_shader.js --kat) is run once for the RNG stream:
rng_kat.npz.  manifest.json records the effective host state and NaN counts.

usage: python3 oracle/gen/make_golden.py [config-name ...]
"""
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
GOLD = os.path.join(REPO, "tests", "golden")
GEN = os.path.join(REPO, "oracle", "_gen")
REFBIN = os.path.join(REPO, "oracle", "_ref")
W = H = 64  # default fixture size; configs may set "fixture_size"


def sh(cmd, **kw):
    return subprocess.run(cmd, check=True, capture_output=True, text=True, **kw)


def build_glrun():
    os.makedirs(REFBIN, exist_ok=True)
    out = os.path.join(REFBIN, "glrun")
    sh(["gcc", "-O2", "-o", out, os.path.join(HERE, "glrun.c"), "-ldl"])
    return out


def cam_args(cfg, cfgs):
    c = cfg["camera"] or cfgs["default_camera"]
    v = list(c["origin"]) + list(c["lookat"]) + [c["fov"], c["aperture"], c["focalLength"]]
    return ["--cam"] + ["%r" % float(x) for x in v]


def parse_host_state(state):
    """defines/constants strings -> {name: value} (no reference text kept)."""
    defs = {}
    for d in state["defines"]:
        name = d.split("#define")[1].strip()
        defs[name] = not d.lstrip().startswith("//")
    consts = {}
    for c in state["constants"]:
        lhs, rhs = c.split("=")
        name = lhs.split()[-1]
        v = rhs.strip().rstrip(";").strip()
        consts[name] = True if v == "true" else False if v == "false" else (float(v) if "." in v else int(v))
    return defs, consts


def run_config(glrun, cfgs, cfg):
    name = cfg["name"]
    frag = os.path.join(GEN, name + ".frag")
    st = sh(["node", os.path.join(HERE, "make_shader.js"), os.path.join(GOLD, "configs.json"), name, frag])
    defs, consts = parse_host_state(json.loads(st.stdout))
    frames = int(cfg["frames"])
    W, H = cfg.get("fixture_size", [64, 64])
    restir = bool(defs.get("USE_RESTIR"))
    prefix = os.path.join(GEN, name)
    cmd = [glrun, "--frag", frag, "--w", str(W), "--h", str(H), "--single", "--out", prefix] + cam_args(cfg, cfgs)
    if restir:
        cmd.append("--restir-out")
    if cfg.get("time_ms"):  # u_time of pass k = t0 + (k-1)*dt (RENDER_MODE 1 configs)
        cmd += ["--time", repr(float(cfg["time_ms"][0])), "--dtime", repr(float(cfg["time_ms"][1]))]
    # asset textures (u_tex0..3 = GL units 1..4, u_rnd_tex = unit 5; index.js:149-163)
    sys.path.insert(0, os.path.dirname(HERE))
    from textures import cubemap_for, textures_for
    faces = cubemap_for(cfg)
    if faces is not None:  # u_cubemap = GL unit 6, faces in the reference's upload order
        fn = "%s_cube.rgb8" % prefix
        np.concatenate([np.ascontiguousarray(f, np.uint8).ravel() for f in faces]).tofile(fn)
        cmd += ["--cube", str(faces[0].shape[0]), fn]
    for unit, img in textures_for(cfg).items():
        fn = "%s_tex%d.rgba8" % (prefix, unit)
        np.ascontiguousarray(img, np.uint8).tofile(fn)
        cmd += ["--tex", str(unit + 1), str(img.shape[1]), str(img.shape[0]), fn]
    skipped = []
    if cfg.get("tiles"):
        return run_tiled(cfg, cmd, prefix, W, H, restir, defs, consts)
    if cfg.get("frame_timeout"):
        # Per-frame mode (volumetric configs): SwiftShader 4.1 does not finish
        # some passes of these shaders (a pass of 8x8 pixels either renders in
        # ~2 s or runs for > 5 min), so every u_frame is its own glrun call
        # with a time limit; frames that do not finish are skipped and
        # recorded, the fixture keeps the first `frames` that do.
        ids = []
        for k in range(1, int(cfg.get("frame_tries", 4 * frames)) + 1):
            try:
                sh(cmd + ["--frames", "1", "--frame0", str(k)], timeout=float(cfg["frame_timeout"]))
                ids.append(k)
            except subprocess.TimeoutExpired:
                skipped.append(k)
            if len(ids) == frames:
                break
        if not ids:
            raise RuntimeError("%s: no frame finished within %s s" % (name, cfg["frame_timeout"]))
    else:
        ids = list(range(1, frames + 1))
        # volumetric shaders take SwiftShader hours: RT0_GOLDEN_TIMEOUT
        sh(cmd + ["--frames", str(frames)], timeout=int(os.environ.get("RT0_GOLDEN_TIMEOUT", "1800")))

    def load(tag):
        return np.stack([np.fromfile("%s_f%d_%s.bin" % (prefix, k, tag), dtype=np.float32).reshape(H, W, 4)
                         for k in ids])

    out = {"samples": load("c")}
    if cfg.get("events") and not restir:
        # the first-event records: the instrumented shader's run, kept where its
        # image equals the plain run's bit for bit
        ifrag = frag[:-len(".frag")] + "_events.frag"
        with open(ifrag, "w") as f:
            f.write(instrument_events(open(frag).read()))
        eprefix = prefix + "_ev"
        ecmd = list(cmd)
        ecmd[ecmd.index("--frag") + 1] = ifrag
        ecmd[ecmd.index("--out") + 1] = eprefix
        sh(ecmd + ["--restir-out", "--frames", str(frames)], timeout=int(os.environ.get("RT0_GOLDEN_TIMEOUT", "1800")))
        ev = {tag: np.stack([np.fromfile("%s_f%d_%s.bin" % (eprefix, k, tag), dtype=np.float32).reshape(H, W, 4)
                             for k in ids]) for tag in "cra"}
        same = (ev["c"] == out["samples"]).all(-1) | (np.isnan(ev["c"]).all(-1) & np.isnan(out["samples"]).all(-1))
        out["exec_events"] = np.concatenate([ev["r"], ev["a"]], axis=-1)  # (F, H, W, 8)
        out["events_valid"] = same
    if cfg.get("frame_timeout"):
        out["frames"] = np.asarray(ids, np.int32)  # u_frame of each samples[i]
    if restir:
        out["restir_main"] = load("r")
        out["restir_aux"] = load("a")
    np.savez_compressed(os.path.join(GOLD, name + ".npz"), **out)
    nan = int(np.isnan(out["samples"][..., :3]).any(axis=-1).sum())
    return {"defines": defs, "constants": consts, "frames": ids, "skipped_frames": skipped, "width": W, "height": H,
            "restir": restir, "nan_pixels": nan,
            "mean_rgb": [float(x) for x in np.nanmean(out["samples"][..., :3], axis=(0, 1, 2))]}


def swiftshader_dir(threads):
    """A working directory whose SwiftShader.ini pins the executor's thread
    count ([Processor] ThreadCount): SwiftShader reads it from the current
    directory.  Default (no ini) = one thread per core."""
    d = tempfile.mkdtemp(prefix="rt0_ss%d_" % threads)
    with open(os.path.join(d, "SwiftShader.ini"), "w") as f:
        f.write("[Processor]\nThreadCount=%d\n" % threads)
    return d


# ---- executor path records (tiled configs with "paths": true) ----
# Textual instrumentation of the expanded reference shader: globals written in
# radiance()'s bounce loop body (raytracer.glsl:1994-2102) record, per lane,
# the iterations the loop body ran, the depth at each (base 16, six iterations
# per float: g_h0..g_h2) and the way each iteration ended (base 8, eight per
# float: g_e0, g_e1; 1 scatter `continue`, 2 miss `break`, 3 light hit, 4 mask
# cut-off, 5 bounce caps, 6 scatter cap, 7 end of body), so every field is an
# integer below 2^24 and exact in fp32 at any depth the fixtures use (the
# round-5 encoding, one float per record, lost late-iteration digits beyond
# 2^24 at 12 bounces); then SCATTERING_EVENTS + 256 DIFF_BOUNCES and
# TRANS_BOUNCES + 256 SPEC_BOUNCES.  main() writes them to the reservoir MRTs,
# which a non-ReSTIR shader leaves at zero (2220-2223).  Writes in the loop
# body are masked like the body itself (mask_kat.py rule 1) -- plain
# statements, no function calls (a call after a `break` still runs, rule 1) --
# so they show what the executor ran.  FragColor is untouched; run_tiled keeps
# a pixel only if the instrumented image equals the plain one bit for bit.
PATH_EV = {1: "S", 2: "m", 3: "L", 4: "k", 5: "T", 6: "X", 7: "."}


def instrument_paths(src):
    def sub(old, new):
        nonlocal src
        assert src.count(old) == 1, old
        src = src.replace(old, new)

    def ev(e):  # the current iteration's exit event
        return "if (g_pit <= 8.0) g_e0 = g_e0 * 8.0 + %d.0; else g_e1 = g_e1 * 8.0 + %d.0;" % (e, e)
    sub("vec3 radiance(Ray r, float seed){",
        "float g_pit = 0.0; float g_h0 = 0.0; float g_h1 = 0.0; float g_h2 = 0.0; float g_e0 = 0.0; float g_e1 = 0.0;\n"
        "vec3 radiance(Ray r, float seed){")
    sub("  for (int depth = 0; depth < MAX_BOUNCES; ++depth){\n",
        "  for (int depth = 0; depth < MAX_BOUNCES; ++depth){\n    g_pit += 1.0;\n"
        "    if (g_pit <= 6.0) g_h0 = g_h0 * 16.0 + float(depth); else if (g_pit <= 12.0) g_h1 = g_h1 * 16.0 + "
        "float(depth); else g_h2 = g_h2 * 16.0 + float(depth);\n")
    sub("max(mask.r, max(mask.g, mask.b)) < 0.01) break;\n            continue;",
        "max(mask.r, max(mask.g, mask.b)) < 0.01) { %s break; }\n"
        "            %s\n            continue;" % (ev(6), ev(1)))
    sub("      if(!bounceIsSpecular && sample_lights) break;",
        "      if(!bounceIsSpecular && sample_lights) { %s break; }" % ev(2))
    sub("#endif\n\n      break;\n    }", "#endif\n      %s\n      break;\n    }" % ev(2))
    sub("      acc += mask * e * misWeight;\n      break;",
        "      acc += mask * e * misWeight;\n      %s\n      break;" % ev(3))
    sub("    if(max(mask.x, max(mask.y, mask.z)) < 0.01) break;",
        "    if(max(mask.x, max(mask.y, mask.z)) < 0.01) { %s break; }" % ev(4))
    sub("SCATTERING_EVENTS >= MAX_SCATTERING_EVENTS ) break;\n  }",
        "SCATTERING_EVENTS >= MAX_SCATTERING_EVENTS ) { %s break; }\n"
        "    %s\n  }" % (ev(5), ev(7)))
    sub("    ReSTIRData = vec4(0.0);\n    ReSTIRAux = vec4(0.0);",
        "    ReSTIRData = vec4(g_pit, g_h0, g_h1, g_h2);\n"
        "    ReSTIRAux = vec4(g_e0, g_e1, float(SCATTERING_EVENTS) + 256.0 * float(DIFF_BOUNCES), "
        "float(TRANS_BOUNCES) + 256.0 * float(SPEC_BOUNCES));")
    return src


# ---- first-event records (configs with "events": true) ----
# For the glossy METAL scenes: what the executor computed along each lane's
# path, written to the reservoir MRTs (a non-ReSTIR shader leaves them at
# zero): [0] the first intersection's t, [1] its texel (the METAL value-noise
# f that sets the glossiness, getTexel 762-768), [2..4] the ray direction
# brdf() leaves after the first bounce (the SDF normal of calcNormal and the
# glossy reflection), [5] the second intersection's t, [6] the path's
# decisions as an integer < 2^24 -- per bounce d < 6 two bits (1 SDF 0 hit,
# 2 another hit, 3 miss) at 2d, and one bit at 12 + d when brdf() added to
# the radiance (its environment NEE ray escaped, 1887-1897; the scenes have no
# lights) -- and [7] the red channel of the first miss's environment sample.
# Plain statements in radiance() (masked like the code around them,
# mask_kat.py rule 1; not inside brdf(), whose ghost calls write globals);
# run_config keeps a pixel-sample only where this image equals the plain one
# bit for bit.  The restatement writes the same record (RT0_DEBUG_EVENTS), so
# each departing pixel's first divergent event is named
# (tests/test_oracle_golden.py test_metal_departures_attributed).
def instrument_events(src):
    def sub(old, new):
        nonlocal src
        assert src.count(old) == 1, old
        src = src.replace(old, new)
    sub("vec3 radiance(Ray r, float seed){",
        "float g_t0 = -1.0; float g_f0 = -1.0; vec3 g_rd1 = vec3(0.0); float g_t1 = -1.0; float g_dec = 0.0; "
        "float g_env = -1.0; float g_pw = 1.0; float g_pb = 4096.0;\n"
        "vec3 radiance(Ray r, float seed){")
    sub("    Hit hit;\n    float t = intersection(r, hit);\n",
        "    Hit hit;\n    float t = intersection(r, hit);\n"
        "    if (depth == 0) { g_t0 = t; g_f0 = hit.texel.r; } else if (depth == 1) { g_t1 = t; }\n"
        "    if (depth > 0) { g_pw *= 4.0; g_pb *= 2.0; }\n"
        "    if (depth < 6) g_dec += (t == INFINITY ? 3.0 : (hit.index == NUM_MESHES ? 1.0 : 2.0)) * g_pw;\n")
    sub("#ifdef USE_CUBEMAP\n        acc += mask * texture(u_cubemap, r.d).rgb;",
        "#ifdef USE_CUBEMAP\n        acc += mask * texture(u_cubemap, r.d).rgb;\n"
        "        if (g_env < 0.0) g_env = texture(u_cubemap, r.d).r;")
    sub("        acc += mask * (vec3(0.5) + vec3(0.5) * cos(TWO_PI * (vec3(0.525, 0.408, 0.409) + vec3(0.9, 0.97, 0.8) * "
        "clamp(r.d.y * 0.6 + 0.5, 0.3, 1.0))));",
        "        acc += mask * (vec3(0.5) + vec3(0.5) * cos(TWO_PI * (vec3(0.525, 0.408, 0.409) + vec3(0.9, 0.97, 0.8) * "
        "clamp(r.d.y * 0.6 + 0.5, 0.3, 1.0))));\n"
        "        if (g_env < 0.0) g_env = 0.5 + 0.5 * cos(TWO_PI * (0.525 + 0.9 * clamp(r.d.y * 0.6 + 0.5, 0.3, 1.0)));")
    sub("    brdf(hit, c, e, t, inside, r, mask, acc, bounceIsSpecular, seed, float(depth));\n",
        "    vec3 g_acc0 = acc;\n"
        "    brdf(hit, c, e, t, inside, r, mask, acc, bounceIsSpecular, seed, float(depth));\n"
        "    if (depth == 0) g_rd1 = r.d;\n"
        "    if (depth < 6 && any(notEqual(acc, g_acc0))) g_dec += g_pb;\n")
    sub("    ReSTIRData = vec4(0.0);\n    ReSTIRAux = vec4(0.0);",
        "    ReSTIRData = vec4(g_t0, g_f0, g_rd1.x, g_rd1.y);\n"
        "    ReSTIRAux = vec4(g_rd1.z, g_t1, g_dec, g_env);")
    return src


def path_conformance(cfg, cfgs, exec_paths, exec_aux):
    """GLSL-semantics path records of the restatement (oracle/rt0_oracle.c
    RT0_DEBUG_PATHS: the same fields, the same encodings) and the lanes whose
    executor record equals them: iterations, depth history, exit events and
    scattering events all the same (the bounce counters are not compared: the
    executor's ghost brdf() calls bump them, mask_kat.py rule 1)."""
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle as O
    F, Hh, Ww = exec_paths.shape[:3]
    o = O.Oracle(cfg, cfgs, width=Ww, height=Hh, overrides={"SWIFTSHADER_GHOST": 1, "RT0_DEBUG_PATHS": 1})
    ref_p, ref_a = [], []
    for k in range(1, F + 1):
        _, m, a = o.frame(k)
        ref_p.append(m)
        ref_a.append(a)
    ref_p, ref_a = np.stack(ref_p), np.stack(ref_a)
    return ((exec_paths == ref_p).all(-1) & (exec_aux[..., :2] == ref_a[..., :2]).all(-1) &
            (np.mod(exec_aux[..., 2], 256.0) == np.mod(ref_a[..., 2], 256.0)))


def run_tiled(cfg, cmd, prefix, W, H, restir, defs, consts):
    """Tiled mode (deep volumetric configs): every (u_frame, tile) is its own
    glrun call with glScissor on the tile and a time limit, run once per
    SwiftShader thread count of cfg["thread_counts"].  A pixel is `valid` when
    its tile finished in every run with the same value: the executor does not
    finish some fragments of these shaders (a tile either renders in ~2 s or
    runs for minutes), and in some branches it reads registers another quad
    left behind, so a full-image render depends on the thread count (measured
    on vol_cornell_2 u_frame 6: ThreadCount 2 changes pixel (x 2, y 6); 1, 3,
    8 and 16 agree).  One 2x2 quad per call shares no registers with another."""
    tw, th = cfg["tiles"]
    frames = int(cfg["frames"])
    tcs = cfg.get("thread_counts", [1, 3])
    dirs = {t: swiftshader_dir(t) for t in tcs}
    jobs = [(k, x, y) for k in range(1, frames + 1) for y in range(0, H, th) for x in range(0, W, tw)]
    paths = bool(cfg.get("paths")) and not restir
    # with path records, the FIRST thread count runs the instrumented shader
    # (its image must equal the plain runs' bit for bit to be kept)
    pcmd = list(cmd)
    if paths:
        fi = cmd.index("--frag") + 1
        ifrag = cmd[fi][:-len(".frag")] + "_paths.frag"
        with open(ifrag, "w") as f:
            f.write(instrument_paths(open(cmd[fi]).read()))
        pcmd[fi] = ifrag
        pcmd.append("--restir-out")

    def run(k, x, y, t):
        out = "%s_k%d_x%d_y%d_t%d" % (prefix, k, x, y, t)
        instr = paths and t == tcs[0]
        try:
            subprocess.run((pcmd if instr else cmd) + ["--frames", "1", "--frame0", str(k), "--scissor", str(x), str(y),
                                                      str(tw), str(th), "--out", out], check=True,
                           capture_output=True, cwd=dirs[t], timeout=float(cfg["tile_timeout"]))
        except subprocess.TimeoutExpired:
            return None
        img = {"c": np.fromfile("%s_f%d_c.bin" % (out, k), dtype=np.float32).reshape(H, W, 4)}
        if instr:
            for tag in "ra":
                img["p" + tag] = np.fromfile("%s_f%d_%s.bin" % (out, k, tag), dtype=np.float32).reshape(H, W, 4)
        if restir:
            for tag in "ra":
                img[tag] = np.fromfile("%s_f%d_%s.bin" % (out, k, tag), dtype=np.float32).reshape(H, W, 4)
        for f in os.listdir(os.path.dirname(out)):
            if f.startswith(os.path.basename(out) + "_"):
                os.remove(os.path.join(os.path.dirname(out), f))
        return img

    def one(job):
        """The tile under every thread count (stopping at the first run that
        does not finish: one quad per call renders the same either way)."""
        imgs = []
        for t in tcs:
            img = run(*job, t)
            if img is None:
                return job, None
            imgs.append(img)
        return job, imgs

    workers = int(os.environ.get("RT0_GOLDEN_WORKERS", "6"))
    with ThreadPoolExecutor(workers) as ex:
        results = list(ex.map(one, jobs))
    samples = np.zeros((frames, H, W, 4), np.float32)
    valid = np.zeros((frames, H, W), bool)
    aux = {tag: np.zeros((frames, H, W, 4), np.float32) for tag in ("ra" if restir else "")}
    if paths:
        aux.update({tag: np.zeros((frames, H, W, 4), np.float32) for tag in ("pr", "pa")})
    timed_out = 0
    for (k, x, y), imgs in results:
        sl = (k - 1, slice(y, y + th), slice(x, x + tw))
        if imgs is None:
            timed_out += 1
            continue
        tile = imgs[0]["c"][y:y + th, x:x + tw]
        same = np.ones(tile.shape[:2], bool)
        for other in imgs[1:]:
            o = other["c"][y:y + th, x:x + tw]
            same &= (o == tile).all(-1) | (np.isnan(o).all(-1) & np.isnan(tile).all(-1))
        samples[sl] = tile
        valid[sl] = same
        for tag in aux:
            aux[tag][sl] = imgs[0][tag][y:y + th, x:x + tw]
    out = {"samples": samples, "valid": valid, "frames": np.arange(1, frames + 1, dtype=np.int32)}
    if restir:
        out["restir_main"], out["restir_aux"] = aux["r"], aux["a"]
    name = cfg["name"]
    extra = {}
    if paths:
        # exec_paths: iterations, depth history, SCATTERING_EVENTS, DIFF_BOUNCES;
        # exec_exits: exit events, TRANS_BOUNCES, 0, SPEC_BOUNCES (instrument_paths)
        out["exec_paths"], out["exec_exits"] = aux["pr"], aux["pa"]
        conf = path_conformance(cfg, json.load(open(os.path.join(GOLD, "configs.json"))), aux["pr"], aux["pa"])
        out["conformant"] = conf & valid
        extra = {"paths": True, "conformant_pixel_samples": int(out["conformant"].sum())}
    np.savez_compressed(os.path.join(GOLD, name + ".npz"), **out)
    v = samples[..., :3][valid]
    return {**extra, "defines": defs, "constants": consts, "frames": list(range(1, frames + 1)), "width": W, "height": H,
            "restir": restir, "tiles": [tw, th], "thread_counts": tcs, "tiles_timed_out": timed_out,
            "tile_jobs": len(jobs), "valid_pixel_samples": int(valid.sum()),
            "nan_pixels": int(np.isnan(v).any(-1).sum()) if v.size else 0,
            "mean_rgb": [float(x) for x in (np.nanmean(v, axis=0) if v.size else [0, 0, 0])]}


def run_kat(glrun, cfgs):
    frag = os.path.join(GEN, "rng_kat.frag")
    sh(["node", os.path.join(HERE, "make_shader.js"), os.path.join(GOLD, "configs.json"),
        "c1_cornell_cos", frag, "--kat"])
    prefix = os.path.join(GEN, "rng_kat")
    frames = 3
    sh([glrun, "--frag", frag, "--w", str(W), "--h", str(H), "--frames", str(frames), "--single",
        "--restir-out", "--out", prefix] + cam_args(cfgs["configs"][0], cfgs))
    arr = {}
    for tag in "cra":
        arr["kat_" + tag] = np.stack([np.fromfile("%s_f%d_%s.bin" % (prefix, k, tag), dtype=np.float32)
                                      .reshape(H, W, 4) for k in range(1, frames + 1)])
    np.savez_compressed(os.path.join(GOLD, "rng_kat.npz"), **arr)


def main():
    cfgs = json.load(open(os.path.join(GOLD, "configs.json")))
    only = set(sys.argv[1:])
    glrun = build_glrun()
    os.makedirs(GEN, exist_ok=True)
    man_path = os.path.join(GOLD, "manifest.json")
    manifest = json.load(open(man_path)) if os.path.exists(man_path) else {}
    manifest["_generator"] = ("oracle/gen/make_golden.py: reference raytracer.glsl expanded by the reference's "
                              "parseShader (tools.js:22-61) + GlslViewport defaults (index.js), executed by "
                              "SwiftShader 4.1 GLES3 (kaleido bundle) via oracle/gen/glrun.c; single-sample "
                              "passes (u_bufferA = 0), 64x64, unpatched powerHeuristic")
    manifest.setdefault("configs", {})
    if not only or "rng_kat" in only:
        run_kat(glrun, cfgs)
    for cfg in cfgs["configs"]:
        if only and cfg["name"] not in only:
            continue
        if cfg.get("unpinned"):  # no reference code for this feature (triangles/BVH): oracle-only config
            continue
        info = run_config(glrun, cfgs, cfg)
        # re-read so that concurrent generator runs (one per slow config) merge
        manifest = json.load(open(man_path)) if os.path.exists(man_path) else manifest
        manifest.setdefault("configs", {})[cfg["name"]] = info
        json.dump(manifest, open(man_path, "w"), indent=1, sort_keys=True)
        print(cfg["name"], info["nan_pixels"], info["mean_rgb"], flush=True)
    json.dump(manifest, open(man_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
