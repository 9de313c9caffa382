"""Pin the CPU restatement (oracle/rt0_oracle.c) to the reference.

The golden fixtures (tests/golden/*.npz) are the reference's own fragment
shader run by SwiftShader (oracle/gen/make_golden.py).  This file checks:
  * the RNG stream -- per-pixel seed (raytracer.glsl:2120), hash (302-306),
    hash2 (308-312) and the bounce/NEE seed schedule -- BIT-EXACTLY;
  * single-sample radiance of every config within the tolerance below;
  * ReSTIR: with the reference's own reservoir buffers of passes k-1..k-3 as
    input, pass k's radiance matches per pixel ("conditional parity"), and,
    with the executor's masked-execution behaviour after `break` modelled
    (SWIFTSHADER_GHOST; pinned by the known-answer shaders of
    oracle/gen/mask_kat.py, tests/golden/mask_kat.json), so do pass k's
    reservoir outputs -- and then the unconditional 6-pass chain.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Tolerance (frozen after measuring restatement vs oracle):
# a pixel matches when every channel satisfies |d| <= 1e-3 * max(1, |ref|);
# transcendental ulp drift (glibc vs SwiftShader) may flip rare discrete
# decisions (shadow ray at an edge, hash < Re, SDF h < EPSILON), so at most
# BAD_FRAC of pixels may differ.  Pixels where the reference is NaN are
# excluded and counted.
REL_TOL = 1e-3
# Menger sponge: every path grazes many SDF edges where mod()/floor() ulp drift
# flips the march (1.2% measured, all flips: median error 0).
# The volumetric fixtures are 8x8 (per-frame generation, make_golden.py): 384
# pixels, so one discrete flip is 0.26%; 2 measured on vol_cornell_2 (a
# shadow ray at the light's silhouette, a scatter-distance boundary).
BAD_FRAC = {"default": 0.005, "c4_mandelbulb_vol": 0.02, "spectral_vol_1l": 0.02, "menger_coat": 0.02,
            # C4 at 12 bounces, tiled + thread-pinned: compared on the ~88% of
            # valid pixel-samples whose bounce loop the executor ran as GLSL
            # says (`conformant`, test_deep_volume_executor_paths); on the rest
            # it departs (mask_kat.py rules 8 and 10: a scatter `continue`
            # retires lanes), measured there, not modelled
            "c4_mandelbulb_deep": 0.02, "c4_mandelbulb_deep_novol": 0.02,
            "vol_cornell_2": 0.011,
            "restir_mis_demo": 0.01,
            # glossy METAL (value-noise roughness) reflections grazing the slab's
            # front edge: SwiftShader's bilinear filtering of the noise texture
            # differs from exact fp32 bilinear by ~6e-4 median (measured with a
            # value_noise KAT shader), enough to move those reflections across
            # the edge; 3.4% measured
            "tex_sdf_metal": 0.04,
            # the same scene under a cubemap: the metal's glossy reflections now
            # see a textured environment instead of the smooth procedural sky
            "cube_sdf_metal": 0.07,
            # the same METAL scene on the reference's own assets: the real
            # noise texture and the 1024^2 Tropical Beach faces give the glossy
            # reflections high-frequency detail; with the executor's texture
            # filter (the default, SWIFTSHADER_TEX_FILTER) 6.3% of pixels
            # differ (24% under exact fp32 bilinear)
            "page_scene0_slabfirst": 0.07,
            # the textured light's emission on the real tex1.png (0.59%; 1.7% fp32)
            "page_scene1": 0.008, "tex_check_assets": 0.001}
# Mean-radiance tolerance (default 2e-3).  cube_sdf_metal: in this SDF-only
# scene SwiftShader's image depends on the ORDER of the two SDF statements
# (mean 0.4244 vs 0.4310 when swapped; with a plain mirror instead of METAL the
# mismatch stays 6.4%), while GLSL semantics -- and the restatement, 0.4177 vs
# 0.4179 -- are order-independent: an executor artefact, DESIGN.md sec. 2.
MEAN_TOL = {"cube_sdf_metal": 0.02,
            # its 3.5% glossy-reflection departures move the mean by 0.2% (either filter)
            "tex_sdf_metal": 0.003,
            # 8x8 per-frame fixtures: one discrete flip onto the light (emission 4)
            # moves the mean of 128-384 samples by up to 0.03
            "c4_mandelbulb_vol": 0.1, "vol_cornell_2": 0.02, "spectral_vol_1l": 0.05,
            "c4_mandelbulb_deep": 0.005, "c4_mandelbulb_deep_novol": 0.005}


def pixel_match(got, ref):
    nan = np.isnan(ref).any(-1)
    d = np.abs(got - ref)
    ok = (d <= REL_TOL * np.maximum(1.0, np.abs(ref))).all(-1) | nan
    return ok, nan


def have(name):
    return os.path.exists(os.path.join(GOLD, name + ".npz"))


def test_rng_seed_bitexact():
    kat = np.load(os.path.join(GOLD, "rng_kat.npz"))
    c = kat["kat_c"]
    for f in range(c.shape[0]):
        for y in range(0, 64, 7):
            for x in range(64):
                s = np.float32(O.pixel_seed(np.float32(x + 0.5), np.float32(y + 0.5), f + 1))
                assert s == c[f, y, x, 0], (f, y, x)


def test_rng_hash_schedule_bitexact():
    kat = np.load(os.path.join(GOLD, "rng_kat.npz"))
    c, r, a = kat["kat_c"], kat["kat_r"], kat["kat_a"]
    f32 = np.float32
    for f in range(c.shape[0]):
        fr = f32(f + 1)
        for y in range(0, 64, 5):
            for x in range(0, 64, 3):
                s = c[f, y, x, 0]
                assert f32(O.hash_(f32(s + f32(13.271)))) == c[f, y, x, 1]
                assert f32(O.hash_(f32(s + f32(63.216)))) == c[f, y, x, 2]
                assert f32(O.hash_(f32(s + f32(496.4562)))) == c[f, y, x, 3]
                assert f32(O.hash_(f32(s + f32(249.1686)))) == a[f, y, x, 2]
                # bounce seed, raytracer.glsl:1810: ((seed + 7.1*f) + 5681.123) + depth*92.13
                b0 = f32(f32(f32(s + f32(f32(7.1) * fr)) + f32(5681.123)) + f32(f32(0.0) * f32(92.13)))
                b3 = f32(f32(f32(s + f32(f32(7.1) * fr)) + f32(5681.123)) + f32(f32(3.0) * f32(92.13)))
                assert (O.hash2(b0, b0) == r[f, y, x, :2]).all()
                assert (O.hash2(b3, b3) == r[f, y, x, 2:]).all()
                # plain-NEE seed + sphere-light offset, raytracer.glsl:1972 / 1190
                n1 = f32(f32(f32(f32(s + f32(f32(8652.1) * fr)) + f32(5681.123)) + f32(f32(1.0) * f32(7895.13)))
                         + f32(23.1656))
                assert (O.hash2(n1, n1) == a[f, y, x, :2]).all()


NON_RESTIR = ["c1_cornell_cos", "c2_cornell_mis_refcaps", "c2_cornell_mis_8", "cornell_nee_plain",
              "c4_mandelbulb_vol", "spectral_vol_1l", "mis_demo_sdfbox", "menger_coat", "thinlens_glass",
              "tex_sdf_metal", "tex_light_sphere", "tex_check_test", "cube_spheres", "cube_sdf_metal",
              "sdf_triprism", "sdf_cone", "spectral_cornell", "vol_cornell_2",
              "page_scene0_slabfirst", "tex_check_assets", "page_scene1", "cube_spheres_assets",
              "c4_mandelbulb_deep", "c4_mandelbulb_deep_novol"]


@pytest.mark.parametrize("name", NON_RESTIR)
def test_oracle_radiance_matches_reference(name, cfgs):
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    # u_frame of each pass (per-frame fixtures skip passes the executor did not finish)
    frames = G["frames"] if "frames" in G else range(1, gold.shape[0] + 1)
    o = O.Oracle(cfg, cfgs, width=gold.shape[2], height=gold.shape[1], overrides={"SWIFTSHADER_GHOST": 1})
    got = np.stack([o.frame(int(k))[0] for k in frames])[..., :3]
    # tiled fixtures: only the pixels whose tile the executor finished, with the
    # same value under two thread counts (oracle/gen/make_golden.py run_tiled);
    # with path records, only the lanes whose bounce loop the executor ran as
    # GLSL says (`conformant`, test_deep_volume_executor_paths)
    valid = G["conformant"] if "conformant" in G else G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    ok, nan = pixel_match(got, gold)
    bad = 1.0 - ok[valid].mean()
    assert bad <= BAD_FRAC.get(name, BAD_FRAC["default"]), "%s: %.4f of pixels differ" % (name, bad)
    assert nan[valid].mean() < 0.001
    # mean radiance agrees tightly (a systematic error would shift it)
    m = ~nan & valid
    assert abs(got[m].mean() - gold[m].mean()) <= MEAN_TOL.get(name, 2e-3) * max(1.0, abs(gold[m].mean()))
    if "conformant" in G:
        # the conformant mask is defined by agreement with this restatement's
        # own path record: a path-structure bug would move lanes out of it
        # instead of failing the check above, so all valid lanes are held too,
        # at the bound the executor's measured departures allow (12% of lanes
        # depart, 75% of those by more than the pixel tolerance)
        allv = G["valid"]
        bad_all = 1.0 - ok[allv].mean()
        assert bad_all <= 0.13, "%s: %.4f of all valid pixel-samples differ" % (name, bad_all)


@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "c5_spectral_sphere"])
def test_oracle_restir_conditional_parity(name, cfgs):
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    o = O.Oracle(cfg, cfgs, width=G["samples"].shape[2], height=G["samples"].shape[1])
    z = np.zeros_like(G["restir_main"][0])

    def out(k, key):
        return G[key][k - 1] if k >= 1 else z

    for k in range(1, G["samples"].shape[0] + 1):
        ins = [out(k - 1, "restir_main"), out(k - 1, "restir_aux"), out(k - 2, "restir_main"),
               out(k - 2, "restir_aux"), out(k - 3, "restir_main"), out(k - 3, "restir_aux")]
        s, _, _ = o.frame(k, ins)
        ok, _ = pixel_match(s[..., :3], G["samples"][k - 1][..., :3])
        assert 1.0 - ok.mean() <= BAD_FRAC.get(name, BAD_FRAC["default"]), (name, k, 1.0 - ok.mean())


def _ghost_expected(name, stop):
    """What the reference executor produces for mask_kat case `name` at a lane
    that breaks at iteration `stop` (rules 1-6 of oracle/gen/mask_kat.py):
    (g0, g1, o0) with g0 = None where the value is undefined (rule 3)."""
    prev = stop - 1  # the lane's previous call (rule 2), none if stop == 0
    val = None
    if name in ("break_then_call", "global_in_callee_if", "nested_break"):
        val, calls, loc = float(prev), stop + 1, float(stop)
    elif name == "nested_call":
        val, calls, loc = 2.0 * (10.0 * prev + 5.0), stop + 1, 10.0 * stop + 5.0
    elif name in ("arg_before_break", "uniform_stop"):
        val, calls, loc = 10.0 * prev + 5.0, stop + 1, 10.0 * stop + 5.0
    elif name == "struct_arg":
        val, calls, loc = 10.0 * prev + 5.0 + 100.0 * prev, stop + 1, 10.0 * stop + 5.0
    elif name == "inout_arg":  # the inout parameter after the previous call: v + 0.5
        val, calls, loc = 10.0 * prev + 5.5 + 1000.0 * prev, stop + 1, 10.0 * stop + 5.0
    elif name == "global_in_loop":  # GLSL semantics (rule 1: loop-body writes are masked)
        val, calls, loc = (float(prev) if stop > 0 else -1.0), stop, float(stop)
        return val, calls, loc
    elif name == "after_continue":  # GLSL semantics (rule 6)
        return (5.0 if stop != 5 else 4.0), 5, 5.0
    if stop == 0 and name in ("global_in_callee_if", "nested_call"):
        calls = None  # the call's effect depends on a parameter (`on`, `b`) that is undefined
    return (val if stop > 0 else None), calls, loc


def test_mask_kat_model():
    """Every output of the executor known-answer shaders follows rules 1-6
    (mask_kat.py) -- the model the restatement's SWIFTSHADER_GHOST and the
    product's rt0_set_executor_compat implement."""
    K = json.load(open(os.path.join(GOLD, "mask_kat.json")))["cases"]
    for name, rows in K.items():
        for r in rows:
            stop = r["stop"]
            if name == "local_array_index":
                # rule 7: iteration i reads arr[0] (= v) instead of the min (0.5 v)
                # when the quad's first lane left the loop before iteration i
                x, y = r["x"], r["y"]
                lane0 = [q for q in rows if q["x"] == x & ~1 and q["y"] == y & ~1][0]["stop"]
                got = r["g"] + r["o"][:2]
                for i in range(6):
                    v = (i + 1) * 10.0 + x + 0.5
                    exp = -1.0 if i > stop else (v if lane0 < i else 0.5 * v)
                    assert got[i] == exp, (name, r, i)
                continue
            if name == "callee_loops":
                # rule 5: loops of <= 4 constant iterations without break/continue
                # are unrolled and run in the ghost call, the others do not
                calls = stop + 1
                assert r["g"] == [2.0 * calls, 3.0 * calls, 4.0 * calls, 5.0 * stop], (name, r)
                assert r["o"] == [9.0 * stop, 2.0 * stop, 2.0 * stop, 3.0 * stop], (name, r)
                continue
            val, calls, loc = _ghost_expected(name, stop)
            assert calls is None or r["g"][1] == calls, (name, r)
            assert r["o"][0] == loc, (name, r)
            if val is not None:
                assert r["g"][0] == val, (name, r)
    # GLSL semantics would give g1 == stop for the break cases: the artefact is real
    assert any(r["g"][1] != r["stop"] for r in K["break_then_call"])


def test_mask_kat_departures():
    """Executor departures from GLSL semantics pinned by known answers
    (oracle/gen/mask_kat.py rules 8-9): a `continue` followed later in the
    loop body by a `break` retires the lane (the construct of the reference's
    volumetric bounce loop, raytracer.glsl:2050 / 2057-2101) -- which is why
    volumetric scenes deeper than one bounce are darker in the reference than
    under GLSL semantics (c4_mandelbulb_deep); the controls and the two-light
    in-scatter construct (2011-2044) run as GLSL says."""
    D = json.load(open(os.path.join(GOLD, "mask_kat.json")))["departures"]
    assert all(r["exec"] == 1.0 and r["glsl"] == 31.0 for r in D["continue_then_break"])
    for name in ("continue_no_break", "break_then_continue", "inscatter_two_lights"):
        assert all(r["exec"] == r["glsl"] for r in D[name]), name
    assert len({r["glsl"] for r in D["inscatter_two_lights"]}) > 3  # the case exercises both lights


def test_deep_volume_executor_paths(cfgs):
    """C4 at its bench depth (12 bounces + medium): the fixture holds, per
    pixel-sample, the record of what the executor ran in radiance()'s bounce
    loop (iterations, depths, exits, scattering events; make_golden.py
    instrument_paths, whose image equals the plain shader's bit for bit).
    The restatement's own record (RT0_DEBUG_PATHS) under GLSL semantics
    reproduces the `conformant` mask exactly, most lanes are conformant, and on
    them the radiance matches tightly (test_oracle_radiance_matches_reference).
    On the other lanes the executor departs from GLSL semantics (rule 10 of
    mask_kat.py among others): measured here, not modelled."""
    name = "c4_mandelbulb_deep"
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    valid, conf = G["valid"], G["conformant"]
    o = O.Oracle(cfg, cfgs, width=16, height=16, overrides={"SWIFTSHADER_GHOST": 1, "RT0_DEBUG_PATHS": 1})
    S, P, X = [], [], []
    for k in G["frames"]:
        s, p, x = o.frame(int(k))
        S.append(s), P.append(p), X.append(x)
    S, P, X = np.stack(S), np.stack(P), np.stack(X)
    ep, ex = G["exec_paths"], G["exec_exits"]
    # iterations, depth history, exit events, scattering events (not the
    # bounce counters, which the executor's ghost calls bump: rule 1)
    mine = ((ep == P).all(-1) & (ex[..., :2] == X[..., :2]).all(-1) &
            (np.mod(ex[..., 2], 256.0) == np.mod(X[..., 2], 256.0)) & valid)
    assert (mine == conf).all()
    assert conf.sum() >= 0.85 * valid.sum(), (int(conf.sum()), int(valid.sum()))
    # the departing lanes, measured: most of them differ, and all one way
    gold = G["samples"][..., :3]
    ok, _ = pixel_match(S[..., :3], gold)
    dep = valid & ~conf
    assert 1.0 - ok[dep].mean() > 0.5
    assert S[..., :3][dep].mean() > gold[dep].mean()


def _path_digits(v, base, n):
    """The n digits (oldest first) of one path-record field."""
    v, d = int(v), []
    for _ in range(n):
        d.append(v % base)
        v //= base
    return d[::-1]


def _path_seq(fields, base, per, n):
    """The first n digits (oldest first) of a path-record sequence spread over
    fields of `per` digits each (make_golden.py instrument_paths: the depth
    history in base 16, six iterations per float; the exit events in base 8,
    eight per float -- every field exact in fp32)."""
    out = []
    for k, v in enumerate(fields):
        m = min(per, n - k * per)
        if m <= 0:
            break
        out += _path_digits(v, base, m)
    return out


def test_deep_volume_departures_accounted(cfgs):
    """Every lane of c4_mandelbulb_deep whose executor record departs from
    GLSL semantics, classified from the fixture's own records
    (exec_paths/exec_exits) against the restatement's (RT0_DEBUG_PATHS):
      (a) retired after a first-iteration scatter `continue` (record: one
          iteration, one event = 1): every such lane meets rule 10's
          condition (mask_kat.py QUAD CONTINUE: GLSL takes the continue in
          iteration 1 and the lane is not its quad's first lane) -- but the
          condition is not sufficient here, most candidates run as GLSL says;
      (b) the first iteration's depth increment lost (depth 0 repeated; its
          exit event missing or recorded) -- only in quads where no lane
          scatters in iteration 1: another mechanism;
      (c) anything else: bounded at 0.5% of the valid lanes.
    Quads are the 2x2 scissor tiles of one glrun call each (tiles [2, 2])."""
    name = "c4_mandelbulb_deep"
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    valid, conf = G["valid"], G["conformant"]
    ep, ex = G["exec_paths"], G["exec_exits"]
    o = O.Oracle(cfg, cfgs, width=16, height=16, overrides={"SWIFTSHADER_GHOST": 1, "RT0_DEBUG_PATHS": 1})
    P, X = [], []
    for k in G["frames"]:
        _, p, x = o.frame(int(k))
        P.append(p), X.append(x)
    P, X = np.stack(P), np.stack(X)
    F, H, W = valid.shape

    def first_event(f, y, x):
        return _path_seq(X[f, y, x, :2], 8, 8, int(P[f, y, x, 0]))[0]

    cand = set()  # rule 10's condition under GLSL semantics
    for f, y, x in zip(*np.nonzero(valid)):
        if int(P[f, y, x, 0]) > 1 and first_event(f, y, x) == 1 and not (x % 2 == 0 and y % 2 == 0):
            cand.add((f, y, x))
    kinds = {"a": [], "b": [], "c": []}
    for f, y, x in zip(*np.nonzero(valid & ~conf)):
        n = int(ep[f, y, x, 0])
        hist, ev = _path_seq(ep[f, y, x, 1:4], 16, 6, n), _path_seq(ex[f, y, x, :2], 8, 8, n)
        if n == 1 and ev == [1]:
            kinds["a"].append((f, y, x))
        elif n >= 2 and hist[0] == 0 and hist[1] == 0:
            kinds["b"].append((f, y, x))
        else:
            kinds["c"].append((f, y, x))
    assert all(p in cand for p in kinds["a"]), "a retirement outside rule 10's condition"
    assert len(kinds["a"]) < len(cand)  # (41 of 351 in the committed fixture)
    for f, y, x in kinds["b"]:
        fy, fx = y & ~1, x & ~1
        quad = [(fy, fx), (fy, fx + 1), (fy + 1, fx), (fy + 1, fx + 1)]
        assert all(first_event(f, a, b) != 1 for a, b in quad if valid[f, a, b])
    assert len(kinds["a"]) + len(kinds["b"]) + len(kinds["c"]) == int((valid & ~conf).sum())
    assert len(kinds["c"]) <= 0.005 * valid.sum(), len(kinds["c"])


def test_mask_kat_quad_continue():
    """Rule 10 (mask_kat.py QUAD CONTINUE): in the reference's bounce-loop
    shape, a lane that takes the scatter `continue` in the loop's first
    iteration is retired -- unless it is the quad's first lane or that lane is
    not covered -- and later continues are honoured.  Some of these quads
    never finish (recorded as HANG: the executor spins in the loop, as in the
    deep volumetric fixture's timed-out tiles); every quad that finishes
    follows the rule."""
    Q = json.load(open(os.path.join(GOLD, "mask_kat.json")))["quad_continue"]
    assert len(Q) >= 20
    retired = finished = hangs = 0
    for case in Q:
        lanes = case["lanes"]
        if lanes[0]["exec"] == "HANG":
            assert all(r["exec"] == "HANG" for r in lanes)
            hangs += 1
            continue
        finished += 1
        lane0 = lanes[0]["covered"]
        for r in lanes:
            if not r["covered"]:
                assert r["exec"] is None
                continue
            cm = case["cms"][r["lane"]]
            retire = (cm & 1) == 1 and r["lane"] != 0 and lane0
            retired += retire
            assert r["exec"] == ("S" if retire else r["glsl"]), (case["cms"], case["cov"], r)
    assert finished >= 15 and retired >= 8 and hangs >= 1, (finished, retired, hangs)
    # a quad where no covered lane continues in the first iteration runs as GLSL says
    calm = [c for c in Q if c["lanes"][0]["exec"] != "HANG"
            and not any(r["covered"] and c["cms"][r["lane"]] & 1 for r in c["lanes"])]
    assert calm and all(r["exec"] in (None, r["glsl"]) for c in calm for r in c["lanes"])


def test_mask_kat_quad_lights():
    """Rule 11 (mask_kat.py QUAD LIGHTS): in brdf's light-loop shape, a lane's
    reads of light_index[i] are right exactly when the quad's first lane runs
    the loop in the same iteration, live or as the ghost call of the iteration
    it breaks in; otherwise both read one stale index -- the end of the loop
    (value 1) without a `continue` before the break, 0 (value 6) with a
    never-taken one.  Re-derived for every pixel of the three shapes."""
    Q = json.load(open(os.path.join(GOLD, "mask_kat.json")))["quad_lights"]
    by = {k: {(r["x"], r["y"]): r for r in v} for k, v in Q.items()}
    stale = {"quad_lights_plain": (1.0,), "quad_lights_shape": (6.0,), "quad_lights_scatter": (1.0, 6.0)}

    def runs(r, d, ghost):  # GLSL: the lane calls nee() in iteration d (ghost: or breaks there and would)
        for e in range(d):
            if not (r["scat"] >> e) & 1 and e == r["stop"]:
                return False
        if (r["scat"] >> d) & 1 or (d == r["stop"] and not ghost):
            return False
        return not (r["spec"] >> d) & 1

    n_right = n_stale = n_ghost = 0
    for name, rows in by.items():
        for (x, y), r in rows.items():
            q0 = rows[(x & ~1, y & ~1)]
            for d in range(4):
                if not runs(r, d, False):
                    assert r["rec"][d] == 0.0, (name, x, y, d)
                elif runs(q0, d, True):
                    assert r["rec"][d] == 10.0, (name, x, y, d)
                    n_right += 1
                    n_ghost += not runs(q0, d, False)
                else:
                    assert r["rec"][d] in stale[name], (name, x, y, d, r["rec"][d])
                    n_stale += 1
    assert n_right >= 60 and n_stale >= 40 and n_ghost >= 4, (n_right, n_stale, n_ghost)


def _res_match(a, b):
    return (np.abs(a - b) <= REL_TOL * np.maximum(1.0, np.abs(b))).all(-1)


@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "c5_spectral_sphere"])
def test_oracle_restir_reservoirs_conditional(name, cfgs):
    """Pass k's reservoir MRTs (g_final_reservoir, raytracer.glsl:2171-2174)
    from the reference's own reservoirs of passes k-1..k-3: >= 99% of pixels
    with the executor model, against 43% (c3) under plain GLSL semantics."""
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    o = O.Oracle(cfg, cfgs, width=G["samples"].shape[2], height=G["samples"].shape[1],
                 overrides={"SWIFTSHADER_GHOST": 1})
    z = np.zeros_like(G["restir_main"][0])

    def out(k, key):
        return G[key][k - 1] if k >= 1 else z

    for k in range(1, G["samples"].shape[0] + 1):
        ins = [out(k - 1, "restir_main"), out(k - 1, "restir_aux"), out(k - 2, "restir_main"),
               out(k - 2, "restir_aux"), out(k - 3, "restir_main"), out(k - 3, "restir_aux")]
        _, m, a = o.frame(k, ins)
        ok = _res_match(m, G["restir_main"][k - 1]) & _res_match(a, G["restir_aux"][k - 1])
        assert ok.mean() >= 0.99, (name, k, ok.mean())


# Unconditional chain vs the reference: per pass <= 1% of pixels
# outside the tolerance, and the relative L2 error of the mean over the passes
# <= 1e-3.  restir_mis_demo is nearly black (mean radiance 6e-5: 0.02-radius
# lights in a closed box); there two to five pixels whose ulp-level flips move
# them by ~1e-4 absolute dominate the relative L2 (3.5e-3 measured), so its
# bound is on the absolute L2 of that mean instead (<= 1e-3 per pixel, RMS).
CHAIN_REL_L2 = {"c3_outdoor_restir": 1e-3, "anim_restir_demo": 1e-3, "c5_spectral_sphere": 1e-3}


@pytest.mark.parametrize("name", ["c3_outdoor_restir", "restir_mis_demo", "anim_restir_demo", "c5_spectral_sphere"])
def test_oracle_restir_chain_matches_reference(name, cfgs):
    """The restatement's own 6-pass ReSTIR swap chain (index.js:795-820), with
    the executor model, against the reference's chained passes."""
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    F, H, W = G["samples"].shape[:3]
    o = O.Oracle(cfg, cfgs, width=W, height=H, overrides={"SWIFTSHADER_GHOST": 1})
    S, M, A = o.frames_restir(F, cfg)
    if cfg.get("time_ms"):  # RENDER_MODE 1 fixture passes are mix(0, sample, 1/u_temporalFrames)
        S = S / np.float32(cfg.get("temporal_frames", 5))
    ok_all = np.ones((H, W), bool)
    for k in range(F):
        ok, _ = pixel_match(S[k][..., :3], G["samples"][k][..., :3])
        ok_all &= ok
        assert 1.0 - ok.mean() <= 0.01, (name, k + 1, 1.0 - ok.mean())
        okr = _res_match(M[k], G["restir_main"][k]) & _res_match(A[k], G["restir_aux"][k])
        assert 1.0 - okr.mean() <= 0.01, (name, k + 1, "reservoirs", 1.0 - okr.mean())
    m, g = S[..., :3].mean(0), G["samples"][..., :3].mean(0)
    if name in CHAIN_REL_L2:  # the restatement has no flipped pixels to exclude here: full image
        assert np.linalg.norm(m - g) / np.linalg.norm(g) <= CHAIN_REL_L2[name]
    else:
        assert np.sqrt(np.mean((m - g) ** 2)) <= 1e-3


def test_oracle_accumulation_is_sequential_sum(cfgs):
    cfg = cfgs["configs"][0]
    o = O.Oracle(cfg, cfgs, width=16, height=16)
    acc = o.accumulate(1, 3)
    ref = np.zeros_like(acc)
    for k in range(1, 4):
        ref[..., :3] += o.frame(k)[0][..., :3]
    assert np.array_equal(acc[..., :3], ref[..., :3])


def test_tex_filter_kat_bitexact():
    """The executor's RGBA8 GL_LINEAR + GL_REPEAT filter (oracle/gen/tex_kat.py:
    known-answer shaders run by the reference's executor) restated as
    tex_fetch_ss (oracle/rt0_oracle.c; the product's tex_rgba8_ss under
    rt0_set_executor_compat): bit-exact on every power-of-two case -- 2x1
    ramps and constants, 1x2, off the 1/4096 grid, one-hot 2x2 taps, wrapped
    coordinates on 64-, 256- and 512-wide textures (the reference's assets
    are 256^2 and 512^2).  On the 53x37 texture 6 of 4096 samples next to a
    texel boundary differ by <= 22 / 65535 (not modelled: no asset is NPOT)."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(os.path.dirname(O.__file__), "librt0_oracle.so"))
    fn = lib.tex_fetch_ss
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                   ctypes.POINTER(ctypes.c_float)]
    K = np.load(os.path.join(GOLD, "tex_filter_kat.npz"))
    out = (ctypes.c_float * 4)()
    for k, name in enumerate(K["names"]):
        tex = np.ascontiguousarray(K["tex_%d" % k])
        uv, n = K["uv_%d" % k], K["n_%d" % k]
        want = n.astype(np.float32) * np.float32(1.0 / 65535.0)  # the executor's readback
        got = np.empty((len(uv), 4), np.float32)
        for i in range(len(uv)):
            fn(tex.ctypes.data, tex.shape[1], tex.shape[0], float(uv[i, 0]), float(uv[i, 1]), out)
            got[i] = out[:]
        if str(name).startswith("npot"):
            bad = (got != want).any(1)
            assert bad.sum() <= 8 and np.abs(got - want).max() <= 24 / 65535.0, (name, bad.sum())
        else:
            assert np.array_equal(got, want), (name, int((got != want).any(1).sum()))


# The executor's texture filter (SWIFTSHADER_TEX_FILTER, the default of the
# restatement and of the product since round 6) against exact fp32 bilinear,
# bad-pixel fractions on the asset fixtures (measured): page_scene0_slabfirst
# 6.3% vs 24.2%, page_scene1 0.59% vs 1.7%, tex_check_assets 0.04% vs 0.49%,
# tex_check_test 0.01% vs 0.12%.  The METAL fixtures on the synthetic noise
# texture do not move (tex_sdf_metal 3.5%, cube_sdf_metal 6.2%).
# name: (bound with the fixed-point filter, at least this much worse in fp32)
TEX_FILTER_BAD = {"page_scene0_slabfirst": (0.07, 0.15), "page_scene1": (0.008, 0.01),
                  "tex_check_assets": (0.001, 0.003), "tex_check_test": (0.001, 0.0008)}


@pytest.mark.parametrize("name", sorted(TEX_FILTER_BAD))
def test_oracle_texture_filter_fixed_vs_float(name, cfgs):
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    frames = G["frames"] if "frames" in G else range(1, gold.shape[0] + 1)
    valid = G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    bad = []
    for tf in (1, 0):
        o = O.Oracle(cfg, cfgs, width=gold.shape[2], height=gold.shape[1],
                     overrides={"SWIFTSHADER_GHOST": 1, "SWIFTSHADER_TEX_FILTER": tf})
        got = np.stack([o.frame(int(k))[0] for k in frames])[..., :3]
        ok, _ = pixel_match(got, gold)
        bad.append(1.0 - ok[valid].mean())
    fixed_bound, float_worse = TEX_FILTER_BAD[name]
    assert bad[0] <= fixed_bound, (name, bad)
    assert bad[1] - bad[0] >= float_worse * 0.9, (name, bad)


def test_cubemap_corner_kat():
    """The executor's seamless cubemap filter (GL_LINEAR on RGB8 faces,
    oracle/gen/tex_kat.py): float bilinear across face edges, and a corner
    footprint's missing texel as the average of the three that meet there
    (oracle cube_sample; the product's cube_sample the same).  Directions
    spread over the sphere and next to the +Z/+X edge and its corners: every
    sample within 5e-4 (the executor's own rounding of the filter)."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(os.path.dirname(O.__file__), "librt0_oracle.so"))
    fn = lib.or_cube_probe
    fn.restype = None
    K = np.load(os.path.join(GOLD, "tex_filter_kat.npz"))
    faces = [np.ascontiguousarray(K["cube_faces"][i]) for i in range(6)]
    ptrs = (ctypes.c_void_p * 6)(*[f.ctypes.data for f in faces])
    out = (ctypes.c_float * 3)()
    for tag in ("spread", "edge"):
        dirs, want = K["cube_dir_" + tag], K["cube_rgb_" + tag]
        got = np.empty_like(want)
        for i, d in enumerate(dirs):
            dd = np.ascontiguousarray(d, np.float32)
            fn(ptrs, faces[0].shape[0], dd.ctypes.data_as(ctypes.c_void_p), out)
            got[i] = out[:]
        err = np.abs(got - want).max()
        assert err <= 5e-4, (tag, float(err))


# Two lights: brdf's surface light loop (raytracer.glsl:1955-1974) reads
# light_index[i] at the index register of the 2x2 quad's first lane
# (SWIFTSHADER_QUAD_LIGHTS, mask_kat.py rule 11, test_mask_kat_quad_lights).
# Measured bad-pixel fractions per quad lane (first | the other three), GLSL
# semantics -> the model: spectral_2l_novol (the KATs' model, no fitting)
# 0.02% | 8.5-8.8% -> 0.11% overall; spectral_vol_2l (the stale value and
# the ghost refresh under the medium's `continue` fitted here) 0% | 25-27% ->
# 0% | 4.1-4.9%, 3.4% overall.  One-light fixtures are unchanged by the
# model (a one-trip loop reads its one element).
QUAD_LIGHTS = {"spectral_vol_2l": (0.04, 0.01), "spectral_2l_novol": (0.003, 2e-3)}


def _two_light(name, cfgs, quad_lights):
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold = G["samples"][..., :3]
    frames = G["frames"] if "frames" in G else range(1, gold.shape[0] + 1)
    o = O.Oracle(cfg, cfgs, width=gold.shape[2], height=gold.shape[1],
                 overrides={"SWIFTSHADER_GHOST": 1, "SWIFTSHADER_QUAD_LIGHTS": quad_lights})
    got = np.stack([o.frame(int(k))[0] for k in frames])[..., :3]
    valid = G["conformant"] if "conformant" in G else G["valid"] if "valid" in G else np.ones(gold.shape[:3], bool)
    ok, _ = pixel_match(got, gold)
    return got, gold, valid, ok


@pytest.mark.parametrize("name", sorted(QUAD_LIGHTS))
def test_two_light_quad_first_lane_is_glsl(name, cfgs):
    """Under GLSL semantics the quad's first lane matches the reference (it is
    the lane whose index register the loop reads) and the other three depart
    -- a quad-coupled executor effect, not a restatement error."""
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    _, _, valid, ok = _two_light(name, cfgs, 0)
    first = valid[:, 0::2, 0::2]
    assert 1.0 - ok[:, 0::2, 0::2][first].mean() <= 0.002
    for ly, lx in ((0, 1), (1, 0), (1, 1)):
        m = valid[:, ly::2, lx::2]
        assert 1.0 - ok[:, ly::2, lx::2][m].mean() >= 0.05, (ly, lx)


@pytest.mark.parametrize("name", sorted(QUAD_LIGHTS))
def test_two_light_executor_quad_lights(name, cfgs):
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    got, gold, valid, ok = _two_light(name, cfgs, 1)
    bound, mean_tol = QUAD_LIGHTS[name]
    bad = 1.0 - ok[valid].mean()
    assert bad <= bound, (name, bad)
    assert abs(got[valid].mean() - gold[valid].mean()) <= mean_tol * max(1.0, abs(gold[valid].mean()))


# First divergent event of every departing pixel of the glossy METAL scenes
# (make_golden.py instrument_events, the restatement's RT0_DEBUG_EVENTS),
# measured (bad pixel-samples of 16 384; round 6):
#   tex_sdf_metal           573: march decisions 401, first-hit normal 171, noise 1
#   cube_sdf_metal         1007: march 751 (with the environment-NEE shadow
#                          rays), normal 250, noise 1, no recorded event 5
#   page_scene0_slabfirst  1035: march 822, normal 195, noise 5, the first
#                          miss's cube sample 4, no recorded event 9
# So the departures are the SDF marches' decisions (hit or miss, which box)
# and calcNormal's four-probe normal, both chaotic under ulp-level map()
# differences -- not the textures' filters: the noise fetch, the cube fetch
# and everything no event records explain at most 0.15% of the pixels.
METAL_EVENTS = ["tex_sdf_metal", "cube_sdf_metal", "page_scene0_slabfirst"]


def _first_divergence(e, r):
    """The first event at which the executor's record e departs from the
    restatement's r (instrument_events' layout)."""
    de, dr = int(e[6]), int(r[6])
    if (de & 3) != (dr & 3):
        return "march"  # the camera ray: hit or miss, which SDF
    if abs(e[1] - r[1]) > 1e-5:
        return "noise"  # the first hit's METAL value noise
    if (np.abs(e[2:5] - r[2:5]) > 1e-4).any():
        return "normal"  # the first bounce's direction: calcNormal + the glossy reflection
    for d in range(6):
        if ((de >> (2 * d)) & 3) != ((dr >> (2 * d)) & 3):
            return "march"  # bounce d's ray
        if ((de >> (12 + d)) & 1) != ((dr >> (12 + d)) & 1):
            return "march"  # bounce d's environment-NEE shadow ray (escaped or not)
    if abs(e[7] - r[7]) > 1e-3:
        return "env"  # the first miss's environment sample
    return "same"  # every recorded event equal


@pytest.mark.parametrize("name", METAL_EVENTS)
def test_metal_departures_attributed(name, cfgs):
    if not have(name):
        pytest.skip("fixture %s not generated" % name)
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    G = np.load(os.path.join(GOLD, name + ".npz"))
    gold, E, ev_ok = G["samples"][..., :3], G["exec_events"], G["events_valid"]
    assert ev_ok.all()  # the instrumented image equals the plain one everywhere
    o = O.Oracle(cfg, cfgs, width=gold.shape[2], height=gold.shape[1],
                 overrides={"SWIFTSHADER_GHOST": 1, "RT0_DEBUG_EVENTS": 1})
    S, R = [], []
    for k in range(1, gold.shape[0] + 1):
        s, m, a = o.frame(k)
        S.append(s[..., :3])
        R.append(np.concatenate([m, a], -1))
    S, R = np.stack(S), np.stack(R)
    ok, _ = pixel_match(S, gold)
    bad = ~ok
    kinds = {}
    for f, y, x in zip(*np.nonzero(bad)):
        k = _first_divergence(E[f, y, x], R[f, y, x])
        kinds[k] = kinds.get(k, 0) + 1
    n = bad.size
    print(name, "bad %.4f" % bad.mean(), kinds)
    assert sum(kinds.values()) == int(bad.sum())
    # the filters (noise texture, cubemap) and anything no event explains
    assert kinds.get("noise", 0) + kinds.get("env", 0) + kinds.get("same", 0) <= 0.0015 * n, kinds
    # the march decisions and the first-hit normal are the departures
    assert kinds.get("march", 0) + kinds.get("normal", 0) >= bad.sum() - 0.0015 * n
    # and they are rare where the image agrees: the executor's decisions equal
    # the restatement's on >= 98% of the matching pixel-samples
    same_dec = E[..., 6] == R[..., 6]
    assert same_dec[ok].mean() >= 0.98
