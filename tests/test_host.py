"""Host-side logic on CPU: the C-ABI library loads and exports include/rt0.h,
the defines/constants/scene parsers reproduce the reference's grammar, and the
Python GlslViewport surface mirrors index.js.  No compute calls (no GPU here).
"""
import ctypes
import os
import re

import numpy as np
import pytest

import rt0

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(REPO, "include", "rt0.h")).read()
    return sorted(set(re.findall(r"\b(rt0_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = rt0.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(rt0.EXPORTS) == syms
    assert b"gfx950" in L.rt0_version()


def test_create_fails_loudly_without_gpu_or_bad_args():
    h = ctypes.c_void_p()
    assert rt0.lib().rt0_create(0, 64, 0, ctypes.byref(h)) == -1
    if not os.path.exists("/dev/kfd"):
        with pytest.raises(rt0.Rt0Error):
            rt0.Renderer(64, 64)


def test_parse_config_reference_defaults():
    vp_defines = ["//#define USE_CUBEMAP", "#define USE_PROCEDURAL_SKY", "#define USE_BIASED_SAMPLING",
                  "//#define USE_BIDIRECTIONAL", "//#define USE_RESTIR", "//#define USE_SPECTRAL",
                  "//#define USE_VOLUMETRICS"]
    cfg = rt0.parse_config(vp_defines, rt0.STATIC_CONSTANTS)
    assert cfg.defines == (1 << 1) | (1 << 2)
    assert (cfg.max_bounces, cfg.max_diff_bounces, cfg.max_spec_bounces, cfg.max_trans_bounces) == (12, 4, 4, 12)
    assert (cfg.max_scattering_events, cfg.marching_steps) == (12, 128)
    assert abs(cfg.fudge_factor - 0.9) < 1e-7
    assert (cfg.sample_lights, cfg.use_mis, cfg.use_restir, cfg.restir_samples, cfg.render_mode) == (1, 0, 0, 16, 0)
    anim = rt0.parse_config(vp_defines, rt0.ANIMATED_CONSTANTS)
    assert (anim.max_bounces, anim.use_restir, anim.render_mode, anim.marching_steps) == (6, 1, 1, 64)


def test_parse_config_rejects_garbage():
    with pytest.raises(rt0.Rt0Error):
        rt0.parse_config(["#define USE_NOTHING"], [])
    with pytest.raises(rt0.Rt0Error):
        rt0.parse_config([], ["const lowp int NOT_A_CONSTANT = 3;"])


def test_scene_parser_cornell(cfgs):
    scene, ns = rt0.scene_from_lines(cfgs["cornell_lines"])
    meshes, ne, nsdf, lights = rt0.parse_scene(scene, [])
    assert (ne, nsdf, lights) == (8, 0, [5])
    types = [m.type for m in meshes]
    assert types == [1, 1, 1, 1, 1, 0, 2, 2]
    assert list(meshes[5].e) == [4.0, 4.0, 4.0] and meshes[5].mat_type == 0
    assert np.allclose(list(meshes[3].c), [0.7, 0.12, 0.05])
    assert np.allclose(list(meshes[7].pos), [-0.45, -1.15, -1.3]) and meshes[7].joker[0] == np.float32(0.7)


def test_scene_parser_handles_reference_comments_and_broadcast():
    text = """// header comment
const bool U_EUCLIDEAN = true;
const Mesh meshes[NUM_MESHES + NUM_SDFS + NUM_MODELS] = Mesh[](
    // Floor  (y = -1.5, normal up)
    Mesh(MAT_CORNELL_WHITE, PLANE,  vec3( 0.0, 1.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)),
    /* a light */ Mesh(MAT_LIGHT_4, SPHERE, vec3(0.0), vec4(0.3))
);
const lowp int light_index[1] = int[](1);"""
    meshes, ne, ns, lights = rt0.parse_scene(text)
    assert (ne, ns, lights) == (2, 0, [1])
    assert list(meshes[1].pos) == [0.0, 0.0, 0.0] and list(meshes[1].joker) == [np.float32(0.3)] * 4


def test_scene_parser_sdf_statements(cfgs):
    cfg = [c for c in cfgs["configs"] if c["name"] == "c4_mandelbulb_vol"][0]
    scene, ns = rt0.scene_from_lines(cfg["scene_lines"])
    stm = [rt0.sdf_statement(i, cfg["sdf_kinds"][i]) for i in range(ns)]
    assert stm[0] == "sdf_meshes[0] = vec2(Mandelbulb(p-meshes[NUM_MESHES + 0].pos), 0.0000);"
    meshes, ne, nsdf, lights = rt0.parse_scene(scene, stm)
    assert (ne, nsdf, lights) == (7, 1, [6])
    assert meshes[7].type == 3 and meshes[7].sdf_kind == 6
    for kind in range(7):
        m, _, _, _ = rt0.parse_scene(scene, [rt0.sdf_statement(0, kind)])
        assert m[7].sdf_kind == kind


def test_scene_parser_errors():
    with pytest.raises(rt0.Rt0Error):
        rt0.parse_scene("Mesh(MAT_NOPE, PLANE, vec3(0.0), vec4(1.0)) light_index[1] = int[](-1);")
    with pytest.raises(rt0.Rt0Error) as e:  # GRID_SDF has no implementation in the reference integrator
        rt0.parse_scene("Mesh(MAT_WHITE, GRID_SDF, vec3(0.0), vec4(1.0)) light_index[1] = int[](-1);")
    assert e.value.code == -3
    # TRIANGLE entries are models (tests/test_models.py)
    assert rt0.parse_scene("Mesh(MAT_WHITE, TRIANGLE, vec3(0.0), vec4(1.0)) light_index[1] = int[](-1);")[0][0].type == 5
    # SDF mesh without a #sdf_meshes statement
    with pytest.raises(rt0.Rt0Error):
        rt0.parse_scene("Mesh(MAT_WHITE, SDF, vec3(0.0), vec4(1.0)) light_index[1] = int[](-1);", [])


def test_no_lights_gives_minus_one(cfgs):
    cfg = [c for c in cfgs["configs"] if c["name"] == "menger_coat"][0]
    scene, ns = rt0.scene_from_lines(cfg["scene_lines"])
    assert "int[](\n-1\n)" in scene
    _, ne, nsdf, lights = rt0.parse_scene(scene, [rt0.sdf_statement(0, 5)])
    assert (ne, nsdf, lights) == (0, 1, [-1])


def test_glslviewport_surface_matches_reference_fields():
    # the fields index.html reads/writes on `sandbox` (index.html:498-1196)
    for name in ("render", "clear", "resize", "setAnimatedMode", "updateFrontTarget"):
        assert callable(getattr(rt0.GlslViewport, name))
    assert len(rt0.STATIC_CONSTANTS) == 13 and len(rt0.ANIMATED_CONSTANTS) == 13


def test_jit_kernels_build_for_every_config(cfgs):
    """The scene-specialised kernel (hipRTC, rt0_jit.cpp) builds for every
    parity config without a device."""
    for cfg in cfgs["configs"]:
        scene, sdf = rt0.scene_strings(cfg, cfgs)
        size = rt0.jit_compile(scene, sdf, rt0.parse_config(*rt0.config_strings(cfg)))
        assert size > 4096, cfg["name"]


def test_bench_workloads_match_the_parity_scenes(cfgs):
    """rt0/workloads.json (read by bench.py, no test imports on the product
    side) describes the same scenes/flags/cameras as the parity fixtures it
    names, up to the documented bench overrides (C4: 12 bounces)."""
    from rt0 import workloads
    by = {c["name"]: c for c in cfgs["configs"]}
    wls = workloads.load_all()
    assert {"c1", "c2", "c3", "c4", "c5"} <= set(wls)
    for key, wl in wls.items():
        cfg = by[wl["fixture"]]
        assert wl["scene_lines"] == (cfg["scene_lines"] or cfgs["cornell_lines"]), key
        assert wl["defines"] == cfg.get("defines", {}), key
        assert wl["camera"] == (cfg.get("camera") or cfgs["default_camera"]), key
        assert wl.get("sdf_kinds", []) == cfg.get("sdf_kinds", []), key
        extra = {k: v for k, v in wl["constants"].items() if cfg.get("constants", {}).get(k) != v}
        assert extra == ({"MAX_BOUNCES": 12} if key == "c4" else {}), (key, extra)
        assert wl.get("models", []) == cfg.get("models", []), key
    assert (wls["c2"]["width"], wls["c2"]["height"], wls["c2"]["spp"]) == (1024, 1024, 64)


def test_bench_flop_model_matches_survey():
    """Cornell intersection() = 150 FLOP; the C2 event counts of
    round 1 (14.64 isect, 7.36 iter, 7.28 nee) give ~4700 FLOP/sample."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from rt0 import workloads
    wl = workloads.get("c2")
    assert bench.isect_flop(wl["scene_lines"]) == 151.0
    fps = bench.flop_per_sample({"samples": 100, "isect": 1464, "iter": 736, "nee": 728, "map": 0}, wl)
    assert 4650 < fps < 4760


def test_jit_walk_module_for_model_scenes(cfgs, tmp_path, monkeypatch):
    """A ReSTIR scene with triangle models gets the occlusion-walk kernel
    (rt0_jit_walk) in its module, and with 16-bit stack entries
    (RT0_BVH_STACK16, the C5 tree's 24-entry stack) the traversal stacks take
    2 B of LDS per entry: 256 x 24 x 2 B per workgroup.  Built with hipRTC,
    no device; rt0_render selects the same key from the built tree.  Runs in
    this process after other compiles, with the environment changed in
    between: hipRTC's private link namespace has its own libc, whose
    `environ` rt0_jit.cpp re-points at every compile (it used to crash here,
    reading the array os.environ had freed)."""
    import glob
    import re
    import subprocess
    cfg = next(c for c in cfgs["configs"] if c["name"] == "c5_spectral_models")
    scene, sdf = rt0.scene_strings(cfg, cfgs)
    rt0.jit_compile(scene, sdf, rt0.parse_config(*rt0.config_strings(cfg)))  # a first compile, default key
    monkeypatch.setenv("RT0_JIT_DUMP", str(tmp_path / "k"))
    monkeypatch.setenv("RT0_BVH_STACK16", "1")
    monkeypatch.setenv("RT0_JIT_STACK", "24")
    for i in range(64):  # grow the environment so its array is reallocated
        monkeypatch.setenv("RT0_TEST_PAD_%d" % i, "x" * 64)

    def compile_lds():
        rt0.jit_compile(scene, sdf, rt0.parse_config(*rt0.config_strings(cfg)))
        co = max(glob.glob(str(tmp_path / "k_*.co")), key=os.path.getmtime)
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                               text=True).stdout
        return co, {m.group(2): int(m.group(1)) for m in
                    re.finditer(r"\.group_segment_fixed_size:\s+(\d+)(?:.|\n)*?\.name:\s+(\S+)", notes)}

    # rt0_set_wavefront(2): wavefront rounds (rt0_jit_wf_shade, _wf_plan, the
    # closest-hit walk rt0_jit_wf_walk), then the deferred-pass kernels
    monkeypatch.setenv("RT0_WAVEFRONT", "2")
    # RT0_JIT_EXTRA: extra hipRTC options (the measurement scripts' probes,
    # scripts/jit_trans_sites.py), recorded in the source and so in the cache key
    monkeypatch.setenv("RT0_JIT_EXTRA", "-DRT0_TEST_EXTRA_OPTION=1")
    co, lds = compile_lds()
    assert "// options: -DRT0_TEST_EXTRA_OPTION=1" in open(co[:-3] + ".hip").read()
    monkeypatch.delenv("RT0_JIT_EXTRA")
    assert {"rt0_jit_wf_shade", "rt0_jit_wf_plan", "rt0_jit_wf_walk", "rt0_jit_nee", "rt0_jit_walk",
            "rt0_jit_resolve"} <= set(lds) and "rt0_jit_pass" not in lds, lds
    # the stack + the LDS treelet (64 BVH nodes of 64 B, rt0_integrator.h bvh_fetch) + the plan prefix
    tl = 64 * 64
    assert 256 * 24 * 2 + tl <= lds["rt0_jit_wf_walk"] <= 256 * 24 * 2 + tl + 2048
    # the default (mode 1: SDF scenes only): the pass kernel
    monkeypatch.setenv("RT0_WAVEFRONT", "1")
    co, lds = compile_lds()
    assert {"rt0_jit_pass", "rt0_jit_nee", "rt0_jit_walk", "rt0_jit_resolve"} <= set(lds), lds
    assert lds["rt0_jit_walk"] == 256 * 24 * 2 + 16 + tl  # the stack + the wave counters + the treelet
    # the pass and light-sampling kernels also hold LDS copies of the scene
    # tables (rt0_integrator.h scene_tables: geometry, material and clamped
    # material, 32 B each per mesh) and the latter the ReSTIR candidates'
    # light table (candidate_table: 32 B per light slot)
    src = open(co[:-3] + ".hip").read()
    k = {n: int(v) for n, v in re.findall(r"\b(kMeshes|kSdfs|kLights|kModels) = (\d+)", src)}
    tables = 96 * (k["kMeshes"] + k["kSdfs"] + k["kModels"])
    assert lds["rt0_jit_pass"] <= 256 * 24 * 2 + 16 + tables + tl
    assert lds["rt0_jit_nee"] == tables + 32 * k["kLights"] + tl  # (+ the treelet its walk code could read)
