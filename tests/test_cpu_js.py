"""The JS CPU integrator (oracle/js/rt0_cpu.js) -- the reported CPU baseline
of bench.py, SURVEY 8d -- renders what the reference renders: checked against
the golden fixtures (the reference shader under SwiftShader) and the C oracle
on the configs it covers (quadrics, SDFs, volumetrics).  CPU only."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "oracle", "js", "cpu_bench.js")
CONFIGS = os.path.join(REPO, "tests", "golden", "configs.json")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is missing")


def js_image(name, w, h, frame0, n, tmp_path, threads=4):
    out = tmp_path / ("%s.f32" % name)
    r = subprocess.run([NODE, BENCH, CONFIGS, name, str(w), str(h), str(threads), "image", str(frame0), str(n),
                        str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return np.fromfile(str(out), np.float32).reshape(h, w, 4)


def match(a, b):
    return ((np.abs(a[..., :3] - b[..., :3]) <= 1e-3 * np.maximum(1.0, np.abs(b[..., :3]))).all(-1)).mean()


@pytest.mark.parametrize("name", ["c1_cornell_cos", "c2_cornell_mis_refcaps", "c2_cornell_mis_8", "cornell_nee_plain",
                                  "thinlens_glass", "menger_coat", "sdf_cone", "sdf_triprism", "mis_demo_sdfbox"])
def test_js_integrator_matches_reference_fixtures(name, cfgs, tmp_path):
    gold = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))["samples"]
    F, H, W = gold.shape[:3]
    for k in (1, F):
        got = js_image(name, W, H, k, 1, tmp_path)
        # SDF scenes: every path grazes many edges (the oracle's own allowance, test_oracle_golden.BAD_FRAC)
        assert match(got, gold[k - 1]) >= (0.98 if name == "menger_coat" else 0.99), (name, k)


def test_js_integrator_matches_c_oracle_accumulated(cfgs, tmp_path):
    cfg = [c for c in cfgs["configs"] if c["name"] == "c2_cornell_mis_8"][0]
    o = O.Oracle(cfg, cfgs, width=48, height=40)
    ref = sum(o.frame(k)[0] for k in (1, 2, 3))
    got = js_image("c2_cornell_mis_8", 48, 40, 1, 3, tmp_path)
    assert match(got, ref) >= 0.99
    assert abs(got[..., :3].mean() - ref[..., :3].mean()) <= 1e-3 * ref[..., :3].mean()


@pytest.mark.parametrize("name", ["c4_mandelbulb_vol", "vol_cornell_2"])
def test_js_integrator_matches_c_oracle_sdf_volumetrics(name, cfgs, tmp_path):
    """C4's feature set (Mandelbulb SDF, homogeneous medium, in-scatter NEE):
    the JS baseline against the C restatement, single-sample frames."""
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    o = O.Oracle(cfg, cfgs, width=24, height=24)
    for k in (1, 2):
        ref = o.frame(k)[0]
        got = js_image(name, 24, 24, k, 1, tmp_path)
        assert match(got, ref) >= 0.99, (name, k)


def test_js_bench_mode_reports_throughput():
    r = subprocess.run([NODE, BENCH, CONFIGS, "c1_cornell_cos", "256", "256", "2", "bench", "0", "8", "0.5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["samples"] > 0 and d["msamples_s"] > 0 and d["threads"] == 2


def test_js_integrator_rejects_features_outside_its_scope(tmp_path):
    r = subprocess.run([NODE, BENCH, CONFIGS, "c3_outdoor_restir", "16", "16", "1", "image", "1", "1",
                        str(tmp_path / "x.f32")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "outside the JS baseline" in r.stderr
