"""bench.py's measurement model on CPU: the FLOP model's terms, the HBM
traffic correction by access shape, the measured VALU rates and the committed
profiles it reads."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_isect_flop_cornell_is_survey_figure():
    wl = json.load(open(os.path.join(REPO, "raytracer-0_amd", "rt0", "workloads.json")))["workloads"]["c2"]
    assert bench.isect_flop(wl["scene_lines"]) == 151.0  # 150


def test_hbm_traffic_by_access_shape():
    pmc = {"counters": {"FETCH_SIZE": 1000.0, "WRITE_SIZE": 300.0}}  # KiB
    fetch, write = 1000.0 * 1024, 300.0 * 1024
    est, lo, hi = bench.hbm_traffic(pmc, "c2", 1000, {})
    assert est == lo == hi == 2.0 * fetch + write  # streams only: FETCH_SIZE x2
    calib = {"k_bilin": 0.5, "k_node64": 0.99}
    acc = 16.0 * 1000
    rest = fetch - acc / 2.0
    est, lo, hi = bench.hbm_traffic(pmc, "c3", 1000, calib)
    assert est == pytest.approx(acc + 0.5 * rest + write)
    assert lo <= est <= hi and hi == pytest.approx(acc + 2.0 * rest + write)
    est5, _, _ = bench.hbm_traffic(pmc, "c5", 1000, calib)
    assert est5 == pytest.approx(acc + 0.99 * rest + write)


def test_committed_profiles_feed_the_bench_line():
    """The files the bench line cites exist and hold what it reads."""
    rates = bench.valu_rates()
    assert rates is not None, "profiles/<round>/valu_peak.json missing"
    ns_valu, ns_trans, src = rates
    assert 0.5 < ns_valu < 2.0 and ns_trans > 2.0 * ns_valu, (ns_valu, ns_trans)  # transcendentals are slow
    calib, csrc = bench.calibration()
    assert csrc and abs(calib["k_stream"] - 2.0) < 0.05
    for c in ("c1", "c2", "c3", "c4", "c5"):
        path, pmc = bench.pmc_summary(c)
        assert pmc is not None, c
        assert {"FETCH_SIZE", "WRITE_SIZE"} <= set(pmc["counters"]), c
        assert pmc["valu"]["SQ_INSTS_VALU"] > pmc["valu"]["SQ_INSTS_VALU_TRANS_F32"] > 0, c


@pytest.mark.parametrize("rd", ["r03", "r04", "r05", "r06"])
def test_roofline_summary_reproduces_committed_table(rd):
    """profiles/<round>/roofline.md is what scripts/roofline_summary.py computes
    from the committed per-workload files (no hand edits)."""
    import subprocess
    d = os.path.join(REPO, "profiles", rd)
    out = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "roofline_summary.py"), d],
                         capture_output=True, text=True, check=True).stdout
    assert out == open(os.path.join(d, "roofline.md")).read()


def test_clock_sampler_reads_the_starred_level(tmp_path):
    """bench.ClockSampler (the bench line's gpu_clock): the starred line of an
    amdgpu pp_dpm_sclk file is the current level; a sampler with no file
    reports why instead of a clock."""
    f = tmp_path / "pp_dpm_sclk"
    f.write_text("0: 500Mhz\n1: 1900Mhz *\n2: 2400Mhz\n")
    s = bench.ClockSampler.__new__(bench.ClockSampler)
    s.path, s.err, s.mhz, s._stop, s._th = str(f), None, [], None, None
    s.start()
    f.write_text("0: 500Mhz\n1: 1900Mhz\n2: 2400Mhz *\n")
    s.stop()
    rep = s.report()
    assert rep["min_mhz"] == 1900.0 and rep["max_mhz"] == 2400.0 and rep["samples"] >= 2
    none = bench.ClockSampler.__new__(bench.ClockSampler)
    none.path, none.err, none.mhz, none._stop, none._th = None, "no pp_dpm_sclk for PCI 0000:05", [], None, None
    none.start()
    none.stop()
    assert none.report() == {"median_mhz": None, "source": None, "error": "no pp_dpm_sclk for PCI 0000:05"}


def test_kt_summary_wavefront_launch_is_its_span(tmp_path):
    """scripts/kt_summary.py on a synthetic kernel trace of two wavefront
    launches whose halves overlap on two streams: a launch's time is its span
    (first dispatch start -> rt0_sum_kernel end), not the sum of its kernels'
    durations; the warm-up launch is skipped."""
    import csv
    import json
    import subprocess
    rows = []

    def k(name, t0, t1):
        rows.append({"Kernel_Name": name, "Start_Timestamp": str(int(t0 * 1e6)), "End_Timestamp": str(int(t1 * 1e6))})

    for base in (0.0, 100.0):  # two launches, ms
        # two halves: shade/plan/march overlapping pairwise
        for h in (0.0, 0.5):
            k("rt0_jit_wf_shade", base + h, base + h + 2.0)
            k("rt0_jit_wf_plan", base + h + 2.0, base + h + 2.1)
            k("rt0_jit_wf_march", base + h + 2.1, base + h + 6.0)
        k("rt0_jit_wf_shade", base + 6.5, base + 7.0)
        k("rt0_jit_wf_shade", base + 6.6, base + 7.1)
        k("rt0_sum_kernel<>", base + 7.1, base + 7.2)
    d = tmp_path / "trace"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "kt.json"
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "kt_summary.py"), str(out), str(d), "1"],
                   check=True, capture_output=True)
    res = json.load(open(out))
    assert res["kept"] == 1 and res["median_ms"] == pytest.approx(7.2, abs=1e-6)
    # the per-kernel busy sums still count both halves
    assert res["per_kernel_median_ms"]["rt0_jit_wf_march"] == pytest.approx(7.8, abs=1e-6)


def test_kt_summary_split_restir_pass_is_its_span(tmp_path):
    """scripts/kt_summary.py with HALVES=3 on a synthetic trace of deferred
    ReSTIR passes split into three row parts on three streams (rt0_host.cpp
    restir_split_pass): a pass is its three parts' pass/nee/walk/resolve
    dispatches, its time their span; per kernel the parts' busy time summed;
    the warm-up pass is skipped."""
    import csv
    import json
    import subprocess
    rows = []

    def k(name, t0, t1):
        rows.append({"Kernel_Name": name, "Start_Timestamp": str(int(t0 * 1e6)), "End_Timestamp": str(int(t1 * 1e6))})

    for base in (0.0, 10.0, 20.0):  # three passes, ms; parts start 0.2 ms apart and overlap
        for h in range(3):
            t = base + 0.2 * h
            k("rt0_jit_pass", t, t + 3.0)
            k("rt0_jit_nee", t + 3.0, t + 5.0)
            k("rt0_jit_walk", t + 5.0, t + 6.0)
            k("rt0_jit_resolve", t + 6.0, t + 6.5)
    d = tmp_path / "trace"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "kt.json"
    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "kt_summary.py"), str(out), str(d), "1"],
                   check=True, capture_output=True, env=dict(os.environ, HALVES="3"))
    res = json.load(open(out))
    assert res["kept"] == 2 and res["median_ms"] == pytest.approx(6.9, abs=1e-6)
    assert res["per_kernel_median_ms"]["rt0_jit_pass"] == pytest.approx(9.0, abs=1e-6)
    assert res["per_kernel_median_ms"]["dispatches_per_pass"]["rt0_jit_resolve"] == 3
