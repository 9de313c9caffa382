#!/usr/bin/env python3
"""Per-workload roofline table from the files scripts/gpu_measure.sh writes
(profiles/r03/: bench_<c>.json, kt_<c>.json, prof_<c>.json, pmc_<c>.json,
calib.json, valu_peak.json).

    python3 scripts/roofline_summary.py profiles/r03 > profiles/r03/roofline.md

For every workload:
  * kernel time: the MEDIAN rocprofv3 duration of rt0_jit_pass over the timed
    steps of a profiled bench run (warm-up launches dropped: kt_summary.py),
    cross-checked against that run's own ms_per_step (kernel ms x launches per
    step must not exceed it) and against the plain run's HIP-event time;
  * achieved = FLOP/sample (bench.py: SURVEY 8d model x counted events of the
    timed frame window) x samples per launch / median kernel time; frac against
    the 157.3 TF spec (packed v_pk_fma_f32) and against the MEASURED scalar
    v_fma_f32 peak of scripts/valu_peak (the compiler emits scalar FMA for this
    kernel: -fno-slp-vectorize);
  * VALU busy: the kernel's wave64 VALU instructions at the MEASURED issue
    time of their class (scripts/valu_peak: non-transcendental = the mean of
    v_add/v_mul/v_fma rates, transcendental = v_exp_f32's), per SIMD, over the
    median kernel time -- the share of time the VALU pipe is occupied;
  * HBM traffic: bench.py's hbm_traffic -- FETCH_SIZE x 1024 B x the
    calibrated factor of the access shape (scripts/fetch_calib: 16-B/lane
    stream x2, 64-B gathers x1, bilinear 2x2 RGBA32F taps x0.5) + WRITE_SIZE;
    a kernel that mixes shapes gets its accumulator stream at x2 and the rest
    at the factor of its dominant shape, with the x0.5 .. x2 range beside it;
    over the median kernel time -> GB/s and the fraction of 8 TB/s;
  * clocks: the GPU clock bench.py sampled during the profiled run (its
    gpu_clock, pp_dpm_sclk) and during the plain run the driver-style line
    comes from, and the frac the kernel reaches at the plain run's clock
    (the profiled median scaled by the clock ratio: these kernels are
    issue-bound, their time follows the shader clock).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import hbm_traffic  # noqa: E402

PEAK_SPEC = 157.3
D = sys.argv[1]


def load(name):
    p = os.path.join(D, name)
    return json.load(open(p)) if os.path.exists(p) else None


calib = load("calib.json") or {}
fac = {k: (v["factor"][-1] if v.get("factor") else None) for k, v in calib.items()}
vp, rate = {}, {}
if os.path.exists(os.path.join(D, "valu_peak.json")):
    for line in open(os.path.join(D, "valu_peak.json")):
        if line.startswith("{"):
            d = json.loads(line)
            vp[d["kernel"]] = d.get("tflops")
            rate[d["kernel"]] = d.get("wave_instr_per_simd_per_ns")
PEAK_SCALAR = vp.get("v_fma_f32", 78.6)
NS_NORM = 3.0 / (rate["v_add_f32"] + rate["v_mul_f32"] + rate["v_fma_f32"]) if rate.get("v_add_f32") else None
NS_TRANS = 1.0 / rate["v_exp_f32"] if rate.get("v_exp_f32") else None

rows = []
for c in ("c1", "c2", "c3", "c4", "c5"):
    b, kt, pr, pmc = load("bench_%s.json" % c), load("kt_%s.json" % c), load("prof_%s.json" % c), load("pmc_%s.json" % c)
    if not (b and kt):
        continue
    R = b["roofline"]
    cfg = b["config"]
    lps = R["launches_per_step"]
    pixels = cfg["width"] * cfg["height"]
    spl = pixels * cfg["spp"] / lps  # samples per launch
    med = kt["median_ms"]
    ach = R["flop_per_sample"] * spl / (med * 1e-3) / 1e12
    row = dict(config=c, msamples_s=b["value"], ms_per_step=b["ms_per_step"], flop_per_sample=R["flop_per_sample"],
               launches_per_step=lps, rocprof_median_ms=med, rocprof_min_ms=kt["min_ms"], rocprof_max_ms=kt["max_ms"],
               hip_event_ms=R["kernel_ms_per_launch"], achieved_tflops=ach, frac_spec=ach / PEAK_SPEC,
               frac_scalar=ach / PEAK_SCALAR, bench_frac=R["frac"])
    clk_b = (b.get("gpu_clock") or {}).get("median_mhz")
    clk_p = ((pr or {}).get("gpu_clock") or {}).get("median_mhz")
    row["bench_clock_mhz"], row["profiled_clock_mhz"] = clk_b, clk_p
    row["frac_spec_at_bench_clock"] = ach * clk_b / clk_p / PEAK_SPEC if clk_b and clk_p else None
    if pr:
        row["profiled_ms_per_step"] = pr["ms_per_step"]
        # the trace median covers every kept dispatch (warm-up steps included), ms_per_step only the timed ones:
        # allow 1% run-to-run jitter between the two windows
        row["check_kernel_x_launches_le_step"] = med * lps <= pr["ms_per_step"] * 1.01
    if pmc:
        clk = pmc.get("clock_ghz_median")
        row["clock_ghz"] = clk
        v = pmc.get("valu", {})
        if v and NS_NORM:
            ns = (v["SQ_INSTS_VALU"] - v["SQ_INSTS_VALU_TRANS_F32"]) * NS_NORM + v["SQ_INSTS_VALU_TRANS_F32"] * NS_TRANS
            row["valu_busy"] = ns / 1024.0 / (med * 1e6)
        row["lane_util"] = pmc.get("valu_lane_utilisation")
        row["stall_share"] = pmc.get("stall_share")
        cnt = pmc.get("counters", {})
        if "FETCH_SIZE" in cnt and "WRITE_SIZE" in cnt:
            fetch, write = cnt["FETCH_SIZE"] * 1024.0, cnt["WRITE_SIZE"] * 1024.0
            est, lo, hi = hbm_traffic(pmc, c, pixels, fac)  # the bench line's own correction
            row.update(fetch_counter_bytes=fetch, write_bytes=write, traffic_est=est, traffic_lo=lo, traffic_hi=hi,
                       hbm_gbs=est / (med * 1e-3) / 1e9, hbm_frac=est / (med * 1e-3) / 8e12,
                       algorithmic_bytes=pmc.get("algorithmic_bytes_per_launch"))
        if pmc.get("valu_mix"):
            row["valu_mix"] = pmc["valu_mix"]
    rows.append(row)
json.dump({"rows": rows, "calibration": fac, "valu_peak_tflops": vp}, open(os.path.join(D, "roofline.json"), "w"),
          indent=1)


def f(x, fmt="%.3f"):
    return "-" if x is None else fmt % x


print("Measured peaks: scalar v_fma_f32 %s TF, packed v_pk_fma_f32 %s TF (scripts/valu_peak.hip; spec 157.3)."
      % (f(vp.get("v_fma_f32"), "%.1f"), f(vp.get("v_pk_fma_f32"), "%.1f")))
print("FETCH_SIZE calibration, true bytes / counter bytes (scripts/fetch_calib.hip): %s." %
      ", ".join("%s x%s" % (k, v) for k, v in fac.items()))
print()
print("| config | Msamples/s | FLOP/sample | kernel ms/launch: rocprof median (min-max) / HIP events | launches x median <= "
      "ms_per_step (profiled run, 1% jitter) | TFLOP/s | frac of 157.3 | frac of scalar peak | clock GHz | VALU busy | "
      "lane util | HBM bytes/launch est. (range) / algorithmic | GB/s | frac of 8 TB/s | clock MHz profiled / "
      "plain run | frac of 157.3 at the plain run's clock |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
for r in rows:
    chk = r.get("check_kernel_x_launches_le_step")
    print("| %s | %.0f | %.0f | %.3f (%.3f-%.3f) / %.3f | %s %s | %.1f | %.3f | %.3f | %s | %s | %s | %s (%s-%s) / %s | %s | %s | %s / %s | %s |" % (
        r["config"], r["msamples_s"], r["flop_per_sample"], r["rocprof_median_ms"], r["rocprof_min_ms"],
        r["rocprof_max_ms"], r["hip_event_ms"],
        "%.2f x %d = %.2f <= %.2f" % (r["rocprof_median_ms"], r["launches_per_step"],
                                      r["rocprof_median_ms"] * r["launches_per_step"], r.get("profiled_ms_per_step", 0)),
        "ok" if chk else ("VIOLATED" if chk is not None else "-"),
        r["achieved_tflops"], r["frac_spec"], r["frac_scalar"], f(r.get("clock_ghz"), "%.2f"),
        f(r.get("valu_busy"), "%.2f"), f(r.get("lane_util"), "%.2f"), f(r.get("traffic_est"), "%.3g"),
        f(r.get("traffic_lo"), "%.3g"), f(r.get("traffic_hi"), "%.3g"), f(r.get("algorithmic_bytes"), "%.3g"),
        f(r.get("hbm_gbs"), "%.0f"), f(r.get("hbm_frac"), "%.3f"), f(r.get("profiled_clock_mhz"), "%.0f"),
        f(r.get("bench_clock_mhz"), "%.0f"), f(r.get("frac_spec_at_bench_clock"), "%.3f")))
