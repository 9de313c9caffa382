#!/usr/bin/env python3
"""bench.py -- Msamples/s of the rt0 HIP integrator on BASELINE.json's workload.

Workload (BASELINE.json configs[1], SURVEY 8d "C2"): 1024x1024 Cornell box
(index.js:54-85, camera index.js:89-95), MIS power heuristic on, 8 bounces
(MAX_BOUNCES = MAX_DIFF_BOUNCES = 8: a true 8-bounce path; the reference's
default MAX_DIFF_BOUNCES=4 variant is reported beside it), 64 spp.
One step = one 64-pass progressive render of the whole image (u_frame 1..64,
i.e. 64 GlslViewport.render() calls) with scene + accumulator resident in HBM.

N GPUs (one process per GPU, torch.distributed.run): the image is split into
16-row bands dealt round-robin over ranks (rt0_set_shard); each rank renders
its bands straight into a band-packed torch buffer (rt0_set_accum_buffer_compact:
the RCCL send buffer as it stands), and rank 0 gathers the bands over RCCL and
reorders them with one index_copy_ inside the timed region ("strong" scaling:
total work fixed).

Prints ONE JSON line on rank 0 (contract in the task statement) with
`roofline` (VALU FP32: algorithmic FLOP/sample from SURVEY 8d x counted events,
over the kernel's HIP-event time; HBM traffic from the committed PMC passes)
and `cpu_baseline` (the JS CPU integrator oracle/js/rt0_cpu.js on
node worker_threads, bounded sample of the same workload), with the C
restatement oracle/rt0_oracle.c (OpenMP) beside it as `cpu_baseline_c`.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "raytracer-0_amd"))
sys.path.insert(0, os.path.join(HERE, "oracle"))

import numpy as np  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X vector FP32 (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0
W = H = 1024
SPP = 64
PROFILE_ROUND = "r01"  # profiles/<round>/ holding the PMC summary of this workload


def flop_per_sample(c, mis=True):
    """SURVEY 8d algorithmic FLOP model: 140 + 150*isect + 130*iter + (140+54*mis)*nee per sample."""
    n = max(1, c["samples"])
    return 140.0 + 150.0 * c["isect"] / n + 130.0 * c["iter"] / n + (140.0 + 54.0 * mis) * c["nee"] / n


def host_threads():
    """Host threads the baselines may use: OMP_NUM_THREADS (16 on the GPU box,
    whose os.cpu_count() shows the whole machine), else up to 16."""
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def cpu_baseline_js(cfg_name, budget_s=10.0):
    """SURVEY 8d's CPU baseline: the JS CPU integrator (oracle/js/rt0_cpu.js,
    fp32 restatement of the same integrator, parity-checked in
    tests/test_cpu_js.py) on node worker_threads, timed on a bounded sample of
    the same workload: rows 480..543 of the 1024^2 image, successive passes
    until the time budget."""
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        return None
    threads = host_threads()
    r = subprocess.run([node, os.path.join(HERE, "oracle", "js", "cpu_bench.js"),
                        os.path.join(HERE, "tests", "golden", "configs.json"), cfg_name, str(W), str(H), str(threads),
                        "bench", "480", "544", str(budget_s)], capture_output=True, text=True, timeout=budget_s * 10 + 60)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}
    d = json.loads(r.stdout)
    return {"value": d["msamples_s"], "unit": "Msamples/s", "cores": d["threads"], "kind": "port",
            "sample": "oracle/js/rt0_cpu.js (JS CPU integrator, node %s worker_threads x%d, %s): rows 480..543 of "
                      "the 1024^2 bench image, successive passes, %d samples in %.1f s"
                      % (d["node"], d["threads"], d["cpu"], d["samples"], d["seconds"])}


def cpu_baseline(cfgs, cfg, budget_s=8.0):
    """Time the C restatement (OpenMP, all host threads we are allowed) on a
    bounded sample of the same workload: full-width 1024 rows x a band of rows,
    8-bounce MIS passes, scaled by samples."""
    import oracle as O
    threads = host_threads()
    rows = 64
    o = O.Oracle(cfg, cfgs, width=W, height=H)
    o.frame(1, rows=(480, 480 + 8), threads=threads)  # warm
    n = 0
    t0 = time.time()
    while time.time() - t0 < budget_s:
        o.frame(1 + n, rows=(480, 480 + rows), threads=threads)
        n += 1
    dt = time.time() - t0
    samples = n * rows * W
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "oracle/rt0_oracle.c (OpenMP x%d), rows 480..%d of the 1024^2 bench image, %d passes "
                      "(%d samples, %.1f s)" % (threads, 480 + rows, n, samples, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2_cornell_mis_8")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", action="store_true", help="also time the MAX_DIFF_BOUNCES=4 variant")
    ap.add_argument("--jit", type=int, default=1, help="1: scene-specialised kernels (default), 0: ahead-of-time")
    args = ap.parse_args()

    import torch
    import rt0
    import oracle as O

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL on ROCm
    cfgs = O.load_configs()
    cfg = [c for c in cfgs["configs"] if c["name"] == args.config][0]

    r = rt0.Renderer(W, H, device=local)
    r.set_jit(bool(args.jit))
    rt0.configure(r, cfg, cfgs)
    band = 16
    nb = H // band
    owned = [b for b in range(nb) if b % world == rank]
    if world > 1:
        # each rank renders its 16-row bands straight into a band-packed
        # accumulator (rt0_set_accum_buffer_compact) that is the RCCL send buffer
        import rt0.shard as shard
        r.set_shard(rank, world, band)
        gather = shard.BandGather(H, W, rank, world, band, "cuda:%d" % local)
        acc = gather.acc
        rows = r.set_accum_buffer_compact(acc.data_ptr())
        assert rows <= acc.shape[0], (rows, acc.shape)
    else:
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:%d" % local)
        r.set_accum_buffer(acc.data_ptr())

    def step(frame0):
        acc.zero_()
        torch.cuda.synchronize()
        r.render(frame0, SPP)  # synchronous: returns after the kernels finished
        if world > 1:
            gather.gather()  # RCCL gather of the HDR bands + one reorder on rank 0

    for i in range(args.warmup):
        step(1)
    kernel_ms = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(1)
        kernel_ms.append(r.last_kernel_ms()[0])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=acc.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1000.0 / args.steps
    total_samples = W * H * SPP * args.steps
    value = total_samples / dt / 1e6

    if rank != 0:
        dist.destroy_process_group()
        return

    # algorithmic FLOPs of the dominant kernel: counted events of the same
    # workload (separate counting kernel instance, outside the timed region)
    r.set_counting(True)
    acc.zero_()
    r.render(1, SPP)
    cnt = r.counters()
    r.set_counting(False)
    fps = flop_per_sample(cnt)
    owned_samples = len(owned) * band * W * SPP
    kern_s = float(np.mean(kernel_ms)) / 1000.0
    achieved_tflops = fps * owned_samples / kern_s / 1e12
    # HBM traffic per launch from the committed rocprofv3 PMC passes of this
    # workload (scripts/gpu_profile.sh -> scripts/pmc_traffic.py; FETCH_SIZE x2
    # gfx950 correction); counters cannot be read from inside this process
    traffic, pmc = None, None
    pmc_path = os.path.join(HERE, "profiles", PROFILE_ROUND, "pmc_summary.json")
    if world == 1 and os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
        traffic = pmc["traffic_bytes_per_launch"]
    out = {
        "metric": "Msamples/sec (pixels x spp / s) at 1024^2 Cornell, 8 bounces",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (the reference's own Cornell scene, index.js:54-85; no external data)",
        "config": {"workload": "%s: 1024x1024 Cornell, MIS power heuristic, MAX_BOUNCES=8, MAX_DIFF_BOUNCES=%d, "
                               "64 spp per step (u_frame 1..64)" % (args.config, cfg["constants"].get(
                                   "MAX_DIFF_BOUNCES", 4)),
                   "width": W, "height": H, "spp": SPP, "parallelism": "row-band x%d (16-row bands)" % world,
                   "kernel": "scene-specialised (hipRTC JIT)" if args.jit else "ahead-of-time"},
        "roofline": {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tflops / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
                     "traffic_unit": "bytes/launch",
                     "traffic_source": ("profiles/%s/pmc_summary.json" % PROFILE_ROUND) if pmc else None,
                     "valu_lane_utilisation": round(pmc["valu_lane_utilisation"], 4) if pmc and "valu_lane_utilisation"
                     in pmc else None,
                     # wave64 VALU instruction = 2 SIMD cycles (transcendental 4,
                     # MI355X_MICROARCH.md constants), over 1024 SIMDs x the live
                     # kernel time at the nominal 2.4 GHz
                     "valu_issue_utilisation": round(2.0 * (pmc["valu"]["SQ_INSTS_VALU"]
                                                           + pmc["valu"]["SQ_INSTS_VALU_TRANS_F32"])
                                                     / (1024 * kern_s * 2.4e9), 4)
                     if pmc and "valu" in pmc and world == 1 else None,
                     "flop_per_sample": round(fps, 1),
                     "events_per_sample": {k: round(cnt[k] / max(1, cnt["samples"]), 3)
                                           for k in ("isect", "iter", "nee")},
                     "kernel_ms_per_launch": round(kern_s * 1000.0, 3),
                     "hbm_bytes_per_launch": W * H * 16 * 2 // world,
                     "note": "FP32 vector kernel (no MFMA): peak = MI355X FP32 vector 157.3 TF; "
                             "FLOP model SURVEY 8d x counted events"},
    }
    if args.secondary:
        sec = [c for c in cfgs["configs"] if c["name"] == "c2_cornell_mis_refcaps"][0]
        rt0.configure(r, sec, cfgs)
        acc.zero_()
        r.render(1, SPP)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            acc.zero_()
            r.render(1, SPP)
        out["secondary_refcaps_Msamples_s"] = round(W * H * SPP * args.steps / (time.perf_counter() - t1) / 1e6 *
                                                    (world if world > 1 else 1), 3)
    if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
        js = cpu_baseline_js(args.config)
        c_port = cpu_baseline(cfgs, cfg)
        out["cpu_baseline"] = js if js and "value" in js else c_port
        out["cpu_baseline_c"] = c_port  # the C oracle on the same sample (OpenMP)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
