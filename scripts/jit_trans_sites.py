#!/usr/bin/env python3
"""Per-source-site census of the transcendental VALU instructions (v_sin, v_cos,
v_sqrt, v_rsq, v_log, v_exp, v_rcp) in a workload's scene-specialised kernel.

    python3 scripts/jit_trans_sites.py c2 [OUT_DIR] [KERNEL]

Compiles the module like scripts/jit_isa.py with line tables
(RT0_JIT_EXTRA=-gline-tables-only: same code, plus .debug_line), disassembles
it with source lines and prints, per source line of the generated JIT source
(rt0_device.h + rt0_integrator.h + the scene), the transcendental opcodes it
owns in KERNEL (default rt0_jit_pass) and the line's text.  Inlined code is
attributed to its innermost source line.  Static counts: how often a site runs
per sample is the event census' business (bench.py events_per_sample).
"""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
LLVM = "/opt/rocm/lib/llvm/bin"
TRANS = re.compile(r"^v_(sin|cos|sqrt|rsq|log|exp|rcp)_f32")


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else "c2"
    out = sys.argv[2] if len(sys.argv) > 2 else tempfile.mkdtemp(prefix="jit_trans_")
    kernel = sys.argv[3] if len(sys.argv) > 3 else "rt0_jit_pass"
    os.makedirs(out, exist_ok=True)
    os.environ["RT0_JIT_EXTRA"] = "-gline-tables-only"
    os.environ["RT0_JIT_DUMP"] = os.path.join(out, "k")
    import rt0
    from rt0 import workloads
    wl = workloads.get(key)
    cfg = {"defines": wl.get("defines", {}), "constants": wl.get("constants", {}), "scene_lines": wl["scene_lines"],
           "sdf_kinds": wl.get("sdf_kinds", []), "camera": wl["camera"]}
    scene, sdf = rt0.scene_strings(cfg, {"cornell_lines": None})
    rt0.jit_compile(scene, sdf, rt0.parse_config(*rt0.config_strings(cfg)))
    co = sorted(glob.glob(os.path.join(out, "k_*.co")), key=os.path.getmtime)[-1]
    src = open(co[:-3] + ".hip").read().splitlines()
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "-l", "--mcpu=gfx950", co], capture_output=True,
                         text=True).stdout
    # every transcendental instruction's address, then its inline stack
    # (llvm-symbolizer --inlines): the site is the first frame outside the
    # one-line math helpers (frcp, frsq, fsqrt, normalize, ...), so a helper's
    # instructions are charged to the line that called it
    addrs, inside = [], False
    for l in dis.splitlines():
        m = re.match(r"[0-9a-f]+ <([^>]+)>:", l)
        if m:
            inside = m.group(1) == kernel
            continue
        t = l.strip().split()
        if inside and t and TRANS.match(t[0]):
            a = re.search(r"//\s*([0-9A-Fa-f]+):", l)
            if a:
                addrs.append((int(a.group(1), 16), t[0].split("_e")[0]))
    sym = subprocess.run([LLVM + "/llvm-symbolizer", "--inlines", "--obj=" + co] + ["0x%x" % a for a, _ in addrs],
                         capture_output=True, text=True).stdout.strip().split("\n\n")
    helpers = {"frcp", "frsq", "fsqrt", "fdiv", "fsin", "fcos", "fsin_rev", "fcos_rev", "fexp", "flog", "normalize",
               "length"}
    sites = collections.defaultdict(collections.Counter)
    chains = {}
    for (a, op), block in zip(addrs, sym):
        lines = block.strip().splitlines()
        frames = [(lines[i].strip(), lines[i + 1].strip()) for i in range(0, len(lines) - 1, 2)]
        site = None
        for fn, loc in frames:
            base = re.sub(r"\(.*", "", fn).split("::")[-1]
            if base not in helpers:
                m = re.search(r":(\d+):", loc)
                site = (int(m.group(1)) if m else None, base)
                break
        sites[site][op] += 1
        chains[site] = " < ".join(re.sub(r"\(.*", "", fn).split("::")[-1] for fn, _ in frames[:4])
    total = sum(sum(c.values()) for c in sites.values())
    print("workload %s, kernel %s: %d transcendental instructions (static) at %d source lines" %
          (key, kernel, total, len(sites)))
    for site, c in sorted(sites.items(), key=lambda kv: -sum(kv[1].values())):
        ln, fn = site if site else (None, "?")
        text = src[ln - 1].strip() if ln and ln <= len(src) else "?"
        print("%5s %-22s %-30s %s" % (ln, fn, " ".join("%s x%d" % kv for kv in sorted(c.items())), text[:100]))


if __name__ == "__main__":
    main()
