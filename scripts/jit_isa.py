#!/usr/bin/env python3
"""Static ISA audit of a bench workload's scene-specialised kernels (no GPU).

    python3 scripts/jit_isa.py c2 [OUT_DIR]

Compiles the workload's JIT module through rt0_jit_compile (hipRTC, the same
source and options rt0_render uses; for scenes with models the LDS stack is
the 48-entry default rather than the built tree's depth), disassembles it and
prints, per kernel: VGPR/SGPR/LDS/spill figures from the code-object notes and
an instruction histogram by class (VALU fp32 add/mul/fma, transcendental,
compare/select, int, cvt, moves, SALU, memory, branches).  OUT_DIR keeps the
generated source, the code object and the disassembly.
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

CLASSES = [
    ("fma_f32", r"^v_(fma|fmac|mad|mac)_f32|^v_fmamk_f32|^v_fmaak_f32"),
    ("pk_f32", r"^v_pk_\w+_f32"),
    ("add_f32", r"^v_(add|sub|subrev)_f32"),
    ("mul_f32", r"^v_mul_f32|^v_mul_legacy_f32"),
    ("minmax_f32", r"^v_(min|max|med3|min3|max3)_f32"),
    ("trans", r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32"),
    ("cmp", r"^v_cmp"),
    ("cndmask", r"^v_cndmask"),
    ("cvt", r"^v_cvt"),
    ("int_valu", r"^v_(add|sub|mul|lshl|lshr|ashr|and|or|xor|bfe|bfi|mad_u|mad_i|min_[iu]|max_[iu]|not|alignbit|perm|subrev)_"),
    ("mov", r"^v_mov|^v_readfirstlane|^v_readlane|^v_writelane|^v_accvgpr"),
    ("other_valu", r"^v_"),
    ("salu", r"^s_(?!cbranch|branch|waitcnt|nop|load|buffer|endpgm|setpc|swappc|getpc)"),
    ("smem", r"^s_(load|buffer)"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc)"),
    ("waitcnt", r"^s_(waitcnt|nop)"),
    ("vmem", r"^(global|buffer|flat|scratch)_"),
    ("lds", r"^ds_"),
]


def classify(op):
    for name, pat in CLASSES:
        if re.match(pat, op):
            return name
    return "other"


def main():
    import rt0
    from rt0 import workloads
    key = sys.argv[1] if len(sys.argv) > 1 else "c2"
    out = sys.argv[2] if len(sys.argv) > 2 else tempfile.mkdtemp(prefix="jit_isa_")
    os.makedirs(out, exist_ok=True)
    wl = workloads.get(key)
    cfg = {"defines": wl.get("defines", {}), "constants": wl.get("constants", {}), "scene_lines": wl["scene_lines"],
           "sdf_kinds": wl.get("sdf_kinds", []), "camera": wl["camera"]}
    scene, sdf = rt0.scene_strings(cfg, {"cornell_lines": None})
    os.environ["RT0_JIT_DUMP"] = os.path.join(out, "k")
    rt0.jit_compile(scene, sdf, rt0.parse_config(*rt0.config_strings(cfg)))
    cos = sorted(glob.glob(os.path.join(out, "k_*.co")), key=os.path.getmtime)
    co = cos[-1]
    notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    dis = subprocess.run([LLVM + "/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True).stdout
    open(co[:-3] + ".s", "w").write(dis)
    print("workload %s: %s" % (key, co))
    for m in re.finditer(r"\.name:\s+(\S+)", notes):
        seg = notes[m.start():]
        nxt = re.search(r"\n\s+- \.", seg[5:])
        seg = seg[:nxt.start() + 5] if nxt else seg
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", seg) or [None, "?"])[1]
        print("  %-16s vgpr %s sgpr %s lds %s spill %s" % (m.group(1), g("vgpr_count"), g("sgpr_count"),
                                                            g("group_segment_fixed_size"), g("vgpr_spill_count")))
    funcs = re.split(r"\n(?=[0-9a-f]+ <[^>]+>:)", dis)
    for f in funcs:
        hm = re.match(r"[0-9a-f]+ <([^>]+)>:", f)
        if not hm or not hm.group(1).startswith("rt0_jit_"):
            continue
        hist = collections.Counter()
        for line in f.splitlines()[1:]:
            t = line.strip().split()
            if not t:
                continue
            hist[classify(t[0])] += 1
        tot = sum(hist.values())
        print("  %s: %d instructions (static)" % (hm.group(1), tot))
        for k, v in hist.most_common():
            print("    %-12s %6d  %5.1f%%" % (k, v, 100.0 * v / tot))


if __name__ == "__main__":
    main()
