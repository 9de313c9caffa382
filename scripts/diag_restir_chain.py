"""Diagnostic (GPU box): the product's ReSTIR chain with executor compat and
the conditional single passes, saved for offline comparison with the fixture.
usage: python scripts/diag_restir_chain.py <config> <out.npz> [jit 0|1]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "raytracer-0_amd"), os.path.join(HERE, "..", "oracle")]
import oracle as O  # noqa: E402  (test infrastructure: fixture loading only)
import rt0  # noqa: E402

name, out = sys.argv[1], sys.argv[2]
jit = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cfgs = O.load_configs()
cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
G = np.load(os.path.join(HERE, "..", "tests", "golden", name + ".npz"))
F, H, W = G["samples"].shape[:3]
res = {}
for compat in (1, 0):
    r = rt0.Renderer(W, H)
    r.set_jit(jit)
    rt0.configure(r, cfg, cfgs)
    r.set_executor_compat(compat)
    zero = np.zeros((H, W, 4), np.float32)
    S, M, A = [], [], []
    for k in range(1, F + 1):
        r.write_accum(zero)
        r.render(k, 1, O.pass_time(cfg, k) if cfg.get("time_ms") else 0.0)
        S.append(r.read_accum())
        m, a = r.read_restir(0)
        M.append(m)
        A.append(a)
    res["chain%d_s" % compat], res["chain%d_m" % compat], res["chain%d_a" % compat] = map(np.stack, (S, M, A))
r = rt0.Renderer(W, H)
r.set_jit(jit)
rt0.configure(r, cfg, cfgs)
C = []
for k in range(1, F + 1):
    r.clear()
    ins = [G["restir_main"][k - j - 1] if k - j >= 1 else None for j in (1, 1, 2, 2, 3, 3)]
    ins = [G[key][k - j - 1] if k - j >= 1 else None
           for j, key in ((1, "restir_main"), (1, "restir_aux"), (2, "restir_main"), (2, "restir_aux"),
                          (3, "restir_main"), (3, "restir_aux"))]
    r.write_restir_inputs(*ins)
    r.render(k, 1)
    C.append(r.read_accum())
res["cond_s"] = np.stack(C)
np.savez_compressed(out, **res)
print("saved", out)
