"""With scripts/ab_r6_wf_shadow_steps.patch applied: whether
RT0_WF_SHADOW_STEPS (shadow-march steps run by the wavefront shade kernel, a
JIT define through RT0_JIT_EXTRA) changes any bit: a 256x256 C4 render
(4 passes) with K = 0 and with each K of argv, compared bit for bit.

    python3 scripts/wf_shadow_check.py 4 8 16
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402


def render(k, key="c4", size=256, frames=4):
    os.environ["RT0_JIT_EXTRA"] = "-DRT0_WF_SHADOW_STEPS=%d" % k
    wl = dict(workloads.get(key))
    r = rt0.Renderer(size, size)
    workloads.configure(r, wl)
    r.render(1, frames)
    img = r.read_accum()
    path = r.last_render_path()
    r.close()
    return img, path


def main():
    base, path = render(0)
    print("K=0", path, float(np.abs(base).mean()), flush=True)
    bad = 0
    for k in [int(a) for a in sys.argv[1:]] or [8]:
        img, p = render(k)
        same = np.array_equal(img.view(np.uint32), base.view(np.uint32))
        print("K=%d" % k, p, "bit-identical" if same else "DIFFERS (%d words)" % int((img != base).sum()), flush=True)
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
