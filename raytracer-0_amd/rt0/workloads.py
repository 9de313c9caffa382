"""Bench workloads: BASELINE.json's configs as scene/host-state descriptions.

Each entry of workloads.json holds what a GlslViewport caller would set for
that configuration -- scene lines in the reference's grammar (index.html:
610-676), `defines`/`constants` by name (index.js:11-35), the camera
(index.js:89-95) -- plus the bench size and passes per step.  bench.py and
scripts/ read these; nothing here imports test or oracle code.
"""
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(_HERE, "workloads.json")


def load_all():
    with open(PATH) as f:
        return json.load(f)["workloads"]


def get(key):
    wl = load_all()
    if key not in wl:
        raise KeyError("unknown workload %r (known: %s)" % (key, ", ".join(sorted(wl))))
    return dict(wl[key], key=key)


def configure(renderer, wl, constants=None):
    """Apply a workload to a Renderer: flags, scene, camera and its models
    (rt0.meshes generators standing in for the absent OBJ assets)."""
    import rt0
    from rt0 import meshes as M
    cfg = {"defines": wl.get("defines", {}), "constants": dict(wl.get("constants", {}), **(constants or {})),
           "scene_lines": wl["scene_lines"], "sdf_kinds": wl.get("sdf_kinds", []), "camera": wl["camera"]}
    rt0.configure(renderer, cfg, {"cornell_lines": None, "default_camera": wl["camera"]})
    gens = {"icosphere": M.icosphere, "wavy_icosphere": M.wavy_icosphere}
    for k, m in enumerate(wl.get("models", [])):
        renderer.set_model(k, *gens[m["kind"]](m["level"]))
    return cfg


def restir(wl):
    return bool(wl.get("defines", {}).get("USE_RESTIR"))


def model_instances(wl):
    """[(positions, triangles, pos, scale, k)] of each TRIANGLE entry k whose
    scale (joker.x) is non-zero, as librt0's BVH build instances them."""
    import rt0
    from rt0 import meshes as M
    gens = {"icosphere": M.icosphere, "wavy_icosphere": M.wavy_icosphere}
    cfg = {"scene_lines": wl["scene_lines"], "sdf_kinds": wl.get("sdf_kinds", [])}
    scene, sdf = rt0.scene_strings(cfg, {"cornell_lines": None})
    meshes, ne, ns, _ = rt0.parse_scene(scene, sdf)
    out = []
    for k, (m, inst) in enumerate(zip(wl.get("models", []), meshes[ne + ns:])):
        if inst.joker[0] != 0.0:
            out.append(gens[m["kind"]](m["level"]) + (list(inst.pos), inst.joker[0], k))
    return out
