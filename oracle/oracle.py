"""ctypes wrapper of the CPU restatement (oracle/rt0_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librt0_oracle.so")
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.or_create.restype = ctypes.c_void_p
        L.or_destroy.argtypes = [ctypes.c_void_p]
        L.or_error.restype = ctypes.c_char_p
        L.or_error.argtypes = [ctypes.c_void_p]
        L.or_set_scene_lines.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.or_set_define.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.or_set_constant.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double]
        fp = ctypes.POINTER(ctypes.c_float)
        L.or_set_camera.argtypes = [ctypes.c_void_p, fp, fp, fp]
        L.or_set_resolution.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.or_render_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint, fp, ctypes.POINTER(fp), fp, fp,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.or_render_accum.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, fp, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.or_hash.restype = ctypes.c_float
        L.or_hash.argtypes = [ctypes.c_float]
        L.or_hash2.argtypes = [ctypes.c_float, ctypes.c_float, fp]
        L.or_set_texture.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_uint8)]
        L.or_set_triangles.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_int]
        L.or_set_cubemap.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))]
        L.or_set_time.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int]
        L.or_pixel_seed.restype = ctypes.c_float
        L.or_pixel_seed.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_uint]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def load_configs():
    with open(os.path.join(GOLDEN, "configs.json")) as f:
        return json.load(f)


class Oracle:
    """One configured oracle instance (scene + flags + camera + resolution)."""

    def __init__(self, cfg, cfgs=None, width=64, height=64, overrides=None):
        cfgs = cfgs or load_configs()
        L = lib()
        self.h = L.or_create()
        self.w, self.hgt = width, height
        lines = cfg["scene_lines"] or cfgs["cornell_lines"]
        kinds = cfg.get("sdf_kinds") or []
        karr = (ctypes.c_int * max(1, len(kinds)))(*kinds)
        self._chk(L.or_set_scene_lines(self.h, "\n".join(lines).encode(), karr, len(kinds)))
        for k, v in cfg.get("defines", {}).items():
            self._chk(L.or_set_define(self.h, k.encode(), int(bool(v))))
        # the reference executor's fixed-point texture filter, as the product's
        # default (rt0_set_texture_filter; SWIFTSHADER_TEX_FILTER 0 = fp32 bilinear)
        consts = {"SWIFTSHADER_TEX_FILTER": 1}
        consts.update(cfg.get("constants", {}))
        consts.update(overrides or {})
        for k, v in consts.items():
            self._chk(L.or_set_constant(self.h, k.encode(), float(v)))
        cam = cfg.get("camera") or cfgs["default_camera"]
        pos = np.array(cam["origin"], np.float32)
        look = np.array(cam["lookat"], np.float32)
        par = np.array([cam["fov"], cam["aperture"], cam["focalLength"]], np.float32)
        L.or_set_camera(self.h, _fp(pos), _fp(look), _fp(par))
        L.or_set_resolution(self.h, width, height)
        self.restir = bool(cfg.get("defines", {}).get("USE_RESTIR"))
        self._tex = {}
        from textures import cubemap_for, textures_for
        for unit, img in textures_for(cfg).items():
            self.set_texture(unit, img)
        faces = cubemap_for(cfg)
        if faces is not None:
            self.set_cubemap(faces)

    def set_time(self, time_ms, temporal_frames=5):
        """u_time / u_temporalFrames (read by RENDER_MODE 1 only)."""
        lib().or_set_time(self.h, float(time_ms), int(temporal_frames))

    def set_triangles(self, v9, model):
        """World-space triangles float32 [n, 9] and their owner model index
        (bit 30 = back-face culling); brute-force closest hit."""
        v = np.ascontiguousarray(v9, np.float32).reshape(-1, 9)
        m = np.ascontiguousarray(model, np.int32).reshape(-1)
        self._tris = (v, m)  # the C side keeps pointers
        self._chk(lib().or_set_triangles(self.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                         m.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), v.shape[0]))

    def set_cubemap(self, faces):
        """u_cubemap: six uint8 [n, n, 3] faces, reference order -X -Y -Z +X +Y +Z."""
        arrs = [np.ascontiguousarray(f, np.uint8) for f in faces]
        self._cube = arrs
        P = ctypes.POINTER(ctypes.c_uint8)
        ptrs = (P * 6)(*[a.ctypes.data_as(P) for a in arrs])
        self._chk(lib().or_set_cubemap(self.h, arrs[0].shape[0], ptrs))

    def set_texture(self, unit, rgba8):
        """u_tex0..3 (unit 0..3) / u_rnd_tex (4): uint8 [h, w, 4], first row = t 0."""
        a = np.ascontiguousarray(rgba8, np.uint8)
        self._tex[unit] = a  # the C side keeps a pointer
        self._chk(lib().or_set_texture(self.h, unit, a.shape[1], a.shape[0],
                                       a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))

    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError(lib().or_error(self.h).decode())

    def __del__(self):
        try:
            lib().or_destroy(self.h)
        except Exception:
            pass

    def frame(self, frame, restir_in=None, rows=None, threads=0, counters=None):
        """One pass (single sample per pixel). Returns (sample, restir_main, restir_aux)."""
        out = np.zeros((self.hgt, self.w, 4), np.float32)
        rm = np.zeros_like(out)
        ra = np.zeros_like(out)
        keep = []
        pin = None
        if restir_in is not None:
            arrs = [np.ascontiguousarray(t, np.float32) for t in restir_in]
            keep = arrs
            pin = (ctypes.POINTER(ctypes.c_float) * 6)(*[_fp(a) for a in arrs])
        r0, r1 = rows or (0, self.hgt)
        c = (ctypes.c_uint64 * 4)() if counters is not None else None
        self._chk(lib().or_render_frame(self.h, frame, _fp(out), pin, _fp(rm), _fp(ra), r0, r1, threads, c))
        if counters is not None:
            counters += np.array(list(c), np.uint64)
        del keep
        return out, rm, ra

    def frames_restir(self, n, cfg=None):
        """Passes 1..n with the reference's ReSTIR swap chain (index.js:795-820);
        returns per-pass samples [n,H,W,4] and reservoirs.  cfg with time_ms
        (RENDER_MODE 1 configs): u_time of pass k = pass_time(cfg, k)."""
        z = np.zeros((self.hgt, self.w, 4), np.float32)
        rbuf, raux, rbuf_back, raux_back, h1, h1a, h2, h2a = z, z, z, z, z, z, z, z
        samples, mains, auxs = [], [], []
        for k in range(1, n + 1):
            if cfg is not None and cfg.get("time_ms"):
                self.set_time(pass_time(cfg, k), cfg.get("temporal_frames", 5))
            s, m, a = self.frame(k, [rbuf_back, raux_back, h1, h1a, h2, h2a])
            rbuf, raux = m, a  # MRT1/2 written this pass
            samples.append(s)
            mains.append(m)
            auxs.append(a)
            o2, o2a = h2, h2a
            h2, h2a = h1, h1a
            h1, h1a = rbuf_back, raux_back
            rbuf_back, raux_back = o2, o2a
            rbuf, rbuf_back = rbuf_back, rbuf
            raux, raux_back = raux_back, raux
        return np.stack(samples), np.stack(mains), np.stack(auxs)

    def accumulate(self, first, n, acc=None, threads=0, counters=None):
        acc = np.zeros((self.hgt, self.w, 4), np.float32) if acc is None else acc
        c = (ctypes.c_uint64 * 4)() if counters is not None else None
        self._chk(lib().or_render_accum(self.h, first, n, _fp(acc), 0, self.hgt, threads, c))
        if counters is not None:
            counters += np.array(list(c), np.uint64)
        return acc


def pass_time(cfg, k):
    """u_time of pass k (1-based) of a RENDER_MODE 1 config: t0 + (k-1)*dt."""
    t0, dt = cfg.get("time_ms") or (0.0, 0.0)
    return float(t0) + float(k - 1) * float(dt)


def hash_(x):
    return lib().or_hash(float(x))


def hash2(x, y):
    out = np.zeros(2, np.float32)
    lib().or_hash2(x, y, _fp(out))
    return out


def pixel_seed(fx, fy, frame):
    return lib().or_pixel_seed(fx, fy, frame)


def write_tris(path, v9, owners):
    """The triangle soup of oracle/js/cpu_bench.js --tris: int32 n, n x 9
    float32 world-space vertices, n int32 owners (entry k | cull bit 30)."""
    v = np.ascontiguousarray(v9, np.float32).reshape(-1, 9)
    m = np.ascontiguousarray(owners, np.int32).reshape(-1)
    with open(path, "wb") as f:
        f.write(np.int32(len(m)).tobytes())
        f.write(v.tobytes())
        f.write(m.tobytes())

