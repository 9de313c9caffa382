"""rt0 -- Python host for the MI355X raytracer-0 backend (ctypes over include/rt0.h).

`GlslViewport` mirrors the reference host class (index.js:3-1105): the same
public fields (defines, constants, scene, sdf_meshes, camera, passes,
max_passes) and methods (render, clear, resize, setAnimatedMode,
updateFrontTarget).  Scene/flag strings use the reference's own grammar, so a
caller written against the reference can drive this backend unchanged.  The
integrator itself runs only in the HIP kernels of librt0.so: there is no CPU
fallback, and every entry point raises if the library or a GPU is missing.
"""
import ctypes
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librt0.so")

RT0_OK = 0
ERRORS = {-1: "RT0_E_ARG", -2: "RT0_E_HIP", -3: "RT0_E_UNSUPPORTED", -4: "RT0_E_STATE"}

DEFINE_NAMES = ["USE_CUBEMAP", "USE_PROCEDURAL_SKY", "USE_BIASED_SAMPLING", "USE_BIDIRECTIONAL",
                "USE_RESTIR", "USE_SPECTRAL", "USE_VOLUMETRICS"]

# C symbols declared by include/rt0.h (checked by tests/test_abi.py)
EXPORTS = ["rt0_create", "rt0_destroy", "rt0_last_error", "rt0_parse_config", "rt0_set_config", "rt0_get_config",
           "rt0_set_scene_glsl", "rt0_set_scene", "rt0_parse_scene_glsl", "rt0_get_scene", "rt0_set_camera", "rt0_render",
           "rt0_render_async", "rt0_sync", "rt0_read_accum", "rt0_write_accum", "rt0_clear", "rt0_resize",
           "rt0_get_size", "rt0_tonemap", "rt0_read_restir", "rt0_write_restir_inputs", "rt0_set_shard",
           "rt0_device_accum", "rt0_set_accum_buffer", "rt0_set_accum_buffer_compact", "rt0_set_restir_buffers", "rt0_device_restir",
           "rt0_set_halo", "rt0_read_halo_misses", "rt0_set_jit", "rt0_set_executor_compat", "rt0_set_texture_filter", "rt0_set_defer_light_sampling", "rt0_set_wavefront", "rt0_jit_compile", "rt0_set_counting",
           "rt0_read_counters", "rt0_read_counters_n", "rt0_last_kernel_ms", "rt0_last_render_path", "rt0_version", "rt0_tonemap_ex", "rt0_png_decode", "rt0_png_read",
           "rt0_png_write", "rt0_pfm_write", "rt0_free", "rt0_set_texture", "rt0_set_cubemap", "rt0_jpeg_decode", "rt0_jpeg_read", "rt0_set_model", "rt0_model_info", "rt0_obj_read",
           "rt0_set_temporal_frames", "rt0_set_viewport", "rt0_scratch_bytes"]

TEX_NOISE = 4  # RT0_TEX_NOISE: the u_rnd_tex unit of rt0_set_texture
TONEMAP_GAMMA, TONEMAP_ACES, TONEMAP_REINHARD = 0, 1, 2
TEX_FILTER_FLOAT, TEX_FILTER_FIXED16 = 0, 1  # rt0_set_texture_filter


class Rt0Error(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (ERRORS.get(code, code), msg))
        self.code = code


class Config(ctypes.Structure):
    """rt0_config, field order = constants[] of index.js:21-35."""
    _fields_ = [("defines", ctypes.c_uint32), ("max_bounces", ctypes.c_int32), ("max_diff_bounces", ctypes.c_int32),
                ("max_spec_bounces", ctypes.c_int32), ("max_trans_bounces", ctypes.c_int32),
                ("max_scattering_events", ctypes.c_int32), ("marching_steps", ctypes.c_int32),
                ("fudge_factor", ctypes.c_float), ("sample_lights", ctypes.c_int32), ("use_mis", ctypes.c_int32),
                ("use_restir", ctypes.c_int32), ("light_path_length", ctypes.c_int32),
                ("restir_samples", ctypes.c_int32), ("render_mode", ctypes.c_int32)]


class Mesh(ctypes.Structure):
    _fields_ = [("c", ctypes.c_float * 3), ("e", ctypes.c_float * 3), ("nt", ctypes.c_float),
                ("mat_type", ctypes.c_int32), ("tex_type", ctypes.c_int32), ("type", ctypes.c_int32),
                ("pos", ctypes.c_float * 3), ("joker", ctypes.c_float * 4), ("sdf_kind", ctypes.c_int32),
                ("tex_c_mask", ctypes.c_float * 3), ("tex_e_mask", ctypes.c_float * 3),
                ("tex_params", ctypes.c_float * 4), ("mat_opts", ctypes.c_uint32)]


_lib = None


def lib():
    """Load librt0.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("librt0.so not built (run `make -C raytracer-0_amd` or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7, and
    # if librt0 bound /opt/rocm's copy first, torch.cuda would later find "No
    # HIP GPUs" (two runtimes over one device).  Importing torch first (when
    # it is installed) makes librt0 resolve to the runtime torch loaded, so
    # torch tensors (sharded accumulators, RCCL buffers) and librt0 share it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    c_void_p, c_int, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    fp = P(ctypes.c_float)
    sig = {
        "rt0_create": (c_int, [c_int, c_int, c_int, P(c_void_p)]),
        "rt0_destroy": (None, [c_void_p]),
        "rt0_last_error": (ctypes.c_char_p, [c_void_p]),
        "rt0_parse_config": (c_int, [P(ctypes.c_char_p), c_int, P(ctypes.c_char_p), c_int, P(Config)]),
        "rt0_set_config": (c_int, [c_void_p, P(Config)]),
        "rt0_get_config": (c_int, [c_void_p, P(Config)]),
        "rt0_set_scene_glsl": (c_int, [c_void_p, ctypes.c_char_p, P(ctypes.c_char_p), c_int]),
        "rt0_set_scene": (c_int, [c_void_p, P(Mesh), c_int, c_int, c_int, P(ctypes.c_int32), c_int]),
        "rt0_parse_scene_glsl": (c_int, [ctypes.c_char_p, P(ctypes.c_char_p), c_int, P(Mesh), c_int, P(c_int),
                                         P(c_int), P(c_int), P(ctypes.c_int32), c_int, P(c_int)]),
        "rt0_get_scene": (c_int, [c_void_p, P(Mesh), c_int, P(c_int), P(c_int), P(c_int), P(ctypes.c_int32), c_int,
                                  P(c_int)]),
        "rt0_set_model": (c_int, [c_void_p, c_int, fp, c_int, P(ctypes.c_int32), c_int]),
        "rt0_model_info": (c_int, [c_void_p, P(c_int), P(c_int)]),
        "rt0_obj_read": (c_int, [ctypes.c_char_p, P(fp), P(c_int), P(P(ctypes.c_int32)), P(c_int)]),
        "rt0_set_camera": (c_int, [c_void_p, fp, fp, fp]),
        "rt0_set_texture": (c_int, [c_void_p, c_int, c_int, c_int, P(ctypes.c_uint8)]),
        "rt0_set_cubemap": (c_int, [c_void_p, c_int, P(P(ctypes.c_uint8))]),
        "rt0_render": (c_int, [c_void_p, ctypes.c_uint32, c_int, c_float]),
        "rt0_render_async": (c_int, [c_void_p, ctypes.c_uint32, c_int, c_float]),
        "rt0_set_temporal_frames": (c_int, [c_void_p, c_int]),
        "rt0_set_viewport": (c_int, [c_void_p, c_int, c_int, c_int, c_int]),
        "rt0_sync": (c_int, [c_void_p]),
        "rt0_read_accum": (c_int, [c_void_p, fp]),
        "rt0_write_accum": (c_int, [c_void_p, fp]),
        "rt0_clear": (c_int, [c_void_p]),
        "rt0_resize": (c_int, [c_void_p, c_int, c_int]),
        "rt0_get_size": (c_int, [c_void_p, P(c_int), P(c_int)]),
        "rt0_tonemap": (c_int, [c_void_p, c_float, P(ctypes.c_uint8)]),
        "rt0_read_restir": (c_int, [c_void_p, c_int, fp, fp]),
        "rt0_write_restir_inputs": (c_int, [c_void_p, fp, fp, fp, fp, fp, fp]),
        "rt0_set_shard": (c_int, [c_void_p, c_int, c_int, c_int]),
        "rt0_device_accum": (c_int, [c_void_p, P(c_void_p), P(c_void_p)]),
        "rt0_set_accum_buffer": (c_int, [c_void_p, c_void_p]),
        "rt0_set_accum_buffer_compact": (c_int, [c_void_p, c_void_p, P(c_int)]),
        "rt0_set_restir_buffers": (c_int, [c_void_p, P(c_void_p)]),
        "rt0_device_restir": (c_int, [c_void_p, c_int, P(c_void_p), P(c_void_p)]),
        "rt0_set_halo": (c_int, [c_void_p, c_int]),
        "rt0_read_halo_misses": (c_int, [c_void_p, P(ctypes.c_uint32), c_int]),
        "rt0_set_jit": (c_int, [c_void_p, c_int]),
        "rt0_set_executor_compat": (c_int, [c_void_p, c_int]),
        "rt0_set_texture_filter": (c_int, [c_void_p, c_int]),
        "rt0_set_defer_light_sampling": (c_int, [c_void_p, c_int]),
        "rt0_set_wavefront": (c_int, [c_void_p, c_int]),
        "rt0_jit_compile": (c_int, [ctypes.c_char_p, P(ctypes.c_char_p), c_int, P(Config), P(ctypes.c_size_t),
                                    ctypes.c_char_p, ctypes.c_size_t]),
        "rt0_set_counting": (c_int, [c_void_p, c_int]),
        "rt0_read_counters": (c_int, [c_void_p, P(ctypes.c_uint64)]),
        "rt0_read_counters_n": (c_int, [c_void_p, P(ctypes.c_uint64), c_int]),
        "rt0_last_kernel_ms": (c_int, [c_void_p, P(c_float), P(c_int)]),
        "rt0_last_render_path": (c_int, [c_void_p]),
        "rt0_scratch_bytes": (c_int, [c_void_p, P(ctypes.c_size_t)]),
        "rt0_version": (ctypes.c_char_p, []),
        "rt0_tonemap_ex": (c_int, [c_void_p, c_float, c_int, P(ctypes.c_uint8)]),
        "rt0_png_decode": (c_int, [c_void_p, ctypes.c_size_t, P(c_int), P(c_int), P(P(ctypes.c_uint8))]),
        "rt0_png_read": (c_int, [ctypes.c_char_p, P(c_int), P(c_int), P(P(ctypes.c_uint8))]),
        "rt0_png_write": (c_int, [ctypes.c_char_p, c_int, c_int, P(ctypes.c_uint8), c_int]),
        "rt0_pfm_write": (c_int, [ctypes.c_char_p, c_int, c_int, fp, c_float]),
        "rt0_free": (None, [c_void_p]),
        "rt0_jpeg_decode": (c_int, [c_void_p, ctypes.c_size_t, P(c_int), P(c_int), P(P(ctypes.c_uint8))]),
        "rt0_jpeg_read": (c_int, [ctypes.c_char_p, P(c_int), P(c_int), P(P(ctypes.c_uint8))]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _fp(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _strarr(items):
    arr = (ctypes.c_char_p * max(1, len(items)))()
    for i, s in enumerate(items):
        arr[i] = s.encode()
    return arr


def parse_config(defines, constants):
    """GlslViewport.defines/.constants string arrays -> Config (index.js:11-35)."""
    cfg = Config()
    rc = lib().rt0_parse_config(_strarr(defines), len(defines), _strarr(constants), len(constants),
                                ctypes.byref(cfg))
    if rc != RT0_OK:
        raise Rt0Error(rc, "cannot parse defines/constants")
    return cfg


# ----------------------------------------------------------------- scene text
def parse_scene(scene_text, sdf_meshes=()):
    """Pure parse of GlslViewport.scene + .sdf_meshes -> (meshes, n_meshes, n_sdfs, light_index);
    meshes also holds the TRIANGLE entries after the SDFs (len(meshes) - n_meshes - n_sdfs models)."""
    meshes = (Mesh * 128)()
    lights = (ctypes.c_int32 * 128)()
    ne, ns, nm, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    sdf = list(sdf_meshes)
    rc = lib().rt0_parse_scene_glsl(scene_text.encode(), _strarr(sdf), len(sdf), meshes, 128, ctypes.byref(ne),
                                    ctypes.byref(ns), ctypes.byref(nm), lights, 128, ctypes.byref(nl))
    if rc != RT0_OK:
        raise Rt0Error(rc, "cannot parse scene")
    return list(meshes[:ne.value + ns.value + nm.value]), ne.value, ns.value, list(lights[:nl.value])


def _check_io(rc, what):
    if rc != 0:
        raise Rt0Error(rc, what)


def png_decode(data):
    """PNG bytes -> [h, w, 4] uint8 (row 0 = the file's first row)."""
    w, h, p = ctypes.c_int(), ctypes.c_int(), ctypes.POINTER(ctypes.c_uint8)()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    _check_io(lib().rt0_png_decode(buf, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)), "png_decode")
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 4)).copy()
    finally:
        lib().rt0_free(p)


def png_read(path):
    w, h, p = ctypes.c_int(), ctypes.c_int(), ctypes.POINTER(ctypes.c_uint8)()
    _check_io(lib().rt0_png_read(str(path).encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)),
              "png_read %s" % path)
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 4)).copy()
    finally:
        lib().rt0_free(p)


def obj_read(path):
    """Wavefront OBJ -> (positions float32 [nv, 3], triangles int32 [nt, 3])."""
    pp, ip = ctypes.POINTER(ctypes.c_float)(), ctypes.POINTER(ctypes.c_int32)()
    nv, nt = ctypes.c_int(), ctypes.c_int()
    _check_io(lib().rt0_obj_read(str(path).encode(), ctypes.byref(pp), ctypes.byref(nv), ctypes.byref(ip),
                                 ctypes.byref(nt)), "obj_read %s" % path)
    try:
        v = np.ctypeslib.as_array(pp, shape=(max(1, nv.value) * 3,))[:nv.value * 3].reshape(-1, 3).copy()
        t = np.ctypeslib.as_array(ip, shape=(max(1, nt.value) * 3,))[:nt.value * 3].reshape(-1, 3).copy()
        return v, t
    finally:
        lib().rt0_free(pp)
        lib().rt0_free(ip)


def jpeg_decode(data):
    """Baseline JPEG bytes -> [h, w, 4] uint8."""
    w, h, p = ctypes.c_int(), ctypes.c_int(), ctypes.POINTER(ctypes.c_uint8)()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    _check_io(lib().rt0_jpeg_decode(buf, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)), "jpeg_decode")
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 4)).copy()
    finally:
        lib().rt0_free(p)


def image_read(path):
    """An asset file -> [h, w, 4] uint8: PNG (textures) or baseline JPEG (the
    reference's cubemap faces), told apart by the file signature."""
    with open(path, "rb") as f:
        head = f.read(2)
    if head == b"\xff\xd8":
        with open(path, "rb") as f:
            return jpeg_decode(f.read())
    return png_read(path)


def png_write(path, rgba, flip_y=False):
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("[h, w, 4] uint8 expected")
    _check_io(lib().rt0_png_write(str(path).encode(), a.shape[1], a.shape[0],
                                  a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), int(bool(flip_y))), "png_write")


def pfm_write(path, rgba, scale=1.0):
    a = np.ascontiguousarray(rgba, dtype=np.float32)
    _check_io(lib().rt0_pfm_write(str(path).encode(), a.shape[1], a.shape[0], _fp(a), scale), "pfm_write")


def jit_compile(scene_text, sdf_meshes, cfg):
    """Build the scene-specialised kernel offline (hipRTC, no device); returns the code-object size."""
    sdf = list(sdf_meshes)
    size = ctypes.c_size_t()
    err = ctypes.create_string_buffer(4096)
    rc = lib().rt0_jit_compile(scene_text.encode(), _strarr(sdf), len(sdf), ctypes.byref(cfg), ctypes.byref(size),
                               err, 4096)
    if rc != RT0_OK:
        raise Rt0Error(rc, err.value.decode(errors="replace"))
    return size.value


def scene_from_lines(lines):
    """The scene textarea -> GLSL `#scene` text, as index.html:610-676 builds it.

    Returns (scene_text, n_sdfs)."""
    n_meshes = n_sdfs = n_models = 0
    u_sphere = u_plane = u_box = False
    lights, text = [], []
    for i, line in enumerate(lines):
        fields = line.split(",")
        mat, typ = fields[0].strip(), fields[1].strip()
        if mat.rfind("MAT_LIGHT") >= 0:
            lights.append(i)
        text.append("Mesh(" + line + ")" + ("," if i != len(lines) - 1 else ""))
        if typ in ("SDF", "GRID_SDF"):
            n_sdfs += 1
        elif typ in ("PLANE", "SPHERE", "BOX"):
            u_sphere |= typ == "SPHERE"
            u_plane |= typ == "PLANE"
            u_box |= typ == "BOX"
            n_meshes += 1
        elif typ == "TRIANGLE":
            n_models += 1
        else:
            raise ValueError("There's no such thing as " + typ)
    if not lights:
        lights.append(-1)
    b = lambda v: "true" if v else "false"  # noqa: E731
    scene = ("const bool U_EUCLIDEAN = %s;\nconst bool U_SPHERE = %s;\nconst bool U_PLANE = %s;\n"
             "const bool U_BOX = %s;\nconst bool U_SDF = %s;\n\nconst lowp int NUM_MESHES = %d;\n"
             "const lowp int NUM_SDFS   = %d;\nconst lowp int NUM_MODELS = %d;\n\n"
             "const Mesh meshes[NUM_MESHES + NUM_SDFS + NUM_MODELS] = Mesh[](\n%s\n);\n\n"
             "const lowp int light_index[%d] = int[](\n%s\n);"
             % (b(n_meshes > 0), b(u_sphere), b(u_plane), b(u_box), b(n_sdfs > 0), n_meshes, n_sdfs, n_models,
                "\n".join(text), len(lights), ", ".join(str(x) for x in lights)))
    return scene, n_sdfs


SDF_PRIMS = ["sdBox", "udRoundBox", "sdSphere", "sdTriPrism", "sdCone", "MengerSponge", "Mandelbulb"]


def sdf_statement(i, kind):
    """index.html:702-717: SDF selector value -> the `#sdf_meshes` statement."""
    m = "meshes[NUM_MESHES + %d]" % i
    args = {0: "p-%s.pos, %s.joker.xyz" % (m, m), 1: "p-%s.pos, %s.joker.xyz, %s.joker.w" % (m, m, m),
            2: "p-%s.pos, %s.joker.x" % (m, m), 3: "p-%s.pos, %s.joker.xy" % (m, m),
            4: "p-%s.pos, %s.joker.xyz" % (m, m), 5: "p-%s.pos, %s.joker.xyz" % (m, m), 6: "p-%s.pos" % m}[kind]
    return "sdf_meshes[%d] = vec2(%s(%s), %.4f);" % (i, SDF_PRIMS[kind], args, i)


# ------------------------------------------------------------------ renderer
class Renderer:
    """Thin owner of one rt0 context (one GPU, one canvas)."""

    def __init__(self, width, height, device=0):
        h = ctypes.c_void_p()
        rc = lib().rt0_create(width, height, device, ctypes.byref(h))
        if rc != RT0_OK:
            raise Rt0Error(rc, "rt0_create(%d, %d, device=%d) failed (no HIP device?)" % (width, height, device))
        self.h = h
        self.width, self.height = width, height

    def _chk(self, rc):
        if rc != RT0_OK:
            raise Rt0Error(rc, lib().rt0_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            lib().rt0_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_config(self, cfg):
        self._chk(lib().rt0_set_config(self.h, ctypes.byref(cfg)))

    def get_config(self):
        cfg = Config()
        self._chk(lib().rt0_get_config(self.h, ctypes.byref(cfg)))
        return cfg

    def set_scene_glsl(self, scene_text, sdf_meshes=()):
        sdf = list(sdf_meshes)
        self._chk(lib().rt0_set_scene_glsl(self.h, scene_text.encode(), _strarr(sdf), len(sdf)))

    def get_scene(self):
        meshes = (Mesh * 128)()
        lights = (ctypes.c_int32 * 128)()
        ne, ns, nm, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(lib().rt0_get_scene(self.h, meshes, 128, ctypes.byref(ne), ctypes.byref(ns), ctypes.byref(nm),
                                      lights, 128, ctypes.byref(nl)))
        return list(meshes[:ne.value + ns.value + nm.value]), ne.value, ns.value, list(lights[:nl.value])

    def set_model(self, k, positions, triangles):
        """Triangle model k of the k-th TRIANGLE entry: float [nv, 3] object-space
        positions, int [nt, 3] vertex indices."""
        v = np.ascontiguousarray(positions, np.float32).reshape(-1, 3)
        t = np.ascontiguousarray(triangles, np.int32).reshape(-1, 3)
        self._chk(lib().rt0_set_model(self.h, k, v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), v.shape[0],
                                      t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), t.shape[0]))

    def model_info(self):
        """(triangles, BVH depth); builds the LBVH now if the scene/models changed."""
        n, d = ctypes.c_int(), ctypes.c_int()
        self._chk(lib().rt0_model_info(self.h, ctypes.byref(n), ctypes.byref(d)))
        return n.value, d.value

    def set_texture(self, unit, rgba8):
        """loadTexture (index.js:699-728): unit 0..3 = u_tex0..3, TEX_NOISE = u_rnd_tex.
        rgba8: uint8 [h, w, 4], first row = the image's top row; None unbinds."""
        if rgba8 is None:
            self._chk(lib().rt0_set_texture(self.h, unit, 0, 0, None))
            return
        a = np.ascontiguousarray(rgba8, np.uint8)
        if a.ndim != 3 or a.shape[2] != 4:
            raise ValueError("texture must be uint8 [h, w, 4]")
        self._chk(lib().rt0_set_texture(self.h, unit, a.shape[1], a.shape[0],
                                        a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))

    def set_cubemap(self, faces):
        """load_cubemap (index.js:298-331): six uint8 [n, n, 3] faces in the
        reference's order -X, -Y, -Z, +X, +Y, +Z (left, bottom, back, right,
        top, front); None unbinds."""
        if faces is None:
            self._chk(lib().rt0_set_cubemap(self.h, 0, None))
            return
        arrs = [np.ascontiguousarray(f, np.uint8) for f in faces]
        if len(arrs) != 6 or any(a.ndim != 3 or a.shape[2] != 3 or a.shape[:2] != arrs[0].shape[:2] or
                                 a.shape[0] != a.shape[1] for a in arrs):
            raise ValueError("six square uint8 [n, n, 3] faces expected")
        ptrs = (ctypes.POINTER(ctypes.c_uint8) * 6)(*[a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) for a in arrs])
        self._chk(lib().rt0_set_cubemap(self.h, arrs[0].shape[0], ptrs))

    def set_camera(self, pos, lookat, params):
        a = [np.asarray(v, np.float32) for v in (pos, lookat, params)]
        self._chk(lib().rt0_set_camera(self.h, *[_fp(x) for x in a]))

    def render(self, first_frame, n_passes, time_ms=0.0):
        self._chk(lib().rt0_render(self.h, first_frame, n_passes, time_ms))

    def set_temporal_frames(self, n):
        """u_temporalFrames: RENDER_MODE 1 running-average length (index.js:236)."""
        self._chk(lib().rt0_set_temporal_frames(self.h, int(n)))

    def set_viewport(self, x, y, w, h):
        """gl.viewport of the following passes (tile rendering); w or h <= 0 = whole canvas."""
        self._chk(lib().rt0_set_viewport(self.h, int(x), int(y), int(w), int(h)))

    def render_async(self, first_frame, n_passes, time_ms=0.0):
        self._chk(lib().rt0_render_async(self.h, first_frame, n_passes, time_ms))

    def sync(self):
        self._chk(lib().rt0_sync(self.h))

    def read_accum(self):
        out = np.empty((self.height, self.width, 4), np.float32)
        self._chk(lib().rt0_read_accum(self.h, _fp(out)))
        return out

    def write_accum(self, a):
        a = np.ascontiguousarray(a, np.float32)
        self._chk(lib().rt0_write_accum(self.h, _fp(a)))

    def clear(self):
        self._chk(lib().rt0_clear(self.h))

    def resize(self, w, h):
        self._chk(lib().rt0_resize(self.h, w, h))
        self.width, self.height = w, h

    def tonemap(self, contribution, mode=TONEMAP_GAMMA):
        """RGBA8 canvas (rows bottom-up, like the accumulator)."""
        out = np.empty((self.height, self.width, 4), np.uint8)
        self._chk(lib().rt0_tonemap_ex(self.h, contribution, mode, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def save_png(self, path, passes, mode=TONEMAP_GAMMA):
        """Tonemapped image (contribution 1/passes) as a top-down PNG."""
        png_write(path, self.tonemap(1.0 / max(1, passes), mode), flip_y=True)

    def save_pfm(self, path, passes):
        """HDR radiance (accumulator / passes) as PFM."""
        pfm_write(path, self.read_accum(), 1.0 / max(1, passes))

    def read_restir(self, which=0):
        m = np.empty((self.height, self.width, 4), np.float32)
        a = np.empty_like(m)
        self._chk(lib().rt0_read_restir(self.h, which, _fp(m), _fp(a)))
        return m, a

    def write_restir_inputs(self, spatial_main=None, spatial_aux=None, h1_main=None, h1_aux=None, h2_main=None,
                            h2_aux=None):
        arrs = [None if x is None else np.ascontiguousarray(x, np.float32)
                for x in (spatial_main, spatial_aux, h1_main, h1_aux, h2_main, h2_aux)]
        self._chk(lib().rt0_write_restir_inputs(self.h, *[_fp(x) for x in arrs]))

    def set_shard(self, shard, n_shards, band_rows=16):
        self._chk(lib().rt0_set_shard(self.h, shard, n_shards, band_rows))

    def device_accum(self):
        d, s = ctypes.c_void_p(), ctypes.c_void_p()
        self._chk(lib().rt0_device_accum(self.h, ctypes.byref(d), ctypes.byref(s)))
        return d.value, s.value

    def set_accum_buffer(self, dptr):
        """Use a caller-owned device buffer (e.g. torch tensor .data_ptr()) as accumulator."""
        self._chk(lib().rt0_set_accum_buffer(self.h, ctypes.c_void_p(dptr) if dptr else None))

    def set_accum_buffer_compact(self, dptr):
        """Band-packed caller-owned accumulator for a shard (after set_shard):
        rows x W x 4 f32 holding only the owned bands; returns rows."""
        rows = ctypes.c_int()
        self._chk(lib().rt0_set_accum_buffer_compact(self.h, ctypes.c_void_p(dptr), ctypes.byref(rows)))
        return rows.value

    def set_restir_buffers(self, dptrs):
        """Use caller-owned device memory (e.g. torch tensors) as the ReSTIR
        reservoir textures: four interleaved main/aux pair buffers of W*H*8
        f32, given as 8 plane pointers with dptrs[2k+1] = dptrs[2k] + 16 bytes
        (a (4, H, W, 2, 4) tensor's [k, :, :, 0] and [k, :, :, 1]); None
        returns to context-owned planes."""
        if dptrs is None:
            self._chk(lib().rt0_set_restir_buffers(self.h, None))
            return
        if len(dptrs) != 8:
            raise ValueError("8 reservoir planes expected")
        arr = (ctypes.c_void_p * 8)(*dptrs)
        self._chk(lib().rt0_set_restir_buffers(self.h, arr))

    def device_restir(self, which=0):
        """Device pointers (main, aux) of the reservoir planes the next pass reads:
        0 = newest output (spatial input), 1/2 = temporal history levels."""
        m, a = ctypes.c_void_p(), ctypes.c_void_p()
        self._chk(lib().rt0_device_restir(self.h, which, ctypes.byref(m), ctypes.byref(a)))
        return m.value, a.value

    def set_halo(self, rows):
        self._chk(lib().rt0_set_halo(self.h, rows))

    def halo_misses(self, reset=True):
        n = ctypes.c_uint32()
        self._chk(lib().rt0_read_halo_misses(self.h, ctypes.byref(n), int(bool(reset))))
        return n.value

    def set_jit(self, on):
        """Scene-specialised (hipRTC) kernels on/off (default on)."""
        self._chk(lib().rt0_set_jit(self.h, int(bool(on))))

    def set_executor_compat(self, on):
        """Reproduce the reference executor's g_final_reservoir stores after a
        `break` (rt0_set_executor_compat); default off = GLSL semantics."""
        self._chk(lib().rt0_set_executor_compat(self.h, int(bool(on))))

    def set_texture_filter(self, mode):
        """GL_LINEAR of the RGBA8 asset / noise textures (rt0_set_texture_filter):
        TEX_FILTER_FIXED16 (default, the reference executor's fixed-point
        filter) or TEX_FILTER_FLOAT (exact fp32 bilinear)."""
        self._chk(lib().rt0_set_texture_filter(self.h, int(mode)))

    def set_defer_light_sampling(self, on):
        """Deferred ReSTIR light sampling (rt0_set_defer_light_sampling);
        default on."""
        self._chk(lib().rt0_set_defer_light_sampling(self.h, int(bool(on))))

    def set_wavefront(self, mode):
        """Wavefront rounds (rt0_set_wavefront): 0 off, 1 / True SDF scenes
        (the default), 2 also ReSTIR scenes with triangle models."""
        self._chk(lib().rt0_set_wavefront(self.h, int(mode)))

    def set_counting(self, on):
        self._chk(lib().rt0_set_counting(self.h, int(bool(on))))

    COUNTER_NAMES = ("isect", "iter", "nee", "map", "samples", "restir", "restir_cand", "restir_ttap",
                     "restir_stap", "bvh_node", "tri")

    def counters(self):
        out = (ctypes.c_uint64 * len(self.COUNTER_NAMES))()
        rc = lib().rt0_read_counters_n(self.h, out, len(out))
        if rc < 0:
            self._chk(rc)
        return dict(zip(self.COUNTER_NAMES, list(out)))

    def samples_bytes(self):
        """Device scratch of frame-chunked launches (rt0_scratch_bytes)."""
        n = ctypes.c_size_t()
        self._chk(lib().rt0_scratch_bytes(self.h, ctypes.byref(n)))
        return n.value

    PATHS = {1: "aot", 2: "pass", 3: "deferred", 4: "wavefront"}

    def last_render_path(self):
        """Kernels of the last render (rt0_last_render_path): 'aot', 'pass',
        'deferred' or 'wavefront' (None before any render)."""
        return self.PATHS.get(lib().rt0_last_render_path(self.h))

    def last_kernel_ms(self):
        ms, n = ctypes.c_float(), ctypes.c_int()
        self._chk(lib().rt0_last_kernel_ms(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


class Vector3:
    """vector.js:2-95 (the camera only needs x/y/z)."""

    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = x, y, z

    def tolist(self):
        return [self.x, self.y, self.z]


class GlslViewport:
    """Drop-in for the reference's GlslViewport (index.js:3-1105) on the rt0 backend.

    Fields and defaults follow index.js:4-103; `render()` is one pass
    (u_frame = ++passes) exactly like index.js:986-1105, `render(n)` batches n
    passes into one kernel launch sequence.  Changing defines/constants/scene/
    sdf_meshes takes effect at the next render() (the reference needs an
    explicit recompile, index.html:1167)."""

    def __init__(self, canvas=None, opts=None, device=0):
        opts = opts or {}
        self.width = opts.get("width", 600)
        self.height = opts.get("height", 600)
        self.tile_rendering = opts.get("tile_rendering", False)
        self.defines = ["//#define USE_CUBEMAP", "#define USE_PROCEDURAL_SKY", "#define USE_BIASED_SAMPLING",
                        "//#define USE_BIDIRECTIONAL", "//#define USE_RESTIR", "//#define USE_SPECTRAL",
                        "//#define USE_VOLUMETRICS"]
        self.constants = list(STATIC_CONSTANTS)
        self.animatedConstants = list(ANIMATED_CONSTANTS)
        self.scene, _ = scene_from_lines(CORNELL_LINES)
        self.sdf_meshes = []
        self.camera = {"origin": Vector3(0.0, 0.0, 2.8), "lookat": Vector3(0.0, 0.0, -1.0), "fov": 50.0,
                       "aperture": 0.0, "focalLength": 3.5}
        self.passes = 0
        self.max_passes = opts.get("max_passes", float("inf"))
        self.animatedScene = False
        self.temporalFrames = 5
        self.loadTime = time.monotonic() * 1000.0  # u_time origin (index.js:986)
        self.paused = opts.get("paused", False)
        # tile rendering (index.js:97-103, 379): 32x32 viewports visited by updateTile()
        self.tile = [0, 0]
        self.tile_size = [32, 32]
        self.total_tiles = [-(-self.width // 32) - 1, -(-self.height // 32) - 1]
        self.viewport = [0, 0, 32, 32] if self.tile_rendering else [0, 0, self.width, self.height]
        self.renderer = Renderer(self.width, self.height, device)
        if opts.get("executorCompat"):  # reservoirs as the reference's GLES executor stores them
            self.renderer.set_executor_compat(True)
        if opts.get("textureFilter") is not None:  # TEX_FILTER_FIXED16 (default) / TEX_FILTER_FLOAT
            self.renderer.set_texture_filter(opts["textureFilter"])
        self._compiled = None
        self.images = {}
        # index.js:256-296: noise image (u_rnd_tex) + opts.textures[0..3]; paths or uint8 arrays
        if opts.get("rndTexture") is not None:
            self.loadTexture({"name": "rnd_tex"}, opts["rndTexture"])
        for i, t in enumerate(opts.get("textures", [])):
            self.loadTexture({"name": "tex%d" % i}, t)
        # index.js:298-331: six faces left, bottom, back, right, top, front (-X -Y -Z +X +Y +Z)
        if opts.get("cubemap") is not None:
            self.loadCubemap(opts["cubemap"])

    def loadCubemap(self, faces):
        """Six faces (paths or uint8 [n, n, 3|4] arrays) in the reference's order."""
        if faces is None:
            self.renderer.set_cubemap(None)
            return
        imgs = [image_read(f) if isinstance(f, str) else np.asarray(f, np.uint8) for f in faces]
        self.renderer.set_cubemap([a[..., :3] for a in imgs])
        for i, a in enumerate(imgs):
            self.images["cubemap_img%d" % i] = a

    def loadTexture(self, opts, img):
        """index.js:699-728 for the asset units (the framebuffers live in librt0)."""
        name = (opts or {}).get("name", "tex0")
        unit = TEX_NOISE if name == "rnd_tex" else int(name[3:])
        if isinstance(img, str):
            img = image_read(img)
        self.renderer.set_texture(unit, img)
        self.images["rnd_img" if unit == TEX_NOISE else "img%d" % unit] = img

    # index.js:384-440 -- uploads camera; here also (re)applies scene + flags
    def updateFrontTarget(self):
        key = (tuple(self.defines), tuple(self.constants), self.scene, tuple(self.sdf_meshes))
        if key != self._compiled:
            self.renderer.set_config(parse_config(self.defines, self.constants))
            self.renderer.set_scene_glsl(self.scene, self.sdf_meshes)
            self._compiled = key
        c = self.camera
        self.renderer.set_camera(c["origin"].tolist(), c["lookat"].tolist(),
                                 [c["fov"], c["aperture"], c["focalLength"]])

    def render(self, n_passes=1, time_ms=None):
        """index.js:986-1105: u_frame = ++passes per pass; accumulate.

        Animated mode (index.js:990-1005) keeps the pass counter cycling
        (passes > 2*temporalFrames -> temporalFrames) so the ReSTIR history
        stays valid, and every pass sees u_time = ms since construction (or
        `time_ms`)."""
        self.updateFrontTarget()
        vp = self.viewport if self.tile_rendering else [0, 0, self.width, self.height]
        self.renderer.set_viewport(*vp)
        t = (time.monotonic() * 1000.0 - self.loadTime) if time_ms is None else float(time_ms)
        if not self.animatedScene:
            first = self.passes + 1
            self.renderer.render(first, n_passes, t)
            self.passes += n_passes
            return
        self.renderer.set_temporal_frames(self.temporalFrames)
        for _ in range(n_passes):
            if self.passes > self.temporalFrames * 2:
                self.passes = self.temporalFrames
            self.passes += 1
            self.renderer.render(self.passes, 1, t)

    def clear(self):
        """index.js:822-880."""
        self.renderer.clear()

    def updateTile(self):
        """index.js:761-792: the next 32x32 viewport (row-major, bottom-up), passes
        restart at 0, and the viewer pauses after the last tile.  As in the
        reference, the edge tile's extent is written through `tile_max`, which is
        the tile_size list itself, so it persists for the following tiles."""
        tile_max = self.tile_size
        self.passes = 0
        if self.tile[0] < self.total_tiles[0]:
            self.tile[0] += 1
            if self.tile[0] == self.total_tiles[0] - 1:
                tile_max[0] = abs(self.width - self.total_tiles[0] * self.tile_size[0])
        else:
            self.tile[0] = 0
            if self.tile[1] < self.total_tiles[1]:
                self.tile[1] += 1
                if self.tile[1] == self.total_tiles[1] - 1:
                    tile_max[1] = abs(self.height - self.total_tiles[1] * self.tile_size[1])
            else:
                self.paused = True
                self.tile[1] = 0
        self.viewport = [self.tile[0] * self.tile_size[0], self.tile[1] * self.tile_size[1], tile_max[0], tile_max[1]]

    def resize(self, v):
        """index.js:471-493: v selects 256..8192 square canvases."""
        size = {0: 256, 1: 512, 2: 1024, 3: 2048, 4: 4096, 5: 8192}.get(v, v)
        self.width = self.height = size
        self.renderer.resize(size, size)
        self.passes = 0
        self.total_tiles = [-(-size // self.tile_size[0]) - 1, -(-size // self.tile_size[1]) - 1]

    def toggleReSTIR(self):
        """index.js:911-927: force USE_RESTIR, use_restir and sample_lights on
        (picked up by the next render(); the reference needs a recompile)."""
        self.defines[4] = "#define USE_RESTIR"
        self.constants[9] = "const bool use_restir = true;"
        self.constants[7] = "const bool sample_lights = true;"

    def getReSTIRDebugInfo(self):
        """index.js:930-938 (the reference reports ReSTIR as active exactly in animated mode)."""
        return {"isReSTIREnabled": self.animatedScene, "temporalFrames": self.temporalFrames,
                "passes": self.passes, "animatedMode": self.animatedScene, "debugViewActive": False}

    def setAnimatedMode(self, is_animated):
        """index.js:940-983: animated constants (RENDER_MODE 1, ReSTIR) or the static ones."""
        self.animatedScene = bool(is_animated)
        if is_animated:
            self.constants = list(self.animatedConstants)
            self.defines[4] = "#define USE_RESTIR"
        else:
            self.constants = list(STATIC_CONSTANTS)
            self.defines[4] = "//#define USE_RESTIR"
        self.clear()

    def accumulator(self):
        return self.renderer.read_accum()

    def image(self):
        """Display pass, tonemapper.glsl:28-33 with u_cont = 1/passes, or 1 for the
        animated running average (index.js:1080-1090)."""
        return self.renderer.tonemap(1.0 if self.animatedScene else 1.0 / max(1, self.passes))


STATIC_CONSTANTS = ["const lowp int MAX_BOUNCES = 12;", "const lowp int MAX_DIFF_BOUNCES = 4;",
                    "const lowp int MAX_SPEC_BOUNCES = 4;", "const lowp int MAX_TRANS_BOUNCES = 12;",
                    "const lowp int MAX_SCATTERING_EVENTS = 12;", "const mediump int MARCHING_STEPS = 128;",
                    "const lowp float FUDGE_FACTOR = 0.9;", "const bool sample_lights = true;",
                    "const bool use_mis = false;", "const bool use_restir = false;",
                    "const lowp int LIGHT_PATH_LENGTH = 2;", "const lowp int RESTIR_SAMPLES = 16;",
                    "const lowp int RENDER_MODE = 0;"]
ANIMATED_CONSTANTS = ["const lowp int MAX_BOUNCES = 6;", "const lowp int MAX_DIFF_BOUNCES = 2;",
                      "const lowp int MAX_SPEC_BOUNCES = 2;", "const lowp int MAX_TRANS_BOUNCES = 4;",
                      "const lowp int MAX_SCATTERING_EVENTS = 4;", "const mediump int MARCHING_STEPS = 64;",
                      "const lowp float FUDGE_FACTOR = 0.9;", "const bool sample_lights = true;",
                      "const bool use_mis = false;", "const bool use_restir = true;",
                      "const lowp int LIGHT_PATH_LENGTH = 1;", "const lowp int RESTIR_SAMPLES = 8;",
                      "const lowp int RENDER_MODE = 1;"]
# index.js:54-85 default scene (Cornell box) in the textarea grammar
CORNELL_LINES = ["MAT_CORNELL_WHITE, PLANE,  vec3( 0.0, 1.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_WHITE, PLANE,  vec3( 0.0,-1.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_WHITE, PLANE,  vec3( 0.0, 0.0, 1.0), vec4(2.5, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_RED,   PLANE,  vec3( 1.0, 0.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_GREEN, PLANE,  vec3(-1.0, 0.0, 0.0), vec4(1.5, 0.0, 0.0, 0.0)",
                 "MAT_LIGHT_4,       SPHERE, vec3( 0.0, 1.4,-1.2), vec4(0.3, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_WHITE, BOX,    vec3( 0.5,-1.0,-1.8), vec4(1.0, 0.0, 0.0, 0.0)",
                 "MAT_CORNELL_WHITE, BOX,    vec3(-0.45,-1.15,-1.3), vec4(0.7, 0.0, 0.0, 0.0)"]


def config_strings(cfg):
    """configs.json entry -> (defines, constants) string arrays in GlslViewport's format."""
    d = ["//#define USE_CUBEMAP", "#define USE_PROCEDURAL_SKY", "#define USE_BIASED_SAMPLING",
         "//#define USE_BIDIRECTIONAL", "//#define USE_RESTIR", "//#define USE_SPECTRAL", "//#define USE_VOLUMETRICS"]
    for k, v in cfg.get("defines", {}).items():
        d[DEFINE_NAMES.index(k)] = ("" if v else "//") + "#define " + k
    consts = list(STATIC_CONSTANTS)
    for k, v in cfg.get("constants", {}).items():
        for i, s in enumerate(consts):
            if (" %s " % k) in s:
                val = ("true" if v else "false") if isinstance(v, bool) else str(v)
                consts[i] = s.split("=")[0] + "= " + val + ";"
                break
        else:
            raise KeyError(k)
    return d, consts


def scene_strings(cfg, cfgs):
    """configs.json entry -> (scene text, sdf_meshes statements)."""
    lines = cfg["scene_lines"] or cfgs["cornell_lines"]
    scene, ns = scene_from_lines(lines)
    kinds = cfg.get("sdf_kinds") or []
    return scene, [sdf_statement(i, kinds[i] if i < len(kinds) else 0) for i in range(ns)]


def configure(renderer, cfg, cfgs):
    """Apply one tests/golden/configs.json entry (scene lines, overrides, camera) to a Renderer."""
    renderer.set_config(parse_config(*config_strings(cfg)))
    renderer.set_scene_glsl(*scene_strings(cfg, cfgs))
    cam = cfg.get("camera") or cfgs["default_camera"]
    renderer.set_camera(cam["origin"], cam["lookat"], [cam["fov"], cam["aperture"], cam["focalLength"]])
