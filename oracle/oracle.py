"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the CPU parity oracle.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module. It wraps ``oracle/_build/libatr_oracle.so`` (built from
``oracle/atr_oracle.c`` by ``oracle/Makefile``), a plain-C restatement of the reference
render path; see that file's header for the per-function reference citations and for
how parity is pinned (SURVEY.md 8(c) probe hashes; DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libatr_oracle.so")

# app.cpp:88-105 constants (benchmark scene)
APP_EYE = (0.1, 2.0, 0.0)
APP_FACING = (-0.1, -0.5, -1.0)
SKY = ((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3)
MODEL_MAT = ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)


class ov3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class om_mesh(C.Structure):
    _fields_ = [("vertices", C.POINTER(ov3)), ("nv", C.c_uint32),
                ("normals", C.POINTER(ov3)), ("nn", C.c_uint32),
                ("texcoords", C.POINTER(ov3)), ("nt", C.c_uint32),
                ("face_v", C.POINTER(C.c_int32)), ("face_tc", C.POINTER(C.c_int32)),
                ("face_n", C.POINTER(C.c_int32)), ("nf", C.c_uint32)]


class om_node(C.Structure):
    _fields_ = [("bmin", C.c_float * 3), ("bmax", C.c_float * 3), ("children", C.c_int32),
                ("prim_off", C.c_uint32), ("prim_cnt", C.c_uint32)]


class om_tree(C.Structure):
    _fields_ = [("nodes", C.POINTER(om_node)), ("nnodes", C.c_int32),
                ("prim_tri", C.POINTER(C.c_float)), ("prim_face", C.POINTER(C.c_uint32)),
                ("nprims", C.c_uint32), ("max_faces", C.c_uint32)]


class om_material(C.Structure):
    _fields_ = [("emission", ov3), ("reflection", ov3), ("scatter", C.c_float)]


class om_sphere(C.Structure):
    _fields_ = [("center", ov3), ("radius", C.c_float), ("material", C.c_int32)]


class om_plane(C.Structure):
    _fields_ = [("normal", ov3), ("distance", C.c_float), ("material", C.c_int32)]


class om_model(C.Structure):
    _fields_ = [("mesh", C.POINTER(om_mesh)), ("tree", C.POINTER(om_tree)),
                ("surrounding_aabb", C.c_float * 6), ("material", C.c_int32)]


class om_scene(C.Structure):
    _fields_ = [("materials", C.POINTER(om_material)), ("nmaterials", C.c_int32),
                ("models", C.POINTER(om_model)), ("nmodels", C.c_int32),
                ("spheres", C.POINTER(om_sphere)), ("nspheres", C.c_int32),
                ("planes", C.POINTER(om_plane)), ("nplanes", C.c_int32)]


class om_camera(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("anti_aliasing", C.c_int32),
                ("spp", C.c_uint32), ("bounce_limit", C.c_int32), ("aspect_ratio", C.c_float),
                ("camera_z", ov3), ("camera_x", ov3), ("camera_y", ov3), ("eye", ov3),
                ("frame_center", ov3), ("h_fov", C.c_float), ("half_pixel_width", C.c_float),
                ("half_pixel_height", C.c_float)]


class om_counters(C.Structure):
    _fields_ = [("n_rays", C.c_uint64), ("n_box", C.c_uint64), ("n_tri", C.c_uint64),
                ("n_leaf", C.c_uint64), ("n_hit", C.c_uint64), ("n_raycasts_ref", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "atr_oracle.c")):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.om_parse_obj.argtypes = [C.c_char_p, C.c_size_t, P(om_mesh)]
        L.om_load_obj.argtypes = [C.c_char_p, P(om_mesh)]
        L.om_free_mesh.argtypes = [P(om_mesh)]
        L.om_get_aabb.argtypes = [P(om_mesh), C.c_float * 6]
        L.om_translate_to.argtypes = [P(om_mesh), C.c_float * 6, ov3]
        L.om_build_tree.argtypes = [P(om_mesh), C.c_uint32, P(om_tree)]
        L.om_free_tree.argtypes = [P(om_tree)]
        L.om_set_camera.argtypes = [P(om_camera), ov3, ov3, C.c_int32, C.c_int32, C.c_int32,
                                    C.c_uint32, C.c_int32, C.c_float]
        L.om_primary_hits.argtypes = [P(om_scene), P(om_camera), C.c_int32, C.c_int32,
                                      C.c_void_p, C.c_void_p, P(om_counters)]
        L.om_primary_leaf_trace.argtypes = [P(om_scene), P(om_camera), C.c_int32, C.c_int32,
                                            C.c_int32, C.c_void_p, C.c_void_p]
        L.om_trace_rays.argtypes = [P(om_scene), C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_void_p, C.c_void_p, C.c_void_p, P(om_counters)]
        L.om_render_rows.argtypes = [P(om_scene), P(om_camera), C.c_uint64, C.c_int32, C.c_int32,
                                     C.c_void_p, C.c_void_p, C.c_void_p, P(om_counters)]
        L.om_render_threaded.argtypes = [P(om_scene), P(om_camera), C.c_uint64, C.c_int32,
                                         C.c_void_p, P(C.c_int64), P(C.c_uint64)]
        L.om_render_threaded.restype = C.c_double
        L.om_render_rows_threaded.argtypes = [P(om_scene), P(om_camera), C.c_uint64, C.c_int32, C.c_int32,
                                              C.c_int32, C.c_int32, P(C.c_uint64), P(C.c_int64)]
        L.om_render_rows_threaded.restype = C.c_double
        L.om_make_tiles.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32]
        L.om_make_tiles.restype = C.c_int32
        L.om_pcg_u32.argtypes = [P(C.c_uint64), C.c_uint64]
        L.om_pcg_u32.restype = C.c_uint32
        L.om_path_rng.argtypes = [C.c_uint64, C.c_int64, C.c_uint32, P(C.c_uint64), P(C.c_uint64)]
        _lib = L
    return _lib


def _v(t):
    return ov3(float(t[0]), float(t[1]), float(t[2]))


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class Camera:
    """set_camera (camera.h:40-45) with the app's eye/facing by default."""

    def __init__(self, width, height, spp=1, bounces=1, aa=False, eye=APP_EYE, facing=APP_FACING,
                 h_fov=1.0):
        self.c = om_camera()
        lib().om_set_camera(C.byref(self.c), _v(eye), _v(facing), int(width), int(height),
                            int(bool(aa)), int(spp), int(bounces), float(h_fov))

    @property
    def width(self):
        return self.c.width

    @property
    def height(self):
        return self.c.height


class Scene:
    """One-model scene as the app builds it (app.cpp:65-146): load OBJ, surrounding AABB,
    translate_to(center), SAH octree with leaf size ``max_faces`` (or brute force)."""

    def __init__(self, obj_path=None, obj_text=None, center=(0.0, -15.0, -38.0), max_faces=300,
                 use_tree=True, materials=(SKY, MODEL_MAT), model_material=1, spheres=(),
                 planes=()):
        L = lib()
        self.mesh = om_mesh()
        if obj_text is not None:
            b = obj_text.encode() if isinstance(obj_text, str) else bytes(obj_text)
            L.om_parse_obj(b, len(b), C.byref(self.mesh))
        else:
            if L.om_load_obj(os.fsencode(obj_path), C.byref(self.mesh)) != 0:
                raise FileNotFoundError(obj_path)
        box = (C.c_float * 6)()
        L.om_get_aabb(C.byref(self.mesh), box)
        if center is not None:
            L.om_translate_to(C.byref(self.mesh), box, _v(center))
        self.surrounding_aabb = np.array(list(box), dtype=np.float32)
        self.tree = None
        if use_tree:
            self.tree = om_tree()
            L.om_build_tree(C.byref(self.mesh), int(max_faces), C.byref(self.tree))
        self._mats = (om_material * len(materials))(
            *[om_material(_v(e), _v(r), float(s)) for e, r, s in materials])
        self._model = om_model()
        self._model.mesh = C.pointer(self.mesh)
        self._model.tree = C.pointer(self.tree) if self.tree is not None else None
        for i in range(6):
            self._model.surrounding_aabb[i] = box[i]
        self._model.material = int(model_material)
        self._spheres = (om_sphere * max(1, len(spheres)))(
            *[om_sphere(_v(c), float(r), int(m)) for c, r, m in spheres])
        self._planes = (om_plane * max(1, len(planes)))(
            *[om_plane(_v(n), float(d), int(m)) for n, d, m in planes])
        self.s = om_scene(self._mats, len(materials), C.pointer(self._model), 1,
                          self._spheres, len(spheres), self._planes, len(planes))

    # ---- introspection ------------------------------------------------------------
    def mesh_arrays(self):
        m = self.mesh
        V = np.ctypeslib.as_array(C.cast(m.vertices, C.POINTER(C.c_float)), (m.nv * 3,)).reshape(-1, 3).copy() if m.nv else np.zeros((0, 3), np.float32)
        N = np.ctypeslib.as_array(C.cast(m.normals, C.POINTER(C.c_float)), (m.nn * 3,)).reshape(-1, 3).copy() if m.nn else np.zeros((0, 3), np.float32)
        FV = np.ctypeslib.as_array(m.face_v, (m.nf * 3,)).reshape(-1, 3).copy() if m.nf else np.zeros((0, 3), np.int32)
        FN = np.ctypeslib.as_array(m.face_n, (m.nf * 3,)).reshape(-1, 3).copy() if m.nf else np.zeros((0, 3), np.int32)
        return V, N, FV, FN

    def tree_arrays(self):
        t = self.tree
        nodes = np.ctypeslib.as_array(C.cast(t.nodes, C.POINTER(C.c_uint8)),
                                      (t.nnodes * C.sizeof(om_node),)).view(
            np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("children", "<i4"),
                      ("prim_off", "<u4"), ("prim_cnt", "<u4")])).copy()
        tri = np.ctypeslib.as_array(t.prim_tri, (max(1, t.nprims) * 9,)).reshape(-1, 9)[:t.nprims].copy()
        face = np.ctypeslib.as_array(t.prim_face, (max(1, t.nprims),))[:t.nprims].copy()
        return nodes, tri, face

    def tree_stats(self):
        nodes, _, _ = self.tree_arrays()
        leaf = nodes["children"] == 0
        return {"nodes": int(len(nodes)), "inner": int((~leaf).sum()), "leaves": int(leaf.sum()),
                "empty_leaves": int((leaf & (nodes["prim_cnt"] == 0)).sum()),
                "leaf_prim_refs": int(nodes["prim_cnt"][leaf].sum()),
                "max_leaf": int(nodes["prim_cnt"][leaf].max()) if leaf.any() else 0}

    # ---- hot path -------------------------------------------------------------------
    def primary_hits(self, cam: Camera, y0=0, y1=None):
        y1 = cam.height if y1 is None else y1
        n = (y1 - y0) * cam.width
        face = np.empty(n, np.uint32)
        t = np.empty(n, np.float32)
        ctr = om_counters()
        lib().om_primary_hits(C.byref(self.s), C.byref(cam.c), y0, y1, _ptr(face), _ptr(t),
                              C.byref(ctr))
        return face.reshape(y1 - y0, cam.width), t.reshape(y1 - y0, cam.width), ctr.as_dict()

    def leaf_trace(self, cam: Camera, cap=64):
        """Per pixel: the leaves its primary ray scans (in order) and its triangle tests."""
        n = cam.width * cam.height
        leaves = np.empty((n, cap), np.int32)
        ntri = np.empty(n, np.uint32)
        lib().om_primary_leaf_trace(C.byref(self.s), C.byref(cam.c), 0, cam.height, cap,
                                    _ptr(leaves), _ptr(ntri))
        return leaves.reshape(cam.height, cam.width, cap), ntri.reshape(cam.height, cam.width)

    def trace(self, orig, dirs):
        orig = np.ascontiguousarray(orig, np.float32)
        dirs = np.ascontiguousarray(dirs, np.float32)
        n = len(orig)
        face = np.empty(n, np.uint32)
        t = np.empty(n, np.float32)
        uv = np.empty((n, 2), np.float32)
        ctr = om_counters()
        lib().om_trace_rays(C.byref(self.s), _ptr(orig), _ptr(dirs), n, _ptr(face), _ptr(t),
                            _ptr(uv), C.byref(ctr))
        return face, t, uv, ctr.as_dict()

    def render(self, cam: Camera, seed: int, y0=0, y1=None):
        y1 = cam.height if y1 is None else y1
        n = (y1 - y0) * cam.width
        rgb = np.empty((n, 3), np.float32)
        fb = np.empty(n, np.uint32)
        casts = np.empty(n, np.uint32)
        ctr = om_counters()
        lib().om_render_rows(C.byref(self.s), C.byref(cam.c), C.c_uint64(seed), y0, y1, _ptr(rgb),
                             _ptr(fb), _ptr(casts), C.byref(ctr))
        shp = (y1 - y0, cam.width)
        return rgb.reshape(shp + (3,)), fb.reshape(shp), casts.reshape(shp), ctr.as_dict()

    def render_rows_threaded(self, cam: Camera, seed: int, threads: int, row0: int, row_step: int, nrows: int):
        """(seconds, traced rays, ray_casts) of a strided row sample on `threads` threads."""
        traced = C.c_uint64(0)
        casts = C.c_int64(0)
        secs = lib().om_render_rows_threaded(C.byref(self.s), C.byref(cam.c), C.c_uint64(seed), int(threads),
                                             int(row0), int(row_step), int(nrows), C.byref(traced), C.byref(casts))
        return secs, int(traced.value), int(casts.value)

    def render_threaded(self, cam: Camera, seed: int, threads: int):
        fb = np.zeros(cam.width * cam.height, np.uint32)
        tot = C.c_int64(0)
        traced = C.c_uint64(0)
        secs = lib().om_render_threaded(C.byref(self.s), C.byref(cam.c), C.c_uint64(seed),
                                        int(threads), _ptr(fb), C.byref(tot), C.byref(traced))
        return secs, fb.reshape(cam.height, cam.width), int(tot.value), int(traced.value)

    def __del__(self):
        try:
            L = lib()
            if self.tree is not None:
                L.om_free_tree(C.byref(self.tree))
            L.om_free_mesh(C.byref(self.mesh))
        except Exception:
            pass


def make_tiles(width, height, threads):
    buf = np.zeros(4 * 65536, np.int32)
    n = lib().om_make_tiles(width, height, threads, _ptr(buf), 65536)
    return buf[:4 * n].reshape(n, 4).copy()


def pcg_sequence(state, stream, n):
    st = C.c_uint64(state)
    return [lib().om_pcg_u32(C.byref(st), C.c_uint64(stream)) for _ in range(n)]


def fnv_hits(face, t):
    """The survey probe's hash: 64-bit FNV over whole u32 words,
    h = (h ^ face) * P; h = (h ^ tbits) * P, pixels in row order from y = 0."""
    h = 1469598103934665603
    P = 1099511628211
    M = (1 << 64) - 1
    f = np.asarray(face, np.uint32).ravel()
    tb = np.asarray(t, np.float32).ravel().view(np.uint32)
    inter = np.empty(2 * len(f), np.uint64)
    inter[0::2] = f
    inter[1::2] = tb
    for w in inter.tolist():
        h = ((h ^ w) * P) & M
    return h
