"""ctypes binding of the C-ABI in ``include/atray.h`` (``atray_amd/_lib/libatray_hip.so``).

The HIP library is the product path: there is no CPU fallback. Loading fails loudly if the
library was not built (``__graft_entry__.build()`` / ``make -C atray_amd/csrc``).

torch is imported before the library is loaded so that both bind the same HIP runtime
(torch's bundled ``libamdhip64.so`` carries the SONAME ``libamdhip64.so.7`` that the library
needs); torch then provides device memory, streams and ``torch.distributed`` (RCCL).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ATRAY_LIB") or os.path.join(HERE, "_lib", "libatray_hip.so")  # ATRAY_LIB: experiment builds only

ATR_LAYOUT_IMAGE = 0
ATR_LAYOUT_PACKED = 1
ATR_PLAN_PRIO = 0x80  # cell plan: raised issue priority (atr_set_cell_plan)


def plan_class(c):
    """Cell plan dispatch class (ATR_PLAN_CLASS): class 7 cells are dispatched first, class 0 last."""
    return (int(c) & 7) << 4
ATR_KERNEL_AUTO, ATR_KERNEL_LANE = 0, 1
ATR_KERNEL_FLAT = 8
ATR_KERNEL_HYBRID = 9
ATR_KERNEL_PATHS = 10
# the kernel variants of the shipping library (atray.h); AUTO picks HYBRID or PATHS
VARIANTS = (ATR_KERNEL_LANE, ATR_KERNEL_FLAT, ATR_KERNEL_HYBRID, ATR_KERNEL_PATHS)
MISS = 0xFFFFFFFF
MAX_FLOAT = np.float32(3.402823466e38)

ERRORS = {-1: "ATR_E_INVALID", -2: "ATR_E_IO", -3: "ATR_E_NOMEM", -4: "ATR_E_NOSCENE",
          -5: "ATR_E_TREE_DEPTH", -6: "ATR_E_TREE_LAYOUT"}


class AtrError(RuntimeError):
    pass


def check(rc, what=""):
    if rc < 0:
        name = ERRORS.get(rc) or (f"hipError {-rc - 1000}" if rc <= -1000 else str(rc))
        raise AtrError(f"{what}: {name}")
    return rc


class atr_vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class atr_material(C.Structure):
    _fields_ = [("emission", atr_vec3), ("reflection", atr_vec3), ("scatter", C.c_float)]


class atr_model(C.Structure):
    _fields_ = [("mesh", C.c_void_p), ("tree", C.c_void_p), ("surrounding_aabb", C.c_float * 6),
                ("material", C.c_int32)]


class atr_sphere(C.Structure):
    _fields_ = [("center", atr_vec3), ("radius", C.c_float), ("material", C.c_int32)]


class atr_plane(C.Structure):
    _fields_ = [("normal", atr_vec3), ("distance", C.c_float), ("material", C.c_int32)]


class atr_camera(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("anti_aliasing", C.c_int32),
                ("samples_per_pixel", C.c_uint32), ("bounce_limit", C.c_int32),
                ("aspect_ratio", C.c_float), ("camera_z", atr_vec3), ("camera_x", atr_vec3),
                ("camera_y", atr_vec3), ("eye", atr_vec3), ("frame_center", atr_vec3),
                ("h_fov", C.c_float), ("half_pixel_width", C.c_float),
                ("half_pixel_height", C.c_float)]


class atr_tile(C.Structure):
    _fields_ = [("min_x", C.c_int32), ("min_y", C.c_int32), ("max_x", C.c_int32),
                ("max_y", C.c_int32)]


class atr_frame(C.Structure):
    _fields_ = [("layout", C.c_int32), ("framebuffer", C.c_void_p), ("hit_face", C.c_void_p),
                ("hit_t", C.c_void_p), ("rgb", C.c_void_p), ("ray_casts", C.c_void_p),
                ("traced_rays", C.c_void_p)]


class atr_tuning(C.Structure):
    _fields_ = [("xcd_chunk", C.c_int32), ("frame_rotate", C.c_int32), ("hybrid_a", C.c_int32),
                ("hybrid_b", C.c_int32), ("path_batch_log2", C.c_int32), ("cluster_size", C.c_int32),
                ("frame_plan", C.c_int32), ("path_camera_occ", C.c_int32), ("path_bounce_occ", C.c_int32),
                ("primary_occ", C.c_int32), ("path_sort_bits", C.c_int32), ("path_split", C.c_int32),
                ("reserved", C.c_int32 * 4)]


# every symbol include/atray.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = [
    "atr_mesh_load_obj", "atr_mesh_parse_obj", "atr_mesh_from_arrays", "atr_mesh_free",
    "atr_mesh_info", "atr_mesh_aabb", "atr_mesh_translate_to", "atr_octree_build", "atr_octree_build_device",
    "atr_octree_from_nodes", "atr_octree_free", "atr_octree_export", "atr_octree_stats", "atr_camera_set",
    "atr_make_tiles", "atr_make_shard_tiles", "atr_create", "atr_destroy", "atr_version",
    "atr_scene_upload", "atr_scene_info", "atr_render_start", "atr_render_start_ex",
    "atr_render_counters", "atr_render_tile_costs", "atr_balance_shard_tiles",
    "atr_render_packed_size", "atr_packed_pixel_map", "atr_unpack", "atr_tile_ray_casts", "atr_render_wait",
    "atr_last_kernel_ms", "atr_device_alloc", "atr_device_free", "atr_memcpy_d2h", "atr_memcpy_h2d",
    "atr_memset_d", "atr_render_start_progressive", "atr_write_bmp", "atr_render_start_frames",
    "atr_render_start_cameras", "atr_mesh_load_obj_threaded", "atr_mesh_parse_obj_threaded",
    "atr_mesh_export", "atr_packed_tile_ray_casts", "atr_set_cell_plan", "atr_render_cell_costs",
    "atr_default_tuning", "atr_set_tuning", "atr_get_tuning", "atr_pack_bgr", "atr_scatter_bgr",
    "atr_pack_bgr_masked_bound", "atr_pack_bgr_masked", "atr_scatter_bgr_masked", "atr_unpack_masked",
    "atr_unpack_masked_ranks",
    "atr_render_plan_info", "atr_workspace_info",
]
# the diagnostic build's extra symbols (include/atray_diag.h; make -C atray_amd/csrc DIAG=1)
DIAG_EXPORTS = ["atr_render_wave_trace", "atr_render_phase_clocks", "atr_render_path_counters",
                "atr_render_simd_counters"]

_lib = None


def lib():
    """Load the HIP engine library (torch first: shared HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (binds libamdhip64.so.7 before our library needs it)
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"atray HIP engine not built: {LIB_PATH} missing "
                          "(run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, vp, i32, u32, i64 = C.POINTER, C.c_void_p, C.c_int32, C.c_uint32, C.c_int64
    sig = {
        "atr_mesh_load_obj": ([C.c_char_p, P(vp)], C.c_int),
        "atr_mesh_parse_obj": ([C.c_char_p, C.c_size_t, P(vp)], C.c_int),
        "atr_mesh_load_obj_threaded": ([C.c_char_p, i32, P(vp)], C.c_int),
        "atr_mesh_parse_obj_threaded": ([C.c_char_p, C.c_size_t, i32, P(vp)], C.c_int),
        "atr_mesh_from_arrays": ([vp, u32, vp, u32, vp, u32, vp, P(vp)], C.c_int),
        "atr_mesh_free": ([vp], None),
        "atr_mesh_info": ([vp, P(u32), P(u32), P(u32)], C.c_int),
        "atr_mesh_export": ([vp, vp, vp, vp, P(u32), vp, vp, vp], C.c_int),
        "atr_mesh_aabb": ([vp, C.c_float * 6], C.c_int),
        "atr_mesh_translate_to": ([vp, C.c_float * 6, atr_vec3], C.c_int),
        "atr_octree_build": ([vp, u32, P(vp)], C.c_int),
        "atr_octree_build_device": ([vp, u32, i32, P(vp), vp], C.c_int),
        "atr_octree_from_nodes": ([i32, vp, vp, vp, vp, u32, vp, vp, P(vp)], C.c_int),
        "atr_octree_free": ([vp], None),
        "atr_octree_export": ([vp, vp, vp, vp, vp, vp, vp], C.c_int),
        "atr_octree_stats": ([vp, i64 * 7], C.c_int),
        "atr_camera_set": ([P(atr_camera), atr_vec3, atr_vec3, i32, i32, i32, u32, i32, C.c_float], C.c_int),
        "atr_make_tiles": ([i32, i32, i32, vp, i32], i32),
        "atr_make_shard_tiles": ([i32, i32, i32, i32, i32, vp, i32], i32),
        "atr_balance_shard_tiles": ([i32, i32, i32, i32, vp, i64, vp], i32),
        "atr_create": ([C.c_int, P(vp)], C.c_int),
        "atr_destroy": ([vp], C.c_int),
        "atr_version": ([], C.c_char_p),
        "atr_scene_upload": ([vp, vp, i32, vp, i32, vp, i32, vp, i32], C.c_int),
        "atr_scene_info": ([vp, P(i64), P(i32), P(i32)], C.c_int),
        "atr_workspace_info": ([vp, P(i32), P(i64)], C.c_int),
        "atr_render_start": ([vp, P(atr_camera), vp, i32, P(atr_frame), C.c_uint64, vp], C.c_int),
        "atr_render_start_ex": ([vp, P(atr_camera), vp, i32, P(atr_frame), C.c_uint64, vp, i32], C.c_int),
        "atr_render_packed_size": ([vp, i32], i64),
        "atr_render_counters": ([vp, P(atr_camera), vp, i32, C.c_uint64, i32, i64 * 10], C.c_int),
        "atr_render_tile_costs": ([vp, P(atr_camera), vp, i32, C.c_uint64, vp], C.c_int),
        "atr_render_wave_trace": ([vp, P(atr_camera), vp, i32, C.c_uint64, i32, vp, i64, P(i64)], C.c_int),
        "atr_packed_pixel_map": ([vp, i32, i32, i32, vp, i64], i64),
        "atr_unpack": ([vp, vp, i32, i32, vp, vp, vp], C.c_int),
        "atr_tile_ray_casts": ([vp, vp, i32, i32, vp, vp, vp], C.c_int),
        "atr_packed_tile_ray_casts": ([vp, vp, i32, i32, i32, vp, i32, i64, vp, vp], C.c_int),
        "atr_set_cell_plan": ([vp, i32, i32, vp], C.c_int),
        "atr_render_phase_clocks": ([vp, P(atr_camera), vp, i32, C.c_uint64, i32, vp], C.c_int),
        "atr_default_tuning": ([P(atr_tuning)], None),
        "atr_set_tuning": ([vp, P(atr_tuning)], C.c_int),
        "atr_get_tuning": ([vp, P(atr_tuning)], C.c_int),
        "atr_pack_bgr": ([vp, vp, i64, vp, vp], C.c_int),
        "atr_render_plan_info": ([vp, vp, i32, i32, i32, vp, vp, i64, vp, P(i64)], C.c_int),
        "atr_scatter_bgr": ([vp, vp, i64, vp, vp, vp], C.c_int),
        "atr_pack_bgr_masked_bound": ([i64], i64),
        "atr_pack_bgr_masked": ([vp, vp, i64, u32, vp, vp, vp], C.c_int),
        "atr_scatter_bgr_masked": ([vp, vp, i64, vp, vp, vp], C.c_int),
        "atr_unpack_masked": ([vp, vp, i32, i32, i32, vp, i32, vp, i64, vp], C.c_int),
        "atr_unpack_masked_ranks": ([vp, i32, vp, vp, i32, i32, vp, vp, i32, vp, i64, vp], C.c_int),
        "atr_render_simd_counters": ([vp, P(atr_camera), vp, i32, C.c_uint64, i32, vp], C.c_int),
        "atr_render_path_counters": ([vp, P(atr_camera), vp, i32, C.c_uint64, i32, vp], C.c_int),
        "atr_render_cell_costs": ([vp, P(atr_camera), C.c_uint64, i32, vp], C.c_int),
        "atr_render_wait": ([vp, u32, P(i32)], C.c_int),
        "atr_render_start_progressive": ([vp, P(atr_camera), vp, i32, P(atr_frame), C.c_uint64, vp, i32, i32],
                                         C.c_int),
        "atr_write_bmp": ([vp, i32, i32, C.c_char_p, C.c_char_p, i32], C.c_int),
        "atr_render_start_frames": ([vp, P(atr_camera), vp, i32, P(atr_frame), i32, i64, C.c_uint64, vp, i32],
                                    C.c_int),
        "atr_render_start_cameras": ([vp, vp, i32, vp, i32, P(atr_frame), i64, C.c_uint64, vp, i32], C.c_int),
        "atr_last_kernel_ms": ([vp, P(C.c_float)], C.c_int),
        "atr_device_alloc": ([vp, C.c_size_t, P(vp)], C.c_int),
        "atr_device_free": ([vp, vp], C.c_int),
        "atr_memcpy_d2h": ([vp, vp, vp, C.c_size_t], C.c_int),
        "atr_memcpy_h2d": ([vp, vp, vp, C.c_size_t], C.c_int),
        "atr_memset_d": ([vp, vp, C.c_int, C.c_size_t], C.c_int),
    }
    for name in [n for n in DIAG_EXPORTS if not hasattr(L, n)]:
        del sig[name]  # product build: the diagnostic entry points are absent
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    global _sig
    _sig = sig
    _lib = L
    return L


_sig = None


def signatures():
    """{symbol: (argtypes, restype)} of the ctypes binding."""
    lib()
    return dict(_sig)


def vec3(t):
    return atr_vec3(float(t[0]), float(t[1]), float(t[2]))


def tiles_array(tiles):
    """(n, 4) int array of inclusive rects -> ctypes atr_tile array."""
    t = np.ascontiguousarray(np.asarray(tiles, dtype=np.int32).reshape(-1, 4))
    arr = (atr_tile * max(1, len(t)))()
    C.memmove(arr, t.ctypes.data, t.nbytes)
    return arr, len(t)


def make_tiles(width, height, threads):
    """Reference tile grid (renderer.cpp:406-445)."""
    L = lib()
    n = L.atr_make_tiles(width, height, threads, None, 0)
    buf = (atr_tile * max(1, n))()
    L.atr_make_tiles(width, height, threads, C.cast(buf, C.c_void_p), n)
    return np.array([[t.min_x, t.min_y, t.max_x, t.max_y] for t in buf[:n]], np.int32).reshape(-1, 4)


def shard_grid(width, height, side):
    """The side x side shard grid, row-major, as an (n, 4) array of inclusive rects."""
    t = []
    for y in range(0, height, side):
        for x in range(0, width, side):
            t.append([x, y, min(x + side, width) - 1, min(y + side, height) - 1])
    return np.array(t, np.int32).reshape(-1, 4)


def balance_shard_tiles(width, height, side, world, costs, rank0_extra=0):
    """Owner rank per grid tile, longest-processing-time-first by measured cost."""
    costs = np.ascontiguousarray(costs, np.int64)
    owner = np.zeros(len(costs), np.int32)
    n = lib().atr_balance_shard_tiles(width, height, side, world, costs.ctypes.data, int(rank0_extra),
                                      owner.ctypes.data)
    if n != len(costs):
        raise AtrError(f"atr_balance_shard_tiles: {n} tiles for {len(costs)} costs")
    return owner


def make_shard_tiles(width, height, side, rank, world):
    L = lib()
    n = L.atr_make_shard_tiles(width, height, side, rank, world, None, 0)
    buf = (atr_tile * max(1, n))()
    L.atr_make_shard_tiles(width, height, side, rank, world, C.cast(buf, C.c_void_p), n)
    return np.array([[t.min_x, t.min_y, t.max_x, t.max_y] for t in buf[:n]], np.int32).reshape(-1, 4)


def write_bmp(pixels, name):
    """BGRX (H, W) u32 image, row 0 = bottom -> '<name>_<id>.bmp' (texture.cpp:66-115); returns the path."""
    px = np.ascontiguousarray(pixels, dtype=np.uint32)
    if px.ndim != 2:
        raise ValueError("write_bmp: pixels must be (height, width)")
    out = C.create_string_buffer(len(os.fsencode(name)) + 32)
    check(lib().atr_write_bmp(px.ctypes.data, px.shape[1], px.shape[0], os.fsencode(name), out, len(out)),
          f"write bmp {name}")
    return os.fsdecode(out.value)


class Mesh:
    """ModelData (model.h:15-23) held by the engine library."""

    def __init__(self, handle):
        self.h = C.c_void_p(handle)

    @classmethod
    def load_obj(cls, path, threads=None):
        """load_model_data; threads None = the library default (host threads, at most 16)."""
        h = C.c_void_p()
        if threads is None:
            check(lib().atr_mesh_load_obj(os.fsencode(path), C.byref(h)), f"load {path}")
        else:
            check(lib().atr_mesh_load_obj_threaded(os.fsencode(path), int(threads), C.byref(h)), f"load {path}")
        return cls(h.value)

    @classmethod
    def parse_obj(cls, text, threads=1):
        b = text.encode() if isinstance(text, str) else bytes(text)
        h = C.c_void_p()
        check(lib().atr_mesh_parse_obj_threaded(b, len(b), int(threads), C.byref(h)), "parse obj")
        return cls(h.value)

    def arrays(self):
        """ModelData copied out: vertices, normals, texcoords (n, 3) f32; face vertex, texcoord
        and normal indices (nfaces, 3) i32, 0-based (-1 = absent)."""
        nv, nn, nf = self.info()
        nt = C.c_uint32()
        check(lib().atr_mesh_export(self.h, None, None, None, C.byref(nt), None, None, None), "mesh export")
        V = np.zeros((max(nv, 1), 3), np.float32)
        N = np.zeros((max(nn, 1), 3), np.float32)
        T = np.zeros((max(nt.value, 1), 3), np.float32)
        FV, FT, FN = (np.zeros((max(nf, 1), 3), np.int32) for _ in range(3))
        check(lib().atr_mesh_export(self.h, V.ctypes.data, N.ctypes.data, T.ctypes.data, C.byref(nt),
                                    FV.ctypes.data, FT.ctypes.data, FN.ctypes.data), "mesh export")
        return V[:nv], N[:nn], T[:nt.value], FV[:nf], FT[:nf], FN[:nf]

    def info(self):
        nv, nn, nf = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().atr_mesh_info(self.h, C.byref(nv), C.byref(nn), C.byref(nf)))
        return nv.value, nn.value, nf.value

    def aabb(self):
        box = (C.c_float * 6)()
        check(lib().atr_mesh_aabb(self.h, box))
        return np.array(list(box), np.float32)

    def translate_to(self, aabb, center):
        box = (C.c_float * 6)(*[float(x) for x in aabb])
        check(lib().atr_mesh_translate_to(self.h, box, vec3(center)))
        return np.array(list(box), np.float32)

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value and _lib is not None:
            _lib.atr_mesh_free(self.h)
            self.h = None


class Octree:
    """KD_Tree (kd_tree.h:38-47): the reference's 8-ary octree, built on the host."""

    def __init__(self, handle):
        self.h = C.c_void_p(handle)

    @classmethod
    def build(cls, mesh: Mesh, max_faces=300):
        h = C.c_void_p()
        check(lib().atr_octree_build(mesh.h, int(max_faces), C.byref(h)), "octree build")
        return cls(h.value)

    @classmethod
    def build_device(cls, mesh: Mesh, max_faces=300, device=0, timings=None):
        """f3: the same build on the GPU (build.hip), bit-identical to build(). `timings`, if a
        dict, receives wall_ms (whole call) and device_ms (build kernels)."""
        h = C.c_void_p()
        ms = (C.c_float * 2)()
        check(lib().atr_octree_build_device(mesh.h, int(max_faces), int(device), C.byref(h), ms),
              "octree build (device)")
        if timings is not None:
            timings["wall_ms"], timings["device_ms"] = float(ms[0]), float(ms[1])
        return cls(h.value)

    @classmethod
    def from_nodes(cls, bounds, children, leaf_first, leaf_count, prim_vertices, prim_face):
        bounds = np.ascontiguousarray(bounds, np.float32)
        children = np.ascontiguousarray(children, np.int32)
        leaf_first = np.ascontiguousarray(leaf_first, np.uint32)
        leaf_count = np.ascontiguousarray(leaf_count, np.uint32)
        prim_vertices = np.ascontiguousarray(prim_vertices, np.float32)
        prim_face = np.ascontiguousarray(prim_face, np.uint32)
        h = C.c_void_p()
        check(lib().atr_octree_from_nodes(len(children), bounds.ctypes.data, children.ctypes.data,
                                          leaf_first.ctypes.data, leaf_count.ctypes.data,
                                          len(prim_face), prim_vertices.ctypes.data,
                                          prim_face.ctypes.data, C.byref(h)), "octree from nodes")
        return cls(h.value)

    def export(self):
        st = self.stats()
        n, p = st["nodes"], st["leaf_prim_refs"]
        bounds = np.zeros((n, 6), np.float32)
        children = np.zeros(n, np.int32)
        first = np.zeros(n, np.uint32)
        count = np.zeros(n, np.uint32)
        verts = np.zeros((max(p, 1), 9), np.float32)
        face = np.zeros(max(p, 1), np.uint32)
        check(lib().atr_octree_export(self.h, bounds.ctypes.data, children.ctypes.data,
                                      first.ctypes.data, count.ctypes.data, verts.ctypes.data,
                                      face.ctypes.data), "octree export")
        return bounds, children, first, count, verts[:p], face[:p]

    def stats(self):
        s = (C.c_int64 * 7)()
        check(lib().atr_octree_stats(self.h, s))
        keys = ["nodes", "inner", "leaves", "empty_leaves", "leaf_prim_refs", "max_leaf", "depth"]
        return dict(zip(keys, [int(x) for x in s]))

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value and _lib is not None:
            _lib.atr_octree_free(self.h)
            self.h = None


def camera(width, height, spp=1, bounces=1, aa=False, eye=(0.1, 2.0, 0.0),
           facing=(-0.1, -0.5, -1.0), h_fov=1.0):
    """set_camera (camera.h:40-45); defaults are the app's (app.cpp:81-88)."""
    cm = atr_camera()
    check(lib().atr_camera_set(C.byref(cm), vec3(eye), vec3(facing), int(width), int(height),
                               int(bool(aa)), int(spp), int(bounces), float(h_fov)), "camera")
    return cm


class Engine:
    """One device context (atr_ctx): scene upload + renders on a HIP stream."""

    def __init__(self, device=0):
        self.h = C.c_void_p()
        check(lib().atr_create(int(device), C.byref(self.h)), "atr_create")
        self.device = device
        self._keep = []

    def upload(self, materials, models, spheres=(), planes=()):
        """materials: [(emission, reflection, scatter)], models: [(Mesh, Octree|None, aabb6, mat)]."""
        mats = (atr_material * len(materials))(
            *[atr_material(vec3(e), vec3(r), float(s)) for e, r, s in materials])
        mods = (atr_model * max(1, len(models)))()
        for i, (mesh, tree, aabb, mat) in enumerate(models):
            mods[i].mesh = mesh.h.value
            mods[i].tree = tree.h.value if tree is not None else None
            for k in range(6):
                mods[i].surrounding_aabb[k] = float(aabb[k])
            mods[i].material = int(mat)
        sph = (atr_sphere * max(1, len(spheres)))(
            *[atr_sphere(vec3(c), float(r), int(m)) for c, r, m in spheres])
        pln = (atr_plane * max(1, len(planes)))(
            *[atr_plane(vec3(n), float(d), int(m)) for n, d, m in planes])
        check(lib().atr_scene_upload(self.h, C.cast(mats, C.c_void_p), len(materials),
                                     C.cast(mods, C.c_void_p), len(models),
                                     C.cast(sph, C.c_void_p), len(spheres),
                                     C.cast(pln, C.c_void_p), len(planes)), "scene upload")
        self._keep = [materials, models]

    def workspace_info(self):
        """Path-engine workspaces held (count, device bytes): atr_workspace_info."""
        n, b = C.c_int32(), C.c_int64()
        check(lib().atr_workspace_info(self.h, C.byref(n), C.byref(b)))
        return {"workspaces": n.value, "device_bytes": b.value}

    def scene_info(self):
        b, n, d = C.c_int64(), C.c_int32(), C.c_int32()
        check(lib().atr_scene_info(self.h, C.byref(b), C.byref(n), C.byref(d)))
        return {"device_bytes": b.value, "max_nodes": n.value, "max_depth": d.value}

    def render_start(self, cam, tiles, frame: atr_frame, seed, stream=None, variant=ATR_KERNEL_AUTO):
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_render_start_ex(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n,
                                        C.byref(frame), C.c_uint64(seed & (2**64 - 1)),
                                        C.c_void_p(stream) if stream else None, int(variant)),
              "render start")

    def render_start_progressive(self, cam, tiles, frame: atr_frame, seed, tiles_per_launch, stream=None,
                                 variant=ATR_KERNEL_AUTO):
        """Live-view render: tiles_per_launch tiles per launch; wait() reports finished tiles."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_render_start_progressive(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n,
                                                 C.byref(frame), C.c_uint64(seed & (2**64 - 1)),
                                                 C.c_void_p(stream) if stream else None, int(variant),
                                                 int(tiles_per_launch)), "progressive render start")

    def render_start_frames(self, cam, tiles, frame: atr_frame, nframes, frame_stride, seed, stream=None,
                            variant=ATR_KERNEL_AUTO):
        """nframes renders in one launch; frame f's outputs at f * frame_stride elements."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_render_start_frames(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n, C.byref(frame),
                                            int(nframes), int(frame_stride), C.c_uint64(seed & (2**64 - 1)),
                                            C.c_void_p(stream) if stream else None, int(variant)),
              "render start frames")

    def render_start_cameras(self, cams, tiles, frame: atr_frame, frame_stride, seed, stream=None,
                             variant=ATR_KERNEL_AUTO):
        """len(cams) frames (at most 24) in one launch, frame f from cams[f]; outputs frame_stride apart."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        ca = (atr_camera * len(cams))(*cams)
        check(lib().atr_render_start_cameras(self.h, C.cast(ca, C.c_void_p), len(cams), C.cast(arr, C.c_void_p), n,
                                             C.byref(frame), int(frame_stride), C.c_uint64(seed & (2**64 - 1)),
                                             C.c_void_p(stream) if stream else None, int(variant)),
              "render start cameras")

    def counters(self, cam, tiles, seed, variant=ATR_KERNEL_AUTO):
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        out = (C.c_int64 * 10)()
        check(lib().atr_render_counters(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n,
                                        C.c_uint64(seed & (2**64 - 1)), int(variant), out), "counters")
        keys = ["n_rays", "n_box", "n_tri", "n_leaf", "wave_tri_iters", "passes", "box_all", "waves",
                "cluster_boxes", "screened"]
        return dict(zip(keys, [int(x) for x in out]))

    def tile_costs(self, cam, tiles, seed):
        """Shader clocks spent per tile by one render of `tiles` (load-balance calibration)."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        out = np.zeros(max(1, n), np.int64)
        check(lib().atr_render_tile_costs(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n,
                                          C.c_uint64(seed & (2**64 - 1)), out.ctypes.data), "tile costs")
        return out[:n]

    def wave_trace(self, cam, tiles, seed, variant=0):
        """Diagnostic: (nblocks, 3) u64 per work block: start, end (100 MHz), HW_ID | XCC_ID << 32."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        nb = C.c_int64()
        args = (self.h, C.byref(cam), C.cast(arr, C.c_void_p), n, C.c_uint64(seed & (2**64 - 1)), int(variant))
        check(lib().atr_render_wave_trace(*args, None, 0, C.byref(nb)), "wave trace")
        out = np.zeros((max(1, nb.value), 3), np.uint64)
        check(lib().atr_render_wave_trace(*args, out.ctypes.data, out.size, C.byref(nb)), "wave trace")
        return out[:nb.value]

    def wait(self, timeout_ms=0xFFFFFFFF):
        done = C.c_int32()
        rc = check(lib().atr_render_wait(self.h, int(timeout_ms), C.byref(done)), "render wait")
        return rc, done.value

    def last_kernel_ms(self):
        ms = C.c_float()
        check(lib().atr_last_kernel_ms(self.h, C.byref(ms)))
        return ms.value

    def unpack(self, tiles, width, packed_ptr, image_ptr, stream=None):
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_unpack(self.h, C.cast(arr, C.c_void_p), n, int(width), C.c_void_p(packed_ptr),
                               C.c_void_p(image_ptr), C.c_void_p(stream) if stream else None), "unpack")

    def tile_ray_casts(self, tiles, width, casts_ptr, out_ptr, stream=None):
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_tile_ray_casts(self.h, C.cast(arr, C.c_void_p), n, int(width),
                                       C.c_void_p(casts_ptr), C.c_void_p(out_ptr),
                                       C.c_void_p(stream) if stream else None), "tile casts")

    def packed_tile_ray_casts(self, tiles, width, height, casts_ptr, nframes, frame_stride, out_ptr, stream=None):
        """out[f * ntiles + i] (device int64) = ray_casts of tile i in PACKED frame f (asynchronous)."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_packed_tile_ray_casts(self.h, C.cast(arr, C.c_void_p), n, int(width), int(height),
                                              C.c_void_p(casts_ptr), int(nframes), int(frame_stride),
                                              C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None),
              "packed tile casts")

    def set_cell_plan(self, width, height, plan=None):
        """Per-8x8-cell split/priority bytes (atr_set_cell_plan); None clears."""
        if plan is None:
            check(lib().atr_set_cell_plan(self.h, int(width), int(height), None), "cell plan")
            return
        plan = np.ascontiguousarray(plan, np.uint8)
        assert plan.size == ((width + 7) // 8) * ((height + 7) // 8)
        check(lib().atr_set_cell_plan(self.h, int(width), int(height), plan.ctypes.data), "cell plan")

    def phase_clocks(self, cam, tiles, seed, variant=ATR_KERNEL_AUTO):
        """Wave clocks in DFS passes, lane-private scans, dealt rounds, whole waves (diagnostic)."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        out = (C.c_int64 * 6)()
        check(lib().atr_render_phase_clocks(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n, C.c_uint64(seed),
                                            int(variant), out), "phase clocks")
        return dict(zip(["pass", "lane_private", "dealt", "wave", "step_prep", "scan"], list(out)))

    def pack_bgr(self, fb_ptr, npixels, out_ptr, stream=None):
        """BGRX u32 -> 3 bytes per pixel (atr_pack_bgr; device pointers, async on `stream`)."""
        check(lib().atr_pack_bgr(self.h, C.c_void_p(fb_ptr), int(npixels), C.c_void_p(out_ptr),
                                 C.c_void_p(stream) if stream else None), "pack bgr")

    def scatter_bgr(self, packed_ptr, npixels, index_ptr, image_ptr, stream=None):
        """3-byte pixels -> BGRX u32 at image[index[i]] (atr_scatter_bgr; device pointers, async)."""
        check(lib().atr_scatter_bgr(self.h, C.c_void_p(packed_ptr), int(npixels), C.c_void_p(index_ptr),
                                    C.c_void_p(image_ptr), C.c_void_p(stream) if stream else None), "scatter bgr")

    def pack_bgr_masked(self, fb_ptr, npixels, background, out_ptr, nbytes_ptr, stream=None):
        """BGRX u32 -> the masked stream (atr_pack_bgr_masked: a bit per pixel, 3 bytes per pixel that
        differs from `background`); its byte count goes to the device int64 at nbytes_ptr."""
        check(lib().atr_pack_bgr_masked(self.h, C.c_void_p(fb_ptr), int(npixels), int(background) & 0xFFFFFFFF,
                                        C.c_void_p(out_ptr), C.c_void_p(nbytes_ptr),
                                        C.c_void_p(stream) if stream else None), "pack bgr masked")

    def scatter_bgr_masked(self, packed_ptr, npixels, index_ptr, image_ptr, stream=None):
        """A masked stream of npixels -> BGRX u32 at image[index[i]] (atr_scatter_bgr_masked)."""
        check(lib().atr_scatter_bgr_masked(self.h, C.c_void_p(packed_ptr), int(npixels), C.c_void_p(index_ptr),
                                           C.c_void_p(image_ptr), C.c_void_p(stream) if stream else None),
              "scatter bgr masked")

    def unpack_masked(self, tiles, width, height, packed_ptr, nframes, image_ptr, image_stride, stream=None):
        """The masked stream of a PACKED render of `tiles` (nframes frames) into IMAGE frames
        image_stride pixels apart (atr_unpack_masked: positions from the tile list's blocks)."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        check(lib().atr_unpack_masked(self.h, C.cast(arr, C.c_void_p), n, int(width), int(height),
                                      C.c_void_p(packed_ptr), int(nframes), C.c_void_p(image_ptr), int(image_stride),
                                      C.c_void_p(stream) if stream else None), "unpack masked")

    def unpack_masked_ranks(self, tiles_list, width, height, packed_ptrs, nframes, image_ptr, image_stride,
                            stream=None, raw=None):
        """Several masked streams (source i: the PACKED render of tiles_list[i], its stream at
        packed_ptrs[i]; with raw[i] true, that render's u32 PACKED frames themselves) into the same
        IMAGE frames in one call (atr_unpack_masked_ranks)."""
        arrs = [t if isinstance(t, tuple) else tiles_array(t) for t in tiles_list]
        n = len(arrs)
        tp = (C.c_void_p * max(1, n))(*[C.cast(a, C.c_void_p) for a, _ in arrs])
        nt = (C.c_int32 * max(1, n))(*[k for _, k in arrs])
        pp = (C.c_void_p * max(1, n))(*[int(p) for p in packed_ptrs])
        rw = (C.c_int32 * max(1, n))(*[int(bool(x)) for x in raw]) if raw is not None else None
        check(lib().atr_unpack_masked_ranks(self.h, n, tp, nt, int(width), int(height), pp, rw, int(nframes),
                                            C.c_void_p(image_ptr), int(image_stride),
                                            C.c_void_p(stream) if stream else None), "unpack masked ranks")

    def plan_info(self, tiles, width, height):
        """The single-frame plan of a tile list (diagnostic): (base index per planned block, masks
        (n, 2) u32, cost per base block) or None before the first planned launch."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        npl = C.c_int64()
        args = (self.h, C.cast(arr, C.c_void_p), n, int(width), int(height))
        check(lib().atr_render_plan_info(*args, None, None, 0, None, C.byref(npl)), "plan info")
        if npl.value == 0:
            return None
        base = np.zeros(npl.value, np.int32)
        masks = np.zeros((npl.value, 2), np.uint32)
        cost = np.zeros(npl.value, np.uint64)  # the base list is shorter than the planned one
        check(lib().atr_render_plan_info(*args, base.ctypes.data, masks.ctypes.data, npl.value, cost.ctypes.data,
                                         C.byref(npl)), "plan info")
        return base, masks, cost

    def tuning(self):
        """The context's scheduling knobs (atr_get_tuning) as a dict."""
        t = atr_tuning()
        check(lib().atr_get_tuning(self.h, C.byref(t)), "get tuning")
        return {f: getattr(t, f) for f, _ in atr_tuning._fields_ if f != "reserved"}

    def set_tuning(self, **kw):
        """Change scheduling knobs (atr_set_tuning); unnamed fields keep their current value. Outputs
        never change; cluster_size applies at the next upload."""
        t = atr_tuning()
        check(lib().atr_get_tuning(self.h, C.byref(t)), "get tuning")
        for k, v in kw.items():
            if k not in {f for f, _ in atr_tuning._fields_} or k == "reserved":
                raise KeyError(k)
            setattr(t, k, int(v))
        check(lib().atr_set_tuning(self.h, C.byref(t)), "set tuning")

    def path_counters(self, cam, tiles, seed, variant=ATR_KERNEL_AUTO):
        """Bounce-loop lane use (diagnostic): wave steps and tracing lanes of bounce 0, 1, >= 2."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        out = (C.c_int64 * 6)()
        check(lib().atr_render_path_counters(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n, C.c_uint64(seed),
                                             int(variant), out), "path counters")
        v = list(out)
        return {"steps": v[:3], "active": v[3:], "lane_use": [a / (64.0 * s) if s else 0.0 for s, a in zip(v[:3], v[3:])]}

    def simd_counters(self, cam, tiles, seed, variant=ATR_KERNEL_AUTO):
        """SIMD efficiency of the clustered scans (diagnostic, atr_render_simd_counters)."""
        arr, n = tiles if isinstance(tiles, tuple) else tiles_array(tiles)
        out = (C.c_int64 * 7)()
        check(lib().atr_render_simd_counters(self.h, C.byref(cam), C.cast(arr, C.c_void_p), n, C.c_uint64(seed),
                                             int(variant), out), "simd counters")
        keys = ["cand_wave_iters", "full_tests", "dfs_wave_iters", "dfs_lane_iters", "dealt_rounds", "dealt_items",
                "rays"]
        return dict(zip(keys, [int(x) for x in out]))

    def cell_costs(self, cam, seed, variant=ATR_KERNEL_AUTO):
        """Shader clocks per 8x8 cell of one full-frame render ((H+7)/8, (W+7)/8)."""
        out = np.zeros(((cam.height + 7) // 8) * ((cam.width + 7) // 8), np.int64)
        check(lib().atr_render_cell_costs(self.h, C.byref(cam), C.c_uint64(seed), int(variant), out.ctypes.data),
              "cell costs")
        return out.reshape((cam.height + 7) // 8, (cam.width + 7) // 8)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().atr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_bgr_masked_bound(npixels):
    """Largest masked exchange stream of npixels pixels, in bytes (atr_pack_bgr_masked_bound)."""
    return int(lib().atr_pack_bgr_masked_bound(int(npixels)))


def packed_size(tiles):
    arr, n = tiles_array(tiles)
    return int(lib().atr_render_packed_size(C.cast(arr, C.c_void_p), n))


def packed_pixel_map(tiles, width, height):
    """Pixel index of every slot of a PACKED render of `tiles` (host-only)."""
    arr, n = tiles_array(tiles)
    L = lib()
    cnt = int(L.atr_packed_pixel_map(C.cast(arr, C.c_void_p), n, int(width), int(height), None, 0))
    out = np.zeros(max(cnt, 1), np.int64)
    L.atr_packed_pixel_map(C.cast(arr, C.c_void_p), n, int(width), int(height), out.ctypes.data, cnt)
    return out[:cnt]
