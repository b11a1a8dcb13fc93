"""Host-side mirror of the reference's render API over the HIP engine.

Names, argument meaning and return conventions follow Source/engine/renderer/renderer.h:
  prep_scene(scene) -> max_nodes                                   (renderer.h:35)
  start_render_from_camera(info, engine)                           (renderer.h:32)
  wait_for_render_from_camera_to_finish(info, engine, ms) -> bool  (renderer.h:33; True = running)
with Scene (scene.h:13-24), Model (model.h:66-71), Material (material.h), RenderSettings
(settings.h), Camera/set_camera (camera.h), RenderTile/RenderInfo (renderer.h:11-30),
load_model_data (OBJ_loader.h:6), get_AABB / translate_to (model.h:41-61,136-152).

The engine replaces the reference's ThreadPool: tiles are the reference grid for `threads`
(renderer.cpp:406-445), every pixel is traced once on the GPU, the framebuffer lands in the
caller's Texture (BGRX u32, row 0 = bottom) and per-tile ray_casts are the reference's sums
over the inclusive tile rects (overlaps counted twice, as the reference's threads do).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import engine as E

SKY_DEFAULT = ((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3)     # app.cpp:91
MODEL_DEFAULT = ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)  # app.cpp:96


@dataclass
class Material:
    emission_color: tuple = (0.0, 0.0, 0.0)
    reflection_color: tuple = (0.0, 0.0, 0.0)
    scatter: float = 0.0


@dataclass
class RenderSettings:
    resolution: tuple = (1280, 720)
    anti_aliasing: bool = False
    samples_per_pixel: int = 5
    bounce_limit: int = 5


@dataclass
class Camera:
    render_settings: RenderSettings
    c: E.atr_camera = None


def set_camera(eye, facing_towards, render_settings: RenderSettings, h_fov=1.0) -> Camera:
    rs = render_settings
    c = E.camera(rs.resolution[0], rs.resolution[1], rs.samples_per_pixel, rs.bounce_limit,
                 rs.anti_aliasing, eye=eye, facing=facing_towards, h_fov=h_fov)
    return Camera(rs, c)


class ModelData:
    def __init__(self, mesh: E.Mesh):
        self.mesh = mesh
        self.material = 0

    @property
    def sizes(self):
        return self.mesh.info()


def load_model_data(path: str) -> ModelData:
    return ModelData(E.Mesh.load_obj(path))


@dataclass
class Model:
    data: ModelData = None
    surrounding_aabb: np.ndarray = None
    kd_tree: Optional[E.Octree] = None
    max_no_faces_per_node: int = 300
    use_kd_tree: bool = True  # renderer.h:8 USE_KD_TREE


def get_AABB(data: ModelData) -> np.ndarray:
    return data.mesh.aabb()


def translate_to(model: Model, center) -> None:
    model.surrounding_aabb = model.data.mesh.translate_to(model.surrounding_aabb, center)


@dataclass
class Scene:
    materials: List[Material] = field(default_factory=list)
    models: List[Model] = field(default_factory=list)
    spheres: list = field(default_factory=list)   # (center, radius, material index)
    planes: list = field(default_factory=list)    # (normal, distance, material index)


def prep_scene(scene: Scene, engine: Optional[E.Engine] = None) -> int:
    """Build every model's octree (kd_tree.cpp:20-64) and upload the flattened scene.
    Plane normals are normalized first (renderer.cpp:267-270). Returns the max node count."""
    max_nodes = 0
    planes = []
    for n, d, m in scene.planes:
        v = np.array(n, np.float32)
        inv = np.float32(1.0) / np.sqrt(np.float32((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))
        planes.append((tuple((v * inv).tolist()), d, m))
    for mdl in scene.models:
        if mdl.use_kd_tree and mdl.kd_tree is None:
            mdl.kd_tree = E.Octree.build(mdl.data.mesh, mdl.max_no_faces_per_node)
        if mdl.kd_tree is not None:
            max_nodes = max(max_nodes, mdl.kd_tree.stats()["nodes"])
    if engine is not None:
        mats = [(m.emission_color, m.reflection_color, m.scatter) for m in scene.materials]
        models = [(m.data.mesh, m.kd_tree if m.use_kd_tree else None, m.surrounding_aabb,
                   m.data.material) for m in scene.models]
        engine.upload(mats, models, scene.spheres, planes)
    return max_nodes


@dataclass
class RenderTile:
    tile: tuple
    ray_casts: int = 0


@dataclass
class RenderInfo:
    camera: Camera
    scene: Scene
    camera_tex: np.ndarray = None   # H x W uint32 BGRX, row 0 = bottom (texture.h:27-38)
    threads: int = 8                # tile grid of renderer.cpp:406 (the reference's pool size)
    seed: int = 0x853C49E6748FEA9B
    jobs: List[RenderTile] = field(default_factory=list)
    jobs_done: int = 0
    total_ray_casts: int = 0
    _dev: dict = field(default_factory=dict)


def start_render_from_camera(info: RenderInfo, engine: E.Engine, tiles_per_launch: int = 0) -> None:
    """renderer.cpp:447-455. tiles_per_launch > 0 renders progressively for a live view
    (app.cpp:162-186): wait_for_render_from_camera_to_finish then reports finished tiles in
    jobs_done and refreshes camera_tex with them while the render runs."""
    import torch
    W, H = info.camera.render_settings.resolution
    tiles = E.make_tiles(W, H, info.threads)
    info.jobs = [RenderTile(tuple(int(v) for v in t)) for t in tiles]
    info.jobs_done = 0
    dev = torch.device("cuda", engine.device)
    fb = torch.zeros(H * W, dtype=torch.int32, device=dev)
    casts = torch.zeros(H * W, dtype=torch.int32, device=dev)
    per_tile = torch.zeros(len(tiles), dtype=torch.int64, device=dev)
    frame = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, casts.data_ptr(), None)
    d = {"fb": fb, "casts": casts, "per_tile": per_tile, "tiles": tiles}
    if tiles_per_launch > 0:
        # own stream, so the live copies (another stream) run beside the render
        rs = torch.cuda.Stream(dev)
        rs.wait_stream(torch.cuda.current_stream(dev))
        d["render_stream"], d["copy_stream"] = rs, torch.cuda.Stream(dev)
        d["host"] = torch.empty(H * W, dtype=torch.int32, pin_memory=True)
        d["stream"] = rs.cuda_stream
        engine.render_start_progressive(info.camera.c, tiles, frame, info.seed, tiles_per_launch, stream=rs.cuda_stream)
    else:
        d["stream"] = torch.cuda.current_stream(dev).cuda_stream
        engine.render_start(info.camera.c, tiles, frame, info.seed, stream=d["stream"])
    info._dev = d


def _live_copy(info: RenderInfo) -> None:
    import torch
    d = info._dev
    W, H = info.camera.render_settings.resolution
    with torch.cuda.stream(d["copy_stream"]):
        d["host"].copy_(d["fb"], non_blocking=True)
    d["copy_stream"].synchronize()
    info.camera_tex = d["host"].numpy().view(np.uint32).reshape(H, W).copy()


def wait_for_render_from_camera_to_finish(info: RenderInfo, engine: E.Engine, ms_to_wait_for: int) -> bool:
    """TRUE while still rendering after the timeout, FALSE once done (renderer.cpp:457-471)."""
    rc, done = engine.wait(ms_to_wait_for)
    d = info._dev
    if rc == 1:
        if "copy_stream" in d and done > info.jobs_done:
            info.jobs_done = done
            _live_copy(info)  # the pixels of the first `done` tiles are final
        return True
    W, H = info.camera.render_settings.resolution
    engine.tile_ray_casts(d["tiles"], W, d["casts"].data_ptr(), d["per_tile"].data_ptr(), d["stream"])
    if "render_stream" in d:
        import torch
        torch.cuda.current_stream(d["fb"].device).wait_stream(d["render_stream"])
    per_tile = d["per_tile"].cpu().numpy()
    for j, c in zip(info.jobs, per_tile.tolist()):
        j.ray_casts = int(c)
    info.total_ray_casts += int(per_tile.sum())
    info.jobs_done = len(info.jobs)
    info.camera_tex = d["fb"].cpu().numpy().view(np.uint32).reshape(H, W)
    return False


def write_to_file(info: RenderInfo, file_name: str) -> str:
    """The app's 'save render' (texture.cpp:66-115 via app.cpp): camera_tex as <file_name>_<id>.bmp."""
    if info.camera_tex is None:
        raise ValueError("write_to_file: nothing rendered yet")
    return E.write_bmp(info.camera_tex, file_name)


def app_scene(obj_path: str, center=(0.0, -15.0, -38.0), use_tree=True, leaf=300) -> Scene:
    """The app's scene (app.cpp:65-146): one model, sky = materials[0], model = materials[5]."""
    mats = [Material(*SKY_DEFAULT), Material((0, 0, 0), (0.2, 0.8, 0.2), 0.3),
            Material((0, 0, 0), (0.4, 0.8, 0.9), 0.9), Material((0, 0.4, 0.6), (0.2, 0.3, 0.2), 0.0),
            Material((0, 0, 0), (0.5, 0.5, 0.5), 0.0), Material(*MODEL_DEFAULT),
            Material((0.8, 0.2, 0.2), (0.92, 0.0, 0.0), 0.3)]
    data = load_model_data(obj_path)
    m = Model(data=data, surrounding_aabb=get_AABB(data), max_no_faces_per_node=leaf,
              use_kd_tree=use_tree)
    translate_to(m, center)
    data.material = 5
    return Scene(materials=mats, models=[m])
