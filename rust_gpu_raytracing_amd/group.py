"""``RendererGroup`` — several GPUs in one process through the C ABI (rt_multi.cpp).

The C-ABI route a Rust host takes to more than one GPU (SURVEY §5, §8b threading
row): ``rt_create_multi`` makes one context per device (rank r on ``devices[r]``,
the 8x8-tile round-robin split of §8e), each driven by its own host thread, and one
RCCL communicator per device (``ncclCommInitAll``); ``rt_gather_frame`` assembles
the frame on a root device with one grouped ``ncclSend``/``ncclRecv``. The
torch.distributed route (one process per GPU, ``distributed.py``) is the other
driver; both render the same bits.

Mirrors :class:`~rust_gpu_raytracing_amd.renderer.Renderer` (itself the mirror of
``Renderer`` in src/renderer.rs:28-320) for the calls a multi-GPU display loop
makes: compute_frame, reset_accumulation, camera updates, readback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from . import buffers as B
from .renderer import Renderer
from .scene import RenderScene

GATHER_PAYLOADS = {"image": N.RT_GATHER_IMAGE, "accumulation": N.RT_GATHER_ACCUMULATION}


class RendererGroup:
    def __init__(self, scene: RenderScene, devices, *, accumulate: bool = True, compute_per_frame: int = 1,
                 camera_rays: np.ndarray | None = None, frame_batch: int | None = None, copy_transport: bool = False,
                 lib=None):
        """``copy_transport``: rt_create_multi_ex(RT_GROUP_COPY_TRANSPORT) -- no RCCL; the gather
        copies blocks device to device, and a device may be listed more than once (several
        ranks on one GPU: the group's N-rank logic on a one-GPU machine)."""
        self._lib = N.load_library() if lib is None else lib
        self.scene = scene
        self.accumulate = accumulate
        self.compute_per_frame = compute_per_frame
        self.width = scene.camera.viewport_width
        self.height = scene.camera.viewport_height
        self.devices = [int(d) for d in devices]
        self._g = None
        rays = scene.camera.recalculate_ray_directions() if camera_rays is None else camera_rays
        self.camera_rays = np.ascontiguousarray(rays, dtype=B.RAY)
        objs, subs, tris = scene.flatten()
        self._keep = [self.camera_rays, scene.materials, scene.spheres, tris, objs, subs]
        info = N.rt_create_info()
        info.width, info.height, info.device = self.width, self.height, 0
        info.camera.origin[:] = [float(x) for x in scene.camera.position]
        info.camera_rays = N.ptr(self.camera_rays)
        info.materials, info.material_count = N.ptr(scene.materials), scene.materials.shape[0]
        info.spheres, info.sphere_count = N.ptr(scene.spheres), scene.spheres.shape[0]
        info.triangles, info.triangle_count = N.ptr(tris), tris.shape[0]
        info.objects, info.object_count = N.ptr(objs), objs.shape[0]
        info.sub_objects, info.sub_object_count = N.ptr(subs), subs.shape[0]
        info.params = N.params_struct(self._params(1))
        info.rank, info.world_size = 0, 1
        devs = (ctypes.c_int32 * len(self.devices))(*self.devices)
        g = ctypes.c_void_p()
        flags = N.RT_GROUP_COPY_TRANSPORT if copy_transport else 0
        rc = self._lib.rt_create_multi_ex(ctypes.byref(info), devs, len(self.devices), flags, ctypes.byref(g))
        N.check(None, rc, self._lib)
        self._g = g
        tex = np.ascontiguousarray(scene.textures, np.uint8)
        layers, th, tw, _ = tex.shape
        self._call("rt_group_upload_textures", N.ptr(tex), tw, th, layers)
        env = np.ascontiguousarray(scene.environment_map, np.uint8)
        eh, ew, _ = env.shape
        self._call("rt_group_upload_env_map", N.ptr(env), ew, eh)
        if frame_batch is not None:
            self._call("rt_group_set_frame_batch", frame_batch)

    def _params(self, accumulation_index: int) -> np.ndarray:
        return self.scene.params(accumulate=int(self.accumulate), compute_per_frame=self.compute_per_frame,
                                 accumulation_index=accumulation_index)

    def _call(self, name, *args):
        if self._g is None:
            raise N.RtError(N.RT_E_INVALID, "renderer group is closed")
        rc = getattr(self._lib, name)(self._g, *args)
        if rc != N.RT_OK:
            msg = self._lib.rt_group_last_error(self._g)
            raise N.RtError(rc, msg.decode() if msg else name)

    @property
    def size(self) -> int:
        return int(self._lib.rt_group_size(self._g))

    def context(self, rank: int) -> int:
        """rank r's rt_ctx* (for single-context entry points while the group is idle)."""
        return self._lib.rt_group_context(self._g, rank)

    def context_view(self, rank: int) -> "Renderer":
        """A Renderer bound to rank r's context, for its single-context calls (timing,
        launch geometry, readback) while the group is idle; closing it leaves the
        context to the group."""
        return _BorrowedContext(self, rank)

    # ------------------------------------------------------------------ reference surface
    def compute_frame(self, bounces: int = 10) -> None:
        """src/renderer.rs:201-252 on every device's tiles (asynchronous)."""
        self._call("rt_group_compute_frame", bounces)

    def reset_accumulation(self) -> None:
        p = N.params_struct(self._params(1))
        self._call("rt_group_reset_accumulation", ctypes.byref(p))

    def update_ray_directions(self, rays: np.ndarray) -> None:
        rays = np.ascontiguousarray(rays, dtype=B.RAY)
        self._call("rt_group_update_ray_directions", N.ptr(rays), rays.shape[0])

    def update_camera(self, camera) -> None:
        """src/renderer.rs:109-129 on every device: reset, new origin, new ray directions."""
        self.scene.camera = camera
        self.reset_accumulation()
        rc = N.rt_ray_camera()
        rc.origin[:] = [float(x) for x in camera.position]
        self._call("rt_group_update_camera", ctypes.byref(rc))
        self.update_ray_directions(camera.recalculate_ray_directions())

    def update_materials(self, materials: np.ndarray) -> None:
        m = np.ascontiguousarray(materials, dtype=B.MATERIAL)
        self._call("rt_group_update_materials", N.ptr(m), m.shape[0])

    def set_frame_batch(self, frames: int) -> None:
        self._call("rt_group_set_frame_batch", frames)

    def synchronize(self) -> None:
        self._call("rt_group_synchronize")

    def gather(self, root: int = 0, what: str = "image") -> None:
        """rt_gather_frame: pack -> grouped ncclSend/ncclRecv -> unpack on `root`
        (stream-ordered, no host wait)."""
        self._call("rt_gather_frame", root, GATHER_PAYLOADS[what])

    def read_output(self, root: int = 0) -> np.ndarray:
        out = np.zeros((self.height, self.width), np.uint32)
        self._call("rt_group_read_output", root, out.ctypes.data)
        return out

    def read_accumulation(self, root: int = 0) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.float32)
        self._call("rt_group_read_accumulation", root, out.ctypes.data)
        return out

    def ray_count(self) -> int:
        v = ctypes.c_uint64()
        self._call("rt_group_ray_count", ctypes.byref(v))
        return int(v.value)

    def reset_ray_count(self) -> None:
        self._call("rt_group_reset_ray_count")

    def close(self) -> None:
        if self._g is not None:
            self._lib.rt_destroy_multi(self._g)
            self._g = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class _BorrowedContext(Renderer):
    """Renderer methods over a group member's context (not owned: close() is a no-op)."""

    def __init__(self, group: RendererGroup, rank: int):  # noqa: D107 - no rt_create here
        self._lib = group._lib
        self.scene = group.scene
        self.accumulate = group.accumulate
        self.compute_per_frame = group.compute_per_frame
        self.width, self.height = group.width, group.height
        self.rank, self.world_size = rank, group.size
        self.device = group.devices[rank]
        self._ctx = ctypes.c_void_p(group.context(rank))

    def close(self) -> None:
        self._ctx = None
