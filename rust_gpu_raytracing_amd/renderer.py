"""``Renderer`` — the host side of the hot path, over the C ABI.

Mirrors ``Renderer`` in src/renderer.rs:28-320 (names, argument meaning and
call order), with wgpu replaced by ``include/rt_abi.h``:

===========================================  ==========================================
reference (src/renderer.rs)                  here
===========================================  ==========================================
``Renderer::new`` :42-101                    ``Renderer(scene, ...)`` -> ``rt_create`` +
                                             ``rt_upload_textures`` + ``rt_upload_env_map``
``reset_accumulation`` :131-151              ``reset_accumulation()`` -> ``rt_reset_accumulation``
``update_scene`` :153-199                    ``update_scene()`` -> ``rt_update_*``, or
                                             ``update_scene(device=True)`` -> ``rt_update_objects``
``compute_frame`` :201-252                   ``compute_frame(bounces)`` -> ``rt_compute_frame``
``on_update`` (camera moved) :109-129        ``update_camera(camera)``
(no readback in the reference)               ``read_output`` / ``read_accumulation``
===========================================  ==========================================

Errors raise :class:`RtError` (the reference panics via ``.expect``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from . import buffers as B
from .scene import RenderScene

REFERENCE_BOUNCES = 10  # compute_shader.wgsl:150


class Renderer:
    def __init__(
        self,
        scene: RenderScene,
        *,
        accumulate: bool = True,
        compute_per_frame: int = 1,
        device: int = 0,
        rank: int = 0,
        world_size: int = 1,
        camera_rays: np.ndarray | None = None,
        device_rays: bool | None = None,
        frame_batch: int | None = None,
        tuning: dict[str, int] | None = None,
        lib=None,
    ):
        """``camera_rays``: explicit per-pixel directions (the reference's ray buffer;
        default: ``scene.camera.recalculate_ray_directions()``). ``device_rays=True``
        computes them on the device from the camera's matrices instead
        (rt_update_camera_matrices; bit-identical, no ray buffer read, but measured
        2% slower on C2 than reading the buffer, so off by default).
        ``frame_batch``: frames one launch may render (rt_set_frame_batch): with
        F > 1, ``compute_frame`` queues frames and launches F at a time (or at the
        next readback / update / sync), each frame's results written as before.
        None keeps the library's default (RT_DEFAULT_FRAME_BATCH, include/rt_abi.h).
        ``tuning``: exact variants of the schedule and acceleration structures for A/B
        runs, {key: value} passed to rt_set_tuning (include/rt_abi.h lists the keys)."""
        self._lib = N.load_library() if lib is None else lib
        self.scene = scene
        self.accumulate = accumulate
        self.compute_per_frame = compute_per_frame
        self.width = scene.camera.viewport_width
        self.height = scene.camera.viewport_height
        self.rank, self.world_size = rank, world_size
        self.device = device
        self._ctx = None
        rays = scene.camera.recalculate_ray_directions() if camera_rays is None else camera_rays
        self.camera_rays = np.ascontiguousarray(rays, dtype=B.RAY)
        objs, subs, tris = scene.flatten()
        self._keep = [self.camera_rays, scene.materials, scene.spheres, tris, objs, subs]

        info = N.rt_create_info()
        info.width, info.height, info.device = self.width, self.height, device
        info.camera.origin[:] = [float(x) for x in scene.camera.position]
        info.camera_rays = N.ptr(self.camera_rays)
        info.materials, info.material_count = N.ptr(scene.materials), scene.materials.shape[0]
        info.spheres, info.sphere_count = N.ptr(scene.spheres), scene.spheres.shape[0]
        info.triangles, info.triangle_count = N.ptr(tris), tris.shape[0]
        info.objects, info.object_count = N.ptr(objs), objs.shape[0]
        info.sub_objects, info.sub_object_count = N.ptr(subs), subs.shape[0]
        info.params = N.params_struct(self._params(accumulation_index=1))
        info.rank, info.world_size = rank, world_size
        ctx = ctypes.c_void_p()
        N.check(None, self._lib.rt_create(ctypes.byref(info), ctypes.byref(ctx)), self._lib)
        self._ctx = ctx
        self._upload_textures()
        self.device_rays = bool(device_rays)
        if self.device_rays:
            self._set_camera_matrices(scene.camera)
        if frame_batch is not None:
            self.set_frame_batch(frame_batch)
        for key, value in (tuning or {}).items():
            self.set_tuning(key, value)

    # ------------------------------------------------------------------ helpers
    def _params(self, accumulation_index: int) -> np.ndarray:
        return self.scene.params(
            accumulate=int(self.accumulate),
            compute_per_frame=self.compute_per_frame,
            accumulation_index=accumulation_index,
        )

    def _call(self, name, *args):
        if self._ctx is None:
            raise N.RtError(N.RT_E_INVALID, "renderer is closed")
        N.check(self._ctx, getattr(self._lib, name)(self._ctx, *args), self._lib)

    def _upload_textures(self):
        tex = np.ascontiguousarray(self.scene.textures, np.uint8)
        layers, th, tw, _ = tex.shape
        self._call("rt_upload_textures", N.ptr(tex), tw, th, layers)
        env = np.ascontiguousarray(self.scene.environment_map, np.uint8)
        eh, ew, _ = env.shape
        self._call("rt_upload_env_map", N.ptr(env), ew, eh)

    # ------------------------------------------------------------------ reference surface
    def reset_accumulation(self) -> None:
        """src/renderer.rs:131-151."""
        p = N.params_struct(self._params(accumulation_index=1))
        self._call("rt_reset_accumulation", ctypes.byref(p))

    def update_scene(self, device: bool = False) -> None:
        """src/renderer.rs:153-199: reset, re-upload spheres, rebuild every object's
        triangles from its edit state (update_triangles + update_sub_objects,
        src/triangle_object.rs:129-150, :199-220), re-upload textures, env map,
        triangles, objects, sub-objects and materials.

        ``device=False`` rebuilds the objects on the host (native builder,
        bit-identical to scene.py) and uploads them, as the reference does.
        ``device=True`` runs the rebuild on the GPU instead (``update_objects``):
        nothing but the 32-B edit state per object crosses PCIe, and the host
        ``scene.objects`` records are left as they were."""
        from . import builder

        self.reset_accumulation()
        s = self.scene
        self._call("rt_update_spheres", N.ptr(s.spheres), s.spheres.shape[0])
        self._upload_textures()
        if device:
            # the device rebuild rewrites bounds only; every other ObjectInfo field
            # (material_index, src/renderer.rs:188-193) comes from the host records
            self._upload_object_fields()
            self.update_objects()
        else:
            self._models = None  # the host path may change the objects: re-upload models for device edits
            for o in s.objects:
                builder.update_object(o, lib=self._lib)
            objs, subs, tris = s.flatten()
            self._keep[3:6] = [tris, objs, subs]
            self._call("rt_update_triangles", N.ptr(tris), tris.shape[0])
            self._call("rt_update_object_info", N.ptr(objs), objs.shape[0])
            self._call("rt_update_sub_object_info", N.ptr(subs), subs.shape[0])
        self._call("rt_update_materials", N.ptr(s.materials), s.materials.shape[0])

    def _upload_object_fields(self) -> None:
        """The host ObjectInfo records with the device's current bounds (a device
        edit leaves the host bounds stale): material index and sub-object range
        reach the device without invalidating the triangle accelerator."""
        objs = np.stack([np.asarray(o.object_info) for o in self.scene.objects]).astype(B.OBJECT_INFO) \
            if self.scene.objects else np.zeros(0, B.OBJECT_INFO)
        if objs.shape[0] == 0:
            return
        dev = np.zeros(objs.shape[0], B.OBJECT_INFO)
        self._call("rt_read_object_info", N.ptr(dev), dev.shape[0])
        merged = objs.copy()
        merged["min_bounds"] = dev["min_bounds"]
        merged["max_bounds"] = dev["max_bounds"]
        merged = np.ascontiguousarray(merged)
        self._call("rt_update_object_info", N.ptr(merged), merged.shape[0])

    def upload_object_models(self) -> None:
        """The objects' normalised points (rt_set_object_models), once, for device-side edits."""
        pts = [np.asarray(o.normalized_points, np.float32).reshape(-1, 9) for o in self.scene.objects]
        self._models = np.ascontiguousarray(np.concatenate(pts) if pts else np.zeros((0, 9), np.float32))
        self._models_key = tuple(id(o) for o in self.scene.objects)
        self._call("rt_set_object_models", N.ptr(self._models), self._models.shape[0])

    def update_objects(self) -> None:
        """update_triangles + update_sub_objects for every object, on the device
        (rt_update_objects): triangles, object and sub-object bounds rebuilt and
        the triangle accelerator refitted, stream-ordered before the next frame."""
        from . import builder

        if getattr(self, "_models", None) is None or \
                getattr(self, "_models_key", None) != tuple(id(o) for o in self.scene.objects):
            self.upload_object_models()
        t = np.ascontiguousarray(np.stack([builder.transform_of(o) for o in self.scene.objects])) \
            if self.scene.objects else np.zeros(0, B.OBJECT_TRANSFORM)
        self._call("rt_update_objects", N.ptr(t), t.shape[0])

    def read_geometry(self):
        """(objects, sub-objects, triangles) as the device holds them (rt_read_*)."""
        objs, subs, tris = self.scene.flatten()
        o = np.zeros(objs.shape[0], B.OBJECT_INFO)
        so = np.zeros(subs.shape[0], B.SUB_OBJECT_INFO)
        t = np.zeros(tris.shape[0], B.TRIANGLE)
        self._call("rt_read_object_info", N.ptr(o), o.shape[0])
        self._call("rt_read_sub_object_info", N.ptr(so), so.shape[0])
        self._call("rt_read_triangles", N.ptr(t), t.shape[0])
        return o, so, t

    def _set_camera_matrices(self, camera) -> None:
        self._inv = [np.ascontiguousarray(camera.inverse_projection, np.float32).reshape(16),
                     np.ascontiguousarray(camera.inverse_view, np.float32).reshape(16)]
        self._call("rt_update_camera_matrices", N.ptr(self._inv[0]), N.ptr(self._inv[1]))

    def update_camera(self, camera) -> None:
        """src/renderer.rs:109-129 after a move: reset, new origin, new ray directions."""
        self.scene.camera = camera
        self.reset_accumulation()
        rc = N.rt_ray_camera()
        rc.origin[:] = [float(x) for x in camera.position]
        self._call("rt_update_camera", ctypes.byref(rc))
        if self.device_rays:
            self._set_camera_matrices(camera)
            return
        self.camera_rays = np.ascontiguousarray(camera.recalculate_ray_directions())
        self._keep[0] = self.camera_rays
        self._call("rt_update_ray_directions", N.ptr(self.camera_rays), self.camera_rays.shape[0])

    def compute_frame(self, bounces: int = REFERENCE_BOUNCES) -> None:
        """src/renderer.rs:201-252 (asynchronous). Called once per frame: one ctypes
        call, the error path only on failure."""
        rc = self._lib.rt_compute_frame(self._ctx, bounces)
        if rc != N.RT_OK:
            if self._ctx is None:
                raise N.RtError(N.RT_E_INVALID, "renderer is closed")
            N.check(self._ctx, rc, self._lib)

    def compute_frames(self, bounces: int = REFERENCE_BOUNCES, frames: int = 1) -> None:
        """``frames`` compute_frame calls fused into one launch (same results;
        rt_compute_frames in include/rt_abi.h). Asynchronous."""
        self._call("rt_compute_frames", bounces, frames)

    def submit_frames(self, bounces: int = REFERENCE_BOUNCES, count: int = 1) -> None:
        """``count`` compute_frame calls in one C call (rt_submit_frames: the host loop a native
        caller runs, without a ctypes round trip per frame). Asynchronous."""
        self._call("rt_submit_frames", bounces, count)

    def set_frame_batch(self, max_frames: int) -> None:
        """rt_set_frame_batch: up to ``max_frames`` queued compute_frame calls per launch."""
        self._call("rt_set_frame_batch", max_frames)

    def frame_batch(self):
        """(max frames per launch, frames queued now)."""
        m, p = ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self._ctx, self._lib.rt_frame_batch(self._ctx, ctypes.byref(m), ctypes.byref(p)), self._lib)
        return m.value, p.value

    def flush(self) -> None:
        """Launch the queued frames now (rt_flush); every other call does so implicitly."""
        self._call("rt_flush")

    # ------------------------------------------------------------------ readback & stats
    def synchronize(self) -> None:
        self._call("rt_synchronize")

    def read_output(self) -> np.ndarray:
        out = np.zeros((self.height, self.width), np.uint32)
        self._call("rt_read_output", N.ptr(out))
        return out

    def read_accumulation(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.float32)
        self._call("rt_read_accumulation", N.ptr(out))
        return out

    def update_texture(self, alignment: int = 256) -> np.ndarray:
        """``Renderer::update_texture`` (src/renderer.rs:254-283), headless: the
        packed output as the Rgba8Unorm display texture the reference copies it
        into, one row every ``calculate_bytes_per_row`` bytes (:285-295). Returns
        the (height, bytes_per_row) u8 staging image; ``image()`` strips the pitch."""
        bpr = int(self._lib.rt_bytes_per_row(self.width, alignment))
        if bpr == 0:
            raise ValueError(f"alignment {alignment} must be a power of two")
        out = np.zeros((self.height, bpr), np.uint8)
        self._call("rt_read_output_pitched", N.ptr(out), bpr)
        return out

    def copy_output_to_device(self, dst_device_ptr: int, bytes_per_row: int) -> None:
        """``Renderer::update_texture`` on the device (src/renderer.rs:254-283): the packed
        output copied into device memory at ``dst_device_ptr`` with a row pitch, stream-ordered
        and asynchronous (rt_copy_output_to_device) -- a display loop's observation point."""
        self._call("rt_copy_output_to_device", ctypes.c_void_p(dst_device_ptr), bytes_per_row)

    def image(self) -> np.ndarray:
        """The displayed frame as an (height, width, 4) RGBA8 array (R first)."""
        return np.ascontiguousarray(self.update_texture()[:, : 4 * self.width].reshape(self.height, self.width, 4))

    def ray_count(self) -> int:
        v = ctypes.c_uint64()
        self._call("rt_ray_count", ctypes.byref(v))
        return v.value

    def reset_ray_count(self) -> None:
        self._call("rt_reset_ray_count")

    @property
    def accumulation_index(self) -> int:
        v = ctypes.c_uint32()
        self._call("rt_accumulation_index", ctypes.byref(v))
        return v.value

    def set_timing(self, enable: bool) -> None:
        self._call("rt_set_timing", int(enable))

    def dispatch_time_total(self):
        """(total milliseconds of timed path-kernel launches, number timed): each launch's
        span on the device clock (rt_set_timing)."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        self._call("rt_dispatch_time_total", ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def set_brute_force(self, enable) -> None:
        """rt_set_brute_force: the reference's own sphere and triangle sweeps (BASELINE config
        5's stress mode) instead of the acceleration structures: True / 1 with the sub-object
        records LDS-tiled, 2 streamed through the scalar cache, False / 0 off."""
        self._call("rt_set_brute_force", int(enable))

    def set_triangle_pruning(self, mode: int) -> None:
        """rt_set_triangle_pruning: distance pruning of the triangle walk.
        1 (default): per-leaf certificates (each triangle's own normal and a derived f32 error
        bound), exact by construction; 0: box culling only (exact); 2: the round-3 relative slack (faster
        on incoherent meshes, not exact)."""
        self._call("rt_set_triangle_pruning", int(mode))

    def set_tuning(self, key: str, value: int) -> None:
        """An exact variant of the schedule or of an acceleration structure (rt_set_tuning)."""
        self._call("rt_set_tuning", key.encode(), int(value))

    def streamed_bytes_l2(self) -> int:
        """Sub-object bytes the brute-force sweeps read from L2 (rt_streamed_bytes_l2)."""
        v = ctypes.c_uint64()
        self._call("rt_streamed_bytes_l2", ctypes.byref(v))
        return v.value

    def streamed_bytes(self) -> int:
        """The brute-force launches' tile-streaming bytes by SURVEY §8d's convention
        (32 B x the swept sub-objects per started 256 rays of a bounce level)."""
        v = ctypes.c_uint64()
        self._call("rt_streamed_bytes", ctypes.byref(v))
        return v.value

    def resolve_time_total(self):
        """(total milliseconds, number) of the timed batches' resolve passes
        (rt_resolve_frames_kernel), which dispatch_time_total does not include."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        self._call("rt_resolve_time_total", ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def reset_timing(self) -> None:
        self._call("rt_reset_timing")

    def owned_pixel_count(self, rank: int | None = None, world_size: int | None = None) -> int:
        v = ctypes.c_uint64()
        r = self.rank if rank is None else rank
        w = self.world_size if world_size is None else world_size
        N.check(self._ctx, self._lib.rt_owned_pixel_count(self._ctx, r, w, ctypes.byref(v)), self._lib)
        return v.value

    def pack_owned_accumulation(self, dst_device_ptr: int) -> None:
        self._call("rt_pack_owned_accumulation", ctypes.c_void_p(dst_device_ptr))

    def unpack_accumulation(self, src_device_ptr: int, src_rank: int, world_size: int, divisor: int) -> None:
        self._call("rt_unpack_accumulation", ctypes.c_void_p(src_device_ptr), src_rank, world_size, divisor)

    def pack_owned_output(self, dst_device_ptr: int) -> None:
        self._call("rt_pack_owned_output", ctypes.c_void_p(dst_device_ptr))

    def unpack_output(self, src_device_ptr: int, src_rank: int, world_size: int) -> None:
        self._call("rt_unpack_output", ctypes.c_void_p(src_device_ptr), src_rank, world_size)

    def unpack_accumulation_ranks(self, src_device_ptr: int, stride_px: int, world_size: int, skip_rank: int,
                                  divisor: int) -> None:
        """Every rank's block of a gather (block r at r * stride_px pixels) but skip_rank's, one launch."""
        self._call("rt_unpack_accumulation_ranks", ctypes.c_void_p(src_device_ptr), stride_px, world_size, skip_rank,
                   divisor)

    def unpack_output_ranks(self, src_device_ptr: int, stride_px: int, world_size: int, skip_rank: int) -> None:
        self._call("rt_unpack_output_ranks", ctypes.c_void_p(src_device_ptr), stride_px, world_size, skip_rank)

    def debug_counters(self, n: int = 8) -> list:
        """Diagnostic builds only: the 8 counters, then per-wave stamps (include/rt_abi.h)."""
        v = (ctypes.c_uint64 * n)()
        N.check(self._ctx, self._lib.rt_debug_counters(self._ctx, v, n), self._lib)
        return list(v)

    def check_leaf_certificates(self) -> tuple:
        """(mismatches, valid, total): the device's leaf certificates re-derived on the host from
        the device's own leaf records, sub-objects and triangles (include/rt_abi.h)."""
        m, v, t = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self._ctx, self._lib.rt_debug_check_leaf_certificates(self._ctx, m, v, t), self._lib)
        return m.value, v.value, t.value

    def set_tile_schedule(self, schedule: int) -> None:
        """0: claim tiles in index order; 1: cost-ordered (most rays of an earlier launch first)."""
        self._call("rt_set_tile_schedule", schedule)

    def tile_schedule_state(self):
        """(order, costs): the next launch's claim order over this rank's tiles and the rays recorded per tile."""
        n = self.owned_pixel_count() // 64
        order = np.zeros(n, np.uint32)
        costs = np.zeros(n, np.uint32)
        self._call("rt_tile_schedule_state", order.ctypes.data_as(ctypes.c_void_p),
                   costs.ctypes.data_as(ctypes.c_void_p))
        return order, costs

    def launch_config(self) -> dict:
        """Geometry of the last launch: workgroup threads, workgroups, LDS bytes, scene staged in LDS."""
        v = [ctypes.c_uint32() for _ in range(4)]
        N.check(self._ctx, self._lib.rt_launch_config(self._ctx, *[ctypes.byref(x) for x in v]), self._lib)
        return dict(zip(("threads", "blocks", "lds_bytes", "scene_in_lds"), (x.value for x in v)))

    def last_launch_passes(self) -> list:
        """Kernels the last launch ran: "path", "primary" (pre-pass), "resolve", "brute",
        "brute_stream" (the brute-force sweep's scalar-cache variant)."""
        v = ctypes.c_uint32()
        N.check(self._ctx, self._lib.rt_last_launch_passes(self._ctx, ctypes.byref(v)), self._lib)
        names = ((N.RT_PASS_PATH, "path"), (N.RT_PASS_PRIMARY, "primary"), (N.RT_PASS_RESOLVE, "resolve"),
                 (N.RT_PASS_BRUTE, "brute"), (N.RT_PASS_BRUTE_STREAM, "brute_stream"))
        return [n for bit, n in names if v.value & bit]

    @property
    def stream_handle(self) -> int:
        return self._lib.rt_stream(self._ctx) or 0

    def close(self) -> None:
        if self._ctx is not None:
            self._lib.rt_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
