"""Several GPUs in one process through the C ABI: rt_create_multi + rt_gather_frame.

The one-GPU test box runs a group of one device: the contexts, the per-device
host threads, ncclCommInitAll and the gather's grouped ncclSend/ncclRecv (the
root's own block goes through RCCL too) all run; the assembled frame must equal a
plain one-context render bit for bit. More devices per group are the driver's
8-GPU node (RCCL runs one rank per device).
"""
import numpy as np
import pytest

from rust_gpu_raytracing_amd import Renderer
from rust_gpu_raytracing_amd.group import RendererGroup
from rust_gpu_raytracing_amd.scene import build_config

pytestmark = pytest.mark.gpu


def _reference(scene, bounces, frames, rays, **kw):
    with Renderer(scene, camera_rays=rays, **kw) as r:
        for _ in range(frames):
            r.compute_frame(bounces)
        return r.read_accumulation(), r.read_output(), r.ray_count()


@pytest.mark.parametrize("config,batch,kw", [
    ("c2_rtiow", 1, {}),
    ("c2_rtiow", 4, {}),
    ("c3_chess", 3, dict(env_size=(512, 256))),
])
def test_gpu_group_gather_matches_single_context(gpu, config, batch, kw):
    scene, bounces = build_config(config, width=200, height=112, **kw)
    rays = scene.camera.recalculate_ray_directions()
    acc_ref, out_ref, n_ref = _reference(scene, bounces, 7, rays)
    with RendererGroup(scene, [0], camera_rays=rays, frame_batch=batch) as g:
        assert g.size == 1
        for _ in range(7):
            g.compute_frame(bounces)
        g.gather(0, "image")
        out = g.read_output(0)
        assert np.array_equal(out, out_ref)
        g.gather(0, "accumulation")
        acc, out2 = g.read_accumulation(0), g.read_output(0)
        assert np.array_equal(acc.view(np.uint32), acc_ref.view(np.uint32))
        assert np.array_equal(out2, out_ref)
        assert g.ray_count() == n_ref


def test_gpu_group_reset_and_updates(gpu):
    """Group-wide reset and material update, then more frames and a gather: the same
    state as one context given the same calls."""
    scene, bounces = build_config("c2_rtiow", width=128, height=72)
    rays = scene.camera.recalculate_ray_directions()
    mats = scene.materials.copy()
    mats["emission_power"][1] = np.float32(2.5)

    with Renderer(scene, camera_rays=rays) as r:
        for _ in range(3):
            r.compute_frame(bounces)
        r.reset_accumulation()
        from rust_gpu_raytracing_amd import _native as N
        r._call("rt_update_materials", N.ptr(mats), mats.shape[0])
        for _ in range(4):
            r.compute_frame(bounces)
        acc_ref, out_ref = r.read_accumulation(), r.read_output()

    with RendererGroup(scene, [0], camera_rays=rays, frame_batch=2) as g:
        for _ in range(3):
            g.compute_frame(bounces)
        g.reset_accumulation()
        g.update_materials(mats)
        for _ in range(4):
            g.compute_frame(bounces)
        g.gather(0, "accumulation")
        assert np.array_equal(g.read_accumulation(0).view(np.uint32), acc_ref.view(np.uint32))
        assert np.array_equal(g.read_output(0), out_ref)


def test_gpu_group_rejects_bad_gather(gpu):
    from rust_gpu_raytracing_amd import RtError

    scene, bounces = build_config("c1_four_spheres", width=64, height=48)
    with RendererGroup(scene, [0], accumulate=False) as g:
        g.compute_frame(bounces)
        with pytest.raises(RtError):
            g.gather(1, "image")  # root out of range
        with pytest.raises(RtError):
            g.gather(0, "accumulation")  # never written without accumulation
        g.gather(0, "image")
        g.synchronize()
