"""Several GPUs in one process through the C ABI: rt_create_multi + rt_gather_frame.

The one-GPU test box runs a group of one device: the contexts, the per-device
host threads, ncclCommInitAll and the gather's grouped ncclSend/ncclRecv (the
root's own block goes through RCCL too) all run; the assembled frame must equal a
plain one-context render bit for bit. RCCL runs one rank per device, so groups of
3 and 4 ranks run here with the copy transport (rt_create_multi_ex with
RT_GROUP_COPY_TRANSPORT: every rank a context and host thread of its own on device
0, the root's N receive slots filled by device copies): the group's N-rank logic --
tile ownership, per-rank threads, the root's slots and unpack -- bit-exact against
one context before the driver's 8-GPU node runs it over RCCL.
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


@pytest.mark.parametrize("n,root,config,batch,kw", [
    (3, 0, "c2_rtiow", 1, {}),
    (3, 2, "c3_chess", 3, dict(env_size=(512, 256))),
    (4, 1, "c2_rtiow", 4, {}),
    (4, 0, "c5_heightfield", None, dict(nx=120, nz=60)),
])
def test_gpu_group_n_ranks_on_one_device(gpu, n, root, config, batch, kw):
    """N ranks on device 0 (copy transport): after 5 frames, both payloads gathered to
    `root` equal one context's render; then a group-wide reset and material update,
    4 more frames, and both gathers again (the second gather's copies wait for the
    first one's unpack)."""
    scene, bounces = build_config(config, width=136, height=80, **kw)
    rays = scene.camera.recalculate_ray_directions()
    mats = scene.materials.copy()
    mats["emission_power"][0] = np.float32(1.75)
    from rust_gpu_raytracing_amd import _native as N

    with Renderer(scene, camera_rays=rays) as r:
        for _ in range(5):
            r.compute_frame(bounces)
        acc1, out1, n1 = r.read_accumulation(), r.read_output(), r.ray_count()
        r.reset_accumulation()
        r._call("rt_update_materials", N.ptr(mats), mats.shape[0])
        for _ in range(4):
            r.compute_frame(bounces)
        acc2, out2, n2 = r.read_accumulation(), r.read_output(), r.ray_count()

    with RendererGroup(scene, [0] * n, camera_rays=rays, frame_batch=batch, copy_transport=True) as g:
        assert g.size == n
        for _ in range(5):
            g.compute_frame(bounces)
        assert g.ray_count() == n1
        g.gather(root, "image")
        assert np.array_equal(g.read_output(root), out1)
        g.gather(root, "accumulation")
        assert np.array_equal(g.read_accumulation(root).view(np.uint32), acc1.view(np.uint32))
        assert np.array_equal(g.read_output(root), out1)
        g.reset_accumulation()
        g.update_materials(mats)
        for _ in range(4):
            g.compute_frame(bounces)
        g.gather(root, "accumulation")
        g.gather(root, "image")
        assert np.array_equal(g.read_accumulation(root).view(np.uint32), acc2.view(np.uint32))
        assert np.array_equal(g.read_output(root), out2)
        assert g.ray_count() == n2


def test_gpu_group_copy_transport_camera_move(gpu):
    """A camera move through a 3-rank copy-transport group (rt_group_update_camera + new ray
    directions + reset), then frames and a gather: one context's render of the same calls."""
    scene, bounces = build_config("c3_chess", width=96, height=64, env_size=(512, 256))
    import copy

    cam2 = copy.deepcopy(scene.camera)
    cam2.position = np.array([1.0, -5.0, 22.0], np.float32)
    cam2.recalculate_view()
    with Renderer(scene) as r:
        for _ in range(2):
            r.compute_frame(bounces)
        r.update_camera(cam2)
        for _ in range(3):
            r.compute_frame(bounces)
        acc_ref, out_ref = r.read_accumulation(), r.read_output()
    scene2, _ = build_config("c3_chess", width=96, height=64, env_size=(512, 256))
    with RendererGroup(scene2, [0, 0, 0], copy_transport=True) as g:
        for _ in range(2):
            g.compute_frame(bounces)
        g.update_camera(cam2)
        for _ in range(3):
            g.compute_frame(bounces)
        g.gather(0, "accumulation")
        assert np.array_equal(g.read_accumulation(0).view(np.uint32), acc_ref.view(np.uint32))
        assert np.array_equal(g.read_output(0), out_ref)
