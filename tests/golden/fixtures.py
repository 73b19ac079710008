"""Golden-fixture cases and helpers shared by make_golden.py and the tests."""
from pathlib import Path

import numpy as np

from rust_gpu_raytracing_amd import buffers as B
from rust_gpu_raytracing_amd.camera import Camera
from rust_gpu_raytracing_amd.scene import RenderScene, SceneObject

GOLDEN_DIR = Path(__file__).resolve().parent

# name -> case. frames are rendered with accumulation_index k = 1..frames.
CASES = {
    # C1 geometry at a small size, 4 bounces, 1 spp, 3 accumulated frames
    "c1_64x48_b4": dict(config="c1_four_spheres", width=64, height=48, bounces=4, frames=3, spp=1, accumulate=1),
    # the reference's own settings: 10 bounces, compute_per_frame 5 (src/main.rs:92)
    "c1_40x24_b10_spp5": dict(config="c1_four_spheres", width=40, height=24, bounces=10, frames=2, spp=5,
                              accumulate=1),
    # non-accumulating path (compute_shader.wgsl:171-175), ragged size (not a multiple of 8)
    "c1_37x21_noacc": dict(config="c1_four_spheres", width=37, height=21, bounces=4, frames=1, spp=1, accumulate=0),
    # C2 RTIOW, 8 bounces
    "c2_64x36_b8": dict(config="c2_rtiow", width=64, height=36, bounces=8, frames=2, spp=1, accumulate=1),
    # C3 chess (triangles + textures + env map), 8 bounces, reduced texture/env sizes
    "c3_64x36_b8": dict(config="c3_chess", width=64, height=36, bounces=8, frames=2, spp=1, accumulate=1,
                        kw=dict(env_size=(256, 128), texture_size=(100, 100))),
}


def scene_inputs(scene: RenderScene) -> dict:
    objs, subs, tris = scene.flatten()
    return dict(
        camera_origin=np.asarray(scene.camera.position, np.float32),
        camera_rays=scene.camera.recalculate_ray_directions(),
        spheres=scene.spheres, materials=scene.materials, triangles=tris, objects=objs, sub_objects=subs,
        textures=np.ascontiguousarray(scene.textures), env=np.ascontiguousarray(scene.environment_map),
        width=np.uint32(scene.camera.viewport_width), height=np.uint32(scene.camera.viewport_height),
    )


def scene_from_inputs(inputs) -> RenderScene:
    """Rebuild a RenderScene whose arrays are exactly the stored inputs."""
    w, h = int(inputs["width"]), int(inputs["height"])
    cam = Camera(w, h, position=np.asarray(inputs["camera_origin"], np.float32))
    objs = []
    objects = np.asarray(inputs["objects"]).astype(B.OBJECT_INFO)
    subs = np.asarray(inputs["sub_objects"]).astype(B.SUB_OBJECT_INFO)
    tris = np.asarray(inputs["triangles"]).astype(B.TRIANGLE)
    for o in objects:
        so = SceneObject(np.array(o, B.OBJECT_INFO), tris[:0])
        objs.append(so)
    scene = RenderScene(np.asarray(inputs["spheres"]).astype(B.SPHERE), np.asarray(inputs["materials"]).astype(B.MATERIAL),
                        objs, np.asarray(inputs["textures"]), np.asarray(inputs["env"]), cam, name="golden")
    scene.flatten = lambda: (objects, subs, tris)  # exact stored arrays, already globally indexed
    return scene


def params_for(scene, case, k):
    return scene.params(accumulate=case["accumulate"], compute_per_frame=case["spp"], accumulation_index=k)


def render_case_with_oracle(inputs, case, threads=0):
    from oracle.oracle import Oracle

    scene = scene_from_inputs(inputs)
    o = Oracle(scene, camera_rays=np.asarray(inputs["camera_rays"]).astype(B.RAY))
    accum = np.zeros((o.height, o.width, 4), np.float32)
    out = np.zeros((o.height, o.width), np.uint32)
    rays = 0
    for k in range(1, case["frames"] + 1):
        rays += o.render_frame(params_for(scene, case, k), case["bounces"], accum, out, threads=threads)
    return accum, out, rays


def load(name):
    with np.load(GOLDEN_DIR / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
