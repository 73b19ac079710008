"""Generate the committed golden fixtures (tests/golden/*.npz) with the CPU oracle.

Each fixture holds the complete kernel inputs (so it does not depend on the
scene builders staying bit-stable) and the oracle's outputs after a sequence of
frames sequenced like Renderer::compute_frame (k = 1, 2, ...):
  inputs : camera_origin, camera_rays, spheres, materials, triangles, objects,
           sub_objects, textures, env, params (per frame), bounces
  outputs: accum (H, W, 4) f32, out (H, W) u32, rays (total counted segments)
The reference itself cannot run here: these pin the oracle and the
HIP kernel to each other and against regressions, not to the WGSL.
Run: python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402
from tests.golden.fixtures import CASES, render_case_with_oracle, scene_inputs  # noqa: E402


def main():
    out_dir = Path(__file__).resolve().parent
    for name, case in CASES.items():
        scene, _ = build_config(case["config"], width=case["width"], height=case["height"], **case.get("kw", {}))
        inputs = scene_inputs(scene)
        accum, out, rays = render_case_with_oracle(inputs, case)
        np.savez_compressed(out_dir / f"{name}.npz", accum=accum, out=out, rays=np.uint64(rays), **inputs)
        print(name, accum.shape, rays, (out_dir / f"{name}.npz").stat().st_size)


if __name__ == "__main__":
    main()
