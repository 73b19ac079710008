"""Probe: one frame rendered as S concurrent launches on S streams (S contexts on
one device, each owning every S-th tile as rank s of world S), against one launch.
Wall time per frame over K frames (analysis tool).

usage: python tools/split_probe.py [config] [frames] [S ...]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c2_rtiow"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
splits = [int(x) for x in sys.argv[3:]] or [1, 2, 3, 4]
scene, bounces = build_config(name)
rays = scene.camera.recalculate_ray_directions()
res = {}
ref = None
for S in splits:
    rs = [Renderer(scene, camera_rays=rays, rank=s, world_size=S) for s in range(S)]
    for _ in range(3):
        for r in rs:
            r.compute_frame(bounces)
    for r in rs:
        r.synchronize()
    best = []
    for _ in range(5):
        for r in rs:
            r.reset_ray_count()
        t0 = time.perf_counter()
        for _ in range(K):
            for r in rs:
                r.compute_frame(bounces)
        for r in rs:
            r.synchronize()
        best.append((time.perf_counter() - t0) * 1e3 / K)
    n = sum(r.ray_count() for r in rs) / K
    acc = np.zeros((scene.camera.viewport_height, scene.camera.viewport_width, 4), np.float32)
    for r in rs:
        a = r.read_accumulation()
        m = np.any(a != 0, axis=-1)
        acc[m] = a[m]
    if ref is None:
        ref = acc
    res[S] = {"ms_per_frame": round(float(np.median(best)), 4), "mray_s": round(n / np.median(best) / 1e3, 1),
              "same_as_first": bool(np.array_equal(acc.view(np.uint32), ref.view(np.uint32)))}
    for r in rs:
        r.close()
print(json.dumps({"config": name, "frames": K, "splits": res}))
