"""Time split of the frame loop from an RT_DIAG build (in-kernel s_memtime stamps).

usage: RT_LIB=build/variants/lib_diag.so python tools/diag_split.py [--frame-batch F] [config ...]
Reports, summed over waves, the share of wave-cycles spent in the traversal
loop (step 4 of the kernel loop); the rest is shading, RNG, refill and
framebuffer I/O. Also: traversal steps per ray and mean lanes per step.
Stamps serialise the wave around each trace: read shares, not absolute times.
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402

SIZES = {"c1_four_spheres": (800, 600), "c2_rtiow": (1920, 1080), "c3_chess": (1920, 1080),
         "c4_mixed": (1920, 1080), "c5_heightfield": (1920, 1080)}

argv = sys.argv[1:]
fb = 1
if argv[:1] == ["--frame-batch"]:
    fb, argv = int(argv[1]), argv[2:]
for name in argv or list(SIZES):
    w, h = SIZES[name]
    scene, bounces = build_config(name, width=w, height=h)
    with Renderer(scene, frame_batch=fb) as r:
        for _ in range(fb):
            r.compute_frame(bounces)
        r.synchronize()
        r.reset_ray_count()
        for _ in range(3 * fb):
            r.compute_frame(bounces)
        c = r.debug_counters(10)
        rays = r.ray_count()
    total, trav, steps, it, step_lanes, shade, refill, setup, leaf_cyc, leaf_steps = c[:10]
    print(json.dumps({"config": name, "frame_batch": fb, "trav_share": trav / total, "shade_share": shade / total,
                      "refill_share": refill / total, "setup_share": setup / total,
                      "rest_share": 1 - (trav + shade + refill + setup) / total,
                      "cycles_per_ray": total / rays, "steps_per_ray": steps / rays,
                      "lanes_per_step": step_lanes / max(steps, 1), "outer_iters_per_ray": it / rays,
                      "leaf_share": leaf_cyc / total, "leaf_steps_per_ray": leaf_steps / rays}))
