"""Time split of the frame loop from an RT_DIAG build (in-kernel s_memtime stamps).

usage: RT_LIB=build/variants/lib_diag.so python tools/diag_split.py [--frame-batch F] [config ...]
Reports, summed over waves, the share of wave-cycles spent in the traversal
loop (step 4 of the kernel loop); the rest is shading, RNG, refill and
framebuffer I/O. Also: traversal steps per ray and mean lanes per step, the lane
occupancy of each phase, the inactive-lane share of the wave cycles by phase, and
which branch the shaded lanes took (sky miss / glass / specular / diffuse).
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
        c = r.debug_counters(28)
        rays = r.ray_count()
    total, trav, steps, it, step_lanes, shade, refill, setup, leaf_cyc, leaf_steps = c[:10]
    sh_pass, sh_lanes, miss, glass, spec, su_pass, su_lanes = c[12:19]
    cert_checks, cert_leaves, cert_tris = c[19:22]  # leaf certificates (certified pruning)
    # sphere-only kernels: wave-level node steps and their lanes, the sphere-group tests run inside
    # them (a group runs for the whole wave when any lane is at a leaf) and the lanes at a leaf
    n_steps, n_step_lanes, n_groups, n_group_lanes = c[22:26]
    # sphere-only kernels since round 6: the group tests run once per block of unrolled node steps
    # for every lane that reached a leaf in it (words 24/25 then count node steps with a lane at a leaf)
    n_blocks, n_block_lanes = c[26:28]
    trav_occ = step_lanes / max(steps, 1) / 64
    shade_occ = sh_lanes / max(sh_pass, 1) / 64
    setup_occ = su_lanes / max(su_pass, 1) / 64
    # inactive-lane share of all wave cycles, by phase: the phase's cycles x (1 - its mean occupancy)
    idle = {"traversal": trav / total * (1 - trav_occ), "shading": shade / total * (1 - shade_occ),
            "setup": setup / total * (1 - setup_occ), "refill_and_rest": (total - trav - shade - setup) / total}
    hits = max(sh_lanes - miss, 1)
    print(json.dumps({"config": name, "frame_batch": fb, "trav_share": trav / total, "shade_share": shade / total,
                      "refill_share": refill / total, "setup_share": setup / total,
                      "rest_share": 1 - (trav + shade + refill + setup) / total,
                      "cycles_per_ray": total / rays, "steps_per_ray": steps / rays,
                      "lanes_per_step": step_lanes / max(steps, 1), "outer_iters_per_ray": it / rays,
                      "leaf_share": leaf_cyc / total, "leaf_steps_per_ray": leaf_steps / rays,
                      "sphere_node_steps": {"per_ray": n_steps / rays, "lanes_per_step": n_step_lanes / max(n_steps, 1),
                                            "steps_with_a_group_test": n_groups / max(n_steps, 1),
                                            "lanes_per_group_test": n_group_lanes / max(n_groups, 1),
                                            "block_group_tests_per_ray": n_blocks / rays,
                                            "lanes_per_block_group_test": n_block_lanes / max(n_blocks, 1)},
                      "leaf_certificates_per_ray": {"checked": cert_checks / rays, "leaves_skipped": cert_leaves / rays,
                                                    "triangles_skipped": cert_tris / rays},
                      "occupancy": {"traversal": trav_occ, "shading": shade_occ, "setup": setup_occ},
                      "inactive_lane_share_by_phase": idle,
                      "shaded_lanes": {"sky_miss": miss / max(sh_lanes, 1), "hit_glass": glass / hits,
                                       "hit_specular": spec / hits, "hit_diffuse": 1 - (glass + spec) / hits},
                      "note": "shading of a hit runs Box-Muller (3 normal draws) for every hit lane"}))
