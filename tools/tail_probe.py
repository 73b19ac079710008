"""Ramp and tail of the persistent grid, from an RT_DIAG_TAIL build.

usage: RT_LIB=build/variants/lib_tail.so python tools/tail_probe.py [--frame-batch F] [--split R/N] [config ...]
With --frame-batch F each probed launch renders a batch of F frames (rt_set_frame_batch).
Per launch: first wave start -> mean/last wave start (ramp), mean/last wave end
(tail), when waves first found the tile queue empty (dry) and how long they ran
after that (drain), in microseconds of the device's 100 MHz real-time clock.
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402

HEADER = 32  # kDiagHeaderWords (csrc/rt_kernel_args.h): counters ahead of the per-wave records
argv = sys.argv[1:]
fb = 1
rank, world = 0, 1
while argv[:1] in (["--frame-batch"], ["--split"]):
    if argv[0] == "--frame-batch":
        fb, argv = int(argv[1]), argv[2:]
    else:  # --split R/N: rank R's share of an N-way tile split (the strong-scaling bench)
        rank, world = map(int, argv[1].split("/"))
        argv = argv[2:]
for name in argv or ["c2_rtiow"]:
    scene, bounces = build_config(name)
    with Renderer(scene, frame_batch=fb, rank=rank, world_size=world) as r:
        for _ in range(fb):
            r.compute_frame(bounces)
        r.synchronize()
        res = []
        for _ in range(5):
            r.reset_ray_count()  # zeroes the diag counters too
            r.reset_timing()
            r.set_timing(True)
            for _ in range(fb):
                r.compute_frame(bounces)
            r.synchronize()
            r.set_timing(False)
            kern_ms, _ = r.dispatch_time_total()
            c = r.debug_counters(HEADER + 2 * 65536)
            waves = np.array(c[HEADER:HEADER + 2 * c[3]], np.float64).reshape(-1, 2)
            t_first = (~np.uint64(c[2])).item()  # stored as the max of ~start
            dry = (waves[:, 0] - t_first) / 100.0   # when the wave first found the queue empty
            dur = (waves[:, 1] - waves[:, 0]) / 100.0  # its drain: queue dry -> wave end
            ends = (waves[:, 1] - t_first) / 100.0
            n = c[3]
            res.append({"waves": n, "ramp_mean_us": (c[4] / n - t_first) / 100, "ramp_last_us": (c[5] - t_first) / 100,
                        "end_mean_us": (c[0] / n - t_first) / 100, "end_last_us": (c[1] - t_first) / 100,
                        "nan_fallbacks": c[6], "longest_wave_us": c[7] / 100, "kernel_us": kern_ms * 1e3,
                        "dry_pct": [round(float(np.percentile(dry, q)), 1) for q in (0, 10, 50, 90, 100)],
                        "drain_pct": [round(float(np.percentile(dur, q)), 1) for q in (10, 50, 90, 99, 100)],
                        "end_pct": [round(float(np.percentile(ends, q)), 1) for q in (10, 50, 90, 99, 100)]})
        print(json.dumps({"config": name, "frame_batch": fb, "split": f"{rank}/{world}", "runs": res[1:]}))
