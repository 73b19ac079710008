"""How far a different-but-valid transcendental library moves the image.

WGSL leaves log/cos/asin/atan2 implementation-defined (compute_shader.wgsl:558-584,
622-627); the oracle and the kernel pin them to the same Cephes-style polynomials, so
they agree bit for bit, but a wgpu/lavapipe run of the reference would use the
driver's own. This tool bounds that gap with evidence: a timing/analysis build whose
Box-Muller log/cos are the hardware approximations (-DRT_EXP_HW_TRANSCENDENTALS,
v_log_f32 / v_cos_f32: a few ulp from the pinned ones) renders N accumulated frames
of a BASELINE configuration, and the per-channel RMS against the oracle's frames is
reported for the averaged colour (accum / (k*c), the value the RGBA8 pack clamps)
and for the packed RGBA8 output (/255), with the fraction of pixels that differ.

usage: python tools/parity_budget.py <variant.so> [--configs c2_rtiow c3_chess] [--frames 16]
(build the variant first: python tools/build_variant.py build/variants/hw_transc.so -DRT_EXP_HW_TRANSCENDENTALS)
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle import oracle as O  # noqa: E402  (analysis tool: the oracle is the checker)
from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd import _native as N  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def rms(a, b):
    a = np.nan_to_num(a.reshape(-1, 4).astype(np.float64), nan=0.0, posinf=0.0, neginf=0.0)
    b = np.nan_to_num(b.reshape(-1, 4).astype(np.float64), nan=0.0, posinf=0.0, neginf=0.0)
    return np.sqrt(((a - b) ** 2).mean(axis=0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant")
    ap.add_argument("--configs", nargs="*", default=["c2_rtiow", "c3_chess"])
    ap.add_argument("--frames", type=int, default=16)
    args = ap.parse_args()
    lib = N.load_library(args.variant)
    for name in args.configs:
        scene, bounces = build_config(name)
        rays = scene.camera.recalculate_ray_directions()
        with Renderer(scene, camera_rays=rays, lib=lib) as r:
            for _ in range(args.frames):
                r.compute_frame(bounces)
            acc_v, out_v, n_v = r.read_accumulation(), r.read_output(), r.ray_count()
        o = O.Oracle(scene, camera_rays=rays)
        acc_o = np.zeros_like(acc_v)
        out_o = np.zeros_like(out_v)
        n_o = 0
        for k in range(1, args.frames + 1):
            n_o += o.render_frame(scene.params(accumulation_index=k), bounces, acc_o, out_o)
        div = float(args.frames)  # k * c after the last frame (k = frames, c = 1)
        col_v, col_o = acc_v / div, acc_o / div
        rgba_v = out_v.view(np.uint8).reshape(out_v.shape + (4,)).astype(np.float64) / 255.0
        rgba_o = out_o.view(np.uint8).reshape(out_o.shape + (4,)).astype(np.float64) / 255.0
        print(json.dumps({
            "config": name, "frames": args.frames, "variant": Path(args.variant).name,
            "rms_colour_per_channel": rms(col_v, col_o).tolist(),
            "rms_rgba8_per_channel": rms(rgba_v, rgba_o).tolist(),
            "pixels_differing": float((acc_v != acc_o).any(axis=-1).mean()),
            "rays_variant": n_v, "rays_oracle": n_o,
            "north_star_tolerance": 1e-4,
        }), flush=True)


if __name__ == "__main__":
    main()
