"""Capture the chess scene's input assets from the reference checkout into a
compact fixture, so the chess configuration (BASELINE.json configs[2]) can be
built on machines without /root/reference (the GPU box).

Writes rust_gpu_raytracing_amd/data/chess_assets.npz:
  stl_<Name>   (n, 3, 3) float32  triangle vertices of 3D_models/<Name>.stl
                                  (binary STL, in file order; normals dropped)
  tex_earth    (400, 400, 4) uint8  textures/earth.png as RGBA8 (alpha 255)
  tex_chess    (400, 400, 4) uint8  textures/chess.png as RGBA8
These are data (meshes and images) decoded to arrays, not reference code.
Run: python tools/make_chess_assets.py [/root/reference]
"""
import struct
import sys
from pathlib import Path

import numpy as np
from PIL import Image

MODELS = ["Wall", "Pawn", "Rook", "Bishop", "Queen", "Knight", "King"]


def read_binary_stl(path: Path) -> np.ndarray:
    data = path.read_bytes()
    (n,) = struct.unpack_from("<I", data, 80)
    assert len(data) == 84 + 50 * n, f"{path} is not a binary STL"
    rec = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("attr", "<u2")]),
                        count=n, offset=84)
    return np.ascontiguousarray(rec["v"], dtype=np.float32)


def main(ref: Path) -> None:
    out = {}
    for name in MODELS:
        out[f"stl_{name}"] = read_binary_stl(ref / "3D_models" / f"{name}.stl")
    out["tex_earth"] = np.asarray(Image.open(ref / "textures" / "earth.png").convert("RGBA"), np.uint8)
    out["tex_chess"] = np.asarray(Image.open(ref / "textures" / "chess.png").convert("RGBA"), np.uint8)
    dst = Path(__file__).resolve().parents[1] / "rust_gpu_raytracing_amd" / "data" / "chess_assets.npz"
    np.savez_compressed(dst, **out)
    print(dst, dst.stat().st_size, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference"))
