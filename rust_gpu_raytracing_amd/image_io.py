"""Headless output of a rendered frame.

The reference only shows ``output_data`` in a window (``copy_buffer_to_texture``
+ ``render_shader.wgsl``, src/renderer.rs:254-283). Here a frame is written to
disk instead: binary PPM (RGB) or PNG (RGBA, 8-bit, no filtering), with the
standard library only. Input is the (height, width, 4) u8 array of
``Renderer.image()`` -- or the packed u32 output, whose byte order is R, G, B, A.
"""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np


def unpack_rgba8(packed: np.ndarray) -> np.ndarray:
    """(h, w) u32 from ``pack_to_u32`` (compute_shader.wgsl:192-208, R in bits 0-7) -> (h, w, 4) u8."""
    p = np.ascontiguousarray(packed, np.uint32)
    return p.astype("<u4").view(np.uint8).reshape(*p.shape, 4)


def _rgba(img: np.ndarray) -> np.ndarray:
    img = np.asarray(img)
    if img.dtype == np.uint32 and img.ndim == 2:
        img = unpack_rgba8(img)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an (h, w, 4) uint8 RGBA image or an (h, w) packed uint32 frame")
    return np.ascontiguousarray(img)


def save_ppm(path, img) -> Path:
    """Binary PPM (P6), alpha dropped."""
    rgba = _rgba(img)
    h, w = rgba.shape[:2]
    path = Path(path)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(rgba[..., :3]).tobytes())
    return path


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def save_png(path, img, level: int = 6) -> Path:
    """8-bit RGBA PNG (colour type 6), filter type 0 on every row."""
    rgba = _rgba(img)
    h, w = rgba.shape[:2]
    raw = np.zeros((h, 1 + 4 * w), np.uint8)  # filter byte 0, then the row
    raw[:, 1:] = rgba.reshape(h, 4 * w)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + \
        _chunk(b"IEND", b"")
    path = Path(path)
    path.write_bytes(data)
    return path


def load_png(path) -> np.ndarray:
    """Reads back what ``save_png`` writes (8-bit RGBA, filter 0 rows): for tests."""
    data = Path(path).read_bytes()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if kind == b"IHDR":
            w, h, depth, ctype, _, _, _ = struct.unpack(">IIBBBBB", body)
            if (depth, ctype) != (8, 6):
                raise ValueError("only 8-bit RGBA PNGs are supported")
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    if np.any(raw[:, 0] != 0):
        raise ValueError("only unfiltered rows are supported")
    return raw[:, 1:].reshape(h, w, 4).copy()
