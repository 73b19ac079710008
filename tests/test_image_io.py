"""Headless display output: row pitch rule, RGBA8 unpacking, PNG/PPM files.

CPU only; the device-side pitched copy is tested in test_gpu_parity.py."""
import numpy as np
import pytest

from rust_gpu_raytracing_amd import image_io as I


@pytest.mark.parametrize("width,align,expect", [
    (800, 256, 3328),    # 3200 B rounded up: the reference's 800-px config breaks its 64-px rule (src/main.rs:51-53)
    (1600, 256, 6400),   # the reference's window width, a multiple of 64 px
    (1920, 256, 7680),
    (1, 256, 256),
    (13, 4, 52),
    (13, 3, 0),          # alignment must be a power of two
    (0, 256, 0),
])
def test_bytes_per_row_matches_calculate_bytes_per_row(native_lib, width, align, expect):
    # src/renderer.rs:285-295: (4*width + alignment - 1) & !(alignment - 1)
    assert native_lib.rt_bytes_per_row(width, align) == expect


def test_unpack_matches_pack_to_u32_layout():
    # pack_to_u32 (compute_shader.wgsl:192-208): R bits 0-7, G 8-15, B 16-23, A 24-31
    packed = np.array([[0x44332211, 0xFF000080]], np.uint32)
    rgba = I.unpack_rgba8(packed)
    assert rgba.shape == (1, 2, 4)
    assert rgba[0, 0].tolist() == [0x11, 0x22, 0x33, 0x44]
    assert rgba[0, 1].tolist() == [0x80, 0, 0, 0xFF]


def test_png_roundtrip_and_packed_input(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    assert np.array_equal(I.load_png(I.save_png(tmp_path / "a.png", img)), img)
    packed = img.reshape(-1, 4).view("<u4").reshape(37, 53)
    assert np.array_equal(I.load_png(I.save_png(tmp_path / "b.png", packed)), img)


def test_ppm_layout(tmp_path):
    img = np.zeros((2, 3, 4), np.uint8)
    img[..., 0] = 7
    img[1, 2] = [1, 2, 3, 4]
    data = I.save_ppm(tmp_path / "a.ppm", img).read_bytes()
    head = b"P6\n3 2\n255\n"
    assert data.startswith(head) and len(data) == len(head) + 2 * 3 * 3
    assert data[-3:] == bytes([1, 2, 3])


def test_rejects_bad_images(tmp_path):
    with pytest.raises(ValueError):
        I.save_png(tmp_path / "x.png", np.zeros((4, 4, 3), np.uint8))
