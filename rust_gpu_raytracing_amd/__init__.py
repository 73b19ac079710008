"""MI355X-native per-pixel path tracer: the hot path of juhotuho10/rust_GPU_raytracing.

``compute_shader.wgsl`` is a hand-written gfx950 HIP kernel behind the C ABI in
``include/rt_abi.h``; :class:`Renderer` mirrors ``src/renderer.rs`` on top of it.
"""
from . import buffers
from ._native import NativeLibraryError, RtError, load_library
from .camera import Camera
from .renderer import REFERENCE_BOUNCES, Renderer
from .scene import CONFIGS, RenderScene, build_config

__all__ = [
    "buffers",
    "Camera",
    "CONFIGS",
    "NativeLibraryError",
    "REFERENCE_BOUNCES",
    "RenderScene",
    "Renderer",
    "RtError",
    "build_config",
    "load_library",
]
