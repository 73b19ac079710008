"""Known-answer tests that pin the CPU oracle (oracle/pathtrace_oracle.c).

The reference has no tests or golden data, so each primitive of
compute_shader.wgsl is checked against an independent computation: pure-Python
integer PCG, libm in double precision, closed-form ray/sphere and ray/triangle
hits, and the SURVEY Appendix B PCG vectors.
"""
import ctypes
import math

import numpy as np
import pytest

from rust_gpu_raytracing_amd import buffers as B
from rust_gpu_raytracing_amd.camera import Camera
from rust_gpu_raytracing_amd.scene import RenderScene, SceneObject, solid_color_image

M32 = 0xFFFFFFFF


def pcg_py(seed: int) -> int:
    """compute_shader.wgsl:587-599 in Python integers."""
    state = (seed * 747796405 + 2891336453) & M32
    word = ((state >> ((state >> 28) + 4)) ^ state) & M32
    word = (word * 277803737) & M32
    return ((word >> 22) ^ word) & M32


# (pixel index, random_index) -> next 4 seeds and their f32 values
APPENDIX_B = [
    (0, 1, 0x00000000, [129708002, 817759070, 2145236065, 2368882721],
     [0.030199997, 0.19039936, 0.49947670, 0.55154848]),
    (1, 1, 0x0004FBE0, [2393977086, 3228683874, 105208503, 3455255200],
     [0.55739123, 0.75173652, 0.024495764, 0.80448931]),
    (1037760, 1, 0xEB6E4800, [727271878, 851565475, 2820831546, 3034249371],
     [0.16933118, 0.19827054, 0.65677601, 0.70646626]),
    (1037760, 7, 0x7003F800, [132734782, 318340152, 394070762, 3221229965],
     [0.030904725, 0.074119344, 0.091751747, 0.75000107]),
]


@pytest.mark.parametrize("idx,k,seed0,seeds,floats", APPENDIX_B)
def test_pcg_appendix_b(oracle_lib, idx, k, seed0, seeds, floats):
    L = oracle_lib.lib()
    seed = (idx * k * 326624) & M32  # compute_shader.wgsl:217
    assert seed == seed0
    s = ctypes.c_uint32(seed)
    py = seed
    for want_seed, want_f in zip(seeds, floats):
        f = L.oracle_random(ctypes.byref(s))
        py = pcg_py(py)
        assert s.value == want_seed == py
        assert np.float32(f) == np.float32(np.float32(want_seed) / np.float32(4294967296.0))
        assert abs(f - want_f) < 1e-7


def test_pcg_matches_python_random_seeds(oracle_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(1)
    for seed in list(rng.integers(0, 2**32, 2000, dtype=np.uint64)) + [0, 1, M32, 2**31]:
        s = ctypes.c_uint32(int(seed))
        f = L.oracle_random(ctypes.byref(s))
        want = pcg_py(int(seed))
        assert s.value == want
        # normalize_u32 (:630-632): f32(value) / f32(U32_MAX), f32(U32_MAX) == 2^32
        assert f == float(np.float32(np.float32(want) / np.float32(2**32)))


def _ulps(got, ref):
    r = np.float32(ref)
    sp = np.spacing(np.abs(r)) if r != 0 else np.float32(1.4e-45)
    return abs(got - ref) / float(sp)


@pytest.mark.parametrize(
    "name,ref,lo,hi,max_ulp",
    [
        ("oracle_logf", math.log, 1e-30, 1.0, 1.5),
        ("oracle_cosf", math.cos, 0.0, 6.2831852, 2.0),
        ("oracle_asinf", math.asin, -1.0, 1.0, 3.0),
        ("oracle_acosf", math.acos, -1.0, 1.0, 2.0),
        ("oracle_atanf", math.atan, -50.0, 50.0, 3.0),
    ],
)
def test_transcendentals_vs_libm(oracle_lib, name, ref, lo, hi, max_ulp):
    fn = getattr(oracle_lib.lib(), name)
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(lo, hi, 20000), np.linspace(lo, hi, 2001)]).astype(np.float32)
    worst = 0.0
    for x in xs:
        got, want = fn(float(x)), ref(float(x))
        if abs(got - want) <= 2.0**-40:  # next to a zero of the function: absolute error is what matters
            continue
        worst = max(worst, _ulps(got, want))
    assert worst <= max_ulp, (name, worst)


def test_atan2_quadrants_and_specials(oracle_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(3)
    worst = 0.0
    for y, x in rng.uniform(-4, 4, (20000, 2)).astype(np.float32):
        worst = max(worst, _ulps(L.oracle_atan2f(float(y), float(x)), math.atan2(float(y), float(x))))
    assert worst <= 3.0
    assert L.oracle_atan2f(0.0, 1.0) == 0.0
    assert L.oracle_atan2f(1.0, 0.0) == np.float32(math.pi / 2)
    assert L.oracle_atan2f(-1.0, 0.0) == -np.float32(math.pi / 2)
    assert L.oracle_atan2f(0.0, -1.0) == np.float32(math.pi)
    assert math.isnan(L.oracle_atan2f(float("nan"), 1.0))


def test_log_edges(oracle_lib):
    L = oracle_lib.lib()
    assert L.oracle_logf(0.0) == -math.inf  # random() == 0 -> rho = inf (reproduced, not fixed)
    assert L.oracle_logf(1.0) == 0.0
    assert math.isnan(L.oracle_logf(-1.0))
    assert abs(L.oracle_logf(1e-40) - math.log(1e-40)) < 1e-4  # denormal input


def test_acos_asin_domain(oracle_lib):
    L = oracle_lib.lib()
    assert math.isnan(L.oracle_acosf(1.0000001))  # |n.y| > 1 after normalize -> NaN uv -> texel 0
    assert math.isnan(L.oracle_asinf(-1.0000001))
    assert L.oracle_acosf(1.0) == 0.0
    assert L.oracle_asinf(1.0) == np.float32(math.pi / 2)


def test_srgb_table(oracle_lib):
    L = oracle_lib.lib()
    t = np.zeros(256, np.float32)
    L.oracle_srgb_table(t.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    c = np.arange(256) / 255.0
    want = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4).astype(np.float32)
    assert np.array_equal(t, want)
    assert t[0] == 0.0 and t[255] == 1.0


@pytest.mark.parametrize(
    "rgba,want",
    [
        ((0.0, 0.0, 0.0, 0.0), 0x00000000),
        ((1.0, 1.0, 1.0, 1.0), 0xFFFFFFFF),
        ((0.5, 0.25, 0.75, 1.0), (127 | (63 << 8) | (191 << 16) | (255 << 24))),  # truncation, not rounding
        ((0.999, 0.0039, 0.00393, 0.5), (254 | (0 << 8) | (1 << 16) | (127 << 24))),
    ],
)
def test_pack_to_u32(oracle_lib, rgba, want):
    L = oracle_lib.lib()
    c = (ctypes.c_float * 4)(*rgba)
    assert L.oracle_pack(c) == want


# ---------------------------------------------------------------- intersection KATs


def _scene(spheres=(), tris=None, n_mat=2):
    sph = np.zeros(len(spheres), B.SPHERE)
    for i, (p, r, m) in enumerate(spheres):
        sph[i]["position"], sph[i]["radius"], sph[i]["material_index"] = p, r, m
    mats = np.zeros(n_mat, B.MATERIAL)
    objs = []
    if tris is not None:
        a, b, c = (np.asarray(x, np.float32) for x in tris)
        t = B.scene_triangles(a, b, c)
        info = np.zeros((), B.OBJECT_INFO)
        allp = np.concatenate([a, b, c])
        info["min_bounds"], info["max_bounds"], info["material_index"] = allp.min(0), allp.max(0), 1
        o = SceneObject(info, t)
        o.create_sub_objects(0, 0)
        objs.append(o)
    tex = np.stack([solid_color_image([1, 1, 1], (2, 2))] * 2)
    env = solid_color_image([0.5, 0.5, 0.5], (4, 2))
    return RenderScene(sph, mats, objs, tex, env, Camera(8, 8))


def _trace(oracle_lib, scene, o, d):
    orc = oracle_lib.Oracle(scene)
    return orc.trace(scene.params(), o, d)


def test_sphere_closed_form(oracle_lib):
    scene = _scene([([0.0, 0.0, -5.0], 1.0, 1)])
    h = _trace(oracle_lib, scene, [0, 0, 0], [0, 0, -1])
    assert h.t == pytest.approx(4.0, abs=1e-6)
    assert (h.nx, h.ny, h.nz) == pytest.approx((0, 0, 1), abs=1e-6)
    assert h.front_face == 1 and h.material_index == 1


def test_inside_sphere_misses(oracle_lib):
    # near root only (:389): a ray starting inside the sphere gets t < 0 and misses it
    scene = _scene([([0.0, 0.0, 0.0], 2.0, 1)])
    h = _trace(oracle_lib, scene, [0, 0, 0], [0, 0, -1])
    assert h.t == np.float32(3.4028235e38)


def test_sphere_tie_first_wins(oracle_lib):
    # two identical spheres: strict `<` keeps the first (:391)
    scene = _scene([([0.0, 0.0, -5.0], 1.0, 0), ([0.0, 0.0, -5.0], 1.0, 1)])
    h = _trace(oracle_lib, scene, [0, 0, 0], [0, 0, -1])
    assert h.material_index == 0


def test_triangle_hit_and_faces(oracle_lib):
    tri = ([[-1.0, -1.0, -3.0]], [[1.0, -1.0, -3.0]], [[0.0, 1.0, -3.0]])
    scene = _scene(tris=tri)
    h = _trace(oracle_lib, scene, [0, 0, 0], [0, 0, -1])
    assert h.t == pytest.approx(3.0, abs=1e-6)
    # calc_normal = ab x ac = +z; det = -dot(d, n) > 0 -> front face, normal = +face_normal
    assert h.front_face == 1 and (h.nx, h.ny, h.nz) == pytest.approx((0, 0, 1))
    h2 = _trace(oracle_lib, scene, [0, 0, -6], [0, 0, 1])
    assert h2.front_face == 0 and (h2.nx, h2.ny, h2.nz) == pytest.approx((0, 0, -1))
    miss = _trace(oracle_lib, scene, [5, 5, 0], [0, 0, -1])
    assert miss.t == np.float32(3.4028235e38)


def test_sphere_triangle_tie_goes_to_triangle(oracle_lib):
    # sphere surface and triangle both at t = 4 exactly: `sphere.t < tri.t` is false -> triangle (:347)
    tri = ([[-1.0, -1.0, -4.0]], [[1.0, -1.0, -4.0]], [[0.0, 1.0, -4.0]])
    scene = _scene([([0.0, 0.0, -5.0], 1.0, 0)], tris=tri)
    h = _trace(oracle_lib, scene, [0, 0, 0], [0, 0, -1])
    assert h.t == 4.0 and h.material_index == 1


def test_triangle_uv_from_object_bounds(oracle_lib):
    # object_texture_coords (:568-578): uv = ((p - min) / (max - min)).xz of the OBJECT box
    tri = ([[0.0, 0.0, 0.0]], [[4.0, 0.0, 0.0]], [[0.0, 0.0, 4.0]])
    scene = _scene(tris=tri)
    h = _trace(oracle_lib, scene, [1.0, -5.0, 1.0], [0, 1, 0])
    assert (h.u, h.v) == pytest.approx((0.25, 0.25))
