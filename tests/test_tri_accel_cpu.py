"""CPU proof-by-test of the triangle accelerator (tests/cpp/tri_exactness.cpp).

The kernel's BVH traversal over (object, sub-object) pairs, restated in C++ with
the same f32 operation order, must pick exactly the triangle, object, facing and
distance of the reference's sequential sweep (compute_shader.wgsl:422-517) —
including first-wins ties (duplicate triangles), objects sharing sub-objects,
grazing rays, and rays lying exactly in a triangle's plane (NaN distance, which
the sweep accepts unconditionally and the kernel hands back to the sweep).
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from rust_gpu_raytracing_amd import buffers as B
from rust_gpu_raytracing_amd.scene import SceneObject, build_config, load_stl_files, load_chess_assets
from tests.adversarial import grazing_rays, tilted_plane_grid

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("tri") / "tri_exactness"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'rust_gpu_raytracing_amd' / 'csrc'}", str(ROOT / "tests" / "cpp" / "tri_exactness.cpp"),
                    str(ROOT / "rust_gpu_raytracing_amd" / "csrc" / "sphere_bvh.cpp"), "-o", str(exe)], check=True)
    return exe


def run(harness, tmp_path, objs, subs, tris, rays, margin=None, env=None):
    for name, arr in (("o", objs), ("s", subs), ("t", tris), ("r", rays.astype(np.float32))):
        np.ascontiguousarray(arr).tofile(tmp_path / f"{name}.bin")
    cmd = [str(harness)] + [str(tmp_path / f"{n}.bin") for n in "ostr"] + ([margin] if margin else [])
    return subprocess.run(cmd, capture_output=True, text=True, env=env)


def random_rays(rng, n, lo, hi, planes_y=()):
    o = rng.uniform(lo, hi, (n, 3))
    tgt = rng.uniform(lo, hi, (n, 3))
    d = (tgt - o) * rng.uniform(0.3, 3.0, (n, 1))
    k = n // 10
    d[:k, 1] = 0.0  # horizontal rays ...
    for i, y in enumerate(planes_y):  # ... some lying exactly in axis-aligned triangle planes (NaN distance)
        o[i * 7:(i + 1) * 7, 1] = y
    d[k:2 * k, 0] = 0.0  # axis-parallel components
    return np.concatenate([o, d], axis=1)


def test_chess_scene_random_rays(harness, tmp_path):
    scene, _ = build_config("c3_chess", width=16, height=16, env_size=(16, 8), texture_size=(8, 8))
    objs, subs, tris = scene.flatten()
    rng = np.random.default_rng(0)
    rays = random_rays(rng, 60000, [-12, -8, -12], [12, 8, 12], planes_y=[float(tris["a"][0][1])])
    out = run(harness, tmp_path, objs, subs, tris, rays)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    assert line(out, "qnodes")[0] == "1"  # quantized nodes walked and checked too


def test_heightfield_and_grazing_rays(harness, tmp_path):
    scene, _ = build_config("c5_heightfield", width=8, height=8, nx=120, nz=60)
    objs, subs, tris = scene.flatten()
    rng = np.random.default_rng(1)
    n = 60000
    o = np.stack([rng.uniform(-20, 20, n), rng.uniform(-3, 0.4, n), rng.uniform(-20, 10, n)], axis=1)
    d = np.stack([rng.uniform(-1, 1, n), rng.uniform(0.0, 0.2, n) ** 3, rng.uniform(-1, 1, n)], axis=1)  # grazing
    out = run(harness, tmp_path, objs, subs, tris, np.concatenate([o, d], axis=1))
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    _, nr, hits, tests, nodes, _ = out.stdout.splitlines()[0].split()
    assert float(tests) < 0.05 * tris.shape[0]  # the accelerator culls
    # the 16-B quantized nodes (tri_qnode.h): every box contains its node's, the walk over them
    # returns the sweep's result on every ray (checked above), and the coarser boxes cost few visits
    q_valid, q_nodes = line(out, "qnodes")
    assert int(q_valid) == 1 and float(q_nodes) < 1.1 * float(nodes)
    # the default global-memory walk: octant layouts + distance pruning, the
    # sweep's result on every ray (checked above) with fewer visits and triangle tests
    p_nodes, p_tests = line(out, "prune")
    assert float(p_nodes) < float(nodes) and float(p_tests) < float(tests)


def test_shared_subobjects_duplicates_and_ties(harness, tmp_path):
    """Objects that share sub-objects (the same triangles reached twice, with
    different object boxes and materials) and exact duplicate triangles: the
    sweep order decides ties."""
    meshes = load_chess_assets()
    objs_l = load_stl_files([("Pawn", 2.0, [0.0, 0.0, 0.0], [90.0, 0.0, 0.0], 1),
                             ("Pawn", 2.0, [0.0, 0.0, 0.0], [90.0, 0.0, 0.0], 2),  # identical copy: full ties
                             ("Rook", 2.0, [0.3, 0.0, 0.2], [90.0, 0.0, 0.0], 3)],
                            {k[4:]: v for k, v in meshes.items() if k.startswith("stl_")})
    objs = np.stack([np.asarray(o.object_info) for o in objs_l]).astype(B.OBJECT_INFO)
    subs = np.concatenate([o.sub_object_info for o in objs_l]).astype(B.SUB_OBJECT_INFO)
    tris = np.concatenate([o.triangles for o in objs_l]).astype(B.TRIANGLE)
    # a 4th object re-using object 0's sub-objects, with a larger box
    extra = objs[0].copy()
    extra["min_bounds"] -= 1.0
    extra["max_bounds"] += 1.0
    objs = np.concatenate([objs, extra[None]]).astype(B.OBJECT_INFO)
    rng = np.random.default_rng(2)
    rays = random_rays(rng, 40000, [-2, -3, -2], [2, 1, 2])
    out = run(harness, tmp_path, objs, subs, tris, rays)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    assert int(out.stdout.splitlines()[0].split()[2]) > 1000  # plenty of hits exercised the tie rule


def test_nan_distance_falls_back_to_the_sweep(harness, tmp_path):
    # a horizontal quad at y = 0.5 and rays lying exactly in its plane: det == 0 and
    # the origin on the plane -> NaN distance, accepted by the sweep (:457)
    a = np.array([[-1, 0.5, -1], [1, 0.5, -1]], np.float32)
    b = np.array([[1, 0.5, -1], [1, 0.5, 1]], np.float32)
    c = np.array([[-1, 0.5, 1], [-1, 0.5, 1]], np.float32)
    t = B.scene_triangles(a, b, c)
    o = SceneObject(np.zeros((), B.OBJECT_INFO), t)
    o.object_info["min_bounds"] = [-1, 0.5, -1]
    o.object_info["max_bounds"] = [1, 0.5, 1]
    o.create_sub_objects(0, 0)
    objs = np.stack([np.asarray(o.object_info)]).astype(B.OBJECT_INFO)
    rays = np.array([[-3, 0.5, 0.1, 1, 0, 0], [0.2, 0.5, -3, 0, 0, 1], [0, 0, 0, 0, 1, 0.01]], np.float32)
    out = run(harness, tmp_path, objs, o.sub_object_info.astype(B.SUB_OBJECT_INFO), t, rays)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    assert int(out.stdout.splitlines()[0].split()[-1]) >= 1  # the fallback ran
    # the kernel's default walk (cooperative leaf batches) met the NaN distance in its merge too
    gap_checked, gap_skipped, coop_leaves, coop_nan = map(int, line(out, "kernel_default"))
    assert coop_leaves > 0 and coop_nan > 0


def test_margin_is_load_bearing(harness, tmp_path):
    scene, _ = build_config("c3_chess", width=16, height=16, env_size=(16, 8), texture_size=(8, 8))
    objs, subs, tris = scene.flatten()
    rays = random_rays(np.random.default_rng(3), 40000, [-12, -8, -12], [12, 8, 12])
    out = run(harness, tmp_path, objs, subs, tris, rays, margin="-0.02")  # shrunken boxes must be caught
    assert out.returncode == 1 and "MISMATCH" in out.stdout


def test_large_sub_objects_and_inconsistent_records(harness, tmp_path):
    """Sub-objects of 20 triangles (leaves beyond the cooperative batch's 7 slots, tested per
    lane) and triangle records whose calc_normal does not follow from their edges (uploaded
    data need not be consistent; certificates are built from the records as stored)."""
    scene, _ = build_config("c5_heightfield", width=8, height=8, nx=40, nz=20)
    obj = scene.objects[0]
    obj.create_sub_objects(0, 0, n=20)
    objs, subs, tris = scene.flatten()
    tris = tris.copy()
    bad = np.arange(0, tris.shape[0], 97)
    tris["calc_normal"][bad] *= np.float32(1.0000001)  # one ulp-ish off: not SceneTriangle::new's result
    rng = np.random.default_rng(5)
    n = 30000
    o = np.stack([rng.uniform(-20, 20, n), rng.uniform(-3, 0.4, n), rng.uniform(-20, 10, n)], axis=1)
    d = np.stack([rng.uniform(-1, 1, n), rng.uniform(0.0, 1.0, n), rng.uniform(-1, 1, n)], axis=1)
    out = run(harness, tmp_path, objs, subs, tris, np.concatenate([o, d], axis=1))
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout


def test_quantized_node_properties(tmp_path):
    """tri_qnode.h on random roots and boxes (1e-30 .. 1e6, denormals, signed zeros, flat
    boxes): the exact decode contains every stored box, and links round-trip."""
    exe = tmp_path / "qnode_props"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'rust_gpu_raytracing_amd' / 'csrc'}", str(ROOT / "tests" / "cpp" / "qnode_props.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "3000"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    assert int(out.stdout.split()[2]) > 100000


def line(out, key):
    return next(x for x in out.stdout.splitlines() if x.startswith(key + " ")).split()[1:]


@pytest.mark.parametrize("seed,h_range,c_range", [(2, (1e-7, 1e-5), (1e-9, 1e-6)), (1, (1e-6, 1e-4), (1e-8, 1e-5)),
                                                  (0, (1e-4, 1e-2), (1e-6, 1e-3))])
def test_adversarial_grazing_rays_certified_pruning(harness, tmp_path, seed, h_range, c_range):
    """Rays built within 1e-9..1e-3 rad of a triangle plane that passes 1e-7..1e-2 from their
    origin, the regime where the reference's f32 distance and barycentrics are dominated by
    rounding. The certified walk (tri_cone.h, the kernel's default) must
    return the sweep's triangle on every ray (the harness exits 1 on the first mismatch); the
    round-3 relative-slack limit (t (1 + 2^-6) + 2^-10 (|o| + E) / |d|, now only an opt-in
    mode) is counted instead, and on the most grazing sets it does miss the sweep's result."""
    objs, subs, tris, _, frame = tilted_plane_grid(seed)
    rays = grazing_rays(frame, 16000, h_range, c_range, seed + 10)
    out = run(harness, tmp_path, objs, subs, tris, rays, env={"TRI_HEUR_COUNT": "1"})
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    misses = int(line(out, "heuristic_misses")[0])
    if c_range[1] <= 1e-5:
        assert misses > 0  # the heuristic slack is not exact: a ray it gets wrong
    nodes, tests, checked, skipped, tris_skipped, valid, total = line(out, "certified")
    assert int(valid) == int(total)  # every leaf of the grid carries a certificate
    if c_range[1] >= 1e-3:
        assert float(skipped) > 0  # and where the bound allows, the certified walk does skip leaves
    # the kernel's default walk on the same rays (exact: checked ray by ray above): the certificate
    # test deferred through node_step's gap (tri_leafcert_skips_gap) and the cooperative leaf batch's
    # merge; the deferred test does run, and skips whole leaves where the bound allows
    gap_checked, gap_skipped, coop_leaves, coop_nan = map(int, line(out, "kernel_default"))
    assert gap_checked > 0 and coop_leaves > 0
    if c_range[1] >= 1e-3:
        assert gap_skipped > 0


def test_certified_pruning_real_scenes(harness, tmp_path):
    """The certified walk on C3's chess scene with random rays: exact, a certificate for every
    leaf, and fewer triangle tests than box culling."""
    scene, _ = build_config("c3_chess", width=16, height=16, env_size=(16, 8), texture_size=(8, 8))
    objs, subs, tris = scene.flatten()
    rays = random_rays(np.random.default_rng(7), 30000, [-12, -8, -12], [12, 8, 12])
    out = run(harness, tmp_path, objs, subs, tris, rays)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout
    nodes, tests, checked, skipped, tris_skipped, valid, total = line(out, "certified")
    assert int(valid) == int(total)
    box_tests = float(out.stdout.splitlines()[0].split()[3])
    assert float(skipped) > 0 and float(tests) < box_tests
