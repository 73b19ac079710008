"""Scene preparation (off the hot path): the arrays the kernel consumes.

* ``SceneObject`` / ``load_stl_files`` restate src/triangle_object.rs:16-331
  (STL placement: rotate, normalise, scale, drop to the surface, translate;
  7-triangle sub-objects with AABBs), in f32 with glam's operation order.
* ``solid_color_image`` restates src/image_texture.rs:40-55.
* ``RenderScene`` mirrors src/renderer.rs:17-26 and ``flatten`` is
  ``get_triangle_data`` (src/renderer.rs:298-320).
* ``build_config`` makes the five BASELINE.json workloads.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import buffers as B
from .camera import Camera

f32 = np.float32
DATA_DIR = Path(__file__).resolve().parent / "data"
SUB_OBJECT_TRIANGLES = 7  # src/triangle_object.rs:125


# --------------------------------------------------------------------------- textures


def solid_color_image(color, size) -> np.ndarray:
    """src/image_texture.rs:40-55: RGBA8 image, ``(c * 255.0) as u8`` per channel, alpha 255."""
    w, h = size
    c = np.asarray(color, np.float32) * f32(255.0)
    rgb = np.clip(np.floor(c), 0, 255).astype(np.uint8)  # Rust `as u8` saturates and truncates
    img = np.empty((h, w, 4), np.uint8)
    img[..., :3] = rgb
    img[..., 3] = 255
    return img


def srgb_encode(linear: np.ndarray) -> np.ndarray:
    """Linear [0,1] -> sRGB-encoded u8 (so that the kernel's Rgba8UnormSrgb decode returns ~linear)."""
    x = np.clip(np.asarray(linear, np.float64), 0.0, 1.0)
    s = np.where(x <= 0.0031308, 12.92 * x, 1.055 * np.power(x, 1.0 / 2.4) - 0.055)
    return np.clip(np.round(s * 255.0), 0, 255).astype(np.uint8)


# --------------------------------------------------------------------------- f32 glam helpers


def _mat3_mul_vec(cols: np.ndarray, v: np.ndarray) -> np.ndarray:
    """glam Mat3A * Vec3A: ((c0*x + c1*y) + c2*z) in f32; v is (n, 3)."""
    v = v.astype(np.float32)
    r = cols[0][None, :] * v[:, 0:1]
    r = r + cols[1][None, :] * v[:, 1:2]
    r = r + cols[2][None, :] * v[:, 2:3]
    return r.astype(np.float32)


def _mat3_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.stack([_mat3_mul_vec(a, b[i][None, :])[0] for i in range(3)]).astype(np.float32)


def _sin_cos(angle: np.float32):
    return f32(math.sin(float(angle))), f32(math.cos(float(angle)))


def rotation_matrix(rotation_deg) -> np.ndarray:
    """``rotate_to_angle`` (src/triangle_object.rs:253-269): Rz * Ry * Rx, columns, f32."""
    k = f32(f32(math.pi) / f32(180.0))
    rx, ry, rz = (f32(d) * k for d in np.asarray(rotation_deg, np.float32))
    sx, cx = _sin_cos(rx)
    sy, cy = _sin_cos(ry)
    sz, cz = _sin_cos(rz)
    mx = np.array([[1, 0, 0], [0, cx, sx], [0, -sx, cx]], np.float32)
    my = np.array([[cy, 0, -sy], [0, 1, 0], [sy, 0, cy]], np.float32)
    mz = np.array([[cz, sz, 0], [-sz, cz, 0], [0, 0, 1]], np.float32)
    return _mat3_mul(_mat3_mul(mz, my), mx)


_F32_MAX = np.float32(np.finfo(np.float32).max)


def _sequential_extreme(col: np.ndarray, lower: bool) -> np.float32:
    """One axis of get_bounding_box's scan: start at +-f32::MAX and replace on a
    strict `<` (`>`), so NaN and values beyond the start never win and of equal
    values (+0 / -0) the first one in point order is kept."""
    cand = col[col < _F32_MAX] if lower else col[col > -_F32_MAX]
    if cand.size == 0:
        return _F32_MAX if lower else -_F32_MAX
    m = cand.min() if lower else cand.max()
    return cand[np.argmax(cand == m)]


def bounding_box(points: np.ndarray):
    """``get_bounding_box`` (src/triangle_object.rs:292-321), bit for bit."""
    pts = np.asarray(points, np.float32).reshape(-1, 3)
    mn = np.array([_sequential_extreme(pts[:, k], True) for k in range(3)], np.float32)
    mx = np.array([_sequential_extreme(pts[:, k], False) for k in range(3)], np.float32)
    return mn, mx


# --------------------------------------------------------------------------- objects


@dataclass
class SceneObject:
    """src/triangle_object.rs:39-52.

    ``normalized_points`` are the model's vertices after normalize_model and
    scale_model (before the drop to the surface), one (3, 3) block per triangle
    in triangle order (the reference keeps a deduplicated vertex list plus
    ``point_indexes``; the vertices are the same). ``rotation`` (degrees),
    ``scale`` and ``transformation`` are the edit state that
    ``update_triangles`` applies (:129-150)."""

    object_info: np.ndarray  # OBJECT_INFO record
    triangles: np.ndarray  # TRIANGLE records
    sub_object_info: np.ndarray = field(default_factory=lambda: np.zeros(0, B.SUB_OBJECT_INFO))
    normalized_points: np.ndarray = field(default_factory=lambda: np.zeros((0, 3), np.float32))
    rotation: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    scale: np.float32 = np.float32(1.0)
    transformation: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    n_sub_object_triangles: int = SUB_OBJECT_TRIANGLES

    @classmethod
    def from_triangles(cls, tri_vertices: np.ndarray, scale: float, coordinates, rotation, material_index: int):
        """``SceneObject::new`` (src/triangle_object.rs:55-127) from (n, 3, 3) STL vertices."""
        assert scale > 0.0, "scale has to be over 0.0"
        pts = np.asarray(tri_vertices, np.float32).reshape(-1, 3)
        # normalize_model, :237-251
        pts = _mat3_mul_vec(rotation_matrix(rotation), pts)
        mn, mx = bounding_box(pts)
        average = ((mn + mx) / f32(2.0)).astype(np.float32)
        d = (mn - mx).astype(np.float32)
        dist = np.sqrt(B.dot_f32(d, d))
        s = f32(1.0) / dist
        pts = (pts * s - average * s).astype(np.float32)
        # scale_model, :278-283
        pts = (pts * f32(scale)).astype(np.float32)
        scaled = pts.copy()
        mn, mx = bounding_box(pts)
        # transform_points_to_surface, :323-331
        surface = ((-mx) * np.array([0, 1, 0], np.float32)).astype(np.float32)  # -max * Vec3A::Y
        pts = (pts + surface).astype(np.float32)
        coords = np.asarray(coordinates, np.float32)
        pts = (pts + coords).astype(np.float32)
        shift = (surface + coords).astype(np.float32)
        mn = (mn + shift).astype(np.float32)
        mx = (mx + shift).astype(np.float32)
        v = pts.reshape(-1, 3, 3)
        tris = B.scene_triangles(v[:, 0], v[:, 1], v[:, 2])
        info = np.zeros((), B.OBJECT_INFO)
        info["min_bounds"] = mn
        info["max_bounds"] = mx
        info["material_index"] = material_index
        # :114-126: scale 1, rotation 0, transformation = coordinates + surface drop
        return cls(info, tris, normalized_points=scaled, scale=f32(1.0), rotation=np.zeros(3, np.float32),
                   transformation=(coords + surface).astype(np.float32))

    def update_triangles(self):
        """src/triangle_object.rs:129-150: rotate the normalised points to
        ``rotation``, scale, translate; new object bounds and triangles."""
        pts = _mat3_mul_vec(rotation_matrix(self.rotation), self.normalized_points)
        pts = (pts * f32(self.scale)).astype(np.float32)
        pts = (pts + np.asarray(self.transformation, np.float32)).astype(np.float32)
        mn, mx = bounding_box(pts)
        self.object_info["min_bounds"] = mn
        self.object_info["max_bounds"] = mx
        v = pts.reshape(-1, 3, 3)
        self.triangles = B.scene_triangles(v[:, 0], v[:, 1], v[:, 2])

    def update_sub_objects(self):
        """src/triangle_object.rs:199-220: sub-object AABBs from the current triangles."""
        n = self.n_sub_object_triangles
        for k in range(self.sub_object_info.shape[0]):
            chunk = self.triangles[k * n:(k + 1) * n]
            allb = np.stack([chunk["min_bounds"], chunk["max_bounds"]], axis=1).reshape(-1, 3)
            mn, mx = bounding_box(allb)
            self.sub_object_info[k]["min_bounds"] = mn
            self.sub_object_info[k]["max_bounds"] = mx

    def set_model_to_surface(self):
        """src/triangle_object.rs:149-154 (``max_bounds * Vec3A::Y``, elementwise in f32)."""
        y = (np.asarray(self.object_info["max_bounds"], np.float32) * np.array([0, 1, 0], np.float32)).astype(np.float32)
        self.transformation = (np.asarray(self.transformation, np.float32) - y).astype(np.float32)

    def reset_rotation(self):
        """src/triangle_object.rs:156-158."""
        self.rotation = np.zeros(3, np.float32)

    def create_sub_objects(self, start_sub: int, start_tri: int, n: int = SUB_OBJECT_TRIANGLES):
        """src/triangle_object.rs:160-197: chunks of ``n`` triangles with their AABBs."""
        count = self.triangles.shape[0]
        n_sub = (count + n - 1) // n
        subs = np.zeros(n_sub, B.SUB_OBJECT_INFO)
        for k in range(n_sub):
            chunk = self.triangles[k * n:(k + 1) * n]
            # the reference interleaves [min0, max0, min1, max1, ...] (:171-174)
            allb = np.stack([chunk["min_bounds"], chunk["max_bounds"]], axis=1).reshape(-1, 3)
            mn, mx = bounding_box(allb)
            subs[k]["min_bounds"] = mn
            subs[k]["max_bounds"] = mx
            subs[k]["first_triangle_index"] = start_tri + k * n
            subs[k]["triangle_count"] = chunk.shape[0]
        self.object_info["first_sub_object_index"] = start_sub
        self.object_info["sub_object_count"] = n_sub
        self.sub_object_info = subs
        return start_sub + n_sub, start_tri + count


def load_stl_files(creations, meshes) -> list:
    """``load_stl_files`` (src/triangle_object.rs:16-37). ``creations`` are
    (model, scale, coordinates, rotation, material_index) tuples; ``meshes`` maps
    a model name to its (n, 3, 3) vertices."""
    objs = []
    sub_i = tri_i = 0
    for model, scale, coords, rot, mat in creations:
        o = SceneObject.from_triangles(meshes[model], scale, coords, rot, mat)
        sub_i, tri_i = o.create_sub_objects(sub_i, tri_i)
        objs.append(o)
    return objs


def load_chess_assets() -> dict:
    path = DATA_DIR / "chess_assets.npz"
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# --------------------------------------------------------------------------- scene


@dataclass
class RenderScene:
    """src/renderer.rs:17-26 plus the camera the frame is rendered from."""

    spheres: np.ndarray
    materials: np.ndarray
    objects: list
    textures: np.ndarray  # (layers, th, tw, 4) uint8, sRGB-encoded
    environment_map: np.ndarray  # (eh, ew, 4) uint8, sRGB-encoded
    camera: Camera
    name: str = "scene"

    @property
    def texture_size(self):
        return (self.textures.shape[2], self.textures.shape[1])

    @property
    def env_map_size(self):
        return (self.environment_map.shape[1], self.environment_map.shape[0])

    def flatten(self):
        """``get_triangle_data`` (src/renderer.rs:298-320)."""
        if self.objects:
            objs = np.stack([np.asarray(o.object_info) for o in self.objects]).astype(B.OBJECT_INFO)
            subs = np.concatenate([o.sub_object_info for o in self.objects]).astype(B.SUB_OBJECT_INFO)
            tris = np.concatenate([o.triangles for o in self.objects]).astype(B.TRIANGLE)
        else:
            objs = np.zeros(0, B.OBJECT_INFO)
            subs = np.zeros(0, B.SUB_OBJECT_INFO)
            tris = np.zeros(0, B.TRIANGLE)
        return np.ascontiguousarray(objs), np.ascontiguousarray(subs), np.ascontiguousarray(tris)

    def params(self, *, accumulate=1, compute_per_frame=1, accumulation_index=1) -> np.ndarray:
        """Params as ``Renderer::reset_accumulation`` builds them (src/renderer.rs:134-147)."""
        tw, th = self.texture_size
        ew, eh = self.env_map_size
        return B.make_params(
            self.camera.viewport_width,
            accumulation_index=accumulation_index,
            accumulate=accumulate,
            sphere_count=self.spheres.shape[0],
            object_count=len(self.objects),
            compute_per_frame=compute_per_frame,
            texture_width=tw,
            texture_height=th,
            texture_count=self.textures.shape[0],
            env_map_width=ew,
            env_map_height=eh,
        )


def _material(texture_index, roughness, emission, specular, scatter, glass, ior):
    m = np.zeros((), B.MATERIAL)
    m["texture_index"] = texture_index
    m["roughness"] = roughness
    m["emission_power"] = emission
    m["specular"] = specular
    m["specular_scatter"] = scatter
    m["glass"] = glass
    m["refraction_index"] = ior
    return m


def _sphere(pos, radius, material_index):
    s = np.zeros((), B.SPHERE)
    s["position"] = pos
    s["radius"] = radius
    s["material_index"] = material_index
    return s


# Materials of src/define_scene.rs:55-253, as
# (texture_index, roughness, emission_power, specular, specular_scatter, glass, refraction_index).
REFERENCE_MATERIALS = [
    (0, 0.4, 0.0, 0.6, 0.0, 1.0, 2.0),    # shiny_green
    (1, 0.9, 0.0, 0.1, 1.0, 0.0, 1.0),    # rough_blue
    (2, 0.7, 5.0, 0.5, 0.1, 0.0, 1.0),    # glossy_pink
    (3, 0.3, 15.0, 0.3, 0.1, 0.0, 1.0),   # shiny_orange
    (4, 0.9, 2.0, 0.0, 1.0, 0.0, 1.0),    # earth_material
    (5, 0.7, 0.0, 0.5, 0.1, 1.0, 1.5),    # shiny_white
] + [(i, 0.9, 0.0, 0.2, 0.2, 0.0, 1.0) for i in range(6, 18)] + [  # 12 chess piece materials
    (18, 0.6, 0.0, 0.3, 0.1, 0.0, 1.0),   # chess_board_material
]

# Texture colours of src/define_scene.rs:24-51 (None = image texture).
REFERENCE_TEXTURE_COLORS = [
    [1.0, 0.0, 0.0], [0.0, 0.6, 1.0], [1.0, 0.1, 0.1], [1.0, 0.7, 0.0], None, [1.0, 1.0, 1.0],
] + [[0.2, 0.2, 0.2]] * 6 + [[1.0, 1.0, 1.0]] * 6 + [None]

# Spheres of src/define_scene.rs:257-276.
REFERENCE_SPHERES = [([1.0, -1.2, -2.0], 0.5, 2), ([-5.0, -2.0, 9.0], 2.0, 4), ([3.0, -25.0, -5.0], 7.0, 3)]


def chess_objects(meshes) -> list:
    """The 34 placements of src/define_scene.rs:278-551."""
    tile = f32(1.51)
    b_pos, w_pos = np.array([5.3, -0.7, 0.0], np.float32), np.array([-5.3, -0.7, 0.0], np.float32)
    b_rot, w_rot = [90.0, 0.0, 0.0], [90.0, 180.0, 0.0]

    def off(x, z):
        return np.array([x, 0.0, z], np.float32)

    queen, king = off(0, f32(0.5) * tile), off(0, f32(-0.5) * tile)
    rook, knight, bishop = off(0, f32(3.5) * tile), off(0, f32(2.5) * tile), off(0, f32(1.5) * tile)
    pawns = [off(-tile, f32(z) * tile) for z in (3.5, 2.5, 1.5, 0.5, -0.5, -1.5, -2.5, -3.5)]
    c = [("Wall", 200.0, [0.0, 7.066, 0.0], [0.0, 0.0, 0.0], 1)]
    c += [("Queen", 2.0, b_pos + queen, b_rot, 6), ("King", 2.0, b_pos + king, b_rot, 7),
          ("Rook", 2.0, b_pos + rook, b_rot, 8), ("Rook", 2.0, b_pos - rook, b_rot, 8),
          ("Knight", 2.0, b_pos + knight, b_rot, 9), ("Knight", 2.0, b_pos - knight, b_rot, 9),
          ("Bishop", 2.0, b_pos + bishop, b_rot, 10), ("Bishop", 2.0, b_pos - bishop, b_rot, 10)]
    c += [("Pawn", 2.0, b_pos + p, b_rot, 11) for p in pawns]
    c += [("Queen", 2.0, w_pos - queen, w_rot, 12), ("King", 2.0, w_pos - king, w_rot, 13),
          ("Rook", 2.0, w_pos + rook, w_rot, 14), ("Rook", 2.0, w_pos - rook, w_rot, 14),
          ("Knight", 2.0, w_pos + knight, w_rot, 15), ("Knight", 2.0, w_pos - knight, w_rot, 15),
          ("Bishop", 2.0, w_pos + bishop, w_rot, 16), ("Bishop", 2.0, w_pos - bishop, w_rot, 16)]
    c += [("Pawn", 2.0, w_pos - p, w_rot, 17) for p in pawns]
    c += [("Wall", 20.0, [0.0, 0.0, 0.0], [0.0, 90.0, 0.0], 18)]
    return load_stl_files(c, meshes)


def procedural_env_map(width: int, height: int, sun=(0.3, 0.28), sun_radius=0.012) -> np.ndarray:
    """Stand-in for env_maps/studio_garden.png (missing from the reference mount,
    SURVEY §2 row 12): sky gradient above the horizon, ground below, a sun disc.
    Row 0 is straight up (v = 0.5 + asin(d.y)/pi with -Y up, compute_shader.wgsl:580-585)."""
    v = (np.arange(height, dtype=np.float64) + 0.5) / height
    elev = (0.5 - v) * math.pi  # +pi/2 at row 0 (zenith)
    t = np.clip(np.sin(elev), 0.0, 1.0)[:, None]
    zenith, horizon, ground = np.array([0.25, 0.45, 0.85]), np.array([0.85, 0.85, 0.8]), np.array([0.12, 0.14, 0.1])
    row = np.where(elev[:, None] >= 0, horizon * (1 - t) + zenith * t, ground)
    img = np.empty((height, width, 4), np.uint8)
    img[..., :3] = srgb_encode(row)[:, None, :]
    img[..., 3] = 255
    # sun disc
    u0, v0 = sun
    r_px = int(math.ceil(sun_radius * max(width, height))) + 1
    cx, cy = int(u0 * width), int(v0 * height)
    ys = np.arange(max(cy - r_px, 0), min(cy + r_px, height))
    xs = np.arange(max(cx - r_px, 0), min(cx + r_px, width))
    yy, xx = np.meshgrid(ys, xs, indexing="ij")
    inside = ((xx + 0.5) / width - u0) ** 2 * (width / height) ** 2 + ((yy + 0.5) / height - v0) ** 2 <= sun_radius**2
    patch = img[ys[0]:ys[-1] + 1, xs[0]:xs[-1] + 1]
    patch[inside, :3] = 255
    return img


def sky_gradient_env_map(width: int, height: int) -> np.ndarray:
    """RTIOW-style sky (white at the horizon/below, blue overhead), -Y up."""
    v = (np.arange(height, dtype=np.float64) + 0.5) / height
    y_up = np.sin((0.5 - v) * math.pi)
    t = (0.5 * (y_up + 1.0))[:, None]
    row = (1.0 - t) * np.array([1.0, 1.0, 1.0]) + t * np.array([0.5, 0.7, 1.0])
    img = np.empty((height, width, 4), np.uint8)
    img[..., :3] = srgb_encode(row)[:, None, :]
    img[..., 3] = 255
    return img


def scene_four_spheres(width=800, height=600) -> RenderScene:
    """Config C1: the 3 reference spheres + a ground sphere, materials 0-3."""
    spheres = np.stack([_sphere(p, r, m) for p, r, m in REFERENCE_SPHERES] +
                       [_sphere([0.0, 1000.5, 0.0], 1000.0, 1)]).astype(B.SPHERE)
    mats = np.stack([_material(*m) for m in REFERENCE_MATERIALS[:5]]).astype(B.MATERIAL)
    tex = np.stack([solid_color_image(c, (4, 4)) for c in REFERENCE_TEXTURE_COLORS[:4]] +
                   [solid_color_image([0.2, 0.4, 0.9], (4, 4))])
    env = solid_color_image([0.2, 0.2, 0.2], (64, 32))
    return RenderScene(spheres, mats, [], tex, env, Camera(width, height), name="four_spheres")


def scene_rtiow(width=1920, height=1080, seed=42) -> RenderScene:
    """Config C2: "Ray Tracing in One Weekend" cover scene, y flipped (the reference's up is -Y).

    Lambertian -> roughness 1, specular 0; metal -> specular 1, specular_scatter = fuzz;
    dielectric -> glass 1, ior 1.5, specular 1 (Schlick reflection). 256 palette
    colours as 1x1 texture layers (the reference's 256-layer limit)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    palette = np.zeros((256, 3))
    palette[0] = [0.5, 0.5, 0.5]
    palette[1] = [1.0, 1.0, 1.0]
    palette[2] = [0.4, 0.2, 0.1]
    palette[3] = [0.7, 0.6, 0.5]
    palette[4:130] = rng.random((126, 3)) * rng.random((126, 3))
    palette[130:256] = 0.5 + 0.5 * rng.random((126, 3))
    spheres, mats = [], []

    def add(pos, r, mat):
        spheres.append(_sphere(pos, r, len(mats)))
        mats.append(_material(*mat))

    add([0.0, 1000.0, 0.0], 1000.0, (0, 1.0, 0.0, 0.0, 1.0, 0.0, 1.0))
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rng.random()
            center = np.array([a + 0.9 * rng.random(), -0.2, b + 0.9 * rng.random()])
            if np.linalg.norm(center - np.array([4.0, -0.2, 0.0])) <= 0.9:
                continue
            if choose < 0.8:
                add(center, 0.2, (int(rng.integers(4, 130)), 1.0, 0.0, 0.0, 1.0, 0.0, 1.0))
            elif choose < 0.95:
                add(center, 0.2, (int(rng.integers(130, 256)), 1.0, 0.0, 1.0, float(0.5 * rng.random()), 0.0, 1.0))
            else:
                add(center, 0.2, (1, 0.0, 0.0, 1.0, 0.0, 1.0, 1.5))
    add([0.0, -1.0, 0.0], 1.0, (1, 0.0, 0.0, 1.0, 0.0, 1.0, 1.5))
    add([-4.0, -1.0, 0.0], 1.0, (2, 1.0, 0.0, 0.0, 1.0, 0.0, 1.0))
    add([4.0, -1.0, 0.0], 1.0, (3, 1.0, 0.0, 1.0, 0.0, 0.0, 1.0))
    tex = np.zeros((256, 1, 1, 4), np.uint8)
    tex[:, 0, 0, :3] = srgb_encode(palette)
    tex[..., 3] = 255
    pos = np.array([13.0, -2.0, 3.0], np.float32)
    cam = Camera(width, height, position=pos, direction=(-pos / np.linalg.norm(pos)).astype(np.float32),
                 vertical_fov=20.0)
    return RenderScene(np.stack(spheres).astype(B.SPHERE), np.stack(mats).astype(B.MATERIAL), [], tex,
                       sky_gradient_env_map(1024, 512), cam, name="rtiow")


def scene_chess(width=1920, height=1080, env_size=(8192, 4096), texture_size=(400, 400)) -> RenderScene:
    """Config C3: the reference's own scene, src/define_scene.rs (5,552 triangles,
    802 sub-objects, 34 objects, 3 spheres, 19 materials), with a procedural
    env map of the reference's size in place of the missing studio_garden.png."""
    assets = load_chess_assets()
    meshes = {k[4:]: v for k, v in assets.items() if k.startswith("stl_")}
    objs = chess_objects(meshes)
    tw, th = texture_size
    layers = []
    for c in REFERENCE_TEXTURE_COLORS:
        layers.append(None if c is None else solid_color_image(c, (tw, th)))
    images = [assets["tex_earth"], assets["tex_chess"]]
    for i, c in enumerate(REFERENCE_TEXTURE_COLORS):
        if c is None:
            img = images.pop(0)
            if img.shape[:2] != (th, tw):
                ys = np.arange(th) * img.shape[0] // th
                xs = np.arange(tw) * img.shape[1] // tw
                img = img[ys][:, xs]
            layers[i] = img
    tex = np.ascontiguousarray(np.stack(layers))
    spheres = np.stack([_sphere(p, r, m) for p, r, m in REFERENCE_SPHERES]).astype(B.SPHERE)
    mats = np.stack([_material(*m) for m in REFERENCE_MATERIALS]).astype(B.MATERIAL)
    env = procedural_env_map(*env_size)
    return RenderScene(spheres, mats, objs, tex, env, Camera(width, height), name="chess")


def scene_mixed(width=3840, height=2160, env_size=(8192, 4096)) -> RenderScene:
    """Config C4: the chess scene plus the RTIOW sphere field (<= 509 spheres),
    scaled down and placed around the board."""
    chess = scene_chess(width, height, env_size=env_size)
    rt = scene_rtiow(8, 8)
    base_mat = chess.materials.shape[0]
    base_tex = chess.textures.shape[0]
    extra = rt.spheres[1:507].copy()  # drop RTIOW's ground sphere: the chess floor is the ground
    extra["position"] = extra["position"] * np.float32(0.9) + np.array([0.0, -0.2, 0.0], np.float32)
    extra["material_index"] += base_mat - 1
    mats = rt.materials[1:507].copy()
    # remap palette textures onto 1-pixel-wide layers is impossible (one texture size);
    # give the field the chess scene's solid layers round-robin instead
    solid = [i for i, c in enumerate(REFERENCE_TEXTURE_COLORS) if c is not None]
    mats["texture_index"] = np.array(solid, np.uint32)[np.arange(mats.shape[0]) % len(solid)]
    spheres = np.concatenate([chess.spheres, extra]).astype(B.SPHERE)
    materials = np.concatenate([chess.materials, mats]).astype(B.MATERIAL)
    del base_tex
    return RenderScene(spheres, materials, chess.objects, chess.textures, chess.environment_map, chess.camera,
                       name="mixed")


def scene_heightfield(width=1920, height=1080, nx=1000, nz=500, seed=7) -> RenderScene:
    """Config C5: one object of 2*nx*nz triangles (1,000,000 by default), a
    random height field under the default camera, solid env map."""
    rng = np.random.Generator(np.random.PCG64(seed))
    xs = np.linspace(-20.0, 20.0, nx + 1, dtype=np.float32)
    zs = np.linspace(-20.0, 10.0, nz + 1, dtype=np.float32)
    hgt = (0.6 * rng.random((nz + 1, nx + 1)) + 0.5).astype(np.float32)
    X, Z = np.meshgrid(xs, zs)
    P = np.stack([X, hgt, Z], axis=-1).astype(np.float32)
    p00, p10, p01, p11 = P[:-1, :-1], P[:-1, 1:], P[1:, :-1], P[1:, 1:]
    a = np.concatenate([p00.reshape(-1, 3), p10.reshape(-1, 3)])
    b = np.concatenate([p10.reshape(-1, 3), p11.reshape(-1, 3)])
    c = np.concatenate([p01.reshape(-1, 3), p01.reshape(-1, 3)])
    tris = B.scene_triangles(a, b, c)
    info = np.zeros((), B.OBJECT_INFO)
    allp = P.reshape(-1, 3)
    mn, mx = bounding_box(allp)
    info["min_bounds"] = mn
    info["max_bounds"] = mx
    info["material_index"] = 0
    # editable like an STL object: its vertices are its "normalised points" at
    # scale 1, rotation 0, no translation (update_triangles reproduces them)
    obj = SceneObject(info, tris, normalized_points=np.stack([a, b, c], axis=1).reshape(-1, 3))
    obj.create_sub_objects(0, 0)
    mats = np.stack([_material(0, 0.9, 0.0, 0.1, 1.0, 0.0, 1.0), _material(1, 0.3, 0.0, 0.8, 0.05, 0.0, 1.0)])
    tex = np.stack([solid_color_image([0.3, 0.6, 0.3], (2, 2)), solid_color_image([0.9, 0.9, 0.9], (2, 2))])
    spheres = np.stack([_sphere([0.0, -1.0, 0.0], 1.0, 1)]).astype(B.SPHERE)
    return RenderScene(spheres, mats.astype(B.MATERIAL), [obj], tex, solid_color_image([0.6, 0.7, 0.9], (64, 32)),
                       Camera(width, height), name="heightfield")


# name -> (builder, bounces) ; SURVEY §8d
CONFIGS = {
    "c1_four_spheres": (scene_four_spheres, 4),
    "c2_rtiow": (scene_rtiow, 8),
    "c3_chess": (scene_chess, 8),
    "c4_mixed": (scene_mixed, 16),
    "c5_heightfield": (scene_heightfield, 8),
}


def build_config(name: str, width=None, height=None, **kw):
    """Return (scene, bounces) for a BASELINE.json configuration, optionally resized."""
    builder, bounces = CONFIGS[name]
    args = {}
    if width is not None:
        args["width"] = width
    if height is not None:
        args["height"] = height
    args.update(kw)
    return builder(**args), bounces
