// rt_scene_math.h — per-element f32 arithmetic of src/triangle_object.rs and
// SceneTriangle::new (src/buffers.rs:66-95), shared by the host builder
// (scene_build.cpp) and the device edit kernels (scene_edit.hip) so that both
// produce the same bits. glam's operation order throughout; compile with
// -ffp-contract=off (and correctly rounded device division/sqrt).
#pragma once
#include <stdint.h>

#include <cmath>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_SCENE_FN __host__ __device__ inline
#else
#define RT_SCENE_FN inline
#endif

namespace rt_scene {

constexpr uint32_t kSubObjectTriangles = 7;  // n_sub_object_triangels, src/triangle_object.rs:125
constexpr float kF32Max = 3.4028235e+38f;

// rt_object_transform (include/rt_abi.h), the edit state of one object.
struct ObjectTransform {
    float rotation[3];
    float scale;
    float transformation[3];
    uint32_t _padding;
};

// What update_triangles applies to each point (:129-134): Rz*Ry*Rx (columns), scale, translation.
struct Placement {
    float rot[9];
    float scale;
    float trans[3];
};

RT_SCENE_FN float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

// glam Mat3A * Vec3A: (c0*x + c1*y) + c2*z, m = 3 columns. `out` may alias `v`.
RT_SCENE_FN void mat3_mul(const float* m, const float* v, float* out) {
    const float x = v[0], y = v[1], z = v[2];
    for (int k = 0; k < 3; k++) out[k] = (m[k] * x + m[3 + k] * y) + m[6 + k] * z;
}

// rotate_to_angle's matrix (:253-269): deg * (PI / 180) in f32, sin/cos of the
// f32 angle rounded from double (glam calls f32 sin/cos; parity unpinned at the
// last bit against the reference's libm), Rz * Ry * Rx.
inline void rotation_matrix(const float* deg, float* out) {
    const float k = 3.14159265358979323846f / 180.0f;
    float s[3], c[3];
    for (int i = 0; i < 3; i++) {
        const float r = deg[i] * k;
        s[i] = (float)std::sin((double)r);
        c[i] = (float)std::cos((double)r);
    }
    const float mx[9] = {1, 0, 0, 0, c[0], s[0], 0, -s[0], c[0]};
    const float my[9] = {c[1], 0, -s[1], 0, 1, 0, s[1], 0, c[1]};
    const float mz[9] = {c[2], s[2], 0, -s[2], c[2], 0, 0, 0, 1};
    float zy[9];
    for (int col = 0; col < 3; col++) mat3_mul(mz, my + 3 * col, zy + 3 * col);
    for (int col = 0; col < 3; col++) mat3_mul(zy, mx + 3 * col, out + 3 * col);
}

inline void placement(const ObjectTransform& t, Placement& p) {
    rotation_matrix(t.rotation, p.rot);
    p.scale = t.scale;
    for (int k = 0; k < 3; k++) p.trans[k] = t.transformation[k];
}

// update_triangles per point (:130-134): rotate, scale_model, transform_model.
RT_SCENE_FN void place_point(const Placement& p, const float* in, float* out) {
    float r[3];
    mat3_mul(p.rot, in, r);
    for (int k = 0; k < 3; k++) out[k] = r[k] * p.scale;
    for (int k = 0; k < 3; k++) out[k] = out[k] + p.trans[k];
}

// get_bounding_box (:292-321): start at +-f32::MAX, replace on a strict < / >.
struct BoxScan {
    float mn[3] = {kF32Max, kF32Max, kF32Max};
    float mx[3] = {-kF32Max, -kF32Max, -kF32Max};
    RT_SCENE_FN void add(const float* p) {
        for (int k = 0; k < 3; k++) {
            if (p[k] < mn[k]) mn[k] = p[k];
            if (p[k] > mx[k]) mx[k] = p[k];
        }
    }
    RT_SCENE_FN void get(float* lo, float* hi) const {
        for (int k = 0; k < 3; k++) {
            lo[k] = mn[k];
            hi[k] = mx[k];
        }
    }
};

// SceneTriangle::new (src/buffers.rs:66-95).
struct TriangleRecord {
    float ab[3], ac[3], calc_normal[3], face_normal[3], mn[3], mx[3];
};

RT_SCENE_FN float vmin(float x, float y) { return x < y ? x : y; }  // SSE minps
RT_SCENE_FN float vmax(float x, float y) { return x > y ? x : y; }  // SSE maxps

RT_SCENE_FN void scene_triangle(const float* a, const float* b, const float* c, TriangleRecord& r) {
    for (int k = 0; k < 3; k++) {
        r.ab[k] = b[k] - a[k];
        r.ac[k] = c[k] - a[k];
    }
    r.calc_normal[0] = r.ab[1] * r.ac[2] - r.ab[2] * r.ac[1];
    r.calc_normal[1] = r.ab[2] * r.ac[0] - r.ab[0] * r.ac[2];
    r.calc_normal[2] = r.ab[0] * r.ac[1] - r.ab[1] * r.ac[0];
    const float inv = 1.0f / std::sqrt(dot3(r.calc_normal, r.calc_normal));
    for (int k = 0; k < 3; k++) {
        r.face_normal[k] = r.calc_normal[k] * inv;
        r.mn[k] = vmin(vmin(a[k], b[k]), c[k]);
        r.mx[k] = vmax(vmax(a[k], b[k]), c[k]);
    }
}

}  // namespace rt_scene
