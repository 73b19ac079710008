// scene_build.cpp — host restatement of src/triangle_object.rs.
//
// STL bytes -> SceneObject::new (rotate, normalise, scale, drop to the surface,
// translate) -> SceneTriangle::new -> 7-triangle sub-objects, and the edit path
// update_triangles / update_sub_objects. Every step is f32 in glam's operation
// order (compiled with -ffp-contract=off): Mat3A * Vec3A = (c0*x + c1*y) + c2*z,
// Vec3A::min/max = SSE minps/maxps (`x < y ? x : y`), length = sqrt of
// (x*x + y*y) + z*z, normalize = v * (1/length). The shared per-element pieces
// (placement of a point, SceneTriangle::new) live in rt_scene_math.h so the
// device rebuild (scene_edit.hip) runs the same arithmetic.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_scene_math.h"

void rt_set_global_error(const std::string& msg);

namespace {

int fail(int code, const std::string& msg) {
    rt_set_global_error(msg);
    return code;
}

bool is_binary_stl(const uint8_t* data, size_t size, uint32_t* n) {
    if (size < 84) return false;
    uint32_t count;
    std::memcpy(&count, data + 80, 4);
    if (84ull + 50ull * count != size) return false;
    *n = count;
    return true;
}

// ASCII STL: "facet ... outer loop / vertex x y z (x3) / endloop / endfacet".
int parse_ascii(const uint8_t* data, size_t size, float* out, uint32_t capacity, uint32_t* count) {
    std::string text(reinterpret_cast<const char*>(data), size);
    size_t pos = 0;
    uint32_t verts = 0;
    while ((pos = text.find("vertex", pos)) != std::string::npos) {
        pos += 6;
        const char* p = text.c_str() + pos;
        char* end = nullptr;
        float v[3];
        for (int k = 0; k < 3; k++) {
            v[k] = std::strtof(p, &end);
            if (end == p) return fail(RT_E_INVALID, "malformed ASCII STL vertex");
            p = end;
        }
        pos = (size_t)(p - text.c_str());
        if (out) {
            if (verts / 3 >= capacity) return fail(RT_E_CAPACITY, "STL has more facets than capacity");
            std::memcpy(out + 3 * verts, v, sizeof(v));
        }
        verts++;
    }
    if (verts % 3) return fail(RT_E_INVALID, "ASCII STL vertex count is not a multiple of 3");
    *count = verts / 3;
    return RT_OK;
}

using namespace rt_scene;

// get_bounding_box (src/triangle_object.rs:292-321), one sequential scan.
void bounding_box(const float* pts, size_t n, float mn[3], float mx[3]) {
    BoxScan b;
    for (size_t i = 0; i < n; i++) b.add(pts + 3 * i);
    b.get(mn, mx);
}

void write_triangle(const float* a, const float* b, const float* c, rt_scene_triangle* t) {
    TriangleRecord r;
    scene_triangle(a, b, c, r);
    std::memset(t, 0, sizeof(*t));
    std::memcpy(t->a, a, 12);
    std::memcpy(t->edge_ab, r.ab, 12);
    std::memcpy(t->edge_ac, r.ac, 12);
    std::memcpy(t->calc_normal, r.calc_normal, 12);
    std::memcpy(t->face_normal, r.face_normal, 12);
    std::memcpy(t->min_bounds, r.mn, 12);
    std::memcpy(t->max_bounds, r.mx, 12);
}

// Bounds of one chunk of triangles: the reference scans [min0, max0, min1, max1, ...] (:171-176).
void chunk_bounds(const rt_scene_triangle* t, uint32_t n, float mn[3], float mx[3]) {
    BoxScan b;
    for (uint32_t i = 0; i < n; i++) {
        b.add(t[i].min_bounds);
        b.add(t[i].max_bounds);
    }
    b.get(mn, mx);
}

}  // namespace

extern "C" {

int rt_stl_triangle_count(const uint8_t* data, size_t size, uint32_t* count) {
    if (!data || !count) return fail(RT_E_INVALID, "data/count is NULL");
    if (is_binary_stl(data, size, count)) return RT_OK;
    if (size >= 5 && std::memcmp(data, "solid", 5) == 0) return parse_ascii(data, size, nullptr, 0, count);
    return fail(RT_E_INVALID, "not an STL file (binary size mismatch and no 'solid' header)");
}

int rt_stl_read(const uint8_t* data, size_t size, float* vertices, uint32_t capacity) {
    if (!data || !vertices) return fail(RT_E_INVALID, "data/vertices is NULL");
    uint32_t n = 0;
    if (is_binary_stl(data, size, &n)) {
        if (n > capacity) return fail(RT_E_CAPACITY, "STL has more facets than capacity");
        for (uint32_t i = 0; i < n; i++)  // 50-byte facet: normal (ignored), 3 vertices, attribute
            std::memcpy(vertices + 9 * (size_t)i, data + 84 + 50 * (size_t)i + 12, 36);
        return RT_OK;
    }
    if (size >= 5 && std::memcmp(data, "solid", 5) == 0) return parse_ascii(data, size, vertices, capacity, &n);
    return fail(RT_E_INVALID, "not an STL file (binary size mismatch and no 'solid' header)");
}

int rt_scene_object_new(const float* stl_vertices, uint32_t triangle_count, float scale, const float coordinates[3],
                        const float rotation[3], uint32_t material_index, float* normalized_points,
                        rt_scene_triangle* triangles, rt_object_info* info, rt_object_transform* state) {
    if (!stl_vertices || !coordinates || !rotation || !normalized_points || !triangles || !info || !state)
        return fail(RT_E_INVALID, "NULL argument");
    if (!(scale > 0.0f)) return fail(RT_E_INVALID, "scale has to be over 0.0");  // :67
    const size_t n = 3 * (size_t)triangle_count;
    std::vector<float> pts(stl_vertices, stl_vertices + 3 * n);
    // normalize_model (:237-251)
    float rot[9];
    rotation_matrix(rotation, rot);
    for (size_t i = 0; i < n; i++) mat3_mul(rot, &pts[3 * i], &pts[3 * i]);
    float mn[3], mx[3];
    bounding_box(pts.data(), n, mn, mx);
    float average[3], d[3];
    for (int k = 0; k < 3; k++) {
        average[k] = (mn[k] + mx[k]) / 2.0f;
        d[k] = mn[k] - mx[k];
    }
    const float s = 1.0f / std::sqrt(dot3(d, d));  // 1 / min.distance(max)
    float shift[3];
    for (int k = 0; k < 3; k++) shift[k] = average[k] * s;
    for (size_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) pts[3 * i + k] = pts[3 * i + k] * s - shift[k];
    // scale_model (:278-283)
    for (size_t i = 0; i < 3 * n; i++) pts[i] = pts[i] * scale;
    std::memcpy(normalized_points, pts.data(), 3 * n * sizeof(float));
    bounding_box(pts.data(), n, mn, mx);
    // transform_points_to_surface (:323-331): -max * Vec3A::Y, then + coordinates
    const float surface[3] = {-mx[0] * 0.0f, -mx[1] * 1.0f, -mx[2] * 0.0f};
    float total[3];
    for (int k = 0; k < 3; k++) total[k] = coordinates[k] + surface[k];
    for (size_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) pts[3 * i + k] = (pts[3 * i + k] + surface[k]) + coordinates[k];
    std::memset(info, 0, sizeof(*info));
    for (int k = 0; k < 3; k++) {
        const float shift_k = surface[k] + coordinates[k];
        info->min_bounds[k] = mn[k] + shift_k;
        info->max_bounds[k] = mx[k] + shift_k;
    }
    info->material_index = material_index;
    for (uint32_t t = 0; t < triangle_count; t++)
        write_triangle(&pts[9 * (size_t)t], &pts[9 * (size_t)t + 3], &pts[9 * (size_t)t + 6], &triangles[t]);
    // the object keeps scale 1, rotation 0 and the total translation (:114-126)
    std::memset(state, 0, sizeof(*state));
    state->scale = 1.0f;
    std::memcpy(state->transformation, total, sizeof(total));
    return RT_OK;
}

int rt_scene_object_create_sub_objects(const rt_scene_triangle* triangles, uint32_t triangle_count,
                                       uint32_t first_sub_object_index, uint32_t first_triangle_index,
                                       rt_object_info* info, rt_sub_object_info* sub_objects) {
    if ((!triangles && triangle_count) || !info || (!sub_objects && triangle_count))
        return fail(RT_E_INVALID, "NULL argument");
    const uint32_t n_sub = (triangle_count + kSubObjectTriangles - 1) / kSubObjectTriangles;
    for (uint32_t k = 0; k < n_sub; k++) {
        const uint32_t first = k * kSubObjectTriangles;
        const uint32_t cnt = std::min(kSubObjectTriangles, triangle_count - first);
        rt_sub_object_info& so = sub_objects[k];
        chunk_bounds(triangles + first, cnt, so.min_bounds, so.max_bounds);
        so.first_triangle_index = first_triangle_index + first;
        so.triangle_count = cnt;
    }
    info->first_sub_object_index = first_sub_object_index;
    info->sub_object_count = n_sub;
    return RT_OK;
}

int rt_scene_object_update(const float* normalized_points, uint32_t triangle_count, const rt_object_transform* state,
                           rt_object_info* info, rt_scene_triangle* triangles, rt_sub_object_info* sub_objects) {
    if ((!normalized_points && triangle_count) || !state || !info || (!triangles && triangle_count))
        return fail(RT_E_INVALID, "NULL argument");
    if (info->sub_object_count && !sub_objects) return fail(RT_E_INVALID, "sub_objects is NULL");
    if (info->sub_object_count != (triangle_count + kSubObjectTriangles - 1) / kSubObjectTriangles)
        return fail(RT_E_INVALID, "sub_object_count must be ceil(triangle_count / 7)");
    const size_t n = 3 * (size_t)triangle_count;
    Placement pl;
    placement(*reinterpret_cast<const ObjectTransform*>(state), pl);
    std::vector<float> pts(3 * n);
    for (size_t i = 0; i < n; i++) place_point(pl, normalized_points + 3 * i, &pts[3 * i]);  // :130-134
    bounding_box(pts.data(), n, info->min_bounds, info->max_bounds);                          // :136-141
    for (uint32_t t = 0; t < triangle_count; t++)                                              // :143-147
        write_triangle(&pts[9 * (size_t)t], &pts[9 * (size_t)t + 3], &pts[9 * (size_t)t + 6], &triangles[t]);
    for (uint32_t k = 0; k < info->sub_object_count; k++) {                                    // :199-220
        const uint32_t first = k * kSubObjectTriangles;
        const uint32_t cnt = std::min(kSubObjectTriangles, triangle_count - first);
        chunk_bounds(triangles + first, cnt, sub_objects[k].min_bounds, sub_objects[k].max_bounds);
    }
    return RT_OK;
}

}  // extern "C"
