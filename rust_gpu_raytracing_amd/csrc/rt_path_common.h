// rt_path_common.h -- the device side of one path segment, shared by the path-tracing kernels
// (pathtrace.hip: the persistent walk, the primary pre-pass, the brute-force wavefront): the
// reference's sphere and triangle tests, its sweep,
// trace_ray's result, the shading of the bounce loop, sampling, packing. Every function follows
// compute_shader.wgsl decision for decision (line numbers in each); the numeric contract is in
// rt_device_math.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_bvh_slab.h"
#include "rt_device_math.h"
#include "rt_kernel_args.h"
#include "tri_qnode.h"

#pragma clang fp contract(off)

using namespace rtk;

namespace {

struct Hit {
    float t;
    f3 p;
    f3 n;
    uint32_t material_index;
    bool front_face;
    float u, v;
};

struct SceneView {
    const float4* sph;        // per slot: centre.xyz, radius^2 (brute-force set, then BVH leaf order)
    const uint32_t* orig;     // per slot: original sphere index
    const uint32_t* sph_mat;  // per original index: material index
    const float4* nodes;      // sphere BVH, 2 float4 per node (sphere_bvh.h)
    const RtMaterial* mat;    // LDS
    const float4* mat_aux;    // LDS (modes 1, 2): per material {1/ior, r0 front, r0 back, roughness/10}, 1x1 texel
    const RtObject* obj;      // LDS
    const float* srgb;        // LDS, 256 entries
    const float4* tri_nodes;  // triangle accelerator nodes (LDS in mode 2, else global)
    const uint4* tri_prims;   // triangle accelerator leaves: object, sub-object, sweep position
    float tri_extent;         // triangle margin scale (device memory: a device refit updates it)
    const RtSubObject* sub;   // sub-object records (LDS in mode 2 when they fit, else global)
    // the quantized triangle nodes (modes 0/1; null: the 32-B nodes) and their grid
    const uint4* tri_q;
    float qox, qoy, qoz, qsx, qsy, qsz;
};

__device__ __forceinline__ f3 ld3(const float4& v) { return mk(v.x, v.y, v.z); }

__device__ __forceinline__ int texel_coord(float c, uint32_t size) {
    // Truncate toward zero, then clamp to [0, size-1]; NaN -> 0 (naga Restrict).
    if (!(c >= 0.0f)) return 0;
    if (c >= (float)size) return (int)size - 1;
    const int i = (int)c;
    return i > (int)size - 1 ? (int)size - 1 : i;
}

__device__ __forceinline__ f4 decode_texel(uint32_t texel, const float* srgb) {
    return f4{srgb[texel & 0xffu], srgb[(texel >> 8) & 0xffu], srgb[(texel >> 16) & 0xffu],
              div_const((float)(texel >> 24), 255.0f, kInv255)};
}

// check_spheres, compute_shader.wgsl:355-404.
//
// The reference sweeps spheres in index order keeping the first of equal
// distances (strict `<`, :391), i.e. it returns the lexicographic minimum of
// (t, index) over spheres with disc >= 0 and t > 0. Here spheres are visited
// in slot order (brute-force set, then BVH leaves), so acceptance compares
// (t, original index) lexicographically, which yields the same sphere in any
// visiting order. `orig` starts at 0 so that t == F32_MAX is never taken.
struct SphereHit {
    float t;
    uint32_t orig;
    uint32_t slot;
};

__device__ __forceinline__ void sphere_candidate(float disc, float b, float two_a, uint32_t orig, uint32_t slot,
                                                 SphereHit& best) {
    if (disc >= 0.0f) {
        const float t = (-b - sqrt_rn_any(disc)) / two_a;
        if (t > 0.0f && (t < best.t || (t == best.t && orig < best.orig))) {
            best.t = t;
            best.orig = orig;
            best.slot = slot;
        }
    }
}

// The reference's per-sphere arithmetic (:372-379), unchanged.
__device__ __forceinline__ float sphere_disc(const float4 s, f3 o, f3 d, float four_a, float& b) {
    const f3 oc = o - ld3(s);
    b = 2.0f * dot(d, oc);
    const float c = dot(oc, oc) - s.w;
    return b * b - four_a * c;
}

// Tests the aligned group of 4 slots starting at `slot` (sphere_bvh.h: padded
// with NaN spheres that no ray hits). All loads are issued together and the
// four tests are independent, so the group costs one LDS round trip.
__device__ __forceinline__ void test_sphere_group(const SceneView& sv, uint32_t slot, f3 o, f3 d, float four_a,
                                                  float two_a, SphereHit& best) {
    const float4 s0 = sv.sph[slot], s1 = sv.sph[slot + 1u], s2 = sv.sph[slot + 2u], s3 = sv.sph[slot + 3u];
    const uint4 og = *reinterpret_cast<const uint4*>(sv.orig + slot);
    float b[4], disc[4];
    disc[0] = sphere_disc(s0, o, d, four_a, b[0]);
    disc[1] = sphere_disc(s1, o, d, four_a, b[1]);
    disc[2] = sphere_disc(s2, o, d, four_a, b[2]);
    disc[3] = sphere_disc(s3, o, d, four_a, b[3]);
    // any(disc[k] >= 0): max of the four (NaN operands ignored, as `NaN >= 0` is false)
    if (fmax_nn(fmax_nn(disc[0], disc[1]), fmax_nn(disc[2], disc[3])) >= 0.0f) {
        sphere_candidate(disc[0], b[0], two_a, og.x, slot, best);
        sphere_candidate(disc[1], b[1], two_a, og.y, slot + 1u, best);
        sphere_candidate(disc[2], b[2], two_a, og.z, slot + 2u, best);
        sphere_candidate(disc[3], b[3], two_a, og.w, slot + 3u, best);
    }
}

// Sphere side: lateral box inflation and depth slack from sphere_cull_bounds
// (rt_bvh_slab.h). Triangle side: covers the f32 rounding of the reference's slab test.
constexpr float kTriMarginScale = 1.0e-5f;

// ray_in_bounds, compute_shader.wgsl:407-419.
__device__ __forceinline__ bool ray_in_bounds(f3 o, f3 inv, const float* mn, const float* mx) {
    const float tminx = (mn[0] - o.x) * inv.x, tmaxx = (mx[0] - o.x) * inv.x;
    const float tminy = (mn[1] - o.y) * inv.y, tmaxy = (mx[1] - o.y) * inv.y;
    const float tminz = (mn[2] - o.z) * inv.z, tmaxz = (mx[2] - o.z) * inv.z;
    const float near_t = fmax_nn(fmax_nn(fmin_nn(tminx, tmaxx), fmin_nn(tminy, tmaxy)), fmin_nn(tminz, tmaxz));
    const float far_t = fmin_nn(fmin_nn(fmax_nn(tminx, tmaxx), fmax_nn(tminy, tmaxy)), fmax_nn(tminz, tmaxz));
    return near_t <= far_t && far_t >= 0.0f;
}

// ray_in_bounds on a 32-B record read as two float4 ({min, first}, {max, count}): the same
// operations (scalar f32: gfx950 issues v_pk_*_f32 at a third of the scalar rate, build.py).
__device__ __forceinline__ bool ray_in_box4(f3 o, f3 inv, float4 lo, float4 hi) {
    const float mn[3] = {lo.x, lo.y, lo.z}, mx[3] = {hi.x, hi.y, hi.z};
    return ray_in_bounds(o, inv, mn, mx);
}

// Closest triangle found so far: distance, position in the reference's sweep
// order (tie-break), triangle and object index, facing.
struct TriHit {
    float t;
    uint32_t seq, tri, obj;
    bool front;
};

// The four vectors of a triangle the intersection test reads (the first 48 B
// of its record; face_normal is read only for the closest hit).
struct TriGeom {
    f3 a, ab, ac, cn;
};
__device__ __forceinline__ TriGeom load_tri(const RtTriangleHot* __restrict__ t, uint32_t i) {
    const float4 p0 = t[i].p0, p1 = t[i].p1, p2 = t[i].p2;
    return TriGeom{mk(p0.x, p0.y, p0.z), mk(p0.w, p1.x, p1.y), mk(p1.z, p1.w, p2.x), mk(p2.y, p2.z, p2.w)};
}

// Leaf certificates (certified pruning) are read by the walks from global memory
// only: node_step records the gap of a leaf box entered beyond the best hit, and the leaf batch
// tests the leaf's certificate with it (C5 11.08 -> 10.81 ms per frame against testing in
// node_step, profiles/r04/r04_k). The LDS-resident walk (mode 2) culls by box alone, exact
// without any bound: the certificate code cost its instances more registers than the triangle
// tests it skipped (C3 0.304 -> 0.335 ms per frame compiled in and off).

// check_triangles, compute_shader.wgsl:422-517: the reference's own sweep over
// objects -> sub-objects -> triangles (first wins on equal distance, `>=`
// rejects, :457). Used when the accelerator is off, and as the fallback for
// the measure-zero NaN-distance case.
__device__ __forceinline__ TriHit sweep_triangles(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d) {
    TriHit th{kF32Max, 0u, 0u, 0u, false};
    float closest = kF32Max;
    const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const uint32_t n_obj = ka.object_count;
    for (uint32_t oi = 0; oi < n_obj; ++oi) {
        const RtObject& ob = sv.obj[oi];
        if (!ray_in_bounds(o, inv, ob.min_bounds, ob.max_bounds)) continue;
        const uint32_t first_sub = ob.first_sub_object_index;
        const uint32_t n_sub = ob.sub_object_count;
        for (uint32_t i = 0; i < n_sub; ++i) {
            const uint32_t si = min(first_sub + i, ka.sub_object_count - 1u);
            const RtSubObject sub = sv.sub[si];
            if (!ray_in_bounds(o, inv, sub.min_bounds, sub.max_bounds)) continue;
            for (uint32_t j = 0; j < sub.triangle_count; ++j) {
                const uint32_t ti = min(sub.first_triangle_index + j, ka.triangle_count - 1u);
                const TriGeom g = load_tri(ka.triangles, ti);
                const float det = -dot(d, g.cn);
                const float inv_det = 1.0f / det;
                const f3 ao = o - g.a;
                const float dist = dot(ao, g.cn) * inv_det;
                if (dist < 0.0f || dist >= closest) continue;
                const f3 dao = cross(ao, d);
                const float v = -dot(g.ab, dao) * inv_det;
                if (v < 0.0f) continue;
                const float u = dot(g.ac, dao) * inv_det;
                if (u < 0.0f) continue;
                const float w = 1.0f - u - v;
                if (w < 0.0f) continue;
                closest = dist;
                th.t = dist;
                th.tri = ti;
                th.obj = oi;
                th.front = det > 0.0f;
            }
        }
    }
    return th;
}

// One ray's closest-hit search, resumable one BVH node at a time so that a
// wave can interleave it with other lanes' shading (see the kernel).
//
// Phase 0 walks the triangle accelerator: a BVH over the
// (object, sub-object) pairs of the reference's sweep; each reached pair runs
// the reference's own object and sub-object ray_in_bounds tests and triangle
// tests, and the winner is the lexicographic minimum of (distance, sweep
// position) — the sweep's first-wins result. A NaN distance (ray lying
// exactly in a triangle's plane) makes the sweep accept later candidates
// unconditionally (:457); if one is met, the lane reruns the sweep itself.
// Phase 1 walks the sphere BVH, pruned by the best sphere and
// the triangle hit (a sphere wins only when strictly closer, :347).
// Phase 2: done.
constexpr uint32_t kNoLeaf = 0xffffffffu;

struct TraceState {
    f3 inv;
    float a4, a2;     // 4*dot(d,d), 2*dot(d,d) (:372-379)
    SlabRay slab;     // the current phase's BVH slab constants (margin folded in, rt_bvh_slab.h)
    float slack;      // depth slack of the sphere walk (0 on the triangle walk)
    float limit;      // pruning distance: min(best sphere, triangle hit) * 1.00001 + slack (inf: none)
    uint32_t node;
    uint32_t phase;
    uint32_t pending;  // postponed leaf (sphere group slot / triangle prim), or kNoLeaf
    float cert_gap;    // deferred leaf certificate test (pending bit 24): the leaf box's gap beyond the best hit
    bool nan_hit;
    SphereHit sph;
    TriHit tri;
};

// A sphere must be strictly closer than the best sphere so far and than the
// triangle hit to win (:347, :391); boxes entered beyond that (with slack for
// the float near root's deviation, ts.slack) cannot hold the winner. Updated
// when either changes.
__device__ __forceinline__ float prune_limit(const TraceState& ts) {
    return fmin_nn(ts.sph.t, ts.tri.t) * 1.00001f + ts.slack;
}

// The round-3 relative-slack pruning (ka.tri_prune_mode 2, opt-in; ka.tri_prune = rho, else 0):
// once a triangle is hit at t, a box whose inflated entry lies beyond t * (1 + rho) + 2^-10
// (|o| + extent) / |d| is skipped. The slack covers the f32 error of the reference's distance
// and barycentrics only for triangles well away from parallel to the ray (that error grows
// as 1/cos): NOT exact -- rays nearly in a triangle's plane close to their origin can lose the
// sweep's winner (tests/test_tri_accel_cpu.py). The default is the certified test below.
constexpr float kTriPruneAbs = 0x1p-10f;
__device__ __forceinline__ float tri_limit(const SceneView& sv, const KernelArgs& ka, f3 o, const TraceState& ts) {
    if (ka.tri_prune == 0.0f || ts.tri.t == kF32Max) return __builtin_inff();
    const float r = sqrt_up(dot(o, o));
    const float sig = kTriPruneAbs * (r + sv.tri_extent) * (__builtin_amdgcn_rsqf(ts.a2 * 0.5f) * 1.001f);
    return ts.tri.t * (1.0f + ka.tri_prune) + sig;
}

// Certified distance pruning (ka.tri_prune_mode 1; tri_cone.h): when the walk
// reaches a leaf whose box it enters beyond the best hit tb, the leaf's certificate proves, per
// triangle, that the reference's test (:449-481) cannot accept it at a distance <= tb; those
// triangles are skipped without being loaded, and the whole leaf when all are. Returns the mask
// of skipped triangles (kLeafCertAll: the leaf). The per-axis entries are the culling slab
// test's own (rt_bvh_slab.h) on the box as the walk decoded it. (The path kernel's walk defers
// this test to its leaf batch, tri_leafcert_skips_gap; the primary pre-pass tests on the spot.)
__device__ __forceinline__ uint32_t tri_leaf_skips(const KernelArgs& ka, uint32_t prim, const SlabRay& sr, f3 o, f3 d,
                                                   float tb, float4 lo, float4 hi) {
    const uint4* rec = reinterpret_cast<const uint4*>(ka.tri_leafcert + prim);
    const uint4 c0 = rec[0], c1 = rec[1];
    const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float t1x = fminf(fmaf(lo.x, sr.ix, sr.lx), fmaf(hi.x, sr.ix, sr.hx));
    const float t1y = fminf(fmaf(lo.y, sr.iy, sr.ly), fmaf(hi.y, sr.iy, sr.hy));
    const float t1z = fminf(fmaf(lo.z, sr.iz, sr.lz), fmaf(hi.z, sr.iz, sr.hz));
    return tri_leafcert_skips(w, tri_cone_ray(o.x, o.y, o.z, d.x, d.y, d.z), tb, t1x, t1y, t1z, fabsf(sr.ix),
                              fabsf(sr.iy), fabsf(sr.iz));
}

// The triangle leaf: the reference's object and sub-object ray_in_bounds tests
// and triangle tests for one (object, sub-object) pair (compute_shader.wgsl:431-500).
// kLazySub (the accelerator in global memory): with the sub-object's triangle range in the
// leaf record, the triangle loads start without the sub-object record, which is loaded and
// its ray_in_bounds test run only for the first candidate that would change the lane's result
// (a new best hit or a NaN distance); if that test fails, no triangle of the leaf counts --
// exactly as the reference, which tests none of them then. Most leaves change nothing, so
// their sub-object record is never read.

// `pending`: the leaf record's index, with the mask of triangles its certificate skips in
// bits 24-30 (tri_leaf_skips; they are not loaded).
template <bool kLazySub = false>
__device__ __forceinline__ void tri_leaf(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts,
                                         uint32_t pending) {
    const uint32_t prim = pending & 0xffffffu;
    uint32_t skip = 0u;
    if ((pending >> 24) & 1u) {  // the certificate test deferred by node_step
        const uint4* rec = reinterpret_cast<const uint4*>(ka.tri_leafcert + prim);
        const uint4 c0 = rec[0], c1 = rec[1];
        const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        skip = tri_leafcert_skips_gap(w, tri_cone_ray(o.x, o.y, o.z, d.x, d.y, d.z), ts.tri.t, ts.cert_gap);
        if (skip == kLeafCertAll) return;
    }
    const uint4 pr = sv.tri_prims[prim];  // object, sub, seq_base, range
    const RtObject& ob = sv.obj[pr.x];
    if (!ray_in_bounds(o, ts.inv, ob.min_bounds, ob.max_bounds)) return;
    uint32_t first, count;
    int sub_state;  // 1: passed, 0: not tested yet
    if (kLazySub && pr.w != 0xffffffffu) {  // kPrimRangeNone (sphere_bvh.h)
        first = pr.w & ((1u << 27) - 1u);
        count = pr.w >> 27;
        sub_state = 0;
    } else {
        const RtSubObject sub = sv.sub[pr.y];
        if (!ray_in_bounds(o, ts.inv, sub.min_bounds, sub.max_bounds)) return;
        first = sub.first_triangle_index;
        count = sub.triangle_count;
        sub_state = 1;
    }
    for (uint32_t j = 0; j < count; ++j) {
        if ((skip >> j) & 1u) continue;
        const uint32_t ti = min(first + j, ka.triangle_count - 1u);
        const uint32_t seq = pr.z + j;
        const TriGeom g = load_tri(ka.triangles, ti);
        const float det = -dot(d, g.cn);
        const float inv_det = 1.0f / det;
        const f3 ao = o - g.a;
        const float dist = dot(ao, g.cn) * inv_det;
        const bool nan_dist = dist != dist;
        if (dist < 0.0f) continue;
        if (!nan_dist && !(dist < ts.tri.t || (dist == ts.tri.t && seq < ts.tri.seq))) continue;
        const f3 dao = cross(ao, d);
        const float v = -dot(g.ab, dao) * inv_det;
        if (v < 0.0f) continue;
        const float u = dot(g.ac, dao) * inv_det;
        if (u < 0.0f) continue;
        const float w = 1.0f - u - v;
        if (w < 0.0f) continue;
        if (kLazySub && sub_state == 0) {
            const RtSubObject sub = sv.sub[pr.y];
            if (!ray_in_bounds(o, ts.inv, sub.min_bounds, sub.max_bounds)) return;
            sub_state = 1;
        }
        if (nan_dist) {
            ts.nan_hit = true;
            continue;
        }
        ts.tri = TriHit{dist, seq, ti, pr.x, det > 0.0f};
    }
}

// trace_ray's result (:342-353): the sphere wins only if strictly closer.
template <bool kTris>
__device__ __forceinline__ Hit trace_end(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, const TraceState& ts) {
    Hit h;
    h.t = kF32Max;
    h.p = mk(0.f, 0.f, 0.f);
    h.n = mk(0.f, 0.f, 0.f);
    h.material_index = 0;
    h.front_face = false;
    h.u = 0.f;
    h.v = 0.f;
    if (kTris && ts.tri.t != kF32Max) {  // found (the sweep can accept a NaN distance, :457)
        const RtObject& ob = sv.obj[ts.tri.obj];
        const f3 fn = ld3(ka.triangles[ts.tri.tri].fn);
        h.front_face = ts.tri.front;
        h.n = ts.tri.front ? fn : -fn;
        h.t = ts.tri.t;
        h.p = o + d * ts.tri.t;
        // object_texture_coords, :568-578 (uv from the OBJECT bounds); unused
        // with 1x1 texture layers, as for spheres below
        if (ka.tex_w != 1u || ka.tex_h != 1u) {
            h.u = (h.p.x - ob.min_bounds[0]) / (ob.max_bounds[0] - ob.min_bounds[0]);
            h.v = (h.p.z - ob.min_bounds[2]) / (ob.max_bounds[2] - ob.min_bounds[2]);
        }
        h.material_index = ob.material_index;
    }
    if (ts.sph.t < h.t) {  // no sphere -> F32_MAX
        // sphere_hit, :530-555, and sphere_texture_coords, :557-566
        const float4 s = sv.sph[ts.sph.slot];
        const float t = ts.sph.t;
        const f3 p = o + d * t;
        const f3 outward = normalize(p - ld3(s));
        h.t = t;
        h.p = p;
        // uv feeds only the texel fetch, and with 1x1 texture layers every uv
        // maps to texel (0, 0) (texel_coord clamps to [0, size-1]): the
        // acos/atan2 are then skipped (bit-identical; 4% of a C2 frame)
        if (ka.tex_w != 1u || ka.tex_h != 1u) {
            const float theta = acosf_c(-outward.y);
            const float phi = atan2f_c(-outward.z, outward.x) + kWgslPi;
            h.u = div_const(phi, kTwoPiWgsl, kInvTwoPiWgsl);  // exact: rt_math_selftest
            h.v = div_const(theta, kWgslPi, kInvWgslPi);
        }
        h.front_face = dot(d, outward) < 0.0f;
        h.n = h.front_face ? outward : -outward;
        h.material_index = sv.sph_mat[ts.sph.orig];
    }
    return h;
}

// sample_texture, compute_shader.wgsl:26-32: the raw RGBA8 texel (decoded later).
__device__ __forceinline__ uint32_t fetch_texture(const KernelArgs& ka, uint32_t layer, float u, float v) {
    const int x = texel_coord(u * (float)(int32_t)ka.texture_width, ka.tex_w);
    const int y = texel_coord(v * (float)(int32_t)ka.texture_height, ka.tex_h);
    const uint32_t l = min(layer, ka.tex_layers - 1u);
    const size_t off = ((size_t)l * ka.tex_h + (size_t)y) * ka.tex_w + (size_t)x;
    return ka.textures[off];
}

__device__ __forceinline__ f4 sample_env(const KernelArgs& ka, const float* srgb, f3 d) {
    // environment_map_coords, :580-585. A coordinate is computed only when the
    // texel depends on it: with every row (column) of the map one colour, any u
    // (v) -- NaN included -- fetches the same texel as column (row) 0.
    int x = 0, y = 0;
    if (!(ka.env_uniform & 1u)) {
        const float u = 0.5f + div_const(atan2f_c(d.z, d.x), kTwoPiWgsl, kInvTwoPiWgsl);
        x = texel_coord(u * (float)(int32_t)ka.env_map_width, ka.env_w);
    }
    if (!(ka.env_uniform & 2u)) {
        const float v = 0.5f + div_const(asinf_c(d.y), kWgslPi, kInvWgslPi);
        y = texel_coord(v * (float)(int32_t)ka.env_map_height, ka.env_h);
    }
    return decode_texel(ka.env[(size_t)y * ka.env_w + (size_t)x], srgb);
}

// State of one path of per_pixel (compute_shader.wgsl:210-314) between bounces.
struct Path {
    f3 o, d;
    f4 light, contrib;
    uint32_t seed;
    uint32_t bounce;
};

// Camera::recalculate_ray_directions (src/camera.rs:139-182) for one pixel, in
// f32 with glam's operation order (Mat4 * Vec4 = ((c0*x + c1*y) + c2*z) + c3*w,
// Vec3A::normalize = v * (1/length)): bit-identical to the host generator
// (rust_gpu_raytracing_amd/camera.py) given the same matrices.
__device__ __forceinline__ f3 mat4_mul_xyz(const float* m, float x, float y, float z, float w, float& out_w) {
    const float r0 = ((m[0] * x + m[4] * y) + m[8] * z) + m[12] * w;
    const float r1 = ((m[1] * x + m[5] * y) + m[9] * z) + m[13] * w;
    const float r2 = ((m[2] * x + m[6] * y) + m[10] * z) + m[14] * w;
    out_w = ((m[3] * x + m[7] * y) + m[11] * z) + m[15] * w;
    return mk(r0, r1, r2);
}

// `cam` is the LDS camera block: inverse projection [16], inverse view [16], aspect.
__device__ __forceinline__ f3 camera_ray(const KernelArgs& ka, const float* cam, uint32_t x, uint32_t y) {
    const float xc = (float)x / (float)ka.width;
    const float yc = (float)y / (float)ka.height;
    const float nx = xc * 2.0f - 1.0f;
    const float ny = yc * 2.0f - 1.0f;
    const float ax = nx * cam[32];
    float tw;
    const f3 t = mat4_mul_xyz(cam, ax, ny, 1.0f, 1.0f, tw);
    const f3 ws = normalize(mk(t.x / tw, t.y / tw, t.z / tw));
    float unused;
    return mat4_mul_xyz(cam + 16, ws.x, ws.y, ws.z, 0.0f, unused);
}

__device__ __forceinline__ f3 pixel_ray(const KernelArgs& ka, const float* cam, uint32_t index, uint32_t x,
                                        uint32_t y) {
    if (ka.gen_rays) return camera_ray(ka, cam, x, y);
    const float4 cr = ka.camera_rays[index];  // binding 1
    return mk(cr.x, cr.y, cr.z);
}

// per_pixel prologue, :212-222, given the pixel's camera ray direction.
__device__ __forceinline__ void start_sample(const KernelArgs& ka, uint32_t index, uint32_t random_index, f3 cam,
                                             Path& p) {
    p.o = mk(ka.camera_origin[0], ka.camera_origin[1], ka.camera_origin[2]);
    p.d = cam;
    p.seed = index * random_index * 326624u;
    const float rx = random01(p.seed), ry = random01(p.seed), rz = random01(p.seed);
    const f3 jit = mk(rx * 2.0f - 1.0f, ry * 2.0f - 1.0f, rz * 2.0f - 1.0f);
    p.d = p.d + jit * 0.0005f;  // not renormalised (:219)
    p.contrib = f4{1.0f, 1.0f, 1.0f, 1.0f};
    p.light = f4{0.0f, 0.0f, 0.0f, 0.0f};
    p.bounce = 0;
}

// The shading half of one iteration of the bounce loop, :228-311, given the
// trace result. Returns true when the path is finished (escaped to the
// environment, or the bounce limit is reached).
// kAux: the material's glass constants come from the LDS table staged with the
// materials (same f32 operations, computed once per workgroup instead of per hit).
template <bool kAux>
__device__ __forceinline__ bool shade(const SceneView& sv, const KernelArgs& ka, Path& p, const Hit& h) {
    if (h.t == kF32Max) {
        const f4 c = sample_env(ka, sv.srgb, p.d);
        p.light.x = p.light.x + c.x * p.contrib.x;
        p.light.y = p.light.y + c.y * p.contrib.y;
        p.light.z = p.light.z + c.z * p.contrib.z;
        p.light.w = p.light.w + c.w * p.contrib.w;
        return true;
    }
    const uint32_t mi = min(h.material_index, ka.material_count - 1u);
    const RtMaterial m = sv.mat[mi];
    // 1x1 texture layers: every uv fetches texel (0, 0) of the material's layer,
    // decoded once per workgroup into the material table (kAux); otherwise the
    // texel load is issued first so that its latency overlaps the draws
    const bool tex1 = kAux && ka.tex_w == 1u && ka.tex_h == 1u;
    uint32_t texel = 0;
    if (!tex1) texel = fetch_texture(ka, m.texture_index, h.u, h.v);
    const float gx = normal01(p.seed);
    const float gy = normal01(p.seed);
    const float gz = normal01(p.seed);
    const f3 diffuse = normalize(h.n + mk(gx, gy, gz));
    const f3 specular = p.d - h.n * (2.0f * dot(h.n, p.d));  // reflect(d, n)
    f4 color;
    if (tex1) {
        const float4 c = sv.mat_aux[2u * mi + 1u];
        color = f4{c.x, c.y, c.z, c.w};
    } else {
        color = decode_texel(texel, sv.srgb);
    }
    const float e = m.emission_power;
    p.light.x = p.light.x + (color.x * e) * p.contrib.x;
    p.light.y = p.light.y + (color.y * e) * p.contrib.y;
    p.light.z = p.light.z + (color.z * e) * p.contrib.z;
    p.light.w = p.light.w + (color.w * e) * p.contrib.w;
    const bool is_glass = m.glass > random01(p.seed);
    bool tint;
    if (is_glass) {
        float ior, r0, rough10;
        if constexpr (kAux) {
            const float4 ax = sv.mat_aux[2u * mi];
            ior = h.front_face ? ax.x : m.refraction_index;
            r0 = h.front_face ? ax.y : ax.z;
            rough10 = ax.w;
        } else {
            ior = m.refraction_index;
            if (h.front_face) ior = 1.0f / ior;
            r0 = (1.0f - ior) / (1.0f + ior);  // specular_percentage, :328-334
            r0 = r0 * r0;
            rough10 = div_const(m.roughness, 10.0f, kInv10);
        }
        const float cos_t = fmin_nn(dot(-p.d, h.n), 1.0f);
        const float sin_t = sqrt_rn_nrm(1.0f - cos_t * cos_t);  // 0, >= 2^-24, or NaN
        const bool reflects = ior * sin_t > 1.0f;
        const float sp = r0 + (1.0f - r0) * pow5(1.0f - cos_t);
        const bool is_spec = (m.specular * sp) > random01(p.seed);
        if (reflects || is_spec) {
            p.d = lerp(specular, diffuse, m.specular_scatter);
            p.o = h.p + h.n * 0.0001f;
            tint = false;
        } else {
            // refract, :316-325
            const f3 perp = (p.d + h.n * cos_t) * ior;
            const float len = sqrt_rn_any(dot(perp, perp));
            const float len_sq = len * len;
            // |1 - len_sq| is 0 or >= 2^-24 (exact difference near 1): sqrt_rn_nrm's domain
            const f3 refr = perp + h.n * (-sqrt_rn_nrm(__builtin_fabsf(1.0f - len_sq)));
            p.d = lerp(refr, diffuse, rough10);
            p.o = h.p - h.n * 0.0001f;
            tint = true;
        }
    } else {
        const bool is_spec = m.specular > random01(p.seed);
        if (is_spec) {
            p.d = lerp(specular, diffuse, m.specular_scatter);
            tint = false;
        } else {
            p.d = lerp(specular, diffuse, m.roughness);
            tint = true;
        }
        p.o = h.p + h.n * 0.0001f;
    }
    if (tint) {
        p.contrib.x = p.contrib.x * color.x;
        p.contrib.y = p.contrib.y * color.y;
        p.contrib.z = p.contrib.z * color.z;
        p.contrib.w = p.contrib.w * color.w;
    }
    p.bounce += 1;
    return p.bounce >= ka.bounces;
}

__device__ __forceinline__ float clamp01(float x) { return fmin_nn(fmax_nn(x, 0.0f), 1.0f); }

// pack_to_u32, compute_shader.wgsl:192-208.
__device__ __forceinline__ uint32_t pack_rgba8(float r, float g, float b, float a) {
    const uint32_t br = (uint32_t)(r * 255.0f) & 0xffu;
    const uint32_t bg = (uint32_t)(g * 255.0f) & 0xffu;
    const uint32_t bb = (uint32_t)(b * 255.0f) & 0xffu;
    const uint32_t ba = (uint32_t)(a * 255.0f) & 0xffu;
    return br | (bg << 8) | (bb << 16) | (ba << 24);
}


// Trace result of a path's first segment, from rt_primary_kernel (below).
struct PrimaryRecord {  // 16 B: {t, id, object | front << 31 | kind << 30, original sphere index}
    float t;
    uint32_t id;     // triangle index, or sphere slot
    uint32_t meta;   // bit 30: sphere; bit 31: front face (triangle); bits 0-29: object
    uint32_t orig;   // sphere: original index
};

template <bool kTris>
__device__ __forceinline__ PrimaryRecord primary_record(const TraceState& ts) {
    // the winner exactly as trace_end picks it: the triangle unless the sphere is strictly closer
    const float tt = kTris ? ts.tri.t : kF32Max;
    if (ts.sph.t < (tt != kF32Max ? tt : kF32Max))
        return PrimaryRecord{ts.sph.t, ts.sph.slot, 1u << 30, ts.sph.orig};
    return PrimaryRecord{tt, ts.tri.tri, (ts.tri.obj & 0x3fffffffu) | (ts.tri.front ? 0x80000000u : 0u), 0u};
}

// The TraceState trace_end rebuilds the same hit from.
__device__ __forceinline__ void primary_state(const PrimaryRecord& r, TraceState& ts) {
    ts.sph = SphereHit{kF32Max, 0u, 0u};
    ts.tri = TriHit{kF32Max, 0u, 0u, 0u, false};
    if (r.meta & (1u << 30)) {
        ts.sph = SphereHit{r.t, r.orig, r.id};
    } else {
        ts.tri = TriHit{r.t, 0u, r.id, r.meta & 0x3fffffffu, (r.meta & 0x80000000u) != 0u};
    }
}

// The wavefront kernel's LDS scene image (brute force) (the persistent kernel's mode 1: spheres in slot
// order, materials + glass constants, objects, sRGB table and camera block); the caller
// synchronises before reading it. Returns the view of it; `cam` receives the camera block.
template <bool kTris, uint32_t kThreads>
__device__ __forceinline__ SceneView brute_stage(const KernelArgs& ka, unsigned char* lds, uint32_t tid, float*& l_cam) {
    // scene staging as the persistent kernel's mode 1 (spheres in slot order, materials + glass
    // constants, objects, sRGB table), then the sub-object tile
    float4* l_sph = reinterpret_cast<float4*>(lds);
    RtMaterial* l_mat = reinterpret_cast<RtMaterial*>(lds + ka.lds_mat_offset);
    float4* l_aux = reinterpret_cast<float4*>(lds + ka.lds_mat_aux_offset);
    RtObject* l_obj = reinterpret_cast<RtObject*>(lds + ka.lds_obj_offset);
    uint32_t* l_orig = reinterpret_cast<uint32_t*>(lds + ka.lds_orig_offset);
    uint32_t* l_smat = reinterpret_cast<uint32_t*>(lds + ka.lds_smat_offset);
    float* l_srgb = reinterpret_cast<float*>(lds + ka.lds_srgb_offset);
    for (uint32_t i = tid; i < ka.sphere_slot_count; i += kThreads) {
        l_sph[i] = ka.sphere_slots[i];
        l_orig[i] = ka.sphere_orig[i];
    }
    for (uint32_t i = tid; i < ka.sphere_count; i += kThreads) l_smat[i] = ka.sphere_material[i];
    for (uint32_t i = tid; i < ka.material_count; i += kThreads) {
        const RtMaterial m = ka.materials[i];
        l_mat[i] = m;
        const float ior_front = 1.0f / m.refraction_index;
        float r0f = (1.0f - ior_front) / (1.0f + ior_front);
        float r0b = (1.0f - m.refraction_index) / (1.0f + m.refraction_index);
        r0f = r0f * r0f;
        r0b = r0b * r0b;
        l_aux[2u * i] = make_float4(ior_front, r0f, r0b, div_const(m.roughness, 10.0f, kInv10));
        const f4 c = decode_texel(ka.textures[min(m.texture_index, ka.tex_layers - 1u)], ka.srgb);
        l_aux[2u * i + 1u] = make_float4(c.x, c.y, c.z, c.w);
    }
    if constexpr (kTris)
        for (uint32_t i = tid; i < ka.object_count; i += kThreads) l_obj[i] = ka.objects[i];
    for (uint32_t i = tid; i < 256u; i += kThreads) l_srgb[i] = ka.srgb[i];
    l_cam = l_srgb + 256;  // camera block for device-side primary rays
    if (tid < 16u) {
        l_cam[tid] = ka.inv_proj[tid];
        l_cam[16u + tid] = ka.inv_view[tid];
    }
    if (tid == 0) l_cam[32] = ka.aspect;
    return SceneView{l_sph, l_orig, l_smat, nullptr, l_mat, l_aux, l_obj, l_srgb, nullptr, nullptr, 0.0f,
                     ka.sub_objects};
}

}  // namespace
