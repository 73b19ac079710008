// scene_edit.hip — device-side scene rebuild after an edit.
//
// Renderer::update_scene (src/renderer.rs:153-199) recomputes every object's
// triangles from its normalised points (SceneObject::update_triangles,
// src/triangle_object.rs:129-150), the object bounds, and the sub-object
// bounds (update_sub_objects, :199-220), on the host, then uploads them. Here
// the same arithmetic (rt_scene_math.h, shared with the host builder) runs on
// the device, and the triangle accelerator's boxes are refitted in place, so an
// edit costs a few small launches and no host round trip:
//
//   rt_edit_triangles_kernel   one thread per triangle: place its 3 points,
//                              SceneTriangle::new -> the 64-B record the path
//                              tracer reads + the per-triangle bounds
//   rt_edit_sub_objects_kernel one thread per sub-object: get_bounding_box over
//                              [min0, max0, min1, max1, ...] of its triangles
//   rt_edit_objects_kernel     one workgroup per object: get_bounding_box over
//                              its placed points, as an order-preserving
//                              reduction (equal to the reference's sequential
//                              scan bit for bit, +0/-0 ties included)
//   rt_refit_tri_bvh_kernel    one workgroup: the accelerator's boxes level by
//                              level, deepest first, and the margin extent
//
// All of it is memory-bound elementwise work (HBM roofline; 36 B in and 112 B
// out per triangle), off the per-frame path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_kernel_args.h"
#include "rt_scene_math.h"
#include "sphere_bvh.h"
#include "tri_cone.h"
#include "tri_qnode.h"

#pragma clang fp contract(off)

using namespace rt_scene;

namespace {

__device__ __forceinline__ void load3(const float* p, float* v) {
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
}

// Order-preserving merge of two get_bounding_box partials (`lo` covers earlier
// points): the later one wins only if strictly smaller / larger, so of equal
// values the first in point order is kept, as in the sequential scan. NaN and
// values beyond the +-f32::MAX start never enter a partial.
__device__ __forceinline__ void merge_box(float* lo_mn, float* lo_mx, const float* hi_mn, const float* hi_mx) {
    for (int k = 0; k < 3; k++) {
        if (hi_mn[k] < lo_mn[k]) lo_mn[k] = hi_mn[k];
        if (hi_mx[k] > lo_mx[k]) lo_mx[k] = hi_mx[k];
    }
}

}  // namespace

extern "C" __global__ void __launch_bounds__(256) rt_edit_triangles_kernel(
    const float* __restrict__ model, const uint32_t* __restrict__ tri_object, const Placement* __restrict__ place,
    uint32_t object_count, uint32_t n_tri, RtTriangleHot* __restrict__ tris, float4* __restrict__ bounds) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tri) return;
    const uint32_t o = tri_object[t];
    if (o >= object_count) return;  // not in an edited object
    const Placement pl = place[o];
    float a[3], b[3], c[3], v[3];
    load3(model + 9 * (size_t)t, v);
    place_point(pl, v, a);
    load3(model + 9 * (size_t)t + 3, v);
    place_point(pl, v, b);
    load3(model + 9 * (size_t)t + 6, v);
    place_point(pl, v, c);
    TriangleRecord r;
    scene_triangle(a, b, c, r);
    tris[t] = pack_triangle(a, r.ab, r.ac, r.calc_normal, r.face_normal);
    bounds[2 * (size_t)t] = make_float4(r.mn[0], r.mn[1], r.mn[2], 0.f);
    bounds[2 * (size_t)t + 1] = make_float4(r.mx[0], r.mx[1], r.mx[2], 0.f);
}

extern "C" __global__ void __launch_bounds__(256) rt_edit_sub_objects_kernel(
    const uint32_t* __restrict__ sub_object, uint32_t object_count, uint32_t n_sub, const float4* __restrict__ bounds,
    RtSubObject* __restrict__ subs) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_sub || sub_object[s] >= object_count) return;
    RtSubObject so = subs[s];
    BoxScan box;
    for (uint32_t i = 0; i < so.triangle_count; i++) {
        const size_t t = (size_t)so.first_triangle_index + i;
        const float4 lo = bounds[2 * t], hi = bounds[2 * t + 1];
        const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
        box.add(l);
        box.add(h);
    }
    box.get(so.min_bounds, so.max_bounds);
    subs[s] = so;
}

// One workgroup per object. Thread i scans a contiguous slice of the object's
// triangles (points in order), then the slices are merged pairwise in order.
constexpr uint32_t kObjThreads = 256;

extern "C" __global__ void __launch_bounds__(kObjThreads) rt_edit_objects_kernel(
    const float* __restrict__ model, const Placement* __restrict__ place, const uint2* __restrict__ object_tris,
    RtObject* __restrict__ objects) {
    __shared__ float s_mn[kObjThreads][3], s_mx[kObjThreads][3];
    const uint32_t o = blockIdx.x;
    const uint2 range = object_tris[o];  // first triangle, count
    const Placement pl = place[o];
    const uint32_t per = (range.y + kObjThreads - 1) / kObjThreads;
    const uint32_t first = range.x + min(range.y, threadIdx.x * per);
    const uint32_t last = range.x + min(range.y, (threadIdx.x + 1) * per);
    BoxScan box;
    for (uint32_t t = first; t < last; t++)
        for (int k = 0; k < 3; k++) {
            float v[3], p[3];
            load3(model + 9 * (size_t)t + 3 * k, v);
            place_point(pl, v, p);
            box.add(p);
        }
    box.get(s_mn[threadIdx.x], s_mx[threadIdx.x]);
    __syncthreads();
    for (uint32_t w = 1; w < kObjThreads; w *= 2) {
        if ((threadIdx.x % (2 * w)) == 0) merge_box(s_mn[threadIdx.x], s_mx[threadIdx.x], s_mn[threadIdx.x + w],
                                                   s_mx[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0 && range.y != 0) {
        RtObject ob = objects[o];
        for (int k = 0; k < 3; k++) {
            ob.min_bounds[k] = s_mn[0][k];
            ob.max_bounds[k] = s_mx[0][k];
        }
        objects[o] = ob;
    }
}

// Refit of the triangle accelerator (sphere_bvh.h TriangleAccel): same
// topology, boxes recomputed from the current sub-object bounds exactly as
// build_triangle_accel sets them (leaf = the sub-object's box, corners
// min/max-ordered; a non-finite box encloses everything), internal nodes =
// union of the two children, processed one depth level at a time, deepest
// first. Also the margin extent (max |coordinate| over finite leaf boxes,
// rounded up), which the path tracer reads from device memory.
constexpr uint32_t kRefitThreads = 1024;

extern "C" __global__ void __launch_bounds__(kRefitThreads) rt_refit_tri_bvh_kernel(
    SphereBvhNode* __restrict__ nodes, const SubObjectPrim* __restrict__ prims, const RtSubObject* __restrict__ subs,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ level_offsets, uint32_t n_levels,
    float* __restrict__ extent_out) {
    __shared__ float s_ext[kRefitThreads];
    float ext = 0.0f;
    for (uint32_t l = 0; l < n_levels; l++) {
        for (uint32_t i = level_offsets[l] + threadIdx.x; i < level_offsets[l + 1]; i += kRefitThreads) {
            const uint32_t n = order[i];
            SphereBvhNode nd = nodes[n];
            if (nd.leaf != kSphereBvhInternal) {
                const RtSubObject s = subs[prims[nd.leaf & 0xffffffu].sub];
                bool finite = true;
                for (int k = 0; k < 3; k++)
                    finite = finite && __builtin_isfinite(s.min_bounds[k]) && __builtin_isfinite(s.max_bounds[k]);
                for (int k = 0; k < 3; k++) {
                    const float a = fminf(s.min_bounds[k], s.max_bounds[k]);
                    const float b = fmaxf(s.min_bounds[k], s.max_bounds[k]);
                    nd.bmin[k] = finite ? a : -3.0e38f;
                    nd.bmax[k] = finite ? b : 3.0e38f;
                    if (finite) ext = fmaxf(ext, fmaxf(fabsf(a), fabsf(b)));
                }
            } else {
                const SphereBvhNode& l0 = nodes[n + 1];
                const SphereBvhNode& r0 = nodes[l0.skip];
                for (int k = 0; k < 3; k++) {
                    nd.bmin[k] = fminf(l0.bmin[k], r0.bmin[k]);
                    nd.bmax[k] = fmaxf(l0.bmax[k], r0.bmax[k]);
                }
            }
            nodes[n] = nd;
        }
        __syncthreads();
    }
    s_ext[threadIdx.x] = ext;
    __syncthreads();
    for (uint32_t w = kRefitThreads / 2; w > 0; w /= 2) {
        if (threadIdx.x < w) s_ext[threadIdx.x] = fmaxf(s_ext[threadIdx.x], s_ext[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *extent_out = __uint_as_float(__float_as_uint(s_ext[0]) + 1u);  // nextafter up
}

hipError_t rt_launch_edit(const float* model, const uint32_t* tri_object, const uint32_t* sub_object,
                          const uint2* object_tris, const Placement* place, uint32_t object_count, uint32_t n_tri,
                          uint32_t n_sub, RtTriangleHot* tris, float4* bounds, RtSubObject* subs, RtObject* objects,
                          hipStream_t stream) {
    if (n_tri) {
        hipLaunchKernelGGL(rt_edit_triangles_kernel, dim3((n_tri + 255) / 256), dim3(256), 0, stream, model,
                           tri_object, place, object_count, n_tri, tris, bounds);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (n_sub) {
        hipLaunchKernelGGL(rt_edit_sub_objects_kernel, dim3((n_sub + 255) / 256), dim3(256), 0, stream, sub_object,
                           object_count, n_sub, bounds, subs);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (object_count) {
        hipLaunchKernelGGL(rt_edit_objects_kernel, dim3(object_count), dim3(kObjThreads), 0, stream, model, place,
                           object_tris, objects);
        return hipGetLastError();
    }
    return hipSuccess;
}

hipError_t rt_launch_refit(SphereBvhNode* nodes, const SubObjectPrim* prims, const RtSubObject* subs,
                           const uint32_t* order, const uint32_t* level_offsets, uint32_t n_levels, float* extent_out,
                           hipStream_t stream) {
    hipLaunchKernelGGL(rt_refit_tri_bvh_kernel, dim3(1), dim3(kRefitThreads), 0, stream, nodes, prims, subs, order,
                       level_offsets, n_levels, extent_out);
    return hipGetLastError();
}

// ---- 16-B quantized copy of the binary triangle accelerator (tri_qnode.h) ----
// grid[0] = {origin.xyz, valid}, grid[1] = {scale.xyz, 0}; with valid = 0 the walk reads the
// 32-B nodes.
// With src / skip (the direction-ordered layouts of order_bvh_by_octant: n_out = 8 x n
// positions, each the node src[i] of the base accelerator with the layout's skip link
// skip[i]), position i of both copies is derived from the base node after every upload or
// refit: out32 (32-B nodes, the layout's links) and q (quantized; a leaf whose skip leaves
// its layout carries kTriQLastLeaf, so the walk ends there instead of at node + 1).
extern "C" __global__ void __launch_bounds__(256) rt_quantize_tri_nodes_kernel(
    const SphereBvhNode* __restrict__ nodes, uint32_t n, const uint32_t* __restrict__ src,
    const uint32_t* __restrict__ skip, uint32_t n_out, SphereBvhNode* __restrict__ out32, uint4* __restrict__ q,
    float4* __restrict__ grid) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    TriQGrid g{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, false};
    if (n != 0) g = tri_qgrid(nodes[0]);
    if (i == 0 && grid) {
        grid[0] = make_float4(g.origin[0], g.origin[1], g.origin[2], g.valid ? 1.f : 0.f);
        grid[1] = make_float4(g.scale[0], g.scale[1], g.scale[2], 0.f);
    }
    if (i >= n_out) return;
    SphereBvhNode nd = nodes[src ? src[i] : i];
    if (src) {
        nd.skip = skip[i];
        if (out32) out32[i] = nd;
    }
    if (!g.valid || !q) return;
    uint32_t w[4];
    tri_qnode(nd, g, w);
    if (src && nd.leaf != kSphereBvhInternal && nd.skip >= n_out) w[3] |= kTriQLastLeaf;
    q[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

hipError_t rt_launch_quantize_tri_nodes(const SphereBvhNode* nodes, uint32_t n, const uint32_t* src,
                                        const uint32_t* skip, uint32_t n_out, SphereBvhNode* out32, uint4* q,
                                        float4* grid, hipStream_t stream) {
    const uint32_t blocks = n_out ? (n_out + 255u) / 256u : 1u;
    hipLaunchKernelGGL(rt_quantize_tri_nodes_kernel, dim3(blocks), dim3(256), 0, stream, nodes, n, src, skip, n_out,
                       out32, q, grid);
    return hipGetLastError();
}

// Leaf certificates (tri_cone.h TriLeafCert), one per leaf record (prim), from its sub-object's
// box and the triangle records the walk's leaf test reads (same index clamp); rebuilt with the
// cones after every change of the accelerator or the triangles.
extern "C" __global__ void __launch_bounds__(256) rt_tri_leafcert_kernel(const SubObjectPrim* __restrict__ prims,
                                                                        uint32_t n_prims,
                                                                        const RtSubObject* __restrict__ subs,
                                                                        const RtTriangleHot* __restrict__ tris,
                                                                        uint32_t n_tri, TriLeafCert* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_prims) return;
    const RtSubObject s = subs[prims[i].sub];
    float lo[3], hi[3];
    for (int k = 0; k < 3; k++) {
        lo[k] = fminf(s.min_bounds[k], s.max_bounds[k]);
        hi[k] = fmaxf(s.min_bounds[k], s.max_bounds[k]);
    }
    const uint32_t cnt = (s.triangle_count <= kLeafCertSlots && n_tri != 0u) ? s.triangle_count : 0u;
    float a[kLeafCertSlots][3], ab[kLeafCertSlots][3], ac[kLeafCertSlots][3], cn[kLeafCertSlots][3];
    for (uint32_t j = 0; j < cnt; ++j) {
        float fn[3];
        unpack_triangle(tris[min(s.first_triangle_index + j, n_tri - 1u)], a[j], ab[j], ac[j], cn[j], fn);
    }
    out[i] = tricone::leafcert_build(cnt, a, ab, ac, cn, lo, hi);
}

hipError_t rt_launch_tri_leafcert(const SubObjectPrim* prims, uint32_t n_prims, const RtSubObject* subs,
                                  const RtTriangleHot* tris, uint32_t n_tri, TriLeafCert* out, hipStream_t stream) {
    if (n_prims == 0 || !out) return hipSuccess;
    hipLaunchKernelGGL(rt_tri_leafcert_kernel, dim3((n_prims + 255u) / 256u), dim3(256), 0, stream, prims, n_prims,
                       subs, tris, n_tri, out);
    return hipGetLastError();
}

// Leaf triangle blocks (KernelArgs::tri_leaftris), one per leaf record, for the cooperative leaf
// batches of the walks from global memory (pathtrace.hip coop_leaf_batch): piece p (0..2) of
// triangle slot j at word 8p + j -- the record's own first 48 B (a, edge_ab, edge_ac,
// calc_normal), bit for bit, at the same index clamp as the per-lane leaf test -- so that the
// 8 lanes testing one leaf read one 128-B line per piece. Slots past the leaf's count, and
// leaves whose triangle range is not in the record (kPrimRangeNone: those are tested per
// lane), are zero. Rebuilt with the certificates after every change of the accelerator or the
// triangles. One thread per word.
extern "C" __global__ void __launch_bounds__(256) rt_tri_leaftris_kernel(const SubObjectPrim* __restrict__ prims,
                                                                        uint32_t n_prims,
                                                                        const RtTriangleHot* __restrict__ tris,
                                                                        uint32_t n_tri, uint4* __restrict__ out) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)n_prims * kLeafTriWords) return;
    const uint32_t i = (uint32_t)(gid / kLeafTriWords), w = (uint32_t)(gid % kLeafTriWords);
    const uint32_t j = w % kLeafTriSlots, piece = w / kLeafTriSlots;
    const uint32_t range = prims[i].range;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (range != kPrimRangeNone && j < (range >> 27) && n_tri != 0u) {
        const uint4* t = reinterpret_cast<const uint4*>(tris + min((range & ((1u << 27) - 1u)) + j, n_tri - 1u));
        v = t[piece];
    }
    out[gid] = v;
}

hipError_t rt_launch_tri_leaftris(const SubObjectPrim* prims, uint32_t n_prims, const RtTriangleHot* tris,
                                  uint32_t n_tri, uint4* out, hipStream_t stream) {
    if (n_prims == 0 || !out) return hipSuccess;
    const uint64_t n = (uint64_t)n_prims * kLeafTriWords;
    hipLaunchKernelGGL(rt_tri_leaftris_kernel, dim3((uint32_t)((n + 255u) / 256u)), dim3(256), 0, stream, prims,
                       n_prims, tris, n_tri, out);
    return hipGetLastError();
}
