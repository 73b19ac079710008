// rt_kernel_args.h — device-side scene records and the kernel argument block.
//
// The records are the reference's GPU layouts (src/buffers.rs:7-129,
// compute_shader.wgsl:43-126) except the triangle, which is repacked on upload
// to the 64 bytes the kernel reads (the reference's 112-byte SceneTriangle
// carries per-triangle bounds the shader never touches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tri_cone.h"

struct RtSphere {  // src/buffers.rs:40-45, 32 B
    float position[3];
    float radius;
    uint32_t material_index;
    uint32_t _pad[3];
};

struct RtMaterial {  // src/buffers.rs:100-109, 32 B
    uint32_t texture_index;
    float roughness;
    float emission_power;
    float specular;
    float specular_scatter;
    float glass;
    float refraction_index;
    uint32_t _pad;
};

struct RtObject {  // src/buffers.rs:113-120, 48 B
    float min_bounds[3];
    uint32_t first_sub_object_index;
    float max_bounds[3];
    uint32_t sub_object_count;
    uint32_t material_index;
    uint32_t _pad[3];
};

struct RtSubObject {  // src/buffers.rs:124-129, 32 B
    float min_bounds[3];
    uint32_t first_triangle_index;
    float max_bounds[3];
    uint32_t triangle_count;
};

// The SceneTriangle fields the kernel reads (src/buffers.rs:49-64), 64 B: the
// four vectors of the intersection test packed into the first 48 B (three
// 16-B loads), face_normal (read only for the closest hit) last. A record never
// straddles a 128-B line, and a sub-object's 7 triangles span 448 B.
struct RtTriangleHot {
    float4 p0;  // a.x a.y a.z edge_ab.x
    float4 p1;  // edge_ab.y edge_ab.z edge_ac.x edge_ac.y
    float4 p2;  // edge_ac.z calc_normal.x calc_normal.y calc_normal.z
    float4 fn;  // face_normal.x face_normal.y face_normal.z 0
};

__host__ __device__ inline RtTriangleHot pack_triangle(const float* a, const float* ab, const float* ac,
                                                       const float* cn, const float* fn) {
    RtTriangleHot h;
    h.p0 = make_float4(a[0], a[1], a[2], ab[0]);
    h.p1 = make_float4(ab[1], ab[2], ac[0], ac[1]);
    h.p2 = make_float4(ac[2], cn[0], cn[1], cn[2]);
    h.fn = make_float4(fn[0], fn[1], fn[2], 0.f);
    return h;
}

__host__ __device__ inline void unpack_triangle(const RtTriangleHot& h, float* a, float* ab, float* ac, float* cn,
                                                float* fn) {
    a[0] = h.p0.x, a[1] = h.p0.y, a[2] = h.p0.z;
    ab[0] = h.p0.w, ab[1] = h.p1.x, ab[2] = h.p1.y;
    ac[0] = h.p1.z, ac[1] = h.p1.w, ac[2] = h.p2.x;
    cn[0] = h.p2.y, cn[1] = h.p2.z, cn[2] = h.p2.w;
    fn[0] = h.fn.x, fn[1] = h.fn.y, fn[2] = h.fn.z;
}

static_assert(sizeof(RtSphere) == 32, "SceneSphere layout");
static_assert(sizeof(RtMaterial) == 32, "SceneMaterial layout");
static_assert(sizeof(RtObject) == 48, "ObjectInfo layout");
static_assert(sizeof(RtSubObject) == 32, "SubObjectInfo layout");
static_assert(sizeof(RtTriangleHot) == 64, "hot triangle layout");

// Cost-ordered tile schedule: buckets of the counting sort (pathtrace.hip,
// sort_tiles_by_cost), whose scratch reuses the LDS tail after the frame loop.
#ifndef RT_ORDER_BUCKETS
#define RT_ORDER_BUCKETS 16
#endif
constexpr uint32_t kOrderBuckets = RT_ORDER_BUCKETS;
// Always staged at the end of the LDS image: the sRGB table (256 floats) and
// the camera block (inverse projection, inverse view, aspect: 33 floats, 160 B
// reserved). After the frame loop the sort's scratch (kOrderBuckets x 16 waves
// + 1 words) reuses it.
constexpr size_t kLdsTailBytes = 1024 + 160;
static_assert(kLdsTailBytes >= (kOrderBuckets * 16 + 1) * 4, "sort scratch fits the LDS tail");

// Cooperative leaf batches (pathtrace.hip coop_leaf_batch): a leaf record's triangle block, and
// the per-wave LDS scratch (one 48-B slot per lane: the ray and leaf of a pending lane, then its
// leaf's result).
constexpr uint32_t kLeafTriSlots = 8;                       // triangle slots per block (7 used)
constexpr uint32_t kLeafTriWords = 3 * kLeafTriSlots;       // uint4 per block (384 B)
constexpr uint32_t kLeafBatchWaveBytes = 64 * 48;

// Diagnostic counters ahead of the per-wave records in KernelArgs::diag
// (RT_DIAG: words 0-25; RT_DIAG_TAIL: words 0-7, then 2 words per wave from here).
constexpr uint32_t kDiagHeaderWords = 32;

struct KernelArgs {
    // framebuffer (bindings 1, 2, 6)
    const float4* __restrict__ camera_rays;
    float4* __restrict__ accum;
    uint32_t* __restrict__ output;
    unsigned long long* __restrict__ ray_counter;
    unsigned long long* __restrict__ diag;          // kDiagHeaderWords counters, then per-wave records (diagnostic builds)
    uint32_t* __restrict__ queue;       // this launch's tile-queue stripe counters (zero at launch start)
    uint32_t* __restrict__ queue_next;  // the next launch's counters, zeroed by this launch
    // cost-ordered tile schedule (pathtrace.hip, sort_tiles_by_cost), null when
    // off: costs[2][owned_tiles], orders[2][owned_tiles], sort flags[2]; launch
    // parity p = sched_bits & 1 records costs[p] and claims in orders[p] (if
    // sched_bits & 2), and its first idle workgroup sorts costs[p^1] (the
    // previous launch's) into orders[p^1] for the next launch
    uint32_t* __restrict__ sched;
    const uint32_t* __restrict__ tile_order;  // = orders[p] when valid, else null (index order)
    uint32_t* __restrict__ tile_cost;         // = costs[p]
    // scene (bindings 3, 4, 5, 7, 8, 10)
    const float4* __restrict__ sphere_slots;      // centre.xyz, radius*radius (f32), kernel order (sphere_bvh.h)
    const uint32_t* __restrict__ sphere_orig;     // slot -> original sphere index
    const uint32_t* __restrict__ sphere_material; // original index -> material index
    const float4* __restrict__ sphere_bvh;        // SphereBvhNode[sphere_nodes] as float4 pairs
    const RtMaterial* __restrict__ materials;
    const RtObject* __restrict__ objects;
    const RtSubObject* __restrict__ sub_objects;
    const RtTriangleHot* __restrict__ triangles;
    const float4* __restrict__ tri_bvh;           // BVH over (object, sub-object) pairs, float4 pairs per node
    const uint4* __restrict__ tri_prims;          // per leaf: object, sub-object, sweep position of its first triangle
    // 16-B quantized copy of tri_bvh (rt_quantize_tri_nodes_kernel) for walks from global memory
    // (LDS modes 0/1); tri_qgrid = {origin.xyz, valid}, {scale.xyz, 0}. Null: the 32-B nodes.
    const uint4* __restrict__ tri_qnodes;
    const float4* __restrict__ tri_qgrid;
    // textures (bindings 9, 11), RGBA8 sRGB, + decode table
    const uint32_t* __restrict__ textures;
    const uint32_t* __restrict__ env;
    const float* __restrict__ srgb;
    float camera_origin[3];
    // device-side primary rays (rt_update_camera_matrices): column-major 4x4
    float inv_proj[16];
    float inv_view[16];
    float aspect;        // f32(width) / f32(height), src/camera.rs:142
    uint32_t gen_rays;   // 1: compute camera rays, 0: read camera_rays
    // Params (binding 0), passed by value at launch
    uint32_t width;
    uint32_t accumulation_index;
    uint32_t accumulate;
    uint32_t sphere_count;
    uint32_t object_count;
    uint32_t sphere_slot_count;  // padded slots (groups of 4, sphere_bvh.h)
    uint32_t sphere_always;   // slots [0, sphere_always) are swept brute force
    uint32_t sphere_nodes;    // BVH nodes over the remaining slots (0: none)
    uint32_t sphere_octant_stride;  // nodes per direction-ordered layout (0: one layout, order_bvh_by_octant)
    uint32_t sphere_boxes_ordered;  // 1: the 8 layouts store boxes as (near, far) corners (slab_hit_ordered)
    float sphere_extent;      // max |centre| + radius over BVH spheres (margin scale)
    float sphere_rmin, sphere_rmax;  // radius range over BVH spheres (culling bounds, rt_bvh_slab.h)
    uint32_t tri_nodes;       // triangle BVH nodes (0 with tri_accel: nothing to hit)
    uint32_t tri_prim_count;  // triangle BVH leaves
    uint32_t tri_accel;       // 1: use the triangle BVH, 0: the reference's sweep
    const float* __restrict__ tri_extent;  // max |coordinate| over sub-object boxes (margin scale), device memory
    // Walks from global memory (LDS modes 0/1): tri_bvh / tri_qnodes hold 8 direction-ordered
    // layouts of tri_octant_stride nodes each (order_bvh_by_octant; tri_nodes = 8 x stride), a
    // ray starts at layout octant(d) x stride; 0: one layout.
    uint32_t tri_octant_stride;
    // distance pruning of the triangle walk, once a triangle is hit at t:
    // tri_prune_mode 1 = certified (a leaf entered beyond t: the triangles its certificate in
    // tri_leafcert -- one per leaf record, tri_prims' indexing -- proves cannot be accepted at a
    // distance <= t are skipped; null: box culling); 2 = the round-3 relative slack (boxes
    // entered beyond t * (1 + tri_prune) + 2^-10 (|o| + extent) / |d|; not exact); 0 = box
    // culling only
    uint32_t tri_prune_mode;
    float tri_prune;
    const TriLeafCert* __restrict__ tri_leafcert;
    // Leaf triangle blocks (walks from global memory, RT_COOP_LEAVES): per leaf record (tri_prims'
    // indexing) kLeafTriWords uint4 -- piece p (0..2) of triangle slot j (0..7) at [8p + j], the
    // first 48 B of the triangle's RtTriangleHot record, so piece p of a leaf's triangles is one
    // 128-B line; slots past the leaf's count are zero. Null: the leaf batches test per lane.
    const uint4* __restrict__ tri_leaftris;
    uint32_t lds_leafbatch_offset;  // per wave kLeafBatchWaveBytes of LDS for the cooperative leaf batch
    uint32_t compute_per_frame;
    uint32_t frames;          // frames rendered by this launch (rt_compute_frames), >= 1
    // Frame-parallel batch (frames > 1, accumulating): the queue holds one unit per
    // (frame, tile) -- queue_units = frames * owned_tiles -- and a finished sample
    // stores its path light to frame_light[(frame * compute_per_frame + sample) *
    // owned_px + local pixel]; rt_resolve_frames_kernel then adds them to the
    // accumulation in the reference's order. Null / owned_tiles otherwise.
    float4* __restrict__ frame_light;
    uint32_t queue_units;
    uint32_t unit_tile_major;  // frame-parallel units: 1 = a tile's frames consecutive, 0 = frame-major
    // launch timing (rt_set_timing), null otherwise: {~earliest workgroup start, latest
    // workgroup end} on the device wall clock
    unsigned long long* __restrict__ launch_clock;
    // coherent primary rays (rt_primary_kernel): one 16-B trace result per (frame, sample, owned
    // pixel), indexed like frame_light; the path kernel starts its paths from them. Null: off.
    uint4* __restrict__ primary;
    uint32_t primary_tile_major;  // the pre-pass takes its (frame, tile) units tile-major (1) or frame-major
    // brute-force launches (rt_brute_wf_kernel): the tile-streaming bytes of SURVEY §8d's
    // convention (32 B x the sweep's sub-objects per 256-ray chunk of a bounce level), and the
    // sub-object bytes the sweeps actually read from L2 (per LDS tile, or per wave when streamed)
    unsigned long long* __restrict__ stream_bytes;
    unsigned long long* __restrict__ l2_stream_bytes;
    // the brute-force wavefront (rt_brute_wf_kernel): per owned pixel slot the path state (4
    // planes of float4: o + seed, d + bounce, light, contribution, plane stride = owned slots),
    // two queues of live slots (ping-pong by bounce level), per pass brute_levels counters
    // (entries of each level's queue, bounces + 1 of them); this launch's pass (frame *
    // compute_per_frame + sample) and bounce level
    float4* __restrict__ brute_paths;
    uint32_t* __restrict__ brute_queue;
    uint32_t* __restrict__ brute_counts;
    uint32_t brute_levels;
    uint32_t brute_pass;
    uint32_t brute_level;
    uint32_t texture_width;
    uint32_t texture_height;
    uint32_t env_map_width;
    uint32_t env_map_height;
    // extents of what is actually allocated (Restrict-policy clamps)
    uint32_t material_count;
    uint32_t sub_object_count;
    uint32_t triangle_count;
    uint32_t tex_w, tex_h, tex_layers;
    uint32_t env_w, env_h;
    uint32_t env_uniform;  // bit 0: env map rows uniform (u unused), bit 1: columns uniform (v unused)
    // launch geometry
    uint32_t height;
    uint32_t bounces;
    uint32_t tiles_x;
    uint32_t owned_tiles;
    uint32_t rank;
    uint32_t world_size;
    uint32_t trav_threshold;  // resume shading once at most this many lanes still traverse
    uint32_t drain_threshold; // decoupled drain (triangle BVH in global memory): the same once the tile
    uint32_t drain_min_steps; // queue is empty and some lane is done, after at least this many steps
    uint32_t leaf_batch;      // test deferred leaves once 8 * pending >= leaf_batch * traversing
    uint32_t queue_stripes;   // tile-queue stripes (one per XCD)
    uint32_t sched_bits;      // cost-ordered schedule: launch parity
    // dynamic LDS carve-up (byte offsets)
    uint32_t lds_mat_offset;
    uint32_t lds_mat_aux_offset;  // per material 2 float4: {1/ior, r0 front face, r0 back face, roughness/10},
                                  // the decoded texel of a 1x1 texture layer (modes 1, 2)
    uint32_t lds_obj_offset;
    uint32_t lds_orig_offset;
    uint32_t lds_smat_offset;
    uint32_t lds_nodes_offset;
    uint32_t lds_tri_nodes_offset;
    uint32_t lds_tri_prims_offset;
    uint32_t lds_sub_offset;  // mode 2: sub-object records staged in LDS at this offset; 0: read from global
    uint32_t lds_stack_offset;    // brute force: the sub-object tiles and hit lists after the scene image
    uint32_t lds_srgb_offset;
};
