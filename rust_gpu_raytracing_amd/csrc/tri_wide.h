// tri_wide.h — the 4-wide triangle accelerator: node and leaf records shared by
// the host builder (tri_wide.cpp), the kernel (pathtrace.hip), the device refit
// (scene_edit.hip) and the CPU exactness harness (tests/cpp/tri_exactness.cpp).
//
// The reference sweeps objects -> sub-objects -> triangles (check_triangles,
// compute_shader.wgsl:422-517). As with the binary accelerator,
// the leaves are the sweep's (object, sub-object) pairs and a reached leaf runs the
// reference's own object and sub-object ray_in_bounds tests and triangle tests;
// interior boxes only cull (inflated per ray by a margin that covers the f32
// rounding of the reference's slab test), so the visited leaf set is a superset of
// the one the sweep tests and, with no distance pruning, the visit order is free:
// the result (lexicographic minimum of (distance, sweep position)) is the sweep's.
//
// What is MI355X-specific is the shape. A binary stackless walk of C5's heightfield
// makes ~150 dependent node loads per ray, each a 32-B piece of an L2 line; here
// one 128-B node (one line) holds four child boxes, tested together, so a walk is
// ~40 node loads. The walk keeps a per-lane stack in LDS (one entry per tree
// level: the first internal child of a node and a mask of its children still to
// visit; a node's internal children are contiguous, so an entry needs no reload
// of the parent).
//
// Leaf records are 64 B and carry everything the leaf test needs: the exact
// sub-object box (for the reference's test), the object, the triangle range, its
// sweep position, and -- "compact" leaves -- the triangles as 4-bit indices into a
// per-leaf block of at most 16 vertices, from which a, edge_ab = b - a, edge_ac =
// c - a and calc_normal = edge_ab x edge_ac are recomputed with the f32 operations
// of SceneTriangle::new (src/buffers.rs:66-95). A leaf is compact only when that
// recomputation reproduces every stored triangle record bit for bit (checked when
// built, and again on the device after every triangle update or edit); otherwise it
// reads the 64-B triangle records. C5's 7-triangle heightfield strips share 15
// vertices: 180 B of vertices instead of 448 B of records per leaf.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_WIDE_FN __host__ __device__ __forceinline__
#else
#define RT_WIDE_FN inline
#endif

constexpr uint32_t kWideArity = 4;
constexpr uint32_t kWideLeafTris = 8;       // triangles per leaf record at most (sub-objects split into chunks)
constexpr uint32_t kWideLeafVerts = 16;     // vertices of a compact leaf at most (4-bit indices)
constexpr uint32_t kWideMaxDepth = 32;      // stack entries the kernel reserves at most (deeper trees: binary walk)
constexpr uint32_t kWideLeafCompact = 0x100u;       // TriLeaf::count_flags: the vertex block is valid now
constexpr uint32_t kWideLeafCompactBuilt = 0x200u;  // the leaf has a vertex block (validity rechecked on updates)

// 128 B, one L2 line. Boxes structure-of-arrays so the four slab tests read
// lo[axis] / hi[axis] of the four slots as float4s.
struct TriWideNode {
    float lo[3][4];       // lo[axis][slot]: the inflation-free box, rounded outward (culling only)
    float hi[3][4];
    // slots [0, n_internal) are internal children, child_base + slot;
    // slots [n_internal, n_internal + n_leaves) are leaves, leaf_base + slot - n_internal;
    // the rest are empty (their boxes are never tested)
    uint32_t child_base;
    uint32_t leaf_base;
    uint32_t slots;       // n_internal | n_leaves << 4
    uint32_t _pad[5];
};
static_assert(sizeof(TriWideNode) == 128, "wide node = one 128-B line");

// 64 B.
struct TriLeaf {
    float mn[3];          // the sub-object's bounds as stored (the reference's ray_in_bounds, :441)
    uint32_t first_tri;   // index of the leaf's first triangle in the triangle buffer
    float mx[3];
    uint32_t seq_base;    // position of that triangle in the reference's sweep order (tie-break, :457)
    uint32_t object;      // object index (its ray_in_bounds, :431; material and uv of a hit, :506, :568)
    uint32_t count_flags; // bits 0-7: triangles; kWideLeafCompactBuilt / kWideLeafCompact: a vertex block exists /
                          // reproduces the triangle records (then the leaf test reads it)
    uint32_t vbase;       // compact: first vertex of the leaf's block in the vertex array
    uint32_t sub;         // sub-object index (the device refit copies its bounds)
    uint32_t idx[4];      // compact: triangle j's vertex k is nibble 3j + k (idx[0] bits 0-3 first)
};
static_assert(sizeof(TriLeaf) == 64, "leaf record");

struct TriVertex {
    float x, y, z;
};
static_assert(sizeof(TriVertex) == 12, "packed vertex");

// SceneTriangle::new's edge and normal arithmetic (src/buffers.rs:66-95, glam
// Vec3A sub and cross in f32): what a compact leaf recomputes per triangle.
RT_WIDE_FN void wide_tri_from_vertices(const TriVertex& a, const TriVertex& b, const TriVertex& c, float* ab,
                                       float* ac, float* cn) {
    ab[0] = b.x - a.x;
    ab[1] = b.y - a.y;
    ab[2] = b.z - a.z;
    ac[0] = c.x - a.x;
    ac[1] = c.y - a.y;
    ac[2] = c.z - a.z;
    cn[0] = ab[1] * ac[2] - ab[2] * ac[1];
    cn[1] = ab[2] * ac[0] - ab[0] * ac[2];
    cn[2] = ab[0] * ac[1] - ab[1] * ac[0];
}

// Vertex index of triangle j, corner k of a compact leaf.
RT_WIDE_FN uint32_t wide_leaf_index(const uint32_t* idx, uint32_t j, uint32_t k) {
    const uint32_t n = 3u * j + k;
    return (idx[n >> 3] >> ((n & 7u) * 4u)) & 0xfu;
}

// ---- host side -----------------------------------------------------------
#include <vector>

#include "rt_abi.h"

// The binary SAH tree the wide one is collapsed from switches to median splits
// where its depth would exceed this, so the wide tree stays within
// kWideMaxDepth levels (a median-split subtree of n leaves is ceil(log2 n) deep).
constexpr uint32_t kWideBinaryDepthCap = 2 * kWideMaxDepth - 2;

struct TriWide {
    std::vector<TriWideNode> nodes;    // nodes[0] is the root
    std::vector<TriLeaf> leaves;
    std::vector<TriVertex> verts;      // compact leaves' vertex blocks
    std::vector<uint32_t> vsrc;        // per vertex: source triangle * 4 + corner (0 a, 1 a + ab, 2 a + ac)
    std::vector<uint32_t> order;       // node indices by depth, deepest level first (device refit)
    std::vector<uint32_t> level_off;   // order[level_off[l], level_off[l + 1]) = level l
    uint32_t depth = 0;                // levels of nodes (the walk's stack needs depth - 1 entries)
    float extent = 0.0f;               // max |coordinate| over finite sub-object boxes (rounded up): margin scale
};

// Build over the first `object_count` objects. `hot16`: the triangle buffer in the
// kernel's 64-B layout (16 floats per triangle), or null for no compact leaves.
void build_triangle_wide(const rt_object_info* objects, uint32_t object_count, const rt_sub_object_info* subs,
                         uint32_t sub_count, const float* hot16, uint32_t n_tri, TriWide* out);

// Makes `leaf` compact when its triangles allow it (appending its vertex block);
// returns whether it did.
bool wide_leaf_make_compact(const float* hot16, uint32_t n_tri, TriLeaf& leaf, std::vector<TriVertex>& verts,
                            std::vector<uint32_t>& vsrc);
