// tri_q4.h -- the 4-wide, 64-byte quantized triangle accelerator for walks from global memory.
//
// The binary accelerator (sphere_bvh.h build_triangle_accel: one leaf per (object, sub-object)
// pair of the reference's sweep, check_triangles, compute_shader.wgsl:422-517) walked from
// global memory costs one dependent 16-B node load per box test, and on C5 nearly every one
// of them misses the CU's L1 and waits for the L2 (~230 L2 requests per ray,
// the walk's bound). Here the same tree is collapsed 4-wide: a node is one 64-B record (half an
// L2 line) holding its four children's boxes and links, so one load tests four boxes and a walk
// makes about a quarter of the dependent loads.
//
//   box[k][0..2]  child k's box as 6 x 16-bit coordinates on the accelerator's quantization grid
//                 (tri_qnode.h: rounded outward, decoded exactly with one FMA): the box of the
//                 binary node the child stands for, so it contains that node's box;
//   ref[k]        kQ4Empty (no child), kQ4Leaf | leaf record (the binary leaf's prim index), or
//                 the index of another 4-wide node.
//
// Exactness: every child is a node of the binary tree and its box contains that node's box, so
// a ray reaches (with the same per-ray culling margin) every leaf the binary walk reaches, and
// the leaf tests are the same; the visiting order does not change the lexicographic (distance,
// sweep position) minimum. The boxes are rebuilt from the binary nodes on the
// device after every upload or refit of the accelerator (tri_q4_fill), like the 16-B copy.
//
// Shared by the host builder (rt_abi.cpp), the device fill kernel (scene_edit.hip), the walk
// (pathtrace.hip) and the CPU exactness harness (tests/cpp/tri_exactness.cpp).
#pragma once

#include <stdint.h>

#include "sphere_bvh.h"
#include "tri_qnode.h"

#if defined(__HIPCC__)
#define RT_Q4_FN __host__ __device__ inline
#else
#define RT_Q4_FN inline
#endif

struct TriQ4Node {
    uint32_t box[4][3];  // lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16 (tri_qnode's words 0-2)
    uint32_t ref[4];
};
static_assert(sizeof(TriQ4Node) == 64, "4-wide node = 64 B");

// Build switch: the 4-wide walk's code is compiled in only with -DRT_Q4=1 (its instructions and
// registers slowed the default binary walk even when switched off at run time: DESIGN.md §5.3e).
#ifndef RT_Q4
#define RT_Q4 0
#endif
constexpr bool kQ4Built = RT_Q4 != 0;

constexpr uint32_t kQ4Empty = 0xffffffffu;
constexpr uint32_t kQ4Leaf = 0x80000000u;
constexpr uint32_t kQ4MaxPrims = 1u << 20;  // leaf records a stack entry can name (larger scenes: binary walk)
// The walk's per-lane stack (LDS): entries a lane may hold; a push beyond it restarts that lane's
// walk on the binary accelerator (exact: a complete walk, merged into the same minimum).
constexpr uint32_t kQ4StackEntries = 16;
constexpr uint32_t kQ4None = 0xffffffffu;  // TraceState::node: no node loaded, pop the stack next
// The primary pre-pass's packet walk: a stack of {node, lane mask} per wave (LDS), 3 entries per
// level at most -- used for trees of depth <= kQ4PacketStack / 3 (deeper: the binary packet walk).
constexpr uint32_t kQ4PacketStack = 64;

// Stack entries: an internal node's index, or kQ4Leaf | prim (bits 0-19) | the 11-bit code of the
// leaf box's certified gap beyond the best hit when it was pushed (bits 20-30: the f32 bits >> 20,
// i.e. the gap truncated toward zero -- a lower bound, so the deferred certificate test stays
// sound; 0: no test). tri_leafcert_skips_gap accepts a gap measured against an earlier, larger
// best distance (tri_cone.h).
RT_Q4_FN uint32_t q4_gap_code(float gap) {
    if (!(gap > 0.0f)) return 0u;
    union {
        float f;
        uint32_t u;
    } v;
    v.f = gap;
    const uint32_t c = v.u >> 20;  // sign 0, exponent and the top 3 mantissa bits
    return c > 0x7ffu ? 0x7ffu : c;
}
RT_Q4_FN float q4_gap_decode(uint32_t code) {
    union {
        float f;
        uint32_t u;
    } v;
    v.u = code << 20;
    return v.f;
}

// ---- host side --------------------------------------------------------------------------
#include <vector>

// The 4-wide tree over a binary accelerator (DFS order, node + 1 = left child, right child =
// the left child's skip; leaves = prim | 1 << 24). `src[4 i + k]` receives the binary node child k
// of node i stands for (kQ4Empty: none); boxes are left to tri_q4_fill. Children of a node are
// opened from the binary tree by largest surface area, as tri_wide.cpp does. Returns false (and
// no tree) when a prim index does not fit a stack entry. `depth` receives the number of levels.
bool build_tri_q4(const std::vector<SphereBvhNode>& bin, std::vector<TriQ4Node>* nodes, std::vector<uint32_t>* src,
                  uint32_t* depth);

// Child k of a node from its binary node, on the grid (tri_qnode's encoding); an empty child
// gets the whole grid (its ref masks it out).
RT_Q4_FN void tri_q4_fill_child(TriQ4Node& nd, uint32_t k, const SphereBvhNode* bin, uint32_t src, const TriQGrid& g) {
    if (src == kQ4Empty) {
        nd.box[k][0] = 0u;
        nd.box[k][1] = 0xffff0000u;
        nd.box[k][2] = 0xffffffffu;
        return;
    }
    uint32_t w[4];
    tri_qnode(bin[src], g, w);
    nd.box[k][0] = w[0];
    nd.box[k][1] = w[1];
    nd.box[k][2] = w[2];
}
