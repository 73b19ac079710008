// rt_treelet.h -- the treelet wavefront's device state (treelet.hip), shared with the host
// (rt_abi.cpp dispatch_treelet) and the host-side treelet builder (sphere_bvh.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Top layouts: 8 direction-ordered pre-order layouts of the part of the triangle accelerator
// above the cut (as order_bvh_by_octant orders the whole tree), 2 float4 per node:
// {min.xyz, skip link}, {max.xyz, leaf word}. Leaf word: kTlInternal, a leaf record index (a leaf
// above the cut), or kTlTreelet | treelet id. A skip link past the layout is kTlEnd.
constexpr uint32_t kTlInternal = 0xffffffffu;
constexpr uint32_t kTlTreelet = 0x40000000u;
constexpr uint32_t kTlEnd = 0x7fffffffu;
constexpr uint32_t kTlNone = 0xffffffffu;
// Largest treelet (nodes of the base layout's pre-order range): its nodes, leaf records and
// leaf triangle blocks in one workgroup's LDS (<= 128 nodes, <= 64 leaves: 29 KB).
constexpr uint32_t kTreeletNodes = 128;
// Rays per work item of a round's treelet walks: a treelet's queue in chunks of this many.
constexpr uint32_t kTlChunk = 1024;

struct TreeletArgs {
    float4* paths;             // 4 planes x n_slots: o + seed, d + bounce, light, contribution
    uint4* walk;               // 2 planes x n_slots: best triangle, {resume position, treelet, rank, -}
    uint32_t* lists;           // walk lists A[2], shading lists R[2], treelet entries: 5 x n_slots slot ids
    uint32_t* ctl;             // list lengths: A[0], A[1], R[0], R[1]; [4]: the round's treelet chunks
    uint4* chunks;             // the round's work list: {treelet, first entry, rays, -}
    uint32_t* sub_cnt;         // per treelet: rays queued this round
    uint32_t* sub_off;         // per treelet: exclusive prefix of sub_cnt (n_sub + 1)
    const uint4* subtrees;     // per treelet: {base root, nodes, first leaf record, leaf records}
    const float4* top;         // the 8 top layouts (top_stride nodes each)
    const float4* base_nodes;  // the base accelerator (pre-order, 2 float4 per node)
    uint32_t top_stride;
    uint32_t n_slots;          // frames x samples x owned pixels of the batch
    uint32_t n_sub;            // treelets
    uint32_t round;            // the wavefront round (its parity selects the lists)
};
