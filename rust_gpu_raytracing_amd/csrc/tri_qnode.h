// tri_qnode.h -- the 16-B quantized copy of the binary triangle accelerator's nodes.
//
// A node of the binary accelerator (sphere_bvh.h SphereBvhNode) is 32 B: two 16-B loads per
// node visit, each its own L1 tag lookup for a lane walking its own path.
// The quantized node holds the same box as 6 x 16-bit grid coordinates rounded OUTWARD, and
// the link word, in 16 B. The grid is 2^k-spaced per axis with its origin on the grid, chosen
// so that origin + q * scale is an exact f32 for every q in [0, 65535]: the decoded box
// (fma(q, scale, origin), exact) contains the stored box, so the kernel's slab test on it
// passes whenever the test on the stored box passes (f32 rounding is monotone): culling stays
// exact. Link word: bit 31 set = leaf, bits 0-23 its record (the next node is always
// node + 1 in pre-order, except for the last leaf of a direction-ordered layout, which also
// carries kTriQLastLeaf: its walk ends there); clear = internal node, the word is its skip link.
// Shared by rt_quantize_tri_nodes_kernel (scene_edit.hip) and the CPU exactness harness.
#pragma once

#include <math.h>
#include <stdint.h>

#include "sphere_bvh.h"

#if defined(__HIPCC__)
#define RT_QN_FN __host__ __device__ inline
#else
#define RT_QN_FN inline
#endif

constexpr uint32_t kTriQLastLeaf = 0x40000000u;  // leaf link word: the walk ends after this leaf
constexpr uint32_t kTriWalkEnd = 0x7fffffffu;     // a node index past every layout

struct TriQGrid {
    float origin[3];
    float scale[3];
    bool valid;  // false: the root box is not finite (a sub-object with non-finite bounds), use 32-B nodes
};

// The grid from the root box alone (every device thread derives the same one).
RT_QN_FN TriQGrid tri_qgrid(const SphereBvhNode& root) {
    TriQGrid g{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, true};
    for (int k = 0; k < 3; k++) {
        const double lo = root.bmin[k], hi = root.bmax[k];
        if (!(lo >= -1.0e30 && hi <= 1.0e30 && lo <= hi)) {
            g.valid = false;
            return g;
        }
        const double amax = fmax(fabs(lo), fabs(hi));
        // scale >= extent / 65000 (q fits 16 bits with room), >= |coordinate| / 2^22 (origin /
        // scale + q stays under 2^24: exact in f32), and >= 2^-60
        const double need = fmax(fmax((hi - lo) / 65000.0, amax / 4194304.0), 8.673617379884035e-19);
        const double s = exp2(ceil(log2(need)));
        g.scale[k] = (float)s;
        g.origin[k] = (float)(floor(lo / s) * s);
    }
    return g;
}

// One node's quantized record: x = lo.x | lo.y << 16, y = lo.z | hi.x << 16, z = hi.y | hi.z << 16,
// w = the link word. A non-finite coordinate (a refit of NaN bounds below a finite root) takes
// the whole grid: the walk reaches the node only through the root's box, which the grid covers.
RT_QN_FN void tri_qnode(const SphereBvhNode& nd, const TriQGrid& g, uint32_t out[4]) {
    uint32_t lo[3], hi[3];
    for (int k = 0; k < 3; k++) {
        const double a = isfinite(nd.bmin[k]) ? floor(((double)nd.bmin[k] - g.origin[k]) / g.scale[k]) : 0.0;
        const double b = isfinite(nd.bmax[k]) ? ceil(((double)nd.bmax[k] - g.origin[k]) / g.scale[k]) : 65535.0;
        lo[k] = (uint32_t)fmin(fmax(a, 0.0), 65535.0);
        hi[k] = (uint32_t)fmin(fmax(b, 0.0), 65535.0);
        // the double arithmetic above can round a coordinate that tiny next to the origin onto
        // the grid point beside it: step outward until the decoded value (the kernel's exact
        // fma) contains the stored one
        if (isfinite(nd.bmin[k]))
            while (lo[k] > 0u && fmaf((float)lo[k], g.scale[k], g.origin[k]) > nd.bmin[k]) lo[k]--;
        if (isfinite(nd.bmax[k]))
            while (hi[k] < 65535u && fmaf((float)hi[k], g.scale[k], g.origin[k]) < nd.bmax[k]) hi[k]++;
    }
    out[0] = lo[0] | (lo[1] << 16);
    out[1] = lo[2] | (hi[0] << 16);
    out[2] = hi[1] | (hi[2] << 16);
    out[3] = nd.leaf != kSphereBvhInternal ? (0x80000000u | (nd.leaf & 0xffffffu)) : nd.skip;
}

// The decoded box, as the kernel computes it (node_step).
RT_QN_FN void tri_qnode_box(const uint32_t q[4], const TriQGrid& g, float lo[3], float hi[3]) {
    lo[0] = fmaf((float)(q[0] & 0xffffu), g.scale[0], g.origin[0]);
    lo[1] = fmaf((float)(q[0] >> 16), g.scale[1], g.origin[1]);
    lo[2] = fmaf((float)(q[1] & 0xffffu), g.scale[2], g.origin[2]);
    hi[0] = fmaf((float)(q[1] >> 16), g.scale[0], g.origin[0]);
    hi[1] = fmaf((float)(q[2] & 0xffffu), g.scale[1], g.origin[1]);
    hi[2] = fmaf((float)(q[2] >> 16), g.scale[2], g.origin[2]);
}
