// pathtrace.hip — the per-pixel path-tracing kernel for gfx950 (CDNA4).
//
// Replaces src/compute_shader.wgsl::main (:146-189) and everything it calls.
// Behaviour is the reference's, decision for decision (SURVEY.md §8a rows
// a6-a18); the numeric contract that makes it bit-exact against the CPU
// oracle is in rt_device_math.h. What is MI355X-specific:
//
//  * Work unit = one 8x8 pixel tile (the reference's workgroup, :146),
//    claimed by persistent wave64s from a device-wide queue; finished lanes
//    are refilled with the tile's next pixels (ballot/mbcnt compaction). Tiles are dealt to ranks
//    round-robin (tile t -> rank t % world) so a multi-GPU split is a launch
//    argument, not a different kernel; seeds depend only on the global pixel
//    index (:217), so any split is bitwise identical to one GPU.
//  * Scene staging: spheres (as centre + radius^2), materials and objects are
//    copied once per workgroup into LDS; every wave then sweeps the sphere and
//    object lists with wave-uniform indices (LDS broadcast reads, no bank
//    conflicts). Sub-objects and triangles are read from HBM/L2 with
//    wave-uniform addresses (scalar loads).
//  * Textures stay RGBA8 (4 B per fetch) and are decoded with a 256-entry
//    sRGB table in LDS, as the Rgba8UnormSrgb format does in hardware.
//  * Counted ray segments are summed per workgroup in LDS and added to one
//    64-bit device counter with a single atomic per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "rt_path_common.h"

// Analysis builds (tools/isa_loops.py, -DRT_ISA_MARKS) tag kernel regions with an
// assembly comment so the tool can find the loop around each; product builds emit nothing.
#ifdef RT_ISA_MARKS
#define RT_ISA_MARK(name) asm volatile("; RT_MARK " name)
#else
#define RT_ISA_MARK(name)
#endif

#pragma clang fp contract(off)

using namespace rtk;

namespace {

// Slab constants and depth bounds of a BVH walk. The triangle walk culls by
// box, and by distance when pruning is on (tri_limit), with no slack.
template <bool kTris>
__device__ __forceinline__ void phase_setup(const SceneView& sv, const KernelArgs& ka, f3 o, float a, uint32_t phase,
                                            TraceState& ts) {
    const float r = sqrt_up(dot(o, o));  // |o| sizes the margins only: an upper bound will do
    float m;
    if (phase == 0) {
        m = kTriMarginScale * (r + sv.tri_extent) + 1.0e-30f;
        ts.slack = 0.0f;
    } else {
        sphere_cull_bounds(r, ka.sphere_extent, ka.sphere_rmin, ka.sphere_rmax, __builtin_amdgcn_rsqf(a), m,
                           ts.slack);
    }
    ts.slab = slab_ray(o.x, o.y, o.z, ts.inv.x, ts.inv.y, ts.inv.z, m);
    ts.limit = phase == 0 ? __builtin_inff() : prune_limit(ts);
    if (kTris && phase == 0) {  // the accelerator layout ordered for this ray's direction octant (global walks)
        const uint32_t oct = (__float_as_uint(ts.inv.x) >> 31) | ((__float_as_uint(ts.inv.y) >> 31) << 1) |
                             ((__float_as_uint(ts.inv.z) >> 31) << 2);
        ts.node = oct * ka.tri_octant_stride;
    }
    if (phase == 1) {  // the sphere BVH layout ordered for this ray's direction octant (sphere_bvh.h)
        const uint32_t oct = (__float_as_uint(ts.inv.x) >> 31) | ((__float_as_uint(ts.inv.y) >> 31) << 1) |
                             ((__float_as_uint(ts.inv.z) >> 31) << 2);
        ts.node = oct * ka.sphere_octant_stride;
        // layouts storing (near, far) corners (sphere-only scenes, set by the host):
        // the plane constants paired the same way, so node_step can skip slab_hit's
        // min/max (rt_bvh_slab.h)
        if constexpr (!kTris)
            if (ka.sphere_boxes_ordered) slab_pair_by_octant(ts.slab);
    }
}

// kTris: the scene has objects (triangles); false compiles the triangle side out.
template <bool kTris>
__device__ __forceinline__ void trace_begin(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts) {
    if constexpr (kTris) {
        ts.inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);  // ray_in_bounds (:407-419) needs the IEEE quotient
    } else {
        // sphere-only scenes use 1/d only in the culling slab test, whose error
        // budget (rt_bvh_slab.h: 16u X for rounding, orders under the margin)
        // covers v_rcp_f32's 1 ulp; the sign (the layout octant) and +-inf for
        // a zero component are exact
        ts.inv = mk(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
    }
    const float a = dot(d, d);
    ts.a4 = 4.0f * a;
    ts.a2 = 2.0f * a;
    ts.sph = SphereHit{kF32Max, 0u, 0u};
    ts.tri = TriHit{kF32Max, 0u, 0u, 0u, false};
    ts.nan_hit = false;
    ts.node = 0;
    ts.pending = kNoLeaf;
    // brute-force sphere set: wave-uniform sweep over groups of 4, then the rest
    // one by one (a sphere's own test is exact, so the visiting order is free)
    // (the slots after the set up to the next group boundary are NaN padding:
    // a remainder of 2-3 spheres takes one group, a lone sphere a single test)
    uint32_t i = 0;
    for (; i + 4u <= ka.sphere_always; i += 4u) test_sphere_group(sv, i, o, d, ts.a4, ts.a2, ts.sph);
    if (ka.sphere_always - i >= 2u) {
        test_sphere_group(sv, i, o, d, ts.a4, ts.a2, ts.sph);
    } else if (ka.sphere_always - i == 1u) {
        float b;
        const float disc = sphere_disc(sv.sph[i], o, d, ts.a4, b);
        sphere_candidate(disc, b, ts.a2, sv.orig[i], i, ts.sph);
    }
    if constexpr (!kTris) {
        ts.phase = 1;
    } else if (!ka.tri_accel) {
        ts.tri = sweep_triangles(sv, ka, o, d);
        ts.phase = 1;
    } else {
        ts.phase = ka.tri_nodes != 0 ? 0u : 1u;
    }
    if (ts.phase == 1 && ka.sphere_nodes == 0) ts.phase = 2;
    phase_setup<kTris>(sv, ka, o, a, ts.phase, ts);
}

// The lane's index in its wave, computed where it is used: an opaque value, so that the compiler
// does not hoist it (and what is derived from it) out of the traversal loop into a register
// held across every node step.
__device__ __forceinline__ uint32_t lane_id_here() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Ends the current BVH walk once its nodes are exhausted and no leaf is pending.
template <bool kTris>
__device__ __forceinline__ void phase_end(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts) {
    if (ts.pending != kNoLeaf) return;
    if (kTris && ts.phase == 0) {
        if (ts.node < ka.tri_nodes) return;
#ifdef RT_DIAG_TAIL
        if (ts.nan_hit) atomicAdd(ka.diag + 6, 1ull);
#endif
        if (ts.nan_hit) ts.tri = sweep_triangles(sv, ka, o, d);  // measure-zero case: the sweep decides
        ts.node = 0;
        ts.phase = ka.sphere_nodes != 0 ? 1u : 2u;
        phase_setup<kTris>(sv, ka, o, ts.a2 * 0.5f, 1, ts);
    } else if (ts.node >= ka.sphere_nodes) {
        ts.phase = 2;
    }
}

// Advances the walk by one BVH node. A reached leaf is not tested here but
// deferred (ts.pending) and the walk goes on past it: the wave tests leaves in
// batches (leaf_step), so the leaf body -- two box tests and up to 7 triangle
// tests with their global loads, or a sphere group -- runs for many lanes at
// once instead of for the few lanes that sit on a leaf in a given step. A lane
// that reaches a second leaf while one is deferred stays on it until the batch.
// Testing a leaf late only delays the pruning distance it would set: the result
// is the lexicographic minimum over the tested primitives either way.
template <bool kTris>
constexpr bool kDeferLeaves = kTris;
// Sphere-only scenes: a lane that reaches a leaf stops walking, and the group tests of the lanes
// waiting at a leaf run together after a block of the wave's unrolled node steps (kTravUnroll),
// once at least kBlockLeafShare eighths of the traversing lanes wait, instead of inside each node
// step for the few lanes at a leaf in that step. The lane resumes with its pruning distance
// updated, so it visits the nodes the on-the-spot test would, in the same order (C2 0.2820 ->
// 0.2481 ms per frame in one process; walking on past the leaf until a second one was slower;
// DESIGN §5.2).
template <bool kTris>
constexpr bool kBlockLeaves = !kTris;
constexpr uint32_t kBlockLeafShare = 3;
// Node steps per wave-wide check of the traversal loop (the ballots of the
// threshold and leaf-batch tests, exec-mask updates). Lanes that finish inside
// the group idle for its remaining steps; the visit order is unchanged.
// Measured (1 -> 3): C2 -2.8%, C3 -10%, C4 -11%, C5 -7%. Round 4, per accelerator placement
// (profiles/r04/r04_z): global-memory walks 3 -> 4 / 5 / 6: C5 -4.0% / -4.3% / -1.6%;
// LDS-resident walks 3 -> 2: C3 -1.2%, C4 (4K) +0.5%. Sphere walks, with the block group tests
// (round 6, profiles/r06/r06l, r06o, r06p): blocks of 4 with the tests once 3/8 of the lanes wait,
// C2 0.2481 ms per frame; 3 / 5 / 6 steps 0.2522 / 0.2503 / 0.2503; every block tested (no
// share) at 3 / 4 / 6 / 8 / 12 steps 0.2675 / 0.2580 / 0.2575 / 0.2614 / 0.2658.
template <int kMode, bool kTris>
constexpr int kTravUnroll = !kTris ? 4 : kMode <= 1 ? 5 : 3;
// Triangle walks: the leaf batch runs after the block's node steps in the same iteration (round 6)
// instead of in an iteration of its own in which the walking lanes idle: the LDS-resident walk
// (mode 2, C3 0.2645 -> 0.2463, C4 1.539 -> 1.416 ms per frame in one process with blocks of 3
// steps; 2 / 4 / 5 steps: C3 0.2492 / 0.2478 / 0.2527, C4 1.460 / 1.413 / 1.437; shares of
// 5/8-8/8 around the default 6/8 no better; profiles/r06/r06r-r06t).
// The walks from global memory keep their batches apart: fusing the cooperative batch the same
// way measured C5 +2.3% (profiles/r06/r06u).
template <int kMode, bool kTris>
constexpr bool kFusedLeaves = kTris && kMode == 2;

// Decoupled drain (see the kernel's step 4): triangle scenes whose accelerator
// is read from global memory (LDS modes 0 and 1).
template <int kMode, bool kTris>
constexpr bool kDrainDecouple = kTris && kMode < 2;

// Walks that read leaf certificates: from global memory only (see tri_leaf).
template <int kMode>
constexpr bool kCertWalk = kMode <= 1;

// A 16-B quantized node decoded (tri_qnode.h): the box exactly (a superset of the 32-B node's
// box), lo.w = the skip link (a leaf's: node + 1, or the end), hi.w = the leaf record or none.
__device__ __forceinline__ void qnode_decode(const SceneView& sv, uint4 q, uint32_t node, float4& lo, float4& hi) {
    lo = make_float4(fmaf((float)(q.x & 0xffffu), sv.qsx, sv.qox), fmaf((float)(q.x >> 16), sv.qsy, sv.qoy),
                     fmaf((float)(q.y & 0xffffu), sv.qsz, sv.qoz), 0.0f);
    hi = make_float4(fmaf((float)(q.y >> 16), sv.qsx, sv.qox), fmaf((float)(q.z & 0xffffu), sv.qsy, sv.qoy),
                     fmaf((float)(q.z >> 16), sv.qsz, sv.qoz), 0.0f);
    const bool is_leaf = (q.w & 0x80000000u) != 0u;
    // a leaf's skip link is node + 1 (pre-order), or the end for a layout's last leaf
    lo.w = __uint_as_float(is_leaf ? ((q.w & kTriQLastLeaf) ? kTriWalkEnd : node + 1u) : q.w);
    hi.w = __uint_as_float(is_leaf ? (q.w & 0xffffffu) : 0xffffffffu);
}

// One node's visit, given its box and links: the box test, the deferred leaf or the sphere
// group, the next node.
template <bool kTris, bool kCert>
__device__ __forceinline__ void node_visit(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts,
                                           bool tri, float4 lo, float4 hi) {
    float near_t, far_t;
    if (!kTris && ka.sphere_boxes_ordered)  // (near, far) corners: no min/max per axis (6 VALU per node step)
        slab_hit_ordered(ts.slab, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, near_t, far_t);
    else
        slab_hit(ts.slab, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, near_t, far_t);
    // enters the inflated box and is not wholly behind the origin; on the sphere
    // side also not beyond the best sphere or the triangle hit (a sphere wins
    // only when strictly closer, :347); ts.slack / ts.limit are 0 / inf on the
    // triangle side
    const bool hit = near_t <= far_t && far_t >= -ts.slack && near_t <= ts.limit;
    const uint32_t leaf = __float_as_uint(hi.w);
    uint32_t skip = 0u;
    if constexpr (kTris && kCert) {
        // certified pruning: a leaf whose box is entered beyond the best triangle hit records
        // the gap of its box beyond that hit, for the leaf batch's certificate test
        if (tri && hit && leaf != 0xffffffffu && ka.tri_leafcert && near_t > ts.tri.t && ts.tri.t != kF32Max &&
            ts.pending == kNoLeaf) {
            const float tbs = ts.tri.t * (1.0f + 0x1p-20f);
            const SlabRay& sr = ts.slab;
            const float gx = (fminf(fmaf(lo.x, sr.ix, sr.lx), fmaf(hi.x, sr.ix, sr.hx)) - tbs) * fabsf(d.x);
            const float gy = (fminf(fmaf(lo.y, sr.iy, sr.ly), fmaf(hi.y, sr.iy, sr.hy)) - tbs) * fabsf(d.y);
            const float gz = (fminf(fmaf(lo.z, sr.iz, sr.lz), fmaf(hi.z, sr.iz, sr.hz)) - tbs) * fabsf(d.z);
            ts.cert_gap = fmaxf(fmaxf(gx, gy), gz) * (1.0f - 0x1p-20f);
            skip = ts.cert_gap > 0.0f ? 1u : 0u;  // (bit 24 of pending: test deferred)
        }
    }
    const bool at_leaf = hit && leaf != 0xffffffffu;
#ifdef RT_DIAG
    if constexpr (!kDeferLeaves<kTris>) {  // node steps and the sphere-group tests inside them, with their lanes
        const uint64_t act = __ballot(true), lf = __ballot(at_leaf);
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(act)) {
            atomicAdd(ka.diag + 22, 1ull);
            atomicAdd(ka.diag + 23, (unsigned long long)__popcll(act));
            if (lf) {
                atomicAdd(ka.diag + 24, 1ull);
                atomicAdd(ka.diag + 25, (unsigned long long)__popcll(lf));
            }
        }
    }
#endif
    if (at_leaf && !kDeferLeaves<kTris> && !kBlockLeaves<kTris>) {
        test_sphere_group(sv, leaf & 0xffffffu, o, d, ts.a4, ts.a2, ts.sph);
        ts.limit = prune_limit(ts);
    } else if (at_leaf) {
        if (ts.pending != kNoLeaf) return;  // blocked until the batch tests the deferred leaf
        ts.pending = (leaf & 0xffffffu) | (skip << 24);
    }
    ts.node = (hit && !at_leaf) ? ts.node + 1u : __float_as_uint(lo.w);
}

// kCert: the walk records leaf-certificate gaps (node_visit) when ka.tri_leafcert is set.
template <bool kTris, bool kCert = true>
__device__ __forceinline__ void node_step(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts) {
    const bool tri = kTris && ts.phase == 0;
    if (kDeferLeaves<kTris> && ts.node >= (tri ? ka.tri_nodes : ka.sphere_nodes))
        return;  // walk over, a leaf still deferred
    if (kBlockLeaves<kTris> && ts.pending != kNoLeaf) return;  // waits for the block's group tests
    float4 lo, hi;
    if (kTris && tri && sv.tri_q) {
        qnode_decode(sv, sv.tri_q[ts.node], ts.node, lo, hi);
    } else {
        const float4* nodes = tri ? sv.tri_nodes : sv.nodes;
        lo = nodes[2u * ts.node];
        hi = nodes[2u * ts.node + 1u];
    }
    node_visit<kTris, kCert>(sv, ka, o, d, ts, tri, lo, hi);
}

template <bool kTris, bool kLazySub = false>
__device__ __forceinline__ void leaf_step(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts) {
    if (kTris && ts.phase == 0) {
        tri_leaf<kLazySub>(sv, ka, o, d, ts, ts.pending);
        ts.limit = tri_limit(sv, ka, o, ts);
    } else {
        test_sphere_group(sv, ts.pending, o, d, ts.a4, ts.a2, ts.sph);
        ts.limit = prune_limit(ts);
    }
    ts.pending = kNoLeaf;
}

// ---- Cooperative leaf batches (walks from global memory) --------------------
//
// A per-lane leaf test loads its up-to-7 triangles with three lane-distinct 16-B loads each:
// 21 L1 tag lookups per leaf, and the L1's tag rate (about one line per cycle per CU) is what
// the global-memory walk is bound by. Here a leaf batch tests the wave's
// pending leaves together instead: the pending lanes publish their ray and leaf in a per-wave
// LDS scratch, and each round 8 lanes per leaf -- lane j the leaf's triangle j -- load the
// leaf's triangle block (KernelArgs::tri_leaftris: piece p of slots 0..7 in one 128-B line),
// so the 21 loads become 3 lines shared by 8 lanes, and 8 leaves are tested per round on all
// 64 lanes. Each lane runs the reference's test (compute_shader.wgsl:445-500) with the same
// f32 operations as tri_leaf; the group's candidates are reduced to the lexicographic minimum
// of (distance, sweep position) and an "any NaN distance" flag, which the leaf's lane then
// merges exactly as tri_leaf's sequential loop would: the sub-object box test (:441) runs if a
// candidate beats the lane's best hit or has a NaN distance; if it fails, nothing of the leaf
// counts; else the NaN flag and the best candidate are taken. (Within a leaf the sequential
// loop's result is that minimum: a candidate's test does not depend on the running best other
// than through "distance < best", which is the minimum's own comparison.)
template <int kMode, bool kTris>
constexpr bool kCoopLeaves = kTris && kMode <= 1;

// LDS written by some lanes of a wave and read by others: the wave's LDS operations complete in
// order, so only the compiler must not move them across this point.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One step of the 8-lane (distance, sequence) minimum: the candidate of lane (DPP `ctrl`).
template <int kCtrl>
__device__ __forceinline__ void coop_min_step(float& cd, uint32_t& cs, uint32_t& ct) {
    const float od = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(cd), kCtrl, 0xf, 0xf, false));
    const uint32_t os = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cs, kCtrl, 0xf, 0xf, false);
    const uint32_t ot = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ct, kCtrl, 0xf, 0xf, false);
    const bool take = od < cd || (od == cd && os < cs);
    cd = take ? od : cd;
    cs = take ? os : cs;
    ct = take ? ot : ct;
}

// `active`: this lane traverses and holds a deferred leaf (a triangle leaf, or a sphere group in
// the sphere phase, which is tested on the spot as in leaf_step). Wave-uniform call; the scratch
// is this wave's 64 x 3 float4 of LDS at ka.lds_leafbatch_offset.
__device__ __forceinline__ void coop_leaf_batch(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts,
                                                bool active, unsigned char* lds) {
    bool want = false;
    uint32_t prim = 0u, range = 0u, seq0 = 0u, obj = 0u, sub = 0u;
    if (active) {
        if (ts.phase == 0) {
            prim = ts.pending & 0xffffffu;
            uint32_t skip = 0u;
            if ((ts.pending >> 24) & 1u) {  // the certificate test deferred by node_step
                const uint4* rec = reinterpret_cast<const uint4*>(ka.tri_leafcert + prim);
                const uint4 c0 = rec[0], c1 = rec[1];
                const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                skip = tri_leafcert_skips_gap(w, tri_cone_ray(o.x, o.y, o.z, d.x, d.y, d.z), ts.tri.t, ts.cert_gap);
            }
            if (skip != kLeafCertAll) {
                const uint4 pr = sv.tri_prims[prim];  // object, sub, seq_base, range
                const RtObject& ob = sv.obj[pr.x];
                if (ray_in_bounds(o, ts.inv, ob.min_bounds, ob.max_bounds)) {  // :431
                    if (pr.w != kPrimRangeNone && (pr.w >> 27) < kLeafTriSlots) {
                        want = true;
                        range = pr.w;
                        seq0 = pr.z;
                        obj = pr.x;
                        sub = pr.y;
                    } else {  // a leaf of more than 7 triangles: the per-lane test (no certificate mask)
                        tri_leaf<true>(sv, ka, o, d, ts, prim);
                        ts.limit = tri_limit(sv, ka, o, ts);
                    }
                }
            }
        } else {
            test_sphere_group(sv, ts.pending, o, d, ts.a4, ts.a2, ts.sph);
            ts.limit = prune_limit(ts);
        }
        ts.pending = kNoLeaf;
    }
    const uint64_t wm = __ballot(want);
    if (wm == 0) return;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4* const scratch = reinterpret_cast<float4*>(lds + ka.lds_leafbatch_offset + wave * kLeafBatchWaveBytes);
    const uint32_t n = (uint32_t)__popcll(wm);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
    if (want) {
        float4* sl = scratch + 3u * rank;
        sl[0] = make_float4(o.x, o.y, o.z, __uint_as_float(prim));
        sl[1] = make_float4(d.x, d.y, d.z, __uint_as_float(range));
        sl[2] = make_float4(__uint_as_float(seq0), __uint_as_float(obj), __uint_as_float(sub), 0.0f);
    }
    wave_lds_sync();
    const uint32_t lane = lane_id_here(), g = lane >> 3, j = lane & 7u;
    for (uint32_t base = 0; base < n; base += 8u) {
        const uint32_t kk = base + g;
        float cd = __builtin_inff();  // no candidate: never accepted (a distance is always < inf there)
        uint32_t cs = 0xffffffffu, ct = 0u;
        bool cnan = false;
        if (kk < n) {
            const float4* sl = scratch + 3u * kk;
            const float4 s0 = sl[0], s1 = sl[1];
            const uint32_t rg = __float_as_uint(s1.w);
            if (j < (rg >> 27)) {
                const uint4* blk = ka.tri_leaftris + (size_t)__float_as_uint(s0.w) * kLeafTriWords + j;
                const uint4 q0 = blk[0], q1 = blk[kLeafTriSlots], q2 = blk[2u * kLeafTriSlots];
                const float4 p0 = make_float4(__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z),
                                              __uint_as_float(q0.w));
                const float4 p1 = make_float4(__uint_as_float(q1.x), __uint_as_float(q1.y), __uint_as_float(q1.z),
                                              __uint_as_float(q1.w));
                const float4 p2 = make_float4(__uint_as_float(q2.x), __uint_as_float(q2.y), __uint_as_float(q2.z),
                                              __uint_as_float(q2.w));
                const TriGeom tg{mk(p0.x, p0.y, p0.z), mk(p0.w, p1.x, p1.y), mk(p1.z, p1.w, p2.x),
                                 mk(p2.y, p2.z, p2.w)};
                const f3 ro = mk(s0.x, s0.y, s0.z), rd = mk(s1.x, s1.y, s1.z);
                // the reference's test, tri_leaf's operations (:449-481)
                const float det = -dot(rd, tg.cn);
                const float inv_det = 1.0f / det;
                const f3 ao = ro - tg.a;
                const float dist = dot(ao, tg.cn) * inv_det;
                const f3 dao = cross(ao, rd);
                const float v = -dot(tg.ab, dao) * inv_det;
                const float u = dot(tg.ac, dao) * inv_det;
                const float w = 1.0f - u - v;
                if (!(dist < 0.0f) && !(v < 0.0f) && !(u < 0.0f) && !(w < 0.0f)) {
                    if (dist != dist) {
                        cnan = true;
                    } else {
                        cd = dist;
                        cs = __float_as_uint(sl[2].x) + j;
                        ct = min((rg & ((1u << 27) - 1u)) + j, ka.triangle_count - 1u) | (det > 0.0f ? 0x80000000u : 0u);
                    }
                }
            }
        }
        // the group's minimum on every lane of it: xor 1, xor 2 (quad), then the other quad
        coop_min_step<0xB1>(cd, cs, ct);
        coop_min_step<0x4E>(cd, cs, ct);
        coop_min_step<0x141>(cd, cs, ct);
        const uint64_t nm = __ballot(cnan);
        if (j == 0u && kk < n)  // slot kk's ray is no longer needed: its result goes there
            scratch[3u * kk] = make_float4(cd, __uint_as_float(cs), __uint_as_float(ct),
                                           __uint_as_float(((nm >> (8u * g)) & 0xffu) != 0u ? 1u : 0u));
    }
    wave_lds_sync();
    if (want) {
        const float4 r = scratch[3u * rank];
        const float4 r2 = scratch[3u * rank + 2u];
        obj = __float_as_uint(r2.y);
        sub = __float_as_uint(r2.z);
        const float rd = r.x;
        const uint32_t rs = __float_as_uint(r.y), rt = __float_as_uint(r.z);
        const bool rnan = __float_as_uint(r.w) != 0u;
        const bool beats = rd < ts.tri.t || (rd == ts.tri.t && rs < ts.tri.seq);
        if (rnan || beats) {
            const RtSubObject so = sv.sub[sub];  // :441, run when the leaf would change the result
            if (ray_in_bounds(o, ts.inv, so.min_bounds, so.max_bounds)) {
                if (rnan) ts.nan_hit = true;
                if (beats) ts.tri = TriHit{rd, rs, rt & 0x7fffffffu, obj, (rt >> 31) != 0u};
            }
        }
        ts.limit = tri_limit(sv, ka, o, ts);
    }
}

}  // namespace

constexpr uint32_t kPrimaryThreads = 1024;  // default: 16 units per workgroup, sharing one LDS image of the scene

// The tile queue, striped over the XCDs. One device-scope atomic counter on a
// single address serialises at the memory side (~15 ns per claim measured:
// that alone capped C1 at 4x below a static schedule). Local tile t belongs to
// stripe t % S (S = 32 by default, 4 per XCD, counters 256 B apart); a wave claims from
// a stripe of its own XCD (HW_REG_XCC_ID), and once that is empty steals from the
// others, checking each with a coherent load before spending an atomic on it.
// Claims stay dynamic, so expensive tiles still balance across waves. The
// counters start at zero: each launch zeroes the other half of the
// double-buffered counter array for the next launch (stream order makes that
// visible). Lane 0 does the memory operations; results are wave-uniform.
constexpr uint32_t kQueueStride = 64;  // u32 between stripe counters (256 B)

// The cost-ordered schedule's device state (KernelArgs::sched).
__device__ __forceinline__ uint32_t* sched_orders(const KernelArgs& ka) { return ka.sched + 2u * ka.owned_tiles; }
__device__ __forceinline__ uint32_t* sched_flags(const KernelArgs& ka) { return ka.sched + 4u * ka.owned_tiles; }

__device__ __forceinline__ uint32_t xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
}

struct TileQueue {
    uint32_t stripe;  // stripe being drained (wave-uniform): the home stripe, then the last one stolen from
    uint32_t empty;   // every stripe was found drained
};

// Returns the claimed queue position in [0, queue_units), or 0xffffffff when
// the queue is empty (unit_tile maps a position to its tile and frame). Stripe
// s holds the positions k * n_str + s; its counter is the next k. One atomic
// on the current stripe; once that is drained, the wave reads every stripe's
// counter at once (lane i the i-th stripe after the current one, one load
// instruction) and claims from the first that has work left, so finding the
// queue empty costs one round trip instead of a walk over the stripes one
// dependent load at a time (up to 31 of them, with the whole wave waiting, when
// the stripes run dry together at the end of a launch).
__device__ __forceinline__ uint32_t claim_tile(const KernelArgs& ka, TileQueue& q) {
    const uint32_t n_str = ka.queue_stripes;
    const uint32_t lane = threadIdx.x & 63u;
    if (q.empty) return 0xffffffffu;
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(ka.queue + q.stripe * kQueueStride, 1u);
    uint64_t pos = (uint64_t)__builtin_amdgcn_readlane(old, 0) * n_str + q.stripe;
    if (pos < ka.queue_units) return (uint32_t)pos;
    while (true) {
        bool open = false;
        if (lane < n_str) {
            uint32_t st = q.stripe + 1u + lane;
            st = st >= n_str ? st - n_str : st;
            const uint32_t v = __hip_atomic_load(ka.queue + st * kQueueStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            open = (uint64_t)v * n_str + st < ka.queue_units;
        }
        const uint64_t m = __ballot(open);
        if (m == 0) {
            q.empty = 1u;
            return 0xffffffffu;
        }
        uint32_t st = q.stripe + 1u + (uint32_t)__builtin_ctzll(m);
        q.stripe = st >= n_str ? st - n_str : st;
        if (lane == 0) old = atomicAdd(ka.queue + q.stripe * kQueueStride, 1u);
        pos = (uint64_t)__builtin_amdgcn_readlane(old, 0) * n_str + q.stripe;
        if (pos < ka.queue_units) return (uint32_t)pos;
    }
}

// Queue position -> local tile (identity unless cost-ordered) and, in a
// frame-parallel batch, the frame: frame-major positions (a cost-ordered launch
// then ends on the last frame's cheapest tiles) or tile-major (a tile's frames
// are claimed one after another: the same camera rays, near-identical primary
// walks). 0xffffffff (empty queue) stays so.
__device__ __forceinline__ uint32_t unit_tile(const KernelArgs& ka, uint32_t pos, uint32_t& frame) {
    if (pos == 0xffffffffu) return pos;
    uint32_t q;
    if (!ka.frame_light) {
        frame = 0u;
        q = pos;
    } else if (ka.unit_tile_major) {
        q = pos / ka.frames;
        frame = pos - q * ka.frames;
    } else {
        frame = pos / ka.owned_tiles;
        q = pos - frame * ka.owned_tiles;
    }
    return ka.tile_order ? ka.tile_order[q] : q;
}

// Cost-ordered schedule support: adds the rays of the pixels this wave just
// finished to their tiles' counters. Finished lanes almost always share one or
// two tiles, so this is one wave reduction and one atomic per distinct tile.
__device__ __forceinline__ void record_tile_cost(uint32_t* cost, bool fin, uint32_t tile, uint32_t n) {
    uint64_t m = __ballot(fin);
    while (m) {
        const uint32_t t = __builtin_amdgcn_readlane(tile, (uint32_t)__builtin_ctzll(m));
        const bool mine = fin && tile == t;
        uint32_t v = mine ? n : 0u;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63u) == 0) atomicAdd(cost + t, v);
        m &= ~__ballot(mine);
    }
}

// The cost-ordered schedule's sort: the tiles of one launch ordered by the
// rays they took, most expensive first, for a later launch to claim in that
// order, so that launches end on cheap tiles (sky) instead of on the long paths
// of expensive ones (paths progress one bounce per wave iteration, so the
// paths in flight when the queue runs dry decide how long the last waves run
// on nearly empty lanes). A stable counting sort into kOrderBuckets buckets
// between 0 and the largest cost. No atomics on shared counters: each wave
// counts its tiles per bucket with ballots, a scan over (bucket, wave) gives
// every wave its slots, and the wave scatters in tile order -- so the result
// is deterministic (and any order renders the same image: pixels are
// independent). No costs recorded: tile index order. Zeroes the costs for
// their next recording. Run by one whole workgroup; `scratch` holds
// kOrderBuckets * 16 + 1 words of LDS (kLdsTailBytes, rt_kernel_args.h).

template <uint32_t kThreads>
__device__ void sort_tiles_by_cost(uint32_t* __restrict__ cost, uint32_t* __restrict__ order, uint32_t n,
                                   uint32_t* scratch) {
    constexpr uint32_t kWaves = kThreads / 64;
    static_assert(kWaves <= 16 && kOrderBuckets * kWaves <= kThreads, "scratch layout / one scan entry per thread");
    uint32_t* slots = scratch;                       // [bucket][wave]: counts, then first slot
    uint32_t* max_cost = scratch + kOrderBuckets * 16;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    if (tid == 0) *max_cost = 0;
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t i = tid; i < n; i += kThreads) m = max(m, cost[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor(m, o));
    if (lane == 0) atomicMax(max_cost, m);
    __syncthreads();
    const uint32_t mx = *max_cost;
    if (mx == 0) {
        for (uint32_t i = tid; i < n; i += kThreads) order[i] = i;
        return;
    }
    const uint64_t mc = (uint64_t)mx + 1u;
    // each wave takes one contiguous range of tiles, 64 per round, so the
    // (bucket, wave) slot order makes the sort stable
    const uint32_t span = ((n + kWaves - 1u) / kWaves + 63u) & ~63u;
    const uint32_t lo = min(n, wave * span), hi = min(n, lo + span);
    auto key = [&](uint32_t i) {  // kOrderBuckets for no tile
        return i < hi ? kOrderBuckets - 1u - (uint32_t)(((uint64_t)cost[i] * kOrderBuckets) / mc) : kOrderBuckets;
    };
    uint32_t cnt = 0;  // lane b < kOrderBuckets: this wave's tiles in bucket b
    for (uint32_t base = lo; base < hi; base += 64u) {
        const uint32_t k = key(base + lane);
        for (uint32_t b = 0; b < kOrderBuckets; ++b) {
            const uint32_t c = (uint32_t)__popcll(__ballot(k == b));
            if (lane == b) cnt += c;
        }
    }
    if (lane < kOrderBuckets) slots[lane * kWaves + wave] = cnt;
    __syncthreads();
    // exclusive scan over (bucket, wave), bucket-major (Hillis-Steele)
    constexpr uint32_t kEntries = kOrderBuckets * kWaves;
    uint32_t v = tid < kEntries ? slots[tid] : 0u;
    const uint32_t own = v;
    for (uint32_t off = 1; off < kEntries; off <<= 1) {
        __syncthreads();
        const uint32_t add = (tid < kEntries && tid >= off) ? slots[tid - off] : 0u;
        __syncthreads();
        v += add;
        if (tid < kEntries) slots[tid] = v;
    }
    __syncthreads();
    if (tid < kEntries) slots[tid] = v - own;
    __syncthreads();
    uint32_t next = lane < kOrderBuckets ? slots[lane * kWaves + wave] : 0u;  // lane b: next slot of bucket b
    for (uint32_t base = lo; base < hi; base += 64u) {
        const uint32_t i = base + lane;
        const uint32_t k = key(i);
        uint32_t pos = 0;
        for (uint32_t b = 0; b < kOrderBuckets; ++b) {
            const uint64_t mb = __ballot(k == b);
            const uint32_t first = __builtin_amdgcn_readlane(next, b);
            if (k == b) pos = first + __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
            if (lane == b) next += (uint32_t)__popcll(mb);
        }
        if (i < hi) {
            order[pos] = i;
            cost[i] = 0;
        }
    }
}

#ifdef RT_DIAG_TAIL
// Diagnostic build only: wave start/end times (s_memrealtime, 100 MHz, one
// clock for the whole device) -> ramp and tail of the persistent grid.
__device__ __forceinline__ unsigned long long realtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#endif

#ifdef RT_DIAG
// Diagnostic build only: wave-level cycle stamps (s_memtime) accumulated per
// wave and added to ka.diag at exit. Never compiled into the product build.
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#endif

// Dynamic LDS image, in this order (all 16-byte aligned):
//   float4   sphere slots[sphere_count]   centre.xyz, radius^2
//   RtMaterial materials[material_count]
//   RtObject objects[object_count]
//   uint32   slot -> original index[sphere_count]
//   uint32   sphere material[sphere_count] (by original index)
//   float4x2 sphere BVH nodes[sphere_nodes]
//   float4x2 triangle accelerator nodes[tri_nodes]      (mode 2)
//   uint4    triangle accelerator leaves[tri_prims]     (mode 2)
//   float    srgb[256]
// kMode 0 keeps the scene in global memory (scenes beyond the LDS budget),
// 1 stages spheres/materials/objects/sphere BVH, 2 also the triangle
// accelerator; the sRGB table is always staged.
//
// Persistent waves with in-wave path regeneration (the "ray compaction across
// bounces"): each wave claims 8x8 tiles from a device-wide queue and keeps all
// 64 lanes busy — whenever lanes' paths finish, __ballot + mbcnt (a wave-wide
// prefix sum) hand those lanes the next pixels of the current tile, so a
// wave never idles behind one long path while work remains. A pixel's samples
// (compute_per_frame) run back to back on one lane, so the accumulation is
// summed in the reference's order (:160-163) and results are bit-identical.
template <int kMode, uint32_t kThreads, bool kTris>
__global__ void __launch_bounds__(kThreads, 1) rt_pathtrace_kernel(KernelArgs ka) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t block_rays;

    const uint32_t tid = threadIdx.x;
    if (ka.launch_clock && tid == 0) atomicMax(ka.launch_clock, ~(unsigned long long)wall_clock64());
    float* l_srgb = reinterpret_cast<float*>(lds + ka.lds_srgb_offset);
    SceneView sv{ka.sphere_slots, ka.sphere_orig, ka.sphere_material, ka.sphere_bvh, ka.materials, nullptr,
                 ka.objects,      l_srgb,         ka.tri_bvh,     ka.tri_prims, kTris ? *ka.tri_extent : 0.0f,
                 ka.sub_objects};
    if constexpr (kTris && kMode <= 1) {
        if (ka.tri_qnodes) {
            const float4 g0 = ka.tri_qgrid[0], g1 = ka.tri_qgrid[1];
            if (g0.w != 0.0f) {
                sv.tri_q = ka.tri_qnodes;
                sv.qox = g0.x;
                sv.qoy = g0.y;
                sv.qoz = g0.z;
                sv.qsx = g1.x;
                sv.qsy = g1.y;
                sv.qsz = g1.z;
            }
        }
    }
    if (tid == 0) block_rays = 0;
    if constexpr (kMode >= 1) {
        float4* l_sph = reinterpret_cast<float4*>(lds);
        RtMaterial* l_mat = reinterpret_cast<RtMaterial*>(lds + ka.lds_mat_offset);
        RtObject* l_obj = reinterpret_cast<RtObject*>(lds + ka.lds_obj_offset);
        uint32_t* l_orig = reinterpret_cast<uint32_t*>(lds + ka.lds_orig_offset);
        uint32_t* l_smat = reinterpret_cast<uint32_t*>(lds + ka.lds_smat_offset);
        float4* l_nodes = reinterpret_cast<float4*>(lds + ka.lds_nodes_offset);
        for (uint32_t i = tid; i < ka.sphere_slot_count; i += kThreads) {
            l_sph[i] = ka.sphere_slots[i];
            l_orig[i] = ka.sphere_orig[i];
        }
        for (uint32_t i = tid; i < ka.sphere_count; i += kThreads) l_smat[i] = ka.sphere_material[i];
        for (uint32_t i = tid; i < 2u * ka.sphere_nodes; i += kThreads) l_nodes[i] = ka.sphere_bvh[i];
        float4* l_aux = reinterpret_cast<float4*>(lds + ka.lds_mat_aux_offset);
        for (uint32_t i = tid; i < ka.material_count; i += kThreads) {
            const RtMaterial m = ka.materials[i];
            l_mat[i] = m;
            // shade()'s glass constants, by the same f32 operations (:320, :328-334, :307)
            const float ior_front = 1.0f / m.refraction_index;
            float r0f = (1.0f - ior_front) / (1.0f + ior_front);
            float r0b = (1.0f - m.refraction_index) / (1.0f + m.refraction_index);
            r0f = r0f * r0f;
            r0b = r0b * r0b;
            l_aux[2u * i] = make_float4(ior_front, r0f, r0b, div_const(m.roughness, 10.0f, kInv10));
            // the decoded texel a 1x1 texture layer gives every hit (sample_texture, :26-32)
            const f4 c = decode_texel(ka.textures[min(m.texture_index, ka.tex_layers - 1u)], ka.srgb);
            l_aux[2u * i + 1u] = make_float4(c.x, c.y, c.z, c.w);
        }
        sv.mat_aux = l_aux;
        if constexpr (kTris)
            for (uint32_t i = tid; i < ka.object_count; i += kThreads) l_obj[i] = ka.objects[i];
        sv.sph = l_sph;
        sv.orig = l_orig;
        sv.sph_mat = l_smat;
        sv.nodes = l_nodes;
        sv.mat = l_mat;
        sv.obj = l_obj;
    }
    if constexpr (kMode == 2) {
        float4* l_tn = reinterpret_cast<float4*>(lds + ka.lds_tri_nodes_offset);
        uint4* l_tp = reinterpret_cast<uint4*>(lds + ka.lds_tri_prims_offset);
        for (uint32_t i = tid; i < 2u * ka.tri_nodes; i += kThreads) l_tn[i] = ka.tri_bvh[i];
        for (uint32_t i = tid; i < ka.tri_prim_count; i += kThreads) l_tp[i] = ka.tri_prims[i];
        sv.tri_nodes = l_tn;
        sv.tri_prims = l_tp;
        if (ka.lds_sub_offset) {  // the leaves' sub-object records too, when they fit
            RtSubObject* l_sub = reinterpret_cast<RtSubObject*>(lds + ka.lds_sub_offset);
            for (uint32_t i = tid; i < ka.sub_object_count; i += kThreads) l_sub[i] = ka.sub_objects[i];
            sv.sub = l_sub;
        }
    }
    for (uint32_t i = tid; i < 256u; i += kThreads) l_srgb[i] = ka.srgb[i];
    float* l_cam = l_srgb + 256;  // camera block for device-side primary rays
    if (tid < 16u) {
        l_cam[tid] = ka.inv_proj[tid];
        l_cam[16u + tid] = ka.inv_view[tid];
    }
    if (tid == 0) l_cam[32] = ka.aspect;
    __syncthreads();

    const bool accumulate = ka.accumulate == 1u;
    const uint32_t samples = accumulate ? ka.compute_per_frame : 1u;  // :158-175

    // Lane states. A lane owns one pixel at a time and one ray of its path.
    constexpr uint32_t kIdle = 0, kSetup = 1, kTrav = 2, kDone = 3, kPrimary = 4;
    uint32_t rays = 0;
    uint32_t lane_tile = 0;  // local tile of the lane's pixel (tile costs)
    uint32_t lane_slot = 0;  // the pixel's slot in its tile (frame-parallel light stores)
    const bool frame_par = ka.frame_light != nullptr;
    uint32_t mode = kIdle;
    uint32_t index = 0, sample = 0, frame = 0;
    float4 pix = make_float4(0.f, 0.f, 0.f, 0.f);
    Path p;
    p.o = p.d = mk(0.f, 0.f, 0.f);
    p.light = p.contrib = f4{0.f, 0.f, 0.f, 0.f};
    p.seed = p.bounce = 0;
    TraceState ts;
    ts.inv = mk(0.f, 0.f, 0.f);
    ts.a4 = ts.a2 = 0.f;
    ts.node = 0;
    ts.phase = 2;
    ts.nan_hit = false;
    ts.sph = SphereHit{kF32Max, 0u, 0u};
    ts.tri = TriHit{kF32Max, 0u, 0u, 0u, false};

    // random_index of a sample (:154, :162): the frame's accumulation index
    // (advanced per frame by the host only when accumulating, src/renderer.rs:216-235)
    // plus the sample number.
    auto random_index = [&]() { return ka.accumulation_index + (accumulate ? frame : 0u) + sample; };
    // A sample just started: with the primary pre-pass (rt_primary_kernel) its first
    // segment's trace result is read back and the lane goes straight to shading it;
    // else the trace starts at the next setup step.
    // (The record is read at the next shading step, where it is used: kPrimary.)
    auto primary_start = [&]() -> uint32_t {
        // (triangle instances only: on a sphere scene the pass measured slower, and the
        // sphere-only kernel keeps none of its code)
        return (kTris && ka.primary && p.bounce < ka.bounces) ? kPrimary : kSetup;
    };

    // A finished sample: pixel_color += per_pixel(...) (:161); then the pixel's
    // next sample (random_index += 1, :162), its next frame (a multi-frame
    // launch runs the frames of one pixel back to back on its lane), or its
    // final write (:164-178).
    // The end of one frame of the pixel (:164-178): the accumulation and the
    // packed output as that frame's dispatch leaves them. Stored where the pixel
    // finishes (holding them back to the next traversal phase measured no
    // faster and costs 6 VGPRs).
    auto store_frame = [&]() {
        float r, g, b, a;
        if (accumulate) {
            const float div = (float)((ka.accumulation_index + frame) * ka.compute_per_frame);
            r = clamp01(pix.x / div);
            g = clamp01(pix.y / div);
            b = clamp01(pix.z / div);
            a = clamp01(pix.w / div);
        } else {
            r = clamp01(p.light.x);
            g = clamp01(p.light.y);
            b = clamp01(p.light.z);
            a = clamp01(p.light.w);
        }
        if (accumulate) ka.accum[index] = pix;      // :164
        ka.output[index] = pack_rgba8(r, g, b, a);  // :178
    };
    auto finish_sample = [&]() {
        if (frame_par) {
            // frame-parallel batch: this sample's light, added to the
            // accumulation in order by rt_resolve_frames_kernel
            const size_t slot = (size_t)(frame * samples + sample) * ((size_t)ka.owned_tiles * 64u) +
                                (size_t)lane_tile * 64u + lane_slot;
            ka.frame_light[slot] = make_float4(p.light.x, p.light.y, p.light.z, p.light.w);
            sample += 1;
            if (sample < samples) {
                start_sample(ka, index, random_index(), pixel_ray(ka, l_cam, index, index % ka.width, index / ka.width),
                             p);
                mode = primary_start();
            } else {
                mode = kIdle;
            }
            return;
        }
        sample += 1;
        if (accumulate) {
            pix.x = pix.x + p.light.x;
            pix.y = pix.y + p.light.y;
            pix.z = pix.z + p.light.z;
            pix.w = pix.w + p.light.w;
        }
        if (sample == samples && frame + 1u < ka.frames) {
            // a multi-frame launch: every frame writes its result, exactly as
            // the sequence of single-frame dispatches it stands for would
            store_frame();
            frame += 1;
            sample = 0;
        }
        if (sample < samples) {
            start_sample(ka, index, random_index(), pixel_ray(ka, l_cam, index, index % ka.width, index / ka.width), p);
            mode = primary_start();
        } else {
            store_frame();
            mode = kIdle;
        }
    };

#ifdef RT_DIAG_TAIL
    const unsigned long long wave_t0 = realtime();
    unsigned long long wave_dry = 0;  // when the queue first came up empty for this wave
#endif
    if (blockIdx.x == 0 && threadIdx.x < ka.queue_stripes) ka.queue_next[threadIdx.x * kQueueStride] = 0u;
    // home stripe: this XCD's (blocks are dealt round-robin over the XCDs, so
    // blockIdx / 8 spreads an XCD's blocks over its stripes when there are more)
    TileQueue queue{(xcc_id() + 8u * (blockIdx.x >> 3)) % ka.queue_stripes, 0u};
    uint32_t tile_frame = 0;         // frame of the claimed unit (frame-parallel batches), wave-uniform
    uint32_t tile = unit_tile(ka, claim_tile(ka, queue), tile_frame);  // wave-uniform
    uint32_t next = 0;               // next pixel slot of `tile`, wave-uniform
#ifdef RT_DIAG
    unsigned long long iters = 0, trav_cyc = 0, steps = 0, step_lanes = 0, shade_cyc = 0, refill_cyc = 0,
                       setup_cyc = 0, leaf_cyc = 0, leaf_steps = 0;
    // lane occupancy by phase (RT_DIAG only): shading passes and the lanes they shade, split by
    // the branch each lane takes (sky miss, glass, specular, diffuse), setup passes and lanes
    unsigned long long shade_passes = 0, shade_lanes = 0, miss_lanes = 0, glass_lanes = 0, spec_lanes = 0,
                       setup_passes = 0, setup_lanes = 0;
    const unsigned long long t_start = stamp();
#endif
    while (true) {
#ifdef RT_DIAG
        ++iters;
        const unsigned long long ts0 = stamp();
#endif
        // 1. Shade the lanes whose trace has finished (:228-311); a sample started by
        // the primary pre-pass has its first trace result in ka.primary.
        bool fin = false;      // a sample finished: its rays go to the tile's cost
        uint32_t fin_rays = 0;
        if (kTris && mode == kPrimary) {
            const uint4 r = ka.primary[(size_t)(frame * samples + sample) * ((size_t)ka.owned_tiles * 64u) +
                                       (size_t)lane_tile * 64u + lane_slot];
            primary_state(PrimaryRecord{__uint_as_float(r.x), r.y, r.z, r.w}, ts);
            mode = kDone;
        }
#ifdef RT_DIAG
        {
            const uint64_t dm = __ballot(mode == kDone);
            if (dm) {
                ++shade_passes;
                shade_lanes += (unsigned long long)__popcll(dm);
            }
        }
#endif
        if (mode == kDone) {
            const Hit h = trace_end<kTris>(sv, ka, p.o, p.d, ts);
#ifdef RT_DIAG
            {
                const bool miss = h.t == kF32Max;
                const RtMaterial dmat = sv.mat[min(h.material_index, ka.material_count - 1u)];
                miss_lanes += (unsigned long long)__popcll(__ballot(miss));
                glass_lanes += (unsigned long long)__popcll(__ballot(!miss && dmat.glass > 0.0f));
                spec_lanes += (unsigned long long)__popcll(__ballot(!miss && !(dmat.glass > 0.0f) && dmat.specular > 0.0f));
            }
#endif
            ++rays;
            RT_ISA_MARK("shade");
            if (shade<(kMode >= 1)>(sv, ka, p, h)) {
                // rays of the sample: one per bounce, plus the escaping one unless the limit ended it
                fin = true;
                fin_rays = p.bounce + (p.bounce < ka.bounces ? 1u : 0u);
                finish_sample();
            } else {
                mode = kSetup;
            }
        }
        if (ka.tile_cost) record_tile_cost(ka.tile_cost, fin, lane_tile, fin_rays);
#ifdef RT_DIAG
        const unsigned long long ts1 = stamp();
        shade_cyc += ts1 - ts0;
#endif
        // 2. Refill: idle lanes take the next pixels of the wave's tile, in slot
        // order (ballot + mbcnt = a wave-wide prefix sum over the idle lanes).
        RT_ISA_MARK("refill");
        while (true) {
            const uint64_t need = __ballot(mode == kIdle);
            if (need == 0 || tile >= ka.owned_tiles) break;
            const uint32_t avail = 64u - next;
            if (mode == kIdle) {
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                if (rank < avail) {
                    const uint32_t slot = next + rank;
                    const uint32_t gt = tile * ka.world_size + ka.rank;
                    const uint32_t x = (gt % ka.tiles_x) * 8u + (slot & 7u);
                    const uint32_t y = (gt / ka.tiles_x) * 8u + (slot >> 3);
                    if (x < ka.width && y < ka.height) {
                        index = y * ka.width + x;  // :148
                        lane_tile = tile;
                        lane_slot = slot;
                        sample = 0;
                        frame = tile_frame;
                        mode = kSetup;
                        if (accumulate && !frame_par) pix = ka.accum[index];  // :156
                        start_sample(ka, index, random_index(), pixel_ray(ka, l_cam, index, x, y), p);
                        mode = primary_start();
                    }
                }
            }
            next += min((uint32_t)__popcll(need), avail);
            if (next == 64u) {
                tile = unit_tile(ka, claim_tile(ka, queue), tile_frame);
                next = 0;
            #ifdef RT_DIAG_TAIL
                if (tile >= ka.owned_tiles && wave_dry == 0) wave_dry = realtime();
#endif
            }
        }
#ifdef RT_DIAG
        const unsigned long long ts2 = stamp();
        refill_cyc += ts2 - ts1;
#endif
        // 3. Start the next ray of every lane that has one (the bounce loop's
        // bound, :226, ends a path without a trace only when bounces == 0).
#ifdef RT_DIAG
        {
            const uint64_t sm = __ballot(mode == kSetup);
            if (sm) {
                ++setup_passes;
                setup_lanes += (unsigned long long)__popcll(sm);
            }
        }
#endif
        RT_ISA_MARK("setup");
        if (mode == kSetup) {
            while (mode == kSetup && p.bounce >= ka.bounces) finish_sample();
            if (mode == kSetup) {
                trace_begin<kTris>(sv, ka, p.o, p.d, ts);
                mode = ts.phase == 2 ? kDone : kTrav;
            }
        }
#ifdef RT_DIAG
        setup_cyc += stamp() - ts2;
#endif
        if (__ballot(mode != kIdle) == 0 && tile >= ka.owned_tiles) break;
        // 4. Traverse. Lanes whose trace finishes wait (kDone) until fewer than
        // `trav_threshold` lanes are still traversing; then the wave goes back
        // to shade and refill them together, so neither the traversal tail nor
        // the shading runs on a nearly empty wave. With no tiles left (the
        // drain) the wave cannot refill, and by default traverses to the end.
        // Instances whose triangle accelerator stays in global memory (long
        // traces: hundreds of dependent loads) decouple the drain instead:
        // after at least `drain_min_steps` steps the wave goes back to
        // shading once at most `drain_threshold` lanes still traverse and
        // some lane is done, so a few very long traces do not hold up the
        // other paths' next bounces (C5: 72 -> 53 ms). Where traces are short
        // an extra shading pass costs more than the wait (C2, C3: measured).
        const bool draining = tile >= ka.owned_tiles;
        uint32_t thresh = draining ? 0u : ka.trav_threshold;
        uint32_t n_active = 64u, min_steps = 0u;
        if constexpr (kDrainDecouple<kMode, kTris>) {
            if (draining) {
                thresh = ka.drain_threshold;
                n_active = (uint32_t)__popcll(__ballot(mode == kTrav || mode == kDone));
                min_steps = ka.drain_min_steps;
            }
        }
#ifdef RT_DIAG
        const unsigned long long t0 = stamp();
#endif
        while (true) {
            const uint64_t trav = __ballot(mode == kTrav);
            const uint32_t n_trav = (uint32_t)__popcll(trav);
            if constexpr (kDrainDecouple<kMode, kTris>) {
                if (trav == 0 || (n_trav <= thresh && n_trav < n_active && min_steps == 0)) break;
                min_steps -= min_steps != 0;
            } else {
                if (n_trav <= thresh || trav == 0) break;
            }
#ifdef RT_DIAG
            ++steps;
            step_lanes += (unsigned long long)n_trav;
#endif
            // Test the deferred leaves once enough of the traversing lanes
            // hold one (ka.leaf_batch eighths); otherwise advance every lane by
            // one node.
            RT_ISA_MARK("traversal");
            bool leaves = false;
            if constexpr (kDeferLeaves<kTris> && !kFusedLeaves<kMode, kTris>) {
                const uint32_t n_pend = (uint32_t)__popcll(__ballot(mode == kTrav && ts.pending != kNoLeaf));
                leaves = 8u * n_pend >= ka.leaf_batch * n_trav;
            }
#ifdef RT_DIAG
            const unsigned long long tl0 = stamp();
#endif
            bool batched = false;
            if constexpr (kCoopLeaves<kMode, kTris>) {
                if (leaves && ka.tri_leaftris) {  // the wave's deferred leaves, cooperatively
                    RT_ISA_MARK("coop_leaf_batch");
                    const bool act = mode == kTrav && ts.pending != kNoLeaf;
                    coop_leaf_batch(sv, ka, p.o, p.d, ts, act, lds);
                    if (act) {
                        phase_end<kTris>(sv, ka, p.o, p.d, ts);
                        if (ts.phase == 2) mode = kDone;
                    }
                    batched = true;
                }
            }
            if (!batched && mode == kTrav && (!leaves || ts.pending != kNoLeaf)) {
                if (kDeferLeaves<kTris> && leaves) {
                    RT_ISA_MARK("leaf_batch");
                    leaf_step<kTris, (kMode <= 1)>(sv, ka, p.o, p.d, ts);
                } else {
                    RT_ISA_MARK("node_step");
                    node_step<kTris, kCertWalk<kMode>>(sv, ka, p.o, p.d, ts);
                }
                phase_end<kTris>(sv, ka, p.o, p.d, ts);
                if (ts.phase == 2) mode = kDone;
                if (!(kDeferLeaves<kTris> && leaves)) {
                    // further node steps before the next wave-wide check (kTravUnroll)
#pragma unroll
                    for (int k = 1; k < kTravUnroll<kMode, kTris>; ++k) {
                        if (mode == kTrav) {
                            node_step<kTris, kCertWalk<kMode>>(sv, ka, p.o, p.d, ts);
                            phase_end<kTris>(sv, ka, p.o, p.d, ts);
                            if (ts.phase == 2) mode = kDone;
                        }
                    }
                }
                if constexpr (kFusedLeaves<kMode, kTris>) {
                    // the leaf batch after the block's node steps, in the same iteration
                    // One kind of leaf per batch in scenes with both walks (C4): the triangle or
                    // the sphere leaves, whichever more lanes hold (the other lanes wait for the
                    // next batch), so the batch does not run both leaf bodies on part of the wave
                    // each (C4 1.410 -> 1.361 ms per frame, profiles/r06/r06y9; the second ballot gated on a sphere BVH
                    // measured C4 1.380).
                    const uint64_t mt = __ballot(mode == kTrav && ts.pending != kNoLeaf && ts.phase == 0);
                    const uint64_t ms = __ballot(mode == kTrav && ts.pending != kNoLeaf && ts.phase != 0);
                    const uint32_t n_p = (uint32_t)__popcll(mt | ms);
                    const uint32_t n_t = (uint32_t)__popcll(__ballot(mode == kTrav));
                    const bool tri_first = __popcll(mt) >= __popcll(ms);
                    if (8u * n_p >= ka.leaf_batch * n_t && mode == kTrav && ts.pending != kNoLeaf &&
                        (ts.phase == 0) == tri_first) {
                        RT_ISA_MARK("leaf_batch");
                        leaf_step<kTris, (kMode <= 1)>(sv, ka, p.o, p.d, ts);
                        phase_end<kTris>(sv, ka, p.o, p.d, ts);
                        if (ts.phase == 2) mode = kDone;
                    }
                }
                if constexpr (kBlockLeaves<kTris>) {
                    // the block's group tests: every lane that reached a leaf in it, together
                    // (the lanes that traversed in this block are the active ones: the ballots count them)
                    const uint32_t n_wait = (uint32_t)__popcll(__ballot(ts.pending != kNoLeaf));
                    const uint32_t n_tr = (uint32_t)__popcll(__ballot(true));
#ifdef RT_DIAG
                    if (8u * n_wait >= kBlockLeafShare * n_tr) {  // the block group tests and their lanes
                        const uint64_t gm = __ballot(mode == kTrav && ts.pending != kNoLeaf);
                        if (gm && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(gm)) {
                            atomicAdd(ka.diag + 26, 1ull);
                            atomicAdd(ka.diag + 27, (unsigned long long)__popcll(gm));
                        }
                    }
#endif
                    if (8u * n_wait >= kBlockLeafShare * n_tr && mode == kTrav && ts.pending != kNoLeaf) {
                        RT_ISA_MARK("sphere_leaves");
                        test_sphere_group(sv, ts.pending, p.o, p.d, ts.a4, ts.a2, ts.sph);
                        ts.limit = prune_limit(ts);
                        ts.pending = kNoLeaf;
                        phase_end<kTris>(sv, ka, p.o, p.d, ts);
                        if (ts.phase == 2) mode = kDone;
                    }
                }
            }
#ifdef RT_DIAG
            if (leaves) {
                leaf_cyc += stamp() - tl0;
                ++leaf_steps;
            }
#endif
        }
#ifdef RT_DIAG
        trav_cyc += stamp() - t0;
#endif
    }
#ifdef RT_DIAG
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(ka.diag + 0, stamp() - t_start);
        atomicAdd(ka.diag + 1, trav_cyc);
        atomicAdd(ka.diag + 2, steps);
        atomicAdd(ka.diag + 3, iters);
        atomicAdd(ka.diag + 4, step_lanes);
        atomicAdd(ka.diag + 5, shade_cyc);
        atomicAdd(ka.diag + 6, refill_cyc);
        atomicAdd(ka.diag + 7, setup_cyc);
        atomicAdd(ka.diag + 8, leaf_cyc);
        atomicAdd(ka.diag + 9, leaf_steps);
        // (RT_DIAG builds do not write the RT_DIAG_TAIL per-wave records: words 12.. are free)
        atomicAdd(ka.diag + 12, shade_passes);
        atomicAdd(ka.diag + 13, shade_lanes);
        atomicAdd(ka.diag + 14, miss_lanes);
        atomicAdd(ka.diag + 15, glass_lanes);
        atomicAdd(ka.diag + 16, spec_lanes);
        atomicAdd(ka.diag + 17, setup_passes);
        atomicAdd(ka.diag + 18, setup_lanes);
    }
#endif
#ifdef RT_DIAG_TAIL
    if ((threadIdx.x & 63u) == 0) {
        const unsigned long long wave_t1 = realtime();
        atomicAdd(ka.diag + 0, wave_t1);
        atomicMax(ka.diag + 1, wave_t1);
        atomicMax(ka.diag + 2, ~wave_t0);  // min start (counters reset to 0)
        atomicAdd(ka.diag + 3, 1ull);
        atomicAdd(ka.diag + 4, wave_t0);
        atomicMax(ka.diag + 5, wave_t0);
        atomicMax(ka.diag + 7, wave_t1 - wave_t0);
        const uint32_t w = blockIdx.x * (kThreads / 64u) + (threadIdx.x >> 6);
        if (w < 65536u) {
            ka.diag[kDiagHeaderWords + 2 * w] = wave_dry ? wave_dry : wave_t1;  // queue dry (tools/tail_probe.py)
            ka.diag[kDiagHeaderWords + 2 * w + 1] = wave_t1;
        }
    }
#endif
    atomicAdd(&block_rays, rays);
    __syncthreads();
    if (tid == 0 && block_rays != 0) atomicAdd(ka.ray_counter, (unsigned long long)block_rays);
    // Cost-ordered schedule: the first workgroup out of work sorts the previous
    // launch's tile costs into the claim order of the next launch, while the
    // rest of the grid drains its last paths (no extra launch, off the
    // critical path). The flags are double-buffered like the queue counters.
    if (ka.sched) {
        const uint32_t par = ka.sched_bits & 1u, n = ka.owned_tiles;
        __shared__ uint32_t sorter;
        if (tid == 0) {
            sorter = atomicAdd(sched_flags(ka) + par, 1u);
            if (blockIdx.x == 0) sched_flags(ka)[par ^ 1u] = 0u;
        }
        __syncthreads();
        if (sorter == 0)
            sort_tiles_by_cost<kThreads>(ka.sched + (par ^ 1u) * n, sched_orders(ka) + (par ^ 1u) * n, n,
                                         reinterpret_cast<uint32_t*>(lds + ka.lds_srgb_offset));
    }
    if (ka.launch_clock) {  // the workgroup's end, once all its waves are done
        __syncthreads();
        if (tid == 0) atomicMax(ka.launch_clock + 1, (unsigned long long)wall_clock64());
    }
}

// Instantiations: LDS mode x workgroup size x triangles present. All waves of
// a workgroup share one LDS copy of the scene, so the best size depends on the
// scene's LDS footprint against the VGPR-limited waves per SIMD; the host picks
// the size with the most resident waves up to a cap (rt_pathtrace_pick_config).
// Sphere-only scenes get kernels without the triangle side (fewer live scalar
// registers: the kernel arguments of the triangle path no longer spill).
// (mode, threads, triangles)
#define RT_FOR_EACH_CONFIG(X)                                                                                   \
    X(0, 256, true) X(0, 512, true) X(0, 1024, true) X(1, 256, true) X(1, 512, true) X(1, 1024, true)          \
    X(2, 256, true) X(2, 512, true) X(2, 1024, true) X(0, 256, false) X(0, 512, false) X(0, 1024, false)       \
    X(1, 256, false) X(1, 512, false) X(1, 1024, false)

// ---- the reference's brute-force sweep as a wavefront (BASELINE.json config 5) -------------
//
// rt_brute_wf_kernel renders frames the way compute_shader.wgsl does -- every sphere tested
// (:355-404), every object's box and every sub-object's box tested in order and the triangles of
// the sub-objects hit (:422-517) -- with no acceleration structure. What is MI355X-specific is
// how the work reaches the lanes. The paths live in HBM (KernelArgs::brute_paths, 64 B per
// pixel slot) and each launch advances one bounce level of one pass (frame, sample) over a
// compacted queue of the slots still alive, so every lane of a sweep carries a live ray (a
// workgroup in lockstep over its 256 pixels idles half its lanes once paths end at different
// bounces: C5 535.7 ms per frame that way). The sub-object records reach the
// lanes either through two LDS tiles per workgroup, the next tile's coalesced loads in flight
// while the current one is tested with broadcast reads, one barrier per tile (mode 1), or
// through the scalar cache, each wave streaming them on its own (mode 2). A sub-object's
// triangles are loaded only by the lanes whose box test passed. Same arithmetic and order as
// the reference's sweep per ray: the first of equal distances wins (`>=` rejects, :457), a NaN
// distance is accepted and makes later candidates accepted (:449-481), spheres by (t, index).
// Per pixel the passes run in order and a finished path adds its light to the accumulation
// then, the reference's sum order (:164-178).
//
// HBM traffic: the framebuffer (52 B/px/frame), texels, and the tile-streaming term
// with its fixed convention of one 256-ray tile -- 32 B x N_sub per started 256 rays of each
// bounce level -- counted in KernelArgs::stream_bytes; the bytes the sweeps actually stream
// from L2 (per LDS tile and workgroup, or per wave in mode 2) in KernelArgs::l2_stream_bytes.
constexpr uint32_t kBruteThreads = 256;  // 4 8x8 tiles per workgroup

// The triangles of one sub-object whose box the ray entered, in the sweep's order (:449-481):
// `>=` rejects a later equal distance, a NaN distance is accepted and then accepts every later one.
__device__ __forceinline__ void brute_sub_triangles(const KernelArgs& ka, f3 o, f3 d, uint32_t first_tri,
                                                    uint32_t count, uint32_t oi, float& closest, TriHit& best) {
    for (uint32_t j = 0; j < count; ++j) {
        const uint32_t ti = min(first_tri + j, ka.triangle_count - 1u);
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
        best = TriHit{dist, 0u, ti, oi, det > 0.0f};
    }
}

constexpr uint32_t kBruteGroup = 4;          // boxes tested per group (see the sweep)
constexpr uint32_t kBruteWfTileSubs = 512;    // sub-object records per LDS tile (x2 buffers)
constexpr uint32_t kBruteWfLoads = 2u * kBruteWfTileSubs / kBruteThreads;  // 16-B loads per thread and tile
static_assert(kBruteWfLoads * kBruteThreads == 2u * kBruteWfTileSubs, "tile = whole 16-B loads per thread");
static_assert(kBruteWfLoads == 4u, "the sweep's tile loads are written out for 4 per thread");
// Rays per thread in a sweep (the LDS-tiled sweep is written for several: each broadcast read of
// a box would serve them all; measured no faster than one, round 5).
constexpr uint32_t kBruteRays = 1;
constexpr uint32_t kBruteChunk = kBruteRays * kBruteThreads;  // queue entries per workgroup pass
// Entries of a ray's list of entered boxes (tile-local u16 indices, LDS) before it is drained.
constexpr uint32_t kBruteHits = 8;
static_assert(kBruteHits >= kBruteGroup, "a group's hits fit a drained list");
// Waves per SIMD requested: the LDS-tiled sweep 4 (its tiles), the streamed sweep 8 (no LDS but
// the hit lists, so the occupancy is set by registers; the shading code spills a little at 8).
constexpr int kBruteWaves = 4, kBruteStreamWaves = 8;

// One pixel slot of the wavefront: its pixel and whether it is inside the image.
struct BruteSlot {
    uint32_t s, index, x, y;
    bool valid;
};
__device__ __forceinline__ BruteSlot brute_slot(const KernelArgs& ka, const uint32_t* q_in, uint32_t level,
                                                uint32_t qi, uint32_t n_in) {
    BruteSlot r;
    const bool have = qi < n_in;
    r.s = have ? (level == 0u ? qi : q_in[qi]) : 0u;
    const uint32_t local_tile = r.s >> 6, lane_slot = r.s & 63u;
    const uint32_t gt = local_tile * ka.world_size + ka.rank;
    r.x = (gt % ka.tiles_x) * 8u + (lane_slot & 7u);
    r.y = (gt / ka.tiles_x) * 8u + (lane_slot >> 3);
    r.valid = have && local_tile < ka.owned_tiles && r.x < ka.width && r.y < ka.height;
    r.index = r.valid ? r.y * ka.width + r.x : 0u;
    return r;
}

__device__ __forceinline__ void brute_load_path(const float4* pl, uint32_t n_slots, uint32_t s, Path& p) {
    const float4 a = pl[s], b = pl[n_slots + s], l = pl[2u * n_slots + s], k = pl[3u * n_slots + s];
    p.o = mk(a.x, a.y, a.z);
    p.seed = __float_as_uint(a.w);
    p.d = mk(b.x, b.y, b.z);
    p.bounce = __float_as_uint(b.w);
    p.light = f4{l.x, l.y, l.z, l.w};
    p.contrib = f4{k.x, k.y, k.z, k.w};
}
__device__ __forceinline__ void brute_store_path(float4* pl, uint32_t n_slots, uint32_t s, const Path& p) {
    pl[s] = make_float4(p.o.x, p.o.y, p.o.z, __uint_as_float(p.seed));
    pl[n_slots + s] = make_float4(p.d.x, p.d.y, p.d.z, __uint_as_float(p.bounce));
    pl[2u * n_slots + s] = make_float4(p.light.x, p.light.y, p.light.z, p.light.w);
    pl[3u * n_slots + s] = make_float4(p.contrib.x, p.contrib.y, p.contrib.z, p.contrib.w);
}

template <bool kTris, bool kStream>
__global__ void __launch_bounds__(kBruteThreads, kStream ? kBruteStreamWaves : kBruteWaves)
    rt_brute_wf_kernel(KernelArgs ka) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t block_rays;
    const uint32_t tid = threadIdx.x;
    if (ka.launch_clock && tid == 0) atomicMax(ka.launch_clock, ~(unsigned long long)wall_clock64());
    const uint32_t n_slots = ka.owned_tiles * 64u;
    const uint32_t level = ka.brute_level;
    uint32_t* counts = ka.brute_counts + (size_t)ka.brute_pass * ka.brute_levels;
    const uint32_t n_in = level == 0u ? n_slots : counts[level];
    if (blockIdx.x * kBruteChunk >= n_in) {  // nothing for this workgroup (the queue shrank)
        if (ka.launch_clock && tid == 0) atomicMax(ka.launch_clock + 1, (unsigned long long)wall_clock64());
        return;
    }
    float* l_cam;
    const SceneView sv = brute_stage<kTris, kBruteThreads>(ka, lds, tid, l_cam);
    uint4* l_tile = reinterpret_cast<uint4*>(lds + ka.lds_stack_offset);  // 2 x kBruteWfTileSubs records
    uint16_t* l_hits = reinterpret_cast<uint16_t*>(l_tile + 4u * kBruteWfTileSubs);  // per thread and ray kBruteHits
    if (tid == 0) block_rays = 0;
    __syncthreads();

    const bool accumulate = ka.accumulate == 1u;
    const uint32_t samples = accumulate ? ka.compute_per_frame : 1u;
    const uint32_t frame = ka.brute_pass / samples, sample = ka.brute_pass % samples;
    const bool last_pass = ka.brute_pass + 1u == ka.frames * samples;
    const uint32_t random_index = ka.accumulation_index + (accumulate ? frame : 0u) + sample;
    const uint32_t* q_in = ka.brute_queue + (size_t)(level & 1u) * n_slots;
    uint32_t* q_out = ka.brute_queue + (size_t)((level + 1u) & 1u) * n_slots;
    float4* pl = ka.brute_paths;
    uint32_t rays = 0;
    uint64_t streamed = 0;  // sub-object records this workgroup's tiles (tid 0) or waves (lane 0 of each) read
    uint32_t chunks = 0;    // 256-ray chunks this workgroup swept (SURVEY §8d's tile convention)
    for (uint32_t c = blockIdx.x; c * kBruteChunk < n_in; c += gridDim.x) {
        ++chunks;
        // the chunk's rays: ray k of this thread is queue entry c * chunk + k * threads + tid
        f3 o[kBruteRays], d[kBruteRays], inv[kBruteRays];
        bool alive[kBruteRays];
        SphereHit sph[kBruteRays];
        TriHit tri[kBruteRays];
        float closest[kBruteRays];
#pragma unroll
        for (uint32_t k = 0; k < kBruteRays; ++k) {
            const BruteSlot bs = brute_slot(ka, q_in, level, c * kBruteChunk + k * kBruteThreads + tid, n_in);
            Path p;
            if (level == 0u) {
                if (bs.valid) {
                    start_sample(ka, bs.index, random_index, pixel_ray(ka, l_cam, bs.index, bs.x, bs.y), p);
                    brute_store_path(pl, n_slots, bs.s, p);  // the state the shading below reloads
                }
            } else if (bs.valid) {
                brute_load_path(pl, n_slots, bs.s, p);
            }
            alive[k] = bs.valid && p.bounce < ka.bounces;
            o[k] = alive[k] ? p.o : mk(0.f, 0.f, 0.f);
            d[k] = alive[k] ? p.d : mk(0.f, 0.f, 1.f);
            inv[k] = mk(1.0f / d[k].x, 1.0f / d[k].y, 1.0f / d[k].z);
            sph[k] = SphereHit{kF32Max, 0u, 0u};
            tri[k] = TriHit{kF32Max, 0u, 0u, 0u, false};
            closest[k] = kF32Max;
            // check_spheres (:355-404), every sphere
            if (alive[k]) {
                const float a = dot(d[k], d[k]);
                for (uint32_t i = 0; i < ka.sphere_slot_count; i += 4u)
                    test_sphere_group(sv, i, o[k], d[k], 4.0f * a, 2.0f * a, sph[k]);
            }
        }
        // check_triangles (:422-517): objects in order, their sub-objects through the LDS tiles
        // (kBruteStream: through the scalar cache, wave by wave)
        if constexpr (kTris && kStream) {
            static_assert(kBruteRays == 1, "the streamed sweep carries one ray per thread");
            uint32_t* l_hits32 = reinterpret_cast<uint32_t*>(l_tile);  // kBruteHits entries per thread
            typedef float rt_v4 __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(4))) const rt_v4 rt_cf4;  // scalar loads (wave-uniform)
            auto ldc = [](rt_cf4* p_, uint32_t i_) {
                const rt_v4 v_ = p_[i_];
                return make_float4(v_.x, v_.y, v_.z, v_.w);
            };
            for (uint32_t oi = 0; oi < ka.object_count; ++oi) {
                const RtObject& ob = sv.obj[oi];
                const bool in_obj = alive[0] && ray_in_bounds(o[0], inv[0], ob.min_bounds, ob.max_bounds);
                if (__ballot(in_obj) == 0ull) continue;  // no lane of the wave enters the object
                const uint32_t first = ob.first_sub_object_index, n_sub = ob.sub_object_count;
                const uint32_t last_sub = ka.sub_object_count - 1u;
                rt_cf4* recs = (rt_cf4*)(const void*)ka.sub_objects;
                if ((tid & 63u) == 0u) streamed += n_sub;  // every wave streams the records itself
                uint32_t cnt = 0u;
                // the entered boxes' triangles, each lane its own list in order (as the tiled sweep)
                auto drain = [&]() {
                    for (uint32_t e = 0; __builtin_amdgcn_ballot_w64(e < cnt) != 0ull; ++e) {
                        if (e < cnt) {
                            const uint32_t si = l_hits32[e * kBruteThreads + tid];
                            const float4 lo = reinterpret_cast<const float4*>(ka.sub_objects)[2u * si];
                            const float4 hi = reinterpret_cast<const float4*>(ka.sub_objects)[2u * si + 1u];
                            brute_sub_triangles(ka, o[0], d[0], __float_as_uint(lo.w), __float_as_uint(hi.w), oi,
                                                closest[0], tri[0]);
                        }
                    }
                    cnt = 0u;
                };
                // groups of 4 records: the next group's scalar loads in flight while this one is tested
                float4 l0, l1, l2, l3, h0, h1, h2, h3;
#define RT_BRUTE_SLOAD(j_)                                                                              \
    {                                                                                                   \
        const uint32_t s0_ = 2u * min(first + (j_), last_sub), s1_ = 2u * min(first + (j_) + 1u, last_sub); \
        const uint32_t s2_ = 2u * min(first + (j_) + 2u, last_sub), s3_ = 2u * min(first + (j_) + 3u, last_sub); \
        n0 = ldc(recs, s0_); m0 = ldc(recs, s0_ + 1u); n1 = ldc(recs, s1_); m1 = ldc(recs, s1_ + 1u);   \
        n2 = ldc(recs, s2_); m2 = ldc(recs, s2_ + 1u); n3 = ldc(recs, s3_); m3 = ldc(recs, s3_ + 1u);   \
    }
                {
                    float4 n0, n1, n2, n3, m0, m1, m2, m3;
                    RT_BRUTE_SLOAD(0u)
                    l0 = n0; l1 = n1; l2 = n2; l3 = n3; h0 = m0; h1 = m1; h2 = m2; h3 = m3;
                }
                uint32_t j0 = 0;
                for (; j0 + 4u <= n_sub; j0 += 4u) {
                    RT_ISA_MARK("brute_box");
                    float4 n0, n1, n2, n3, m0, m1, m2, m3;
                    RT_BRUTE_SLOAD(j0 + 4u)  // (clamped: past the end it rereads the last record)
                    uint32_t bits = 0u;
                    if (in_obj) {
                        bits |= ray_in_box4(o[0], inv[0], l0, h0) ? 1u : 0u;
                        bits |= ray_in_box4(o[0], inv[0], l1, h1) ? 2u : 0u;
                        bits |= ray_in_box4(o[0], inv[0], l2, h2) ? 4u : 0u;
                        bits |= ray_in_box4(o[0], inv[0], l3, h3) ? 8u : 0u;
                    }
                    if (__ballot(bits != 0u) != 0ull) {  // (rare) queue the entered boxes, in order
                        while (bits) {
                            const uint32_t j = __builtin_ctz(bits);
                            bits &= bits - 1u;
                            l_hits32[cnt * kBruteThreads + tid] = first + j0 + j;
                            cnt += 1u;
                        }
                        if (__ballot(cnt + 4u > kBruteHits) != 0ull) drain();
                    }
                    l0 = n0; l1 = n1; l2 = n2; l3 = n3; h0 = m0; h1 = m1; h2 = m2; h3 = m3;
                }
#undef RT_BRUTE_SLOAD
                for (; j0 < n_sub; ++j0) {  // the last 1-3 records
                    const uint32_t si = min(first + j0, last_sub);
                    const float4 lo = ldc(recs, 2u * si), hi = ldc(recs, 2u * si + 1u);
                    if (in_obj && ray_in_box4(o[0], inv[0], lo, hi)) {
                        l_hits32[cnt * kBruteThreads + tid] = si;
                        cnt += 1u;
                    }
                    if (__ballot(cnt + 1u > kBruteHits) != 0ull) drain();
                }
                drain();
            }
        } else if constexpr (kTris) {
            for (uint32_t oi = 0; oi < ka.object_count; ++oi) {
                const RtObject& ob = sv.obj[oi];
                bool in_obj[kBruteRays];
                bool any_in = false;
#pragma unroll
                for (uint32_t k = 0; k < kBruteRays; ++k) {
                    in_obj[k] = alive[k] && ray_in_bounds(o[k], inv[k], ob.min_bounds, ob.max_bounds);
                    any_in |= in_obj[k];
                }
                if (!__syncthreads_or(any_in)) continue;  // (a barrier: the tiles are free)
                const uint32_t first = ob.first_sub_object_index, n_sub = ob.sub_object_count;
                const uint32_t n_tiles = (n_sub + kBruteWfTileSubs - 1u) / kBruteWfTileSubs;
                const uint4* src = reinterpret_cast<const uint4*>(ka.sub_objects);
                const uint32_t last_sub = ka.sub_object_count - 1u;
                // the next tile, in flight: kBruteWfLoads (4) 16-B loads per thread, in named registers
                uint4 r0, r1, r2, r3;
#define RT_BRUTE_LOAD1(k_, rk)                                                                          \
    {                                                                                                   \
        const uint32_t q_ = tid + (k_) * kBruteThreads;                                                 \
        rk = src[2u * min(first + base_ + (min(q_, 2u * nt_ - 1u) >> 1), last_sub) + (q_ & 1u)];       \
    }
#define RT_BRUTE_LOAD_TILE(t)                                                                           \
    {                                                                                                   \
        const uint32_t base_ = (t) * kBruteWfTileSubs, nt_ = min(kBruteWfTileSubs, n_sub - base_);     \
        RT_BRUTE_LOAD1(0u, r0) RT_BRUTE_LOAD1(1u, r1) RT_BRUTE_LOAD1(2u, r2) RT_BRUTE_LOAD1(3u, r3)     \
    }
#define RT_BRUTE_STORE1(k_, rk)                                                                         \
    {                                                                                                   \
        const uint32_t q_ = tid + (k_) * kBruteThreads;                                                 \
        if (q_ < 2u * nt_) dst_[q_] = rk;                                                               \
    }
#define RT_BRUTE_STORE_TILE(t)                                                                          \
    {                                                                                                   \
        uint4* dst_ = l_tile + (size_t)((t) & 1u) * 2u * kBruteWfTileSubs;                             \
        const uint32_t nt_ = min(kBruteWfTileSubs, n_sub - (t) * kBruteWfTileSubs);                     \
        RT_BRUTE_STORE1(0u, r0) RT_BRUTE_STORE1(1u, r1) RT_BRUTE_STORE1(2u, r2) RT_BRUTE_STORE1(3u, r3) \
    }
                if (n_tiles) {
                    RT_BRUTE_LOAD_TILE(0u)
                    RT_BRUTE_STORE_TILE(0u)
                }
                for (uint32_t t = 0; t < n_tiles; ++t) {
                    __syncthreads();  // tile t stored; every reader of tile t - 1's buffer done
                    const uint32_t nt = min(kBruteWfTileSubs, n_sub - t * kBruteWfTileSubs);
                    if (tid == 0) streamed += nt;
                    const bool more = t + 1u < n_tiles;
                    if (more) RT_BRUTE_LOAD_TILE(t + 1u)  // in flight during the tests
                    if (any_in) {
                        const float4* tile = reinterpret_cast<const float4*>(l_tile + (size_t)(t & 1u) * 2u * kBruteWfTileSubs);
                        // A hit box's triangles are tested later, not in the box loop: their loads from
                        // global memory would stall the wave once per hit group. Each ray appends the
                        // tile-local indices of the boxes it enters to its list (LDS, in sweep order);
                        // the lists are drained -- each lane its own entries in order, all lanes' loads
                        // in flight together -- at the end of the tile, or when a list is full. A ray's
                        // triangle tests keep their order, and the box tests do not read `closest`.
                        uint32_t cnt[kBruteRays];
#pragma unroll
                        for (uint32_t k = 0; k < kBruteRays; ++k) cnt[k] = 0u;
                        auto drain = [&]() {
#pragma unroll
                            for (uint32_t k = 0; k < kBruteRays; ++k) {
                                for (uint32_t e = 0; __builtin_amdgcn_ballot_w64(e < cnt[k]) != 0ull; ++e) {
                                    if (e < cnt[k]) {
                                        const uint32_t j = l_hits[(k * kBruteHits + e) * kBruteThreads + tid];
                                        const float4 lo = tile[2u * j], hi = tile[2u * j + 1u];
                                        brute_sub_triangles(ka, o[k], d[k], __float_as_uint(lo.w), __float_as_uint(hi.w),
                                                            oi, closest[k], tri[k]);
                                    }
                                }
                                cnt[k] = 0u;
                            }
                        };
                        // groups of kBruteGroup boxes: the group's LDS reads in flight at once
                        uint32_t j0 = 0;
                        for (; j0 + kBruteGroup <= nt; j0 += kBruteGroup) {
                            RT_ISA_MARK("brute_box");
                            uint32_t bits[kBruteRays];
                            uint32_t any = 0u;
#pragma unroll
                            for (uint32_t k = 0; k < kBruteRays; ++k) bits[k] = 0u;
#pragma unroll
                            for (uint32_t j = 0; j < kBruteGroup; ++j) {  // broadcast reads
                                const float4 lo = tile[2u * (j0 + j)], hi = tile[2u * (j0 + j) + 1u];
#pragma unroll
                                for (uint32_t k = 0; k < kBruteRays; ++k)
                                    bits[k] |= (in_obj[k] & ray_in_box4(o[k], inv[k], lo, hi)) ? 1u << j : 0u;
                            }
#pragma unroll
                            for (uint32_t k = 0; k < kBruteRays; ++k) any |= bits[k];
                            if (any) {  // (rare) append the hit boxes, in order
                                bool full = false;
#pragma unroll
                                for (uint32_t k = 0; k < kBruteRays; ++k) {
                                    while (bits[k]) {
                                        const uint32_t j = __builtin_ctz(bits[k]);
                                        bits[k] &= bits[k] - 1u;
                                        l_hits[(k * kBruteHits + cnt[k]) * kBruteThreads + tid] = (uint16_t)(j0 + j);
                                        cnt[k] += 1u;
                                    }
                                    full |= cnt[k] + kBruteGroup > kBruteHits;  // the next group might not fit
                                }
                                if (__builtin_amdgcn_ballot_w64(full) != 0ull) drain();
                            }
                        }
                        for (; j0 < nt; ++j0) {  // (a tile of fewer than kBruteGroup-aligned boxes)
                            const float4 lo = tile[2u * j0], hi = tile[2u * j0 + 1u];
#pragma unroll
                            for (uint32_t k = 0; k < kBruteRays; ++k) {
                                if (in_obj[k] && ray_in_box4(o[k], inv[k], lo, hi)) {
                                    l_hits[(k * kBruteHits + cnt[k]) * kBruteThreads + tid] = (uint16_t)j0;
                                    cnt[k] += 1u;
                                }
                            }
                            bool full = false;
#pragma unroll
                            for (uint32_t k = 0; k < kBruteRays; ++k) full |= cnt[k] + 1u > kBruteHits;
                            if (__builtin_amdgcn_ballot_w64(full) != 0ull) drain();
                        }
                        drain();
                    }
                    if (more) RT_BRUTE_STORE_TILE(t + 1u)
                }
#undef RT_BRUTE_LOAD1
#undef RT_BRUTE_LOAD_TILE
#undef RT_BRUTE_STORE1
#undef RT_BRUTE_STORE_TILE
            }
        }
        // shading, ray by ray: the path state again from HBM
#pragma unroll
        for (uint32_t k = 0; k < kBruteRays; ++k) {
            const BruteSlot bs = brute_slot(ka, q_in, level, c * kBruteChunk + k * kBruteThreads + tid, n_in);
            Path p;
            if (bs.valid) brute_load_path(pl, n_slots, bs.s, p);
            bool done = bs.valid && !alive[k];  // bounces == 0: the path ends untraced
            if (alive[k]) {
                ++rays;
                TraceState ts;
                ts.sph = sph[k];
                ts.tri = tri[k];
                const Hit h = trace_end<kTris>(sv, ka, o[k], d[k], ts);
                done = shade<true>(sv, ka, p, h);
            }
            const bool cont = alive[k] && !done;
            if (cont) brute_store_path(pl, n_slots, bs.s, p);
            // the live slots to the next level's queue (wave-aggregated)
            const uint64_t m = __ballot(cont);
            if (m) {
                const uint32_t lane = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                uint32_t base = 0u;
                if ((tid & 63u) == (uint32_t)__builtin_ctzll(m)) base = atomicAdd(counts + level + 1u, (uint32_t)__popcll(m));
                base = __builtin_amdgcn_readlane(base, (uint32_t)__builtin_ctzll(m));
                if (cont) q_out[base + lane] = bs.s;
            }
            if (done) {  // the sample's light (:164-178), in pass order per pixel
                float r, g, b, al;
                if (accumulate) {
                    float4 pix = ka.accum[bs.index];
                    pix.x = pix.x + p.light.x;
                    pix.y = pix.y + p.light.y;
                    pix.z = pix.z + p.light.z;
                    pix.w = pix.w + p.light.w;
                    ka.accum[bs.index] = pix;
                    const float div = (float)((ka.accumulation_index + ka.frames - 1u) * ka.compute_per_frame);
                    r = clamp01(pix.x / div);
                    g = clamp01(pix.y / div);
                    b = clamp01(pix.z / div);
                    al = clamp01(pix.w / div);
                } else {
                    r = clamp01(p.light.x);
                    g = clamp01(p.light.y);
                    b = clamp01(p.light.z);
                    al = clamp01(p.light.w);
                }
                if (last_pass) ka.output[bs.index] = pack_rgba8(r, g, b, al);
            }
        }
    }
    atomicAdd(&block_rays, rays);
    __syncthreads();
    if (tid == 0 && block_rays) atomicAdd(ka.ray_counter, (unsigned long long)block_rays);
    // the tile-streaming term of SURVEY §8d -- 32 B x the sweep's sub-objects per 256 rays of the
    // level -- and the records the sweeps actually read from L2
    if (tid == 0 && ka.stream_bytes && kTris && chunks) {
        uint64_t n_sub = 0;
        for (uint32_t oi = 0; oi < ka.object_count; ++oi) n_sub += sv.obj[oi].sub_object_count;
        atomicAdd(ka.stream_bytes, (unsigned long long)(chunks * n_sub * 32ull));
    }
    if (streamed && ka.l2_stream_bytes) atomicAdd(ka.l2_stream_bytes, (unsigned long long)streamed * 32ull);
    if (ka.launch_clock) {
        __syncthreads();
        if (tid == 0) atomicMax(ka.launch_clock + 1, (unsigned long long)wall_clock64());
    }
}

// ---- coherent primary rays: a packet pre-pass -----------------------------------
//
// The first segment of every path starts at the camera, and the 64 primary rays
// of an 8x8 tile (one wave here) differ only by the pixel step and the reference's
// +-0.0005 jitter (compute_shader.wgsl:212-222): they reach nearly the same nodes
// and leaves. The path kernel's walk is per lane and asynchronous, so each lane
// loads its own copy of every node, sub-object and triangle record (C5: ~1,750 L1
// accesses per ray, the TCP's tag lookups being the binding unit). rt_primary_kernel
// instead walks each unit's rays as one packet: the node index is wave-uniform,
// a node is entered when any lane's ray enters it (each lane still applies its own
// culling test and its own exact leaf tests, so every lane gets exactly its own
// result: the lexicographic minimum over a superset of its own candidate set),
// and the node, sub-object and triangle records are read at wave-uniform
// addresses -- one scalar load or LDS broadcast for the whole wave. It writes
// each (frame, sample, pixel)'s trace result (the winner of trace_ray, :342-353:
// sphere or triangle, distance, index, object, facing) as one 16-B record; the
// path kernel starts those paths from the record instead of tracing their first
// segment. Everything after the first segment is unchanged.
template <int kMode, bool kTris, uint32_t kThreads, uint32_t kMinWaves>
__global__ void __launch_bounds__(kThreads, kMinWaves) rt_primary_kernel(KernelArgs ka) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t tid = threadIdx.x;
    // rt_set_timing: the pre-pass opens the launch's device span (the path kernel closes it)
    if (ka.launch_clock && tid == 0) atomicMax(ka.launch_clock, ~(unsigned long long)wall_clock64());
    float* l_srgb = reinterpret_cast<float*>(lds + ka.lds_srgb_offset);
    float* l_cam = l_srgb + 256;
    SceneView sv{ka.sphere_slots, ka.sphere_orig, ka.sphere_material, ka.sphere_bvh, ka.materials, nullptr,
                 ka.objects,      l_srgb,         ka.tri_bvh,     ka.tri_prims, kTris ? *ka.tri_extent : 0.0f,
                 ka.sub_objects};
    if constexpr (kMode >= 1) {  // what the walks read (the path kernel's mode 1 / 2 image)
        float4* l_sph = reinterpret_cast<float4*>(lds);
        RtObject* l_obj = reinterpret_cast<RtObject*>(lds + ka.lds_obj_offset);
        uint32_t* l_orig = reinterpret_cast<uint32_t*>(lds + ka.lds_orig_offset);
        float4* l_nodes = reinterpret_cast<float4*>(lds + ka.lds_nodes_offset);
        for (uint32_t i = tid; i < ka.sphere_slot_count; i += kThreads) {
            l_sph[i] = ka.sphere_slots[i];
            l_orig[i] = ka.sphere_orig[i];
        }
        for (uint32_t i = tid; i < 2u * ka.sphere_nodes; i += kThreads) l_nodes[i] = ka.sphere_bvh[i];
        if constexpr (kTris)
            for (uint32_t i = tid; i < ka.object_count; i += kThreads) l_obj[i] = ka.objects[i];
        sv.sph = l_sph;
        sv.orig = l_orig;
        sv.nodes = l_nodes;
        sv.obj = l_obj;
    }
    if constexpr (kMode == 2) {
        float4* l_tn = reinterpret_cast<float4*>(lds + ka.lds_tri_nodes_offset);
        uint4* l_tp = reinterpret_cast<uint4*>(lds + ka.lds_tri_prims_offset);
        for (uint32_t i = tid; i < 2u * ka.tri_nodes; i += kThreads) l_tn[i] = ka.tri_bvh[i];
        for (uint32_t i = tid; i < ka.tri_prim_count; i += kThreads) l_tp[i] = ka.tri_prims[i];
        sv.tri_nodes = l_tn;
        sv.tri_prims = l_tp;
        if (ka.lds_sub_offset) {
            RtSubObject* l_sub = reinterpret_cast<RtSubObject*>(lds + ka.lds_sub_offset);
            for (uint32_t i = tid; i < ka.sub_object_count; i += kThreads) l_sub[i] = ka.sub_objects[i];
            sv.sub = l_sub;
        }
    }
    if (tid < 16u) {
        l_cam[tid] = ka.inv_proj[tid];
        l_cam[16u + tid] = ka.inv_view[tid];
    }
    if (tid == 0) l_cam[32] = ka.aspect;
    __syncthreads();

    // one wave per (frame, local tile) unit, frame-major
    const uint32_t unit = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / 64u) + (tid >> 6));
    if (unit >= ka.queue_units) return;  // the whole wave
    // unit -> (frame, tile): frame-major, or tile-major (a tile's frames on consecutive waves of
    // a workgroup: their packets walk nearly the same nodes, so the later ones find them in the
    // CU's caches)
    const uint32_t n_frames = ka.queue_units / ka.owned_tiles;
    const uint32_t frame = ka.primary_tile_major ? unit % n_frames : unit / ka.owned_tiles;
    const uint32_t local_tile = ka.primary_tile_major ? unit / n_frames : unit - frame * ka.owned_tiles;
    const uint32_t slot = tid & 63u;
    const uint32_t gt = local_tile * ka.world_size + ka.rank;
    const uint32_t x = (gt % ka.tiles_x) * 8u + (slot & 7u);
    const uint32_t y = (gt / ka.tiles_x) * 8u + (slot >> 3);
    const bool valid = x < ka.width && y < ka.height;
    const uint32_t index = valid ? y * ka.width + x : 0u;
    const bool accumulate = ka.accumulate == 1u;
    const uint32_t samples = accumulate ? ka.compute_per_frame : 1u;
    const size_t owned_px = (size_t)ka.owned_tiles * 64u;
    const f3 cam = pixel_ray(ka, l_cam, index, x, y);
    for (uint32_t sample = 0; sample < samples; ++sample) {
        Path p;
        start_sample(ka, index, ka.accumulation_index + (accumulate ? frame : 0u) + sample, cam, p);
        const f3 o = p.o, d = p.d;
        TraceState ts;
        trace_begin<kTris>(sv, ka, o, d, ts);  // brute-force spheres, slab constants, phase
        if constexpr (kTris) {
            if (ts.phase == 0) {
                // the triangle accelerator as a packet: wave-uniform node (the layout of the
                // first lane's direction octant), per-lane culling and pruning
                uint32_t node = __builtin_amdgcn_readfirstlane(ts.node);
                while (node < ka.tri_nodes) {
                    const float4 lo = sv.tri_nodes[2u * node], hi = sv.tri_nodes[2u * node + 1u];
                    float near_t, far_t;
                    slab_hit(ts.slab, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, near_t, far_t);
                    bool hit = valid && near_t <= far_t && far_t >= 0.0f && near_t <= ts.limit;
                    const uint32_t leaf = __float_as_uint(hi.w);
                    uint32_t skip = 0u;  // certified pruning: the lane's own leaf certificate test
                    if (kCertWalk<kMode> && hit && leaf != 0xffffffffu && ka.tri_leafcert && near_t > ts.tri.t &&
                        ts.tri.t != kF32Max) {
                        skip = tri_leaf_skips(ka, leaf & 0xffffffu, ts.slab, o, d, ts.tri.t, lo, hi);
                        if (skip == kLeafCertAll) hit = false;
                    }
                    const bool any = __ballot(hit) != 0;
                    if (any && leaf != 0xffffffffu && hit) {
                        // (its certificate tested above: bit 24 of the argument would mean "deferred")
                        tri_leaf<(kMode <= 1)>(sv, ka, o, d, ts, leaf & 0xffffffu);
                        ts.limit = tri_limit(sv, ka, o, ts);
                    }
                    node = (any && leaf == 0xffffffffu) ? node + 1u : __float_as_uint(lo.w);
                }
                if (ts.nan_hit) ts.tri = sweep_triangles(sv, ka, o, d);  // measure-zero case: the sweep decides
                ts.phase = ka.sphere_nodes != 0 ? 1u : 2u;
                ts.node = 0;
                if (ts.phase == 1) phase_setup<kTris>(sv, ka, o, ts.a2 * 0.5f, 1, ts);
            }
        }
        if (ts.phase == 1) {
            // the sphere BVH as a packet over layout 0 (a complete walk whatever the octant,
            // boxes stored as min/max there): per-lane culling and pruning
            const uint32_t n0 = ka.sphere_octant_stride ? ka.sphere_octant_stride : ka.sphere_nodes;
            SlabRay sr = slab_ray(o.x, o.y, o.z, ts.inv.x, ts.inv.y, ts.inv.z, 0.0f);
            {
                // the lane's own margin (phase_setup's), without the octant pairing
                const float r = sqrt_up(dot(o, o));
                float m, slack;
                sphere_cull_bounds(r, ka.sphere_extent, ka.sphere_rmin, ka.sphere_rmax,
                                   __builtin_amdgcn_rsqf(ts.a2 * 0.5f), m, slack);
                sr = slab_ray(o.x, o.y, o.z, ts.inv.x, ts.inv.y, ts.inv.z, m);
                ts.slack = slack;
                ts.limit = prune_limit(ts);
            }
            uint32_t node = 0;
            while (node < n0) {
                const float4 lo = sv.nodes[2u * node], hi = sv.nodes[2u * node + 1u];
                float near_t, far_t;
                slab_hit(sr, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, near_t, far_t);
                const bool hit = valid && near_t <= far_t && far_t >= -ts.slack && near_t <= ts.limit;
                const bool any = __ballot(hit) != 0;
                const uint32_t leaf = __float_as_uint(hi.w);
                if (any && leaf != 0xffffffffu && hit) {
                    test_sphere_group(sv, leaf & 0xffffffu, o, d, ts.a4, ts.a2, ts.sph);
                    ts.limit = prune_limit(ts);
                }
                node = (any && leaf == 0xffffffffu) ? node + 1u : __float_as_uint(lo.w);
            }
        }
        if (valid)
            reinterpret_cast<uint4*>(ka.primary)[(size_t)(frame * samples + sample) * owned_px +
                                                 (size_t)local_tile * 64u + slot] = [&] {
                const PrimaryRecord r = primary_record<kTris>(ts);
                return make_uint4(__float_as_uint(r.t), r.id, r.meta, r.orig);
            }();
    }
}

namespace {
// Dynamic LDS above 64 KiB must be opted into per kernel.
hipError_t allow_big_lds(const void* fn) {
    int dev = 0, max_optin = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&max_optin, hipDeviceAttributeSharedMemPerBlockOptin, dev);
    if (e != hipSuccess || max_optin <= 0) return hipSuccess;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, max_optin - 256);
}
}  // namespace

hipError_t rt_launch_pathtrace(const KernelArgs& ka, int mode, bool tris, uint32_t threads, size_t lds_bytes,
                               uint32_t blocks, hipStream_t stream) {
#define RT_LAUNCH(M, T, TR)                                                                                    \
    if (mode == M && threads == T && tris == TR) {                                                            \
        hipLaunchKernelGGL((rt_pathtrace_kernel<M, T, TR>), dim3(blocks), dim3(T), lds_bytes, stream, ka);    \
        return hipGetLastError();                                                                             \
    }
    RT_FOR_EACH_CONFIG(RT_LAUNCH)
#undef RT_LAUNCH
    return hipErrorInvalidValue;
}

size_t rt_brute_wf_tile_bytes(bool stream) {
    if (stream) return (size_t)kBruteThreads * kBruteHits * 4u;  // the hit lists only (u32 entries)
    return 2u * (size_t)kBruteWfTileSubs * sizeof(RtSubObject) + (size_t)kBruteThreads * kBruteRays * kBruteHits * 2u;
}

uint32_t rt_brute_wf_chunk() { return kBruteChunk; }

// One (pass, bounce level) of the wavefront; `blocks` workgroups stride over the level's queue.
hipError_t rt_launch_brute_wf(const KernelArgs& ka, bool tris, bool scalar_stream, size_t lds_bytes, uint32_t blocks,
                              hipStream_t stream) {
    if (blocks == 0) return hipSuccess;
    const void* fn = tris ? (scalar_stream ? reinterpret_cast<const void*>(&rt_brute_wf_kernel<true, true>)
                                           : reinterpret_cast<const void*>(&rt_brute_wf_kernel<true, false>))
                          : reinterpret_cast<const void*>(&rt_brute_wf_kernel<false, false>);
    if (lds_bytes > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        if (e != hipSuccess) return hipErrorInvalidConfiguration;
    }
    if (tris && scalar_stream)
        hipLaunchKernelGGL((rt_brute_wf_kernel<true, true>), dim3(blocks), dim3(kBruteThreads), lds_bytes, stream, ka);
    else if (tris)
        hipLaunchKernelGGL((rt_brute_wf_kernel<true, false>), dim3(blocks), dim3(kBruteThreads), lds_bytes, stream, ka);
    else
        hipLaunchKernelGGL((rt_brute_wf_kernel<false, false>), dim3(blocks), dim3(kBruteThreads), lds_bytes, stream, ka);
    return hipGetLastError();
}

hipError_t rt_launch_primary(const KernelArgs& ka, int mode, bool tris, size_t lds_bytes, uint32_t threads,
                             uint32_t min_waves, hipStream_t stream) {
    if (threads == 0) threads = kPrimaryThreads;
    const uint32_t per = threads / 64u;
    const uint32_t blocks = (ka.queue_units + per - 1u) / per;
    if (blocks == 0) return hipSuccess;
#define RT_PRIMARY(M, TR, T, W)                                                                                \
    if (mode == M && tris == TR && threads == T && min_waves == W) {                                           \
        if (lds_bytes > 64u * 1024u) {                                                                         \
            hipError_t e = allow_big_lds(reinterpret_cast<const void*>(&rt_primary_kernel<M, TR, T, W>));     \
            if (e != hipSuccess) return e;                                                                     \
        }                                                                                                      \
        hipLaunchKernelGGL((rt_primary_kernel<M, TR, T, W>), dim3(blocks), dim3(T), lds_bytes, stream, ka);   \
        return hipGetLastError();                                                                              \
    }
    // (mode, triangles, workgroup size, minimum waves per SIMD: 0 = the compiler's choice)
    RT_PRIMARY(1, true, 64, 0) RT_PRIMARY(1, true, 128, 0) RT_PRIMARY(1, true, 256, 0) RT_PRIMARY(1, true, 256, 8)
    RT_PRIMARY(1, true, 512, 0) RT_PRIMARY(1, true, 1024, 0) RT_PRIMARY(2, true, 1024, 0)
#undef RT_PRIMARY
    return hipErrorInvalidValue;
}

// Picks the workgroup size for this LDS mode and footprint: the most resident
// waves per CU up to kTargetWavesPerCu (measured on C2: 16 waves/CU beat 18
// and 20 — the per-lane BVH traversal is LDS-latency bound and more waves only
// add contention), ties to the smaller workgroup.
constexpr int kDefaultWavesPerCu = 16;

hipError_t rt_pathtrace_pick_config(int mode, bool tris, size_t lds_bytes, size_t lds_bytes_per_thread,
                                    uint32_t force_threads, uint32_t waves_cap, uint32_t* threads,
                                    int* blocks_per_cu) {
    const int kTargetWavesPerCu = waves_cap ? (int)waves_cap : kDefaultWavesPerCu;
    int best_waves = -1;
    // lds_bytes_per_thread: the cooperative leaf batch's per-wave scratch (grows with the workgroup size)
#define RT_OCC(M, T, TR)                                                                                  \
    if (mode == M && tris == TR) {                                                                        \
        int n = 0;                                                                                        \
        hipError_t e = allow_big_lds(reinterpret_cast<const void*>(&rt_pathtrace_kernel<M, T, TR>));     \
        if (e != hipSuccess) return e;                                                                    \
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rt_pathtrace_kernel<M, T, TR>, T,           \
                                                         lds_bytes + (size_t)T * lds_bytes_per_thread);  \
        if (e != hipSuccess) return e;                                                                    \
        const int waves = std::min(n * (int)(T / 64), kTargetWavesPerCu);                                 \
        if (n > 0 && (force_threads ? force_threads == T : waves > best_waves)) {                         \
            best_waves = waves;                                                                           \
            *threads = T;                                                                                 \
            *blocks_per_cu = force_threads ? n : std::max(1, std::min(n, kTargetWavesPerCu / (int)(T / 64))); \
        }                                                                                                 \
    }
    RT_FOR_EACH_CONFIG(RT_OCC)
#undef RT_OCC
    if (best_waves <= 0) return hipErrorInvalidConfiguration;
    return hipSuccess;
}

// Gather support: pack the accumulation of this rank's tiles, in
// local-tile order (64 float4 per tile), into a contiguous buffer.
extern "C" __global__ void __launch_bounds__(256) rt_pack_tiles_kernel(const float4* __restrict__ accum,
                                                                      float4* __restrict__ dst, uint32_t width,
                                                                      uint32_t height, uint32_t tiles_x,
                                                                      uint32_t owned_tiles, uint32_t rank,
                                                                      uint32_t world) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t local_tile = gid >> 6;
    if (local_tile >= owned_tiles) return;
    const uint32_t lane = (uint32_t)(gid & 63u);
    const uint32_t tile = (uint32_t)local_tile * world + rank;
    const uint32_t x = (tile % tiles_x) * 8u + (lane & 7u);
    const uint32_t y = (tile / tiles_x) * 8u + (lane >> 3);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (x < width && y < height) v = accum[(size_t)y * width + x];
    dst[gid] = v;
}

// Unpack: blockIdx.y selects the source rank first_rank + blockIdx.y, whose
// packed block starts at src + blockIdx.y * stride_px; skip_rank's block (the
// destination's own tiles, already in place) is left out. One launch unpacks
// every rank's block of a gather.
__device__ __forceinline__ uint32_t owned_tiles_of(uint32_t n_tiles, uint32_t rank, uint32_t world) {
    return rank < n_tiles ? (n_tiles - rank + world - 1u) / world : 0u;
}

extern "C" __global__ void __launch_bounds__(256) rt_unpack_tiles_kernel(
    const float4* __restrict__ src, float4* __restrict__ accum, uint32_t* __restrict__ output, uint32_t width,
    uint32_t height, uint32_t tiles_x, uint32_t n_tiles, uint32_t first_rank, uint32_t world, uint64_t stride_px,
    uint32_t skip_rank, float divisor) {
    const uint32_t rank = first_rank + blockIdx.y;
    if (rank == skip_rank) return;
    src += (uint64_t)blockIdx.y * stride_px;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t local_tile = gid >> 6;
    if (local_tile >= owned_tiles_of(n_tiles, rank, world)) return;
    const uint32_t lane = (uint32_t)(gid & 63u);
    const uint32_t tile = (uint32_t)local_tile * world + rank;
    const uint32_t x = (tile % tiles_x) * 8u + (lane & 7u);
    const uint32_t y = (tile / tiles_x) * 8u + (lane >> 3);
    if (x >= width || y >= height) return;
    const float4 v = src[gid];
    const size_t idx = (size_t)y * width + x;
    accum[idx] = v;
    output[idx] = pack_rgba8(clamp01(v.x / divisor), clamp01(v.y / divisor), clamp01(v.z / divisor),
                             clamp01(v.w / divisor));
}

// The end of a frame-parallel batch: for each owned pixel, the accumulation
// plus every (frame, sample) light in the reference's order -- frame k's samples
// k, k+1, ..., then frame k+1's (compute_shader.wgsl:156-164, src/renderer.rs:216-235)
// -- so the sum is bit-identical to the frames rendered one after another; then
// the accumulation and the last frame's packed output (:166-178). One thread per
// owned pixel slot, coalesced: HBM-bound (16 + 16 * frames * samples + 20 B/px).
// A 16-B load of data read once (nontemporal: it does not displace cached lines).
typedef float StreamF4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    const StreamF4 v = __builtin_nontemporal_load(reinterpret_cast<const StreamF4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void resolve_pixel(float4* __restrict__ accum, uint32_t* __restrict__ output,
                                              const float4* __restrict__ light, uint32_t width, uint32_t height,
                                              uint32_t tiles_x, uint32_t owned_tiles, uint32_t rank, uint32_t world,
                                              uint32_t k0, uint32_t samples, uint32_t frames) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t owned_px = (uint64_t)owned_tiles * 64u;
    if (gid >= owned_px) return;
    const uint32_t lane = (uint32_t)(gid & 63u);
    const uint32_t tile = (uint32_t)(gid >> 6) * world + rank;
    const uint32_t x = (tile % tiles_x) * 8u + (lane & 7u);
    const uint32_t y = (tile / tiles_x) * 8u + (lane >> 3);
    if (x >= width || y >= height) return;
    const size_t idx = (size_t)y * width + x;
    float4 pix = accum[idx];
    const uint32_t n = frames * samples;
    // the lights are read once: groups of kGroup loads in flight together (streaming,
    // nontemporal), then added in the reference's order
    constexpr uint32_t kGroup = 8;
    const float4* src = light + gid;
    uint32_t i = 0;
    for (; i + kGroup <= n; i += kGroup) {
        float4 l[kGroup];
#pragma unroll
        for (uint32_t k = 0; k < kGroup; k++) l[k] = ld_stream(src + (size_t)(i + k) * owned_px);
#pragma unroll
        for (uint32_t k = 0; k < kGroup; k++) {
            pix.x = pix.x + l[k].x;
            pix.y = pix.y + l[k].y;
            pix.z = pix.z + l[k].z;
            pix.w = pix.w + l[k].w;
        }
    }
    for (; i < n; i++) {
        const float4 l = ld_stream(src + (size_t)i * owned_px);
        pix.x = pix.x + l.x;
        pix.y = pix.y + l.y;
        pix.z = pix.z + l.z;
        pix.w = pix.w + l.w;
    }
    accum[idx] = pix;
    const float div = (float)((k0 + frames - 1u) * samples);
    output[idx] = pack_rgba8(clamp01(pix.x / div), clamp01(pix.y / div), clamp01(pix.z / div), clamp01(pix.w / div));
}

extern "C" __global__ void __launch_bounds__(256) rt_resolve_frames_kernel(
    float4* __restrict__ accum, uint32_t* __restrict__ output, const float4* __restrict__ light, uint32_t width,
    uint32_t height, uint32_t tiles_x, uint32_t owned_tiles, uint32_t rank, uint32_t world, uint32_t k0,
    uint32_t samples, uint32_t frames, unsigned long long* __restrict__ clock) {
    // clock (rt_set_timing): {~earliest workgroup start, latest workgroup end}, stamped by the
    // first and the last kResolveStampBlocks workgroups only (workgroups start in index order
    // and take the same time): thousands of workgroups each adding two atomics on the same two
    // words cost tens of microseconds at the end of the pass
    constexpr uint32_t kResolveStampBlocks = 64;
    const bool first = blockIdx.x < kResolveStampBlocks;
    const bool last = blockIdx.x + kResolveStampBlocks >= gridDim.x;
    if (clock && first && threadIdx.x == 0) atomicMax(clock, ~(unsigned long long)wall_clock64());
    resolve_pixel(accum, output, light, width, height, tiles_x, owned_tiles, rank, world, k0, samples, frames);
    if (clock && last) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(clock + 1, (unsigned long long)wall_clock64());
    }
}

hipError_t rt_launch_resolve(float4* accum, uint32_t* output, const float4* light, uint32_t width, uint32_t height,
                             uint32_t tiles_x, uint32_t owned_tiles, uint32_t rank, uint32_t world, uint32_t k0,
                             uint32_t samples, uint32_t frames, unsigned long long* clock, hipStream_t stream) {
    const uint64_t threads = (uint64_t)owned_tiles * 64u;
    const uint32_t blocks = (uint32_t)((threads + 255u) / 256u);
    hipLaunchKernelGGL(rt_resolve_frames_kernel, dim3(blocks), dim3(256), 0, stream, accum, output, light, width,
                       height, tiles_x, owned_tiles, rank, world, k0, samples, frames, clock);
    return hipGetLastError();
}

// The packed RGBA8 output, one u32 per pixel, both ways (non-accumulating renders).
// (Unpacking: blockIdx.y selects the source rank, as in rt_unpack_tiles_kernel.)
extern "C" __global__ void __launch_bounds__(256) rt_pack_output_kernel(
    const uint32_t* __restrict__ output, uint32_t* __restrict__ dst, uint32_t width, uint32_t height,
    uint32_t tiles_x, uint32_t n_tiles, uint32_t first_rank, uint32_t world, uint64_t stride_px, uint32_t skip_rank,
    uint32_t unpack) {
    const uint32_t rank = first_rank + blockIdx.y;
    if (rank == skip_rank) return;
    dst += (uint64_t)blockIdx.y * stride_px;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t local_tile = gid >> 6;
    if (local_tile >= owned_tiles_of(n_tiles, rank, world)) return;
    const uint32_t lane = (uint32_t)(gid & 63u);
    const uint32_t tile = (uint32_t)local_tile * world + rank;
    const uint32_t x = (tile % tiles_x) * 8u + (lane & 7u);
    const uint32_t y = (tile / tiles_x) * 8u + (lane >> 3);
    const bool inside = x < width && y < height;
    const size_t idx = (size_t)y * width + x;
    uint32_t* out = const_cast<uint32_t*>(output);
    if (unpack) {
        if (inside) out[idx] = dst[gid];
    } else {
        dst[gid] = inside ? output[idx] : 0u;
    }
}

static uint32_t owned_tiles_host(uint32_t n_tiles, uint32_t rank, uint32_t world) {
    return rank < n_tiles ? (n_tiles - rank + world - 1u) / world : 0u;
}

// Packs rank `first_rank`'s output (ranks == 1, unpack false), or unpacks the
// blocks of ranks [first_rank, first_rank + ranks) except skip_rank, block r at
// packed + (r - first_rank) * stride_px.
hipError_t rt_launch_pack_output(uint32_t* output, uint32_t* packed, uint32_t width, uint32_t height, uint32_t tiles_x,
                                 uint32_t n_tiles, uint32_t first_rank, uint32_t ranks, uint32_t world,
                                 uint64_t stride_px, uint32_t skip_rank, bool unpack, hipStream_t stream) {
    const uint64_t threads = (uint64_t)owned_tiles_host(n_tiles, first_rank, world) * 64u;  // the first rank has the most
    const uint32_t blocks = (uint32_t)((threads + 255u) / 256u);
    if (blocks == 0 || ranks == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_pack_output_kernel, dim3(blocks, ranks), dim3(256), 0, stream, output, packed, width, height,
                       tiles_x, n_tiles, first_rank, world, stride_px, skip_rank, unpack ? 1u : 0u);
    return hipGetLastError();
}

hipError_t rt_launch_pack(const float4* accum, float4* dst, uint32_t width, uint32_t height, uint32_t tiles_x,
                          uint32_t owned_tiles, uint32_t rank, uint32_t world, hipStream_t stream) {
    const uint64_t threads = (uint64_t)owned_tiles * 64u;
    const uint32_t blocks = (uint32_t)((threads + 255u) / 256u);
    hipLaunchKernelGGL(rt_pack_tiles_kernel, dim3(blocks), dim3(256), 0, stream, accum, dst, width, height, tiles_x,
                       owned_tiles, rank, world);
    return hipGetLastError();
}

hipError_t rt_launch_unpack(const float4* src, float4* accum, uint32_t* output, uint32_t width, uint32_t height,
                            uint32_t tiles_x, uint32_t n_tiles, uint32_t first_rank, uint32_t ranks, uint32_t world,
                            uint64_t stride_px, uint32_t skip_rank, float divisor, hipStream_t stream) {
    const uint64_t threads = (uint64_t)owned_tiles_host(n_tiles, first_rank, world) * 64u;  // the first rank has the most
    const uint32_t blocks = (uint32_t)((threads + 255u) / 256u);
    if (blocks == 0 || ranks == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_unpack_tiles_kernel, dim3(blocks, ranks), dim3(256), 0, stream, src, accum, output, width,
                       height, tiles_x, n_tiles, first_rank, world, stride_px, skip_rank, divisor);
    return hipGetLastError();
}

// Exhaustive device check of the fast exact-arithmetic helpers in
// rt_device_math.h against the IEEE operations they replace (rt_math_selftest).
// which: 0 sqrt_rn_nrm over its domain, 1 x / 2pi, 2 x / pi, 3 x / 255, 4 x / 10,
// each over all 2^32 f32 bit patterns (sqrt: those in its domain).
extern "C" __global__ void __launch_bounds__(256) rt_math_selftest_kernel(uint32_t which,
                                                                         unsigned long long* mismatches,
                                                                         uint32_t* first_bad) {
    unsigned long long bad = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const uint32_t bits = (uint32_t)i;
        const float x = __uint_as_float(bits);
        float got, want;
        if (which == 0) {
            const float ax = __builtin_fabsf(x);
            if (ax != 0.0f && ax < 0x1p-96f) continue;  // outside the domain (tiny and denormal)
            got = sqrt_rn_nrm(x);
            want = __builtin_sqrtf(x);
        } else if (which == 1) {
            got = div_const(x, kTwoPiWgsl, kInvTwoPiWgsl);
            want = x / kTwoPiWgsl;
        } else if (which == 2) {
            got = div_const(x, kWgslPi, kInvWgslPi);
            want = x / kWgslPi;
        } else if (which == 3) {
            got = div_const(x, 255.0f, kInv255);
            want = x / 255.0f;
        } else if (which == 4) {
            got = div_const(x, 10.0f, kInv10);
            want = x / 10.0f;
        } else {
            // every value random01 returns: its seed word / 2^32 (the seed is any u32)
            const float u = (float)bits / 4294967296.0f;
            if (which == 5) {
                got = logf_u01(u);
                want = logf_c(u);
            } else {
                const float theta = kBoxMullerTwoPi * u;
                got = cosf_box(theta);
                want = cosf_c(theta);
            }
        }
        const bool same = __float_as_uint(got) == __float_as_uint(want) || (got != got && want != want);
        if (!same) {
            ++bad;
            atomicMin(first_bad, bits);
        }
    }
    if (bad) atomicAdd(mismatches, bad);
}

hipError_t rt_launch_math_selftest(uint32_t which, unsigned long long* mismatches, uint32_t* first_bad,
                                   hipStream_t stream) {
    hipLaunchKernelGGL(rt_math_selftest_kernel, dim3(8192), dim3(256), 0, stream, which, mismatches, first_bad);
    return hipGetLastError();
}
