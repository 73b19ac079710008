// treelet.hip -- the triangle walk of scenes whose accelerator lives in global memory, as a
// wavefront over treelets.
//
// The persistent path kernel walks each lane's ray through the accelerator on its own: on C5
// (1M triangles, 286k nodes per layout) every node, certificate and triangle block a lane reads
// is a lane-divergent load, the L1 serves a third of them, and the walk is bound by the L2
// requests of the misses (§5.3e). Here the rays of a whole batch of frames are walked together
// instead, and the accelerator is cut into subtrees of at most kTreeletNodes nodes (the treelets):
//
//   * top walk (rt_tl_top_kernel): each ray walks the part of the tree above the cut in its
//     direction-ordered layout (nodes shared by all rays: L1/L2 hits) until it enters a treelet;
//     it is then queued on that treelet, with the position to resume at;
//   * treelet walk (rt_tl_subtree_kernel): one workgroup per treelet stages the treelet's nodes,
//     leaf records and triangle blocks in LDS once, and walks every ray queued on it from there;
//     the rays then go back to the top walk;
//   * shading (rt_tl_shade_kernel): a ray whose walk is over is shaded (the reference's bounce
//     loop body, compute_shader.wgsl:228-311) and its next segment joins the top walk; the first
//     segments come from the coherent primary pre-pass (rt_primary_kernel), as in the path
//     kernel. Each (frame, sample) path writes its light to the batch's light buffer, which
//     rt_resolve_frames_kernel adds to the accumulation in the reference's order.
//
// Exactness: a ray's result is the lexicographic minimum of (distance, sweep position) over the
// triangles of the leaves whose boxes it enters (each leaf merged exactly as the cooperative leaf
// batch merges it: object box, then the sub-object box only when a candidate would change the
// result, :431-500), whatever order the leaves are met in -- the same minimum the path kernel's
// walk and the reference's sweep return. A NaN distance hands the ray to the sweep itself, as
// everywhere. Spheres: only the brute-force sphere set (scenes with no sphere BVH), swept at
// shading time as trace_begin sweeps it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_path_common.h"
#include "rt_treelet.h"

namespace {

constexpr uint32_t kTlThreads = 256;
constexpr uint32_t kTlSteps = 4;  // treelet node steps per leaf-pass check
constexpr uint32_t kTlTopSteps = 8;  // top-walk node steps per refill check

// The list and counter block of a round (TreeletArgs::lists, ::ctl): walk lists A[2] and shading
// lists R[2] of slot ids, by round parity, and the treelet entries of the round.
__device__ __forceinline__ uint32_t* tl_walk_list(const TreeletArgs& ta, uint32_t q) { return ta.lists + (size_t)q * ta.n_slots; }
__device__ __forceinline__ uint32_t* tl_shade_list(const TreeletArgs& ta, uint32_t q) {
    return ta.lists + (size_t)(2u + q) * ta.n_slots;
}
__device__ __forceinline__ uint32_t* tl_entries(const TreeletArgs& ta) { return ta.lists + (size_t)4u * ta.n_slots; }

// Appends `slot` for the lanes with `want` (wave-aggregated: one atomic per wave).
__device__ __forceinline__ void tl_append(uint32_t* list, uint32_t* count, bool want, uint32_t slot) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const uint32_t lead = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0u;
    if ((threadIdx.x & 63u) == lead) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, lead);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (want) list[base + rank] = slot;
}

// A rank in the queue of treelet `target` (kTlNone: none) for every lane: the wave's lanes are
// grouped by treelet, one atomic per group (its leader's), ranks by mbcnt within the group.
__device__ __forceinline__ uint32_t tl_enqueue(uint32_t* counts, uint32_t target) {
    bool pending = target != kTlNone;
    uint32_t rank = 0u;
    for (;;) {
        const uint64_t m = __ballot(pending);
        if (m == 0) break;
        const uint32_t lead = (uint32_t)__builtin_ctzll(m);
        const uint32_t lt = (uint32_t)__builtin_amdgcn_readlane((int)target, (int)lead);
        const bool mine = pending && target == lt;
        const uint64_t g = __ballot(mine);
        uint32_t base = 0u;
        if ((threadIdx.x & 63u) == lead) base = atomicAdd(counts + lt, (uint32_t)__popcll(g));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)lead);
        if (mine) {
            rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(g >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)g, 0u));
            pending = false;
        }
    }
    return rank;
}

// A slot's pixel: slot = (frame * samples + sample) * owned_px + local pixel (frame_light's indexing).
struct TlPixel {
    uint32_t index, x, y, frame, sample;
    bool valid;
};
__device__ __forceinline__ TlPixel tl_pixel(const KernelArgs& ka, uint32_t slot, uint32_t samples) {
    const uint32_t owned_px = ka.owned_tiles * 64u;
    const uint32_t pass = slot / owned_px, lp = slot - pass * owned_px;
    TlPixel r;
    r.frame = pass / samples;
    r.sample = pass - r.frame * samples;
    const uint32_t gt = (lp >> 6) * ka.world_size + ka.rank, lane = lp & 63u;
    r.x = (gt % ka.tiles_x) * 8u + (lane & 7u);
    r.y = (gt / ka.tiles_x) * 8u + (lane >> 3);
    r.valid = r.x < ka.width && r.y < ka.height;
    r.index = r.valid ? r.y * ka.width + r.x : 0u;
    return r;
}

// Path state: 4 planes of float4 (o + seed, d + bounce, light, contribution).
__device__ __forceinline__ void tl_load_path(const TreeletArgs& ta, uint32_t s, Path& p) {
    const float4* pl = ta.paths;
    const size_t n = ta.n_slots;
    const float4 a = pl[s], b = pl[n + s], l = pl[2 * n + s], k = pl[3 * n + s];
    p.o = mk(a.x, a.y, a.z);
    p.seed = __float_as_uint(a.w);
    p.d = mk(b.x, b.y, b.z);
    p.bounce = __float_as_uint(b.w);
    p.light = f4{l.x, l.y, l.z, l.w};
    p.contrib = f4{k.x, k.y, k.z, k.w};
}
__device__ __forceinline__ void tl_store_path(const TreeletArgs& ta, uint32_t s, const Path& p) {
    float4* pl = ta.paths;
    const size_t n = ta.n_slots;
    pl[s] = make_float4(p.o.x, p.o.y, p.o.z, __uint_as_float(p.seed));
    pl[n + s] = make_float4(p.d.x, p.d.y, p.d.z, __uint_as_float(p.bounce));
    pl[2 * n + s] = make_float4(p.light.x, p.light.y, p.light.z, p.light.w);
    pl[3 * n + s] = make_float4(p.contrib.x, p.contrib.y, p.contrib.z, p.contrib.w);
}

// Walk state plane 0: the best triangle {t, sweep position, triangle | front << 31, object |
// nan << 31}; plane 1: {top position to resume at, treelet queued on (kTlNone: none), rank in
// its queue, -}.
__device__ __forceinline__ void tl_load_best(const TreeletArgs& ta, uint32_t s, TraceState& ts) {
    const uint4 w = ta.walk[s];
    ts.tri = TriHit{__uint_as_float(w.x), w.y, w.z & 0x7fffffffu, w.w & 0x7fffffffu, (w.z >> 31) != 0u};
    ts.nan_hit = (w.w >> 31) != 0u;
}
__device__ __forceinline__ void tl_store_best(const TreeletArgs& ta, uint32_t s, const TraceState& ts) {
    ta.walk[s] = make_uint4(__float_as_uint(ts.tri.t), ts.tri.seq, ts.tri.tri | (ts.tri.front ? 0x80000000u : 0u),
                            ts.tri.obj | (ts.nan_hit ? 0x80000000u : 0u));
}

// The triangle walk's slab constants (phase_setup's phase 0: box culling with the margin).
__device__ __forceinline__ void tl_ray_setup(const KernelArgs& ka, f3 o, f3 d, TraceState& ts) {
    ts.inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);  // ray_in_bounds (:407-419) needs the IEEE quotient
    const float m = kTriMarginScale * (sqrt_up(dot(o, o)) + *ka.tri_extent) + 1.0e-30f;
    ts.slab = slab_ray(o.x, o.y, o.z, ts.inv.x, ts.inv.y, ts.inv.z, m);
}

__device__ __forceinline__ uint32_t tl_octant(f3 inv) {
    return (__float_as_uint(inv.x) >> 31) | ((__float_as_uint(inv.y) >> 31) << 1) | ((__float_as_uint(inv.z) >> 31) << 2);
}

}  // namespace

// Shading: the first segments (kFirst: every slot of the batch, traced by the primary pre-pass)
// or the rays the top walk finished last round. A path that goes on gets its next ray queued for
// the top walk (list A[q]); a finished one stores its light.
template <bool kFirst>
__global__ void __launch_bounds__(kTlThreads) rt_tl_shade_kernel(KernelArgs ka, TreeletArgs ta) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t block_rays;
    const uint32_t tid = threadIdx.x;
    const uint32_t q = ta.round & 1u;
    const uint32_t count = kFirst ? ta.n_slots : ta.ctl[2u + q];
    if (blockIdx.x * kTlThreads >= count) return;
    float* l_cam;
    const SceneView sv = brute_stage<true, kTlThreads>(ka, lds, tid, l_cam);
    if (tid == 0) block_rays = 0;
    __syncthreads();
    const uint32_t samples = ka.compute_per_frame;
    const uint32_t* in = tl_shade_list(ta, q);
    uint32_t rays = 0;
    for (uint32_t base = blockIdx.x * kTlThreads; base < count; base += gridDim.x * kTlThreads) {
        const uint32_t i = base + tid;
        bool active = i < count;
        const uint32_t slot = active ? (kFirst ? i : in[i]) : 0u;
        Path p;
        TraceState ts;
        if (kFirst) {
            const TlPixel px = tl_pixel(ka, slot, samples);
            active = active && px.valid;
            if (active) {
                start_sample(ka, px.index, ka.accumulation_index + px.frame + px.sample,
                             pixel_ray(ka, l_cam, px.index, px.x, px.y), p);
                const uint4 r = ka.primary[slot];
                primary_state(PrimaryRecord{__uint_as_float(r.x), r.y, r.z, r.w}, ts);
            }
        } else if (active) {
            tl_load_path(ta, slot, p);
            tl_load_best(ta, slot, ts);
            // the brute-force sphere set (trace_begin's sweep; these scenes have no sphere BVH)
            ts.sph = SphereHit{kF32Max, 0u, 0u};
            const float a = dot(p.d, p.d);
            uint32_t k = 0;
            for (; k + 4u <= ka.sphere_always; k += 4u) test_sphere_group(sv, k, p.o, p.d, 4.0f * a, 2.0f * a, ts.sph);
            if (ka.sphere_always - k >= 2u) {
                test_sphere_group(sv, k, p.o, p.d, 4.0f * a, 2.0f * a, ts.sph);
            } else if (ka.sphere_always - k == 1u) {
                float b;
                const float disc = sphere_disc(sv.sph[k], p.o, p.d, 4.0f * a, b);
                sphere_candidate(disc, b, 2.0f * a, sv.orig[k], k, ts.sph);
            }
        }
        bool go_on = false;
        if (active) {
            ++rays;
            const Hit h = trace_end<true>(sv, ka, p.o, p.d, ts);
            if (shade<true>(sv, ka, p, h)) {
                ka.frame_light[slot] = make_float4(p.light.x, p.light.y, p.light.z, p.light.w);
            } else {
                go_on = true;
                tl_store_path(ta, slot, p);
                ta.walk[slot] = make_uint4(__float_as_uint(kF32Max), 0u, 0u, 0u);
                const f3 inv = mk(1.0f / p.d.x, 1.0f / p.d.y, 1.0f / p.d.z);
                ta.walk[ta.n_slots + slot] = make_uint4(tl_octant(inv) * ta.top_stride, kTlNone, 0u, 0u);
            }
        }
        tl_append(tl_walk_list(ta, q), ta.ctl + q, go_on, slot);
    }
    atomicAdd(&block_rays, rays);
    __syncthreads();
    if (tid == 0 && block_rays) atomicAdd(ka.ray_counter, (unsigned long long)block_rays);
}

// The top walk: every ray of A[q] from its resume position in its direction's top layout, until
// it enters a treelet (queued there, counted in sub_cnt) or its walk is over (queued for shading
// next round: R[q ^ 1]). Leaves above the cut are tested on the spot.
__global__ void __launch_bounds__(kTlThreads) rt_tl_top_kernel(KernelArgs ka, TreeletArgs ta) {
    __shared__ uint32_t s_next;
    const uint32_t q = ta.round & 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) ta.ctl[2u + q] = 0u;  // R[q] was shaded (the previous kernel)
    const uint32_t count = ta.ctl[q];
    // the block's share of A[q]; each lane takes the share's next ray when its walk stops
    const uint32_t per = (count + gridDim.x - 1u) / gridDim.x;
    const uint32_t lo = min(count, blockIdx.x * per), hi = min(count, lo + per);
    if (lo >= hi) return;
    if (threadIdx.x == 0) s_next = lo;
    __syncthreads();
    const SceneView sv{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ka.objects, nullptr, nullptr,
                       ka.tri_prims, *ka.tri_extent, ka.sub_objects};
    const uint32_t* in = tl_walk_list(ta, q);
    const size_t n = ta.n_slots;
    uint32_t slot = 0u, pos = kTlEnd, target = kTlNone;
    bool live = false;
    f3 o = mk(0.0f, 0.0f, 0.0f), d = o;
    TraceState ts;
    for (;;) {
        const uint64_t idle = __ballot(!live);
        if (idle != 0u) {
            const uint32_t lead = (uint32_t)__builtin_ctzll(idle);
            uint32_t b0 = 0u;
            if ((threadIdx.x & 63u) == lead) b0 = atomicAdd(&s_next, (uint32_t)__popcll(idle));
            b0 = (uint32_t)__builtin_amdgcn_readlane((int)b0, (int)lead);
            const uint32_t k = b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!live && k < hi) {
                slot = in[k];
                const float4 a = ta.paths[slot], b = ta.paths[n + slot];
                o = mk(a.x, a.y, a.z);
                d = mk(b.x, b.y, b.z);
                tl_load_best(ta, slot, ts);
                tl_ray_setup(ka, o, d, ts);
                pos = ta.walk[n + slot].x;
                target = kTlNone;
                live = true;
            }
        }
        if (__ballot(live) == 0u) break;
        for (uint32_t step = 0; step < kTlTopSteps && live && target == kTlNone && pos < kTlEnd; ++step) {
            const float4 blo = ta.top[2u * pos], bhi = ta.top[2u * pos + 1u];
            float near_t, far_t;
            slab_hit(ts.slab, blo.x, blo.y, blo.z, bhi.x, bhi.y, bhi.z, near_t, far_t);
            const bool hit = near_t <= far_t && far_t >= 0.0f;
            const uint32_t leaf = __float_as_uint(bhi.w);
            if (hit && leaf == kTlInternal) {
                pos += 1u;
                continue;
            }
            if (hit && (leaf & kTlTreelet)) target = leaf & ~kTlTreelet;
            else if (hit) tri_leaf<true>(sv, ka, o, d, ts, leaf & 0xffffffu);  // a leaf above the cut (its record index)
            pos = __float_as_uint(blo.w);
        }
        const bool stop = live && (target != kTlNone || pos >= kTlEnd);
        const bool finished = stop && target == kTlNone;
        if (finished && ts.nan_hit) {  // measure-zero case: the sweep decides
            ts.tri = sweep_triangles(sv, ka, o, d);
            ts.nan_hit = false;
        }
        // queue ranks: one atomic per distinct treelet of the wave (coherent rays enter the same
        // treelets; an atomic per ray serialises on the hot ones)
        const uint32_t rank = tl_enqueue(ta.sub_cnt, stop ? target : kTlNone);
        if (stop) {
            tl_store_best(ta, slot, ts);
            ta.walk[n + slot] = finished ? make_uint4(kTlEnd, kTlNone, 0u, 0u) : make_uint4(pos, target, rank, 0u);
        }
        tl_append(tl_shade_list(ta, q ^ 1u), ta.ctl + 2u + (q ^ 1u), finished, slot);
        if (stop) live = false;
    }
}

// Exclusive prefix of the treelets' queue lengths, and the round's work list: each treelet's
// queue cut into chunks of at most kTlChunk rays, {treelet, first entry, rays} (a hot treelet --
// the ground under the camera -- is walked by many workgroups at once). One workgroup of 1024
// threads; it also zeroes the queue lengths for the next round's top walk (their last reader).
__global__ void __launch_bounds__(1024) rt_tl_scan_kernel(TreeletArgs ta) {
    __shared__ uint32_t part[1024], cpart[1024];
    const uint32_t tid = threadIdx.x, n = ta.n_sub;
    const uint32_t per = (n + 1023u) / 1024u, lo = min(n, tid * per), hi = min(n, lo + per);
    uint32_t s = 0, c = 0;
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t m = ta.sub_cnt[k];
        s += m;
        c += (m + kTlChunk - 1u) / kTlChunk;
    }
    part[tid] = s;
    cpart[tid] = c;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {
        const uint32_t add = tid >= off ? part[tid - off] : 0u;
        const uint32_t cadd = tid >= off ? cpart[tid - off] : 0u;
        __syncthreads();
        part[tid] += add;
        cpart[tid] += cadd;
        __syncthreads();
    }
    uint32_t run = part[tid] - s, crun = cpart[tid] - c;  // exclusive
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t m = ta.sub_cnt[k];
        ta.sub_off[k] = run;
        for (uint32_t j = 0; j < m; j += kTlChunk) ta.chunks[crun++] = make_uint4(k, run + j, min(kTlChunk, m - j), 0u);
        run += m;
        ta.sub_cnt[k] = 0u;
    }
    if (tid == 1023u) ta.ctl[4] = cpart[1023];
}

// Queue entries in treelet order: entries[sub_off[t] + rank] = slot.
__global__ void __launch_bounds__(kTlThreads) rt_tl_scatter_kernel(TreeletArgs ta) {
    const uint32_t q = ta.round & 1u;
    const uint32_t count = ta.ctl[q];
    const uint32_t* in = tl_walk_list(ta, q);
    uint32_t* entries = tl_entries(ta);
    for (uint32_t i = blockIdx.x * kTlThreads + threadIdx.x; i < count; i += gridDim.x * kTlThreads) {
        const uint32_t slot = in[i];
        const uint4 w = ta.walk[ta.n_slots + slot];
        if (w.y != kTlNone) entries[ta.sub_off[w.y] + w.z] = slot;
    }
}

// One leaf of a treelet from LDS: the object box (:431), the leaf's candidates as the
// cooperative leaf batch tests and merges them (tri_leaf's operations, :449-481), and the
// sub-object box (:441) only when a candidate would change the result.
__device__ __forceinline__ void tl_leaf_lds(const SceneView& sv, const KernelArgs& ka, f3 o, f3 d, TraceState& ts,
                                            const uint4 pr, const uint4* blk, uint32_t record) {
    const RtObject& ob = ka.objects[pr.x];  // object, sub-object, sweep position, range
    if (!ray_in_bounds(o, ts.inv, ob.min_bounds, ob.max_bounds)) return;
    if (pr.w == kPrimRangeNone || (pr.w >> 27) >= kLeafTriSlots) {
        tri_leaf<true>(sv, ka, o, d, ts, record);  // no triangle block: from global memory
        return;
    }
    const uint32_t cnt = pr.w >> 27, first = pr.w & ((1u << 27) - 1u);
    float cd = __builtin_inff();
    uint32_t cs = 0xffffffffu, ct = 0u;
    bool cnan = false;
    for (uint32_t j = 0; j < cnt; ++j) {
        const uint4 q0 = blk[j], q1 = blk[kLeafTriSlots + j], q2 = blk[2u * kLeafTriSlots + j];
        const f3 ta_ = mk(__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z));
        const f3 cn = mk(__uint_as_float(q2.y), __uint_as_float(q2.z), __uint_as_float(q2.w));
        const float det = -dot(d, cn);
        const float inv_det = 1.0f / det;
        const f3 ao = o - ta_;
        const float dist = dot(ao, cn) * inv_det;
        // (a distance beyond the best hit cannot win; NaN goes on)
        if (dist < 0.0f || dist > ts.tri.t) continue;
        const f3 ab = mk(__uint_as_float(q0.w), __uint_as_float(q1.x), __uint_as_float(q1.y));
        const f3 ac = mk(__uint_as_float(q1.z), __uint_as_float(q1.w), __uint_as_float(q2.x));
        const f3 dao = cross(ao, d);
        const float v = -dot(ab, dao) * inv_det;
        if (v < 0.0f) continue;
        const float u = dot(ac, dao) * inv_det;
        if (u < 0.0f) continue;
        const float w = 1.0f - u - v;
        if (w < 0.0f) continue;
        if (dist != dist) {
            cnan = true;
        } else {
            const uint32_t seq = pr.z + j;
            if (dist < cd || (dist == cd && seq < cs)) {
                cd = dist;
                cs = seq;
                ct = min(first + j, ka.triangle_count - 1u) | (det > 0.0f ? 0x80000000u : 0u);
            }
        }
    }
    const bool beats = cd < ts.tri.t || (cd == ts.tri.t && cs < ts.tri.seq);
    if (cnan || beats) {
        const RtSubObject so = ka.sub_objects[pr.y];
        if (ray_in_bounds(o, ts.inv, so.min_bounds, so.max_bounds)) {
            if (cnan) ts.nan_hit = true;
            if (beats) ts.tri = TriHit{cd, cs, ct & 0x7fffffffu, pr.x, (ct >> 31) != 0u};
        }
    }
}

// The treelet walks, a chunk of a treelet's queue per workgroup step: the treelet's nodes (the
// base layout's pre-order range), leaf records and leaf triangle blocks staged in LDS, then the
// chunk's rays walked from there; the rays go back to the top walk (A[q ^ 1]).
__global__ void __launch_bounds__(kTlThreads) rt_tl_subtree_kernel(KernelArgs ka, TreeletArgs ta) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t s_next, s_out;
    const uint32_t tid = threadIdx.x, q = ta.round & 1u;
    if (blockIdx.x == 0 && tid == 0) ta.ctl[q] = 0u;  // A[q] was walked and scattered (the previous kernels)
    const uint32_t n_chunks = ta.ctl[4];
    const SceneView sv{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ka.objects, nullptr, nullptr,
                       ka.tri_prims, *ka.tri_extent, ka.sub_objects};
    const uint32_t* all_entries = tl_entries(ta);
    uint32_t* out_list = tl_walk_list(ta, q ^ 1u);
    uint32_t staged = kTlNone;
    for (uint32_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        const uint4 ch = ta.chunks[c];  // treelet, first entry, rays
        const uint32_t t = ch.x, n = ch.z;
        const uint4 st = ta.subtrees[t];  // root (base layout), nodes, first leaf record, leaf records
        const uint32_t root = st.x, nn = st.y, p0 = st.z, np = st.w;
        float4* l_nodes = reinterpret_cast<float4*>(lds);
        uint4* l_prims = reinterpret_cast<uint4*>(lds + (size_t)nn * 32u);
        uint4* l_tris = l_prims + np;
        __syncthreads();  // the previous chunk's readers are done (LDS image, s_next, s_out)
        if (t != staged) {
            const float4* g_nodes = ta.base_nodes + 2u * (size_t)root;
            for (uint32_t k = tid; k < 2u * nn; k += kTlThreads) l_nodes[k] = g_nodes[k];
            for (uint32_t k = tid; k < np; k += kTlThreads) l_prims[k] = ka.tri_prims[p0 + k];
            const uint4* g_tris = ka.tri_leaftris + (size_t)p0 * kLeafTriWords;
            for (uint32_t k = tid; k < np * kLeafTriWords; k += kTlThreads) l_tris[k] = g_tris[k];
            staged = t;
        }
        // every ray of the chunk goes back to the top walk: one append for the chunk
        if (tid == 0) {
            s_next = 0u;
            s_out = atomicAdd(ta.ctl + (q ^ 1u), n);
        }
        __syncthreads();
        const uint32_t* entries = all_entries + ch.y;
        for (uint32_t k = tid; k < n; k += kTlThreads) out_list[s_out + k] = entries[k];
        // Each lane walks one ray at a time and takes the chunk's next ray when it is done
        // (claims by wave, from an LDS counter). Up to kTlSteps node steps per check; a lane that
        // reaches a leaf waits with it, and the waiting lanes' leaves are tested together once
        // they are at least as many as the walking lanes. The walk culls by box only, so the
        // leaves' order does not matter (lexicographic minimum).
        uint32_t slot = 0u, node = nn, pend = kTlNone;
        bool live = false;
        f3 o = mk(0.0f, 0.0f, 0.0f), d = o;
        TraceState ts;
        for (;;) {
            const uint64_t idle = __ballot(!live);
            if (idle != 0u) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(idle);
                uint32_t b0 = 0u;
                if ((tid & 63u) == lead) b0 = atomicAdd(&s_next, (uint32_t)__popcll(idle));
                b0 = (uint32_t)__builtin_amdgcn_readlane((int)b0, (int)lead);
                const uint32_t k = b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (!live && k < n) {
                    slot = entries[k];
                    const size_t ns = ta.n_slots;
                    const float4 a = ta.paths[slot], b = ta.paths[ns + slot];
                    o = mk(a.x, a.y, a.z);
                    d = mk(b.x, b.y, b.z);
                    tl_load_best(ta, slot, ts);
                    tl_ray_setup(ka, o, d, ts);
                    node = 0u;
                    pend = kTlNone;
                    live = true;
                }
            }
            if (__ballot(live) == 0u) break;
            for (uint32_t step = 0; step < kTlSteps && live && pend == kTlNone && node < nn; ++step) {
                const float4 lo = l_nodes[2u * node], hi = l_nodes[2u * node + 1u];
                float near_t, far_t;
                slab_hit(ts.slab, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, near_t, far_t);
                const bool hit = near_t <= far_t && far_t >= 0.0f;
                const uint32_t leaf = __float_as_uint(hi.w);
                if (hit && leaf == kTlInternal) {
                    node += 1u;
                    continue;
                }
                if (hit) pend = (leaf & 0xffffffu) - p0;  // (a leaf word: record | count << 24)
                node = __float_as_uint(lo.w) - root;      // the skip link, local
            }
            const uint64_t waiting = __ballot(pend != kTlNone);
            const uint64_t walking = __ballot(live && pend == kTlNone && node < nn);
            if (waiting != 0u && (walking == 0u || __popcll(waiting) >= __popcll(walking)) && pend != kTlNone) {
                tl_leaf_lds(sv, ka, o, d, ts, l_prims[pend], l_tris + (size_t)pend * kLeafTriWords, p0 + pend);
                pend = kTlNone;
            }
            if (live && pend == kTlNone && node >= nn) {  // left the treelet: its best hit so far
                tl_store_best(ta, slot, ts);
                live = false;
            }
        }
    }
}

// The top layouts' boxes from the base accelerator's nodes (after every upload or refit; the
// links are the host's): node i = box of base node src[i], skip link and leaf word from links[i].
__global__ void __launch_bounds__(256) rt_tl_derive_top_kernel(const float4* __restrict__ base, const uint32_t* __restrict__ src,
                                                               const uint2* __restrict__ links, float4* __restrict__ top,
                                                               uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const float4 lo = base[2u * src[i]], hi = base[2u * src[i] + 1u];
    const uint2 l = links[i];
    top[2u * i] = make_float4(lo.x, lo.y, lo.z, __uint_as_float(l.x));
    top[2u * i + 1u] = make_float4(hi.x, hi.y, hi.z, __uint_as_float(l.y));
}

// Closes a timed batch's device span (rt_set_timing): stream-ordered after its last kernel.
__global__ void rt_tl_stamp_kernel(unsigned long long* clock) {
    if (threadIdx.x == 0) atomicMax(clock + 1, (unsigned long long)wall_clock64());
}

hipError_t rt_launch_tl_derive_top(const float4* base, const uint32_t* src, const uint2* links, float4* top, uint32_t n,
                                   hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_tl_derive_top_kernel, dim3((n + 255u) / 256u), dim3(256), 0, stream, base, src, links, top, n);
    return hipGetLastError();
}

size_t rt_tl_subtree_lds_bytes(uint32_t nodes, uint32_t prims) {
    return (size_t)nodes * 32u + (size_t)prims * 16u + (size_t)prims * kLeafTriWords * 16u;
}

// One round of the wavefront (host loop: rt_abi.cpp dispatch_treelet). kind 0: shade the
// first segments, 1: shade R[q], 2: top walk, 3: scan, 4: scatter, 5: treelet walks, 6: stamp.
hipError_t rt_launch_tl(int kind, const KernelArgs& ka, const TreeletArgs& ta, uint32_t blocks, size_t lds_bytes,
                        hipStream_t stream) {
    switch (kind) {
        case 0:
        case 1: {
            const void* fn = kind == 0 ? reinterpret_cast<const void*>(&rt_tl_shade_kernel<true>)
                                       : reinterpret_cast<const void*>(&rt_tl_shade_kernel<false>);
            if (lds_bytes > 64u * 1024u) {
                const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
                if (e != hipSuccess) return e;
            }
            if (kind == 0)
                hipLaunchKernelGGL(rt_tl_shade_kernel<true>, dim3(blocks), dim3(kTlThreads), lds_bytes, stream, ka, ta);
            else
                hipLaunchKernelGGL(rt_tl_shade_kernel<false>, dim3(blocks), dim3(kTlThreads), lds_bytes, stream, ka, ta);
            break;
        }
        case 2:
            hipLaunchKernelGGL(rt_tl_top_kernel, dim3(blocks), dim3(kTlThreads), 0, stream, ka, ta);
            break;
        case 3:
            hipLaunchKernelGGL(rt_tl_scan_kernel, dim3(1), dim3(1024), 0, stream, ta);
            break;
        case 4:
            hipLaunchKernelGGL(rt_tl_scatter_kernel, dim3(blocks), dim3(kTlThreads), 0, stream, ta);
            break;
        case 5:
            if (lds_bytes > 64u * 1024u) {
                const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&rt_tl_subtree_kernel),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(rt_tl_subtree_kernel, dim3(blocks), dim3(kTlThreads), lds_bytes, stream, ka, ta);
            break;
        case 6:
            hipLaunchKernelGGL(rt_tl_stamp_kernel, dim3(1), dim3(64), 0, stream, ka.launch_clock);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
