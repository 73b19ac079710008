#include <functional>
// sphere_bvh.cpp — binned-SAH BVH over spheres, flattened depth-first with
// skip links for stackless traversal on the GPU.
#include "sphere_bvh.h"

#include <algorithm>
#include <limits>
#include <cmath>
#include <numeric>

namespace {

constexpr uint32_t kSweepMax = 4096;  // larger subtrees split by the binned SAH (build time)

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const double* a, const double* b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], a[k]);
            hi[k] = std::max(hi[k], b[k]);
        }
    }
    void grow(const Box& o) { grow(o.lo, o.hi); }
    double area() const {
        if (lo[0] > hi[0]) return 0.0;
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct Prim {
    Box box;
    double c[3];
    uint32_t orig;
};

struct Builder {
    std::vector<Prim>& prims;
    std::vector<SphereBvhNode>& nodes;
    std::vector<uint32_t> leaf_order;
    uint32_t leaf_max = kSphereBvhLeafMax;
    bool sweep_sah = true;  // exact SAH over sorted centroids on all three axes (subtrees <= kSweepMax)
    uint32_t max_depth = 0xffffffffu;

    // Builds the subtree over prims[begin, end) at node index `at` (pre-order),
    // `depth` levels below the root.
    void build(uint32_t begin, uint32_t end, uint32_t depth = 0) {
        const uint32_t at = (uint32_t)nodes.size();
        nodes.push_back(SphereBvhNode{});
        Box box, cbox;
        for (uint32_t i = begin; i < end; i++) {
            box.grow(prims[i].box);
            cbox.grow(prims[i].c, prims[i].c);
        }
        for (int k = 0; k < 3; k++) {  // round outward to f32
            nodes[at].bmin[k] = std::nextafter((float)box.lo[k], -INFINITY);
            nodes[at].bmax[k] = std::nextafter((float)box.hi[k], INFINITY);
        }
        const uint32_t n = end - begin;
        if (n <= leaf_max) {
            nodes[at].leaf = (uint32_t)leaf_order.size() | (n << 24);
            for (uint32_t i = begin; i < end; i++) leaf_order.push_back(prims[i].orig);
            nodes[at].skip = (uint32_t)nodes.size();
            return;
        }
        // levels a balanced split of the rest needs: ceil(log2(ceil(n / leaf_max)))
        uint32_t need = 0;
        for (uint64_t c = ((uint64_t)n + leaf_max - 1) / leaf_max; c > 1; c = (c + 1) / 2) need++;
        if (max_depth != 0xffffffffu && depth + need + 1 >= max_depth) {
            // median split on the widest centroid axis: depth stays bounded
            int axis = 0;
            for (int k = 1; k < 3; k++)
                if (cbox.hi[k] - cbox.lo[k] > cbox.hi[axis] - cbox.lo[axis]) axis = k;
            std::stable_sort(prims.begin() + begin, prims.begin() + end,
                             [&](const Prim& a, const Prim& b) { return a.c[axis] < b.c[axis]; });
            const uint32_t mid = begin + n / 2;
            nodes[at].leaf = kSphereBvhInternal;
            build(begin, mid, depth + 1);
            build(mid, end, depth + 1);
            nodes[at].skip = (uint32_t)nodes.size();
            return;
        }
        if (sweep_sah && n <= kSweepMax) {
            // exact SAH: every split of the centroid order on each axis, cost
            // area(left) * n_left + area(right) * n_right (replayed C2 rays: 17.3 ->
            // 16.1 node visits and 5.66 -> 5.47 sphere tests per ray against the
            // 16-bin SAH on the widest axis below)
            double best = INFINITY;
            int best_axis = -1;
            uint32_t best_i = 0;
            std::vector<double> right_area(n + 1);
            for (int ax = 0; ax < 3; ax++) {
                std::stable_sort(prims.begin() + begin, prims.begin() + end,
                                 [&](const Prim& a, const Prim& b) { return a.c[ax] < b.c[ax]; });
                Box r;
                for (uint32_t i = n; i > 0; i--) {
                    r.grow(prims[begin + i - 1].box);
                    right_area[i - 1] = r.area();
                }
                Box l;
                for (uint32_t i = 1; i < n; i++) {
                    l.grow(prims[begin + i - 1].box);
                    const double cost = l.area() * i + right_area[i] * (n - i);
                    if (cost < best) {
                        best = cost;
                        best_axis = ax;
                        best_i = i;
                    }
                }
            }
            std::stable_sort(prims.begin() + begin, prims.begin() + end,
                             [&](const Prim& a, const Prim& b) { return a.c[best_axis] < b.c[best_axis]; });
            const uint32_t mid = begin + best_i;
            nodes[at].leaf = kSphereBvhInternal;
            build(begin, mid, depth + 1);
            build(mid, end, depth + 1);
            nodes[at].skip = (uint32_t)nodes.size();
            return;
        }
        // binned SAH along the widest centroid axis
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (cbox.hi[k] - cbox.lo[k] > cbox.hi[axis] - cbox.lo[axis]) axis = k;
        const double span = cbox.hi[axis] - cbox.lo[axis];
        uint32_t mid = begin + n / 2;
        if (span > 0.0) {
            constexpr int kBins = 16;
            Box bins[kBins];
            uint32_t cnt[kBins] = {};
            auto bin_of = [&](const Prim& p) {
                int b = (int)((p.c[axis] - cbox.lo[axis]) / span * kBins);
                return std::min(std::max(b, 0), kBins - 1);
            };
            for (uint32_t i = begin; i < end; i++) {
                const int b = bin_of(prims[i]);
                bins[b].grow(prims[i].box);
                cnt[b]++;
            }
            double best = INFINITY;
            int best_split = -1;
            for (int s = 1; s < kBins; s++) {
                Box l, r;
                uint32_t nl = 0, nr = 0;
                for (int b = 0; b < s; b++) {
                    if (cnt[b]) l.grow(bins[b]);
                    nl += cnt[b];
                }
                for (int b = s; b < kBins; b++) {
                    if (cnt[b]) r.grow(bins[b]);
                    nr += cnt[b];
                }
                if (nl == 0 || nr == 0) continue;
                const double cost = l.area() * nl + r.area() * nr;
                if (cost < best) {
                    best = cost;
                    best_split = s;
                }
            }
            if (best_split > 0) {
                auto it = std::stable_partition(prims.begin() + begin, prims.begin() + end,
                                                [&](const Prim& p) { return bin_of(p) < best_split; });
                mid = (uint32_t)(it - prims.begin());
            } else {
                std::stable_sort(prims.begin() + begin, prims.begin() + end,
                                 [&](const Prim& a, const Prim& b) { return a.c[axis] < b.c[axis]; });
            }
        }
        if (mid == begin || mid == end) mid = begin + n / 2;
        nodes[at].leaf = kSphereBvhInternal;
        build(begin, mid, depth + 1);
        build(mid, end, depth + 1);
        nodes[at].skip = (uint32_t)nodes.size();
    }
};

}  // namespace

void build_box_bvh(const std::vector<float>& lo, const std::vector<float>& hi, uint32_t leaf_max,
                   std::vector<SphereBvhNode>* nodes, std::vector<uint32_t>* leaf_order, uint32_t max_depth) {
    const size_t n = lo.size() / 3;
    std::vector<Prim> prims(n);
    for (size_t i = 0; i < n; i++) {
        for (int k = 0; k < 3; k++) {
            prims[i].box.lo[k] = lo[3 * i + k];
            prims[i].box.hi[k] = hi[3 * i + k];
            prims[i].c[k] = 0.5 * ((double)lo[3 * i + k] + (double)hi[3 * i + k]);
        }
        prims[i].orig = (uint32_t)i;
    }
    nodes->clear();
    leaf_order->clear();
    if (n == 0) return;
    Builder b{prims, *nodes, {}, leaf_max};
    b.max_depth = max_depth;
    b.build(0, (uint32_t)n);
    *leaf_order = std::move(b.leaf_order);
}

bool box_layout_orderable(const std::vector<SphereBvhNode>& nodes) {
    for (const SphereBvhNode& nd : nodes)
        for (int k = 0; k < 3; k++)
            if (!(nd.bmin[k] <= nd.bmax[k]) || !(std::fabs(nd.bmin[k]) <= 1e8f) || !(std::fabs(nd.bmax[k]) <= 1e8f))
                return false;
    return true;
}

void order_bvh_by_octant(const std::vector<SphereBvhNode>& in, std::vector<SphereBvhNode>* out, bool swap_boxes,
                         std::vector<uint32_t>* src_index) {
    out->clear();
    if (src_index) src_index->clear();
    const uint32_t n = (uint32_t)in.size();
    if (n == 0) return;
    out->reserve(8 * (size_t)n);
    const uint32_t end_all = 8u * n;
    for (uint32_t oct = 0; oct < 8; oct++) {
        const uint32_t base = (uint32_t)out->size();
        // pre-order re-emission (recursion depth = tree depth)
        std::function<void(uint32_t)> emit = [&](uint32_t src) {
            const uint32_t at = (uint32_t)out->size();
            out->push_back(in[src]);
            if (src_index) src_index->push_back(src);
            if (swap_boxes)  // (near corner, far corner) for this octant
                for (int k = 0; k < 3; k++)
                    if ((oct >> k) & 1u) std::swap(out->back().bmin[k], out->back().bmax[k]);
            if (in[src].leaf == kSphereBvhInternal) {
                uint32_t a = src + 1, b = in[src + 1].skip;  // left child, right child
                int axis = 0;
                double best = -1.0, diff = 0.0;
                for (int k = 0; k < 3; k++) {
                    const double ca = 0.5 * ((double)in[a].bmin[k] + (double)in[a].bmax[k]);
                    const double cb = 0.5 * ((double)in[b].bmin[k] + (double)in[b].bmax[k]);
                    if (std::fabs(cb - ca) > best) {
                        best = std::fabs(cb - ca);
                        axis = k;
                        diff = cb - ca;
                    }
                }
                const bool negative = (oct >> axis) & 1u;  // this octant's rays travel towards -axis
                if ((diff < 0.0) != negative) std::swap(a, b);  // a: met first along the travel direction
                emit(a);
                emit(b);
            }
            const uint32_t after = (uint32_t)out->size();
            (*out)[at].skip = after == base + n ? end_all : after;
        };
        emit(0);
    }
}

void build_triangle_accel(const rt_object_info* objects, uint32_t object_count, const rt_sub_object_info* subs,
                          uint32_t sub_count, TriangleAccel* out) {
    out->prims.clear();
    out->nodes.clear();
    out->extent = 0.0f;
    std::vector<SubObjectPrim> prims;
    std::vector<float> lo, hi;
    double extent = 0.0;
    uint32_t seq = 0;
    for (uint32_t o = 0; o < object_count; o++) {
        for (uint32_t i = 0; i < objects[o].sub_object_count; i++) {
            const uint32_t si = objects[o].first_sub_object_index + i;
            if (si >= sub_count) break;  // validated on the host; never taken
            const rt_sub_object_info& s = subs[si];
            const uint32_t base = seq;
            seq += s.triangle_count;
            if (s.triangle_count == 0) continue;
            bool finite = true;
            for (int k = 0; k < 3; k++) finite = finite && std::isfinite(s.min_bounds[k]) && std::isfinite(s.max_bounds[k]);
            prims.push_back(SubObjectPrim{o, si, base, prim_range(s.first_triangle_index, s.triangle_count)});
            for (int k = 0; k < 3; k++) {
                // the reference's slab test is symmetric in min/max (:414-415); a
                // non-finite box can still pass it on its other axes (NaN operands
                // are ignored), so it gets a box that every ray enters
                const float a = finite ? std::min(s.min_bounds[k], s.max_bounds[k]) : -3.0e38f;
                const float b = finite ? std::max(s.min_bounds[k], s.max_bounds[k]) : 3.0e38f;
                lo.push_back(a);
                hi.push_back(b);
                if (finite) extent = std::max(extent, std::max(std::fabs((double)a), std::fabs((double)b)));
            }
        }
    }
    std::vector<uint32_t> order;
    build_box_bvh(lo, hi, 1, &out->nodes, &order);
    out->prims.reserve(order.size());
    for (uint32_t p : order) out->prims.push_back(prims[p]);
    out->extent = std::nextafter((float)extent, INFINITY);
}

void build_sphere_slots(const rt_scene_sphere* s, uint32_t count, bool use_bvh, SphereSlots* out, uint32_t leaf_max) {
    out->n_always = 0;
    out->slot_sph.clear();
    out->slot_orig.clear();
    out->nodes.clear();
    out->extent = 0.0f;

    auto push_slot = [&](uint32_t i) {
        const rt_scene_sphere& sp = s[i];
        out->slot_sph.insert(out->slot_sph.end(),
                             {sp.position[0], sp.position[1], sp.position[2], sp.radius * sp.radius});
        out->slot_orig.push_back(i);
    };

    // Extent of each sphere from the origin; the handful of huge/far spheres
    // (a ground sphere of radius 1000) stay in the brute-force set so that the
    // per-ray BVH margin, proportional to the BVH spheres' extent, stays small.
    std::vector<double> ext(count);
    for (uint32_t i = 0; i < count; i++) {
        const rt_scene_sphere& sp = s[i];
        ext[i] = std::sqrt((double)sp.position[0] * sp.position[0] + (double)sp.position[1] * sp.position[1] +
                           (double)sp.position[2] * sp.position[2]) +
                 std::fabs((double)sp.radius);
    }
    std::vector<bool> in_bvh(count, false);
    if (use_bvh && count >= 16) {
        std::vector<double> sorted(ext);
        std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
        const double cap = 8.0 * std::max(sorted[count / 2], 1e-30);
        for (uint32_t i = 0; i < count; i++) in_bvh[i] = std::isfinite(ext[i]) && ext[i] <= cap;
    }
    // Pad to a multiple of kSphereGroup with slots no ray can hit (NaN centre:
    // disc is NaN, never >= 0), so the kernel reads spheres in aligned groups.
    auto pad_group = [&]() {
        while (out->slot_orig.size() % kSphereGroup) {
            const float qnan = std::numeric_limits<float>::quiet_NaN();
            out->slot_sph.insert(out->slot_sph.end(), {qnan, qnan, qnan, qnan});
            out->slot_orig.push_back(kSphereDummyOrig);
        }
    };
    for (uint32_t i = 0; i < count; i++)
        if (!in_bvh[i]) push_slot(i);
    out->n_always = (uint32_t)out->slot_orig.size();  // swept in groups of 4, then one by one
    pad_group();  // BVH leaves start group-aligned

    std::vector<Prim> prims;
    double extent = 0.0, r_min = INFINITY, r_max = 0.0;
    for (uint32_t i = 0; i < count; i++) {
        if (!in_bvh[i]) continue;
        const rt_scene_sphere& sp = s[i];
        Prim p;
        const double r = std::fabs((double)sp.radius);
        r_min = std::min(r_min, r);
        r_max = std::max(r_max, r);
        for (int k = 0; k < 3; k++) {
            p.c[k] = sp.position[k];
            p.box.lo[k] = p.c[k] - r;
            p.box.hi[k] = p.c[k] + r;
        }
        p.orig = i;
        prims.push_back(p);
        extent = std::max(extent, ext[i]);
    }
    if (prims.size() < 2) {  // nothing worth a tree: brute-force everything
        out->slot_sph.resize(4 * out->n_always);
        out->slot_orig.resize(out->n_always);
        for (const Prim& p : prims) push_slot(p.orig);
        out->n_always = (uint32_t)out->slot_orig.size();
        pad_group();
        return;
    }
    const uint32_t lmax = std::min<uint32_t>(leaf_max ? leaf_max : kSphereBvhLeafMax, kSphereGroup);
    Builder b{prims, out->nodes, {}, lmax};
    b.build(0, (uint32_t)prims.size());
    // one aligned group of kSphereGroup slots per leaf (padded), in node order
    for (SphereBvhNode& nd : out->nodes) {
        if (nd.leaf == kSphereBvhInternal) continue;
        const uint32_t first = nd.leaf & 0xffffffu, cnt = nd.leaf >> 24;
        const uint32_t slot = (uint32_t)out->slot_orig.size();
        for (uint32_t k = 0; k < cnt; k++) push_slot(b.leaf_order[first + k]);
        pad_group();
        nd.leaf = slot | (kSphereGroup << 24);
    }
    out->extent = std::nextafter((float)extent, INFINITY);
    // radii are f32 already: r_min is exact, r_max too (kept as the float value)
    out->r_min = (float)r_min;
    out->r_max = (float)r_max;
}

