// tri_wide.cpp — host builder of the 4-wide triangle accelerator (tri_wide.h).
//
// 1. Leaves: the reference's sweep order -- objects, their sub-objects, their
//    triangles (check_triangles, compute_shader.wgsl:422-517) -- cut into records
//    of at most kWideLeafTris triangles (a sub-object of more triangles becomes
//    several records with the same box: its test is per sub-object either way).
// 2. A binary SAH tree over the leaves' boxes (build_box_bvh, depth-capped),
//    collapsed into 4-wide nodes by repeatedly opening the child of largest
//    surface area; a node's internal children are allocated contiguously, and so
//    are its leaf records.
// 3. Compact leaves: the distinct vertices of a leaf's triangles (a, fl(a + ab),
//    fl(a + ac), deduplicated by bit pattern), kept only when recomputing every
//    triangle's edges and normal from them reproduces its record exactly.
#include "tri_wide.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>

#include "sphere_bvh.h"

namespace {

// The culling box of a leaf: its sub-object box with min/max ordered, or an
// all-enclosing box when a bound is not finite (the reference's slab test can
// still pass such a box on its other axes, NaN operands being ignored).
void leaf_cull_box(const float* mn, const float* mx, float* lo, float* hi, bool* finite_out) {
    bool finite = true;
    for (int k = 0; k < 3; k++) finite = finite && std::isfinite(mn[k]) && std::isfinite(mx[k]);
    for (int k = 0; k < 3; k++) {
        lo[k] = finite ? std::min(mn[k], mx[k]) : -3.0e38f;
        hi[k] = finite ? std::max(mn[k], mx[k]) : 3.0e38f;
    }
    *finite_out = finite;
}

float box_area(const float* lo, const float* hi) {
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0f;
    return (float)(2.0 * (dx * dy + dy * dz + dz * dx));
}

// a, ab, ac, cn of triangle i in the 64-B hot layout (16 floats: a.xyz ab.x |
// ab.yz ac.xy | ac.z cn.xyz | fn.xyz 0), rt_kernel_args.h RtTriangleHot.
void hot_fields(const float* hot16, uint32_t i, float* a, float* ab, float* ac, float* cn) {
    const float* p = hot16 + 16 * (size_t)i;
    a[0] = p[0], a[1] = p[1], a[2] = p[2];
    ab[0] = p[3], ab[1] = p[4], ab[2] = p[5];
    ac[0] = p[6], ac[1] = p[7], ac[2] = p[8];
    cn[0] = p[9], cn[1] = p[10], cn[2] = p[11];
}

bool same_bits(const float* x, const float* y, int n) { return std::memcmp(x, y, sizeof(float) * n) == 0; }

}  // namespace

bool wide_leaf_make_compact(const float* hot16, uint32_t n_tri, TriLeaf& leaf, std::vector<TriVertex>& verts,
                            std::vector<uint32_t>& vsrc) {
    const uint32_t count = leaf.count_flags & 0xffu;
    TriVertex v[kWideLeafVerts];
    uint32_t src[kWideLeafVerts];
    uint32_t nv = 0;
    uint32_t idx[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < count; j++) {
        const uint32_t t = leaf.first_tri + j;
        if (t >= n_tri) return false;
        float a[3], ab[3], ac[3], cn[3];
        hot_fields(hot16, t, a, ab, ac, cn);
        const TriVertex corner[3] = {{a[0], a[1], a[2]},
                                     {a[0] + ab[0], a[1] + ab[1], a[2] + ab[2]},
                                     {a[0] + ac[0], a[1] + ac[1], a[2] + ac[2]}};
        uint32_t id[3];
        for (uint32_t k = 0; k < 3; k++) {
            uint32_t f = 0;
            while (f < nv && std::memcmp(&v[f], &corner[k], sizeof(TriVertex)) != 0) f++;
            if (f == nv) {
                if (nv == kWideLeafVerts) return false;
                v[nv] = corner[k];
                src[nv] = t * 4u + k;
                nv++;
            }
            id[k] = f;
            const uint32_t n = 3u * j + k;
            idx[n >> 3] |= f << ((n & 7u) * 4u);
        }
        // the recomputation must give the record's own bits
        float rab[3], rac[3], rcn[3];
        wide_tri_from_vertices(v[id[0]], v[id[1]], v[id[2]], rab, rac, rcn);
        if (!same_bits(&v[id[0]].x, a, 3) || !same_bits(rab, ab, 3) || !same_bits(rac, ac, 3) || !same_bits(rcn, cn, 3))
            return false;
    }
    leaf.vbase = (uint32_t)verts.size();
    for (uint32_t f = 0; f < nv; f++) {
        verts.push_back(v[f]);
        vsrc.push_back(src[f]);
    }
    std::memcpy(leaf.idx, idx, sizeof(idx));
    leaf.count_flags |= kWideLeafCompact | kWideLeafCompactBuilt;
    return true;
}

void build_triangle_wide(const rt_object_info* objects, uint32_t object_count, const rt_sub_object_info* subs,
                         uint32_t sub_count, const float* hot16, uint32_t n_tri, TriWide* out) {
    *out = TriWide{};
    // 1. leaves in sweep order
    std::vector<TriLeaf> leaves;
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
            float clo[3], chi[3];
            bool finite;
            leaf_cull_box(s.min_bounds, s.max_bounds, clo, chi, &finite);
            if (finite)
                for (int k = 0; k < 3; k++)
                    extent = std::max(extent, std::max(std::fabs((double)clo[k]), std::fabs((double)chi[k])));
            for (uint32_t j0 = 0; j0 < s.triangle_count; j0 += kWideLeafTris) {
                TriLeaf L{};
                std::memcpy(L.mn, s.min_bounds, 12);
                std::memcpy(L.mx, s.max_bounds, 12);
                L.first_tri = s.first_triangle_index + j0;
                L.seq_base = base + j0;
                L.object = o;
                L.count_flags = std::min<uint32_t>(kWideLeafTris, s.triangle_count - j0);
                L.sub = si;
                leaves.push_back(L);
                lo.insert(lo.end(), clo, clo + 3);
                hi.insert(hi.end(), chi, chi + 3);
            }
        }
    }
    out->extent = std::nextafter((float)extent, INFINITY);
    if (leaves.empty()) return;

    // 2. binary SAH tree, collapsed to 4-wide
    std::vector<SphereBvhNode> bin;
    std::vector<uint32_t> order;
    build_box_bvh(lo, hi, 1, &bin, &order, kWideBinaryDepthCap);
    auto is_leaf = [&](uint32_t b) { return bin[b].leaf != kSphereBvhInternal; };
    auto area = [&](uint32_t b) { return box_area(bin[b].bmin, bin[b].bmax); };
    auto children_of = [&](uint32_t b, uint32_t* kids) {  // up to 4 binary nodes under wide node b
        uint32_t n = 0;
        if (is_leaf(b)) {
            kids[n++] = b;  // a tree that is a single leaf
            return n;
        }
        kids[n++] = b + 1;
        kids[n++] = bin[b + 1].skip;
        while (n < kWideArity) {
            int best = -1;
            float best_a = -1.0f;
            for (uint32_t i = 0; i < n; i++)
                if (!is_leaf(kids[i]) && area(kids[i]) > best_a) {
                    best_a = area(kids[i]);
                    best = (int)i;
                }
            if (best < 0) break;
            const uint32_t c = kids[best];
            kids[best] = c + 1;
            kids[n++] = bin[c + 1].skip;
        }
        // slot order: internal children first, then leaves, each in the binary tree's order
        std::sort(kids, kids + n, [&](uint32_t x, uint32_t y) {
            const bool lx = is_leaf(x), ly = is_leaf(y);
            return lx != ly ? ly : x < y;
        });
        return n;
    };
    std::vector<TriWideNode>& nodes = out->nodes;
    std::vector<uint32_t> node_depth;
    std::vector<uint32_t> bin_of;  // wide node -> the binary node it expands
    nodes.emplace_back();
    bin_of.push_back(0);
    node_depth.push_back(0);
    // breadth of allocation: a node's internal children get consecutive indices when
    // the node is filled; filling then proceeds depth-first
    std::function<void(uint32_t)> fill = [&](uint32_t w) {
        uint32_t kids[kWideArity];
        const uint32_t n = children_of(bin_of[w], kids);
        TriWideNode nd{};
        for (int k = 0; k < 3; k++)
            for (uint32_t s = 0; s < kWideArity; s++) {
                nd.lo[k][s] = 0.0f;
                nd.hi[k][s] = 0.0f;
            }
        uint32_t n_int = 0;
        for (uint32_t s = 0; s < n; s++) n_int += is_leaf(kids[s]) ? 0u : 1u;
        nd.child_base = (uint32_t)nodes.size();
        nd.leaf_base = (uint32_t)out->leaves.size();
        nd.slots = n_int | ((n - n_int) << 4);
        std::vector<uint32_t> to_fill;
        for (uint32_t s = 0; s < n; s++) {
            const uint32_t b = kids[s];
            for (int k = 0; k < 3; k++) {
                nd.lo[k][s] = bin[b].bmin[k];
                nd.hi[k][s] = bin[b].bmax[k];
            }
            if (is_leaf(b))
                out->leaves.push_back(leaves[order[bin[b].leaf & 0xffffffu]]);
            else
                to_fill.push_back(b);
        }
        for (uint32_t b : to_fill) {
            nodes.emplace_back();
            bin_of.push_back(b);
            node_depth.push_back(node_depth[w] + 1);
        }
        nodes[w] = nd;
        for (uint32_t i = 0; i < n_int; i++) fill(nd.child_base + i);
    };
    fill(0);
    // leaf slot boxes: the exact culling boxes (the binary builder rounded them outward)
    for (TriWideNode& nd : nodes)
        for (uint32_t r = 0; r < (nd.slots >> 4); r++) {
            const uint32_t s = (nd.slots & 0xfu) + r;
            const TriLeaf& L = out->leaves[nd.leaf_base + r];
            float clo[3], chi[3];
            bool finite;
            leaf_cull_box(L.mn, L.mx, clo, chi, &finite);
            for (int k = 0; k < 3; k++) {
                nd.lo[k][s] = clo[k];
                nd.hi[k][s] = chi[k];
            }
        }
    uint32_t max_depth = 0;
    for (uint32_t d : node_depth) max_depth = std::max(max_depth, d);
    out->depth = max_depth + 1;
    // refit order: nodes by depth, deepest level first
    out->level_off.assign(max_depth + 2, 0);
    for (uint32_t d : node_depth) out->level_off[max_depth - d + 1]++;
    for (size_t l = 1; l < out->level_off.size(); l++) out->level_off[l] += out->level_off[l - 1];
    std::vector<uint32_t> fillp(out->level_off.begin(), out->level_off.end() - 1);
    out->order.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) out->order[fillp[max_depth - node_depth[i]]++] = (uint32_t)i;

    // 3. compact leaves
    if (hot16)
        for (TriLeaf& L : out->leaves) wide_leaf_make_compact(hot16, n_tri, L, out->verts, out->vsrc);
}
