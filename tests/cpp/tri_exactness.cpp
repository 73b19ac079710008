// CPU check of the triangle accelerator used by rt_pathtrace_kernel: the
// kernel's BVH traversal logic (same f32 operation order, -ffp-contract=off)
// must return exactly the triangle, object and distance of the reference's
// sequential sweep (check_triangles, compute_shader.wgsl:422-517).
// The binary walk over the 16-B quantized nodes (tri_qnode.h) is checked the same way, ray
// by ray; every quantized box must contain its node's box.
// usage: tri_exactness <objects.bin> <subs.bin> <tris.bin> <rays.f32> [margin_scale]
//   -> "ok <rays> <hits> <avg_tri_tests> <avg_nodes> <nan_fallbacks>"
//      "qnodes <valid> <avg_nodes>"
//   or the first mismatch
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "rt_bvh_slab.h"
#include "sphere_bvh.h"
#include "tri_cone.h"
#include "tri_qnode.h"

static const float F32_MAX_ = 3.4028235e+38f;
struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V ld(const float* p) { return {p[0], p[1], p[2]}; }

template <typename T>
static std::vector<T> load(const char* path) {
    std::vector<T> v;
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    T x;
    while (fread(&x, sizeof(T), 1, f) == 1) v.push_back(x);
    fclose(f);
    return v;
}

static bool rib(V o, V inv, const float* mn, const float* mx) {
    float a0 = (mn[0] - o.x) * inv.x, a1 = (mx[0] - o.x) * inv.x;
    float b0 = (mn[1] - o.y) * inv.y, b1 = (mx[1] - o.y) * inv.y;
    float c0 = (mn[2] - o.z) * inv.z, c1 = (mx[2] - o.z) * inv.z;
    float n = std::fmax(std::fmax(std::fmin(a0, a1), std::fmin(b0, b1)), std::fmin(c0, c1));
    float f = std::fmin(std::fmin(std::fmax(a0, a1), std::fmax(b0, b1)), std::fmax(c0, c1));
    return n <= f && f >= 0.0f;
}

struct Res { float t; int tri; int obj; int front; };

static long g_tests = 0, g_nodes = 0, g_nan = 0;

static Res sweep(const std::vector<rt_object_info>& ob, const std::vector<rt_sub_object_info>& sb,
                 const std::vector<rt_scene_triangle>& tr, V o, V d) {
    float closest = F32_MAX_;
    Res r{F32_MAX_, -1, -1, 0};
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    for (size_t oi = 0; oi < ob.size(); oi++) {
        if (!rib(o, inv, ob[oi].min_bounds, ob[oi].max_bounds)) continue;
        for (uint32_t i = 0; i < ob[oi].sub_object_count; i++) {
            const rt_sub_object_info& s = sb[ob[oi].first_sub_object_index + i];
            if (!rib(o, inv, s.min_bounds, s.max_bounds)) continue;
            for (uint32_t j = 0; j < s.triangle_count; j++) {
                const rt_scene_triangle& t = tr[s.first_triangle_index + j];
                V cn = ld(t.calc_normal);
                float det = -dot(d, cn), inv_det = 1.0f / det;
                V ao = sub(o, ld(t.a));
                float dist = dot(ao, cn) * inv_det;
                if (dist < 0.0f || dist >= closest) continue;
                V dao = cross(ao, d);
                float v = -dot(ld(t.edge_ab), dao) * inv_det;
                if (v < 0.0f) continue;
                float u = dot(ld(t.edge_ac), dao) * inv_det;
                if (u < 0.0f) continue;
                float w = 1.0f - u - v;
                if (w < 0.0f) continue;
                closest = dist;
                r = {dist, (int)(s.first_triangle_index + j), (int)oi, det > 0.0f};
            }
        }
    }
    return r;
}

static long g_qnodes = 0;
static bool g_lazy = false;  // the kernel's kLazySub leaf: the sub-object box tested at the first candidate
static const std::vector<uint32_t>* g_q = nullptr;  // quantized records (4 words per node), or null
static TriQGrid g_grid;
// the kernel's global-memory walk (round 3): the direction-ordered layouts (order_bvh_by_octant,
// quantized with the last-leaf flag as rt_quantize_tri_nodes_kernel derives them) and distance
// pruning with the kernel's limit (pathtrace.hip tri_limit)
static const std::vector<SphereBvhNode>* g_oct = nullptr;
static const std::vector<uint32_t>* g_qoct = nullptr;
static float g_prune = 0.0f;
static long g_prune_nodes = 0, g_prune_tests = 0;
static bool g_heur_count = false;
static long g_heur_miss = 0;
static long g_exact_nodes = 0, g_exact_tests = 0;
// certified pruning (tri_cone.h): the leaf certificates, per prim (the kernel's default walk)
static const std::vector<TriLeafCert>* g_lcert = nullptr;
static long g_lcert_leaves = 0, g_lcert_skipped = 0, g_lcert_tris = 0;
static uint32_t g_subtree_max = 0;
// experiment (TRI_DEPTH_HIST): the kernel-default walk's node visits and box hits by tree depth
static std::vector<uint8_t> g_depth;
static long g_depth_visits[64] = {0};
static long g_depth_entries[64] = {0};  // the kernel-default walk's box hits by depth (subtrees entered)
// the kernel's default walk since round 5 (pathtrace.hip): the certificate test deferred to the
// leaf batch through the gap node_step records (tri_leafcert_skips_gap, RT_LEAFCERT_DEFER) and the
// leaf's triangles tested as a cooperative batch -- every candidate on its own, then the
// lexicographic minimum and a NaN flag merged by the leaf's lane (coop_leaf_batch)
static bool g_kernel_default = false;
static long g_gap_checked = 0, g_gap_skipped = 0, g_coop_leaves = 0, g_coop_nan = 0;

static Res accel(const TriangleAccel& A, const std::vector<rt_object_info>& ob, const std::vector<rt_sub_object_info>& sb,
                 const std::vector<rt_scene_triangle>& tr, V o, V d, float scale) {
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    float m = scale * (std::sqrt(dot(o, o)) + A.extent) + 1.0e-30f;
    float best = F32_MAX_;
    uint32_t best_seq = 0;
    Res r{F32_MAX_, -1, -1, 0};
    bool nan_hit = false;
    const SlabRay sr = slab_ray(o.x, o.y, o.z, inv.x, inv.y, inv.z, m);
    const std::vector<SphereBvhNode>& NS = g_oct ? *g_oct : A.nodes;
    const std::vector<uint32_t>* QS = g_oct ? g_qoct : g_q;
    uint32_t n = (uint32_t)NS.size();
    uint32_t node = 0;
    if (g_oct) {
        uint32_t ib[3];
        memcpy(ib, &inv, 12);
        node = ((ib[0] >> 31) | ((ib[1] >> 31) << 1) | ((ib[2] >> 31) << 2)) * (uint32_t)A.nodes.size();
    }
    float limit = INFINITY;
    const TriConeRay tcr = tri_cone_ray(o.x, o.y, o.z, d.x, d.y, d.z);
    const float sig = 0x1p-10f * (std::sqrt(dot(o, o)) + A.extent) * (1.0f / std::sqrt(dot(d, d)) * 1.001f);
    while (node < n) {
        SphereBvhNode nd = NS[node];
        if (g_prune != 0.0f) g_prune_nodes++;
        if (QS) {  // the kernel's quantized-node walk: the decoded box and the link word
            if (!g_lazy) g_qnodes++;
            const uint32_t* q = &(*QS)[4 * (size_t)node];
            tri_qnode_box(q, g_grid, nd.bmin, nd.bmax);
            const bool is_leaf = (q[3] & 0x80000000u) != 0u;
            nd.leaf = is_leaf ? (q[3] & 0xffffffu) : kSphereBvhInternal;
            nd.skip = is_leaf ? ((q[3] & kTriQLastLeaf) ? kTriWalkEnd : node + 1) : q[3];
        } else if (!g_lazy) {
            g_nodes++;
        }
        if (g_lcert) g_exact_nodes++;
        if (g_kernel_default && !g_depth.empty()) g_depth_visits[std::min<int>(g_depth[node], 63)]++;
        float nt, ft;  // the kernel's slab test (rt_bvh_slab.h)
        slab_hit(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2], nt, ft);
        bool hit = nt <= ft && ft >= 0.0f && nt <= limit;
        uint32_t skip = 0u;  // leaf certificate: triangles proven beyond the best hit
        if (g_lcert && g_subtree_max && hit && nd.leaf == kSphereBvhInternal && best != F32_MAX_ && nt > best) {
            // experiment (TRI_SUBTREE_MAX): an ideal certificate for small subtrees -- every leaf's
            // own certificate evaluated on this node's box entry
            uint32_t tri_count = 0;
            for (uint32_t q = node; q < nd.skip && q < n; q++)
                if (NS[q].leaf != kSphereBvhInternal) tri_count += sb[A.prims[NS[q].leaf & 0xffffffu].sub].triangle_count;
            if (tri_count <= g_subtree_max) {
                const float t1x = fminf(fmaf(nd.bmin[0], sr.ix, sr.lx), fmaf(nd.bmax[0], sr.ix, sr.hx));
                const float t1y = fminf(fmaf(nd.bmin[1], sr.iy, sr.ly), fmaf(nd.bmax[1], sr.iy, sr.hy));
                const float t1z = fminf(fmaf(nd.bmin[2], sr.iz, sr.lz), fmaf(nd.bmax[2], sr.iz, sr.hz));
                bool all = true;
                for (uint32_t q = node; q < nd.skip && q < n && all; q++)
                    if (NS[q].leaf != kSphereBvhInternal)
                        all = tri_leafcert_skips((*g_lcert)[NS[q].leaf & 0xffffffu].w, tcr, best, t1x, t1y, t1z,
                                                 fabsf(sr.ix), fabsf(sr.iy), fabsf(sr.iz)) == kLeafCertAll;
                if (all) hit = false;
            }
        }
        if (g_kernel_default && !g_depth.empty() && hit) g_depth_entries[std::min<int>(g_depth[node], 63)]++;
        if (g_lcert && hit && nd.leaf != kSphereBvhInternal && best != F32_MAX_ && nt > best) {
            const float t1x = fminf(fmaf(nd.bmin[0], sr.ix, sr.lx), fmaf(nd.bmax[0], sr.ix, sr.hx));
            const float t1y = fminf(fmaf(nd.bmin[1], sr.iy, sr.ly), fmaf(nd.bmax[1], sr.iy, sr.hy));
            const float t1z = fminf(fmaf(nd.bmin[2], sr.iz, sr.lz), fmaf(nd.bmax[2], sr.iz, sr.hz));
            if (g_kernel_default) {
                // node_step's gap (pathtrace.hip, RT_LEAFCERT_DEFER), then the leaf batch's test
                const float tbs = best * (1.0f + 0x1p-20f);
                const float gx = (t1x - tbs) * fabsf(d.x), gy = (t1y - tbs) * fabsf(d.y), gz = (t1z - tbs) * fabsf(d.z);
                const float gap = fmaxf(fmaxf(gx, gy), gz) * (1.0f - 0x1p-20f);
                skip = gap > 0.0f ? tri_leafcert_skips_gap((*g_lcert)[nd.leaf & 0xffffffu].w, tcr, best, gap) : 0u;
                g_gap_checked += gap > 0.0f;
                g_gap_skipped += skip == kLeafCertAll;
            } else {
                skip = tri_leafcert_skips((*g_lcert)[nd.leaf & 0xffffffu].w, tcr, best, t1x, t1y, t1z, fabsf(sr.ix),
                                          fabsf(sr.iy), fabsf(sr.iz));
            }
            g_lcert_leaves++;
            if (skip == kLeafCertAll) {
                hit = false;
                g_lcert_skipped++;
            }
        }
        if (hit && nd.leaf != kSphereBvhInternal) {
            const SubObjectPrim& p = A.prims[nd.leaf & 0xffffffu];
            const rt_object_info& OB = ob[p.object];
            const rt_sub_object_info& s = sb[p.sub];
            const bool lazy = g_lazy && p.range != kPrimRangeNone;
            int sub_state = lazy ? 0 : 1;
            const uint32_t first = lazy ? (p.range & ((1u << 27) - 1u)) : s.first_triangle_index;
            const uint32_t count = lazy ? (p.range >> 27) : s.triangle_count;
            if (lazy && (first != s.first_triangle_index || count != s.triangle_count)) {
                printf("PRIM RANGE mismatch\n");
                exit(1);
            }
            if (g_kernel_default && lazy && count < 8u && rib(o, inv, OB.min_bounds, OB.max_bounds)) {
                // coop_leaf_batch: every triangle tested on its own (lane j), the group's minimum of
                // (distance, sweep position) and NaN flag, then the leaf's lane merges
                g_coop_leaves++;
                float cd = INFINITY;
                uint32_t cs = 0xffffffffu;
                int cti = -1, cfront = 0;
                bool cnan = false;
                for (uint32_t j = 0; j < count; j++) {
                    g_exact_tests++;
                    const rt_scene_triangle& t = tr[std::min<uint32_t>(first + j, (uint32_t)tr.size() - 1u)];
                    V cn = ld(t.calc_normal);
                    float det = -dot(d, cn), inv_det = 1.0f / det;
                    V ao = sub(o, ld(t.a));
                    float dist = dot(ao, cn) * inv_det;
                    V dao = cross(ao, d);
                    float v = -dot(ld(t.edge_ab), dao) * inv_det;
                    float u = dot(ld(t.edge_ac), dao) * inv_det;
                    float w = 1.0f - u - v;
                    if (dist < 0.0f || v < 0.0f || u < 0.0f || w < 0.0f) continue;
                    if (dist != dist) { cnan = true; continue; }
                    const uint32_t seq = p.seq_base + j;
                    if (dist < cd || (dist == cd && seq < cs)) {
                        cd = dist;
                        cs = seq;
                        cti = (int)(first + j);
                        cfront = det > 0.0f;
                    }
                }
                const bool beats = cd < best || (cd == best && cs < best_seq);
                if ((cnan || beats) && rib(o, inv, s.min_bounds, s.max_bounds)) {
                    if (cnan) { nan_hit = true; g_coop_nan++; }
                    if (beats) {
                        best = cd;
                        best_seq = cs;
                        r = {cd, cti, (int)p.object, cfront};
                    }
                }
            } else if (rib(o, inv, OB.min_bounds, OB.max_bounds) && (lazy || rib(o, inv, s.min_bounds, s.max_bounds))) {
                for (uint32_t j = 0; j < count; j++) {
                    if ((skip >> j) & 1u) {
                        g_lcert_tris++;
                        continue;
                    }
                    if (!g_q && !g_lazy) g_tests++;
                    if (g_prune != 0.0f) g_prune_tests++;
                    if (g_lcert) g_exact_tests++;
                    uint32_t ti = first + j, seq = p.seq_base + j;
                    const rt_scene_triangle& t = tr[ti];
                    V cn = ld(t.calc_normal);
                    float det = -dot(d, cn), inv_det = 1.0f / det;
                    V ao = sub(o, ld(t.a));
                    float dist = dot(ao, cn) * inv_det;
                    bool nan_dist = dist != dist;
                    if (dist < 0.0f) continue;
                    if (!nan_dist && !(dist < best || (dist == best && seq < best_seq))) continue;
                    V dao = cross(ao, d);
                    float v = -dot(ld(t.edge_ab), dao) * inv_det;
                    if (v < 0.0f) continue;
                    float u = dot(ld(t.edge_ac), dao) * inv_det;
                    if (u < 0.0f) continue;
                    float w = 1.0f - u - v;
                    if (w < 0.0f) continue;
                    if (sub_state == 0) {
                        if (!rib(o, inv, s.min_bounds, s.max_bounds)) break;
                        sub_state = 1;
                    }
                    if (nan_dist) { nan_hit = true; continue; }
                    best = dist;
                    best_seq = seq;
                    r = {dist, (int)ti, (int)p.object, det > 0.0f};
                    if (g_prune != 0.0f) limit = best * (1.0f + g_prune) + sig;
                }
            }
        }
        node = (hit && nd.leaf == kSphereBvhInternal) ? node + 1 : nd.skip;
    }
    if (nan_hit) {
        g_nan++;
        return sweep(ob, sb, tr, o, d);
    }
    return r;
}

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    auto ob = load<rt_object_info>(argv[1]);
    auto sb = load<rt_sub_object_info>(argv[2]);
    auto tr = load<rt_scene_triangle>(argv[3]);
    auto rays = load<float>(argv[4]);
    float scale = argc > 5 ? (float)atof(argv[5]) : 1.0e-5f;
    g_heur_count = getenv("TRI_HEUR_COUNT") != nullptr;
    if (getenv("TRI_SUBTREE_MAX")) g_subtree_max = (uint32_t)atoi(getenv("TRI_SUBTREE_MAX"));
    TriangleAccel A;
    build_triangle_accel(ob.data(), (uint32_t)ob.size(), sb.data(), (uint32_t)sb.size(), &A);
    // the quantized copy, as rt_quantize_tri_nodes_kernel makes it; each box must contain its node's
    std::vector<uint32_t> qn(4 * A.nodes.size());
    g_grid = A.nodes.empty() ? TriQGrid{} : tri_qgrid(A.nodes[0]);
    if (g_grid.valid) {
        for (size_t i = 0; i < A.nodes.size(); i++) {
            tri_qnode(A.nodes[i], g_grid, &qn[4 * i]);
            float lo[3], hi[3];
            tri_qnode_box(&qn[4 * i], g_grid, lo, hi);
            for (int k = 0; k < 3; k++)
                if (!(lo[k] <= A.nodes[i].bmin[k] && hi[k] >= A.nodes[i].bmax[k])) {
                    printf("QNODE BOX node %zu axis %d: [%.9g %.9g] does not contain [%.9g %.9g]\n", i, k, lo[k], hi[k],
                           A.nodes[i].bmin[k], A.nodes[i].bmax[k]);
                    return 1;
                }
        }
    }
    // leaf certificates, per prim (rt_tri_leafcert_kernel derives them the same way)
    std::vector<TriLeafCert> lcert(A.prims.size());
    long lcert_valid = 0;
    for (size_t pi = 0; pi < A.prims.size(); pi++) {
        const rt_sub_object_info& sbi = sb[A.prims[pi].sub];
        float lo[3], hi[3];
        for (int k = 0; k < 3; k++) {
            lo[k] = fminf(sbi.min_bounds[k], sbi.max_bounds[k]);
            hi[k] = fmaxf(sbi.min_bounds[k], sbi.max_bounds[k]);
        }
        const uint32_t cnt = sbi.triangle_count <= kLeafCertSlots ? sbi.triangle_count : 0u;
        float ta[kLeafCertSlots][3], tab[kLeafCertSlots][3], tac[kLeafCertSlots][3], tcn[kLeafCertSlots][3];
        for (uint32_t j = 0; j < cnt; j++) {
            const rt_scene_triangle& t = tr[sbi.first_triangle_index + j];
            memcpy(ta[j], t.a, 12);
            memcpy(tab[j], t.edge_ab, 12);
            memcpy(tac[j], t.edge_ac, 12);
            memcpy(tcn[j], t.calc_normal, 12);
        }
        lcert[pi] = tricone::leafcert_build(cnt, ta, tab, tac, tcn, lo, hi);
        lcert_valid += lcert[pi].w[7] != kLeafCertNone;
    }
    std::vector<SphereBvhNode> oct;
    std::vector<uint32_t> qoct;
    order_bvh_by_octant(A.nodes, &oct, false, nullptr);
    if (g_grid.valid) {
        qoct.resize(4 * oct.size());
        for (size_t i = 0; i < oct.size(); i++) {
            tri_qnode(oct[i], g_grid, &qoct[4 * i]);
            if (oct[i].leaf != kSphereBvhInternal && oct[i].skip >= oct.size()) qoct[4 * i + 3] |= kTriQLastLeaf;
        }
    }
    if (getenv("TRI_DEPTH_HIST") && !oct.empty()) {
        g_depth.assign(oct.size(), 0);
        for (size_t i = 0; i < oct.size(); i++)
            if (oct[i].leaf == kSphereBvhInternal && i + 1 < oct.size()) {
                g_depth[i + 1] = g_depth[i] + 1;
                if (oct[i + 1].skip < oct.size()) g_depth[oct[i + 1].skip] = g_depth[i] + 1;
            }
    }
    long n = (long)rays.size() / 6, hits = 0;
    for (long i = 0; i < n; i++) {
        V o = ld(&rays[6 * i]), d = ld(&rays[6 * i + 3]);
        Res a = sweep(ob, sb, tr, o, d), b = accel(A, ob, sb, tr, o, d, scale);
        Res e = b;
        if (g_grid.valid) {
            g_q = &qn;
            e = accel(A, ob, sb, tr, o, d, scale);
            g_q = nullptr;
        }
        g_lazy = true;  // the mode-1 kernel's walk: quantized nodes (when valid) and lazy sub-object tests
        g_q = g_grid.valid ? &qn : nullptr;
        Res f = accel(A, ob, sb, tr, o, d, scale);
        // the default global-memory walk: octant layouts (quantized when valid), lazy sub-objects, pruning
        g_oct = oct.empty() ? nullptr : &oct;
        g_qoct = g_grid.valid ? &qoct : nullptr;
        g_prune = 1.0f / 64.0f;
        Res h = accel(A, ob, sb, tr, o, d, scale);
        if (g_heur_count) {  // TRI_HEUR_COUNT: the heuristic slack's misses are counted, not fatal
            uint32_t ta, th;
            memcpy(&ta, &a.t, 4);
            memcpy(&th, &h.t, 4);
            if (ta != th || a.tri != h.tri || a.obj != h.obj || a.front != h.front) g_heur_miss++;
            h = a;
        }
        g_prune = 0.0f;
        // the certified walk (tri_cone.h leaf certificates) over the same layouts
        g_lcert = &lcert;
        Res x = accel(A, ob, sb, tr, o, d, scale);
        // the kernel's default walk (round 5): deferred certificate test + cooperative leaf batches
        g_kernel_default = true;
        const long saved_nodes = g_exact_nodes, saved_tests = g_exact_tests;
        Res y = accel(A, ob, sb, tr, o, d, scale);
        g_exact_nodes = saved_nodes;
        g_exact_tests = saved_tests;
        g_kernel_default = false;
        g_lcert = nullptr;
        g_oct = nullptr;
        g_qoct = nullptr;
        g_q = nullptr;
        g_lazy = false;
        const Res* const walks[] = {&b, &e, &f, &h, &x, &y};
        const char* const names[] = {"binary", "qnodes", "qnodes+lazy", "octants+prune", "certified", "kernel-default"};
        for (int wi = 0; wi < 6; wi++) {
            const Res* w = walks[wi];
            uint32_t ta, tb;
            memcpy(&ta, &a.t, 4);
            memcpy(&tb, &w->t, 4);
            if (ta != tb || a.tri != w->tri || a.obj != w->obj || a.front != w->front) {
                printf("MISMATCH (%s) ray %ld o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) sweep=(%d/%d %.9g) accel=(%d/%d %.9g)\n",
                       names[wi], i, o.x, o.y, o.z, d.x, d.y, d.z, a.obj, a.tri, a.t, w->obj, w->tri, w->t);
                return 1;
            }
        }
        hits += a.tri >= 0;
    }
    printf("ok %ld %ld %.2f %.2f %ld\n", n, hits, (double)g_tests / n, (double)g_nodes / n, g_nan);
    printf("qnodes %d %.2f\n", g_grid.valid ? 1 : 0, (double)g_qnodes / n);
    printf("prune %.2f %.2f\n", (double)g_prune_nodes / n, (double)g_prune_tests / n);
    printf("certified %.2f %.2f %.2f %.2f %.2f %ld %zu\n", (double)g_exact_nodes / n, (double)g_exact_tests / n,
           (double)g_lcert_leaves / n, (double)g_lcert_skipped / n, (double)g_lcert_tris / n, lcert_valid,
           lcert.size());
    printf("heuristic_misses %ld\n", g_heur_miss);
    printf("kernel_default %ld %ld %ld %ld\n", g_gap_checked, g_gap_skipped, g_coop_leaves, g_coop_nan);
    if (!g_depth.empty()) {  // depth, visits per ray at that depth, nodes of one layout at that depth
        std::vector<long> per(64, 0);
        for (size_t i = 0; i < A.nodes.size(); i++) per[std::min<int>(g_depth[i], 63)]++;
        for (int k = 0; k < 64; k++)
            if (per[k] || g_depth_visits[k])
                printf("depth %d %.3f %.3f %ld\n", k, (double)g_depth_visits[k] / n, (double)g_depth_entries[k] / n, per[k]);
    }
    return 0;
}
