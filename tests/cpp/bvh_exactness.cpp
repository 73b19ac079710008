// CPU check of the sphere-BVH culling used by rt_pathtrace_kernel: for many
// rays, the kernel's traversal logic (restated here in the same f32 operation
// order, compiled with -ffp-contract=off) must return exactly the sphere and
// t of the reference's brute-force scan (compute_shader.wgsl:355-404).
// usage: bvh_exactness <n_rays> <seed>   -> prints "ok <rays> <hits> <avg_tests>" or the first mismatch
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rt_bvh_slab.h"
#include "sphere_bvh.h"

static const float F32_MAX_ = 3.4028235e+38f;
struct V { float x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static float fmin_nn(float a, float b) { return std::fmin(a, b); }
static float fmax_nn(float a, float b) { return std::fmax(a, b); }

struct Res { float t; int idx; };

static Res brute(const std::vector<rt_scene_sphere>& s, V o, V d) {
    float closest = F32_MAX_;
    int ci = -1;
    float a = dot(d, d);
    for (size_t i = 0; i < s.size(); i++) {
        V oc = sub(o, V{s[i].position[0], s[i].position[1], s[i].position[2]});
        float b = 2.0f * dot(d, oc);
        float c = dot(oc, oc) - s[i].radius * s[i].radius;
        float disc = b * b - 4.0f * a * c;
        if (disc < 0.0f) continue;
        float t = (-b - std::sqrt(disc)) / (2.0f * a);
        if (t > 0.0f && t < closest) { closest = t; ci = (int)i; }
    }
    return {closest, ci};
}

static long g_tests = 0;
static long g_disc_pos = 0, g_accept = 0;
static long g_nodes = 0;

static void cand(const SphereSlots& sl, uint32_t slot, V o, V d, float four_a, float two_a, float& bt, uint32_t& bo, bool& found) {
    const float* q = &sl.slot_sph[4 * slot];
    V oc = sub(o, V{q[0], q[1], q[2]});
    float b = 2.0f * dot(d, oc);
    float c = dot(oc, oc) - q[3];
    float disc = b * b - four_a * c;
    g_tests++;
    if (disc >= 0.0f) {
        g_disc_pos++;
        float t = (-b - std::sqrt(disc)) / two_a;
        uint32_t orig = sl.slot_orig[slot];
        if (t > 0.0f && (t < bt || (t == bt && orig < bo))) { bt = t; bo = orig; found = true; g_accept++; }
    }
}

// Experiment (ORDERED=1): ordered stack traversal, both child boxes tested at
// each internal node, nearer first. g_nodes counts box tests.
static Res ordered_like(const SphereSlots& sl, V o, V d) {
    float bt = F32_MAX_;
    uint32_t bo = 0;
    bool found = false;
    float a = dot(d, d), four_a = 4.0f * a, two_a = 2.0f * a;
    for (uint32_t i = 0; i < sl.n_always; i++) cand(sl, i, o, d, four_a, two_a, bt, bo, found);
    if (sl.nodes.empty()) return {bt, found ? (int)bo : -1};
    float lateral, slack;
    sphere_cull_bounds(std::sqrt(dot(o, o)), sl.extent, sl.r_min, sl.r_max, 1.0f / std::sqrt(a), lateral, slack);
    V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const SlabRay sr = slab_ray(o.x, o.y, o.z, inv.x, inv.y, inv.z, lateral);
    auto box = [&](uint32_t n, float& nt) {
        g_nodes++;
        const SphereBvhNode& nd = sl.nodes[n];
        float near_t, far_t;
        slab_hit(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2], near_t, far_t);
        nt = near_t;
        return near_t <= far_t && far_t >= -slack && near_t <= bt * 1.00001f + slack;
    };
    uint32_t stack[64]; float st[64]; int sp = 0;
    float nt0;
    if (!box(0, nt0)) return {bt, found ? (int)bo : -1};
    stack[sp] = 0; st[sp++] = nt0;
    while (sp) {
        --sp;
        uint32_t n = stack[sp];
        if (st[sp] > bt * 1.00001f + slack) continue;
        for (;;) {
            const SphereBvhNode& nd = sl.nodes[n];
            if (nd.leaf != kSphereBvhInternal) {
                uint32_t first = nd.leaf & 0xffffffu, cnt = nd.leaf >> 24;
                for (uint32_t k = 0; k < cnt; k++) cand(sl, first + k, o, d, four_a, two_a, bt, bo, found);
                break;
            }
            uint32_t l = n + 1, r = sl.nodes[n + 1].skip;
            float tl, tr;
            bool hl = box(l, tl), hr = box(r, tr);
            if (hl && hr) {
                if (tr < tl) { std::swap(l, r); std::swap(tl, tr); }
                stack[sp] = r; st[sp++] = tr; n = l;
            } else if (hl) n = l; else if (hr) n = r; else break;
        }
    }
    return {bt, found ? (int)bo : -1};
}

// The kernel walks the direction-ordered layouts (order_bvh_by_octant) unless
// SINGLE_LAYOUT is set: g_oct holds them for the scene under test.
static std::vector<SphereBvhNode> g_oct;
static bool g_oct_ordered = false;  // g_oct stores (near, far) corners per octant (box-ordered layouts)
static long g_slab_diff = 0;        // slab_hit_ordered != slab_hit on the same inputs (must stay 0)

static Res kernel_like(const SphereSlots& sl, V o, V d) {
    float bt = F32_MAX_;
    uint32_t bo = 0;
    bool found = false;
    float a = dot(d, d), four_a = 4.0f * a, two_a = 2.0f * a;
    for (uint32_t i = 0; i < sl.n_always; i++) cand(sl, i, o, d, four_a, two_a, bt, bo, found);
    const uint32_t n = (uint32_t)sl.nodes.size();
    if (n) {
        // the kernel's culling bounds (rt_bvh_slab.h); LAT_SCALE / SLACK_SCALE
        // shrink them to show the check is not vacuous
        float lateral, slack;
        sphere_cull_bounds(std::sqrt(dot(o, o)), sl.extent, sl.r_min, sl.r_max, 1.0f / std::sqrt(a), lateral, slack);
        if (getenv("LAT_SCALE")) lateral *= (float)atof(getenv("LAT_SCALE"));
        if (getenv("SLACK_SCALE")) slack *= (float)atof(getenv("SLACK_SCALE"));
        V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        if (getenv("INV_ULP")) {
            // sphere-only kernels take 1/d from v_rcp_f32 (<= 1 ulp): each component
            // one ulp up or down, chosen per ray and axis
            static uint32_t h = 0x9e3779b9u;
            auto nudge = [&](float v) {
                h = h * 747796405u + 2891336453u;
                return std::isfinite(v) ? std::nextafter(v, (h >> 31) ? INFINITY : -INFINITY) : v;
            };
            inv = {nudge(inv.x), nudge(inv.y), nudge(inv.z)};
        }
        SlabRay sr = slab_ray(o.x, o.y, o.z, inv.x, inv.y, inv.z, lateral);  // the kernel's slab test
        const bool oct = !getenv("SINGLE_LAYOUT");
        if (oct && g_oct.size() != 8 * (size_t)n) {
            // the sphere-only kernels' layouts: boxes as (near, far) corners when exact
            g_oct_ordered = !getenv("UNORDERED_BOXES") && box_layout_orderable(sl.nodes);
            order_bvh_by_octant(sl.nodes, &g_oct, g_oct_ordered);
        }
        if (oct && g_oct_ordered) slab_pair_by_octant(sr);
        const SphereBvhNode* nodes = oct ? g_oct.data() : sl.nodes.data();
        const uint32_t total = oct ? 8 * n : n;
        uint32_t node = oct ? n * ((std::signbit(inv.x) ? 1u : 0u) | (std::signbit(inv.y) ? 2u : 0u) |
                                   (std::signbit(inv.z) ? 4u : 0u))
                            : 0u;
        while (node < total) {
            g_nodes++;
            const SphereBvhNode& nd = nodes[node];
            float near_t, far_t;
            slab_hit(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2], near_t, far_t);
            if (oct && g_oct_ordered) {  // what the sphere-only kernels compute: must be the same values
                float n2, f2;
                slab_hit_ordered(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2], n2, f2);
                if (!(n2 == near_t || (n2 != n2 && near_t != near_t)) || !(f2 == far_t || (f2 != f2 && far_t != far_t)))
                    g_slab_diff++;
                near_t = n2;
                far_t = f2;
            }
            bool hit = near_t <= far_t && far_t >= -slack && near_t <= bt * 1.00001f + slack;
            if (hit && nd.leaf != kSphereBvhInternal) {
                uint32_t first = nd.leaf & 0xffffffu, cnt = nd.leaf >> 24;
                for (uint32_t k = 0; k < cnt; k++) cand(sl, first + k, o, d, four_a, two_a, bt, bo, found);
            }
            node = (hit && nd.leaf == kSphereBvhInternal) ? node + 1 : nd.skip;
        }
    }
    return {bt, found ? (int)bo : -1};
}

static int replay(const char* rays_path, const char* sph_path) {
    FILE* f = fopen(sph_path, "rb");
    std::vector<rt_scene_sphere> s;
    rt_scene_sphere sp;
    while (fread(&sp, sizeof(sp), 1, f) == 1) s.push_back(sp);
    fclose(f);
    SphereSlots sl;
    build_sphere_slots(s.data(), (uint32_t)s.size(), true, &sl);
    f = fopen(rays_path, "rb");
    float q[6];
    long n = 0, bad = 0;
    g_tests = 0;
    std::vector<uint32_t> visits;  // node visits per ray (distribution)
    while (fread(q, sizeof(q), 1, f) == 1) {
        V o{q[0], q[1], q[2]}, d{q[3], q[4], q[5]};
        const long before = g_nodes;
        Res a = brute(s, o, d), b = getenv("ORDERED") ? ordered_like(sl, o, d) : kernel_like(sl, o, d);
        visits.push_back((uint32_t)(g_nodes - before));
        uint32_t ta, tb;
        memcpy(&ta, &a.t, 4);
        memcpy(&tb, &b.t, 4);
        bad += (a.idx != b.idx || ta != tb);
        n++;
    }
    fclose(f);
    printf("replay rays %ld mismatches %ld spheres %zu always %u nodes %zu | per ray: node visits %.2f sphere tests %.2f"
           " disc>=0 %.2f accepted %.2f\n",
           n, bad, s.size(), sl.n_always, sl.nodes.size(), (double)g_nodes / n, (double)g_tests / n,
           (double)g_disc_pos / n, (double)g_accept / n);
    if (!visits.empty()) {
        std::sort(visits.begin(), visits.end());
        auto pct = [&](double q) { return visits[(size_t)(q * (visits.size() - 1))]; };
        printf("node visits per ray: p10 %u p50 %u p90 %u p99 %u max %u\n", pct(0.1), pct(0.5), pct(0.9), pct(0.99),
               visits.back());
    }
    if (g_slab_diff) printf("slab_hit_ordered differs from slab_hit on %ld box tests\n", g_slab_diff);
    return (bad || g_slab_diff) ? 1 : 0;
}

// Adversarial sets for the derived bound (rt_bvh_slab.h): BVH spheres with
// radii log-uniform over 1e-3..1e3 (centres 1e3..2e3 from the origin, so every sphere is in the
// BVH), and rays tangent to a random sphere in exact arithmetic -- the reference's discriminant
// within a few ulp of 0 -- from origins 1..1e6 radii away along the tangent, nudged across the
// tangent by a few ulp; plus rays aimed at the centre from far away, and directions scaled to
// |d| from 1e-12 (below the bound's admitted range: no culling) to 1e6.
static int adversarial(long n_rays, unsigned seed) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<rt_scene_sphere> s;
    for (int i = 0; i < 600; i++) {
        double th = U(rng) * 6.283185307179586, ph = std::acos(2.0 * U(rng) - 1.0), R = 1000.0 + 1000.0 * U(rng);
        rt_scene_sphere sp{};
        sp.position[0] = (float)(R * std::sin(ph) * std::cos(th));
        sp.position[1] = (float)(R * std::cos(ph));
        sp.position[2] = (float)(R * std::sin(ph) * std::sin(th));
        sp.radius = (float)std::pow(10.0, -3.0 + 6.0 * U(rng));
        sp.material_index = (uint32_t)i;
        s.push_back(sp);
    }
    SphereSlots sl;
    build_sphere_slots(s.data(), (uint32_t)s.size(), true, &sl);
    if (sl.nodes.empty() || sl.n_always != 0) { printf("adversarial scene not fully in the BVH\n"); return 2; }
    long hits = 0, near_zero = 0;
    for (long r = 0; r < n_rays; r++) {
        const rt_scene_sphere& sp = s[rng() % s.size()];
        const double C[3] = {sp.position[0], sp.position[1], sp.position[2]}, rad = sp.radius;
        double n[3] = {U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5};
        double ln = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        for (double& v : n) v /= ln;
        double t[3] = {U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5};  // a tangent direction: t - (t.n) n
        const double tn = t[0] * n[0] + t[1] * n[1] + t[2] * n[2];
        for (int k = 0; k < 3; k++) t[k] -= tn * n[k];
        const double lt = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        for (double& v : t) v /= lt;
        const double L = rad * std::pow(10.0, 6.0 * U(rng));  // |o - tangent point| / r in 1..1e6
        V o, d;
        const int kind = (int)(r % 4);
        if (kind <= 2) {  // tangent in exact arithmetic, nudged by a few ulp across it
            const double nudge = (double)((int)(rng() % 9) - 4) * std::ldexp(1.0, std::ilogb((float)rad) - 23);
            o = {(float)(C[0] + (rad + nudge) * n[0] - L * t[0]), (float)(C[1] + (rad + nudge) * n[1] - L * t[1]),
                 (float)(C[2] + (rad + nudge) * n[2] - L * t[2])};
            d = {(float)t[0], (float)t[1], (float)t[2]};
            if (kind == 2) d = {(float)(t[0] + 1e-7 * n[0]), (float)(t[1] + 1e-7 * n[1]), (float)(t[2] + 1e-7 * n[2])};
        } else {  // aimed at the centre from 1..1e6 radii away (the near root far from the origin)
            o = {(float)(C[0] + L * n[0]), (float)(C[1] + L * n[1]), (float)(C[2] + L * n[2])};
            d = {(float)-n[0], (float)-n[1], (float)-n[2]};
        }
        const float scale = (float)std::pow(10.0, -12.0 + 18.0 * U(rng) * U(rng) + (r % 16 == 0 ? 0.0 : 11.0));
        d = {d.x * scale, d.y * scale, d.z * scale};
        {
            // how often the reference's discriminant sits near 0 for the chosen sphere (within 2^-16 of b^2)
            V oc = sub(o, V{sp.position[0], sp.position[1], sp.position[2]});
            float b = 2.0f * dot(d, oc), c = dot(oc, oc) - sp.radius * sp.radius;
            float disc = b * b - 4.0f * dot(d, d) * c;
            near_zero += std::fabs(disc) <= std::ldexp(std::fabs(b * b), -16);
        }
        Res a = brute(s, o, d), b = kernel_like(sl, o, d);
        uint32_t ta, tb;
        memcpy(&ta, &a.t, 4);
        memcpy(&tb, &b.t, 4);
        if (a.idx != b.idx || ta != tb) {
            printf("MISMATCH adversarial ray %ld kind %d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) brute=(%d %.9g) bvh=(%d %.9g)\n",
                   r, kind, o.x, o.y, o.z, d.x, d.y, d.z, a.idx, a.t, b.idx, b.t);
            return 1;
        }
        hits += a.idx >= 0;
    }
    printf("ok adversarial %ld %ld %.1f near_zero_disc %ld\n", n_rays, hits, (double)g_tests / n_rays, near_zero);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 3 && strcmp(argv[1], "--replay") == 0) return replay(argv[2], argv[3]);
    long n_rays = argc > 1 ? atol(argv[1]) : 200000;
    unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1;
    if (argc > 3 && strcmp(argv[3], "adv") == 0) return adversarial(n_rays, seed);
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    // RTIOW-like field + ground + a few big spheres + duplicates (ties) + touching spheres
    std::vector<rt_scene_sphere> s;
    auto add = [&](float x, float y, float z, float r) {
        rt_scene_sphere sp{}; sp.position[0] = x; sp.position[1] = y; sp.position[2] = z; sp.radius = r;
        sp.material_index = (uint32_t)s.size(); s.push_back(sp);
    };
    add(0, 1000, 0, 1000);
    for (int a = -11; a < 11; a++)
        for (int b = -11; b < 11; b++) add(a + 0.9f * U(rng), -0.2f, b + 0.9f * U(rng), 0.2f);
    add(0, -1, 0, 1); add(-4, -1, 0, 1); add(4, -1, 0, 1);
    add(4, -1, 0, 1);           // exact duplicate: tie must go to the lower index
    add(4.5f, -1.2f, 0.3f, 0.7f);  // overlapping
    add(0.0f, -3.0f, 0.0f, 0.001f); // tiny
    SphereSlots sl;
    build_sphere_slots(s.data(), (uint32_t)s.size(), true, &sl);
    if (sl.nodes.empty()) { printf("no bvh built\n"); return 2; }
    // structural checks
    std::vector<int> seen(s.size(), 0);
    for (uint32_t i = 0; i < sl.slot_orig.size(); i++) {
        if (sl.slot_orig[i] == kSphereDummyOrig) {  // padding: a NaN sphere no ray can hit
            if (!std::isnan(sl.slot_sph[4 * i])) { printf("padding slot %u is not NaN\n", i); return 1; }
            continue;
        }
        seen[sl.slot_orig[i]]++;
    }
    for (size_t i = 0; i < s.size(); i++) if (seen[i] != 1) { printf("slot coverage broken at %zu\n", i); return 1; }
    // the kernel reads aligned groups of kSphereGroup slots: brute-force prefix and every leaf
    if (sl.slot_orig.size() % kSphereGroup) { printf("slot groups unaligned\n"); return 1; }
    for (const SphereBvhNode& nd : sl.nodes)
        if (nd.leaf != kSphereBvhInternal && ((nd.leaf & 0xffffffu) % kSphereGroup || (nd.leaf >> 24) != kSphereGroup)) {
            printf("leaf group unaligned\n");
            return 1;
        }
    long hits = 0;
    for (long r = 0; r < n_rays; r++) {
        V o, d;
        int kind = r % 5;
        if (kind == 0) {  // camera-like
            o = {13.0f + U(rng), -2.0f - U(rng), 3.0f + U(rng)};
            d = {-13.0f + 6 * (U(rng) - 0.5f), 2.0f + 2 * (U(rng) - 0.5f), -3.0f + 6 * (U(rng) - 0.5f)};
        } else if (kind <= 2) {  // secondary from a sphere surface, offset like the shader (+-n*1e-4)
            const rt_scene_sphere& sp = s[1 + (rng() % (s.size() - 1))];
            V n{U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f};
            float inv = 1.0f / std::sqrt(dot(n, n));
            n = {n.x * inv, n.y * inv, n.z * inv};
            float off = (kind == 1 ? 1.0f : -1.0f) * 0.0001f;
            o = {sp.position[0] + n.x * sp.radius + n.x * off, sp.position[1] + n.y * sp.radius + n.y * off,
                 sp.position[2] + n.z * sp.radius + n.z * off};
            d = {U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f};
            if (r % 7 == 0) d = {n.z, 0.0f, -n.x};  // tangent
        } else if (kind == 3) {  // from the ground, far out
            o = {200 * (U(rng) - 0.5f), -0.0001f, 200 * (U(rng) - 0.5f)};
            d = {U(rng) - 0.5f, -U(rng), U(rng) - 0.5f};
        } else {  // axis-parallel and tiny components, aimed at sphere centres
            const rt_scene_sphere& sp = s[rng() % s.size()];
            o = {sp.position[0] + 5 * (U(rng) - 0.5f), sp.position[1] - 3, sp.position[2]};
            d = {0.0f, 1.0f, (r % 3 == 0) ? 1e-30f : 0.0f};
            if (r % 2) d = {sp.position[0] - o.x, sp.position[1] - o.y + sp.radius * (U(rng) - 0.5f) * 2, sp.position[2] - o.z};
        }
        float scale = 0.5f + 2.0f * U(rng);  // non-unit directions (jitter breaks unit length, :219)
        d = {d.x * scale, d.y * scale, d.z * scale};
        Res a = brute(s, o, d), b = getenv("ORDERED") ? ordered_like(sl, o, d) : kernel_like(sl, o, d);
        uint32_t ta, tb;
        memcpy(&ta, &a.t, 4);
        memcpy(&tb, &b.t, 4);
        if (a.idx != b.idx || ta != tb) {
            printf("MISMATCH ray %ld kind %d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) brute=(%d %.9g) bvh=(%d %.9g)\n", r,
                   kind, o.x, o.y, o.z, d.x, d.y, d.z, a.idx, a.t, b.idx, b.t);
            return 1;
        }
        hits += a.idx >= 0;
    }
    if (g_slab_diff) { printf("slab_hit_ordered differs from slab_hit on %ld box tests\n", g_slab_diff); return 1; }
    printf("ok %ld %ld %.1f %zu ordered_boxes %d\n", n_rays, hits, (double)g_tests / n_rays, s.size(), (int)g_oct_ordered);
    return 0;
}
