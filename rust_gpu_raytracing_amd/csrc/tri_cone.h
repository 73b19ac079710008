// tri_cone.h -- certified distance pruning of the triangle walk.
//
// Once a walk holds a triangle hit at distance tb, a triangle may be skipped only if the
// reference's f32 test (compute_shader.wgsl:449-481) cannot accept it with a distance <= tb.
//
// The bound (derived in DESIGN.md §5.3c). If the f32 test accepts triangle T with
// distance t, the point o + t d lies within
//     delta_T = (b_T (t |d| + |o|) + k_T) / c_T,     c_T = |d . N| / (|d| |N|),
// of T, where b_T and k_T depend only on T's stored record (its f32 calc_normal n may
// differ from the exact N = ab x ac: |N - n| enters both), the triangle's corners may lie
// outside its sub-object box by at most what k_T adds, and u = 2^-24:
//     b_T = (|N - n| + 8u |n| + 32u |ab| |ac|) / |N|
//     k_T = b_T |a| + (|ab| + |ac|) (|N - n| + 8u |n|) / |N| + excess_T + 2u (|ab| + |ac|)
// So the ray, which holds that point at parameter t <= tb, enters T's leaf box inflated by
// delta_T no later than t. Conversely, when the inflated box's entry (a certified lower
// bound) lies beyond tb, the reference cannot accept T at a distance <= tb: T cannot change
// the walk's lexicographic (distance, sweep position) minimum, ties included (strict).
//
// What carries c_T: a leaf's certificate (TriLeafCert) holds each of its triangles' own
// normal, so c_T is bounded per triangle. Round 4 first bounded c_T per BVH node with a
// normal cone over every triangle below; on the BASELINE scenes no cone above the leaves
// is narrow enough (C3 closed meshes and C5's spiky heightfield face every direction) and
// the cones pruned 0.00 (C3) / 3.7 (C5) of ~7 / ~225 node visits per ray, so the walks use
// the leaf certificates alone.
//
// Shared by the device builder (rt_tri_leafcert_kernel, scene_edit.hip), the walks
// (pathtrace.hip) and the CPU exactness harness (tests/cpp/tri_exactness.cpp).
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define RT_TC_FN __host__ __device__ inline
#else
#define RT_TC_FN inline
#endif

// Smallest lower bound of c_T the walk accepts (below it delta is too large to prune anyway).
constexpr float kTriConeCMin = 1.0e-4f;

namespace tricone {

constexpr double kU = 5.9604644775390625e-8;  // 2^-24
// Magnitudes under which no step of the reference's test overflows or leaves the normal f32
// range (the walk checks 1e-5 <= |d| <= 1e5 and |o| <= 1e15 per ray):
constexpr double kMaxCoord = 1.0e15;   // |a|
constexpr double kMaxEdge = 1.0e9;     // |ab|, |ac|
constexpr double kMaxNormal = 1.0e18;  // |calc_normal|
constexpr double kMinNormal = 1.0e-15; // |N| = |ab x ac| below this: degenerate, not prunable

RT_TC_FN double dd(float v) { return (double)v; }
RT_TC_FN float f_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = nextafterf(f, -INFINITY);
    return f;
}
RT_TC_FN float f_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = nextafterf(f, INFINITY);
    return f;
}
RT_TC_FN double len3(double x, double y, double z) { return sqrt(x * x + y * y + z * z); }

// One triangle's certificate terms (double): its unit normal and error coefficients b, k.
struct Acc {
    double ax, ay, az;  // the unit normal N / |N|, valid when n > 0
    double b, k;
    uint32_t n;         // 1 once a triangle was added
    bool valid;
};

RT_TC_FN Acc acc_empty() { return Acc{0.0, 0.0, 0.0, 0.0, 0.0, 0u, true}; }

// One triangle record (the f32 values the kernel reads: a, edge_ab, edge_ac,
// calc_normal) of a leaf whose sub-object box is [lo, hi].
RT_TC_FN void acc_add_triangle(Acc& acc, const float a[3], const float ab[3], const float ac[3], const float cn[3],
                               const float lo[3], const float hi[3]) {
    const double Nx = dd(ab[1]) * dd(ac[2]) - dd(ab[2]) * dd(ac[1]);
    const double Ny = dd(ab[2]) * dd(ac[0]) - dd(ab[0]) * dd(ac[2]);
    const double Nz = dd(ab[0]) * dd(ac[1]) - dd(ab[1]) * dd(ac[0]);
    const double NN = len3(Nx, Ny, Nz);
    const double nn = len3(dd(cn[0]), dd(cn[1]), dd(cn[2]));
    const double e = len3(Nx - dd(cn[0]), Ny - dd(cn[1]), Nz - dd(cn[2])) * (1.0 + 1e-5) + 1e-300;
    const double pa = len3(dd(a[0]), dd(a[1]), dd(a[2]));
    const double pab = len3(dd(ab[0]), dd(ab[1]), dd(ab[2]));
    const double pac = len3(dd(ac[0]), dd(ac[1]), dd(ac[2]));
    bool ok = NN >= kMinNormal && NN <= kMaxNormal && nn <= kMaxNormal && pa <= kMaxCoord && pab <= kMaxEdge &&
              pac <= kMaxEdge && e < 1e300;
    for (int i = 0; i < 3; i++) ok = ok && isfinite(lo[i]) && isfinite(hi[i]) && lo[i] <= hi[i];
    if (!ok) {
        acc.valid = false;
        return;
    }
    // the triangle's corners a, a + ab, a + ac (exact in double up to 2^-53 relative)
    // beyond the sub-object box
    double ex2 = 0.0;
    for (int c = 0; c < 3; c++) {
        double q2 = 0.0;
        for (int i = 0; i < 3; i++) {
            const double p = dd(a[i]) + (c == 1 ? dd(ab[i]) : c == 2 ? dd(ac[i]) : 0.0);
            const double over = fmax(0.0, fmax(dd(lo[i]) - p, p - dd(hi[i])));
            q2 += over * over;
        }
        ex2 = fmax(ex2, q2);
    }
    const double excess = sqrt(ex2) * (1.0 + 1e-12) + 1e-15 * (pa + pab + pac);
    const double b = (e + 8.0 * kU * nn + 32.0 * kU * pab * pac) / NN;
    // + 1e-15: absolute rounding of products that underflow (each <= 2^-150) over |det| >= 5e-25
    const double k = b * pa + (pab + pac) * (e + 8.0 * kU * nn) / NN + excess + 2.0 * kU * (pab + pac) + 1e-15;
    acc.b = fmax(acc.b, b);
    acc.k = fmax(acc.k, k);
    acc.ax = Nx / NN;
    acc.ay = Ny / NN;
    acc.az = Nz / NN;
    acc.n = 1u;
}

}  // namespace tricone

// ---- Per-triangle certificates of a leaf ("leaf certificates") ----
//
// A node's cone must hold every normal below it, and on meshes whose facets face every
// direction (C5's spiky heightfield: 64% of the nodes a ray enters beyond its hit carry no
// cone at all) it proves nothing. A leaf holds at most a few triangles, so its record keeps
// each triangle's own normal instead: 7 octahedral-encoded unit normals (16 + 16 bits,
// checked at build time to lie within kLeafCertNormalErr of +-N/|N|) and the leaf's error
// coefficients b, k (bf16, rounded up). The walk bounds c_T from below per triangle and
// skips every triangle whose own delta_T keeps it beyond tb -- without loading it -- and the
// whole leaf when all are skipped. Leaves with more than 7 triangles, or an invalid
// triangle (tri_cone.h's admitted magnitudes), carry no certificate (w[7] = kLeafCertNone).
// Slots past the leaf's count repeat triangle 0's normal, so they are skipped exactly when
// triangle 0 is, and "all 7 bits" means "every triangle of the leaf".
struct TriLeafCert {
    uint32_t w[8];  // w[j], j < 7: octahedral normal of the leaf's triangle j; w[7]: bf16 b | bf16 k << 16
};
static_assert(sizeof(TriLeafCert) == 32, "leaf certificate layout");

constexpr uint32_t kLeafCertNone = 0xffffffffu;
constexpr uint32_t kLeafCertSlots = 7u;
constexpr uint32_t kLeafCertAll = (1u << kLeafCertSlots) - 1u;
// Largest |n_T - (+-v)| allowed between the unit normal and the decoded (unit-scaled) direction;
// 16-bit octahedral quantization stays under ~1e-4, the builder refuses a record above this.
constexpr float kLeafCertNormalErr = 0x1p-12f;

// Octahedral decode, exact in f32: every value is a multiple of 2^-15 in [-1, 1]. |v| lies in
// [1/sqrt(3), 1]; v is not normalised (|d.v| / |d| <= |d.v| / (|d| |v|) is the bound used).
RT_TC_FN void leafcert_decode(uint32_t q, float& x, float& y, float& z) {
    const float px = (float)((int)(q & 0xffffu) - 32768) * 0x1p-15f;
    const float py = (float)((int)(q >> 16) - 32768) * 0x1p-15f;
    const float pz = (1.0f - fabsf(px)) - fabsf(py);
    if (pz < 0.0f) {
        x = copysignf(1.0f - fabsf(py), px);
        y = copysignf(1.0f - fabsf(px), py);
    } else {
        x = px;
        y = py;
    }
    z = pz;
}

// bf16 of a non-negative value, rounded up (0xffff: not representable / invalid).
RT_TC_FN uint32_t leafcert_bf16_up(double v) {
    if (!(v >= 0.0) || !(v < 1.0e30)) return 0xffffu;
    uint32_t bits;
    const float f = tricone::f_up(v);
    __builtin_memcpy(&bits, &f, 4);
    if (bits & 0xffffu) bits += 0x10000u;  // positive finite: a larger magnitude
    return bits >> 16;
}
RT_TC_FN float leafcert_bf16(uint32_t h) {
    const uint32_t bits = h << 16;
    float f;
    __builtin_memcpy(&f, &bits, 4);
    return f;
}

namespace tricone {

// Encodes the unit direction (x, y, z) (double); returns false when the decoded direction
// is not within kLeafCertNormalErr (minus a margin for the double evaluation) of it.
RT_TC_FN bool leafcert_encode(double x, double y, double z, uint32_t& q) {
    const double s = fabs(x) + fabs(y) + fabs(z);
    if (!(s > 0.0)) return false;
    double px = x / s, py = y / s;
    if (z < 0.0) {
        const double tx = (1.0 - fabs(py)) * (px >= 0.0 ? 1.0 : -1.0);
        const double ty = (1.0 - fabs(px)) * (py >= 0.0 ? 1.0 : -1.0);
        px = tx;
        py = ty;
    }
    long qx = lround(px * 32768.0) + 32768, qy = lround(py * 32768.0) + 32768;
    qx = qx < 0 ? 0 : qx > 65535 ? 65535 : qx;
    qy = qy < 0 ? 0 : qy > 65535 ? 65535 : qy;
    q = (uint32_t)qx | ((uint32_t)qy << 16);
    float fx, fy, fz;
    leafcert_decode(q, fx, fy, fz);
    const double l = len3(fx, fy, fz);
    if (!(l > 0.5)) return false;
    const double ex = fx / l - x, ey = fy / l - y, ez = fz / l - z;
    const double fxn = fx / l + x, fyn = fy / l + y, fzn = fz / l + z;
    const double e = fmin(len3(ex, ey, ez), len3(fxn, fyn, fzn));
    return e <= (double)kLeafCertNormalErr * 0.99;
}

// The certificate of one leaf: its sub-object box [lo, hi] and its n triangles' records.
RT_TC_FN TriLeafCert leafcert_build(uint32_t n, const float (*a)[3], const float (*ab)[3], const float (*ac)[3],
                                    const float (*cn)[3], const float lo[3], const float hi[3]) {
    TriLeafCert c;
    for (uint32_t j = 0; j < 8u; j++) c.w[j] = 0u;
    c.w[7] = kLeafCertNone;
    if (n == 0u || n > kLeafCertSlots) return c;
    double b = 0.0, k = 0.0;
    for (uint32_t j = 0; j < n; j++) {
        Acc acc = acc_empty();
        acc_add_triangle(acc, a[j], ab[j], ac[j], cn[j], lo, hi);
        if (!acc.valid) return c;
        b = fmax(b, acc.b);
        k = fmax(k, acc.k);
        if (!leafcert_encode(acc.ax, acc.ay, acc.az, c.w[j])) {
            c.w[7] = kLeafCertNone;
            return c;
        }
    }
    for (uint32_t j = n; j < kLeafCertSlots; j++) c.w[j] = c.w[0];
    const uint32_t hb = leafcert_bf16_up(b * (1.0 + 1e-6)), hk = leafcert_bf16_up(k * (1.0 + 1e-6) + 1e-30);
    if (hb == 0xffffu || hk == 0xffffu) return c;
    c.w[7] = hb | (hk << 16);
    return c;
}

}  // namespace tricone

// Per-ray constants of the certified test: d, an upper bound of |d| and of |o|, and
// the reciprocal lower bound 1/|d| (all from the kernel's f32 values, rounded the safe way).
struct TriConeRay {
    float dx, dy, dz;
    float dlen_hi, inv_dlen_lo, olen_hi;
};

RT_TC_FN TriConeRay tri_cone_ray(float ox, float oy, float oz, float dx, float dy, float dz) {
    const float dd2 = (dx * dx + dy * dy) + dz * dz;
    const float oo2 = (ox * ox + oy * oy) + oz * oz;
    TriConeRay r;
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
    r.dlen_hi = sqrtf(dd2) * 1.000001f;
    r.inv_dlen_lo = (1.0f / sqrtf(dd2)) * 0.999999f;
    r.olen_hi = sqrtf(oo2) * 1.000001f;
    return r;
}

// The triangles of a leaf (certificate w, as stored) that cannot pass the reference's test
// at a distance <= tb, as a mask over the 7 slots (kLeafCertAll: the whole leaf). t1x..z: the
// culling slab test's per-axis entry parameters of the leaf box (inflated by the culling
// margin; rt_bvh_slab.h), aix..z: |1/d| as capped there. c_T is bounded from the triangle's
// own normal, with one division per leaf: a triangle is skipped when its delta_T = num / c_T keeps
// the inflated box's entry beyond tb on some axis a, i.e. when
//     c_T > num |1/d_a| s / (t1_a - tb s)   for an axis with t1_a > tb s,
// evaluated with margins that round every step toward "do not skip".
RT_TC_FN uint32_t tri_leafcert_skips(const uint32_t* w, const TriConeRay& r, float tb, float t1x, float t1y, float t1z,
                                     float aix, float aiy, float aiz) {
    if (w[7] == kLeafCertNone || !(r.dlen_hi <= 1.0e5f) || !(r.olen_hi <= 1.0e15f) || !(r.inv_dlen_lo <= 1.0e5f))
        return 0u;
    const float b = leafcert_bf16(w[7] & 0xffffu), k = leafcert_bf16(w[7] >> 16);
    const float s = 1.0f + 0x1p-20f;
    const float tbs = tb * s;
    const float num = (b * (tb * r.dlen_hi + r.olen_hi) + k) * 1.00001f;
    // smallest c_T that skips: min over axes entered beyond tb (others give +inf or NaN, ignored)
    const float gx = t1x - tbs, gy = t1y - tbs, gz = t1z - tbs;
    float need = INFINITY;
    if (gx > 0.0f) need = fminf(need, (num * aix * s) / gx);
    if (gy > 0.0f) need = fminf(need, (num * aiy * s) / gy);
    if (gz > 0.0f) need = fminf(need, (num * aiz * s) / gz);
    need = fmaxf(need * 1.0001f, fmaxf(kTriConeCMin, 4.0f * b));
    if (!(need < 1.0f)) return 0u;
    // c_T >= |d.v| / |d| - kLeafCertNormalErr (|v| <= 1), the dot's rounding in the 1e-6
    const float thr = need + kLeafCertNormalErr + 1.0e-6f;
    uint32_t m = 0u;
    for (uint32_t j = 0; j < kLeafCertSlots; j++) {
        float vx, vy, vz;
        leafcert_decode(w[j], vx, vy, vz);
        const float cp = fabsf((r.dx * vx + r.dy * vy) + r.dz * vz) * r.inv_dlen_lo;
        if (cp * 0.999999f > thr) m |= 1u << j;
    }
    return m;
}

// The same test with the box entry condensed into one distance, for walks that defer it to
// their leaf batches: gap = max over axes of (t1_a - tb0 s) |d_a| (1 - 2^-20), the distance
// (lower bound) by which the leaf box's inflated-slab entry lies beyond tb0 >= tb along some
// axis; with delta_T < gap that axis still enters beyond tb. (|d_a| <= 1 / |1/d_a| as capped,
// up to the rounding the 2^-20 covers.)
RT_TC_FN uint32_t tri_leafcert_skips_gap(const uint32_t* w, const TriConeRay& r, float tb, float gap) {
    if (w[7] == kLeafCertNone || !(gap > 0.0f) || !(r.dlen_hi <= 1.0e5f) || !(r.olen_hi <= 1.0e15f) ||
        !(r.inv_dlen_lo <= 1.0e5f))
        return 0u;
    const float b = leafcert_bf16(w[7] & 0xffffu), k = leafcert_bf16(w[7] >> 16);
    const float num = (b * (tb * r.dlen_hi + r.olen_hi) + k) * 1.00001f;
    const float need = fmaxf((num / gap) * 1.0001f, fmaxf(kTriConeCMin, 4.0f * b));
    if (!(need < 1.0f)) return 0u;
    const float thr = need + kLeafCertNormalErr + 1.0e-6f;
    uint32_t m = 0u;
    for (uint32_t j = 0; j < kLeafCertSlots; j++) {
        float vx, vy, vz;
        leafcert_decode(w[j], vx, vy, vz);
        const float cp = fabsf((r.dx * vx + r.dy * vy) + r.dz * vz) * r.inv_dlen_lo;
        if (cp * 0.999999f > thr) m |= 1u << j;
    }
    return m;
}
