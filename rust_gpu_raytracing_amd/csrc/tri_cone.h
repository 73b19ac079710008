// tri_cone.h -- certified distance pruning of the triangle walk.
//
// Once a walk holds a triangle hit at distance tb, a node may be skipped only if no
// triangle below it can pass the reference's f32 test (compute_shader.wgsl:449-481)
// with a distance <= tb. Per node this header keeps what proves it: a double cone
// bounding the directions of every triangle normal N = ab x ac below the node (axis A,
// half-angle phi; N and -N alike), and two coefficients b, k of the f32 error bound.
//
// The bound (derived in DESIGN.md §5.3c). If the f32 test accepts triangle T with
// distance t, the point o + t d lies within
//     delta_T = (b_T (t |d| + |o|) + k_T) / c_T,     c_T = |d . N| / (|d| |N|),
// of T, where b_T and k_T depend only on T's stored record (its f32 calc_normal n may
// differ from the exact N: |N - n| enters both), the triangle's corners may lie outside
// its sub-object box by at most what k_T adds, and u = 2^-24:
//     b_T = (|N - n| + 8u |n| + 32u |ab| |ac|) / |N|
//     k_T = b_T |a| + (|ab| + |ac|) (|N - n| + 8u |n|) / |N| + excess_T + 2u (|ab| + |ac|)
// So the ray, which holds that point at parameter t <= tb, enters the node box
// inflated by delta = max_T delta_T no later than t. Conversely, when the inflated
// box's entry (a certified lower bound, tri_cone_prunes) lies beyond tb, every
// triangle below the node that the reference could accept has distance > tb: the
// node cannot change the walk's lexicographic (distance, sweep position) minimum,
// ties included (strict). c_T is bounded below from the cone: with psi the angle
// between d and the axis (folded to [0, pi/2]), c_T >= cos(psi + phi) whenever
// psi + phi < pi/2. A node whose cone is wider than a hemisphere, or whose
// triangles have a non-finite or degenerate record, is never pruned: it is walked
// with box culling alone, which is exact without any bound.
//
// Shared by the device builder (rt_tri_cones_kernel, scene_edit.hip), the walks
// (pathtrace.hip) and the CPU exactness harness (tests/cpp/tri_exactness.cpp).
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define RT_TC_FN __host__ __device__ inline
#else
#define RT_TC_FN inline
#endif

struct TriCone {
    float ax, ay, az;  // cone axis (unit up to f32 rounding)
    float cos_lo;      // cos(phi + slack), rounded down
    float sin_hi;      // sin(phi + slack), rounded up
    float b, k;        // error coefficients (header comment), rounded up
    uint32_t flags;    // kTriConeValid | kTriConeNarrow
};
static_assert(sizeof(TriCone) == 32, "cone record layout");

constexpr uint32_t kTriConeValid = 1u;   // every triangle below has a finite, non-degenerate record
constexpr uint32_t kTriConeNarrow = 2u;  // phi < pi/2: the cone can bound c_T away from 0
constexpr uint32_t kTriConePrunable = kTriConeValid | kTriConeNarrow;

// Smallest cone lower bound the walk accepts (below it delta is too large to prune anyway).
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

// Running state of a cone/coefficient build over a node's triangles (double).
struct Acc {
    double ax, ay, az;  // axis (unit), valid when n > 0
    double phi;         // half-angle (radians), an upper bound
    double b, k;
    uint32_t n;         // triangles (or children) merged
    bool valid;
};

RT_TC_FN Acc acc_empty() { return Acc{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0u, true}; }

RT_TC_FN double angle_between(double x0, double y0, double z0, double x1, double y1, double z1) {
    // both unit; |cos| folded (N and -N alike); acos error covered by the +1e-9 slack of the callers
    double c = fabs(x0 * x1 + y0 * y1 + z0 * z1);
    c = c > 1.0 ? 1.0 : c;
    return acos(c);
}

// Adds a cone (unit axis x, half-angle p) to acc: the new axis is the sign-aligned
// sum of the two axes, the new half-angle the larger of (angle to each old axis +
// its half-angle). Conservative: every direction in either cone is in the result.
RT_TC_FN void acc_add_cone(Acc& acc, double x, double y, double z, double p) {
    if (acc.n == 0u) {
        acc.ax = x;
        acc.ay = y;
        acc.az = z;
        acc.phi = p;
        acc.n = 1u;
        return;
    }
    const double s = (acc.ax * x + acc.ay * y + acc.az * z) < 0.0 ? -1.0 : 1.0;
    // weight the running axis by its count so a leaf's axis is near the normals' mean
    const double w = (double)acc.n;
    double nx = acc.ax * w + s * x, ny = acc.ay * w + s * y, nz = acc.az * w + s * z;
    const double l = len3(nx, ny, nz);
    if (!(l > 1e-12)) {  // opposite axes cancel: keep the old axis
        nx = acc.ax;
        ny = acc.ay;
        nz = acc.az;
    } else {
        nx /= l;
        ny /= l;
        nz /= l;
    }
    const double p_old = angle_between(nx, ny, nz, acc.ax, acc.ay, acc.az) + acc.phi;
    const double p_new = angle_between(nx, ny, nz, x, y, z) + p;
    acc.ax = nx;
    acc.ay = ny;
    acc.az = nz;
    acc.phi = (p_old > p_new ? p_old : p_new) + 1e-9;
    acc.n += 1u;
}

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
    acc_add_cone(acc, Nx / NN, Ny / NN, Nz / NN, 1e-9);
}

// A merged node: both children's triangles.
RT_TC_FN void acc_add_acc(Acc& acc, const Acc& c) {
    acc.valid = acc.valid && c.valid;
    acc.b = fmax(acc.b, c.b);
    acc.k = fmax(acc.k, c.k);
    if (c.n > 0u) {
        const uint32_t n = acc.n;
        acc_add_cone(acc, c.ax, c.ay, c.az, c.phi);
        acc.n = n + c.n;
    }
}

// The f32 record. Slack on the angle covers the axis' f32 rounding (<= ~2^-23 rad) and
// the kernel's evaluation of cos(psi) (tri_cone_prunes).
RT_TC_FN TriCone acc_record(const Acc& acc) {
    TriCone r{0.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0u};
    if (!acc.valid || acc.n == 0u) return r;
    r.flags = kTriConeValid;
    r.b = f_up(acc.b * (1.0 + 1e-6));
    r.k = f_up(acc.k * (1.0 + 1e-6) + 1e-30);
    const double phi = acc.phi + 1e-6;
    if (phi < 1.5707963267948966 - 1e-6) {
        r.flags |= kTriConeNarrow;
        r.ax = (float)acc.ax;
        r.ay = (float)acc.ay;
        r.az = (float)acc.az;
        r.cos_lo = f_down(cos(phi) - 1e-12);
        r.sin_hi = f_up(sin(phi) + 1e-12);
    }
    return r;
}

// Back to the double state (for a parent's merge): phi from the stored, conservative
// cos/sin; a record that is not narrow has no usable axis (phi = pi/2 stays pi/2 up).
RT_TC_FN Acc acc_from_record(const TriCone& r) {
    Acc a = acc_empty();
    a.valid = (r.flags & kTriConeValid) != 0u;
    a.b = r.b;
    a.k = r.k;
    a.n = 1u;
    if (r.flags & kTriConeNarrow) {
        const double l = len3(r.ax, r.ay, r.az);
        a.ax = r.ax / l;
        a.ay = r.ay / l;
        a.az = r.az / l;
        a.phi = atan2((double)r.sin_hi, (double)r.cos_lo) + 1e-9;
    } else {
        a.ax = 1.0;
        a.phi = 3.2;  // wider than a hemisphere: every merge stays wide
    }
    return a;
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

// True when the node (cone record c) cannot hold a triangle the reference accepts at a
// distance <= tb. t1x..z: the culling slab test's per-axis entry parameters of the node box
// (inflated by the culling margin; rt_bvh_slab.h), aix..z: |1/d| as capped there.
// Every step rounds toward "do not prune" (DESIGN.md §5.3c).
RT_TC_FN bool tri_cone_prunes(const TriCone& c, const TriConeRay& r, float tb, float t1x, float t1y, float t1z,
                              float aix, float aiy, float aiz) {
    if ((c.flags & kTriConePrunable) != kTriConePrunable || !(r.dlen_hi <= 1.0e5f) || !(r.olen_hi <= 1.0e15f) ||
        !(r.inv_dlen_lo <= 1.0e5f))
        return false;
    // cos(psi) = |d.A| / |d| to within 1e-6 (f32 dot, |A| = 1 +- 2^-23)
    const float cp = fabsf((r.dx * c.ax + r.dy * c.ay) + r.dz * c.az) * r.inv_dlen_lo;
    const float cl = fmaxf(cp - 1.0e-6f, 0.0f);
    const float su = sqrtf(fmaxf(1.0f - cl * cl, 0.0f) + 4.0e-6f);
    const float clb = (cl * c.cos_lo - su * c.sin_hi) - 1.0e-6f;
    if (!(clb >= kTriConeCMin) || !(clb >= 4.0f * c.b)) return false;
    const float num = (c.b * (tb * r.dlen_hi + r.olen_hi) + c.k) * 1.00001f;
    const float delta = (num / clb) * 1.00001f;
    const float s = 1.0f + 0x1p-20f;
    const float nx = t1x - (delta * aix) * s;
    const float ny = t1y - (delta * aiy) * s;
    const float nz = t1z - (delta * aiz) * s;
    return fmaxf(fmaxf(nx, ny), nz) > tb * s;
}
