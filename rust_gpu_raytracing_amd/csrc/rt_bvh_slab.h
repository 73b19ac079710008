// rt_bvh_slab.h — the BVH culling slab test, shared by the kernel and the CPU
// exactness harnesses (tests/cpp/*_exactness.cpp), so both run the same f32
// arithmetic.
//
// Culling only: a node box inflated by a per-ray margin m is tested, and the
// margin covers the rounding of the reference's own
// sphere and slab arithmetic with orders of magnitude to spare. This test is
// therefore free to use its own arithmetic: per axis
//     t_lo = (lo - m - o) * inv = fma(lo, inv, -(o + m) * inv)
//     t_hi = (hi + m - o) * inv = fma(hi, inv, -(o - m) * inv)
// one FMA per plane with the ray constants precomputed, instead of sub, sub,
// mul. Its error in position units is <= ~u (|lo| + |o| + m) << m.
// A zero (or denormal) direction component makes 1/d infinite, and an FMA of
// an infinite slope can produce a NaN for only one of the two planes, which the
// NaN-ignoring min/max would turn into a false miss; |inv| is therefore capped
// at 1e30: such a ray moves < 1e-21 along that axis over any parameter range a
// hit can lie in, and an origin inside the inflated slab by >= m/2 still yields
// t_lo <= -5e23 <= +5e23 <= t_hi (unconstrained), one outside it an entry far
// beyond every other axis' exit (a miss) -- a superset of the exact answer.
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define RT_SLAB_FN __host__ __device__ __forceinline__
#else
#define RT_SLAB_FN inline
#endif

struct SlabRay {
    float ix, iy, iz;     // 1/d, |.| capped at 1e30
    float lx, ly, lz;     // -(o + m) * inv
    float hx, hy, hz;     // -(o - m) * inv
};

RT_SLAB_FN float slab_cap_inv(float v) { return fabsf(v) > 1e30f ? copysignf(1e30f, v) : v; }

// v where keep, else +inf: a bitwise merge, so the compiler cannot branch around v's arithmetic.
RT_SLAB_FN float keep_or_inf(float v, bool keep) {
    const unsigned m = 0u - (unsigned)keep;
    unsigned b;
    __builtin_memcpy(&b, &v, 4);
    b = (b & m) | (0x7f800000u & ~m);
    float r;
    __builtin_memcpy(&r, &b, 4);
    return r;
}

// Upper bounds for quantities that only size the margins (bigger = more
// conservative): 1/x and sqrt(x) from the hardware approximations (<= 1 ulp)
// rounded up by 1.000001 (~8.4u), on the host from the IEEE results.
RT_SLAB_FN float rcp_up(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x) * 1.000001f;
#else
    return (1.0f / x) * 1.000001f;
#endif
}
RT_SLAB_FN float sqrt_up(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x) * 1.000001f;
#else
    return sqrtf(x) * 1.000001f;
#endif
}

// inv: the ray's 1/d (exact, as the reference computes it); m: the margin.
RT_SLAB_FN SlabRay slab_ray(float ox, float oy, float oz, float inv_x, float inv_y, float inv_z, float m) {
    SlabRay r;
    r.ix = slab_cap_inv(inv_x);
    r.iy = slab_cap_inv(inv_y);
    r.iz = slab_cap_inv(inv_z);
    r.lx = -(ox + m) * r.ix;
    r.ly = -(oy + m) * r.iy;
    r.lz = -(oz + m) * r.iz;
    r.hx = -(ox - m) * r.ix;
    r.hy = -(oy - m) * r.iy;
    r.hz = -(oz - m) * r.iz;
    return r;
}

// Culling bounds of the sphere BVH for one ray. A BVH sphere (centre C, f32
// radius r, rho = fl(r * r), r' = sqrt(rho) <= r (1 + u)) may be skipped only where the
// reference's own test (check_spheres, compute_shader.wgsl:372-391) cannot accept it. Inputs are
// the f32 values the kernel reads; u = 2^-24, gamma_k = k u / (1 - k u); x = o - C exactly,
// X = |o| + extent >= |x| + r (extent = max over BVH spheres of |C| + r, rounded up).
//
// The reference computes, one rounding per operation: oc = fl(o - C) (|oc - x| <= u |x|),
// a = fl(d.d), g = fl(d.oc), b = 2 g, q = fl(oc.oc), c = fl(q - rho), disc = fl(fl(b b) -
// fl(4 a c)). Its exact counterpart D = B^2 - 4 A Cc with A = d.d, B = 2 d.x, Cc = x.x - rho is
// 4 |d|^2 (rho - p^2), p the distance from C to the ray's line. With the standard dot-product
// bound |fl(v.w) - v.w| <= gamma_3 |v| |w|:
//   |g - d.x|       <= (gamma_3 (1 + u) + u) |d| X                  =: e_g |d| X,  e_g <= 4.01u
//   |fl(b b) - B^2| <= |d|^2 X^2 (8 e_g + 4 e_g^2 + 4u (1 + e_g)^2)  <= 36.2u |d|^2 X^2
//   |a - A|         <= gamma_3 |d|^2
//   |q - x.x|       <= (2u + u^2 + gamma_3 (1 + u)^2) X^2           =: e_q X^2,    e_q <= 5.01u
//   |c - Cc|        <= e_q X^2 + u (q + rho) <= (e_q + u (1 + e_q)) X^2 + u rho
//   |fl(4 a c) - 4 A Cc| <= 4 |d|^2 ((gamma_3 + e_q + u) X^2 + (gamma_3 + u) rho) (1 + 4u)
//                        + 4u |d|^2 (1 + gamma_3) (X^2 + rho)  <= |d|^2 (40.1u X^2 + 20.1u rho)
//   |disc - D| <= the two above + u |fl(b b) - fl(4 a c)|, and |fl(b b) - fl(4 a c)| <=
//   |D| + both <= 4.01 |d|^2 (X^2 + rho), so
//       |disc - D| <= |d|^2 (81u X^2 + 25u rho) + E_sub,
// every second-order term above absorbed in the rounded-up integer coefficients (they are
// O(u^2), below 10^-5 of u), and E_sub <= 20 x 2^-150 the absolute rounding of products that
// underflow. Overflow cannot let the test accept: an infinite or NaN b b, 4 a c or disc makes
// disc NaN, -inf, or +inf with t = -inf or NaN, all rejected by `t > 0`. The bound is used only
// for |d|^2 >= 2^-60 (below that E_sub / |d|^2 is not negligible: sphere_cull_bounds returns
// infinite bounds, the walk culls nothing and tests every BVH sphere -- exact).
//
//  * lateral (position units, the box inflation). disc >= 0 => D >= -|disc - D| =>
//    p^2 <= rho + delta, delta = 6.25u rho + 20.25u X^2 + E_sub / (4 |d|^2) (<= 6.25u rho + 20.25u
//    X^2 + 1e-27), so p - r' <= min(delta / (2 r'), sqrt(delta)) <= min(13.25u X^2 / r_min,
//    7 sqrt(u) X) + 1e-13 (X >= r' >= r_min). The box the builder stores contains C +- r rounded
//    outward, and r' - r <= u r; this slab test's own rounding in position units is <= 4u (|lo| +
//    |o| + m) <= 16u X (its FMA form, above). The margin below uses 40u X^2 / r_min and
//    4.4e-3 X (>= 3x and 2.5x the derived terms) + 16u X + 16u r_max + 1e-6.
//  * slack (parameter units, for the depth tests `far >= -slack` and `near <= limit + slack`).
//    The accepted root t = fl(fl(-b - fl(sqrt(disc))) / fl(2 a)) is within
//    (|b - B| + sqrt|disc - D| + u |b + s|) / (2 a) (1 + gamma_3) + 3u |t| of t_ref = (-B -
//    sqrt(max(D, 0))) / (2 A): the exact entry point when the line meets the sphere, else the
//    closest-approach parameter, whose point lies within the lateral bound of C. So |t - t_ref|
//    <= (4.5 sqrt(u) X + 2.5 sqrt(u) r' + 12u X) / |d| + 3u |t| <= (1.1e-3 X + 6.2e-4 r_max +
//    15u X) / |d| (|t| <= X / |d| for an accepted root), and the point o + t_ref d lies in the
//    laterally inflated box: its slab entry is <= t_ref <= t + slack, its exit >= t - slack. The
//    slack below is 4.4e-3 (X + r_max) + 32u X, over |d| rounded down (>= 2.5x the derived one).
// Hence a box whose inflated entry lies beyond limit + slack (limit = the best sphere's t x
// 1.00001, or the triangle hit: a sphere wins only if strictly closer, :347, :391), or whose
// exit lies before -slack, holds no sphere the reference accepts with a distance that could win.
// With the RTIOW field (r = 0.2, X ~ 30) the lateral inflation is ~0.011.
// Evidence: tests/cpp/bvh_exactness.cpp (RTIOW-like scene, replayed frames, and the adversarial
// sets: radii 1e-3..1e3, tangent rays with the discriminant within a few ulp of 0 from 1..1e6
// radii away, |d| from 1e-12 to 1e6); the lateral bound cut to 0.03x fails there.
RT_SLAB_FN void sphere_cull_bounds(float olen, float extent, float r_min, float r_max, float inv_dlen,
                                   float& lateral, float& slack) {
    const float u = 5.9604645e-8f;  // 2^-24
    const float X = (olen + extent) * 1.0000005f;
    const float quad = r_min > 0.0f ? ((40.0f * u) * (X * X)) * rcp_up(r_min) : INFINITY;  // >= 3 x 13.25u X^2 / r_min
    const float lin = 4.4e-3f * X;                                               // >= 2.5 x 7 sqrt(u) X
    // |d|^2 < 2^-60 (or not finite): outside the bound's range, no culling. Merged by bit mask,
    // not by a select: the compiler turns `in_range ? expr : INFINITY` into a branch around the
    // expression, and that branch on the ray setup of every segment cost the sphere walk 1.4%
    // (round 6 bisect, profiles/r06/r06a, r06h)
    const bool in_range = inv_dlen <= 0x1p30f;
    lateral = keep_or_inf(fminf(quad, lin) + (16.0f * u) * X + (16.0f * u) * r_max + 1.0e-6f, in_range);
    slack = keep_or_inf((4.4e-3f * (X + r_max) + (32.0f * u) * X) * (inv_dlen * 1.01f) + 1.0e-30f, in_range);
}

// near/far parameters of the inflated box [lo, hi] (min/max ignore NaN operands).
RT_SLAB_FN void slab_hit(const SlabRay& r, float lox, float loy, float loz, float hix, float hiy, float hiz,
                         float& near_t, float& far_t) {
    const float tx0 = fmaf(lox, r.ix, r.lx), tx1 = fmaf(hix, r.ix, r.hx);
    const float ty0 = fmaf(loy, r.iy, r.ly), ty1 = fmaf(hiy, r.iy, r.hy);
    const float tz0 = fmaf(loz, r.iz, r.lz), tz1 = fmaf(hiz, r.iz, r.hz);
    near_t = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
    far_t = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
}

// slab_hit with the per-axis entry parameters kept (near_t = their maximum, the same operations):
// the certified pruning's gap of a leaf box beyond the best hit reads them (tri_cone.h).
RT_SLAB_FN void slab_hit_axes(const SlabRay& r, float lox, float loy, float loz, float hix, float hiy, float hiz,
                              float& t1x, float& t1y, float& t1z, float& far_t) {
    const float tx0 = fmaf(lox, r.ix, r.lx), tx1 = fmaf(hix, r.ix, r.hx);
    const float ty0 = fmaf(loy, r.iy, r.ly), ty1 = fmaf(hiy, r.iy, r.hy);
    const float tz0 = fmaf(loz, r.iz, r.lz), tz1 = fmaf(hiz, r.iz, r.hz);
    t1x = fminf(tx0, tx1);
    t1y = fminf(ty0, ty1);
    t1z = fminf(tz0, tz1);
    far_t = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
}

// Box-ordered layouts (order_bvh_by_octant with swap_boxes): layout k stores
// every box as (near corner, far corner) for rays of direction octant k, i.e.
// bmin/bmax swapped on the axes where bit k is set (the ray travels towards
// -axis). The ray's constants are paired the same way (slab_pair_by_octant: l*
// with the near corner, h* with the far one), so each slab's nearer plane is
// known and the test needs no min/max per axis. It is the same arithmetic as
// slab_hit on the unswapped box: for lo <= hi and a finite slope, rounding is
// monotone, so fma(lo, ix, lx) <= fma(hi, ix, hx) when ix >= 0 and >= when
// ix < 0 -- exactly the operands slab_hit's min/max would pick. The NaN-free
// premise (|plane * ix| <= 1e8 * 1e30 stays finite) is what box_layout_orderable
// checks on the host; a NaN origin makes both planes of an axis NaN, which both
// forms ignore alike.
RT_SLAB_FN void slab_pair_by_octant(SlabRay& r) {
    const bool nx = signbit(r.ix), ny = signbit(r.iy), nz = signbit(r.iz);
    const float lx = nx ? r.hx : r.lx, hx = nx ? r.lx : r.hx;
    const float ly = ny ? r.hy : r.ly, hy = ny ? r.ly : r.hy;
    const float lz = nz ? r.hz : r.lz, hz = nz ? r.lz : r.hz;
    r.lx = lx;
    r.hx = hx;
    r.ly = ly;
    r.hy = hy;
    r.lz = lz;
    r.hz = hz;
}

// near/far parameters of a box stored as (near corner n, far corner f).
RT_SLAB_FN void slab_hit_ordered(const SlabRay& r, float nx, float ny, float nz, float fx, float fy, float fz,
                                 float& near_t, float& far_t) {
    near_t = fmaxf(fmaxf(fmaf(nx, r.ix, r.lx), fmaf(ny, r.iy, r.ly)), fmaf(nz, r.iz, r.lz));
    far_t = fminf(fminf(fmaf(fx, r.ix, r.hx), fmaf(fy, r.iy, r.hy)), fmaf(fz, r.iz, r.hz));
}
