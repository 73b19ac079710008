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

// Culling bounds of the sphere BVH for one ray, with X =
// |o| + extent >= |o - C| for every BVH sphere (centre C, radius r in
// [r_min, r_max]) and u = 2^-24:
//
//  * lateral (position units, the box inflation). The reference's float
//    discriminant (:372-379) differs from the exact 4|d|^2 (r^2 - p^2) (p = the
//    distance from C to the ray line) by at most |d|^2 (80u X^2 + 24u r^2) to
//    first order, so `disc >= 0` implies p^2 <= r^2 (1 + 8u) + 20u X^2, i.e.
//    p - r <= min(10u X^2 / r, sqrt(20u) X) + 4u r. Taken 4x, plus the
//    builder's f32 box rounding and this slab test's own (<= ~2u X each, 16u X
//    allowed).
//  * slack (parameter units, for the depth tests `far >= -slack` and
//    `near <= limit + slack`). The float near root lies at most
//    sqrt(|E|) / (2|d|^2) <= sqrt(20u) (X + r) / |d| (+ ~6u X / |d| of
//    rounding) before the exact entry point, or -- for a line that misses the
//    exact sphere but still has disc >= 0 -- before the closest-approach point,
//    which lies inside the laterally inflated box. Taken 4x.
//
// With the RTIOW field (r = 0.2, X ~ 30) the lateral inflation is ~0.011
// instead of the 0.12 of the r-independent sqrt(u) X bound alone.
RT_SLAB_FN void sphere_cull_bounds(float olen, float extent, float r_min, float r_max, float inv_dlen,
                                   float& lateral, float& slack) {
    const float u = 5.9604645e-8f;  // 2^-24
    const float X = (olen + extent) * 1.0000005f;
    const float quad = r_min > 0.0f ? ((40.0f * u) * (X * X)) * rcp_up(r_min) : INFINITY;  // 4 x 10u X^2 / r
    const float lin = 4.4e-3f * X;                                               // ~4 x sqrt(20u) X
    lateral = fminf(quad, lin) + (16.0f * u) * X + (16.0f * u) * r_max + 1.0e-6f;
    slack = (4.4e-3f * (X + r_max) + (32.0f * u) * X) * (inv_dlen * 1.01f) + 1.0e-30f;
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
