// rt_device_math.h — the f32 numeric contract on the device.
//
// The reference kernel (src/compute_shader.wgsl) makes its path decisions by
// comparing floats against RNG draws (:256, :274, :298) and hit distances
// against each other (:347, :391, :457); a 1-ulp difference anywhere flips a
// path. Parity with the CPU oracle is therefore bit-exact by construction:
// every function here is a fixed sequence of IEEE binary32 +,-,*,/ and sqrt
// (correctly rounded; the file is compiled with -ffp-contract=off and
// -fhip-fp32-correctly-rounded-divide-sqrt, denormals preserved), and the
// transcendentals WGSL leaves implementation-defined are pinned to
// Cephes-style f32 range reductions + minimax polynomials (<=3 ulp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace rtk {

constexpr float kF32Max = 3.4028235e+38f;   // compute_shader.wgsl:1
constexpr float kWgslPi = 3.1415926536f;    // compute_shader.wgsl:3 (f32: 3.14159274)
constexpr float kTwoPiWgsl = 2.0f * kWgslPi;
constexpr float kBoxMullerTwoPi = 6.2831850051879883f;  // `2.0 * 3.1415926` folded to f32, :624
// RN(1/c) for div_const (compile-time f32 divisions are correctly rounded)
constexpr float kInvTwoPiWgsl = 1.0f / kTwoPiWgsl;
constexpr float kInvWgslPi = 1.0f / kWgslPi;
constexpr float kInv255 = 1.0f / 255.0f;
constexpr float kInv10 = 1.0f / 10.0f;
constexpr float kPiO2 = 1.5707963267948966f;
constexpr float kPiO4 = 0.7853981633974483f;
constexpr float kPi = 3.141592653589793f;

struct f3 {
    float x, y, z;
};
struct f4 {
    float x, y, z, w;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// min/max returning the non-NaN operand (v_min_f32/v_max_f32 IEEE-mode semantics).
__device__ __forceinline__ float fmin_nn(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float fmax_nn(float a, float b) { return __builtin_fmaxf(a, b); }
#ifndef RT_SQRT_SPLIT
#define RT_SQRT_SPLIT 1
#endif
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// Correctly rounded sqrt for x in {+-0} U [2^-96, +inf] (NaN and negative x give
// NaN): the core of the compiler's IEEE expansion -- hardware v_sqrt_f32, then
// pick among s - 1ulp, s, s + 1ulp by the sign of the exact FMA residual --
// without the denormal rescaling and the special-value select the general case
// needs (16 -> 10 VALU). Used only where the argument is provably in that
// domain (each call site says why); rt_math_selftest checks it bit for bit
// against __builtin_sqrtf over every such f32 on the device.
__device__ __forceinline__ float sqrt_rn_nrm(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    return r;
}

// x / c for a constant c > 1, correctly rounded: q = x * RN(1/c) corrected once
// by the exact residual x - q*c (3 VALU + selects instead of the 10-instruction
// general division). The residual is not exact for quotients near the
// denormal range, so |x| < 2^-100 (and zeros, for their sign) take the IEEE
// division, a branch no lane takes in practice. Valid for the constants below
// only: rt_math_selftest compares it with IEEE x / c for all 2^32 f32 x.
__device__ __forceinline__ float div_const(float x, float c, float rc) {
    if (__builtin_fabsf(x) < 0x1p-100f) return x / c;
    const float q = x * rc;
    const float r = __builtin_fmaf(-q, c, x);
    const float q2 = __builtin_fmaf(r, rc, q);
    return __builtin_isinf(x) ? q : q2;
}
// Correctly rounded sqrt for any x: the short form on its proven domain (x >=
// 2^-96, +inf included), the IEEE expansion for zeros, tiny and denormal x,
// negatives and NaN (a branch whose slow side is all but never taken).
__device__ __forceinline__ float sqrt_rn_any(float x) {
#if RT_SQRT_SPLIT
    if (__builtin_expect(x >= 0x1p-96f, 1)) return sqrt_rn_nrm(x);
#endif
    return sqrt_rn(x);
}
__device__ __forceinline__ f3 normalize(f3 v) { return v * (1.0f / sqrt_rn_any(dot(v, v))); }
__device__ __forceinline__ f3 lerp(f3 a, f3 b, float t) { return a + (b - a) * t; }

__device__ __forceinline__ float logf_c(float x) {
    uint32_t b = __float_as_uint(x);
    if (x != x) return x;
    if (x < 0.0f) return __uint_as_float(0x7fc00000u);
    if (x == 0.0f) return -__builtin_inff();
    if (x == __builtin_inff()) return x;
    int e = 0;
    if (b < 0x00800000u) {  // denormal: scale into the normal range
        x = x * 8388608.0f;
        b = __float_as_uint(x);
        e = -23;
    }
    e += (int)((b >> 23) & 0xffu) - 126;
    float m = __uint_as_float((b & 0x007fffffu) | 0x3f000000u);  // [0.5, 1)
    if (m < 0.70710678118654752f) {
        e -= 1;
        m = m + m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = y * m - 1.1514610310e-1f;
    y = y * m + 1.1676998740e-1f;
    y = y * m - 1.2420140846e-1f;
    y = y * m + 1.4249322787e-1f;
    y = y * m - 1.6668057665e-1f;
    y = y * m + 2.0000714765e-1f;
    y = y * m - 2.4999993993e-1f;
    y = y * m + 3.3333331174e-1f;
    y = y * m * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    return r + 0.693359375f * fe;
}

// cos for the Box-Muller angle, |x| <= 2*pi (the contract's range; the
// oracle's only extra branch is for |x| > 8192, unreachable here).
__device__ __forceinline__ float cosf_c(float x) {
    if (x != x) return x;
    x = x < 0.0f ? -x : x;
    int j = (int)(1.27323954473516f * x);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y = y + 1.0f;
    }
    j &= 7;
    bool neg = false;
    if (j > 3) {
        j -= 4;
        neg = !neg;
    }
    if (j > 1) neg = !neg;
    const float r = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    const float z = r * r;
    float res;
    if (j == 1 || j == 2) {
        float p = -1.9515295891e-4f;
        p = p * z + 8.3321608736e-3f;
        p = p * z - 1.6666654611e-1f;
        res = p * z * r + r;
    } else {
        float p = 2.443315711809948e-5f;
        p = p * z - 1.388731625493765e-3f;
        p = p * z + 4.166664568298827e-2f;
        res = p * z * z - 0.5f * z + 1.0f;
    }
    return neg ? -res : res;
}

__device__ __forceinline__ float atanf_pos(float x) {
    float w;
    if (x > 2.414213562373095f) {
        w = kPiO2;
        x = -1.0f / x;
    } else if (x > 0.4142135623730950f) {
        w = kPiO4;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        w = 0.0f;
    }
    const float z = x * x;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    return w + (p * z * x + x);
}

__device__ __forceinline__ float atan2f_c(float y, float x) {
    if (x != x || y != y) return x + y;
    if (x == 0.0f) {
        if (y < 0.0f) return -kPiO2;
        if (y == 0.0f) return 0.0f;
        return kPiO2;
    }
    if (y == 0.0f) return x < 0.0f ? kPi : 0.0f;
    const float w = x < 0.0f ? (y < 0.0f ? -kPi : kPi) : 0.0f;
    const float q = y / x;
    if (q != q) return w + q;
    const float a = q < 0.0f ? -atanf_pos(-q) : atanf_pos(q);
    return w + a;
}

__device__ __forceinline__ float asinf_c(float x) {
    if (x != x) return x;
    const float a = x < 0.0f ? -x : x;
    if (a > 1.0f) return __uint_as_float(0x7fc00000u);
    float z;
    if (a < 1.0e-4f) {
        z = a;
    } else {
        float t, zz;
        const bool flag = a > 0.5f;
        if (flag) {
            zz = 0.5f * (1.0f - a);
            t = sqrt_rn_nrm(zz);  // zz = (1 - a)/2, a in (0.5, 1]: 0 or a multiple of 2^-25
        } else {
            t = a;
            zz = t * t;
        }
        float p = 4.2163199048e-2f;
        p = p * zz + 2.4181311049e-2f;
        p = p * zz + 4.5470025998e-2f;
        p = p * zz + 7.4953002686e-2f;
        p = p * zz + 1.6666752422e-1f;
        z = p * zz * t + t;
        if (flag) {
            z = z + z;
            z = kPiO2 - z;
        }
    }
    return x < 0.0f ? -z : z;
}

__device__ __forceinline__ float acosf_c(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return __uint_as_float(0x7fc00000u);
    // the arguments are 0 or multiples of 2^-25 (Sterbenz): sqrt_rn_nrm's domain
    if (x < -0.5f) return kPi - 2.0f * asinf_c(sqrt_rn_nrm(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asinf_c(sqrt_rn_nrm(0.5f * (1.0f - x)));
    return kPiO2 - asinf_c(x);
}

__device__ __forceinline__ float pow5(float x) {
    const float x2 = x * x;
    return (x2 * x2) * x;
}

// logf_c and cosf_c restricted to what normal01 feeds them: r = random01() in
// {0} U [2^-32, 1] (never NaN, negative, infinite or denormal) and
// theta = kBoxMullerTwoPi * r in [0, 2*pi]. Same operations on that domain,
// without the special-value branches and with both polynomials evaluated and
// selected (branch-free: the lanes of a wave disagree on the octant anyway).
// rt_math_selftest (which 5, 6) compares them bit for bit with logf_c / cosf_c
// over all 2^32 values random01 can return.
__device__ __forceinline__ float logf_u01(float x) {
    const uint32_t b = __float_as_uint(x);
    int e = (int)((b >> 23) & 0xffu) - 126;
    float m = __uint_as_float((b & 0x007fffffu) | 0x3f000000u);  // [0.5, 1)
    const bool lo = m < 0.70710678118654752f;
    e = lo ? e - 1 : e;
    m = lo ? m + m - 1.0f : m - 1.0f;
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = y * m - 1.1514610310e-1f;
    y = y * m + 1.1676998740e-1f;
    y = y * m - 1.2420140846e-1f;
    y = y * m + 1.4249322787e-1f;
    y = y * m - 1.6668057665e-1f;
    y = y * m + 2.0000714765e-1f;
    y = y * m - 2.4999993993e-1f;
    y = y * m + 3.3333331174e-1f;
    y = y * m * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    const float r = m + y;
    return x == 0.0f ? -__builtin_inff() : r + 0.693359375f * fe;
}

__device__ __forceinline__ float cosf_box(float x) {
    int j = (int)(1.27323954473516f * x);
    float y = (float)j;
    const bool odd = (j & 1) != 0;
    j = odd ? j + 1 : j;
    y = odd ? y + 1.0f : y;
    j &= 7;
    const bool neg = (j > 3) != ((j & 3) > 1);
    j &= 3;
    const float r = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    const float z = r * r;
    float ps = -1.9515295891e-4f;
    ps = ps * z + 8.3321608736e-3f;
    ps = ps * z - 1.6666654611e-1f;
    const float s_res = ps * z * r + r;
    float pc = 2.443315711809948e-5f;
    pc = pc * z - 1.388731625493765e-3f;
    pc = pc * z + 4.166664568298827e-2f;
    const float c_res = pc * z * z - 0.5f * z + 1.0f;
    const float res = (j == 1 || j == 2) ? s_res : c_res;
    return neg ? -res : res;
}

// PCG hash RNG, compute_shader.wgsl:587-599 + normalize_u32 :630-632.
__device__ __forceinline__ float random01(uint32_t& seed) {
    const uint32_t state = seed * 747796405u + 2891336453u;
    uint32_t word = (state >> ((state >> 28u) + 4u)) ^ state;
    word = word * 277803737u;
    seed = (word >> 22u) ^ word;
    return (float)seed / 4294967296.0f;  // f32(U32_MAX) == 2^32
}

// normal_distribution, compute_shader.wgsl:622-628 (theta drawn before rho).
__device__ __forceinline__ float normal01(uint32_t& seed) {
    const float theta = kBoxMullerTwoPi * random01(seed);
    // -2 log(r), r in {0} U [2^-32, 1]: -0, +inf, or >= 1.1e-7 (sqrt_rn_nrm's domain)
#ifdef RT_EXP_HW_TRANSCENDENTALS  // timing experiment only: hardware log/cos (not the contract)
    const float rho = sqrt_rn_nrm(-2.0f * __logf(random01(seed)));
    return rho * __cosf(theta);
#else
    const float rho = sqrt_rn_nrm(-2.0f * logf_u01(random01(seed)));
    return rho * cosf_box(theta);
#endif
}

}  // namespace rtk
