/*
 * pathtrace_oracle.c — CPU ORACLE (test infrastructure, never shipped).
 *
 * A scalar, strict-IEEE restatement of the reference's per-pixel path tracer
 * `src/compute_shader.wgsl` (juhotuho10/rust_GPU_raytracing). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (rust_gpu_raytracing_amd/) never does.
 *
 * PARITY UNPINNED against the reference itself: the reference is Rust + WGSL on
 * wgpu/Vulkan; no Rust toolchain, no Vulkan ICD and no WGSL compiler exist in
 * this image, and the reference ships no tests, golden images or known-answer
 * vectors. The oracle is pinned instead by
 *   - known-answer tests of each primitive against independent computations
 *     (pure-Python integer PCG, libm in double precision, closed-form
 *     sphere/triangle hits), tests/test_oracle_*.py;
 *   - the SURVEY.md Appendix B PCG vectors;
 *   - committed golden images produced by this file (tests/golden/).
 *
 * Numeric contract (shared with the HIP kernel): every f32
 * operation is a single IEEE-754 binary32 op, round-to-nearest, no FMA
 * contraction (build with -ffp-contract=off), denormals preserved. WGSL
 * leaves transcendentals implementation-defined; this contract fixes them to
 * the f32 algorithms below (Cephes-style range reduction + minimax
 * polynomials, ~1-2 ulp, checked against libm in double by the tests).
 * `pow(x, 5.0)` is x*x*x*x*x; `normalize(v)` is v * (1/sqrt(dot(v,v)));
 * dot is ((x*x' + y*y') + z*z'); min/max return the non-NaN operand.
 *
 * Out-of-range behaviour follows naga's "Restrict" policy (SURVEY Appendix A
 * item 8): texel coordinates are truncated toward zero and clamped to
 * [0, size-1] (NaN -> 0); texture layer clamped to [0, layers-1].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define F32_MAX 3.4028235e+38f            /* compute_shader.wgsl:1 */
#define WGSL_PI 3.1415926536f             /* compute_shader.wgsl:3 (rounds to 3.14159274f) */
#define TILE 8                            /* 8x8 pixel tiles */

/* ---------------- POD layouts: src/buffers.rs:7-129 ---------------------- */
typedef struct { uint32_t screen_width, accumulation_index, accumulate, sphere_count, object_count,
                 compute_per_frame, texture_width, texture_height, texture_count, env_map_width,
                 env_map_height, _pad; } OParams;                          /* 48 B */
typedef struct { float x, y, z; uint32_t _pad; } OVec;                   /* 16 B: Ray, RayCamera */
typedef struct { float pos[3]; float radius; uint32_t material_index; uint32_t _pad[3]; } OSphere;
typedef struct { float a[3]; uint32_t p0; float ab[3]; uint32_t p1; float ac[3]; uint32_t p2;
                 float cn[3]; uint32_t p3; float fn[3]; uint32_t p4; float mn[3]; uint32_t p5;
                 float mx[3]; uint32_t p6; } OTriangle;                  /* 112 B */
typedef struct { uint32_t texture_index; float roughness, emission_power, specular, specular_scatter,
                 glass, refraction_index; uint32_t _pad; } OMaterial;    /* 32 B */
typedef struct { float mn[3]; uint32_t first_sub; float mx[3]; uint32_t sub_count; uint32_t material_index;
                 uint32_t _pad[3]; } OObject;                            /* 48 B */
typedef struct { float mn[3]; uint32_t first_tri; float mx[3]; uint32_t tri_count; } OSub; /* 32 B */

typedef char oracle_size_check[(sizeof(OParams) == 48 && sizeof(OSphere) == 32 && sizeof(OTriangle) == 112 &&
                                sizeof(OMaterial) == 32 && sizeof(OObject) == 48 && sizeof(OSub) == 32) ? 1 : -1];

/* Everything bound to the compute pipeline (compute_shader.wgsl:12-23). */
typedef struct {
    const float* camera_origin;      /* binding 3, 3 floats */
    const OVec* camera_rays;         /* binding 1 */
    const OMaterial* materials; uint32_t material_count;
    const OSphere* spheres; uint32_t sphere_capacity;
    const OTriangle* triangles; uint32_t triangle_count;
    const OObject* objects; uint32_t object_capacity;
    const OSub* subs; uint32_t sub_count;
    const uint8_t* textures; uint32_t tex_w, tex_h, tex_layers;  /* binding 9, RGBA8 sRGB */
    const uint8_t* env; uint32_t env_w, env_h;                   /* binding 11, RGBA8 sRGB */
} OScene;

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

static inline v3 mk3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3s(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
static inline v3 neg3(v3 a) { return mk3(-a.x, -a.y, -a.z); }
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline v3 cross3(v3 a, v3 b) {
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float ofminf(float a, float b) { if (a != a) return b; if (b != b) return a; return b < a ? b : a; }
static inline float ofmaxf(float a, float b) { if (a != a) return b; if (b != b) return a; return b > a ? b : a; }
static inline v3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ---------------- numeric contract: transcendentals --------------------- */

#define C_PIO2F 1.5707963267948966f
#define C_PIO4F 0.7853981633974483f
#define C_PIF 3.141592653589793f

float oracle_logf(float x) {
    if (x != x) return x;
    if (x < 0.0f) return u2f(0x7fc00000u);
    if (x == 0.0f) return -INFINITY;
    if (x == INFINITY) return x;
    uint32_t b = f2u(x);
    int e = 0;
    if (b < 0x00800000u) { x = x * 8388608.0f; b = f2u(x); e = -23; }   /* denormal: scale by 2^23 */
    e += (int)((b >> 23) & 0xffu) - 126;
    float m = u2f((b & 0x007fffffu) | 0x3f000000u);                       /* m in [0.5, 1) */
    if (m < 0.70710678118654752f) { e -= 1; m = m + m - 1.0f; } else { m = m - 1.0f; }
    float z = m * m;
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
    float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    r = r + 0.693359375f * fe;
    return r;
}

float oracle_cosf(float x) {
    if (x != x) return x;
    if (x == INFINITY || x == -INFINITY) return u2f(0x7fc00000u);
    x = x < 0.0f ? -x : x;
    if (x > 8192.0f) {            /* outside the reduction's accuracy range: never reached by the path */
        return (float)cos((double)x);
    }
    int sign = 1;
    int j = (int)(1.27323954473516f * x);
    float y = (float)j;
    if (j & 1) { j += 1; y = y + 1.0f; }
    j &= 7;
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    float r = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float z = r * r;
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
    return sign < 0 ? -res : res;
}

static float oatanf_pos(float x) { /* x >= 0, finite or +inf */
    float y, w;
    if (x > 2.414213562373095f) { w = C_PIO2F; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { w = C_PIO4F; x = (x - 1.0f) / (x + 1.0f); }
    else { w = 0.0f; }
    float z = x * x;
    float p = 8.05374449538e-2f;
    p = p * z - 1.38776856032e-1f;
    p = p * z + 1.99777106478e-1f;
    p = p * z - 3.33329491539e-1f;
    y = w + (p * z * x + x);
    return y;
}

float oracle_atanf(float x) {
    if (x != x) return x;
    if (x < 0.0f) return -oatanf_pos(-x);
    return oatanf_pos(x);
}

float oracle_atan2f(float y, float x) {
    if (x != x || y != y) return x + y;
    if (x == 0.0f) {
        if (y < 0.0f) return -C_PIO2F;
        if (y == 0.0f) return 0.0f;
        return C_PIO2F;
    }
    if (y == 0.0f) {
        if (x < 0.0f) return C_PIF;
        return 0.0f;
    }
    float w;
    if (x < 0.0f) w = (y < 0.0f) ? -C_PIF : C_PIF;
    else w = 0.0f;
    return w + oracle_atanf(y / x);
}

float oracle_asinf(float x) {
    if (x != x) return x;
    float a = x < 0.0f ? -x : x;
    if (a > 1.0f) return u2f(0x7fc00000u);
    float z;
    if (a < 1.0e-4f) {
        z = a;
    } else {
        float t, zz;
        int flag;
        if (a > 0.5f) { zz = 0.5f * (1.0f - a); t = sqrtf(zz); flag = 1; }
        else { t = a; zz = t * t; flag = 0; }
        float p = 4.2163199048e-2f;
        p = p * zz + 2.4181311049e-2f;
        p = p * zz + 4.5470025998e-2f;
        p = p * zz + 7.4953002686e-2f;
        p = p * zz + 1.6666752422e-1f;
        z = p * zz * t + t;
        if (flag) { z = z + z; z = C_PIO2F - z; }
    }
    return x < 0.0f ? -z : z;
}

float oracle_acosf(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return u2f(0x7fc00000u);
    if (x < -0.5f) return C_PIF - 2.0f * oracle_asinf(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * oracle_asinf(sqrtf(0.5f * (1.0f - x)));
    return C_PIO2F - oracle_asinf(x);
}

static inline float opow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

static inline v3 onormalize(v3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return mul3s(v, inv); }
static inline float olength(v3 v) { return sqrtf(dot3(v, v)); }

/* ---------------- RNG: compute_shader.wgsl:587-632 ----------------------- */

float oracle_random(uint32_t* seed) {
    uint32_t state = *seed * 747796405u + 2891336453u;
    uint32_t word = (state >> ((state >> 28u) + 4u)) ^ state;
    word = word * 277803737u;
    *seed = (word >> 22u) ^ word;
    return (float)(*seed) / 4294967296.0f;     /* f32(U32_MAX) rounds to 2^32 */
}

static inline float onormal_distribution(uint32_t* seed) {       /* :622-628 */
    float theta = 6.2831850051879883f * oracle_random(seed);      /* 2.0 * 3.1415926 folded to f32 */
    float rho = sqrtf(-2.0f * oracle_logf(oracle_random(seed)));
    return rho * oracle_cosf(theta);
}

/* ---------------- textures: compute_shader.wgsl:26-40 -------------------- */

static float g_srgb[256];
static int g_srgb_ready = 0;

void oracle_srgb_table(float out[256]) {
    for (int i = 0; i < 256; i++) {
        double c = (double)i / 255.0;
        double l = c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4);
        out[i] = (float)l;
    }
}

static void ensure_srgb(void) {
    if (!g_srgb_ready) {
        oracle_srgb_table(g_srgb);
        g_srgb_ready = 1;
    }
}

static inline int texel_coord(float c, uint32_t size) {
    if (!(c >= 0.0f)) return 0;           /* negative or NaN */
    if (c >= (float)size) return (int)size - 1;
    int i = (int)c;
    return i > (int)size - 1 ? (int)size - 1 : i;
}

static inline v4 decode_texel(const uint8_t* p) {
    v4 r = {g_srgb[p[0]], g_srgb[p[1]], g_srgb[p[2]], (float)p[3] / 255.0f};
    return r;
}

static v4 sample_texture(const OScene* s, const OParams* pr, uint32_t index, float u, float v) {
    int x = texel_coord(u * (float)(int32_t)pr->texture_width, s->tex_w);
    int y = texel_coord(v * (float)(int32_t)pr->texture_height, s->tex_h);
    uint32_t layer = index >= s->tex_layers ? s->tex_layers - 1 : index;
    size_t off = (((size_t)layer * s->tex_h + (size_t)y) * s->tex_w + (size_t)x) * 4;
    return decode_texel(s->textures + off);
}

static v4 sample_env(const OScene* s, const OParams* pr, float u, float v) {
    int x = texel_coord(u * (float)(int32_t)pr->env_map_width, s->env_w);
    int y = texel_coord(v * (float)(int32_t)pr->env_map_height, s->env_h);
    size_t off = ((size_t)y * s->env_w + (size_t)x) * 4;
    return decode_texel(s->env + off);
}

/* ---------------- intersection: compute_shader.wgsl:342-585 -------------- */

typedef struct {
    float t;
    v3 p, n;
    uint32_t material_index;
    int front_face;
    float u, v;
} OHit;

static inline OHit omiss(void) {
    OHit h;
    memset(&h, 0, sizeof(h));
    h.t = F32_MAX;
    return h;
}

static OHit check_spheres(const OScene* s, const OParams* pr, v3 o, v3 d) {   /* :355-404 */
    float closest = F32_MAX;
    int closest_i = -1;
    float a = dot3(d, d);
    int n = (int)pr->sphere_count;
    for (int i = 0; i < n; i++) {
        const OSphere* sp = &s->spheres[i];
        v3 oc = sub3(o, ld3(sp->pos));
        float b = 2.0f * dot3(d, oc);
        float c = dot3(oc, oc) - sp->radius * sp->radius;
        float disc = b * b - 4.0f * a * c;
        if (disc < 0.0f) continue;
        float t = (-b - sqrtf(disc)) / (2.0f * a);
        if (t > 0.0f && t < closest) { closest = t; closest_i = i; }
    }
    if (closest_i < 0) return omiss();
    /* sphere_hit, :530-555 */
    const OSphere* sp = &s->spheres[closest_i];
    OHit h;
    h.t = closest;
    h.p = add3(o, mul3s(d, closest));
    v3 outward = onormalize(sub3(h.p, ld3(sp->pos)));
    /* sphere_texture_coords, :557-566 */
    float theta = oracle_acosf(-outward.y);
    float phi = oracle_atan2f(-outward.z, outward.x) + WGSL_PI;
    h.u = phi / (2.0f * WGSL_PI);
    h.v = theta / WGSL_PI;
    h.front_face = dot3(d, outward) < 0.0f;
    h.n = h.front_face ? outward : neg3(outward);
    h.material_index = sp->material_index;
    return h;
}

static inline int ray_in_bounds(v3 o, v3 d, const float* mn, const float* mx) {   /* :407-419 */
    v3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    v3 tmin = mk3((mn[0] - o.x) * inv.x, (mn[1] - o.y) * inv.y, (mn[2] - o.z) * inv.z);
    v3 tmax = mk3((mx[0] - o.x) * inv.x, (mx[1] - o.y) * inv.y, (mx[2] - o.z) * inv.z);
    v3 t1 = mk3(ofminf(tmin.x, tmax.x), ofminf(tmin.y, tmax.y), ofminf(tmin.z, tmax.z));
    v3 t2 = mk3(ofmaxf(tmin.x, tmax.x), ofmaxf(tmin.y, tmax.y), ofmaxf(tmin.z, tmax.z));
    float near_t = ofmaxf(ofmaxf(t1.x, t1.y), t1.z);
    float far_t = ofminf(ofminf(t2.x, t2.y), t2.z);
    return near_t <= far_t && far_t >= 0.0f;
}

static OHit check_triangles(const OScene* s, const OParams* pr, v3 o, v3 d) {   /* :422-517 */
    float closest = F32_MAX;
    OHit best = omiss();
    for (uint32_t oi = 0; oi < pr->object_count; oi++) {
        const OObject* ob = &s->objects[oi];
        if (!ray_in_bounds(o, d, ob->mn, ob->mx)) continue;
        for (uint32_t i = 0; i < ob->sub_count; i++) {
            uint32_t si = ob->first_sub + i;
            if (si >= s->sub_count) si = s->sub_count - 1;
            const OSub* sub = &s->subs[si];
            if (!ray_in_bounds(o, d, sub->mn, sub->mx)) continue;
            for (uint32_t j = 0; j < sub->tri_count; j++) {
                uint32_t ti = sub->first_tri + j;
                if (ti >= s->triangle_count) ti = s->triangle_count - 1;
                const OTriangle* tr = &s->triangles[ti];
                v3 cn = ld3(tr->cn);
                float det = -dot3(d, cn);
                float inv_det = 1.0f / det;
                v3 ao = sub3(o, ld3(tr->a));
                float dist = dot3(ao, cn) * inv_det;
                if (dist < 0.0f || dist >= closest) continue;
                v3 dao = cross3(ao, d);
                float v = -dot3(ld3(tr->ab), dao) * inv_det;
                if (v < 0.0f) continue;
                float u = dot3(ld3(tr->ac), dao) * inv_det;
                if (u < 0.0f) continue;
                float w = 1.0f - u - v;
                if (w < 0.0f) continue;
                v3 fn = ld3(tr->fn);
                best.front_face = det > 0.0f;
                best.n = best.front_face ? fn : neg3(fn);
                closest = dist;
                best.t = dist;
                best.p = add3(o, mul3s(d, dist));
                /* object_texture_coords, :568-578 */
                float rx = ob->mx[0] - ob->mn[0], rz = ob->mx[2] - ob->mn[2];
                best.u = (best.p.x - ob->mn[0]) / rx;
                best.v = (best.p.z - ob->mn[2]) / rz;
                best.material_index = ob->material_index;
            }
        }
    }
    return best;
}

/* Optional trace log (test/analysis only): records (o, d) of every trace_ray
 * call, for replaying real ray distributions through traversal experiments.
 * Only meaningful with one thread. */
static float* g_trace_log = 0;
static uint64_t g_trace_cap = 0, g_trace_n = 0;

void oracle_set_trace_log(float* buf, uint64_t cap) {
    g_trace_log = buf;
    g_trace_cap = cap;
    g_trace_n = 0;
}

uint64_t oracle_trace_log_count(void) { return g_trace_n; }

static inline OHit trace_ray(const OScene* s, const OParams* pr, v3 o, v3 d) {   /* :342-353 */
    if (g_trace_log && g_trace_n < g_trace_cap) {
        float* q = g_trace_log + 6 * g_trace_n++;
        q[0] = o.x; q[1] = o.y; q[2] = o.z; q[3] = d.x; q[4] = d.y; q[5] = d.z;
    }
    OHit hs = check_spheres(s, pr, o, d);
    OHit ht = check_triangles(s, pr, o, d);
    return hs.t < ht.t ? hs : ht;
}

/* Exposed for known-answer tests: closest hit of one ray. */
typedef struct { float t, px, py, pz, nx, ny, nz, u, v; uint32_t material_index; int32_t front_face; } OHitOut;

void oracle_trace(const OScene* s, const OParams* pr, const float* o, const float* d, OHitOut* out) {
    ensure_srgb();
    OHit h = trace_ray(s, pr, ld3(o), ld3(d));
    out->t = h.t; out->px = h.p.x; out->py = h.p.y; out->pz = h.p.z;
    out->nx = h.n.x; out->ny = h.n.y; out->nz = h.n.z; out->u = h.u; out->v = h.v;
    out->material_index = h.material_index; out->front_face = h.front_face;
}

/* ---------------- per_pixel: compute_shader.wgsl:210-339 ----------------- */

static v4 per_pixel(const OScene* s, const OParams* pr, uint32_t index, uint32_t bounces, uint32_t random_index,
                    uint64_t* rays) {
    v3 o = ld3(s->camera_origin);
    const OVec* cr = &s->camera_rays[index];
    v3 d = mk3(cr->x, cr->y, cr->z);
    uint32_t seed = index * random_index * 326624u;
    {   /* random_scaler(&seed) * 0.0005, :612-620 */
        float rx = oracle_random(&seed), ry = oracle_random(&seed), rz = oracle_random(&seed);
        v3 j = mk3(rx * 2.0f - 1.0f, ry * 2.0f - 1.0f, rz * 2.0f - 1.0f);
        d = add3(d, mul3s(j, 0.0005f));
    }
    v4 contrib = {1.0f, 1.0f, 1.0f, 1.0f};
    v4 light = {0.0f, 0.0f, 0.0f, 0.0f};
    for (uint32_t i = 0; i < bounces; i++) {
        OHit h = trace_ray(s, pr, o, d);
        (*rays)++;
        if (h.t == F32_MAX) {
            /* environment_map_coords, :580-585 */
            float u = 0.5f + oracle_atan2f(d.z, d.x) / (2.0f * WGSL_PI);
            float v = 0.5f + oracle_asinf(d.y) / WGSL_PI;
            v4 c = sample_env(s, pr, u, v);
            light.x = light.x + c.x * contrib.x; light.y = light.y + c.y * contrib.y;
            light.z = light.z + c.z * contrib.z; light.w = light.w + c.w * contrib.w;
            break;
        }
        uint32_t mi = h.material_index >= s->material_count ? s->material_count - 1 : h.material_index;
        const OMaterial* m = &s->materials[mi];
        float gx = onormal_distribution(&seed);
        float gy = onormal_distribution(&seed);
        float gz = onormal_distribution(&seed);
        v3 diffuse = onormalize(add3(h.n, mk3(gx, gy, gz)));
        v3 specular = sub3(d, mul3s(h.n, 2.0f * dot3(h.n, d)));      /* reflect(d, n) */
        v4 color = sample_texture(s, pr, m->texture_index, h.u, h.v);
        float e = m->emission_power;
        light.x = light.x + (color.x * e) * contrib.x; light.y = light.y + (color.y * e) * contrib.y;
        light.z = light.z + (color.z * e) * contrib.z; light.w = light.w + (color.w * e) * contrib.w;
        int is_glass = m->glass > oracle_random(&seed);
        if (is_glass) {
            float ior = m->refraction_index;
            if (h.front_face) ior = 1.0f / ior;
            float cos_t = ofminf(dot3(neg3(d), h.n), 1.0f);
            float sin_t = sqrtf(1.0f - cos_t * cos_t);
            int reflects = ior * sin_t > 1.0f;
            float r0 = (1.0f - ior) / (1.0f + ior);                  /* specular_percentage, :328-334 */
            r0 = r0 * r0;
            float sp = r0 + (1.0f - r0) * opow5(1.0f - cos_t);
            int is_spec = (m->specular * sp) > oracle_random(&seed);
            if (reflects || is_spec) {
                d = add3(specular, mul3s(sub3(diffuse, specular), m->specular_scatter));
                o = add3(h.p, mul3s(h.n, 0.0001f));
            } else {
                /* refract, :316-325 */
                v3 perp = mul3s(add3(d, mul3s(h.n, cos_t)), ior);
                float len = olength(perp);
                float len_sq = len * len;
                v3 par = mul3s(h.n, -sqrtf(fabsf(1.0f - len_sq)));
                v3 refr = add3(perp, par);
                d = add3(refr, mul3s(sub3(diffuse, refr), m->roughness / 10.0f));
                o = sub3(h.p, mul3s(h.n, 0.0001f));
                contrib.x = contrib.x * color.x; contrib.y = contrib.y * color.y;
                contrib.z = contrib.z * color.z; contrib.w = contrib.w * color.w;
            }
        } else {
            int is_spec = m->specular > oracle_random(&seed);
            if (is_spec) {
                d = add3(specular, mul3s(sub3(diffuse, specular), m->specular_scatter));
            } else {
                d = add3(specular, mul3s(sub3(diffuse, specular), m->roughness));
                contrib.x = contrib.x * color.x; contrib.y = contrib.y * color.y;
                contrib.z = contrib.z * color.z; contrib.w = contrib.w * color.w;
            }
            o = add3(h.p, mul3s(h.n, 0.0001f));
        }
    }
    return light;
}

/* pack_to_u32, :192-208 */
uint32_t oracle_pack(const float* c) {
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        float x = c[i] * 255.0f;
        uint32_t b = (uint32_t)x & 0xffu;
        r |= b << (8 * i);
    }
    return r;
}

static inline float oclamp01(float x) { return ofminf(ofmaxf(x, 0.0f), 1.0f); }

/* main, :146-189, for one pixel. */
static uint64_t shade_pixel(const OScene* s, const OParams* pr, uint32_t index, uint32_t bounces, float* acc4,
                            uint32_t* out1) {
    uint64_t rays = 0;
    uint32_t random_index = pr->accumulation_index;
    float rc[4];
    if (pr->accumulate == 1) {
        v4 px = {acc4[0], acc4[1], acc4[2], acc4[3]};
        for (uint32_t i = 0; i < pr->compute_per_frame; i++) {
            v4 l = per_pixel(s, pr, index, bounces, random_index, &rays);
            px.x = px.x + l.x; px.y = px.y + l.y; px.z = px.z + l.z; px.w = px.w + l.w;
            random_index = random_index + 1u;
        }
        acc4[0] = px.x; acc4[1] = px.y; acc4[2] = px.z; acc4[3] = px.w;
        float div = (float)(pr->accumulation_index * pr->compute_per_frame);
        rc[0] = oclamp01(px.x / div); rc[1] = oclamp01(px.y / div);
        rc[2] = oclamp01(px.z / div); rc[3] = oclamp01(px.w / div);
    } else {
        v4 l = per_pixel(s, pr, index, bounces, random_index, &rays);
        rc[0] = oclamp01(l.x); rc[1] = oclamp01(l.y); rc[2] = oclamp01(l.z); rc[3] = oclamp01(l.w);
    }
    *out1 = oracle_pack(rc);
    return rays;
}

/* One dispatch over the pixels of `height` rows owned by `rank` of `world`
 * (8x8 tile t -> rank t % world). accum/out are full row-major framebuffers.
 * Returns the number of counted ray segments. */
uint64_t oracle_render_frame(const OScene* s, const OParams* pr, uint32_t height, uint32_t bounces, uint32_t rank,
                             uint32_t world, float* accum, uint32_t* out, int n_threads) {
    ensure_srgb();
    uint32_t w = pr->screen_width;
    uint32_t tiles_x = (w + TILE - 1) / TILE, tiles_y = (height + TILE - 1) / TILE;
    int64_t n_tiles = (int64_t)tiles_x * tiles_y;
    uint64_t total = 0;
    if (world == 0) world = 1;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : total) num_threads(n_threads)
#endif
    for (int64_t t = 0; t < n_tiles; t++) {
        if ((uint64_t)t % world != rank) continue;
        uint32_t tx = (uint32_t)(t % tiles_x), ty = (uint32_t)(t / tiles_x);
        for (uint32_t yy = 0; yy < TILE; yy++) {
            uint32_t y = ty * TILE + yy;
            if (y >= height) break;
            for (uint32_t xx = 0; xx < TILE; xx++) {
                uint32_t x = tx * TILE + xx;
                if (x >= w) break;
                uint32_t idx = y * w + x;
                total += shade_pixel(s, pr, idx, bounces, accum + 4 * (size_t)idx, out + idx);
            }
        }
    }
    (void)n_threads;
    return total;
}

/* Shade an explicit list of pixel indices (for sampled parity checks at full
 * resolution). accum_io/out are indexed by position in the list, not by pixel
 * index: accum_io[4*i..] holds the accumulation of pixels[i] on entry. */
uint64_t oracle_render_pixels(const OScene* s, const OParams* pr, uint32_t bounces, const uint32_t* pixels,
                              uint64_t n, float* accum_io, uint32_t* out, int n_threads) {
    ensure_srgb();
    uint64_t total = 0;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total) num_threads(n_threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; i++) {
        uint32_t idx = pixels[i];
        float acc[4] = {accum_io[4 * i], accum_io[4 * i + 1], accum_io[4 * i + 2], accum_io[4 * i + 3]};
        uint32_t o1;
        total += shade_pixel(s, pr, idx, bounces, acc, &o1);
        accum_io[4 * i] = acc[0]; accum_io[4 * i + 1] = acc[1]; accum_io[4 * i + 2] = acc[2];
        accum_io[4 * i + 3] = acc[3];
        out[i] = o1;
    }
    (void)n_threads;
    return total;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
