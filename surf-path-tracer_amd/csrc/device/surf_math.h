/*
 * surf_math.h -- arithmetic shared by the HIP kernels (and compiled for the host
 * so CPU tests can check it against glibc).
 *
 * Bit-exactness rules, all required for the GPU to reproduce the CPU
 * reference's float stream (surf_math.h/.cpp of the reference):
 *   - built with -ffp-contract=off (no FMA contraction of a*b+c);
 *   - f32 division and sqrt correctly rounded (hipcc default on gfx950);
 *   - min/max are the reference's ternaries (NaN semantics differ from fminf);
 *   - operation order follows the reference expression by expression;
 *   - sinf/cosf/expf are restatements of glibc 2.35's x86-64 FMA variants
 *     (ARM optimized-routines algorithms, evaluated in f64 with explicit fma),
 *     verified bit-exact against glibc for every float in [0, 6.3] (sin/cos)
 *     and [-110, 0] (exp) -- tools/verify_libm.c.
 */
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define SURF_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define SURF_HD static inline
#endif

namespace surfdev {

constexpr float kFarAway = 1e30f;
constexpr float kEps = 1e-5f;
constexpr float kInvPi = 0.31830988618379067153777f;
constexpr float k2Pi = 6.28318530717958647692528f;

struct V3 { float x, y, z; };

SURF_HD V3 mk3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
SURF_HD V3 add(V3 a, V3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
SURF_HD V3 sub(V3 a, V3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
SURF_HD V3 mul(V3 a, V3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
SURF_HD V3 scl(V3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }      /* Float3 * F32 */
SURF_HD V3 lscl(float s, V3 a) { return mk3(s * a.x, s * a.y, s * a.z); }     /* F32 * Float3 */
SURF_HD V3 divs(V3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
SURF_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
SURF_HD V3 cross(V3 a, V3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
SURF_HD V3 normalize(V3 a) { float inv = 1.0f / sqrtf(dot(a, a)); return scl(a, inv); }
SURF_HD float tmin(float a, float b) { return a < b ? a : b; }
SURF_HD float tmax(float a, float b) { return a > b ? a : b; }

/* ---- RNG, surf_math.cpp:31-95 ---- */
SURF_HD uint32_t wangHash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
SURF_HD uint32_t initSeed(uint32_t s) { return wangHash((s + 1u) * 0x11u); }
SURF_HD uint32_t rndU(uint32_t& s) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
SURF_HD float rndF(uint32_t& s) { return (float)rndU(s) * 2.3283064365387e-10f; }
SURF_HD float rndRange(uint32_t& s, float lo, float hi) { float r = hi - lo; return (rndF(s) * r) + lo; }
SURF_HD uint32_t rndRangeU(uint32_t& s, uint32_t lo, uint32_t hi) { return (rndU(s) + lo) % hi; }

/* ---- bit casts (memcpy lowers to a register move on both sides) ---- */
SURF_HD uint32_t f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
SURF_HD float u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
SURF_HD uint64_t d2u(double d) { uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
SURF_HD double u2d(uint64_t u) { double d; __builtin_memcpy(&d, &u, 8); return d; }
SURF_HD double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* ---- glibc 2.35 sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c, sincosf.h;
 *      x86-64 FMA ifunc variant).  Valid for |y| < 120 (the path tracer calls
 *      them with theta = 2*pi*r1 in [0, 2*pi]); larger inputs fall back to the
 *      f64 library call (not bit-exact, never reached by the renderer). ---- */
/* constants of __sincosf_table[0] (sincosf_data.c, !TOINT_INTRINSICS form);
 * table[1] negates c0..c4 and keeps s1..s3, selected here by `neg`. */
SURF_HD uint32_t absTop12(float x) { return (f2u(x) >> 20) & 0x7ff; }
SURF_HD float sincosPoly(double x, double x2, bool neg, int n) {
    if ((n & 1) == 0) {
        const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7, s3c = -0x1.994eb3774cf24p-13;
        double x3 = x * x2;
        double s1 = fmad(x2, s3c, s2c);
        double x7 = x3 * x2;
        double s = fmad(x3, s1c, x);
        return (float)fmad(x7, s1, s);
    }
    const double c0 = neg ? -0x1p0 : 0x1p0;
    const double c1c = neg ? 0x1.ffffffd0c621cp-2 : -0x1.ffffffd0c621cp-2;
    const double c2c = neg ? -0x1.55553e1068f19p-5 : 0x1.55553e1068f19p-5;
    const double c3c = neg ? 0x1.6c087e89a359dp-10 : -0x1.6c087e89a359dp-10;
    const double c4c = neg ? -0x1.99343027bf8c3p-16 : 0x1.99343027bf8c3p-16;
    double x4 = x2 * x2;
    double c2 = fmad(x2, c4c, c3c);
    double c1 = fmad(x2, c1c, c0);
    double x6 = x4 * x2;
    double c = fmad(x4, c2c, c1);
    return (float)fmad(x6, c2, c);
}
SURF_HD float glibcSinCos(float y, int cosine) {
    const uint32_t top = absTop12(y);
    double x = (double)y;
    if (top < absTop12(0x1.921fb6p-1f)) {                    /* |y| < pi/4 */
        if (top < absTop12(0x1p-12f)) return cosine ? 1.0f : y;
        return sincosPoly(x, x * x, false, cosine);
    }
    if (top < absTop12(120.0f)) {
        const double hpiInv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
        double r = x * hpiInv;
        int n = (((int32_t)r) + 0x800000) >> 24;
        x = fmad(-(double)n, hpi, x);
        const int q = n & 3;
        const double s = (q == 1 || q == 2) ? -1.0 : 1.0;    /* sign[] = {1,-1,-1,1} */
        return sincosPoly(x * s, x * x, (n & 2) != 0, cosine ? (n ^ 1) : n);
    }
    return cosine ? (float)cos((double)y) : (float)sin((double)y);
}
SURF_HD float gSinf(float y) { return glibcSinCos(y, 0); }
SURF_HD float gCosf(float y) { return glibcSinCos(y, 1); }
/* sinf(y) and cosf(y) with one shared range reduction (glibc's s_sincosf.c
 * uses the same reduction and polynomials as s_sinf.c / s_cosf.c, so both
 * results are bit-identical to the separate calls); the cosine polynomial is
 * finished before the sine one starts, which keeps the f64 temporaries of the
 * two from being live at once. */
SURF_HD void gSinCosf(float y, float& sn, float& cs) {
    const uint32_t top = absTop12(y);
    double x = (double)y;
    if (top < absTop12(0x1.921fb6p-1f)) {                    /* |y| < pi/4 */
        if (top < absTop12(0x1p-12f)) { sn = y; cs = 1.0f; return; }
        const double x2 = x * x;
        cs = sincosPoly(x, x2, false, 1);
        sn = sincosPoly(x, x2, false, 0);
        return;
    }
    if (top < absTop12(120.0f)) {
        const double hpiInv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
        double r = x * hpiInv;
        int n = (((int32_t)r) + 0x800000) >> 24;
        x = fmad(-(double)n, hpi, x);
        const int q = n & 3;
        const double sg = (q == 1 || q == 2) ? -1.0 : 1.0;   /* sign[] = {1,-1,-1,1} */
        const bool neg = (n & 2) != 0;
        const double xs = x * sg, x2 = x * x;
        cs = sincosPoly(xs, x2, neg, n ^ 1);
        sn = sincosPoly(xs, x2, neg, n);
        return;
    }
    sn = (float)sin((double)y);
    cs = (float)cos((double)y);
}

/* ---- glibc 2.35 expf (e_expf.c + e_exp2f_data.c, N = 32, FMA variant) ---- */
SURF_HD float gExpf(float x) {
    const uint32_t top = absTop12(x);
    if (top >= absTop12(88.0f)) {
        const uint32_t ux = f2u(x);
        if (ux == 0xff800000u) return 0.0f;                  /* -inf */
        if (top >= absTop12(__builtin_inff())) return x + x; /* nan / +inf */
        if (x > 0x1.62e42ep6f) return __builtin_inff();
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    const uint64_t tab[32] = {
        0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
        0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
        0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
        0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
        0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
        0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
        0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
        0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
    const double N = 32.0;
    const double invLn2N = 0x1.71547652b82fep+0 * N;
    const double shift = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-5 / N / N / N, C1 = 0x1.ebfce50fac4f3p-3 / N / N, C2 = 0x1.62e42ff0c52d6p-1 / N;
    const double xd = (double)x;
    double kd = fmad(invLn2N, xd, shift);
    const uint64_t ki = d2u(kd);
    kd -= shift;
    const double r = fmad(invLn2N, xd, -kd);
    uint64_t t = tab[ki % 32];
    t += ki << (52 - 5);
    const double s = u2d(t);
    const double z = fmad(C0, r, C1);
    const double r2 = r * r;
    double y = fmad(C2, r, 1.0);
    y = fmad(z, r2, y);
    y = y * s;
    return (float)y;
}

/* ---- AABB slab test, bvh.cpp:40-66 (rd = 1/d precomputed: same values) ---- */
SURF_HD float slab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                   V3 o, V3 rd, float depth) {
    float tx0 = (mnx - o.x) * rd.x, tx1 = (mxx - o.x) * rd.x;
    float t0 = tmin(tx0, tx1), t1 = tmax(tx0, tx1);
    float ty0 = (mny - o.y) * rd.y, ty1 = (mxy - o.y) * rd.y;
    t0 = tmax(t0, tmin(ty0, ty1));
    t1 = tmin(t1, tmax(ty0, ty1));
    float tz0 = (mnz - o.z) * rd.z, tz1 = (mxz - o.z) * rd.z;
    t0 = tmax(t0, tmin(tz0, tz1));
    t1 = tmin(t1, tmax(tz0, tz1));
    return (t1 >= t0 && t0 < depth && t1 > 0.0f) ? t0 : kFarAway;
}

/* Same value as slab() (up to the sign of a zero, which only ever meets
 * comparisons) when no NaN can arise: o, rd and the box finite.  Then every
 * (b - o) * rd is finite or +-inf, never 0 * inf, so the ternary min/max of
 * the reference equal IEEE min/max and fold to v_min3/v_max3. */
SURF_HD float slabFinite(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                         V3 o, V3 rd, float depth) {
    const float tx0 = (mnx - o.x) * rd.x, tx1 = (mxx - o.x) * rd.x;
    const float ty0 = (mny - o.y) * rd.y, ty1 = (mxy - o.y) * rd.y;
    const float tz0 = (mnz - o.z) * rd.z, tz1 = (mxz - o.z) * rd.z;
    const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
    const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return (t1 >= t0 && t0 < depth && t1 > 0.0f) ? t0 : kFarAway;
}

SURF_HD bool finite3(V3 v) { return fabsf(v.x) <= 3.40282347e38f && fabsf(v.y) <= 3.40282347e38f && fabsf(v.z) <= 3.40282347e38f; }

/* ---- Moller-Trumbore, mesh.cpp:23-62, with e1 = v1-v0, e2 = v2-v0 precomputed
 *      (the same f32 subtraction the reference performs per test). ---- */
SURF_HD bool triHit(V3 v0, V3 e1, V3 e2, V3 o, V3 d, float& depth, float& hu, float& hv) {
    V3 h = cross(d, e2);
    float a = dot(e1, h);
    if (fabsf(a) < kEps) return false;
    float f = 1.0f / a;
    V3 s = sub(o, v0);
    float u = f * dot(s, h);
    if (0.0f > u || u > 1.0f) return false;
    V3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (0.0f > v || (u + v) > 1.0f) return false;
    float t = f * dot(e2, q);
    if (!(kEps <= t && t < depth)) return false;
    depth = t; hu = u; hv = v;
    return true;
}

/* triHit without early exits, for lanes that each test a different triangle
 * (the leaf of a wave walk): the same operations and the same four rejection
 * tests (each negated as written, so NaN operands reject exactly where
 * triHit's branches do), combined with bitwise ands so no lane mask is saved
 * and restored per test.  t, u, v are meaningful only when it returns true;
 * depth is not updated (the caller accepts hits in triangle order). */
SURF_HD bool triHitFlat(V3 v0, V3 e1, V3 e2, V3 o, V3 d, float depth, float& t, float& hu, float& hv) {
    const V3 h = cross(d, e2);
    const float a = dot(e1, h);
    const float f = 1.0f / a;
    const V3 s = sub(o, v0);
    const float u = f * dot(s, h);
    const V3 q = cross(s, e1);
    const float v = f * dot(d, q);
    t = f * dot(e2, q);
    hu = u; hv = v;
    const bool k0 = !(fabsf(a) < kEps);
    const bool k1 = !((0.0f > u) | (u > 1.0f));
    const bool k2 = !((0.0f > v) | ((u + v) > 1.0f));
    const bool k3 = (kEps <= t) & (t < depth);
    return k0 & k1 & k2 & k3;
}

/* ---- glm mat4 * vec4, pairwise column sums (type_mat4x4.inl) ---- */
SURF_HD float mrow(const float* m, int i, float x, float y, float z, float w) {
    float a = m[0 + i] * x + m[4 + i] * y;
    float b = m[8 + i] * z + m[12 + i] * w;
    return a + b;
}

}  // namespace surfdev
