// pt_math.h — bit-exact arithmetic of the reference trace loop, for gfx950 and host.
//
// Everything here must produce the same bits as the reference compiled with
// g++ -O3 for x86-64 (no FMA): the translation units that include this header
// are built with -ffp-contract=off and IEEE division/sqrt (see Makefile).
//
// Reference semantics reproduced (file:line into the reference tree):
//   LCG                       rng.h:14-20   state' = 1664525*state + 1013904223 mod 2^32,
//                                           rand01 = (float)state / 2^32 (can be 1.0f)
//   std::min/std::max         aabb.h:24-25  (b<a)?b:a / (a<b)?b:a, and min_element /
//                                           max_element scan order for the 3-way forms,
//                                           so NaN behaves as in the reference
//   |a| < EPS                 triangle.h:31 EPS = 1e-6 is a double; for float |a| the
//                                           compare is exactly |a| < 0x1.0c6f7cp-20f
//   acosf                     glibc 2.35 e_acosf.c (fdlibm), float arithmetic
//   sincosf                   glibc 2.35 s_sincosf.c (double polynomial)
// Both libm restatements equal the host glibc on every input of the path's
// domain (tests/test_math.py); on the GPU they are checked against the oracle.
#pragma once

#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#endif

#if defined(__HIPCC__)
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD inline
#endif

namespace pt {

// ------------------------------------------------------------------ bits
PT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
PT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// ------------------------------------------------------------------ vec3
struct v3 {
    float x, y, z;
};
PT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
PT_HD v3 add(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_HD v3 sub(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_HD v3 mul(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_HD v3 scale(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
PT_HD v3 neg(v3 a) { return v3{-a.x, -a.y, -a.z}; }
PT_HD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD v3 cross(v3 a, v3 b) {
    return v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// ------------------------------------------------------------------ exact rcp / sqrt
// Correctly rounded 1/a and sqrt(x) in fewer instructions than the IEEE division and
// square-root expansions (12 and 15 VALU ops on gfx950). The fast sequences are exact
// on a range of inputs, established by sweeping EVERY float of that range on the GPU
// (pt_debug_sweep; tests/test_gpu_parity.py::test_fast_exact_math_sweep re-checks all
// 2^32 inputs of the guarded functions on each GPU run); outside it the IEEE operation
// runs (a branch no lane of a wave normally takes).
//   rcp:  v_rcp_f32, then one Newton step with FMA; exact for |a| in [2^-126, 2^126]
//   sqrt: v_sqrt_f32, then the +-1 ulp residual fix-up; exact for x in [2^-100, 2^100]
// On the host (oracle, CPU builds) they are the IEEE operations themselves.
PT_HD float rcp_exact(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float m = __builtin_fabsf(a);
    if (__builtin_expect(!(m >= 0x1p-126f && m <= 0x1p126f), 0)) return 1.0f / a;
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = __builtin_fmaf(-a, r, 1.0f);
    return __builtin_fmaf(e, r, r);
#else
    return 1.0f / a;
#endif
}

PT_HD float sqrt_exact(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_expect(!(x >= 0x1p-100f && x <= 0x1p100f), 0)) return __builtin_sqrtf(x);
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) - 1u);
    const float su = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    float r = rd <= 0.0f ? sd : s;
    r = ru > 0.0f ? su : r;
    return r;
#else
    return __builtin_sqrtf(x);
#endif
}

// vec3::normalize = *this / length(): three correctly rounded divisions.
PT_HD v3 normalize(v3 a) {
    float len = sqrt_exact(dot(a, a));
    return v3{a.x / len, a.y / len, a.z / len};
}

// a / b given y = RN(1/b) (rcp_exact): q0 = RN(a y), the exact remainder r = a - b q0
// (one FMA), then RN(q0 + r y). Markstein's theorem (P. Markstein, IBM J. Res. Dev. 34(1),
// 1990; Muller et al., Handbook of Floating-Point Arithmetic, §4.7): with y within half an
// ulp of 1/b and q0 within one ulp of a/b, that is the correctly rounded quotient, barring
// underflow / overflow of q0, r and the result — here ruled out by |a|, |b| in
// [2^-60, 2^60] (callers check) — and a = 0 (RN(q0 + r y) would lose the sign of -0).
// Checked on the GPU against IEEE division over 2^32 such pairs (pt_debug_sweep 4).
PT_HD float div_by_rcp(float a, float b, float y) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float q0 = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
#else
    (void)y;
    return a / b;
#endif
}

// vec3::normalize (linalg.h:149-151) with the three divisions by one reciprocal: exact
// when |len| and every nonzero |component| lie in [2^-60, 2^60] and no component is 0
// (div_by_rcp); otherwise the IEEE divisions. Same bits as normalize in every case.
PT_HD v3 normalize_fast(v3 a) {
    const float len = sqrt_exact(dot(a, a));
    const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    if (__builtin_expect(m >= 0x1p-60f && mx <= 0x1p60f && len >= 0x1p-60f && len <= 0x1p60f, 1)) {
        const float y = rcp_exact(len);
        return v3{div_by_rcp(a.x, len, y), div_by_rcp(a.y, len, y), div_by_rcp(a.z, len, y)};
    }
    return v3{a.x / len, a.y / len, a.z / len};
}

PT_HD float std_max(float a, float b) { return (a < b) ? b : a; }
PT_HD float std_min(float a, float b) { return (b < a) ? b : a; }
PT_HD float std_min3(float a, float b, float c) {
    float r = a;
    r = (b < r) ? b : r;
    r = (c < r) ? c : r;
    return r;
}
PT_HD float std_max3(float a, float b, float c) {
    float r = a;
    r = (r < b) ? b : r;
    r = (r < c) ? c : r;
    return r;
}

// ------------------------------------------------------------------ LCG
struct Lcg {
    uint32_t s;
    PT_HD float next01() {
        s = 1664525u * s + 1013904223u;
        return (float)s * 0x1p-32f;  // == (float)s / 2^32 exactly
    }
};

// ------------------------------------------------------------------ AABB slab (aabb.h:20-29)
PT_HD bool slab_hit(v3 lb, v3 rt, v3 o, v3 inv) {
    float t1x = (lb.x - o.x) * inv.x, t1y = (lb.y - o.y) * inv.y, t1z = (lb.z - o.z) * inv.z;
    float t2x = (rt.x - o.x) * inv.x, t2y = (rt.y - o.y) * inv.y, t2z = (rt.z - o.z) * inv.z;
    float tmax = std_min3(std_max(t1x, t2x), std_max(t1y, t2y), std_max(t1z, t2z));
    float tmin = std_max3(std_min(t1x, t2x), std_min(t1y, t2y), std_min(t1z, t2z));
    return !(tmax < 0) && (tmin <= tmax);
}

// Same result as slab_hit whenever inv has no infinite component. Then no slab value
// can be NaN (box and origin are finite, 0 * finite = 0), and without NaN the
// reference's compare-select min/max equal IEEE min/max up to the sign of a zero,
// which neither `tmax < 0` nor `tmin <= tmax` can observe. Lowers to v_min3/v_max3.
PT_HD bool slab_hit_finite(v3 lb, v3 rt, v3 o, v3 inv) {
    float t1x = (lb.x - o.x) * inv.x, t1y = (lb.y - o.y) * inv.y, t1z = (lb.z - o.z) * inv.z;
    float t2x = (rt.x - o.x) * inv.x, t2y = (rt.y - o.y) * inv.y, t2z = (rt.z - o.z) * inv.z;
    float tmax = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x, t2x), __builtin_fmaxf(t1y, t2y)),
                                 __builtin_fmaxf(t1z, t2z));
    float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x, t2x), __builtin_fminf(t1y, t2y)),
                                 __builtin_fminf(t1z, t2z));
    // !(tmax < 0) && tmin <= tmax  <=>  max(tmin, 0) <= tmax  (no NaN here)
    return __builtin_fmaxf(tmin, 0.0f) <= tmax;
}

PT_HD bool all_finite(v3 a) {
    return __builtin_fabsf(a.x) < __builtin_inff() && __builtin_fabsf(a.y) < __builtin_inff() &&
           __builtin_fabsf(a.z) < __builtin_inff();
}

// ------------------------------------------------------------------ Möller–Trumbore (triangle.h:25-44)
// e1 = v2 - v1 and e2 = v3 - v1 are precomputed on the host with the same float ops.
PT_HD bool tri_hit(v3 v1, v3 e1, v3 e2, v3 o, v3 d, float& t) {
    v3 h = cross(d, e2);
    float a = dot(e1, h);
    // (double)|a| < 1e-6  <=>  |a| <= 1e-6f (0x1.0c6f7ap-20)  <=>  |a| < 0x1.0c6f7cp-20f
    if (__builtin_fabsf(a) < 0x1.0c6f7cp-20f) return false;
    float f = rcp_exact(a);
    v3 s = sub(o, v1);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    v3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    t = f * dot(e2, q);
    return t > 0.0f;
}

// tri_hit with the same operations and the same result, for lanes that all run the whole
// test (the flat path's pair rounds: 64 different (ray, triangle) pairs, so no early exit
// is ever taken by a whole wave): no branches, and 1/a without the range guard. Requires
// |a| <= 2^126: a = e1 . (d x e2) with |d| ~ 1, so |a| < 2^124 whenever every vertex
// coordinate is below 2^60 in magnitude (the host checks before enabling it); |a| below
// the EPS threshold only clears `ok`. NaN behaves as in tri_hit: every rejection is a
// comparison that is false for NaN, so a NaN u or v passes through to `t > 0`.
PT_HD bool tri_hit_nb(v3 v1, v3 e1, v3 e2, v3 o, v3 d, float& t) {
    v3 h = cross(d, e2);
    float a = dot(e1, h);
    const bool ok = !(__builtin_fabsf(a) < 0x1.0c6f7cp-20f);
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_rcpf(a);
    const float f = __builtin_fmaf(__builtin_fmaf(-a, r, 1.0f), r, r);  // rcp_exact's fast branch
#else
    const float f = 1.0f / a;
#endif
    v3 s = sub(o, v1);
    float u = f * dot(s, h);
    v3 q = cross(s, e1);
    float v = f * dot(d, q);
    t = f * dot(e2, q);
    return ok && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) && t > 0.0f;
}

// ------------------------------------------------------------------ acosf (fdlibm)
// The restatement: glibc's float acosf (fdlibm e_acosf.c) as g++ compiles it for the
// reference (IEEE division and sqrt, no FMA).
PT_HD float acosf_ref(float x) {
    const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const float p0 = 1.6666667163e-01f, p1 = -3.2556581497e-01f, p2 = 2.0121252537e-01f,
                p3 = -4.0055535734e-02f, p4 = 7.9153501429e-04f, p5 = 3.4793309169e-05f;
    const float q1 = -2.4033949375e+00f, q2 = 2.0209457874e+00f, q3 = -6.8828397989e-01f,
                q4 = 7.7038154006e-02f;
    const uint32_t ux = f2u(x), ax = ux & 0x7fffffffu;
    if (ax >= 0x3f800000u) {
        if (ax == 0x3f800000u) return (ux >> 31) ? pi + 2.0f * pio2_lo : 0.0f;
        return (x - x) / (x - x);
    }
    if (ax < 0x3f000000u) {  // |x| < 0.5
        if (ax <= 0x32800000u) return pio2_hi + pio2_lo;
        float z = x * x;
        float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
        float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
        float r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (ux >> 31) {  // x <= -0.5
        float z = (1.0f + x) * 0.5f;
        float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
        float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
        float s = __builtin_sqrtf(z);
        float r = p / q;
        float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    // x >= 0.5
    float z = (1.0f - x) * 0.5f;
    float s = __builtin_sqrtf(z);
    float df = u2f(f2u(s) & 0xfffff000u);
    float c = (z - df * df) / (s + df);
    float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
    float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
    float r = p / q;
    float w = r * s + c;
    return 2.0f * (df + w);
}

// Device form: the three cases of acosf_ref as one instruction stream (every lane runs
// the polynomial, both divisions and the sqrt once; the case picks the result), each
// division as rcp_exact + one Markstein correction (div_by_rcp) and sqrt_exact. Not
// claimed for every (p, q) — but acosf_fast(x) == acosf_ref(x) for EVERY float x in
// [-1, 1], the whole domain the path reaches (argument 2u - 1, material.h:9), by
// exhaustive GPU sweep (pt_debug_sweep 2, tests/test_gpu_parity.py). Cases split over a
// wave otherwise cost the sum of the three branches.
PT_HD float acosf_fast(float x) {
    const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const float p0 = 1.6666667163e-01f, p1 = -3.2556581497e-01f, p2 = 2.0121252537e-01f,
                p3 = -4.0055535734e-02f, p4 = 7.9153501429e-04f, p5 = 3.4793309169e-05f;
    const float q1 = -2.4033949375e+00f, q2 = 2.0209457874e+00f, q3 = -6.8828397989e-01f,
                q4 = 7.7038154006e-02f;
    const uint32_t ux = f2u(x), ax = ux & 0x7fffffffu;
    if (__builtin_expect(ax >= 0x3f800000u || ax <= 0x32800000u, 0)) return acosf_ref(x);  // |x| >= 1, tiny
    const bool small = ax < 0x3f000000u;
    // 1 + x for x <= -0.5 and 1 - x for x >= 0.5 are both 1 - |x|
    const float z = small ? x * x : (1.0f - u2f(ax)) * 0.5f;
    const float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
    const float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
    const float r = div_by_rcp(p, q, rcp_exact(q));
    const float zs = small ? 0.25f : z;  // |x| < 0.5 uses neither s nor c
    const float s = sqrt_exact(zs);
    const float df = u2f(f2u(s) & 0xfffff000u);
    const float sd = s + df;
    const float c = div_by_rcp(zs - df * df, sd, rcp_exact(sd));
    const float v_small = pio2_hi - (x - (pio2_lo - x * r));
    const float v_neg = pi - 2.0f * (s + (r * s - pio2_lo));
    const float v_pos = 2.0f * (df + (r * s + c));
    return small ? v_small : ((ux >> 31) ? v_neg : v_pos);
}

// ------------------------------------------------------------------ sincosf (double kernel)
// The restatement: glibc's sincosf (the double-precision polynomial kernel, no FMA as
// g++ compiles it for x86-64). Valid for |y| < 120 (top12 < 0x42F); the path only
// evaluates |y| <= 2*pi.
PT_HD void sincosf_ref(float y, float& sin_out, float& cos_out) {
    const uint32_t t12 = (f2u(y) >> 20) & 0x7ffu;
    double x = (double)y;
    int n = 0;
    double csign = 1.0;
    if (t12 < 0x3f4u) {  // |y| < pi/4
        if (t12 < 0x398u) {  // |y| < 2^-12
            sin_out = y;
            cos_out = 1.0f;
            return;
        }
    } else {
        double r = x * 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
        n = ((int32_t)r + 0x800000) >> 24;
        x = -(double)n * 0x1.921FB54442D18p0 + x;  // x - n * pi/2
        if ((n & 3) == 1 || (n & 3) == 2) x = -x;  // sign[n & 3] = {1,-1,-1,1}
        // sincos_poly is called with (x * s, x * x): x2 uses the unsigned x, same value.
        if (n & 2) csign = -1.0;
    }
    const double c0 = csign * 0x1p0, c1 = csign * -0x1.ffffffd0c621cp-2,
                 c2 = csign * 0x1.55553e1068f19p-5, c3 = csign * -0x1.6c087e89a359dp-10,
                 c4 = csign * 0x1.99343027bf8c3p-16;
    const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7, s3c = -0x1.994eb3774cf24p-13;
    double x2 = x * x;
    double x4 = x2 * x2, x3 = x2 * x;
    double cc2 = x2 * c4 + c3, ss1 = x2 * s3c + s2c;
    double cc1 = x2 * c1 + c0, x5 = x3 * x2, x6 = x4 * x2;
    double s = x3 * s1c + x, c = x4 * c2 + cc1;
    float sv = (float)(x5 * ss1 + s), cv = (float)(x6 * cc2 + c);
    if (n & 1) {
        sin_out = cv;
        cos_out = sv;
    } else {
        sin_out = sv;
        cos_out = cv;
    }
}

// Device form: one instruction stream for every |y| >= 2^-12 — the range reduction runs
// for |y| < pi/4 too, where it yields n = 0 and x unchanged, i.e. the unreduced case —
// with the double polynomial and the reduction FMA-contracted (glibc's own
// __sincosf_fma variant does the same on FMA hosts), and the cosine's sign applied to
// the result (rounding is symmetric, so the polynomial of the negated coefficients is
// the negated polynomial; the cosine term is never 0 here). sincosf_fast ==
// sincosf_ref for EVERY float in [-2, 7] (theta in [-pi/2, pi/2], phi in [0, 2*pi]),
// by exhaustive GPU sweep (pt_debug_sweep 3).
PT_HD void sincosf_fast(float y, float& sin_out, float& cos_out) {
    const uint32_t t12 = (f2u(y) >> 20) & 0x7ffu;
    const double y0 = (double)y;
    const double rr = y0 * 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
    const int n = ((int32_t)rr + 0x800000) >> 24;
    double x = __builtin_fma(-(double)n, 0x1.921FB54442D18p0, y0);
    if ((n & 3) == 1 || (n & 3) == 2) x = -x;
    const double c0 = 0x1p0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16;
    const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7, s3c = -0x1.994eb3774cf24p-13;
    const double x2 = x * x;
    const double x4 = x2 * x2, x3 = x2 * x;
    const double cc2 = __builtin_fma(x2, c4, c3), ss1 = __builtin_fma(x2, s3c, s2c);
    const double cc1 = __builtin_fma(x2, c1, c0), x5 = x3 * x2, x6 = x4 * x2;
    const double s = __builtin_fma(x3, s1c, x), c = __builtin_fma(x4, c2, cc1);
    const float sv = (float)__builtin_fma(x5, ss1, s);
    float cv = (float)__builtin_fma(x6, cc2, c);
    if (n & 2) cv = -cv;
    const bool swap = (n & 1) != 0, tiny = t12 < 0x398u;  // |y| < 2^-12: (y, 1)
    sin_out = tiny ? y : (swap ? cv : sv);
    cos_out = tiny ? 1.0f : (swap ? sv : cv);
}

// What the path calls: the fast forms on the device, the restatements on the host.
#if defined(__HIP_DEVICE_COMPILE__)
constexpr bool kFastLibm = true;
#else
constexpr bool kFastLibm = false;
#endif
PT_HD float acosf_path(float x) { return kFastLibm ? acosf_fast(x) : acosf_ref(x); }
PT_HD void sincosf_path(float y, float& s, float& c) {
    if (kFastLibm) sincosf_fast(y, s, c);
    else sincosf_ref(y, s, c);
}

// ------------------------------------------------------------------ BRDF (material.h:6-25)
// hemisphere_sample: u first, then v (separate declarators are sequenced).
PT_HD v3 hemisphere_dir(Lcg& g, v3 n) {
    float u = g.next01();
    float v = g.next01();
#ifdef PT_EXP_CHEAP_LIBM  // timing experiment only (wrong images): hardware approximations
    float theta = (float)((double)acosf(2.0f * u - 1.0f) - 1.57079632679489661923);
    float phi = (float)(6.28318530717958647692 * (double)v);
    float st = __sinf(theta), ct = __cosf(theta), sp = __sinf(phi), cp = __cosf(phi);
#else
    float theta = (float)((double)acosf_path(2.0f * u - 1.0f) - 1.57079632679489661923);  // - M_PI_2
    float phi = (float)(6.28318530717958647692 * (double)v);                                // 2 * M_PI * v
    float st, ct, sp, cp;
    sincosf_path(theta, st, ct);
    sincosf_path(phi, sp, cp);
#endif
    v3 smp = v3{ct * cp, ct * sp, st};
    return dot(smp, n) < 0.0f ? neg(smp) : smp;
}

// hemisphere_sample's theta part by table: theta = acosf(x) - M_PI_2 for x = 2u - 1, and
// its sine and cosine, depend on x alone, and x = fl(2u - 1) for every u the LCG yields
// (rand01 = (float)state / 2^32) lies on the grid k 2^-24 of [-1, 1] (all 2^32 states
// checked: tests/test_math.py), so (sin theta, cos theta) for all 2^25 + 1 grid values fit
// one table, built on the device by the same exact functions (pt_theta_table_kernel).
// Index of x in it: x 2^24 + 2^24 (both steps exact).
PT_HD int theta_index(float x) { return (int)(x * 0x1p24f) + (1 << 24); }
constexpr int kThetaEntries = (1 << 25) + 1;

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
// hemisphere_dir with (sin theta, cos theta) from the table: u, then v, as the reference
// draws them; phi's sincosf is computed. Same bits as hemisphere_dir.
__device__ __forceinline__ v3 hemisphere_dir_tab(Lcg& g, v3 n, const float2* __restrict__ tab) {
    float u = g.next01();
    float v = g.next01();
    const float2 sct = tab[theta_index(2.0f * u - 1.0f)];  // (sin theta, cos theta)
    float phi = (float)(6.28318530717958647692 * (double)v);  // 2 * M_PI * v
    float sp, cp;
    sincosf_path(phi, sp, cp);
    v3 smp = v3{sct.y * cp, sct.y * sp, sct.x};
    return dot(smp, n) < 0.0f ? neg(smp) : smp;
}
#endif

// specular_sample: vec3(rand01(), rand01(), rand01()) is evaluated right to left by
// g++, so the first draw is z. Returns false if the rejection loop hit `max_iter`.
PT_HD bool specular_dir(Lcg& g, v3 d, v3 n, float rough, int max_iter, v3& out) {
    v3 refl = sub(d, scale(n, 2.0f * dot(d, n)));
    v3 ret;
    int it = 0;
    do {
        float jz = g.next01();
        float jy = g.next01();
        float jx = g.next01();
        v3 j = v3{(jx - 0.5f) * rough, (jy - 0.5f) * rough, (jz - 0.5f) * rough};
        ret = add(refl, j);
        if (++it >= max_iter) {
            out = normalize(ret);
            return false;
        }
    } while (dot(ret, n) < 0.0f);
    out = normalize(ret);
    return true;
}

}  // namespace pt
