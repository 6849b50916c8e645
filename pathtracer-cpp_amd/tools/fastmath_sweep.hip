// Exploratory exhaustive sweep: candidate fast float sequences vs the IEEE-exact ones,
// over every float bit pattern in a range, on the GPU. Prints mismatch counts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "pt_math.h"
using namespace pt;

__device__ __forceinline__ float rcp_nr(float a) {
    float r = __builtin_amdgcn_rcpf(a);
    float e = __builtin_fmaf(-a, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp_nr2(float a) {  // NR then one residual correction
    float r = rcp_nr(a);
    float e = __builtin_fmaf(-a, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float sqrt_hw(float x) { return __builtin_amdgcn_sqrtf(x); }
// sqrt: hw estimate then residual-based +-1ulp fix (no scaling)
__device__ __forceinline__ float sqrt_fix(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    float sd = __uint_as_float(__float_as_uint(s) - 1), su = __uint_as_float(__float_as_uint(s) + 1);
    float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    s = rd <= 0.0f ? sd : s;
    s = ru > 0.0f ? su : s;
    return s;
}

// glibc sincosf kernel with FMA contraction in the double polynomial
__device__ __forceinline__ void sincos_fma(float y, float& sin_out, float& cos_out) {
    const uint32_t t12 = (f2u(y) >> 20) & 0x7ffu;
    double x = (double)y;
    int n = 0;
    double csign = 1.0;
    if (t12 < 0x3f4u) {
        if (t12 < 0x398u) { sin_out = y; cos_out = 1.0f; return; }
    } else {
        double r = x * 0x1.45F306DC9C883p+23;
        n = ((int32_t)r + 0x800000) >> 24;
        x = MODE_RR ? __builtin_fma(-(double)n, 0x1.921FB54442D18p0, x) : x - (double)n * 0x1.921FB54442D18p0;
        if ((n & 3) == 1 || (n & 3) == 2) x = -x;
        if (n & 2) csign = -1.0;
    }
    const double c0 = csign * 0x1p0, c1 = csign * -0x1.ffffffd0c621cp-2,
                 c2 = csign * 0x1.55553e1068f19p-5, c3 = csign * -0x1.6c087e89a359dp-10,
                 c4 = csign * 0x1.99343027bf8c3p-16;
    const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7, s3c = -0x1.994eb3774cf24p-13;
    double x2 = x * x;
    double x4 = x2 * x2, x3 = x2 * x;
    double cc2 = __builtin_fma(x2, c4, c3), ss1 = __builtin_fma(x2, s3c, s2c);
    double cc1 = __builtin_fma(x2, c1, c0), x5 = x3 * x2, x6 = x4 * x2;
    double s = __builtin_fma(x3, s1c, x), c = __builtin_fma(x4, c2, cc1);
    float sv = (float)__builtin_fma(x5, ss1, s), cv = (float)__builtin_fma(x6, cc2, c);
    if (n & 1) { sin_out = cv; cos_out = sv; } else { sin_out = sv; cos_out = cv; }
}
#ifndef MODE_RR
#define MODE_RR 0
#endif

// fdlibm acosf with p/q as p * rcp(q) + one Markstein correction, sqrt via sqrt_exact
__device__ __forceinline__ float div_mk(float p, float q) {
    const float y = rcp_exact(q);
    const float q0 = p * y;
    const float rem = __builtin_fmaf(-q, q0, p);
    return __builtin_fmaf(rem, y, q0);
}
__device__ __forceinline__ float div_rcp(float p, float q) { return p * rcp_exact(q); }
template <int V>
__device__ __forceinline__ float acosf_v(float x) {
    auto DIV = [](float a, float b) { return V == 0 ? a / b : V == 1 ? div_mk(a, b) : div_rcp(a, b); };
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
    if (ax < 0x3f000000u) {
        if (ax <= 0x32800000u) return pio2_hi + pio2_lo;
        float z = x * x;
        float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
        float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
        float r = DIV(p, q);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (ux >> 31) {
        float z = (1.0f + x) * 0.5f;
        float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
        float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
        float s = sqrt_exact(z);
        float r = DIV(p, q);
        float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    float z = (1.0f - x) * 0.5f;
    float s = sqrt_exact(z);
    float df = u2f(f2u(s) & 0xfffff000u);
    float c = DIV(z - df * df, s + df);
    float p = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
    float q = 1.0f + z * (q1 + z * (q2 + z * (q3 + z * q4)));
    float r = DIV(p, q);
    float w = r * s + c;
    return 2.0f * (df + w);
}

__global__ void sweep(int which, uint32_t lo, uint64_t n, unsigned long long* bad, uint32_t* first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long nb = 0;
    for (; i < n; i += stride) {
        const uint32_t bits = lo + (uint32_t)i;
        const float x = __uint_as_float(bits);
        if (x != x) continue;
        float got, want;
        switch (which) {
            case 0: got = __builtin_amdgcn_rcpf(x); want = 1.0f / x; break;
            case 1: got = rcp_nr(x); want = 1.0f / x; break;
            case 2: got = rcp_nr2(x); want = 1.0f / x; break;
            case 3: got = sqrt_hw(x); want = __builtin_sqrtf(x); break;
            case 4: got = sqrt_fix(x); want = __builtin_sqrtf(x); break;
            case 5: got = acosf_v<1>(x); want = acosf_ref(x); break;
            case 6: got = acosf_v<2>(x); want = acosf_ref(x); break;
            case 7: { float a, b, c2, d2; sincos_fma(x, a, b); sincosf_ref(x, c2, d2);
                      got = a; want = c2; if (__float_as_uint(b) != __float_as_uint(d2)) { got = 1; want = 2; } } break;
            case 8: got = acosf_v<0>(x); want = acosf_ref(x); break;
            default: got = want = 0; break;
        }
        if (__float_as_uint(got) != __float_as_uint(want)) {
            nb++;
            atomicMin(first, bits);
        }
    }
    if (nb) atomicAdd(bad, nb);
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 4);
    struct R { int which; const char* name; uint32_t lo, hi; };
    const R runs[] = {
        {0, "rcp_hw  all positive", 0x00000000u, 0x7f800000u},
        {1, "rcp_nr  all positive", 0x00000000u, 0x7f800000u},
        {1, "rcp_nr  [2^-126, 2^126]", 0x00800000u, 0x7e800000u},
        {1, "rcp_nr  [1e-6, 2^100]", 0x358637bdu, 0x71800000u},
        {2, "rcp_nr2 all positive", 0x00000000u, 0x7f800000u},
        {2, "rcp_nr2 [2^-126, 2^126]", 0x00800000u, 0x7e800000u},
        {3, "sqrt_hw all positive", 0x00000000u, 0x7f800000u},
        {3, "sqrt_hw [2^-100, 2^100]", 0x0d800000u, 0x71800000u},
        {4, "sqrt_fix all positive", 0x00000000u, 0x7f800000u},
        {4, "sqrt_fix [2^-100, 2^100]", 0x0d800000u, 0x71800000u},
        {8, "acosf sqrt_exact [0,1]", 0x00000000u, 0x3f800000u},
        {8, "acosf sqrt_exact [-1,0]", 0x80000000u, 0xbf800000u},
        {5, "acosf markstein [0,1]", 0x00000000u, 0x3f800000u},
        {5, "acosf markstein [-1,0]", 0x80000000u, 0xbf800000u},
        {6, "acosf p*rcp(q) [0,1]", 0x00000000u, 0x3f800000u},
        {6, "acosf p*rcp(q) [-1,0]", 0x80000000u, 0xbf800000u},
        {7, "sincos fma [0,7]", 0x00000000u, 0x40e00000u},
        {7, "sincos fma [-2,0]", 0x80000000u, 0xc0000000u},
    };
    for (const R& r : runs) {
        hipMemset(bad, 0, 8);
        hipMemset(first, 0xff, 4);
        hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0, r.which, r.lo, (uint64_t)(r.hi - r.lo) + 1, bad, first);
        unsigned long long hb; uint32_t hf;
        hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
        printf("%-28s mismatches %llu  first 0x%08x (%a)\n", r.name, hb, hf, (double)__builtin_bit_cast(float, hf));
    }
    return 0;
}
