// valu_ubench — issue cost of the VALU forms the trace kernels choose between (gfx950).
//
// Each kernel runs kIters iterations of 8 independent dependency chains of one
// instruction form (inline asm, so the compiler cannot fuse or reorder them), on a
// full grid (many waves per SIMD), and reports the wall time per wave-instruction
// per SIMD, i.e. the throughput cost the trace kernels pay:
//   fma       v_fma_f32
//   pk_fma    v_pk_fma_f32           (2 lanes of f32 per instruction)
//   pk_mul    v_pk_mul_f32
//   fma_mix   v_fma_mix_f32 (f16 multiplicand from a register half, f32 addend)
//   cvt_ub    v_cvt_f32_ubyte0
//   fma_f64   v_fma_f64
//   rcp       v_rcp_f32
//   addc      v_addc_co_u32 (VOP3, SGPR carry-in)
//   max3      v_max3_f32
//   add       v_add_f32 (VOP2)
//   mov       v_mov_b32 (VOP1)
//   and       v_and_b32 (VOP2, integer)
//   cndmask   v_cndmask_b32 (VOP2, VCC select)
//   cmp       v_cmp_lt_f32 (VOPC, writes VCC)
//   fma_lo32  v_fma_f32 with EXEC = lanes 0..31 (one 32-lane half of the wave)
//   fma_1     v_fma_f32 with EXEC = lane 0
//   fma_even  v_fma_f32 with EXEC = the even lanes (both halves partly active)
//   fmac, mul, mul_neg (VOP3 for the modifier), min, cndmask_vcc (VOP2), cndmask_sgpr (VOP3),
//   add_u32, lshl, cmp_sgpr (VOP3 compare to an SGPR pair), sub, add_abs (VOP3), mov_dpp,
//   fma+add / mul+add / max3+min (two forms alternating), fma_2lanes / fma_4 / fma_16 (EXEC)
//   mul_lo_u32, mad_u24, mul_u24, lshl_add, cvt_f32_u32, or_sdwa (SDWA word select), perm,
//   mul_f64, cvt_f64_f32, max3+mul / fma_mix+mul (a main-port form beside a second-port one)
// SQ_ACTIVE_INST_VALU2 (rocprofv3) counts the instructions issued on the SIMD's second VALU
// port: a form that appears there can dual-issue beside a main-port instruction.
// usage: valu_ubench [waves_per_simd] [op ...]   (ops by name; default all)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

constexpr int kIters = 4096;

#define CHAIN8(INSN)       \
    INSN(a0) INSN(a1) INSN(a2) INSN(a3) INSN(a4) INSN(a5) INSN(a6) INSN(a7)

template <int kOp>
__global__ void __launch_bounds__(256) ubench(float* out, float s) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = p0, p5 = p1, p6 = p2, p7 = p3;
    const f2 ps = {s, s};
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    uint32_t u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6,
             u7 = u0 + 7;
    const unsigned long long carry = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    const uint32_t h = 0x3c003c00u;  // (1.0h, 1.0h)
    const int lane = threadIdx.x & 63;
    const bool on = kOp == 14 ? lane < 32 : kOp == 15 ? lane == 0 : kOp == 16 ? (lane & 1) == 0
                    : kOp == 32 ? (lane & 31) == 0 : kOp == 33 ? lane < 4 : kOp == 34 ? lane < 16 : true;
    if constexpr (kOp == 21) asm volatile("v_cmp_gt_u32 vcc, 32, %0" : : "v"(lane) : "vcc");
    if (on)
    for (int i = 0; i < kIters; i++) {
        if constexpr (kOp == 0) {
#define I(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 1) {
#define I(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(ps));
            I(p0) I(p1) I(p2) I(p3) I(p4) I(p5) I(p6) I(p7)
#undef I
        } else if constexpr (kOp == 2) {
#define I(x) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(ps));
            I(p0) I(p1) I(p2) I(p3) I(p4) I(p5) I(p6) I(p7)
#undef I
        } else if constexpr (kOp == 3) {
#define I(x) asm volatile("v_fma_mix_f32 %0, %1, %0, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(h));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 4) {
#define I(x) asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(x) : "v"(u0 + i));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 5) {
#define I(x) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(x));
            I(d0) I(d1) I(d2) I(d3) I(d4) I(d5) I(d6) I(d7)
#undef I
        } else if constexpr (kOp == 6) {
#define I(x) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 7) {
#define I(x) asm volatile("v_addc_co_u32_e64 %0, vcc, %0, %0, %1" : "+v"(x) : "s"(carry) : "vcc");
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 8) {
#define I(x) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 9) {
#define I(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 10) {
#define I(x) asm volatile("v_mov_b32 %0, %0" : "+v"(x));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 11) {
#define I(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(a0)
#undef I
        } else if constexpr (kOp == 12) {
#define I(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(s) : "vcc");
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 13) {
#define I(x) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(x), "v"(s) : "vcc");
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 17) {
#define I(x) asm volatile("v_fmac_f32_e32 %0, %1, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 18) {
#define I(x) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 19) {
#define I(x) asm volatile("v_mul_f32_e64 %0, -%0, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 20) {
#define I(x) asm volatile("v_min_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 21) {  // VCC set once before the loop (no clobber: no hazard nops)
#define I(x) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 22) {
#define I(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(s), "s"(carry));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 23) {
#define I(x) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(a0)
#undef I
        } else if constexpr (kOp == 24) {
#define I(x) asm volatile("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(x));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 25) {  // compare to an SGPR pair (VOP3), 8 independent destinations
            unsigned long long m0, m1, m2, m3;
            asm volatile("v_cmp_lt_f32_e64 %0, %4, %5\n v_cmp_lt_f32_e64 %1, %4, %6\n"
                         " v_cmp_lt_f32_e64 %2, %4, %7\n v_cmp_lt_f32_e64 %3, %4, %8\n"
                         " v_cmp_lt_f32_e64 %0, %4, %9\n v_cmp_lt_f32_e64 %1, %4, %10\n"
                         " v_cmp_lt_f32_e64 %2, %4, %11\n v_cmp_lt_f32_e64 %3, %4, %5"
                         : "=&s"(m0), "=&s"(m1), "=&s"(m2), "=&s"(m3)
                         : "v"(s), "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6));
            u0 += (uint32_t)(m0 ^ m1 ^ m2 ^ m3);
        } else if constexpr (kOp == 26) {  // VOP3 fma and VOP2 add alternating
#define F(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
#define A(x) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            F(a0) A(a1) F(a2) A(a3) F(a4) A(a5) F(a6) A(a7)
#undef F
#undef A
        } else if constexpr (kOp == 27) {  // VOP2 add and mul alternating
#define M(x) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
#define A(x) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            M(a0) A(a1) M(a2) A(a3) M(a4) A(a5) M(a6) A(a7)
#undef M
#undef A
        } else if constexpr (kOp == 28) {
#define I(x) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 29) {
#define I(x) asm volatile("v_sub_f32_e32 %0, %1, %0" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 30) {  // VOP3 max3 and VOP2 min alternating
#define X(x) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(x) : "v"(s));
#define N(x) asm volatile("v_min_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            X(a0) N(a1) X(a2) N(a3) X(a4) N(a5) X(a6) N(a7)
#undef X
#undef N
        } else if constexpr (kOp == 31) {
#define I(x) asm volatile("v_add_f32_e64 %0, |%0|, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 35) {  // 32-bit integer multiply (the LCG's a * s)
#define I(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 36) {  // 24-bit multiply-add
#define I(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 37) {
#define I(x) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 38) {
#define I(x) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 39) {
#define I(x) asm volatile("v_cvt_f32_u32_e32 %0, %1" : "=v"(x) : "v"(u0 + i));
            CHAIN8(I)
#undef I
        } else if constexpr (kOp == 40) {  // SDWA: the high word of a register, zero-extended, or'ed
#define I(x) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 41) {
#define I(x) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(u7));
            I(u0) I(u1) I(u2) I(u3) I(u4) I(u5) I(u6) I(u7)
#undef I
        } else if constexpr (kOp == 42) {
#define I(x) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(x));
            I(d0) I(d1) I(d2) I(d3) I(d4) I(d5) I(d6) I(d7)
#undef I
        } else if constexpr (kOp == 43) {
#define I(x) asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(x) : "v"(s));
            I(d0) I(d1) I(d2) I(d3) I(d4) I(d5) I(d6) I(d7)
#undef I
        } else if constexpr (kOp == 44) {  // max3 and mul alternating (a main-port form beside a second-port one)
#define X(x) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(x) : "v"(s));
#define M(x) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            X(a0) M(a1) X(a2) M(a3) X(a4) M(a5) X(a6) M(a7)
#undef X
#undef M
        } else if constexpr (kOp == 45) {  // fma_mix and mul alternating
#define X(x) asm volatile("v_fma_mix_f32 %0, %1, %0, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(h));
#define M(x) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(x) : "v"(s));
            X(a0) M(a1) X(a2) M(a3) X(a4) M(a5) X(a6) M(a7)
#undef X
#undef M
        } else {  // 14..16, 32..34: v_fma_f32 under a partial EXEC mask (the branch is outside the loop)
#define I(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
            CHAIN8(I)
#undef I
        }
    }
    const float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y + p4.x + p5.y + p6.x + p7.y +
                    (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) + (float)(u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7);
    if (r == 12345.0f) out[0] = r;  // keeps every chain live
}

template <int kOp>
double run(const char* name, int blocks, float* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(ubench<kOp>, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(ubench<kOp>, dim3(blocks), dim3(256), 0, 0, out, 0.5f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    int dev = 0, cus = 0, clk_khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    // wave-instructions per SIMD = waves per SIMD x iterations x 8
    const double waves_per_simd = (double)blocks * 4 / (cus * 4.0);
    const double insts = waves_per_simd * kIters * 8;
    const double cyc = ms * 1e-3 * clk_khz * 1e3 / insts;
    printf("%-8s %6.2f cycles per wave-instruction per SIMD (%.3f ms)\n", name, cyc, ms);
    return cyc;
}

struct Op {
    const char* name;
    double (*fn)(const char*, int, float*);
};

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 8;
    int dev = 0, cus = 0, clk_khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
    float* out = nullptr;
    if (hipMalloc((void**)&out, 4) != hipSuccess) return 1;
    printf("%d CUs, %d waves per SIMD, clock attribute %.0f MHz\n", cus, wps, clk_khz / 1e3);
    const Op ops[] = {{"fma", run<0>},      {"pk_fma", run<1>},  {"pk_mul", run<2>},   {"fma_mix", run<3>},
                      {"cvt_ub", run<4>},   {"fma_f64", run<5>}, {"rcp", run<6>},      {"addc", run<7>},
                      {"max3", run<8>},     {"add", run<9>},     {"mov", run<10>},     {"and", run<11>},
                      {"cndmask", run<12>}, {"cmp", run<13>},    {"fma_lo32", run<14>}, {"fma_1", run<15>},
                      {"fma_even", run<16>}, {"fmac", run<17>},   {"mul", run<18>},      {"mul_neg", run<19>},
                      {"min", run<20>},      {"cndmask_vcc", run<21>}, {"cndmask_sgpr", run<22>},
                      {"add_u32", run<23>},  {"lshl", run<24>},  {"cmp_sgpr", run<25>}, {"fma+add", run<26>},
                      {"mul+add", run<27>},  {"mov_dpp", run<28>}, {"sub", run<29>},    {"max3+min", run<30>},
                      {"add_abs", run<31>},  {"fma_2lanes", run<32>}, {"fma_4", run<33>}, {"fma_16", run<34>},
                      {"mul_lo_u32", run<35>}, {"mad_u24", run<36>}, {"mul_u24", run<37>}, {"lshl_add", run<38>},
                      {"cvt_f32_u32", run<39>}, {"or_sdwa", run<40>}, {"perm", run<41>}, {"mul_f64", run<42>},
                      {"cvt_f64_f32", run<43>}, {"max3+mul", run<44>}, {"fma_mix+mul", run<45>}};
    for (const Op& op : ops) {
        bool want = argc <= 2;
        for (int i = 2; i < argc; i++) want = want || strcmp(argv[i], op.name) == 0;
        if (want) op.fn(op.name, blocks, out);
    }
    (void)hipFree(out);
    return 0;
}
