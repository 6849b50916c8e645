// pt_trace.h — device code of the trace megakernel (gfx950).
//
// Compiled twice: offline into libpt_hip.so (generic kernels, pt_kernel.hip) and at
// scene-upload time through hipRTC (pt_rtc.cpp), where the flat leaf-box test is a
// generated function with the scene's box planes as constants. Keep this header
// free of host-only includes (hipRTC provides no C library headers).
//
// One persistent launch per sample batch. Every lane runs its own path state
// machine: one loop iteration = one path segment (BVH::intersect + shading,
// bvh.h:156-183 + render.h:36-61 unrolled). A lane whose path ends writes the
// sample's radiance and starts its next sample in the next iteration; lanes whose
// work item is exhausted refill from a wave-private pool (ballot + mbcnt prefix),
// refilled by one global atomic per kChunk items.
//
// Accumulation order is the reference's (render.h:84, image.h:27-40): each sample's
// radiance goes to an HBM slab [sample][pixel][rgb]; pt_accumulate_kernel adds the
// slab into the per-pixel float32 running sum in sample order, so items may run in
// any order on any lane or GPU and the image is still bit-identical.
#pragma once

#include "pt_hip.h"
#include "pt_math.h"

namespace pt {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxSpecularIters = 1 << 16;  // bound for material.h:20-23 (reference: unbounded)
#ifndef PT_CHUNK  // >= kWave (64)
#define PT_CHUNK 1024  // Cornell headline: 64 -> 18.6, 128 -> 36.8, 256 -> 42.8, 1024 -> 43.1, 4096 -> 42.6 Grays/s
#endif
constexpr int kChunk = PT_CHUNK;             // most work items claimed per wave per atomic (host clamps: TraceArgs::chunk)
static_assert(kChunk >= kWave, "a work-pool refill must cover one claim of every lane of a wave");
constexpr int kMaxFlatLeaves = 64;

#ifndef PT_WAVES
#define PT_WAVES 7  // waves per SIMD the trace kernel is register-allocated for (<= 72 VGPRs)
#endif

// Diagnostic build only (make stamps -> lib/libpt_hip_stamps.so): per-wave s_memtime
// deltas of the loop's sections, summed into TraceArgs::stamps. Never in the product build.
#ifdef PT_STAMPS
#define PT_STAMP(v)                                  \
    __builtin_amdgcn_sched_barrier(0);               \
    const uint64_t v = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);
#define PT_STAMP_ADD(i, a, b) stamp_acc[i] += (b) - (a);
#elif defined(PT_MARKS)
// Static-analysis build (never the product): an assembly comment per stamp point, so the
// instructions of each section can be counted in the kernel's .s (scripts/section_isa.py).
#define PT_STAMP(v)                       \
    __builtin_amdgcn_sched_barrier(0);    \
    asm volatile("; @mark " #v);          \
    __builtin_amdgcn_sched_barrier(0);
#define PT_STAMP_ADD(i, a, b)
#else
#define PT_STAMP(v)
#define PT_STAMP_ADD(i, a, b)
#endif
constexpr int kStampSections = 23;  // start, box mask, pair phase, shade, fold, intersect, waves,
                                    // pair iterations, pairs, pair rounds, max pairs of a lane;
                                    // wide: 10 outer iterations, 11 shading lanes, 12 new paths,
                                    // 13 drain rounds, 14 drained entries, 15 end-of-iteration
                                    // drain rounds, 16 path ends; wide launch timeline (100 MHz
                                    // s_memrealtime ticks): 17 ~(first wave start), 18 last wave
                                    // end, 19 ~(first exhaustion of the work), 20 sum of wave
                                    // lifetimes, 21 sum of (wave end - its exhaustion), 22 last
                                    // exhaustion

// hipRTC flat kernels (pt_kernel.hip: flat_mask_source). PT_ADDC_MASK: the lane's leaf
// mask is assembled by a carry chain, one v_addc per leaf with the box test's lane mask as
// the carry-in (the compiler's own form, cndmask + shift + or3, took ~60 instructions for
// Cornell's 32 leaves: 55.3 -> 58.4 Grays/s). PT_PK_PLANES: plane values in pairs with
// packed FP32 ops (same IEEE operations; measured 3 % slower, off).
#ifndef PT_PK_PLANES
#define PT_PK_PLANES 0
#endif
// Wave issue priority (s_setprio) for latency-bound phases: with it, a wave in its pair
// phase (LDS queue -> ds_bpermute -> triangle reads -> atomic, a dependent chain) is
// issued ahead of the SIMD's other waves and leaves that phase sooner (Cornell +2.3 %).
#ifndef PT_PRIO_PAIRS
#define PT_PRIO_PAIRS 1
#endif
#ifndef PT_PRIO_MASK
#define PT_PRIO_MASK 0
#endif
#ifndef PT_PRIO_FOLD
#define PT_PRIO_FOLD 0
#endif
#ifndef PT_PRIO_SHADE
#define PT_PRIO_SHADE 0
#endif
#ifndef PT_PRIO_DRAIN
#define PT_PRIO_DRAIN 2  // wide drains (the same kind of chain): +0.3-0.6 %
#endif
#ifndef PT_PRIO_STEP
#define PT_PRIO_STEP 0
#endif
#ifndef PT_WIDE_THR_SCALE  // the wide step loop's bar scales with the lanes holding paths (0: fixed bar, A/B)
#define PT_WIDE_THR_SCALE 1
#endif
// PT_WIDE_ADDC / PT_WIDE_FAST_M: the wide node test builds its child mask by the same
// carry chain and bounds the margin's M by 255 |A| + |B| (one FMA per axis): 162 -> 155
// VALU per node test, config 4 16.07 -> 16.54 Grays/s.
#ifndef PT_WIDE_ADDC
#define PT_WIDE_ADDC 1
#endif
#ifndef PT_WIDE_FAST_M
#define PT_WIDE_FAST_M 1
#endif
#ifndef PT_ADDC_MASK
#define PT_ADDC_MASK 1
#endif
// PT_SIGN_MASK (the wide node test; the hipRTC flat mask has its own switch,
// PT_FLAT_SIGN_MASK, off: there the extra second-port forms cost more than the main-port
// slots saved, -1.9 % on Cornell and -3.5 % on config 3 against +0.6 % on config 4 for the
// wide walk, profiles/r05_ab): a box's pass bit from sign bits instead of a compare. With tmin3 the largest
// entry value and tmax the least exit value, the test max(tmin3, 0) <= tmax holds exactly when
// neither tmax - tmin3 nor tmax is negative, i.e. when the sign bit of
// bits(tmax - tmin3) | bits(tmax) is clear: the subtraction and the OR dual-issue on the
// second VALU port, and v_alignbit_b32 shifts that sign bit into the lane's mask (fail bits)
// in one main-port instruction, where the compare-based form takes a max(., 0), a compare and
// a carry add. Exact: no operand is NaN or infinite (finite inverse direction, bounded
// coordinates), tmax - tmin3 is +0 when they are equal and negative otherwise (denormals
// kept), and tmax is never -0 (an exit value fl(q A + B) with B = fl(b + m), m >= 2^-99: a
// zero sum is +0, and a nonzero exact sum is a multiple of 2^-124 (|A| >= 2^-100 (1 - 2^-23),
// scale exponents >= -100), so it does not round to zero).
#ifndef PT_SIGN_MASK
#define PT_SIGN_MASK 1
#endif
// |1 / d| <= 2^60 and |o| < 2^60 (the sign-bit box mask's domain; NaN fails both)
__device__ __forceinline__ bool bounded_ray(v3 o, v3 inv) {
    const float ri = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(inv.x), __builtin_fabsf(inv.y)), __builtin_fabsf(inv.z));
    const float ro = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)), __builtin_fabsf(o.z));
    return ri <= 0x1p60f && ro < 0x1p60f;
}
// fail = 2 fail + (sign bit of f): one v_alignbit_b32 (({fail, f} >> 31) & 0xffffffff)
__device__ __forceinline__ uint32_t shl1_add_sign(uint32_t fail, uint32_t f) {
    return __builtin_amdgcn_alignbit(fail, f, 31u);
}
// bits(tmax - tmin3) | bits(tmax): sign bit set iff the box test max(tmin3, 0) <= tmax fails
__device__ __forceinline__ uint32_t box_fail_bits(float tmin3, float tmax) {
    return __float_as_uint(tmax - tmin3) | __float_as_uint(tmax);
}
// hipRTC flat kernels: the clamp of tmin to 0 shared by the boxes whose terms coincide
// (PT_SHARED_CLAMP: 13 fewer main-port max per Cornell wave-iteration; Cornell +0.6 %,
// modified Cornell +1.4-3 %). PT_MULTI_LEAF_OR (one select + or per multi-leaf box instead
// of one carry add per leaf) measured -1.1 % with the compiler's lowering (it turns the
// doublings into shifts and or3s, all main-port forms) and -2 % with them forced into
// v_add_u32 / v_or_b32 (dbl_u32, or_if_bit: 11 fewer main-port slots per wave-iteration,
// but the live patterns spill); off.
#ifndef PT_SHARED_CLAMP
#define PT_SHARED_CLAMP 1
#endif
#ifndef PT_MULTI_LEAF_OR
#define PT_MULTI_LEAF_OR 0
#endif

typedef float f2v __attribute__((ext_vector_type(2)));

// 2x + (this lane's bit of the lane mask m): one v_addc with m as the carry-in.
__device__ __forceinline__ uint32_t shl1_add_bit(uint32_t x, unsigned long long m) {
    uint32_t r;
    unsigned long long c;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(c) : "v"(x), "s"(m));
    return r;
}

// 2x as one v_add_u32 (a form that dual-issues on the second VALU port; the compiler's own
// lowering of x + x merges doublings into shifts, which do not).
__device__ __forceinline__ uint32_t dbl_u32(uint32_t x) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
}

// x | (this lane's bit of m ? pattern : 0): the bits of every leaf of a multi-leaf box.
__device__ __forceinline__ uint32_t or_if_bit(uint32_t x, uint32_t pattern, unsigned long long m) {
    uint32_t t, r;
    asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(t) : "v"(pattern), "s"(m));
    asm("v_or_b32_e32 %0, %1, %2" : "=v"(r) : "v"(t), "v"(x));
    return r;
}

// Leaf boxes of the flat path, passed by value in the kernel-argument segment so the
// generic wave-uniform box loop reads them with scalar loads (SGPR operands). Identical
// boxes are stored once (the two triangles of a quad share one): box u carries the mask of
// the leaves it bounds (Cornell: 20 boxes for 32 leaves).
struct FlatLeaves {
    float box[kMaxFlatLeaves][6];            // distinct leaf boxes, lb.xyz, rt.xyz; padded to a multiple of 4
    unsigned long long bits[kMaxFlatLeaves];  // leaves of box u (bit k = leaf k); 0 for padding
};

// Unsigned 32-bit division by a divisor fixed for the launch (Granlund & Montgomery,
// "Division by invariant integers using multiplication", 1994, round-up form): exact
// for every 32-bit numerator. Integer division has no hardware instruction on gfx950;
// this is a mul_hi and four adds/shifts. Host side: make_fastdiv (pt_kernel.hip).
struct FastDiv {
    uint32_t d, m, sh1, sh2;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
    const uint32_t t = __umulhi(f.m, n);
    return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

struct TraceArgs {
    const float4* __restrict__ nodes;
    const float4* __restrict__ tris;
    const float4* __restrict__ mats;
    const float4* __restrict__ leaves;     // flat leaf list (2 x float4 per leaf, rank order)
    const uint4* __restrict__ wide;        // wide tree (kNodeU4<W> uint4 per node, pt_internal.h)
    const float4* __restrict__ wtris;      // wide-leaf-order triangles (4 float4 each, pt_internal.h)
    const float4* __restrict__ nrm;        // wide: {n.xyz, material id} per rank position
    const float4* __restrict__ umats;      // wide: distinct materials (2 float4 each)
    float* __restrict__ radiance;          // [s_count][npix][3]
    unsigned long long* __restrict__ ctr;  // [0] work head, [1] rays, [2] (unused), [3] runaway
    unsigned long long* __restrict__ work; // the work head (ctr + 0)
    unsigned long long* stamps;            // PT_STAMPS builds: kStampSections cycle sums
    unsigned long long total_items;
    float pos_x, pos_y, pos_z;
    float col0_x, col0_y, col0_z;  // camera transform columns (camera.h:67-71)
    float col1_x, col1_y, col1_z;
    float col2_x, col2_y, col2_z;
    float half_vres_x, half_vres_y, cell;  // v_res / 2 (camera.h:65-66)
    float cz_col0, cz_col1, cz_col2;       // -distance * column z (one rounding each, as on the host)
    int W, npix;
    int part_index, part_count, band_rows;
    int depth;
    uint32_t seed;
    int s_begin, s_count, per_item;
    int stack_size;                      // deferred-left-child stack entries per lane
    int rec_size;                        // path records per lane (depth - 1)
    int num_node4, num_tri4, num_mat4;   // float4 counts of the scene arrays (LDS copy)
    int num_umat4;                       // wide: float4 count of umats
    int num_leaves;                      // flat leaf list length (kFlat kernels)
    int num_boxes_padded;                // distinct flat leaf boxes (flat.box), rounded up to a multiple of 4
    int force_exact_slab;                // test hook PT_FORCE_EXACT_SLAB: 1 never take the IEEE path,
                                         // 2 only in odd waves of a block (mixed waves)
    int wide_thresh;                     // kWide: shade once fewer lanes than this still traverse
    int chunk;                           // items per work-pool refill, kWave..kChunk (small launches: fewer, so every wave gets work)
    uint32_t static_items;               // items each wave starts with, no atomic: wave w's are
                                         // [w static_items, (w + 1) static_items)
    unsigned long long static_base;      // grid waves x static_items: where the refills' items begin
    int pair_queue;                      // kFlat: (lane, leaf) queue entries per wave (0 = per-lane loop)
    int regen_thresh;                    // generate camera rays once this many lanes want one
    int wide_queue;                      // kWide: triangle-queue entries per wave
    int wide_rows;                       // kWide: stack rows of the wide walk
    int wide_top;                        // kWide: nodes [0, wide_top) are read from the block's LDS copy
    uint32_t wide_nodes;                 // kWide: nodes in `wide`
    float wide_span_x, wide_span_y, wide_span_z;  // kWide, float planes: max |plane| per axis (the margin's bound)
    int wide_single;                     // kWide: every leaf holds one triangle (leaf k's is leaf_base + k)
    int wide_compact;                    // kWide: wtris holds 3-float4 records {v1, rank} {v2, v3.x} {v3.yz}
    int tri_fast;                        // kWide: triangle tests by tri_hit_nb (vertex coordinates < 2^60)
    int* __restrict__ exact_stack;       // kWide: [grid][exact_rows][kBlock] stacks of the exact binary walk
    int exact_rows;
    // Fused accumulation (fused_accumulate_chunk): while this launch traces its batch, its
    // waves also add the PREVIOUS batch's slab (acc_src, acc_count samples) into the running
    // sum acc_sum, 64 pixels per chunk, chunk head ctr[2]; acc_chunks = 0: none.
    const float* __restrict__ acc_src;
    float* __restrict__ acc_sum;
    int acc_count, acc_first, acc_chunks, acc_every;
    FastDiv div_npix, div_w, div_band;   // item -> (sample block, pixel), pixel -> row, row -> band
    const float2* __restrict__ theta_tab;  // PT_THETA_TAB: (sin, cos) of theta per grid x (hemisphere_dir_tab)
    int theta_lanes;                       // PT_THETA_TAB 2: waves with at most this many sampling lanes use it
    int dark;                              // every DIFFUSE / SPECULAR material is dark (finish_path's skip)
    // Flagged slab (dark scenes, round 5): only a path that does not end dark stores its record,
    // and sets its bit in `flags`; the accumulation adds only flagged records. An unflagged
    // record would be +0, and adding +0 changes no running sum (a sum that starts at +0 is never
    // -0 under round-to-nearest). nullptr: every path stores and every record is added (dense
    // slab). Bit layout (flags_pm): 0, bit i = record i of this launch's slab (sample-major, as
    // the records); 1 (round 6, frames of several launches), word g * npix + q holds pixel q's
    // samples [32 g, 32 g + 32) (flag_word): a pixel's 32 samples are one load for the sum.
    uint32_t* __restrict__ flags;
    int flags_pm;
    const uint32_t* __restrict__ acc_flags;  // the previous batch's flags (fused accumulation)
    FlatLeaves flat;                     // kFlat kernels with the generic box loop
};

// compact row r of this part -> image row h (row h belongs to part (h / band) % parts)
__device__ __forceinline__ int part_row(const TraceArgs& A, int r) {
    const int k = (int)fdiv((uint32_t)r, A.div_band), i = r - k * A.band_rows;
    return (k * A.part_count + A.part_index) * A.band_rows + i;
}

struct NodeBox {
    v3 lb, rt;
    int a, b;
};

__device__ __forceinline__ NodeBox load_node(const float4* __restrict__ nodes, int n) {
    const float4 p = nodes[2 * n], q = nodes[2 * n + 1];
    return NodeBox{v3{p.x, p.y, p.z}, v3{p.w, q.x, q.y}, __float_as_int(q.z), __float_as_int(q.w)};
}

template <bool kFiniteInv>
__device__ __forceinline__ bool box_hit(v3 lb, v3 rt, v3 o, v3 inv) {
    return kFiniteInv ? slab_hit_finite(lb, rt, o, inv) : slab_hit(lb, rt, o, inv);
}

// BVH::intersect (bvh.h:156-183) in child-pair form. The reference pops a node, tests
// its box, then tests a leaf's triangles or pushes left and right (right is popped
// first). Here both children's boxes are tested when their parent is processed (a box
// test is a pure function, so testing it earlier changes nothing), the right subtree
// is entered first and only a hit left sibling is deferred on the stack: the sequence
// of triangle tests — and so the first-found winner among equal t — is the reference's.
template <bool kFiniteInv, typename NodePtr, typename TriPtr>
__device__ __forceinline__ int intersect_tree(NodePtr nodes, TriPtr tris, int* __restrict__ stk, int tid, v3 o,
                                              v3 d, v3 inv, float& t_out) {
    int hit = -1;
    float t = 1e30f;
    int sp = 0;
    const NodeBox root = load_node(nodes, 0);
    int ca = root.a, cb = root.b;
    bool go = box_hit<kFiniteInv>(root.lb, root.rt, o, inv);
    while (go) {
        if (ca >= 0) {
            const NodeBox L = load_node(nodes, ca);
            const NodeBox R = load_node(nodes, ca + 1);
            const bool hl = box_hit<kFiniteInv>(L.lb, L.rt, o, inv);
            const bool hr = box_hit<kFiniteInv>(R.lb, R.rt, o, inv);
            if (hr) {
                if (hl) {
                    stk[sp * kBlock + tid] = ca;
                    sp++;
                }
                ca = R.a;
                cb = R.b;
                continue;
            }
            if (hl) {
                ca = L.a;
                cb = L.b;
                continue;
            }
        } else {
            for (int i = -ca - 1; i <= cb; i++) {
                const float4 t0 = tris[3 * i], t1 = tris[3 * i + 1], t2 = tris[3 * i + 2];
                float tt;
                if (tri_hit(v3{t0.x, t0.y, t0.z}, v3{t0.w, t1.x, t1.y}, v3{t1.z, t1.w, t2.x}, o, d, tt) && tt < t) {
                    t = tt;
                    hit = i;
                }
            }
        }
        if (sp == 0) break;
        sp--;
        const float4 q = nodes[2 * stk[sp * kBlock + tid] + 1];
        ca = __float_as_int(q.z);
        cb = __float_as_int(q.w);
    }
    t_out = t;
    return hit;
}

// Generic flat box test: every distinct leaf box of the kernel-argument table, 4 per
// iteration; a passing box sets the bits of all its leaves.
struct TableBoxMask {
    static constexpr bool kMask32 = false;     // leaf bits fit 32 bits
    static constexpr bool kSingleTri = false;  // leaf k holds exactly triangle rank k
    static constexpr bool kSpecular = true;    // the scene may hold SPECULAR materials
    static constexpr bool kTriFast = false;    // pair rounds use tri_hit_nb (vertex coordinates < 2^60)
    static constexpr bool kSignMask = false;   // box bits from sign bits (PT_SIGN_MASK; bounded inverse directions)
    static constexpr bool kAlbedoX2 = false;   // the block's material copy holds 2 * albedo (finish_path)
    static constexpr bool kDarkKnown = false;  // kDark is not known at compile time: finish_path reads A.dark
    static constexpr bool kBoxPairs = false;   // mask bits are leaves (hipRTC kernels may use box-level pairs)
    static constexpr int kBoxes = 0;
    static constexpr uint16_t kBoxTab[1] = {0};
    static constexpr bool kDark = false;
    __device__ __forceinline__ static unsigned long long mask(const TraceArgs& A, v3 o, v3 inv) {
        const float(*box)[6] = A.flat.box;
        unsigned long long m = 0;
        const int n = A.num_boxes_padded;
        for (int k = 0; k < n; k += 4) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float* b = box[k + j];
                if (slab_hit_finite(v3{b[0], b[1], b[2]}, v3{b[3], b[4], b[5]}, o, inv)) m |= A.flat.bits[k + j];
            }
        }
        return m;
    }
};

// The kernel-argument box table with the scene flags a hipRTC scene kernel bakes in, for the
// scenes BVH::build makes (round 6, pt_flat_fast.hip): every leaf one triangle, vertex
// coordinates below 2^60, a dark scene with the pre-doubled albedo allowed (host: the same
// gates as the hipRTC source), leaf bits in 32 bits or not, the specular sampler or not. It
// runs a cold first frame while the scene kernel compiles: 81 % of the scene kernel's speed
// on Cornell against 71 % for TableBoxMask (profiles/r06_cold).
template <bool kSpec, bool kM32>
struct FastTableMask : TableBoxMask {
    static constexpr bool kMask32 = kM32;
    static constexpr bool kSingleTri = true;
    static constexpr bool kSpecular = kSpec;
    static constexpr bool kTriFast = true;
    static constexpr bool kAlbedoX2 = true;
    static constexpr bool kDarkKnown = true;
    static constexpr bool kDark = true;
};

// Triangle phase of the flat path for one lane: the triangles of the leaves in `mask`,
// in rank order, so the first strict minimum is the reference's winner (bvh.h:171).
template <typename TriPtr, typename LeafPtr>
__device__ __forceinline__ int flat_tri_loop(unsigned long long mask, LeafPtr lleaves, TriPtr tris, v3 o, v3 d,
                                             float& t_out) {
    int hit = -1;
    float t = 1e30f;
    while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        const float4 b = lleaves[2 * k + 1];
        const int last = __float_as_int(b.w);
        for (int i = __float_as_int(b.z); i <= last; i++) {
            const float4 t0 = tris[3 * i], t1 = tris[3 * i + 1], t2 = tris[3 * i + 2];
            float tt;
            if (tri_hit(v3{t0.x, t0.y, t0.z}, v3{t0.w, t1.x, t1.y}, v3{t1.z, t1.w, t2.x}, o, d, tt) && tt < t) {
                t = tt;
                hit = i;
            }
        }
    }
    t_out = t;
    return hit;
}

// flat_tri_loop for a box mask (box-level pairs): box u's one or two triangles (boxtab[u] =
// rank0 | rank1 << 8, 0xff = none). Boxes are not visited in rank order, so the winner is the
// least (t, rank) pair, as the pair phase's atomic min picks it (bvh.h:171's first strict
// minimum in rank order).
__device__ __forceinline__ int flat_box_loop(unsigned long long mask, const uint16_t* __restrict__ boxtab,
                                             const float4* __restrict__ tris, v3 o, v3 d, float& t_out) {
    int hit = -1;
    float t = 1e30f;
    while (mask) {
        const int u = __builtin_ctzll(mask);
        mask &= mask - 1;
        const uint32_t code = boxtab[u];
        for (int j = 0; j < 2; j++) {
            const uint32_t r = j ? code >> 8 : code & 0xffu;
            if (r == 0xffu) continue;
            const int i = (int)r;
            const float4 t0 = tris[3 * i], t1 = tris[3 * i + 1], t2 = tris[3 * i + 2];
            float tt;
            if (tri_hit(v3{t0.x, t0.y, t0.z}, v3{t0.w, t1.x, t1.y}, v3{t1.z, t1.w, t2.x}, o, d, tt) &&
                (tt < t || (tt == t && i < hit))) {
                t = tt;
                hit = i;
            }
        }
    }
    t_out = t;
    return hit;
}

// BVH::intersect for scenes with <= 64 leaves, as a flat leaf list.
// With finite inv the slab test is monotone under box containment, so a leaf box
// passes only if every ancestor box passes: the triangles the reference tests are
// exactly those of leaves whose own box passes, whatever the tree. Step 1 tests every
// leaf box wave-uniformly (BoxMask: the kernel-argument table, or a hipRTC-generated
// function with the scene's planes as constants); step 2 tests each lane's passing
// leaves in rank order, so the first strict minimum is the reference's winner (bvh.h:171).
template <typename BoxMask, typename TriPtr, typename LeafPtr>
__device__ __forceinline__ int intersect_flat(const TraceArgs& A, LeafPtr lleaves, TriPtr tris, v3 o, v3 d, v3 inv,
                                              float& t_out, const uint16_t* __restrict__ boxtab) {
    if constexpr (BoxMask::kBoxPairs) return flat_box_loop(BoxMask::mask(A, o, inv), boxtab, tris, o, d, t_out);
    return flat_tri_loop(BoxMask::mask(A, o, inv), lleaves, tris, o, d, t_out);
}

// Inclusive prefix sum over the wave's 64 lanes; every lane must be active (DPP row
// shifts within rows of 16, then the row-15 / row-31 broadcasts of gfx9).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Order this wave's LDS writes before its later LDS reads of other lanes' slots.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float lane_float(int addr, float v) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

// The flat path with the triangle phase spread over the wave. Per lane, the reference
// tests the triangles of its passing leaves and keeps the first strict minimum in rank
// order (bvh.h:171): the least (t, rank) pair among hits with t < 1e30f (FLOAT_INF, the
// initial t). A lane's loop over its own leaves would cost the wave max-over-lanes
// iterations; here the (lane, leaf) pairs of the whole wave go to an LDS queue (wave
// prefix sum of the popcounts) and every round tests 64 of them, one per lane, with the
// owner's ray fetched by ds_bpermute. Each hit is reduced into the owner's slot with a
// 64-bit LDS atomic min of (t bits, rank): t > 0, so its bits order like its value, and
// equal t resolves to the lower rank — exactly the reference's winner, in any order.
// Must be called by all 64 lanes (wave-uniform control flow); `mask` = the lane's
// passing leaves (0 for a lane without a ray). The queue is the wave's own LDS array of
// A.pair_queue 16-bit entries (lane << 6 | leaf), written linearly; when the wave's pairs
// exceed it, the lanes test their own leaves in a loop (flat_tri_loop, same result).
template <typename BoxMask, typename TriPtr, typename LeafPtr>
__device__ __forceinline__ int intersect_flat_pairs(const TraceArgs& A, unsigned long long mask, LeafPtr lleaves,
                                                    TriPtr tris, uint16_t* __restrict__ queue,
                                                    unsigned long long* __restrict__ best, int tid, int lane, v3 o,
                                                    v3 d, float& t_out, const uint16_t* __restrict__ boxtab) {
    const uint32_t c = (uint32_t)__popcll(mask);
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (total > (uint32_t)A.pair_queue) {
        if constexpr (BoxMask::kBoxPairs) return flat_box_loop(mask, boxtab, tris, o, d, t_out);
        return flat_tri_loop(mask, lleaves, tris, o, d, t_out);
    }
    best[tid] = ~0ull;
    uint16_t* at = queue + (incl - c);
    // Two entries per iteration (the second predicated on a second bit): the loop runs
    // max-over-lanes popcount / 2 times (Cornell: 9.3 leaves for the busiest lane), and
    // the tag is kept in a register rather than re-formed every iteration (+0.8 %).
    uint32_t tag = (uint32_t)lane << 6;
    asm volatile("" : "+v"(tag));
    if constexpr (BoxMask::kMask32) {
        uint32_t m = (uint32_t)mask;
        while (m) {
            const uint32_t b0 = (uint32_t)__builtin_ctz(m);
            m &= m - 1;
            at[0] = (uint16_t)(tag | b0);
            if (m) {
                at[1] = (uint16_t)(tag | (uint32_t)__builtin_ctz(m));
                m &= m - 1;
            }
            at += 2;
        }
    } else {
        while (mask) {
            const uint32_t b0 = (uint32_t)__builtin_ctzll(mask);
            mask &= mask - 1;
            at[0] = (uint16_t)(tag | b0);
            if (mask) {
                at[1] = (uint16_t)(tag | (uint32_t)__builtin_ctzll(mask));
                mask &= mask - 1;
            }
            at += 2;
        }
    }
    wave_lds_sync();
    unsigned long long* wbest = best + (tid - lane);
    for (uint32_t base = 0; base < total; base += kWave) {
        const uint32_t p = base + (uint32_t)lane;
        const uint32_t e = p < total ? (uint32_t)queue[p] : 0u;
        const int owner = (int)(e >> 6), leaf = (int)(e & 63u);
        const int addr = owner << 2;
        const v3 ro{lane_float(addr, o.x), lane_float(addr, o.y), lane_float(addr, o.z)};
        const v3 rd{lane_float(addr, d.x), lane_float(addr, d.y), lane_float(addr, d.z)};
        if (BoxMask::kBoxPairs && p < total) {
            // a (lane, box) pair: the box's one or two triangles (boxtab: rank0 | rank1 << 8)
            const uint32_t code = boxtab[leaf];
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const uint32_t r = j ? code >> 8 : code & 0xffu;
                if (j == 0 || r != 0xffu) {  // every box bounds at least one leaf
                    const int i = (int)r;
                    const float4 t0 = tris[3 * i], t1 = tris[3 * i + 1], t2 = tris[3 * i + 2];
                    const v3 v1{t0.x, t0.y, t0.z}, e1{t0.w, t1.x, t1.y}, e2{t1.z, t1.w, t2.x};
                    float tt;
                    const bool h = BoxMask::kTriFast ? tri_hit_nb(v1, e1, e2, ro, rd, tt) : tri_hit(v1, e1, e2, ro, rd, tt);
                    if (h && tt < 1e30f)
                        atomicMin(wbest + owner, ((unsigned long long)__float_as_uint(tt) << 32) | (uint32_t)i);
                }
            }
        } else if (p < total) {
            int first = leaf, last = leaf;
            if constexpr (!BoxMask::kSingleTri) {
                const float4 b = lleaves[2 * leaf + 1];
                first = __float_as_int(b.z);
                last = __float_as_int(b.w);
            }
            for (int i = first; i <= last; i++) {
                const float4 t0 = tris[3 * i], t1 = tris[3 * i + 1], t2 = tris[3 * i + 2];
                const v3 v1{t0.x, t0.y, t0.z}, e1{t0.w, t1.x, t1.y}, e2{t1.z, t1.w, t2.x};
                float tt;
                const bool h = BoxMask::kTriFast ? tri_hit_nb(v1, e1, e2, ro, rd, tt) : tri_hit(v1, e1, e2, ro, rd, tt);
#ifdef PT_EXP_DUP_PAIR  // measurement only: the pair's triangle test once more
                {
                    v3 o2 = ro;
                    asm volatile("" : "+v"(o2.x));
                    float t2;
                    const bool h2 = BoxMask::kTriFast ? tri_hit_nb(v1, e1, e2, o2, rd, t2) : tri_hit(v1, e1, e2, o2, rd, t2);
                    asm volatile("" ::"v"(t2), "v"((int)h2));
                }
#endif
                if (h && tt < 1e30f)
                    atomicMin(wbest + owner, ((unsigned long long)__float_as_uint(tt) << 32) | (uint32_t)i);
            }
        }
    }
    wave_lds_sync();
    const unsigned long long kb = best[tid];
    if ((uint32_t)kb == 0xffffffffu) {
        t_out = 1e30f;
        return -1;
    }
    t_out = __uint_as_float((uint32_t)(kb >> 32));
    return (int)(uint32_t)kb;
}

#ifndef PT_THETA_TAB
// hemisphere_sample's theta terms from the device table (hemisphere_dir_tab): 0 never, 1
// always, 2 (default) in waves where at most A.theta_lanes lanes sample — scenes that mix
// specular and diffuse materials (config 3: +6.9 %); in all-diffuse scenes most lanes sample
// and the table's random reads cost more than they save (Cornell -8 % with 1), so the host
// passes theta_lanes = 0 there (profiles/r04_theta)
#define PT_THETA_TAB 2
#endif

// PT_FLAT_ONLY (the hipRTC scene kernel's source): the wide walk and the tree-walk bodies
// below are not compiled (less to parse in the hipRTC compile a cold process waits for).
#ifndef PT_FLAT_ONLY
// ---- wide tree walk (kWide kernels)
//
// Node format (host: build_wide, pt_internal.h): kNodeU4<W> uint4 per node, BFS order.
//   u[0..2] origin O (float), u[3] meta = (ex+128) | (ey+128) << 8 | (ez+128) << 16 | ni << 24 | nl << 28
//   u[4] child_base, u[5] leaf_base, u[6..7] cumulative triangle end offset of leaf k (byte k)
//   u[8..] per axis a: byte planes lo.a[W] hi.a[W] hi.a[W] lo.a[W] (kF16 = false), or
//          binary16 planes lo.a[W] hi.a[W] (kF16)
// Slots [0, ni) are inner children (node child_base + j), [ni, ni + nl) leaves.
// Float planes (plane format kPF = 2, round 6): u[0] child_base | ni << 24 | nl << 28,
//   u[1] leaf_base, u[2..3] leaf ends, then per axis a lo.a[W] hi.a[W] as floats from u[4].
template <int W, int kPF = 1>
constexpr int kNodeU4 = kPF == 2 ? 1 + 3 * W / 2 : W == 8 ? 8 : 5;

// Byte planes: a ray's (entry, exit) run on axis a starts at byte 32 + 16 QW a + t_a of a
// node: t_a = 0 gives (lo, hi) for 1 / d >= 0, t_a = 8 QW gives (hi, lo) for 1 / d < 0
// (octant order), fixed for the whole walk. Half planes: the entry run is at
// 32 + 4 W a + t_a (t_a = 0: lo, 2 W: hi) and the exit run at the other. t_a is re-made per
// node from the sign's lane mask (scalar registers) by one select, so no vector register
// holds it across the walk (the 8-wide walk is at its 80-register budget).
__device__ __forceinline__ uint32_t lane_sel(uint32_t a, uint32_t b, unsigned long long m) {
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// The words of a node one ray needs: the header and its entry / exit planes per axis
// (W bytes or W halves each).
template <int W, bool kF16>
struct WideNode {
    static constexpr int kWords = kF16 ? W / 2 : W / 4;
    uint4 h0, h1;
    uint32_t en[3][kWords], ex[3][kWords];
};

// Per-lane byte offsets (from the node's start) of the entry and exit runs of each axis.
template <int W, bool kF16>
struct WideOff {
    uint32_t en[3], ex[3];
};

#ifndef PT_WIDE_EXIT_SUB
#define PT_WIDE_EXIT_SUB 1
#endif
// The constant part of an exit run's offset that the loads add (PT_WIDE_EXIT_SUB; a buffer
// load takes it as its scalar offset: the compiler cannot fold it into the immediate field of
// a per-lane offset formed by a subtraction)
template <int W>
__device__ __forceinline__ constexpr uint32_t wide_exit_c(int a) { return PT_WIDE_EXIT_SUB ? 32u + 4u * W * a : 0u; }
// The select picks between nb and nb + 2 W (one v_cndmask per run); the constant part
// 32 + 4 W a is left for the load instruction's immediate offset field.
template <int W, bool kF16>
__device__ __forceinline__ WideOff<W, kF16> wide_offsets(uint32_t nb, const unsigned long long (&neg)[3]) {
    WideOff<W, kF16> f;
    const uint32_t nb2 = nb + 2u * W;
#if PT_WIDE_EXIT_SUB
    // the exit run is the other one: (nb + nb2) - entry, one v_sub_u32 (second VALU port)
    // instead of a second select (main port) per axis
    const uint32_t both = nb + nb2;
#endif
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if constexpr (kF16) {
#if PT_WIDE_EXIT_SUB
            const uint32_t e = lane_sel(nb, nb2, neg[a]);
            f.en[a] = e + (32u + 4u * W * a);
            f.ex[a] = both - e;  // + wide_exit_c<W>(a), added by the loads (buffer loads: soffset)
#else
            f.en[a] = lane_sel(nb, nb2, neg[a]) + (32u + 4u * W * a);
            f.ex[a] = lane_sel(nb2, nb, neg[a]) + (32u + 4u * W * a);
#endif
        } else {
            f.en[a] = lane_sel(nb, nb2, neg[a]) + (32u + 4u * W * a);  // (entry, exit) in one run
            f.ex[a] = 0u;
        }
    }
    return f;
}

// LDS copy of the top levels: plain LDS loads at byte offset nb (+ the plane runs).
template <int W, bool kF16>
__device__ __forceinline__ WideNode<W, kF16> load_wide_node_lds(const char* __restrict__ base, uint32_t nb,
                                                                const WideOff<W, kF16>& off) {
    WideNode<W, kF16> n;
    n.h0 = *reinterpret_cast<const uint4*>(base + nb);
    n.h1 = *reinterpret_cast<const uint4*>(base + nb + 16);
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if constexpr (kF16 && W == 8) {
            const uint4 e = *reinterpret_cast<const uint4*>(base + off.en[a]);
            const uint4 x = *reinterpret_cast<const uint4*>(base + off.ex[a] + wide_exit_c<W>(a));
            n.en[a][0] = e.x, n.en[a][1] = e.y, n.en[a][2] = e.z, n.en[a][3] = e.w;
            n.ex[a][0] = x.x, n.ex[a][1] = x.y, n.ex[a][2] = x.z, n.ex[a][3] = x.w;
        } else if constexpr (kF16) {
            const uint2 e = *reinterpret_cast<const uint2*>(base + off.en[a]);
            const uint2 x = *reinterpret_cast<const uint2*>(base + off.ex[a] + wide_exit_c<W>(a));
            n.en[a][0] = e.x, n.en[a][1] = e.y;
            n.ex[a][0] = x.x, n.ex[a][1] = x.y;
        } else if constexpr (W == 8) {
            const uint4 v = *reinterpret_cast<const uint4*>(base + off.en[a]);
            n.en[a][0] = v.x;
            n.en[a][1] = v.y;
            n.ex[a][0] = v.z;
            n.ex[a][1] = v.w;
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(base + off.en[a]);
            n.en[a][0] = v.x;
            n.ex[a][0] = v.y;
        }
    }
    return n;
}

// Global tree: buffer loads, a 32-bit per-lane byte offset from the tree's base in
// scalar registers (no 64-bit address arithmetic per load).
template <int W, bool kF16>
__device__ __forceinline__ WideNode<W, kF16> load_wide_node_buf(__amdgpu_buffer_rsrc_t r, uint32_t nb,
                                                                const WideOff<W, kF16>& off) {
    WideNode<W, kF16> n;
    const auto h0 = __builtin_amdgcn_raw_buffer_load_b128(r, nb, 0, 0);
    const auto h1 = __builtin_amdgcn_raw_buffer_load_b128(r, nb + 16u, 0, 0);
    n.h0 = make_uint4(h0[0], h0[1], h0[2], h0[3]);
    n.h1 = make_uint4(h1[0], h1[1], h1[2], h1[3]);
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if constexpr (kF16 && W == 8) {
            const auto e = __builtin_amdgcn_raw_buffer_load_b128(r, off.en[a], 0, 0);
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off.ex[a], (int)wide_exit_c<W>(a), 0);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                n.en[a][i] = e[i];
                n.ex[a][i] = x[i];
            }
        } else if constexpr (kF16) {
            const auto e = __builtin_amdgcn_raw_buffer_load_b64(r, off.en[a], 0, 0);
            const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off.ex[a], (int)wide_exit_c<W>(a), 0);
            n.en[a][0] = e[0], n.en[a][1] = e[1];
            n.ex[a][0] = x[0], n.ex[a][1] = x[1];
        } else if constexpr (W == 8) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off.en[a], 0, 0);
            n.en[a][0] = v[0];
            n.en[a][1] = v[1];
            n.ex[a][0] = v[2];
            n.ex[a][1] = v[3];
        } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off.en[a], 0, 0);
            n.en[a][0] = v[0];
            n.ex[a][0] = v[1];
        }
    }
    return n;
}

// The walk of BVH::intersect (bvh.h:156-183) over the quantised wide tree. Child box on
// axis a (real numbers): [O + lo 2^e, O + hi 2^e], which contains the reference's box.
// Its slab value at plane q is computed as fl(q A + B) with A = 2^e inv (exact) and
// B = fl(fl(O - o) inv); against the reference's fl(fl(L - o) inv) at any plane L inside
// the node's range that differs by at most 5.01 u M (u = 2^-24, M = max(|B|, |Q A + B|)
// over the axes, Q = 255 for byte planes, 2047 for half planes). The test widens every
// child's [tmin, tmax] by folding a margin into B: entry planes use fl(B - m), exit planes
// fl(B + m), m = 2^-19 M + 2^-99, which covers that difference plus the two extra
// roundings (< 3 u M), so every child whose exact box passes the reference's test passes
// here (and so does each ancestor, by containment). Valid while |inv| <= 2^60 and |o|,
// |coordinates| < 2^64 (no overflow; the kernel checks the ray, the host the scene).
// Octant order: for inv < 0 the hi plane is the entry plane — the ray loads its own runs
// (wide_offsets). Byte planes: children in pairs with packed FMAs (v_pk_fma_f32: two IEEE
// fmas) after one byte conversion per plane; half planes: one v_fma_mix_f32 per plane
// (the binary16 integer converted exactly inside the fused multiply-add).
template <int W>
struct WideHits {
    uint32_t inner, leaf;  // passing inner slots (bit j = slot j), passing leaves (bit k = leaf k)
    uint32_t child_base, leaf_base, ends_lo, ends_hi;
};


__device__ __forceinline__ float byte_f(uint32_t w, int j) { return (float)((w >> (8 * (j & 3))) & 255u); }

// slab values of children j and j + 1 on one axis: fl(q A + B) for the bytes of word w
__device__ __forceinline__ f2v slab_pair(uint32_t w, int j, float A, float B) {
    const f2v qv = {byte_f(w, j), byte_f(w, j + 1)};
    const f2v av = {A, A}, bv = {B, B};
    return __builtin_elementwise_fma(qv, av, bv);
}

// fl(q A + B) for the binary16 plane q in the low / high half of w (one fused operation:
// the exact f16 -> f32 conversion of q, the product and the sum rounded once)
__device__ __forceinline__ float slab_half_lo(uint32_t w, float A, float B) {
    return __builtin_fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu)), A, B);
}
__device__ __forceinline__ float slab_half_hi(uint32_t w, float A, float B) {
    return __builtin_fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16)), A, B);
}

template <int W, bool kF16>
__device__ __forceinline__ WideHits<W> wide_node_test(const WideNode<W, kF16>& nd, v3 o, v3 inv) {
    constexpr float kQ = kF16 ? 2047.0f : 255.0f;
    const uint32_t meta = nd.h0.w;
    const float Ax = __builtin_ldexpf(inv.x, (int)(meta & 255u) - 128);
    const float Ay = __builtin_ldexpf(inv.y, (int)((meta >> 8) & 255u) - 128);
    const float Az = __builtin_ldexpf(inv.z, (int)((meta >> 16) & 255u) - 128);
    const float Bx = (__uint_as_float(nd.h0.x) - o.x) * inv.x;
    const float By = (__uint_as_float(nd.h0.y) - o.y) * inv.y;
    const float Bz = (__uint_as_float(nd.h0.z) - o.z) * inv.z;
#if PT_WIDE_FAST_M
    // M' = Q |A| + |B| >= max(|B|, |Q A + B|): a larger M only widens the margin
    const float Mx = __builtin_fmaf(kQ, __builtin_fabsf(Ax), __builtin_fabsf(Bx));
    const float My = __builtin_fmaf(kQ, __builtin_fabsf(Ay), __builtin_fabsf(By));
    const float Mz = __builtin_fmaf(kQ, __builtin_fabsf(Az), __builtin_fabsf(Bz));
#else
    const float Mx = __builtin_fmaxf(__builtin_fabsf(Bx), __builtin_fabsf(__builtin_fmaf(kQ, Ax, Bx)));
    const float My = __builtin_fmaxf(__builtin_fabsf(By), __builtin_fabsf(__builtin_fmaf(kQ, Ay, By)));
    const float Mz = __builtin_fmaxf(__builtin_fabsf(Bz), __builtin_fabsf(__builtin_fmaf(kQ, Az, Bz)));
#endif
    const float m = __builtin_fmaf(__builtin_fmaxf(__builtin_fmaxf(Mx, My), Mz), 0x1p-19f, 0x1p-99f);
    const float Enx = Bx - m, Eny = By - m, Enz = Bz - m;  // entry planes, lowered
    const float Exx = Bx + m, Exy = By + m, Exz = Bz + m;  // exit planes, raised
    uint32_t hits = 0;
#if PT_SIGN_MASK
    uint32_t fbits[W];
#elif PT_WIDE_ADDC
    bool pass[W];
#endif
#pragma unroll
    for (int j = 0; j < W; j += 2) {
        f2v enx, eny, enz, exx, exy, exz;
        if constexpr (kF16) {
            const int w = j >> 1;
            enx = f2v{slab_half_lo(nd.en[0][w], Ax, Enx), slab_half_hi(nd.en[0][w], Ax, Enx)};
            eny = f2v{slab_half_lo(nd.en[1][w], Ay, Eny), slab_half_hi(nd.en[1][w], Ay, Eny)};
            enz = f2v{slab_half_lo(nd.en[2][w], Az, Enz), slab_half_hi(nd.en[2][w], Az, Enz)};
            exx = f2v{slab_half_lo(nd.ex[0][w], Ax, Exx), slab_half_hi(nd.ex[0][w], Ax, Exx)};
            exy = f2v{slab_half_lo(nd.ex[1][w], Ay, Exy), slab_half_hi(nd.ex[1][w], Ay, Exy)};
            exz = f2v{slab_half_lo(nd.ex[2][w], Az, Exz), slab_half_hi(nd.ex[2][w], Az, Exz)};
        } else {
            const int w = j >> 2;
            enx = slab_pair(nd.en[0][w], j, Ax, Enx);
            eny = slab_pair(nd.en[1][w], j, Ay, Eny);
            enz = slab_pair(nd.en[2][w], j, Az, Enz);
            exx = slab_pair(nd.ex[0][w], j, Ax, Exx);
            exy = slab_pair(nd.ex[1][w], j, Ay, Exy);
            exz = slab_pair(nd.ex[2][w], j, Az, Exz);
        }
#pragma unroll
        for (int c = 0; c < 2; c++) {
#if PT_SIGN_MASK
            const float tmin3 = __builtin_fmaxf(__builtin_fmaxf(enx[c], eny[c]), enz[c]);
            const float tmax = __builtin_fminf(__builtin_fminf(exx[c], exy[c]), exz[c]);
            fbits[j + c] = box_fail_bits(tmin3, tmax);
#else
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(enx[c], eny[c]), enz[c]), 0.0f);
            const float tmax = __builtin_fminf(__builtin_fminf(exx[c], exy[c]), exz[c]);
#if PT_WIDE_ADDC
            pass[j + c] = tmin <= tmax;
#else
            hits |= (tmin <= tmax) ? (1u << (j + c)) : 0u;
#endif
#endif
        }
    }
#if PT_SIGN_MASK
    // bit j = child j fails, shifted in high child first; the passing children are the others
    uint32_t fail = 0;
#pragma unroll
    for (int j = W - 1; j >= 0; j--) fail = shl1_add_sign(fail, fbits[j]);
    hits = ~fail;
#elif PT_WIDE_ADDC
    // bit j = child j, assembled high child first by a carry chain (as the flat box mask)
#pragma unroll
    for (int j = W - 1; j >= 0; j--) hits = shl1_add_bit(hits, __builtin_amdgcn_ballot_w64(pass[j]));
#endif
    const uint32_t ni = (meta >> 24) & 15u, nl = meta >> 28;
    hits &= (1u << (ni + nl)) - 1u;
    return WideHits<W>{hits & ((1u << ni) - 1u), hits >> ni, nd.h1.x, nd.h1.y, nd.h1.z, nd.h1.w};
}

// ---- float planes (kPF = 2, PT_WIDE_PLANES=f32)
//
// The child planes are the reference's own float boxes (bvh.h:12-16), so a node carries no
// origin or scale and the per-node header arithmetic of the quantised test (2^e inv, the
// origin's B, the margin bound) is gone. A plane's slab value is fl(L inv + C) with C a
// per-ray constant: C_en = fl(-o inv - m) for entry planes, C_ex = fl(-o inv + m) for exit
// planes, m = 2^-22 (|o| + S) |inv| + 2^-99 per axis, S = max |plane| of the tree on that
// axis (wide_ray_consts, once per ray segment). Two children per v_pk_fma_f32.
//
// Conservative (every child whose box passes the reference's aabb.h:20-29 test passes
// here): with x = (L - o) inv exact, the reference's r = fl(fl(L - o) inv) is within
// 2.01 u |x| + 2^-150 of x (u = 2^-24; a subnormal difference is exact), |x| <=
// (|L| + |o|) |inv|; ours before its last rounding is s = L inv + C = x + m + b (m - o inv),
// |b| <= u. So s - r >= m (1 - u) - u |o inv| - 2.01 u (S + |o|) |inv| - 2^-150 > 0 because
// the computed m >= 4 u (1 - u)^3 (|o| + S) |inv| + 2^-99 (1 - u) exceeds 3.01 u (|o| + S)
// |inv| + 2^-150 strictly; rounding is monotone, so fl(s) >= r for exit planes, and the
// mirror argument gives fl(s) <= r for entry planes. Then tmin3 <= the reference's tmin
// and tmax >= its tmax. The sign-bit mask (box_fail_bits) stays exact: a -0 exit value
// means s <= 0 (round to nearest never gives -0 for a positive sum), so the reference's
// value on that axis r < s <= 0 and the reference rejects the box too. Valid under the walk's ray bound (|inv| <= 2^60, |o| <
// 2^64) and the host's plane bound (|L| < 2^64): no overflow. An empty slot (lo = +inf,
// hi = -inf) gives tmin3 = +inf, tmax = -inf and fails; the slot mask drops it anyway.
// The nine per-ray operands of the plane FMAs packed into five register pairs, each FMA
// broadcasting one half of a pair to both children by op_sel (pk_fma_bc): the compiler's own
// v_pk_fma_f32 for {a, a} operands holds a duplicated copy of every broadcast value (nine more
// registers, which spilled). p[0] = {inv.x, inv.y}, p[1] = {inv.z, C_en.x}, p[2] = {C_en.y,
// C_en.z}, p[3] = {C_ex.x, C_ex.y}, p[4] = {C_ex.z, -}.
struct WideRay {
    f2v p[5];
};

__device__ __forceinline__ WideRay wide_ray_consts(const TraceArgs& A, v3 o, v3 inv) {
    const float mx = __builtin_fmaf((__builtin_fabsf(o.x) + A.wide_span_x) * __builtin_fabsf(inv.x), 0x1p-22f, 0x1p-99f);
    const float my = __builtin_fmaf((__builtin_fabsf(o.y) + A.wide_span_y) * __builtin_fabsf(inv.y), 0x1p-22f, 0x1p-99f);
    const float mz = __builtin_fmaf((__builtin_fabsf(o.z) + A.wide_span_z) * __builtin_fabsf(inv.z), 0x1p-22f, 0x1p-99f);
    WideRay r;
    r.p[0] = f2v{inv.x, inv.y};
    r.p[1] = f2v{inv.z, __builtin_fmaf(-o.x, inv.x, -mx)};
    r.p[2] = f2v{__builtin_fmaf(-o.y, inv.y, -my), __builtin_fmaf(-o.z, inv.z, -mz)};
    r.p[3] = f2v{__builtin_fmaf(-o.x, inv.x, mx), __builtin_fmaf(-o.y, inv.y, my)};
    r.p[4] = f2v{__builtin_fmaf(-o.z, inv.z, mz), 0.0f};
    return r;
}

// {a.x b[BH] + c[CH], a.y b[BH] + c[CH]}: two IEEE fmas (v_pk_fma_f32), b and c broadcast
// from half BH / CH of their pairs
template <int BH, int CH>
__device__ __forceinline__ f2v pk_fma_bc(f2v a, f2v b, f2v c) {
    f2v r;
    if constexpr (BH == 0 && CH == 0)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else if constexpr (BH == 0 && CH == 1)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else if constexpr (BH == 1 && CH == 0)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int W>
struct WideNodeF {
    uint4 h;
    float en[3][W], ex[3][W];  // the ray's entry run (lo for 1 / d >= 0, else hi) and exit run per axis
};

// Per-lane byte offsets of the entry and exit runs of each axis (as wide_offsets: one
// select per axis, the exit run by a subtraction; the constant 16 + 8 W a is left to the
// loads' offset fields).
template <int W>
__device__ __forceinline__ void wide_offsets_f32(uint32_t nb, const unsigned long long (&neg)[3], uint32_t (&en)[3],
                                                 uint32_t (&ex)[3]) {
    const uint32_t nb2 = nb + 4u * W;
    const uint32_t both = nb + nb2;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const uint32_t e = lane_sel(nb, nb2, neg[a]);
        en[a] = e;
        ex[a] = both - e;
    }
}

template <int W>
__device__ __forceinline__ WideNodeF<W> load_wide_node_f32_lds(const char* __restrict__ base, uint32_t nb,
                                                             const uint32_t (&en)[3], const uint32_t (&ex)[3]) {
    WideNodeF<W> n;
    n.h = *reinterpret_cast<const uint4*>(base + nb);
#pragma unroll
    for (int a = 0; a < 3; a++) {
#pragma unroll
        for (int i = 0; i < W; i += 4) {
            const float4 e = *reinterpret_cast<const float4*>(base + en[a] + 16 + 8 * W * a + 4 * i);
            const float4 x = *reinterpret_cast<const float4*>(base + ex[a] + 16 + 8 * W * a + 4 * i);
            n.en[a][i] = e.x, n.en[a][i + 1] = e.y, n.en[a][i + 2] = e.z, n.en[a][i + 3] = e.w;
            n.ex[a][i] = x.x, n.ex[a][i + 1] = x.y, n.ex[a][i + 2] = x.z, n.ex[a][i + 3] = x.w;
        }
    }
    return n;
}

template <int W>
__device__ __forceinline__ WideNodeF<W> load_wide_node_f32_buf(__amdgpu_buffer_rsrc_t r, uint32_t nb,
                                                             const uint32_t (&en)[3], const uint32_t (&ex)[3]) {
    WideNodeF<W> n;
    const auto h = __builtin_amdgcn_raw_buffer_load_b128(r, nb, 0, 0);
    n.h = make_uint4(h[0], h[1], h[2], h[3]);
#pragma unroll
    for (int a = 0; a < 3; a++) {
#pragma unroll
        for (int i = 0; i < W; i += 4) {
            const auto e = __builtin_amdgcn_raw_buffer_load_b128(r, en[a] + (uint32_t)(16 + 8 * W * a + 4 * i), 0, 0);
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, ex[a], 16 + 8 * W * a + 4 * i, 0);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                n.en[a][i + k] = __uint_as_float(e[k]);
                n.ex[a][i + k] = __uint_as_float(x[k]);
            }
        }
    }
    return n;
}

template <int W>
__device__ __forceinline__ WideHits<W> wide_node_test_f32(const WideNodeF<W>& nd, const WideRay& wr) {
    uint32_t fbits[W];
#pragma unroll
    for (int j = 0; j < W; j += 2) {
        const f2v enx = pk_fma_bc<0, 1>(f2v{nd.en[0][j], nd.en[0][j + 1]}, wr.p[0], wr.p[1]);
        const f2v eny = pk_fma_bc<1, 0>(f2v{nd.en[1][j], nd.en[1][j + 1]}, wr.p[0], wr.p[2]);
        const f2v enz = pk_fma_bc<0, 1>(f2v{nd.en[2][j], nd.en[2][j + 1]}, wr.p[1], wr.p[2]);
        const f2v exx = pk_fma_bc<0, 0>(f2v{nd.ex[0][j], nd.ex[0][j + 1]}, wr.p[0], wr.p[3]);
        const f2v exy = pk_fma_bc<1, 1>(f2v{nd.ex[1][j], nd.ex[1][j + 1]}, wr.p[0], wr.p[3]);
        const f2v exz = pk_fma_bc<0, 0>(f2v{nd.ex[2][j], nd.ex[2][j + 1]}, wr.p[1], wr.p[4]);
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const float tmin3 = __builtin_fmaxf(__builtin_fmaxf(enx[c], eny[c]), enz[c]);
            const float tmax = __builtin_fminf(__builtin_fminf(exx[c], exy[c]), exz[c]);
            fbits[j + c] = box_fail_bits(tmin3, tmax);
        }
    }
    uint32_t fail = 0;
#pragma unroll
    for (int j = W - 1; j >= 0; j--) fail = shl1_add_sign(fail, fbits[j]);
    const uint32_t hd = nd.h.x;
    const uint32_t ni = (hd >> 24) & 15u, nl = hd >> 28;
    const uint32_t hits = ~fail & ((1u << (ni + nl)) - 1u);
    return WideHits<W>{hits & ((1u << ni) - 1u), hits >> ni, hd & 0xffffffu, nd.h.y, nd.h.z, nd.h.w};
}

// Triangle range of leaf k of a node: [leaf_base + end[k - 1], leaf_base + end[k]).
template <int W>
__device__ __forceinline__ void wide_leaf_range(const WideHits<W>& h, int k, int& first, int& count) {
    const uint32_t ends = k < 4 ? h.ends_lo : h.ends_hi;
    const int end = (int)((ends >> (8 * (k & 3))) & 255u);
    int begin = 0;
    if (k > 0) {
        const uint32_t pe = (k - 1) < 4 ? h.ends_lo : h.ends_hi;
        begin = (int)((pe >> (8 * ((k - 1) & 3))) & 255u);
    }
    first = (int)h.leaf_base + begin;
    count = end - begin;
}

// One triangle of a wide leaf against a ray (the queue's test). A hit counts only if the
// leaf's EXACT box passes the reference's slab test too (aabb.h:20-29; inv finite, so the
// IEEE form is exact, pt_math.h): with the conservative node test that makes the set of
// counted hits exactly the reference's. Reduces (t bits, rank) into *slot.
// fast: tri_hit_nb (branch-free; the lanes of a drain round test different (ray,
// triangle) pairs, so tri_hit's early exits rarely skip work for the whole wave).
// inv: the ray's 1 / d (bvh.h:157), as its owner lane computed it for the walk.
__device__ __forceinline__ void wide_tri_test(const float4* __restrict__ wtris, int i, v3 o, v3 d, v3 inv,
                                              unsigned long long* slot, bool fast, bool compact) {
    float tt;
    if (compact) {
        // {v1, rank} {v2, v3.x} {v3.yz}: e1 = v2 - v1, e2 = v3 - v1 as triangle.h:28 forms
        // them; the leaf's box (one triangle: its AABB, aabb.h:16-19) is the vertices'
        // component min / max, equal to the reference's as real numbers (all the slab test
        // depends on: slab_hit_finite)
        const float4 t0 = wtris[3 * i], t1 = wtris[3 * i + 1], t2 = wtris[3 * i + 2];
        const v3 v1{t0.x, t0.y, t0.z}, v2{t1.x, t1.y, t1.z}, v3_{t1.w, t2.x, t2.y};
        const v3 e1 = sub(v2, v1), e2 = sub(v3_, v1);
        const bool h = fast ? tri_hit_nb(v1, e1, e2, o, d, tt) : tri_hit(v1, e1, e2, o, d, tt);
#ifdef PT_EXP_DUP_TRI  // measurement only: the triangle test once more
        {
            v3 o2 = o;
            asm volatile("" : "+v"(o2.x));
            float t2;
            const bool h2 = fast ? tri_hit_nb(v1, e1, e2, o2, d, t2) : tri_hit(v1, e1, e2, o2, d, t2);
            asm volatile("" ::"v"(t2), "v"((int)h2));
        }
#endif
        if (h && tt < 1e30f) {
            const v3 lb{__builtin_fminf(__builtin_fminf(v1.x, v2.x), v3_.x),
                        __builtin_fminf(__builtin_fminf(v1.y, v2.y), v3_.y),
                        __builtin_fminf(__builtin_fminf(v1.z, v2.z), v3_.z)};
            const v3 rt{__builtin_fmaxf(__builtin_fmaxf(v1.x, v2.x), v3_.x),
                        __builtin_fmaxf(__builtin_fmaxf(v1.y, v2.y), v3_.y),
                        __builtin_fmaxf(__builtin_fmaxf(v1.z, v2.z), v3_.z)};
#ifdef PT_EXP_DUP_XBOX  // measurement only: a hit's exact leaf-box check once more
            {
                v3 o2 = o;
                asm volatile("" : "+v"(o2.x));
                const bool x2 = slab_hit_finite(lb, rt, o2, inv);
                asm volatile("" ::"v"((int)x2));
            }
#endif
            if (slab_hit_finite(lb, rt, o, inv))
                atomicMin(slot, ((unsigned long long)__float_as_uint(tt) << 32) | (unsigned long long)__float_as_uint(t0.w));
        }
        return;
    }
    // the exact leaf box (t2.zw, t3) is loaded with the triangle: a hit round then waits for
    // one memory trip, not two
    const float4 t0 = wtris[4 * i], t1 = wtris[4 * i + 1], t2 = wtris[4 * i + 2], t3 = wtris[4 * i + 3];
    const v3 v1{t0.x, t0.y, t0.z}, e1{t0.w, t1.x, t1.y}, e2{t1.z, t1.w, t2.x};
    const bool h = fast ? tri_hit_nb(v1, e1, e2, o, d, tt) : tri_hit(v1, e1, e2, o, d, tt);
    if (h && tt < 1e30f) {
        if (slab_hit_finite(v3{t2.z, t2.w, t3.x}, v3{t3.y, t3.z, t3.w}, o, inv))
            atomicMin(slot, ((unsigned long long)__float_as_uint(tt) << 32) | (unsigned long long)__float_as_uint(t2.y));
    }
}

// Drain the wave's triangle queue: 64 entries per round, one per lane, the owner's ray
// (o, d and the 1 / d it walks with, so the exact leaf-box check of a hit needs no
// divisions here) by ds_bpermute; all lanes call it. `all`: drain completely, else only
// full rounds. Entries: kSingle (every leaf holds one triangle) one word, triangle << 6 |
// owner lane; else two words, (first triangle, owner lane << 26 | count - 1). The two
// forms are separate loops, so neither carries the other's registers.
template <bool kSingle>
__device__ __forceinline__ void wide_queue_drain_t(const uint32_t* __restrict__ wq, int& qn, bool all,
                                                   const float4* __restrict__ wtris,
                                                   unsigned long long* __restrict__ wbest, int lane, v3 o, v3 d,
                                                   v3 inv, bool fast, bool compact, unsigned long long& n_rounds,
                                                   unsigned long long& n_ents) {
    while (qn >= kWave || (all && qn > 0)) {
        const int base = qn > kWave ? qn - kWave : 0;
        n_rounds += 1;  // diagnostic counts (PT_STAMPS builds; dead code otherwise)
        n_ents += (unsigned long long)(qn - base);
        const bool valid = lane < qn - base;
        int first, owner;
        uint32_t cnt = 0u;
        if constexpr (kSingle) {
            const uint32_t e = valid ? wq[base + lane] : 0u;
            first = (int)(e >> 6);
            owner = (int)(e & 63u);
        } else {
            const uint2 e = valid ? reinterpret_cast<const uint2*>(wq)[base + lane] : make_uint2(0u, 0u);
            first = (int)e.x;
            owner = (int)(e.y >> 26);
            cnt = e.y & 0x3ffffffu;
        }
        const int addr = owner << 2;
        const v3 ro{lane_float(addr, o.x), lane_float(addr, o.y), lane_float(addr, o.z)};
        const v3 rd{lane_float(addr, d.x), lane_float(addr, d.y), lane_float(addr, d.z)};
        const v3 ri{lane_float(addr, inv.x), lane_float(addr, inv.y), lane_float(addr, inv.z)};
#ifdef PT_EXP_DUP_DRAINQ  // measurement only: the round's queue read and owner fetches once more
        {
            int b2 = base;
            asm volatile("" : "+v"(b2));
            const uint32_t e2 = valid ? wq[(b2 + lane) * (kSingle ? 1 : 2)] : 0u;
            const int a2 = (int)(e2 & 63u) << 2;
            const float f0 = lane_float(a2, o.x), f1 = lane_float(a2, o.y), f2 = lane_float(a2, o.z);
            const float f3 = lane_float(a2, d.x), f4 = lane_float(a2, d.y), f5 = lane_float(a2, d.z);
            const float f6 = lane_float(a2, inv.x), f7 = lane_float(a2, inv.y), f8 = lane_float(a2, inv.z);
            asm volatile("" ::"v"(f0), "v"(f1), "v"(f2), "v"(f3), "v"(f4), "v"(f5), "v"(f6), "v"(f7), "v"(f8));
        }
#endif
        if (valid) {
            if constexpr (kSingle) {
                wide_tri_test(wtris, first, ro, rd, ri, wbest + owner, fast, compact);
            } else {
                const int last = first + (int)cnt;
                for (int i = first; i <= last; i++) wide_tri_test(wtris, i, ro, rd, ri, wbest + owner, fast, compact);
            }
        }
        qn = base;
    }
}

__device__ __forceinline__ void wide_queue_drain(const uint32_t* __restrict__ wq, int& qn, bool all,
                                                 const float4* __restrict__ wtris,
                                                 unsigned long long* __restrict__ wbest, int lane, v3 o, v3 d,
                                                 v3 inv, bool fast, bool single, bool compact,
                                                 unsigned long long& n_rounds, unsigned long long& n_ents) {
    if (PT_PRIO_DRAIN) __builtin_amdgcn_s_setprio(PT_PRIO_DRAIN);
    wave_lds_sync();
    if (single) wide_queue_drain_t<true>(wq, qn, all, wtris, wbest, lane, o, d, inv, fast, compact, n_rounds, n_ents);
    else wide_queue_drain_t<false>(wq, qn, all, wtris, wbest, lane, o, d, inv, fast, compact, n_rounds, n_ents);
    wave_lds_sync();
    if (PT_PRIO_DRAIN) __builtin_amdgcn_s_setprio(0);
}

// One wide-walk step for the lanes with `on` (all 64 lanes call it): test the current
// node's children, queue the triangles of its passing leaves (wave prefix sum of the
// entry counts; a step whose entries exceed the queue tests them per lane), then move to
// the first passing inner child or pop the stack. Stack entry: child_base << 8 | the
// node's passing inner slots not yet taken. Returns true for an `on` lane whose walk is
// complete. Node `cur` < A.wide_top is read from the block's LDS copy of the top levels.
#ifndef PT_WIDE_LDS_TOP
#define PT_WIDE_LDS_TOP 1  // 0: every node read from global memory (A/B hook; the LDS copy is then unused)
#endif
template <int W, int kPF>
__device__ __forceinline__ bool wide_step_q(const TraceArgs& A, const uint4* __restrict__ top,
                                            int* __restrict__ stk, int tid, int lane, bool on, v3 o, v3 d,
                                            v3 inv, const WideRay& wr, const unsigned long long (&neg)[3], int& cur,
                                            int& sp, uint32_t* __restrict__ wq, int& qn, int qcap,
                                            unsigned long long* __restrict__ wbest, unsigned long long& n_rounds,
                                            unsigned long long& n_ents) {
    constexpr bool kF16 = kPF == 1;
    constexpr int NU = kNodeU4<W, kPF>;
    // only the masks need a value on lanes that are not stepping (the bases and leaf ends
    // are read only under a set bit): no register moves for the rest
    WideHits<W> h;
    h.inner = 0u;
    h.leaf = 0u;
    if (on && kPF == 2) {
        const uint32_t nb = (uint32_t)cur * (16u * NU);  // < 2^31: at most 2^24 nodes
        uint32_t en[3], ex[3];
        wide_offsets_f32<W>(nb, neg, en, ex);
        WideNodeF<W> nd;
        if (PT_WIDE_LDS_TOP && cur < A.wide_top) {
            nd = load_wide_node_f32_lds<W>(reinterpret_cast<const char*>(top), nb, en, ex);
        } else {
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint4*>(A.wide), (short)0, (int)(A.wide_nodes * 16u * NU), 0x00020000);
            nd = load_wide_node_f32_buf<W>(r, nb, en, ex);
        }
        h = wide_node_test_f32<W>(nd, wr);
#ifdef PT_EXP_DUP_NODE  // measurement only: the node test once more (its VALU cost by difference)
        {
            WideRay w2 = wr;
            asm volatile("" : "+v"(w2.p[0]));
            const WideHits<W> h2 = wide_node_test_f32<W>(nd, w2);
            asm volatile("" ::"v"(h2.inner), "v"(h2.leaf));
        }
#endif
    } else if (on) {
        const uint32_t nb = (uint32_t)cur * (16u * NU);  // < 2^31: at most 2^24 nodes
        const WideOff<W, kF16> off = wide_offsets<W, kF16>(nb, neg);
#ifdef PT_EXP_DUP_OFFS  // measurement only: the node's load offsets once more
        {
            int c2 = cur;
            asm volatile("" : "+v"(c2));
            const WideOff<W, kF16> o2 = wide_offsets<W, kF16>((uint32_t)c2 * (16u * NU), neg);
            asm volatile("" ::"v"(o2.en[0]), "v"(o2.en[1]), "v"(o2.en[2]), "v"(o2.ex[0]), "v"(o2.ex[1]), "v"(o2.ex[2]));
        }
#endif
        WideNode<W, kF16> nd;
        if (PT_WIDE_LDS_TOP && cur < A.wide_top) {
            nd = load_wide_node_lds<W, kF16>(reinterpret_cast<const char*>(top), nb, off);
        } else {
            // num_records: the tree's bytes (< 2^31); a load past it would read zeros
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint4*>(A.wide), (short)0, (int)(A.wide_nodes * 16u * NU), 0x00020000);
            nd = load_wide_node_buf<W, kF16>(r, nb, off);
        }
        h = wide_node_test<W, kF16>(nd, o, inv);
#ifdef PT_EXP_DUP_NODE  // measurement only: the node test once more (its VALU cost by difference)
        {
            v3 o2 = o;
            asm volatile("" : "+v"(o2.x));
            const WideHits<W> h2 = wide_node_test<W, kF16>(nd, o2, inv);
            asm volatile("" ::"v"(h2.inner), "v"(h2.leaf));
        }
#endif
    }
    const uint32_t c = (uint32_t)__popc(h.leaf);
    const uint32_t incl = wave_incl_scan(c);
    const int total = __builtin_amdgcn_readlane((int)incl, 63);
#ifdef PT_EXP_DUP_SCAN  // measurement only: the step's popcount + wave prefix sum once more
    {
        uint32_t l2 = h.leaf;
        asm volatile("" : "+v"(l2));
        const uint32_t i2 = wave_incl_scan((uint32_t)__popc(l2));
        const int t2 = __builtin_amdgcn_readlane((int)i2, 63);
        asm volatile("" ::"v"(i2), "s"(t2));
    }
#endif
    if (total > 0) {
        if (qn + total > qcap)
            wide_queue_drain(wq, qn, true, A.wtris, wbest, lane, o, d, inv, A.tri_fast != 0, A.wide_single != 0,
                             A.wide_compact != 0, n_rounds, n_ents);
        uint32_t lm = h.leaf;
        if (total <= qcap) {
            uint32_t at = (uint32_t)qn + incl - c;
            if (A.wide_single) {  // leaf k's one triangle is leaf_base + k: no range decode, one word
#ifdef PT_EXP_DUP_ENQ  // measurement only: the enqueue loop once more (the same entries written twice)
                {
                    uint32_t l2 = lm, at2 = at;
                    asm volatile("" : "+v"(l2), "+v"(at2));
                    while (l2) {
                        const int k = __builtin_ctz(l2);
                        l2 &= l2 - 1;
                        wq[at2++] = ((h.leaf_base + (uint32_t)k) << 6) | (uint32_t)lane;
                    }
                    asm volatile("" ::: "memory");
                }
#endif
                while (lm) {
                    const int k = __builtin_ctz(lm);
                    lm &= lm - 1;
                    wq[at++] = ((h.leaf_base + (uint32_t)k) << 6) | (uint32_t)lane;
                }
            } else {
                uint2* wq2 = reinterpret_cast<uint2*>(wq);
                while (lm) {
                    const int k = __builtin_ctz(lm);
                    lm &= lm - 1;
                    int first, count;
                    wide_leaf_range<W>(h, k, first, count);
                    wq2[at++] = make_uint2((uint32_t)first, ((uint32_t)lane << 26) | (uint32_t)(count - 1));
                }
            }
            qn += total;
        } else {  // more entries than the queue holds: this lane tests its own (exact either way)
            while (lm) {
                const int k = __builtin_ctz(lm);
                lm &= lm - 1;
                int first, count;
                wide_leaf_range<W>(h, k, first, count);
                for (int i = first; i < first + count; i++)
                    wide_tri_test(A.wtris, i, o, d, inv, wbest + lane, A.tri_fast != 0, A.wide_compact != 0);
            }
        }
    }
    if (!on) return false;
#ifdef PT_EXP_DUP_STACK  // measurement only: the push / pop decisions once more (same stack writes)
    {
        uint32_t in2 = h.inner;
        int sp2 = sp;
        asm volatile("" : "+v"(in2), "+v"(sp2));
        int cur2 = 0;
        if (in2) {
            const uint32_t rest = in2 & (in2 - 1);
            if (rest) stk[sp2 * kBlock + tid] = (int)((h.child_base << 8) | rest);
            cur2 = (int)h.child_base + __builtin_ctz(in2);
        } else if (sp2 > 0) {
            const uint32_t e = (uint32_t)stk[(sp2 - 1) * kBlock + tid];
            cur2 = (int)(e >> 8) + __builtin_ctz(e & 255u);
        }
        asm volatile("" ::"v"(cur2) : "memory");
    }
#endif
    if (h.inner) {
        const int j = __builtin_ctz(h.inner);
        const uint32_t rest = h.inner & (h.inner - 1);
        if (rest) {
            stk[sp * kBlock + tid] = (int)((h.child_base << 8) | rest);
            sp++;
        }
        cur = (int)h.child_base + j;
        return false;
    }
    if (sp == 0) return true;
    const uint32_t e = (uint32_t)stk[(sp - 1) * kBlock + tid];
    uint32_t m = e & 255u;
    const int j = __builtin_ctz(m);
    m &= m - 1;
    if (m) stk[(sp - 1) * kBlock + tid] = (int)((e & ~255u) | m);
    else sp--;
    cur = (int)(e >> 8) + j;
    return false;
}
#endif  // PT_FLAT_ONLY

// ---- pieces of the path loop shared by the megakernel bodies

// Wave-private pool of work items [next, end), refilled kChunk items at a time by one
// atomic: a single global counter saturates near 88 returning atomics/us
// (MI355X_MICROARCH.md, row "dequeue"), which one claim per wave-iteration reaches.
// Every wave starts with a static range of items (no atomic): a launch's ~7k waves would
// otherwise all queue on the counter at once (~80 us), and a small launch (config 1: 1M
// items, 64-item refills) would spend most of its time in that queue.
// Item numbers fit 32 bits: total_items < 2^31 (host check) and the head passes the end by
// at most one claim per wave (< 2^24 items), so the pool is held in two 32-bit registers.
struct Pool {
    uint32_t next = 0, end = 0;
    uint32_t acc_left = 0;  // refills until the next fused accumulation chunk (its cadence)
};

__device__ __forceinline__ Pool pool_start(const TraceArgs& A) {
    const uint32_t w = blockIdx.x * (uint32_t)(kBlock / kWave) + (threadIdx.x >> 6);
    Pool p;
    p.next = w * A.static_items;
    p.end = p.next + A.static_items;
    p.acc_left = (uint32_t)A.acc_every;
    return p;
}

// The kernel arguments re-read from the kernarg segment (one TraceArgs at offset 0): the
// fused accumulation's fields are loaded where they are used instead of being held in
// SGPRs for the whole megakernel (they would push other arguments into VGPR spill lanes).
__device__ __forceinline__ const __attribute__((address_space(4))) TraceArgs* kernarg_args() {
    const __attribute__((address_space(4))) TraceArgs* K =
        (const __attribute__((address_space(4))) TraceArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(K));
    return K;
}

// Radiance slab layout: [sample][pixel][rgb], one 12-B record per sample (a finished path
// stores it with one instruction; the [rgb][sample][pixel] planes of rounds 1-3 took three:
// +0.1-0.5 %, profiles/r04_slab_rgb). Sample s of pixel q:
__device__ __forceinline__ float3 slab_at(const float* __restrict__ src, size_t s, uint32_t q, uint32_t npix) {
    return *reinterpret_cast<const float3*>(src + 3 * (s * npix + q));
}
// The flag word of a flagged slab (TraceArgs::flags) holding sample s (of the launch) of pixel
// q: pixel-major within groups of 32 samples (bit s & 31).
__device__ __forceinline__ size_t flag_word(uint32_t s, uint32_t q, uint32_t npix) {
    return (size_t)(s >> 5) * npix + q;
}

// Pixel q's samples [0, n) of a slab added to (x, y, z) in sample order (image.h:27-31: sum =
// sum + sample); with flags, only the flagged records (the others are +0, §TraceArgs::flags).
// Pixel-major bits (pm): one flag word per 32 samples, then its set bits' records read and
// added in order; kParallel (the separate pass, pt_accumulate_kernel: a frame of few pixels —
// one rank's share — is latency-bound there) loads 8 words and up to 8 records at once.
// Sample-major bits: kDepth samples' bits gathered into a mask (one load each), then the set
// ones' records read and added in order (kParallel: 32 samples, all their records at once;
// inside the trace kernels, whose registers are spoken for: 8, one record at a time).
template <bool kParallel = false>
__device__ __forceinline__ void slab_sum(const float* __restrict__ src, const uint32_t* __restrict__ flags, int pm,
                                         int n, uint32_t q, uint32_t npix, float& x, float& y, float& z) {
    int s = 0;
    if (flags && pm) {
        const int nw = (n + 31) >> 5;  // bits of samples >= n are never set
        int g = 0;
        if constexpr (kParallel) {
            for (; g + 8 <= nw; g += 8) {
                uint32_t m[8];
#pragma unroll
                for (int j = 0; j < 8; j++) m[j] = flags[flag_word((uint32_t)(g + j) << 5, q, npix)];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    // 64 samples: up to 8 flagged records loaded at once (a lane's lot is ~1),
                    // then added in sample order; a slot past the lane's last record adds +0,
                    // which changes no running sum (§TraceArgs::flags)
                    unsigned long long mm = (unsigned long long)m[2 * h + 1] << 32 | m[2 * h];
                    const int base = (g + 2 * h) << 5;
                    while (mm) {
                        float3 v[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            v[k] = make_float3(0.0f, 0.0f, 0.0f);
                            if (mm) {
                                const int b = __builtin_ctzll(mm);
                                mm &= mm - 1;
                                v[k] = slab_at(src, (size_t)(base + b), q, npix);
                            }
                        }
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            x += v[k].x;
                            y += v[k].y;
                            z += v[k].z;
                        }
                    }
                }
            }
        }
        for (; g < nw; g++) {
            uint32_t m = flags[flag_word((uint32_t)g << 5, q, npix)];
            while (m) {
                const int b = __builtin_ctz(m);
                m &= m - 1;
                const float3 v = slab_at(src, (size_t)((g << 5) + b), q, npix);
                x += v.x;
                y += v.y;
                z += v.z;
            }
        }
        return;
    }
    if (flags) {
        constexpr int kDepth = kParallel ? 32 : 8;
        for (; s + kDepth <= n; s += kDepth) {
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < kDepth; j++) {
                const size_t i = (size_t)(s + j) * npix + q;
                m |= ((flags[i >> 5] >> (uint32_t)(i & 31)) & 1u) << j;
            }
            if constexpr (kParallel) {
                // every flagged record of the group loaded at once (one more round trip per
                // group, not one per record), then added in sample order
                if (m) {
                    float3 v[kDepth];
#pragma unroll
                    for (int j = 0; j < kDepth; j++)
                        if ((m >> j) & 1u) v[j] = slab_at(src, (size_t)(s + j), q, npix);
#pragma unroll
                    for (int j = 0; j < kDepth; j++)
                        if ((m >> j) & 1u) {
                            x += v[j].x;
                            y += v[j].y;
                            z += v[j].z;
                        }
                }
            } else {
                while (m) {
                    const int j = __builtin_ctz(m);
                    m &= m - 1;
                    const float3 v = slab_at(src, (size_t)(s + j), q, npix);
                    x += v.x;
                    y += v.y;
                    z += v.z;
                }
            }
        }
        for (; s < n; s++) {
            const size_t i = (size_t)s * npix + q;
            if ((flags[i >> 5] >> (uint32_t)(i & 31)) & 1u) {
                const float3 v = slab_at(src, (size_t)s, q, npix);
                x += v.x;
                y += v.y;
                z += v.z;
            }
        }
        return;
    }
    for (; s + 4 <= n; s += 4) {  // 4 samples' loads in flight, added in sample order
        float3 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = slab_at(src, (size_t)(s + j), q, npix);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            x += v[j].x;
            y += v[j].y;
            z += v[j].z;
        }
    }
    for (; s < n; s++) {
        const float3 v = slab_at(src, (size_t)s, q, npix);
        x += v.x;
        y += v.y;
        z += v.z;
    }
}

// One chunk of the fused accumulation: pixels [64 c, 64 c + 64) of the previous batch's
// slab added into the running sum in sample order, exactly pt_accumulate_kernel's
// arithmetic (image.h:27-31: sum = sum + sample, sample by sample) without its /spp (the
// last batch always goes through pt_accumulate_kernel). A pixel's chunk runs in exactly
// one launch, after the launch that wrote its slab, so the order of the sums is the
// reference's. Wave-uniform: all 64 lanes call. Returns false once no chunk is left.
__device__ __forceinline__ bool fused_accumulate_chunk(int lane) {
#ifdef PT_EXP_NO_ACC  // timing experiment only (wrong images): no fused accumulation
    return false;
#endif
    const auto* K = kernarg_args();
    unsigned long long c = 0;
    if (lane == 0) c = atomicAdd(K->ctr + 2, 1ull);
    c = __builtin_amdgcn_readfirstlane((uint32_t)c);
    if (c >= (unsigned long long)K->acc_chunks) return false;
    const uint32_t npix = (uint32_t)K->npix, q = (uint32_t)c * kWave + (uint32_t)lane;
    if (q < npix) {
        float* __restrict__ sum = K->acc_sum;
        const float* __restrict__ src = K->acc_src;
        const int n = K->acc_count;
        float x = 0.0f, y = 0.0f, z = 0.0f;
        if (!K->acc_first) {
            x = sum[q];
            y = sum[npix + q];
            z = sum[2 * (size_t)npix + q];
        }
        slab_sum(src, K->acc_flags, K->flags_pm, n, q, npix, x, y, z);
        sum[q] = x;
        sum[npix + q] = y;
        sum[2 * (size_t)npix + q] = z;
    }
    return true;
}

// After a refill of the work pool: every acc_every-th refill of a wave runs one chunk of
// the fused accumulation, so the previous batch's slab is summed while this one traces
// (HBM reads under VALU-bound tracing) rather than in a separate pass between launches.
__device__ __forceinline__ void after_refill(const TraceArgs& A, int lane, Pool& pool) {
    if (A.acc_chunks > 0 && --pool.acc_left == 0) {  // every acc_every-th refill (a countdown, no division)
        pool.acc_left = (uint32_t)A.acc_every;
        fused_accumulate_chunk(lane);
    }
}

// Before a wave exits: the chunks nobody has taken yet.
__device__ __forceinline__ void drain_accumulate(const TraceArgs& A, int lane) {
    if (A.acc_chunks > 0)
        while (fused_accumulate_chunk(lane)) {
        }
}

// Give every lane with `need` its next work item (q = pixel of the part, samples
// [s, s_end)); lanes past the last item get alive = false. Wave-uniform: all lanes call.
__device__ __forceinline__ void claim_work(const TraceArgs& A, int lane, bool need, Pool& pool, bool& alive, int& q,
                                           int& s, int& s_end) {
    const unsigned long long want = __ballot(need);
    if (want == 0ull) return;
    const uint32_t cnt = (uint32_t)__popcll(want);
    const uint32_t avail = pool.end - pool.next;
    uint32_t fresh = 0;
    if (avail < cnt) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(A.work, (unsigned long long)A.chunk);
        fresh = (uint32_t)A.static_base + __builtin_amdgcn_readfirstlane((uint32_t)b);
    }
    if (need) {
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
        const uint32_t item = rank < avail ? pool.next + rank : fresh + (rank - avail);
        if (item >= (uint32_t)A.total_items) {
            alive = false;
        } else {
            const uint32_t blk = fdiv(item, A.div_npix);
            q = (int)(item - blk * (uint32_t)A.npix);
            s = A.s_begin + (int)blk * A.per_item;
            s_end = min(s + A.per_item, A.s_begin + A.s_count);
        }
    }
    if (avail < cnt) {
        pool.next = fresh + (cnt - avail);
        pool.end = fresh + (uint32_t)A.chunk;
        after_refill(A, lane, pool);
    } else {
        pool.next += cnt;
    }
}

// claim_work for one-sample items (flat kernel; the host sets per_item = 1): each lane
// with `need` gets an item index, which is also its sample's slab offset
// (slab_index); lanes past the last item get alive = false.
__device__ __forceinline__ void claim_item(const TraceArgs& A, int lane, bool need, Pool& pool, bool& alive,
                                           uint32_t& item_out) {
    const unsigned long long want = __ballot(need);
    if (want == 0ull) return;
    const uint32_t cnt = (uint32_t)__popcll(want);
    const uint32_t avail = pool.end - pool.next;
    uint32_t fresh = 0;
    if (avail < cnt) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(A.work, (unsigned long long)A.chunk);
        fresh = (uint32_t)A.static_base + __builtin_amdgcn_readfirstlane((uint32_t)b);
    }
    if (need) {
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
        const uint32_t item = rank < avail ? pool.next + rank : fresh + (rank - avail);
        if (item >= (uint32_t)A.total_items) alive = false;
        else item_out = item;  // total_items < 2^31 (host check)
    }
    if (avail < cnt) {
        pool.next = fresh + (cnt - avail);
        pool.end = fresh + (uint32_t)A.chunk;
        after_refill(A, lane, pool);
    } else {
        pool.next += cnt;
    }
}

// camera.h:63-73 with the per-sample reseed of pt_sample_seed
#ifndef PT_CAM_KERNARG
#define PT_CAM_KERNARG 1  // 0: camera fields from the kernel's argument registers (A/B hook)
#endif
// The camera's fields are read from the kernarg segment here (scalar loads at the use)
// rather than held in SGPRs across the megakernel loop, where they pushed other uniform
// values into VGPR spill lanes (each reload a v_readlane on the VALU).
__device__ __forceinline__ void camera_ray(const TraceArgs& A, int q, int s, Lcg& g, v3& o, v3& d) {
    const auto* K = PT_CAM_KERNARG ? kernarg_args() : nullptr;
    const TraceArgs& C = PT_CAM_KERNARG ? *(const TraceArgs*)K : A;
    const int r = (int)fdiv((uint32_t)q, C.div_w);
    const int px = q - r * C.W;
    const int py = part_row(C, r);
    g.s = pt_sample_seed((uint32_t)(py * C.W + px), (uint32_t)s, C.seed);
    const float jy = g.next01();  // g++ evaluates the y argument first
    const float jx = g.next01();
    const float cx = ((float)px + jx) * C.cell - C.half_vres_x;
    const float cy = ((float)py + jy) * C.cell - C.half_vres_y;
    // the z term (-distance) * column z is the same float product for every ray: the host
    // forms it (uniform operands stay in SGPRs instead of taking VGPRs)
    d = normalize_fast(v3{cx * C.col0_x + cy * C.col0_y + C.cz_col0, cx * C.col1_x + cy * C.col1_y + C.cz_col1,
                     cx * C.col2_x + cy * C.col2_y + C.cz_col2});
    o = v3{C.pos_x, C.pos_y, C.pos_z};
}

// trace() after BVH::intersect (render.h:41-57) for segment k of the path. Returns
// true when the path ends here (L = this segment's radiance); otherwise records
// (tri, cos) for the fold and moves (o, d) to the next segment.
// kSpecular = false: the scene has no SPECULAR material (hipRTC kernels know the scene),
// so the specular sampler is not compiled in.
// kIds: `tris` is the wide path's nrm array ({n.xyz, material id} per triangle) and `mats`
// the distinct-material table; the path record then holds the material row, not the
// triangle (finish_path reads the same table). Otherwise mats/tris are per triangle.
template <bool kSpecular = true, typename RecT = int, bool kIds = false>
__device__ __forceinline__ bool shade(const TraceArgs& A, const float4* __restrict__ mats,
                                      const float4* __restrict__ tris, RecT* __restrict__ rec_tri,
                                      float* __restrict__ rec_cos, int tid, int hit, float t, Lcg& g, v3& o, v3& d,
                                      int& k, v3& L) {
    L = v3{0.0f, 0.0f, 0.0f};
    if (hit < 0) return true;  // miss -> 0 (also depth <= 0)
#ifdef PT_EXP_DUP_SHADE  // measurement only: the hit record and material reads, face-forward and hit point once more
    {
        int h2 = hit;
        asm volatile("" : "+v"(h2));
        const float4 tn2 = kIds ? tris[h2] : tris[3 * h2 + 2];
        const int row2 = kIds ? __float_as_int(tn2.w) : h2;
        const float4 m02 = mats[2 * row2], m12 = mats[2 * row2 + 1];
        v3 n2 = kIds ? v3{tn2.x, tn2.y, tn2.z} : v3{tn2.y, tn2.z, tn2.w};
        if (!(dot(n2, d) < 0.0f)) n2 = neg(n2);
        const v3 hp2 = add(o, scale(d, t));
        asm volatile("" ::"v"(m02.x), "v"(m12.x), "v"(hp2.x), "v"(hp2.y), "v"(hp2.z), "v"(n2.x), "v"(n2.y), "v"(n2.z));
    }
#endif
    float4 tn;
    int row = hit;
    if constexpr (kIds) {
        tn = tris[hit];
        row = __float_as_int(tn.w);
    }
    const float4 m0 = mats[2 * row], m1 = mats[2 * row + 1];
    const int type = __float_as_int(m0.x);
    if (type == PT_MAT_EMIT) {
        L = v3{m1.x, m1.y, m1.z};
        return true;
    }
    if (k + 1 >= A.depth) {
        // Last segment: trace(depth-1 == 0) returns 0, so the result is
        // emission + ((2*0)*albedo)*cos; the BRDF draw only advanced the
        // per-sample stream, which ends here.
        L = v3{m1.x + 0.0f * m0.y, m1.y + 0.0f * m0.z, m1.z + 0.0f * m0.w};
        return true;
    }
    v3 n;
    if constexpr (kIds) {
        n = v3{tn.x, tn.y, tn.z};
    } else {
        tn = tris[3 * hit + 2];
        n = v3{tn.y, tn.z, tn.w};
    }
    if (!(dot(n, d) < 0.0f)) n = neg(n);  // triangle.h:48
    const v3 hp = add(o, scale(d, t));
    v3 nd;
    if (kSpecular && type == PT_MAT_SPECULAR) {
        if (!specular_dir(g, d, n, m1.w, kMaxSpecularIters, nd)) atomicAdd(A.ctr + 3, 1ull);
#ifdef PT_EXP_DUP_SPEC  // measurement only: the specular sample (rejection loop) once more
        {
            Lcg g2 = g;
            asm volatile("" : "+v"(g2.s));
            v3 x;
            specular_dir(g2, d, n, m1.w, kMaxSpecularIters, x);
            asm volatile("" ::"v"(x.x), "v"(x.y), "v"(x.z));
        }
#endif
    } else {
#ifdef PT_EXP_NO_BRDF  // timing experiment only (wrong images): no hemisphere sample
        nd = n;
#else
#if PT_THETA_TAB == 1
        nd = hemisphere_dir_tab(g, n, kernarg_args()->theta_tab);
#elif PT_THETA_TAB == 2
        // by wave: few lanes sampling -> the table (little memory traffic, the computed form
        // would run at low lane utilisation); many -> computed (no table traffic)
        if ((int)__popcll(__ballot(true)) <= kernarg_args()->theta_lanes)
            nd = hemisphere_dir_tab(g, n, kernarg_args()->theta_tab);
        else
            nd = hemisphere_dir(g, n);
#else
        nd = hemisphere_dir(g, n);
#endif
#ifdef PT_EXP_DUP_BRDF  // measurement only: the hemisphere sample once more
        {
            Lcg g2 = g;
            asm volatile("" : "+v"(g2.s));
            const v3 x = hemisphere_dir(g2, n);
            asm volatile("" ::"v"(x.x), "v"(x.y), "v"(x.z));
        }
#endif
#endif
#if defined(PT_EXP_COHERENT_DIR) || defined(PT_EXP_OCTANT_DIR)
        // timing experiments only (wrong images): bounds on what regrouping a wave's bounce
        // rays by direction could gain. COHERENT: every sampling lane of the wave takes the
        // first sampling lane's direction w, mirrored into its own hemisphere (+-w: two
        // directions per wave, the most coherent a regroup could get). OCTANT: each component
        // takes the sign of w's where the result stays in the lane's hemisphere (the sign
        // agreement a regroup by octant would give), else the lane keeps its sample.
        {
            const v3 w = v3{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(nd.x))),
                            __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(nd.y))),
                            __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(nd.z)))};
#ifdef PT_EXP_COHERENT_DIR
            nd = dot(w, n) < 0.0f ? neg(w) : w;
#else
            const v3 c = v3{__builtin_copysignf(nd.x, w.x), __builtin_copysignf(nd.y, w.y), __builtin_copysignf(nd.z, w.z)};
            if (dot(c, n) >= 0.0f) nd = c;
#endif
        }
#endif
    }
    rec_tri[k * kBlock + tid] = (RecT)row;
    rec_cos[k * kBlock + tid] = dot(n, nd);
    o = add(hp, scale(n, 1e-4f));  // SHIFT_BIAS, render.h:16, 52
    d = nd;
    k++;
    return false;
}

// Slab record of sample s of pixel q (the radiance slab is [sample][pixel][rgb]).
__device__ __forceinline__ uint32_t slab_index(const TraceArgs& A, int s, int q) {
    return (uint32_t)(s - A.s_begin) * (uint32_t)A.npix + (uint32_t)q;  // < 2^31 (host check)
}

// Unwind the recursion, L = emit + ((2 * L) * albedo) * cos (render.h:60), and store
// the sample's radiance at slab offset `at`.
// kAlbedoX2: `mats` holds a' = 2 * albedo (exact: a power-of-two scaling), and a level is
// emit + (L * a') * cos. Same bits: 2 * L is exact while |L| < 2^127, so (2L) * a and
// L * (2a) are the same real product rounded once (subnormal results included); the host
// enables it only when every material is finite and the radiance bound over PT_MAX_DEPTH
// levels stays below 2^125 (pt_kernel.hip: albedo_x2_ok). Saves the 3 doublings per level.
// Dark paths (PT_DARK_SKIP): when every material a path can bounce on (DIFFUSE, SPECULAR)
// has emission exactly +0 in all channels and a finite albedo (the host's `dark` flag), a
// path whose end value L is +0 in all channels unwinds to +0: each level is
// e + (L a) c = +0 + (+-0) = +0 (a finite, c finite, e = +0). Only paths that end on an
// emitter (1.4-1.7 % of paths in configs 2-5) unwind; the others store L as it is, and a
// wave runs the unwinding only when one of its ending lanes needs it.
#ifndef PT_DARK_SKIP
#define PT_DARK_SKIP 1
#endif
template <typename RecT, bool kAlbedoX2 = false, bool kDarkKnown = false, bool kDark = false>
__device__ __forceinline__ void finish_path(const TraceArgs& A, const float4* __restrict__ mats,
                                            const RecT* __restrict__ rec_tri, const float* __restrict__ rec_cos,
                                            int tid, int k, v3 L, uint32_t at) {
#ifdef PT_EXP_NO_FOLD  // timing experiment only (wrong images): skip the unwinding
    k = 0;
#endif
    // a dark path's unwinding is L itself (+0): the wave skips it unless a lane needs it
    const bool unwind = !(PT_DARK_SKIP && (kDarkKnown ? kDark : kernarg_args()->dark != 0) &&
                          (__float_as_uint(L.x) | __float_as_uint(L.y) | __float_as_uint(L.z)) == 0u);
    if (unwind) {
#ifndef PT_FOLD_UNROLL
#define PT_FOLD_UNROLL 1
#endif
    if (PT_FOLD_UNROLL && kernarg_args()->rec_size <= 4) {  // uniform; re-read, not held in a spilled SGPR
        // depth <= 5: every record of the path is loaded up front (predicated on j < k),
        // so the unwinding waits for two LDS round trips instead of two per level
        int tj[4];
        float cj[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            tj[j] = 0;
            cj[j] = 0.0f;
            if (j < k) {
                tj[j] = (int)rec_tri[j * kBlock + tid];
                cj[j] = rec_cos[j * kBlock + tid];
            }
        }
        float4 m0[4], m1[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (j < k) {
                m0[j] = mats[2 * tj[j]];
                m1[j] = mats[2 * tj[j] + 1];
            }
#pragma unroll
        for (int j = 3; j >= 0; j--)
            if (j < k) {
                if constexpr (kAlbedoX2)
                    L = v3{m1[j].x + (L.x * m0[j].y) * cj[j], m1[j].y + (L.y * m0[j].z) * cj[j],
                           m1[j].z + (L.z * m0[j].w) * cj[j]};
                else
                    L = v3{m1[j].x + ((2.0f * L.x) * m0[j].y) * cj[j], m1[j].y + ((2.0f * L.y) * m0[j].z) * cj[j],
                           m1[j].z + ((2.0f * L.z) * m0[j].w) * cj[j]};
            }
    } else {
        for (int j = k - 1; j >= 0; j--) {
            const int tj = (int)rec_tri[j * kBlock + tid];
            const float cj = rec_cos[j * kBlock + tid];
            const float4 m0 = mats[2 * tj], m1 = mats[2 * tj + 1];
            if constexpr (kAlbedoX2)
                L = v3{m1.x + (L.x * m0.y) * cj, m1.y + (L.y * m0.z) * cj, m1.z + (L.z * m0.w) * cj};
            else
                L = v3{m1.x + ((2.0f * L.x) * m0.y) * cj, m1.y + ((2.0f * L.y) * m0.z) * cj,
                       m1.z + ((2.0f * L.z) * m0.w) * cj};
        }
    }
    }  // unwind
#ifdef PT_EXP_DUP_FOLD  // measurement only: the unwinding once more (records re-read, result dropped)
    {
        v3 L2 = L;
        asm volatile("" : "+v"(L2.x));
        for (int j = k - 1; j >= 0; j--) {
            const int tj = (int)rec_tri[j * kBlock + tid];
            const float cj = rec_cos[j * kBlock + tid];
            const float4 m0 = mats[2 * tj], m1 = mats[2 * tj + 1];
            L2 = v3{m1.x + ((2.0f * L2.x) * m0.y) * cj, m1.y + ((2.0f * L2.y) * m0.z) * cj,
                    m1.z + ((2.0f * L2.z) * m0.w) * cj};
        }
        asm volatile("" ::"v"(L2.x), "v"(L2.y), "v"(L2.z));
    }
#endif
#ifdef PT_EXP_NO_STORE  // timing experiment only (wrong images): no radiance stores
    if (L.x == 12345.0f)
#endif
    // a flagged slab takes only the records of paths that do not end dark (TraceArgs::flags)
    uint32_t* fl = kernarg_args()->flags;
    if (unwind || !fl)
        *reinterpret_cast<float3*>(A.radiance + 3 * (size_t)at) = make_float3(L.x, L.y, L.z);  // slab_at's layout
    if (unwind && fl) {  // rare (paths that end on an emitter): at = sample * npix + pixel
        if (kernarg_args()->flags_pm) {
            const uint32_t sm = fdiv(at, A.div_npix), q = at - sm * (uint32_t)A.npix;
            atomicOr(fl + flag_word(sm, q, (uint32_t)A.npix), 1u << (sm & 31u));
        } else {
            atomicOr(fl + (at >> 5), 1u << (at & 31u));
        }
    }
}

// ray count: wave reduction, one atomic per wave
__device__ __forceinline__ void count_rays(const TraceArgs& A, int lane, uint32_t n_rays) {
    unsigned long long r = n_rays;
    for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off);
    if (lane == 0) atomicAdd(A.ctr + 1, r);
}

// ray count kept per wave (a scalar): one atomic per wave at the end
__device__ __forceinline__ void count_rays_wave(const TraceArgs& A, int lane, unsigned long long n_rays) {
    if (lane == 0) atomicAdd(A.ctr + 1, n_rays);
}

// The megakernel body of the flat path (scenes with <= 64 leaves).
// BoxMask: the leaf-box test (the kernel-argument table, or the hipRTC-generated one with
// the scene's planes as constants). One loop iteration = one path segment of every lane.
// LDS (small, so that many blocks fit): [triangles: num_tri4 float4] [materials:
// num_mat4 float4] [pair queues: pair_queue x uint16 per wave] [records: rec_size x
// kBlock x (uint16 triangle, float cos)] [best: kBlock x u64]. The node array and the
// leaf list are read from global memory (L1/L2): only the rare exact walk (a zero
// direction component) and queue overflows touch them; the exact walk's stack is in HBM.
// threadIdx.x re-read at a use: the per-lane LDS addresses formed from it (best[tid], the
// path records) are then computed where they are used instead of being held across the
// megakernel loop, where the register budgets (flat: 72, 8-wide walk: 80) spilled them to
// scratch (each reload a scratch load and a vmcnt(0) wait).
#ifndef PT_FRESH_TID
#define PT_FRESH_TID 1  // 0: plain threadIdx.x (A/B hook)
#endif
__device__ __forceinline__ int fresh_tid() {
    int t = (int)threadIdx.x;
    if (PT_FRESH_TID) asm volatile("" : "+v"(t));
    return t;
}

// The flat kernel's path-record bases, formed from the kernarg segment where they are used
// (scalar loads and adds) instead of being held in SGPRs across the loop (spilled to VGPR
// lanes at the hipRTC kernel's register budget).
struct FlatRecs {
    uint16_t* tri;
    float* cos;
};
__device__ __forceinline__ FlatRecs flat_records(float4* lds4) {
    const auto* K = kernarg_args();
    uint16_t* rt = reinterpret_cast<uint16_t*>(lds4 + K->num_tri4 + K->num_mat4) + (kBlock / kWave) * K->pair_queue;
    return FlatRecs{rt, reinterpret_cast<float*>(rt + K->rec_size * kBlock)};
}

template <typename BoxMask>
__device__ __forceinline__ void trace_body_flat(const TraceArgs& A) {
    extern __shared__ float4 lds4[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    float4* s_tris = lds4;
    float4* s_mats = s_tris + A.num_tri4;
    uint16_t* queues = reinterpret_cast<uint16_t*>(s_mats + A.num_mat4);
    uint16_t* rec_tri = queues + (kBlock / kWave) * A.pair_queue;
    float* rec_cos = reinterpret_cast<float*>(rec_tri + A.rec_size * kBlock);
    unsigned long long* best = reinterpret_cast<unsigned long long*>(rec_cos + A.rec_size * kBlock);
    float4* next_ray = reinterpret_cast<float4*>(best + kBlock);  // prefetched camera ray: d.xyz, LCG state
    uint32_t* next_at = reinterpret_cast<uint32_t*>(next_ray + kBlock);  // its item = slab offset
    uint16_t* boxtab = reinterpret_cast<uint16_t*>(next_at + kBlock);     // box-level pairs: box -> its triangles
    if constexpr (BoxMask::kBoxPairs)
        for (int i = tid; i < BoxMask::kBoxes; i += kBlock) boxtab[i] = BoxMask::kBoxTab[i];
    for (int i = tid; i < A.num_tri4; i += kBlock) s_tris[i] = A.tris[i];
    for (int i = tid; i < A.num_mat4; i += kBlock) {
        float4 m = A.mats[i];
        if (BoxMask::kAlbedoX2 && !(i & 1)) m = make_float4(m.x, 2.0f * m.y, 2.0f * m.z, 2.0f * m.w);  // row's albedo
        s_mats[i] = m;
    }
    __syncthreads();
    const float4* __restrict__ mats = s_mats;
    const float4* __restrict__ tris = s_tris;
    uint16_t* wq = queues + __builtin_amdgcn_readfirstlane(tid >> 6) * A.pair_queue;
    int* xstk = A.exact_stack + (size_t)blockIdx.x * A.exact_rows * kBlock;

    bool alive = true;      // the lane's generator may still produce paths
    bool active = false;    // lane has a path in flight (slab offset `at`)
    bool has_next = false;  // lane's next camera ray waits in next_ray / next_at (LDS)
    uint32_t at = 0;
    Lcg g{0};
    v3 o{0, 0, 0}, d{0, 0, 0};
    int k = 0;
    unsigned long long n_rays = 0;  // this wave's segments (wave-uniform)
    Pool pool = pool_start(A);
#ifdef PT_STAMPS
    uint64_t stamp_acc[kStampSections] = {};
#endif

    while (true) {
        PT_STAMP(st_a)
        // Camera rays are generated one path ahead, and only once at least
        // A.regen_thresh lanes of the wave want one (or nothing else is left to do):
        // the generator then runs with many lanes active instead of the few whose path
        // just ended. A lane idles only when its path ends before its slot is refilled.
        // The prefetched ray lives in LDS, not in registers (fewer VGPRs -> more waves).
        const bool want = alive && !has_next;
        const int n_want = (int)__popcll(__ballot(want));
        if (n_want > 0 && (n_want >= A.regen_thresh || !__any(active || has_next))) {
            uint32_t item = 0;
            claim_item(A, lane, want, pool, alive, item);
            if (want && alive) {
                const uint32_t blk = fdiv(item, A.div_npix);  // item = blk * npix + q, sample s_begin + blk
                Lcg gn{0};
                v3 on, nd;
                camera_ray(A, (int)(item - blk * (uint32_t)A.npix), A.s_begin + (int)blk, gn, on, nd);
#ifdef PT_EXP_DUP_CAMF  // measurement only: the camera ray once more
                {
                    uint32_t it2 = item;
                    asm volatile("" : "+v"(it2));
                    Lcg g2{0};
                    v3 o2, d2;
                    camera_ray(A, (int)(it2 - blk * (uint32_t)A.npix), A.s_begin + (int)blk, g2, o2, d2);
                    asm volatile("" ::"v"(d2.x), "v"(d2.y), "v"(d2.z), "v"(g2.s));
                }
#endif
                next_ray[fresh_tid()] = make_float4(nd.x, nd.y, nd.z, __uint_as_float(gn.s));
                next_at[fresh_tid()] = item;
                has_next = true;
            }
        }
        if (!active && has_next) {
            const int t0 = fresh_tid();
            const float4 nr = next_ray[t0];
            at = next_at[t0];
            g.s = __float_as_uint(nr.w);
            d = v3{nr.x, nr.y, nr.z};
            o = v3{A.pos_x, A.pos_y, A.pos_z};
            k = 0;
            active = true;
            has_next = false;
        }
        if (!__any(active)) break;
        PT_STAMP(st_b)

        // ---- BVH::intersect (bvh.h:156-183); trace(depth == 0) returns 0 without
        // intersecting (render.h:37)
        float t = 0.0f;
        int hit = -1;
        const bool tr = active && A.depth > 0;
        if (A.depth > 0) n_rays += (unsigned long long)__popcll(__ballot(tr));
        // bvh.h:157 inv = 1 / d. Waves whose lanes all have finite inv take the IEEE
        // min/max slab test (identical result, see slab_hit_finite).
        const v3 inv{rcp_exact(d.x), rcp_exact(d.y), rcp_exact(d.z)};
        const bool forced = A.force_exact_slab == 1 || (A.force_exact_slab == 2 && ((tid >> 6) & 1));
        // with the sign-bit box mask (BoxMask::kSignMask) the wave's plane values must stay
        // finite: |1 / d| <= 2^60 and |o| < 2^60 (scene coordinates < 2^60: the host's
        // condition), so |t| < 2^122; others take the exact walk as zero components do
        const bool fast = !forced && __all(!tr || (BoxMask::kSignMask ? bounded_ray(o, inv) : all_finite(inv)));
        if (fast && A.pair_queue > 0) {
            // wave-uniform branch: all 64 lanes take part in the pair queue
            if (PT_PRIO_MASK) __builtin_amdgcn_s_setprio(PT_PRIO_MASK);
            unsigned long long mask = BoxMask::mask(A, o, inv);
#ifdef PT_EXP_DUP_MASK  // measurement only: the leaf-box mask once more
            {
                v3 o2 = o;
                asm volatile("" : "+v"(o2.x));
                const unsigned long long m2 = BoxMask::mask(A, o2, inv);
                asm volatile("" ::"v"((uint32_t)m2), "v"((uint32_t)(m2 >> 32)));
            }
#endif
            if (PT_PRIO_MASK) __builtin_amdgcn_s_setprio(0);
            if (!tr) mask = 0ull;
            PT_STAMP(st_b2)
            PT_STAMP_ADD(1, st_b, st_b2)
#ifdef PT_STAMPS
            {
                const uint32_t pc = (uint32_t)__popcll(mask);
                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(pc), 63);
                int mx = (int)pc;
                for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off));
                stamp_acc[7] += 1;
                stamp_acc[8] += tot;
                stamp_acc[9] += (tot + 63) / 64;
                stamp_acc[10] += (uint32_t)mx;
            }
#endif
#ifdef PT_EXP_NO_PAIRS  // timing experiment only (wrong images): first passing leaf, no triangle test
            hit = mask ? __builtin_ctzll(mask) : -1;
            t = 1.0f;
#else
            if (PT_PRIO_PAIRS) __builtin_amdgcn_s_setprio(PT_PRIO_PAIRS);
            hit = intersect_flat_pairs<BoxMask>(A, mask, A.leaves, tris, wq, best, fresh_tid(), lane, o, d, t, boxtab);
            if (PT_PRIO_PAIRS) __builtin_amdgcn_s_setprio(0);
#endif
            PT_STAMP(st_b3)
            PT_STAMP_ADD(2, st_b2, st_b3)
        } else if (tr) {
            if (fast) hit = intersect_flat<BoxMask>(A, A.leaves, tris, o, d, inv, t, boxtab);
            else hit = intersect_tree<false>(A.nodes, tris, xstk, tid, o, d, inv, t);
        }
        PT_STAMP(st_c)

        bool end = false;
        v3 L{0.0f, 0.0f, 0.0f};
        if (PT_PRIO_SHADE) __builtin_amdgcn_s_setprio(PT_PRIO_SHADE);
        if (active) {
            const FlatRecs R = flat_records(lds4);
            end = shade<BoxMask::kSpecular>(A, mats, tris, R.tri, R.cos, fresh_tid(), hit, t, g, o, d, k, L);
        }
        if (PT_PRIO_SHADE) __builtin_amdgcn_s_setprio(0);
        PT_STAMP(st_d)
        if (end) {
            if (PT_PRIO_FOLD) __builtin_amdgcn_s_setprio(PT_PRIO_FOLD);
            const FlatRecs R = flat_records(lds4);
            finish_path<uint16_t, BoxMask::kAlbedoX2, BoxMask::kDarkKnown, BoxMask::kDark>(A, mats, R.tri, R.cos,
                                                                                        fresh_tid(), k, L, at);
            if (PT_PRIO_FOLD) __builtin_amdgcn_s_setprio(0);
            active = false;
        }
        PT_STAMP(st_e)
        PT_STAMP_ADD(0, st_a, st_b)
        PT_STAMP_ADD(5, st_b, st_c)  // whole intersection (1 + 2 + other paths)
        PT_STAMP_ADD(3, st_c, st_d)
        PT_STAMP_ADD(4, st_d, st_e)
    }
#ifdef PT_STAMPS
    if (lane == 0 && A.stamps) {
        for (int i = 0; i < kStampSections; i++)
            if (i != 6) atomicAdd(A.stamps + i, (unsigned long long)stamp_acc[i]);
        atomicAdd(A.stamps + 6, 1ull);
    }
#endif
    drain_accumulate(A, lane);
    count_rays_wave(A, lane, n_rays);
}

#ifndef PT_FLAT_ONLY
// The megakernel body of the binary-tree walk (child-pair form, intersect_tree): the
// generic path for scenes the flat list and the wide tree do not cover. kLdsScene: node,
// triangle and material arrays copied to LDS. One loop iteration = one path segment of
// every lane. LDS: [scene copy (kLdsScene)] [stack: stack_size x kBlock int]
// [records: rec_size x kBlock x (int, float)]
template <bool kLdsScene>
__device__ __forceinline__ void trace_body(const TraceArgs& A) {
    extern __shared__ float4 lds4[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int scene4 = kLdsScene ? (A.num_node4 + A.num_tri4 + A.num_mat4) : 0;
    float4* s_nodes = lds4;
    float4* s_tris = lds4 + A.num_node4;
    float4* s_mats = s_tris + A.num_tri4;
    int* stk = reinterpret_cast<int*>(lds4 + scene4);
    int* rec_tri = stk + A.stack_size * kBlock;
    float* rec_cos = reinterpret_cast<float*>(rec_tri + A.rec_size * kBlock);
    if (kLdsScene) {
        for (int i = tid; i < A.num_node4; i += kBlock) s_nodes[i] = A.nodes[i];
        for (int i = tid; i < A.num_tri4; i += kBlock) s_tris[i] = A.tris[i];
        for (int i = tid; i < A.num_mat4; i += kBlock) s_mats[i] = A.mats[i];
        __syncthreads();
    }
    const float4* __restrict__ mats = kLdsScene ? s_mats : A.mats;
    const float4* __restrict__ tris = kLdsScene ? s_tris : A.tris;

    bool alive = true;      // the lane's generator may still produce paths
    bool active = false;    // lane has a path in flight (pixel q, sample s)
    bool has_next = false;  // lane holds its next camera ray (pixel gq, sample gs - 1)
    int gq = 0, gs = 0, gs_end = 0;  // generator: work item, samples [gs, gs_end) left
    int q = 0, s = 0;
    uint32_t next_state = 0;  // LCG state after the camera draws of the next path
    v3 next_d{0, 0, 0};
    Lcg g{0};
    v3 o{0, 0, 0}, d{0, 0, 0};
    int k = 0;
    unsigned long long n_rays = 0;  // this wave's segments (wave-uniform)
    Pool pool = pool_start(A);

    while (true) {
        // camera rays one path ahead, generated once A.regen_thresh lanes want one
        const bool want = alive && !has_next;
        const int n_want = (int)__popcll(__ballot(want));
        if (n_want > 0 && (n_want >= A.regen_thresh || !__any(active || has_next))) {
            claim_work(A, lane, want && gs == gs_end, pool, alive, gq, gs, gs_end);
            if (want && alive) {
                Lcg gn{0};
                v3 on;
                camera_ray(A, gq, gs, gn, on, next_d);
                next_state = gn.s;
                gs++;
                has_next = true;
            }
        }
        if (!active && has_next) {
            q = gq;
            s = gs - 1;
            g.s = next_state;
            d = next_d;
            o = v3{A.pos_x, A.pos_y, A.pos_z};
            k = 0;
            active = true;
            has_next = false;
        }
        if (!__any(active)) break;

        // ---- BVH::intersect (bvh.h:156-183); trace(depth == 0) returns 0 (render.h:37)
        float t = 0.0f;
        int hit = -1;
        const bool tr = active && A.depth > 0;
        if (A.depth > 0) n_rays += (unsigned long long)__popcll(__ballot(tr));
        const v3 inv{rcp_exact(d.x), rcp_exact(d.y), rcp_exact(d.z)};  // bvh.h:157
        const bool forced = A.force_exact_slab == 1 || (A.force_exact_slab == 2 && ((tid >> 6) & 1));
        const bool fast = !forced && __all(!tr || all_finite(inv));
        if (tr) {
            if (fast)
                hit = kLdsScene ? intersect_tree<true>(s_nodes, s_tris, stk, tid, o, d, inv, t)
                                : intersect_tree<true>(A.nodes, A.tris, stk, tid, o, d, inv, t);
            else
                hit = kLdsScene ? intersect_tree<false>(s_nodes, s_tris, stk, tid, o, d, inv, t)
                                : intersect_tree<false>(A.nodes, A.tris, stk, tid, o, d, inv, t);
        }
        bool end = false;
        v3 L{0.0f, 0.0f, 0.0f};
        if (active) end = shade(A, mats, tris, rec_tri, rec_cos, tid, hit, t, g, o, d, k, L);
        if (end) {
            finish_path(A, mats, rec_tri, rec_cos, tid, k, L, slab_index(A, s, q));
            active = false;
        }
    }
    drain_accumulate(A, lane);
    count_rays_wave(A, lane, n_rays);
}

// The megakernel body for big scenes (wide tree read through L1/L2/MALL, its top levels
// from LDS): the wide walk is resumable, so a lane keeps its traversal state across loop
// iterations. The wave steps its traversing lanes until fewer than A.wide_thresh of them
// remain, then shades the lanes whose walk finished and starts their next segment (or
// sample), and resumes: traversal steps run with most lanes busy instead of waiting for
// the longest walk in the wave (Aila & Laine 2009's persistent while-while with dynamic
// ray fetch). Rays outside the quantised test's range (a zero or tiny direction
// component, a far origin) take the exact compare-select walk of the binary tree.
// LDS: [top nodes: wide_top x kNodeU4 uint4] [stack: wide_rows x kBlock int]
// [best: kBlock x u64] [records: rec_size x kBlock x (float, row)]
// [queues: wide_queue entries per wave, 1 word each for single-triangle leaves, else 2]
template <bool B, typename T, typename F>
struct PickT {
    using type = T;
};
template <typename T, typename F>
struct PickT<false, T, F> {
    using type = F;
};

template <int W, int kPF, bool kLdsMats>
__device__ __forceinline__ void trace_body_wide(const TraceArgs& A) {
    extern __shared__ float4 lds4[];
    constexpr int NU = kNodeU4<W, kPF>;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    float4* s_mats = lds4;  // kLdsMats: the distinct materials
    uint4* top = reinterpret_cast<uint4*>(s_mats + (kLdsMats ? A.num_umat4 : 0));
    int* stk = reinterpret_cast<int*>(top + A.wide_top * NU);
    unsigned long long* best = reinterpret_cast<unsigned long long*>(stk + A.wide_rows * kBlock);
    // path records: cos (float) then the material row, one byte when the distinct-material
    // table is in LDS (<= kMaxLdsMaterials rows), else an int
    using RecW = typename PickT<kLdsMats, uint8_t, int>::type;
    float* rec_cos = reinterpret_cast<float*>(best + kBlock);
    RecW* rec_tri = reinterpret_cast<RecW*>(rec_cos + A.rec_size * kBlock);
    // the queues last: their size (words per entry) does not move the other arrays
    uint32_t* queues = reinterpret_cast<uint32_t*>(rec_tri + A.rec_size * kBlock);
    const int qwords = A.wide_single ? 1 : 2;  // words per queue entry
    for (int i = tid; i < A.wide_top * NU; i += kBlock) top[i] = A.wide[i];
    if constexpr (kLdsMats)
        for (int i = tid; i < A.num_umat4; i += kBlock) s_mats[i] = A.umats[i];
    __syncthreads();
    // materials by row of the distinct table (records hold rows), normals from nrm
    const float4* __restrict__ mats = kLdsMats ? s_mats : A.umats;
    const float4* __restrict__ nrm = A.nrm;
    // wave-uniform bases (scalar registers)
    unsigned long long* wbest = best + __builtin_amdgcn_readfirstlane(tid - lane);
    uint32_t* wq = queues + __builtin_amdgcn_readfirstlane(tid >> 6) * A.wide_queue * qwords;

    bool alive = true;    // lane may still get work
    bool active = false;  // lane has a path in flight
    bool trav = false;    // lane's wide walk in progress
    bool done = false;    // lane's intersection result ready for shading
    int s = 0, s_end = 0, q = 0;
    Lcg g{0};
    v3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    WideRay wr{};  // float planes: the segment's per-ray constants (wide_ray_consts)
    int k = 0;
    int cur = 0, sp = 0;
    int qn = 0;  // wave-uniform queue length
    unsigned long long n_rays = 0;  // this wave's segments (wave-uniform)
    Pool pool = pool_start(A);
    const int thresh = A.wide_thresh;
    unsigned long long d_rounds = 0, d_ents = 0, f_rounds = 0, f_ents = 0;  // drain counts (PT_STAMPS)
#ifdef PT_STAMPS
    uint64_t stamp_acc[kStampSections] = {};
    const uint64_t tl_start = __builtin_amdgcn_s_memrealtime();
    uint64_t tl_exhaust = 0;
#endif

    while (true) {
        PT_STAMP(st_a)
#ifdef PT_STAMPS
        stamp_acc[10] += 1;
#endif
        claim_work(A, lane, alive && !active && (s == s_end), pool, alive, q, s, s_end);
#ifdef PT_STAMPS
        if (tl_exhaust == 0 && __ballot(!alive) != 0ull) tl_exhaust = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef PT_EXP_DUP_CLAIM  // measurement only: the claim's item arithmetic once more (no pool change)
        {
            int need2 = alive && !active ? 1 : 0;
            asm volatile("" : "+v"(need2));
            const unsigned long long want2 = __ballot(need2 != 0);
            if (need2) {
                const uint32_t rank2 =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(want2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want2, 0u));
                const uint32_t item2 = pool.next + rank2;
                const uint32_t blk2 = fdiv(item2, A.div_npix);
                const int q2 = (int)(item2 - blk2 * (uint32_t)A.npix);
                asm volatile("" ::"v"(q2), "v"(blk2));
            }
        }
#endif
#ifdef PT_STAMPS
        stamp_acc[12] += (uint64_t)__popcll(__ballot(alive && !active));
#endif
        if (alive && !active) {
            camera_ray(A, q, s, g, o, d);
#ifdef PT_EXP_DUP_CAM  // measurement only: the camera ray once more
            {
                Lcg g2{0};
                v3 o2, d2;
                int q2 = q;
                asm volatile("" : "+v"(q2));
                camera_ray(A, q2, s, g2, o2, d2);
                asm volatile("" ::"v"(d2.x), "v"(d2.y), "v"(d2.z), "v"(g2.s));
            }
#endif
            k = 0;
            active = true;
        }
        if (!__any(active)) break;
        const bool start = active && !trav && !done;
        if (A.depth > 0) n_rays += (unsigned long long)__popcll(__ballot(start));
        if (start) {  // start this segment's BVH::intersect; the result goes to best[tid]
            best[fresh_tid()] = ~0ull;  // miss; also trace(depth == 0) returns 0 without intersecting (render.h:37)
            done = true;
            if (A.depth > 0) {
                inv = v3{rcp_exact(d.x), rcp_exact(d.y), rcp_exact(d.z)};  // bvh.h:157
#ifdef PT_EXP_DUP_START  // measurement only: the segment start's 1 / d and range checks once more
                {
                    v3 d2 = d;
                    asm volatile("" : "+v"(d2.x));
                    const v3 i2{rcp_exact(d2.x), rcp_exact(d2.y), rcp_exact(d2.z)};
                    const float r2 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(i2.x), __builtin_fabsf(i2.y)),
                                                     __builtin_fabsf(i2.z));
                    asm volatile("" ::"v"(r2), "v"(i2.x), "v"(i2.y), "v"(i2.z));
                }
#endif
                const float ri = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(inv.x), __builtin_fabsf(inv.y)),
                                                 __builtin_fabsf(inv.z));
                const float ro = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(o.x), __builtin_fabsf(o.y)),
                                                 __builtin_fabsf(o.z));
                if (!A.force_exact_slab && ri <= 0x1p60f && ro < 0x1p64f) {
                    if constexpr (kPF == 2) wr = wide_ray_consts(A, o, inv);
                    cur = 0;
                    sp = 0;
                    trav = true;
                    done = false;
                } else {
                    // rare (a zero or tiny direction component): its binary-tree stack is in
                    // HBM, so LDS holds only the wide walk's rows
                    float tx;
                    const int hx = intersect_tree<false>(A.nodes, A.tris,
                                                         A.exact_stack + (size_t)blockIdx.x * A.exact_rows * kBlock,
                                                         tid, o, d, inv, tx);
                    if (hx >= 0) best[fresh_tid()] = ((unsigned long long)__float_as_uint(tx) << 32) | (uint32_t)hx;
                }
            }
        }
        PT_STAMP(st_b)
        PT_STAMP_ADD(0, st_a, st_b)
        // the lanes whose 1 / d is negative, per axis (their octant's plane order)
        const unsigned long long neg[3] = {__builtin_amdgcn_ballot_w64(inv.x < 0.0f),
                                           __builtin_amdgcn_ballot_w64(inv.y < 0.0f),
                                           __builtin_amdgcn_ballot_w64(inv.z < 0.0f)};
        // float planes: the walk reads 1 / d from the packed pairs (one copy of it in registers)
        const v3 winv = kPF == 2 ? v3{wr.p[0].x, wr.p[0].y, wr.p[1].x} : inv;
        // The step loop hands the wave back to shading once fewer than `thresh` of its 64 lanes
        // traverse. At the end of the work fewer lanes hold paths, and a fixed bar then let
        // each outer iteration take one step and a forced drain; the bar scales with the
        // lanes that hold paths (the same bar while all 64 do). Round 6: the launch's drain.
#if PT_WIDE_THR_SCALE
        const int thr = (thresh * (int)__popcll(__ballot(active)) + kWave - 1) / kWave;
#else
        const int thr = thresh;
#endif
        while (__any(trav)) {
#ifdef PT_STAMPS
            stamp_acc[7] += 1;
            stamp_acc[8] += (uint64_t)__popcll(__ballot(trav));
#endif
            PT_STAMP(st_s0)
            if (PT_PRIO_STEP) __builtin_amdgcn_s_setprio(PT_PRIO_STEP);
            const bool fin = wide_step_q<W, kPF>(A, top, stk, tid, lane, trav, o, d, winv, wr, neg, cur, sp, wq, qn,
                                                 A.wide_queue, wbest, d_rounds, d_ents);
            if (PT_PRIO_STEP) __builtin_amdgcn_s_setprio(0);
            if (fin) {
                trav = false;
                done = true;
            }
            PT_STAMP(st_s1)
            PT_STAMP_ADD(1, st_s0, st_s1)
            if (qn >= kWave) {
#ifdef PT_STAMPS
                stamp_acc[9] += 1;
#endif
                wide_queue_drain(wq, qn, false, A.wtris, wbest, lane, o, d, winv, A.tri_fast != 0, A.wide_single != 0,
                                 A.wide_compact != 0, d_rounds, d_ents);
            }
            PT_STAMP(st_s2)
            PT_STAMP_ADD(2, st_s1, st_s2)
#ifdef PT_EXP_DUP_LOOPCTL  // measurement only: the step loop's exit test once more
            {
                int t2 = trav ? 1 : 0;
                asm volatile("" : "+v"(t2));
                const int n2 = (int)__popcll(__ballot(t2 != 0));
                asm volatile("" ::"s"(n2));
            }
#endif
            if ((int)__popcll(__ballot(trav)) < thr) break;
        }
        PT_STAMP(st_c)
        if (qn > 0)
            wide_queue_drain(wq, qn, true, A.wtris, wbest, lane, o, d, winv, A.tri_fast != 0, A.wide_single != 0,
                             A.wide_compact != 0, f_rounds, f_ents);
        PT_STAMP(st_d)
        PT_STAMP_ADD(2, st_c, st_d)
#ifdef PT_STAMPS
        stamp_acc[11] += (uint64_t)__popcll(__ballot(done));
#endif
        if (done) {
            done = false;
            const unsigned long long kb = best[fresh_tid()];
            const int hit = (uint32_t)kb == 0xffffffffu ? -1 : (int)(uint32_t)kb;
            const float t = hit < 0 ? 1e30f : __uint_as_float((uint32_t)(kb >> 32));
            v3 L;
            const bool end = shade<true, RecW, true>(A, mats, nrm, rec_tri, rec_cos, fresh_tid(), hit, t, g, o, d, k, L);
            PT_STAMP(st_e)
            PT_STAMP_ADD(3, st_d, st_e)
#ifdef PT_STAMPS
            stamp_acc[16] += (uint64_t)__popcll(__ballot(end));
#endif
            if (end) {
                finish_path(A, mats, rec_tri, rec_cos, fresh_tid(), k, L, slab_index(A, s, q));
                s++;
                active = false;
            }
            PT_STAMP(st_f)
            PT_STAMP_ADD(4, st_e, st_f)
        }
    }
#ifdef PT_STAMPS
    stamp_acc[13] = d_rounds + f_rounds;
    stamp_acc[14] = d_ents + f_ents;
    stamp_acc[15] = f_rounds;
    {
        const uint64_t tl_end = __builtin_amdgcn_s_memrealtime();
        if (tl_exhaust == 0) tl_exhaust = tl_end;
        stamp_acc[20] = tl_end - tl_start;
        stamp_acc[21] = tl_end - tl_exhaust;
        if (lane == 0 && A.stamps) {
            atomicMax(A.stamps + 17, (unsigned long long)~tl_start);
            atomicMax(A.stamps + 18, (unsigned long long)tl_end);
            atomicMax(A.stamps + 19, (unsigned long long)~tl_exhaust);
            atomicMax(A.stamps + 22, (unsigned long long)tl_exhaust);
        }
    }
    if (lane == 0 && A.stamps) {
        for (int i = 0; i < kStampSections; i++)
            if (i != 6 && (i < 17 || i == 20 || i == 21)) atomicAdd(A.stamps + i, (unsigned long long)stamp_acc[i]);
        atomicAdd(A.stamps + 6, 1ull);
    }
#else
    (void)d_rounds, (void)d_ents, (void)f_rounds, (void)f_ents;
#endif
    drain_accumulate(A, lane);
    count_rays_wave(A, lane, n_rays);
}
#endif  // PT_FLAT_ONLY

}  // namespace pt
