// pt_kernel.hip — gfx950 megakernel for the reference's per-pixel trace loop,
// plus the device-side context of libpt_hip.so.
//
// One persistent launch per sample batch. Every lane runs its own path state
// machine: one loop iteration = one path segment (BVH::intersect + shading,
// bvh.h:156-183 + render.h:36-61 unrolled). A lane whose path ends writes the
// sample's radiance and immediately starts the next sample of its work item;
// lanes whose item is exhausted refill through a wave-aggregated atomic
// (ballot + popcount + mbcnt prefix: one global atomic per wave per refill).
// So lanes never wait for the longest path in their wave to finish its sample.
//
// Accumulation order is the reference's (render.h:84, image.h:27-40): each
// sample's radiance is stored to an HBM slab [rgb][sample][pixel]; a second
// kernel adds the slab into the per-pixel float32 running sum in sample order
// and divides by spp at the end. Items can therefore run in any order on any
// lane/GPU and the image is still bit-identical to the sequential loop.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "pt_internal.h"
#include "pt_math.h"

namespace pt {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxSpecularIters = 1 << 16;  // bound for material.h:20-23 (reference: unbounded)
constexpr int kChunk = 256;                  // work items claimed per wave per atomic

// Diagnostic build only (make STAMPS=1 -> lib/libpt_hip_stamps.so): per-wave s_memtime
// deltas of the loop's sections, summed into TraceArgs::stamps. Never in the product build.
#ifdef PT_STAMPS
#define PT_STAMP(v)                      \
    __builtin_amdgcn_sched_barrier(0);   \
    const uint64_t v = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);
#define PT_STAMP_ADD(i, a, b) stamp_acc[i] += (b) - (a);
#else
#define PT_STAMP(v)
#define PT_STAMP_ADD(i, a, b)
#endif
[[maybe_unused]] constexpr int kStampSections = 6;

#ifndef PT_BOX_KERNARG
#define PT_BOX_KERNARG 1  // flat leaf boxes from the kernel-argument segment (scalar loads)
#endif
constexpr int kMaxFlatLeaves = 64;

// Leaf boxes of the flat path, passed by value in the kernel-argument segment so the
// wave-uniform box loop reads them with scalar loads (SGPR operands, no VMEM waits).
struct FlatLeaves {
    float box[kMaxFlatLeaves][6];  // lb.xyz, rt.xyz; padded to a multiple of 4
};

struct TraceArgs {
    const float4* __restrict__ nodes;
    const float4* __restrict__ tris;
    const float4* __restrict__ mats;
    const float4* __restrict__ leaves;     // flat leaf list (2 x float4 per leaf, rank order)
    float* __restrict__ radiance;          // [3][s_count][npix]
    unsigned long long* __restrict__ ctr;  // [0] work head, [1] rays, [2] (unused), [3] runaway
    unsigned long long total_items;
    float pos_x, pos_y, pos_z;
    float col0_x, col0_y, col0_z;  // camera transform columns (camera.h:67-71)
    float col1_x, col1_y, col1_z;
    float col2_x, col2_y, col2_z;
    float vres_x, vres_y, cell, dist;
    int W, npix;
    int part_index, part_count, band_rows;
    int depth;
    uint32_t seed;
    int s_begin, s_count, per_item;
    int stack_size;  // deferred-left-child stack entries per lane
    int rec_size;    // path records per lane (depth - 1)
    int num_node4, num_tri4, num_mat4;  // float4 counts of the scene arrays (LDS copy)
    int num_leaves;                      // flat leaf list length (kFlat kernels)
    int force_exact_slab;                // test hook (PT_FORCE_EXACT_SLAB=1): never take the IEEE path
    unsigned long long* stamps;          // PT_STAMPS builds: kStampSections cycle sums
    float zero;                          // 0.0f at run time (diagnostic ablation builds)
    int num_leaves_padded;               // num_leaves rounded up to a multiple of 4
    FlatLeaves flat;                     // kFlat kernels only
};

// compact row r of this part -> image row h (row h belongs to part (h / band) % parts)
__device__ __forceinline__ int part_row(const TraceArgs& A, int r) {
    const int k = r / A.band_rows, i = r - k * A.band_rows;
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

// BVH::intersect (bvh.h:156-183) in child-pair form. The reference pops a node, tests
// its box, then tests a leaf's triangles or pushes left and right (right is popped
// first). Here both children's boxes are tested when their parent is processed (a box
// test is a pure function, so testing it earlier changes nothing), the right subtree
// is entered first and only a hit left sibling is deferred on the stack: the sequence
// of triangle tests — and so the first-found winner among equal t — is the reference's.
template <bool kFiniteInv>
__device__ __forceinline__ bool box_hit(v3 lb, v3 rt, v3 o, v3 inv) {
    return kFiniteInv ? slab_hit_finite(lb, rt, o, inv) : slab_hit(lb, rt, o, inv);
}

template <bool kFiniteInv, typename NodePtr, typename TriPtr>
__device__ __forceinline__ int intersect_scene(NodePtr nodes, TriPtr tris, int* __restrict__ stk, int tid, v3 o,
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

// BVH::intersect for scenes with <= 64 leaves, as a flat leaf list (see DESIGN.md
// "Exact traversal by leaf rank"). With finite inv the slab test is monotone under
// box containment, so a leaf box passes only if every ancestor box passes: the
// triangles the reference tests are exactly those of leaves whose own box passes,
// whatever the tree. Step 1 tests every leaf box in a wave-uniform loop (boxes come
// through scalar loads); step 2 tests each lane's passing leaves in rank order, so
// the first strict minimum is the reference's winner (bvh.h:171).
template <typename TriPtr, typename LeafPtr>
__device__ __forceinline__ int intersect_flat(const TraceArgs& A, LeafPtr lleaves, TriPtr tris, v3 o, v3 d, v3 inv,
                                              float& t_out, uint64_t& stamp_mid, float stamp_zero) {
    // Step 1: every leaf box, wave-uniform, kU per iteration (independent chains).
#ifndef PT_BOX_UNROLL
#define PT_BOX_UNROLL 4
#endif
    constexpr int kU = PT_BOX_UNROLL;
#if PT_BOX_KERNARG
    const float(*box)[6] = A.flat.box;
#endif
    uint32_t lo = 0, hi = 0;
    const int n = A.num_leaves_padded;
    for (int k = 0; k < n; k += kU) {
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < kU; j++) {
#if PT_BOX_KERNARG
            const float* b = box[k + j];
            const v3 blb{b[0], b[1], b[2]}, brt{b[3], b[4], b[5]};
#else
            const float4 p = A.leaves[2 * (k + j)], q = A.leaves[2 * (k + j) + 1];
            const v3 blb{p.x, p.y, p.z}, brt{p.w, q.x, q.y};
#endif
            bits |= slab_hit_finite(blb, brt, o, inv) ? (1u << j) : 0u;
        }
        if (k < 32) lo |= bits << k;
        else hi |= bits << (k - 32);
    }
#ifdef PT_ABLATE_BOX2  // diagnostic: run the box loop a second time (cost of one pass = delta)
    {
        uint32_t lo2 = 0, hi2 = 0;
        const v3 inv2{inv.x + stamp_zero, inv.y, inv.z};
        for (int k = 0; k < n; k += 4) {
            bool h[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float* b = box[k + j];
                h[j] = slab_hit_finite(v3{b[0], b[1], b[2]}, v3{b[3], b[4], b[5]}, o, inv2);
            }
            const uint32_t bits = (h[0] ? 1u : 0u) | (h[1] ? 2u : 0u) | (h[2] ? 4u : 0u) | (h[3] ? 8u : 0u);
            if (k < 32) lo2 |= bits << k;
            else hi2 |= bits << (k - 32);
        }
        if (stamp_zero != 0.0f) { lo &= lo2; hi &= hi2; }
    }
#endif
    unsigned long long mask = ((unsigned long long)hi << 32) | lo;
    mask &= A.num_leaves >= 64 ? ~0ull : ((1ull << A.num_leaves) - 1);  // padding bits
#ifdef PT_STAMPS
    PT_STAMP(st_mid)
    stamp_mid = st_mid;
#else
    (void)stamp_mid;
    (void)stamp_zero;
#endif
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

#ifndef PT_WAVES
#define PT_WAVES 7  // waves per SIMD the trace kernel is register-allocated for (<= 72 VGPRs)
#endif
template <bool kLdsScene, bool kFlat>
__global__ __launch_bounds__(kBlock, PT_WAVES) void pt_trace_kernel(TraceArgs A) {
    extern __shared__ float4 lds4[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    // LDS: [scene copy (kLdsScene)] [stack: stack_size x kBlock int] [records: rec_size x kBlock x (int,float)]
    const int leaf4 = kFlat ? 2 * A.num_leaves : 0;
    const int scene4 = kLdsScene ? (A.num_node4 + A.num_tri4 + A.num_mat4 + leaf4) : 0;
    float4* s_nodes = lds4;
    float4* s_tris = lds4 + A.num_node4;
    float4* s_mats = s_tris + A.num_tri4;
    float4* s_leaves = s_mats + A.num_mat4;
    int* stk = reinterpret_cast<int*>(lds4 + scene4);
    int* rec_tri = stk + A.stack_size * kBlock;
    float* rec_cos = reinterpret_cast<float*>(rec_tri + A.rec_size * kBlock);
    if (kLdsScene) {
        for (int i = tid; i < A.num_node4; i += kBlock) s_nodes[i] = A.nodes[i];
        for (int i = tid; i < A.num_tri4; i += kBlock) s_tris[i] = A.tris[i];
        for (int i = tid; i < A.num_mat4; i += kBlock) s_mats[i] = A.mats[i];
        for (int i = tid; i < leaf4; i += kBlock) s_leaves[i] = A.leaves[i];
        __syncthreads();
    }
    const float4* __restrict__ mats = kLdsScene ? s_mats : A.mats;
    const float4* __restrict__ tris = kLdsScene ? s_tris : A.tris;

    bool alive = true;    // lane may still get work
    bool active = false;  // lane has a path in flight
    int s = 0, s_end = 0, q = 0;
    Lcg g{0};
    v3 o{0, 0, 0}, d{0, 0, 0};
    int k = 0;
    uint32_t n_rays = 0;
    // Wave-private pool of work items [pool_next, pool_end), refilled kChunk items at a
    // time by one atomic: a single global counter saturates near 88 returning atomics/us
    // (MI355X_MICROARCH.md, row "dequeue"), which one claim per wave-iteration reaches.
    unsigned long long pool_next = 0, pool_end = 0;
#ifdef PT_STAMPS
    uint64_t stamp_acc[kStampSections] = {0, 0, 0, 0, 0, 0};
#endif

    while (true) {
        PT_STAMP(st_a)
        const bool need = alive && !active && (s == s_end);
        const unsigned long long want = __ballot(need);
        if (want != 0ull) {  // wave-uniform
            const unsigned long long cnt = (unsigned long long)__popcll(want);
            const unsigned long long avail = pool_end - pool_next;
            unsigned long long fresh = 0;
            if (avail < cnt) {
                unsigned long long b = 0;
                if (lane == 0) b = atomicAdd(A.ctr, (unsigned long long)kChunk);
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
                const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
                fresh = ((unsigned long long)hi << 32) | lo;
            }
            if (need) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
                const unsigned long long item = rank < avail ? pool_next + rank : fresh + (rank - avail);
                if (item >= A.total_items) {
                    alive = false;
                } else {
                    const unsigned long long blk = item / (unsigned long long)A.npix;
                    q = (int)(item - blk * (unsigned long long)A.npix);
                    s = A.s_begin + (int)blk * A.per_item;
                    s_end = min(s + A.per_item, A.s_begin + A.s_count);
                }
            }
            if (avail < cnt) {
                pool_next = fresh + (cnt - avail);
                pool_end = fresh + kChunk;
            } else {
                pool_next += cnt;
            }
        }
        if (alive && !active) {
            if (alive) {
                // camera.h:63-73 with the per-sample reseed of pt_sample_seed
                const int r = q / A.W;
                const int px = q - r * A.W;
                const int py = part_row(A, r);
                g.s = pt_sample_seed((uint32_t)(py * A.W + px), (uint32_t)s, A.seed);
                const float jy = g.next01();  // g++ evaluates the y argument first
                const float jx = g.next01();
                const float cx = ((float)px + jx) * A.cell - A.vres_x / 2.0f;
                const float cy = ((float)py + jy) * A.cell - A.vres_y / 2.0f;
                const float cz = -A.dist;
                d = normalize(v3{cx * A.col0_x + cy * A.col0_y + cz * A.col0_z,
                                 cx * A.col1_x + cy * A.col1_y + cz * A.col1_z,
                                 cx * A.col2_x + cy * A.col2_y + cz * A.col2_z});
                o = v3{A.pos_x, A.pos_y, A.pos_z};
                k = 0;
                active = true;
            }
        }
        if (!__any(active)) break;
        PT_STAMP(st_b)

        // ---- BVH::intersect (bvh.h:156-183); trace(depth == 0) returns 0 without
        // intersecting (render.h:37)
        float t = 0.0f;
        int hit = -1;
        uint64_t stamp_mid = 0;
        if (active && A.depth > 0) {
            // bvh.h:157 inv = 1 / d. Waves whose lanes all have finite inv take the
            // IEEE min/max slab test (identical result, see slab_hit_finite).
            const v3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
            if (!A.force_exact_slab && __all(all_finite(inv))) {
                if (kFlat)
                    hit = intersect_flat(A, s_leaves, s_tris, o, d, inv, t, stamp_mid, A.zero);
                else
                    hit = kLdsScene ? intersect_scene<true>(s_nodes, s_tris, stk, tid, o, d, inv, t)
                                    : intersect_scene<true>(A.nodes, A.tris, stk, tid, o, d, inv, t);
            } else {
                hit = kLdsScene ? intersect_scene<false>(s_nodes, s_tris, stk, tid, o, d, inv, t)
                                : intersect_scene<false>(A.nodes, A.tris, stk, tid, o, d, inv, t);
            }
            n_rays++;
        }
        PT_STAMP(st_c)

        // ---- trace() body (render.h:41-57)
        bool end = false;
        v3 L{0.0f, 0.0f, 0.0f};
        if (active) {
            if (hit < 0) {
                end = true;  // miss -> 0 (also depth <= 0)
            } else {
                const float4 m0 = mats[2 * hit], m1 = mats[2 * hit + 1];
                const int type = __float_as_int(m0.x);
                if (type == PT_MAT_EMIT) {
                    end = true;
                    L = v3{m1.x, m1.y, m1.z};
                } else if (k + 1 >= A.depth) {
                    // Last segment: trace(depth-1 == 0) returns 0, so the result is
                    // emission + ((2*0)*albedo)*cos; the BRDF draw only advanced the
                    // per-sample stream, which ends here.
                    end = true;
                    L = v3{m1.x + 0.0f * m0.y, m1.y + 0.0f * m0.z, m1.z + 0.0f * m0.w};
                } else {
                    const float4 tn = tris[3 * hit + 2];
                    v3 n{tn.y, tn.z, tn.w};
                    if (!(dot(n, d) < 0.0f)) n = neg(n);  // triangle.h:48
                    const v3 hp = add(o, scale(d, t));
                    v3 nd;
                    if (type == PT_MAT_SPECULAR) {
                        if (!specular_dir(g, d, n, m1.w, kMaxSpecularIters, nd)) atomicAdd(A.ctr + 3, 1ull);
                    } else {
                        nd = hemisphere_dir(g, n);
                    }
                    rec_tri[k * kBlock + tid] = hit;
                    rec_cos[k * kBlock + tid] = dot(n, nd);
                    o = add(hp, scale(n, 1e-4f));  // SHIFT_BIAS, render.h:16, 52
                    d = nd;
                    k++;
                }
            }
        }
        PT_STAMP(st_d)
        if (end) {
            // Unwind the recursion: L = emit + ((2 * L) * albedo) * cos  (render.h:60)
            for (int j = k - 1; j >= 0; j--) {
                const int tj = rec_tri[j * kBlock + tid];
                const float cj = rec_cos[j * kBlock + tid];
                const float4 m0 = mats[2 * tj], m1 = mats[2 * tj + 1];
                L = v3{m1.x + ((2.0f * L.x) * m0.y) * cj, m1.y + ((2.0f * L.y) * m0.z) * cj,
                       m1.z + ((2.0f * L.z) * m0.w) * cj};
            }
            const size_t plane = (size_t)A.s_count * (size_t)A.npix;
            const size_t at = (size_t)(s - A.s_begin) * (size_t)A.npix + (size_t)q;
            A.radiance[at] = L.x;
            A.radiance[plane + at] = L.y;
            A.radiance[2 * plane + at] = L.z;
            s++;
            active = false;
        }
        PT_STAMP(st_e)
        PT_STAMP_ADD(0, st_a, st_b)
        PT_STAMP_ADD(1, st_b, st_c)
#ifdef PT_STAMPS
        {
            const uint64_t mid = __builtin_amdgcn_readfirstlane((uint32_t)stamp_mid) |
                                 ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(stamp_mid >> 32)) << 32);
            if (mid) stamp_acc[4] += mid - st_b;
        }
#endif
        PT_STAMP_ADD(2, st_c, st_d)
        PT_STAMP_ADD(3, st_d, st_e)
    }
#ifdef PT_STAMPS
    if (lane == 0 && A.stamps) {
        for (int i = 0; i < 5; i++) atomicAdd(A.stamps + i, (unsigned long long)stamp_acc[i]);
        atomicAdd(A.stamps + 5, 1ull);
    }
#endif

    // ---- ray count: wave reduction, one atomic per wave
    unsigned long long r = n_rays;
    for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off);
    if (lane == 0) atomicAdd(A.ctr + 1, r);
}
// Running per-pixel sum in sample order (image.h:27-31 via render.h:84), then /spp
// (image.h:37-40) on the last batch; output interleaved RGB rows of this part.
__global__ __launch_bounds__(kBlock) void pt_accumulate_kernel(const float* __restrict__ radiance,
                                                               float* __restrict__ accum, float* __restrict__ out,
                                                               int npix, int s_count, int first, int last,
                                                               float spp) {
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= npix) return;
    const size_t plane = (size_t)s_count * (size_t)npix;
    float x = first ? 0.0f : accum[q];
    float y = first ? 0.0f : accum[npix + q];
    float z = first ? 0.0f : accum[2 * (size_t)npix + q];
    for (int sl = 0; sl < s_count; sl++) {
        const size_t at = (size_t)sl * npix + q;
        x += radiance[at];
        y += radiance[plane + at];
        z += radiance[2 * plane + at];
    }
    if (last) {
        out[3 * (size_t)q] = x / spp;
        out[3 * (size_t)q + 1] = y / spp;
        out[3 * (size_t)q + 2] = z / spp;
    } else {
        accum[q] = x;
        accum[npix + q] = y;
        accum[2 * (size_t)npix + q] = z;
    }
}

// Device copies of the math primitives, for the GPU math known-answer tests.
__global__ void pt_math_kernel(int which, const float* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (which == 0) {
        out[i] = acosf_ref(in[i]);
    } else if (which == 1) {
        float sv, cv;
        sincosf_ref(in[i], sv, cv);
        out[2 * i] = sv;
        out[2 * i + 1] = cv;
    } else if (which == 2) {
        // BRDF from an LCG state: in = {state_bits, type, rough, dx, dy, dz, nx, ny, nz} per item
        const float* a = in + 9 * (size_t)i;
        Lcg g{__float_as_uint(a[0])};
        const int type = __float_as_int(a[1]);
        const v3 dd{a[3], a[4], a[5]}, nn{a[6], a[7], a[8]};
        v3 r;
        if (type == PT_MAT_SPECULAR) specular_dir(g, dd, nn, a[2], kMaxSpecularIters, r);
        else r = hemisphere_dir(g, nn);
        out[4 * i] = r.x;
        out[4 * i + 1] = r.y;
        out[4 * i + 2] = r.z;
        out[4 * i + 3] = __uint_as_float(g.s);
    }
}

}  // namespace pt

using namespace pt;

struct pt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int num_cus = 0;
    // scene
    float4* d_nodes = nullptr;
    float4* d_tris = nullptr;
    float4* d_mats = nullptr;
    float4* d_leaves = nullptr;
    std::vector<f4> flat_host;  // leaf boxes for the kernel-argument table
    PackedScene meta;
    bool have_scene = false;
    // buffers
    float* d_radiance = nullptr;
    size_t radiance_floats = 0;
    float* d_accum = nullptr;
    size_t accum_floats = 0;
    float* d_out = nullptr;
    size_t out_floats = 0;
    unsigned long long* d_ctr = nullptr;
    unsigned long long* d_stamps = nullptr;  // PT_STAMPS builds only
};

namespace {

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return set_error(PT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int ensure(float** p, size_t* cap, size_t n) {
    if (*cap >= n && *p) return PT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(float)));
    *cap = n;
    return PT_OK;
}

size_t lds_scene_budget() {
    const char* e = getenv("PT_LDS_SCENE_BYTES");
    if (e && *e) return (size_t)strtoull(e, nullptr, 0);
    return 32 * 1024;
}

size_t batch_bytes_budget() {
    const char* e = getenv("PT_BATCH_BYTES");
    if (e && *e) return (size_t)strtoull(e, nullptr, 0);
    return (size_t)4 << 30;  // 4 GiB radiance slab: ~340 spp of a 1024^2 frame per launch
}

}  // namespace

extern "C" {

int pt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pt_ctx_create(int device, pt_ctx** out) {
    if (!out) return set_error(PT_E_ARG, "pt_ctx_create: out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(PT_E_HIP, "no HIP device available");
    if (device < 0 || device >= n) return set_error(PT_E_ARG, "device %d out of range (have %d)", device, n);
    HIP_TRY(hipSetDevice(device));
    pt_ctx* c = new pt_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return set_error(PT_E_HIP, "hipGetDeviceProperties failed");
    }
    c->num_cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void**)&c->d_ctr, 4 * sizeof(unsigned long long)) != hipSuccess) {
        pt_ctx_destroy(c);
        return set_error(PT_E_HIP, "stream/counter allocation failed");
    }
    *out = c;
    return PT_OK;
}

void pt_ctx_destroy(pt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : {(void*)c->d_nodes, (void*)c->d_tris, (void*)c->d_mats, (void*)c->d_leaves, (void*)c->d_radiance,
                    (void*)c->d_accum, (void*)c->d_out, (void*)c->d_ctr, (void*)c->d_stamps})
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int pt_ctx_set_scene(pt_ctx* c, const pt_scene* scene) {
    if (!c) return set_error(PT_E_ARG, "context is NULL");
    PackedScene ps;
    int rc = pack_scene(scene, ps);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    for (float4** p : {&c->d_nodes, &c->d_tris, &c->d_mats, &c->d_leaves}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    c->have_scene = false;
    HIP_TRY(hipMalloc((void**)&c->d_nodes, ps.nodes.size() * sizeof(float4)));
    HIP_TRY(hipMalloc((void**)&c->d_tris, ps.tris.size() * sizeof(float4)));
    HIP_TRY(hipMalloc((void**)&c->d_mats, ps.mats.size() * sizeof(float4)));
    HIP_TRY(hipMemcpyAsync(c->d_nodes, ps.nodes.data(), ps.nodes.size() * sizeof(float4), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_tris, ps.tris.data(), ps.tris.size() * sizeof(float4), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_mats, ps.mats.data(), ps.mats.size() * sizeof(float4), hipMemcpyHostToDevice,
                           c->stream));
    if (!ps.leaves.empty()) {
        HIP_TRY(hipMalloc((void**)&c->d_leaves, ps.leaves.size() * sizeof(float4)));
        HIP_TRY(hipMemcpyAsync(c->d_leaves, ps.leaves.data(), ps.leaves.size() * sizeof(float4),
                               hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    ps.nodes.clear();
    ps.tris.clear();
    ps.mats.clear();
    c->flat_host = ps.leaves;
    ps.leaves.clear();
    c->meta = ps;
    c->have_scene = true;
    return PT_OK;
}

int pt_ctx_render(pt_ctx* c, const pt_camera* cam, const pt_params* prm, float* out, int out_is_device,
                  pt_stats* stats) {
    const auto t_start = std::chrono::steady_clock::now();
    if (!c || !cam || !prm || !out) return set_error(PT_E_ARG, "pt_ctx_render: NULL argument");
    if (!c->have_scene) return set_error(PT_E_ARG, "pt_ctx_render: no scene set");
    const int W = cam->res[0], H = cam->res[1];
    if (W <= 0 || H <= 0) return set_error(PT_E_ARG, "camera resolution must be positive");
    const int parts = prm->part_count > 0 ? prm->part_count : 1;
    const int band = prm->band_rows > 0 ? prm->band_rows : 1;
    if (prm->part_index < 0 || prm->part_index >= parts) return set_error(PT_E_ARG, "part_index out of range");
    if (prm->depth > PT_MAX_DEPTH) return set_error(PT_E_ARG, "depth %d exceeds PT_MAX_DEPTH", prm->depth);
    const int rows = pt_part_rows(H, prm->part_index, parts, band);
    const long long npix_ll = (long long)rows * W;
    if (npix_ll > (1ll << 30)) return set_error(PT_E_ARG, "too many pixels for one part");
    const int npix = (int)npix_ll;
    const int spp = prm->spp > 0 ? prm->spp : 0;
    HIP_TRY(hipSetDevice(c->device));

    // batch size: radiance slab of 3 * batch * npix floats within the budget
    int batch = prm->batch_spp > 0 ? prm->batch_spp : 0;
    if (batch <= 0) {
        const size_t per_sample = 3 * sizeof(float) * (size_t)std::max(npix, 1);
        batch = (int)std::max<size_t>(1, batch_bytes_budget() / per_sample);
    }
    batch = std::max(1, std::min(batch, std::max(spp, 1)));
    const int per_item = prm->samples_per_item > 0 ? std::min(prm->samples_per_item, batch) : std::min(2, batch);

    int rc;
    if ((rc = ensure(&c->d_radiance, &c->radiance_floats, 3 * (size_t)batch * npix))) return rc;
    if ((rc = ensure(&c->d_accum, &c->accum_floats, 3 * (size_t)npix))) return rc;
    float* dst = out;
    if (!out_is_device) {
        if ((rc = ensure(&c->d_out, &c->out_floats, 3 * (size_t)npix))) return rc;
        dst = c->d_out;
    }

    const int rec = std::max(1, prm->depth - 1);
    const int stack = std::max(1, c->meta.tree_depth);
    const int node4 = 2 * c->meta.num_nodes, tri4 = 3 * c->meta.num_tris, mat4 = 2 * c->meta.num_tris;
    const size_t work_lds = sizeof(int) * (size_t)kBlock * (stack + 2 * rec);
    // Flat leaf list for scenes with <= 64 leaves (Cornell: 32); PT_FLAT=0 disables it.
    const char* fenv = getenv("PT_FLAT");
    const bool flat = c->meta.num_leaves > 0 && c->meta.num_leaves <= kMaxFlatLeaves && !(fenv && *fenv == '0');
    const int leaf4 = flat ? 2 * c->meta.num_leaves : 0;
    const size_t scene_lds = sizeof(float4) * ((size_t)node4 + tri4 + mat4 + leaf4);
    // Small scenes (Cornell: 5.6 KB) live in LDS; big ones are read through L1/L2/MALL.
    const bool lds_scene = flat || (scene_lds <= lds_scene_budget() && scene_lds + work_lds <= 64 * 1024);
    const size_t lds_bytes = work_lds + (lds_scene ? scene_lds : 0);
    if (lds_bytes > 160 * 1024)
        return set_error(PT_E_ARG, "BVH depth (%d) x path depth needs %zu B of LDS", stack, lds_bytes);
    auto kern = flat ? pt_trace_kernel<true, true> : lds_scene ? pt_trace_kernel<true, false> : pt_trace_kernel<false, false>;
    int blocks_per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks_per_cu, kern, kBlock, lds_bytes));
    blocks_per_cu = std::max(1, blocks_per_cu);

    TraceArgs A;
    memset(&A, 0, sizeof(A));
    A.nodes = c->d_nodes;
    A.tris = c->d_tris;
    A.mats = c->d_mats;
    A.leaves = c->d_leaves;
    A.num_leaves = flat ? c->meta.num_leaves : 0;
    A.num_leaves_padded = (A.num_leaves + 3) & ~3;
    for (int k = 0; k < A.num_leaves_padded; k++) {
        const f4* L = &c->flat_host[2 * (k < A.num_leaves ? k : 0)];
        const float b6[6] = {L[0].x, L[0].y, L[0].z, L[0].w, L[1].x, L[1].y};
        memcpy(A.flat.box[k], b6, sizeof(b6));
    }
    A.radiance = c->d_radiance;
    A.ctr = c->d_ctr;
    A.pos_x = cam->pos[0];
    A.pos_y = cam->pos[1];
    A.pos_z = cam->pos[2];
    const float* T = cam->transform;  // rows right, up, -forward; columns feed get_ray's dots
    A.col0_x = T[0]; A.col0_y = T[3]; A.col0_z = T[6];
    A.col1_x = T[1]; A.col1_y = T[4]; A.col1_z = T[7];
    A.col2_x = T[2]; A.col2_y = T[5]; A.col2_z = T[8];
    A.vres_x = cam->v_res[0];
    A.vres_y = cam->v_res[1];
    A.cell = cam->cell_size;
    A.dist = cam->distance;
    A.W = W;
    A.npix = npix;
    A.part_index = prm->part_index;
    A.part_count = parts;
    A.band_rows = band;
    A.depth = prm->depth;
    A.seed = prm->seed;
    A.per_item = per_item;
    A.stack_size = stack;
    A.rec_size = rec;
    A.num_node4 = node4;
    A.num_tri4 = tri4;
    A.num_mat4 = mat4;
    {
        const char* fe = getenv("PT_FORCE_EXACT_SLAB");
        A.force_exact_slab = (fe && *fe == '1') ? 1 : 0;
    }

    HIP_TRY(hipMemsetAsync(c->d_ctr, 0, 4 * sizeof(unsigned long long), c->stream));
#ifdef PT_STAMPS
    if (!c->d_stamps) HIP_TRY(hipMalloc((void**)&c->d_stamps, kStampSections * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(c->d_stamps, 0, kStampSections * sizeof(unsigned long long), c->stream));
    A.stamps = c->d_stamps;
#endif
    std::vector<hipEvent_t> ev;
    auto cleanup = [&]() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    };
    int launches = 0;
    const int acc_grid = (npix + kBlock - 1) / kBlock;
    if (spp == 0 || npix == 0) {
        if (npix > 0) {
            // No samples: the reference divides the zero image by 0 (render.h:97).
            hipLaunchKernelGGL(pt_accumulate_kernel, dim3(acc_grid), dim3(kBlock), 0, c->stream, c->d_radiance,
                               c->d_accum, dst, npix, 0, 1, 1, (float)spp);
        }
    }
    for (int s0 = 0; s0 < spp && npix > 0; s0 += batch) {
        const int sc = std::min(batch, spp - s0);
        A.s_begin = s0;
        A.s_count = sc;
        const unsigned long long blocks_of_samples = (unsigned long long)((sc + per_item - 1) / per_item);
        A.total_items = blocks_of_samples * (unsigned long long)npix;
        const unsigned long long want_blocks = (A.total_items + kBlock - 1) / kBlock;
        const int grid = (int)std::min<unsigned long long>(want_blocks, (unsigned long long)blocks_per_cu * c->num_cus);
        hipEvent_t e0, e1, e2;
        if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess ||
            hipEventCreate(&e2) != hipSuccess) {
            cleanup();
            return set_error(PT_E_HIP, "hipEventCreate failed");
        }
        ev.push_back(e0);
        ev.push_back(e1);
        ev.push_back(e2);
        (void)hipMemsetAsync(c->d_ctr, 0, sizeof(unsigned long long), c->stream);  // work head only
        (void)hipEventRecord(e0, c->stream);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds_bytes, c->stream, A);
        (void)hipEventRecord(e1, c->stream);
        hipLaunchKernelGGL(pt_accumulate_kernel, dim3(acc_grid), dim3(kBlock), 0, c->stream, c->d_radiance,
                           c->d_accum, dst, npix, sc, s0 == 0 ? 1 : 0, s0 + sc >= spp ? 1 : 0, (float)spp);
        (void)hipEventRecord(e2, c->stream);
        launches++;
    }
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
        cleanup();
        return set_error(PT_E_HIP, "kernel launch failed: %s", hipGetErrorString(le));
    }
    unsigned long long h_ctr[4] = {0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(h_ctr, c->d_ctr, sizeof(h_ctr), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && !out_is_device)
        e = hipMemcpyAsync(out, dst, 3 * (size_t)npix * sizeof(float), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        cleanup();
        return set_error(PT_E_HIP, "render failed: %s", hipGetErrorString(e));
    }
#ifdef PT_STAMPS
    {
        unsigned long long hs[kStampSections];
        if (hipMemcpy(hs, c->d_stamps, sizeof(hs), hipMemcpyDeviceToHost) == hipSuccess) {
            const double tot = (double)(hs[0] + hs[1] + hs[2] + hs[3]);
            fprintf(stderr,
                    "[stamps] waves %llu  cycles/wave %.3g  start %.1f%%  traverse %.1f%% (flat box loop %.1f%%)  "
                    "shade %.1f%%  fold %.1f%%\n",
                    hs[5], tot / (double)(hs[5] ? hs[5] : 1), 100 * hs[0] / tot, 100 * hs[1] / tot,
                    100 * hs[4] / tot, 100 * hs[2] / tot, 100 * hs[3] / tot);
        }
    }
#endif
    double kms = 0, rms = 0;
    for (size_t i = 0; i + 2 < ev.size(); i += 3) {
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, ev[i], ev[i + 1]);
        (void)hipEventElapsedTime(&b, ev[i + 1], ev[i + 2]);
        kms += a;
        rms += b;
    }
    cleanup();
    if (stats) {
        stats->rays = h_ctr[1];
        stats->paths = (uint64_t)spp * (uint64_t)npix;
        stats->runaway = h_ctr[3];
        stats->kernel_ms = kms;
        stats->reduce_ms = rms;
        stats->trace_launches = launches;
        stats->rows = rows;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    if (h_ctr[3] != 0)
        return set_error(PT_E_RUNAWAY, "%llu specular rejection loops hit the %d-iteration bound", h_ctr[3],
                         kMaxSpecularIters);
    return PT_OK;
}

int pt_render_f32(const pt_scene* scene, const pt_camera* cam, const pt_params* params, float* out_rgb,
                  pt_stats* stats) {
    if (!params) return set_error(PT_E_ARG, "params is NULL");
    if (scene && scene->num_tris <= 0) return set_error(PT_E_EMPTY, "No triangles in scene.");
    pt_ctx* c = nullptr;
    int rc = pt_ctx_create(0, &c);
    if (rc) return rc;
    rc = pt_ctx_set_scene(c, scene);
    if (!rc) {
        pt_params p = *params;
        p.part_index = 0;
        p.part_count = 1;
        if (p.band_rows <= 0) p.band_rows = 1;
        rc = pt_ctx_render(c, cam, &p, out_rgb, 0, stats);
    }
    pt_ctx_destroy(c);
    return rc;
}

// GPU copies of the math primitives (test hook): which = 0 acosf, 1 sincosf, 2 BRDF.
int pt_debug_math(int device, int which, const float* in, int n, float* out) {
    if (!in || !out || n <= 0 || which < 0 || which > 2) return set_error(PT_E_ARG, "pt_debug_math: bad argument");
    HIP_TRY(hipSetDevice(device));
    const size_t in_n = (size_t)n * (which == 2 ? 9 : 1), out_n = (size_t)n * (which == 0 ? 1 : which == 1 ? 2 : 4);
    float *di = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc((void**)&di, in_n * sizeof(float)));
    if (hipMalloc((void**)&dout, out_n * sizeof(float)) != hipSuccess) {
        (void)hipFree(di);
        return set_error(PT_E_HIP, "hipMalloc failed");
    }
    hipError_t e = hipMemcpy(di, in, in_n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(pt_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, which, di, dout, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, out_n * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(di);
    (void)hipFree(dout);
    if (e != hipSuccess) return set_error(PT_E_HIP, "pt_debug_math: %s", hipGetErrorString(e));
    return PT_OK;
}

}  // extern "C"
