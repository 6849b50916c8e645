// pt_internal.h — declarations shared by pt_host.cpp (host C++) and pt_kernel.hip.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "pt_hip.h"

namespace pt {

// Record the error message of the calling thread and return `code`.
int set_error(int code, const char* fmt, ...);

// Test / tuning hooks (PT_FLAT, PT_WIDE, PT_PAIRS, PT_BATCH_BYTES, ...): the value of
// environment variable `name`, or nullptr. Hooks are honoured only when PT_TEST_HOOKS=1
// was set when the library first looked (once per process), so a stray variable in a
// user's environment never changes which kernel or queue size the product runs.
const char* hook_env(const char* name);

struct f4 {
    float x, y, z, w;
};

// Device layout of a scene (see DESIGN.md "Data layout in HBM"):
//   nodes: 2 x f4 per node   {lb.xyz, rt.x}, {rt.y, rt.z, a, b}, renumbered so that the two
//          children of every interior node are adjacent (left = a, right = a + 1; the
//          reference builder already emits them so, bvh.h:142-152). Root = node 0.
//          interior: a = left (>= 1), b = 0; leaf: a = -(tri_start+1), b = tri_end
//          (bit-cast ints). Traversal order depends only on the tree, not on numbering.
//   tris : 3 x f4 per tri_idx POSITION i (triangle tri_idx[i]):
//          {v1.xyz, e1.x}, {e1.yz, e2.xy}, {e2.z, n.xyz}   e1 = v2-v1, e2 = v3-v1,
//          n = normalize(cross(e1, e2)) (triangle.h:28-29, 46-47), computed on the host
//   mats : 2 x f4 per position {type, color.rgb}, {emit.rgb, roughness}
//   Triangle positions are renumbered into the reference's visit RANK: the order in
//   which BVH::intersect would test them if every box passed (right subtree first,
//   bvh.h:177-178; ascending tri_idx position inside a leaf). The first strict minimum
//   in rank order is then the reference's winner for any traversal order.
//   leaves: 2 x f4 per leaf in rank order {lb.xyz, rt.x}, {rt.y, rt.z, first, last}
//          (first/last = rank positions, bit-cast ints) — the flat leaf list.
//   wide: the binary tree collapsed into nodes of `wide_width` (4 or 8) children with
//          quantised child boxes, built only when the flat-leaf argument holds
//          (partition + containment). Nodes in BFS order (root 0; the first levels
//          form an index prefix, staged in LDS by the kernel); the inner children of a
//          node are consecutive nodes from child_base, slots [0, ni); its leaf children
//          follow in slots [ni, ni + nl), their triangles consecutive in `wtris` from
//          leaf_base. Per node kWideNodeU4[W] uint4:
//            [0] O.x O.y O.z (float), meta = (ex+128) | (ey+128) << 8 | (ez+128) << 16
//                | ni << 24 | nl << 28
//            [1] child_base, leaf_base, end[0..3], end[4..7] (bytes: cumulative end
//                offset of leaf k's triangles from leaf_base)
//            [2..] per axis a (x, y, z), `wide_fmt` kWideF16 (default): binary16 integers
//                lo.a[W] hi.a[W] in 0..2047, so a ray reads its entry run at lo or hi
//                and its exit run at the other (the sign of its 1 / d); otherwise bytes
//                lo.a[W] hi.a[W] hi.a[W] lo.a[W] in 0..255, one (entry, exit) run.
//                8-wide: 128 B per node, one cache line, in either format.
//          Child box on axis a: [O + lo * 2^e, O + hi * 2^e] (reals), containing the
//          reference's child box; the kernel's test is conservative,
//          exactness comes from the exact leaf box checked on every triangle hit.
//          `wide_fmt` kWideF32 (round 6): no quantisation — the child
//          planes are the reference's own float boxes. Per node 1 + 3 W / 2 uint4:
//            [0] child_base | ni << 24 | nl << 28, leaf_base, end[0..3], end[4..7]
//            [1..] per axis a: lo.a[W] hi.a[W] (float; an empty slot lo = +inf, hi = -inf)
//          8-wide: 208 B per node; 4-wide: 112 B.
//   wtris: 4 x f4 per triangle in wide-leaf order: {v1.xyz, e1.x}, {e1.yz, e2.xy},
//          {e2.z, rank (bits), leaf lb.xy}, {leaf lb.z, leaf rt.xyz}; or, when every
//          leaf holds one triangle (`wide_compact`), 3 x f4: {v1.xyz, rank (bits)},
//          {v2.xyz, v3.x}, {v3.yz, 0, 0} (edges and the leaf box formed by the kernel).
//   nrm  : (wide path) 1 x f4 per rank position {n.xyz, material id (bits)}: the shading
//          normal and the row of the triangle's material in `umats`
//   umats: (wide path) 2 x f4 per DISTINCT material, same layout as `mats` (the wide
//          kernel keeps them in LDS when there are at most kMaxLdsMaterials)
// Child-plane formats of the wide tree.
constexpr int kWideByte = 0, kWideF16 = 1, kWideF32 = 2;
constexpr int kWideNodeU4(int W, int fmt) { return fmt == kWideF32 ? 1 + 3 * W / 2 : W == 8 ? 8 : 5; }
constexpr int kMaxLdsMaterials = 64;
// With the table in LDS the path records hold a material row in ONE byte (trace_body_wide):
// the LDS form is only ever chosen for at most kMaxLdsRowsByte rows, whatever the tuning hook.
constexpr int kMaxLdsRowsByte = 256;
static_assert(kMaxLdsMaterials <= kMaxLdsRowsByte, "LDS material rows must fit the 8-bit path records");
// LDS per CU the blocks of one kernel can count on, and the granule a block's LDS is
// rounded to: 6 blocks of 26,816 B run together, 6 of 27,072 B do not (measured on the wide
// kernel on gfx950 / MI355X, profiles/r03z_lds), although 160 KiB would hold them. Applied
// only on that architecture, and never above the device's reported LDS per CU
// (lds_usable_per_cu, pt_kernel.hip).
constexpr size_t kLdsUsable = 161280;
constexpr size_t kLdsGranule = 256;
constexpr int kPairQueueMin = 256;  // shortest flat pair queue (entries per wave) the launch picks for occupancy

struct PackedScene {
    std::vector<f4> nodes, tris, mats, leaves, wide, wtris, nrm, umats;
    int32_t num_umats = 0;
    int32_t num_leaves = 0;
    int32_t num_wide = 0, wide_width = 0;
    int32_t wide_depth = 0;  // wide levels; the walk holds at most wide_depth - 1 pending stack entries
                             // (one per level above the current node; the last level has no inner nodes)
    int32_t wide_top = 0;    // nodes of the first wide levels that fit the LDS top-of-tree budget
    int32_t wide_fmt = kWideByte;  // child planes: bytes 0..255, binary16 integers 0..2047, or floats
    float wide_span[3] = {0, 0, 0};  // kWideF32: max |plane| per axis (the per-ray margin's bound)
    bool wide_single = false;  // every wide leaf holds exactly one triangle (BVH::build's output)
    bool wide_compact = false;  // wtris holds the 3-f4 records of single-triangle leaves
    int32_t num_nodes = 0, num_tris = 0;
    int32_t stack_size = 0;  // max LIFO occupancy of BVH::intersect over this tree
    int32_t tree_depth = 0;  // max root-to-leaf edge count (child-pair traversal stack bound)
    bool coords_small = false;  // every vertex coordinate below 2^60 in magnitude (tri_hit_nb's precondition)
};

// Validate the node graph and pack it. Returns PT_OK or an error code.
int pack_scene(const pt_scene* s, PackedScene& out);

// A context's HIP stream (hipStream_t) and device gamma/quantisation (pt_kernel.hip):
// `rows` x W linear pixels at d_lin -> bytes at d_dst (flip: last row first); synchronous.
void* ctx_stream(pt_ctx* c);
int rgb8_device(pt_ctx* c, const float* d_lin, int rows, int W, float gamma, int flip, uint8_t* d_dst);
// The flat path's table kernel with a scene's flags baked in (pt_flat_fast.hip): every leaf one
// triangle, coordinates below 2^60, a dark scene with pre-doubled albedo; `specular`: the scene
// holds a SPECULAR material, `mask32`: at most 32 leaves. A __global__ function's address.
void* flat_fast_kernel(bool specular, bool mask32);
// Free a context's radiance slabs and flag words (allocated again by its next render).
int ctx_release_slabs(pt_ctx* c);
// pt_debug_counter's context counters (pt_kernel.hip): 0 contexts created, 1 scene uploads.
int64_t kernel_counter(int which);

}  // namespace pt
