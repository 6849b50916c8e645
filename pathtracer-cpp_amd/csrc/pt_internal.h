// pt_internal.h — declarations shared by pt_host.cpp (host C++) and pt_kernel.hip.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "pt_hip.h"

namespace pt {

// Record the error message of the calling thread and return `code`.
int set_error(int code, const char* fmt, ...);

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
//   wide: the binary tree collapsed into nodes of `wide_width` (4 or 8) children, built
//          only when the flat-leaf argument holds (partition + containment). Per node
//          `wide_width * 2` float4, fields SoA across the children:
//          lb.x[W] lb.y[W] lb.z[W] rt.x[W] rt.y[W] rt.z[W] ref[W] last[W]
//          child box = the reference's own node box (exact; leaf boxes decide which
//          triangles are tested). ref >= 0: wide node index; leaf: ref = -(first+1),
//          last = last rank position; empty slot: ref = INT32_MIN. Root = wide node 0.
struct PackedScene {
    std::vector<f4> nodes, tris, mats, leaves, wide;
    int32_t num_leaves = 0;
    int32_t num_wide = 0, wide_width = 0;
    int32_t wide_depth = 0;  // max pending (node, child mask) entries of the wide walk
    int32_t num_nodes = 0, num_tris = 0;
    int32_t stack_size = 0;  // max LIFO occupancy of BVH::intersect over this tree
    int32_t tree_depth = 0;  // max root-to-leaf edge count (child-pair traversal stack bound)
};

// Validate the node graph and pack it. Returns PT_OK or an error code.
int pack_scene(const pt_scene* s, PackedScene& out);

}  // namespace pt
