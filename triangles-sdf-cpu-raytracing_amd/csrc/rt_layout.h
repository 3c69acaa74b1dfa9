// rt_layout.h -- device-resident scene layouts (HBM) shared by the host
// scene builder (rt_host.cpp) and the HIP kernels (rt_device.hip).
//
// The layouts are re-designed for one-thread-per-pixel traversal on CDNA4;
// they carry exactly the values the reference computes with, so the kernels
// reproduce the reference arithmetic bit for bit:
//
//  * GNode: one BVH8 INNER node (triangles_raytracing.hpp:10-36). The reference
//    node is Box8 SoA (192 B) + realCount + offset, with leaves as separate
//    nodes. Here a node carries its 8 child boxes in AoS order (child c at
//    box[c][0..5]: xMin xMax yMin yMax zMin zMax -- the same floats as the
//    reference Box8, the min/max of an axis adjacent so a slab pair is one
//    64-bit register pair for the packed-math unit) and 8 child WORDS; a
//    leaf child is referenced directly by its triangle range, so leaves cost
//    no node fetch. Unused slots
//    (c >= realCount) hold +inf boxes: under the ISPC slab formula
//    (ray_pack.ispc:241-273) such a box always yields -1 (miss), so the kernel
//    may compute or skip them identically. 224 B = 7 x 32 B.
//  * GTri: one triangle in leaf order: v0 (after the reference's /w,
//    triangles_raytracing.cpp:307-309), e1 = v1-v0, e2 = v2-v0 (the first ops
//    of ray_pack.ispc:140-141, exact float subtractions done once on the host)
//    and the original triangle index (OBJ face order) in v0's w slot.
//  * Octree: SoA split of the 36-byte SDFOctreeNode (octree_raytracing.hpp:8-18)
//    into child words (4 B/node, all an inner-node visit needs) and 32-B
//    aligned corner values (read only at leaves).
#pragma once
#include <stdint.h>

namespace rtl {

constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kInvalidChild = 0xFFFFFFFFu;
// leaf child word: kLeafBit | (first_tri << 3) | (ntri - 1), ntri in [1, 8]
constexpr uint32_t kMaxLeafFirstTri = (1u << 28) - 1u;

struct alignas(32) GNode {
  float box[8][6];
  uint32_t child[8];
};
static_assert(sizeof(GNode) == 224, "GNode must be 224 bytes");

struct alignas(16) GTri {
  float v0x, v0y, v0z;
  uint32_t orig_id;
  float e1x, e1y, e1z, pad1;
  float e2x, e2y, e2z, pad2;
};
static_assert(sizeof(GTri) == 48, "GTri must be 48 bytes");

// Octree child word: 0 = leaf that can hit (march it); kOctNeverHits = leaf
// that the reference rejects before marching (isEmpty() or every corner
// >= HIT_EPS, octree_raytracing.cpp:125-133); otherwise childrenOffset.
constexpr uint32_t kOctNeverHits = 0xFFFFFFFFu;

// Device word of an octree node: `child` as above, and for an inner node the
// masks of its 8 children (bit k = child id k, (x<<2)|(y<<1)|z):
//   bits 0-7  the child's subtree can produce a hit (a leaf that can hit, or an
//             inner node with such a leaf below it); the reference's recursion
//             into any other child returns false whatever the ray
//             (octree_raytracing.cpp:122-133, 166-202), so the traversal may skip it;
//   bits 8-15 the child is a leaf that can hit (march it without loading its word).
struct alignas(8) OctWord {
  uint32_t child;
  uint32_t masks;
};

struct alignas(32) OctVals {
  float v[8];
};

}  // namespace rtl
