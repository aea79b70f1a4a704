// bvh_build.h -- host-side binned-SAH BVH2 builder for the device scene (replaces the reference's
// SAH kd-tree build, KdTree.hs:107-203, which stays in the oracle).  Node format: dev_scene.h.
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

namespace bvh {

struct Box { float lo[3], hi[3]; };

struct Result {
  std::vector<float> nodes;      // 16 floats per node
  std::vector<uint32_t> refs;    // leaf slots
  int depth = 0, leaves = 0, max_leaf = 0;
};

// boxes[i] bounds item i whose leaf reference word is refs_in[i].
// Throws std::runtime_error if a leaf would exceed 255 items at the depth cap.
Result build(const std::vector<Box>& boxes, const std::vector<uint32_t>& refs_in, int max_leaf = 4,
             int max_depth = 31);

// The same BVH2 as a threaded depth-first entry list for wave-coherent (packet) traversal: one
// entry per non-empty child box, 8 words each: lo.xyz, hi.xyz, leaf code (~(first << 8 | count),
// the BVH2 link) or -1 for an inner entry, skip = index of the entry after its subtree.  An inner
// entry's first child is the next entry; entries.size() / 8 ends the walk.
std::vector<float> threaded(const Result& R);

// The same BVH2 collapsed into a 4-wide BVH (dev_scene.h, 28 floats = 7 float4 per node): each node
// takes its BVH2 children and repeatedly opens the inner child with the largest surface area until
// it has four (or only leaves are left).  Child k's box is lo.x/lo.y/lo.z/hi.x/hi.y/hi.z in lane k
// of words 0-5; word 6 holds the four links (>= 0 inner node, leaf code ~(first << 8 | count) as in
// the BVH2, EMPTY4 for an unused slot).  Leaf codes and the leaf-ref array are the BVH2's.  Nodes are
// breadth-first (LDS prefix).  stack_need bounds the traversal stack: the largest sum over a
// root-to-node chain of (hit children - 1) pushed at each node.
constexpr int32_t EMPTY4 = (int32_t)0x80000000;
struct Result4 {
  std::vector<float> nodes;      // 28 floats per node
  int depth = 0, stack_need = 0;
};
Result4 collapse4(const Result& R);

// The same BVH4 with its child boxes quantized to one byte per plane: 16 words (4 float4 = 64 B, not
// 112) per node -- words 0-2 the node's origin (its children's lowest corner), 3-5 the per-axis scale
// 2^e, 6-8 the children's lo.x / lo.y / lo.z bytes (child k in byte k), 9-11 the hi bytes, 12-15 the
// links as in collapse4.  A plane decodes as dequant(q, scale, origin): q x 2^e is exact, the sum
// rounds once, on the host as on the device (dev_trace.h Traversal4).  Each q is chosen so the
// decoded plane lies outside the float box (lo rounds down, hi up): a superset, so the traversal
// finds every hit the float tree finds.  An empty slot holds lo bytes 255, hi 0 (its link marks it).
// Throws std::runtime_error on a box that cannot be encoded (non-finite bounds).
std::vector<uint32_t> quantize4(const Result4& Q);
inline float dequant(uint32_t q, float scale, float origin) { return std::fmaf((float)q, scale, origin); }

}  // namespace bvh
