// bvh_build.h -- host-side binned-SAH BVH2 builder for the device scene (replaces the reference's
// SAH kd-tree build, KdTree.hs:107-203, which stays in the oracle).  Node format: dev_scene.h.
#pragma once
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

}  // namespace bvh
