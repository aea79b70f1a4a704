// dev_scene.h -- HBM layout of the flattened scene on the MI355X (all SoA / 16-B aligned records).
//
//  BVH2 nodes        4 x float4 per node (64 B): both children's AABBs + child links, so one node
//                    fetch tests two boxes.  child link >= 0: inner node; < 0: leaf = ~(first<<8|count)
//  leaf refs         u32 per leaf slot: (kind << 30) | local index   (kind 0 tri, 1 shape, 2 fractal)
//  tri_geo           3 x float4 per triangle: v0.xyz e1.x | e1.yz e2.xy | e2.z - - -  (48 B, the
//                    Moller-Trumbore inputs of TriangleMesh.hs:140-207; e1 = p2 - p1, e2 = p3 - p1)
//  tri_pts           9 floats per triangle (p1 p2 p3, for hit reconstruction at shade time)
//  shapes            DevShape records (w2o used by traversal, o2w by shading)
#pragma once
#include <stdint.h>
#include "../../../include/bling_scene.h"

namespace bd {

constexpr uint32_t REF_TRI = 0u, REF_SHAPE = 1u, REF_FRACTAL = 2u;
constexpr uint32_t REF_NONE = 0xFFFFFFFFu;

struct DevShape {
  int32_t kind, material, light, prim;
  float params[4];
  float w2o[16];
  float o2w[16];
};

struct DevScene {
  // acceleration structure
  const float4* nodes;
  const uint32_t* leaf_refs;
  uint32_t num_nodes;
  // geometry
  const float4* tri_geo;
  const float* tri_pts;
  const float* tri_uvs;
  const float* tri_normals;     // nullptr if no mesh has shading normals
  const uint8_t* tri_has_n;
  const int32_t* tri_material;
  const int32_t* tri_prim;      // triangle -> reference prim id
  const DevShape* shapes;
  bling_fractal fractal;
  int32_t fractal_prim;
  // appearance
  const bling_material* materials;
  const bling_texture* textures;
  const bling_light* lights;    // dist pointers rewritten to device memory
  int32_t num_lights;
  bling_camera camera;
  float filter_table[256];
  float filter_w, filter_h;
  // render configuration
  int32_t sampler, nu, nv, spp, max_depth, sample_depth;
  int32_t width, height;
  int32_t ex0, ex1, ey0, ey1, ext_w;
};

}  // namespace bd
