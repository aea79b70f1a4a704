// dev_scene.h -- HBM layout of the flattened scene on the MI355X (all SoA / 16-B aligned records).
//
//  BVH2 nodes        4 x float4 per node (64 B): both children's AABBs + child links, so one node
//                    fetch tests two boxes.  child link >= 0: inner node; < 0: leaf = ~(first<<8|count)
//  BVH4 nodes        7 x float4 per node (112 B), the same tree 4-wide (bvh::collapse4, Traversal4),
//                    (4 x float4 = 64 B quantized, bvh::quantize4, in BLING_QBVH4 experiment builds)
//  leaf refs         u32 per leaf slot: (kind << 30) | local index   (kind 0 tri, 1 shape, 2 fractal)
//  tri_geo           3 x float4 per triangle: v0.xyz e1.x | e1.yz e2.xy | e2.z - - -  (48 B, the
//                    Moller-Trumbore inputs of TriangleMesh.hs:140-207; e1 = p2 - p1, e2 = p3 - p1)
//  tri_frame         4 float4 per triangle: dpdu, dpdv, normal, uvs (dev_shade.h tri_frame_build)
//  shapes            DevShape records (w2o used by traversal, o2w by shading)
#pragma once
#include <stdint.h>
#include "../../../include/bling_scene.h"

namespace bd {

// Pointers into HBM are typed: fields loaded from the DevScene record would otherwise be generic
// pointers and every access a FLAT load (slower issue, and each one waits on both vmcnt and
// lgkmcnt).  Scene memory is never written while a kernel runs, so (BLING_SCENE_CONST, the default)
// it is typed constant (address space 4): no store of the kernel can alias it, so its loads may be
// scheduled and reused across the path-state stores, and a wave-uniform address becomes a scalar
// load; address space 1 (global) otherwise.
#ifndef BLING_SCENE_CONST
#define BLING_SCENE_CONST 1
#endif
#if BLING_SCENE_CONST
#define BLING_SCENE_AS 4
#else
#define BLING_SCENE_AS 1
#endif
template <class T>
using gptr = const __attribute__((address_space(BLING_SCENE_AS))) T*;

template <class T>
__host__ __device__ inline gptr<T> as_global(const T* p) { return (gptr<T>)p; }

// Back to generic pointers / references for helpers that take plain C++ types; after inlining the
// address-space inference pass sees through the cast and keeps the typed loads.
template <class T>
__device__ __forceinline__ const T* gen(gptr<T> p) { return (const T*)p; }
template <class T>
__device__ __forceinline__ const T& gen(const __attribute__((address_space(BLING_SCENE_AS))) T& r) { return *(const T*)&r; }

// Scene feature set.  Every kernel is instantiated for a few feature profiles (core.hip); a scene
// runs on the smallest profile that covers what it uses, so BSDF / light / shape code the scene can
// never reach is not compiled into its kernels (register pressure and code size of k_shade).
enum : uint32_t {
  FT_MATTE = 1u << 0, FT_PLASTIC = 1u << 1, FT_GLASS = 1u << 2, FT_METAL = 1u << 3, FT_MIRROR = 1u << 4,
  FT_GRAPHPAPER = 1u << 5, FT_AREA = 1u << 6, FT_ENV_CONST = 1u << 7, FT_ENV_SKY = 1u << 8,
  FT_SPHERE = 1u << 9, FT_TRI_NORMALS = 1u << 10, FT_FRACTAL = 1u << 11, FT_TRIS = 1u << 12,
  FT_SHAPES2 = 1u << 13,      // disk, cylinder, box (Shape.hs:86-155)
  FT_TRANSMATTE = 1u << 14,   // translucentMatte: Lambert / OrenNayar BRDF + BTDF
  FT_SHINYMETAL = 1u << 15,   // mkShinyMetal: conductor microfacet + conductor specular reflection
  FT_SUBSTRATE = 1u << 16,    // mkSubstrate: FresnelBlend lobe, anisotropic distribution
  FT_BUMP = 1u << 17,         // bumpMapped materials (shading frame from a displacement texture)
  FT_PROCTEX = 1u << 18,      // per-hit computed spectra (blend / gradient / checker), cellNoise
  FT_DELTA = 1u << 19,        // point / directional lights
  FT_ENV_IMG = 1u << 20,      // infinite lights with an image map (l { file "x.hdr" })
  FT_MULTI_LIGHT = 1u << 21,  // more than one light: profiles without it assume light 0 (one_light)
  FT_ALL = (1u << 22) - 1u
};
// Profiles without FT_MULTI_LIGHT serve scenes with at most one light: the sampled light (and a hit
// light) is light 0 in every lane, so its record and its shape's are wave-uniform and are read
// through the constant address space -- scalar loads into SGPRs, once per wave -- instead of a
// vector load per lane (light_rec, light_shape).  Scene records are never written while a kernel runs.
template <uint32_t F>
constexpr bool one_light() { return !(F & FT_MULTI_LIGHT); }
template <class T>
using cptr = const __attribute__((address_space(4))) T*;
constexpr uint32_t FT_INF = FT_ENV_CONST | FT_ENV_SKY | FT_ENV_IMG;
constexpr uint32_t FT_OREN = FT_MATTE | FT_TRANSMATTE;                 // OrenNayar lobes
constexpr uint32_t FT_DIFFUSE = FT_MATTE | FT_PLASTIC | FT_TRANSMATTE;  // Lambertian / OrenNayar lobes
constexpr uint32_t FT_MICRO = FT_PLASTIC | FT_METAL | FT_SHINYMETAL;
constexpr uint32_t FT_COND = FT_METAL | FT_SHINYMETAL;                 // conductor Fresnel
constexpr uint32_t FT_SREFL = FT_GLASS | FT_MIRROR | FT_SHINYMETAL;    // specular reflection lobes
constexpr uint32_t FT_TWO_LOBES = FT_PLASTIC | FT_GLASS | FT_TRANSMATTE | FT_SHINYMETAL;
constexpr uint32_t FT_NONQUAD = FT_SPHERE | FT_SHAPES2;                // shapes other than quads

constexpr uint32_t REF_TRI = 0u, REF_SHAPE = 1u, REF_FRACTAL = 2u;
// entries - 1 of the guide table behind each Dist2D CDF on the device (core.hip, sample_c1d)
constexpr int kCdfGuide = 64;
constexpr uint32_t REF_NONE = 0xFFFFFFFFu;

struct DevShape {
  int32_t kind, material, light, prim;
  float params[8];
  float w2o[16];
  float o2w[16];
};

// Exact unsigned 32-bit division by a run-time constant (Granlund-Montgomery round-up method):
// q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(m, n), l = ceil(log2 d), m = 2^32 (2^l - d) / d + 1.
// Exact for every 32-bit n (verified exhaustively over d in tests/test_rng_loader.py); replaces
// the ~40-instruction integer division of `quot`/`rem` by spp and nu on the sampler's hot path.
struct FastDiv {
  uint32_t d, m, s;                 // s = l - 1; d == 1 is the identity (m unused)
  __host__ static FastDiv make(uint32_t d) {
    FastDiv f{d, 0u, 0u};
    if (d > 1) {
      uint32_t l = 32u - (uint32_t)__builtin_clz(d - 1u);
      f.m = (uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1u);
      f.s = l - 1u;
    }
    return f;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    if (d == 1u) return n;
    uint32_t t = __umulhi(m, n);
    return (t + ((n - t) >> 1)) >> s;
  }
  __device__ __forceinline__ uint32_t mod(uint32_t n) const { return n - div(n) * d; }
};

struct DevScene {
  // acceleration structure
  gptr<float4> nodes;
  gptr<uint32_t> leaf_refs;
  gptr<float4> leaf_geo;        // per leaf slot: the primitive's record with its ref (dev_trace.h LeafRec)
  uint32_t num_nodes;
  // geometry
  gptr<float4> tri_geo;
  gptr<float4> tri_frame;
  gptr<float> tri_normals;      // nullptr if no mesh has shading normals
  gptr<uint8_t> tri_has_n;
  gptr<int32_t> tri_material;
  gptr<int32_t> tri_prim;       // triangle -> reference prim id
  gptr<DevShape> shapes;
  bling_fractal fractal;
  int32_t fractal_prim;
  float fractal_pw[32];         // (float)(order^k), k = 0..31, as Int (64-bit) powers (Fractal.hs:97)
  // appearance
  gptr<bling_material> materials;
  gptr<bling_texture> textures;
  gptr<bling_scalar_texture> stex;   // scalar textures evaluated at a hit (substrate parameters)
  gptr<bling_image> images;     // texture images, texel pointers rewritten to device memory
  gptr<bling_light> lights;     // dist pointers rewritten to device memory
  int32_t num_lights;
  bling_camera camera;
  float filter_table[256];
  float filter_w, filter_h;
  // render configuration
  int32_t sampler, nu, nv, spp, max_depth, sample_depth;
  int32_t integrator;           // bling_integrator_kind
  int32_t n1d, n2d;             // stratified dimensions the integrator requests (Path 4 sd / 3 sd, DL 2 md)
  FastDiv fd_spp, fd_nu;        // exact quot/rem by spp and nu
  uint32_t perm_mask_spp;       // Kensler permutation mask for l = spp
  float inv_spp, inv_nu, inv_nv;   // 1 / (float)spp etc., rounded once on the host (binary32)
  int32_t width, height;
  int32_t ex0, ex1, ey0, ey1, ext_w;
  // LDS plan of the traversal kernels (core.hip: plan_lds): BFS prefix of the nodes, and the whole
  // triangle / leaf-ref arrays when they fit, copied into dynamic LDS at block start; stack rows.
  uint32_t lds_nodes, lds_tris, lds_refs, stack_depth;
  // The same tree collapsed to 4 children per node (bvh::collapse4; 7 float4 = 112 B per node: the
  // four child boxes as lo.x / lo.y / lo.z / hi.x / hi.y / hi.z quads, then the four links; BLING_QBVH4
  // experiment builds: bvh::quantize4's 4 float4 = 64 B, one byte per plane, unless all in LDS), used by
  // the queue traversal kernels of profiles without fractals (dev_trace.h Traversal4).  Its own LDS
  // plan: node prefix, triangles / refs, stack4_lds stack rows in LDS; rows stack4_lds .. stack4_need
  // - 1 spill to stack4_ovf (row r - stack4_lds, lane = global thread id of the persistent grid).
  gptr<float4> nodes4;
  int32_t* stack4_ovf;
  uint32_t num_nodes4, lds4_nodes, lds4_tris, lds4_refs, stack4_lds, stack4_need, stack4_lanes;
  uint32_t lds4_shapes;   // BVH4 plan: shape records 0 .. lds4_shapes - 1 copied to LDS (dev_trace.h lds_setup)
  // threaded depth-first entry list of the same BVH (bvh::threaded; 2 float4 per entry) for the
  // wave-coherent traversal kernels, used when the scene is small (pkt_n > 0; core.hip upload)
  gptr<float4> pkt;
  uint32_t pkt_n;
  uint32_t pkt_refs;            // leaf refs of that BVH (the packet kernels keep the first 64 in a VGPR)
  uint32_t sample_major;        // camera-sample slot order of a tile (wavefront.h k_raygen): 1 for pkt scenes
  uint32_t bf_tris, bf_shapes;  // > 0: the queue traversal kernels test every primitive (dev_trace.h
                                // brute_walk; core.hip upload: scenes of a few dozen primitives)
  uint32_t sh_inline;           // 1: the shading kernel tests the light-sample shadow rays itself against
                                // the LDS copy of the whole BVH4 (wavefront.h inline_shadow; core.hip upload)
  // boundingSphere of the scene's worldBounds (AABB.hs:62-66; the kd-tree bounds: union of the
  // reference primitive bounds), for infinite-light photon emission (Light.hs:190-208)
  float world_c[3], world_r;
  // that union itself: the reference tests every query against it first (kdTreePrimitive's
  // intersectAABB b r, KdTree.hs:236-244), and a ray it rejects misses the scene (dev_trace.h kd_root)
  float kd_lo[3], kd_hi[3];
};

}  // namespace bd
