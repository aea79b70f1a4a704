// core.hip -- the MI355X path-tracing core behind include/bling.h.
//
// One render pass (Rendering.hs:127-140) runs as a wavefront of paths in HBM, chunked by tiles:
//   k_raygen          camera samples of the chunk's 16x16 tiles (Sampling.hs:112-132, Camera.hs:49-76)
//   per path vertex   k_trace_closest -> k_trace_any -> k_resolve -> k_shade over compacted queues
//                     (wavefront.h; Integrator/Path.hs:41-87, Scene.hs:61-118)
//   k_film            per-tile filtered splat into LDS + merge into the film (Image.hs:108-299)
// Path state is SoA (one 64-B record per spectrum) indexed through compacted queues.  Traversal
// uses the LDS stack of dev_trace.h.
#include "core_internal.h"

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <thread>

using namespace bd;
using namespace bcore;

namespace {

thread_local std::string g_err;

// largest threaded BVH (child boxes) walked by the wave-coherent kernels.  A/B on MI355X
// (DESIGN.md 3): sun-sky (8 entries) closest-hit -11 %; cornell-box (30) +28 %, so it stays per-lane
constexpr uint32_t kPacketMaxEntries = 16;
// primitives up to which the traversal kernels test every primitive instead of walking a tree:
// sun-sky's 4 shapes, closest-hit 108 -> 93 ms per C4 pass; cornell's 31 primitives measured even
// (closest 28.9 -> 28.4 ms, any-hit 8.6 -> 9.4: profiles/r05_ab_session.txt r05h-l), so they walk
// the BVH4
constexpr uint32_t kBruteMax = 16;
static_assert(2 * kPacketMaxEntries <= 64, "the packet kernels hold the entry list in one VGPR float4 per lane");
// scenes with at most this many analytic shapes keep their shape records in the BVH4 kernels' LDS
constexpr uint32_t kLdsShapesMax = 8;
// dynamic LDS of the shading kernel's in-line shadow test: 4 blocks x (36 KiB ring + 4 KiB) = 160 KiB
constexpr size_t kShadeLdsMax = 4096;

// LDS plan of the traversal kernels: keep a block at <= 30 KiB so five 256-thread blocks fit a CU's
// 160 KiB.  The stack takes depth x 1 KiB; small scenes then go to LDS whole, larger ones keep the
// breadth-first node prefix (the top levels every ray visits).
void plan_lds(DevScene& S, uint32_t nodes, uint32_t tris, uint32_t refs, uint32_t depth) {
  constexpr size_t kBudget = 30 * 1024;
  S.stack_depth = depth;
  const size_t stack = (size_t)4 * TRACE_BLOCK * depth;
  const size_t avail = kBudget > stack ? kBudget - stack : 0;
  const size_t ref_b = (size_t)16 * ((refs + 3) / 4);
  if ((size_t)64 * nodes + lds_tri_bytes(tris) + ref_b <= avail) {
    S.lds_nodes = nodes; S.lds_tris = tris; S.lds_refs = refs;
    return;
  }
  S.lds_tris = 0;
  S.lds_refs = ref_b <= avail / 4 ? refs : 0;
  const size_t left = avail - (S.lds_refs ? ref_b : 0);
  S.lds_nodes = (uint32_t)std::min<size_t>(nodes, left / 64);
}

// LDS plan of the BVH4 (Traversal4): a 26-KiB block budget, so six 256-thread blocks share a CU's
// 160 KiB -- the meshes-profile kernel's 78 VGPRs allow six waves per SIMD, and occupancy beats a
// longer node prefix (A/B on C3, profiles/r02_ab_lds4_budget_s5.txt: 20 / 26 / 30 / 40 / 53 KiB ->
// 5 002 / 5 046 / 4 822 / 4 518 / 3 009 Mrays/s).  When the tree,
// triangles, refs and the whole stack bound fit, everything goes to LDS (lds_all4).  Otherwise
// stack4_lds rows of the stack stay in LDS (12: flat from 8 to 20 rows on C3), the
// rest spill to global rows, and the breadth-first node prefix (and the refs, if small) take what is
// left (node_b bytes a node: 112, or 64 quantized in BLING_QBVH4 experiment builds).
void plan_lds4(DevScene& S, uint32_t nodes, uint32_t tris, uint32_t refs, uint32_t need, uint32_t shapes, size_t node_b) {
  constexpr size_t kBudget = (size_t)26 * 1024;
  const size_t ref_b = (size_t)16 * ((refs + 3) / 4);
  S.stack4_need = need;
  // shape records (176 B each) go to LDS whole when the scene has a few: cornell's light quad
  const uint32_t sh = shapes <= kLdsShapesMax ? shapes : 0u;
  S.lds4_shapes = sh;
  if (lds_bytes4(nodes, tris, refs, need, sh, false) <= kBudget) {
    S.lds4_nodes = nodes; S.lds4_tris = tris; S.lds4_refs = refs; S.stack4_lds = need;
    return;
  }
  const uint32_t rows = std::max(1u, std::min(12u, need));
  S.stack4_lds = rows;
  const size_t stack = (size_t)4 * TRACE_BLOCK * rows + sizeof(DevShape) * sh;
  const size_t avail = kBudget > stack ? kBudget - stack : 0;
  S.lds4_tris = 0;
  S.lds4_refs = ref_b <= avail / 4 ? refs : 0;
  const size_t left = avail - (S.lds4_refs ? ref_b : 0);
  S.lds4_nodes = (uint32_t)std::min<size_t>(nodes, left / node_b);
}

// Everything upload_scene and the kernels assume of a scene description, checked on the host before
// any device work (bling_scene_validate runs it without a device): render config, texture graphs
// (computed textures at the top, their children stored), host-folded material spectra, light
// count, images and the textures and environment maps that index them.
void validate_scene(const bling_scene_desc* d) {
  if (!d) throw std::invalid_argument("null argument");
  if (d->config.width <= 0 || d->config.height <= 0) throw std::invalid_argument("bad render config");
  if (d->config.renderer == BLING_RENDERER_SPPM) {
    // eye trees are walked depth-first with one parked sibling per level (k_sppm_eye)
    if (d->config.max_depth < 1 || d->config.max_depth > SPPM_MAX_DEPTH)
      throw std::invalid_argument("sppm maxDepth outside [1, " + std::to_string(SPPM_MAX_DEPTH) + "]");
    if (d->config.sppm_photons < 1 || d->config.sppm_threads < 1) throw std::invalid_argument("bad sppm photon count");
  } else if (d->config.spp <= 0) {
    throw std::invalid_argument("bad render config");
  } else if (d->config.integrator == BLING_INTEGRATOR_DIRECT) {
    // the tree is walked depth-first with one parked sibling per level (k_shade_dl): bound it
    if (d->config.max_depth < 1 || d->config.max_depth > kMaxDlDepth)
      throw std::invalid_argument("directLighting maxDepth outside [1, " + std::to_string(kMaxDlDepth) + "]");
  } else if (d->config.integrator != BLING_INTEGRATOR_PATH) {
    throw std::invalid_argument("unknown surface integrator");
  }
  for (uint32_t k = 0; k < d->num_textures; ++k) {     // computed textures: children the device resolves
    const bling_texture& t = d->textures[k];
    auto simple = [&](int32_t ti) {
      return ti >= 0 && (uint32_t)ti < d->num_textures && d->textures[ti].kind <= BLING_TEX_GRAPHPAPER;
    };
    auto stex_ok = [&](int32_t si) { return si >= 0 && (uint32_t)si < d->num_scalar_textures; };
    bool ok = true;
    if (t.kind == BLING_TEX_BLEND) ok = simple(t.tex1) && simple(t.tex2) && stex_ok(t.stex);
    else if (t.kind == BLING_TEX_CHECKER) ok = simple(t.tex1) && simple(t.tex2);
    else if (t.kind == BLING_TEX_GRADIENT) {
      ok = t.tex2 >= 1 && t.tex1 >= 0 && (uint64_t)t.tex1 + (uint64_t)t.tex2 <= d->num_textures && stex_ok(t.stex);
      for (int32_t s = 0; ok && s < t.tex2; ++s) ok = d->textures[t.tex1 + s].kind == BLING_TEX_CONST;
    } else if (t.kind == BLING_TEX_GRAPHPAPER) ok = simple(t.tex1) && simple(t.tex2);
    else ok = t.kind == BLING_TEX_CONST || t.kind == BLING_TEX_IMAGE;   // the image index is checked below
    if (!ok) throw std::invalid_argument("texture " + std::to_string(k) + ": malformed or nested computed texture");
  }
  for (uint32_t k = 0; k < d->num_scalar_textures; ++k) {
    const bling_scalar_texture& t = d->scalar_textures[k];
    bool ok = t.kind >= BLING_STEX_CONST && t.kind <= BLING_STEX_IMAGE;
    if (t.kind == BLING_STEX_SCALE) ok = t.child >= 0 && (uint32_t)t.child < d->num_scalar_textures;
    if (t.kind == BLING_STEX_CRYSTAL)
      ok = t.octaves >= 1 && t.child >= 0 && (uint64_t)t.child + (uint64_t)t.octaves <= d->num_scalar_textures;
    if (!ok) throw std::invalid_argument("scalar texture " + std::to_string(k) + ": malformed");
  }
  for (uint32_t k = 0; k < d->num_materials; ++k) {
    // transMatte / shinyMetal / substrate spectra are folded on the host (sClamp, conductor terms):
    // make_bsdf reads their textures' constant values directly, so nothing computed may sit there
    const bling_material& m = d->materials[k];
    int nt = 0;
    if (m.kind == BLING_MAT_TRANSMATTE) nt = 2;
    else if (m.kind == BLING_MAT_SHINYMETAL) nt = 4;
    else if (m.kind == BLING_MAT_SUBSTRATE) nt = 3;
    for (int j = 0; j < nt; ++j) {
      const int32_t ti = m.tex[j];
      if (ti < 0 || (uint32_t)ti >= d->num_textures || d->textures[ti].kind != BLING_TEX_CONST)
        throw std::invalid_argument("material " + std::to_string(k) + ": texture " + std::to_string(j) +
                                    " must be a constant spectrum (folded on the host)");
    }
  }
  // the path state packs a light index (and a hit light + 1) into 8 bits each (wavefront.h vf_*)
  if (d->num_lights > 254) throw std::invalid_argument("more than 254 lights");
  for (uint32_t k = 0; k < d->num_lights; ++k) {
    const bling_light& l = d->lights[k];
    if (l.kind == BLING_LIGHT_INFINITE && l.env_kind == BLING_ENV_IMAGE && (l.env_w <= 0 || l.env_h <= 0 || !l.env_texels))
      throw std::invalid_argument("infinite light: empty image map");
  }
  for (uint32_t k = 0; k < d->num_images; ++k) {
    const bling_image& im = d->images[k];
    if (im.width <= 0 || im.height <= 0 || !im.texels || (im.channels != 1 && im.channels != 16))
      throw std::invalid_argument("texture image: bad size, channels or texels");
  }
  for (uint32_t k = 0; k < d->num_textures; ++k) {
    const bling_texture& t = d->textures[k];
    if (t.kind == BLING_TEX_IMAGE && (t.tex1 < 0 || (uint32_t)t.tex1 >= d->num_images || d->images[t.tex1].channels != 16))
      throw std::invalid_argument("image texture " + std::to_string(k) + ": no spectral image");
  }
  for (uint32_t k = 0; k < d->num_scalar_textures; ++k) {
    const bling_scalar_texture& t = d->scalar_textures[k];
    if (t.kind == BLING_STEX_IMAGE && (t.child < 0 || (uint32_t)t.child >= d->num_images || d->images[t.child].channels != 1))
      throw std::invalid_argument("scalar image texture " + std::to_string(k) + ": no greyscale image");
  }
}

// one thread per triangle: its shading frame (dev_shade.h tri_frame_build)
__global__ void k_tri_frames(const float* __restrict__ pts, const float* __restrict__ uvs, float4* __restrict__ out,
                             uint32_t n) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) tri_frame_build(pts + (size_t)9 * t, uvs + (size_t)6 * t, out + (size_t)4 * t);
}

void upload_scene(bling_ctx* c, const bling_scene_desc* d) {
  HIPCHK(hipSetDevice(c->device));
  DevScene& S = c->S;
  S = DevScene{};
  const uint32_t nt = d->num_triangles, ns = d->num_shapes;
  // --- triangles: MT record (v0, e1 = p2 - p1, e2 = p3 - p1) and shading data
  std::vector<float4> geo((size_t)3 * nt);
  std::vector<float> pts((size_t)9 * nt);
  for (uint32_t t = 0; t < nt; ++t) {
    const uint32_t* ix = d->tri_indices + 3 * t;
    float p[3][3];
    for (int k = 0; k < 3; ++k)
      for (int a = 0; a < 3; ++a) { p[k][a] = d->vertices[3 * ix[k] + a]; pts[9 * t + 3 * k + a] = p[k][a]; }
    float e1[3], e2[3];
    for (int a = 0; a < 3; ++a) { e1[a] = p[1][a] - p[0][a]; e2[a] = p[2][a] - p[0][a]; }
    geo[3 * t + 0] = make_float4(p[0][0], p[0][1], p[0][2], e1[0]);
    geo[3 * t + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
    geo[3 * t + 2] = make_float4(e2[2], 0.f, 0.f, 0.f);
  }
  c->tri_geo.upload(geo.data(), geo.size());
  {                                   // per-triangle shading frames (dev_shade.h tri_frame_build)
    DBuf<float> dpts, duvs;
    dpts.upload(pts.data(), pts.size());
    duvs.upload(d->tri_uvs, (size_t)6 * nt);
    c->tri_frame.alloc((size_t)4 * nt);
    if (nt) {
      k_tri_frames<<<(nt + 255) / 256, 256, 0, c->stream>>>(dpts.p, duvs.p, c->tri_frame.p, nt);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(c->stream));
    }
  }
  c->tri_material.upload(d->tri_material, nt);
  if (d->tri_normals && d->tri_has_normals) {
    c->tri_normals.upload(d->tri_normals, (size_t)9 * nt);
    c->tri_has_n.upload(d->tri_has_normals, nt);
  } else { c->tri_normals.free(); c->tri_has_n.free(); }
  // --- primitive list (reference order) -> BVH items
  std::vector<int32_t> tri_prim(nt, -1), shape_prim(ns, -1);
  int32_t fractal_prim = -1;
  std::vector<bvh::Box> boxes;
  std::vector<uint32_t> refs;
  for (uint32_t i = 0; i < d->num_prims; ++i) {
    int kind = d->prim_kind[i], idx = d->prim_index[i];
    bvh::Box b;
    for (int a = 0; a < 3; ++a) { b.lo[a] = INFINITY; b.hi[a] = -INFINITY; }
    if (kind == 0) {
      tri_prim[idx] = (int32_t)i;
      for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) { float v = pts[9 * idx + 3 * k + a]; b.lo[a] = std::min(b.lo[a], v); b.hi[a] = std::max(b.hi[a], v); }
      refs.push_back((REF_TRI << 30) | (uint32_t)idx);
    } else if (kind == 1) {
      shape_prim[idx] = (int32_t)i;
      const bling_shape& s = d->shapes[idx];
      float mn[3], mx[3];
      const float* P = s.params;                                   // objectBounds (Shape.hs:299-311)
      if (s.kind == BLING_SHAPE_QUAD) { mn[0] = -P[0]; mn[1] = -P[1]; mn[2] = 0.f; mx[0] = P[0]; mx[1] = P[1]; mx[2] = 0.f; }
      else if (s.kind == BLING_SHAPE_DISK) { mn[0] = -P[1]; mn[1] = -P[1]; mn[2] = P[0]; mx[0] = P[1]; mx[1] = P[1]; mx[2] = P[0]; }
      else if (s.kind == BLING_SHAPE_CYLINDER) { mn[0] = -P[0]; mn[1] = -P[0]; mn[2] = P[1]; mx[0] = P[0]; mx[1] = P[0]; mx[2] = P[2]; }
      else if (s.kind == BLING_SHAPE_BOX) { for (int a = 0; a < 3; ++a) { mn[a] = P[a]; mx[a] = P[3 + a]; } }
      else { for (int a = 0; a < 3; ++a) { mn[a] = -P[0]; mx[a] = P[0]; } }
      for (int cidx = 0; cidx < 8; ++cidx) {
        float q[3] = {(cidx & 4) ? mx[0] : mn[0], (cidx & 2) ? mx[1] : mn[1], (cidx & 1) ? mx[2] : mn[2]};
        const float* m = s.o2w;
        float w = m[12] * q[0] + m[13] * q[1] + m[14] * q[2] + m[15];
        for (int a = 0; a < 3; ++a) {
          float v = m[4 * a] * q[0] + m[4 * a + 1] * q[1] + m[4 * a + 2] * q[2] + m[4 * a + 3];
          if (w != 1.f) v /= w;
          b.lo[a] = std::min(b.lo[a], v); b.hi[a] = std::max(b.hi[a], v);
        }
      }
      refs.push_back((REF_SHAPE << 30) | (uint32_t)idx);
    } else {
      fractal_prim = (int32_t)i;
      const float fr = d->fractal.kind == BLING_FRACTAL_JULIA ? 1.7321f : 1.4143f;   // entry spheres r^2 = 3 / 2
      for (int a = 0; a < 3; ++a) { b.lo[a] = -fr; b.hi[a] = fr; }
      refs.push_back((REF_FRACTAL << 30));
    }
    boxes.push_back(b);
  }
  {
    // worldBounds of the reference's kd-tree (union of the primitive bounds; the fractals' are
    // mkMandelBulb's +-2.5 and the Julia radius sqrt 3, not the tighter BVH entry spheres)
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < d->num_prims; ++i) {
      bvh::Box b = boxes[i];
      if (d->prim_kind[i] == 2) {
        const float fr = d->fractal.kind == BLING_FRACTAL_JULIA ? sqrtf(3.f) : 2.5f;
        for (int a = 0; a < 3; ++a) { b.lo[a] = -fr; b.hi[a] = fr; }
      }
      for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    float dd[3];
    for (int a = 0; a < 3; ++a) { S.world_c[a] = lo[a] + (hi[a] - lo[a]) * 0.5f; dd[a] = hi[a] - S.world_c[a]; }
    S.world_r = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
    for (int a = 0; a < 3; ++a) { S.kd_lo[a] = lo[a]; S.kd_hi[a] = hi[a]; }
  }
  // Leaves of at most two primitives: the all-LDS BVH4 kernel tests two primitives per step, so a
  // leaf costs one step (A/B, profiles/r02_ab_bvh_leaf_s5.txt: C2 closest-hit 37.4 -> 31.5 ms per
  // pass against leaves of up to 4; C3, C4 and C5 within noise).
  bvh::Result R = bvh::build(boxes, refs, 2);
  c->nodes.upload(reinterpret_cast<const float4*>(R.nodes.data()), R.nodes.size() / 4);
  c->refs.upload(R.refs.data(), R.refs.size());
  {
    // the primitives' records in leaf order, the ref in each (dev_trace.h LeafRec): the BVH4 kernels
    // with a global fallback test a leaf primitive with one dependent load instead of two
    std::vector<float4> lg((size_t)3 * (R.refs.size() + 1), make_float4(0.f, 0.f, 0.f, 0.f));
    for (size_t j = 0; j < R.refs.size(); ++j) {
      const uint32_t ref = R.refs[j], idx = ref & 0x3FFFFFFFu;
      if ((ref >> 30) == REF_TRI) { lg[3 * j] = geo[3 * idx]; lg[3 * j + 1] = geo[3 * idx + 1]; }
      float rf;
      std::memcpy(&rf, &ref, sizeof rf);
      lg[3 * j + 2] = make_float4((ref >> 30) == REF_TRI ? geo[3 * idx + 2].x : 0.f, rf, 0.f, 0.f);
    }
    c->leaf_geo.upload(lg.data(), lg.size());
  }
  c->bvh_depth = R.depth; c->bvh_leaves = R.leaves; c->bvh_max_leaf = R.max_leaf;
  if (R.depth > STACK_DEPTH - 1) throw std::runtime_error("BVH deeper than the traversal stack");
  c->features = bfeat::scene_features(d);
  static_assert(FT_PROCTEX == bfeat::PROCTEX && FT_BUMP == bfeat::BUMP && FT_MATTE == bfeat::MATTE &&
                FT_MULTI_LIGHT == bfeat::MULTI_LIGHT, "feature bits");
  plan_lds(S, (uint32_t)(R.nodes.size() / 16), nt, (uint32_t)R.refs.size(), (uint32_t)R.depth + 1);
  c->lds_trace = lds_bytes(S.lds_nodes, S.lds_tris, S.lds_refs, S.stack_depth);
  c->lds_all = S.lds_nodes == (uint32_t)(R.nodes.size() / 16) && S.lds_tris == nt && S.lds_refs == (uint32_t)R.refs.size();
  {
    // the 4-wide tree for the queue traversal kernels of non-fractal profiles (Traversal4)
    const bvh::Result4 Q = bvh::collapse4(R);
    const uint32_t n4 = (uint32_t)(Q.nodes.size() / 28);
    plan_lds4(S, n4, nt, (uint32_t)R.refs.size(), (uint32_t)std::max(1, Q.stack_need), ns, kQuantBvh4 ? 64 : 112);
    c->lds_all4 = S.lds4_nodes == n4 && S.lds4_tris == nt && S.lds4_refs == (uint32_t)R.refs.size() &&
                  S.stack4_lds == S.stack4_need && S.lds4_shapes == ns;
    const bool quantized = kQuantBvh4 && !c->lds_all4;
    // the all-LDS kernels lay the primitives out in leaf order (dev_trace.h lds_setup<..., LEAF>)
    c->lds_trace4 = c->lds_all4 ? lds_bytes4_leaf(S.lds4_nodes, S.lds4_refs, S.stack4_lds, S.lds4_shapes)
                                : lds_bytes4(S.lds4_nodes, S.lds4_tris, S.lds4_refs, S.stack4_lds, S.lds4_shapes, quantized);
    // one node format per scene: float, or quantized in BLING_QBVH4 builds unless all in LDS (Traversal4)
    if (!quantized) {
      c->nodes4.upload(reinterpret_cast<const float4*>(Q.nodes.data()), Q.nodes.size() / 4);
    } else {
      const std::vector<uint32_t> qn = bvh::quantize4(Q);
      c->nodes4.upload(reinterpret_cast<const float4*>(qn.data()), qn.size() / 4);
    }
    c->bvh4_depth = Q.depth;
    S.num_nodes4 = n4;
    // in-line shadow test of the cornell profile's shading kernel (wavefront.h inline_shadow): the
    // whole tree in LDS, a stack bound within the register stack (dev_trace.h occluded_lds),
    // and an LDS copy small enough that four shading blocks (36 KiB of ring each) still share a CU.
    // Experiment builds only (BLING_INLINE_SHADOW=1); BLING_INLINE_SHADOW=0 in the environment then
    // turns it off (A/B measurements).
    {
      const char* env = std::getenv("BLING_INLINE_SHADOW");
      const size_t bytes = lds_bytes4_leaf(n4, (uint32_t)R.refs.size(), 0u, ns);
      const bool on = BLING_INLINE_SHADOW && !(env && env[0] == '0') && c->lds_all4 && fractal_prim < 0 &&
                      S.stack4_need <= (uint32_t)kShadowStack && bytes <= kShadeLdsMax;
      S.sh_inline = on ? 1u : 0u;
      c->lds_shade = on ? bytes : 0u;
    }
    S.stack4_lanes = 0;
    if (S.stack4_need > S.stack4_lds) {
      int cus = 256;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) cus = 256;
      S.stack4_lanes = (uint32_t)cus * 2048u;           // every resident lane of a persistent grid
      c->stack4_ovf.alloc((size_t)(S.stack4_need - S.stack4_lds) * S.stack4_lanes);
    } else {
      c->stack4_ovf.free();
    }
  }
  {
    // small scenes walk the threaded BVH wave-coherently (packet_walk, dev_trace.h): at most
    // kPacketMaxEntries child boxes, no fractal
    const std::vector<float> th = bvh::threaded(R);
    const uint32_t ne = (uint32_t)(th.size() / 8);
    const bool on = fractal_prim < 0 && ne > 0 && ne <= kPacketMaxEntries;
    c->pkt.upload(reinterpret_cast<const float4*>(th.data()), th.size() / 4);
    S.pkt = as_global(c->pkt.p);
    S.pkt_n = on ? ne : 0u;
    S.pkt_refs = (uint32_t)R.refs.size();
    S.sample_major = on ? 1u : 0u;       // k_raygen's slot order: see there
  }
  {
    // scenes of at most kBruteMax primitives test all of them per ray (brute_walk, dev_trace.h) instead
    // of walking a tree; BLING_BRUTE=<n> sets the limit (0: never), for A/B measurements
    const char* env = std::getenv("BLING_BRUTE");
    const uint32_t lim = env ? (uint32_t)std::strtoul(env, nullptr, 10) : kBruteMax;
    const bool on = fractal_prim < 0 && nt + ns > 0 && nt + ns <= lim && R.refs.size() == (size_t)nt + ns;
    S.bf_tris = on ? nt : 0u;
    S.bf_shapes = on ? ns : 0u;
  }
  c->tri_prim.upload(tri_prim.data(), nt);
  c->shape_prim.upload(shape_prim.data(), ns);
  // --- shapes
  std::vector<DevShape> sh(ns);
  for (uint32_t k = 0; k < ns; ++k) {
    const bling_shape& s = d->shapes[k];
    sh[k].kind = s.kind; sh[k].material = s.material; sh[k].light = s.light; sh[k].prim = shape_prim[k];
    std::memcpy(sh[k].params, s.params, sizeof sh[k].params);
    std::memcpy(sh[k].w2o, s.w2o, 64);
    std::memcpy(sh[k].o2w, s.o2w, 64);
  }
  c->shapes.upload(sh.data(), ns);
  c->materials.upload(d->materials, d->num_materials);
  c->textures.upload(d->textures, d->num_textures);
  c->stex.upload(d->scalar_textures, d->num_scalar_textures);
  // --- lights: rewrite the Dist2D pointers to device copies
  // the path state packs a light index (and a hit light + 1) into 8 bits each (wavefront.h vf_*)
  std::vector<bling_light> lights(d->lights, d->lights + d->num_lights);
  c->light_arrays.clear();
  auto up = [&](const float* h, size_t n) -> const float* {
    if (!h || !n) return nullptr;
    c->light_arrays.emplace_back(new DBuf<float>());
    c->light_arrays.back()->upload(h, n);
    return c->light_arrays.back()->p;
  };
  // Each CDF travels with a guide table behind it (the device layout of dev_shade.h
  // sample_c1d): g[k] = the first index whose CDF value is >= k / kCdfGuide (k = 0 .. kCdfGuide),
  // so a search for u starts in [g[floor(u kCdfGuide)], g[floor(u kCdfGuide) + 1]] instead of the
  // whole row (the sun-sky map's 641-entry rows: 10 dependent loads -> 1 to 3).  The marginal
  // buffer also carries the sky's Perez denominators (host libm, as the oracle evaluates them).
  auto with_guide = [&](const float* cdf, size_t n, size_t rows, std::vector<float>& out) {
    out.assign(cdf, cdf + n * rows);
    for (size_t r = 0; r < rows; ++r) {
      const float* row = cdf + r * n;
      size_t i = 0;
      for (int k = 0; k <= kCdfGuide; ++k) {
        const float t = (float)k / (float)kCdfGuide;
        while (i < n && !(row[i] >= t)) ++i;
        uint32_t gi = (uint32_t)i;
        float f;
        std::memcpy(&f, &gi, 4);
        out.push_back(f);
      }
    }
  };
  for (auto& l : lights) {
    if (l.kind != BLING_LIGHT_INFINITE) continue;
    size_t nu = l.dist_nu, nv = l.dist_nv;
    std::vector<float> rows, marg;
    with_guide(l.dist_cdf, nu + 1, nv, rows);
    with_guide(l.marg_cdf, nv + 1, 1, marg);
    float den[3] = {0.f, 0.f, 0.f};
    if (l.env_kind == BLING_ENV_SUNSKY) {
      const float* ps[3] = {l.perez_x, l.perez_y, l.perez_Y};
      const float st = l.sun_theta, cst = bcr::cosf(st);
      for (int k = 0; k < 3; ++k) {                  // perez's denominator (SunSky.hs:81-86)
        const float* q = ps[k];
        den[k] = (1.f + q[0] * bcr::expf(q[1])) * (1.f + q[2] * bcr::expf(q[3] * st)) + q[4] * cst * cst;
      }
    }
    marg.insert(marg.end(), den, den + 3);
    if (l.env_kind == BLING_ENV_IMAGE) {
      l.env_texels = up(l.env_texels, (size_t)l.env_w * l.env_h * 16);
    }
    l.dist_func = up(l.dist_func, nu * nv);
    l.dist_cdf = up(rows.data(), rows.size());
    l.dist_func_int = up(l.dist_func_int, nv);
    l.marg_func = up(l.marg_func, nv);
    l.marg_cdf = up(marg.data(), marg.size());
  }
  c->lights.upload(lights.data(), lights.size());
  // --- texture images: texel tables in device memory
  std::vector<bling_image> images(d->images, d->images + d->num_images);
  for (auto& im : images) im.texels = up(im.texels, (size_t)im.width * im.height * im.channels);
  c->images.upload(images.data(), images.size());
  // --- DevScene
  S.nodes = as_global(c->nodes.p); S.leaf_refs = as_global(c->refs.p); S.leaf_geo = as_global(c->leaf_geo.p); S.num_nodes = (uint32_t)c->nodes.n / 4;
  S.nodes4 = as_global(c->nodes4.p); S.stack4_ovf = c->stack4_ovf.p;
  S.tri_geo = as_global(c->tri_geo.p); S.tri_frame = as_global(c->tri_frame.p);
  S.tri_normals = as_global(c->tri_normals.p); S.tri_has_n = as_global(c->tri_has_n.p);
  S.tri_material = as_global(c->tri_material.p); S.tri_prim = as_global(c->tri_prim.p);
  S.shapes = as_global(c->shapes.p);
  S.fractal = d->fractal; S.fractal_prim = fractal_prim;
  {
    long long pw = 1;                     // order ^ k is a Haskell Int: 8^14 needs 64 bits
    for (int k = 0; k < 32; ++k) { S.fractal_pw[k] = (float)pw; pw *= (long long)d->fractal.order; }
    if (d->fractal.present && (d->fractal.iterations < 0 || d->fractal.iterations > 32))
      throw std::runtime_error("fractal iterations outside [0, 32]");
  }
  S.materials = as_global(c->materials.p); S.textures = as_global(c->textures.p); S.stex = as_global(c->stex.p); S.lights = as_global(c->lights.p);
  S.images = as_global(c->images.p);
  S.num_lights = (int32_t)d->num_lights;
  S.camera = d->camera;
  std::memcpy(S.filter_table, d->filter.table, sizeof S.filter_table);
  S.filter_w = d->filter.width; S.filter_h = d->filter.height;
  const bling_render_config& cfg = d->config;
  S.sampler = cfg.sampler; S.nu = cfg.nu; S.nv = cfg.nv; S.spp = cfg.spp;
  S.max_depth = cfg.max_depth; S.sample_depth = cfg.sample_depth;
  S.integrator = cfg.integrator;
  if (S.integrator == BLING_INTEGRATOR_DIRECT) S.n1d = S.n2d = 2 * cfg.max_depth;   // DirectLighting.hs:17-18
  else { S.n1d = 4 * cfg.sample_depth; S.n2d = 3 * cfg.sample_depth; }              // Path.hs:26-28
  if (cfg.spp > (1 << 24)) throw std::runtime_error("more than 2^24 samples per pixel (the sampler's permutation, counter_rng.h)");
  S.fd_spp = FastDiv::make((uint32_t)std::max(1, cfg.spp));
  S.fd_nu = FastDiv::make((uint32_t)std::max(1, cfg.nu));
  {
    uint32_t w = (uint32_t)std::max(1, cfg.spp) - 1u;                 // brng::permute's mask
    w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
    S.perm_mask_spp = w;
  }
  S.inv_spp = 1.f / (float)cfg.spp; S.inv_nu = 1.f / (float)cfg.nu; S.inv_nv = 1.f / (float)cfg.nv;
  S.width = cfg.width; S.height = cfg.height;
  float fw = d->filter.width, fh = d->filter.height;
  S.ex0 = (int)floorf(0.5f - fw); S.ex1 = (int)floorf(0.5f + (float)cfg.width + fw);      // Image.hs:162-168
  S.ey0 = (int)floorf(0.5f - fh); S.ey1 = (int)floorf(0.5f + (float)cfg.height + fh);
  S.ext_w = S.ex1 - S.ex0 + 1;
  c->num_prims = d->num_prims;
  if ((int)std::ceil(fw) + 17 > FILM_TILE_MAX || (int)std::ceil(fh) + 17 > FILM_TILE_MAX)
    throw std::runtime_error("filter wider than the LDS film tile supports");
  c->counters.alloc(1);
  c->dscene.upload(&S, 1);
  c->film_dev.free();
  c->cfg = cfg;
  c->sppm.free_all();
}

int run_wave(bling_ctx* c, const WaveState& W, uint32_t n, uint32_t seed, uint32_t pass, bool stats,
             WaveTiming* tm = nullptr) {
  int launches = 0;
  with_profile(c->features, [&](auto prof) {
    launches = run_wave_prof<decltype(prof)::value>(c, W, n, seed, pass, stats, tm);
  });
  return launches;
}

void launch_trace(bling_ctx* c, const float* rays, uint32_t n, int any_hit, float* t, uint32_t* prim, float* bary) {
  with_profile(c->features, [&](auto prof) { launch_trace_prof<decltype(prof)::value>(c, rays, n, any_hit, t, prim, bary); });
}

// The tile-image slot of a filter (BLING_PASS_TILE_IMAGES): the largest mkImageTile image
// (Image.hs:108-120), w = x1 - max(0, x0) + floor(0.5 + fw) <= 15 + floor(0.5 + fw).
void tile_slot(const DevScene& S, int* sw, int* sh) {
  *sw = 15 + (int)std::floor(0.5f + S.filter_w);
  *sh = 15 + (int)std::floor(0.5f + S.filter_h);
}

// splitWindow over the sample extent (Sampling.hs:55-58), filtered by the stride (a sub-sample of
// the pass) and dealt round-robin to the shard
std::vector<TileDesc> pass_tiles(const DevScene& S, int rank, int world, int stride) {
  world = std::max(1, world); stride = std::max(1, stride);
  if (rank < 0 || rank >= world) throw std::invalid_argument("shard rank outside [0, world)");
  const uint32_t spp = (uint32_t)S.spp;
  std::vector<TileDesc> tiles;
  int k = 0;
  for (int y = S.ey0; y <= S.ey1; y += 16)
    for (int x = S.ex0; x <= S.ex1; x += 16, ++k) {
      if (k % stride != 0 || (k / stride) % world != rank) continue;
      TileDesc t{x, std::min(x + 15, S.ex1), y, std::min(y + 15, S.ey1), 0, 0};
      t.count = (uint32_t)((t.x1 - t.x0 + 1) * (t.y1 - t.y0 + 1)) * spp;
      tiles.push_back(t);
    }
  return tiles;
}

// Film splat of a chunk's tiles: the register-window kernel for the filter widths the configs use,
// the per-sample LDS-atomic kernel otherwise.  timg != NULL: the chunk's tile images into their slots.
void launch_film(bling_ctx* c, const WaveState& P, unsigned n_tiles, float* film_dev, float* timg) {
  const float fw = c->S.filter_w, fh = c->S.filter_h;
  const int kx = 2 * (int)std::floor(0.5f + fw) + 1, ky = 2 * (int)std::floor(0.5f + fh) + 1;
  int sw, sh;
  tile_slot(c->S, &sw, &sh);
  hipStream_t s = c->stream;
  if (kx == 5 && ky == 5)
    k_film_gather<5><<<n_tiles, 256 * film_split<5>(), 0, s>>>(c->dscene.p, P, c->tiles_dev.p, film_dev, timg, sw, sh);
  else if (kx == 7 && ky == 7)
    k_film_gather<7><<<n_tiles, 256 * film_split<7>(), 0, s>>>(c->dscene.p, P, c->tiles_dev.p, film_dev, timg, sw, sh);
  else
    k_film<<<n_tiles, 256, 0, s>>>(c->dscene.p, P, c->tiles_dev.p, film_dev, timg, sw, sh);
}

int render(bling_ctx* c, const bling_pass_params* p, float* film_dev, bling_stats* st) {
  const DevScene& S = c->S;
  uint32_t spp = (uint32_t)S.spp;
  const std::vector<TileDesc> tiles = pass_tiles(S, p->shard_rank, p->shard_world, p->tile_stride);
  float* timg = (p->flags & BLING_PASS_TILE_IMAGES) ? static_cast<float*>(p->tiles_device) : nullptr;
  if ((p->flags & BLING_PASS_TILE_IMAGES) && !timg) throw std::invalid_argument("BLING_PASS_TILE_IMAGES without tiles_device");
  int slot_w, slot_h;
  tile_slot(S, &slot_w, &slot_h);
  const size_t slot_floats = (size_t)slot_w * slot_h * 4;
  if (timg && p->tiles_capacity < tiles.size() * slot_floats)
    throw std::invalid_argument("tiles_capacity " + std::to_string(p->tiles_capacity) + " floats < the " +
                                std::to_string(tiles.size() * slot_floats) + " this shard's tile images need");
  uint64_t total = 0;
  for (auto& t : tiles) total += t.count;
  // Default wave: the whole pass when it fits in half of the free HBM (C2: 67.7 M paths, ~33 GB
  // of path state on a 288 GB MI355X) -- one wave means 8 launches per bounce in total instead of
  // per chunk, and full-device waves at the deep bounces.
  uint64_t want = p->chunk_paths > 0 ? (uint64_t)p->chunk_paths : total;
  if (p->chunk_paths <= 0) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
      // half of (free + what this context already holds): the same answer on every pass, so a
      // pass never re-allocates the path state the previous one sized (C3: 140 GB per hipMalloc)
      const uint64_t pb = c->path_bytes();
      const uint64_t held = (uint64_t)c->cap * pb;
      const uint64_t fit = std::max<uint64_t>(((uint64_t)free_b + held) / 2 / pb, 1u << 20);
      if (want > fit) {
        // equal waves instead of full waves plus a small remainder; one tile of slack because
        // waves are cut at tile boundaries
        uint32_t max_tile = 0;
        for (auto& t : tiles) max_tile = std::max(max_tile, t.count);
        const uint64_t waves = (total + fit - 1) / fit;
        want = std::min<uint64_t>(fit, (total + waves - 1) / waves + max_tile);
      }
    } else {
      want = std::min<uint64_t>(want, 1u << 22);
    }
  }
  want = std::min<uint64_t>(want, (uint64_t)1 << 31);
  uint32_t chunk = (uint32_t)std::max<uint64_t>(want, 256u * spp);
  c->ensure_paths((uint32_t)std::min<uint64_t>(chunk, std::max<uint64_t>(total, 1)));
  chunk = std::min<uint32_t>(chunk, c->cap);
  WaveState P = c->state();
  hipStream_t s = c->stream;
  HIPCHK(hipMemsetAsync(c->counters.p, 0, sizeof(Counters), s));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1));
  hipEvent_t eb0, eb1, ef1;
  HIPCHK(hipEventCreate(&eb0)); HIPCHK(hipEventCreate(&eb1)); HIPCHK(hipEventCreate(&ef1));
  HIPCHK(hipEventRecord(e0, s));
  uint64_t samples = 0, launches = 0;
  const bool stats_on = (p->flags & BLING_PASS_TRAVERSAL_STATS) != 0;
  WaveTiming tm;
  tm.on = (p->flags & BLING_PASS_KERNEL_TIMING) != 0;
  double ms_closest = 0.0, ms_shade = 0.0;
  uint64_t n_closest = 0, n_shade = 0;
  double ms_bounce = 0.0, ms_film = 0.0;
  size_t t0 = 0;
  std::vector<TileDesc> batch;
  c->tiles_dev.alloc(std::max<size_t>(1, tiles.size()));
  while (t0 < tiles.size()) {
    batch.clear();
    uint32_t off = 0, maxc = 0;
    size_t t1 = t0;
    while (t1 < tiles.size() && off + tiles[t1].count <= chunk) {
      TileDesc t = tiles[t1]; t.offset = off; off += t.count; maxc = std::max(maxc, t.count); batch.push_back(t); ++t1;
    }
    HIPCHK(hipMemcpyAsync(c->tiles_dev.p, batch.data(), batch.size() * sizeof(TileDesc), hipMemcpyHostToDevice, s));
    dim3 g((maxc + 255) / 256, (unsigned)batch.size());
    k_reset_queues<<<1, 64, 0, s>>>(P.qcount, off);
    k_raygen<<<g, 256, 0, s>>>(c->dscene.p, P, c->tiles_dev.p, p->seed, p->pass_index);
    HIPCHK(hipEventRecord(eb0, s));
    launches += (uint64_t)run_wave(c, P, off, p->seed, p->pass_index, stats_on, &tm);
    HIPCHK(hipEventRecord(eb1, s));
    launch_film(c, P, (unsigned)batch.size(), film_dev, timg ? timg + t0 * slot_floats : nullptr);
    HIPCHK(hipEventRecord(ef1, s));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // the tile table is reused by the next chunk
    samples += off;
    t0 = t1;
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, eb0, eb1));
    HIPCHK(hipEventElapsedTime(&b, eb1, ef1));
    ms_bounce += a; ms_film += b;
    for (size_t k = 0; k + 1 < tm.ev.size(); k += 2) {
      float m = 0.f;
      HIPCHK(hipEventElapsedTime(&m, tm.ev[k], tm.ev[k + 1]));
      ms_closest += m; ++n_closest;
      (void)hipEventDestroy(tm.ev[k]); (void)hipEventDestroy(tm.ev[k + 1]);
    }
    tm.ev.clear();
    for (size_t k = 0; k + 1 < tm.ev_shade.size(); k += 2) {
      float m = 0.f;
      HIPCHK(hipEventElapsedTime(&m, tm.ev_shade[k], tm.ev_shade[k + 1]));
      ms_shade += m; ++n_shade;
      (void)hipEventDestroy(tm.ev_shade[k]); (void)hipEventDestroy(tm.ev_shade[k + 1]);
    }
    tm.ev_shade.clear();
  }
  HIPCHK(hipEventRecord(e1, s));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
  (void)hipEventDestroy(eb0); (void)hipEventDestroy(eb1); (void)hipEventDestroy(ef1);
  Counters hc;
  HIPCHK(hipMemcpy(&hc, c->counters.p, sizeof hc, hipMemcpyDeviceToHost));
  std::memcpy(c->stream_bytes, hc.sb, sizeof c->stream_bytes);
  if (st) {
    std::memset(st, 0, sizeof *st);
    st->camera_samples = samples;
    st->rays_camera = hc.cam; st->rays_continuation = hc.cont; st->rays_mis = hc.mis; st->rays_shadow = hc.shadow;
    st->dropped_samples = hc.dropped;
    st->tiles = tiles.size();
    st->ms_total = ms;
    st->ms_bounce = ms_bounce; st->ms_film = ms_film;
    st->bounce_launches = launches;
    st->path_vertices = hc.vertices;
    st->node_visits = hc.node_visits; st->tri_tests = hc.tri_tests; st->shape_tests = hc.shape_tests;
    st->march_ticks = hc.march_ticks;
    st->closest_node_visits = hc.c_node_visits; st->closest_tri_tests = hc.c_tri_tests;
    st->closest_shape_tests = hc.c_shape_tests; st->closest_march_ticks = hc.c_march_ticks;
    st->ms_closest = ms_closest; st->closest_launches = n_closest;
    st->ms_shade = ms_shade; st->shade_launches = n_shade;
  }
  return BLING_OK;
}


// addTile of tile images into a device film: for each (tile list, buffer) pair, slot k of the buffer
// holds tile k of the list (slots of this context's tile_slot); one launch over all of them
void add_tiles(bling_ctx* c, const std::vector<std::pair<const std::vector<TileDesc>*, const float*>>& sets,
               float* film_dev) {
  int sw, sh;
  tile_slot(c->S, &sw, &sh);
  const size_t slot = (size_t)sw * sh;
  std::vector<TileSrc> t;
  for (const auto& s : sets)
    for (size_t k = 0; k < s.first->size(); ++k) {
      const TileDesc& d = (*s.first)[k];
      t.push_back(TileSrc{reinterpret_cast<const float4*>(s.second) + k * slot, std::max(0, d.x0), std::max(0, d.y0)});
    }
  if (t.empty()) return;
  c->tile_src.upload(t.data(), t.size());
  k_add_tiles<<<(unsigned)t.size(), 256, 0, c->stream>>>(c->tile_src.p, film_dev, c->S.width, c->S.height, sw, sh);
  HIPCHK(hipGetLastError());
}

// One pass over every device of the context (bling_create with n_devices > 1).  The caller's shard
// (rank, world) is dealt further over the n devices: device j renders the tiles of shard
// (rank + world j, world n), i.e. tile k (after the stride) when k % (world n) == rank + world j.
// Devices render concurrently, one host thread each, every one into its own tile-image buffer
// (BLING_PASS_TILE_IMAGES: ~1/n of the pass's tiles with their aprons, 2.4 MB per device for C2 at
// n = 8 instead of a 16 MiB film).  Once all succeeded, each peer pushes its buffer into its landing
// buffer on the primary with its own stream (the copies run concurrently over the xGMI links), the
// primary waits for them and adds every device's tile images into the caller's film (addTile).  A
// failed pass leaves the caller's film untouched.  Replaces the spark fan-out `parBuffer
// numCapabilities` of prender (Rendering.hs:111-140, :118) and its addTile merge.
int render_fanout(bling_ctx* c, const bling_pass_params* p, float* film_dev, bling_stats* st) {
  if (c->peers.empty()) return render(c, p, film_dev, st);
  if (p->flags & BLING_PASS_TILE_IMAGES) throw std::invalid_argument("BLING_PASS_TILE_IMAGES on a multi-device context");
  const int nd = 1 + (int)c->peers.size();
  const int world = std::max(1, p->shard_world), rank = p->shard_rank;
  int sw, sh;
  tile_slot(c->S, &sw, &sh);
  const size_t slot_floats = (size_t)sw * sh * 4;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<bling_stats> sts(nd);
  std::vector<std::string> errs(nd);
  std::vector<int> rcs(nd, BLING_OK);
  std::vector<std::vector<TileDesc>> dtiles(nd);
  for (int j = 0; j < nd; ++j) dtiles[j] = pass_tiles(c->S, rank + world * j, world * nd, p->tile_stride);
  std::vector<std::thread> th;
  for (int j = 0; j < nd; ++j) {
    th.emplace_back([&, j] {
      try {
        bling_ctx* d = j == 0 ? c : c->peers[j - 1].get();
        HIPCHK(hipSetDevice(d->device));
        bling_pass_params pp = *p;
        pp.shard_world = world * nd;
        pp.shard_rank = rank + world * j;
        const size_t need = std::max<size_t>(1, dtiles[j].size() * slot_floats);
        if (d->pass_tiles.n < need) d->pass_tiles.alloc(need);
        pp.flags |= BLING_PASS_TILE_IMAGES;
        pp.tiles_device = d->pass_tiles.p;
        pp.tiles_capacity = d->pass_tiles.n;
        rcs[j] = render(d, &pp, nullptr, &sts[j]);
      } catch (const std::exception& e) {
        errs[j] = e.what();
        rcs[j] = BLING_EHIP;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int j = 0; j < nd; ++j)
    if (rcs[j] != BLING_OK) throw HipError("device " + std::to_string(j) + ": " + (errs[j].empty() ? "render failed" : errs[j]));
  // merge: peers push concurrently, the primary adds after their copies
  while (c->stage.size() < (size_t)nd) c->stage.emplace_back(new DBuf<float>());
  struct Events {                      // destroyed on every exit path, after the streams drained
    std::vector<hipEvent_t> e;
    std::vector<hipStream_t> drain;
    ~Events() {
      for (hipStream_t s : drain) (void)hipStreamSynchronize(s);
      for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x);
    }
  } ev;
  ev.e.assign(nd, nullptr);
  std::vector<hipEvent_t>& done = ev.e;
  for (int j = 1; j < nd; ++j) {
    bling_ctx* d = c->peers[j - 1].get();
    const size_t bytes = dtiles[j].size() * slot_floats * sizeof(float);
    if (!bytes) continue;
    HIPCHK(hipSetDevice(c->device));
    if (c->stage[j]->n < dtiles[j].size() * slot_floats) c->stage[j]->alloc(dtiles[j].size() * slot_floats);
    HIPCHK(hipSetDevice(d->device));
    ev.drain.push_back(d->stream);
    HIPCHK(hipMemcpyPeerAsync(c->stage[j]->p, c->device, d->pass_tiles.p, d->device, bytes, d->stream));
    HIPCHK(hipEventCreateWithFlags(&done[j], hipEventDisableTiming));
    HIPCHK(hipEventRecord(done[j], d->stream));
  }
  HIPCHK(hipSetDevice(c->device));
  for (int j = 1; j < nd; ++j)
    if (done[j]) HIPCHK(hipStreamWaitEvent(c->stream, done[j], 0));
  std::vector<std::pair<const std::vector<TileDesc>*, const float*>> sets;
  for (int j = 0; j < nd; ++j) sets.emplace_back(&dtiles[j], j == 0 ? c->pass_tiles.p : c->stage[j]->p);
  ev.drain.push_back(c->stream);
  // one launch over every device's tile images.  Not bit-reproducible, like the single-device pass:
  // the film pixels under overlapping aprons, and each tile image's own LDS accumulation, take their
  // float additions in arrival order (tests/test_multidevice.py checks the sums to a tolerance;
  // INTEGRATION.md "Reproducibility" tells callers)
  add_tiles(c, sets, film_dev);
  if (st) {
    bling_stats a = sts[0];
    for (int j = 1; j < nd; ++j) {
      const bling_stats& b = sts[j];
      a.camera_samples += b.camera_samples; a.rays_camera += b.rays_camera; a.rays_continuation += b.rays_continuation;
      a.rays_mis += b.rays_mis; a.rays_shadow += b.rays_shadow; a.dropped_samples += b.dropped_samples;
      a.tiles += b.tiles; a.bounce_launches += b.bounce_launches; a.path_vertices += b.path_vertices;
      a.node_visits += b.node_visits; a.tri_tests += b.tri_tests; a.shape_tests += b.shape_tests;
      a.march_ticks += b.march_ticks;
      // kernel times: the slowest device's (as ms_bounce / ms_film), launches counted once
      a.ms_closest = std::max(a.ms_closest, b.ms_closest); a.ms_shade = std::max(a.ms_shade, b.ms_shade);
      a.closest_node_visits += b.closest_node_visits; a.closest_tri_tests += b.closest_tri_tests;
      a.closest_shape_tests += b.closest_shape_tests; a.closest_march_ticks += b.closest_march_ticks;
      a.ms_bounce = std::max(a.ms_bounce, b.ms_bounce); a.ms_film = std::max(a.ms_film, b.ms_film);
    }
    a.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *st = a;
  }
  return BLING_OK;
}

template <class F>
int guarded(F f) {
  try {
    return f();
  } catch (const HipError& e) {
    g_err = e.what();
    return BLING_EHIP;
  } catch (const std::bad_alloc&) {
    g_err = "out of memory";
    return BLING_ENOMEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return BLING_EINVAL;
  }
}

}  // namespace

extern "C" {

int bling_create(const int* device_ids, int n_devices, bling_ctx** out) {
  return guarded([&] {
    if (!out) throw std::invalid_argument("out is NULL");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) { g_err = "no HIP device"; return BLING_ENODEV; }
    if (n_devices < 0 || (n_devices > 0 && !device_ids)) throw std::invalid_argument("bad device list");
    if (n_devices > 64) throw std::invalid_argument("more than 64 devices");
    const int nd = std::max(1, n_devices);
    std::vector<int> ids(nd, 0);
    for (int j = 0; j < n_devices; ++j) {
      ids[j] = device_ids[j];
      if (ids[j] < 0 || ids[j] >= count) throw std::invalid_argument("bad device id " + std::to_string(ids[j]));
    }
    // a repeated id would silently fan a multi-GPU caller out onto one device: refused, except under
    // the test hook that exercises the fan-out on a one-GPU box (BLING_ALLOW_REPEATED_DEVICES=1)
    const char* rep = std::getenv("BLING_ALLOW_REPEATED_DEVICES");
    if (!(rep && rep[0] == '1'))
      for (int j = 0; j < n_devices; ++j)
        for (int k = 0; k < j; ++k)
          if (ids[j] == ids[k])
            throw std::invalid_argument("device id " + std::to_string(ids[j]) + " repeated in the device list");
    auto make = [](int dev) {
      auto x = std::make_unique<bling_ctx>();
      x->device = dev;
      HIPCHK(hipSetDevice(dev));
      HIPCHK(hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking));
      return x;
    };
    auto c = make(ids[0]);
    // further devices: peer contexts of the fan-out (render_fanout); the primary reads their films
    // over xGMI, so peer access is enabled where the pair supports it (a repeated id -- test hook
    // only -- runs two contexts on one device)
    for (int j = 1; j < nd; ++j) {
      c->peers.push_back(make(ids[j]));
      if (ids[j] != ids[0]) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, ids[0], ids[j]) == hipSuccess && can) {
          HIPCHK(hipSetDevice(ids[0]));
          hipError_t e = hipDeviceEnablePeerAccess(ids[j], 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
          (void)hipGetLastError();
        }
      }
    }
    HIPCHK(hipSetDevice(ids[0]));
    *out = c.release();
    return BLING_OK;
  });
}

int bling_scene_upload(bling_ctx* c, const bling_scene_desc* d) {
  return guarded([&] {
    if (!c || !d) throw std::invalid_argument("null argument");
    validate_scene(d);
    // no pass may mix a new scene on one device with an old or half-uploaded one on another: the
    // context and every peer lose their scene first and get it back only once all uploads succeeded
    c->has_scene = false;
    for (auto& q : c->peers) q->has_scene = false;
    upload_scene(c, d);
    for (auto& q : c->peers) upload_scene(q.get(), d);   // replicated scene (8e)
    HIPCHK(hipSetDevice(c->device));
    for (auto& q : c->peers) q->has_scene = true;
    c->has_scene = true;
    return BLING_OK;
  });
}

int bling_scene_validate(const bling_scene_desc* d) {
  return guarded([&] {
    validate_scene(d);
    return BLING_OK;
  });
}

int bling_render_pass_device(bling_ctx* c, const bling_pass_params* p, void* film, bling_stats* st) {
  return guarded([&] {
    if (!c || !p || (!film && !(p->flags & BLING_PASS_TILE_IMAGES))) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    return render_fanout(c, p, static_cast<float*>(film), st);
  });
}

int bling_render_pass(bling_ctx* c, const bling_pass_params* p, float* film_out, bling_stats* st) {
  return guarded([&] {
    if (!c || !p) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    size_t n = (size_t)c->S.width * c->S.height * 4;
    if (c->film_dev.n != n) c->film_dev.alloc(n);
    if (film_out) HIPCHK(hipMemcpy(c->film_dev.p, film_out, n * sizeof(float), hipMemcpyHostToDevice));
    else HIPCHK(hipMemset(c->film_dev.p, 0, n * sizeof(float)));
    int rc = render_fanout(c, p, c->film_dev.p, st);
    if (rc == BLING_OK && film_out) HIPCHK(hipMemcpy(film_out, c->film_dev.p, n * sizeof(float), hipMemcpyDeviceToHost));
    return rc;
  });
}

static int sample_li_impl(bling_ctx* c, uint32_t seed, uint32_t pass_index, const int32_t* samples, size_t n, float* L_out,
                   float* img_out, bling_stats* st, float* vtx_out) {
  return guarded([&] {
    if (!c || !samples || !L_out) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    if (n == 0) return BLING_OK;
    if (n > (1u << 24)) throw std::invalid_argument("too many samples");
    HIPCHK(hipSetDevice(c->device));
    const DevScene& S = c->S;
    for (size_t k = 0; k < n; ++k) {
      int x = samples[3 * k], y = samples[3 * k + 1], m = samples[3 * k + 2];
      if (x < S.ex0 || x > S.ex1 || y < S.ey0 || y > S.ey1 || m < 0 || m >= S.spp)
        throw std::invalid_argument("sample outside the sample extent");
    }
    c->ensure_paths((uint32_t)n);
    DBuf<float4> lfull;
    lfull.alloc((size_t)4 * c->cap);
    DBuf<int32_t> list;
    list.upload(samples, 3 * n);
    WaveState P = c->state();
    P.Lfull = lfull.p;
    DBuf<float> vtx;
    if (vtx_out) {
      const size_t nv = n * BLING_DV_DEPTHS * BLING_DV_FIELDS;
      std::vector<float> nan(nv, std::numeric_limits<float>::quiet_NaN());
      vtx.upload(nan.data(), nv);
      P.dbg = vtx.p;
    }
    hipStream_t s = c->stream;
    HIPCHK(hipMemsetAsync(c->counters.p, 0, sizeof(Counters), s));
    unsigned blocks = (unsigned)((n + 255) / 256);
    k_reset_queues<<<1, 64, 0, s>>>(P.qcount, (uint32_t)n);
    k_raygen_list<<<blocks, 256, 0, s>>>(c->dscene.p, P, list.p, (uint32_t)n, seed, pass_index);
    run_wave(c, P, (uint32_t)n, seed, pass_index, false);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(L_out, lfull.p, n * 16 * sizeof(float), hipMemcpyDeviceToHost));
    if (vtx_out) HIPCHK(hipMemcpy(vtx_out, vtx.p, vtx.n * sizeof(float), hipMemcpyDeviceToHost));
    if (img_out) {
      std::vector<float2> im(n);
      HIPCHK(hipMemcpy(im.data(), c->img.p, n * sizeof(float2), hipMemcpyDeviceToHost));
      for (size_t k = 0; k < n; ++k) { img_out[2 * k] = im[k].x; img_out[2 * k + 1] = im[k].y; }
    }
    if (st) {
      Counters hc;
      HIPCHK(hipMemcpy(&hc, c->counters.p, sizeof hc, hipMemcpyDeviceToHost));
      std::memset(st, 0, sizeof *st);
      st->camera_samples = n;
      st->rays_camera = hc.cam; st->rays_continuation = hc.cont; st->rays_mis = hc.mis; st->rays_shadow = hc.shadow;
      st->dropped_samples = hc.dropped;
    }
    return BLING_OK;
  });
}

int bling_pass_tile_layout(bling_ctx* c, const bling_pass_params* p, int32_t* origins_out, size_t* n_tiles,
                           int32_t* slot_w, int32_t* slot_h) {
  return guarded([&] {
    if (!c || !p || !n_tiles) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    const std::vector<TileDesc> tiles = pass_tiles(c->S, p->shard_rank, p->shard_world, p->tile_stride);
    *n_tiles = tiles.size();
    int sw, sh;
    tile_slot(c->S, &sw, &sh);
    if (slot_w) *slot_w = sw;
    if (slot_h) *slot_h = sh;
    if (origins_out)
      for (size_t k = 0; k < tiles.size(); ++k) {
        origins_out[2 * k] = std::max(0, tiles[k].x0);
        origins_out[2 * k + 1] = std::max(0, tiles[k].y0);
      }
    return BLING_OK;
  });
}

static void check_tiles_capacity(bling_ctx* c, const bling_pass_params* p, size_t n_tiles) {
  int sw, sh;
  tile_slot(c->S, &sw, &sh);
  const size_t need = n_tiles * (size_t)sw * sh * 4;
  if (p->tiles_capacity < need)
    throw std::invalid_argument("tiles_capacity " + std::to_string(p->tiles_capacity) + " floats < the " +
                                std::to_string(need) + " a shard's tile images need");
}

int bling_film_add_tiles(bling_ctx* c, const bling_pass_params* p, const void* tiles_device, void* film_device) {
  return guarded([&] {
    if (!c || !p || !tiles_device || !film_device) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    const std::vector<TileDesc> tiles = pass_tiles(c->S, p->shard_rank, p->shard_world, p->tile_stride);
    check_tiles_capacity(c, p, tiles.size());
    add_tiles(c, {{&tiles, static_cast<const float*>(tiles_device)}}, static_cast<float*>(film_device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BLING_OK;
  });
}

int bling_film_add_shards(bling_ctx* c, const bling_pass_params* p, const void* const* tiles_devices, void* film_device) {
  return guarded([&] {
    if (!c || !p || !tiles_devices || !film_device) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    const int world = std::max(1, p->shard_world);
    std::vector<std::vector<TileDesc>> tiles(world);
    std::vector<std::pair<const std::vector<TileDesc>*, const float*>> sets;
    for (int r = 0; r < world; ++r) {
      if (!tiles_devices[r]) throw std::invalid_argument("null tile buffer");
      tiles[r] = pass_tiles(c->S, r, world, p->tile_stride);
      check_tiles_capacity(c, p, tiles[r].size());
      sets.emplace_back(&tiles[r], static_cast<const float*>(tiles_devices[r]));
    }
    add_tiles(c, sets, static_cast<float*>(film_device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return BLING_OK;
  });
}

namespace {
// One pass of bling_render with exact per-window reports (single-device contexts, host film): the
// pass is rendered into its tile images on the device (BLING_PASS_TILE_IMAGES), which come back to
// the host; bling_render then adds them into the film one window after another, in the pass's
// window order, reporting SamplesAdded with the film up to that window (Rendering.hs:130-134).
int region_pass(bling_ctx* c, const bling_pass_params& p, bling_stats* st, std::vector<TileDesc>& tiles,
                std::vector<float>& images, int& sw, int& sh) {
  return guarded([&] {
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    tiles = pass_tiles(c->S, p.shard_rank, p.shard_world, p.tile_stride);
    tile_slot(c->S, &sw, &sh);
    const size_t slot = (size_t)sw * sh * 4, need = std::max<size_t>(1, tiles.size() * slot);
    if (c->pass_tiles.n < need) c->pass_tiles.alloc(need);
    bling_pass_params pt = p;
    pt.flags |= BLING_PASS_TILE_IMAGES;
    pt.tiles_device = c->pass_tiles.p;
    pt.tiles_capacity = c->pass_tiles.n;
    const int rc = render(c, &pt, nullptr, st);
    if (rc != BLING_OK) return rc;
    images.resize(tiles.size() * slot);
    HIPCHK(hipMemcpy(images.data(), c->pass_tiles.p, images.size() * sizeof(float), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}
// addTile of one tile image slot (the layout film_flush writes) into a host film: k_add_tiles' rule
// (zero pixels and pixels past the film skipped), one tile at a time in the caller's order
void add_tile_host(float* film, int width, int height, const float* img, int ox, int oy, int sw, int sh) {
  for (int y = 0; y < sh; ++y)
    for (int x = 0; x < sw; ++x) {
      const int gx = ox + x, gy = oy + y;
      if (gx >= width || gy >= height) continue;
      const float* v = img + 4 * ((size_t)y * sw + x);
      if (v[0] == 0.f && v[1] == 0.f && v[2] == 0.f && v[3] == 0.f) continue;
      float* o = film + 4 * ((size_t)gy * width + gx);
      o[0] += v[0]; o[1] += v[1]; o[2] += v[2]; o[3] += v[3];
    }
}
}  // namespace

int bling_render(bling_ctx* c, const bling_pass_params* p, float* film_out, bling_progress_fn report, void* user,
                 bling_stats* st) {
  if (!report) { g_err = "bling_render needs a progress reporter"; return BLING_EINVAL; }
  if (!p) { g_err = "null argument"; return BLING_EINVAL; }
  bling_pass_params pp = *p;
  bling_stats sum;
  std::memset(&sum, 0, sizeof sum);
  // per-window reports with the film up to each window need the tile images on the host: single
  // device, host film (a multi-device pass merges on the device; its reports follow the pass)
  const bool exact = (pp.flags & BLING_PASS_REGION_EVENTS) && film_out && c && c->peers.empty();
  std::vector<TileDesc> rtiles;
  std::vector<float> rimages;
  int rsw = 0, rsh = 0;
  for (;;) {
    bling_stats one;
    const int rc = exact ? region_pass(c, pp, &one, rtiles, rimages, rsw, rsh) : bling_render_pass(c, &pp, film_out, &one);
    if (rc != BLING_OK) return rc;
    sum.camera_samples += one.camera_samples; sum.rays_camera += one.rays_camera;
    sum.rays_continuation += one.rays_continuation; sum.rays_mis += one.rays_mis; sum.rays_shadow += one.rays_shadow;
    sum.dropped_samples += one.dropped_samples; sum.tiles += one.tiles; sum.ms_total += one.ms_total;
    sum.ms_bounce += one.ms_bounce; sum.ms_film += one.ms_film; sum.bounce_launches += one.bounce_launches;
    sum.path_vertices += one.path_vertices; sum.node_visits += one.node_visits; sum.tri_tests += one.tri_tests;
    sum.shape_tests += one.shape_tests; sum.ms_closest += one.ms_closest; sum.closest_launches += one.closest_launches;
    sum.march_ticks += one.march_ticks; sum.closest_node_visits += one.closest_node_visits;
    sum.closest_tri_tests += one.closest_tri_tests; sum.closest_shape_tests += one.closest_shape_tests;
    sum.closest_march_ticks += one.closest_march_ticks; sum.ms_shade += one.ms_shade;
    sum.shade_launches += one.shade_launches;
    if (st) *st = sum;
    if (pp.flags & BLING_PASS_REGION_EVENTS) {                     // forM_ ... RegionStarted w, SamplesAdded w img'
      const std::vector<TileDesc> tiles = exact ? rtiles : pass_tiles(c->S, pp.shard_rank, pp.shard_world, pp.tile_stride);
      for (size_t k = 0; k < tiles.size(); ++k) {
        const TileDesc& t = tiles[k];
        const bling_progress rs{BLING_PROGRESS_REGION_STARTED, (int32_t)pp.pass_index, nullptr, 1.f, nullptr,
                                {t.x0, t.x1, t.y0, t.y1}};
        (void)report(user, &rs);
        if (exact)                                                    // addTile of this window (Rendering.hs:133)
          add_tile_host(film_out, c->S.width, c->S.height, rimages.data() + k * (size_t)rsw * rsh * 4,
                        std::max(0, t.x0), std::max(0, t.y0), rsw, rsh);
        const bling_progress sa{BLING_PROGRESS_SAMPLES_ADDED, (int32_t)pp.pass_index, film_out, 1.f, nullptr,
                                {t.x0, t.x1, t.y0, t.y1}};
        (void)report(user, &sa);
      }
    }
    const bling_progress ev{BLING_PROGRESS_PASS_DONE, (int32_t)pp.pass_index, film_out, 1.f, &one, {0, 0, 0, 0}};
    if (!report(user, &ev)) return BLING_OK;                      // PassDone ... >>= \cont -> ...
    ++pp.pass_index;
  }
}

int bling_debug_scene_info(bling_ctx* c, char* buf, size_t size, size_t* len) {
  if (!c) { g_err = "null argument"; return BLING_EINVAL; }
  if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_EINVAL; }
  const DevScene& S = c->S;
  char tmp[1024];
  const int n = std::snprintf(tmp, sizeof tmp,
      "{\"prims\": %u, \"bvh_depth\": %d, \"bvh_leaves\": %d, \"bvh4_nodes\": %u, \"bvh4_depth\": %d, "
      "\"stack4_need\": %u, \"lds_all4\": %d, \"lds_trace4\": %zu, \"pkt_n\": %u, \"bf_prims\": %u, \"sh_inline\": %u, "
      "\"lds_shade\": %zu, \"features\": %u}",
      c->num_prims, c->bvh_depth, c->bvh_leaves, S.num_nodes4, c->bvh4_depth, S.stack4_need, c->lds_all4 ? 1 : 0,
      c->lds_trace4, S.pkt_n, S.bf_tris + S.bf_shapes, S.sh_inline, c->lds_shade, c->features);
  if (n < 0) { g_err = "format error"; return BLING_EINVAL; }
  if (len) *len = (size_t)n;
  if (buf && size) { std::strncpy(buf, tmp, size - 1); buf[size - 1] = '\0'; }
  return BLING_OK;
}

int bling_debug_stream_bytes(bling_ctx* c, uint64_t* out, size_t n, size_t* n_streams) {
  if (!c) { g_err = "null argument"; return BLING_EINVAL; }
  if (n_streams) *n_streams = BLING_N_STREAMS;
  if (!BLING_STREAM_STATS) { g_err = "stream byte counts need a BLING_STREAM_STATS build"; return BLING_EUNSUPPORTED; }
  if (out) std::memcpy(out, c->stream_bytes, std::min<size_t>(n, 2 * BLING_N_STREAMS) * sizeof(uint64_t));
  return BLING_OK;
}

int bling_sample_li(bling_ctx* c, uint32_t seed, uint32_t pass_index, const int32_t* samples, size_t n, float* L_out,
                    float* img_out, bling_stats* st) {
  return sample_li_impl(c, seed, pass_index, samples, n, L_out, img_out, st, nullptr);
}

int bling_sample_li_vertices(bling_ctx* c, uint32_t seed, uint32_t pass_index, const int32_t* samples, size_t n,
                             float* L_out, float* vtx_out) {
  if (!BLING_DEBUG_VERTEX) { g_err = "per-vertex records need a BLING_DEBUG_VERTEX build"; return BLING_EUNSUPPORTED; }
  if (!vtx_out) { g_err = "vtx_out is NULL"; return BLING_EINVAL; }
  if (c && c->S.integrator != BLING_INTEGRATOR_PATH) { g_err = "per-vertex records: Path integrator only"; return BLING_EUNSUPPORTED; }
  return sample_li_impl(c, seed, pass_index, samples, n, L_out, nullptr, nullptr, vtx_out);
}

int bling_trace(bling_ctx* c, const float* rays, size_t n, int any_hit, float* t_out, uint32_t* prim_out, float* bary_out) {
  return guarded([&] {
    if (!c || !rays || !prim_out) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    if (n == 0) return BLING_OK;
    HIPCHK(hipSetDevice(c->device));
    c->tr_rays.upload(rays, 8 * n);
    c->tr_t.alloc(n); c->tr_prim.alloc(n); c->tr_bary.alloc(2 * n);
    HIPCHK(hipMemsetAsync(c->counters.p, 0, sizeof(Counters), c->stream));
    launch_trace(c, c->tr_rays.p, (uint32_t)n, any_hit, c->tr_t.p, c->tr_prim.p, c->tr_bary.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(prim_out, c->tr_prim.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (t_out) HIPCHK(hipMemcpy(t_out, c->tr_t.p, n * sizeof(float), hipMemcpyDeviceToHost));
    if (bary_out) HIPCHK(hipMemcpy(bary_out, c->tr_bary.p, 2 * n * sizeof(float), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}

int bling_trace_device(bling_ctx* c, const void* rays, size_t n, int any_hit, void* t_dev, void* prim_dev, void* bary_dev,
                       int repeats, double* ms_out) {
  return guarded([&] {
    if (!c || !rays || !prim_dev) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    HIPCHK(hipSetDevice(c->device));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, c->stream));
    for (int r = 0; r < std::max(1, repeats); ++r)
      launch_trace(c, static_cast<const float*>(rays), (uint32_t)n, any_hit, static_cast<float*>(t_dev),
                   static_cast<uint32_t*>(prim_dev), static_cast<float*>(bary_dev));
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e1, c->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    if (ms_out) *ms_out = ms / std::max(1, repeats);
    return BLING_OK;
  });
}

int bling_sppm_pass(bling_ctx* c, uint32_t seed, uint32_t pass_index, float* film_out, float* splat_out,
                    bling_sppm_stats* st) {
  return guarded([&] {
    if (!c) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    if (c->cfg.renderer != BLING_RENDERER_SPPM) throw std::invalid_argument("the uploaded scene's renderer is not sppm");
    if (c->features & FT_PROCTEX) {
      g_err = "sppm: blend / gradient / checker / cellNoise textures are not supported by the SPPM renderer";
      return BLING_EUNSUPPORTED;
    }
    HIPCHK(hipSetDevice(c->device));
    if (!c->sppm.ready) sppm_init(c);
    SppmState& P = c->sppm;
    const size_t nf = (size_t)c->S.width * c->S.height * 4, ns = (size_t)c->S.width * c->S.height * 3;
    if (film_out) HIPCHK(hipMemcpy(P.film.p, film_out, nf * sizeof(float), hipMemcpyHostToDevice));
    else HIPCHK(hipMemset(P.film.p, 0, nf * sizeof(float)));
    if (splat_out) HIPCHK(hipMemcpy(P.splat.p, splat_out, ns * sizeof(float), hipMemcpyHostToDevice));
    else HIPCHK(hipMemset(P.splat.p, 0, ns * sizeof(float)));
    if (st) std::memset(st, 0, sizeof *st);
    if ((c->features & ~kProfiles[0]) == 0u) sppm_pass_t<kProfiles[0]>(c, seed, pass_index, st);
    else sppm_pass_t<kSppmAll>(c, seed, pass_index, st);
    if (film_out) HIPCHK(hipMemcpy(film_out, P.film.p, nf * sizeof(float), hipMemcpyDeviceToHost));
    if (splat_out) HIPCHK(hipMemcpy(splat_out, P.splat.p, ns * sizeof(float), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}

int bling_sppm_pixel_stats(bling_ctx* c, float* r2_out, float* n_out, size_t* n_pixels) {
  return guarded([&] {
    if (!c) throw std::invalid_argument("null argument");
    if (!c->has_scene) { g_err = "no scene uploaded"; return BLING_ENOSCENE; }
    if (c->cfg.renderer != BLING_RENDERER_SPPM) throw std::invalid_argument("the uploaded scene's renderer is not sppm");
    if (c->features & FT_PROCTEX) {
      g_err = "sppm: blend / gradient / checker / cellNoise textures are not supported by the SPPM renderer";
      return BLING_EUNSUPPORTED;
    }
    HIPCHK(hipSetDevice(c->device));
    if (!c->sppm.ready) sppm_init(c);
    SppmState& P = c->sppm;
    if (n_pixels) *n_pixels = P.n_stats;
    if (r2_out) HIPCHK(hipMemcpy(r2_out, P.r2.p, P.n_stats * sizeof(float), hipMemcpyDeviceToHost));
    if (n_out) HIPCHK(hipMemcpy(n_out, P.nacc.p, P.n_stats * sizeof(float), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}

int bling_debug_sppm_hitpoints(bling_ctx* c, float* pos_r2, uint64_t* keys, size_t cap, size_t* n) {
  return guarded([&] {
    if (!c) throw std::invalid_argument("null argument");
    if (!c->sppm.ready) { g_err = "no SPPM pass has run"; return BLING_EINVAL; }
    HIPCHK(hipSetDevice(c->device));
    SppmState& P = c->sppm;
    uint32_t cnt = 0;
    HIPCHK(hipMemcpy(&cnt, P.hp_count.p, sizeof cnt, hipMemcpyDeviceToHost));
    const size_t m = std::min<size_t>(cnt, P.hp_cap);
    if (n) *n = m;
    const size_t k = std::min(m, cap);
    if (pos_r2 && k) HIPCHK(hipMemcpy(pos_r2, P.hp_pos.p, k * sizeof(float4), hipMemcpyDeviceToHost));
    if (keys && k) HIPCHK(hipMemcpy(keys, P.hp_key.p, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}

int bling_debug_sppm_buckets(bling_ctx* c, uint32_t* bstart, uint32_t* items, float* mr, size_t cap_b, size_t cap_i,
                             size_t* nb, size_t* ni) {
  return guarded([&] {
    if (!c) throw std::invalid_argument("null argument");
    if (!c->sppm.ready) { g_err = "no SPPM pass has run"; return BLING_EINVAL; }
    HIPCHK(hipSetDevice(c->device));
    SppmState& P = c->sppm;
    SppmGrid g;
    HIPCHK(hipMemcpy(&g, P.grid.p, sizeof g, hipMemcpyDeviceToHost));
    if (nb) *nb = (size_t)g.cnt + 1;
    if (ni) *ni = g.items;
    if (bstart && cap_b >= (size_t)g.cnt + 1) HIPCHK(hipMemcpy(bstart, P.bstart.p, ((size_t)g.cnt + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (items && cap_i >= g.items && g.items) HIPCHK(hipMemcpy(items, P.items.p, (size_t)g.items * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (mr && cap_i >= g.items && g.items) HIPCHK(hipMemcpy(mr, P.kd_mr.p, (size_t)g.items * sizeof(float), hipMemcpyDeviceToHost));
    return BLING_OK;
  });
}

int bling_sppm_reset(bling_ctx* c) {
  return guarded([&] {
    if (!c) throw std::invalid_argument("null argument");
    HIPCHK(hipSetDevice(c->device));
    c->sppm.free_all();
    return BLING_OK;
  });
}

void bling_destroy(bling_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  delete c;
}

const char* bling_last_error(void) { return g_err.c_str(); }

const char* bling_version(void) { return "bling-mi355x core 0.1 (gfx950, wavefront path tracer, BVH2 + LDS stack)"; }

}  // extern "C"
