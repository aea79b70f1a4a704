// dev_trace.h -- ray / scene intersection on CDNA4: BVH2 traversal with an LDS-resident short
// stack (one column per lane, conflict-free), plus the primitive tests the reference runs inside
// its kd-tree leaves: Moller-Trumbore triangles (TriangleMesh.hs:140-207), object-space Quad and
// Sphere through the shape's world->object transform (Geometry.hs:14-37, Shape.hs:157-284) and the
// Mandelbulb distance-estimator march (Fractal.hs:37-137).
//
// Closest-hit semantics match Primitive.near (Primitive.hs:29-32): a primitive hit is accepted when
// tmin <= t <= current tmax, so a later-tested primitive wins exact ties.
#pragma once
#include <type_traits>
#include "dev_common.h"
#include "dev_scene.h"
#include "dev_shapes.h"
#include "../common/cr_math.h"
#include "../common/fast_cr.h"

// The march inside the traversal kernels (Julia scenes, and the batch bling_trace / SPPM walks):
// march iterations per traversal step (8 measured best with batching), and the number of lanes
// whose potential is decided that a batched finish() waits for (A/B on C5, round 1: off 166, 8: 179,
// 16: 202, 32: 214, 48: 216, 64: 171 Mrays/s)
constexpr int kMarchK = 8;
constexpr int kMarchBatch = 32;

namespace bd {

constexpr int TRACE_BLOCK = 256;   // threads per block of every tracing kernel
constexpr int STACK_DEPTH = 32;    // BVH depth is capped at 31 by the builder
constexpr int32_t bvh4_empty = (int32_t)0x80000000;   // unused BVH4 child slot (bvh::EMPTY4)

// The queue traversal kernels of a profile walk the BVH4 unless the profile has fractals.
template <uint32_t F>
constexpr bool use_bvh4() { return !(F & FT_FRACTAL); }

// Per-block LDS copy of the hot acceleration data (dynamic shared memory, sized by the host from
// DevScene::lds_*): node / triangle / leaf-ref loads below the cached counts are LDS reads instead
// of L1/L2 round trips.  The traversal stack lives behind them, one column per lane.
// Triangles sit in LDS as their 48-B records (v0.xyz e1.x | e1.yz e2.xy | e2.z, unused) plus a plane
// of e2.z: a primitive test reads two ds_read_b128 (16 lanes a group over all 64 banks; the 48-B stride
// keeps 16 consecutive triangles on 16 distinct bank quads) and one ds_read_b32 from consecutive dwords
// (bank = index mod 32).  Reading e2.z from the record instead made the compiler split the loads into
// b128 + b96 + a read2_b32 at dwords 12 t + 7 / 12 t + 8, which fall on only 8 of the 32 banks.
// (A 32-B record, e1.yz e2.xy packed next to v0, measured worse: 2 t mod 16 has 8 values, SQ 1.27
// conflicts per LDS instruction against 0.73, gpurun_out/r06h_sqtri36.)
//
// The all-LDS BVH4 kernels (ALLL: the whole tree in LDS) keep their primitives in leaf order
// instead (`leaf`, lds_setup<..., LEAF = true>): leaf slot j of the tree's ref list holds a 48-B
// record {v0.xyz e1.x | e1.yz e2.xy | e2.z, ref, -, -} (a shape's slot: zeros and its ref), plus one
// zero record past the end.  A leaf's primitive test then reads its record from the slot index it
// already holds -- the ref comes with the geometry -- instead of the ref first and the triangle one
// dependent LDS round trip later, and a step's two tests (leaves of at most two primitives) issue
// their loads together.  The prims of every leaf are tested in the same order as before.
struct LdsScene {
  const float4* nodes; uint32_t n_nodes;
  const float4* tris; uint32_t n_tris;
  const float* tri_e2z;
  const uint32_t* refs; uint32_t n_refs;
  int32_t* stack;
  const DevShape* shapes; uint32_t n_shapes;     // BVH4 plan only (0 otherwise)
  const float4* leaf = nullptr;                  // LEAF layout: 3 float4 per leaf slot (+ 1 zero record)
};
constexpr uint32_t kShapeQuads = sizeof(DevShape) / 16;   // float4 per DevShape record
static_assert(sizeof(DevShape) % 16 == 0, "DevShape must be a whole number of float4");

__host__ __device__ inline size_t lds_tri_bytes(uint32_t n_tris) { return (size_t)48 * n_tris + (size_t)16 * ((n_tris + 3) / 4); }
__host__ __device__ inline size_t lds_bytes(uint32_t n_nodes, uint32_t n_tris, uint32_t n_refs, uint32_t depth) {
  return (size_t)64 * n_nodes + lds_tri_bytes(n_tris) + (size_t)16 * ((n_refs + 3) / 4) + (size_t)4 * TRACE_BLOCK * depth;
}

// LDS bytes of the BVH4 plan (Traversal4): nodes (112 B float, 64 B quantized), triangles, refs,
// shape records, the stack rows that live in LDS.
__host__ __device__ inline size_t lds_bytes4(uint32_t n_nodes, uint32_t n_tris, uint32_t n_refs, uint32_t rows,
                                             uint32_t n_shapes, bool quantized) {
  return (size_t)(quantized ? 64 : 112) * n_nodes + lds_tri_bytes(n_tris) + (size_t)16 * ((n_refs + 3) / 4) + sizeof(DevShape) * n_shapes +
         (size_t)4 * TRACE_BLOCK * rows;
}
// the same for the all-LDS kernels' LEAF layout: nodes, leaf records (refs + 1), shapes, stack rows
// plus two spare rows (the branch-free pushes store up to two rows past the top, Traversal4::step)
__host__ __device__ inline size_t lds_bytes4_leaf(uint32_t n_nodes, uint32_t n_refs, uint32_t rows, uint32_t n_shapes) {
  return (size_t)112 * n_nodes + (size_t)48 * (n_refs + 1) + sizeof(DevShape) * n_shapes + (size_t)4 * TRACE_BLOCK * (rows + 2);
}

// Copies the planned prefixes into LDS; every thread of the block must call it.  B4: the BVH4 plan;
// QN: its nodes are the quantized ones (BLING_QBVH4 builds: every BVH4 kernel but the all-LDS one).
template <bool B4 = false, bool QN = false, bool LEAF = false>
DEV LdsScene lds_setup(const DevScene& S, float4* smem) {
  static_assert(B4 || !QN, "only the BVH4 has quantized nodes");
  static_assert(!LEAF || (B4 && !QN), "the leaf layout is the all-LDS float BVH4's");
  LdsScene L;
  if constexpr (LEAF) {                          // all-LDS BVH4: nodes | leaf records | shapes | stack
    L.n_nodes = S.lds4_nodes; L.n_tris = S.lds4_tris; L.n_refs = S.lds4_refs; L.n_shapes = S.lds4_shapes;
    float4* nd = smem;
    float4* lf = nd + 7 * L.n_nodes;
    for (uint32_t q = threadIdx.x; q < 7 * L.n_nodes; q += blockDim.x) nd[q] = gen(S.nodes4[q]);
    for (uint32_t q = threadIdx.x; q < 3 * (L.n_refs + 1); q += blockDim.x) {
      const uint32_t j = q / 3, part = q - 3 * j;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (j < L.n_refs) {
        const uint32_t ref = S.leaf_refs[j];
        const bool tri = (ref >> 30) == REF_TRI;
        const uint32_t idx = ref & 0x3FFFFFFFu;
        if (part < 2u) { if (tri) v = gen(S.tri_geo[3 * idx + part]); }
        else v = make_float4(tri ? gen(S.tri_geo[3 * idx + 2]).x : 0.f, __uint_as_float(ref), 0.f, 0.f);
      }
      lf[q] = v;
    }
    float4* sp = lf + 3 * (L.n_refs + 1);
    const gptr<float4> ssrc = as_global(reinterpret_cast<const float4*>(gen(S.shapes)));
    for (uint32_t q = threadIdx.x; q < kShapeQuads * L.n_shapes; q += blockDim.x) sp[q] = gen(ssrc[q]);
    L.nodes = nd; L.leaf = lf;
    L.tris = nullptr; L.tri_e2z = nullptr; L.refs = nullptr;
    L.shapes = reinterpret_cast<const DevShape*>(sp);
    L.stack = reinterpret_cast<int32_t*>(sp + kShapeQuads * L.n_shapes) + threadIdx.x;
    __syncthreads();
    return L;
  }
  L.n_nodes = B4 ? S.lds4_nodes : S.lds_nodes;
  L.n_tris = B4 ? S.lds4_tris : S.lds_tris;
  L.n_refs = B4 ? S.lds4_refs : S.lds_refs;
  constexpr uint32_t nq = QN ? 4u : (B4 ? 7u : 4u);   // float4 per node
  const gptr<float4> src = B4 ? S.nodes4 : S.nodes;
  float4* nd = smem;
  float4* tr = nd + nq * L.n_nodes;
  float4* rf = tr + 3 * L.n_tris;
  for (uint32_t q = threadIdx.x; q < nq * L.n_nodes; q += blockDim.x) nd[q] = gen(src[q]);
  for (uint32_t q = threadIdx.x; q < 3 * L.n_tris; q += blockDim.x) tr[q] = gen(S.tri_geo[q]);
  for (uint32_t q = threadIdx.x; q < (L.n_refs + 3) / 4; q += blockDim.x) {
    uint32_t b = 4 * q;
    rf[q] = make_float4(__uint_as_float(S.leaf_refs[b]), __uint_as_float(b + 1 < L.n_refs ? S.leaf_refs[b + 1] : 0u),
                        __uint_as_float(b + 2 < L.n_refs ? S.leaf_refs[b + 2] : 0u),
                        __uint_as_float(b + 3 < L.n_refs ? S.leaf_refs[b + 3] : 0u));
  }
  // BVH4 plan: the first lds4_shapes shape records (small scenes: all of them, e.g. cornell's
  // light quad, which ~19 % of its closest-hit rays test) -- no global load in the all-LDS kernel
  L.n_shapes = B4 ? S.lds4_shapes : 0u;
  float4* sp = rf + (L.n_refs + 3) / 4;
  const gptr<float4> ssrc = as_global(reinterpret_cast<const float4*>(gen(S.shapes)));
  for (uint32_t q = threadIdx.x; q < kShapeQuads * L.n_shapes; q += blockDim.x) sp[q] = gen(ssrc[q]);
  float* ez = reinterpret_cast<float*>(sp + kShapeQuads * L.n_shapes);
  for (uint32_t q = threadIdx.x; q < L.n_tris; q += blockDim.x) ez[q] = gen(S.tri_geo[3 * q + 2]).x;
  L.nodes = nd; L.tris = tr; L.refs = reinterpret_cast<const uint32_t*>(rf);
  L.shapes = reinterpret_cast<const DevShape*>(sp);
  L.tri_e2z = ez;
  L.stack = reinterpret_cast<int32_t*>(sp + kShapeQuads * L.n_shapes + (L.n_tris + 3) / 4) + threadIdx.x;
  __syncthreads();
  return L;
}

struct HitRec { float t; uint32_t ref; float b1, b2; };
struct TraceCount { uint32_t nodes, tris, shapes, ticks; };

// The reference's first test of every query: kdTreePrimitive's `intersectAABB b r >>= trav` (closest)
// and `maybe False tr (intersectAABB b r)` (any hit; KdTree.hs:236-244) against the kd-tree's bounds b,
// the union of the primitive bounds (DevScene::kd_lo / kd_hi).  intersectAABB (AABB.hs:79-94) narrows
// [rayMin, rayMax] slab by slab with Haskell's max / min and 1 / d per axis (inv: rcp_cr, = 1.f / d bit
// for bit) and gives up as soon as near > far.  near only grows and far only shrinks (hmax / hmin never
// take a NaN operand's side), so testing near > far once at the end gives the same answer without
// branches.  The device's BVH boxes are padded, so without this test a ray that grazes the bounds
// where a primitive's edge lies on them (the box's entry t one ulp past its exit t) finds the
// primitive, which the reference never tests: C2's floor edge at y = z = 0 under the round-6 sampler
// (tests/test_kd_root.py).
// Where the test runs: the kernel that makes a ray, once per ray with the lanes it has anyway
// (camera rays in k_raygen, continuation / BSDF-MIS / shadow rays in the shading kernels), not the
// traversal kernels.  There it sat in the lane-refill branch, which the wave enters at almost every
// step, and cost the all-LDS closest-hit kernel 10 % (C2 30.4 -> 33.5 ms per pass, gpurun_out/r06f).
// A rejected closest-hit ray carries the sign bit of its direction record's w (dir.w = pc, mdir.w =
// the MIS weight, both >= 0: readers take fabsf), and the traversal kernels start it finished (a
// miss); a rejected shadow ray gets tmin = +inf, which no box or primitive test passes (unoccluded).
// Batch queries (bling_trace) and SPPM walk with the test at the start (Traversal::reject_outside).
#ifndef BLING_KD_ROOT
#define BLING_KD_ROOT 1   // 0: measurement-only builds (what the test costs)
#endif
struct KdBox { float lo[3], hi[3]; };
DEV KdBox kd_box(const DevScene& S) {
  KdBox b;
#pragma unroll
  for (int a = 0; a < 3; ++a) { b.lo[a] = S.kd_lo[a]; b.hi[a] = S.kd_hi[a]; }
  return b;
}
DEV bool kd_root(const KdBox& b, const Ray& r, V3 inv) {
  if (!BLING_KD_ROOT) return true;
  float nr = r.tmin, fr = r.tmax;
  const float o[3] = {r.o.x, r.o.y, r.o.z}, iv[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float tn = (b.lo[a] - o[a]) * iv[a], tf = (b.hi[a] - o[a]) * iv[a];
    const bool sw = tn > tf;
    nr = hmax(nr, sw ? tf : tn);
    fr = hmin(fr, sw ? tn : tf);
  }
  return !(nr > fr);
}
DEV bool kd_root(const DevScene& S, const Ray& r) {
  return kd_root(kd_box(S), r, mk(bfast::rcp_cr(r.d.x), bfast::rcp_cr(r.d.y), bfast::rcp_cr(r.d.z)));
}
// the flag's encodings (see above)
DEV float kd_flag_w(float w, bool inside) { return inside ? w : __builtin_copysignf(w, -1.f); }
DEV bool kd_rejected(float w) { return __builtin_signbit(w) != 0; }

// ---------------------------------------------------------------- triangles
DEV bool tri_test(float4 g0, float4 g1, float4 g2, const Ray& r, float tmax, float* t_out, float* b1o, float* b2o) {
  V3 p1 = mk(g0.x, g0.y, g0.z);
  V3 e1 = mk(g0.w, g1.x, g1.y);
  V3 e2 = mk(g1.z, g1.w, g2.x);
  V3 s1 = cross(r.d, e2);
  float divisor = dot(s1, e1);
  if (divisor == 0.f) return false;
  float inv = bfast::rcp_cr(divisor);                     // = 1.f / divisor for every input (fast_cr.h)
  V3 dd = r.o - p1;
  float b1 = dot(dd, s1) * inv;
  if (b1 < 0.f || b1 > 1.f) return false;
  V3 s2 = cross(dd, e1);
  float b2 = dot(r.d, s2) * inv;
  if (b2 < 0.f || b1 + b2 > 1.f) return false;
  float t = dot(e2, s2) * inv;
  if (t < r.tmin || t > tmax) return false;
  *t_out = t; *b1o = b1; *b2o = b2;
  return true;
}
// tri_test without its early exits, for the all-LDS kernels: every value is computed (the same
// operations in the same order, so the same bits) and the exits' conditions are combined at the end,
// each in its original form -- a NaN barycentric or t passes its test there as it does in tri_test.
// The wave runs every operation of tri_test anyway whenever one lane gets past an exit; without the
// exits it saves their exec-mask bookkeeping and branches (the all-LDS kernels issue 0.38 SALU per
// VALU instruction, r05_c2_sq_summary).
DEV bool tri_test_nb(float4 g0, float4 g1, float e2z, const Ray& r, float tmax, float* t_out, float* b1o, float* b2o) {
  const V3 p1 = mk(g0.x, g0.y, g0.z);
  const V3 e1 = mk(g0.w, g1.x, g1.y);
  const V3 e2 = mk(g1.z, g1.w, e2z);
  const V3 s1 = cross(r.d, e2);
  const float divisor = dot(s1, e1);
  const float inv = bfast::rcp_cr(divisor);     // its out-of-range inputs behind a wave-uniform test
  const V3 dd = r.o - p1;
  const float b1 = dot(dd, s1) * inv;
  const V3 s2 = cross(dd, e1);
  const float b2 = dot(r.d, s2) * inv;
  const float t = dot(e2, s2) * inv;
  *t_out = t; *b1o = b1; *b2o = b2;
  return !(divisor == 0.f) & !(b1 < 0.f || b1 > 1.f) & !(b2 < 0.f || b1 + b2 > 1.f) & !(t < r.tmin || t > tmax);
}

// ---------------------------------------------------------------- shapes (object space)
DEV bool quad_test(float sx, float sy, const Ray& r, float tmax, float* t_out) {      // Shape.hs:157-171
  if (fabsf(r.d.z) < 1e-7f) return false;
  float t = -(r.o.z) / r.d.z;
  if (t < r.tmin || t > tmax) return false;
  V3 p = ray_at(r, t);
  if (fabsf(p.x) > sx || fabsf(p.y) > sy) return false;
  *t_out = t;
  return true;
}
DEV bool sphere_test(float rad, const Ray& r, float tmax, float* t_out) {              // Shape.hs:173-187
  float a = sqlen(r.d), b = 2.f * dot(r.o, r.d), c = sqlen(r.o) - (rad * rad);
  float t1, t2;
  if (!solve_quadric(a, b, c, &t1, &t2)) return false;
  if (t1 > tmax) return false;
  if (t2 < r.tmin) return false;
  float t = t1 < r.tmin ? t2 : t1;
  if (t > tmax) return false;
  *t_out = t;
  return true;
}
DEV bool sphere_any(float rad, const Ray& r) {                                         // Shape.hs:275-284
  float a = sqlen(r.d), b = 2.f * dot(r.o, r.d), c = sqlen(r.o) - (rad * rad);
  float t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > r.tmax || t1 < r.tmin) return false;
  if (t0 < r.tmin) return t1 < r.tmax;
  return true;
}
DEV Ray to_object(const DevShape& s, const Ray& r) {                                   // transRay w2o
  return Ray{xpoint(s.w2o, r.o), xvector(s.w2o, r.d), r.tmin, r.tmax};
}

// ---------------------------------------------------------------- mandelbulb (Fractal.hs)
// bulbPower of an order other than 8 (Fractal.hs:103-137 general branch): binary64 acos / atan2 /
// pow / sin / cos (cr_math.h).  Kept out of line: inlined, its temporaries raised the march
// kernels' register demand above their occupancy floor although no config uses another order.
__attribute__((noinline)) __device__ V3 bulb_power_n(V3 p, int n) {
  float wr = len(p);
  float wo = bcr::acosf(p.y / wr), wi = bcr::atan2f(p.x, p.z), fn = (float)n;
  float wrp = bcr::powf(wr, fn), wop = wo * fn, wip = wi * fn;
  const bcr::SinCos so = bcr::sincosf(wop), si = bcr::sincosf(wip);
  return vs(mk(so.s * si.s, so.c, so.s * si.c), wrp);
}
DEV V3 bulb_power(V3 p, int n) {
  if (n == 8) {
    float x = p.x, y = p.y, z = p.z;
    float x2 = x * x, y2 = y * y, z2 = z * z;
    float x4 = x2 * x2, y4 = y2 * y2, z4 = z2 * z2;
    float k3 = x2 + z2;
    float k2p = sqrtf(k3 * k3 * k3 * k3 * k3 * k3 * k3);
    if (k2p <= 0.f) return mk(0.f, 0.f, 0.f);
    float k2 = 1.f / k2p;
    float k1 = x4 + y4 + z4 - 6.f * y2 * z2 - 6.f * x2 * y2 + 2.f * z2 * x2;
    float k4 = x2 - y2 + z2;
    float wx = 64.f * x * y * z * (x2 - z2) * k4 * (x4 - 6.f * x2 * z2 + z4) * k1 * k2;
    float wy = -(16.f * y2 * k3 * k4 * k4) + k1 * k1;
    float wz = -(8.f * y * k4 * (x4 * x4 - 28.f * x4 * x2 * z2 + 70.f * x4 * z4 - 28.f * x2 * z2 * z4 + z4 * z4) * k1 * k2);
    return mk(wx, wy, wz);
  }
  return bulb_power_n(p, n);
}
DEV float mandel_potential(int order, int its, V3 pos) {
  V3 z = pos;
  for (int n = its + 1;; --n) {
    if (n == 1) return 0.f;
    V3 zp = bulb_power(z, order) + pos;
    if (sqlen(zp) > 2.5f) {
      // order ^ (1 + its - n) is a Haskell Int (64-bit): 8^14 overflows 32 bits
      long long pw = 1;
      for (int k = 0; k < 1 + its - n; ++k) pw *= order;
      return bcr::logf(len(zp)) / (float)pw;
    }
    z = zp;
  }
}
DEV float mandel_dist(int order, int its, float eps, V3 p, V3* g) {
  float pot = mandel_potential(order, its, p);
  if (pot == 0.f) { *g = mk(0.f, 1.f, 0.f); return 0.f; }
  V3 gp = mk(mandel_potential(order, its, p + mk(eps, 0.f, 0.f)), mandel_potential(order, its, p + mk(0.f, eps, 0.f)),
             mandel_potential(order, its, p + mk(0.f, 0.f, eps)));
  *g = vs(gp - mk(pot, pot, pot), 1.f / eps);
  return (0.5f / bcr::expf(pot)) * bcr::sinhf(pot) / len(*g);
}
// mandelInter's start (Fractal.hs:23-36): entry distance into the r^2 = 2 sphere, or tmin inside it
DEV bool mandel_entry(const Ray& r, float* d) {
  float c = sqlen(r.o) - 2.f;
  if (c <= 0.f) { *d = r.tmin; return true; }
  float a = sqlen(r.d), b = 2.f * dot(r.d, r.o), t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > r.tmax || t1 < r.tmin) return false;
  *d = t0;
  return true;
}
DEV bool mandel_march(const bling_fractal& f, const Ray& r, float* d_out, V3* p_out, V3* n_out) {
  float d;
  if (!mandel_entry(r, &d)) return false;
  float l = len(r.d);
  Ray rn{r.o, vs(r.d, 1.f / l), r.tmin * l, r.tmax * l};
  for (int guard = 0; guard < 100000; ++guard) {
    V3 p = ray_at(rn, d);
    if (sqlen(p) > 2.5f) return false;
    V3 g;
    float dist = mandel_dist(f.order, f.iterations, f.epsilon, p, &g);
    if (dist < f.epsilon) { *d_out = d; *p_out = p; *n_out = normalize(g); return true; }
    d = d + dist;
  }
  return false;
}

// mandel_march as a resumable state machine: one iter() is one iteration of mandelPotential's loop
// (one bulbPower), so the lanes of a wave stay converged however differently their rays march, and
// a finished march frees its lane at once; finish() is the rare part (the potentials' log, the
// gradient and the DE step's exp / sinh), which callers run batched over many lanes.  The four
// potentials of a DE step are taken two at a time: (p, p + eps ex), then (p + eps ey, p + eps ez).
// The two potentials of a pair run in the two halves of packed binary32 registers, so the order-8
// closed-form bulbPower issues as v_pk_mul_f32 / v_pk_add_f32 (two IEEE results per instruction).
// Each component sees exactly the operations of mandel_potential in the same order -- packing
// changes no rounding -- so hits stay bit-identical; the only extra work is the p + eps ex
// potential of a final step whose potential at p is 0.
typedef float f2v __attribute__((ext_vector_type(2)));
struct V3x2 { f2v x, y, z; };
DEV V3x2 v3x2(V3 a, V3 b) { V3x2 r; r.x = f2v{a.x, b.x}; r.y = f2v{a.y, b.y}; r.z = f2v{a.z, b.z}; return r; }
DEV V3 lane0(const V3x2& v) { return mk(v.x.x, v.y.x, v.z.x); }
DEV V3 lane1(const V3x2& v) { return mk(v.x.y, v.y.y, v.z.y); }
DEV V3x2 bulb_power2(const V3x2& p, int n) {
  if (n != 8) return v3x2(bulb_power(lane0(p), n), bulb_power(lane1(p), n));
  const f2v x = p.x, y = p.y, z = p.z;                 // bulb_power's order-8 closed form, per lane
  const f2v x2 = x * x, y2 = y * y, z2 = z * z;
  const f2v x4 = x2 * x2, y4 = y2 * y2, z4 = z2 * z2;
  const f2v k3 = x2 + z2;
  const f2v k37 = k3 * k3 * k3 * k3 * k3 * k3 * k3;
  const f2v k2p = f2v{bfast::sqrt_cr(k37.x), bfast::sqrt_cr(k37.y)};   // = sqrtf, 1.f / x (fast_cr.h)
  const f2v k2 = f2v{bfast::rcp_cr(k2p.x), bfast::rcp_cr(k2p.y)};
  const f2v k1 = x4 + y4 + z4 - 6.f * y2 * z2 - 6.f * x2 * y2 + 2.f * z2 * x2;
  const f2v k4 = x2 - y2 + z2;
  const f2v wx = 64.f * x * y * z * (x2 - z2) * k4 * (x4 - 6.f * x2 * z2 + z4) * k1 * k2;
  const f2v wy = -(16.f * y2 * k3 * k4 * k4) + k1 * k1;
  const f2v wz = -(8.f * y * k4 * (x4 * x4 - 28.f * x4 * x2 * z2 + 70.f * x4 * z4 - 28.f * x2 * z2 * z4 + z4 * z4) * k1 * k2);
  V3x2 r;                                              // k2p <= 0: bulb_power's early (0, 0, 0)
  r.x = f2v{k2p.x <= 0.f ? 0.f : wx.x, k2p.y <= 0.f ? 0.f : wx.y};
  r.y = f2v{k2p.x <= 0.f ? 0.f : wy.x, k2p.y <= 0.f ? 0.f : wy.y};
  r.z = f2v{k2p.x <= 0.f ? 0.f : wz.x, k2p.y <= 0.f ? 0.f : wz.y};
  return r;
}

struct MandelMarch2 {
  V3 rnd, p;                    // normalised ray direction, march point
  float d, pot, gx;             // distance, potential at p, potential at p + eps ex
  V3x2 pos, z;                  // the pair's potential inputs and iterates
  int32_t na, nb, steps, phase; // loop counters (0 = start the pair), steps, pair 0 / 1
  int32_t ran;                  // potentials the last iter() advanced (work counters: 0, 1 or 2)
  bool da, db;                  // potential decided (escaped or iterations spent)
  DEV void start(const Ray& r, float d0) {
    float l = len(r.d);
    rnd = vs(r.d, 1.f / l);
    d = d0; na = 0; nb = 0; steps = 0; phase = 0;
  }
  // one bulbPower iteration of both potentials of the pair: 1 = both decided, 0 = running, -1 = miss
  DEV int iter(const bling_fractal& f, const V3& o) {
    if (na == 0) {
      V3 a, b;
      if (phase == 0) {
        if (steps >= 100000) return -1;
        p = o + vs(rnd, d);                            // ray_at(rn, d)
        if (sqlen(p) > 2.5f) return -1;
        a = p; b = p + mk(f.epsilon, 0.f, 0.f);
      } else {
        a = p + mk(0.f, f.epsilon, 0.f); b = p + mk(0.f, 0.f, f.epsilon);
      }
      pos = v3x2(a, b); z = pos;
      na = nb = f.iterations + 1; da = db = false;
    }
    if (na == 1) da = true;                            // mandelPotential's n == 1: 0
    if (nb == 1) db = true;
    ran = (da ? 0 : 1) + (db ? 0 : 1);
    if (da && db) return 1;
    V3x2 zp = bulb_power2(z, f.order);
    zp.x = zp.x + pos.x; zp.y = zp.y + pos.y; zp.z = zp.z + pos.z;
    const f2v q = zp.x * zp.x + zp.y * zp.y + zp.z * zp.z;          // sqlen, per lane
    // per lane: a running potential takes the iterate and escapes or counts down (selects, no branches)
    const bool ra = !da, rb = !db;
    z.x = f2v{ra ? zp.x.x : z.x.x, rb ? zp.x.y : z.x.y};
    z.y = f2v{ra ? zp.y.x : z.y.x, rb ? zp.y.y : z.y.y};
    z.z = f2v{ra ? zp.z.x : z.z.x, rb ? zp.z.y : z.z.y};
    const bool ea = q.x > 2.5f, eb = q.y > 2.5f;
    na -= (ra && !ea) ? 1 : 0;
    nb -= (rb && !eb) ? 1 : 0;
    da = da || ea;
    db = db || eb;
    return (da && db) ? 1 : 0;
  }
  // the pair's potentials (log of the escaped iterate / order ^ k, or 0), then the DE step:
  // 0 = running (the next iter starts the next pair), 1 = hit (d; normal in *nrm)
  DEV int finish(const bling_fractal& f, const float* pw_tab, V3* nrm) {
    const float va = na == 1 ? 0.f : bcr::logf(len(lane0(z))) / pw_tab[1 + f.iterations - na];
    const float vb = nb == 1 ? 0.f : bcr::logf(len(lane1(z))) / pw_tab[1 + f.iterations - nb];
    na = 0; nb = 0;
    if (phase == 0) {
      pot = va;
      if (pot == 0.f) { *nrm = normalize(mk(0.f, 1.f, 0.f)); return 1; }   // mandelDist = 0 < eps
      gx = vb; phase = 1;
      return 0;
    }
    V3 g = vs(mk(gx, va, vb) - mk(pot, pot, pot), 1.f / f.epsilon);
    float dist = (0.5f / bcr::expf(pot)) * bcr::sinhf(pot) / len(g);
    if (dist < f.epsilon) { *nrm = normalize(g); return 1; }
    d = d + dist;
    phase = 0; ++steps;
    return 0;
  }
  DEV int tick(const bling_fractal& f, const float* pw_tab, const V3& o, V3* nrm) {
    const int s = iter(f, o);
    return s > 0 ? finish(f, pw_tab, nrm) : s;
  }
};

using MarchState = MandelMarch2;

// ---------------------------------------------------------------- Julia quaternion fractal
// Fractal.hs:148-281 (mkJuliaQuat, traverseJulia, iter, normalJulia), same operation order
struct Quat { float r, x, y, z; };
DEV Quat qadd(Quat a, Quat b) { return Quat{a.r + b.r, a.x + b.x, a.y + b.y, a.z + b.z}; }
DEV Quat qsub(Quat a, Quat b) { return Quat{a.r - b.r, a.x - b.x, a.y - b.y, a.z - b.z}; }
DEV float qlen(Quat q) { return sqrtf(q.r * q.r + q.x * q.x + q.y * q.y + q.z * q.z); }
DEV Quat qsq(Quat q) {
  const float tr = 2.f * q.r;
  return Quat{q.r * q.r - (q.x * q.x + q.y * q.y + q.z * q.z), tr * q.x, tr * q.y, tr * q.z};
}
DEV Quat qmul2(Quat q, Quat p) {                 // qscale (qmul q p) 2
  V3 c = cross(mk(q.x, q.y, q.z), mk(p.x, p.y, p.z));
  const float r1 = q.r, r2 = p.r;
  Quat m{r1 * r2 - (q.x * p.x + q.y * p.y + q.z * p.z), c.x + r1 * p.x + r2 * q.x, c.y + r1 * p.y + r2 * q.y,
         c.z + r1 * p.z + r2 * q.z};
  return Quat{m.r * 2.f, 2.f * m.x, 2.f * m.y, 2.f * m.z};
}
DEV Quat qpromote(V3 p) { return Quat{p.x, p.y, p.z, 0.f}; }
constexpr float JULIA_R2 = 3.f;                  // juliaRadius2

// One tick = one step of `iter` (the next iterate and its derivative); a DE step ends when the
// iterate escapes (|q| > 4) or the iterations run out.  Unlike the Mandelbulb, the hit is checked
// against the (normalised) ray extent (onRay, Fractal.hs:193).
struct JuliaMarch {
  V3 rnd;
  float d, tmin, tmax;                           // normalised-ray distance and extent
  Quat q, qp;
  int32_t i, steps;                              // iterations left (-1: start a DE step)
  // prepare (Fractal.hs:162-172) on the normalised ray
  DEV bool start(const Ray& r) {
    const float l = len(r.d);
    rnd = vs(r.d, 1.f / l);
    tmin = r.tmin * l; tmax = r.tmax * l;
    const float c = sqlen(r.o) - JULIA_R2;
    if (c <= 0.f) d = tmin;
    else {
      float a = sqlen(rnd), b = 2.f * dot(rnd, r.o), t0, t1;
      if (!solve_quadric(a, b, c, &t0, &t1)) return false;
      if (t0 > tmax || t1 < tmin) return false;
      d = t0;
    }
    i = -1; steps = 0;
    return true;
  }
  // 0 = running, 1 = hit (d), -1 = miss
  DEV int tick(const bling_fractal& f, const V3& o) {
    const Quat c{f.julia_c[0], f.julia_c[1], f.julia_c[2], f.julia_c[3]};
    if (i < 0) {
      if (steps >= 100000) return -1;
      V3 p = o + vs(rnd, d);
      if (sqlen(p) > JULIA_R2 + f.epsilon) return -1;
      q = qpromote(p); qp = Quat{1.f, 0.f, 0.f, 0.f}; i = f.iterations;      // qzero
    }
    const Quat q2 = qadd(qsq(q), c), qp2 = qmul2(q, qp);
    if (i == 0 || qlen(q) > 4.f) {
      const float nz = qlen(q2);
      const float dist = (0.5f * nz * bcr::logf(nz)) / qlen(qp2);
      if (dist < f.epsilon) return (d >= tmin && d <= tmax) ? 1 : -1;
      d = d + dist; i = -1; ++steps;
      return 0;
    }
    q = q2; qp = qp2; --i;
    return 0;
  }
};
// normalJulia (Fractal.hs:203-223)
DEV V3 julia_normal(const bling_fractal& f, V3 p) {
  const Quat c{f.julia_c[0], f.julia_c[1], f.julia_c[2], f.julia_c[3]};
  const Quat qp = qpromote(p);
  const Quat dx = qpromote(mk(f.epsilon, 0.f, 0.f)), dy = qpromote(mk(0.f, f.epsilon, 0.f)), dz = qpromote(mk(0.f, 0.f, f.epsilon));
  Quat v0 = qsub(qp, dx), v1 = qadd(qp, dx), v2 = qsub(qp, dy), v3 = qadd(qp, dy), v4 = qsub(qp, dz), v5 = qadd(qp, dz);
  for (int n = 0; n < f.iterations; ++n) {
    v0 = qadd(c, qsq(v0)); v1 = qadd(c, qsq(v1)); v2 = qadd(c, qsq(v2));
    v3 = qadd(c, qsq(v3)); v4 = qadd(c, qsq(v4)); v5 = qadd(c, qsq(v5));
  }
  return normalize(mk(qlen(v1) - qlen(v0), qlen(v3) - qlen(v2), qlen(v5) - qlen(v4)));
}

// ---------------------------------------------------------------- BVH2 traversal
DEV bool box2(const float4& n0, const float4& n1, const float4& n2, V3 o, V3 inv, float tmin, float tmax, float* tn0,
              float* tn1, bool* h1) {
  // child 0: lo (n0.x,n0.y,n0.z) hi (n0.w,n1.x,n1.y); child 1: lo (n1.z,n1.w,n2.x) hi (n2.y,n2.z,n2.w)
  float ax = (n0.x - o.x) * inv.x, bx = (n0.w - o.x) * inv.x;
  float ay = (n0.y - o.y) * inv.y, by = (n1.x - o.y) * inv.y;
  float az = (n0.z - o.z) * inv.z, bz = (n1.y - o.z) * inv.z;
  float lo0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
  float hi0 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
  float cx = (n1.z - o.x) * inv.x, dx = (n2.y - o.x) * inv.x;
  float cy = (n1.w - o.y) * inv.y, dy = (n2.z - o.y) * inv.y;
  float cz = (n2.x - o.z) * inv.z, dz = (n2.w - o.z) * inv.z;
  float lo1 = fmaxf(fmaxf(fminf(cx, dx), fminf(cy, dy)), fmaxf(fminf(cz, dz), tmin));
  float hi1 = fminf(fminf(fmaxf(cx, dx), fmaxf(cy, dy)), fminf(fmaxf(cz, dz), tmax));
  *tn0 = lo0; *tn1 = lo1;
  *h1 = lo1 <= hi1;
  return lo0 <= hi0;
}

// One analytic shape (record s, from LDS or global memory) against the ray in object space
// (Shape.hs:157-284); closest mode updates h (ref = the shape's) when tmin <= t <= h.t.
template <bool ANY, uint32_t F>
DEV bool shape_hit_rec(const DevShape& s, uint32_t ref, const Ray& r, HitRec& h) {
  Ray ro = to_object(s, Ray{r.o, r.d, r.tmin, h.t});
  const bool quad = !(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD;
  float t;
  if ((F & FT_SHAPES2) && !quad && s.kind != BLING_SHAPE_SPHERE) {            // disk, cylinder, box
    if (ANY) return shape2_test(s, ro, ro.tmax, true, &t);
    if (!shape2_test(s, ro, h.t, false, &t)) return false;
  } else {
    if (ANY) return quad ? quad_test(s.params[0], s.params[1], ro, ro.tmax, &t) : sphere_any(s.params[0], ro);
    if (!(quad ? quad_test(s.params[0], s.params[1], ro, h.t, &t) : sphere_test(s.params[0], ro, h.t, &t))) return false;
  }
  h.t = t; h.ref = ref; h.b1 = 0.f; h.b2 = 0.f;
  return true;
}

// One leaf primitive against the ray (Primitive.near's fold step, Primitive.hs:29-43): closest
// mode updates h when tmin <= t <= h.t; ANY returns true on any hit.
template <bool ANY, uint32_t F, bool ALLL = false>
DEV bool prim_hit_ref(const DevScene& S, const LdsScene& L, uint32_t ref, const Ray& r, HitRec& h, TraceCount& tc) {
  uint32_t kind = ref >> 30, idx = ref & 0x3FFFFFFFu;
  if ((F & FT_TRIS) && kind == REF_TRI) {
    ++tc.tris;
    float t, b1, b2;
    float4 g0, g1, g2;
    // the empty asm statements keep each branch's loads in that branch: without them the compiler
    // sinks the loads both branches share into one FLAT load through a merged pointer (waits on
    // vmcnt and lgkmcnt, and is slower than ds_read for the LDS case)
    if (ALLL || idx < L.n_tris) {
      g0 = L.tris[3 * idx]; g1 = L.tris[3 * idx + 1]; g2 = make_float4(L.tri_e2z[idx], 0.f, 0.f, 0.f);
      asm volatile("" ::: "memory");
    }
    else { g0 = gen(S.tri_geo[3 * idx]); g1 = gen(S.tri_geo[3 * idx + 1]); g2 = gen(S.tri_geo[3 * idx + 2]); asm volatile("" ::: "memory"); }
    if (!tri_test(g0, g1, g2, r, h.t, &t, &b1, &b2)) return false;
    if (!ANY) { h.t = t; h.ref = ref; h.b1 = b1; h.b2 = b2; }
    return true;
  }
  if (!(F & FT_FRACTAL) || kind == REF_SHAPE) {
    ++tc.shapes;
    if ((ALLL && use_bvh4<F>()) || idx < L.n_shapes) {   // planned into LDS (BVH4 ALLL: every shape)
      const bool hit = shape_hit_rec<ANY, F>(L.shapes[idx], ref, r, h);
      asm volatile("" ::: "memory");                      // see the triangle loads: no merged FLAT load
      return hit;
    }
    const bool hit = shape_hit_rec<ANY, F>(gen(S.shapes[idx]), ref, r, h);
    asm volatile("" ::: "memory");
    return hit;
  }
  ++tc.shapes;
  float d; V3 p, n;
  if (!mandel_march(S.fractal, Ray{r.o, r.d, r.tmin, ANY ? r.tmax : h.t}, &d, &p, &n)) return false;
  if (!ANY) { h.t = d; h.ref = ref; h.b1 = 0.f; h.b2 = 0.f; }
  return true;
}
// The LEAF layout's record of leaf slot j (lds_setup<..., true>) and its test: prim_hit_ref's
// arithmetic and update rule for the ref the record carries.
struct LeafRec { float4 a, b; float2 c; };      // c = (e2.z, ref)
DEV LeafRec leaf_rec(const LdsScene& L, uint32_t j) {
  LeafRec q;
  q.a = L.leaf[3 * j]; q.b = L.leaf[3 * j + 1];
  q.c = *reinterpret_cast<const float2*>(L.leaf + 3 * j + 2);
  return q;
}
// Records j and j + 1 (contiguous) in six explicit LDS reads: left to itself the compiler splits the
// float4 loads into ds_read2_b32 / ds_read_b96 pieces (four-cycle, 32-bank instructions).  The
// s_waitcnt inside makes the values safe to use when the statement ends.
DEV void leaf_rec2(const LdsScene& L, uint32_t j, LeafRec& q0, LeafRec& q1) {
  const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float4*)(L.leaf + 3 * j);
  asm volatile(
      "ds_read_b128 %0, %6\n\t"
      "ds_read_b128 %1, %6 offset:16\n\t"
      "ds_read_b64 %2, %6 offset:32\n\t"
      "ds_read_b128 %3, %6 offset:48\n\t"
      "ds_read_b128 %4, %6 offset:64\n\t"
      "ds_read_b64 %5, %6 offset:80\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(q0.a), "=&v"(q0.b), "=&v"(q0.c), "=&v"(q1.a), "=&v"(q1.b), "=&v"(q1.c)
      : "v"(addr)
      : "memory");
}
DEV LeafRec leaf_rec1(const LdsScene& L, uint32_t j) {
  LeafRec q;
  const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float4*)(L.leaf + 3 * j);
  asm volatile(
      "ds_read_b128 %0, %3\n\t"
      "ds_read_b128 %1, %3 offset:16\n\t"
      "ds_read_b64 %2, %3 offset:32\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(q.a), "=&v"(q.b), "=&v"(q.c)
      : "v"(addr)
      : "memory");
  return q;
}
// 1: a step loads both records of a two-primitive leaf before the first test (leaf_rec2); 0: one
// record before each test (fewer live registers)
#ifndef BLING_LEAF_PAIR
#define BLING_LEAF_PAIR 0
#endif
constexpr bool kLeafPair = BLING_LEAF_PAIR != 0;
template <bool ANY, uint32_t F>
DEV bool leaf_hit(const LdsScene& L, const LeafRec& q, const Ray& r, HitRec& h, TraceCount& tc) {
  const uint32_t ref = __float_as_uint(q.c.y);
  if ((F & FT_TRIS) && (ref >> 30) == REF_TRI) {
    ++tc.tris;
    float t, b1, b2;
    if (!tri_test_nb(q.a, q.b, q.c.x, r, h.t, &t, &b1, &b2)) return false;
    if (!ANY) { h.t = t; h.ref = ref; h.b1 = b1; h.b2 = b2; }
    return true;
  }
  ++tc.shapes;                                   // the all-LDS BVH4 holds every shape record
  const bool hit = shape_hit_rec<ANY, F>(L.shapes[ref & 0x3FFFFFFFu], ref, r, h);
  asm volatile("" ::: "memory");
  return hit;
}

// The BVH4 kernels with a global fallback: leaf slot j's record from S.leaf_geo (the same records
// in global memory, core.hip upload), so the test waits on one dependent load, not on the ref and
// then the triangle.  Shapes keep their records in LDS when planned there (prim_hit_ref's rule).
template <bool ANY, uint32_t F>
DEV bool leaf_hit_global(const DevScene& S, const LdsScene& L, uint32_t j, const Ray& r, HitRec& h, TraceCount& tc) {
  const gptr<float4> p = S.leaf_geo + 3 * j;
  LeafRec q;
  q.a = gen(p[0]); q.b = gen(p[1]);
  const float4 c = gen(p[2]);
  q.c = make_float2(c.x, c.y);
  const uint32_t ref = __float_as_uint(q.c.y);
  if ((F & FT_TRIS) && (ref >> 30) == REF_TRI) {
    ++tc.tris;
    float t, b1, b2;
    if (!tri_test_nb(q.a, q.b, q.c.x, r, h.t, &t, &b1, &b2)) return false;
    if (!ANY) { h.t = t; h.ref = ref; h.b1 = b1; h.b2 = b2; }
    return true;
  }
  ++tc.shapes;
  const uint32_t idx = ref & 0x3FFFFFFFu;
  if (idx < L.n_shapes) {
    const bool hit = shape_hit_rec<ANY, F>(L.shapes[idx], ref, r, h);
    asm volatile("" ::: "memory");               // see prim_hit_ref: no merged FLAT load
    return hit;
  }
  const bool hit = shape_hit_rec<ANY, F>(gen(S.shapes[idx]), ref, r, h);
  asm volatile("" ::: "memory");
  return hit;
}

template <bool ANY, uint32_t F, bool ALLL = false>
DEV bool prim_hit(const DevScene& S, const LdsScene& L, uint32_t slot, const Ray& r, HitRec& h, TraceCount& tc) {
  if constexpr (ALLL && use_bvh4<F>()) return leaf_hit<ANY, F>(L, leaf_rec(L, slot), r, h, tc);
  const uint32_t ref = (ALLL || slot < L.n_refs) ? L.refs[slot] : S.leaf_refs[slot];
  return prim_hit_ref<ANY, F, ALLL>(S, L, ref, r, h, tc);
}

// One child box of a BVH2 node against the ray, the arithmetic of box2 for a single box.
DEV bool box1(const float4& a, const float4& b, V3 o, V3 inv, float tmin, float tmax) {
  // lo (a.x, a.y, a.z) hi (a.w, b.x, b.y)
  const float ax = (a.x - o.x) * inv.x, bx = (a.w - o.x) * inv.x;
  const float ay = (a.y - o.y) * inv.y, by = (b.x - o.y) * inv.y;
  const float az = (a.z - o.z) * inv.z, bz = (b.y - o.z) * inv.z;
  const float lo = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
  const float hi = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
  return lo <= hi;
}

// Wave-coherent (packet) traversal of the threaded BVH (bvh::threaded, DevScene::pkt) for scenes
// whose whole tree is a few dozen entries: the 64 rays of a wave walk the entry list together.  An
// entry is entered when ANY lane's ray hits its box (with that lane's current closest t); a lane
// tests a leaf's primitives only where its own box test passed, so every lane sees exactly the
// primitives its own BVH2 traversal would test (culling is conservative: padded boxes), and only
// the order of the tests differs.  The walk index, the entry and the primitive records are
// wave-uniform -- scalar loads, no per-lane stack, no divergent refill -- which is what the
// per-lane traversal spends most of its issue slots on for small scenes.
// Returns when the walk ends or, for ANY, when no lane is still looking.
// The walk reads its entries and leaf refs from registers, not memory: each wave loads the whole
// list once (packet_regs: lane l holds float4 l of the list and leaf ref l) and an entry is eight
// v_readlane by the wave-uniform walk index, so the walk's dependent chain holds no load latency;
// shape records come from LDS (packet_lds).
struct PacketRegs { float4 ent; uint32_t ref; };
DEV PacketRegs packet_regs(const DevScene& S) {
  const uint32_t lane = threadIdx.x & 63u;
  PacketRegs p;
  p.ent = lane < 2u * S.pkt_n ? gen(S.pkt[lane]) : make_float4(0.f, 0.f, 0.f, 0.f);
  p.ref = lane < S.pkt_refs ? S.leaf_refs[lane] : 0u;
  return p;
}
DEV float4 lane_f4(const float4& v, uint32_t l) {
  return make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.z), l)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.w), l)));
}
// The scene's shape records (S.lds4_shapes of them: all, when there are few) in dynamic LDS; every
// thread of the block must call it.
DEV LdsScene packet_lds(const DevScene& S, float4* smem) {
  LdsScene L{nullptr, 0u, nullptr, 0u, nullptr, nullptr, 0u, nullptr, nullptr, 0u};
  L.n_shapes = S.lds4_shapes;
  const gptr<float4> ssrc = as_global(reinterpret_cast<const float4*>(gen(S.shapes)));
  for (uint32_t q = threadIdx.x; q < kShapeQuads * L.n_shapes; q += blockDim.x) smem[q] = gen(ssrc[q]);
  L.shapes = reinterpret_cast<const DevShape*>(smem);
  __syncthreads();
  return L;
}
template <bool ANY, uint32_t F>
DEV void packet_walk(const DevScene& S, const LdsScene& L, const PacketRegs& P, const Ray& r, bool active, HitRec& h,
                     TraceCount& tc) {
  const V3 inv = mk(bfast::rcp_cr(r.d.x), bfast::rcp_cr(r.d.y), bfast::rcp_cr(r.d.z));
  const uint32_t n = S.pkt_n;
  uint32_t k = 0;
  while (k < n) {
    const float4 a = lane_f4(P.ent, 2 * k), b = lane_f4(P.ent, 2 * k + 1);
    const bool hb = active && box1(a, b, r.o, inv, r.tmin, ANY ? r.tmax : h.t);
    ++tc.nodes;
    const int32_t code = __float_as_int(b.z);
    const uint32_t skip = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(b.w));
    if (__ballot(hb) == 0ull) { k = skip; continue; }
    if (code == -1) { ++k; continue; }
    const uint32_t lc = ~(uint32_t)code, first = lc >> 8, cnt = lc & 0xFFu;
    for (uint32_t q = 0; q < cnt; ++q) {
      const uint32_t sl = first + q;
      const uint32_t ref = sl < 64u ? (uint32_t)__builtin_amdgcn_readlane((int)P.ref, sl)
                                    : (uint32_t)__builtin_amdgcn_readfirstlane((int)S.leaf_refs[sl]);
      if (hb && prim_hit_ref<ANY, F, false>(S, L, ref, r, h, tc) && ANY) { h.ref = 0u; active = false; }
    }
    if (ANY && __ballot(active) == 0ull) return;
    k = skip;
  }
}

// Two triangles' Moller-Trumbore tests (tri_test) in the two halves of packed binary32 registers: each
// half runs exactly tri_test's operations in its order (v_pk_mul_f32 / v_pk_add_f32 round each half as
// the scalar instruction would; no contraction), and the outcome is computed without branches.
// ok0 / ok1: triangle a / b passes every test but the upper bound on t, which the caller applies in
// the triangles' order (tmin <= t <= the closest t so far, Primitive.near).
struct TriHit2 { f2v t, b1, b2; bool ok0, ok1; };
DEV f2v rcp2_cr(f2v x) {                                   // bfast::rcp_cr of both halves, one branch
  const bool in0 = __builtin_fabsf(x.x) >= 0x1p-125f && __builtin_fabsf(x.x) <= 0x1p125f;
  const bool in1 = __builtin_fabsf(x.y) >= 0x1p-125f && __builtin_fabsf(x.y) <= 0x1p125f;
  const f2v y = f2v{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)};
  const f2v e = f2v{__builtin_fmaf(-x.x, y.x, 1.f), __builtin_fmaf(-x.y, y.y, 1.f)};
  f2v r = f2v{__builtin_fmaf(e.x, y.x, y.x), __builtin_fmaf(e.y, y.y, y.y)};
  if (!(in0 && in1)) { r.x = in0 ? r.x : 1.f / x.x; r.y = in1 ? r.y : 1.f / x.y; }
  return r;
}
DEV TriHit2 tri_test2(const float4* A, const float4* B, const Ray& r) {
  const f2v p1x = f2v{A[0].x, B[0].x}, p1y = f2v{A[0].y, B[0].y}, p1z = f2v{A[0].z, B[0].z};
  const f2v e1x = f2v{A[0].w, B[0].w}, e1y = f2v{A[1].x, B[1].x}, e1z = f2v{A[1].y, B[1].y};
  const f2v e2x = f2v{A[1].z, B[1].z}, e2y = f2v{A[1].w, B[1].w}, e2z = f2v{A[2].x, B[2].x};
  const f2v dx = r.d.x, dy = r.d.y, dz = r.d.z;
  const f2v s1x = dy * e2z - dz * e2y, s1y = -(dx * e2z - dz * e2x), s1z = dx * e2y - dy * e2x;   // cross(d, e2)
  const f2v dv = s1x * e1x + s1y * e1y + s1z * e1z;                                                // dot(s1, e1)
  const f2v inv = rcp2_cr(dv);
  const f2v ddx = r.o.x - p1x, ddy = r.o.y - p1y, ddz = r.o.z - p1z;
  TriHit2 h;
  h.b1 = (ddx * s1x + ddy * s1y + ddz * s1z) * inv;
  const f2v s2x = ddy * e1z - ddz * e1y, s2y = -(ddx * e1z - ddz * e1x), s2z = ddx * e1y - ddy * e1x;  // cross(dd, e1)
  h.b2 = (dx * s2x + dy * s2y + dz * s2z) * inv;
  const f2v bs = h.b1 + h.b2;
  h.t = (e2x * s2x + e2y * s2y + e2z * s2z) * inv;
  h.ok0 = dv.x != 0.f && !(h.b1.x < 0.f || h.b1.x > 1.f) && !(h.b2.x < 0.f || bs.x > 1.f) && !(h.t.x < r.tmin);
  h.ok1 = dv.y != 0.f && !(h.b1.y < 0.f || h.b1.y > 1.f) && !(h.b2.y < 0.f || bs.y > 1.f) && !(h.t.y < r.tmin);
  return h;
}

// Exhaustive queries for scenes of a few dozen primitives (DevScene::bf_tris + bf_shapes > 0, core.hip
// upload): every lane tests its ray against every triangle, then every shape, in one wave-uniform
// order.  The records are read through the constant address space at a wave-uniform index, i.e. as
// scalar loads into SGPRs that the 64 lanes share: no node visits, no stack, no divergent walk and
// no LDS.  The triangles go two at a time through tri_test2 (packed, branch-free).  Closest mode
// keeps Primitive.near's rule (a later-tested hit with tmin <= t <= h.t replaces the current one)
// over this fixed order; only exact ties between distinct primitives see the order (the BVH walks'
// orders differ from the oracle's as well).  ANY returns once no lane of the wave is still looking.
template <class T>
using kptr = const __attribute__((address_space(4))) T*;
template <bool ANY, uint32_t F>
DEV void brute_walk(const DevScene& S, const Ray& r, bool active, HitRec& h, TraceCount& tc) {
  const kptr<float4> tg = (kptr<float4>)S.tri_geo;
  const uint32_t nt = S.bf_tris, ns = S.bf_shapes;
  if (ANY && __ballot(active) == 0ull) return;
  for (uint32_t i = 0; i < nt; i += 2) {
    const uint32_t j = i + 1 < nt ? i + 1 : i;           // an odd count tests the last triangle twice
    const float4* A = (const float4*)(tg + 3 * i);       // generic again; address-space inference keeps
    const float4* B = (const float4*)(tg + 3 * j);       // the constant loads (scalar, wave-uniform)
    const TriHit2 q = tri_test2(A, B, r);
    if (active) tc.tris += j > i ? 2u : 1u;
    if (ANY) {
      const bool hit = (q.ok0 && !(q.t.x > r.tmax)) || (j > i && q.ok1 && !(q.t.y > r.tmax));
      if (active && hit) { h.ref = 0u; active = false; }
      if (__ballot(active) == 0ull) return;
    } else {
      if (active && q.ok0 && !(q.t.x > h.t)) { h.t = q.t.x; h.ref = (REF_TRI << 30) | i; h.b1 = q.b1.x; h.b2 = q.b2.x; }
      if (active && j > i && q.ok1 && !(q.t.y > h.t)) { h.t = q.t.y; h.ref = (REF_TRI << 30) | j; h.b1 = q.b1.y; h.b2 = q.b2.y; }
    }
  }
  const kptr<DevShape> sg = (kptr<DevShape>)S.shapes;
  for (uint32_t k = 0; k < ns; ++k) {
    const DevShape& s = *(const DevShape*)(sg + k);
    if (active) {
      ++tc.shapes;
      if (shape_hit_rec<ANY, F>(s, (REF_SHAPE << 30) | k, r, h) && ANY) { h.ref = 0u; active = false; }
    }
    if (ANY && __ballot(active) == 0ull) return;
  }
}

// One ray's BVH2 traversal as a resumable state machine: step() visits one node (both child boxes,
// leaf children tested in place) and reports completion.  The queue kernels interleave step()
// with refilling finished lanes, so a wave keeps 64 rays in flight instead of idling its early
// finishers until the slowest ray of the batch is done.
// ALLL: the whole BVH, triangle set and leaf-ref list are LDS-resident (plan_lds), so no access
// needs a global fallback (fewer VGPRs, no branch per fetch).
template <bool ANY, uint32_t F, bool ALLL = false>
struct Traversal {
  static constexpr int32_t NONE = 0x7FFFFFFF;   // no inner node selected: pop the stack next
  Ray r;
  V3 inv;
  HitRec h;
  int32_t node, sp;
  uint32_t pfirst, pcount;                       // pending leaf: primitives still to test
  bool marching;                                 // FT_FRACTAL: a fractal march is in progress
  bool mpend;                                    // kMarchBatch: decided potential awaits finish()
  bool pre;                                      // Mandelbulb marched ahead (k_march): result in mres
  float mres;                                    //   the march's hit distance, or < 0 for none
  uint32_t mref;
  union { MarchState mm; JuliaMarch jm; };       // by S.fractal.kind (uniform)

  // rejected: the ray's kd_root test failed where it was made -- start finished, a miss
  DEV void init(const Ray& ray, bool rejected = false) {
    r = ray;
    inv = mk(bfast::rcp_cr(r.d.x), bfast::rcp_cr(r.d.y), bfast::rcp_cr(r.d.z));
    h.t = r.tmax; h.ref = REF_NONE; h.b1 = h.b2 = 0.f;
    node = rejected ? NONE : 0; sp = 0; pfirst = 0u; pcount = 0u;   // NONE, sp 0: done
    marching = false; mpend = false; pre = false; mres = -1.f; mref = 0u;
  }
  DEV void reject_outside(const DevScene& S) { if (!kd_root(kd_box(S), r, inv)) node = NONE; }
  DEV void take(int32_t link) {                  // link: inner node index, leaf code (< 0) or NONE
    if (link < 0) { uint32_t code = ~(uint32_t)link; pfirst = code >> 8; pcount = code & 0xFFu; node = NONE; }
    else node = link;
  }
  // One unit of work: an inner-node visit (both child boxes) OR one primitive test, so the lanes
  // of a wave diverge over at most one node visit plus one primitive per iteration (leaf loops of
  // up to 2 x 4 primitives no longer serialise the whole wave).
  // Returns true when finished: closest -> h holds the nearest hit (REF_NONE on a miss);
  // ANY -> h.ref != REF_NONE iff occluded.
  DEV bool step(const DevScene& S, const LdsScene& L, TraceCount& tc) {
    if (F & FT_FRACTAL) {
      if (marching) {                            // kMarchK bulbPower iterations of the march
        V3 nrm;
        int res = 0;
        const bool julia = S.fractal.kind == BLING_FRACTAL_JULIA;
        if (kMarchBatch > 0 && !julia) {
          // a lane whose potential is decided waits (mpend) until kMarchBatch lanes of the
          // marching set have one, or until no marching lane is still iterating
#pragma unroll
          for (int u = 0; u < kMarchK; ++u) {
            if (res == 0 && !mpend) {
              const int s = mm.iter(S.fractal, r.o);
              tc.ticks += mm.ran;                    // potential iterations (the reference's work)
              if (s < 0) res = -1; else mpend = s > 0;
            }
            const unsigned long long pm = __ballot(res == 0 && mpend), am = __ballot(res == 0);
            if (pm != 0ull && (__popcll(pm) >= kMarchBatch || pm == am) && res == 0 && mpend) {
              mpend = false;
              res = mm.finish(S.fractal, S.fractal_pw, &nrm);
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < kMarchK; ++u) {
            if (res == 0) {
              res = julia ? jm.tick(S.fractal, r.o) : mm.tick(S.fractal, S.fractal_pw, r.o, &nrm);
              ++tc.ticks;
            }
          }
        }
        if (res == 0) return false;
        marching = false;
        if (res > 0) {
          if (ANY) { h.ref = 0u; return true; }
          h.t = julia ? jm.d : mm.d;                  // mandelInter ignores rayMax (T10); Julia checked onRay
          h.ref = mref; h.b1 = 0.f; h.b2 = 0.f;
        }
        ++pfirst; --pcount;
        return false;
      }
      if (pcount > 0u) {
        const uint32_t ref = (ALLL || pfirst < L.n_refs) ? L.refs[pfirst] : S.leaf_refs[pfirst];
        if ((ref >> 30) == REF_FRACTAL) {
          ++tc.shapes;
          float d0;
          const Ray re{r.o, r.d, r.tmin, ANY ? r.tmax : h.t};
          const bool in = S.fractal.kind == BLING_FRACTAL_JULIA ? jm.start(re) : mandel_entry(re, &d0);
          if (in && pre) {                       // marched by k_march from the same entry point
            ++pfirst; --pcount;
            if (mres >= 0.f) {
              if (ANY) { h.ref = 0u; return true; }
              h.t = mres; h.ref = ref; h.b1 = 0.f; h.b2 = 0.f;   // mandelInter ignores rayMax (T10)
            }
            return false;
          }
          if (in) {
            if (S.fractal.kind != BLING_FRACTAL_JULIA) mm.start(r, d0);
            marching = true; mref = ref;
          } else {
            ++pfirst; --pcount;
          }
          return false;
        }
      }
    }
    // "if-if" step: a lane that tests the last primitive of its leaf goes on to the next node in the
    // same iteration (the wave runs both phases whenever any lane needs them, so this progress is
    // free); the order of node visits and primitive tests per ray is unchanged
    if (pcount > 0u) {
      if (prim_hit<ANY, F, ALLL>(S, L, pfirst, r, h, tc) && ANY) { h.ref = 0u; return true; }
      ++pfirst; --pcount;
      if (pcount > 0u || ((F & FT_FRACTAL) && marching)) return false;
    }
    if (node == NONE) {
      if (sp == 0) return true;
      --sp;
      take(L.stack[sp * TRACE_BLOCK]);
      if (node == NONE) return false;            // popped a leaf: its primitives come next
    }
    float4 n0, n1, n2, n3;
    if (ALLL || (uint32_t)node < L.n_nodes) {
      const float4* np = L.nodes + 4 * node;
      n0 = np[0]; n1 = np[1]; n2 = np[2]; n3 = np[3];
      asm volatile("" ::: "memory");             // see prim_hit: no merged FLAT load
    } else {
      n0 = gen(S.nodes[4 * node]); n1 = gen(S.nodes[4 * node + 1]); n2 = gen(S.nodes[4 * node + 2]); n3 = gen(S.nodes[4 * node + 3]);
      asm volatile("" ::: "memory");
    }
    ++tc.nodes;
    float t0, t1;
    bool h1;
    bool h0 = box2(n0, n1, n2, r.o, inv, r.tmin, h.t, &t0, &t1, &h1);
    int32_t c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y);
    if (h0 && h1) {
      bool first0 = t0 <= t1;
      if (F & FT_FRACTAL) {
        // mandelInter ignores rayMax (trap T10), so the order in which a fractal and a nearer
        // primitive are tested decides the hit.  Fractal scenes keep the order of the leaf fold
        // (leaves before inner children, leaves in child order), which agrees with the
        // reference's kd traversal on the golden rays; other scenes go near-first.
        const bool l0 = c0 < 0, l1 = c1 < 0;
        first0 = (l0 != l1) ? l0 : (l0 ? true : first0);
      }
      L.stack[sp * TRACE_BLOCK] = first0 ? c1 : c0;
      ++sp;
      take(first0 ? c0 : c1);
    } else if (h0) {
      take(c0);
    } else if (h1) {
      take(c1);
    } else {
      node = NONE;
    }
    return false;
  }
};

#ifndef BLING_QBVH4
#define BLING_QBVH4 0
#endif
constexpr bool kQuantBvh4 = BLING_QBVH4 != 0;   // experiment builds only (see Traversal4)

// Primitives of a leaf tested per Traversal4 step: two for the all-LDS kernel (fewer loop
// iterations of the small, issue-bound walk: C2 closest-hit 40.2 -> 37.7 ms per pass), one with a
// global fallback (two measured -4 % on C3; profiles/r02_ab_prim_unroll_s5.txt).
// One ray's traversal of the 4-wide tree (DevScene::nodes4), the same resumable unit steps as
// Traversal: a step visits one BVH4 node (four child boxes) or tests one primitive.  Hit children
// are ordered near-first by their entry distance (five compare-exchanges), the nearest is taken and
// the others pushed farthest-first.  Against the BVH2 this halves the dependent node fetches per ray
// (cornell 7.6 -> ~4 visits, ducky 12.1 -> ~6), which is what the latency-bound kernels wait on.
// The stack keeps S.stack4_lds rows in LDS; deeper rows (never on small trees: the host plans the
// whole bound into LDS when it fits, and ALLL implies it) go to S.stack4_ovf.
// Node format: float nodes (7 float4).  An experiment build with BLING_QBVH4=1 gives every BVH4
// kernel but the all-LDS one quantized nodes instead (bvh::quantize4, 4 float4 = 64 B: 43 % fewer
// bytes and load instructions per visit, 1.75x the LDS node prefix), each plane decoded with one
// convert and one fma, bit for bit the host's bvh::dequant -- boxes that contain the float boxes, so
// the same primitives are reached (parity green, 61 tests).  Measured on MI355X it loses: C3 5 842 ->
// 5 656 Mrays/s (-3 %; profiles/r04_ab_session.txt r04u): the meshes traversal waits on dependent
// node latency, not on bytes, and the decode adds issue slots to every visit.  The host uploads one
// format per scene (core.hip upload).
// Not used by fractal profiles, whose leaf-order rule (trap T10) is written for the BVH2.
#ifndef BLING_ANY_UNSORTED
#define BLING_ANY_UNSORTED 1
#endif
constexpr bool kAnyUnsorted = BLING_ANY_UNSORTED != 0;
#ifndef BLING_TRAV_VOTE
#define BLING_TRAV_VOTE 0
#endif
constexpr bool kTravVote = BLING_TRAV_VOTE != 0;
#ifndef BLING_PUSH_NB
#define BLING_PUSH_NB 1
#endif
constexpr bool kPushNb = BLING_PUSH_NB != 0;   // all-LDS kernels: branch-free pushes (Traversal4::step)
#ifndef BLING_LEAF_GLOBAL
#define BLING_LEAF_GLOBAL 1
#endif
constexpr bool kLeafGlobal = BLING_LEAF_GLOBAL != 0;   // global-fallback kernels: leaf_hit_global
template <bool ANY, uint32_t F, bool ALLL = false>
struct Traversal4 {
  static constexpr int32_t NONE = 0x7FFFFFFF;
  static constexpr int kPrimUnroll = ALLL ? 2 : 1;
  Ray r;
  V3 inv;
  HitRec h;
  int32_t node, sp;
  uint32_t pfirst, pcount;

  DEV void init(const Ray& ray, bool rejected = false) {      // rejected: see Traversal::init
    r = ray;
    inv = mk(bfast::rcp_cr(r.d.x), bfast::rcp_cr(r.d.y), bfast::rcp_cr(r.d.z));
    h.t = r.tmax; h.ref = REF_NONE; h.b1 = h.b2 = 0.f;
    node = rejected ? NONE : 0; sp = 0; pfirst = 0u; pcount = 0u;
  }
  DEV void take(int32_t link) {
    if (link < 0) { uint32_t code = ~(uint32_t)link; pfirst = code >> 8; pcount = code & 0xFFu; node = NONE; }
    else node = link;
  }
  DEV void push(const DevScene& S, const LdsScene& L, int32_t v) {
    if (ALLL || (uint32_t)sp < S.stack4_lds) L.stack[sp * TRACE_BLOCK] = v;
    else S.stack4_ovf[(size_t)((uint32_t)sp - S.stack4_lds) * S.stack4_lanes + blockIdx.x * blockDim.x + threadIdx.x] = v;
    ++sp;
  }
  DEV int32_t pop(const DevScene& S, const LdsScene& L) {
    --sp;
    if (ALLL || (uint32_t)sp < S.stack4_lds) return L.stack[sp * TRACE_BLOCK];
    return S.stack4_ovf[(size_t)((uint32_t)sp - S.stack4_lds) * S.stack4_lanes + blockIdx.x * blockDim.x + threadIdx.x];
  }
  // four planes of one axis from their bytes: bvh::dequant, (float)q x 2^e exact, one rounding
  DEV static float4 dequant4(uint32_t w, float s, float o) {
    return make_float4(__builtin_fmaf((float)(w & 0xFFu), s, o), __builtin_fmaf((float)((w >> 8) & 0xFFu), s, o),
                       __builtin_fmaf((float)((w >> 16) & 0xFFu), s, o), __builtin_fmaf((float)(w >> 24), s, o));
  }
  DEV static void cx(float& ka, int32_t& la, float& kb, int32_t& lb) {
    const bool sw = kb < ka;
    const float k = sw ? kb : ka; kb = sw ? ka : kb; ka = k;
    const int32_t l = sw ? lb : la; lb = sw ? la : lb; la = l;
  }
  DEV bool step(const DevScene& S, const LdsScene& L, TraceCount& tc) {
    if constexpr (ALLL && kTravVote) {
      // experiment builds (BLING_TRAV_VOTE): one phase per iteration for the whole wave -- primitive
      // tests when at least half of the calling lanes have some pending, else node visits
      const bool wp = pcount > 0u;
      const bool prim_phase = 2 * __popcll(__ballot(wp)) >= __popcll(__ballot(true));
      if (prim_phase != wp) return false;
      if (wp) {
        if (prim_hit<ANY, F, ALLL>(S, L, pfirst, r, h, tc) && ANY) { h.ref = 0u; return true; }
        ++pfirst; --pcount;
#pragma unroll
        for (int u = 1; u < kPrimUnroll; ++u) {
          if (pcount > 0u) {
            if (prim_hit<ANY, F, ALLL>(S, L, pfirst, r, h, tc) && ANY) { h.ref = 0u; return true; }
            ++pfirst; --pcount;
          }
        }
        return false;
      }
    }
    if constexpr (ALLL && !kTravVote) {
      if (pcount > 0u) {                         // a whole leaf (at most two primitives) per step
        // both records' loads issue together; the second may be the zero record past the last leaf
        // slot, and is tested only when the leaf has it
        if constexpr (kLeafPair) {
          LeafRec q0, q1;
          leaf_rec2(L, pfirst, q0, q1);
          if (leaf_hit<ANY, F>(L, q0, r, h, tc) && ANY) { h.ref = 0u; return true; }
          if (pcount > 1u && leaf_hit<ANY, F>(L, q1, r, h, tc) && ANY) { h.ref = 0u; return true; }
        } else {
          if (leaf_hit<ANY, F>(L, leaf_rec1(L, pfirst), r, h, tc) && ANY) { h.ref = 0u; return true; }
          if (pcount > 1u && leaf_hit<ANY, F>(L, leaf_rec1(L, pfirst + 1u), r, h, tc) && ANY) { h.ref = 0u; return true; }
        }
        pfirst += min(pcount, 2u); pcount -= min(pcount, 2u);
        if (pcount > 0u) return false;
      }
    } else if (pcount > 0u) {                    // "if-if": see Traversal::step
      if (((kLeafGlobal && !ALLL) ? leaf_hit_global<ANY, F>(S, L, pfirst, r, h, tc) : prim_hit<ANY, F, ALLL>(S, L, pfirst, r, h, tc)) && ANY) {
        h.ref = 0u;
        return true;
      }
      ++pfirst; --pcount;
#pragma unroll
      for (int u = 1; u < kPrimUnroll; ++u) {    // further primitives of the same leaf, same order
        if (pcount > 0u) {
          if (prim_hit<ANY, F, ALLL>(S, L, pfirst, r, h, tc) && ANY) { h.ref = 0u; return true; }
          ++pfirst; --pcount;
        }
      }
      if (pcount > 0u) return false;
    }
    if (node == NONE) {
      if (sp == 0) return true;
      take(pop(S, L));
      if (node == NONE) return false;            // popped a leaf: its primitives come next
    }
    float4 lx, ly, lz, hx, hy, hz, lk;
    if constexpr (ALLL || !kQuantBvh4) {
      if (ALLL || (uint32_t)node < L.n_nodes) {
        const float4* np = L.nodes + 7 * node;
        lx = np[0]; ly = np[1]; lz = np[2]; hx = np[3]; hy = np[4]; hz = np[5]; lk = np[6];
        asm volatile("" ::: "memory");           // see prim_hit: no merged FLAT load
      } else {
        const gptr<float4> np = S.nodes4 + 7 * node;
        lx = gen(np[0]); ly = gen(np[1]); lz = gen(np[2]); hx = gen(np[3]); hy = gen(np[4]); hz = gen(np[5]); lk = gen(np[6]);
        asm volatile("" ::: "memory");
      }
    } else {
      float4 qa, qb, qc;
      if ((uint32_t)node < L.n_nodes) {
        const float4* np = L.nodes + 4 * node;
        qa = np[0]; qb = np[1]; qc = np[2]; lk = np[3];
        asm volatile("" ::: "memory");
      } else {
        const gptr<float4> np = S.nodes4 + 4 * node;
        qa = gen(np[0]); qb = gen(np[1]); qc = gen(np[2]); lk = gen(np[3]);
        asm volatile("" ::: "memory");
      }
      // words: origin xyz, scale x | scale yz, lo bytes x y | lo bytes z, hi bytes x y z
      lx = dequant4(__float_as_uint(qb.z), qa.w, qa.x); ly = dequant4(__float_as_uint(qb.w), qb.x, qa.y);
      lz = dequant4(__float_as_uint(qc.x), qb.y, qa.z); hx = dequant4(__float_as_uint(qc.y), qa.w, qa.x);
      hy = dequant4(__float_as_uint(qc.z), qb.x, qa.y); hz = dequant4(__float_as_uint(qc.w), qb.y, qa.z);
    }
    ++tc.nodes;
    const float ox = r.o.x, oy = r.o.y, oz = r.o.z, tmin = r.tmin, tmax = h.t;
    float key[4];
    int32_t lnk[4] = {__float_as_int(lk.x), __float_as_int(lk.y), __float_as_int(lk.z), __float_as_int(lk.w)};
    const float blx[4] = {lx.x, lx.y, lx.z, lx.w}, bly[4] = {ly.x, ly.y, ly.z, ly.w}, blz[4] = {lz.x, lz.y, lz.z, lz.w};
    const float bhx[4] = {hx.x, hx.y, hx.z, hx.w}, bhy[4] = {hy.x, hy.y, hy.z, hy.w}, bhz[4] = {hz.x, hz.y, hz.z, hz.w};
    int nh = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {                // box1's slab arithmetic per child
      const float ax = (blx[k] - ox) * inv.x, bx = (bhx[k] - ox) * inv.x;
      const float ay = (bly[k] - oy) * inv.y, by = (bhy[k] - oy) * inv.y;
      const float az = (blz[k] - oz) * inv.z, bz = (bhz[k] - oz) * inv.z;
      const float lo = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
      const float hi = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
      const bool hit = lo <= hi && lnk[k] != bvh4_empty;
      key[k] = hit ? fminf(lo, 3.0e38f) : INFINITY;
      nh += hit ? 1 : 0;
    }
    if (nh == 0) { node = NONE; return false; }
    if (ANY && kAnyUnsorted) {                   // any-hit is order-free: no near-first sort
      int32_t first = NONE;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (key[k] != INFINITY) {
          if (first == NONE) first = lnk[k];
          else push(S, L, lnk[k]);
        }
      }
      take(first);
      return false;
    }
    cx(key[0], lnk[0], key[1], lnk[1]);
    cx(key[2], lnk[2], key[3], lnk[3]);
    cx(key[0], lnk[0], key[2], lnk[2]);
    cx(key[1], lnk[1], key[3], lnk[3]);
    cx(key[1], lnk[1], key[2], lnk[2]);
    if constexpr (ALLL && kPushNb) {
      // the same pushes (lnk[nh - 1] .. lnk[1], farthest first) as three unconditional stores to rows
      // sp .. sp + 2 (the host plans spare rows) and one add: no branch per push
      const int32_t s0 = nh > 3 ? lnk[3] : (nh > 2 ? lnk[2] : lnk[1]);
      const int32_t s1 = nh > 3 ? lnk[2] : lnk[1];
      L.stack[sp * TRACE_BLOCK] = s0;
      L.stack[(sp + 1) * TRACE_BLOCK] = s1;
      L.stack[(sp + 2) * TRACE_BLOCK] = lnk[1];
      sp += nh - 1;
      take(lnk[0]);
      return false;
    }
    if (nh > 3) push(S, L, lnk[3]);
    if (nh > 2) push(S, L, lnk[2]);
    if (nh > 1) push(S, L, lnk[1]);
    take(lnk[0]);
    return false;
  }
};

// Any-hit query of one ray against the LDS copy of the whole BVH4 (lds_all4 scenes), for the shading
// kernel's in-line shadow test (wavefront.h inline_shadow): the same padded boxes, slab arithmetic
// and primitive tests as Traversal4<true, F, true>, with the stack in registers (a shift register of
// kShadowStack entries, static indices only -- the host enables it only when the tree's exact stack
// bound fits) instead of LDS rows.  Any-hit is order-free: true iff some primitive tests a hit in
// [tmin, tmax], whatever the visiting order, so the answer is the traversal kernel's.
constexpr int kShadowStack = 8;
template <uint32_t F>
DEV bool occluded_lds(const DevScene& S, const LdsScene& L, const Ray& r) {
  const V3 inv = mk(bfast::rcp_cr(r.d.x), bfast::rcp_cr(r.d.y), bfast::rcp_cr(r.d.z));
  HitRec h{r.tmax, REF_NONE, 0.f, 0.f};
  TraceCount tc{0u, 0u, 0u, 0u};
  int32_t stk[kShadowStack];
#pragma unroll
  for (int i = 0; i < kShadowStack; ++i) stk[i] = 0;
  int sp = 0;
  int32_t link = 0;                               // the root
  for (;;) {
    bool next = false;                            // a hit child taken directly (Traversal4's order of pushes)
    if (link < 0) {                               // a leaf: its primitives
      const uint32_t code = ~(uint32_t)link, first = code >> 8, cnt = code & 0xFFu;
      for (uint32_t q = 0; q < cnt; ++q)
        if (prim_hit<true, F, true>(S, L, first + q, r, h, tc)) return true;
    } else {                                      // an inner node: one hit child next, the others pushed
      const float4* np = L.nodes + 7 * link;
      const float4 lx = np[0], ly = np[1], lz = np[2], hx = np[3], hy = np[4], hz = np[5], lk = np[6];
      const int32_t lnk[4] = {__float_as_int(lk.x), __float_as_int(lk.y), __float_as_int(lk.z), __float_as_int(lk.w)};
      const float blx[4] = {lx.x, lx.y, lx.z, lx.w}, bly[4] = {ly.x, ly.y, ly.z, ly.w}, blz[4] = {lz.x, lz.y, lz.z, lz.w};
      const float bhx[4] = {hx.x, hx.y, hx.z, hx.w}, bhy[4] = {hy.x, hy.y, hy.z, hy.w}, bhz[4] = {hz.x, hz.y, hz.z, hz.w};
      int32_t take = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {               // Traversal4's slab arithmetic per child
        const float ax = (blx[k] - r.o.x) * inv.x, bx = (bhx[k] - r.o.x) * inv.x;
        const float ay = (bly[k] - r.o.y) * inv.y, by = (bhy[k] - r.o.y) * inv.y;
        const float az = (blz[k] - r.o.z) * inv.z, bz = (bhz[k] - r.o.z) * inv.z;
        const float lo = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), r.tmin));
        const float hi = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), h.t));
        if (lo <= hi && lnk[k] != bvh4_empty) {
          if (!next) { take = lnk[k]; next = true; }
          else if (sp < kShadowStack) {           // never full: the host enables this for stack bounds <= 8
#pragma unroll
            for (int i = kShadowStack - 1; i > 0; --i) stk[i] = stk[i - 1];
            stk[0] = lnk[k];
            ++sp;
          }
        }
      }
      link = take;
    }
    if (next) continue;
    if (sp == 0) return false;
    link = stk[0];
#pragma unroll
    for (int i = 0; i < kShadowStack - 1; ++i) stk[i] = stk[i + 1];
    --sp;
  }
}

template <bool ANY, uint32_t F, bool ALLL>
using QTraversal = typename std::conditional<use_bvh4<F>(), Traversal4<ANY, F, ALLL>, Traversal<ANY, F, ALLL>>::type;

// Whole traversal of one ray (bling_trace batches).
template <bool ANY, uint32_t F>
DEV bool trace(const DevScene& S, const LdsScene& L, const Ray& r, HitRec& h, TraceCount& tc) {
  Traversal<ANY, F> tv;
  tv.init(r);
  tv.reject_outside(S);
  while (!tv.step(S, L, tc)) {}
  h = tv.h;
  return h.ref != REF_NONE;
}

}  // namespace bd
