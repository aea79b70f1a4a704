// sppm.h -- the SPPM renderer (Renderer/SPPM.hs) on the device, a second consumer of the trace
// core.  One pass (onePass, SPPM.hs:424-460):
//   k_sppm_eye      one random camera sample per sample-extent pixel; each thread walks its
//                   sample's ray tree depth-first (traceCam / followCam, :89-131), appends a hit
//                   point at every hit with a non-specular lobe and writes Ls for the tile film
//   k_film          addSample of Ls (the path core's tile film, wavefront.h)
//   k_sppm_reduce   largest radius^2 and hit-point bounds -> the hash grid (mkHash, :316-349)
//   k_sppm_cells    count -> scan -> fill: hit point ids per hash bucket (CSR)
//   k_sppm_kd       each bucket's kd-tree (mkKdTree, :363-389), implicit in the bucket's order
//   k_sppm_photon   one thread per photon (tracePhoton / followPhoton, :181-239): every hit with a
//                   non-specular lobe splats into the pixels of the hit points around it
//   k_sppm_stats    mergeStats + statsUpdate (:259-291)
// Each hit point stores its BSDF record (~200 B: lobes with texture pointers, frame, normal) so a
// photon pair costs one load and evalBsdf, not a re-shade of the hit.  Splats and counts are float / u32 atomics: the sum order differs
// from the reference's per-thread images, the set of contributions does not.
#pragma once
#include "wavefront.h"

namespace bd {

constexpr uint32_t DIM_SPPM_1D = 0x100000u, DIM_SPPM_2D = 0x200000u, SPPM_PHOTON_PIXEL = 0x80000000u;
constexpr int SPPM_MAX_DEPTH = 16;               // eye-tree depth bound (one parked sibling per level)
constexpr int SPPM_PHOTON_BOUNCES = 1 << 16;     // exit bound of the (unbounded) photon walk

struct SppmGrid { float lo[3]; float scale; float r2max; uint32_t cnt; uint32_t items; uint32_t pad; };

struct SppmBufs {
  float4* hp_pos;        // shading point p.xyz, r2
  float4* hp_hit;        // closest hit: t, ref, b1, b2
  float4* hp_o;          // eye ray o.xyz, imageX
  float4* hp_d;          // eye ray d.xyz, imageY
  float4* hp_f;          // [cap][4] throughput t of the node (hpF)
  Bsdf* hp_bsdf;         // the hit point's BSDF (hpBsdf), built once by the eye pass
  uint32_t* hp_count;    // hit points appended (may exceed hp_cap: the host re-runs the eye pass)
  uint32_t hp_cap;
  float* r2;             // psR2 per stats pixel (windowPixels entries)
  float* nacc;           // psN
  uint32_t* cnt;         // [threads][n_stats] photon hits per pixel and photon sampler (psM per seed)
  uint32_t n_stats;
  SppmGrid* grid;
  uint32_t* bstart;      // [cells + 1] bucket offsets
  uint32_t* bcur;        // [cells] fill cursors
  uint32_t* items;       // hit point ids, bucket by bucket; k_sppm_kd reorders each bucket into its kd-tree
  uint32_t items_cap;
  unsigned long long* hp_key;   // pixel << 24 | eye-tree node id: the kd-tree's tie order
  float* kd_mr;          // per items entry: the node's mr at a pivot position (k_sppm_kd)
  float* kd_c;           // per items entry: scratch of k_sppm_kd (r2 of a pivot, r of a leaf)
  float* splat;          // W * H * 3 (X, Y, Z), accumulated
  unsigned long long* ctr;   // [0] eye rays, [1] photon rays, [2] photon/hit-point pairs, [3] dropped
};

// sIdx (SPPM.hs:266-270), literally: row stride xEnd - xStart, truncation towards zero
DEV int64_t sppm_sidx(const DevScene& S, float px, float py) {
  const int64_t w = S.ex1 - S.ex0, h = S.ey1 - S.ey0;
  const int64_t ix = min(w, (int64_t)px), iy = min(h, (int64_t)py);
  return w * (iy - S.ey0) + (ix - S.ex0);
}

// hash (SPPM.hs:303-305) on 64-bit Int (wrapping products), abs, `rem cnt`, clamped
DEV uint32_t sppm_bucket(int64_t x, int64_t y, int64_t z, uint32_t cnt) {
  uint64_t hv = ((uint64_t)x * 73856093ull) ^ ((uint64_t)y * 19349663ull) ^ ((uint64_t)z * 83492791ull);
  int64_t a = (int64_t)hv;
  if (a < 0) a = (int64_t)(0ull - (uint64_t)a);
  int64_t r = a % (int64_t)cnt;
  return (uint32_t)max((int64_t)0, min((int64_t)cnt - 1, r));
}

DEV bool has_non_specular(const Bsdf& b) {                                          // bsdfHasNonSpecular
  bool r = false;
#pragma unroll
  for (int i = 0; i < 2; ++i) if (i < b.n && !has_flag(b.b[i], F_SPEC)) r = true;
  return r;
}

// ------------------------------------------------------------------ eye pass
struct SppmPend { float4 o, d; Sp t; };

template <uint32_t F>
static __global__ __launch_bounds__(256) void k_sppm_eye(const DevScene* __restrict__ Sptr, SppmBufs B, WaveState W,
                                                  const TileDesc* __restrict__ tiles, uint32_t seed, uint32_t pass) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup(S, smem);
  const TileDesc td = tiles[blockIdx.y];
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long rays = 0, dropped = 0;
  if (j < td.count) {
    const int tw = td.x1 - td.x0 + 1;
    const int ix = td.x0 + (int)(j % (uint32_t)tw), iy = td.y0 + (int)(j / (uint32_t)tw);
    const uint32_t pixel = (uint32_t)((iy - S.ey0) * S.ext_w + (ix - S.ex0));
    const uint32_t sk = brng::sample_key(brng::pixel_key(seed, pass, pixel), 0u);
    // mkRandomSampler 1 camera sample (Sampling.hs:101-110)
    const float ox = brng::u01(brng::draw(sk, brng::DIM_RAND_CAM)), oy = brng::u01(brng::draw(sk, brng::DIM_RAND_CAM + 1));
    const float lu = brng::u01(brng::draw(sk, brng::DIM_RAND_CAM + 2)), lv = brng::u01(brng::draw(sk, brng::DIM_RAND_CAM + 3));
    const float px = (float)ix + ox, py = (float)iy + oy;
    Ray ray = fire_ray(S.camera, px, py, lu, lv);
    const float r2 = B.r2[sppm_sidx(S, px, py)];
    SppmPend pend[SPPM_MAX_DEPTH];
    int np = 0, depth = 0;
    uint32_t id = 1u;
    Sp t = sconst(1.f), Ls = sconst(0.f);
    for (;;) {
      bool next = false;
      Ray nray;
      Sp nt;
      int ndepth = 0;
      uint32_t nid = 0u;
      ++rays;
      HitRec h;
      TraceCount tc{0u, 0u, 0u, 0u};
      if (!trace<false, F>(S, L, ray, h, tc)) {                          // escaped (SPPM.hs:74-75, 116)
        Sp sum = sconst(0.f);
        for (int l = 0; l < S.num_lights; ++l) sum = sum + light_le<F>(gen(S.lights[l]), ray.d);
        Ls = Ls + t * sum;
      } else {
        const float4 hv = make_float4(h.t, __uint_as_float(h.ref), h.b1, h.b2);
        DG dgg, dgs;
        float eps;
        int mat, hit_light;
        hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
        Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs);
        const V3 wo = -ray.d;
        if (hit_light >= 0 && dot(dgg.n, ray.d) > 0.f)                   // intLe int (-wo) (:122, trap T6)
          Ls = Ls + t * sload(gen(S.lights[hit_light]).radiance);
        if (has_non_specular(bsdf)) {
          const uint32_t slot = atomicAdd(B.hp_count, 1u);
          if (slot < B.hp_cap) {
            B.hp_pos[slot] = make_float4(bsdf.p.x, bsdf.p.y, bsdf.p.z, r2);
            B.hp_hit[slot] = hv;
            B.hp_o[slot] = make_float4(ray.o.x, ray.o.y, ray.o.z, px);
            B.hp_d[slot] = make_float4(ray.d.x, ray.d.y, ray.d.z, py);
            store_sp(B.hp_f, slot, t);
            B.hp_bsdf[slot] = bsdf;
            B.hp_key[slot] = (unsigned long long)pixel << 24 | id;
          }
        }
        if (depth + 1 != S.max_depth) {                                  // children at maxDepth do nothing
          const float4 po = make_float4(bsdf.p.x, bsdf.p.y, bsdf.p.z, eps);
#pragma unroll
          for (int c = 0; c < 2; ++c) {                                  // followCam Reflection, then Transmission
            const uint32_t cid = 2u * id + (uint32_t)c;
            const float bc = brng::u01(brng::draw(sk, DIM_SPPM_1D + cid));
            const float b1 = brng::u01(brng::draw(sk, DIM_SPPM_2D + 2u * cid));
            const float b2 = brng::u01(brng::draw(sk, DIM_SPPM_2D + 2u * cid + 1u));
            Sp f; V3 wi;
            const float pdf = sample_bsdf_spec<F>(bsdf, wo, c == 0 ? F_REFL : F_TRANS, bc, b1, b2, f, wi);
            if (pdf == 0.f || is_black(f)) continue;
            if (!next) {
              next = true; nray = Ray{bsdf.p, wi, eps, INFINITY}; nt = f * t; ndepth = depth + 1; nid = cid;
            } else if (np < SPPM_MAX_DEPTH) {                            // park the transmission sibling
              pend[np].o = po;
              pend[np].d = make_float4(wi.x, wi.y, wi.z, __uint_as_float(((uint32_t)(depth + 1) << 24) | cid));
              pend[np].t = f * t;
              ++np;
            }
          }
        }
      }
      if (!next) {
        if (np == 0) break;
        --np;
        const float4 o = pend[np].o, d = pend[np].d;
        const uint32_t code = __float_as_uint(d.w);
        nray = Ray{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, INFINITY};
        nt = pend[np].t; ndepth = (int)(code >> 24); nid = code & 0xFFFFFFu;
      }
      ray = nray; t = nt; depth = ndepth; id = nid;
    }
    const uint32_t i = td.offset + j;
    W.img[i] = make_float2(px, py);
    if (s_bad(Ls)) { W.result[i] = make_float4(0.f, 0.f, 0.f, 0.f); dropped = 1; }
    else {
      float x, y, z;
      to_xyz(Ls, &x, &y, &z);
      W.result[i] = make_float4(x, y, z, 1.f);
    }
  }
  const unsigned long long wr = wave_sum_u64(rays), wd = wave_sum_u64(dropped);
  if ((threadIdx.x & 63) == 0) {
    if (wr) atomicAdd(&B.ctr[0], wr);
    if (wd) atomicAdd(&B.ctr[3], wd);
  }
}

// ------------------------------------------------------------------ hash grid (mkHash)
// One block: max r2 (foldl' max from 0) and the hit-point bounds; the grid bounds are
// (min p) - r, (max p) + r (the union of every mkAABB (p - r) (p + r), rounding being monotonic).
static __global__ __launch_bounds__(1024) void k_sppm_reduce(SppmBufs B) {
  __shared__ float red[7][1024];
  const uint32_t n = min(*B.hp_count, B.hp_cap);
  float r2m = 0.f, lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float4 p = B.hp_pos[i];
    r2m = p.w <= r2m ? r2m : p.w;
    lo[0] = fminf(lo[0], p.x); lo[1] = fminf(lo[1], p.y); lo[2] = fminf(lo[2], p.z);
    hi[0] = fmaxf(hi[0], p.x); hi[1] = fmaxf(hi[1], p.y); hi[2] = fmaxf(hi[2], p.z);
  }
  red[0][threadIdx.x] = r2m;
  for (int a = 0; a < 3; ++a) { red[1 + a][threadIdx.x] = lo[a]; red[4 + a][threadIdx.x] = hi[a]; }
  __syncthreads();
  for (uint32_t s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const uint32_t o = threadIdx.x + s;
      red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][o]);
      for (int a = 0; a < 3; ++a) {
        red[1 + a][threadIdx.x] = fminf(red[1 + a][threadIdx.x], red[1 + a][o]);
        red[4 + a][threadIdx.x] = fmaxf(red[4 + a][threadIdx.x], red[4 + a][o]);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float r = sqrtf(red[0][0]);
    SppmGrid g;
    for (int a = 0; a < 3; ++a) g.lo[a] = red[1 + a][0] - r;
    g.scale = 1.f / (2.f * r);
    g.r2max = red[0][0];
    g.cnt = n;
    g.items = 0u;
    g.pad = 0u;
    *B.grid = g;
  }
}

// the cells a hit point's own radius overlaps (mkHash insertion, SPPM.hs:329-344)
DEV void sppm_cell_range(const SppmGrid& g, float4 p, int64_t c0[3], int64_t c1[3]) {
  const float rp = sqrtf(p.w);
  const float pc[3] = {p.x, p.y, p.z};
  for (int a = 0; a < 3; ++a) {
    c0[a] = (int64_t)(g.scale * fabsf((pc[a] - rp) - g.lo[a]));
    c1[a] = (int64_t)(g.scale * fabsf((pc[a] + rp) - g.lo[a]));
  }
}

template <bool FILL>
static __global__ __launch_bounds__(256) void k_sppm_cells(SppmBufs B) {
  const SppmGrid g = *B.grid;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.cnt) return;
  const float4 p = B.hp_pos[i];
  if (p.w == 0.f) return;                                             // unless (r2p == 0)
  int64_t c0[3], c1[3];
  sppm_cell_range(g, p, c0, c1);
  for (int64_t x = c0[0]; x <= c1[0]; ++x)
    for (int64_t y = c0[1]; y <= c1[1]; ++y)
      for (int64_t z = c0[2]; z <= c1[2]; ++z) {
        const uint32_t b = sppm_bucket(x, y, z, g.cnt);
        if (FILL) B.items[atomicAdd(&B.bcur[b], 1u)] = i;
        else atomicAdd(&B.bstart[b], 1u);
      }
}

// exclusive scan of the bucket counts in one block (cells = hit points, a few 10^5): bstart[cnt]
// = total entries; bcur = bstart
static __global__ __launch_bounds__(1024) void k_sppm_scan(SppmBufs B) {
  __shared__ uint32_t part[1024];
  const uint32_t n = B.grid->cnt;
  const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = min(n, threadIdx.x * per), b1 = min(n, b0 + per);
  uint32_t s = 0;
  for (uint32_t k = b0; k < b1; ++k) s += B.bstart[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < blockDim.x; off <<= 1) {                 // Hillis-Steele inclusive scan
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (uint32_t k = b0; k < b1; ++k) {
    const uint32_t c = B.bstart[k];
    B.bstart[k] = run; B.bcur[k] = run;
    run += c;
  }
  if (threadIdx.x == blockDim.x - 1) { B.bstart[n] = part[threadIdx.x]; B.grid->items = part[threadIdx.x]; }
}

// ------------------------------------------------------------------ per-bucket kd-tree
// mkKdTree (SPPM.hs:363-389) as an implicit tree over the bucket's range of `items` -- the oracle's
// sppm_kd_build, which documents the layout: a range of more than five entries is a Node whose pivot
// is the entry of rank (u - l) `quot` 2 on axis depth `rem` 3 (ties by hp_key), the smaller ones
// left, the rest right; kd_mr at the pivot's position is the node's mr, max (hpR2 pivot) (max lr rr)
// with a Leaf's value sqrt of its largest r2.  One thread per bucket; the ranges are sorted top-down
// (heapsort: no recursion, no scratch stack beyond a fixed array), the mr values from the final order.
struct KdRange { uint32_t l, u, depth; };
constexpr int SPPM_KD_STACK = 64;        // > 2 log2(entries): a range's depth never exceeds 32
DEV bool kd_less(const SppmBufs& B, uint32_t a, uint32_t b, int axis) {
  const float4 pa = B.hp_pos[a], pb = B.hp_pos[b];
  const float ca = axis == 0 ? pa.x : (axis == 1 ? pa.y : pa.z), cb = axis == 0 ? pb.x : (axis == 1 ? pb.y : pb.z);
  return ca < cb || (!(cb < ca) && B.hp_key[a] < B.hp_key[b]);
}
DEV void kd_sift(const SppmBufs& B, uint32_t* v, uint32_t root, uint32_t n, int axis) {
  for (;;) {
    uint32_t c = 2u * root + 1u;
    if (c >= n) return;
    if (c + 1u < n && kd_less(B, v[c], v[c + 1u], axis)) ++c;
    if (!kd_less(B, v[root], v[c], axis)) return;
    const uint32_t t = v[root]; v[root] = v[c]; v[c] = t;
    root = c;
  }
}
DEV void kd_sort(const SppmBufs& B, uint32_t* v, uint32_t n, int axis) {          // heapsort, ascending
  for (uint32_t i = n / 2u; i-- > 0u;) kd_sift(B, v, i, n, axis);
  for (uint32_t e = n; e-- > 1u;) {
    const uint32_t t = v[0]; v[0] = v[e]; v[e] = t;
    kd_sift(B, v, 0u, e, axis);
  }
}
static __global__ __launch_bounds__(256) void k_sppm_kd(SppmBufs B) {
  const SppmGrid g = *B.grid;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= g.cnt) return;
  const uint32_t b0 = B.bstart[b], b1 = B.bstart[b + 1];
  if (b1 <= b0) return;
  uint32_t* v = B.items + b0;
  float* c = B.kd_c + b0;
  float* mr = B.kd_mr + b0;
  KdRange st[SPPM_KD_STACK];
  int sp = 0;
  st[sp++] = KdRange{0u, b1 - b0, 0u};
  while (sp > 0) {                                                    // order and contributions
    const KdRange r = st[--sp];
    if (r.u - r.l <= 5u) {
      float m = 0.f;
      for (uint32_t i = r.l; i < r.u; ++i) m = hmax(m, B.hp_pos[v[i]].w);   // foldl' (\m hp -> max m r2) 0
      const float lv = sqrtf(m);
      for (uint32_t i = r.l; i < r.u; ++i) c[i] = lv;
      continue;
    }
    kd_sort(B, v + r.l, r.u - r.l, (int)(r.depth % 3u));
    const uint32_t m = r.l + (r.u - r.l) / 2u;
    c[m] = B.hp_pos[v[m]].w;
    if (sp + 2 > SPPM_KD_STACK) break;                                // cannot happen: depth <= 32
    st[sp++] = KdRange{m + 1u, r.u, r.depth + 1u};
    st[sp++] = KdRange{r.l, m, r.depth + 1u};
  }
  st[sp++] = KdRange{0u, b1 - b0, 0u};
  while (sp > 0) {                                                    // mr of every node
    const KdRange r = st[--sp];
    if (r.u - r.l <= 5u) continue;
    const uint32_t m = r.l + (r.u - r.l) / 2u;
    float x = 0.f;                                                    // values are >= 0: max is order-free
    for (uint32_t i = r.l; i < r.u; ++i) x = hmax(x, c[i]);
    mr[m] = x;
    st[sp++] = KdRange{m + 1u, r.u, r.depth + 1u};
    st[sp++] = KdRange{r.l, m, r.depth + 1u};
  }
}

// treeLookup (SPPM.hs:391-404) over bucket range [b0, b1): a Node tests its pivot, then descends
// left when pos - mr <= split and right when pos + mr >= split; a Leaf tests each of its entries
// against its own radius.  fn(i) for every hit point i found, left subtrees before right ones.
template <class Fn>
DEV void kd_lookup(const SppmBufs& B, uint32_t b0, uint32_t b1, V3 p, Fn&& fn) {
  KdRange st[SPPM_KD_STACK];
  int sp = 0;
  if (b1 > b0) st[sp++] = KdRange{b0, b1, 0u};
  const uint32_t* v = B.items;
  while (sp > 0) {
    const KdRange r = st[--sp];
    if (r.u - r.l <= 5u) {
      for (uint32_t e = r.l; e < r.u; ++e) {
        const uint32_t i = v[e];
        const float4 hp = B.hp_pos[i];
        if (sqlen(mk(hp.x, hp.y, hp.z) - p) <= hp.w) fn(i, hp);
      }
      continue;
    }
    const uint32_t m = r.l + (r.u - r.l) / 2u;
    const uint32_t i = v[m];
    const float4 hp = B.hp_pos[i];
    const uint32_t axis = r.depth % 3u;
    const float split = axis == 0u ? hp.x : (axis == 1u ? hp.y : hp.z);
    const float pos = axis == 0u ? p.x : (axis == 1u ? p.y : p.z);
    const float x = B.kd_mr[m];
    if (sqlen(mk(hp.x, hp.y, hp.z) - p) <= hp.w) fn(i, hp);
    if (sp + 2 > SPPM_KD_STACK) break;                                // cannot happen: depth <= 32
    if (pos + x >= split) st[sp++] = KdRange{m + 1u, r.u, r.depth + 1u};   // popped after the left subtree
    if (pos - x <= split) st[sp++] = KdRange{r.l, m, r.depth + 1u};
  }
}

// ------------------------------------------------------------------ photon pass
// Photon sampler: "thread" k's mkStratifiedSampler sn sn over one pixel with n1d = 7, n2d = 5
// (SPPM.hs:442, 470-473), the counter-RNG restatement of rnd' / rnd2D' (Sampling.hs:203-221)
struct PhotonSampler {
  uint32_t pk, n, spp, sn;
  float inv_spp, inv_sn;
  uint32_t sk;                                    // sample_key(pk, n) (common/counter_rng.h)
  DEV float rnd1(int dim) const {
    if (dim < 7) {
      const uint32_t j = brng::permute(n, spp, brng::draw(brng::sample_key(pk, brng::ALL_SAMPLES), brng::DIM_1D_PERM + dim));
      const float jit = brng::u01(brng::draw(sk, brng::DIM_1D_J + dim));
      return fminf(ALMOST_ONE, ((float)j + jit) * inv_spp);
    }
    return brng::u01(brng::draw(sk, brng::DIM_FRESH1D + dim));
  }
  DEV void rnd2(int dim, float* a, float* b) const {
    if (dim < 5) {
      const uint32_t j = brng::permute(n, spp, brng::draw(brng::sample_key(pk, brng::ALL_SAMPLES), brng::DIM_2D_PERM + dim));
      const float ju = brng::u01(brng::draw(sk, brng::DIM_2D_J + 2 * dim));
      const float jv = brng::u01(brng::draw(sk, brng::DIM_2D_J + 2 * dim + 1));
      const int u = (int)(j / sn), v = (int)(j % sn);                   // quotRem i nu (trap T5)
      *a = fminf(ALMOST_ONE, ((float)u + ju) * inv_sn);
      *b = fminf(ALMOST_ONE, ((float)v + jv) * inv_sn);
      return;
    }
    *a = brng::u01(brng::draw(sk, brng::DIM_FRESH2D + 2 * dim));
    *b = brng::u01(brng::draw(sk, brng::DIM_FRESH2D + 2 * dim + 1));
  }
};

// sample' (Light.hs:166-213) -> Le, ray, normal at the light, pdf
template <uint32_t F>
DEV float light_ray(const DevScene& S, const bling_light& L, float uo1, float uo2, float ud1, float ud2, Sp& li,
                    Ray& ray, V3& n) {
  if ((F & FT_DELTA) && L.kind >= BLING_LIGHT_POINT) {
    const V3 v = mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]);
    li = sload(L.radiance);
    if (L.kind == BLING_LIGHT_POINT) {                               // sample' PointLight (Light.hs:210-213)
      const V3 d = uniform_sample_sphere(ud1, ud2);
      ray = Ray{v, d, 0.f, INFINITY};
      n = d;
      return 1.f / (2.f * PI);             // uniformSpherePdf = 1 / (2 pi) as written (Montecarlo.hs:188-190)
    }
    const V3 c = mk(S.world_c[0], S.world_c[1], S.world_c[2]);        // sample' Directional (Light.hs:181-187)
    const float wr = S.world_r;
    const LC cs = coordinate_system(v);                               // coordinateSystem''
    float d1, d2;
    concentric_sample_disk(uo1, uo2, &d1, &d2);
    const V3 pd = c + vs(vs(cs.s, d1) + vs(cs.t, d2), wr);
    ray = Ray{pd + vs(v, wr), -v, 0.f, INFINITY};
    n = -v;
    return 1.f / (PI * wr * wr);
  }
  if (!(F & FT_INF) || L.kind == BLING_LIGHT_AREA) {
    const DevShape& s = gen(S.shapes[L.shape]);
    V3 ps, ns;
    if ((F & FT_SHAPES2) && s.kind >= BLING_SHAPE_DISK) shape2_sample(s, uo1, uo2, &ps, &ns);
    else if (!(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD) {
      ps = mk(lerpf(uo1, -s.params[0], s.params[0]), lerpf(uo2, -s.params[1], s.params[1]), 0.f);
      ns = mk(0.f, 0.f, -1.f);                                        // sampleShape' Quad (trap T6)
    } else {
      V3 q = uniform_sample_sphere(uo1, uo2);                          // sampleShape' Sphere
      ps = vs(q, s.params[0]); ns = q;
    }
    const V3 org = xpoint(s.o2w, ps);
    n = normalize(xnormal(s.w2o, ns));
    float dx, dy;
    concentric_sample_disk(ud1, ud2, &dx, &dy);                         // cosineSampleHemisphere' (Montecarlo.hs:152-158)
    const V3 wi = local_to_world(coordinate_system(n), mk(dx, dy, sqrtf(hmax(0.f, 1.f - dx * dx - dy * dy))));
    li = sload(L.radiance);
    ray = Ray{org, wi, 1e-3f, INFINITY};
    return INV_PI * (1.f / shape_area<F>(s)) * fabsf(dot(n, wi));
  }
  float u, v, mpdf;
  sample_c2d(L, ud1, ud2, &u, &v, &mpdf);
  li = sconst(0.f); ray = Ray{mk(0.f, 0.f, 0.f), mk(0.f, 1.f, 0.f), 0.f, 0.f}; n = mk(0.f, 1.f, 0.f);
  if (mpdf == 0.f) return 0.f;
  li = env_eval<F>(L, u, v);
  const float th = v * PI, phi = u * 2.f * PI;
  const bcr::SinCos sct = bcr::sincosf(th), scp = bcr::sincosf(phi);
  const float sint = sct.s;
  const V3 d = xvector(L.l2w, mk(sint * scp.c, sint * scp.s, sct.c));
  const V3 c = mk(S.world_c[0], S.world_c[1], S.world_c[2]);
  const float wr = S.world_r;
  const LC cs = coordinate_system(-d);
  float d1, d2;
  concentric_sample_disk(uo1, uo2, &d1, &d2);
  const V3 pd = c + vs(vs(cs.s, d1) + vs(cs.t, d2), wr);
  ray = Ray{pd + vs(d, wr), -d, 0.f, INFINITY};
  n = d;
  const float pdDir = mpdf / (2.f * PI * PI * sint), pdArea = 1.f / (PI * wr * wr);
  return sint == 0.f ? 0.f : pdDir * pdArea;
}

template <uint32_t F>
static __global__ __launch_bounds__(256) void k_sppm_photon(const DevScene* __restrict__ Sptr, SppmBufs B, uint32_t nth,
                                                     uint32_t sn, uint32_t seed, uint32_t pass) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup(S, smem);
  const uint32_t spp = sn * sn;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long rays = 0, pairs = 0, dropped = 0;
  if (gid < nth * spp) {
    const uint32_t k = gid / spp;
    const uint32_t ppk = brng::pixel_key(seed, pass, SPPM_PHOTON_PIXEL | k), pn = gid - k * spp;
    PhotonSampler ps{ppk, pn, spp, sn, 1.f / (float)spp, 1.f / (float)sn, brng::sample_key(ppk, pn)};
    const SppmGrid g = *B.grid;
    uint32_t* cnt = B.cnt + (size_t)k * B.n_stats;
    const float ul = ps.rnd1(0);
    float uo1, uo2, ud1, ud2;
    ps.rnd2(0, &uo1, &uo2);
    ps.rnd2(1, &ud1, &ud2);
    float pdf = 0.f;                                                    // sampleLightRay (Scene.hs:121-135)
    Sp li; Ray ray; V3 nl;
    if (S.num_lights > 0) {
      const int lc = S.num_lights;
      const int ln = lc == 1 ? 0 : min((int)floorf(ul * (float)lc), lc - 1);
      pdf = light_ray<F>(S, gen(S.lights[ln]), uo1, uo2, ud1, ud2, li, ray, nl);
      if (lc > 1) pdf = pdf / (float)lc;
    }
    bool alive = pdf > 0.f;
    if (alive) {
      li = sscale(li, fabsf(dot(nl, -ray.d)) / pdf);
      alive = !is_black(li);
    }
    for (int d = 0; alive && d < SPPM_PHOTON_BOUNCES; ++d) {
      const V3 wi = -ray.d;
      ++rays;
      HitRec h;
      TraceCount tc{0u, 0u, 0u, 0u};
      if (!trace<false, F>(S, L, ray, h, tc)) break;
      const float4 hv = make_float4(h.t, __uint_as_float(h.ref), h.b1, h.b2);
      DG dgg, dgs;
      float eps;
      int mat, hit_light;
      hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
      const Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs);
      const V3 p = bsdf.p, ng = bsdf.ng;
      if (has_non_specular(bsdf) && g.cnt > 0u) {                       // hashLookup (SPPM.hs:307-314)
        const V3 q = p - mk(g.lo[0], g.lo[1], g.lo[2]);
        const uint32_t b = sppm_bucket((int64_t)fabsf(q.x * g.scale), (int64_t)fabsf(q.y * g.scale),
                                       (int64_t)fabsf(q.z * g.scale), g.cnt);
        kd_lookup(B, B.bstart[b], B.bstart[b + 1], p, [&](uint32_t i, const float4& hp) {
          ++pairs;
          const float4 ho = B.hp_o[i], hd = B.hp_d[i];
          const Bsdf hb = B.hp_bsdf[i];
          const Sp f = eval_bsdf<F>(hb, -mk(hd.x, hd.y, hd.z), wi);
          const Sp l = sscale(load_sp(B.hp_f, i) * f * li, 1.f / (fabsf(dot(wi, ng)) * hp.w * PI));
          const int sx = (int)floorf(ho.w), sy = (int)floorf(hd.w);     // splatSample (Image.hs:201-221)
          if (sx >= 0 && sy >= 0 && sx < S.width && sy < S.height) {
            if (s_bad(l)) ++dropped;
            else {
              float x, y, z;
              to_xyz(l, &x, &y, &z);
              float* o = B.splat + 3 * ((size_t)sy * S.width + sx);
              atomicAdd(&o[0], x); atomicAdd(&o[1], y); atomicAdd(&o[2], z);
            }
          }
          atomicAdd(&cnt[sppm_sidx(S, ho.w, hd.w)], 1u);
        });
      }
      const float ubc = ps.rnd1(1 + d * 2);
      float ub1, ub2;
      ps.rnd2(2 + d, &ub1, &ub2);
      Sp f; V3 wo; int fl;
      const float spdf = sample_bsdf<F, true>(bsdf, wi, ubc, ub1, ub2, f, wo, fl);   // sampleAdjBsdf
      const float pcont = d > 7 ? 0.8f : 1.f;
      const Sp li2 = sscale(f * li, 1.f / pcont);
      if (spdf == 0.f || is_black(li2)) break;
      if (ps.rnd1(2 + d * 2) > pcont) break;
      ray = Ray{p, wo, eps, INFINITY};
      li = li2;
    }
  }
  const unsigned long long wr = wave_sum_u64(rays), wp = wave_sum_u64(pairs), wd = wave_sum_u64(dropped);
  if ((threadIdx.x & 63) == 0) {
    if (wr) atomicAdd(&B.ctr[1], wr);
    if (wp) atomicAdd(&B.ctr[2], wp);
    if (wd) atomicAdd(&B.ctr[3], wd);
  }
}

// ------------------------------------------------------------------ pixel statistics
// mergeStats in seed order, literally m[i] := m'[i + m[i]] (SPPM.hs:259-262; an index past the end
// reads 0), then statsUpdate (:272-291); clears the per-seed counts for the next pass
static __global__ __launch_bounds__(256) void k_sppm_stats(SppmBufs B, uint32_t nth, float alpha) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_stats) return;
  uint32_t m = 0u;
  for (uint32_t k = 0; k < nth; ++k) {
    const uint64_t j = (uint64_t)i + m;
    m = j < B.n_stats ? B.cnt[(size_t)k * B.n_stats + j] : 0u;
  }
  if (m > 0u) {
    const float r2 = B.r2[i], n = B.nacc[i], mf = (float)m;
    const float n2 = n + alpha * mf;
    const float ratio = n2 / (n + mf);
    B.r2[i] = r2 * ratio;
    B.nacc[i] = n2;
  }
}

}  // namespace bd
