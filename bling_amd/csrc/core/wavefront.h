// wavefront.h -- the per-bounce kernels of the MI355X path integrator (Integrator/Path.hs:41-87)
// and of the DirectLighting integrator (Integrator/DirectLighting.hs:22-57, k_shade_dl).
//
// One path vertex = four launches over compacted work queues (wave-aggregated appends):
//   k_shade(d)          hit reconstruction, BSDF (Material.hs), one-light MIS estimate set-up
//                       (Scene.hs:61-118): emits the BSDF-MIS ray + its candidate contribution, the
//                       light-sample shadow ray + its candidate, Russian roulette and the
//                       continuation ray (Path.hs:68-87)
//   k_trace_closest     closest-hit queries of {MIS rays of d} + {continuation rays of d+1}
//   k_trace_any         any-hit queries of the shadow rays of d
//   k_resolve(d)        L += T_d * (intl + (ls + bs)) with the visibility / MIS-hit outcomes; finalises
//                       paths that stopped at d
// Trace kernels hold no spectra and run at high occupancy; k_shade holds no traversal.  All
// per-path state is SoA in HBM; a spectrum is one 64-B record per path (4 x float4), so a lane
// touches whole cache-line halves whatever order the compacted queues visit paths in.
#pragma once
#include "dev_shade.h"
#include "dev_trace.h"

namespace bd {

// Occupancy targets (waves per SIMD) the register allocator must meet; 0 = compiler's choice.
// Build-time knobs for experiments (make variant); the defaults are the measured best.
#ifndef BLING_SHADE_WAVES
#define BLING_SHADE_WAVES 0
#endif
#ifndef BLING_RESOLVE_WAVES
#define BLING_RESOLVE_WAVES 0
#endif
// Shading kernels of the profiles with glass / substrate / bump lobes need more than 256 VGPRs
// unconstrained (k_shade of the sun-sky profile: 260, one wave per SIMD); they are held to >= 2
// waves per SIMD (<= 256 VGPRs).  A/B on MI355X, C4: 3 558 -> 5 155 Mrays/s; the other profiles keep
// the compiler's choice (cornell's 159 VGPRs at 3 waves: forcing 2 measured -6 %).
// The sun-sky profile (glass / metal / plastic spheres under the sky, no meshes) is latency bound
// (SQ wait 0.53 of its cycles at two waves); at three waves it spills 380 B per lane and still runs
// faster (A/B on one box, profiles/r02_ab_shade_waves.txt: C4 +2.8 %; the meshes profile at three
// waves: C3 -2.7 %, so it keeps the compiler's choice).
template <uint32_t F>
constexpr int shade_min_waves() {
  return BLING_SHADE_WAVES > 0 ? BLING_SHADE_WAVES
       : ((F & FT_ENV_SKY) && (F & FT_GLASS) && !(F & (FT_TRIS | FT_SUBSTRATE | FT_BUMP))) ? 3
       : ((F & (FT_GLASS | FT_SUBSTRATE | FT_BUMP)) ? 2 : 1);
}
template <uint32_t F>
constexpr int shade_max_waves() { return BLING_SHADE_WAVES > 0 ? BLING_SHADE_WAVES : 8; }
#define SHADE_OCC __attribute__((amdgpu_waves_per_eu(shade_min_waves<F>(), shade_max_waves<F>())))
#ifndef BLING_TRACE_WAVES
#define BLING_TRACE_WAVES 0    // build knob (A/B): minimum waves per SIMD of k_trace_closest, 0 = per profile
#endif
// The fractal profiles' closest-hit kernel (the paired march) sits just above the 168 VGPRs of
// three waves per SIMD; it is held to three.  The all-LDS BVH4 kernel (ALLL: small scenes, no global
// fallback) is held to eight (70 -> 64 VGPRs; A/B on C2, profiles/r02_ab_occupancy_s5.txt: closest
// 41.4 -> 40.1 ms/pass; the same floor on the meshes profile's global-fallback kernel lost 10 % on C3,
// so it applies to ALLL only).  The other kernels keep the compiler's choice.
#ifndef BLING_ALLL_WAVES
#define BLING_ALLL_WAVES 8     // build knob (A/B): the all-LDS BVH4 kernels' occupancy floor
#endif
#ifndef BLING_ANY_OCC
#define BLING_ANY_OCC 0        // build knob (A/B): 1 = k_trace_any takes the same occupancy floor
#endif
template <uint32_t F, bool ALLL>
constexpr int trace_min_waves() {
  return BLING_TRACE_WAVES > 0 ? BLING_TRACE_WAVES
       : ((F & FT_FRACTAL) ? 3 : ((ALLL && use_bvh4<F>()) ? BLING_ALLL_WAVES : 1));
}
#define TRACE_OCC __attribute__((amdgpu_waves_per_eu(trace_min_waves<F, ALLL>(), 8)))
#if BLING_ANY_OCC
#define ANY_OCC TRACE_OCC
#else
#define ANY_OCC
#endif
#if BLING_RESOLVE_WAVES > 0
#define RESOLVE_OCC __attribute__((amdgpu_waves_per_eu(BLING_RESOLVE_WAVES, BLING_RESOLVE_WAVES)))
#else
#define RESOLVE_OCC
#endif

#ifndef BLING_FUSED
#define BLING_FUSED 1   // build knob for A/B: 0 = separate k_resolve and k_shade launches (core_wave.h)
#endif

constexpr uint32_t FL_ALIVE = 1u << 31, FL_SPEC = 1u << 30;
constexpr uint32_t VF_SH = 1u, VF_MIS = 2u, VF_TERM = 4u;
constexpr uint32_t ENTRY_CONT = 0u, ENTRY_MIS = 1u;

enum QueueId : int { Q_SHADE0 = 0, Q_SHADE1 = 1, Q_CLOSEST = 2, Q_ANY = 3, Q_RESOLVE = 4, Q_N = 5 };

struct WaveState {
  float4* org;        // p.xyz, eps : origin + tmin of the MIS ray (= the continuation's for Path)
  float4* corg;       // continuation (camera at d = 0) ray origin + tmin: aliases org for Path;
                      // its own array for DirectLighting, whose popped sibling rays start elsewhere
  float4* dir;        // continuation (camera at d = 0) ray direction
  float4* mis_dir;    // BSDF-MIS ray direction
  float4* sh_o;       // shadow ray o.xyz, tmin
  float4* sh_d;       // shadow ray d.xyz, tmax
  float4* hit;        // closest hit of the continuation ray: t, ref, b1, b2
  float2* mis_hit;    // closest hit of the MIS ray: t, ref
  uint32_t* occ;      // shadow ray occluded (1) / visible (0)
  float4* T;          // [cap][4] throughput of the vertex being shaded
  float4* Tn;         // [cap][4] throughput after the continuation sample
  float4* L;          // [cap][4] radiance so far
  float4* lsc;        // [cap][4] light-sampling candidate  sc (w / pdf) (f * Li)
  float4* bsc;        // [cap][4] BSDF-sampling f (weight in mis_dir.w)
  float4* fac;        // factored profiles: (s1 of the BSDF-MIS f, s1, s2 of the light-sample f, w / pdf)
  uint32_t* rtex;     // factored profiles: byte offset of the lobe's spectrum in S.textures (~0u = white)
  uint32_t* flags;    // FL_ALIVE | FL_SPEC | depth
  uint32_t* vflags;   // VF_* | (intl light + 1) << 8 | light index << 16
  uint32_t* pixel;    // sample-extent pixel index
  uint32_t* nidx;     // sample number within the pixel
  float2* img;        // imageX, imageY
  float4* result;     // X, Y, Z, 1 (or 0 = dropped)
  float4* Lfull;      // [cap][4] final spectrum (parity hook only, may be NULL)
  uint32_t* queue[Q_N];
  uint32_t* qcount;   // Q_N counters
  uint8_t* qflag;     // per shade-queue entry: QF_* bits written by k_shade, compacted by k_compact_*
  uint32_t* blk;      // compaction: per-block counts / offsets [nb][4], then totals [4]
  // DirectLighting only (NULL for Path): the pending specular-transmission sibling of level j
  // (1 <= j < maxDepth) of each sample's depth-first walk, slot j at [j * cap + i]
  float4* dl_org;     // p.xyz, eps
  float4* dl_dir;     // wi
  float4* dl_T;       // [levels * cap][4] weight of the pending ray
  uint32_t* dl_mask;  // bit j set = slot j pending
  float* dbg;         // per-vertex debug records (bling_sample_li_vertices; BLING_DEBUG_VERTEX builds only)
  uint32_t cap;
};

// Per-vertex debug records (BLING_DEBUG_VERTEX builds, `make variant V=dbg`): BLING_DV_FIELDS floats
// per path vertex, field map in include/bling.h; the oracle writes the same fields
// (oracle_sample_li_vertices), so the first differing field names the first diverging operation.
#ifndef BLING_DEBUG_VERTEX
#define BLING_DEBUG_VERTEX 0
#endif
#if BLING_DEBUG_VERTEX
#define DVREC(W, i, d, f, v) \
  do { if ((W).dbg && (d) >= 0 && (d) < BLING_DV_DEPTHS) (W).dbg[((size_t)(i) * BLING_DV_DEPTHS + (d)) * BLING_DV_FIELDS + (f)] = (v); } while (0)
#else
#define DVREC(W, i, d, f, v) do { } while (0)
#endif
#define DVREC3(W, i, d, f, v) do { DVREC(W, i, d, f, (v).x); DVREC(W, i, d, (f) + 1, (v).y); DVREC(W, i, d, (f) + 2, (v).z); } while (0)

// Queue membership bits emitted by k_shade for entry e of its input queue.
constexpr uint32_t QF_RESOLVE = 1u, QF_ANY = 2u, QF_MIS = 4u, QF_CONT = 8u;
constexpr uint32_t COMPACT_CHUNK = 4096;   // shade-queue entries per compaction block (4 waves x 1024)

struct Counters {
  unsigned long long cam, cont, mis, shadow, dropped, node_visits, tri_tests, shape_tests, vertices, march_ticks;
  unsigned long long c_node_visits, c_tri_tests, c_shape_tests, c_march_ticks;   // closest-hit kernel only
};

// wave-aggregated queue append; every active lane calls it (pred may be false)
DEV uint32_t wave_append(uint32_t* counter, bool pred) {
  unsigned long long mask = __ballot(pred);
  if (!pred) return 0u;
  uint32_t lane = threadIdx.x & 63u;
  uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
  uint32_t base = 0u;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
  base = __shfl(base, (int)leader, 64);
  return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

// Spectrum records.  Record layout ([n][4] float4: one 64-B record per index) for the SPPM hit
// points and the parity hook; path-state spectra use the tiled layout below.
DEV void store_sp(float4* dst, uint32_t i, const Sp& s) {
  float4* p = dst + 4 * (size_t)i;
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = make_float4(s.v[4 * q], s.v[4 * q + 1], s.v[4 * q + 2], s.v[4 * q + 3]);
}
DEV Sp load_sp(const float4* src, uint32_t i) {
  const float4* p = src + 4 * (size_t)i;
  Sp s;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = p[q];
    s.v[4 * q] = v.x; s.v[4 * q + 1] = v.y; s.v[4 * q + 2] = v.z; s.v[4 * q + 3] = v.w;
  }
  return s;
}

// Path-state spectra (T, Tn, L, lsc, bsc, dl_T).  Default: the record layout (one 64-B record per
// path).  BLING_SP_TILED=1 stores tiles of 64 paths instead (quarter q of path i at float4
// ((i / 64) * 4 + q) * 64 + i % 64: one load instruction of a wave over 64 consecutive ids reads
// 1 KiB contiguous), which measured slower because the compacted queues are sparse in path ids, so
// a tile line is mostly unused (A/B on MI355X, profiles/r02_ab_bvh4_sp.txt: C2 6 083 tiled vs 6 867
// records, C3 4 070 vs 4 203, C4 5 608 vs 5 738 Mrays/s).
#ifndef BLING_SP_TILED
#define BLING_SP_TILED 0
#endif
DEV size_t sp_at(uint32_t i, int q) {
#if BLING_SP_TILED
  return ((size_t)(i & ~63u) << 2) + (size_t)q * 64u + (i & 63u);
#else
  return 4 * (size_t)i + (size_t)q;
#endif
}
DEV void store_ps(float4* dst, uint32_t i, const Sp& s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[sp_at(i, q)] = make_float4(s.v[4 * q], s.v[4 * q + 1], s.v[4 * q + 2], s.v[4 * q + 3]);
}
DEV Sp load_ps(const float4* src, uint32_t i) {
  Sp s;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = src[sp_at(i, q)];
    s.v[4 * q] = v.x; s.v[4 * q + 1] = v.y; s.v[4 * q + 2] = v.z; s.v[4 * q + 3] = v.w;
  }
  return s;
}

DEV void finalize(const WaveState& W, uint32_t i, const Sp& L, unsigned long long& dropped) {
  W.flags[i] = 0u;
  if (W.Lfull) store_sp(W.Lfull, i, L);
  if (s_bad(L)) { W.result[i] = make_float4(0.f, 0.f, 0.f, 0.f); dropped++; return; }   // Image.hs:253-256
  float x, y, z;
  to_xyz(L, &x, &y, &z);
  W.result[i] = make_float4(x, y, z, 1.f);
}

// Traversal work counters (node fetches, triangle / shape tests) for the roofline freeze tool; the
// production launch compiles them out (STATS = false).  Ray counts come from the queue lengths
// (k_stage), never from per-wave atomics.
template <bool STATS, bool CLOSEST = false>
DEV void flush_trace_stats(Counters* C, const TraceCount& tc) {
  if (!STATS) return;
  unsigned long long nv = wave_sum_u64((unsigned long long)tc.nodes);
  unsigned long long nt = wave_sum_u64((unsigned long long)tc.tris);
  unsigned long long ns = wave_sum_u64((unsigned long long)tc.shapes);
  unsigned long long nk = wave_sum_u64((unsigned long long)tc.ticks);
  if ((threadIdx.x & 63) == 0) {
    if (nv) atomicAdd(&C->node_visits, nv);
    if (nt) atomicAdd(&C->tri_tests, nt);
    if (ns) atomicAdd(&C->shape_tests, ns);
    if (nk) atomicAdd(&C->march_ticks, nk);
    if (CLOSEST) {                         // the roofline's work basis: closest-hit queries only
      if (nv) atomicAdd(&C->c_node_visits, nv);
      if (nt) atomicAdd(&C->c_tri_tests, nt);
      if (ns) atomicAdd(&C->c_shape_tests, ns);
      if (nk) atomicAdd(&C->c_march_ticks, nk);
    }
  }
}
DEV void flush_dropped(Counters* C, unsigned long long drop) {
  if (__ballot(drop != 0ull) == 0ull) return;
  drop = wave_sum_u64(drop);
  if ((threadIdx.x & 63) == 0) atomicAdd(&C->dropped, drop);
}

// ------------------------------------------------------------------ closest / any traversal
// Both traversal kernels are persistent over their queue: lane-level refill (a lane whose ray is
// done writes its result and starts the next queue entry at once, Traversal::step).
//
// Refill order is wave-coherent: wave w owns the 64-entry queue chunks w, w + nw, w + 2 nw, ...
// and hands the next consecutive entries of its current chunk to its free lanes (rank among the
// free lanes).  The ray records a wave loads (and the hit records it stores) therefore stay inside
// a few cache lines per refill.  A per-lane grid stride (entry e, e + grid, ...) scatters every
// refilled lane to its own line: PMC FETCH_SIZE measured 275 B per closest ray for the 36 B the
// ray stream needs.
constexpr uint32_t FEED_CHUNK = 64;
// Traversal steps per refill check: three for the global-fallback kernels (the refill's ballots and
// queue loads amortised over several steps: C3 closest-hit 160 / 149 / 138 ms per pass with one /
// two / three), one for the all-LDS kernel, whose short walks lose more to lanes idling after an
// early finish (C2 37.7 -> 43.2 with two; profiles/r02_ab_trace_steps_s5.txt).  Build knob
// BLING_TRACE_STEPS forces a count for A/B.
#ifndef BLING_TRACE_STEPS
#define BLING_TRACE_STEPS 0
#endif
template <bool ALLL>
constexpr int trace_steps() { return BLING_TRACE_STEPS > 0 ? BLING_TRACE_STEPS : (ALLL ? 1 : 3); }

struct WaveFeed {
  uint32_t chunk, cur, end, n, nw;
  DEV void init(uint32_t n_) {
    n = n_;
    nw = gridDim.x * (blockDim.x >> 6);
    chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    open();
  }
  DEV void open() {
    const uint64_t c0 = (uint64_t)chunk * FEED_CHUNK;
    cur = c0 < n ? (uint32_t)c0 : n;
    end = (uint32_t)((uint64_t)cur + FEED_CHUNK < n ? cur + FEED_CHUNK : n);
  }
  // Free lanes (live == false) receive consecutive entries; returns true for a lane that got entry *e.
  DEV bool take(bool live, uint32_t* e) {
    bool got = false;
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const bool want = !live && !got;
      const unsigned long long m = __ballot(want);
      if (m == 0ull || cur >= end) break;
      const uint32_t avail = end - cur;
      const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (want && rank < avail) { *e = cur + rank; got = true; }
      const uint32_t used = min((uint32_t)__popcll(m), avail);
      cur += used;
      if (cur == end) { chunk += nw; open(); }
    }
    return got;
  }
};
template <uint32_t F, bool STATS, bool ALLL>
static __global__ __launch_bounds__(256) TRACE_OCC void k_trace_closest(const DevScene* __restrict__ Sptr, WaveState W,
                                                                 Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup<use_bvh4<F>()>(S, smem);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_CLOSEST];
  const uint32_t* q = W.queue[Q_CLOSEST];
  WaveFeed feed;
  feed.init(n);
  TraceCount tc{0u, 0u, 0u, 0u};
  QTraversal<false, F, ALLL> tv;
  bool live = false;
  uint32_t ent = 0u, e = 0u;
  for (;;) {
    if (feed.take(live, &e)) {
      ent = q[e];
      const uint32_t i = ent >> 1;
      const float4 o = ((ent & 1u) == ENTRY_CONT ? W.corg : W.org)[i];
      const float4 d = (ent & 1u) == ENTRY_CONT ? W.dir[i] : W.mis_dir[i];
      tv.init(Ray{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, INFINITY});
      live = true;
    }
    if (__ballot(live) == 0ull) break;
#pragma unroll
    for (int u = 0; u < trace_steps<ALLL>(); ++u) {
      if (live && tv.step(S, L, tc)) {
        const uint32_t i = ent >> 1;
        if ((ent & 1u) == ENTRY_CONT) W.hit[i] = make_float4(tv.h.t, __uint_as_float(tv.h.ref), tv.h.b1, tv.h.b2);
        else W.mis_hit[i] = make_float2(tv.h.t, __uint_as_float(tv.h.ref));
        live = false;
      }
    }
  }
  flush_trace_stats<STATS, true>(C, tc);
}

template <uint32_t F, bool STATS, bool ALLL>
static __global__ __launch_bounds__(256) ANY_OCC void k_trace_any(const DevScene* __restrict__ Sptr, WaveState W,
                                                   Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup<use_bvh4<F>()>(S, smem);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_ANY];
  const uint32_t* q = W.queue[Q_ANY];
  WaveFeed feed;
  feed.init(n);
  TraceCount tc{0u, 0u, 0u, 0u};
  QTraversal<true, F, ALLL> tv;
  bool live = false;
  uint32_t i = 0u, e = 0u;
  for (;;) {
    if (feed.take(live, &e)) {
      i = q[e];
      const float4 o = W.sh_o[i], d = W.sh_d[i];
      tv.init(Ray{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, d.w});
      live = true;
    }
    if (__ballot(live) == 0ull) break;
#pragma unroll
    for (int u = 0; u < trace_steps<ALLL>(); ++u) {
      if (live && tv.step(S, L, tc)) {
        W.occ[i] = tv.h.ref != REF_NONE ? 1u : 0u;
        live = false;
      }
    }
  }
  flush_trace_stats<STATS>(C, tc);
}

// Wave-coherent variants for small scenes (DevScene::pkt_n > 0, dev_trace.h packet_walk): wave w
// takes the 64-entry queue chunks w, w + nw, ... and walks the threaded BVH once per chunk with all
// of its rays.  Same queue, ray and hit records as the per-lane kernels above.
template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_closest_pkt(const DevScene* __restrict__ Sptr, WaveState W,
                                                                 Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_CLOSEST];
  const uint32_t* q = W.queue[Q_CLOSEST];
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk * 64u < n; chunk += nw) {
    const uint32_t e = chunk * 64u + (threadIdx.x & 63u);
    const bool live = e < n;
    const uint32_t ent = live ? q[e] : 0u;
    const uint32_t i = ent >> 1;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f), d = make_float4(0.f, 0.f, 1.f, 0.f);
    if (live) {
      o = ((ent & 1u) == ENTRY_CONT ? W.corg : W.org)[i];
      d = (ent & 1u) == ENTRY_CONT ? W.dir[i] : W.mis_dir[i];
    }
    const Ray r{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, INFINITY};
    HitRec h{INFINITY, REF_NONE, 0.f, 0.f};
    packet_walk<false, F>(S, r, live, h, tc);
    if (live) {
      if ((ent & 1u) == ENTRY_CONT) W.hit[i] = make_float4(h.t, __uint_as_float(h.ref), h.b1, h.b2);
      else W.mis_hit[i] = make_float2(h.t, __uint_as_float(h.ref));
    }
  }
  flush_trace_stats<STATS, true>(C, tc);
}

template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_any_pkt(const DevScene* __restrict__ Sptr, WaveState W,
                                                             Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_ANY];
  const uint32_t* q = W.queue[Q_ANY];
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk * 64u < n; chunk += nw) {
    const uint32_t e = chunk * 64u + (threadIdx.x & 63u);
    const bool live = e < n;
    const uint32_t i = live ? q[e] : 0u;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f), d = make_float4(0.f, 0.f, 1.f, 0.f);
    if (live) { o = W.sh_o[i]; d = W.sh_d[i]; }
    const Ray r{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, d.w};
    HitRec h{d.w, REF_NONE, 0.f, 0.f};
    packet_walk<true, F>(S, r, live, h, tc);
    if (live) W.occ[i] = h.ref != REF_NONE ? 1u : 0u;
  }
  flush_trace_stats<STATS>(C, tc);
}

// ------------------------------------------------------------------ shading
// Factored candidates.  In a profile whose materials are all matte (one Lambertian or Oren-Nayar
// lobe over a texture spectrum r) and whose lights are all area lights (Li = the light's constant
// radiance), the two candidate spectra of a vertex are
//   light sample:  lsc = ((0 + (r * s1) * s2) * Le) * (w / pdf)     (evalBsdf, sampleLightMis)
//   BSDF sample:   bsc = r * s1                                      (sampleBsdf, sampleBsdfMis)
// so k_shade stores the four scalars and the texture (20 B) instead of two 64-B spectra, and
// k_resolve expands them with the same operations in the same order: bit-identical candidates,
// 216 fewer bytes of HBM traffic per path vertex.
#ifndef BLING_FACTORED
#define BLING_FACTORED 1   // build knob for A/B (make variant DEFS=-DBLING_FACTORED=0)
#endif
template <uint32_t F>
constexpr bool factored() { return BLING_FACTORED && (F & ~(FT_MATTE | FT_AREA | FT_TRIS)) == 0; }

// sampleOneLight set-up (Scene.hs:61-118): picks the light with 1D dimension dl1, emits the BSDF-MIS
// ray (1D db1 + 2D db2) and the light-sample shadow ray (2D dl2) with their candidate contributions;
// k_resolve completes the estimate once both rays are traced.
template <uint32_t F>
DEV void direct_setup(const DevScene& S, const WaveState& W, uint32_t i, const SampleKey& k, const Bsdf& bsdf, V3 wo,
                      V3 p, float eps, int dl1, int dl2, int db1, int db2, uint32_t& vf, bool& app_mis, bool& app_sh,
                      int dvd = -1) {
  int lc = S.num_lights;
  if (lc > 0) {
    float lNumU = rnd1(S, k, dl1);
    int ln = lc == 1 ? 0 : min((int)floorf(lNumU * (float)lc), lc - 1);
    const bling_light& Lt = gen(S.lights[ln]);
    vf |= (uint32_t)ln << 16;
    if constexpr (factored<F>()) {
      const float* r = bsdf.n ? bsdf.b[0].r : nullptr;
      float fm = 0.f, fs1 = 0.f, fs2 = 0.f, wpdf = 0.f;
      {                                                              // sampleBsdfMis (Scene.hs:71-82)
        float lb1, lb2; rnd2(S, k, db2, &lb1, &lb2);
        float s; V3 bwi;
        const float bpdf = sample_bsdf_diffuse1<F>(bsdf, wo, lb1, lb2, s, bwi);
        DVREC3(W, i, dvd, 18, bwi); DVREC(W, i, dvd, 21, bpdf);
        if (!(bpdf == 0.f) && !is_black(diffuse1_f(r, s))) {
          const float lpdf = light_pdf<F>(S, Lt, p, bwi);
          W.mis_dir[i] = make_float4(bwi.x, bwi.y, bwi.z, power_heuristic(bpdf, lpdf));
          fm = s;
          vf |= VF_MIS;
          app_mis = true;
        }
      }
      {                                                              // sampleLightMis (Scene.hs:61-69)
        float ld1, ld2; rnd2(S, k, dl2, &ld1, &ld2);
        LightSample smp = light_sample<F>(S, Lt, p, eps, ld1, ld2);
        DVREC3(W, i, dvd, 14, smp.wi); DVREC(W, i, dvd, 17, smp.pdf);
        float s1, s2;
        if (!(smp.pdf == 0.f) && !is_black(smp.li) && eval_bsdf_diffuse1<F>(bsdf, wo, smp.wi, s1, s2) &&
            !is_black(diffuse1_e(r, s1, s2))) {
          const float w = power_heuristic(smp.pdf, bsdf_pdf<F>(bsdf, wo, smp.wi));
          wpdf = w / smp.pdf; fs1 = s1; fs2 = s2;
          W.sh_o[i] = make_float4(smp.ray.o.x, smp.ray.o.y, smp.ray.o.z, smp.ray.tmin);
          W.sh_d[i] = make_float4(smp.ray.d.x, smp.ray.d.y, smp.ray.d.z, smp.ray.tmax);
          vf |= VF_SH;
          app_sh = true;
        }
      }
      if (app_mis || app_sh) {
        W.fac[i] = make_float4(fm, fs1, fs2, wpdf);
        W.rtex[i] = r ? (uint32_t)((const char*)r - (const char*)gen(S.textures)) : ~0u;
      }
      return;
    }
    // BSDF half of estimateDirect: sampleBsdfMis (Scene.hs:71-82)
    {
      float lBc = rnd1(S, k, db1);
      float lb1, lb2; rnd2(S, k, db2, &lb1, &lb2);
      Sp bf; V3 bwi; int bfl;
      float bpdf = sample_bsdf<F>(bsdf, wo, lBc, lb1, lb2, bf, bwi, bfl);
      DVREC3(W, i, dvd, 18, bwi); DVREC(W, i, dvd, 21, bpdf);
      if (!(bpdf == 0.f) && !is_black(bf)) {
        float lpdf = light_pdf<F>(S, Lt, p, bwi);
        float w = power_heuristic(bpdf, lpdf);
        // f and w are kept apart: k_resolve forms sc w (f * Le) in the reference's order once
        // the MIS ray's hit is known
        store_ps(W.bsc, i, bf);
        W.mis_dir[i] = make_float4(bwi.x, bwi.y, bwi.z, w);
        vf |= VF_MIS;
        app_mis = true;
      }
    }
    // light half: sampleLightMis (Scene.hs:61-69)
    {
      float ld1, ld2; rnd2(S, k, dl2, &ld1, &ld2);
      LightSample smp = light_sample<F>(S, Lt, p, eps, ld1, ld2);
      DVREC3(W, i, dvd, 14, smp.wi); DVREC(W, i, dvd, 17, smp.pdf);
      if (!(smp.pdf == 0.f) && !is_black(smp.li)) {
        Sp f = eval_bsdf<F>(bsdf, wo, smp.wi);
        if (!is_black(f)) {
          float w = power_heuristic(smp.pdf, bsdf_pdf<F>(bsdf, wo, smp.wi));
          store_ps(W.lsc, i, sscale(f * smp.li, w / smp.pdf));
          W.sh_o[i] = make_float4(smp.ray.o.x, smp.ray.o.y, smp.ray.o.z, smp.ray.tmin);
          W.sh_d[i] = make_float4(smp.ray.d.x, smp.ray.d.y, smp.ray.d.z, smp.ray.tmax);
          vf |= VF_SH;
          app_sh = true;
        }
      }
    }
  }
}

// Hit reconstruction (mkIntersection + shadingGeometry, Primitive.hs:57-65) from a closest-hit
// record {t, ref, b1, b2}: geometric and shading DG, the ray epsilon, the material and the area
// light of a hit shape (-1 if none).
template <uint32_t F>
DEV void hit_geometry(const DevScene& S, const Ray& ray, const float4 hv, DG& dgg, DG& dgs, float& eps, int& mat,
                      int& hit_light) {
  const uint32_t ref = __float_as_uint(hv.y);
  uint32_t kind = ref >> 30, idx = ref & 0x3FFFFFFFu;
  hit_light = -1;
  if (kind == REF_TRI) {
    dgg = tri_dg(S, idx, ray, hv.x, hv.z, hv.w);
    eps = 1e-3f * hv.x;
    mat = S.tri_material[idx];
  } else if (!(F & FT_FRACTAL) || kind == REF_SHAPE) {
    const DevShape& sh = gen(S.shapes[idx]);
    dgg = shape_dg<F>(sh, ray, hv.x);
    eps = 5e-4f * hv.x;
    mat = sh.material;
    hit_light = sh.light;
  } else {
    // the march's last point and gradient (mandel_march): p = ray_at(rn, t) on the normalised
    // ray, n = normalize(grad) from mandelDist there -- not a second march
    const float l = len(ray.d);
    const V3 pp = ray.o + vs(vs(ray.d, 1.f / l), hv.x);
    V3 nn;
    if (S.fractal.kind == BLING_FRACTAL_JULIA) {
      nn = julia_normal(S.fractal, pp);                             // normalJulia (Fractal.hs:203-223)
    } else {
      V3 gg;
      mandel_dist(S.fractal.order, S.fractal.iterations, S.fractal.epsilon, pp, &gg);
      nn = normalize(gg);
    }
    LC c = coordinate_system(nn);                                   // mkDg' (DG.hs:53-56)
    dgg.p = pp; dgg.n = nn; dgg.u = 0.f; dgg.v = 0.f; dgg.dpdu = c.s; dgg.dpdv = c.t;
    eps = S.fractal.epsilon * 2.f;
    mat = S.fractal.material;
  }
  dgs = dgg;
  if ((F & FT_TRI_NORMALS) && kind == REF_TRI && S.tri_normals && S.tri_has_n[idx]) {       // triangleShadingGeometry (TriangleMesh.hs:122-134)
    const float* nn = gen(S.tri_normals) + 9 * idx;
    float b1 = hv.z, b2 = hv.w, b0 = 1.f - b1 - b2;
    V3 nsp = sm(b0, mk(nn[0], nn[1], nn[2])) + sm(b1, mk(nn[3], nn[4], nn[5])) + sm(b2, mk(nn[6], nn[7], nn[8]));
    V3 ns = normalize(nsp);
    V3 ssp = normalize(dgg.dpdu);
    V3 tsp = cross(ssp, ns);
    if (sqlen(tsp) > 0.f) { dgs.dpdu = cross(normalize(tsp), ns); dgs.dpdv = normalize(tsp); }
    else { LC c = coordinate_system(ns); dgs.dpdu = c.s; dgs.dpdv = c.t; }
    dgs.n = ns;
  }
}

// L + T (intl + (ls + bs)) of the vertex whose shadow / BSDF-MIS rays were just traced
// (sampleOneLight's completion, Scene.hs:61-118, and Path.hs:73-79's accumulation), in the
// reference's operation order.  T is the vertex's throughput (Tv).
template <uint32_t F>
// first: the vertex is the camera path's first (depth 0), whose L = 0 and T = 1 are implicit (the
// Path integrator's raygen stores neither; see k_raygen).
DEV Sp resolve_L(const DevScene& S, const WaveState& W, uint32_t i, uint32_t vf, const float4* Tv, bool first = false,
                 int dvd = -1) {
  int lc = S.num_lights;
  Sp ld = sconst(0.f);
  if (lc > 0) {
    Sp ls = sconst(0.f), bs = sconst(0.f);
    const int ln = (int)(vf >> 16);
    float4 fc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* rf = nullptr;                                        // factored: the lobe's spectrum
    if constexpr (factored<F>()) {
      if (vf & (VF_SH | VF_MIS)) {
        fc = W.fac[i];
        const uint32_t off = W.rtex[i];
        rf = off == ~0u ? nullptr : (const float*)((const char*)gen(S.textures) + off);
      }
      if ((vf & VF_SH) && W.occ[i] == 0u)
        ls = sscale(diffuse1_e(rf, fc.y, fc.z) * sload(gen(S.lights[ln]).radiance), fc.w);
    } else {
      if ((vf & VF_SH) && W.occ[i] == 0u) ls = load_ps(W.lsc, i);
    }
    if (vf & VF_SH) DVREC(W, i, dvd, 28, W.occ[i] ? 1.f : 0.f);
    if (vf & VF_MIS) {                                                // sampleBsdfMis (Scene.hs:71-82)
      const bling_light& Lt = gen(S.lights[ln]);
      float2 mh = W.mis_hit[i];
      uint32_t ref = __float_as_uint(mh.y);
      DVREC(W, i, dvd, 29, ref == REF_NONE ? INFINITY : mh.x);
      float4 d = W.mis_dir[i];
      V3 wi = mk(d.x, d.y, d.z);
      if (ref == REF_NONE) {
        const Sp bf = factored<F>() ? diffuse1_f(rf, fc.x) : load_ps(W.bsc, i);
        bs = sscale(bf * light_le<F>(Lt, wi), d.w);                  // le l ray
      } else if ((ref >> 30) == REF_SHAPE) {
        const DevShape& hs = gen(S.shapes[ref & 0x3FFFFFFFu]);
        if (hs.light == ln) {                                         // l' == l (Light.hs:48-50)
          float4 o = W.org[i];
          DG dg = shape_dg<F>(hs, Ray{mk(o.x, o.y, o.z), wi, o.w, INFINITY}, mh.x);
          Sp le = dot(dg.n, -wi) > 0.f ? sload(gen(S.lights[ln]).radiance) : sconst(0.f);   // intLe (-wi): trap T6
          const Sp bf = factored<F>() ? diffuse1_f(rf, fc.x) : load_ps(W.bsc, i);
          bs = sscale(bf * le, d.w);
        }
      }
    }
    ld = ls + bs;
    if (lc > 1) ld = sscale(ld, (float)lc);
  }
  int il = (int)((vf >> 8) & 0xFFu) - 1;
  Sp lhere = (il >= 0 ? sload(gen(S.lights[il]).radiance) : sconst(0.f)) + ld;
  const Sp L0 = first ? sconst(0.f) : load_ps(W.L, i);
  const Sp T0 = first ? sconst(1.f) : load_ps(Tv, i);
#if BLING_DEBUG_VERTEX
  {
    const Sp Lr = L0 + T0 * lhere;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < 16; ++q) { a += lhere.v[q]; b += Lr.v[q]; }
    DVREC(W, i, dvd, 30, a); DVREC(W, i, dvd, 31, b);
  }
#endif
  return L0 + T0 * lhere;
}

// Vertex d of path i (Path.hs:68-87 with sampleOneLight's set-up) once its continuation ray hit
// something below maxDepth: hit reconstruction, BSDF, the one-light estimate's two rays and
// candidates, Russian roulette and the continuation (throughput Tcur -> Tnext).  Returns the
// queue-membership bits of the vertex (QF_*).
#if !defined(BLING_SHADE_EARLY_T)
#define BLING_SHADE_EARLY_T 1
#endif
template <uint32_t F>
constexpr bool shade_early_t() {
  // throughput loaded with the hit record (A/B +1 % on C2); the sun-sky profile, which spills,
  // loads it after the light sample instead (+2 % on C4, profiles/r02_ab_shade_s5.txt)
  return BLING_SHADE_EARLY_T && !((F & FT_ENV_SKY) && (F & FT_GLASS) && !(F & (FT_TRIS | FT_SUBSTRATE | FT_BUMP)));
}
template <uint32_t F>
DEV uint32_t shade_vertex(const DevScene& S, const WaveState& W, uint32_t i, int depth, uint32_t seed, uint32_t pass,
                          const float4* Tcur, float4* Tnext, uint32_t fl, float4 hv, const Ray& ray,
                          uint32_t pix, uint32_t nid) {
  const bool spec = (fl & FL_SPEC) != 0;
  bool app_sh = false, app_mis = false, app_cont = false;
  SampleKey k = sample_key(seed, pass, pix, nid);
  Sp T;
  if constexpr (shade_early_t<F>()) T = depth == 0 ? sconst(1.f) : load_ps(Tcur, i);   // issued before any store of this vertex
  DG dgg, dgs;
  float eps;
  int mat, hit_light;
  hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
  DVREC3(W, i, depth, 0, ray.o); DVREC3(W, i, depth, 3, ray.d); DVREC(W, i, depth, 6, hv.x);
  DVREC3(W, i, depth, 10, dgg.n); DVREC(W, i, depth, 13, eps);
  int intl_light = (spec && hit_light >= 0 && dot(dgg.n, ray.d) > 0.f) ? hit_light : -1;   // intLe rd (trap T6)
  float ttmp[(F & FT_PROCTEX) ? 32 : 1];  // computed spectra of the BSDF (FT_PROCTEX profiles)
  Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs, ttmp);
  V3 wo = -ray.d;
  V3 p = bsdf.p;
  DVREC3(W, i, depth, 7, p);
  uint32_t vf = ((uint32_t)(intl_light + 1) & 0xFFu) << 8;
  direct_setup<F>(S, W, i, k, bsdf, wo, p, eps, 1 + 4 * depth, 1 + 3 * depth, 2 + 4 * depth, 2 + 3 * depth, vf,
                  app_mis, app_sh, depth);
  // Russian roulette + continuation (Path.hs:68-87)
  if constexpr (!shade_early_t<F>()) T = depth == 0 ? sconst(1.f) : load_ps(Tcur, i);
  float pc = depth <= 7 ? 1.f : hmin(0.75f, sY(T));
  float x = rnd1(S, k, 3 + 4 * depth);
  DVREC(W, i, depth, 26, pc); DVREC(W, i, depth, 27, x);
  bool cont = !(x > pc);
  if (cont) {
    float uc = rnd1(S, k, 0 + 4 * depth);
    float ud1, ud2; rnd2(S, k, 0 + 3 * depth, &ud1, &ud2);
    Sp cf; V3 cwi; int cfl;
    float cpdf = sample_bsdf<F>(bsdf, wo, uc, ud1, ud2, cf, cwi, cfl);
    DVREC3(W, i, depth, 22, cwi); DVREC(W, i, depth, 25, cpdf);
    cont = !(cpdf == 0.f || is_black(cf));
    if (cont) {
      store_ps(Tnext, i, sscale(cf * T, 1.f / pc));
      W.dir[i] = make_float4(cwi.x, cwi.y, cwi.z, 0.f);
      W.flags[i] = FL_ALIVE | (((cfl & F_SPEC) == F_SPEC) ? FL_SPEC : 0u) | (uint32_t)(depth + 1);
      app_cont = true;
    }
  }
  if (!cont) vf |= VF_TERM;
  W.org[i] = make_float4(p.x, p.y, p.z, eps);
  W.vflags[i] = vf;
  return QF_RESOLVE | (app_sh ? QF_ANY : 0u) | (app_mis ? QF_MIS : 0u) | (app_cont ? QF_CONT : 0u);
}

// A path whose continuation ray of depth d missed, or that reached maxDepth: Le of the escaped ray
// after a specular bounce (Path.hs:80), then the sample is done (Path.hs:83, 87).
template <uint32_t F>
DEV void shade_end(const DevScene& S, const WaveState& W, uint32_t i, const float4* Tcur, bool spec_miss, V3 rd, Sp L,
                   unsigned long long& n_drop, bool first) {
  if (spec_miss) {
    Sp T = first ? sconst(1.f) : load_ps(Tcur, i);
    Sp sum = sconst(0.f);
    for (int l = 0; l < S.num_lights; ++l) sum = sum + light_le<F>(gen(S.lights[l]), rd);
    L = L + T * sum;
  }
  finalize(W, i, L, n_drop);
}

// Path vertex d over a queue of paths.  FUSED = false: the queue holds the paths alive at d (the
// camera paths at d = 0); T is their throughput, the continuation's goes to Tn.  FUSED = true
// (d >= 1): the queue holds every path that had a vertex at d - 1 (k_compact's resolve list), and
// the kernel first resolves that vertex (resolve_L with Tprev = T), then -- unless the path stopped
// there -- shades vertex d with the resolved L (Tcur = Tn; the continuation's throughput goes to T,
// whose slot of path i only this path's thread reads).  One launch instead of k_resolve + k_shade:
// the two kernels' independent path loads are in flight together.  Per path, every operation and
// its order is unchanged.
//
// Wave compaction (BLING_SHADE_COMPACT): a wave takes 64 consecutive queue entries, resolves them
// and ends every path that stops here (terminated at d - 1, missed, or at maxDepth) in place; the
// paths that get a vertex at d go into a per-wave ring of 128 (path, entry) pairs in LDS, and the
// wave shades 64 of them at once whenever the ring holds 64.  Escaping / terminating paths no
// longer idle the lanes of the shading code (C4 measured 0.30 VALU lane utilisation in the fused
// shade without it).  The shading order of paths changes, their arithmetic does not; qflag stays
// indexed by queue entry, so the compacted queues keep their order.
#ifndef BLING_SHADE_COMPACT
#define BLING_SHADE_COMPACT 1
#endif
#ifndef BLING_SHADE_DUAL
#define BLING_SHADE_DUAL 0   // build knob (A/B): two queue chunks per wave iteration, both resolves' loads in flight
#endif
constexpr uint32_t SHADE_RING = BLING_SHADE_DUAL ? 256 : 128;
// BLING_SHADE_HOIST: the path's flags and hit record are loaded with the resolve loads and handed to
// the shading lane through the ring (1: +0.8 % C2, +2.2 % C4, profiles/r02_ab_shade_hoist_s5.txt);
// 2 also hands over the ray and the sample-key inputs (A/B knob).
#ifndef BLING_SHADE_HOIST
#define BLING_SHADE_HOIST 1
#endif
#ifndef BLING_SHADE_QPREFETCH
#define BLING_SHADE_QPREFETCH 1   // queue entry of the next chunk loaded one iteration ahead (C4 +1 %, C2 neutral; A/B knob)
#endif
template <uint32_t F, bool FUSED>
static __global__ __launch_bounds__(256) SHADE_OCC void k_shade(const DevScene* __restrict__ Sptr, WaveState W, int depth, int qin,
                                               uint32_t seed, uint32_t pass, Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[qin];
  const uint32_t* q = W.queue[qin];
  unsigned long long n_drop = 0;
  const float4* Tcur = FUSED ? W.Tn : W.T;
  float4* Tnext = FUSED ? W.T : W.Tn;
#if BLING_SHADE_COMPACT
  __shared__ uint32_t ring_i[4][SHADE_RING], ring_e[4][SHADE_RING];
#if BLING_SHADE_HOIST
  __shared__ uint32_t ring_f[4][SHADE_RING];
  __shared__ float4 ring_h[4][SHADE_RING];
#endif
#if BLING_SHADE_HOIST > 1
  __shared__ float4 ring_o[4][SHADE_RING], ring_d[4][SHADE_RING];
  __shared__ uint32_t ring_p[4][SHADE_RING], ring_n[4][SHADE_RING];
#endif
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  uint32_t head = 0u, cnt = 0u;                                         // wave-uniform ring state
  auto shade_from_ring = [&](uint32_t slot) {
    const uint32_t i = ring_i[wv][slot], e = ring_e[wv][slot];
#if BLING_SHADE_HOIST > 1
    const uint32_t fl = ring_f[wv][slot], pix = ring_p[wv][slot], nid = ring_n[wv][slot];
    const float4 hv = ring_h[wv][slot], ro = ring_o[wv][slot], rdv = ring_d[wv][slot];
#elif BLING_SHADE_HOIST
    const uint32_t fl = ring_f[wv][slot], pix = W.pixel[i], nid = W.nidx[i];
    const float4 hv = ring_h[wv][slot], ro = W.corg[i], rdv = W.dir[i];
#else
    const uint32_t fl = W.flags[i], pix = W.pixel[i], nid = W.nidx[i];
    const float4 hv = W.hit[i], ro = W.corg[i], rdv = W.dir[i];
#endif
    const Ray ray{mk(ro.x, ro.y, ro.z), mk(rdv.x, rdv.y, rdv.z), ro.w, INFINITY};
    W.qflag[e] = (uint8_t)shade_vertex<F>(S, W, i, depth, seed, pass, Tcur, Tnext, fl, hv, ray, pix, nid);
  };
#if BLING_SHADE_DUAL
  static_assert(BLING_SHADE_HOIST == 1, "the dual-chunk loop hands flags and hit over through the ring");
  for (uint32_t base = (blockIdx.x * (blockDim.x >> 6) + wv) * 128u; base < n; base += nwaves * 128u) {
    uint32_t ee[2], ii[2] = {0u, 0u}, ff[2] = {0u, 0u}, vv[2] = {0u, 0u};
    float4 hh[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    Sp LL[2];
    bool ok[2], vert[2] = {false, false};
#pragma unroll
    for (int u = 0; u < 2; ++u) {               // loads of both entries first (no stores in between)
      ee[u] = base + (uint32_t)u * 64u + lane;
      ok[u] = ee[u] < n;
      if (ok[u]) { ii[u] = q[ee[u]]; }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (ok[u]) {
        ff[u] = W.flags[ii[u]]; hh[u] = W.hit[ii[u]];
        if constexpr (FUSED) vv[u] = W.vflags[ii[u]];
      }
    }
    if constexpr (FUSED) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (ok[u]) LL[u] = resolve_L<F>(S, W, ii[u], vv[u], W.T, depth == 1, depth - 1);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!ok[u]) continue;
      const uint32_t i = ii[u], e = ee[u];
      bool ends = false;
      if constexpr (FUSED) {
        if (vv[u] & VF_TERM) { finalize(W, i, LL[u], n_drop); ends = true; }   // the path stopped at d - 1
      }
      if (!ends) {
        const uint32_t ref = __float_as_uint(hh[u].y);
        if (ref != REF_NONE && depth != S.max_depth) {
          if constexpr (FUSED) store_ps(W.L, i, LL[u]);
          vert[u] = true;
        } else {
          Sp L;
          if constexpr (FUSED) L = LL[u]; else L = depth == 0 ? sconst(0.f) : load_ps(W.L, i);
          const float4 rdv = W.dir[i];
          shade_end<F>(S, W, i, Tcur, ref == REF_NONE && (ff[u] & FL_SPEC) != 0, mk(rdv.x, rdv.y, rdv.z), L, n_drop,
                       depth == 0);
        }
      }
      if (!vert[u]) W.qflag[e] = 0u;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned long long m = __ballot(vert[u]);
      if (vert[u]) {
        const uint32_t slot = (head + cnt + (uint32_t)__popcll(m & below)) & (SHADE_RING - 1u);
        ring_i[wv][slot] = ii[u]; ring_e[wv][slot] = ee[u];
        ring_f[wv][slot] = ff[u]; ring_h[wv][slot] = hh[u];
      }
      cnt += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (cnt >= 64u) {                                                 // a full wave of vertices
        shade_from_ring((head + lane) & (SHADE_RING - 1u));
        head = (head + 64u) & (SHADE_RING - 1u);
        cnt -= 64u;
      }
    }
  }
#else
#if BLING_SHADE_QPREFETCH
  // the next chunk's queue entry is loaded one iteration ahead (its latency overlaps this chunk)
  uint32_t qnext = 0u;
  {
    const uint32_t e0 = (blockIdx.x * (blockDim.x >> 6) + wv) * 64u + lane;
    if (e0 < n) qnext = q[e0];
  }
#endif
  for (uint32_t base = (blockIdx.x * (blockDim.x >> 6) + wv) * 64u; base < n; base += nwaves * 64u) {
    const uint32_t e = base + lane;
#if BLING_SHADE_QPREFETCH
    const uint32_t qcur = qnext;
    if (e + nwaves * 64u < n) qnext = q[e + nwaves * 64u];
#endif
    bool vert = false;
    uint32_t i = 0u, fl = 0u;
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
#if BLING_SHADE_HOIST > 1
    float4 ro = hv, rdv = hv;
    uint32_t pix = 0u, nid = 0u;
#endif
    if (e < n) {
#if BLING_SHADE_QPREFETCH
      i = qcur;
#else
      i = q[e];
#endif
#if BLING_SHADE_HOIST
      fl = W.flags[i];                          // issued together with the resolve loads
      hv = W.hit[i];
#endif
#if BLING_SHADE_HOIST > 1
      ro = W.corg[i]; rdv = W.dir[i]; pix = W.pixel[i]; nid = W.nidx[i];
#endif
      Sp L;
      bool ends = false;
      if constexpr (FUSED) {
        const uint32_t vfp = W.vflags[i];
        L = resolve_L<F>(S, W, i, vfp, W.T, depth == 1, depth - 1);
        if (vfp & VF_TERM) { finalize(W, i, L, n_drop); ends = true; }     // the path stopped at d - 1
      }
      if (!ends) {
#if !BLING_SHADE_HOIST
        fl = W.flags[i];
        hv = W.hit[i];
#endif
        const uint32_t ref = __float_as_uint(hv.y);
        if (ref != REF_NONE && depth != S.max_depth) {
          if constexpr (FUSED) store_ps(W.L, i, L);
          vert = true;
        } else {
          if constexpr (!FUSED) L = depth == 0 ? sconst(0.f) : load_ps(W.L, i);
          const float4 rdv = W.dir[i];
          shade_end<F>(S, W, i, Tcur, ref == REF_NONE && (fl & FL_SPEC) != 0, mk(rdv.x, rdv.y, rdv.z), L, n_drop, depth == 0);
        }
      }
      if (!vert) W.qflag[e] = 0u;
    }
    const unsigned long long m = __ballot(vert);
    if (vert) {
      const uint32_t slot = (head + cnt + (uint32_t)__popcll(m & below)) & (SHADE_RING - 1u);
      ring_i[wv][slot] = i; ring_e[wv][slot] = e;
#if BLING_SHADE_HOIST
      ring_f[wv][slot] = fl; ring_h[wv][slot] = hv;
#endif
#if BLING_SHADE_HOIST > 1
      ring_o[wv][slot] = ro; ring_d[wv][slot] = rdv; ring_p[wv][slot] = pix; ring_n[wv][slot] = nid;
#endif
    }
    cnt += (uint32_t)__popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (cnt >= 64u) {                                                   // a full wave of vertices
      shade_from_ring((head + lane) & (SHADE_RING - 1u));
      head = (head + 64u) & (SHADE_RING - 1u);
      cnt -= 64u;
    }
  }
#endif  // BLING_SHADE_DUAL
  if (lane < cnt) shade_from_ring((head + lane) & (SHADE_RING - 1u));   // the rest of the ring
#else
  const uint32_t gstride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gstride) {
    uint32_t i = q[e];
    Sp L;
    if constexpr (FUSED) {
      const uint32_t vfp = W.vflags[i];
      L = resolve_L<F>(S, W, i, vfp, W.T, depth == 1, depth - 1);
      if (vfp & VF_TERM) {                                              // the path stopped at d - 1
        finalize(W, i, L, n_drop);
        W.qflag[e] = 0u;
        continue;
      }
    }
    const uint32_t fl = W.flags[i];
    const float4 hv = W.hit[i], ro = W.corg[i], rdv = W.dir[i];
    const uint32_t ref = __float_as_uint(hv.y);
    const Ray ray{mk(ro.x, ro.y, ro.z), mk(rdv.x, rdv.y, rdv.z), ro.w, INFINITY};
    if (ref != REF_NONE && depth != S.max_depth) {
      if constexpr (FUSED) store_ps(W.L, i, L);
      W.qflag[e] = (uint8_t)shade_vertex<F>(S, W, i, depth, seed, pass, Tcur, Tnext, fl, hv, ray, W.pixel[i], W.nidx[i]);
    } else {
      if constexpr (!FUSED) L = depth == 0 ? sconst(0.f) : load_ps(W.L, i);
      shade_end<F>(S, W, i, Tcur, ref == REF_NONE && (fl & FL_SPEC) != 0, ray.d, L, n_drop, depth == 0);
      W.qflag[e] = 0u;
    }
  }
#endif
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ DirectLighting vertex
// directLighting / cont (Integrator/DirectLighting.hs:22-57) as a depth-first walk of each sample's
// ray tree with one ray in flight: a hit node emits the one-light estimate (dimensions 2d, 2d + 1)
// plus Le towards wo through k_resolve with its weight T, then continues into its specular
// reflection child and parks the transmission child in slot d + 1; a node without children (or a
// miss, which adds black) resumes the deepest parked sibling.  Depth is per path (flags).
template <uint32_t F>
static __global__ __launch_bounds__(256) SHADE_OCC void k_shade_dl(const DevScene* __restrict__ Sptr, WaveState W, int qin, uint32_t seed,
                                                  uint32_t pass, Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[qin];
  const uint32_t* q = W.queue[qin];
  unsigned long long n_drop = 0;
  const size_t cap = W.cap;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint32_t i = q[e];
    const uint32_t fl = W.flags[i];
    const int d = (int)(fl & 0xFFu);
    const float4 hv = W.hit[i], ro = W.corg[i], rdv = W.dir[i];
    const Ray ray{mk(ro.x, ro.y, ro.z), mk(rdv.x, rdv.y, rdv.z), ro.w, INFINITY};
    const bool hit = __float_as_uint(hv.y) != REF_NONE;
    bool app_sh = false, app_mis = false, next = false;
    uint32_t mask = W.dl_mask[i], vf = 0u;
    float4 no = ro, nd = rdv;
    int nlev = 0;
    if (hit) {
      const Sp T = load_ps(W.T, i);
      SampleKey k = sample_key(seed, pass, W.pixel[i], W.nidx[i]);
      DG dgg, dgs;
      float eps;
      int mat, hit_light;
      hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
      const V3 wo = -ray.d;
      const int intl = (hit_light >= 0 && dot(dgg.n, wo) > 0.f) ? hit_light : -1;     // intLe int wo
      float ttmp[(F & FT_PROCTEX) ? 32 : 1];  // computed spectra of the BSDF (FT_PROCTEX profiles)
      Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs, ttmp);
      const V3 p = bsdf.p;
      vf = ((uint32_t)(intl + 1) & 0xFFu) << 8;
      direct_setup<F>(S, W, i, k, bsdf, wo, p, eps, 2 * d, 2 * d, 1 + 2 * d, 1 + 2 * d, vf, app_mis, app_sh);
      if (d + 1 != S.max_depth) {                                          // cont: d == md -> black
        Sp fr, ft; V3 wr, wt;
        const bool hr = !(sample_bsdf_spec<F>(bsdf, wo, F_REFL, fr, wr) == 0.f);
        const bool ht = !(sample_bsdf_spec<F>(bsdf, wo, F_TRANS, ft, wt) == 0.f);
        const float4 po = make_float4(p.x, p.y, p.z, eps);
        if (hr) {
          next = true; no = po; nd = make_float4(wr.x, wr.y, wr.z, 0.f); nlev = d + 1;
          store_ps(W.Tn, i, fr * T);
        }
        if (ht) {
          if (hr) {                                                        // park the sibling
            const size_t slot = (size_t)(d + 1) * cap + i;
            W.dl_org[slot] = po;
            W.dl_dir[slot] = make_float4(wt.x, wt.y, wt.z, 0.f);
            store_ps(W.dl_T + 4 * (size_t)(d + 1) * cap, i, ft * T);
            mask |= 1u << (d + 1);
          } else {
            next = true; no = po; nd = make_float4(wt.x, wt.y, wt.z, 0.f); nlev = d + 1;
            store_ps(W.Tn, i, ft * T);
          }
        }
      }
      W.org[i] = make_float4(p.x, p.y, p.z, eps);
    }
    if (!next && mask != 0u) {                                             // resume the deepest sibling
      const int j = 31 - __clz(mask);
      const size_t slot = (size_t)j * cap + i;
      mask &= ~(1u << j);
      next = true; no = W.dl_org[slot]; nd = W.dl_dir[slot]; nlev = j;
      store_ps(W.Tn, i, load_ps(W.dl_T + 4 * (size_t)j * cap, i));
    }
    W.dl_mask[i] = mask;
    if (next) {
      W.corg[i] = no;
      W.dir[i] = nd;
      W.flags[i] = FL_ALIVE | (uint32_t)nlev;
    } else if (!hit) {
      finalize(W, i, load_ps(W.L, i), n_drop);
    }
    if (hit) W.vflags[i] = vf | (next ? 0u : VF_TERM);                     // k_resolve finalises on TERM
    W.qflag[e] = (uint8_t)((hit ? QF_RESOLVE : 0u) | (app_sh ? QF_ANY : 0u) | (app_mis ? QF_MIS : 0u) |
                           (next ? QF_CONT : 0u));
  }
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ resolve
template <uint32_t F>
static __global__ __launch_bounds__(256) RESOLVE_OCC void k_resolve(const DevScene* __restrict__ Sptr, WaveState W,
                                                 Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_RESOLVE];
  const uint32_t* q = W.queue[Q_RESOLVE];
  unsigned long long n_drop = 0;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    uint32_t i = q[e];
    uint32_t vf = W.vflags[i];
    Sp L = resolve_L<F>(S, W, i, vf, W.T);
    if (vf & VF_TERM) finalize(W, i, L, n_drop);
    else store_ps(W.L, i, L);
  }
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ camera rays
struct TileDesc { int x0, x1, y0, y1; uint32_t offset, count; };

DEV void init_path(const DevScene& S, const WaveState& W, uint32_t i, int ix, int iy, uint32_t n, uint32_t seed,
                   uint32_t pass) {
  uint32_t pixel = (uint32_t)((iy - S.ey0) * S.ext_w + (ix - S.ex0));
  SampleKey k = sample_key(seed, pass, pixel, n);
  float ox, oy, lu, lv;
  camera_sample(S, k, &ox, &oy, &lu, &lv);
  float imx = (float)ix + ox, imy = (float)iy + oy;
  Ray r = fire_ray(S.camera, imx, imy, lu, lv);
  W.corg[i] = make_float4(r.o.x, r.o.y, r.o.z, r.tmin);             // = org for Path
  W.dir[i] = make_float4(r.d.x, r.d.y, r.d.z, 0.f);
  if (W.dl_mask) W.dl_mask[i] = 0u;
  if (!(BLING_FUSED && S.integrator == BLING_INTEGRATOR_PATH)) {
    // the fused Path pipeline takes the first vertex's T = 1 and L = 0 as constants (k_shade at
    // depth 0, resolve_L at depth 1): 128 B per path neither written here nor read back
    store_ps(W.T, i, sconst(1.f));
    store_ps(W.L, i, sconst(0.f));
  }
  W.flags[i] = FL_ALIVE | FL_SPEC;
  W.pixel[i] = pixel;
  W.nidx[i] = n;
  W.img[i] = make_float2(imx, imy);
  W.result[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  W.queue[Q_SHADE0][i] = i;
  W.queue[Q_CLOSEST][i] = (i << 1) | ENTRY_CONT;
}

static __global__ __launch_bounds__(256) void k_raygen(const DevScene* __restrict__ Sptr, WaveState W,
                                                const TileDesc* __restrict__ tiles, uint32_t seed, uint32_t pass) {
  const DevScene& S = *Sptr;
  const TileDesc td = tiles[blockIdx.y];
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= td.count) return;
  uint32_t pt = S.fd_spp.div(j), n = j - pt * (uint32_t)S.spp;
  int tw = td.x1 - td.x0 + 1;
  int ix = td.x0 + (int)(pt % (uint32_t)tw), iy = td.y0 + (int)(pt / (uint32_t)tw);   // coverWindow: y outer
  init_path(S, W, td.offset + j, ix, iy, n, seed, pass);
}

static __global__ __launch_bounds__(256) void k_raygen_list(const DevScene* __restrict__ Sptr, WaveState W,
                                                     const int32_t* __restrict__ list, uint32_t n_list, uint32_t seed,
                                                     uint32_t pass) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_list) return;
  init_path(*Sptr, W, i, list[3 * i], list[3 * i + 1], (uint32_t)list[3 * i + 2], seed, pass);
}

// queue counters for a fresh wave of n paths: SHADE0 = CLOSEST = n, the rest 0
static __global__ void k_reset_queues(uint32_t* qcount, uint32_t n) {
  if (threadIdx.x < Q_N) qcount[threadIdx.x] = (threadIdx.x == Q_SHADE0 || threadIdx.x == Q_CLOSEST) ? n : 0u;
}
// Before shade(d): the trace / resolve queues of this iteration are consumed.  Account the rays
// they held (Q_CLOSEST = continuation (camera at d = 0) rays of d + MIS rays of d - 1; Q_ANY =
// shadow rays of d - 1; the shade input = paths alive at d), then clear them and the next shade queue.
// Fused mode (k_shade<F, true>): the shade input is the resolve list of d - 1, and the scan left
// the number of paths alive at d (continuation rays) in the Q_RESOLVE counter.
static __global__ void k_stage(uint32_t* qcount, int qin, int depth, Counters* C, int fused) {
  if (threadIdx.x != 0) return;
  unsigned long long alive = (fused && depth > 0) ? qcount[Q_RESOLVE] : qcount[qin];
  unsigned long long closest = qcount[Q_CLOSEST], any = qcount[Q_ANY];
  if (depth == 0) C->cam += alive; else C->cont += alive;
  C->mis += closest - alive;
  C->shadow += any;
  C->vertices += alive;
}

// ------------------------------------------------------------------ queue compaction
// Order-preserving stream compaction of k_shade's flags into the next queues: block b owns shade
// entries [b * 4096, (b + 1) * 4096), wave w of it 1024 consecutive ones.  count -> scan -> scatter,
// three small launches instead of same-address atomics from every wave (those serialise across
// the 8 XCDs and cost milliseconds per bounce).  Closest queue = all MIS entries, then all
// continuation entries, each in shade-queue order (paths stay in raygen order: coherent rays).
DEV void wave_counts(const uint8_t* __restrict__ flag, uint32_t wb, uint32_t n, uint32_t cnt[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0u;
  for (uint32_t k = 0; k < 16; ++k) {
    uint32_t e = wb + k * 64u + lane;
    uint32_t f = e < n ? flag[e] : 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) cnt[c] += (uint32_t)__popcll(__ballot((f >> c) & 1u));
  }
}

static __global__ __launch_bounds__(256) void k_compact_count(WaveState W, int qin) {
  __shared__ uint32_t s[4][4];
  const uint32_t n = W.qcount[qin];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t wb = blockIdx.x * COMPACT_CHUNK + w * 1024u;
  uint32_t cnt[4];
  wave_counts(W.qflag, wb, n, cnt);
  if (lane == 0) for (int c = 0; c < 4; ++c) s[w][c] = cnt[c];
  __syncthreads();
  if (threadIdx.x < 4) W.blk[4 * blockIdx.x + threadIdx.x] = s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x];
}

// one block of 1024: exclusive scan of the per-block counts; queue lengths for the next launches
// fused: the next shade input (qin ^ 1) is the resolve list, and Q_RESOLVE's counter carries the
// continuation count (k_stage); otherwise the next shade input is the continuation list.
static __global__ __launch_bounds__(1024) void k_compact_scan(WaveState W, uint32_t nb, int qin, int fused) {
  __shared__ uint32_t s[1024][4];
  const uint32_t t = threadIdx.x;
  const uint32_t seg = (nb + 1023u) / 1024u, b0 = t * seg, b1 = min(nb, b0 + seg);
  uint32_t sum[4] = {0u, 0u, 0u, 0u};
  for (uint32_t b = b0; b < b1; ++b)
    for (int c = 0; c < 4; ++c) sum[c] += W.blk[4 * b + c];
  for (int c = 0; c < 4; ++c) s[t][c] = sum[c];
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {          // Hillis-Steele inclusive scan
    uint32_t v[4];
    for (int c = 0; c < 4; ++c) v[c] = t >= off ? s[t - off][c] : 0u;
    __syncthreads();
    for (int c = 0; c < 4; ++c) s[t][c] += v[c];
    __syncthreads();
  }
  uint32_t run[4];
  for (int c = 0; c < 4; ++c) run[c] = s[t][c] - sum[c];
  for (uint32_t b = b0; b < b1; ++b)
    for (int c = 0; c < 4; ++c) { uint32_t x = W.blk[4 * b + c]; W.blk[4 * b + c] = run[c]; run[c] += x; }
  if (t == 1023) {
    const uint32_t tr = s[t][0], ta = s[t][1], tm = s[t][2], tc = s[t][3];
    W.blk[4 * nb + 0] = tm;                                   // MIS total = start of the continuation part
    W.qcount[Q_RESOLVE] = fused ? tc : tr;
    W.qcount[Q_ANY] = ta;
    W.qcount[Q_CLOSEST] = tm + tc;
    W.qcount[qin ^ 1] = fused ? tr : tc;
  }
}

static __global__ __launch_bounds__(256) void k_compact_scatter(WaveState W, uint32_t nb, int qin, int fused) {
  __shared__ uint32_t s[4][4];
  const uint32_t n = W.qcount[qin];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t wb = blockIdx.x * COMPACT_CHUNK + w * 1024u;
  if (blockIdx.x * COMPACT_CHUNK >= n) return;               // whole block past the queue
  uint32_t cnt[4];
  wave_counts(W.qflag, wb, n, cnt);
  if (lane == 0) for (int c = 0; c < 4; ++c) s[w][c] = cnt[c];
  __syncthreads();
  uint32_t off[4];
  for (int c = 0; c < 4; ++c) {
    off[c] = W.blk[4 * blockIdx.x + c];
    for (uint32_t v = 0; v < w; ++v) off[c] += s[v][c];
  }
  const uint32_t mis_total = W.blk[4 * nb];
  const uint32_t* qi = W.queue[qin];
  uint32_t* qr = fused ? W.queue[qin ^ 1] : W.queue[Q_RESOLVE];
  uint32_t* qa = W.queue[Q_ANY];
  uint32_t* qc = W.queue[Q_CLOSEST];
  uint32_t* qn = fused ? nullptr : W.queue[qin ^ 1];
  const unsigned long long below = (1ull << lane) - 1ull;
  for (uint32_t k = 0; k < 16; ++k) {
    uint32_t e = wb + k * 64u + lane;
    uint32_t f = 0u, i = 0u;
    if (e < n) { f = W.qflag[e]; i = qi[e]; }
    unsigned long long m0 = __ballot(f & QF_RESOLVE), m1 = __ballot(f & QF_ANY);
    unsigned long long m2 = __ballot(f & QF_MIS), m3 = __ballot(f & QF_CONT);
    if (f & QF_RESOLVE) qr[off[0] + __popcll(m0 & below)] = i;
    if (f & QF_ANY) qa[off[1] + __popcll(m1 & below)] = i;
    if (f & QF_MIS) qc[off[2] + __popcll(m2 & below)] = (i << 1) | ENTRY_MIS;
    if (f & QF_CONT) {
      uint32_t pos = off[3] + __popcll(m3 & below);
      qc[mis_total + pos] = (i << 1) | ENTRY_CONT;
      if (!fused) qn[pos] = i;
    }
    off[0] += __popcll(m0); off[1] += __popcll(m1); off[2] += __popcll(m2); off[3] += __popcll(m3);
  }
}

// ------------------------------------------------------------------ film
// addSample into the reference's tile image (mkImageTile, Image.hs:108-120, 250-299), then addTile.
constexpr int FILM_TILE_MAX = 32;
static __global__ __launch_bounds__(256) void k_film(const DevScene* __restrict__ Sptr, WaveState W,
                                              const TileDesc* __restrict__ tiles, float* __restrict__ film) {
  __shared__ float img[FILM_TILE_MAX * FILM_TILE_MAX * 4];
  const DevScene& S = *Sptr;
  const TileDesc td = tiles[blockIdx.x];
  float fw = S.filter_w, fh = S.filter_h;
  int ox = max(0, td.x0), oy = max(0, td.y0);
  int w = td.x1 - ox + (int)floorf(0.5f + fw), h = td.y1 - oy + (int)floorf(0.5f + fh);
  for (int q = threadIdx.x; q < FILM_TILE_MAX * FILM_TILE_MAX * 4; q += blockDim.x) img[q] = 0.f;
  __syncthreads();
  float ifw = 1.f / fw, ifh = 1.f / fw;                                  // trap T12
  for (uint32_t j = threadIdx.x; j < td.count; j += blockDim.x) {
    uint32_t i = td.offset + j;
    float4 r = W.result[i];
    if (r.w == 0.f) continue;
    float2 im = W.img[i];
    float dx = im.x - 0.5f, dy = im.y - 0.5f;
    int x0 = max(ox, (int)ceilf(dx - fw)), x1 = min(ox + w - 1, (int)floorf(dx + fw));
    int y0 = max(oy, (int)ceilf(dy - fh)), y1 = min(oy + h - 1, (int)floorf(dy + fh));
    for (int y = y0; y <= y1; ++y) {
      int fy = min((int)floorf(fabsf(((float)y - dy) * ifh * 16.f)), 15);
      for (int x = x0; x <= x1; ++x) {
        int fx = min((int)floorf(fabsf(((float)x - dx) * ifw * 16.f)), 15);
        float fltw = S.filter_table[fy * 16 + fx];
        float* o = &img[4 * ((x - ox) + (y - oy) * FILM_TILE_MAX)];
        atomicAdd(&o[0], fltw);
        atomicAdd(&o[1], r.x * fltw);
        atomicAdd(&o[2], r.y * fltw);
        atomicAdd(&o[3], r.z * fltw);
      }
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < w * h; q += blockDim.x) {
    int x = q % w, y = q / w;
    int gx = x + ox, gy = y + oy;
    if (gx >= S.width || gy >= S.height) continue;
    const float* s = &img[4 * (x + y * FILM_TILE_MAX)];
    if (s[0] == 0.f && s[1] == 0.f && s[2] == 0.f && s[3] == 0.f) continue;
    float* o = film + 4 * ((size_t)gy * S.width + gx);
    atomicAdd(&o[0], s[0]); atomicAdd(&o[1], s[1]); atomicAdd(&o[2], s[2]); atomicAdd(&o[3], s[3]);
  }
}

// Register-accumulating film splat: thread t owns source pixel t of the tile and sums the filtered
// contributions of all its samples to the K x K window of output pixels around it in registers
// (K = 2 * floor(0.5 + fw) + 1: 5 for the width-2 filters of C1/C2/C4/C5, 7 for C3's width 3), then
// adds the window into the tile image in LDS once.  Same pixel ranges, table lookups and tile
// clipping as k_film (addSample, Image.hs:250-299); ~K*K*4 LDS atomics per source pixel instead of
// ~K*K*4 per sample.
template <int K>
static __global__ __launch_bounds__(256) void k_film_gather(const DevScene* __restrict__ Sptr, WaveState W,
                                                     const TileDesc* __restrict__ tiles, float* __restrict__ film) {
  __shared__ float img[FILM_TILE_MAX * FILM_TILE_MAX * 4];
  __shared__ float tbl[256];
  constexpr int R = K / 2;
  const DevScene& S = *Sptr;
  const TileDesc td = tiles[blockIdx.x];
  const float fw = S.filter_w, fh = S.filter_h;
  const int ox = max(0, td.x0), oy = max(0, td.y0);
  const int w = td.x1 - ox + (int)floorf(0.5f + fw), h = td.y1 - oy + (int)floorf(0.5f + fh);
  for (int q = threadIdx.x; q < FILM_TILE_MAX * FILM_TILE_MAX * 4; q += blockDim.x) img[q] = 0.f;
  tbl[threadIdx.x] = S.filter_table[threadIdx.x];
  __syncthreads();
  const float ifw = 1.f / fw, ifh = 1.f / fw;                            // trap T12
  const int tw = td.x1 - td.x0 + 1, npix = tw * (td.y1 - td.y0 + 1);
  const uint32_t spp = (uint32_t)S.spp;
  const int pt = threadIdx.x;
  if (pt < npix) {
    const int ix = td.x0 + pt % tw, iy = td.y0 + pt / tw;
    float acc[K][K][4];
#pragma unroll
    for (int b = 0; b < K; ++b)
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[b][a][c] = 0.f;
    const uint32_t base = td.offset + (uint32_t)pt * spp;
    for (uint32_t n = 0; n < spp; ++n) {
      const float4 r = W.result[base + n];
      if (r.w == 0.f) continue;
      const float2 im = W.img[base + n];
      const float dx = im.x - 0.5f, dy = im.y - 0.5f;
      const int x0 = max(ox, (int)ceilf(dx - fw)), x1 = min(ox + w - 1, (int)floorf(dx + fw));
      const int y0 = max(oy, (int)ceilf(dy - fh)), y1 = min(oy + h - 1, (int)floorf(dy + fh));
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const int y = iy - R + b;
        if (y < y0 || y > y1) continue;
        const int fy = min((int)floorf(fabsf(((float)y - dy) * ifh * 16.f)), 15);
#pragma unroll
        for (int a = 0; a < K; ++a) {
          const int x = ix - R + a;
          if (x < x0 || x > x1) continue;
          const int fx = min((int)floorf(fabsf(((float)x - dx) * ifw * 16.f)), 15);
          const float fltw = tbl[fy * 16 + fx];
          acc[b][a][0] += fltw;
          acc[b][a][1] += r.x * fltw;
          acc[b][a][2] += r.y * fltw;
          acc[b][a][3] += r.z * fltw;
        }
      }
    }
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int y = iy - R + b;
      if (y < oy || y >= oy + h) continue;
#pragma unroll
      for (int a = 0; a < K; ++a) {
        const int x = ix - R + a;
        if (x < ox || x >= ox + w) continue;
        if (acc[b][a][0] == 0.f && acc[b][a][1] == 0.f && acc[b][a][2] == 0.f && acc[b][a][3] == 0.f) continue;
        float* o = &img[4 * ((x - ox) + (y - oy) * FILM_TILE_MAX)];
#pragma unroll
        for (int c = 0; c < 4; ++c) atomicAdd(&o[c], acc[b][a][c]);
      }
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < w * h; q += blockDim.x) {
    int x = q % w, y = q / w;
    int gx = x + ox, gy = y + oy;
    if (gx >= S.width || gy >= S.height) continue;
    const float* sp = &img[4 * (x + y * FILM_TILE_MAX)];
    if (sp[0] == 0.f && sp[1] == 0.f && sp[2] == 0.f && sp[3] == 0.f) continue;
    float* o = film + 4 * ((size_t)gy * S.width + gx);
    atomicAdd(&o[0], sp[0]); atomicAdd(&o[1], sp[1]); atomicAdd(&o[2], sp[2]); atomicAdd(&o[3], sp[3]);
  }
}

}  // namespace bd
