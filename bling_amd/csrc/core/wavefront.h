// wavefront.h -- the per-bounce kernels of the MI355X path integrator (Integrator/Path.hs:41-87)
// and of the DirectLighting integrator (Integrator/DirectLighting.hs:22-57, k_shade_dl).
//
// One path vertex d = three launches over compacted work queues:
//   k_trace_closest     closest-hit queries of {continuation rays of d} + {BSDF-MIS rays of d - 1}
//   k_trace_any         any-hit queries of the light-sample shadow rays of d - 1
//   k_shade<F, true>    resolve vertex d - 1 (L += T (Le + lc (ls vis + bs)), Scene.hs:61-118 and
//                       Path.hs:73-79), finish the paths that stop, and shade vertex d: hit
//                       reconstruction, BSDF, the one-light estimate's two rays and candidates,
//                       Russian roulette and the continuation (Path.hs:54-87)
// then an order-preserving compaction of the shade launch's queue flags into the next queues.
//
// Path state follows the queue.  The state of a path lives in one of two ping-pong sets (PathSet)
// at a slot: the queue entry of the launch that wrote it.  A shade launch reads its inputs from the
// current set at the slots its queue lists (gathers over the previous launch's entries: dense, since
// most paths survive a bounce) and writes every vertex it shades to the next set at a slot of its
// own entry chunk: the chunk's new vertices take its first slots in entry order (round 5) --
// consecutive lanes, consecutive slots, coalesced full-line stores -- and the trace kernels
// of the next vertex read and write that set at the slots their queues list.  A path's sample id
// (raygen order) travels in its record; only the finished radiance is written by sample id.  Per
// path a set holds 64-B records: the ray / hit / metadata record, the estimate record (BSDF-MIS
// direction and weight, factored candidates, the traced outcomes, the continuation's factors) and the
// throughput and radiance spectra, so a gather pays whole lines.
// DirectLighting walks a per-sample tree with parked siblings; it runs in place (one set, slot =
// sample id).
#pragma once
#include "../../../include/bling.h"
#include "dev_shade.h"
#include "dev_trace.h"

namespace bd {

// Occupancy targets (waves per SIMD) the register allocator must meet.
// Shading kernels of the profiles with glass / substrate / bump lobes need more than 256 VGPRs
// unconstrained (k_shade of the sun-sky profile: 260, one wave per SIMD); they are held to >= 2
// waves per SIMD (<= 256 VGPRs).  A/B on MI355X, C4: 3 558 -> 5 155 Mrays/s; the other profiles keep
// the compiler's choice (cornell's 159 VGPRs at 3 waves: forcing 2 measured -6 %).
// The sun-sky profile (glass / metal / plastic spheres under the sky, no meshes) is latency bound;
// at three waves it spills and still runs faster (round 2 A/B, profiles/r02_ab_shade_waves.txt:
// C4 +2.8 %; the meshes profile at three waves: C3 -2.7 %, so it keeps the compiler's choice).
constexpr int kSkyWaves = 3;
// Round 3 (one-call-site shading, ring-carried hit / metadata / sY(T)): the cornell profile at four
// waves (128 VGPRs, 48 B of scratch) and the meshes profile at three (168, 80 B) beat the compiler's
// choice of three (145) and two (199): C2 +1.5 %, C3 +2.6 % (profiles/r03_ab_occupancy.txt); the
// sun-sky profile at two waves lost 14 % against three.  Round 5 moved cornell back to three (below).
// Round 5: the cornell profile's k_shade at three waves (168 VGPRs, 60 B scratch) against four (128,
// 88 B): C2 +0.5 % and +0.4 % on two boxes (profiles/r05_ab_session.txt r05b, r05f).
// Round 6: with the v2 sampler and the triangle frames it needs 134 VGPRs at three waves; at four
// (128 VGPRs, 28 B scratch) shade 42.3 -> 41.1 ms per pass, C2 +0.7 % (profiles/r06_ab_session.txt r06s2l)
#ifndef BLING_CORNELL_SHADE_WAVES
#define BLING_CORNELL_SHADE_WAVES 4   // experiment builds may override (make variant DEFS=...)
#endif
template <uint32_t F>
constexpr int shade_min_waves() {
  return ((F & FT_ENV_SKY) && (F & FT_GLASS) && !(F & (FT_TRIS | FT_SUBSTRATE | FT_BUMP))) ? kSkyWaves
       : ((F & (FT_GLASS | FT_SUBSTRATE | FT_BUMP)) ? 2
       : (F == (FT_MATTE | FT_AREA | FT_TRIS) ? BLING_CORNELL_SHADE_WAVES : ((F & FT_TRIS) ? 3 : 1)));
}
#define SHADE_OCC __attribute__((amdgpu_waves_per_eu(shade_min_waves<F>(), 8)))
// The fractal profiles' closest-hit kernel (the paired march) sits just above the 168 VGPRs of
// three waves per SIMD; it is held to three.  The all-LDS BVH4 kernel (ALLL: small scenes, no global
// fallback) is held to eight (70 -> 64 VGPRs; A/B on C2, profiles/r02_ab_occupancy_s5.txt: closest
// 41.4 -> 40.1 ms/pass; the same floor on the meshes profile's global-fallback kernel lost 10 % on C3,
// so it applies to ALLL only).  The other kernels keep the compiler's choice.
#ifndef BLING_ALLL_WAVES
#define BLING_ALLL_WAVES 8   // experiment builds may override
#endif
template <uint32_t F, bool ALLL>
constexpr int trace_min_waves() { return (F & FT_FRACTAL) ? 3 : ((ALLL && use_bvh4<F>()) ? BLING_ALLL_WAVES : 1); }
#define TRACE_OCC __attribute__((amdgpu_waves_per_eu(trace_min_waves<F, ALLL>(), 8)))

// Per-vertex flags (the .x word of the metadata record)
constexpr uint32_t VF_SH = 1u, VF_MIS = 2u, VF_TERM = 4u;   // shadow ray / BSDF-MIS ray set up; path ends
constexpr uint32_t VF_SPEC = 8u;                            // Path: the continuation sample was specular
constexpr uint32_t VF_OCC = 0x200u;                         // in-line shadow test: the shadow ray is occluded
// bits 4-8: DirectLighting depth of the next ray; bits 16-23: the light hit (intLe) + 1; bits 24-31:
// the light sampled (sampleOneLight) -- scenes hold at most 254 lights (upload checks)
DEV uint32_t vf_depth(uint32_t vf) { return (vf >> 4) & 31u; }
DEV int vf_intl(uint32_t vf) { return (int)((vf >> 16) & 0xFFu) - 1; }
DEV int vf_light(uint32_t vf) { return (int)(vf >> 24); }
DEV uint32_t vf_make(int intl, int depth) { return ((uint32_t)(intl + 1) & 0xFFu) << 16 | ((uint32_t)depth & 31u) << 4; }
constexpr uint32_t ENTRY_CONT = 0u, ENTRY_MIS = 1u;

enum QueueId : int { Q_SHADE0 = 0, Q_SHADE1 = 1, Q_CLOSEST = 2, Q_ANY = 3, Q_RESOLVE = 4, Q_N = 5 };

// One set of path state, indexed by slot, as SoA arrays: a launch's lanes touch consecutive (or
// nearly consecutive, per-bounce dense) slots, so each field is a coalesced stream and a kernel reads
// only the fields it needs (the trace kernels: 32 B of ray, 16 B of hit).
//   org   p.xyz, eps      origin + tmin of the BSDF-MIS and continuation rays (camera ray at d = 0)
//   dir   d.xyz, -        continuation (camera) ray direction
//   hit   t, ref, b1, b2  closest hit of the continuation ray (k_trace_closest)
//   meta  vf, pixel, n, sid   per-vertex flags, sample-extent pixel, sample number, sample id
//   mdir  wi.xyz, w       BSDF-MIS ray direction and its MIS weight
//   mhit  t, ref          BSDF-MIS ray's closest hit (k_trace_closest)
//   occ   0 / 1           the shadow ray is occluded (k_trace_any)
//   fac   s1 f_mis, s1, s2, w / pdf    factored candidates (factored profiles)
//   cf    s1, pc, rtex, - factored profiles: the continuation's f = r s1, the RR pc and the lobe
//                         spectrum's byte offset, so the next launch forms T' = (f T) / pc itself
//   sh_o, sh_d            the light sample's shadow ray (o, tmin | d, tmax)
//   T (throughput of the vertex), Tn (after the continuation; non-factored profiles), L (radiance so
//   far), lsc / bsc (light- / BSDF-sample candidates; non-factored profiles): 16-band spectra, one
//   64-B record per slot.
struct PathSet {
  float4 *org, *dir, *hit;
  uint4* meta;
  float4* mdir;
  float2* mhit;
  uint32_t* occ;
  float4 *fac, *cf, *sh_o, *sh_d;
  float4 *T, *Tn, *L, *lsc, *bsc;
};

// a vertex's estimate as its shade launch writes it and the next launch's resolve reads it
struct Est { float4 mdir, fac, cf; float2 mhit; uint32_t occ; };
DEV Est load_est(const PathSet& P, uint32_t s, uint32_t vf, bool factored_) {
  Est m;
  m.mdir = P.mdir[s];
  m.mhit = (vf & 2u) ? P.mhit[s] : make_float2(0.f, 0.f);
  m.occ = (vf & 1u) ? P.occ[s] : 0u;
  m.fac = factored_ ? P.fac[s] : make_float4(0.f, 0.f, 0.f, 0.f);
  m.cf = factored_ ? P.cf[s] : make_float4(0.f, 0.f, 0.f, 0.f);
  return m;
}
// The same record loaded without waiting for the metadata: the traced outcomes (mhit, occ) are read
// whatever the flags say (their slots always exist; a value whose ray was not traced is never used),
// so every load of the record issues together with the metadata's instead of one memory latency
// after it.  The flags still select what the resolve uses.
DEV Est load_est_eager(const PathSet& P, uint32_t s, bool factored_, bool occ = true) {
  Est m;
  m.mdir = P.mdir[s];
  m.mhit = P.mhit[s];
  m.occ = occ ? P.occ[s] : 0u;
  m.fac = factored_ ? P.fac[s] : make_float4(0.f, 0.f, 0.f, 0.f);
  m.cf = factored_ ? P.cf[s] : make_float4(0.f, 0.f, 0.f, 0.f);
  return m;
}

struct WaveState {
  PathSet cur;        // the set the queues index (read side; the trace kernels also write it)
  PathSet nxt;        // the set a Path shade launch writes (at its entry chunks' slots); the host
                      // swaps cur / nxt after it.  DirectLighting: nxt == cur, slot = sample id
  float4* corg;       // DirectLighting: continuation ray origin + tmin by sample id (its popped
                      // sibling rays start away from the vertex whose MIS ray is traced alongside)
  float2* img;        // by sample id: imageX, imageY
  float4* result;     // by sample id: X, Y, Z, 1 (or 0 = dropped)
  float4* Lfull;      // by sample id: [n][4] final spectrum (parity hook only, may be NULL)
  float* dbg;         // by sample id: per-vertex debug records (bling_sample_li_vertices; BLING_DEBUG_VERTEX builds only)
  float* march_t;     // Mandelbulb scenes: per entry of the closest / any queue, the k_march result
                      // (hit distance, or -1); NULL when the traversal kernels march themselves
  uint32_t* queue[Q_N];
  uint32_t* qcount;   // Q_N counters
  uint8_t* qflag;     // per shade-queue entry: QF_* bits written by k_shade, compacted by k_compact_*
  uint32_t* blk;      // compaction: per-block counts / offsets [nb][4], then totals [4]
  unsigned long long* sb;   // BLING_STREAM_STATS builds: Counters::sb of the pass (else unused)
  // DirectLighting only (NULL for Path), by sample id: the pending specular-transmission sibling of
  // level j (1 <= j < maxDepth) of each sample's depth-first walk, slot j at [j * cap + i]
  float4* dl_org;     // p.xyz, eps
  float4* dl_dir;     // wi
  float4* dl_T;       // [levels * cap][4] weight of the pending ray
  uint32_t* dl_mask;  // bit j set = slot j pending
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
  unsigned long long sb[2 * BLING_N_STREAMS];   // BLING_STREAM_STATS: k_shade's bytes per stream (read, write)
};

// Path-state bytes of the shading kernel per stream (bling_debug_stream_bytes, include/bling.h):
// counted where the algorithm needs a record -- a field the path uses, written once, read back
// once -- whatever the code loads besides (e.g. the eager mhit / occ loads), so the roofline's
// algorithmic bytes are a floor of the DRAM traffic.  Only BLING_STREAM_STATS builds count.
#ifndef BLING_STREAM_STATS
#define BLING_STREAM_STATS 0
#endif
enum StreamId : int { SB_QUEUE, SB_HIT, SB_META, SB_ORG, SB_DIR, SB_MDIR, SB_MHIT, SB_OCC, SB_FAC, SB_CF, SB_T, SB_L,
                      SB_TN, SB_LSC, SB_BSC, SB_SHO, SB_SHD, SB_RESULT, SB_QFLAG };
static_assert(SB_QFLAG + 1 == BLING_N_STREAMS, "stream list of include/bling.h");
DEV void sb_count(unsigned long long* sb, int k, bool wr, uint32_t bytes, bool pred) {
#if BLING_STREAM_STATS
  const unsigned long long m = __ballot(pred);
  const uint32_t lead = (uint32_t)__ffsll((long long)__ballot(1)) - 1u;
  if (m && sb && (threadIdx.x & 63u) == lead) atomicAdd(&sb[2 * k + (wr ? 1 : 0)], (unsigned long long)__popcll(m) * bytes);
#else
  (void)sb; (void)k; (void)wr; (void)bytes; (void)pred;
#endif
}
#define SBR(W, k, bytes, pred) sb_count((W).sb, (k), false, (bytes), (pred))
#define SBW(W, k, bytes, pred) sb_count((W).sb, (k), true, (bytes), (pred))

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

// Spectrum records: one 64-B record per index ([n][4] float4).
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

DEV void finalize(const WaveState& W, uint32_t sid, const Sp& L, unsigned long long& dropped) {
  SBW(W, SB_RESULT, 16, true);
  if (W.Lfull) store_sp(W.Lfull, sid, L);
  if (s_bad(L)) { W.result[sid] = make_float4(0.f, 0.f, 0.f, 0.f); dropped++; return; }   // Image.hs:253-256
  float x, y, z;
  to_xyz(L, &x, &y, &z);
  W.result[sid] = make_float4(x, y, z, 1.f);
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
// early finish (C2 37.7 -> 43.2 with two; profiles/r02_ab_trace_steps_s5.txt).
template <bool ALLL>
constexpr int trace_steps() { return ALLL ? 1 : 3; }

// Queue-in-register refill (take_q): measured on MI355X (profiles/r05_ab_session.txt r05g) C2
// neutral (+0.2 %), C3 -3.4 % (the meshes profile's closest kernel 78 -> 82 VGPRs, 6 -> 5 waves), so
// experiment builds only (BLING_FEED_QREG=1)
#ifndef BLING_FEED_QREG
#define BLING_FEED_QREG 0
#endif
constexpr bool kFeedQreg = BLING_FEED_QREG != 0;
struct WaveFeed {
  uint32_t chunk, cur, end, n, nw;
  // queue-in-register mode (init with a queue): lane l holds entry l of the current chunk (qv) and of
  // the wave's next chunk (qn, loaded one chunk ahead), so a refill reads its entry with one lane
  // shuffle instead of a dependent global load before the ray's own loads
  const uint32_t* q = nullptr;
  uint32_t qv = 0u, qn = 0u;
  DEV uint32_t chunk_entry(uint32_t c) const {
    const uint64_t i = (uint64_t)c * FEED_CHUNK + (threadIdx.x & 63u);
    return i < n ? q[i] : 0u;
  }
  DEV void init(uint32_t n_, const uint32_t* queue = nullptr) {
    n = n_;
    nw = gridDim.x * (blockDim.x >> 6);
    chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    q = queue;
    if (kFeedQreg && q) { qv = chunk_entry(chunk); qn = chunk_entry(chunk + nw); }
    open();
  }
  DEV void open() {
    const uint64_t c0 = (uint64_t)chunk * FEED_CHUNK;
    cur = c0 < n ? (uint32_t)c0 : n;
    end = (uint32_t)((uint64_t)cur + FEED_CHUNK < n ? cur + FEED_CHUNK : n);
  }
  // take() in queue-in-register mode: *v = the queue entry q[*e]
  DEV bool take_q(bool live, uint32_t* e, uint32_t* v) {
    if constexpr (!kFeedQreg) {                   // experiment builds: the entry loaded per refill
      const bool got = take(live, e);
      if (got) *v = q[*e];
      return got;
    }
    bool got = false;
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const bool want = !live && !got;
      const unsigned long long m = __ballot(want);
      if (m == 0ull || cur >= end) break;
      const uint32_t avail = end - cur;
      const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      const uint32_t val = (uint32_t)__shfl((int)qv, (int)((cur + rank) & (FEED_CHUNK - 1u)), 64);
      if (want && rank < avail) { *e = cur + rank; *v = val; got = true; }
      const uint32_t used = min((uint32_t)__popcll(m), avail);
      cur += used;
      if (cur == end) {
        chunk += nw;
        open();
        qv = qn;
        if (cur < end) qn = chunk_entry(chunk + nw);
      }
    }
    return got;
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

// The closest-hit query of entry ent = slot << 1 | kind of the current set: a continuation ray
// (origin org, or DirectLighting's corg; direction dir) or a BSDF-MIS ray (org, mdir).
// rej: the producer's kd_root test rejected the ray (dev_trace.h kd_flag_w): it misses.
DEV Ray closest_ray(const WaveState& W, uint32_t ent, bool& rej) {
  const uint32_t s = ent >> 1;
  const bool cont = (ent & 1u) == ENTRY_CONT;
  const float4 o = (cont && W.corg) ? W.corg[s] : W.cur.org[s];
  const float4 d = cont ? W.cur.dir[s] : W.cur.mdir[s];
  rej = kd_rejected(d.w);
  return Ray{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, INFINITY};
}
DEV void closest_store(const WaveState& W, uint32_t ent, const HitRec& h) {
  const uint32_t s = ent >> 1;
  if ((ent & 1u) == ENTRY_CONT) W.cur.hit[s] = make_float4(h.t, __uint_as_float(h.ref), h.b1, h.b2);
  else W.cur.mhit[s] = make_float2(h.t, __uint_as_float(h.ref));
}
DEV Ray shadow_ray(const WaveState& W, uint32_t s) {
  const float4 o = W.cur.sh_o[s], d = W.cur.sh_d[s];
  return Ray{mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), o.w, d.w};
}
DEV void shadow_store(const WaveState& W, uint32_t s, bool occluded) { W.cur.occ[s] = occluded ? 1u : 0u; }

template <uint32_t F, bool STATS, bool ALLL>
static __global__ __launch_bounds__(256) TRACE_OCC void k_trace_closest(const DevScene* __restrict__ Sptr, WaveState W,
                                                                 Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup<use_bvh4<F>(), use_bvh4<F>() && !ALLL && kQuantBvh4, ALLL && use_bvh4<F>()>(S, smem);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_CLOSEST];
  const uint32_t* q = W.queue[Q_CLOSEST];
  WaveFeed feed;
  feed.init(n, q);
  TraceCount tc{0u, 0u, 0u, 0u};
  QTraversal<false, F, ALLL> tv;
  bool live = false;
  uint32_t ent = 0u, e = 0u;
  for (;;) {
    if (feed.take_q(live, &e, &ent)) {
      bool rej;
      const Ray r = closest_ray(W, ent, rej);
      tv.init(r, rej);
      if constexpr ((F & FT_FRACTAL) != 0) {
        if (W.march_t) { tv.pre = true; tv.mres = W.march_t[e]; }
      }
      live = true;
    }
    if (__ballot(live) == 0ull) break;
#pragma unroll
    for (int u = 0; u < trace_steps<ALLL>(); ++u) {
      if (live && tv.step(S, L, tc)) {
        closest_store(W, ent, tv.h);
        live = false;
      }
    }
  }
  flush_trace_stats<STATS, true>(C, tc);
}

template <uint32_t F, bool STATS, bool ALLL>
static __global__ __launch_bounds__(256) TRACE_OCC void k_trace_any(const DevScene* __restrict__ Sptr, WaveState W,
                                                   Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup<use_bvh4<F>(), use_bvh4<F>() && !ALLL && kQuantBvh4, ALLL && use_bvh4<F>()>(S, smem);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_ANY];
  const uint32_t* q = W.queue[Q_ANY];
  WaveFeed feed;
  feed.init(n, q);
  TraceCount tc{0u, 0u, 0u, 0u};
  QTraversal<true, F, ALLL> tv;
  bool live = false;
  uint32_t s = 0u, e = 0u;
  for (;;) {
    if (feed.take_q(live, &e, &s)) {
      tv.init(shadow_ray(W, s));                 // rejected shadow rays carry tmin = +inf
      if constexpr ((F & FT_FRACTAL) != 0) {
        if (W.march_t) { tv.pre = true; tv.mres = W.march_t[e]; }
      }
      live = true;
    }
    if (__ballot(live) == 0ull) break;
#pragma unroll
    for (int u = 0; u < trace_steps<ALLL>(); ++u) {
      if (live && tv.step(S, L, tc)) {
        shadow_store(W, s, tv.h.ref != REF_NONE);
        live = false;
      }
    }
  }
  flush_trace_stats<STATS>(C, tc);
}

// ------------------------------------------------------------------ Mandelbulb pre-march
// The Mandelbulb's march (mandelInter, Fractal.hs:23-137) depends on the ray and its entry point
// into the r^2 = 2 sphere only: it ignores rayMax (trap T10), and the entry distance t0 does not
// depend on the traversal's current closest t, which only decides whether the fractal leaf is
// entered at all.  So every query of a queue whose ray enters the sphere within [tmin, tmax]
// (closest-hit queries: tmax = inf, a superset of the entries the traversal will accept) is marched
// here, before its traversal kernel, which then takes the stored result at the fractal leaf with
// the same entry test.  Same operations from the same start, so the same hits bit for bit.
// Without the BVH walk, its stack and its refill bookkeeping in the same kernel, the march runs
// with fewer registers and every lane of a wave is marching (round 3: C5 260 -> 325 Mrays/s with
// per-lane rays and batched finishes, profiles/r03_ab_premarch.txt).
//
// k_march_jobs: the march with the lanes decoupled from the rays (per-lane rays: 325, jobs: 382 Mrays/s
// on C5, profiles/r03_ab_march_jobs.txt).  A DE step needs four
// potentials at p, p + eps x, p + eps y, p + eps z, which depend on p only: two independent pair
// jobs (the paired march's two halves).  Each wave keeps MJ_SLOTS rays in LDS; a lane holds one pair
// job in registers and iterates it; a decided pair leaves |z| and the loop counter of both of its
// potentials in the ray's record, and the second of a ray's two jobs to finish puts the ray on the
// ready list.  Once MJ_FIN rays are ready (or no job is left), the wave's lanes take one ready ray
// each and run the rest of the DE step -- the four logarithms, the gradient, exp / sinh, the step --
// and either end the ray or post its next two jobs.  So the bulbPower iterations run on every lane
// that has a job, whatever the escape counts of the rays, and the transcendental tail runs on up to
// 64 rays at once.  The operations of every potential and every step are MandelMarch2's, in the same
// order (the p + eps y / z pair of a final step whose potential at p is 0 is evaluated in vain).
// Tuned on C5 (profiles/r03_ab_march_tuning*.txt): 80 slots (64: -2.4 %, 96: -1.7 %), a finish once
// 48 rays are ready (32: -0.3 %, 40 / 64: -1 to -2 %), 4 iterations between the refill / finish
// checks (2: -3 %, 8: -1.5 %, 16: -17 %).
constexpr uint32_t MJ_SLOTS = 80, MJ_JOBS = 256, MJ_FIN = 48, MJ_K = 4;
static_assert(2 * MJ_SLOTS <= MJ_JOBS, "job ring holds two jobs per ray");
// 6 592 B per wave, 26 368 B per block: six blocks (the kernel's 77 VGPRs allow six waves per SIMD)
// share a CU's 160 KiB.  At 7 552 B (32-bit loop counters, a separate done word) only five fitted,
// so LDS, not registers, held the march at five waves per SIMD.  The loop counters are at most
// iterations + 1 (the host premarches only scenes with iterations < 32 767) and the steps below the
// 100 000 cap, so the pair count of a step rides in the top two bits of its steps word.
struct MarchSlots {                 // per wave, in LDS
  float o[3][MJ_SLOTS], rn[3][MJ_SLOTS], p[3][MJ_SLOTS], d[MJ_SLOTS];
  float zl[4][MJ_SLOTS];            // |z| of the escaped iterate of potential k of the current step
  int16_t zn[4][MJ_SLOTS];          // its loop counter at the decision (1 = iterations spent)
  uint32_t sd[MJ_SLOTS];            // steps | (pairs of the step decided) << 30
  uint32_t ent[MJ_SLOTS];
  uint16_t jobs[MJ_JOBS];           // ring of pair jobs: slot << 1 | pair
  uint16_t ready[MJ_SLOTS], freel[MJ_SLOTS];
};
static_assert(6 * 4 * sizeof(MarchSlots) <= 160 * 1024, "six 4-wave blocks of march slots per CU");

// wave-uniform ring bookkeeping: the lanes with pred get consecutive positions from base
DEV uint32_t lane_rank(bool pred, unsigned long long* m) {
  *m = __ballot(pred);
  return (uint32_t)__popcll(*m & ((1ull << (threadIdx.x & 63u)) - 1ull));
}
DEV void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <uint32_t F, bool STATS, bool ANYQ>
static __global__ __launch_bounds__(256) void k_march_jobs(const DevScene* __restrict__ Sptr, WaveState W,
                                                       Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[ANYQ ? Q_ANY : Q_CLOSEST];
  const uint32_t* q = W.queue[ANYQ ? Q_ANY : Q_CLOSEST];
  __shared__ MarchSlots ms_all[4];
  MarchSlots& M = ms_all[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63u;
  const bling_fractal& fr = S.fractal;
  const int its = fr.iterations;
  const float eps = fr.epsilon;
  WaveFeed feed;
  feed.init(n);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t k = lane; k < MJ_SLOTS; k += 64u) M.freel[k] = (uint16_t)k;
  // wave-uniform ring positions (free slots, jobs, ready rays) and the number of rays in slots
  uint32_t fhead = 0u, ftail = MJ_SLOTS, jhead = 0u, jtail = 0u, rhead = 0u, rtail = 0u, inuse = 0u;
  // the lane's pair job
  bool job = false, da = false, db = false;
  uint32_t jslot = 0u, jpair = 0u;
  int32_t na = 0, nb = 0;
  V3x2 pos, z;
  wave_sync_lds();
  // a bound every wave reaches (no legal march comes near it: the reference's own 100 000-step cap
  // bounds a ray): the grid drains even if the bookkeeping below were ever wrong
  uint32_t guard = 0u;
  // posts the two pair jobs of a ray whose march point p is set (every posting lane calls it with
  // post = true; all lanes call it)
  auto post_jobs = [&](bool post, uint32_t slot) {
    unsigned long long m;
    const uint32_t r = lane_rank(post, &m);
    if (post) { M.jobs[(jtail + 2u * r) % MJ_JOBS] = (uint16_t)(slot << 1); M.jobs[(jtail + 2u * r + 1u) % MJ_JOBS] = (uint16_t)(slot << 1 | 1u); }
    jtail += 2u * (uint32_t)__popcll(m);
  };
  // a ray ends: its result goes out, its slot back to the free list
  auto end_ray = [&](bool end, uint32_t slot, float t) {
    unsigned long long m;
    const uint32_t r = lane_rank(end, &m);
    if (end) { W.march_t[M.ent[slot]] = t; M.freel[(ftail + r) % MJ_SLOTS] = (uint16_t)slot; }
    ftail += (uint32_t)__popcll(m);
    inuse -= (uint32_t)__popcll(m);
  };
  for (;; ++guard) {
    if (guard > (1u << 26)) break;
    // 1. new rays into free slots: the sphere entry, the first march point, its two jobs
    if (feed.cur < feed.end) {                         // queue entries left (WaveFeed::open)
      const uint32_t nfree = ftail - fhead;
      const bool want = lane < nfree;                 // the first nfree lanes may take a query
      uint32_t e = 0u;
      const bool got = feed.take(!want, &e);
      unsigned long long mg;
      const uint32_t rg = lane_rank(got, &mg);
      uint32_t slot = 0u;
      bool post = false, miss = false;
      if (got) {
        slot = M.freel[(fhead + rg) % MJ_SLOTS];
        bool rj;                                        // a rejected ray misses anyway: its march goes unused
        const Ray r = ANYQ ? shadow_ray(W, q[e]) : closest_ray(W, q[e], rj);
        float d0;
        if (mandel_entry(Ray{r.o, r.d, r.tmin, ANYQ ? r.tmax : INFINITY}, &d0)) {
          const V3 rnd = vs(r.d, 1.f / len(r.d));        // MandelMarch2::start
          const V3 p = r.o + vs(rnd, d0);                 // its first iter(): ray_at(rn, d)
          M.o[0][slot] = r.o.x; M.o[1][slot] = r.o.y; M.o[2][slot] = r.o.z;
          M.rn[0][slot] = rnd.x; M.rn[1][slot] = rnd.y; M.rn[2][slot] = rnd.z;
          M.p[0][slot] = p.x; M.p[1][slot] = p.y; M.p[2][slot] = p.z;
          M.d[slot] = d0; M.sd[slot] = 0u; M.ent[slot] = e;
          post = !(sqlen(p) > 2.5f);
          miss = !post;
        } else {
          W.march_t[e] = -1.f;
          miss = true;
          M.ent[slot] = e;
        }
      }
      fhead += (uint32_t)__popcll(mg);
      inuse += (uint32_t)__popcll(mg);
      wave_sync_lds();
      end_ray(miss, slot, -1.f);
      post_jobs(post, slot);
      wave_sync_lds();
    }
    if (inuse == 0u) {
      if (feed.cur >= feed.end) break;
      continue;
    }
    // 2. MJ_K iterations of the lanes' pair jobs; free lanes take queued jobs first
#pragma unroll 1
    for (int u = 0; u < MJ_K; ++u) {
      {
        unsigned long long m;
        const uint32_t r = lane_rank(!job, &m);
        const uint32_t avail = jtail - jhead;
        if (!job && r < avail) {
          const uint32_t jb = M.jobs[(jhead + r) % MJ_JOBS];
          jslot = jb >> 1; jpair = jb & 1u;
          const V3 p = mk(M.p[0][jslot], M.p[1][jslot], M.p[2][jslot]);
          V3 a, b;
          if (jpair == 0u) { a = p; b = p + mk(eps, 0.f, 0.f); }
          else { a = p + mk(0.f, eps, 0.f); b = p + mk(0.f, 0.f, eps); }
          pos = v3x2(a, b); z = pos;
          na = nb = its + 1; da = db = false;
          job = true;
        }
        jhead += min((uint32_t)__popcll(m), avail);
      }
      bool fin = false;
      if (job) {                                        // MandelMarch2::iter, one bulbPower per potential
        if (na == 1) da = true;
        if (nb == 1) db = true;
        if (!(da && db)) {
          tc.ticks += (da ? 0u : 1u) + (db ? 0u : 1u);
          V3x2 zp = bulb_power2(z, fr.order);
          zp.x = zp.x + pos.x; zp.y = zp.y + pos.y; zp.z = zp.z + pos.z;
          const f2v qq = zp.x * zp.x + zp.y * zp.y + zp.z * zp.z;
          const bool ra = !da, rb = !db;
          z.x = f2v{ra ? zp.x.x : z.x.x, rb ? zp.x.y : z.x.y};
          z.y = f2v{ra ? zp.y.x : z.y.x, rb ? zp.y.y : z.y.y};
          z.z = f2v{ra ? zp.z.x : z.z.x, rb ? zp.z.y : z.z.y};
          const bool ea = qq.x > 2.5f, eb = qq.y > 2.5f;
          na -= (ra && !ea) ? 1 : 0;
          nb -= (rb && !eb) ? 1 : 0;
          da = da || ea;
          db = db || eb;
        }
        if (da && db) {                                 // the pair is decided: leave it with its ray
          const uint32_t k0 = 2u * jpair;
          M.zl[k0][jslot] = na == 1 ? 0.f : len(lane0(z)); M.zn[k0][jslot] = (int16_t)na;
          M.zl[k0 + 1][jslot] = nb == 1 ? 0.f : len(lane1(z)); M.zn[k0 + 1][jslot] = (int16_t)nb;
          fin = (atomicAdd(&M.sd[jslot], 1u << 30) >> 30) == 1u;   // the ray's second pair
          job = false;
        }
      }
      {
        unsigned long long m;
        const uint32_t r = lane_rank(fin, &m);
        if (fin) M.ready[(rtail + r) % MJ_SLOTS] = (uint16_t)jslot;
        rtail += (uint32_t)__popcll(m);
      }
      wave_sync_lds();
    }
    // 3. the rest of the DE step for up to 64 ready rays, once MJ_FIN are ready or no job is left
    const uint32_t nready = rtail - rhead;
    const bool jobs_left = (jtail != jhead) || __ballot(job) != 0ull;
    if (nready >= MJ_FIN || (nready > 0u && !jobs_left)) {
      const uint32_t take = min(nready, 64u);
      bool post = false, end = false;
      float tres = -1.f;
      uint32_t slot = 0u;
      if (lane < take) {
        slot = M.ready[(rhead + lane) % MJ_SLOTS];
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {                   // MandelMarch2::finish's potentials
          const int32_t nk = M.zn[k][slot];
          v[k] = nk == 1 ? 0.f : bcr::logf(M.zl[k][slot]) / S.fractal_pw[1 + its - nk];
        }
        float d = M.d[slot];
        const float pot = v[0];
        if (pot == 0.f) { end = true; tres = d; }       // mandelDist = 0 < eps: a hit
        else {
          const V3 g = vs(mk(v[1], v[2], v[3]) - mk(pot, pot, pot), 1.f / eps);
          const float dist = (0.5f / bcr::expf(pot)) * bcr::sinhf(pot) / len(g);
          if (dist < eps) { end = true; tres = d; }
          else {
            d = d + dist;
            const int32_t st = (int32_t)(M.sd[slot] & 0x3FFFFFFFu) + 1;
            if (st >= 100000) { end = true; }             // the next step's start: a miss
            else {
              const V3 o = mk(M.o[0][slot], M.o[1][slot], M.o[2][slot]);
              const V3 rnd = mk(M.rn[0][slot], M.rn[1][slot], M.rn[2][slot]);
              const V3 p = o + vs(rnd, d);
              if (sqlen(p) > 2.5f) end = true;
              else {
                M.p[0][slot] = p.x; M.p[1][slot] = p.y; M.p[2][slot] = p.z;
                M.d[slot] = d; M.sd[slot] = (uint32_t)st;
                post = true;
              }
            }
          }
        }
      }
      rhead += take;
      wave_sync_lds();
      end_ray(end, slot, tres);
      post_jobs(post, slot);
      wave_sync_lds();
    }
  }
  if (STATS) {
    const unsigned long long nk = wave_sum_u64((unsigned long long)tc.ticks);
    if (lane == 0 && nk) {
      atomicAdd(&C->march_ticks, nk);
      if (!ANYQ) atomicAdd(&C->c_march_ticks, nk);
    }
  }
}

// Wave-coherent variants for small scenes (DevScene::pkt_n > 0, dev_trace.h packet_walk): wave w
// takes the 64-entry queue chunks w, w + nw, ... and walks the threaded BVH once per chunk with all
// of its rays.  Same queue, ray and hit records as the per-lane kernels above.
template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_closest_pkt(const DevScene* __restrict__ Sptr, WaveState W,
                                                                 Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = packet_lds(S, smem);
  const PacketRegs P = packet_regs(S);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_CLOSEST];
  const uint32_t* q = W.queue[Q_CLOSEST];
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk * 64u < n; chunk += nw) {
    const uint32_t e = chunk * 64u + (threadIdx.x & 63u);
    const bool live = e < n;
    const uint32_t ent = live ? q[e] : 0u;
    bool rej = false;
    const Ray r = live ? closest_ray(W, ent, rej) : Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f, INFINITY};
    HitRec h{INFINITY, REF_NONE, 0.f, 0.f};
    packet_walk<false, F>(S, L, P, r, live && !rej, h, tc);
    if (live) closest_store(W, ent, h);
  }
  flush_trace_stats<STATS, true>(C, tc);
}

template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_any_pkt(const DevScene* __restrict__ Sptr, WaveState W,
                                                             Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = packet_lds(S, smem);
  const PacketRegs P = packet_regs(S);
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_ANY];
  const uint32_t* q = W.queue[Q_ANY];
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk * 64u < n; chunk += nw) {
    const uint32_t e = chunk * 64u + (threadIdx.x & 63u);
    const bool live = e < n;
    const uint32_t s = live ? q[e] : 0u;
    const Ray r = live ? shadow_ray(W, s) : Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f, 0.f};
    HitRec h{r.tmax, REF_NONE, 0.f, 0.f};
    packet_walk<true, F>(S, L, P, r, live, h, tc);
    if (live) shadow_store(W, s, h.ref != REF_NONE);
  }
  flush_trace_stats<STATS>(C, tc);
}

// Exhaustive variants for scenes of a few dozen primitives (DevScene::bf_tris + bf_shapes > 0,
// dev_trace.h brute_walk): the same chunk loop, queue, ray and hit records as the packet kernels.
template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_closest_bf(const DevScene* __restrict__ Sptr, WaveState W,
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
    bool rej = false;
    const Ray r = live ? closest_ray(W, ent, rej) : Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f, INFINITY};
    HitRec h{INFINITY, REF_NONE, 0.f, 0.f};
    brute_walk<false, F>(S, r, live && !rej, h, tc);
    if (live) closest_store(W, ent, h);
  }
  flush_trace_stats<STATS, true>(C, tc);
}

template <uint32_t F, bool STATS>
static __global__ __launch_bounds__(256) void k_trace_any_bf(const DevScene* __restrict__ Sptr, WaveState W,
                                                            Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_ANY];
  const uint32_t* q = W.queue[Q_ANY];
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  TraceCount tc{0u, 0u, 0u, 0u};
  for (uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk * 64u < n; chunk += nw) {
    const uint32_t e = chunk * 64u + (threadIdx.x & 63u);
    const bool live = e < n;
    const uint32_t s = live ? q[e] : 0u;
    const Ray r = live ? shadow_ray(W, s) : Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f, 0.f};
    HitRec h{r.tmax, REF_NONE, 0.f, 0.f};
    brute_walk<true, F>(S, r, live, h, tc);
    if (live) shadow_store(W, s, h.ref != REF_NONE);
  }
  flush_trace_stats<STATS>(C, tc);
}

// ------------------------------------------------------------------ shading
// Factored candidates.  In a profile whose materials are all matte (one Lambertian or Oren-Nayar
// lobe over a texture spectrum r) and whose lights are all area lights (Li = the light's constant
// radiance), the two candidate spectra of a vertex are
//   light sample:  lsc = ((0 + (r * s1) * s2) * Le) * (w / pdf)     (evalBsdf, sampleLightMis)
//   BSDF sample:   bsc = r * s1                                      (sampleBsdf, sampleBsdfMis)
// and the continuation's throughput is (r * s1 * T) / pc, so k_shade stores scalars (fac, cf) and the
// texture offset (cf.z) instead of three 64-B spectra, and the next launch expands them
// with the same operations in the same order: bit-identical candidates and throughputs.
template <uint32_t F>
constexpr bool factored() { return (F & ~(FT_MATTE | FT_AREA | FT_TRIS)) == 0; }

// In-line shadow test (the cornell profile, DevScene::sh_inline scenes: the whole BVH4, triangles,
// refs and shapes in LDS and a stack bound that fits dev_trace.h's register stack).  The shading
// lane that sets up the light sample's shadow ray tests it itself against the block's LDS copy of
// the tree (occluded_lds) and keeps the answer in the vertex flags (VF_OCC), instead of storing the
// ray (32 B) for k_trace_any, which then does not run, and reading its 4-B answer back.  The answer
// is the same: any-hit is order-free.  The check order of sampleLightMis (lpdf, Li, f, occluded;
// Scene.hs:61-69) is kept: the ray is tested only when the other three passed.  Its query still
// counts as a shadow ray (QF_ANY).
// Measured on MI355X and left out of the product build (BLING_INLINE_SHADOW=1 experiment builds
// only; profiles/r05_ab_session.txt): on C2 the in-line walk cost k_shade as much as the any-hit
// launch it replaces (shade 49.7 -> 58.4 ms per pass, k_trace_any's ~9 ms gone, 9 487 -> 9 516
// Mrays/s) -- the walk runs at k_shade's four waves without lane refill -- and compiling it in
// raised k_shade's scratch (88 -> 136 B) even with the test switched off.
#ifndef BLING_INLINE_SHADOW
#define BLING_INLINE_SHADOW 0
#endif
template <uint32_t F>
constexpr bool inline_shadow() { return BLING_INLINE_SHADOW && F == (FT_MATTE | FT_AREA | FT_TRIS); }

// the factored lobe's spectrum from its byte offset in S.textures (~0u = white)
DEV const float* lobe_r(const DevScene& S, uint32_t off) {
#if defined(BLING_SCENE_LOAD_EXPERIMENT)                              // measurement-only builds
  (void)S; (void)off; return nullptr;
#endif
  return off == ~0u ? nullptr : (const float*)((const char*)gen(S.textures) + off);
}

// sampleOneLight set-up (Scene.hs:61-118): picks the light with 1D dimension dl1, emits the BSDF-MIS
// ray (1D db1 + 2D db2) and the light-sample shadow ray (2D dl2) with their candidate contributions
// into set O at slot o; the next shade launch completes the estimate once both rays are traced.
// m[] is the estimate record being assembled (written by the caller).
template <uint32_t F>
DEV void direct_setup(const DevScene& S, const WaveState& W, const PathSet& O, uint32_t o, const SampleKey& k,
                      const Bsdf& bsdf, V3 wo, V3 p, float eps, int dl1, int dl2, int db1, int db2, uint32_t& vf,
                      bool& app_mis, bool& app_sh, Est& m, uint32_t sid, int dvd = -1, Ray* shr = nullptr) {
  (void)W; (void)sid;
  int lc = S.num_lights;
  if (lc > 0) {
    float lNumU = rnd1(S, k, dl1);
    int ln = lc == 1 ? 0 : min((int)floorf(lNumU * (float)lc), lc - 1);
    const bling_light& Lt = light_rec<F>(S, ln);
    vf |= (uint32_t)ln << 24;
    if constexpr (factored<F>()) {
      const float* r = bsdf.n ? bsdf.b[0].r : nullptr;
      float fm = 0.f, fs1 = 0.f, fs2 = 0.f, wpdf = 0.f;
      {                                                              // sampleBsdfMis (Scene.hs:71-82)
        float lb1, lb2; rnd2(S, k, db2, &lb1, &lb2);
        float s; V3 bwi;
        const float bpdf = sample_bsdf_diffuse1<F>(bsdf, wo, lb1, lb2, s, bwi);
        DVREC3(W, sid, dvd, 18, bwi); DVREC(W, sid, dvd, 21, bpdf);
        if (!(bpdf == 0.f) && !is_black(diffuse1_f(r, s))) {
          const float lpdf = light_pdf<F>(S, Lt, p, bwi);
          m.mdir = make_float4(bwi.x, bwi.y, bwi.z,               // the MIS ray Ray p wi eps infinity
                               kd_flag_w(power_heuristic(bpdf, lpdf), kd_root(S, Ray{p, bwi, eps, INFINITY})));
          fm = s;
          vf |= VF_MIS;
          app_mis = true;
        }
      }
      {                                                              // sampleLightMis (Scene.hs:61-69)
        float ld1, ld2; rnd2(S, k, dl2, &ld1, &ld2);
        LightSample smp = light_sample<F>(S, Lt, p, bsdf.cs.n, eps, ld1, ld2);
        DVREC3(W, sid, dvd, 14, smp.wi); DVREC(W, sid, dvd, 17, smp.pdf);
        float s1, s2;
        if (!(smp.pdf == 0.f) && !is_black(smp.li) && eval_bsdf_diffuse1<F>(bsdf, wo, smp.wi, s1, s2) &&
            !is_black(diffuse1_e(r, s1, s2))) {
          const float w = smp.delta ? 1.f : power_heuristic(smp.pdf, bsdf_pdf<F>(bsdf, wo, smp.wi));
          wpdf = w / smp.pdf; fs1 = s1; fs2 = s2;
          const float stmin = kd_root(S, smp.ray) ? smp.ray.tmin : INFINITY;   // +inf: rejected (kd_root)
          if (shr) { *shr = smp.ray; shr->tmin = stmin; }           // tested by the caller (inline_shadow)
          else {
            O.sh_o[o] = make_float4(smp.ray.o.x, smp.ray.o.y, smp.ray.o.z, stmin);
            O.sh_d[o] = make_float4(smp.ray.d.x, smp.ray.d.y, smp.ray.d.z, smp.ray.tmax);
          }
          vf |= VF_SH;
          app_sh = true;
        }
      }
      m.fac = make_float4(fm, fs1, fs2, wpdf);
      return;
    }
    // BSDF half of estimateDirect: sampleBsdfMis (Scene.hs:71-82)
    {
      float lBc = rnd1(S, k, db1);
      float lb1, lb2; rnd2(S, k, db2, &lb1, &lb2);
      Sp bf; V3 bwi; int bfl;
      float bpdf = sample_bsdf<F>(bsdf, wo, lBc, lb1, lb2, bf, bwi, bfl);
      DVREC3(W, sid, dvd, 18, bwi); DVREC(W, sid, dvd, 21, bpdf);
      if (!(bpdf == 0.f) && !is_black(bf)) {
        float lpdf = light_pdf<F>(S, Lt, p, bwi);
        float w = power_heuristic(bpdf, lpdf);
        // f and w are kept apart: the resolve forms sc w (f * Le) in the reference's order once
        // the MIS ray's hit is known
        store_sp(O.bsc, o, bf);
        m.mdir = make_float4(bwi.x, bwi.y, bwi.z, kd_flag_w(w, kd_root(S, Ray{p, bwi, eps, INFINITY})));
        vf |= VF_MIS;
        app_mis = true;
      }
    }
    // light half: sampleLightMis (Scene.hs:61-69)
    {
      float ld1, ld2; rnd2(S, k, dl2, &ld1, &ld2);
      LightSample smp = light_sample<F>(S, Lt, p, bsdf.cs.n, eps, ld1, ld2);
      DVREC3(W, sid, dvd, 14, smp.wi); DVREC(W, sid, dvd, 17, smp.pdf);
      if (!(smp.pdf == 0.f) && !is_black(smp.li)) {
        float dps[2] = {__builtin_nanf(""), __builtin_nanf("")};    // Blinn powers shared by eval and pdf
        Sp f = eval_bsdf<F>(bsdf, wo, smp.wi, dps);
        if (!is_black(f)) {
          // delta lights (point, directional): sScale (f * li) (1 / lpdf), no MIS weight (Scene.hs:65)
          float w = smp.delta ? 1.f : power_heuristic(smp.pdf, bsdf_pdf<F>(bsdf, wo, smp.wi, dps));
          store_sp(O.lsc, o, sscale(f * smp.li, w / smp.pdf));
          O.sh_o[o] = make_float4(smp.ray.o.x, smp.ray.o.y, smp.ray.o.z, kd_root(S, smp.ray) ? smp.ray.tmin : INFINITY);
          O.sh_d[o] = make_float4(smp.ray.d.x, smp.ray.d.y, smp.ray.d.z, smp.ray.tmax);
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
    LC c = coordinate_system(nn);                                   // mkDg' (DifferentialGeometry.hs:53-56)
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

// L + T (intl + (ls + bs)) of the vertex at slot s of the current set, whose shadow / BSDF-MIS rays
// were just traced (sampleOneLight's completion, Scene.hs:61-118, and Path.hs:73-79's accumulation),
// in the reference's operation order.  m = the slot's estimate record, T0 = the vertex's throughput.
// first: the vertex is the camera path's first (depth 0), whose L = 0 is implicit.
template <uint32_t F>
DEV Sp resolve_L(const DevScene& S, const WaveState& W, uint32_t s, uint32_t vf, const Est& m, const Sp& T0,
                 bool first, uint32_t sid, int dvd, const float4& o) {
  (void)sid;
  int lc = S.num_lights;
  Sp ld = sconst(0.f);
  if (lc > 0) {
    Sp ls = sconst(0.f), bs = sconst(0.f);
    const int ln = vf_light(vf);
    float4 fc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* rf = nullptr;                                        // factored: the lobe's spectrum
    if constexpr (factored<F>()) {
      if (vf & (VF_SH | VF_MIS)) {
        fc = m.fac;
        rf = lobe_r(S, __float_as_uint(m.cf.z));
      }
      if ((vf & VF_SH) && m.occ == 0u)
        ls = sscale(diffuse1_e(rf, fc.y, fc.z) * sload(light_rec<F>(S, ln).radiance), fc.w);
    } else {
      if ((vf & VF_SH) && m.occ == 0u) ls = load_sp(W.cur.lsc, s);
      SBR(W, SB_LSC, 64, (vf & VF_SH) && m.occ == 0u);
    }
    if (vf & VF_SH) DVREC(W, sid, dvd, 28, m.occ ? 1.f : 0.f);
    if (vf & VF_MIS) {                                                // sampleBsdfMis (Scene.hs:71-82)
      const bling_light& Lt = light_rec<F>(S, ln);
      const uint32_t ref = __float_as_uint(m.mhit.y);
      const float4 d = m.mdir;
      V3 wi = mk(d.x, d.y, d.z);
      DVREC(W, sid, dvd, 29, ref == REF_NONE ? INFINITY : m.mhit.x);
      if (ref == REF_NONE) {
        const Sp bf = factored<F>() ? diffuse1_f(rf, fc.x) : load_sp(W.cur.bsc, s);
        SBR(W, SB_BSC, 64, !factored<F>());
        bs = sscale(bf * light_le<F>(Lt, wi), fabsf(d.w));           // le l ray (w: the kd_root flag's sign)
      } else if ((ref >> 30) == REF_SHAPE) {
        const DevShape& hs = gen(S.shapes[ref & 0x3FFFFFFFu]);
        SBR(W, SB_BSC, 64, !factored<F>() && hs.light == ln);
        if (hs.light == ln) {                                         // l' == l (Light.hs:48-50)
          DG dg = shape_dg<F>(hs, Ray{mk(o.x, o.y, o.z), wi, o.w, INFINITY}, m.mhit.x);
          Sp le = dot(dg.n, -wi) > 0.f ? sload(gen(S.lights[ln]).radiance) : sconst(0.f);   // intLe (-wi): trap T6
          const Sp bf = factored<F>() ? diffuse1_f(rf, fc.x) : load_sp(W.cur.bsc, s);
          bs = sscale(bf * le, fabsf(d.w));
        }
      }
    }
    ld = ls + bs;
    if (lc > 1) ld = sscale(ld, (float)lc);
  }
  const int il = vf_intl(vf);
  Sp lhere = (il >= 0 ? sload(light_rec<F>(S, il).radiance) : sconst(0.f)) + ld;
  const Sp L0 = first ? sconst(0.f) : load_sp(W.cur.L, s);
#if BLING_DEBUG_VERTEX
  {
    const Sp Lr = L0 + T0 * lhere;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < 16; ++q) { a += lhere.v[q]; b += Lr.v[q]; }
    DVREC(W, sid, dvd, 30, a); DVREC(W, sid, dvd, 31, b);
  }
#endif
  return L0 + T0 * lhere;
}

// The throughput of the vertex a continuation ray of slot s leads to, from the throughput Tv of the
// vertex that sampled it (Path.hs:82: t' = f t / pc).  The shading launch stores f and pc, not t':
// factored profiles the factors of f = r s1 (cf.x, texture offset cf.z) and pc in cf.y; the others
// the spectrum f (Tn) and pc in the continuation direction's w.  The next launch, which holds Tv
// anyway, forms t' with the same operations, so the shading phase needs only sY(T) (the RR bound)
// instead of the 16-band throughput.
template <uint32_t F>
DEV Sp next_throughput(const DevScene& S, const PathSet& P, uint32_t s, const float4 cf, const Sp& Tv, float pc) {
  if constexpr (factored<F>()) {
    (void)pc;
    const Sp f = diffuse1_f(lobe_r(S, __float_as_uint(cf.z)), cf.x);
    return sscale(f * Tv, 1.f / cf.y);
  } else {
    (void)cf;
    return sscale(load_sp(P.Tn, s) * Tv, 1.f / pc);
  }
}

// Vertex d of a path (Path.hs:68-87 with sampleOneLight's set-up) once its continuation ray hit
// something below maxDepth: hit reconstruction, BSDF, the one-light estimate's two rays and
// candidates, Russian roulette and the continuation.  Writes the vertex to slot o of the output set
// O.  ty = sY of the vertex's throughput (Russian roulette's bound; read only beyond depth 7).
// Returns the queue-membership bits of the vertex (QF_*).
template <uint32_t F>
DEV uint32_t shade_vertex(const DevScene& S, const WaveState& W, const PathSet& O, uint32_t o, int depth, uint32_t seed,
                          uint32_t pass, float ty, uint32_t vfin, float4 hv, const Ray& ray, uint32_t pix,
                          uint32_t nid, uint32_t sid, const LdsScene* Lsh = nullptr) {
  const bool spec = (vfin & VF_SPEC) != 0;
  bool app_sh = false, app_mis = false, app_cont = false;
  SampleKey k = sample_key(seed, pass, pix, nid);
  DG dgg, dgs;
  float eps;
  int mat, hit_light;
  hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
  DVREC3(W, sid, depth, 0, ray.o); DVREC3(W, sid, depth, 3, ray.d); DVREC(W, sid, depth, 6, hv.x);
  DVREC3(W, sid, depth, 10, dgg.n); DVREC(W, sid, depth, 13, eps);
  int intl_light = (spec && hit_light >= 0 && dot(dgg.n, ray.d) > 0.f) ? hit_light : -1;   // intLe rd (trap T6)
  float ttmp[(F & FT_PROCTEX) ? 32 : 1];  // computed spectra of the BSDF (FT_PROCTEX profiles)
  Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs, ttmp);
  V3 wo = -ray.d;
  V3 p = bsdf.p;
  DVREC3(W, sid, depth, 7, p);
  uint32_t vf = vf_make(intl_light, 0);
  Est m;
  m.mdir = make_float4(0.f, 0.f, 0.f, 0.f);
  m.fac = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* r = (factored<F>() && bsdf.n) ? bsdf.b[0].r : nullptr;
  const uint32_t rtex = r ? (uint32_t)((const char*)r - (const char*)gen(S.textures)) : ~0u;
  // Russian roulette + continuation (Path.hs:68-87)
  float pc = depth <= 7 ? 1.f : hmin(0.75f, ty);
  float x = rnd1(S, k, 3 + 4 * depth);
  DVREC(W, sid, depth, 26, pc); DVREC(W, sid, depth, 27, x);
  bool cont = !(x > pc);
  float s1c = 0.f;
  V3 cwi = mk(0.f, 0.f, 0.f);
  if (cont) {
    float uc = rnd1(S, k, 0 + 4 * depth);
    float ud1, ud2; rnd2(S, k, 0 + 3 * depth, &ud1, &ud2);
    int cfl = F_REFL | F_DIFF;
    float cpdf;
    if constexpr (factored<F>()) {
      (void)uc;
      cpdf = sample_bsdf_diffuse1<F>(bsdf, wo, ud1, ud2, s1c, cwi);   // one diffuse lobe: f = r s1
      cont = !(cpdf == 0.f || is_black(diffuse1_f(r, s1c)));
    } else {
      Sp cf;
      cpdf = sample_bsdf<F>(bsdf, wo, uc, ud1, ud2, cf, cwi, cfl);
      cont = !(cpdf == 0.f || is_black(cf));
      if (cont) store_sp(O.Tn, o, cf);                                // t' = (f t) / pc: next launch
      SBW(W, SB_TN, 64, cont);
    }
    DVREC3(W, sid, depth, 22, cwi); DVREC(W, sid, depth, 25, cpdf);
    if (cont) {
      if ((cfl & F_SPEC) == F_SPEC) vf |= VF_SPEC;
      app_cont = true;
    }
  }
  if (!cont) vf |= VF_TERM;
  // the continuation is written before the one-light estimate is set up, so none of its state is
  // live across that (the sample dimensions are independent draws: the order changes no value)
  if constexpr (factored<F>()) O.cf[o] = make_float4(s1c, pc, __uint_as_float(rtex), 0.f);
  O.org[o] = make_float4(p.x, p.y, p.z, eps);
  // the continuation ray Ray p wi eps infinity (Path.hs:79) with its kd_root flag (dev_trace.h)
  O.dir[o] = make_float4(cwi.x, cwi.y, cwi.z, kd_flag_w(pc, !cont || kd_root(S, Ray{p, cwi, eps, INFINITY})));
  Ray shr{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f, 0.f};
  direct_setup<F>(S, W, O, o, k, bsdf, wo, p, eps, 1 + 4 * depth, 1 + 3 * depth, 2 + 4 * depth, 2 + 3 * depth, vf,
                  app_mis, app_sh, m, sid, depth, Lsh ? &shr : nullptr);
  O.mdir[o] = m.mdir;
  if constexpr (factored<F>()) O.fac[o] = m.fac;
  if constexpr (inline_shadow<F>()) {
    if (Lsh && app_sh && occluded_lds<F>(S, *Lsh, shr)) vf |= VF_OCC;      // sampleLightMis's `occluded`
  }
  O.meta[o] = make_uint4(vf, pix, nid, sid);
  // what the next launches need of the vertex: cf (factored: the continuation's factors and the
  // lobe offset the candidates use), the origin of the continuation / MIS rays, the continuation
  // direction and pc, the MIS direction and weight, the candidates' scalars, the metadata; the
  // shadow ray and, in the spectral profiles, the candidate spectra
  SBW(W, SB_CF, 16, factored<F>() && (app_cont || app_sh || app_mis));
  SBW(W, SB_ORG, 16, app_cont || app_mis);
  SBW(W, SB_DIR, 16, app_cont);
  SBW(W, SB_MDIR, 16, app_mis);
  SBW(W, SB_FAC, 16, factored<F>() && (app_sh || app_mis));
  SBW(W, SB_META, 16, true);
  SBW(W, SB_SHO, 16, app_sh && !Lsh);
  SBW(W, SB_SHD, 16, app_sh && !Lsh);
  SBW(W, SB_LSC, 64, !factored<F>() && app_sh);
  SBW(W, SB_BSC, 64, !factored<F>() && app_mis);
  return QF_RESOLVE | (app_sh ? QF_ANY : 0u) | (app_mis ? QF_MIS : 0u) | (app_cont ? QF_CONT : 0u);
}

// A path whose continuation ray of depth d missed, or that reached maxDepth: Le of the escaped ray
// after a specular bounce (Path.hs:80), then the sample is done (Path.hs:83, 87).
template <uint32_t F>
DEV void shade_end(const DevScene& S, const WaveState& W, uint32_t sid, const Sp& T, bool spec_miss, V3 rd, Sp L,
                   unsigned long long& n_drop) {
  if (spec_miss) {
    Sp sum = sconst(0.f);
#if !defined(BLING_SKY_COST_EXPERIMENT)        // measurement-only builds: what the escaped rays' Le costs
    for (int l = 0; l < S.num_lights; ++l) sum = sum + light_le<F>(gen(S.lights[l]), rd);
#endif
    L = L + T * sum;
  }
  finalize(W, sid, L, n_drop);
}

// Path vertex d over a queue of slots of the current set.  FUSED = false (d = 0): the queue holds
// the camera paths.  FUSED = true (d >= 1): the queue holds every path that had a vertex at d - 1
// (the compaction's resolve list); the kernel first resolves that vertex, then -- unless the path
// stopped there -- shades vertex d with the resolved L.  One launch instead of a resolve and a shade
// launch: their independent path loads are in flight together.  The vertices shaded from a 64-entry
// chunk of the queue are written to the first slots of that chunk in the next set (W.nxt).
//
// Wave compaction: a wave takes 64 consecutive queue entries, resolves them and ends every path that
// stops here (terminated at d - 1, missed, or at maxDepth) in place; the paths that get a vertex at
// d go into a per-wave ring of 128 (slot, entry) pairs in LDS, and the wave shades 64 of them at
// once whenever the ring holds 64.  Escaping / terminating paths no longer idle the lanes of the
// shading code (round 2, C4 measured 0.30 VALU lane utilisation in the fused shade without it).
// The shading order of paths changes, their arithmetic does not; qflag stays indexed by queue entry,
// so the compacted queues keep their order.
constexpr uint32_t SHADE_RING = 128;
template <uint32_t F, bool FUSED>
static __global__ __launch_bounds__(256) SHADE_OCC void k_shade(const DevScene* __restrict__ Sptr, WaveState W, int depth, int qin,
                                               uint32_t seed, uint32_t pass, Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[qin];
  const uint32_t* q = W.queue[qin];
  unsigned long long n_drop = 0;
  // in-line shadow test: the block's LDS copy of the whole BVH4 (dynamic LDS behind the ring)
  LdsScene Lsh{nullptr, 0u, nullptr, 0u, nullptr, nullptr, 0u, nullptr, nullptr, 0u};
  bool inl = false;
  if constexpr (inline_shadow<F>()) {
    extern __shared__ float4 smem[];
    inl = S.sh_inline != 0u;
    if (inl) Lsh = lds_setup<true, false, true>(S, smem);
  }
  // the ring hands a vertex's slot, entry, hit and metadata records and sY(T) from the resolve phase
  // to the shading lane, so the shading phase loads only the ray (org, dir) from the path set
  __shared__ uint32_t ring_e[4][SHADE_RING];
  __shared__ float ring_y[4][SHADE_RING];
  __shared__ float4 ring_h[4][SHADE_RING];
  __shared__ uint4 ring_m[4][SHADE_RING];
  __shared__ float4 ring_o[4][SHADE_RING], ring_d[4][SHADE_RING];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  uint32_t head = 0u, cnt = 0u;                                         // wave-uniform ring state
  auto shade_from_ring = [&](uint32_t slot) __attribute__((always_inline)) {
    const uint32_t e = ring_e[wv][slot];
    const float4 ro = ring_o[wv][slot], rdv = ring_d[wv][slot];
    const float4 hv = ring_h[wv][slot];
    const uint4 meta = ring_m[wv][slot];
    const Ray ray{mk(ro.x, ro.y, ro.z), mk(rdv.x, rdv.y, rdv.z), ro.w, INFINITY};
    W.qflag[e] = (uint8_t)shade_vertex<F>(S, W, W.nxt, e, depth, seed, pass, ring_y[wv][slot], meta.x, hv, ray, meta.y,
                                          meta.z, meta.w, inl ? &Lsh : nullptr);
  };
  // the next chunk's queue entry is loaded one iteration ahead (its latency overlaps this chunk)
  uint32_t qnext = 0u;
  {
    const uint32_t e0 = (blockIdx.x * (blockDim.x >> 6) + wv) * 64u + lane;
    if (e0 < n) qnext = q[e0];
  }
  // One call site of the shading code (a second one, for the ring's tail, made the compiler outline
  // it as a function in the largest profiles: a call with its register saves and stack frame).
  uint32_t base = (blockIdx.x * (blockDim.x >> 6) + wv) * 64u;
  for (;;) {
    const bool more = base < n;                                         // wave-uniform
    if (more) {
      const uint32_t e = base + lane;
      const uint32_t qcur = qnext;
      if (e + nwaves * 64u < n) qnext = q[e + nwaves * 64u];
      bool vert = false;
      uint32_t s = 0u;
      float ty = 0.f;
      float4 hv = make_float4(0.f, 0.f, 0.f, 0.f), ro = hv, rdv = hv;
      uint4 meta = make_uint4(0u, 0u, 0u, 0u);
      if (e < n) {
        s = qcur;
        // every record of the slot is loaded at once (no load waits on another's value): hit,
        // metadata, the ray of the vertex (the ring hands it to the shading lane) and the estimate
        hv = W.cur.hit[s];
        meta = W.cur.meta[s];
        ro = W.cur.org[s];
        rdv = W.cur.dir[s];
        // the path gets a vertex at d unless it stopped at d - 1, missed, or is at maxDepth
        vert = !(FUSED && (meta.x & VF_TERM)) && __float_as_uint(hv.y) != REF_NONE && depth != S.max_depth;
      }
      // Dense output slots: the chunk's k new vertices take slots base .. base + k - 1 of the next set
      // in lane order (their entries' order, so the compacted queues keep the same order), and the
      // chunk's other slots get an empty flag.  The next launches then gather a dense prefix of every
      // 64-slot chunk instead of the entries of the vertices that survived.  Slots are addresses
      // only; no value depends on them.
      const unsigned long long msk = __ballot(vert);
      const uint32_t nv = (uint32_t)__popcll(msk);
      const uint32_t o = base + (uint32_t)__popcll(msk & below);
      if (e < n) {
        if (lane >= nv) W.qflag[base + lane] = 0u;
        Sp L = sconst(0.f);
        bool ends = false;
        Est m;
        m.cf = make_float4(0.f, 0.f, 0.f, 0.f);
        Sp Tp = sconst(1.f);                                                  // T(d - 1)
        if constexpr (FUSED) {
#if defined(BLING_LAZY_EST)                                           // experiment builds only
          m = load_est(W.cur, s, meta.x, factored<F>());
#else
          m = load_est_eager(W.cur, s, factored<F>(), !inl);
#endif
          if (inl) m.occ = (meta.x & VF_OCC) ? 1u : 0u;                  // tested in line at d - 1
          if (depth > 1) Tp = load_sp(W.cur.T, s);
          L = resolve_L<F>(S, W, s, meta.x, m, Tp, depth == 1, meta.w, depth - 1, ro);
          SBR(W, SB_MDIR, 16, (meta.x & VF_MIS) != 0u);
          SBR(W, SB_MHIT, 8, (meta.x & VF_MIS) != 0u);
          SBR(W, SB_OCC, 4, !inl && (meta.x & VF_SH) != 0u);
          SBR(W, SB_FAC, 16, factored<F>() && (meta.x & (VF_SH | VF_MIS)) != 0u);
          SBR(W, SB_T, 64, depth > 1);
          SBR(W, SB_L, 64, depth > 1);
          if (meta.x & VF_TERM) { finalize(W, meta.w, L, n_drop); ends = true; }   // the path stopped at d - 1
        }
        if (!ends) {
          const uint32_t ref = __float_as_uint(hv.y);
          const bool spec_miss = ref == REF_NONE && (meta.x & VF_SPEC) != 0;
          const bool hit = ref != REF_NONE && depth != S.max_depth;          // == vert here
          // T(d): 1 for the camera path (depth 0), else formed from T(d - 1) and the stored f, pc
          Sp Td = sconst(1.f);
          if (FUSED && (hit || spec_miss)) Td = next_throughput<F>(S, W.cur, s, m.cf, Tp, fabsf(rdv.w));
          SBR(W, SB_TN, 64, FUSED && !factored<F>() && (hit || spec_miss));
          SBR(W, SB_CF, 16, FUSED && factored<F>() && ((hit || spec_miss) || (meta.x & (VF_SH | VF_MIS)) != 0u));
          // the vertex's ray: shading needs org and dir, a specular miss dir, T' of a spectral
          // profile dir.w (pc); the resolve needs org for a BSDF-MIS ray that hit the sampled light
          SBR(W, SB_DIR, 16, hit || spec_miss);
          SBR(W, SB_ORG, 16, hit || (FUSED && (meta.x & VF_MIS) != 0u && __float_as_uint(m.mhit.y) != REF_NONE &&
                                     (__float_as_uint(m.mhit.y) >> 30) == REF_SHAPE));
          SBW(W, SB_L, 64, FUSED && hit);
          SBW(W, SB_T, 64, FUSED && hit);
          if (hit) {
            if constexpr (FUSED) {
              store_sp(W.nxt.L, o, L);
              store_sp(W.nxt.T, o, Td);                                      // T(d), for the resolve of d
            }
            if (depth > 7) ty = sY(Td);                                      // Russian roulette's bound
          } else {
            shade_end<F>(S, W, meta.w, Td, spec_miss, mk(rdv.x, rdv.y, rdv.z), L, n_drop);
          }
        }
        SBR(W, SB_QUEUE, 4, true);
        SBR(W, SB_HIT, 16, true);
        SBR(W, SB_META, 16, true);
        SBW(W, SB_QFLAG, 1, true);
      }
      if (vert) {
        const uint32_t slot = (head + cnt + (uint32_t)__popcll(msk & below)) & (SHADE_RING - 1u);
        ring_e[wv][slot] = o; ring_y[wv][slot] = ty;
        ring_h[wv][slot] = hv; ring_m[wv][slot] = meta;
        ring_o[wv][slot] = ro; ring_d[wv][slot] = rdv;
      }
      cnt += (uint32_t)__popcll(msk);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      base += nwaves * 64u;
    }
    // a full wave of vertices, or the rest of the ring once the queue is done (cnt < 64 then)
    if (cnt >= 64u || (!more && cnt > 0u)) {
      const uint32_t take = cnt < 64u ? cnt : 64u;
      if (lane < take) shade_from_ring((head + lane) & (SHADE_RING - 1u));
      head = (head + take) & (SHADE_RING - 1u);
      cnt -= take;
    }
    if (!more && cnt == 0u) break;
  }
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ DirectLighting vertex
// directLighting / cont (Integrator/DirectLighting.hs:22-57) as a depth-first walk of each sample's
// ray tree with one ray in flight: a hit node emits the one-light estimate (dimensions 2d, 2d + 1)
// plus Le towards wo through k_resolve with its weight T, then continues into its specular
// reflection child and parks the transmission child in slot d + 1; a node without children (or a
// miss, which adds black) resumes the deepest parked sibling.  Depth is per path (vf bits 4-8).
// Runs in place: one set, slot = sample id.
template <uint32_t F>
static __global__ __launch_bounds__(256) SHADE_OCC void k_shade_dl(const DevScene* __restrict__ Sptr, WaveState W, int qin, uint32_t seed,
                                                  uint32_t pass, Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[qin];
  const uint32_t* q = W.queue[qin];
  unsigned long long n_drop = 0;
  const size_t cap = W.cap;
  const PathSet& P = W.cur;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint32_t i = q[e];
    const uint4 meta = P.meta[i];
    const int d = (int)vf_depth(meta.x);
    const float4 hv = P.hit[i], ro = W.corg[i], rdv = P.dir[i];
    const Ray ray{mk(ro.x, ro.y, ro.z), mk(rdv.x, rdv.y, rdv.z), ro.w, INFINITY};
    const bool hit = __float_as_uint(hv.y) != REF_NONE;
    bool app_sh = false, app_mis = false, next = false;
    uint32_t mask = W.dl_mask[i], vf = 0u;
    float4 no = ro, nd = rdv;
    int nlev = 0;
    if (hit) {
      const Sp T = load_sp(P.T, i);
      SampleKey k = sample_key(seed, pass, meta.y, meta.z);
      DG dgg, dgs;
      float eps;
      int mat, hit_light;
      hit_geometry<F>(S, ray, hv, dgg, dgs, eps, mat, hit_light);
      const V3 wo = -ray.d;
      const int intl = (hit_light >= 0 && dot(dgg.n, wo) > 0.f) ? hit_light : -1;     // intLe int wo
      float ttmp[(F & FT_PROCTEX) ? 32 : 1];  // computed spectra of the BSDF (FT_PROCTEX profiles)
      Bsdf bsdf = make_bsdf<F>(S, mat, dgg, dgs, ttmp);
      const V3 p = bsdf.p;
      vf = vf_make(intl, 0);
      Est m;
      m.mdir = make_float4(0.f, 0.f, 0.f, 0.f);
      m.fac = make_float4(0.f, 0.f, 0.f, 0.f);
      const float* lr = (factored<F>() && bsdf.n) ? bsdf.b[0].r : nullptr;
      const uint32_t rtex = lr ? (uint32_t)((const char*)lr - (const char*)gen(S.textures)) : ~0u;
      direct_setup<F>(S, W, P, i, k, bsdf, wo, p, eps, 2 * d, 2 * d, 1 + 2 * d, 1 + 2 * d, vf, app_mis, app_sh, m, i);
      P.mdir[i] = m.mdir;
      if constexpr (factored<F>()) { P.fac[i] = m.fac; P.cf[i] = make_float4(0.f, 1.f, __uint_as_float(rtex), 0.f); }
      if (d + 1 != S.max_depth) {                                          // cont: d == md -> black
        Sp fr, ft; V3 wr, wt;
        const bool hr = !(sample_bsdf_spec<F>(bsdf, wo, F_REFL, fr, wr) == 0.f);
        const bool ht = !(sample_bsdf_spec<F>(bsdf, wo, F_TRANS, ft, wt) == 0.f);
        const float4 po = make_float4(p.x, p.y, p.z, eps);
        if (hr) {
          next = true; no = po; nd = make_float4(wr.x, wr.y, wr.z, 0.f); nlev = d + 1;
          store_sp(P.Tn, i, fr * T);
        }
        if (ht) {
          if (hr) {                                                        // park the sibling
            const size_t slot = (size_t)(d + 1) * cap + i;
            W.dl_org[slot] = po;
            W.dl_dir[slot] = make_float4(wt.x, wt.y, wt.z, 0.f);
            store_sp(W.dl_T + 4 * (size_t)(d + 1) * cap, i, ft * T);
            mask |= 1u << (d + 1);
          } else {
            next = true; no = po; nd = make_float4(wt.x, wt.y, wt.z, 0.f); nlev = d + 1;
            store_sp(P.Tn, i, ft * T);
          }
        }
      }
      P.org[i] = make_float4(p.x, p.y, p.z, eps);
    }
    if (!next && mask != 0u) {                                             // resume the deepest sibling
      const int j = 31 - __clz(mask);
      const size_t slot = (size_t)j * cap + i;
      mask &= ~(1u << j);
      next = true; no = W.dl_org[slot]; nd = W.dl_dir[slot]; nlev = j;
      store_sp(P.Tn, i, load_sp(W.dl_T + 4 * (size_t)j * cap, i));
    }
    W.dl_mask[i] = mask;
    if (next) {
      W.corg[i] = no;
      nd.w = kd_flag_w(0.f, kd_root(S, Ray{mk(no.x, no.y, no.z), mk(nd.x, nd.y, nd.z), no.w, INFINITY}));
      P.dir[i] = nd;
    } else if (!hit) {
      finalize(W, i, load_sp(P.L, i), n_drop);
    }
    // k_resolve finalises on TERM; the depth bits carry the next ray's level
    P.meta[i] = make_uint4((hit ? (vf | (next ? 0u : VF_TERM)) : 0u) | vf_make(-1, nlev), meta.y, meta.z, meta.w);
    W.qflag[e] = (uint8_t)((hit ? QF_RESOLVE : 0u) | (app_sh ? QF_ANY : 0u) | (app_mis ? QF_MIS : 0u) |
                           (next ? QF_CONT : 0u));
  }
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ resolve (DirectLighting)
// in place, slot = sample id: L += T (Le + one-light estimate); finalise on TERM
template <uint32_t F>
static __global__ __launch_bounds__(256) void k_resolve(const DevScene* __restrict__ Sptr, WaveState W,
                                                 Counters* __restrict__ C) {
  const DevScene& S = *Sptr;
  const uint32_t n = *(volatile uint32_t*)&W.qcount[Q_RESOLVE];
  const uint32_t* q = W.queue[Q_RESOLVE];
  unsigned long long n_drop = 0;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const uint32_t i = q[e];
    const uint32_t vf = W.cur.meta[i].x;
    const Est m = load_est(W.cur, i, vf, factored<F>());
    const Sp L = resolve_L<F>(S, W, i, vf, m, load_sp(W.cur.T, i), false, i, -1, W.cur.org[i]);
    if (vf & VF_TERM) finalize(W, i, L, n_drop);
    else store_sp(W.cur.L, i, L);
  }
  flush_dropped(C, n_drop);
}

// ------------------------------------------------------------------ camera rays
struct TileDesc { int x0, x1, y0, y1; uint32_t offset, count; };

// camera sample i (raygen order = sample id = slot of the current set)
DEV void init_path(const DevScene& S, const WaveState& W, uint32_t i, int ix, int iy, uint32_t n, uint32_t seed,
                   uint32_t pass) {
  uint32_t pixel = (uint32_t)((iy - S.ey0) * S.ext_w + (ix - S.ex0));
  SampleKey k = sample_key(seed, pass, pixel, n);
  float ox, oy, lu, lv;
  camera_sample(S, k, &ox, &oy, &lu, &lv);
  float imx = (float)ix + ox, imy = (float)iy + oy;
  Ray r = fire_ray(S.camera, imx, imy, lu, lv);
  const float4 ro = make_float4(r.o.x, r.o.y, r.o.z, r.tmin);
  W.cur.org[i] = ro;
  W.cur.dir[i] = make_float4(r.d.x, r.d.y, r.d.z, kd_flag_w(0.f, kd_root(S, r)));   // kd_root flag (dev_trace.h)
  W.cur.meta[i] = make_uint4(VF_SPEC, pixel, n, i);                     // the camera "bounce" is specular (Path.hs:38)
  if (W.dl_mask) {
    // DirectLighting keeps T and L in its one set (the Path pipeline takes the camera path's T = 1
    // and L = 0 as constants)
    W.dl_mask[i] = 0u;
    W.corg[i] = ro;
    store_sp(W.cur.T, i, sconst(1.f));
    store_sp(W.cur.L, i, sconst(0.f));
  }
  W.img[i] = make_float2(imx, imy);
  W.result[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  W.queue[Q_SHADE0][i] = i;
  W.queue[Q_CLOSEST][i] = (i << 1) | ENTRY_CONT;
}

// Slot order of a tile's camera samples (DevScene::sample_major).  Pixel-major (slot = pixel x spp
// + n) puts one pixel's samples side by side, so the first bounce of a wave traces 64 samples of one
// pixel; sample-major (slot = n x pixels + pixel) puts a tile's pixels side by side, so the film
// gather's per-pixel sample loop reads consecutive slots across the lanes of a wave (coalesced)
// instead of one line per lane.  Each path's arithmetic and each pixel's summation order are the
// same in both.  Measured on MI355X (profiles/r04_ab_session.txt r04x): C4 +1.6 %, C2 +0.3 %, C3
// -2.7 % (the per-lane traversal of the meshes loses first-bounce coherence), so the host picks
// sample-major for the scenes that walk the packet kernels (core.hip upload).
static __global__ __launch_bounds__(256) void k_raygen(const DevScene* __restrict__ Sptr, WaveState W,
                                                const TileDesc* __restrict__ tiles, uint32_t seed, uint32_t pass) {
  const DevScene& S = *Sptr;
  const TileDesc td = tiles[blockIdx.y];
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= td.count) return;
  int tw = td.x1 - td.x0 + 1;
  uint32_t pt, n;
  if (S.sample_major) {
    const uint32_t npix = (uint32_t)(tw * (td.y1 - td.y0 + 1));
    n = j / npix; pt = j - n * npix;
  } else {
    pt = S.fd_spp.div(j); n = j - pt * (uint32_t)S.spp;
  }
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
// Path (fused) mode: the shade input is the resolve list of d - 1, and the scan left the number of
// paths alive at d (continuation rays) in the Q_RESOLVE counter.
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
    // Path (fused): the next queues list the entries themselves -- the shade launch wrote each
    // vertex to slot e of the next set; DirectLighting (in place): the sample ids
    if (e < n) { f = W.qflag[e]; i = fused ? e : qi[e]; }
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
// The end of a film kernel: the block's tile image (LDS, FILM_TILE_MAX stride) is either added into
// the film (addTile, Image.hs:178-199), or -- tile-image mode (tiles != NULL, BLING_PASS_TILE_IMAGES)
// -- written whole, zero-padded, into the block's slot of sw x sh x 4 floats, so a multi-rank pass
// can gather the compact tile images and add them on one device (k_add_tiles).
DEV void film_flush(const DevScene& S, const float* img, int ox, int oy, int w, int h, float* __restrict__ film,
                    float* __restrict__ tiles, int sw, int sh) {
  if (tiles) {
    float4* slot = reinterpret_cast<float4*>(tiles) + (size_t)blockIdx.x * sw * sh;
    for (int q = threadIdx.x; q < sw * sh; q += blockDim.x) {
      const int x = q % sw, y = q / sw;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (x < w && y < h && x + ox < S.width && y + oy < S.height)
        v = *reinterpret_cast<const float4*>(&img[4 * (x + y * FILM_TILE_MAX)]);
      slot[q] = v;
    }
    return;
  }
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

static __global__ __launch_bounds__(256) void k_film(const DevScene* __restrict__ Sptr, WaveState W,
                                              const TileDesc* __restrict__ tiles, float* __restrict__ film,
                                              float* __restrict__ timg, int sw, int sh) {
  __shared__ __attribute__((aligned(16))) float img[FILM_TILE_MAX * FILM_TILE_MAX * 4];
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
  film_flush(S, img, ox, oy, w, h, film, timg, sw, sh);
}

// Register-accumulating film splat: thread t owns source pixel t of the tile and sums the filtered
// contributions of all its samples to the K x K window of output pixels around it in registers
// (K = 2 * floor(0.5 + fw) + 1: 5 for the width-2 filters of C1/C2/C4/C5, 7 for C3's width 3), then
// adds the window into the tile image in LDS once.  Same pixel ranges, table lookups and tile
// clipping as k_film (addSample, Image.hs:250-299); ~K*K*4 LDS atomics per source pixel instead of
// ~K*K*4 per sample.
// Round 6: for K = 5, two threads per source pixel (blocks of 512), each owning a band of the
// window's rows (0-2 / 3-4): 150 -> 106 VGPRs, four waves per SIMD instead of three, with twice the
// threads walking samples.  Each thread reads its pixel's samples and does its rows' arithmetic
// exactly as before; a window pixel's sum over one source pixel's samples is still formed in sample
// order by one thread.  K = 7 keeps one thread per pixel: split, it needs 166 VGPRs, three waves,
// which a 512-thread block (two waves per SIMD) cannot fill.
#ifndef BLING_FILM_SPLIT5
#define BLING_FILM_SPLIT5 2
#endif
template <int K>
constexpr int film_split() { return K <= 5 ? BLING_FILM_SPLIT5 : 1; }
template <int K>
static __global__ __launch_bounds__(256 * film_split<K>()) void k_film_gather(const DevScene* __restrict__ Sptr, WaveState W,
                                                     const TileDesc* __restrict__ tiles, float* __restrict__ film,
                                                     float* __restrict__ timg, int sw, int sh) {
  __shared__ __attribute__((aligned(16))) float img[FILM_TILE_MAX * FILM_TILE_MAX * 4];
  __shared__ float tbl[256];
  constexpr int R = K / 2;
  constexpr int KB = (K + film_split<K>() - 1) / film_split<K>();   // window rows per thread
  const DevScene& S = *Sptr;
  const TileDesc td = tiles[blockIdx.x];
  const float fw = S.filter_w, fh = S.filter_h;
  const int ox = max(0, td.x0), oy = max(0, td.y0);
  const int w = td.x1 - ox + (int)floorf(0.5f + fw), h = td.y1 - oy + (int)floorf(0.5f + fh);
  for (int q = threadIdx.x; q < FILM_TILE_MAX * FILM_TILE_MAX * 4; q += blockDim.x) img[q] = 0.f;
  if (threadIdx.x < 256) tbl[threadIdx.x] = S.filter_table[threadIdx.x];
  __syncthreads();
  const float ifw = 1.f / fw, ifh = 1.f / fw;                            // trap T12
  const int tw = td.x1 - td.x0 + 1, npix = tw * (td.y1 - td.y0 + 1);
  const uint32_t spp = (uint32_t)S.spp;
  const int pt = threadIdx.x & 255;
  const int b0 = (int)(threadIdx.x >> 8) * KB;                        // this thread's first window row
  if (pt < npix) {
    const int ix = td.x0 + pt % tw, iy = td.y0 + pt / tw;
    float acc[KB][K][4];
#pragma unroll
    for (int b = 0; b < KB; ++b)
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[b][a][c] = 0.f;
    // slot of sample n of this pixel: base + n x stride (k_raygen's order)
    const uint32_t base = td.offset + (S.sample_major ? (uint32_t)pt : (uint32_t)pt * spp);
    const uint32_t stride = S.sample_major ? (uint32_t)npix : 1u;
    // the next sample's records are loaded one iteration ahead: their latency overlaps this
    // sample's window arithmetic
    float4 rn = W.result[base];
    float2 imn = W.img[base];
    for (uint32_t n = 0; n < spp; ++n) {
      const float4 r = rn;
      const float2 im = imn;
      if (n + 1 < spp) { rn = W.result[base + (n + 1) * stride]; imn = W.img[base + (n + 1) * stride]; }
      if (r.w == 0.f) continue;
      const float dx = im.x - 0.5f, dy = im.y - 0.5f;
      const int x0 = max(ox, (int)ceilf(dx - fw)), x1 = min(ox + w - 1, (int)floorf(dx + fw));
      const int y0 = max(oy, (int)ceilf(dy - fh)), y1 = min(oy + h - 1, (int)floorf(dy + fh));
#pragma unroll
      for (int b = 0; b < KB; ++b) {
        const int y = iy - R + b0 + b;
        if (b0 + b >= K || y < y0 || y > y1) continue;
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
    for (int b = 0; b < KB; ++b) {
      const int y = iy - R + b0 + b;
      if (b0 + b >= K || y < oy || y >= oy + h) continue;
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
  film_flush(S, img, ox, oy, w, h, film, timg, sw, sh);
}

// addTile of gathered tile images (Image.hs:178-199): block k adds the slot tiles[k].src (sw x sh x 4
// floats, the layout film_flush writes) at its tile's image origin; zero pixels and pixels past the
// film skipped.  One launch merges every rank's (or device's) images.
struct TileSrc { const float4* src; int ox, oy; };
static __global__ __launch_bounds__(256) void k_add_tiles(const TileSrc* __restrict__ tiles, float* __restrict__ film,
                                                   int width, int height, int sw, int sh) {
  const TileSrc t = tiles[blockIdx.x];
  for (int q = threadIdx.x; q < sw * sh; q += blockDim.x) {
    const int gx = t.ox + q % sw, gy = t.oy + q / sw;
    if (gx >= width || gy >= height) continue;
    const float4 v = t.src[q];
    if (v.x == 0.f && v.y == 0.f && v.z == 0.f && v.w == 0.f) continue;
    float* d = film + 4 * ((size_t)gy * width + gx);
    atomicAdd(&d[0], v.x); atomicAdd(&d[1], v.y); atomicAdd(&d[2], v.z); atomicAdd(&d[3], v.w);
  }
}

}  // namespace bd
