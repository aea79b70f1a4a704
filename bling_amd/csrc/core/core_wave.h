// core_wave.h -- the per-vertex launch sequence of one wave of paths (Path and DirectLighting) and
// batch traversal, as templates over the kernel feature profile.  Included only by the profile units
// prof_<k>.hip, each of which instantiates one profile.
#pragma once
#include "core_internal.h"

namespace bcore {

// Batch traversal for bling_trace (Scene.scIntersect / Scene.occluded).
template <bool ANY, uint32_t F>
static __global__ __launch_bounds__(256) void k_trace(const DevScene* __restrict__ Sptr, const float* __restrict__ rays, uint32_t n,
                                               float* __restrict__ t_out, uint32_t* __restrict__ prim_out,
                                               float* __restrict__ bary_out, const int32_t* __restrict__ shape_prim,
                                               Counters* __restrict__ C) {
  extern __shared__ float4 smem[];
  const DevScene& S = *Sptr;
  const LdsScene L = lds_setup(S, smem);
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  TraceCount tc{0u, 0u, 0u, 0u};
  if (i < n) {
    Ray r{mk(rays[i], rays[n + i], rays[2 * (size_t)n + i]), mk(rays[3 * (size_t)n + i], rays[4 * (size_t)n + i], rays[5 * (size_t)n + i]),
          rays[6 * (size_t)n + i], rays[7 * (size_t)n + i]};
    HitRec h;
    if (ANY) {
      prim_out[i] = trace<true, F>(S, L, r, h, tc) ? 1u : 0u;
    } else if (trace<false, F>(S, L, r, h, tc)) {
      uint32_t kind = h.ref >> 30, idx = h.ref & 0x3FFFFFFFu;
      uint32_t pid;
      float b1 = h.b1, b2 = h.b2;
      if (kind == REF_TRI) pid = (uint32_t)S.tri_prim[idx];
      else if (kind == REF_SHAPE) {
        pid = (uint32_t)shape_prim[idx];
        DG dg = shape_dg<F>(gen(S.shapes[idx]), r, h.t);
        b1 = dg.u; b2 = dg.v;
      } else pid = (uint32_t)S.fractal_prim;
      if (t_out) t_out[i] = h.t;
      prim_out[i] = pid;
      if (bary_out) { bary_out[2 * i] = b1; bary_out[2 * i + 1] = b2; }
    } else {
      if (t_out) t_out[i] = INFINITY;
      prim_out[i] = BLING_MISS;
      if (bary_out) { bary_out[2 * i] = 0.f; bary_out[2 * i + 1] = 0.f; }
    }
  }
  unsigned long long nv = wave_sum_u64((unsigned long long)tc.nodes);
  unsigned long long nt = wave_sum_u64((unsigned long long)tc.tris);
  unsigned long long ns = wave_sum_u64((unsigned long long)tc.shapes);
  if ((threadIdx.x & 63) == 0) {
    if (nv) atomicAdd(&C->node_visits, nv);
    if (nt) atomicAdd(&C->tri_tests, nt);
    if (ns) atomicAdd(&C->shape_tests, ns);
  }
}

// The traversal launches of one wave: the exhaustive kernels for scenes of a few dozen primitives
// (DevScene::bf_tris + bf_shapes > 0), the wave-coherent packet kernels when the scene's threaded BVH
// is small (DevScene::pkt_n > 0), else the per-lane kernels; never the first two for fractal scenes.
template <uint32_t F, bool STATS, bool ALLL>
struct TraceLaunch {
  bling_ctx* c;
  bool pkt, bf;
  unsigned gc, ga;
  size_t lds() const { return use_bvh4<F>() ? c->lds_trace4 : c->lds_trace; }
  size_t pkt_lds() const { return sizeof(DevShape) * c->S.lds4_shapes; }   // packet_lds
  TraceLaunch(bling_ctx* c_, uint32_t n) : c(c_), pkt(false), bf(false), gc(1), ga(1) {
    if constexpr (!(F & FT_FRACTAL)) {
      bf = c->S.bf_tris + c->S.bf_shapes > 0;
      pkt = !bf && c->S.pkt_n > 0;
      if (bf) {
        gc = persistent_grid(k_trace_closest_bf<F, STATS>, 0, 2 * n);
        ga = persistent_grid(k_trace_any_bf<F, STATS>, 0, n);
        return;
      }
      if (pkt) {
        gc = persistent_grid(k_trace_closest_pkt<F, STATS>, pkt_lds(), 2 * n);
        ga = persistent_grid(k_trace_any_pkt<F, STATS>, pkt_lds(), n);
        return;
      }
    }
    gc = persistent_grid(k_trace_closest<F, STATS, ALLL>, lds(), 2 * n);
    ga = persistent_grid(k_trace_any<F, STATS, ALLL>, lds(), n);
    if constexpr (use_bvh4<F>()) {
      if ((size_t)std::max(gc, ga) * 256 > c->S.stack4_lanes && c->S.stack4_need > c->S.stack4_lds)
        throw std::runtime_error("BVH4 stack overflow rows sized for fewer lanes than the traversal grid");
    }
  }
  void closest(const WaveState& W) const {
    if constexpr (!(F & FT_FRACTAL)) {
      if (bf) { k_trace_closest_bf<F, STATS><<<gc, 256, 0, c->stream>>>(c->dscene.p, W, c->counters.p); return; }
      if (pkt) { k_trace_closest_pkt<F, STATS><<<gc, 256, pkt_lds(), c->stream>>>(c->dscene.p, W, c->counters.p); return; }
    }
    k_trace_closest<F, STATS, ALLL><<<gc, 256, lds(), c->stream>>>(c->dscene.p, W, c->counters.p);
  }
  void any(const WaveState& W) const {
    if constexpr (!(F & FT_FRACTAL)) {
      if (bf) { k_trace_any_bf<F, STATS><<<ga, 256, 0, c->stream>>>(c->dscene.p, W, c->counters.p); return; }
      if (pkt) { k_trace_any_pkt<F, STATS><<<ga, 256, pkt_lds(), c->stream>>>(c->dscene.p, W, c->counters.p); return; }
    }
    k_trace_any<F, STATS, ALLL><<<ga, 256, lds(), c->stream>>>(c->dscene.p, W, c->counters.p);
  }
};

// The shading launches go through host wrappers, so that a large profile can compile its shading
// kernels in units of their own (prof_<k>a / b.hip) beside the traversal / compaction pipeline.
template <uint32_t F, bool FUSED>
void shade_launch(unsigned gs, size_t lds, hipStream_t s, const DevScene* d, const WaveState& W, int depth, int qin,
                  uint32_t seed, uint32_t pass, Counters* C) {
  k_shade<F, FUSED><<<gs, 256, lds, s>>>(d, W, depth, qin, seed, pass, C);
}
template <uint32_t F>
void shade_dl_launch(unsigned gs, hipStream_t s, const DevScene* d, const WaveState& W, int qin, uint32_t seed,
                     uint32_t pass, Counters* C) {
  k_shade_dl<F><<<gs, 256, 0, s>>>(d, W, qin, seed, pass, C);
}

template <uint32_t F, bool STATS, bool ALLL>
int run_wave_t(bling_ctx* c, WaveState W, uint32_t n, uint32_t seed, uint32_t pass, WaveTiming* tm) {
  hipStream_t s = c->stream;
  const DevScene* d = c->dscene.p;
  Counters* C = c->counters.p;
  const unsigned gs = grid_for(n);
  const TraceLaunch<F, STATS, ALLL> tl(c, n);
  const uint32_t nb = (n + COMPACT_CHUNK - 1) / COMPACT_CHUNK;
  // the shading kernel tests the shadow rays itself (wavefront.h inline_shadow): no any-hit launch
  const bool inl = inline_shadow<F>() && c->S.sh_inline != 0u;
  const size_t lshade = inl ? c->lds_shade : 0;
  // Mandelbulb scenes: each traversal launch is preceded by the march of its queue (k_march), whose
  // results the traversal kernels read at the fractal leaf; Julia scenes march inside the traversal
  bool premarch = false;
  unsigned gmc = 1, gma = 1;
  if constexpr ((F & FT_FRACTAL) != 0) {
    // (k_march_jobs keeps 16-bit loop counters: deeper iteration counts march in the traversal)
    premarch = W.march_t != nullptr && c->S.fractal.kind == BLING_FRACTAL_MANDELBULB && c->S.fractal.iterations < 32767;
    if (premarch) {
      gmc = persistent_grid(k_march_jobs<F, STATS, false>, 0, 2 * n);
      gma = persistent_grid(k_march_jobs<F, STATS, true>, 0, n);
    }
  }
  if (!premarch) W.march_t = nullptr;
  auto march = [&](bool anyq) {
    if constexpr ((F & FT_FRACTAL) != 0) {
      if (!premarch) return;
      if (anyq) k_march_jobs<F, STATS, true><<<gma, 256, 0, s>>>(d, W, C);
      else k_march_jobs<F, STATS, false><<<gmc, 256, 0, s>>>(d, W, C);
    } else {
      (void)anyq;
    }
  };
  int launches = 0;
  for (int depth = 0; depth <= c->S.max_depth; ++depth) {
    if (tm && tm->on) {                // the closest-hit queries' time includes their march
      hipEvent_t a, b;
      HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b));
      tm->ev.push_back(a); tm->ev.push_back(b);
      HIPCHK(hipEventRecord(a, s));
      march(false);
      tl.closest(W);
      HIPCHK(hipEventRecord(b, s));
    } else {
      march(false);
      tl.closest(W);
    }
    if (depth > 0 && !inl) {
      march(true);
      tl.any(W);
      ++launches;
    }
    int qin = depth & 1;
    k_stage<<<1, 64, 0, s>>>(W.qcount, qin, depth, C, 1);
    if (depth > 0) {
      // resolve(d - 1) + shade(d) over the resolve list of d - 1 (wavefront.h k_shade<F, true>):
      // reads the current set at the listed slots, writes vertex d to the next set at its entries
      if (tm && tm->on) {
        hipEvent_t a, b;
        HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b));
        tm->ev_shade.push_back(a); tm->ev_shade.push_back(b);
        HIPCHK(hipEventRecord(a, s));
        shade_launch<F, true>(gs, lshade, s, d, W, depth, qin, seed, pass, C);
        HIPCHK(hipEventRecord(b, s));
      } else {
        shade_launch<F, true>(gs, lshade, s, d, W, depth, qin, seed, pass, C);
      }
    } else if (tm && tm->on) {        // depth 0 is timed with the fused launches (ms_shade)
      hipEvent_t a, b;
      HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b));
      tm->ev_shade.push_back(a); tm->ev_shade.push_back(b);
      HIPCHK(hipEventRecord(a, s));
      shade_launch<F, false>(gs, lshade, s, d, W, depth, qin, seed, pass, C);
      HIPCHK(hipEventRecord(b, s));
    } else {
      shade_launch<F, false>(gs, lshade, s, d, W, depth, qin, seed, pass, C);
    }
    std::swap(W.cur, W.nxt);           // the queues built next index the set just written
    if (depth < c->S.max_depth) {      // shade at maxDepth finalises every path: nothing to queue
      k_compact_count<<<nb, 256, 0, s>>>(W, qin);
      k_compact_scan<<<1, 1024, 0, s>>>(W, nb, qin, 1);
      k_compact_scatter<<<nb, 256, 0, s>>>(W, nb, qin, 1);
      launches += 3;
    }
    launches += 3;
  }
  return launches;
}

// DirectLighting: one tree node per path per step.  The number of steps depends on the specular
// trees, so the shade-queue length is read back after each compaction (one 4-byte copy per step);
// the walk ends once no path has a ray left and the last step's shadow / MIS rays are resolved.
template <uint32_t F, bool STATS, bool ALLL>
int run_wave_dl_t(bling_ctx* c, WaveState W, uint32_t n, uint32_t seed, uint32_t pass, WaveTiming* tm) {
  hipStream_t s = c->stream;
  const DevScene* d = c->dscene.p;
  Counters* C = c->counters.p;
  const unsigned gs = grid_for(n), gr = grid_for(n);
  const TraceLaunch<F, STATS, ALLL> tl(c, n);
  const uint32_t nb = (n + COMPACT_CHUNK - 1) / COMPACT_CHUNK;
  const int max_steps = (1 << c->S.max_depth);        // a tree of depth < maxDepth has < 2^maxDepth nodes
  W.march_t = nullptr;                                // the traversal kernels march themselves
  uint32_t live = n;
  int launches = 0;
  for (int step = 0;; ++step) {
    if (tm && tm->on) {
      hipEvent_t a, b;
      HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b));
      tm->ev.push_back(a); tm->ev.push_back(b);
      HIPCHK(hipEventRecord(a, s));
      tl.closest(W);
      HIPCHK(hipEventRecord(b, s));
    } else {
      tl.closest(W);
    }
    ++launches;
    if (step > 0) {
      tl.any(W);
      k_resolve<F><<<gr, 256, 0, s>>>(d, W, C);
      std::swap(W.cur.T, W.cur.Tn);      // in place: the next node's weight becomes its T
      W.nxt = W.cur;
      launches += 2;
    }
    if (live == 0) break;
    if (step >= max_steps) throw std::runtime_error("directLighting walk did not terminate");
    const int qin = step & 1;
    k_stage<<<1, 64, 0, s>>>(W.qcount, qin, step, C, 0);
    shade_dl_launch<F>(gs, s, d, W, qin, seed, pass, C);
    k_compact_count<<<nb, 256, 0, s>>>(W, qin);
    k_compact_scan<<<1, 1024, 0, s>>>(W, nb, qin, 0);
    k_compact_scatter<<<nb, 256, 0, s>>>(W, nb, qin, 0);
    launches += 5;
    HIPCHK(hipMemcpyAsync(&live, W.qcount + (qin ^ 1), sizeof live, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  return launches;
}

template <uint32_t F>
int run_wave_prof(bling_ctx* c, const WaveState& W, uint32_t n, uint32_t seed, uint32_t pass, bool stats, WaveTiming* tm) {
  const bool all = use_bvh4<F>() ? c->lds_all4 : c->lds_all;
  if (c->S.integrator == BLING_INTEGRATOR_DIRECT) {
    if (all)
      return stats ? run_wave_dl_t<F, true, true>(c, W, n, seed, pass, tm) : run_wave_dl_t<F, false, true>(c, W, n, seed, pass, tm);
    return stats ? run_wave_dl_t<F, true, false>(c, W, n, seed, pass, tm) : run_wave_dl_t<F, false, false>(c, W, n, seed, pass, tm);
  }
  if (all)
    return stats ? run_wave_t<F, true, true>(c, W, n, seed, pass, tm) : run_wave_t<F, false, true>(c, W, n, seed, pass, tm);
  return stats ? run_wave_t<F, true, false>(c, W, n, seed, pass, tm) : run_wave_t<F, false, false>(c, W, n, seed, pass, tm);
}

template <uint32_t F>
void launch_trace_prof(bling_ctx* c, const float* rays, uint32_t n, int any_hit, float* t, uint32_t* prim, float* bary) {
  unsigned blocks = (n + 255) / 256;
  hipStream_t s = c->stream;
  const DevScene* d = c->dscene.p;
  if (any_hit) k_trace<true, F><<<blocks, 256, c->lds_trace, s>>>(d, rays, n, t, prim, bary, c->shape_prim.p, c->counters.p);
  else k_trace<false, F><<<blocks, 256, c->lds_trace, s>>>(d, rays, n, t, prim, bary, c->shape_prim.p, c->counters.p);
}

}  // namespace bcore

#define BLING_SHADE_ARGS unsigned, size_t, hipStream_t, const DevScene*, const WaveState&, int, int, uint32_t, uint32_t, Counters*
#define BLING_SHADE_DL_ARGS unsigned, hipStream_t, const DevScene*, const WaveState&, int, uint32_t, uint32_t, Counters*
#ifdef BLING_STUB_PROFILE
// Experiment builds only (make variant ... STUB="4 5"): the profile's entry points throw instead of
// compiling its kernels, so an A/B build of the bench profiles takes minutes less.  Never in `make all`.
#define BLING_INSTANTIATE_PROFILE(K)                                                                              \
  namespace bcore {                                                                                               \
  template <> int run_wave_prof<kProfiles[K]>(bling_ctx*, const WaveState&, uint32_t, uint32_t, uint32_t, bool,   \
                                              WaveTiming*) { throw std::runtime_error("profile stubbed in this experiment build"); } \
  template <> void launch_trace_prof<kProfiles[K]>(bling_ctx*, const float*, uint32_t, int, float*, uint32_t*, float*) { \
    throw std::runtime_error("profile stubbed in this experiment build"); }                                       \
  }
#define BLING_INSTANTIATE_PROFILE_SPLIT(K) BLING_INSTANTIATE_PROFILE(K)
#define BLING_INSTANTIATE_SHADE(K, FUSED)
#define BLING_INSTANTIATE_SHADE_DL(K)
#else
#define BLING_INSTANTIATE_PROFILE(K)                                                                              \
  namespace bcore {                                                                                               \
  template int run_wave_prof<kProfiles[K]>(bling_ctx*, const WaveState&, uint32_t, uint32_t, uint32_t, bool,      \
                                           WaveTiming*);                                                          \
  template void launch_trace_prof<kProfiles[K]>(bling_ctx*, const float*, uint32_t, int, float*, uint32_t*, float*); \
  }
// split profiles: this unit compiles the pipeline without the shading kernels, whose launch wrappers
// the shade units instantiate (BLING_INSTANTIATE_SHADE / _SHADE_DL in prof_<k>a.hip / prof_<k>b.hip)
#define BLING_INSTANTIATE_PROFILE_SPLIT(K)                                                                        \
  namespace bcore {                                                                                               \
  extern template void shade_launch<kProfiles[K], true>(BLING_SHADE_ARGS);                                        \
  extern template void shade_launch<kProfiles[K], false>(BLING_SHADE_ARGS);                                       \
  extern template void shade_dl_launch<kProfiles[K]>(BLING_SHADE_DL_ARGS);                                        \
  }                                                                                                               \
  BLING_INSTANTIATE_PROFILE(K)
#define BLING_INSTANTIATE_SHADE(K, FUSED)                                                                         \
  namespace bcore {                                                                                               \
  template void shade_launch<kProfiles[K], FUSED>(BLING_SHADE_ARGS);                                              \
  }
#define BLING_INSTANTIATE_SHADE_DL(K)                                                                             \
  namespace bcore {                                                                                               \
  template void shade_dl_launch<kProfiles[K]>(BLING_SHADE_DL_ARGS);                                               \
  }
#endif
