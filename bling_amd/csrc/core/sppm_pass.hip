// sppm_pass.hip -- host driver of one SPPM pass (Renderer/SPPM.hs onePass) over the kernels of sppm.h.
#include "core_internal.h"

namespace bcore {

// ------------------------------------------------------------------ SPPM pass (sppm.h)
static SppmBufs sppm_bufs(bling_ctx* c) {
  SppmState& P = c->sppm;
  SppmBufs B{};
  B.hp_pos = P.hp_pos.p; B.hp_hit = P.hp_hit.p; B.hp_o = P.hp_o.p; B.hp_d = P.hp_d.p; B.hp_f = P.hp_f.p;
  B.hp_bsdf = P.hp_bsdf.p;
  B.hp_count = P.hp_count.p; B.hp_cap = P.hp_cap;
  B.r2 = P.r2.p; B.nacc = P.nacc.p; B.cnt = P.cnt.p; B.n_stats = P.n_stats;
  B.grid = P.grid.p; B.bstart = P.bstart.p; B.bcur = P.bcur.p; B.items = P.items.p; B.items_cap = P.items_cap;
  B.hp_key = P.hp_key.p; B.kd_mr = P.kd_mr.p; B.kd_c = P.kd_c.p;
  B.splat = P.splat.p; B.ctr = P.ctr.p;
  return B;
}


static void sppm_alloc_hitpoints(SppmState& P, uint32_t cap) {
  P.hp_cap = cap;
  for (auto* b : {&P.hp_pos, &P.hp_hit, &P.hp_o, &P.hp_d}) b->alloc(cap);
  P.hp_f.alloc((size_t)4 * cap);
  P.hp_bsdf.alloc(cap);
  P.hp_key.alloc(cap);
  P.bstart.alloc((size_t)cap + 1);
  P.bcur.alloc(cap);
}

void sppm_init(bling_ctx* c) {
  SppmState& P = c->sppm;
  const DevScene& S = c->S;
  const int ext_h = S.ey1 - S.ey0 + 1;
  P.n_ext = (uint32_t)S.ext_w * (uint32_t)ext_h;
  P.n_stats = P.n_ext;                                                 // windowPixels (Sampling.hs:60-62)
  P.nth = (uint32_t)std::max(1, c->cfg.sppm_threads);
  std::vector<float> r2(P.n_stats, c->cfg.sppm_radius * c->cfg.sppm_radius);
  P.r2.upload(r2.data(), r2.size());
  P.nacc.alloc(P.n_stats);
  HIPCHK(hipMemset(P.nacc.p, 0, P.n_stats * sizeof(float)));
  P.cnt.alloc((size_t)P.nth * P.n_stats);
  // the extent's 16 x 16 tiles (splitWindow), one camera sample per pixel, in tile order
  std::vector<TileDesc> tl;
  uint32_t off = 0;
  for (int y = S.ey0; y <= S.ey1; y += 16)
    for (int x = S.ex0; x <= S.ex1; x += 16) {
      TileDesc t{x, std::min(x + 15, S.ex1), y, std::min(y + 15, S.ey1), off, 0u};
      t.count = (uint32_t)((t.x1 - t.x0 + 1) * (t.y1 - t.y0 + 1));
      off += t.count;
      tl.push_back(t);
    }
  P.n_tiles = (uint32_t)tl.size();
  P.tiles.upload(tl.data(), tl.size());
  P.result.alloc(P.n_ext); P.img.alloc(P.n_ext);
  P.hp_count.alloc(1); P.grid.alloc(1); P.ctr.alloc(4);
  sppm_alloc_hitpoints(P, 2 * P.n_ext);
  P.splat.alloc((size_t)S.width * S.height * 3);
  P.film.alloc((size_t)S.width * S.height * 4);
  P.ready = true;
}

template <uint32_t F>
static void sppm_launch_eye(bling_ctx* c, const WaveState& W, uint32_t seed, uint32_t pass) {
  SppmState& P = c->sppm;
  HIPCHK(hipMemsetAsync(P.hp_count.p, 0, sizeof(uint32_t), c->stream));
  HIPCHK(hipMemsetAsync(P.ctr.p, 0, 4 * sizeof(unsigned long long), c->stream));
  k_sppm_eye<F><<<dim3(1, P.n_tiles), TRACE_BLOCK, c->lds_trace, c->stream>>>(c->dscene.p, sppm_bufs(c), W, P.tiles.p,
                                                                             seed, pass);
  HIPCHK(hipGetLastError());
}

template <uint32_t F>
void sppm_pass_t(bling_ctx* c, uint32_t seed, uint32_t pass, bling_sppm_stats* st) {
  SppmState& P = c->sppm;
  const DevScene& S = c->S;
  hipStream_t s = c->stream;
  hipEvent_t e0, e1, e2, e3;
  HIPCHK(hipEventCreate(&e0)); HIPCHK(hipEventCreate(&e1)); HIPCHK(hipEventCreate(&e2)); HIPCHK(hipEventCreate(&e3));
  HIPCHK(hipEventRecord(e0, s));
  WaveState W{};
  W.result = P.result.p; W.img = P.img.p;
  // mkHitPoints; an overflowing hit-point buffer is grown and the (deterministic) pass re-run
  sppm_launch_eye<F>(c, W, seed, pass);
  uint32_t nhp = 0;
  HIPCHK(hipMemcpyAsync(&nhp, P.hp_count.p, sizeof nhp, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (nhp > P.hp_cap) {
    sppm_alloc_hitpoints(P, nhp + nhp / 4 + 1024);
    sppm_launch_eye<F>(c, W, seed, pass);
  }
  k_film<<<P.n_tiles, 256, 0, s>>>(c->dscene.p, W, P.tiles.p, P.film.p, nullptr, 0, 0);
  HIPCHK(hipEventRecord(e1, s));
  // mkHash: grid, bucket counts, offsets, entries
  HIPCHK(hipMemsetAsync(P.grid.p, 0, sizeof(SppmGrid), s));
  if (nhp > 0) {
    k_sppm_reduce<<<1, 1024, 0, s>>>(sppm_bufs(c));
    HIPCHK(hipMemsetAsync(P.bstart.p, 0, ((size_t)nhp + 1) * sizeof(uint32_t), s));
    const unsigned gb = (nhp + 255u) / 256u;
    k_sppm_cells<false><<<gb, 256, 0, s>>>(sppm_bufs(c));
    k_sppm_scan<<<1, 1024, 0, s>>>(sppm_bufs(c));
    SppmGrid g;
    HIPCHK(hipMemcpyAsync(&g, P.grid.p, sizeof g, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (g.items > P.items_cap) {
      P.items_cap = g.items + g.items / 4 + 1024;
      P.items.alloc(P.items_cap); P.kd_mr.alloc(P.items_cap); P.kd_c.alloc(P.items_cap);
    }
    k_sppm_cells<true><<<gb, 256, 0, s>>>(sppm_bufs(c));
    k_sppm_kd<<<gb, 256, 0, s>>>(sppm_bufs(c));                           // a kd-tree per bucket
  }
  HIPCHK(hipEventRecord(e2, s));
  // photons (threads x sn^2, SPPM.hs:441-453, 474)
  const uint32_t sn = (uint32_t)std::max(1, (int)std::ceil(std::sqrt((float)c->cfg.sppm_photons / (float)P.nth)));
  const uint64_t nph = (uint64_t)P.nth * sn * sn;
  if (nph > 0xFFFFFFFFull || (uint64_t)sn * sn > (1u << 24)) throw std::invalid_argument("too many photons per pass");
  HIPCHK(hipMemsetAsync(P.cnt.p, 0, (size_t)P.nth * P.n_stats * sizeof(uint32_t), s));
  k_sppm_photon<F><<<(unsigned)((nph + 255) / 256), TRACE_BLOCK, c->lds_trace, s>>>(c->dscene.p, sppm_bufs(c), P.nth, sn,
                                                                                   seed, pass);
  HIPCHK(hipGetLastError());
  k_sppm_stats<<<(P.n_stats + 255) / 256, 256, 0, s>>>(sppm_bufs(c), P.nth, c->cfg.sppm_alpha);
  HIPCHK(hipEventRecord(e3, s));
  unsigned long long ctr[4];
  HIPCHK(hipMemcpyAsync(ctr, P.ctr.p, sizeof ctr, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (st) {
    float a = 0.f, b = 0.f, t = 0.f;
    HIPCHK(hipEventElapsedTime(&a, e0, e1)); HIPCHK(hipEventElapsedTime(&b, e1, e2)); HIPCHK(hipEventElapsedTime(&t, e0, e3));
    st->hitpoints = std::min(nhp, P.hp_cap);
    st->photons = nph;
    st->cam_rays = ctr[0]; st->photon_rays = ctr[1]; st->photon_hits = ctr[2]; st->dropped = ctr[3];
    st->ms_eye = a; st->ms_hash = b; st->ms_photon = t - a - b; st->ms_total = t;
  }
  for (auto e : {e0, e1, e2, e3}) (void)hipEventDestroy(e);
  (void)S;
}

template void sppm_pass_t<kProfiles[0]>(bling_ctx*, uint32_t, uint32_t, bling_sppm_stats*);
template void sppm_pass_t<kSppmAll>(bling_ctx*, uint32_t, uint32_t, bling_sppm_stats*);

}  // namespace bcore
