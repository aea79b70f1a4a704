// core_internal.h -- host-side state of the MI355X core shared by its translation units:
// the context (bling_ctx), device buffers, kernel feature profiles and the per-profile entry points
// that the profile units (prof_*.hip) instantiate.  Splitting the kernel instantiations by profile
// lets the build compile them in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/bling.h"
#include "../common/scene_features.h"
#include "bvh_build.h"
#include "wavefront.h"
#include "sppm.h"

namespace bcore {
using namespace bd;

struct HipError : std::runtime_error { using std::runtime_error::runtime_error; };

#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) throw HipError(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ device buffers
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  DBuf(const DBuf&) = delete;              // owns device memory: never copied
  DBuf& operator=(const DBuf&) = delete;
  void alloc(size_t count) {
    free();
    if (count == 0) return;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    n = count;
  }
  void upload(const T* h, size_t count) {
    alloc(count);
    if (count) HIPCHK(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
  }
  void free() { if (p) { (void)hipFree(p); p = nullptr; n = 0; } }
  ~DBuf() { free(); }
};


// device bytes per path in flight, for sizing waves: per path set the SoA streams of wavefront.h
// PathSet (org, dir, hit, meta, mdir, fac, cf, sh_o, sh_d: 16 B each; mhit 8 B; occ 4 B), T and L
// (64 B each) and, for the non-factored profiles, Tn, lsc and bsc (64 B each); two sets for the Path
// pipeline, plus result, img, six queue words and the queue flag
constexpr uint64_t kSetBytes = 9 * 16 + 8 + 4 + 64 + 64;
constexpr uint64_t kSetSpectraBytes = 3 * 64;
constexpr uint64_t kPathFixedBytes = 16 + 8 + 6 * 4 + 1 + 4 + 2 * 4;   // ... + the k_march results (2 words)
// DirectLighting adds the continuation origin, the sibling mask and one parked ray (org, dir,
// weight) per level below maxDepth
constexpr uint64_t kDlSlotBytes = 16 + 16 + 64;
constexpr int kMaxDlDepth = 16;

// SPPM renderer state (sppm.h): hit points, hash grid and the per-pixel statistics that persist
// across passes (reset by a scene upload or bling_sppm_reset)
struct SppmState {
  bool ready = false;
  uint32_t hp_cap = 0, items_cap = 0, n_stats = 0, nth = 0, n_tiles = 0, n_ext = 0;
  DBuf<float4> hp_pos, hp_hit, hp_o, hp_d, hp_f, result;
  DBuf<Bsdf> hp_bsdf;
  DBuf<float2> img;
  DBuf<uint32_t> hp_count, cnt, bstart, bcur, items;
  DBuf<float> r2, nacc, splat, film, kd_mr, kd_c;
  DBuf<unsigned long long> hp_key;
  DBuf<SppmGrid> grid;
  DBuf<unsigned long long> ctr;
  DBuf<TileDesc> tiles;
  void free_all() {
    for (auto* b : {&hp_pos, &hp_hit, &hp_o, &hp_d, &hp_f, &result}) b->free();
    img.free(); hp_bsdf.free();
    for (auto* b : {&hp_count, &cnt, &bstart, &bcur, &items}) b->free();
    for (auto* b : {&r2, &nacc, &splat, &film, &kd_mr, &kd_c}) b->free();
    hp_key.free(); grid.free(); ctr.free(); tiles.free();
    ready = false; hp_cap = items_cap = 0;
  }
};

}  // namespace bcore

// the context lives in the global namespace (include/bling.h declares `struct bling_ctx`)
using namespace bd;
using namespace bcore;

struct bling_ctx {
  using WaveState = bd::WaveState;
  int device = 0;
  hipStream_t stream = nullptr;
  bool has_scene = false;
  DevScene S{};
  // scene memory
  DBuf<float4> nodes, tri_geo, pkt;   // BVH2 nodes, triangle records, threaded entry list
  DBuf<float4> leaf_geo;              // triangle records in leaf order, each with its ref (Traversal4)
  DBuf<uint32_t> refs;
  DBuf<float> tri_normals;
  DBuf<float4> tri_frame;
  DBuf<uint8_t> tri_has_n;
  DBuf<int32_t> tri_material, tri_prim, shape_prim;
  DBuf<DevShape> shapes;
  DBuf<bling_material> materials;
  DBuf<bling_texture> textures;
  DBuf<bling_scalar_texture> stex;
  DBuf<bling_light> lights;
  DBuf<bling_image> images;
  std::vector<std::unique_ptr<DBuf<float>>> light_arrays;   // Dist2D tables, env maps, texture images
  // path state (WaveState): two sets of per-slot records (PathSet), by-sample arrays, queues
  uint32_t cap = 0;
  struct SetBufs {
    DBuf<float4> org, dir, hit, mdir, fac, cf, sh_o, sh_d, T, Tn, L, lsc, bsc;
    DBuf<uint4> meta;
    DBuf<float2> mhit;
    DBuf<uint32_t> occ;
    void alloc(uint32_t n, bool spectra) {
      for (auto* b : {&org, &dir, &hit, &mdir, &fac, &cf, &sh_o, &sh_d}) b->alloc(n);
      meta.alloc(n); mhit.alloc(n); occ.alloc(n);
      T.alloc((size_t)4 * n); L.alloc((size_t)4 * n);
      if (spectra) { Tn.alloc((size_t)4 * n); lsc.alloc((size_t)4 * n); bsc.alloc((size_t)4 * n); }
      else { Tn.free(); lsc.free(); bsc.free(); }
    }
    void free() {
      for (auto* b : {&org, &dir, &hit, &mdir, &fac, &cf, &sh_o, &sh_d, &T, &Tn, &L, &lsc, &bsc}) b->free();
      meta.free(); mhit.free(); occ.free();
    }
    PathSet view() const {
      return PathSet{org.p, dir.p, hit.p, meta.p, mdir.p, mhit.p, occ.p, fac.p, cf.p, sh_o.p, sh_d.p,
                     T.p, Tn.p, L.p, lsc.p, bsc.p};
    }
  } set[2];
  bool sets_spectra = false, sets_two = false;     // layout of the allocated sets
  DBuf<float4> corg, dl_org, dl_dir, dl_T;          // DirectLighting only
  DBuf<uint32_t> dl_mask;
  int dl_levels = 0;                                // slots allocated per path (0 = Path)
  DBuf<float4> result;
  DBuf<float2> img;
  DBuf<uint32_t> qmem, qcount, blk;
  DBuf<float> march;                                 // k_march results, one per closest / any queue entry
  DBuf<uint8_t> qflag;
  DBuf<TileDesc> tiles_dev;
  DBuf<Counters> counters;
  uint64_t stream_bytes[2 * BLING_N_STREAMS] = {};   // Counters::sb of the last pass (BLING_STREAM_STATS)
  DBuf<DevScene> dscene;      // the DevScene record in device memory (kernels take a pointer)
  DBuf<float> film_dev;
  // trace scratch
  DBuf<float> tr_rays, tr_t, tr_bary;
  DBuf<uint32_t> tr_prim;
  // bvh stats
  int bvh_depth = 0, bvh_leaves = 0, bvh_max_leaf = 0, bvh4_depth = 0;
  uint32_t num_prims = 0;
  uint32_t features = FT_ALL;   // scene_features() of the uploaded scene
  size_t lds_trace = 0;         // dynamic LDS bytes of the traversal kernels
  bool lds_all = false;         // the whole BVH, triangle set and leaf refs are LDS-resident
  size_t lds_trace4 = 0;        // the same for the BVH4 plan (queue traversal kernels, dev_trace.h Traversal4)
  size_t lds_shade = 0;         // dynamic LDS of k_shade: the BVH4 copy of its in-line shadow test (or 0)
  bool lds_all4 = false;
  DBuf<float4> nodes4;          // BVH4 nodes
  DBuf<int32_t> stack4_ovf;     // BVH4 stack rows beyond the LDS ones
  bling_render_config cfg{};    // the uploaded scene's renderer configuration
  SppmState sppm;
  // Multi-device fan-out (bling_create with n_devices > 1): one context per further device; every
  // device renders its share as tile images, the peers push theirs over xGMI into stage, and the
  // primary adds them all (Rendering.hs:118).
  std::vector<std::unique_ptr<bling_ctx>> peers;
  DBuf<float> pass_tiles;          // this device's tile images of the pass (BLING_PASS_TILE_IMAGES)
  DBuf<TileSrc> tile_src;          // the merge's per-tile sources (k_add_tiles)
  std::vector<std::unique_ptr<DBuf<float>>> stage;  // primary: landing buffer of peer j's tile images

  ~bling_ctx() {
    peers.clear();                          // each peer frees its memory on its own device
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamDestroy(stream);
  }

  int want_dl_levels() const { return S.integrator == BLING_INTEGRATOR_DIRECT ? S.max_depth : 0; }
  // the uploaded scene's kernel profile keeps the three non-factored spectra per slot (wavefront.h
  // factored()); DirectLighting runs in place on one set
  bool want_spectra() const;
  bool want_two_sets() const { return S.integrator != BLING_INTEGRATOR_DIRECT; }
  uint64_t path_bytes() const {
    const uint64_t set_b = kSetBytes + (want_spectra() ? kSetSpectraBytes : 0);
    return (want_two_sets() ? 2 : 1) * set_b + kPathFixedBytes + (want_dl_levels() ? 20 + kDlSlotBytes * want_dl_levels() : 0);
  }

  void ensure_paths(uint32_t n) {
    const int lv = want_dl_levels();
    const bool sp = want_spectra(), two = want_two_sets();
    const bool relayout = lv != dl_levels || sp != sets_spectra || two != sets_two;
    if (n <= cap && !relayout) return;
    cap = std::max(cap, (n + 255u) & ~255u);
    dl_levels = lv; sets_spectra = sp; sets_two = two;
    set[0].alloc(cap, sp);
    if (two) set[1].alloc(cap, sp); else set[1].free();
    if (lv) {
      corg.alloc(cap); dl_mask.alloc(cap);
      dl_org.alloc((size_t)lv * cap); dl_dir.alloc((size_t)lv * cap); dl_T.alloc((size_t)4 * lv * cap);
    } else {
      for (auto* b : {&corg, &dl_org, &dl_dir, &dl_T}) b->free();
      dl_mask.free();
    }
    result.alloc(cap); img.alloc(cap);
    qmem.alloc((size_t)6 * cap);     // SHADE0, SHADE1, CLOSEST (2 cap), ANY, RESOLVE
    march.alloc((size_t)2 * cap);    // reused: closest-queue results, then any-queue results
    qcount.alloc(Q_N);
    qflag.alloc(cap);
    blk.alloc((size_t)4 * (cap / COMPACT_CHUNK + 2));
  }
  WaveState state() {
    WaveState W{};
    W.cur = set[0].view();
    W.nxt = sets_two ? set[1].view() : W.cur;
    W.corg = dl_levels ? corg.p : nullptr;
    W.img = img.p; W.result = result.p;
    W.Lfull = nullptr; W.dbg = nullptr;
    W.march_t = march.p;             // run_wave_t keeps it for Mandelbulb scenes only (k_march)
    W.dl_org = dl_levels ? dl_org.p : nullptr; W.dl_dir = dl_levels ? dl_dir.p : nullptr;
    W.dl_T = dl_levels ? dl_T.p : nullptr; W.dl_mask = dl_levels ? dl_mask.p : nullptr;
    W.queue[Q_SHADE0] = qmem.p;
    W.queue[Q_SHADE1] = qmem.p + cap;
    W.queue[Q_CLOSEST] = qmem.p + 2 * (size_t)cap;
    W.queue[Q_ANY] = qmem.p + 4 * (size_t)cap;
    W.queue[Q_RESOLVE] = qmem.p + 5 * (size_t)cap;
    W.qcount = qcount.p;
    W.qflag = qflag.p;
    W.blk = blk.p;
    W.sb = counters.p ? counters.p->sb : nullptr;
    W.cap = cap;
    return W;
  }
};

namespace bcore {

// Kernel profiles: feature sets the kernels are compiled for.  A scene runs on the first profile
// that covers its features (scene_features.h); the last one covers everything.
// The cornell and sun-sky profiles serve one-light scenes only (dev_scene.h one_light): their light
// record -- for the sun-sky profile the sky model's constants -- is read with scalar loads (sun-sky
// one-light: C4 9 170 -> 9 789 Mrays/s, shade 873 -> 806 ms per pass, profiles/r06_ab_session.txt
// r06s2w); the others serve any number.
constexpr uint32_t kProfiles[] = {
    FT_MATTE | FT_AREA | FT_TRIS,                                                         // cornell
    FT_MATTE | FT_PLASTIC | FT_AREA | FT_ENV_CONST | FT_TRIS | FT_TRI_NORMALS | FT_MULTI_LIGHT,   // meshes
    FT_MATTE | FT_PLASTIC | FT_GLASS | FT_METAL | FT_MIRROR | FT_GRAPHPAPER | FT_AREA | FT_ENV_CONST |
        FT_ENV_SKY | FT_SPHERE,                                                           // analytic shapes (sun-sky)
    FT_MATTE | FT_GRAPHPAPER | FT_AREA | FT_ENV_CONST | FT_ENV_SKY | FT_FRACTAL | FT_MULTI_LIGHT,   // mandelbulb
    FT_ALL & ~(FT_FRACTAL | FT_PROCTEX),                                                  // surfaces
    FT_ALL,
};

// SPPM keeps each hit point's BSDF record between its eye and photon passes; computed spectra
// (FT_PROCTEX) live only while one thread shades, so SPPM runs without them (bling_sppm_pass
// refuses such scenes).  Photons leave area, infinite, point and directional lights (sppm.h light_ray).
constexpr uint32_t kSppmAll = FT_ALL & ~FT_PROCTEX;

template <size_t I = 0, class Fn>
void with_profile(uint32_t need, Fn&& fn) {
  constexpr uint32_t P = kProfiles[I];
  if constexpr (I + 1 < sizeof(kProfiles) / sizeof(kProfiles[0])) {
    if ((need & ~P) != 0u) return with_profile<I + 1>(need, fn);
  }
  fn(std::integral_constant<uint32_t, P>{});
}

inline uint32_t profile_of(uint32_t need) {
  uint32_t p = 0;
  with_profile(need, [&](auto prof) { p = decltype(prof)::value; });
  return p;
}

}  // namespace bcore

inline bool bling_ctx::want_spectra() const {
  bool full = true;
  bcore::with_profile(features, [&](auto prof) { full = !bd::factored<decltype(prof)::value>(); });
  return full || S.integrator == BLING_INTEGRATOR_DIRECT;
}

namespace bcore {

// Drive one wave of n freshly generated paths to completion (Path.hs:41-87 for every path).
// Queue lengths stay on the device: every launch is a grid-stride loop that reads the live count
// itself, so the host never synchronises inside the loop.
struct WaveTiming {
  bool on = false;
  std::vector<hipEvent_t> ev;      // pairs around each k_trace_closest launch
  std::vector<hipEvent_t> ev_shade;   // pairs around each fused resolve + shade launch
};

inline unsigned grid_for(uint32_t items) {
  constexpr uint32_t kMaxBlocks = 256 * 8;       // 8 blocks of 256 per CU, grid-stride beyond
  return std::max(1u, std::min((items + 255u) / 256u, kMaxBlocks));
}

// Grid of a persistent (grid-stride, lane-refill) kernel: exactly the blocks that are co-resident
// on the device, so no second partial round of blocks idles most CUs at the tail.
template <class K>
unsigned persistent_grid(K kernel, size_t lds, uint32_t items) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  const uint32_t cap = (uint32_t)(cus * per_cu);
  return std::max(1u, std::min((items + 255u) / 256u, cap));
}

// Per-profile entry points, explicitly instantiated by prof_<k>.hip (one unit per kProfiles entry;
// the largest profiles compile their shading kernels in prof_<k>a / b (/ c).hip beside it, so
// the build runs them in parallel) and sppm_pass.hip.
template <uint32_t F>
int run_wave_prof(bling_ctx* c, const WaveState& W, uint32_t n, uint32_t seed, uint32_t pass, bool stats, WaveTiming* tm);
template <uint32_t F>
void launch_trace_prof(bling_ctx* c, const float* rays, uint32_t n, int any_hit, float* t, uint32_t* prim, float* bary);
template <uint32_t F>
void sppm_pass_t(bling_ctx* c, uint32_t seed, uint32_t pass, bling_sppm_stats* st);
void sppm_init(bling_ctx* c);

}  // namespace bcore
