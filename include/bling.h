/*
 * bling.h -- C ABI of the MI355X-native intersection + path-integration core (libbling_hip.so).
 *
 * This is the drop-in seam for bling's per-sample hot path.  The reference has no FFI; its plug-in
 * point is the Renderer class, `render :: a -> RenderJob -> ProgressReporter -> IO ()`
 * (src/lib/Graphics/Bling/Rendering.hs:77-78), whose sampler renderer `prender`
 * (Rendering.hs:111-150) drives Sampling.runSample -> Camera.fireRay -> Integrator.Path.nextVertex
 * (Integrator/Path.hs:41-87) -> Scene.scIntersect/occluded (Scene.hs:45-51) -> KdTree traversal
 * (Primitive/KdTree.hs:210-246) -> Shape/Triangle intersect.  Each entry point below names the
 * reference interface it replaces.  Conventions:
 *   - return 0 on success, a negative BLING_E* code on failure; no C++ exception crosses the ABI;
 *   - host buffers are caller-owned and copied; device memory is owned by the context unless an
 *     entry point says it takes a device pointer;
 *   - a context is used by one host thread at a time; every call blocks until its result is ready.
 */
#ifndef BLING_H
#define BLING_H

#include <stddef.h>
#include <stdint.h>
#include "bling_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BLING_OK           0
#define BLING_EINVAL      -1   /* bad argument                                  */
#define BLING_ENODEV      -2   /* no usable HIP device                          */
#define BLING_EHIP        -3   /* a HIP runtime call failed                     */
#define BLING_ENOSCENE    -4   /* no scene uploaded                             */
#define BLING_EUNSUPPORTED -5  /* scene feature not implemented on the device   */
#define BLING_ENOMEM      -6

#define BLING_MISS 0xFFFFFFFFu

typedef struct bling_ctx bling_ctx;

/* One render pass = every camera sample of the sample extent once (Rendering.hs:127-140).
 * Samples are keyed by (seed, pass_index, pixel, sample, dimension) through the counter RNG that
 * replaces the per-tile MWC streams of Random.hs:56-62 / Rendering.hs:128. */
typedef struct bling_pass_params {
    uint32_t seed;
    uint32_t pass_index;
    int32_t  shard_rank;       /* of the tiles the stride keeps, the m-th (m = k / tile_stride) */
    int32_t  shard_world;      /* is rendered iff m % shard_world == shard_rank; 1 = all of them */
    int32_t  tile_stride;      /* >1: keep only tiles k with k % tile_stride == 0 (sub-sample)  */
    int32_t  chunk_paths;      /* paths in flight per wave (0 = default)                       */
    uint32_t flags;            /* BLING_PASS_* bits                                            */
    void*    tiles_device;     /* BLING_PASS_TILE_IMAGES: device buffer of the pass's tile images */
    uint64_t tiles_capacity;   /* floats tiles_device holds (and, for bling_film_add_*, each rank's
                                  buffer): the core refuses (BLING_EINVAL) a layout that needs more,
                                  so a buffer sized for another shard / stride is never overrun */
} bling_pass_params;

#define BLING_PASS_TRAVERSAL_STATS 1u  /* count node fetches / triangle / shape tests (slower)   */
#define BLING_PASS_KERNEL_TIMING   2u  /* HIP events around every closest-hit launch (roofline)  */
/* Tile images instead of a film (the multi-rank merge): the pass writes each of its
 * tiles' mkImageTile images (Image.hs:108-120) -- slot k = the k-th tile the shard / stride select,
 * in splitWindow order, slot_w x slot_h x 4 floats, zero padded, every slot written whole -- into
 * tiles_device on device_ids[0]; the film argument is ignored (may be NULL).  Single-device
 * contexts only.  bling_pass_tile_layout gives the slot count, size and origins; a rank gathers the
 * others' slots and adds them with bling_film_add_tiles (addTile, Image.hs:178-199). */
#define BLING_PASS_TILE_IMAGES     4u
/* bling_render only: RegionStarted / SamplesAdded reports per sample window before each PassDone */
#define BLING_PASS_REGION_EVENTS   8u

typedef struct bling_stats {
    uint64_t camera_samples;   /* paths started                                               */
    uint64_t rays_camera;      /* closest-hit queries of camera rays                          */
    uint64_t rays_continuation;/* closest-hit queries of BSDF-sampled continuation rays        */
    uint64_t rays_mis;         /* closest-hit queries of BSDF-sampled MIS rays (Scene.hs:71-82)  */
    uint64_t rays_shadow;      /* any-hit queries of light-sample shadow rays (Scene.hs:45-47)  */
    uint64_t dropped_samples;  /* NaN / Inf samples skipped by addSample (Image.hs:253-256)     */
    uint64_t tiles;            /* tiles rendered by this call                                  */
    double   ms_total;         /* device wall time of the pass (HIP events)                    */
    double   ms_bounce;        /* path-vertex pipeline time (HIP events on the core's stream)   */
    double   ms_film;          /* film splat + merge                                           */
    uint64_t bounce_launches;  /* number of path-vertex pipeline launches                      */
    uint64_t path_vertices;    /* alive paths entering a bounce launch, summed                 */
    uint64_t node_visits;      /* BVH2 nodes fetched (64 B each)                               */
    uint64_t tri_tests;        /* triangle tests (48 B records)                                */
    uint64_t shape_tests;      /* instanced shape / fractal tests                              */
    double   ms_closest;       /* BLING_PASS_KERNEL_TIMING: summed k_trace_closest launch times */
    uint64_t closest_launches; /* BLING_PASS_KERNEL_TIMING: k_trace_closest launches timed      */
    uint64_t march_ticks;      /* BLING_PASS_TRAVERSAL_STATS: Mandelbulb march iterations (one
                                  bulbPower each, Fractal.hs:90-137)                            */
    /* BLING_PASS_TRAVERSAL_STATS, closest-hit queries only (the four counts above include the
       shadow rays' any-hit traversals): the work basis of the closest-hit kernel's roofline */
    uint64_t closest_node_visits, closest_tri_tests, closest_shape_tests, closest_march_ticks;
    double   ms_shade;         /* BLING_PASS_KERNEL_TIMING: summed launch times of the shading
                                  kernel: depth 0 and the fused resolve + shade launches      */
    uint64_t shade_launches;   /* BLING_PASS_KERNEL_TIMING: shade launches timed                */
} bling_stats;

/* Replaces: the process-wide GHC RTS + spark pool (bling.cabal:98-103, Rendering.hs:118).
 * device_ids: n_devices HIP device ordinals (NULL / 0 = device 0).  With n_devices > 1 the context
 * fans every bling_render_pass[_device] out over all of them: the scene is
 * replicated at upload, each device renders an interleaved share of the pass's tiles concurrently
 * as tile images (BLING_PASS_TILE_IMAGES), every peer pushes its images over xGMI onto
 * device_ids[0] (concurrent copies, one per peer stream), and they are added there (addTile) once
 * every device has succeeded, before the call returns.  bling_trace, bling_sample_li and the SPPM
 * calls run on device_ids[0] only.  One process per GPU (torch.distributed / RCCL) instead passes
 * one id per process and uses the shard fields.  A device id listed twice is BLING_EINVAL (unless
 * the environment sets BLING_ALLOW_REPEATED_DEVICES=1, a test hook that runs the fan-out with two
 * contexts on one GPU). */
int bling_create(const int* device_ids, int n_devices, bling_ctx** out);

/* Replaces: Scene.mkScene -> KdTree.mkKdTree (Scene.hs:37-43, KdTree.hs:107-139).  Builds a binned
 * SAH BVH2 on the host, flattens triangles/shapes/materials/lights to SoA and uploads them. */
int bling_scene_upload(bling_ctx* ctx, const bling_scene_desc* desc);

/* The checks bling_scene_upload makes of a scene description before any device work (render
 * config, texture graphs, host-folded material spectra, lights, images), without a context or a
 * device: the parser's error path (parseJob, IO/RenderJob.hs:31-34, and the `fail` paths of
 * IO/ParserCore.hs:147-186, fail at parse time) for a description built
 * elsewhere.  BLING_OK or BLING_EINVAL with bling_last_error() set. */
int bling_scene_validate(const bling_scene_desc* desc);

/* Replaces: prender's onePass (Rendering.hs:127-140) for the `sampler` renderer with its `path`
 * (Integrator/Path.hs) or `directLighting` (Integrator/DirectLighting.hs) surface integrator,
 * selected by desc->config.integrator at upload (directLighting maxDepth must lie in [1, 16]).
 * film_out: host buffer of width*height*4 floats (W, X, Y, Z per pixel, Image.hs:64-71),
 * ACCUMULATED into (pass several passes to get the progressive sum); may be NULL.  On a multi-device
 * context the film holds the sum over all devices; stats sum the counts (times: the slowest device,
 * ms_total = host wall time of the whole fan-out including the film merge). */
int bling_render_pass(bling_ctx* ctx, const bling_pass_params* p, float* film_out,
                      bling_stats* stats);

/* Replaces: prender's whole progressive loop with its ProgressReporter (Rendering.hs:60-78, 111-140):
 * passes p->pass_index, p->pass_index + 1, ... each accumulated into film_out (host, width*height*4,
 * as bling_render_pass; may be NULL), and after each one report(user, &ev) with ev.kind =
 * BLING_PROGRESS_PASS_DONE, the pass number, the accumulated film (finalImg) and splat weight 1
 * (`PassDone pass img' 1`); the loop stops when report returns 0 (`if cont then onePass (pass + 1)`).
 * With BLING_PASS_REGION_EVENTS in p->flags, each PassDone is preceded by prender's per-tile
 * reports (`RegionStarted w`, then `SamplesAdded w img'`, Rendering.hs:130-134) for every sample
 * window of the pass in tile order; their return values are ignored, as the reference ignores them.
 * The device renders the pass as a whole into its tile images; with a host film on a single-device
 * context they come back to the host and are added one window after another (addTile in the
 * reference's window order), so every SamplesAdded carries the film up to and including its window,
 * as the reference's does.  On a multi-device context (or with film_out NULL) the reports follow the
 * pass and carry the film after the whole pass.  stats (may be NULL)
 * sums the counts of every pass and takes the times' sum.  report must not be NULL (the reference
 * always has a reporter). */
typedef struct bling_progress {
    int32_t      kind;         /* BLING_PROGRESS_* (the constructors of Progress, Rendering.hs:60-73) */
    int32_t      pass;         /* progPassNum (every kind: the pass the event belongs to)        */
    const float* film;         /* finalImg / SamplesAdded's image: film_out after this pass, or (single
                                  device) up to this window; NULL if film_out is NULL or for
                                  RegionStarted                                                   */
    float        splat_weight; /* splatWeight (1)                                                */
    const struct bling_stats* pass_stats;   /* PassDone: this pass's counters and times (not the running
                                               sum); NULL otherwise                                */
    int32_t      region[4];    /* RegionStarted / SamplesAdded: the SampleWindow x0, x1, y0, y1 (inclusive) */
} bling_progress;
#define BLING_PROGRESS_STARTED        0
#define BLING_PROGRESS_SAMPLES_ADDED  1
#define BLING_PROGRESS_REGION_STARTED 2
#define BLING_PROGRESS_PASS_DONE      3
typedef int (*bling_progress_fn)(void* user, const bling_progress* ev);
int bling_render(bling_ctx* ctx, const bling_pass_params* p, float* film_out, bling_progress_fn report, void* user,
                 bling_stats* stats);

/* Same as bling_render_pass, but accumulates into a DEVICE film buffer (width*height*4 floats on
 * device_ids[0]) that the caller owns -- e.g. a tensor later reduced over RCCL. */
int bling_render_pass_device(bling_ctx* ctx, const bling_pass_params* p, void* film_device,
                             bling_stats* stats);

/* The tile-image layout of a pass (BLING_PASS_TILE_IMAGES) with p's shard and stride: *n_tiles
 * slots of *slot_w x *slot_h x 4 floats (15 + floor(0.5 + filter width) square for the square
 * filters); origins_out (2 ints per slot: the tile image's film x, y) may be NULL. */
int bling_pass_tile_layout(bling_ctx* ctx, const bling_pass_params* p, int32_t* origins_out, size_t* n_tiles,
                           int32_t* slot_w, int32_t* slot_h);

/* addTile (Image.hs:178-199) of the tile images of p's shard / stride (tiles_device, written by a
 * BLING_PASS_TILE_IMAGES pass of that shard, possibly on another rank) into film_device (width *
 * height * 4 floats), both device buffers on device_ids[0]. */
int bling_film_add_tiles(bling_ctx* ctx, const bling_pass_params* p, const void* tiles_device, void* film_device);

/* The same for every rank of a multi-rank pass at once (the merge after the gather): tiles_devices
 * holds p->shard_world device pointers, rank r's tile images (shard (r, shard_world), p's stride);
 * one launch adds them all into film_device. */
int bling_film_add_shards(bling_ctx* ctx, const bling_pass_params* p, const void* const* tiles_devices,
                          void* film_device);

/* Replaces: Scene.scIntersect / Scene.occluded for a batch (Scene.hs:45-51 -> KdTree.hs:236-246).
 * rays_soa: 8 planes of n floats (ox, oy, oz, dx, dy, dz, tmin, tmax).
 * closest (any_hit=0): t_out[n], prim_out[n] (index into desc->prim_kind order, BLING_MISS on
 * miss), bary_out[2n] (triangle b1,b2 / shape u,v); any_hit=1: prim_out[i] = 1 if occluded else 0
 * (t_out, bary_out may be NULL).  Host buffers. */
int bling_trace(bling_ctx* ctx, const float* rays_soa, size_t n, int any_hit,
                float* t_out, uint32_t* prim_out, float* bary_out);

/* Device-pointer variant of bling_trace for benchmarks (no host copies); timing via ms_out. */
int bling_trace_device(bling_ctx* ctx, const void* rays_soa_dev, size_t n, int any_hit,
                       void* t_dev, void* prim_dev, void* bary_dev, int repeats, double* ms_out);

/* Parity hook: radiance of individual camera samples, Path.li for sample n of extent pixel
 * (x, y) (Integrator/Path.hs:38-39 after Camera.fireRay).  samples: 3 ints (x, y, n) per sample;
 * L_out: 16 floats per sample (the spectrum before addSample's NaN filter); img_out: 2 floats per
 * sample (imageX, imageY), may be NULL.  Host buffers. */
int bling_sample_li(bling_ctx* ctx, uint32_t seed, uint32_t pass_index, const int32_t* samples, size_t n,
                    float* L_out, float* img_out, bling_stats* stats);

/* Debug hook (parity diagnosis): bling_sample_li plus one record of BLING_DV_FIELDS floats per path
 * vertex (vertex d of sample k at vtx_out[(k * BLING_DV_DEPTHS + d) * BLING_DV_FIELDS]; NaN where a
 * vertex or field was not reached).  The oracle's oracle_sample_li_vertices writes the same fields,
 * so the first field where the two differ names the first operation that diverges.  Only a build
 * with BLING_DEBUG_VERTEX (`make variant V=dbg DEFS=-DBLING_DEBUG_VERTEX=1`) records; the product
 * library returns BLING_EUNSUPPORTED.  Path integrator only.  Fields, in the vertex's order:
 *   0-2 ray origin, 3-5 ray direction, 6 hit t (Path.hs:41, scIntersect)
 *   7-9 shading point p, 10-12 geometric normal, 13 ray epsilon (mkIntersection, DG)
 *   14-16 light-sample wi, 17 its pdf (Light.sample, Scene.hs:61-69)
 *   18-20 BSDF-MIS wi, 21 its pdf (sampleBsdf, Scene.hs:71-82)
 *   22-24 continuation wi, 25 its pdf (Path.hs:74-79)
 *   26 Russian-roulette pc, 27 its uniform (Path.hs:68-72)
 *   28 shadow ray occluded (1 / 0), 29 BSDF-MIS ray hit t (inf = miss)
 *   30 sum of the vertex's 16-band radiance term, 31 sum of L after the vertex (Path.hs:73-79) */
#define BLING_DV_DEPTHS 16
#define BLING_DV_FIELDS 32
int bling_sample_li_vertices(bling_ctx* ctx, uint32_t seed, uint32_t pass_index, const int32_t* samples, size_t n,
                             float* L_out, float* vtx_out);

/* ---- SPPM renderer (Renderer/SPPM.hs), the second consumer of the trace core ---- */
typedef struct bling_sppm_stats {
    uint64_t hitpoints;        /* hit points recorded by the eye pass (mkHitPoints)              */
    uint64_t photons;          /* photons emitted: sppm_threads * sn^2 (SPPM.hs:449, 474)         */
    uint64_t photon_rays;      /* closest-hit queries of photon segments (followPhoton)           */
    uint64_t photon_hits;      /* (photon hit, hit point) pairs within the hit point's radius      */
    uint64_t cam_rays;         /* closest-hit queries of eye rays (traceCam)                      */
    uint64_t dropped;          /* NaN / Inf eye samples and splats skipped                        */
    double   ms_total, ms_eye, ms_hash, ms_photon;   /* device time (HIP events)                  */
} bling_sppm_stats;

/* Replaces: SPPM's onePass (Renderer/SPPM.hs:424-460) for a scene whose renderer block is
 * `sppm photonCount maxDepth radius [alpha]` (maxDepth in [1, 16]): one random camera sample per
 * sample-extent pixel builds the hit points (their Ls is addSample'd into film_out, W*H*4), then
 * sppm_threads * sn^2 photons splat into splat_out (W*H*3 XYZ, splatSample); both host buffers are
 * ACCUMULATED into and may be NULL.  The per-pixel radius statistics (psR2, psN) live in the
 * context and carry over to the next pass; pass_index numbers passes from 1 like onePass.  The
 * reference's image of pass k is getPixel with splat weight 1 / (threads * k * sn^2) (:460). */
int bling_sppm_pass(bling_ctx* ctx, uint32_t seed, uint32_t pass_index, float* film_out, float* splat_out,
                    bling_sppm_stats* stats);

/* The per-pixel statistics (PixelStats psR2 / psN, SPPM.hs:245-257) over the sample extent, in
 * sIdx order (windowPixels entries, written to *n_pixels); r2_out / n_out may be NULL. */
int bling_sppm_pixel_stats(bling_ctx* ctx, float* r2_out, float* n_out, size_t* n_pixels);

/* Restarts the SPPM statistics (every radius back to the scene's initial radius). */
int bling_sppm_reset(bling_ctx* ctx);

/* Diagnostics: the hit points of the last SPPM pass, in the device's (arbitrary) order -- shading
 * point and radius^2 (4 floats each) and the key pixel << 24 | eye-tree node id that orders the
 * kd-trees' ties.  *n receives the count; at most cap are copied (either array may be NULL). */
int bling_debug_sppm_hitpoints(bling_ctx* ctx, float* pos_r2, uint64_t* keys, size_t cap, size_t* n);
/* Diagnostics: the last SPPM pass's hash buckets as its kd-trees laid them out (k_sppm_kd): bucket
 * offsets (*nb = buckets + 1), hit point indices per bucket in kd order, and per entry the node's
 * mr at pivot positions (*ni entries).  Arrays are copied only when their capacity suffices. */
int bling_debug_sppm_buckets(bling_ctx* ctx, uint32_t* bstart, uint32_t* items, float* mr, size_t cap_b,
                             size_t cap_i, size_t* nb, size_t* ni);

/* Diagnostics (no reference counterpart): the path-state bytes the shading kernel k_shade moved in
 * the context's last bling_render_pass*, per stream and direction -- out[2 k] read, out[2 k + 1]
 * written, stream k in the order BLING_STREAM_NAMES lists -- counted where the algorithm needs
 * them (a record the path uses), for the roofline's algorithmic bytes (DESIGN.md "Roofline").
 * Counted only by a BLING_STREAM_STATS build (make variant V=streams DEFS=-DBLING_STREAM_STATS=1);
 * other builds return BLING_EUNSUPPORTED.  *n_streams receives the stream count; out may be NULL. */
#define BLING_STREAM_NAMES "queue,hit,meta,org,dir,mdir,mhit,occ,fac,cf,T,L,Tn,lsc,bsc,sh_o,sh_d,result,qflag"
#define BLING_N_STREAMS 19
int bling_debug_stream_bytes(bling_ctx* ctx, uint64_t* out, size_t n, size_t* n_streams);

/* The uploaded scene's acceleration / kernel plan as one JSON object (BVH2 and BVH4 depth and
 * sizes, the BVH4 stack bound, the LDS plans, the packet walk, the in-line shadow test), written
 * NUL-terminated into buf (at most size bytes); *len (may be NULL) receives the full length.
 * Diagnostics for bench.py and the tests; no reference counterpart. */
int bling_debug_scene_info(bling_ctx* ctx, char* buf, size_t size, size_t* len);

/* Frees every device resource of the context. */
void bling_destroy(bling_ctx* ctx);

/* Thread-local description of the last error on this thread. */
const char* bling_last_error(void);

/* Build identification (arch, compile flags) for reports. */
const char* bling_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BLING_H */
