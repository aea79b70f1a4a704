"""Host-side mirror of the reference's renderer interface over the MI355X core (libbling_hip.so).

Reference interface (src/lib/Graphics/Bling/Rendering.hs):
  * ``class Renderer a where render :: a -> RenderJob -> ProgressReporter -> IO ()``   (:77-78)
  * ``SamplerRenderer`` / ``prender``: progressive passes, each pass = every tile once (:252-296)
  * ``Progress`` events ``Started``/``RegionStarted``/``SamplesAdded``/``PassDone`` (:60-73); the
    reporter returns False to stop after a pass (:136-137)
Here the per-pass work is one ``bling_render_pass`` call (the whole tile list on the GPU), so the
progress stream is ``Started`` then one ``PassDone`` per pass.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _ffi
from .scene import Job

DEFAULT_SEED = 0x0B11A6   # master seed of the benchmark


class BlingError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"bling error {rc}: {msg}")
        self.rc = rc


def _check(rc: int):
    if rc != 0:
        raise BlingError(rc, _ffi.hip().bling_last_error().decode())


class Context:
    """One bling_ctx (bling_create / bling_destroy) on one HIP device, or on several: a list of
    device ids makes every render pass fan out over all of them inside the library (include/bling.h,
    bling_create), with the summed film on the first device."""

    def __init__(self, device: int | list[int] = 0):
        lib = _ffi.hip()
        h = C.c_void_p()
        ids = [device] if isinstance(device, int) else list(device)
        dev = (C.c_int * len(ids))(*ids)
        _check(lib.bling_create(dev, len(ids), C.byref(h)))
        self._h = h
        self.device = ids[0]
        self.devices = ids
        self.job: Job | None = None

    def upload(self, job: Job):
        """bling_scene_upload (replaces Scene.mkScene -> mkKdTree)."""
        _check(_ffi.hip().bling_scene_upload(self._h, C.c_void_p(job.desc)))
        self.job = job

    def render_pass(self, seed=DEFAULT_SEED, pass_index=0, shard=(0, 1), tile_stride=1, chunk_paths=0,
                    film: np.ndarray | None = None, flags=0):
        """One pass into a host film (accumulated). Returns (film, Stats)."""
        job = self.job
        if film is None:
            film = np.zeros(job.width * job.height * 4, np.float32)
        pp = _ffi.PassParams(seed, pass_index, shard[0], shard[1], tile_stride, chunk_paths, flags)
        st = _ffi.Stats()
        _check(_ffi.hip().bling_render_pass(self._h, C.byref(pp), _ffi.f32ptr(film), C.byref(st)))
        return film, st

    def render_loop(self, report, seed=DEFAULT_SEED, first_pass=1, film: np.ndarray | None = None, shard=(0, 1),
                    tile_stride=1, regions=None):
        """bling_render: passes first_pass, first_pass + 1, ... into a host film until report(pass,
        film, stats) returns False (prender's onePass loop with its ProgressReporter,
        Rendering.hs:127-140); stats is that pass's own bling_stats as a dict.  With regions (a
        callable), every pass first reports prender's per-window events as regions(kind, pass,
        (x0, x1, y0, y1), film) with kind "region_started" (film None) or "samples_added"
        (BLING_PASS_REGION_EVENTS).  Returns (film, Stats summed over the passes)."""
        job = self.job
        if film is None:
            film = np.zeros(job.width * job.height * 4, np.float32)
        flags = _ffi.PASS_REGION_EVENTS if regions is not None else 0
        pp = _ffi.PassParams(seed, first_pass, shard[0], shard[1], tile_stride, 0, flags)
        st = _ffi.Stats()
        err = []
        kinds = {_ffi.PROGRESS_REGION_STARTED: "region_started", _ffi.PROGRESS_SAMPLES_ADDED: "samples_added"}

        def cb(_user, ev):
            try:
                e = ev.contents
                if e.kind in kinds:
                    regions(kinds[e.kind], int(e.pass_), tuple(int(v) for v in e.region),
                            film if e.kind == _ffi.PROGRESS_SAMPLES_ADDED else None)
                    return 1
                assert e.kind == _ffi.PROGRESS_PASS_DONE
                one = e.pass_stats.contents.as_dict() if e.pass_stats else {}
                return 1 if report(int(e.pass_), film, one) else 0
            except Exception as ex:          # never unwind through the C frame
                err.append(ex)
                return 0
        fn = _ffi.ProgressFn(cb)
        _check(_ffi.hip().bling_render(self._h, C.byref(pp), _ffi.f32ptr(film), fn, None, C.byref(st)))
        if err:
            raise err[0]
        return film, st

    def scene_info(self) -> dict:
        """bling_debug_scene_info: the uploaded scene's acceleration / kernel plan."""
        import json
        buf = C.create_string_buffer(1024)
        _check(_ffi.hip().bling_debug_scene_info(self._h, buf, len(buf), None))
        return json.loads(buf.value.decode())

    def stream_bytes(self) -> dict:
        """bling_debug_stream_bytes: k_shade's path-state bytes of the last pass per stream,
        {name: (read, written)} (BLING_STREAM_STATS builds only)."""
        n = C.c_size_t()
        out = (C.c_uint64 * (2 * len(_ffi.STREAM_NAMES)))()
        _check(_ffi.hip().bling_debug_stream_bytes(self._h, out, len(out), C.byref(n)))
        return {k: (int(out[2 * i]), int(out[2 * i + 1])) for i, k in enumerate(_ffi.STREAM_NAMES)}

    def render_pass_device(self, film_ptr: int, seed=DEFAULT_SEED, pass_index=0, shard=(0, 1), tile_stride=1,
                           chunk_paths=0, flags=0):
        """One pass accumulated into a device film (e.g. ``torch_tensor.data_ptr()``)."""
        pp = _ffi.PassParams(seed, pass_index, shard[0], shard[1], tile_stride, chunk_paths, flags)
        st = _ffi.Stats()
        _check(_ffi.hip().bling_render_pass_device(self._h, C.byref(pp), C.c_void_p(film_ptr), C.byref(st)))
        return st

    def tile_layout(self, shard=(0, 1), tile_stride=1):
        """bling_pass_tile_layout: (origins (n, 2) int32, slot_w, slot_h) of a tile-image pass."""
        pp = _ffi.PassParams(0, 0, shard[0], shard[1], tile_stride, 0, 0, None)
        n, sw, sh = C.c_size_t(), C.c_int32(), C.c_int32()
        _check(_ffi.hip().bling_pass_tile_layout(self._h, C.byref(pp), None, C.byref(n), C.byref(sw), C.byref(sh)))
        org = np.zeros((n.value, 2), np.int32)
        if n.value:
            _check(_ffi.hip().bling_pass_tile_layout(self._h, C.byref(pp), org.ctypes.data_as(C.POINTER(C.c_int32)),
                                                     C.byref(n), C.byref(sw), C.byref(sh)))
        return org, sw.value, sh.value

    @staticmethod
    def _tiles_buf(buf, capacity):
        """(device pointer, floats it holds) of a tile-image buffer.  A tensor-like buffer (anything
        with data_ptr() and numel(), e.g. a torch tensor) carries its own size (capacity, if given,
        may only lower it); a raw integer pointer must come with its capacity -- the core refuses a
        layout that needs more floats than that (include/bling.h bling_pass_params.tiles_capacity)."""
        if hasattr(buf, "data_ptr") and hasattr(buf, "numel"):
            # the capacity is counted in float32 slots: refuse any other element type (a float16
            # tensor's numel would claim twice the bytes it holds) and host tensors
            dt = getattr(buf, "dtype", None)
            if dt is not None and str(dt) not in ("torch.float32", "float32"):
                raise ValueError(f"tile-image buffer must be float32, got {dt}")
            if hasattr(buf, "is_cuda") and not buf.is_cuda:
                raise ValueError("tile-image buffer must be a device tensor")
            n = int(buf.numel())
            return int(buf.data_ptr()), n if capacity is None else min(n, int(capacity))
        if capacity is None:
            raise ValueError("tiles_capacity is required with a raw device pointer (pass the tensor to size it)")
        return int(buf), int(capacity)

    def render_pass_tiles(self, tiles, seed=DEFAULT_SEED, pass_index=0, shard=(0, 1), tile_stride=1,
                          chunk_paths=0, flags=0, tiles_capacity=None):
        """One pass written as tile images into a device buffer (BLING_PASS_TILE_IMAGES, layout
        tile_layout) instead of a film -- the per-rank half of the multi-GPU merge.  tiles: a device
        tensor, or a raw pointer with tiles_capacity (floats)."""
        ptr, cap = self._tiles_buf(tiles, tiles_capacity)
        pp = _ffi.PassParams(seed, pass_index, shard[0], shard[1], tile_stride, chunk_paths,
                             flags | _ffi.PASS_TILE_IMAGES, C.c_void_p(ptr), cap)
        st = _ffi.Stats()
        _check(_ffi.hip().bling_render_pass_device(self._h, C.byref(pp), None, C.byref(st)))
        return st

    def film_add_tiles(self, tiles, film_ptr: int, shard=(0, 1), tile_stride=1, tiles_capacity=None):
        """bling_film_add_tiles: addTile of one shard's tile images into a device film."""
        ptr, cap = self._tiles_buf(tiles, tiles_capacity)
        pp = _ffi.PassParams(0, 0, shard[0], shard[1], tile_stride, 0, 0, None, cap)
        _check(_ffi.hip().bling_film_add_tiles(self._h, C.byref(pp), C.c_void_p(ptr), C.c_void_p(film_ptr)))

    def film_add_shards(self, tiles_list, film_ptr: int, tile_stride=1, tiles_capacity=None):
        """bling_film_add_shards: every rank's tile images (rank r's buffer tiles_list[r]) into a
        device film in one launch -- rank 0's merge after the gather.  The capacity checked against
        each rank's layout is the smallest buffer's (tensors), or tiles_capacity (raw pointers)."""
        world = len(tiles_list)
        bufs = [self._tiles_buf(b, tiles_capacity) for b in tiles_list]
        pp = _ffi.PassParams(0, 0, 0, world, tile_stride, 0, 0, None, min(c for _, c in bufs))
        arr = (C.c_void_p * world)(*[C.c_void_p(p) for p, _ in bufs])
        _check(_ffi.hip().bling_film_add_shards(self._h, C.byref(pp), arr, C.c_void_p(film_ptr)))

    def trace(self, rays_soa: np.ndarray, any_hit: bool = False):
        """Scene.scIntersect / Scene.occluded for a batch of rays (8 x n SoA)."""
        rays_soa = np.ascontiguousarray(rays_soa, np.float32)
        n = rays_soa.shape[1]
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.uint32)
        bary = np.zeros(2 * n, np.float32)
        _check(_ffi.hip().bling_trace(self._h, _ffi.f32ptr(rays_soa), n, 1 if any_hit else 0, _ffi.f32ptr(t),
                                      _ffi.u32ptr(prim), _ffi.f32ptr(bary)))
        return t, prim, bary.reshape(n, 2)

    def sample_li(self, samples: np.ndarray, seed=DEFAULT_SEED, pass_index=0):
        """Per-sample Path.li on the device; samples = int32 (k, 3) of (x, y, n)."""
        samples = np.ascontiguousarray(samples, np.int32)
        n = samples.shape[0]
        L = np.zeros((n, 16), np.float32)
        img = np.zeros((n, 2), np.float32)
        st = _ffi.Stats()
        lib = _ffi.hip()
        lib.bling_sample_li.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t,
                                        _ffi.c_f32p, _ffi.c_f32p, C.POINTER(_ffi.Stats)]
        _check(lib.bling_sample_li(self._h, seed, pass_index, samples.ctypes.data_as(C.POINTER(C.c_int32)), n,
                                   _ffi.f32ptr(L), _ffi.f32ptr(img), C.byref(st)))
        return L, img, st

    def sample_li_vertices(self, samples: np.ndarray, seed=DEFAULT_SEED, pass_index=0):
        """sample_li plus the per-vertex debug records (include/bling.h BLING_DV_*): (L (k, 16),
        vtx (k, 16, 32)).  Needs the BLING_DEBUG_VERTEX build (BLING_HIP_VARIANT=dbg); the product
        library raises BlingError(BLING_EUNSUPPORTED)."""
        samples = np.ascontiguousarray(samples, np.int32)
        n = samples.shape[0]
        L = np.zeros((n, 16), np.float32)
        vtx = np.zeros((n, 16, 32), np.float32)
        lib = _ffi.hip()
        lib.bling_sample_li_vertices.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t,
                                                 _ffi.c_f32p, _ffi.c_f32p]
        _check(lib.bling_sample_li_vertices(self._h, seed, pass_index, samples.ctypes.data_as(C.POINTER(C.c_int32)), n,
                                            _ffi.f32ptr(L), _ffi.f32ptr(vtx)))
        return L, vtx

    def sppm_pass(self, seed=DEFAULT_SEED, pass_index=1, film: np.ndarray | None = None,
                  splat: np.ndarray | None = None):
        """One SPPM onePass (Renderer/SPPM.hs:424-460) into host film (W,X,Y,Z) and splat (X,Y,Z)
        buffers, both accumulated.  Returns (film, splat, SppmStats)."""
        job = self.job
        if film is None:
            film = np.zeros(job.width * job.height * 4, np.float32)
        if splat is None:
            splat = np.zeros(job.width * job.height * 3, np.float32)
        st = _ffi.SppmStats()
        _check(_ffi.hip().bling_sppm_pass(self._h, seed, pass_index, _ffi.f32ptr(film), _ffi.f32ptr(splat),
                                          C.byref(st)))
        return film, splat, st

    def sppm_pixel_stats(self):
        """(psR2, psN) over the sample extent in sIdx order."""
        n = C.c_size_t()
        _check(_ffi.hip().bling_sppm_pixel_stats(self._h, None, None, C.byref(n)))
        r2 = np.zeros(n.value, np.float32)
        nn = np.zeros(n.value, np.float32)
        _check(_ffi.hip().bling_sppm_pixel_stats(self._h, _ffi.f32ptr(r2), _ffi.f32ptr(nn), C.byref(n)))
        return r2, nn

    def sppm_hitpoints(self):
        """bling_debug_sppm_hitpoints: (pos_r2 (n, 4) float32, keys (n,) uint64) of the last SPPM pass."""
        n = C.c_size_t()
        _check(_ffi.hip().bling_debug_sppm_hitpoints(self._h, None, None, 0, C.byref(n)))
        pos = np.zeros((n.value, 4), np.float32)
        keys = np.zeros(n.value, np.uint64)
        _check(_ffi.hip().bling_debug_sppm_hitpoints(self._h, _ffi.f32ptr(pos.reshape(-1)),
                                                     keys.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n)))
        return pos, keys

    def sppm_buckets(self):
        """bling_debug_sppm_buckets: (bstart, items, mr) of the last SPPM pass's kd-tree buckets."""
        nb, ni = C.c_size_t(), C.c_size_t()
        _check(_ffi.hip().bling_debug_sppm_buckets(self._h, None, None, None, 0, 0, C.byref(nb), C.byref(ni)))
        bs = np.zeros(nb.value, np.uint32); it = np.zeros(ni.value, np.uint32); mr = np.zeros(ni.value, np.float32)
        u32 = C.POINTER(C.c_uint32)
        _check(_ffi.hip().bling_debug_sppm_buckets(self._h, bs.ctypes.data_as(u32), it.ctypes.data_as(u32), _ffi.f32ptr(mr),
                                                   nb.value, ni.value, C.byref(nb), C.byref(ni)))
        return bs, it, mr

    def sppm_reset(self):
        _check(_ffi.hip().bling_sppm_reset(self._h))

    def close(self):
        if self._h:
            _ffi.hip().bling_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- Renderer interface
@dataclass
class Progress:
    kind: str                     # "Started" | "PassDone"
    pass_num: int = 0
    film: np.ndarray | None = None
    stats: dict = field(default_factory=dict)


class SamplerRenderer:
    """``SamplerRenderer`` with the path integrator (Rendering.hs:111-140) on the MI355X core."""

    def __init__(self, device: int = 0, seed: int = DEFAULT_SEED):
        self.device = device
        self.seed = seed

    def render(self, job: Job, report) -> np.ndarray:
        """Passes 1, 2, ... through bling_render (the core's own pass loop) until the reporter
        returns False; each PassDone carries the accumulated film."""
        ctx = Context(self.device)
        ctx.upload(job)
        report(Progress("Started"))
        film, _ = ctx.render_loop(lambda p, f, st: bool(report(Progress("PassDone", p, f, st))), seed=self.seed,
                                  first_pass=1)
        ctx.close()
        return film


class SPPMRenderer:
    """``instance Renderer SPPM`` (Renderer/SPPM.hs:466-480) on the MI355X core: passes 1, 2, ...
    until the reporter returns False; each PassDone carries the film, the photon splat and the
    splat weight 1 / (threads * pass * sn^2) that getPixel applies (:460)."""

    def __init__(self, device: int = 0, seed: int = DEFAULT_SEED):
        self.device = device
        self.seed = seed

    def render(self, job: Job, report):
        cfg = job.config
        threads = max(1, cfg.sppm_threads)
        sn = max(1, int(np.ceil(np.sqrt(np.float32(cfg.sppm_photons) / np.float32(threads)))))
        ctx = Context(self.device)
        ctx.upload(job)
        film = np.zeros(job.width * job.height * 4, np.float32)
        splat = np.zeros(job.width * job.height * 3, np.float32)
        report(Progress("Started"))
        p = 1
        while True:
            film, splat, st = ctx.sppm_pass(seed=self.seed, pass_index=p, film=film, splat=splat)
            info = st.as_dict()
            info["splat"] = splat
            info["splat_weight"] = 1.0 / (threads * p * sn * sn)
            if not report(Progress("PassDone", p, film, info)):
                break
            p += 1
        ctx.close()
        return film, splat


def render(job: Job, passes: int = 1, device: int = 0, seed: int = DEFAULT_SEED) -> np.ndarray:
    """Render `passes` progressive passes (the commented bling CLI harness renders exactly one,
    src/cmdline/Main.hs:15-26)."""
    count = {"n": 0}

    def rep(pr: Progress) -> bool:
        if pr.kind == "PassDone":
            count["n"] += 1
            return count["n"] < passes
        return True

    return SamplerRenderer(device, seed).render(job, rep)
