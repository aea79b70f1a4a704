"""ORACLE ctypes wrapper -- test infrastructure only.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product
package.  Loads oracle/_build/liboracle.so (built by ``make oracle``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "liboracle.so")
f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)


class OracleStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("rays_camera", C.c_uint64), ("rays_continuation", C.c_uint64),
                ("rays_mis", C.c_uint64), ("rays_shadow", C.c_uint64), ("dropped", C.c_uint64),
                ("kd_nodes", C.c_uint64), ("kd_leaf_prims", C.c_uint64), ("seconds", C.c_double)]

    def rays(self) -> int:
        return int(self.rays_camera + self.rays_continuation + self.rays_mis + self.rays_shadow)


class OracleSppmStats(C.Structure):
    _fields_ = [("hitpoints", C.c_uint64), ("photons", C.c_uint64), ("photon_rays", C.c_uint64),
                ("photon_hits", C.c_uint64), ("cam_rays", C.c_uint64), ("dropped", C.c_uint64),
                ("seconds", C.c_double)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        L.oracle_build.argtypes = [C.c_void_p]
        L.oracle_build.restype = C.c_void_p
        L.oracle_free.argtypes = [C.c_void_p]
        L.oracle_info.argtypes = [C.c_void_p]
        L.oracle_info.restype = C.c_char_p
        L.oracle_render.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, f32p, C.POINTER(OracleStats)]
        L.oracle_render_shard.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, f32p,
                                          C.POINTER(OracleStats)]
        L.oracle_sample_li.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, f32p, f32p,
                                       C.POINTER(OracleStats)]
        L.oracle_sample_li_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int), C.c_size_t, f32p,
                                             f32p, C.c_int, C.POINTER(OracleStats)]
        L.oracle_sample_li_vertices.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int), C.c_size_t,
                                                f32p, f32p, C.c_int]
        L.oracle_set_libm32.argtypes = [C.c_int]
        L.oracle_sppm_set_lookup.argtypes = [C.c_int]
        L.oracle_sppm_hitpoints.argtypes = [C.c_void_p, f32p, C.POINTER(C.c_uint64), C.c_size_t]
        L.oracle_sppm_hitpoints.restype = C.c_size_t
        L.oracle_sppm_buckets.argtypes = [C.c_void_p, u32p, u32p, f32p, C.POINTER(C.c_size_t)]
        L.oracle_sppm_buckets.restype = C.c_size_t
        L.oracle_cr_eval.argtypes = [C.c_int, f32p, f32p, f32p, C.c_size_t]
        L.oracle_render_tiles.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int,
                                          f32p, C.POINTER(C.c_int), C.POINTER(OracleStats)]
        L.oracle_camera_ray.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, f32p]
        L.oracle_trace.argtypes = [C.c_void_p, f32p, C.c_size_t, C.c_int, f32p, u32p, f32p, C.POINTER(OracleStats)]
        L.oracle_sampler_probe.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_int, f32p]
        L.oracle_hash5.argtypes = [C.c_uint32] * 5
        L.oracle_hash5.restype = C.c_uint32
        L.oracle_permute.argtypes = [C.c_uint32] * 3
        L.oracle_permute.restype = C.c_uint32
        L.oracle_concentric_disk.argtypes = [C.c_float, C.c_float, f32p]
        L.oracle_solve_quadric.argtypes = [C.c_float, C.c_float, C.c_float, f32p]
        L.oracle_solve_quadric.restype = C.c_int
        L.oracle_fr_dielectric.argtypes = [C.c_float, C.c_float, C.c_float, f32p]
        L.oracle_fr_conductor.argtypes = [f32p, f32p, C.c_float, f32p]
        L.oracle_fblend_eval.argtypes = [f32p, f32p, f32p, f32p, f32p, f32p, f32p]
        L.oracle_aniso_d.argtypes = [C.c_float, C.c_float, f32p]
        L.oracle_aniso_d.restype = C.c_float
        L.oracle_tri_probe.argtypes = [f32p, f32p, f32p]
        L.oracle_tri_probe.restype = C.c_int
        L.oracle_bxdf_probe.argtypes = [C.c_void_p, C.c_int, C.c_int, f32p, f32p, f32p, f32p]
        L.oracle_bxdf_probe.restype = C.c_int
        L.oracle_light_sample_probe.argtypes = [C.c_void_p, C.c_int, f32p, C.c_float, C.c_float, C.c_float, f32p]
        L.oracle_light_pdf_probe.argtypes = [C.c_void_p, C.c_int, f32p, f32p]
        L.oracle_light_pdf_probe.restype = C.c_float
        L.oracle_env_probe.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_float, f32p]
        L.oracle_fire_ray_probe.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_float, f32p]
        L.oracle_stex_probe.argtypes = [C.c_void_p, C.c_int, f32p]
        L.oracle_stex_probe.restype = C.c_float
        L.oracle_stex_probe_uv.argtypes = [C.c_void_p, C.c_int, f32p, C.c_float, C.c_float]
        L.oracle_stex_probe_uv.restype = C.c_float
        L.oracle_spectrum_probe.argtypes = [C.c_void_p, C.c_int, f32p, C.c_float, C.c_float, f32p]
        L.oracle_bump_probe.argtypes = [C.c_void_p, C.c_int, f32p, f32p]
        L.oracle_extent.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        L.oracle_set_rng.argtypes = [C.c_void_p, C.c_int]
        L.oracle_mwc_probe.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, u32p]
        L.oracle_sppm_new.argtypes = [C.c_void_p]
        L.oracle_sppm_new.restype = C.c_void_p
        L.oracle_sppm_free.argtypes = [C.c_void_p]
        L.oracle_sppm_pass.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, f32p, f32p,
                                       C.POINTER(OracleSppmStats)]
        L.oracle_sppm_pixel_stats.argtypes = [C.c_void_p, f32p, f32p]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(f32p)


class Oracle:
    """CPU restatement of the reference hot path over a parsed Job (bling_amd.scene.Job)."""

    def __init__(self, job):
        self.job = job  # keeps the desc alive
        self.h = lib().oracle_build(job.desc)

    def info(self) -> str:
        return lib().oracle_info(self.h).decode()

    def set_rng(self, mode: str) -> None:
        """Sampler RNG of render / render_tiles: "counter" (the product's, default) or "mwc" (the
        reference's MWC8222 tile streams, for statistical convergence checks only)."""
        if lib().oracle_set_rng(self.h, {"counter": 0, "mwc": 1}[mode]) < 0:
            raise ValueError(mode)

    def render(self, seed=0x0B11A6, pass_index=0, tile_stride=1, threads=0, film=None, shard=(0, 1)):
        w, h = self.job.width, self.job.height
        if film is None:
            film = np.zeros(w * h * 4, np.float32)
        st = OracleStats()
        rc = lib().oracle_render_shard(self.h, seed, pass_index, shard[0], shard[1], tile_stride, threads, _fp(film),
                                       C.byref(st))
        if rc != 0:
            raise RuntimeError("oracle_render failed (renderer is not sampler/path?)")
        return film, st

    def tile_slot(self):
        """(slot_w, slot_h) of a tile image: the largest mkImageTile of the filter."""
        return self.job.tile_slot()

    def render_tiles(self, seed=0x0B11A6, pass_index=0, shard=(0, 1), tile_stride=1, threads=0):
        """One shard's tile images: (tiles (n, slot_h, slot_w, 4), origins (n, 2), stats)."""
        sw, sh = self.tile_slot()
        (x0, x1, y0, y1), nt = self.extent()
        cap = nt // max(1, tile_stride) + 1
        tiles = np.zeros((cap, sh, sw, 4), np.float32)
        org = np.zeros((cap, 2), np.int32)
        st = OracleStats()
        n = lib().oracle_render_tiles(self.h, seed, pass_index, shard[0], shard[1], tile_stride, threads, _fp(tiles),
                                      org.ctypes.data_as(C.POINTER(C.c_int)), C.byref(st))
        if n < 0:
            raise RuntimeError("oracle_render_tiles failed")
        return tiles[:n], org[:n], st

    def sample_li(self, px, py, n, seed=0x0B11A6, pass_index=0):
        L = np.zeros(16, np.float32)
        xy = np.zeros(2, np.float32)
        st = OracleStats()
        lib().oracle_sample_li(self.h, seed, pass_index, px, py, n, _fp(L), _fp(xy), C.byref(st))
        return L, xy, st

    def sample_li_batch(self, samples: np.ndarray, seed=0x0B11A6, pass_index=0, threads=0):
        """sample_li over an int32 (k, 3) array of (x, y, n): (L (k, 16), img (k, 2), stats)."""
        samples = np.ascontiguousarray(samples, np.int32)
        k = samples.shape[0]
        L = np.zeros((k, 16), np.float32)
        xy = np.zeros((k, 2), np.float32)
        st = OracleStats()
        lib().oracle_sample_li_batch(self.h, seed, pass_index, samples.ctypes.data_as(C.POINTER(C.c_int)), k, _fp(L),
                                     _fp(xy), threads, C.byref(st))
        return L, xy, st

    def sample_li_vertices(self, samples: np.ndarray, seed=0x0B11A6, pass_index=0, threads=0):
        """Per-vertex debug records of sample_li (Path integrator): (L (k, 16), vtx (k, 16, 32)),
        NaN where a vertex / field was not reached.  Field map: include/bling.h BLING_DV_*."""
        samples = np.ascontiguousarray(samples, np.int32)
        k = samples.shape[0]
        L = np.zeros((k, 16), np.float32)
        vtx = np.zeros((k, 16, 32), np.float32)
        if lib().oracle_sample_li_vertices(self.h, seed, pass_index, samples.ctypes.data_as(C.POINTER(C.c_int)), k,
                                           _fp(L), _fp(vtx), threads) != 0:
            raise RuntimeError("oracle_sample_li_vertices: Path integrator only")
        return L, vtx

    def camera_ray(self, px, py, n, seed=0x0B11A6, pass_index=0):
        out = np.zeros(8, np.float32)
        lib().oracle_camera_ray(self.h, seed, pass_index, px, py, n, _fp(out))
        return out

    def trace(self, rays_soa: np.ndarray, any_hit=False):
        rays_soa = np.ascontiguousarray(rays_soa, np.float32)
        n = rays_soa.shape[1]
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.uint32)
        bary = np.zeros(2 * n, np.float32)
        st = OracleStats()
        lib().oracle_trace(self.h, _fp(rays_soa), n, 1 if any_hit else 0, _fp(t), prim.ctypes.data_as(u32p),
                           _fp(bary), C.byref(st))
        return t, prim, bary.reshape(n, 2), st

    def sampler_probe(self, px, py, n, kind, dim=0, seed=0x0B11A6, pass_index=0):
        out = np.zeros(4, np.float32)
        lib().oracle_sampler_probe(self.h, seed, pass_index, px, py, n, kind, dim, _fp(out))
        return out

    def extent(self):
        o = (C.c_int * 4)()
        nt = lib().oracle_extent(self.h, o)
        return tuple(o), nt

    def close(self):
        if self.h:
            lib().oracle_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OracleSppm:
    """CPU restatement of the SPPM renderer (Renderer/SPPM.hs); pixel statistics persist across passes."""

    def hitpoints(self):
        """(pos_r2 (n, 4) float32, keys (n,) uint64) of the last pass, in the oracle's order."""
        n = lib().oracle_sppm_hitpoints(self.h, None, None, 0)
        pos = np.zeros((n, 4), np.float32)
        keys = np.zeros(n, np.uint64)
        lib().oracle_sppm_hitpoints(self.h, _fp(pos.reshape(-1)), keys.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        return pos, keys

    def buckets(self):
        """(bstart, items, mr) of the last pass's kd-tree buckets."""
        n = C.c_size_t()
        nb = lib().oracle_sppm_buckets(self.h, None, None, None, C.byref(n))
        bs = np.zeros(nb, np.uint32); it = np.zeros(n.value, np.uint32); mr = np.zeros(n.value, np.float32)
        lib().oracle_sppm_buckets(self.h, bs.ctypes.data_as(u32p), it.ctypes.data_as(u32p), _fp(mr), C.byref(n))
        return bs, it, mr

    @staticmethod
    def set_lookup(all_within: bool):
        """Measurement only: True = every bucket entry within its radius instead of treeLookup's walk."""
        lib().oracle_sppm_set_lookup(1 if all_within else 0)

    def __init__(self, job):
        self.job = job
        self.oracle = Oracle(job)
        self.h = lib().oracle_sppm_new(self.oracle.h)
        if not self.h:
            raise RuntimeError("scene renderer is not sppm")
        (x0, x1, y0, y1), _ = self.oracle.extent()
        self.n_stats = (x1 - x0 + 1) * (y1 - y0 + 1)

    def render_pass(self, seed=0x0B11A6, pass_index=1, threads=0, film=None, splat=None):
        w, h = self.job.width, self.job.height
        film = np.zeros(w * h * 4, np.float32) if film is None else film
        splat = np.zeros(w * h * 3, np.float32) if splat is None else splat
        st = OracleSppmStats()
        if lib().oracle_sppm_pass(self.h, seed, pass_index, threads, _fp(film), _fp(splat), C.byref(st)) != 0:
            raise RuntimeError("oracle_sppm_pass failed")
        return film, splat, st

    def pixel_stats(self):
        r2 = np.zeros(self.n_stats, np.float32)
        n = np.zeros(self.n_stats, np.float32)
        lib().oracle_sppm_pixel_stats(self.h, _fp(r2), _fp(n))
        return r2, n

    def close(self):
        if self.h:
            lib().oracle_sppm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


CR_FUNCS = ["sin", "cos", "tan", "asin", "acos", "atan", "exp", "log", "sinh", "atan2", "pow", "sincos_s", "sincos_c"]


def cr_eval(name: str, x: np.ndarray, y: np.ndarray | None = None) -> np.ndarray:
    """common/cr_math.h's binary32 function `name` over x (and y for atan2 / pow), on the host."""
    x = np.ascontiguousarray(x, np.float32)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    out = np.zeros_like(x)
    if lib().oracle_cr_eval(CR_FUNCS.index(name), _fp(x), None if yy is None else _fp(yy), _fp(out), len(x)) != 0:
        raise ValueError(name)
    return out


def hash5(seed, pss, pixel, sample, dim) -> int:
    return int(lib().oracle_hash5(seed, pss, pixel, sample, dim))


def permute(i, l, p) -> int:
    return int(lib().oracle_permute(i, l, p))
