"""ctypes bindings for the two product shared libraries.

* ``libbling_host.so``  -- the `.bling` loader + film output (include/bling_host.h)
* ``libbling_hip.so``   -- the MI355X core (include/bling.h)

Both are built in-tree by ``make`` (see ``__graft_entry__.build``).  Nothing here falls back to a
CPU implementation: if the HIP library cannot be loaded, :func:`hip` raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(_HERE, "_lib")

c_f32p = C.POINTER(C.c_float)
c_u32p = C.POINTER(C.c_uint32)


PASS_TRAVERSAL_STATS = 1   # BLING_PASS_TRAVERSAL_STATS
PASS_KERNEL_TIMING = 2     # BLING_PASS_KERNEL_TIMING
PASS_TILE_IMAGES = 4       # BLING_PASS_TILE_IMAGES
PASS_REGION_EVENTS = 8     # BLING_PASS_REGION_EVENTS (bling_render only)


class PassParams(C.Structure):
    """bling_pass_params (include/bling.h)."""
    _fields_ = [("seed", C.c_uint32), ("pass_index", C.c_uint32), ("shard_rank", C.c_int32),
                ("shard_world", C.c_int32), ("tile_stride", C.c_int32), ("chunk_paths", C.c_int32),
                ("flags", C.c_uint32), ("tiles_device", C.c_void_p), ("tiles_capacity", C.c_uint64)]


class Stats(C.Structure):
    """bling_stats (include/bling.h)."""
    _fields_ = [("camera_samples", C.c_uint64), ("rays_camera", C.c_uint64),
                ("rays_continuation", C.c_uint64), ("rays_mis", C.c_uint64),
                ("rays_shadow", C.c_uint64), ("dropped_samples", C.c_uint64),
                ("tiles", C.c_uint64), ("ms_total", C.c_double), ("ms_bounce", C.c_double),
                ("ms_film", C.c_double), ("bounce_launches", C.c_uint64), ("path_vertices", C.c_uint64),
                ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64), ("shape_tests", C.c_uint64),
                ("ms_closest", C.c_double), ("closest_launches", C.c_uint64), ("march_ticks", C.c_uint64),
                ("closest_node_visits", C.c_uint64), ("closest_tri_tests", C.c_uint64),
                ("closest_shape_tests", C.c_uint64), ("closest_march_ticks", C.c_uint64),
                ("ms_shade", C.c_double), ("shade_launches", C.c_uint64)]

    def rays(self) -> int:
        return int(self.rays_camera + self.rays_continuation + self.rays_mis + self.rays_shadow)

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class SppmStats(C.Structure):
    """bling_sppm_stats (include/bling.h)."""
    _fields_ = [("hitpoints", C.c_uint64), ("photons", C.c_uint64), ("photon_rays", C.c_uint64),
                ("photon_hits", C.c_uint64), ("cam_rays", C.c_uint64), ("dropped", C.c_uint64),
                ("ms_total", C.c_double), ("ms_eye", C.c_double), ("ms_hash", C.c_double),
                ("ms_photon", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class RenderConfig(C.Structure):
    _fields_ = [("renderer", C.c_int32), ("sampler", C.c_int32), ("nu", C.c_int32), ("nv", C.c_int32),
                ("spp", C.c_int32), ("max_depth", C.c_int32), ("sample_depth", C.c_int32),
                ("width", C.c_int32), ("height", C.c_int32), ("integrator", C.c_int32),
                ("sppm_photons", C.c_int32), ("sppm_radius", C.c_float), ("sppm_alpha", C.c_float),
                ("sppm_threads", C.c_int32)]


_host = None
_hip = None


def host() -> C.CDLL:
    global _host
    if _host is None:
        lib = C.CDLL(os.path.join(LIBDIR, "libbling_host.so"))
        lib.bling_host_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
        lib.bling_host_load.restype = C.c_int
        lib.bling_host_desc.argtypes = [C.c_void_p]
        lib.bling_host_desc.restype = C.c_void_p
        lib.bling_host_summary.argtypes = [C.c_void_p]
        lib.bling_host_summary.restype = C.c_char_p
        lib.bling_host_free.argtypes = [C.c_void_p]
        lib.bling_host_config.argtypes = [C.c_void_p, C.POINTER(RenderConfig)]
        lib.bling_host_filter_size.argtypes = [C.c_void_p, c_f32p]
        lib.bling_host_filter_table.argtypes = [C.c_void_p, c_f32p]
        lib.bling_host_counts.argtypes = [C.c_void_p, c_u32p]
        lib.bling_host_last_error.restype = C.c_char_p
        lib.bling_host_film_to_rgb.argtypes = [c_f32p, C.c_int, C.c_int, c_f32p]
        lib.bling_host_write_hdr.argtypes = [C.c_char_p, c_f32p, C.c_int, C.c_int]
        lib.bling_host_write_hdr.restype = C.c_int
        lib.bling_host_rgb_pixels.argtypes = [c_f32p, C.c_int, C.c_int, C.POINTER(C.c_uint8)]
        lib.bling_host_write_png.argtypes = [C.c_char_p, c_f32p, C.c_int, C.c_int]
        lib.bling_host_write_png.restype = C.c_int
        _host = lib
    return _host


HIP_SYMBOLS = ["bling_create", "bling_scene_upload", "bling_scene_validate", "bling_render_pass", "bling_render_pass_device",
               "bling_trace", "bling_trace_device", "bling_sample_li", "bling_sample_li_vertices", "bling_pass_tile_layout",
               "bling_film_add_tiles", "bling_film_add_shards", "bling_sppm_pass", "bling_sppm_pixel_stats", "bling_sppm_reset",
               "bling_render", "bling_debug_stream_bytes", "bling_debug_scene_info", "bling_debug_sppm_hitpoints", "bling_debug_sppm_buckets", "bling_destroy", "bling_last_error", "bling_version"]


class Progress(C.Structure):
    """bling_progress (include/bling.h): one report of bling_render (PassDone, or with
    PASS_REGION_EVENTS the per-window RegionStarted / SamplesAdded)."""
    _fields_ = [("kind", C.c_int32), ("pass_", C.c_int32), ("film", C.POINTER(C.c_float)), ("splat_weight", C.c_float),
                ("pass_stats", C.POINTER(Stats)), ("region", C.c_int32 * 4)]


PROGRESS_STARTED, PROGRESS_SAMPLES_ADDED, PROGRESS_REGION_STARTED, PROGRESS_PASS_DONE = 0, 1, 2, 3
ProgressFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(Progress))
STREAM_NAMES = "queue,hit,meta,org,dir,mdir,mhit,occ,fac,cf,T,L,Tn,lsc,bsc,sh_o,sh_d,result,qflag".split(",")


def hip() -> C.CDLL:
    """Load libbling_hip.so (raises OSError if it was not built -- no silent fallback)."""
    global _hip
    if _hip is None:
        # BLING_HIP_VARIANT=<v> loads the experiment build libbling_hip_<v>.so (make variant V=<v>)
        var = os.environ.get("BLING_HIP_VARIANT", "")
        path = os.path.join(LIBDIR, f"libbling_hip_{var}.so" if var else "libbling_hip.so")
        if not os.path.exists(path):
            raise OSError(f"{path} missing: run `make` (the HIP core has no CPU fallback)")
        lib = C.CDLL(path)
        lib.bling_create.argtypes = [C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]
        lib.bling_create.restype = C.c_int
        lib.bling_scene_upload.argtypes = [C.c_void_p, C.c_void_p]
        lib.bling_scene_upload.restype = C.c_int
        if hasattr(lib, "bling_scene_validate"):      # older experiment builds (BLING_HIP_VARIANT) lack it
            lib.bling_scene_validate.argtypes = [C.c_void_p]
            lib.bling_scene_validate.restype = C.c_int
        lib.bling_render_pass.argtypes = [C.c_void_p, C.POINTER(PassParams), c_f32p, C.POINTER(Stats)]
        lib.bling_render_pass.restype = C.c_int
        lib.bling_render_pass_device.argtypes = [C.c_void_p, C.POINTER(PassParams), C.c_void_p, C.POINTER(Stats)]
        lib.bling_render_pass_device.restype = C.c_int
        lib.bling_pass_tile_layout.argtypes = [C.c_void_p, C.POINTER(PassParams), C.POINTER(C.c_int32),
                                               C.POINTER(C.c_size_t), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.bling_pass_tile_layout.restype = C.c_int
        lib.bling_film_add_tiles.argtypes = [C.c_void_p, C.POINTER(PassParams), C.c_void_p, C.c_void_p]
        lib.bling_film_add_tiles.restype = C.c_int
        lib.bling_film_add_shards.argtypes = [C.c_void_p, C.POINTER(PassParams), C.POINTER(C.c_void_p), C.c_void_p]
        lib.bling_film_add_shards.restype = C.c_int
        lib.bling_trace.argtypes = [C.c_void_p, c_f32p, C.c_size_t, C.c_int, c_f32p, c_u32p, c_f32p]
        lib.bling_trace.restype = C.c_int
        lib.bling_trace_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_int, C.POINTER(C.c_double)]
        lib.bling_trace_device.restype = C.c_int
        lib.bling_sppm_pass.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, c_f32p, c_f32p, C.POINTER(SppmStats)]
        lib.bling_sppm_pass.restype = C.c_int
        lib.bling_sppm_pixel_stats.argtypes = [C.c_void_p, c_f32p, c_f32p, C.POINTER(C.c_size_t)]
        lib.bling_sppm_pixel_stats.restype = C.c_int
        lib.bling_sppm_reset.argtypes = [C.c_void_p]
        lib.bling_sppm_reset.restype = C.c_int
        if hasattr(lib, "bling_render"):              # older experiment builds lack the pass loop
            lib.bling_render.argtypes = [C.c_void_p, C.POINTER(PassParams), c_f32p, ProgressFn, C.c_void_p,
                                         C.POINTER(Stats)]
            lib.bling_render.restype = C.c_int
        lib.bling_debug_sppm_hitpoints.argtypes = [C.c_void_p, c_f32p, C.POINTER(C.c_uint64), C.c_size_t,
                                                   C.POINTER(C.c_size_t)]
        lib.bling_debug_sppm_hitpoints.restype = C.c_int
        lib.bling_debug_sppm_buckets.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), c_f32p,
                                                 C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        lib.bling_debug_sppm_buckets.restype = C.c_int
        lib.bling_debug_scene_info.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
        lib.bling_debug_scene_info.restype = C.c_int
        if hasattr(lib, "bling_debug_stream_bytes"):
            lib.bling_debug_stream_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t,
                                                     C.POINTER(C.c_size_t)]
            lib.bling_debug_stream_bytes.restype = C.c_int
        lib.bling_destroy.argtypes = [C.c_void_p]
        lib.bling_last_error.restype = C.c_char_p
        lib.bling_version.restype = C.c_char_p
        _hip = lib
    return _hip


def f32ptr(a):
    return a.ctypes.data_as(c_f32p)


def u32ptr(a):
    return a.ctypes.data_as(c_u32p)
