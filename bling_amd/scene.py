"""Scene loading (host side of the boundary) and the benchmark configurations.

`parse_job` mirrors the reference's ``parseJob :: FilePath -> IO (Either ParseError (RenderJob,
AnyRenderer))`` (src/lib/Graphics/Bling/IO/RenderJob.hs:31-34): it returns a :class:`Job` holding
the flattened scene description the MI355X core consumes.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "fixtures", "scenes")


class ParseError(RuntimeError):
    pass


@dataclass(frozen=True)
class BenchConfig:
    """One row of BASELINE.json `configs`: scene file + in-place overrides."""
    name: str
    scene: str
    overrides: str
    gpus: int

    @property
    def path(self) -> str:
        return os.path.join(SCENES, self.scene)


# Overrides follow SURVEY.md 8(d): imageSize patched in place (T2), path renderer forced (T1).
CONFIGS = {
    "C1": BenchConfig("C1", "cornell-box.bling", "image=256,256;stratified=2,2;path=15,3;force_path=1", 0),
    "C2": BenchConfig("C2", "cornell-box.bling", "image=1024,1024;stratified=8,8;path=15,3;force_path=1", 1),
    "C3": BenchConfig("C3", "ducky.bling", "image=1920,1080;stratified=16,16;path=5,3;force_path=1", 1),
    "C4": BenchConfig("C4", "sun-sky.bling", "image=2048,2048;random=512;path=7,4;force_path=1", 4),
    "C5": BenchConfig("C5", "mandelbulb.bling", "image=4096,4096;stratified=32,32;path=5,2;force_path=1", 8),
}


# Feature scenes of this repository (fixtures/scenes), in the reference grammar, for parity tests
# of components beyond the benchmark configs.
FEATURE_SCENES = {
    "X1": BenchConfig("X1", "shapes-materials.bling", "", 0),   # disk / cylinder / box, transMatte, shinyMetal
    "X2": BenchConfig("X2", "heightmap-sinc.bling", "", 0),     # heightMap (fBm), shading normals, sinc 4
    "X3": BenchConfig("X3", "julia.bling", "", 0),              # quaternion Julia fractal (DE march)
    "X4": BenchConfig("X4", "direct-lighting.bling", "", 0),    # directLighting integrator, specular trees
    "X5": BenchConfig("X5", "cornell-box.bling", "", 0),        # SPPM as shipped (area light, matte)
    "X6": BenchConfig("X6", "sun-sky.bling", "", 0),            # SPPM as shipped (sun/sky photons, glass trees)
    "X7": BenchConfig("X7", "substrate-materials.bling", "", 0),  # substrate (FresnelBlend, anisotropic)
    "X8": BenchConfig("X8", "substrate.bling", "", 0),          # the reference's substrate.bling as shipped (fBm depth)
    "X9": BenchConfig("X9", "bumpmap.bling", "", 0),            # the reference's bumpmap.bling as shipped (fBm bump)
    "X10": BenchConfig("X10", "cellnoise.bling", "", 0),        # the reference's cellnoise.bling as shipped
    "X11": BenchConfig("X11", "procedural-textures.bling", "", 0),  # blend / gradient / checker, 4 cellNoise kinds
    "X12": BenchConfig("X12", "crystal-constenv.bling", "", 0),  # crystal.bling, constant env (its .hdr is not shipped)
    "X13": BenchConfig("X13", "delta-lights.bling", "", 0),     # point + directional lights next to an area light
    "X14": BenchConfig("X14", "image-textures.bling", "", 0),   # PNG image textures (uv / planar, bump), HDR env map
    "X15": BenchConfig("X15", "envmap.bling", "", 0),           # HDR env map over constant materials (no per-hit textures)
    "X16": BenchConfig("X16", "bezier.bling", "", 0),           # Bezier patches (tesselateBezier) as a shading-normal mesh
}


class Job:
    """A parsed `.bling` job: RenderJob + the sampler/path renderer configuration."""

    def __init__(self, path: str, overrides: str | None = None):
        lib = _ffi.host()
        h = C.c_void_p()
        rc = lib.bling_host_load(path.encode(), overrides.encode() if overrides else None, C.byref(h))
        if rc != 0:
            raise ParseError(lib.bling_host_last_error().decode())
        self._h = h
        self._lib = lib
        self.path = path
        self.overrides = overrides
        cfg = _ffi.RenderConfig()
        lib.bling_host_config(h, C.byref(cfg))
        self.config = cfg
        fw = np.zeros(2, np.float32)
        lib.bling_host_filter_size(h, _ffi.f32ptr(fw))
        self.filter_size = (float(fw[0]), float(fw[1]))

    @property
    def desc(self) -> int:
        """Address of the bling_scene_desc (valid while this Job lives)."""
        return self._lib.bling_host_desc(self._h)

    @property
    def width(self) -> int:
        return self.config.width

    @property
    def height(self) -> int:
        return self.config.height

    @property
    def spp(self) -> int:
        return self.config.spp

    def filter_table(self) -> np.ndarray:
        out = np.zeros(256, np.float32)
        self._lib.bling_host_filter_table(self._h, _ffi.f32ptr(out))
        return out.reshape(16, 16)

    def counts(self) -> dict:
        out = np.zeros(6, np.uint32)
        self._lib.bling_host_counts(self._h, _ffi.u32ptr(out))
        return dict(zip(("triangles", "shapes", "fractal", "prims", "lights", "features"), (int(v) for v in out)))

    def summary(self) -> str:
        return self._lib.bling_host_summary(self._h).decode()

    def extent(self):
        """sampleExtent (Image.hs:162-168) -> (x0, x1, y0, y1), inclusive."""
        fw, fh = self.filter_size
        f32 = np.float32
        x0 = int(np.floor(f32(0.5) - f32(fw)))
        x1 = int(np.floor(f32(f32(0.5) + f32(self.width)) + f32(fw)))
        y0 = int(np.floor(f32(0.5) - f32(fh)))
        y1 = int(np.floor(f32(f32(0.5) + f32(self.height)) + f32(fh)))
        return x0, x1, y0, y1

    def num_tiles(self) -> int:
        x0, x1, y0, y1 = self.extent()
        return ((x1 - x0) // 16 + 1) * ((y1 - y0) // 16 + 1)

    def tile_slot(self):
        """(slot_w, slot_h): the largest mkImageTile image of this filter (Image.hs:108-120), the slot
        size of the tile images a multi-rank pass gathers (include/bling.h BLING_PASS_TILE_IMAGES)."""
        fw, fh = self.filter_size
        f32 = np.float32
        return 15 + int(np.floor(f32(0.5) + f32(fw))), 15 + int(np.floor(f32(0.5) + f32(fh)))

    def shard_tiles(self, rank: int = 0, world: int = 1, stride: int = 1):
        """Tile-image origins (ox, oy) of the shard's tiles in slot order: splitWindow's tiles k with
        k % stride == 0 and (k / stride) % world == rank (core.hip render, oracle_render_shard)."""
        x0, x1, y0, y1 = self.extent()
        out, k = [], 0
        for y in range(y0, y1 + 1, 16):
            for x in range(x0, x1 + 1, 16):
                if k % stride == 0 and (k // stride) % world == rank:
                    out.append((max(0, x), max(0, y)))
                k += 1
        return np.array(out, np.int32).reshape(-1, 2)

    def camera_samples(self) -> int:
        x0, x1, y0, y1 = self.extent()
        return (x1 - x0 + 1) * (y1 - y0 + 1) * self.spp

    def close(self):
        if self._h:
            self._lib.bling_host_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def parse_job(path: str, overrides: str | None = None) -> Job:
    return Job(path, overrides)


def load_config(name: str, overrides_extra: str | None = None) -> Job:
    c = CONFIGS[name] if name in CONFIGS else FEATURE_SCENES[name]
    ov = ";".join(x for x in (c.overrides, overrides_extra) if x)
    return Job(c.path, ov or None)


def film_to_rgb(film: np.ndarray, w: int, h: int) -> np.ndarray:
    """getPixel + xyzToRgb (Image.hs:302-315) for a (h*w*4) film."""
    film = np.ascontiguousarray(film, np.float32).reshape(-1)
    out = np.zeros(w * h * 3, np.float32)
    _ffi.host().bling_host_film_to_rgb(_ffi.f32ptr(film), w, h, _ffi.f32ptr(out))
    return out.reshape(h, w, 3)


def write_hdr(path: str, rgb: np.ndarray):
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w, _ = rgb.shape
    if _ffi.host().bling_host_write_hdr(path.encode(), _ffi.f32ptr(rgb.reshape(-1)), w, h) != 0:
        raise IOError(_ffi.host().bling_host_last_error().decode())
