"""Film output of a pass: the reference's tonemap and image writers over the host library.

Reference (src/lib/Graphics/Bling):
  * ``getPixel`` / ``xyzToRgb`` (Image.hs:302-315, Spectrum.hs:162-168)  -> :func:`to_rgb`
  * ``rgbPixels`` (gamma 2.2, clamp, round; Image.hs:317-331)            -> :func:`rgb_pixels`
  * ``writePng`` / ``writeRgbe`` (IO/Bitmap.hs:37-41)                     -> :func:`write_png`, :func:`write_hdr`
  * ``progressWriter`` (IO/Progress.hs:23-36): ``<base>-NNNNN.png`` and ``.hdr`` at every PassDone
    -> :func:`progress_writer`
The film is the (W, X, Y, Z) array a pass accumulates (``bling_render_pass``), shape (h * w * 4,).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi


def _film(film, w, h):
    f = np.ascontiguousarray(film, np.float32).reshape(-1)
    if f.size != w * h * 4:
        raise ValueError(f"film has {f.size} floats, expected {w} x {h} x 4")
    return f


def to_rgb(film, w: int, h: int) -> np.ndarray:
    """Linear RGB (h, w, 3) float32: XYZ / W, then xyzToRgb."""
    f = _film(film, w, h)
    rgb = np.zeros(w * h * 3, np.float32)
    _ffi.host().bling_host_film_to_rgb(_ffi.f32ptr(f), w, h, _ffi.f32ptr(rgb))
    return rgb.reshape(h, w, 3)


def rgb_pixels(film, w: int, h: int) -> np.ndarray:
    """8-bit display pixels (h, w, 3) uint8 of rgbPixels."""
    f = _film(film, w, h)
    out = np.zeros(w * h * 3, np.uint8)
    _ffi.host().bling_host_rgb_pixels(_ffi.f32ptr(f), w, h, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out.reshape(h, w, 3)


def write_png(path: str, film, w: int, h: int) -> None:
    f = _film(film, w, h)
    if _ffi.host().bling_host_write_png(path.encode(), _ffi.f32ptr(f), w, h) != 0:
        raise OSError(_ffi.host().bling_host_last_error().decode())


def write_hdr(path: str, film, w: int, h: int) -> None:
    rgb = np.ascontiguousarray(to_rgb(film, w, h).reshape(-1))
    if _ffi.host().bling_host_write_hdr(path.encode(), _ffi.f32ptr(rgb), w, h) != 0:
        raise OSError(_ffi.host().bling_host_last_error().decode())


def progress_writer(base: str, w: int, h: int):
    """progressWriter: a ProgressReporter (bling_amd.render.Progress -> bool) that writes every
    completed pass to ``<base>-NNNNN.png`` and ``.hdr`` and asks to continue."""
    def report(pr) -> bool:
        if pr.kind == "PassDone" and pr.film is not None:
            name = f"{base}-{pr.pass_num:05d}"
            print(f"\nWriting {name}...")
            write_png(name + ".png", pr.film, w, h)
            write_hdr(name + ".hdr", pr.film, w, h)
        return True
    return report
