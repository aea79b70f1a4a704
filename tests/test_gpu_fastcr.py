"""Exhaustive device check of common/fast_cr.h: the march's reciprocal and square root
(bfast::rcp_cr / sqrt_cr, used by the paired Mandelbulb march in dev_trace.h) return exactly
`1.f / x` and `sqrtf(x)` for all 2^32 binary32 inputs on gfx950 -- the condition for the march
staying bit-identical to mandel_march and the oracle."""
import ctypes as C
import json
import os

import pytest

from parity_util import report

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bling_amd", "_lib",
                   "libbling_mathcheck.so")


def test_mathcheck_library_exports():
    lib = C.CDLL(LIB)
    assert hasattr(lib, "bling_mathcheck")


@pytest.mark.gpu
def test_fast_cr_exhaustive():
    lib = C.CDLL(LIB)
    out = (C.c_ulonglong * 4)()
    assert lib.bling_mathcheck(out) == 0
    rec = {"rcp_mismatch": out[0], "sqrt_mismatch": out[1], "first_rcp": hex(out[2]), "first_sqrt": hex(out[3])}
    report("fast_cr_exhaustive", inputs=1 << 32, **rec)
    assert out[0] == 0 and out[1] == 0, json.dumps(rec)
