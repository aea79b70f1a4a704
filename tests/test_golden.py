"""The oracle reproduces the committed golden vectors bit-for-bit (tests/golden/make_golden.py).

Golden vectors are the parity anchor for this path (the reference's own tests pin no hot-path value,
SURVEY.md 8c): any change to the oracle's arithmetic shows up here, and tests/test_gpu_parity.py
checks the HIP core against the same files."""
import os

import numpy as np
import pytest

from bling_amd.scene import load_config
from oracle_py import Oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEED = 0x0B11A6


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "C5", "X1", "X2", "X3", "X4", "X7", "X10", "X11", "X12", "X13",
                                  "X14", "X15", "X16"])
def test_trace_golden(name):
    g = np.load(os.path.join(GOLD, f"trace_{name}.npz"))
    orc = Oracle(load_config(name, str(g["overrides"]) or None))
    t, prim, bary, _ = orc.trace(g["rays"])
    np.testing.assert_array_equal(prim, g["prim"])
    np.testing.assert_array_equal(t, g["t"])
    np.testing.assert_array_equal(bary, g["bary"])
    _, occ, _, _ = orc.trace(g["rays"], any_hit=True)
    np.testing.assert_array_equal(occ, g["occluded"])


@pytest.mark.parametrize("name", ["C1", "X1", "X2", "X3", "X4", "X7", "X8", "X9", "X10", "X11", "X12", "X13",
                                  "X14", "X15", "X16"])
def test_sample_li_golden(name):
    g = np.load(os.path.join(GOLD, f"sample_li_{name}.npz"))
    orc = Oracle(load_config(name, str(g["overrides"]) or None))
    for i, (x, y, n) in enumerate(g["samples"][:64]):
        L, img, _ = orc.sample_li(int(x), int(y), int(n), seed=SEED)
        np.testing.assert_array_equal(L, g["L"][i])
        np.testing.assert_array_equal(img, g["img"][i])


def test_film_golden():
    g = np.load(os.path.join(GOLD, "film_C1_48.npz"))
    film, st = Oracle(load_config("C1", str(g["overrides"]))).render(seed=SEED, pass_index=0, threads=1)
    np.testing.assert_array_equal(film.reshape(g["film"].shape), g["film"])
    assert [st.samples, st.rays_camera, st.rays_continuation, st.rays_mis, st.rays_shadow] == list(g["counts"])
