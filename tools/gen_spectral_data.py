#!/usr/bin/env python3
"""Generate bling_amd/csrc/common/spectral_data.h from the reference's Spectrum.hs / SunSky.hs.

Runs only in the build container (where /root/reference exists).  The committed output holds
DERIVED numeric data only (16-band averages, XYZ constants, and the raw public CIE / Preetham
curve samples the host loader needs); no reference source text is kept.

Every derived value is computed in IEEE binary32 exactly as the reference's Float code does:
  - literals are rounded to Float correctly (Haskell `fromRational`), not via double;
  - `fromSpd`   : Spectrum.hs:329-335  (16 bands over [400,700] via `avgSpd`)
  - `avgSpd`    : Spectrum.hs:297-305  (RegularSpd: slice average, n = length amps)
  - `evalSpd`   : Spectrum.hs:271-280  (RegularSpd linear interpolation)
  - `spdToXYZ`  : Spectrum.hs:319-326  (1 nm sums over [cieStart..cieEnd] = [360..830])
  - `spectrumCieYSum` : Spectrum.hs:346-347 (V.sum = left fold from 0)
  - `lerp`      : Math.hs:108-110
"""
import re
import sys
from fractions import Fraction

import numpy as np

F = np.float32
REF = "/root/reference/src/lib/Graphics/Bling"


def f32_exact(s: str) -> np.float32:
    """Correctly rounded decimal -> binary32 (ties to even), like GHC's fromRational."""
    q = Fraction(s)
    if q == 0:
        return F(0.0)
    d = F(float(q))  # candidate (may be off by one ulp due to double rounding)
    best = None
    for c in (np.nextafter(d, F(-np.inf)), d, np.nextafter(d, F(np.inf))):
        err = abs(Fraction(float(c)) - q)
        if best is None or err < best[0] or (err == best[0] and (c.view(np.uint32) & 1) == 0):
            best = (err, c)
    return F(best[1])


def grab_list(text: str, name: str):
    """Return the number literals of the first `[ ... ]` after `name =` (or `name = f`)."""
    m = re.search(r"^%s\s*=" % re.escape(name), text, re.M)
    if not m:
        raise KeyError(name)
    i = text.index("[", m.end())
    j = text.index("]", i)
    body = text[i + 1:j]
    return [tok for tok in re.findall(r"[-+]?\d+\.?\d*(?:[eE][-+]?\d+)?", body)]


def lerp(t, v1, v2):
    return F(F(F(1) - t) * v1) + F(t * v2)


def eval_regular(l0, l1, amps, lam):
    """evalSpd (RegularSpd l0 l1 amps) lam  -- Spectrum.hs:271-280."""
    n = len(amps)
    if lam <= l0:
        return amps[0]
    if lam >= l1:
        return amps[-1]
    d1 = F(F(1) / F(F(l1 - l0) / F(n - 1)))
    x = F(F(lam - l0) * d1)
    b0 = int(np.floor(x))
    b1 = min(b0 + 1, n - 1)
    dx = F(x - F(b0))
    return F(F(F(1) - dx) * amps[b0]) + F(dx * amps[b1])


def avg_regular(s0, s1, amps, l0, l1):
    """avgSpd (RegularSpd s0 s1 amps) l0 l1 -- Spectrum.hs:297-305."""
    n = len(amps)
    if l1 <= s0:
        return amps[0]
    if l0 >= s1:
        return amps[-1]
    i0 = max(0, min(n, int(np.floor(F(F(n) * F(F(l0 - s0) / F(s1 - s0)))))))
    i1 = max(0, min(n, int(np.floor(F(F(n) * F(F(l1 - s0) / F(s1 - s0)))))))
    acc = F(0)
    sl = amps[i0:i1 + 1]
    assert len(sl) == i1 - i0 + 1, "slice out of range"
    for a in sl:
        acc = F(acc + a)
    return F(acc / F(len(sl)))


def from_spd_regular(s0, s1, amps):
    """fromSpd -- Spectrum.hs:329-335 (bands = 16, [400,700])."""
    out = []
    for i in range(16):
        l0 = lerp(F(F(i) / F(16)), F(400), F(700))
        l1 = lerp(F(F(i + 1) / F(16)), F(400), F(700))
        out.append(avg_regular(F(s0), F(s1), amps, l0, l1))
    return out


def fsum(xs):
    acc = F(0)
    for x in xs:
        acc = F(acc + x)
    return acc


def hexf(x):
    return float(x).hex() + "f"


def main(out_path):
    spec = open(f"{REF}/Spectrum.hs").read()
    sky = open(f"{REF}/SunSky.hs").read()

    cie = {c: [f32_exact(t) for t in grab_list(spec, f"cie{c}Values")] for c in "XYZ"}
    assert all(len(v) == 471 for v in cie.values())
    s012 = [[f32_exact(t) for t in grab_list(spec, f"cieS{k}")] for k in range(3)]
    assert all(len(v) == 54 for v in s012)
    bases = ["Red", "Green", "Blue", "Cyan", "Magenta", "Yellow", "White"]
    refl = [[f32_exact(t) for t in grab_list(spec, f"rgbRefl{b}")] for b in bases]
    illum = [[f32_exact(t) for t in grab_list(spec, f"rgbIllum{b}")] for b in bases]

    cie_bands = {c: from_spd_regular(360, 830, cie[c]) for c in "XYZ"}
    ysum = fsum(cie_bands["Y"])
    refl_bands = [from_spd_regular(380, 720, v) for v in refl]
    illum_bands = [from_spd_regular(380, 720, v) for v in illum]

    # spdToXYZ for the S0/S1/S2 daylight basis (Spectrum.hs:234-251, 319-326)
    lams = [F(l) for l in range(360, 831)]
    cx = [eval_regular(F(360), F(830), cie["X"], l) for l in lams]
    cy = [eval_regular(F(360), F(830), cie["Y"], l) for l in lams]
    cz = [eval_regular(F(360), F(830), cie["Z"], l) for l in lams]
    yint = fsum(cy)
    sxyz = []
    for k in range(3):
        vs = [eval_regular(F(300), F(830), s012[k], l) for l in lams]
        x = fsum([F(a * b) for a, b in zip(cx, vs)])
        y = fsum([F(a * b) for a, b in zip(cy, vs)])
        z = fsum([F(a * b) for a, b in zip(cz, vs)])
        sxyz.append((F(x / yint), F(y / yint), F(z / yint)))

    # Preetham sun attenuation curves (SunSky.hs:127-157), raw samples for the host loader.
    sol = [f32_exact(t) for t in grab_list(sky, "solCurve")]

    def irregular(name):
        m = re.search(r"^%s\s*=" % name, sky, re.M)
        seg = sky[m.end():]
        end = seg.find("\n\n")
        seg = seg[:end if end > 0 else len(seg)]
        lists = re.findall(r"\[([^\]]*)\]", seg)
        nums = [re.findall(r"[-+]?\d+\.?\d*(?:[eE][-+]?\d+)?", l) for l in lists]
        return [f32_exact(t) for t in nums[0]], [f32_exact(t) for t in nums[1]]

    ko = irregular("koCurve")
    kg = irregular("kgCurve")
    kwa = irregular("kwaCurve")

    L = []
    w = L.append
    w("/* GENERATED by tools/gen_spectral_data.py -- do not edit.")
    w(" * Derived binary32 data for the bling spectral model (16 bands, 400-700 nm).")
    w(" * Sources (reference, read in the build container): Spectrum.hs fromSpd/avgSpd/spdToXYZ,")
    w(" * SunSky.hs solCurve/koCurve/kgCurve/kwaCurve.  Values are hex-float exact. */")
    w("#pragma once")
    w("#define BLING_NBANDS 16")

    def arr(name, vals):
        w(f"static constexpr float {name}[{len(vals)}] = {{")
        for i in range(0, len(vals), 4):
            w("   " + ", ".join(hexf(v) for v in vals[i:i + 4]) + ",")
        w("};")

    arr("BLING_CIE_X_BANDS", cie_bands["X"])
    arr("BLING_CIE_Y_BANDS", cie_bands["Y"])
    arr("BLING_CIE_Z_BANDS", cie_bands["Z"])
    w(f"static constexpr float BLING_CIE_Y_SUM = {hexf(ysum)};")
    w("/* order: red, green, blue, cyan, magenta, yellow, white */")
    w("static constexpr float BLING_RGB_REFL_BANDS[7][16] = {")
    for b in refl_bands:
        w("   {" + ", ".join(hexf(v) for v in b) + "},")
    w("};")
    w("static constexpr float BLING_RGB_ILLUM_BANDS[7][16] = {")
    for b in illum_bands:
        w("   {" + ", ".join(hexf(v) for v in b) + "},")
    w("};")
    w("static constexpr float BLING_S_XYZ[3][3] = {")
    for t in sxyz:
        w("   {" + ", ".join(hexf(v) for v in t) + "},")
    w("};")
    arr("BLING_SOL_CURVE_380_750", sol)
    for nm, (ls, vs) in (("KO", ko), ("KG", kg), ("KWA", kwa)):
        arr(f"BLING_{nm}_LAMBDA", ls)
        arr(f"BLING_{nm}_VALUE", vs)
    open(out_path, "w").write("\n".join(L) + "\n")
    print("wrote", out_path)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "bling_amd/csrc/common/spectral_data.h")
