#!/usr/bin/env python3
"""Loader coverage of the reference's example scenes, in THIS container only
(the reference tree does not exist on the GPU box):

  python tools/scan_examples.py [/root/reference/examples]

Parses every ``*.bling`` with the host loader (path renderer forced) and prints, per scene, either
the prim / light counts and feature bits or the loader's error.  Several examples are stale and
fail in the reference's own parser too (``rgb`` instead of ``rgbR``/``rgbI``, ``stratified
xSamples``, a top-level ``shape`` object): the loader rejects those in the same place.
"""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bling_amd.scene import ParseError, parse_job  # noqa: E402


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/examples"
    ok = 0
    files = sorted(glob.glob(os.path.join(base, "*.bling")))
    for p in files:
        try:
            j = parse_job(p, "force_path=1")
            print(f"OK   {os.path.basename(p):28s} {j.counts()}")
            ok += 1
        except ParseError as e:
            print(f"FAIL {os.path.basename(p):28s} {str(e)[:160]}")
    print(f"{ok} / {len(files)} scenes load")


if __name__ == "__main__":
    main()
