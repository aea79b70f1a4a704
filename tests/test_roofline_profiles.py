"""The committed round-4 roofline is reproducible from profiles/ alone:
tools/roofline_check.py recomputes each bench line's shading-kernel and closest-hit fractions from
the counted stream bytes and the rocprofv3 kernel-trace summary committed beside it, requires them
to match the line within 5 %, and requires the counted algorithmic bytes to stay below the PMC DRAM
bytes of the same workload.  Also checks that every file of one config's session carries the same
source digest as its bench line.  CPU only (reads JSON / CSV)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
CFGS = ["C2", "C3", "C4"]


def test_roofline_check_passes_on_committed_round4_profiles():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_check.py"), "r04"] + CFGS,
                       capture_output=True, text=True, timeout=120)
    res = json.loads(r.stdout)
    assert r.returncode == 0, r.stdout
    assert sorted(x["config"] for x in res) == CFGS
    for x in res:
        names = {c["check"] for c in x["checks"]}
        assert {"shade frac from profiles", "shade algorithmic <= PMC DRAM bytes", "closest frac from profiles"} <= names


@pytest.mark.parametrize("cfg", CFGS)
def test_session_files_share_the_bench_line_digest(cfg):
    c = cfg.lower()
    line = json.load(open(os.path.join(PROF, f"r04_{c}_bench.json")))
    digest = line["config"]["source_digest"]
    roof = line["roofline"]
    shade = roof if roof.get("kernel", "").startswith("k_shade") else roof["secondary"]
    assert shade["bytes_source_current"] and shade["traffic_source_current"]
    for kind in ("shade_streams", "shade_traffic", "trace_closest_traffic"):
        d = json.load(open(os.path.join(PROF, f"r04_{c}_{kind}.json")))
        assert d.get("source_digest") == digest, (kind, d.get("source_digest"), digest)
