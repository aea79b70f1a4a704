"""Quantized BVH4 nodes (bvh::quantize4, bling_amd/csrc/core/bvh_build.cpp): the decoded child boxes
contain the float boxes on random scenes (unit, offset 1e5, flat, wide, tiny), every plane within one
quantization step, links unchanged -- so Traversal4's quantized walk reaches every primitive the float
walk reaches.  Builds tests/cpp/bvh_quant_check.cpp with g++ against the builder's own source.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_quantized_bvh4_boxes_contain_float_boxes(tmp_path):
    exe = tmp_path / "bvh_quant_check"
    src = [os.path.join(ROOT, "tests", "cpp", "bvh_quant_check.cpp"),
           os.path.join(ROOT, "bling_amd", "csrc", "core", "bvh_build.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe)] + src, check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("planes") == 5
