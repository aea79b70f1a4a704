"""The C-ABI boundary: every entry point declared in include/*.h is exported by the
built libraries, the ctypes mirrors match the C structs' layouts, and the device library reports
missing GPUs as an error code instead of falling back to anything.  No GPU compute call is made."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bling_amd", "_lib")

DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_][\w\s]*?[\s\*]+(bling_\w+)\s*\(", re.M)


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(DECL.findall(text)))


@pytest.fixture(scope="module")
def libs(built):
    hip = os.path.join(LIB, "libbling_hip.so")
    if not os.path.exists(hip):
        pytest.skip("libbling_hip.so not built (run __graft_entry__.build())")
    return C.CDLL(os.path.join(LIB, "libbling_host.so")), C.CDLL(hip)


def test_headers_declare_the_boundary():
    core = declared("bling.h")
    for f in ("bling_create", "bling_scene_upload", "bling_render_pass", "bling_render_pass_device",
              "bling_trace", "bling_sample_li", "bling_destroy", "bling_last_error"):
        assert f in core, f
    assert "bling_host_load" in declared("bling_host.h")


@pytest.mark.parametrize("header,which", [("bling.h", 1), ("bling_host.h", 0)])
def test_every_declared_symbol_is_exported(libs, header, which):
    lib = libs[which]
    missing = [f for f in declared(header) if not hasattr(lib, f)]
    assert not missing, f"{header}: not exported: {missing}"


def test_struct_layouts_match_ctypes(libs):
    from bling_amd import _ffi
    # offsets of the appended fields pin the whole layout (natural alignment, no packing)
    assert _ffi.PassParams.tiles_device.offset == 8 * 4 and _ffi.PassParams.tiles_capacity.offset == 8 * 4 + 8
    assert C.sizeof(_ffi.PassParams) == 8 * 4 + 16
    assert C.sizeof(_ffi.Progress) == 4 + 4 + 8 + 8 + 8 + 16 and _ffi.Progress.film.offset == 8
    assert _ffi.Progress.pass_stats.offset == 24 and _ffi.Progress.region.offset == 32
    assert _ffi.Stats.ms_closest.offset == 15 * 8
    assert _ffi.Stats.march_ticks.offset == 17 * 8
    assert _ffi.Stats.closest_march_ticks.offset == 21 * 8
    assert _ffi.Stats.ms_shade.offset == 22 * 8
    assert C.sizeof(_ffi.Stats) == 24 * 8


def test_no_device_is_an_error_not_a_fallback(libs):
    """Without a HIP device bling_create must fail loudly (BLING_ENODEV), never run on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    hip = libs[1]
    hip.bling_last_error.restype = C.c_char_p
    out = C.c_void_p()
    rc = hip.bling_create(None, 0, C.byref(out))
    assert rc != 0 and not out.value
    assert hip.bling_last_error()


def test_product_does_not_link_the_oracle(libs):
    """The shipped libraries never reference oracle symbols (the oracle is test infrastructure)."""
    for name in ("libbling_hip.so", "libbling_host.so"):
        blob = open(os.path.join(LIB, name), "rb").read()
        assert b"oracle_" not in blob, name


def test_struct_layouts_match_the_c_compiler(tmp_path):
    """sizeof / offsetof of the ABI structs as gcc lays out include/bling.h, against the ctypes mirror."""
    import subprocess
    from bling_amd import _ffi
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "bling.h"\nint main(void) {\n'
                   '  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(bling_pass_params), offsetof(bling_pass_params, flags),\n'
                   '         offsetof(bling_pass_params, tiles_device), sizeof(bling_stats), offsetof(bling_stats, ms_shade),\n'
                   '         offsetof(bling_pass_params, tiles_capacity), sizeof(bling_progress), offsetof(bling_progress, film),\n'
                   '         offsetof(bling_progress, pass_stats), offsetof(bling_progress, region));\n'
                   '  return 0;\n}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(_ffi.PassParams), _ffi.PassParams.flags.offset, _ffi.PassParams.tiles_device.offset,
                   C.sizeof(_ffi.Stats), _ffi.Stats.ms_shade.offset, _ffi.PassParams.tiles_capacity.offset,
                   C.sizeof(_ffi.Progress), _ffi.Progress.film.offset, _ffi.Progress.pass_stats.offset,
                   _ffi.Progress.region.offset]


def test_stream_names_match_the_header():
    """The Python stream list of bling_debug_stream_bytes is the header's BLING_STREAM_NAMES."""
    import re
    from bling_amd import _ffi
    text = open(os.path.join(ROOT, "include", "bling.h")).read()
    names = re.search(r'#define BLING_STREAM_NAMES "([^"]+)"', text).group(1).split(",")
    n = int(re.search(r"#define BLING_N_STREAMS (\d+)", text).group(1))
    assert names == _ffi.STREAM_NAMES and len(names) == n


def test_every_scene_passes_upload_validation(libs):
    """bling_scene_validate runs bling_scene_upload's checks without a device: every benchmark
    config and feature scene the loader accepts must pass them (the checks and the loader's texture,
    material and light kinds must not drift apart), and a malformed description must fail."""
    from bling_amd import _ffi
    from bling_amd.scene import CONFIGS, FEATURE_SCENES, load_config
    hip = _ffi.hip()
    for name in list(CONFIGS) + list(FEATURE_SCENES):
        job = load_config(name)
        rc = hip.bling_scene_validate(C.c_void_p(job.desc))
        assert rc == 0, f"{name}: {hip.bling_last_error().decode()}"
    assert hip.bling_scene_validate(None) != 0
