"""The C-ABI library loads and exports every entry point include/az_engine.h declares
(no compute calls: runs without a GPU); without a device it fails loudly."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "az_engine.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(az_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_core_entry_points():
    names = declared()
    for n in ("az_engine_create", "az_net_forward", "az_net_predict_batch", "az_search_run", "az_search_select",
              "az_search_apply", "az_search_add_noise", "az_selfplay_step"):
        assert n in names


def test_library_exports_every_declared_symbol():
    import az_amd._lib as L
    assert os.path.exists(L.LIB_PATH), "build libaz_hip.so first (__graft_entry__.build())"
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared()) == set(L.EXPORTS), "ctypes binding out of sync with the header"


def test_no_device_fails_loudly():
    import az_amd
    from az_amd._lib import lib
    n = ctypes.c_int(0)
    try:
        import torch
        has_gpu = torch.cuda.device_count() > 0
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(az_amd.AzError, match="HIP"):
        az_amd.Engine(0)
    assert lib().az_last_error()


def test_header_is_plain_c_and_links(tmp_path):
    """A C99 translation unit (what a cgo / JNI / N-API binding compiles) includes the header with
    -Wall -Werror, links against libaz_hip.so and runs: without a device az_engine_create returns
    an error code and az_last_error names it; with one it creates and destroys an engine."""
    import shutil
    import subprocess
    import az_amd._lib as L
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "t.c"
    src.write_text('''#include "az_engine.h"
#include <stdio.h>
int main(void) {
    az_engine* e = 0;
    int r = az_engine_create(0, &e);
    if (r != 0) { printf("err %d %s\\n", r, az_last_error()); return 0; }
    az_engine_destroy(e);
    printf("ok\\n");
    return 0;
}
''')
    exe = tmp_path / "t"
    libdir = os.path.dirname(L.LIB_PATH)
    subprocess.run([cc, "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-L", libdir,
                    "-laz_hip", "-Wl,-rpath," + libdir, "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=120).stdout
    assert out.startswith("ok") or ("err" in out and "HIP" in out), out
