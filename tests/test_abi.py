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
