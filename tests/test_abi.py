"""The C-ABI library builds for gfx950, loads, and exports every entry point
include/fsg.h declares (CPU only: no compute call is made here)."""
import ctypes
import os
import re

import pytest

from fluvio_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "fsg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fsg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("fsg_engine_new", "fsg_chain_builder_add_smart_module", "fsg_chain_builder_initialize",
                 "fsg_chain_process", "fsg_chain_process_batch", "fsg_chain_process_slice",
                 "fsg_allreduce_state", "fsg_state_collect", "fsg_state_allreduce"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _ffi.lib()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    # and the ctypes signature table covers the whole header
    assert set(_declared()) == set(_ffi.SIGNATURES)


def test_abi_version():
    assert _ffi.lib().fsg_abi_version() == _ffi.ABI_VERSION == 6


def test_gfx950_code_object_embedded():
    data = open(_ffi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_is_a_loud_error():
    """Without a GPU, engine creation fails with FSG_E_DEVICE (no CPU fallback)."""
    n = ctypes.c_int(-1)
    _ffi.lib().fsg_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    rc = _ffi.lib().fsg_engine_new(0, ctypes.byref(h))
    assert rc == _ffi.FSG_E_DEVICE
    from fluvio_amd.smartengine import DeviceError, SmartEngine
    with pytest.raises(DeviceError):
        SmartEngine(0)
