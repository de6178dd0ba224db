"""ctypes binding of libfsg.so (include/fsg.h).

This is the Python analogue of the reference-side FFI crate a maintainer would
add (INTEGRATION.md shows the Rust `extern "C"` block).  Loading fails loudly if
the HIP library has not been built: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FSG_LIB") or os.path.join(_HERE, "_lib", "libfsg.so")
CSRC = os.path.join(_HERE, "csrc")

FSG_OK = 0
FSG_E_UNKNOWN = -1
FSG_E_INIT = -2
FSG_E_DECODING_BASE_INPUT = -11
FSG_E_DECODING_RECORDS = -22
FSG_E_ENCODING_OUTPUT = -33
FSG_E_UNKNOWN_SM = -100
FSG_E_INSTANTIATE = -101
FSG_E_STORE_MEMORY = -102
FSG_E_UNSUPPORTED = -103
FSG_E_IO = -104
FSG_E_INVALID_ARG = -105
FSG_E_LOOKBACK = -106
FSG_LOOKBACK_NONE, FSG_LOOKBACK_LAST, FSG_LOOKBACK_AGE = 0, 1, 2
FSG_E_DEVICE = -200
ABI_VERSION = 6  # include/fsg.h FSG_ABI_VERSION: the struct layouts below


class fsg_param(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("value", ctypes.c_char_p)]


class fsg_metrics(ctypes.Structure):
    _fields_ = [("bytes_in", ctypes.c_uint64), ("records_out", ctypes.c_uint64),
                ("invocation_count", ctypes.c_uint64), ("fuel_used", ctypes.c_uint64)]


class fsg_runtime_error(ctypes.Structure):
    _fields_ = [("hint", ctypes.POINTER(ctypes.c_char)), ("hint_len", ctypes.c_size_t),
                ("offset", ctypes.c_int64), ("kind", ctypes.c_int32), ("has_key", ctypes.c_int32),
                ("key", ctypes.POINTER(ctypes.c_uint8)), ("key_len", ctypes.c_size_t),
                ("value", ctypes.POINTER(ctypes.c_uint8)), ("value_len", ctypes.c_size_t)]


class fsg_output(ctypes.Structure):
    _fields_ = [("records", ctypes.POINTER(ctypes.c_uint8)), ("records_len", ctypes.c_size_t),
                ("n_records", ctypes.c_uint32), ("has_error", ctypes.c_int32),
                ("error", fsg_runtime_error)]


class fsg_batch_output(ctypes.Structure):
    _fields_ = [("batch", ctypes.POINTER(ctypes.c_uint8)), ("batch_len", ctypes.c_size_t),
                ("base_offset", ctypes.c_int64), ("last_offset_delta", ctypes.c_int32),
                ("n_records", ctypes.c_uint32), ("has_error", ctypes.c_int32),
                ("error", fsg_runtime_error)]


class fsg_lookback(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("stage", ctypes.c_uint32), ("last", ctypes.c_uint64),
                ("age_ms", ctypes.c_uint64)]


READ_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(fsg_lookback),
                           ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t))


class fsg_timings(ctypes.Structure):
    _fields_ = [("eval_ms", ctypes.c_float), ("plan_ms", ctypes.c_float), ("write_ms", ctypes.c_float),
                ("crc_ms", ctypes.c_float), ("total_ms", ctypes.c_float), ("in_bytes", ctypes.c_uint64),
                ("out_bytes", ctypes.c_uint64), ("n_batches", ctypes.c_uint64),
                ("n_records_in", ctypes.c_uint64), ("eval_path", ctypes.c_uint32), ("deferred", ctypes.c_uint32),
                ("text_ms", ctypes.c_float), ("order_ms", ctypes.c_float), ("chunks", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


VP = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
U8P = ctypes.c_char_p
SZ = ctypes.c_size_t

# every symbol include/fsg.h declares, with (restype, argtypes)
SIGNATURES = {
    "fsg_last_error_message": (ctypes.c_char_p, []),
    "fsg_abi_version": (ctypes.c_int, []),
    "fsg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "fsg_engine_new": (ctypes.c_int, [ctypes.c_int, PP]),
    "fsg_engine_free": (None, [VP]),
    "fsg_chain_builder_new": (ctypes.c_int, [PP]),
    "fsg_chain_builder_set_store_memory_limit": (ctypes.c_int, [VP, SZ]),
    "fsg_chain_builder_add_smart_module": (ctypes.c_int, [VP, ctypes.POINTER(fsg_param), SZ, ctypes.c_int16,
                                                          U8P, SZ, ctypes.c_int32, U8P, SZ]),
    "fsg_chain_builder_initialize": (ctypes.c_int, [VP, VP, PP]),
    "fsg_chain_builder_free": (None, [VP]),
    "fsg_chain_process": (ctypes.c_int, [VP, U8P, SZ, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(fsg_metrics), ctypes.POINTER(ctypes.POINTER(fsg_output))]),
    "fsg_chain_process_batch": (ctypes.c_int, [VP, U8P, SZ, ctypes.c_uint64, ctypes.POINTER(fsg_metrics),
                                               ctypes.POINTER(ctypes.POINTER(fsg_batch_output))]),
    "fsg_chain_look_back": (ctypes.c_int, [VP, READ_FN, VP, ctypes.POINTER(fsg_metrics),
                                           ctypes.POINTER(fsg_runtime_error)]),
    "fsg_runtime_error_free": (None, [ctypes.POINTER(fsg_runtime_error)]),
    "fsg_chain_builder_set_lookback": (ctypes.c_int, [VP, SZ, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64]),
    "fsg_chain_get_accumulator": (ctypes.c_int, [VP, SZ, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                                 ctypes.POINTER(SZ)]),
    "fsg_chain_last_timings": (ctypes.c_int, [VP, ctypes.POINTER(fsg_timings)]),
    "fsg_chain_free": (None, [VP]),
    "fsg_output_free": (None, [ctypes.POINTER(fsg_output)]),
    "fsg_batch_output_free": (None, [ctypes.POINTER(fsg_batch_output)]),
    "fsg_free": (None, [VP]),
    "fsg_host_cache_trim": (None, []),
    "fsg_slice_upload": (ctypes.c_int, [VP, VP, SZ, PP]),
    "fsg_slice_info": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "fsg_slice_free": (None, [VP]),
    "fsg_slice_device_framed": (ctypes.c_int, [VP]),
    "fsg_slice_reframe": (ctypes.c_int, [VP]),
    "fsg_slice_verify_crc_start": (ctypes.c_int, [VP]),
    "fsg_slice_verify_crc": (ctypes.c_int, [VP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_float)]),
    "fsg_chain_process_slice": (ctypes.c_int, [VP, VP, ctypes.c_uint64, ctypes.POINTER(fsg_metrics),
                                               ctypes.POINTER(ctypes.POINTER(fsg_batch_output))]),
    "fsg_chain_output_device": (ctypes.c_int, [VP, PP, ctypes.POINTER(SZ)]),
    "fsg_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "fsg_engine_comm_init": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    "fsg_allreduce_state": (ctypes.c_int, [VP, VP, SZ, ctypes.c_int]),
    "fsg_chain_allreduce_state": (ctypes.c_int, [VP, VP, SZ, ctypes.c_int]),
    "fsg_last_store_memory": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)] * 3),
    "fsg_state_new": (ctypes.c_int, [VP, SZ, ctypes.c_int, PP]),
    "fsg_state_collect": (ctypes.c_int, [VP, SZ, VP]),
    "fsg_state_allreduce": (ctypes.c_int, [VP]),
    "fsg_state_read": (ctypes.c_int, [VP, VP, SZ]),
    "fsg_state_device": (ctypes.c_int, [VP, PP]),
    "fsg_state_free": (None, [VP]),
    "fsg_keyed_new": (ctypes.c_int, [VP, PP]),
    "fsg_keyed_reset": (ctypes.c_int, [VP]),
    "fsg_keyed_collect": (ctypes.c_int, [VP, VP, SZ]),
    "fsg_keyed_allreduce": (ctypes.c_int, [VP, ctypes.POINTER(SZ), ctypes.POINTER(SZ)]),
    "fsg_keyed_read": (ctypes.c_int, [VP, VP, SZ, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                                      SZ]),
    "fsg_keyed_device": (ctypes.c_int, [VP, PP, PP, PP]),
    "fsg_keyed_free": (None, [VP]),
    "fsg_chain_group_process_slices": (ctypes.c_int, [PP, PP, SZ, ctypes.c_uint64, ctypes.POINTER(fsg_metrics),
                                                      ctypes.POINTER(ctypes.POINTER(fsg_batch_output)),
                                                      ctypes.POINTER(ctypes.c_int)]),
}

FSG_DTYPE_I32, FSG_DTYPE_U32, FSG_DTYPE_I64, FSG_DTYPE_U64, FSG_DTYPE_F64 = range(5)

_lib = None


def build() -> str:
    """Compile libfsg.so for gfx950 (hipcc cross-compiles without a GPU)."""
    env = dict(os.environ)
    subprocess.run(["make", "-s", "-j8", "-C", CSRC], check=True, env=env)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libfsg.so not built ({LIB_PATH}); run fluvio_amd._ffi.build() "
                               "— the GPU engine has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        got = L.fsg_abi_version()
        if got != ABI_VERSION:  # a stale libfsg.so would write past these structs
            raise RuntimeError(f"{LIB_PATH}: ABI version {got}, this binding expects {ABI_VERSION}; rebuild it")
        _lib = L
    return _lib


_debug = None


def debug_lib():
    """The host-only test hook library (libfsg_debug.so: the regex -> DFA compiler
    with no GPU); never part of libfsg.so or of any process call."""
    global _debug
    if _debug is None:
        path = os.path.join(_HERE, "_lib", "libfsg_debug.so")
        if not os.path.exists(path):
            raise RuntimeError(f"libfsg_debug.so not built ({path}); run fluvio_amd._ffi.build()")
        D = ctypes.CDLL(path)
        D.fsg_debug_regex_match.restype = ctypes.c_int
        D.fsg_debug_regex_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p, SZ, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        D.fsg_debug_regex_error.restype = ctypes.c_int
        D.fsg_debug_regex_error.argtypes = [ctypes.c_char_p, ctypes.c_char_p, SZ]
        _debug = D
    return _debug


_hooks = None


def hooks_lib():
    """The GPU test-hook library (libfsg_hooks.so, linked against libfsg.so):
    the keyed merge over simulated ranks; never part of libfsg.so's C ABI."""
    global _hooks
    if _hooks is None:
        lib()  # libfsg.so first (the hooks library resolves against it)
        path = os.path.join(_HERE, "_lib", "libfsg_hooks.so")
        if not os.path.exists(path):
            raise RuntimeError(f"libfsg_hooks.so not built ({path}); run fluvio_amd._ffi.build()")
        H = ctypes.CDLL(path)
        H.fsg_keyed_allreduce_sim.restype = ctypes.c_int
        H.fsg_keyed_allreduce_sim.argtypes = [VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                               PP, PP, ctypes.POINTER(ctypes.c_uint64), PP, ctypes.POINTER(SZ),
                                               ctypes.POINTER(SZ)]
        _hooks = H
    return _hooks


def buf_ptr(data):
    """(pointer, length) of a bytes-like object without copying (bytes or numpy uint8)."""
    if isinstance(data, (bytes, bytearray)):
        b = bytes(data)
        return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), len(b), b
    import numpy as np
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return ctypes.c_void_p(a.ctypes.data), a.nbytes, a


def last_error() -> str:
    m = lib().fsg_last_error_message()
    return m.decode("utf-8", "replace") if m else ""
