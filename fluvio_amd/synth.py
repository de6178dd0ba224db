"""Synthetic fetch slices for tests and bench.py (see fluvio_amd/tools/synth.c).

kind 1: C1 regex workload (256 B printable ASCII, ~50 % SSN), seed 0xF100
kind 2: C2 JSON logs (~1 KB, ~50 % contain "timeout"), seed 0xF101
kind 3: decimal i32 values (aggregate-sum / filter_map), seed 0xF105
kind 4: edge cases (empty values, keys, invalid UTF-8, multi-byte UTF-8)
kind 5: C4 JSON arrays of 1-16 ints / short ASCII strings (array_map), seed 0xF104
"""
import ctypes
import os

import numpy as np

from . import _ffi

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libfsg_synth.so")
_lib = None

SEEDS = {1: 0xF100, 2: 0xF101, 3: 0xF105, 4: 0xF1EE, 5: 0xF104}
REC_BYTES = {1: 272, 2: 1100, 3: 16, 4: 64, 5: 200}


def _l():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            _ffi.build()
        L = ctypes.CDLL(_LIB)
        L.synth_slice.restype = ctypes.c_size_t
        L.synth_slice.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64,
                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        _lib = L
    return _lib


def make_slice_array(kind: int, nrec: int, seed: int = None, base_offset: int = 0,
                     max_section: int = 16384) -> np.ndarray:
    """The encoded batches (file format) holding `nrec` records, as a uint8 array
    (no copy; for the multi-GB bench slices)."""
    seed = SEEDS[kind] if seed is None else seed
    cap = nrec * REC_BYTES[kind] + (nrec // 4 + 16) * 64 + (1 << 16)
    buf = np.empty(cap, dtype=np.uint8)
    n = _l().synth_slice(kind, nrec, seed, base_offset, buf.ctypes.data, cap, max_section)
    if n == 0 and nrec:
        raise RuntimeError("synth buffer too small")
    return buf[:n]


def make_slice(kind: int, nrec: int, seed: int = None, base_offset: int = 0, max_section: int = 16384) -> bytes:
    """Returns the encoded batches (file format) holding `nrec` records."""
    return make_slice_array(kind, nrec, seed, base_offset, max_section).tobytes()
