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


def last_int_sum() -> int:
    """The sum of the integers of the last kind-3 slice generated (the
    generator's own ground truth, for aggregate-sum checks without a GPU)."""
    L = _l()
    L.synth_last_sum.restype = ctypes.c_int64
    return int(L.synth_last_sum())


def make_keyed_slices(partitions: int = 64, nrec: int = 5000, nkeys: int = 10000, seed: int = 0xF106,
                      owned=None, key_sums: dict = None) -> dict:
    """C5 keyed: records `{"repo-NNNN": n}` (aggregate-json input), the record
    key = the repo name, routed to partition SipHash(key) mod P exactly as
    fluvio's producer does (partitioning.rs:70-83), so every key lives in one
    partition.  ~16 KiB batches (tools/synth.c synth_keyed); returns
    {partition: slice bytes} for `owned` (all partitions by default)."""
    from . import partitions as PT
    keys = [b"repo-%04d" % i for i in range(nkeys)]
    by_p = {}
    for k in keys:
        by_p.setdefault(PT.partition_siphash(k, partitions), []).append(k)
    L = _l()
    L.synth_keyed.restype = ctypes.c_size_t
    L.synth_keyed.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t]
    L.synth_key_sums.argtypes = [ctypes.c_void_p]
    L.synth_key_sums.restype = None
    out = {}
    for p in (owned if owned is not None else range(partitions)):
        ks = by_p.get(p) or [b"repo-none"]
        sums = np.zeros(len(ks), dtype=np.uint64)
        L.synth_key_sums(sums.ctypes.data if key_sums is not None else None)
        blob = b"".join(ks)
        off = np.zeros(len(ks) + 1, dtype=np.uint32)
        off[1:] = np.cumsum([len(k) for k in ks])
        cap = nrec * 80 + 65536
        buf = np.zeros(cap, dtype=np.uint8)
        n = L.synth_keyed(blob, off.ctypes.data, len(ks), nrec, seed * 1000003 + p, 0, buf.ctypes.data, cap)
        L.synth_key_sums(None)
        assert n, "synth_keyed: buffer too small"
        out[p] = buf[:n].tobytes()
        if key_sums is not None:  # the generator's ground truth: committed values per key
            for k, v in zip(ks, sums.tolist()):
                if v:
                    key_sums[k] = key_sums.get(k, 0) + int(v)
    return out
