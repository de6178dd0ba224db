"""ctypes wrapper of the CPU oracle (oracle/fsg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / timed CPU baseline.  The product
path (fluvio_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, Iterable, List, Optional, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libfsg_oracle.so")
_lib = None


class _Result(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int),
        ("bytes", ctypes.POINTER(ctypes.c_uint8)),
        ("bytes_len", ctypes.c_size_t),
        ("n_records", ctypes.c_uint32),
        ("base_offset", ctypes.c_int64),
        ("last_offset_delta", ctypes.c_int32),
        ("has_error", ctypes.c_int),
        ("hint", ctypes.POINTER(ctypes.c_char)),  # hint_len bytes (a serde text may hold a NUL)
        ("hint_len", ctypes.c_size_t),
        ("err_offset", ctypes.c_int64),
        ("err_kind", ctypes.c_int32),
        ("has_key", ctypes.c_int),
        ("key", ctypes.POINTER(ctypes.c_uint8)),
        ("key_len", ctypes.c_size_t),
        ("value", ctypes.POINTER(ctypes.c_uint8)),
        ("value_len", ctypes.c_size_t),
        ("message", ctypes.c_char_p),
        ("m_bytes_in", ctypes.c_uint64),
        ("m_records_out", ctypes.c_uint64),
        ("m_invocations", ctypes.c_uint64),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_crc32c.restype = ctypes.c_uint32
        L.orc_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_chain_new.restype = ctypes.c_void_p
        L.orc_chain_free.argtypes = [ctypes.c_void_p]
        L.orc_chain_add.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.c_char_p,
                                    ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.orc_chain_process.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.POINTER(_Result)]
        L.orc_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64,
                                        ctypes.POINTER(_Result)]
        L.orc_chain_accumulator.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                            ctypes.POINTER(ctypes.c_size_t)]
        L.orc_chain_look_back.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.POINTER(_Result)]
        L.orc_result_free.argtypes = [ctypes.POINTER(_Result)]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_regex_is_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_int)]
        L.orc_json_structured_log.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.orc_json_struct.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                      ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.orc_json_array_map.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_size_t)),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.orc_json_project.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_size_t)]
        for fn in (L.orc_decompress, L.orc_compress):
            fn.restype = ctypes.c_int
        L.orc_decompress.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.orc_compress.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.orc_xxh32.restype = ctypes.c_uint32
        L.orc_xxh32.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.orc_varint_encode.restype = ctypes.c_size_t
        L.orc_varint_encode.argtypes = [ctypes.c_int64, ctypes.c_char_p]
        L.orc_siphash.restype = ctypes.c_uint64
        L.orc_siphash.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                  ctypes.c_size_t]
        _lib = L
    return _lib


def siphash(c_rounds: int, d_rounds: int, k0: int, k1: int, data: bytes) -> int:
    return lib().orc_siphash(c_rounds, d_rounds, k0, k1, data, len(data))


def crc32c(data: bytes) -> int:
    return lib().orc_crc32c(data, len(data))


CODECS = {"gzip": 1, "snappy": 2, "lz4": 3, "zstd": 4}


def decompress(codec: int, data: bytes):
    """Compression::uncompress (fsg_codec.c): bytes, or None on a decode error."""
    p, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = lib().orc_decompress(codec, data, len(data), ctypes.byref(p), ctypes.byref(n))
    if rc == -1:
        return None
    if rc:
        raise OracleError(rc, "unsupported codec")
    out = ctypes.string_at(p, n.value)
    lib().orc_free(p)
    return out


def compress(codec: int, data: bytes, flags: int = 0) -> bytes:
    """Test-data encoders: 1 gzip (flags = zlib level), 2 snappy frame, 3 lz4 frame."""
    p, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = lib().orc_compress(codec, data, len(data), flags, ctypes.byref(p), ctypes.byref(n))
    if rc:
        raise OracleError(rc, "compress")
    out = ctypes.string_at(p, n.value)
    lib().orc_free(p)
    return out


def xxh32(data: bytes, seed: int = 0) -> int:
    return lib().orc_xxh32(data, len(data), seed)


def varint_encode(v: int) -> bytes:
    buf = ctypes.create_string_buffer(16)
    n = lib().orc_varint_encode(v, buf)
    return buf.raw[:n]


def regex_is_match(pattern: str, text: bytes) -> bool:
    m = ctypes.c_int(0)
    rc = lib().orc_regex_is_match(pattern.encode(), text, len(text), ctypes.byref(m))
    if rc:
        raise ValueError(f"oracle regex status {rc}")
    return bool(m.value)


def _json_result(rc, msg, ml):
    if rc == 0:
        return None
    if rc == 1:
        text = ctypes.string_at(msg.value, ml.value)
        lib().orc_free(msg)
        return text.decode("utf-8", "replace") if isinstance(text, bytes) else text
    raise OracleError(rc, "outside the serde_json restatement")


def json_structured_log(value: bytes):
    """serde_json::from_slice::<StructuredLog>: ("ok", level 0..3) or ("err", Display text)."""
    lv = ctypes.c_int(0)
    msg = ctypes.c_void_p()
    ml = ctypes.c_size_t(0)
    rc = lib().orc_json_structured_log(value, len(value), ctypes.byref(lv), ctypes.byref(msg), ctypes.byref(ml))
    err = _json_result(rc, msg, ml)
    return ("ok", lv.value) if err is None else ("err", err)


def json_array_map(value: bytes):
    """array_map_json_array: ("ok", [canonical element bytes]) / ("err", Display text);
    raises OracleError(-103) outside the restatement."""
    el = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))()
    ln = ctypes.POINTER(ctypes.c_size_t)()
    cnt = ctypes.c_size_t()
    msg = ctypes.c_void_p()
    ml = ctypes.c_size_t(0)
    rc = lib().orc_json_array_map(value, len(value), ctypes.byref(el), ctypes.byref(ln), ctypes.byref(cnt),
                                  ctypes.byref(msg), ctypes.byref(ml))
    if rc == 0:
        out = [ctypes.string_at(el[i], ln[i]) for i in range(cnt.value)]
        for i in range(cnt.value):
            lib().orc_free(el[i])
        lib().orc_free(el)
        lib().orc_free(ln)
        return "ok", out
    err = _json_result(rc, msg, ml)
    return "err", err


def json_project(value: bytes, field: str = "message"):
    """map_json_project: ("ok", canonical bytes or None if the field is absent) / ("err", text)."""
    out = ctypes.POINTER(ctypes.c_uint8)()
    ol = ctypes.c_size_t()
    found = ctypes.c_int()
    msg = ctypes.c_void_p()
    ml = ctypes.c_size_t(0)
    rc = lib().orc_json_project(value, len(value), field.encode(), ctypes.byref(out), ctypes.byref(ol),
                                ctypes.byref(found), ctypes.byref(msg), ctypes.byref(ml))
    if rc == 0:
        if not found.value:
            return "ok", None
        v = ctypes.string_at(out, ol.value)
        lib().orc_free(out)
        return "ok", v
    return "err", _json_result(rc, msg, ml)


def json_struct(value: bytes, name: str, fields):
    """Generic derive(Deserialize) struct (fields "f" = String, "f=a|b" = unit enum)."""
    arr = (ctypes.c_char_p * len(fields))(*[f.encode() for f in fields])
    vals = (ctypes.c_int * len(fields))()
    msg = ctypes.c_void_p()
    ml = ctypes.c_size_t(0)
    rc = lib().orc_json_struct(value, len(value), name.encode(), arr, len(fields), vals, ctypes.byref(msg),
                               ctypes.byref(ml))
    err = _json_result(rc, msg, ml)
    return ("ok", list(vals)) if err is None else ("err", err)


class OracleError(Exception):
    def __init__(self, status: int, message: str = ""):
        super().__init__(f"oracle status {status}: {message}")
        self.status = status
        self.message = message


def _take(r: _Result) -> Dict:
    def raw(p, n):
        return ctypes.string_at(p, n) if n else b""

    out = {
        "status": r.status,
        "bytes": raw(r.bytes, r.bytes_len),
        "n_records": r.n_records,
        "base_offset": r.base_offset,
        "last_offset_delta": r.last_offset_delta,
        "error": None,
        "metrics": {"bytes_in": r.m_bytes_in, "records_out": r.m_records_out,
                    "invocation_count": r.m_invocations},
    }
    if r.has_error:
        out["error"] = {
            "hint": ctypes.string_at(r.hint, r.hint_len).decode("utf-8", "replace"),
            "offset": r.err_offset,
            "kind": r.err_kind,
            "key": raw(r.key, r.key_len) if r.has_key else None,
            "value": raw(r.value, r.value_len),
        }
    return out


class OracleChain:
    """A chain of built-in SmartModules identified by reference module name."""

    def __init__(self, modules: Iterable[Tuple[str, Optional[Dict[str, str]], Optional[bytes]]] = ()):
        self._h = ctypes.c_void_p(lib().orc_chain_new())
        self.n = 0
        for spec in modules:
            name, params, acc = (tuple(spec) + (None, None))[:3]
            self.add(name, params or {}, acc)

    def add(self, name: str, params: Dict[str, str], acc: Optional[bytes] = None) -> None:
        items = list(params.items())
        keys = (ctypes.c_char_p * max(1, len(items)))(*[k.encode() for k, _ in items])
        vals = (ctypes.c_char_p * max(1, len(items)))(*[v.encode() for _, v in items])
        msg = ctypes.c_void_p()
        rc = lib().orc_chain_add(self._h, name.encode(), keys, vals, len(items), acc or b"",
                                 len(acc or b""), 1 if acc is not None else 0, ctypes.byref(msg))
        text = ""
        if msg.value:
            text = ctypes.string_at(msg.value).decode()
            lib().orc_free(msg)
        if rc:
            raise OracleError(rc, text)
        self.n += 1

    def process(self, raw: bytes, base_offset: int = 0, base_timestamp: int = -1) -> Dict:
        r = _Result()
        lib().orc_chain_process(self._h, raw, len(raw), base_offset, base_timestamp, ctypes.byref(r))
        try:
            return _take(r)
        finally:
            lib().orc_result_free(ctypes.byref(r))

    def process_batch(self, slice_bytes: bytes, max_bytes: int = (1 << 64) - 1) -> Dict:
        r = _Result()
        lib().orc_process_batch(self._h, slice_bytes, len(slice_bytes), max_bytes, ctypes.byref(r))
        try:
            return _take(r)
        finally:
            lib().orc_result_free(ctypes.byref(r))

    def look_back(self, stage: int, raw: bytes) -> Dict:
        """look_back of one stage over encoded records (Vec<Record>); "error" is the
        SmartModuleLookbackRuntimeError (hint, offset, key, value)."""
        r = _Result()
        lib().orc_chain_look_back(self._h, stage, raw, len(raw), ctypes.byref(r))
        try:
            return _take(r)
        finally:
            lib().orc_result_free(ctypes.byref(r))

    def accumulator(self, stage: int) -> bytes:
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        rc = lib().orc_chain_accumulator(self._h, stage, ctypes.byref(p), ctypes.byref(n))
        if rc:
            raise OracleError(rc)
        data = ctypes.string_at(p, n.value) if n.value else b""
        lib().orc_free(p)
        return data

    def __del__(self):
        try:
            if self._h:
                lib().orc_chain_free(self._h)
                self._h = None
        except Exception:
            pass
