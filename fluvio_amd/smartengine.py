"""Host-side mirror of the fluvio-smartengine API over the MI355X C ABI.

Same names, argument meaning and error behaviour as the reference (paths
relative to /root/reference):

  SmartEngine                 crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:26-41
  SmartModuleChainBuilder     engine.rs:49-111
  SmartModuleChainInstance    engine.rs:118-218 (process, look_back)
  SmartModuleConfig(+Builder) crates/fluvio-smartengine/src/engine/config.rs:33-74
  SmartModuleInitialData      config.rs:11-28
  SmartModuleChainMetrics     crates/fluvio-smartengine/src/engine/metrics.rs:6-41
  SmartModuleInput/Output     crates/fluvio-smartmodule/src/input.rs:82-184, output.rs:12-42
  SmartModuleTransformRuntimeError  crates/fluvio-protocol/src/link/smartmodule.rs:12-72
  EngineError                 crates/fluvio-smartengine/src/engine/error.rs:1-13
  process_batch               crates/fluvio-spu/src/smartengine/batch.rs:41-142

SmartModule bytes are chosen at chain-build time: ``builtin("regex-filter")``
returns the ``b"\\0fsg"`` descriptor of a GPU built-in; real wasm (``b"\\0asm"``)
is rejected with ``UnknownSmartModule`` exactly where the reference's
``create_transform`` would fail for a module it cannot run.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from . import _ffi
from .protocol import Batch, Record, decode_batch, decode_records, encode_records

DEFAULT_SMARTENGINE_VERSION = 22  # input.rs:14 SMARTMODULE_TIMESTAMPS_VERSION

BUILTINS = ("filter", "filter_init", "filter_with_param", "regex-filter", "filter_regex", "filter_odd",
            "map", "map_double", "filter_map", "aggregate-sum", "aggregate", "aggregate-json", "filter_json",
            "array_map_json_array", "map_json_project")


def builtin(name: str) -> bytes:
    """Module bytes selecting a GPU built-in SmartModule by its reference name."""
    return b"\0fsg" + name.encode()


# ---------------------------------------------------------------------------
# errors (EngineError + guest status enums)
# ---------------------------------------------------------------------------
class EngineError(Exception):
    code = _ffi.FSG_E_UNKNOWN

    def __init__(self, message: str = "", code: Optional[int] = None):
        super().__init__(message)
        if code is not None:
            self.code = code


class UnknownSmartModule(EngineError):
    code = _ffi.FSG_E_UNKNOWN_SM


class Instantiate(EngineError):
    code = _ffi.FSG_E_INSTANTIATE


class StoreMemoryExceeded(EngineError):
    """EngineError::StoreMemoryExceeded{current, requested, max} (error.rs:2-13)."""
    code = _ffi.FSG_E_STORE_MEMORY

    def __init__(self, message: str = "", code: Optional[int] = None):
        super().__init__(message, code)
        c, r, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _ffi.lib().fsg_last_store_memory(ctypes.byref(c), ctypes.byref(r), ctypes.byref(m))
        self.current, self.requested, self.max = c.value, r.value, m.value


class SmartModuleInitError(EngineError):
    """SmartModuleInitRuntimeError surfaced by initialize() (init.rs:42-66)."""
    code = _ffi.FSG_E_INIT


class SmartModuleTransformErrorStatus(EngineError):
    """A negative guest return code (error.rs:17-34): DecodingBaseInput, ..."""


class Unsupported(EngineError):
    code = _ffi.FSG_E_UNSUPPORTED


class IoError(EngineError):
    code = _ffi.FSG_E_IO


class DeviceError(EngineError):
    code = _ffi.FSG_E_DEVICE


_ERRORS = {
    _ffi.FSG_E_UNKNOWN_SM: UnknownSmartModule, _ffi.FSG_E_INSTANTIATE: Instantiate,
    _ffi.FSG_E_STORE_MEMORY: StoreMemoryExceeded, _ffi.FSG_E_INIT: SmartModuleInitError,
    _ffi.FSG_E_DECODING_BASE_INPUT: SmartModuleTransformErrorStatus,
    _ffi.FSG_E_DECODING_RECORDS: SmartModuleTransformErrorStatus,
    _ffi.FSG_E_ENCODING_OUTPUT: SmartModuleTransformErrorStatus,
    _ffi.FSG_E_UNKNOWN: SmartModuleTransformErrorStatus,
    _ffi.FSG_E_UNSUPPORTED: Unsupported, _ffi.FSG_E_IO: IoError, _ffi.FSG_E_DEVICE: DeviceError,
}


def _check(rc: int) -> None:
    if rc != 0:
        cls = _ERRORS.get(rc, EngineError)
        raise cls(_ffi.last_error(), rc)


# ---------------------------------------------------------------------------
# config
# ---------------------------------------------------------------------------
@dataclass
class SmartModuleInitialData:
    accumulator: Optional[bytes] = None

    @staticmethod
    def none() -> "SmartModuleInitialData":
        return SmartModuleInitialData(None)

    @staticmethod
    def with_aggregate(accumulator: bytes) -> "SmartModuleInitialData":
        return SmartModuleInitialData(bytes(accumulator))


@dataclass(frozen=True)
class Lookback:
    """Lookback (fluvio-smartengine engine/config.rs:45-49): Last(n) or Age{age, last}."""
    last: int
    age_ms: Optional[int] = None

    @staticmethod
    def Last(n: int) -> "Lookback":  # noqa: N802 (the reference's variant name)
        return Lookback(n)

    @staticmethod
    def Age(age_ms: int, last: int) -> "Lookback":  # noqa: N802
        return Lookback(last, age_ms)


@dataclass
class SmartModuleLookbackRuntimeError(Exception):
    """SmartModuleLookbackRuntimeError (fluvio-protocol link/smartmodule.rs:150-176)."""
    hint: str
    offset: int
    record_key: Optional[bytes]
    record_value: bytes

    def __str__(self) -> str:
        def disp(b: Optional[bytes]) -> str:
            if b is None:
                return "NULL"
            try:
                return b.decode("utf-8")
            except UnicodeDecodeError:
                return f"Binary: {len(b)} bytes"
        return (f"{self.hint}\n\nSmartModule Lookback Error: \n    Offset: {self.offset}\n"
                f"    Key: {disp(self.record_key)}\n    Value: {disp(self.record_value)}")


@dataclass
class SmartModuleConfig:
    params: Dict[str, str] = field(default_factory=dict)
    initial_data: SmartModuleInitialData = field(default_factory=SmartModuleInitialData)
    version: Optional[int] = None
    lookback: Optional[object] = None

    @staticmethod
    def builder() -> "SmartModuleConfigBuilder":
        return SmartModuleConfigBuilder()

    def get_version(self) -> int:
        return DEFAULT_SMARTENGINE_VERSION if self.version is None else self.version


class SmartModuleConfigBuilder:
    def __init__(self):
        self._c = SmartModuleConfig()

    def param(self, key: str, value: str) -> "SmartModuleConfigBuilder":
        self._c.params[key] = value
        return self

    def params(self, params: Dict[str, str]) -> "SmartModuleConfigBuilder":
        self._c.params = dict(params)
        return self

    def initial_data(self, data: SmartModuleInitialData) -> "SmartModuleConfigBuilder":
        self._c.initial_data = data
        return self

    def version(self, v: int) -> "SmartModuleConfigBuilder":
        self._c.version = v
        return self

    def lookback(self, lb) -> "SmartModuleConfigBuilder":
        self._c.lookback = lb
        return self

    def build(self) -> SmartModuleConfig:
        return self._c


class SmartModuleChainMetrics:
    def __init__(self):
        self._m = _ffi.fsg_metrics()

    def bytes_in(self) -> int:
        return self._m.bytes_in

    def records_out(self) -> int:
        return self._m.records_out

    def invocation_count(self) -> int:
        return self._m.invocation_count

    def fuel_used(self) -> int:
        return self._m.fuel_used


# ---------------------------------------------------------------------------
# input / output
# ---------------------------------------------------------------------------
@dataclass
class SmartModuleInput:
    raw_bytes: bytes
    base_offset: int = 0
    base_timestamp: int = 0

    @staticmethod
    def new(raw_bytes: bytes, base_offset: int, base_timestamp: int) -> "SmartModuleInput":
        return SmartModuleInput(bytes(raw_bytes), base_offset, base_timestamp)

    @staticmethod
    def try_from_records(records: List[Record], version: int = DEFAULT_SMARTENGINE_VERSION) -> "SmartModuleInput":
        return SmartModuleInput(encode_records(records), 0, 0)

    def set_base_offset(self, v: int) -> None:
        self.base_offset = v

    def set_base_timestamp(self, v: int) -> None:
        self.base_timestamp = v


@dataclass
class SmartModuleTransformRuntimeError(Exception):
    hint: str
    offset: int
    kind: int
    record_key: Optional[bytes]
    record_value: bytes

    KIND_NAMES = {0: "Filter", 1: "Map", 2: "ArrayMap", 3: "Aggregate", 4: "FilterMap"}

    def __str__(self) -> str:  # Display (link/smartmodule.rs:46-64)
        def disp(b: Optional[bytes]) -> str:
            if b is None:
                return "NULL"
            try:
                return b.decode("utf-8")
            except UnicodeDecodeError:
                return f"Binary: {len(b)} bytes"
        return (f"{self.hint}\n\nSmartModule Info: \n    Type: {self.KIND_NAMES.get(self.kind, self.kind)}\n"
                f"    Offset: {self.offset}\n    Key: {disp(self.record_key)}\n    Value: {disp(self.record_value)}")


def _runtime_error(e: _ffi.fsg_runtime_error) -> SmartModuleTransformRuntimeError:
    return SmartModuleTransformRuntimeError(
        hint=ctypes.string_at(e.hint, e.hint_len).decode("utf-8", "replace") if e.hint_len else "",
        offset=e.offset, kind=e.kind,
        record_key=ctypes.string_at(e.key, e.key_len) if e.has_key else None,
        record_value=ctypes.string_at(e.value, e.value_len) if e.value_len else b"")


@dataclass
class SmartModuleOutput:
    raw_successes: bytes  # encoded Vec<Record>
    error: Optional[SmartModuleTransformRuntimeError] = None

    @property
    def successes(self) -> List[Record]:
        return decode_records(self.raw_successes)


@dataclass
class BatchOutput:
    """(Batch, Option<SmartModuleTransformRuntimeError>) of SPU process_batch."""
    raw: bytes
    base_offset: int
    last_offset_delta: int
    n_records: int
    error: Optional[SmartModuleTransformRuntimeError] = None

    def batch(self):
        return decode_batch(self.raw)[0]

    def records(self) -> List[Record]:
        return self.batch().memory_records()


# ---------------------------------------------------------------------------
# engine / builder / chain
# ---------------------------------------------------------------------------
class SmartEngine:
    """SmartEngine::new — binds one MI355X (default: LOCAL_RANK or 0)."""

    def __init__(self, device: Optional[int] = None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        h = ctypes.c_void_p()
        _check(_ffi.lib().fsg_engine_new(device, ctypes.byref(h)))
        self._h = h
        self.device = device

    @staticmethod
    def new() -> "SmartEngine":
        return SmartEngine()

    def comm_init(self, unique_id: bytes, nranks: int, rank: int) -> None:
        _check(_ffi.lib().fsg_engine_comm_init(self._h, unique_id, nranks, rank))

    def allreduce_state(self, dev_ptr: int, count: int, dtype: int = _ffi.FSG_DTYPE_I32) -> None:
        """RCCL sum of `count` state elements in HBM across the engine's communicator."""
        _check(_ffi.lib().fsg_allreduce_state(self._h, ctypes.c_void_p(dev_ptr), count, dtype))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value and _ffi._lib is not None:
            _ffi.lib().fsg_engine_free(h)
            self._h = None


class PartitionState:
    """Per-partition aggregate state vector in HBM (fsg_state_*): one i32 slot
    per topic partition, filled device-to-device from each partition's
    aggregate-sum chain and merged across GPUs with an RCCL all-reduce."""

    def __init__(self, engine: SmartEngine, count: int, dtype: int = _ffi.FSG_DTYPE_I32):
        h = ctypes.c_void_p()
        _check(_ffi.lib().fsg_state_new(engine._h, count, dtype, ctypes.byref(h)))
        self._h, self._engine, self.count, self.dtype = h, engine, count, dtype

    def collect(self, slot: int, chain: "SmartModuleChainInstance") -> None:
        _check(_ffi.lib().fsg_state_collect(self._h, slot, chain._h))

    def allreduce(self) -> None:
        _check(_ffi.lib().fsg_state_allreduce(self._h))

    def device_ptr(self) -> int:
        p = ctypes.c_void_p()
        _check(_ffi.lib().fsg_state_device(self._h, ctypes.byref(p)))
        return p.value or 0

    def read(self) -> List[int]:
        import array
        a = array.array("i" if self.dtype == _ffi.FSG_DTYPE_I32 else "q", [0] * self.count)
        addr, _ = a.buffer_info()
        _check(_ffi.lib().fsg_state_read(self._h, ctypes.c_void_p(addr), self.count * a.itemsize))
        return list(a)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value and _ffi._lib is not None:
            _ffi.lib().fsg_state_free(h)
            self._h = None


def process_slices(chains, slices, max_bytes: int = (1 << 64) - 1, metrics=None, download: bool = False):
    """fsg_chain_group_process_slices: every chain over its resident slice in one
    call (the partitions a rank owns), outputs left in HBM unless `download`;
    aggregate-json's stream-order walks run as one launch over all chains.
    Returns the BatchOutputs when downloading."""
    n = len(chains)
    assert len(slices) == n
    ch = (ctypes.c_void_p * n)(*[c._h.value if isinstance(c._h, ctypes.c_void_p) else c._h for c in chains])
    sl = (ctypes.c_void_p * n)(*[s._h.value if isinstance(s._h, ctypes.c_void_p) else s._h for s in slices])
    rcs = (ctypes.c_int * max(n, 1))()
    m = None
    if metrics is not None:
        m = (_ffi.fsg_metrics * n)()
    outs = (ctypes.POINTER(_ffi.fsg_batch_output) * n)() if download else None
    rc = _ffi.lib().fsg_chain_group_process_slices(ch, sl, n, max_bytes, m, outs, rcs)
    if download:
        res = [chains[i]._batch_result(outs[i]) if outs[i] else None for i in range(n)]
    _check(rc)
    if metrics is not None:
        for i in range(n):
            metrics[i]._m.bytes_in += m[i].bytes_in
            metrics[i]._m.records_out += m[i].records_out
            metrics[i]._m.invocation_count += m[i].invocation_count
            metrics[i]._m.fuel_used += m[i].fuel_used
    return res if download else None


class KeyedState:
    """Topic-wide keyed totals of aggregate-json chains (fsg_keyed_*): collect
    each owned partition's map (exact keys, device side), then `allreduce()`
    builds the topic key dictionary over the engine's communicator (RCCL
    all-gather of the key lists, dense K-slot u32 all-reduce), or locally on one
    rank.  `read()` -> {key bytes: u32 total}."""

    def __init__(self, engine: "SmartEngine"):
        h = ctypes.c_void_p()
        _check(_ffi.lib().fsg_keyed_new(engine._h, ctypes.byref(h)))
        self._h = h
        self._engine = engine
        self.n_keys = 0
        self.key_bytes = 0

    def reset(self) -> None:
        _check(_ffi.lib().fsg_keyed_reset(self._h))

    def collect(self, chain: "SmartModuleChainInstance", stage: int = 0) -> None:
        _check(_ffi.lib().fsg_keyed_collect(self._h, chain._h, stage))

    def allreduce(self) -> int:
        n, b = ctypes.c_size_t(), ctypes.c_size_t()
        _check(_ffi.lib().fsg_keyed_allreduce(self._h, ctypes.byref(n), ctypes.byref(b)))
        self.n_keys, self.key_bytes = n.value, b.value
        return n.value

    def allreduce_simulated(self, me: int, ranks) -> int:
        """fsg_keyed_allreduce_sim: this table as rank `me`, `ranks[r]` = rank r's
        (key list with None for a dead entry, values) for r != me."""
        from . import partitions as PT
        nr = len(ranks)
        n = (ctypes.c_uint64 * nr)()
        alen = (ctypes.c_uint64 * nr)()
        dptr, aptr, vptr = (ctypes.c_void_p * nr)(), (ctypes.c_void_p * nr)(), (ctypes.c_void_p * nr)()
        keep = []
        for r, item in enumerate(ranks):
            if r == me or item is None:
                continue
            keys, vals = item
            desc, arena = PT.keyed_desc(keys)
            d = (ctypes.c_uint64 * max(len(desc), 1))(*desc)
            a = ctypes.create_string_buffer(arena, max(len(arena), 1))
            v = (ctypes.c_uint32 * max(len(vals), 1))(*vals)
            keep += [d, a, v]
            n[r], alen[r] = len(desc), len(arena)
            dptr[r], aptr[r], vptr[r] = ctypes.cast(d, ctypes.c_void_p), ctypes.cast(a, ctypes.c_void_p), \
                ctypes.cast(v, ctypes.c_void_p)
        nk, b = ctypes.c_size_t(), ctypes.c_size_t()
        _check(_ffi.hooks_lib().fsg_keyed_allreduce_sim(self._h, nr, me, n, dptr, aptr, alen, vptr, ctypes.byref(nk),
                                                  ctypes.byref(b)))
        self.n_keys, self.key_bytes = nk.value, b.value
        return nk.value

    def read(self) -> Dict[bytes, int]:
        n = self.n_keys
        keys = ctypes.create_string_buffer(max(self.key_bytes, 1))
        offs = (ctypes.c_uint64 * (n + 1))()
        vals = (ctypes.c_uint32 * max(n, 1))()
        _check(_ffi.lib().fsg_keyed_read(self._h, keys, self.key_bytes, offs, vals, n))
        raw = keys.raw
        return {raw[offs[i]:offs[i + 1]]: int(vals[i]) for i in range(n)}

    def close(self) -> None:
        if self._h:
            _ffi.lib().fsg_keyed_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(_ffi.lib().fsg_comm_unique_id(buf))
    return buf.raw


class SmartModuleChainBuilder:
    def __init__(self):
        self._mods: List[Tuple[SmartModuleConfig, bytes]] = []
        self._limit: Optional[int] = None

    @staticmethod
    def default() -> "SmartModuleChainBuilder":
        return SmartModuleChainBuilder()

    @staticmethod
    def from_pair(config: SmartModuleConfig, module: bytes) -> "SmartModuleChainBuilder":
        b = SmartModuleChainBuilder()
        b.add_smart_module(config, module)
        return b

    def add_smart_module(self, config: SmartModuleConfig, module: bytes) -> None:
        self._mods.append((config, bytes(module)))

    def set_store_memory_limit(self, max_memory_bytes: int) -> None:
        self._limit = max_memory_bytes

    def initialize(self, engine: SmartEngine) -> "SmartModuleChainInstance":
        L = _ffi.lib()
        b = ctypes.c_void_p()
        _check(L.fsg_chain_builder_new(ctypes.byref(b)))
        if self._limit is not None:
            L.fsg_chain_builder_set_store_memory_limit(b, self._limit)
        for idx, (cfg, module) in enumerate(self._mods):
            items = list(cfg.params.items())
            arr = (_ffi.fsg_param * max(1, len(items)))()
            for i, (k, v) in enumerate(items):
                arr[i].key = k.encode()
                arr[i].value = v.encode()
            acc = cfg.initial_data.accumulator
            _check(L.fsg_chain_builder_add_smart_module(
                b, arr, len(items), cfg.get_version(), acc or b"", len(acc or b""), 1 if acc is not None else 0,
                module, len(module)))
            lb = cfg.lookback
            if lb is not None:
                kind = _ffi.FSG_LOOKBACK_LAST if lb.age_ms is None else _ffi.FSG_LOOKBACK_AGE
                _check(L.fsg_chain_builder_set_lookback(b, idx, kind, lb.last, lb.age_ms or 0))
        c = ctypes.c_void_p()
        _check(L.fsg_chain_builder_initialize(b, engine._h, ctypes.byref(c)))  # consumes the builder
        return SmartModuleChainInstance(c, engine, len(self._mods))


class SmartModuleChainInstance:
    def __init__(self, handle: ctypes.c_void_p, engine: SmartEngine, n: int):
        self._h = handle
        self._engine = engine  # keep the engine alive
        self.n_instances = n

    def process(self, input: SmartModuleInput,
                metrics: Optional[SmartModuleChainMetrics] = None) -> SmartModuleOutput:
        m = metrics._m if metrics is not None else None
        out = ctypes.POINTER(_ffi.fsg_output)()
        _check(_ffi.lib().fsg_chain_process(self._h, input.raw_bytes, len(input.raw_bytes), input.base_offset,
                                            input.base_timestamp, ctypes.byref(m) if m is not None else None,
                                            ctypes.byref(out)))
        try:
            o = out.contents
            raw = ctypes.string_at(o.records, o.records_len) if o.records_len else b"\0\0\0\0"
            err = _runtime_error(o.error) if o.has_error else None
            return SmartModuleOutput(raw, err)
        finally:
            _ffi.lib().fsg_output_free(out)

    def look_back(self, read_fn: Callable, metrics: Optional[SmartModuleChainMetrics] = None) -> None:
        """SmartModuleChainInstance::look_back (engine.rs:187-218): read_fn(Lookback)
        returns the records (a list of Record, or an encoded Vec<Record>) the
        stage's look_back runs over; a record error raises
        SmartModuleLookbackRuntimeError."""
        keep = []

        def _read(user, lbp, recs, ln):
            try:
                lb = lbp.contents
                got = read_fn(Lookback(lb.last, None if lb.kind == _ffi.FSG_LOOKBACK_LAST else lb.age_ms))
                raw = got if isinstance(got, (bytes, bytearray)) else encode_records(list(got))
                buf = ctypes.create_string_buffer(bytes(raw), max(1, len(raw)))
                keep.append(buf)
                recs[0] = ctypes.cast(buf, ctypes.c_void_p)
                ln[0] = len(raw)
                return 0
            except Exception:  # noqa: BLE001 (the read failed: io::Error for look_back)
                return 1

        cb = _ffi.READ_FN(_read)
        err = _ffi.fsg_runtime_error()
        rc = _ffi.lib().fsg_chain_look_back(self._h, cb, None, ctypes.byref(metrics._m) if metrics else None,
                                            ctypes.byref(err))
        if rc == _ffi.FSG_E_LOOKBACK:
            e = _runtime_error(err)
            _ffi.lib().fsg_runtime_error_free(ctypes.byref(err))
            raise SmartModuleLookbackRuntimeError(e.hint, e.offset, e.record_key, e.record_value)
        _check(rc)

    def accumulator(self, stage: int) -> bytes:
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        _check(_ffi.lib().fsg_chain_get_accumulator(self._h, stage, ctypes.byref(p), ctypes.byref(n)))
        data = ctypes.string_at(p, n.value) if n.value else b""
        _ffi.lib().fsg_free(p)
        return data


    def last_timings(self) -> Dict[str, float]:
        t = _ffi.fsg_timings()
        _check(_ffi.lib().fsg_chain_last_timings(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in _ffi.fsg_timings._fields_}

    def _batch_result(self, out) -> BatchOutput:
        try:
            o = out.contents
            n = o.batch_len
            if n < (1 << 31):
                raw = ctypes.string_at(o.batch, n)
            else:  # string_at takes a C int size
                raw = bytearray(n)
                ctypes.memmove((ctypes.c_char * n).from_buffer(raw), o.batch, n)
            err = _runtime_error(o.error) if o.has_error else None
            return BatchOutput(raw, o.base_offset, o.last_offset_delta, o.n_records, err)
        finally:
            _ffi.lib().fsg_batch_output_free(out)

    def process_batch(self, slice_bytes: bytes, max_bytes: int = (1 << 64) - 1,
                      metrics: Optional[SmartModuleChainMetrics] = None) -> BatchOutput:
        out = ctypes.POINTER(_ffi.fsg_batch_output)()
        _check(_ffi.lib().fsg_chain_process_batch(self._h, slice_bytes, len(slice_bytes), max_bytes,
                                                  ctypes.byref(metrics._m) if metrics else None,
                                                  ctypes.byref(out)))
        return self._batch_result(out)

    def process_slice(self, sl: "ResidentSlice", max_bytes: int = (1 << 64) - 1,
                      metrics: Optional[SmartModuleChainMetrics] = None, download: bool = True):
        out = ctypes.POINTER(_ffi.fsg_batch_output)()
        _check(_ffi.lib().fsg_chain_process_slice(self._h, sl._h, max_bytes,
                                                  ctypes.byref(metrics._m) if metrics else None,
                                                  ctypes.byref(out) if download else None))
        return self._batch_result(out) if download else None

    def output_device(self) -> Tuple[int, int]:
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _check(_ffi.lib().fsg_chain_output_device(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value or 0, n.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value and _ffi._lib is not None:
            _ffi.lib().fsg_chain_free(h)
            self._h = None


class ResidentSlice:
    """A fetch slice of stored batches ingested into HBM once (FileBatchIterator framing)."""

    def __init__(self, engine: SmartEngine, slice_bytes: bytes):
        h = ctypes.c_void_p()
        ptr, n, keep = _ffi.buf_ptr(slice_bytes)
        _check(_ffi.lib().fsg_slice_upload(engine._h, ptr, n, ctypes.byref(h)))
        del keep
        self._h = h
        self._engine = engine
        nb, nr, by = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _ffi.lib().fsg_slice_info(h, ctypes.byref(nb), ctypes.byref(nr), ctypes.byref(by))
        self.n_batches, self.n_records, self.bytes = nb.value, nr.value, by.value
        self.device_framed = bool(_ffi.lib().fsg_slice_device_framed(h))

    def reframe(self):
        """Frame the resident bytes again on the device, as a freshly fetched
        slice (the fetch-shaped measurement: framing + verify + process)."""
        _check(_ffi.lib().fsg_slice_reframe(self._h))

    def verify_crc_start(self):
        """Start the CRC32C check on the slice's own stream and return at
        once; the next verify_crc() returns its result."""
        _check(_ffi.lib().fsg_slice_verify_crc_start(self._h))

    def verify_crc(self):
        """CRC32C of every stored batch checked on the GPU (report only: the
        reference never verifies).  Returns (mismatches, first bad batch or -1,
        kernel ms)."""
        nb, fb, ms = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_float()
        _check(_ffi.lib().fsg_slice_verify_crc(self._h, ctypes.byref(nb), ctypes.byref(fb), ctypes.byref(ms)))
        return nb.value, fb.value, ms.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value and _ffi._lib is not None:
            _ffi.lib().fsg_slice_free(h)
            self._h = None


def process_batch(chain: SmartModuleChainInstance, slice_bytes: bytes, max_bytes: int,
                  metrics: Optional[SmartModuleChainMetrics] = None
                  ) -> Tuple[Batch, Optional[SmartModuleTransformRuntimeError]]:
    """fluvio-spu process_batch (batch.rs:41-142): returns (Batch, Option<error>)."""
    out = chain.process_batch(slice_bytes, max_bytes, metrics)
    b = out.batch()
    batch = Batch(base_offset=b.base_offset, header=b.header, records=b.memory_records())
    return batch, out.error
