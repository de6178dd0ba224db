"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's own known answers.  Bit-exact on output batch bytes (incl. CRC32C),
error records, metrics and aggregate state.

Every test here needs an MI355X (marked gpu).
"""
import random
import struct

import os

import pytest

from fluvio_amd import protocol as P
from fluvio_amd import synth
from fluvio_amd.smartengine import (IoError, SmartEngine, SmartModuleChainBuilder, SmartModuleChainMetrics,
                                    SmartModuleConfig, SmartModuleInitError, SmartModuleInitialData,
                                    SmartModuleInput, SmartModuleTransformErrorStatus, UnknownSmartModule,
                                    Unsupported, ResidentSlice, StoreMemoryExceeded, builtin)
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    return SmartEngine(0)


def gpu_chain(engine, modules, limit=None):
    b = SmartModuleChainBuilder.default()
    if limit is not None:
        b.set_store_memory_limit(limit)
    for name, params, acc in modules:
        cb = SmartModuleConfig.builder().params(params or {})
        if acc is not None:
            cb.initial_data(SmartModuleInitialData.with_aggregate(acc))
        b.add_smart_module(cb.build(), builtin(name))
    return b.initialize(engine)


def orc_chain(modules):
    return O.OracleChain([(n, p or {}, a) for n, p, a in modules])


def mods(spec):
    return [(m[0], m[1], m[2].encode() if isinstance(m[2], str) else m[2]) for m in spec]


def assert_same_error(ge, oe):
    if oe is None:
        assert ge is None
        return
    assert ge is not None
    assert ge.hint == oe["hint"]
    assert ge.offset == oe["offset"]
    assert ge.kind == oe["kind"]
    assert ge.record_key == oe["key"]
    assert ge.record_value == oe["value"]


def check_batch(engine, modules, slice_bytes, max_bytes=(1 << 64) - 1, calls=1):
    g = gpu_chain(engine, modules)
    o = orc_chain(modules)
    for _ in range(calls):
        gm = SmartModuleChainMetrics()
        try:
            gout = g.process_batch(slice_bytes, max_bytes, gm)
            gerr = None
        except Exception as e:  # noqa: BLE001
            gout, gerr = None, e
        oout = o.process_batch(slice_bytes, max_bytes)
        if oout["status"] != 0:
            assert gerr is not None, f"oracle status {oout['status']}, gpu succeeded"
            assert getattr(gerr, "code", None) == oout["status"], (gerr, oout["status"])
            continue
        assert gerr is None, gerr
        assert gout.raw == oout["bytes"], "output batch bytes differ"
        assert gout.base_offset == oout["base_offset"]
        assert gout.last_offset_delta == oout["last_offset_delta"]
        assert gout.n_records == oout["n_records"]
        assert_same_error(gout.error, oout["error"])
        om = oout["metrics"]
        assert gm.bytes_in() == om["bytes_in"]
        assert gm.invocation_count() == om["invocation_count"]
        assert gm.records_out() == om["records_out"]
        assert gm.fuel_used() == 0
    for i, m in enumerate(modules):
        if m[0] in ("aggregate-sum", "aggregate", "aggregate-json"):
            assert g.accumulator(i) == o.accumulator(i)
    return gout


# ---------------------------------------------------------------------------
# reference known answers
# ---------------------------------------------------------------------------
def test_kat_chain_cases(engine, kats):
    for case in kats["chain"]:
        modules = mods(case["modules"])
        agg = next((i for i, m in enumerate(modules) if m[0].startswith("aggregate")), None)
        g = gpu_chain(engine, modules)
        for call in case["calls"]:
            inp = SmartModuleInput.try_from_records([P.Record.new(v) for v in call["values"]])
            out = g.process(inp)
            assert out.error is None
            assert [r.value for r in out.successes] == [v.encode() for v in call["expect"]], case["name"]
            if "acc" in call:  # transforms/aggregate.rs:157,185,207: the stored accumulator
                assert g.accumulator(agg) == call["acc"].encode(), case["name"]


def test_kat_init_errors(engine, kats):
    for c in kats["init_errors"]:
        with pytest.raises(SmartModuleInitError) as e:
            gpu_chain(engine, [(c["module"], c["params"], None)])
        assert str(e.value) == c["message"]


def test_kat_survey_guest(engine, kats):
    g = kats["survey_guest"]
    ch = gpu_chain(engine, [(g["module"], {}, None)])
    recs = [P.Record.new(v) for v in g["ok"]["values"]]
    for i, r in enumerate(recs):
        r.preamble.offset_delta = i
    out = ch.process(SmartModuleInput(P.encode_records(recs), g["ok"]["base_offset"], 0))
    assert out.raw_successes.hex() == g["ok"]["expect_successes"]
    assert out.error is None
    u = g["utf8"]
    recs = [P.Record.new(bytes.fromhex(v)) for v in u["values_hex"]]
    for i, r in enumerate(recs):
        r.preamble.offset_delta = i
    out = ch.process(SmartModuleInput(P.encode_records(recs), u["base_offset"], 0))
    assert [r.value for r in out.successes] == [v.encode() for v in u["expect_values"]]
    e = out.error
    assert (e.hint, e.offset, e.kind, e.record_key, e.record_value.hex()) == (
        u["error"]["hint"], u["error"]["offset"], u["error"]["kind"], None, u["error"]["value"])


def test_kat_process_batch(engine, kats):
    for case in kats["process_batch"]:
        modules = mods(case["modules"])
        out = check_batch(engine, modules, bytes.fromhex(case["slice"]), case["max_bytes"])
        exp = case["expect"]
        b = out.batch()
        recs = b.memory_records()
        assert b.base_offset == exp["base_offset"]
        assert [r.value for r in recs] == [v.encode() for v in exp["values"]], case["name"]
        if "next_offset" in exp:
            assert b.base_offset + b.header.last_offset_delta + 1 == exp["next_offset"]
        if "error" in exp:
            assert out.error.hint == exp["error"]["hint"]
            assert out.error.offset == exp["error"]["offset"]


def test_unknown_module(engine):
    b = SmartModuleChainBuilder.default()
    b.add_smart_module(SmartModuleConfig.builder().build(), b"\0asm\x01\0\0\0")
    with pytest.raises(UnknownSmartModule):
        b.initialize(engine)
    b = SmartModuleChainBuilder.default()
    b.add_smart_module(SmartModuleConfig.builder().build(), builtin("no-such-module"))
    with pytest.raises(UnknownSmartModule):
        b.initialize(engine)


# ---------------------------------------------------------------------------
# randomized parity over synthetic slices
# ---------------------------------------------------------------------------
CHAINS = {
    "filter": [("filter", {}, None)],
    "filter_init_timeout": [("filter_init", {"key": "timeout"}, None)],
    "filter_with_param": [("filter_with_param", {}, None)],
    "regex_ssn": [("regex-filter", {"regex": r"\d{3}-\d{2}-\d{4}"}, None)],
    "filter_regex": [("filter_regex", {}, None)],
    "regex_level": [("regex-filter", {"regex": r'^\{"level":"(warn|error)"'}, None)],
    "regex_unbounded": [("regex-filter", {"regex": r"a.*c\d+$"}, None)],
    "regex_unicode": [("regex-filter", {"regex": r"é|\d\d"}, None)],
    "regex_word_boundary": [("regex-filter", {"regex": r"\btimeout\b|\b\d{3}\b"}, None)],
    "regex_case_insensitive": [("regex-filter", {"regex": r"(?i)TIMEOUT|(?i:ssn)\s"}, None)],
    "regex_posix": [("regex-filter", {"regex": r"[[:digit:]]{3}-[[:digit:]]{2}|^[[:upper:]]"}, None)],
    "regex_unicode_word": [("regex-filter", {"regex": r"\w+é|\p{Lu}\p{Ll}+\d|\P{L}{4}$"}, None)],
    "regex_multiline": [("regex-filter", {"regex": r"(?m)^\d+$|x$|^\{\x22level"}, None)],
    "regex_verbose": [("regex-filter", {"regex": r"(?x) time out \s* \d  # the timeout records"}, None)],
    "regex_ascii_only": [("regex-filter", {"regex": r"(?-u)\w\d{2}\s"}, None)],
    "regex_script_fold": [("regex-filter", {"regex": r"(?i)\p{Greek}|É\p{Alphabetic}|\p{Emoji_Presentation}|TIME\p{Ll}"}, None)],
    "map_then_regex_ci": [("map", {}, None), ("regex-filter", {"regex": r"(?i)error"}, None)],
    "map": [("map", {}, None)],
    "filter_json": [("filter_json", {}, None)],
    "filter_json_then_map": [("filter_json", {}, None), ("map", {}, None)],
    "map_then_filter_json": [("map", {}, None), ("filter_json", {}, None)],
    "double_then_filter_json": [("map_double", {}, None), ("filter_json", {}, None)],
    "filter_json_then_filter": [("filter_json", {}, None), ("filter_init", {"key": "timeout"}, None)],
    "filter_then_filter_json": [("filter_init", {"key": "a"}, None), ("filter_json", {}, None)],
    "filter_then_map": [("filter_init", {"key": "timeout"}, None), ("map", {}, None)],
    "map_then_filter": [("map", {}, None), ("filter_init", {"key": "TIMEOUT"}, None)],
    "map_then_lower_filter": [("map", {}, None), ("filter_init", {"key": "timeout"}, None)],
    "filter_odd": [("filter_odd", {}, None)],
    "map_double": [("map_double", {}, None)],
    "filter_map": [("filter_map", {}, None)],
    "map_double_filter_map": [("map_double", {}, None), ("filter_map", {}, None)],
    "agg_sum": [("aggregate-sum", {}, b"7")],
    "filter_agg_sum": [("filter_with_param", {"key": "1"}, None), ("aggregate-sum", {}, None)],
    "array_map": [("array_map_json_array", {}, None)],
    "filter_array_map": [("filter_with_param", {"key": "1"}, None), ("array_map_json_array", {}, None)],
    "map_array_map": [("map", {}, None), ("array_map_json_array", {}, None)],
    "project": [("map_json_project", {}, None)],
    "filter_project_map": [("filter_init", {"key": "timeout"}, None), ("map_json_project", {}, None), ("map", {}, None)],
    "project_level_filter": [("map_json_project", {"field": "level"}, None), ("filter_init", {"key": "warn"}, None)],
    "map_project_upper": [("map", {}, None), ("map_json_project", {"field": "MESSAGE"}, None)],
    "empty": [],
}
# string-concatenating aggregate: output grows quadratically, small slices only
CONCAT_CHAINS = {
    "agg_concat": [("aggregate", {}, b"A")],
    "filter_agg_concat": [("filter", {}, None), ("aggregate", {}, None)],
    "map_agg_concat": [("map", {}, None), ("aggregate", {}, b"x")],
    "filter_map_agg_concat": [("filter_map", {}, None), ("aggregate", {}, b"")],
    "agg_concat_bad_acc": [("aggregate", {}, b"ok\xff")],
}


@pytest.mark.parametrize("kind,n", [(1, 3000), (2, 2000), (3, 5000), (4, 4000), (5, 3000)])
@pytest.mark.parametrize("chain", sorted(CHAINS))
def test_random_parity(engine, chain, kind, n):
    sl = synth.make_slice(kind, n, base_offset=1000)
    check_batch(engine, CHAINS[chain], sl)


# ---------------------------------------------------------------------------
# k_arr_lean (fsg_array.hip): array_map alone, lane per record; arrays outside
# its grammar (floats, nested values, escapes, leading zeros, -0, long ints,
# non-ASCII, errors) defer their batch to the exact kernel
# ---------------------------------------------------------------------------
def _array_slice(seed, nbatches=80, odd=0.1):
    import random
    rng = random.Random(seed)
    good = ["1", "-7", "0", "123456789012345678", "true", "false", "null", '"ab c"', '""', '"x,]"', "-42"]
    weird = ["1.5", "1e3", "01", "-0", "1234567890123456789012", "[1]", '{"a":1}', '"\\n"', '"\u00e9"', '"é"',
             "tru", "nul", "-", "+1"]
    out, base = b"", 0
    for bi in range(nbatches):
        b = P.Batch(base_offset=base)
        nrec = rng.choice([1, 3, 40, 64, 65, 130, 200])
        for _ in range(nrec):
            els = [rng.choice(good) for _ in range(rng.randint(0, 12))]
            if rng.random() < odd / nrec * 4:
                els.insert(rng.randint(0, len(els)), rng.choice(weird))
            sep = rng.choice([",", ", ", " ,", "\n,\t"])
            v = rng.choice(["", " ", "\n"]) + "[" + rng.choice(["", " "]) + sep.join(els) + rng.choice(["", " "]) + "]"
            if odd and rng.random() < 0.003:
                v = rng.choice(["", "[1,2", "x", "[1,]", "[,]"])
            key = None if rng.random() < 0.7 else b"k"
            r = P.Record.new_key_value(key, v.encode())
            if rng.random() < 0.1:
                r.headers = 2
            b.add_record(r)
        enc = b.encode()
        if len(enc) - 57 > 16000:
            continue
        out += enc
        base += nrec + rng.randint(0, 5)
    return out


@pytest.mark.parametrize("seed,odd", [(1, 0.0), (2, 0.1), (3, 0.5)])
def test_array_lean_parity(engine, seed, odd):
    sl = _array_slice(seed, odd=odd)
    check_batch(engine, CHAINS["array_map"], sl)
    check_batch(engine, CHAINS["array_map"], sl, max_bytes=20000)
    g = gpu_chain(engine, CHAINS["array_map"])
    if orc_chain(CHAINS["array_map"]).process_batch(sl)["status"] == 0:
        g.process_batch(sl)
        t = g.last_timings()
        assert t["eval_path"] == 3, t  # FSG_EVAL_ARRAY
        if odd == 0.0:
            assert t["deferred"] < t["n_batches"] // 10, t
    # the C4 synthetic arrays: every batch on the lean path
    sl2 = synth.make_slice(5, 20000, base_offset=3)
    check_batch(engine, CHAINS["array_map"], sl2)
    g.process_batch(sl2)
    assert g.last_timings()["deferred"] == 0


def test_array_lean_rebase_and_varint_edges(engine):
    """k_arr_lean / k_arr_write edges: offset rebases of 1..5 varint bytes,
    element varint + text lengths around the inner-length threshold (L = 50 .. 60
    against 60 - vsize(rel)), texts of 64+ bytes (two-byte length varints),
    batches of more than 256 records (the writer's record chunks) and outputs
    spanning several 16 KiB staging rounds."""
    rng = random.Random(7)
    sl, base = b"", 0
    jumps = [0, 70, 20000, 3_000_000, 2**31]
    for k in range(15):
        b = P.Batch(base_offset=base)
        kind = k % 3
        nrec = (40, 900, 3)[kind]
        for j in range(nrec):
            if kind == 1:
                v = "[%d]" % j if j % 7 else "[]"
            else:
                els = ['"' + "s" * rng.randrange(44, 70) + '"' for _ in range(rng.randint(1, 4))]
                els.append(str(rng.randint(-99, 99)))
                rng.shuffle(els)
                v = "[" + ",".join(els) + "]"
            b.add_record(P.Record.new(v.encode()))
        sl += b.encode()
        base += nrec + jumps[k % 5]
    check_batch(engine, CHAINS["array_map"], sl)
    check_batch(engine, CHAINS["array_map"], sl, max_bytes=50000)
    g = gpu_chain(engine, CHAINS["array_map"])
    g.process_batch(sl)
    t = g.last_timings()
    assert t["eval_path"] == 3 and t["deferred"] == 0, t


# ---------------------------------------------------------------------------
# composed chains: stages after an array_map, an aggregate or a stateful
# filter (engine.rs:147-167 feeds each stage's successes to the next); the
# GPU runs them as segments (fsg_runtime.cpp run_composed)
# ---------------------------------------------------------------------------
COMPOSED = {
    "array_map_filter": [("array_map_json_array", {}, None), ("filter_init", {"key": "a"}, None)],
    "array_map_map": [("array_map_json_array", {}, None), ("map", {}, None)],
    "array_map_filter_odd": [("array_map_json_array", {}, None), ("filter_odd", {}, None)],
    "array_map_filter_map_double": [("array_map_json_array", {}, None), ("filter_map", {}, None),
                                    ("map_double", {}, None)],
    "filter_array_map_regex": [("filter_with_param", {"key": "1"}, None), ("array_map_json_array", {}, None),
                               ("regex-filter", {"regex": r"^-?\d{2}$|[xyz]"}, None)],
    "array_map_twice": [("array_map_json_array", {}, None), ("array_map_json_array", {}, None)],
    "agg_sum_filter_odd": [("aggregate-sum", {}, b"7"), ("filter_odd", {}, None)],
    "agg_sum_filter": [("aggregate-sum", {}, None), ("filter_init", {"key": "5"}, None), ("map", {}, None)],
    "agg_sum_agg_sum": [("aggregate-sum", {}, None), ("aggregate-sum", {}, b"3")],
    "hashset_map": [("filter_hashset", {}, None), ("map", {}, None)],
    "hashset_filter_odd": [("filter_hashset", {"count": "50"}, None), ("filter_odd", {}, None)],
    "look_back_filter_map": [("filter_look_back", {}, None), ("filter_map", {}, None)],
    "aggj_filter": [("aggregate-json", {}, None), ("filter_init", {"key": "repo-0001"}, None)],
    "map_agg_concat_filter": [("map", {}, None), ("aggregate", {}, b"x"), ("filter_init", {"key": "X"}, None)],
}


@pytest.mark.parametrize("kind,n", [(1, 800), (2, 600), (3, 2500), (4, 2500), (5, 1500)])
@pytest.mark.parametrize("chain", sorted(COMPOSED))
def test_composed_chain_parity(engine, chain, kind, n):
    if chain == "map_agg_concat_filter":
        n = min(n, 300)  # the concat output grows quadratically
    sl = synth.make_slice(kind, n, base_offset=500)
    check_batch(engine, COMPOSED[chain], sl, calls=2)


@pytest.mark.parametrize("max_bytes", [0, 100, 5000, 60000])
@pytest.mark.parametrize("chain", ["array_map_filter_odd", "agg_sum_filter_odd", "hashset_map"])
def test_composed_chain_max_bytes(engine, chain, max_bytes):
    sl = synth.make_slice(5 if chain.startswith("array") else 3, 2000, base_offset=9)
    check_batch(engine, COMPOSED[chain], sl, max_bytes, calls=2)


def test_composed_chain_keyed_errors(engine):
    """aggregate-json then a filter over keyed records with bad values (the
    aggregate's error batch passes through the filter), then process()."""
    for seed in (1, 3):
        check_batch(engine, COMPOSED["aggj_filter"], _keyed_slice(seed, bad=0.02), calls=2)
    modules = COMPOSED["array_map_filter_odd"]
    g, o = gpu_chain(engine, modules), orc_chain(modules)
    for b in P.decode_batches(synth.make_slice(5, 400)):
        gout = g.process(SmartModuleInput(b.records_bytes, b.base_offset, b.header.first_timestamp))
        oout = o.process(b.records_bytes, b.base_offset, b.header.first_timestamp)
        assert oout["status"] == 0
        assert gout.raw_successes == oout["bytes"]
        assert_same_error(gout.error, oout["error"])


@pytest.mark.parametrize("max_bytes", [0, 1, 100, 5000, 40000, 300000])
@pytest.mark.parametrize("chain", ["filter_init_timeout", "filter_then_map", "filter_map", "agg_sum"])
def test_max_bytes_cut(engine, chain, max_bytes):
    kind = 3 if chain in ("filter_map", "agg_sum") else 2
    sl = synth.make_slice(kind, 1500, base_offset=77)
    check_batch(engine, CHAINS[chain], sl, max_bytes)


def test_aggregate_state_across_calls(engine):
    sl = synth.make_slice(3, 3000)
    check_batch(engine, CHAINS["agg_sum"], sl, calls=3)
    check_batch(engine, [("aggregate-sum", {}, b"\xff\xfe")], sl)  # invalid UTF-8 accumulator
    check_batch(engine, [("aggregate-sum", {}, b" 2147483647\n")], sl)  # wrapping sum


def test_process_parity(engine):
    """SmartModuleChainInstance::process on single inputs (per-batch API)."""
    for chain in ("filter_init_timeout", "regex_ssn", "filter_odd", "filter_then_map", "filter_map", "empty"):
        modules = CHAINS[chain]
        g, o = gpu_chain(engine, modules), orc_chain(modules)
        for kind in (1, 2, 4):
            sl = synth.make_slice(kind, 300)
            for b in P.decode_batches(sl):
                gm = SmartModuleChainMetrics()
                gout = g.process(SmartModuleInput(b.records_bytes, b.base_offset, b.header.first_timestamp), gm)
                oout = o.process(b.records_bytes, b.base_offset, b.header.first_timestamp)
                assert oout["status"] == 0
                assert gout.raw_successes == oout["bytes"], chain
                assert_same_error(gout.error, oout["error"])
                assert gm.bytes_in() == oout["metrics"]["bytes_in"]
                assert gm.records_out() == oout["metrics"]["records_out"]


def test_ingest_slice_reused_across_calls(engine):
    """process_batch / process stage their input in the chain's own ingest slice
    (kept at the largest size seen): shrinking, growing, compressed, empty and
    one-record inputs through ONE chain each match the oracle."""
    from tests.compressed_slices import recompress
    modules = CHAINS["filter_init_timeout"]
    g, o = gpu_chain(engine, modules), orc_chain(modules)
    big = synth.make_slice(2, 3000, base_offset=5)
    small = synth.make_slice(2, 7, base_offset=90)
    comp = recompress(synth.make_slice(2, 400, base_offset=3), [1, 2, 3, 0])
    one = next(iter(P.decode_batches(synth.make_slice(2, 40))))
    for step in ("big", "small", "one", "comp", "empty", "one", "big", "small", "comp", "one"):
        if step == "one":
            gout = g.process(SmartModuleInput(one.records_bytes, one.base_offset, one.header.first_timestamp))
            oout = o.process(one.records_bytes, one.base_offset, one.header.first_timestamp)
            assert oout["status"] == 0
            assert gout.raw_successes == oout["bytes"], step
            assert_same_error(gout.error, oout["error"])
            continue
        sl = {"big": big, "small": small, "comp": comp, "empty": b""}[step]
        gout = g.process_batch(sl)
        oout = o.process_batch(sl)
        assert oout["status"] == 0, step
        assert gout.raw == oout["bytes"], step
        assert gout.n_records == oout["n_records"], step
        assert_same_error(gout.error, oout["error"])


def test_staged_download_large_output(engine):
    """Outputs of 128 MiB and more come back through two pinned 32 MiB chunks
    (DMA of one overlapping the host copy of the other): byte-exact with the
    oracle over a ~150 MB decode-and-return batch (chunk count not a multiple of 2,
    last chunk partial)."""
    sl = synth.make_slice(2, 150_000, base_offset=77)
    g, o = gpu_chain(engine, []), orc_chain([])
    gout = g.process_batch(sl)
    oout = o.process_batch(sl)
    assert oout["status"] == 0
    assert len(oout["bytes"]) >= 128 << 20
    assert gout.raw == oout["bytes"]
    del gout, oout


def test_large_records_beyond_window(engine):
    """Records larger than the 17 KB LDS window take the global-memory path."""
    batches = b""
    base = 0
    for size in (100, 20000, 17380, 17400, 70000, 5):
        b = P.Batch(base_offset=base, header=P.BatchHeader(producer_id=0))
        for j in range(3):
            v = (b"x" * (size - 9)) + (b"timeout" if j != 1 else b"nothing") + b"\xc3\xa9"
            b.add_record(P.Record.new(v))
        batches += b.encode()
        base += 3
    for chain in ("filter_init_timeout", "map", "regex_unbounded", "filter_then_map"):
        check_batch(engine, CHAINS[chain], batches)


def test_edge_slices(engine):
    chain = CHAINS["filter_init_timeout"]
    good = synth.make_slice(2, 100)
    # empty slice
    check_batch(engine, chain, b"")
    # batch with zero records, negative count
    e = P.Batch(base_offset=5).encode()
    check_batch(engine, chain, e + good)
    neg = bytearray(e)
    neg[57:61] = struct.pack(">i", -3)
    check_batch(engine, chain, bytes(neg))
    # truncated slice -> io error after processing the good batches
    check_batch(engine, chain, good + good[:100])
    # gzip bits on a section that is not gzip -> the iterator's io::Error, like the oracle
    comp = bytearray(good)
    comp[22] |= 1
    check_batch(engine, chain, bytes(comp))
    # zstd bits on a section that is not zstd -> io::Error, like the oracle
    comp[22] = (comp[22] & ~7) | 4
    check_batch(engine, chain, bytes(comp))
    # a record whose length claims more than the section -> decoding error (-11)
    bad = bytearray(good)
    bad[61] = 0x7E
    check_batch(engine, chain, bytes(bad))
    # count larger than the records present -> decoding error
    more = bytearray(e)
    more[57:61] = struct.pack(">i", 2)
    check_batch(engine, chain, bytes(more))
    # empty chain on a malformed section -> io error
    check_batch(engine, [], bytes(more))


def _frame_walk(sl):
    """FileBatchIterator::next (crates/fluvio-storage/src/iterators.rs:55-160) as
    a plain walk: (batches, records, header bytes, tail) — tail 'io' / 'unsup'."""
    pos, nb, nrec, hb, tail = 0, 0, 0, 0, None
    while pos < len(sl):
        if len(sl) - pos < 57:
            tail = "io"
            break
        blen, = struct.unpack_from(">i", sl, pos + 8)
        attrs, = struct.unpack_from(">h", sl, pos + 21)
        if blen < 45 or len(sl) - pos - 57 < blen - 45:
            tail = "io"
            break
        if attrs & 7:  # (these test sections are not really compressed: decoding fails -> io)
            tail = "unsup" if (attrs & 7) == 4 else "io"
            break
        rem = blen - 45
        if rem >= 4:
            c, = struct.unpack_from(">i", sl, pos + 57)
            nrec += min(max(c, 0), (rem - 4) // 7)
        nb += 1
        hb += 57 + rem
        pos += 57 + rem
    return nb, nrec, hb, tail


def test_device_framing(engine):
    """The slice framed on the device (magic-2 candidates, pointer doubling from
    position 0) equals the host walk; a batch without magic 2 on the chain
    sends the slice to the host walk, with the same framing."""
    import random
    rng = random.Random(7)
    good = synth.make_slice(2, 3000)
    small = synth.make_slice(1, 2000)
    nomagic = bytearray(good)
    nomagic[16] = 1  # the first batch's magic byte
    cases = [(good, True), (small, True), (good + small, True), (good + good[:40], True),
             (good + good[:300], True), (P.Batch(base_offset=5).encode() + good, True), (bytes(nomagic), False)]
    comp = bytearray(good)
    # a compressed batch in the middle: the walk stops there (unsupported)
    pos, k = 0, 0
    while k < 20:
        blen, = struct.unpack_from(">i", good, pos + 8)
        pos += 12 + blen
        k += 1
    comp[pos + 22] |= 2
    cases.append((bytes(comp), False))  # a compressed batch: host walk + GPU decompression (fails: io)
    # random bytes with magic-2 noise between batches are never on the chain
    noisy = bytearray(good)
    for _ in range(2000):
        i = rng.randrange(len(noisy))
        if noisy[i] == 0x20:
            noisy[i] = 2
    cases.append((bytes(noisy), True))
    for sl, dev in cases:
        rs = ResidentSlice(engine, sl)
        nb, nrec, hb, tail = _frame_walk(sl)
        assert (rs.n_batches, rs.n_records, rs.bytes) == (nb, nrec, hb)
        assert rs.device_framed == dev
    for sl, _ in cases:
        if _frame_walk(sl)[3] == "unsup":
            with pytest.raises(Unsupported):
                gpu_chain(engine, CHAINS["filter_init_timeout"]).process_batch(sl)
        else:
            check_batch(engine, CHAINS["filter_init_timeout"], sl)


def test_unicode_word_boundaries(engine):
    """\\b / \\B on non-ASCII values: Unicode word boundaries between code points
    (the marked full DFA, a marker with each code point's \\w class before its
    bytes), like the oracle's Pike VM; a (?-u) \\b stays outside the GPU subset:
    FSG_E_UNSUPPORTED when (and only when) such a record is reached in stream order."""
    check_batch(engine, [("regex-filter", {"regex": r"\w+"}, None)], _one_record_slice("caf\u00e9".encode()))
    b = P.Batch()
    for v in ("abc", "caf\u00e9", "xyz", "x\u00e9", "\u00e9x", "\u03c9 x", "\u263a\u263ax", "na\u0301x"):
        b.add_record(P.Record.new(v))
    for pat in (r"\bx", r"x\b", r"\Bx", r"\b\w+\b", r"(?i)\bCAF\u00c9\b", r"\b\u03c9\b"):
        chain = [("regex-filter", {"regex": pat}, None)]
        check_batch(engine, chain, synth.make_slice(4, 500))
        check_batch(engine, chain, b.encode())
    for pat in (r"\p{IsGreek}", r"\p{sc=IsGreek}\s", r"\p{Is_L}{3}",  # symbolic_name_normalize's "is" prefix
                r"\p{GCB=Extend}", r"\p{WB=ALetter}{2}\p{SB=Lower}"):  # break property values
        check_batch(engine, [("regex-filter", {"regex": pat}, None)], b.encode())
    chain = [("regex-filter", {"regex": r"(?-u:\b)x"}, None)]
    with pytest.raises(Unsupported):
        gpu_chain(engine, chain).process_batch(b.encode())
    check_batch(engine, chain, b.encode())


def test_version_uncertain_code_points(engine):
    """regex-filter emulates regex-syntax 0.6.27 (Unicode 14) and filter_regex
    0.7.1 (Unicode 15); this build's tables are Unicode 13 (unicodedata) and
    the regex module's newer UCD.  A table-dependent pattern (\\d \\w \\p,
    (?i), Unicode \\b) meeting a code point whose class differs between them
    (U+1FAE8, assigned in 15; U+0295, Ll -> Lo in 14) is FSG_E_UNSUPPORTED on
    the GPU and in the oracle; literal / '.' patterns decide it."""
    b = P.Batch()
    for v in ("abc", "café", "x \U0001FAE8 y", "zz ʕ"):
        b.add_record(P.Record.new(v))
    for pat in (r"\w+é", r"\d", r"(?i)ZZ", r"\p{Ll}", r"\bq"):
        chain = [("regex-filter", {"regex": pat}, None)]
        with pytest.raises(Unsupported):
            gpu_chain(engine, chain).process_batch(b.encode())
        check_batch(engine, chain, b.encode())
    for pat in (r"zz", r"é", r"x . y", r"[^a]"):
        check_batch(engine, [("regex-filter", {"regex": pat}, None)], b.encode())
    # a \p name regex-syntax rejects (a Unicode 16 script): the regex crate's error Display
    with pytest.raises(SmartModuleInitError) as e:
        gpu_chain(engine, [("regex-filter", {"regex": r"a\p{Garay}"}, None)])
    assert str(e.value) == ("regex parse error:\n    a\\p{Garay}\n     ^^^^^^^^^\nerror: Unicode property not found"
                            "\n\nSmartModule Init Error: \n")


def test_unsupported_mid_stream_leaves_state(engine):
    """FSG_E_UNSUPPORTED in batch 1 of 3 (a (?-u) \\b on a non-ASCII value):
    the caller falls back and replays the input, so the aggregate accumulator
    and the dedup set must not move past batch 0 (the advisor's round-5 case)."""
    rx = ("regex-filter", {"regex": r"(?-u:\b)\d"}, None)
    sl = b""
    for base, vals in ((0, ["5", "7"]), (10, ["8", "\u00e95"]), (20, ["9"])):
        b = P.Batch(base_offset=base)
        for v in vals:
            b.add_record(P.Record.new(v.encode()))
        sl += b.encode()
    b0 = P.Batch(base_offset=0)
    for v in ("5", "7"):
        b0.add_record(P.Record.new(v.encode()))
    first = b0.encode()
    assert sl.startswith(first)
    g = gpu_chain(engine, [rx, ("aggregate-sum", {}, b"100")])
    with pytest.raises(Unsupported):
        g.process_batch(sl)
    assert g.accumulator(1) == b"100"
    o = orc_chain([rx, ("aggregate-sum", {}, b"100")])
    assert g.process_batch(first).raw == o.process_batch(first)["bytes"]
    assert g.accumulator(1) == o.accumulator(1) == b"112"
    h = gpu_chain(engine, [rx, ("filter_hashset", {}, None)])
    with pytest.raises(Unsupported):
        h.process_batch(sl)
    oh = orc_chain([rx, ("filter_hashset", {}, None)])
    r = h.process_batch(first)
    assert r.raw == oh.process_batch(first)["bytes"] and r.n_records == 2


def test_resident_slice_matches_process_batch(engine):
    sl = synth.make_slice(2, 4000)
    ch = gpu_chain(engine, CHAINS["filter_then_map"])
    rs = ResidentSlice(engine, sl)
    a = ch.process_slice(rs)
    b = ch.process_batch(sl)
    assert a.raw == b.raw
    o = orc_chain(CHAINS["filter_then_map"]).process_batch(sl)
    assert a.raw == o["bytes"]
    t = ch.last_timings()
    assert t["eval_ms"] > 0 and t["out_bytes"] == len(a.raw)


def test_large_output_crc(engine):
    """An output batch above 512 MiB: the CRC combine shifts by more than 2^32
    bits (x^(2^32) != x mod the Castagnoli polynomial, so no exponent wrap is
    allowed).  Checked byte-for-byte against the oracle and by recomputing the
    CRC32C of the returned batch."""
    sl = synth.make_slice_array(2, 640_000)  # ~650 MB in, all records kept by `map`
    rs = ResidentSlice(engine, sl)
    ch = gpu_chain(engine, CHAINS["map"])
    out = ch.process_slice(rs).raw
    assert len(out) > (512 << 20)
    assert struct.unpack(">I", out[17:21])[0] == O.crc32c(out[21:])
    o = orc_chain(CHAINS["map"]).process_batch(sl.tobytes())
    assert out == o["bytes"]


# ---------------------------------------------------------------------------
# JSON-field filter (examples/filter_json): serde_json semantics incl. error hints
# ---------------------------------------------------------------------------
def _one_record_slice(value: bytes, base: int = 0) -> bytes:
    b = P.Batch(base_offset=base)
    b.add_record(P.Record.new(value))
    return b.encode()


def test_filter_json_string_debug_texts(engine):
    """serde's "invalid type: string .." with Rust's str Debug of any string
    (control / format / separator / private-use / unassigned chars and
    combining marks as \\u{..}): error hint bit-exact with the oracle, as one
    record and as the first error in a batch."""
    import json as _json
    from tests.test_json_oracle import DEBUG_STRINGS
    for s in DEBUG_STRINGS:
        for ascii_only in (True, False):
            doc = _json.dumps(s, ensure_ascii=ascii_only).encode()
            check_batch(engine, CHAINS["filter_json"], _one_record_slice(doc))
    # a NUL inside the error text (unknown variant of the raw string) crosses with hint_len
    check_batch(engine, CHAINS["filter_json"], _one_record_slice(b'{"level":"in\\u0000fo","message":"m"}'))
    b = P.Batch()
    for v in (b'{"level":"info","message":"a"}', b'{"level":"warn","message":"b"}',
              _json.dumps("x\u200d\u0301\x1b y").encode(), b'{"level":"info","message":"c"}'):
        b.add_record(P.Record.new(v))
    check_batch(engine, CHAINS["filter_json"], b.encode())


def test_filter_json_fuzz_one_record(engine):
    """Every document of the corpus (valid, mutated, hand-picked error cases) as a
    one-record batch: output, error hint text, offset and value bit-exact."""
    from tests import jsongen
    for doc in jsongen.corpus(7, 150, 450):
        check_batch(engine, CHAINS["filter_json"], _one_record_slice(doc))


def test_filter_json_first_error_in_stream(engine):
    from tests import jsongen
    import random
    rng = random.Random(11)
    good = [jsongen.valid_doc(rng).encode() for _ in range(400)]
    bad = [b'{"level":"info","message":5}', b'{"level":"nope","message":"m"}', b"[1,2",
           b'{"level":"warn","message":"x"} trailing']
    sl = b""
    base = 0
    for k in range(40):
        b = P.Batch(base_offset=base)
        for j in range(10):
            v = good[k * 10 + j]
            if k == 23 and j == 6:
                v = bad[k % len(bad)]
            b.add_record(P.Record.new(v))
        sl += b.encode()
        base += 10
    for chain in ("filter_json", "filter_json_then_map", "map_then_filter_json", "filter_json_then_filter",
                  "filter_then_filter_json"):
        check_batch(engine, CHAINS[chain], sl)
        check_batch(engine, CHAINS[chain], sl, max_bytes=20000)


def test_filter_json_lean_batches(engine):
    """Batches of 1..64 records mixing documents the fast path decides, ones only
    the exact restatement decides (escapes, nesting, whitespace, non-ASCII,
    enum maps) and ones that fail: every batch bit-exact with the oracle."""
    from tests import jsongen
    import random
    rng = random.Random(3)
    docs = jsongen.corpus(13, 300, 120)
    simple = [b'{"level":"%s","message":"m %d","n":-1.5e3,"t":true,"z":null,"s":"x"}' % (
        rng.choice(jsongen.LEVELS).encode(), i) for i in range(200)]
    sl, base = b"", 0
    for k in range(60):
        b = P.Batch(base_offset=base)
        n = rng.choice([1, 7, 15, 40, 64])
        for j in range(n):
            pool = simple if k % 3 else docs
            b.add_record(P.Record.new(rng.choice(pool)))
        sl += b.encode()
        base += n
    for chain in ("filter_json", "filter_json_then_filter", "filter_then_filter_json"):
        check_batch(engine, CHAINS[chain], sl)


def test_project_lean_batches(engine):
    """Field projection on the lean path (flat objects, fsg_kernels.hip
    lean_json_stage): batches of 1..64 records mixing documents it decides
    (string / integer / literal values, duplicate keys: last wins, missing
    field: dropped) with ones only the exact restatement decides (floats,
    -0, escapes, nesting) and ones that fail; every batch bit-exact with the
    oracle or reported unsupported for a document the device defers to it."""
    from tests import jsongen
    import random
    rng = random.Random(9)
    docs = [d for d in jsongen.corpus(19, 300, 120) if not _project_may_be_unsupported(d)]
    simple = []
    for i in range(300):
        k = rng.random()
        if k < 0.2:
            simple.append(b'{"level":"info","message":"m %d","n":%d,"t":true}' % (i, rng.randint(-10**12, 10**12)))
        elif k < 0.4:
            simple.append(b'{"message":%d,"x":null,"message":"last %d"}' % (i, i))  # duplicate: last wins
        elif k < 0.6:
            simple.append(b'{"a":"b","c":false}')                                   # no field: dropped
        elif k < 0.8:
            simple.append(b'{ "message" : -%d , "level" : "warn" }' % (i + 1))     # whitespace, integer
        else:
            simple.append(b'{"message":"%s"}' % (b"x" * rng.randint(0, 300)))
    sl, base = b"", 0
    for k in range(60):
        b = P.Batch(base_offset=base)
        n = rng.choice([1, 7, 15, 40, 64])
        for j in range(n):
            pool = simple if k % 3 else docs
            b.add_record(P.Record.new(rng.choice(pool)))
        sl += b.encode()
        base += n
    for chain in ("project", "filter_project_map", "project_level_filter"):
        check_batch(engine, CHAINS[chain], sl)


def test_project_synthetic_logs(engine):
    """C3 on the bench's C2 documents: filter -> projection of `message` ->
    uppercase, and projections of other fields, batch by batch."""
    sl = synth.make_slice(2, 3000)
    out = check_batch(engine, CHAINS["filter_project_map"], sl)
    assert 0 < out.n_records < 3000
    for f in ("level", "ts", "nope"):
        check_batch(engine, [("map_json_project", {"field": f}, None)], sl)


def test_filter_json_synthetic_logs(engine):
    """C2 records are StructuredLog documents: keep level > debug."""
    sl = synth.make_slice(2, 3000)
    out = check_batch(engine, CHAINS["filter_json"], sl)
    assert 0 < out.n_records < 3000


FJ_CHAINS = [
    [("filter_json", {}, None)],
    [("filter_json", {}, None), ("map", {}, None)],
    [("filter_init", {"key": "timeout"}, None), ("filter_json", {}, None)],
    [("filter_json", {}, None), ("filter_init", {"key": "tim"}, None)],  # short needle: lean kernel, not flat
    [("filter_init", {"key": "timeout"}, None), ("map_json_project", {"field": "message"}, None), ("map", {}, None)],
    [("map_json_project", {}, None)],
    [("map_json_project", {"field": "ts"}, None)],
    [("filter_init", {"key": "warn"}, None), ("map_json_project", {"field": "level"}, None)],
    [("filter_json", {}, None), ("map_json_project", {"field": "host"}, None)],
]


def _fj_docs(rng):
    """Values for the flat JSON path: ones it decides (flat objects, ' ' only,
    every value kind, strings across 16-byte chunks and 1 KiB rounds) beside
    ones it must hand to k_eval (escapes, tabs, nesting, floats under a
    projection, duplicates, missing fields, bad variants, trailing bytes,
    non-ASCII, unterminated strings)."""
    lv = ["debug", "info", "warn", "error"]
    good, odd = [], []
    for i in range(400):
        msg = "".join(rng.choice("abcdefgh ij") for _ in range(rng.choice([0, 1, 5, 14, 15, 16, 17, 31, 63, 200,
                                                                              1000, 1100, 2500])))
        if rng.random() < 0.4:
            msg = msg[: len(msg) // 2] + "timeout" + msg[len(msg) // 2:]
        sp = " " * rng.choice([0, 0, 0, 1, 3])
        extra = rng.choice(['"ts":%d' % rng.randrange(10**9), '"ok":true', '"no":false', '"z":null',
                            '"n":-%d' % rng.randrange(1, 10**6), '"s":"svc-%02d"' % rng.randrange(100), '"e":""'])
        members = ['"level"%s:%s"%s"' % (sp, sp, rng.choice(lv)), '"message":%s"%s"' % (sp, msg), extra,
                   '"host":"h-%04d"' % rng.randrange(10**4)]
        rng.shuffle(members)
        pre = " " * rng.randrange(0, 18)
        good.append((pre + "{" + sp + ("," + sp).join(members) + sp + "}" + sp).encode())
    odd += [b'{"level":"info","message":"a\\nb"}', b'{"level":"info","message":"a\tb"}',
            b'{"level":"info","message":"x","n":1.5}', b'{"level":"info","message":"x","n":2e3}',
            b'{"level":"info","message":"x","n":-0}', b'{"level":"info","message":"x","n":01}',
            b'{"level":"info","message":"x","o":{"a":1}}', b'{"level":"info","message":"x","a":[1,2]}',
            b'{"level":"info","level":"warn","message":"x"}', b'{"message":"x"}', b'{"level":"info"}',
            b'{"level":"INFO","message":"x"}', b'{"level":1,"message":"x"}', b'{"level":"info","message":5}',
            b'{"level":"info","message":"x"} x', b'{"level":"info","message":"x"}}', b'{}', b'',
            b'["info","x"]', b'{"level":"info","message":"caf\xc3\xa9"}', b'{"level":"info","message":"x',
            b'{"level":"info","message":"x","t":tru}', b'{"level":"info","message":"x","t":truex}',
            b'{"level":"info","message":"x","n":12345678901234567890}', b'{"level":"info","message":"x",}',
            b'{"level":"info" "message":"x"}', b'{"level":"info","message":"x"\n}', b'{"\xff":1}',
            b'{"level":"info","message":"x","n":-}', b'{"level":"info","message":"x","n":1.}',
            b'{"level":"info","message":"x","n":1e}', b'{"message":"timeout","message":"again"}']
    return good, odd


@pytest.mark.parametrize("ci", range(len(FJ_CHAINS)))
def test_fjson_path_parity(engine, ci):
    """The flat JSON path (FSG_EVAL_FJSON: k_flat_scan's JSON-interesting
    chunks + k_fj_decide) against the oracle: clean batches it decides alone,
    batches with one odd document (deferred whole to k_eval), strings that end
    at every offset of a 16-byte chunk and messages longer than the two
    preloaded bitmap rounds."""
    import random
    rng = random.Random(77 + ci)
    good, odd = _fj_docs(rng)
    sl, base = b"", 0
    for k in range(90):
        b = P.Batch(base_offset=base)
        n = rng.choice([1, 2, 9, 16, 33, 64])
        for j in range(n):
            doc = rng.choice(odd) if (k % 5 == 4 and j == n // 2) else rng.choice(good)
            b.add_record(P.Record.new_key_value(b"k%d" % j if j % 3 == 0 else None, doc))
        sl += b.encode()
        base += n
    chain = FJ_CHAINS[ci]
    check_batch(engine, chain, sl)
    g = gpu_chain(engine, chain)
    g.process_batch(sl)
    t = g.last_timings()
    short = any(m[0] == "filter_init" and len(m[1]["key"]) < 4 for m in chain)
    assert t["eval_path"] == (1 if short else 6), t
    if not short:
        assert 0 < t["deferred"] < t["n_batches"], t


def test_fjson_string_ends_every_offset(engine):
    """Strings ending at each byte of a chunk, keys and values straddling
    chunk and 1 KiB round edges, values starting at every alignment."""
    sl, base = b"", 0
    for shift in range(0, 48):
        b = P.Batch(base_offset=base)
        for i in range(20):
            msg = "m" * (i * 7 + shift)
            doc = ('{"level":"%s","message":"%s","n":%d}' % (["debug", "info"][i % 2], msg, i)).encode()
            b.add_record(P.Record.new(b" " * (shift % 5) + doc))
        sl += b.encode()
        base += 20
    for chain in ([("filter_json", {}, None)], [("map_json_project", {}, None), ("map", {}, None)]):
        check_batch(engine, chain, sl)
        g = gpu_chain(engine, chain)
        g.process_batch(sl)
        t = g.last_timings()
        assert t["eval_path"] == 6 and t["deferred"] == 0, t


# ---------------------------------------------------------------------------
# k_eval_lean (one wave per batch) vs the exact path: every needle-length mode,
# upper-cased scans, keys, empty values, needles at value edges or spanning
# into the next record, non-ASCII values and > 64 records (both deferred to the
# exact kernel), mixed in one slice
# ---------------------------------------------------------------------------
def _lean_slice(seed=7, nbatches=40):
    import random
    rnd = random.Random(seed)
    words = ["timeout", "time", "out", "info", "warn", "level", "a", "TIMEOUT", "tim", "eout", "xx", "é", "\xff"]
    out = b""
    base = 0
    for bi in range(nbatches):
        b = P.Batch(base_offset=base)
        nrec = rnd.choice([1, 3, 15, 63, 64, 65]) if bi % 3 else rnd.randint(1, 20)
        size = rnd.choice([0, 5, 40, 200, 900])
        for _ in range(nrec):
            parts = []
            while sum(len(p) for p in parts) < size:
                pool = words if bi >= nbatches - 2 else (words[:12] if bi % 5 == 0 else words[:11])
                w = rnd.choice(pool)
                parts.append(w)
            v = "".join(parts)[: size or None] if rnd.random() < 0.5 else " ".join(parts)
            enc = v.encode("utf-8") if "\xff" not in v else v.replace("\xff", "").encode() + b"\xff"
            key = None if rnd.random() < 0.7 else rnd.choice([b"", b"timeout", b"k\x80y"])
            r = P.Record.new_key_value(key, enc)
            b.add_record(r)
        enc_b = b.encode()
        if len(enc_b) - 57 > 16384:
            continue
        out += enc_b
        base += nrec + rnd.randint(0, 3)
    return out


@pytest.mark.parametrize("chain", [
    [("filter_init", {"key": "timeout"}, None)],          # m >= 7: aligned 4-gram rotations
    [("filter_init", {"key": "level"}, None)],            # 4 <= m <= 6
    [("filter_init", {"key": "ti"}, None)],               # m < 4
    [("filter", {}, None)],                               # 'a'
    [("filter_init", {"key": ""}, None)],                 # empty needle: UTF-8 check only
    [("map", {}, None), ("filter_init", {"key": "TIMEOUT"}, None)],
    [("map", {}, None), ("filter_init", {"key": "LEVEL"}, None)],
    [("filter_init", {"key": "out"}, None), ("map", {}, None), ("filter_init", {"key": "TIME"}, None)],
    [("map", {}, None)],
    [],
    [("regex-filter", {"regex": r"ti.e"}, None)],                        # lean regex: <= 16-state DFA
    [("regex-filter", {"regex": r"^(time|level)"}, None)],
    [("regex-filter", {"regex": r"out$|^a"}, None)],
    [("regex-filter", {"regex": r"^$"}, None)],                           # empty values only
    [("regex-filter", {"regex": r"(a|b)?"}, None)],                       # matches the empty string
    [("filter_regex", {}, None)],
    [("map", {}, None), ("regex-filter", {"regex": r"TI[M]E"}, None)],   # upper-cased rows
    [("filter_init", {"key": "o"}, None), ("regex-filter", {"regex": r"t\w{2}e"}, None)],
    [("regex-filter", {"regex": r"[a-z]{2}\d"}, None), ("filter_init", {"key": "out"}, None)],
])
def test_lean_path_parity(engine, chain):
    check_batch(engine, chain, _lean_slice())
    check_batch(engine, chain, _lean_slice(seed=11, nbatches=25))


RX_FLAT_CHAINS = [
    [("regex-filter", {"regex": r"\d{3}-\d{2}-\d{4}"}, None)],          # C1: max_len 11, anchor-free
    [("filter_regex", {}, None)],                                          # the same DFA, keep non-matches
    [("regex-filter", {"regex": r"^\d{2}"}, None)],                      # begin anchor: head scans
    [("regex-filter", {"regex": r"\d-\d$"}, None)],                      # end anchor: tail scans
    [("regex-filter", {"regex": r"x?"}, None)],                           # matches the empty string
    [("map", {}, None), ("regex-filter", {"regex": r"AB\d"}, None)],     # upper-cased rows
    [("regex-filter", {"regex": r"\d{14}"}, None)],                        # max_len 14: four context dwords
    [("regex-filter", {"regex": r"[a-c]b{5}"}, None)],                     # max_len 6: two context dwords
    [("regex-filter", {"regex": r"q"}, None)],                            # max_len 1: no context
]


def _rx_slice(seed):
    """Values of every length 0..70 and a few long ones, an SSN (or other
    digit runs) at every offset around the value's start, end and 16-byte
    chunk edges, digits in the record headers around it, some non-ASCII
    batches (deferred) and keys."""
    rnd = random.Random(seed)
    out, base = b"", 0
    for bi in range(60):
        b = P.Batch(base_offset=base)
        n = rnd.choice([1, 5, 17, 40, 64])
        for j in range(n):
            L = rnd.choice(list(range(0, 71)) + [200, 1000, 3000])
            v = bytearray(rnd.choice(b"abcxyzAB ,.;:") for _ in range(L))
            if L >= 11 and rnd.random() < 0.6:
                p = rnd.choice([0, 1, L - 11, L - 12, rnd.randrange(L - 10)])
                v[p:p + 11] = b"%03d-%02d-%04d" % (rnd.randrange(1000), rnd.randrange(100), rnd.randrange(10000))
            elif L >= 3 and rnd.random() < 0.3:
                v[0:2] = b"%02d" % rnd.randrange(100)
                v[-3:] = b"%d-%d" % (rnd.randrange(10), rnd.randrange(10))
            if L >= 14 and rnd.random() < 0.2:
                p = rnd.randrange(L - 13)
                v[p:p + 14] = b"%014d" % rnd.randrange(10 ** 14) if rnd.random() < 0.5 else b"cbbbbb12345678"
            if bi % 13 == 12 and j == 0:
                v += "é".encode()
            b.add_record(P.Record.new_key_value(b"123-45-6789" if j % 7 == 3 else None, bytes(v)))
        out += b.encode()
        base += n
    return out


@pytest.mark.parametrize("ci", range(len(RX_FLAT_CHAINS)))
def test_rx_flat_path(engine, ci, monkeypatch):
    """The flat regex path (FSG_EVAL_RX: k_rx_scan window bits + k_rx_decide
    with the edge scans) against the oracle's Pike VM, taken whatever the
    record sizes (FSG_FRX_MIN_REC=0: by default only slices of records
    averaging >= 512 bytes take it)."""
    monkeypatch.setenv("FSG_FRX_MIN_REC", "0")
    chain = RX_FLAT_CHAINS[ci]
    for seed in (1, 2):
        sl = _rx_slice(seed)
        check_batch(engine, chain, sl)
        g = gpu_chain(engine, chain)
        g.process_batch(sl)
        t = g.last_timings()
        assert t["eval_path"] == 7 and 0 < t["deferred"] < t["n_batches"], t  # FSG_EVAL_RX
    sl = synth.make_slice(1, 3000)
    check_batch(engine, chain, sl)


# ---------------------------------------------------------------------------
# string-concatenating aggregate (examples/aggregate) and array_map
# (examples/array_map_json_array): variable-size outputs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind,n", [(1, 150), (3, 1500), (4, 900), (5, 600)])
@pytest.mark.parametrize("chain", sorted(CONCAT_CHAINS))
def test_aggregate_concat_parity(engine, chain, kind, n):
    sl = synth.make_slice(kind, n, base_offset=5)
    check_batch(engine, CONCAT_CHAINS[chain], sl, calls=2)


@pytest.mark.parametrize("max_bytes", [0, 50, 4000, 200000])
def test_aggregate_concat_max_bytes(engine, max_bytes):
    check_batch(engine, CONCAT_CHAINS["agg_concat"], synth.make_slice(3, 900), max_bytes, calls=2)


def _check_array_doc(engine, doc):
    sl = _one_record_slice(doc, base=3)
    try:
        check_batch(engine, CHAINS["array_map"], sl)
    except AssertionError as e:
        raise AssertionError(f"doc {doc!r}: {e}") from e


def test_array_map_fuzz_one_record(engine):
    """Every document (valid, mutated, hand-picked errors) as a one-record batch:
    exploded records bit-exact, or the serde_json error hint/offset/value."""
    from tests import jsongen
    docs = jsongen.ARRAY_FIXED + jsongen.array_corpus(3, 250, 350)
    docs += jsongen.array_corpus(4, 60, 0, sorted_keys=False) + jsongen.array_corpus(6, 60, 0, ints_only=False)
    docs += jsongen.array_corpus(8, 80, 40, sorted_keys=False, ints_only=False)
    for doc in docs:
        _check_array_doc(engine, doc)


def _json_batches_slice(seed, nbatch=40, per=30):
    """Many batches of array documents with floats, keys out of order, whitespace
    and escapes (elements measured and written by k_canon_len / k_write_canon)
    mixed with batches of verbatim integer arrays."""
    from tests import jsongen
    rng = random.Random(seed)
    out = b""
    off = 0
    for k in range(nbatch):
        b = P.Batch(base_offset=off)
        for _ in range(per):
            if k % 3 == 0:
                doc = "[" + ",".join(str(rng.randrange(-999, 999)) for _ in range(rng.randrange(6))) + "]"
            else:
                doc = jsongen.array_doc(rng, sorted_keys=rng.random() < 0.5, ints_only=False)
            b.add_record(P.Record.new(doc.encode()))
        out += b.encode()
        off += per
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_array_map_canonical_batches(engine, seed):
    sl = _json_batches_slice(seed)
    check_batch(engine, CHAINS["array_map"], sl)
    check_batch(engine, CHAINS["array_map"], sl, max_bytes=30000)
    check_batch(engine, [("array_map_json_array", {}, None), ("filter_with_param", {"key": "."}, None)], sl)
    check_batch(engine, [("map", {}, None), ("array_map_json_array", {}, None)], sl)


def test_array_map_first_error_in_stream(engine):
    from tests import jsongen
    import random
    rng = random.Random(21)
    good = [jsongen.array_doc(rng).encode() for _ in range(600)]
    sl, base = b"", 0
    for k in range(60):
        b = P.Batch(base_offset=base)
        for j in range(10):
            v = good[k * 10 + j]
            if k == 37 and j == 4:
                v = b'[1,"x",]'
            b.add_record(P.Record.new(v))
        sl += b.encode()
        base += 10
    for chain in ("array_map", "filter_array_map"):
        check_batch(engine, CHAINS[chain], sl)
        check_batch(engine, CHAINS[chain], sl, max_bytes=30000)


def test_array_map_long_and_rewritten_elements(engine):
    """Elements above the lane-copy size (whole-wave copies), elements whose
    canonical form differs from the source (whitespace, \\u and \\/ escapes),
    uppercased input (map -> array_map)."""
    long_s = '"' + "x" * 3000 + '"'
    docs = [f"[{long_s},1,{long_s}]", "[" + ",".join(['"' + "y" * k + '"' for k in range(0, 200, 7)]) + "]",
            '[ "a\\u0041" , [ 1 , 2 ] , {"k" : "v\\/"} ]', "[" + ",".join(str(10**k) for k in range(19)) + "]",
            '["' + "\\u00e9" * 40 + '"]', '[[' + "1," * 400 + '1]]', '["abc","def"]', '[true,"t"]']
    sl, base = b"", 0
    for d in docs:
        b = P.Batch(base_offset=base)
        b.add_record(P.Record.new(d.encode()))
        b.add_record(P.Record.new(b'["tail"]'))
        sl += b.encode()
        base += 2
    for chain in ("array_map", "map_array_map"):
        check_batch(engine, CHAINS[chain], sl)


def test_array_map_c4_synthetic(engine):
    """C4 (BASELINE configs[3]): JSON arrays of 1-16 ints / short strings."""
    sl = synth.make_slice(5, 20000)
    out = check_batch(engine, CHAINS["array_map"], sl)
    assert out.n_records > 5 * 20000
    check_batch(engine, CHAINS["array_map"], sl, max_bytes=100000)


# ---------------------------------------------------------------------------
# per-partition aggregate state in HBM + RCCL merge (one rank on this box;
# the partition sharding / merge logic at world size 2 is tests/test_partitions.py)
# ---------------------------------------------------------------------------
def test_partition_state_rccl_one_rank():
    from fluvio_amd.smartengine import PartitionState, comm_unique_id
    eng = SmartEngine(0)
    eng.comm_init(comm_unique_id(), 1, 0)
    st = PartitionState(eng, 8)
    expect = []
    for p in range(8):
        sl = synth.make_slice(3, 1500 + 200 * p, seed=0xF105 + p)
        ch = gpu_chain(eng, [("aggregate-sum", {}, b"3" if p == 2 else None)])
        for _ in range(1 + p % 2):
            ch.process_batch(sl)
        st.collect(p, ch)
        expect.append(int(ch.accumulator(0)))
        o = orc_chain([("aggregate-sum", {}, b"3" if p == 2 else None)])
        for _ in range(1 + p % 2):
            o.process_batch(sl)
        assert ch.accumulator(0) == o.accumulator(0)
    st.allreduce()
    assert st.read() == expect
    # the raw-pointer entry on the same HBM vector: a second all-reduce over one rank is the identity
    eng.allreduce_state(st.device_ptr(), 8)
    assert st.read() == expect


def test_store_memory_exceeded_numbers(engine):
    ch = gpu_chain(engine, CHAINS["filter"], limit=1000)
    with pytest.raises(StoreMemoryExceeded) as e:
        ch.process_batch(synth.make_slice(2, 100))
    assert e.value.max == 1000 and e.value.requested > 1000


def test_crc_tables_on_every_device():
    """Engines on two devices in one process: each device gets its own CRC
    tables (fsg_kernels.hip upload_crc_tables), so both output CRCs are right."""
    import ctypes
    from fluvio_amd import _ffi
    n = ctypes.c_int(0)
    _ffi.lib().fsg_device_count(ctypes.byref(n))
    if n.value < 2:
        pytest.skip("one GPU on this box")
    sl = synth.make_slice(2, 500)
    ref = orc_chain(CHAINS["map"]).process_batch(sl)["bytes"]
    for d in (0, 1):
        e = SmartEngine(d)
        assert gpu_chain(e, CHAINS["map"]).process_batch(sl).raw == ref


# ---------------------------------------------------------------------------
# field projection (map_json_project, C3): parity unpinned by the reference
# (no such module ships in it); checked against the oracle's definition
# ---------------------------------------------------------------------------
def _project_may_be_unsupported(doc: bytes) -> bool:
    """Documents the device projection reports as unsupported
    (fsg_json_dev.h run_project): a key with an escape (it could decode to the
    field name), or a projected value that is not already serde_json's text
    (escapes, floats, objects that need re-ordering).  A coarse superset: any
    backslash, any fraction / exponent, any object inside an object."""
    import re
    return b"\\" in doc or re.search(rb"[0-9][.eE]", doc) is not None or \
        re.search(rb":\s*[\[{]", doc) is not None


def test_project_fuzz_one_record(engine):
    from tests import jsongen
    n_unsup = 0
    for doc in jsongen.corpus(17, 150, 350):
        sl = _one_record_slice(doc)
        for chain in ("project", "project_level_filter"):
            try:
                check_batch(engine, CHAINS[chain], sl)
            except AssertionError as e:
                if "Unsupported" in str(e) and _project_may_be_unsupported(doc):
                    n_unsup += 1
                    continue
                raise AssertionError(f"doc {doc!r}: {e}") from e
    assert n_unsup < 150  # most documents take the device path


def test_project_c3_chain_errors_in_stream(engine):
    """C3: filter -> projection -> uppercase, with projection errors and an
    error in a later stage after the value was narrowed (double_then... on text)."""
    from tests import jsongen
    import random
    rng = random.Random(5)
    good = [jsongen.valid_doc(rng).encode() for _ in range(500)]
    sl, base = b"", 0
    for k in range(50):
        b = P.Batch(base_offset=base)
        for j in range(10):
            v = good[k * 10 + j]
            if k == 31 and j == 2:
                v = b'{"message": "timeout x", "level": 5, "message": [1, 2'
            b.add_record(P.Record.new(v))
        sl += b.encode()
        base += 10
    for chain in ("filter_project_map", "project", "map_project_upper"):
        check_batch(engine, CHAINS[chain], sl)
        check_batch(engine, CHAINS[chain], sl, max_bytes=5000)
    # a stage erring on the projected (narrowed) value reports that value
    check_batch(engine, [("map_json_project", {}, None), ("filter_odd", {}, None)], sl)


# ---------------------------------------------------------------------------
# aggregate-json (examples/aggregate-json: HashMap<String, u32> += per key,
# the C5 keyed aggregate): every record's output = the pretty map after it, its
# keys in the guest HashMap's bucket order (SipHash-1-3 under the wasm32
# RandomState sequence, hashbrown's groups: oracle hb_*, tests/rust_hashmap.py),
# the stored accumulator, errors; byte-for-byte against the oracle
# ---------------------------------------------------------------------------
def _keyed_slice(seed, nbatches=30, nkeys=40, bad=0.0, escapes=False):
    import json
    import random
    rng = random.Random(seed)
    keys = ["repo-%04d" % i for i in range(nkeys)]
    out, base = b"", 0
    for _ in range(nbatches):
        b = P.Batch(base_offset=base)
        n = rng.choice([1, 5, 17, 64, 100])
        for _ in range(n):
            if rng.random() < bad:
                v = rng.choice([b'{"a": -3}', b'{"a": "x"}', b"[1,2]", b'{"a": 4294967296}', b'{"a": 1', b"7"])
            else:
                d = {}
                for _ in range(rng.randint(0, 3)):
                    d[rng.choice(keys)] = rng.randint(0, 2 ** 32 - 1) if rng.random() < 0.1 else rng.randint(0, 1000)
                v = json.dumps(d, separators=(",", ":") if rng.random() < 0.5 else (", ", ": ")).encode()
                if rng.random() < 0.05:
                    v = v.replace(b"}", b', "repo-0001": 2}') if len(d) else v  # duplicate key: last wins
            key = None if rng.random() < 0.8 else b"k"
            b.add_record(P.Record.new_key_value(key, v))
        out += b.encode()
        base += n
    return out


AGGJ_CHAINS = {
    "aggj": [("aggregate-json", {}, None)],
    "aggj_acc": [("aggregate-json", {}, b'{\n  "repo-0003": 10,\n  "z\\"q": 1\n}')],
    "aggj_bad_acc": [("aggregate-json", {}, b"not json")],
    # '{' then a failure: the visitor's map and HashMap::default() both draw a RandomState
    "aggj_brace_bad_acc": [("aggregate-json", {}, b' {"repo-0002": "x"}')],
    # a repeated key: HashMap::insert reserves before it finds the key (the layout can grow)
    "aggj_dup_acc": [("aggregate-json", {}, b'{"a": 1, "b": 2, "c": 3, "a": 4, "d": 5, "e": 6, "f": 7, "a": 9}')],
    "filter_aggj": [("filter_init", {"key": "repo-000"}, None), ("aggregate-json", {}, None)],
    "map_aggj": [("map", {}, None), ("aggregate-json", {}, b'{"REPO-0001": 5}')],
}


@pytest.mark.parametrize("chain", sorted(AGGJ_CHAINS))
@pytest.mark.parametrize("seed,bad", [(1, 0.0), (2, 0.0), (3, 0.01)])
def test_aggregate_json_parity(engine, chain, seed, bad):
    check_batch(engine, AGGJ_CHAINS[chain], _keyed_slice(seed, bad=bad), calls=2)


@pytest.mark.parametrize("max_bytes", [0, 300, 20000])
def test_aggregate_json_max_bytes(engine, max_bytes):
    check_batch(engine, AGGJ_CHAINS["aggj"], _keyed_slice(5, nbatches=12), max_bytes, calls=2)


def test_aggregate_json_many_blocks(engine):
    """~15K records: hundreds of 32-record blocks, each replayed by its own wave
    from the per-block rows (k_aggj_bsum / k_aggj_colscan / k_aggj_text)."""
    check_batch(engine, AGGJ_CHAINS["aggj"], _keyed_slice(11, nbatches=400, nkeys=300), calls=2)


def test_aggregate_json_large_dictionary(engine):
    """More than kAjLds (4096) keys: the values replay in the block rows in HBM
    instead of LDS; the second call starts from an accumulator of >4096 keys."""
    import json
    out, base = b"", 0
    for bi in range(12):
        b = P.Batch(base_offset=base)
        for r in range(8):
            d = {"k%05d" % (bi * 512 + r * 64 + j): bi + r + j for j in range(64)}
            d["k00001"] = 7  # an old key again
            b.add_record(P.Record.new(json.dumps(d).encode()))
        out += b.encode()
        base += 8
    check_batch(engine, AGGJ_CHAINS["aggj"], out, calls=2)


# ---------------------------------------------------------------------------
# C5 at its configuration on one rank: 64 partitions, each partition's chain,
# output batches and accumulator against the oracle over two calls, the
# per-partition i32 vector merged by RCCL (fsg_state_*), the keyed totals of
# the aggregate-json maps merged through the C ABI by exact key (fsg_keyed_*:
# RCCL all-gather of the key lists, union dictionary, dense u32 all-reduce)
# ---------------------------------------------------------------------------
C5_PARTS = 64


@pytest.fixture(scope="module")
def comm_engine():
    from fluvio_amd.smartengine import comm_unique_id
    eng = SmartEngine(0)
    eng.comm_init(comm_unique_id(), 1, 0)
    return eng


def _same_batch(g_out, o_res):
    assert o_res["status"] == 0
    assert g_out.raw == o_res["bytes"]
    assert_same_error(g_out.error, o_res["error"])


def test_c5_agg_sum_64_partitions(comm_engine):
    from fluvio_amd.smartengine import PartitionState
    from fluvio_amd import partitions as PT
    st = PartitionState(comm_engine, C5_PARTS)
    expect = []
    for p in range(C5_PARTS):
        acc = b"-2147483000" if p == 5 else (b"17" if p % 9 == 0 else None)
        mods = [("aggregate-sum", {}, acc)]
        g, o = gpu_chain(comm_engine, mods), orc_chain(mods)
        for call in range(2):
            sl = synth.make_slice(3, 700 + 37 * p + 500 * call, seed=0xC5 + 131 * p + call, base_offset=1000 * call)
            _same_batch(g.process_batch(sl), o.process_batch(sl))
            assert g.accumulator(0) == o.accumulator(0)
        st.collect(p, g)
        expect.append(int(o.accumulator(0)))
    st.allreduce()
    assert st.read() == [PT.wrap_i32(v) for v in expect]


def _oracle_map(o):
    import json
    a = o.accumulator(0)
    return {k.encode(): v for k, v in json.loads(a).items()} if a else {}


def test_c5_keyed_64_partitions(comm_engine):
    """aggregate-json per partition over {"repo-NNNN": n} records routed by
    SipHash (1024 keys), two calls; three partitions start from an accumulator
    naming keys other partitions own, so the merge really sums across
    partitions; the topic totals (exact keys) == the oracle's maps summed."""
    from fluvio_amd.smartengine import KeyedState
    slices = synth.make_keyed_slices(C5_PARTS, 1500, 1024)
    ks = KeyedState(comm_engine)
    expect, chains = {}, []
    for p in range(C5_PARTS):
        acc = b'{"repo-0001": 4000000000, "other": 3}' if p in (3, 40, 63) else None
        mods = [("aggregate-json", {}, acc)]
        g, o = gpu_chain(comm_engine, mods), orc_chain(mods)
        for call in range(2):
            _same_batch(g.process_batch(slices[p]), o.process_batch(slices[p]))
        assert g.accumulator(0) == o.accumulator(0)
        for k, v in _oracle_map(o).items():
            expect[k] = (expect.get(k, 0) + v) & 0xFFFFFFFF
        ks.collect(g)
        chains.append(g)
    assert ks.allreduce() == len(expect) > 1000
    assert ks.read() == expect
    # another merge round over the same states (reset, collect, all-reduce)
    ks.reset()
    for g in chains:
        ks.collect(g)
    ks.allreduce()
    assert ks.read() == expect
    # a chain that never ran contributes its initial accumulator
    ks.collect(gpu_chain(comm_engine, [("aggregate-json", {}, b'{"fresh": 9, "other": 1}')]))
    ks.allreduce()
    e2 = dict(expect)
    e2[b"fresh"] = 9
    e2[b"other"] = e2[b"other"] + 1
    assert ks.read() == e2


def test_keyed_table_growth_and_dead_copies(engine):
    """Many chains with overlapping keys into one table: the table grows
    (rehash) and equal keys inserted concurrently leave one live copy."""
    import json
    from fluvio_amd.smartengine import KeyedState
    ks = KeyedState(engine)
    expect = {}
    for c in range(6):
        d = {"k%05d" % ((c * 700 + j) % 3000): j + c for j in range(900)}
        acc = json.dumps(d).encode()
        g = gpu_chain(engine, [("aggregate-json", {}, acc)])
        for k, v in d.items():
            expect[k.encode()] = (expect.get(k.encode(), 0) + v) & 0xFFFFFFFF
        ks.collect(g)
    ks.allreduce()
    assert ks.read() == expect



def test_aggregate_json_process_kat(engine):
    """One `process` call (engine.rs:135): the per-record pretty maps and the
    stored accumulator, as the oracle has them."""
    g = gpu_chain(engine, AGGJ_CHAINS["aggj"])
    o = orc_chain(AGGJ_CHAINS["aggj"])
    vals = [b'{"a":1}', b'{"b":2,"a":3}', b'{}', b'{"c": 1, "c": 7}']
    out = g.process(SmartModuleInput.try_from_records([P.Record.new(v) for v in vals]))
    ref = o.process(P.encode_records([P.Record.new(v) for v in vals]))
    assert [r.value for r in out.successes] == [r.value for r in P.decode_records(ref["bytes"])]
    # bucket order under k0 = 7 (the fourth record's accumulator map): b, a, c (tests/rust_hashmap.py)
    assert out.successes[-1].value == b'{\n  "b": 2,\n  "a": 4,\n  "c": 7\n}'
    assert g.accumulator(0) == o.accumulator(0)


# ---------------------------------------------------------------------------
# stateful filters with look_back: filter_look_back (keep above
# PREV) and filter_hashset (dedup over a BoundedHashSet), last stage of a chain
# ---------------------------------------------------------------------------
def test_look_back_kats(engine, kats):
    """engine.rs:388-470, filter_hashset test_set, SPU produce.rs:522-1020 (a
    chain per produce request / per replica), stream_fetch.rs:2483-2605."""
    from fluvio_amd.smartengine import Lookback, SmartModuleLookbackRuntimeError
    from tests.lookback_steps import run_lookback_case

    for case in kats["look_back"]:
        name, params = case["module"]

        def new_chain(lb, name=name, params=params):
            b = SmartModuleChainBuilder.default()
            cb = SmartModuleConfig.builder().params(params)
            if lb:
                cb.lookback(Lookback.Last(lb[1]) if lb[0] == "last" else Lookback.Age(lb[2], lb[1]))
            b.add_smart_module(cb.build(), builtin(name))
            return b.initialize(engine), SmartModuleChainMetrics()

        def look_back(ch, values):
            chain, m = ch
            before = m.invocation_count()
            seen = []
            try:
                chain.look_back(lambda lb: seen.append(lb) or [P.Record.new(v) for v in values], m)
                err = None
            except SmartModuleLookbackRuntimeError as e:
                err = {"hint": e.hint, "offset": e.offset, "key": e.record_key, "value": e.record_value}
            assert len(seen) == 1  # read_fn is asked once, for the stage's Lookback
            return err, m.invocation_count() - before

        def process(ch, values):
            chain, m = ch
            before = m.invocation_count()
            out = chain.process(SmartModuleInput.try_from_records([P.Record.new(v) for v in values]), m)
            assert out.error is None
            return [r.value for r in out.successes], m.invocation_count() - before

        run_lookback_case(case, new_chain, look_back, process)


def test_look_back_not_configured(engine):
    """No Lookback on the config, or a module without look_back: read_fn is never called."""
    from fluvio_amd.smartengine import Lookback
    for mods, lb in (([("filter_hashset", {}, None)], None), ([("filter", {}, None)], Lookback.Last(3))):
        b = SmartModuleChainBuilder.default()
        cb = SmartModuleConfig.builder().params(mods[0][1])
        if lb:
            cb.lookback(lb)
        b.add_smart_module(cb.build(), builtin(mods[0][0]))
        ch = b.initialize(engine)
        m = SmartModuleChainMetrics()
        ch.look_back(lambda _lb: pytest.fail("read_fn called"), m)
        assert m.invocation_count() == 0 and m.bytes_in() == 0


SF_CHAINS = {
    "look_back": [("filter_look_back", {}, None)],
    "map_double_look_back": [("map_double", {}, None), ("filter_look_back", {}, None)],
    "dedup": [("filter_hashset", {}, None)],
    "dedup_evicting": [("filter_hashset", {"count": "40"}, None)],
    "dedup_zero": [("filter_hashset", {"count": "0"}, None)],
    "map_dedup": [("map", {}, None), ("filter_hashset", {"count": "500"}, None)],
    "filter_dedup": [("filter_with_param", {"key": "1"}, None), ("filter_hashset", {}, None)],
    # an integer stage before the dedup: the set holds the records' text (a segment boundary)
    "map_double_dedup": [("map_double", {}, None), ("filter_hashset", {"count": "300"}, None)],
    "filter_map_dedup": [("filter_map", {}, None), ("filter_hashset", {}, None)],
    "map_double_odd_dedup": [("map_double", {}, None), ("filter_odd", {}, None), ("filter_hashset", {}, None)],
}


def check_sequence(engine, modules, calls, look_back=None):
    """One GPU chain and one oracle chain through a sequence of process_batch
    calls [(slice, max_bytes)], optionally after a look_back over `look_back`
    (encoded records), compared call by call."""
    from fluvio_amd.smartengine import Lookback, SmartModuleLookbackRuntimeError
    b = SmartModuleChainBuilder.default()
    for i, (name, params, acc) in enumerate(modules):
        cb = SmartModuleConfig.builder().params(params or {})
        if look_back is not None and i == len(modules) - 1:
            cb.lookback(Lookback.Last(1000))
        b.add_smart_module(cb.build(), builtin(name))
    g = b.initialize(engine)
    o = orc_chain(modules)
    if look_back is not None:
        ol = o.look_back(len(modules) - 1, look_back)
        try:
            g.look_back(lambda _lb: look_back)
            assert ol["error"] is None
        except SmartModuleLookbackRuntimeError as e:
            oe = ol["error"]
            assert oe is not None
            assert (e.hint, e.offset, e.record_key, e.record_value) == (oe["hint"], oe["offset"], oe["key"],
                                                                         oe["value"])
    for sl, max_bytes in calls:
        gm = SmartModuleChainMetrics()
        oout = o.process_batch(sl, max_bytes)
        if oout["status"] != 0:
            with pytest.raises(Exception):
                g.process_batch(sl, max_bytes, gm)
            continue
        gout = g.process_batch(sl, max_bytes, gm)
        assert gout.raw == oout["bytes"], "output batch bytes differ"
        assert gout.n_records == oout["n_records"]
        assert_same_error(gout.error, oout["error"])
        assert gm.records_out() == oout["metrics"]["records_out"]
        assert gm.bytes_in() == oout["metrics"]["bytes_in"]


@pytest.mark.parametrize("kind,n", [(3, 6000), (4, 3000), (1, 1500)])
@pytest.mark.parametrize("chain", sorted(SF_CHAINS))
def test_stateful_filter_parity(engine, chain, kind, n):
    """Three different slices through one chain: the state carries across calls."""
    calls = [(synth.make_slice(kind, n, seed=synth.SEEDS[kind] + k, base_offset=500 + 7 * n * k), (1 << 64) - 1)
             for k in range(3)]
    check_sequence(engine, SF_CHAINS[chain], calls)


@pytest.mark.parametrize("max_bytes", [0, 100, 3000, 40000])
@pytest.mark.parametrize("chain", ["look_back", "dedup", "dedup_evicting"])
def test_stateful_filter_max_bytes(engine, chain, max_bytes):
    """The batch cut by max_bytes was processed (its state kept), later ones not."""
    calls = [(synth.make_slice(3, 4000, seed=0x51 + k, base_offset=100 + 5000 * k), max_bytes) for k in range(3)]
    check_sequence(engine, SF_CHAINS[chain], calls)


@pytest.mark.parametrize("chain", ["look_back", "dedup", "dedup_evicting"])
def test_stateful_filter_after_look_back(engine, chain):
    lb_ok = P.encode_records([P.Record.new(str(v)) for v in (5, -3, 700, 12, 12, 999, 40)])
    calls = [(synth.make_slice(3, 5000, seed=0x77), (1 << 64) - 1)]
    check_sequence(engine, SF_CHAINS[chain], calls, look_back=lb_ok)
    lb_bad = P.encode_records([P.Record.new(v) for v in (b"5", b"900", b"x1", b"\xff")])  # stops at the first error
    check_sequence(engine, SF_CHAINS[chain], calls, look_back=lb_bad)


def test_dedup_large_sequential(engine):
    """Evictions across many batches (the sequential BoundedHashSet walk)."""
    calls = [(synth.make_slice(3, 40000, seed=0x99 + k), (1 << 64) - 1) for k in range(2)]
    check_sequence(engine, [("filter_hashset", {"count": "1500"}, None)], calls)
    check_sequence(engine, [("filter_hashset", {"count": "1000000"}, None)], calls)


# ---------------------------------------------------------------------------
# CRC32C verify on ingest (north_star): report only, processing unchanged
# ---------------------------------------------------------------------------
def test_verify_crc_on_ingest(engine):
    for kind, n in ((2, 3000), (1, 5000), (3, 20000), (4, 2000)):
        sl = synth.make_slice(kind, n, base_offset=9)
        batches = list(P.decode_batches(sl))
        rs = ResidentSlice(engine, sl)
        bad, first, _ms = rs.verify_crc()
        assert (bad, first) == (0, -1), kind
        # the oracle's CRC32C of each batch's covered bytes matches the stored one
        pos = 0
        for b in batches:
            blen = struct.unpack(">i", sl[pos + 8:pos + 12])[0]
            assert O.crc32c(sl[pos + 21:pos + 12 + blen]) == struct.unpack(">I", sl[pos + 17:pos + 21])[0]
            pos += 12 + blen
        # corrupt three batches (a record byte, a header byte in the CRC range, the stored CRC itself)
        corrupt = bytearray(sl)
        starts = []
        pos = 0
        while pos < len(sl):
            starts.append(pos)
            pos += 12 + struct.unpack(">i", sl[pos + 8:pos + 12])[0]
        picks = sorted({1 % len(starts), len(starts) // 2, len(starts) - 1})
        for j, bi in enumerate(picks):
            p0 = starts[bi]
            off = [p0 + 70, p0 + 30, p0 + 18][j % 3]
            corrupt[off] ^= 0x40
        rs2 = ResidentSlice(engine, bytes(corrupt))
        bad, first, _ms = rs2.verify_crc()
        assert (bad, first) == (len(picks), picks[0]), kind
        # started on the slice's stream, processed beside it, collected after
        modules = [("filter_init", {"key": "timeout"}, None)]
        rs2.verify_crc_start()
        out = gpu_chain(engine, modules).process_slice(rs2).raw
        assert rs2.verify_crc()[:2] == (len(picks), picks[0]), kind
        assert out == orc_chain(modules).process_batch(bytes(corrupt))["bytes"], kind
    # the reference never checks: a corrupted CRC field does not change process_batch
    sl = synth.make_slice(2, 2000)
    c = bytearray(sl)
    c[17] ^= 0xFF
    modules = [("filter_init", {"key": "timeout"}, None)]
    assert gpu_chain(engine, modules).process_batch(bytes(c)).raw == orc_chain(modules).process_batch(bytes(c))["bytes"]


def test_verify_crc_large_batches(engine):
    """Batches beyond the 16 KiB window (one wave folds many 1 KiB rounds)."""
    sl = synth.make_slice(2, 3000, max_section=300000)
    rs = ResidentSlice(engine, sl)
    assert rs.verify_crc()[:2] == (0, -1)


def test_verify_blocks_every_shape(engine):
    """k_verify_crc over batches of every size class (a few units, a few
    KiB, beyond one wave's 1 KiB round) at every alignment, with corruptions
    in the first and last units, the middle and the stored CRC; the count
    and first bad batch match the CPU check, also when started beside
    process_batch after a reframe."""
    rnd = random.Random(11)
    sizes = [rnd.randint(1, 6) for _ in range(300)] + [rnd.randint(20, 200) for _ in range(60)] + \
        [rnd.randint(1500, 4000) for _ in range(8)] + [9000]
    rnd.shuffle(sizes)
    raw, starts, base = b"", [], 0
    for n in sizes:
        recs = []
        for i in range(n):
            r = P.Record.new_key_value(None, bytes(rnd.choice(b"abcdefgh") for _ in range(rnd.randint(2, 90))))
            r.preamble.offset_delta = i
            recs.append(r.encode())
        starts.append(len(raw))
        raw += _raw_batch(base, recs)
        base += n
    rs = ResidentSlice(engine, raw)
    assert rs.n_batches == len(sizes) and rs.device_framed
    assert rs.verify_crc()[:2] == (0, -1)
    c = bytearray(raw)
    picks = sorted(rnd.sample(range(len(sizes)), 40))
    for bi in picks:
        p0 = starts[bi]
        end = p0 + 12 + struct.unpack(">i", raw[p0 + 8:p0 + 12])[0]
        # (header bytes the framing reads stay intact: batch length, magic, attributes, record count)
        off = rnd.choice([p0 + 17 + rnd.randint(0, 3), p0 + 27 + rnd.randint(0, 29), max(p0 + 61, end - 1 - rnd.randint(0, 40)),
                          rnd.randint(p0 + 61, end - 1)])
        c[off] ^= 1 << rnd.randint(0, 7)
    want = sum(1 for i, p0 in enumerate(starts)
               if O.crc32c(bytes(c[p0 + 21:p0 + 12 + struct.unpack(">i", raw[p0 + 8:p0 + 12])[0]]))
               != struct.unpack(">I", bytes(c[p0 + 17:p0 + 21]))[0])
    assert want == len(picks)
    rs2 = ResidentSlice(engine, bytes(c))
    assert rs2.verify_crc()[:2] == (len(picks), picks[0])
    rs2.reframe()
    rs2.verify_crc_start()
    assert rs2.verify_crc()[:2] == (len(picks), picks[0])


def test_reframe_resident_slice(engine):
    """fsg_slice_reframe (the fetch-shaped step): the HBM-resident bytes framed
    again on the device give the same batches, CRC verdicts and process_batch
    output, call after call."""
    sl = synth.make_slice(2, 3000, base_offset=4)
    rs = ResidentSlice(engine, sl)
    nb, nr = rs.n_batches, rs.n_records
    g = gpu_chain(engine, CHAINS["filter_init_timeout"])
    ref = orc_chain(CHAINS["filter_init_timeout"]).process_batch(sl)["bytes"]
    for i in range(4):
        rs.reframe()
        if i % 2:  # the bench's fetch step: the verify beside process_batch
            rs.verify_crc_start()
            assert g.process_slice(rs).raw == ref
            assert rs.verify_crc()[:2] == (0, -1)
        else:
            assert rs.verify_crc()[:2] == (0, -1)
            assert g.process_slice(rs).raw == ref
    rs.verify_crc_start()
    rs.reframe()  # waits for the verify in flight; its result stays collectable
    assert rs.verify_crc()[:2] == (0, -1)
    assert (rs.n_batches, rs.n_records) == (nb, nr)



def test_reframe_host_framed_slice_is_unsupported(engine):
    """fsg_slice_reframe on a slice the host walk framed (no magic 2 at position
    0): FSG_E_UNSUPPORTED before anything is reset, so the slice keeps its
    batches and still processes exactly like the oracle."""
    nomagic = bytearray(synth.make_slice(2, 1500))
    nomagic[16] = 1
    nomagic = bytes(nomagic)
    rs = ResidentSlice(engine, nomagic)
    assert not rs.device_framed
    with pytest.raises(Unsupported):
        rs.reframe()
    g = gpu_chain(engine, CHAINS["filter_init_timeout"])
    o = orc_chain(CHAINS["filter_init_timeout"]).process_batch(nomagic)
    out = g.process_slice(rs)
    assert out.raw == o["bytes"] and out.n_records == o["n_records"] > 0


def test_array_map_many_tiny_batches_near_store_limit(engine):
    """The lean array path's per-batch element bitmaps (~4.4 KB a batch) are this
    engine's scratch, not guest memory: 3,000 one-record batches run under a
    4 MB store limit, as the reference (limit per guest call = per batch)
    runs them."""
    out, base = b"", 0
    for i in range(3000):
        b = P.Batch(base_offset=base)
        b.add_record(P.Record.new(b"[1,2]" if i % 3 else b'["a",7,null]'))
        out += b.encode()
        base += 1
    g = gpu_chain(engine, CHAINS["array_map"], limit=4 << 20)
    o = orc_chain(CHAINS["array_map"]).process_batch(out)
    r = g.process_batch(out)
    assert r.raw == o["bytes"] and r.n_records == o["n_records"]
    assert g.last_timings()["eval_path"] == 3  # FSG_EVAL_ARRAY


def test_group_order_walk_timing(engine):
    """fsg_timings.order_ms: the aggregate-json order walk's own duration: the
    group's one launch (the same for every chain of a group call), a chain's
    own launch outside a group."""
    from fluvio_amd.smartengine import process_slices
    slices = synth.make_keyed_slices(4, 800, 64)
    chains = [gpu_chain(engine, [("aggregate-json", {}, None)]) for _ in range(4)]
    rs = [ResidentSlice(engine, slices[p]) for p in range(4)]
    process_slices(chains, rs)
    ts = [c.last_timings() for c in chains]
    assert all(t["order_ms"] > 0 for t in ts), ts
    assert len({t["order_ms"] for t in ts}) == 1
    chains[0].process_slice(rs[0])
    assert chains[0].last_timings()["order_ms"] > 0
    g = gpu_chain(engine, CHAINS["filter_init_timeout"])
    g.process_batch(synth.make_slice(2, 300))
    assert g.last_timings()["order_ms"] == 0

# ---------------------------------------------------------------------------
# compressed record sections decompressed on the GPU at ingest
# ---------------------------------------------------------------------------
from tests.compressed_slices import recompress  # noqa: E402

COMPRESSED_CHAINS = ["filter_init_timeout", "filter_then_map", "regex_ssn", "filter_json", "empty", "project"]


@pytest.mark.parametrize("codecs,flags", [([1], 0), ([2], 0), ([3], 0), ([3], 15), ([2], 3), ([0, 3, 2, 1], {3: 7, 1: 9}),
                                          ([1, 0], 1), ([4], 0), ([4], 0x100 | 19), ([4], 0x200 | 0x400 | 0x800),
                                          ([0, 4, 2, 4, 1], {4: 0x100 | 7})])
@pytest.mark.parametrize("chain", COMPRESSED_CHAINS)
def test_compressed_slice_parity(engine, chain, codecs, flags):
    kind = 1 if chain == "regex_ssn" else 2
    sl = synth.make_slice(kind, 1200, base_offset=300)
    check_batch(engine, CHAINS[chain], recompress(sl, codecs, flags))


def test_decompression_bomb_is_store_memory(engine):
    """A small gzip section that inflates past the chain's store limit is
    StoreMemoryExceeded before anything is allocated (the reference's guest would
    need that much memory for the batch: engine.rs:24, limiter.rs:18-35), not a
    device allocation failure; under the limit the same kind of slice decodes."""
    import gzip
    from tests.compressed_slices import batches
    sl = synth.make_slice(2, 300)
    pos, blen = next(batches(sl))
    hdr = bytearray(sl[pos:pos + 57])
    sec = gzip.compress(b"\0" * (8 << 20), 9)  # 8 MiB of zeros in ~8 KiB
    assert len(sec) < 64 << 10
    hdr[21:23] = struct.pack(">h", (struct.unpack(">h", bytes(hdr[21:23]))[0] & ~7) | 1)
    hdr[8:12] = struct.pack(">i", 45 + len(sec))
    hdr[17:21] = struct.pack(">I", O.crc32c(bytes(hdr[21:57]) + sec))
    bomb = bytes(hdr) + sec
    ch = gpu_chain(engine, CHAINS["filter_init_timeout"], limit=4 << 20)
    with pytest.raises(StoreMemoryExceeded) as e:
        ch.process_batch(bomb + sl)
    assert e.value.max == 4 << 20 and e.value.requested == 8 << 20
    # the chain is still usable, and a slice within the limit goes through
    check_batch(engine, CHAINS["filter_init_timeout"], recompress(sl, [1]))
    assert ch.process_batch(sl).raw == orc_chain(CHAINS["filter_init_timeout"]).process_batch(sl)["bytes"]


@pytest.mark.parametrize("chain", ["filter_map", "agg_sum", "filter_odd"])
def test_compressed_int_chains(engine, chain):
    sl = synth.make_slice(3, 20000, base_offset=7)
    check_batch(engine, CHAINS[chain], recompress(sl, [3, 1, 2, 4], {3: 3}))


@pytest.mark.parametrize("level", [1, 3, 9, 19])
def test_zstd_large_sections(engine, level):
    """zstd over ~300 KiB record sections: several 128 KiB blocks per frame,
    Huffman literals with 4 streams, FSE / repeat / predefined sequence tables,
    repeat offsets across blocks; C2 JSON logs and C4 arrays."""
    for kind, n in ((2, 1500), (5, 6000)):
        sl = synth.make_slice(kind, n, base_offset=3, max_section=300000)
        check_batch(engine, CHAINS["filter_init_timeout" if kind == 2 else "array_map"],
                    recompress(sl, [4], 0x100 | level))


def test_compressed_resident_and_errors(engine):
    sl = synth.make_slice(2, 2000)
    csl = recompress(sl, [2, 3])
    rs = ResidentSlice(engine, csl)
    assert not rs.device_framed and rs.n_records == 2000
    assert rs.verify_crc()[:2] == (0, -1)  # checked on the stored (compressed) bytes at ingest
    rs.verify_crc_start()  # nothing to start: the ingest result is returned
    assert rs.verify_crc()[:2] == (0, -1)
    from tests.compressed_slices import batches
    crc_bad = bytearray(csl)
    crc_bad[list(batches(csl))[4][0] + 18] ^= 1  # batch 4's stored CRC
    rsb = ResidentSlice(engine, bytes(crc_bad))
    assert rsb.verify_crc()[:2] == (1, 4) and rsb.n_records == 2000
    modules = [("filter_init", {"key": "timeout"}, None)]
    out = gpu_chain(engine, modules).process_batch(csl)
    assert out.raw == orc_chain(modules).process_batch(csl)["bytes"]
    assert out.raw[22] & 7 == 2  # set_compression: the first surviving batch's codec
    # a batch that fails to decode (checksum / stream error): io::Error at that batch
    for codecs, flags in (([3], 3), ([2], 0), ([1], 0)):
        bad = recompress(sl, codecs, flags, corrupt={3: 50})
        check_batch(engine, modules, bad)
        assert orc_chain(modules).process_batch(bad)["status"] == -104  # FSG_E_IO
    # zstd bits on uncompressed sections: not zstd frames -> io::Error, like the oracle
    z = bytearray(recompress(sl, [0]))
    z[22] = (z[22] & ~7) | 4
    check_batch(engine, modules, bytes(z))
    # corrupted zstd sections (content checksum on): both sides stop at that batch
    for off in (5, 30, 60, 200):
        bad = recompress(sl, [4], 0x100, corrupt={2: off})
        check_batch(engine, modules, bad)


# ---------------------------------------------------------------------------
# substring / uppercase edge cases on the lean path: records with keys,
# non-zero headers, long timestamp / offset varints, needles across 16-byte
# chunks and 1 KiB wave loads, non-ASCII values (deferred batches)
# ---------------------------------------------------------------------------
def _flat_slice(seed=3, nbatches=60, words=None):
    import random
    rnd = random.Random(seed)
    words = words or ["timeout", "time", "out", "level", "lev", "TIMEOUT", "eout", "xx", "y" * 13, "é"]
    out = b""
    base = 5
    for bi in range(nbatches):
        b = P.Batch(base_offset=base)
        b.header.first_timestamp = rnd.choice([-1, 0, 1 << 40])
        nrec = rnd.choice([1, 2, 15, 40, 64, 65]) if bi % 4 else rnd.randint(0, 8)
        size = rnd.choice([0, 3, 16, 61, 250, 1000])
        for i in range(nrec):
            parts = []
            while sum(len(p) + 1 for p in parts) < size:
                pool = words if bi % 7 == 6 else words[:-1]  # every 7th batch may hold a non-ASCII value
                parts.append(rnd.choice(pool))
            v = rnd.choice(["", " ", "-"]).join(parts)[: size or None]
            key = None if rnd.random() < 0.6 else rnd.choice([b"", b"timeout", b"k" * 40])
            r = P.Record.new_key_value(key, v.encode())
            if rnd.random() < 0.2:
                r.headers = rnd.choice([1, -3, 60])
            b.add_record(r)
            if rnd.random() < 0.2:  # long varints: timestamp / offset deltas far from zero
                r.preamble.timestamp_delta = rnd.choice([1 << 33, -(1 << 20), 300])
        enc = b.encode()
        if len(enc) - 57 > 16384:
            continue
        out += enc
        base += max(nrec, 1) + rnd.randint(0, 3)
    return out


FLAT_CHAINS = [
    [("filter_init", {"key": "timeout"}, None)],
    [("filter_init", {"key": "level"}, None)],                     # 4..6 bytes: first 4-gram at every position
    [("filter_init", {"key": "time"}, None)],
    [("filter_init", {"key": "yyyyyyyyyyyyyyyyyyyyyyyyyy"}, None)],  # 26 bytes across chunks
    [("map", {}, None), ("filter_init", {"key": "TIMEOUT"}, None)],
    [("filter_init", {"key": "out"}, None)],                       # 3 bytes: k_eval_lean
    [("filter_init", {"key": "timeout"}, None), ("map", {}, None), ("filter_init", {"key": "LEVEL"}, None)],
    [("filter_init", {"key": ""}, None), ("map", {}, None)],
    [("map", {}, None)],
]


@pytest.mark.parametrize("ci", range(len(FLAT_CHAINS)))
@pytest.mark.parametrize("seed", [3, 4])
def test_flat_path_parity(engine, ci, seed):
    chain = FLAT_CHAINS[ci]
    sl = _flat_slice(seed)
    check_batch(engine, chain, sl)
    g = gpu_chain(engine, chain)
    g.process_batch(sl)
    t = g.last_timings()
    # one substring stage with a needle of >= 4 bytes: the flat path (FSG_EVAL_FLAT),
    # else k_eval_lean (FSG_EVAL_LEAN)
    subs = [m for m in chain if m[0] == "filter_init"]
    flat = len(subs) == 1 and len(subs[0][1]["key"]) >= 4
    assert t["eval_path"] == (4 if flat else 1), t
    assert 0 < t["deferred"] < t["n_batches"], t  # the non-ASCII / 65-record batches go to k_eval
    # the same chain over the synthetic C2 logs: nothing deferred
    sl2 = synth.make_slice(2, 3000, base_offset=9)
    check_batch(engine, chain, sl2)


def test_flat_needle_at_window_edges(engine):
    """A 7-byte needle at every offset around 16-byte chunks and 1 KiB loads
    (the flat path's edge chunks: starts before the value, ends past it)."""
    for shift in range(0, 40, 3):
        b = P.Batch(base_offset=100 + shift)
        for i in range(16):
            pad = 1024 * (i % 3) - 40 + shift + i
            v = ("x" * max(pad, 0) + "timeout" + "z" * (i * 7)).encode()
            b.add_record(P.Record.new(v))
        b2 = P.Batch(base_offset=200)
        b2.add_record(P.Record.new(b"timeou"))
        check_batch(engine, [("filter_init", {"key": "timeout"}, None)], b.encode() + b2.encode())


def test_flat_edges_exhaustive(engine):
    """The flat path's per-chunk bits against every value / chunk alignment:
    values of 0..40 bytes at every offset, the needle at every position of the
    value and just outside it (in the record header and trailer bytes), a
    needle byte in the previous record's value, high bytes in the header
    varints only (ASCII values) and in the value (deferred)."""
    out, base = b"", 0
    for vlen in list(range(0, 41)) + [255, 1000]:
        b = P.Batch(base_offset=base)
        for pos in range(-3, vlen + 2, 1 if vlen < 41 else 97):
            v = bytearray(b"a" * vlen)
            if 0 <= pos and pos + 4 <= vlen:
                v[pos:pos + 4] = b"tiMe"
            elif pos < 0 and vlen >= 4 + pos:
                v[0:4 + pos] = b"tiMe"[-pos:]  # a partial needle at the value start
            elif pos > vlen - 4 and pos < vlen:
                v[pos:] = b"tiMe"[: vlen - pos]  # a partial needle at the value end
            b.add_record(P.Record.new_key_value(b"ti" if pos % 5 == 0 else None, bytes(v)))
        out += b.encode()
        base += 200
    hb = P.Batch(base_offset=base)
    for i in range(20):
        hb.add_record(P.Record.new(("x" * (i * 9) + "tiMe" + "\u00e9" * (i % 2)).encode()))
    out += hb.encode()
    for needle in ["tiMe", "tiMea", "atiMe"]:
        g = gpu_chain(engine, [("filter_init", {"key": needle}, None)])
        check_batch(engine, [("filter_init", {"key": needle}, None)], out)
        g.process_batch(out)
        assert g.last_timings()["eval_path"] == 4


@pytest.mark.parametrize("d", [1, 2, 3])
def test_flat_scan_slice_start_candidate(engine, d):
    """The slice's first aligned dword (the first batch's base offset, big
    endian) equals the needle's 4-gram at offset d: the long-needle candidate
    would start d bytes before the slice.  No occurrence, no read before it."""
    needle =("wvu"[: d] + "ABCD" + "qrstu")[: max(7, d + 4)]
    assert needle[d:d + 4] == "ABCD"
    b = P.Batch(base_offset=0x41424344 << 32)
    for i in range(20):
        b.add_record(P.Record.new(("ABCD" + "z" * i + (needle if i % 3 == 0 else "")).encode()))
    b2 = P.Batch(base_offset=(0x41424344 << 32) + 100)  # two batches: the flat path (one takes k_eval)
    b2.add_record(P.Record.new(needle.encode()))
    sl = b.encode() + b2.encode()
    assert sl[:4] == b"ABCD"
    chain = [("filter_init", {"key": needle}, None)]
    check_batch(engine, chain, sl)
    g = gpu_chain(engine, chain)
    g.process_batch(sl)
    assert g.last_timings()["eval_path"] == 4


@pytest.mark.parametrize("nr", range(2, 9))
def test_keyed_merge_simulated_ranks(engine, nr):
    """The multi-rank branch of fsg_keyed_allreduce (maxn / maxb padding,
    rank-offset arenas, union ids by first occurrence in rank order, dense
    placement per rank) on one GPU: this table is rank `me` of `nr`, the other
    ranks' gathered key lists come from the host (unequal counts, shared and
    disjoint keys, dead entries, empty ranks).  Totals against a host union."""
    import json
    import random
    from fluvio_amd.smartengine import KeyedState
    rng = random.Random(100 + nr)
    pool = ["k%03d" % i for i in range(70)] + ["", "x" * 40, "é"]
    me = rng.randrange(nr)
    local = {}
    ks = KeyedState(engine)
    for c in range(rng.choice([1, 3])):  # this rank's table: chains that never ran (initial accumulators)
        d = {k: rng.randint(0, 2 ** 32 - 1) for k in rng.sample(pool, rng.randint(0, 30))}
        ks.collect(gpu_chain(engine, [("aggregate-json", {}, json.dumps(d).encode())]))
        for k, v in d.items():
            local[k.encode()] = (local.get(k.encode(), 0) + v) & 0xFFFFFFFF
    ranks, expect = [], dict(local)
    for r in range(nr):
        if r == me:
            ranks.append(None)
            continue
        keys = [k.encode() for k in rng.sample(pool, rng.choice([0, 1, 7, 40, 70]))]
        keys = [None if rng.random() < 0.1 else k for k in keys]
        vals = [rng.randint(0, 2 ** 32 - 1) for _ in keys]
        for k, v in zip(keys, vals):
            if k is not None:
                expect[k] = (expect.get(k, 0) + v) & 0xFFFFFFFF
        ranks.append((keys, vals))
    assert ks.allreduce_simulated(me, ranks) == len(expect)
    assert ks.read() == expect


def test_group_process_slices(comm_engine):
    """fsg_chain_group_process_slices: 24 chains in one call (aggregate-json
    partitions whose stream-order walks run as one launch, beside filter,
    aggregate-sum and composed chains, an aggregate-json partition with record
    errors, one with no records), two calls; every chain's output batch and
    accumulator as the oracle has them."""
    from fluvio_amd.smartengine import ResidentSlice, process_slices
    keyed = synth.make_keyed_slices(16, 900, 300)
    cases = []
    for p in range(16):
        acc = b'{"repo-0001": 7, "zz": 1}' if p == 5 else None
        cases.append(([("aggregate-json", {}, acc)], keyed[p]))
    cases.append((CHAINS["filter_init_timeout"], synth.make_slice(2, 500, seed=4)))
    cases.append((CHAINS["agg_sum"], synth.make_slice(3, 2000, seed=5)))
    cases.append(([("aggregate-json", {}, None), ("filter_init", {"key": "repo-000"}, None)], keyed[0]))
    cases.append(([("filter_init", {"key": "repo"}, None), ("aggregate-json", {}, None)], keyed[1]))
    cases.append(([("aggregate-json", {}, None)], P.Batch(base_offset=3).encode()))  # no records
    cases.append(([("aggregate-json", {}, None)], keyed[2]))
    cases.append(([("aggregate-json", {}, None)], _keyed_slice(7, nbatches=8, bad=0.05)))
    cases.append(([("aggregate-json", {}, None)], _keyed_slice(8, nbatches=6)))
    gs = [gpu_chain(comm_engine, m) for m, _ in cases]
    os_ = [orc_chain(m) for m, _ in cases]
    rs = [ResidentSlice(comm_engine, sl) for _, sl in cases]
    for call in range(2):
        outs = process_slices(gs, rs, download=True)
        for i, (m, sl) in enumerate(cases):
            _same_batch(outs[i], os_[i].process_batch(sl))
            if m[-1][0] in ("aggregate-json", "aggregate-sum"):
                assert gs[i].accumulator(len(m) - 1) == os_[i].accumulator(len(m) - 1), (call, i)


# ---------------------------------------------------------------------------
# par_frame (k_eval<kOpsInt / kOpsAll>): batches of more than 128 small records
# framed in parallel (successor^32 by squaring, one lane per 32 records); a
# malformed length, a header count other than the records present, or any
# record whose fields do not tile it leaves the batch to the serial walk
# ---------------------------------------------------------------------------
def _raw_batch(base, raws, count=None):
    h = P.BatchHeader()
    h.last_offset_delta = len(raws) - 1
    body = struct.pack(">hiqqqhi", h.attributes, h.last_offset_delta, h.first_timestamp, h.max_time_stamp,
                       h.producer_id, h.producer_epoch, h.first_sequence)
    recs = struct.pack(">I", len(raws) if count is None else count & 0xFFFFFFFF) + b"".join(raws)
    body += recs
    return struct.pack(">qiibI", base, P.BATCH_HEADER_SIZE + len(recs), h.partition_leader_epoch, h.magic,
                       P.crc32c(body)) + body


def _small_records(rnd, n, bad_value=None, keys=True, hi=99999):
    out = []
    for i in range(n):
        v = str(rnd.randint(-hi, hi)).encode() if rnd.random() < 0.9 else str(rnd.randint(0, 9)).encode()
        if bad_value is not None and i == bad_value:
            v = b"12x"
        k = None if (not keys or rnd.random() < 0.8) else rnd.choice([b"", b"k", b"key7"])
        r = P.Record.new_key_value(k, v)
        r.preamble.offset_delta = i
        out.append(r.encode())
    return out


def _noncanonical_len(raw):
    ln, pos = P.varint_decode(raw, 0)
    z = (ln << 1) & 0xFF  # zigzag of a small non-negative length, one byte
    assert z < 0x80
    return bytes([z | 0x80, 0x00]) + raw[pos:]


def _par_slices():
    rnd = random.Random(5)
    good = b""
    base = 0
    for n in (129, 200, 700, 1000, 1500, 2000):
        good += _raw_batch(base, _small_records(rnd, n))
        base += n + 2
    cases = {"good": good}
    recs = _small_records(rnd, 900)
    r = bytearray(recs[611])  # key tag 2: Record::decode fails ("not valid bool value")
    ln, pos = P.varint_decode(bytes(r), 0)
    i = pos + 1
    _, i = P.varint_decode(bytes(r), i)
    _, i = P.varint_decode(bytes(r), i)
    r[i] = 2
    cases["bad_tag"] = good + _raw_batch(base, recs[:611] + [bytes(r)] + recs[612:])
    recs = _small_records(rnd, 800)
    cases["count_low"] = _raw_batch(0, recs[:400]) + _raw_batch(400, recs, count=799)
    cases["count_high"] = _raw_batch(0, recs[:300]) + _raw_batch(300, recs, count=801)
    recs = _small_records(rnd, 1200)
    cases["noncanonical"] = _raw_batch(0, [_noncanonical_len(x) if j % 97 == 5 else x for j, x in enumerate(recs)])
    cases["parse_error"] = good + _raw_batch(base, _small_records(rnd, 1300, bad_value=1000))
    cases["unkeyed_2300"] = _raw_batch(0, _small_records(rnd, 2300, keys=False))  # beyond the window: serial walk
    short = b""
    for j, n in enumerate((1800, 1500, 1100, 130)):  # resident sections of up to ~1,800 records
        short += _raw_batch(j * 2000, _small_records(rnd, n, keys=False, hi=9 if n > 1500 else 999))
    cases["short"] = short
    return cases


@pytest.mark.parametrize("chain", [
    [("filter_odd", {}, None)],
    [("map_double", {}, None)],
    [("filter_map", {}, None)],
    [("aggregate-sum", {}, b"7")],
    [("filter_with_param", {"key": "1"}, None), ("aggregate-sum", {}, None)],
    [("filter_hashset", {}, None)],
    [("map_double", {}, None), ("filter_map", {}, None)],
    [("regex-filter", {"regex": r"\d"}, None), ("filter_odd", {}, None)],  # k_eval<kOpsAll>
])
def test_par_frame_many_small_records(engine, chain):
    for name, sl in _par_slices().items():
        try:
            check_batch(engine, chain, sl)
        except AssertionError as e:
            raise AssertionError(f"slice {name}: {e}") from e


def _bad_tag_batch(base, n=20, at=7):
    raws = []
    for i in range(n):
        r = P.Record.new_key_value(None, str(i * 3 + 1).encode())
        r.preamble.offset_delta = i
        raws.append(bytearray(r.encode()))
    r = raws[at]  # len, attr, ts, od, then the key tag
    _, i = P.varint_decode(bytes(r), 0)
    i += 1
    _, i = P.varint_decode(bytes(r), i)
    _, i = P.varint_decode(bytes(r), i)
    r[i] = 2
    return _raw_batch(base, [bytes(x) for x in raws])


@pytest.mark.parametrize("chain,kind", [
    ([("aggregate-sum", {}, b"7")], "int"),
    ([("filter_with_param", {"key": "1"}, None), ("aggregate-sum", {}, None)], "int"),
    ([("aggregate", {}, b"A")], "int"),
    ([("aggregate-json", {}, None)], "json"),
    ([("filter_hashset", {}, None)], "int"),
    ([("filter_look_back", {}, None)], "int"),
])
def test_state_kept_before_decode_error(engine, chain, kind):
    """A batch that fails to decode ends process_batch with the error, but the
    calls that completed before it changed the chain's state (the reference's
    batch loop returns at `process(input)?`): the next call sees that state."""
    if kind == "int":
        rnd = random.Random(9)
        good = b"".join(_raw_batch(j * 100, _small_records(rnd, 40, keys=False, hi=500)) for j in range(3))
        later = _raw_batch(1000, _small_records(rnd, 30, keys=False, hi=500))
    else:
        good = _keyed_slice(4, nbatches=5)
        later = _keyed_slice(5, nbatches=3)
    g = gpu_chain(engine, chain)
    o = orc_chain(chain)
    bad = good + _bad_tag_batch(5000)
    oo = o.process_batch(bad, (1 << 64) - 1)
    assert oo["status"] != 0
    with pytest.raises(Exception) as ei:
        g.process_batch(bad, (1 << 64) - 1, SmartModuleChainMetrics())
    assert getattr(ei.value, "code", None) == oo["status"]
    for i, m in enumerate(chain):
        if m[0] in ("aggregate-sum", "aggregate", "aggregate-json"):
            assert g.accumulator(i) == o.accumulator(i)
    gout = g.process_batch(later, (1 << 64) - 1, SmartModuleChainMetrics())
    oo = o.process_batch(later, (1 << 64) - 1)
    assert oo["status"] == 0
    assert gout.raw == oo["bytes"]
    for i, m in enumerate(chain):
        if m[0] in ("aggregate-sum", "aggregate", "aggregate-json"):
            assert g.accumulator(i) == o.accumulator(i)


# ---------------------------------------------------------------------------
# long verbatim records (k_write_lean's staged units and its wave path for
# batches beyond the staging buffer): keys up to 210 B, values of 0..2000 B,
# uppercase maps, offset-delta rebasing across batches with gaps
# ---------------------------------------------------------------------------
def _long_slice(seed, nbatches=50):
    rnd = random.Random(seed)
    words = ["timeout", "level", "warn", "x", "é", "abc", "TIME", "out"]
    out, base = b"", 0
    for bi in range(nbatches):
        b = P.Batch(base_offset=base)
        n = rnd.choice([1, 2, 7, 13, 40, 64, 70])
        for i in range(n):
            if rnd.random() < 0.75:
                size = rnd.randint(128, 2000)
            else:
                size = rnd.randint(0, 127)
            v = ""
            while len(v) < size:
                v += rnd.choice(words) + rnd.choice(["", " ", "-"])
            enc = v.encode()[:size] if rnd.random() < 0.5 else v.encode()
            if bi >= nbatches - 3 and rnd.random() < 0.05:
                enc = enc + b"\xff"  # invalid UTF-8 near the end: the filters' error path
            key = None if rnd.random() < 0.7 else rnd.choice([b"", b"k", b"timeout" * 30])
            r = P.Record.new_key_value(key, enc)
            r.preamble.offset_delta = i
            r.preamble.timestamp_delta = rnd.choice([0, 5, 300, 1 << 20])
            b.records.append(r)
        b.header.last_offset_delta = n - 1
        enc_b = b.encode()
        out += enc_b
        base += n + rnd.choice([0, 0, 1, 100, 5000])
    return out


@pytest.mark.parametrize("chain", [
    [("filter_init", {"key": "timeout"}, None)],
    [("filter_init", {"key": "out"}, None)],
    [("map", {}, None)],
    [("map", {}, None), ("filter_init", {"key": "TIMEOUT"}, None)],
    [],
    [("regex-filter", {"regex": r"warn|x"}, None)],
])
def test_writer_long_records(engine, chain):
    for seed in (1, 2, 3):
        sl = _long_slice(seed)
        check_batch(engine, chain, sl)
        check_batch(engine, chain, sl, max_bytes=len(sl) // 3)


@pytest.mark.parametrize("chain", [
    [("aggregate-sum", {}, b"7")],
    [("aggregate-sum", {}, b" -5 ")],
    [("filter_odd", {}, None)],
    [("map_double", {}, None)],
    [("map_double", {}, None), ("filter_map", {}, None)],
    [("filter_map", {}, None), ("aggregate-sum", {}, None)],
])
def test_int_path_edge_values(engine, chain):
    """k_eval_int on the values its branches special-case, with no deferral:
    '+' signs, -0, the i32 bounds, map_double / the aggregate's sum wrapping,
    and (aggregate-sum alone, which trims) surrounding whitespace; batches of
    more than 128 records, every output record and accumulator vs the oracle."""
    rnd = random.Random(5)
    agg_only = chain[0][0] == "aggregate-sum"
    pool = ["+7", "-0", "0", "2147483647", "-2147483648", "1073741824", "-1073741825", "+0", "-1", "12"]
    if agg_only:
        pool += [" 12\t", "\t-3", "+4 ", "\n2147483647\r", " 0 ", "\x0b9\x0c"]
    sl, base = b"", 0
    for k in range(12):
        n = rnd.choice([129, 200, 300])
        b = P.Batch(base_offset=base)
        for j in range(n):
            b.add_record(P.Record.new(rnd.choice(pool).encode()))
        sl += b.encode()
        base += n
    g = gpu_chain(engine, chain)
    o = orc_chain(chain)
    for _ in range(2):
        gout = g.process_batch(sl)
        oo = o.process_batch(sl, (1 << 64) - 1)
        assert oo["status"] == 0
        assert gout.raw == oo["bytes"]
        t = g.last_timings()
        assert t["eval_path"] == 5 and t["deferred"] == 0, t  # FSG_EVAL_INT
        for i, m in enumerate(chain):
            if m[0] == "aggregate-sum":
                assert g.accumulator(i) == o.accumulator(i)


@pytest.mark.parametrize("chain", [
    [("aggregate-sum", {}, b"7")],
    [("filter_odd", {}, None)],
    [("map_double", {}, None), ("filter_map", {}, None)],
    [("filter_map", {}, None), ("aggregate-sum", {}, None)],
])
def test_int_path_taken_and_exact(engine, chain):
    """k_eval_int (FSG_EVAL_INT) runs for integer chains over many small records:
    the C5 generator's slice (1,000+ decimal records per batch) decides every
    batch there (no deferral) and matches the oracle; a malformed batch in the
    stream is deferred to k_eval and still matches; the slice's record starts
    are computed once and reused by the next call."""
    sl = synth.make_slice(3, 20000, seed=11)
    g = gpu_chain(engine, chain)
    o = orc_chain(chain)
    rs = ResidentSlice(engine, sl)
    for _ in range(2):  # the second call reuses the slice's record starts
        gout = g.process_slice(rs)
        oo = o.process_batch(sl, (1 << 64) - 1)
        assert oo["status"] == 0
        assert gout.raw == oo["bytes"]
        t = g.last_timings()
        assert t["eval_path"] == 5 and t["deferred"] == 0, t  # FSG_EVAL_INT
    for i, m in enumerate(chain):
        if m[0] == "aggregate-sum":
            assert g.accumulator(i) == o.accumulator(i)
    # a batch the lean kernel defers (a non-digit value mid-stream; a key tag of 2 at the end)
    rnd = random.Random(3)
    mixed = sl + _raw_batch(10 ** 6, _small_records(rnd, 900, bad_value=450, hi=999)) + _bad_tag_batch(2 * 10 ** 6)
    check_batch(engine, chain, mixed)


PIPE_CHAINS = ["filter_init_timeout", "regex_ssn", "filter_json", "filter_project_map", "map", "empty"]


def _pipe_slices():
    """Host slices of many 48 KiB chunks: batches straddling chunk ends, a
    batch larger than a chunk (a longer chunk), a leading run of batches no
    filter keeps (the output batch starts in a later chunk), and a tail of
    edge-case records (invalid UTF-8, odd JSON: errors in a late chunk)."""
    logs = synth.make_slice(2, 1500) + synth.make_slice(2, 150, seed=5, base_offset=10_000, max_section=200_000) + \
        synth.make_slice(2, 1500, seed=6, base_offset=20_000)
    ints_first = synth.make_slice(3, 30_000, base_offset=0) + synth.make_slice(2, 1500, seed=8, base_offset=100_000)
    edge_tail = synth.make_slice(2, 2000, seed=9) + synth.make_slice(4, 3000, base_offset=50_000)
    return {"logs": logs, "ints_first": ints_first, "edge_tail": edge_tail}


@pytest.mark.parametrize("name", PIPE_CHAINS)
def test_pipelined_process_batch(engine, monkeypatch, name):
    """fsg_chain_process_batch of a host slice larger than two chunks runs
    pipelined (upload of piece k+1, processing of chunk k and download of chunk
    k-1 overlap; chunk k > 0 continues the output batch an earlier chunk
    started, the CRC32C combined on the host): the output batch, its header,
    error and metrics equal the oracle's process_batch of the whole slice, for
    an unlimited max_bytes and cuts in the first and in a later chunk."""
    monkeypatch.setenv("FSG_PIPE_CHUNK", str(48 << 10))  # read when the chain is built
    for key, sl in _pipe_slices().items():
        for max_bytes in ((1 << 64) - 1, len(sl) // 3, 5000):
            check_batch(engine, CHAINS[name], sl, max_bytes=max_bytes)
        g = gpu_chain(engine, CHAINS[name])
        try:
            g.process_batch(sl)
        except Exception:  # noqa: BLE001 (a status error: check_batch compared it)
            continue
        assert g.last_timings()["chunks"] >= 1, key
    g = gpu_chain(engine, CHAINS[name])
    g.process_batch(_pipe_slices()["logs"])
    assert g.last_timings()["chunks"] > 4


def test_filter_json_deeply_nested_ignored_values(engine):
    """serde_json skips a field StructuredLog does not name with ignore_value,
    whose frame stack is a Vec with no depth limit (de.rs): on the GPU the
    exact kernel keeps 256 levels of frames in registers (the round-5 stack had
    64), so an ignored value nested 65..256 deep is decided like the oracle's
    restatement (and its syntax errors found at the same position)."""
    b = P.Batch()
    for depth in (1, 63, 64, 65, 100, 128, 129, 200, 255, 256):
        for opener, closer in (("[", "]"), ('{"a":', "}")):
            inner = "1" if opener == "[" else "2"
            v = '{"level":"warn","extra":' + opener * depth + inner + closer * depth + ',"message":"m"}'
            b.add_record(P.Record.new(v.encode()))
    for depth in (70, 250):  # unbalanced: the EOF / comma errors at the same byte
        b.add_record(P.Record.new(('{"level":"error","x":' + "[" * depth + "1" + "]" * (depth - 1) + "}").encode()))
    sl = b.encode()
    check_batch(engine, CHAINS["filter_json"], sl)
    # one record per batch, so each error stops only its own call
    for depth in (65, 256):
        check_batch(engine, CHAINS["filter_json"], _one_record_slice(
            ('{"level":"info","extra":' + "[" * depth + "]" * depth + "}").encode()))
