"""Writes tests/golden/kats.json: known-answer vectors for the SmartModule path.

Every EXPECTED value below is transcribed from an assertion in the reference's
own tests (file:line cited next to it, paths relative to /root/reference), or
from the output of the reference's compiled guest recorded in SURVEY.md §8c.
The INPUT bytes are built here with the host codec (fluvio_amd/protocol.py) to
reproduce the inputs those tests construct (BatchProducer, Record::new, ...).
Nothing here is computed by the oracle or by the product.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from fluvio_amd.protocol import (Batch, BatchHeader, Record, encode_records)  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "kats.json")


def recs(values, offset_deltas=True):
    rs = [Record.new(v) for v in values]
    if offset_deltas:
        for i, r in enumerate(rs):
            r.preamble.offset_delta = i
    return rs


def producer_batch(base_offset, values, producer_id=0, ts_delta=False):
    """fluvio-protocol/src/fixture.rs:42-54 (BatchProducer::generate_batch), with the
    base offset assigned by the replica on write (offsets are consecutive)."""
    b = Batch(base_offset=base_offset, header=BatchHeader(magic=2, producer_id=producer_id,
                                                         producer_epoch=-1))
    for i, v in enumerate(values):
        r = Record.new(v)
        if ts_delta:
            r.preamble.timestamp_delta = i
        b.add_record(r)
    return b.encode()


def filter_values(n):
    """fluvio-spu/src/services/public/tests/mod.rs:25-45 (create_filter_records)."""
    return [("b" * 100 if i == 0 else "a" * 100 if i == 1 else "z" * 100) for i in range(n)]


def main():
    k = {}
    k["varint"] = {
        "source": "crates/fluvio-protocol/src/core/varint.rs:93-103,126-136",
        "cases": [[0, "00"], [-1, "01"], [1, "02"], [63, "7e"], [7, "0e"], [10, "14"], [4, "08"],
                  [8191, "fe7f"], [-134217729, "8180808001"]],
    }
    k["record_dog"] = {
        "source": "crates/fluvio-protocol/src/record/data.rs:653-666",
        "bytes": bytes([0x12, 0x0, 0x0, 0x2, 0x0, 0x6, 0x64, 0x6F, 0x67, 0x0]).hex(),
        "offset_delta": 1, "value": "dog", "write_size": 10,
    }
    # batch.rs:548-575: one record "test" pushed directly (last_offset_delta stays -1)
    b = Batch(header=BatchHeader(first_timestamp=1555478494747, max_time_stamp=1555478494747))
    b.records.append(Record.new(b"test"))
    b2 = Batch(header=BatchHeader(first_timestamp=1555478494747, max_time_stamp=1555478494747))
    b2.records.append(Record.new(b"test"))
    b2.header.attributes |= 0x10
    b2.schema_id = 42
    k["crc"] = {
        "source": "crates/fluvio-protocol/src/record/batch.rs:574,627",
        "cases": [{"batch": b.encode().hex(), "crc": 1430948200},
                  {"batch": b2.encode().hex(), "crc": 2943551365}],
    }
    k["produce_records"] = {
        "source": "crates/fluvio-spu/src/smartengine/produce_batch.rs:124,128",
        "cases": [{"records": encode_records(recs(["soup"])).hex(),
                   "expect": b"\0\0\0\x01\x14\0\0\0\0\x08soup\0".hex()},
                  {"records": encode_records(recs(["fries"])).hex(),
                   "expect": b"\0\0\0\x01\x16\0\0\0\0\nfries\0".hex()}],
    }

    # --- SmartModuleChainInstance::process cases (SmartEngine unit tests) -----
    chain = []

    def case(name, source, modules, calls):
        chain.append({"name": name, "source": source, "modules": modules, "calls": calls})

    # inputs are SmartModuleInput::try_from_records(vec![Record::new(..)]) -> offset_delta 0
    case("filter", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/filter.rs:37-58",
         [["filter", {}, None]],
         [{"values": ["hello world"], "expect": []},
          {"values": ["apple", "fruit"], "expect": ["apple"]}])
    case("map", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/map.rs:18-41",
         [["map", {}, None]],
         [{"values": ["apple", "fruit"], "expect": ["APPLE", "FRUIT"]}])
    case("filter_map", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/filter_map.rs:21-43",
         [["filter_map", {}, None]],
         [{"values": ["10", "11"], "expect": ["5"]}])
    case("chain_filter_map", "crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:259-311",
         [["filter_init", {"key": "a"}, None], ["map", {}, None]],
         [{"values": ["hello world"], "expect": []},
          {"values": ["apple", "fruit", "banana"], "expect": ["APPLE", "BANANA"]}])
    case("chain_filter_aggregate", "crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:315-384",
         [["filter_init", {"key": "a"}, None], ["aggregate", {}, "zero"]],
         [{"values": ["apple", "fruit", "banana"], "expect": ["zeroapple", "zeroapplebanana"]},
          {"values": ["nothing"], "expect": []},
          {"values": ["elephant"], "expect": ["zeroapplebananaelephant"]}])
    case("aggregate_ok", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/aggregate.rs:124-221",
         [["aggregate", {}, None]],
         [{"values": ["a"], "expect": ["a"], "acc": "a"},
          {"values": ["b"], "expect": ["ab"], "acc": "ab"},
          {"values": [], "expect": [], "acc": "ab"},
          {"values": ["c"], "expect": ["abc"]}])
    case("aggregate_with_initial", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/aggregate.rs:223-255",
         [["aggregate", {}, "a"]],
         [{"values": ["b"], "expect": ["ab"]}])
    case("array_map", "crates/fluvio-smartengine/src/engine/wasmtime/transforms/array_map.rs:41-52",
         [["array_map_json_array", {}, None]],
         [{"values": ['["Apple","Banana","Cranberry"]'], "expect": ['"Apple"', '"Banana"', '"Cranberry"']}])
    case("empty_chain", "crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:477-498",
         [], [{"values": ["input"], "expect": ["input"]}])
    k["chain"] = chain
    k["init_errors"] = [
        {"source": "crates/fluvio-smartengine/src/engine/wasmtime/transforms/filter.rs:62-81",
         "module": "filter_init", "params": {}, "message": "Missing param key\n\nSmartModule Init Error: \n"},
        {"source": "smartmodule/regex-filter/src/lib.rs:13-22",
         "module": "regex-filter", "params": {}, "message": "Missing param regex\n\nSmartModule Init Error: \n"},
    ]

    # --- reference guest output recorded in SURVEY.md §8c (compiled reference
    # fixture crates/fluvio-smartmodule/fixtures/smartmodule.wasm = contains('a'))
    k["survey_guest"] = {
        "source": "SURVEY.md §8c (reference compiled guest, recorded during the survey)",
        "module": "filter",
        "ok": {"values": ["apple", "fruit", "banana", "hello world"], "base_offset": 0,
               "expect_successes": "0000000216000000000a6170706c650018000004000c62616e616e6100",
               "expect_error_tag": "00"},
        "utf8": {"values_hex": ["6170706c65", "ff61"], "base_offset": 100,
                 "expect_values": ["apple"],
                 "error": {"hint": "invalid utf-8 sequence of 1 bytes from index 0", "offset": 101,
                           "kind": 0, "key": None, "value": "ff61"}},
    }

    # --- SPU process_batch over stored batches ----------------------------
    spu = []
    # stream_fetch.rs:441-476: 2 filter records at offset 0 -> 1 record, offset_delta 1
    s1 = producer_batch(0, filter_values(2))
    spu.append({"name": "filter_first_fetch",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:441-476",
                "modules": [["filter", {}, None]], "slice": s1.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 1, "values": ["a" * 100],
                           "offset_deltas": [1]}})
    # stream_fetch.rs:480-537: fetch from offset 2 over [raw(2)@2, filter(3)@4, filter(3)@7]
    s2 = (producer_batch(2, [bytes([10, 20])] * 2, producer_id=12) + producer_batch(4, filter_values(3))
          + producer_batch(7, filter_values(3)))
    spu.append({"name": "filter_across_batches",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:480-537",
                "modules": [["filter", {}, None]], "slice": s2.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 4, "n_records": 2, "values": ["a" * 100, "a" * 100],
                           "next_offset": 10}})
    # stream_fetch.rs:839-969: three batches of 10 filter records, max_bytes 250
    s3 = b"".join(producer_batch(10 * i, filter_values(10)) for i in range(3))
    spu.append({"name": "filter_max_bytes",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:870-920",
                "modules": [["filter", {}, None]], "slice": s3.hex(), "max_bytes": 250,
                "expect": {"base_offset": 0, "n_records": 2, "values": ["a" * 100, "a" * 100],
                           "next_offset": 20}})
    s3b = producer_batch(20, filter_values(10))
    spu.append({"name": "filter_max_bytes_second_fetch",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:922-960",
                "modules": [["filter", {}, None]], "slice": s3b.hex(), "max_bytes": 250,
                "expect": {"base_offset": 20, "n_records": 1, "values": ["a" * 100],
                           "next_offset": 30}})
    # stream_fetch.rs:704-803: filter_odd over "0".."9","ten" -> 5 records + error at offset 10
    s4 = producer_batch(0, [str(i) for i in range(10)] + ["ten"])
    spu.append({"name": "filter_odd_error",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:744-795",
                "modules": [["filter_odd", {}, None]], "slice": s4.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 5, "values": ["0", "2", "4", "6", "8"],
                           "error": {"offset": 10, "key": None, "value": "ten", "kind": 0,
                                     "hint": "Oops something went wrong\n\nCaused by:\n   0: Failed to parse int\n   1: invalid digit found in string"}}})
    # stream_fetch.rs:1438-1530: aggregate (concat, initial "A") over "0".."4"
    s5 = producer_batch(0, [str(i) for i in range(5)])
    spu.append({"name": "aggregate_single_batch",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:1481-1528",
                "modules": [["aggregate", {}, "A"]], "slice": s5.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 5,
                           "values": ["A0", "A01", "A012", "A0123", "A01234"]}})
    # stream_fetch.rs:1551-1709: aggregate over two batches "0".."2" @0 and "3".."5" @3
    s5b = producer_batch(0, ["0", "1", "2"]) + producer_batch(3, ["3", "4", "5"])
    spu.append({"name": "aggregate_multi_batch",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:1672-1693",
                "modules": [["aggregate", {}, "A"]], "slice": s5b.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 6, "next_offset": 6,
                           "values": ["A0", "A01", "A012", "A0123", "A01234", "A012345"]}})
    # stream_fetch.rs:1933-2020: filter_map over 11,22,33,44,55 -> "11","22"
    s6 = producer_batch(0, ["11", "22", "33", "44", "55"])
    spu.append({"name": "filter_map",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:1933-2020",
                "modules": [["filter_map", {}, None]], "slice": s6.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 2, "values": ["11", "22"]}})
    # stream_fetch.rs:1838-1893: one record serde_json::to_string(&(0..10)) -> "0".."9"
    s7 = producer_batch(0, ["[0,1,2,3,4,5,6,7,8,9]"])
    spu.append({"name": "array_map_ints",
                "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:1838-1893",
                "modules": [["array_map_json_array", {}, None]], "slice": s7.hex(), "max_bytes": 10000,
                "expect": {"base_offset": 0, "n_records": 10, "values": [str(i) for i in range(10)]}})
    k["process_batch"] = spu

    # serde / serde_json error texts asserted by the reference's own tests (the
    # JSON-field filter's error hints are serde_json::Error Display strings)
    k["serde_json"] = [
        {"name": "missing_field_position",
         "source": "crates/fluvio-version-manager/src/common/manifest.rs:88-101 (serde_json::from_str)",
         "input": '{\n"foo": "bar",\n"hello": "world"\n}', "struct": "VersionManifest",
         "fields": ["channel=stable|latest", "version"],
         "expect": "missing field `channel` at line 4 column 1", "match": "exact"},
        {"name": "unknown_variant_one_of",
         "source": "crates/fluvio-connector-package/src/config/mod.rs:738-742 (serde::de::Error::unknown_variant)",
         "input": '{"compression":"gzipaoeu"}', "struct": "ProducerParameters",
         "fields": ["compression=none|gzip|snappy|lz4|zstd"],
         "expect": "unknown variant `gzipaoeu`, expected one of `none`, `gzip`, `snappy`, `lz4`, `zstd`",
         "match": "prefix"},
        {"name": "unexpected_string_debug",
         "source": "crates/fluvio-connector-package/src/config/mod.rs:746-750 (serde::de::Unexpected::Str)",
         "input": '"1aoeu"', "struct": "Batch", "fields": ["size"],
         "expect": 'string "1aoeu"', "match": "contains"},
    ]

    # stateful filters with look_back (f4).  A "chain" step list runs on one
    # chain instance: look_back over the given records (Lookback::Last(n) read by
    # the SPU from the replica's last n records), process of one input, or
    # "new_chain" (the SPU builds a new SmartModuleContext per produce request /
    # stream, and a recreated replica re-runs look_back).
    lb = []
    lb.append({"name": "chain_filter_look_back",
               "source": "crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:388-428",
               "module": ["filter_look_back", {}], "lookback": ["last", 1, 0],
               "steps": [{"look_back": ["2"]}, {"process": ["1", "2", "3"], "expect": ["3"]}],
               "invocation_count": 2})
    lb.append({"name": "chain_filter_look_back_error_propagated",
               "source": "crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:433-470",
               "module": ["filter_look_back", {}], "lookback": ["last", 1, 0],
               "steps": [{"look_back": ["wrong str"],
                          "error": {"hint": "invalid digit found in string", "offset": 0, "key": None,
                                    "value": "wrong str"}}],
               "invocation_count": 1})
    lb.append({"name": "bounded_hash_set",
               "source": "smartmodule/examples/filter_hashset/src/lib.rs:83-104 (test_set, limit 3)",
               "module": ["filter_hashset", {"count": "3"}], "lookback": None,
               "steps": [{"process": ["1", "3", "2", "3", "1", "5", "1"], "expect": ["1", "3", "2", "5", "1"]}]})
    # produce.rs:522-700: a chain per produce request, look_back over the replica's last record
    stored = []
    steps = []
    for vals, last, exp in [(["1", "2", "3"], 1, ["1", "2", "3"]), (["1", "2", "3", "4", "5"], 1, ["4", "5"]),
                            (["1", "2"], 0, ["1", "2"]), (["1", "2"], None, ["1", "2"])]:
        steps.append({"new_chain": None if last is None else ["last", last, 0]})
        if last is not None:
            steps.append({"look_back": stored[len(stored) - last:] if last else []})
        steps.append({"process": vals, "expect": exp})
        stored += exp
    assert stored == ["1", "2", "3", "4", "5", "1", "2", "1", "2"]  # produce.rs:656-700
    lb.append({"name": "produce_basic_with_lookback",
               "source": "crates/fluvio-spu/src/services/public/tests/produce.rs:522-700",
               "module": ["filter_look_back", {}], "lookback": ["last", 1, 0], "steps": steps})
    # produce.rs:840-1020: dedup (filter_hashset, count 6, Lookback::Last(6)) built once per
    # replica with look_back at init (replica_state.rs:391-406); the replica is recreated once
    stored = []
    steps = [{"look_back": []}]
    for vals, exp in [(["1", "2", "3", "1"], ["1", "2", "3"]), (["1", "2", "4", "5", "6"], ["4", "5", "6"]),
                      (["7", "1", "2"], ["7", "1", "2"])]:
        steps.append({"process": vals, "expect": exp})
        stored += exp
    steps.append({"new_chain": ["last", 6, 0]})
    steps.append({"look_back": stored[-6:]})
    steps.append({"process": ["7", "8"], "expect": ["8"]})
    stored += ["8"]
    assert stored == ["1", "2", "3", "4", "5", "6", "7", "1", "2", "8"]  # produce.rs:1014-1018
    lb.append({"name": "produce_with_deduplication",
               "source": "crates/fluvio-spu/src/services/public/tests/produce.rs:840-1020",
               "module": ["filter_hashset", {"count": "6"}], "lookback": ["last", 6, 0], "steps": steps})
    # stream_fetch.rs:2483-2605: a stream per fetch, look_back over the last record
    steps = [{"look_back": ["3"]}, {"process": ["1", "10", "2", "11", "3"], "expect": ["10", "11"]},
             {"new_chain": ["last", 1, 0]}, {"look_back": ["13"]},
             {"process": ["1", "10", "2", "11", "3", "10", "14", "13"], "expect": ["14"]},
             {"new_chain": ["last", 0, 0]}, {"look_back": []},
             {"process": ["1", "10", "2", "11", "3", "10", "14", "13"], "expect": ["1", "10", "11", "14"]}]
    lb.append({"name": "stream_fetch_filter_lookback",
               "source": "crates/fluvio-spu/src/services/public/tests/stream_fetch.rs:2483-2605",
               "module": ["filter_look_back", {}], "lookback": ["last", 1, 0], "steps": steps})
    k["look_back"] = lb

    with open(OUT, "w") as f:
        json.dump(k, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
