"""Pins the CPU oracle (oracle/) against the reference's own known answers
(tests/golden/kats.json, every expected value cited to a reference test).

CPU only: no GPU, no product library involved.
"""
import re
import struct

import pytest

from fluvio_amd import protocol as P
from oracle import oracle as O


def _vals(raw):
    return [r.value for r in P.decode_records(raw)]


def test_varint_table(kats):
    for v, hx in kats["varint"]["cases"]:
        assert O.varint_encode(v).hex() == hx
        assert P.varint_encode(v).hex() == hx
        assert P.varint_decode(bytes.fromhex(hx)) == (v, len(hx) // 2)


def test_record_dog(kats):
    k = kats["record_dog"]
    raw = bytes.fromhex(k["bytes"])
    recs = P.decode_records(struct.pack(">I", 1) + raw)
    assert recs[0].preamble.offset_delta == k["offset_delta"]
    assert recs[0].value == k["value"].encode()
    assert recs[0].write_size() == k["write_size"]
    # oracle decode -> encode round trip through the empty chain
    out = O.OracleChain().process(struct.pack(">I", 1) + raw)
    assert out["bytes"] == struct.pack(">I", 1) + raw


def test_crc_kats(kats):
    for c in kats["crc"]["cases"]:
        b = bytes.fromhex(c["batch"])
        crc_field = struct.unpack(">I", b[17:21])[0]
        assert crc_field == c["crc"]  # host codec reproduces the KAT
        assert O.crc32c(b[21:]) == c["crc"]  # oracle CRC over attributes..records


def test_produce_records(kats):
    for c in kats["produce_records"]["cases"]:
        assert c["records"] == c["expect"]
        out = O.OracleChain().process(bytes.fromhex(c["records"]))
        assert out["bytes"].hex() == c["expect"]


def _records_input(values, base_offset=0):
    return P.encode_records([P.Record.new(v) for v in values])


@pytest.mark.parametrize("case_idx", range(9))
def test_chain_cases(kats, case_idx):
    case = kats["chain"][case_idx]
    chain = O.OracleChain([(m, p, a.encode() if a is not None else None)
                           for m, p, a in case["modules"]])
    agg_stage = next((i for i, m in enumerate(case["modules"]) if m[0].startswith("aggregate")), None)
    for call in case["calls"]:
        out = chain.process(_records_input(call["values"]))
        assert out["status"] == 0
        assert out["error"] is None
        assert _vals(out["bytes"]) == [v.encode() for v in call["expect"]], case["name"]
        if "acc" in call:
            assert chain.accumulator(agg_stage) == call["acc"].encode()


def test_init_errors(kats):
    for c in kats["init_errors"]:
        with pytest.raises(O.OracleError) as e:
            O.OracleChain([(c["module"], c["params"], None)])
        assert e.value.status == -2
        assert e.value.message == c["message"]


def test_survey_guest_vectors(kats):
    g = kats["survey_guest"]
    ok = g["ok"]
    recs = [P.Record.new(v) for v in ok["values"]]
    for i, r in enumerate(recs):
        r.preamble.offset_delta = i
    out = O.OracleChain([(g["module"], {}, None)]).process(P.encode_records(recs), ok["base_offset"])
    assert out["bytes"].hex() == ok["expect_successes"]
    assert out["error"] is None
    u = g["utf8"]
    recs = [P.Record.new(bytes.fromhex(v)) for v in u["values_hex"]]
    for i, r in enumerate(recs):
        r.preamble.offset_delta = i
    out = O.OracleChain([(g["module"], {}, None)]).process(P.encode_records(recs), u["base_offset"])
    assert _vals(out["bytes"]) == [v.encode() for v in u["expect_values"]]
    e = out["error"]
    assert e["hint"] == u["error"]["hint"]
    assert e["offset"] == u["error"]["offset"]
    assert e["kind"] == u["error"]["kind"]
    assert e["key"] is None
    assert e["value"].hex() == u["error"]["value"]


def test_process_batch_cases(kats):
    for case in kats["process_batch"]:
        chain = O.OracleChain([(m, p, a.encode() if a is not None else None)
                               for m, p, a in case["modules"]])
        out = chain.process_batch(bytes.fromhex(case["slice"]), case["max_bytes"])
        exp = case["expect"]
        assert out["status"] == 0, case["name"]
        b, end = P.decode_batch(out["bytes"])
        assert end == len(out["bytes"])
        assert b.base_offset == exp["base_offset"], case["name"]
        recs = b.memory_records()
        assert len(recs) == exp["n_records"], case["name"]
        assert [r.value for r in recs] == [v.encode() for v in exp["values"]], case["name"]
        if "offset_deltas" in exp:
            assert [r.preamble.offset_delta for r in recs] == exp["offset_deltas"]
        if "next_offset" in exp:
            # stream_fetch.rs:487-492: next_filter_offset = base_offset + last_offset_delta + 1
            assert b.base_offset + b.header.last_offset_delta + 1 == exp["next_offset"], case["name"]
        # CRC is over attributes..records and batch_len matches
        assert b.header.crc == P.crc32c(out["bytes"][21:])
        assert b.batch_len == len(out["bytes"]) - 12
        if "error" in exp:
            e = out["error"]
            assert e is not None
            for f in ("offset", "kind", "hint"):
                assert e[f] == exp["error"][f], (case["name"], f)
            assert e["key"] is None
            assert e["value"] == exp["error"]["value"].encode()
        else:
            assert out["error"] is None


@pytest.mark.parametrize("pattern,texts", [
    (r"\d{3}-\d{2}-\d{4}", ["my ssn is 123-45-6789 ok", "123-45-678", "x1234-56-78901", "", "12-345-6789"]),
    (r"[A-Z]", ["AA", "aa", "a1b2", "zZ"]),
    (r"^ab|cd$", ["abx", "xab", "xcd", "cdx", "ab", ""]),
    (r"a(b|c)*d", ["ad", "abcbd", "abxd", "zzabbbbbccd"]),
    (r"colou?r\s+\w+", ["color red", "colour  blue", "colr x", "color"]),
    (r"[^a-c]x", ["ax", "dx", "x", "abcx"]),
    (r"a.c", ["abc", "a\nc", "aéc", "ac"]),
    (r"x{2,3}y", ["xy", "xxy", "xxxxy"]),
    (r"", ["", "anything"]),
    # word boundaries (ASCII text: Unicode \b and Python's agree), inline flags, \A / \z
    (r"\bfoo\b", ["a foo b", "afoo b", "foo", "foo_", "(foo)", ""]),
    (r"\Bar\B", ["bars", "ar", "bar", "xarx"]),
    (r"\b", ["", " ", "a"]),
    (r"x\b|\by", ["x", "xa", "ay", "a y"]),
    (r"(?i)timeout", ["TimeOut", "TIMEOUT", "time out", "timeouts"]),
    (r"(?i)[a-f]{2}\d", ["AB1", "aB2", "ag3"]),
    (r"(?i:ab)c", ["ABc", "abC", "aBc"]),
    (r"(?i)[^k]", ["K", "k", "x"]),
    (r"(?i)sk", ["SK", "\u017fK", "s\u212a", "sx"]),
    (r"(?s)a.b", ["a\nb", "axb"]),
    (r"\Aab", ["ab", "xab"]),
])
def test_regex_oracle_vs_python_re(pattern, texts):
    """Cross-check the oracle's regex engine with Python's independent `re` on
    inputs where Rust regex and Python re agree (no `$` before a trailing \\n,
    ASCII \\w).  Pins the restatement of regex is_match (third-party crate
    regex 1.6.0/1.8.1, absent from /root/reference)."""
    for t in texts:
        py = pattern.replace(r"\z", r"\Z")
        assert O.regex_is_match(pattern, t.encode()) == (re.search(py, t) is not None), (pattern, t)


def test_regex_unicode_classes():
    # \d is Unicode Nd in Rust regex (Arabic-Indic digits match), '.' is a scalar value
    assert O.regex_is_match(r"\d\d\d", "١٢٣".encode())
    assert O.regex_is_match(r"^.$", "é".encode())
    assert not O.regex_is_match(r"^..$", "é".encode())
    assert O.regex_is_match(r"\s", "a　b".encode())


def test_look_back_kats(kats):
    """filter_look_back / filter_hashset with look_back: engine.rs:388-470,
    filter_hashset test_set, SPU produce.rs:522-1020, stream_fetch.rs:2483-2605."""
    from tests.lookback_steps import run_lookback_case

    def new_chain(lb):
        return O.OracleChain([tuple(case["module"]) + (None,)])

    def look_back(ch, values):
        r = ch.look_back(0, P.encode_records([P.Record.new(v) for v in values]))
        assert r["status"] == 0
        return r["error"], r["metrics"]["invocation_count"]

    def process(ch, values):
        r = ch.process(P.encode_records([P.Record.new(v) for v in values]))
        assert r["status"] == 0 and r["error"] is None
        return _vals(r["bytes"]), r["metrics"]["invocation_count"]

    assert len(kats["look_back"]) >= 6
    for case in kats["look_back"]:
        run_lookback_case(case, new_chain, look_back, process)


def test_hashset_init_count_param():
    with pytest.raises(O.OracleError) as e:
        O.OracleChain([("filter_hashset", {"count": "many"}, None)])
    assert e.value.message == "invalid digit found in string\n\nSmartModule Init Error: \n"
    O.OracleChain([("filter_hashset", {"count": "+7"}, None)])  # usize::from_str takes a leading '+'
    with pytest.raises(O.OracleError):
        O.OracleChain([("filter_hashset", {"count": "4294967296"}, None)])  # usize is u32 on wasm32


def test_regex_posix_classes():
    """[[:name:]] ASCII classes (regex-syntax ClassAsciiKind; Python re has none)."""
    m = lambda p, t: O.regex_is_match(p, t.encode())  # noqa: E731
    assert m(r"^[[:digit:]]{3}$", "123") and not m(r"^[[:digit:]]{3}$", "12a")
    assert m(r"[[:^alpha:]]", "ab1") and not m(r"[[:^alpha:]]", "abc")
    assert m(r"^[[:xdigit:][:space:]]+$", "fF 09\t") and not m(r"^[[:xdigit:]]+$", "fg")
    assert m(r"[[:punct:]]", "a,b") and not m(r"[[:punct:]]", "ab")
    assert m(r"(?i)^[[:upper:]]+$", "abC") and not m(r"^[[:upper:]]+$", "abC")
