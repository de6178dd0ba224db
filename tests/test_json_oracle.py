"""The serde_json restatement in oracle/fsg_json.c (test infrastructure):
pinned by the serde / serde_json error texts the reference's own tests assert,
and cross-checked against Python's independent `json` parser on the
accept/reject decision and the decoded level (error *texts* beyond the pinned
fixtures follow serde_json 1.0.96's source)."""
import json

import pytest

from oracle import oracle as O
from tests import jsongen

LEVELS = jsongen.LEVELS


def test_reference_serde_fixtures(kats):
    for case in kats["serde_json"]:
        st, msg = O.json_struct(case["input"].encode(), case["struct"], case["fields"])
        assert st == "err", case["name"]
        if case["match"] == "exact":
            assert msg == case["expect"], case["name"]
        elif case["match"] == "prefix":
            assert msg.startswith(case["expect"]), (case["name"], msg)
        else:
            assert case["expect"] in msg, (case["name"], msg)


class Pairs(list):
    pass


def _lone_surrogate(s):
    return isinstance(s, str) and any(0xD800 <= ord(c) <= 0xDFFF for c in s)


def _level(v):
    """LogLevel from a decoded JSON value: index, or None (error), or 'skip'."""
    if isinstance(v, str):
        if _lone_surrogate(v):
            return "skip"
        return LEVELS.index(v) if v in LEVELS else None
    if isinstance(v, Pairs):  # {"variant": null}
        if len(v) != 1:
            return None
        k, x = v[0]
        if _lone_surrogate(k):
            return "skip"
        return LEVELS.index(k) if (k in LEVELS and x is None) else None
    return None


def python_verdict(doc: bytes):
    """("ok", level) / ("err",) by Python's json, or None where the two libraries'
    rules differ by design (non-ASCII, lone surrogates, NaN/Infinity)."""
    if any(b >= 0x80 for b in doc) or b"NaN" in doc or b"Infinity" in doc:
        return None
    try:
        v = json.loads(doc, object_pairs_hook=Pairs)
    except RecursionError:
        return None
    except ValueError:
        return ("err",)
    if isinstance(v, Pairs):
        seen = {}
        for k, x in v:
            if _lone_surrogate(k):
                return None
            if k in ("level", "message"):
                if k in seen:
                    return ("err",)  # duplicate field
                seen[k] = x
        if "level" not in seen or "message" not in seen:
            return ("err",)
        lv, msg = _level(seen["level"]), seen["message"]
    elif isinstance(v, list):
        if len(v) != 2:
            return ("err",)
        lv, msg = _level(v[0]), v[1]
    else:
        return ("err",)
    if lv == "skip" or _lone_surrogate(msg):
        return None
    if lv is None or not isinstance(msg, str):
        return ("err",)
    return ("ok", lv)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_python_json(seed):
    checked = 0
    for doc in jsongen.corpus(seed, 300, 900):
        pv = python_verdict(doc)
        if pv is None:
            continue
        try:
            ov = O.json_structured_log(doc)
        except O.OracleError:
            continue  # outside the restatement (float / Debug-escaped text)
        assert ov[0] == pv[0], (doc, ov, pv)
        if pv[0] == "ok":
            assert ov[1] == pv[1], (doc, ov, pv)
        checked += 1
    assert checked > 900


def test_oracle_error_texts():
    """serde_json Display strings for the error kinds (positions as serde_json's
    position_of_index of the reader index when the error is raised)."""
    cases = {
        b'': "EOF while parsing a value at line 1 column 0",
        b'{"level":"info"}': "missing field `message` at line 1 column 16",
        b'{"level":"info","level":"warn","message":"x"}': "duplicate field `level` at line 1 column 23",
        b'["warn"]': "invalid length 1, expected struct StructuredLog with 2 elements at line 1 column 8",
        b'{"level":"INFO","message":"m"}':
            "unknown variant `INFO`, expected one of `debug`, `info`, `warn`, `error` at line 1 column 15",
        b'"hello"': 'invalid type: string "hello", expected struct StructuredLog at line 1 column 7',
        b'{"level":"info","message":5}': "invalid type: integer `5`, expected a string at line 1 column 27",
        b'{"level":"info","message":"x"} x': "trailing characters at line 1 column 32",
        b'{"level":"info","message":"x",}': "trailing comma at line 1 column 31",
        b'\n\n  {"level"\n:\n"info"}': "missing field `message` at line 5 column 7",
        # a NUL in the text (the raw variant string): carried with its length
        b'{"level":"in\\u0000fo","message":"m"}':
            "unknown variant `in\x00fo`, expected one of `debug`, `info`, `warn`, `error` at line 1 column 21",
    }
    for doc, want in cases.items():
        assert O.json_structured_log(doc) == ("err", want), doc


# strings serde reports with Rust's str Debug ("invalid type: string ...")
DEBUG_STRINGS = ["tab\there", "esc\x1b[31m", "del\x7f", "bel\u0007", "nul\u0000x", "caf\u00e9", "na\u0301x",
                 "zwj\u200dx", "nbsp\u00a0x", "ls\u2028x", "shy\u00adx", "pua\ue000", "nonchar\uffff",
                 "last\U0010ffff", "emoji\U0001f600", "quote'\"s", "back\\slash", "\u0300lead", "cjk\u4e2d",
                 "arabic\u0645\u0631\u062d\u0628\u0627", "vs\ufe0f", "tag\U000e0041", "\u0085nel"]


def _rust_str_debug(s):
    """<str as Debug>::fmt restated from its documented rules (Rust 1.75
    core::fmt / char::escape_debug_ext): independent of the oracle's C."""
    import unicodedata
    import regex
    out = ['"']
    for ch in s:
        cp = ord(ch)
        esc = {0: "\\0", 9: "\\t", 10: "\\n", 13: "\\r", 0x5C: "\\\\", 0x22: '\\"'}.get(cp)
        cat = unicodedata.category(ch)
        if esc is not None:
            out.append(esc)
        elif (cat != "Cn" and regex.match(r"\p{Grapheme_Extend}", ch)) or \
                (cat in ("Cc", "Cf", "Cs", "Co", "Cn", "Zl", "Zp", "Zs") and ch != " "):
            out.append("\\u{%x}" % cp)
        else:
            out.append(ch)
    return "".join(out) + '"'


def test_oracle_string_debug_texts():
    """serde's Unexpected::Str through Rust's str Debug: control, format,
    separator, private-use and unassigned chars and combining marks as
    \\u{..}; printable non-ASCII as is (parity unpinned: no reference fixture;
    checked against a separate restatement of the rules)."""
    import json as _json
    for s, ascii_only in [(s, a) for s in DEBUG_STRINGS for a in (True, False)]:
        doc = _json.dumps(s, ensure_ascii=ascii_only).encode()  # \\u escapes, or raw UTF-8
        col = len(doc)
        want = "invalid type: string %s, expected struct StructuredLog at line 1 column %d" % (_rust_str_debug(s), col)
        got = O.json_structured_log(doc)
        assert got == ("err", want), (s, got, want)


# ---------------------------------------------------------------------------
# array_map_json_array: from_slice::<Vec<Value>> + to_string per element
# ---------------------------------------------------------------------------
class _SerdeF64(float):
    """a number serde_json reads as f64 (tests/test_json_float.py serde_read)"""


def _serde_float(t):
    from tests.test_json_float import serde_read
    r = serde_read(t)
    if r[0] == "range":
        raise ValueError("number out of range")
    return _SerdeF64(r[1]) if r[0] == "f64" else int(t)


def _py_loads(d):
    return json.loads(d, parse_float=_serde_float, parse_int=_serde_float)


def _py_canon(v):
    """serde_json::to_string of a Value as Python's json writes it: compact,
    BTreeMap (sorted) keys, raw non-ASCII, \\u00xx lowercase for other controls;
    f64 through the ryu model of tests/test_json_float.py."""
    from tests.test_json_float import ryu_py

    def enc(x):
        if isinstance(x, _SerdeF64):
            return ryu_py(float(x))
        if isinstance(x, dict):
            return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + enc(x[k]) for k in sorted(x)) + "}"
        if isinstance(x, list):
            return "[" + ",".join(enc(y) for y in x) + "]"
        return json.dumps(x, ensure_ascii=False)
    return enc(v).encode()


def test_array_map_reference_kat(kats):
    case = next(c for c in kats["chain"] if c["name"] == "array_map")
    st, els = O.json_array_map(case["calls"][0]["values"][0].encode())
    assert st == "ok" and els == [e.encode() for e in case["calls"][0]["expect"]]


@pytest.mark.parametrize("sorted_keys", [True, False])
def test_array_map_oracle_vs_python_json(sorted_keys):
    """Accept/reject and every canonical element against Python's independent
    json module (valid documents: identical; Python is laxer on floats, which the
    restatement leaves unsupported)."""
    docs = jsongen.array_corpus(5, 400, 0, sorted_keys=sorted_keys, ints_only=True)
    for d in docs:
        st, els = O.json_array_map(d)
        assert st == "ok", (d, els)
        assert els == [_py_canon(v) for v in json.loads(d)], d


def test_array_map_oracle_errors_and_floats():
    for d in jsongen.ARRAY_FIXED + jsongen.array_corpus(9, 0, 300):
        st, res = O.json_array_map(d)
        try:
            py = _py_loads(d)
            py_ok = isinstance(py, list)
        except (ValueError, RecursionError):
            py_ok = False
        if st == "ok":
            assert py_ok, d
            assert res == [_py_canon(v) for v in py], d
        else:
            assert " at line " in res, (d, res)
            if py_ok:  # Python accepts lone surrogates and deeper nesting than serde's limit 128
                assert b"\\ud8" in d or b"\\udc" in d or d.count(b"[") >= 128, (d, res)


# ---------------------------------------------------------------------------
# the lean filter_json fast path's token DFA (fluvio_amd/csrc/fsg_json_dfa.h):
# whatever it accepts, the serde_json restatement accepts with the same level
# ---------------------------------------------------------------------------
def _dfa_probe():
    import ctypes
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "oracle", "_build", "libjson_dfa_probe.so")
    src = os.path.join(root, "tests", "native", "json_dfa_probe.cpp")
    hdr = os.path.join(root, "fluvio_amd", "csrc", "fsg_json_dfa.h")
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.dirname(hdr), src, "-o", out],
                       check=True)
    L = ctypes.CDLL(out)
    L.json_dfa_probe.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]

    def probe(v):
        lv = ctypes.c_int(-1)
        return L.json_dfa_probe(v, len(v), ctypes.byref(lv)), lv.value
    return probe


def test_lean_json_dfa_only_accepts_what_serde_accepts():
    from fluvio_amd import protocol as P
    from fluvio_amd import synth
    probe = _dfa_probe()
    docs = jsongen.corpus(21, 600, 900)
    docs += [b'{"level":"info","message":"m","n":%s}' % n for n in
             (b"0", b"-0", b"01", b"1.", b"1.5", b"-", b"1e", b"1e+", b"1E-7", b"2e10", b"-12.5e+3", b"00", b"1 2")]
    docs += [b'{"level":"info","message":"m","t":%s}' % t for t in
             (b"true", b"tru", b"truee", b"false", b"fals", b"null", b"nul", b"nulll", b"t rue", b"True")]
    docs += [b'{"level":"info","message":"x","level":"warn"}', b'{"message":"x"}', b'{ "level" : "warn" , "message" : "y" }',
             b'{"level":"warn","message":"y"} ', b' {"level":"warn","message":"y"}', b'{"level":"warn","message":"y"}}',
             b'{"level":"warn","message":"y",}', b'{"level":"warn" "message":"y"}', b'{"level":"warnx","message":"y"}']
    accepted = 0
    for d in docs:
        ok, lv = probe(d)
        if ok:
            accepted += 1
            assert O.json_structured_log(d) == ("ok", lv), d
    assert accepted >= 10
    # the bench's C2 documents are all decided by the fast path
    for b in P.decode_batches(synth.make_slice(2, 300)):
        for r in b.memory_records():
            ok, lv = probe(r.value)
            assert ok and O.json_structured_log(r.value) == ("ok", lv)


# ---------------------------------------------------------------------------
# map_json_project (C3 field projection, defined by the oracle: parity
# unpinned by the reference) against Python's json on the accept/reject
# decision and the projected text
# ---------------------------------------------------------------------------
def test_project_oracle_vs_python_json():
    docs = jsongen.corpus(31, 300, 300) + [b'{"message":"a","message":"b"}', b'{"a":{"message":1}}', b"{}",
                                           b'{"message":[3,{"b":1,"a":2}]}', b'{"message":null}']
    seen_ok = seen_none = 0
    for d in docs:
        try:
            st, v = O.json_project(d)
        except O.OracleError as e:
            assert e.status == -103
            continue
        try:
            py = _py_loads(d)
        except (ValueError, RecursionError):
            py = ValueError
        if st == "ok":
            assert isinstance(py, dict), d
            if "message" in py:
                assert v == _py_canon(py["message"]), d
                seen_ok += 1
            else:
                assert v is None, d
                seen_none += 1
        else:
            assert " at line " in v, (d, v)
            if isinstance(py, dict):  # Python accepts lone surrogates / deeper nesting
                import re
                assert re.search(rb"\\u[dD][89a-fA-F]", d) or d.count(b"[") >= 60, (d, v)
    assert seen_ok > 100 and seen_none > 0


# ---------------------------------------------------------------------------
# aggregate-json (examples/aggregate-json: HashMap<String, u32> += per key,
# to_vec_pretty): the oracle against the Python model of the guest's HashMap
# (tests/rust_hashmap.py: SipHash-1-3 under the wasm32 RandomState sequence,
# hashbrown's bucket order), including error hints
# ---------------------------------------------------------------------------
def test_aggregate_json_oracle_vs_python_model():
    from fluvio_amd import protocol as P
    from tests import rust_hashmap as H
    from tests.test_hashmap_order import _py_u32_map
    import random
    rng = random.Random(12)
    keys = ["repo-%d" % i for i in range(12)] + ["é", 'q"uote', "tab\t"]
    for trial in range(40):
        acc0 = rng.choice([b"", b"{}", b'{"repo-1": 5}', b"nope", b'{"a": 1, "a": 2}', b'{"x":-1}'])
        vals = []
        for _ in range(rng.randint(1, 12)):
            k = rng.random()
            if k < 0.8:
                d = {rng.choice(keys): rng.randint(0, 2 ** 32 - 1) for _ in range(rng.randint(0, 3))}
                vals.append(json.dumps(d, ensure_ascii=rng.random() < 0.5).encode())
            elif k < 0.9:
                vals.append(b'{"repo-1": 1, "repo-1": 7}')
            else:
                vals.append(rng.choice([b'{"a": -1}', b'{"a": "s"}', b"[1]", b'{"a": 4294967296}', b"{", b'{"a":1}x']))
        ch = O.OracleChain([("aggregate-json", {}, acc0)])
        out = ch.process(P.encode_records([P.Record.new(v) for v in vals]))
        model = H.AggregateJson(acc0, _py_u32_map)
        expect = []
        for v in vals:
            o = model.call(v)
            if o is None:
                break
            expect.append(o)
        err = len(expect) < len(vals)
        got = [r.value for r in P.decode_records(out["bytes"])]
        assert got == expect, (acc0, vals)
        assert (out["error"] is not None) == err, (vals, out["error"])
        if err:
            assert " at line " in out["error"]["hint"]
