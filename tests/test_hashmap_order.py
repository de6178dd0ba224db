"""aggregate-json output order (CPU): SipHash vectors, hand-traced hashbrown
layouts, and the C oracle against the Python model (tests/rust_hashmap.py) over
random record streams.  See rust_hashmap.py for what is restated and why the
order is deterministic on the reference's wasm32 target."""
import json
import os
import random
import subprocess
import sys

import pytest

from fluvio_amd import protocol as P
from oracle import oracle as O
from tests import rust_hashmap as H

K0 = int.from_bytes(bytes(range(8)), "little")
K1 = int.from_bytes(bytes(range(8, 16)), "little")


def test_siphash_24_published_vectors():
    """SipHash-2-4 (Aumasson & Bernstein, appendix A / vectors.h): key 00..0f."""
    for impl in (lambda m: O.siphash(2, 4, K0, K1, m), lambda m: H.siphash(K0, K1, m, 2, 4)):
        assert impl(b"") == 0x726FDB47DD0E0E31
        assert impl(bytes(range(15))) == 0xA129CA6149BE45E5


def test_siphash_24_matches_python_hash():
    """CPython 3.10's bytes hash is SipHash-2-4 keyed by zeros under PYTHONHASHSEED=0."""
    msgs = [b"abc", b"hello world!!", b"x" * 40, bytes(range(200))]
    out = subprocess.check_output([sys.executable, "-c", "import sys;[print(hash(m)) for m in %r]" % (msgs,)],
                                  env=dict(os.environ, PYTHONHASHSEED="0")).decode().split()
    for m, py in zip(msgs, out):
        v = O.siphash(2, 4, 0, 0, m)
        assert (v - (1 << 64) if v >> 63 else v) == int(py)
        assert H.siphash(0, 0, m, 2, 4) == v


def test_siphash_13_rust_vector():
    """SipHash-1-3 (std's DefaultHasher): Rust's own test vector for the empty
    message under key 00..0f (library/core/tests/hash/sip.rs, test_siphash_1_3:
    dc c4 0f 05 58 01 ac ab, little-endian)."""
    assert O.siphash(1, 3, K0, K1, b"").to_bytes(8, "little") == bytes.fromhex("dcc40f055801acab")
    assert H.siphash(K0, K1, b"", 1, 3) == O.siphash(1, 3, K0, K1, b"")
    rng = random.Random(5)
    for n in range(0, 40):
        m = bytes(rng.randrange(256) for _ in range(n))
        k0, k1 = rng.getrandbits(64), rng.getrandbits(64)
        assert O.siphash(1, 3, k0, k1, m) == H.siphash(k0, k1, m, 1, 3)


def test_str_hash_low_bits():
    """The probe positions used in the hand traces below (h1 = hash as u32)."""
    h = {k: H.str_hash(1, k) & 0xFFFFFFFF for k in (b"a", b"b", b"c", b"d", b"e")}
    assert [h[k] & 3 for k in (b"a", b"b", b"c")] == [3, 3, 0]
    assert [h[k] & 7 for k in (b"a", b"b", b"c", b"d", b"e")] == [3, 7, 4, 3, 5]
    assert H.str_hash(1, b"a") == O.siphash(1, 3, 1, 2, b"a\xff")


def test_hashbrown_hand_trace():
    """HashMap::insert of a, b, c, d, e under RandomState (1, 2):
    a: reserve -> 4 buckets, h&3 = 3 -> bucket 3.
    b: h&3 = 3 full; the group at 3 reads ctrl[3..11): bucket 3, then EMPTY
       padding -> index (3 + 1) & 3 = 0, which is empty -> bucket 0.
    c: h&3 = 0 full -> bucket 1.
    d: items 3 = capacity 3 -> grow to 8, re-insert in bucket order b(0) c(1)
       a(3) with h&7 = 7, 4, 3 -> b@7 c@4 a@3; then d: h&7 = 3, 4 full -> @5.
    e: h&7 = 5 full -> @6.
    Iteration (bucket order): a c d e b."""
    t = H.RawTable(1)
    for k in (b"a", b"b", b"c", b"d", b"e"):
        t.insert(k, 1)
    assert [k for k, _ in t.iter_slots()] == [b"a", b"c", b"d", b"e", b"b"]


def test_aggregate_json_hand_trace_oracle():
    """One aggregate-json call, empty accumulator, record {"a":1,...,"e":1}:
    the accumulator does not parse (no '{'): HashMap::default() draws k0 = 1;
    the record's map draws k0 = 2.  Record map (k0 = 2, h&3 / h&7 of a..e:
    0/0, 3/7, 0/4, 3/3, 0/0): a@0 b@3 c@1, grow (a c b -> a@0 c@4 b@7), d@3,
    e: 0 full -> @1 => bucket order a e d c b.  Added into the accumulator map
    (k0 = 1) in that order: a@3, e@1 (h&3 = 1), d: 3 full -> group padding ->
    @0; c: grow (d e a -> d@3 e@5 a@4), c: 4, 5 full -> @6; b@7 => d a e c b."""
    rec = b'{"a":1,"b":1,"c":1,"d":1,"e":1}'
    ch = O.OracleChain([("aggregate-json", {}, None)])
    out = ch.process(P.encode_records([P.Record.new(rec)]))
    got = P.decode_records(out["bytes"])[0].value
    assert got == b'{\n  "d": 1,\n  "a": 1,\n  "e": 1,\n  "c": 1,\n  "b": 1\n}'
    m = H.AggregateJson(b"", _py_u32_map)
    assert m.call(rec) == got


def _py_u32_map(doc: bytes):
    """The (key bytes, u32) pairs of a JSON object in text order, or None where
    serde_json::from_slice::<HashMap<String, u32>> fails."""
    class _Pairs(list):
        pass
    try:
        pairs = json.loads(doc, object_pairs_hook=_Pairs, parse_float=lambda x: (_ for _ in ()).throw(ValueError()),
                           parse_constant=lambda x: (_ for _ in ()).throw(ValueError()))
    except (ValueError, RecursionError):
        return None
    if not isinstance(pairs, _Pairs):
        return None
    for _k, v in pairs:
        if isinstance(v, bool) or not isinstance(v, int) or not (0 <= v < 2 ** 32):
            return None
    return [(k.encode(), v) for k, v in pairs]


@pytest.mark.parametrize("seed", range(6))
def test_aggregate_json_oracle_vs_model_streams(seed):
    """Random record streams over several process() calls of one instance (the
    RandomState counter carries across calls), keys 1..70 so maps cross the
    4 / 8 / 16 / 32 / 64 / 128 bucket boundaries; accumulators that parse, do
    not parse, and parse after '{' fails (two draws)."""
    rng = random.Random(seed)
    nkeys = rng.choice([6, 20, 70])
    keys = ["repo-%d" % i for i in range(nkeys)] + ["é", 'q"uote', "tab\t"]
    acc0 = rng.choice([None, b"{}", b'{"repo-1": 5}', b"nope", b'{"a": 1, "a": 2}', b'{"x":-1}', b"  {\"x\": \"s\"}"])
    ch = O.OracleChain([("aggregate-json", {}, acc0)])
    model = H.AggregateJson(acc0 or b"", _py_u32_map)
    for call in range(3):
        vals = []
        for _ in range(rng.randint(1, 30)):
            if rng.random() < 0.97:
                d = {rng.choice(keys): rng.randint(0, 2 ** 32 - 1) for _ in range(rng.randint(0, 9))}
                v = json.dumps(d, ensure_ascii=rng.random() < 0.5).encode()
                if d and rng.random() < 0.1:
                    v = v[:-1] + b', "%s": 3}' % rng.choice(keys).encode()  # duplicate key: last wins
                vals.append(v)
            else:
                vals.append(rng.choice([b'{"a": -1}', b'  {"a": "s"}', b"[1]", b"7", b"  "]))
        out = ch.process(P.encode_records([P.Record.new(v) for v in vals]))
        got = [r.value for r in P.decode_records(out["bytes"])]
        expect = []
        for v in vals:
            o = model.call(v)
            if o is None:
                break
            expect.append(o)
        assert got == expect, (seed, call)
        assert (out["error"] is not None) == (len(expect) < len(vals))
        assert ch.accumulator(0) == model.acc
