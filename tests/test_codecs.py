"""Record-section codecs: the oracle's restatement of
fluvio-compression (gzip / snappy frame / lz4 frame) pinned by independent
implementations (Python gzip/zlib, the xxhash module), encoder round trips,
the produce_batch.rs KAT, and process_batch over compressed slices."""
import gzip
import random
import struct
import zlib

import pytest

from fluvio_amd import protocol as P
from fluvio_amd import synth
from oracle import oracle as O
from tests.compressed_slices import recompress


def test_produce_batch_iterator_kat():
    """produce_batch.rs:124-153: a gzip batch of "soup" and an lz4 batch of
    "fries" decompress to these record sections."""
    for codec, v, exp in ((1, "soup", b"\0\0\0\x01\x14\0\0\0\0\x08soup\0"),
                          (3, "fries", b"\0\0\0\x01\x16\0\0\0\0\nfries\0")):
        sec = P.encode_records([P.Record.new(v)])
        assert sec == exp
        assert O.decompress(codec, O.compress(codec, sec)) == exp


def test_lib_rs_round_trip_text():
    """fluvio-compression gzip.rs / snappy.rs / lz4.rs test_compress_decompress."""
    text = b"FLUVIO_AAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA"
    for codec in (1, 2, 3, 4):
        c = O.compress(codec, text)
        assert len(c) < len(text)
        assert O.decompress(codec, c) == text


@pytest.mark.parametrize("n", [0, 1, 4, 13, 300, 5000, 70000, 200000])
def test_round_trips_and_independent_pins(n):
    rng = random.Random(n)
    data = bytes(rng.choice(b"abcdefgh  xyz0123{}\":,") for _ in range(n))
    for codec, flags in ((1, [0, 1, 9]), (2, [0, 1, 2]), (3, [0, 1, 2, 3, 4, 8, 15, 16, 31]),
                         (4, [0, 3, 19, 0x100, 0x200, 0x400, 0x800])):
        for f in flags:
            assert O.decompress(codec, O.compress(codec, data, f)) == data, (codec, f)
    assert O.decompress(1, gzip.compress(data)) == data          # Python's gzip encoder
    assert zlib.decompress(O.compress(1, data), 31) == data       # Python's inflate
    xxhash = pytest.importorskip("xxhash")
    assert O.xxh32(data) == xxhash.xxh32(data).intdigest()


def test_corrupt_inputs_are_errors():
    data = b"abcabcabcabcabcabc-" * 500
    for codec, f in ((1, 0), (2, 0), (3, 3), (3, 0), (4, 0x100)):
        c = bytearray(O.compress(codec, data, f))
        bad = 0
        for off in range(0, len(c), max(1, len(c) // 40)):
            t = bytearray(c)
            t[off] ^= 0x5A
            if O.decompress(codec, bytes(t)) is None:
                bad += 1
        assert bad > 0
        assert O.decompress(codec, bytes(c[:-3])) is None  # truncated
    # zstd (the crate's streaming Decoder): a bare magic, an empty input and
    # bytes after the last frame are "incomplete frame" / unknown-frame errors
    assert O.decompress(4, b"\x28\xb5\x2f\xfd") is None
    assert O.decompress(4, b"") is None
    assert O.decompress(4, O.compress(4, data) + b"\0\0") is None
    assert O.decompress(4, O.compress(4, data, 0x800)) == data  # a skippable frame first


@pytest.mark.parametrize("codecs", [[1], [2], [3], [0, 3, 2, 1]])
def test_process_batch_over_compressed_slice(codecs):
    """FileBatchIterator decompresses each batch: process_batch over the
    compressed slice equals the uncompressed one, apart from the output header's
    compression bits (set_compression of the first surviving batch) and CRC."""
    sl = synth.make_slice(2, 1500, base_offset=11)
    csl = recompress(sl, codecs)
    for mods in ([("filter_init", {"key": "timeout"}, None)], [("map", {}, None)], []):
        a = O.OracleChain(mods).process_batch(sl)
        b = O.OracleChain(mods).process_batch(csl)
        assert a["status"] == b["status"] == 0
        ra, rb = bytearray(a["bytes"]), bytearray(b["bytes"])
        first = next(i for i, c in enumerate(codecs * 10000) if True)  # noqa: F841
        assert rb[22] & 7 == (codecs[0] if a["n_records"] else 0) or a["n_records"] == 0
        ra[17:23] = rb[17:23] = b"\0" * 6
        assert ra == rb
        assert a["metrics"] == b["metrics"]


def test_process_batch_decode_error_is_io():
    sl = synth.make_slice(3, 2000)
    csl = recompress(sl, [3], flags=3, corrupt={1: 40})
    r = O.OracleChain([("filter_map", {}, None)]).process_batch(csl)
    assert r["status"] == -104  # io::Error from the iterator
