"""Compressed fetch slices for the decompression tests: every
stored batch of a synthetic slice re-stored with its record section (u32 count +
records) compressed by the codec the batch's attributes name, as
Batch::<RawRecords>::try_from does (fluvio-protocol record/batch.rs:212-233),
batch_len and CRC32C recomputed.  The encoders are the oracle's test-data
encoders (oracle/fsg_codec.c) and Python's gzip."""
import struct

from oracle import oracle as O


def batches(sl: bytes):
    pos = 0
    while pos < len(sl):
        blen = struct.unpack(">i", sl[pos + 8:pos + 12])[0]
        yield pos, blen
        pos += 12 + blen


def recompress(sl: bytes, codecs, flags=0, corrupt=None) -> bytes:
    """codecs: list cycled over the batches (0 = leave uncompressed); flags:
    encoder flags per codec (int or dict codec -> int); corrupt: {batch index:
    byte offset into the compressed section to flip}."""
    out = bytearray()
    for i, (pos, blen) in enumerate(batches(sl)):
        hdr = bytearray(sl[pos:pos + 57])
        sec = sl[pos + 57:pos + 12 + blen]
        codec = codecs[i % len(codecs)]
        if codec:
            f = flags.get(codec, 0) if isinstance(flags, dict) else flags
            sec = bytearray(O.compress(codec, sec, f))
            if corrupt and i in corrupt:
                sec[corrupt[i] % len(sec)] ^= 0x5A
            sec = bytes(sec)
            attrs = (struct.unpack(">h", bytes(hdr[21:23]))[0] & ~7) | codec
            hdr[21:23] = struct.pack(">h", attrs)
        hdr[8:12] = struct.pack(">i", 45 + len(sec))
        hdr[17:21] = struct.pack(">I", O.crc32c(bytes(hdr[21:57]) + sec))
        out += hdr + sec
    return bytes(out)
