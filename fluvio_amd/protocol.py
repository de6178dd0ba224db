"""Host-side mirror of the fluvio-protocol data-plane types used on the
SmartModule path: zigzag varints, ``Record``/``RecordHeader``/``RecordData``,
``Vec<Record>`` and file-format ``Batch`` with CRC32C.

This module only builds and parses wire bytes on the host (inputs handed to the
C ABI, outputs handed back).  All per-record work of the hot path runs in the
HIP kernels of ``fluvio_amd/csrc``.

Reference (paths relative to /root/reference):
  varint            crates/fluvio-protocol/src/core/varint.rs:13-80
  Record            crates/fluvio-protocol/src/record/data.rs:375-562
  RecordData        crates/fluvio-protocol/src/record/data.rs:186-227
  Batch/BatchHeader crates/fluvio-protocol/src/record/batch.rs:86-93, 398-430, 444-508
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

BATCH_HEADER_SIZE = 45  # batch.rs:499-508
BATCH_PREAMBLE_SIZE = 12
BATCH_FILE_HEADER_SIZE = BATCH_PREAMBLE_SIZE + BATCH_HEADER_SIZE
NO_TIMESTAMP = -1
ATTR_SCHEMA_PRESENT = 0x10
ATTR_COMPRESSION_CODEC_MASK = 0x07


def _i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def varint_encode(num: int) -> bytes:
    """variant_encode (varint.rs:43-66) including its `>> 31` / `0xffffff80` quirk."""
    v = _i64((num << 1) ^ (num >> 31))
    out = bytearray()
    while v & 0xFFFFFF80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v & 0xFF)
    return bytes(out)


def varint_size(num: int) -> int:
    return len(varint_encode(num))


def varint_decode(buf: bytes, pos: int = 0) -> Tuple[int, int]:
    """varint_decode (varint.rs:13-40): returns (value, new_pos); raises EOFError."""
    num = 0
    shift = 0
    while True:
        if pos >= len(buf):
            raise EOFError("varint decoding no more bytes left")
        b = buf[pos]
        pos += 1
        num |= (b & 0x7F) << (shift & 63)
        shift += 7
        if not b & 0x80:
            break
    num = _i64(num)
    return _i64((num >> 1) ^ -(num & 1)), pos


@dataclass
class RecordHeader:
    attributes: int = 0
    timestamp_delta: int = 0
    offset_delta: int = 0


@dataclass
class Record:
    """`Record<RecordData>` (data.rs:413)."""

    value: bytes = b""
    key: Optional[bytes] = None
    preamble: RecordHeader = field(default_factory=RecordHeader)
    headers: int = 0

    @staticmethod
    def new(value) -> "Record":
        return Record(value=value.encode() if isinstance(value, str) else bytes(value))

    @staticmethod
    def new_key_value(key, value) -> "Record":
        k = None if key is None else (key.encode() if isinstance(key, str) else bytes(key))
        v = value.encode() if isinstance(value, str) else bytes(value)
        return Record(value=v, key=k)

    def offset_delta(self) -> int:
        return self.preamble.offset_delta

    def timestamp_delta(self) -> int:
        return self.preamble.timestamp_delta

    # -- codec ---------------------------------------------------------
    def _inner(self) -> bytes:
        out = bytearray()
        out.append(self.preamble.attributes & 0xFF)
        out += varint_encode(self.preamble.timestamp_delta)
        out += varint_encode(self.preamble.offset_delta)
        if self.key is None:
            out.append(0)
        else:
            out.append(1)
            out += varint_encode(len(self.key))
            out += self.key
        out += varint_encode(len(self.value))
        out += self.value
        out += varint_encode(self.headers)
        return bytes(out)

    def encode(self) -> bytes:
        inner = self._inner()
        return varint_encode(len(inner)) + inner

    def write_size(self) -> int:
        return len(self.encode())


def encode_records(records: List[Record]) -> bytes:
    """`Vec<Record>` encode: u32 BE count + records (encoder.rs:49-77)."""
    return struct.pack(">I", len(records)) + b"".join(r.encode() for r in records)


def decode_records(buf: bytes) -> List[Record]:
    """`Vec<Record>` decode (decoder.rs:43-63 + data.rs:534-562)."""
    if len(buf) < 4:
        raise EOFError("vec len")
    (cnt,) = struct.unpack(">i", buf[:4])
    pos = 4
    out: List[Record] = []
    for _ in range(max(cnt, 0)):
        ln, pos = varint_decode(buf, pos)
        if len(buf) - pos < ln:
            raise EOFError("not enough for record")
        if pos >= len(buf):
            raise EOFError("attributes")
        attr = buf[pos]
        pos += 1
        attr = attr - 256 if attr >= 128 else attr
        ts, pos = varint_decode(buf, pos)
        od, pos = varint_decode(buf, pos)
        if pos >= len(buf):
            raise EOFError("key tag")
        tag = buf[pos]
        pos += 1
        if tag > 1:
            raise ValueError("not valid bool value")
        key = None
        if tag == 1:
            kl, pos = varint_decode(buf, pos)
            kl = kl & ((1 << 64) - 1)
            take = min(kl, len(buf) - pos)
            key = bytes(buf[pos:pos + take])
            pos += take
        vl, pos = varint_decode(buf, pos)
        vl = vl & ((1 << 64) - 1)
        take = min(vl, len(buf) - pos)
        value = bytes(buf[pos:pos + take])
        pos += take
        hdr, pos = varint_decode(buf, pos)
        out.append(Record(value=value, key=key, preamble=RecordHeader(attr, ts, od), headers=hdr))
    return out


# ---------------------------------------------------------------------------
# CRC32C (host-side helper for building small inputs; the product computes the
# output-batch CRC on the GPU)
# ---------------------------------------------------------------------------
_CRC_TAB = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TAB.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    tab = _CRC_TAB
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


@dataclass
class BatchHeader:
    partition_leader_epoch: int = -1
    magic: int = 2
    crc: int = 0
    attributes: int = 0
    last_offset_delta: int = -1
    first_timestamp: int = NO_TIMESTAMP
    max_time_stamp: int = NO_TIMESTAMP
    producer_id: int = -1
    producer_epoch: int = -1
    first_sequence: int = -1


@dataclass
class Batch:
    """`Batch<MemoryRecords>` (batch.rs:86) with its file-format encoder."""

    base_offset: int = 0
    header: BatchHeader = field(default_factory=BatchHeader)
    records: List[Record] = field(default_factory=list)
    schema_id: int = 0

    def add_record(self, record: Record) -> None:
        """Batch::add_records + update_offset_deltas (batch.rs:276-291)."""
        self.records.append(record)
        for i, r in enumerate(self.records):
            r.preamble.offset_delta = i
        self.header.last_offset_delta = len(self.records) - 1

    def has_schema(self) -> bool:
        return bool(self.header.attributes & ATTR_SCHEMA_PRESENT)

    def encode(self) -> bytes:
        """Batch::encode (batch.rs:398-430): CRC32C over attributes..records."""
        h = self.header
        body = struct.pack(">hiqqqhi", h.attributes, h.last_offset_delta, h.first_timestamp,
                           h.max_time_stamp, h.producer_id, h.producer_epoch, h.first_sequence)
        if self.has_schema():
            body += struct.pack(">I", self.schema_id)
        recs = encode_records(self.records)
        body += recs
        crc = crc32c(body)
        batch_len = BATCH_HEADER_SIZE + len(recs) + (4 if self.has_schema() else 0)
        return struct.pack(">qiibI", self.base_offset, batch_len, h.partition_leader_epoch,
                           h.magic, crc) + body


@dataclass
class DecodedBatch:
    base_offset: int
    batch_len: int
    header: BatchHeader
    records_bytes: bytes

    def memory_records(self) -> List[Record]:
        return decode_records(self.records_bytes)


def decode_batch(buf: bytes, pos: int = 0) -> Tuple[DecodedBatch, int]:
    """File-format batch decode (batch.rs:163-180 + Decoder for Batch)."""
    base_offset, batch_len, ple, magic, crc = struct.unpack_from(">qiibI", buf, pos)
    attrs, lod, fts, mts, pid, pep, fseq = struct.unpack_from(">hiqqqhi", buf, pos + 21)
    hdr = BatchHeader(ple, magic, crc, attrs, lod, fts, mts, pid, pep, fseq)
    start = pos + BATCH_FILE_HEADER_SIZE
    end = pos + BATCH_PREAMBLE_SIZE + batch_len
    return DecodedBatch(base_offset, batch_len, hdr, bytes(buf[start:end])), end


def decode_batches(buf: bytes) -> List[DecodedBatch]:
    out, pos = [], 0
    while pos < len(buf):
        b, pos = decode_batch(buf, pos)
        out.append(b)
    return out
