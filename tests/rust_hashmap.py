"""Python model of the aggregate-json guest's map order (test infrastructure).

smartmodule/examples/aggregate-json/src/lib.rs:22-36 deserializes the
accumulator and the record into `HashMap<String, u32>` (std), adds the record's
map into the accumulator's with the entry API and writes `to_vec_pretty` of
the accumulator's map: the output keys come in the map's iteration order.  The
module is built with Rust 1.75 (the repository root's rust-toolchain.toml; a
guest built from smartmodule/cargo_template, which pins `stable`, may carry a
newer hashbrown whose order differs: a known limit) for
wasm32-unknown-unknown, where that order is deterministic:

* `RandomState::new()` (std/src/hash/random.rs) takes its keys from a
  thread-local seeded once by `sys::hashmap_random_keys()`, which is the
  constant `(1, 2)` on this target (std/src/sys/unsupported/common.rs), and
  bumps k0 by one per call.  Every map the guest creates draws one: serde's
  HashMap visitor (`with_capacity_and_hasher(0, S::default())`, only once
  serde_json's deserialize_map has seen '{') and `unwrap_or_default()`'s
  `HashMap::default()` when the accumulator does not parse.
* The hasher is SipHash-1-3 (core/src/hash/sip.rs) keyed (k0, k1); a String
  hashes as its bytes followed by 0xFF (`Hasher::write_str`).
* The table is hashbrown 0.14 (std's backend in 1.75) with its generic
  8-byte control groups (`GroupWord = u64` on wasm32): buckets a power of two,
  h1 = the hash as a 32-bit usize, triangular probing by groups, trailing
  control bytes mirroring the first group, a fix-up scan from bucket 0 for
  tables smaller than a group, growth 0 -> 4 -> 8 -> 2x (capacity 3, 7, then
  7/8 of the buckets), `HashMap::insert` reserving one slot before it looks
  the key up, the entry API reserving only for a vacant key, resize
  re-inserting in bucket order, iteration in bucket order.

This module restates that literally over control bytes; oracle/fsg_oracle.c
(hb_*) is the C restatement the GPU is checked against, and the device
(fsg_keyed.hip k_aggj_order) uses a rotated-window formulation of the same
probe.  No reference fixture holds an aggregate-json output with two or more
keys, so beyond SipHash's published vectors this order is parity-unpinned.
"""
M64 = (1 << 64) - 1
GROUP = 8
EMPTY = 0xFF


def _rotl(x, b):
    return ((x << b) | (x >> (64 - b))) & M64


def siphash(k0, k1, msg, c=1, d=3):
    """SipHash-c-d (64-bit output) of `msg` under keys k0, k1."""
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rnd():
        nonlocal v0, v1, v2, v3
        v0 = (v0 + v1) & M64
        v1 = _rotl(v1, 13) ^ v0
        v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & M64
        v3 = _rotl(v3, 16) ^ v2
        v0 = (v0 + v3) & M64
        v3 = _rotl(v3, 21) ^ v0
        v2 = (v2 + v1) & M64
        v1 = _rotl(v1, 17) ^ v2
        v2 = _rotl(v2, 32)

    n = len(msg)
    full = n - n % 8
    for i in range(0, full, 8):
        m = int.from_bytes(msg[i:i + 8], "little")
        v3 ^= m
        for _ in range(c):
            rnd()
        v0 ^= m
    b = ((n & 0xFF) << 56) | int.from_bytes(msg[full:] + bytes(8 - (n - full)), "little")
    v3 ^= b
    for _ in range(c):
        rnd()
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(d):
        rnd()
    return v0 ^ v1 ^ v2 ^ v3


def str_hash(k0, key: bytes, k1=2):
    """`key.hash(&mut DefaultHasher)` for a String under RandomState (k0, k1)."""
    return siphash(k0, k1, key + b"\xff", 1, 3)


def bucket_mask_to_capacity(mask):
    return mask if mask < 8 else ((mask + 1) // 8) * 7


def capacity_to_buckets(cap):
    if cap < 8:
        return 4 if cap < 4 else 8
    adj = cap * 8 // 7
    return 1 << (adj - 1).bit_length()


class RawTable:
    """hashbrown RawTable<(String, u32)> with generic 8-byte groups."""

    def __init__(self, k0, k1=2):
        self.k0, self.k1 = k0, k1
        self.buckets = 0          # 0: the empty singleton
        self.ctrl = [EMPTY] * GROUP
        self.slot = []
        self.items = 0
        self.where = {}           # key -> bucket (equality lookups)

    def hash(self, key):
        return str_hash(self.k0, key, self.k1)

    def growth_left(self):
        return (bucket_mask_to_capacity(self.buckets - 1) if self.buckets else 0) - self.items

    def _set_ctrl(self, i, c):
        mask = self.buckets - 1
        self.ctrl[i] = c
        self.ctrl[((i - GROUP) & mask) + GROUP] = c

    def _find_insert_slot(self, h):
        mask = self.buckets - 1
        pos, stride = (h & 0xFFFFFFFF) & mask, 0
        while True:
            group = self.ctrl[pos:pos + GROUP]
            for bit, c in enumerate(group):
                if c & 0x80:  # EMPTY or DELETED
                    idx = (pos + bit) & mask
                    if not (self.ctrl[idx] & 0x80):  # fix_insert_slot: table smaller than a group
                        idx = next(i for i, c2 in enumerate(self.ctrl[:GROUP]) if c2 & 0x80)
                    return idx
            stride += GROUP
            pos = (pos + stride) & mask

    def _place(self, key, val, h):
        i = self._find_insert_slot(h)
        self._set_ctrl(i, ((h & 0xFFFFFFFF) >> 25) & 0x7F)
        self.slot[i] = [key, val]
        self.where[key] = i
        self.items += 1

    def _resize(self, cap):
        old = self.iter_slots()
        self.buckets = capacity_to_buckets(cap)
        self.ctrl = [EMPTY] * (self.buckets + GROUP)
        self.slot = [None] * self.buckets
        self.items = 0
        self.where = {}
        for k, v in old:
            self._place(k, v, self.hash(k))

    def reserve1(self):
        if self.growth_left() < 1:
            full = bucket_mask_to_capacity(self.buckets - 1) if self.buckets else 0
            self._resize(max(self.items + 1, full + 1))

    def insert(self, key, val):
        """HashMap::insert (find_or_find_insert_slot reserves first)."""
        self.reserve1()
        if key in self.where:
            self.slot[self.where[key]][1] = val
        else:
            self._place(key, val, self.hash(key))

    def entry_add(self, key, val):
        """`entry(key).and_modify(|s| *s += v).or_insert(v)` (u32 wrapping)."""
        if key in self.where:
            s = self.slot[self.where[key]]
            s[1] = (s[1] + val) & 0xFFFFFFFF
        else:
            self.reserve1()
            self._place(key, val, self.hash(key))

    def iter_slots(self):
        return [(s[0], s[1]) for s in self.slot if s is not None]


def pretty(pairs):
    """serde_json::to_vec_pretty of a map of strings to u32."""
    import json
    if not pairs:
        return b"{}"
    return ("{\n" + ",\n".join("  %s: %d" % (json.dumps(k.decode("utf-8"), ensure_ascii=False), v)
                                for k, v in pairs) + "\n}").encode()


def ws_first(doc: bytes):
    i = 0
    while i < len(doc) and doc[i] in b" \t\n\r":
        i += 1
    return doc[i:i + 1]


class AggregateJson:
    """One aggregate-json wasm instance: the accumulator and the RandomState
    counter persist across calls.  `parse(doc)` -> list of (key bytes, u32) in
    text order, or None when serde_json rejects the document."""

    def __init__(self, acc: bytes, parse):
        self.acc = acc
        self.parse = parse
        self.k0 = 1

    def _draw(self):
        k = self.k0
        self.k0 += 1
        return k

    def call(self, value: bytes):
        """The record's output value, or None for an error (the chain stops)."""
        pairs = self.parse(self.acc)
        k_acc = self._draw() if ws_first(self.acc) == b"{" else None
        if pairs is None:
            k_acc = self._draw()  # unwrap_or_default: HashMap::default()
            pairs = []
        acc = RawTable(k_acc)
        for k, v in pairs:
            acc.insert(k, v)
        rec_pairs = self.parse(value)
        k_rec = self._draw() if ws_first(value) == b"{" else None
        if rec_pairs is None:
            return None
        rec = RawTable(k_rec)
        for k, v in rec_pairs:
            rec.insert(k, v)
        for k, v in rec.iter_slots():
            acc.entry_add(k, v)
        self.acc = pretty(acc.iter_slots())
        return self.acc
