"""Topic partitions across GPUs: key routing, rank ownership, state merge.

Fluvio's only scale-out axis is the topic partition.  Keyed records are routed
by SipHash-2-4 of the key (siphasher 1.0.0 `sip::SipHasher`, keys 0/0, over the
`Hash` encoding of a byte slice: usize length prefix then the bytes) modulo
the partition count; unkeyed records go round-robin
(crates/fluvio/src/producer/partitioning.rs:51-83).  Every partition has its
own SmartModule chain instance and therefore its own aggregate accumulator
(crates/fluvio-spu/src/smartengine/context.rs:25-30): partitions never
exchange data.

On MI355X the partitions of a topic are sharded p -> rank p mod N (one process
per GPU).  Filters, maps and array_map need no collective at all.  The only
exchange is the merge of per-partition aggregate state: each rank fills the
slots of the partitions it owns (zeros elsewhere) and one all-reduce (sum)
yields the topic-wide table on every rank — RCCL over xGMI on the GPU path
(`PartitionState.allreduce`, fsg_state_allreduce), torch.distributed on the
CPU test path.
"""
from __future__ import annotations

import struct
from typing import Callable, Dict, Iterable, List, Optional, Sequence

_M64 = (1 << 64) - 1


def _rotl(x: int, b: int) -> int:
    return ((x << b) | (x >> (64 - b))) & _M64


def siphash24(data: bytes, k0: int = 0, k1: int = 0) -> int:
    """SipHash-2-4 (Aumasson & Bernstein), 64-bit output."""
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rounds(n):
        nonlocal v0, v1, v2, v3
        for _ in range(n):
            v0 = (v0 + v1) & _M64
            v1 = _rotl(v1, 13) ^ v0
            v0 = _rotl(v0, 32)
            v2 = (v2 + v3) & _M64
            v3 = _rotl(v3, 16) ^ v2
            v0 = (v0 + v3) & _M64
            v3 = _rotl(v3, 21) ^ v0
            v2 = (v2 + v1) & _M64
            v1 = _rotl(v1, 17) ^ v2
            v2 = _rotl(v2, 32)

    n = len(data)
    full = n - n % 8
    for i in range(0, full, 8):
        m = struct.unpack_from("<Q", data, i)[0]
        v3 ^= m
        rounds(2)
        v0 ^= m
    tail = data[full:] + bytes(7 - n % 8)
    m = ((n & 0xFF) << 56) | struct.unpack("<Q", tail + b"\0")[0]
    v3 ^= m
    rounds(2)
    v0 ^= m
    v2 ^= 0xFF
    rounds(4)
    return v0 ^ v1 ^ v2 ^ v3


def partition_siphash(key: bytes, partition_count: int) -> int:
    """partitioning.rs:70-83: `key.hash(&mut SipHasher::new())` % partitions.
    `<[u8] as Hash>::hash` writes the length as a native-endian usize (8 bytes on
    the 64-bit client) before the bytes.

    Parity unpinned: SipHash-2-4 itself is pinned by siphasher's test vectors
    (tests/test_partitions.py), but no fixture in the reference tree holds a
    key -> partition pair, so the length-prefix assumption above is a restatement
    of std's `Hash for [u8]`, not checked against the reference client."""
    return siphash24(struct.pack("<Q", len(key)) + key) % partition_count


class RoundRobin:
    """SiphashRoundRobinPartitioner (partitioning.rs:39-68)."""

    def __init__(self):
        self.index = 0

    def partition(self, key: Optional[bytes], partition_count: int) -> int:
        if key is not None:
            return partition_siphash(key, partition_count)
        p = self.index % partition_count
        self.index = (self.index + 1) & 0xFFFFFFFF
        return p


def owned_partitions(partition_count: int, world: int, rank: int) -> List[int]:
    """Partitions of a topic this rank processes (p -> rank p mod world)."""
    return [p for p in range(partition_count) if p % world == rank]


def route(records: Iterable, partition_count: int, key_of: Callable = lambda r: r.key) -> Dict[int, list]:
    """Split producer records into per-partition lists, in send order."""
    rr = RoundRobin()
    out: Dict[int, list] = {p: [] for p in range(partition_count)}
    for r in records:
        out[rr.partition(key_of(r), partition_count)].append(r)
    return out


def wrap_i32(v: int) -> int:
    return (v + (1 << 31)) % (1 << 32) - (1 << 31)


def local_state_vector(partition_count: int, states: Dict[int, int]) -> List[int]:
    """This rank's slots of the topic state vector: its partitions' aggregate
    accumulators, zero for partitions other ranks own."""
    vec = [0] * partition_count
    for p, v in states.items():
        vec[p] = wrap_i32(v)
    return vec


def merge_states_torch(vec: Sequence[int]) -> List[int]:
    """All-reduce (sum, wrapping i32) of a state vector over torch.distributed
    (gloo on CPU ranks).  The GPU path does the same with RCCL on HBM-resident
    state (smartengine.PartitionState.allreduce)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(vec), dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


def union_dictionary(key_lists: Sequence[Sequence[bytes]]) -> Dict[bytes, int]:
    """The topic key dictionary of fsg_keyed_allreduce: the keys of every rank's
    list in rank order, each id given at its first occurrence, so every rank that
    holds the same gathered lists builds the same dictionary."""
    ids: Dict[bytes, int] = {}
    for keys in key_lists:
        for k in keys:
            if k not in ids:
                ids[k] = len(ids)
    return ids


KD_LEN_DEAD = 0xFFFFFF  # fsg_keyed.hip kKdLenDead: a descriptor with no key (a lost duplicate / padding)


def keyed_desc(keys: Sequence[Optional[bytes]]):
    """One rank's send buffers of fsg_keyed_allreduce (k_kd_desc): per key a u64
    descriptor `arena offset | length << 40` (None = a dead entry) and the key
    bytes packed in an arena."""
    desc, arena = [], bytearray()
    for k in keys:
        if k is None:
            desc.append(KD_LEN_DEAD << 40)
            continue
        desc.append(len(arena) | (len(k) << 40))
        arena += k
    return desc, bytes(arena)


def gather_shape(counts: Sequence[Sequence[int]]):
    """maxn / maxb of the all-gathers from every rank's (keys, arena bytes):
    at least one entry and 16 bytes, bytes rounded up to 16."""
    maxn = max([1] + [int(c[0]) for c in counts])
    maxb = max([16] + [int(c[1]) for c in counts])
    return maxn, (maxb + 15) & ~15


def union_from_gathered(gdesc: Sequence[int], garena: bytes, maxn: int, maxb: int):
    """k_kd_union / k_kd_first / k_kd_ids over the gathered buffers: item
    g = rank * maxn + i, a live item's key at garena[rank * maxb + off ..], union
    ids by first occurrence in item (rank-major) order.  -> (id per item or None,
    union keys in id order)."""
    ids: Dict[bytes, int] = {}
    gid: List[Optional[int]] = []
    for g, d in enumerate(gdesc):
        ln = d >> 40
        if ln == KD_LEN_DEAD:
            gid.append(None)
            continue
        off = (g // maxn) * maxb + (d & ((1 << 40) - 1))
        k = bytes(garena[off:off + ln])
        if k not in ids:
            ids[k] = len(ids)
        gid.append(ids[k])
    return gid, list(ids)


def merge_keyed(local: Dict[bytes, int], dist=None, group=None) -> Dict[bytes, int]:
    """Topic-wide per-key totals of aggregate-json states in the C ABI's shape
    (fsg_keyed_allreduce, fsg_runtime.cpp): all-gather every rank's (keys, arena
    bytes); all-gather the key descriptors (padded to maxn with dead entries) and
    the arenas (padded to maxb); the union dictionary built identically on every
    rank; this rank's values scattered into a dense K-slot table; one all-reduce
    (sum, u32 wrapping).  gloo on CPU ranks; the GPU path runs the same steps on
    HBM with RCCL (smartengine.KeyedState)."""
    import torch
    keys = list(local)
    desc, arena = keyed_desc(keys)
    multi = dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1
    nr = dist.get_world_size(group) if multi else 1
    me = dist.get_rank(group) if multi else 0
    cnt = torch.tensor([len(desc), len(arena)], dtype=torch.int64)
    gcnt = [torch.zeros(2, dtype=torch.int64) for _ in range(nr)]
    if multi:
        dist.all_gather(gcnt, cnt, group=group)
    else:
        gcnt = [cnt]
    maxn, maxb = gather_shape([c.tolist() for c in gcnt])
    # u64 descriptors travel as int64 bit patterns
    ld = torch.tensor([d - (1 << 64) if d >> 63 else d for d in desc + [KD_LEN_DEAD << 40] * (maxn - len(desc))],
                      dtype=torch.int64)
    la = torch.zeros(maxb, dtype=torch.uint8)
    if arena:
        la[:len(arena)] = torch.frombuffer(bytearray(arena), dtype=torch.uint8)
    gd = [torch.zeros(maxn, dtype=torch.int64) for _ in range(nr)]
    ga = [torch.zeros(maxb, dtype=torch.uint8) for _ in range(nr)]
    if multi:
        dist.all_gather(gd, ld, group=group)
        dist.all_gather(ga, la, group=group)
    else:
        gd, ga = [ld], [la]
    gdesc = [int(x) & _M64 for t in gd for x in t.tolist()]
    garena = b"".join(bytes(t.tolist()) for t in ga)
    gid, ukeys = union_from_gathered(gdesc, garena, maxn, maxb)
    dense = torch.zeros(len(ukeys), dtype=torch.int64)
    for i, k in enumerate(keys):  # k_kd_place: this rank's items
        dense[gid[me * maxn + i]] += int(local[k])
    if multi:
        dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=group)
    return {k: int(dense[i]) & 0xFFFFFFFF for i, k in enumerate(ukeys)}
