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


def merge_keyed(local: Dict[bytes, int], dist=None, group=None) -> Dict[bytes, int]:
    """Topic-wide per-key totals of aggregate-json states with the shape of the
    C ABI's merge (fsg_keyed_allreduce): every rank's exact key list all-gathered,
    the union dictionary built in rank order, this rank's values scattered into a
    dense K-slot table, one all-reduce (sum), u32 wrapping.  gloo on CPU ranks;
    the GPU path runs the same steps on HBM with RCCL (smartengine.KeyedState)."""
    import torch
    keys = list(local)
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        gathered = [None] * dist.get_world_size(group)
        dist.all_gather_object(gathered, keys, group=group)
    else:
        gathered = [keys]
    ids = union_dictionary(gathered)
    dense = torch.zeros(len(ids), dtype=torch.int64)
    for k, v in local.items():
        dense[ids[k]] += int(v)
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=group)
    return {k: int(dense[i]) & 0xFFFFFFFF for k, i in ids.items()}
