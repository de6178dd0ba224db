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
    the 64-bit client) before the bytes."""
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


def fnv1a64(key: bytes) -> int:
    """The key fingerprint of fsg_chain_keyed_state (FNV-1a 64)."""
    h = 14695981039346656037
    for c in key:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def merge_keyed_torch(fp, val, dist=None, group=None):
    """Topic totals of aggregate-json states (C5 keyed): every rank's (key
    fingerprint, u32 value) pairs gathered with one all_gather (RCCL on GPU
    tensors, gloo on CPU ones), then summed per key (u32 wrapping) on the
    tensors' device.  `fp` int64 (the u64 bits), `val` int64.  Returns
    (fingerprints, sums) sorted by fingerprint, identical on every rank."""
    import torch
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        world = dist.get_world_size(group)
        n = torch.tensor([fp.numel()], dtype=torch.int64, device=fp.device)
        dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
        m = int(n.item())
        pad = m - fp.numel()
        fpp = torch.cat([fp, torch.zeros(pad, dtype=torch.int64, device=fp.device)])
        valp = torch.cat([val, torch.zeros(pad, dtype=torch.int64, device=fp.device)])
        okp = torch.cat([torch.ones(fp.numel(), dtype=torch.int64, device=fp.device),
                         torch.zeros(pad, dtype=torch.int64, device=fp.device)])
        packed = torch.stack([fpp, valp, okp])                   # one collective for the three rows
        bufs = [torch.empty_like(packed) for _ in range(world)]
        dist.all_gather(bufs, packed, group=group)
        allp = torch.cat(bufs, dim=1)
        keep = allp[2] == 1
        fp, val = allp[0][keep], allp[1][keep]
    if fp.numel() == 0:
        return fp, val
    keys, inv = torch.unique(fp, sorted=True, return_inverse=True)
    sums = torch.zeros(keys.numel(), dtype=torch.int64, device=fp.device)
    sums.index_add_(0, inv, val)
    return keys, sums & 0xFFFFFFFF
