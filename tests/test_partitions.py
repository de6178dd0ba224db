"""Partition sharding and the aggregate-state merge, CPU only.

The producer's key routing (crates/fluvio/src/producer/partitioning.rs:51-83),
rank ownership p -> rank p mod N, and the all-reduce merge of per-partition
aggregate accumulators, run as two gloo ranks on the CPU.  Per-partition states
come from the CPU oracle (aggregate-sum chains, one per partition, like the
SPU's per-partition SmartModuleContext, context.rs:25-30); the merged vector
must equal the single-process table over all partitions.
"""
import os
import socket

import pytest

from fluvio_amd import partitions as PT
from fluvio_amd import protocol as P

N_PART = 8


def test_siphash24_reference_vectors():
    # SipHash paper, Appendix A (key 00..0f): empty input and the 15-byte 00..0e example
    k0 = int.from_bytes(bytes(range(8)), "little")
    k1 = int.from_bytes(bytes(range(8, 16)), "little")
    assert PT.siphash24(b"", k0, k1) == 0x726FDB47DD0E0E31
    assert PT.siphash24(bytes(range(15)), k0, k1) == 0xA129CA6149BE45E5


def test_round_robin_like_reference():
    # partitioning.rs:104-121 (test_round_robin_individual)
    rr = PT.RoundRobin()
    assert [rr.partition(None, 3) for _ in range(6)] == [0, 1, 2, 0, 1, 2]
    # keyed records are stable per key, spread over the partitions
    ps = {PT.partition_siphash(f"key-{i}".encode(), N_PART) for i in range(200)}
    assert ps == set(range(N_PART))
    assert PT.partition_siphash(b"abc", 64) == PT.partition_siphash(b"abc", 64)


def test_ownership_covers_every_partition_once():
    for world in (1, 2, 3, 8):
        seen = sorted(p for r in range(world) for p in PT.owned_partitions(64, world, r))
        assert seen == list(range(64))


def topic_records(n=3000, seed=5):
    import random
    rng = random.Random(seed)
    return [(f"user-{rng.randrange(500)}".encode(), str(rng.randrange(-1000, 1001)).encode()) for _ in range(n)]


def partition_slice(recs, base=0):
    """Stored batches of one partition (~16 KB record sections)."""
    out, b, off = b"", P.Batch(base_offset=base), base
    for k, v in recs:
        b.add_record(P.Record.new_key_value(k, v))
        if len(b.records) == 200:
            out += b.encode()
            off += len(b.records)
            b = P.Batch(base_offset=off)
    if b.records:
        out += b.encode()
    return out


def partition_states(owned, routed):
    from oracle.oracle import OracleChain
    states = {}
    for p in owned:
        ch = OracleChain([("aggregate-sum", {}, None)])
        r = ch.process_batch(partition_slice(routed[p]))
        assert r["status"] == 0 and r["error"] is None
        acc = ch.accumulator(0)
        states[p] = int(acc) if acc else 0
    return states


def _rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    routed = PT.route(topic_records(), N_PART, key_of=lambda r: r[0])
    owned = PT.owned_partitions(N_PART, world, rank)
    vec = PT.local_state_vector(N_PART, partition_states(owned, routed))
    merged = PT.merge_states_torch(vec)
    with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
        f.write(" ".join(map(str, merged)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(180)
def test_two_rank_state_merge(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    routed = PT.route(topic_records(), N_PART, key_of=lambda r: r[0])
    expect = PT.local_state_vector(N_PART, partition_states(range(N_PART), routed))
    assert any(expect)
    for r in range(world):
        got = [int(x) for x in open(tmp_path / f"rank{r}.txt").read().split()]
        assert got == expect
    # each partition's state is the running i32 sum of its own records only
    for p in range(N_PART):
        assert expect[p] == PT.wrap_i32(sum(int(v) for _, v in routed[p]))


# ---------------------------------------------------------------------------
# C5 keyed (aggregate-json): per-key u32 sums, keys routed by SipHash so a key
# lives in one partition; the topic-wide table = all ranks' (fingerprint, value)
# key lists gathered, the union dictionary, a dense all-reduce (partitions.merge_keyed,
# the shape of fsg_keyed_allreduce)
# ---------------------------------------------------------------------------
K_PART, K_REC, K_KEYS = 8, 1500, 64


def keyed_pairs(owned):
    """This rank's keyed table: the oracle's aggregate-json accumulator (the
    pretty map after the partition's last record) of every owned partition,
    summed by exact key (a key lives in one partition)."""
    import json
    from fluvio_amd import synth
    from oracle.oracle import OracleChain
    slices = synth.make_keyed_slices(K_PART, K_REC, K_KEYS, owned=list(owned))
    local = {}
    for p in owned:
        ch = OracleChain([("aggregate-json", {}, None)])
        r = ch.process_batch(slices[p])
        assert r["status"] == 0 and r["error"] is None
        for k, v in json.loads(ch.accumulator(0)).items():
            local[k.encode()] = (local.get(k.encode(), 0) + v) & 0xFFFFFFFF
    return local


def keyed_expect():
    """Per-key totals straight from the generated records (all partitions)."""
    import json
    from fluvio_amd import synth
    tot = {}
    for p, sl in synth.make_keyed_slices(K_PART, K_REC, K_KEYS).items():
        for b in P.decode_batches(sl):
            for rec in b.memory_records():
                for k, v in json.loads(rec.value).items():
                    assert PT.partition_siphash(k.encode(), K_PART) == p  # routed by key
                    tot[k.encode()] = (tot.get(k.encode(), 0) + v) & 0xFFFFFFFF
    return tot


def _keyed_rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    merged = PT.merge_keyed(keyed_pairs(PT.owned_partitions(K_PART, world, rank)), dist=dist)
    with open(os.path.join(outdir, f"keyed{rank}.txt"), "w") as f:
        f.write(" ".join(f"{k.decode()}:{v}" for k, v in merged.items()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_keyed_merge(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_keyed_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    expect = keyed_expect()
    assert len(expect) > K_PART
    for r in range(world):
        got = {k.encode(): int(v) for k, v in (x.split(":") for x in open(tmp_path / f"keyed{r}.txt").read().split())}
        assert got == expect


@pytest.mark.parametrize("nr", range(2, 9))
def test_union_of_simulated_ranks(nr):
    """The union step of fsg_keyed_allreduce on N = 2..8 simulated gathered key
    lists (unequal counts, shared and disjoint keys, dead entries, padding to
    maxn / maxb) against a host union built straight from the key lists."""
    import random
    rng = random.Random(nr)
    pool = [b"k%03d" % i for i in range(60)] + [b"", b"x" * 40, "é".encode()]
    lists = []
    for r in range(nr):
        n = rng.choice([0, 1, 5, 17, 40])
        ks = rng.sample(pool, min(n, len(pool)))
        lists.append([None if rng.random() < 0.1 else k for k in ks])
    sends = [PT.keyed_desc(ks) for ks in lists]
    maxn, maxb = PT.gather_shape([(len(d), len(a)) for d, a in sends])
    gdesc, garena = [], b""
    for d, a in sends:
        gdesc += d + [PT.KD_LEN_DEAD << 40] * (maxn - len(d))
        garena += a + bytes(maxb - len(a))
    gid, ukeys = PT.union_from_gathered(gdesc, garena, maxn, maxb)
    expect = PT.union_dictionary([[k for k in ks if k is not None] for ks in lists])
    assert ukeys == list(expect)
    for r, ks in enumerate(lists):
        for i, k in enumerate(ks):
            assert gid[r * maxn + i] == (None if k is None else expect[k])
        for i in range(len(ks), maxn):
            assert gid[r * maxn + i] is None
