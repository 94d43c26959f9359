"""CPU tests of the multi-GPU path: RaftGroupId placement (java.util.UUID.hashCode, RaftId.java:
119-122) and the node-wide stats all-reduce, run as a world_size-2 gloo job (the GPU job uses
the same code over RCCL).  No data-path collective exists: shards are disjoint."""
import os
import socket

import numpy as np
import pytest

from ratis_amd import shard


def java_hash(msb: int, lsb: int) -> int:
    """java.util.UUID.hashCode() written out with Java int/long semantics."""
    def to_long(x):
        x &= (1 << 64) - 1
        return x - (1 << 64) if x >> 63 else x

    def to_int(x):
        x &= (1 << 32) - 1
        return x - (1 << 32) if x >> 31 else x

    hilo = to_long(msb ^ lsb)
    return to_int(to_int(hilo >> 32) ^ to_int(hilo))


def test_uuid_hash_known_values():
    cases = [(0, 0, 0), (1, 0, 1), (-1, 0, 0), (1 << 32, 0, 1),
             (0x123456789ABCDEF0, 0x0FEDCBA987654321, None), (-(1 << 63), 5, None)]
    for msb, lsb, want in cases:
        got = int(shard.java_uuid_hash(np.array([msb], np.int64), np.array([lsb], np.int64))[0])
        assert got == java_hash(msb, lsb)
        if want is not None:
            assert got == want


def test_uuid_hash_random_matches_java_semantics():
    msb, lsb = shard.random_group_ids(5000, seed=3)
    got = shard.java_uuid_hash(msb, lsb)
    for i in range(0, 5000, 97):
        assert int(got[i]) == java_hash(int(msb[i]), int(lsb[i]))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_shards_partition_all_groups(n):
    msb, lsb = shard.random_group_ids(80_000, seed=11)
    s = shard.shard_of(msb, lsb, n)
    assert s.min() >= 0 and s.max() < n
    counts = np.bincount(s, minlength=n)
    assert counts.sum() == 80_000
    assert counts.min() > 0.9 * 80_000 / n     # hash spreads groups evenly


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import oracle as orc
        from ratis_amd import workload
        # bench.py's sharding: the job's RaftGroupIds, this rank keeps floorMod(hash, world)
        msb, lsb = shard.random_group_ids(20_000 * world, seed=workload.SEED)
        mine = np.nonzero(shard.shard_of(msb, lsb, world) == rank)[0]
        # per-rank snapshot (the GPU job runs the HIP kernel here; the CPU test uses the oracle)
        h = workload.stable_tier(mine.size, seed=workload.SEED + 1000 * rank)
        ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=-1, commit_in=h.commit,
                             term_start=h.term_start)
        adv = int(np.unpackbits(ref["advanced_bits"].view(np.uint8), bitorder="little")[: h.n].sum())
        stats = shard.allreduce_stats({"groups_evaluated": int(mine.size), "commits_advanced": adv})
        q.put((rank, int(mine.size), adv, stats, mine[:5].tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shard_and_stats_allreduce():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, n0, a0, s0, _), (_, n1, a1, s1, _) = res
    assert n0 + n1 == 40_000                      # disjoint and complete
    for s in (s0, s1):                            # every rank sees the node-wide sums
        assert s["groups_evaluated"] == 40_000
        assert s["commits_advanced"] == a0 + a1


def test_library_shard_of_matches_java_floor_mod():
    """rh_shard_of (the C ABI's RaftGroupId placement, used by rh_node routing) equals
    Math.floorMod(UUID.hashCode(), n) for every n = 1..8 -- a pure host function, no GPU."""
    from ratis_amd import groups
    msb, lsb = shard.random_group_ids(3000, seed=17)
    for n in range(1, 9):
        want = shard.shard_of(msb, lsb, n)
        got = np.array([groups.shard_of(int(a), int(b), n) for a, b in zip(msb, lsb)])
        assert np.array_equal(got, want), n
    with pytest.raises(Exception):
        groups.shard_of(1, 2, 0)
