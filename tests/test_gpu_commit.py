"""GPU parity of the batched quorum-commit kernel against the CPU oracle (bit-exact).

Every launch goes through the C ABI (rh_commit_soa_launch; the resident table is in
test_gpu_table.py).  The oracle is
oracle/ratis_oracle.c (orc_commit_soa), itself pinned in tests/test_oracle.py."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _bits(words, n):
    w = np.asarray(words).view(np.uint64)
    return np.unpackbits(w.view(np.uint8), bitorder="little")[:n].astype(bool)


def _run_gpu(ctx, follower, flush, conf, commit, ts, mode=0, gap=-1, levels=True, col_stride=None):
    import torch

    from ratis_amd import engine
    F, n = follower.shape
    dev = "cuda"
    if col_stride is not None and col_stride != n:
        big = torch.full((F, col_stride), -7, dtype=torch.int64, device=dev)
        big[:, :n] = torch.from_numpy(follower).to(dev)
        fi = big[:, :n]          # strided view: col_stride passes through the ABI
    else:
        fi = torch.from_numpy(np.ascontiguousarray(follower)).to(dev)
    t = engine.CommitTier(follower_index=fi, self_index=torch.from_numpy(flush).to(dev),
                          conf=torch.from_numpy(conf.astype(np.uint32).view(np.int32)).to(dev),
                          commit_in=torch.from_numpy(commit).to(dev), term_start=torch.from_numpy(ts).to(dev),
                          gap_threshold=gap)
    t.alloc_outputs(mode=mode, levels=levels)
    engine.commit_launch(ctx, [t], mode=mode)
    torch.cuda.synchronize()
    out = {"min": t.min_out.cpu().numpy(), "valid": _bits(t.valid_bits.cpu().numpy(), n)}
    if mode == 0:
        out["commit"] = t.commit_out.cpu().numpy()
        out["adv"] = _bits(t.advanced_bits.cpu().numpy(), n)
    if levels or mode == 1:
        out["maj"] = t.maj_out.cpu().numpy()
        out["max"] = t.max_out.cpu().numpy()
    return out


def _check(ctx, orc, follower, flush, conf, commit, ts, mode=0, gap=-1, col_stride=None):
    got = _run_gpu(ctx, follower, flush, conf, commit, ts, mode=mode, gap=gap, col_stride=col_stride)
    ref = orc.commit_soa(follower, flush, conf, mode=mode, gap=gap,
                         commit_in=commit if mode == 0 else None, term_start=ts if mode == 0 else None)
    n = flush.size
    v_ref = _bits(ref["valid_bits"], n)
    assert np.array_equal(got["valid"], v_ref)
    assert np.array_equal(got["min"], ref["min"])
    assert np.array_equal(got["maj"], ref["maj"])
    assert np.array_equal(got["max"], ref["max"])
    if mode == 0:
        assert np.array_equal(got["commit"], ref["commit"])
        assert np.array_equal(got["adv"], _bits(ref["advanced_bits"], n))
    return got


def _random_case(rng, F, n, lo=-1, hi=60, full_masks=False):
    follower = rng.integers(lo, hi, size=(F, n)).astype(np.int64)
    flush = rng.integers(lo, hi, size=n).astype(np.int64)
    commit = rng.integers(lo, hi, size=n).astype(np.int64)
    ts = rng.integers(0, hi, size=n).astype(np.int64)
    fm = (1 << F) - 1
    newm = rng.integers(0, 1 << F, size=n).astype(np.uint32)
    oldm = rng.integers(0, 1 << F, size=n).astype(np.uint32)
    flags = rng.integers(0, 16, size=n).astype(np.uint32)
    if full_masks:
        newm[:] = fm
    conf = ((newm & fm) | ((flags & 1) << 14) | (((flags >> 1) & 1) << 15) | ((oldm & fm) << 16)
            | (((flags >> 2) & 1) << 30) | (np.uint32(1) << 31)).astype(np.uint32)
    inactive = rng.random(n) < 0.05
    conf[inactive] &= np.uint32(0x7FFFFFFF)
    return follower, flush, conf, commit, ts


@pytest.mark.parametrize("F", list(range(1, 15)))
def test_every_follower_width(ctx, orc, F):
    rng = np.random.default_rng(100 + F)
    n = 3001  # ragged: not a multiple of the 512-group tile
    for gap in (-1, 0, 9):
        _check(ctx, orc, *_random_case(rng, F, n), mode=0, gap=gap)
    _check(ctx, orc, *_random_case(rng, F, n), mode=1)


def test_golden_cases_on_gpu(ctx, orc):
    cases = json.load(open(os.path.join(HERE, "golden", "commit_cases.json")))["cases"]
    F = 4
    n = len(cases)
    follower = np.full((F, n), -1, dtype=np.int64)
    flush = np.zeros(n, dtype=np.int64)
    commit = np.zeros(n, dtype=np.int64)
    ts = np.zeros(n, dtype=np.int64)
    conf = np.zeros(n, dtype=np.uint32)
    gaps = set(c["gap"] for c in cases)
    for gap in gaps:
        idx = [i for i, c in enumerate(cases) if c["gap"] == gap]
        for j, i in enumerate(idx):
            c = cases[i]
            k = len(c["followers"])
            follower[:k, i] = c["followers"]
            flush[i] = c["self_index"]
            commit[i] = c["last_committed"]
            ts[i] = c["term_start"]
            nm = sum(b << q for q, b in enumerate(c["in_new"]))
            om = sum(b << q for q, b in enumerate(c["in_old"]))
            conf[i] = nm | (c["include_self"] << 14) | (c["transitional"] << 15) | (om << 16) | (
                c["include_self_old"] << 30) | (1 << 31)
        got = _run_gpu(ctx, follower[:, idx], flush[idx], conf[idx], commit[idx], ts[idx], mode=0, gap=gap)
        for j, i in enumerate(idx):
            c = cases[i]
            exp = c["expected"]
            assert got["valid"][j] == (exp is not None), c["name"]
            if exp is not None:
                assert (got["min"][j], got["maj"][j], got["max"][j]) == (exp["min"], exp["majority"], exp["max"]), c["name"]
            assert got["commit"][j] == c["expected_commit"], c["name"]


def test_extreme_values_and_ties(ctx, orc):
    rng = np.random.default_rng(11)
    F, n = 6, 4096
    pool = np.array([-(1 << 63), -2, -1, 0, 1, 2, (1 << 62), (1 << 63) - 1], dtype=np.int64)
    follower = pool[rng.integers(0, pool.size, size=(F, n))]
    flush = pool[rng.integers(0, pool.size, size=n)]
    commit = pool[rng.integers(0, pool.size, size=n)]
    ts = pool[rng.integers(0, pool.size, size=n)]
    _, _, conf, _, _ = _random_case(rng, F, n)
    for gap in (-1, 0, 1, (1 << 63) - 1):
        _check(ctx, orc, follower, flush, conf, commit, ts, mode=0, gap=gap)


def test_padded_column_stride_scalar_path(ctx, orc):
    rng = np.random.default_rng(12)
    F, n = 4, 1000
    _check(ctx, orc, *_random_case(rng, F, n), mode=0, gap=3, col_stride=1027)  # odd stride: no 16-B loads


def test_fused_multi_tier_launch_and_compaction(ctx, orc):
    import torch

    from ratis_amd import engine, workload
    tiers_h = workload.commit_snapshot(200_000, joint_frac=0.1, peers=5, seed=77)
    tiers_h.append(workload.stable_tier(50_000, seed=78, peers=3))
    tiers_h.append(workload.stable_tier(7_777, seed=79, peers=9))   # F=8: second kernel class
    tiers = []
    total = sum(t.n for t in tiers_h)
    adv_rows = torch.empty(total, dtype=torch.int64, device="cuda")
    adv_commit = torch.empty(total, dtype=torch.int64, device="cuda")
    adv_count = torch.zeros(1, dtype=torch.int64, device="cuda")
    base = 0
    for h in tiers_h:
        t = workload.to_device(h, gap_threshold=2048).alloc_outputs(mode=0, levels=True)
        t.adv_rows, t.adv_commit, t.adv_count, t.adv_row_base = adv_rows, adv_commit, adv_count, base
        base += h.n
        tiers.append(t)
    engine.commit_launch(ctx, tiers, mode=0)
    torch.cuda.synchronize()
    all_adv = []
    base = 0
    for h, t in zip(tiers_h, tiers):
        ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=2048, commit_in=h.commit, term_start=h.term_start)
        assert np.array_equal(t.commit_out.cpu().numpy(), ref["commit"])
        assert np.array_equal(t.min_out.cpu().numpy(), ref["min"])
        assert np.array_equal(t.maj_out.cpu().numpy(), ref["maj"])
        assert np.array_equal(t.max_out.cpu().numpy(), ref["max"])
        adv = _bits(ref["advanced_bits"], h.n)
        assert np.array_equal(_bits(t.advanced_bits.cpu().numpy(), h.n), adv)
        assert np.array_equal(_bits(t.valid_bits.cpu().numpy(), h.n), _bits(ref["valid_bits"], h.n))
        all_adv.append(np.nonzero(adv)[0] + base)
        base += h.n
    k = int(adv_count.item())
    exp_rows = np.concatenate(all_adv)
    assert k == exp_rows.size and k > 0
    rows = adv_rows[:k].cpu().numpy()
    order = np.argsort(rows)
    assert np.array_equal(rows[order], exp_rows)
    commits = np.concatenate([t.commit_out.cpu().numpy() for t in tiers])
    assert np.array_equal(adv_commit[:k].cpu().numpy()[order], commits[exp_rows])


def test_full_size_config3_parity(ctx, orc):
    """BASELINE config 3 at full size: 1M groups x 5 peers, 10% joint, both gap settings."""
    import torch

    from ratis_amd import engine, workload
    tiers_h = workload.commit_snapshot(1_000_000, joint_frac=0.1, peers=5)
    for gap in (-1, 2048):
        tiers = [workload.to_device(h, gap_threshold=gap).alloc_outputs(mode=0) for h in tiers_h]
        engine.commit_launch(ctx, tiers, mode=0)
        torch.cuda.synchronize()
        for h, t in zip(tiers_h, tiers):
            ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=gap, commit_in=h.commit,
                                 term_start=h.term_start)
            assert np.array_equal(t.commit_out.cpu().numpy(), ref["commit"])
            assert np.array_equal(t.min_out.cpu().numpy(), ref["min"])
            adv = _bits(ref["advanced_bits"], h.n)
            assert np.array_equal(_bits(t.advanced_bits.cpu().numpy(), h.n), adv)
            assert 0.01 < adv.mean() < 0.99   # both branches of the commit decision are exercised


def test_full_size_config2_parity(ctx, orc):
    """BASELINE config 2 at full size: 100k groups x 3 peers (stable confs), both gap settings."""
    import torch

    from ratis_amd import engine, workload
    tiers_h = workload.commit_snapshot(100_000, joint_frac=0.0, peers=3)
    for gap in (-1, 2048):
        tiers = [workload.to_device(h, gap_threshold=gap).alloc_outputs(mode=0) for h in tiers_h]
        engine.commit_launch(ctx, tiers, mode=0)
        torch.cuda.synchronize()
        for h, t in zip(tiers_h, tiers):
            ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=gap, commit_in=h.commit,
                                 term_start=h.term_start)
            assert np.array_equal(t.commit_out.cpu().numpy(), ref["commit"])
            assert np.array_equal(t.min_out.cpu().numpy(), ref["min"])


def test_full_size_config4_sharded(ctx, orc):
    """BASELINE config 4 at full size: 8M groups x 5 peers (10 % joint) placed on 8 shards by
    floorMod(RaftGroupId.hashCode(), 8) (shard.py), each shard launched on its own as one rank
    would.  Every shard equals the oracle, and the shards together equal one launch over all 8M
    groups (groups are independent: sharding changes nothing)."""
    import torch

    from ratis_amd import engine, shard, workload
    n = 8_000_000
    tiers_h = workload.commit_snapshot(n, joint_frac=0.1, peers=5, seed=workload.SEED + 4)
    msb, lsb = shard.random_group_ids(n, seed=44)
    sh = shard.shard_of(msb, lsb, 8)
    counts = np.bincount(sh, minlength=8)
    assert counts.min() > 0.95 * n / 8 and counts.max() < 1.05 * n / 8   # hash spreads evenly
    off = 0
    whole = {}
    for ti, h in enumerate(tiers_h):
        idx_all = np.arange(off, off + h.n)
        off += h.n
        ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=-1, commit_in=h.commit,
                             term_start=h.term_start)
        got_commit = np.empty(h.n, np.int64)
        got_min = np.empty(h.n, np.int64)
        for r in range(8):
            sel = np.nonzero(sh[idx_all] == r)[0]
            part = workload.HostTier(h.follower[:, sel], h.flush[sel], h.commit[sel], h.term_start[sel],
                                     h.conf[sel], h.voters_union[sel])
            t = workload.to_device(part).alloc_outputs(mode=0)
            engine.commit_launch(ctx, [t], mode=0)
            torch.cuda.synchronize()
            got_commit[sel] = t.commit_out.cpu().numpy()
            got_min[sel] = t.min_out.cpu().numpy()
            del t
        assert np.array_equal(got_commit, ref["commit"]), ti
        assert np.array_equal(got_min, ref["min"]), ti
        whole[ti] = got_commit
    tiers = [workload.to_device(h).alloc_outputs(mode=0) for h in tiers_h]
    engine.commit_launch(ctx, tiers, mode=0)
    torch.cuda.synchronize()
    for ti, t in enumerate(tiers):
        assert np.array_equal(t.commit_out.cpu().numpy(), whole[ti])


@pytest.mark.parametrize("F", [1, 2, 4, 6, 7, 13])
def test_malformed_conf_words_raw_launch(ctx, orc, F):
    """a conf word naming a follower slot >= F (new or old mask) on the raw
    rh_commit_soa_launch path is malformed for the tier: no result, no commit advance (never a
    majority over fewer voters), exactly as the oracle's SoA driver rules."""
    rng = np.random.default_rng(500 + F)
    n = 5000
    follower, flush, conf, commit, ts = _random_case(rng, F, n)
    extra_new = (rng.integers(1, 1 << (14 - F), size=n) << F).astype(np.uint32) if F < 14 else 0
    extra_old = (rng.integers(1, 1 << (14 - F), size=n) << F).astype(np.uint32) if F < 14 else 0
    which = rng.integers(0, 4, size=n)
    conf = conf | np.where(which == 1, extra_new, 0).astype(np.uint32)
    conf = conf | (np.where(which == 2, extra_old, 0).astype(np.uint32) << 16)
    conf = conf.astype(np.uint32)
    got = _check(ctx, orc, follower, flush, conf, commit, ts, mode=0, gap=-1)
    bad = (which == 1) | (which == 2)
    assert not got["valid"][bad].any()
    assert np.array_equal(got["commit"][bad], commit[bad])
    assert got["valid"][~bad].any()


@pytest.mark.parametrize("F", [1, 2, 4, 6, 7, 11, 14])
def test_tiled_layout(ctx, orc, F):
    """rh_commit_soa.tile_stride (AoSoA tiles of 128 groups) gives the plain layout's results:
    both gap settings, COMMIT and WATCH (levels), a ragged last tile."""
    import torch

    from ratis_amd import engine
    rng = np.random.default_rng(700 + F)
    n = 128 * 37 + 45
    follower, flush, conf, commit, ts = _random_case(rng, F, n)
    for mode, gap in ((0, -1), (0, 9), (1, -1)):
        t = engine.TiledCommitTier.from_arrays(follower, flush, conf, commit, ts, gap_threshold=gap, levels=True)
        engine.commit_launch(ctx, [t], mode=mode)
        torch.cuda.synchronize()
        ref = orc.commit_soa(follower, flush, conf, mode=mode, gap=gap,
                             commit_in=commit if mode == 0 else None, term_start=ts if mode == 0 else None)
        assert np.array_equal(_bits(t.valid_bits.cpu().numpy(), n), _bits(ref["valid_bits"], n))
        for col, key in (("min_out", "min"), ("maj_out", "maj"), ("max_out", "max")):
            assert np.array_equal(t.column(col).cpu().numpy(), ref[key]), col
        if mode == 0:
            assert np.array_equal(t.column("commit_out").cpu().numpy(), ref["commit"])
            assert np.array_equal(_bits(t.advanced_bits.cpu().numpy(), n), _bits(ref["advanced_bits"], n))
        # the inputs are untouched (outputs live in their own columns of each tile)
        assert np.array_equal(t.column("self").cpu().numpy(), flush)


def test_tiled_layout_config3_full_size(ctx, orc):
    """BASELINE config 3 (1M groups x 5 peers, 10 % joint: an F=4 and an F=6 tier in one launch)
    in the tiled layout, every group against the oracle."""
    import torch

    from ratis_amd import engine, workload
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 3)
    tiers = [workload.to_device_tiled(h) for h in host]
    engine.commit_launch(ctx, tiers)
    torch.cuda.synchronize()
    for h, t in zip(host, tiers):
        ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=-1, commit_in=h.commit, term_start=h.term_start)
        assert np.array_equal(t.column("commit_out").cpu().numpy(), ref["commit"])
        assert np.array_equal(t.column("min_out").cpu().numpy(), ref["min"])


def test_tiled_layout_rejects_bad_strides(ctx):
    from ratis_amd import _lib, engine
    rng = np.random.default_rng(5)
    t = engine.TiledCommitTier.from_arrays(*_random_case(rng, 4, 300))
    s = t.to_struct(0)
    for field, bad in (("tile_stride", s.tile_stride + 8), ("col_stride", 64), ("tile_stride", 512)):
        arr = (_lib.RhCommitSoa * 1)(t.to_struct(0))
        setattr(arr[0], field, bad)
        assert _lib.load().rh_commit_soa_launch(ctx.handle, arr, 1, None) == _lib.RH_E_INVAL


def test_prepared_launches_match_per_call_launches(ctx, orc):
    """engine.prepare_commit / prepare_lease / prepare_leader (argument arrays built once, as the
    bench's timed loops use them) give the oracle's results, launched repeatedly."""
    import torch

    from ratis_amd import engine, workload
    host = workload.commit_snapshot(30_000, joint_frac=0.10, peers=5, seed=91)
    ct = [engine.TiledCommitTier.from_arrays(h.follower, h.flush, h.conf, h.commit, h.term_start) for h in host]
    now, rng = 1 << 60, np.random.default_rng(92)
    lin = [now - rng.integers(0, 200_000_000, size=h.n, dtype=np.int64) for h in host]
    ts = [now - rng.integers(-1_000_000, 300_000_000, size=h.follower.shape, dtype=np.int64) for h in host]
    lt = [engine.TiledLeaseTier.from_arrays(t, h.conf, li) for t, h, li in zip(ts, host, lin)]
    launches = (engine.prepare_commit(ct), engine.prepare_lease(lt, now, 100), engine.prepare_leader(ct, lt, now, 100))
    for k, p in enumerate(launches):
        for _ in range(3):
            p(ctx)
        torch.cuda.synchronize()
        for h, c, l, t, li in zip(host, ct, lt, ts, lin):
            rc = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, commit_in=h.commit, term_start=h.term_start)
            assert np.array_equal(c.column("commit_out").cpu().numpy(), rc["commit"])
            if k >= 1:   # the lease half has run
                rl = orc.lease_soa(t, h.conf, li, now, 100)
                assert np.array_equal(l.lease_out.cpu().numpy(), rl["lease"])
                nw = (h.n + 63) // 64
                assert np.array_equal(l.has_lease_bits[:nw].cpu().numpy().view(np.uint64), rl["has_lease_bits"])
