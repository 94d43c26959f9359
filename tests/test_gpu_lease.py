"""GPU parity of the batched leader-lease kernel (rh_lease_soa_launch) against the oracle's literal
LeaderStateImpl.hasLease / LeaderLease.extend restatement (orc_lease_soa, cross-checked against
an independent Python restatement in tests/test_oracle.py).  Bit-exact: lease timestamps,
hasLease bits and extended bits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MS = 1_000_000
NOW = 1_700_000_000_000_000_000


def random_lease_tier(rng, n, F, timeout_ms=100, joint_rate=0.2, boundary_rate=0.05):
    ts = NOW - rng.integers(-5 * MS, 3 * timeout_ms * MS, size=(F, n), dtype=np.int64)
    if F:   # exact millisecond boundaries of the activity test
        m = rng.random((F, n)) < boundary_rate
        ts[m] = NOW - timeout_ms * MS + rng.integers(-1, 2, int(m.sum()))
    full = (1 << F) - 1
    new = rng.integers(0, full + 1, n) if F else np.zeros(n, np.int64)
    old = rng.integers(0, full + 1, n) if F else np.zeros(n, np.int64)
    self_new = rng.random(n) < 0.9
    trans = rng.random(n) < joint_rate
    self_old = rng.random(n) < 0.8
    active = rng.random(n) < 0.97
    conf = (new | (self_new.astype(np.int64) << 14) | (trans.astype(np.int64) << 15) | (old << 16)
            | (self_old.astype(np.int64) << 30) | (active.astype(np.int64) << 31)).astype(np.uint32)
    lease_in = NOW - rng.integers(0, 2 * timeout_ms * MS, n, dtype=np.int64)
    return ts, conf, lease_in


def run_gpu(ctx, ts, conf, lease_in, timeout_ms, enabled=None, alias=False, pad=0):
    import torch

    from ratis_amd import engine
    dev = torch.device("cuda")
    F, n = ts.shape
    tsd = torch.zeros((F, n + pad), dtype=torch.int64, device=dev)
    tsd[:, :n] = torch.from_numpy(ts)
    t = engine.LeaseTier(follower_ts=tsd, conf=torch.from_numpy(conf.view(np.int32)).to(dev),
                         lease_in=torch.from_numpy(lease_in).to(dev),
                         enabled_bits=None if enabled is None else torch.from_numpy(enabled.view(np.int64)).to(dev))
    if alias:
        t.lease_out = t.lease_in
    t.alloc_outputs()
    engine.lease_launch(ctx, [t], NOW, timeout_ms)
    torch.cuda.synchronize()
    nw = (n + 63) // 64
    return (t.lease_out.cpu().numpy(), t.has_lease_bits[:nw].cpu().numpy().view(np.uint64),
            t.extended_bits[:nw].cpu().numpy().view(np.uint64))


def assert_same(ref, got):
    lease, has, ext = got
    assert np.array_equal(lease, ref["lease"])
    assert np.array_equal(has, ref["has_lease_bits"])
    assert np.array_equal(ext, ref["extended_bits"])


@pytest.mark.parametrize("F", list(range(0, 15)))
def test_lease_every_follower_count(ctx, orc, F):
    rng = np.random.default_rng(1000 + F)
    n = 20_000 + F * 37          # not a multiple of 64
    ts, conf, lease_in = random_lease_tier(rng, n, F)
    en = rng.integers(0, 1 << 63, (n + 63) // 64, dtype=np.int64).astype(np.uint64) | np.uint64(0xF0F0F0F0F0F0F0F0)
    ref = orc.lease_soa(ts, conf, lease_in, NOW, 100, en)
    assert_same(ref, run_gpu(ctx, ts, conf, lease_in, 100, enabled=en))
    ref = orc.lease_soa(ts, conf, lease_in, NOW, 100)
    assert_same(ref, run_gpu(ctx, ts, conf, lease_in, 100, alias=True, pad=45))


@pytest.mark.parametrize("timeout_ms", [0, 1, 100, 5000])
def test_lease_timeouts_and_extremes(ctx, orc, timeout_ms):
    rng = np.random.default_rng(timeout_ms)
    n, F = 5000, 4
    ts, conf, lease_in = random_lease_tier(rng, n, F, timeout_ms=max(timeout_ms, 1), joint_rate=0.5)
    # far-past and slightly-future timestamps (|now - t| well below 2^62)
    ts[0, ::11] = NOW - (1 << 61)
    ts[1, ::13] = NOW + 3 * MS
    lease_in[::17] = NOW + 2 * MS
    lease_in[::19] = NOW - (1 << 60)
    ref = orc.lease_soa(ts, conf, lease_in, NOW, timeout_ms)
    assert_same(ref, run_gpu(ctx, ts, conf, lease_in, timeout_ms))


def test_lease_multi_tier_and_counts(ctx, orc):
    import torch

    from ratis_amd import engine
    rng = np.random.default_rng(77)
    tiers, refs = [], []
    for F, n in ((2, 70_001), (4, 900_000), (9, 3_333), (6, 100_000)):
        ts, conf, lease_in = random_lease_tier(rng, n, F)
        refs.append(orc.lease_soa(ts, conf, lease_in, NOW, 150))
        t = engine.LeaseTier(follower_ts=torch.from_numpy(ts).cuda(), conf=torch.from_numpy(conf.view(np.int32)).cuda(),
                             lease_in=torch.from_numpy(lease_in).cuda()).alloc_outputs()
        tiers.append(t)
    engine.lease_launch(ctx, tiers, NOW, 150)
    torch.cuda.synchronize()
    for t, ref in zip(tiers, refs):
        nw = (t.n + 63) // 64
        assert np.array_equal(t.lease_out.cpu().numpy(), ref["lease"])
        assert np.array_equal(t.has_lease_bits[:nw].cpu().numpy().view(np.uint64), ref["has_lease_bits"])
        assert np.array_equal(t.extended_bits[:nw].cpu().numpy().view(np.uint64), ref["extended_bits"])


def test_lease_bad_arguments(ctx):
    import torch

    from ratis_amd import _lib, engine
    t = engine.LeaseTier(follower_ts=torch.zeros((15, 8), dtype=torch.int64, device="cuda"),
                         conf=torch.zeros(8, dtype=torch.int32, device="cuda"),
                         lease_in=torch.zeros(8, dtype=torch.int64, device="cuda")).alloc_outputs()
    with pytest.raises(_lib.IllegalArgumentError):
        engine.lease_launch(ctx, [t], NOW, 100)
    t2 = engine.LeaseTier(follower_ts=torch.zeros((2, 8), dtype=torch.int64, device="cuda"),
                          conf=torch.zeros(8, dtype=torch.int32, device="cuda"),
                          lease_in=torch.zeros(8, dtype=torch.int64, device="cuda")).alloc_outputs()
    with pytest.raises(_lib.IllegalArgumentError):
        engine.lease_launch(ctx, [t2], NOW, -1)


@pytest.mark.parametrize("timeout_ms", [0, 1, 7, 9_223_372_036_854, 9_223_372_036_855, (1 << 62)])
def test_lease_ms_threshold_exact(ctx, orc, timeout_ms):
    """The kernel's division-free form of elapsedTimeMs < timeout (d <= lim(T)) at every edge of the
    truncating millisecond division: d = k*10^6 - 1, k*10^6, k*10^6 + 1 for k around T and around
    -1, 0, and the saturation of T*10^6 near INT64_MAX."""
    rng = np.random.default_rng(5 + timeout_ms % 1000)
    T = min(timeout_ms, 9_223_372_036_854)
    ks = [-2, -1, 0, 1, T - 1, T, T + 1]
    ds = sorted({k * MS + e for k in ks for e in (-1, 0, 1) if abs(k * MS + e) < (1 << 62)})
    n, F = 4 * len(ds) * 8, 4
    ts, conf, lease_in = random_lease_tier(rng, n, F, timeout_ms=100, joint_rate=0.3)
    pick = np.array(ds, dtype=np.int64)
    ts[:, :] = NOW - pick[rng.integers(0, len(ds), size=(F, n))]
    lease_in[:] = NOW - pick[rng.integers(0, len(ds), size=n)]
    ref = orc.lease_soa(ts, conf, lease_in, NOW, timeout_ms)
    assert_same(ref, run_gpu(ctx, ts, conf, lease_in, timeout_ms))


@pytest.mark.parametrize("F", [0, 1, 4, 7, 9])
def test_lease_malformed_conf_words(ctx, orc, F):
    """A conf word naming a follower slot >= F is malformed for the tier: no lease, no extension,
    lease unchanged -- the same rule as the commit kernel and the oracle."""
    rng = np.random.default_rng(77 + F)
    n = 4096
    ts, conf, lease_in = random_lease_tier(rng, n, F)
    which = rng.integers(0, 3, size=n)
    hi_new = np.uint32(1 << F) if F < 14 else np.uint32(0)
    conf = (conf | np.where(which == 1, hi_new, 0).astype(np.uint32)
            | (np.where(which == 2, hi_new, 0).astype(np.uint32) << 16)).astype(np.uint32)
    got = run_gpu(ctx, ts, conf, lease_in, 100)
    assert_same(orc.lease_soa(ts, conf, lease_in, NOW, 100), got)
    bad = which > 0
    has = np.unpackbits(got[1].view(np.uint8), bitorder="little")[:n].astype(bool)
    assert not has[bad].any() and np.array_equal(got[0][bad], lease_in[bad])


def test_leader_fused_launch_equals_separate(ctx, orc):
    """rh_leader_soa_launch (updateCommit + hasLease of the same divisions in one kernel, wider
    tiers in their own launches) gives exactly the oracle's commit and lease results."""
    import torch

    from ratis_amd import engine, workload
    rng = np.random.default_rng(31)
    tiers_h = workload.commit_snapshot(150_000, joint_frac=0.1, peers=5, seed=41)
    tiers_h.append(workload.stable_tier(5_000, seed=42, peers=10))   # F = 9: outside the fused classes
    ctiers = [workload.to_device(h, gap_threshold=2048).alloc_outputs(mode=0) for h in tiers_h]
    lease_in = []
    ltiers = []
    for h in tiers_h:
        ts = NOW - rng.integers(-5 * MS, 300 * MS, size=h.follower.shape, dtype=np.int64)
        lin = NOW - rng.integers(0, 200 * MS, h.n, dtype=np.int64)
        lease_in.append((ts, h.conf, lin))
        ltiers.append(engine.LeaseTier(follower_ts=torch.from_numpy(ts).cuda(),
                                       conf=torch.from_numpy(h.conf.view(np.int32)).cuda(),
                                       lease_in=torch.from_numpy(lin).cuda()).alloc_outputs())
    engine.leader_launch(ctx, ctiers, ltiers, NOW, 100)
    torch.cuda.synchronize()
    for h, t in zip(tiers_h, ctiers):
        ref = orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=2048, commit_in=h.commit, term_start=h.term_start)
        assert np.array_equal(t.commit_out.cpu().numpy(), ref["commit"])
        assert np.array_equal(t.min_out.cpu().numpy(), ref["min"])
    for (ts, conf, lin), t in zip(lease_in, ltiers):
        nw = (t.n + 63) // 64
        got = (t.lease_out.cpu().numpy(), t.has_lease_bits[:nw].cpu().numpy().view(np.uint64),
               t.extended_bits[:nw].cpu().numpy().view(np.uint64))
        assert_same(orc.lease_soa(ts, conf, lin, NOW, 100), got)


@pytest.mark.parametrize("F", [0, 1, 3, 4, 6, 7, 8, 11, 14])
def test_lease_tiled_layout(ctx, orc, F):
    """The TILED layout (rh_lease_soa.tile_stride: 128-group tiles holding every per-group column)
    gives the oracle's results for every follower-count class, incl. a partial last tile and an
    enabled-bit column."""
    import torch

    from ratis_amd import engine
    rng = np.random.default_rng(3000 + F)
    n = 9_000 + 77 * F            # partial last tile, not a multiple of 64
    ts, conf, lease_in = random_lease_tier(rng, n, F)
    en = rng.integers(0, 1 << 63, (n + 63) // 64, dtype=np.int64).astype(np.uint64) | np.uint64(0x0FF00FF00FF00FF0)
    t = engine.TiledLeaseTier.from_arrays(ts, conf, lease_in)
    t.enabled_bits = torch.from_numpy(en.view(np.int64)).cuda()
    engine.lease_launch(ctx, [t], NOW, 100)
    torch.cuda.synchronize()
    nw = (n + 63) // 64
    ref = orc.lease_soa(ts, conf, lease_in, NOW, 100, en)
    assert_same(ref, (t.lease_out.cpu().numpy(), t.has_lease_bits[:nw].cpu().numpy().view(np.uint64),
                      t.extended_bits[:nw].cpu().numpy().view(np.uint64)))


def test_leader_launch_tiled_commit_and_lease(ctx, orc):
    """rh_leader_soa_launch over tiled commit tiers and tiled lease tiers of the same groups (the
    bench's fused configuration) equals the oracle on both halves."""
    import torch

    from ratis_amd import engine, workload
    host = workload.commit_snapshot(40_000, joint_frac=0.10, peers=5, seed=77)
    rng = np.random.default_rng(78)
    ctiers, ltiers, refs = [], [], []
    for h in host:
        ct = engine.TiledCommitTier.from_arrays(h.follower, h.flush, h.conf, h.commit, h.term_start)
        ts = NOW - rng.integers(-MS, 300 * MS, size=h.follower.shape, dtype=np.int64)
        lin = NOW - rng.integers(0, 200 * MS, size=h.n, dtype=np.int64)
        ctiers.append(ct)
        ltiers.append(engine.TiledLeaseTier.from_arrays(ts, h.conf, lin))
        refs.append((orc.commit_soa(h.follower, h.flush, h.conf, mode=0, commit_in=h.commit, term_start=h.term_start),
                     orc.lease_soa(ts, h.conf, lin, NOW, 100)))
    engine.leader_launch(ctx, ctiers, ltiers, NOW, 100)
    torch.cuda.synchronize()
    for ct, lt, (rc, rl), h in zip(ctiers, ltiers, refs, host):
        assert np.array_equal(ct.column("commit_out").cpu().numpy(), rc["commit"])
        nw = (h.n + 63) // 64
        assert np.array_equal(lt.lease_out.cpu().numpy(), rl["lease"])
        assert np.array_equal(lt.has_lease_bits[:nw].cpu().numpy().view(np.uint64), rl["has_lease_bits"])
