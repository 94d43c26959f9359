"""GPU parity of the delta path's ordering and concurrency (rh_push_deltas, the multi-producer
staging and the three-phase device apply, ratis_hip.h rh_delta / groups.cpp).

The reference updates a FollowerInfo one call at a time: RaftLogIndex.updateToMax (matchIndex,
commitIndex: FollowerInfoImpl.java:93-105), setUnconditionally (setSnapshotIndex:
FollowerInfoImpl.java:147-151), Timestamp / AtomicBoolean sets for the lease state
(FollowerInfoImpl.java:241-243, LeaderLease.java:37-38).  Here every batch -- one push, many pushes
staged together, pushes from several producer threads -- must leave each cell where applying its
deltas one by one in call order leaves it: the last SET wins and only the MAX deltas after it count,
SET-after-MAX and MAX-after-SET on one cell included.  The last tests check that a thread waiting
for a watch / lease / commit evaluation does not hold up a producer (no table lock across a device
wait) and that a control op on a slot comes after the deltas staged for it."""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

IMIN = np.iinfo(np.int64).min
SELF, ACTIVE = 1 << 14, 1 << 31
COL_FLUSH, COL_COMMITTED, COL_LEASE, COL_LEASE_ON = 32, 33, 36, 37
OP_MAX, OP_SET = 0, 1
F = 4   # followers 0..3: a width-4 tier


def cols():
    return ([k for k in range(F)] + [16 + k for k in range(F)] + [48 + k for k in range(F)]
            + [COL_FLUSH, COL_COMMITTED, COL_LEASE, COL_LEASE_ON])


class Cells:
    """One-by-one RaftLogIndex / Timestamp / AtomicBoolean semantics per (slot, column)."""

    def __init__(self, slots, flush, commit):
        self.v = {}
        for s in slots:
            for c in cols():
                if c < 32:
                    self.v[(s, c)] = -1                      # new FollowerInfo (FII:42-43)
                elif c >= 48 or c == COL_LEASE:
                    self.v[(s, c)] = IMIN                    # no timestamp / lease yet
                elif c == COL_LEASE_ON:
                    self.v[(s, c)] = 0
            self.v[(s, COL_FLUSH)] = flush
            self.v[(s, COL_COMMITTED)] = commit

    def apply(self, d):
        for x in d:
            s, c, op, v = int(x["slot"]), int(x["column"]), int(x["op"]), int(x["value"])
            if c == COL_LEASE_ON:   # AtomicBoolean: SET stores v != 0, MAX ORs it
                b = int(v != 0)
                self.v[(s, c)] = b if op == OP_SET else (self.v[(s, c)] | b)
            else:
                self.v[(s, c)] = v if op == OP_SET else max(self.v[(s, c)], v)


def started_table(ctx, n_slots, capacity=256, flush=1000, commit=900):
    from ratis_amd import groups
    tab = groups.RaftGroupTable(ctx, capacity=capacity)
    conf = (0b1111 | SELF | ACTIVE) & 0xFFFFFFFF
    for s in range(n_slots):
        tab.start(s, conf, flush, commit, 0)
    return tab, Cells(range(n_slots), flush, commit)


def check(tab, cells, slots):
    for c in cols():
        got = tab.read(c)
        for s in slots:
            assert got[s] == cells.v[(s, c)], (s, c, int(got[s]), cells.v[(s, c)])


def random_batch(rng, slots, k, set_frac=0.4):
    from ratis_amd.groups import make_deltas
    cs = np.array(cols())
    s = rng.choice(slots, size=k)
    c = rng.choice(cs, size=k)
    op = np.where(rng.random(k) < set_frac, OP_SET, OP_MAX)
    v = rng.integers(-5, 60, size=k) * 7 + 1000   # few distinct values: ties and reversals
    v = np.where(c == COL_LEASE_ON, rng.integers(-2, 3, size=k), v)
    return make_deltas(s, c, v, op)


def test_hand_sequences_on_one_cell(ctx):
    """SET-after-MAX, MAX-after-SET, SET-SET-MAX, MAX below a SET, and the lease flag's SET 0 then
    MAX of a non-zero value -- each sequence inside ONE push and again spread over many pushes."""
    from ratis_amd.groups import make_deltas
    seqs = [
        [(OP_MAX, 100), (OP_SET, 50), (OP_MAX, 70)],            # -> 70
        [(OP_SET, 200), (OP_MAX, 150)],                         # -> 200
        [(OP_MAX, 300), (OP_SET, 10), (OP_SET, 20), (OP_MAX, 15)],   # -> 20
        [(OP_SET, 5), (OP_MAX, 5), (OP_MAX, 4), (OP_SET, 3)],   # -> 3
        [(OP_MAX, 7), (OP_MAX, 9), (OP_MAX, 8)],                # -> 9
    ]
    lease_seqs = [[(OP_SET, 0), (OP_MAX, -3)], [(OP_SET, 5), (OP_MAX, 0)], [(OP_MAX, 1), (OP_SET, 0)]]
    for spread in (False, True):
        tab, cells = started_table(ctx, 16)
        rows = []
        for i, seq in enumerate(seqs):
            for c in (0, 17, 50, COL_FLUSH, COL_LEASE):
                rows += [(i, c, op, v) for op, v in seq]
        for i, seq in enumerate(lease_seqs):
            rows += [(8 + i, COL_LEASE_ON, op, v) for op, v in seq]
        d = make_deltas([r[0] for r in rows], [r[1] for r in rows], [r[3] for r in rows], [r[2] for r in rows])
        if spread:
            for x in d:
                tab.push(x.reshape(1))
        else:
            tab.push(d)
        cells.apply(d)
        check(tab, cells, range(16))
        assert tab.read(0)[0] == 70 and tab.read(0)[2] == 20 and tab.read(COL_LEASE_ON)[8] == 1
        tab.close()


@pytest.mark.parametrize("calls", [1, 37])
def test_random_conflicting_batches(ctx, calls):
    """20k deltas on 16 slots x 16 cells (every cell hit ~80 times, 40 % SETs) in one push or split
    over many pushes staged into one device batch, then evaluations in between."""
    rng = np.random.default_rng(11 + calls)
    tab, cells = started_table(ctx, 16)
    for rnd in range(3):
        d = random_batch(rng, np.arange(16), 20_000)
        cuts = np.sort(rng.choice(np.arange(1, d.size), size=calls - 1, replace=False)) if calls > 1 else []
        for part in np.split(d, cuts):
            tab.push(part)
        cells.apply(d)
        check(tab, cells, range(16))
        tab.update_commit()   # an evaluation submits the staged deltas: the next round is a new batch
    tab.close()


def test_batches_larger_than_a_staging_slot(ctx):
    """A push that spans staging slots (> RH_DELTA_SLOT deltas) keeps its order across the split."""
    from ratis_amd import _lib
    from ratis_amd.groups import make_deltas
    rng = np.random.default_rng(5)
    tab, cells = started_table(ctx, 4)
    n = _lib.RH_DELTA_SLOT + 4321
    s = rng.integers(0, 4, size=n)
    c = rng.integers(0, F, size=n)
    op = np.where(rng.random(n) < 0.3, OP_SET, OP_MAX)
    v = rng.integers(0, 1 << 40, size=n)
    d = make_deltas(s, c, v, op)
    tab.push(d)
    # one-by-one result per cell: the max of the MAXes after the last SET (and the SET itself)
    for slot in range(4):
        for k in range(F):
            m = (s == slot) & (c == k)
            idx = np.nonzero(m)[0]
            sets = idx[op[idx] == OP_SET]
            if sets.size:
                last = sets[-1]
                after = idx[idx > last]
                want = max([int(v[last])] + [int(v[j]) for j in after if op[j] == OP_MAX])
            else:
                want = max(-1, int(v[idx].max()))
            cells.v[(slot, k)] = want
    check(tab, cells, range(4))
    tab.close()


def test_concurrent_producers_keep_each_threads_order(ctx):
    """8 producer threads push their own slots' conflicting SET / MAX sequences in random-sized
    calls at the same time (plus MAX deltas to one shared flushIndex): every cell ends where its
    thread's one-by-one order puts it; the shared cell holds the max."""
    from ratis_amd.groups import make_deltas
    T, per = 8, 6
    tab, cells = started_table(ctx, T * per + 1)
    shared = T * per
    seqs = []
    for t in range(T):
        rng = np.random.default_rng(100 + t)
        d = random_batch(rng, np.arange(t * per, (t + 1) * per), 30_000)
        extra = make_deltas(np.full(500, shared), COL_FLUSH, rng.integers(1000, 1 << 30, size=500), OP_MAX)
        d = np.concatenate([d, extra])
        d = d[rng.permutation(d.size)]   # shared MAXes interleaved (order-free)
        d_own = d[d["slot"] != shared]
        seqs.append((d, d_own))
    errors = []

    def producer(t):
        try:
            rng = np.random.default_rng(7 + t)
            d = seqs[t][0]
            i = 0
            while i < d.size:
                k = int(rng.integers(1, 800))
                tab.push(d[i:i + k])
                i += k
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    th = [threading.Thread(target=producer, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(T):
        cells.apply(seqs[t][1])
        sh = seqs[t][0][seqs[t][0]["slot"] == shared]
        cells.apply(sh)
    check(tab, cells, range(T * per + 1))
    tab.close()


def test_control_op_follows_deltas_staged_for_its_slot(ctx):
    """Deltas staged for slot 1, then rh_group_start(1) (a new leader term): the deltas land on
    the old row, which the start resets (every FollowerInfo new at -1).  Deltas staged for slot 2
    while slot 3 starts are kept."""
    from ratis_amd.groups import make_deltas
    tab, cells = started_table(ctx, 4)
    conf = (0b1111 | SELF | ACTIVE) & 0xFFFFFFFF
    tab.push(make_deltas([1, 1, 2, 2], [0, COL_FLUSH, 0, 17], [500, 2000, 600, 700]))
    tab.start(1, conf, 1000, 900, 0)
    tab.stop(3)
    tab.start(3, conf, 1000, 900, 0)
    m, f = tab.read(0), tab.read(17)
    assert m[1] == -1 and tab.read(COL_FLUSH)[1] == 1000
    assert m[2] == 600 and f[2] == 700
    tab.close()


def _spin(tab, ms):
    """Occupies the table's stream for ~ms with a spin kernel (torch.cuda._sleep)."""
    import torch
    stream = torch.cuda.ExternalStream(tab._lib.rh_ctx_stream(tab.ctx.handle))
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(ms * 2_000_000))


@pytest.mark.parametrize("what", ["watch", "lease", "commit"])
def test_wait_does_not_block_producers(ctx, orc, what):
    """A thread waits for a watch / lease / commit evaluation queued behind a ~150 ms spin kernel on a
    200k-group table; meanwhile another thread pushes deltas.  The push returns before the wait
    does, and the results equal the table model's."""
    from ratis_amd import groups
    from tests.table_model import TableModel
    n = 200_000
    rng = np.random.default_rng(3)
    tab = groups.RaftGroupTable(ctx, capacity=n)
    model = TableModel(n)
    conf = np.full(n, (0b1111 | SELF | ACTIVE) & 0xFFFFFFFF, np.uint32)
    flush = rng.integers(10_000, 20_000, n)
    commit = flush - 5000
    match = (flush - rng.integers(0, 8000, (F, n))).astype(np.int64)
    tab.load(0, conf, flush, commit, np.zeros(n, np.int64), match=match)
    model.load(0, conf, flush, commit, np.zeros(n, np.int64), match=match)
    assert np.array_equal(tab.update_commit().advanced_slots, model.commit_batch(orc)[0])
    tab.commit_index_changed()
    model.watch(orc)
    d = groups.make_deltas(rng.integers(0, n, 5000), rng.integers(0, F, 5000), rng.integers(15_000, 25_000, 5000))
    _spin(tab, 150)
    t0 = time.perf_counter()
    if what == "watch":
        tab.watch_async()
    elif what == "lease":
        tab.lease_async(1 << 50, 100)
    else:
        tk = tab.commit_async()
    done = {}

    def waiter():
        if what == "watch":
            done["r"] = tab.watch_wait()
        elif what == "lease":
            done["r"] = tab.lease_wait()
        else:
            done["r"] = tab.commit_wait(tk)
        done["t"] = time.perf_counter()
    th = threading.Thread(target=waiter)
    th.start()
    time.sleep(0.02)
    tab.push(d)
    t_push = time.perf_counter()
    th.join()
    assert t_push < done["t"], (t_push - t0, done["t"] - t0)
    assert done["t"] - t0 > 0.05   # the wait really waited for the spin
    # the evaluation in flight saw the state before the push; the next one sees the push
    if what == "commit":
        a_s, a_c, _, _ = model.commit_batch(orc)
        assert np.array_equal(done["r"].advanced_slots, a_s) and np.array_equal(done["r"].advanced_commit, a_c)
    model.apply(d)
    a_s, a_c, w_s, w_m = model.commit_batch(orc)
    got = tab.update_commit()
    assert np.array_equal(got.advanced_slots, a_s) and np.array_equal(got.advanced_commit, a_c)
    assert np.array_equal(got.watch_all_slots, w_s) and np.array_equal(got.watch_all_min, w_m)
    assert np.array_equal(tab.read(0), model.column(0))
    tab.close()


def test_staging_slots_reused_without_evaluations(ctx):
    """Batches submitted by reads and zero-copy submits with no evaluation in between -- so no
    evaluation's event frees a slot applied in place, and the next user of the slot must record and
    wait for one itself (groups.cpp slot_event) -- with sizes on both sides of the in-place bound
    (65536 deltas: the slot read in place, or first copied to HBM): every cell ends where the
    one-by-one order puts it."""
    rng = np.random.default_rng(65536)
    tab, cells = started_table(ctx, 64)
    slots = np.arange(64)
    for i, k in enumerate([100, 3000, 70_000, 500, 65_536, 65_537, 20, 40_000, 7, 1]):
        d = random_batch(rng, slots, k)
        if i % 3 == 2:   # a producer-filled slot (rh_deltas_acquire / submit)
            ring = tab.acquire_deltas()
            ring[: d.size] = d
            tab.submit_deltas(d.size)
        else:
            tab.push(d)
            tab.read(0)   # submits the staged batch: no evaluation
        cells.apply(d)
    check(tab, cells, slots)
    tab.close()
