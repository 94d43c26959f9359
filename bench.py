#!/usr/bin/env python3
"""Benchmark of the BASELINE.json hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

Headline (`value`): quorum-commit updates/s at BASELINE config 3 per GPU -- 1M RaftGroups x 5
peers, 10% in joint consensus (old+new) -- weak-scaled: each rank owns the groups whose
RaftGroupId hash maps to it (RaftId.java:119-122), 1M per GPU, no inter-GPU traffic on the
hot path.  A step = one fused commit launch (LeaderStateImpl.updateCommit +
RaftLogBase.updateCommitIndex for every group) over one 1M-group batch already resident in HBM.
Steps rotate over 8 distinct batches (615 MB > the 256 MiB Infinity Cache) so every step reads
HBM, not a cache.  Also reported in the same JSON line:
  * crc32c: SegmentedRaftLog frame verification GB/s (config 5: 256 x 32 MiB segments of 4 KiB
    frames = 8 GiB per GPU), its roofline and CPU baseline;
  * read_path: segment framing (SegmentedRaftLogReader walk) and framing + CRC verify
    (LogSegment.readSegmentFile) GB/s over the same config-5 segments;
  * lease: batched LeaderStateImpl.hasLease / LeaderLease.extend checks/s over the same 1M groups;
  * pcie: host-buffer-inclusive rates for both paths;
  * cpu_baseline: the oracle (a scalar C port of the reference's Java arithmetic) timed on this
    host on a bounded sample, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "quorum commit updates/sec @1M groups×5 peers; log CRC32C GB/s; % HBM peak"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--groups-per-gpu", type=int, default=1_000_000)
    p.add_argument("--rotate", type=int, default=8)
    p.add_argument("--gap", type=int, default=-1)
    p.add_argument("--layout", choices=["tiled", "plain"], default="tiled",
                   help="commit tiers in the tiled (AoSoA, rh_commit_soa.tile_stride) or plain SoA layout")
    p.add_argument("--crc-segments", type=int, default=256, help="32 MiB segments per GPU (0 = skip CRC)")
    p.add_argument("--crc-steps", type=int, default=20)
    p.add_argument("--crc-warmup", type=int, default=30, help="untimed config-5 CRC passes before the timed ones")
    p.add_argument("--ragged-segments", type=int, default=256,
                   help="32 MiB segments of 64-2048 B frames per GPU for the ragged read path (0 = skip)")
    p.add_argument("--no-lease", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="time the commit / lease / fused legs as one captured HIP graph of the K launches "
                        "(measured equal or 1-2 %% slower than the prebuilt stream launches: profiles/r02/graph_timing/)")
    p.add_argument("--lease-layout", choices=["tiled", "plain"], default="tiled",
                   help="rh_lease_soa layout of the lease leg (tile_stride), as --layout for commit")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pcie", action="store_true")
    p.add_argument("--pmc-json", default=None, help="default: the newest profiles/r*/pmc_traffic.json")
    return p.parse_args()


def load_pmc(path):
    """Per-unit HBM traffic measured by rocprofv3 PMC passes (scripts/pmc.sh + pmc_summary.py),
    committed under profiles/rNN/.  Used only to fill roofline.traffic.  Without --pmc-json every
    profiles/r*/pmc_traffic.json is read oldest first, so each kernel's figure comes from the newest
    round that measured it; "_src" records which file that was per kernel."""
    import glob
    paths = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    out = {"_src": {}}
    for p in paths:
        try:
            d = json.load(open(p))
        except Exception:
            continue
        for k, v in d.items():
            out[k] = v
            if k.endswith("_bytes_per_unit"):
                out["_src"][k[: -len("_bytes_per_unit")]] = os.path.relpath(p, ROOT)
    return out


class _Legs:
    """roctx ranges naming the bench's timed legs (rocprofv3 --marker-trace records them): every
    kernel dispatch of a profiled run is attributed to the leg whose range holds it
    (scripts/prof_legs.py), so each roofline's avg_launch_ms can be checked against the kernel
    trace.  Without the profiler the calls are no-ops; without the library, nothing is called."""

    def __init__(self):
        import ctypes
        self._lib = None
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                self._lib = lib
                break
            except (OSError, AttributeError):
                continue

    def push(self, name: str, steps: int = 1) -> None:
        """Opens the range of a leg that times `steps` steps (the name carries the count)."""
        if self._lib is not None:
            self._lib.roctxRangePushA(f"leg:{name}#{steps}".encode())

    def pop(self) -> None:
        if self._lib is not None:
            self._lib.roctxRangePop()


LEGS = _Legs()


def cpu_threads() -> int:
    """Threads for the all-core CPU baseline: this process's CPU affinity, capped at the 16-CPU
    share a one-GPU box gives a job (nproc there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def host_cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def timed_passes(items, fn, seconds: float) -> dict:
    """Runs fn(*item) repeatedly on one thread per item for `seconds`; fn returns the units one
    pass processed.  Returns the aggregate units/s over the wall time of all threads."""
    import threading
    units = [0] * len(items)
    passes = [0] * len(items)
    t0 = time.perf_counter()
    stop = t0 + seconds

    def run(i):
        while time.perf_counter() < stop:
            units[i] += fn(*items[i])
            passes[i] += 1
    th = [threading.Thread(target=run, args=(i,)) for i in range(len(items))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return {"rate": sum(units) / dt, "passes": sum(passes), "seconds": dt}


class _producers:
    """bench_support/libbench_producers.so: a pool of native threads standing in for the Java
    RPC threads that write rh_delta records into the acquired staging slot (bench-only)."""

    def __init__(self, threads: int):
        import ctypes
        path = os.path.join(ROOT, "bench_support", "_build", "libbench_producers.so")
        self._lib = ctypes.CDLL(path)
        self._lib.bp_create.restype = ctypes.c_void_p
        self._lib.bp_create.argtypes = [ctypes.c_int]
        self._lib.bp_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        self._lib.bp_destroy.argtypes = [ctypes.c_void_p]
        self._lib.bp_push.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t]
        self._lib.bp_threads.argtypes = [ctypes.c_void_p]
        self._pool = self._lib.bp_create(int(threads))
        if not self._pool:
            raise RuntimeError("bp_create failed")

    def fill(self, dst: int, src: int, nbytes: int) -> None:
        if self._lib.bp_fill(self._pool, dst, src, nbytes) != 0:
            raise RuntimeError("bp_fill failed")

    def push(self, fn: int, node: int, src: int, shares: int, chunk: int) -> int:
        """Every producer pushes its share of src (record offsets `shares`) through fn(node, ...)."""
        return self._lib.bp_push(self._pool, fn, node, src, shares, chunk)

    def threads(self) -> int:
        return self._lib.bp_threads(self._pool)

    def close(self) -> None:
        if self._pool:
            self._lib.bp_destroy(self._pool)
            self._pool = None


class HostShift:
    """A workload.HostTier with every index column translated by d (the rotating batches)."""

    def __init__(self, h, d):
        self.follower, self.flush, self.commit, self.term_start = h.follower + d, h.flush + d, h.commit + d, h.term_start + d
        self.conf = h.conf


def out_col(t, name):
    """An output column of a plain (CommitTier) or tiled (TiledCommitTier) commit tier."""
    return t.column(name) if hasattr(t, "column") else getattr(t, name)


def captured(launches, steps: int, ctx, use_graph: bool):
    """The K timed launches of a leg (launches[i % R] for i < K) as one callable: replayed from a
    HIP graph captured once (the kernels run back to back without the host in between), or -- if
    capture is off or fails -- issued one by one.  Returns (run, mode)."""
    import torch
    if use_graph:
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(steps):
                    launches[i % len(launches)](ctx, None)   # on the capture stream
            torch.cuda.synchronize()
            return (lambda stream: g.replay()), "hipGraph"
        except Exception as e:  # noqa: BLE001 -- report and time the plain launches instead
            print(f"bench: graph capture failed ({e}); timing stream launches", file=sys.stderr)

    def run(stream):
        for i in range(steps):
            launches[i % len(launches)](ctx, stream)
    return run, "stream"


def delta_streaming(ctx, host, steps: int = 12, fill_threads: int = 16, reps: int = 5, sink=None) -> dict:
    """The operating mode the Java module uses: one resident RaftGroupTable (stable F=4 and joint
    F=6 tiers), FollowerInfo / flush-index updates written in place into the pinned delta ring
    (rh_deltas_acquire / submit: H2D + device apply, which marks the touched groups dirty), then
    rh_commit_batch_async over the dirty groups with its advanced-group events written straight
    into host-mapped memory.  One step = one 16-byte delta per group (90 % a follower matchIndex,
    10 % the leader flushIndex) + one batched updateCommit.  Pipelined: the host fills step s+1
    while the device applies and evaluates step s, and collects step s-1's events meanwhile.
    Wall-clock per step; the stages are also timed on their own."""
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(99)
    n_all = sum(h.n for h in host)
    tab = groups.RaftGroupTable(ctx, capacity=n_all)
    if sink is not None:
        tab.set_event_sink(sink)
    first, bases = 0, []
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        bases.append(first)
        first += h.n
    per = []   # fresh deltas for every step of every run (a re-applied MAX delta advances nothing)
    for s in range(steps * reps + 3):
        parts = []
        for h, b in zip(host, bases):
            F = h.follower.shape[0]
            slot = rng.permutation(h.n)
            is_flush = rng.random(h.n) < 0.10
            col = rng.integers(0, 4, size=h.n)          # followers 0..3 exist in both tiers
            cur = np.where(is_flush, h.flush[slot], h.follower[col, slot])
            parts.append(groups.make_deltas(b + slot, np.where(is_flush, _lib.RH_COL_FLUSH, col),
                                            cur + (s + 1) * 512))
            del F
        per.append(np.concatenate(parts))
    nbytes = per[0].nbytes

    prod = _producers(fill_threads)

    def fill(ring, d):
        # the producers' writes into the pinned ring (bench_support/producers.c: fill_threads native
        # threads, each copying one contiguous share of the step's deltas)
        prod.fill(ring.ctypes.data, d.ctypes.data, d.nbytes)

    def step(d):
        ring = tab.acquire_deltas()
        fill(ring, d)
        tab.submit_deltas(d.size)
        return tab.commit_async(watch_all=False)

    tk = step(per[0])
    tab.commit_wait_counts(tk)
    # pipelined (the timed figure): `reps` runs of `steps` steps, the median run reported (one
    # run of a dozen sub-millisecond steps is at the mercy of a single host hiccup)
    runs = []
    for rep in range(reps):
        LEGS.push("delta_streaming", steps)
        t0 = time.perf_counter()
        inflight, advanced = [], 0
        for s in range(1, steps + 1):
            inflight.append(step(per[rep * steps + s]))
            if len(inflight) > 2:   # two evaluations in flight while the host fills the next step
                advanced += tab.commit_wait_counts(inflight.pop(0))[0]
        for tk in inflight:
            advanced += tab.commit_wait_counts(tk)[0]
        runs.append((time.perf_counter() - t0) / steps)
        LEGS.pop()
    dt = float(np.median(runs))
    # stages on their own: host fill of the pinned ring; device part (H2D + apply + evaluation +
    # events) with the ring already filled, synchronous
    last = steps * reps
    f0 = time.perf_counter()
    for s in range(3):
        ring = tab.acquire_deltas()
        fill(ring, per[last + 1])
        tab.submit_deltas(0)
    fill_s = (time.perf_counter() - f0) / 3
    ring = tab.acquire_deltas()
    fill(ring, per[last + 2])
    g0 = time.perf_counter()
    tab.submit_deltas(per[last + 2].size)
    tab.commit_wait_counts(tab.commit_async(watch_all=False))
    dev_s = time.perf_counter() - g0
    tab.close()
    prod.close()
    return {"commit_updates_per_s_incl_pcie": round(n_all / dt, 1), "ms_per_step": round(dt * 1e3, 3),
            "ms_per_step_runs": [round(x * 1e3, 3) for x in runs], "runs": f"median of {reps} runs of {steps} steps",
            "deltas_per_step": n_all, "delta_bytes_h2d_per_step": nbytes,
            "h2d_bound_ms": round(nbytes / 50e9 * 1e3, 3),
            "stage_ms": {"host_fill_pinned_ring": round(fill_s * 1e3, 3), "fill_threads": fill_threads,
                         "device_h2d_apply_evaluate_events": round(dev_s * 1e3, 3)},
            "advanced_per_step": round(advanced / steps, 1),
            "path": "rh_deltas_acquire/submit (pinned ring, 16 B deltas, H2D + apply marking dirty groups) + "
                    "rh_commit_batch_async/_wait (dirty-group evaluation, advanced events in host-mapped "
                    "memory), pipelined: the host fill of step s+1 and its H2D (copy stream, double-buffered "
                    "device slots) overlap the apply and evaluation of step s"}


def reply_mix_leg(host, threads: int = 16, steps: int = 8, active_frac: float = 0.25, repeat_frac: float = 0.25,
                  chunk: int = 4096) -> dict:
    """The delta path the Java module runs (HipLeaderBookkeeper: per-thread DeltaBuffers of 4096
    deltas pushed through rh_node_push_deltas by their own producer threads, the multi-producer
    staging, then the pump's updateCommit + commitIndexChanged), fed the reference's per-reply
    mix.  Per step a quarter of config 3's divisions are active; each gets one flushIndex MAX (the
    log worker, SegmentedRaftLogWorker.java:419-431) and one reply from each of its 4 followers --
    SET lastRespondedAppendEntriesSendTime, MAX matchIndex, MAX commitIndex
    (GrpcLogAppender.java:491, 516; FollowerInfoImpl.java:93-105, 241-243) -- and a quarter of the
    followers reply twice in the step (SET after SET on one cell, later MAXes).  `threads` native
    producers own the divisions d % threads (an appender thread serves its followers' replies in
    order).  Pipelined as the pump: step s's evaluations are in flight while the producers push
    step s+1.  PCIe included (the deltas are host memory).  Parity: after the run, every
    follower's matchIndex / commitIndex / timestamp and every flushIndex equals the one-by-one
    result, and each step's advanced set equals an oracle evaluation of the same snapshot."""
    import ctypes

    from oracle import oracle as orc
    from ratis_amd import _lib, groups
    lib = _lib.load()
    rng = np.random.default_rng(123)
    n_all = sum(h.n for h in host)
    node = groups.RaftNode(0, n_all, devices=[0])
    tab = node.tables[0]
    first = 0
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower,
                 fcommit=h.follower - 3)
        first += h.n
    tab.commit_wait_counts(tab.commit_async(watch_all=True))   # the load marked every row dirty
    tab.watch_async()
    tab.watch_wait()
    com0 = tab.read(_lib.RH_COL_COMMITTED)
    match = np.concatenate([h.follower[:4] for h in host], axis=1)   # followers 0..3 exist in both tiers
    fcom = match - 3
    ts = np.full((4, n_all), np.iinfo(np.int64).min, np.int64)   # no timestamp yet (rh_groups_load)
    flush = np.concatenate([h.flush for h in host])
    T = threads
    A = int(n_all * active_frac)
    per_step = []
    for s in range(steps + 1):
        act = np.sort(rng.choice(n_all, A, replace=False))
        owner = act % T
        act = act[np.argsort(owner, kind="stable")]
        owner = act % T
        # first part, 13 deltas per active division: flush MAX, then each follower's reply
        flush_v = flush[act] + rng.integers(1, 600, A)
        m1 = match[:, act] + rng.integers(1, 500, (4, A))
        t1 = (s * 10 + 1) * 1_000_000 + np.arange(4)[:, None]
        c1 = np.maximum(fcom[:, act], m1 - rng.integers(0, 64, (4, A)))
        first_part = np.zeros((A, 13), dtype=groups.DELTA_DTYPE)
        first_part["slot"] = act[:, None]
        first_part["column"][:, 0], first_part["value"][:, 0] = _lib.RH_COL_FLUSH, flush_v
        for k in range(4):
            b = 1 + 3 * k
            first_part["column"][:, b], first_part["op"][:, b], first_part["value"][:, b] = _lib.RH_COL_TS(k), _lib.RH_OP_SET, t1[k]
            first_part["column"][:, b + 1], first_part["value"][:, b + 1] = _lib.rh_col_match(k), m1[k]
            first_part["column"][:, b + 2], first_part["value"][:, b + 2] = _lib.rh_col_fcommit(k), c1[k]
        # second replies (repeat_frac of the (division, follower) pairs): later send time, further
        # matchIndex -- or a stale one, which the MAX ignores
        rep = rng.random((4, A)) < repeat_frac
        kk, jj = np.nonzero(rep)
        m2 = m1[kk, jj] + rng.integers(-50, 400, kk.size)
        t2 = t1[kk, 0] + 5_000_000
        c2 = np.maximum(c1[kk, jj], m2 - 10)
        second = np.zeros((kk.size, 3), dtype=groups.DELTA_DTYPE)
        second["slot"] = act[jj][:, None]
        second["column"][:, 0], second["op"][:, 0], second["value"][:, 0] = 48 + kk, _lib.RH_OP_SET, t2
        second["column"][:, 1], second["value"][:, 1] = kk, m2
        second["column"][:, 2], second["value"][:, 2] = 16 + kk, c2
        # the one-by-one state after the step (the parity reference)
        flush[act] = np.maximum(flush[act], flush_v)
        match[:, act] = np.maximum(match[:, act], m1)
        fcom[:, act] = np.maximum(fcom[:, act], c1)
        ts[:, act] = t1
        np.maximum.at(match, (kk, act[jj]), m2)
        np.maximum.at(fcom, (kk, act[jj]), c2)
        ts[kk, act[jj]] = t2
        # producer t's share: its divisions' first parts, then their second replies
        sown = owner[jj]
        so = np.argsort(sown, kind="stable")
        second = second[so]
        shares = [0]
        parts = []
        for t in range(T):
            a = first_part[owner == t].reshape(-1)
            b = second[sown[so] == t].reshape(-1)
            parts += [a, b]
            shares.append(shares[-1] + a.size + b.size)
        per_step.append((np.concatenate(parts), np.array(shares, dtype=np.uint64), int(A * 4 + kk.size)))
    prod = _producers(T)
    if prod.threads() != T:
        T = prod.threads()
    push_fn = ctypes.cast(lib.rh_node_push_deltas, ctypes.c_void_p).value
    node_h = node._h.value

    def push(d, sh):
        if prod.push(push_fn, node_h, d.ctypes.data, sh.ctypes.data, chunk) != 0:
            raise RuntimeError("rh_node_push_deltas failed in a producer thread")
    push(*per_step[0][:2])   # warm-up step (not timed)
    tk = tab.commit_async(watch_all=True)
    tab.watch_async()
    tab.commit_wait_counts(tk)
    tab.watch_wait_count()
    LEGS.push("reply_mix", steps)
    t0 = time.perf_counter()
    inflight = None
    advanced = 0
    push_s = 0.0
    for s in range(1, steps + 1):
        p0 = time.perf_counter()
        push(*per_step[s][:2])
        push_s += time.perf_counter() - p0
        if inflight is not None:   # the previous step's evaluations, in flight while this step pushed
            advanced += tab.commit_wait_counts(inflight)[0]
            tab.watch_wait_count()
        inflight = tab.commit_async(watch_all=True)
        tab.watch_async()
    advanced += tab.commit_wait_counts(inflight)[0]
    tab.watch_wait_count()
    dt = (time.perf_counter() - t0) / steps
    LEGS.pop()
    ok = (np.array_equal(tab.read(_lib.RH_COL_FLUSH), flush)
          and all(np.array_equal(tab.read(_lib.rh_col_match(k)), match[k]) for k in range(4))
          and all(np.array_equal(tab.read(_lib.rh_col_fcommit(k)), fcom[k]) for k in range(4))
          and all(np.array_equal(tab.read(_lib.RH_COL_TS(k)), ts[k]) for k in range(4)))
    # every index only grows here, and updateCommit's rule is monotone in them (a commit accepted at
    # one step is <= the final snapshot's, which passes the term check too): the commit the
    # pipelined evaluations reached is the oracle's rule on the final snapshot from the start commit
    conf = np.concatenate([h.conf for h in host])
    tstart = np.concatenate([h.term_start for h in host])
    com = tab.read(_lib.RH_COL_COMMITTED)
    lo = 0
    for h in host:
        hi = lo + h.n
        fol = h.follower.copy()
        fol[:4] = match[:, lo:hi]
        r = orc.commit_soa(fol, flush[lo:hi], conf[lo:hi], mode=0, gap=-1, commit_in=com0[lo:hi], term_start=tstart[lo:hi])
        ok &= bool(np.array_equal(r["commit"], com[lo:hi]))
        lo = hi
    n_deltas = int(np.mean([p[0].size for p in per_step[1:]]))
    replies = int(np.mean([p[2] for p in per_step[1:]]))
    prod.close()
    node.close()
    return {"ms_per_step": round(dt * 1e3, 3), "ms_producers_per_step": round(push_s / steps * 1e3, 3),
            "replies_per_s_incl_pcie": round(replies / dt, 1),
            "deltas_per_s_incl_pcie": round(n_deltas / dt, 1), "replies_per_step": replies,
            "deltas_per_step": n_deltas, "delta_bytes_h2d_per_step": n_deltas * 16,
            "h2d_bound_ms": round(n_deltas * 16 / 50e9 * 1e3, 3), "producer_threads": T,
            "deltas_per_push_call": chunk, "active_divisions_per_step": A, "advanced_per_step": round(advanced / steps, 1),
            "parity_ok": bool(ok),
            "path": "per-thread buffers -> rh_node_push_deltas from every producer thread at once (multi-producer "
                    "staging: one CAS per call, copies in parallel) -> H2D per full 1M-delta slot + three-phase apply "
                    "(last SET wins, later MAXes) -> rh_commit_batch_async + rh_watch_levels_async per step, "
                    "pipelined one step deep"}


def _placeholder_frames(rng, nbytes: int, lo: int = 64, hi: int = 2048):
    """A flush batch as SegmentedRaftLogOutputStream.write lays it out (varint32(n) || n entry bytes
    || 4-byte trailer), trailers zero, ~nbytes long: (image uint8, frame offsets, frame lengths)."""
    sizes, total = [], 0
    while total < nbytes:
        n = int(rng.integers(lo, hi + 1))
        v = 1 if n < 128 else 2
        sizes.append((n, v))
        total += v + n + 4
    img = rng.integers(0, 256, total, dtype=np.uint8)
    off = np.empty(len(sizes), dtype=np.uint64)
    ln = np.empty(len(sizes), dtype=np.uint32)
    pos = 0
    for i, (n, v) in enumerate(sizes):
        off[i], ln[i] = pos, v + n + 4
        if v == 1:
            img[pos] = n
        else:
            img[pos], img[pos + 1] = (n & 0x7F) | 0x80, n >> 7
        img[pos + v + n: pos + v + n + 4] = 0
        pos += v + n + 4
    return img, off, ln


def write_stamp_leg(ctx, reps: int = 25) -> dict:
    """The write side's decision input: the trailers of one flush batch stamped
    on the GPU from a registered host buffer (rh_crc32c_stamp_host: H2D of the batch + the CRC kernel
    + D2H of 4 B per frame + the host writing the trailers; host wall clock per call) against the
    oracle's PureJavaCrc32C restatement (slicing-by-8 C, one core) over the same frames -- at flush
    sizes up to raft.server.log.write.buffer.size's default 8 MiB.  The crossover is the smallest
    measured flush from which the GPU call is faster; the Java module stamps on the GPU from there
    (the writer seam).  Entries of 64-2048 B."""
    import time

    from oracle import oracle as orc
    from ratis_amd import _lib, engine
    lib, olib = _lib.load(), orc.load()
    rng = np.random.default_rng(17)
    out = {"sizes": [], "frames": [], "gpu_us": [], "gpu_GBps": [], "cpu_1core_us": [], "cpu_1core_GBps": []}
    parity = True
    for nbytes in (16 << 10, 32 << 10, 64 << 10, 128 << 10, 256 << 10, 1 << 20, 8 << 20):
        img, off, ln = _placeholder_frames(rng, nbytes)
        buf = img.copy()
        crc = np.zeros(off.size, dtype=np.uint32)
        # both sides timed at their C ABI with the pointers prepared once -- the form of the Java
        # module's JNI call (numpy's per-call pointer conversions cost ~1.4 us each, on both sides)
        pb, po, pl, pi, pc = (a.ctypes.data for a in (buf, off, ln, img, crc))
        with engine.HostRegistration(ctx, buf):
            engine.stamp_host(ctx, buf, off, ln)   # warm-up (staging, code objects)
            g = []
            for _ in range(reps):
                t0 = time.perf_counter()
                rc = lib.rh_crc32c_stamp_host(ctx.handle, pb, buf.size, po, pl, off.size)
                g.append(time.perf_counter() - t0)
                assert rc == 0, rc
        c = []
        for _ in range(reps):
            t0 = time.perf_counter()
            olib.orc_crc32c_frames(pi, po, pl, off.size, pc)
            c.append(time.perf_counter() - t0)
        end = (off + ln.astype(np.uint64)).astype(np.int64)
        stored = ((buf[end - 4].astype(np.uint32) << 24) | (buf[end - 3].astype(np.uint32) << 16)
                  | (buf[end - 2].astype(np.uint32) << 8) | buf[end - 1].astype(np.uint32))
        parity &= bool(np.array_equal(stored, crc))
        gs, cs = float(np.median(g)), float(np.median(c))
        out["sizes"].append(int(img.size))
        out["frames"].append(int(off.size))
        out["gpu_us"].append(round(gs * 1e6, 1))
        out["gpu_GBps"].append(round(img.size / gs / 1e9, 2))
        out["cpu_1core_us"].append(round(cs * 1e6, 1))
        out["cpu_1core_GBps"].append(round(img.size / cs / 1e9, 2))
    faster = [s for s, a, b in zip(out["sizes"], out["gpu_us"], out["cpu_1core_us"]) if a < b]
    out["crossover_bytes"] = min(faster) if faster else None
    out["parity_ok"] = parity
    out["note"] = ("GPU: rh_crc32c_stamp_host from a registered (page-locked) buffer, PCIe both ways included "
                   "(zero-copy plan up to ~7 MiB: the kernel reads the mapped buffer); CPU: the oracle's C "
                   "slicing-by-8 restatement of PureJavaCrc32C on one core (no JVM on the box: the Java "
                   "PureJavaCrc32C is not faster than this); both timed at the C ABI with pointers prepared "
                   "once (the JNI call's form); median of %d calls" % reps)
    return out


def queue_gate(stream, cycles: int = 400_000) -> None:
    """Occupies `stream` for ~0.2 ms with a spin kernel (torch.cuda._sleep) so that the launches the
    host enqueues next are all queued before the GPU reaches the timed region's start event: the
    region then times back-to-back device work, not the host's enqueue rate."""
    import torch
    try:
        with torch.cuda.stream(stream):
            torch.cuda._sleep(cycles)
    except Exception:  # noqa: BLE001 -- no spin kernel in this build: time without the gate
        pass


def table_commit_leg(ctx, host, reps: int = 16, fracs=(1.0, 0.1, 0.01), pmc=None) -> dict:
    """The kernel the Java module drives: rh_commit_batch over the resident table (config-3
    groups, stable F=4 and joint F=6 tiers, 128-row tiled layout), after deltas marked `frac` of the
    groups dirty (one matchIndex / flushIndex update per dirty group, as delta_streaming's steps).
    One evaluation = one kernel that evaluates the dirty rows and writes its event records straight
    into the result lists (the tile kernel over every 128-row tile, or the list kernel over the
    dirty-row lists when few rows can be dirty); the library's timing events (rh_groups_timing: HIP
    events on the evaluation's own launch, stamped at its kernel boundaries by hipExtLaunchKernel)
    time it on the table's stream, HIP events around rh_commit_batch_async the call.  Every sink:
    RH_EVENTS_HOST_MAPPED (the lists are pinned host memory, written across PCIe), RH_EVENTS_DEVICE
    (the lists in HBM, _wait copies the counted prefix) and RH_EVENTS_AUTO (the default, what the
    Java module and rh_node run: DEVICE for tile evaluations, HOST_MAPPED for list evaluations).
    `roofline` = AUTO's evaluation, events included.  The tables' events must be identical."""
    import ctypes
    import time

    import torch

    from ratis_amd import _lib, groups
    lib = _lib.load()
    rng = np.random.default_rng(7)
    n_all = sum(h.n for h in host)
    F = [h.follower.shape[0] for h in host]
    stream = torch.cuda.ExternalStream(lib.rh_ctx_stream(ctx.handle))
    tabs = {}
    names = {_lib.RH_EVENTS_HOST_MAPPED: "host_mapped", _lib.RH_EVENTS_DEVICE: "device", _lib.RH_EVENTS_AUTO: "auto"}
    for sink in (_lib.RH_EVENTS_HOST_MAPPED, _lib.RH_EVENTS_DEVICE, _lib.RH_EVENTS_AUTO):
        tab = groups.RaftGroupTable(ctx, capacity=n_all)
        first = 0
        for h in host:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        tab.set_event_sink(sink)
        tab.set_timing(True)
        tab.commit_wait_counts(tab.commit_async(watch_all=False))   # the load marked every row dirty
        tabs[sink] = tab
    # the reference rate for the event records: GPU stores into mapped pinned memory (the same path)
    from ratis_amd import engine
    pcie_write_gbps = engine.pcie_write_probe(ctx, 32 << 20, 9)
    cur_f = np.concatenate([h.follower[:4] for h in host], axis=1)   # followers 0..3 exist in both tiers
    cur_s = np.concatenate([h.flush for h in host])
    out = {}
    for frac in fracs:
        k = n_all if frac >= 1.0 else int(n_all * frac)
        res = {}
        for r in range(reps + 1):
            slot = rng.permutation(n_all)[:k] if k < n_all else rng.permutation(n_all)
            is_flush = rng.random(k) < 0.10
            col = rng.integers(0, 4, size=k)
            val = np.where(is_flush, cur_s[slot], cur_f[col, slot]) + 512
            cur_s[slot[is_flush]] = val[is_flush]
            cur_f[col[~is_flush], slot[~is_flush]] = val[~is_flush]
            d = groups.make_deltas(slot, np.where(is_flush, _lib.RH_COL_FLUSH, col), val)
            got = {}
            for sink, tab in tabs.items():
                tab.push(d)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                LEGS.push(f"table_{frac * 100:g}pct_{names[sink]}" if r else "table_warmup")
                queue_gate(stream)   # the evaluation is enqueued before the GPU reaches e0
                torch.cuda.synchronize()   # (the gate: the host clock below starts on an idle GPU)
                t_h0 = time.perf_counter()
                e0.record(stream)
                tk = tab.commit_async(watch_all=True)
                e1.record(stream)
                raw = _lib.RhCommitOut()
                _lib.check(lib.rh_commit_batch_wait(tab.handle, tk, ctypes.byref(raw)))
                t_h1 = time.perf_counter()   # the records are in the pinned lists: what the pump waits for
                got[sink] = groups.CommitResult(raw)
                torch.cuda.synchronize()
                LEGS.pop()
                if r:   # the first round is a warm-up
                    res.setdefault((sink, "call"), []).append(e0.elapsed_time(e1))
                    res.setdefault((sink, "host"), []).append((t_h1 - t_h0) * 1e3)
                    sp = tab.last_timing_split()
                    res.setdefault((sink, "eval"), []).append(sp["eval_ms"])
                    res.setdefault((sink, "submit"), []).append(sp["submit_ms"])
                    res.setdefault((sink, "events"), []).append(sp["events_ms"])
                    res.setdefault((sink, "gather"), []).append(sp["gather_ms"])
                    res.setdefault((sink, "list"), []).append(sp["list"])
            a = got[_lib.RH_EVENTS_DEVICE]
            ok = all(np.array_equal(a.advanced_slots, b.advanced_slots) and np.array_equal(a.advanced_commit, b.advanced_commit)
                     and np.array_equal(a.watch_all_slots, b.watch_all_slots) and np.array_equal(a.watch_all_min, b.watch_all_min)
                     for b in got.values())
            res["sinks_agree"] = res.get("sinks_agree", True) and bool(ok)
            res["advanced"] = int(a.advanced_slots.size)
            res["watch_all"] = int(a.watch_all_slots.size)
        med = {key: float(np.median(v)) for key, v in res.items() if isinstance(key, tuple)}
        eval_ms = float(np.median(res[(_lib.RH_EVENTS_AUTO, "eval")]))   # the module's sink
        # algorithmic bytes of the evaluation kernel: 1 dirty byte per row; per dirty row its
        # columns (F matchIndex, conf, commit, flush, term start, previous watch-ALL level; the row
        # slot only where the kernel writes records) and the flag clear; per event the 8 B commit /
        # watch level and (advanced) the 1 B watch-dirty flag it stores, and -- a list evaluation of
        # (AUTO) only -- the 16 B record it writes (tile evaluations and larger
        # list evaluations into AUTO write event bits instead: rh_table_gather_commit builds the
        # records from the table on the side stream)
        n_f4 = host[0].n
        f_mean = (n_f4 * F[0] + (n_all - n_f4) * (F[1] if len(F) > 1 else F[0])) / n_all
        list_mode = bool(np.all(res[(_lib.RH_EVENTS_AUTO, "list")]))
        pinned = list_mode   # groups.cpp RH_LIST_PINNED_MAX: every AUTO list evaluation writes its records
        rec = 16 if pinned else 0
        per_dirty = 8 * f_mean + 4 + (4 if pinned else 0) + 8 + 8 + 8 + 8 + 1
        alg = n_all * 1 + k * per_dirty + res["advanced"] * (rec + 8 + 1) + res["watch_all"] * (rec + 8)
        if not list_mode:
            alg += n_all / 4   # the event masks: 2 bits per row
        ach = alg / (eval_ms * 1e-3) / 1e9
        case = {"dirty_groups": k, "advanced": res["advanced"], "watch_all_changed": res["watch_all"],
                "ms_evaluation": round(eval_ms, 4), "list_mode": list_mode,
                "sinks_agree": res["sinks_agree"]}
        ev_bytes = 16 * (res["advanced"] + res["watch_all"])   # rh_index_event records into the pinned lists
        for sink, nm in names.items():
            case[nm] = {"ms_evaluation": round(med[(sink, "eval")], 4),
                        "ms_submit": round(med[(sink, "submit")], 4),
                        "ms_events": round(med[(sink, "events")], 4),
                        "ms_gather_kernel": round(med[(sink, "gather")], 4),
                        "ms_async_to_records_host": round(med[(sink, "host")], 4),
                        "ms_commit_batch_async_hip_events": round(med[(sink, "call")], 4)}
        ev_ms = med[(_lib.RH_EVENTS_AUTO, "events")]
        ga_ms = med[(_lib.RH_EVENTS_AUTO, "gather")]
        case["events"] = {"records": res["advanced"] + res["watch_all"], "bytes": ev_bytes,
                          "ms_auto": round(ev_ms, 4), "ms_gather_kernel_auto": round(ga_ms, 4),
                          "GBps_gather_kernel": round(ev_bytes / (ga_ms * 1e-3) / 1e9, 2) if ga_ms > 0 else None,
                          "note": ("AUTO: ms_auto from the evaluation's end until the records are in the pinned lists "
                                   "(the REGION gather on the side stream with its launch and cross-stream wait; "
                                   "~0 when the list kernel wrote them itself), ms_gather_kernel_auto the gather "
                                   "kernel at its boundaries; rh_groups_last_timing_split")}
        if pcie_write_gbps and ga_ms > 0:
            case["events"]["pcie_write_GBps"] = round(pcie_write_gbps, 2)
            case["events"]["gather_vs_pcie_bound"] = round(ga_ms / (ev_bytes / (pcie_write_gbps * 1e9) * 1e3), 3)
        case["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBPS, 4), "algorithmic_bytes_per_launch": int(alg),
                            "kernel": ("table_list_kernel<false>" if list_mode else "table_commit_kernel_rank<false>")
                            + (" (RH_EVENTS_AUTO: records into the pinned lists)" if pinned
                               else " (RH_EVENTS_AUTO: event masks; records rebuilt by the gather)"),
                            # PMC passes (scripts/prof_kernels.py table case) run the all-dirty step
                            "traffic": (round(pmc["table_bytes_per_unit"] * n_all)
                                        if frac >= 1.0 and pmc and "table_bytes_per_unit" in pmc else None),
                            "traffic_source": (pmc or {}).get("_src", {}).get("table") if frac >= 1.0 else None}
        out[f"dirty_{frac * 100:g}pct"] = case
    for tab in tabs.values():
        tab.close()
    out["pcie_write_GBps"] = round(pcie_write_gbps, 2)
    out["workload"] = (f"resident table of {n_all} config-3 groups (F=4 and F=6 tiers); deltas mark the dirty "
                       "fraction, then one rh_commit_batch (RH_COMMIT_WATCH_ALL) per step; median of "
                       f"{reps} steps per case; auto is the sink the Java module runs")
    return out


def tick_leg(ctx, host, ks=(256, 2048), reps: int = 50) -> dict:
    """The Java pump's sparse tick end to end (HipLeaderBookkeeper.tick, groups.LeaderPump.tick): k
    follower replies -- a matchIndex and a commitIndex MAX for k / 2 random divisions of config 3's
    1M, as FollowerInfo.updateMatchIndex / updateCommitIndex emit them (FollowerInfoImpl.java:93-105)
    -- pushed, then updateCommit and commitIndexChanged put in flight together and waited for, their
    event records read (LeaderStateImpl.java:946-950, 612-622: the reference runs them per reply event
    per division).  Host wall clock from the push to the last wait, median and p90 of `reps` ticks
    (no timing events on the table: they would lengthen the tick); the event records stay in the
    library's pinned lists (the JNI glue's copy into the Java arrays is not included)."""
    import time

    from ratis_amd import groups
    n_all = sum(h.n for h in host)
    tab = groups.RaftGroupTable(ctx, capacity=n_all)
    first = 0
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    tab.commit_wait_counts(tab.commit_async(watch_all=True))
    tab.watch_async()
    tab.watch_wait_count()
    match = np.concatenate([h.follower[:4] for h in host], axis=1)
    rng = np.random.default_rng(5)
    out = {}
    for k in ks:
        ms = {"tick_async": [], "two_calls": []}
        n_adv = 0
        for r in range(2 * reps + 6):   # the two forms alternate tick by tick
            fused = r % 2 == 0
            slot = rng.choice(n_all, size=k // 2, replace=False)
            col = rng.integers(0, 4, size=slot.size)
            match[col, slot] += rng.integers(1, 300, size=slot.size)
            d = groups.make_deltas(np.concatenate([slot, slot]), np.concatenate([col, 16 + col]),
                                   np.concatenate([match[col, slot], match[col, slot] - 2]))
            LEGS.push((f"tick_k{k}" if fused else f"tick2_k{k}") if r >= 6 else "tick_warmup")
            t0 = time.perf_counter()
            tab.push(d)
            if fused:   # rh_tick_async: both evaluations in one launch (the pump's call)
                tk = tab.tick_async(watch_all=True)
            else:       # the same as two calls: two launches
                tk = tab.commit_async(watch_all=True)
                tab.watch_async()
            na, _ = tab.commit_wait_counts(tk)
            tab.watch_wait_count()
            t1 = time.perf_counter()
            LEGS.pop()
            if r >= 6:
                ms["tick_async" if fused else "two_calls"].append((t1 - t0) * 1e3)
                n_adv += na if fused else 0
        med = float(np.median(ms["tick_async"]))
        out[f"replies_{k}"] = {
            "ms_tick_median": round(med, 4), "ms_tick_p90": round(float(np.percentile(ms["tick_async"], 90)), 4),
            "replies_per_s": round(k / (med * 1e-3), 1),
            "ms_two_calls_median": round(float(np.median(ms["two_calls"])), 4),
            "commits_advanced_per_tick": round(n_adv / reps, 1)}
    tab.close()
    out["workload"] = (f"resident table of {n_all} config-3 groups; per tick k deltas (k/2 replies x matchIndex + "
                       f"commitIndex), push + rh_tick_async (both evaluations, one launch) + both waits (the pump's "
                       f"order); two_calls: commit_async + watch_async instead, ticks alternating; host wall clock, "
                       f"median of {reps} ticks each")
    return out


def table_watch_leg(ctx, host, reps: int = 16, fracs=(1.0, 0.1, 0.01)) -> dict:
    """commitIndexChanged over the resident table (LeaderStateImpl.java:612-622, rh_watch_levels_async
    / _wait), the other evaluation the Java pump runs every tick: the followers' commitIndex deltas
    (FollowerInfo.updateCommitIndex, one per dirty group: follower 0..3, +512 over its current value)
    mark `frac` of config 3's 1M groups, then one watch evaluation per step, timed at its kernel
    boundaries (rh_groups_timing).  Two tables fed the same deltas -- AUTO (the module's sink: a
    tile evaluation writes 2 bits per row -- changed, valid -- and rh_table_gather_watch rebuilds the
    level records from the table on the side stream; a list evaluation writes its records itself,
    across PCIe) and HOST_MAPPED (records across PCIe from the kernel) -- must
    report the same levels.  Algorithmic bytes of the evaluation: 1 B watch-dirty flag per row; per
    dirty row 8F follower commitIndex, 8 commit (the self value), 24 previous levels, 4 conf, 1 flag
    clear; per changed row the 24 B of levels stored, plus the 4 B row slot and 32 B record when the
    kernel writes records, or the masks (n / 4 B) in tile mode."""
    import torch

    from ratis_amd import _lib, groups
    rng = np.random.default_rng(11)
    n_all = sum(h.n for h in host)
    F = [h.follower.shape[0] for h in host]
    tabs = {}
    for sink in (_lib.RH_EVENTS_AUTO, _lib.RH_EVENTS_HOST_MAPPED):
        tab = groups.RaftGroupTable(ctx, capacity=n_all)
        first = 0
        for h in host:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        tab.set_event_sink(sink)
        tab.set_timing(True)
        tab.commit_wait_counts(tab.commit_async(watch_all=False))
        tab.watch_async()
        tab.watch_wait_count()
        tabs[sink] = tab
    commit = np.concatenate([h.commit for h in host])
    cur = np.tile(commit - 2048, (4, 1))   # follower commitIndex, below the leader's (all -1 after the load)
    stream = torch.cuda.ExternalStream(_lib.load().rh_ctx_stream(ctx.handle))
    out = {}
    for frac in fracs:
        k = n_all if frac >= 1.0 else int(n_all * frac)
        res = {"eval": [], "list": []}
        agree, changed = True, 0
        for r in range(reps + 1):
            slot = rng.permutation(n_all)[:k] if k < n_all else rng.permutation(n_all)
            col = rng.integers(0, 4, size=k)
            val = cur[col, slot] + 512
            cur[col, slot] = val
            d = groups.make_deltas(slot, 16 + col, val)
            got = {}
            for sink, tab in tabs.items():
                tab.push(d)
                LEGS.push(f"twatch_{frac * 100:g}pct" if (r and sink == _lib.RH_EVENTS_AUTO) else "twatch_warmup")
                queue_gate(stream)
                tab.watch_async()
                got[sink] = tab.watch_wait()
                torch.cuda.synchronize()
                LEGS.pop()
                if r and sink == _lib.RH_EVENTS_AUTO:
                    sp = tab.last_timing_split()
                    res["eval"].append(sp["eval_ms"])
                    res.setdefault("events", []).append(sp["events_ms"])
                    res.setdefault("gather", []).append(sp["gather_ms"])
                    res.setdefault("submit", []).append(sp["submit_ms"])
                    res["list"].append(sp["list"])
            a, b = got[_lib.RH_EVENTS_AUTO], got[_lib.RH_EVENTS_HOST_MAPPED]
            agree &= bool(np.array_equal(a, b))
            changed = int(a.size)
        eval_ms = float(np.median(res["eval"]))
        list_mode = bool(np.all(res["list"]))
        n_f4 = host[0].n
        f_mean = (n_f4 * F[0] + (n_all - n_f4) * (F[1] if len(F) > 1 else F[0])) / n_all
        pinned = list_mode   # groups.cpp RH_LIST_PINNED_MAX: records into the pinned list
        alg = n_all * 1 + k * (8 * f_mean + 8 + 24 + 4 + (4 if pinned else 0) + 1) + changed * ((32 if pinned else 0) + 24)
        if not list_mode:
            alg += n_all / 4   # the event masks: 2 bits per row
        ach = alg / (eval_ms * 1e-3) / 1e9
        ev_ms = float(np.median(res["events"]))
        out[f"dirty_{frac * 100:g}pct"] = {
            "dirty_groups": k, "levels_changed": changed, "ms_evaluation": round(eval_ms, 4), "list_mode": list_mode,
            "sinks_agree": agree, "ms_submit": round(float(np.median(res["submit"])), 4),
            "events": {"records": changed, "bytes": 32 * changed, "ms_auto": round(ev_ms, 4),
                       "ms_gather_kernel_auto": round(float(np.median(res["gather"])), 4)},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "algorithmic_bytes_per_launch": int(alg),
                         "kernel": ("table_list_kernel<true>" if list_mode else "table_commit_kernel_rank<true>")
                         + (" (records into the pinned list)" if pinned else " (event masks; records rebuilt by the gather)")}}
    for tab in tabs.values():
        tab.close()
    out["workload"] = (f"resident table of {n_all} config-3 groups; follower commitIndex deltas mark the dirty "
                       f"fraction, then one rh_watch_levels_async / _wait per step (AUTO sink); median of {reps} steps")
    return out


def ragged_read_path(ctx, args, rank, stream, barrier, max_over_ranks, sum_over_ranks, pmc=None) -> dict:
    """Segments of differently sized frames (64-2048 B, seeded random payloads, 1 in 10^5 frames
    with a flipped payload bit): framing alone (the serial walk defers each segment after its first
    window to the piece-parallel pass) and rh_segments_read_launch (framing + CRC verify + verdict).
    Parity: the frame table equals the generator's, the mismatch set equals the planted set, and
    two whole segments equal the oracle's literal reader walk."""
    import torch

    from oracle import oracle as orc
    from ratis_amd import _lib, engine, workload
    dev = torch.device("cuda")
    rs = workload.synth_ragged_segments(ctx, n_segments=args.ragged_segments, min_frame=64, max_frame=2048,
                                        seed=workload.SEED + 31 * rank + 5, corrupt_rate=1e-5)
    n, size = rs.n_segments, rs.segment_size
    nf = int(rs.seg_nframes.sum())
    cap = int(rs.seg_nframes.max()) + 16
    sb = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, dtype=torch.int64, device=dev) * size,
                             seg_len=torch.full((n,), size, dtype=torch.int64, device=dev), frames_per_seg_cap=cap)
    steps = max(2, args.crc_steps // 2)
    for _ in range(2):
        engine.segments_scan(ctx, sb, stream=stream)
    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    LEGS.push("ragged_framing", steps)
    e0.record(stream)
    for _ in range(steps):
        engine.segments_scan(ctx, sb, stream=stream)
    e1.record(stream)
    barrier()
    LEGS.pop()
    scan_ms = e0.elapsed_time(e1) / steps
    frame_ok = (int(sb.total_frames.item()) == nf and torch.equal(sb.frame_off[:nf], rs.batch.frame_off)
                and torch.equal(sb.frame_len[:nf], rs.batch.frame_len))
    fbatch = engine.SegmentBatch(buf=rs.batch.buf, seg_off=sb.seg_off, seg_len=sb.seg_len, frames_per_seg_cap=cap)
    for _ in range(2):
        fout = engine.read_segments_fused(ctx, fbatch, stream=stream)
    barrier()
    LEGS.push("ragged_read_launch", steps)
    e0.record(stream)
    for _ in range(steps):
        fout = engine.read_segments_fused(ctx, fbatch, stream=stream)
    e1.record(stream)
    barrier()
    LEGS.pop()
    rl_ms = e0.elapsed_time(e1) / steps
    fbad = np.nonzero(np.unpackbits(fout["bad_bits"].cpu().numpy().view(np.uint8), bitorder="little")[:nf])[0]
    clean = torch.ones(nf, dtype=torch.bool, device=dev)
    clean[torch.from_numpy(rs.corrupted).to(dev)] = False
    rl_ok = bool(np.array_equal(fbad, rs.corrupted)
                 and torch.equal(fout["crc_out"][:nf][clean], rs.batch.crc_out[:nf][clean]))
    orc_ok = True
    for sgi in (0, n - 1):
        img = rs.batch.buf[sgi * size:(sgi + 1) * size].cpu().numpy()
        ro, rl, _, rst, rstop = orc.segment_scan(img)
        k = int(sb.seg_first[sgi].item())
        m = int(sb.seg_nframes[sgi].item())
        orc_ok &= (int(sb.seg_status[sgi].item()), int(sb.seg_stop[sgi].item()), m) == (rst, rstop, len(ro)) or \
            rst == -2  # a planted corruption: the literal reader stops at its checksum
        orc_ok &= bool(np.array_equal(sb.frame_off[k:k + len(ro)].cpu().numpy() - sgi * size, ro))
    seg_bytes = n * size
    tot = sum_over_ranks(seg_bytes)
    read_alg = seg_bytes + nf * (12 + 12 + 4)
    read_ach = read_alg / (rl_ms * 1e-3) / 1e9
    out = {"workload": f"{n} x 32 MiB segments/GPU, frames of 64-2048 B ({nf} frames/GPU, {rs.corrupted.size} corrupted)",
           "framing_GBps": round(tot / (max_over_ranks(scan_ms) * 1e-3) / 1e9, 1), "ms_framing": round(scan_ms, 4),
           "framing_note": ("serial walk of the first window, then piece-parallel framing (128 KiB pieces: LDS guess "
                            "over 16 KiB, lane walks over HBM headers recording frame lengths and the next piece's "
                            "merge, stitch in parallel passes, list expansion into the slots), resume pass"),
           "read_launch_GBps": round(tot / (max_over_ranks(rl_ms) * 1e-3) / 1e9, 1), "ms_read_launch": round(rl_ms, 4),
           "parity_ok": bool(frame_ok and rl_ok and orc_ok),
           "parity_check": "frame table == generator's, mismatch set == planted set, CRCs == stamped, 2 segments == oracle reader",
           "roofline": {"bound": "hbm", "achieved": round(read_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(read_ach / HBM_PEAK_GBPS, 4),
                        "kernel": "rh_segments_read_launch (piece framing + crc_pack_kernel slot mode + verdict)",
                        "algorithmic_bytes_per_launch": read_alg, "avg_launch_ms": round(rl_ms, 4),
                        # every kernel of one read launch, PMC (scripts/pmc_ragged.py), per segment byte
                        "traffic": (round(pmc["ragged_read_bytes_per_unit"] * seg_bytes)
                                    if pmc and "ragged_read_bytes_per_unit" in pmc else None),
                        "traffic_source": (pmc or {}).get("_src", {}).get("ragged_read")}}
    del sb, fbatch, fout, rs
    return out


def _summary(line: dict) -> dict:
    """Compact copies of the headline figures of every leg (see the legs for how each is measured)."""
    def g(d, *ks):
        for k in ks:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d
    out = {"commit": {"G_updates_per_s": round(line["value"] / 1e9, 2), "us_per_launch": round(line["ms_per_step"] * 1e3, 2),
                      "hbm_frac": line["roofline"]["frac"], "pmc_over_alg": None}}
    r = line["roofline"]
    if r.get("traffic"):
        out["commit"]["pmc_over_alg"] = round(r["traffic"] / r["algorithmic_bytes_per_launch"], 3)
    c = g(line, "crc32c", "roofline")
    if c:
        out["crc32c_config5"] = {"TBps": round(c["achieved"] / 1e3, 2), "hbm_frac": c["frac"],
                                 "pmc_over_alg": round(c["traffic"] / c["algorithmic_bytes_per_launch"], 3) if c.get("traffic") else None}
    rp = g(line, "crc32c", "read_path")
    if rp and g(rp, "roofline", "frac") is not None:
        out["read_path_hbm_frac"] = rp["roofline"]["frac"]
    lr = g(line, "lease", "roofline")
    if lr:
        out["lease_hbm_frac"] = lr["frac"]
    fr = g(line, "lease", "fused_with_commit", "roofline")
    if fr:
        out["fused_commit_lease_hbm_frac"] = fr["frac"]
    tc = g(line, "pcie", "delta_streaming", "table_commit")
    if tc:
        t = {}
        for k in ("dirty_100pct", "dirty_10pct", "dirty_1pct"):
            if k in tc:
                a = tc[k].get("auto", {})
                t[k] = {"eval_us": round(tc[k]["ms_evaluation"] * 1e3, 2), "frac": tc[k]["roofline"]["frac"],
                        "host_wait_us": round(a["ms_async_to_records_host"] * 1e3, 1) if "ms_async_to_records_host" in a else None,
                        "events_us": round(a["ms_events"] * 1e3, 1) if "ms_events" in a else None,
                        "gather_us": round(tc[k]["events"]["ms_gather_kernel_auto"] * 1e3, 1),
                        "gather_vs_pcie_bound": g(tc[k], "events", "gather_vs_pcie_bound")}
        t["pcie_write_GBps"] = tc.get("pcie_write_GBps")
        out["table_commit"] = t
    tw = g(line, "pcie", "delta_streaming", "table_watch")
    if tw:
        out["table_watch_eval_us"] = {k: round(tw[k]["ms_evaluation"] * 1e3, 2) for k in ("dirty_100pct", "dirty_10pct", "dirty_1pct") if k in tw}
    tk = g(line, "pcie", "delta_streaming", "tick")
    if tk:
        out["pump_tick_us"] = {k: round(v["ms_tick_median"] * 1e3, 1) for k, v in tk.items() if isinstance(v, dict)}
        out["pump_tick_two_calls_us"] = {k: round(v["ms_two_calls_median"] * 1e3, 1) for k, v in tk.items()
                                         if isinstance(v, dict)}
    ws = g(line, "pcie", "write_stamp")
    if ws:
        out["write_stamp_16KiB_us"] = ws["gpu_us"][0]
    cb = line.get("cpu_baseline") or {}
    if cb:
        out["cpu_baseline"] = {"G_updates_per_s": round(cb["value"] / 1e9, 3), "cores": cb["cores"],
                               "crc_GBps": g(cb, "crc32c", "value")}
    out["parity_ok"] = line.get("parity_ok")
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from ratis_amd import _lib, engine, shard, workload

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # RH_BENCH_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N > 1 path on a 1-GPU box
    # (ranks share the device; timings are not per-GPU figures).  The driver's runs use RCCL with
    # one rank per GPU, where local % device_count() == local.
    backend = os.environ.get("RH_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        local %= torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    n_gpus = world
    dev = torch.device("cuda", local)
    ctx = engine.Context(local)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x: int) -> int:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.int64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    # ------------------------------------------------------------------ commit workload
    # RaftGroupIds for the whole job (1M per GPU); this rank keeps floorMod(UUID.hashCode(), N).
    msb, lsb = shard.random_group_ids(args.groups_per_gpu * n_gpus, seed=workload.SEED)
    mine = shard.shard_of(msb, lsb, n_gpus) == rank
    n_mine = int(mine.sum())
    host = workload.commit_snapshot(n_mine, joint_frac=0.10, peers=5, seed=workload.SEED + 1000 * rank)
    alg_bytes = sum(h.algorithmic_bytes() for h in host)      # per launch (per batch)
    # R rotating batches: batch r = batch 0 translated by r * 2^44 (every index column and the
    # term start).  The commit arithmetic is translation-equivariant, so batch r's results are
    # batch 0's + r * 2^44 (INT64_MIN stays for empty groups) -- checked after the timed loop.
    SHIFT = 1 << 44

    def make_batch(r, layout):
        tiers = []
        for h in host:
            d = r * SHIFT
            if layout == "tiled":
                t = engine.TiledCommitTier.from_arrays(h.follower + d, h.flush + d, h.conf, h.commit + d,
                                                       h.term_start + d, device=dev, gap_threshold=args.gap)
            else:
                t = workload.to_device(HostShift(h, d), device=dev, gap_threshold=args.gap)
                t.alloc_outputs(mode=_lib.RH_MODE_COMMIT)
            tiers.append(t)
        return tiers
    batches = [make_batch(r, args.layout) for r in range(args.rotate)]
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    # launch arguments built once per batch (engine.PreparedLaunch): the timed loop is one C-ABI
    # call per step, so the host enqueues faster than the kernels run
    commit_launches = [engine.prepare_commit(b) for b in batches]
    for i in range(args.warmup):
        commit_launches[i % args.rotate](ctx, stream)
    barrier()
    run_commit, launch_mode = captured(commit_launches, args.steps, ctx, args.graph)
    barrier()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    LEGS.push("commit", args.steps)
    queue_gate(stream)
    wall0 = time.perf_counter()
    t0.record(stream)
    run_commit(stream)
    t1.record(stream)
    barrier()
    wall = time.perf_counter() - wall0
    LEGS.pop()
    elapsed_ms = max_over_ranks(t0.elapsed_time(t1))
    # average launch duration over the timed region (back-to-back launches on one stream, so it
    # includes the ~1-2 us kernel boundaries; rocprofv3's per-kernel average is kernel-only)
    kern_ms = t0.elapsed_time(t1) / args.steps
    total_groups = sum_over_ranks(n_mine)
    value = total_groups * args.steps / (elapsed_ms / 1e3)

    # ---- correctness of the timed outputs: batch 0 vs the oracle, batch r by equivariance
    from oracle import oracle as orc
    check_ok = True
    ref0 = []
    for h in host:
        ref0.append(orc.commit_soa(h.follower, h.flush, h.conf, mode=0, gap=args.gap, commit_in=h.commit,
                                   term_start=h.term_start))
    for r, tiers in enumerate(batches[: min(args.rotate, args.steps)]):
        for h, t, ref in zip(host, tiers, ref0):
            got_c = out_col(t, "commit_out").cpu().numpy()
            got_m = out_col(t, "min_out").cpu().numpy()
            want_m = np.where(ref["min"] == np.iinfo(np.int64).min, ref["min"], ref["min"] + r * SHIFT)
            check_ok &= bool(np.array_equal(got_c, ref["commit"] + r * SHIFT) and np.array_equal(got_m, want_m))
    advanced = 0
    for h, t in zip(host, batches[0]):
        advanced += int(np.unpackbits(t.advanced_bits.cpu().numpy().view(np.uint8))[: h.n].sum())

    pmc = load_pmc(args.pmc_json)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": (round(pmc["commit_bytes_per_unit"] * n_mine) if "commit_bytes_per_unit" in pmc else None),
                "traffic_source": pmc["_src"].get("commit"),
                "kernel": f"commit_kernel_rank (fused stable F=4 + joint F=6 tiers, {args.layout} layout)",
                "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": round(kern_ms, 5)}

    # ------------------------------------------------------------------ leader lease (same groups)
    # Run right after the commit leg, before the 1.5 ms CRC / read-path launches: after those the
    # chip's clocks sat lower for the following short launches (round 2: 14.35 us per lease pass in
    # the driver's run vs 12.6 us under rocprof with the leg in this position).
    lease = {}
    lease_inputs = []
    if not args.no_lease:
        NOW = 1 << 60
        MS = 1_000_000
        TIMEOUT_MS = 100
        rng = np.random.default_rng(workload.SEED + 5 + rank)
        for h in host:
            ts = NOW - rng.integers(-MS, 3 * TIMEOUT_MS * MS, size=h.follower.shape, dtype=np.int64)
            lin = NOW - rng.integers(0, 2 * TIMEOUT_MS * MS, size=h.n, dtype=np.int64)
            lease_inputs.append((ts, h.conf, lin))
        lbatches = []
        for r in range(args.rotate):
            tiers = []
            for ts, conf, lin in lease_inputs:
                if args.lease_layout == "tiled":
                    tiers.append(engine.TiledLeaseTier.from_arrays(ts + r * SHIFT, conf, lin + r * SHIFT, device=dev))
                    continue
                t = engine.LeaseTier(follower_ts=torch.from_numpy(ts + r * SHIFT).to(dev),
                                     conf=torch.from_numpy(conf.view(np.int32)).to(dev),
                                     lease_in=torch.from_numpy(lin + r * SHIFT).to(dev))
                tiers.append(t.alloc_outputs())
            lbatches.append(tiers)
        lease_launches = [engine.prepare_lease(lbatches[r], NOW + r * SHIFT, TIMEOUT_MS) for r in range(args.rotate)]
        for i in range(args.warmup):
            lease_launches[i % args.rotate](ctx, stream)
        barrier()
        run_lease, _ = captured(lease_launches, args.steps, ctx, args.graph)
        barrier()
        l0, l1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        LEGS.push("lease", args.steps)
        queue_gate(stream)
        l0.record(stream)
        run_lease(stream)
        l1.record(stream)
        barrier()
        LEGS.pop()
        lease_kern_ms = l0.elapsed_time(l1) / args.steps
        lease_ms = max_over_ranks(lease_kern_ms)
        lease_ok = True
        for r, tiers in enumerate(lbatches[: min(args.rotate, args.steps)]):
            for (ts, conf, lin), t in zip(lease_inputs, tiers):
                ref = orc.lease_soa(ts, conf, lin, NOW, TIMEOUT_MS)
                nw = (t.n + 63) // 64
                lease_ok &= bool(np.array_equal(t.lease_out.cpu().numpy(), ref["lease"] + r * SHIFT)
                                 and np.array_equal(t.has_lease_bits[:nw].cpu().numpy().view(np.uint64),
                                                    ref["has_lease_bits"]))
        lease_alg = sum(ts.size * 8 + conf.size * 4 + lin.size * 16 + 2 * ((lin.size + 63) // 64) * 8
                        for ts, conf, lin in lease_inputs)
        lease_ach = lease_alg / (lease_kern_ms * 1e-3) / 1e9
        lease = {"checks_per_s": round(total_groups / (lease_ms * 1e-3), 1), "unit": "hasLease checks/s (whole job)",
                 "ms_per_pass": round(lease_ms, 5), "parity_ok": lease_ok, "timeout_ms": TIMEOUT_MS,
                 "roofline": {"bound": "hbm", "achieved": round(lease_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                              "frac": round(lease_ach / HBM_PEAK_GBPS, 4), "kernel": f"lease_kernel<0,7,true,8> (F=4 and F=6 tiers in one launch, {args.lease_layout} layout)",
                              "traffic": (round(pmc["lease_bytes_per_unit"] * n_mine) if "lease_bytes_per_unit" in pmc
                                          else None),
                              "traffic_source": pmc["_src"].get("lease"),
                              "algorithmic_bytes_per_launch": lease_alg}}
        # ---- the fused launch: updateCommit + hasLease of the same 1M divisions in ONE kernel
        # (rh_leader_soa_launch), rotating over the same batches
        leader_launches = [engine.prepare_leader(batches[r], lbatches[r], NOW + r * SHIFT, TIMEOUT_MS)
                           for r in range(args.rotate)]
        for i in range(args.warmup):
            leader_launches[i % args.rotate](ctx, stream)
        barrier()
        run_leader, _ = captured(leader_launches, args.steps, ctx, args.graph)
        barrier()
        LEGS.push("fused", args.steps)
        queue_gate(stream)
        l0.record(stream)
        run_leader(stream)
        l1.record(stream)
        barrier()
        LEGS.pop()
        fused_kern_ms = l0.elapsed_time(l1) / args.steps
        fused_ms = max_over_ranks(fused_kern_ms)
        fused_ok = True
        for r in range(min(args.rotate, args.steps)):
            for h, t, ref in zip(host, batches[r], ref0):
                want_m = np.where(ref["min"] == np.iinfo(np.int64).min, ref["min"], ref["min"] + r * SHIFT)
                fused_ok &= bool(np.array_equal(out_col(t, "commit_out").cpu().numpy(), ref["commit"] + r * SHIFT)
                                 and np.array_equal(out_col(t, "min_out").cpu().numpy(), want_m))
            for (ts, conf, lin), t in zip(lease_inputs, lbatches[r]):
                ref = orc.lease_soa(ts, conf, lin, NOW, TIMEOUT_MS)
                nw = (t.n + 63) // 64
                fused_ok &= bool(np.array_equal(t.lease_out.cpu().numpy(), ref["lease"] + r * SHIFT)
                                 and np.array_equal(t.has_lease_bits[:nw].cpu().numpy().view(np.uint64),
                                                    ref["has_lease_bits"]))
        fused_alg = alg_bytes + lease_alg
        fused_ach = fused_alg / (fused_kern_ms * 1e-3) / 1e9
        lease["fused_with_commit"] = {
            "ms_per_launch": round(fused_ms, 5), "parity_ok": fused_ok,
            "updates_per_s": round(total_groups / (fused_ms * 1e-3), 1),
            "note": "one rh_leader_soa_launch per step: updateCommit (config 3 tiers) + hasLease (same groups) "
                    "in one kernel; vs the two separate launches "
                    f"{round(kern_ms + lease_kern_ms, 5)} ms",
            "roofline": {"bound": "hbm", "achieved": round(fused_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(fused_ach / HBM_PEAK_GBPS, 4), "kernel": "leader_kernel (commit_kernel_rank + lease blocks)",
                         "algorithmic_bytes_per_launch": fused_alg, "avg_launch_ms": round(fused_kern_ms, 5)}}
        del lbatches

    # ------------------------------------------------------------------ PCIe-inclusive commit
    pcie = {}
    if not args.no_pcie:
        hb = []
        for h in host:
            hb.append({k: torch.from_numpy(np.ascontiguousarray(v)).pin_memory()
                       for k, v in (("f", h.follower), ("s", h.flush), ("c", h.commit), ("t", h.term_start),
                                    ("w", h.conf.view(np.int32)))})
        outs = [torch.empty(h.n, dtype=torch.int64).pin_memory() for h in host]
        tiers = make_batch(0, "plain")
        reps = 5
        torch.cuda.synchronize()
        pa = torch.cuda.Event(enable_timing=True)
        pb = torch.cuda.Event(enable_timing=True)
        pa.record(stream)
        for _ in range(reps):
            for t, b in zip(tiers, hb):
                t.follower_index.copy_(b["f"], non_blocking=True)
                t.self_index.copy_(b["s"], non_blocking=True)
                t.commit_in.copy_(b["c"], non_blocking=True)
                t.term_start.copy_(b["t"], non_blocking=True)
                t.conf.copy_(b["w"], non_blocking=True)
            engine.commit_launch(ctx, tiers, stream=stream)
            for t, o in zip(tiers, outs):
                o.copy_(t.commit_out, non_blocking=True)
        pb.record(stream)
        torch.cuda.synchronize()
        ms = pa.elapsed_time(pb) / reps
        pcie["commit_updates_per_s_incl_pcie"] = round(n_mine / (ms * 1e-3), 1)
        pcie["commit_ms_incl_pcie_full_snapshot"] = round(ms, 4)
        pcie["note"] = "full snapshot H2D (pinned) + kernel + commit D2H per batch"
        pcie["delta_streaming"] = delta_streaming(ctx, host, fill_threads=cpu_threads())
        pcie["delta_streaming"]["table_commit"] = table_commit_leg(ctx, host, pmc=pmc)
        pcie["delta_streaming"]["table_watch"] = table_watch_leg(ctx, host)
        pcie["delta_streaming"]["tick"] = tick_leg(ctx, host)
        pcie["delta_streaming"]["reply_mix"] = reply_mix_leg(host, threads=cpu_threads())
        pcie["write_stamp"] = write_stamp_leg(ctx)

    # ------------------------------------------------------------------ CRC32C (config 5)
    crc = {}
    frames_verified = bytes_verified = mismatches = 0
    if args.crc_segments > 0:
        ss = workload.synth_segments(ctx, n_segments=args.crc_segments, seed=workload.SEED + 77 * rank,
                                     device=dev)
        fb = ss.batch
        # warm up until the launch time has settled: right after the commit and lease legs the
        # first config-5 passes run 1.53 -> 2.07 -> 1.55 ms over ~20 launches (a clock / power
        # transient seen in the run8 kernel trace, profiles/r02/crc_warmup/); 2 passes left it
        # inside the timed region
        for i in range(max(2, args.crc_warmup)):
            engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, stream=stream)
        barrier()
        c0 = torch.cuda.Event(enable_timing=True)
        c1 = torch.cuda.Event(enable_timing=True)
        LEGS.push("crc", args.crc_steps)
        c0.record(stream)
        for i in range(args.crc_steps):
            engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, stream=stream)
        c1.record(stream)
        barrier()
        LEGS.pop()
        crc_kern_ms = c0.elapsed_time(c1) / args.crc_steps
        crc_ms = max_over_ranks(crc_kern_ms)
        fb.n_bad.zero_()
        fb.bad_bits.zero_()
        engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, stream=stream)
        torch.cuda.synchronize()
        bad = np.nonzero(np.unpackbits(fb.bad_bits.cpu().numpy().view(np.uint8), bitorder="little")[: fb.n])[0]
        frames_verified = fb.n * (args.crc_steps + 3)
        bytes_verified = frames_verified * ss.frame_size
        mismatches = int(bad.size)
        # parity of the timed kernel's outputs: EVERY frame's CRC against the oracle over the same
        # bytes (16 host threads), and the mismatch set against the oracle's own comparison of
        # each stored trailer -- independent of the generator's GPU-stamped trailers
        t_or = time.perf_counter()
        img = fb.buf.cpu().numpy()
        want_crc, want_bad = orc.crc32c_frames_all(img, fb.frame_off.cpu().numpy(), fb.frame_len.cpu().numpy(),
                                                   threads=cpu_threads())
        crc_ok = bool(np.array_equal(fb.crc_out.cpu().numpy().view(np.uint32), want_crc)
                      and np.array_equal(bad, np.nonzero(want_bad)[0]) and np.array_equal(bad, ss.corrupted))
        crc_check_s = time.perf_counter() - t_or
        del img, want_crc, want_bad
        frame_bytes = ss.frame_bytes
        meta_bytes = fb.n * (8 + 4 + 4)   # offset + length read, crc written (bits negligible)
        crc_alg = frame_bytes + meta_bytes
        total_frame_bytes = sum_over_ranks(frame_bytes)
        crc_gbps = total_frame_bytes / (crc_ms * 1e-3) / 1e9
        crc_ach = crc_alg / (crc_kern_ms * 1e-3) / 1e9
        crc = {"GBps": round(crc_gbps, 1), "unit": "GB/s (frame bytes, whole job)",
               "workload": f"config5: {args.crc_segments} x 32 MiB segments/GPU, 4 KiB frames "
                           f"({fb.n} frames/GPU, {ss.corrupted.size} corrupted)",
               "ms_per_pass": round(crc_ms, 4), "mismatches_found": int(bad.size), "parity_ok": crc_ok,
               "parity_check": f"all {fb.n} frames vs the oracle ({crc_check_s:.1f} s on {cpu_threads()} threads)",
               "roofline": {"bound": "hbm", "achieved": round(crc_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(crc_ach / HBM_PEAK_GBPS, 4),
                            "traffic": (round(pmc["crc_bytes_per_unit"] * fb.n) if "crc_bytes_per_unit" in pmc else None),
                            "traffic_source": pmc["_src"].get("crc"),
                            "kernel": "crc_frames_kernel (16 lanes x 64 B per 1 KiB window, copy-free 3-slot ring, LDS-staged frame table, 2 fold chains/lane)",
                            "algorithmic_bytes_per_launch": crc_alg, "avg_launch_ms": round(crc_kern_ms, 4)}}
        # ---- read path: framing walk, then framing + verify, over the same segment images
        n_seg = args.crc_segments
        sb = engine.SegmentBatch(buf=fb.buf,
                                 seg_off=torch.arange(n_seg, dtype=torch.int64, device=dev) * ss.segment_size,
                                 seg_len=torch.full((n_seg,), ss.segment_size, dtype=torch.int64, device=dev),
                                 frames_per_seg_cap=ss.frames_per_segment + 16)
        for _ in range(2):
            engine.segments_scan(ctx, sb, stream=stream)
        barrier()
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        LEGS.push("framing", args.crc_steps)
        f0.record(stream)
        for _ in range(args.crc_steps):
            engine.segments_scan(ctx, sb, stream=stream)
        f1.record(stream)
        barrier()
        LEGS.pop()
        scan_ms = f0.elapsed_time(f1) / args.crc_steps
        nfr_found = int(sb.total_frames.item())
        frame_ok = (nfr_found == fb.n and torch.equal(sb.frame_off[:fb.n], fb.frame_off)
                    and torch.equal(sb.frame_len[:fb.n], fb.frame_len)
                    and bool((sb.seg_status[:n_seg] == _lib.RH_SEG_END).all()))
        rb = engine.FrameBatch(buf=fb.buf, frame_off=sb.frame_off[:fb.n], frame_len=sb.frame_len[:fb.n])
        rb.alloc_outputs()
        barrier()
        LEGS.push("framing_plus_verify", args.crc_steps)
        f0.record(stream)
        for _ in range(args.crc_steps):
            engine.segments_scan(ctx, sb, stream=stream)
            engine.crc32c_frames(ctx, rb, flags=_lib.RH_CRC_VERIFY, stream=stream)
        f1.record(stream)
        barrier()
        LEGS.pop()
        read_ms = f0.elapsed_time(f1) / args.crc_steps
        # rh_segments_read_launch (LogSegment.readSegmentFile in one call): framing walk + CRC over
        # the slotted frame table + verdict
        fbatch = engine.SegmentBatch(buf=fb.buf, seg_off=sb.seg_off, seg_len=sb.seg_len,
                                     frames_per_seg_cap=ss.frames_per_segment + 16)
        for _ in range(2):
            fout = engine.read_segments_fused(ctx, fbatch, stream=stream)
        barrier()
        LEGS.push("read_launch", args.crc_steps)
        f0.record(stream)
        for _ in range(args.crc_steps):
            fout = engine.read_segments_fused(ctx, fbatch, stream=stream)
        f1.record(stream)
        barrier()
        LEGS.pop()
        rl_ms = f0.elapsed_time(f1) / args.crc_steps
        fbad = np.nonzero(np.unpackbits(fout["bad_bits"].cpu().numpy().view(np.uint8), bitorder="little")[: fb.n])[0]
        rl_ok = bool(np.array_equal(fbad, ss.corrupted) and int(fbatch.total_frames.item()) == fb.n
                     and torch.equal(fbatch.frame_off[: fb.n], fb.frame_off)
                     and torch.equal(fout["crc_out"][: fb.n], fb.crc_out[: fb.n]))
        del fbatch, fout
        seg_bytes = n_seg * ss.segment_size
        tot_seg_bytes = sum_over_ranks(seg_bytes)
        # framing + verify (the read path): the CRC pass reads every frame byte, the framing walk
        # only headers + the padding tail; algorithmic bytes = segment bytes + frame table
        # (12 B/frame written by the walk, read by the CRC pass) + 4 B/frame CRC out
        read_alg = seg_bytes + fb.n * (12 + 12 + 4)
        read_ach = read_alg / (read_ms * 1e-3) / 1e9
        crc["read_path"] = {
            "framing_GBps": round(tot_seg_bytes / (max_over_ranks(scan_ms) * 1e-3) / 1e9, 1),
            "framing_note": ("segment bytes framed per second; the walk reads frame headers (LDS windows, "
                             "then a header fast-forward straight through HBM over runs of equal-length "
                             "frames) and the padding tail, not the payload: latency-bound, not HBM-bound"),
            "framing_traffic_bytes": (round(pmc["framing_bytes_per_unit"] * n_seg) if "framing_bytes_per_unit" in pmc
                                      else None),
            "framing_plus_verify_GBps": round(tot_seg_bytes / (max_over_ranks(read_ms) * 1e-3) / 1e9, 1),
            "read_launch_GBps": round(tot_seg_bytes / (max_over_ranks(rl_ms) * 1e-3) / 1e9, 1),
            "ms_read_launch": round(rl_ms, 4), "read_launch_parity_ok": rl_ok,
            "read_launch_note": "rh_segments_read_launch (walk + CRC + verdict in one call)",
            "unit": "GB/s (segment bytes, whole job)", "frames_found": nfr_found, "parity_ok": bool(frame_ok),
            "ms_framing": round(scan_ms, 4), "ms_framing_plus_verify": round(read_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(read_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(read_ach / HBM_PEAK_GBPS, 4),
                         "traffic": ((round(pmc["framing_bytes_per_unit"] * n_seg) if "framing_bytes_per_unit" in pmc
                                      else 0) + round(pmc.get("crc_bytes_per_unit", 0) * fb.n)) or None,
                         "traffic_source": [pmc["_src"].get("framing"), pmc["_src"].get("crc")],
                         "kernel": "segment_walk_kernel<32768> (+ scan, compact) then crc_frames_kernel",
                         "algorithmic_bytes_per_launch": read_alg}}
        del sb, rb
        if not args.no_pcie:
            # host image of 8 segments (256 MiB) -> H2D pinned + verify
            nseg = min(8, args.crc_segments)
            hsz = nseg * ss.segment_size
            himg = fb.buf[:hsz].cpu().pin_memory()
            nfr = nseg * ss.frames_per_segment
            sub = engine.FrameBatch(buf=torch.empty(hsz, dtype=torch.uint8, device=dev),
                                    frame_off=fb.frame_off[:nfr].clone(), frame_len=fb.frame_len[:nfr].clone())
            sub.alloc_outputs()
            hcrc = torch.empty(nfr, dtype=torch.int32).pin_memory()
            torch.cuda.synchronize()
            pa = torch.cuda.Event(enable_timing=True)
            pb = torch.cuda.Event(enable_timing=True)
            pa.record(stream)
            for _ in range(3):
                sub.buf.copy_(himg, non_blocking=True)
                engine.crc32c_frames(ctx, sub, flags=_lib.RH_CRC_VERIFY, stream=stream)
                hcrc.copy_(sub.crc_out, non_blocking=True)
            pb.record(stream)
            torch.cuda.synchronize()
            ms = pa.elapsed_time(pb) / 3
            pcie["crc32c_GBps_incl_pcie"] = round(nfr * ss.frame_size / (ms * 1e-3) / 1e9, 2)
        del ss, fb
        torch.cuda.empty_cache()
        if args.ragged_segments:
            crc["read_path"]["ragged"] = ragged_read_path(ctx, args, rank, stream, barrier, max_over_ranks,
                                                          sum_over_ranks, pmc=pmc)
            torch.cuda.empty_cache()

    # ------------------------------------------------------------------ CPU baseline (rank 0, N = 1)
    # The oracle (scalar C restatement of the reference's Java arithmetic), timed on this host on a
    # bounded sample: once on 1 thread, once on every core of this job's CPU share (ctypes drops the
    # GIL, so Python threads run the C passes in parallel over static slices).
    cpu = None
    cpu_note = None
    if world > 1:
        cpu_note = ("measured on rank 0 at N = 1 only (the bench contract): the per-GPU work is the same "
                    "1M-group snapshot, so the N = 1 line's cpu_baseline is the host-core figure for every N")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_threads()
        # each thread owns a static slice of BOTH tiers (stable F=4 and joint F=6) of the snapshot
        def slices(h, i, k):
            p = slice(h.n * i // k, h.n * (i + 1) // k)
            return (np.ascontiguousarray(h.follower[:, p]), h.flush[p].copy(), h.conf[p].copy(), h.commit[p].copy(),
                    h.term_start[p].copy())
        items = [tuple(slices(h, i, threads) for h in host) for i in range(threads)]

        def commit_pass(*tiers):
            for f, sf, c, ci, ts in tiers:
                orc.commit_soa(f, sf, c, mode=0, gap=args.gap, commit_in=ci, term_start=ts)
            return sum(t[1].size for t in tiers)
        one = timed_passes([tuple(slices(h, 0, 1) for h in host)], commit_pass, 4.0)
        allc = timed_passes(items, commit_pass, 4.0)
        n_groups = sum(h.n for h in host)
        cpu = {"value": round(allc["rate"], 1), "unit": "updates/s", "cores": threads, "kind": "port",
               "sample": f"{allc['passes']} passes of orc_commit_soa over {threads} static slices of the whole "
                         f"{n_groups}-group snapshot (stable F=4 and joint F=6 tiers; {allc['seconds']:.1f} s; scalar C "
                         f"restatement of LeaderStateImpl.getMajorityMin/updateCommit + RaftLogBase.updateCommitIndex, "
                         f"getSorted with the insertion sort Arrays.sort(long[]) runs below 47 elements, "
                         f"{threads} threads)",
               "single_core": {"value": round(one["rate"], 1), "cores": 1,
                               "sample": f"{one['passes']} passes over the whole snapshot ({one['seconds']:.1f} s)"},
               "host": host_cpu_model()}
        if args.crc_segments > 0:
            rng = np.random.default_rng(5)
            nseg = 8
            fps = (32 << 20) // 4096 - 1
            sample = rng.integers(0, 256, size=nseg * (32 << 20), dtype=np.uint8)
            offs = (np.repeat(np.arange(nseg) * (32 << 20), fps) + 8
                    + np.tile(np.arange(fps) * 4096, nseg)).astype(np.uint64)
            lens = np.full(offs.size, 4096, dtype=np.uint32)

            def crc_pass(o, ln):
                orc.crc32c_frames(sample, o, ln)
                return o.size * 4096
            cparts = [slice(offs.size * i // threads, offs.size * (i + 1) // threads) for i in range(threads)]
            one = timed_passes([(offs, lens)], crc_pass, 4.0)
            allc = timed_passes([(offs[p].copy(), lens[p].copy()) for p in cparts], crc_pass, 4.0)
            crc["cpu_baseline"] = {
                "value": round(allc["rate"] / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
                "sample": f"{allc['passes']} slice passes over 8 x 32 MiB segment images ({offs.size} 4 KiB frames) "
                          f"split across {threads} threads, PureJavaCrc32C slicing-by-8 restatement ({allc['seconds']:.1f} s)",
                "single_core": {"value": round(one["rate"] / 1e9, 3), "cores": 1,
                                "sample": f"{one['passes']} passes over the 8 images ({one['seconds']:.1f} s)"}}
        if lease_inputs:
            ts, conf, lin = lease_inputs[0]
            lparts = [slice(conf.size * i // threads, conf.size * (i + 1) // threads) for i in range(threads)]

            def lease_pass(t, c, li):
                orc.lease_soa(t, c, li, 1 << 60, 100)
                return c.size
            one = timed_passes([(ts, conf, lin)], lease_pass, 3.0)
            allc = timed_passes([(np.ascontiguousarray(ts[:, p]), conf[p].copy(), lin[p].copy()) for p in lparts],
                                lease_pass, 3.0)
            lease["cpu_baseline"] = {
                "value": round(allc["rate"], 1), "unit": "checks/s", "cores": threads, "kind": "port",
                "sample": f"{allc['passes']} slice passes of orc_lease_soa over the {conf.size}-group stable tier "
                          f"split across {threads} threads ({allc['seconds']:.1f} s, literal LeaderLease restatement)",
                "single_core": {"value": round(one["rate"], 1), "cores": 1,
                                "sample": f"{one['passes']} passes over the whole tier ({one['seconds']:.1f} s)"}}

    stats = shard.allreduce_stats({"groups_evaluated": n_mine * args.steps, "commits_advanced": advanced,
                                   "frames_verified": frames_verified, "bytes_verified": bytes_verified,
                                   "crc_mismatches": mismatches}, device=dev)

    # The metric's second half (log CRC32C GB/s, config 5) also rides inside the two objects the
    # driver keeps whole (roofline, cpu_baseline): its parsed copy drops the long nested legs.
    if crc.get("roofline"):
        r = crc["roofline"]
        roofline["crc32c"] = {"GBps_whole_job": crc["GBps"], "achieved": r["achieved"], "frac": r["frac"],
                              "avg_launch_ms": r["avg_launch_ms"], "traffic": r["traffic"],
                              "traffic_source": r["traffic_source"], "kernel": "crc_frames_kernel",
                              "algorithmic_bytes_per_launch": r["algorithmic_bytes_per_launch"],
                              "parity_ok": crc.get("parity_ok")}
    if cpu is not None and crc.get("cpu_baseline"):
        cpu["crc32c"] = {k: crc["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind")}
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "updates/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_ms / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {"workload": "config3: 1M RaftGroups x 5 peers per GPU, 10% joint consensus (old+new conf), "
                               "updateCommit + updateCommitIndex per group",
                   "groups_per_gpu": args.groups_per_gpu, "groups_this_job": total_groups, "peers": 5,
                   "joint_fraction": 0.10, "gap_threshold": args.gap, "rotating_batches": args.rotate,
                   "layout": args.layout, "timed_launches": launch_mode,
                   "sharding": f"RaftGroupId UUID.hashCode() floorMod {n_gpus}"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        **({"cpu_baseline_note": cpu_note} if cpu_note else {}),
        "crc32c": crc,
        "lease": lease,
        "pcie": pcie,
        "parity_ok": check_ok,
        "advanced_groups_batch0_rank0": advanced,
        "stats": stats,
        "wall_s_timed_region": round(wall, 4),
    }
    # The driver keeps the last ~2000 characters of this line: the figures a reader looks for first,
    # again, compactly, at its end (every one of them is in the legs above with its method).
    line["summary"] = _summary(line)
    if rank == 0:
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
