"""Host model of the resident group table for the parity tests -- TEST INFRASTRUCTURE ONLY.

It keeps, per slot, what the reference keeps per leader division and replays the reference's
semantics step by step; the commit arithmetic itself is the oracle's (orc_commit_soa):

  start     new LeaderStateImpl: every FollowerInfo is new, matchIndex = commitIndex = -1
            (FollowerInfoImpl.java:42-43; LeaderStateImpl.java:421-430, 681-692)
  reconf    conf change: follower k keeps old follower src[k]'s FollowerInfo or gets a new one
            (LeaderStateImpl.java:624-633, 681-692, 704-724, 1064-1074)
  deltas    RaftLogIndex.updateToMax (FollowerInfoImpl.java:93-105) / setUnconditionally
            (FollowerInfoImpl.java:147-151), applied one by one in array order
  commit    updateCommit() for every started slot (LeaderStateImpl.java:946-950, 1015-1026):
            the slots whose commit index advanced, and the slots whose watch-ALL level changed
  watch     commitIndexChanged() (LeaderStateImpl.java:606-622): slots whose levels changed

Follower columns a slot's tier does not have (beyond its width, ratis_hip.h) read -1, exactly as
the table reports them.
"""
from __future__ import annotations

import numpy as np

MAXF = 14
IMIN = np.iinfo(np.int64).min
COL_FLUSH, COL_COMMITTED = 32, 33
OP_MAX, OP_SET = 0, 1


def needed_width(conf: int) -> int:
    m = (conf & 0x3FFF) | ((conf >> 16) & 0x3FFF)
    return m.bit_length()


def tier_width(conf: int) -> int:
    w = needed_width(conf)
    return 2 if w <= 2 else 2 * ((w + 1) // 2)


class TableModel:
    def __init__(self, capacity: int, gap: int = -1):
        self.cap, self.gap = capacity, gap
        self.started = np.zeros(capacity, bool)
        self.conf = np.zeros(capacity, np.uint32)
        self.width = np.zeros(capacity, np.int64)
        self.match = np.full((MAXF, capacity), -1, np.int64)
        self.fcommit = np.full((MAXF, capacity), -1, np.int64)
        self.flush = np.zeros(capacity, np.int64)
        self.commit = np.zeros(capacity, np.int64)
        self.tstart = np.zeros(capacity, np.int64)
        self.wall = np.full(capacity, IMIN, np.int64)
        self.wlev = np.full((3, capacity), IMIN, np.int64)

    # -- control ---------------------------------------------------------------------------
    def start(self, slot, conf, flush, commit, tstart):
        self.started[slot] = True
        self.conf[slot] = conf
        self.width[slot] = tier_width(conf)
        self.match[:, slot] = -1
        self.fcommit[:, slot] = -1
        self.flush[slot], self.commit[slot], self.tstart[slot] = flush, commit, tstart
        self.wall[slot] = IMIN
        self.wlev[:, slot] = IMIN

    def reconf(self, slot, conf, src=None):
        assert self.started[slot]
        old_w = int(self.width[slot])
        new_w = tier_width(conf)
        src = list(range(MAXF)) if src is None else list(src) + [-1] * (MAXF - len(src))
        m = np.full(MAXF, -1, np.int64)
        f = np.full(MAXF, -1, np.int64)
        for k in range(new_w):
            s = src[k]
            if 0 <= s < old_w:
                m[k], f[k] = self.match[s, slot], self.fcommit[s, slot]
        self.match[:, slot], self.fcommit[:, slot] = m, f
        self.conf[slot] = conf
        self.width[slot] = new_w

    def stop(self, slot):
        self.started[slot] = False

    def load(self, first, conf, flush, commit, tstart, match=None, fcommit=None):
        for i in range(conf.size):
            s = first + i
            self.start(s, int(conf[i]), int(flush[i]), int(commit[i]), int(tstart[i]))
            w = int(self.width[s])
            for arr, dst in ((match, self.match), (fcommit, self.fcommit)):
                if arr is not None:
                    k = min(w, arr.shape[0])
                    dst[:k, s] = arr[:k, i]

    # -- deltas ----------------------------------------------------------------------------
    def apply(self, d):
        if d.size == 0:
            return
        if not (d["op"] == OP_SET).any():
            self._apply_max(d)
            return
        for x in d:   # sequential semantics
            self._apply_one(int(x["slot"]), int(x["column"]), int(x["op"]), int(x["value"]))

    def _cell(self, slot, col):
        if col < 16:
            return self.match, col
        if col < 32:
            return self.fcommit, col - 16
        return None, col

    def _apply_one(self, slot, col, op, v):
        if col == COL_FLUSH:
            self.flush[slot] = v if op == OP_SET else max(self.flush[slot], v)
        elif col == COL_COMMITTED:
            self.commit[slot] = v if op == OP_SET else max(self.commit[slot], v)
        else:
            arr, k = self._cell(slot, col)
            arr[k, slot] = v if op == OP_SET else max(arr[k, slot], v)

    def _apply_max(self, d):
        s = d["slot"].astype(np.int64)
        c = d["column"].astype(np.int64)
        v = d["value"].astype(np.int64)
        m = c < 16
        np.maximum.at(self.match, (c[m], s[m]), v[m])
        m = (c >= 16) & (c < 32)
        np.maximum.at(self.fcommit, (c[m] - 16, s[m]), v[m])
        m = c == COL_FLUSH
        np.maximum.at(self.flush, s[m], v[m])
        m = c == COL_COMMITTED
        np.maximum.at(self.commit, s[m], v[m])

    # -- evaluation ------------------------------------------------------------------------
    def _soa(self, orc, mode):
        idx = np.nonzero(self.started)[0]
        col = self.match if mode == 0 else self.fcommit
        self_i = self.flush if mode == 0 else self.commit
        r = orc.commit_soa(np.ascontiguousarray(col[:, idx]), self_i[idx], self.conf[idx], mode=mode,
                           gap=self.gap if mode == 0 else -1, commit_in=self.commit[idx], term_start=self.tstart[idx])
        return idx, r

    def commit_batch(self, orc):
        idx, r = self._soa(orc, 0)
        adv = r["commit"] != self.commit[idx]
        chg = r["min"] != self.wall[idx]
        self.commit[idx] = r["commit"]
        self.wall[idx] = r["min"]
        return idx[adv], r["commit"][adv], idx[chg], r["min"][chg]

    def watch(self, orc):
        idx, r = self._soa(orc, 1)
        new = np.stack([r["min"], r["maj"], r["max"]])
        chg = (new != self.wlev[:, idx]).any(axis=0)
        self.wlev[:, idx] = new
        valid = np.unpackbits(r["valid_bits"].view(np.uint8), bitorder="little")[: idx.size].astype(bool)
        return idx[chg], new[:, chg], valid[chg]

    def column(self, col):
        """What rh_groups_read returns for every slot."""
        out = np.full(self.cap, IMIN, np.int64)
        s = self.started
        if col < 16 or 16 <= col < 32:
            arr, k = self._cell(0, col)
            v = arr[k].copy()
            v[k >= self.width] = -1
            out[s] = v[s]
        elif col == COL_FLUSH:
            out[s] = self.flush[s]
        elif col == COL_COMMITTED:
            out[s] = self.commit[s]
        elif col == 34:
            out[s] = self.conf[s].astype(np.int64)
        elif col == 35:
            out[s] = self.tstart[s]
        return out
