/*
 * Server-level leader bookkeeping on the GPU: one instance per RaftServerProxy (RaftServerProxy.java:
 * 89-150 holds every division of a server) when raft.server.hip.commit.backend = hip.
 *
 * It replaces, for every leader division at once, what LeaderStateImpl does per division:
 *   - the FollowerInfoMap and the MinMajorityMax arithmetic (LeaderStateImpl.java:230-294, 904-984):
 *     follower slots k per division, the membership word of RaftConfigurationImpl's conf / oldConf
 *     restricted to peers with a FollowerInfo (LeaderStateImpl.java:291-293);
 *   - the per-division EventProcessor thread and its UPDATE_COMMIT queue (LeaderStateImpl.java:111-188,
 *     791-816): producers append 16-byte deltas; ONE pump thread pushes them and runs the batched
 *     updateCommit over the dirty divisions;
 *   - RaftLogBase.updateCommitIndex's decision (RaftLogBase.java:121-142).
 * The follow-up the reference runs after a successful updateCommitIndex -- getEntries, the real
 * ServerState.updateCommitIndex, StateMachineUpdater.notifyUpdater, watch release -- stays in the
 * division's LeaderStateImpl (Callback.onCommit), for the advanced divisions only.
 */
package org.apache.ratis.hip;

import org.apache.ratis.protocol.RaftGroupId;
import org.apache.ratis.protocol.RaftPeerId;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.Collection;
import java.util.Deque;
import java.util.HashMap;
import java.util.Map;
import java.util.UUID;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.locks.LockSupport;

public final class HipLeaderBookkeeper implements AutoCloseable {
  /** What a division's LeaderStateImpl does with the GPU's decisions (run on the pump thread). */
  public interface Callback {
    /** updateCommit(majority, min) found a new commit index (LeaderStateImpl.java:1015-1026). */
    void onCommit(long newCommitIndex);
    /** watchRequests.update(ALL, min) with a changed level (LeaderStateImpl.java:1025). */
    void onWatchAll(long min);
  }

  private final RatisHip hip;
  private final long capacity;
  private final Deque<Integer>[] freeSlots;
  private final Map<Integer, Division> divisions = new ConcurrentHashMap<>();
  private final ByteBuffer deltas;         // producers' deltas (node slots), drained by the pump
  private final Object deltaLock = new Object();
  private final Thread pump;
  private final long tickNanos;
  private volatile boolean watchAll;       // some division has ALL-level watch requests
  private volatile boolean running = true;
  private volatile long leaseTimeoutMs = -1;  // LeaderLease.leaseTimeoutMs; -1: no lease batches
  private volatile long[] leaseBits;          // last rh_node_lease_batch: bit = node slot has the lease

  @SuppressWarnings("unchecked")
  public HipLeaderBookkeeper(int deviceMask, long capacityPerShard, long gapThreshold, long tickMicros)
      throws IOException {
    this.hip = new RatisHip(deviceMask, capacityPerShard, gapThreshold);
    this.capacity = capacityPerShard;
    this.freeSlots = new Deque[hip.getShards()];
    for (int s = 0; s < freeSlots.length; s++) {
      freeSlots[s] = new ArrayDeque<>();
      for (long i = capacityPerShard - 1; i >= 0; i--) {
        freeSlots[s].push((int) i);
      }
    }
    this.deltas = ByteBuffer.allocateDirect(RatisHip.DELTA_BYTES << 20).order(ByteOrder.LITTLE_ENDIAN);
    this.tickNanos = TimeUnit.MICROSECONDS.toNanos(tickMicros);
    this.pump = new Thread(this::pumpLoop, "ratis-hip-commit-pump");
    this.pump.setDaemon(true);
    this.pump.start();
  }

  public void setWatchAll(boolean enabled) {
    this.watchAll = enabled;
  }

  /** rpc.timeout.min x read.leader.lease.timeout.ratio (LeaderLease.java:45-48); the pump then
   * evaluates hasLease() for every division each tick. */
  public void setLeaseTimeoutMs(long ms) {
    this.leaseTimeoutMs = ms;
  }

  /** A new leader division (new LeaderStateImpl, LeaderStateImpl.java:365-430). */
  public synchronized Division register(RaftGroupId groupId, RaftPeerId selfId, Callback callback) {
    final UUID u = groupId.getUuid();
    final int shard = hip.shardOf(u.getMostSignificantBits(), u.getLeastSignificantBits());
    final Integer slot = freeSlots[shard].poll();
    if (slot == null) {
      throw new IllegalStateException("ratis-hip: shard " + shard + " is full (" + capacity + " divisions)");
    }
    final int nodeSlot = (int) (shard * capacity + slot);
    final Division d = new Division(nodeSlot, selfId, callback);
    divisions.put(nodeSlot, d);
    return d;
  }

  synchronized void release(Division d) {
    divisions.remove(d.nodeSlot);
    freeSlots[(int) (d.nodeSlot / capacity)].push((int) (d.nodeSlot % capacity));
  }

  /** Appends one delta; the caller holds deltaLock (one ordered stream of deltas and control ops). */
  private void putDeltaLocked(int nodeSlot, int column, int op, long value) {
    if (deltas.remaining() < RatisHip.DELTA_BYTES) {
      drainDeltas();
    }
    RatisHip.putDelta(deltas, nodeSlot, column, op, value);
  }

  private void drainDeltas() {
    final int n = deltas.position() / RatisHip.DELTA_BYTES;
    if (n == 0) {
      return;
    }
    try {
      hip.pushDeltas(deltas, n);
    } catch (IOException e) {
      throw new IllegalStateException("ratis-hip: pushDeltas failed", e);
    }
    deltas.clear();
  }

  private void pumpLoop() {
    final int cap = (int) Math.min(Integer.MAX_VALUE - 8, capacity * hip.getShards());
    final int[] advSlot = new int[cap];
    final long[] advCommit = new long[cap];
    final int[] wallSlot = new int[cap];
    final long[] wallMin = new long[cap];
    while (running) {
      LockSupport.parkNanos(tickNanos);
      synchronized (deltaLock) {
        drainDeltas();
      }
      final long counts;
      try {
        counts = watchAll ? hip.commitBatch(advSlot, advCommit, wallSlot, wallMin)
                          : hip.commitBatch(advSlot, advCommit, null, null);
      } catch (IOException e) {
        throw new IllegalStateException("ratis-hip: commitBatch failed", e);
      }
      final int nAdv = (int) Math.min(counts >>> 32, cap);
      for (int i = 0; i < nAdv; i++) {
        final Division d = divisions.get(advSlot[i]);
        if (d != null) {
          d.callback.onCommit(advCommit[i]);
        }
      }
      final int nWall = (int) Math.min(counts & 0xFFFFFFFFL, cap);
      for (int i = 0; i < nWall; i++) {
        final Division d = divisions.get(wallSlot[i]);
        if (d != null) {
          d.callback.onWatchAll(wallMin[i]);
        }
      }
      final long timeout = leaseTimeoutMs;
      if (timeout >= 0) {  // LeaderStateImpl.hasLease for every division: extend + isValid
        final long[] bits = new long[(cap + 63) / 64];
        try {
          hip.leaseBatch(System.nanoTime(), timeout, bits);
        } catch (IOException e) {
          throw new IllegalStateException("ratis-hip: leaseBatch failed", e);
        }
        leaseBits = bits;
      }
    }
  }

  @Override
  public void close() throws IOException {
    running = false;
    LockSupport.unpark(pump);
    try {
      pump.join();
    } catch (InterruptedException e) {
      Thread.currentThread().interrupt();
    }
    hip.close();
  }

  /** The width of the device tier a membership word puts a division in (groups.cpp needed_width). */
  static int tierWidth(int conf) {
    final int mask = (conf & 0x3FFF) | ((conf >>> RatisHip.CONF_OLD_SHIFT) & 0x3FFF);
    return Math.max(2, (32 - Integer.numberOfLeadingZeros(mask) + 1) & ~1);
  }

  /**
   * One leader division's handle: its node slot and the numbering of its followers.
   *
   * Deltas and the control calls (start / reconf / stop) go through one ordered stream under
   * deltaLock: buffered deltas are pushed before a control call reaches the library, so a delta
   * never lands on a slot after it was stopped (or recycled), and a delta is only emitted for a
   * column the division's current tier has (rh_push_deltas rejects the others).  Dropping a
   * follower column outside the tier loses nothing the commit rule reads: that slot is not in the
   * membership word, and the widening reconf starts it at -1, as a new FollowerInfoImpl does
   * (FollowerInfoImpl.java:42-43); the follower's next reply carries its current matchIndex.
   */
  public final class Division {
    private final int nodeSlot;
    private final RaftPeerId selfId;
    private final Callback callback;
    private final Map<RaftPeerId, Integer> followerSlot = new HashMap<>();   // peers with a FollowerInfo
    private boolean started;   // guarded by deltaLock
    private int width;         // follower columns of the device tier; guarded by deltaLock

    Division(int nodeSlot, RaftPeerId selfId, Callback callback) {
      this.nodeSlot = nodeSlot;
      this.selfId = selfId;
      this.callback = callback;
    }

    private void emit(int follower, int column, int op, long value) {
      synchronized (deltaLock) {
        if (!started || follower >= width) {
          return;
        }
        putDeltaLocked(nodeSlot, column, op, value);
      }
      LockSupport.unpark(pump);
    }

    /** addSenders (LeaderStateImpl.java:681-692): the peer gets a FollowerInfo and a slot. */
    public synchronized int addFollower(RaftPeerId peer) {
      final Integer k = followerSlot.get(peer);
      if (k != null) {
        return k;
      }
      for (int s = 0; s < RatisHip.MAX_FOLLOWERS; s++) {
        if (!followerSlot.containsValue(s)) {
          followerSlot.put(peer, s);
          // a new FollowerInfoImpl starts at matchIndex = commitIndex = -1 (FollowerInfoImpl.java:42-43);
          // a recycled slot still holds its previous peer's indices
          emit(s, RatisHip.colMatch(s), RatisHip.OP_SET, -1L);
          emit(s, RatisHip.colFollowerCommit(s), RatisHip.OP_SET, -1L);
          emit(s, RatisHip.colTs(s), RatisHip.OP_SET, System.nanoTime());  // lastRpcTime (FollowerInfoImpl.java:58)
          return s;
        }
      }
      throw new IllegalStateException("ratis-hip: more than " + RatisHip.MAX_FOLLOWERS + " followers");
    }

    /** stopAndRemoveSenders (LeaderStateImpl.java:694-702): the slot becomes reusable. */
    public synchronized void removeFollower(RaftPeerId peer) {
      followerSlot.remove(peer);
    }

    /**
     * The membership word of conf / oldConf (RaftConfigurationImpl.java:142-195) restricted to
     * peers with a FollowerInfo, as getFollowerInfos filters them (LeaderStateImpl.java:291-293).
     */
    public synchronized int confWord(Collection<RaftPeerId> conf, Collection<RaftPeerId> oldConf) {
      int n = 0;
      int o = 0;
      for (RaftPeerId p : conf) {
        final Integer k = followerSlot.get(p);
        if (k != null) {
          n |= 1 << k;
        }
      }
      if (oldConf != null) {
        for (RaftPeerId p : oldConf) {
          final Integer k = followerSlot.get(p);
          if (k != null) {
            o |= 1 << k;
          }
        }
      }
      return RatisHip.confWord(n, conf.contains(selfId), oldConf != null, o,
          oldConf != null && oldConf.contains(selfId), true);
    }

    /** Leader start: every FollowerInfo new (-1); StartupLogEntry index = termStart (LeaderStateImpl.java:296-301). */
    public void start(int conf, long flushIndex, long commitIndex, long termStart) throws IOException {
      synchronized (deltaLock) {
        drainDeltas();
        hip.start(nodeSlot, conf, flushIndex, commitIndex, termStart);
        width = tierWidth(conf);
        started = true;
      }
    }

    /**
     * Conf change (applyOldNewConf / replicateNewConf, LeaderStateImpl.java:624-633, 1064-1074):
     * the membership word changes and every slot keeps its follower's indices (a new peer's slot
     * was reset to -1 when addFollower gave it out; a slot the wider tier adds starts at -1).
     */
    public void reconf(int conf) throws IOException {
      final byte[] src = new byte[RatisHip.MAX_FOLLOWERS];
      for (int k = 0; k < src.length; k++) {
        src[k] = (byte) k;
      }
      synchronized (deltaLock) {
        if (!started) {
          return;
        }
        drainDeltas();
        hip.reconf(nodeSlot, conf, src);
        width = tierWidth(conf);
      }
    }

    /** Step-down (LeaderStateImpl.stop, LeaderStateImpl.java:470-490): the node slot is released. */
    public void stop() throws IOException {
      synchronized (deltaLock) {
        if (!started) {
          return;
        }
        drainDeltas();
        started = false;
        hip.stop(nodeSlot);
      }
      release(this);
    }

    // ---- producers (called where the reference updates FollowerInfo / the flush index) -------
    /** FollowerInfo.updateMatchIndex (FollowerInfoImpl.java:93-95), after the RPC reply. */
    public void matchIndex(int followerSlot, long value) {
      emit(followerSlot, RatisHip.colMatch(followerSlot), RatisHip.OP_MAX, value);
    }

    /** FollowerInfo.setSnapshotIndex (FollowerInfoImpl.java:147-151): matchIndex set as is. */
    public void snapshotIndex(int followerSlot, long value) {
      emit(followerSlot, RatisHip.colMatch(followerSlot), RatisHip.OP_SET, value);
    }

    /** FollowerInfo.updateCommitIndex (FollowerInfoImpl.java:103-105). */
    public void followerCommitIndex(int followerSlot, long value) {
      emit(followerSlot, RatisHip.colFollowerCommit(followerSlot), RatisHip.OP_MAX, value);
    }

    /** The leader's flush-index advance (SegmentedRaftLogWorker.java:419-431). */
    public void flushIndex(long value) {
      emit(-1, RatisHip.COL_FLUSH, RatisHip.OP_MAX, value);
    }

    /** A commit index raised outside updateCommit (RaftLogBase.updateSnapshotIndex, :155-166). */
    public void committedIndex(long value) {
      emit(-1, RatisHip.COL_COMMITTED, RatisHip.OP_MAX, value);
    }

    // ---- leader lease (LeaderStateImpl.hasLease, LeaderLease) --------------------------------
    /** The division's LeaderLease (lease = now, enabled per config) with every follower stamped now. */
    public void leaseStart(long nowNanos, boolean enabled) throws IOException {
      synchronized (deltaLock) {
        if (!started) {
          return;
        }
        drainDeltas();
        hip.leaseStart(nodeSlot, nowNanos, enabled);
      }
    }

    /** FollowerInfo.updateLastRespondedAppendEntriesSendTime (FollowerInfoImpl.java:241-243). */
    public void lastResponded(int followerSlot, long sendTimeNanos) {
      emit(followerSlot, RatisHip.colTs(followerSlot), RatisHip.OP_SET, sendTimeNanos);
    }

    /** LeaderLease.getAndSetEnabled (LeaderStateImpl.java:478, 744, 1042, 1226). */
    public void leaseEnabled(boolean enabled) {
      emit(-1, RatisHip.COL_LEASE_ON, RatisHip.OP_SET, enabled ? 1L : 0L);
    }

    /** enabled && (singleton || the lease, extended if it could be, is valid) at the last tick. */
    public boolean hasLease() {
      final long[] bits = leaseBits;
      return bits != null && ((bits[nodeSlot >>> 6] >>> (nodeSlot & 63)) & 1L) != 0;
    }
  }
}
