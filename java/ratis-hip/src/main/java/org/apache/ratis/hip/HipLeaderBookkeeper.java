/*
 * Server-level leader bookkeeping on the GPU: one instance per RaftServerProxy (RaftServerProxy.java:
 * 89-150 holds every division of a server) when raft.server.hip.commit.backend = hip.
 *
 * It replaces, for every leader division at once, what LeaderStateImpl does per division:
 *   - the FollowerInfoMap and the MinMajorityMax arithmetic (LeaderStateImpl.java:230-294, 904-984):
 *     follower slots k per division, the membership word of RaftConfigurationImpl's conf / oldConf
 *     restricted to peers with a FollowerInfo (LeaderStateImpl.java:291-293);
 *   - the per-division EventProcessor thread and its UPDATE_COMMIT queue (LeaderStateImpl.java:111-188,
 *     791-816): producers append 16-byte deltas to a buffer of their own thread (no lock shared
 *     between producers; a full buffer is pushed by its producer, the multi-producer rh_push_deltas);
 *     ONE pump thread pushes what is left each tick and runs the batched updateCommit over the dirty
 *     divisions;
 *   - RaftLogBase.updateCommitIndex's decision (RaftLogBase.java:121-142);
 *   - commitIndexChanged()'s watch levels (LeaderStateImpl.java:606-622) over the divisions whose
 *     follower commitIndex or leader commitIndex changed;
 *   - LeaderStateImpl.hasLease / LeaderLease.extend (LeaderStateImpl.java:1229-1249, LeaderLease.java).
 * The follow-up the reference runs after a decision -- getEntries, the real
 * ServerState.updateCommitIndex, StateMachineUpdater.notifyUpdater, the WatchRequests updates,
 * notifySenders -- stays in the division's LeaderStateImpl (Callback), for the divisions with an
 * event only.
 *
 * One pump tick: push the buffered deltas; put every shard's updateCommit evaluation, its
 * commitIndexChanged evaluation and (with a lease timeout) its hasLease pass in flight -- every GPU
 * busy before any wait; then per shard, wait and hand the advanced commits and changed watch-ALL
 * levels to the divisions, then commitIndexChanged's levels, then publish the lease bitmap; recycle
 * the slots released during the tick.  Nothing is allocated per tick: every result array is sized
 * once, per shard capacity, and reused shard after shard.
 *
 * FALLBACK.  A division the GPU table cannot hold leaves it for good and reverts to the reference's
 * own per-division path (updateCommit / commitIndexChanged / hasLease in LeaderStateImpl; the
 * FollowerInfos are kept by Java in both modes): a 15th follower slot (the table has 14 per
 * division; a joint change of two 8-peer confs reaches 15), a full shard at register, a control
 * call the library rejects (RH_E_RANGE / RH_E_INVAL) or fails, and -- for every division -- a pump
 * that died.  Division.isFallback() is what every seam checks; Callback.onFallback() lets the
 * division catch up in Java at once; getFallbackCount() / getFallbackCount(reason) count them
 * (SURVEY section 7: "fall back to the CPU path.  Count that fallback").
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
import java.util.Queue;
import java.util.UUID;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.ConcurrentLinkedQueue;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.atomic.AtomicBoolean;
import java.util.concurrent.atomic.AtomicLongArray;
import java.util.concurrent.atomic.AtomicReferenceArray;
import java.util.concurrent.locks.LockSupport;
import java.util.concurrent.locks.ReentrantReadWriteLock;

public final class HipLeaderBookkeeper implements AutoCloseable {
  /** What a division's LeaderStateImpl does with the GPU's decisions (run on the pump thread). */
  public interface Callback {
    /** updateCommit(majority, min) found a new commit index (LeaderStateImpl.java:1015-1024). */
    void onCommit(long newCommitIndex);
    /** updateCommit(majority, min)'s watchRequests.update(ALL, min), the level changed (LeaderStateImpl.java:1025). */
    void onWatchAll(long min);
    /** commitIndexChanged()'s levels changed (LeaderStateImpl.java:612-622): ALL_COMMITTED = min,
     *  MAJORITY_COMMITTED = majority, MAJORITY = max; the division then runs notifySenders(). */
    void onWatchLevels(long min, long majority, long max);
    /** The division left the GPU table (see FALLBACK above): from now on it runs the reference's
     *  per-division path; it should evaluate updateCommit / commitIndexChanged once now. */
    void onFallback();
  }

  /** Why a division runs the Java path. */
  public enum FallbackReason { SHARD_FULL, FOLLOWER_SLOTS, REJECTED, DEVICE_ERROR, PUMP_FAILED }

  private final RatisHip hip;
  private final int shards;
  private final int capacity;                        // divisions per shard
  private final Deque<Integer>[] freeSlots;
  private final Deque<Integer> pendingFree = new ArrayDeque<>();   // released during the current tick
  private final Map<Integer, Division> divisions = new ConcurrentHashMap<>();
  /** Deltas per producer thread: an appender thread (GrpcLogAppender / LogAppenderDefault, one per
   *  follower) or the log worker writes into its own buffer, so producers never contend with each
   *  other -- only, briefly, with the pump flushing that buffer. */
  private static final int BUFFER_DELTAS = 4096;
  private final Queue<DeltaBuffer> buffers = new ConcurrentLinkedQueue<>();
  private final ThreadLocal<DeltaBuffer> localBuffer = ThreadLocal.withInitial(this::newBuffer);
  private final AtomicBoolean wake = new AtomicBoolean();   // one unpark of the pump per tick at most
  private final Thread pump;
  private final long tickNanos;
  private volatile boolean running = true;
  private volatile Throwable failure;                // set when the pump died: no more results, no lease
  private volatile long leaseTimeoutMs = -1;  // LeaderLease.leaseTimeoutMs; -1: no lease batches
  private final AtomicLongArray fallbacks = new AtomicLongArray(FallbackReason.values().length);

  // ---- pump-thread result arrays: one shard's worth, reused for every shard and every tick -----
  private final int[] advSlot;
  private final long[] advCommit;
  private final int[] wallSlot;
  private final long[] wallMin;
  private final int[] wSlot;
  private final long[] wMin;
  private final long[] wMaj;
  private final long[] wMax;
  private final boolean[] wValid;
  private final long[] tickets;

  /**
   * The lease bitmap of one shard, published by the pump under a sequence number (odd while being
   * written; every field is read and written with volatile / ordered accesses, so a reader that
   * sees the same even number before and after its reads saw one consistent bitmap).  A bit
   * answers hasLease() only until validUntil: the batch was evaluated at evaluation time + margin
   * (a lease valid then is valid at every earlier moment: LeaderLease only moves forward), and
   * after validUntil the bitmap says nothing -- a stalled or dead pump turns every lease off
   * instead of freezing it (LeaderLease.java:60-62 checks at call time).
   */
  private static final class LeaseBits {
    final AtomicLongArray bits;
    volatile long seq;
    volatile long validUntil;   // System.nanoTime() bound of this bitmap
    volatile long batch;        // leaseBatchCount when it was evaluated

    LeaseBits(int words) {
      this.bits = new AtomicLongArray(words);
    }
  }

  private final LeaseBits[][] lease;       // [shard][2]: written alternately
  private final int[] leaseCurrent;        // [shard] which of the two is published (pump-owned)
  private final AtomicReferenceArray<LeaseBits> leasePublished;
  private final long[] leaseScratch;       // the native batch's output, copied into a LeaseBits
  private volatile long leaseBatchCount;   // batches started so far
  private final long leaseMarginNanos;

  @SuppressWarnings("unchecked")
  public HipLeaderBookkeeper(int deviceMask, long capacityPerShard, long gapThreshold, long tickMicros)
      throws IOException {
    if (capacityPerShard < 1 || capacityPerShard > Integer.MAX_VALUE - 8) {
      throw new IllegalArgumentException("capacityPerShard out of range: " + capacityPerShard);
    }
    this.hip = new RatisHip(deviceMask, capacityPerShard, gapThreshold);
    this.shards = hip.getShards();
    this.capacity = (int) capacityPerShard;
    this.freeSlots = new Deque[shards];
    for (int s = 0; s < shards; s++) {
      freeSlots[s] = new ArrayDeque<>();
      for (int i = capacity - 1; i >= 0; i--) {
        freeSlots[s].push(i);
      }
    }
    this.tickNanos = TimeUnit.MICROSECONDS.toNanos(tickMicros);
    // a bitmap stays meaningful for two ticks: long enough for the next one to replace it
    this.leaseMarginNanos = 2 * tickNanos;
    this.advSlot = new int[capacity];
    this.advCommit = new long[capacity];
    this.wallSlot = new int[capacity];
    this.wallMin = new long[capacity];
    this.wSlot = new int[capacity];
    this.wMin = new long[capacity];
    this.wMaj = new long[capacity];
    this.wMax = new long[capacity];
    this.wValid = new boolean[capacity];
    this.tickets = new long[shards];
    final int words = (capacity + 63) / 64;
    this.lease = new LeaseBits[shards][2];
    this.leaseCurrent = new int[shards];
    this.leasePublished = new AtomicReferenceArray<>(shards);
    this.leaseScratch = new long[words];
    for (int s = 0; s < shards; s++) {
      lease[s][0] = new LeaseBits(words);
      lease[s][1] = new LeaseBits(words);
      leasePublished.set(s, lease[s][0]);   // batch 0: answers no division (see hasLease)
    }
    this.pump = new Thread(this::pumpLoop, "ratis-hip-commit-pump");
    this.pump.setDaemon(true);
    this.pump.start();
  }

  /** rpc.timeout.min x read.leader.lease.timeout.ratio (LeaderLease.java:45-48); the pump then
   * evaluates hasLease() for every division each tick. */
  public void setLeaseTimeoutMs(long ms) {
    this.leaseTimeoutMs = ms;
  }

  /** Why the pump stopped, or null while it runs. */
  public Throwable getFailure() {
    return failure;
  }

  /** Divisions that fell back to the Java path so far (every reason). */
  public long getFallbackCount() {
    long n = 0;
    for (int i = 0; i < fallbacks.length(); i++) {
      n += fallbacks.get(i);
    }
    return n;
  }

  public long getFallbackCount(FallbackReason reason) {
    return fallbacks.get(reason.ordinal());
  }

  /**
   * A new leader division (new LeaderStateImpl, LeaderStateImpl.java:365-430).  Never fails: a
   * division the GPU cannot take (its shard is full, or the pump has failed) is returned in
   * fallback, and the caller runs the reference's path for it.
   */
  public synchronized Division register(RaftGroupId groupId, RaftPeerId selfId, Callback callback) {
    if (failure != null) {
      return fallenBack(selfId, callback, FallbackReason.PUMP_FAILED);
    }
    final UUID u = groupId.getUuid();
    final int shard = hip.shardOf(u.getMostSignificantBits(), u.getLeastSignificantBits());
    final Integer slot = freeSlots[shard].poll();
    if (slot == null) {
      return fallenBack(selfId, callback, FallbackReason.SHARD_FULL);
    }
    final int nodeSlot = shard * capacity + slot;
    final Division d = new Division(nodeSlot, selfId, callback);
    divisions.put(nodeSlot, d);
    return d;
  }

  /** A division that never enters the table (no slot): the Java path from the start. */
  private Division fallenBack(RaftPeerId selfId, Callback callback, FallbackReason reason) {
    final Division d = new Division(-1, selfId, callback);
    d.fallback = true;
    fallbacks.incrementAndGet(reason.ordinal());
    return d;
  }

  /**
   * The division is gone: no event reaches it from now on (it leaves the map), and its slot waits
   * for the end of the current pump tick before it can be handed out again -- an evaluation that
   * was in flight when the division stopped can only deliver to an empty map entry, never to a
   * new division that took the slot over.
   */
  synchronized void release(Division d) {
    divisions.remove(d.nodeSlot);
    pendingFree.add(d.nodeSlot);
  }

  private synchronized void recycleSlots() {
    for (Integer s; (s = pendingFree.poll()) != null; ) {
      freeSlots[s / capacity].push(s % capacity);
    }
  }

  /**
   * One producer thread's deltas, in its call order.  Its monitor is taken by that producer (append,
   * and push when full) and by whoever flushes every buffer (the pump each tick, a control call
   * before it reaches the library): a buffer is pushed whole under its monitor, so one thread's
   * deltas reach the library in order.  Uncontended in the common case.
   */
  private final class DeltaBuffer {
    private final ByteBuffer bb =
        ByteBuffer.allocateDirect(RatisHip.DELTA_BYTES * BUFFER_DELTAS).order(ByteOrder.LITTLE_ENDIAN);

    synchronized void put(int nodeSlot, int column, int op, long value) {
      if (bb.remaining() < RatisHip.DELTA_BYTES) {
        flushLocked();
      }
      RatisHip.putDelta(bb, nodeSlot, column, op, value);
    }

    synchronized void flush() {
      flushLocked();
    }

    private void flushLocked() {
      final int n = bb.position() / RatisHip.DELTA_BYTES;
      if (n == 0) {
        return;
      }
      try {
        hip.pushDeltas(bb, n);   // multi-producer: other buffers push concurrently
      } catch (IOException e) {
        throw new IllegalStateException("ratis-hip: pushDeltas failed", e);
      }
      bb.clear();
    }
  }

  private DeltaBuffer newBuffer() {
    final DeltaBuffer b = new DeltaBuffer();
    buffers.add(b);
    return b;
  }

  /** Pushes every producer's buffered deltas (the pump each tick; a control call before it runs). */
  private void flushAllDeltas() {
    for (DeltaBuffer b : buffers) {
      b.flush();
    }
  }

  private void pumpLoop() {
    try {
      while (running) {
        LockSupport.parkNanos(tickNanos);
        wake.set(false);   // deltas emitted from here on may unpark the pump once more
        tick();
      }
    } catch (Throwable t) {
      failure = t;   // results stop; hasLease() turns false at once (see Division.hasLease)
      // every division reverts to the reference's per-division path
      for (Division d : divisions.values()) {
        d.fallBack(FallbackReason.PUMP_FAILED);
      }
    }
  }

  /** One pump tick (see the class comment). */
  void tick() throws IOException {
    flushAllDeltas();
    final long timeout = leaseTimeoutMs;
    final long batch = timeout >= 0 ? ++leaseBatchCount : 0;
    final long now = System.nanoTime();
    // every shard's updateCommit(), then commitIndexChanged() (one call: the commits the first stores
    // are the second's input; one launch when both kinds' dirty divisions are listed) and hasLease():
    // all shards in flight before any wait
    for (int s = 0; s < shards; s++) {
      tickets[s] = hip.tickAsync(s, RatisHip.COMMIT_WATCH_ALL);
      if (timeout >= 0) {
        hip.leaseAsync(s, now + leaseMarginNanos, timeout);
      }
    }
    for (int s = 0; s < shards; s++) {
      final long counts = hip.commitWait(s, tickets[s], advSlot, advCommit, wallSlot, wallMin);
      final int base = s * capacity;
      final int nAdv = (int) Math.min(counts >>> 32, capacity);
      for (int i = 0; i < nAdv; i++) {
        final Division d = divisions.get(base + advSlot[i]);
        if (d != null) {
          d.callback.onCommit(advCommit[i]);
        }
      }
      final int nWall = (int) Math.min(counts & 0xFFFFFFFFL, capacity);
      for (int i = 0; i < nWall; i++) {
        final Division d = divisions.get(base + wallSlot[i]);
        if (d != null) {
          d.callback.onWatchAll(wallMin[i]);
        }
      }
      // commitIndexChanged() of the divisions whose follower / leader commitIndex changed
      final int n = Math.min(hip.watchWait(s, wSlot, wMin, wMaj, wMax, wValid), capacity);
      for (int i = 0; i < n; i++) {
        if (!wValid[i]) {
          continue;   // getMajorityMin was Optional.empty(): no watch update (LeaderStateImpl.java:613)
        }
        final Division d = divisions.get(base + wSlot[i]);
        if (d != null) {
          d.callback.onWatchLevels(wMin[i], wMaj[i], wMax[i]);
        }
      }
      if (timeout >= 0) {  // LeaderStateImpl.hasLease for every division: extend + isValid
        hip.leaseWait(s, leaseScratch);
        final int next = leaseCurrent[s] ^ 1;
        final LeaseBits lb = lease[s][next];
        lb.seq = lb.seq + 1;                        // odd: being written (only the pump writes)
        for (int w = 0; w < leaseScratch.length; w++) {
          lb.bits.lazySet(w, leaseScratch[w]);
        }
        lb.validUntil = now + leaseMarginNanos;
        lb.batch = batch;
        lb.seq = lb.seq + 1;
        leaseCurrent[s] = next;
        leasePublished.set(s, lb);
      }
    }
    recycleSlots();
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
   * Deltas and the control calls (start / reconf / stop) are ordered per division by its
   * read-write lock: producers emit under the READ lock (any number at once, each into its own
   * thread's buffer), a control call holds the WRITE lock while it pushes every buffer and then
   * calls the library -- so a delta emitted before the call reaches the library before it, none is
   * emitted during it, and a delta never lands on a slot after it was stopped (or recycled).  A
   * delta is only emitted for a column the division's current tier has (rh_push_deltas rejects the
   * others).  Dropping a follower column outside the tier loses nothing the commit rule reads: that
   * slot is not in the membership word, and the widening reconf starts it at -1, as a new
   * FollowerInfoImpl does (FollowerInfoImpl.java:42-43); the follower's next reply carries its
   * current matchIndex.
   */
  public final class Division {
    private final int nodeSlot;   // -1: never had one (fell back at register)
    private final RaftPeerId selfId;
    private final Callback callback;
    private final Map<RaftPeerId, Integer> followerSlot = new HashMap<>();   // peers with a FollowerInfo
    private final ReentrantReadWriteLock order = new ReentrantReadWriteLock();
    private boolean started;   // guarded by `order` (written under the write lock)
    private int width;         // follower columns of the device tier; guarded by `order`
    private volatile boolean fallback;   // the reference's per-division path from now on
    private volatile long leaseArmedAfter = Long.MAX_VALUE;   // lease batches up to this one predate leaseStart

    Division(int nodeSlot, RaftPeerId selfId, Callback callback) {
      this.nodeSlot = nodeSlot;
      this.selfId = selfId;
      this.callback = callback;
    }

    /** True once the division runs the reference's own path (every seam checks this). */
    public boolean isFallback() {
      return fallback;
    }

    /**
     * Leaves the GPU table for good (see FALLBACK in the class comment): the slot is stopped and
     * released, later deltas are dropped, and the division is told to evaluate in Java now.
     * Idempotent; never throws (a device error while stopping is moot: nothing reads the slot).
     */
    void fallBack(FallbackReason reason) {
      boolean release = false;
      order.writeLock().lock();
      try {
        if (fallback) {
          return;
        }
        fallback = true;
        leaseArmedAfter = Long.MAX_VALUE;
        if (nodeSlot >= 0) {
          release = true;
          if (started) {
            started = false;
            try {
              flushAllDeltas();
              hip.stop(nodeSlot);
            } catch (IOException | RuntimeException ignored) {
              // the slot is released below and never evaluated for this division again
            }
          }
        }
      } finally {
        order.writeLock().unlock();
      }
      fallbacks.incrementAndGet(reason.ordinal());
      if (release) {
        release(this);
      }
      callback.onFallback();
    }

    private void emit(int follower, int column, int op, long value) {
      order.readLock().lock();
      try {
        if (!started || follower >= width) {
          return;
        }
        localBuffer.get().put(nodeSlot, column, op, value);
      } finally {
        order.readLock().unlock();
      }
      if (!wake.get() && wake.compareAndSet(false, true)) {
        LockSupport.unpark(pump);   // the first delta since the pump's last wake-up only
      }
    }

    /**
     * addSenders (LeaderStateImpl.java:681-692): the peer gets a FollowerInfo and a slot.  Returns
     * the slot, or -1 once the division is in fallback -- which a 15th follower puts it in.
     */
    public synchronized int addFollower(RaftPeerId peer) {
      if (fallback) {
        return -1;
      }
      final Integer k = followerSlot.get(peer);
      if (k != null) {
        return k;
      }
      for (int s = 0; s < RatisHip.MAX_FOLLOWERS; s++) {
        if (!followerSlot.containsValue(s)) {
          followerSlot.put(peer, s);
          resetFollowerSlot(s);
          return s;
        }
      }
      fallBack(FallbackReason.FOLLOWER_SLOTS);   // more than 14 followers: the Java path holds any number
      return -1;
    }

    /**
     * A new FollowerInfoImpl starts at matchIndex = commitIndex = -1 (FollowerInfoImpl.java:42-43)
     * and lastRpcTime = now (:58).  A recycled slot still holds its previous peer's values, and that
     * peer's last deltas may still sit in any producer thread's buffer -- buffers are pushed in
     * registration order, so a reset SET buffered by this thread could reach the library before a
     * stale MAX buffered by another, and the new follower would inherit the old matchIndex.  So,
     * under the write lock (no delta is emitted meanwhile): every buffer is pushed first, then the
     * three SETs go straight to the library, after every delta of the previous occupant.
     */
    private void resetFollowerSlot(int s) {
      order.writeLock().lock();
      try {
        if (!started || s >= width) {
          return;   // not in the tier: a widening reconf starts the column at -1
        }
        flushAllDeltas();
        final ByteBuffer bb =
            ByteBuffer.allocateDirect(3 * RatisHip.DELTA_BYTES).order(ByteOrder.LITTLE_ENDIAN);
        RatisHip.putDelta(bb, nodeSlot, RatisHip.colMatch(s), RatisHip.OP_SET, -1L);
        RatisHip.putDelta(bb, nodeSlot, RatisHip.colFollowerCommit(s), RatisHip.OP_SET, -1L);
        RatisHip.putDelta(bb, nodeSlot, RatisHip.colTs(s), RatisHip.OP_SET, System.nanoTime());
        hip.pushDeltas(bb, 3);
      } catch (IOException e) {
        throw new IllegalStateException("ratis-hip: pushDeltas failed", e);
      } finally {
        order.writeLock().unlock();
      }
    }

    /**
     * stopAndRemoveSenders (LeaderStateImpl.java:694-702): the slot becomes reusable.  The peer's
     * buffered deltas are pushed now, under the write lock, so none of them can follow the reset
     * of the slot's next occupant.
     */
    public synchronized void removeFollower(RaftPeerId peer) {
      followerSlot.remove(peer);
      order.writeLock().lock();
      try {
        if (started) {
          flushAllDeltas();
        }
      } finally {
        order.writeLock().unlock();
      }
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

    /**
     * Leader start: every FollowerInfo new (-1); StartupLogEntry index = termStart
     * (LeaderStateImpl.java:296-301).  A start the library rejects or fails puts the division in
     * fallback instead of failing the leader.
     */
    public void start(int conf, long flushIndex, long commitIndex, long termStart) {
      FallbackReason why = null;
      order.writeLock().lock();
      try {
        if (fallback) {
          return;
        }
        try {
          flushAllDeltas();
          hip.start(nodeSlot, conf, flushIndex, commitIndex, termStart);
          width = tierWidth(conf);
          started = true;
        } catch (IllegalArgumentException e) {
          why = FallbackReason.REJECTED;
        } catch (IOException | RuntimeException e) {
          why = FallbackReason.DEVICE_ERROR;
        }
      } finally {
        order.writeLock().unlock();
      }
      if (why != null) {
        fallBack(why);
      }
    }

    /**
     * Conf change (applyOldNewConf / replicateNewConf, LeaderStateImpl.java:624-633, 1064-1074):
     * the membership word changes and every slot keeps its follower's indices (a new peer's slot
     * was reset to -1 when addFollower gave it out; a slot the wider tier adds starts at -1).  A
     * reconf the library rejects (RH_E_RANGE: no row in the wider tier) or fails puts the division
     * in fallback.
     */
    public void reconf(int conf) {
      final byte[] src = new byte[RatisHip.MAX_FOLLOWERS];
      for (int k = 0; k < src.length; k++) {
        src[k] = (byte) k;
      }
      FallbackReason why = null;
      order.writeLock().lock();
      try {
        if (!started || fallback) {
          return;
        }
        try {
          flushAllDeltas();
          hip.reconf(nodeSlot, conf, src);
          width = tierWidth(conf);
        } catch (IllegalArgumentException e) {
          why = FallbackReason.REJECTED;
        } catch (IOException | RuntimeException e) {
          why = FallbackReason.DEVICE_ERROR;
        }
      } finally {
        order.writeLock().unlock();
      }
      if (why != null) {
        fallBack(why);
      }
    }

    /** Step-down (LeaderStateImpl.stop, LeaderStateImpl.java:470-490): the node slot is released. */
    public void stop() throws IOException {
      order.writeLock().lock();
      try {
        if (!started) {
          return;
        }
        flushAllDeltas();
        started = false;
        leaseArmedAfter = Long.MAX_VALUE;
        hip.stop(nodeSlot);
      } finally {
        order.writeLock().unlock();
      }
      release(this);
    }

    // ---- producers (called where the reference updates FollowerInfo / the flush index) -------
    // Each is a no-op for a follower without a slot (-1) and once the division is in fallback.
    /** FollowerInfo.updateMatchIndex (FollowerInfoImpl.java:93-95), after the RPC reply. */
    public void matchIndex(int followerSlot, long value) {
      if (followerSlot >= 0) {
        emit(followerSlot, RatisHip.colMatch(followerSlot), RatisHip.OP_MAX, value);
      }
    }

    /** FollowerInfo.setSnapshotIndex (FollowerInfoImpl.java:147-151): matchIndex set as is. */
    public void snapshotIndex(int followerSlot, long value) {
      if (followerSlot >= 0) {
        emit(followerSlot, RatisHip.colMatch(followerSlot), RatisHip.OP_SET, value);
      }
    }

    /** FollowerInfo.updateCommitIndex (FollowerInfoImpl.java:103-105): the pump's next watchLevels
     *  reports the division if its commitIndexChanged() levels moved. */
    public void followerCommitIndex(int followerSlot, long value) {
      if (followerSlot >= 0) {
        emit(followerSlot, RatisHip.colFollowerCommit(followerSlot), RatisHip.OP_MAX, value);
      }
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
    public void leaseStart(long nowNanos, boolean enabled) {
      FallbackReason why = null;
      order.writeLock().lock();
      try {
        if (!started || fallback) {
          return;
        }
        try {
          flushAllDeltas();
          // batches already started may predate this lease: only a later one answers hasLease()
          leaseArmedAfter = leaseBatchCount;
          hip.leaseStart(nodeSlot, nowNanos, enabled);
        } catch (IllegalArgumentException e) {
          why = FallbackReason.REJECTED;
        } catch (IOException | RuntimeException e) {
          why = FallbackReason.DEVICE_ERROR;
        }
      } finally {
        order.writeLock().unlock();
      }
      if (why != null) {
        fallBack(why);
      }
    }

    /** FollowerInfo.updateLastRespondedAppendEntriesSendTime (FollowerInfoImpl.java:241-243). */
    public void lastResponded(int followerSlot, long sendTimeNanos) {
      if (followerSlot >= 0) {
        emit(followerSlot, RatisHip.colTs(followerSlot), RatisHip.OP_SET, sendTimeNanos);
      }
    }

    /** LeaderLease.getAndSetEnabled (LeaderStateImpl.java:478, 744, 1042, 1226). */
    public void leaseEnabled(boolean enabled) {
      emit(-1, RatisHip.COL_LEASE_ON, RatisHip.OP_SET, enabled ? 1L : 0L);
    }

    /**
     * enabled && (singleton || the lease, extended if it could be, is valid), as of the latest
     * lease batch -- evaluated for a moment at least as late as now, so a true answer holds now.
     * False when no such batch exists: the pump has not run one since leaseStart, it has stalled
     * past the bitmap's validity, or it has failed; and in fallback (the caller then asks the
     * reference's LeaderLease instead).
     */
    public boolean hasLease() {
      if (failure != null || fallback || nodeSlot < 0) {
        return false;
      }
      final int shard = nodeSlot / capacity;
      final int slot = nodeSlot % capacity;
      for (;;) {
        final LeaseBits lb = leasePublished.get(shard);
        final long seq = lb.seq;
        if ((seq & 1) != 0) {
          continue;   // being rewritten: the pump published the other one meanwhile
        }
        final boolean bit = ((lb.bits.get(slot >>> 6) >>> (slot & 63)) & 1L) != 0;
        final long validUntil = lb.validUntil;
        final long batch = lb.batch;
        if (lb.seq != seq) {
          continue;
        }
        return bit && batch > leaseArmedAfter && System.nanoTime() - validUntil <= 0;
      }
    }
  }
}
