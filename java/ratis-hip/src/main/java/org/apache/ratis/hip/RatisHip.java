/*
 * ratis-hip: JNI binding of libratis_hip (include/ratis_hip.h in the ratis_amd repository), the
 * MI355X leader-bookkeeping engine.  One RatisHip per RaftServerProxy wraps an rh_node: one
 * resident group table per GPU of the device mask, RaftGroups placed by
 * floorMod(RaftGroupId.hashCode(), #GPUs) (RaftId.java:119-122).
 *
 * Java 8 compatible (the reference's CI baseline, .github/workflows/ci.yaml:51).  Not compiled in
 * the ratis_amd repository (its image has no JDK); the native half is java/ratis-hip/src/main/
 * native/ratis_hip_jni.c, which the repository's tests compile against the C ABI.
 *
 * Error mapping (ratis_hip.h): RH_E_INVAL / RH_E_RANGE -> IllegalArgumentException (as the
 * reference throws for bad arguments, e.g. LeaderStateImpl.java:396-399), every other negative
 * status -> IOException; a frame whose checksum does not verify -> ChecksumException at its offset
 * (SegmentedRaftLogReader.java:330-336) in the callers.  Array and buffer sizes are checked here
 * (and again in the native half) before any native call reads or writes them.
 */
package org.apache.ratis.hip;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

public final class RatisHip implements AutoCloseable {
  static {
    System.loadLibrary("ratis_hip_jni");   // links libratis_hip.so
  }

  // ---- membership word (ratis_hip.h, RH_CONF_*) ---------------------------------------------
  public static final int MAX_FOLLOWERS = 14;
  public static final int CONF_SELF = 1 << 14;
  public static final int CONF_TRANSITIONAL = 1 << 15;
  public static final int CONF_OLD_SHIFT = 16;
  public static final int CONF_SELF_OLD = 1 << 30;
  public static final int CONF_ACTIVE = 1 << 31;

  /** rh_conf_pack: bit k of newMask / oldMask = follower slot k is a voter of conf / oldConf. */
  public static int confWord(int newMask, boolean includeSelf, boolean transitional, int oldMask,
      boolean includeSelfOld, boolean active) {
    return (newMask & 0x3FFF) | (includeSelf ? CONF_SELF : 0) | (transitional ? CONF_TRANSITIONAL : 0)
        | ((oldMask & 0x3FFF) << CONF_OLD_SHIFT) | (includeSelfOld ? CONF_SELF_OLD : 0) | (active ? CONF_ACTIVE : 0);
  }

  // ---- deltas (rh_delta: u32 slot, u8 column, u8 op, u16 reserved, i64 value; 16 bytes) -----
  public static final int DELTA_BYTES = 16;
  public static int colMatch(int followerSlot) { return followerSlot; }
  public static int colFollowerCommit(int followerSlot) { return 16 + followerSlot; }
  public static final int COL_FLUSH = 32;
  public static final int COL_COMMITTED = 33;
  public static final int COL_LEASE = 36;     // LeaderLease.lease (nanos)
  public static final int COL_LEASE_ON = 37;  // LeaderLease.enabled (getAndSetEnabled)
  public static int colTs(int followerSlot) { return 48 + followerSlot; }  // lastRespondedAppendEntriesSendTime
  public static final int OP_MAX = 0;   // RaftLogIndex.updateToMax
  public static final int OP_SET = 1;   // RaftLogIndex.setUnconditionally (setSnapshotIndex)
  public static final int COMMIT_WATCH_ALL = 1;

  // ---- segment read verdicts (ratis_hip.h RH_SEG_*) -----------------------------------------
  public static final int SEG_END = 1;
  public static final int SEG_PARTIAL = 2;
  public static final int SEG_E_OVERSIZE = -1;
  public static final int SEG_E_CHECKSUM = -2;
  public static final int SEG_E_PADDING = -3;
  public static final int SEG_E_VARINT = -4;
  public static final int SEG_E_HEADER = -5;
  public static final int SEG_E_CAPACITY = -6;
  public static final int SEG_E_RANGE = -7;

  /** Writes one delta at the buffer's position (little-endian) and advances it. */
  public static void putDelta(ByteBuffer ring, int slotInShard, int column, int op, long value) {
    ring.putInt(slotInShard).put((byte) column).put((byte) op).putShort((short) 0).putLong(value);
  }

  private long node;        // rh_node*
  private final int shards;
  private final long capacityPerShard;

  public RatisHip(int deviceMask, long capacityPerShard, long gapThreshold) throws IOException {
    this.node = nodeCreate0(deviceMask, capacityPerShard, gapThreshold);
    this.shards = nodeShards0(node);
    this.capacityPerShard = capacityPerShard;
  }

  public int getShards() { return shards; }
  public long getCapacityPerShard() { return capacityPerShard; }

  /** Math.floorMod(UUID.hashCode(), shards) computed by the library (rh_shard_of). */
  public int shardOf(long uuidMsb, long uuidLsb) {
    return shardOf0(uuidMsb, uuidLsb, shards);
  }

  private void checkShard(int shard) {
    if (shard < 0 || shard >= shards) {
      throw new IllegalArgumentException("no shard " + shard + " (" + shards + " shards)");
    }
  }

  private static void checkLength(String what, int length, long needed) {
    if (length < needed) {
      throw new IllegalArgumentException(what + ".length = " + length + " < " + needed);
    }
  }

  // ---- division lifecycle (node slots = shard * capacityPerShard + slot in shard) ------------
  /** New LeaderStateImpl: every FollowerInfo new (index -1); termStart = StartupLogEntry index. */
  public void start(int nodeSlot, int conf, long flushIndex, long commitIndex, long termStart) throws IOException {
    groupStart0(node, nodeSlot, conf, flushIndex, commitIndex, termStart);
  }

  /** Conf change: src[k] = old follower slot kept by new slot k, or -1 for a new FollowerInfo. */
  public void reconf(int nodeSlot, int conf, byte[] src) throws IOException {
    if (src != null) {
      checkLength("src", src.length, MAX_FOLLOWERS);
    }
    groupReconf0(node, nodeSlot, conf, src);
  }

  public void stop(int nodeSlot) throws IOException {
    groupStop0(node, nodeSlot);
  }

  // ---- delta producers ---------------------------------------------------------------------
  /** Validated push of the n deltas at the start of a direct buffer (node slots); returns when the
   * buffer may be reused. */
  public void pushDeltas(ByteBuffer direct, int n) throws IOException {
    if (!direct.isDirect()) {
      throw new IllegalArgumentException("pushDeltas needs a direct buffer");
    }
    if (n < 0 || (long) n * DELTA_BYTES > direct.capacity()) {
      throw new IllegalArgumentException("pushDeltas: " + n + " deltas do not fit the buffer's "
          + direct.capacity() + " bytes");
    }
    pushDeltas0(node, direct, n);
  }

  /**
   * Zero-copy path of one shard: the next pinned staging slot as a little-endian direct buffer
   * (capacity RH_DELTA_SLOT deltas, slots relative to the shard) to fill with {@link #putDelta}.
   * Hand it back with {@link #submitDeltas}; one acquire/submit pair at a time per shard.
   */
  public ByteBuffer acquireDeltas(int shard) throws IOException {
    checkShard(shard);
    return acquire0(node, shard).order(ByteOrder.LITTLE_ENDIAN);
  }

  public void submitDeltas(int shard, int n) throws IOException {
    checkShard(shard);
    submit0(node, shard, n);
  }

  // ---- consumers ---------------------------------------------------------------------------
  /**
   * Batched LeaderStateImpl.updateCommit() over every shard's dirty divisions.  Fills
   * advSlot/advCommit with the node slots whose commit index advanced and the new value, and
   * (with COMMIT_WATCH_ALL) wallSlot/wallMin with the changed watch-ALL levels.  Returns
   * (long) nAdvanced << 32 | nWatchAll; counts beyond the arrays are truncated.
   */
  public long commitBatch(int[] advSlot, long[] advCommit, int[] wallSlot, long[] wallMin) throws IOException {
    checkLength("advCommit", advCommit.length, advSlot.length);
    if (wallSlot != null) {
      checkLength("wallMin", wallMin.length, wallSlot.length);
    }
    return commitBatch0(node, advSlot, advCommit, wallSlot, wallMin);
  }

  /** rh_commit_batch_async on one shard: the evaluation is in flight when this returns. */
  public long commitAsync(int shard, int flags) throws IOException {
    checkShard(shard);
    return commitAsync0(node, shard, flags);
  }

  /**
   * rh_tick_async on one shard: {@link #commitAsync} then {@link #watchAsync} in one call (one kernel
   * launch when both kinds' dirty divisions are listed).  Collect with {@link #commitWait} (the
   * returned ticket) and {@link #watchWait}.
   */
  public long tickAsync(int shard, int flags) throws IOException {
    checkShard(shard);
    return tickAsync0(node, shard, flags);
  }

  /**
   * rh_commit_batch_wait on one shard: the shard's events (slots WITHIN the shard) copied into the
   * caller's arrays, which must hold the shard capacity.  Returns nAdvanced << 32 | nWatchAll.
   */
  public long commitWait(int shard, long ticket, int[] advSlot, long[] advCommit, int[] wallSlot, long[] wallMin)
      throws IOException {
    checkShard(shard);
    checkLength("advSlot", advSlot.length, capacityPerShard);
    checkLength("advCommit", advCommit.length, capacityPerShard);
    checkLength("wallSlot", wallSlot.length, capacityPerShard);
    checkLength("wallMin", wallMin.length, capacityPerShard);
    return commitWait0(node, shard, ticket, advSlot, advCommit, wallSlot, wallMin);
  }

  /** Batched commitIndexChanged() of one shard: changed {min, majority, max} levels (slots within
   * the shard).  Every array must hold the shard capacity. */
  public int watchLevels(int shard, int[] slot, long[] min, long[] majority, long[] max, boolean[] valid)
      throws IOException {
    checkShard(shard);
    checkLength("slot", slot.length, capacityPerShard);
    checkLength("min", min.length, capacityPerShard);
    checkLength("majority", majority.length, capacityPerShard);
    checkLength("max", max.length, capacityPerShard);
    checkLength("valid", valid.length, capacityPerShard);
    return watchLevels0(node, shard, slot, min, majority, max, valid);
  }

  /** rh_watch_levels_async on one shard: commitIndexChanged() of its dirty divisions in flight
   *  (after the shard's commit evaluation, in stream order). */
  public void watchAsync(int shard) throws IOException {
    checkShard(shard);
    watchAsync0(node, shard);
  }

  /** rh_watch_levels_wait on one shard: the outstanding evaluation's changed levels, as
   *  {@link #watchLevels}.  Every array must hold the shard capacity. */
  public int watchWait(int shard, int[] slot, long[] min, long[] majority, long[] max, boolean[] valid)
      throws IOException {
    checkShard(shard);
    checkLength("slot", slot.length, capacityPerShard);
    checkLength("min", min.length, capacityPerShard);
    checkLength("majority", majority.length, capacityPerShard);
    checkLength("max", max.length, capacityPerShard);
    checkLength("valid", valid.length, capacityPerShard);
    return watchWait0(node, shard, slot, min, majority, max, valid);
  }

  /** Where every shard's result lists are assembled (rh_groups_set_event_sink): EVENTS_AUTO (the
   *  default), EVENTS_HOST_MAPPED or EVENTS_DEVICE.  Not while an evaluation is outstanding. */
  public void setEventSink(int sink) throws IOException {
    for (int s = 0; s < shards; s++) {
      setEventSink0(node, s, sink);
    }
  }

  public static final int EVENTS_HOST_MAPPED = 0;
  public static final int EVENTS_DEVICE = 1;
  /** The default: HBM lists for evaluations over every tile, pinned lists for dirty-row-list ones. */
  public static final int EVENTS_AUTO = 2;

  // ---- leader lease (LeaderStateImpl.hasLease, LeaderLease) ----------------------------------
  /** A new LeaderLease for the division (lease = now, enabled per config) with every follower slot
   * stamped now, as a new LeaderStateImpl creates them (LeaderLease.java:37-38, FollowerInfoImpl.java:58).
   * Later replies go in as COL_TS deltas (updateLastRespondedAppendEntriesSendTime). */
  public void leaseStart(int slot, long nowNanos, boolean enabled) throws IOException {  // node slot
    leaseStart0(node, slot, nowNanos, enabled);
  }

  /** hasLease() of every node slot at nowNanos (without isRunning()/isReady()); extended leases
   * stay in the table.  bits[s / 64] bit s % 64 = slot s; bits.length >= ceil(slots / 64). */
  public void leaseBatch(long nowNanos, long timeoutMs, long[] bits) throws IOException {
    checkLength("bits", bits.length, (shards * capacityPerShard + 63) / 64);
    leaseBatch0(node, nowNanos, timeoutMs, bits);
  }

  /** hasLease() of one shard's slots at nowNanos; bits.length >= ceil(capacityPerShard / 64). */
  public void leaseBatch(int shard, long nowNanos, long timeoutMs, long[] bits) throws IOException {
    checkShard(shard);
    checkLength("bits", bits.length, (capacityPerShard + 63) / 64);
    leaseBatchShard0(node, shard, nowNanos, timeoutMs, bits);
  }

  /** rh_lease_batch_async on one shard: its hasLease() pass at nowNanos in flight. */
  public void leaseAsync(int shard, long nowNanos, long timeoutMs) throws IOException {
    checkShard(shard);
    leaseAsync0(node, shard, nowNanos, timeoutMs);
  }

  /** rh_lease_batch_wait on one shard: the outstanding pass's bitmap; bits.length >=
   *  ceil(capacityPerShard / 64). */
  public void leaseWait(int shard, long[] bits) throws IOException {
    checkShard(shard);
    checkLength("bits", bits.length, (capacityPerShard + 63) / 64);
    leaseWait0(node, shard, bits);
  }

  // ---- checksums (SegmentedRaftLogReader.decodeEntry, batched over a segment) ---------------
  /**
   * PCIe-inclusive verification of the frames of one segment image held in a direct buffer (from
   * its position to its limit): every frame's PureJavaCrc32C (crcOut, optional) and the mismatch
   * bitmap (badBits, optional); returns the number of mismatches.
   */
  public long verifyFrames(int shard, ByteBuffer segment, long[] frameOff, int[] frameLen, int[] crcOut,
      long[] badBits) throws IOException {
    checkShard(shard);
    if (!segment.isDirect()) {
      throw new IllegalArgumentException("verifyFrames needs a direct buffer");
    }
    final int n = frameOff.length;
    checkLength("frameLen", frameLen.length, n);
    if (crcOut != null) {
      checkLength("crcOut", crcOut.length, n);
    }
    if (badBits != null) {
      checkLength("badBits", badBits.length, (n + 63) / 64);
    }
    return verifyHost0(node, shard, segment, segment.position(), segment.remaining(), frameOff, frameLen, n, crcOut,
        badBits);
  }

  @Override
  public void close() throws IOException {
    if (node != 0) {
      nodeDestroy0(node);
      node = 0;
    }
  }

  // ---- a bare context for the log read path (HipLogReader) -----------------------------------
  static native long ctxCreate0(int device) throws IOException;
  static native void ctxDestroy0(long ctx) throws IOException;
  /** rh_segments_read_host over image[0, imageLen) of a direct buffer; per segment s:
   * segInts[3s..3s+2] = status, n_ok, n_frames; segLongs[2s..2s+1] = stop, first_frame. */
  static native long readSegments0(long ctx, ByteBuffer image, long imageLen, long[] segOff, long[] segLen, int nSeg,
      int maxOp, int capPerSeg, long[] frameOff, int[] frameLen, int[] frameCrc, int[] segInts, long[] segLongs)
      throws IOException;

  /** rh_crc32c_stamp_host over buf[0, bufLen) of a direct buffer. */
  static native void stampHost0(long ctx, ByteBuffer buf, long bufLen, long[] off, int[] len, int n) throws IOException;
  /** rh_host_register / rh_host_unregister of a whole direct buffer. */
  static native void hostRegister0(long ctx, ByteBuffer buf) throws IOException;
  static native void hostUnregister0(long ctx, ByteBuffer buf) throws IOException;

  private static native long nodeCreate0(int deviceMask, long capacityPerShard, long gap) throws IOException;
  private static native void nodeDestroy0(long node) throws IOException;
  private static native int nodeShards0(long node);
  private static native int shardOf0(long msb, long lsb, int shards);
  private static native void groupStart0(long node, int slot, int conf, long flush, long commit, long termStart)
      throws IOException;
  private static native void groupReconf0(long node, int slot, int conf, byte[] src) throws IOException;
  private static native void groupStop0(long node, int slot) throws IOException;
  private static native void pushDeltas0(long node, ByteBuffer direct, int n) throws IOException;
  private static native ByteBuffer acquire0(long node, int shard) throws IOException;
  private static native void submit0(long node, int shard, int n) throws IOException;
  private static native long commitBatch0(long node, int[] advSlot, long[] advCommit, int[] wallSlot, long[] wallMin)
      throws IOException;
  private static native long commitAsync0(long node, int shard, int flags) throws IOException;
  private static native long tickAsync0(long node, int shard, int flags) throws IOException;
  private static native long commitWait0(long node, int shard, long ticket, int[] advSlot, long[] advCommit,
      int[] wallSlot, long[] wallMin) throws IOException;
  private static native int watchLevels0(long node, int shard, int[] slot, long[] min, long[] majority, long[] max,
      boolean[] valid) throws IOException;
  private static native void watchAsync0(long node, int shard) throws IOException;
  private static native int watchWait0(long node, int shard, int[] slot, long[] min, long[] majority, long[] max,
      boolean[] valid) throws IOException;
  private static native void setEventSink0(long node, int shard, int sink) throws IOException;
  private static native void leaseAsync0(long node, int shard, long nowNanos, long timeoutMs) throws IOException;
  private static native void leaseWait0(long node, int shard, long[] bits) throws IOException;
  private static native void leaseStart0(long node, int slot, long nowNanos, boolean enabled) throws IOException;
  private static native void leaseBatch0(long node, long nowNanos, long timeoutMs, long[] bits) throws IOException;
  private static native void leaseBatchShard0(long node, int shard, long nowNanos, long timeoutMs, long[] bits)
      throws IOException;
  private static native long verifyHost0(long node, int shard, ByteBuffer seg, long pos, long len, long[] off,
      int[] flen, int n, int[] crc, long[] bad) throws IOException;
}
