/*
 * The checksum backend of the segmented log's bulk load (raft.server.hip.checksum.backend = hip):
 * SegmentedRaftLog.loadLogSegments (SegmentedRaftLog.java:248-276) reads many segment files at
 * server start; each is walked and checksummed by SegmentedRaftLogReader.decodeEntry
 * (SegmentedRaftLogReader.java:291-341: PureJavaCrc32C over every entry) through
 * LogSegment.readSegmentFile (LogSegment.java:166-196).  Here the files' bytes go to the GPU in one
 * rh_segments_read_host call (framing walk + CRC32C of every frame + the reader's verdict per file)
 * and come back as, per file, the verified frame table and how the reader would have ended; the
 * caller (LogSegment, through the seams patch) parses the accepted entries from the same image and
 * raises what the reader would have raised -- ChecksumException at the failing entry's offset,
 * IOException / CorruptedFileException for the framing errors -- under its CorruptionPolicy.
 *
 * No LogEntryProto parsing here (ratis-hip does not depend on ratis-proto); a Segment exposes the
 * bytes of each accepted entry.  Files are read into one direct buffer per batch; a file the GPU
 * could not walk (more frames than the per-file slot count, RH_SEG_E_CAPACITY) reports
 * {@link Segment#usable()} = false and is left to the Java reader.
 */
package org.apache.ratis.hip;

import java.io.File;
import java.io.IOException;
import java.io.RandomAccessFile;
import java.nio.ByteBuffer;
import java.nio.channels.FileChannel;
import java.util.List;

public final class HipLogReader implements AutoCloseable {
  private static HipLogReader instance;

  /** The process-wide reader on the lowest GPU of the mask (one context; calls are serialised). */
  public static synchronized HipLogReader get(int deviceMask) throws IOException {
    if (instance == null) {
      if (deviceMask == 0) {
        throw new IllegalArgumentException("empty device mask");
      }
      instance = new HipLogReader(Integer.numberOfTrailingZeros(deviceMask));
    }
    return instance;
  }

  private long ctx;   // rh_ctx*

  private HipLogReader(int device) throws IOException {
    this.ctx = RatisHip.ctxCreate0(device);
  }

  /** One file's outcome. */
  public static final class Segment {
    private final Batch batch;
    private final int index;

    Segment(Batch batch, int index) {
      this.batch = batch;
      this.index = index;
    }

    /** RatisHip.SEG_* verdict of the reader over this file. */
    public int status() {
      return batch.segInts[3 * index];
    }

    /** False when the GPU walk could not cover the file: read it with the Java reader. */
    public boolean usable() {
      final int s = status();
      return s != RatisHip.SEG_E_CAPACITY && s != RatisHip.SEG_E_RANGE;
    }

    /** Entries the reader returns before it stops. */
    public int entries() {
      return batch.segInts[3 * index + 1];
    }

    /** Offset in the file where the reader stopped: the failing entry, or the end. */
    public long stopOffset() {
      return batch.segLongs[2 * index];
    }

    private int frame(int k) {
      if (k < 0 || k >= entries()) {
        throw new IndexOutOfBoundsException("entry " + k + " of " + entries());
      }
      return (int) batch.segLongs[2 * index + 1] + k;
    }

    /** Offset of entry k's frame (its varint) in the file. */
    public long frameOffset(int k) {
      return batch.frameOff[frame(k)] - batch.fileStart[index];
    }

    /** The LogEntryProto bytes of entry k (between its varint and its checksum), as a read-only view. */
    public ByteBuffer entryBytes(int k) {
      final int f = frame(k);
      final long off = batch.frameOff[f];
      final int len = batch.frameLen[f];
      int v = 1;   // varint32 length prefix: 1..5 bytes, 7 bits each
      while ((batch.image.get((int) off + v - 1) & 0x80) != 0) {
        v++;
      }
      final ByteBuffer b = batch.image.duplicate();
      b.limit((int) (off + len - 4)).position((int) (off + v));
      return b.slice().asReadOnlyBuffer();
    }

    /** PureJavaCrc32C.getValue() of entry k's frame, as computed on the GPU. */
    public int checksum(int k) {
      return batch.frameCrc[frame(k)];
    }
  }

  /** The files of one rh_segments_read_host call. */
  public static final class Batch {
    final ByteBuffer image;
    final long[] fileStart;
    final long[] frameOff;
    final int[] frameLen;
    final int[] frameCrc;
    final int[] segInts;
    final long[] segLongs;

    Batch(ByteBuffer image, long[] fileStart, long[] frameOff, int[] frameLen, int[] frameCrc, int[] segInts,
        long[] segLongs) {
      this.image = image;
      this.fileStart = fileStart;
      this.frameOff = frameOff;
      this.frameLen = frameLen;
      this.frameCrc = frameCrc;
      this.segInts = segInts;
      this.segLongs = segLongs;
    }

    public int size() {
      return fileStart.length;
    }

    public Segment segment(int i) {
      return new Segment(this, i);
    }
  }

  /**
   * Reads `files` into one image and runs the read path over it.  framesPerFile bounds the entries
   * of any one file (closed segments: end - start + 1 from the file name, plus slack for the
   * garbage the reader skips after the last index); maxOpSize = the reader's limit
   * (raft.server.log.appender.buffer.byte-limit).  The image must stay under 2 GiB.
   */
  public synchronized Batch read(List<File> files, int framesPerFile, int maxOpSize) throws IOException {
    final int n = files.size();
    final long[] start = new long[n];
    final long[] len = new long[n];
    long total = 0;
    for (int i = 0; i < n; i++) {
      start[i] = total;
      len[i] = files.get(i).length();
      total += (len[i] + 255) & ~255L;   // 256-byte aligned file starts
    }
    if (total > Integer.MAX_VALUE - 256) {
      throw new IllegalArgumentException("segment batch of " + total + " bytes: split it below 2 GiB");
    }
    final ByteBuffer image = ByteBuffer.allocateDirect((int) Math.max(total, 1));
    for (int i = 0; i < n; i++) {
      try (RandomAccessFile f = new RandomAccessFile(files.get(i), "r"); FileChannel ch = f.getChannel()) {
        final ByteBuffer dst = image.duplicate();
        dst.position((int) start[i]).limit((int) (start[i] + len[i]));
        while (dst.hasRemaining()) {
          if (ch.read(dst) < 0) {
            throw new IOException("file shrank while reading: " + files.get(i));
          }
        }
      }
    }
    final int cap = Math.max(framesPerFile, 1);
    final long frames = Math.min((long) cap * n, Integer.MAX_VALUE - 8);
    final long[] frameOff = new long[(int) frames];
    final int[] frameLen = new int[(int) frames];
    final int[] frameCrc = new int[(int) frames];
    final int[] segInts = new int[3 * n];
    final long[] segLongs = new long[2 * n];
    RatisHip.readSegments0(ctx, image, total, start, len, n, maxOpSize, cap, frameOff, frameLen, frameCrc, segInts,
        segLongs);
    return new Batch(image, start, frameOff, frameLen, frameCrc, segInts, segLongs);
  }

  @Override
  public synchronized void close() throws IOException {
    if (ctx != 0) {
      RatisHip.ctxDestroy0(ctx);
      ctx = 0;
    }
  }
}
