/*
 * The checksum backend of the segmented log's bulk load (raft.server.hip.checksum.backend = hip):
 * SegmentedRaftLog.loadLogSegments (SegmentedRaftLog.java:248-276) reads many segment files at
 * server start; each is walked and checksummed by SegmentedRaftLogReader.decodeEntry
 * (SegmentedRaftLogReader.java:291-341: PureJavaCrc32C over every entry) through
 * LogSegment.readSegmentFile (LogSegment.java:166-196).  Here the files' bytes go to a GPU in one
 * rh_segments_read_host call per batch (framing walk + CRC32C of every frame + the reader's verdict
 * per file) and come back as, per file, the verified frame table and how the reader would have
 * ended; the caller (LogSegment, through the seams patch) parses the accepted entries from the same
 * image and raises what the reader would have raised -- ChecksumException at the failing entry's
 * offset, IOException / CorruptedFileException for the framing errors -- under its CorruptionPolicy.
 *
 * No LogEntryProto parsing here (ratis-hip does not depend on ratis-proto); a Segment exposes the
 * bytes of each accepted entry.  A file the GPU could not walk (more frames than the per-file slot
 * count, RH_SEG_E_CAPACITY) reports {@link Segment#usable()} = false and is left to the Java reader.
 *
 * Memory.  The reference streams one file at a time (SegmentedRaftLog.java:248-276).  A
 * {@link Pipeline} keeps that bound: it reads and verifies batch k + 1 on a loader thread while the
 * caller loads batch k's segments, with exactly two image buffers (each at most one batch), and a
 * batch's buffer goes back to the loader as soon as the caller moves past its last segment.  The
 * frame tables are sized per batch and bounded (MAX_FRAMES_PER_BATCH slots).
 *
 * GPUs.  One context per GPU of the device mask; batches and concurrent callers (one
 * SegmentedRaftLog per division loads at server start) are spread over them round robin, each
 * context serving one call at a time.
 */
package org.apache.ratis.hip;

import java.io.File;
import java.io.IOException;
import java.io.InterruptedIOException;
import java.io.RandomAccessFile;
import java.nio.ByteBuffer;
import java.nio.channels.FileChannel;
import java.util.ArrayList;
import java.util.Collections;
import java.util.List;
import java.util.concurrent.ArrayBlockingQueue;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.atomic.AtomicInteger;

public final class HipLogReader implements AutoCloseable {
  /** Frame slots of one batch (16 B of heap each: offset, length, CRC): callers cut batches so that
   *  files x framesPerFile stays under this, and a file needing more is left to the Java reader. */
  public static final int MAX_FRAMES_PER_BATCH = 1 << 24;

  private static HipLogReader instance;

  /** The process-wide reader over the GPUs of the mask. */
  public static synchronized HipLogReader get(int deviceMask) throws IOException {
    if (instance == null) {
      if (deviceMask == 0) {
        throw new IllegalArgumentException("empty device mask");
      }
      instance = new HipLogReader(deviceMask);
    }
    return instance;
  }

  private final long[] ctx;      // rh_ctx* per GPU of the mask
  private final Object[] ctxLock;
  private final AtomicInteger nextCtx = new AtomicInteger();

  private HipLogReader(int deviceMask) throws IOException {
    final List<Long> c = new ArrayList<>();
    try {
      for (int d = 0; d < 32; d++) {
        if ((deviceMask >>> d & 1) != 0) {
          c.add(RatisHip.ctxCreate0(d));
        }
      }
    } catch (IOException | RuntimeException e) {
      for (long h : c) {
        RatisHip.ctxDestroy0(h);
      }
      throw e;
    }
    this.ctx = new long[c.size()];
    this.ctxLock = new Object[c.size()];
    for (int i = 0; i < ctx.length; i++) {
      ctx[i] = c.get(i);
      ctxLock[i] = new Object();
    }
  }

  public int getDevices() {
    return ctx.length;
  }

  /** One file's outcome.  From a Pipeline: valid until the pipeline's next call to next(). */
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

  /** What one batch reads: its files and the frame slots each may fill. */
  public static final class Plan {
    final List<File> files;
    final int framesPerFile;

    public Plan(List<File> files, int framesPerFile) {
      if (files.isEmpty() || framesPerFile < 1 || (long) framesPerFile * files.size() > MAX_FRAMES_PER_BATCH) {
        throw new IllegalArgumentException("a batch of " + files.size() + " files x " + framesPerFile
            + " frame slots: needs 1..MAX_FRAMES_PER_BATCH slots");
      }
      this.files = Collections.unmodifiableList(new ArrayList<>(files));
      this.framesPerFile = framesPerFile;
    }

    /** Image bytes (256-byte aligned file starts). */
    long imageBytes() {
      long total = 0;
      for (File f : files) {
        total += (f.length() + 255) & ~255L;
      }
      return total;
    }
  }

  /**
   * Reads `files` into one image and runs the read path over it.  framesPerFile bounds the entries
   * of any one file (closed segments: end - start + 1 from the file name, plus slack for the
   * garbage the reader skips after the last index); maxOpSize = the reader's limit
   * (raft.server.log.appender.buffer.byte-limit).  The image must stay under 2 GiB.
   */
  public Batch read(List<File> files, int framesPerFile, int maxOpSize) throws IOException {
    final Plan p = new Plan(files, framesPerFile);
    return readInto(null, p, maxOpSize, nextCtx.getAndIncrement());
  }

  private Batch readInto(ByteBuffer buf, Plan plan, int maxOpSize, int ctxIndex) throws IOException {
    final List<File> files = plan.files;
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
    final ByteBuffer image = buf != null && buf.capacity() >= total ? buf
        : ByteBuffer.allocateDirect((int) Math.max(total, 1));
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
    final int cap = plan.framesPerFile;
    final int frames = cap * n;   // <= MAX_FRAMES_PER_BATCH (Plan)
    final long[] frameOff = new long[frames];
    final int[] frameLen = new int[frames];
    final int[] frameCrc = new int[frames];
    final int[] segInts = new int[3 * n];
    final long[] segLongs = new long[2 * n];
    final int c = Math.floorMod(ctxIndex, ctx.length);
    synchronized (ctxLock[c]) {
      if (ctx[c] == 0) {
        throw new IOException("HipLogReader is closed");
      }
      RatisHip.readSegments0(ctx[c], image, total, start, len, n, maxOpSize, cap, frameOff, frameLen, frameCrc,
          segInts, segLongs);
    }
    return new Batch(image, start, frameOff, frameLen, frameCrc, segInts, segLongs);
  }

  // ---- the write side of the same backend (HipFrameStamper) -----------------------------------
  /** Page-locks a direct buffer (the log worker's reused write buffer) for DMA from every GPU. */
  void register(ByteBuffer direct) throws IOException {
    synchronized (ctxLock[0]) {
      RatisHip.hostRegister0(ctx[0], direct);
    }
  }

  void unregister(ByteBuffer direct) throws IOException {
    synchronized (ctxLock[0]) {
      if (ctx[0] != 0) {
        RatisHip.hostUnregister0(ctx[0], direct);
      }
    }
  }

  /** rh_crc32c_stamp_host: the trailers of frames [off[i], off[i] + len[i]) of buf[0, limit)
   *  written in place (big-endian PureJavaCrc32C of the bytes before each). */
  void stampFrames(ByteBuffer direct, int limit, long[] off, int[] len, int n) throws IOException {
    final int c = Math.floorMod(nextCtx.getAndIncrement(), ctx.length);
    synchronized (ctxLock[c]) {
      if (ctx[c] == 0) {
        throw new IOException("HipLogReader is closed");
      }
      RatisHip.stampHost0(ctx[c], direct, limit, off, len, n);
    }
  }

  /** The bulk load of one directory: batch k + 1 read and verified while the caller loads batch k. */
  public Pipeline pipeline(List<Plan> plans, int maxOpSize) {
    return new Pipeline(plans, maxOpSize);
  }

  /**
   * Segments in plan order.  Two image buffers: the loader thread fills one while the caller
   * consumes the other; the caller's buffer returns to the loader when next() moves past the last
   * segment of its batch, so the direct memory in use never exceeds two batch images.
   */
  public final class Pipeline implements AutoCloseable {
    private final BlockingQueue<Object> ready = new ArrayBlockingQueue<>(1);   // a Batch, or the loader's failure
    private final BlockingQueue<ByteBuffer> free = new ArrayBlockingQueue<>(2);
    private final Thread loader;
    private final int batches;
    private int taken;
    private Batch current;
    private int index;

    Pipeline(List<Plan> plans, int maxOpSize) {
      this.batches = plans.size();
      long max = 1;
      for (Plan p : plans) {
        max = Math.max(max, p.imageBytes());
      }
      if (max > Integer.MAX_VALUE - 256) {
        throw new IllegalArgumentException("segment batch of " + max + " bytes: split it below 2 GiB");
      }
      final int bytes = (int) max;
      free.add(ByteBuffer.allocateDirect(bytes));
      free.add(ByteBuffer.allocateDirect(bytes));
      final int first = nextCtx.getAndAdd(plans.size());
      this.loader = new Thread(() -> {
        try {
          for (int k = 0; k < plans.size(); k++) {
            final ByteBuffer buf = free.take();   // blocks while both images are in use
            ready.put(readInto(buf, plans.get(k), maxOpSize, first + k));
          }
        } catch (InterruptedException e) {
          Thread.currentThread().interrupt();
        } catch (Throwable t) {
          try {
            ready.put(t);   // after the batch the caller has not taken yet, if any
          } catch (InterruptedException e) {
            Thread.currentThread().interrupt();
          }
        }
      }, "ratis-hip-log-loader");
      loader.setDaemon(true);
      loader.start();
    }

    /** The next file's outcome (plan order), valid until the following call. */
    public Segment next() throws IOException {
      if (current == null || index == current.size()) {
        if (current != null) {
          free.offer(current.image);   // the previous batch is consumed: its image goes back to the loader
          current = null;
        }
        if (taken == batches) {
          throw new IllegalStateException("no more segments");
        }
        final Object o;
        try {
          o = ready.take();
        } catch (InterruptedException e) {
          Thread.currentThread().interrupt();
          throw new InterruptedIOException("interrupted while the GPU read the log");
        }
        if (o instanceof IOException) {
          throw (IOException) o;
        } else if (o instanceof Throwable) {
          throw new IOException("the GPU log read failed", (Throwable) o);
        }
        current = (Batch) o;
        index = 0;
        taken++;
      }
      return current.segment(index++);
    }

    @Override
    public void close() {
      loader.interrupt();
      try {
        loader.join();
      } catch (InterruptedException e) {
        Thread.currentThread().interrupt();
      }
      current = null;
      ready.clear();
      free.clear();
    }
  }

  @Override
  public void close() throws IOException {
    for (int i = 0; i < ctx.length; i++) {
      synchronized (ctxLock[i]) {
        if (ctx[i] != 0) {
          RatisHip.ctxDestroy0(ctx[i]);
          ctx[i] = 0;
        }
      }
    }
  }
}
