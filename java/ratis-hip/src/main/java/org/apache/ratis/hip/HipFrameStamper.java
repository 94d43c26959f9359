/*
 * The write side of the checksum backend (raft.server.hip.checksum.backend = hip): the trailers of a
 * flush batch, stamped in one call.
 *
 * The reference computes each entry's trailer as it serialises the entry into the log worker's write
 * buffer (SegmentedRaftLogOutputStream.write, SegmentedRaftLogOutputStream.java:86-110: reset(),
 * update(varint || entry), putInt(getValue())).  With a stamper the stream writes a placeholder and
 * records the frame here; just before the buffer goes to the file (BufferedWriteChannel.flushBuffer,
 * the worker's flush, SegmentedRaftLogWorker.java:746-752) stamp() writes every pending trailer:
 * on the GPU (rh_crc32c_stamp_host: the batch crosses PCIe from the page-locked write buffer, 4 B per
 * frame come back) when the batch holds at least minGpuBytes, else with the caller's own
 * PureJavaCrc32C, frame by frame, exactly as write() would have.  The bytes written to the file are
 * the reference's either way.  minGpuBytes is the crossover measured by bench.py's write_stamp leg
 * (INTEGRATION.md): below it the PCIe round trip costs more than the CPU checksum.
 *
 * A GPU call that fails never fails the flush: the same frames are stamped by the CPU path, the
 * failure is counted (getGpuFailures), and after MAX_GPU_FAILURES of them the stamper stays on the
 * CPU.  The write buffer is page-locked lazily, at the first batch large enough for the GPU, so a
 * worker whose batches never reach minGpuBytes pins no host memory.
 *
 * Single-threaded, like BufferedWriteChannel (the log worker's thread).
 */
package org.apache.ratis.hip;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.Arrays;

public final class HipFrameStamper implements AutoCloseable {
  /** What write() computes for one frame: PureJavaCrc32C.getValue() after reset() and update() over
   *  the frame without its trailer (the view's [position, limit)). */
  public interface FrameChecksum {
    int crc(ByteBuffer frameWithoutTrailer);
  }

  /** Flush batches from this size on go to the GPU (bench.py write_stamp leg: crossover_bytes). */
  public static final int DEFAULT_MIN_GPU_BYTES = 64 << 10;
  /** GPU failures after which the stamper stays on the CPU path. */
  static final int MAX_GPU_FAILURES = 3;

  private final HipLogReader gpu;
  private final int minGpuBytes;
  private final ByteBuffer writeBuffer;
  private boolean registered;       // writeBuffer page-locked (at the first GPU-sized batch)
  private long gpuFailures;
  private long[] off = new long[1024];
  private int[] len = new int[1024];
  private int n;
  private long bytes;
  private long gpuBatches;
  private long cpuBatches;

  /** writeBuffer: the worker's reused direct write buffer, page-locked (from its first GPU-sized batch
   *  on) for the stamper's lifetime. */
  public HipFrameStamper(int deviceMask, int minGpuBytes, ByteBuffer writeBuffer) throws IOException {
    if (minGpuBytes < 0) {
      throw new IllegalArgumentException("minGpuBytes < 0: " + minGpuBytes);
    }
    this.gpu = HipLogReader.get(deviceMask);
    this.minGpuBytes = minGpuBytes;
    this.writeBuffer = writeBuffer;
  }

  /** A frame whose trailer is a placeholder: [pos, pos + length) of the write buffer, length = varint
   *  + entry + 4. */
  public void add(int pos, int length) {
    if (n == off.length) {
      off = Arrays.copyOf(off, 2 * n);
      len = Arrays.copyOf(len, 2 * n);
    }
    off[n] = pos;
    len[n] = length;
    n++;
    bytes += length;
  }

  /**
   * Writes every pending trailer of buf (its frames lie in [0, position)): the GPU for a batch of at
   * least minGpuBytes, else cpu per frame (as write() does).  Returns whether the GPU stamped it.
   */
  public boolean stamp(ByteBuffer buf, FrameChecksum cpu) throws IOException {
    if (n == 0) {
      return false;
    }
    boolean onGpu = false;
    if (bytes >= minGpuBytes && buf.isDirect() && gpuFailures < MAX_GPU_FAILURES) {
      try {
        if (!registered && buf == writeBuffer) {
          gpu.register(writeBuffer);
          registered = true;
        }
        gpu.stampFrames(buf, buf.position(), off, len, n);
        onGpu = true;
        gpuBatches++;
      } catch (IOException | RuntimeException e) {
        gpuFailures++;   // the CPU path below stamps the same frames: the file gets the reference's bytes
      }
    }
    if (!onGpu) {
      for (int i = 0; i < n; i++) {
        final int pos = (int) off[i];
        final int end = pos + len[i] - 4;
        final ByteBuffer d = buf.duplicate();
        d.position(pos).limit(end);
        buf.putInt(end, cpu.crc(d));
      }
      cpuBatches++;
    }
    // only now is every pending trailer written: a batch whose CPU path threw keeps its frames, and
    // the next stamp() (the close() flush included) writes them
    n = 0;
    bytes = 0;
    return onGpu;
  }

  /** Batches stamped on the GPU / by the CPU so far. */
  public long getGpuBatches() {
    return gpuBatches;
  }

  public long getCpuBatches() {
    return cpuBatches;
  }

  /** GPU calls that failed (their batches were stamped by the CPU path). */
  public long getGpuFailures() {
    return gpuFailures;
  }

  @Override
  public void close() throws IOException {
    if (registered) {
      registered = false;
      gpu.unregister(writeBuffer);
    }
  }
}
