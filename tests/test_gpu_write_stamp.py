"""GPU parity of the write side over host buffers (rh_crc32c_stamp_host): a flush batch of frames
written with placeholder trailers, stamped in one call, must equal byte for byte what the oracle's
writer (orc_frame_write = SegmentedRaftLogOutputStream.write, OUT:86-110: varint32(n) || entry ||
big-endian PureJavaCrc32C) produces for the same entries -- at the flush sizes the bench compares
(64 KiB, 1 MiB, 8 MiB = raft.server.log.write.buffer.size's default), from pageable and from
registered (page-locked) memory, with frames at any offset of the buffer and the bytes around them
untouched; malformed tables stamp nothing."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _flush_batch(orc, rng, nbytes, lo=1, hi=2040, lead=0):
    """Entries of random sizes framed by the oracle writer until ~nbytes; returns (expected image,
    placeholder image with zero trailers, frame offsets, frame lengths)."""
    parts, off, ln = [], [], []
    pos = lead
    while pos < nbytes:
        proto = rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8).tobytes()
        fr = orc.frame_write(proto)
        off.append(pos)
        ln.append(len(fr))
        parts.append(np.frombuffer(fr, dtype=np.uint8))
        pos += len(fr)
    want = np.concatenate([rng.integers(0, 256, lead, dtype=np.uint8)] + parts + [rng.integers(0, 256, 37, dtype=np.uint8)])
    buf = want.copy()
    off = np.array(off, dtype=np.uint64)
    ln = np.array(ln, dtype=np.uint32)
    for o, l in zip(off, ln):
        buf[int(o) + int(l) - 4: int(o) + int(l)] = 0
    return want, buf, off, ln


@pytest.mark.parametrize("nbytes", [64 << 10, 1 << 20, 8 << 20])
def test_stamped_flush_batch_equals_oracle_writer(ctx, orc, nbytes):
    from ratis_amd import engine
    rng = np.random.default_rng(nbytes)
    want, buf, off, ln = _flush_batch(orc, rng, nbytes, lead=int(rng.integers(0, 300)))
    engine.stamp_host(ctx, buf, off, ln)
    assert np.array_equal(buf, want)
    # the same from page-locked memory (the worker's write buffer is registered once)
    want2, buf2, off2, ln2 = _flush_batch(orc, rng, nbytes, lo=100, hi=4000)
    with engine.HostRegistration(ctx, buf2):
        engine.stamp_host(ctx, buf2, off2, ln2)
    assert np.array_equal(buf2, want2)


def test_stamp_edge_frames_and_errors(ctx, orc):
    from ratis_amd import _lib, engine
    rng = np.random.default_rng(5)
    # an empty entry (5-byte frame), 1-byte entries, a multi-byte varint (>= 128 B) entry, a 300 KiB entry
    protos = [b"", b"\x01", bytes(range(200)), rng.integers(0, 256, 300 << 10, dtype=np.uint8).tobytes(), b"\x07" * 127]
    frames = [orc.frame_write(p) for p in protos]
    want = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    ln = np.array([len(f) for f in frames], dtype=np.uint32)
    buf = want.copy()
    for o, l in zip(off, ln):
        buf[int(o) + int(l) - 4: int(o) + int(l)] = 0xAB
    engine.stamp_host(ctx, buf, off, ln)
    assert np.array_equal(buf, want)
    engine.stamp_host(ctx, buf, off[:0], ln[:0])            # no frames: nothing to do
    before = buf.copy()
    buf[int(off[1]) + int(ln[1]) - 4] ^= 0xFF
    spoiled = buf.copy()
    with pytest.raises(_lib.IllegalArgumentError):           # a frame past the buffer end: nothing stamped
        engine.stamp_host(ctx, buf, np.append(off, buf.size - 2), np.append(ln, 8))
    assert np.array_equal(buf, spoiled)
    with pytest.raises(_lib.IllegalArgumentError):           # shorter than its trailer
        engine.stamp_host(ctx, buf, off[:1], np.array([3], dtype=np.uint32))
    engine.stamp_host(ctx, buf, off, ln)
    assert np.array_equal(buf, before)


def _frames(orc, rng, sizes, gap=0):
    """One frame per entry size, gap random bytes between frames; returns (expected image,
    placeholder image, offsets, lengths)."""
    parts, off, ln = [], [], []
    pos = 0
    for sz in sizes:
        g = rng.integers(0, 256, int(rng.integers(0, gap + 1)) if gap else 0, dtype=np.uint8)
        parts.append(g)
        pos += g.size
        fr = np.frombuffer(orc.frame_write(rng.integers(0, 256, int(sz), dtype=np.uint8).tobytes()), dtype=np.uint8)
        off.append(pos)
        ln.append(fr.size)
        parts.append(fr)
        pos += fr.size
    want = np.concatenate(parts)
    buf = want.copy()
    for o, l in zip(off, ln):
        buf[o + l - 4: o + l] = 0x5A
    return want, buf, np.array(off, dtype=np.uint64), np.array(ln, dtype=np.uint32)


@pytest.mark.parametrize("case", ["512_window", "513_serial", "long_frame_over_512", "shuffled_with_gaps"])
def test_stamp_plan_boundaries(ctx, orc, case):
    """rh_crc32c_stamp_host's plan choice (rh_api.cpp, RH_STAMP_PLAN 2): up to 512 frames one
    window-kernel batch, more frames one lane each (frames up to 64 KiB), more frames with a longer
    one on the window kernel over several batches; and a table whose frames are not in buffer order
    with bytes between them (only the covered span crosses PCIe)."""
    from ratis_amd import engine
    rng = np.random.default_rng(len(case))
    if case == "512_window":
        sizes = rng.integers(0, 700, 512)
    elif case == "513_serial":
        sizes = rng.integers(0, 700, 513)
    elif case == "long_frame_over_512":
        sizes = np.append(rng.integers(0, 700, 599), 70 << 10)
        rng.shuffle(sizes)
    else:
        sizes = rng.integers(0, 3000, 300)
    want, buf, off, ln = _frames(orc, rng, sizes, gap=40 if case == "shuffled_with_gaps" else 0)
    if case == "shuffled_with_gaps":
        p = rng.permutation(off.size)
        off, ln = off[p], ln[p]
    engine.stamp_host(ctx, buf, off, ln)
    assert np.array_equal(buf, want)


@pytest.mark.parametrize("case", ["16k", "64k_unaligned", "1m_groups", "tiny_entries", "1024_frames", "1025_frames",
                                  "shuffled_with_gaps", "long_frame_fallback", "8m_over_groups", "max_payloads",
                                  "ends_at_registration_end"])
def test_stamp_zero_copy_registered(ctx, orc, case):
    """The zero-copy plan (rh_api.cpp stamp_zero_copy, rh_internal.h StampArgs): a registered buffer,
    payloads under 16 KiB, at most 96 workgroups of 64 KiB span / 1024 windows / 1024 frames.  Frames
    at unaligned offsets (the span's 16-byte rounding), empty and 1..3-byte payloads (windows that
    are all leading bytes), workgroup splits by frame count and by span, frames out of buffer order
    (a new workgroup whenever a frame starts before its group), and batches the plan does not take
    (a 20 KiB payload, an 8 MiB batch over 96 workgroups) -- every trailer equal to the oracle
    writer's and every other byte untouched."""
    from ratis_amd import engine
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    gap = 0
    if case == "16k":
        sizes = rng.integers(64, 2048, 16)
    elif case == "64k_unaligned":
        sizes = rng.integers(1, 2048, 60)
        gap = 13
    elif case == "1m_groups":
        sizes = rng.integers(64, 2048, 1000)
    elif case == "tiny_entries":
        sizes = np.concatenate([np.zeros(40, np.int64), rng.integers(0, 4, 200), rng.integers(60, 70, 50)])
        rng.shuffle(sizes)
    elif case == "1024_frames":
        sizes = rng.integers(0, 100, 1024)
    elif case == "1025_frames":
        sizes = rng.integers(0, 100, 1025)
    elif case == "shuffled_with_gaps":
        sizes = rng.integers(0, 5000, 200)
        gap = 40
    elif case == "long_frame_fallback":
        sizes = np.append(rng.integers(0, 700, 50), 20 << 10)
    elif case == "max_payloads":   # payloads just under 16 KiB: 256 windows, every shift map staged
        sizes = np.append(rng.integers(16300, 16378, 12), rng.integers(0, 100, 30))
        rng.shuffle(sizes)
    elif case == "ends_at_registration_end":
        sizes = rng.integers(1, 3000, 40)
    else:
        sizes = rng.integers(64, 2048, 8000)
    want, buf, off, ln = _frames(orc, rng, sizes, gap=gap)
    lead = int(rng.integers(1, 16))   # the batch starts off a 16-byte boundary of the registration
    tail = 0 if case == "ends_at_registration_end" else 21   # (or ends exactly where it ends)
    want = np.concatenate([np.full(lead, 0xC3, np.uint8), want, np.full(tail, 0x3C, np.uint8)])
    buf = np.concatenate([np.full(lead, 0xC3, np.uint8), buf, np.full(tail, 0x3C, np.uint8)])
    off = off + np.uint64(lead)
    if case == "shuffled_with_gaps":
        p = rng.permutation(off.size)
        off, ln = off[p], ln[p]
    with engine.HostRegistration(ctx, buf):
        engine.stamp_host(ctx, buf, off, ln)
        assert np.array_equal(buf, want)
        engine.stamp_host(ctx, buf, off, ln)   # restamping stamped frames: the same bytes
        assert np.array_equal(buf, want)
