"""GPU parity of the fused read path (rh_segments_read_launch: framing walk + CRC32C verify of every
frame in one pass = LogSegment.readSegmentFile, LogSegment.java:166-196) against the oracle's
orc_segment_scan, which runs SegmentedRaftLogReader's verifyHeader / decodeEntry (with its
checksum, RDR:327-336) / verifyTerminator literally, and against the two-pass path's framing.

Covered: every damage kind of test_gpu_segment (header, truncation, varint, oversize, padding,
flipped payload bits), frames long enough to leave the LDS ring (folded from HBM), thousands of
tiny frames per window (the per-step frame/unit list fills up), CRC spans of 2 and 3 bytes (the
reset() state reaches past the message), the TestRaftLogReadWrite segment and config-5 segments
with planted corruptions."""
import os

import numpy as np
import pytest

from .test_gpu_segment import HEADER, KINDS, make_segment, pack, speculation_images

pytestmark = pytest.mark.gpu


def run_fused(ctx, buf, offs, lens, max_op=4 << 20, cap=4096):
    import torch

    from ratis_amd import engine
    dev = torch.device("cuda")
    b = engine.SegmentBatch(buf=torch.from_numpy(buf).to(dev), seg_off=torch.from_numpy(offs).to(dev),
                            seg_len=torch.from_numpy(lens).to(dev), max_op=max_op, frames_per_seg_cap=cap)
    out = engine.read_segments_fused(ctx, b)
    torch.cuda.synchronize()
    return b, out


def _bits(words, n):
    return np.unpackbits(np.asarray(words).view(np.uint64).view(np.uint8), bitorder="little")[:n].astype(bool)


def check_fused(ctx, orc, b, out, buf, offs, lens, max_op=4 << 20, cap=4096):
    import torch

    from ratis_amd import engine
    # 1. the reader's verdict per segment == the literal reader (framing + checksum)
    n_ok, st, stop = out["n_ok"].cpu().numpy(), out["status"].cpu().numpy(), out["stop"].cpu().numpy()
    for s in range(len(offs)):
        ro, _, _, rst, rstop = orc.segment_scan(buf[offs[s]: offs[s] + lens[s]], max_op=max_op)
        assert (st[s], stop[s], n_ok[s]) == (rst, rstop, len(ro)), s
    # 2. framing outputs == the two-pass framing walk on the same buffer
    b2 = engine.SegmentBatch(buf=b.buf, seg_off=b.seg_off, seg_len=b.seg_len, max_op=max_op, frames_per_seg_cap=cap)
    engine.segments_scan(ctx, b2)
    torch.cuda.synchronize()
    for name in ("seg_nframes", "seg_status", "seg_stop", "seg_first"):
        assert torch.equal(getattr(b, name)[: len(offs)], getattr(b2, name)[: len(offs)]), name
    total = int(b.total_frames.item())
    assert total == int(b2.total_frames.item())
    assert torch.equal(b.frame_off[:total], b2.frame_off[:total])
    assert torch.equal(b.frame_len[:total], b2.frame_len[:total])
    # 3. every frame's CRC == PureJavaCrc32C over varint||proto; mismatch bit == (stored != computed)
    fo = b.frame_off[:total].cpu().numpy()
    fl = b.frame_len[:total].cpu().numpy()
    got = out["crc_out"][:total].cpu().numpy().view(np.uint32)
    want, _ = orc.crc32c_frames(buf, fo.astype(np.uint64), fl.astype(np.uint32))
    assert np.array_equal(got, want)
    stored = np.array([int.from_bytes(buf[o + l - 4: o + l].tobytes(), "big") for o, l in zip(fo, fl)], np.uint32)
    bad = _bits(out["bad_bits"].cpu().numpy(), total)
    assert np.array_equal(bad, stored != want)
    assert int(out["n_bad"].item()) == int(bad.sum())
    return total


@pytest.mark.parametrize("big", [False, True])
def test_fused_matches_reader_every_kind(ctx, orc, big):
    rng = np.random.default_rng(70 + big)
    kinds = [KINDS[i % len(KINDS)] for i in range(len(KINDS) * 6)]
    made = [make_segment(orc, rng, k, big) for k in kinds]
    buf, offs, lens = pack([m[0] for m in made], rng)
    b, out = run_fused(ctx, buf, offs, lens)
    check_fused(ctx, orc, b, out, buf, offs, lens)
    from ratis_amd import _lib
    st = set(out["status"].cpu().numpy().tolist())
    for code in (_lib.RH_SEG_END, _lib.RH_SEG_PARTIAL, _lib.RH_SEG_E_OVERSIZE, _lib.RH_SEG_E_PADDING,
                 _lib.RH_SEG_E_VARINT, _lib.RH_SEG_E_HEADER, _lib.RH_SEG_E_CHECKSUM):
        assert code in st, code


def test_fused_long_frames_folded_from_hbm(ctx, orc):
    """Frames from 20 KiB to 600 KiB (past the 64 KiB ring), between runs of small frames, some
    with a flipped bit: the long ones are folded straight from HBM by one group."""
    rng = np.random.default_rng(5)
    images = []
    for i in range(10):
        protos = []
        for j in range(int(rng.integers(3, 12))):
            n = int(rng.integers(20_000, 600_000)) if rng.random() < 0.4 else int(rng.integers(1, 5000))
            protos.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        frames = [orc.frame_write(p) for p in protos]
        body = bytearray(HEADER + b"".join(frames) + bytes(int(rng.integers(0, 3000))))
        if i % 3 == 1:  # corrupt one byte inside a long frame's payload
            starts = np.cumsum([8] + [len(f) for f in frames])
            k = int(np.argmax([len(f) for f in frames]))
            body[int(starts[k]) + len(frames[k]) // 2] ^= 0x40
        images.append(bytes(body))
    buf, offs, lens = pack(images, rng)
    b, out = run_fused(ctx, buf, offs, lens)
    check_fused(ctx, orc, b, out, buf, offs, lens)
    assert int(out["n_bad"].item()) >= 3


def test_fused_tiny_frames_and_short_spans(ctx, orc):
    """~2000 frames per 16 KiB window (the per-step list caps at 256 frames / 512 units and the walk
    resumes inside the window) and 1- and 2-byte protos, whose CRC spans of 2 and 3 bytes leave part
    of reset()'s 0xFFFFFFFF past the message."""
    rng = np.random.default_rng(8)
    images = []
    for i in range(6):
        fr = [orc.frame_write(bytes(rng.integers(0, 256, 1 + (j % 3), dtype=np.uint8))) for j in range(6000 + 17 * i)]
        body = bytearray(HEADER + b"".join(fr) + bytes(100))
        if i % 2:
            body[int(rng.integers(8, len(body) - 200))] ^= 1
        images.append(bytes(body))
    buf, offs, lens = pack(images, rng)
    b, out = run_fused(ctx, buf, offs, lens, cap=8192)
    total = check_fused(ctx, orc, b, out, buf, offs, lens, cap=8192)
    assert total > 30_000


def test_fused_frame_capacity(ctx, orc):
    from ratis_amd import _lib
    rng = np.random.default_rng(3)
    img = HEADER + b"".join(orc.frame_write(bytes([7]) * 5) for _ in range(100)) + bytes(100)
    buf, offs, lens = pack([img, img], rng)
    b, out = run_fused(ctx, buf, offs, lens, cap=64)
    assert list(b.seg_status.cpu().numpy()) == [_lib.RH_SEG_E_CAPACITY] * 2
    assert list(out["n_ok"].cpu().numpy()) == [64, 64]


def test_fused_raftlog_readwrite_golden(ctx, orc):
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "raftlog_rw.npz"))
    img = np.asarray(z["image"], dtype=np.uint8)
    bad = img.copy()
    bad[100] ^= 0xFF   # TestRaftLogReadWrite's corruption case: byte 100 flipped (:239-268)
    rng = np.random.default_rng(0)
    buf, offs, lens = pack([img.tobytes(), img.tobytes() + bytes(4096), bad.tobytes()], rng)
    b, out = run_fused(ctx, buf, offs, lens)
    check_fused(ctx, orc, b, out, buf, offs, lens)
    assert list(out["n_ok"].cpu().numpy())[:2] == [100, 100]


def test_fused_config5_segments(ctx, orc):
    """32 MiB segments of 4 KiB frames with planted corruptions: the frame
    table equals the generator's and the mismatch set equals the planted set."""
    import torch

    from ratis_amd import engine, workload
    ss = workload.synth_segments(ctx, n_segments=6, corrupt_rate=3e-4, seed=41)
    n = ss.n_segments
    b = engine.SegmentBatch(buf=ss.batch.buf, seg_off=torch.arange(n, dtype=torch.int64, device="cuda") * ss.segment_size,
                            seg_len=torch.full((n,), ss.segment_size, dtype=torch.int64, device="cuda"),
                            frames_per_seg_cap=ss.frames_per_segment + 16)
    out = engine.read_segments_fused(ctx, b)
    torch.cuda.synchronize()
    nf = n * ss.frames_per_segment
    assert int(b.total_frames.item()) == nf
    assert torch.equal(b.frame_off[:nf], ss.batch.frame_off) and torch.equal(b.frame_len[:nf], ss.batch.frame_len)
    bad = np.nonzero(_bits(out["bad_bits"].cpu().numpy(), nf))[0]
    assert np.array_equal(bad, ss.corrupted) and ss.corrupted.size > 0
    fps = ss.frames_per_segment
    ok = out["n_ok"].cpu().numpy()
    for sgi in range(n):
        mine = ss.corrupted[(ss.corrupted >= sgi * fps) & (ss.corrupted < (sgi + 1) * fps)]
        assert int(ok[sgi]) == (int(mine[0]) - sgi * fps if mine.size else fps), sgi
    idx = np.linspace(0, nf - 1, 48).astype(np.int64)
    offs = b.frame_off.cpu().numpy()
    got = out["crc_out"].cpu().numpy().view(np.uint32)
    for i in idx:
        fr = ss.batch.buf[int(offs[i]): int(offs[i]) + ss.frame_size - 4].cpu().numpy().tobytes()
        assert orc.crc32c(fr) == int(got[i])


def test_fused_bad_arguments(ctx):
    import torch

    from ratis_amd import _lib, engine
    dev = torch.device("cuda")
    b = engine.SegmentBatch(buf=torch.zeros(16, dtype=torch.uint8, device=dev),
                            seg_off=torch.zeros(1, dtype=torch.int64, device=dev),
                            seg_len=torch.full((1,), 16, dtype=torch.int64, device=dev), frames_per_seg_cap=0)
    with pytest.raises(_lib.IllegalArgumentError):
        engine.read_segments_fused(ctx, b)


def test_fused_speculative_walk_edges(ctx, orc):
    """The fused walker's speculation (test_gpu_segment.speculation_images)."""
    rng = np.random.default_rng(123)
    buf, offs, lens = pack(speculation_images(orc, rng), rng)
    b, out = run_fused(ctx, buf, offs, lens, cap=1024)
    check_fused(ctx, orc, b, out, buf, offs, lens, cap=1024)


def test_fused_ragged_segments_with_corruption(ctx, orc):
    """Ragged frame lengths with planted corruptions through rh_segments_read_launch: the mismatch
    set is exactly the planted set and every segment stops at its first planted frame."""
    import torch

    from ratis_amd import engine, workload
    rs = workload.synth_ragged_segments(ctx, 6, segment_size=2 << 20, min_frame=20, max_frame=3000, seed=9,
                                        corrupt_rate=3e-4)
    n = rs.n_segments
    b = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * rs.segment_size,
                            seg_len=torch.full((n,), rs.segment_size, device="cuda", dtype=torch.int64),
                            frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
    out = engine.read_segments_fused(ctx, b)
    torch.cuda.synchronize()
    nf = int(rs.seg_nframes.sum())
    assert int(b.total_frames.item()) == nf
    bad = np.nonzero(_bits(out["bad_bits"].cpu().numpy(), nf))[0]
    assert np.array_equal(bad, rs.corrupted) and rs.corrupted.size > 0
    first = np.concatenate([[0], np.cumsum(rs.seg_nframes)[:-1]])
    ok = out["n_ok"].cpu().numpy()
    for sgi in range(n):
        mine = rs.corrupted[(rs.corrupted >= first[sgi]) & (rs.corrupted < first[sgi] + rs.seg_nframes[sgi])]
        assert int(ok[sgi]) == (int(mine[0] - first[sgi]) if mine.size else int(rs.seg_nframes[sgi])), sgi


@pytest.mark.parametrize("lo,hi", [(20, 1500), (1200, 6000)])
def test_fused_ragged_both_crc_plans_against_oracle(ctx, orc, lo, hi):
    """Ragged segments through rh_segments_read_launch under both CRC plans -- the length-class
    split with the dense outputs written by the CRC pass (mean slot length <= 2 KiB) and the
    window kernel followed by the compaction pass (longer frames): the reader's verdict, the frame
    table, every dense CRC and mismatch bit against the oracle, with planted corruptions."""
    from ratis_amd import workload
    rs = workload.synth_ragged_segments(ctx, 5, segment_size=2 << 20, min_frame=lo, max_frame=hi, seed=17 + lo,
                                        corrupt_rate=3e-3)
    n, size = rs.n_segments, rs.segment_size
    cap = int(rs.seg_nframes.max()) + 16
    split = (n * size) / (n * cap) <= 2048
    assert split == (hi <= 1500)
    buf = rs.batch.buf.cpu().numpy()
    offs = np.arange(n, dtype=np.int64) * size
    lens = np.full(n, size, dtype=np.int64)
    b, out = run_fused(ctx, buf, offs, lens, cap=cap)
    total = check_fused(ctx, orc, b, out, buf, offs, lens, cap=cap)
    assert total == int(rs.seg_nframes.sum())
    bad = np.nonzero(_bits(out["bad_bits"].cpu().numpy(), total))[0]
    assert np.array_equal(bad, rs.corrupted) and rs.corrupted.size > 0


@pytest.mark.parametrize("big", [False, True])
def test_host_image_read_path_matches_reader(ctx, orc, big):
    """rh_segments_read_host (the Java module's bulk LogSegment load: host image in, the reader's
    verdict and the verified frame table out, PCIe included) against the literal reader, per
    segment: status, stop offset, accepted entries, their offsets / lengths and CRCs."""
    from ratis_amd import _lib, engine
    rng = np.random.default_rng(170 + big)
    kinds = [KINDS[i % len(KINDS)] for i in range(len(KINDS) * 4)]
    made = [make_segment(orc, rng, k, big) for k in kinds]
    buf, offs, lens = pack([m[0] for m in made], rng)
    r = engine.read_segments_host(ctx, buf, offs, lens)
    seen = set()
    for s in range(len(offs)):
        ro, rl, rc, rst, rstop = orc.segment_scan(buf[offs[s]: offs[s] + lens[s]])
        assert (r["status"][s], r["stop"][s], r["n_ok"][s]) == (rst, rstop, len(ro)), s
        f0 = r["first_frame"][s]
        k = len(ro)
        assert np.array_equal(r["frame_off"][f0:f0 + k] - offs[s], ro), s
        assert np.array_equal(r["frame_len"][f0:f0 + k], rl), s
        assert np.array_equal(r["frame_crc"][f0:f0 + k], rc), s
        seen.add(int(rst))
    assert {_lib.RH_SEG_END, _lib.RH_SEG_PARTIAL, _lib.RH_SEG_E_CHECKSUM, _lib.RH_SEG_E_HEADER} <= seen
    # a segment with more frames than frames_per_seg_cap is reported, not truncated silently
    # (unless the reader already stops at a checksum failure inside the slots it has)
    r2 = engine.read_segments_host(ctx, buf, offs, lens, frames_per_seg_cap=2)
    n_cap = 0
    for s in range(len(offs)):
        ro, _, _, rst, _ = orc.segment_scan(buf[offs[s]: offs[s] + lens[s]])
        if len(ro) > 2:
            assert r2["status"][s] == _lib.RH_SEG_E_CAPACITY, s
            n_cap += 1
        elif rst == _lib.RH_SEG_E_CHECKSUM and len(ro) < 2:
            assert r2["status"][s] == _lib.RH_SEG_E_CHECKSUM, s
    assert n_cap > 0


def test_fused_ragged_bench_scale_against_oracle(ctx, orc):
    """The ragged read path at the bench's own scale per segment (32 x 32 MiB = 1 GiB, 64-2048 B
    frames, corruptions planted at the bench's rate), checked against the oracle -- not only against
    the generator's self-stamped trailers: every segment's verdict, stop offset and accepted frame
    table against the literal reader (orc_segment_scan), every frame's CRC recomputed from the bytes
    by the oracle (16 host threads), and the mismatch set against the oracle's own stored-vs-computed
    comparison AND the planted set."""
    import torch

    from ratis_amd import engine, workload
    rs = workload.synth_ragged_segments(ctx, 32, segment_size=32 << 20, min_frame=64, max_frame=2048,
                                        seed=workload.SEED + 4242, corrupt_rate=1e-5)
    n, size = rs.n_segments, rs.segment_size
    cap = int(rs.seg_nframes.max()) + 16
    b = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * size,
                            seg_len=torch.full((n,), size, device="cuda", dtype=torch.int64), frames_per_seg_cap=cap)
    out = engine.read_segments_fused(ctx, b)
    torch.cuda.synchronize()
    total = int(b.total_frames.item())
    assert total == int(rs.seg_nframes.sum()) > 500_000
    buf = rs.batch.buf.cpu().numpy()
    fo = b.frame_off[:total].cpu().numpy().astype(np.uint64)
    fl = b.frame_len[:total].cpu().numpy().astype(np.uint32)
    first = b.seg_first[:n].cpu().numpy()
    n_ok, st, stop = out["n_ok"].cpu().numpy(), out["status"].cpu().numpy(), out["stop"].cpu().numpy()
    for s in range(n):
        seg = buf[s * size: (s + 1) * size]
        ro, rl, rc, rst, rstop = orc.segment_scan(seg, cap=cap)
        assert (st[s], stop[s], n_ok[s]) == (rst, rstop, len(ro)), s
        k = len(ro)
        assert np.array_equal(fo[first[s]: first[s] + k].astype(np.int64) - s * size, ro), s
        assert np.array_equal(fl[first[s]: first[s] + k], rl), s
    crc, bad_ref = orc.crc32c_frames_all(buf, fo, fl, threads=16)
    assert np.array_equal(out["crc_out"][:total].cpu().numpy().view(np.uint32), crc)
    bad = _bits(out["bad_bits"].cpu().numpy(), total)
    assert np.array_equal(bad, bad_ref)
    assert np.array_equal(np.nonzero(bad)[0], rs.corrupted) and rs.corrupted.size > 0
    assert int(out["n_bad"].item()) == int(bad.sum())
