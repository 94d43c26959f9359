"""The JNI glue executed: java/ratis-hip/src/main/native/ratis_hip_jni.c,
compiled unchanged with a fake JNIEnv (tests/jni_harness/fake_jni.c: Java arrays and direct
buffers are views of numpy memory, ThrowNew records the exception) and called through ctypes the
way RatisHip.java calls it.  Every native the pump (HipLeaderBookkeeper.tick) and the checksum
backend (HipLogReader, HipFrameStamper) use runs against the same rh_* calls made directly on a
twin table and against the oracle / table model; short arrays, a buffer position beyond the
buffer, heap buffers and library rejections raise the exception class RatisHip.java documents
(RH_E_INVAL / RH_E_RANGE -> IllegalArgumentException, the rest -> IOException), and every array
the glue pins is released."""
import ctypes
import os

import numpy as np
import pytest
import torch  # noqa: F401 -- torch's HIP runtime must be the process's first (the harness links libratis_hip)

from tests.table_model import COL_FLUSH, TableModel
from tests.test_gpu_table import conf_word, random_deltas

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "jni_harness", "_build", "libratis_hip_jni_test.so")
NATIVES = ["nodeCreate0", "nodeDestroy0", "nodeShards0", "shardOf0", "groupStart0", "groupReconf0", "groupStop0",
           "pushDeltas0", "acquire0", "submit0", "commitBatch0", "commitAsync0", "tickAsync0", "commitWait0", "watchLevels0",
           "watchAsync0", "watchWait0", "setEventSink0", "leaseStart0", "leaseBatch0", "leaseBatchShard0",
           "leaseAsync0", "leaseWait0", "verifyHost0", "ctxCreate0", "ctxDestroy0", "readSegments0", "stampHost0",
           "hostRegister0", "hostUnregister0"]
IAE, IOE = "java/lang/IllegalArgumentException", "java/io/IOException"

P, L, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32


def jint(w: int) -> int:
    """A u32 conf word as the Java int RatisHip passes."""
    return w - (1 << 32) if w >= (1 << 31) else w


class Jni:
    """RatisHip's natives over the fake JNIEnv (every call: env + class, then the Java arguments)."""

    def __init__(self):
        self.h = ctypes.CDLL(HARNESS)
        self.h.fj_env.restype = P
        self.h.fj_array.restype = P
        self.h.fj_array.argtypes = [ctypes.c_int, ctypes.c_int32, P]
        self.h.fj_buffer.restype = P
        self.h.fj_buffer.argtypes = [P, L, ctypes.c_int]
        self.h.fj_buffer_address.restype = P
        self.h.fj_buffer_address.argtypes = [P]
        self.h.fj_buffer_capacity.restype = L
        self.h.fj_buffer_capacity.argtypes = [P]
        self.h.fj_take_exception.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        self.h.fj_pins_outstanding.restype = ctypes.c_long
        self.env = self.h.fj_env()
        self.keep = []

    def fn(self, name, res, *args):
        f = getattr(self.h, "Java_org_apache_ratis_hip_RatisHip_" + name)
        f.restype = res
        f.argtypes = [P, P] + list(args)
        return lambda *a: f(self.env, None, *a)

    def arr(self, a):
        """A Java array over numpy memory (None -> null)."""
        if a is None:
            return None
        assert a.flags["C_CONTIGUOUS"]
        self.keep.append(a)
        return self.h.fj_array(a.itemsize, a.size, a.ctypes.data)

    def buf(self, a, direct=True):
        self.keep.append(a)
        return self.h.fj_buffer(a.ctypes.data, a.nbytes, 1 if direct else 0)

    def exception(self):
        c, m = ctypes.create_string_buffer(96), ctypes.create_string_buffer(512)
        return (c.value.decode(), m.value.decode()) if self.h.fj_take_exception(c, 96, m, 512) else None

    def expect(self, cls):
        e = self.exception()
        assert e is not None and e[0] == cls, e
        return e[1]

    def clean(self):
        e = self.exception()
        assert e is None, e
        assert self.h.fj_pins_outstanding() == 0


@pytest.fixture(scope="module")
def jni():
    if not os.path.exists(HARNESS):
        pytest.skip("JNI harness not built (python -c 'import __graft_entry__ as g; g.build()')")
    return Jni()


def test_harness_exports_every_native():
    """CPU-side: the harness library exists after build() and exports every RatisHip native."""
    assert os.path.exists(HARNESS), "build() builds tests/jni_harness"
    h = ctypes.CDLL(HARNESS)
    for n in NATIVES:
        assert hasattr(h, "Java_org_apache_ratis_hip_RatisHip_" + n), n


@pytest.mark.gpu
def test_pump_natives_against_direct_calls_and_model(jni, ctx, orc):
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(77)
    cap = 4000
    node_create = jni.fn("nodeCreate0", L, I, L, L)
    node = node_create(1, cap, -1)
    jni.clean()
    assert node
    twin = groups.RaftNode(1, cap)
    model = TableModel(cap)
    try:
        assert jni.fn("nodeShards0", I, L)(node) == 1
        assert jni.fn("shardOf0", I, L, L, I)(123, 456, 8) == groups.shard_of(123, 456, 8)
        start = jni.fn("groupStart0", None, L, I, I, L, L, L)
        slots = np.arange(0, 3000)
        for s in slots:
            w = conf_word(int(rng.integers(1, 1 << 4)) if s % 5 else int(rng.integers(1, 1 << 6)))
            b = int(rng.integers(1 << 20, 1 << 30))
            start(node, int(s), jint(w), b, b - 100, b - 400)
            twin.start(int(s), w, b, b - 100, b - 400)
            model.start(int(s), w, b, b - 100, b - 400)
        jni.clean()
        push = jni.fn("pushDeltas0", None, L, P, I)
        commit_async = jni.fn("commitAsync0", L, L, I, I)
        tick_async = jni.fn("tickAsync0", L, L, I, I)
        commit_wait = jni.fn("commitWait0", L, L, I, L, P, P, P, P)
        watch_async = jni.fn("watchAsync0", None, L, I)
        watch_wait = jni.fn("watchWait0", I, L, I, P, P, P, P, P)
        watch_levels = jni.fn("watchLevels0", I, L, I, P, P, P, P, P)
        a_slot, a_val = np.zeros(cap, np.int32), np.zeros(cap, np.int64)
        w_slot, w_val = np.zeros(cap, np.int32), np.zeros(cap, np.int64)
        l_slot, l_min, l_maj, l_max = (np.zeros(cap, np.int32), np.zeros(cap, np.int64), np.zeros(cap, np.int64),
                                       np.zeros(cap, np.int64))
        l_valid = np.zeros(cap, np.uint8)
        for step in range(4):
            d = random_deltas(rng, model, slots, int(rng.choice([300, 6000])))
            dbuf = np.zeros(d.size + 7, dtype=d.dtype)   # the direct buffer is larger than the deltas
            dbuf[: d.size] = d
            push(node, jni.buf(dbuf.view(np.uint8)), d.size)
            twin.push(d)
            model.apply(d)
            jni.clean()
            if step == 2:   # the pump's call: both evaluations (rh_tick_async)
                tk = tick_async(node, 0, _lib.RH_COMMIT_WATCH_ALL)
            else:
                tk = commit_async(node, 0, _lib.RH_COMMIT_WATCH_ALL)
            tk2 = twin.tables[0].commit_async(watch_all=True)
            if step == 0:
                watch_async(node, 0)
            counts = commit_wait(node, 0, tk, jni.arr(a_slot), jni.arr(a_val), jni.arr(w_slot), jni.arr(w_val))
            jni.clean()
            na, nw = counts >> 32, counts & 0xFFFFFFFF
            got = twin.tables[0].commit_wait(tk2)
            a_s, a_c, ws, wm = model.commit_batch(orc)
            o = np.argsort(a_slot[:na], kind="stable")
            assert np.array_equal(a_slot[:na][o], got.advanced_slots) and np.array_equal(a_val[:na][o], got.advanced_commit)
            assert np.array_equal(a_slot[:na][o].astype(np.int64), a_s) and np.array_equal(a_val[:na][o], a_c)
            o = np.argsort(w_slot[:nw], kind="stable")
            assert np.array_equal(w_slot[:nw][o].astype(np.int64), ws) and np.array_equal(w_val[:nw][o], wm)
            if step % 2 == 0:
                n = watch_wait(node, 0, jni.arr(l_slot), jni.arr(l_min), jni.arr(l_maj), jni.arr(l_max), jni.arr(l_valid))
            else:
                n = watch_levels(node, 0, jni.arr(l_slot), jni.arr(l_min), jni.arr(l_maj), jni.arr(l_max), jni.arr(l_valid))
            jni.clean()
            ev = twin.tables[0].commit_index_changed()
            m_s, m_lev, m_valid = model.watch(orc)
            o = np.argsort(l_slot[:n], kind="stable")
            assert np.array_equal(l_slot[:n][o].astype(np.int64), m_s) and np.array_equal(l_slot[:n][o], ev["slot"])
            assert np.array_equal(l_min[:n][o], m_lev[0]) and np.array_equal(l_maj[:n][o], m_lev[1])
            assert np.array_equal(l_max[:n][o], m_lev[2]) and np.array_equal(l_valid[:n][o].astype(bool), m_valid)
        # leases: leaseStart0 + leaseAsync0 / leaseWait0 and leaseBatchShard0 against the twin
        lease_start = jni.fn("leaseStart0", None, L, I, L, ctypes.c_uint8)
        lease_async = jni.fn("leaseAsync0", None, L, I, L, L)
        lease_wait = jni.fn("leaseWait0", None, L, I, P)
        lease_shard = jni.fn("leaseBatchShard0", None, L, I, L, L, P)
        now = 1 << 50
        for s in slots[::3]:
            lease_start(node, int(s), now, 1)
            twin.lease_start(int(s), now, True)
        jni.clean()
        bits = np.zeros((cap + 63) // 64, np.int64)
        some = []
        for dt, asy in ((50_000_000, True), (150_000_000, False)):
            if asy:
                lease_async(node, 0, now + dt, 100)
                lease_wait(node, 0, jni.arr(bits))
            else:
                lease_shard(node, 0, now + dt, 100, jni.arr(bits))
            jni.clean()
            want = twin.lease_batch(now + dt, 100)
            got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:cap].astype(bool)
            assert np.array_equal(got, want)
            some.append(int(got.sum()))
        assert some[0] > 0 and some[1] == 0   # lease from the start at 50 ms; lapsed, no replies at 150 ms
        # errors: short arrays, superseded tickets, bad slots, heap buffers, unknown sinks
        tk = commit_async(node, 0, _lib.RH_COMMIT_WATCH_ALL)
        d = random_deltas(rng, model, slots, 500)
        model.apply(d)
        commit_wait(node, 0, tk, jni.arr(a_slot), jni.arr(a_val), jni.arr(w_slot), jni.arr(w_val))
        jni.clean()
        push(node, jni.buf(np.ascontiguousarray(d).view(np.uint8)), d.size)
        tk = commit_async(node, 0, _lib.RH_COMMIT_WATCH_ALL)
        short = np.zeros(1, np.int32)
        commit_wait(node, 0, tk, jni.arr(short), jni.arr(a_val), jni.arr(w_slot), jni.arr(w_val))
        assert "shorter" in jni.expect(IAE)
        commit_wait(node, 0, tk - 3, jni.arr(a_slot), jni.arr(a_val), jni.arr(w_slot), jni.arr(w_val))
        jni.expect(IOE)                                          # RH_E_STATE: superseded ticket
        start(node, cap + 5, jint(conf_word(1)), 1, 1, 1)
        jni.expect(IAE)                                          # RH_E_INVAL: node slot out of range
        push(node, jni.buf(np.ascontiguousarray(d).view(np.uint8), direct=False), d.size)
        assert "direct" in jni.expect(IAE)                       # a heap buffer has no address
        push(node, jni.buf(np.ascontiguousarray(d[:2]).view(np.uint8)), 5)
        jni.expect(IAE)                                          # n beyond the buffer's capacity
        jni.fn("setEventSink0", None, L, I, I)(node, 0, 9)
        jni.expect(IAE)
        watch_wait(node, 0, jni.arr(l_slot), jni.arr(l_min), jni.arr(l_maj), jni.arr(l_max), jni.arr(l_valid))
        jni.expect(IOE)                                          # nothing in flight: RH_E_STATE
        lease_wait(node, 0, jni.arr(np.zeros(1, np.int64)))
        jni.expect(IOE)
        assert jni.h.fj_pins_outstanding() == 0
    finally:
        jni.fn("nodeDestroy0", None, L)(node)
        jni.clean()
        twin.close()


@pytest.mark.gpu
def test_log_reader_and_writer_natives(jni, ctx, orc):
    """readSegments0 (HipLogReader), verifyHost0 (RatisHip.verifyFrames, with a non-zero buffer
    position), stampHost0 / hostRegister0 (HipFrameStamper) against the library and the oracle."""
    from ratis_amd import engine, segment
    rng = np.random.default_rng(3)
    ctx_create = jni.fn("ctxCreate0", L, I)
    h = ctx_create(0)
    jni.clean()
    try:
        # three segment files of entries, one corrupted, in one image (256-byte aligned starts)
        files, offs = [], []
        for k in range(3):
            protos = segment.simple_operation_entries(int(rng.integers(50, 400)), term=k + 1)
            img, fo0, fl0 = segment.build_segment(protos)
            crc0, _ = orc.crc32c_frames(img, fo0, fl0)   # the writer's trailers (OUT:100-107)
            for o, l, c in zip(fo0.astype(np.int64), fl0.astype(np.int64), crc0):
                img[o + l - 4: o + l] = np.frombuffer(int(c).to_bytes(4, "big"), np.uint8)
            if k == 1:
                img[len(img) // 2] ^= 0x40
            files.append(np.concatenate([img, np.zeros(int(rng.integers(0, 300)), np.uint8)]))
        pos = 0
        for f in files:
            offs.append(pos)
            pos += (f.size + 255) // 256 * 256
        image = np.zeros(pos, np.uint8)
        for o, f in zip(offs, files):
            image[o: o + f.size] = f
        so, sl = np.array(offs, np.int64), np.array([f.size for f in files], np.int64)
        capf = 512
        fo, fl, fc = np.zeros(3 * capf, np.int64), np.zeros(3 * capf, np.int32), np.zeros(3 * capf, np.int32)
        si, sg = np.zeros(9, np.int32), np.zeros(6, np.int64)
        read = jni.fn("readSegments0", L, L, P, L, P, P, I, I, I, P, P, P, P, P)
        total = read(h, jni.buf(image), image.size, jni.arr(so), jni.arr(sl), 3, 4 << 20, capf, jni.arr(fo),
                     jni.arr(fl), jni.arr(fc), jni.arr(si), jni.arr(sg))
        jni.clean()
        want = engine.read_segments_host(ctx, image, so, sl, frames_per_seg_cap=capf)
        assert total == want["total"]
        assert np.array_equal(si[0::3], want["status"]) and np.array_equal(si[1::3], want["n_ok"])
        assert np.array_equal(si[2::3], want["n_frames"]) and np.array_equal(sg[0::2], want["stop"])
        assert np.array_equal(fo[:total], want["frame_off"]) and np.array_equal(fc[:total].view(np.uint32), want["frame_crc"])
        for k, f in enumerate(files):                             # the reader's verdict per file
            ro, _, _, rst, rstop = orc.segment_scan(f)
            assert (int(sg[2 * k]), int(si[3 * k + 1])) == (rstop, len(ro)) or si[3 * k] == -2
        read(h, jni.buf(image), image.size, jni.arr(so), jni.arr(sl), 3, 4 << 20, capf, jni.arr(fo), jni.arr(fl),
             jni.arr(fc), jni.arr(si[:8]), jni.arr(sg))
        assert "segInts" in jni.expect(IAE)
        # verifyHost0 over the first file's frames at a non-zero buffer position
        node = jni.fn("nodeCreate0", L, I, L, L)(1, 16, -1)
        jni.clean()
        try:
            lead = 777
            seg = files[0]
            n0 = int(want["n_frames"][0])
            off = want["frame_off"][:n0].astype(np.int64)
            ln = want["frame_len"][:n0].astype(np.int32)
            bufm = np.concatenate([rng.integers(0, 256, lead, dtype=np.uint8), seg])
            crc = np.zeros(n0, np.int32)
            bad = np.zeros((n0 + 63) // 64, np.int64)
            verify = jni.fn("verifyHost0", L, L, I, P, L, L, P, P, I, P, P)
            nb = verify(node, 0, jni.buf(bufm), lead, seg.size, jni.arr(off), jni.arr(ln), n0, jni.arr(crc), jni.arr(bad))
            jni.clean()
            ref, nbad = orc.crc32c_frames(seg, off.astype(np.uint64), ln.astype(np.uint32))
            assert nb == nbad == 0 and np.array_equal(crc.view(np.uint32), ref)
            verify(node, 0, jni.buf(bufm), lead + 1, seg.size, jni.arr(off), jni.arr(ln), n0, jni.arr(crc), jni.arr(bad))
            assert "outside" in jni.expect(IAE)                  # [position, limit) beyond the buffer
            verify(node, 0, jni.buf(bufm), lead, seg.size, jni.arr(off), jni.arr(ln[:3]), n0, jni.arr(crc), jni.arr(bad))
            jni.expect(IAE)                                      # frameLen shorter than n
        finally:
            jni.fn("nodeDestroy0", None, L)(node)
            jni.clean()
        # stampHost0 from a registered buffer: the oracle writer's bytes
        protos = [rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes() for _ in range(300)]
        frames = [orc.frame_write(p) for p in protos]
        wantb = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
        off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.int64)
        ln = np.array([len(f) for f in frames], np.int32)
        wb = np.zeros(wantb.size + 4096, np.uint8)
        wb[: wantb.size] = wantb
        for o, l in zip(off, ln):
            wb[o + l - 4: o + l] = 0
        jbuf = jni.buf(wb)
        jni.fn("hostRegister0", None, L, P)(h, jbuf)
        jni.clean()
        jni.fn("stampHost0", None, L, P, L, P, P, I)(h, jbuf, wantb.size, jni.arr(off), jni.arr(ln), ln.size)
        jni.clean()
        assert np.array_equal(wb[: wantb.size], wantb)
        jni.fn("stampHost0", None, L, P, L, P, P, I)(h, jbuf, wantb.size - 1, jni.arr(off), jni.arr(ln), ln.size)
        jni.expect(IAE)                                          # the last frame ends past bufLen
        jni.fn("hostUnregister0", None, L, P)(h, jbuf)
        jni.clean()
    finally:
        jni.fn("ctxDestroy0", None, L)(h)
        jni.clean()
