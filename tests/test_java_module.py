"""The Java side of the drop-in (java/ratis-hip, java/patches): checked without a JDK.

* ratis_hip_jni.c is type-checked by gcc against include/ratis_hip.h (and a test-only subset of
  jni.h), so every call into the C ABI matches its prototype;
* every `native` method of RatisHip.java has a JNI function of the same name and parameter types;
* the seams patch applies cleanly to the reference files it edits (when /root/reference exists), and
  the LeaderStateImpl seams only call methods HipLeaderBookkeeper.Division defines.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "ratis-hip", "src", "main")
JNI_C = os.path.join(JAVA, "native", "ratis_hip_jni.c")
RATIS_HIP_JAVA = os.path.join(JAVA, "java", "org", "apache", "ratis", "hip", "RatisHip.java")
BOOKKEEPER_JAVA = os.path.join(JAVA, "java", "org", "apache", "ratis", "hip", "HipLeaderBookkeeper.java")
PATCH = os.path.join(ROOT, "java", "patches", "0001-ratis-hip-backend-switch-and-seams.patch")
REFERENCE = "/root/reference"

JAVA_TO_JNI = {
    "int": "jint", "long": "jlong", "boolean": "jboolean", "void": "void",
    "int[]": "jintArray", "long[]": "jlongArray", "byte[]": "jbyteArray", "boolean[]": "jbooleanArray",
    "ByteBuffer": "jobject",
}


def _java_natives():
    src = open(RATIS_HIP_JAVA).read()
    out = {}
    for m in re.finditer(r"(?:private )?static native (\S+) (\w+)\(([^)]*)\)", src, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = [" ".join(p.split()[:-1]) for p in params.split(",") if p.strip()]
        out[name] = (JAVA_TO_JNI[ret], [JAVA_TO_JNI[t] for t in types])
    return out


def _c_natives():
    src = open(JNI_C).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT (\w+) JNICALL CLS\((\w+)\)\(JNIEnv\* env, jclass c((?:,[^)]*)?)\)", src, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = [p.split()[0] for p in params.split(",") if p.strip()]
        out[name] = (ret, types)
    return out


def test_jni_source_typechecks_against_abi_header():
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    r = subprocess.run([cc, "-std=c11", "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-parameter",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"), JNI_C],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_method_is_implemented_with_matching_types():
    java, c = _java_natives(), _c_natives()
    assert java, "no native methods parsed"
    assert set(java) == set(c), (set(java) ^ set(c))
    for name, sig in java.items():
        assert c[name] == sig, (name, sig, c[name])


def test_seams_call_only_division_methods():
    patch = open(PATCH).read()
    book = open(BOOKKEEPER_JAVA).read()
    division = book[book.index("public final class Division"):]
    methods = {m.group(1): len([p for p in m.group(2).split(",") if p.strip()])
               for m in re.finditer(r"public (?:synchronized )?\w+ (\w+)\(([^)]*)\)", division)}
    added = "\n".join(l for l in patch.splitlines() if l.startswith("+") and not l.startswith("+++"))
    called = set(re.findall(r"(?<![.\w])hip\.(\w+)\(", added))
    assert called, "no seam calls found"
    assert called <= set(methods), called - set(methods)
    assert methods["reconf"] == 1   # LeaderStateImpl passes only the new membership word


def test_seams_patch_applies_to_reference(tmp_path):
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference tree not present")
    files = re.findall(r"^diff --git a/(\S+) b/", open(PATCH).read(), re.M)
    assert "ratis-server/src/main/java/org/apache/ratis/server/impl/LeaderStateImpl.java" in files
    assert "ratis-server-api/src/main/java/org/apache/ratis/server/RaftServerConfigKeys.java" in files
    for f in files:   # copies only: the reference tree stays untouched
        dst = tmp_path / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(os.path.join(REFERENCE, f), dst)
    r = subprocess.run(["git", "apply", "--check", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _method_body(src: str, signature: str) -> str:
    """The text of a Java method body from `signature` to its matching closing brace."""
    i = src.index(signature)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError("unbalanced braces after " + signature)


def test_pump_runs_watch_levels_and_watch_all_without_allocating():
    """commitIndexChanged (LeaderStateImpl.java:606-622) and updateCommit's watch ALL (:1025) in HIP
    mode: every tick evaluates with RH_COMMIT_WATCH_ALL, puts every shard's commit, watch and lease
    passes in flight before any wait (rh_tick_async: commit + watch in one call; rh_lease_batch_async),
    waits them per shard, and allocates nothing (result arrays sized once per shard capacity)."""
    book = open(BOOKKEEPER_JAVA).read()
    tick = _method_body(book, "void tick()")
    assert "hip.tickAsync(s, RatisHip.COMMIT_WATCH_ALL)" in tick
    assert "hip.commitWait(" in tick and "hip.watchWait(" in tick and "hip.leaseWait(" in tick
    assert "onWatchLevels(" in tick and "onWatchAll(" in tick and "onCommit(" in tick
    assert not re.search(r"\bnew\b", tick), "tick() allocates"
    assert "capacity * hip.getShards()" not in book and "capacity * shards" not in book
    # every shard's three passes are issued in the first loop, before the first wait
    first_wait = tick.index("hip.commitWait(")
    for call in ("hip.tickAsync(", "hip.leaseAsync("):
        assert tick.index(call) < first_wait, call
    assert "hip.watchLevels(" not in tick and "hip.leaseBatch(" not in tick


def test_seams_implement_every_callback_and_the_checksum_backend():
    book = open(BOOKKEEPER_JAVA).read()
    iface = _method_body(book, "public interface Callback")
    callbacks = set(re.findall(r"void (\w+)\(", iface))
    assert callbacks == {"onCommit", "onWatchAll", "onWatchLevels", "onFallback"}
    patch = open(PATCH).read()
    added = "\n".join(l[1:] for l in patch.splitlines() if l.startswith("+") and not l.startswith("+++"))
    cb = _method_body(added, "private final class HipCallback implements HipLeaderBookkeeper.Callback")
    assert set(re.findall(r"public void (\w+)\(", cb)) == callbacks
    handler = _method_body(added, "private void updateFromHip()")
    for level in ("ALL,", "ALL_COMMITTED,", "MAJORITY_COMMITTED,", "MAJORITY,"):
        assert f"ReplicationLevel.{level}" in handler, level
    assert "notifySenders()" in handler
    # the checksum backend: SegmentedRaftLog's bulk load goes through the GPU read path and
    # LogSegment parses the verified entries, raising the reader's exceptions
    assert "HipLogReader.get(hipDeviceMask)" in added and "cache.loadSegment(pi, keepEntryInCache, logConsumer, v)" in added
    reader = _method_body(added, "static int readSegmentFileHip(")
    assert "verified.entryBytes(k)" in reader and "throwReaderFailure(file, verified)" in reader
    failure = _method_body(added, "private static void throwReaderFailure(")
    assert "new ChecksumException(" in failure and "new CorruptedFileException(" in failure


def test_log_reader_native_matches_the_abi():
    """HipLogReader's native (readSegments0) packs rh_segment_result as the header defines it."""
    jni = open(JNI_C).read()
    body = jni[jni.index("CLS(readSegments0)"):]
    assert "rh_segments_read_host(" in body
    for f in ("status", "n_ok", "n_frames", "stop", "first_frame"):
        assert f"res[s].{f}" in body, f
    hdr = open(os.path.join(ROOT, "include", "ratis_hip.h")).read()
    assert "int rh_segments_read_host(" in hdr


def _patched_java(path_suffix: str) -> str:
    """The reference file as the seams patch leaves it (requires /root/reference)."""
    import tempfile
    files = re.findall(r"^diff --git a/(\S+) b/", open(PATCH).read(), re.M)
    f = next(x for x in files if x.endswith(path_suffix))
    with tempfile.TemporaryDirectory() as d:
        dst = os.path.join(d, f)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(os.path.join(REFERENCE, f), dst)
        r = subprocess.run(["git", "apply", "--include", f, PATCH], cwd=d, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        return open(dst).read()


def _added_lines() -> str:
    patch = open(PATCH).read()
    return "\n".join(l[1:] for l in patch.splitlines() if l.startswith("+") and not l.startswith("+++"))


def test_fallback_replaces_every_membership_failure():
    """HIP mode never fails a leader for what the GPU table cannot hold (fall back to
    the CPU path and count it): no seam throws for membership size, the bookkeeper counts fallbacks
    by reason, a 15th follower / full shard / rejected or failed control call / dead pump each put
    the division in fallback, and the division then answers through the reference's path."""
    book = open(BOOKKEEPER_JAVA).read()
    added = _added_lines()
    # no seam turns a library rejection into an exception any more
    assert "ratis-hip start failed" not in added and "ratis-hip reconf failed" not in added
    assert "more than \" + RatisHip.MAX_FOLLOWERS" not in book
    assert not re.search(r"throw new IllegalStateException\(\"ratis-hip: (shard|more than)", book)
    # the stat and its reasons
    assert "public long getFallbackCount()" in book and "public long getFallbackCount(FallbackReason reason)" in book
    reasons = set(re.findall(r"FallbackReason\.(\w+)", book))
    assert reasons >= {"SHARD_FULL", "FOLLOWER_SLOTS", "REJECTED", "DEVICE_ERROR", "PUMP_FAILED"}, reasons
    add = _method_body(book, "public synchronized int addFollower(")
    assert "fallBack(FallbackReason.FOLLOWER_SLOTS)" in add and "return -1;" in add
    reg = _method_body(book, "public synchronized Division register(")
    assert "FallbackReason.SHARD_FULL" in reg and "throw" not in reg
    for m in ("public void start(", "public void reconf(", "public void leaseStart("):
        body = _method_body(book, m)
        assert "FallbackReason.REJECTED" in body and "FallbackReason.DEVICE_ERROR" in body, m
        assert "catch (IllegalArgumentException" in body, m
    pump = _method_body(book, "private void pumpLoop()")
    assert "d.fallBack(FallbackReason.PUMP_FAILED)" in pump
    fb = _method_body(book, "void fallBack(FallbackReason reason)")
    assert "callback.onFallback()" in fb and "hip.stop(nodeSlot)" in fb and "release(this)" in fb
    # producers ignore a follower without a slot
    for m in ("public void matchIndex(", "public void snapshotIndex(", "public void followerCommitIndex(",
              "public void lastResponded("):
        assert "followerSlot >= 0" in _method_body(book, m), m
    assert "fallback" in _method_body(book, "public boolean hasLease()")
    # the seams: every HIP branch of LeaderStateImpl is taken only while the division is active
    assert "private boolean hipActive()" in added
    assert "return hip != null && !hip.isFallback();" in added
    branches = re.findall(r"if \((hip != null|hipActive\(\))[^)]*\)", added)
    null_only = [b for b in re.findall(r"if \(hip != null\)", added)]
    # `hip != null` remains only where fallback does not matter: start (a fallen-back division
    # ignores it), stop / removeFollower (harmless), and the UPDATE_COMMIT handler (applies GPU decisions)
    assert len(null_only) <= 4, null_only
    assert sum(1 for b in branches if b == "hipActive()") >= 10
    cb = _method_body(added, "public void onFallback()")
    assert "eventQueue.submit(updateCommitEvent)" in cb and "commitIndexChanged()" in cb


def test_hip_mode_does_not_rerun_the_java_arithmetic():
    """In HIP mode LeaderStateImpl no longer evaluates getMajorityMin in Java: updateCommit's
    follow-up runs notifySenders() instead of commitIndexChanged() (LeaderStateImpl.java:1009), and
    checkStaging marks the division for the GPU instead of executing updateCommit (:866); the
    UPDATE_COMMIT event runs the Java updateCommit() only in JAVA mode or after a fallback."""
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference tree not present")
    src = _patched_java("server/impl/LeaderStateImpl.java")
    assert "new StateUpdateEvent(StateUpdateEvent.Type.UPDATE_COMMIT, this::onUpdateCommitEvent)" in src
    assert "hipUpdateEvent" not in src
    handler = _method_body(src, "private void onUpdateCommitEvent()")
    assert "updateFromHip();" in handler and "if (!hipActive())" in handler and "updateCommit();" in handler
    follow = _method_body(src, "private void updateCommit(LogEntryHeader[] entriesToCommit)")
    i = follow.index("if (hipActive())")
    assert follow.index("notifySenders();", i) < follow.index("commitIndexChanged();", i)
    staging = _method_body(src, "private void checkStaging()")
    i = staging.index("if (hipActive())")
    assert staging.index("submitUpdateCommitEvent();", i) < staging.index("updateCommitEvent.execute();", i)
    # the only Java getMajorityMin callers left run in JAVA mode / fallback
    assert _method_body(src, "private void onUpdateCommitEvent()").count("updateCommit()") == 1


def test_bulk_load_streams_batches_with_two_images():
    """SegmentedRaftLog.loadLogSegments no longer materialises every batch before loading: it takes
    segments one by one from a HipLogReader.Pipeline (batch k + 1 read and verified while batch k
    loads), which holds exactly two image buffers and hands a batch's back after its last segment;
    batches are planned under HIP_BATCH_BYTES and MAX_FRAMES_PER_BATCH frame slots (no silent
    clamp of the frame table).  A failure to create the pipeline or of one of its batches falls back
    to the reference's reader for the remaining segments."""
    added = _added_lines()
    assert "List<HipLogReader.Segment>" not in added
    assert "HipLogReader.Pipeline verified = null;" in added and "v = verified.next();" in added
    # a GPU that fails never fails the load: the rest is read by the reference's reader
    assert "verified = hipVerify(paths);" in added and "closeQuietly(verified);" in added
    assert added.count("} catch (IOException | RuntimeException e) {") >= 2
    plan = _method_body(added, "private HipLogReader.Pipeline hipVerify(")
    assert "HipLogReader.MAX_FRAMES_PER_BATCH" in plan and "new HipLogReader.Plan(" in plan
    assert "reader.pipeline(plans, maxOp)" in plan
    reader = open(os.path.join(JAVA, "java", "org", "apache", "ratis", "hip", "HipLogReader.java")).read()
    pipe = _method_body(reader, "Pipeline(List<Plan> plans, int maxOpSize)")
    assert pipe.count("free.add(ByteBuffer.allocateDirect(bytes))") == 2
    assert "free.take()" in pipe and "ready.put(readInto(buf," in pipe
    nxt = _method_body(reader, "public Segment next()")
    assert "free.offer(current.image)" in nxt
    assert "Integer.MAX_VALUE - 8" not in reader          # the old silent clamp
    assert "MAX_FRAMES_PER_BATCH" in _method_body(reader, "public Plan(List<File> files, int framesPerFile)")
    # one context per GPU of the mask, batches spread round robin
    assert "RatisHip.ctxCreate0(d)" in reader and "Math.floorMod(ctxIndex, ctx.length)" in reader


def test_writer_seam_stamps_flush_batches():
    """The write side (north_star: the PureJavaCrc32C/Checksum call sites): in
    HIP checksum mode SegmentedRaftLogOutputStream.write (OUT:86-110) leaves a placeholder trailer
    and records the frame; BufferedWriteChannel.flushBuffer stamps every pending trailer just before
    the buffer goes to the file -- on the GPU from the measured crossover (bench.py write_stamp leg,
    HipFrameStamper.DEFAULT_MIN_GPU_BYTES, the config key's default), else PureJavaCrc32C per frame;
    the worker registers its write buffer once and unregisters it before freeing it."""
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference tree not present")
    chan = _patched_java("segmented/BufferedWriteChannel.java")
    flush = _method_body(chan, "private void flushBuffer()")
    assert flush.index("beforeFlush.accept(writeBuffer)") < flush.index("writeBuffer.flip()")
    outs = _patched_java("segmented/SegmentedRaftLogOutputStream.java")
    write = _method_body(outs, "public void write(LogEntryProto entry)")
    i = write.index("if (stamper != null)")
    assert "buf.putInt(0);" in write[i:] and "stamper.add(pos, total);" in write[i:]
    assert "checksum.update(duplicated);" in write   # the reference path stays for JAVA mode
    assert "out.setBeforeFlush(buf -> stamper.stamp(buf, frame -> {" in outs
    worker = _patched_java("segmented/SegmentedRaftLogWorker.java")
    assert "this.hipStamper = newHipStamper(properties, writeBuffer);" in worker
    assert "preallocatedSize, writeBuffer, hipStamper);" in worker
    close = _method_body(worker, "void close()")
    assert close.index("IOUtils.cleanup(LOG, hipStamper)") < close.index("PlatformDependent.freeDirectBuffer(writeBuffer)")
    keys = _patched_java("server/RaftServerConfigKeys.java")
    assert 'CHECKSUM_GPU_MIN_BYTES_DEFAULT = SizeInBytes.valueOf("64KB")' in keys
    stamper = open(os.path.join(JAVA, "java", "org", "apache", "ratis", "hip", "HipFrameStamper.java")).read()
    assert "DEFAULT_MIN_GPU_BYTES = 64 << 10" in stamper
    st = _method_body(stamper, "public boolean stamp(ByteBuffer buf, FrameChecksum cpu)")
    assert "bytes >= minGpuBytes" in st and "gpu.stampFrames(buf, buf.position(), off, len, n)" in st
    assert "cpu.crc(d)" in st
    # a failing GPU call falls back to the CPU path for the same frames (never fails the flush);
    # the pending frames are dropped only after one path wrote every trailer
    g, c = st.index("gpu.stampFrames("), st.index("cpu.crc(d)")
    assert "catch (IOException | RuntimeException e)" in st[g:c] and "gpuFailures++" in st[g:c]
    assert "finally" not in st and st.rindex("n = 0;") > c
    assert "gpu.register(writeBuffer)" in st   # page-locked lazily, at the first GPU-sized batch
    jni = open(JNI_C).read()
    assert "rh_crc32c_stamp_host(C(ctx)" in jni and "rh_host_register(C(ctx)" in jni


def test_cache_miss_reload_reads_through_the_gpu():
    """Missing item #3 of round 3: a cache miss (LogSegment.LogEntryLoader.load, LogSegment.java:
    265-293) re-reads its segment file. In HIP checksum mode the cache hands every segment it adds
    (addSegment, setOpenSegment) the device mask, and the loader reads the file through
    HipLogReader (framing + every entry's CRC on the GPU) and decodes it with readSegmentFileHip;
    a GPU failure falls back to the reference's readSegmentFile, never fails the read."""
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference tree not present")
    seg = _patched_java("segmented/LogSegment.java")
    load = _method_body(seg, "public LogEntryProto load(LogRecord key)")
    i = load.index("hipDeviceMask != 0 ? hipReload(file, startEnd) : null")
    assert load.index("readSegmentFileHip(file, startEnd, getLogCorruptionPolicy(), verified, reload)") > i
    assert "readSegmentFile(file, startEnd, maxOpSize, getLogCorruptionPolicy(), raftLogMetrics, reload)" in load
    rl = _method_body(seg, "private HipLogReader.Segment hipReload(File file, LogSegmentStartEnd startEnd)")
    assert "HipLogReader.get(hipDeviceMask).read(Collections.singletonList(file)" in rl
    assert "HipLogReader.MAX_FRAMES_PER_BATCH" in rl and "return null;" in rl
    cache = _patched_java("segmented/SegmentedRaftLogCache.java")
    assert "RaftServerConfigKeys.Hip.checksumBackend(properties) == RaftServerConfigKeys.Hip.Backend.HIP" in cache
    for m in ("void addSegment(LogSegment segment)", "private void setOpenSegment(LogSegment openSegment)"):
        assert "setHipDeviceMask(hipDeviceMask);" in _method_body(cache, m), m
