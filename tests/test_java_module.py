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
    mode: every tick evaluates with RH_COMMIT_WATCH_ALL and runs watchLevels on every shard, and
    allocates nothing (result arrays sized once per shard capacity)."""
    book = open(BOOKKEEPER_JAVA).read()
    tick = _method_body(book, "void tick()")
    assert "hip.commitAsync(s, RatisHip.COMMIT_WATCH_ALL)" in tick
    assert "hip.commitWait(" in tick and "hip.watchLevels(" in tick
    assert "onWatchLevels(" in tick and "onWatchAll(" in tick and "onCommit(" in tick
    assert not re.search(r"\bnew\b", tick), "tick() allocates"
    assert "capacity * hip.getShards()" not in book and "capacity * shards" not in book


def test_seams_implement_every_callback_and_the_checksum_backend():
    book = open(BOOKKEEPER_JAVA).read()
    iface = _method_body(book, "public interface Callback")
    callbacks = set(re.findall(r"void (\w+)\(", iface))
    assert callbacks == {"onCommit", "onWatchAll", "onWatchLevels"}
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
