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
    for m in re.finditer(r"private static native (\S+) (\w+)\(([^)]*)\)", src, re.S):
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
