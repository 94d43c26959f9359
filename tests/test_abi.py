"""CPU tests of the C-ABI boundary: the library loads, exports every function include/ratis_hip.h
declares, and the ctypes mirrors of the C structs have the C layout (no compute calls)."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ratis_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s+\**\s*(rh_[a-z0-9_]+)\s*\(", src, flags=re.M)
    inline = set(re.findall(r"static\s+inline\s+\w+\s+(rh_[a-z0-9_]+)\s*\(", src))
    return sorted(set(names) - inline)


def test_header_parses_into_function_list():
    names = declared_functions()
    for must in ("rh_init", "rh_commit_soa_launch", "rh_crc32c_frames_launch", "rh_push_deltas",
                 "rh_commit_batch", "rh_commit_batch_async", "rh_group_reconf", "rh_node_create",
                 "rh_crc32c_verify_host"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from ratis_amd import _lib
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes table covers exactly the declared surface
    assert sorted(_lib.exported_symbols()) == declared_functions()


def test_abi_version_and_error_slot():
    from ratis_amd import _lib
    lib = _lib.load()
    assert lib.rh_abi_version() == 1
    assert isinstance(lib.rh_last_error(), bytes)


def test_invalid_arguments_fail_without_gpu():
    """Argument validation happens before any device call (no GPU needed)."""
    from ratis_amd import _lib
    lib = _lib.load()
    assert lib.rh_commit_soa_launch(None, None, 1, None) == _lib.RH_E_INVAL
    assert b"ctx" in lib.rh_last_error()
    assert lib.rh_groups_create(None, 10, -1, None) == _lib.RH_E_INVAL
    assert lib.rh_node_create(0, 10, -1, None) == _lib.RH_E_INVAL
    assert lib.rh_commit_batch(None, 0, None) == _lib.RH_E_INVAL
    assert lib.rh_push_deltas(None, None, 0) == _lib.RH_E_INVAL
    assert lib.rh_crc32c_frames_launch(None, None, 0, None) == _lib.RH_E_INVAL
    with pytest.raises(_lib.IllegalArgumentError):
        _lib.check(lib.rh_lease_soa_launch(None, None, 1, None))


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "ratis_hip.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("rh_commit_soa %zu\n", sizeof(rh_commit_soa));
  printf("rh_frames %zu\n", sizeof(rh_frames));
  printf("rh_delta %zu\n", sizeof(rh_delta));
  printf("rh_index_event %zu\n", sizeof(rh_index_event));
  printf("rh_watch_event %zu\n", sizeof(rh_watch_event));
  printf("rh_commit_out %zu\n", sizeof(rh_commit_out));
  F(rh_index_event, slot) F(rh_index_event, reserved) F(rh_index_event, value)
  F(rh_watch_event, slot) F(rh_watch_event, valid) F(rh_watch_event, min) F(rh_watch_event, majority)
  F(rh_watch_event, max)
  F(rh_commit_out, advanced) F(rh_commit_out, n_advanced) F(rh_commit_out, watch_all) F(rh_commit_out, n_watch_all)
  printf("rh_segments %zu\n", sizeof(rh_segments));
  printf("rh_lease_soa %zu\n", sizeof(rh_lease_soa));
  printf("rh_segments_crc %zu\n", sizeof(rh_segments_crc));
  F(rh_segments_crc, scratch_crc) F(rh_segments_crc, seg_ok) F(rh_segments_crc, seg_read_status)
  F(rh_segments_crc, seg_read_stop) F(rh_segments_crc, crc_out) F(rh_segments_crc, bad_bits) F(rh_segments_crc, n_bad)
  F(rh_commit_soa, n) F(rh_commit_soa, n_followers) F(rh_commit_soa, mode) F(rh_commit_soa, gap_threshold)
  F(rh_commit_soa, follower_index) F(rh_commit_soa, col_stride) F(rh_commit_soa, self_index)
  F(rh_commit_soa, commit_in) F(rh_commit_soa, term_start) F(rh_commit_soa, conf) F(rh_commit_soa, commit_out)
  F(rh_commit_soa, min_out) F(rh_commit_soa, maj_out) F(rh_commit_soa, max_out) F(rh_commit_soa, valid_bits)
  F(rh_commit_soa, advanced_bits) F(rh_commit_soa, adv_rows) F(rh_commit_soa, adv_commit)
  F(rh_commit_soa, adv_count) F(rh_commit_soa, adv_cap) F(rh_commit_soa, adv_row_base)
  F(rh_commit_soa, tile_stride)
  F(rh_frames, buf) F(rh_frames, buf_len) F(rh_frames, frame_off) F(rh_frames, frame_len) F(rh_frames, n)
  F(rh_frames, init_state) F(rh_frames, reserved) F(rh_frames, crc_out) F(rh_frames, bad_bits) F(rh_frames, n_bad)
  F(rh_delta, slot) F(rh_delta, column) F(rh_delta, op) F(rh_delta, reserved) F(rh_delta, value)
  F(rh_segments, buf) F(rh_segments, buf_len) F(rh_segments, seg_off) F(rh_segments, seg_len)
  F(rh_segments, n_seg) F(rh_segments, max_op) F(rh_segments, frames_per_seg_cap) F(rh_segments, scratch_off)
  F(rh_segments, scratch_len) F(rh_segments, frame_off) F(rh_segments, frame_len) F(rh_segments, frame_cap)
  F(rh_segments, seg_first) F(rh_segments, seg_nframes) F(rh_segments, seg_status) F(rh_segments, seg_stop)
  F(rh_segments, total_frames)
  F(rh_lease_soa, n) F(rh_lease_soa, n_followers) F(rh_lease_soa, reserved) F(rh_lease_soa, now_nanos)
  F(rh_lease_soa, timeout_ms) F(rh_lease_soa, follower_ts) F(rh_lease_soa, col_stride) F(rh_lease_soa, conf)
  F(rh_lease_soa, lease_in) F(rh_lease_soa, enabled_bits) F(rh_lease_soa, lease_out)
  F(rh_lease_soa, has_lease_bits) F(rh_lease_soa, extended_bits) F(rh_lease_soa, tile_stride)
  printf("rh_segment_result %zu\n", sizeof(rh_segment_result));
  F(rh_segment_result, status) F(rh_segment_result, n_ok) F(rh_segment_result, stop)
  F(rh_segment_result, first_frame) F(rh_segment_result, n_frames) F(rh_segment_result, reserved)
  printf("conf %u\n", rh_conf_pack(0x5, 1, 1, 0x3, 1, 1));
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    from ratis_amd import _lib
    src = tmp_path / "layout.c"
    src.write_text(C_LAYOUT)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    vals = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    assert int(vals["rh_commit_soa"]) == ctypes.sizeof(_lib.RhCommitSoa)
    assert int(vals["rh_frames"]) == ctypes.sizeof(_lib.RhFrames)
    assert int(vals["rh_delta"]) == ctypes.sizeof(_lib.RhDelta)
    assert int(vals["rh_segments"]) == ctypes.sizeof(_lib.RhSegments)
    assert int(vals["rh_lease_soa"]) == ctypes.sizeof(_lib.RhLeaseSoa)
    assert int(vals["rh_segments_crc"]) == ctypes.sizeof(_lib.RhSegmentsCrc)
    assert int(vals["rh_segment_result"]) == ctypes.sizeof(_lib.RhSegmentResult) == 32
    assert int(vals["rh_delta"]) == 16 and int(vals["rh_index_event"]) == 16 and int(vals["rh_watch_event"]) == 32
    from ratis_amd import groups
    assert groups.DELTA_DTYPE.itemsize == 16 and groups.INDEX_EVENT_DTYPE.itemsize == 16
    assert groups.WATCH_EVENT_DTYPE.itemsize == 32
    for cname, cls in (("rh_commit_soa", _lib.RhCommitSoa), ("rh_frames", _lib.RhFrames), ("rh_delta", _lib.RhDelta),
                       ("rh_segments", _lib.RhSegments), ("rh_lease_soa", _lib.RhLeaseSoa),
                       ("rh_segments_crc", _lib.RhSegmentsCrc), ("rh_index_event", _lib.RhIndexEvent),
                       ("rh_watch_event", _lib.RhWatchEvent), ("rh_commit_out", _lib.RhCommitOut),
                       ("rh_segment_result", _lib.RhSegmentResult)):
        for fname, _ in cls._fields_:
            assert int(vals[f"{cname}.{fname}"]) == getattr(cls, fname).offset, (cname, fname)
    assert int(vals["conf"]) == _lib.conf_pack(0x5, True, True, 0x3, True, True)


def test_host_crc32c_update_matches_the_oracle(orc):
    """rh_crc32c_update (SURVEY 8(b)'s pure host rh_crc32c: Checksum.update on PureJavaCrc32C's
    internal state) against the oracle's PJC restatement: RFC 3720 answers through getValue(),
    chained updates over every alignment and span length near the 8-byte steps, and the NULL /
    empty spans.  A host function: runs here, without a GPU."""
    import json

    import numpy as np

    from ratis_amd import engine
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "crc_reference.json")))
    for v in ref["rfc3720"]:
        st = engine.crc32c_update_host(0xFFFFFFFF, bytes.fromhex(v["hex"]))
        assert (~st) & 0xFFFFFFFF == int(v["crc"], 16), v["name"]
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=5000, dtype=np.uint8).tobytes()
    for a in range(0, 17):
        for n in (0, 1, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1000):
            st0 = int(rng.integers(0, 1 << 32))
            assert engine.crc32c_update_host(st0, data[a:a + n]) == orc.crc32c_update(st0, data[a:a + n]), (a, n)
    st = 0xFFFFFFFF
    for a, b in ((0, 3), (3, 11), (11, 4000), (4000, 5000)):
        st = engine.crc32c_update_host(st, data[a:b])
    assert (~st) & 0xFFFFFFFF == orc.crc32c(data)
    from ratis_amd import _lib
    assert _lib.load().rh_crc32c_update(0x1234, None, 10) == 0x1234
