"""ctypes binding of libratis_hip.so (include/ratis_hip.h).

The product path is the HIP library: if ``ratis_amd/lib/libratis_hip.so`` is missing this module
raises on import of any compute entry point -- there is no CPU fallback anywhere in
``ratis_amd``.  Structures below mirror the C structs field by field (checked against the
header by ``tests/test_abi.py``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libratis_hip.so")
# A/B builds of the same sources (scripts/ab_build.sh) are loaded by the tuning scripts through
# RATIS_HIP_LIB; the product, tests, smoke() and bench.py use LIB_PATH.
LIB_PATH = os.environ.get("RATIS_HIP_LIB", LIB_PATH)

RH_OK = 0
RH_E_INVAL = -1
RH_E_RANGE = -2
RH_E_DEVICE = -3
RH_E_NOMEM = -4
RH_E_STATE = -5

RH_MAX_FOLLOWERS = 14
RH_CONF_SELF = 1 << 14
RH_CONF_TRANSITIONAL = 1 << 15
RH_CONF_OLD_SHIFT = 16
RH_CONF_SELF_OLD = 1 << 30
RH_CONF_ACTIVE = 1 << 31
RH_MODE_COMMIT = 0
RH_MODE_WATCH = 1
RH_MAX_TIERS = 4

RH_COL_FLUSH = 32
RH_COL_COMMITTED = 33
RH_COL_CONF = 34
RH_COL_TERM_START = 35
RH_COL_LEASE = 36
RH_COL_LEASE_ON = 37


def RH_COL_TS(k: int) -> int:
    return 48 + k
RH_OP_MAX = 0
RH_OP_SET = 1
RH_DELTA_SLOT = 1 << 20
RH_COMMIT_WATCH_ALL = 1
RH_EVENTS_HOST_MAPPED = 0
RH_EVENTS_DEVICE = 1
RH_EVENTS_AUTO = 2

RH_CRC_VERIFY = 1
RH_CRC_STAMP = 2


def rh_col_match(k: int) -> int:
    return k


def rh_col_fcommit(k: int) -> int:
    return 16 + k


def conf_pack(new_mask: int, include_self: bool, transitional: bool, old_mask: int,
              include_self_old: bool, active: bool = True) -> int:
    """Python twin of ``rh_conf_pack`` (ratis_hip.h)."""
    return ((new_mask & 0x3FFF) | (RH_CONF_SELF if include_self else 0)
            | (RH_CONF_TRANSITIONAL if transitional else 0)
            | ((old_mask & 0x3FFF) << RH_CONF_OLD_SHIFT)
            | (RH_CONF_SELF_OLD if include_self_old else 0)
            | (RH_CONF_ACTIVE if active else 0))


class RhCommitSoa(ctypes.Structure):
    _fields_ = [
        ("n", c_uint64),
        ("n_followers", c_uint32),
        ("mode", c_int32),
        ("gap_threshold", c_int64),
        ("follower_index", c_void_p),
        ("col_stride", c_uint64),
        ("self_index", c_void_p),
        ("commit_in", c_void_p),
        ("term_start", c_void_p),
        ("conf", c_void_p),
        ("commit_out", c_void_p),
        ("min_out", c_void_p),
        ("maj_out", c_void_p),
        ("max_out", c_void_p),
        ("valid_bits", c_void_p),
        ("advanced_bits", c_void_p),
        ("adv_rows", c_void_p),
        ("adv_commit", c_void_p),
        ("adv_count", c_void_p),
        ("adv_cap", c_uint64),
        ("adv_row_base", c_uint64),
        ("tile_stride", c_uint64),
    ]


class RhDelta(ctypes.Structure):
    _fields_ = [("slot", c_uint32), ("column", ctypes.c_uint8), ("op", ctypes.c_uint8), ("reserved", ctypes.c_uint16),
                ("value", c_int64)]


class RhIndexEvent(ctypes.Structure):
    _fields_ = [("slot", c_uint32), ("reserved", c_uint32), ("value", c_int64)]


class RhWatchEvent(ctypes.Structure):
    _fields_ = [("slot", c_uint32), ("valid", c_uint32), ("min", c_int64), ("majority", c_int64), ("max", c_int64)]


class RhCommitOut(ctypes.Structure):
    _fields_ = [("advanced", c_void_p), ("n_advanced", c_uint64), ("watch_all", c_void_p), ("n_watch_all", c_uint64)]


class RhFrames(ctypes.Structure):
    _fields_ = [
        ("buf", c_void_p),
        ("buf_len", c_uint64),
        ("frame_off", c_void_p),
        ("frame_len", c_void_p),
        ("n", c_uint64),
        ("init_state", c_uint32),
        ("reserved", c_uint32),
        ("crc_out", c_void_p),
        ("bad_bits", c_void_p),
        ("n_bad", c_void_p),
    ]


class RhLeaseSoa(ctypes.Structure):
    _fields_ = [
        ("n", c_uint64),
        ("n_followers", c_uint32),
        ("reserved", c_uint32),
        ("now_nanos", c_int64),
        ("timeout_ms", c_int64),
        ("follower_ts", c_void_p),
        ("col_stride", c_uint64),
        ("conf", c_void_p),
        ("lease_in", c_void_p),
        ("enabled_bits", c_void_p),
        ("lease_out", c_void_p),
        ("has_lease_bits", c_void_p),
        ("extended_bits", c_void_p),
        ("tile_stride", c_uint64),
    ]


RH_SEG_END = 1
RH_SEG_PARTIAL = 2
RH_SEG_E_OVERSIZE = -1
RH_SEG_E_CHECKSUM = -2
RH_SEG_E_PADDING = -3
RH_SEG_E_VARINT = -4
RH_SEG_E_HEADER = -5
RH_SEG_E_CAPACITY = -6
RH_SEG_E_RANGE = -7


class RhSegments(ctypes.Structure):
    _fields_ = [
        ("buf", c_void_p),
        ("buf_len", c_uint64),
        ("seg_off", c_void_p),
        ("seg_len", c_void_p),
        ("n_seg", c_uint64),
        ("max_op", c_uint32),
        ("frames_per_seg_cap", c_uint32),
        ("scratch_off", c_void_p),
        ("scratch_len", c_void_p),
        ("frame_off", c_void_p),
        ("frame_len", c_void_p),
        ("frame_cap", c_uint64),
        ("seg_first", c_void_p),
        ("seg_nframes", c_void_p),
        ("seg_status", c_void_p),
        ("seg_stop", c_void_p),
        ("total_frames", c_void_p),
    ]


class RhSegmentsCrc(ctypes.Structure):
    _fields_ = [
        ("scratch_crc", c_void_p),
        ("seg_ok", c_void_p),
        ("seg_read_status", c_void_p),
        ("seg_read_stop", c_void_p),
        ("crc_out", c_void_p),
        ("bad_bits", c_void_p),
        ("n_bad", c_void_p),
    ]


class RhSegmentResult(ctypes.Structure):
    _fields_ = [("status", c_int32), ("n_ok", c_uint32), ("stop", c_uint64), ("first_frame", c_uint64),
                ("n_frames", c_uint32), ("reserved", c_uint32)]


# name -> (restype, argtypes); every function declared in include/ratis_hip.h
_SIGNATURES = {
    "rh_abi_version": (c_int, []),
    "rh_last_error": (c_char_p, []),
    "rh_device_count": (c_int, [POINTER(c_int)]),
    "rh_init": (c_int, [c_int, POINTER(c_void_p)]),
    "rh_shutdown": (c_int, [c_void_p]),
    "rh_synchronize": (c_int, [c_void_p]),
    "rh_ctx_stream": (c_void_p, [c_void_p]),
    "rh_commit_soa_launch": (c_int, [c_void_p, POINTER(RhCommitSoa), c_int, c_void_p]),
    "rh_groups_create": (c_int, [c_void_p, c_uint64, c_int64, POINTER(c_void_p)]),
    "rh_groups_destroy": (c_int, [c_void_p]),
    "rh_groups_set_event_sink": (c_int, [c_void_p, c_int]),
    "rh_group_start": (c_int, [c_void_p, c_uint32, c_uint32, c_int64, c_int64, c_int64]),
    "rh_group_reconf": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p]),
    "rh_group_stop": (c_int, [c_void_p, c_uint32]),
    "rh_group_tier": (c_int, [c_void_p, c_uint32, POINTER(c_uint32)]),
    "rh_group_lease_start": (c_int, [c_void_p, c_uint32, c_int64, c_int]),
    "rh_lease_batch": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_void_p), POINTER(c_uint64)]),
    "rh_node_group_lease_start": (c_int, [c_void_p, c_uint32, c_int64, c_int]),
    "rh_node_lease_batch": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_uint64]),
    "rh_groups_load": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "rh_push_deltas": (c_int, [c_void_p, c_void_p, c_size_t]),   # rh_delta*: groups._addr
    "rh_deltas_acquire": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_size_t)]),
    "rh_deltas_submit": (c_int, [c_void_p, c_size_t]),
    "rh_commit_batch": (c_int, [c_void_p, c_uint32, POINTER(RhCommitOut)]),
    "rh_commit_batch_async": (c_int, [c_void_p, c_uint32, POINTER(c_uint64)]),
    "rh_commit_batch_wait": (c_int, [c_void_p, c_uint64, POINTER(RhCommitOut)]),
    "rh_watch_levels": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint64)]),
    "rh_watch_levels_async": (c_int, [c_void_p]),
    "rh_tick_async": (c_int, [c_void_p, c_uint32, POINTER(c_uint64)]),
    "rh_groups_timing": (c_int, [c_void_p, c_int]),
    "rh_groups_last_timing": (c_int, [c_void_p, POINTER(ctypes.c_float), POINTER(c_int)]),
    "rh_groups_last_timing_split": (c_int, [c_void_p, POINTER(ctypes.c_float), POINTER(ctypes.c_float),
                                            POINTER(ctypes.c_float), POINTER(ctypes.c_float), POINTER(c_int)]),
    "rh_pcie_write_probe": (c_int, [c_void_p, c_uint64, c_int, POINTER(ctypes.c_float)]),
    "rh_watch_levels_wait": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint64)]),
    "rh_lease_batch_async": (c_int, [c_void_p, c_int64, c_int64]),
    "rh_lease_batch_wait": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint64)]),
    "rh_node_watch_levels": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "rh_groups_read": (c_int, [c_void_p, c_uint32, c_uint32, ctypes.c_uint8, c_void_p]),
    "rh_shard_of": (c_int, [c_uint64, c_uint64, c_int]),
    "rh_node_create": (c_int, [c_uint32, c_uint64, c_int64, POINTER(c_void_p)]),
    "rh_node_create_devices": (c_int, [POINTER(c_int), c_int, c_uint64, c_int64, POINTER(c_void_p)]),
    "rh_node_destroy": (c_int, [c_void_p]),
    "rh_node_shards": (c_int, [c_void_p]),
    "rh_node_groups": (c_void_p, [c_void_p, c_int]),
    "rh_node_ctx": (c_void_p, [c_void_p, c_int]),
    "rh_node_group_start": (c_int, [c_void_p, c_uint32, c_uint32, c_int64, c_int64, c_int64]),
    "rh_node_group_reconf": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p]),
    "rh_node_group_stop": (c_int, [c_void_p, c_uint32]),
    "rh_node_push_deltas": (c_int, [c_void_p, c_void_p, c_size_t]),   # rh_delta*: groups._addr
    "rh_node_commit_batch": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, POINTER(c_uint64), c_void_p, c_uint64,
                                     POINTER(c_uint64)]),
    "rh_crc32c_frames_launch": (c_int, [c_void_p, POINTER(RhFrames), c_uint32, c_void_p]),
    "rh_crc32c": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, POINTER(c_uint32)]),
    "rh_crc32c_update": (c_uint32, [c_uint32, c_void_p, c_uint64]),
    "rh_crc32c_stamp_host": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64]),
    "rh_host_register": (c_int, [c_void_p, c_void_p, c_uint64]),
    "rh_host_unregister": (c_int, [c_void_p, c_void_p]),
    "rh_crc32c_verify_host": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64, c_void_p,
                                      c_void_p, POINTER(c_uint64)]),
    "rh_lease_soa_launch": (c_int, [c_void_p, POINTER(RhLeaseSoa), c_int, c_void_p]),
    "rh_leader_soa_launch": (c_int, [c_void_p, POINTER(RhCommitSoa), c_int, POINTER(RhLeaseSoa), c_int, c_void_p]),
    "rh_segments_scan_launch": (c_int, [c_void_p, POINTER(RhSegments), c_void_p]),
    "rh_segments_read_launch": (c_int, [c_void_p, POINTER(RhSegments), POINTER(RhSegmentsCrc), c_void_p]),
    "rh_segments_read_host": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64, c_uint32, c_uint32,
                                      c_void_p, c_void_p, c_void_p, c_uint64, POINTER(RhSegmentResult),
                                      POINTER(c_uint64)]),
}


class RatisHipError(RuntimeError):
    """A libratis_hip call returned a negative RH_E_* status."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code


class IllegalArgumentError(RatisHipError, ValueError):
    """RH_E_INVAL / RH_E_RANGE: the Java binding maps these to IllegalArgumentException."""


_lib = None


def load() -> ctypes.CDLL:
    """Loads libratis_hip.so (once).  Raises if the native library has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libratis_hip.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C ratis_amd/csrc). "
            "ratis_amd has no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> int:
    if rc >= 0:
        return rc
    msg = load().rh_last_error()
    msg = msg.decode() if msg else ""
    if rc in (RH_E_INVAL, RH_E_RANGE):
        raise IllegalArgumentError(rc, msg)
    raise RatisHipError(rc, msg)


def exported_symbols() -> list[str]:
    return sorted(_SIGNATURES)
