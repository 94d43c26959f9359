"""SegmentedRaftLog segment images: frame layout and LogEntryProto encoding (host side).

Frame layout (SegmentedRaftLogOutputStream.java:74-110)::

    varint32(n) || LogEntryProto (n bytes) || CRC32C(varint || proto) as big-endian u32

Segment file (SegmentedRaftLogFormat.java:30-80, SegmentedRaftLogOutputStream.java:40-70)::

    "RaftLog1" || frame* || zero padding (preallocation fill / terminator)

The CRC trailer is filled by the GPU (``RH_CRC_STAMP``, the batched write side) -- this module
only lays out bytes.  Protobuf wire encoding follows protobuf 3.25 (shaded in
ratis-thirdparty-misc 1.1.0): fields in field-number order, proto3 defaults omitted.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

HEADER = b"RaftLog1"            # SegmentedRaftLogFormat.java:30-34
TRAILER = 4                     # 4-byte checksum (SegmentedRaftLogOutputStream.java:80-84)
SEGMENT_SIZE_MAX = 32 << 20     # raft.server.log.segment.size.max (RaftServerConfigKeys.java:455-456)
MAX_OP_SIZE = 4 << 20           # raft.server.log.appender.buffer.byte-limit (SegmentedRaftLogCache.java:437)


def varint_size(v: int) -> int:
    """CodedOutputStream.computeUInt32SizeNoTag / computeUInt64SizeNoTag."""
    n = 1
    while v >= 0x80:
        v >>= 7
        n += 1
    return n


def varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field_varint(num: int, v: int) -> bytes:
    return b"" if v == 0 else varint(num << 3) + varint(v)


def _field_bytes(num: int, b: Optional[bytes]) -> bytes:
    return b"" if not b else varint((num << 3) | 2) + varint(len(b)) + b


def state_machine_log_entry(log_data: bytes = b"", sm_data: Optional[bytes] = None, sm_type: int = 0,
                            client_id: Optional[bytes] = None, call_id: int = 0) -> bytes:
    """StateMachineLogEntryProto (Raft.proto:72-91) as built by
    LogProtoUtils.toStateMachineLogEntryProto (LogProtoUtils.java:221-232)."""
    sme = None
    if sm_data is not None:  # StateMachineEntryProto{stateMachineData = 1}
        sme = _field_bytes(1, sm_data)
    return (_field_bytes(1, log_data) + (varint((2 << 3) | 2) + varint(len(sme)) + sme if sme is not None else b"")
            + _field_varint(13, sm_type) + _field_bytes(14, client_id) + _field_varint(15, call_id))


def log_entry(term: int, index: int, sm_entry: Optional[bytes] = None, metadata_commit: Optional[int] = None) -> bytes:
    """LogEntryProto (Raft.proto:97-106): term = 1, index = 2, stateMachineLogEntry = 3,
    metadataEntry = 5 (LogProtoUtils.toLogEntryProto, LogProtoUtils.java:126-140)."""
    body = _field_varint(1, term) + _field_varint(2, index)
    if sm_entry is not None:
        body += varint((3 << 3) | 2) + varint(len(sm_entry)) + sm_entry
    elif metadata_commit is not None:
        m = _field_varint(1, metadata_commit)
        body += varint((5 << 3) | 2) + varint(len(m)) + m
    return body


def frame_bytes(proto: bytes) -> bytes:
    """varint || proto || 4 zero bytes (CRC placeholder, stamped on the GPU)."""
    return varint(len(proto)) + proto + b"\0" * TRAILER


def build_segment(protos: Sequence[bytes], preallocate_to: Optional[int] = None,
                  with_header: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Lays out a segment image.  Returns (image uint8, frame_off int64, frame_len int32).

    ``frame_len`` is the whole frame (varint + proto + 4), i.e. what LogSegment.getEntrySize
    accounts for (LogSegment.java:71-84)."""
    parts: List[bytes] = [HEADER] if with_header else []
    pos = len(HEADER) if with_header else 0
    offs, lens = [], []
    for p in protos:
        fb = frame_bytes(p)
        offs.append(pos)
        lens.append(len(fb))
        parts.append(fb)
        pos += len(fb)
    img = b"".join(parts)
    if preallocate_to is not None and preallocate_to > len(img):
        img += b"\0" * (preallocate_to - len(img))
    return (np.frombuffer(img, dtype=np.uint8).copy(), np.asarray(offs, dtype=np.int64),
            np.asarray(lens, dtype=np.int32))


def simple_operation_entries(n: int, term: int = 0, first_index: int = 0, client_id: bytes = bytes(16),
                             first_call_id: int = 1) -> List[bytes]:
    """The entries TestRaftLogReadWrite writes: SimpleOperation("m"+i) at (term, i)
    (TestRaftLogReadWrite.java:92-103, RaftTestUtil.java:411-431)."""
    return [log_entry(term, first_index + i,
                      state_machine_log_entry(log_data=f"m{i}".encode(), client_id=client_id,
                                              call_id=first_call_id + i))
            for i in range(n)]


def fixed_size_entry_prefix(term: int, index: int, proto_len: int) -> bytes:
    """Header bytes of a LogEntryProto{term, index, stateMachineLogEntry{logData}} whose total
    encoded size is exactly ``proto_len``; the logData bytes follow.  Used by the 4 KiB-frame
    synthetic workload."""
    head = _field_varint(1, term) + _field_varint(2, index)
    # solve for logData length L: head + 1 + vs(len_sm) + len_sm = proto_len, len_sm = 1 + vs(L) + L
    for L in range(proto_len, -1, -1):
        len_sm = 1 + varint_size(L) + L
        total = len(head) + 1 + varint_size(len_sm) + len_sm
        if total == proto_len:
            return head + varint((3 << 3) | 2) + varint(len_sm) + varint((1 << 3) | 2) + varint(L)
        if total < proto_len:
            break
    raise ValueError(f"no LogEntryProto encoding of exactly {proto_len} bytes for ({term}, {index})")
