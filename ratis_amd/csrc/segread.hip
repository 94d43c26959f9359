// SegmentedRaftLog read path on gfx950 (MI355X): LogSegment.readSegmentFile in one call --
// framing walk, CRC32C verification of every frame, and the reader's verdict per segment.
//
// Reference semantics (ratis tree, ratis-server/.../raftlog/segmented/ unless noted):
//   LogSegment.readSegmentFile               LogSegment.java:166-196
//   SegmentedRaftLogReader.decodeEntry       SegmentedRaftLogReader.java:291-341 (the reader stops
//                                            at the first frame whose CRC does not verify:
//                                            ChecksumException, :327-336)
//
// Pipeline (all on the caller's stream):
//   1. segment_walk_kernel (segment.hip): framing into the per-segment slotted frame table, then
//      the scan + compaction into the dense frame table;
//   2. the CRC pass (crc32c.hip) in slot mode over the slotted table: per-slot CRCs, each
//      segment's first bad slot atomically lowered in seg_ok, and -- under the length-class plan
//      -- the dense per-frame CRCs and mismatch bits (optional outputs);
//   3. segment_compact_crc_kernel, after the window-only plan: those dense outputs from the slots;
//   4. segment_verdict_kernel: n_ok / status / stop per segment.
// The walk reads frame headers (header fast-forward over runs of equal-length frames), the CRC
// pass reads every frame byte once.  Integer work, no MFMA.
#include "rh_internal.h"

namespace {

// Dense frame table + CRC results: segment s's frames land at seg_first[s]...; the mismatch bit
// compares the computed CRC with the frame's stored big-endian trailer.
__global__ __launch_bounds__(256) void segment_compact_crc_kernel(const uint8_t* buf, uint64_t n_seg, uint32_t cap,
                                                                  const uint64_t* scratch_off,
                                                                  const uint32_t* scratch_len,
                                                                  const uint32_t* scratch_crc,
                                                                  const uint32_t* seg_nframes,
                                                                  const uint64_t* seg_first, uint64_t frame_cap,
                                                                  uint32_t* crc_out, uint64_t* bad_bits) {
    for (uint64_t s = blockIdx.x; s < n_seg; s += gridDim.x) {
        const uint32_t n = seg_nframes[s] < cap ? seg_nframes[s] : cap;
        const uint64_t first = seg_first[s];
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t d = first + i;
            if (d >= frame_cap) break;
            const uint64_t o = scratch_off[s * (uint64_t)cap + i];
            const uint32_t l = scratch_len[s * (uint64_t)cap + i];
            const uint32_t c = scratch_crc[s * (uint64_t)cap + i];
            if (crc_out) crc_out[d] = c;
            if (bad_bits) {
                const uint8_t* tr = buf + o + l - 4;
                const uint32_t stored = ((uint32_t)tr[0] << 24) | ((uint32_t)tr[1] << 16) | ((uint32_t)tr[2] << 8) | tr[3];
                if (stored != c) atomicOr(reinterpret_cast<unsigned long long*>(bad_bits + (d >> 6)), 1ull << (d & 63));
            }
        }
    }
}

// The reader's verdict per segment from the first bad slot (seg_ok pre-set to 0xFFFFFFFF, lowered
// by the CRC pass): decodeEntry throws ChecksumException at the first frame whose CRC does not
// verify (RDR:327-336), so the segment reads as that many frames, stopped at that frame's offset.
__global__ __launch_bounds__(256) void segment_verdict_kernel(const uint64_t* seg_off, const uint32_t* seg_nframes,
                                                              const int32_t* seg_status, const uint64_t* seg_stop,
                                                              const uint64_t* scratch_off, uint64_t n_seg, uint32_t cap,
                                                              uint32_t* seg_ok, int32_t* seg_rstatus,
                                                              uint64_t* seg_rstop) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_seg; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t nfr = seg_nframes[s];
        const uint32_t nfs = nfr < cap ? nfr : cap;
        const uint32_t fb = seg_ok[s];
        const bool bad = fb < nfs;
        seg_ok[s] = bad ? fb : nfr;
        seg_rstatus[s] = bad ? RH_SEG_E_CHECKSUM : seg_status[s];
        seg_rstop[s] = bad ? scratch_off[s * (uint64_t)cap + fb] - seg_off[s] : seg_stop[s];
    }
}

}  // namespace

int rh_segments_read_impl(rh_ctx* ctx, const rh_segments* g, const rh_segments_crc* c, hipStream_t stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: ctx == NULL");
    if (!g || !c) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: segs/crc == NULL");
    if (g->n_seg == 0) return RH_OK;
    if (!c->scratch_crc || !c->seg_ok || !c->seg_read_status || !c->seg_read_stop)
        return rh::fail(RH_E_INVAL, "rh_segments_read_launch: scratch_crc, seg_ok, seg_read_status, seg_read_stop required");
    if (!ctx->d_slice) return rh::fail(RH_E_STATE, "rh_segments_read_launch: CRC tables not uploaded");
    int rc = rh_segments_launch_impl(ctx, g, stream);  // walk + scan + compaction (validates g)
    if (rc != RH_OK) return rc;
    RH_HIP(hipMemsetAsync(c->seg_ok, 0xFF, (size_t)g->n_seg * 4, stream));
    // dense per-frame CRCs / mismatch bits: the length-class plan writes them from the CRC pass
    // (frame seg_first[s] + slot); after the window-only plan a compaction pass gathers them
    if (c->bad_bits) RH_HIP(hipMemsetAsync(c->bad_bits, 0, (size_t)((g->frame_cap + 63) / 64) * 8, stream));
    bool dense = false;
    rc = rh_crc_verify_slots(ctx, g, c, stream, &dense);
    if (rc != RH_OK) return rc;
    if ((c->crc_out || c->bad_bits) && !dense) {
        const int cus = ctx->num_cus > 0 ? ctx->num_cus : 256;
        const uint64_t cgrid = g->n_seg < (uint64_t)cus * 8 ? g->n_seg : (uint64_t)cus * 8;
        hipLaunchKernelGGL(segment_compact_crc_kernel, dim3((uint32_t)cgrid), dim3(256), 0, stream, g->buf, g->n_seg,
                           g->frames_per_seg_cap, g->scratch_off, g->scratch_len, c->scratch_crc, g->seg_nframes,
                           g->seg_first, g->frame_cap, c->crc_out, c->bad_bits);
        RH_HIP(hipGetLastError());
    }
    const uint64_t vgrid = (g->n_seg + 255) / 256 < 1024 ? (g->n_seg + 255) / 256 : 1024;
    hipLaunchKernelGGL(segment_verdict_kernel, dim3((uint32_t)vgrid), dim3(256), 0, stream, g->seg_off, g->seg_nframes,
                       g->seg_status, g->seg_stop, g->scratch_off, g->n_seg, g->frames_per_seg_cap, c->seg_ok,
                       c->seg_read_status, c->seg_read_stop);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
