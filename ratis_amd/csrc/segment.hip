// SegmentedRaftLog segment framing on gfx950: the reader's varint walk, batched over segments.
//
// Reference semantics (ratis-server/.../raftlog/segmented/):
//   SegmentedRaftLogReader.verifyHeader     SegmentedRaftLogReader.java:179-205
//   SegmentedRaftLogReader.decodeEntry      SegmentedRaftLogReader.java:291-341 (size/EOF rules;
//                                           the CRC itself is rh_crc32c_frames_launch's job)
//   SegmentedRaftLogReader.verifyTerminator SegmentedRaftLogReader.java:251-280
//   LimitedInputStream.checkLimit           SegmentedRaftLogReader.java:66-82
//   SegmentedRaftLogFormat header/terminator SegmentedRaftLogFormat.java:30-80
//
// The walk is a serial chain (each frame's length is a varint at its start), so the parallelism
// is across segments: one 256-thread block per segment, two blocks per CU.  The segment streams
// through a 2 x 32 KiB LDS ring; wave 0 walks the frames that start in the current window
// (speculating on runs of equal-length frames: lane j checks the header at p + j*s), the block's
// loads of the window after next are in flight meanwhile, and a run that leaves the window is
// followed straight through HBM reading frame headers only.  Terminator padding is checked by
// the whole block.  Frames are written to a per-segment slotted table, then compacted.
#include "rh_internal.h"

namespace {

constexpr int kScanThreads = 1024;

struct SegArgs {
    const uint8_t* buf;
    int64_t buf_len;
    const uint64_t* seg_off;
    const uint64_t* seg_len;
    uint64_t n_seg;
    uint32_t max_op;
    uint32_t cap;
    uint64_t* scratch_off;
    uint32_t* scratch_len;
    uint32_t* seg_nframes;
    int32_t* seg_status;
    uint64_t* seg_stop;
    // piece-parallel framing hooks (framing of irregular logs, see "Piece-parallel framing" below)
    uint32_t bail_min;            // > 0: defer a segment whose window walk is mostly scalar steps
                                  // and that has at least bail_min bytes left (first pass)
    uint32_t* seg_gmax;           // [n_seg] optional: largest frame length the walk saw
    const uint64_t* resume_pos;   // non-NULL: resume pass -- only deferred segments are walked,
    const uint32_t* resume_nfr;   // from resume_pos[s] with resume_nfr[s] frames already found
};

constexpr int kWalking = 0;
constexpr int kTermPending = 100;
constexpr int kDeferred = 101;  // internal: handed to the piece-parallel pass (never returned)
constexpr int kBailScalar = 8;  // scalar-walked frames in one window that make a segment defer

__device__ __forceinline__ int varint32_size(uint32_t v) {
    if ((v & (~0u << 7)) == 0) return 1;
    if ((v & (~0u << 14)) == 0) return 2;
    if ((v & (~0u << 21)) == 0) return 3;
    if ((v & (~0u << 28)) == 0) return 4;
    return 5;
}

struct __attribute__((aligned(4))) u32x4s {
    uint32_t x, y, z, w;
};

// ---- one 256-thread block per segment, double-buffered windows ----------------------------------
// The segment is cut into W-byte windows on a 16-B aligned grid.  Two windows live in an LDS ring
// (2W bytes); while the walker (thread 0) walks the frames that START in window k, the block's
// loads of window k+2 are in flight in registers, so HBM latency overlaps the serial walk.  Ring
// index of segment byte p = (p - A) & (2W - 1), A = the grid origin (-15..0).  A frame whose
// length jumps past window k+1 restarts the pipeline at the window holding the new position.
constexpr int kBlock2 = 256;

// Block-uniform 64-bit value, pinned to SGPRs (keeps the walker's compares scalar).
// Per-frame outputs of the serial walk are staged one per lane (frame k -> lane k % 64) and
// written 64 at a time as one coalesced store, instead of a single-lane store per frame.
__device__ __forceinline__ void stage_put(uint64_t& so, uint32_t& sl, int lane, uint32_t k, uint64_t off,
                                          uint32_t len) {
    const bool me = lane == (int)(k & 63u);
    so = me ? off : so;
    sl = me ? len : sl;
}
__device__ __forceinline__ void stage_flush(uint64_t* so, uint32_t* sl, int lane, uint32_t n, uint64_t o,
                                            uint32_t l) {
    if ((uint32_t)lane < n) {
        so[lane] = o;
        sl[lane] = l;
    }
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int W>
struct Win {
    static constexpr int PER = W / (kBlock2 * 16);  // 16-B loads per thread per window
    u32x4s r[PER];

    __device__ __forceinline__ void load(const uint8_t* seg, int64_t L, int64_t wstart, int t) {
        if (wstart >= 0 && wstart + W <= L) {
            // whole window inside the segment (block-uniform branch): PER independent 16-B loads
            // in flight together -- no per-chunk guard, so no s_waitcnt between them
#pragma unroll
            for (int i = 0; i < PER; ++i)
                r[i] = *reinterpret_cast<const u32x4s*>(seg + wstart + (int64_t)(i * kBlock2 + t) * 16);
            return;
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int64_t p = wstart + (int64_t)(i * kBlock2 + t) * 16;
            u32x4s v{0, 0, 0, 0};
            if (p >= 0 && p + 16 <= L) {
                v = *reinterpret_cast<const u32x4s*>(seg + p);
            } else if (p < L && p + 16 > 0) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int k = p < 0 ? (int)-p : 0; k < 16 && p + k < L; ++k)
                    w[k >> 2] |= (uint32_t)seg[p + k] << (8 * (k & 3));
                v = {w[0], w[1], w[2], w[3]};
            }
            r[i] = v;
        }
    }
    __device__ __forceinline__ void store(uint8_t* ring, int slot, int t) const {
#pragma unroll
        for (int i = 0; i < PER; ++i)
            *reinterpret_cast<u32x4s*>(ring + slot * W + (i * kBlock2 + t) * 16) = r[i];
        // mirror of the ring's first 16 bytes past its end: an 8-byte read at any q0 <= 2W-4
        // needs no wrap-around
        if (slot == 0 && t == 0) *reinterpret_cast<u32x4s*>(ring + 2 * W) = r[0];
    }
};

template <int W>
__global__ __launch_bounds__(kBlock2) void segment_walk_kernel(SegArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];  // [2W + 16]: 2 windows + mirror
    __shared__ int sh_status;
    __shared__ long long sh_pos;
    __shared__ uint32_t sh_nfr;
    __shared__ unsigned long long sh_min;
    constexpr int64_t MASK = 2 * W - 1;
    const int t = threadIdx.x;
    for (uint64_t s = blockIdx.x; s < a.n_seg; s += gridDim.x) {
        // a descriptor outside buf is a caller error, reported as RH_SEG_E_RANGE (never clamped:
        // a cut-off tail would read as a half-written last entry)
        const uint64_t soff = a.seg_off[s], slen = a.seg_len[s];
        const bool range_bad = soff > (uint64_t)a.buf_len || slen > (uint64_t)a.buf_len - soff;
        const int64_t base = uniform64(range_bad ? 0 : (int64_t)soff);
        const int64_t L = uniform64(range_bad ? 0 : (int64_t)slen);
        const uint8_t* seg = a.buf + base;
        const int64_t A = (base & ~(int64_t)15) - base;
        if (a.resume_pos) {  // resume pass: deferred segments only, from where the pieces stopped
            if (a.seg_status[s] != kDeferred) continue;  // block-uniform
            if (t == 0) {
                sh_status = kWalking;
                sh_pos = (long long)a.resume_pos[s];
                // never past the slot table, whatever the piece pass left (room = cap - nfr below)
                sh_nfr = a.resume_nfr[s] < a.cap ? a.resume_nfr[s] : a.cap;
            }
        } else if (t == 0) {  // verifyHeader (RDR:179-205)
            const char H[8] = {'R', 'a', 'f', 't', 'L', 'o', 'g', '1'};
            const int64_t rl = L < 8 ? L : 8;
            int match = 0, bad = 0;
            for (int i = 0; i < rl; ++i) {
                const uint8_t b = seg[i];
                if (match == i && b == (uint8_t)H[i]) match = i + 1;
                else if (b != 0) bad = 1;
            }
            const bool ok = rl == 8 && match == 8;
            sh_status = range_bad ? RH_SEG_E_RANGE
                                  : ok ? (8 >= L ? RH_SEG_END : kWalking) : (bad ? RH_SEG_E_HEADER : RH_SEG_END);
            sh_pos = ok && !range_bad ? 8 : 0;
            sh_nfr = 0;
        }
        __syncthreads();
        int status = sh_status;
        int64_t pos = sh_pos;
        Win<W> nxt;
        // wave 0's speculation state: the last two frame lengths (equal = a run worth speculating on)
        uint32_t last_fl = 0, prev_fl = 1;
        uint32_t gmax = 0;  // largest frame length walked (sizes the piece pass's guess filter)
        while (status == kWalking) {
            // (re)start the pipeline at the window holding pos
            int64_t k = (pos - A) / W;
            {
                Win<W> cur;
                cur.load(seg, L, A + k * W, t);
                cur.store(ring, (int)(k & 1), t);
            }
            nxt.load(seg, L, A + (k + 1) * W, t);
            for (;;) {
                nxt.store(ring, (int)((k + 1) & 1), t);   // ring now holds windows k, k+1
                __syncthreads();
                nxt.load(seg, L, A + (k + 2) * W, t);       // in flight during the walk
                if (t < 64) {
                    // wave 0 walks, wave-uniformly (lane 0 stores the single-frame steps)
                    const int lane = t;
                    const int64_t wend = A + (k + 1) * W;
                    uint32_t nfr = sh_nfr;
                    int st = kWalking;
                    int64_t p = pos;
                    uint32_t nscalar = 0;  // frames of this window walked one at a time
                    while (p < wend) {
                        {
                            // Speculative run (a run of equal lengths was seen): lane j checks the
                            // frame at p + j * s, s = the last length, with the fast loop's folded
                            // predicate; the leading run of lanes that pass with length s is
                            // accepted at once (frame j + 1 starts at p + (j + 1) s iff frames
                            // 0..j all have length s).  Exact; a mismatch ends the run.
                            const int64_t pend = wend < L - 8 ? wend : L - 8;
                            if (last_fl == prev_fl && last_fl <= (1u << 25) && L <= 0x7fffffff && pend > p) {
                                const uint32_t sd = last_fl, p32 = (uint32_t)p, pend32 = (uint32_t)pend;
                                const uint32_t c = p32 + (uint32_t)lane * sd;
                                const bool okp = c < pend32;
                                const uint32_t q = (uint32_t)(((okp ? c : p32) - A) & MASK);
                                const uint32_t q0 = q & ~3u;
                                const uint32_t lo = *reinterpret_cast<const uint32_t*>(ring + q0);
                                const uint32_t hi = *reinterpret_cast<const uint32_t*>(ring + q0 + 4);  // mirror
                                const uint32_t v = (uint32_t)(((uint64_t)hi << 32 | lo) >> (8 * (q & 3)));
                                const uint32_t stop4 = ~v & 0x80808080u;
                                const int vl = (__builtin_ctz(stop4 | 0x80000000u) >> 3) + 1;
                                const uint32_t nn = ((v & 0x7fu) | ((v >> 1) & 0x3f80u) | ((v >> 2) & 0x1fc000u) |
                                                     ((v >> 3) & 0xfe00000u)) &
                                                    (0xffffffffu >> (32 - 7 * vl));
                                const uint32_t vs = nn < (1u << 7) ? 1u : nn < (1u << 14) ? 2u : nn < (1u << 21) ? 3u : 4u;
                                const uint32_t fl = vs + nn + 4;
                                const uint32_t left = okp ? (uint32_t)L - c : 0u;
                                const bool ok = okp && (v & 0xffu) != 0 && stop4 != 0 && fl == sd &&
                                                fl <= (left < a.max_op ? left : a.max_op) && nfr + (uint32_t)lane < a.cap;
                                const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
                                const uint32_t nacc = __builtin_amdgcn_readfirstlane(~m ? (uint32_t)__builtin_ctzll(~m) : 64u);
                                if (nacc) {
                                    if ((uint32_t)lane < nacc) {
                                        a.scratch_off[s * (uint64_t)a.cap + nfr + lane] = (uint64_t)base + c;
                                        a.scratch_len[s * (uint64_t)a.cap + nfr + lane] = sd;
                                    }
                                    nfr += nacc;
                                    p += (int64_t)nacc * sd;
                                    gmax = sd > gmax ? sd : gmax;
                                    if (nacc == 64) continue;
                                }
                                if (p >= wend) break;
                                if (p < pend) prev_fl = 0;  // a different frame ended the run: scalar loop
                            }
                        }
                        {
                            // Fast loop for the common case, every check folded into two
                            // predicates: a non-zero first byte and a varint of <= 4 bytes wholly
                            // before EOF (p < pend), and a frame within maxOpSize and EOF.
                            // Anything else drops to the rule-by-rule step below (same results).
                            const int64_t pend = wend < L - 8 ? wend : L - 8;
                            const uint32_t room = a.cap - nfr;
                            uint64_t* so = a.scratch_off + s * (uint64_t)a.cap + nfr;
                            uint32_t* sl = a.scratch_len + s * (uint64_t)a.cap + nfr;
                            uint32_t k = 0;
                            if (L <= 0x7fffffff && pend > p) {  // 32-bit offsets: all-scalar compares
                                uint64_t st_o = 0;
                                uint32_t st_l = 0;
                                uint32_t p32 = (uint32_t)p;
                                const uint32_t pend32 = (uint32_t)pend, L32 = (uint32_t)L, mo = a.max_op;
                                uint32_t q = (uint32_t)((p - A) & MASK);
                                while (p32 < pend32 && k < room) {
                                    const uint32_t q0 = q & ~3u;
                                    // wave-uniform: one readfirstlane, then the decode runs on the SALU
                                    const uint32_t lo = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(ring + q0));
                                    const uint32_t hi = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(ring + q0 + 4));  // mirror
                                    const uint32_t v = (uint32_t)(((uint64_t)hi << 32 | lo) >> (8 * (q & 3)));
                                    const uint32_t stop4 = ~v & 0x80808080u;
                                    if ((v & 0xffu) == 0 || stop4 == 0) break;
                                    const int vl = (__builtin_ctz(stop4) >> 3) + 1;
                                    const uint32_t nn = ((v & 0x7fu) | ((v >> 1) & 0x3f80u) | ((v >> 2) & 0x1fc000u) |
                                                         ((v >> 3) & 0xfe00000u)) &
                                                        (0xffffffffu >> (32 - 7 * vl));
                                    const uint32_t vs =
                                        nn < (1u << 7) ? 1u : nn < (1u << 14) ? 2u : nn < (1u << 21) ? 3u : 4u;
                                    const uint32_t fl = vs + nn + 4;  // nn < 2^28: no overflow
                                    const uint32_t left = L32 - p32;
                                    if (fl > (left < mo ? left : mo)) break;
                                    stage_put(st_o, st_l, lane, k, (uint64_t)base + p32, fl);
                                    if ((k & 63u) == 63u) stage_flush(so + (k - 63), sl + (k - 63), lane, 64, st_o, st_l);
                                    ++k;
                                    p32 += fl;
                                    gmax = fl > gmax ? fl : gmax;
                                    q = (q + fl) & (uint32_t)MASK;
                                    prev_fl = last_fl;
                                    last_fl = fl;
                                    if (fl == prev_fl) break;  // a run: back to speculation
                                }
                                stage_flush(so + (k & ~63u), sl + (k & ~63u), lane, k & 63u, st_o, st_l);
                                p = p32;
                            }
                            nfr += k;
                            nscalar += k;
                        }
                        if (p >= wend) break;
                        if (p >= L) {
                            st = RH_SEG_END;
                            break;
                        }
                        // general step: bytes p..p+4 from two aligned LDS dwords
                        const uint32_t q = (uint32_t)((p - A) & MASK);
                        const uint32_t q0 = q & ~3u;
                        const uint32_t lo = *reinterpret_cast<const uint32_t*>(ring + q0);
                        const uint32_t hi = *reinterpret_cast<const uint32_t*>(ring + ((q0 + 4) & MASK));
                        const uint64_t x = ((uint64_t)hi << 32 | lo) >> (8 * (q & 3));
                        if ((x & 0xff) == 0) {  // terminator (SegmentedRaftLogFormat.isTerminator)
                            st = kTermPending;
                            break;
                        }
                        // CodedInputStream.readRawVarint32(firstByte, in): 7 bits per byte, int
                        // arithmetic (bits past 31 dropped); EOF inside the varint -> truncatedMessage
                        const uint64_t stop = ~x & 0x8080808080ull;
                        const int vlen = stop ? (__builtin_ctzll(stop) >> 3) + 1 : 6;
                        const int64_t avail = L - p;
                        uint32_t result = (uint32_t)((x & 0x7f) | ((x >> 1) & 0x3f80) | ((x >> 2) & 0x1fc000) |
                                                     ((x >> 3) & 0xfe00000) | ((x >> 4) & 0x7f0000000ull));
                        if (vlen < 5) result &= (1u << (7 * vlen)) - 1u;
                        if (avail < (vlen < 5 ? vlen : 5)) {
                            st = RH_SEG_E_VARINT;
                            break;
                        }
                        if (vlen == 6) {  // discard up to 5 more bytes of a 64-bit varint
                            bool done = false;
                            for (int i = 5; i < 10 && i < avail; ++i) {
                                if ((ring[(p + i - A) & MASK] & 0x80) == 0) {
                                    done = true;
                                    break;
                                }
                            }
                            if (!done) {
                                st = RH_SEG_E_VARINT;
                                break;
                            }
                        }
                        const int32_t n = (int32_t)result;
                        if (n > (int32_t)a.max_op) {
                            st = RH_SEG_E_OVERSIZE;
                            break;
                        }
                        if (n < 0) {
                            st = RH_SEG_E_VARINT;
                            break;
                        }
                        const int64_t total = (int64_t)varint32_size((uint32_t)n) + n;
                        if (total > (int64_t)a.max_op) {
                            st = RH_SEG_E_OVERSIZE;
                            break;
                        }
                        if (p + total > L) {
                            st = RH_SEG_PARTIAL;
                            break;
                        }
                        // readInt: checkLimit(1) before each of the 4 reads (RDR:66-82)
                        const int64_t lim_room = (int64_t)a.max_op - total;  // reads allowed by the limit
                        const int64_t eof_room = L - p - total;             // bytes before EOF
                        if (lim_room < 4 || eof_room < 4) {
                            st = lim_room <= eof_room ? RH_SEG_E_OVERSIZE : RH_SEG_PARTIAL;
                            break;
                        }
                        if (nfr >= a.cap) {
                            st = RH_SEG_E_CAPACITY;
                            break;
                        }
                        if (lane == 0) {
                            a.scratch_off[s * (uint64_t)a.cap + nfr] = (uint64_t)(base + p);
                            a.scratch_len[s * (uint64_t)a.cap + nfr] = (uint32_t)(total + 4);
                        }
                        ++nfr;
                        ++nscalar;
                        p += total + 4;
                        prev_fl = last_fl;
                        last_fl = (uint32_t)(total + 4);
                        gmax = last_fl > gmax ? last_fl : gmax;
                    }
                    // An irregular log (frames of differing lengths: the window went mostly one
                    // frame at a time) with a long way to go is handed to the piece-parallel pass.
                    if (a.bail_min && st == kWalking && nscalar >= (uint32_t)kBailScalar && L - p >= (int64_t)a.bail_min)
                        st = kDeferred;
                    // Header fast-forward: the window ended inside a run of equal lengths s, so
                    // the run is followed straight through HBM, reading only frame HEADERS: each
                    // round lane j loads the headers at p + j*s and p + (64+j)*s (two 8-byte
                    // reads) and the leading run of frames that pass the fast loop's predicate
                    // with length s is accepted -- up to 128 frames per round trip, the payload
                    // bytes never touched (they are the CRC pass's).  The first frame that breaks
                    // the run (or the segment tail) sends the block back to the LDS window walk,
                    // restarting the ring at the new position.
                    if (st == kWalking && p >= wend && last_fl == prev_fl && last_fl != 0 &&
                        last_fl <= (1u << 24) && L <= 0x7fffffff) {
                        const uint32_t sd = last_fl, pend32 = (uint32_t)(L - 8 > 0 ? L - 8 : 0);
                        for (;;) {
                            if (p >= (int64_t)pend32) break;
                            const uint32_t p32 = (uint32_t)p;
                            uint32_t okm[2];
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const uint32_t cj = p32 + (uint32_t)(lane + 64 * h) * sd;  // < 2^31 + 2^31
                                const bool okp = cj < pend32;
                                const uint64_t ga = (uint64_t)base + (okp ? cj : p32);
                                const uint32_t* wp = reinterpret_cast<const uint32_t*>(a.buf + (ga & ~3ull));
                                const uint32_t lo = wp[0], hi = wp[1];
                                const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (ga & 3)));
                                const uint32_t stop4 = ~v & 0x80808080u;
                                const int vl = (__builtin_ctz(stop4 | 0x80000000u) >> 3) + 1;
                                const uint32_t nn = ((v & 0x7fu) | ((v >> 1) & 0x3f80u) | ((v >> 2) & 0x1fc000u) |
                                                     ((v >> 3) & 0xfe00000u)) &
                                                    (0xffffffffu >> (32 - 7 * vl));
                                const uint32_t vs = nn < (1u << 7) ? 1u : nn < (1u << 14) ? 2u : nn < (1u << 21) ? 3u : 4u;
                                const uint32_t fl = vs + nn + 4;
                                const uint32_t left = okp ? (uint32_t)L - cj : 0u;
                                const bool ok = okp && (v & 0xffu) != 0 && stop4 != 0 && fl == sd &&
                                                fl <= (left < a.max_op ? left : a.max_op) &&
                                                nfr + (uint32_t)(lane + 64 * h) < a.cap;
                                const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
                                okm[h] = __builtin_amdgcn_readfirstlane(~m ? (uint32_t)__builtin_ctzll(~m) : 64u);
                            }
                            const uint32_t nacc = okm[0] < 64 ? okm[0] : 64 + okm[1];
                            for (uint32_t j = (uint32_t)lane; j < nacc; j += 64) {
                                a.scratch_off[s * (uint64_t)a.cap + nfr + j] = (uint64_t)base + p32 + j * sd;
                                a.scratch_len[s * (uint64_t)a.cap + nfr + j] = sd;
                            }
                            nfr += nacc;
                            p += (int64_t)nacc * sd;
                            if (nacc < 128) break;
                        }
                    }
                    if (lane == 0) {
                        sh_status = st;
                        sh_pos = p;
                        sh_nfr = nfr;
                    }
                }
                __syncthreads();
                status = sh_status;
                pos = sh_pos;
                if (status != kWalking) break;
                if (pos >= A + (k + 2) * W) break;  // jumped past the ring: restart there
                ++k;
            }
        }
        if (status == kTermPending) {
            // verifyTerminator (RDR:251-280): the first non-zero byte in [pos, L), block-wide
            if (t == 0) sh_min = (unsigned long long)L;
            __syncthreads();
            const int64_t q0 = ((base + pos) & ~(int64_t)15) - base;
            bool found = false;
            for (int64_t q = q0; q < L && !found; q += (int64_t)W) {
                Win<W> c;
                c.load(seg, L, q, t);
                unsigned long long my = (unsigned long long)L;
#pragma unroll
                for (int i = 0; i < Win<W>::PER; ++i) {
                    const uint32_t ww[4] = {c.r[i].x, c.r[i].y, c.r[i].z, c.r[i].w};
                    const int64_t p = q + (int64_t)(i * kBlock2 + t) * 16;
                    for (int j = 0; j < 4; ++j) {
                        if (ww[j] == 0) continue;
                        for (int b = 0; b < 4; ++b) {
                            const int64_t pb = p + 4 * j + b;
                            if (((ww[j] >> (8 * b)) & 0xff) && pb >= pos && pb < L && (unsigned long long)pb < my)
                                my = (unsigned long long)pb;
                        }
                    }
                }
                if (my < (unsigned long long)L) atomicMin(&sh_min, my);
                __syncthreads();
                found = sh_min < (unsigned long long)L;
                __syncthreads();
            }
            if (found) {
                status = RH_SEG_E_PADDING;
                pos = (int64_t)sh_min;
            } else {
                status = RH_SEG_END;
            }
        }
        if (t == 0) {
            a.seg_nframes[s] = sh_nfr;
            a.seg_status[s] = status;
            a.seg_stop[s] = (uint64_t)pos;
        }
        if (a.seg_gmax && t == 0) a.seg_gmax[s] = gmax;  // thread 0 = wave 0's lane 0
        __syncthreads();
    }
}

// Exclusive scan of seg_nframes (capped at cap) -> seg_first, total_frames.  One block.
__global__ __launch_bounds__(kScanThreads) void segment_scan_kernel(const uint32_t* nframes, uint64_t n_seg,
                                                                    uint32_t cap, uint64_t* seg_first,
                                                                    unsigned long long* total) {
    __shared__ uint64_t part[kScanThreads];
    const int t = threadIdx.x;
    const uint64_t per = (n_seg + kScanThreads - 1) / kScanThreads;
    const uint64_t lo = t * per, hi = lo + per < n_seg ? lo + per : n_seg;
    uint64_t sum = 0;
    for (uint64_t i = lo; i < hi; ++i) sum += nframes[i] < cap ? nframes[i] : cap;
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < kScanThreads; d <<= 1) {  // Hillis-Steele inclusive scan
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0;
    for (uint64_t i = lo; i < hi; ++i) {
        seg_first[i] = run;
        run += nframes[i] < cap ? nframes[i] : cap;
    }
    if (t == kScanThreads - 1) *total = part[t];
}

// Work items of kCompactSlots slots of one segment each (a segment of 32k frames spreads over
// several CUs: one block per segment left most of the chip idle).
constexpr uint32_t kCompactSlots = 4096;
__global__ __launch_bounds__(256) void segment_compact_kernel(const uint64_t* scratch_off, const uint32_t* scratch_len,
                                                              const uint32_t* nframes, const uint64_t* seg_first,
                                                              uint64_t n_seg, uint32_t cap, uint64_t* frame_off,
                                                              uint32_t* frame_len, uint64_t frame_cap) {
    const uint64_t per = (cap + kCompactSlots - 1) / kCompactSlots;
    for (uint64_t it = blockIdx.x; it < n_seg * per; it += gridDim.x) {
        const uint64_t s = it / per;
        const uint32_t lo = (uint32_t)(it - s * per) * kCompactSlots;
        const uint32_t n = nframes[s] < cap ? nframes[s] : cap;
        if (lo >= n) continue;  // block-uniform
        const uint32_t hi = n - lo < kCompactSlots ? n : lo + kCompactSlots;
        const uint64_t first = seg_first[s];
        for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
            if (first + i < frame_cap) {
                frame_off[first + i] = scratch_off[s * (uint64_t)cap + i];
                frame_len[first + i] = scratch_len[s * (uint64_t)cap + i];
            }
        }
    }
}

// ---- Piece-parallel framing (irregular logs) -----------------------------------------------------
// The frame chain is serial, so a segment of differently sized frames walks one frame per step
// (above).  A segment the walk defers (kDeferred: its window went mostly one frame at a time) is
// cut into pieces of kPiece bytes from the deferral point p_d, and the chain is found in parallel:
//   piece_guess_kernel  one 512-thread block per piece, the piece's first kGuessWin bytes in LDS.
//                       Piece 0 starts at p_d.  Piece i >= 1 GUESSES its first frame: candidate
//                       starts B_i, B_i + 1, ... are walked in rounds of 512 (one lane each) with
//                       the fast-path rules; a walk survives if it leaves the window, or ends where
//                       the rest of the window is zero (a terminator) or at EOF; it dies at any other
//                       unparseable header or at a frame longer than gmax (2 x the largest frame
//                       the deferring walk saw).  The lowest survivor is the guess g_i.
//   piece_walk_kernel   one lane per piece, headers straight from HBM: walks from g_i to the piece
//                       end -- frame count, exit (first position >= B_{i+1}, or where the fast walk
//                       ended) and the walk's frame lengths (the list, up to kList frames).
//   piece_stitch_kernel one wave per segment, in piece order: the true entry e_i of piece i is the
//                       exit of piece i-1's true walk.  Walks are deterministic, so once the walk
//                       from e_i reaches a position of the guessed walk the two coincide.  e_i is
//                       usually g_i itself or on the listed walk (a false candidate that survives
//                       has merged into the true chain); otherwise the walk from e_i steps through
//                       HBM until it meets a listed position (the wave holds them all and checks
//                       each step with one ballot), or to the piece end if it never does.  The
//                       result never depends on the guess -- a bad guess only costs those steps.
//                       Per piece: entry, frame count, first slot and the steps before the merge;
//                       per segment: where the fast walk ended.
//   piece_write_kernel  one wave per piece: the frames before the merge walked from the entry, the
//                       rest expanded from the list (a wave prefix sum of lengths, 64 frames per
//                       store), or -- list incomplete -- walked from the entry.
//   segment_walk_kernel (resume pass) takes each deferred segment from where the fast walk ended,
//                       with the full decodeEntry / verifyTerminator rules (usually the terminator).
// A frame is taken by the pieces only if it passes the fast loop's checks (non-zero first byte,
// varint of <= 4 bytes, frame within maxOpSize and EOF, header more than 8 bytes before EOF), the
// frames the serial walk accepts without its rule-by-rule step; everything else is the resume
// pass's.  Integer byte work, no MFMA: the guess pass streams 1/8 of the bytes through LDS, the
// walks touch one header per frame.
#ifndef RH_PIECE_BYTES  // A/B builds override (scripts/ab_build.sh)
#define RH_PIECE_BYTES 131072
#define RH_PIECE_LIST 1024
#endif
constexpr uint32_t kPiece = RH_PIECE_BYTES;  // bytes per piece (or twice that: see piece_plan_kernel)
#ifndef RH_PIECE_ADAPT  // A/B builds override: 0 = every segment at kPiece
#define RH_PIECE_ADAPT 1
#endif
constexpr uint32_t kBigPieceMean = 512;  // mean frame bytes from which a segment takes 2 kPiece
#ifndef RH_HUGE_PIECE_MEAN  // A/B builds override: mean frame bytes from which a segment takes 4 kPiece
#define RH_HUGE_PIECE_MEAN 0xFFFFFFFFull
#endif
#ifndef RH_GUESS_WIN  // A/B builds override (scripts/ab_build.sh)
#define RH_GUESS_WIN 16384
#define RH_PIECE_THREADS 256
#endif
constexpr uint32_t kGuessWin = RH_GUESS_WIN;  // bytes of a piece the guess pass looks at
constexpr uint32_t kGuessLds = kGuessWin + 64;
constexpr int kPieceThreads = RH_PIECE_THREADS;
#ifndef RH_GUESS_BLOCKS_PER_CU  // A/B builds override (scripts/ab_build.sh)
#define RH_GUESS_BLOCKS_PER_CU 6
#endif
// Guess-pass grid size: blocks LAUNCHED per CU (the grid of persistent blocks that take pieces in
// turn), not a residency figure -- how many are resident at once is set by their LDS (~16.5 KB
// each) and waves.  6 per CU beat 4 and 8 on grid / tail balance (profiles/r02/guess_grid/).
constexpr int kGuessBlocksPerCu = RH_GUESS_BLOCKS_PER_CU;
constexpr uint32_t kList = RH_PIECE_LIST;  // frame lengths (u16) a guessed walk records
constexpr uint32_t kListPerLane = kList / 64;
constexpr uint32_t kAList = 16;  // merge-walk frame lengths kept per piece (the true frames before the meeting)
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Frame length of the header v (bytes p..p+3, little-endian) if it passes the fast-path checks,
// else 0.  left = L - p.  (Same folded predicate as the walk's fast loop.)
__device__ __forceinline__ uint32_t fast_frame_len(uint32_t v, uint32_t left, uint32_t max_op) {
    const uint32_t stop4 = ~v & 0x80808080u;
    const int vl = (__builtin_ctz(stop4 | 0x80000000u) >> 3) + 1;
    const uint32_t nn = ((v & 0x7fu) | ((v >> 1) & 0x3f80u) | ((v >> 2) & 0x1fc000u) | ((v >> 3) & 0xfe00000u)) &
                        (0xffffffffu >> (32 - 7 * vl));
    const uint32_t vs = nn < (1u << 7) ? 1u : nn < (1u << 14) ? 2u : nn < (1u << 21) ? 3u : 4u;
    const uint32_t fl = vs + nn + 4;
    const bool ok = (v & 0xffu) != 0 && stop4 != 0 && fl <= (left < max_op ? left : max_op);
    return ok ? fl : 0u;
}

// 4 header bytes at absolute buffer offset ga, read from HBM as two aligned dwords.
__device__ __forceinline__ uint32_t hbm_header(const uint8_t* buf, uint64_t ga) {
    const uint32_t* wp = reinterpret_cast<const uint32_t*>(buf + (ga & ~3ull));
    return (uint32_t)((((uint64_t)wp[1] << 32) | wp[0]) >> (8 * (ga & 3)));
}

// Fast-path frame length at segment position p, from HBM; 0 = the fast walk ends at p.
__device__ __forceinline__ uint32_t hbm_frame_len(const uint8_t* buf, uint64_t base, uint32_t p, uint32_t L,
                                                  uint32_t max_op) {
    return p + 8 < L ? fast_frame_len(hbm_header(buf, base + p), L - p, max_op) : 0u;
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        v += lane >= d ? u : 0u;
    }
    return v;
}

struct PieceArgs {
    const uint8_t* buf;
    uint64_t buf_len;
    const uint64_t* seg_off;
    const uint64_t* seg_len;
    uint64_t n_seg;
    uint32_t max_op;
    uint32_t cap;                // frames_per_seg_cap
    uint64_t piece_cap;          // work items the scratch holds
    const int32_t* seg_status;   // kDeferred = piece pass
    const uint64_t* seg_stop;    // p_d
    const uint32_t* seg_nframes; // frames found before p_d
    const uint32_t* seg_gmax;
    uint32_t* piece_first;       // [n_seg] first work item of the segment
    uint32_t* piece_cnt;         // [n_seg] pieces of the segment (0: serial resume from p_d)
    uint32_t* seg_psz;           // [n_seg] piece size of the segment (bytes)
    uint32_t* piece_seg;         // [piece_cap] segment of each work item (kNone: none)
    unsigned int* n_pieces;      // work items in use
    uint32_t* guess;             // [piece_cap] g (kNone: no survivor)
    uint4* gwalk;                // [piece_cap] walk from g: {g, count, exit, ended | list_ok << 1}
    uint16_t* plen;              // [piece_cap][kList] frame lengths of that walk
    uint16_t* alen;              // [piece_cap][kAList] frame lengths of the merge walk (pre) up to the meeting
    uint4* walk;                 // [piece_cap] true walk: {entry, count, first slot, merge steps | kNone}
    uint4* pre;                  // [piece_cap] merge from the assumed entry (piece_walk_kernel)
    uint64_t* resume_pos;        // [n_seg]
    uint32_t* resume_nfr;        // [n_seg]
    uint64_t* scratch_off;
    uint32_t* scratch_len;
};

// Segment-relative bounds of piece i: [Bi, Bn).
__device__ __forceinline__ void piece_bounds(uint32_t pd, uint32_t L, uint32_t i, uint32_t P, uint32_t& Bi,
                                             uint32_t& Bn) {
    Bi = pd + i * P;
    Bn = L - Bi > P ? Bi + P : L;
}

// One block: pieces per deferred segment (prefix sum) and the work-item -> segment map.
__global__ __launch_bounds__(kScanThreads) void piece_plan_kernel(PieceArgs a) {
    __shared__ uint64_t part[kScanThreads];
    const int t = threadIdx.x;
    const uint64_t per = (a.n_seg + kScanThreads - 1) / kScanThreads;
    const uint64_t lo = t * per, hi = lo + per < a.n_seg ? lo + per : a.n_seg;
    // Piece size per segment: kPiece, or 2 kPiece for a log whose frames the deferring walk saw
    // average >= kBigPieceMean bytes (a piece's walk is a chain of one header load per frame, its
    // guess a fixed cost: long frames afford longer pieces -- 64-2048 B frames +7 % read launch at
    // 256 KiB, 64-512 B frames -6 % framing, same-box A/B, profiles/r03/piece_size/)
    auto psize_of = [&](uint64_t s) -> uint32_t {
        const uint64_t pd = a.seg_stop[s], nf = a.seg_nframes[s];
        if (!RH_PIECE_ADAPT || !nf) return kPiece;
        const uint64_t mean = pd / nf;
        return mean >= RH_HUGE_PIECE_MEAN ? 4 * kPiece : mean >= kBigPieceMean ? 2 * kPiece : kPiece;
    };
    auto pieces_of = [&](uint64_t s) -> uint64_t {
        if (a.seg_status[s] != kDeferred) return 0;
        const uint64_t L = a.seg_len[s], pd = a.seg_stop[s];
        if (L > 0x7fffffffull || pd >= L) return 0;
        const uint64_t P = psize_of(s);
        return (L - pd + P - 1) / P;
    };
    uint64_t sum = 0;
    for (uint64_t s = lo; s < hi; ++s) sum += pieces_of(s);
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < kScanThreads; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    // the prefix is monotone: the segments that fit are a prefix of the deferred ones, and the
    // work items in use end where the last of them ends (*n_pieces zeroed by the host)
    uint64_t run = t ? part[t - 1] : 0;
    for (uint64_t s = lo; s < hi; ++s) {
        const uint64_t np = pieces_of(s);
        const bool fits = run + np <= a.piece_cap;  // else: this segment walks serially
        a.piece_first[s] = (uint32_t)(fits ? run : 0);
        a.piece_cnt[s] = (uint32_t)(fits ? np : 0);
        a.seg_psz[s] = psize_of(s);
        if (fits && np) {  // 16-byte stores over the aligned middle (a store per piece was ~10 us)
            uint64_t w = run;
            const uint64_t e = run + np;
            for (; w < e && (reinterpret_cast<uintptr_t>(a.piece_seg + w) & 15u); ++w) a.piece_seg[w] = (uint32_t)s;
            for (; w + 4 <= e; w += 4) *reinterpret_cast<uint4*>(a.piece_seg + w) = make_uint4(s, s, s, s);
            for (; w < e; ++w) a.piece_seg[w] = (uint32_t)s;
            atomicMax(a.n_pieces, (unsigned int)(run + np));
        }
        run += np;
    }
}

// The guess per piece (see above).  Block-uniform control; LDS holds the guess window.  The next
// piece's window is loaded into registers while the candidate rounds of this one run (its HBM
// latency was the larger part of a piece's time), then stored into LDS after the last round.
__global__ __launch_bounds__(kPieceThreads) void piece_guess_kernel(PieceArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t img[kGuessLds];
    __shared__ unsigned int sh_best;
    __shared__ unsigned int sh_zero;  // image index where the all-zero tail of the window starts
    constexpr uint32_t kPer = (kGuessLds + kPieceThreads * 16 - 1) / (kPieceThreads * 16);
    const int t = threadIdx.x;
    const unsigned int total = *a.n_pieces;
    struct Item {
        uint32_t s, Bi, We, L, o0, ilen, gmax;
        uint64_t base;
    };
    // the next work item at or after w (stride gridDim.x) that needs a guess; a segment's first
    // piece starts at the deferral point, a true frame position (no guess)
    auto find = [&](unsigned int w) -> unsigned int {
        for (; w < total; w += gridDim.x) {
            const uint32_t s = a.piece_seg[w];
            if (s == kNone) continue;  // block-uniform
            if (w == a.piece_first[s]) {
                if (t == 0) a.guess[w] = (uint32_t)a.seg_stop[s];
                continue;
            }
            return w;
        }
        return total;
    };
    // image: segment bytes [Bi - o0, Bi - o0 + kGuessLds) on a 16-byte grid, zero past the region
    // end min(We + 32, L); image index of segment position p = p - Bi + o0
    auto describe = [&](unsigned int w) -> Item {
        Item it{};
        if (w >= total) return it;
        it.s = a.piece_seg[w];
        it.base = a.seg_off[it.s];
        it.L = (uint32_t)a.seg_len[it.s];
        uint32_t Bn;
        piece_bounds((uint32_t)a.seg_stop[it.s], it.L, w - a.piece_first[it.s], a.seg_psz[it.s], it.Bi, Bn);
        // frames longer than gmax (2x the largest the serial walk saw) kill a candidate; the window
        // is 4 gmax (4..16 KiB) so that a false start cannot leave it in a step or two
        const uint32_t gm0 = a.seg_gmax[it.s] * 2u;
        it.gmax = gm0 < 1024u ? 1024u : gm0 > kGuessWin ? kGuessWin : gm0;
        const uint32_t win = 4u * it.gmax < 4096u ? 4096u : 4u * it.gmax > kGuessWin ? kGuessWin : 4u * it.gmax;
        it.We = Bn - it.Bi > win ? it.Bi + win : Bn;  // guess window end
        it.o0 = (uint32_t)((it.base + it.Bi) & 15u);
        const uint32_t rend = it.L - it.We > 32u ? it.We + 32u : it.L;
        it.ilen = rend - it.Bi + it.o0;
        return it;
    };
    u32x4s v[kPer];
    auto issue = [&](const Item& it) {  // every load in flight before any use
        const uint8_t* src = a.buf + it.base + it.Bi - it.o0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t c = ((uint32_t)t + k * kPieceThreads) * 16u;
            v[k] = u32x4s{0, 0, 0, 0};
            if (c + 16 <= it.ilen) v[k] = *reinterpret_cast<const u32x4s*>(src + c);
        }
    };
    unsigned int w = find(blockIdx.x);
    Item cur = describe(w);
    if (w < total) issue(cur);
    while (w < total) {
        if (t == 0) {
            sh_best = kNone;
            sh_zero = 0;
        }
        unsigned int lastnz = 0;  // 1 + highest image index holding a non-zero byte (this thread)
        const uint8_t* src = a.buf + cur.base + cur.Bi - cur.o0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t c = ((uint32_t)t + k * kPieceThreads) * 16u;
            if (c >= kGuessLds) continue;
            if (c < cur.ilen && c + 16 > cur.ilen) {
                uint32_t wv[4] = {0, 0, 0, 0};
                for (uint32_t b = 0; c + b < cur.ilen; ++b) wv[b >> 2] |= (uint32_t)src[c + b] << (8 * (b & 3));
                v[k] = {wv[0], wv[1], wv[2], wv[3]};
            }
            *reinterpret_cast<u32x4s*>(img + c) = v[k];
            const uint32_t ww[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int q = 3; q >= 0; --q)
                if (ww[q]) {
                    const unsigned int e = c + 4u * q + 4u - (__builtin_clz(ww[q]) >> 3);
                    lastnz = e > lastnz ? e : lastnz;
                    break;
                }
        }
        __syncthreads();
        if (lastnz) atomicMax(&sh_zero, lastnz);
        // the next piece's window into registers while this one's rounds run
        const unsigned int w2 = find(w + gridDim.x);
        const Item nxt = describe(w2);
        if (w2 < total) issue(nxt);
        __syncthreads();
        const uint32_t Bi = cur.Bi, We = cur.We, L = cur.L, o0 = cur.o0;
        const uint32_t zpos = sh_zero >= o0 ? Bi + sh_zero - o0 : Bi;  // segment position
        const uint32_t gmax = cur.gmax;
        const uint32_t ncand = We - Bi < 4u * gmax ? We - Bi : 4u * gmax;
        // rounds of kPieceThreads candidate starts until one survives.  The walk is a lockstep
        // loop of predicated steps (one uniform branch per step): a candidate's chain
        //   leaves the window, or reaches the rule-by-rule step's EOF zone   -> survives
        //   reaches a header the fast path rejects                          -> survives iff the
        //                                                                      rest is zero (terminator)
        //   meets a frame longer than gmax (implausible for this log)       -> dies
        const uint32_t* img32 = reinterpret_cast<const uint32_t*>(img);
        const uint32_t qend = We - Bi + o0;                        // window end (image index)
        const uint32_t qeof = L >= Bi + 8 ? L - 8 - Bi + o0 : 0u;  // p + 8 >= L  <=>  q >= qeof
        const uint32_t qz = zpos - Bi + o0;
        for (uint32_t r0 = 0; r0 < ncand; r0 += kPieceThreads) {
            const uint32_t ci = r0 + (uint32_t)t;
            uint32_t q = ci + o0;  // image index of the walk position p = Bi + q - o0
            bool run = ci < ncand, surv = false;
            while (__any(run)) {
                const bool out = q >= qend || q >= qeof;
                const uint32_t qa = out ? 0u : q;  // in-image address for the lanes that read
                const uint32_t wi = qa >> 2;
                const uint32_t hv = __builtin_amdgcn_alignbyte(img32[wi + 1], img32[wi], qa & 3u);
                const uint32_t fl = fast_frame_len(hv, L - (Bi + q - o0), a.max_op);
                surv = surv || (run && (out || (fl == 0 && q >= qz)));
                run = run && !out && fl != 0 && fl <= gmax;
                q += run ? fl : 0u;
            }
            if (surv) atomicMin(&sh_best, ci);
            __syncthreads();
            const unsigned int best = sh_best;
            __syncthreads();  // read by all before the next round may lower it
            if (best != kNone) break;  // block-uniform
        }
        if (t == 0) a.guess[w] = sh_best == kNone ? kNone : Bi + sh_best;
        __syncthreads();
        w = w2;
        cur = nxt;
    }
}

// The same guess with ONE WAVE per piece and every lane busy.  In the rounds above a wave walks
// until its longest-lived candidate dies (~9 steps for the longest of 64 false chains), while a
// false candidate dies after ~2 steps on average: three quarters of the lane-steps were idle
// (PMC: ~6,300 VALU instructions per piece, issue-bound).  Here candidates are handed out in
// increasing order to whichever lanes are free after each step (refill); a candidate that
// survives lowers `best`, candidates above `best` are dropped and no longer handed out, and the
// piece is done when no lane is walking: every candidate below `best` has then died, so `best` is
// the LOWEST survivor -- the guess the rounds produce, exactly.
#ifndef RH_GUESS_REFILL  // A/B builds override: 0 = the block rounds above
#define RH_GUESS_REFILL 1
#endif
#ifndef RH_GUESS_WAVE_BLOCKS_PER_CU
#define RH_GUESS_WAVE_BLOCKS_PER_CU 8  // 8 x 16.5 KB windows of LDS per CU
#endif
constexpr int kGuessWaveBlocksPerCu = RH_GUESS_WAVE_BLOCKS_PER_CU;
#ifndef RH_GUESS_SLOTS  // A/B builds override: candidate slots per lane in the refill loop
#define RH_GUESS_SLOTS 1
#endif
#ifndef RH_GUESS_WIN_MULT  // A/B builds override: survival window = this many gmax (4..16 KiB)
#define RH_GUESS_WIN_MULT 4
#endif
constexpr uint32_t kWinMult = RH_GUESS_WIN_MULT;

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_xor(v, d, 64);
        v = u < v ? u : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_xor(v, d, 64);
        v = u > v ? u : v;
    }
    return v;
}

__global__ __launch_bounds__(64) void piece_guess_wave_kernel(PieceArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t img[kGuessLds];
    constexpr uint32_t kPer = (kGuessLds + 64 * 16 - 1) / (64 * 16);
    const int t = threadIdx.x;
    const unsigned int total = *a.n_pieces;
    struct Item {
        uint32_t s, Bi, We, L, o0, ilen, gmax;
        uint64_t base;
    };
    auto find = [&](unsigned int w) -> unsigned int {  // as piece_guess_kernel
        for (; w < total; w += gridDim.x) {
            const uint32_t s = a.piece_seg[w];
            if (s == kNone) continue;
            if (w == a.piece_first[s]) {
                if (t == 0) a.guess[w] = (uint32_t)a.seg_stop[s];
                continue;
            }
            return w;
        }
        return total;
    };
    auto describe = [&](unsigned int w) -> Item {  // as piece_guess_kernel
        Item it{};
        if (w >= total) return it;
        it.s = a.piece_seg[w];
        it.base = a.seg_off[it.s];
        it.L = (uint32_t)a.seg_len[it.s];
        uint32_t Bn;
        piece_bounds((uint32_t)a.seg_stop[it.s], it.L, w - a.piece_first[it.s], a.seg_psz[it.s], it.Bi, Bn);
        const uint32_t gm0 = a.seg_gmax[it.s] * 2u;
        it.gmax = gm0 < 1024u ? 1024u : gm0 > kGuessWin ? kGuessWin : gm0;
        const uint32_t win = kWinMult * it.gmax < 4096u ? 4096u : kWinMult * it.gmax > kGuessWin ? kGuessWin : kWinMult * it.gmax;
        it.We = Bn - it.Bi > win ? it.Bi + win : Bn;
        it.o0 = (uint32_t)((it.base + it.Bi) & 15u);
        const uint32_t rend = it.L - it.We > 32u ? it.We + 32u : it.L;
        it.ilen = rend - it.Bi + it.o0;
        return it;
    };
    u32x4s v[kPer];
    auto issue = [&](const Item& it) {
        const uint8_t* src = a.buf + it.base + it.Bi - it.o0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t c = ((uint32_t)t + k * 64u) * 16u;
            v[k] = u32x4s{0, 0, 0, 0};
            if (c + 16 <= it.ilen) v[k] = *reinterpret_cast<const u32x4s*>(src + c);
        }
    };
    unsigned int w = find(blockIdx.x);
    Item cur = describe(w);
    if (w < total) issue(cur);
    while (w < total) {
        const uint8_t* src = a.buf + cur.base + cur.Bi - cur.o0;
        const uint32_t qend0 = cur.We - cur.Bi + cur.o0;  // window end (image index)
        bool tailnz = false;  // a non-zero 16 bytes wholly in [window end, region end)
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t c = ((uint32_t)t + k * 64u) * 16u;
            if (c >= kGuessLds) continue;
            if (c < cur.ilen && c + 16 > cur.ilen) {
                uint32_t wv[4] = {0, 0, 0, 0};
                for (uint32_t b = 0; c + b < cur.ilen; ++b) wv[b >> 2] |= (uint32_t)src[c + b] << (8 * (b & 3));
                v[k] = {wv[0], wv[1], wv[2], wv[3]};
            }
            *reinterpret_cast<u32x4s*>(img + c) = v[k];
            tailnz = tailnz || (c >= qend0 && c + 16 <= cur.ilen && (v[k].x | v[k].y | v[k].z | v[k].w) != 0);
        }
        // Where the window's all-zero tail starts (the terminator test of the survival rule) matters
        // only if it starts inside the window: a non-zero byte past the window end rules that out
        // (every mid-segment piece); else the exact position, from the registers still held.
        unsigned int zimg = cur.ilen;
        if (!__any(tailnz)) {
            unsigned int lastnz = 0;
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                const uint32_t c = ((uint32_t)t + k * 64u) * 16u;
                if (c >= kGuessLds) continue;
                const uint32_t ww[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                for (int q = 3; q >= 0; --q)
                    if (ww[q]) {
                        const unsigned int e = c + 4u * q + 4u - (__builtin_clz(ww[q]) >> 3);
                        lastnz = e > lastnz ? e : lastnz;
                        break;
                    }
            }
            zimg = wave_max_u32(lastnz);
        }
        __syncthreads();  // the window is in LDS (one wave: a wait, not a rendezvous)
        const unsigned int w2 = find(w + gridDim.x);
        const Item nxt = describe(w2);
        if (w2 < total) issue(nxt);
        const uint32_t Bi = cur.Bi, We = cur.We, L = cur.L, o0 = cur.o0;
        const uint32_t zpos = zimg >= o0 ? Bi + zimg - o0 : Bi;
        const uint32_t gmax = cur.gmax;
        const uint32_t ncand = We - Bi < 4u * gmax ? We - Bi : 4u * gmax;
        const uint32_t* img32 = reinterpret_cast<const uint32_t*>(img);
        const uint32_t qend = We - Bi + o0;
        const uint32_t qeof = L >= Bi + 8 ? L - 8 - Bi + o0 : 0u;
        const uint32_t qz = zpos - Bi + o0;
        uint32_t best = kNone, limit = ncand;
#if RH_GUESS_SLOTS == 1
        uint32_t next = 64u;
        uint32_t cand = (uint32_t)t, q = cand + o0;
        bool run = cand < limit;
        while (__any(run)) {
            const bool out = q >= qend || q >= qeof;
            const uint32_t qa = out ? 0u : q;
            const uint32_t wi = qa >> 2;
            const uint32_t hv = __builtin_amdgcn_alignbyte(img32[wi + 1], img32[wi], qa & 3u);
            const uint32_t fl = fast_frame_len(hv, L - (Bi + q - o0), a.max_op);
            const bool surv = run && (out || (fl == 0 && q >= qz));
            if (__any(surv)) {  // rare: the true chain (or a false one) left the window
                best = min(best, wave_min_u32(surv ? cand : kNone));
                limit = best;
            }
            run = run && !surv && !out && fl != 0 && fl <= gmax && cand < limit;
            q += run ? fl : 0u;
            // refill: free lanes take the next candidates, in lane order
            const uint64_t freeb = __ballot(!run);
            if (freeb != 0 && next < limit) {
                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(freeb >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)freeb, 0u));
                if (!run) {
                    cand = next + k;
                    q = cand + o0;
                    run = cand < limit;
                }
                next += (uint32_t)__popcll(freeb);
            }
        }
#else
        // two candidate slots per lane, walked in lockstep (their LDS reads issued together: the
        // loop is latency-bound); refill hands the next candidates to slot A's free lanes, then
        // slot B's, in lane order -- still every candidate below the lowest survivor is walked
        // until it dies, so the guess is the same
        uint32_t next = 128u;
        uint32_t candA = (uint32_t)t, qA = candA + o0, candB = 64u + (uint32_t)t, qB = candB + o0;
        bool runA = candA < limit, runB = candB < limit;
        while (__any(runA || runB)) {
            const bool outA = qA >= qend || qA >= qeof, outB = qB >= qend || qB >= qeof;
            const uint32_t qa = outA ? 0u : qA, qb = outB ? 0u : qB;
            const uint32_t hvA = __builtin_amdgcn_alignbyte(img32[(qa >> 2) + 1], img32[qa >> 2], qa & 3u);
            const uint32_t hvB = __builtin_amdgcn_alignbyte(img32[(qb >> 2) + 1], img32[qb >> 2], qb & 3u);
            const uint32_t flA = fast_frame_len(hvA, L - (Bi + qA - o0), a.max_op);
            const uint32_t flB = fast_frame_len(hvB, L - (Bi + qB - o0), a.max_op);
            const bool survA = runA && (outA || (flA == 0 && qA >= qz));
            const bool survB = runB && (outB || (flB == 0 && qB >= qz));
            if (__any(survA || survB)) {
                const uint32_t sA = survA ? candA : kNone, sB = survB ? candB : kNone;
                best = min(best, wave_min_u32(sA < sB ? sA : sB));
                limit = best;
            }
            runA = runA && !survA && !outA && flA != 0 && flA <= gmax && candA < limit;
            runB = runB && !survB && !outB && flB != 0 && flB <= gmax && candB < limit;
            qA += runA ? flA : 0u;
            qB += runB ? flB : 0u;
            const uint64_t fa = __ballot(!runA), fb = __ballot(!runB);
            if ((fa | fb) != 0 && next < limit) {
                const uint32_t na = (uint32_t)__popcll(fa);
                const uint32_t ka = __builtin_amdgcn_mbcnt_hi((uint32_t)(fa >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fa, 0u));
                const uint32_t kb = na + __builtin_amdgcn_mbcnt_hi((uint32_t)(fb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fb, 0u));
                if (!runA) {
                    candA = next + ka;
                    qA = candA + o0;
                    runA = candA < limit;
                }
                if (!runB) {
                    candB = next + kb;
                    qB = candB + o0;
                    runB = candB < limit;
                }
                next += na + (uint32_t)__popcll(fb);
            }
        }
#endif
        if (t == 0) a.guess[w] = best == kNone ? kNone : Bi + best;
        __syncthreads();  // the window may be overwritten
        w = w2;
        cur = nxt;
    }
}

// The walk from p to the piece end through HBM headers, recording the frame lengths in pl.  The
// lengths are buffered in registers and stored 8 at a time (16 B): on gfx9 vmcnt counts stores too,
// and a store per frame made every header load wait for the previous frame's store first (the
// loop's dependent chain then paid two memory round trips per frame).  __restrict__: the header
// loads never alias the list.
__device__ __forceinline__ uint32_t walk_piece(const uint8_t* __restrict__ buf, uint16_t* __restrict__ pl, uint64_t base,
                                               uint32_t p, uint32_t Bn, uint32_t L, uint32_t max_op, uint32_t& cnt,
                                               uint32_t& ended, uint32_t& lok) {
    uint32_t acc[4] = {0, 0, 0, 0};
    while (p < Bn) {
        const uint32_t fl = hbm_frame_len(buf, base, p, L, max_op);
        if (fl == 0) {
            ended = 1;
            break;
        }
        if (cnt < kList) {
            const uint32_t k = cnt & 7u;
            const uint32_t v = (fl < 65536u ? fl : 0xFFFFu) << (16 * (k & 1u));
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) acc[q] = (k >> 1) == q ? ((k & 1u) ? acc[q] | v : v) : acc[q];
            lok &= fl < 65536u ? 1u : 0u;
            if (k == 7u) *reinterpret_cast<uint4*>(pl + (cnt - 7u)) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        }
        ++cnt;
        p += fl;
    }
    const uint32_t c = cnt < kList ? cnt : kList;  // the lengths of a partial last group of 8
    for (uint32_t k = c & ~7u; k < c; ++k) pl[k] = (uint16_t)(acc[(k & 7u) >> 1] >> (16 * (k & 1u)));
    return p;
}

// One lane per piece: the walk from the guess (see above), headers from HBM.
__global__ __launch_bounds__(256) void piece_walk_kernel(PieceArgs a) {
    const unsigned int total = *a.n_pieces;
    for (unsigned int w = blockIdx.x * blockDim.x + threadIdx.x; w < total; w += gridDim.x * blockDim.x) {
        const uint32_t s = a.piece_seg[w];
        if (s == kNone) continue;
        const uint32_t g = a.guess[w];
        uint16_t* pl = a.plen + (uint64_t)w * kList;
        uint32_t cnt = 0, p = g, ended = 0, lok = 1;
        if (g != kNone) {
            const uint64_t base = a.seg_off[s];
            const uint32_t L = (uint32_t)a.seg_len[s];
            uint32_t Bi, Bn;
            piece_bounds((uint32_t)a.seg_stop[s], L, w - a.piece_first[s], a.seg_psz[s], Bi, Bn);
            p = walk_piece(a.buf, pl, base, p, Bn, L, a.max_op, cnt, ended, lok);
        }
        a.gwalk[w] = make_uint4(g, cnt, p, ended | (lok << 1));
        // The next piece's merge (see piece_stitch_kernel): if this walk is the true one, the next
        // piece's true entry is its exit p.  Almost every guess is a false start whose chain merged
        // into the true one, so walk from p (chain A) and from the next guess (chain B) in position
        // order until they meet: A's steps before the meeting point are the true frames the guessed
        // walk missed, B's the false ones it has.  Headers from HBM; bounded, else left to the stitch.
        // pre[w + 1] = {assumed entry, A steps, met ? B steps : A's exit, met | ended << 1}.
        if (w == a.piece_first[s]) a.pre[w] = make_uint4(kNone, 0, 0, 0);
        if (w + 1 < total && a.piece_seg[w + 1] == s) {
            uint4 pr = make_uint4(kNone, 0, 0, 0);
            const uint32_t gb = a.guess[w + 1];
            if (g != kNone && !ended && gb != kNone) {
                const uint64_t base = a.seg_off[s];
                const uint32_t L = (uint32_t)a.seg_len[s];
                uint32_t Bi, Bn;
                piece_bounds((uint32_t)a.seg_stop[s], L, w + 1 - a.piece_first[s], a.seg_psz[s], Bi, Bn);
                uint32_t pa = p, pb = gb, ma = 0, mb = 0, fa_end = 0, steps = 0;
                uint32_t al[kAList / 2] = {};  // A's frame lengths (u16 pairs), stored once at the end
                bool alfit = true;             // every one of them below 64 KiB
                bool bdone = false, met = false, give_up = false;
                while (true) {
                    if (pa == pb) {
                        met = true;
                        break;
                    }
                    if (pa >= Bn) break;  // not met: A's walk (to the piece end) is the true one
                    if (bdone && pa > pb) {  // B died before A reached it: a false survivor -- the
                        give_up = true;      // rest of A's walk is the stitch's (windowed) walk
                        break;
                    }
                    if (++steps > 48) {
                        give_up = true;
                        break;
                    }
                    if (pa < pb || bdone) {
                        const uint32_t fl = hbm_frame_len(a.buf, base, pa, L, a.max_op);
                        if (fl == 0) {
                            fa_end = 1;
                            break;
                        }
                        if (ma < kAList) {
                            const uint32_t v = (fl & 0xFFFFu) << (16 * (ma & 1u));
                            alfit = alfit && fl < 65536u;
#pragma unroll
                            for (uint32_t q = 0; q < kAList / 2; ++q) al[q] = (ma >> 1) == q ? (al[q] | v) : al[q];
                        }
                        pa += fl;
                        ++ma;
                    } else {
                        const uint32_t fl = pb < Bn ? hbm_frame_len(a.buf, base, pb, L, a.max_op) : 0u;
                        if (fl == 0) bdone = true;  // B's walk ends at pb (a meeting is still possible there)
                        else {
                            pb += fl;
                            ++mb;
                        }
                    }
                }
                if (!give_up) {
                    // bit 2: al holds every one of A's frames before the meeting (the write uses them)
                    const bool alok = met && ma <= kAList && alfit;
                    pr = make_uint4(p, ma, met ? mb : pa, (met ? 1u : 0u) | (fa_end << 1) | (alok ? 4u : 0u));
                    if (alok) {
                        uint4* dst = reinterpret_cast<uint4*>(a.alen + (uint64_t)(w + 1) * kAList);
                        dst[0] = make_uint4(al[0], al[1], al[2], al[3]);
                        dst[1] = make_uint4(al[4], al[5], al[6], al[7]);
                    }
                }
            }
            a.pre[w + 1] = pr;
        }
    }
}

// The true walk of piece w from entry e (!= its guess g): through HBM headers until it meets a
// listed position of the guessed walk (from there the two coincide) or passes the listed part or
// ends.  Wave-uniform; the guessed walk's positions are rebuilt in registers (lane l: frames
// [16 l, 16 l + 16)).  In: gr = gwalk[w].  Out: cnt / x / ended of the true walk, msteps = steps
// before the meeting point (kNone: never met).
struct MergeOut {
    uint32_t cnt, x, ended, msteps;
};
// The walk streams the segment through two 8 KiB LDS windows (the next one loaded while the
// current one is walked): a false-survivor guess leaves a whole piece (~125 frames) to walk, and a
// header load per frame from HBM made that one memory round trip per frame.
#ifndef RH_MERGE_WIN
#define RH_MERGE_WIN 8192
#endif
constexpr uint32_t kMergeWin = RH_MERGE_WIN;
constexpr uint32_t kMergePer = kMergeWin / (64 * 16);  // 16-B loads per lane per window
// rec (LDS, kList entries): the true walk's frame lengths as walked (lane 0 stores them).
__device__ __forceinline__ MergeOut merge_walk(const PieceArgs& a, uint32_t w, uint4 gr, uint32_t e, uint32_t Bn,
                                               uint64_t base, uint32_t L, int lane, uint8_t* ring, uint16_t* rec) {
    const uint32_t g = gr.x, gfl = gr.w;
    uint32_t cnt = gr.y, x = gr.z;
    const uint32_t nl = (g != kNone && (gfl & 2u)) ? (cnt < kList ? cnt : kList) : 0u;
    uint32_t pos[kListPerLane];
    uint32_t run = 0;
    const uint16_t* pl = a.plen + (uint64_t)w * kList + (uint32_t)lane * kListPerLane;
#pragma unroll
    for (uint32_t k = 0; k < kListPerLane; ++k) {
        const uint32_t idx = (uint32_t)lane * kListPerLane + k;
        pos[k] = run;
        run += idx < nl ? (uint32_t)pl[k] : 0u;
    }
    const uint32_t incl = wave_incl_scan(run, lane);
    const uint32_t off = g + incl - run;
#pragma unroll
    for (uint32_t k = 0; k < kListPerLane; ++k) pos[k] = (uint32_t)lane * kListPerLane + k < nl ? off + pos[k] : kNone;
    const uint32_t last = nl ? g + __builtin_amdgcn_readlane(incl, 63) : 0u;  // end of the listed part
    uint32_t p = e, m = 0, ended = 0;
    bool met = false;
    // windows: absolute buffer addresses [W, W + kMergeWin), W 16-B aligned; slot 0/1 of ring
    u32x4s nx[kMergePer];
    auto fetch = [&](uint64_t W) {
#pragma unroll
        for (uint32_t k = 0; k < kMergePer; ++k) {
            const uint64_t q = W + ((uint64_t)k * 64 + (uint64_t)lane) * 16;
            nx[k] = q + 16 <= a.buf_len ? *reinterpret_cast<const u32x4s*>(a.buf + q) : u32x4s{0, 0, 0, 0};
        }
    };
    auto put = [&](uint32_t slot) {
#pragma unroll
        for (uint32_t k = 0; k < kMergePer; ++k)
            *reinterpret_cast<u32x4s*>(ring + slot * kMergeWin + ((uint32_t)k * 64 + (uint32_t)lane) * 16) = nx[k];
    };
    uint64_t Wc = (base + p) & ~15ull, Wn = Wc + kMergeWin;
    uint32_t slot = 0;
    fetch(Wc);
    put(0);
    fetch(Wn);
    while (p < Bn) {
        if (p < last) {
            uint32_t jl = kNone;
#pragma unroll
            for (uint32_t k = 0; k < kListPerLane; ++k)
                if (pos[k] == p) jl = (uint32_t)lane * kListPerLane + k;
            const uint64_t hit = __builtin_amdgcn_ballot_w64(jl != kNone);
            if (hit) {
                const uint32_t jj = __builtin_amdgcn_readlane(jl, __builtin_ctzll(hit));
                cnt = m + cnt - jj;  // x, ended: the guessed walk's
                met = true;
                break;
            }
        }
        if (p + 8 >= L) {  // hbm_frame_len's EOF zone: the fast walk ends
            ended = 1;
            break;
        }
        const uint64_t q = base + p;
        if ((q & ~3ull) + 8 > Wc + kMergeWin) {  // the header is not inside the current window
            if ((q & ~3ull) >= Wn && (q & ~3ull) + 8 <= Wn + kMergeWin) {
                slot ^= 1u;
                put(slot);  // the prefetched next window
                Wc = Wn;
            } else {        // a long frame jumped past it: load the window at q
                Wc = q & ~15ull;
                fetch(Wc);
                slot ^= 1u;
                put(slot);
            }
            Wn = Wc + kMergeWin;
            fetch(Wn);
        }
        const uint32_t o = (uint32_t)((q & ~3ull) - Wc) + slot * kMergeWin;
        const uint32_t hv = __builtin_amdgcn_alignbyte(*reinterpret_cast<const uint32_t*>(ring + o + 4),
                                                       *reinterpret_cast<const uint32_t*>(ring + o), (uint32_t)(q & 3u));
        const uint32_t fl = fast_frame_len(hv, L - p, a.max_op);
        if (fl == 0) {
            ended = 1;
            break;
        }
        if (lane == 0 && m < kList) rec[m] = (uint16_t)(fl < 65536u ? fl : 0u);
        ++m;
        p += fl;
    }
    if (!met) return MergeOut{m, p, ended, kNone};
    return MergeOut{cnt, x, gfl & 1u, m};
}

// One wave per segment: the true chain through the pieces (see above).  Control is wave-uniform.
__global__ __launch_bounds__(64) void piece_stitch_kernel(PieceArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[2 * kMergeWin];  // merge_walk's windows
    __shared__ uint16_t rec[kList];                                        // ... and its frame lengths
    const uint64_t s = blockIdx.x;
#ifdef RH_STITCH_STATS
    const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t_1 = 0, t_2 = 0;
    uint32_t npass = 0, nser = 0, n_mw = 0;
    uint64_t t_mw = 0;
#endif
    if (s >= a.n_seg || a.seg_status[s] != kDeferred) return;
    const int lane = threadIdx.x;
    const uint64_t base = a.seg_off[s];
    const uint32_t L = (uint32_t)a.seg_len[s];
    const uint32_t pd = (uint32_t)a.seg_stop[s];
    const uint32_t np = a.piece_cnt[s], pf = a.piece_first[s], PS = a.seg_psz[s];  // pieces, first, size
    uint32_t e = pd, total = a.seg_nframes[s];
    uint64_t rpos = pd;
    uint32_t rnfr = total;
    bool done = false;
    uint32_t j = 0;  // pieces [0, j) resolved (their walk entries written)
    constexpr uint32_t K = 8;  // pieces per lane in a parallel pass (512 = 64 MiB of segment)
    const uint4 kDefault = make_uint4(0, 0, 0, kNone);
    while (j < np && !done) {
        // ---- parallel pass over pieces j + lane K + k: each takes as its entry the previous
        // piece's guessed exit (the first one: the true entry e).  While every piece's true exit
        // is its guessed exit, those entries are the true ones and a piece's walk follows from
        // pre / gwalk alone; the pass stops at the first piece where that fails (unknown merge,
        // exit differing, walk ended, a frame spanning the piece, slot capacity).
        const uint32_t P = np - j < 64 * K ? np - j : 64 * K;
        uint4 gr[K], pr[K];
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t i = (uint32_t)lane * K + k;
            gr[k] = make_uint4(kNone, 0, 0, 0);
            pr[k] = make_uint4(kNone, 0, 0, 0);
            if (i < P) {
                gr[k] = a.gwalk[pf + j + i];
                pr[k] = a.pre[pf + j + i];
            }
        }
#ifdef RH_STITCH_STATS
        if (!t_1) t_1 = __builtin_amdgcn_s_memrealtime() + (gr[0].x & 0);
        ++npass;
#endif
        const uint32_t prevx = (uint32_t)__shfl_up((int)gr[K - 1].z, 1, 64);
        uint32_t ent[K], cnt[K], xx[K], ms[K], incl[K], excl[K];
        bool kn[K], en[K];
        uint32_t run = 0;
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t i = (uint32_t)lane * K + k;
            ent[k] = k ? gr[k - 1].z : (lane ? prevx : e);
            uint32_t Bi, Bn;
            piece_bounds(pd, L, j + i, PS, Bi, Bn);
            kn[k] = i < P && ent[k] < Bn;
            cnt[k] = gr[k].y;
            xx[k] = gr[k].z;
            en[k] = gr[k].w & 1u;
            ms[k] = 0;
            if (ent[k] != gr[k].x) {
                if (pr[k].x == ent[k]) {
                    if (pr[k].w & 1u) {  // met after pr.y true and pr.z false frames
                        cnt[k] = pr[k].y + gr[k].y - pr[k].z;
                        ms[k] = pr[k].y;
                    } else {  // never met: the true walk is the merge walk's
                        cnt[k] = pr[k].y;
                        xx[k] = pr[k].z;
                        en[k] = (pr[k].w >> 1) & 1u;
                        ms[k] = kNone;
                    }
                } else {
                    kn[k] = false;
                }
            }
            excl[k] = run;
            run += kn[k] ? cnt[k] : 0u;
            incl[k] = run;
        }
        const uint32_t lincl = wave_incl_scan(run, lane);
        const uint32_t lexcl = lincl - run;
        uint32_t kb = K;  // this lane's first piece that breaks the chain
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            incl[k] += lexcl;  // frames of the pass up to and including piece k
            excl[k] += lexcl;  // ... before piece k
            kn[k] = kn[k] && total + incl[k] <= a.cap;
            const bool chain = kn[k] && !en[k] && xx[k] == gr[k].z;  // the next entry is true
            if (kb == K && !chain) kb = k;
        }
        const uint32_t first = wave_min_u32(kb < K ? (uint32_t)lane * K + kb : kNone);  // wave-uniform
        // values of the piece `first` (or of the pass's last piece) from the lane holding it
        const uint32_t at = first < P ? first : P - 1;
        const uint32_t atk = at % K;
        uint32_t v_incl = 0, v_excl = 0, v_x = 0, v_ent = 0, v_en = 0, v_kn = 0;
#pragma unroll
        for (uint32_t k = 0; k < K; ++k)
            if (k == atk) {
                v_incl = incl[k];
                v_excl = excl[k];
                v_x = xx[k];
                v_ent = ent[k];
                v_en = en[k];
                v_kn = kn[k];
            }
        const int src = (int)(at / K);
        v_incl = (uint32_t)__shfl((int)v_incl, src);
        v_excl = (uint32_t)__shfl((int)v_excl, src);
        v_x = (uint32_t)__shfl((int)v_x, src);
        v_ent = (uint32_t)__shfl((int)v_ent, src);
        v_en = (uint32_t)__shfl((int)v_en, src);
        v_kn = (uint32_t)__shfl((int)v_kn, src);
        const bool all = first >= P;  // every piece of the pass chains
        const uint32_t ntake = all ? P : (v_kn ? first + 1 : first);
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t i = (uint32_t)lane * K + k;
            if (i < ntake) a.walk[pf + j + i] = make_uint4(ent[k], cnt[k], total + incl[k] - cnt[k], ms[k]);
        }
        if (all || v_kn) {
            j += ntake;
            total += v_incl;
            if (!all && v_en) {
                rpos = v_x;
                rnfr = total;
                done = true;
            } else {
                e = v_x;  // the next pass starts from the true exit
            }
            continue;
        }
        // ---- piece j + first: the serial merge walk from its true entry ----
#ifdef RH_STITCH_STATS
        ++nser;
        if (!t_2) t_2 = __builtin_amdgcn_s_memrealtime();
#endif
        j += first;
        total += v_excl;  // the frames of the pieces before it
        e = v_ent;
        const uint32_t w = pf + j;
        uint32_t Bi, Bn;
        piece_bounds(pd, L, j, PS, Bi, Bn);
        if (e >= Bn) {  // a frame spans this piece: nothing starts in it
            if (lane == 0) a.walk[w] = make_uint4(e, 0, total, kNone);
            ++j;
            continue;
        }
        const uint4 g4 = a.gwalk[w];
        const uint4 p4 = a.pre[w];
        const uint32_t g = __builtin_amdgcn_readfirstlane(g4.x);
        uint32_t cnt1 = __builtin_amdgcn_readfirstlane(g4.y);
        uint32_t x1 = __builtin_amdgcn_readfirstlane(g4.z);
        const uint32_t gfl = __builtin_amdgcn_readfirstlane(g4.w);
        uint32_t ended = gfl & 1u, msteps = 0;
        const uint32_t pe = __builtin_amdgcn_readfirstlane(p4.x);
        if (pe == e && g != e) {  // piece_walk_kernel's merge from this entry
            const uint32_t ma = __builtin_amdgcn_readfirstlane(p4.y);
            const uint32_t z = __builtin_amdgcn_readfirstlane(p4.z);
            const uint32_t fm = __builtin_amdgcn_readfirstlane(p4.w);
            if (fm & 1u) {
                cnt1 = ma + cnt1 - z;
                msteps = ma;
            } else {
                cnt1 = ma;
                x1 = z;
                ended = (fm >> 1) & 1u;
                msteps = kNone;
            }
        } else if (g != e) {
#ifdef RH_STITCH_STATS
            const uint64_t tm0 = __builtin_amdgcn_s_memrealtime();
#endif
            const MergeOut r = merge_walk(a, w, make_uint4(g, cnt1, x1, gfl), e, Bn, base, L, lane, ring, rec);
#ifdef RH_STITCH_STATS
            t_mw += __builtin_amdgcn_s_memrealtime() + (r.cnt & 0) - tm0;
            n_mw += r.msteps == kNone ? r.cnt : r.msteps;
#endif
            cnt1 = r.cnt;
            x1 = r.x;
            ended = r.ended;
            msteps = r.msteps;
            if (msteps == kNone) {
                // never met: the walk just made IS the piece's true walk -- its lengths become the
                // piece's list and its guessed walk, so piece_write expands them (instead of
                // re-walking every frame of the piece through HBM)
                const uint32_t nr = cnt1 < kList ? cnt1 : kList;
                bool fits = cnt1 <= kList;
                __builtin_amdgcn_wave_barrier();
                uint16_t* pl = a.plen + (uint64_t)w * kList;
                for (uint32_t i = (uint32_t)lane; i < nr; i += 64) {
                    const uint16_t v = rec[i];
                    pl[i] = v;
                    fits = fits && v != 0;
                }
                fits = __builtin_amdgcn_ballot_w64(!fits) == 0;
                if (lane == 0) a.gwalk[w] = make_uint4(e, cnt1, x1, ended | (fits ? 2u : 0u));
                msteps = 0;
            }
        }
        if (total + cnt1 > a.cap) {  // the slot capacity ends inside this piece: serial from e
            rpos = e;
            rnfr = total;
            done = true;
            break;
        }
        if (lane == 0) a.walk[w] = make_uint4(e, cnt1, total, msteps);
        total += cnt1;
        ++j;
        if (ended) {
            rpos = x1;
            rnfr = total;
            done = true;
            break;
        }
        e = x1;
    }
    if (done)
        for (uint32_t i = j + (uint32_t)lane; i < np; i += 64) a.walk[pf + i] = kDefault;
    if (!done) {  // unreachable (a header within 8 bytes of EOF ends every fast walk); be exact anyway
        rpos = e;
        rnfr = total;
    }
    if (lane == 0) {
        a.resume_pos[s] = rpos;
        a.resume_nfr[s] = rnfr;
    }
#ifdef RH_STITCH_STATS
    const uint64_t t_3 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
        printf("STITCH seg %u np %u passes %u serial %u t0 %llu loads %u first_serial %u end %u merge_walk %u steps %u\n",
               (unsigned)s, np, npass, nser, (unsigned long long)t_0, (unsigned)(t_1 - t_0),
               (unsigned)(t_2 ? t_2 - t_0 : 0), (unsigned)(t_3 - t_0), (unsigned)t_mw, n_mw);
#endif
}

// One wave per piece: the piece's frames into the segment's slots (see above).
__global__ __launch_bounds__(256) void piece_write_kernel(PieceArgs a) {
    const unsigned int total = *a.n_pieces;
    const int lane = threadIdx.x & 63;
    const unsigned int nwaves = gridDim.x * (blockDim.x >> 6);
    for (unsigned int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w < total; w += nwaves) {
        const uint32_t s = a.piece_seg[w];
        if (s == kNone) continue;  // wave-uniform
        const uint4 r = a.walk[w];
        if (r.y == 0) continue;
        const uint64_t base = a.seg_off[s];
        const uint32_t L = (uint32_t)a.seg_len[s];
        uint64_t* so = a.scratch_off + s * (uint64_t)a.cap + r.z;
        uint32_t* sl = a.scratch_len + s * (uint64_t)a.cap + r.z;
        const uint4 gw = a.gwalk[w];
        const uint32_t m = r.w;
        if (m != kNone && (gw.w & 2u) && gw.y <= kList) {
            // frames [0, m): the true walk from the entry -- the lengths piece_walk_kernel's merge
            // walk kept (pre bit 2, same entry), else walked again; [m, count): list entries [jj, gcnt)
            const uint4 pr = a.pre[w];
            if (m > 0 && pr.x == r.x && (pr.w & 4u) && pr.y == m) {
                const uint32_t len = (uint32_t)lane < m ? (uint32_t)a.alen[(uint64_t)w * kAList + lane] : 0u;
                const uint32_t incl = wave_incl_scan(len, lane);
                if ((uint32_t)lane < m) {
                    so[lane] = base + r.x + incl - len;
                    sl[lane] = len;
                }
            } else if (lane == 0) {
                uint32_t p = r.x;
                for (uint32_t k = 0; k < m; ++k) {
                    const uint32_t fl = hbm_frame_len(a.buf, base, p, L, a.max_op);
                    so[k] = base + p;
                    sl[k] = fl;
                    p += fl;
                }
            }
            const uint32_t jj = gw.y - (r.y - m);
            const uint16_t* pl = a.plen + (uint64_t)w * kList;
            uint32_t run = gw.x;  // position of list entry c
            for (uint32_t c = 0; c < gw.y; c += 64) {
                const uint32_t idx = c + (uint32_t)lane;
                const uint32_t len = idx < gw.y ? (uint32_t)pl[idx] : 0u;
                const uint32_t incl = wave_incl_scan(len, lane);
                if (idx >= jj && idx < gw.y) {
                    const uint32_t k = m + idx - jj;
                    so[k] = base + run + incl - len;
                    sl[k] = len;
                }
                run += __builtin_amdgcn_readlane(incl, 63);
            }
            continue;
        }
        if (lane != 0) continue;
        uint32_t p = r.x;
        for (uint32_t k = 0; k < r.y; ++k) {
            const uint32_t fl = hbm_frame_len(a.buf, base, p, L, a.max_op);
            so[k] = base + p;
            sl[k] = fl;
            p += fl;
        }
    }
}

#ifdef RH_AB_FENCE_PROBE
__global__ void empty_probe_kernel(int) {}
#endif

constexpr int kWalkWindow = 32768;  // 2 x 32 KiB LDS ring + mirror: two blocks per CU

hipError_t launch_walk(const SegArgs& a, int cus, hipStream_t stream) {
    constexpr int lds = 2 * kWalkWindow + 16;
    // once per process (thread-safe static initialisation)
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(segment_walk_kernel<kWalkWindow>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (attr != hipSuccess) return attr;
    const uint64_t cap = (uint64_t)cus * 2;
    const uint64_t grid = a.n_seg < cap ? a.n_seg : cap;
    hipLaunchKernelGGL((segment_walk_kernel<kWalkWindow>), dim3((uint32_t)grid), dim3(kBlock2), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

int rh_segments_scan_counts(const uint32_t* nframes, uint64_t n_seg, uint32_t cap, uint64_t* seg_first,
                            unsigned long long* total, hipStream_t stream) {
    hipLaunchKernelGGL(segment_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, nframes, n_seg, cap, seg_first, total);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_segments_launch_impl(rh_ctx* ctx, const rh_segments* g, hipStream_t stream) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_segments_scan_launch: segs == NULL");
    if (g->n_seg == 0) return RH_OK;
    if (!g->buf || !g->seg_off || !g->seg_len || !g->scratch_off || !g->scratch_len || !g->frame_off ||
        !g->frame_len || !g->seg_first || !g->seg_nframes || !g->seg_status || !g->seg_stop || !g->total_frames)
        return rh::fail(RH_E_INVAL, "rh_segments_scan_launch: every array is required");
    if (g->frames_per_seg_cap == 0) return rh::fail(RH_E_INVAL, "rh_segments_scan_launch: frames_per_seg_cap == 0");
    if (g->max_op == 0 || g->max_op > 0x7FFFFFFFu) return rh::fail(RH_E_INVAL, "rh_segments_scan_launch: bad max_op");
    if (g->buf_len > (uint64_t)INT64_MAX) return rh::fail(RH_E_RANGE, "rh_segments_scan_launch: buf_len too large");
    SegArgs a{};
    a.buf = g->buf;
    a.buf_len = (int64_t)g->buf_len;
    a.seg_off = g->seg_off;
    a.seg_len = g->seg_len;
    a.n_seg = g->n_seg;
    a.max_op = g->max_op;
    a.cap = g->frames_per_seg_cap;
    a.scratch_off = g->scratch_off;
    a.scratch_len = g->scratch_len;
    a.seg_nframes = g->seg_nframes;
    a.seg_status = g->seg_status;
    a.seg_stop = g->seg_stop;
    const int cus = ctx && ctx->num_cus > 0 ? ctx->num_cus : 256;
    // Piece-pass scratch (stream-ordered, from the context's pool): per segment 28 B, per piece
    // 56 + 2 kList + 2 kAList B.  piece_cap bounds the pieces of non-overlapping segments; segments beyond it
    // walk serially.
    const uint64_t n_seg = g->n_seg;
    const uint64_t piece_cap = g->buf_len / kPiece + n_seg + 1;
    const size_t bytes = (size_t)piece_cap * (56 + 2 * kList + 2 * kAList) + (size_t)n_seg * 28 + 64;
    rh::PoolScratch scratch(stream);  // released on every exit path (after the last pass using it)
    RH_HIP(scratch.alloc(ctx, bytes));
    uint8_t* sp = scratch.bytes();
    PieceArgs pa{};
    pa.gwalk = reinterpret_cast<uint4*>(sp);
    pa.walk = pa.gwalk + piece_cap;
    pa.pre = pa.walk + piece_cap;
    pa.resume_pos = reinterpret_cast<uint64_t*>(pa.pre + piece_cap);
    pa.piece_first = reinterpret_cast<uint32_t*>(pa.resume_pos + n_seg);
    pa.piece_cnt = pa.piece_first + n_seg;
    uint32_t* seg_gmax = pa.piece_cnt + n_seg;
    pa.seg_gmax = seg_gmax;
    pa.resume_nfr = seg_gmax + n_seg;
    pa.seg_psz = pa.resume_nfr + n_seg;
    pa.n_pieces = reinterpret_cast<unsigned int*>(pa.seg_psz + n_seg);
    pa.piece_seg = reinterpret_cast<uint32_t*>(pa.n_pieces + 4);
    pa.guess = pa.piece_seg + piece_cap;
    pa.plen = reinterpret_cast<uint16_t*>(pa.guess + piece_cap);
    pa.alen = pa.plen + (size_t)piece_cap * kList;
    pa.buf = g->buf;
    pa.buf_len = g->buf_len;
    pa.seg_off = g->seg_off;
    pa.seg_len = g->seg_len;
    pa.n_seg = n_seg;
    pa.max_op = g->max_op;
    pa.cap = g->frames_per_seg_cap;
    pa.piece_cap = piece_cap;
    pa.seg_status = g->seg_status;
    pa.seg_stop = g->seg_stop;
    pa.seg_nframes = g->seg_nframes;
    pa.scratch_off = g->scratch_off;
    pa.scratch_len = g->scratch_len;
    // 1. serial walk; irregular segments with >= 2 pieces to go are deferred
    a.bail_min = 2 * kPiece;
    a.seg_gmax = seg_gmax;
    RH_HIP(launch_walk(a, cus, stream));
    // 2-6. piece-parallel framing of the deferred segments
    RH_HIP(hipMemsetAsync(pa.n_pieces, 0, sizeof(unsigned int), stream));
    hipLaunchKernelGGL(piece_plan_kernel, dim3(1), dim3(kScanThreads), 0, stream, pa);
    RH_HIP(hipGetLastError());
    if (RH_GUESS_REFILL)
        hipLaunchKernelGGL(piece_guess_wave_kernel, dim3((uint32_t)(kGuessWaveBlocksPerCu * cus)), dim3(64), 0, stream, pa);
    else
        hipLaunchKernelGGL(piece_guess_kernel, dim3((uint32_t)(kGuessBlocksPerCu * cus)), dim3(kPieceThreads), 0, stream, pa);
    RH_HIP(hipGetLastError());
    const uint64_t wgrid = (piece_cap + 255) / 256 < (uint64_t)cus * 8 ? (piece_cap + 255) / 256 : (uint64_t)cus * 8;
    hipLaunchKernelGGL(piece_walk_kernel, dim3((uint32_t)wgrid), dim3(256), 0, stream, pa);
    RH_HIP(hipGetLastError());
#ifdef RH_AB_FENCE_PROBE
    hipLaunchKernelGGL(empty_probe_kernel, dim3((uint32_t)n_seg), dim3(64), 0, stream, 0);
#endif
    hipLaunchKernelGGL(piece_stitch_kernel, dim3((uint32_t)n_seg), dim3(64), 0, stream, pa);
    RH_HIP(hipGetLastError());
    const uint64_t pgrid = (piece_cap + 3) / 4 < (uint64_t)cus * 8 ? (piece_cap + 3) / 4 : (uint64_t)cus * 8;
    hipLaunchKernelGGL(piece_write_kernel, dim3((uint32_t)pgrid), dim3(256), 0, stream, pa);
    RH_HIP(hipGetLastError());
    // 6. the deferred segments' ends (terminator check, rule-by-rule steps) and serial leftovers
    a.bail_min = 0;
    a.seg_gmax = nullptr;
    a.resume_pos = pa.resume_pos;
    a.resume_nfr = pa.resume_nfr;
    RH_HIP(launch_walk(a, cus, stream));
    hipLaunchKernelGGL(segment_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, g->seg_nframes, g->n_seg,
                       g->frames_per_seg_cap, g->seg_first, g->total_frames);
    RH_HIP(hipGetLastError());
    const uint64_t citems = g->n_seg * ((g->frames_per_seg_cap + kCompactSlots - 1) / kCompactSlots);
    const uint64_t cgrid = citems < (uint64_t)cus * 8 ? citems : (uint64_t)cus * 8;
    hipLaunchKernelGGL(segment_compact_kernel, dim3((uint32_t)cgrid), dim3(256), 0, stream, g->scratch_off,
                       g->scratch_len, g->seg_nframes, g->seg_first, g->n_seg, g->frames_per_seg_cap, g->frame_off,
                       g->frame_len, g->frame_cap);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
