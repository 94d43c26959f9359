// Fused SegmentedRaftLog read path on gfx950 (MI355X): the framing walk and the CRC32C
// verification of every frame in ONE pass over HBM.
//
// Reference semantics (ratis tree, ratis-server/.../raftlog/segmented/ unless noted):
//   LogSegment.readSegmentFile               LogSegment.java:166-196
//   SegmentedRaftLogReader.verifyHeader      SegmentedRaftLogReader.java:179-205
//   SegmentedRaftLogReader.decodeEntry       SegmentedRaftLogReader.java:291-341 (size/EOF rules,
//                                            CRC32C over varint||proto, big-endian trailer)
//   SegmentedRaftLogReader.verifyTerminator  SegmentedRaftLogReader.java:251-280
//   PureJavaCrc32C.reset/update/getValue     ratis-common/.../util/PureJavaCrc32C.java:43-91
//
// The two-pass path (segment_walk_kernel2, then crc_frames_kernel5 over the frame table) streams
// every segment byte from HBM twice.  Here one 1024-thread workgroup per CU owns one segment at a
// time and streams it once through a ring of four 16 KiB LDS windows (register-staged, two
// windows in flight ahead of the ring).  In step k:
//   * wave 0 walks the frames that START in window k.  The walk is a serial chain, so the wave
//     speculates on it: lane j decodes the header at p + j*s, s = the last frame's length, and the
//     run of lanes whose frame passes decodeEntry's common-case checks with length s is accepted
//     at once (exact: frame j+1 starts at p+(j+1)s iff frames 0..j all have length s).  Anything
//     else -- a different length, the terminator, an error, a frame longer than the ring -- is
//     decided rule by rule, in the order segment_walk_kernel2 applies the rules, for one frame.
//     Accepted frames go to the scratch frame table and to an LDS list, each frame's CRC span cut
//     into end-anchored units of 16 lanes x S bytes;
//   * waves 1-15 (60 groups of 16 lanes) fold the units listed in step k-1 straight out of the
//     ring: slicing-by-4 from 16 lane-interleaved copies of the tables (one v_perm per lookup
//     address), a per-lane zero advance to the unit end, a 16-lane DPP XOR reduce; the group that
//     finishes a frame's last unit (LDS counter) advances every unit register to the frame end in
//     parallel (lane u: nibble tables of "u units of zeros"), XOR-reduces, applies reset()'s
//     0xFFFFFFFF and compares the big-endian trailer.
// The steady-state step has no out-of-line calls, no fences and no spills, so the only waits on
// the window loads in flight are the ones that store them into the ring two steps later.
// Frames that do not fit the resident ring are folded by one group straight from HBM.
// Table/XOR integer work, no MFMA.  Algorithmic bytes = the segment bytes.
#include "rh_internal.h"

namespace {

constexpr int kWalking = 0;
constexpr int kTermPending = 100;

constexpr int kThreads = 1024;
constexpr int kW = 16384;                    // window bytes
constexpr int kRing = 4 * kW;                // resident ring: windows k-1 .. k+2
constexpr uint32_t kRMask = kRing - 1;
constexpr int kQ = 16;                       // lanes per unit
constexpr int kFCap = 128;                   // frames listed per step
constexpr int kUCap = 256;                   // units listed per step
constexpr int kGroups = (kThreads / 64 - 1) * (64 / kQ);  // 60 CRC groups (waves 1..15)
constexpr uint32_t kHbmUnit = 0xFFFFu;       // unit marker: fold the whole frame from HBM
constexpr int kChunk = 15;                   // unit registers combined per combine pass
constexpr uint32_t kNoCombine = 0x80000000u; // Frame.ufirst flag: CRC finished by its folder

// Dynamic LDS (the kernel declares no static LDS, so a byte offset is the LDS address itself).
// [0, 64 KiB): slicing tables, [256 e][4 k][16 c] u32 (addressed absolutely by fold4)
constexpr uint32_t kOffLane = 65536;                     // [8 k][16 nibble][16 lane]: lane -> unit end
constexpr uint32_t kOffUd = kOffLane + 8192;             // [8 k][16 nibble][16 d]: d units of zeros
constexpr uint32_t kOffRing = kOffUd + 8192;             // 4 windows + 16-byte mirror
constexpr uint32_t kOffFt = kOffRing + kRing + 16;       // [3][kFCap] Frame (walked, folded, combined)
constexpr uint32_t kOffUm = kOffFt + 3 * kFCap * 16;     // [3][kUCap] u32: frame | unit << 16
constexpr uint32_t kOffPart = kOffUm + 3 * kUCap * 4;    // [2][kUCap] u32: unit CRC registers
constexpr uint32_t kOffTrail = kOffPart + 2 * kUCap * 4; // [2][kFCap] u32: stored (big-endian) CRC
constexpr uint32_t kOffSh = kOffTrail + 2 * kFCap * 4;   // Shared
constexpr uint32_t kOffProf = kOffSh + 128;              // [16] u64: PROF counters
constexpr uint32_t kLdsBytes = kOffProf + 128;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct Frame {
    int64_t off;      // segment-relative start
    uint32_t len;     // whole frame: varint + proto + 4
    uint32_t ufirst;  // index of its first unit in the list | kNoCombine
};

struct Shared {
    long long pos;
    int status;
    uint32_t nfr;                     // frames found in the segment so far
    uint32_t nf[3], nu[3], fbase[3];  // per list buffer: frames, units, index of the first frame
    uint32_t first_bad;               // smallest frame index whose CRC did not verify
    uint32_t nbad;
    uint32_t stride;                  // the walker's speculation stride (last frame length)
    unsigned long long term_min;
};
static_assert(sizeof(Shared) <= 128, "Shared");

struct ReadArgs {
    const uint8_t* buf;
    int64_t buf_len;
    const uint64_t* seg_off;
    const uint64_t* seg_len;
    uint64_t n_seg;
    uint32_t max_op;
    uint32_t cap;
    uint64_t* scratch_off;
    uint32_t* scratch_len;
    uint32_t* scratch_crc;
    uint32_t* seg_nframes;
    int32_t* seg_status;
    uint64_t* seg_stop;
    uint32_t* seg_ok;
    int32_t* seg_rstatus;
    uint64_t* seg_rstop;
    unsigned long long* n_bad;
    const uint32_t* slice;  // [4][256]
    const uint32_t* rd;     // [8][16][16] lane -> unit end, then [8][16][16] d units (build_read_tables)
};

struct __attribute__((aligned(4))) u32x4s {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ uint32_t varint32_size(uint32_t v) {
    return (v >> 7) == 0 ? 1u : (v >> 14) == 0 ? 2u : (v >> 21) == 0 ? 3u : (v >> 28) == 0 ? 4u : 5u;
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u32 lds_u32x4;
typedef __attribute__((address_space(3))) Frame LFrame;
typedef __attribute__((address_space(3))) Shared LShared;

template <typename T>
__device__ __forceinline__ T* lds_at(uint32_t byte_addr) {
    return reinterpret_cast<T*>(static_cast<uintptr_t>(byte_addr));
}
__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) { return *lds_at<lds_u32>(byte_addr); }

// Barrier for LDS hand-offs only: the staged window loads stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// 16 bytes of the segment at window start w0 for thread t (bytes outside [0, L) read as zero).
__device__ __forceinline__ u32x4s load16(const uint8_t* seg, int64_t L, int64_t w0, int t) {
    const int64_t p = w0 + 16 * (int64_t)t;
    if (p >= 0 && p + 16 <= L) return *reinterpret_cast<const u32x4s*>(seg + p);
    uint32_t w[4] = {0, 0, 0, 0};
    if (p < L && p + 16 > 0)
        for (int k = p < 0 ? (int)-p : 0; k < 16 && p + k < L; ++k) w[k >> 2] |= (uint32_t)seg[p + k] << (8 * (k & 3));
    return u32x4s{w[0], w[1], w[2], w[3]};
}

// Window `win` into its ring slot (win & 3); slot 0 is mirrored past the ring end so an 8-byte
// read at any ring offset needs no wrap-around.
__device__ __forceinline__ void store16(int64_t win, const u32x4s& v, int t) {
    const uint32_t slot = (uint32_t)(win & 3);
    const v4u32 x = {v.x, v.y, v.z, v.w};
    *lds_at<lds_u32x4>(kOffRing + slot * kW + 16 * t) = x;
    if (slot == 0 && t == 0) *lds_at<lds_u32x4>(kOffRing + kRing) = x;
}

// 4 bytes of the segment at ring offset q (little-endian).
__device__ __forceinline__ uint32_t ring_peek4(uint32_t q) {
    const uint32_t q0 = q & ~3u;
    const uint32_t lo = lds_word(kOffRing + q0);
    const uint32_t hi = lds_word(kOffRing + q0 + 4);  // mirror covers q0 = kRing - 4
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (q & 3)));
}

// Slicing-by-4 step from the 16-copy tables: entry e of table k for lane copy c sits at byte
// e << 8 | k << 6 | c << 2, so the address of byte j of x is one v_perm into lb[k] = k << 6 | c << 2.
// Odd 16-lane groups swap the bytes of x pairwise (lb[4] = perm selector) and address tables k ^ 1
// (lb[k]), so the two groups of a half-wave read disjoint bank halves: conflict free.
__device__ __forceinline__ uint32_t fold4(uint32_t r, uint32_t w, const uint32_t (&lb)[5]) {
    const uint32_t x0 = r ^ w;
    const uint32_t x = __builtin_amdgcn_perm(x0, x0, lb[4]);
    return lds_word(__builtin_amdgcn_perm(x, lb[3], 0x03020400u)) ^ lds_word(__builtin_amdgcn_perm(x, lb[2], 0x03020500u)) ^
           lds_word(__builtin_amdgcn_perm(x, lb[1], 0x03020600u)) ^ lds_word(__builtin_amdgcn_perm(x, lb[0], 0x03020700u));
}

// Linear zero-advance of register r by the nibble tables at `tab` ([8 k][16 nibble][16 col]), column c.
__device__ __forceinline__ uint32_t nib_adv(uint32_t tab, uint32_t r, uint32_t c) {
    uint32_t z = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) z ^= lds_word(tab + ((((uint32_t)k * 16 + ((r >> (4 * k)) & 15u)) * 16 + c) << 2));
    return z;
}

// XOR over the 16 lanes of a DPP row; every lane gets the result.
__device__ __forceinline__ uint32_t row_xor16(uint32_t r) {
    r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x141, 0xF, 0xF, false);  // row_half_mirror
    r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x140, 0xF, 0xF, false);  // row_mirror
    return r;
}

// CRC register contribution of unit wi (of nwu) of the frame whose CRC span is [fo, fo + span),
// folded by a 16-lane group (lane gl); every lane returns the reduced value.  Unit wi covers
// [E - (nwu - wi) * U, E - (nwu - 1 - wi) * U) (E = fo + span), lane gl its S-byte slice gl.
// Bytes before fo are zeroed and reset()'s 0xFFFFFFFF is XOR-ed into the frame's first 4 bytes
// (CRC linearity: a zero register absorbing leading zeros stays zero).  Positions are relative to
// fo (spans < 2^31); the bytes come from the LDS ring at ring offset fq + position.
template <int S>
__device__ __forceinline__ uint32_t fold_unit(uint32_t fq, uint32_t sh, int32_t span, int nwu, int wi, int gl,
                                              const uint32_t (&lb)[5]) {
    constexpr int U = kQ * S;
    const int32_t be = span - (nwu - 1 - wi) * U - (kQ - 1 - gl) * S;  // lane chunk end, rel. to fo
    const bool act = be > 0;
    const int32_t b0 = be - S - (int32_t)sh;  // fo + b0 is 4-byte aligned in memory
    uint32_t d[S / 4 + 1];
    const uint32_t q = fq + (uint32_t)b0;
#pragma unroll
    for (int i = 0; i <= S / 4; ++i) d[i] = lds_word(kOffRing + ((q + 4u * i) & kRMask));
    if (act && b0 < 4) {
        const int qc = b0 < -48 ? -48 : b0;
#pragma unroll
        for (int i = 0; i <= S / 4; ++i) {
            const int qq = qc + 4 * i;
            uint32_t v = d[i];
            v = (qq <= -4) ? 0u : (qq < 0 ? (v & (0xFFFFFFFFu << (8 * -qq))) : v);
            const uint32_t up = (qq >= 0 && qq < 4) ? (0xFFFFFFFFu >> (8 * qq)) : 0u;
            const uint32_t dn = (qq < 0 && qq > -4) ? (0xFFFFFFFFu << (8 * -qq)) : 0u;
            d[i] = v ^ up ^ dn;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < S / 4; ++j) r = fold4(r, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), lb);
    r = nib_adv(kOffLane, r, (uint32_t)gl);
    return row_xor16(act ? r : 0u);
}

// Register-light twin of fold_unit<S, false> for frames folded straight from HBM (rare): the
// same lane slices and head handling, one dword at a time in a rolled loop (keeps the unrolled
// ring fold's register budget intact -- a spill would put a vmcnt(0) into every step).
template <int S>
__device__ __forceinline__ uint32_t fold_unit_hbm(const uint8_t* fseg, uint32_t sh, int32_t span, int nwu, int wi,
                                                  int gl, const uint32_t (&lb)[5]) {
    constexpr int U = kQ * S;
    const int32_t be = span - (nwu - 1 - wi) * U - (kQ - 1 - gl) * S;
    const bool act = be > 0;
    const int32_t b0 = be - S - (int32_t)sh;
    auto word = [&](int i) -> uint32_t {
        const int32_t p = b0 + 4 * i;
        uint32_t v = (act && p + 4 > 0 && p < span) ? *reinterpret_cast<const uint32_t*>(fseg + p) : 0u;
        if (p < 4) {  // bytes before the frame start -> 0; reset()'s 0xFFFFFFFF into bytes 0..3
            const int qq = p < -48 ? -48 : p;
            v = (qq <= -4) ? 0u : (qq < 0 ? (v & (0xFFFFFFFFu << (8 * -qq))) : v);
            v ^= (qq >= 0 && qq < 4) ? (0xFFFFFFFFu >> (8 * qq)) : 0u;
            v ^= (qq < 0 && qq > -4) ? (0xFFFFFFFFu << (8 * -qq)) : 0u;
        }
        return v;
    };
    uint32_t r = 0, prev = word(0);
#pragma unroll 1
    for (int j = 0; j < S / 4; ++j) {
        const uint32_t nx = word(j + 1);
        r = fold4(r, __builtin_amdgcn_alignbyte(nx, prev, sh), lb);
        prev = nx;
    }
    r = nib_adv(kOffLane, r, (uint32_t)gl);
    return row_xor16(act ? r : 0u);
}

// Tuning instrumentation (rh_segments_read_profile): per-block cycle counters, PROF kernels only.
// [0] segment loop, [1] walker (t 0), [2] fold+combine phase (t 64), [3] t 0 wait at the step-end
// barrier, [4] steps, [5] t 64 wait at the step-start barrier, [6] frames walked, [7] frames by
// speculation, [8] t 64 between the barriers (ring advance), [9] fold+combine phase (t 1008)
__device__ unsigned long long g_rd_prof[1024][16];
bool g_rd_prof_on = false;

// One walker step (wave 0, every lane, wave-uniform control flow): the frames that start in
// window k, decided by decodeEntry's rules, are recorded in the scratch frame table and listed
// (frame, units) in list buffer wb.  Returns the frames accepted by speculation.
template <int S>
__device__ __forceinline__ uint32_t walk_window(const ReadArgs& a, int64_t L, int64_t A, int64_t base, uint64_t slot0,
                                                int64_t k, int wb, int lane) {
    constexpr int U = kQ * S;
    const lds_u8* ring = lds_at<const lds_u8>(kOffRing);
    LShared& Sh = *lds_at<LShared>(kOffSh);
    const int64_t wend = A + (k + 1) * kW;
    const int64_t ring_hi = A + (k + 3) * kW;  // resident through the next step
    int64_t p = uniform64(Sh.pos);
    uint32_t nfr = uni(Sh.nfr), nf = 0, nu = 0, stride = uni(Sh.stride), spec = 0;
    const uint32_t cap = a.cap, max_op = a.max_op;
    int st = kWalking;
    LFrame* f = lds_at<LFrame>(kOffFt) + wb * kFCap;
    lds_u32* u = lds_at<lds_u32>(kOffUm) + wb * kUCap;
    // speculation bounds (32-bit positions): header bytes before pend, frame end before rhi
    const int64_t pend64 = wend < L - 8 ? wend : L - 8;
    const bool fast_ok = L <= 0x7fffffff;
    const uint32_t pend = pend64 > 0 ? (uint32_t)pend64 : 0u;
    const uint32_t rhi = ring_hi < L ? (uint32_t)ring_hi : (uint32_t)L;
    const uint32_t Aneg = (uint32_t)(-A);
    while (p < wend) {
        // ---- speculative run: lane j checks the frame at p + j * stride ----
        if (fast_ok && p < (int64_t)pend) {
            const uint32_t s = stride <= (1u << 25) ? stride : 0u;  // 63 * 2^25 + 2^31 < 2^32
            const uint32_t p32 = (uint32_t)p;
            const uint32_t c = p32 + (uint32_t)lane * s;
            const bool okp = lane == 0 || (s != 0 && c < pend);
            const uint32_t v = ring_peek4(((okp ? c : p32) + Aneg) & kRMask);
            const uint32_t stop4 = ~v & 0x80808080u;
            const uint32_t vl = (uint32_t)(__builtin_ctz(stop4 | 0x80000000u) >> 3) + 1;
            const uint32_t nn = ((v & 0x7fu) | ((v >> 1) & 0x3f80u) | ((v >> 2) & 0x1fc000u) | ((v >> 3) & 0xfe00000u)) &
                                (0xffffffffu >> (32 - 7 * vl));
            const uint32_t fl = varint32_size(nn) + nn + 4;  // nn < 2^28: no overflow
            // common case of decodeEntry: non-zero first byte, <= 4-byte varint, frame within
            // maxOpSize and EOF (and, here, inside the resident ring)
            const uint32_t room = okp && c < rhi ? rhi - c : 0u;
            const uint32_t lim = max_op < room ? max_op : room;
            bool ok = okp && (v & 0xffu) != 0 && stop4 != 0 && fl <= lim && nfr + (uint32_t)lane < cap;
            const uint32_t fl0 = uni(fl);
            if (lane != 0) ok = ok && fl == s && fl0 == s;
            const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
            uint32_t nacc = ~m ? (uint32_t)__builtin_ctzll(~m) : 64u;
            const uint32_t nw = (fl0 - 4 + U - 1) / U;
            if (nacc) {
                if (nacc > kFCap - nf) nacc = kFCap - nf;
                if (nu + nacc * nw > kUCap) nacc = (kUCap - nu) / nw;
            }
            nacc = uni(nacc);
            if (nacc) {
                if ((uint32_t)lane < nacc) {
                    const uint32_t cj = p32 + (uint32_t)lane * fl0;
                    a.scratch_off[slot0 + nfr + lane] = (uint64_t)base + cj;
                    a.scratch_len[slot0 + nfr + lane] = fl0;
                    f[nf + lane].off = cj;
                    f[nf + lane].len = fl0;
                    f[nf + lane].ufirst = (nu + (uint32_t)lane * nw) | (nw == 1 ? kNoCombine : 0u);
                }
                // unit entries, the whole wave at once: entry e = frame e / nw, unit e % nw
                const uint32_t ne = nacc * nw;
#pragma clang loop vectorize(disable) unroll(disable)
                for (uint32_t e = (uint32_t)lane; e < ne; e += 64) {
                    const uint32_t fj = e / nw;
                    u[nu + e] = (nf + fj) | ((e - fj * nw) << 16);
                }
                p += (int64_t)nacc * fl0;
                nfr += nacc;
                nf += nacc;
                nu += nacc * nw;
                stride = fl0;
                spec += nacc;
                continue;
            }
        }
        // ---- one frame, rule by rule (decodeEntry, RDR:291-341) ----
        if (p >= L) {
            st = RH_SEG_END;
            break;
        }
        const uint32_t q = (uint32_t)((p - A) & kRMask);
        const uint32_t q0 = q & ~3u;
        const uint32_t lo = uni(*reinterpret_cast<const lds_u32*>(ring + q0));  // scalar from here
        const uint32_t hi = uni(*reinterpret_cast<const lds_u32*>(ring + q0 + 4));  // mirror
        const uint64_t x = ((uint64_t)hi << 32 | lo) >> (8 * (q & 3));
        if ((x & 0xff) == 0) {  // terminator (SegmentedRaftLogFormat.isTerminator)
            st = kTermPending;
            break;
        }
        // CodedInputStream.readRawVarint32(firstByte, in): 7 bits per byte, int
        // arithmetic; EOF inside the varint -> truncatedMessage
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
            bool fin = false;
            for (int i = 5; i < 10 && i < avail; ++i) {
                if ((uni(ring[(uint32_t)(p + i - A) & kRMask]) & 0x80) == 0) {
                    fin = true;
                    break;
                }
            }
            if (!fin) {
                st = RH_SEG_E_VARINT;
                break;
            }
        }
        const int32_t n = (int32_t)result;
        if (n > (int32_t)max_op) {
            st = RH_SEG_E_OVERSIZE;
            break;
        }
        if (n < 0) {
            st = RH_SEG_E_VARINT;
            break;
        }
        const int64_t total = (int64_t)varint32_size((uint32_t)n) + n;
        if (total > (int64_t)max_op) {  // checkBufferSize
            st = RH_SEG_E_OVERSIZE;
            break;
        }
        if (p + total > L) {  // readFully EOF
            st = RH_SEG_PARTIAL;
            break;
        }
        // readInt: checkLimit(1) before each of the 4 reads (RDR:66-82)
        const int64_t lim_room = (int64_t)max_op - total, eof_room = L - p - total;
        if (lim_room < 4 || eof_room < 4) {
            st = lim_room <= eof_room ? RH_SEG_E_OVERSIZE : RH_SEG_PARTIAL;
            break;
        }
        if (nfr >= cap) {
            st = RH_SEG_E_CAPACITY;
            break;
        }
        const int64_t fl = total + 4;
        const uint32_t nwu = (uint32_t)((total + U - 1) / U);
        const bool in_ring = p + fl <= ring_hi;
        const uint32_t need = in_ring ? nwu : 1u;
        if (nf == kFCap || nu + need > kUCap) break;  // list full: resume here next step
        if (lane == 0) {
            a.scratch_off[slot0 + nfr] = (uint64_t)(base + p);
            a.scratch_len[slot0 + nfr] = (uint32_t)fl;
            f[nf].off = p;
            f[nf].len = (uint32_t)fl;
            f[nf].ufirst = nu | (in_ring && nwu > 1 ? 0u : kNoCombine);
        }
#pragma clang loop vectorize(disable) unroll(disable)
        for (uint32_t w = (uint32_t)lane; w < need; w += 64) u[nu + w] = nf | ((in_ring ? w : kHbmUnit) << 16);
        ++nfr;
        ++nf;
        nu += need;
        p += fl;
        stride = (uint32_t)fl;
    }
    if (lane == 0) {
        Sh.status = st;
        Sh.pos = p;
        Sh.nfr = nfr;
        Sh.stride = stride;
        Sh.nf[wb] = nf;
        Sh.nu[wb] = nu;
        Sh.fbase[wb] = nfr - nf;
    }
    return spec;
}

template <int S, bool PROF>
__global__ __launch_bounds__(kThreads) void segment_read_kernel(ReadArgs a) {
    constexpr int U = kQ * S;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_at assumes base 0
    uint32_t* L32 = reinterpret_cast<uint32_t*>(lds);
    LFrame* ft = lds_at<LFrame>(kOffFt);
    lds_u32* um = lds_at<lds_u32>(kOffUm);
    lds_u32* part = lds_at<lds_u32>(kOffPart);
    lds_u32* trail = lds_at<lds_u32>(kOffTrail);
    LShared& Sh = *lds_at<LShared>(kOffSh);
    const lds_u8* ring = lds_at<const lds_u8>(kOffRing);

    const int t = threadIdx.x;
    for (int i = t; i < 16384; i += kThreads) L32[i] = a.slice[((i >> 4) & 3) * 256 + (i >> 6)];
    for (int i = t; i < 4096; i += kThreads) L32[kOffLane / 4 + i] = a.rd[i];
    const int wave = t >> 6;
    const int lane = t & 63;
    const int gl = t & 15;
    const int grp = (wave - 1) * 4 + ((t >> 4) & 3);
    const uint32_t gpar = (uint32_t)(t >> 4) & 1u;
    uint32_t lb[5];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = (((uint32_t)k ^ gpar) << 6) | ((uint32_t)gl << 2);
    lb[4] = gpar ? 0x02030001u : 0x03020100u;
    typedef __attribute__((address_space(3))) unsigned long long lds_u64;
    lds_u64* pc = lds_at<lds_u64>(kOffProf);  // PROF counters, kept out of the VGPR budget
    if (PROF && t < 16) pc[t] = 0;
    __syncthreads();

    for (uint64_t s = blockIdx.x; s < a.n_seg; s += gridDim.x) {
        const unsigned long long t_seg = PROF ? __builtin_readcyclecounter() : 0;
        const int64_t base = uniform64((int64_t)a.seg_off[s]);
        int64_t L = (int64_t)a.seg_len[s];
        if (base > a.buf_len) L = 0;
        else if (L > a.buf_len - base) L = a.buf_len - base;  // never read past the buffer
        L = uniform64(L);
        const uint8_t* seg = a.buf + base;
        const int64_t A = (base & ~(int64_t)15) - base;  // window grid origin: seg + A is 16-B aligned
        const uint32_t Aneg = (uint32_t)(-A);
        const uint64_t slot0 = s * (uint64_t)a.cap;
        if (t == 0) {  // verifyHeader (RDR:179-205)
            const char H[8] = {'R', 'a', 'f', 't', 'L', 'o', 'g', '1'};
            const int64_t rl = L < 8 ? L : 8;
            int match = 0, bad = 0;
            for (int i = 0; i < rl; ++i) {
                const uint8_t b = seg[i];
                if (match == i && b == (uint8_t)H[i]) match = i + 1;
                else if (b != 0) bad = 1;
            }
            const bool ok = rl == 8 && match == 8;
            Sh.status = ok ? (8 >= L ? RH_SEG_END : kWalking) : (bad ? RH_SEG_E_HEADER : RH_SEG_END);
            Sh.pos = ok ? 8 : 0;
            Sh.nfr = 0;
            Sh.stride = 0;
            for (int i = 0; i < 3; ++i) Sh.nf[i] = Sh.nu[i] = Sh.fbase[i] = 0;
            Sh.first_bad = 0xFFFFFFFFu;
            Sh.nbad = 0;
        }
        __syncthreads();
        int status = Sh.status;
        int64_t pos = Sh.pos;

        // Three-stage pipeline over list buffers: in step `stp` the walker fills list stp % 3,
        // the folders fold the units of list (stp - 1) % 3 into part[stp & 1], and the combiners
        // finish the frames of list (stp - 2) % 3 from part[~stp & 1] and trail[~stp & 1].
        // mode: 0 walk, 1 prime the ring then walk, 2 drain one step (fold) then prime,
        // 3 drain two steps (fold, combine) then finish, 4 finished
        int mode = status == kWalking ? 1 : 4;
        int64_t k = 0;
        uint32_t stp = 0;
        int drain = 0;
        bool adv = false;
        u32x4s R0{0, 0, 0, 0}, R1{0, 0, 0, 0};  // windows k+3, k+4 in flight (R1: even windows)
        while (mode != 4) {
            if (mode == 1) {
                k = (pos - A) / kW;
                const u32x4s w0 = load16(seg, L, A + k * kW, t);
                const u32x4s w1 = load16(seg, L, A + (k + 1) * kW, t);
                const u32x4s w2 = load16(seg, L, A + (k + 2) * kW, t);
                store16(k, w0, t);
                store16(k + 1, w1, t);
                store16(k + 2, w2, t);
                if (k & 1) {
                    R1 = load16(seg, L, A + (k + 3) * kW, t);
                    R0 = load16(seg, L, A + (k + 4) * kW, t);
                } else {
                    R0 = load16(seg, L, A + (k + 3) * kW, t);
                    R1 = load16(seg, L, A + (k + 4) * kW, t);
                }
                mode = 0;
            }
            const uint32_t wl = stp % 3, fl3 = (stp + 2) % 3, cl3 = (stp + 1) % 3;
            const uint32_t pbw = stp & 1, pbr = pbw ^ 1;
            unsigned long long t0 = PROF ? __builtin_readcyclecounter() : 0;
            lds_barrier();  // ring holds windows k-1..k+1 (+ k+2); the previous step's lists are complete
            if (adv) {
                // deferred advance: window k+2 into the slot of window k-2 (folded last step); it
                // is first read next step, and this step's own stores are not yet in the wave's
                // vmcnt queue ahead of the staged load
                if (k & 1) {
                    store16(k + 2, R0, t);
                    R0 = load16(seg, L, A + (k + 4) * kW, t);
                } else {
                    store16(k + 2, R1, t);
                    R1 = load16(seg, L, A + (k + 4) * kW, t);
                }
                adv = false;
            }
            const unsigned long long t1 = PROF ? __builtin_readcyclecounter() : 0;
            if (PROF && t == 64) pc[5] += t1 - t0;
            if (PROF && t == 0) pc[4] += 1;
            if (wave == 0) {
                __builtin_amdgcn_s_setprio(3);  // the serial walk is the step's critical path
                if (mode == 0) {
                    const uint32_t nfr0 = PROF ? Sh.nfr : 0;
                    const uint32_t sp = walk_window<S>(a, L, A, base, slot0, k, (int)wl, lane);
                    if (PROF && lane == 0) {
                        pc[6] += Sh.nfr - nfr0;
                        pc[7] += sp;
                    }
                } else if (lane == 0) {
                    Sh.nf[wl] = 0;
                    Sh.nu[wl] = 0;
                }
                __builtin_amdgcn_s_setprio(0);
            } else {
                // ---- fold: units of list fl3 (RDR:327-336) ----
                {
                    const uint32_t nu_p = Sh.nu[fl3], fbase = Sh.fbase[fl3];
                    const LFrame* f = ft + fl3 * kFCap;
                    const lds_u32* u = um + fl3 * kUCap;
                    for (uint32_t x = (uint32_t)grp; x < nu_p; x += kGroups) {
                        const uint32_t e = u[x];
                        const uint32_t j = e & 0xFFFFu, wi = e >> 16;
                        const int64_t fo = f[j].off;
                        const int32_t span = (int32_t)f[j].len - 4;  // varint + proto
                        const int nwu = (span + U - 1) / U;
                        const uint32_t sh = (uint32_t)(base + fo + span) & 3u;
                        uint32_t R;
                        const uint8_t* tr;  // big-endian trailer bytes
                        if (wi == kHbmUnit) {
                            const uint8_t* fseg = seg + fo;
                            R = 0;
#pragma unroll 1
                            for (int w = 0; w < nwu; ++w)
                                R = nib_adv(kOffUd, R, 1u) ^ fold_unit_hbm<S>(fseg, sh, span, nwu, w, gl, lb);
                            tr = fseg + span;
                        } else {
                            R = fold_unit<S>((uint32_t)fo + Aneg, sh, span, nwu, (int)wi, gl, lb);
                            tr = nullptr;
                        }
                        uint32_t stored = 0;
                        if (gl == 0 && (wi == kHbmUnit || (int)wi == nwu - 1)) {
                            uint32_t b[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                b[i] = tr ? tr[i] : ring[(uint32_t)(fo + span + i - A) & kRMask];
                            stored = (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3];
                        }
                        if (gl == 0) {
                            if (wi == kHbmUnit || nwu == 1) {
                                // getValue() after reset(); update(frame, 0, span)
                                const uint32_t value = ~(R ^ (span < 4 ? 0xFFFFFFFFu >> (8 * span) : 0u));
                                const uint32_t idx = fbase + j;
                                a.scratch_crc[slot0 + idx] = value;
                                if (stored != value) {
                                    __hip_atomic_fetch_min(&Sh.first_bad, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    __hip_atomic_fetch_add(&Sh.nbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                            } else {
                                part[pbw * kUCap + x] = R;
                                if ((int)wi == nwu - 1) trail[pbw * kFCap + j] = stored;
                            }
                        }
                    }
                }
                // ---- combine: frames of list cl3, every unit register advanced to the frame end
                // in parallel (lane g takes unit c0 + g, d = units after it in its chunk) ----
                {
                    const uint32_t nf_c = Sh.nf[cl3], fbase = Sh.fbase[cl3];
                    const LFrame* f = ft + cl3 * kFCap;
                    for (uint32_t j = (uint32_t)(kGroups - 1 - grp); j < nf_c; j += kGroups) {
                        const uint32_t uf = f[j].ufirst;
                        if (uf & kNoCombine) continue;
                        const int32_t span = (int32_t)f[j].len - 4;
                        const int nwu = (span + U - 1) / U;
                        uint32_t R = 0;
                        for (int c0 = 0; c0 < nwu; c0 += kChunk) {
                            const int m = nwu - c0 < kChunk ? nwu - c0 : kChunk;
                            const uint32_t pv = gl < m ? part[pbr * kUCap + uf + c0 + gl] : 0u;
                            const uint32_t z = gl < m ? nib_adv(kOffUd, pv, (uint32_t)(m - 1 - gl)) : 0u;
                            R = nib_adv(kOffUd, R, (uint32_t)m) ^ row_xor16(z);
                        }
                        if (gl == 0) {
                            const uint32_t value = ~(R ^ (span < 4 ? 0xFFFFFFFFu >> (8 * span) : 0u));
                            const uint32_t idx = fbase + j;
                            a.scratch_crc[slot0 + idx] = value;
                            if (trail[pbr * kFCap + j] != value) {
                                __hip_atomic_fetch_min(&Sh.first_bad, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                __hip_atomic_fetch_add(&Sh.nbad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        }
                    }
                }
            }
            if (PROF) {
                t0 = __builtin_readcyclecounter();
                if (t == 0) pc[1] += t0 - t1;
                if (t == 64) pc[2] += t0 - t1;
                if (t == 1008) pc[9] += t0 - t1;
            }
            lds_barrier();  // the walk, folds and combines of this step are done
            const unsigned long long t2 = PROF ? __builtin_readcyclecounter() : 0;
            if (PROF && t == 0) pc[3] += t2 - t0;
            ++stp;
            if (mode == 3) {
                if (--drain == 0) break;
                continue;
            }
            if (mode == 2) {
                mode = 1;
                continue;
            }
            status = Sh.status;
            pos = Sh.pos;
            if (status != kWalking) {
                mode = 3;  // fold the last list, then combine it
                drain = 2;
            } else if (pos >= A + (k + 2) * kW) {
                mode = 2;  // a frame jumped past the ring: fold the list, restart at pos
            } else if (pos >= A + (k + 1) * kW) {
                ++k;  // advance; window k+2 is stored at the start of the next step
                adv = true;
            }
            // else the list filled up inside window k: walk it again next step
            if (PROF && t == 64) pc[8] += __builtin_readcyclecounter() - t2;
        }

        if (status == kTermPending) {
            // verifyTerminator (RDR:251-280): the first non-zero byte in [pos, L), block-wide
            if (t == 0) Sh.term_min = (unsigned long long)L;
            __syncthreads();
            const int64_t q0 = ((base + pos) & ~(int64_t)15) - base;
            bool found = false;
            for (int64_t q = q0; q < L && !found; q += kW) {
                const u32x4s c = load16(seg, L, q, t);
                const uint32_t ww[4] = {c.x, c.y, c.z, c.w};
                unsigned long long my = (unsigned long long)L;
                const int64_t p = q + 16 * (int64_t)t;
                for (int j = 0; j < 4; ++j) {
                    if (ww[j] == 0) continue;
                    for (int bb = 0; bb < 4; ++bb) {
                        const int64_t pb = p + 4 * j + bb;
                        if (((ww[j] >> (8 * bb)) & 0xff) && pb >= pos && pb < L && (unsigned long long)pb < my)
                            my = (unsigned long long)pb;
                    }
                }
                if (my < (unsigned long long)L)
                    __hip_atomic_fetch_min(&Sh.term_min, my, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __syncthreads();
                found = Sh.term_min < (unsigned long long)L;
                __syncthreads();
            }
            if (found) {
                status = RH_SEG_E_PADDING;
                pos = (int64_t)Sh.term_min;
            } else {
                status = RH_SEG_END;  // stop stays at the terminator (the segment's logical end)
            }
        }
        if (t == 0) {
            const uint32_t nfr = Sh.nfr, fb = Sh.first_bad;
            const bool bad = fb < nfr;
            a.seg_nframes[s] = nfr;
            a.seg_status[s] = status;
            a.seg_stop[s] = (uint64_t)pos;
            a.seg_ok[s] = bad ? fb : nfr;
            a.seg_rstatus[s] = bad ? RH_SEG_E_CHECKSUM : status;
            a.seg_rstop[s] = bad ? a.scratch_off[slot0 + fb] - (uint64_t)base : (uint64_t)pos;
            if (a.n_bad && Sh.nbad) atomicAdd(a.n_bad, (unsigned long long)Sh.nbad);
        }
        __syncthreads();
        if (PROF && t == 0) pc[0] += __builtin_readcyclecounter() - t_seg;
    }
    if (PROF && blockIdx.x < 1024) {
        __syncthreads();
        if (t < 16) g_rd_prof[blockIdx.x][t] += pc[t];
    }
}

// Dense frame table + CRC results: segment s's frames land at seg_first[s]...; the mismatch bit
// compares the computed CRC with the frame's stored big-endian trailer.
__global__ __launch_bounds__(256) void segment_compact_crc_kernel(ReadArgs a, const uint64_t* seg_first,
                                                                  uint64_t* frame_off, uint32_t* frame_len,
                                                                  uint64_t frame_cap, uint32_t* crc_out,
                                                                  uint64_t* bad_bits) {
    for (uint64_t s = blockIdx.x; s < a.n_seg; s += gridDim.x) {
        const uint32_t n = a.seg_nframes[s] < a.cap ? a.seg_nframes[s] : a.cap;
        const uint64_t first = seg_first[s];
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t d = first + i;
            if (d >= frame_cap) break;
            const uint64_t o = a.scratch_off[s * (uint64_t)a.cap + i];
            const uint32_t l = a.scratch_len[s * (uint64_t)a.cap + i];
            const uint32_t c = a.scratch_crc[s * (uint64_t)a.cap + i];
            frame_off[d] = o;
            frame_len[d] = l;
            if (crc_out) crc_out[d] = c;
            if (bad_bits) {
                const uint8_t* tr = a.buf + o + l - 4;
                const uint32_t stored = ((uint32_t)tr[0] << 24) | ((uint32_t)tr[1] << 16) | ((uint32_t)tr[2] << 8) | tr[3];
                if (stored != c) atomicOr(reinterpret_cast<unsigned long long*>(bad_bits + (d >> 6)), 1ull << (d & 63));
            }
        }
    }
}

// Fused-read variants (identical results): the unit's lane slice S in bytes.
// 0 / 1: segment_read_kernel with 36 / 20-byte CRC units (one pass over HBM, LDS ring);
// 2 (default): framing walk (segment_walk_kernel2, header fast-forward) then crc_frames_kernel8 over
// the slotted frame table, then the verdict -- two passes, but the walk reads headers only.
constexpr int kNumReadVariants = 3;
constexpr int kReadS[kNumReadVariants] = {36, 20, 0};
int g_read_variant = 2;

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

template <int S>
hipError_t launch_read(const ReadArgs& a, uint64_t grid, hipStream_t stream) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(segment_read_kernel<S, false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(segment_read_kernel<S, true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (g_rd_prof_on)
        hipLaunchKernelGGL((segment_read_kernel<S, true>), dim3((uint32_t)grid), dim3(kThreads), kLdsBytes, stream, a);
    else
        hipLaunchKernelGGL((segment_read_kernel<S, false>), dim3((uint32_t)grid), dim3(kThreads), kLdsBytes, stream, a);
    return hipGetLastError();
}

// Host: the fused kernel's advance tables for lane slice S (unit U = 16 S):
// [8 k][16 nibble][16 lane]: lane g -> unit end (S (15 - g) zero bytes), then
// [8 k][16 nibble][16 d]: d units (d U zero bytes).  Nibble tables from byte tables: the image
// of nibble v at nibble position k is byte table k/2 at v << 4 (k & 1).
std::vector<uint32_t> build_read_tables(int S) {
    std::vector<uint32_t> out(4096);
    uint32_t tab[4][256];
    for (int c = 0; c < 16; ++c) {
        rh::build_crc_shift_table((uint64_t)S * (uint64_t)(15 - c), tab);
        for (int k = 0; k < 8; ++k)
            for (int v = 0; v < 16; ++v) out[(k * 16 + v) * 16 + c] = tab[k >> 1][v << (4 * (k & 1))];
    }
    for (int d = 0; d < 16; ++d) {
        rh::build_crc_shift_table((uint64_t)16 * S * (uint64_t)d, tab);
        for (int k = 0; k < 8; ++k)
            for (int v = 0; v < 16; ++v) out[2048 + (k * 16 + v) * 16 + d] = tab[k >> 1][v << (4 * (k & 1))];
    }
    return out;
}

}  // namespace

int rh_segments_read_set_variant_impl(int v) {
    if (v < 0 || v >= kNumReadVariants)
        return rh::fail(RH_E_RANGE, "rh_segments_read_set_variant: variant out of range [0, 2]");
    g_read_variant = v;
    return RH_OK;
}

int rh_segments_read_impl(rh_ctx* ctx, const rh_segments* g, const rh_segments_crc* c, hipStream_t stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: ctx == NULL");
    if (!g || !c) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: segs/crc == NULL");
    if (g->n_seg == 0) return RH_OK;
    if (!g->buf || !g->seg_off || !g->seg_len || !g->scratch_off || !g->scratch_len || !g->frame_off ||
        !g->frame_len || !g->seg_first || !g->seg_nframes || !g->seg_status || !g->seg_stop || !g->total_frames)
        return rh::fail(RH_E_INVAL, "rh_segments_read_launch: every rh_segments array is required");
    if (!c->scratch_crc || !c->seg_ok || !c->seg_read_status || !c->seg_read_stop)
        return rh::fail(RH_E_INVAL, "rh_segments_read_launch: scratch_crc, seg_ok, seg_read_status, seg_read_stop required");
    if (g->frames_per_seg_cap == 0) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: frames_per_seg_cap == 0");
    if (g->max_op == 0 || g->max_op > 0x7FFFFFFFu) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: bad max_op");
    if (g->buf_len > (uint64_t)INT64_MAX) return rh::fail(RH_E_RANGE, "rh_segments_read_launch: buf_len too large");
    if (!ctx->d_slice) return rh::fail(RH_E_STATE, "rh_segments_read_launch: CRC tables not uploaded");
    const int v = g_read_variant;
    if (v == 2) {
        int rc = rh_segments_launch_impl(ctx, g, stream);  // walk + scan + compaction
        if (rc != RH_OK) return rc;
        RH_HIP(hipMemsetAsync(c->seg_ok, 0xFF, (size_t)g->n_seg * 4, stream));
        rc = rh_crc_verify_slots(ctx, g, c, stream);
        if (rc != RH_OK) return rc;
        if (c->crc_out || c->bad_bits) {  // dense per-frame CRCs / mismatch bits
            if (c->bad_bits) RH_HIP(hipMemsetAsync(c->bad_bits, 0, (size_t)((g->frame_cap + 63) / 64) * 8, stream));
            ReadArgs a{};
            a.buf = g->buf;
            a.n_seg = g->n_seg;
            a.cap = g->frames_per_seg_cap;
            a.scratch_off = g->scratch_off;
            a.scratch_len = g->scratch_len;
            a.scratch_crc = c->scratch_crc;
            a.seg_nframes = g->seg_nframes;
            const int cus = ctx->num_cus > 0 ? ctx->num_cus : 256;
            const uint64_t cgrid = g->n_seg < (uint64_t)cus * 8 ? g->n_seg : (uint64_t)cus * 8;
            hipLaunchKernelGGL(segment_compact_crc_kernel, dim3((uint32_t)cgrid), dim3(256), 0, stream, a, g->seg_first,
                               g->frame_off, g->frame_len, g->frame_cap, c->crc_out, c->bad_bits);
            RH_HIP(hipGetLastError());
        }
        const uint64_t vgrid = (g->n_seg + 255) / 256 < 1024 ? (g->n_seg + 255) / 256 : 1024;
        hipLaunchKernelGGL(segment_verdict_kernel, dim3((uint32_t)vgrid), dim3(256), 0, stream, g->seg_off, g->seg_nframes,
                           g->seg_status, g->seg_stop, g->scratch_off, g->n_seg, g->frames_per_seg_cap, c->seg_ok,
                           c->seg_read_status, c->seg_read_stop);
        RH_HIP(hipGetLastError());
        return RH_OK;
    }
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (!ctx->d_read_tables[v]) {
            const std::vector<uint32_t> t = build_read_tables(kReadS[v]);
            RH_HIP(hipMalloc(&ctx->d_read_tables[v], t.size() * 4));
            RH_HIP(hipMemcpy(ctx->d_read_tables[v], t.data(), t.size() * 4, hipMemcpyHostToDevice));
        }
    }
    ReadArgs a{};
    a.buf = g->buf;
    a.buf_len = (int64_t)g->buf_len;
    a.seg_off = g->seg_off;
    a.seg_len = g->seg_len;
    a.n_seg = g->n_seg;
    a.max_op = g->max_op;
    a.cap = g->frames_per_seg_cap;
    a.scratch_off = g->scratch_off;
    a.scratch_len = g->scratch_len;
    a.scratch_crc = c->scratch_crc;
    a.seg_nframes = g->seg_nframes;
    a.seg_status = g->seg_status;
    a.seg_stop = g->seg_stop;
    a.seg_ok = c->seg_ok;
    a.seg_rstatus = c->seg_read_status;
    a.seg_rstop = c->seg_read_stop;
    a.n_bad = c->n_bad;
    a.slice = ctx->d_slice;
    a.rd = ctx->d_read_tables[v];
    const int cus = ctx->num_cus > 0 ? ctx->num_cus : 256;
    const uint64_t grid = g->n_seg < (uint64_t)cus ? g->n_seg : (uint64_t)cus;
    RH_HIP(v == 0 ? launch_read<36>(a, grid, stream) : launch_read<20>(a, grid, stream));
    int rc = rh_segments_scan_counts(g->seg_nframes, g->n_seg, g->frames_per_seg_cap, g->seg_first, g->total_frames,
                                     stream);
    if (rc != RH_OK) return rc;
    if (c->bad_bits) RH_HIP(hipMemsetAsync(c->bad_bits, 0, (size_t)((g->frame_cap + 63) / 64) * 8, stream));
    const uint64_t cgrid = g->n_seg < (uint64_t)cus * 8 ? g->n_seg : (uint64_t)cus * 8;
    hipLaunchKernelGGL(segment_compact_crc_kernel, dim3((uint32_t)cgrid), dim3(256), 0, stream, a, g->seg_first,
                       g->frame_off, g->frame_len, g->frame_cap, c->crc_out, c->bad_bits);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_segments_read_profile_impl(int enable, uint64_t* out, uint64_t n) {
    if (out && n) {
        RH_HIP(hipDeviceSynchronize());
        const uint64_t m = n < 1024 * 16 ? n : 1024 * 16;
        RH_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rd_prof), m * sizeof(uint64_t), 0, hipMemcpyDeviceToHost));
    }
    if (enable >= 0) {
        if (enable) {
            static const unsigned long long zero[1024 * 16] = {};
            RH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rd_prof), zero, sizeof(zero), 0, hipMemcpyHostToDevice));
        }
        g_rd_prof_on = enable != 0;
    }
    return RH_OK;
}
