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
//   * wave 0, lane 0 walks the frames that START in window k with decodeEntry's rule-by-rule
//     checks (the same decisions as segment_walk_kernel2) and lists them in an LDS frame table,
//     each frame's CRC span cut into end-anchored 576-byte units (16 lanes x 36 bytes);
//   * waves 1-15 (60 groups of 16 lanes) fold the units listed in step k-1 straight out of the
//     ring: slicing-by-4 from 16 lane-interleaved copies of the tables (one v_perm per lookup
//     address, as crc_frames_kernel5), a per-lane zero advance to the unit end, a 16-lane XOR
//     reduce; the group that finishes a frame's last unit (LDS counter) combines the units with
//     576-byte zero advances, applies reset()'s 0xFFFFFFFF and compares the trailer.
// A 36-byte lane stride (9 dwords, odd) puts the 16 ring reads of a group on 16 distinct banks.
// Frames that do not fit the resident ring (longer than ~2 windows) are folded by one group
// straight from HBM.  Table/XOR integer work, no MFMA.  Algorithmic bytes = the segment bytes.
#include "rh_internal.h"

namespace {

constexpr int kWalking = 0;
constexpr int kTermPending = 100;

constexpr int kThreads = 1024;
constexpr int kW = 16384;                    // window bytes
constexpr int kRing = 4 * kW;                // resident ring: windows k-1 .. k+2
constexpr uint32_t kRMask = kRing - 1;
constexpr int kQ = 16, kS = 36, kU = kQ * kS;  // unit = 16 lanes x 36 B = 576 B
constexpr int kFCap = 256;                   // frames listed per step
constexpr int kUCap = 512;                   // units listed per step
constexpr int kGroups = (kThreads / 64 - 1) * (64 / kQ);  // 60 CRC groups (waves 1..15)
constexpr uint32_t kHbmUnit = 0xFFFFu;       // unit marker: fold the whole frame from HBM

// Dynamic LDS (the kernel declares no static LDS, so a byte offset is the LDS address itself).
// [0, 64 KiB): slicing tables, [256 e][4 k][16 c] u32 (addressed absolutely by fold4)
constexpr uint32_t kOffLane = 65536;                     // [8 k][16 nibble][16 lane] u32 = 8 KiB
constexpr uint32_t kOffZu = kOffLane + 8192;             // [4][256] u32: advance over 576 zeros
constexpr uint32_t kOffRing = kOffZu + 4096;             // 4 windows + 16-byte mirror
constexpr uint32_t kOffFt = kOffRing + kRing + 16;       // [2][kFCap] Frame
constexpr uint32_t kOffUm = kOffFt + 2 * kFCap * 16;     // [2][kUCap] u32: frame | unit << 16
constexpr uint32_t kOffPart = kOffUm + 2 * kUCap * 4;    // [kUCap] u32: unit CRC registers
constexpr uint32_t kOffDone = kOffPart + kUCap * 4;      // [kFCap] u32: units finished per frame
constexpr uint32_t kOffSh = kOffDone + kFCap * 4;        // Shared
constexpr uint32_t kLdsBytes = kOffSh + 128;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct Frame {
    int64_t off;   // segment-relative start
    uint32_t len;  // whole frame: varint + proto + 4
    uint32_t pad;
};

struct Shared {
    long long pos;
    int status;
    uint32_t nfr;                     // frames found in the segment so far
    uint32_t nf[2], nu[2], fbase[2];  // per list buffer: frames, units, index of the first frame
    uint32_t first_bad;               // smallest frame index whose CRC did not verify
    uint32_t nbad;
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
    const uint32_t* lane;   // rh::build_crc_lane_tables(16, 36): [8][16][32]
    const uint32_t* zu;     // [4][256]: advance over 576 zero bytes
};

struct __attribute__((aligned(4))) u32x4s {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ int varint32_size(uint32_t v) {
    return (v >> 7) == 0 ? 1 : (v >> 14) == 0 ? 2 : (v >> 21) == 0 ? 3 : (v >> 28) == 0 ? 4 : 5;
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) {
    return *reinterpret_cast<lds_u32_t*>(static_cast<uintptr_t>(byte_addr));
}

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
__device__ __forceinline__ void store16(uint8_t* ring, int64_t win, const u32x4s& v, int t) {
    const int slot = (int)(win & 3);
    *reinterpret_cast<u32x4s*>(ring + slot * kW + 16 * t) = v;
    if (slot == 0 && t == 0) *reinterpret_cast<u32x4s*>(ring + kRing) = v;
}

// Slicing-by-4 step from the 16-copy tables: entry e of table k for lane copy c sits at byte
// e << 8 | k << 6 | c << 2, so the address of byte j of x is one v_perm into lb[k] = k << 6 | c << 2.
__device__ __forceinline__ uint32_t fold4(uint32_t r, uint32_t w, const uint32_t (&lb)[4]) {
    const uint32_t x = r ^ w;
    return lds_word(__builtin_amdgcn_perm(x, lb[3], 0x03020400u)) ^ lds_word(__builtin_amdgcn_perm(x, lb[2], 0x03020500u)) ^
           lds_word(__builtin_amdgcn_perm(x, lb[1], 0x03020600u)) ^ lds_word(__builtin_amdgcn_perm(x, lb[0], 0x03020700u));
}

__device__ __forceinline__ uint32_t zshift(const uint32_t* tab, uint32_t r) {
    return tab[r & 0xffu] ^ tab[256 + ((r >> 8) & 0xffu)] ^ tab[512 + ((r >> 16) & 0xffu)] ^ tab[768 + (r >> 24)];
}

// CRC register contribution of unit `wi` (of `nwu`) of the frame whose CRC span is [fo, E),
// folded by a 16-lane group (lane gl); every lane of the group returns the reduced value.
// Unit wi covers [E - (nwu - wi) * 576, E - (nwu - 1 - wi) * 576), lane gl its 36-byte slice
// gl.  Bytes before fo are zeroed and reset()'s 0xFFFFFFFF is XOR-ed into the frame's first 4
// bytes (CRC linearity: a zero register absorbing leading zeros stays zero).  FROM_RING: bytes
// come from the LDS ring (ring offset of segment byte p = (p - A) & kRMask), else from HBM.
template <bool FROM_RING>
__device__ __forceinline__ uint32_t fold_unit(const uint8_t* ring, const uint8_t* seg, int64_t A, uint32_t sh,
                                              int64_t fo, int64_t E, int nwu, int wi, int gl,
                                              const uint32_t (&lb)[4], const uint32_t* lanetab) {
    const int64_t be = E - (int64_t)(nwu - 1 - wi) * kU - (int64_t)(kQ - 1 - gl) * kS;
    const bool act = be > fo;
    const int64_t b0 = be - kS - sh;  // seg + b0 is 4-byte aligned
    uint32_t d[kS / 4 + 1];
    if (FROM_RING) {
        const uint32_t q = (uint32_t)(b0 - A);
#pragma unroll
        for (int i = 0; i <= kS / 4; ++i) d[i] = *reinterpret_cast<const uint32_t*>(ring + ((q + 4u * i) & kRMask));
    } else {
#pragma unroll
        for (int i = 0; i <= kS / 4; ++i) {
            const int64_t p = b0 + 4 * i;
            d[i] = (act && p + 4 > fo && p < E) ? *reinterpret_cast<const uint32_t*>(seg + p) : 0u;
        }
    }
    const int64_t q0 = b0 - fo;
    if (act && q0 < 4) {
        const int qc = q0 < -48 ? -48 : (int)q0;
#pragma unroll
        for (int i = 0; i <= kS / 4; ++i) {
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
    for (int j = 0; j < kS / 4; ++j) r = fold4(r, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), lb);
    uint32_t z = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) z ^= lanetab[((k * 16 + ((r >> (4 * k)) & 15u)) << 4) + gl];
    r = act ? z : 0u;
#pragma unroll
    for (int m = 1; m < kQ; m <<= 1) r ^= __shfl_xor(r, m);
    return r;
}

// A frame that does not fit the resident ring: all of its units folded by one group from HBM
// (out of line: rare, and it keeps the hot path's registers free).
__device__ __noinline__ uint32_t fold_frame_hbm(const uint8_t* seg, int64_t A, uint32_t sh, int64_t fo, int64_t E,
                                                int nwu, int gl, const uint32_t* lanetab, const uint32_t* zu) {
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)k << 6) | ((uint32_t)gl << 2);
    uint32_t R = 0;
    for (int w = 0; w < nwu; ++w)
        R = zshift(zu, R) ^ fold_unit<false>(nullptr, seg, A, sh, fo, E, nwu, w, gl, lb, lanetab);
    return R;
}

// One walker step (wave 0, lane 0; out of line to keep the fold's registers free): the frames
// that start in window k, decided by decodeEntry's rules in the order segment_walk_kernel2 applies
// them, are recorded in the scratch frame table and listed (frame, units) in list buffer wb.
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) Frame LFrame;
typedef __attribute__((address_space(3))) Shared LShared;

__device__ __noinline__ void walk_window(uint64_t* scratch_off, uint32_t* scratch_len, uint32_t max_op, uint32_t cap,
                                         int64_t L, int64_t A, int64_t base, uint64_t slot0, int64_t k, int wb) {
    const lds_u8* ring = reinterpret_cast<const lds_u8*>(static_cast<uintptr_t>(kOffRing));
    LShared& S = *reinterpret_cast<LShared*>(static_cast<uintptr_t>(kOffSh));
    // ---- walk the frames that start in window k (decodeEntry, RDR:291-341) ----
    const int64_t wend = A + (k + 1) * kW;
    const int64_t ring_hi = A + (k + 3) * kW;  // resident through the next step
    int64_t p = S.pos;
    uint32_t nfr = S.nfr, nf = 0, nu = 0;
    int st = kWalking;
    LFrame* f = reinterpret_cast<LFrame*>(static_cast<uintptr_t>(kOffFt)) + wb * kFCap;
    lds_u32* u = reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(kOffUm)) + wb * kUCap;
    while (p < wend) {
        if (p >= L) {
            st = RH_SEG_END;
            break;
        }
        const uint32_t q = (uint32_t)((p - A) & kRMask);
        const uint32_t q0 = q & ~3u;
        const uint32_t lo = *reinterpret_cast<const lds_u32*>(ring + q0);
        const uint32_t hi = *reinterpret_cast<const lds_u32*>(ring + q0 + 4);  // mirror
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
                if ((ring[(uint32_t)(p + i - A) & kRMask] & 0x80) == 0) {
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
        const uint32_t nwu = (uint32_t)((total + kU - 1) / kU);
        const bool in_ring = p + fl <= ring_hi;
        const uint32_t need = in_ring ? nwu : 1u;
        if (nf == kFCap || nu + need > kUCap) break;  // list full: resume here next step
        scratch_off[slot0 + nfr] = (uint64_t)(base + p);
        scratch_len[slot0 + nfr] = (uint32_t)fl;
        f[nf].off = p;
        f[nf].len = (uint32_t)fl;
        for (uint32_t w = 0; w < need; ++w) u[nu + w] = nf | ((in_ring ? w : kHbmUnit) << 16);
        ++nfr;
        ++nf;
        nu += need;
        p += fl;
    }
    S.status = st;
    S.pos = p;
    S.nfr = nfr;
    S.nf[wb] = nf;
    S.nu[wb] = nu;
    S.fbase[wb] = nfr - nf;
}

__global__ __launch_bounds__(kThreads) void segment_read_kernel(ReadArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    uint32_t* L32 = reinterpret_cast<uint32_t*>(lds);
    uint8_t* ring = lds + kOffRing;
    Frame* ft = reinterpret_cast<Frame*>(lds + kOffFt);
    uint32_t* um = reinterpret_cast<uint32_t*>(lds + kOffUm);
    uint32_t* part = reinterpret_cast<uint32_t*>(lds + kOffPart);
    uint32_t* done = reinterpret_cast<uint32_t*>(lds + kOffDone);
    Shared& S = *reinterpret_cast<Shared*>(lds + kOffSh);
    const uint32_t* lanetab = reinterpret_cast<const uint32_t*>(lds + kOffLane);
    const uint32_t* zu = reinterpret_cast<const uint32_t*>(lds + kOffZu);

    const int t = threadIdx.x;
    for (int i = t; i < 16384; i += kThreads) L32[i] = a.slice[((i >> 4) & 3) * 256 + (i >> 6)];
    for (int i = t; i < 2048; i += kThreads) L32[kOffLane / 4 + i] = a.lane[(i >> 4) * 32 + (i & 15)];
    for (int i = t; i < 1024; i += kThreads) L32[kOffZu / 4 + i] = a.zu[i];
    for (int i = t; i < kFCap; i += kThreads) done[i] = 0;
    const int wave = t >> 6;
    const int gl = t & 15;
    const int grp = (wave - 1) * 4 + ((t >> 4) & 3);
    const int glead = (t & 63) & ~15;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)k << 6) | ((uint32_t)gl << 2);
    __syncthreads();

    for (uint64_t s = blockIdx.x; s < a.n_seg; s += gridDim.x) {
        const int64_t base = uniform64((int64_t)a.seg_off[s]);
        int64_t L = (int64_t)a.seg_len[s];
        if (base > a.buf_len) L = 0;
        else if (L > a.buf_len - base) L = a.buf_len - base;  // never read past the buffer
        L = uniform64(L);
        const uint8_t* seg = a.buf + base;
        const int64_t A = (base & ~(int64_t)15) - base;  // window grid origin: seg + A is 16-B aligned
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
            S.status = ok ? (8 >= L ? RH_SEG_END : kWalking) : (bad ? RH_SEG_E_HEADER : RH_SEG_END);
            S.pos = ok ? 8 : 0;
            S.nfr = 0;
            S.nf[0] = S.nf[1] = S.nu[0] = S.nu[1] = S.fbase[0] = S.fbase[1] = 0;
            S.first_bad = 0xFFFFFFFFu;
            S.nbad = 0;
        }
        __syncthreads();
        int status = S.status;
        int64_t pos = S.pos;

        // mode: 0 walk, 1 prime the ring then walk, 2 drain the listed frames then prime,
        // 3 drain the listed frames then finish, 4 finished
        int mode = status == kWalking ? 1 : 4;
        int64_t k = 0;
        u32x4s R0{0, 0, 0, 0}, R1{0, 0, 0, 0};  // windows k+3, k+4 in flight (R1: even windows)
        int wb = 0;                              // list buffer the walker fills this step
        while (mode != 4) {
            if (mode == 1) {
                k = (pos - A) / kW;
                const u32x4s w0 = load16(seg, L, A + k * kW, t);
                const u32x4s w1 = load16(seg, L, A + (k + 1) * kW, t);
                const u32x4s w2 = load16(seg, L, A + (k + 2) * kW, t);
                store16(ring, k, w0, t);
                store16(ring, k + 1, w1, t);
                store16(ring, k + 2, w2, t);
                if (k & 1) {
                    R1 = load16(seg, L, A + (k + 3) * kW, t);
                    R0 = load16(seg, L, A + (k + 4) * kW, t);
                } else {
                    R0 = load16(seg, L, A + (k + 3) * kW, t);
                    R1 = load16(seg, L, A + (k + 4) * kW, t);
                }
                mode = 0;
            }
            lds_barrier();  // ring holds windows k-1..k+2; the previous step's list is complete
            if (t == 0) {
                if (mode == 0) {
                    walk_window(a.scratch_off, a.scratch_len, a.max_op, a.cap, L, A, base, slot0, k, wb);
                } else {
                    S.nf[wb] = 0;
                    S.nu[wb] = 0;
                }
            }
            if (wave > 0) {
                // ---- CRC32C of the frames listed in the previous step (RDR:327-336) ----
                const int pb = wb ^ 1;
                const uint32_t nu_p = S.nu[pb], fbase = S.fbase[pb];
                const Frame* f = ft + pb * kFCap;
                const uint32_t* u = um + pb * kUCap;
                for (uint32_t x = (uint32_t)grp; x < nu_p; x += kGroups) {
                    const uint32_t e = u[x];
                    const uint32_t j = e & 0xFFFFu, wi = e >> 16;
                    const int64_t fo = f[j].off;
                    const int64_t total = (int64_t)f[j].len - 4;  // varint + proto
                    const int64_t E = fo + total;
                    const int nwu = (int)((total + kU - 1) / kU);
                    const uint32_t sh = (uint32_t)(base + E) & 3u;
                    uint32_t R = 0;
                    bool fin;
                    if (wi == kHbmUnit) {
                        R = fold_frame_hbm(seg, A, sh, fo, E, nwu, gl, lanetab, zu);
                        fin = true;
                    } else {
                        const uint32_t r = fold_unit<true>(ring, seg, A, sh, fo, E, nwu, (int)wi, gl, lb, lanetab);
                        if (nwu == 1) {
                            R = r;
                            fin = true;
                        } else {
                            uint32_t old = 0;
                            if (gl == 0) {
                                part[x] = r;
                                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                                old = atomicAdd(&done[j], 1u);
                            }
                            old = __shfl(old, glead);
                            fin = old == (uint32_t)nwu - 1;
                            if (fin && gl == 0) {
                                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                                const uint32_t u0 = x - wi;
                                for (int w = 0; w < nwu; ++w) R = zshift(zu, R) ^ part[u0 + w];
                                done[j] = 0;
                            }
                        }
                    }
                    if (fin && gl == 0) {
                        // getValue() after reset(); update(frame, 0, total)
                        const uint32_t value = ~(R ^ (total < 4 ? 0xFFFFFFFFu >> (8 * total) : 0u));
                        uint32_t b[4];
                        for (int i = 0; i < 4; ++i)
                            b[i] = wi == kHbmUnit ? seg[E + i] : ring[(uint32_t)(E + i - A) & kRMask];
                        const uint32_t stored = (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3];  // big-endian
                        const uint32_t idx = fbase + j;
                        a.scratch_crc[slot0 + idx] = value;
                        if (stored != value) {
                            atomicMin(&S.first_bad, idx);
                            atomicAdd(&S.nbad, 1u);
                        }
                    }
                }
            }
            lds_barrier();  // the walk and the folds of this step are done
            const int cur = mode;
            wb ^= 1;
            if (cur == 3) break;
            if (cur == 2) {
                mode = 1;
                continue;
            }
            status = S.status;
            pos = S.pos;
            if (status != kWalking) {
                mode = 3;
            } else if (pos >= A + (k + 2) * kW) {
                mode = 2;  // a frame jumped past the ring: drain the list, restart at pos
            } else if (pos >= A + (k + 1) * kW) {
                // advance: window k+3 replaces window k-1 (its frames were folded this step)
                if (k & 1) {
                    store16(ring, k + 3, R1, t);
                    R1 = load16(seg, L, A + (k + 5) * kW, t);
                } else {
                    store16(ring, k + 3, R0, t);
                    R0 = load16(seg, L, A + (k + 5) * kW, t);
                }
                ++k;
            }
            // else the list filled up inside window k: walk it again next step
        }

        if (status == kTermPending) {
            // verifyTerminator (RDR:251-280): the first non-zero byte in [pos, L), block-wide
            if (t == 0) S.term_min = (unsigned long long)L;
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
                if (my < (unsigned long long)L) atomicMin(&S.term_min, my);
                __syncthreads();
                found = S.term_min < (unsigned long long)L;
                __syncthreads();
            }
            if (found) {
                status = RH_SEG_E_PADDING;
                pos = (int64_t)S.term_min;
            } else {
                status = RH_SEG_END;  // stop stays at the terminator (the segment's logical end)
            }
        }
        if (t == 0) {
            const uint32_t nfr = S.nfr, fb = S.first_bad;
            const bool bad = fb < nfr;
            a.seg_nframes[s] = nfr;
            a.seg_status[s] = status;
            a.seg_stop[s] = (uint64_t)pos;
            a.seg_ok[s] = bad ? fb : nfr;
            a.seg_rstatus[s] = bad ? RH_SEG_E_CHECKSUM : status;
            a.seg_rstop[s] = bad ? a.scratch_off[slot0 + fb] - (uint64_t)base : (uint64_t)pos;
            if (a.n_bad && S.nbad) atomicAdd(a.n_bad, (unsigned long long)S.nbad);
        }
        __syncthreads();
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

}  // namespace

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
    if (!ctx->d_slice || !ctx->d_lane16_s36 || !ctx->d_zu576)
        return rh::fail(RH_E_STATE, "rh_segments_read_launch: CRC tables not uploaded");
    static bool attr_set = false;
    if (!attr_set) {
        RH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(segment_read_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes));
        attr_set = true;
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
    a.lane = ctx->d_lane16_s36;
    a.zu = ctx->d_zu576;
    const int cus = ctx->num_cus > 0 ? ctx->num_cus : 256;
    const uint64_t grid = g->n_seg < (uint64_t)cus ? g->n_seg : (uint64_t)cus;
    hipLaunchKernelGGL(segment_read_kernel, dim3((uint32_t)grid), dim3(kThreads), kLdsBytes, stream, a);
    RH_HIP(hipGetLastError());
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
