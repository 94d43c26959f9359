// CRC32C (PureJavaCrc32C) over SegmentedRaftLog frames, for gfx950 (MI355X).
//
// Reference semantics:
//   PureJavaCrc32C.update/getValue/reset    PureJavaCrc32C.java:43-152 (tables :158-688)
//   frame CRC = CRC32C(varint || proto), big-endian trailer
//                                            SegmentedRaftLogOutputStream.java:86-110
//   verification                             SegmentedRaftLogReader.java:327-336
//
// Structure (crc_frames_kernel).  A frame's CRC-covered span is cut into end-anchored 1 KiB
// windows; a window is folded by one 16-lane group of a wave, lane g taking the 64-byte chunk
// [end - (16-g)*64, end - (15-g)*64).  Every lane folds its chunk into a CRC register that
// starts at zero (slicing-by-4, two independent chains of 8 words joined by a 32-zero-byte
// advance), advances it over the 64*(15-g) zero bytes after its chunk with 8 nibble lookups into
// lane-specific tables, and a 4-step DPP XOR reduce over the 16-lane row gives the window's
// register; windows chain with a 1 KiB zero-advance.  CRC linearity makes this exact: bytes
// before the frame start contribute nothing to a zero register, and the initial state I
// (0xFFFFFFFF after reset()) is injected by XOR-ing it into the first 4 message bytes.
//
// LDS.  The 4 slicing tables are replicated 32 times and interleaved so that lane l always
// reads bank (l & 31) and the address of byte j of a register is one v_perm_b32 (128 KiB); the
// lane tables (16 KiB) use the same bank = lane & 31 layout.  One 1024-thread workgroup per CU,
// persistent over 512-frame batches whose frame table is staged in LDS.
//
// No MFMA: CRC is table/XOR integer work and the kernel is HBM-bound.
#include "rh_internal.h"

#include <vector>

namespace {

// ---- host: zero-advance linear maps ------------------------------------------------------
struct Map32 {
    uint32_t col[32];  // image of bit i
};

uint32_t apply(const Map32& m, uint32_t x) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i)
        if (x >> i & 1u) r ^= m.col[i];
    return r;
}

Map32 compose(const Map32& a, const Map32& b) {  // a o b
    Map32 r{};
    for (int i = 0; i < 32; ++i) r.col[i] = apply(a, b.col[i]);
    return r;
}

}  // namespace
namespace rh {

void build_crc_slice_tables(CrcTables* t) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? 0x82F63B78u : 0u);
        t->slice[0][i] = c;
    }
    for (int k = 1; k < 4; ++k)
        for (int i = 0; i < 256; ++i)
            t->slice[k][i] = (t->slice[k - 1][i] >> 8) ^ t->slice[0][t->slice[k - 1][i] & 0xffu];
}

void build_crc_shift_table(uint64_t nbytes, uint32_t out[4][256]) {
    CrcTables st;
    build_crc_slice_tables(&st);
    Map32 one{};  // advance over one zero byte: r -> (r >> 8) ^ T0[r & 0xff]
    for (int i = 0; i < 32; ++i) {
        const uint32_t x = 1u << i;
        one.col[i] = (x >> 8) ^ st.slice[0][x & 0xffu];
    }
    Map32 acc{};
    for (int i = 0; i < 32; ++i) acc.col[i] = 1u << i;  // identity
    Map32 p = one;
    for (uint64_t n = nbytes; n; n >>= 1) {
        if (n & 1u) acc = compose(p, acc);
        p = compose(p, p);
    }
    for (int k = 0; k < 4; ++k)
        for (int b = 0; b < 256; ++b) out[k][b] = apply(acc, (uint32_t)b << (8 * k));
}

// Lane-distance tables: lane g of a Q-lane window advances its chunk CRC over
// 64*(Q-1-g) zero bytes with 8 nibble lookups.  Layout [Q/32 halves][8 nibbles][16][32 copies]:
// copy c (= lane & 31) holds the map of lane position (half*32 + c) mod Q, so every lane reads
// LDS bank (lane & 31) -- conflict free.
std::vector<uint32_t> build_crc_lane_tables(int Q, int S) {
    const int halves = Q > 32 ? Q / 32 : 1;
    std::vector<uint32_t> out((size_t)halves * 8 * 16 * 32);
    CrcTables st;
    build_crc_slice_tables(&st);
    Map32 one{};
    for (int i = 0; i < 32; ++i) {
        const uint32_t x = 1u << i;
        one.col[i] = (x >> 8) ^ st.slice[0][x & 0xffu];
    }
    for (int h = 0; h < halves; ++h)
        for (int c = 0; c < 32; ++c) {
            const int g = (h * 32 + c) % Q;
            const uint64_t nbytes = (uint64_t)S * (uint64_t)(Q - 1 - g);
            Map32 acc{};
            for (int i = 0; i < 32; ++i) acc.col[i] = 1u << i;
            Map32 p = one;
            for (uint64_t n = nbytes; n; n >>= 1) {
                if (n & 1u) acc = compose(p, acc);
                p = compose(p, p);
            }
            for (int k = 0; k < 8; ++k)
                for (int nib = 0; nib < 16; ++nib)
                    out[(((size_t)h * 8 + k) * 16 + nib) * 32 + c] = apply(acc, (uint32_t)nib << (4 * k));
        }
    return out;
}

namespace {
Map32 zero_byte_map() {  // advance over one zero byte: r -> (r >> 8) ^ T0[r & 0xff]
    CrcTables st;
    build_crc_slice_tables(&st);
    Map32 one{};
    for (int i = 0; i < 32; ++i) {
        const uint32_t x = 1u << i;
        one.col[i] = (x >> 8) ^ st.slice[0][x & 0xffu];
    }
    return one;
}

Map32 map_pow(Map32 p, uint64_t n) {
    Map32 acc{};
    for (int i = 0; i < 32; ++i) acc.col[i] = 1u << i;
    for (; n; n >>= 1) {
        if (n & 1u) acc = compose(p, acc);
        p = compose(p, p);
    }
    return acc;
}

// Inverse over GF(2) by Gauss-Jordan on the rows (the zero-byte advance is invertible: the
// Castagnoli polynomial has a non-zero constant term, so x is a unit modulo it).
Map32 invert(const Map32& m) {
    uint32_t row[32], inv[32];
    for (int r = 0; r < 32; ++r) {
        row[r] = 0;
        for (int c = 0; c < 32; ++c) row[r] |= ((m.col[c] >> r) & 1u) << c;
        inv[r] = 1u << r;
    }
    for (int c = 0; c < 32; ++c) {
        int p = c;
        while (p < 32 && !((row[p] >> c) & 1u)) ++p;
        if (p == 32) return Map32{};  // singular (not reached)
        std::swap(row[p], row[c]);
        std::swap(inv[p], inv[c]);
        for (int r = 0; r < 32; ++r)
            if (r != c && ((row[r] >> c) & 1u)) {
                row[r] ^= row[c];
                inv[r] ^= inv[c];
            }
    }
    Map32 out{};
    for (int c = 0; c < 32; ++c)
        for (int r = 0; r < 32; ++r) out.col[c] |= ((inv[r] >> c) & 1u) << r;
    return out;
}
}  // namespace

std::vector<uint32_t> build_crc_inverse_lane_tables() {
    const Map32 back = invert(zero_byte_map());
    std::vector<uint32_t> out((size_t)32 * 8 * 16);
    for (int c = 0; c < 32; ++c) {
        const Map32 m = map_pow(back, (uint64_t)64 * (uint64_t)(31 - c));
        for (int k = 0; k < 8; ++k)
            for (int nib = 0; nib < 16; ++nib) out[((size_t)c * 8 + k) * 16 + nib] = apply(m, (uint32_t)nib << (4 * k));
    }
    return out;
}

std::vector<uint32_t> build_crc_init_terms(uint32_t init) {
    CrcTables st;
    build_crc_slice_tables(&st);
    std::vector<uint32_t> out((size_t)kCrcInitSpan + 1);
    uint32_t x = init;
    for (uint32_t k = 0; k <= kCrcInitSpan; ++k) {
        out[k] = x;
        x = (x >> 8) ^ st.slice[0][x & 0xffu];
    }
    return out;
}

}  // namespace rh

namespace {

struct FrameArgs {
    const uint8_t* buf;
    uint8_t* wbuf;
    int64_t buf_len;
    const uint64_t* off;
    const uint32_t* len;
    uint64_t n;
    uint32_t init;
    uint32_t flags;
    uint32_t* crc_out;
    uint64_t* bad_bits;
    unsigned long long* n_bad;
    const uint32_t* slice;   // [4][256] global
    const uint32_t* shift32; // [4][256]: advance over 32 zero bytes (fold chain combine)
    const uint32_t* lanetab; // lane-distance nibble tables (build_crc_lane_tables(16, 64))
    const uint32_t* zwin;    // [4][256]: advance over one 1 KiB window
    // slot mode (the read path): the frame table is rh_segments' slotted scratch table, entry
    // f = segment f / slot_cap, slot f % slot_cap, valid below min(slot_nframes[seg], slot_cap);
    // a mismatch also lowers seg_first_bad[seg] to the slot index (atomicMin)
    const uint32_t* slot_nframes;
    uint32_t slot_cap;
    uint32_t* seg_first_bad;
    // slot mode, dense outputs (the read path's crc_out / bad_bits): slot s of segment g is frame
    // seg_first[g] + s of the dense table (below frame_cap)
    const uint64_t* seg_first;
    uint32_t* dense_crc;
    uint64_t* dense_bad;
    uint64_t frame_cap;
    // crc_frames_kernel<true> (the lane split's window pass): its frames are widx[0 .. counts[0])
    const uint32_t* counts;
    const uint32_t* widx;
};

__device__ __forceinline__ uint32_t zshift(const uint32_t* tab, uint32_t r) {
    return tab[r & 0xffu] ^ tab[256 + ((r >> 8) & 0xffu)] ^ tab[512 + ((r >> 16) & 0xffu)] ^ tab[768 + (r >> 24)];
}

// 16 bytes at a 4-aligned address.
struct __attribute__((aligned(4))) u32x4a {
    uint32_t x, y, z, w;
};

// Slicing table k lives in 64 KiB region (k >> 1), half (k & 1): entry e of lane copy c at byte
// (k>>1)<<16 | e<<8 | (k&1)<<7 | c<<2, so ds_read_b32 bank = c = lane & 31 (conflict free) and
// the address of byte j of the register x is ONE v_perm_b32: byte j of x dropped into bits
// 8..15 of the lane's base word for that table.
// Absolute LDS address: the kernel has no static LDS, so its dynamic region starts at 0 and a
// byte offset is the LDS address itself (saves the base add per lookup).
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_word(const uint32_t*, uint32_t byte_addr) {
    return *reinterpret_cast<lds_u32_t*>(static_cast<uintptr_t>(byte_addr));
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// The register after folding one word: x = register ^ word (the word's bytes already XOR-ed in);
// returns that register ^ `wn` -- with wn = the next word this is the next step's x, so a word costs
// four v_perm and two bitop3 (the four lookups and the next word joined in two 3-input XORs).
__device__ __forceinline__ uint32_t fold_x(const uint32_t* lds, uint32_t x, const uint32_t (&lb)[4], uint32_t wn) {
    // selector: out byte0 = lb.b0 (0), byte1 = x.byte j (4 + j), byte2 = lb.b2 (2), byte3 = lb.b3 (3)
    const uint32_t a3 = __builtin_amdgcn_perm(x, lb[3], 0x03020400u);  // byte 0 of x -> T3
    const uint32_t a2 = __builtin_amdgcn_perm(x, lb[2], 0x03020500u);  // byte 1 -> T2
    const uint32_t a1 = __builtin_amdgcn_perm(x, lb[1], 0x03020600u);  // byte 2 -> T1
    const uint32_t a0 = __builtin_amdgcn_perm(x, lb[0], 0x03020700u);  // byte 3 -> T0
    return xor3(xor3(lds_word(lds, a3), lds_word(lds, a2), lds_word(lds, a1)), lds_word(lds, a0), wn);
}

// zshift(tab, r) ^ extra
__device__ __forceinline__ uint32_t zshift_x(const uint32_t* tab, uint32_t r, uint32_t extra) {
    return xor3(xor3(tab[r & 0xffu], tab[256 + ((r >> 8) & 0xffu)], tab[512 + ((r >> 16) & 0xffu)]), tab[768 + (r >> 24)],
                extra);
}

// A lane table's map of the register r (8 nibble-indexed lookups, copy c of each table entry).
__device__ __forceinline__ uint32_t lane_advance(const uint32_t* tab, uint32_t c, uint32_t r) {
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = tab[c + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
    return xor3(xor3(xor3(t[0], t[1], t[2]), t[3], t[4]), t[5], t[6]) ^ t[7];
}

// Start of a frame inside a lane's chunk: the chunk's aligned words d[0..16] start q0l bytes
// after the frame start (q0l < 4: the chunk holds frame bytes 0..3).  Bytes before the frame are
// zeroed (a zero register absorbs leading zeros) and reset()'s state is XOR-ed into frame bytes
// 0..3, so folding the chunk from a zero register is folding the frame from `init`.
// Word i starts s = -(q0l + 4i) bytes before the frame start: it keeps its bytes >= s
// (mask ~0 << 8 clamp(s, 0, 4)) and takes init shifted by s bytes, i.e. the low word of
// (init << 32) >> (32 - 8 clamp(s, -4, 4)) -- both ends of that clamp give 0 (a 64-bit shift by
// 0 or 64 = 0 mod 64 of a value whose low half is 0).  Lanes with `on` false: s <= -4 everywhere.
__device__ __forceinline__ void mask_frame_start(uint32_t (&d)[18], int64_t q0l, bool on, uint32_t init) {
    const int32_t s8_0 = on ? -8 * (int32_t)q0l : -32;  // 8 s for word 0 (q0l in (-68, 4) when on)
    const uint64_t X = (uint64_t)init << 32;
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        const int32_t s8 = s8_0 - 32 * i;
        const int32_t k = min(max(s8, 0), 32);   // garbage bits at the word's low end (v_med3)
        const int32_t m = min(max(s8, -32), 32);
        const uint32_t keep = (uint32_t)(~0ull << k);
        const uint32_t inj = (uint32_t)(X >> ((uint32_t)(32 - m) & 63u));
        d[i] = (d[i] & keep) ^ inj;
    }
}

// A frame's results: its CRC, and when `bad` (VERIFY mismatch, or malformed) its bad bit and count;
// in slot mode also the segment's first bad slot and the dense per-frame outputs.
template <typename A>
__device__ __forceinline__ void emit_frame(const A& a, uint64_t f, uint32_t value, bool bad) {
    if (a.crc_out) a.crc_out[f] = value;
    if (bad) {
        if (a.bad_bits) atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
    }
    if (a.seg_first_bad || a.seg_first) {  // slot mode (32-bit: the launcher keeps n below 2^32)
        const uint32_t seg = (uint32_t)f / a.slot_cap, slot = (uint32_t)f - seg * a.slot_cap;
        if (bad && a.seg_first_bad) atomicMin(a.seg_first_bad + seg, slot);
        if (a.seg_first) {
            const uint64_t d = a.seg_first[seg] + slot;
            if (d < a.frame_cap) {
                if (a.dense_crc) a.dense_crc[d] = value;
                if (bad && a.dense_bad)
                    atomicOr(reinterpret_cast<unsigned long long*>(a.dense_bad + (d >> 6)), 1ull << (d & 63));
            }
        }
    }
}

// ---- the kernel: copy-free prefetch ring, frame metadata staged in LDS ------------------------
//   * the loop body is unrolled over the 3 ring slots with static roles (load slot i+2 while
//     folding slot i): a window's data is consumed two windows after its load was issued, and
//     every wait in the loop is a counted vmcnt(N);
//   * the frame table is staged per block in batches of 512 frames into LDS (one drain per batch),
//     and each 16-lane group takes the batch's next frame whenever it finishes one;
//   * the trailer for VERIFY comes from the last window's own chunk (one extra dword per lane), so
//     the verify needs no dependent byte loads; the group's lane 15 (whose chunk ends at the CRC
//     span's end) finalises the frame;
//   * inactive lanes load from the buffer start instead of zero-filling registers in flight.
// Frames whose chunks could leave the buffer (within 67 bytes of its start or 8 of its end),
// malformed and empty ones take a guarded byte path after the batch's main loop.
// Chunk-count classes and the kernel each goes to (microbench over uniform and ragged shapes,
// profiles/r02/crc_lanes/): spans up to 768 B on 4 lanes per frame, up to 1536 B on 8; longer
// spans fill the 1 KiB windows well enough that the window kernel's per-frame dynamic assignment
// wins (4 KiB frames: 4.3 vs 3.8 TB/s on 16 lanes per frame).
#ifndef RH_Q4_CHUNKS  // A/B builds override (scripts/ab_build.sh)
#define RH_Q4_CHUNKS 12
#define RH_LANE_CHUNKS 24
#endif
constexpr int kQ4Chunks = RH_Q4_CHUNKS;
constexpr int kLaneChunks = RH_LANE_CHUNKS;  // CRC spans up to 1536 B go to the lane kernels
constexpr int kClasses = kLaneChunks + 1;  // class 0: window kernel; class c: c chunks of 64 B
constexpr uint64_t kLaneMeanMax = 2048;    // mean frame length (buf_len / n) up to which the split runs

// Batch table per block: 512 frames x 15 B (start, span, path, guarded list), or in the listed
// variant 416 x 19 B (+ frame number): what 160 KiB of LDS leaves next to 152 KiB of tables.
constexpr int kBatchOf(bool listed) { return listed ? 416 : 512; }
constexpr int kBatch = kBatchOf(false);
struct Meta {
    int64_t o;    // frame start (bytes)
    uint32_t lc;  // CRC-covered length
    uint32_t fl;  // 0 = fast path; 1 = slow path (guarded), 2 = malformed
};

constexpr int kCrcThreads = 1024;
constexpr int kCrcLdsOf(bool listed) { return 128 * 1024 + 16384 + 8192 + kBatchOf(listed) * (listed ? 19 : 15) + 16; }
static_assert(kCrcLdsOf(false) <= 160 * 1024 && kCrcLdsOf(true) <= 160 * 1024, "LDS budget");

// LISTED = false: every frame of the table (the plan for logs of long entries, config 5).
// LISTED = true: the frames the length-class split left to this kernel, widx[0 .. counts[0]).
template <bool LISTED>
__global__ __launch_bounds__(kCrcThreads) void crc_frames_kernel(FrameArgs a) {
    constexpr int kBatch = kBatchOf(LISTED);
    constexpr int CH = 2;  // independent fold chains per lane (measured: 1 / 4 chains are slower)
    constexpr int Q = 16, S = 64;
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int kSliceBytes = 128 * 1024;
    constexpr int kLaneWords = 8 * 16 * 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    const uint64_t n_all = LISTED ? (uint64_t)a.counts[0] : a.n;
    if (LISTED && (uint64_t)blockIdx.x * kBatch >= n_all) return;  // no batch: skip the table fill
    uint32_t* llane = lds + kSliceBytes / 4;
    uint32_t* lzw = llane + kLaneWords;
    uint32_t* lch = lzw + 1024;  // [4][256]: advance over 64 / CH zero bytes (chain combine)
    // batch frame table, struct-of-arrays: start, CRC-covered length, path; then the guarded list
    int64_t* mo = reinterpret_cast<int64_t*>(lch + 1024);
    uint32_t* mlc = reinterpret_cast<uint32_t*>(mo + kBatch);
    uint32_t* mf = mlc + kBatch;  // LISTED: frame number
    uint8_t* mfl = reinterpret_cast<uint8_t*>(LISTED ? mf + kBatch : mlc + kBatch);
    uint16_t* slow = reinterpret_cast<uint16_t*>(mfl + kBatch);  // [kBatch] guarded-path frames
    uint32_t* nslow = reinterpret_cast<uint32_t*>(slow + kBatch);
    uint32_t* nexti = nslow + 1;  // next batch frame to hand out (dynamic assignment)
    auto meta = [&](uint32_t j) { return Meta{mo[j], mlc[j], mfl[j]}; };
    for (int i = threadIdx.x; i < kSliceBytes / 4; i += blockDim.x) {
        const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
        lds[i] = a.slice[((region * 2 + half) << 8) | e];
    }
    for (int i = threadIdx.x; i < kLaneWords; i += blockDim.x) llane[i] = a.lanetab[i];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lzw[i] = a.zwin[i];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lch[i] = a.shift32[i];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const uint32_t c = lane & 31;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | (c << 2);
    const int gl = lane & (Q - 1);
    const uint32_t grp = (uint32_t)t >> 4;  // 64 groups per block
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;
    const uint32_t tl = trailer ? 4u : 0u;

    for (uint64_t b0f = (uint64_t)blockIdx.x * kBatch; b0f < n_all; b0f += (uint64_t)gridDim.x * kBatch) {
        const uint32_t nb = (uint32_t)(n_all - b0f < (uint64_t)kBatch ? n_all - b0f : (uint64_t)kBatch);
        __syncthreads();  // previous batch done with meta / slow
        if (t == 0) {
            *nslow = 0;
            *nexti = 0;
        }
        __syncthreads();
        if ((uint32_t)t < nb) {
            const uint64_t f = LISTED ? (uint64_t)a.widx[b0f + (uint64_t)t] : b0f + (uint64_t)t;
            if (LISTED) mf[t] = (uint32_t)f;
            const uint64_t o = a.off[f];
            const int64_t L = (int64_t)a.len[f];
            const bool malformed = o > (uint64_t)a.buf_len || L > a.buf_len - (int64_t)o || (trailer && L < 4);
            Meta m;
            m.o = (int64_t)o;
            m.lc = malformed ? 0u : (uint32_t)(L - (int64_t)tl);
            const int64_t E = m.o + (int64_t)m.lc;
            const bool unsafe = m.o < 67 || E + 8 > a.buf_len || m.lc < 8;
            m.fl = malformed ? 2u : (unsafe ? 1u : 0u);
            if (a.slot_nframes) {  // slot mode: slots past the segment's frame count are skipped
                const uint32_t seg = (uint32_t)f / a.slot_cap, slot = (uint32_t)f - seg * a.slot_cap;
                const uint32_t nfs = a.slot_nframes[seg];
                if (slot >= (nfs < a.slot_cap ? nfs : a.slot_cap)) m.fl = 3u;
            }
            mo[t] = m.o;
            mlc[t] = m.lc;
            mfl[t] = (uint8_t)m.fl;
            if (m.fl == 1u || m.fl == 2u) slow[atomicAdd(nslow, 1u)] = (uint16_t)t;
        }
        __syncthreads();

        // ---- fast path: each group walks the windows of the frames it takes from the batch ----
        struct Task {
            uint32_t j;   // batch-local frame (>= nb: none)
            uint32_t wi;  // window
        };
        // Frames are handed out dynamically: a group that finishes a frame takes the batch's next
        // fast-path frame (one LDS atomic by the group's lane 0, broadcast to its 16 lanes), so
        // groups stay balanced when frame lengths differ.  Control is uniform within a group.
        auto grab = [&]() -> uint32_t {
            uint32_t j;
            do {
                uint32_t v = 0;
                if (gl == 0) v = atomicAdd(nexti, 1u);
                j = (uint32_t)__shfl((int)v, lane & ~(Q - 1));
            } while (j < nb && mfl[j] != 0);
            return j < nb ? j : nb;
        };
        auto next = [&](Task x) {
            if (x.j >= nb) return x;
            const uint32_t nw = (mlc[x.j] + (uint32_t)W - 1) / (uint32_t)W;
            if (x.wi + 1 < nw) return Task{x.j, x.wi + 1};
            return Task{grab(), 0u};
        };
        // chunk of lane gl in task x: [be - S, be), be = E - (nw - 1 - wi) W - (Q - 1 - gl) S
        auto load = [&](Task x, uint32_t (&dd)[18]) {
            const uint8_t* src = a.buf;
            if (x.j < nb) {
                const Meta m = meta(x.j);
                const int64_t E = m.o + (int64_t)m.lc;
                const int64_t nw = ((int64_t)m.lc + W - 1) / W;
                const int64_t be = E - (nw - 1 - (int64_t)x.wi) * W - (int64_t)(Q - 1 - gl) * S;
                const int64_t b0 = be - S - (int64_t)(E & 3);
                if (be > m.o) src = a.buf + b0;  // inactive lanes: the buffer start (never used)
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4a v = *reinterpret_cast<const u32x4a*>(src + 16 * q);
                dd[4 * q] = v.x;
                dd[4 * q + 1] = v.y;
                dd[4 * q + 2] = v.z;
                dd[4 * q + 3] = v.w;
            }
            dd[16] = *reinterpret_cast<const uint32_t*>(src + 64);
            dd[17] = *reinterpret_cast<const uint32_t*>(src + 68);
        };
        uint32_t R = 0;
        auto fold = [&](Task x, uint32_t (&d)[18]) {
            if (x.j >= nb) return;
            const Meta m = meta(x.j);
            const int64_t E = m.o + (int64_t)m.lc;
            const int64_t nw = ((int64_t)m.lc + W - 1) / W;
            const uint32_t sh = (uint32_t)(E & 3);
            const int64_t be = E - (nw - 1 - (int64_t)x.wi) * W - (int64_t)(Q - 1 - gl) * S;
            const bool act = be > m.o;
            const int64_t q0l = be - S - (int64_t)sh - m.o;  // chunk start (aligned) rel. to frame start
            if (__any(act && q0l < 4)) mask_frame_start(d, q0l, act && q0l < 4, a.init);
            // CH independent chains of 16 / CH words (the LDS round trips overlap), joined by
            // Horner steps over 64 / CH zero bytes: CRC(A||B) = adv_|B|(crc A) ^ crc B from zero
            constexpr int LW = 16 / CH;
            uint32_t rc[CH];
            if (__all(sh == 0 || !act)) {
#pragma unroll
                for (int q = 0; q < CH; ++q) rc[q] = d[q * LW];
#pragma unroll
                for (int j = 0; j < LW; ++j)
#pragma unroll
                    for (int q = 0; q < CH; ++q) rc[q] = fold_x(lds, rc[q], lb, j + 1 < LW ? d[q * LW + j + 1] : 0u);
            } else {
                auto wd = [&](int q, int j) { return __builtin_amdgcn_alignbyte(d[q * LW + j + 1], d[q * LW + j], sh); };
#pragma unroll
                for (int q = 0; q < CH; ++q) rc[q] = wd(q, 0);
#pragma unroll
                for (int j = 0; j < LW; ++j)
#pragma unroll
                    for (int q = 0; q < CH; ++q) rc[q] = fold_x(lds, rc[q], lb, j + 1 < LW ? wd(q, j + 1) : 0u);
            }
            uint32_t r = rc[0];
#pragma unroll
            for (int q = 1; q < CH; ++q) r = zshift_x(lch, r, rc[q]);
            r = act ? lane_advance(llane, c, r) : 0u;
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x141, 0xF, 0xF, false);  // row_half_mirror
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x140, 0xF, 0xF, false);  // row_mirror
            R = zshift_x(lzw, R, r);
            if ((int64_t)x.wi + 1 >= nw) {
                if (gl == Q - 1) {  // this lane's chunk ends at E: d[16..17] hold bytes E - sh .. E + 8 - sh
                    const uint64_t f = LISTED ? (uint64_t)mf[x.j] : b0f + x.j;
                    uint32_t state = R;
                    if (m.lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * m.lc));
                    const uint32_t value = ~state;
                    bool bad = false;
                    if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t le = __builtin_amdgcn_alignbyte(d[17], d[16], sh);
                        bad = __builtin_bswap32(le) != value;  // big-endian trailer
                    }
                    emit_frame(a, f, value, bad);
                }
                R = 0;
            }
        };
        Task T0{a.buf_len >= 128 ? grab() : nb, 0u};  // tiny buffers: every frame is guarded
        Task T1 = next(T0);
        Task T2 = next(T1);
        uint32_t d0[18], d1[18], d2[18];
        if (__any(T0.j < nb)) {
            load(T0, d0);
            load(T1, d1);
        }
        while (__any(T0.j < nb)) {
            load(T2, d2);
            fold(T0, d0);
            T0 = next(T2);
            if (!__any(T1.j < nb)) break;
            load(T0, d0);
            fold(T1, d1);
            T1 = next(T0);
            if (!__any(T2.j < nb)) break;
            load(T1, d1);
            fold(T2, d2);
            T2 = next(T1);
        }

        // ---- guarded path: frames near the buffer ends, malformed and empty spans ----
        __syncthreads();
        const uint32_t ns = *nslow;
        for (uint32_t i = grp; i < ns; i += 64) {
            const uint32_t j = slow[i];
            const Meta m = meta(j);
            const uint64_t f = LISTED ? (uint64_t)mf[j] : b0f + j;
            if (m.fl == 2) {
                if (gl == 0) emit_frame(a, f, 0u, true);
                continue;
            }
            const int64_t E = m.o + (int64_t)m.lc;
            const int64_t nw = ((int64_t)m.lc + W - 1) / W;
            uint32_t Rs = 0;
            for (int64_t wi = 0; wi < nw; ++wi) {
                const int64_t be = E - (nw - 1 - wi) * W - (int64_t)(Q - 1 - gl) * S;
                const int64_t bs = be - S > m.o ? be - S : m.o;
                uint32_t r = 0;
                // byte-wise, reset()'s state in bytes 0..3; T0 from this lane's LDS copy (a global
                // table made every byte a dependent L2 round trip: ~13 us per 1 KiB window)
#pragma unroll 4
                for (int64_t p = bs; p < be; ++p) {
                    uint32_t b = a.buf[p];
                    if (p - m.o < 4) b ^= (a.init >> (8 * (p - m.o))) & 0xffu;
                    r = (r >> 8) ^ lds_word(lds, (((r ^ b) & 0xffu) << 8) | (c << 2));
                }
                uint32_t z = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) z ^= llane[c + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
                r = be > m.o ? z : 0u;
#pragma unroll
                for (int dlt = 1; dlt < Q; dlt <<= 1) r ^= __shfl_xor(r, dlt);
                Rs = zshift(lzw, Rs) ^ r;
            }
            if (gl == 0) {
                uint32_t state = Rs;
                if (m.lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * m.lc));
                const uint32_t value = ~state;
                bool bad = false;
                if (a.flags & RH_CRC_STAMP) {
                    a.wbuf[E + 0] = (uint8_t)(value >> 24);
                    a.wbuf[E + 1] = (uint8_t)(value >> 16);
                    a.wbuf[E + 2] = (uint8_t)(value >> 8);
                    a.wbuf[E + 3] = (uint8_t)value;
                } else if (a.flags & RH_CRC_VERIFY) {
                    const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                            ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                    bad = stored != value;
                }
                emit_frame(a, f, value, bad);
            }
        }
    }
}

// ---- lane-per-frame path --------------------------------------------------------------------
// The window kernel's cost is per 1 KiB window, however little of it a short frame fills (it is
// VALU-issue bound: ~0.25 ns of the chip per window).  Frames whose CRC span is at most
// kLaneChunks x 64 B are instead folded one frame per lane: a lane walks its frame's end-anchored
// 64-byte chunks and carries its register from chunk to chunk, so the work is proportional to the
// frame's bytes and needs no cross-lane combine.  A counting sort by chunk count (classify +
// scatter) makes the 64 frames of a wave the same length, so the wave's lanes start and finish
// their frames together (the start-of-frame masking and the trailer check are wave-uniform steps).
// Long frames and frames the fast path cannot load safely stay on the window kernel (class 0).
constexpr int kLaneLds = 128 * 1024 + 4096 + 16384 + 4096;
constexpr int kSortThreads = 256, kSortPer = 8, kSortTile = kSortThreads * kSortPer;

struct LaneRec {  // one frame of the lane path, records ascending by chunk count
    int64_t o;    // frame start
    uint32_t lc;  // CRC-covered length (8 .. 4096)
    uint32_t f;   // frame number (output index)
};

// A frame's table entry, loaded unconditionally (every load of a thread's frames in flight before
// any is used: a dependent, conditional load chain per slot left the prepass waiting on memory).
struct FrameIn {
    uint64_t o;
    uint32_t len;
    uint32_t nfs;  // slot mode: frames of the slot's segment
};
__device__ __forceinline__ FrameIn load_frame(const FrameArgs& a, uint64_t f) {
    FrameIn x{0, 0, 0};
    if (f < a.n) {
        x.o = a.off[f];
        x.len = a.len[f];
        if (a.slot_nframes) x.nfs = a.slot_nframes[(uint32_t)f / a.slot_cap];  // 32-bit: n < 2^32
    }
    return x;
}

// class of frame f (-1: none, or an empty slot of the slotted read-path table: no output at all)
__device__ __forceinline__ int crc_class(const FrameArgs& a, uint64_t f, const FrameIn& x, int64_t& o_out,
                                         uint32_t& lc_out) {
    if (f >= a.n) return -1;
    if (a.slot_nframes) {
        const uint32_t slot = (uint32_t)f % a.slot_cap;
        if (slot >= (x.nfs < a.slot_cap ? x.nfs : a.slot_cap)) return -1;
    }
    const uint32_t tl = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) ? 4u : 0u;
    const uint64_t o = x.o;
    const int64_t L = (int64_t)x.len;
    // the window kernel's fast-path rules (malformed / guarded frames are its business)
    if (o > (uint64_t)a.buf_len || L > a.buf_len - (int64_t)o || L < (int64_t)tl) return 0;
    const int64_t lc = L - (int64_t)tl, E = (int64_t)o + lc;
    if ((int64_t)o < 67 || E + 8 > a.buf_len || lc < 8 || lc > (int64_t)kLaneChunks * 64) return 0;
    o_out = (int64_t)o;
    lc_out = (uint32_t)lc;
    return (int)((lc + 63) >> 6);
}

// counts[c] = frames of class c; each thread takes kSortPer frames per round, loads first
__global__ __launch_bounds__(kSortThreads) void crc_classify_kernel(FrameArgs a, uint32_t* counts) {
    __shared__ uint32_t h[kClasses];
    for (int i = threadIdx.x; i < kClasses; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t step = (uint64_t)gridDim.x * kSortTile;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kSortTile; t0 < a.n; t0 += step) {
        FrameIn x[kSortPer];
#pragma unroll
        for (int k = 0; k < kSortPer; ++k) x[k] = load_frame(a, t0 + (uint64_t)k * kSortThreads + threadIdx.x);
#pragma unroll
        for (int k = 0; k < kSortPer; ++k) {
            int64_t o;
            uint32_t lc;
            const int c = crc_class(a, t0 + (uint64_t)k * kSortThreads + threadIdx.x, x[k], o, lc);
            const int c0 = __shfl(c, 0);
            if (__all(c == c0)) {  // a wave of one class (uniform logs): one atomic
                if ((threadIdx.x & 63) == 0 && c0 >= 0) atomicAdd(&h[c0], 64u);
            } else if (c >= 0) {
                atomicAdd(&h[c], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kClasses; i += blockDim.x)
        if (h[i]) atomicAdd(&counts[i], h[i]);
}

// Scatter: lane-path records by ascending chunk count into rec[], the window kernel's frame numbers
// into widx[].  cursor[c] (zeroed) hands each block its range within class c.
__global__ __launch_bounds__(kSortThreads) void crc_scatter_kernel(FrameArgs a, const uint32_t* counts, uint32_t* cursor,
                                                                   LaneRec* rec, uint32_t* widx) {
    __shared__ uint32_t h[kClasses], base[kClasses];
    for (int i = threadIdx.x; i < kClasses; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kSortTile;
    int cls[kSortPer];
    uint32_t rank[kSortPer], lcs[kSortPer];
    int64_t os[kSortPer];
    FrameIn x[kSortPer];
#pragma unroll
    for (int k = 0; k < kSortPer; ++k) x[k] = load_frame(a, t0 + (uint64_t)k * kSortThreads + threadIdx.x);
#pragma unroll
    for (int k = 0; k < kSortPer; ++k) {
        const uint64_t f = t0 + (uint64_t)k * kSortThreads + threadIdx.x;
        cls[k] = crc_class(a, f, x[k], os[k], lcs[k]);
        const int c0 = __shfl(cls[k], 0);
        if (__all(cls[k] == c0)) {  // a wave of one class: one atomic, ranks by lane
            uint32_t b = 0;
            if ((threadIdx.x & 63) == 0 && c0 >= 0) b = atomicAdd(&h[c0], 64u);
            rank[k] = (uint32_t)__shfl((int)b, 0) + (uint32_t)(threadIdx.x & 63);
        } else {
            rank[k] = cls[k] >= 0 ? atomicAdd(&h[cls[k]], 1u) : 0u;
        }
    }
    __syncthreads();
    __shared__ uint32_t cnt[kClasses];
    if (threadIdx.x < kClasses) cnt[threadIdx.x] = counts[threadIdx.x];  // one load per class, in parallel
    __syncthreads();
    if (threadIdx.x < kClasses) {
        const int c = threadIdx.x;
        uint32_t b = 0;  // class c's first record: classes 1..c-1 before it (class 0: its own list)
        for (int j = 1; j < c; ++j) b += cnt[j];
        base[c] = b + (h[c] ? atomicAdd(&cursor[c], h[c]) : 0u);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortPer; ++k) {
        const uint64_t f = t0 + (uint64_t)k * kSortThreads + threadIdx.x;
        if (cls[k] > 0) {
            LaneRec r;
            r.o = os[k];
            r.lc = lcs[k];
            r.f = (uint32_t)f;
            rec[base[cls[k]] + rank[k]] = r;
        } else if (cls[k] == 0) {
            widx[base[0] + rank[k]] = (uint32_t)f;
        }
    }
}

struct LaneArgs {
    const uint8_t* buf;
    uint8_t* wbuf;
    const LaneRec* rec;
    const uint32_t* counts;
    uint32_t init;
    uint32_t flags;
    uint32_t* crc_out;
    uint64_t* bad_bits;
    unsigned long long* n_bad;
    const uint32_t* slice;
    const uint32_t* shift32;
    const uint32_t* lanetab;  // Q > 1: lane-distance tables build_crc_lane_tables(Q, 64)
    const uint32_t* zwin;     // Q > 1: advance over one Q x 64-byte window
    uint32_t cls_lo, cls_hi;  // the chunk-count classes this launch folds
    uint32_t slot_cap;
    uint32_t* seg_first_bad;
    const uint64_t* seg_first;
    uint32_t* dense_crc;
    uint64_t* dense_bad;
    uint64_t frame_cap;
};

// One wave = one group of G = 64 / Q consecutive records, Q lanes per frame (lane l: record
// G g + l / Q, chunk position l % Q); groups g = wave, wave + waves, ... (the records ascend by
// length, so every wave gets a like mix).  A frame's CRC span is cut into end-anchored windows of
// Q chunks of 64 B.  A group runs nmax = its longest frame's window count steps; window k of the
// group ends at E - W (nmax - 1 - k) for every frame, so shorter frames start later and all end at
// step nmax - 1.  Q = 1: the lane carries its register from chunk to chunk (no combine).  Q > 1:
// every chunk is folded from zero and the window's register is the XOR of the chunks advanced
// over the bytes after them (lane tables + DPP reduce), windows chained by a W-byte advance.
// Same 3-slot register ring with static roles as the window kernel.
template <int Q>
__global__ __launch_bounds__(kCrcThreads) void crc_lanes_kernel(LaneArgs a) {
    constexpr int kSliceBytes = 128 * 1024;
    constexpr int kWaves = kCrcThreads / 64;
    constexpr int G = 64 / Q;
    constexpr int64_t W = 64 * Q;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    uint32_t nbeg = 0, nrec = 0;  // this launch's records: rec[nbeg, nbeg + nrec)
    for (uint32_t c = 1; c <= a.cls_hi; ++c) {
        const uint32_t k = a.counts[c];
        if (c < a.cls_lo) nbeg += k;
        else nrec += k;
    }
    const LaneRec* rec = a.rec + nbeg;
    const uint32_t ngroups = (nrec + G - 1) / G;
    if ((uint32_t)blockIdx.x * kWaves >= ngroups) return;  // no group for this block
    uint32_t* lch = lds + kSliceBytes / 4;
    uint32_t* llane = lch + 1024;
    uint32_t* lzw = llane + 4096;
    for (int i = threadIdx.x; i < kSliceBytes / 4; i += blockDim.x) {
        const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
        lds[i] = a.slice[((region * 2 + half) << 8) | e];
    }
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lch[i] = a.shift32[i];
    if constexpr (Q > 1) {
        for (int i = threadIdx.x; i < 4096; i += blockDim.x) llane[i] = a.lanetab[i];
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) lzw[i] = a.zwin[i];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int gl = lane & (Q - 1);  // chunk position within the window
    const uint32_t c = lane & 31;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | (c << 2);
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
    const uint32_t nwv = gridDim.x * kWaves;

    struct Rec {
        int64_t o;
        uint32_t lc;
        uint32_t f;  // 0xFFFFFFFF: no frame in this lane
    };
    struct Task {
        Rec r;
        int64_t be;     // end of this lane's chunk: E - W (nmax - 1 - k) - 64 (Q - 1 - gl)
        uint32_t g;     // group (>= ngroups: done)
        uint32_t k;     // step
        uint32_t nmax;  // steps of the group
    };
    // Record of this lane's frame in group g.  The load is issued unconditionally (clamped index),
    // so every step issues the same vector memory operations and the compiler's vmcnt waits stay
    // counted -- a conditional load here cost a full drain of the ring at each group change.
    auto fetch = [&](uint32_t g) -> Rec {
        const uint64_t i = (uint64_t)g * G + (uint64_t)(lane / Q);
        const bool ok = g < ngroups && i < nrec;
        const LaneRec x = rec[ok ? i : 0];
        return Rec{x.o, x.lc, ok ? x.f : 0xFFFFFFFFu};
    };
    auto enter = [&](uint32_t g, const Rec& r) -> Task {
        Task t{r, 0, g, 0u, 0u};
        if (g < ngroups) {
            const uint32_t last = nrec - 1 - g * G < (uint32_t)(G - 1) ? nrec - 1 - g * G : (uint32_t)(G - 1);
            const uint32_t nw = (uint32_t)(((int64_t)r.lc + W - 1) / W);  // longest frame: the last one
            t.nmax = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)nw, (int)(last * Q)));
            t.be = r.o + (int64_t)r.lc - W * (int64_t)(t.nmax - 1) - 64 * (int64_t)(Q - 1 - gl);
        }
        return t;
    };
    Rec pre = fetch(wv + nwv);  // record of the group after the newest task's group
    auto next = [&](const Task& x) -> Task {
        Task t = x;
        if (x.g < ngroups) t = x.k + 1 < x.nmax ? Task{x.r, x.be + W, x.g, x.k + 1, x.nmax} : enter(x.g + nwv, pre);
        pre = fetch(t.g + nwv);  // every step (see fetch)
        return t;
    };
    // chunk of task x in this lane: [be - 64, be); loads 72 bytes from the 4-aligned
    // b0 = be - 64 - (E & 3) (the last 8 hold the trailer)
    auto load = [&](const Task& x, uint32_t (&dd)[18]) {
        const uint8_t* src = a.buf;
        if (x.g < ngroups && x.r.f != 0xFFFFFFFFu && x.be > x.r.o)
            src = a.buf + (x.be - 64 - (int64_t)((uint32_t)x.r.o + x.r.lc & 3u));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4a v = *reinterpret_cast<const u32x4a*>(src + 16 * q);
            dd[4 * q] = v.x;
            dd[4 * q + 1] = v.y;
            dd[4 * q + 2] = v.z;
            dd[4 * q + 3] = v.w;
        }
        dd[16] = *reinterpret_cast<const uint32_t*>(src + 64);
        dd[17] = *reinterpret_cast<const uint32_t*>(src + 68);
    };
    uint32_t R = 0;  // the frame's register over its windows (chunks, Q = 1) so far
    auto fold = [&](const Task& x, uint32_t (&d)[18]) {
        if (x.g >= ngroups) return;
        const bool valid = x.r.f != 0xFFFFFFFFu;
        const int64_t E = x.r.o + (int64_t)x.r.lc;
        const uint32_t sh = (uint32_t)(E & 3);
        const int64_t be = x.be;
        const bool act = valid && be > x.r.o;
        const int64_t q0l = be - 64 - (int64_t)sh - x.r.o;
        if (__any(act && q0l < 4)) mask_frame_start(d, q0l, act && q0l < 4, a.init);
        // two chains of 8 words, joined over 32 zero bytes
        auto chains = [&](auto W) {
            uint32_t x0 = (Q == 1 ? R : 0u) ^ W(0), x1 = W(8);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                x0 = fold_x(lds, x0, lb, j < 7 ? W(j + 1) : 0u);
                x1 = fold_x(lds, x1, lb, j < 7 ? W(9 + j) : 0u);
            }
            return zshift_x(lch, x0, x1);
        };
        uint32_t r;
        if (__all(sh == 0 || !act))
            r = chains([&](int i) { return d[i]; });
        else
            r = chains([&](int i) { return __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh); });
        if constexpr (Q == 1) {
            R = act ? r : 0u;
        } else {
            r = act ? lane_advance(llane, c, r) : 0u;
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
            if constexpr (Q >= 4) r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x4E, 0xF, 0xF, false);
            if constexpr (Q >= 8) r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x141, 0xF, 0xF, false);
            if constexpr (Q >= 16) r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x140, 0xF, 0xF, false);
            R = zshift_x(lzw, R, r);
        }
        if (x.k + 1 == x.nmax) {  // every frame of the group ends at this step
            if (valid && gl == Q - 1) {  // the lane whose chunk ends at E
                const uint32_t value = ~R;
                bool bad = false;
                if (a.flags & RH_CRC_STAMP) {
                    a.wbuf[E + 0] = (uint8_t)(value >> 24);
                    a.wbuf[E + 1] = (uint8_t)(value >> 16);
                    a.wbuf[E + 2] = (uint8_t)(value >> 8);
                    a.wbuf[E + 3] = (uint8_t)value;
                } else if (a.flags & RH_CRC_VERIFY) {
                    bad = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[17], d[16], sh)) != value;
                }
                emit_frame(a, x.r.f, value, bad);
            }
            R = 0;
        }
    };
    Task T0 = enter(wv, fetch(wv));
    Task T1 = next(T0);
    Task T2 = next(T1);
    uint32_t d0[18], d1[18], d2[18];
    if (T0.g < ngroups) {
        load(T0, d0);
        load(T1, d1);
    }
    while (T0.g < ngroups) {
        load(T2, d2);
        fold(T0, d0);
        T0 = next(T2);
        if (T1.g >= ngroups) break;
        load(T0, d0);
        fold(T1, d1);
        T1 = next(T0);
        if (T2.g >= ngroups) break;
        load(T1, d1);
        fold(T2, d2);
        T2 = next(T1);
    }
}

template <int Q>
hipError_t launch_lanes(const LaneArgs& l, uint64_t n, uint64_t cus, hipStream_t stream) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_lanes_kernel<Q>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLaneLds);
    if (attr != hipSuccess) return attr;
    constexpr uint64_t per_block = (uint64_t)(kCrcThreads / 64) * (64 / Q);  // frames of one round of groups
    const uint64_t grid = (n + per_block - 1) / per_block < cus ? (n + per_block - 1) / per_block : cus;
    hipLaunchKernelGGL(crc_lanes_kernel<Q>, dim3((uint32_t)grid), dim3(kCrcThreads), kLaneLds, stream, l);
    return hipGetLastError();
}

// ---- packed path: every frame's 64-byte chunks packed across the wave, in table order -----------
// The lane kernels above fold whole windows of Q chunks per frame, so a frame pays up to a window
// of padding, the start-of-frame masking runs in every window that holds a frame start, and the
// frames must first be sorted by length.  Here a wave takes 64 frames of the table in order (a
// task) and folds their chunks back to back, 64 chunks per step, whatever the frames' lengths:
//   * a frame's span is cut into end-anchored chunks 0..k (k = ceil(span / 64) - 1); chunk 0 (the
//     one holding the frame start, bytes before it zeroed) is folded for all 64 frames in ONE
//     masked pass per task, so the steps fold chunks 1..k unmasked;
//   * reset()'s state is not injected into the bytes: it enters as A^span(init), one table lookup
//     per frame (initv), A = the zero-byte advance;
//   * in a step, lane l holds packed chunk 64 s + l; its register R (folded from zero) is advanced
//     to the end of its 32-lane half with the lane table of distance 64 (31 - l mod 32) (LDS,
//     bank = lane & 31, conflict free), a prefix XOR inside each half (DPP) sums every frame's
//     chunks there, and the part of a frame begun before the half enters as one uniform 2 KiB
//     advance (scalar table loads) -- the frame's register at the end of the half;
//   * a frame ending in the step stores that value; the task's emit pass moves it back to the frame
//     end with the inverse lane map (global table, once per frame), XORs the init term and checks
//     or stamps the trailer.
// Chunk k - m of a frame ending at E covers [E - 64 (m + 1), E - 64 m): the wave's loads of a step
// are one contiguous run when its frames are contiguous (a segment's frame table).
// Frames the fast path cannot load safely, malformed ones and spans over kCrcInitSpan go to a list
// for the window kernel (crc_frames_kernel<true>).
// Steps of loads in flight per wave beyond the one being folded: 1 (two register sets, 16 waves
// per CU) or 2 (three sets; the registers that takes allow 12 waves per CU).
#ifndef RH_PACK_DEPTH
#define RH_PACK_DEPTH 1
#endif
constexpr int kPackThreads = RH_PACK_DEPTH >= 2 ? 768 : kCrcThreads;
constexpr int kPackWaves = kPackThreads / 64;
constexpr int kPackTabBytes = 128 * 1024 + 4096 + 16384;  // slicing tables, 32-byte join, lane maps
// Fold chains per 64-byte chunk: 2 (8 words each, one 32-byte join) or 4 (4 words each, joined as
// a tree: two 16-byte joins, then one 32-byte join; the 16-byte table takes the last 4 KiB of LDS).
#ifndef RH_PACK_CHAINS
#define RH_PACK_CHAINS 2
#endif
constexpr int kPackLds = kPackTabBytes + kPackWaves * 512 +  // + per wave: 64 step marks, 64 frame values
                         (RH_PACK_CHAINS == 4 ? 4096 : 0);
static_assert(kPackLds <= 160 * 1024, "LDS budget");

struct PackArgs {
    FrameArgs f;                       // buffers, outputs, slot-mode fields (f.n = table entries)
    const uint32_t* ftab;              // build_crc_lane_tables(32, 64)
    const uint32_t* inv;               // build_crc_inverse_lane_tables()
    const uint32_t* z16;               // [4][256] advance over 16 zero bytes (RH_PACK_CHAINS 4)
    const uint32_t* z64;               // [4][256] advance over 64 zero bytes
    const uint32_t* z2k;               // [4][256] advance over 2048 zero bytes (uniform lookups)
    const uint32_t* z4k;               // [4][256] advance over 4096 zero bytes (uniform lookups)
    const uint32_t* initv;             // [kCrcInitSpan + 1]: A^k(init)
    const uint64_t* seg_first;         // slot mode: dense frame d lives in segment upper_bound - 1
    const unsigned long long* total;   // slot mode: frames in the dense numbering
    uint64_t n_seg;
    uint32_t* counts;                  // counts[0]: frames listed for the window kernel (zeroed)
    uint32_t* widx;
};

typedef __attribute__((address_space(4))) const uint32_t const_u32_t;
// Zero-advance of a wave-uniform register: scalar loads through the constant cache.
__device__ __forceinline__ uint32_t zshift_uniform(const uint32_t* tab, uint32_t r) {
    r = __builtin_amdgcn_readfirstlane(r);
    const_u32_t* t = (const_u32_t*)tab;
    return t[r & 0xffu] ^ t[256 + ((r >> 8) & 0xffu)] ^ t[512 + ((r >> 16) & 0xffu)] ^ t[768 + (r >> 24)];
}

// Inclusive XOR prefix inside each 32-lane half (row shifts, then row 0 / row 2's last lane into
// rows 1 / 3).
__device__ __forceinline__ uint32_t half_prefix_xor(uint32_t x) {
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    return x;
}

__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d, 64);
        v += lane >= d ? u : 0u;
    }
    return v;
}

// 64 bytes at the 4-aligned b0 plus the next word: the chunk [b0 + sh, b0 + sh + 64).
__device__ __forceinline__ void load_chunk(const uint8_t* src, uint32_t (&d)[17]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32x4a v = *reinterpret_cast<const u32x4a*>(src + 16 * q);
        d[4 * q] = v.x;
        d[4 * q + 1] = v.y;
        d[4 * q + 2] = v.z;
        d[4 * q + 3] = v.w;
    }
    d[16] = *reinterpret_cast<const uint32_t*>(src + 64);
}

// CRC register of the 16 words (from zero), XOR `extra`: two chains of 8 joined over 32 zero bytes
// (`extra` rides in the second chain's last fold).
__device__ __forceinline__ uint32_t fold16(const uint32_t* lds, const uint32_t* lch, const uint32_t (&w)[16],
                                           const uint32_t (&lb)[4], uint32_t extra = 0u) {
    uint32_t x0 = w[0], x1 = w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        x0 = fold_x(lds, x0, lb, j < 7 ? w[j + 1] : 0u);
        x1 = fold_x(lds, x1, lb, j < 7 ? w[9 + j] : extra);
    }
    return zshift_x(lch, x0, x1);
}

// The same over four chains of 4 words: half the dependent LDS rounds per chain, three joins.
__device__ __forceinline__ uint32_t fold16_4(const uint32_t* lds, const uint32_t* lch, const uint32_t* lz16,
                                             const uint32_t (&w)[16], const uint32_t (&lb)[4], uint32_t extra = 0u) {
    uint32_t x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = w[4 * q];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = fold_x(lds, x[q], lb, j < 3 ? w[4 * q + j + 1] : (q == 3 ? extra : 0u));
    return zshift_x(lch, zshift_x(lz16, x[0], x[1]), zshift_x(lz16, x[2], x[3]));
}

// A/B: 1 folds chunk 0 in the steps (a per-lane mask on every word of every step) instead of one
// masked chunk-0 pass per task.  It removes the chunk-0 pass's refetched lines (ragged 64-2048 B,
// 64 x 32 MiB: FETCH_SIZE 2545 -> 2402 MB) but the masking makes the step VALU-heavier: crc_pack
// 1054 -> 1086 us at 128 segments (profiles/r04/ragged_c0/).  Off.
#ifndef RH_PACK_C0STEP
#define RH_PACK_C0STEP 0
#endif

template <bool SLOT>
__global__ __launch_bounds__(kPackThreads) void crc_pack_kernel(PackArgs pk_arg) {
    // slot variant: fields read from the kernarg segment where used (scalar loads the compiler can
    // repeat), not held in SGPRs across the step loop -- its extra pointers spilled
    const PackArgs& p = SLOT ? rh::kernarg_struct<PackArgs>() : pk_arg;
    const FrameArgs& a = p.f;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    const uint64_t nfr = SLOT ? (uint64_t)*p.total : a.n;
    const uint64_t ntask = (nfr + 63) / 64;
    if ((uint64_t)blockIdx.x * kPackWaves >= ntask) return;  // block-uniform
    constexpr int kSliceBytes = 128 * 1024;
    uint32_t* lch = lds + kSliceBytes / 4;
    uint32_t* lf = lch + 1024;
    for (int i = threadIdx.x; i < kSliceBytes / 4; i += blockDim.x) {
        const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
        lds[i] = a.slice[((region * 2 + half) << 8) | e];
    }
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lch[i] = a.shift32[i];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lf[i] = p.ftab[i];
    uint32_t* lz16 = lds + kPackTabBytes / 4 + kPackWaves * 128;
    if (RH_PACK_CHAINS == 4)
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) lz16[i] = p.z16[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | (c << 2);
    auto fold = [&](const uint32_t (&w)[16], uint32_t extra) {
        if constexpr (RH_PACK_CHAINS == 4) return fold16_4(lds, lch, lz16, w, lb, extra);
        else return fold16(lds, lch, w, lb, extra);
    };
    const uint32_t wid = threadIdx.x >> 6;
    uint32_t* mark = lds + kPackTabBytes / 4 + wid * 128;  // [64] step marks
    uint32_t* vst = mark + 64;                               // [64] frame registers (end of half)
    const uint32_t tl = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) ? 4u : 0u;
    const uint32_t hs = (uint32_t)lane & 32u;

    for (uint64_t t = (uint64_t)blockIdx.x * kPackWaves + wid; t < ntask; t += (uint64_t)gridDim.x * kPackWaves) {
        // ---- the task's 64 frames: lane j holds frame j ----
        const uint64_t d = t * 64 + (uint64_t)lane;
        const bool have = d < nfr;
        uint32_t f = (uint32_t)d;  // table entry (the launcher keeps tables below 2^32 entries)
        if (SLOT) {
            // the task's first frame: the largest segment with seg_first <= 64 t (seg_first[0] = 0),
            // a wave-uniform search (scalar loads); a lane past that segment's end steps forward
            const const_u32_t* sf = (const const_u32_t*)p.seg_first;  // u64 entries as u32 pairs
            auto first_of = [&](uint64_t s) -> uint64_t {
                const uint32_t i = __builtin_amdgcn_readfirstlane((uint32_t)s);
                return ((uint64_t)sf[2 * (uint64_t)i + 1] << 32) | sf[2 * (uint64_t)i];
            };
            const uint64_t d0 = t * 64;
            uint64_t lo = 0, hi = p.n_seg;
            while (hi - lo > 1) {
                const uint64_t mid = (lo + hi) >> 1;
                if (first_of(mid) <= d0) lo = mid;
                else hi = mid;
            }
            uint64_t seg = lo;
            uint64_t next = seg + 1 < p.n_seg ? first_of(seg + 1) : ~0ull;
            uint64_t base = first_of(seg);
            while (__any(have && d >= next)) {  // rare: the task crosses into later segments
                if (have && d >= next) {
                    ++seg;
                    base = next;
                    next = seg + 1 < p.n_seg ? p.seg_first[seg + 1] : ~0ull;
                }
            }
            f = (uint32_t)(seg * (uint64_t)a.slot_cap + (d - base));
        }
        uint64_t o = 0;
        uint32_t L = 0;
        if (have) {
            o = a.off[f];
            L = a.len[f];
        }
        const bool malformed = o > (uint64_t)a.buf_len || (int64_t)L > a.buf_len - (int64_t)o || L < tl;
        const int64_t lcs = (int64_t)L - (int64_t)tl;
        const int64_t E = (int64_t)o + lcs;
        // (frames within 67 bytes of the buffer start: chunk 0's words before byte 0 load as zero)
        const bool pk = have && !malformed && E + 8 <= a.buf_len && lcs >= 8 && lcs <= (int64_t)rh::kCrcInitSpan;
        const bool left = have && !pk;
        const uint64_t lb_left = __ballot(left);
        if (lb_left) {  // the window kernel's frames (guarded, malformed, long)
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(p.counts, (uint32_t)__popcll(lb_left));
            base = (uint32_t)__shfl((int)base, 0);
            if (left)
                p.widx[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(lb_left >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lb_left, 0u))] =
                    (uint32_t)f;
        }
        const uint32_t lc = pk ? (uint32_t)lcs : 0u;
        const uint32_t k = pk ? (lc - 1) >> 6 : 0u;  // chunks after chunk 0
        // packed chunks per frame: 1..k (chunk 0 in its own pass) or 0..k (chunk 0 in the steps)
        const uint32_t kp = RH_PACK_C0STEP ? (pk ? k + 1u : 0u) : k;
        const uint32_t Qi = wave_scan_add(kp, lane);
        const uint32_t Q = Qi - kp;                  // packed position of the frame's first packed chunk
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)Qi, 63);
        const uint32_t sh = (uint32_t)E & 3u;
        // trailer and init term (needed at the end of the task; loaded now)
        uint32_t tw0 = 0, tw1 = 0, iv = 0;
        if (pk) {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(a.buf + (E & ~(int64_t)3));
            tw0 = tp[0];
            tw1 = tp[1];
            iv = p.initv[lc];
        }
        mark[lane] = 0;
        // ---- chunk 0 of every frame: bytes before the frame start zeroed ----
        uint32_t f0 = 0, fs = 0;
        if (!RH_PACK_C0STEP) {
            uint32_t dd[17];
            const int64_t b0 = E - 64 * (int64_t)k - 64 - (int64_t)sh;  // chunk 0's 4-aligned start
            if (__any(pk && b0 < 0)) {  // a frame near the buffer start (rare): word by word
#pragma unroll
                for (int i = 0; i < 17; ++i)
                    dd[i] = pk && b0 + 4 * i >= 0 ? *reinterpret_cast<const uint32_t*>(a.buf + b0 + 4 * i) : 0u;
            } else {
                load_chunk(pk ? a.buf + b0 : a.buf, dd);
            }
            uint32_t w[16];
            const int32_t g8 = 8 * (int32_t)((k + 1) * 64 - lc);  // 8 x bytes before the frame
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int32_t kk = min(max(g8 - 32 * i, 0), 32);
                w[i] = __builtin_amdgcn_alignbyte(dd[i + 1], dd[i], sh) & (uint32_t)(~0ull << kk);
            }
            f0 = fold(w, 0u);
            fs = 0;
            if (k > 0) {  // chunk 0 seen from the end of chunk 1
#pragma unroll
                for (int q = 0; q < 4; ++q) fs ^= p.z64[256 * q + ((f0 >> (8 * q)) & 0xffu)];
            }
        }

        // ---- steps: 64 packed chunks (1..k of the frames, in order) each ----
        struct Step {
            uint32_t j, i, m, fs;  // frame lane, chunk index, chunks after it, chunk-0 term
            int64_t be;            // chunk end
            uint32_t sh;
            int32_t g8;            // RH_PACK_C0STEP: 8 x the bytes before the frame start (chunk 0)
            bool valid;
        };
        auto map = [&](uint32_t s, uint32_t jprev) -> Step {
            if (kp > 0 && (Q >> 6) == s) mark[Q & 63u] = ((s + 1u) << 8) | (uint32_t)lane;
            __builtin_amdgcn_wave_barrier();
            const uint32_t rd = mark[lane];
            const uint64_t M = __ballot((rd >> 8) == s + 1u) & (~0ull >> (63 - lane));
            const int src = M ? 63 - __builtin_clzll(M) : 0;
            const uint32_t jr = (uint32_t)__shfl((int)rd, src) & 0xffu;
            Step x;
            x.j = M ? jr : jprev;
            const uint32_t P = s * 64u + (uint32_t)lane;
            x.valid = P < T;
            const uint32_t Qj = (uint32_t)__shfl((int)Q, (int)x.j);
            const uint32_t kj = (uint32_t)__shfl((int)k, (int)x.j);
            const uint32_t elo = (uint32_t)__shfl((int)(uint32_t)E, (int)x.j);
            const uint32_t ehi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)E >> 32), (int)x.j);
            x.fs = RH_PACK_C0STEP ? 0u : (uint32_t)__shfl((int)fs, (int)x.j);
            x.i = P - Qj + (RH_PACK_C0STEP ? 0u : 1u);
            x.m = kj - x.i;
            x.g8 = 0;
            if (RH_PACK_C0STEP) {
                const uint32_t lcj = (uint32_t)__shfl((int)lc, (int)x.j);
                x.g8 = x.i == 0u ? 8 * (int32_t)((kj + 1u) * 64u - lcj) : 0;
            }
            const int64_t Ej = (int64_t)(((uint64_t)ehi << 32) | elo);
            x.be = Ej - 64 * (int64_t)x.m;
            x.sh = elo & 3u;
            return x;
        };
        auto load = [&](const Step& x, uint32_t (&dd)[17]) {
            const int64_t b0 = x.be - 64 - (int64_t)x.sh;
            if (RH_PACK_C0STEP && __any(x.valid && b0 < 0)) {  // chunk 0 of a frame near the buffer start (rare)
#pragma unroll
                for (int i = 0; i < 17; ++i)
                    dd[i] = x.valid && b0 + 4 * i >= 0 ? *reinterpret_cast<const uint32_t*>(a.buf + b0 + 4 * i) : 0u;
                return;
            }
            load_chunk(x.valid ? a.buf + b0 : a.buf, dd);
        };
        const uint32_t nsteps = (T + 63) >> 6;
        uint32_t carry = 0;  // register of the frame running past the previous step (at its end)
        // one step: fold `cur` (its chunk in dc) while step s + D's map and loads go out into nx / dn
        // (pm: step s + D - 1, whose last lane's frame carries into step s + D)
        constexpr uint32_t D = RH_PACK_DEPTH;
        auto step = [&](uint32_t s, Step& cur, uint32_t (&dc)[17], const Step& pm, Step& nx, uint32_t (&dn)[17]) {
            if (s + D < nsteps) {
                nx = map(s + D, (uint32_t)__builtin_amdgcn_readlane((int)pm.j, 63));
                load(nx, dn);
            }
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                w[i] = __builtin_amdgcn_alignbyte(dc[i + 1], dc[i], cur.sh);
                if (RH_PACK_C0STEP) {  // chunk 0: the bytes before the frame start zeroed
                    const int32_t kk = min(max(cur.g8 - 32 * i, 0), 32);
                    w[i] &= (uint32_t)(~0ull << kk);
                }
            }
            const uint32_t R = fold(w, !RH_PACK_C0STEP && cur.i == 1u ? cur.fs : 0u);
            const uint32_t K0 = zshift_uniform(p.z2k, carry);  // off the step's dependent chain
            const uint32_t C4 = zshift_uniform(p.z4k, carry);
            const uint32_t y = cur.valid ? lane_advance(lf, c, R) : 0u;
            const uint32_t px = half_prefix_xor(y);
            const int a0 = lane - (int)cur.i + (RH_PACK_C0STEP ? 0 : 1);  // lane of the frame's first packed chunk (may be < 0)
            const bool cont = a0 < (int)hs;        // the frame began before this half
            const int src = (cont ? (int)hs : a0) - 1;
            const uint32_t before = (uint32_t)__shfl((int)px, src < 0 ? 0 : src);
            const uint32_t seg = px ^ (cont ? 0u : (src >= (int)hs ? before : 0u));
            const uint64_t contM = __ballot(cont);
            // the carried frame at the end of half 0 (K0) and of half 1 -- by linearity the half-1
            // term splits into Z2k(half 0's running frame) ^ Z4k(carry): only the former waits on
            // this step's prefix
            const uint32_t s31 = (uint32_t)__builtin_amdgcn_readlane((int)seg, 31);
            const uint32_t K1 = zshift_uniform(p.z2k, s31) ^ (((contM >> 31) & 1u) ? C4 : 0u);
            const uint32_t tot = seg ^ (cont ? (hs ? K1 : K0) : 0u);
            const bool ends = cur.valid && cur.m == 0u;
            if (ends) vst[cur.j] = tot;
            const uint64_t runM = __ballot(cur.valid && cur.m != 0u);
            carry = ((runM >> 63) & 1u) ? (uint32_t)__builtin_amdgcn_readlane((int)tot, 63) : 0u;
        };
        // D + 1 register sets in turn (no copy of a prefetched chunk from one set to another)
        Step sa{}, sb{};
        uint32_t da[17], db[17];
        if (nsteps) {
            sa = map(0, 0);
            load(sa, da);
        }
        if constexpr (D == 1) {
            for (uint32_t s = 0; s < nsteps; s += 2) {
                step(s, sa, da, sa, sb, db);
                if (s + 1 >= nsteps) break;
                step(s + 1, sb, db, sb, sa, da);
            }
        } else {
            Step sc{};
            uint32_t dd3[17];
            if (nsteps > 1) {
                sb = map(1, (uint32_t)__builtin_amdgcn_readlane((int)sa.j, 63));
                load(sb, db);
            }
            for (uint32_t s = 0; s < nsteps; s += 3) {
                step(s, sa, da, sb, sc, dd3);
                if (s + 1 >= nsteps) break;
                step(s + 1, sb, db, sc, sa, da);
                if (s + 2 >= nsteps) break;
                step(s + 2, sc, dd3, sa, sb, db);
            }
        }
        __builtin_amdgcn_wave_barrier();

        // ---- emit: frame lane j finishes frame j ----
        if (pk) {
            uint32_t V = f0;
            if (RH_PACK_C0STEP || k > 0) {
                const uint32_t tot = vst[lane];
                const uint32_t* im = p.inv + (size_t)((Q + kp - 1u) & 31u) * 128u;   // its last chunk's position
                V = 0;
#pragma unroll
                for (int q = 0; q < 8; ++q) V ^= im[q * 16 + ((tot >> (4 * q)) & 15u)];
            }
            const uint32_t value = ~(V ^ iv);
            bool bad = false;
            if (a.flags & RH_CRC_STAMP) {
                a.wbuf[E + 0] = (uint8_t)(value >> 24);
                a.wbuf[E + 1] = (uint8_t)(value >> 16);
                a.wbuf[E + 2] = (uint8_t)(value >> 8);
                a.wbuf[E + 3] = (uint8_t)value;
            } else if (a.flags & RH_CRC_VERIFY) {
                bad = __builtin_bswap32(__builtin_amdgcn_alignbyte(tw1, tw0, sh)) != value;
            }
            if (!SLOT) {
                emit_frame(a, f, value, bad);
            } else {  // emit_frame's slot mode, with the dense index already known
                if (a.crc_out) a.crc_out[f] = value;
                if (bad) {
                    if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    const uint32_t seg = f / a.slot_cap;
                    if (a.seg_first_bad) atomicMin(a.seg_first_bad + seg, f - seg * a.slot_cap);
                }
                if (d < a.frame_cap) {
                    if (a.dense_crc) a.dense_crc[d] = value;
                    if (bad && a.dense_bad)
                        atomicOr(reinterpret_cast<unsigned long long*>(a.dense_bad + (d >> 6)), 1ull << (d & 63));
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// A^k(init) for k = 0..kCrcInitSpan (a start state other than reset()'s; that one is cached in ctx)
__global__ __launch_bounds__(256) void crc_init_terms_kernel(const uint32_t* shift, uint32_t init, uint32_t* out) {
    const uint32_t kk = blockIdx.x * blockDim.x + threadIdx.x;
    if (kk > rh::kCrcInitSpan) return;
    uint32_t x = init;
    for (int b = 0; b < 16; ++b)
        if ((kk >> b) & 1u) x = zshift(shift + (size_t)b * 1024, x);
    out[kk] = x;
}

// Slot mode of the packed kernel (the read path): dense frame numbering over the slotted table.
struct SlotPlan {
    const uint64_t* seg_first = nullptr;
    const unsigned long long* total = nullptr;
    uint64_t n_seg = 0;
};

#ifndef RH_CRC_PACK  // A/B builds override: 0 = the length-class split (classify / sort / lane kernels)
#define RH_CRC_PACK 1
#endif

// packed kernel -> window kernel over the frames it lists, all on `stream`.
int launch_pack(rh_ctx* ctx, FrameArgs a, const SlotPlan& sp, hipStream_t stream) {
    static const hipError_t attr = [] {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_pack_kernel<false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kPackLds);
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_pack_kernel<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kPackLds);
        return e;
    }();
    RH_HIP(attr);
    const uint64_t cus = (uint64_t)(ctx->num_cus > 0 ? ctx->num_cus : 256);
    // scratch: counts, the window kernel's list widx[n], the init terms of a non-reset start state
    const bool own_init = a.init != 0xFFFFFFFFu;
    const size_t o_widx = 256, o_init = o_widx + ((size_t)a.n * 4 + 255) / 256 * 256;
    const size_t bytes = o_init + (own_init ? ((size_t)rh::kCrcInitSpan + 1) * 4 : 0);
    rh::PoolScratch scratch(stream);
    RH_HIP(scratch.alloc(ctx, bytes));
    uint32_t* counts = reinterpret_cast<uint32_t*>(scratch.bytes());
    uint32_t* widx = reinterpret_cast<uint32_t*>(scratch.bytes() + o_widx);
    RH_HIP(hipMemsetAsync(counts, 0, 4, stream));
    PackArgs p{};
    p.initv = ctx->d_initff;
    if (own_init) {
        uint32_t* iv = reinterpret_cast<uint32_t*>(scratch.bytes() + o_init);
        hipLaunchKernelGGL(crc_init_terms_kernel, dim3((rh::kCrcInitSpan + 256) / 256), dim3(256), 0, stream, ctx->d_shift,
                           a.init, iv);
        RH_HIP(hipGetLastError());
        p.initv = iv;
    }
    p.f = a;
    p.ftab = ctx->d_lane16 + (size_t)4 * 4096;  // Q = 32
    p.inv = ctx->d_inv32;
    p.z16 = ctx->d_shift + (size_t)4 * 1024;
    p.z64 = ctx->d_shift + (size_t)6 * 1024;
    p.z2k = ctx->d_shift + (size_t)11 * 1024;
    p.z4k = ctx->d_shift + (size_t)12 * 1024;
    p.seg_first = sp.seg_first;
    p.total = sp.total;
    p.n_seg = sp.n_seg;
    p.counts = counts;
    p.widx = widx;
    if (sp.total) {
        hipLaunchKernelGGL(crc_pack_kernel<true>, dim3((uint32_t)cus), dim3(kPackThreads), kPackLds, stream, p);
    } else {
        const uint64_t tasks = (a.n + 63) / 64, blocks = (tasks + kPackWaves - 1) / kPackWaves;
        hipLaunchKernelGGL(crc_pack_kernel<false>, dim3((uint32_t)(blocks < cus ? blocks : cus)), dim3(kPackThreads),
                           kPackLds, stream, p);
    }
    RH_HIP(hipGetLastError());
    a.counts = counts;
    a.widx = widx;
    constexpr uint64_t kBL = kBatchOf(true);
    const uint64_t wgrid = (a.n + kBL - 1) / kBL < cus ? (a.n + kBL - 1) / kBL : cus;
    hipLaunchKernelGGL(crc_frames_kernel<true>, dim3((uint32_t)wgrid), dim3(kCrcThreads), kCrcLdsOf(true), stream, a);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

// classify -> scatter -> lane kernels (4 and 8 lanes per frame) -> window kernel over the rest,
// all on `stream`.
int launch_frames(rh_ctx* ctx, FrameArgs a, hipStream_t stream, bool* dense_written = nullptr,
                  const SlotPlan& sp = SlotPlan{}, bool force_window = false) {
    static const hipError_t attr = [] {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_frames_kernel<false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kCrcLdsOf(false));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_frames_kernel<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kCrcLdsOf(true));
        return e;
    }();
    RH_HIP(attr);
    if (a.n > 0xFFFFFFFFull) return rh::fail(RH_E_RANGE, "CRC launch: more than 2^32 - 1 frames in one launch");
    a.slice = ctx->d_slice;
    a.shift32 = ctx->d_shift + (size_t)5 * 1024;  // 2^5 = 32 bytes: the fold-chain join
    a.zwin = ctx->d_shift + (size_t)10 * 1024;    // 2^10 = one 1 KiB window
    a.lanetab = ctx->d_lane16 + (size_t)3 * 4096;  // Q = 16
    const uint64_t cus = (uint64_t)(ctx->num_cus > 0 ? ctx->num_cus : 256);
    // The lane split pays a classify + scatter pass (~4 % of a config-5 launch); it is taken when the
    // buffer's mean frame length buf_len / n is at most kLaneMeanMax -- logs of short entries.
    // Logs of long frames (config 5's 4 KiB) and single spans stay on the window kernel alone.
    bool window_only = force_window || a.buf_len / a.n > kLaneMeanMax;
#ifdef RH_AB_WINDOW_ONLY  // A/B build (scripts/ab_build.sh): every frame on the window kernel
    window_only = true;
#endif
#ifdef RH_AB_PACK_ALL  // A/B build: every frame table on the packed kernel
    window_only = false;
#endif
    if (window_only) {
        // slot mode: the dense outputs are left to the caller's compaction (a dependent seg_first
        // load at every frame's end costs the window kernel more than that pass, config 5: -4 %)
        a.seg_first = nullptr;
        a.dense_crc = nullptr;
        a.dense_bad = nullptr;
        if (dense_written) *dense_written = false;
        const uint64_t wgrid = (a.n + kBatch - 1) / kBatch < cus ? (a.n + kBatch - 1) / kBatch : cus;
        hipLaunchKernelGGL(crc_frames_kernel<false>, dim3((uint32_t)wgrid), dim3(kCrcThreads), kCrcLdsOf(false),
                           stream, a);
        RH_HIP(hipGetLastError());
        return RH_OK;
    }
    if (dense_written) *dense_written = a.seg_first != nullptr;
    if (RH_CRC_PACK && (sp.total || !a.slot_nframes)) return launch_pack(ctx, a, sp, stream);
    // scratch: counts[kClasses], cursor[kClasses], rec[n], widx[n]
    const size_t o_rec = 1024, o_widx = o_rec + (size_t)a.n * sizeof(LaneRec), bytes = o_widx + (size_t)a.n * 4;
    rh::PoolScratch scratch(stream);  // released on every exit path
    RH_HIP(scratch.alloc(ctx, bytes));
    uint8_t* sb = scratch.bytes();
    uint32_t* counts = reinterpret_cast<uint32_t*>(sb);
    uint32_t* cursor = counts + kClasses;
    LaneRec* rec = reinterpret_cast<LaneRec*>(sb + o_rec);
    uint32_t* widx = reinterpret_cast<uint32_t*>(sb + o_widx);
    RH_HIP(hipMemsetAsync(counts, 0, 2 * kClasses * sizeof(uint32_t), stream));
    const uint64_t ntile = (a.n + kSortTile - 1) / kSortTile;
    const uint64_t cgrid = ntile < cus * 8 ? ntile : cus * 8;
    hipLaunchKernelGGL(crc_classify_kernel, dim3((uint32_t)cgrid), dim3(kSortThreads), 0, stream, a, counts);
    RH_HIP(hipGetLastError());
    hipLaunchKernelGGL(crc_scatter_kernel, dim3((uint32_t)((a.n + kSortTile - 1) / kSortTile)), dim3(kSortThreads), 0,
                       stream, a, counts, cursor, rec, widx);
    RH_HIP(hipGetLastError());
    LaneArgs l{};
    l.buf = a.buf;
    l.wbuf = a.wbuf;
    l.rec = rec;
    l.counts = counts;
    l.init = a.init;
    l.flags = a.flags;
    l.crc_out = a.crc_out;
    l.bad_bits = a.bad_bits;
    l.n_bad = a.n_bad;
    l.slice = a.slice;
    l.shift32 = a.shift32;
    l.slot_cap = a.slot_cap;
    l.seg_first_bad = a.seg_first_bad;
    l.seg_first = a.seg_first;
    l.dense_crc = a.dense_crc;
    l.dense_bad = a.dense_bad;
    l.frame_cap = a.frame_cap;
    // 4 lanes per frame for classes 1..12, 8 for 13..24 (lane tables: Q = 2, 4, 8, 16 at 4096 words each)
    l.lanetab = ctx->d_lane16 + (size_t)1 * 4096;
    l.zwin = ctx->d_shift + (size_t)8 * 1024;
    l.cls_lo = 1;
    l.cls_hi = kQ4Chunks;
    RH_HIP(launch_lanes<4>(l, a.n, cus, stream));
    l.lanetab = ctx->d_lane16 + (size_t)2 * 4096;
    l.zwin = ctx->d_shift + (size_t)9 * 1024;
    l.cls_lo = kQ4Chunks + 1;
    l.cls_hi = kLaneChunks;
    RH_HIP(launch_lanes<8>(l, a.n, cus, stream));
    a.counts = counts;
    a.widx = widx;
    constexpr uint64_t kBL = kBatchOf(true);
    const uint64_t wgrid = (a.n + kBL - 1) / kBL < cus ? (a.n + kBL - 1) / kBL : cus;
    hipLaunchKernelGGL(crc_frames_kernel<true>, dim3((uint32_t)wgrid), dim3(kCrcThreads), kCrcLdsOf(true), stream, a);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

}  // namespace

int rh_crc_upload_tables(rh_ctx* ctx) {
    rh::CrcTables t;
    rh::build_crc_slice_tables(&t);
    RH_HIP(hipMalloc(&ctx->d_slice, sizeof(t.slice)));
    RH_HIP(hipMemcpy(ctx->d_slice, t.slice, sizeof(t.slice), hipMemcpyHostToDevice));
    // zero-advance maps for every power of two 2^0 .. 2^40 bytes
    constexpr int kPow = 41;
    std::vector<uint32_t> sh((size_t)kPow * 1024);
    for (int m = 0; m < kPow; ++m)
        rh::build_crc_shift_table(1ull << m, reinterpret_cast<uint32_t(*)[256]>(sh.data() + (size_t)m * 1024));
    RH_HIP(hipMalloc(&ctx->d_shift, sh.size() * 4));
    RH_HIP(hipMemcpy(ctx->d_shift, sh.data(), sh.size() * 4, hipMemcpyHostToDevice));
    // lane-distance tables for Q = 2, 4, 8, 16, 32 lanes per window (4096 words each)
    std::vector<uint32_t> lt;
    for (int q = 2; q <= 32; q *= 2) {
        const std::vector<uint32_t> t = rh::build_crc_lane_tables(q, 64);
        lt.insert(lt.end(), t.begin(), t.end());
    }
    RH_HIP(hipMalloc(&ctx->d_lane16, lt.size() * 4));
    RH_HIP(hipMemcpy(ctx->d_lane16, lt.data(), lt.size() * 4, hipMemcpyHostToDevice));
    // packed kernel: inverse lane maps and reset()'s init term per span length
    const std::vector<uint32_t> inv = rh::build_crc_inverse_lane_tables();
    RH_HIP(hipMalloc(&ctx->d_inv32, inv.size() * 4));
    RH_HIP(hipMemcpy(ctx->d_inv32, inv.data(), inv.size() * 4, hipMemcpyHostToDevice));
    const std::vector<uint32_t> iff = rh::build_crc_init_terms(0xFFFFFFFFu);
    RH_HIP(hipMalloc(&ctx->d_initff, iff.size() * 4));
    RH_HIP(hipMemcpy(ctx->d_initff, iff.data(), iff.size() * 4, hipMemcpyHostToDevice));
    ctx->h_initff = iff;
    uint32_t s8[8][256];
    for (int k = 0; k < 8; ++k)
        for (int b = 0; b < 256; ++b)
            s8[k][b] = k < 4 ? t.slice[k][b] : (s8[k - 1][b] >> 8) ^ t.slice[0][s8[k - 1][b] & 0xffu];
    RH_HIP(hipMalloc(&ctx->d_slice8, sizeof(s8)));
    RH_HIP(hipMemcpy(ctx->d_slice8, s8, sizeof(s8), hipMemcpyHostToDevice));
    return RH_OK;
}

// ---- small flush batches: one lane per frame ----------------------------------------------------
// The write side's batches (rh_crc32c_stamp_host) are a few to a few thousand short frames, where the
// window and packed kernels' fixed costs (128-156 KiB of LDS tables staged per workgroup, a second
// launch) dominate.  Here a lane folds its own frame with PJC's own slicing-by-8 (PJC:54-91: eight
// table lookups per 8-byte word, T[k] = the register after a byte and k zero bytes), the 8 KiB of
// tables built in LDS from the context's four slicing-by-4 tables.  Latency-bound per lane (one
// dependent table round per 8 bytes), parallel over frames.  Frames must be well formed (the caller
// checks): [off, off + len) inside the buffer and len >= 4 under STAMP / VERIFY.  Only the CRCs are
// written (crc_out, required): under STAMP the caller writes the trailers from them (the host copy is
// the one that goes to the file), so the device image is never written.
__global__ __launch_bounds__(64) void crc_serial_kernel(const uint8_t* __restrict__ buf,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len, uint64_t n,
                                                         uint32_t init, uint32_t flags, const uint32_t* __restrict__ slice4,
                                                         uint32_t* crc_out) {
    __shared__ uint32_t T[8][256];
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[i >> 8][i & 255] = slice4[i];
    __syncthreads();
    for (int k = 4; k < 8; ++k) {   // T[k][b] = T[k-1][b] advanced over one more zero byte
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
            const uint32_t x = T[k - 1][i];
            T[k][i] = (x >> 8) ^ T[0][x & 0xffu];
        }
        __syncthreads();
    }
    const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    const uint8_t* p = buf + off[f];
    const uint32_t span = (flags & (RH_CRC_STAMP | RH_CRC_VERIFY)) ? len[f] - 4 : len[f];
    const uint8_t* e = p + span;
    uint32_t c = init;
    auto step8 = [&](uint32_t lo, uint32_t hi) {   // one PJC slicing-by-8 round over 8 bytes
        lo ^= c;
        c = T[7][lo & 0xffu] ^ T[6][(lo >> 8) & 0xffu] ^ T[5][(lo >> 16) & 0xffu] ^ T[4][lo >> 24] ^
            T[3][hi & 0xffu] ^ T[2][(hi >> 8) & 0xffu] ^ T[1][(hi >> 16) & 0xffu] ^ T[0][hi >> 24];
    };
    while (p < e && (reinterpret_cast<uintptr_t>(p) & 15)) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xffu];
    // 128 bytes per round, the next round's eight 16-byte loads issued before this round's fold:
    // the lane's memory latency hides behind its LDS chain (two buffers with static roles)
    typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
    v4u32 qa[8], qb[8];
    auto load128 = [&](v4u32 (&q)[8], const uint8_t* src) {
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = reinterpret_cast<const v4u32*>(src)[k];
    };
    auto fold128 = [&](const v4u32 (&q)[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            step8(q[k].x, q[k].y);
            step8(q[k].z, q[k].w);
        }
    };
    if (p + 128 <= e) load128(qa, p);
    while (p + 128 <= e) {
        if (p + 256 <= e) load128(qb, p + 128);
        fold128(qa);
        p += 128;
        if (p + 128 > e) break;
        if (p + 256 <= e) load128(qa, p + 128);
        fold128(qb);
        p += 128;
    }
    for (; p + 8 <= e; p += 8) {
        const uint64_t w = *reinterpret_cast<const uint64_t*>(p);
        step8((uint32_t)w, (uint32_t)(w >> 32));
    }
    while (p < e) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xffu];
    crc_out[f] = ~c;   // getValue()
}

int rh_crc_serial_launch(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream) {
    if (f->n == 0) return RH_OK;
    if (!f->crc_out) return rh::fail(RH_E_INVAL, "crc serial launch: crc_out required");
    // one wave per workgroup: the frames spread over as many CUs as there are waves of them
    hipLaunchKernelGGL(crc_serial_kernel, dim3((uint32_t)((f->n + 63) / 64)), dim3(64), 0, stream, f->buf,
                       f->frame_off, f->frame_len, f->n, f->init_state, flags, ctx->d_slice, f->crc_out);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_crc_launch_impl(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream, bool window_only) {
    if (!f) return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: frames == NULL");
    if ((flags & ~(RH_CRC_VERIFY | RH_CRC_STAMP)) || flags == (RH_CRC_VERIFY | RH_CRC_STAMP))
        return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: flags must be 0, VERIFY or STAMP");
    if (f->n == 0) return RH_OK;
    if (!f->buf || !f->frame_off || !f->frame_len)
        return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: buf, frame_off, frame_len required");
    if (f->buf_len > (uint64_t)INT64_MAX) return rh::fail(RH_E_RANGE, "rh_crc32c_frames_launch: buf_len too large");
    FrameArgs a{};
    a.buf = f->buf;
    a.wbuf = f->buf;
    a.buf_len = (int64_t)f->buf_len;
    a.off = f->frame_off;
    a.len = f->frame_len;
    a.n = f->n;
    a.init = f->init_state;
    a.flags = flags;
    a.crc_out = f->crc_out;
    a.bad_bits = f->bad_bits;
    a.n_bad = f->n_bad;
    return launch_frames(ctx, a, stream, nullptr, SlotPlan{}, window_only);
}

// The read path's CRC pass (rh_segments_read_launch): the kernel over the slotted frame table the
// framing walk left in segs->scratch_off/len, VERIFY, CRCs into crc->scratch_crc (slot-indexed),
// mismatches counted in crc->n_bad and the first bad slot of each segment atomically lowered in
// crc->seg_ok (pre-set to 0xFFFFFFFF by the caller).
int rh_crc_verify_slots(rh_ctx* ctx, const rh_segments* g, const rh_segments_crc* c, hipStream_t stream,
                        bool* dense_written) {
    FrameArgs a{};
    a.buf = g->buf;
    a.wbuf = nullptr;
    a.buf_len = (int64_t)g->buf_len;
    a.off = g->scratch_off;
    a.len = g->scratch_len;
    a.n = g->n_seg * (uint64_t)g->frames_per_seg_cap;
    a.init = 0xFFFFFFFFu;
    a.flags = RH_CRC_VERIFY;
    a.crc_out = c->scratch_crc;
    a.bad_bits = nullptr;
    a.n_bad = c->n_bad;
    a.slot_nframes = g->seg_nframes;
    a.slot_cap = g->frames_per_seg_cap;
    a.seg_first_bad = c->seg_ok;
    if (c->crc_out || c->bad_bits) {  // dense per-frame outputs straight from the CRC pass
        a.seg_first = g->seg_first;
        a.dense_crc = c->crc_out;
        a.dense_bad = c->bad_bits;
        a.frame_cap = g->frame_cap;
    }
    SlotPlan sp;
    sp.seg_first = g->seg_first;
    sp.total = g->total_frames;
    sp.n_seg = g->n_seg;
    return launch_frames(ctx, a, stream, dense_written, sp);
}

// ---- small flush batches from a registered buffer: zero-copy, one launch ---------------------------
// (rh_internal.h, StampArgs.)  Every byte a workgroup needs -- its span across PCIe, its frame
// records across PCIe, the slicing-by-8 table and the shift maps its frames need from HBM -- lands
// in LDS by LDS-DMA (16 B per lane, no registers), all issued before the first barrier: one PCIe
// round trip.  Thread t owns a run of frames for the window-count scan (wave scans + the wave
// totals scanned by wave 0); windows are then dealt round robin: window w's frame by binary search
// of the scan, j = its rank from the payload's end.  A window: 17 aligned LDS words funnel-shifted
// to its byte position, the leading bytes outside the frame zeroed (a zero register absorbs
// leading zeros), eight slicing-by-8 rounds (PJC:54-91) from a zero register, then advanced over
// the 64 j bytes after it (j's set bits: the maps over 64 * 2^b zero bytes) and XOR-ed into its
// frame's accumulator: a frame's register is A^len(init) ^ XOR of its windows' terms (the CRC is
// affine in the register and linear in the bytes).
namespace {
constexpr uint32_t kStampWaves = kStampThreads / 64;
constexpr uint32_t kStampFpt = kStampMaxFrames / kStampThreads;   // frames per thread in the scan
constexpr uint32_t kStampLdsT = 8 * 1024 + kStampShifts * 4096;  // tables
constexpr uint32_t kStampLdsF = kStampMaxFrames * 16;            // frame records
constexpr uint32_t kStampLds = kStampLdsT + kStampLdsF + 16 * (kStampWaves + 1) + kStampFront + kStampSpan + 16;
static_assert(kStampLds <= 160 * 1024, "LDS budget");
static_assert(kStampMaxFrames % kStampThreads == 0, "frames per thread");

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// pieces [0, n) of 16 B from global `src` to LDS `dst` (16-B aligned both), the workgroup's waves
// each taking runs of 64 pieces (one LDS-DMA instruction: wave-uniform LDS base + lane * 16)
__device__ __forceinline__ void dma16(const uint8_t* src, uint8_t* dst, uint32_t n, uint32_t wave, uint32_t lane) {
    for (uint32_t p0 = 64u * wave; p0 < n; p0 += 64u * kStampWaves) {
        const uint32_t i = p0 + lane;
        if (i < n)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 16ull * i), (lds_void_t*)(dst + 16u * i), 16, 0, 0);
    }
}

__global__ __launch_bounds__(kStampThreads) void crc_stamp_mapped_kernel(StampArgs arg) {
    (void)arg;
    const StampArgs& A = rh::kernarg_struct<StampArgs>();   // uniform index: scalar loads
    extern __shared__ __attribute__((aligned(16))) uint8_t sb[];
    const uint32_t* T = reinterpret_cast<const uint32_t*>(sb);   // [8][256]
    const uint32_t* Z = T + 8 * 256;                            // [n_shift][4][256]
    uint4* fr = reinterpret_cast<uint4*>(sb + kStampLdsT);      // [frame_n]: pos, payload, acc, prefix
    uint32_t* wsum = reinterpret_cast<uint32_t*>(sb + kStampLdsT + kStampLdsF);   // [kStampWaves + 1]
    uint8_t* img = sb + kStampLdsT + kStampLdsF + 16 * (kStampWaves + 1);         // kStampFront + span + 16
    const StampGroup& g = A.g[blockIdx.x];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t nq = (g.bytes_n >> 12) / 16, F = g.bytes_n & 4095u;
    dma16(reinterpret_cast<const uint8_t*>(g.src), img + kStampFront, nq, wave, lane);
    dma16(reinterpret_cast<const uint8_t*>(A.frames + g.frame_first), reinterpret_cast<uint8_t*>(fr), F, wave, lane);
    dma16(reinterpret_cast<const uint8_t*>(A.slice8), sb, 512, wave, lane);
    dma16(reinterpret_cast<const uint8_t*>(A.shift64), sb + 8 * 1024, 256 * A.n_shift, wave, lane);
    __syncthreads();   // (waits for the LDS-DMA)
    // windows per frame, scanned: thread t's frames [kStampFpt t, + kStampFpt)
    uint32_t own = 0;
#pragma unroll
    for (uint32_t k = 0; k < kStampFpt; ++k) {
        const uint32_t f = kStampFpt * t + k;
        if (f < F) own += (fr[f].y + 63u) / 64u;
    }
    uint32_t incl = own;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, d);
        if ((int)lane >= d) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (wave == 0) {   // exclusive scan of the wave totals (lanes < kStampWaves)
        const uint32_t v = lane < kStampWaves ? wsum[lane] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < (int)kStampWaves; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d);
            if ((int)lane >= d) x += y;
        }
        if (lane < kStampWaves) wsum[lane] = x - v;
        if (lane == kStampWaves - 1) wsum[kStampWaves] = x;
    }
    __syncthreads();
    uint32_t run = wsum[wave] + incl - own;
#pragma unroll
    for (uint32_t k = 0; k < kStampFpt; ++k) {
        const uint32_t f = kStampFpt * t + k;
        if (f < F) {
            fr[f].w = run;
            run += (fr[f].y + 63u) / 64u;
        }
    }
    const uint32_t n_win = wsum[kStampWaves];
    __syncthreads();
    for (uint32_t wi = t; wi < n_win; wi += kStampThreads) {
        uint32_t lo = 0, hi = F;   // the frame f with prefix[f] <= wi < prefix[f] + its windows
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (fr[mid].w <= wi) lo = mid; else hi = mid;
        }
        const uint32_t f = lo, j = wi - fr[f].w, fp = fr[f].x;
        const int32_t P = (int32_t)(fp + fr[f].y) - 64 * (int32_t)(j + 1);   // the window's first byte
        const uint32_t pos = (uint32_t)P, lead = P < (int32_t)fp ? fp - (uint32_t)P : 0u;
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(img + (pos & ~3u));
        uint32_t W[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) W[i] = wp[i];
        const uint32_t sh = pos & 3u;
        uint32_t D[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t x = __builtin_amdgcn_alignbyte(W[i + 1], W[i], sh);
            const int32_t z = (int32_t)lead - 4 * i;   // bytes of this word before the frame
            D[i] = z >= 4 ? 0u : (z <= 0 ? x : x & (~0u << (8 * z)));
        }
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t lo8 = D[2 * k] ^ c, hi8 = D[2 * k + 1];
            c = xor3(xor3(T[7 * 256 + (lo8 & 0xffu)], T[6 * 256 + ((lo8 >> 8) & 0xffu)], T[5 * 256 + ((lo8 >> 16) & 0xffu)]),
                     xor3(T[4 * 256 + (lo8 >> 24)], T[3 * 256 + (hi8 & 0xffu)], T[2 * 256 + ((hi8 >> 8) & 0xffu)]),
                     T[256 + ((hi8 >> 16) & 0xffu)] ^ T[hi8 >> 24]);
        }
#pragma unroll
        for (uint32_t b = 0; b < kStampShifts; ++b)
            if ((j >> b) & 1u) c = zshift(Z + b * 1024, c);
        atomicXor(&fr[f].z, c);
    }
    __syncthreads();
    for (uint32_t f = t; f < F; f += kStampThreads) A.crc_out[g.frame_first + f] = ~fr[f].z;   // getValue()
    __threadfence_system();   // this wave's CRC stores performed (system scope) before the flag
    __syncthreads();
    if (t == 0) __hip_atomic_store(A.done + blockIdx.x, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

int rh_crc_stamp_mapped_launch(const StampArgs& a, uint32_t n_groups, hipStream_t stream) {
    if (n_groups == 0 || n_groups > kStampMaxGroups) return rh::fail(RH_E_INVAL, "crc stamp (mapped): group count");
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_stamp_mapped_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kStampLds);
    RH_HIP(attr);
    hipLaunchKernelGGL(crc_stamp_mapped_kernel, dim3(n_groups), dim3(kStampThreads), kStampLds, stream, a);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
