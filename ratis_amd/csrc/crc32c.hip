// CRC32C (PureJavaCrc32C) over SegmentedRaftLog frames, for gfx950 (MI355X).
//
// Reference semantics:
//   PureJavaCrc32C.update/getValue/reset    PureJavaCrc32C.java:43-152 (tables :158-688)
//   frame CRC = CRC32C(varint || proto), big-endian trailer
//                                            SegmentedRaftLogOutputStream.java:86-110
//   verification                             SegmentedRaftLogReader.java:327-336
//
// Structure.  A frame's CRC-covered span is cut into end-anchored windows of W = Q*S bytes;
// each window is handled by Q consecutive lanes of a wave, lane i taking the contiguous chunk
// [end - (Q-i)*S, end - (Q-i-1)*S) of the window.  Every lane folds its chunk into a CRC
// register that starts at zero (slicing-by-4, 4 byte-tables), and the Q partial registers are
// combined with a log2(Q)-level tree: left' = Z_d(left) ^ right, where Z_d advances a register
// over d zero bytes (a 4x256 byte-table per power-of-two d).  CRC linearity makes this exact:
// bytes before the frame start contribute nothing to a zero register, and the initial state
// I (0xFFFFFFFF after reset()) is injected by XOR-ing it into the first 4 message bytes.
//
// LDS.  The 4 slicing tables are replicated 32 times and interleaved so that lane l always
// reads bank (l & 31): the data-dependent lookups are bank-conflict free (a random byte index
// into a shared table would cost ~3.4 LDS cycles per 32-lane group instead of 1).  128 KiB of
// tables + 4 KiB per tree level => one 1024-thread workgroup per CU, persistent over frames.
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

// Lane-distance tables for the v4 kernel: lane g of a Q-lane window advances its chunk CRC over
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
    const uint32_t* shift;   // [levels][4][256] global: level j advances S*2^j, last = W
    const uint32_t* shift32; // [4][256]: advance over 32 zero bytes (v3/v4, ILP = 2)
    const uint32_t* lanetab; // v4: lane-distance nibble tables (build_crc_lane_tables)
    const uint32_t* zwin;    // v4: [4][256] advance over one window (Q*64 bytes)
    // v8 slot mode (the read path): the frame table is rh_segments' slotted scratch table, entry
    // f = segment f / slot_cap, slot f % slot_cap, valid below min(slot_nframes[seg], slot_cap);
    // a mismatch also lowers seg_first_bad[seg] to the slot index (atomicMin)
    const uint32_t* slot_nframes;
    uint32_t slot_cap;
    uint32_t* seg_first_bad;
};

template <bool REPL>
__device__ __forceinline__ uint32_t slice_lookup(const uint32_t* lds, int k, uint32_t e, uint32_t c) {
    if (REPL) return lds[(k << 13) | (e << 5) | c];
    return lds[(k << 8) | e];
}

template <bool REPL>
__device__ __forceinline__ uint32_t fold_word(const uint32_t* lds, uint32_t r, uint32_t w, uint32_t c) {
    const uint32_t x = r ^ w;
    return slice_lookup<REPL>(lds, 3, x & 0xffu, c) ^ slice_lookup<REPL>(lds, 2, (x >> 8) & 0xffu, c) ^
           slice_lookup<REPL>(lds, 1, (x >> 16) & 0xffu, c) ^ slice_lookup<REPL>(lds, 0, x >> 24, c);
}

template <bool REPL>
__device__ __forceinline__ uint32_t fold_byte(const uint32_t* lds, uint32_t r, uint32_t b, uint32_t c) {
    return (r >> 8) ^ slice_lookup<REPL>(lds, 0, (r ^ b) & 0xffu, c);
}

__device__ __forceinline__ uint32_t zshift(const uint32_t* tab, uint32_t r) {
    return tab[r & 0xffu] ^ tab[256 + ((r >> 8) & 0xffu)] ^ tab[512 + ((r >> 16) & 0xffu)] ^ tab[768 + (r >> 24)];
}

// One little-endian dword at byte offset p (4-aligned) of a buffer of `lim` bytes; bytes at or
// past `lim` read as zero and are never touched.
__device__ __forceinline__ uint32_t load_dword_clamped(const uint8_t* buf, int64_t p, int64_t lim) {
    if (p + 4 <= lim) return *reinterpret_cast<const uint32_t*>(buf + p);
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i)
        if (p + i < lim) v |= (uint32_t)buf[p + i] << (8 * i);
    return v;
}

// Same as load_dword_clamped for the rare dword that crosses the buffer end (out of line).
__device__ __noinline__ uint32_t load_dword_clamped_slow(const uint8_t* buf, int64_t p, int64_t lim) {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i)
        if (p + i >= 0 && p + i < lim) v |= (uint32_t)buf[p + i] << (8 * i);
    return v;
}

// 4-byte-aligned 16-byte vector for non-temporal loads (the builtin needs a vector type).
typedef uint32_t u32x4v __attribute__((ext_vector_type(4), aligned(4)));
struct __attribute__((aligned(4))) u32x4a {
    uint32_t x, y, z, w;
};

// Dwords [16*blk, 16*blk+16) after the 4-aligned byte offset b0; dwords >= need read as 0.
__device__ __forceinline__ void load_block(uint32_t (&d)[16], const uint8_t* buf, int64_t b0, int blk,
                                           int need, int64_t lim) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int idx = 16 * blk + 4 * q;
        const int64_t p = b0 + 4 * (int64_t)idx;
        if (idx < need && p + 16 <= lim) {
            const u32x4a v = *reinterpret_cast<const u32x4a*>(buf + p);
            d[4 * q] = v.x;
            d[4 * q + 1] = v.y;
            d[4 * q + 2] = v.z;
            d[4 * q + 3] = v.w;
        } else if (idx < need) {
#pragma unroll
            for (int i = 0; i < 4; ++i) d[4 * q + i] = load_dword_clamped(buf, p + 4 * i, lim);
        } else {
            d[4 * q] = d[4 * q + 1] = d[4 * q + 2] = d[4 * q + 3] = 0;
        }
    }
}

// Q lanes per frame window, S bytes per lane (multiple of 16), REPL = replicated tables.
template <int Q, int S, bool REPL>
__global__ __launch_bounds__(1024) void crc_frames_kernel(FrameArgs a) {
    constexpr int W = Q * S;
    constexpr int LOGQ = __builtin_ctz(Q);
    constexpr int NB = S / 64;                    // 64-byte blocks per full chunk
    static_assert(S % 64 == 0, "chunk must be a multiple of 64 bytes");
    constexpr int kSliceWords = REPL ? 4 * 256 * 32 : 4 * 256;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* lslice = lds;
    uint32_t* lshift = lds + kSliceWords;  // [LOGQ + 1][1024]

    // ---- stage tables into LDS ----
    for (int i = threadIdx.x; i < kSliceWords; i += blockDim.x) {
        if (REPL) {
            const int k = i >> 13, e = (i >> 5) & 255;
            lslice[i] = a.slice[(k << 8) | e];
        } else {
            lslice[i] = a.slice[i];
        }
    }
    for (int i = threadIdx.x; i < (LOGQ + 1) * 1024; i += blockDim.x) lshift[i] = a.shift[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    const int gl = lane & (Q - 1);            // position inside the window group
    const int gid = lane / Q;                 // group inside the wave
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    for (uint64_t f0 = wave * kGroupsPerWave; f0 < a.n; f0 += nwaves * kGroupsPerWave) {
        const uint64_t f = f0 + gid;
        const bool active = f < a.n;
        uint64_t o = 0;
        int64_t Lc = 0;
        bool malformed = false;  // frame outside the buffer, or shorter than its trailer
        if (active) {
            o = a.off[f];
            const int64_t L = (int64_t)a.len[f];
            malformed = o > (uint64_t)a.buf_len || L > a.buf_len - (int64_t)o || (trailer && L < 4);
            Lc = malformed ? 0 : L - (trailer ? 4 : 0);
        }
        const int64_t E = (int64_t)o + Lc;              // end of the CRC-covered span
        const int64_t nw = (Lc + W - 1) / W;            // windows of this frame (0 if empty)
        const uint32_t sh = (uint32_t)(E & 3);          // byte misalignment of every word

        // Wave-uniform trip count: the largest window count among the wave's groups.
        int64_t nw_max = nw;
        if (kGroupsPerWave > 1) {
#pragma unroll
            for (int d = Q; d < 64; d <<= 1) {
                const int64_t other = __shfl_xor(nw_max, d);
                nw_max = other > nw_max ? other : nw_max;
            }
        }

        uint32_t R = 0;  // running register of the frame (meaningful in the group leader)
        for (int64_t wi = 0; wi < nw_max; ++wi) {
            const bool win_active = wi < nw;
            // chunk [cs, be) of this lane
            const int64_t be = E - (nw - 1 - wi) * (int64_t)W - (int64_t)(Q - 1 - gl) * S;
            const int64_t cs = be - S;
            const int64_t bs = cs > (int64_t)o ? cs : (int64_t)o;  // bytes before o are zero
            int64_t cnt = be - bs;
            if (!win_active || cnt < 0) cnt = 0;
            const int h = (int)(cnt & 3);                          // head bytes (straddling lane)
            const int nwords = (int)(cnt >> 2);
            const int64_t A = bs + h;                              // first word's address
            uint32_t r = 0;
            // The initial state I is XOR-ed into message positions 0..3 (byte k of I at position
            // k).  Those positions can be split over two lanes when the first lane holds < 4
            // bytes, so the injection is by position: p0 = message position of this chunk.
            const int64_t p0 = bs - (int64_t)o;

            // head bytes (at most 3, only the lane that holds the frame start)
            if (h) {
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    if (i < h) {
                        uint32_t b = a.buf[bs + i];
                        if (p0 + i < 4) b ^= (a.init >> (8 * (p0 + i))) & 0xffu;
                        r = fold_byte<REPL>(lslice, r, b, c);
                    }
            }
            // words: 64-byte blocks loaded as 16-byte pieces from the 4-aligned base b0,
            // realigned by `sh`; block blk+1 is in flight while block blk is folded.  Loads
            // never touch [buf_len, ...): pieces crossing it are read per dword / per byte.
            if (nwords > 0) {
                const int64_t b0 = A - sh;                 // 4-aligned
                const int need = nwords + (sh ? 1 : 0);    // dwords needed from b0
                uint32_t cur[16], nxt[16];
                load_block(cur, a.buf, b0, 0, need, a.buf_len);
#pragma unroll
                for (int blk = 0; blk < NB; ++blk) {
                    if (blk + 1 < NB) {
                        load_block(nxt, a.buf, b0, blk + 1, need, a.buf_len);
                    } else {
                        nxt[0] = (16 * NB < need) ? load_dword_clamped(a.buf, b0 + 64 * NB, a.buf_len) : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        if (16 * blk + j < nwords) {
                            const uint32_t hi = (j < 15) ? cur[j + 1] : nxt[0];
                            uint32_t w = sh ? __builtin_amdgcn_alignbyte(hi, cur[j], sh) : cur[j];
                            if (blk == 0 && j == 0 && p0 + h < 4) w ^= a.init >> (8 * (p0 + h));
                            r = fold_word<REPL>(lslice, r, w, c);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 16; ++j) cur[j] = nxt[j];
                }
            }
            // init bytes that fall beyond a sub-4-byte message are handled after the loop
            // ---- tree combine across the Q lanes of the window ----
#pragma unroll
            for (int j = 0; j < LOGQ; ++j) {
                const uint32_t t = zshift(lshift + j * 1024, r);
                const uint32_t p = __shfl_down(r, 1 << j);
                r = t ^ p;
            }
            if (win_active) R = zshift(lshift + LOGQ * 1024, R) ^ r;
        }

        if (active && gl == 0) {
            uint32_t state = R;
            if (Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * Lc));
            const uint32_t value = ~state;  // getValue()
            if (a.crc_out) a.crc_out[f] = malformed ? 0u : value;
            if (malformed) {
                if (a.bad_bits) atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                if (a.n_bad) atomicAdd(a.n_bad, 1ull);
            } else if (a.flags & RH_CRC_STAMP) {
                a.wbuf[E + 0] = (uint8_t)(value >> 24);
                a.wbuf[E + 1] = (uint8_t)(value >> 16);
                a.wbuf[E + 2] = (uint8_t)(value >> 8);
                a.wbuf[E + 3] = (uint8_t)value;
            } else if (a.flags & RH_CRC_VERIFY) {
                const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                        ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                if (stored != value) {
                    if (a.bad_bits) atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                             1ull << (f & 63));
                    if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                }
            }
        }
    }
}

// ---- v2: flattened (frame, window) cursor per lane group, one window of data in flight ------
// Each Q-lane group walks its frames window by window; the chunk of the NEXT window (possibly
// of the next frame) is loaded before the current one is folded, so HBM latency overlaps the
// table work.  Chunk = 64 bytes per lane (S = 64): 17 dwords in registers per window.
struct Cursor {
    uint64_t f;        // frame index (>= n: exhausted)
    int64_t o, Lc, E;  // frame start, CRC-covered length, end
    int64_t nw, wi;    // windows of the frame, current window
    uint32_t sh;       // E & 3
    bool malformed;
};

__device__ __forceinline__ void cursor_frame(const FrameArgs& a, bool trailer, int64_t W, Cursor& c) {
    c.wi = 0;
    c.malformed = false;
    c.o = c.Lc = c.E = c.nw = 0;
    c.sh = 0;
    if (c.f >= a.n) return;
    const uint64_t o = a.off[c.f];
    const int64_t L = (int64_t)a.len[c.f];
    c.malformed = o > (uint64_t)a.buf_len || L > a.buf_len - (int64_t)o || (trailer && L < 4);
    c.o = (int64_t)o;
    c.Lc = c.malformed ? 0 : L - (trailer ? 4 : 0);
    c.E = c.o + c.Lc;
    c.nw = (c.Lc + W - 1) / W;
    c.sh = (uint32_t)(c.E & 3);
}

// Chunk geometry of lane `gl` in window `wi` of the cursor's frame.
struct Chunk {
    int64_t bs, A, p0;
    int cnt, h, nwords;
};

template <int Q, int S>
__device__ __forceinline__ Chunk chunk_of(const Cursor& c, int gl) {
    constexpr int64_t W = (int64_t)Q * S;
    Chunk k;
    const int64_t be = c.E - (c.nw - 1 - c.wi) * W - (int64_t)(Q - 1 - gl) * S;
    const int64_t cs = be - S;
    k.bs = cs > c.o ? cs : c.o;
    int64_t cnt = be - k.bs;
    if (c.wi >= c.nw || cnt < 0) cnt = 0;
    k.cnt = (int)cnt;
    k.h = k.cnt & 3;
    k.nwords = k.cnt >> 2;
    k.A = k.bs + k.h;
    k.p0 = k.bs - c.o;
    return k;
}

template <int Q, int S, bool REPL>
__global__ __launch_bounds__(REPL ? 1024 : 256) void crc_frames_kernel2(FrameArgs a) {
    static_assert(S == 64, "v2 keeps one 64-byte chunk per lane in registers");
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int LOGQ = __builtin_ctz(Q);
    constexpr int kSliceWords = REPL ? 4 * 256 * 32 : 4 * 256;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* lslice = lds;
    uint32_t* lshift = lds + kSliceWords;
    for (int i = threadIdx.x; i < kSliceWords; i += blockDim.x) {
        if (REPL) {
            const int k = i >> 13, e = (i >> 5) & 255;
            lslice[i] = a.slice[(k << 8) | e];
        } else {
            lslice[i] = a.slice[i];
        }
    }
    for (int i = threadIdx.x; i < (LOGQ + 1) * 1024; i += blockDim.x) lshift[i] = a.shift[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    const int gl = lane & (Q - 1);
    const int gid = lane / Q;
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t fstride = nwaves * kGroupsPerWave;
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    Cursor cur;
    cur.f = wave * kGroupsPerWave + gid;
    cursor_frame(a, trailer, W, cur);
    // skip frames with no window (empty / malformed) after finalising them
    uint32_t d[17];
    auto load_chunk = [&](const Cursor& cc, uint32_t (&dd)[17]) {
        const Chunk k = chunk_of<Q, S>(cc, gl);
        const int need = k.nwords + (cc.sh ? 1 : 0);
        const int64_t b0 = k.A - cc.sh;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int idx = 4 * q;
            const int64_t p = b0 + 16 * q;
            if (idx < need && p + 16 <= a.buf_len) {
                const u32x4a v = *reinterpret_cast<const u32x4a*>(a.buf + p);
                dd[idx] = v.x;
                dd[idx + 1] = v.y;
                dd[idx + 2] = v.z;
                dd[idx + 3] = v.w;
            } else if (idx < need) {
#pragma unroll
                for (int i = 0; i < 4; ++i) dd[idx + i] = load_dword_clamped(a.buf, p + 4 * i, a.buf_len);
            } else {
                dd[idx] = dd[idx + 1] = dd[idx + 2] = dd[idx + 3] = 0;
            }
        }
        dd[16] = (16 < need) ? load_dword_clamped(a.buf, b0 + 64, a.buf_len) : 0u;
    };
    if (cur.f < a.n) load_chunk(cur, d);
    uint32_t R = 0;
    while (__any(cur.f < a.n)) {
        // next cursor + its data, issued before folding the current window
        Cursor nxt = cur;
        if (cur.f < a.n) {
            if (cur.wi + 1 < cur.nw) {
                nxt.wi = cur.wi + 1;
            } else {
                nxt.f = cur.f + fstride;
                cursor_frame(a, trailer, W, nxt);
            }
        }
        uint32_t dn[17];
        if (nxt.f < a.n) load_chunk(nxt, dn);

        // fold the current window's chunk
        uint32_t r = 0;
        if (cur.f < a.n && cur.wi < cur.nw) {
            const Chunk k = chunk_of<Q, S>(cur, gl);
            if (k.h) {
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    if (i < k.h) {
                        uint32_t b = a.buf[k.bs + i];
                        if (k.p0 + i < 4) b ^= (a.init >> (8 * (k.p0 + i))) & 0xffu;
                        r = fold_byte<REPL>(lslice, r, b, c);
                    }
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (j < k.nwords) {
                    uint32_t w = cur.sh ? __builtin_amdgcn_alignbyte(d[j + 1], d[j], cur.sh) : d[j];
                    if (j == 0 && k.p0 + k.h < 4) w ^= a.init >> (8 * (k.p0 + k.h));
                    r = fold_word<REPL>(lslice, r, w, c);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < LOGQ; ++j) {
            const uint32_t t = zshift(lshift + j * 1024, r);
            const uint32_t p = __shfl_down(r, 1 << j);
            r = t ^ p;
        }
        if (cur.f < a.n) {
            if (cur.wi < cur.nw) R = zshift(lshift + LOGQ * 1024, R) ^ r;
            if (cur.wi + 1 >= cur.nw) {  // frame complete: finalise in the group leader
                if (gl == 0) {
                    const uint64_t f = cur.f;
                    uint32_t state = R;
                    if (cur.Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * cur.Lc));
                    const uint32_t value = ~state;
                    const int64_t E = cur.E;
                    if (a.crc_out) a.crc_out[f] = cur.malformed ? 0u : value;
                    if (cur.malformed) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    } else if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                                ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                         1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        }
                    }
                }
                R = 0;
            }
        }
        cur = nxt;
#pragma unroll
        for (int j = 0; j < 17; ++j) d[j] = dn[j];
    }
}

// ---- v3: branch-free fold ----------------------------------------------------------------
// Every lane folds exactly 16 words (its end-anchored 64-byte chunk).  Bytes of the chunk that
// lie before the frame start are zeroed once after the load (a zero register absorbing leading
// zero bytes stays zero, so this equals folding only the real bytes), and the initial state is
// XOR-ed into the dwords that hold message positions 0..3.  Only the (at most one per window)
// lane whose chunk crosses the frame start, or whose loads would cross a buffer edge, takes
// the guarded load path.  ILP = 2 folds the two 32-byte halves as independent chains and joins
// them with one 32-byte zero-advance: the serial LDS-latency chain per window halves.
template <int Q, int ILP, bool REPL>
__global__ __launch_bounds__(REPL ? 1024 : 256) void crc_frames_kernel3(FrameArgs a) {
    constexpr int S = 64;
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int LOGQ = __builtin_ctz(Q);
    constexpr int kSliceWords = REPL ? 4 * 256 * 32 : 4 * 256;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* lslice = lds;
    uint32_t* lshift = lds + kSliceWords;          // [LOGQ + 1] levels, S*2^j then W
    uint32_t* lhalf = lshift + (LOGQ + 1) * 1024;  // 32-byte zero-advance (ILP = 2)
    for (int i = threadIdx.x; i < kSliceWords; i += blockDim.x) {
        if (REPL) {
            const int k = i >> 13, e = (i >> 5) & 255;
            lslice[i] = a.slice[(k << 8) | e];
        } else {
            lslice[i] = a.slice[i];
        }
    }
    for (int i = threadIdx.x; i < (LOGQ + 1) * 1024; i += blockDim.x) lshift[i] = a.shift[i];
    if (ILP == 2)
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) lhalf[i] = a.shift32[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    const int gl = lane & (Q - 1);
    const int gid = lane / Q;
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t fstride = nwaves * kGroupsPerWave;
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    // loads the 17 dwords of this lane's chunk in window `cc.wi`, pre-masked and init-injected
    auto load_chunk = [&](const Cursor& cc, uint32_t (&dd)[17]) {
        const int64_t be = cc.E - (cc.nw - 1 - cc.wi) * W - (int64_t)(Q - 1 - gl) * S;
        const int64_t cs = be - S;
        const int64_t b0 = cs - cc.sh;  // 4-aligned
        const bool fast = cs >= cc.o && b0 + 68 <= a.buf_len;
        if (fast) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4a v = *reinterpret_cast<const u32x4a*>(a.buf + b0 + 16 * q);
                dd[4 * q] = v.x;
                dd[4 * q + 1] = v.y;
                dd[4 * q + 2] = v.z;
                dd[4 * q + 3] = v.w;
            }
            dd[16] = cc.sh ? *reinterpret_cast<const uint32_t*>(a.buf + b0 + 64) : 0u;
        } else {
            // guarded path: only dwords overlapping [o, be) are read; none outside the buffer
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int64_t p = b0 + 4 * i;  // 4-aligned
                uint32_t v = 0;
                if (p + 4 > cc.o && p < be) {
                    if (p >= 0 && p + 4 <= a.buf_len)
                        v = *reinterpret_cast<const uint32_t*>(a.buf + p);
                    else
                        v = load_dword_clamped_slow(a.buf, p, a.buf_len);
                    const int64_t lead = cc.o - p;  // bytes of this dword before the frame start
                    if (lead > 0) v &= 0xFFFFFFFFu << (8 * (uint32_t)lead);
                }
                dd[i] = v;
            }
        }
        // initial state at message positions 0..3: dword i covers positions q0+4i .. q0+4i+3
        const int64_t q0l = b0 - cc.o;
        if (q0l < 4 && q0l > -72) {
            const int q0 = (int)q0l;
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int q = q0 + 4 * i;
                const uint32_t up = (q >= 0 && q < 4) ? (a.init >> (8 * q)) : 0u;
                const uint32_t dn = (q < 0 && q > -4) ? (a.init << (8 * -q)) : 0u;
                dd[i] ^= up | dn;
            }
        }
    };
    auto fold16 = [&](const uint32_t (&dd)[17], uint32_t sh) -> uint32_t {
        if (ILP == 2) {
            uint32_t ra = 0, rb = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t wa = __builtin_amdgcn_alignbyte(dd[j + 1], dd[j], sh);
                const uint32_t wb = __builtin_amdgcn_alignbyte(dd[j + 9], dd[j + 8], sh);
                ra = fold_word<REPL>(lslice, ra, wa, c);
                rb = fold_word<REPL>(lslice, rb, wb, c);
            }
            return zshift(lhalf, ra) ^ rb;
        } else {
            uint32_t r = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) r = fold_word<REPL>(lslice, r, __builtin_amdgcn_alignbyte(dd[j + 1], dd[j], sh), c);
            return r;
        }
    };

    Cursor cur;
    cur.f = wave * kGroupsPerWave + gid;
    cursor_frame(a, trailer, W, cur);
    uint32_t d[17];
    if (cur.f < a.n && cur.wi < cur.nw) load_chunk(cur, d);
    uint32_t R = 0;
    while (__any(cur.f < a.n)) {
        Cursor nxt = cur;
        if (cur.f < a.n) {
            if (cur.wi + 1 < cur.nw) {
                nxt.wi = cur.wi + 1;
            } else {
                nxt.f = cur.f + fstride;
                cursor_frame(a, trailer, W, nxt);
            }
        }
        uint32_t dn[17];
        if (nxt.f < a.n && nxt.wi < nxt.nw) load_chunk(nxt, dn);

        uint32_t r = 0;
        if (cur.f < a.n && cur.wi < cur.nw) r = fold16(d, cur.sh);
#pragma unroll
        for (int j = 0; j < LOGQ; ++j) {
            const uint32_t t = zshift(lshift + j * 1024, r);
            const uint32_t p = __shfl_down(r, 1 << j);
            r = t ^ p;
        }
        if (cur.f < a.n) {
            if (cur.wi < cur.nw) R = zshift(lshift + LOGQ * 1024, R) ^ r;
            if (cur.wi + 1 >= cur.nw) {
                if (gl == 0) {
                    const uint64_t f = cur.f;
                    uint32_t state = R;
                    if (cur.Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * cur.Lc));
                    const uint32_t value = ~state;
                    const int64_t E = cur.E;
                    if (a.crc_out) a.crc_out[f] = cur.malformed ? 0u : value;
                    if (cur.malformed) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    } else if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                                ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                         1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        }
                    }
                }
                R = 0;
            }
        }
        cur = nxt;
#pragma unroll
        for (int j = 0; j < 17; ++j) d[j] = dn[j];
    }
}

// ---- v4: per-lane zero-advance instead of a tree ------------------------------------------
// A window is Q lanes x 64 bytes.  Each lane folds its 16 words (slicing-by-4, replicated
// tables), advances the partial register over the 64*(Q-1-g) bytes that follow its chunk in the
// window with 8 conflict-free nibble lookups into lane-specific tables, and the group XOR-reduces
// (log2 Q shuffles).  Frame-start masking and initial-state injection run only on windows that
// contain a frame start (wave-uniform test); a frame's windows are chained by its leader lane
// with one window-length zero-advance.
template <int Q, int ILP, bool REPL>
__global__ __launch_bounds__(1024) void crc_frames_kernel4(FrameArgs a) {
    constexpr int S = 64;
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int kSliceWords = REPL ? 4 * 256 * 32 : 4 * 256;
    constexpr int kLaneWords = (Q > 32 ? Q / 32 : 1) * 8 * 16 * 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* lslice = lds;
    uint32_t* llane = lslice + kSliceWords;
    uint32_t* lzw = llane + kLaneWords;
    uint32_t* lhalf = lzw + 1024;
    for (int i = threadIdx.x; i < kSliceWords; i += blockDim.x) {
        if (REPL) {
            const int k = i >> 13, e = (i >> 5) & 255;
            lslice[i] = a.slice[(k << 8) | e];
        } else {
            lslice[i] = a.slice[i];
        }
    }
    for (int i = threadIdx.x; i < kLaneWords; i += blockDim.x) llane[i] = a.lanetab[i];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        lzw[i] = a.zwin[i];
        if (ILP == 2) lhalf[i] = a.shift32[i];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    const uint32_t lbase = (Q > 32 ? (uint32_t)(lane >> 5) * (8 * 16 * 32) : 0u) + c;
    const int gl = lane & (Q - 1);
    const int gid = lane / Q;
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t fstride = nwaves * kGroupsPerWave;
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    auto load_chunk = [&](const Cursor& cc, uint32_t (&dd)[17]) {
        const bool act = cc.f < a.n && cc.wi < cc.nw;
        const int64_t be = cc.E - (cc.nw - 1 - cc.wi) * W - (int64_t)(Q - 1 - gl) * S;
        const int64_t b0 = be - S - cc.sh;  // 4-aligned
        const bool safe = !act || (b0 >= 0 && b0 + 68 <= a.buf_len);
        if (__all(safe)) {
            if (act) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const u32x4a v = *reinterpret_cast<const u32x4a*>(a.buf + b0 + 16 * q);
                    dd[4 * q] = v.x;
                    dd[4 * q + 1] = v.y;
                    dd[4 * q + 2] = v.z;
                    dd[4 * q + 3] = v.w;
                }
                dd[16] = *reinterpret_cast<const uint32_t*>(a.buf + b0 + 64);
            } else {
#pragma unroll
                for (int i = 0; i < 17; ++i) dd[i] = 0;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int64_t p = b0 + 4 * i;
                uint32_t v = 0;
                if (act && p + 4 > cc.o && p < be) {
                    if (p >= 0 && p + 4 <= a.buf_len)
                        v = *reinterpret_cast<const uint32_t*>(a.buf + p);
                    else
                        v = load_dword_clamped_slow(a.buf, p, a.buf_len);
                }
                dd[i] = v;
            }
        }
    };

    Cursor cur;
    cur.f = wave * kGroupsPerWave + gid;
    cursor_frame(a, trailer, W, cur);
    uint32_t d[17];
    load_chunk(cur, d);
    uint32_t R = 0;
    while (__any(cur.f < a.n)) {
        Cursor nxt = cur;
        if (cur.f < a.n) {
            if (cur.wi + 1 < cur.nw) {
                nxt.wi = cur.wi + 1;
            } else {
                nxt.f = cur.f + fstride;
                cursor_frame(a, trailer, W, nxt);
            }
        }
        uint32_t dn[17];
        load_chunk(nxt, dn);

        const bool act = cur.f < a.n && cur.wi < cur.nw;
        // message position of dword 0 of this lane's chunk
        const int64_t q0l = cur.E - (cur.nw - 1 - cur.wi) * W - (int64_t)(Q - gl) * S - cur.sh - cur.o;
        const bool special = act && q0l < 4;
        if (__any(special)) {
            // zero bytes before the frame start; XOR the initial state into positions 0..3
            const int64_t qc = q0l < -80 ? -80 : (q0l > 4 ? 4 : q0l);
            const int q0 = (int)qc;
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int q = q0 + 4 * i;
                uint32_t v = act ? d[i] : 0u;
                v = (q <= -4) ? 0u : (q < 0 ? (v & (0xFFFFFFFFu << (8 * -q))) : v);
                const uint32_t up = (q >= 0 && q < 4) ? (a.init >> (8 * q)) : 0u;
                const uint32_t dn2 = (q < 0 && q > -4) ? (a.init << (8 * -q)) : 0u;
                d[i] = (act && special) ? (v ^ up ^ dn2) : d[i];
            }
        }
        // fold 16 words
        uint32_t r;
        const uint32_t sh = cur.sh;
        if (ILP == 2) {
            uint32_t ra = 0, rb = 0;
            if (__all(sh == 0 || !act)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    ra = fold_word<REPL>(lslice, ra, d[j], c);
                    rb = fold_word<REPL>(lslice, rb, d[j + 8], c);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    ra = fold_word<REPL>(lslice, ra, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), c);
                    rb = fold_word<REPL>(lslice, rb, __builtin_amdgcn_alignbyte(d[j + 9], d[j + 8], sh), c);
                }
            }
            r = zshift(lhalf, ra) ^ rb;
        } else {
            r = 0;
            if (__all(sh == 0 || !act)) {
#pragma unroll
                for (int j = 0; j < 16; ++j) r = fold_word<REPL>(lslice, r, d[j], c);
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    r = fold_word<REPL>(lslice, r, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), c);
            }
        }
        // advance over the rest of the window: 8 nibble lookups, lane-specific map, bank = lane&31
        uint32_t z = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) z ^= llane[lbase + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
        r = act ? z : 0u;
#pragma unroll
        for (int dlt = 1; dlt < Q; dlt <<= 1) r ^= __shfl_xor(r, dlt);
        if (cur.f < a.n) {
            if (act) R = zshift(lzw, R) ^ r;
            if (cur.wi + 1 >= cur.nw) {
                if (gl == 0) {
                    const uint64_t f = cur.f;
                    uint32_t state = R;
                    if (cur.Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * cur.Lc));
                    const uint32_t value = ~state;
                    const int64_t E = cur.E;
                    if (a.crc_out) a.crc_out[f] = cur.malformed ? 0u : value;
                    if (cur.malformed) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    } else if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                                ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                         1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        }
                    }
                }
                R = 0;
            }
        }
        cur = nxt;
#pragma unroll
        for (int j = 0; j < 17; ++j) d[j] = dn[j];
    }
}

// ---- v5: v4 + one-instruction table addressing + deeper prefetch --------------------------
// Slicing table k lives in 64 KiB region (k >> 1), half (k & 1): entry e of lane copy c at byte
// (k>>1)<<16 | e<<8 | (k&1)<<7 | c<<2, so ds_read_b32 bank = c = lane & 31 (conflict free) and
// the address of byte j of the register x is ONE v_perm_b32: byte j of x dropped into bits
// 8..15 of the lane's base word for that table.  PF windows of chunk data are in flight.
// Absolute LDS address: the v5 kernel has no static LDS, so its dynamic region starts at 0 and a
// byte offset is the LDS address itself (saves the base add per lookup).
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_word(const uint32_t*, uint32_t byte_addr) {
    return *reinterpret_cast<lds_u32_t*>(static_cast<uintptr_t>(byte_addr));
}

__device__ __forceinline__ uint32_t fold_word_perm(const uint32_t* lds, uint32_t r, uint32_t w,
                                                   const uint32_t (&lb)[4]) {
    const uint32_t x = r ^ w;
    // selector: out byte0 = lb.b0 (0), byte1 = x.byte j (4 + j), byte2 = lb.b2 (2), byte3 = lb.b3 (3)
    const uint32_t a3 = __builtin_amdgcn_perm(x, lb[3], 0x03020400u);  // byte 0 of x -> T3
    const uint32_t a2 = __builtin_amdgcn_perm(x, lb[2], 0x03020500u);  // byte 1 -> T2
    const uint32_t a1 = __builtin_amdgcn_perm(x, lb[1], 0x03020600u);  // byte 2 -> T1
    const uint32_t a0 = __builtin_amdgcn_perm(x, lb[0], 0x03020700u);  // byte 3 -> T0
    return lds_word(lds, a3) ^ lds_word(lds, a2) ^ lds_word(lds, a1) ^ lds_word(lds, a0);
}

template <int PF>
struct ChunkRing {
    uint32_t d[PF + 1][17];
};

template <int Q, int PF, bool NT = false>
__global__ __launch_bounds__(1024) void crc_frames_kernel5(FrameArgs a) {
    constexpr int S = 64;
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int kSliceBytes = 128 * 1024;
    constexpr int kLaneWords = (Q > 32 ? Q / 32 : 1) * 8 * 16 * 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    uint32_t* llane = lds + kSliceBytes / 4;
    uint32_t* lzw = llane + kLaneWords;
    for (int i = threadIdx.x; i < kSliceBytes / 4; i += blockDim.x) {
        // word i at byte 4i = region<<16 | e<<8 | half<<7 | c<<2
        const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
        lds[i] = a.slice[((region * 2 + half) << 8) | e];
    }
    for (int i = threadIdx.x; i < kLaneWords; i += blockDim.x) llane[i] = a.lanetab[i];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lzw[i] = a.zwin[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | (c << 2);
    const uint32_t lbase = (Q > 32 ? (uint32_t)(lane >> 5) * (8 * 16 * 32) : 0u) + c;
    const int gl = lane & (Q - 1);
    const int gid = lane / Q;
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t fstride = nwaves * kGroupsPerWave;
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    auto advance = [&](const Cursor& cc) {
        Cursor nx = cc;
        if (cc.f < a.n) {
            if (cc.wi + 1 < cc.nw) {
                nx.wi = cc.wi + 1;
            } else {
                nx.f = cc.f + fstride;
                cursor_frame(a, trailer, W, nx);
            }
        }
        return nx;
    };
    auto load_chunk = [&](const Cursor& cc, uint32_t (&dd)[17]) {
        const bool act = cc.f < a.n && cc.wi < cc.nw;
        const int64_t be = cc.E - (cc.nw - 1 - cc.wi) * W - (int64_t)(Q - 1 - gl) * S;
        const int64_t b0 = be - S - cc.sh;
        const bool safe = act ? (b0 >= 0 && b0 + 68 <= a.buf_len) : a.buf_len >= 68;
        if (__all(safe)) {
            // every lane loads (inactive lanes from the buffer start; their data is never used:
            // the fold masks r with act): no divergent zero-fill of registers a load may still
            // be writing, which would make the compiler drain the whole prefetch (vmcnt(0))
            const uint8_t* src = a.buf + (act ? b0 : 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (NT) {
                    const u32x4v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(src + 16 * q));
                    dd[4 * q] = v.x;
                    dd[4 * q + 1] = v.y;
                    dd[4 * q + 2] = v.z;
                    dd[4 * q + 3] = v.w;
                } else {
                    const u32x4a v = *reinterpret_cast<const u32x4a*>(src + 16 * q);
                    dd[4 * q] = v.x;
                    dd[4 * q + 1] = v.y;
                    dd[4 * q + 2] = v.z;
                    dd[4 * q + 3] = v.w;
                }
            }
            dd[16] = *reinterpret_cast<const uint32_t*>(src + 64);
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int64_t p = b0 + 4 * i;
                uint32_t v = 0;
                if (act && p + 4 > cc.o && p < be) {
                    if (p >= 0 && p + 4 <= a.buf_len)
                        v = *reinterpret_cast<const uint32_t*>(a.buf + p);
                    else
                        v = load_dword_clamped_slow(a.buf, p, a.buf_len);
                }
                dd[i] = v;
            }
        }
    };

    Cursor cq[PF + 1];
    uint32_t dq[PF + 1][17];
    cq[0].f = wave * kGroupsPerWave + gid;
    cursor_frame(a, trailer, W, cq[0]);
    load_chunk(cq[0], dq[0]);
#pragma unroll
    for (int p = 1; p < PF; ++p) {
        cq[p] = advance(cq[p - 1]);
        load_chunk(cq[p], dq[p]);
    }
    uint32_t R = 0;
    while (__any(cq[0].f < a.n)) {
        cq[PF] = advance(cq[PF - 1]);
        load_chunk(cq[PF], dq[PF]);
        const Cursor& cur = cq[0];
        uint32_t (&d)[17] = dq[0];

        const bool act = cur.f < a.n && cur.wi < cur.nw;
        const int64_t q0l = cur.E - (cur.nw - 1 - cur.wi) * W - (int64_t)(Q - gl) * S - cur.sh - cur.o;
        const bool special = act && q0l < 4;
        if (__any(special)) {
            const int64_t qc = q0l < -80 ? -80 : (q0l > 4 ? 4 : q0l);
            const int q0 = (int)qc;
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int q = q0 + 4 * i;
                uint32_t v = act ? d[i] : 0u;
                v = (q <= -4) ? 0u : (q < 0 ? (v & (0xFFFFFFFFu << (8 * -q))) : v);
                const uint32_t up = (q >= 0 && q < 4) ? (a.init >> (8 * q)) : 0u;
                const uint32_t dn2 = (q < 0 && q > -4) ? (a.init << (8 * -q)) : 0u;
                d[i] = (act && special) ? (v ^ up ^ dn2) : d[i];
            }
        }
        uint32_t r = 0;
        const uint32_t sh = cur.sh;
        if (__all(sh == 0 || !act)) {
#pragma unroll
            for (int j = 0; j < 16; ++j) r = fold_word_perm(lds, r, d[j], lb);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) r = fold_word_perm(lds, r, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), lb);
        }
        uint32_t z = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) z ^= llane[lbase + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
        r = act ? z : 0u;
#pragma unroll
        for (int dlt = 1; dlt < Q; dlt <<= 1) r ^= __shfl_xor(r, dlt);
        if (cur.f < a.n) {
            if (act) R = zshift(lzw, R) ^ r;
            if (cur.wi + 1 >= cur.nw) {
                if (gl == 0) {
                    const uint64_t f = cur.f;
                    uint32_t state = R;
                    if (cur.Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * cur.Lc));
                    const uint32_t value = ~state;
                    const int64_t E = cur.E;
                    if (a.crc_out) a.crc_out[f] = cur.malformed ? 0u : value;
                    if (cur.malformed) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    } else if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                                ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                         1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        }
                    }
                }
                R = 0;
            }
        }
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            cq[p] = cq[p + 1];
#pragma unroll
            for (int j = 0; j < 17; ++j) dq[p][j] = dq[p + 1][j];
        }
    }
}

// v7: v5 with S bytes per lane chunk (S = 128: the per-window cursor, load-address and combine
// work is amortised over twice the bytes).
template <int Q, int S, int PF>
__global__ __launch_bounds__(1024) void crc_frames_kernel7(FrameArgs a) {
    constexpr int NW = S / 4;  // words per lane chunk
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int kSliceBytes = 128 * 1024;
    constexpr int kLaneWords = (Q > 32 ? Q / 32 : 1) * 8 * 16 * 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    uint32_t* llane = lds + kSliceBytes / 4;
    uint32_t* lzw = llane + kLaneWords;
    for (int i = threadIdx.x; i < kSliceBytes / 4; i += blockDim.x) {
        // word i at byte 4i = region<<16 | e<<8 | half<<7 | c<<2
        const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
        lds[i] = a.slice[((region * 2 + half) << 8) | e];
    }
    for (int i = threadIdx.x; i < kLaneWords; i += blockDim.x) llane[i] = a.lanetab[i];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lzw[i] = a.zwin[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint32_t c = lane & 31;
    uint32_t lb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lb[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | (c << 2);
    const uint32_t lbase = (Q > 32 ? (uint32_t)(lane >> 5) * (8 * 16 * 32) : 0u) + c;
    const int gl = lane & (Q - 1);
    const int gid = lane / Q;
    constexpr int kGroupsPerWave = 64 / Q;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t fstride = nwaves * kGroupsPerWave;
    const bool trailer = (a.flags & (RH_CRC_VERIFY | RH_CRC_STAMP)) != 0;

    auto advance = [&](const Cursor& cc) {
        Cursor nx = cc;
        if (cc.f < a.n) {
            if (cc.wi + 1 < cc.nw) {
                nx.wi = cc.wi + 1;
            } else {
                nx.f = cc.f + fstride;
                cursor_frame(a, trailer, W, nx);
            }
        }
        return nx;
    };
    auto load_chunk = [&](const Cursor& cc, uint32_t (&dd)[NW + 1]) {
        const bool act = cc.f < a.n && cc.wi < cc.nw;
        const int64_t be = cc.E - (cc.nw - 1 - cc.wi) * W - (int64_t)(Q - 1 - gl) * S;
        const int64_t b0 = be - S - cc.sh;
        const bool safe = !act || (b0 >= 0 && b0 + S + 4 <= a.buf_len);
        if (__all(safe)) {
            if (act) {
#pragma unroll
                for (int q = 0; q < NW / 4; ++q) {
                    const u32x4a v = *reinterpret_cast<const u32x4a*>(a.buf + b0 + 16 * q);
                    dd[4 * q] = v.x;
                    dd[4 * q + 1] = v.y;
                    dd[4 * q + 2] = v.z;
                    dd[4 * q + 3] = v.w;
                }
                dd[NW] = *reinterpret_cast<const uint32_t*>(a.buf + b0 + S);
            } else {
#pragma unroll
                for (int i = 0; i < NW + 1; ++i) dd[i] = 0;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NW + 1; ++i) {
                const int64_t p = b0 + 4 * i;
                uint32_t v = 0;
                if (act && p + 4 > cc.o && p < be) {
                    if (p >= 0 && p + 4 <= a.buf_len)
                        v = *reinterpret_cast<const uint32_t*>(a.buf + p);
                    else
                        v = load_dword_clamped_slow(a.buf, p, a.buf_len);
                }
                dd[i] = v;
            }
        }
    };

    Cursor cq[PF + 1];
    uint32_t dq[PF + 1][NW + 1];
    cq[0].f = wave * kGroupsPerWave + gid;
    cursor_frame(a, trailer, W, cq[0]);
    load_chunk(cq[0], dq[0]);
#pragma unroll
    for (int p = 1; p < PF; ++p) {
        cq[p] = advance(cq[p - 1]);
        load_chunk(cq[p], dq[p]);
    }
    uint32_t R = 0;
    while (__any(cq[0].f < a.n)) {
        cq[PF] = advance(cq[PF - 1]);
        load_chunk(cq[PF], dq[PF]);
        const Cursor& cur = cq[0];
        uint32_t (&d)[NW + 1] = dq[0];

        const bool act = cur.f < a.n && cur.wi < cur.nw;
        const int64_t q0l = cur.E - (cur.nw - 1 - cur.wi) * W - (int64_t)(Q - gl) * S - cur.sh - cur.o;
        const bool special = act && q0l < 4;
        if (__any(special)) {
            const int64_t qc = q0l < -(S + 16) ? -(S + 16) : (q0l > 4 ? 4 : q0l);
            const int q0 = (int)qc;
#pragma unroll
            for (int i = 0; i < NW + 1; ++i) {
                const int q = q0 + 4 * i;
                uint32_t v = act ? d[i] : 0u;
                v = (q <= -4) ? 0u : (q < 0 ? (v & (0xFFFFFFFFu << (8 * -q))) : v);
                const uint32_t up = (q >= 0 && q < 4) ? (a.init >> (8 * q)) : 0u;
                const uint32_t dn2 = (q < 0 && q > -4) ? (a.init << (8 * -q)) : 0u;
                d[i] = (act && special) ? (v ^ up ^ dn2) : d[i];
            }
        }
        uint32_t r = 0;
        const uint32_t sh = cur.sh;
        if (__all(sh == 0 || !act)) {
#pragma unroll
            for (int j = 0; j < NW; ++j) r = fold_word_perm(lds, r, d[j], lb);
        } else {
#pragma unroll
            for (int j = 0; j < NW; ++j) r = fold_word_perm(lds, r, __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh), lb);
        }
        uint32_t z = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) z ^= llane[lbase + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
        r = act ? z : 0u;
#pragma unroll
        for (int dlt = 1; dlt < Q; dlt <<= 1) r ^= __shfl_xor(r, dlt);
        if (cur.f < a.n) {
            if (act) R = zshift(lzw, R) ^ r;
            if (cur.wi + 1 >= cur.nw) {
                if (gl == 0) {
                    const uint64_t f = cur.f;
                    uint32_t state = R;
                    if (cur.Lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * cur.Lc));
                    const uint32_t value = ~state;
                    const int64_t E = cur.E;
                    if (a.crc_out) a.crc_out[f] = cur.malformed ? 0u : value;
                    if (cur.malformed) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    } else if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                                ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)),
                                         1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        }
                    }
                }
                R = 0;
            }
        }
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            cq[p] = cq[p + 1];
#pragma unroll
            for (int j = 0; j < NW + 1; ++j) dq[p][j] = dq[p + 1][j];
        }
    }
}


// ---- v8: v5's fold with a copy-free prefetch ring and frame metadata staged in LDS -----------
// v5 rotates its register ring by copying (dq[p] = dq[p + 1]), which makes the compiler wait for
// the load it just issued (vmcnt(0) at the loop head), and reads each frame's offset/length from
// HBM right when it needs them, which drains every load in flight.  v8 keeps the same 16-lane x
// 64-byte fold and lane-distance tables, but
//   * the loop body is unrolled over the 3 ring slots with static roles (load slot i+2 while
//     folding slot i): a window's data is consumed two windows after its load was issued, and
//     every wait in the loop is a counted vmcnt(N);
//   * the frame table is staged per block in batches of 512 frames into LDS (one drain per batch),
//     group g of the block taking frames g, g+64, ... of the batch;
//   * the trailer for VERIFY comes from the last window's own chunk (one extra dword per lane), so
//     the verify needs no dependent byte loads; the group's lane 15 (whose chunk ends at the CRC
//     span's end) finalises the frame;
//   * inactive lanes load from the buffer start instead of zero-filling registers in flight.
// Frames whose chunks could leave the buffer (within 67 bytes of its start or 8 of its end),
// malformed and empty ones take a guarded byte path after the batch's main loop.
constexpr int kV8Batch = 512;
struct MetaV8 {
    int64_t o;    // frame start (bytes)
    uint32_t lc;  // CRC-covered length
    uint32_t fl;  // 0 = fast path; 1 = slow path (guarded), 2 = malformed
};

template <int PF, int CH = 1, bool ABLATE = false>
__global__ __launch_bounds__(1024) void crc_frames_kernel8(FrameArgs a) {
    static_assert(PF == 2, "v8 ring: 3 slots");
    static_assert(CH == 1 || CH == 2 || CH == 4, "fold chains per lane");
    constexpr int Q = 16, S = 64;
    constexpr int64_t W = (int64_t)Q * S;
    constexpr int kSliceBytes = 128 * 1024;
    constexpr int kLaneWords = 8 * 16 * 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (__builtin_amdgcn_groupstaticsize() != 0) __builtin_trap();  // lds_word assumes base 0
    uint32_t* llane = lds + kSliceBytes / 4;
    uint32_t* lzw = llane + kLaneWords;
    uint32_t* lch = lzw + 1024;  // [4][256]: advance over 64 / CH zero bytes (chain combine)
    // batch frame table, struct-of-arrays: start, CRC-covered length, path; then the guarded list
    int64_t* mo = reinterpret_cast<int64_t*>(lch + 1024);
    uint32_t* mlc = reinterpret_cast<uint32_t*>(mo + kV8Batch);
    uint8_t* mfl = reinterpret_cast<uint8_t*>(mlc + kV8Batch);
    uint16_t* slow = reinterpret_cast<uint16_t*>(mfl + kV8Batch);  // [kV8Batch] guarded-path frames
    uint32_t* nslow = reinterpret_cast<uint32_t*>(slow + kV8Batch);
    auto meta = [&](uint32_t j) { return MetaV8{mo[j], mlc[j], mfl[j]}; };
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

    for (uint64_t b0f = (uint64_t)blockIdx.x * kV8Batch; b0f < a.n; b0f += (uint64_t)gridDim.x * kV8Batch) {
        const uint32_t nb = (uint32_t)(a.n - b0f < (uint64_t)kV8Batch ? a.n - b0f : (uint64_t)kV8Batch);
        __syncthreads();  // previous batch done with meta / slow
        if (t == 0) *nslow = 0;
        __syncthreads();
        if ((uint32_t)t < nb) {
            const uint64_t f = b0f + (uint64_t)t;
            const uint64_t o = a.off[f];
            const int64_t L = (int64_t)a.len[f];
            const bool malformed = o > (uint64_t)a.buf_len || L > a.buf_len - (int64_t)o || (trailer && L < 4);
            MetaV8 m;
            m.o = (int64_t)o;
            m.lc = malformed ? 0u : (uint32_t)(L - (int64_t)tl);
            const int64_t E = m.o + (int64_t)m.lc;
            const bool unsafe = m.o < 67 || E + 8 > a.buf_len || m.lc < 8;
            m.fl = malformed ? 2u : (unsafe ? 1u : 0u);
            if (a.slot_nframes) {  // slot mode: slots past the segment's frame count are skipped
                const uint32_t nfs = a.slot_nframes[f / a.slot_cap];
                if (f % a.slot_cap >= (nfs < a.slot_cap ? nfs : a.slot_cap)) m.fl = 3u;
            }
            mo[t] = m.o;
            mlc[t] = m.lc;
            mfl[t] = (uint8_t)m.fl;
            if (m.fl == 1u || m.fl == 2u) slow[atomicAdd(nslow, 1u)] = (uint16_t)t;
        }
        __syncthreads();

        // ---- fast path: group grp walks the windows of batch frames grp, grp + 64, ... ----
        struct Task {
            uint32_t j;   // batch-local frame (>= nb: none)
            uint32_t wi;  // window
        };
        auto skip = [&](uint32_t j) {  // next fast-path frame at or after j (stride 64)
            while (j < nb && mfl[j] != 0) j += 64;
            return j;
        };
        auto next = [&](Task x) {
            if (x.j >= nb) return x;
            const uint32_t nw = (mlc[x.j] + (uint32_t)W - 1) / (uint32_t)W;
            if (x.wi + 1 < nw) return Task{x.j, x.wi + 1};
            return Task{skip(x.j + 64), 0u};
        };
        // chunk of lane gl in task x: [be - S, be), be = E - (nw - 1 - wi) W - (Q - 1 - gl) S
        auto load = [&](Task x, uint32_t (&dd)[18]) {
            const uint8_t* src = a.buf;
            if (x.j < nb) {
                const MetaV8 m = meta(x.j);
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
            const MetaV8 m = meta(x.j);
            const int64_t E = m.o + (int64_t)m.lc;
            const int64_t nw = ((int64_t)m.lc + W - 1) / W;
            const uint32_t sh = (uint32_t)(E & 3);
            const int64_t be = E - (nw - 1 - (int64_t)x.wi) * W - (int64_t)(Q - 1 - gl) * S;
            const bool act = be > m.o;
            const int64_t q0l = be - S - (int64_t)sh - m.o;  // chunk start (aligned) rel. to frame start
            if (__any(act && q0l < 4)) {
                const int q0 = (int)(q0l < -80 ? -80 : (q0l > 4 ? 4 : q0l));
#pragma unroll
                for (int i = 0; i < 17; ++i) {
                    const int q = q0 + 4 * i;
                    uint32_t v = d[i];
                    v = (q <= -4) ? 0u : (q < 0 ? (v & (0xFFFFFFFFu << (8 * -q))) : v);
                    const uint32_t up = (q >= 0 && q < 4) ? (a.init >> (8 * q)) : 0u;
                    const uint32_t dn2 = (q < 0 && q > -4) ? (a.init << (8 * -q)) : 0u;
                    d[i] = (act && q0l < 4) ? (v ^ up ^ dn2) : d[i];
                }
            }
            // CH independent chains of 16 / CH words (the LDS round trips overlap), joined by
            // Horner steps over 64 / CH zero bytes: CRC(A||B) = adv_|B|(crc A) ^ crc B from zero
            constexpr int LW = 16 / CH;
            uint32_t rc[CH];
#pragma unroll
            for (int q = 0; q < CH; ++q) rc[q] = 0;
            if (ABLATE) {
            } else if (__all(sh == 0 || !act)) {
#pragma unroll
                for (int j = 0; j < LW; ++j)
#pragma unroll
                    for (int q = 0; q < CH; ++q) rc[q] = fold_word_perm(lds, rc[q], d[q * LW + j], lb);
            } else {
#pragma unroll
                for (int j = 0; j < LW; ++j)
#pragma unroll
                    for (int q = 0; q < CH; ++q)
                        rc[q] = fold_word_perm(lds, rc[q], __builtin_amdgcn_alignbyte(d[q * LW + j + 1], d[q * LW + j], sh), lb);
            }
            uint32_t r = rc[0];
#pragma unroll
            for (int q = 1; q < CH; ++q) r = zshift(lch, r) ^ rc[q];
            if (ABLATE) {  // access-pattern ablation: same loads and outputs, no table work
                r = 0;
#pragma unroll
                for (int j = 0; j < 17; ++j) r ^= d[j];
            }
            uint32_t z = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) z ^= llane[c + ((uint32_t)(k * 16) + ((r >> (4 * k)) & 15u)) * 32u];
            r = act ? z : 0u;
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x141, 0xF, 0xF, false);  // row_half_mirror
            r ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x140, 0xF, 0xF, false);  // row_mirror
            R = zshift(lzw, R) ^ r;
            if ((int64_t)x.wi + 1 >= nw) {
                if (gl == Q - 1) {  // this lane's chunk ends at E: d[16..17] hold bytes E - sh .. E + 8 - sh
                    const uint64_t f = b0f + x.j;
                    uint32_t state = R;
                    if (m.lc < 4) state ^= (uint32_t)((uint64_t)a.init >> (8 * m.lc));
                    const uint32_t value = ~state;
                    if (a.crc_out) a.crc_out[f] = value;
                    if (a.flags & RH_CRC_STAMP) {
                        a.wbuf[E + 0] = (uint8_t)(value >> 24);
                        a.wbuf[E + 1] = (uint8_t)(value >> 16);
                        a.wbuf[E + 2] = (uint8_t)(value >> 8);
                        a.wbuf[E + 3] = (uint8_t)value;
                    } else if (a.flags & RH_CRC_VERIFY) {
                        const uint32_t le = __builtin_amdgcn_alignbyte(d[17], d[16], sh);
                        const uint32_t stored = __builtin_bswap32(le);  // big-endian trailer
                        if (stored != value) {
                            if (a.bad_bits)
                                atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                            if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                            if (a.seg_first_bad) atomicMin(a.seg_first_bad + f / a.slot_cap, (uint32_t)(f % a.slot_cap));
                        }
                    }
                }
                R = 0;
            }
        };
        Task T0{a.buf_len >= 128 ? skip(grp) : nb, 0u};  // tiny buffers: every frame is guarded
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
            const MetaV8 m = meta(j);
            const uint64_t f = b0f + j;
            if (m.fl == 2) {
                if (gl == 0) {
                    if (a.crc_out) a.crc_out[f] = 0u;
                    if (a.bad_bits) atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                    if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                    if (a.seg_first_bad) atomicMin(a.seg_first_bad + f / a.slot_cap, (uint32_t)(f % a.slot_cap));
                }
                continue;
            }
            const int64_t E = m.o + (int64_t)m.lc;
            const int64_t nw = ((int64_t)m.lc + W - 1) / W;
            uint32_t Rs = 0;
            for (int64_t wi = 0; wi < nw; ++wi) {
                const int64_t be = E - (nw - 1 - wi) * W - (int64_t)(Q - 1 - gl) * S;
                const int64_t bs = be - S > m.o ? be - S : m.o;
                uint32_t r = 0;
                for (int64_t p = bs; p < be; ++p) {  // byte-wise, reset()'s state in bytes 0..3
                    uint32_t b = a.buf[p];
                    if (p - m.o < 4) b ^= (a.init >> (8 * (p - m.o))) & 0xffu;
                    r = (r >> 8) ^ a.slice[(r ^ b) & 0xffu];
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
                if (a.crc_out) a.crc_out[f] = value;
                if (a.flags & RH_CRC_STAMP) {
                    a.wbuf[E + 0] = (uint8_t)(value >> 24);
                    a.wbuf[E + 1] = (uint8_t)(value >> 16);
                    a.wbuf[E + 2] = (uint8_t)(value >> 8);
                    a.wbuf[E + 3] = (uint8_t)value;
                } else if (a.flags & RH_CRC_VERIFY) {
                    const uint32_t stored = ((uint32_t)a.buf[E] << 24) | ((uint32_t)a.buf[E + 1] << 16) |
                                            ((uint32_t)a.buf[E + 2] << 8) | (uint32_t)a.buf[E + 3];
                    if (stored != value) {
                        if (a.bad_bits)
                            atomicOr(reinterpret_cast<unsigned long long*>(a.bad_bits + (f >> 6)), 1ull << (f & 63));
                        if (a.n_bad) atomicAdd(a.n_bad, 1ull);
                        if (a.seg_first_bad) atomicMin(a.seg_first_bad + f / a.slot_cap, (uint32_t)(f % a.slot_cap));
                    }
                }
            }
        }
    }
}


struct Variant {
    int q, s;
    bool repl;
};

constexpr Variant kVariants[] = {
    {64, 64, true},    // 0: one wave per 4 KiB window (default)
    {16, 256, true},   // 1: four 4 KiB windows per wave
    {8, 512, true},    // 2: eight 4 KiB windows per wave
    {64, 64, false},   // 3: shared (non-replicated) tables, for the bank-conflict A/B
    {64, 64, true},    // 4: v2 (window prefetch), replicated tables
    {64, 64, false},   // 5: v2, shared tables, 4 workgroups per CU
    {16, 64, true},    // 6: v2, 16 lanes x 64 B = 1 KiB windows
    {64, 64, true},    // 7: v3 branch-free fold, ILP 1
    {64, 64, true},    // 8: v3, ILP 2
    {16, 64, true},    // 9: v3, 16 lanes, ILP 2
    {64, 64, false},   // 10: v3, shared tables, ILP 2, 4 workgroups per CU
    {16, 64, true},    // 11: v4, 16 lanes x 64 B windows, ILP 1
    {16, 64, true},    // 12: v4, ILP 2
    {32, 64, true},    // 13: v4, 32 lanes, ILP 2
    {16, 64, true},    // 14: v5 (perm addressing), prefetch 1 window
    {16, 64, true},    // 15: v5, prefetch 2 windows
    {16, 64, true},    // 16: v5, prefetch 3 windows
    {32, 64, true},    // 17: v5, 32 lanes, prefetch 2
    {16, 128, true},   // 18: v7 (v5 with 128-byte lane chunks, 2 KiB windows), prefetch 1
    {16, 128, true},   // 19: v7, prefetch 2
    {8, 128, true},    // 20: v7, 8 lanes x 128 B = 1 KiB windows, prefetch 1
    {16, 64, true},    // 21: v5 (15) with non-temporal 16-byte loads, prefetch 2
    {16, 64, true},    // 22: v5 with non-temporal loads, prefetch 1
    {16, 64, true},    // 23: v8 (v5 fold, copy-free 3-slot ring, LDS-staged frame metadata)
    {16, 64, true},    // 24: v8 with 2 independent fold chains per lane
    {16, 64, true},    // 25: v8 with 4 independent fold chains per lane
    {16, 64, true},    // 26: ABLATION ONLY (wrong CRCs): v8's loads and stores without the table fold
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
constexpr int kAblationVariant = 26;  // launchable by index for A/B, not counted as a CRC kernel

int g_default_variant = 24;  // v8 with 2 fold chains per lane (fastest measured)

template <int Q, int S, bool REPL, int V = 1, int ILP = 1>
int launch_variant(rh_ctx* ctx, const FrameArgs& fa, hipStream_t stream) {
    constexpr int LOGQ = __builtin_ctz(Q);
    constexpr size_t lds = V >= 9 ? (size_t)128 * 1024 + 16384 + 8192 + kV8Batch * 15 + 16
                         : V >= 5 ? (size_t)128 * 1024 + (size_t)(Q > 32 ? Q / 32 : 1) * 16384 + 4096
                         : V == 4 ? (REPL ? 4 * 256 * 32 * 4 : 4 * 256 * 4) + (size_t)(Q > 32 ? Q / 32 : 1) * 16384 + 4096 +
                                        (ILP == 2 ? 4096 : 0)
                                  : (REPL ? 4 * 256 * 32 * 4 : 4 * 256 * 4) + (size_t)(LOGQ + 1) * 4096 + (ILP == 2 ? 4096 : 0);
    static_assert(lds <= 160 * 1024, "LDS budget");
    const int block = REPL ? 1024 : 256;
    const int per_cu = REPL ? 1 : 4;
    void (*kern)(FrameArgs);
    if constexpr (V == 12)
        kern = crc_frames_kernel8<ILP, 1, true>;
    else if constexpr (V == 9 || V == 10 || V == 11)
        kern = crc_frames_kernel8<ILP, V == 9 ? 1 : (V == 10 ? 2 : 4)>;
    else if constexpr (V == 7)
        kern = crc_frames_kernel7<Q, S, ILP>;
    else if constexpr (V == 5 || V == 8)
        kern = crc_frames_kernel5<Q, ILP, V == 8>;  // ILP carries the prefetch depth; 8 = NT loads
    else if constexpr (V == 4)
        kern = crc_frames_kernel4<Q, ILP, REPL>;
    else if constexpr (V == 3)
        kern = crc_frames_kernel3<Q, ILP, REPL>;
    else if constexpr (V == 2)
        kern = crc_frames_kernel2<Q, S, REPL>;
    else
        kern = crc_frames_kernel<Q, S, REPL>;
    static bool attr_set = false;
    if (!attr_set) {
        RH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = true;
    }
    const uint64_t groups = (fa.n + (64 / Q) - 1) / (64 / Q);   // wave-iterations needed
    uint64_t grid = (uint64_t)ctx->num_cus * per_cu;
    const uint64_t need = V >= 9 ? (fa.n + kV8Batch - 1) / kV8Batch : (groups + (block / 64) - 1) / (block / 64);
    if (need < grid) grid = need ? need : 1;
    FrameArgs a = fa;
    // per-level shift tables: S*2^j for j < LOGQ, then W
    a.shift = ctx->d_shift + (size_t)__builtin_ctz(S) * 1024;
    a.shift32 = ctx->d_shift + (size_t)(V == 11 ? 4 : 5) * 1024;  // v8 chain combine: 64 / CH bytes
    a.zwin = ctx->d_shift + (size_t)__builtin_ctz(Q * S) * 1024;
    if constexpr (S == 128)
        a.lanetab = Q == 16 ? ctx->d_lane16_s128 : ctx->d_lane8_s128;
    else
        a.lanetab = Q == 16 ? ctx->d_lane16 : (Q == 32 ? ctx->d_lane32 : ctx->d_lane64);
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(block), lds, stream, a);
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
    uint32_t** dst[6] = {&ctx->d_lane16, &ctx->d_lane32, &ctx->d_lane64, &ctx->d_lane16_s128, &ctx->d_lane8_s128,
                         &ctx->d_lane16_s36};
    const int qs[6] = {16, 32, 64, 16, 8, 16};
    const int ss[6] = {64, 64, 64, 128, 128, 36};
    {
        uint32_t zu[4][256];
        rh::build_crc_shift_table(576, zu);
        RH_HIP(hipMalloc(&ctx->d_zu576, sizeof(zu)));
        RH_HIP(hipMemcpy(ctx->d_zu576, zu, sizeof(zu), hipMemcpyHostToDevice));
    }
    for (int i = 0; i < 6; ++i) {
        std::vector<uint32_t> lt = rh::build_crc_lane_tables(qs[i], ss[i]);
        RH_HIP(hipMalloc(dst[i], lt.size() * 4));
        RH_HIP(hipMemcpy(*dst[i], lt.data(), lt.size() * 4, hipMemcpyHostToDevice));
    }
    return RH_OK;
}

int rh_crc_launch_variant(rh_ctx* ctx, const rh_frames* f, uint32_t flags, int variant, hipStream_t stream) {
    if (!f) return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: frames == NULL");
    if ((flags & ~(RH_CRC_VERIFY | RH_CRC_STAMP)) || flags == (RH_CRC_VERIFY | RH_CRC_STAMP))
        return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: flags must be 0, VERIFY or STAMP");
    if (f->n == 0) return RH_OK;
    if (!f->buf || !f->frame_off || !f->frame_len)
        return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: buf, frame_off, frame_len required");
    if (variant < 0 || variant >= kNumVariants) return rh::fail(RH_E_INVAL, "unknown CRC kernel variant");
    FrameArgs a{};
    a.buf = f->buf;
    a.wbuf = f->buf;
    if (f->buf_len > (uint64_t)INT64_MAX) return rh::fail(RH_E_RANGE, "rh_crc32c_frames_launch: buf_len too large");
    a.buf_len = (int64_t)f->buf_len;
    a.off = f->frame_off;
    a.len = f->frame_len;
    a.n = f->n;
    a.init = f->init_state;
    a.flags = flags;
    a.crc_out = f->crc_out;
    a.bad_bits = f->bad_bits;
    a.n_bad = f->n_bad;
    a.slice = ctx->d_slice;
    switch (variant) {
        case 0: return launch_variant<64, 64, true>(ctx, a, stream);
        case 1: return launch_variant<16, 256, true>(ctx, a, stream);
        case 2: return launch_variant<8, 512, true>(ctx, a, stream);
        case 3: return launch_variant<64, 64, false>(ctx, a, stream);
        case 4: return launch_variant<64, 64, true, 2>(ctx, a, stream);
        case 5: return launch_variant<64, 64, false, 2>(ctx, a, stream);
        case 6: return launch_variant<16, 64, true, 2>(ctx, a, stream);
        case 7: return launch_variant<64, 64, true, 3, 1>(ctx, a, stream);
        case 8: return launch_variant<64, 64, true, 3, 2>(ctx, a, stream);
        case 9: return launch_variant<16, 64, true, 3, 2>(ctx, a, stream);
        case 10: return launch_variant<64, 64, false, 3, 2>(ctx, a, stream);
        case 11: return launch_variant<16, 64, true, 4, 1>(ctx, a, stream);
        case 12: return launch_variant<16, 64, true, 4, 2>(ctx, a, stream);
        case 13: return launch_variant<32, 64, true, 4, 2>(ctx, a, stream);
        case 14: return launch_variant<16, 64, true, 5, 1>(ctx, a, stream);
        case 15: return launch_variant<16, 64, true, 5, 2>(ctx, a, stream);
        case 16: return launch_variant<16, 64, true, 5, 3>(ctx, a, stream);
        case 17: return launch_variant<32, 64, true, 5, 2>(ctx, a, stream);
        case 18: return launch_variant<16, 128, true, 7, 1>(ctx, a, stream);
        case 19: return launch_variant<16, 128, true, 7, 2>(ctx, a, stream);
        case 20: return launch_variant<8, 128, true, 7, 1>(ctx, a, stream);
        case 21: return launch_variant<16, 64, true, 8, 2>(ctx, a, stream);
        case 22: return launch_variant<16, 64, true, 8, 1>(ctx, a, stream);
        case 23: return launch_variant<16, 64, true, 9, 2>(ctx, a, stream);
        case 24: return launch_variant<16, 64, true, 10, 2>(ctx, a, stream);
        case 25: return launch_variant<16, 64, true, 11, 2>(ctx, a, stream);
        case 26: return launch_variant<16, 64, true, 12, 2>(ctx, a, stream);
    }
    return rh::fail(RH_E_INVAL, "unknown CRC kernel variant");
}

int rh_crc_launch_impl(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream) {
    return rh_crc_launch_variant(ctx, f, flags, g_default_variant, stream);
}

int rh_crc_set_default_variant(int v) {
    if (v < 0 || v >= kAblationVariant) return rh::fail(RH_E_INVAL, "unknown CRC kernel variant");
    g_default_variant = v;
    return RH_OK;
}

int rh_crc_num_variants() { return kAblationVariant; }  // exact variants 0..25

// The read path's CRC pass (rh_segments_read_launch, default variant): crc_frames_kernel8 over the
// slotted frame table the framing walk left in segs->scratch_off/len, VERIFY, CRCs into
// crc->scratch_crc (slot-indexed), mismatches counted in crc->n_bad and the first bad slot of each
// segment atomically lowered in crc->seg_ok (pre-set to 0xFFFFFFFF by the caller).
int rh_crc_verify_slots(rh_ctx* ctx, const rh_segments* g, const rh_segments_crc* c, hipStream_t stream) {
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
    a.slice = ctx->d_slice;
    a.slot_nframes = g->seg_nframes;
    a.slot_cap = g->frames_per_seg_cap;
    a.seg_first_bad = c->seg_ok;
    return launch_variant<16, 64, true, 10, 2>(ctx, a, stream);
}
