// Batched quorum commit for gfx950 (MI355X).
//
// Restates, per RaftGroup, the leader's commit decision of the reference:
//   LeaderStateImpl.getMajorityMin        LeaderStateImpl.java:956-984
//   LeaderStateImpl.getSorted             LeaderStateImpl.java:1076-1095
//   MinMajorityMax.valueOf / combine      LeaderStateImpl.java:904-944
//   LeaderStateImpl.updateCommit(maj,min) LeaderStateImpl.java:1015-1026
//   RaftLogBase.updateCommitIndex         RaftLogBase.java:121-142
// and, in WATCH mode, LeaderStateImpl.commitIndexChanged (LeaderStateImpl.java:612-622).
//
// Per-group arithmetic: commit_eval.h.  Layout: one struct-of-arrays "tier" per follower-slot
// count F, either plain (every column a contiguous int64 array over the tier's groups) or tiled
// (tiles of 128 groups holding 128 elements of every column back to back, so one wave's loads
// are one contiguous run); either way a wave's load of one column is one coalesced 1 KiB request
// (2 groups per lane, 16 B per lane).  The order statistics over <= F+1 voters are
// integer compare/select work in registers -- rank masks for F <= 6 (commit_kernel_rank), a
// Batcher merge-exchange network for wider tiers (commit_kernel_net) -- no MFMA (this is not a
// contraction).  The kernel is HBM-bound: 8(F+1)+20 bytes read and 16 bytes written per group.
#include "rh_internal.h"
#include "commit_eval.h"
#include "lease_eval.h"

namespace {

#ifndef RH_COMMIT_XCD
#define RH_COMMIT_XCD 0
#endif
#ifndef RH_COMMIT_BLOCK   // A/B: threads per commit_kernel_rank / _net workgroup (the fused leader kernel keeps 256)
#define RH_COMMIT_BLOCK 256
#endif
constexpr int kBlock = RH_COMMIT_BLOCK;
constexpr int kLeaderBlock = 256;      // 4 waves
#ifndef RH_COMMIT_WAVES  // A/B builds override (scripts/ab_build.sh): waves per SIMD the F <= 6 kernels are pinned to
#define RH_COMMIT_WAVES 8
#endif
constexpr int kGroupsPerLane = 2;      // 16-byte loads per column per lane
#ifndef RH_COMMIT_BITS_DIRECT  // 1 = each wave stores its bit words itself (no LDS staging, no barrier)
#define RH_COMMIT_BITS_DIRECT 1
#endif
#ifndef RH_COMMIT_ABL_NOEVAL  // ablation only (wrong results): trivial arithmetic instead of eval_group
#define RH_COMMIT_ABL_NOEVAL 0
#endif
#ifndef RH_COMMIT_NTS  // 1 = non-temporal result stores (A/B: plain stores measured 0.2 us faster per 1M-group launch)
#define RH_COMMIT_NTS 0
#endif

struct TierArgs {
    rh_commit_soa t;
    uint64_t stride;        // elements between follower columns
    uint64_t tile64;        // tiled layout: int64 elements between tiles (0 = plain columns)
    uint64_t tile32;        // tiled layout: uint32 elements between tiles
    uint32_t block_begin;   // first block of this tier in the launch
    uint32_t n_blocks;
    bool vec_ok;            // every column 16-byte aligned: full tiles use 16-byte loads
};

// Element index of group r in a per-group column: plain (r) or tiled (tile * tile elems + r % 128).
__device__ __forceinline__ uint64_t ix64(const TierArgs& ta, uint64_t r) {
    return ta.tile64 ? (r >> 7) * ta.tile64 + (r & 127u) : r;
}
__device__ __forceinline__ uint64_t ix32(const TierArgs& ta, uint64_t r) {
    return ta.tile32 ? (r >> 7) * ta.tile32 + (r & 127u) : r;
}

// The block -> tier map leads the struct (one scalar load), then the tiers' arguments.
struct LaunchArgs {
    uint32_t n_tiers;
    uint32_t begin[RH_MAX_TIERS];   // = tier[i].block_begin
    uint32_t pad[3];
    TierArgs tier[RH_MAX_TIERS];
};

using rh_bits::spread32;

typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

// A 128-group sub-tile of one wave: lane l holds rows r0 = base + 2l and r0 + 1.
template <int F>
struct SubTile {
    int64_t fv[2][F];
    int64_t self[2], cin[2], tstart[2];
    uint32_t w[2];
};

// 16-byte column load; NT marks it non-temporal (streamed once, no reuse in L2/MALL).
template <bool NT, typename V>
__device__ __forceinline__ V ld16(const void* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
    return *reinterpret_cast<const V*>(p);
}

template <int F, bool VEC, bool NT = false>
__device__ __forceinline__ void load_sub(const TierArgs& ta, uint64_t r0, bool commit_mode, SubTile<F>& st) {
    const rh_commit_soa& t = ta.t;
    if (VEC) {
        const uint64_t e = ix64(ta, r0), e32 = ix32(ta, r0);  // r0 even: e, e + 1 in one tile
#pragma unroll
        for (int k = 0; k < F; ++k) {
            const v2i64 x = ld16<NT, v2i64>(t.follower_index + (uint64_t)k * ta.stride + e);
            st.fv[0][k] = x.x;
            st.fv[1][k] = x.y;
        }
        const v2i64 s = ld16<NT, v2i64>(t.self_index + e);
        st.self[0] = s.x;
        st.self[1] = s.y;
        const v2u32 c = NT ? __builtin_nontemporal_load(reinterpret_cast<const v2u32*>(t.conf + e32))
                           : *reinterpret_cast<const v2u32*>(t.conf + e32);
        st.w[0] = c.x;
        st.w[1] = c.y;
        if (commit_mode) {
            const v2i64 ci = ld16<NT, v2i64>(t.commit_in + e);
            const v2i64 ts = ld16<NT, v2i64>(t.term_start + e);
            st.cin[0] = ci.x;
            st.cin[1] = ci.y;
            st.tstart[0] = ts.x;
            st.tstart[1] = ts.y;
        } else {
            st.cin[0] = st.cin[1] = st.tstart[0] = st.tstart[1] = 0;
        }
    } else {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const uint64_t r = r0 + g;
            const bool in = r < t.n;
            const uint64_t e = ix64(ta, r);
#pragma unroll
            for (int k = 0; k < F; ++k) st.fv[g][k] = in ? t.follower_index[(uint64_t)k * ta.stride + e] : 0;
            st.self[g] = in ? t.self_index[e] : 0;
            st.w[g] = in ? t.conf[ix32(ta, r)] : 0u;  // rows past n: inactive padding
            st.cin[g] = (in && commit_mode) ? t.commit_in[e] : 0;
            st.tstart[g] = (in && commit_mode) ? t.term_start[e] : 0;
        }
    }
}

template <bool NT>
__device__ __forceinline__ void st16(int64_t* p, int64_t a, int64_t b) {
    v2i64 v;
    v.x = a;
    v.y = b;
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<v2i64*>(p));
    else
        *reinterpret_cast<v2i64*>(p) = v;
}

template <int F, bool VEC, bool RANK = false, bool NTS = false>
__device__ __forceinline__ void compute_store_sub(const TierArgs& ta, uint64_t wbase, bool commit_mode,
                                                  const SubTile<F>& st, uint64_t (&bits)[2][8]) {
    constexpr int N = F + 1;
    const rh_commit_soa& t = ta.t;
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = wbase + 2 * (uint64_t)lane;

    // ---- getMajorityMin (LSI:956-984) + updateCommit(majority, min) (LSI:1015-1026) ----
    const int64_t gap = commit_mode ? t.gap_threshold : -1;  // 2-arg overload passes -1 (LSI:952-954)
    bool valid[2], adv[2];
    int64_t mn[2], mj[2], mx[2], cout[2];
    bool trans[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) trans[g] = (st.w[g] & RH_CONF_ACTIVE) && (st.w[g] & RH_CONF_TRANSITIONAL);
    const bool any_trans = __any(trans[0] || trans[1]);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        int64_t vals[N];
#pragma unroll
        for (int k = 0; k < F; ++k) vals[k] = st.fv[g][k];
        vals[F] = st.self[g];
#if RH_COMMIT_ABL_NOEVAL
        (void)any_trans;
        valid[g] = (st.w[g] & RH_CONF_ACTIVE) != 0;
        mn[g] = vals[0];
#pragma unroll
        for (int k = 1; k < N; ++k) mn[g] ^= vals[k];   // every loaded column stays live
        mj[g] = mn[g] + 1;
        mx[g] = mn[g] + 2;
#else
        rh_eval::eval_group<F, RANK>(vals, st.w[g], gap, any_trans, valid[g], mn[g], mj[g], mx[g]);
#endif
        adv[g] = commit_mode && rh_eval::commit_decision(valid[g], mj[g], st.cin[g], st.self[g], st.tstart[g], cout[g]);
        if (!commit_mode) cout[g] = st.cin[g];
    }

    // ---- stores ----
    if (VEC) {
        const uint64_t e = ix64(ta, r0);
        if (commit_mode) st16<NTS>(t.commit_out + e, cout[0], cout[1]);
        if (t.min_out) st16<NTS>(t.min_out + e, mn[0], mn[1]);
        if (t.maj_out) st16<NTS>(t.maj_out + e, mj[0], mj[1]);
        if (t.max_out) st16<NTS>(t.max_out + e, mx[0], mx[1]);
    } else {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const uint64_t r = r0 + g;
            if (r < t.n) {
                const uint64_t e = ix64(ta, r);
                if (commit_mode) t.commit_out[e] = cout[g];
                if (t.min_out) t.min_out[e] = mn[g];
                if (t.maj_out) t.maj_out[e] = mj[g];
                if (t.max_out) t.max_out[e] = mx[g];
            }
        }
    }

    // ---- per-wave bit words: bit j of word (wbase/64 + h) is row wbase + 64h + j ----
    // Lane p fetches the 2 rows of lane 32h + p/2 (one ds_bpermute per word) and keeps row p & 1,
    // so one ballot per word and column yields the word directly (no scalar bit interleave: the
    // scalar unit is shared by the CU's waves).  Staged in LDS; run_tile stores the block's words.
    const int wave = threadIdx.x >> 6;
    if (t.valid_bits || t.advanced_bits) {
        const int packed = (valid[0] ? 1 : 0) | (valid[1] ? 2 : 0) | (adv[0] ? 4 : 0) | (adv[1] ? 8 : 0);
        const int lo = __shfl(packed, lane >> 1), hi = __shfl(packed, 32 + (lane >> 1));
        const int sel = lane & 1;
        const uint64_t v0 = __ballot((lo >> sel) & 1), v1 = __ballot((hi >> sel) & 1);
        const uint64_t a0 = __ballot((lo >> (2 + sel)) & 1), a1 = __ballot((hi >> (2 + sel)) & 1);
#if RH_COMMIT_BITS_DIRECT
        // A/B: every wave stores its own two words per column (no LDS staging, no block barrier)
        (void)wave;
        (void)bits;
        const uint64_t word = (wbase >> 6) + (uint64_t)lane;
        if (lane < 2 && word < ((t.n + 63) >> 6)) {
            if (t.valid_bits) t.valid_bits[word] = lane ? v1 : v0;
            if (t.advanced_bits) t.advanced_bits[word] = lane ? a1 : a0;
        }
#else
        if (lane < 2) {
            bits[0][2 * wave + lane] = lane ? v1 : v0;
            bits[1][2 * wave + lane] = lane ? a1 : a0;
        }
#endif
    }

    // ---- compacted advanced list: one atomic per wave ----
    const uint64_t ae = t.adv_rows ? __ballot(adv[0]) : 0ull, ao = t.adv_rows ? __ballot(adv[1]) : 0ull;
    if (t.adv_rows && (ae | ao)) {
        const uint32_t cnt = __popcll(ae) + __popcll(ao);
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(t.adv_count, (unsigned long long)cnt);
        base = __shfl(base, 0);
        const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
        uint64_t pos = base + __popcll(ae & lt) + __popcll(ao & lt);
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (adv[g]) {
                if (pos < t.adv_cap) {
                    t.adv_rows[pos] = t.adv_row_base + r0 + g;
                    t.adv_commit[pos] = cout[g];
                }
                ++pos;
            }
        }
    }
}

// One wave = one 128-group sub-tile: all loads of the tile are issued before any compute.  The
// block's bit words (8 per column) leave through LDS in one 64-byte store per column.
template <int F, bool RANK, bool NT, bool NTS, int BLOCK>
__device__ __forceinline__ void run_tile(const TierArgs& ta, uint64_t tile) {
    constexpr uint64_t kWaveGroups = 128;
    __shared__ uint64_t bits[2][8];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t wchunk = tile * (kWaveGroups * (BLOCK / 64)) + (uint64_t)wave * kWaveGroups;
    const bool commit_mode = ta.t.mode == RH_MODE_COMMIT;
    if (wchunk < ta.t.n) {
        const bool full = wchunk + kWaveGroups <= ta.t.n && ta.vec_ok;
        SubTile<F> st;
        if (full) {
            load_sub<F, true, NT>(ta, wchunk + 2 * lane, commit_mode, st);
            compute_store_sub<F, true, RANK, NTS>(ta, wchunk, commit_mode, st, bits);
        } else {
            load_sub<F, false>(ta, wchunk + 2 * lane, commit_mode, st);
            compute_store_sub<F, false, RANK>(ta, wchunk, commit_mode, st, bits);
        }
    }
    if (RH_COMMIT_BITS_DIRECT || BLOCK != 256 || (!ta.t.valid_bits && !ta.t.advanced_bits)) return;  // block-uniform
    __syncthreads();
    if (threadIdx.x < 16) {
        const int col = threadIdx.x >> 3, k = threadIdx.x & 7;
        uint64_t* dst = col ? ta.t.advanced_bits : ta.t.valid_bits;
        const uint64_t word = tile * 8 + (uint64_t)k;
        if (dst && word < ((ta.t.n + 63) >> 6)) dst[word] = bits[col][k];
    }
}

template <int F, int FHI, bool RANK, bool NT, bool NTS, int BLOCK>
__device__ __forceinline__ void dispatch_f(const TierArgs& ta, uint64_t tile) {
    if (ta.t.n_followers == F)
        run_tile<F, RANK, NT, NTS, BLOCK>(ta, tile);
    else if constexpr (F < FHI)
        dispatch_f<F + 1, FHI, RANK, NT, NTS, BLOCK>(ta, tile);
}

__device__ __forceinline__ int tier_of_block(const LaunchArgs& args, uint32_t b) {
    int ti = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < (int)args.n_tiers && b >= args.begin[i]) ti = i;
    return ti;
}

// Tiers with F <= 6: rank-mask order statistics (no sorted copies), non-temporal loads and
// stores (every byte is touched once), and the register budget pinned to 64 VGPRs so 8 waves fit
// per SIMD: a 1M-group launch (7813 waves of 128 groups) is resident in one round on 256 CUs.
// One launch covers every tier of the class; blocks are assigned to tiers in order and the F
// switch is block-uniform, so it costs no divergence.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(RH_COMMIT_WAVES, 8))) void commit_kernel_rank(
    const LaunchArgs a) {
    const LaunchArgs& args = rh::kernarg_struct<LaunchArgs>();  // scalar loads, no scratch copy
    const int ti = tier_of_block(args, blockIdx.x);
    const TierArgs& ta = args.tier[ti];
    uint32_t j = blockIdx.x - ta.block_begin;
#if RH_COMMIT_XCD   // A/B: each XCD (blocks dealt round robin) streams one contiguous eighth of the tier
    {
        const uint32_t n = ta.n_blocks, x = j % 8u, q = n / 8u, r = n % 8u;
        j = x * q + (x < r ? x : r) + j / 8u;
    }
#endif
    dispatch_f<1, 6, true, true, RH_COMMIT_NTS, kBlock>(ta, (uint64_t)j);
}

// Tiers with F = 7..14 (8..15 voters): a Batcher network per conf (rank masks of 8+ values do
// not stay in registers).
__global__ __launch_bounds__(kBlock) void commit_kernel_net(const LaunchArgs a) {
    const LaunchArgs& args = rh::kernarg_struct<LaunchArgs>();
    const int ti = tier_of_block(args, blockIdx.x);
    const TierArgs& ta = args.tier[ti];
    dispatch_f<7, 14, false, false, false, kBlock>(ta, (uint64_t)(blockIdx.x - ta.block_begin));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Kernel arguments for the tiers whose F lies in [flo, fhi].  Blocks go to the widest tiers first:
// a joint-consensus tier (two confs, 7 voters) costs several times a stable tier's compute per
// group, and its blocks dispatched last were the launch's tail (config 3: 17.2 -> 16.1 us).
void build_args(const rh_commit_soa* tiers, int n_tiers, int flo, int fhi, LaunchArgs& args, uint64_t& blocks,
                int block = kBlock) {
    const uint64_t kTile = (uint64_t)block * kGroupsPerLane;  // groups per workgroup
    args = LaunchArgs{};
    blocks = 0;
    int order[RH_MAX_TIERS];
    for (int i = 0; i < n_tiers; ++i) order[i] = i;
    for (int i = 1; i < n_tiers; ++i)  // stable insertion sort by descending width
        for (int j = i; j > 0 && tiers[order[j]].n_followers > tiers[order[j - 1]].n_followers; --j) {
            const int x = order[j];
            order[j] = order[j - 1];
            order[j - 1] = x;
        }
    for (int oi = 0; oi < n_tiers; ++oi) {
        const rh_commit_soa& t = tiers[order[oi]];
        if ((int)t.n_followers < flo || (int)t.n_followers > fhi || t.n == 0) continue;
        TierArgs& ta = args.tier[args.n_tiers++];
        ta.t = t;
        ta.stride = t.col_stride ? t.col_stride : t.n;
        ta.tile64 = t.tile_stride / 8;
        ta.tile32 = t.tile_stride / 4;
        ta.block_begin = (uint32_t)blocks;
        args.begin[args.n_tiers - 1] = (uint32_t)blocks;
        ta.n_blocks = (uint32_t)((t.n + kTile - 1) / kTile);
        const bool cm = t.mode == RH_MODE_COMMIT;
        ta.vec_ok = aligned16(t.follower_index) && (ta.stride % 2 == 0) && aligned16(t.self_index) &&
                    (reinterpret_cast<uintptr_t>(t.conf) & 7u) == 0 &&
                    (!cm || (aligned16(t.commit_in) && aligned16(t.term_start) && aligned16(t.commit_out))) &&
                    (!t.min_out || aligned16(t.min_out)) && (!t.maj_out || aligned16(t.maj_out)) &&
                    (!t.max_out || aligned16(t.max_out));
        blocks += ta.n_blocks;
    }
}

// One launch over the tiers whose F lies in [flo, fhi].
int launch_class(const rh_commit_soa* tiers, int n_tiers, int flo, int fhi, hipStream_t stream) {
    LaunchArgs args;
    uint64_t blocks = 0;
    build_args(tiers, n_tiers, flo, fhi, args, blocks);
    if (args.n_tiers == 0) return RH_OK;
    if (blocks > 0x7FFFFFFFull) return rh::fail(RH_E_RANGE, "commit launch: too many groups");
    const dim3 g((uint32_t)blocks), b(kBlock);
    if (flo == 1)
        hipLaunchKernelGGL(commit_kernel_rank, g, b, 0, stream, args);
    else
        hipLaunchKernelGGL(commit_kernel_net, g, b, 0, stream, args);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

// ---- fused commit + lease launch (rh_leader_soa_launch) -------------------------------------------
// The leader's per-heartbeat bookkeeping of every division in ONE launch: blocks [0, commit_blocks)
// run updateCommit over the commit tiers (as commit_kernel_rank), the rest hasLease over the lease
// tiers (as lease_kernel<0, 7>).  One launch ramp and tail instead of two; both halves fit the
// same 64-VGPR / 8-waves-per-SIMD budget.
struct LeaderArgs {
    LaunchArgs commit;
    rh_lease::LeaseLaunch lease;
    uint32_t commit_blocks;
};

__global__ __launch_bounds__(kLeaderBlock) __attribute__((amdgpu_waves_per_eu(RH_COMMIT_WAVES, 8))) void leader_kernel(const LeaderArgs arg) {
    const LeaderArgs& a = rh::kernarg_struct<LeaderArgs>();
    const uint32_t b = blockIdx.x;
    if (b < a.commit_blocks) {
        const int ti = tier_of_block(a.commit, b);
        const TierArgs& ta = a.commit.tier[ti];
        dispatch_f<1, 6, true, true, RH_COMMIT_NTS, kLeaderBlock>(ta, (uint64_t)(b - ta.block_begin));
    } else {
        rh_lease::lease_block(a.lease, (uint64_t)(b - a.commit_blocks));
    }
}

int validate(const rh_commit_soa* tiers, int n_tiers) {
    if (!tiers || n_tiers < 1 || n_tiers > RH_MAX_TIERS)
        return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: n_tiers must be in [1, RH_MAX_TIERS]");
    for (int i = 0; i < n_tiers; ++i) {
        const rh_commit_soa& t = tiers[i];
        if (t.n_followers < 1 || t.n_followers > RH_MAX_FOLLOWERS)
            return rh::fail(RH_E_RANGE, "rh_commit_soa_launch: n_followers must be in [1, 14]");
        if (t.mode != RH_MODE_COMMIT && t.mode != RH_MODE_WATCH)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: unknown mode");
        if (t.n == 0) continue;
        if (!t.follower_index || !t.self_index || !t.conf)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: follower_index/self_index/conf required");
        if (t.tile_stride == 0 && t.col_stride != 0 && t.col_stride < t.n)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: col_stride < n");
        if (t.tile_stride != 0 && (t.tile_stride % 16 != 0 || t.col_stride < RH_TILE_GROUPS ||
                                   t.tile_stride < 8ull * RH_TILE_GROUPS))
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: tiled layout needs tile_stride % 16 == 0, "
                                        "tile_stride >= 1024 and col_stride >= 128");
        if (t.mode == RH_MODE_COMMIT && (!t.commit_in || !t.term_start || !t.commit_out))
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: COMMIT needs commit_in, term_start, commit_out");
        if (t.mode == RH_MODE_COMMIT && t.gap_threshold < -1)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: gap_threshold must be -1 or >= 0");
        if (t.adv_rows && (!t.adv_commit || !t.adv_count))
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: adv_rows needs adv_commit and adv_count");
    }
    return RH_OK;
}

}  // namespace

int rh_commit_launch_impl(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, hipStream_t stream) {
    (void)ctx;
    int rc = validate(tiers, n_tiers);
    if (rc == RH_OK) rc = launch_class(tiers, n_tiers, 1, 6, stream);
    return rc != RH_OK ? rc : launch_class(tiers, n_tiers, 7, 14, stream);
}

int rh_leader_launch_impl(rh_ctx* ctx, const rh_commit_soa* commit, int n_commit, const rh_lease_soa* lease,
                          int n_lease, hipStream_t stream) {
    (void)ctx;
    int rc = validate(commit, n_commit);
    if (rc == RH_OK) rc = rh_lease_validate(lease, n_lease);
    if (rc != RH_OK) return rc;
    LeaderArgs a;
    uint64_t cb = 0, lb = 0;
    build_args(commit, n_commit, 1, 6, a.commit, cb, kLeaderBlock);
    rh_lease::build_lease_args(lease, n_lease, 0, 7, a.lease, lb);
    if (cb + lb > 0x7FFFFFFFull) return rh::fail(RH_E_RANGE, "rh_leader_soa_launch: too many groups");
    a.commit_blocks = (uint32_t)cb;
    if (cb + lb) {
        hipLaunchKernelGGL(leader_kernel, dim3((uint32_t)(cb + lb)), dim3(kLeaderBlock), 0, stream, a);
        RH_HIP(hipGetLastError());
    }
    // tiers outside the fused kernel's classes: their own launches (same stream, same results)
    rc = launch_class(commit, n_commit, 7, 14, stream);
    return rc != RH_OK ? rc : rh_lease_launch_class(lease, n_lease, 8, 14, stream);
}
