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
// Layout: one struct-of-arrays "tier" per follower-slot count F.  Every column is a contiguous
// int64 array over the tier's groups, so a wave's loads of one column are one coalesced
// 1 KiB request (2 groups per lane, 16 B per lane).  The k-th order statistic over <= F+1
// voters is a Batcher merge-exchange network in registers with non-voters padded to
// INT64_MAX -- integer compare/select work, no MFMA (this is not a contraction).  The kernel
// is HBM-bound: 8(F+1)+20 bytes read and 16 bytes written per group.
#include "rh_internal.h"
#include "sortnet.h"

#include <climits>

namespace {

constexpr int kBlock = 256;            // 4 waves
constexpr int kGroupsPerLane = 2;      // 16-byte loads per column per lane
// Launch variant (identical results; scripts/microbench.py A/B).  Default 14: rank-mask
// selection at 8 waves/SIMD with non-temporal loads and stores (fastest measured).
int g_commit_variant = 14;
constexpr int kVariantT[] = {1, 2, 4};
// 0-2: v1 with T = 1, 2, 4 sub-tiles per wave (F classes [1,7] and [8,14])
// 3:   v1, T = 1, F classes [1,4], [5,7], [8,14] (narrower register allocation)
// 4-6: v2 persistent + prefetch, F classes [1,4], [5,7], [8,14]; 3/4/5 waves per SIMD
// 7:   v2, F classes [1,7], [8,14], 4 waves per SIMD
// 8:   v3 rank-mask selection, 64-VGPR budget (8 waves/SIMD), F classes [1,6], [7,14]
// 9:   v3 rank-mask selection, unpinned budget, F classes [1,7], [8,14]
// 10/11: v3 (8) with 512 / 1024-thread workgroups (fewer dispatches)
// 12/13: v3 (8) with non-temporal loads, 256 / 512-thread workgroups
// 14:    v3 (12) with non-temporal stores as well
// 15:    v1 (0) with non-temporal loads
constexpr int kNumCommitVariants = 16;

// Order statistics of the voters selected by `member` (bit i = slot i, bit N-1 = self):
// getSorted (LSI:1076-1095) + MinMajorityMax.valueOf(sorted, gap) (LSI:926-943).
// Non-members sort to the end as INT64_MAX; k < n so they are never selected.
template <int N>
__device__ __forceinline__ void order_stats(const int64_t (&vals)[N], uint32_t member, int64_t gap,
                                            int64_t& mn, int64_t& mj, int64_t& mx) {
    int64_t s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = ((member >> i) & 1u) ? vals[i] : INT64_MAX;
    rh_sort::sort_net<N>(s);
    const int n = __builtin_popcount(member);
    const int k = (n - 1) >> 1;  // getMajority: sorted[(length - 1) / 2]
    mn = s[0];
    mj = s[0];
    mx = s[0];
#pragma unroll
    for (int j = 1; j < N; ++j) {
        mj = (j == k) ? s[j] : mj;
        mx = (j == n - 1) ? s[j] : mx;
    }
    // gapThreshold clamp; Java long subtraction wraps (LSI:929-933).
    if (gap != -1 && (int64_t)((uint64_t)mj - (uint64_t)mn) > gap) mj = mn;
}

// Same result as order_stats, from rank masks shared by the new and the old conf.
template <int N>
__device__ __forceinline__ void order_stats_rank(const int64_t (&vals)[N], const uint32_t (&less)[N],
                                                 uint32_t member, int64_t gap, int64_t& mn, int64_t& mj,
                                                 int64_t& mx) {
    const int n = __builtin_popcount(member);
    rh_sort::select_ranks<N>(vals, less, member, (n - 1) >> 1, n, mn, mj, mx);
    if (gap != -1 && (int64_t)((uint64_t)mj - (uint64_t)mn) > gap) mj = mn;
}

struct TierArgs {
    rh_commit_soa t;
    uint64_t stride;        // elements between follower columns
    uint32_t block_begin;   // first block of this tier in the launch
    uint32_t n_blocks;
    bool vec_ok;            // every column 16-byte aligned: full tiles use 16-byte loads
};

struct LaunchArgs {
    TierArgs tier[RH_MAX_TIERS];
    int n_tiers;
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
#pragma unroll
        for (int k = 0; k < F; ++k) {
            const v2i64 x = ld16<NT, v2i64>(t.follower_index + (uint64_t)k * ta.stride + r0);
            st.fv[0][k] = x.x;
            st.fv[1][k] = x.y;
        }
        const v2i64 s = ld16<NT, v2i64>(t.self_index + r0);
        st.self[0] = s.x;
        st.self[1] = s.y;
        const v2u32 c = NT ? __builtin_nontemporal_load(reinterpret_cast<const v2u32*>(t.conf + r0))
                           : *reinterpret_cast<const v2u32*>(t.conf + r0);
        st.w[0] = c.x;
        st.w[1] = c.y;
        if (commit_mode) {
            const v2i64 ci = ld16<NT, v2i64>(t.commit_in + r0);
            const v2i64 ts = ld16<NT, v2i64>(t.term_start + r0);
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
#pragma unroll
            for (int k = 0; k < F; ++k) st.fv[g][k] = in ? t.follower_index[(uint64_t)k * ta.stride + r] : 0;
            st.self[g] = in ? t.self_index[r] : 0;
            st.w[g] = in ? t.conf[r] : 0u;  // rows past n: inactive padding
            st.cin[g] = (in && commit_mode) ? t.commit_in[r] : 0;
            st.tstart[g] = (in && commit_mode) ? t.term_start[r] : 0;
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
                                                  const SubTile<F>& st) {
    constexpr int N = F + 1;
    const rh_commit_soa& t = ta.t;
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = wbase + 2 * (uint64_t)lane;

    // ---- getMajorityMin (LSI:956-984) ----
    const int64_t gap = commit_mode ? t.gap_threshold : -1;  // 2-arg overload passes -1 (LSI:952-954)
    bool valid[2], adv[2];
    int64_t mn[2], mj[2], mx[2], cout[2];
    const uint32_t fmask = (1u << F) - 1u;
    bool trans[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) trans[g] = (st.w[g] & RH_CONF_ACTIVE) && (st.w[g] & RH_CONF_TRANSITIONAL);
    const bool any_trans = __any(trans[0] || trans[1]);

#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const uint32_t w = st.w[g];
        int64_t vals[N];
#pragma unroll
        for (int k = 0; k < F; ++k) vals[k] = st.fv[g][k];
        vals[F] = st.self[g];
        const uint32_t mnew = (w & fmask) | (((w >> 14) & 1u) << F);
        const uint32_t mold = ((w >> RH_CONF_OLD_SHIFT) & fmask) | (((w >> 30) & 1u) << F);
        // followers.isEmpty() && !includeSelf -> Optional.empty()  (LSI:964-966, 976-978)
        const bool v = (w & RH_CONF_ACTIVE) && mnew != 0 && (!trans[g] || mold != 0);
        int64_t a0, a1, a2;
        if (RANK) {
            uint32_t less[N];
            rh_sort::rank_masks<N>(vals, less);
            order_stats_rank<N>(vals, less, mnew ? mnew : 1u, gap, a0, a1, a2);
            if (any_trans) {
                if (trans[g]) {  // combine(): element-wise min (LSI:915-920)
                    int64_t b0, b1, b2;
                    order_stats_rank<N>(vals, less, mold ? mold : 1u, gap, b0, b1, b2);
                    a0 = b0 < a0 ? b0 : a0;
                    a1 = b1 < a1 ? b1 : a1;
                    a2 = b2 < a2 ? b2 : a2;
                }
            }
        } else {
            order_stats<N>(vals, mnew ? mnew : 1u, gap, a0, a1, a2);
            if (any_trans) {
                if (trans[g]) {  // combine(): element-wise min (LSI:915-920)
                    int64_t b0, b1, b2;
                    order_stats<N>(vals, mold ? mold : 1u, gap, b0, b1, b2);
                    a0 = b0 < a0 ? b0 : a0;
                    a1 = b1 < a1 ? b1 : a1;
                    a2 = b2 < a2 ? b2 : a2;
                }
            }
        }
        valid[g] = v;
        mn[g] = v ? a0 : INT64_MIN;
        mj[g] = v ? a1 : INT64_MIN;
        mx[g] = v ? a2 : INT64_MIN;
        // ---- updateCommit(majority, min) (LSI:1015-1026) -> RaftLogBase.updateCommitIndex ----
        // old = lastCommitted; if (majority > old) { newCommit = min(majority, flushIndex);
        //   if (old < newCommit && termAt(newCommit) == currentTerm) commit = newCommit; }
        const int64_t old = st.cin[g];
        const int64_t flush = st.self[g];
        const int64_t nc = a1 < flush ? a1 : flush;
        const bool a = commit_mode && v && a1 > old && old < nc && nc >= st.tstart[g];
        adv[g] = a;
        cout[g] = a ? nc : old;
    }

    // ---- stores ----
    if (VEC) {
        if (commit_mode) st16<NTS>(t.commit_out + r0, cout[0], cout[1]);
        if (t.min_out) st16<NTS>(t.min_out + r0, mn[0], mn[1]);
        if (t.maj_out) st16<NTS>(t.maj_out + r0, mj[0], mj[1]);
        if (t.max_out) st16<NTS>(t.max_out + r0, mx[0], mx[1]);
    } else {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const uint64_t r = r0 + g;
            if (r < t.n) {
                if (commit_mode) t.commit_out[r] = cout[g];
                if (t.min_out) t.min_out[r] = mn[g];
                if (t.maj_out) t.maj_out[r] = mj[g];
                if (t.max_out) t.max_out[r] = mx[g];
            }
        }
    }

    // ---- per-wave bit words: bit j of word (wbase/64 + h) is row wbase + 64h + j ----
    const uint64_t ve = __ballot(valid[0]), vo = __ballot(valid[1]);
    const uint64_t ae = __ballot(adv[0]), ao = __ballot(adv[1]);
    if (wbase < t.n) {
        // ballots are wave-uniform: interleave them on the scalar unit, then lanes 0/1 store
        const uint64_t word = wbase >> 6;
        const uint64_t nwords = (t.n + 63) >> 6;
        if (t.valid_bits) {
            const uint64_t w0 = spread32(ve) | (spread32(vo) << 1);
            const uint64_t w1 = spread32(ve >> 32) | (spread32(vo >> 32) << 1);
            if (lane < 2 && word + lane < nwords) t.valid_bits[word + lane] = lane ? w1 : w0;
        }
        if (t.advanced_bits) {
            const uint64_t w0 = spread32(ae) | (spread32(ao) << 1);
            const uint64_t w1 = spread32(ae >> 32) | (spread32(ao >> 32) << 1);
            if (lane < 2 && word + lane < nwords) t.advanced_bits[word + lane] = lane ? w1 : w0;
        }
    }

    // ---- compacted advanced list: one atomic per wave ----
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

// One workgroup tile = 4 waves x T sub-tiles of 128 groups.  All T sub-tiles' loads are
// issued before any compute, so a wave keeps T x (F+3) x 1 KiB in flight.
template <int F, int T, bool RANK = false, int BLK = kBlock, bool NT = false, bool NTS = false>
__device__ __forceinline__ void run_tile(const TierArgs& ta, uint64_t tile) {
    constexpr uint64_t kWaveGroups = 128ull * T;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t wchunk = tile * (kWaveGroups * (BLK / 64)) + (uint64_t)wave * kWaveGroups;
    const bool commit_mode = ta.t.mode == RH_MODE_COMMIT;
    if (wchunk >= ta.t.n) return;
    const bool full = wchunk + kWaveGroups <= ta.t.n && ta.vec_ok;
    SubTile<F> st[T];
    if (full) {
#pragma unroll
        for (int s = 0; s < T; ++s) load_sub<F, true, NT>(ta, wchunk + 128 * s + 2 * lane, commit_mode, st[s]);
#pragma unroll
        for (int s = 0; s < T; ++s) compute_store_sub<F, true, RANK, NTS>(ta, wchunk + 128 * s, commit_mode, st[s]);
    } else {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            load_sub<F, false>(ta, wchunk + 128 * s + 2 * lane, commit_mode, st[s]);
            compute_store_sub<F, false, RANK>(ta, wchunk + 128 * s, commit_mode, st[s]);
        }
    }
}


// ---- v2: persistent waves, software-pipelined over 128-group units -------------------------
// Each wave walks units u = wave, wave + nwaves, ... over all tiers of the launch and issues the
// loads of its next unit before computing the current one, so the HBM stream of the next unit
// overlaps the sorting-network work of this one (v1 runs ~1.5 "rounds" of waves with no such
// overlap).  A unit never crosses a tier, so F is wave-uniform per unit.
template <int F>
__device__ __forceinline__ void unit_load(const TierArgs& ta, uint64_t ubase, bool commit_mode, bool full,
                                          SubTile<F>& st) {
    const uint64_t r0 = ubase + 2 * (uint64_t)(threadIdx.x & 63);
    if (full)
        load_sub<F, true>(ta, r0, commit_mode, st);
    else
        load_sub<F, false>(ta, r0, commit_mode, st);
}

template <int F>
__device__ __forceinline__ void unit_compute(const TierArgs& ta, uint64_t ubase, bool commit_mode, bool full,
                                             const SubTile<F>& st) {
    if (full)
        compute_store_sub<F, true>(ta, ubase, commit_mode, st);
    else
        compute_store_sub<F, false>(ta, ubase, commit_mode, st);
}

struct UnitRef {
    int tier;
    uint64_t base;  // first row of the unit in its tier
    bool valid;
};

__device__ __forceinline__ UnitRef unit_ref(const LaunchArgs& args, uint64_t u) {
    UnitRef r{0, 0, false};
#pragma unroll
    for (int i = 0; i < RH_MAX_TIERS; ++i) {
        if (i < args.n_tiers) {
            const uint64_t nu = (uint64_t)args.tier[i].n_blocks;  // here: units (128 groups) of tier i
            if (!r.valid && u < nu) {
                r.tier = i;
                r.base = u * 128;
                r.valid = true;
            }
            if (!r.valid) u -= nu;
        }
    }
    return r;
}

template <int F>
__device__ __forceinline__ void run_units(const LaunchArgs& args, uint64_t u0, uint64_t stride, uint64_t n_units) {
    // all units of this wave have the same F only if the launch holds one F; otherwise units of
    // other widths are skipped here and handled by their own dispatch_f2 instantiation.
    SubTile<F> cur, nxt;
    uint64_t u = u0;
    // find first unit of width F
    auto next_of_width = [&](uint64_t from) -> uint64_t {
        for (uint64_t v = from; v < n_units; v += stride) {
            const UnitRef r = unit_ref(args, v);
            if ((int)args.tier[r.tier].t.n_followers == F) return v;
        }
        return n_units;
    };
    u = next_of_width(u);
    if (u >= n_units) return;
    UnitRef rc = unit_ref(args, u);
    bool cfull = rc.base + 128 <= args.tier[rc.tier].t.n && args.tier[rc.tier].vec_ok;
    bool ccm = args.tier[rc.tier].t.mode == RH_MODE_COMMIT;
    unit_load<F>(args.tier[rc.tier], rc.base, ccm, cfull, cur);
    while (true) {
        const uint64_t un = next_of_width(u + stride);
        UnitRef rn{0, 0, false};
        bool nfull = false, ncm = false;
        if (un < n_units) {
            rn = unit_ref(args, un);
            nfull = rn.base + 128 <= args.tier[rn.tier].t.n && args.tier[rn.tier].vec_ok;
            ncm = args.tier[rn.tier].t.mode == RH_MODE_COMMIT;
            unit_load<F>(args.tier[rn.tier], rn.base, ncm, nfull, nxt);
        }
        unit_compute<F>(args.tier[rc.tier], rc.base, ccm, cfull, cur);
        if (un >= n_units) break;
        u = un;
        rc = rn;
        cfull = nfull;
        ccm = ncm;
        cur = nxt;
    }
}

template <int F, int FHI>
__device__ __forceinline__ void dispatch_f2(const LaunchArgs& args, uint32_t fmask, uint64_t u0, uint64_t stride,
                                            uint64_t n_units) {
    if (fmask & (1u << F)) run_units<F>(args, u0, stride, n_units);
    if constexpr (F < FHI) dispatch_f2<F + 1, FHI>(args, fmask, u0, stride, n_units);
}

template <int FLO, int FHI>
__global__ __launch_bounds__(kBlock) void commit_kernel_v2(const LaunchArgs args, uint32_t fmask, uint64_t n_units) {
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t stride = (uint64_t)gridDim.x * (kBlock / 64);
    dispatch_f2<FLO, FHI>(args, fmask, wave, stride, n_units);
}

}  // namespace

namespace {

template <int F, int FHI, int T, bool RANK = false, int BLK = kBlock, bool NT = false, bool NTS = false>
__device__ __forceinline__ void dispatch_f(const TierArgs& ta, uint64_t tile) {
    if (ta.t.n_followers == F)
        run_tile<F, T, RANK, BLK, NT, NTS>(ta, tile);
    else if constexpr (F < FHI)
        dispatch_f<F + 1, FHI, T, RANK, BLK, NT, NTS>(ta, tile);
}

// One launch evaluates every tier whose F lies in [FLO, FHI]; blocks are assigned to tiers
// in order.  The F switch is block-uniform, so it costs no divergence.
template <int FLO, int FHI, int T>
__global__ __launch_bounds__(kBlock) void commit_kernel(const LaunchArgs args) {
    const uint32_t b = blockIdx.x;
    int ti = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < args.n_tiers && b >= args.tier[i].block_begin) ti = i;
    const TierArgs& ta = args.tier[ti];
    dispatch_f<FLO, FHI, T>(ta, (uint64_t)(b - ta.block_begin));
}

// v3: rank-mask order statistics (no sorted copies) with the register budget pinned to 64
// VGPRs, so 8 waves fit per SIMD: a 1M-group launch (7813 waves of 128 groups) is resident in
// one round on 256 CUs instead of ~1.5 rounds at 5 waves/SIMD.
template <int FLO, int FHI, int BLK = kBlock, bool NT = false, bool NTS = false>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(8, 8))) void commit_kernel_r8(
    const LaunchArgs args) {
    const uint32_t b = blockIdx.x;
    int ti = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < args.n_tiers && b >= args.tier[i].block_begin) ti = i;
    const TierArgs& ta = args.tier[ti];
    dispatch_f<FLO, FHI, 1, true, BLK, NT, NTS>(ta, (uint64_t)(b - ta.block_begin));
}

// v1 (sorting network, T = 1) with non-temporal loads.
template <int FLO, int FHI>
__global__ __launch_bounds__(kBlock) void commit_kernel_nt(const LaunchArgs args) {
    const uint32_t b = blockIdx.x;
    int ti = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < args.n_tiers && b >= args.tier[i].block_begin) ti = i;
    const TierArgs& ta = args.tier[ti];
    dispatch_f<FLO, FHI, 1, false, kBlock, true>(ta, (uint64_t)(b - ta.block_begin));
}

template <int FLO, int FHI>
__global__ __launch_bounds__(kBlock) void commit_kernel_r(const LaunchArgs args) {
    const uint32_t b = blockIdx.x;
    int ti = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < args.n_tiers && b >= args.tier[i].block_begin) ti = i;
    const TierArgs& ta = args.tier[ti];
    dispatch_f<FLO, FHI, 1, true>(ta, (uint64_t)(b - ta.block_begin));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <int FLO, int FHI>
void launch_t(int T, uint32_t blocks, const LaunchArgs& args, hipStream_t stream) {
    switch (T) {
        case 1: hipLaunchKernelGGL((commit_kernel<FLO, FHI, 1>), dim3(blocks), dim3(kBlock), 0, stream, args); break;
        case 2: hipLaunchKernelGGL((commit_kernel<FLO, FHI, 2>), dim3(blocks), dim3(kBlock), 0, stream, args); break;
        default: hipLaunchKernelGGL((commit_kernel<FLO, FHI, 4>), dim3(blocks), dim3(kBlock), 0, stream, args); break;
    }
}

int g_num_cus = 256;

// v2 launch over the tiers whose F lies in [flo, fhi]: n_blocks holds units of 128 groups.
int launch_class_v2(const rh_commit_soa* tiers, int n_tiers, int flo, int fhi, int waves_per_simd,
                    hipStream_t stream) {
    LaunchArgs args{};
    uint64_t units = 0;
    uint32_t fmask = 0;
    for (int i = 0; i < n_tiers; ++i) {
        const rh_commit_soa& t = tiers[i];
        if ((int)t.n_followers < flo || (int)t.n_followers > fhi || t.n == 0) continue;
        TierArgs& ta = args.tier[args.n_tiers++];
        ta.t = t;
        ta.stride = t.col_stride ? t.col_stride : t.n;
        ta.block_begin = 0;
        ta.n_blocks = (uint32_t)((t.n + 127) / 128);
        const bool cm = t.mode == RH_MODE_COMMIT;
        ta.vec_ok = aligned16(t.follower_index) && (ta.stride % 2 == 0) && aligned16(t.self_index) &&
                    (reinterpret_cast<uintptr_t>(t.conf) & 7u) == 0 &&
                    (!cm || (aligned16(t.commit_in) && aligned16(t.term_start) && aligned16(t.commit_out))) &&
                    (!t.min_out || aligned16(t.min_out)) && (!t.maj_out || aligned16(t.maj_out)) &&
                    (!t.max_out || aligned16(t.max_out));
        units += ta.n_blocks;
        fmask |= 1u << t.n_followers;
    }
    if (args.n_tiers == 0) return RH_OK;
    uint64_t waves = (uint64_t)g_num_cus * 4 * waves_per_simd;
    if (waves > units) waves = units;
    const uint32_t blocks = (uint32_t)((waves + 3) / 4);
    if (flo == 1 && fhi == 4)
        hipLaunchKernelGGL((commit_kernel_v2<1, 4>), dim3(blocks), dim3(kBlock), 0, stream, args, fmask, units);
    else if (flo == 5 && fhi == 7)
        hipLaunchKernelGGL((commit_kernel_v2<5, 7>), dim3(blocks), dim3(kBlock), 0, stream, args, fmask, units);
    else if (flo == 1 && fhi == 7)
        hipLaunchKernelGGL((commit_kernel_v2<1, 7>), dim3(blocks), dim3(kBlock), 0, stream, args, fmask, units);
    else
        hipLaunchKernelGGL((commit_kernel_v2<8, 14>), dim3(blocks), dim3(kBlock), 0, stream, args, fmask, units);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int launch_class(const rh_commit_soa* tiers, int n_tiers, int flo, int fhi, int variant, hipStream_t stream) {
    const int T = kVariantT[variant < 3 ? variant : 0];
    const int blk = (variant == 10 || variant == 13) ? 512 : variant == 11 ? 1024 : kBlock;
    const uint64_t kTile = (uint64_t)(flo == 1 ? blk : kBlock) * kGroupsPerLane * T;  // groups per workgroup
    LaunchArgs args{};
    uint64_t blocks = 0;
    for (int i = 0; i < n_tiers; ++i) {
        const rh_commit_soa& t = tiers[i];
        if ((int)t.n_followers < flo || (int)t.n_followers > fhi || t.n == 0) continue;
        TierArgs& ta = args.tier[args.n_tiers++];
        ta.t = t;
        ta.stride = t.col_stride ? t.col_stride : t.n;
        ta.block_begin = (uint32_t)blocks;
        ta.n_blocks = (uint32_t)((t.n + kTile - 1) / kTile);
        const bool cm = t.mode == RH_MODE_COMMIT;
        ta.vec_ok = aligned16(t.follower_index) && (ta.stride % 2 == 0) && aligned16(t.self_index) &&
                    (reinterpret_cast<uintptr_t>(t.conf) & 7u) == 0 &&
                    (!cm || (aligned16(t.commit_in) && aligned16(t.term_start) && aligned16(t.commit_out))) &&
                    (!t.min_out || aligned16(t.min_out)) && (!t.maj_out || aligned16(t.maj_out)) &&
                    (!t.max_out || aligned16(t.max_out));
        blocks += ta.n_blocks;
    }
    if (args.n_tiers == 0) return RH_OK;
    if (blocks > 0x7FFFFFFFull) return rh::fail(RH_E_RANGE, "commit launch: too many groups");
    if (variant >= 8 && flo == 1) {  // rank-mask selection, T = 1
        const dim3 g((uint32_t)blocks), b(blk);
        if (variant == 10)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6, 512>), g, b, 0, stream, args);
        else if (variant == 11)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6, 1024>), g, b, 0, stream, args);
        else if (variant == 12)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6, 256, true>), g, b, 0, stream, args);
        else if (variant == 13)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6, 512, true>), g, b, 0, stream, args);
        else if (variant == 14)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6, 256, true, true>), g, b, 0, stream, args);
        else if (variant == 15)
            hipLaunchKernelGGL((commit_kernel_nt<1, 7>), g, b, 0, stream, args);
        else if (fhi == 6)
            hipLaunchKernelGGL((commit_kernel_r8<1, 6>), g, b, 0, stream, args);
        else
            hipLaunchKernelGGL((commit_kernel_r<1, 7>), g, b, 0, stream, args);
    } else if (flo == 7)  // wide tiers: sorting network (rank masks of 8+ values would not unroll)
        launch_t<7, 14>(T, (uint32_t)blocks, args, stream);
    else if (flo == 1 && fhi == 4)
        launch_t<1, 4>(T, (uint32_t)blocks, args, stream);
    else if (flo == 5 && fhi == 7)
        launch_t<5, 7>(T, (uint32_t)blocks, args, stream);
    else if (fhi <= 7)
        launch_t<1, 7>(T, (uint32_t)blocks, args, stream);
    else
        launch_t<8, 14>(T, (uint32_t)blocks, args, stream);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

}  // namespace

int rh_commit_set_variant_impl(int v) {
    if (v < 0 || v >= kNumCommitVariants) return rh::fail(RH_E_INVAL, "unknown commit kernel variant");
    g_commit_variant = v;
    return RH_OK;
}

int rh_commit_num_variants_impl() { return kNumCommitVariants; }

int rh_commit_launch_impl(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, hipStream_t stream) {
    if (ctx && ctx->num_cus > 0) g_num_cus = ctx->num_cus;
    const int variant = g_commit_variant;
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
        if (t.col_stride != 0 && t.col_stride < t.n)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: col_stride < n");
        if (t.mode == RH_MODE_COMMIT && (!t.commit_in || !t.term_start || !t.commit_out))
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: COMMIT needs commit_in, term_start, commit_out");
        if (t.mode == RH_MODE_COMMIT && t.gap_threshold < -1)
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: gap_threshold must be -1 or >= 0");
        if (t.adv_rows && (!t.adv_commit || !t.adv_count))
            return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: adv_rows needs adv_commit and adv_count");
    }
    int rc = RH_OK;
    if (variant == 15) {
        rc = launch_class(tiers, n_tiers, 1, 7, variant, stream);
        return rc != RH_OK ? rc : launch_class(tiers, n_tiers, 8, 14, variant, stream);
    }
    if (variant == 8 || variant >= 10) {
        rc = launch_class(tiers, n_tiers, 1, 6, variant, stream);
        return rc != RH_OK ? rc : launch_class(tiers, n_tiers, 7, 14, variant, stream);
    }
    if (variant == 9) {
        rc = launch_class(tiers, n_tiers, 1, 7, variant, stream);
        return rc != RH_OK ? rc : launch_class(tiers, n_tiers, 8, 14, variant, stream);
    }
    if (variant <= 2) {
        rc = launch_class(tiers, n_tiers, 1, 7, variant, stream);
    } else if (variant == 3) {
        rc = launch_class(tiers, n_tiers, 1, 4, variant, stream);
        if (rc == RH_OK) rc = launch_class(tiers, n_tiers, 5, 7, variant, stream);
    } else if (variant <= 6) {
        rc = launch_class_v2(tiers, n_tiers, 1, 4, variant - 1, stream);
        if (rc == RH_OK) rc = launch_class_v2(tiers, n_tiers, 5, 7, variant - 1, stream);
    } else {
        rc = launch_class_v2(tiers, n_tiers, 1, 7, 4, stream);
    }
    if (rc != RH_OK) return rc;
    if (variant <= 3) return launch_class(tiers, n_tiers, 8, 14, variant, stream);
    return launch_class_v2(tiers, n_tiers, 8, 14, 4, stream);
}

// ---- delta application: RaftLogIndex.updateToMax per (slot, column) ----------------------
namespace {

__global__ __launch_bounds__(256) void apply_deltas_kernel(const rh_delta* __restrict__ d, uint64_t n,
                                                           uint64_t capacity, uint64_t stride,
                                                           uint32_t nf, int64_t* match, int64_t* fcommit,
                                                           int64_t* flush, int64_t* commit) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rh_delta x = d[i];
    if (x.slot >= capacity) return;  // validated on the host; never trust the ring blindly
    int64_t* p = nullptr;
    if (x.column < nf)
        p = match + (uint64_t)x.column * stride + x.slot;
    else if (x.column >= 16 && x.column < 16 + nf)
        p = fcommit + (uint64_t)(x.column - 16) * stride + x.slot;
    else if (x.column == RH_COL_FLUSH)
        p = flush + x.slot;
    else if (x.column == RH_COL_COMMITTED)
        p = commit + x.slot;
    if (p) atomicMax(reinterpret_cast<long long*>(p), (long long)x.value);
}

}  // namespace

int rh_apply_deltas_impl(hipStream_t stream, const rh_delta* d_deltas, uint64_t n, uint64_t capacity,
                         uint64_t stride, uint32_t n_followers, int64_t* match, int64_t* fcommit,
                         int64_t* flush, int64_t* commit) {
    if (n == 0) return RH_OK;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(apply_deltas_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, d_deltas, n,
                       capacity, stride, n_followers, match, fcommit, flush, commit);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
