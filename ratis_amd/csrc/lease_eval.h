// Leader-lease evaluation for one wave of 128 groups, shared by the lease kernels (lease.hip) and
// the fused commit + lease launch (commit.hip).  See lease.hip for the reference mapping.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "../../include/ratis_hip.h"
#include "sortnet.h"

namespace rh_lease {

constexpr int kLeaseBlock = 256;

typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
using rh_bits::spread32;

// Timestamp.elapsedTimeMs < timeout, division-free: for timeout T >= 0 (the launcher rejects T < 0),
// trunc(d / 10^6) < T  <=>  d <= lim(T), lim(0) = -10^6, lim(T >= 1) = T * 10^6 - 1 (saturating).
// One int64 compare instead of a 64-bit division by a constant per timestamp.
__device__ __forceinline__ int64_t ms_limit(int64_t T) {
    return T == 0 ? -1000000 : (T > INT64_MAX / 1000000 ? INT64_MAX : T * 1000000 - 1);
}
__device__ __forceinline__ bool ms_below(int64_t d, int64_t lim) { return d <= lim; }

// ((cnt-1)/2)-th smallest of the members' elapsed times; 0 (= currentTime()) for an empty list.
template <int F>
__device__ __forceinline__ int64_t majority_ack_elapsed(const int64_t (&d)[F > 0 ? F : 1], uint32_t member) {
    if constexpr (F == 0) {
        return 0;
    } else {
        const int cnt = __builtin_popcount(member);
        int64_t s[F];
#pragma unroll
        for (int i = 0; i < F; ++i) s[i] = ((member >> i) & 1u) ? d[i] : INT64_MAX;
        rh_sort::sort_net<F>(s);
        const int k = (cnt - 1) >> 1;
        int64_t r = s[0];
#pragma unroll
        for (int j = 1; j < F; ++j) r = (j == k) ? s[j] : r;
        return cnt ? r : 0;
    }
}

// PeerConfiguration.hasMajority(activePeers, includeSelf) with peers = followers in `mask` (+ self)
__device__ __forceinline__ bool has_majority(uint32_t mask, uint32_t active, bool self) {
    if (mask == 0 && !self) return true;
    const int num = (self ? 1 : 0) + __builtin_popcount(mask & active);
    return num > (__builtin_popcount(mask) + (self ? 1 : 0)) / 2;
}

// hasLease() for one group (see the file header for the elapsed-time form).
// `never` (bit k = follower k has no timestamp yet; the resident table's unstamped columns) makes
// a follower inactive and the oldest: it is never the majority-ack time when extend() runs.
template <int F>
__device__ __forceinline__ void lease_one(const rh_lease_soa& t, const int64_t (&ts)[F > 0 ? F : 1], uint32_t w,
                                          int64_t lin, bool en, bool in, int64_t& lout, bool& has, bool& ext,
                                          uint32_t never = 0u) {
    const int64_t now = t.now_nanos;
    const int64_t lim = ms_limit(t.timeout_ms);
    int64_t d[F > 0 ? F : 1];
    uint32_t act = 0;
#pragma unroll
    for (int k = 0; k < F; ++k) {
        const bool nv = (never >> k) & 1u;
        d[k] = nv ? INT64_MAX : (int64_t)((uint64_t)now - (uint64_t)ts[k]);
        act |= (!nv && ms_below(d[k], lim) ? 1u : 0u) << k;
    }
    const uint32_t nm = w & 0x3FFFu, om = (w >> 16) & 0x3FFFu;
    const bool self = (w & RH_CONF_SELF) != 0, self_old = (w & RH_CONF_SELF_OLD) != 0;
    // a word naming a follower slot >= F is malformed for this tier: treated as inactive (no
    // lease, no extension), the same rule as the commit kernel and the oracle
    constexpr uint32_t fm = (1u << F) - 1u;
    const bool trans = (w & RH_CONF_TRANSITIONAL) != 0,
               active = (w & RH_CONF_ACTIVE) != 0 && ((nm | om) & ~fm) == 0;
    // RaftConfigurationImpl.isSingleton (RCI:296-298)
    const int cur_size = __builtin_popcount(nm) + (self ? 1 : 0);
    const int prev_size = trans ? __builtin_popcount(om) + (self_old ? 1 : 0) : 0;
    const bool singleton = cur_size == 1 && prev_size <= 1;
    const bool valid_in = singleton || ms_below((int64_t)((uint64_t)now - (uint64_t)lin), lim);
    const bool maj = has_majority(nm, act, self) && (!trans || has_majority(om, act, self_old));
    ext = in && active && en && !valid_in && maj;
    lout = lin;
    has = in && active && en && valid_in;
    if (ext) {
        const int64_t dc = majority_ack_elapsed<F>(d, nm);
        const int64_t dold = trans ? majority_ack_elapsed<F>(d, om) : 0;  // old == null -> currentTime()
        // Timestamp.earliest(a, b) = a.compareTo(b) > 0 ? b : a, with a - b == dold - dc (wrapping)
        const int64_t dn = (int64_t)((uint64_t)dold - (uint64_t)dc) > 0 ? dold : dc;
        lout = (int64_t)((uint64_t)now - (uint64_t)dn);
        has = singleton || ms_below(dn, lim);
    }
}

// One wave = 128 groups, lane l holds groups 2l and 2l+1: every column is one 16-byte load per
// lane (VEC; needs an even col_stride and 16-byte aligned columns) and the two ballots of the
// wave interleave into its two bit words.
template <bool NT, typename V>
__device__ __forceinline__ V lease_ld(const V* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int F, bool VEC, bool NT>
__device__ __forceinline__ void lease_wave(const rh_lease_soa& t, uint64_t wbase) {
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = wbase + 2 * (uint64_t)lane;
    const bool in0 = r0 < t.n, in1 = r0 + 1 < t.n;
    // element index of group r0 in an int64 / uint32 column: plain (r0) or tiled (tile * elements
    // per tile + r0 % 128); r0 is even, so r0 + 1 is the next element in both layouts
    const uint64_t e = t.tile_stride ? (r0 >> 7) * (t.tile_stride >> 3) + (r0 & 127u) : r0;
    const uint64_t e32 = t.tile_stride ? (r0 >> 7) * (t.tile_stride >> 2) + (r0 & 127u) : r0;
    int64_t ts0[F > 0 ? F : 1], ts1[F > 0 ? F : 1];
    uint32_t w0 = 0, w1 = 0;
    int64_t l0 = 0, l1 = 0;
    if (VEC && in1) {
#pragma unroll
        for (int k = 0; k < F; ++k) {
            const v2i64 x = lease_ld<NT>(reinterpret_cast<const v2i64*>(t.follower_ts + (uint64_t)k * t.col_stride + e));
            ts0[k] = x.x;
            ts1[k] = x.y;
        }
        const v2u32 c = lease_ld<NT>(reinterpret_cast<const v2u32*>(t.conf + e32));
        const v2i64 li = lease_ld<NT>(reinterpret_cast<const v2i64*>(t.lease_in + e));
        w0 = c.x;
        w1 = c.y;
        l0 = li.x;
        l1 = li.y;
    } else {
#pragma unroll
        for (int k = 0; k < F; ++k) {
            ts0[k] = in0 ? t.follower_ts[(uint64_t)k * t.col_stride + e] : t.now_nanos;
            ts1[k] = in1 ? t.follower_ts[(uint64_t)k * t.col_stride + e + 1] : t.now_nanos;
        }
        w0 = in0 ? t.conf[e32] : 0u;
        w1 = in1 ? t.conf[e32 + 1] : 0u;
        l0 = in0 ? t.lease_in[e] : 0;
        l1 = in1 ? t.lease_in[e + 1] : 0;
    }
    // r0 is even, so both groups' bits live in the same enabled word
    const uint64_t ew = (t.enabled_bits && in0) ? t.enabled_bits[r0 >> 6] : ~0ull;
    const bool e0 = (ew >> (r0 & 63)) & 1ull;
    const bool e1 = (ew >> ((r0 + 1) & 63)) & 1ull;
    int64_t o0, o1;
    bool h0, h1, x0, x1;
    lease_one<F>(t, ts0, w0, l0, e0, in0, o0, h0, x0);
    lease_one<F>(t, ts1, w1, l1, e1, in1, o1, h1, x1);
    if (VEC && in1) {
        *reinterpret_cast<v2i64*>(t.lease_out + e) = v2i64{o0, o1};
    } else {
        if (in0) t.lease_out[e] = o0;
        if (in1) t.lease_out[e + 1] = o1;
    }
    const uint64_t he = __ballot(h0), ho = __ballot(h1);
    const uint64_t xe = __ballot(x0), xo = __ballot(x1);
    const uint64_t word = wbase >> 6;
    const uint64_t nwords = (t.n + 63) >> 6;
    if (lane < 2 && word + lane < nwords) {
        const uint64_t hw = lane ? (spread32(he >> 32) | (spread32(ho >> 32) << 1))
                                 : (spread32(he) | (spread32(ho) << 1));
        t.has_lease_bits[word + lane] = hw;
        if (t.extended_bits) {
            const uint64_t xw = lane ? (spread32(xe >> 32) | (spread32(xo >> 32) << 1))
                                     : (spread32(xe) | (spread32(xo) << 1));
            t.extended_bits[word + lane] = xw;
        }
    }
}

// All tiers of a follower-count class in one launch: block b belongs to the tier whose block
// range holds it (block-uniform), then a block-uniform switch on F.
struct LeaseLaunch {
    rh_lease_soa t[RH_MAX_TIERS];
    uint64_t first_block[RH_MAX_TIERS + 1];
    uint32_t vec_mask;
    int n_tiers;
};

template <int F, int FHI, bool NT>
__device__ __forceinline__ void lease_dispatch(const rh_lease_soa& t, bool vec, uint64_t wbase) {
    if constexpr (F <= FHI) {
        if ((int)t.n_followers == F) {
            if (vec) lease_wave<F, true, NT>(t, wbase);
            else lease_wave<F, false, NT>(t, wbase);
        } else {
            lease_dispatch<F + 1, FHI, NT>(t, vec, wbase);
        }
    }
}

constexpr uint64_t kGroupsPerBlock = kLeaseBlock / 64 * 128;

// Kernel arguments for the tiers whose F lies in [flo, fhi] (host side).
inline int build_lease_args(const rh_lease_soa* tiers, int n_tiers, int flo, int fhi, LeaseLaunch& a,
                            uint64_t& blocks) {
    a = LeaseLaunch{};
    blocks = 0;
    // blocks to the widest tiers first (their per-group work is the launch's tail otherwise)
    int order[RH_MAX_TIERS];
    for (int i = 0; i < n_tiers; ++i) order[i] = i;
    for (int i = 1; i < n_tiers; ++i)
        for (int j = i; j > 0 && tiers[order[j]].n_followers > tiers[order[j - 1]].n_followers; --j) {
            const int x = order[j];
            order[j] = order[j - 1];
            order[j - 1] = x;
        }
    for (int oi = 0; oi < n_tiers; ++oi) {
        const rh_lease_soa& t = tiers[order[oi]];
        if (t.n == 0 || (int)t.n_followers < flo || (int)t.n_followers > fhi) continue;
        const bool vec = (t.n_followers == 0 || t.col_stride % 2 == 0) && t.tile_stride % 16 == 0 &&
                         (t.n_followers == 0 || ((uintptr_t)t.follower_ts & 15) == 0) &&
                         ((uintptr_t)t.conf & 7) == 0 && ((uintptr_t)t.lease_in & 15) == 0 &&
                         ((uintptr_t)t.lease_out & 15) == 0;
        a.t[a.n_tiers] = t;
        a.first_block[a.n_tiers] = blocks;
        a.vec_mask |= (vec ? 1u : 0u) << a.n_tiers;
        ++a.n_tiers;
        blocks += (t.n + kGroupsPerBlock - 1) / kGroupsPerBlock;
    }
    a.first_block[a.n_tiers] = blocks;
    return RH_OK;
}

// One block of the F <= 7 class (non-temporal loads), block index b within the class's blocks.
__device__ __forceinline__ void lease_block(const LeaseLaunch& a, uint64_t b) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < a.n_tiers && b >= a.first_block[i]) k = i;
    const rh_lease_soa& t = a.t[k];
    const uint64_t wbase = ((b - a.first_block[k]) * kLeaseBlock / 64 + (threadIdx.x >> 6)) * 128;
    if (wbase >= t.n) return;
    lease_dispatch<0, 7, true>(t, (a.vec_mask >> k) & 1u, wbase);
}

}  // namespace rh_lease
