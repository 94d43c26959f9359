// Batched leader-lease check/extension on gfx950: LeaderStateImpl.hasLease() for every group.
//
// Reference semantics (ratis-server/.../server/impl/):
//   LeaderStateImpl.hasLease / checkLeaderLease   LeaderStateImpl.java:1229-1249
//   LeaderLease.isValid / extend                  LeaderLease.java:60-85
//   LeaderLease.getMaxTimestampWithMajorityAck    LeaderLease.java:90-103
//   RaftConfigurationImpl.hasMajority/isSingleton RaftConfigurationImpl.java:265-298
//   PeerConfiguration.hasMajority                 PeerConfiguration.java:152-169
//   Timestamp.compareTo / earliest / elapsedTimeMs Timestamp.java:51-56, 87-112
//
// Work is done on elapsed times d = now - t (wrapping int64).  For |d| < 2^62 (every realistic
// nanoTime) Timestamp.compareTo(a, b) == sign(d_b - d_a), so "sort ascending by timestamp, take
// element size/2" is "take the ((size-1)/2)-th smallest elapsed time" -- the same order statistic
// the commit kernel takes, here over the followers only (self has no FollowerInfo).  One group
// per lane, column loads coalesced across the wave, hasLease/extended bits by wave ballot.
#include "rh_internal.h"
#include "sortnet.h"

namespace {

constexpr int kLeaseBlock = 256;

struct LeaseArgs {
    rh_lease_soa t;
};

__device__ __forceinline__ int64_t elapsed_ms(int64_t d) { return d / 1000000; }  // truncating, as Java

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

template <int F>
__global__ __launch_bounds__(kLeaseBlock) void lease_kernel(LeaseArgs a) {
    const rh_lease_soa& t = a.t;
    const uint64_t i = (uint64_t)blockIdx.x * kLeaseBlock + threadIdx.x;
    const bool in = i < t.n;
    const uint32_t w = in ? t.conf[i] : 0u;
    const int64_t lin = in ? t.lease_in[i] : 0;
    const bool en = t.enabled_bits ? ((t.enabled_bits[i >> 6] >> (i & 63)) & 1ull) : true;
    const int64_t now = t.now_nanos;
    int64_t d[F > 0 ? F : 1];
    uint32_t act = 0;
#pragma unroll
    for (int k = 0; k < F; ++k) {
        const int64_t ts = in ? t.follower_ts[(uint64_t)k * t.col_stride + i] : now;
        d[k] = (int64_t)((uint64_t)now - (uint64_t)ts);
        act |= (elapsed_ms(d[k]) < t.timeout_ms ? 1u : 0u) << k;
    }
    const uint32_t nm = w & 0x3FFFu, om = (w >> 16) & 0x3FFFu;
    const bool self = (w & RH_CONF_SELF) != 0, self_old = (w & RH_CONF_SELF_OLD) != 0;
    const bool trans = (w & RH_CONF_TRANSITIONAL) != 0, active = (w & RH_CONF_ACTIVE) != 0;
    // RaftConfigurationImpl.isSingleton (RCI:296-298)
    const int cur_size = __builtin_popcount(nm) + (self ? 1 : 0);
    const int prev_size = trans ? __builtin_popcount(om) + (self_old ? 1 : 0) : 0;
    const bool singleton = cur_size == 1 && prev_size <= 1;
    const bool valid_in = singleton || elapsed_ms((int64_t)((uint64_t)now - (uint64_t)lin)) < t.timeout_ms;
    const bool maj = has_majority(nm, act, self) && (!trans || has_majority(om, act, self_old));
    const bool extend = in && active && en && !valid_in && maj;
    int64_t lout = lin;
    bool has = in && active && en && valid_in;
    if (extend) {
        const int64_t dc = majority_ack_elapsed<F>(d, nm);
        const int64_t dold = trans ? majority_ack_elapsed<F>(d, om) : 0;  // old == null -> currentTime()
        // Timestamp.earliest(a, b) = a.compareTo(b) > 0 ? b : a, with a - b == dold - dc (wrapping)
        const int64_t dn = (int64_t)((uint64_t)dold - (uint64_t)dc) > 0 ? dold : dc;
        lout = (int64_t)((uint64_t)now - (uint64_t)dn);
        has = singleton || elapsed_ms(dn) < t.timeout_ms;
    }
    if (in) t.lease_out[i] = lout;
    const uint64_t hb = __ballot(has);
    const uint64_t xb = __ballot(extend);
    const int lane = threadIdx.x & 63;
    const uint64_t word = i >> 6;
    if (lane == 0 && (word << 6) < t.n) {
        t.has_lease_bits[word] = hb;
        if (t.extended_bits) t.extended_bits[word] = xb;
    }
}

template <int F>
void launch_f(const rh_lease_soa& t, hipStream_t stream) {
    LeaseArgs a{t};
    const uint64_t blocks = (t.n + kLeaseBlock - 1) / kLeaseBlock;
    hipLaunchKernelGGL(lease_kernel<F>, dim3((uint32_t)blocks), dim3(kLeaseBlock), 0, stream, a);
}

template <int F = 0>
void dispatch(const rh_lease_soa& t, hipStream_t stream) {
    if constexpr (F <= 14) {
        if ((int)t.n_followers == F) launch_f<F>(t, stream);
        else dispatch<F + 1>(t, stream);
    }
}

}  // namespace

int rh_lease_launch_impl(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, hipStream_t stream) {
    (void)ctx;
    if (!tiers || n_tiers < 1 || n_tiers > RH_MAX_TIERS)
        return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: n_tiers must be in [1, RH_MAX_TIERS]");
    for (int k = 0; k < n_tiers; ++k) {
        const rh_lease_soa& t = tiers[k];
        if (t.n_followers > 14) return rh::fail(RH_E_RANGE, "rh_lease_soa_launch: n_followers must be in [0, 14]");
        if (t.n == 0) continue;
        if (!t.conf || !t.lease_in || !t.lease_out || !t.has_lease_bits || (t.n_followers && !t.follower_ts))
            return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: conf/lease_in/lease_out/has_lease_bits required");
        if (t.n_followers && t.col_stride < t.n) return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: col_stride < n");
        if (t.timeout_ms < 0) return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: timeout_ms < 0");
        if (t.n > (uint64_t)UINT32_MAX * kLeaseBlock) return rh::fail(RH_E_RANGE, "rh_lease_soa_launch: n too large");
    }
    for (int k = 0; k < n_tiers; ++k) {
        if (tiers[k].n == 0) continue;
        dispatch(tiers[k], stream);
        RH_HIP(hipGetLastError());
    }
    return RH_OK;
}
