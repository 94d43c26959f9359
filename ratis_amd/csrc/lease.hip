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
// the commit kernel takes, here over the followers only (self has no FollowerInfo).  Two groups
// per lane with 16-byte column loads, all tiers of a follower-count class in one launch,
// hasLease/extended bits by wave ballot.
#include "rh_internal.h"
#include "lease_eval.h"

#ifndef RH_LEASE_NT      // A/B: non-temporal column loads in the F <= 7 kernel
#define RH_LEASE_NT 1
#endif
#ifndef RH_LEASE_WAVES   // A/B: waves per SIMD the F <= 7 kernel is pinned to
#define RH_LEASE_WAVES 8
#endif

namespace {

using namespace rh_lease;

template <int FLO, int FHI, bool NT, int MINW>
__global__ __launch_bounds__(kLeaseBlock) __attribute__((amdgpu_waves_per_eu(MINW, 8))) void lease_kernel(LeaseLaunch arg) {
    const LeaseLaunch& a = rh::kernarg_struct<LeaseLaunch>();
    const uint64_t b = blockIdx.x;
    int k = 0;
#pragma unroll
    for (int i = 1; i < RH_MAX_TIERS; ++i)
        if (i < a.n_tiers && b >= a.first_block[i]) k = i;
    const rh_lease_soa& t = a.t[k];
    const uint64_t wbase = ((b - a.first_block[k]) * kLeaseBlock / 64 + (threadIdx.x >> 6)) * 128;
    if (wbase >= t.n) return;
    lease_dispatch<FLO, FHI, NT>(t, (a.vec_mask >> k) & 1u, wbase);
}

}  // namespace

int rh_lease_launch_class(const rh_lease_soa* tiers, int n_tiers, int flo, int fhi, hipStream_t stream) {
    LeaseLaunch a{};
    uint64_t blocks = 0;
    build_lease_args(tiers, n_tiers, flo, fhi, a, blocks);
    if (a.n_tiers == 0) return RH_OK;
    if (blocks > 0x7fffffffull) return rh::fail(RH_E_RANGE, "rh_lease_soa_launch: too many groups");
    const dim3 g((uint32_t)blocks), b(kLeaseBlock);
    // F <= 7: non-temporal loads (every byte is read once), register budget pinned to 8
    // waves/SIMD so a 1M-group launch is resident in one round; wider tiers: plain loads
    if (flo != 0)
        hipLaunchKernelGGL((lease_kernel<8, 14, false, 1>), g, b, 0, stream, a);
    else
        hipLaunchKernelGGL((lease_kernel<0, 7, RH_LEASE_NT != 0, RH_LEASE_WAVES>), g, b, 0, stream, a);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_lease_validate(const rh_lease_soa* tiers, int n_tiers) {
    if (!tiers || n_tiers < 1 || n_tiers > RH_MAX_TIERS)
        return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: n_tiers must be in [1, RH_MAX_TIERS]");
    for (int k = 0; k < n_tiers; ++k) {
        const rh_lease_soa& t = tiers[k];
        if (t.n_followers > 14) return rh::fail(RH_E_RANGE, "rh_lease_soa_launch: n_followers must be in [0, 14]");
        if (t.n == 0) continue;
        if (!t.conf || !t.lease_in || !t.lease_out || !t.has_lease_bits || (t.n_followers && !t.follower_ts))
            return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: conf/lease_in/lease_out/has_lease_bits required");
        if (t.tile_stride) {
            if (t.tile_stride % 16) return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: tile_stride not a multiple of 16");
            if (t.n_followers && t.col_stride < RH_TILE_GROUPS)
                return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: tiled col_stride < 128");
        } else if (t.n_followers && t.col_stride < t.n) {
            return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: col_stride < n");
        }
        if (t.timeout_ms < 0) return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: timeout_ms < 0");
        if (t.n > (uint64_t)UINT32_MAX * kLeaseBlock) return rh::fail(RH_E_RANGE, "rh_lease_soa_launch: n too large");
    }
    return RH_OK;
}

int rh_lease_launch_impl(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, hipStream_t stream) {
    (void)ctx;
    int rc = rh_lease_validate(tiers, n_tiers);
    if (rc == RH_OK) rc = rh_lease_launch_class(tiers, n_tiers, 0, 7, stream);
    return rc != RH_OK ? rc : rh_lease_launch_class(tiers, n_tiers, 8, 14, stream);
}
