// Per-group evaluation shared by the raw SoA commit kernels (commit.hip) and the resident-table
// kernels (table.hip): LeaderStateImpl.getMajorityMin + RaftLogBase.updateCommitIndex for ONE
// group held in registers.
//   LeaderStateImpl.getMajorityMin        LeaderStateImpl.java:956-984
//   LeaderStateImpl.getSorted             LeaderStateImpl.java:1076-1095
//   MinMajorityMax.valueOf / combine      LeaderStateImpl.java:904-944
//   LeaderStateImpl.updateCommit(maj,min) LeaderStateImpl.java:1015-1026
//   RaftLogBase.updateCommitIndex         RaftLogBase.java:121-142
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "../../include/ratis_hip.h"
#include "sortnet.h"

namespace rh_eval {

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

// getMajorityMin (LSI:956-984) for one group: vals[0..F) = the follower index column (matchIndex
// or commitIndex), vals[F] = self (flushIndex or lastCommittedIndex), w = the membership word.
// any_trans (wave-uniform) skips the old-conf pass for waves without a transitional group.
// Invalid (inactive, Optional.empty() or a malformed word) -> valid = false, levels INT64_MIN.
template <int F, bool RANK>
__device__ __forceinline__ void eval_group(const int64_t (&vals)[F + 1], uint32_t w, int64_t gap, bool any_trans,
                                           bool& valid, int64_t& mn, int64_t& mj, int64_t& mx) {
    constexpr int N = F + 1;
    const uint32_t fmask = (1u << F) - 1u;
    const bool trans = (w & RH_CONF_ACTIVE) && (w & RH_CONF_TRANSITIONAL);
    const uint32_t mnew = (w & fmask) | (((w >> 14) & 1u) << F);
    const uint32_t mold = ((w >> RH_CONF_OLD_SHIFT) & fmask) | (((w >> 30) & 1u) << F);
    // followers.isEmpty() && !includeSelf -> Optional.empty()  (LSI:964-966, 976-978).
    // A word naming a follower slot >= F is malformed for this tier: no result, no commit
    // (ABI rule shared with the lease kernel and the oracle; never a smaller quorum).
    const bool fits = ((w & 0x3FFFu) & ~fmask) == 0 && (((w >> RH_CONF_OLD_SHIFT) & 0x3FFFu) & ~fmask) == 0;
    const bool v = (w & RH_CONF_ACTIVE) && fits && mnew != 0 && (!trans || mold != 0);
    int64_t a0, a1, a2;
    if (RANK) {
        uint32_t less[N];
        rh_sort::rank_masks<N>(vals, less);
        order_stats_rank<N>(vals, less, mnew ? mnew : 1u, gap, a0, a1, a2);
        if (any_trans) {
            if (trans) {  // combine(): element-wise min (LSI:915-920)
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
            if (trans) {  // combine(): element-wise min (LSI:915-920)
                int64_t b0, b1, b2;
                order_stats<N>(vals, mold ? mold : 1u, gap, b0, b1, b2);
                a0 = b0 < a0 ? b0 : a0;
                a1 = b1 < a1 ? b1 : a1;
                a2 = b2 < a2 ? b2 : a2;
            }
        }
    }
    valid = v;
    mn = v ? a0 : INT64_MIN;
    mj = v ? a1 : INT64_MIN;
    mx = v ? a2 : INT64_MIN;
}

// updateCommit(majority, min) (LSI:1015-1026) -> RaftLogBase.updateCommitIndex (RLB:121-142):
// old = lastCommitted; if (majority > old) { newCommit = min(majority, flushIndex);
//   if (old < newCommit && termAt(newCommit) == currentTerm) commit = newCommit; }
// with termAt(i) == currentTerm <=> i >= term_start for i <= flushIndex.
__device__ __forceinline__ bool commit_decision(bool valid, int64_t majority, int64_t old, int64_t flush,
                                                int64_t term_start, int64_t& out) {
    const int64_t nc = majority < flush ? majority : flush;
    const bool a = valid && majority > old && old < nc && nc >= term_start;
    out = a ? nc : old;
    return a;
}

}  // namespace rh_eval
