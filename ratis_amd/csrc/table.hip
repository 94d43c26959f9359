// Device side of the resident group table (rh_groups, include/ratis_hip.h) for gfx950.
//
//   table_apply_kernel    FollowerInfo.updateMatchIndex / updateCommitIndex (RaftLogIndex.updateToMax,
//                         FollowerInfoImpl.java:93-105), setSnapshotIndex's setUnconditionally
//                         (FollowerInfoImpl.java:147-151), the flush-index advance
//                         (SegmentedRaftLogWorker.java:419-431) -- and the event each one submits
//                         (submitUpdateCommitEvent, LeaderStateImpl.java:846-854, 900-902): the
//                         touched row is marked dirty.
//   table_control_kernel  leader start (new FollowerInfos at -1, FollowerInfoImpl.java:42-43),
//                         conf change with follower carry-over / reset, step down.
//   table_commit_kernel   LeaderStateImpl.updateCommit() (COMMIT) or commitIndexChanged() (WATCH)
//                         over the DIRTY rows of every tier; only changed results become events,
//                         written straight into host-mapped pinned memory.
//   table_lease_kernel    LeaderStateImpl.hasLease() (LSI:1229-1249) with LeaderLease.extend (LL:67-84)
//                         for every started slot: lease_eval.h's arithmetic over the follower
//                         timestamp columns, the lease stored in place, a slot-indexed bitmap out.
//   table_read_kernel     slot-ordered read-back of one column.
//
// Rows of a tier are laid out exactly like an rh_commit_soa tier (column-major, 16-byte aligned
// columns), so the per-group arithmetic is commit_eval.h's, shared with the raw SoA kernels.
// Integer compare/select work, no MFMA; HBM-bound over the dirty rows.
#include "rh_internal.h"
#include "commit_eval.h"
#include "lease_eval.h"

namespace {

using rh::CtrlOp;
using rh::TableDev;
using rh::TableEvents;
using rh::TableTier;

typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool locate(const TableDev& T, uint32_t slot, const TableTier*& tt, uint32_t& row) {
    if ((uint64_t)slot >= T.capacity) return false;
    const uint32_t m = T.slot_map[slot];
    if (m == rh::kNoRow) return false;
    const uint32_t t = m >> 28;
    if (t >= (uint32_t)rh::kTableTiers) return false;
    tt = &T.tier[t];
    row = m & rh::kRowMask;
    return row < tt->rows;
}

// ---- deltas --------------------------------------------------------------------------------------
// phase 0 applies the batch's SET deltas (plain stores), phase 1 its MAX deltas (atomicMax): the
// host orders batches so that this equals applying them one by one (ratis_hip.h, rh_delta).
__global__ __launch_bounds__(256) void table_apply_kernel(TableDev Targ, const rh_delta* __restrict__ d, uint64_t n,
                                                          int phase) {
    // the tier is picked per thread: index the argument in the kernarg segment (scalar loads), not
    // the by-value copy, which the compiler spilled whole into scratch (984 B per lane, 8x slower)
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rh_delta x = d[i];
    if (x.op != (phase == 0 ? RH_OP_SET : RH_OP_MAX)) return;
    const TableTier* tt;
    uint32_t row;
    if (!locate(T, x.slot, tt, row)) return;  // stopped slot / out of range: ignored
    int64_t* p = nullptr;
    bool commit_ev = false, watch_ev = false;
    const uint32_t c = x.column;
    if (c == RH_COL_LEASE_ON) {  // AtomicBoolean: SET stores, MAX ORs
        if (phase == 0)
            tt->lon[row] = x.value != 0;
        else if (x.value != 0)
            tt->lon[row] = 1;
        return;
    }
    if (c >= 48 && c < 64) {
        if (c - 48 < tt->width) p = tt->fts + (uint64_t)(c - 48) * tt->rows + row;
    } else if (c == RH_COL_LEASE) {
        p = tt->lease + row;
    } else if (c < 16) {
        if (c < tt->width) p = tt->match + (uint64_t)c * tt->rows + row;
        commit_ev = true;
    } else if (c < 32) {
        if (c - 16 < tt->width) p = tt->fcommit + (uint64_t)(c - 16) * tt->rows + row;
        watch_ev = true;
    } else if (c == RH_COL_FLUSH) {
        p = tt->flush + row;
        commit_ev = true;
    } else if (c == RH_COL_COMMITTED) {
        p = tt->commit + row;
        commit_ev = watch_ev = true;
    }
    if (!p) return;
    if (phase == 0)
        *p = x.value;
    else
        atomicMax(reinterpret_cast<long long*>(p), (long long)x.value);
    if (commit_ev) tt->dirty[row] = 1;
    if (watch_ev) tt->wdirty[row] = 1;
}

// ---- control ops ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void table_control_kernel(TableDev T, const CtrlOp* __restrict__ ops, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const CtrlOp op = ops[i];
    if (op.kind == rh::kCtrlStop) {
        const TableTier& s = T.tier[op.src >> 28];
        const uint32_t r = op.src & rh::kRowMask;
        s.conf[r] = 0u;
        s.dirty[r] = 0;
        s.wdirty[r] = 0;
        s.lon[r] = 0;
        s.row_slot[r] = rh::kNoRow;
        T.slot_map[op.slot] = rh::kNoRow;
        return;
    }
    const TableTier& D = T.tier[op.dst >> 28];
    const uint32_t r = op.dst & rh::kRowMask;
    const uint64_t R = D.rows;
    if (op.kind == rh::kCtrlStart) {
        for (uint32_t k = 0; k < D.width; ++k) {
            D.match[k * R + r] = -1;   // RaftLog.INVALID_LOG_INDEX (FollowerInfoImpl.java:42-43)
            D.fcommit[k * R + r] = -1;
            D.fts[k * R + r] = rh::kNoTimestamp;
        }
        D.lease[r] = rh::kNoTimestamp;  // rh_group_lease_start sets the LeaderLease
        D.lon[r] = 0;
        D.flush[r] = op.flush;
        D.commit[r] = op.commit;
        D.tstart[r] = op.tstart;
        D.wall[r] = INT64_MIN;
        D.wmin[r] = INT64_MIN;
        D.wmaj[r] = INT64_MIN;
        D.wmax[r] = INT64_MIN;
    } else {  // MOVE (to another tier) or RECONF (same row): follower columns through the map
        const TableTier& S = T.tier[op.src >> 28];
        const uint32_t sr = op.src & rh::kRowMask;
        const uint64_t SR = S.rows;
        int64_t m[RH_MAX_FOLLOWERS], f[RH_MAX_FOLLOWERS], ts[RH_MAX_FOLLOWERS];
        for (uint32_t k = 0; k < D.width; ++k) {  // read all first: RECONF may permute in place
            const int src = op.map[k];
            const bool keep = src >= 0 && (uint32_t)src < S.width;
            m[k] = keep ? S.match[(uint64_t)src * SR + sr] : -1;
            f[k] = keep ? S.fcommit[(uint64_t)src * SR + sr] : -1;
            ts[k] = keep ? S.fts[(uint64_t)src * SR + sr] : rh::kNoTimestamp;
        }
        for (uint32_t k = 0; k < D.width; ++k) {
            D.match[k * R + r] = m[k];
            D.fcommit[k * R + r] = f[k];
            D.fts[k * R + r] = ts[k];
        }
        if (op.kind == rh::kCtrlMove) {
            D.flush[r] = S.flush[sr];
            D.commit[r] = S.commit[sr];
            D.tstart[r] = S.tstart[sr];
            D.wall[r] = S.wall[sr];
            D.wmin[r] = S.wmin[sr];
            D.wmaj[r] = S.wmaj[sr];
            D.wmax[r] = S.wmax[sr];
            D.lease[r] = S.lease[sr];
            D.lon[r] = S.lon[sr];
            S.lon[sr] = 0;
            S.conf[sr] = 0u;
            S.dirty[sr] = 0;
            S.wdirty[sr] = 0;
            S.row_slot[sr] = rh::kNoRow;
        }
    }
    D.conf[r] = op.conf;
    D.row_slot[r] = op.slot;
    D.dirty[r] = 1;
    D.wdirty[r] = 1;
    T.slot_map[op.slot] = op.dst;
}

// ---- updateCommit / commitIndexChanged over the dirty rows ---------------------------------------
struct TierRange {
    uint32_t block_begin[rh::kTableTiers + 1];  // blocks of tier t: [block_begin[t], block_begin[t+1])
};

constexpr int kTBlock = 256;  // 4 waves x 128 rows

template <int F, bool RANK, bool WATCH>
__device__ __forceinline__ void table_wave(const TableDev& T, const TableTier& tt, uint64_t wbase,
                                           const TableEvents& ev) {
    constexpr int N = F + 1;
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = wbase + 2 * (uint64_t)lane;  // rows is a multiple of 128: r0 + 1 < rows
    uint8_t* dflag = WATCH ? tt.wdirty : tt.dirty;
    const uint16_t dd = *reinterpret_cast<const uint16_t*>(dflag + r0);
    const bool d0 = (dd & 0xFFu) != 0, d1 = (dd >> 8) != 0;
    const bool need = d0 || d1;
    if (!__any(need)) return;  // the whole 128-row sub-tile is clean: nothing read
    int64_t fv[2][F], self[2] = {0, 0}, cin[2] = {0, 0}, ts[2] = {0, 0};
    int64_t p0[2] = {0, 0}, p1[2] = {0, 0}, p2[2] = {0, 0};
    uint32_t w[2] = {0u, 0u};
    if (need) {
        const int64_t* col = WATCH ? tt.fcommit : tt.match;
#pragma unroll
        for (int k = 0; k < F; ++k) {
            const v2i64 x = *reinterpret_cast<const v2i64*>(col + (uint64_t)k * tt.rows + r0);
            fv[0][k] = x.x;
            fv[1][k] = x.y;
        }
        const v2u32 c = *reinterpret_cast<const v2u32*>(tt.conf + r0);
        w[0] = d0 ? c.x : 0u;  // a clean row is evaluated as inactive and produces nothing
        w[1] = d1 ? c.y : 0u;
        const v2i64 cm = *reinterpret_cast<const v2i64*>(tt.commit + r0);
        cin[0] = cm.x;
        cin[1] = cm.y;
        if (WATCH) {
            self[0] = cm.x;  // lastCommittedIndex is the self value (LSI:613)
            self[1] = cm.y;
            const v2i64 a = *reinterpret_cast<const v2i64*>(tt.wmin + r0);
            const v2i64 b = *reinterpret_cast<const v2i64*>(tt.wmaj + r0);
            const v2i64 e = *reinterpret_cast<const v2i64*>(tt.wmax + r0);
            p0[0] = a.x, p0[1] = a.y, p1[0] = b.x, p1[1] = b.y, p2[0] = e.x, p2[1] = e.y;
        } else {
            const v2i64 fl = *reinterpret_cast<const v2i64*>(tt.flush + r0);
            const v2i64 st = *reinterpret_cast<const v2i64*>(tt.tstart + r0);
            self[0] = fl.x, self[1] = fl.y, ts[0] = st.x, ts[1] = st.y;
            if (ev.wall) {  // watch-ALL levels are compared only when reported (RH_COMMIT_WATCH_ALL)
                const v2i64 wa = *reinterpret_cast<const v2i64*>(tt.wall + r0);
                p0[0] = wa.x, p0[1] = wa.y;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < F; ++k) fv[0][k] = fv[1][k] = 0;
    }
    const int64_t gap = WATCH ? -1 : T.gap;  // commitIndexChanged uses the 2-arg overload (gap -1)
    bool trans[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) trans[g] = (w[g] & RH_CONF_ACTIVE) && (w[g] & RH_CONF_TRANSITIONAL);
    const bool any_trans = __any(trans[0] || trans[1]);
    bool adv[2] = {false, false}, chg[2] = {false, false}, valid[2];
    int64_t mn[2], mj[2], mx[2], nc[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        int64_t vals[N];
#pragma unroll
        for (int k = 0; k < F; ++k) vals[k] = fv[g][k];
        vals[F] = self[g];
        rh_eval::eval_group<F, RANK>(vals, w[g], gap, any_trans, valid[g], mn[g], mj[g], mx[g]);
        const bool dg = g ? d1 : d0;
        if (WATCH) {
            chg[g] = dg && (mn[g] != p0[g] || mj[g] != p1[g] || mx[g] != p2[g]);
        } else {
            adv[g] = dg && rh_eval::commit_decision(valid[g], mj[g], cin[g], self[g], ts[g], nc[g]);
            chg[g] = dg && ev.wall && mn[g] != p0[g];  // watch-ALL level changed (LSI:1025)
        }
    }
    // stores: only what changed, plus clearing the dirty flags of this lane's rows
    if (need) *reinterpret_cast<uint16_t*>(dflag + r0) = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const uint64_t r = r0 + g;
        if (WATCH) {
            if (chg[g]) {
                tt.wmin[r] = mn[g];
                tt.wmaj[r] = mj[g];
                tt.wmax[r] = mx[g];
            }
        } else {
            if (adv[g]) {
                tt.commit[r] = nc[g];
                tt.wdirty[r] = 1;  // the commit index changed: commitIndexChanged follows (LSI:1003)
            }
            if (chg[g]) tt.wall[r] = mn[g];
        }
    }
    // events: one atomic per wave and event kind, records written to host-mapped memory
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (!WATCH) {
        const uint64_t ae = __ballot(adv[0]), ao = __ballot(adv[1]);
        if (ae | ao) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(&ev.counts[0], (unsigned long long)(__popcll(ae) + __popcll(ao)));
            base = __shfl(base, 0);
            uint64_t pos = base + __popcll(ae & lt) + __popcll(ao & lt);
#pragma unroll
            for (int g = 0; g < 2; ++g)
                if (adv[g]) {
                    if (pos < ev.cap) {
                        rh_index_event e{tt.row_slot[r0 + g], 0u, nc[g]};
                        ev.adv[pos] = e;
                    }
                    ++pos;
                }
        }
    }
    const uint64_t ce = __ballot(chg[0]), co = __ballot(chg[1]);
    if (ce | co) {
        unsigned long long base = 0;
        if (lane == 0)
            base = atomicAdd(&ev.counts[WATCH ? 2 : 1], (unsigned long long)(__popcll(ce) + __popcll(co)));
        base = __shfl(base, 0);
        uint64_t pos = base + __popcll(ce & lt) + __popcll(co & lt);
#pragma unroll
        for (int g = 0; g < 2; ++g)
            if (chg[g]) {
                if (pos < ev.cap) {
                    const uint32_t slot = tt.row_slot[r0 + g];
                    if (WATCH) {
                        rh_watch_event e{slot, valid[g] ? 1u : 0u, mn[g], mj[g], mx[g]};
                        ev.watch[pos] = e;
                    } else {
                        rh_index_event e{slot, 0u, mn[g]};
                        ev.wall[pos] = e;
                    }
                }
                ++pos;
            }
    }
}

template <int F, int FHI, bool RANK, bool WATCH>
__device__ __forceinline__ void table_dispatch(const TableDev& T, int t, uint64_t wbase, const TableEvents& ev) {
    if ((int)rh::width_of_tier(t) == F)
        table_wave<F, RANK, WATCH>(T, T.tier[t], wbase, ev);
    else if constexpr (F + 2 <= FHI)
        table_dispatch<F + 2, FHI, RANK, WATCH>(T, t, wbase, ev);
}

// Widths 2..6: rank-mask order statistics; widths 8..14: Batcher networks (commit.hip's split).
template <bool WATCH, int FLO, int FHI>
__global__ __launch_bounds__(kTBlock) void table_commit_kernel(TableDev T, TierRange tr, TableEvents ev) {
    const uint32_t b = blockIdx.x;
    int t = 0;
#pragma unroll
    for (int i = 1; i < rh::kTableTiers; ++i)
        if (b >= tr.block_begin[i]) t = i;
    const uint64_t wbase = ((uint64_t)(b - tr.block_begin[t]) * (kTBlock / 64) + (threadIdx.x >> 6)) * 128;
    if (wbase >= T.tier[t].rows) return;
    table_dispatch<FLO, FHI, FLO <= 6, WATCH>(T, t, wbase, ev);
}

// ---- hasLease over every started row -------------------------------------------------------------
template <int F>
__global__ __launch_bounds__(256) void table_lease_kernel(TableTier tt, int64_t now, int64_t timeout_ms,
                                                          uint64_t* __restrict__ slot_bits) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= tt.rows) return;
    const uint32_t w = tt.conf[r];
    if (!(w & RH_CONF_ACTIVE)) return;  // free row
    int64_t ts[F];
    uint32_t never = 0;
#pragma unroll
    for (int k = 0; k < F; ++k) {
        ts[k] = tt.fts[(uint64_t)k * tt.rows + r];
        never |= (ts[k] == rh::kNoTimestamp ? 1u : 0u) << k;
    }
    rh_lease_soa t{};
    t.now_nanos = now;
    t.timeout_ms = timeout_ms;
    int64_t lout;
    bool has, ext;
    rh_lease::lease_one<F>(t, ts, w, tt.lease[r], tt.lon[r] != 0, true, lout, has, ext, never);
    if (ext) tt.lease[r] = lout;
    if (has) {
        const uint32_t slot = tt.row_slot[r];
        atomicOr(reinterpret_cast<unsigned long long*>(slot_bits + (slot >> 6)), 1ull << (slot & 63));
    }
}

template <int F>
void launch_lease_width(const TableTier& tt, int64_t now, int64_t timeout_ms, uint64_t* bits, hipStream_t s) {
    hipLaunchKernelGGL((table_lease_kernel<F>), dim3((tt.rows + 255) / 256), dim3(256), 0, s, tt, now, timeout_ms, bits);
}

// ---- read-back -------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void table_read_kernel(TableDev T, uint32_t first, uint32_t n, uint32_t column,
                                                         int64_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TableTier* tt;
    uint32_t row;
    int64_t v = INT64_MIN;
    if (locate(T, first + i, tt, row)) {
        const uint64_t R = tt->rows;
        if (column < 16) v = column < tt->width ? tt->match[column * R + row] : -1;
        else if (column < 32) v = column - 16 < tt->width ? tt->fcommit[(column - 16) * R + row] : -1;
        else if (column == RH_COL_FLUSH) v = tt->flush[row];
        else if (column == RH_COL_COMMITTED) v = tt->commit[row];
        else if (column == RH_COL_CONF) v = (int64_t)tt->conf[row];
        else if (column == RH_COL_TERM_START) v = tt->tstart[row];
        else if (column == RH_COL_LEASE) v = tt->lease[row];
        else if (column == RH_COL_LEASE_ON) v = (int64_t)tt->lon[row];
        else if (column >= 48 && column < 64) v = column - 48 < tt->width ? tt->fts[(column - 48) * R + row] : rh::kNoTimestamp;
    }
    out[i] = v;
}

}  // namespace

int rh_table_apply_deltas(const rh::TableDev& t, const rh_delta* d_deltas, uint64_t n, int phase, hipStream_t stream) {
    if (n == 0) return RH_OK;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(table_apply_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, t, d_deltas, n, phase);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_table_control(const rh::TableDev& t, const rh::CtrlOp* d_ops, uint64_t n, hipStream_t stream) {
    if (n == 0) return RH_OK;
    hipLaunchKernelGGL(table_control_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, t, d_ops, n);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_table_commit(const rh::TableDev& t, int mode, const rh::TableEvents& ev, hipStream_t stream) {
    // one launch per width class over every non-empty tier of the class
    for (int cls = 0; cls < 2; ++cls) {
        TierRange tr{};
        uint32_t blocks = 0;
        for (int i = 0; i < rh::kTableTiers; ++i) {
            tr.block_begin[i] = blocks;
            const bool in_cls = cls == 0 ? i <= 2 : i >= 3;
            if (in_cls && t.tier[i].rows) blocks += (uint32_t)(t.tier[i].rows / (2 * kTBlock) + (t.tier[i].rows % (2 * kTBlock) != 0));
        }
        tr.block_begin[rh::kTableTiers] = blocks;
        if (blocks == 0) continue;
        const dim3 g(blocks), b(kTBlock);
        if (mode == RH_MODE_WATCH) {
            if (cls == 0) hipLaunchKernelGGL((table_commit_kernel<true, 2, 6>), g, b, 0, stream, t, tr, ev);
            else hipLaunchKernelGGL((table_commit_kernel<true, 8, 14>), g, b, 0, stream, t, tr, ev);
        } else {
            if (cls == 0) hipLaunchKernelGGL((table_commit_kernel<false, 2, 6>), g, b, 0, stream, t, tr, ev);
            else hipLaunchKernelGGL((table_commit_kernel<false, 8, 14>), g, b, 0, stream, t, tr, ev);
        }
        RH_HIP(hipGetLastError());
    }
    return RH_OK;
}

int rh_table_lease(const rh::TableDev& t, int64_t now_nanos, int64_t timeout_ms, uint64_t* d_slot_bits,
                   hipStream_t stream) {
    for (int i = 0; i < rh::kTableTiers; ++i) {
        const TableTier& tt = t.tier[i];
        if (!tt.rows) continue;
        switch (tt.width) {
            case 2: launch_lease_width<2>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 4: launch_lease_width<4>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 6: launch_lease_width<6>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 8: launch_lease_width<8>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 10: launch_lease_width<10>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 12: launch_lease_width<12>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            case 14: launch_lease_width<14>(tt, now_nanos, timeout_ms, d_slot_bits, stream); break;
            default: return rh::fail(RH_E_STATE, "rh_lease_batch: unexpected tier width");
        }
        RH_HIP(hipGetLastError());
    }
    return RH_OK;
}

int rh_table_read(const rh::TableDev& t, uint32_t first, uint32_t n, uint8_t column, int64_t* d_out,
                  hipStream_t stream) {
    if (n == 0) return RH_OK;
    hipLaunchKernelGGL(table_read_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, t, first, n, (uint32_t)column, d_out);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
