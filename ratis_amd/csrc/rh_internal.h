// Internal declarations shared by the libratis_hip translation units (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ratis_hip.h"

namespace rh {

// Thread-local error slot behind rh_last_error().
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define RH_HIP(call)                                          \
    do {                                                      \
        hipError_t _e = (call);                               \
        if (_e != hipSuccess) return ::rh::hip_fail(_e, #call); \
    } while (0)

// ---- CRC32C constants (reflected Castagnoli 0x82F63B78, PureJavaCrc32C.java:154-688) ----
// Slicing tables T_k[b] = CRC register after absorbing byte b followed by k zero bytes.
// shift tables Z_j: linear map "advance the register over 2^j * unit zero bytes", 4 x 256.
struct CrcTables {
    uint32_t slice[4][256];
};
void build_crc_slice_tables(CrcTables* t);
// Zero-advance map for `nbytes` zero bytes, as 4 byte-indexed tables (out[4][256]).
void build_crc_shift_table(uint64_t nbytes, uint32_t out[4][256]);
std::vector<uint32_t> build_crc_lane_tables(int Q, int S);
// Packed CRC kernel: inverse lane maps (advance BACK over 64 (31 - c) zero bytes, c = 0..31,
// nibble layout [c][8][16]) and the init term A^k(init) for spans k = 0..kCrcInitSpan.
std::vector<uint32_t> build_crc_inverse_lane_tables();
constexpr uint32_t kCrcInitSpan = 65535;
std::vector<uint32_t> build_crc_init_terms(uint32_t init);

// The kernel's by-value argument struct, addressed in the kernarg segment (address space 4).
// Indexing a tier array of the argument with a block-dependent index through this pointer gives
// scalar loads from the kernarg segment; indexing the by-value parameter directly can make the
// compiler copy the whole struct into scratch first (seen at 440-1240 bytes per lane).  Valid
// for kernels whose only explicit argument is that struct (it then starts the segment).
template <typename T>
__device__ __forceinline__ const T& kernarg_struct() {
    return *(const T*)(__builtin_amdgcn_kernarg_segment_ptr());
}

// ---- resident table (rh_groups) device layout --------------------------------------------------
// Tier t holds slots whose conf names follower slots < width = 2 (t + 1); every column is a
// contiguous array over the tier's rows (row space), so the commit kernels see a tier exactly as
// an rh_commit_soa.  slot_map: slot -> (tier << 28) | row, kNoRow = stopped.
constexpr int kTableTiers = 7;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr uint32_t kRowMask = 0x0FFFFFFFu;
__host__ __device__ inline int tier_of_width(uint32_t w) { return w <= 2 ? 0 : (int)((w + 1) / 2) - 1; }
__host__ __device__ inline uint32_t width_of_tier(int t) { return 2u * (uint32_t)(t + 1); }

struct TableTier {
    uint32_t width = 0;         // follower columns F
    uint32_t rows = 0;          // allocated rows (column stride), multiple of 128
    int64_t* match = nullptr;   // [F][rows] FollowerInfo.matchIndex
    int64_t* fcommit = nullptr; // [F][rows] FollowerInfo.commitIndex
    int64_t* flush = nullptr;   // [rows] leader flushIndex
    int64_t* commit = nullptr;  // [rows] leader commitIndex (lastCommittedIndex)
    int64_t* tstart = nullptr;  // [rows] first index of the current term
    uint32_t* conf = nullptr;   // [rows] membership word (0 on free rows)
    uint32_t* row_slot = nullptr;  // [rows] row -> slot
    int64_t* wall = nullptr;    // [rows] last watch-ALL level of updateCommit (INT64_MIN = none)
    int64_t* wmin = nullptr;    // [rows] last commitIndexChanged levels
    int64_t* wmaj = nullptr;
    int64_t* wmax = nullptr;
    uint8_t* dirty = nullptr;   // [rows] 1 = updateCommit pending
    uint8_t* wdirty = nullptr;  // [rows] 1 = commitIndexChanged pending
    int64_t* fts = nullptr;     // [F][rows] FollowerInfo.lastRespondedAppendEntriesSendTime (nanos,
                                //           kNoTimestamp until the module sets it)
    int64_t* lease = nullptr;   // [rows] LeaderLease.lease (nanos)
    uint8_t* lon = nullptr;     // [rows] LeaderLease.enabled
};
// A follower column that has no lastRespondedAppendEntriesSendTime yet (a FollowerInfo the module
// has not stamped): never active, never the majority-ack time.
constexpr int64_t kNoTimestamp = INT64_MIN;

struct TableDev {
    TableTier tier[kTableTiers];
    uint32_t* slot_map = nullptr;  // [capacity]
    uint64_t capacity = 0;
    int64_t gap = -1;
};

// Control operations on rows (rh_group_start / reconf / stop), applied in parallel by
// table_control_kernel: within one launch every slot and every destination row appears once and
// no destination row is a source row (the host splits and defers row reuse to guarantee it).
enum CtrlKind : uint32_t { kCtrlStart = 1, kCtrlMove = 2, kCtrlStop = 3, kCtrlReconf = 4 };
struct CtrlOp {
    uint32_t kind;
    uint32_t slot;
    uint32_t dst;     // (tier << 28) | row written (START / MOVE / RECONF)
    uint32_t src;     // (tier << 28) | row read (MOVE / RECONF) or freed (STOP)
    uint32_t conf;
    int8_t map[RH_MAX_FOLLOWERS];  // dst follower column k <- src column map[k] (-1: new FollowerInfo)
    uint16_t pad;
    int64_t flush, commit, tstart;  // START
};

// Event sinks of the table kernels.  Records go to adv / wall / watch (host-mapped pinned memory,
// or HBM under RH_EVENTS_DEVICE).  Every workgroup takes its range of the lists from one device
// counter word (kind 0 in the low 32 bits, kind 1 in the high 32) and writes the end of its range
// (packed the same way) into its own entry of `block_end`, host-mapped memory: the host reads the
// list lengths as the maxima over those entries, so no memset and no read-back of the counter sits
// on the stream.  The counters alternate between two words per kind of evaluation: a launch
// counts into `counts` and clears `counts_next`, the word the following evaluation counts into.
struct TableEvents {
    rh_index_event* adv = nullptr;     // COMMIT: advanced
    rh_index_event* wall = nullptr;    // COMMIT: watch-ALL changes
    rh_watch_event* watch = nullptr;   // WATCH: level changes
    unsigned long long* counts = nullptr;       // device word of this evaluation (zero at launch)
    unsigned long long* counts_next = nullptr;  // device word of the next one: cleared by block 0
    uint64_t* block_end = nullptr;              // host-mapped [blocks]: packed end of each block's range
    uint32_t block_base = 0;                     // this launch's first entry in block_end
    uint64_t cap = 0;
};
// Workgroups the table evaluation launches for a table (both width classes): the size of the
// block_end array an evaluation needs.
uint32_t table_commit_blocks(const TableDev& t);

}  // namespace rh

struct rh_ctx {
    int device = -1;
    hipStream_t stream = nullptr;
    int num_cus = 0;
    // device copies of the CRC tables
    uint32_t* d_slice = nullptr;   // [4][256]
    uint32_t* d_shift = nullptr;   // [41][4][256]: zero-advance maps over 2^m bytes, m = 0..40
    uint32_t* d_lane16 = nullptr;  // lane-distance nibble tables (Q = 2, 4, 8, 16, 32 lanes x 64 B)
    uint32_t* d_inv32 = nullptr;   // [32][8][16] inverse lane maps of the packed CRC kernel
    uint32_t* d_initff = nullptr;  // [kCrcInitSpan + 1] advance of reset()'s 0xFFFFFFFF over k zero bytes
    std::mutex pool_mu;  // guards the pool's creation
    void* h_pinned = nullptr;
    size_t pinned_bytes = 0;
    hipMemPool_t pool = nullptr;  // stream-ordered scratch (rh::pool_alloc)
};

// Launchers implemented in the .hip files (device pointers, async on `stream`).
namespace rh {
// Stream-ordered device scratch from the context's memory pool (created on first use, keeps its
// memory cached between calls): free with hipFreeAsync on the same stream.
hipError_t pool_alloc(rh_ctx* ctx, void** p, size_t bytes, hipStream_t stream);
// Pool scratch released (hipFreeAsync on its stream) on every exit path, error returns included.
struct PoolScratch {
    void* p = nullptr;
    hipStream_t s;
    explicit PoolScratch(hipStream_t stream) : s(stream) {}
    ~PoolScratch() {
        if (p) (void)hipFreeAsync(p, s);
    }
    PoolScratch(const PoolScratch&) = delete;
    PoolScratch& operator=(const PoolScratch&) = delete;
    hipError_t alloc(rh_ctx* ctx, size_t bytes) { return pool_alloc(ctx, &p, bytes, s); }
    uint8_t* bytes() const { return static_cast<uint8_t*>(p); }
};
}  // namespace rh

int rh_commit_launch_impl(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, hipStream_t stream);
// Resident table kernels (table.hip): delta apply (phase 0 = SET deltas, 1 = MAX deltas),
// control ops, and updateCommit / commitIndexChanged over the dirty rows of every tier.
int rh_table_apply_deltas(const rh::TableDev& t, const rh_delta* d_deltas, uint64_t n, int phase, hipStream_t stream);
int rh_table_control(const rh::TableDev& t, const rh::CtrlOp* d_ops, uint64_t n, hipStream_t stream);
int rh_table_commit(const rh::TableDev& t, int mode, const rh::TableEvents& ev, hipStream_t stream);
int rh_table_lease(const rh::TableDev& t, int64_t now_nanos, int64_t timeout_ms, uint64_t* d_slot_bits,
                   hipStream_t stream);
int rh_table_read(const rh::TableDev& t, uint32_t first, uint32_t n, uint8_t column, int64_t* d_out,
                  hipStream_t stream);
int rh_crc_launch_impl(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream);
int rh_crc_upload_tables(rh_ctx* ctx);
int rh_segments_launch_impl(rh_ctx* ctx, const rh_segments* segs, hipStream_t stream);
int rh_segments_read_impl(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, hipStream_t stream);
// *dense_written: whether the pass also wrote crc->crc_out / bad_bits (the length-class plan);
// else the caller compacts them from the slots.
int rh_crc_verify_slots(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, hipStream_t stream,
                        bool* dense_written);
int rh_lease_launch_impl(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, hipStream_t stream);
int rh_lease_validate(const rh_lease_soa* tiers, int n_tiers);
int rh_lease_launch_class(const rh_lease_soa* tiers, int n_tiers, int flo, int fhi, hipStream_t stream);
int rh_leader_launch_impl(rh_ctx* ctx, const rh_commit_soa* commit, int n_commit, const rh_lease_soa* lease,
                          int n_lease, hipStream_t stream);
