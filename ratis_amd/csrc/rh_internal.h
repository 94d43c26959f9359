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
// Tier t holds slots whose conf names follower slots < width = 2 (t + 1).  Rows come in TILES of
// kTileRows = 128 (one wave of the evaluation kernel: two rows per lane): a tile holds its 128
// elements of every column back to back, so one wave's reads of a column are one contiguous 1 KiB
// run and an updateCommit evaluation reads ONE contiguous run per tile (the rh_commit_soa TILED
// layout, commit.hip).  Byte offsets inside a tile of a tier with F follower columns (tile::):
//
//   [0, 128)      dirty    u8    1 = updateCommit pending (UPDATE_COMMIT event, LSI:846-854)
//   [128, 256)    wdirty   u8    1 = commitIndexChanged pending
//   [256, 384)    lon      u8    LeaderLease.enabled
//   [512, 1024)   conf     u32   membership word (0 on free rows)
//   [1024, 1536)  row_slot u32   row -> slot (kNoRow on free rows)
//   then int64 columns of 1 KiB each, addressed by these offsets (tile::match(k) ...):
//   match[F] flush tstart commit wall | fcommit[F] wmin wmaj wmax | fts[F] lease
//   and stored (tile::pair_off) as the commit column, then three sections of records of
//   kGroupRows rows: [match[F] flush tstart wall] [fcommit[F] wmin wmaj wmax] [fts[F] lease] --
//   each section still one contiguous run per tile.
//
// COMMIT reads dirty + [conf .. wall] (one run), WATCH wdirty + conf, row_slot, commit, fcommit..wmax,
// the lease pass conf + fts + lease.  slot_map: slot -> (tier << 28) | row, kNoRow = stopped.
// Beside the tiles a per-tier SUMMARY of two bytes per tile (sum[2 tile] = some row of the tile is
// dirty, sum[2 tile + 1] = some row is wdirty), set by every kernel that sets a flag: an evaluation
// wave whose tile is clean returns after reading that byte, without touching the tile.
constexpr int kTableTiers = 7;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr uint32_t kRowMask = 0x0FFFFFFFu;
constexpr uint32_t kTileRows = 128;
__host__ __device__ inline int tier_of_width(uint32_t w) { return w <= 2 ? 0 : (int)((w + 1) / 2) - 1; }
__host__ __device__ inline uint32_t width_of_tier(int t) { return 2u * (uint32_t)(t + 1); }

namespace tile {
constexpr uint32_t kDirty = 0, kWdirty = 128, kLon = 256, kConf = 512, kSlot = 1024, kMatch = 1536;
__host__ __device__ constexpr uint32_t match(uint32_t k) { return kMatch + 1024u * k; }
__host__ __device__ constexpr uint32_t flush(uint32_t F) { return kMatch + 1024u * F; }
__host__ __device__ constexpr uint32_t tstart(uint32_t F) { return flush(F) + 1024u; }
__host__ __device__ constexpr uint32_t commit(uint32_t F) { return flush(F) + 2048u; }
__host__ __device__ constexpr uint32_t wall(uint32_t F) { return flush(F) + 3072u; }
__host__ __device__ constexpr uint32_t fcommit(uint32_t F, uint32_t k) { return kMatch + 1024u * (F + 4 + k); }
__host__ __device__ constexpr uint32_t wmin(uint32_t F) { return fcommit(F, F); }
__host__ __device__ constexpr uint32_t wmaj(uint32_t F) { return wmin(F) + 1024u; }
__host__ __device__ constexpr uint32_t wmax(uint32_t F) { return wmin(F) + 2048u; }
__host__ __device__ constexpr uint32_t fts(uint32_t F, uint32_t k) { return kMatch + 1024u * (2 * F + 7 + k); }
__host__ __device__ constexpr uint32_t lease(uint32_t F) { return fts(F, F); }
__host__ __device__ constexpr uint32_t bytes(uint32_t F) { return kMatch + 1024u * (3 * F + 8); }
// Byte offset in a tile of the 16 bytes that hold rows 2p and 2p + 1 of the int64 column at tile
// offset `off` (a match / flush / ... offset above; row 2p + 1 at + 8).  Round 5: the commit column
// stays a column (both evaluations read it); the others are grouped in three sections --
// [match[F] flush tstart wall] | [fcommit[F] wmin wmaj wmax] | [fts[F] lease] -- each stored as
// records of kGroupRows rows (per record: each column's kGroupRows values in turn), so a row's
// updateCommit inputs are F + 3 values kGroupRows x 8 bytes apart instead of 1 KiB apart (list
// mode: fewer random lines per row), while a tile wave still reads each section as one contiguous
// run.  kGroupRows = 128 is the plain column layout.
#ifndef RH_TABLE_GROUP
#define RH_TABLE_GROUP 128
#endif
constexpr uint32_t kGroupRows = RH_TABLE_GROUP;
static_assert(kGroupRows >= 2 && kGroupRows <= 128 && (kGroupRows & (kGroupRows - 1)) == 0, "a power of two");
__host__ __device__ constexpr uint32_t pair_off(uint32_t F, uint32_t off, uint32_t p) {
    const uint32_t c = (off - kMatch) >> 10;   // int64 column index in the tile:: order
    const uint32_t r = 2u * p;
    if (c == F + 2) return kMatch + 16u * p;   // commit
    const uint32_t base = c < F + 4 ? kMatch + 1024u : c < 2 * F + 7 ? kMatch + 1024u * (F + 4) : kMatch + 1024u * (2 * F + 7);
    const uint32_t ns = c < 2 * F + 7 ? F + 3 : F + 1;
    const uint32_t j = c < F + 2 ? c : c < F + 4 ? c - 1 : c < 2 * F + 7 ? c - (F + 4) : c - (2 * F + 7);
    return base + (r / kGroupRows) * (kGroupRows * 8u * ns) + j * 8u * kGroupRows + 8u * (r % kGroupRows);
}
// Byte offset in a tile of element r (0..127) of the column at tile offset `off`, element size sz.
__host__ __device__ constexpr uint32_t elem_off(uint32_t F, uint32_t off, uint32_t r, uint32_t sz) {
    return off >= kMatch ? pair_off(F, off, r >> 1) + 8u * (r & 1u) : off + r * sz;
}
}  // namespace tile

struct TableTier {
    uint32_t width = 0;         // follower columns F
    uint32_t rows = 0;          // allocated rows, a multiple of kTileRows
    uint8_t* base = nullptr;    // [rows / 128] tiles of tile::bytes(width)
    uint8_t* sum = nullptr;     // [rows / 128][2] tile summaries (dirty, wdirty)
    // Delta order keys, laid out like `base` (the key of the int64 cell at tile offset o, row r, sits at
    // the same offset of `shadow`; the u8 lease-enabled cell's key uses the conf / row-slot bytes,
    // which no delta targets): (batch generation << 32) | index in the batch of the cell's last SET.
    uint8_t* shadow = nullptr;
    // element `r` of the column at tile offset `off` (element size sizeof(T))
    template <typename T>
    __host__ __device__ T* at(uint32_t off, uint64_t r) const {
        return reinterpret_cast<T*>(base + (r >> 7) * (uint64_t)tile::bytes(width) +
                                    tile::elem_off(width, off, (uint32_t)(r & 127), (uint32_t)sizeof(T)));
    }
    // the order key of the delta target at tile offset `off` (int64 column, or tile::kLon)
    __host__ __device__ unsigned long long* key(uint32_t off, uint64_t r) const {
        const uint32_t o = off == tile::kLon ? tile::kConf : off;
        return reinterpret_cast<unsigned long long*>(shadow + (r >> 7) * (uint64_t)tile::bytes(width) +
                                                     tile::elem_off(width, o, (uint32_t)(r & 127), 8u));
    }
    __host__ __device__ int64_t* i64(uint32_t off, uint64_t r) const { return at<int64_t>(off, r); }
    __host__ __device__ uint32_t* u32(uint32_t off, uint64_t r) const { return at<uint32_t>(off, r); }
    __host__ __device__ uint8_t* u8(uint32_t off, uint64_t r) const { return at<uint8_t>(off, r); }
    __host__ __device__ uint8_t* summary(uint64_t r, int watch) const { return sum + 2 * (r >> 7) + watch; }
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

// Event lists of the evaluation kernels, written straight into the result lists of the sink
// (pinned host memory or HBM).  A workgroup gathers its records (LDS), takes ONE range of each list
// with ONE device-scope atomic on the evaluation's counter word `cnt` and copies them out
// contiguously.  The word holds kind 0 in bits [0, cbits) and kind 1 in [cbits, 2 cbits) (advanced /
// watch-ALL for COMMIT, level changes for WATCH; cbits = 24 for capacities below 2^24, else 28)
// and, when they fit above (`packed`: always in the list kernel, whose grid is at most 240
// workgroups; in the tile kernels below 2^16 workgroups at cbits 24), the workgroups done -- so one
// atomic both reserves a workgroup's range and tells the last one the totals.  Otherwise the tile
// kernels count themselves on the separate `done` word.  The workgroup completing the
// evaluation's count (done_target: the workgroups of every launch of it) writes the two list
// lengths to counts_out (host-mapped) and zeroes the words for the next evaluation: no gather
// pass, no memset, no count read-back on the stream.
constexpr int kHeads = 8;          // dirty-row list regions, one per XCD head (below)
constexpr int kHeadStride = 32;    // u64 words between head / counter words: each on its own 256-B line
struct TableEvents {
    rh_index_event* adv = nullptr;     // COMMIT: advanced (the result list)
    rh_index_event* wall = nullptr;    // COMMIT: watch-ALL changes, or null (not reported)
    rh_watch_event* watch = nullptr;   // WATCH: level changes
    uint64_t cap = 0;                  // records per list
    unsigned long long* cnt = nullptr; // the evaluation's counter word (zero at its first launch)
    unsigned int* done = nullptr;      // workgroups done in this launch (zero at launch)
    uint64_t* counts_out = nullptr;    // [2] list lengths (host-mapped)
    uint32_t cbits = 28;               // bits per count in `cnt`
    int packed = 0;                    // tile kernels: the done count rides in `cnt` above the counts
    uint32_t done_target = 0;          // tile kernels: workgroups done that end the evaluation (0: not this launch)
    unsigned long long* lheads_next = nullptr;  // the other list-head set of the evaluated kind: cleared
    // REGION mode (tile kernels into the DEVICE / AUTO sinks): no counter atomic, no LDS staging.
    // Workgroup gb (block_base + its block index: the evaluation's launches number their workgroups
    // on) has descriptor gb, kTableDesc u32 at bdesc + gb * kTableDesc, and writes no records: the
    // descriptor is the totals (u64: list a | list b << 32) and per wave four u64 masks, bit L for
    // rows 2L / 2L + 1 -- COMMIT: advanced rows, then changed watch-ALL rows; WATCH: rows whose
    // levels changed, then which of them are valid.  The evaluation has stored the new values in the
    // table, so rh_table_gather_commit / _watch rebuild the records from the masks and the table's
    // columns (the host orders every later writer of those columns after the gather).  (One
    // returning atomic per workgroup on one word, at every workgroup's end, cost the 1M-row
    // evaluation 4.5 us; the COMMIT records themselves 1.6 us of the 19.3.)
    uint32_t* bdesc = nullptr;
    uint32_t block_base = 0;
    // REGION mode of the list kernel: descriptor gb = pass * grid + workgroup, wave w's masks at
    // [1 + 4 w] (bit j: the wave's lane j's listed row in that pass) and [3 + 4 w] (COMMIT: watch-ALL
    // changed; WATCH: valid), [2 + 4 w] = [4 + 4 w] = 0.  list_passes: the host's bound on the passes
    // (rh::table_list_passes); descriptors of passes the evaluation does not run are zeroed.
    uint32_t list_passes = 0;
};
// The fused tick's events (rh_tick_async, table_tick_kernel): both evaluations' records straight
// into the pinned lists.  cnt: three u64 words kHeadStride apart -- the commit lists' counter
// (advanced | watch-ALL << 32), the level records' counter, the workgroups done (u32) -- zero between
// launches (the last workgroup zeroes them).
struct TickEvents {
    rh_index_event* adv = nullptr;
    rh_index_event* wall = nullptr;    // null: watch-ALL changes not reported
    rh_watch_event* watch = nullptr;
    uint64_t cap = 0;
    unsigned long long* cnt = nullptr;
    uint64_t* counts_c = nullptr;      // [2] host-mapped: advanced, watch-ALL
    uint64_t* counts_w = nullptr;      // [2] host-mapped: level records, 0
    unsigned long long* lheads_next_c = nullptr;   // the other list-head sets: cleared
    unsigned long long* lheads_next_w = nullptr;
};
// Tile-kernel workgroup: RH_TABLE_BLOCK_WAVES waves, one 128-row tile each.  REGION mode: records
// per workgroup region (its rows) and u32 counts per workgroup descriptor (2 totals + 2 per wave).
#ifndef RH_TABLE_BLOCK_WAVES   // A/B builds (both table.hip and groups.cpp see it)
#define RH_TABLE_BLOCK_WAVES 2
#endif
constexpr uint32_t kTableRecs = RH_TABLE_BLOCK_WAVES * 128;
constexpr uint32_t kTableDesc = 2 + 8 * RH_TABLE_BLOCK_WAVES;   // u32: COMMIT's u64 totals + 4 u64 masks per wave
// DIRTY-ROW LISTS (list mode).  While the host knows that few rows can be dirty (the deltas and
// control ops since the last evaluation of a kind bound the rows they can mark), every 0 -> 1
// transition of a row's dirty / wdirty flag (found with a 32-bit atomicOr on the flag's word) also
// appends the row to a list: kHeads regions (one per XCD head, the writer's blockIdx & 7) of `cap`
// entries, each with its own head word; an entry is (tier << 28) | row.  The evaluation then runs
// over the listed rows only (table_list_kernel: work proportional to the dirty rows, not to the
// table).  Two head sets per kind alternate: appends go to `heads`; the evaluation that consumes
// them clears the other set.
struct TableLists {
    uint32_t* rows = nullptr;            // [kHeads][cap] entries: (tier << 28) | row within the tier
    unsigned long long* heads = nullptr; // [kHeads] words, kHeadStride apart (null: no list)
    uint32_t cap = 0;
};

// Workgroups the table evaluation launches for a table (both width classes).
uint32_t table_commit_blocks(const TableDev& t);
// The list kernel's grid for `rows_hint` marked rows, a bound on its passes over lists of at most
// `rows` entries (each pass: one entry per lane of every wave), and the most descriptors a
// REGION-mode list evaluation of lists of capacity `cap` per region can write.
uint32_t table_list_grid(uint64_t rows_hint);
uint32_t table_list_passes(uint32_t grid, uint64_t rows);
uint64_t table_list_desc_blocks(uint64_t cap);
// A REGION-mode list evaluation's rows, for its gather: the list (entries per region: cap) and grid.
struct ListRegion {
    const uint32_t* rows = nullptr;   // null: a tile evaluation
    uint32_t cap = 0;
    uint32_t grid = 0;
};

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
    uint32_t* d_slice8 = nullptr;  // [8][256]: PureJavaCrc32C's slicing-by-8 tables (T[k] = T[k-1] + one zero byte)
    std::vector<uint32_t> h_initff;  // host copy of d_initff (rh_crc32c_stamp_host's zero-copy plan)
    unsigned int stamp_seq = 0;   // zero-copy plan: the last call's completion number
    std::mutex pool_mu;  // guards the pool's creation
    std::mutex stage_mu;  // guards the pinned staging below (rh_crc32c_stamp_host's frame table / CRCs)
    void* h_pinned = nullptr;
    size_t pinned_bytes = 0;
    hipMemPool_t pool = nullptr;  // stream-ordered scratch (rh::pool_alloc)
    // Pinned bounce buffers for transfers of CALLER host memory (rh::h2d / rh::d2h): the HIP runtime
    // is never handed pageable memory the library does not own (it would page-lock it behind the
    // call, and a lock that outlives the caller's buffer is a GPU mapping of freed pages -- DESIGN
    // §11).  Two buffers of kBounceBytes, each with the event of the last copy that used it.
    std::mutex bounce_mu;
    uint8_t* bounce[2] = {nullptr, nullptr};
    hipEvent_t bounce_ev[2] = {nullptr, nullptr};
    bool bounce_used[2] = {false, false};
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

// Transfers between CALLER host memory and the device on `s`.  A range inside one registration the
// runtime knows (rh_host_register, hipHostMalloc) is copied directly; any other range goes through
// the context's pinned bounce buffers in kBounceBytes chunks (the memcpy of chunk k + 1 overlaps the
// DMA of chunk k).  h2d: enqueued, `src` reusable on return.  d2h: `dst` holds the bytes on return
// (it waits for the stream).
constexpr uint64_t kBounceBytes = 4ull << 20;
// (*dev: the device address of p, when registered)
bool host_registered(const void* p, uint64_t n, void** dev = nullptr);
int h2d(rh_ctx* ctx, void* dst, const void* src, uint64_t n, hipStream_t s);
int d2h(rh_ctx* ctx, void* dst, const void* src, uint64_t n, hipStream_t s);
}  // namespace rh

int rh_commit_launch_impl(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, hipStream_t stream);
// Resident table kernels (table.hip): delta apply (phase 0 = SET deltas, 1 = MAX deltas),
// control ops, and updateCommit / commitIndexChanged over the dirty rows of every tier.
// Phases of one batch (rh_delta order semantics, ratis_hip.h): kApplyKeys records each SET target's
// last SET (the highest batch index: its order key in the tier's shadow), kApplySet stores the SET
// that holds its target's key, kApplyMax applies the MAX deltas that come after their target's last
// SET (all of them when gen == 0: a batch without SETs).  gen: the batch generation (>= 1) of the
// keys, 0 for a batch without SETs.
enum ApplyPhase : int { kApplySet = 0, kApplyMax = 1, kApplyKeys = 2 };
// resolved: the deltas' slot fields hold row codes (tier << 28 | row), resolved by rh_push_deltas.
int rh_table_apply_deltas(const rh::TableDev& t, const rh_delta* d_deltas, uint64_t n, int phase, uint32_t gen,
                          const rh::TableLists& lc, const rh::TableLists& lw, hipStream_t stream, bool resolved);
// List-mode evaluation of the listed rows of one kind (mode); COMMIT appends the rows whose commit
// advanced to the watch list `lw` (when it is maintained).  Events as rh_table_commit.
// t0 / t1 (may be null): timing events stamped at the evaluation's kernel boundaries.
int rh_table_commit_lists(const rh::TableDev& t, int mode, const rh::TableLists& l, const rh::TableLists& lw,
                          const rh::TableEvents& ev, hipStream_t stream, hipEvent_t t0, hipEvent_t t1, uint64_t rows_hint);
int rh_table_control(const rh::TableDev& t, const rh::CtrlOp* d_ops, uint64_t n, hipStream_t stream);
// The pump's tick in one launch: updateCommit over the commit list lc, commitIndexChanged over the rows
// of the watch list lw and the rows whose commit advanced (table.hip, table_tick_kernel).
int rh_table_tick_lists(const rh::TableDev& t, const rh::TableLists& lc, const rh::TableLists& lw, const rh::TickEvents& ev,
                        hipStream_t stream, hipEvent_t t0, hipEvent_t t1, uint64_t rows_hint);
// spec: issue every column load with the dirty-flag load (a large part of the table is dirty).
int rh_table_commit(const rh::TableDev& t, int mode, const rh::TableEvents& ev, bool spec, hipStream_t stream,
                    hipEvent_t t0, hipEvent_t t1);
// Copies the counted prefixes of HBM result lists into the pinned lists (device pointers of the
// host mapping): list a (records of rec_bytes0 = 16 or 32 B, length counts[0]) and, if b is not
// null, list b (16 B records, length counts[1]); counts = the host-mapped lengths the evaluation
// published.  Enqueued on `stream` (ordered after the evaluation by the caller).
// REGION mode, COMMIT: the records of an evaluation (its clipped table `t`, as given to
// rh_table_commit) rebuilt from the descriptors' masks and the table's row-slot, commit and
// watch-ALL columns into the pinned lists adv_out / wall_out (device pointers; wall_out null: no
// watch-ALL list), lengths to counts_out.  Nothing may write those columns between the evaluation
// and this kernel (groups.cpp gather_fence).
// A list evaluation's records (lr.rows set): the same, its rows from the list entries of the masks'
// lanes -- nothing may append to that list either until the gather has run.
// t0 / t1 (may be null): timing events stamped at the gather kernel's boundaries.
int rh_table_gather_commit(const rh::TableDev& t, const uint32_t* bdesc, uint32_t n_blocks, rh_index_event* adv_out,
                           rh_index_event* wall_out, uint64_t* counts_out, hipStream_t stream,
                           const rh::ListRegion& lr = rh::ListRegion{}, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// REGION mode, WATCH: the level records (slot, valid, min, majority, max) of an evaluation rebuilt
// the same way from the masks (changed rows, valid flags) and the row-slot / wmin / wmaj / wmax
// columns into the pinned list `out` (device pointer), its length to counts_out[0].
int rh_table_gather_watch(const rh::TableDev& t, const uint32_t* bdesc, uint32_t n_blocks, rh_watch_event* out,
                          uint64_t* counts_out, hipStream_t stream, const rh::ListRegion& lr = rh::ListRegion{},
                          hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// n 64-bit words from device memory to a host-mapped pinned buffer (device view), as GPU writes.
int rh_table_copy_words(const uint64_t* src, uint64_t* dst, uint64_t n, hipStream_t stream);
int rh_table_drain(const uint64_t* counts, const void* a, void* a_out, const void* b, void* b_out, uint32_t rec_bytes0,
                   uint64_t cap, hipStream_t stream);
// Initialises tiles [first_tile, n_tiles) of a tier as free rows (conf 0, row_slot kNoRow, clean).
int rh_table_init_tiles(const rh::TableTier& t, uint32_t first_tile, uint32_t n_tiles, hipStream_t stream);
// hasLease over every row into the zeroed bitmap d_slot_bits; the launch also zeroes d_clear_bits
// (clear_words words: the next pass's bitmap).
int rh_table_lease(const rh::TableDev& t, int64_t now_nanos, int64_t timeout_ms, uint64_t* d_slot_bits,
                   uint64_t* d_clear_bits, uint32_t clear_words, hipStream_t stream);
int rh_table_read(const rh::TableDev& t, uint32_t first, uint32_t n, uint8_t column, int64_t* d_out,
                  hipStream_t stream);
// window_only: every frame on the window kernel (one launch, no packed pass): small batches
int rh_crc_launch_impl(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream, bool window_only = false);
// One lane per frame (crc_serial_kernel): small batches of well-formed frames (no bad bits / counts).
int rh_crc_serial_launch(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream);

// rh_crc32c_stamp_host's zero-copy plan (a buffer registered with rh_host_register): one launch,
// no copies, no device scratch.  The batch's frames are dealt in order to workgroups of at most
// kStampSpan bytes of span and kStampMaxWin 64-byte windows (the host sizes them so that the
// batch spreads over up to kStampMaxGroups CUs).  Workgroup g moves its span straight from the
// mapped host buffer, its frame records from the mapped staging and the CRC tables from HBM into
// LDS (LDS-DMA, one round trip), cuts every payload into windows from its end (a scan of the
// window counts; each window's frame found by binary search), folds the windows (the first one's
// bytes before the frame masked), and XORs each window's register, advanced over the bytes after
// it in its frame, into its frame's accumulator (seeded with reset()'s term for the frame's
// length).  The CRCs go to mapped pinned memory, then the workgroup's done flag.
#ifndef RH_STAMP_THREADS      // A/B: threads per workgroup
#define RH_STAMP_THREADS 128
#endif
struct StampGroup {
    uint64_t src;          // device address (host mapping) of the span's first byte, 16-B aligned
    uint32_t frame_first;  // its frames: records / CRCs [frame_first, + frame_n)
    uint32_t bytes_n;      // span bytes (a multiple of 16, <= kStampSpan) << 12 | frame_n
};
constexpr uint32_t kStampThreads = RH_STAMP_THREADS;
constexpr uint32_t kStampSpan = 64 << 10;   // span bytes per workgroup at most (its LDS image)
constexpr uint32_t kStampMaxWin = 1024;     // windows per workgroup at most
constexpr uint32_t kStampMaxFrames = 1024;  // frames per workgroup at most
constexpr uint32_t kStampShifts = 8;        // windows after a window in its frame: < 2^kStampShifts
constexpr uint32_t kStampMaxGroups = 128;   // workgroups per launch (descriptors: kernel arguments)
constexpr uint32_t kStampFront = 64;        // LDS image bytes before the span (a first window starts <= 63 B early)
static_assert(kStampSpan < (1u << 20) && kStampMaxFrames < 4096 && kStampThreads % 64 == 0, "StampGroup.bytes_n");
// frame record in the staging (16 B: one LDS-DMA piece): x = LDS byte position of the payload,
// y = payload bytes, z = reset()'s term for them, w = 0 (the kernel's window prefix)
struct StampArgs {
    StampGroup g[kStampMaxGroups];
    const uint4* frames;        // mapped pinned, per frame
    uint32_t* crc_out;          // mapped pinned, per frame
    unsigned int* done;         // mapped pinned, per workgroup: `seq` once its CRCs are stored
    const uint32_t* slice8;     // device [8][256]
    const uint32_t* shift64;    // device: the zero-advance maps over 64 * 2^b bytes, b = 0..7
    unsigned int seq;
    uint32_t n_shift;           // maps staged (the longest frame's windows - 1 < 2^n_shift)
};
int rh_crc_stamp_mapped_launch(const StampArgs& a, uint32_t n_groups, hipStream_t stream);
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
