// libratis_hip C ABI (include/ratis_hip.h): contexts, the resident group table, host-buffer
// conveniences.  Kernels live in commit.hip and crc32c.hip.
#include <algorithm>
#include <cstring>
#include <string>
#include <new>
#include <vector>

#include "rh_internal.h"

#define RH_EXPORT extern "C" __attribute__((visibility("default")))

namespace rh {

static thread_local std::string t_err;

void set_error(const std::string& msg) { t_err = msg; }

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    t_err = std::string(what) + ": " + hipGetErrorString(e);
    return RH_E_DEVICE;
}

}  // namespace rh

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// The stream is used exactly as given (NULL = the HIP null stream, which is also what a
// PyTorch default stream reports); the context stream is only used by the rh_groups calls.
hipStream_t pick_stream(rh_ctx*, void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

// ---- rh_groups ---------------------------------------------------------------------------
struct rh_groups {
    rh_ctx* ctx = nullptr;
    uint64_t capacity = 0;
    uint64_t stride = 0;  // padded column length (multiple of 64 => 16-byte aligned columns)
    uint32_t nf = 0;
    int64_t gap = -1;
    int64_t* match = nullptr;    // [nf][stride]
    int64_t* fcommit = nullptr;  // [nf][stride]
    int64_t* flush = nullptr;    // [stride]
    int64_t* commit = nullptr;   // [stride]
    int64_t* tstart = nullptr;   // [stride]
    uint32_t* conf = nullptr;    // [stride]
    int64_t* min_out = nullptr;  // [stride]
    int64_t* maj_out = nullptr;  // [stride]
    int64_t* max_out = nullptr;  // [stride]
    uint64_t* valid_bits = nullptr;
    uint64_t* adv_rows = nullptr;
    int64_t* adv_commit = nullptr;
    unsigned long long* adv_count = nullptr;
    // delta staging: two pinned host slots (the producer fills one while the other's H2D is in
    // flight) and one device buffer (stream order serialises H2D -> apply -> next H2D)
    std::mutex mu;
    rh_delta* h_ring[2] = {nullptr, nullptr};
    hipEvent_t ring_free[2] = {nullptr, nullptr};  // recorded after the slot's H2D
    bool ring_used[2] = {false, false};
    int ring_next = 0;
    int ring_acquired = -1;                        // slot handed out by rh_deltas_acquire
    rh_delta* d_deltas = nullptr;
    size_t delta_cap = 0;
};

// ---- context -----------------------------------------------------------------------------
RH_EXPORT int rh_abi_version(void) { return RH_ABI_VERSION; }

RH_EXPORT const char* rh_last_error(void) { return rh::t_err.c_str(); }

RH_EXPORT int rh_device_count(int* out) {
    if (!out) return rh::fail(RH_E_INVAL, "rh_device_count: out == NULL");
    int n = 0;
    RH_HIP(hipGetDeviceCount(&n));
    *out = n;
    return RH_OK;
}

RH_EXPORT int rh_init(int device, rh_ctx** out) {
    if (!out) return rh::fail(RH_E_INVAL, "rh_init: out == NULL");
    *out = nullptr;
    int n = 0;
    RH_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return rh::fail(RH_E_INVAL, "rh_init: no such device");
    DeviceGuard g(device);
    if (!g.ok) return rh::fail(RH_E_DEVICE, "rh_init: hipSetDevice failed");
    hipDeviceProp_t prop;
    RH_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return rh::fail(RH_E_DEVICE, std::string("rh_init: libratis_hip is built for gfx950, device is ") +
                                         prop.gcnArchName);
    rh_ctx* ctx = new (std::nothrow) rh_ctx();
    if (!ctx) return rh::fail(RH_E_NOMEM, "rh_init: out of host memory");
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return rh::hip_fail(e, "hipStreamCreateWithFlags");
    }
    int rc = rh_crc_upload_tables(ctx);
    if (rc != RH_OK) {
        (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return rc;
    }
    *out = ctx;
    return RH_OK;
}

RH_EXPORT int rh_shutdown(rh_ctx* ctx) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_shutdown: ctx == NULL");
    DeviceGuard g(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_slice);
    (void)hipFree(ctx->d_shift);
    (void)hipFree(ctx->d_lane16);
    (void)hipFree(ctx->d_scratch);
    if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return RH_OK;
}

RH_EXPORT int rh_synchronize(rh_ctx* ctx) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_synchronize: ctx == NULL");
    DeviceGuard g(ctx->device);
    RH_HIP(hipStreamSynchronize(ctx->stream));
    return RH_OK;
}

RH_EXPORT void* rh_ctx_stream(rh_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// ---- commit ------------------------------------------------------------------------------
RH_EXPORT int rh_commit_soa_launch(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_commit_launch_impl(ctx, tiers, n_tiers, pick_stream(ctx, stream));
}

namespace {

template <typename T>
int dalloc(T** p, size_t count) {
    if (count == 0) {
        *p = nullptr;
        return RH_OK;
    }
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) return rh::fail(RH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return RH_OK;
}

void free_groups(rh_groups* g) {
    (void)hipFree(g->match);
    (void)hipFree(g->fcommit);
    (void)hipFree(g->flush);
    (void)hipFree(g->commit);
    (void)hipFree(g->tstart);
    (void)hipFree(g->conf);
    (void)hipFree(g->min_out);
    (void)hipFree(g->maj_out);
    (void)hipFree(g->max_out);
    (void)hipFree(g->valid_bits);
    (void)hipFree(g->adv_rows);
    (void)hipFree(g->adv_commit);
    (void)hipFree(g->adv_count);
    (void)hipFree(g->d_deltas);
    for (int i = 0; i < 2; ++i) {
        if (g->h_ring[i]) (void)hipHostFree(g->h_ring[i]);
        if (g->ring_free[i]) (void)hipEventDestroy(g->ring_free[i]);
    }
}

// Waits until ring slot i may be overwritten (its previous H2D has completed).
int ring_wait(rh_groups* g, int i) {
    if (g->ring_used[i]) RH_HIP(hipEventSynchronize(g->ring_free[i]));
    return RH_OK;
}

// Enqueues H2D of the first n deltas of slot i and the device apply; does not wait.
int ring_submit(rh_groups* g, int i, size_t n) {
    hipStream_t s = g->ctx->stream;
    RH_HIP(hipMemcpyAsync(g->d_deltas, g->h_ring[i], n * sizeof(rh_delta), hipMemcpyHostToDevice, s));
    RH_HIP(hipEventRecord(g->ring_free[i], s));
    g->ring_used[i] = true;
    g->ring_next = i ^ 1;
    return rh_apply_deltas_impl(s, g->d_deltas, n, g->capacity, g->stride, g->nf, g->match, g->fcommit, g->flush,
                                g->commit);
}

// Fills n int64 with `v` on `s` (hipMemsetD32-free: a tiny kernel is overkill, use a host pattern).
int fill_i64(int64_t* d, uint64_t n, int64_t v, hipStream_t s) {
    if (n == 0) return RH_OK;
    if (v == -1) {
        RH_HIP(hipMemsetAsync(d, 0xFF, n * sizeof(int64_t), s));
        return RH_OK;
    }
    std::vector<int64_t> h(n, v);
    RH_HIP(hipMemcpyAsync(d, h.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
    RH_HIP(hipStreamSynchronize(s));
    return RH_OK;
}

bool conf_fits(uint32_t conf, uint32_t nf) {
    const uint32_t fmask = (1u << nf) - 1u;
    const uint32_t newf = conf & 0x3FFFu, oldf = (conf >> RH_CONF_OLD_SHIFT) & 0x3FFFu;
    return (newf & ~fmask) == 0 && (oldf & ~fmask) == 0;
}

}  // namespace

RH_EXPORT int rh_groups_create(rh_ctx* ctx, uint64_t capacity, uint32_t n_followers, int64_t gap_threshold,
                               rh_groups** out) {
    if (!ctx || !out) return rh::fail(RH_E_INVAL, "rh_groups_create: ctx/out == NULL");
    *out = nullptr;
    if (capacity == 0) return rh::fail(RH_E_INVAL, "rh_groups_create: capacity == 0");
    if (n_followers < 1 || n_followers > RH_MAX_FOLLOWERS)
        return rh::fail(RH_E_RANGE, "rh_groups_create: n_followers must be in [1, 14]");
    if (gap_threshold < -1) return rh::fail(RH_E_INVAL, "rh_groups_create: gap_threshold must be -1 or >= 0");
    DeviceGuard dg(ctx->device);
    rh_groups* g = new (std::nothrow) rh_groups();
    if (!g) return rh::fail(RH_E_NOMEM, "rh_groups_create: out of host memory");
    g->ctx = ctx;
    g->capacity = capacity;
    g->stride = (capacity + 63) / 64 * 64;
    g->nf = n_followers;
    g->gap = gap_threshold;
    const uint64_t S = g->stride;
    int rc = RH_OK;
    if (rc == RH_OK) rc = dalloc(&g->match, (size_t)n_followers * S);
    if (rc == RH_OK) rc = dalloc(&g->fcommit, (size_t)n_followers * S);
    if (rc == RH_OK) rc = dalloc(&g->flush, S);
    if (rc == RH_OK) rc = dalloc(&g->commit, S);
    if (rc == RH_OK) rc = dalloc(&g->tstart, S);
    if (rc == RH_OK) rc = dalloc(&g->conf, S);
    if (rc == RH_OK) rc = dalloc(&g->min_out, S);
    if (rc == RH_OK) rc = dalloc(&g->maj_out, S);
    if (rc == RH_OK) rc = dalloc(&g->max_out, S);
    if (rc == RH_OK) rc = dalloc(&g->valid_bits, S / 64);
    if (rc == RH_OK) rc = dalloc(&g->adv_rows, S);
    if (rc == RH_OK) rc = dalloc(&g->adv_commit, S);
    if (rc == RH_OK) rc = dalloc(&g->adv_count, 1);
    g->delta_cap = RH_DELTA_SLOT;
    if (rc == RH_OK) rc = dalloc(&g->d_deltas, g->delta_cap);
    for (int i = 0; i < 2 && rc == RH_OK; ++i) {
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&g->h_ring[i]), g->delta_cap * sizeof(rh_delta));
        if (e != hipSuccess) rc = rh::fail(RH_E_NOMEM, "hipHostMalloc(delta staging)");
        if (rc == RH_OK && hipEventCreateWithFlags(&g->ring_free[i], hipEventDisableTiming) != hipSuccess)
            rc = rh::fail(RH_E_DEVICE, "hipEventCreate(delta staging)");
    }
    hipStream_t s = ctx->stream;
    // every index starts at INVALID_LOG_INDEX (-1), every slot inactive (conf 0)
    if (rc == RH_OK) rc = fill_i64(g->match, (uint64_t)n_followers * S, -1, s);
    if (rc == RH_OK) rc = fill_i64(g->fcommit, (uint64_t)n_followers * S, -1, s);
    if (rc == RH_OK) rc = fill_i64(g->flush, S, -1, s);
    if (rc == RH_OK) rc = fill_i64(g->commit, S, -1, s);
    if (rc == RH_OK) rc = fill_i64(g->tstart, S, INT64_MAX, s);
    if (rc == RH_OK) {
        hipError_t e = hipMemsetAsync(g->conf, 0, S * sizeof(uint32_t), s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = rh::hip_fail(e, "rh_groups_create: init");
    }
    if (rc != RH_OK) {
        free_groups(g);
        delete g;
        return rc;
    }
    *out = g;
    return RH_OK;
}

RH_EXPORT int rh_groups_destroy(rh_groups* g) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_destroy: NULL");
    DeviceGuard dg(g->ctx->device);
    (void)hipStreamSynchronize(g->ctx->stream);
    free_groups(g);
    delete g;
    return RH_OK;
}

RH_EXPORT int rh_group_set(rh_groups* g, uint64_t slot, uint32_t conf, int64_t flush_index, int64_t commit_index,
                           int64_t term_start) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_group_set: groups == NULL");
    return rh_groups_load(g, slot, 1, nullptr, nullptr, &flush_index, &commit_index, &term_start, &conf);
}

RH_EXPORT int rh_groups_load(rh_groups* g, uint64_t first, uint64_t n, const int64_t* match,
                             const int64_t* fcommit, const int64_t* flush, const int64_t* commit,
                             const int64_t* term_start, const uint32_t* conf) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_load: groups == NULL");
    if (first > g->capacity || n > g->capacity - first)
        return rh::fail(RH_E_INVAL, "rh_groups_load: rows out of range");
    if (n == 0) return RH_OK;
    if (conf)
        for (uint64_t i = 0; i < n; ++i)
            if (!conf_fits(conf[i], g->nf))
                return rh::fail(RH_E_INVAL, "rh_groups_load: conf word names a follower slot >= n_followers");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    hipStream_t s = g->ctx->stream;
    const uint64_t S = g->stride;
    for (uint32_t k = 0; k < g->nf; ++k) {
        if (match) RH_HIP(hipMemcpyAsync(g->match + k * S + first, match + (uint64_t)k * n, n * 8, hipMemcpyHostToDevice, s));
        if (fcommit)
            RH_HIP(hipMemcpyAsync(g->fcommit + k * S + first, fcommit + (uint64_t)k * n, n * 8, hipMemcpyHostToDevice, s));
    }
    if (flush) RH_HIP(hipMemcpyAsync(g->flush + first, flush, n * 8, hipMemcpyHostToDevice, s));
    if (commit) RH_HIP(hipMemcpyAsync(g->commit + first, commit, n * 8, hipMemcpyHostToDevice, s));
    if (term_start) RH_HIP(hipMemcpyAsync(g->tstart + first, term_start, n * 8, hipMemcpyHostToDevice, s));
    if (conf) RH_HIP(hipMemcpyAsync(g->conf + first, conf, n * 4, hipMemcpyHostToDevice, s));
    RH_HIP(hipStreamSynchronize(s));
    return RH_OK;
}

RH_EXPORT int rh_push_deltas(rh_groups* g, const rh_delta* deltas, size_t n) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_push_deltas: groups == NULL");
    if (n == 0) return RH_OK;
    if (!deltas) return rh::fail(RH_E_INVAL, "rh_push_deltas: deltas == NULL");
    for (size_t i = 0; i < n; ++i) {
        const rh_delta& d = deltas[i];
        const uint32_t c = d.column;
        const bool ok_col = c < g->nf || (c >= 16 && c < 16 + g->nf) || c == RH_COL_FLUSH || c == RH_COL_COMMITTED;
        if (d.slot >= g->capacity || !ok_col)
            return rh::fail(RH_E_INVAL, "rh_push_deltas: delta " + std::to_string(i) + " has a bad slot/column");
    }
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->ring_acquired >= 0) return rh::fail(RH_E_STATE, "rh_push_deltas: a staging slot is acquired");
    for (size_t done = 0; done < n;) {
        const size_t m = std::min(n - done, g->delta_cap);
        const int i = g->ring_next;
        int rc = ring_wait(g, i);
        if (rc == RH_OK) {
            std::memcpy(g->h_ring[i], deltas + done, m * sizeof(rh_delta));
            rc = ring_submit(g, i, m);
        }
        if (rc != RH_OK) return rc;
        done += m;
    }
    return RH_OK;
}

RH_EXPORT int rh_deltas_acquire(rh_groups* g, rh_delta** out_buf, size_t* out_cap) {
    if (!g || !out_buf || !out_cap) return rh::fail(RH_E_INVAL, "rh_deltas_acquire: NULL argument");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->ring_acquired >= 0) return rh::fail(RH_E_STATE, "rh_deltas_acquire: a slot is already acquired");
    const int i = g->ring_next;
    int rc = ring_wait(g, i);
    if (rc != RH_OK) return rc;
    g->ring_acquired = i;
    *out_buf = g->h_ring[i];
    *out_cap = g->delta_cap;
    return RH_OK;
}

RH_EXPORT int rh_deltas_submit(rh_groups* g, size_t n) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_deltas_submit: groups == NULL");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    const int i = g->ring_acquired;
    if (i < 0) return rh::fail(RH_E_STATE, "rh_deltas_submit: no slot acquired");
    if (n > g->delta_cap) return rh::fail(RH_E_INVAL, "rh_deltas_submit: n exceeds the slot capacity");
    g->ring_acquired = -1;
    if (n == 0) return RH_OK;
    return ring_submit(g, i, n);
}

namespace {

rh_commit_soa table_tier(rh_groups* g, int mode) {
    rh_commit_soa t{};
    t.n = g->capacity;
    t.n_followers = g->nf;
    t.mode = mode;
    t.gap_threshold = mode == RH_MODE_COMMIT ? g->gap : -1;
    t.col_stride = g->stride;
    t.conf = g->conf;
    if (mode == RH_MODE_COMMIT) {
        t.follower_index = g->match;
        t.self_index = g->flush;
        t.commit_in = g->commit;
        t.term_start = g->tstart;
        t.commit_out = g->commit;
        t.min_out = g->min_out;
        t.adv_rows = g->adv_rows;
        t.adv_commit = g->adv_commit;
        t.adv_count = g->adv_count;
        t.adv_cap = g->stride;
    } else {
        t.follower_index = g->fcommit;
        t.self_index = g->commit;  // lastCommittedIndex is the self value (LSI:613)
        t.min_out = g->min_out;
        t.maj_out = g->maj_out;
        t.max_out = g->max_out;
        t.valid_bits = g->valid_bits;
    }
    return t;
}

}  // namespace

RH_EXPORT int rh_commit_batch(rh_groups* g, uint64_t* out_slots, int64_t* out_commit, size_t cap, size_t* out_n,
                              int64_t* out_min) {
    if (!g || !out_n) return rh::fail(RH_E_INVAL, "rh_commit_batch: groups/out_n == NULL");
    if (cap && (!out_slots || !out_commit)) return rh::fail(RH_E_INVAL, "rh_commit_batch: output arrays required");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    hipStream_t s = g->ctx->stream;
    RH_HIP(hipMemsetAsync(g->adv_count, 0, sizeof(unsigned long long), s));
    rh_commit_soa t = table_tier(g, RH_MODE_COMMIT);
    int rc = rh_commit_launch_impl(g->ctx, &t, 1, s);
    if (rc != RH_OK) return rc;
    unsigned long long cnt = 0;
    RH_HIP(hipMemcpyAsync(&cnt, g->adv_count, sizeof(cnt), hipMemcpyDeviceToHost, s));
    if (out_min) RH_HIP(hipMemcpyAsync(out_min, g->min_out, g->capacity * 8, hipMemcpyDeviceToHost, s));
    RH_HIP(hipStreamSynchronize(s));
    const size_t m = std::min<size_t>((size_t)cnt, cap);
    if (m) {
        RH_HIP(hipMemcpyAsync(out_slots, g->adv_rows, m * 8, hipMemcpyDeviceToHost, s));
        RH_HIP(hipMemcpyAsync(out_commit, g->adv_commit, m * 8, hipMemcpyDeviceToHost, s));
        RH_HIP(hipStreamSynchronize(s));
    }
    *out_n = (size_t)cnt;
    return RH_OK;
}

RH_EXPORT int rh_watch_levels(rh_groups* g, int64_t* out_min, int64_t* out_maj, int64_t* out_max,
                              uint64_t* out_valid_bits) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_watch_levels: groups == NULL");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    hipStream_t s = g->ctx->stream;
    rh_commit_soa t = table_tier(g, RH_MODE_WATCH);
    int rc = rh_commit_launch_impl(g->ctx, &t, 1, s);
    if (rc != RH_OK) return rc;
    const size_t n8 = g->capacity * 8;
    if (out_min) RH_HIP(hipMemcpyAsync(out_min, g->min_out, n8, hipMemcpyDeviceToHost, s));
    if (out_maj) RH_HIP(hipMemcpyAsync(out_maj, g->maj_out, n8, hipMemcpyDeviceToHost, s));
    if (out_max) RH_HIP(hipMemcpyAsync(out_max, g->max_out, n8, hipMemcpyDeviceToHost, s));
    if (out_valid_bits)
        RH_HIP(hipMemcpyAsync(out_valid_bits, g->valid_bits, (g->capacity + 63) / 64 * 8, hipMemcpyDeviceToHost, s));
    RH_HIP(hipStreamSynchronize(s));
    return RH_OK;
}

RH_EXPORT int rh_groups_read_commit(rh_groups* g, uint64_t first, uint64_t n, int64_t* out) {
    if (!g || (!out && n)) return rh::fail(RH_E_INVAL, "rh_groups_read_commit: NULL argument");
    if (first > g->capacity || n > g->capacity - first)
        return rh::fail(RH_E_INVAL, "rh_groups_read_commit: rows out of range");
    if (n == 0) return RH_OK;
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    RH_HIP(hipMemcpyAsync(out, g->commit + first, n * 8, hipMemcpyDeviceToHost, g->ctx->stream));
    RH_HIP(hipStreamSynchronize(g->ctx->stream));
    return RH_OK;
}

// ---- CRC32C --------------------------------------------------------------------------------
RH_EXPORT int rh_crc32c_frames_launch(rh_ctx* ctx, const rh_frames* frames, uint32_t flags, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_crc32c_frames_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_crc_launch_impl(ctx, frames, flags, pick_stream(ctx, stream));
}

// ---- leader lease ----------------------------------------------------------------------------
RH_EXPORT int rh_lease_soa_launch(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_lease_soa_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_lease_launch_impl(ctx, tiers, n_tiers, pick_stream(ctx, stream));
}

// ---- segment framing -------------------------------------------------------------------------
RH_EXPORT int rh_segments_scan_launch(rh_ctx* ctx, const rh_segments* segs, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_segments_scan_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_segments_launch_impl(ctx, segs, pick_stream(ctx, stream));
}

RH_EXPORT int rh_segments_read_launch(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_segments_read_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_segments_read_impl(ctx, segs, crc, pick_stream(ctx, stream));
}

RH_EXPORT int rh_crc32c(rh_ctx* ctx, uint32_t crc_state, const void* data, uint64_t n, uint32_t* out_state) {
    if (!ctx || !out_state) return rh::fail(RH_E_INVAL, "rh_crc32c: ctx/out_state == NULL");
    if (n && !data) return rh::fail(RH_E_INVAL, "rh_crc32c: data == NULL");
    if (n > 0x7FFFFFFFull) return rh::fail(RH_E_RANGE, "rh_crc32c: span longer than 2^31 - 1 (Java int length)");
    *out_state = crc_state;
    if (n == 0) return RH_OK;
    DeviceGuard g(ctx->device);
    std::lock_guard<std::mutex> lk(ctx->mu);
    const size_t o_len = (n + 255) / 256 * 256, total = o_len + 256;
    if (ctx->scratch_bytes < total) {
        (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
        hipError_t e = hipMalloc(&ctx->d_scratch, total);
        if (e != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_crc32c: device scratch");
        ctx->scratch_bytes = total;
    }
    uint8_t* base = static_cast<uint8_t*>(ctx->d_scratch);
    hipStream_t s = ctx->stream;
    // frame table of one span: offset 0 (8 B), length n (4 B), crc out (4 B)
    struct {
        uint64_t off;
        uint32_t len;
        uint32_t crc;
    } hdr{0, (uint32_t)n, 0};
    RH_HIP(hipMemcpyAsync(base, data, n, hipMemcpyHostToDevice, s));
    RH_HIP(hipMemcpyAsync(base + o_len, &hdr, sizeof(hdr), hipMemcpyHostToDevice, s));
    rh_frames f{};
    f.buf = base;
    f.buf_len = n;
    f.frame_off = reinterpret_cast<const uint64_t*>(base + o_len);
    f.frame_len = reinterpret_cast<const uint32_t*>(base + o_len + 8);
    f.n = 1;
    f.init_state = crc_state;
    f.crc_out = reinterpret_cast<uint32_t*>(base + o_len + 12);
    int rc = rh_crc_launch_impl(ctx, &f, 0, s);
    if (rc != RH_OK) return rc;
    uint32_t value = 0;
    RH_HIP(hipMemcpyAsync(&value, base + o_len + 12, 4, hipMemcpyDeviceToHost, s));
    RH_HIP(hipStreamSynchronize(s));
    *out_state = ~value;  // getValue() = ~crc
    return RH_OK;
}

RH_EXPORT int rh_crc32c_verify_host(rh_ctx* ctx, const uint8_t* seg, uint64_t seg_len, const uint64_t* frame_off,
                                    const uint32_t* frame_len, uint64_t n, uint32_t* crc_out, uint64_t* bad_bits,
                                    uint64_t* n_bad) {
    if (!ctx || !n_bad) return rh::fail(RH_E_INVAL, "rh_crc32c_verify_host: ctx/n_bad == NULL");
    if (n && (!seg || !frame_off || !frame_len)) return rh::fail(RH_E_INVAL, "rh_crc32c_verify_host: NULL input");
    *n_bad = 0;
    if (n == 0) return RH_OK;
    DeviceGuard g(ctx->device);
    std::lock_guard<std::mutex> lk(ctx->mu);
    const size_t nwords = (n + 63) / 64;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_seg = 0, o_off = al(seg_len), o_len = o_off + al(n * 8), o_crc = o_len + al(n * 4),
                 o_bad = o_crc + al(n * 4), o_cnt = o_bad + al(nwords * 8), total = o_cnt + 256;
    if (ctx->scratch_bytes < total) {
        (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
        hipError_t e = hipMalloc(&ctx->d_scratch, total);
        if (e != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_crc32c_verify_host: device scratch");
        ctx->scratch_bytes = total;
    }
    uint8_t* base = static_cast<uint8_t*>(ctx->d_scratch);
    hipStream_t s = ctx->stream;
    RH_HIP(hipMemcpyAsync(base + o_seg, seg, seg_len, hipMemcpyHostToDevice, s));
    RH_HIP(hipMemcpyAsync(base + o_off, frame_off, n * 8, hipMemcpyHostToDevice, s));
    RH_HIP(hipMemcpyAsync(base + o_len, frame_len, n * 4, hipMemcpyHostToDevice, s));
    RH_HIP(hipMemsetAsync(base + o_bad, 0, nwords * 8 + 256, s));
    rh_frames f{};
    f.buf = base + o_seg;
    f.buf_len = seg_len;
    f.frame_off = reinterpret_cast<const uint64_t*>(base + o_off);
    f.frame_len = reinterpret_cast<const uint32_t*>(base + o_len);
    f.n = n;
    f.init_state = 0xFFFFFFFFu;
    f.crc_out = reinterpret_cast<uint32_t*>(base + o_crc);
    f.bad_bits = reinterpret_cast<uint64_t*>(base + o_bad);
    f.n_bad = reinterpret_cast<unsigned long long*>(base + o_cnt);
    int rc = rh_crc_launch_impl(ctx, &f, RH_CRC_VERIFY, s);
    if (rc != RH_OK) return rc;
    unsigned long long cnt = 0;
    if (crc_out) RH_HIP(hipMemcpyAsync(crc_out, base + o_crc, n * 4, hipMemcpyDeviceToHost, s));
    if (bad_bits) RH_HIP(hipMemcpyAsync(bad_bits, base + o_bad, nwords * 8, hipMemcpyDeviceToHost, s));
    RH_HIP(hipMemcpyAsync(&cnt, base + o_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
    RH_HIP(hipStreamSynchronize(s));
    *n_bad = cnt;
    return RH_OK;
}
