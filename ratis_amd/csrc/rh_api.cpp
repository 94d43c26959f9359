// libratis_hip C ABI (include/ratis_hip.h): contexts, the resident group table, host-buffer
// conveniences.  Kernels live in commit.hip and crc32c.hip.
#include <algorithm>
#include <atomic>
#include <chrono>
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

hipError_t rh::pool_alloc(rh_ctx* ctx, void** p, size_t bytes, hipStream_t stream) {
    {
        std::lock_guard<std::mutex> lk(ctx->pool_mu);
        if (!ctx->pool) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = ctx->device;
            hipError_t e = hipMemPoolCreate(&ctx->pool, &props);
            if (e != hipSuccess) {
                ctx->pool = nullptr;
                return e;
            }
            uint64_t keep = UINT64_MAX;  // never trim between calls
            e = hipMemPoolSetAttribute(ctx->pool, hipMemPoolAttrReleaseThreshold, &keep);
            if (e != hipSuccess) return e;
        }
    }
    return hipMallocFromPoolAsync(p, bytes, ctx->pool, stream);
}

// Releases everything the context owns.  The device is drained first -- not only the context's
// stream: pool scratch is freed stream-ordered on whatever stream a launch was given (PoolScratch),
// and a zero-copy stamp may still be completing -- and a fault of that work is returned (the context
// is released all the same), never dropped.
RH_EXPORT int rh_shutdown(rh_ctx* ctx) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_shutdown: ctx == NULL");
    DeviceGuard g(ctx->device);
    hipError_t err = hipStreamSynchronize(ctx->stream);
    const hipError_t e2 = hipDeviceSynchronize();
    if (err == hipSuccess) err = e2;
    (void)hipFree(ctx->d_slice);
    (void)hipFree(ctx->d_shift);
    (void)hipFree(ctx->d_lane16);
    (void)hipFree(ctx->d_inv32);
    (void)hipFree(ctx->d_initff);
    (void)hipFree(ctx->d_slice8);
    if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
    for (int i = 0; i < 2; ++i) {
        if (ctx->bounce[i]) (void)hipHostFree(ctx->bounce[i]);
        if (ctx->bounce_ev[i]) (void)hipEventDestroy(ctx->bounce_ev[i]);
    }
    if (ctx->pool) (void)hipMemPoolDestroy(ctx->pool);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    if (err != hipSuccess) return rh::hip_fail(err, "rh_shutdown: the context's last work");
    return RH_OK;
}

RH_EXPORT int rh_synchronize(rh_ctx* ctx) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_synchronize: ctx == NULL");
    DeviceGuard g(ctx->device);
    RH_HIP(hipStreamSynchronize(ctx->stream));   // (a zero-copy stamp's launch included)
    return RH_OK;
}

// ---- diagnostics: the rate of GPU stores into mapped pinned memory -------------------------------------
// The reference rate for the kernels that write event records across PCIe (the table's gather / drain,
// the hasLease bitmap copy): `bytes` copied from HBM into a mapped pinned buffer by the same 16-byte
// store kernel (rh_table_copy_words), `reps` times on the context stream; *ms = the median launch.
RH_EXPORT int rh_pcie_write_probe(rh_ctx* ctx, uint64_t bytes, int reps, float* ms) {
    if (!ctx || !ms || reps < 1 || bytes < 16 || bytes > (1ull << 32))
        return rh::fail(RH_E_INVAL, "rh_pcie_write_probe: ctx/ms NULL, reps < 1 or bytes outside [16, 4 GiB]");
    DeviceGuard g(ctx->device);
    const uint64_t words = bytes / 8;
    uint64_t* d_src = nullptr;
    void* h_dst = nullptr;
    uint64_t* d_dst = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<float> t;
    int rc = RH_OK;
    if (hipMalloc(reinterpret_cast<void**>(&d_src), words * 8) != hipSuccess ||
        hipHostMalloc(&h_dst, words * 8, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&d_dst), h_dst, 0) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
        rc = rh::fail(RH_E_NOMEM, "rh_pcie_write_probe: buffers");
    }
    if (rc == RH_OK && hipMemsetAsync(d_src, 0x5A, words * 8, ctx->stream) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_pcie_write_probe: memset");
    for (int r = 0; r <= reps && rc == RH_OK; ++r) {   // r = 0: warm-up
        if (hipEventRecord(e0, ctx->stream) != hipSuccess) rc = rh::fail(RH_E_DEVICE, "rh_pcie_write_probe: event");
        if (rc == RH_OK) rc = rh_table_copy_words(d_src, d_dst, words, ctx->stream);
        if (rc == RH_OK && (hipEventRecord(e1, ctx->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess))
            rc = rh::fail(RH_E_DEVICE, "rh_pcie_write_probe: launch");
        float x = 0;
        if (rc == RH_OK && r > 0 && hipEventElapsedTime(&x, e0, e1) == hipSuccess) t.push_back(x);
    }
    if (rc == RH_OK && t.empty()) rc = rh::fail(RH_E_DEVICE, "rh_pcie_write_probe: no timing");
    if (rc == RH_OK) {
        std::sort(t.begin(), t.end());
        *ms = t[t.size() / 2];
    }
    (void)hipStreamSynchronize(ctx->stream);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (h_dst) (void)hipHostFree(h_dst);
    (void)hipFree(d_src);
    return rc;
}

// ---- transfers of caller host memory (rh_internal.h) ------------------------------------------------
bool rh::host_registered(const void* p, uint64_t n, void** dev) {
    if (n == 0) return true;
    void *d0 = nullptr, *d1 = nullptr;
    if (hipHostGetDevicePointer(&d0, const_cast<void*>(p), 0) != hipSuccess ||
        hipHostGetDevicePointer(&d1, const_cast<uint8_t*>(static_cast<const uint8_t*>(p)) + n - 1, 0) != hipSuccess ||
        static_cast<uint8_t*>(d1) - static_cast<uint8_t*>(d0) != (ptrdiff_t)(n - 1)) {
        (void)hipGetLastError();   // a pageable range: not an error
        return false;
    }
    if (dev) *dev = d0;
    return true;
}

namespace {
// The bounce buffers and their events (under bounce_mu).
int bounce_reserve(rh_ctx* ctx) {
    for (int i = 0; i < 2; ++i) {
        if (!ctx->bounce[i] && hipHostMalloc(reinterpret_cast<void**>(&ctx->bounce[i]), rh::kBounceBytes, 0) != hipSuccess) {
            ctx->bounce[i] = nullptr;
            return rh::fail(RH_E_NOMEM, "pinned bounce buffer");
        }
        if (!ctx->bounce_ev[i]) RH_HIP(hipEventCreateWithFlags(&ctx->bounce_ev[i], hipEventDisableTiming));
    }
    return RH_OK;
}
}  // namespace

int rh::h2d(rh_ctx* ctx, void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (n == 0) return RH_OK;
    if (host_registered(src, n)) {
        RH_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s));
        return RH_OK;
    }
    std::lock_guard<std::mutex> lk(ctx->bounce_mu);
    int rc = bounce_reserve(ctx);
    if (rc != RH_OK) return rc;
    const uint8_t* in = static_cast<const uint8_t*>(src);
    uint8_t* out = static_cast<uint8_t*>(dst);
    for (uint64_t off = 0, k = 0; off < n; off += kBounceBytes, ++k) {
        const int i = (int)(k & 1);
        const uint64_t c = std::min<uint64_t>(kBounceBytes, n - off);
        if (ctx->bounce_used[i]) RH_HIP(hipEventSynchronize(ctx->bounce_ev[i]));   // its last copy has read it
        std::memcpy(ctx->bounce[i], in + off, c);
        RH_HIP(hipMemcpyAsync(out + off, ctx->bounce[i], c, hipMemcpyHostToDevice, s));
        RH_HIP(hipEventRecord(ctx->bounce_ev[i], s));
        ctx->bounce_used[i] = true;
    }
    return RH_OK;
}

int rh::d2h(rh_ctx* ctx, void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (n == 0) return RH_OK;
    if (host_registered(dst, n)) {
        RH_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s));
        RH_HIP(hipStreamSynchronize(s));
        return RH_OK;
    }
    std::lock_guard<std::mutex> lk(ctx->bounce_mu);
    int rc = bounce_reserve(ctx);
    if (rc != RH_OK) return rc;
    const uint8_t* in = static_cast<const uint8_t*>(src);
    uint8_t* out = static_cast<uint8_t*>(dst);
    // chunk k lands in buffer k & 1; the host drains chunk k - 1 while chunk k is in flight
    const uint64_t chunks = (n + kBounceBytes - 1) / kBounceBytes;
    for (uint64_t k = 0; k <= chunks; ++k) {
        if (k < chunks) {
            const int i = (int)(k & 1);
            if (ctx->bounce_used[i]) RH_HIP(hipEventSynchronize(ctx->bounce_ev[i]));
            const uint64_t off = k * kBounceBytes, c = std::min<uint64_t>(kBounceBytes, n - off);
            RH_HIP(hipMemcpyAsync(ctx->bounce[i], in + off, c, hipMemcpyDeviceToHost, s));
            RH_HIP(hipEventRecord(ctx->bounce_ev[i], s));
            ctx->bounce_used[i] = true;
        }
        if (k > 0) {
            const int i = (int)((k - 1) & 1);
            const uint64_t off = (k - 1) * kBounceBytes, c = std::min<uint64_t>(kBounceBytes, n - off);
            RH_HIP(hipEventSynchronize(ctx->bounce_ev[i]));
            std::memcpy(out + off, ctx->bounce[i], c);
        }
    }
    return RH_OK;
}



RH_EXPORT void* rh_ctx_stream(rh_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// ---- commit ------------------------------------------------------------------------------
RH_EXPORT int rh_commit_soa_launch(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_commit_soa_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_commit_launch_impl(ctx, tiers, n_tiers, pick_stream(ctx, stream));
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

RH_EXPORT int rh_leader_soa_launch(rh_ctx* ctx, const rh_commit_soa* commit, int n_commit, const rh_lease_soa* lease,
                                   int n_lease, void* stream) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_leader_soa_launch: ctx == NULL");
    DeviceGuard g(ctx->device);
    return rh_leader_launch_impl(ctx, commit, n_commit, lease, n_lease, pick_stream(ctx, stream));
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

// ---- single span on the host: the SURVEY 8(b) rh_crc32c contract (pure, reentrant) -------------
// PureJavaCrc32C's register (PJC:54-91: c = (c >>> 8) ^ T[(c ^ b) & 0xff], reflected Castagnoli
// polynomial 0x82F63B78, no inversion inside update) is exactly what the SSE4.2 CRC32 instruction
// advances, 8 bytes per instruction; without it, a byte-wise table built once.  Not a fallback of the
// batched paths: those stay on the GPU; this serves the odd single span where a PCIe round trip would
// cost more than the span (a snapshot file's checksum, a Java caller's one-off update).
namespace {
const uint32_t* host_crc_table() {
    static const std::vector<uint32_t> t = [] {
        std::vector<uint32_t> v(256);
        for (uint32_t b = 0; b < 256; ++b) {
            uint32_t c = b;
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            v[b] = c;
        }
        return v;
    }();
    return t.data();
}

__attribute__((target("sse4.2"))) uint32_t crc_sse42(uint32_t c, const uint8_t* p, uint64_t n) {
    uint64_t c64 = c;
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7); --n) c64 = __builtin_ia32_crc32qi((uint32_t)c64, *p++);
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        c64 = __builtin_ia32_crc32di(c64, w);
    }
    for (; n; --n) c64 = __builtin_ia32_crc32qi((uint32_t)c64, *p++);
    return (uint32_t)c64;
}
}  // namespace

RH_EXPORT uint32_t rh_crc32c_update(uint32_t crc_state, const void* data, uint64_t n) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (!p || n == 0) return crc_state;
    static const bool sse42 = __builtin_cpu_supports("sse4.2");
    if (sse42) return crc_sse42(crc_state, p, n);
    const uint32_t* t = host_crc_table();
    uint32_t c = crc_state;
    for (uint64_t i = 0; i < n; ++i) c = (c >> 8) ^ t[(c ^ p[i]) & 0xffu];
    return c;
}

RH_EXPORT int rh_crc32c(rh_ctx* ctx, uint32_t crc_state, const void* data, uint64_t n, uint32_t* out_state) {
    if (!ctx || !out_state) return rh::fail(RH_E_INVAL, "rh_crc32c: ctx/out_state == NULL");
    if (n && !data) return rh::fail(RH_E_INVAL, "rh_crc32c: data == NULL");
    if (n > 0x7FFFFFFFull) return rh::fail(RH_E_RANGE, "rh_crc32c: span longer than 2^31 - 1 (Java int length)");
    *out_state = crc_state;
    if (n == 0) return RH_OK;
    DeviceGuard g(ctx->device);
    // per-call stream-ordered scratch from the context's pool (no shared staging buffer); the work
    // is enqueued on the context stream, so concurrent callers are safe but run one after another
    const size_t o_len = (n + 255) / 256 * 256, total = o_len + 256;
    hipStream_t s = ctx->stream;
    rh::PoolScratch scratch(s);  // released on every exit path
    if (scratch.alloc(ctx, total) != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_crc32c: device scratch");
    uint8_t* base = scratch.bytes();
    // frame table of one span: offset 0 (8 B), length n (4 B), crc out (4 B)
    struct {
        uint64_t off;
        uint32_t len;
        uint32_t crc;
    } hdr{0, (uint32_t)n, 0};
    int rc = rh::h2d(ctx, base, data, n, s);
    if (rc == RH_OK) rc = rh::h2d(ctx, base + o_len, &hdr, sizeof(hdr), s);
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    rh_frames f{};
    f.buf = base;
    f.buf_len = n;
    f.frame_off = reinterpret_cast<const uint64_t*>(base + o_len);
    f.frame_len = reinterpret_cast<const uint32_t*>(base + o_len + 8);
    f.n = 1;
    f.init_state = crc_state;
    f.crc_out = reinterpret_cast<uint32_t*>(base + o_len + 12);
    rc = rh_crc_launch_impl(ctx, &f, 0, s);
    uint32_t value = 0;
    if (rc == RH_OK) rc = rh::d2h(ctx, &value, base + o_len + 12, 4, s);
    RH_HIP(hipStreamSynchronize(s));
    if (rc != RH_OK) return rc;
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
    const size_t nwords = (n + 63) / 64;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_seg = 0, o_off = al(seg_len), o_len = o_off + al(n * 8), o_crc = o_len + al(n * 4),
                 o_bad = o_crc + al(n * 4), o_cnt = o_bad + al(nwords * 8), total = o_cnt + 256;
    hipStream_t s = ctx->stream;
    rh::PoolScratch scratch(s);  // per-call stream-ordered scratch (as rh_crc32c), freed on every exit
    if (scratch.alloc(ctx, total) != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_crc32c_verify_host: device scratch");
    uint8_t* base = scratch.bytes();
    int rc = rh::h2d(ctx, base + o_seg, seg, seg_len, s);
    if (rc == RH_OK) rc = rh::h2d(ctx, base + o_off, frame_off, n * 8, s);
    if (rc == RH_OK) rc = rh::h2d(ctx, base + o_len, frame_len, n * 4, s);
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
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
    rc = rh_crc_launch_impl(ctx, &f, RH_CRC_VERIFY, s);
    unsigned long long cnt = 0;
    if (rc == RH_OK && crc_out) rc = rh::d2h(ctx, crc_out, base + o_crc, n * 4, s);
    if (rc == RH_OK && bad_bits) rc = rh::d2h(ctx, bad_bits, base + o_bad, nwords * 8, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, &cnt, base + o_cnt, sizeof(cnt), s);
    RH_HIP(hipStreamSynchronize(s));
    if (rc != RH_OK) return rc;
    *n_bad = cnt;
    return RH_OK;
}

// ---- write side: the trailers of a flush batch (SegmentedRaftLogOutputStream.write, OUT:86-110) ----
RH_EXPORT int rh_host_register(rh_ctx* ctx, void* p, uint64_t n) {
    if (!ctx || !p || n == 0) return rh::fail(RH_E_INVAL, "rh_host_register: ctx/p == NULL or n == 0");
    DeviceGuard g(ctx->device);
    // every GPU's contexts may read it; mapped: rh_crc32c_stamp_host's kernel reads and stamps it in place
    RH_HIP(hipHostRegister(p, n, hipHostRegisterPortable | hipHostRegisterMapped));
    return RH_OK;
}

// The GPU's mapping of the buffer goes away here: every launch that may still read it -- a zero-copy
// stamp of this or any other context (the registration is portable) returns on polled flags, before
// its completion -- is drained first, and a fault of that work is returned.
RH_EXPORT int rh_host_unregister(rh_ctx* ctx, void* p) {
    if (!ctx || !p) return rh::fail(RH_E_INVAL, "rh_host_unregister: ctx/p == NULL");
    DeviceGuard g(ctx->device);
    const hipError_t e = hipDeviceSynchronize();
    RH_HIP(hipHostUnregister(p));
    if (e != hipSuccess) return rh::hip_fail(e, "rh_host_unregister: work still reading the buffer");
    return RH_OK;
}

// rh_crc32c_stamp_host's plan (A/B builds override): 0 = the span and the frame table copied in,
// one lane per frame (crc_serial_kernel), the CRCs copied back, trailers written by the host; 1 =
// the same copies around the window kernel; 2 = the span copied in, the window kernel reading the
// frame table from and writing the CRCs to the mapped pinned staging (one copy, no D2H).  (Reading
// the frames themselves across PCIe would leave the batch's first frame -- within 67 bytes of the
// mapping's start -- to the window kernel's byte-wise guarded path: a PCIe round trip per 4 bytes.)
#ifndef RH_STAMP_PLAN
#define RH_STAMP_PLAN 2
#endif
// plan 0: frames up to this length go one lane per frame; longer ones to the streaming plans
constexpr uint64_t kSerialMaxFrame = 64 << 10;

#ifndef RH_STAMP_ZERO_COPY   // A/B: the zero-copy plan for registered buffers (1) or never (0)
#define RH_STAMP_ZERO_COPY 1
#endif
#ifndef RH_STAMP_SPIN        // A/B: the zero-copy plan's completion by a polled flag (1) or the stream (0)
#define RH_STAMP_SPIN 1
#endif

namespace {
// Grows the context's pinned staging to `bytes` (under stage_mu).
int stage_reserve(rh_ctx* ctx, uint64_t bytes) {
    if (ctx->pinned_bytes >= bytes) return RH_OK;
    RH_HIP(hipStreamSynchronize(ctx->stream));   // a zero-copy launch may still map the old staging
    if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
    ctx->h_pinned = nullptr;
    ctx->pinned_bytes = 0;
    const size_t want = std::max<size_t>(bytes, (size_t)1 << 20);
    if (hipHostMalloc(&ctx->h_pinned, want, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
        return rh::fail(RH_E_NOMEM, "rh_crc32c_stamp_host: pinned staging");
    ctx->pinned_bytes = want;
    return RH_OK;
}

constexpr int kNotPlanned = 1;   // stamp_zero_copy: the batch does not fit the plan (nothing done)

// rh_crc32c_stamp_host's zero-copy plan (rh_internal.h, StampArgs): the frames dealt in their order
// to workgroups of at most `cap` bytes of span (cap: the batch over 3/4 of kStampMaxGroups
// workgroups, at least kStampThreads windows' worth), kStampMaxWin windows and kStampMaxFrames
// frames; the frame records and CRCs in the pinned staging.  Needs the batch's span inside a
// mapped registration of `buf` (rh_host_register), every payload under 64 * 2^kStampShifts bytes
// and at most kStampMaxGroups workgroups.  Caller holds stage_mu.
int stamp_zero_copy(rh_ctx* ctx, uint8_t* buf, uint64_t lo, uint64_t hi, const uint64_t* frame_off,
                    const uint32_t* frame_len, uint64_t n, uint64_t max_len) {
    // groups of `cap` span bytes: 3/4 of the workgroup limit, the rest slack for frames that do not
    // pack to the cap (a 1 MiB batch of <= 2 KiB entries: ~100 workgroups)
    const uint64_t cap = std::min<uint64_t>(kStampSpan, std::max<uint64_t>(64ull * kStampThreads,
                                                                            ((hi - lo) / (kStampMaxGroups * 3 / 4) + 15) & ~15ull));
    if (!RH_STAMP_ZERO_COPY || max_len - 4 >= (64ull << kStampShifts) || ctx->h_initff.empty() ||
        hi - lo > (uint64_t)kStampMaxGroups * 3 / 4 * kStampSpan)   // would not fit the workgroups
        return kNotPlanned;
    // the workgroups move 16-byte pieces from (offset & ~15) up to (end + 15) & ~15 of `buf`: that
    // whole range, not only the frames, must be mapped for the GPU.  A registration maps whole pages,
    // so the pieces' ends may pass the registered bytes within the pages the frames occupy; past
    // them only if the registration goes on (a batch ending within 15 bytes of a registration that
    // ends on a page boundary would otherwise read the next page -- a GPU page fault)
    const uint64_t r_lo = lo & ~15ull, r_hi = (hi + 15) & ~15ull;
    const auto page = [](const uint8_t* p) { return reinterpret_cast<uintptr_t>(p) >> 12; };
    const uint64_t c_lo = page(buf + r_lo) == page(buf + lo) ? lo : r_lo;
    const uint64_t c_hi = page(buf + r_hi - 1) == page(buf + hi - 1) ? hi : r_hi;
    void* d_c = nullptr;
    if (!rh::host_registered(buf + c_lo, c_hi - c_lo, &d_c)) return kNotPlanned;   // the copying plan
    uint8_t* d_lo = static_cast<uint8_t*>(d_c) + (lo - c_lo);
    StampArgs A{};
    auto al = [](uint64_t x) { return (x + 255) / 256 * 256; };
    const uint64_t o_fr = 0, o_crc = al(n * 16), o_done = o_crc + al(n * 4);
    int rc = stage_reserve(ctx, o_done + al(kStampMaxGroups * 4));
    if (rc != RH_OK) return rc;
    uint8_t* st = static_cast<uint8_t*>(ctx->h_pinned);
    uint4* fr = reinterpret_cast<uint4*>(st + o_fr);
    uint32_t ng = 0, g_win = 0, max_w = 1;
    uint64_t g_lo = 0, g_hi = 0, g_first = 0;
    StampGroup* g = nullptr;
    auto close = [&](uint64_t end) {   // group g's frames [g_first, end): positions in its LDS image
        const uint64_t base = g_lo & ~15ull;
        g->src = reinterpret_cast<uint64_t>(d_lo) + base - lo;
        g->bytes_n = (uint32_t)(((g_hi + 15) & ~15ull) - base) << 12 | (uint32_t)(end - g_first);
        for (uint64_t k = g_first; k < end; ++k) fr[k].x = (uint32_t)(kStampFront + frame_off[k] - base);
    };
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t o = frame_off[i], p = frame_len[i] - 4;
        const uint32_t nw = (uint32_t)((p + 63) / 64);
        max_w = std::max(max_w, nw);
        const uint64_t nlo = std::min(g_lo, o), nhi = std::max(g_hi, o + p);
        if (!g || o < g_lo || ((nhi + 15) & ~15ull) - (nlo & ~15ull) > cap || g_win + nw > kStampMaxWin ||
            i - g_first == kStampMaxFrames) {   // a new workgroup (a frame before the group's start: a new base)
            if (g) close(i);
            if (ng == kStampMaxGroups) return kNotPlanned;
            g = &A.g[ng++];
            g->frame_first = (uint32_t)i;
            g_first = i;
            g_lo = o;
            g_hi = o + p;
            g_win = 0;
        } else {
            g_hi = nhi;
        }
        g_win += nw;
        fr[i].y = (uint32_t)p;
        fr[i].z = ctx->h_initff[p];
        fr[i].w = 0;
    }
    close(n);
    // the shift maps the frames need: j < max_w windows after a window
    uint32_t n_shift = 0;
    while ((1u << n_shift) < max_w) ++n_shift;
    // completion: each workgroup stores the call's number to its flag word in the staging after
    // its CRCs; the host polls them -- a few microseconds less than the stream's completion signal
    // (hipStreamSynchronize follows when a flag is late, and reports any fault)
    volatile unsigned int* done = reinterpret_cast<volatile unsigned int*>(st + o_done);
    for (uint32_t k = 0; k < ng; ++k) done[k] = 0u;
    uint8_t* dst = nullptr;
    RH_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dst), st, 0));
    A.frames = reinterpret_cast<const uint4*>(dst + o_fr);
    A.crc_out = reinterpret_cast<uint32_t*>(dst + o_crc);
    A.done = reinterpret_cast<unsigned int*>(dst + o_done);
    A.slice8 = ctx->d_slice8;
    A.shift64 = ctx->d_shift + (size_t)6 * 1024;   // 2^6 = 64 bytes, then 128, ... (consecutive maps)
    A.seq = ++ctx->stamp_seq;
    if (A.seq == 0) A.seq = ctx->stamp_seq = 1;
    A.n_shift = n_shift;
    hipStream_t s = ctx->stream;
    rc = rh_crc_stamp_mapped_launch(A, ng, s);
    if (rc != RH_OK) return rc;
    bool seen = false;
    if (RH_STAMP_SPIN) {
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t k = 0;
        for (uint32_t it = 0;; ++it) {
            while (k < ng && done[k] == A.seq) ++k;
            if (k == ng) {
                seen = true;
                break;
            }
            if ((it & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    // returned on the flags: every workgroup has made its last access (the flag store); the launch's
    // completion -- and a fault of it -- is met by the next synchronisation of the context stream
    // (rh_synchronize, the staging's growth), rh_host_unregister and rh_shutdown (device drains)
    if (!seen) RH_HIP(hipStreamSynchronize(s));
    const uint32_t* crc = reinterpret_cast<const uint32_t*>(st + o_crc);
    for (uint64_t i = 0; i < n; ++i) {   // buf.putInt((int) checksum.getValue()): big-endian
        uint8_t* t = buf + frame_off[i] + frame_len[i] - 4;
        const uint32_t v = crc[i];
        t[0] = (uint8_t)(v >> 24);
        t[1] = (uint8_t)(v >> 16);
        t[2] = (uint8_t)(v >> 8);
        t[3] = (uint8_t)v;
    }
    return RH_OK;
}
}  // namespace

RH_EXPORT int rh_crc32c_stamp_host(rh_ctx* ctx, uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off,
                                   const uint32_t* frame_len, uint64_t n) {
    if (!ctx) return rh::fail(RH_E_INVAL, "rh_crc32c_stamp_host: ctx == NULL");
    if (n == 0) return RH_OK;
    if (!buf || !frame_off || !frame_len) return rh::fail(RH_E_INVAL, "rh_crc32c_stamp_host: NULL input");
    if (n >= (1ull << 32)) return rh::fail(RH_E_RANGE, "rh_crc32c_stamp_host: n >= 2^32");
    // every frame must lie in the buffer and hold its trailer: nothing is stamped otherwise
    uint64_t lo = UINT64_MAX, hi = 0, max_len = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t o = frame_off[i], l = frame_len[i];
        max_len = std::max(max_len, l);
        if (l < 4 || o > buf_len || l > buf_len - o)
            return rh::fail(RH_E_INVAL, "rh_crc32c_stamp_host: frame " + std::to_string(i) +
                                            " is shorter than its trailer or outside the buffer");
        lo = std::min(lo, o);
        hi = std::max(hi, o + l);
    }
    DeviceGuard g(ctx->device);
    hipStream_t s = ctx->stream;
    // the frame table (offsets relative to the span's start, lengths) and the CRCs in the context's
    // pinned staging
    auto al = [](uint64_t x) { return (x + 255) / 256 * 256; };
    const uint64_t span = hi - lo;
    const uint64_t t_off = 0, t_len = al(n * 8), t_crc = t_len + al(n * 4), t_bytes = t_crc + al(n * 4);
    std::lock_guard<std::mutex> lk(ctx->stage_mu);
    const int zc = stamp_zero_copy(ctx, buf, lo, hi, frame_off, frame_len, n, max_len);
    if (zc != kNotPlanned) return zc;
    const int rs = stage_reserve(ctx, t_bytes);
    if (rs != RH_OK) return rs;
    uint8_t* st = static_cast<uint8_t*>(ctx->h_pinned);
    // the device image has kPad bytes before the span and after it: no frame lies within the window
    // kernel's guard distances of the image ends (67 B before, 8 B after), so none takes its byte-wise
    // guarded path (one dependent load per byte)
    constexpr uint64_t kPad = 128;
    uint64_t* rel = reinterpret_cast<uint64_t*>(st + t_off);
    for (uint64_t i = 0; i < n; ++i) rel[i] = frame_off[i] - lo + kPad;
    std::memcpy(st + t_len, frame_len, n * 4);
    rh_frames f{};
    f.buf_len = kPad + span + kPad;
    f.n = n;
    f.init_state = 0xFFFFFFFFu;   // checksum.reset() before every entry (OUT:100-103)
    // only the span the frames cover crosses PCIe (a flush batch is one contiguous run); the CRCs
    // come back as 4 B per frame and the host writes the big-endian trailers
    const uint64_t o_img = 0, o_tab = al(kPad + span + kPad), total = o_tab + (RH_STAMP_PLAN == 2 ? 0 : t_bytes);
    const uint32_t* crc = reinterpret_cast<const uint32_t*>(st + t_crc);
    rh::PoolScratch scratch(s);
    if (scratch.alloc(ctx, total) != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_crc32c_stamp_host: device scratch");
    uint8_t* base = scratch.bytes();
    int rc = rh::h2d(ctx, base + o_img + kPad, buf + lo, span, s);
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    f.buf = base + o_img;
    // the CRCs come back (crc_out) and the host writes the trailers; the device copy is not stamped
    if (RH_STAMP_PLAN == 2) {   // the frame table and the CRCs through the staging's device mapping
        uint8_t* dst = nullptr;
        RH_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dst), st, 0));
        f.frame_off = reinterpret_cast<const uint64_t*>(dst + t_off);
        f.frame_len = reinterpret_cast<const uint32_t*>(dst + t_len);
        f.crc_out = reinterpret_cast<uint32_t*>(dst + t_crc);
        // up to one window-kernel batch (512 frames, one workgroup) on the window kernel; more
        // frames one lane each over many CUs (its single workgroup per 512 frames would serialise
        // them; measured 996 frames: 88 vs 94 us per call)
        rc = (n > 512 && max_len <= kSerialMaxFrame) ? rh_crc_serial_launch(ctx, &f, RH_CRC_STAMP, s)
                                                   : rh_crc_launch_impl(ctx, &f, RH_CRC_STAMP, s, true);
    } else {
        RH_HIP(hipMemcpyAsync(base + o_tab, st, t_crc, hipMemcpyHostToDevice, s));
        f.frame_off = reinterpret_cast<const uint64_t*>(base + o_tab + t_off);
        f.frame_len = reinterpret_cast<const uint32_t*>(base + o_tab + t_len);
        f.crc_out = reinterpret_cast<uint32_t*>(base + o_tab + t_crc);
        rc = (RH_STAMP_PLAN == 0 && max_len <= kSerialMaxFrame) ? rh_crc_serial_launch(ctx, &f, RH_CRC_STAMP, s)
                                                              : rh_crc_launch_impl(ctx, &f, RH_CRC_STAMP, s, true);
        if (rc == RH_OK) RH_HIP(hipMemcpyAsync(st + t_crc, base + o_tab + t_crc, n * 4, hipMemcpyDeviceToHost, s));
    }
    RH_HIP(hipStreamSynchronize(s));
    if (rc != RH_OK) return rc;
    for (uint64_t i = 0; i < n; ++i) {   // buf.putInt((int) checksum.getValue()): big-endian
        uint8_t* t = buf + frame_off[i] + frame_len[i] - 4;
        const uint32_t c = crc[i];
        t[0] = (uint8_t)(c >> 24);
        t[1] = (uint8_t)(c >> 16);
        t[2] = (uint8_t)(c >> 8);
        t[3] = (uint8_t)c;
    }
    return RH_OK;
}

// ---- host-image read path (LogSegment.readSegmentFile over many files in one call) -------------
RH_EXPORT int rh_segments_read_host(rh_ctx* ctx, const uint8_t* image, uint64_t image_len, const uint64_t* seg_off,
                                    const uint64_t* seg_len, uint64_t n_seg, uint32_t max_op,
                                    uint32_t frames_per_seg_cap, uint64_t* frame_off, uint32_t* frame_len,
                                    uint32_t* frame_crc, uint64_t frame_cap, rh_segment_result* results,
                                    uint64_t* n_frames_total) {
    if (!ctx || !n_frames_total) return rh::fail(RH_E_INVAL, "rh_segments_read_host: ctx/n_frames_total == NULL");
    *n_frames_total = 0;
    if (n_seg == 0) return RH_OK;
    if (!seg_off || !seg_len || !results || (image_len && !image))
        return rh::fail(RH_E_INVAL, "rh_segments_read_host: NULL input");
    if (frame_cap && (!frame_off || !frame_len)) return rh::fail(RH_E_INVAL, "rh_segments_read_host: NULL frame arrays");
    if (frames_per_seg_cap == 0) return rh::fail(RH_E_INVAL, "rh_segments_read_host: frames_per_seg_cap == 0");
    if (n_seg > (1ull << 32)) return rh::fail(RH_E_RANGE, "rh_segments_read_host: too many segments");
    DeviceGuard g(ctx->device);
    const uint64_t slots = n_seg * (uint64_t)frames_per_seg_cap;
    const uint64_t dcap = std::max<uint64_t>(1, std::min<uint64_t>(frame_cap, slots));
    auto al = [](uint64_t x) { return (x + 255) / 256 * 256; };
    // device layout: image | seg_off | seg_len | scratch off/len/crc | dense off/len/crc | per-segment
    // first/nframes/status/stop/ok/read_status/read_stop | total
    uint64_t o = 0;
    const uint64_t o_img = o; o += al(image_len);
    const uint64_t o_soff = o; o += al(n_seg * 8);
    const uint64_t o_slen = o; o += al(n_seg * 8);
    const uint64_t o_xoff = o; o += al(slots * 8);
    const uint64_t o_xlen = o; o += al(slots * 4);
    const uint64_t o_xcrc = o; o += al(slots * 4);
    const uint64_t o_foff = o; o += al(dcap * 8);
    const uint64_t o_flen = o; o += al(dcap * 4);
    const uint64_t o_fcrc = o; o += al(dcap * 4);
    const uint64_t o_first = o; o += al(n_seg * 8);
    const uint64_t o_nfr = o; o += al(n_seg * 4);
    const uint64_t o_st = o; o += al(n_seg * 4);
    const uint64_t o_stop = o; o += al(n_seg * 8);
    const uint64_t o_ok = o; o += al(n_seg * 4);
    const uint64_t o_rst = o; o += al(n_seg * 4);
    const uint64_t o_rstop = o; o += al(n_seg * 8);
    const uint64_t o_tot = o; o += 256;
    hipStream_t s = ctx->stream;
    rh::PoolScratch scratch(s);
    if (scratch.alloc(ctx, o) != hipSuccess) return rh::fail(RH_E_NOMEM, "rh_segments_read_host: device scratch");
    uint8_t* b = scratch.bytes();
    int rc = rh::h2d(ctx, b + o_img, image, image_len, s);
    if (rc == RH_OK) rc = rh::h2d(ctx, b + o_soff, seg_off, n_seg * 8, s);
    if (rc == RH_OK) rc = rh::h2d(ctx, b + o_slen, seg_len, n_seg * 8, s);
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    rh_segments sg{};
    sg.buf = b + o_img;
    sg.buf_len = image_len;
    sg.seg_off = reinterpret_cast<const uint64_t*>(b + o_soff);
    sg.seg_len = reinterpret_cast<const uint64_t*>(b + o_slen);
    sg.n_seg = n_seg;
    sg.max_op = max_op;
    sg.frames_per_seg_cap = frames_per_seg_cap;
    sg.scratch_off = reinterpret_cast<uint64_t*>(b + o_xoff);
    sg.scratch_len = reinterpret_cast<uint32_t*>(b + o_xlen);
    sg.frame_off = reinterpret_cast<uint64_t*>(b + o_foff);
    sg.frame_len = reinterpret_cast<uint32_t*>(b + o_flen);
    sg.frame_cap = dcap;
    sg.seg_first = reinterpret_cast<uint64_t*>(b + o_first);
    sg.seg_nframes = reinterpret_cast<uint32_t*>(b + o_nfr);
    sg.seg_status = reinterpret_cast<int32_t*>(b + o_st);
    sg.seg_stop = reinterpret_cast<uint64_t*>(b + o_stop);
    sg.total_frames = reinterpret_cast<unsigned long long*>(b + o_tot);
    rh_segments_crc cr{};
    cr.scratch_crc = reinterpret_cast<uint32_t*>(b + o_xcrc);
    cr.seg_ok = reinterpret_cast<uint32_t*>(b + o_ok);
    cr.seg_read_status = reinterpret_cast<int32_t*>(b + o_rst);
    cr.seg_read_stop = reinterpret_cast<uint64_t*>(b + o_rstop);
    cr.crc_out = reinterpret_cast<uint32_t*>(b + o_fcrc);
    rc = rh_segments_read_impl(ctx, &sg, &cr, s);
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    std::vector<uint64_t> first, rstop;
    std::vector<uint32_t> nfr, ok;
    std::vector<int32_t> rst;
    try {
        first.resize(n_seg);
        rstop.resize(n_seg);
        nfr.resize(n_seg);
        ok.resize(n_seg);
        rst.resize(n_seg);
    } catch (...) {
        (void)hipStreamSynchronize(s);
        return rh::fail(RH_E_NOMEM, "rh_segments_read_host: out of host memory");
    }
    unsigned long long total = 0;
    rc = rh::d2h(ctx, first.data(), b + o_first, n_seg * 8, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, nfr.data(), b + o_nfr, n_seg * 4, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, ok.data(), b + o_ok, n_seg * 4, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, rst.data(), b + o_rst, n_seg * 4, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, rstop.data(), b + o_rstop, n_seg * 8, s);
    if (rc == RH_OK) rc = rh::d2h(ctx, &total, b + o_tot, sizeof(total), s);
    const uint64_t nout = std::min<uint64_t>(total, frame_cap);
    if (rc == RH_OK && nout) {
        rc = rh::d2h(ctx, frame_off, b + o_foff, nout * 8, s);
        if (rc == RH_OK) rc = rh::d2h(ctx, frame_len, b + o_flen, nout * 4, s);
        if (rc == RH_OK && frame_crc) rc = rh::d2h(ctx, frame_crc, b + o_fcrc, nout * 4, s);
    }
    if (rc != RH_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    for (uint64_t i = 0; i < n_seg; ++i) {
        rh_segment_result& r = results[i];
        r.status = rst[i];
        r.n_frames = std::min<uint32_t>(nfr[i], frames_per_seg_cap);
        r.n_ok = std::min<uint32_t>(ok[i], r.n_frames);
        r.stop = rstop[i];
        r.first_frame = first[i];
        r.reserved = 0;
    }
    *n_frames_total = total;
    return RH_OK;
}
