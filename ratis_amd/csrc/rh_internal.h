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

}  // namespace rh

struct rh_ctx {
    int device = -1;
    hipStream_t stream = nullptr;
    int num_cus = 0;
    // device copies of the CRC tables
    uint32_t* d_slice = nullptr;   // [4][256]
    uint32_t* d_shift = nullptr;   // [41][4][256]: zero-advance maps over 2^m bytes, m = 0..40
    uint32_t* d_lane16 = nullptr;  // lane-distance nibble tables of the 16-lane x 64-byte fold
    // scratch for host-buffer convenience calls
    std::mutex mu;
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    void* h_pinned = nullptr;
    size_t pinned_bytes = 0;
};

// Launchers implemented in the .hip files (device pointers, async on `stream`).
int rh_commit_launch_impl(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, hipStream_t stream);
int rh_apply_deltas_impl(hipStream_t stream, const rh_delta* d_deltas, uint64_t n, uint64_t capacity,
                         uint64_t stride, uint32_t n_followers, int64_t* match, int64_t* fcommit,
                         int64_t* flush, int64_t* commit);
int rh_crc_launch_impl(rh_ctx* ctx, const rh_frames* f, uint32_t flags, hipStream_t stream);
int rh_crc_upload_tables(rh_ctx* ctx);
int rh_segments_launch_impl(rh_ctx* ctx, const rh_segments* segs, hipStream_t stream);
int rh_segments_read_impl(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, hipStream_t stream);
int rh_crc_verify_slots(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, hipStream_t stream);
int rh_lease_launch_impl(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, hipStream_t stream);
