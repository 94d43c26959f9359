// Standalone A/B (tuning only, not part of libratis_hip): the real commit kernel vs a kernel
// with the identical SoA access pattern (same loads, same 16-byte stores) but trivial compute.
// If the stream-only kernel is much faster, the commit kernel is compute/latency-bound.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 commit_ablation.hip ../../ratis_amd/csrc/commit.hip \
//         ../../ratis_amd/csrc/crc32c.hip ../../ratis_amd/csrc/rh_api.cpp -o ablation
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/ratis_hip.h"

typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

template <int F>
__global__ __launch_bounds__(256) void stream_only(const int64_t* __restrict__ fol, uint64_t stride,
                                                   const int64_t* __restrict__ self, const int64_t* __restrict__ cin,
                                                   const int64_t* __restrict__ ts, const uint32_t* __restrict__ conf,
                                                   int64_t* __restrict__ cout, int64_t* __restrict__ mout, uint64_t n) {
    const uint64_t r0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (r0 + 1 >= n) return;
    v2i64 acc = *reinterpret_cast<const v2i64*>(self + r0);
#pragma unroll
    for (int k = 0; k < F; ++k) {
        const v2i64 x = *reinterpret_cast<const v2i64*>(fol + k * stride + r0);
        acc.x = acc.x < x.x ? acc.x : x.x;
        acc.y = acc.y < x.y ? acc.y : x.y;
    }
    const v2i64 c = *reinterpret_cast<const v2i64*>(cin + r0);
    const v2i64 t = *reinterpret_cast<const v2i64*>(ts + r0);
    const v2u32 w = *reinterpret_cast<const v2u32*>(conf + r0);
    v2i64 o;
    o.x = (w.x & 1u) ? c.x : t.x;
    o.y = (w.y & 1u) ? c.y : t.y;
    *reinterpret_cast<v2i64*>(cout + r0) = o;
    *reinterpret_cast<v2i64*>(mout + r0) = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Tier {
    int F; uint64_t n;
    int64_t *fol, *self, *cin, *ts, *cout, *mout; uint32_t* conf;
};

int main() {
    const uint64_t N = 1000000, R = 8;
    std::vector<Tier> tiers;
    const int Fs[2] = {4, 6};
    const uint64_t ns[2] = {900000, 100000};
    for (uint64_t r = 0; r < R; ++r)
        for (int i = 0; i < 2; ++i) {
            Tier t{Fs[i], ns[i]};
            CK(hipMalloc(&t.fol, 8 * t.n * t.F));
            CK(hipMalloc(&t.self, 8 * t.n)); CK(hipMalloc(&t.cin, 8 * t.n)); CK(hipMalloc(&t.ts, 8 * t.n));
            CK(hipMalloc(&t.cout, 8 * t.n)); CK(hipMalloc(&t.mout, 8 * t.n)); CK(hipMalloc(&t.conf, 4 * t.n));
            std::vector<int64_t> h(t.n * t.F);
            for (uint64_t j = 0; j < h.size(); ++j) h[j] = (int64_t)((j * 2654435761ull) & 0xFFFFF) + (1ll << 30);
            CK(hipMemcpy(t.fol, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
            CK(hipMemcpy(t.self, h.data(), 8 * t.n, hipMemcpyHostToDevice));
            CK(hipMemcpy(t.cin, h.data() + 1, 8 * t.n, hipMemcpyHostToDevice));
            CK(hipMemcpy(t.ts, h.data() + 2, 8 * t.n, hipMemcpyHostToDevice));
            std::vector<uint32_t> c(t.n, (1u << 31) | (1u << 14) | ((1u << t.F) - 1));
            CK(hipMemcpy(t.conf, c.data(), 4 * t.n, hipMemcpyHostToDevice));
            tiers.push_back(t);
        }
    rh_ctx* ctx = nullptr;
    if (rh_init(0, &ctx) != 0) { printf("rh_init: %s\n", rh_last_error()); return 1; }
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const double alg = 76.96e6;
    for (int round = 0; round < 3; ++round) {
        // the shipped kernel
        {
            CK(hipEventRecord(a, 0));
            for (int it = 0; it < 40; ++it) {
                rh_commit_soa s[2] = {};
                for (int i = 0; i < 2; ++i) {
                    Tier& t = tiers[(it % R) * 2 + i];
                    s[i].n = t.n; s[i].n_followers = t.F; s[i].mode = RH_MODE_COMMIT; s[i].gap_threshold = -1;
                    s[i].follower_index = t.fol; s[i].self_index = t.self; s[i].commit_in = t.cin;
                    s[i].term_start = t.ts; s[i].conf = t.conf; s[i].commit_out = t.cout; s[i].min_out = t.mout;
                }
                if (rh_commit_soa_launch(ctx, s, 2, nullptr) != 0) { printf("%s\n", rh_last_error()); return 1; }
            }
            CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"kernel\": \"commit_real\", \"us\": %.2f, \"GBps\": %.1f}\n", ms * 1e3 / 40, alg / (ms / 40 * 1e-3) / 1e9);
        }
        // stream-only: one launch per tier (2 launches per batch)
        CK(hipEventRecord(a, 0));
        for (int it = 0; it < 40; ++it)
            for (int i = 0; i < 2; ++i) {
                Tier& t = tiers[(it % R) * 2 + i];
                const uint32_t blocks = (uint32_t)((t.n / 2 + 255) / 256);
                if (t.F == 4)
                    hipLaunchKernelGGL(stream_only<4>, dim3(blocks), dim3(256), 0, 0, t.fol, t.n, t.self, t.cin, t.ts, t.conf, t.cout, t.mout, t.n);
                else
                    hipLaunchKernelGGL(stream_only<6>, dim3(blocks), dim3(256), 0, 0, t.fol, t.n, t.self, t.cin, t.ts, t.conf, t.cout, t.mout, t.n);
            }
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"kernel\": \"stream_only_2launch\", \"us\": %.2f, \"GBps\": %.1f}\n", ms * 1e3 / 40, alg / (ms / 40 * 1e-3) / 1e9);
        // stream-only, stable tier only (one launch, 900k groups)
        CK(hipEventRecord(a, 0));
        for (int it = 0; it < 40; ++it) {
            Tier& t = tiers[(it % R) * 2];
            const uint32_t blocks = (uint32_t)((t.n / 2 + 255) / 256);
            hipLaunchKernelGGL(stream_only<4>, dim3(blocks), dim3(256), 0, 0, t.fol, t.n, t.self, t.cin, t.ts, t.conf, t.cout, t.mout, t.n);
        }
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"kernel\": \"stream_only_stable900k\", \"us\": %.2f, \"GBps\": %.1f}\n", ms * 1e3 / 40, 900000.0 * 76 / (ms / 40 * 1e-3) / 1e9);
    }
    return 0;
}
