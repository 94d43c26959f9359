// Standalone access-pattern probe (tuning only, not part of libratis_hip): the commit kernel's
// per-group traffic (F = 4: 7 int64 + 1 u32 read, 2 int64 written) laid out three ways, each over
// 8 rotating 1M-group batches (> the Infinity Cache), trivial compute:
//   soa    -- one array per column (the rh_commit_soa layout): a wave touches 10 separate 1 KiB runs
//   tiled  -- per 128-group tile all columns back to back (AoSoA): a wave touches one 8.5 KiB run
//   flat   -- the same byte counts as one contiguous read stream and one write stream
//   hipcc --offload-arch=gfx950 -O3 scripts/ablation/layout_probe.hip -o scripts/ablation/layout_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

constexpr int F = 4;
constexpr uint64_t N = 1 << 20;  // groups per batch (multiple of 128)
constexpr int R = 8;

template <bool NT>
__device__ __forceinline__ v2i64 ld(const long long* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(p));
    return *reinterpret_cast<const v2i64*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(long long* p, v2i64 v) {
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<v2i64*>(p));
    else
        *reinterpret_cast<v2i64*>(p) = v;
}

__device__ __forceinline__ void body(v2i64 f[F], v2i64 s, v2i64 c, v2i64 t, v2u32 w, v2i64& o, v2i64& m) {
    m = s;
#pragma unroll
    for (int k = 0; k < F; ++k) {
        m.x = m.x < f[k].x ? m.x : f[k].x;
        m.y = m.y < f[k].y ? m.y : f[k].y;
    }
    o.x = (w.x & 1u) ? c.x : t.x;
    o.y = (w.y & 1u) ? c.y : t.y;
}

// soa: columns [F][N], self, cin, ts [N], conf [N] u32; out, min [N]
template <bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_soa(const long long* fol,
    const long long* self, const long long* cin, const long long* ts, const unsigned* conf, long long* out,
    long long* mn) {
    const uint64_t r = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    v2i64 f[F];
#pragma unroll
    for (int k = 0; k < F; ++k) f[k] = ld<NT>(fol + k * N + r);
    const v2i64 s = ld<NT>(self + r), c = ld<NT>(cin + r), t = ld<NT>(ts + r);
    const v2u32 w = *reinterpret_cast<const v2u32*>(conf + r);
    v2i64 o, m;
    body(f, s, c, t, w, o, m);
    st<NT>(out + r, o);
    st<NT>(mn + r, m);
}

// tiled: tile of 128 groups = [F+3][128] int64 then [128] u32 (8.5 KiB), outputs [2][128] int64
constexpr uint64_t kTileIn = (F + 3) * 128 * 8 + 128 * 4;
constexpr uint64_t kTileOut = 2 * 128 * 8;
template <bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_tiled(const char* in, char* outp) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const long long* tin = reinterpret_cast<const long long*>(in + wave * kTileIn);
    v2i64 f[F];
#pragma unroll
    for (int k = 0; k < F; ++k) f[k] = ld<NT>(tin + k * 128 + 2 * lane);
    const v2i64 s = ld<NT>(tin + F * 128 + 2 * lane), c = ld<NT>(tin + (F + 1) * 128 + 2 * lane),
                t = ld<NT>(tin + (F + 2) * 128 + 2 * lane);
    const v2u32 w = *reinterpret_cast<const v2u32*>(reinterpret_cast<const unsigned*>(tin + (F + 3) * 128) + 2 * lane);
    v2i64 o, m;
    body(f, s, c, t, w, o, m);
    long long* tout = reinterpret_cast<long long*>(outp + wave * kTileOut);
    st<NT>(tout + 2 * lane, o);
    st<NT>(tout + 128 + 2 * lane, m);
}

// flat: each lane reads kTileIn/64 bytes as 16-byte loads strided by the wave (like a copy)
template <bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_flat(const char* in, char* outp) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const v4u32* p = reinterpret_cast<const v4u32*>(in + wave * kTileIn);
    constexpr int kLd = (int)(kTileIn / 16 / 64);  // 8 full loads + a remainder
    v4u32 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
        const v4u32 v = NT ? __builtin_nontemporal_load(p + i * 64 + lane) : p[i * 64 + lane];
        acc ^= v;
    }
    if (lane < (int)((kTileIn / 16) % 64)) acc ^= p[kLd * 64 + lane];
    v4u32* q = reinterpret_cast<v4u32*>(outp + wave * kTileOut);
    q[lane] = acc;
    q[64 + lane] = acc + 1u;
}

int main() {
    const uint64_t in_b = N / 128 * kTileIn, out_b = N / 128 * kTileOut;
    char *in[R], *out[R];
    for (int i = 0; i < R; ++i) {
        CK(hipMalloc(&in[i], in_b));
        CK(hipMalloc(&out[i], out_b));
        CK(hipMemset(in[i], i + 1, in_b));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int steps = 200;
    const dim3 grid(N / 512), block(256);
    const double bytes = (double)in_b + (double)out_b;
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 2 * R; ++i) launch(i % R);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < steps; ++i) launch(i % R);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / steps;
        std::printf("{\"layout\": \"%s\", \"us_per_launch\": %.2f, \"TBps\": %.3f}\n", name, us, bytes / us / 1e6);
    };
    for (int nt = 0; nt < 2; ++nt) {
        run(nt ? "soa_nt" : "soa", [&](int i) {
            const long long* b = reinterpret_cast<const long long*>(in[i]);
            const long long* fol = b;
            const long long* self = b + F * N;
            const long long* cin = self + N;
            const long long* ts = cin + N;
            const unsigned* conf = reinterpret_cast<const unsigned*>(ts + N);
            long long* o = reinterpret_cast<long long*>(out[i]);
            if (nt)
                hipLaunchKernelGGL(k_soa<true>, grid, block, 0, 0, fol, self, cin, ts, conf, o, o + N);
            else
                hipLaunchKernelGGL(k_soa<false>, grid, block, 0, 0, fol, self, cin, ts, conf, o, o + N);
        });
        run(nt ? "tiled_nt" : "tiled", [&](int i) {
            if (nt)
                hipLaunchKernelGGL(k_tiled<true>, grid, block, 0, 0, in[i], out[i]);
            else
                hipLaunchKernelGGL(k_tiled<false>, grid, block, 0, 0, in[i], out[i]);
        });
        run(nt ? "flat_nt" : "flat", [&](int i) {
            if (nt)
                hipLaunchKernelGGL(k_flat<true>, grid, block, 0, 0, in[i], out[i]);
            else
                hipLaunchKernelGGL(k_flat<false>, grid, block, 0, 0, in[i], out[i]);
        });
    }
    CK(hipDeviceSynchronize());
    return 0;
}
