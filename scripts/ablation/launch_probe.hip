// Launch fixed-cost probe (tuning only, not part of libratis_hip): what a back-to-back launch on
// one stream costs before any bytes move, against the headline kernel's 1M-group launch shape
// (1954 workgroups of 256 threads, an ~800-byte by-value argument struct).
//   empty1        1 workgroup, no memory access
//   emptyG        1954 workgroups, no memory access
//   emptyG_arg    the same with an 800-byte argument struct read by every wave (scalar loads)
//   touchG        1954 workgroups, one 16-byte load + store per lane from one of 8 rotating
//                 buffers of 77 MB (every launch touches pages the previous one did not)
//   touchG_warm   the same on one buffer (pages and lines warm)
//   stream        the tiled commit probe: 61 MB read + 16 MB written per launch, 8 rotating batches
// Each is timed back to back with HIP events (200 launches); run under rocprofv3 --kernel-trace for
// per-dispatch durations.
//   hipcc --offload-arch=gfx950 -O3 scripts/ablation/launch_probe.hip -o scripts/ablation/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef long long v2i64 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

constexpr uint64_t N = 1000000;
constexpr int R = 8;
constexpr uint32_t G = (N + 511) / 512;
struct Big {
    const char* p[4];
    uint64_t v[96];
};

__global__ __launch_bounds__(256) void k_empty(int* flag) {
    if (flag && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *flag = 1;
}
__global__ __launch_bounds__(256) void k_empty_arg(const Big b) {
    const Big& a = *(const Big*)(__builtin_amdgcn_kernarg_segment_ptr());
    uint64_t s = 0;
    for (int i = 0; i < 96; i += 8) s += a.v[i];
    if (s == 0x123456789ull && threadIdx.x == 0) *(int*)a.p[0] = 1;
}
__global__ __launch_bounds__(256) void k_touch(const char* in, char* out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const v2i64 v = *reinterpret_cast<const v2i64*>(in + i * 32);
    *reinterpret_cast<v2i64*>(out + i * 16) = v + 1;
}
constexpr int F = 4;
constexpr uint64_t kTileIn = (F + 3) * 128 * 8 + 128 * 4;
constexpr uint64_t kTileOut = 2 * 128 * 8;
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_stream(const char* in, char* outp) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const long long* tin = reinterpret_cast<const long long*>(in + wave * kTileIn);
    v2i64 f[F + 3];
#pragma unroll
    for (int k = 0; k < F + 3; ++k) f[k] = __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(tin + k * 128 + 2 * lane));
    const unsigned w = reinterpret_cast<const unsigned*>(tin + (F + 3) * 128)[2 * lane];
    v2i64 m = f[0];
#pragma unroll
    for (int k = 1; k < F + 3; ++k) {
        m.x = m.x < f[k].x ? m.x : f[k].x;
        m.y = m.y < f[k].y ? m.y : f[k].y;
    }
    long long* tout = reinterpret_cast<long long*>(outp + wave * kTileOut);
    __builtin_nontemporal_store(m, reinterpret_cast<v2i64*>(tout + 2 * lane));
    __builtin_nontemporal_store(m + (long long)w, reinterpret_cast<v2i64*>(tout + 128 + 2 * lane));
}

int main() {
    const uint64_t in_b = (uint64_t)G * 4 * kTileIn, out_b = (uint64_t)G * 4 * kTileOut;
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
    Big big{};
    big.p[0] = in[0];
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 2 * R; ++i) launch(i % R);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < steps; ++i) launch(i % R);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"%s\", \"us_per_launch\": %.2f}\n", name, ms * 1e3 / steps);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("empty1", [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, nullptr); });
        run("emptyG", [&](int) { hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, 0, nullptr); });
        run("emptyG_arg", [&](int) { hipLaunchKernelGGL(k_empty_arg, dim3(G), dim3(256), 0, 0, big); });
        run("touchG", [&](int i) { hipLaunchKernelGGL(k_touch, dim3(G), dim3(256), 0, 0, in[i], out[i]); });
        run("touchG_warm", [&](int) { hipLaunchKernelGGL(k_touch, dim3(G), dim3(256), 0, 0, in[0], out[0]); });
        run("stream", [&](int i) { hipLaunchKernelGGL(k_stream, dim3(G), dim3(256), 0, 0, in[i], out[i]); });
    }
    CK(hipDeviceSynchronize());
    return 0;
}
