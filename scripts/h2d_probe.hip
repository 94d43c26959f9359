// Host -> device transfer probe for the delta-streaming path (16 MB per step): one SDMA copy,
// the copy split over 2 / 4 streams, and a kernel pulling the bytes from host-mapped pinned
// memory.  Build: hipcc --offload-arch=gfx950 -O2 scripts/h2d_probe.hip -o scripts/h2d_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void pull(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = __builtin_nontemporal_load(src + i);
}

int main() {
    const size_t bytes = 16000000;
    void* h = nullptr;
    void* d = nullptr;
    CK(hipHostMalloc(&h, bytes, hipHostMallocMapped));
    CK(hipMalloc(&d, bytes));
    void* hd = nullptr;
    CK(hipHostGetDevicePointer(&hd, h, 0));
    for (size_t i = 0; i < bytes; ++i) static_cast<unsigned char*>(h)[i] = (unsigned char)i;
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipEvent_t done[4];
    for (auto& e : done) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const int reps = 20;
    for (int parts : {1, 2, 4}) {
        for (int warm = 0; warm < 2; ++warm) {
            CK(hipEventRecord(e0, st[0]));
            for (int r = 0; r < reps; ++r) {
                for (int p = 1; p < parts; ++p) CK(hipStreamWaitEvent(st[p], e0, 0));
                const size_t chunk = bytes / parts;
                for (int p = 0; p < parts; ++p)
                    CK(hipMemcpyAsync(static_cast<char*>(d) + p * chunk, static_cast<char*>(h) + p * chunk,
                                      p == parts - 1 ? bytes - p * chunk : chunk, hipMemcpyHostToDevice, st[p]));
                for (int p = 1; p < parts; ++p) {
                    CK(hipEventRecord(done[p], st[p]));
                    CK(hipStreamWaitEvent(st[0], done[p], 0));
                }
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"sdma_h2d\", \"streams\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", parts, ms / reps,
                    bytes / (ms / reps * 1e-3) / 1e9);
    }
    for (int blocks : {256, 1024, 4096}) {
        for (int warm = 0; warm < 2; ++warm) {
            CK(hipEventRecord(e0, st[0]));
            for (int r = 0; r < reps; ++r)
                hipLaunchKernelGGL(pull, dim3(blocks), dim3(256), 0, st[0], static_cast<const v4u*>(hd),
                                   static_cast<v4u*>(d), bytes / 16);
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"kernel_pull\", \"blocks\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", blocks, ms / reps,
                    bytes / (ms / reps * 1e-3) / 1e9);
    }
    for (int parts : {1, 2}) {  // device -> host for comparison
        CK(hipEventRecord(e0, st[0]));
        for (int r = 0; r < reps; ++r) {
            const size_t chunk = bytes / parts;
            for (int p = 1; p < parts; ++p) CK(hipStreamWaitEvent(st[p], e0, 0));
            for (int p = 0; p < parts; ++p)
                CK(hipMemcpyAsync(static_cast<char*>(h) + p * chunk, static_cast<char*>(d) + p * chunk, chunk,
                                  hipMemcpyDeviceToHost, st[p]));
            for (int p = 1; p < parts; ++p) {
                CK(hipEventRecord(done[p], st[p]));
                CK(hipStreamWaitEvent(st[0], done[p], 0));
            }
        }
        CK(hipEventRecord(e1, st[0]));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"sdma_d2h\", \"streams\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", parts, ms / reps,
                    bytes / (ms / reps * 1e-3) / 1e9);
    }
    CK(hipDeviceSynchronize());
    CK(hipHostFree(h));
    CK(hipFree(d));
    return 0;
}
