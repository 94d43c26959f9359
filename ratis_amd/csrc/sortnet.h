// Batcher merge-exchange sorting network on int64 registers, generated at compile time.
// Shared by the commit (order statistics of match indices) and lease (order statistics of
// follower response times) kernels, with the ballot bit-word helper both use.
#pragma once
#include <cstdint>

namespace rh_sort {

// Knuth, TAOCP 5.2.2, Algorithm M.
struct Net {
    int n = 0;
    int a[128] = {};
    int b[128] = {};
};

constexpr Net make_net(int N) {
    Net net{};
    if (N < 2) return net;
    int t = 0;
    while ((1 << t) < N) ++t;
    int p = 1 << (t - 1);
    while (p > 0) {
        int q = 1 << (t - 1), r = 0, d = p;
        while (true) {
            for (int i = 0; i < N - d; ++i)
                if ((i & p) == r) {
                    net.a[net.n] = i;
                    net.b[net.n] = i + d;
                    ++net.n;
                }
            if (q == p) break;
            d = q - p;
            q >>= 1;
            r = p;
        }
        p >>= 1;
    }
    return net;
}

template <int N>
constexpr Net kNet = make_net(N);

template <int N, int I = 0>
__device__ __forceinline__ void sort_net(int64_t (&v)[N]) {
    if constexpr (I < kNet<N>.n) {
        constexpr int a = kNet<N>.a[I];
        constexpr int b = kNet<N>.b[I];
        const int64_t x = v[a], y = v[b];
        const bool lt = x < y;
        v[a] = lt ? x : y;
        v[b] = lt ? y : x;
        sort_net<N, I + 1>(v);
    }
}

}  // namespace rh_sort

namespace rh_bits {

// Interleave the low 32 bits of x with zeros (bit i -> bit 2i): two per-lane ballots of a wave
// that holds 2 groups per lane become the group-ordered bit words.
__device__ __forceinline__ uint64_t spread32(uint64_t x) {
    x &= 0xFFFFFFFFull;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

}  // namespace rh_bits
