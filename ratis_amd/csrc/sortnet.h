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

namespace rh_sort {

// Rank masks for order statistics without sorting (fewer live registers than a network on
// copies, and one pass serves several member masks -- new and old conf of a joint group).
// Bit j of less[i] is set iff element j precedes element i in the stable ascending order
// (v[j] < v[i], or v[j] == v[i] and j < i).  For a member mask m, the member i with
// popcount(less[i] & m) == r is the r-th smallest member: the same value Arrays.sort puts at
// index r (ties are equal values, so the order among them does not matter).
template <int N>
__device__ __forceinline__ void rank_masks(const int64_t (&v)[N], uint32_t (&less)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) less[i] = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = i + 1; j < N; ++j) {
            const bool jfirst = v[j] < v[i];
            less[i] |= jfirst ? (1u << j) : 0u;
            less[j] |= jfirst ? 0u : (1u << i);
        }
}

// min / element of rank k / max of the members of m (m != 0, n = popcount(m), k < n).
template <int N>
__device__ __forceinline__ void select_ranks(const int64_t (&v)[N], const uint32_t (&less)[N], uint32_t m,
                                             int k, int n, int64_t& mn, int64_t& mk, int64_t& mx) {
    mn = v[0];
    mk = v[0];
    mx = v[0];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool in = (m >> i) & 1u;
        const int r = __builtin_popcount(less[i] & m);
        mn = (in && r == 0) ? v[i] : mn;
        mk = (in && r == k) ? v[i] : mk;
        mx = (in && r == n - 1) ? v[i] : mx;
    }
}

}  // namespace rh_sort
