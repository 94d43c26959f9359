// Host-side check of the resident table's tile layout (rh_internal.h, tile::): for every width,
// the byte ranges of every column element of a 128-row tile -- flag and u32 columns, and the int64
// columns through tile::pair_off / elem_off for the build's RH_TABLE_GROUP -- lie inside the tile,
// cover its int64 region exactly once, and each lane's row pair is one aligned 16-byte piece.
// Built and run by tests/test_table_layout.py (hipcc, host code only).
#include "rh_internal.h"

#include <cstdio>
#include <vector>

int main() {
    using namespace rh::tile;
    int bad = 0;
    for (uint32_t F = 2; F <= 14; F += 2) {
        std::vector<int> used(bytes(F), 0);
        auto mark = [&](uint32_t off, uint32_t sz) {
            for (uint32_t r = 0; r < 128; ++r) {
                const uint32_t o = elem_off(F, off, r, sz);
                if (o + sz > bytes(F)) {
                    ++bad;
                    continue;
                }
                for (uint32_t b = 0; b < sz; ++b) ++used[o + b];
            }
        };
        mark(kDirty, 1);
        mark(kWdirty, 1);
        mark(kLon, 1);
        mark(kConf, 4);
        mark(kSlot, 4);
        for (uint32_t c = 0; c < 3 * F + 8; ++c) mark(kMatch + 1024 * c, 8);
        for (uint32_t i = 0; i < bytes(F); ++i)
            if (used[i] > 1 || (i >= kMatch && used[i] != 1)) ++bad;
        for (uint32_t c = 0; c < 3 * F + 8; ++c)
            for (uint32_t p = 0; p < 64; ++p) {
                const uint32_t col = kMatch + 1024 * c, o = pair_off(F, col, p);
                if (o % 16 || elem_off(F, col, 2 * p, 8) != o || elem_off(F, col, 2 * p + 1, 8) != o + 8) ++bad;
            }
    }
    std::printf("layout violations: %d\n", bad);
    return bad != 0;
}
