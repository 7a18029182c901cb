// ccj_items.h — the k_iloop work items of one level and shard.  They depend only
// on n, the level and the shard (not on the sequence), so ccj_create builds them once.
//
// One item = one workgroup = a tile of IT_TI consecutive closing pairs x one 64-lane chunk of the
// free index (ccj_kernels.hip k_iloop), role << 30 | f1 << 20 | tile << 10 | chunk:
//   PL (role 0): own a in [6, t]:   pairs (i, i+a), i = 1+IT_TI*tile ... <= m; lanes k from i0+a+2
//   PR (role 1): own a in [0, t-6]: pairs (k, k+t-a), k = a+3+IT_TI*tile ... <= m+a+2; lanes i from 1
//   PM (role 2): g in [4, m+1]:     pairs (j, j+g), j = 3+IT_TI*tile ... <= n-g-2; lanes i from
//                                   max(1, j0-t+2); every rank walks them and stores its own a only
// with m = n-t-2.  PL/PR with a or b = 6 have no candidates (source levels >= 3 need a, b >= 7)
// but still store the "no interior loop" value k_level4d reads.
#pragma once
#include <stdint.h>
#include <vector>
#include "ccj_energy.h"
#include "ccj_engine.h"

namespace ccj {

inline void level_iloop_items(int n, int t, int G, int r, std::vector<uint32_t> &out) {
    const int m = n - t - 2;
    if (m <= 0 || t < 4) return;  // PM from t = 4 (a, b >= 2), PL / PR from t = 6
    auto push = [&](uint32_t role, int f1, int tile, int chunks) {
        for (int c = 0; c < chunks; ++c)
            out.push_back((role << 30) | ((uint32_t)f1 << 20) | ((uint32_t)tile << 10) | (uint32_t)c);
    };
    const int nown = shard_count(t, G, r);
    for (int o = 0; o < nown; ++o) {  // PL: own a >= 6
        const int a = shard_a(o, G, r);
        if (a < 6) continue;
        for (int x = 0; 1 + IT_TI * x <= m; ++x) push(0, a, x, (m - IT_TI * x + 63) / 64);
    }
    for (int o = 0; o < nown; ++o) {  // PR: own a with b = t-a >= 6
        const int a = shard_a(o, G, r);
        if (t - a < 6) continue;
        for (int x = 0; IT_TI * x < m; ++x) push(1, a, x, (imin(IT_TI * (x + 1), m) + 63) / 64);
    }
    for (int g = 4; g <= m + 1; ++g) {  // PM
        for (int x = 0; 3 + IT_TI * x <= n - g - 2; ++x) {
            const int j0 = 3 + IT_TI * x;
            const int ilo = imax(1, j0 - t + 2), ihi = imin(j0 + IT_TI - 3, n - g - t);
            if (ihi >= ilo) push(2, g, x, (ihi - ilo + 1 + 63) / 64);
        }
    }
}

}  // namespace ccj
