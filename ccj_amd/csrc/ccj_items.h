// ccj_items.h — enumeration of the k_iloop work items of one level and shard, shared
// by the GPU builder (k_items, ccj_kernels.hip) and the host's count pass (ccj_host.cc): both must
// produce the same per-level counts, since the host sizes the k_iloop launches from them.
//
// A "row" is one closing pair; its items are the chunks of cw cells (k_iloop: IL_CW = 128, one wave
// holding two 64-lane halves; k_pf_iloop: 64) of the cells that share it:
//   PL (role 0): for own a in [6, t], i in [1, m]:   pair (i, i+a),  chunks over h <= m-i
//   PR (role 1): for own a in [0, t-6], q < m:        pair (k, k+t-a), k = q+a+3, chunks over i <= q+1
//   PM (role 2): for h in [2, m-1], j in [1, n]:      pair (j, k = j+h+2), chunks over the own a in [alo, ahi]
// ("own": the rank's a-blocks, ccj_engine.h shard_a; every a when unsharded).  An item is
// role << 30 | f1 << 20 | f2 << 10 | chunk.  pt(i, j) is the pair type of (i, j), 0 = cannot pair.
#pragma once
#include "ccj_energy.h"
#include "ccj_engine.h"

namespace ccj {

constexpr int IL_CW = 128;  // cells per k_iloop work item (MFE)
// k_items splits each (level, shard) into KI_SPLIT consecutive runs of rows, one workgroup each, so
// the count and write passes run KI_SPLIT workgroups per level in parallel (one per level: 0.31 ms
// per sequence at n=200, a serial walk of up to 130 chunks of rows per workgroup)
constexpr int KI_SPLIT = 16;
CCJ_HD void ki_split_rows(int nrows, int s, int &lo, int &hi) {
    const int per = (nrows + KI_SPLIT - 1) / KI_SPLIT;
    lo = imin(nrows, s * per);
    hi = imin(nrows, lo + per);
}

struct ItemRows {
    int m, oPL0, nPLa, nPRa, nPL, nPR, nPM;
};

// rows of level t for rank r of G
CCJ_HD ItemRows item_rows(int n, int t, int G, int r) {
    ItemRows R;
    R.m = n - t - 2;
    R.oPL0 = shard_ceil(6, G, r);
    R.nPLa = imax(0, shard_count(t, G, r) - R.oPL0);
    R.nPRa = t >= 6 ? shard_count(t - 6, G, r) : 0;
    R.nPL = R.nPLa * R.m;
    R.nPR = R.nPRa * R.m;
    R.nPM = imax(0, R.m - 2) * n;
    return R;
}

// rank r's a-blocks of a PM pair (j, k = j+h+2) at level t: own indices [o0, o1]
CCJ_HD void pm_own_range(int n, int t, int j, int k, int G, int r, int &o0, int &o1) {
    const int alo = imax(2, t - (n - k)), ahi = imin(t - 2, j - 1);
    o0 = shard_ceil(alo, G, r);
    o1 = ahi >= alo ? shard_count(ahi, G, r) - 1 : o0 - 1;
}

// items of row x and the first of them (chunk 0); 0 when the pair cannot pair
template <class PT>
CCJ_HD int item_row(const PT &pt, int n, int t, const ItemRows &R, int x, int G, int r, uint32_t &it0, int cw = 64) {
    const int m = R.m;
    if (x < R.nPL) {
        const int a = shard_a(R.oPL0 + x / m, G, r), i = 1 + x % m;
        it0 = (0u << 30) | ((uint32_t)a << 20) | ((uint32_t)i << 10);
        return pt(i, i + a) > 0 ? (m - i) / cw + 1 : 0;
    }
    x -= R.nPL;
    if (x < R.nPR) {
        const int a = shard_a(x / m, G, r), q = x % m;
        const int k = q + a + 3, b = t - a;
        it0 = (1u << 30) | ((uint32_t)a << 20) | ((uint32_t)q << 10);
        return pt(k, k + b) > 0 ? q / cw + 1 : 0;
    }
    x -= R.nPR;
    const int h = 2 + x / n, j = 1 + x % n;
    const int k = j + h + 2;
    if (k > n) return 0;
    int o0, o1;
    pm_own_range(n, t, j, k, G, r, o0, o1);
    if (o0 > o1 || pt(j, k) <= 0) return 0;
    it0 = (2u << 30) | ((uint32_t)h << 20) | ((uint32_t)j << 10);
    return (o1 - o0) / cw + 1;
}

// The same count as summing item_row over every row of the level, with the rows walked in tight
// loops over contiguous pair-type rows (host count pass of ccj_reset: ~10x faster).  pt is the
// [w][p] pair-type table with row stride rs.
inline long long count_level_items(const int8_t *pt, int rs, int n, int t, int G, int r, int cw = 64) {
    const ItemRows R = item_rows(n, t, G, r);
    const int m = R.m;
    long long cnt = 0;
    for (int o = R.oPL0; o < R.oPL0 + R.nPLa; ++o) {  // PL: pair (i, i+a)
        const int a = shard_a(o, G, r);
        const int8_t *row = pt + (size_t)a * rs;
        for (int i = 1; i <= m; ++i)
            if (row[i] > 0) cnt += (m - i) / cw + 1;
    }
    for (int o = 0; o < R.nPRa; ++o) {  // PR: pair (k, k+b), k = q+a+3
        const int a = shard_a(o, G, r), b = t - a;
        const int8_t *row = pt + (size_t)b * rs + a + 3;
        for (int q = 0; q < m; ++q)
            if (row[q] > 0) cnt += q / cw + 1;
    }
    for (int h = 2; h <= m - 1; ++h) {  // PM: pair (j, k = j+h+2)
        const int g = h + 2;
        const int8_t *row = pt + (size_t)g * rs;
        for (int j = 1; j + g <= n; ++j) {
            if (row[j] <= 0) continue;
            int o0, o1;
            pm_own_range(n, t, j, j + g, G, r, o0, o1);
            if (o0 <= o1) cnt += (o1 - o0) / cw + 1;
        }
    }
    return cnt;
}

}  // namespace ccj
