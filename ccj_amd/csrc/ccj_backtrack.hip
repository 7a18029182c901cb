// ccj_backtrack.hip — exterior W and the whole traceback on the GPU.
//
// The reference runs W (W_final.cc:68-79) and the traceback (W_final::backtrack :175-719,
// pseudo_loop::backtrack pseudo_loop.cc:861-2820) on the host over the filled matrices.  Doing it
// here removes the 2.9 GB device-to-host copy of the 4-D matrices (n=200) from every fold: only
// W, the pair list f[] and an exit record come back, and fill_structure (W_final.cc:764-819)
// stays on the host.
//
// One workgroup (CCJ_BT_WAVES waves, default 8) does the traceback.  Nodes are popped from an LDS
// stack in the reference's LIFO order; every case is the reference's argmin with its strict `<`
// (first minimum in loop order) computed as a parallel scan: each lane evaluates a strided subset
// of the case's candidates and a lexicographic (value, position) reduction picks the first
// minimum (see scan() for how short and long scans are spread).  Loops that the
// reference runs one after another are scanned one after another, each result compared strictly
// with the running minimum, so ties resolve exactly as in the sequential code.  The host
// restatement (ccj_host.cc, Backtracker) is the same algorithm over the host mirror; the GPU tests
// check both against the reference.
#include <hip/hip_runtime.h>

#include "ccj_backtrack.h"
#include "ccj_energy.h"
#include "ccj_engine.h"

using namespace ccj;

namespace {

constexpr int BIG = 0x7fffffff;  // "no candidate" in a scan

// reference getters over device memory (same semantics as HostView in ccj_host.cc)
struct DV {
    const DevTables &T;
    int n, rs;
    const int *W;
    mutable int bad;  // Matrix4D::get_uc assert (matrices.hh:167) hit by this lane
    // the small tables every candidate reads (k_backtrack: copies in LDS; else T's)
    const short *S, *S1;
    const int8_t *pair, *rtype;
    const LvlDev *ld;

    __device__ __forceinline__ int pr(int i, int j) const { return pair[S[i] * 8 + S[j]]; }
    __device__ __forceinline__ int a2(const int *A, int i, int j) const { return A[(j - i) * rs + i]; }
    // s_energy_matrix.hh:37-43
    __device__ __forceinline__ int V(int i, int j) const { return i >= j ? INF : a2(T.V, i, j); }
    __device__ __forceinline__ int Vtype(int i, int j) const { return T.Vt[(j - i) * rs + i]; }
    __device__ __forceinline__ int WM(int i, int j) const { return i >= j ? INF : a2(T.WM, i, j); }
    __device__ __forceinline__ int WMv(int i, int j) const { return i >= j ? INF : a2(T.WMv, i, j); }
    __device__ __forceinline__ int WMp(int i, int j) const { return i >= j ? INF : a2(T.WMp, i, j); }
    // TriangleMatrix::get (matrices.hh:38-41)
    __device__ __forceinline__ int Pg(int i, int j) const { return i > j ? INF : a2(T.P, i, j); }
    __device__ __forceinline__ int WBPg(int i, int j) const { return i > j ? INF : a2(T.WBP, i, j); }
    __device__ __forceinline__ int WPPg(int i, int j) const { return i > j ? INF : a2(T.WPP, i, j); }
    // pseudo_loop.cc:647-661
    __device__ __forceinline__ int WB(int i, int j) const {
        if (i <= 0 || j <= 0 || i > n || j > n) return INF;
        if (i > j) return 0;
        return imin(T.pen.cp * (j - i + 1), WBPg(i, j));
    }
    __device__ __forceinline__ int WP(int i, int j) const {
        if (i <= 0 || j <= 0 || i > n || j > n) return INF;
        if (i > j) return 0;
        return imin(T.pen.PUP * (j - i + 1), WPPg(i, j));
    }
    // Matrix4D::get (matrices.hh:177-182) with get_uc's live assert
    __device__ __forceinline__ int g4(int x, int i, int j, int k, int l) const {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (i <= 0 || l > n) {
            bad = 1;
            return INF;
        }
        const int t = (j - i) + (l - k), m = n - t - 2, h = k - j - 2, a = j - i;
        const LvlDev L = ld[t];
        const long long cell = (long long)a * L.M + h * m - ((h * (h - 1)) >> 1) + i - 1;
        if (!T.mat5 && rec_only(x)) return rec_get(T, x, L, cell);  // record-only matrix (ccj_engine.h)
        return (int)T.d4[L.lb + (long long)mslot(x) * L.C + cell];
    }
    __device__ __forceinline__ bool can_pair(int i, int j) const { return (j - i > TURN) && pr(i, j) > 0; }  // pseudo_loop.hh:131-135
    // pseudo_loop.cc:822-840 (lrint = round-half-even in double)
    __device__ __forceinline__ int compute_int(int i, int j, int k, int l) const {
        return E_IntLoop(T.prm, T.lx, k - i - 1, j - l - 1, pr(i, j), rtype[pr(k, l)], S1[i + 1], S1[j - 1], S1[k - 1],
                         S1[l + 1]);
    }
    __device__ __forceinline__ int e_stP(int i, int j) const {
        if (i + 1 == j - 1) return INF;
        return (int)rint(T.e_stP * (double)compute_int(i, j, i + 1, j - 1));
    }
    __device__ __forceinline__ int e_intP(int i, int ip, int jp, int j) const { return (int)rint(T.e_intP * (double)compute_int(i, j, ip, jp)); }
};

__device__ __forceinline__ int lane_id() { return (int)threadIdx.x; }

__device__ __forceinline__ void wreduce(int &v, int &x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int v2 = __shfl_xor(v, o), x2 = __shfl_xor(x, o);
        if (v2 < v || (v2 == v && x2 < x)) {
            v = v2;
            x = x2;
        }
    }
}

// The traceback workgroup has BT_MAXW waves at most.  Every wave walks the same nodes in lockstep
// (all control flow is uniform: it depends only on scan results, which every lane holds).  A scan
// of at most REPL_MAX candidates is evaluated by every wave redundantly (lane x: x, x+64, ...) and
// reduced inside the wave — no barrier; a longer one is spread over the whole workgroup (thread t:
// t, t+blockDim, ...) and the waves' partial minima meet in LDS.  Either way every lane ends with
// the lexicographic (value, position) minimum, i.e. the reference's first strict minimum.
constexpr int BT_MAXW = 16;
constexpr int BT_WAVES_DEFAULT = 8;
constexpr int REPL_MAX = 64;

__device__ __forceinline__ void block_reduce(int &v, int &x) {
    __shared__ int rv[BT_MAXW], rx[BT_MAXW];
    const int w = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6);
    if ((threadIdx.x & 63) == 0) {
        rv[w] = v;
        rx[w] = x;
    }
    __syncthreads();
    for (int q = 0; q < nw; ++q) {
        const int v2 = rv[q], x2 = rx[q];
        if (v2 < v || (v2 == v && x2 < x)) {
            v = v2;
            x = x2;
        }
    }
    __syncthreads();  // rv/rx are reused by the next scan
}

// first minimum (value, position) over candidate positions [0, count) in loop order
template <class F>
__device__ __forceinline__ void scan(int count, F f, int &bv, int &bx) {
    int v = BIG, x = BIG;
    const bool spread = count > REPL_MAX && blockDim.x > 64;
    const int c0 = spread ? (int)threadIdx.x : (int)(threadIdx.x & 63), dc = spread ? (int)blockDim.x : 64;
    for (int c = c0; c < count; c += dc) {
        const int t = f(c);
        if (t < v) {
            v = t;
            x = c;
        }
    }
    wreduce(v, x);
    if (spread) block_reduce(v, x);
    bv = v;
    bx = x;
}

template <class F>
__device__ __forceinline__ int wmin(int count, F f) {
    int v = BIG, x = 0;
    const bool spread = count > REPL_MAX && blockDim.x > 64;
    const int c0 = spread ? (int)threadIdx.x : (int)(threadIdx.x & 63), dc = spread ? (int)blockDim.x : 64;
    for (int c = c0; c < count; c += dc) v = imin(v, f(c));
    wreduce(v, x);
    if (spread) block_reduce(v, x);
    return v;
}

// One pass over candidates that yields both the first minimum (value, position) of f(c).x and the
// minimum of f(c).y: a get_P?iloop value (pairable inner pairs only, .y) and the argmin its
// P_P?iloop node takes next over the same candidates (no can_pair filter, .x)
template <class F>
__device__ __forceinline__ void scan2(int count, F f, int &fmin, int &bv, int &bx) {
    int v = BIG, x = BIG, fm = BIG, z = 0;
    const bool spread = count > REPL_MAX && blockDim.x > 64;
    const int c0 = spread ? (int)threadIdx.x : (int)(threadIdx.x & 63), dc = spread ? (int)blockDim.x : 64;
    for (int c = c0; c < count; c += dc) {
        const int2 t = f(c);
        if (t.x < v) {
            v = t.x;
            x = c;
        }
        fm = imin(fm, t.y);
    }
    wreduce(v, x);
    wreduce(fm, z);
    if (spread) {
        block_reduce(v, x);
        block_reduce(fm, z);
    }
    fmin = fm;
    bv = v;
    bx = x;
}

// W_final.cc:118-173
__device__ int E_ext_Stem(const DV &H, int dangles, int vij, int vi1j, int vij1, int vi1j1, int i, int j) {
    const short *S = H.S;
    const int n = H.n;
    int e = INF, en;
    int tt = H.pr(i, j);
    en = vij;
    if (en != INF) {
        if (dangles == 2) en += E_ExtLoop(H.T.prm, tt, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1);
        else en += E_ExtLoop(H.T.prm, tt, -1, -1);
        e = imin(e, en);
    }
    if (dangles == 1) {
        tt = H.pr(i + 1, j);
        en = (j - i - 1 > TURN) ? vi1j : INF;
        if (en != INF) en += E_ExtLoop(H.T.prm, tt, S[i], -1);
        e = imin(e, en);
        tt = H.pr(i, j - 1);
        en = (j - 1 - i > TURN) ? vij1 : INF;
        if (en != INF) en += E_ExtLoop(H.T.prm, tt, -1, S[j]);
        e = imin(e, en);
        tt = H.pr(i + 1, j - 1);
        en = (j - 1 - i - 1 > TURN) ? vi1j1 : INF;
        if (en != INF) en += E_ExtLoop(H.T.prm, tt, S[i], S[j]);
        e = imin(e, en);
    }
    return e;
}

// W_final.cc:68-79.  W[j] = min(W[j-1], min_k W[k-1] + S(k,j)) with
//   S(k,j) = min(E_ext_Stem(V(k..j) ...), min(P(k,j), P(k+1,j), P(k,j-1), P(k+1,j-1)) + PS),
// since the reference's two terms share the W[k-1] addend.  k_w_terms evaluates every S(k,j) in
// parallel; k_compute_W then runs the recurrence in one wave, j ascending, k over the lanes.
__global__ __launch_bounds__(256) void k_w_terms(DevTables T, int *S) {
    const int n = T.n;
    DV H{T, n, T.rs, nullptr, 0, T.S, T.S1, T.pair, T.rtype, T.ld};
    const int j = blockIdx.y + TURN + 1;
    const int k = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (j > n || k > j - TURN - 1) return;
    const int e2 = E_ext_Stem(H, T.dangles, H.V(k, j), H.V(k + 1, j), H.V(k, j - 1), H.V(k + 1, j - 1), k, j);
    const int e3 = imin(imin(H.Pg(k, j), H.Pg(k + 1, j)), imin(H.Pg(k, j - 1), H.Pg(k + 1, j - 1))) + T.pen.PS;
    S[(size_t)j * T.rs + k] = imin(e2, e3);
}

// The recurrence with W held in registers: W[x] lives in lane x % 64, slot x / 64 (Q slots cover
// 0..n), so a step is a register pass plus a wave reduction — no LDS, no barrier — and the S row
// of step j+1 is loaded while step j reduces, which hides the load latency behind the chain.
template <int Q>
__global__ __launch_bounds__(64) void k_compute_W_reg(DevTables T, const int *S, int *Wout) {
    const int n = T.n, lane = (int)threadIdx.x;
    int w[Q], s_cur[Q], s_nxt[Q];
    // S(k, j) for k = lane + 64q + 1, which adds to W[k-1] = w[q]; k runs 1 .. j-TURN-1
    auto load = [&](int j, int *s) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int k = lane + 64 * q + 1;
            s[q] = (j <= n && k <= j - TURN - 1) ? S[(size_t)j * T.rs + k] : BIG;
        }
    };
#pragma unroll
    for (int q = 0; q < Q; ++q) w[q] = 0;
    load(TURN + 1, s_cur);
    int wprev = 0;
    for (int j = TURN + 1; j <= n; ++j) {
        load(j + 1, s_nxt);
        int m = INF;
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (s_cur[q] != BIG) m = imin(m, w[q] + s_cur[q]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = imin(m, __shfl_xor(m, o));
        wprev = imin(wprev, m);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (lane + 64 * q == j) w[q] = wprev;
            s_cur[q] = s_nxt[q];
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (lane + 64 * q <= n) Wout[lane + 64 * q] = w[q];
}

__global__ __launch_bounds__(64) void k_compute_W(DevTables T, const int *S, int *Wout) {
    extern __shared__ int Ws[];
    const int n = T.n;
    for (int j = lane_id(); j <= n; j += 64) Ws[j] = 0;
    __syncthreads();
    for (int j = TURN + 1; j <= n; ++j) {
        const int *Sj = S + (size_t)j * T.rs;
        int m = INF;
        for (int k = 1 + lane_id(); k <= j - TURN - 1; k += 64) m = imin(m, ((k > 1) ? Ws[k - 1] : 0) + Sj[k]);
        int x = 0;
        wreduce(m, x);
        if (lane_id() == 0) Ws[j] = imin(Ws[j - 1], m);
        __syncthreads();
    }
    for (int j = lane_id(); j <= n; j += 64) Wout[j] = Ws[j];
}

struct Bt {
    const DV &H;
    Interval *stk;
    int cap, sp;
    int *f_pair;
    int8_t *f_type;
    BtOut st;  // uniform
    // the interior-loop argmin a P_PL / PR / PM / PO node computed with its get_P?iloop value, for
    // the P_P?iloop node it pushes (popped next); type 0: none
    struct IlCache { int type, i, j, k, l, bv, bx; };
    mutable IlCache ilc{0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ bool il_cached(int type, int i, int j, int k, int l, int &bv, int &bx) const {
        const bool hit = ilc.type == type && ilc.i == i && ilc.j == j && ilc.k == k && ilc.l == l;
        if (hit) {
            bv = ilc.bv;
            bx = ilc.bx;
        }
        ilc.type = 0;
        return hit;
    }

    __device__ __forceinline__ void push(int i, int j, int k, int l, int type) {
        if (sp >= cap) {
            st.status = BT_OVERFLOW;
            return;
        }
        if (lane_id() == 0) stk[sp] = Interval{i, j, k, l, type};
        ++sp;
    }
    __device__ __forceinline__ void push2(int i, int j, int type) { push(i, j, 0, 0, type); }
    // pseudo_loop::insert_node(i, j, k, l, type): fields i, j(=l of the region), k(=j), l(=k)
    __device__ __forceinline__ void push4(int i, int j, int k, int l, int type) { push(i, j, k, l, type); }
    __device__ __forceinline__ void pairup(int p, int q, int type) {
        if (lane_id() == 0) {
            f_pair[p] = q;
            f_pair[q] = p;
            f_type[p] = (int8_t)type;
            f_type[q] = (int8_t)type;
        }
    }
    __device__ __forceinline__ void die(int prefix, int node) {
        st.status = BT_DIE;
        st.prefix = prefix;
        st.node = node;
    }
    __device__ __forceinline__ bool in_range4(int i, int j, int k, int l) const {
        const int n = H.n;
        return !(i <= 0 || j <= 0 || k <= 0 || l <= 0 || i > n || j > n || k > n || l > n);
    }
    __device__ __forceinline__ static bool order4(int i, int j, int k, int l) { return i <= j && j < k - 1 && k <= l; }

    // get_P?iloop, value only, with can_pair (pseudo_loop.cc:682-808)
    __device__ __forceinline__ int get_PLiloop(int i, int j, int k, int l) const {
        if (!order4(i, j, k, l) || !H.can_pair(i, j)) return INF;
        int mn = INF;
        if (i + TURN + 2 < j) mn = H.g4(PL, i + 1, j - 1, k, l) + H.e_stP(i, j);
        const int nd = imin(j, i + MAXLOOP) - (i + 1);
        int fm, bv, bx;
        scan2(imax(nd, 0) * 32, [&](int c) {
            const int d = i + 1 + (c >> 5), dp = j - 1 - (c & 31);
            if (dp <= imax(d + TURN, j - MAXLOOP)) return make_int2(BIG, BIG);
            const int v = H.e_intP(i, d, dp, j) + H.g4(PL, d, dp, k, l);
            return make_int2(v, H.can_pair(d, dp) ? v : BIG);
        }, fm, bv, bx);
        ilc = IlCache{P_PLiloop, i, j, k, l, bv, bx};
        return imin(mn, fm);
    }
    __device__ __forceinline__ int get_PRiloop(int i, int j, int k, int l) const {
        if (!order4(i, j, k, l) || !H.can_pair(k, l)) return INF;
        int mn = INF;
        if (k + TURN + 2 < l) mn = H.g4(PR, i, j, k + 1, l - 1) + H.e_stP(k, l);
        const int nd = imin(l, k + MAXLOOP) - (k + 1);
        int fm, bv, bx;
        scan2(imax(nd, 0) * 32, [&](int c) {
            const int d = k + 1 + (c >> 5), dp = l - 1 - (c & 31);
            if (dp <= imax(d + TURN, l - MAXLOOP)) return make_int2(BIG, BIG);
            const int v = H.e_intP(k, d, dp, l) + H.g4(PR, i, j, d, dp);
            return make_int2(v, H.can_pair(d, dp) ? v : BIG);
        }, fm, bv, bx);
        ilc = IlCache{P_PRiloop, i, j, k, l, bv, bx};
        return imin(mn, fm);
    }
    __device__ __forceinline__ int get_PMiloop(int i, int j, int k, int l) const {
        if (!order4(i, j, k, l) || !H.can_pair(j, k)) return INF;
        int mn = INF;
        if (i < j && k < l) mn = H.g4(PM, i, j - 1, k + 1, l) + H.e_stP(j - 1, k + 1);
        const int nd = (j - 1) - imax(i, j - MAXLOOP);
        const int min_dp = imin(l, k + MAXLOOP);
        int fm, bv, bx;
        scan2(imax(nd, 0) * 32, [&](int c) {
            const int d = j - 1 - (c >> 5), dp = k + 1 + (c & 31);
            if (dp >= min_dp) return make_int2(BIG, BIG);
            const int v = H.e_intP(d, j, k, dp) + H.g4(PM, i, d, dp, l);
            return make_int2(v, H.can_pair(d, dp) ? v : BIG);
        }, fm, bv, bx);
        ilc = IlCache{P_PMiloop, i, j, k, l, bv, bx};
        return imin(mn, fm);
    }
    __device__ __forceinline__ int get_POiloop(int i, int j, int k, int l) const {
        if (!order4(i, j, k, l) || !H.can_pair(i, l)) return INF;
        int mn = INF;
        if (i < j && k < l) mn = H.g4(PO, i + 1, j, k, l - 1) + H.e_stP(i, l);
        const int nd = imin(j, i + MAXLOOP) - (i + 1);
        const int min_dp = imax(l - MAXLOOP, k);
        int fm, bv, bx;
        scan2(imax(nd, 0) * 32, [&](int c) {
            const int d = i + 1 + (c >> 5), dp = l - 1 - (c & 31);
            if (dp <= min_dp) return make_int2(BIG, BIG);
            const int v = H.e_intP(i, d, dp, l) + H.g4(PO, d, j, dp, k);
            return make_int2(v, H.can_pair(d, dp) ? v : BIG);
        }, fm, bv, bx);
        ilc = IlCache{P_POiloop, i, j, k, l, bv, bx};
        return imin(mn, fm);
    }
    __device__ __forceinline__ int get_PXmloop(int m10, int m01, int i2, int j2, int k2, int l2, int i, int j, int k, int l) const {
        if (!order4(i, j, k, l)) return INF;
        const int b1 = H.g4(m10, i2, j2, k2, l2) + H.T.pen.ap + H.T.pen.bp;
        const int b2 = H.g4(m01, i2, j2, k2, l2) + H.T.pen.ap + H.T.pen.bp;
        return imin(b1, b2);
    }

    // one node (W_final::backtrack W_final.cc:175-719, pseudo_loop::backtrack pseudo_loop.cc:861-2820)
    __device__ __forceinline__ void node(const Interval &cur);
    __device__ __forceinline__ void bt_loop(const Interval &cur);
    __device__ __forceinline__ void bt_free(const Interval &cur);
    __device__ __forceinline__ void bt_wm(const Interval &cur);
    __device__ __forceinline__ void bt_wmv(const Interval &cur);
    __device__ __forceinline__ void bt_wmp(const Interval &cur);
    __device__ __forceinline__ void pl(const Interval &cur);
};

__device__ __forceinline__ void Bt::node(const Interval &cur) {
    switch (cur.type) {
        case LOOP: bt_loop(cur); break;
        case FREE: bt_free(cur); break;
        case M_WM: bt_wm(cur); break;
        case M_WMv: bt_wmv(cur); break;
        case M_WMp: bt_wmp(cur); break;
        case P_PK: case P_PL: case P_PR: case P_PM: case P_PO: case P_PfromL: case P_PfromR: case P_PfromM:
        case P_PfromO: case P_PLiloop: case P_PLiloop5: case P_PLmloop: case P_PLmloop00: case P_PLmloop01:
        case P_PLmloop10: case P_PRiloop: case P_PRiloop5: case P_PRmloop: case P_PRmloop00: case P_PRmloop01:
        case P_PRmloop10: case P_PMiloop: case P_PMiloop5: case P_PMmloop: case P_PMmloop00: case P_PMmloop01:
        case P_PMmloop10: case P_POiloop: case P_POiloop5: case P_POmloop: case P_POmloop00: case P_POmloop01:
        case P_POmloop10: case P_WB: case P_WBP: case P_WP: case P_WPP: case P_P:
            pl(cur);
            break;
        default:
            ++st.n_snbh;  // "Should not be here!" (A-B1: P_PfromMprime / P_PfromMdoubleprime)
    }
}

__device__ __forceinline__ void Bt::bt_loop(const Interval &cur) {
    const int i = cur.i, j = cur.j;
    if (i >= j) return;
    const int type = H.Vtype(i, j);
    if (lane_id() == 0) {
        f_pair[i] = j;
        f_pair[j] = i;
    }
    if (type == T_HAIRP) {
        pairup(i, j, T_HAIRP);
    } else if (type == T_INTER) {
        pairup(i, j, T_INTER);
        // W_final.cc:198-226: k ascending, l descending, first strict minimum
        const int max_ip = imin(j - TURN - 2, i + MAXLOOP + 1);
        int bv, bx;
        scan(imax(max_ip - i, 0) * 32, [&](int c) {
            const int k = i + 1 + (c >> 5), l = j - 1 - (c & 31);
            const int min_l = imax(k + TURN + 1 + MAXLOOP + 2, k + j - i) - MAXLOOP - 2;
            if (l < min_l) return BIG;
            return E_IntLoop(H.T.prm, H.T.lx, k - i - 1, j - l - 1, H.pr(i, j), H.rtype[H.pr(k, l)], H.S1[i + 1],
                             H.S1[j - 1], H.S1[k - 1], H.S1[l + 1]) + H.V(k, l);
        }, bv, bx);
        int best_ip = j, best_jp = i;
        if (bv < INF) {
            best_ip = i + 1 + (bx >> 5);
            best_jp = j - 1 - (bx & 31);
        }
        if (best_ip < best_jp) push2(best_ip, best_jp, LOOP);
        else {
            st.status = BT_INTER;
            st.args[0] = i;
            st.args[1] = j;
            st.args[2] = best_ip;
            st.args[3] = best_jp;
        }
    } else if (type == T_MULTI) {
        pairup(i, j, T_MULTI);
        const short *S = H.S;
        const ccj_energy_params *P = H.T.prm;
        const int tt = H.pr(j, i);
        // W_final.cc:228-300: per k (ascending) rows 1..8 in order
        int bv, bx;
        scan(imax(j - 1 - i, 0) * 8, [&](int c) {
            const int k = i + 1 + (c >> 3), row = (c & 7) + 1;
            switch (row) {
                case 1: return H.WM(i + 1, k - 1) + imin(H.WMv(k, j - 1), H.WMp(k, j - 1)) + E_MLstem(P, tt, -1, -1) + P->MLclosing;
                case 2: return H.WM(i + 2, k - 1) + imin(H.WMv(k, j - 1), H.WMp(k, j - 1)) + E_MLstem(P, tt, -1, S[i + 1]) +
                               P->MLclosing + P->MLbase;
                case 3: return H.WM(i + 1, k - 1) + imin(H.WMv(k, j - 2), H.WMp(k, j - 2)) + E_MLstem(P, tt, S[j - 1], -1) +
                               P->MLclosing + P->MLbase;
                case 4: return H.WM(i + 2, k - 1) + imin(H.WMv(k, j - 2), H.WMp(k, j - 2)) + E_MLstem(P, tt, S[j - 1], S[i + 1]) +
                               P->MLclosing + 2 * P->MLbase;
                case 5: return (k - i - 1) * P->MLbase + H.WMp(k, j - 1) + E_MLstem(P, tt, -1, -1) + P->MLclosing;
                case 6:  // the reference re-tests the previous tmp when the guard fails: no new candidate
                    if ((k - (i + 1) - 1) < 0) return BIG;
                    return (k - (i + 1) - 1) * P->MLbase + H.WMp(k, j - 1) + E_MLstem(P, tt, -1, S[i + 1]) + P->MLclosing + P->MLbase;
                case 7: return (k - i - 1) * P->MLbase + H.WMp(k, j - 2) + E_MLstem(P, tt, S[j - 1], -1) + P->MLclosing + P->MLbase;
                default:
                    if ((k - (i + 1) - 1) < 0) return BIG;
                    return (k - (i + 1) - 1) * P->MLbase + H.WMp(k, j - 2) + E_MLstem(P, tt, S[j - 1], S[i + 1]) + P->MLclosing +
                           2 * P->MLbase;
            }
        }, bv, bx);
        if (bv < INF) {
            const int best_k = i + 1 + (bx >> 3), best_row = (bx & 7) + 1;
            switch (best_row) {
                case 1: push2(i + 1, best_k - 1, M_WM); push2(best_k, j - 1, M_WM); break;
                case 2: push2(i + 2, best_k - 1, M_WM); push2(best_k, j - 1, M_WM); break;
                case 3: push2(i + 1, best_k - 1, M_WM); push2(best_k, j - 2, M_WM); break;
                case 4: push2(i + 2, best_k - 1, M_WM); push2(best_k, j - 2, M_WM); break;
                case 5: push2(best_k, j - 1, M_WM); break;
                case 6: push2(best_k, j - 1, M_WM); break;
                case 7: push2(best_k, j - 2, M_WM); break;
                case 8: push2(best_k, j - 2, M_WM); break;
            }
        }
    }
}

__device__ __forceinline__ void Bt::bt_free(const Interval &cur) {
    const int j = cur.j, n = H.n;
    if (j == 1) return;
    const short *S = H.S;
    const int dangles = H.T.dangles;
    const int *W = H.W;
    int mn = INF, best_row = -1, best_i = -1;
    if (W[j - 1] < mn) {
        mn = W[j - 1];
        best_row = 0;
    }
    // W_final.cc:316-360: i ascending, rows 1..4
    int bv, bx;
    scan((j - 1) * 4, [&](int c) {
        const int i = 1 + (c >> 2), row = (c & 3) + 1;
        const int acc = (i > 1) ? W[i - 1] : 0;
        if (row == 1) {
            const int eij = H.V(i, j);
            if (eij >= INF) return BIG;
            if (dangles == 2) return eij + E_ExtLoop(H.T.prm, H.pr(i, j), i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1) + acc;
            return eij + E_ExtLoop(H.T.prm, H.pr(i, j), -1, -1) + acc;
        }
        if (dangles != 1) return BIG;
        if (row == 2) {
            const int eij = H.V(i + 1, j);
            return eij < INF ? eij + E_ExtLoop(H.T.prm, H.pr(i + 1, j), S[i], -1) + acc : BIG;
        }
        if (row == 3) {
            const int eij = H.V(i, j - 1);
            return eij < INF ? eij + E_ExtLoop(H.T.prm, H.pr(i, j - 1), -1, S[j]) + acc : BIG;
        }
        const int eij = H.V(i + 1, j - 1);
        return eij < INF ? eij + E_ExtLoop(H.T.prm, H.pr(i + 1, j - 1), S[i], S[j]) + acc : BIG;
    }, bv, bx);
    if (bv < mn) {
        mn = bv;
        best_i = 1 + (bx >> 2);
        best_row = (bx & 3) + 1;
    }
    // W_final.cc:362-395: P rows 5..8
    scan((j - 1) * 4, [&](int c) {
        const int i = 1 + (c >> 2), row = (c & 3) + 5;
        const int acc = (i - 1 > 0) ? W[i - 1] : 0;
        int eij;
        if (row == 5) eij = H.Pg(i, j);
        else if (dangles != 1) return BIG;
        else if (row == 6) eij = H.Pg(i + 1, j);
        else if (row == 7) eij = H.Pg(i, j - 1);
        else eij = H.Pg(i + 1, j - 1);
        return eij < INF ? eij + H.T.pen.PS + acc : BIG;
    }, bv, bx);
    if (bv < mn) {
        mn = bv;
        best_i = 1 + (bx >> 2);
        best_row = (bx & 3) + 5;
    }
    switch (best_row) {
        case 0: push2(1, j - 1, FREE); break;
        case 1: push2(best_i, j, LOOP); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
        case 2: push2(best_i + 1, j, LOOP); if (best_i >= 1) push2(1, best_i, FREE); break;
        case 3: push2(best_i, j - 1, LOOP); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
        case 4: push2(best_i + 1, j - 1, LOOP); if (best_i >= 1) push2(1, best_i, FREE); break;
        case 5: push2(best_i, j, P_P); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
        case 6: push2(best_i + 1, j, P_P); if (best_i >= 1) push2(1, best_i, FREE); break;
        case 7: push2(best_i, j - 1, P_P); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
        case 8: push2(best_i + 1, j - 1, P_P); if (best_i >= 1) push2(1, best_i, FREE); break;
    }
}

__device__ __forceinline__ void Bt::bt_wm(const Interval &cur) {
    const int i = cur.i, j = cur.j;
    const int MLb = H.T.prm->MLbase;
    int mn = H.WM(i, j - 1) + MLb;
    int best_k = j, best_row = 5;
    // W_final.cc:408-440: k ascending, rows 1..4
    int bv, bx;
    scan(imax(j - TURN - i, 0) * 4, [&](int c) {
        const int k = i + (c >> 2), row = (c & 3) + 1;
        switch (row) {
            case 1: return (k - i) * MLb + H.WMv(k, j);
            case 2: return (k - i) * MLb + H.WMp(k, j);
            case 3: return H.WM(i, k - 1) + H.WMv(k, j);
            default: return H.WM(i, k - 1) + H.WMp(k, j);
        }
    }, bv, bx);
    if (bv < mn) {
        best_k = i + (bx >> 2);
        best_row = (bx & 3) + 1;
    }
    switch (best_row) {
        case 1: push2(best_k, j, M_WMv); break;
        case 2: push2(best_k, j, M_WMp); break;
        case 3: push2(i, best_k - 1, M_WM); push2(best_k, j, M_WMv); break;
        case 4: push2(i, best_k - 1, M_WM); push2(best_k + 1, j, M_WMp); break;  // A-B3
        case 5: push2(i, j - 1, M_WM); break;
    }
}

__device__ __forceinline__ void Bt::bt_wmv(const Interval &cur) {
    const int i = cur.i, j = cur.j, n = H.n;
    const short *S = H.S;
    const ccj_energy_params *P = H.T.prm;
    const int si = S[i], sj = S[j];
    const int si1 = (i > 1) ? S[i - 1] : -1;
    const int sj1 = (j < n) ? S[j + 1] : -1;
    int tt = H.pr(i, j);
    int mn = H.V(i, j) + ((H.T.dangles == 2) ? E_MLstem(P, tt, si1, sj1) : E_MLstem(P, tt, -1, -1));
    int best_row = 1;
    if (H.T.dangles == 1) {
        tt = H.pr(i + 1, j);
        int tmp = H.V(i + 1, j) + E_MLstem(P, tt, si, -1) + P->MLbase;
        if (tmp < mn) { mn = tmp; best_row = 2; }
        tt = H.pr(i, j - 1);
        tmp = H.V(i, j - 1) + E_MLstem(P, tt, -1, sj) + P->MLbase;
        if (tmp < mn) { mn = tmp; best_row = 3; }
        tt = H.pr(i + 1, j - 1);
        tmp = H.V(i + 1, j - 1) + E_MLstem(P, tt, si, sj) + 2 * P->MLbase;
        if (tmp < mn) { mn = tmp; best_row = 4; }
    }
    const int tmp = H.WMv(i, j - 1) + P->MLbase;
    if (tmp < mn) { mn = tmp; best_row = 5; }
    switch (best_row) {
        case 1: push2(i, j, LOOP); break;
        case 2: push2(i + 1, j, LOOP); break;
        case 3: push2(i, j - 1, LOOP); break;
        case 4: push2(i + 1, j - 1, LOOP); break;
        case 5: push2(i, j - 1, M_WMv); break;
    }
}

__device__ __forceinline__ void Bt::bt_wmp(const Interval &cur) {
    const int i = cur.i, j = cur.j;
    const int mn = H.Pg(i, j) + H.T.pen.PSM + H.T.pen.b;
    const int tmp = H.WMp(i, j - 1) + H.T.prm->MLbase;
    if (tmp < mn) push2(i, j - 1, M_WMp);  // case 1 is commented out in the reference (A-B2)
}

__device__ __forceinline__ void Bt::pl(const Interval &cur) {
    const Penalties &pe = H.T.pen;
    const int PB = pe.PB, bp = pe.bp, cp = pe.cp, ap = pe.ap, n = H.n;
    const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
    int bv, bx;
    switch (cur.type) {
        case P_P: {
            if (i >= l) return die(1, P_P);
            // first (j,d,k) in the reference loop order whose PK(i,j,d+1,k)+PK(j+1,d,k+1,l) is P(i,l)
            // (pseudo_loop.cc:867-896): k_pterm keeps it with the minimum (T.Pk)
            int best_d = 0, best_j = 0, best_k = 0;
            const int target = H.Pg(i, l);
            if (l - i >= 3 && target < INF / 2) {
                const unsigned long long key = H.T.Pk[(l - i) * H.rs + i];
                const unsigned sig = (unsigned)(l - i), kk = (unsigned)(key & 0xffffffffull);
                best_j = i + (int)(kk / (sig * sig));
                best_d = i + (int)((kk / sig) % sig);
                best_k = i + (int)(kk % sig);
            }
            push4(i, best_k, best_j, best_d + 1, P_PK);
            push4(best_j + 1, l, best_d, best_k + 1, P_PK);
        } break;

        case P_PK: {
            if (!order4(i, j, k, l)) return die(2, P_PK);
            if (!in_range4(i, j, k, l)) return die(4, P_PK);
            int mn = INF, best_row = -1, best_d = -1;
            scan(imax(j - i - 1, 0), [&](int c) { const int d = i + 1 + c; return H.g4(PK, i, d, k, l) + H.WP(d + 1, j); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 1; best_d = i + 1 + bx; }
            scan(imax(l - k - 1, 0), [&](int c) { const int d = k + 1 + c; return H.g4(PK, i, j, d, l) + H.WP(k, d - 1); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 2; best_d = k + 1 + bx; }
            int tmp = H.g4(PL, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
            tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
            tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 5; best_d = -1; }
            tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 6; best_d = -1; }
            switch (best_row) {
                case 1: if (best_d > -1) { push4(i, l, best_d, k, P_PK); push2(best_d + 1, j, P_WP); } break;
                case 2: if (best_d > -1) { push4(i, l, j, best_d, P_PK); push2(k, best_d - 1, P_WP); } break;
                case 3: push4(i, l, j, k, P_PL); break;
                case 4: push4(i, l, j, k, P_PM); break;
                case 5: push4(i, l, j, k, P_PR); break;
                case 6: push4(i, l, j, k, P_PO); break;
            }
        } break;

        case P_PL: {
            if (!order4(i, j, k, l)) return die(2, P_PL);
            if (!in_range4(i, j, k, l)) return die(4, P_PL);
            int mn = INF, tmp, best_row = -1;
            if (H.pr(i, j) > 0) {
                tmp = get_PLiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = get_PXmloop(PLmloop10, PLmloop01, i + 1, j - 1, k, l, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                if (j >= i + TURN + 1) { tmp = H.g4(PfromL, i + 1, j - 1, k, l); if (tmp < mn) { mn = tmp; best_row = 3; } }
            }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_PLiloop); break;
                case 2: push4(i, l, j, k, P_PLmloop); break;
                case 3: push4(i + 1, l, j - 1, k, P_PfromL); pairup(i, j, P_PL); break;
            }
        } break;

        case P_PR: {
            if (!order4(i, j, k, l)) return die(3, P_PR);
            if (i < 0 || j < 0 || k < 0 || l < 0 || i >= n || j >= n || k >= n || l >= n) return die(4, P_PR);  // A-B5
            int mn = INF, tmp, best_row = -1;
            if (H.pr(k, l) > 0) {
                tmp = get_PRiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = get_PXmloop(PRmloop10, PRmloop01, i, j, k + 1, l - 1, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                if (l >= k + TURN + 1) { tmp = H.g4(PfromR, i, j, k + 1, l - 1); if (tmp < mn) { mn = tmp; best_row = 3; } }
            }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_PRiloop); break;
                case 2: push4(i, l, j, k, P_PRmloop); break;
                case 3: push4(i, l - 1, j, k + 1, P_PfromR); pairup(k, l, P_PR); break;
            }
        } break;

        case P_PM: {
            if (!order4(i, j, k, l)) return die(2, P_PM);
            if (!in_range4(i, j, k, l)) return die(4, P_PM);
            if (i == j && k == l) { pairup(j, k, P_PM); return; }
            int mn = INF, tmp, best_row = -1;
            if (H.pr(j, k) > 0) {
                tmp = get_PMiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = get_PXmloop(PMmloop10, PMmloop01, i, j - 1, k + 1, l, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                if (k >= j + TURN - 1) { tmp = H.g4(PfromM, i, j - 1, k + 1, l); if (tmp < mn) { mn = tmp; best_row = 3; } }
            }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_PMiloop); break;
                case 2: push4(i, l, j, k, P_PMmloop); break;
                case 3: push4(i, l, j - 1, k + 1, P_PfromM); pairup(j, k, P_PM); break;
            }
        } break;

        case P_PO: {
            if (!order4(i, j, k, l)) return die(2, P_PO);
            if (!in_range4(i, j, k, l)) return die(4, P_PO);
            int mn = INF, tmp, best_row = -1;
            if (H.pr(i, l) > 0) {
                tmp = get_POiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = get_PXmloop(POmloop10, POmloop01, i + 1, j, k, l - 1, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                if (l >= i + TURN + 1) { tmp = H.g4(PfromO, i + 1, j, k, l - 1); if (tmp < mn) { mn = tmp; best_row = 3; } }
            }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_POiloop); break;
                case 2: push4(i, l, j, k, P_POmloop); break;
                case 3: push4(i + 1, l - 1, j, k, P_PfromO); pairup(i, l, P_PO); break;
            }
        } break;

        case P_PfromL: {
            if (!order4(i, j, k, l)) return die(0, P_PfromL);
            if (!in_range4(i, j, k, l)) return die(0, P_PfromL);
            if (i == j && k == l) return;
            int mn = INF, tmp, best_row = -1, best_d = -1;
            scan(imax(j - i - 1, 0) * 2, [&](int c) {
                const int d = i + 1 + (c >> 1);
                return (c & 1) ? H.g4(PfromL, i, d, k, l) + H.WP(d + 1, j) : H.g4(PfromL, d, j, k, l) + H.WP(i, d - 1);
            }, bv, bx);
            if (bv < mn) { mn = bv; best_row = (bx & 1) + 1; best_d = i + 1 + (bx >> 1); }
            tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
            tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
            tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 5; best_d = -1; }
            switch (best_row) {
                case 1: if (best_d > -1) { push4(best_d, l, j, k, P_PfromL); push2(i, best_d - 1, P_WP); } break;
                case 2: if (best_d > -1) { push4(i, l, best_d, k, P_PfromL); push2(best_d + 1, j, P_WP); } break;
                case 3: push4(i, l, j, k, P_PR); break;
                case 4: push4(i, l, j, k, P_PM); break;
                case 5: push4(i, l, j, k, P_PO); break;
            }
        } break;

        case P_PfromR: {
            if (!order4(i, j, k, l)) return die(0, P_PfromR);
            if (!in_range4(i, j, k, l)) return die(5, P_PfromR);
            if (i == j && k == l) return;
            int mn = INF, tmp, best_row = -1, best_d = -1;
            scan(imax(l - k - 1, 0) * 2, [&](int c) {
                const int d = k + 1 + (c >> 1);
                return (c & 1) ? H.g4(PfromR, i, j, k, d) + H.WP(d + 1, l) : H.g4(PfromR, i, j, d, l) + H.WP(k, d - 1);
            }, bv, bx);
            if (bv < mn) { mn = bv; best_row = (bx & 1) + 1; best_d = k + 1 + (bx >> 1); }
            tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
            tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
            switch (best_row) {
                case 1: if (best_d > -1) { push4(i, l, j, best_d, P_PfromR); push2(k, best_d - 1, P_WP); } break;
                case 2: if (best_d > -1) { push4(i, best_d, j, k, P_PfromR); push2(best_d + 1, l, P_WP); } break;
                case 3: push4(i, l, j, k, P_PM); break;
                case 4: push4(i, l, j, k, P_PO); break;
            }
        } break;

        case P_PfromM: {
            if (!order4(i, j, k, l)) return die(0, P_PfromM);
            if (!in_range4(i, j, k, l)) return die(0, P_PfromM);
            if (i == j && k == l) return;
            scan(imax(j - i - 1, 0), [&](int c) { const int d = i + 1 + c; return H.g4(PfromMprime, i, d, k, l) + H.WP(d + 1, j); }, bv, bx);
            if (bv < INF) {
                const int best_d = i + 1 + bx;
                push4(i, l, best_d, k, P_PfromMprime);
                push2(best_d + 1, j, P_WP);
            }
        } break;

        case P_PfromO: {
            if (!order4(i, j, k, l)) return die(2, P_PfromO);
            if (!in_range4(i, j, k, l)) return die(5, P_PfromO);
            if (i == j && k == l) return;
            int mn = INF, tmp, best_row = -1, best_d = -1;
            scan(imax(j - i - 1, 0), [&](int c) { const int d = i + 1 + c; return H.g4(PfromO, d, j, k, l) + H.WP(i, d - 1); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 1; best_d = i + 1 + bx; }
            scan(imax(l - k - 1, 0), [&](int c) { const int d = k + 1 + c; return H.g4(PfromO, i, j, k, d) + H.WP(d + 1, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 2; best_d = k + 1 + bx; }
            tmp = H.g4(PL, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
            tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
            switch (best_row) {
                case 1: if (best_d > -1) { push4(best_d, l, j, k, P_PfromO); push2(i, best_d - 1, P_WP); } break;
                case 2: if (best_d > -1) { push4(i, best_d, j, k, P_PfromO); push2(best_d + 1, l, P_WP); } break;
                case 3: push4(i, l, j, k, P_PL); break;
                case 4: push4(i, l, j, k, P_PR); break;
            }
        } break;

        case P_WB: {
            if (i <= 0 || l <= 0 || i > n || l > n) return die(4, P_WB);
            if (i > l) return;
            int mn = INF, best_row = -1;
            int tmp = H.WBPg(i, l); if (tmp < mn) { mn = tmp; best_row = 1; }
            tmp = cp * (l - i + 1); if (tmp < mn) { mn = tmp; best_row = 2; }
            if (best_row == 1) push2(i, l, P_WBP);
        } break;

        case P_WBP: {
            if (i > l) return die(1, P_WBP);
            if (i <= 0 || l <= 0 || i > n || l > n) return die(4, P_WBP);
            int mn = INF, best_row = -1, best_d = -1;
            scan((l - i) * 2, [&](int c) {
                const int d = i + (c >> 1);
                return (c & 1) ? H.WB(i, d - 1) + H.Pg(d, l) + pe.PSM + pe.PPS : H.WB(i, d - 1) + H.V(d, l) + bp + pe.PPS;
            }, bv, bx);
            if (bv < mn) { mn = bv; best_row = (bx & 1) + 1; best_d = i + (bx >> 1); }
            const int tmp = H.WBPg(i, l - 1) + cp;
            if (tmp < mn) { mn = tmp; best_row = 3; }
            switch (best_row) {
                case 1: push2(i, best_d - 1, P_WB); push2(best_d, l, LOOP); break;
                case 2: push2(i, best_d - 1, P_WB); push2(best_d, l, P_P); break;
                case 3: push2(i, l - 1, P_WBP); break;
            }
        } break;

        case P_WP: {
            if (i <= 0 || l <= 0 || i > n || l > n) return die(4, P_WP);
            if (i > l) return;
            int mn = INF, best_row = -1;
            int tmp = H.WPPg(i, l); if (tmp < mn) { mn = tmp; best_row = 1; }
            tmp = pe.PUP * (l - i + 1); if (tmp < mn) { mn = tmp; best_row = 2; }
            if (best_row == 1) push2(i, l, P_WPP);
        } break;

        case P_WPP: {
            if (i > l) return die(1, P_WPP);
            if (i <= 0 || l <= 0 || i > n || l > n) return die(4, P_WPP);
            int mn = INF, best_row = -1, best_d = -1;
            scan((l - i) * 2, [&](int c) {
                const int d = i + (c >> 1);
                return (c & 1) ? H.WP(i, d - 1) + H.Pg(d, l) + pe.PSP + pe.PPS : H.WP(i, d - 1) + H.V(d, l) + 0 + pe.PPS;
            }, bv, bx);
            if (bv < mn) { mn = bv; best_row = (bx & 1) + 1; best_d = i + (bx >> 1); }
            const int tmp = H.WPPg(i, l - 1) + pe.PUP;
            if (tmp < mn) { mn = tmp; best_row = 3; }
            switch (best_row) {
                case 1: push2(i, best_d - 1, P_WP); push2(best_d, l, LOOP); break;
                case 2: push2(i, best_d - 1, P_WP); push2(best_d, l, P_P); break;
                case 3: push2(i, l - 1, P_WPP); break;
            }
        } break;

        case P_PLiloop: {
            if (!(i < j && j < k - 1 && k < l)) return die(2, P_PLiloop);
            if (!in_range4(i, j, k, l)) return die(6, P_PLiloop);
            pairup(i, j, P_PLiloop);
            int mn = INF, best_row = -1, best_d = -1, best_dp = -1;
            if (H.pr(i, j) > 0) {
                const int tmp = H.g4(PL, i + 1, j - 1, k, l) + H.e_stP(i, j);  // no i+TURN+2<j test here
                if (tmp < mn) { mn = tmp; best_row = 1; }
                const int nd = imin(j, i + MAXLOOP) - (i + 1);
                if (!il_cached(P_PLiloop, i, j, k, l, bv, bx))
                    scan(imax(nd, 0) * 32, [&](int c) {  // d ascending, dp descending; no can_pair filter
                        const int d = i + 1 + (c >> 5), dp = j - 1 - (c & 31);
                        if (dp <= imax(d + TURN, j - MAXLOOP)) return BIG;
                        return H.e_intP(i, d, dp, j) + H.g4(PL, d, dp, k, l);
                    }, bv, bx);
                if (bv < mn) { mn = bv; best_d = i + 1 + (bx >> 5); best_dp = j - 1 - (bx & 31); best_row = 2; }
            }
            switch (best_row) {
                case 1: push4(i + 1, l, j - 1, k, P_PL); break;
                case 2: push4(best_d, l, best_dp, k, P_PL); break;
            }
        } break;

        case P_PLmloop: {
            if (!order4(i, j, k, l)) return die(2, P_PLmloop);
            if (!in_range4(i, j, k, l)) return die(4, P_PLmloop);
            pairup(i, j, P_PLmloop);
            const int br1 = H.g4(PLmloop10, i + 1, j - 1, k, l) + ap + bp;
            const int br2 = H.g4(PLmloop01, i + 1, j - 1, k, l) + ap + bp;
            if (br1 < br2) push4(i + 1, l, j - 1, k, P_PLmloop10);
            else push4(i + 1, l, j - 1, k, P_PLmloop01);
        } break;

        case P_PLmloop00: {
            if (!order4(i, j, k, l)) return die(2, P_PLmloop00);
            if (!in_range4(i, j, k, l)) return die(4, P_PLmloop00);
            const int mn = H.g4(PL, i, j, k, l) + bp;
            scan((j - i + 1) * 2, [&](int c) {  // d ascending; row 2 (d > i) then row 3 (d < j)
                const int d = i + (c >> 1);
                if (!(c & 1)) return d > i ? H.WB(i, d - 1) + H.g4(PLmloop00, d, j, k, l) : BIG;
                return d < j ? H.g4(PLmloop00, i, d, k, l) + H.WB(d + 1, j) : BIG;
            }, bv, bx);
            if (bv < mn) {
                const int best_d = i + (bx >> 1);
                if (!(bx & 1)) { push4(best_d, l, j, k, P_PLmloop00); push2(i, best_d - 1, P_WB); }
                else { push4(i, l, best_d, k, P_PLmloop00); push2(best_d + 1, j, P_WB); }
            } else {
                push4(i, l, j, k, P_PL);
            }
        } break;

        case P_PLmloop01: {
            if (!order4(i, j, k, l)) return die(2, P_PLmloop01);
            if (!in_range4(i, j, k, l)) return die(4, P_PLmloop01);
            scan(j - i, [&](int c) { const int d = i + c; return H.g4(PLmloop00, i, d, k, l) + H.WBPg(d + 1, j); }, bv, bx);
            const int best_d = bv < INF ? i + bx : -1;
            push4(i, l, best_d, k, P_PLmloop00);
            push2(best_d + 1, j, P_WBP);
        } break;

        case P_PLmloop10: {
            if (!order4(i, j, k, l)) return die(2, P_PLmloop10);
            if (!in_range4(i, j, k, l)) return die(4, P_PLmloop10);
            scan((j - i) * 2, [&](int c) {  // d = i+1..j; row 1, then row 2 if d < j
                const int d = i + 1 + (c >> 1);
                if (!(c & 1)) return H.WBPg(i, d - 1) + H.g4(PLmloop00, d, j, k, l);
                return d < j ? H.g4(PLmloop10, i, d, k, l) + H.WB(d + 1, j) : BIG;
            }, bv, bx);
            if (bv < INF) {
                const int best_d = i + 1 + (bx >> 1);
                if (!(bx & 1)) { push2(i, best_d - 1, P_WBP); push4(best_d, l, j, k, P_PLmloop00); }
                else { push4(i, l, best_d, k, P_PLmloop10); push2(best_d + 1, j, P_WB); }
            }
        } break;

        case P_PRiloop: {
            if (!order4(i, j, k, l)) return die(2, P_PRiloop);
            if (!in_range4(i, j, k, l)) return die(4, P_PRiloop);
            pairup(k, l, P_PRiloop);
            int mn = INF, best_row = -1, best_d = -1, best_dp = -1;
            if (H.pr(k, l) > 0) {
                const int tmp = H.g4(PR, i, j, k + 1, l - 1) + H.e_stP(k, l);
                if (tmp < mn) { mn = tmp; best_row = 1; }
                const int nd = imin(l, k + MAXLOOP) - (k + 1);
                if (!il_cached(P_PRiloop, i, j, k, l, bv, bx))
                    scan(imax(nd, 0) * 32, [&](int c) {
                        const int d = k + 1 + (c >> 5), dp = l - 1 - (c & 31);
                        if (dp <= imax(d + TURN, l - MAXLOOP)) return BIG;
                        return H.e_intP(k, d, dp, l) + H.g4(PR, i, j, d, dp);
                    }, bv, bx);
                if (bv < mn) { mn = bv; best_d = k + 1 + (bx >> 5); best_dp = l - 1 - (bx & 31); best_row = 2; }
            }
            switch (best_row) {
                case 1: push4(i, l - 1, j, k + 1, P_PR); break;
                case 2: push4(i, best_dp, j, best_d, P_PR); break;
            }
        } break;

        case P_PRmloop: {
            if (!order4(i, j, k, l)) return die(2, P_PRmloop);
            if (!in_range4(i, j, k, l)) return die(4, P_PRmloop);
            pairup(k, l, P_PRmloop);
            const int br1 = H.g4(PRmloop10, i, j, k + 1, l - 1) + ap + bp;
            const int br2 = H.g4(PRmloop01, i, j, k + 1, l - 1) + ap + bp;
            if (br1 < br2) push4(i, l - 1, j, k + 1, P_PRmloop10);
            else push4(i, l - 1, j, k + 1, P_PRmloop01);
        } break;

        case P_PRmloop00: {
            if (!order4(i, j, k, l)) return die(2, P_PRmloop00);
            if (!in_range4(i, j, k, l)) return die(4, P_PRmloop00);
            const int mn = H.g4(PR, i, j, k, l) + bp;
            scan((l - k + 1) * 2, [&](int c) {
                const int d = k + (c >> 1);
                if (!(c & 1)) return d > k ? H.WB(k, d - 1) + H.g4(PRmloop00, i, j, d, l) : BIG;
                return d < l ? H.g4(PRmloop00, i, j, k, d) + H.WB(d + 1, l) : BIG;
            }, bv, bx);
            if (bv < mn) {  // A-B4: (i,j,k,l) argument order
                const int best_d = k + (bx >> 1);
                if (!(bx & 1)) { push4(i, j, best_d, l, P_PRmloop00); push2(k, best_d - 1, P_WB); }
                else { push4(i, j, k, best_d, P_PRmloop00); push2(best_d + 1, l, P_WB); }
            } else {
                push4(i, j, k, l, P_PR);
            }
        } break;

        case P_PRmloop01: {
            if (!order4(i, j, k, l)) return die(2, P_PRmloop01);
            if (!in_range4(i, j, k, l)) return die(4, P_PRmloop01);
            const int mn = H.g4(PRmloop01, i, j, k, l - 1) + cp;
            scan(l - k, [&](int c) { const int d = k + c; return H.g4(PRmloop00, i, j, k, d) + H.WBPg(d + 1, l); }, bv, bx);
            if (bv < mn) {
                const int best_d = k + bx;
                push2(best_d + 1, l, P_WBP);
                push4(i, best_d, j, k, P_PRmloop00);
            } else {
                push4(i, l - 1, j, k, P_PRmloop01);
            }
        } break;

        case P_PRmloop10: {
            if (!order4(i, j, k, l)) return die(2, P_PRmloop10);
            if (!in_range4(i, j, k, l)) return die(4, P_PRmloop10);
            const int mn = H.g4(PRmloop10, i, j, k + 1, l) + cp;
            scan(l - k, [&](int c) { const int d = k + 1 + c; return H.WBPg(k, d - 1) + H.g4(PRmloop00, i, j, d, l); }, bv, bx);
            if (bv < mn) {
                const int best_d = k + 1 + bx;
                push2(k, best_d - 1, P_WBP);
                push4(i, l, j, best_d, P_PRmloop00);
            } else {
                push4(i, l, j, k + 1, P_PRmloop10);
            }
        } break;

        case P_PMiloop: {
            if (!order4(i, j, k, l)) return die(2, P_PMiloop);
            if (!in_range4(i, j, k, l)) return die(4, P_PMiloop);
            pairup(j, k, P_PMiloop);
            int mn = INF, best_d = -1, best_dp = -1, best_row = -1;
            if (H.pr(j, k) > 0) {
                const int tmp = H.g4(PM, i, j - 1, k + 1, l) + H.e_stP(j - 1, k + 1);
                if (tmp < mn) { mn = tmp; best_row = 1; }
                const int nd = (j - 1) - imax(i, j - MAXLOOP);
                const int min_dp = imin(l, k + MAXLOOP);
                if (!il_cached(P_PMiloop, i, j, k, l, bv, bx))
                    scan(imax(nd, 0) * 32, [&](int c) {  // d descending, dp ascending
                        const int d = j - 1 - (c >> 5), dp = k + 1 + (c & 31);
                        if (dp >= min_dp) return BIG;
                        return H.e_intP(d, j, k, dp) + H.g4(PM, i, d, dp, l);
                    }, bv, bx);
                if (bv < mn) { mn = bv; best_d = j - 1 - (bx >> 5); best_dp = k + 1 + (bx & 31); best_row = 2; }
            }
            switch (best_row) {
                case 1: push4(i, l, j - 1, k + 1, P_PM); break;
                case 2: push4(i, l, best_d, best_dp, P_PM); break;
            }
        } break;

        case P_PMmloop: {
            if (!order4(i, j, k, l)) return die(2, P_PMmloop);
            if (!in_range4(i, j, k, l)) return die(4, P_PMmloop);
            pairup(j, k, P_PMmloop);
            const int br1 = H.g4(PMmloop10, i, j - 1, k + 1, l) + ap + bp;
            const int br2 = H.g4(PMmloop01, i, j - 1, k + 1, l) + ap + bp;
            if (br1 < br2) push4(i, l, j - 1, k + 1, P_PMmloop10);
            else push4(i, l, j - 1, k + 1, P_PMmloop01);
        } break;

        case P_PMmloop00: {
            if (!order4(i, j, k, l)) return die(2, P_PMmloop00);
            if (!in_range4(i, j, k, l)) return die(4, P_PMmloop00);
            pairup(j, k, P_PMmloop);
            int mn = H.g4(PM, i, j, k, l) + bp, best_row = 1, best_d = -1;
            scan(j - i, [&](int c) { const int d = i + c; return H.WB(d + 1, j) + H.g4(PMmloop00, i, d, k, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 2; best_d = i + bx; }
            scan(l - k, [&](int c) { const int d = k + 1 + c; return H.g4(PMmloop00, i, j, d, l) + H.WB(k, d - 1); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 3; best_d = k + 1 + bx; }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_PM); break;
                case 2: push4(i, l, best_d, k, P_PMmloop00); push2(best_d + 1, j, P_WB); break;
                case 3: push4(i, l, j, best_d, P_PMmloop00); push2(k, best_d - 1, P_WB); break;
            }
        } break;

        case P_PMmloop01: {
            if (!order4(i, j, k, l)) return die(2, P_PMmloop01);
            if (!in_range4(i, j, k, l)) return die(4, P_PMmloop01);
            const int mn = H.g4(PMmloop01, i, j, k + 1, l) + cp;
            scan(l - k, [&](int c) { const int d = k + 1 + c; return H.g4(PMmloop00, i, j, d, l) + H.WBPg(k, d - 1); }, bv, bx);
            if (bv < mn) {
                const int best_d = k + 1 + bx;
                push4(i, l, j, best_d, P_PMmloop00);
                push2(k, best_d - 1, P_WBP);
            } else {
                push4(i, l, j, k + 1, P_PMmloop01);
            }
        } break;

        case P_PMmloop10: {
            if (!order4(i, j, k, l)) return die(2, P_PMmloop10);
            if (!in_range4(i, j, k, l)) return die(4, P_PMmloop10);
            const int mn = H.g4(PMmloop10, i, j - 1, k, l) + cp;
            scan(imax(j - i - 1, 0), [&](int c) { const int d = i + 1 + c; return H.WBPg(d, j) + H.g4(PMmloop00, i, d - 1, k, l); }, bv, bx);
            if (bv < mn) {
                const int best_d = i + 1 + bx;
                push4(i, l, best_d - 1, k, P_PMmloop00);
                push2(best_d, j, P_WBP);
            } else {
                push4(i, l, j - 1, k, P_PMmloop10);
            }
        } break;

        case P_POiloop: {
            if (!in_range4(i, j, k, l)) return die(4, P_POiloop);
            if (!order4(i, j, k, l)) return die(2, P_POiloop);
            pairup(i, l, P_POiloop);
            int mn = INF, best_d = -1, best_dp = -1, best_row = -1;
            if (H.pr(i, l) > 0) {
                const int tmp = H.g4(PO, i + 1, j, k, l - 1) + H.e_stP(i, l);
                if (tmp < mn) { mn = tmp; best_row = 1; }
                const int nd = imin(j, i + MAXLOOP) - (i + 1);
                const int min_dp = imax(l - MAXLOOP, k);
                if (!il_cached(P_POiloop, i, j, k, l, bv, bx))
                    scan(imax(nd, 0) * 32, [&](int c) {  // reads PO(d,j,dp,k) with dp > k: always INF (A-Q5)
                        const int d = i + 1 + (c >> 5), dp = l - 1 - (c & 31);
                        if (dp <= min_dp) return BIG;
                        return H.e_intP(i, d, dp, l) + H.g4(PO, d, j, dp, k);
                    }, bv, bx);
                if (bv < mn) { mn = bv; best_row = 2; best_d = i + 1 + (bx >> 5); best_dp = l - 1 - (bx & 31); }
            }
            switch (best_row) {
                case 1: push4(i + 1, l - 1, j, k, P_PO); break;
                case 2: push4(best_d, k, j, best_dp, P_PO); break;
            }
        } break;

        case P_POmloop: {
            if (!order4(i, j, k, l)) return die(2, P_POmloop);
            if (!in_range4(i, j, k, l)) return die(4, P_POmloop);
            pairup(i, l, P_POmloop);
            const int br1 = H.g4(POmloop10, i + 1, j, k, l - 1) + ap + bp;
            const int br2 = H.g4(POmloop01, i + 1, j, k, l - 1) + ap + bp;
            if (br1 < br2) push4(i + 1, l - 1, j, k, P_POmloop10);
            else push4(i + 1, l - 1, j, k, P_POmloop01);
        } break;

        case P_POmloop00: {
            if (!order4(i, j, k, l)) return die(2, P_POmloop00);
            if (!in_range4(i, j, k, l)) return die(4, P_POmloop00);
            int mn = H.g4(PO, i, j, k, l) + bp, best_row = 1, best_d = -1;
            scan(j - i, [&](int c) { const int d = i + 1 + c; return H.WB(i, d - 1) + H.g4(POmloop00, d, j, k, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 2; best_d = i + 1 + bx; }
            scan(l - k, [&](int c) { const int d = k + c; return H.g4(POmloop00, i, j, k, d) + H.WB(d + 1, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 3; best_d = k + bx; }
            switch (best_row) {
                case 1: push4(i, l, j, k, P_PO); break;
                case 2: push4(best_d, l, j, k, P_POmloop00); push2(i, best_d - 1, P_WBP); break;  // sic
                case 3: push4(i, best_d, j, k, P_POmloop00); push2(best_d + 1, l, P_WB); break;
            }
        } break;

        case P_POmloop01: {
            if (!order4(i, j, k, l)) return die(2, P_POmloop01);
            if (!in_range4(i, j, k, l)) return die(4, P_POmloop01);
            scan(l - k, [&](int c) { const int d = k + c; return H.g4(POmloop00, i, j, k, d) + H.WBPg(d + 1, l); }, bv, bx);
            const int best_d = bv < INF ? k + bx : -1;
            push4(i, best_d, j, k, P_POmloop00);
            push2(best_d + 1, l, P_WBP);
        } break;

        case P_POmloop10: {
            if (!order4(i, j, k, l)) return die(2, P_POmloop10);
            if (!in_range4(i, j, k, l)) return die(4, P_POmloop10);
            int mn = INF, best_row = -1, best_d = -1;
            scan(j - i, [&](int c) { const int d = i + 1 + c; return H.WBPg(i, d - 1) + H.g4(POmloop00, d, j, k, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 1; best_d = i + 1 + bx; }
            scan(imax(l - k - 1, 0), [&](int c) { const int d = k + 1 + c; return H.g4(POmloop10, i, j, k, d) + H.WB(d + 1, l); }, bv, bx);
            if (bv < mn) { mn = bv; best_row = 2; best_d = k + 1 + bx; }
            switch (best_row) {
                case 1: push4(best_d, l, j, k, P_POmloop00); push2(i, best_d - 1, P_WBP); break;
                case 2: push4(i, best_d, j, k, P_POmloop10); push2(best_d + 1, l, P_WB); break;
            }
        } break;

        default:
            break;  // P_PLiloop5 etc.: no case in pseudo_loop::backtrack
    }
}

// one workgroup of 1..BT_MAXW waves; LDS: the node stack (cap entries)
__global__ __launch_bounds__(64 * BT_MAXW) void k_backtrack(DevTables T, const int *W, int *f_pair, int8_t *f_type, BtOut *out, int cap,
                                                            int lds_ld) {
    extern __shared__ Interval stk[];
    const int n = T.n;
    // LDS copies of the small tables behind every candidate's first loads (sequence, pair types,
    // level descriptors), placed after the node stack; the descriptors only when they fit (lds_ld)
    short *sS = (short *)(stk + cap), *sS1 = sS + (n + 2);
    int8_t *sPair = (int8_t *)(sS1 + (n + 2)), *sRt = sPair + 64;
    LvlDev *sLd = (LvlDev *)(((unsigned long long)(sRt + 8) + 15) & ~15ull);
    for (int x = (int)threadIdx.x; x < n + 2; x += (int)blockDim.x) {
        sS[x] = T.S[x];
        sS1[x] = T.S1[x];
    }
    for (int x = (int)threadIdx.x; x < 72; x += (int)blockDim.x) {
        if (x < 64) sPair[x] = T.pair[x];
        else sRt[x - 64] = T.rtype[x - 64];
    }
    if (lds_ld)
        for (int x = (int)threadIdx.x; x < T.nlev; x += (int)blockDim.x) sLd[x] = T.ld[x];
    DV H{T, n, T.rs, W, 0, sS, sS1, sPair, sRt, lds_ld ? sLd : T.ld};
    for (int x = (int)threadIdx.x; x <= n; x += (int)blockDim.x) {
        f_pair[x] = -1;
        f_type[x] = (int8_t)T_NONE;
    }
    __syncthreads();  // the pair list is cleared before lane 0 starts writing pairs
    Bt B{H, stk, cap, 0, f_pair, f_type, BtOut{}};
    B.push2(1, n, FREE);  // W_final.cc:84-99
    __syncthreads();
    while (B.sp > 0 && B.st.status == BT_OK) {
        const Interval cur = stk[B.sp - 1];
        __syncthreads();  // every lane has read the top before lane 0 overwrites it
        --B.sp;
        ++B.st.steps;
        B.node(cur);
        // a get_uc assert on any lane of any wave; the barrier also publishes lane 0's pushes
        if (__syncthreads_or(H.bad)) B.st.status = BT_ASSERT;
    }
    if (lane_id() == 0) *out = B.st;
}

}  // namespace

extern "C" int ccjk_compute_W(const void *Tv, int *W, int *S, void *stream) {
    const DevTables *T = (const DevTables *)Tv;
    const int n = T->n;
    if (n > TURN) {
        hipLaunchKernelGGL(k_w_terms, dim3((unsigned)((n + 255) / 256), (unsigned)(n - TURN)), dim3(256), 0,
                           (hipStream_t)stream, *T, S);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    const hipStream_t s = (hipStream_t)stream;
    switch ((n + 64) / 64) {  // slots for W[0..n]
        case 1: hipLaunchKernelGGL(k_compute_W_reg<1>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 2: hipLaunchKernelGGL(k_compute_W_reg<2>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 3: hipLaunchKernelGGL(k_compute_W_reg<3>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 4: hipLaunchKernelGGL(k_compute_W_reg<4>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 5: hipLaunchKernelGGL(k_compute_W_reg<5>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 6: hipLaunchKernelGGL(k_compute_W_reg<6>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 7: hipLaunchKernelGGL(k_compute_W_reg<7>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        case 8: hipLaunchKernelGGL(k_compute_W_reg<8>, dim3(1), dim3(64), 0, s, *T, S, W); break;
        default: hipLaunchKernelGGL(k_compute_W, dim3(1), dim3(64), (n + 1) * sizeof(int), s, *T, S, W);
    }
    return (int)hipGetLastError();
}

extern "C" int ccjk_backtrack(const void *Tv, const int *W, int *f_pair, int8_t *f_type, BtOut *out, int stack_cap,
                              void *stream) {
    const DevTables *T = (const DevTables *)Tv;
    static const int waves = [] {
        const char *e = getenv("CCJ_BT_WAVES");
        const int w = e ? atoi(e) : BT_WAVES_DEFAULT;
        return w < 1 ? 1 : (w > BT_MAXW ? BT_MAXW : w);
    }();
    // dynamic LDS: the node stack, then the small tables (k_backtrack); the level descriptors too
    // while the whole stays within 64 KB
    const size_t base = (size_t)stack_cap * sizeof(Interval) + 4 * ((size_t)T->n + 2) + 72 + 16;
    const size_t with_ld = base + (size_t)T->nlev * sizeof(LvlDev);
    const int lds_ld = with_ld <= 65536 ? 1 : 0;
    hipLaunchKernelGGL(k_backtrack, dim3(1), dim3(64 * waves), lds_ld ? with_ld : base, (hipStream_t)stream, *T, W, f_pair,
                       f_type, out, stack_cap, lds_ld);
    return (int)hipGetLastError();
}
