// ccj_kernels.hip — hand-written HIP kernels (gfx950, wave64) for the CCJ MFE fill.
//
// Schedule: for sigma = 0..n-1
//     k_diag2d(sigma)   : every 2-D interval value of span sigma (V, P, WBP, WPP, WMv, WMp, WM)
//     k_level4d(t=sigma): every 4-D cell of level t = (j-i)+(l-k), all 22 gap matrices
// Level t reads only 4-D levels < t and 2-D spans <= t-1; span sigma reads 4-D levels <= sigma-3.
// Within a cell the 22 recurrences run in the reference's order (pseudo_loop.cc:85-127), so the
// same-cell reads (PfromL/PfromR/PfromO/PK read PL/PR/PM/PO of the cell) see the finished
// values and the P?mloop00 seeds see the initial 32767.
// All arithmetic is int32 min-plus; storage is int16 with the reference clamp at 32767.
#include <hip/hip_runtime.h>
#include "ccj_engine.h"
#include "ccj_energy.h"

using namespace ccj;

namespace {

__device__ __forceinline__ int clamp_store(int v) { return v >= INTERN_INF ? INTERN_INF : v; }

// 4-D read of matrix x at level tp, block ap, row hp, position ip (reference Matrix4D::get on a
// cell known to be valid).  tp/ap are wave-uniform, so the LevelDesc loads are scalar.
__device__ __forceinline__ int ld4(const DevTables &T, int x, int tp, int ap, int hp, int ip) {
#ifdef CCJ_DEBUG_BOUNDS
    // debug build: every read must be a valid cell of an earlier level (else flag, no access)
    if (tp < 0 || tp >= T.nlev || ap < 0 || ap > tp || hp < 0 || hp >= T.lv[tp].m || ip < 1 ||
        ip > T.lv[tp].m - hp || x < 0 || x >= NMAT4) {
        atomicOr(T.err, 4);
        return 0;
    }
#endif
    const LevelDesc &L = T.lv[tp];
    const int off = x * L.C + ap * L.M + hp * L.m - ((hp * (hp - 1)) >> 1) + ip - 1;
    return (int)L.base[off];
}

#ifdef CCJ_DEBUG_BOUNDS
__device__ int *g_dbg_err;
#endif

template <class TT>
__device__ __forceinline__ int at2(const TT *A, int rs, int p, int q) {
#ifdef CCJ_DEBUG_BOUNDS
    if (p < 1 || q < p || q > rs - 2) {
        atomicOr(g_dbg_err, 8);
        return 0;
    }
#endif
    return (int)A[(q - p) * rs + p];
}

// s_energy_matrix.hh:37-43 getters: INF for i >= j
__device__ __forceinline__ int gV(const DevTables &T, int i, int j) { return i >= j ? INF : at2(T.V, T.rs, i, j); }
__device__ __forceinline__ int gWM(const DevTables &T, int i, int j) { return i >= j ? INF : at2(T.WM, T.rs, i, j); }
__device__ __forceinline__ int gWMv(const DevTables &T, int i, int j) { return i >= j ? INF : at2(T.WMv, T.rs, i, j); }
__device__ __forceinline__ int gWMp(const DevTables &T, int i, int j) { return i >= j ? INF : at2(T.WMp, T.rs, i, j); }

__device__ __forceinline__ int ptype(const DevTables &T, int i, int j) { return T.pt[(j - i) * T.rs + i]; }

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = imin(v, __shfl_xor(v, o, 64));
    return v;
}

// min over the 256-thread block, result returned to every thread
__device__ __forceinline__ int block_min(int v, int *red) {
    v = wave_min(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return imin(imin(red[0], red[1]), imin(red[2], red[3]));
}

// s_energy_matrix.cc:54-112
__device__ int E_MLStem_d(const DevTables &T, int vij, int vi1j, int vij1, int vi1j1, int i, int j) {
    const ccj_energy_params *P = T.prm;
    const short *S = T.S;
    const int n = T.n;
    int e = INF, en;
    int type = T.pair[S[i] * 8 + S[j]];
    en = vij;
    if (en != INF) {
        if (T.dangles == 2) en += E_MLstem(P, type, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1);
        else en += E_MLstem(P, type, -1, -1);
        e = imin(e, en);
    }
    if (T.dangles == 1) {
        const int mm5 = S[i], mm3 = S[j];
        en = (j - i - 1 > TURN) ? vi1j : INF;
        if (en != INF) { en += P->MLbase + E_MLstem(P, T.pair[S[i + 1] * 8 + S[j]], mm5, -1); e = imin(e, en); }
        en = (j - 1 - i > TURN) ? vij1 : INF;
        if (en != INF) { en += P->MLbase + E_MLstem(P, T.pair[S[i] * 8 + S[j - 1]], -1, mm3); e = imin(e, en); }
        en = (j - 1 - i - 1 > TURN) ? vi1j1 : INF;
        if (en != INF) { en += 2 * P->MLbase + E_MLstem(P, T.pair[S[i + 1] * 8 + S[j - 1]], mm5, mm3); e = imin(e, en); }
    }
    return e;
}

// s_energy_matrix.cc:122-205
__device__ int E_MbLoop_d(const DevTables &T, int WM2ij, int WM2ip1j, int WM2ijm1, int WM2ip1jm1, int i, int j) {
    const ccj_energy_params *P = T.prm;
    const short *S = T.S;
    int e = INF, en;
    const int tt = T.pair[S[j] * 8 + S[i]];
    switch (T.dangles) {
        case 2:
            e = WM2ij;
            if (e != INF) e += E_MLstem(P, tt, S[j - 1], S[i + 1]) + P->MLclosing;
            break;
        case 1:
            e = WM2ij;
            if (e != INF) e += E_MLstem(P, tt, -1, -1) + P->MLclosing;
            en = WM2ip1j;
            if (en != INF) en += E_MLstem(P, tt, -1, S[i + 1]) + P->MLclosing + P->MLbase;
            e = imin(e, en);
            en = WM2ijm1;
            if (en != INF) en += E_MLstem(P, tt, S[j - 1], -1) + P->MLclosing + P->MLbase;
            e = imin(e, en);
            en = WM2ip1jm1;
            if (en != INF) en += E_MLstem(P, tt, S[j - 1], S[i + 1]) + P->MLclosing + 2 * P->MLbase;
            e = imin(e, en);
            break;
        case 0:
            e = WM2ij;
            if (e != INF) e += E_MLstem(P, tt, -1, -1) + P->MLclosing;
            break;
    }
    return e;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// 2-D init: reference initial values (h_struct.hh:100 V = 10000 'N'; matrices.hh:25 INF+1)
// ------------------------------------------------------------------------------------------
__global__ void k_init2d(DevTables T, int total) {
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < total; x += gridDim.x * blockDim.x) {
        T.V[x] = 10000;
        T.Vt[x] = 'N';
        T.WM[x] = T.WMv[x] = T.WMp[x] = INF + 1;
        T.P[x] = T.WBP[x] = T.WPP[x] = INF + 1;
        T.WB[x] = 0;
        T.WP[x] = 0;
    }
}

// ------------------------------------------------------------------------------------------
// e_intP table: IE[u1][u2][w][p] = lrint(e_intP * E_IntLoop(...)) for outer (p, p+w) and inner
// (p+u1+1, p+w-u2-1)  (pseudo_loop.cc:822-826, 836-840).  The reference skips a candidate unless
// both pairs can pair (get_P?iloop's can_pair tests); such entries hold 32767, and the matrix value
// they are added to is then the never-set 32767 of that pair, so the sum can never
// undercut a stored value (all stores clamp at 32767).
// ------------------------------------------------------------------------------------------
__global__ void k_precompute_ie(DevTables T) {
    const int n = T.n, rs = T.rs;
    const int w = blockIdx.y;          // outer span
    const int uu = blockIdx.z;         // u1*29+u2
    const int u1 = uu / IE_U, u2 = uu - u1 * IE_U;
    for (int p = 1 + blockIdx.x * blockDim.x + threadIdx.x; p + w <= n; p += gridDim.x * blockDim.x) {
        const int q = p + w;
        const int d = p + u1 + 1, dp = q - u2 - 1;
        int16_t out = INTERN_INF;
        if (dp - d >= 1) {
            const int t1 = T.pair[T.S[p] * 8 + T.S[q]];
            const int t2 = T.pair[T.S[d] * 8 + T.S[dp]];
            const int e = E_IntLoop(T.prm, T.lx, u1, u2, t1, T.rtype[t2], T.S1[p + 1], T.S1[q - 1], T.S1[d - 1],
                                    T.S1[dp + 1]);
            const int v = (int)rint(T.e_intP * (double)e);
            if (t1 > 0 && t2 > 0) {
                // the reference only visits candidates with can_pair() on both pairs
                if (v < -32768 || v >= INTERN_INF) atomicOr(T.err, 1);
                out = (int16_t)v;
            }
        }
        T.ie[((size_t)uu * (n + 1) + w) * rs + p] = out;
    }
}

// ------------------------------------------------------------------------------------------
// 2-D anti-diagonal sigma: one 256-thread workgroup per interval (i, l = i+sigma).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_diag2d(DevTables T, int sigma) {
#ifdef CCJ_DEBUG_BOUNDS
    g_dbg_err = T.err;
#endif
    __shared__ int red[4];
    __shared__ int sh_v, sh_p;
    const int n = T.n, rs = T.rs;
    const int i = blockIdx.x + 1;
    const int l = i + sigma;
    if (l > n) return;
    const int tid = threadIdx.x;
    const ccj_energy_params *Pp = T.prm;
    const int cell = sigma * rs + i;

    // ---- V(i,l): s_energy_matrix.cc:315-358
    {
        const int tc = ptype(T, i, l);
        int best_int = INF;
        const int max_k = imin(l - TURN - 2, i + MAXLOOP + 1);
        const int off = imax(TURN + 1, sigma - MAXLOOP - 2);  // min_l = k + off  (:292)
        const int nk = max_k - i;
        for (int idx = tid; idx < nk * 32; idx += 256) {
            const int k = i + 1 + (idx >> 5);
            const int lp = l - 1 - (idx & 31);
            if (lp < k + off) continue;
            const int e = E_IntLoop(Pp, T.lx, k - i - 1, l - lp - 1, tc, T.rtype[ptype(T, k, lp)], T.S1[i + 1],
                                    T.S1[l - 1], T.S1[k - 1], T.S1[lp + 1]) + gV(T, k, lp);
            best_int = imin(best_int, e);
        }
        int best_vm = INF;  // compute_energy_VM :243-268
        const int MLb = Pp->MLbase;
        for (int k = i + 1 + tid; k <= l - 3; k += 256) {
            int A = gWM(T, i + 1, k - 1) + gWMv(T, k, l - 1);
            A = imin(A, gWM(T, i + 1, k - 1) + gWMp(T, k, l - 1));
            A = imin(A, (k - i - 1) * MLb + gWMp(T, k, l - 1));
            int B = gWM(T, i + 2, k - 1) + gWMv(T, k, l - 1);
            B = imin(B, gWM(T, i + 2, k - 1) + gWMp(T, k - 1, l - 1));  // sic (A-Q7)
            B = imin(B, (k - (i + 1) - 1) * MLb + gWMp(T, k, l - 1));
            int C = gWM(T, i + 1, k - 1) + gWMv(T, k, l - 2);
            C = imin(C, gWM(T, i + 1, k - 1) + gWMp(T, k, l - 2));
            C = imin(C, (k - i - 1) * MLb + gWMp(T, k, l - 2));
            int D = gWM(T, i + 2, k - 1) + gWMv(T, k, l - 2);
            D = imin(D, gWM(T, i + 2, k - 1) + gWMp(T, k, l - 2));
            D = imin(D, (k - (i + 1) - 1) * MLb + gWMp(T, k, l - 2));
            best_vm = imin(best_vm, E_MbLoop_d(T, A, B, C, D, i, l));
        }
        best_int = block_min(best_int, red);
        best_vm = block_min(best_vm, red);
        if (tid == 0) {
            const int en[3] = {T.hp[cell], best_int, best_vm};
            int mn = INF / 2, rank = -1;
            for (int x = 0; x < 3; ++x)
                if (en[x] < mn) { mn = en[x]; rank = x; }
            int v = 10000;
            int8_t ty = 'N';
            if (mn < INF / 2) {
                v = mn;
                ty = rank == 0 ? 'H' : rank == 1 ? 'I' : 'M';
                T.V[cell] = v;
                T.Vt[cell] = ty;
            }
            sh_v = v;
        }
    }

    // ---- P(i,l): pseudo_loop.cc:166-179 (PK of levels <= sigma-3 only)
    {
        int best = INF;
        const int sq = sigma * sigma;
        for (int idx = tid; idx < sq; idx += 256) {
            const int j = i + idx / sigma;
            const int d = i + idx % sigma;
            if (!(j < d && d <= l - 2)) continue;
            const int a1 = j - i, h1 = d - 1 - j;  // PK(i, j, d+1, k)
            const int a2 = d - j - 1;              // PK(j+1, d, k+1, l)
            for (int k = d + 1; k < l; ++k) {
                const int b1 = k - d - 1, h2 = k - 1 - d, b2 = l - k - 1;
                const int v = ld4(T, PK, a1 + b1, a1, h1, i) + ld4(T, PK, a2 + b2, a2, h2, j + 1);
                best = imin(best, v);
            }
        }
        best = block_min(best, red);
        if (tid == 0) {
            int p = INF + 1;
            if (best < INF / 2) { p = best; T.P[cell] = p; }
            sh_p = p;
        }
        __syncthreads();
    }
    const int v_il = sh_v, p_il = sh_p;

    // ---- WBP / WPP: pseudo_loop.cc:134-164 (+ the WB/WP getters :647-661)
    {
        const Penalties &pe = T.pen;
        int bb = INF, bw = INF;
        for (int d = i + tid; d < l; d += 256) {
            // get_WB(i, i-1) is 0, except get_WB(1, 0) which is INF (j <= 0 test first, :648)
            const int wb = (d == i) ? (i == 1 ? INF : 0) : T.WB[(d - 1 - i) * rs + i];
            const int wp = (d == i) ? (i == 1 ? INF : 0) : T.WP[(d - 1 - i) * rs + i];
            const int vd = (d == i) ? v_il : T.V[(l - d) * rs + d];
            const int pd = (d == i) ? p_il : T.P[(l - d) * rs + d];
            bb = imin(bb, imin(wb + vd + pe.bp + pe.PPS, wb + pd + pe.PSM + pe.PPS));
            bw = imin(bw, imin(wp + vd + 0 + pe.PPS, wp + pd + pe.PSP + pe.PPS));
        }
        bb = block_min(bb, red);
        bw = block_min(bw, red);
        if (tid == 0) {
            const int b3 = (sigma == 0 ? INF : T.WBP[(sigma - 1) * rs + i]) + pe.cp;
            int m = imin(bb, b3);
            int wbp = INF + 1;
            if (m < INF / 2) { wbp = m; T.WBP[cell] = m; }
            T.WB[cell] = imin(pe.cp * (sigma + 1), wbp);
            const int c3 = (sigma == 0 ? INF : T.WPP[(sigma - 1) * rs + i]) + pe.PUP;
            m = imin(bw, c3);
            int wpp = INF + 1;
            if (m < INF / 2) { wpp = m; T.WPP[cell] = m; }
            T.WP[cell] = imin(pe.PUP * (sigma + 1), wpp);
        }
    }

    // ---- WMv / WMp / WM: s_energy_matrix.cc:206-241 (only for j-i+1 >= 4)
    if (sigma >= 3) {
        const Penalties &pe = T.pen;
        const int MLb = Pp->MLbase;
        int best = INF;
        for (int k = l - TURN - 1 - tid; k >= i; k -= 256) {
            const int vkl = (k == i) ? v_il : gV(T, k, l);
            const int wm_kj = E_MLStem_d(T, vkl, gV(T, k + 1, l), gV(T, k, l - 1), gV(T, k + 1, l - 1), k, l);
            const int pkl = (k == i) ? p_il : T.P[(l - k) * rs + k];
            const int wmb_kj = pkl + pe.PSM + pe.b;
            const int base = (k - i) * MLb;
            const int wmi = gWM(T, i, k - 1);
            best = imin(best, imin(imin(base + wm_kj, base + wmb_kj), imin(wmi + wm_kj, wmi + wmb_kj)));
        }
        best = block_min(best, red);
        if (tid == 0) {
            const int prev = (sigma - 1) * rs + i;  // raw (i, l-1)
            const int emv = E_MLStem_d(T, v_il, gV(T, i + 1, l), gV(T, i, l - 1), gV(T, i + 1, l - 1), i, l);
            T.WMv[cell] = imin(emv, T.WMv[prev] + MLb);
            T.WMp[cell] = imin(p_il + pe.PSM + pe.b, T.WMp[prev] + MLb);
            T.WM[cell] = imin(best, T.WM[prev] + MLb);
        }
    }
}

// ------------------------------------------------------------------------------------------
// 4-D level t: one lane per cell (i,j,k,l); all lanes of a wave share (t, a) so every loop
// bound is wave-uniform.  pseudo_loop.cc:181-644, 663-808.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_level4d(DevTables T, int t, int wavesPerA) {
#ifdef CCJ_DEBUG_BOUNDS
    g_dbg_err = T.err;
#endif
    const int n = T.n, rs = T.rs;
    const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int a = __builtin_amdgcn_readfirstlane(gw / wavesPerA);
    if (a > t) return;
    const int chunk = gw - a * wavesPerA;
    const int m = n - t - 2;
    const int Mt = (m * (m + 1)) >> 1;
    const int c = chunk * 64 + lane;
    if (c >= Mt) return;
    // row h: largest h with G(h) = h*m - h(h-1)/2 <= c
    const float tm = 2.0f * m + 1.0f;
    int h = (int)((tm - sqrtf(tm * tm - 8.0f * (float)c)) * 0.5f);
    h = imax(0, imin(h, m - 1));
    while (h > 0 && h * m - ((h * (h - 1)) >> 1) > c) --h;
    while (h + 1 < m && (h + 1) * m - (((h + 1) * h) >> 1) <= c) ++h;
    const int Gh = h * m - ((h * (h - 1)) >> 1);
    const int b = t - a;
    const int i = c - Gh + 1;
    const int g = h + 2;
    const int j = i + a, k = j + g, l = k + b;

    const Penalties pe = T.pen;
    const int bp = pe.bp, cp = pe.cp, PB = pe.PB, apbp2 = pe.ap + 2 * pe.bp;
    const int *WB = T.WB, *WP = T.WP, *WBPr = T.WBP;
#define L4(x, dt, ap_, dh, di) ld4(T, (x), t - (dt), (ap_), h + (dh), i + (di))
#ifdef CCJ_DEBUG_BOUNDS
#define IE_CHECK(u1_, u2_, w_, p_) \
    if ((u1_) < 0 || (u1_) >= IE_U || (u2_) < 0 || (u2_) >= IE_U || (w_) < 0 || (w_) > n || (p_) < 1 || (p_) + (w_) > n) atomicOr(T.err, 16)
#else
#define IE_CHECK(u1_, u2_, w_, p_)
#endif
#define W2(A, p, q) at2((A), rs, (p), (q))

    int mv;
    // ---- multiloop-spanning-band recurrences (pseudo_loop.cc:445-644) ----
    // PLmloop00 (:445-463): seed PL(i,j,k,l) is the not-yet-computed 32767
    mv = INTERN_INF + bp;
    for (int s = 1; s <= a; ++s) {
        mv = imin(mv, W2(WB, i, i + s - 1) + L4(PLmloop00, s, a - s, 0, s));
        mv = imin(mv, L4(PLmloop00, s, a - s, s, 0) + W2(WB, j - s + 1, j));
    }
    const int vPLm00 = mv;
    // PLmloop01 (:465-476)
    mv = INF;
    for (int s = 1; s <= a; ++s) mv = imin(mv, L4(PLmloop00, s, a - s, s, 0) + W2(WBPr, j - s + 1, j));
    const int vPLm01 = mv;
    // PLmloop10 (:478-493)
    mv = INF;
    for (int s = 1; s <= a; ++s) {
        mv = imin(mv, W2(WBPr, i, i + s - 1) + L4(PLmloop00, s, a - s, 0, s));
        if (s < a) mv = imin(mv, L4(PLmloop10, a - s, s, a - s, 0) + W2(WB, i + s + 1, j));
    }
    const int vPLm10 = mv;
    // PRmloop00 (:495-513)
    mv = INTERN_INF + bp;
    for (int s = 1; s <= b; ++s) mv = imin(mv, W2(WB, k, k + s - 1) + L4(PRmloop00, s, a, s, 0));
    for (int s = 0; s < b; ++s) mv = imin(mv, L4(PRmloop00, b - s, a, 0, 0) + W2(WB, k + s + 1, l));
    const int vPRm00 = mv;
    // PRmloop01 (:516-528)
    mv = (b >= 1 ? L4(PRmloop01, 1, a, 0, 0) : INF) + cp;
    for (int s = 0; s < b; ++s) mv = imin(mv, L4(PRmloop00, b - s, a, 0, 0) + W2(WBPr, k + s + 1, l));
    const int vPRm01 = mv;
    // PRmloop10 (:530-542)
    mv = (b >= 1 ? L4(PRmloop10, 1, a, 1, 0) : INF) + cp;
    for (int s = 1; s <= b; ++s) mv = imin(mv, W2(WBPr, k, k + s - 1) + L4(PRmloop00, s, a, s, 0));
    const int vPRm10 = mv;
    // PMmloop00 (:544-560)
    mv = INTERN_INF + bp;
    for (int s = 1; s <= a; ++s) mv = imin(mv, L4(PMmloop00, s, a - s, s, 0) + W2(WB, j - s + 1, j));
    for (int s = 1; s <= b; ++s) mv = imin(mv, L4(PMmloop00, s, a, s, 0) + W2(WB, k, k + s - 1));
    const int vPMm00 = mv;
    // PMmloop01 (:563-575)
    mv = (b >= 1 ? L4(PMmloop01, 1, a, 1, 0) : INF) + cp;
    for (int s = 0; s < b; ++s) mv = imin(mv, L4(PMmloop00, b - s, a, 0, 0) + W2(WBPr, k + s + 1, l));
    const int vPMm01 = mv;
    // PMmloop10 (:577-593)
    mv = (a >= 1 ? L4(PMmloop10, 1, a - 1, 1, 0) : INF) + cp;
    for (int s = 1; s <= a; ++s) mv = imin(mv, W2(WBPr, i, i + s - 1) + L4(PMmloop00, s, a - s, 0, s));
    for (int s = 1; s < b; ++s) mv = imin(mv, L4(PMmloop10, b - s, a, 0, 0) + W2(WB, k + s + 1, l));
    const int vPMm10 = mv;
    // POmloop00 (:595-612)
    mv = INTERN_INF + bp;
    for (int s = 1; s <= a; ++s) mv = imin(mv, W2(WB, i, i + s - 1) + L4(POmloop00, s, a - s, 0, s));
    for (int s = 0; s < b; ++s) mv = imin(mv, L4(POmloop00, b - s, a, 0, 0) + W2(WB, k + s + 1, l));
    const int vPOm00 = mv;
    // POmloop01 (:615-627)
    mv = INF;
    for (int s = 0; s < b; ++s) mv = imin(mv, L4(POmloop00, b - s, a, 0, 0) + W2(WBPr, k + s + 1, l));
    const int vPOm01 = mv;
    // POmloop10 (:629-644)
    mv = INF;
    for (int s = 1; s <= a; ++s) mv = imin(mv, W2(WBPr, i, i + s - 1) + L4(POmloop00, s, a - s, 0, s));
    for (int s = 1; s < b; ++s) mv = imin(mv, L4(POmloop10, b - s, a, 0, 0) + W2(WB, k + s + 1, l));
    const int vPOm10 = mv;

    const size_t ie_w = (size_t)(n + 1) * rs;  // stride between (u1,u2) planes of IE
    // ---- PL (:232-253) with get_PLiloop (:682-703), get_PLmloop (:705-715)
    int vPL = INF;
    if (ptype(T, i, j) > 0) {
        int b1 = INF;
        if (a > TURN) {
            if (a > TURN + 2) b1 = L4(PL, 2, a - 2, 1, 1) + W2(T.est, i, j);
            const int mu1 = imin(a, MAXLOOP) - 2;
            for (int u1 = 0; u1 <= mu1; ++u1) {
                const int mu2 = imin(a - u1 - 6, MAXLOOP - 2);
                const int16_t *ie = T.ie + (size_t)(u1 * IE_U) * ie_w + (size_t)a * rs + i;
                for (int u2 = 0; u2 <= mu2; ++u2) {
                    IE_CHECK(u1, u2, a, i);
                    b1 = imin(b1, (int)ie[u2 * ie_w] + L4(PL, 2 + u1 + u2, a - 2 - u1 - u2, u2 + 1, 1 + u1));
                }
            }
        }
        const int b2 = (a >= 2) ? imin(L4(PLmloop10, 2, a - 2, 1, 1), L4(PLmloop01, 2, a - 2, 1, 1)) + apbp2 : INF;
        const int b3 = (a >= TURN + 1) ? L4(PfromL, 2, a - 2, 1, 1) : INF;
        vPL = imin(imin(b1, b2), b3);
    }
    // ---- PR (:255-275) with get_PRiloop (:717-738), get_PRmloop (:740-750)
    int vPR = INF;
    if (ptype(T, k, l) > 0) {
        int b1 = INF;
        if (b > TURN) {
            if (b > TURN + 2) b1 = L4(PR, 2, a, 1, 0) + W2(T.est, k, l);
            const int mu1 = imin(b, MAXLOOP) - 2;
            for (int u1 = 0; u1 <= mu1; ++u1) {
                const int mu2 = imin(b - u1 - 6, MAXLOOP - 2);
                const int16_t *ie = T.ie + (size_t)(u1 * IE_U) * ie_w + (size_t)b * rs + k;
                for (int u2 = 0; u2 <= mu2; ++u2) {
                    IE_CHECK(u1, u2, b, k);
                    b1 = imin(b1, (int)ie[u2 * ie_w] + L4(PR, 2 + u1 + u2, a, 1 + u1, 0));
                }
            }
        }
        const int b2 = (b >= 2) ? imin(L4(PRmloop10, 2, a, 1, 0), L4(PRmloop01, 2, a, 1, 0)) + apbp2 : INF;
        const int b3 = (b >= TURN + 1) ? L4(PfromR, 2, a, 1, 0) : INF;
        vPR = imin(imin(b1, b2), b3);
    }
    // ---- PM (:277-300) with get_PMiloop (:752-773), get_PMmloop (:775-785)
    int vPM = INF;
    if (ptype(T, j, k) > 0) {
        int b1 = INF;
        const bool inner = (a >= 1 && b >= 1);
        if (g > TURN) {
            if (inner) b1 = L4(PM, 2, a - 1, 2, 0) + W2(T.est, j - 1, k + 1);
            const int mu1 = imin(a - 2, MAXLOOP - 2);
            const int mu2 = imin(b - 2, MAXLOOP - 2);
            for (int u1 = 0; u1 <= mu1; ++u1) {
                const int16_t *ie = T.ie + (size_t)(u1 * IE_U) * ie_w + (size_t)(g + 2 + u1) * rs + (j - 1 - u1);
                for (int u2 = 0; u2 <= mu2; ++u2) {
                    IE_CHECK(u1, u2, g + 2 + u1 + u2, j - 1 - u1);
                    b1 = imin(b1, (int)ie[(size_t)u2 * ie_w + (size_t)u2 * rs] +
                                      L4(PM, 2 + u1 + u2, a - 1 - u1, 2 + u1 + u2, 0));
                }
            }
        }
        const int b2 = inner ? imin(L4(PMmloop10, 2, a - 1, 2, 0), L4(PMmloop01, 2, a - 1, 2, 0)) + apbp2 : INF;
        const int b3 = inner ? L4(PfromM, 2, a - 1, 2, 0) : INF;
        const int b4 = (a == 0 && b == 0) ? 0 : INF;
        vPM = imin(imin(b1, b2), imin(b3, b4));
    }
    // ---- PO (:302-322) with get_POiloop (:787-808; interior branch is dead, A-Q5), get_POmloop (:810-820)
    int vPO = INF;
    if (ptype(T, i, l) > 0) {
        const bool inner = (a >= 1 && b >= 1);
        int b1 = INF;
        if (l - i > TURN && inner) b1 = L4(PO, 2, a - 1, 0, 1) + W2(T.est, i, l);
        const int b2 = inner ? imin(L4(POmloop10, 2, a - 1, 0, 1), L4(POmloop01, 2, a - 1, 0, 1)) + apbp2 : INF;
        const int b3 = (inner && l - i >= TURN + 1) ? L4(PfromO, 2, a - 1, 0, 1) : INF;
        vPO = imin(imin(b1, b2), b3);
    }
    // values as stored (Matrix4D::set clamp / never-set 32767), read back by same-cell terms
    const int sPL = clamp_store(vPL), sPR = clamp_store(vPR), sPM = clamp_store(vPM), sPO = clamp_store(vPO);

    // ---- PfromL (:354-374)
    int b1 = INF, b2 = INF;
    for (int s = 1; s < a; ++s) {
        b1 = imin(b1, L4(PfromL, s, a - s, 0, s) + W2(WP, i, i + s - 1));
        b2 = imin(b2, L4(PfromL, a - s, s, a - s, 0) + W2(WP, i + s + 1, j));
    }
    const int vPfromL = imin(imin(b1, b2), imin(imin(sPR, sPM), sPO) + PB);
    // ---- PfromR (:376-394)
    b1 = INF; b2 = INF;
    for (int s = 1; s < b; ++s) {
        b1 = imin(b1, L4(PfromR, s, a, s, 0) + W2(WP, k, k + s - 1));
        b2 = imin(b2, L4(PfromR, b - s, a, 0, 0) + W2(WP, k + s + 1, l));
    }
    const int vPfromR = imin(imin(b1, b2), imin(sPM, sPO) + PB);
    // ---- PfromM (:396-407)
    mv = INF;
    for (int s = 1; s < a; ++s) mv = imin(mv, L4(PfromMprime, a - s, s, a - s, 0) + W2(WP, i + s + 1, j));
    const int vPfromM = mv;
    // ---- PfromMprime (:409-420) with get_PfromMdoubleprime (:663-679); d < l so never the base case
    mv = INF;
    for (int s = 1; s < b; ++s)
        mv = imin(mv, imin(L4(PL, s, a, s, 0), L4(PR, s, a, s, 0)) + PB + W2(WP, k, k + s - 1));
    const int vPfromMp = mv;
    // ---- PfromO (:422-443)
    b1 = INF; b2 = INF;
    for (int s = 1; s < a; ++s) b1 = imin(b1, L4(PfromO, s, a - s, 0, s) + W2(WP, i, i + s - 1));
    for (int s = 1; s < b; ++s) b2 = imin(b2, L4(PfromO, b - s, a, 0, 0) + W2(WP, k + s + 1, l));
    const int vPfromO = imin(imin(b1, b2), imin(sPL, sPR) + PB);
    // ---- PK (:181-202)
    b1 = INF; b2 = INF;
    for (int s = 1; s < a; ++s) b1 = imin(b1, L4(PK, a - s, s, a - s, 0) + W2(WP, i + s + 1, j));
    for (int s = 1; s < b; ++s) b2 = imin(b2, L4(PK, s, a, s, 0) + W2(WP, k, k + s - 1));
    const int vPK = imin(imin(b1, b2), imin(imin(sPL, sPM), imin(sPR, sPO)) + PB);
#undef L4
#undef W2
#undef IE_CHECK

    // ---- stores: one coalesced int16 per matrix
    const LevelDesc &L = T.lv[t];
#ifdef CCJ_DEBUG_BOUNDS
    if (i < 1 || i > m - h || h >= m) { atomicOr(T.err, 32); return; }
#endif
    int16_t *dst = L.base + a * L.M + Gh + (i - 1);
    const int C = L.C;
    dst[PK * C] = (int16_t)clamp_store(vPK);
    dst[PL * C] = (int16_t)sPL;
    dst[PR * C] = (int16_t)sPR;
    dst[PM * C] = (int16_t)sPM;
    dst[PO * C] = (int16_t)sPO;
    dst[PfromL * C] = (int16_t)clamp_store(vPfromL);
    dst[PfromR * C] = (int16_t)clamp_store(vPfromR);
    dst[PfromM * C] = (int16_t)clamp_store(vPfromM);
    dst[PfromMprime * C] = (int16_t)clamp_store(vPfromMp);
    dst[PfromO * C] = (int16_t)clamp_store(vPfromO);
    dst[PLmloop00 * C] = (int16_t)clamp_store(vPLm00);
    dst[PLmloop01 * C] = (int16_t)clamp_store(vPLm01);
    dst[PLmloop10 * C] = (int16_t)clamp_store(vPLm10);
    dst[PRmloop00 * C] = (int16_t)clamp_store(vPRm00);
    dst[PRmloop01 * C] = (int16_t)clamp_store(vPRm01);
    dst[PRmloop10 * C] = (int16_t)clamp_store(vPRm10);
    dst[PMmloop00 * C] = (int16_t)clamp_store(vPMm00);
    dst[PMmloop01 * C] = (int16_t)clamp_store(vPMm01);
    dst[PMmloop10 * C] = (int16_t)clamp_store(vPMm10);
    dst[POmloop00 * C] = (int16_t)clamp_store(vPOm00);
    dst[POmloop01 * C] = (int16_t)clamp_store(vPOm01);
    dst[POmloop10 * C] = (int16_t)clamp_store(vPOm10);
}

// ------------------------------------------------------------------------------------------
extern "C" int ccjk_init2d(const DevTables *T, void *stream) {
    const int total = (T->n + 1) * T->rs;
    hipLaunchKernelGGL(k_init2d, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, *T, total);
    return (int)hipGetLastError();
}

extern "C" int ccjk_precompute_ie(const DevTables *T, void *stream) {
    const int n = T->n;
    dim3 grid((n + 255) / 256, n + 1, IE_U * IE_U);
    hipLaunchKernelGGL(k_precompute_ie, grid, dim3(256), 0, (hipStream_t)stream, *T);
    return (int)hipGetLastError();
}

extern "C" int ccjk_diag2d(const DevTables *T, int sigma, void *stream) {
    const int nb = T->n - sigma;
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(k_diag2d, dim3(nb), dim3(256), 0, (hipStream_t)stream, *T, sigma);
    return (int)hipGetLastError();
}

extern "C" int ccjk_level4d(const DevTables *T, int t, void *stream) {
    const int m = T->n - t - 2;
    if (m <= 0) return 0;
    const int Mt = m * (m + 1) / 2;
    const int wavesPerA = (Mt + 63) / 64;
    const long waves = (long)(t + 1) * wavesPerA;
    const long blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(k_level4d, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *T, t, wavesPerA);
    return (int)hipGetLastError();
}
