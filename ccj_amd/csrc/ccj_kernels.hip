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
#include <stdlib.h>
#include "ccj_engine.h"
#include "ccj_energy.h"
#include "ccj_items.h"

using namespace ccj;

#ifdef CCJ_WG_TIMELINE
// Measurement build only (tools/wg_timeline.py): around one armed level L, every wave of the fill's
// kernels stamps the 100 MHz constant clock at entry and exit, with a tag (a-block and roles for the
// level kernels) and its hardware slot (HW_ID: wave / SIMD / CU / SE bits; XCD by round robin), one
// 32-byte entry per wave, written by lane 0 through a plain vector store.  g_tl[kind][blockIdx *
// waves per block + wave in block]; kinds: 0 k_level4d(L), 1 k_level4d_lead(L), 2..4 k_iloop(L+1..L+3),
// 5..6 k_ppush(L-1..L), 7 k_diag2d(L-1..L) (sigma in the tag).
constexpr int TL_CAP = 1 << 15, TL_KINDS = 8;
__device__ int g_tl_level = -1;
__device__ ulonglong4 g_tl[TL_KINDS][TL_CAP];
struct TLStamp {
    int slot;
    unsigned long long t0;
    unsigned meta = 0xffffffffu;  // level-kernel grid-tail waves that return before their a-block is known
    // kind_of(L) -> the kind of this launch when level L is armed, or -1
    template <class K>
    __device__ __forceinline__ explicit TLStamp(K kind_of) {
        const int kind = kind_of(g_tl_level);
        const int wpb = (int)(blockDim.x >> 6);
        const int s = (int)blockIdx.x * wpb + (int)(threadIdx.x >> 6);
        slot = (g_tl_level >= 0 && kind >= 0 && s < TL_CAP && (threadIdx.x & 63) == 0) ? kind * TL_CAP + s : -1;
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ ~TLStamp() {
        if (slot < 0) return;
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, all 32 bits
        (&g_tl[0][0])[slot] = make_ulonglong4(t0, t1, meta, hw | (unsigned long long)(blockIdx.x % 8) << 32);
    }
};
#define TL_STAMP(expr_) TLStamp tl_stamp_([&](int L_) -> int { return (expr_); })
#define TL_META(v_) (tl_stamp_.meta = (unsigned)(v_))
#else
#define TL_STAMP(expr_)
#define TL_META(v_)
#endif

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
    const int mp = T.n - tp - 2;
    const int Mp = (mp * (mp + 1)) >> 1;
    const int off = mslot(x) * (tp + 1) * Mp + ap * Mp + hp * mp - ((hp * (hp - 1)) >> 1) + ip - 1;
    return (int)T.d4[T.lb[tp] + off];
}

#ifdef CCJ_DEBUG_BOUNDS
__device__ int *g_dbg_err;
#define IE_CHECK(u1_, u2_, w_, p_) \
    if ((u1_) < 0 || (u1_) >= IE_U || (u2_) < 0 || (u2_) >= IE_U || (w_) < 0 || (w_) > n || (p_) < 1 || (p_) + (w_) > n) atomicOr(T.err, 16)
#else
#define IE_CHECK(u1_, u2_, w_, p_)
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
#define W2E(A, p, q) ((int)(A)[((q) - (p)) * rs + (p)])

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
        T.Pk[x] = ~0ull;
        T.WB[x] = 0;
        T.WP[x] = 0;
        T.WBW[x] = make_int2(INF + 1, 0);
    }
}

// ------------------------------------------------------------------------------------------
// e_intP of one pseudoknot interior loop: lrint(e_intP * E_IntLoop(...)) for outer (p, p+w) and
// inner (p+u1+1, p+w-u2-1) (pseudo_loop.cc:822-826, 836-840).  The reference skips a candidate
// unless both pairs can pair (get_P?iloop's can_pair tests): 32767 then, and the matrix value it
// would be added to is the never-set 32767 of that pair, so the sum can never
// undercut a stored value (all stores clamp at 32767).  k_build_il evaluates it for every list
// entry (each candidate once per list), k_precompute_ie for u1 = u2 = 0 (k_level4d's stack-like
// interior loop, the plane T.ie).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int e_intP(const DevTables &T, int u1, int u2, int p, int q) {
    const int d = p + u1 + 1, dp = q - u2 - 1;
    if (dp - d < 1) return INTERN_INF;
    const int t1 = T.pair[T.S[p] * 8 + T.S[q]];
    const int t2 = T.pair[T.S[d] * 8 + T.S[dp]];
    if (t1 <= 0 || t2 <= 0) return INTERN_INF;  // the reference only visits candidates with can_pair() on both pairs
    const int e = E_IntLoop(T.prm, T.lx, u1, u2, t1, T.rtype[t2], T.S1[p + 1], T.S1[q - 1], T.S1[d - 1], T.S1[dp + 1]);
    const int v = (int)rint(T.e_intP * (double)e);
    if (v < -32768 || v >= INTERN_INF) atomicOr(T.err, 1);
    return v;
}

__global__ void k_precompute_ie(DevTables T) {
    const int n = T.n, rs = T.rs;
    const int w = blockIdx.y;  // outer span
    for (int p = 1 + blockIdx.x * blockDim.x + threadIdx.x; p + w <= n; p += gridDim.x * blockDim.x)
        T.ie[(size_t)w * rs + p] = (int16_t)e_intP(T, 0, 0, p, p + w);
}

// ------------------------------------------------------------------------------------------
// 2-D anti-diagonal sigma: one 256-thread workgroup per interval (i, l = i+sigma).
// ------------------------------------------------------------------------------------------
// Band-sharded fills partition each span: interval i belongs to rank (i-1) % G, and
// the level-sigma exchange carries the span's values to the other ranks (k_dtail_pack / _unpack).
__global__ __launch_bounds__(256) void k_diag2d(DevTables T, int sigma, int G, int rank) {
#ifdef CCJ_DEBUG_BOUNDS
    g_dbg_err = T.err;
#endif
    TL_STAMP(sigma == L_ - 1 || sigma == L_ ? 7 : -1);
    TL_META(sigma);
    __shared__ int red[4];
    __shared__ int sh_v, sh_p;
    const int n = T.n, rs = T.rs;
    const int i = (int)blockIdx.x * G + rank + 1;
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

    // ---- P(i,l) was reduced into T.Pk by k_ppush (ordered before this kernel by an event)
    if (tid == 0) {  // value half of the (value, first split) minimum; never set -> INF+1
        const unsigned long long pk = T.Pk[cell];
        sh_p = pk == ~0ull ? INF + 1 : (int)((unsigned)(pk >> 32) - 0x80000000u);
        T.P[cell] = sh_p;
    }
    __syncthreads();
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
            T.WBW[cell] = make_int2(wbp, T.WP[cell]);  // the pair the level loops load
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

// readlane of a 64-bit value (two 32-bit readlanes)
__device__ __forceinline__ unsigned long long rdl64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// ------------------------------------------------------------------------------------------
// P(i, i+sigma) = min over i<=j<d<k<l of PK(i,j,d+1,k) + PK(j+1,d,k+1,l)   (pseudo_loop.cc:166-179),
// pushed by level.  A term of P(i, i+sigma) reads A = PK(i,j,d+1,k) at level t1 = jo+(ko-do-1) and
// B = PK(j+1,d,k+1,l) at level t2 = (do-jo-1)+(sigma-ko-1), with t1 + t2 = sigma-3 (offsets
// jo = j-i, do = d-i, ko = k-i).  k_ppush(T), enqueued after level T, evaluates every term with
// max(t1, t2) = T: part A t1 = T (t2 <= T), part B t2 = T (t1 < T).  That completes P(T+3) (the
// last span whose terms all sit at levels <= T) and leaves partial minima of P(sigma > T+3) in T.Pk.  The gain: the level-T operand of a term is the same cell for
// PP_S consecutive spans, so a wave loads it once and pairs it with PP_S partners (1 + 1/PP_S loads
// per term instead of 2), and it is the level just written (L2 / MALL resident).
//   part A wave: (jo, 64 consecutive i, PP_S consecutive t2), loop h1 = do-jo-1 ascending:
//       A = level T, block jo, row h1, position i          (once per h1)
//       B = level t2, block h1, row T-jo, position i+jo+1  (per t2, valid while h1 <= t2)
//   part B wave: (a2 = do-jo-1, 64 consecutive l, PP_S consecutive t1), loop h2 = ko-do-1 descending:
//       B = level T, block a2, row h2, position l-h2-T-2            (once per h2)
//       A = level t1, block t1-h2, row a2, position l-T-3-t1 = i    (per t1, valid while h2 <= t1)
// Both loops visit the terms of one output in ascending (jo, do, ko) order, so a strict < keeps the
// reference's first minimum within a wave; across waves a 64-bit atomicMin on
// (P + 2^31) << 32 | (j-i, d-i, k-i) key keeps it: T.Pk starts all-ones ("never set"; every
// candidate is <= 65534 < INF/2, A-Q4), k_diag2d(sigma) takes P from it and the P_P traceback
// (pseudo_loop.cc:867-896) its first split, without a rescan.
// ------------------------------------------------------------------------------------------

// k_ppush's operands as buffer loads: a wave reads PK at level lev and at the PP_S consecutive levels
// o0 .. o0+ns-1, each set within 4 GB of its lowest level's start (ccj_create checks it; ~300 MB at
// n=200, above 2 GB from n ~ 470, hence unsigned offsets), so each is one buffer
// (base = that level's start) and an operand is (uniform byte offset, lane byte offset) = (soffset,
// voffset): no 64-bit address per load (as row pointers the compiler ran out of SGPRs and formed a
// 64-bit VGPR address for most of them)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pk_src(const DevTables &T, int t) {
    const unsigned long long v = (unsigned long long)(T.d4 + T.ld[t].lb);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((unsigned long long)hi << 32) | lo), (short)0, -1, 0x00020000);
}
// PK at (level t, block a, row h, position pos) read through the buffer of level tb <= t: soff =
// 2 * (the row's start relative to tb's start), voff = 2 * (pos - 1)
__device__ __forceinline__ int pk_buf(const DevTables &T, __amdgpu_buffer_rsrc_t src, int soff, int voff, int t, int a, int h,
                                      int pos) {
#ifdef CCJ_DEBUG_BOUNDS
    if (t < 0 || t >= T.nlev || a < 0 || a > t || h < 0 || h >= T.n - t - 2 || pos < 1 || pos > T.n - t - 2 - h) {
        atomicOr(T.err, 32);
        return 0;
    }
#endif
    (void)T; (void)t; (void)a; (void)h; (void)pos;
    return (int)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(src, voff, soff, 0);
}

// A wave's running minimum per span is one int: (value << 10) + code, code = the step's position in
// the reference order (h1 in part A, 1023 - h2 in part B; n <= 1023), so v_min keeps the first
// minimum.  Steps that are not terms of a span (h > its t) add PP_OFF and never win.
constexpr int PP_OFF = 1 << 30;

template <int PP_S, int PP_U>
__global__ __launch_bounds__(256) void k_ppush(DevTables T, int lev, int ngrp, int npairs, int hs_len, int blocksA, int G,
                                               int rank, int nout) {
    TL_STAMP(lev == L_ - 1 ? 5 : lev == L_ ? 6 : -1);
    TL_META(lev);
    const int n = T.n, rs = T.rs;
    const int lane = threadIdx.x & 63;
    const int partB = (int)blockIdx.x >= blocksA;
    // wave-uniform (readfirstlane: lets the compiler keep every index below in SGPRs)
    const int item = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - (partB ? blocksA : 0)) * 4 + (int)(threadIdx.x >> 6));
    // item = (pair * nout + own outer) * ngrp + g; outer = jo (part A) / a2 (part B), rank r of G
    // taking outer = r, r+G, ... (band sharding: every rank pushes its share of the terms into its
    // own T.Pk and the P spans are min-combined in the level exchange); pair = one
    // (chunk c of PP_S spans, slice hs = [hs*hs_len, +hs_len) of the inner loop h1 / h2), so long
    // loops spread over waves.  Chunk c's inner loop runs over h < min((c+1)*PP_S, nmax), so it has
    // ceil(that / hs_len) slices; the pairs are enumerated chunk by chunk (part A's count, nmax).
    // g (64 consecutive intervals) varies fastest, so the 4 waves of a workgroup read adjacent
    // segments of the same operand rows: the 128-byte lines a misaligned segment straddles are
    // shared inside one CU (and its XCD's L2) instead of fetched by two XCDs.
    const int g = item % ngrp;
    int pr = item / ngrp;
    const int outer = rank + G * (pr % nout);
    pr /= nout;
    if (pr >= npairs) return;  // whole wave
    const int nmax = imin(lev, n - 4 - lev) + 1;
    int c = 0;
    for (;; ++c) {  // scalar: at most nmax / PP_S steps
        const int cnt = (imin((c + 1) * PP_S, nmax) + hs_len - 1) / hs_len;
        if (pr < cnt) break;
        pr -= cnt;
    }
    const int hs = pr;
    const int nother = (partB ? imin(lev - 1, n - 4 - lev) : imin(lev, n - 4 - lev)) + 1;  // t2 (A) / t1 (B) count
    const int o0 = c * PP_S;
    if (o0 >= nother) return;
    const int ns = imin(PP_S, nother - o0);
    const int h_lo = hs * hs_len;
    const int hmax = imin(o0 + ns - 1, h_lo + hs_len - 1);
    if (h_lo > hmax) return;
    int bv[PP_S];
#pragma unroll
    for (int s = 0; s < PP_S; ++s) bv[s] = 0x7fffffff;
    const int mT = n - lev - 2;
    const LvlDev *__restrict__ LD = T.ld;
    const int Mlev = LD[lev].M;
    const long long lbo = LD[o0].lb;  // the other operand's buffer: levels o0 .. o0+ns-1
    const __amdgpu_buffer_rsrc_t srcT = pk_src(T, lev), srcO = pk_src(T, o0);
    auto Grow = [&](int m_, int h) { return h * m_ - ((h * (h - 1)) >> 1); };
    if (!partB) {
        const int jo = outer, b1 = lev - jo;
        const int i = 1 + g * 64 + lane;
        if (1 + g * 64 > n - (lev + 3 + o0)) return;  // no lane has an interval of the shortest span
        const int sA0 = 2 * (jo * Mlev);  // + 2 G(h) per step
        // B of span s: the row's start relative to level o0 plus the lane's position (voffset, fixed
        // per lane) and the block h1 (soffset h1 * 2M, per step)
        int voB[PP_S], Ms2[PP_S];
#pragma unroll
        for (int s = 0; s < PP_S; ++s) {
            const int t2 = imin(o0 + s, o0 + ns - 1);
            Ms2[s] = __builtin_amdgcn_readfirstlane(2 * LD[t2].M);  // uniform: a per-lane soffset would be a waterfall loop
            // unsigned: below 4 GB by ccj_create's k_ppush span check, possibly above 2 GB (n >~ 470)
            voB[s] = (int)((unsigned)(2 * (LD[t2].lb - lbo + Grow(n - t2 - 2, b1))) + 2u * (unsigned)(imin(i, n - (lev + 3 + t2)) + jo));
        }
        // PP_U steps per iteration, all PP_U * (PP_S + 1) loads in flight together (the steps of a
        // short tail re-read the last one and are masked)
        for (int h1 = h_lo; h1 <= hmax; h1 += PP_U) {
            int va[PP_U], vb[PP_U][PP_S], hh[PP_U];
#pragma unroll
            for (int u = 0; u < PP_U; ++u) hh[u] = imin(h1 + u, hmax);
#pragma unroll
            for (int u = 0; u < PP_U; ++u) {
                const int h = hh[u];
                va[u] = pk_buf(T, srcT, sA0 + 2 * Grow(mT, h), 2 * (imin(i, mT - h) - 1), lev, jo, h, imin(i, mT - h));
                // every load unconditional (steps with h1 > t2 read a clamped valid cell and are
                // masked)
#pragma unroll
                for (int s = 0; s < PP_S; ++s) {
                    const int t2 = imin(o0 + s, o0 + ns - 1), hc = imin(h, t2);
                    vb[u][s] = pk_buf(T, srcO, hc * Ms2[s], voB[s], t2, hc, b1, imin(i, n - (lev + 3 + t2)) + jo + 1);
                }
            }
#pragma unroll
            for (int u = 0; u < PP_U; ++u) {
                const bool live = h1 + u <= hmax;
#pragma unroll
                for (int s = 0; s < PP_S; ++s) {
                    const int code = (live && s < ns && hh[u] <= o0 + s) ? hh[u] : PP_OFF;
                    bv[s] = imin(bv[s], ((va[u] + vb[u][s]) << 10) + code);
                }
            }
        }
#pragma unroll
        for (int s = 0; s < PP_S; ++s) {
            const int sg = lev + 3 + o0 + s;
            if (s < ns && i + sg <= n && bv[s] < (PP_OFF >> 1)) {
                const unsigned dd = (unsigned)(jo + 1 + (bv[s] & 1023)), ko = dd + 1u + (unsigned)b1;
                const unsigned key = ((unsigned)jo * (unsigned)sg + dd) * (unsigned)sg + ko;
                atomicMin(T.Pk + sg * rs + i, ((unsigned long long)((unsigned)(bv[s] >> 10) + 0x80000000u) << 32) | key);
            }
        }
    } else {
        const int a2 = outer;
        const int l = lev + 4 + o0 + g * 64 + lane;
        if (lev + 4 + o0 + g * 64 > n) return;
        const int lc = imin(l, n);
        const int sB0 = 2 * (a2 * Mlev);  // + 2 G(h) per step
        // A of span s: row start relative to level o0 plus the lane's position (voffset), block
        // t1-h2 (soffset (t1-h2) * 2M, per step)
        int voA[PP_S], Ms2[PP_S];
#pragma unroll
        for (int s = 0; s < PP_S; ++s) {
            const int t1 = imin(o0 + s, o0 + ns - 1);
            Ms2[s] = __builtin_amdgcn_readfirstlane(2 * LD[t1].M);
            voA[s] = (int)((unsigned)(2 * (LD[t1].lb - lbo + Grow(n - t1 - 2, a2))) + 2u * (unsigned)(imax(1, lc - (lev + 3 + t1)) - 1));
        }
        for (int h2 = hmax; h2 >= h_lo; h2 -= PP_U) {  // PP_U steps per iteration, as in part A
            int vb[PP_U], va[PP_U][PP_S], hh[PP_U];
#pragma unroll
            for (int u = 0; u < PP_U; ++u) hh[u] = imax(h2 - u, h_lo);
#pragma unroll
            for (int u = 0; u < PP_U; ++u) {
                const int h = hh[u];
                const int pb = imax(1, imin(lc - h - lev - 2, mT - h));
                vb[u] = pk_buf(T, srcT, sB0 + 2 * Grow(mT, h), 2 * (pb - 1), lev, a2, h, pb);
#pragma unroll
                for (int s = 0; s < PP_S; ++s) {  // unconditional loads, clamped and masked as in part A
                    const int t1 = imin(o0 + s, o0 + ns - 1), hc = imin(h, t1);
                    va[u][s] = pk_buf(T, srcO, (t1 - hc) * Ms2[s], voA[s], t1, t1 - hc, a2, imax(1, lc - (lev + 3 + t1)));
                }
            }
#pragma unroll
            for (int u = 0; u < PP_U; ++u) {
                const bool live = h2 - u >= h_lo;
#pragma unroll
                for (int s = 0; s < PP_S; ++s) {
                    const int code = (live && s < ns && hh[u] <= o0 + s) ? 1023 - hh[u] : PP_OFF;
                    bv[s] = imin(bv[s], ((va[u][s] + vb[u]) << 10) + code);
                }
            }
        }
#pragma unroll
        for (int s = 0; s < PP_S; ++s) {
            const int sg = lev + 3 + o0 + s;
            const int i = l - sg;
            if (s < ns && l <= n && i >= 1 && bv[s] < (PP_OFF >> 1)) {
                const unsigned h2 = 1023u - (unsigned)(bv[s] & 1023);
                const unsigned jo = (unsigned)(o0 + s) - h2, dd = jo + 1u + (unsigned)a2, ko = dd + 1u + h2;
                const unsigned key = (jo * (unsigned)sg + dd) * (unsigned)sg + ko;
                atomicMin(T.Pk + sg * rs + i, ((unsigned long long)((unsigned)(bv[s] >> 10) + 0x80000000u) << 32) | key);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Interior-loop candidate lists (once per problem, after k_precompute_ie).
// For pair (p, q = p+w):
//   il  — loops closed by (p,q) around an inner pair (d,dp) = (p+1+u1, q-1-u2), the window of
//         get_PLiloop / get_PRiloop (pseudo_loop.cc:694-700, 729-735): u1 <= min(w,30)-2,
//         u2 <= min(w-u1-6, 28);
//   ilm — loops closed by an outer pair (d,dp) = (p-1-u1, q+1+u2) around (p,q), the window of
//         get_PMiloop (pseudo_loop.cc:762-768) without its cell-dependent bounds (u1 <= a-2,
//         u2 <= b-2 are checked per lane by k_iloop).
// Only candidates whose other pair can pair are kept (the reference skips the rest: can_pair),
// in order of dt = 2+u1+u2 (the source level distance), u1 ascending; seg[dt] is the first entry
// of dt.  One wave per pair: the window's validity and energies are gathered at once (lane = u1)
// into LDS, then compacted per dt (lane = u1, ballot).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_build_il(DevTables T) {
    __shared__ int16_t es[IE_U][IE_U + 1];  // [u1][u2]: the window's energies
    __shared__ uint32_t vb[IE_U];            // [u1]: bit u2 = the candidate is kept
    const int n = T.n, rs = T.rs;
    const int p = blockIdx.x + 1, w = blockIdx.y, kind = blockIdx.z;
    const int q = p + w;
    if (q > n) return;
    // k_iloop reads only the lists of pairs that can pair (its items exist only for those)
    if (T.pt[(size_t)w * rs + p] <= 0) return;
    const int lane = threadIdx.x;
    const size_t pidx = (size_t)w * rs + p;
    uint32_t *seg = (kind ? T.ilmseg : T.ilseg) + pidx * IL_SEG;
    uint2 *ent = (kind ? T.ilm : T.il) + pidx * IL_CAP;
    // the whole window at once (lane = u1, every u2): one memory round trip for its loads
    if (lane < IE_U) {
        const int u1 = lane;
        uint32_t bits = 0;
#pragma unroll
        for (int u2 = 0; u2 < IE_U; ++u2) {
            bool valid = false;
            int e = 0;
            if (kind == 0) {
                const int d = p + 1 + u1, dp = q - 1 - u2;
                if (u1 <= imin(w, MAXLOOP) - 2 && u2 <= imin(w - u1 - 6, MAXLOOP - 2) && T.pt[(dp - d) * rs + d] > 0) {
                    valid = true;
                    e = e_intP(T, u1, u2, p, q);
                }
            } else {
                const int d = p - 1 - u1, dp = q + 1 + u2;
                if (d >= 1 && dp <= n && T.pt[(dp - d) * rs + d] > 0) {
                    valid = true;
                    e = e_intP(T, u1, u2, d, dp);
                }
            }
            es[u1][u2] = (int16_t)e;
            bits |= (valid ? 1u : 0u) << u2;
        }
        vb[u1] = bits;
    }
    __syncthreads();
    int cnt = 0;
    for (int dt = 0; dt < IL_SEG; ++dt) {
        if (lane == 0) seg[dt] = (uint32_t)cnt;
        const int u1 = lane, u2 = dt - 2 - lane;
        const bool valid = dt >= 2 && u1 < IE_U && u2 >= 0 && u2 < IE_U && ((vb[u1] >> u2) & 1u);
        const unsigned long long mask = __ballot(valid);
        if (valid)
            ent[cnt + __popcll(mask & ((1ull << lane) - 1))] =
                make_uint2(((uint32_t)dt << 21) | ((uint32_t)u1 << 16) | (uint32_t)(uint16_t)es[u1][u2], (uint32_t)(2 * u1 * dt));
        cnt += __popcll(mask);
    }
    // null tail: dt 63 addresses the sentinel pad (32767), energy 32767 -> 65534, never below a clamped result
    if (lane < IL_B) ent[cnt + lane] = make_uint2((63u << 21) | (uint32_t)INTERN_INF, 0u);
}

// ------------------------------------------------------------------------------------------
// k_iloop work items, built on the GPU once per sequence (ccj_create / ccj_reset).  One wave of
// k_iloop per item; an item is a closing pair that can pair plus a 64-lane chunk of the cells that
// share it (role << 30 | f1 << 20 | f2 << 10 | chunk):
//   PL (role 0): for own a in [6, t], i in [1, m]:   pair (i, i+a),  chunks over h <= m-i
//   PR (role 1): for own a in [0, t-6], q < m:        pair (k, k+t-a), k = q+a+3, chunks over i <= q+1
//   PM (role 2): for h in [2, m-1], j in [1, n]:      pair (j, k = j+h+2), chunks over the own a in [alo, ahi]
// ("own": the rank's a-blocks, ccj_engine.h shard_a; every a when unsharded)
// in this enumeration order (measured no slower than heaviest-list-first).  KI_SPLIT workgroups per
// (level t, shard r) each walk one run of its "rows" (one closing pair each) 256 at a time; pass 0
// counts the items of each run, pass 1 writes them at offs[(t*G+r)*KI_SPLIT+s] + an exclusive scan
// of the row counts.
// ------------------------------------------------------------------------------------------
// the row enumeration (ItemRows, item_row) is shared with the host's count pass: ccj_items.h
struct DevPT {
    const DevTables *T;
    __device__ int operator()(int i, int j) const { return ptype(*T, i, j); }
};

__global__ __launch_bounds__(256) void k_items(DevTables T, int G, int rank, int simulate,
                                               long long *counts, const long long *__restrict__ offs, uint32_t *items,
                                               int pass) {
    __shared__ int wsum[4];
    __shared__ long long tot;
    // workgroup = (level t, shard r, split s): rows [lo, hi) of the level (ccj_items.h ki_split_rows)
    const int bs = blockIdx.x, b = bs / KI_SPLIT, sp = bs - b * KI_SPLIT, t = b / G, r = b - t * G;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool mine = simulate || r == rank;
    if (!mine || t < 4 || t >= T.nlev) {
        if (pass == 0 && tid == 0) counts[bs] = 0;
        return;  // whole workgroup
    }
    const ItemRows R = item_rows(T.n, t, G, r);
    const DevPT pt{&T};
    int lo, hi;
    ki_split_rows(R.nPL + R.nPR + R.nPM, sp, lo, hi);
    long long base = pass ? offs[bs] : 0;
    for (int c0 = lo; c0 < hi; c0 += 256) {
        const int x = c0 + tid;
        uint32_t it0 = 0;
        const int cnt = x < hi ? item_row(pt, T.n, t, R, x, G, r, it0, IL_CW) : 0;
        // exclusive scan of cnt over the workgroup: wave scan, then the wave totals
        int inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        int before = 0;
        for (int v = 0; v < w; ++v) before += wsum[v];
        const int chunk_total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (pass) {
            const long long pos = base + before + inc - cnt;
            for (int c = 0; c < cnt; ++c) items[pos + c] = it0 | (uint32_t)c;
        }
        base += chunk_total;
        __syncthreads();  // wsum is rewritten by the next chunk
    }
    if (pass == 0 && tid == 0) {
        tot = base;
        counts[bs] = tot;
    }
}

extern "C" int ccjk_items(const DevTables *T, int G, int rank, int simulate, long long *counts, const long long *offs,
                          uint32_t *items, int pass, void *stream) {
    const int blocks = T->n * G * KI_SPLIT;
    if (blocks <= 0) return 0;
    hipLaunchKernelGGL(k_items, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *T, G, rank, simulate, counts,
                       offs, items, pass);
    return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Interior loops of level t (get_PLiloop / get_PRiloop / get_PMiloop, pseudo_loop.cc:682-773).
// One wave per closing pair and run of cells sharing it, so the pair test, the candidate list and
// the loop energies are wave-uniform (scalar loads) and only candidates whose inner pair can pair
// are visited; the partner value comes from the PLx/PRx/PMx copy, contiguous along the lanes.
//   PL: wave = (a, i, h-chunk), lanes h  — closing pair (i, j)
//   PR: wave = (a, q, i-chunk), lanes i  — closing pair (k, l), q = i+h-1 = k-a-3
//   PM: wave = (h, j, a-chunk), lanes a  — pair (j, k), per-lane window u1 <= a-2, u2 <= b-2
// The minimum (clamped like a store) goes into the cell's PL/PR/PM slot of level t, where
// k_level4d(t) picks it up.  The candidate with no unpaired base (u1 = u2 = 0, source level t-2)
// reads the same inner cell as the stack term, so k_level4d(t) evaluates it there; k_iloop(t)
// walks the lists from dt = 3 on and needs levels <= t-3 only, a whole level of slack.
// ------------------------------------------------------------------------------------------
// Each list entry's partner address is A[dt] + B[u1] (+ 2*u1*dt for PL/PM) bytes + the lane's
// offset: A (64-bit, per source level) and B (per u1) are per-wave tables held one value per lane
// and fetched with readlane, so an entry costs a few scalar ops and one load on a uniform base.
// IL_B entries are loaded together (one s_load burst), then IL_B partner values, then reduced.
// Null tail entries (dt 63) hit the sentinel pad, so the last batch needs no masking (PL/PR: cnt is the
// whole list; PM stops early and substitutes null entries).
// Loads at wave-uniform addresses of data no kernel of the fill writes (candidate lists, segment
// tables): through the constant address space, so they are scalar (SMEM) loads.  As plain global
// loads the compiler cannot prove them unclobbered (the kernel stores to T.d4), emits vector loads
// plus readfirstlane, and a wave waiting for its next list entries then waits for every partner
// load before them too (vmcnt counts in order): one memory latency per batch instead of one per
// two batches.
__device__ __forceinline__ uint32_t ld_const(const uint32_t *p) {
    return *(const __attribute__((address_space(4))) uint32_t *)(unsigned long long)p;  // inttoptr: no flat cast
}
__device__ __forceinline__ uint2 ld_const(const uint2 *p) {
    const unsigned long long v = *(const __attribute__((address_space(4))) unsigned long long *)(unsigned long long)p;
    return make_uint2((unsigned)v, (unsigned)(v >> 32));
}
__device__ __forceinline__ const uint2 *uni_ptr(const uint2 *p) {
    const unsigned long long v = (unsigned long long)p;
    return (const uint2 *)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v)) |
                           ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32)) << 32));
}
__device__ __forceinline__ int il_u1(uint32_t x) { return (int)((x >> 16) & 31u); }
__device__ __forceinline__ int il_dt(uint32_t x) { return (int)(x >> 21); }
__device__ __forceinline__ int il_e(uint32_t x) { return (int)(int16_t)(x & 0xffffu); }

// min over the wave's candidate list of energy + partner value (PL/PR/PM interior loops).
// Software-pipelined one batch deep: the entries and partner loads of batch k+1 are issued before
// batch k is reduced, so a wave keeps 2*IL_B partner loads in flight.  PAIR: the wave holds two
// 64-cell chunks of its row (lane offsets lofs2 and lofs2b) and loads both partners of every
// entry, so a list entry's decode and address cost is paid once per 128 cells; half as many
// entries per batch keep the loads in flight (and the registers) at 2*IL_B.
template <bool CROSS, bool PMWIN, bool PAIR>
__device__ __forceinline__ int2 il_scan(const DevTables &T, const uint2 *__restrict__ ent, int cnt,
                                        __amdgpu_buffer_rsrc_t src, int Atab, int Btab, unsigned lofs2, int as, int bs,
                                        unsigned lofs2b, int asb, int bsb) {
    constexpr int NB = PAIR ? IL_B / 2 : IL_B;
    int b1 = INF, b2 = INF;
    cnt = __builtin_amdgcn_readfirstlane(cnt);
    if (cnt <= 0) return make_int2(b1, b2);
    ent = uni_ptr(ent);
    // a batch of NB entries (8 or 16 bytes x NB) as ONE scalar load: s_load_dwordx16 / x8 (as NB
    // separate dwordx2 loads the compiler computed a 64-bit address per entry)
    typedef unsigned ent_vec __attribute__((ext_vector_type(2 * NB)));
    auto fetch = [&](int e0, uint2 *E) {
        const ent_vec v = *(const __attribute__((address_space(4))) ent_vec *)(unsigned long long)(ent + e0);
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            E[u] = make_uint2(v[2 * u], v[2 * u + 1]);
            // PM stops at dt <= t-2, before the list's null tail: past cnt, substitute a null entry
            if (PMWIN && e0 + u >= cnt) E[u] = make_uint2((63u << 21) | (uint32_t)INTERN_INF, 0u);
        }
    };
    auto issue = [&](const uint2 *E, int *v, int *w) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int dt = il_dt(E[u].x), u1 = il_u1(E[u].x);
            // the partner's byte offset from the wave's buffer base: A[dt] + B[u1] (+ 2 u1 dt), all
            // 32-bit and wave-uniform, so it is the load's soffset and the lane's offset its voffset
            // (a 64-bit address per candidate cost a 64-bit VALU add and a third readlane)
            unsigned off = (unsigned)__builtin_amdgcn_readlane(Btab, u1) + (unsigned)__builtin_amdgcn_readlane(Atab, dt);
            if (CROSS) off += E[u].y;
#ifdef CCJ_DEBUG_BOUNDS
            {   // the partner must lie inside its copy (the null target is the pad in front of a level)
                bool bad = false;
                for (int c = 0; c < (PAIR ? 2 : 1); ++c) {
                    const unsigned o = off + (c ? lofs2b : lofs2);
                    bad = bad || o >= (unsigned)T.xspan;
                }
                if (bad || (dt != 63 && (dt < 2 || dt > 2 * MAXLOOP - 2))) {
                    if (atomicOr(T.err, 64) == 0)
                        printf("k_iloop OOB: dt %d u1 %d off %u lofs2 %u lofs2b %u pair %d\n", dt, u1, off, lofs2, lofs2b,
                               (int)PAIR);
                    v[u] = w[u] = 0;
                    continue;
                }
            }
#endif
#ifdef CCJ_ABLATE_ILHOT
            // timing only: every partner read hits the same cache-resident line (wrong results)
            off &= 0u;
#endif
            v[u] = (int)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(src, (int)lofs2, (int)off, 0);
            if (PAIR) w[u] = (int)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(src, (int)lofs2b, (int)off, 0);
        }
    };
    auto reduce = [&](const uint2 *E, const int *v, const int *w) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int e = il_e(E[u].x), c = e + v[u];
            if (PMWIN) {
                const int u1 = il_u1(E[u].x), u2 = il_dt(E[u].x) - 2 - u1;
                // get_PMiloop: d > i, dp < l.  Branch-free (a select of constants): a branch here
                // splits the loop body, and the compiler then sign-extends the next batch's loads
                // in the latch, draining every load before the back-edge
                b1 = imin(b1, c + (((u1 > as - 2) | (u2 > bs - 2)) ? INF : 0));
                if (PAIR) b2 = imin(b2, e + w[u] + (((u1 > asb - 2) | (u2 > bsb - 2)) ? INF : 0));
            } else {
                b1 = imin(b1, c);
                if (PAIR) b2 = imin(b2, e + w[u]);
            }
        }
    };
    // Ping-pong buffers, two batches per trip: a batch's registers are written only after the
    // batch they replace was reduced, so the loop carries no register copies.  (With one buffer
    // and a copy per trip, the copy of a just-issued load made the compiler wait for every load
    // before the back-edge: one full memory latency per batch instead of overlapped batches.)
    uint2 Ea[NB], Eb[NB];
    int va[NB], vb[NB], wa[NB], wb[NB];
    fetch(0, Ea);
    issue(Ea, va, wa);
    int e0 = NB;
#pragma unroll 1
    while (true) {
        if (e0 >= cnt) {
            reduce(Ea, va, wa);
            break;
        }
        fetch(e0, Eb);
        issue(Eb, vb, wb);
        reduce(Ea, va, wa);
        e0 += NB;
        if (e0 >= cnt) {
            reduce(Eb, vb, wb);
            break;
        }
        fetch(e0, Ea);
        issue(Ea, va, wa);
        reduce(Eb, vb, wb);
        e0 += NB;
    }
    return make_int2(b1, b2);
}

// The same minimum for a wave whose row has at most 32 cells: the wave is G groups of W lanes
// (il_groups), each group holding the whole row and walking every G-th list entry (entry
// e0+g+G*u), so the list takes 1/G of the iterations; the groups are min-reduced at the end
// (lanes rl, rl+W, ..., rl+(G-1)W; rl unused with power-of-two W).  The
// entry is per lane here, so the A/B tables are read with ds_bpermute instead of readlane.  All 64
// lanes run the scan (bpermute sources must be live).
__device__ __forceinline__ int bperm(int v, int l) { return __builtin_amdgcn_ds_bpermute(l << 2, v); }

#ifndef CCJ_ILG_B
#define CCJ_ILG_B 4
#endif
constexpr int ILG_B = CCJ_ILG_B;  // entries per lane per batch in the grouped walk (registers: 8 waves/SIMD)
template <bool CROSS, bool PMWIN>
__device__ __forceinline__ int il_scan_g(const DevTables &T, const uint2 *__restrict__ ent, int cnt, __amdgpu_buffer_rsrc_t src,
                                         int Atab, int Btab, unsigned lofs2, int as, int bs, int G, int W, int g, int rl) {
    int b1 = INF;
    if (cnt <= 0) return b1;
    // only the packed word is loaded (the cross term 2*u1*dt is recomputed): half the registers
    const uint32_t nul = (63u << 21) | (uint32_t)INTERN_INF;
    auto fetch = [&](int e0, uint32_t *E) {
#pragma unroll
        for (int u = 0; u < ILG_B; ++u) {
            const int e = e0 + g + G * u;
            E[u] = ent[imin(e, cnt - 1)].x;
            if (e >= cnt) E[u] = nul;
        }
    };
    auto issue = [&](const uint32_t *E, int *v) {
#pragma unroll
        for (int u = 0; u < ILG_B; ++u) {
            const int dt = il_dt(E[u]), u1 = il_u1(E[u]);
            // per-lane entries: the offset from the wave's buffer base is per lane (voffset)
            unsigned off = (unsigned)bperm(Btab, u1) + (unsigned)bperm(Atab, dt) + lofs2;
            if (CROSS) off += (unsigned)(2 * u1 * dt);
#ifdef CCJ_DEBUG_BOUNDS
            if (off >= (unsigned)T.xspan || (dt != 63 && (dt < 2 || dt > 2 * MAXLOOP - 2))) {
                if (atomicOr(T.err, 64) == 0) printf("k_iloop (grouped, G %d) OOB: dt %d u1 %d\n", G, dt, u1);
                v[u] = 0;
                continue;
            }
#endif
#ifdef CCJ_ABLATE_ILHOT
            off = lofs2;  // timing only: every partner read on the lane's own line of the pad
#endif
            v[u] = (int)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(src, (int)off, 0, 0);
        }
    };
    auto reduce = [&](const uint32_t *E, const int *v) {
#pragma unroll
        for (int u = 0; u < ILG_B; ++u) {
            const int c = il_e(E[u]) + v[u];
            if (PMWIN) {
                const int u1 = il_u1(E[u]), u2 = il_dt(E[u]) - 2 - u1;
                b1 = imin(b1, c + (((u1 > as - 2) | (u2 > bs - 2)) ? INF : 0));
            } else {
                b1 = imin(b1, c);
            }
        }
    };
    // Ping-pong as in il_scan, with the (per-lane, vector-memory) entries loaded one batch ahead:
    // loads return in order, so waiting for batch k+1's entries also waits for batch k's partners;
    // issuing k+1's partners together with k+2's entries keeps two loads per lane in flight
    // across each wait instead of one.
    uint32_t Ea[ILG_B], Eb[ILG_B];
    int va[ILG_B], vb[ILG_B];
    const int stepE = G * ILG_B;
    fetch(0, Ea);
    issue(Ea, va);
    fetch(stepE, Eb);
    int e0 = stepE;
#pragma unroll 1
    while (true) {
        if (e0 >= cnt) {
            reduce(Ea, va);
            break;
        }
        issue(Eb, vb);
        reduce(Ea, va);
        fetch(e0 + stepE, Ea);
        e0 += stepE;
        if (e0 >= cnt) {
            reduce(Eb, vb);
            break;
        }
        issue(Ea, va);
        reduce(Eb, vb);
        fetch(e0 + stepE, Eb);
        e0 += stepE;
    }
    for (int off = W; off < 64; off <<= 1) b1 = imin(b1, __shfl_xor(b1, off));
    return b1;
}

// Lane groups for a row of nact cells: W lanes per group (one per cell, W >= nact, a power of two
// >= 8), G = 64/W groups; lane = gq*W + rl.  Rows above 32 cells keep one group (the scalar list
// walk).  (Groups of exactly nact lanes, W not a power of two, measured the same.)
struct ILGroups { int G, W, gq, rl; };
__device__ __forceinline__ ILGroups il_groups(int nact, int lane) {
    const int W = nact > 32 ? 64 : nact > 16 ? 32 : nact > 8 ? 16 : 8;
    return {64 / W, W, lane / W, lane & (W - 1)};
}

// The partner buffer of one k_iloop wave: every copy row its candidates read lies in the source
// levels t-58 .. t-3, at most a few GB past the sentinel pad (T.xpad elements of 32767) in front of
// the lowest one, so the wave addresses them as 32-bit byte offsets from that pad (buffer loads:
// soffset = the candidate's uniform offset, voffset = the lane's).  A null list entry (dt 63, the
// lane-63 A entry) lands in the pad: 32767, never below a clamped result.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t il_src(const int16_t *base) {
    const unsigned long long v = (unsigned long long)base;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((unsigned long long)hi << 32) | lo), (short)0, -1, 0x00020000);
}

#ifdef CCJ_ABLATE_ILHALF
#define ILHALF(x) ((x) >> 1)  // timing only: every list walked half way (wrong results; the marginal cost of k_iloop's work)
#else
#define ILHALF(x) (x)
#endif
// one wave per work item: a closing pair that can pair and up to IL_CW (two 64-lane chunks) of
// its cells (ccj_items.h, built by k_items in enumeration order)
constexpr int IL_WPB = 4;  // waves (consecutive items) per k_iloop workgroup (1, 2, 8, 16 measured +3.6 ... +9 ms)
__global__ __launch_bounds__(64 * IL_WPB) void k_iloop(DevTables T, int t, long long first, int nitems, int G_SH, int rank) {
    TL_STAMP(t >= L_ + 1 && t <= L_ + 3 ? 2 + t - L_ - 1 : -1);
    TL_META(t);
    const int n = T.n, rs = T.rs, m = n - t - 2;
    const int lane = threadIdx.x & 63;
    const int w = (int)blockIdx.x * IL_WPB + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= nitems) return;
    const uint32_t it = T.items[first + w];
    const int role = (int)(it >> 30), f1 = (int)((it >> 20) & 1023u), f2 = (int)((it >> 10) & 1023u);
    const int zc = (int)(it & 1023u);
    const LvlDev Lt = T.ld[t];
    const int tl = t - lane;  // A-table lane L describes source level t-L (dt = L)
    const bool lvl_ok = lane >= 2 && lane <= 2 * MAXLOOP - 2 && tl >= 0;
    const long long BIAS = (long long)(n + 64) * (n + 64);  // keeps B >= 0
    // the wave's buffer base: the sentinel pad in front of the lowest source level's copies
    const int tlo = imax(0, t - (2 * MAXLOOP - 2));
    const long long xb = T.ldx[tlo].lbx - T.xpad, pb = T.ldx[tlo].pmb - T.xpad;  // elements
    const __amdgpu_buffer_rsrc_t src = il_src(role == 2 ? T.pmx + pb : T.d4x + xb);
    if (role == 0) {
        // PL: wave = (a, i, h-chunk), lanes h; closing pair (i, j)
        const int a = f1, i = f2, len = m - i + 1, h0 = zc * IL_CW;
        const ILGroups lg = il_groups(imin(64, len - h0), lane);
        const int G = lg.G, gq = lg.gq;
        const bool pair = len - h0 > 64;  // a second 64-cell chunk (wave-uniform)
        const int h = h0 + lg.rl, hb = h + 64;
        const bool act = h <= m - i, actb = pair && hb <= m - i;
        const unsigned lofs2 = 2u * (unsigned)(act ? h : m - i);  // idle lanes re-read a valid cell
        const unsigned lofs2b = 2u * (unsigned)(actb ? hb : m - i);
        const size_t pidx = (size_t)a * rs + i;
        // PLx(t-dt, a-dt, h+dt-1-u1, i+1+u1) = lbx + (a-dt)M + x(m+dt) - x(x-1)/2 + dt-1-u1 + h, x = i+u1
        //   = [lbx + (a-dt)M + i*m + i*dt + dt-1] + [u1*m - x(x-1)/2 - u1] + u1*dt
        const int x = i + lane;
        const int Btab = (int)(2 * ((long long)lane * m - ((long long)x * (x - 1) >> 1) - lane + BIAS));
        int Atab = 0;
        if (lvl_ok && a >= lane)
            Atab = (int)(unsigned)(2 * (T.ldx[tl].lbx - xb + (long long)(a - lane) * T.ld[tl].M + (long long)i * m +
                                        (long long)i * lane + lane - 1 - BIAS));
        const int B0 = __builtin_amdgcn_readlane(Btab, 0);
        if (lane == 63) Atab = -B0;
        const int e0 = (int)ld_const(T.ilseg + pidx * IL_SEG + 3);
        const uint2 *le = T.il + pidx * IL_CAP + e0;
        const int lc = ILHALF((int)ld_const(T.ilseg + pidx * IL_SEG + IL_SEG - 1) - e0);
        const int2 bm = G > 1  ? make_int2(il_scan_g<true, false>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, G, lg.W, gq, lg.rl), INF)
                        : pair ? il_scan<true, false, true>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, lofs2b, 0, 0)
                               : il_scan<true, false, false>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, 0u, 0, 0);
#ifdef CCJ_DEBUG_BOUNDS
        if ((act && (a < 0 || a > t || h < 0 || h >= m || i < 1 || i > m - h)) || (actb && hb >= m)) {
            atomicOr(T.err, 128);
            return;
        }
#endif
        int16_t *dl = T.d4 + Lt.lb + (long long)mslot(PL) * Lt.C + a * Lt.M + i - 1;
        if (act && gq == 0) dl[h * m - ((h * (h - 1)) >> 1)] = (int16_t)clamp_store(bm.x);
        if (actb) dl[hb * m - ((hb * (hb - 1)) >> 1)] = (int16_t)clamp_store(bm.y);
    } else if (role == 1) {
        // PR: wave = (a, q, i-chunk), lanes i; closing pair (k, l), q = i+h-1 = k-a-3
        const int a = f1, q = f2;
        const int b = t - a;
        const int k = q + a + 3;
        const int i0 = zc * IL_CW;
        const ILGroups lg = il_groups(imin(64, q + 1 - i0), lane);
        const int G = lg.G, gq = lg.gq;
        const bool pair = q + 1 - i0 > 64;
        const int i = i0 + lg.rl + 1, ib = i + 64;
        const bool act = i <= q + 1, actb = pair && ib <= q + 1;
        const unsigned lofs2 = 2u * (unsigned)((act ? i : q + 1) - 1);
        const unsigned lofs2b = 2u * (unsigned)((actb ? ib : q + 1) - 1);
        const int h = q + 1 - i, hb = q + 1 - ib;
        const size_t pidx = (size_t)b * rs + k;
        // PRx(t-dt, a, h+1+u1, i) = lbx + C + a*M + qq(qq+1)/2 + i-1, qq = q+1+u1
        const int qq = q + 1 + lane;
        const int Btab = qq * (qq + 1);  // bytes
        int Atab = 0;
        if (lvl_ok) Atab = (int)(unsigned)(2 * (T.ldx[tl].lbx - xb + T.ld[tl].C + (long long)a * T.ld[tl].M));
        const int B0 = __builtin_amdgcn_readlane(Btab, 0);
        if (lane == 63) Atab = -B0;
        const int e0 = (int)ld_const(T.ilseg + pidx * IL_SEG + 3);
        const uint2 *le = T.il + pidx * IL_CAP + e0;
        const int lc = ILHALF((int)ld_const(T.ilseg + pidx * IL_SEG + IL_SEG - 1) - e0);
        const int2 bm = G > 1  ? make_int2(il_scan_g<false, false>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, G, lg.W, gq, lg.rl), INF)
                        : pair ? il_scan<false, false, true>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, lofs2b, 0, 0)
                               : il_scan<false, false, false>(T, le, lc, src, Atab, Btab, lofs2, 0, 0, 0u, 0, 0);
#ifdef CCJ_DEBUG_BOUNDS
        if ((act && (a < 0 || a > t || h < 0 || h >= m || i < 1 || i > m - h)) || (actb && (hb < 0 || ib > m - hb))) {
            atomicOr(T.err, 128);
            return;
        }
#endif
        int16_t *dr = T.d4 + Lt.lb + (long long)mslot(PR) * Lt.C + a * Lt.M;
        if (act && gq == 0) dr[h * m - ((h * (h - 1)) >> 1) + i - 1] = (int16_t)clamp_store(bm.x);
        if (actb) dr[hb * m - ((hb * (hb - 1)) >> 1) + ib - 1] = (int16_t)clamp_store(bm.y);
    } else {
        // PM: wave = (h, j, a-chunk), lanes a; pair (j, k), per-lane window u1 <= a-2, u2 <= b-2
        const int h = f1, j = f2;
        const int g = h + 2, k = j + g;
        // the rank's own a-blocks in the window (all of [alo, ahi] when unsharded): lanes = own index
        int o0, o1;
        pm_own_range(n, t, j, k, G_SH, rank, o0, o1);  // ccj_items.h
        const int oz = zc * IL_CW;
        const ILGroups lg = il_groups(imin(64, o1 - o0 - oz + 1), lane);
        const int G = lg.G, gq = lg.gq;
        const bool pair = o1 - o0 - oz + 1 > 64;
        const int o = o0 + oz + lg.rl, ob = o + 64;
        const bool act = o <= o1, actb = pair && ob <= o1;
        const int a = shard_a(imin(o, o1), G_SH, rank), ab = shard_a(imin(ob, o1), G_SH, rank);
        const int as = a;
        const unsigned lofs2 = 2u * (unsigned)as, lofs2b = 2u * (unsigned)ab;
        const size_t pidx = (size_t)g * rs + j;
        // PMx(t-dt, a-1-u1, h+dt, j-1-u1) = pmb + (h+dt)*n*(t+1-dt) + (j-2-u1)(t+1-dt) - 1-u1 + a
        //   = [pmb + (h+dt)*n*(t+1-dt) + (j-2)(t+1-dt) - 1] + [-u1(t+2)] + u1*dt
        // Lanes outside the get_PMiloop window read another cell of the same level (h+dt >= 4:
        // in bounds) and are masked.
        const int Btab = (int)(2 * (-(long long)lane * (t + 2) + BIAS));
        int Atab = 0;
        if (lvl_ok)
            Atab = (int)(unsigned)(2 * (T.ldx[tl].pmb - pb + ((long long)(h + lane) * n + (j - 2)) * (tl + 1) - 1 - BIAS));
        const int B0 = __builtin_amdgcn_readlane(Btab, 0);
        if (lane == 63) Atab = -B0;
        // entries with dt > t-2 fit no cell of this level
        const int cnt = (int)ld_const(T.ilmseg + pidx * IL_SEG + imin(t - 1, IL_SEG - 1));
        const int e0 = (int)ld_const(T.ilmseg + pidx * IL_SEG + 3);
        const uint2 *le = T.ilm + pidx * IL_CAP + e0;
        const int2 bm = G > 1  ? make_int2(il_scan_g<true, true>(T, le, ILHALF(cnt - e0), src, Atab, Btab, lofs2, as, t - as, G, lg.W, gq, lg.rl), INF)
                        : pair ? il_scan<true, true, true>(T, le, ILHALF(cnt - e0), src, Atab, Btab, lofs2, as, t - as, lofs2b, ab, t - ab)
                               : il_scan<true, true, false>(T, le, ILHALF(cnt - e0), src, Atab, Btab, lofs2, as, t - as, 0u, 0, 0);
#ifdef CCJ_DEBUG_BOUNDS
        if ((act && (a < 0 || a > t || h < 0 || h >= m || (j - a) < 1 || (j - a) > m - h)) ||
            (actb && (ab < 0 || ab > t || (j - ab) < 1 || (j - ab) > m - h))) {
            atomicOr(T.err, 128);
            return;
        }
#endif
        int16_t *dm = T.d4 + Lt.lb + (long long)mslot(PM) * Lt.C + h * m - ((h * (h - 1)) >> 1) + j - 1;
        if (act && gq == 0) dm[a * Lt.M - a] = (int16_t)clamp_store(bm.x);
        if (actb) dm[ab * Lt.M - ab] = (int16_t)clamp_store(bm.y);
    }
}

// ------------------------------------------------------------------------------------------
// AoS loop records (ccj_engine.h RecType): pack / unpack int16 pairs
__device__ __forceinline__ unsigned pk16(int lo, int hi) { return (unsigned)(uint16_t)lo | ((unsigned)(uint16_t)hi << 16); }
__device__ __forceinline__ int lo16(unsigned w) { return (int)(int16_t)(w & 0xffffu); }
__device__ __forceinline__ int hi16(unsigned w) { return (int)w >> 16; }

// ints per lane a leader's split wave hands to part 0: the followers' slices r = 1..R-1 of one side
constexpr int LEAD_RED = 15 * SHARE_R;

// split-point sharing (ccj_engine.h): the SHARE_R W values of one split step, one per follower
typedef int wv_t __attribute__((ext_vector_type(SHARE_R)));
// partial record: up to 7 int16 fields (min-clamped like a store), slot 7 = 32767
__device__ __forceinline__ uint4 pack_acc(const int *f, int nf) {
    int c[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) c[x] = x < nf ? clamp_store(f[x]) : INTERN_INF;
    return make_uint4(pk16(c[0], c[1]), pk16(c[2], c[3]), pk16(c[4], c[5]), pk16(c[6], c[7]));
}

// the three records of one cell (values as stored, i.e. already clamped)
__device__ __forceinline__ void write_records(const DevTables &T, long long lr, int C, unsigned cell, int Lm00, int Mm00,
                                              int Om00, int fL, int fO, int Lm10, int fMp, int K, int Rm00, int fR,
                                              int PLR, int Mm10, int Om10) {
    uint4 *rp = T.rec + lr;
    rp[cell] = make_uint4(pk16(Lm00, Mm00), pk16(Om00, fL), pk16(fO, Lm10), pk16(fMp, K));
    T.rk[(lr >> 1) + cell] = make_uint3(pk16(Rm00, Mm00), pk16(fR, PLR), pk16(K, INTERN_INF));
    rp[(unsigned)C + cell] = make_uint4(pk16(Rm00, Mm00), pk16(Om00, Mm10), pk16(Om10, fR), pk16(fO, INTERN_INF));
}


// Software-pipelined split scan: visits s = s0, s0+step, ... <= last, issuing the loads of step
// s+step before reducing step s (mask: 0 while s < mlim, INF on the last split point).  The loads
// return raw registers (records, (WBP, WP) pairs) and every field is unpacked in the reduce, so
// nothing waits on a load before its step is reduced; and the two buffers alternate (ping-pong),
// so the loop carries no register copies.  (Round 2 before this: unpack at load time and
// `cur = nxt` each trip, which made the compiler wait for every load of the next step before the
// back-edge — one full memory latency per split step.)
template <class V, class LD, class ST>
__device__ __forceinline__ void pipe_scan(int s, int step, int last, int mlim, LD ld, ST st) {
    V A = ld(s);
#pragma unroll 1
    for (;;) {
        int sn = s + step;
        if (sn > last) {
            st(A, s < mlim ? 0 : INF);
            return;
        }
        const V B = ld(sn);
        st(A, s < mlim ? 0 : INF);
        s = sn;
        sn = s + step;
        if (sn > last) {
            st(B, s < mlim ? 0 : INF);
            return;
        }
        A = ld(sn);
        st(B, s < mlim ? 0 : INF);
        s = sn;
    }
}
// The one-buffer loop shape (`cur = nxt`), kept for the leaders' loops: their ping-pong form needs
// 241 VGPRs instead of ~150 (2 waves/SIMD) and measured fill +5 ms.  (Peeling the
// final, possibly masked, step so the other steps skip the mask adds — ~15% of a leader step's
// VALU — measured fill +1.7 ms: 146 instead of 130 VGPRs, the leaders are not VALU-bound.)
template <class V, class LD, class ST>
__device__ __forceinline__ void pipe_scan_lead(int s, int step, int last, int mlim, LD ld, ST st) {
    V cur = ld(s);
    for (;;) {
        const int sn = s + step;
        const V nxt = ld(imin(sn, last));
        st(cur, s < mlim ? 0 : INF);
        if (sn > last) break;
        cur = nxt;
        s = sn;
    }
}


// ------------------------------------------------------------------------------------------
// 4-D level t: one lane per cell (i,j,k,l); all lanes of a wave share (t, a) so every loop bound
// is wave-uniform.  pseudo_loop.cc:181-644, 663-808.
//
// Addressing.  A neighbour at (t-dt, a', h+dh, i+di) of matrix x is element
//     x*C' + a'*M' + [dh*m + dh*dt - dh(dh-1)/2 + di]   (wave-uniform: SGPRs)
//   + L0 + h*(dt-dh)                                   (per lane: VGPR)
// of level t' = t-dt, whose base/C'/M' come from one 16-byte descriptor (T.ld[t']).  L0 is the
// cell's own in-block offset.  Loops walk these terms incrementally, so a read costs ~one scalar
// add plus one vector add; every read is a coalesced global load.
//
// The split-point loops of the 22 recurrences are fused into one loop over the (i,j) gap ("a-loop")
// and one over the (k,l) gap ("b-loop"): each neighbour value is loaded once and feeds every
// recurrence that reads it (11a + 13b loads per cell instead of 14a + 16b).  The interior-loop
// windows are walked by source level dt (outer) so the level descriptor is loaded once per dt.
// ------------------------------------------------------------------------------------------
template <bool LEAD>
__device__ __forceinline__ void level4d_body(const DevTables &T, int t, int wavesPerA, int split, int G, int rank, int nblk,
                                             int copies) {
#ifdef CCJ_DEBUG_BOUNDS
    g_dbg_err = T.err;
#endif
    TL_STAMP(t == L_ ? (LEAD ? 1 : 0) : -1);
    // split > 1 (late, narrow levels): the split waves of one 64-cell chunk share the a/b loops
    // (step s = part + 1, part + 1 + split, ...) and min-reduce their partial results through LDS.
    extern __shared__ int red[];  // [chunk][part-1][22][64], split > 1 only
    const int n = T.n, rs = T.rs;
    const int bid = blockIdx.x;
    const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int part = wib % split;
    const int cpb = (int)(blockDim.x >> 6) / split;  // chunks per block
    const int gw = __builtin_amdgcn_readfirstlane(bid * cpb + wib / split);
    const int lane = threadIdx.x & 63;
    // this launch computes nblk a-blocks of level t: rank's own blocks shard_a(0 .. nblk-1) (all of
    // them when unsharded, ccj_engine.h), or on leader launches the rank's list T.lord
    const int a_rel = __builtin_amdgcn_readfirstlane(gw / wavesPerA);
    if (split == 1 && a_rel >= nblk) return;
    const bool wave_ok = a_rel < nblk;  // grid tail (split > 1 keeps the wave for the barrier)
    const int oi = wave_ok ? a_rel : nblk - 1;
    int a = shard_a(oi, G, rank);
    if (LEAD && T.lord) a = T.lord[T.lord_off[t * G + rank] + oi];
    const int chunk = wave_ok ? gw - a_rel * wavesPerA : 0;
    const int m = n - t - 2;
    const int Mt = (m * (m + 1)) >> 1;
    const int c_raw = chunk * 64 + lane;
    if (split == 1 && c_raw >= Mt) return;
    const bool lane_ok = wave_ok && c_raw < Mt;
    const int c = imin(c_raw, Mt - 1);  // idle lanes shadow the last cell (valid reads, no store)
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
    const unsigned L0 = (unsigned)(Gh + i - 1);
    const unsigned uh = (unsigned)h;

    const Penalties pe = T.pen;
    const int bp = pe.bp, cp = pe.cp, PB = pe.PB, apbp2 = pe.ap + 2 * pe.bp;
    const int *__restrict__ WB = T.WB;
    const int *__restrict__ WP = T.WP;
    const int *__restrict__ WBPr = T.WBP;
    const int2 *__restrict__ WBW = T.WBW;
    const LvlDev *__restrict__ LD = T.ld;
    const int16_t *__restrict__ D4 = T.d4;
#define LDX(lp, L, x, U, ln) ((int)(lp)[(unsigned)(mslot(x) * (L).C + (U)) + (ln)])
    // WB of an interval of `len` bases from its WBP, as k_diag2d stores it (get_WB,
    // pseudo_loop.cc:647-653: min(cp*len, WBP)): one load fewer per split side
#define WBD(wbp, len) imin(cp * (len), (wbp))
#ifdef CCJ_DEBUG_BOUNDS
#define CHK(dt, ap_, dh, di) \
    if ((dt) < 1 || (dt) > t || (ap_) < 0 || (ap_) > t - (dt) || h + (dh) >= m + (dt) || i + (di) < 1 || \
        i + (di) > m + (dt) - h - (dh)) atomicOr(T.err, 4)
#define CHKR(idx) \
    if ((long long)(idx) < 0 || (long long)(idx) >= T.nrec) atomicOr(T.err, 8)
#define CHKK(idx) \
    if ((long long)(idx) < 0 || (long long)(idx) >= T.nrec / 2) atomicOr(T.err, 8)
#define CHKA(idx) \
    if (!T.acc || (long long)(idx) >= T.accC) atomicOr(T.err, 256)
#else
#define CHK(dt, ap_, dh, di)
#define CHKR(idx)
#define CHKK(idx)
#define CHKA(idx)
#endif

    // The a- and b-loops are software-pipelined: the loads of step s+split are issued before the
    // values of step s are consumed, so every wave keeps two steps of loads in flight.  The terms
    // with d strictly inside the gap (s < a, s < b) are masked on the last step by adding INF;
    // their loads still hit valid cells.
    // ---- split-point sharing roles (ccj_engine.h), wave-uniform: 0 = own full scan, 1 = leader
    // (full scan, also for the next SHARE_R-1 cells of its columns), 2 = follower (scans only the
    // split points 1..a%R / 1..b%R, takes the rest from its leader's partial record).  A leader's
    // W(i-r, .) / W(., j+r) operands have spans up to a+r-1 <= t-1 only if b >= r (a-side) / a >= r
    // (b-side), so columns with a short other gap keep full scans.
    const bool grp = t >= T.g_lo && t < T.g_hi;
    const int ra = a % SHARE_R, rb = b % SHARE_R;
    const int arole = (grp && b >= SHARE_R - 1) ? (ra == 0 ? 1 : (t - ra >= T.g_lo ? 2 : 0)) : 0;
    const int brole = (grp && a >= SHARE_R - 1) ? (rb == 0 ? 1 : (t - rb >= T.g_lo ? 2 : 0)) : 0;
    // On sharing levels every wave with a long scan (a leader, or a full scan on either side) runs
    // in its own launch (k_level4d_lead: more registers, scans split over several waves); the plain
    // kernel keeps the cells that only follow (short scans, full occupancy).
    TL_META((unsigned)a | (unsigned)part << 10 | (unsigned)arole << 13 | (unsigned)brole << 15 | 1u << 20);
    if (grp && LEAD != (arole != 2 || brole != 2)) return;
    TL_META((unsigned)a | (unsigned)part << 10 | (unsigned)arole << 13 | (unsigned)brole << 15);
    // last split step this cell scans itself
    const int a_stop = arole == 2 ? ra : a;
    const int b_stop = brole == 2 ? rb : b;

    // ---- fused a-loop: split point d inside [i, j] ----
    const int seed = INTERN_INF + bp;  // A-Q3 seeds
    int pLm00 = seed, pLm01 = INF, pLm10 = INF, pMm00 = seed, pMm10 = INF;
    int pOm00 = seed, pOm10 = INF;
    int fL1 = INF, fL2 = INF, fM = INF, fO1 = INF, pK1 = INF;
    struct AV { int2 w2i, w2j; uint4 wi, wj; int s; };  // raw loads of one split step
    auto load_a = [&](int s) {
        AV v;
        v.s = s;
        const int r2 = (s - 1) * rs, jl = j - s + 1;
        v.w2i = WBW[r2 + i];  // (WBP, WP) of (i, i+s-1)
        v.w2j = WBW[r2 + jl];  // (WBP, WP) of (j-s+1, j)
        CHK(s, a - s, 0, s);
        CHK(s, a - s, s, 0);
#ifdef CCJ_ABLATE_LOCAL
        const LvlDev L = LD[t - 1];  // timing only: every step re-reads one level (cache-resident)
        s = 1;
#else
        const LvlDev L = LD[t - s];
#endif
        const int Ui = (a - s) * L.M + s;                          // X(d,j,k,l), d = i+s: lane L0 + h*s
        const int Uj = (a - s) * L.M + s * m + ((s * (s + 1)) >> 1);  // X(i,d,k,l), d = j-s: lane L0
        const unsigned lh = L0 + uh * (unsigned)s;
        // one RA record per side (ccj_engine.h): x = Lm00|Mm00, y = Om00|fL, z = fO|Lm10, w = fMp|K
        const uint4 *rp = T.rec + L.lr;
        CHKR(L.lr + (unsigned)Ui + lh);
        CHKR(L.lr + (unsigned)Uj + L0);
        v.wi = rp[(unsigned)Ui + lh];
        v.wj = rp[(unsigned)Uj + L0];
        return v;
    };
    auto step_a = [&](const AV &v, int mask) {
        const int wbp_i = v.w2i.x, wp_i = v.w2i.y, wbp_j = v.w2j.x, wp_j = v.w2j.y;
        const int wb_i = WBD(wbp_i, v.s), wb_j = WBD(wbp_j, v.s);
        const int Lm00i = lo16(v.wi.x), Mm00i = hi16(v.wi.x), Om00i = lo16(v.wi.y), fLi = hi16(v.wi.y), fOi = lo16(v.wi.z);
        const int Lm00j = lo16(v.wj.x), Mm00j = hi16(v.wj.x), fLj = hi16(v.wj.y), Lm10j = hi16(v.wj.z);
        const int fMpj = lo16(v.wj.w), Kj = hi16(v.wj.w);
        pLm00 = imin(pLm00, imin(wb_i + Lm00i, Lm00j + wb_j));  // :449-458
        pLm01 = imin(pLm01, Lm00j + wbp_j);                     // :468-471
        pLm10 = imin(pLm10, wbp_i + Lm00i);                     // :481-483
        pMm00 = imin(pMm00, Mm00j + wb_j);                      // :548-551
        pMm10 = imin(pMm10, wbp_i + Mm00i);                     // :581-584
        pOm00 = imin(pOm00, wb_i + Om00i);                      // :599-602
        pOm10 = imin(pOm10, wbp_i + Om00i);                     // :632-635
        fL1 = imin(fL1, fLi + wp_i + mask);        // PfromL(d,j,k,l) + WP(i,d-1)      :357-359
        fO1 = imin(fO1, fOi + wp_i + mask);        // PfromO(d,j,k,l) + WP(i,d-1)      :425-427
        pLm10 = imin(pLm10, Lm10j + wb_j + mask);  // PLmloop10(i,d,k,l) + WB(d+1,j)   :484-486
        fL2 = imin(fL2, fLj + wp_j + mask);        // PfromL(i,d,k,l) + WP(d+1,j)      :360-361
        fM = imin(fM, fMpj + wp_j + mask);         // PfromMprime(i,d,k,l) + WP(d+1,j) :399-401
        pK1 = imin(pK1, Kj + wp_j + mask);         // PK(i,d,k,l) + WP(d+1,j)          :184-187
    };
    // a-leader: one scan of s = 1..a for this cell (r = 0) and its followers r = 1..R-1:
    //   i side: cell (i-r, j, k, l) (level t+r, block a+r, row h), term X(i+s,j,k,l) + W(i-r, i+s-1)
    //   j side: cell (i, j+r, k, l) (level t+r, block a+r, row h-r), term X(i,j-s,k,l) + W(j-s+1, j+r)
    // Both followers mask the same last split point (d = j / d = i) as the leader.
    auto lead_a = [&]() {
        int AI_[SHARE_R][7], AJ_[SHARE_R][7];
#pragma unroll
        for (int r = 0; r < SHARE_R; ++r)
#pragma unroll
            for (int f = 0; f < 7; ++f) AI_[r][f] = AJ_[r][f] = INF;
        struct LA { uint4 wi, wj; int2 q[SHARE_R], p[SHARE_R]; int s; };  // raw loads of one split step
        auto ld = [&](int s) {
            LA v;
            v.s = s;
            const LvlDev L = LD[t - s];
            const int Ui = (a - s) * L.M + s;
            const int Uj = (a - s) * L.M + s * m + ((s * (s + 1)) >> 1);
            const unsigned lh = L0 + uh * (unsigned)s;
            const uint4 *rp = T.rec + L.lr;
            CHKR(L.lr + (unsigned)Ui + lh);
            CHKR(L.lr + (unsigned)Uj + L0);
            v.wi = rp[(unsigned)Ui + lh];
            v.wj = rp[(unsigned)Uj + L0];
            // span-major rows: W(i-r, i+s-1) and W(j-s+1, j+r) have span s-1+r, coalesced along the lanes
#pragma unroll
            for (int r = 0; r < SHARE_R; ++r) {
                const int o = (s - 1 + r) * rs;
#ifdef CCJ_ABLATE_WHOT
                // timing only: every W operand load on one cache-resident line (wrong results)
                v.q[r] = WBW[(lane & 15) + 0 * (o + i - r)];
                v.p[r] = WBW[(lane & 15) + 16 + 0 * (o + j - s)];
#else
                v.q[r] = WBW[o + i - r];
                v.p[r] = WBW[o + j - s + 1];
#endif
            }
            return v;
        };
        auto st = [&](const LA &v, int mask) {
            const int Lm00i = lo16(v.wi.x), Mm00i = hi16(v.wi.x), Om00i = lo16(v.wi.y), fLi = hi16(v.wi.y);
            const int fOi = lo16(v.wi.z);
            const int Lm00j = lo16(v.wj.x), Mm00j = hi16(v.wj.x), fLj = hi16(v.wj.y), Lm10j = hi16(v.wj.z);
            const int fMpj = lo16(v.wj.w), Kj = hi16(v.wj.w);
#pragma unroll
            for (int r = 0; r < SHARE_R; ++r) {
                const int wbpi = v.q[r].x, wpi = v.q[r].y, wbi = WBD(wbpi, v.s + r);
                const int wbpj = v.p[r].x, wpj = v.p[r].y, wbj = WBD(wbpj, v.s + r);
                int *I = AI_[r], *J = AJ_[r];
                I[0] = imin(I[0], wbi + Lm00i);          // PLmloop00 :449-458
                I[1] = imin(I[1], wbpi + Lm00i);         // PLmloop10 :481-483
                I[2] = imin(I[2], wbpi + Mm00i);         // PMmloop10 :581-584
                I[3] = imin(I[3], wbi + Om00i);          // POmloop00 :599-602
                I[4] = imin(I[4], wbpi + Om00i);         // POmloop10 :632-635
                I[5] = imin(I[5], fLi + wpi + mask);     // PfromL    :357-359
                I[6] = imin(I[6], fOi + wpi + mask);     // PfromO    :425-427
                J[0] = imin(J[0], Lm00j + wbj);          // PLmloop00
                J[1] = imin(J[1], Lm00j + wbpj);         // PLmloop01 :468-471
                J[2] = imin(J[2], Mm00j + wbj);          // PMmloop00 :548-551
                J[3] = imin(J[3], Lm10j + wbj + mask);   // PLmloop10 :484-486
                J[4] = imin(J[4], fLj + wpj + mask);     // PfromL    :360-361
                J[5] = imin(J[5], fMpj + wpj + mask);    // PfromM    :399-401
                J[6] = imin(J[6], Kj + wpj + mask);      // PK        :184-187
            }
        };
        if (1 + part <= a) pipe_scan_lead<LA>(1 + part, split, a, a, ld, st);
        // slices handed over through the ring: the followers' (r >= 1); r = 0 stays in this wave's
        // accumulators
        constexpr int r0 = 1;
        if (split > 1) {  // the split waves' slices meet in part 0
            int *slot = red + (wib / split) * (split - 1) * LEAD_RED * 64 + lane;
            if (part > 0) {
#pragma unroll
                for (int r = 0; r < SHARE_R; ++r)
#pragma unroll
                    for (int f = 0; f < 7; ++f) {
                        if (r < r0) continue;
                        slot[((part - 1) * LEAD_RED + r * 14 + f) * 64] = AI_[r][f];
                        slot[((part - 1) * LEAD_RED + r * 14 + 7 + f) * 64] = AJ_[r][f];
                    }
            }
            __syncthreads();
            if (part == 0)
                for (int p = 1; p < split; ++p)
#pragma unroll
                    for (int r = 0; r < SHARE_R; ++r)
#pragma unroll
                        for (int f = 0; f < 7; ++f) {
                            if (r < r0) continue;
                            AI_[r][f] = imin(AI_[r][f], slot[((p - 1) * LEAD_RED + r * 14 + f) * 64]);
                            AJ_[r][f] = imin(AJ_[r][f], slot[((p - 1) * LEAD_RED + r * 14 + 7 + f) * 64]);
                        }
            __syncthreads();
        }
        {
        pLm00 = imin(pLm00, imin(AI_[0][0], AJ_[0][0]));
        pLm10 = imin(AI_[0][1], AJ_[0][3]);
        pMm10 = AI_[0][2];
        pOm00 = imin(pOm00, AI_[0][3]);
        pOm10 = AI_[0][4];
        fL1 = AI_[0][5];
        fO1 = AI_[0][6];
        pLm01 = AJ_[0][1];
        pMm00 = imin(pMm00, AJ_[0][2]);
        fL2 = AJ_[0][4];
        fM = AJ_[0][5];
        pK1 = AJ_[0][6];
        }
        if (!lane_ok || part != 0) return;
#ifdef CCJ_ABLATE_NOACC  // timing only: no partial-record stores (followers read stale partials)
        return;
#endif
#pragma unroll
        for (int r = 0; r < SHARE_R; ++r) {
            if (r < r0) continue;
            const int tf = t + r;
            if (tf >= T.g_hi) break;
            const int Mf = LD[tf].M, mf = m - r;
            uint4 *ring = T.acc + (long long)((tf % SHARE_SLOTS) * SHARE_NACC) * T.accC;
            if (i - r >= 1) {
                const unsigned idx = (unsigned)((a + r) * Mf) + L0 - (unsigned)(r * (h + 1));
                CHKA(idx);
                ring[(long long)AI * T.accC + idx] = pack_acc(AI_[r], 7);
            }
            if (h - r >= 0) {
                const int hh = h - r;
                const unsigned idx = (unsigned)((a + r) * Mf + hh * mf - ((hh * (hh - 1)) >> 1) + i - 1);
                CHKA(idx);
                ring[(long long)AJ * T.accC + idx] = pack_acc(AJ_[r], 7);
            }
        }
    };
#ifdef CCJ_ABLATE_LINEAR
    if (a < 0)
#endif
    if (arole == 1 && LEAD) {
        lead_a();
    } else if (1 + part <= a_stop) {
        pipe_scan<AV>(1 + part, split, a_stop, a, load_a, step_a);
    }
    // the ring record of the a-loop: a follower's leader partial (split points a%R+1 .. a)
    if (arole == 2) {
        const uint4 *ring = T.acc + (long long)((t % SHARE_SLOTS) * SHARE_NACC) * T.accC;
        const unsigned idx = (unsigned)(a * Mt) + L0;
        CHKA(idx);
        const uint4 pi = ring[(long long)AI * T.accC + idx], pj = ring[(long long)AJ * T.accC + idx];
        pLm00 = imin(pLm00, imin(lo16(pi.x), lo16(pj.x)));
        pLm10 = imin(pLm10, imin(hi16(pi.x), hi16(pj.y)));
        pMm10 = imin(pMm10, lo16(pi.y));
        pOm00 = imin(pOm00, hi16(pi.y));
        pOm10 = imin(pOm10, lo16(pi.z));
        fL1 = imin(fL1, hi16(pi.z));
        fO1 = imin(fO1, lo16(pi.w));
        pLm01 = imin(pLm01, hi16(pj.x));
        pMm00 = imin(pMm00, lo16(pj.y));
        fL2 = imin(fL2, lo16(pj.z));
        fM = imin(fM, hi16(pj.z));
        pK1 = imin(pK1, lo16(pj.w));
    }
    // ---- fused b-loop: split point d inside [k, l] ----
    int pRm00 = seed, pRm01 = INF, pRm10 = INF, pMm01 = INF, pOm01 = INF;
    int fR1 = INF, fR2 = INF, fMp = INF, fO2 = INF, pK2 = INF;
    struct BV { int2 w2k, w2l; uint3 wk; uint4 wl; int s; };  // raw loads of one split step
    auto load_b = [&](int s) {
        BV v;
        v.s = s;
        const int r2 = (s - 1) * rs, ll = l - s + 1;
        v.w2k = WBW[r2 + k];   // (WBP, WP) of (k, k+s-1)
        v.w2l = WBW[r2 + ll];  // (WBP, WP) of (l-s+1, l)
        CHK(s, a, s, 0);
        CHK(s, a, 0, 0);
#ifdef CCJ_ABLATE_LOCAL
        const LvlDev L = LD[t - 1];  // timing only: every step re-reads one level (cache-resident)
        s = 1;
#else
        const LvlDev L = LD[t - s];
#endif
        const int Uk = a * L.M + s * m + ((s * (s + 1)) >> 1);  // X(i,j,d,l), d = k+s: lane L0
        const int Ul = a * L.M;                                 // X(i,j,k,d), d = l-s: lane L0 + h*s
        const unsigned lh = L0 + uh * (unsigned)s;
        // RK at X(i,j,d,l): x = Rm00|Mm00, y = fR|min(PL,PR), z = K|-
        // RL at X(i,j,k,d): x = Rm00|Mm00, y = Om00|Mm10, z = Om10|fR, w = fO|-
        const uint4 *rp = T.rec + L.lr;
        const uint3 *kp = T.rk + (L.lr >> 1);
        CHKK((L.lr >> 1) + (unsigned)Uk + L0);
        CHKR(L.lr + L.C + (unsigned)Ul + lh);
        v.wk = kp[(unsigned)Uk + L0];
        v.wl = rp[(unsigned)(L.C + Ul) + lh];
        return v;
    };
    auto step_b = [&](const BV &v, int mask) {
        const int wbp_k = v.w2k.x, wp_k = v.w2k.y, wbp_l = v.w2l.x, wp_l = v.w2l.y;
        const int wb_k = WBD(wbp_k, v.s), wb_l = WBD(wbp_l, v.s);
        const int Rm00k = lo16(v.wk.x), Mm00k = hi16(v.wk.x), fRk = lo16(v.wk.y), PLRk = hi16(v.wk.y), Kk = lo16(v.wk.z);
        const int Rm00l = lo16(v.wl.x), Mm00l = hi16(v.wl.x), Om00l = lo16(v.wl.y), Mm10l = hi16(v.wl.y);
        const int Om10l = lo16(v.wl.z), fRl = hi16(v.wl.z), fOl = lo16(v.wl.w);
        pRm00 = imin(pRm00, imin(wb_k + Rm00k, Rm00l + wb_l));  // :499-508
        pRm10 = imin(pRm10, wbp_k + Rm00k);                     // :534-537
        pRm01 = imin(pRm01, Rm00l + wbp_l);                     // :520-523
        pMm00 = imin(pMm00, Mm00k + wb_k);                      // :552-555
        pMm01 = imin(pMm01, Mm00l + wbp_l);                     // :567-570
        pOm00 = imin(pOm00, Om00l + wb_l);                      // :603-606
        pOm01 = imin(pOm01, Om00l + wbp_l);                     // :618-621
        fR1 = imin(fR1, fRk + wp_k + mask);               // PfromR(i,j,d,l) + WP(k,d-1)     :379-381
        fMp = imin(fMp, PLRk + PB + wp_k + mask);         // PfromM'' (:663-679) + WP(k,d-1) :412-414
        pK2 = imin(pK2, Kk + wp_k + mask);                // PK(i,j,d,l) + WP(k,d-1)         :189-192
        pMm10 = imin(pMm10, Mm10l + wb_l + mask);         // PMmloop10(i,j,k,d) + WB(d+1,l)  :585-588
        pOm10 = imin(pOm10, Om10l + wb_l + mask);         // POmloop10(i,j,k,d) + WB(d+1,l)  :636-639
        fR2 = imin(fR2, fRl + wp_l + mask);               // PfromR(i,j,k,d) + WP(d+1,l)     :382-383
        fO2 = imin(fO2, fOl + wp_l + mask);               // PfromO(i,j,k,d) + WP(d+1,l)     :429-431
    };
    // b-leader: one scan of s = 1..b for this cell and its followers r = 1..R-1:
    //   k side: cell (i, j, k-r, l) (level t+r, block a, row h-r), term X(i,j,k+s,l) + W(k-r, k+s-1)
    //   l side: cell (i, j, k, l+r) (level t+r, block a, row h),   term X(i,j,k,l-s) + W(l-s+1, l+r)
    auto lead_b = [&]() {
        int AK_[SHARE_R][6], AL_[SHARE_R][9];
#pragma unroll
        for (int r = 0; r < SHARE_R; ++r) {
#pragma unroll
            for (int f = 0; f < 6; ++f) AK_[r][f] = INF;
#pragma unroll
            for (int f = 0; f < 9; ++f) AL_[r][f] = INF;
        }
        struct LB { uint3 wk; uint4 wl; int2 q[SHARE_R], p[SHARE_R]; int s; };  // raw loads of one split step
        auto ld = [&](int s) {
            LB v;
            v.s = s;
            const LvlDev L = LD[t - s];
            const int Uk = a * L.M + s * m + ((s * (s + 1)) >> 1);
            const int Ul = a * L.M;
            const unsigned lh = L0 + uh * (unsigned)s;
            const uint4 *rp = T.rec + L.lr;
            const uint3 *kp = T.rk + (L.lr >> 1);
            CHKK((L.lr >> 1) + (unsigned)Uk + L0);
            CHKR(L.lr + L.C + (unsigned)Ul + lh);
            v.wk = kp[(unsigned)Uk + L0];
            v.wl = rp[(unsigned)(L.C + Ul) + lh];
#pragma unroll
            for (int r = 0; r < SHARE_R; ++r) {
                const int o = (s - 1 + r) * rs;
#ifdef CCJ_ABLATE_WHOT
                v.q[r] = WBW[(lane & 15) + 0 * (o + k - r)];
                v.p[r] = WBW[(lane & 15) + 16 + 0 * (o + l - s)];
#else
                v.q[r] = WBW[o + k - r];
                v.p[r] = WBW[o + l - s + 1];
#endif
            }
            return v;
        };
        auto st = [&](const LB &v, int mask) {
            const int Rm00k = lo16(v.wk.x), Mm00k = hi16(v.wk.x), fRk = lo16(v.wk.y), PLRk = hi16(v.wk.y);
            const int Kk = lo16(v.wk.z);
            const int Rm00l = lo16(v.wl.x), Mm00l = hi16(v.wl.x), Om00l = lo16(v.wl.y), Mm10l = hi16(v.wl.y);
            const int Om10l = lo16(v.wl.z), fRl = hi16(v.wl.z), fOl = lo16(v.wl.w);
#pragma unroll
            for (int r = 0; r < SHARE_R; ++r) {
                const int wbpk = v.q[r].x, wpk = v.q[r].y, wbk = WBD(wbpk, v.s + r);
                const int wbpl = v.p[r].x, wpl_ = v.p[r].y, wbl = WBD(wbpl, v.s + r);
                int *K = AK_[r], *Q = AL_[r];
                K[0] = imin(K[0], wbk + Rm00k);             // PRmloop00 :499-508
                K[1] = imin(K[1], wbpk + Rm00k);            // PRmloop10 :534-537
                K[2] = imin(K[2], Mm00k + wbk);             // PMmloop00 :552-555
                K[3] = imin(K[3], fRk + wpk + mask);        // PfromR    :379-381
                K[4] = imin(K[4], PLRk + PB + wpk + mask);  // PfromMprime :412-414
                K[5] = imin(K[5], Kk + wpk + mask);         // PK        :189-192
                Q[0] = imin(Q[0], Rm00l + wbl);             // PRmloop00
                Q[1] = imin(Q[1], Rm00l + wbpl);            // PRmloop01 :520-523
                Q[2] = imin(Q[2], Mm00l + wbpl);            // PMmloop01 :567-570
                Q[3] = imin(Q[3], Om00l + wbl);             // POmloop00 :603-606
                Q[4] = imin(Q[4], Om00l + wbpl);            // POmloop01 :618-621
                Q[5] = imin(Q[5], Mm10l + wbl + mask);      // PMmloop10 :585-588
                Q[6] = imin(Q[6], Om10l + wbl + mask);      // POmloop10 :636-639
                Q[7] = imin(Q[7], fRl + wpl_ + mask);       // PfromR    :382-383
                Q[8] = imin(Q[8], fOl + wpl_ + mask);       // PfromO    :429-431
            }
        };
        if (1 + part <= b) pipe_scan_lead<LB>(1 + part, split, b, b, ld, st);
        constexpr int r0 = 1;
        if (split > 1) {
            int *slot = red + (wib / split) * (split - 1) * LEAD_RED * 64 + lane;
            if (part > 0) {
#pragma unroll
                for (int r = 0; r < SHARE_R; ++r) {
                    if (r < r0) continue;
#pragma unroll
                    for (int f = 0; f < 6; ++f) slot[((part - 1) * LEAD_RED + r * 15 + f) * 64] = AK_[r][f];
#pragma unroll
                    for (int f = 0; f < 9; ++f) slot[((part - 1) * LEAD_RED + r * 15 + 6 + f) * 64] = AL_[r][f];
                }
            }
            __syncthreads();
            if (part == 0)
                for (int p = 1; p < split; ++p)
#pragma unroll
                    for (int r = 0; r < SHARE_R; ++r) {
                        if (r < r0) continue;
#pragma unroll
                        for (int f = 0; f < 6; ++f)
                            AK_[r][f] = imin(AK_[r][f], slot[((p - 1) * LEAD_RED + r * 15 + f) * 64]);
#pragma unroll
                        for (int f = 0; f < 9; ++f)
                            AL_[r][f] = imin(AL_[r][f], slot[((p - 1) * LEAD_RED + r * 15 + 6 + f) * 64]);
                    }
            __syncthreads();
        }
        {
        pRm00 = imin(pRm00, imin(AK_[0][0], AL_[0][0]));
        pRm10 = AK_[0][1];
        pMm00 = imin(pMm00, AK_[0][2]);
        fR1 = AK_[0][3];
        fMp = AK_[0][4];
        pK2 = AK_[0][5];
        pRm01 = AL_[0][1];
        pMm01 = AL_[0][2];
        pOm00 = imin(pOm00, AL_[0][3]);
        pOm01 = AL_[0][4];
        pMm10 = imin(pMm10, AL_[0][5]);
        pOm10 = imin(pOm10, AL_[0][6]);
        fR2 = AL_[0][7];
        fO2 = AL_[0][8];
        }
        if (!lane_ok || part != 0) return;
#ifdef CCJ_ABLATE_NOACC
        return;
#endif
#pragma unroll
        for (int r = 0; r < SHARE_R; ++r) {
            if (r < r0) continue;
            const int tf = t + r;
            if (tf >= T.g_hi) break;
            const int Mf = LD[tf].M, mf = m - r;
            uint4 *ring = T.acc + (long long)((tf % SHARE_SLOTS) * SHARE_NACC) * T.accC;
            if (h - r >= 0) {  // k side: AK slots 0..5 (12 bytes; slot 6 belongs to the l-side leader)
                const int hh = h - r;
                const unsigned idx = (unsigned)(a * Mf + hh * mf - ((hh * (hh - 1)) >> 1) + i - 1);
                CHKA(idx);
                const uint4 v = pack_acc(AK_[r], 6);
                *(uint3 *)(ring + (long long)AK * T.accC + idx) = make_uint3(v.x, v.y, v.z);
            }
            if (i <= m - h - r) {  // l side: AL, and its 9th field into AK slot 6 of the same cell
                const unsigned idx = (unsigned)(a * Mf) + L0 - (unsigned)(h * r);
                CHKA(idx);
                ring[(long long)AL * T.accC + idx] = pack_acc(AL_[r], 8);
                // bytes 12..15 of AK (slot 6 and the unused slot 7): with the k side's 12 bytes the
                // whole 16-byte record is written (measured equal to a 2-byte store of slot 6)
                ((unsigned *)(ring + (long long)AK * T.accC + idx))[3] = pk16(clamp_store(AL_[r][8]), INTERN_INF);
            }
        }
    };
#ifdef CCJ_ABLATE_LINEAR
    if (b < 0)
#endif
    if (brole == 1 && LEAD) {
        lead_b();
    } else if (1 + part <= b_stop) {
        pipe_scan<BV>(1 + part, split, b_stop, b, load_b, step_b);
    }
    if (brole == 2) {  // the b-loop's ring record (as for the a-loop)
        const uint4 *ring = T.acc + (long long)((t % SHARE_SLOTS) * SHARE_NACC) * T.accC;
        const unsigned idx = (unsigned)(a * Mt) + L0;
        CHKA(idx);
        const uint4 pk = ring[(long long)AK * T.accC + idx], pl = ring[(long long)AL * T.accC + idx];
        pRm00 = imin(pRm00, imin(lo16(pk.x), lo16(pl.x)));
        pRm10 = imin(pRm10, hi16(pk.x));
        pMm00 = imin(pMm00, lo16(pk.y));
        fR1 = imin(fR1, hi16(pk.y));
        fMp = imin(fMp, lo16(pk.z));
        pK2 = imin(pK2, hi16(pk.z));
        fO2 = imin(fO2, lo16(pk.w));
        pRm01 = imin(pRm01, hi16(pl.x));
        pMm01 = imin(pMm01, lo16(pl.y));
        pOm00 = imin(pOm00, hi16(pl.y));
        pOm01 = imin(pOm01, lo16(pl.z));
        pMm10 = imin(pMm10, hi16(pl.z));
        pOm10 = imin(pOm10, lo16(pl.w));
        fR2 = imin(fR2, hi16(pl.w));
    }
    if (split > 1) {
        // min-reduce the split waves' partial a/b-loop results; part 0 finishes the cell
        int acc[22] = {pLm00, pLm01, pLm10, pMm00, pMm10, pOm00, pOm10, fL1, fL2, fM, fO1, pK1,
                       pRm00, pRm01, pRm10, pMm01, pOm01, fR1, fR2, fMp, fO2, pK2};
        const int cl = wib / split;
        int *slot = red + ((cl * (split - 1) + (part - 1)) * 22) * 64 + lane;
        if (part > 0)
#pragma unroll
            for (int x = 0; x < 22; ++x) slot[x * 64] = acc[x];
        __syncthreads();
        if (part > 0) return;
        for (int p = 1; p < split; ++p) {
            const int *src = red + ((cl * (split - 1) + (p - 1)) * 22) * 64 + lane;
#pragma unroll
            for (int x = 0; x < 22; ++x) acc[x] = imin(acc[x], src[x * 64]);
        }
        pLm00 = acc[0]; pLm01 = acc[1]; pLm10 = acc[2]; pMm00 = acc[3]; pMm10 = acc[4]; pOm00 = acc[5];
        pOm10 = acc[6]; fL1 = acc[7]; fL2 = acc[8]; fM = acc[9]; fO1 = acc[10]; pK1 = acc[11];
        pRm00 = acc[12]; pRm01 = acc[13]; pRm10 = acc[14]; pMm01 = acc[15]; pOm01 = acc[16]; fR1 = acc[17];
        fR2 = acc[18]; fMp = acc[19]; fO2 = acc[20]; pK2 = acc[21];
        if (!lane_ok) return;
    }
    // ---- single-step seeds (:519, :533, :566, :580), level t-1
    int vPRm01 = pRm01, vPRm10 = pRm10, vPMm01 = pMm01, vPMm10 = pMm10;
    {
        const int16_t *dummy = D4;
        (void)dummy;
        if (t >= 1) {
            const LvlDev L = LD[t - 1];
            const int16_t *lp = D4 + L.lb;
            if (b >= 1) {
                vPRm01 = imin(vPRm01, LDX(lp, L, PRmloop01, a * L.M, L0 + uh) + cp);          // (i,j,k,l-1)
                vPRm10 = imin(vPRm10, LDX(lp, L, PRmloop10, a * L.M + m + 1, L0) + cp);       // (i,j,k+1,l)
                vPMm01 = imin(vPMm01, LDX(lp, L, PMmloop01, a * L.M + m + 1, L0) + cp);       // (i,j,k+1,l)
            }
            // PMmloop10 from the RL record (d4 does not store it: ccj_engine.h rec_only)
            if (a >= 1) vPMm10 = imin(vPMm10, hi16(T.rec[L.lr + (unsigned)(L.C + (a - 1) * L.M + m + 1) + L0].y) + cp);  // (i,j-1,k,l)
        }
    }
    const int vPLm00 = pLm00, vPLm01 = pLm01, vPLm10 = pLm10, vPRm00 = pRm00, vPMm00 = pMm00;
    const int vPOm00 = pOm00, vPOm01 = pOm01, vPOm10 = pOm10;

    // ---- level t-2 neighbours of PL/PR/PM/PO (stack terms, get_P?mloop, PfromX)
    const LvlDev L2 = LD[t >= 2 ? t - 2 : 0];
    const int16_t *lp2 = D4 + L2.lb;
    // the record-carried matrices of those neighbours (PLmloop10, PfromL, PfromR, PMmloop10,
    // POmloop10, PfromO; ccj_engine.h rec_only) from their loop records: one 16-byte load per cell
    const uint4 *rp2 = T.rec + L2.lr;
    // own slots of level t: k_iloop(t) left the interior-loop minima of PL/PR/PM there
    const LvlDev Lt = LD[t];
    const int C = Lt.C;
    int16_t *dst = T.d4 + Lt.lb + (long long)a * Mt + L0;
    // ---- PL (:232-253) with get_PLiloop (:682-703, k_iloop), get_PLmloop (:705-715)
    int vPL = INF;
    const bool pl_ok = ptype(T, i, j) > 0;
    if (pl_ok) {
        int b1 = INF;
        const int Uin = (a - 2) * L2.M + m + 3;  // (i+1, j-1, k, l): lane L0 + h
        if (a > TURN + 2) {
            // stack (:692-694) and, on the same inner cell, the interior loop with no unpaired base
            // (d, dp) = (i+1, j-1); k_iloop(t) did the rest of get_PLiloop (source levels <= t-3)
            const int pin = LDX(lp2, L2, PL, Uin, L0 + uh);
            b1 = pin + W2E(T.est, i, j);
#ifndef CCJ_ABLATE_ILOOP
            b1 = imin(b1, imin(pin + W2E(T.ie, i, j), (int)dst[mslot(PL) * C]));
#endif
        }
        const uint4 ra = (a >= 2) ? rp2[(unsigned)Uin + L0 + uh] : make_uint4(0, 0, 0, 0);  // RA: ., .|fL, .|Lm10, .
        const int b2 = (a >= 2) ? imin(hi16(ra.z), LDX(lp2, L2, PLmloop01, Uin, L0 + uh)) + apbp2 : INF;
        const int b3 = (a >= TURN + 1) ? hi16(ra.y) : INF;
        vPL = imin(imin(b1, b2), b3);
    }
    // ---- PR (:255-275) with get_PRiloop (:717-738, k_iloop), get_PRmloop (:740-750)
    int vPR = INF;
    const bool pr_ok = ptype(T, k, l) > 0;
    if (pr_ok) {
        int b1 = INF;
        const int Uin = a * L2.M + m + 2;  // (i, j, k+1, l-1): lane L0 + h
        if (b > TURN + 2) {
            const int pin = LDX(lp2, L2, PR, Uin, L0 + uh);  // stack and (d, dp) = (k+1, l-1)
            b1 = pin + W2E(T.est, k, l);
#ifndef CCJ_ABLATE_ILOOP
            b1 = imin(b1, imin(pin + W2E(T.ie, k, l), (int)dst[mslot(PR) * C]));
#endif
        }
        const int b2 = (b >= 2) ? imin(LDX(lp2, L2, PRmloop10, Uin, L0 + uh), LDX(lp2, L2, PRmloop01, Uin, L0 + uh)) + apbp2 : INF;
        const int b3 = (b >= TURN + 1) ? lo16(T.rk[(L2.lr >> 1) + (unsigned)Uin + L0 + uh].y) : INF;  // RK: ., fR|.
        vPR = imin(imin(b1, b2), b3);
    }
    // ---- PM (:277-300) with get_PMiloop (:752-773, k_iloop), get_PMmloop (:775-785)
    int vPM = INF;
    const bool pm_ok = ptype(T, j, k) > 0;
    if (pm_ok) {
        int b1 = INF;
        const bool inner = (a >= 1 && b >= 1);
        const int Uin = (a - 1) * L2.M + 2 * m + 3;  // (i, j-1, k+1, l): lane L0
        if (g > TURN && inner) {
            const int pin = LDX(lp2, L2, PM, Uin, L0);  // stack and (d, dp) = (j-1, k+1)
            b1 = pin + W2E(T.est, j - 1, k + 1);
#ifndef CCJ_ABLATE_ILOOP
            if (a >= 2 && b >= 2) b1 = imin(b1, imin(pin + W2E(T.ie, j - 1, k + 1), (int)dst[mslot(PM) * C]));
#endif
        }
        const int b2 = inner ? imin(hi16(rp2[(unsigned)(L2.C + Uin) + L0].y), LDX(lp2, L2, PMmloop01, Uin, L0)) + apbp2 : INF;  // RL: ., .|Mm10
        const int b3 = inner ? LDX(lp2, L2, PfromM, Uin, L0) : INF;
        const int b4 = (a == 0 && b == 0) ? 0 : INF;
        vPM = imin(imin(b1, b2), imin(b3, b4));
    }
    // ---- PO (:302-322) with get_POiloop (:787-808; interior branch is dead, A-Q5), get_POmloop (:810-820)
    int vPO = INF;
    if (ptype(T, i, l) > 0) {
        const bool inner = (a >= 1 && b >= 1);
        const int Uin = (a - 1) * L2.M + 1;  // (i+1, j, k, l-1): lane L0 + 2h
        int b1 = INF;
        if (l - i > TURN && inner) b1 = LDX(lp2, L2, PO, Uin, L0 + 2 * uh) + W2E(T.est, i, l);
        const uint4 rl = inner ? rp2[(unsigned)(L2.C + Uin) + L0 + 2 * uh] : make_uint4(0, 0, 0, 0);  // RL: ., ., Om10|., fO|.
        const int b2 = inner ? imin(lo16(rl.z), LDX(lp2, L2, POmloop01, Uin, L0 + 2 * uh)) + apbp2 : INF;
        const int b3 = (inner && l - i >= TURN + 1) ? lo16(rl.w) : INF;
        vPO = imin(imin(b1, b2), b3);
    }
#undef LDX
#undef WBD
#undef CHK
#undef CHKR
#undef CHKA
    // values as stored (Matrix4D::set clamp / never-set 32767), read back by same-cell terms
    const int sPL = clamp_store(vPL), sPR = clamp_store(vPR), sPM = clamp_store(vPM), sPO = clamp_store(vPO);
    const int vPfromL = imin(imin(fL1, fL2), imin(imin(sPR, sPM), sPO) + PB);   // :354-374
    const int vPfromR = imin(imin(fR1, fR2), imin(sPM, sPO) + PB);             // :376-394
    const int vPfromM = fM;                                                     // :396-407
    const int vPfromMp = fMp;                                                   // :409-420
    const int vPfromO = imin(imin(fO1, fO2), imin(sPL, sPR) + PB);             // :422-443
    const int vPK = imin(imin(pK1, pK2), imin(imin(sPL, sPM), imin(sPR, sPO)) + PB);  // :181-202

    // ---- stores: one coalesced int16 per matrix
#ifdef CCJ_DEBUG_BOUNDS
    if (i < 1 || i > m - h || h >= m) { atomicOr(T.err, 32); return; }
#endif
    dst[mslot(PK) * C] = (int16_t)clamp_store(vPK);
    dst[mslot(PL) * C] = (int16_t)sPL;
    dst[mslot(PR) * C] = (int16_t)sPR;
    dst[mslot(PM) * C] = (int16_t)sPM;
    dst[mslot(PO) * C] = (int16_t)sPO;
    if (T.mat5) dst[mslot(PfromL) * C] = (int16_t)clamp_store(vPfromL);  // record-carried (ccj_engine.h rec_only)
    if (T.mat5) dst[mslot(PfromR) * C] = (int16_t)clamp_store(vPfromR);  // record-carried (ccj_engine.h rec_only)
    dst[mslot(PfromM) * C] = (int16_t)clamp_store(vPfromM);
    if (T.mat5) dst[mslot(PfromMprime) * C] = (int16_t)clamp_store(vPfromMp);  // record-carried (ccj_engine.h rec_only)
    if (T.mat5) dst[mslot(PfromO) * C] = (int16_t)clamp_store(vPfromO);  // record-carried (ccj_engine.h rec_only)
    if (T.mat5) dst[mslot(PLmloop00) * C] = (int16_t)clamp_store(vPLm00);  // record-carried (ccj_engine.h rec_only)
    dst[mslot(PLmloop01) * C] = (int16_t)clamp_store(vPLm01);
    if (T.mat5) dst[mslot(PLmloop10) * C] = (int16_t)clamp_store(vPLm10);  // record-carried (ccj_engine.h rec_only)
    if (T.mat5) dst[mslot(PRmloop00) * C] = (int16_t)clamp_store(vPRm00);  // record-carried (ccj_engine.h rec_only)
    dst[mslot(PRmloop01) * C] = (int16_t)clamp_store(vPRm01);
    dst[mslot(PRmloop10) * C] = (int16_t)clamp_store(vPRm10);
    if (T.mat5) dst[mslot(PMmloop00) * C] = (int16_t)clamp_store(vPMm00);  // record-carried (ccj_engine.h rec_only)
    dst[mslot(PMmloop01) * C] = (int16_t)clamp_store(vPMm01);
    if (T.mat5) dst[mslot(PMmloop10) * C] = (int16_t)clamp_store(vPMm10);  // record-carried (ccj_engine.h rec_only)
    if (T.mat5) dst[mslot(POmloop00) * C] = (int16_t)clamp_store(vPOm00);  // record-carried (ccj_engine.h rec_only)
    dst[mslot(POmloop01) * C] = (int16_t)clamp_store(vPOm01);
    if (T.mat5) dst[mslot(POmloop10) * C] = (int16_t)clamp_store(vPOm10);  // record-carried (ccj_engine.h rec_only)
    // loop records and interior-loop copies (the copies only where a later k_iloop can read them:
    // its pair can pair); in sharded fills the other ranks' cells get both from k_unpack
    if (!copies) return;
#ifndef CCJ_ABLATE_NOREC  // timing only: no loop-record stores (the split loops then read stale records)
    write_records(T, Lt.lr, C, (unsigned)(a * Mt) + L0, clamp_store(vPLm00), clamp_store(vPMm00), clamp_store(vPOm00),
                  clamp_store(vPfromL), clamp_store(vPfromO), clamp_store(vPLm10), clamp_store(vPfromMp),
                  clamp_store(vPK), clamp_store(vPRm00), clamp_store(vPfromR), imin(sPL, sPR), clamp_store(vPMm10),
                  clamp_store(vPOm10));
#endif
#ifdef CCJ_ABLATE_NOCOPY
    return;  // timing only: no interior-loop copies (k_iloop then reads stale values)
#endif
    const LvlX X = T.ldx[t];
    if (pl_ok) T.d4x[X.lbx + (long long)a * Mt + (i - 1) * m - (((i - 1) * (i - 2)) >> 1) + h] = (int16_t)sPL;
    if (pr_ok) {
        const int q = i + h - 1;
        T.d4x[X.lbx + C + (long long)a * Mt + ((q * (q + 1)) >> 1) + i - 1] = (int16_t)sPR;
    }
    if (pm_ok) T.pmx[X.pmb + ((long long)h * n + j - 1) * (t + 1) + a] = (int16_t)sPM;
}

// The two launches of a level (ccjk_level4d / ccjk_level4d_lead): the plain cells (short scans)
// and, on the split-sharing levels, the long-scan cells with their larger register budget.
__global__ __launch_bounds__(512) void k_level4d(DevTables T, int t, int wavesPerA, int split, int G, int rank, int nblk, int copies) {
    level4d_body<false>(T, t, wavesPerA, split, G, rank, nblk, copies);
}
__global__ __launch_bounds__(512) void k_level4d_lead(DevTables T, int t, int wavesPerA, int split, int G, int rank, int nblk,
                                                      int copies) {
    level4d_body<true>(T, t, wavesPerA, split, G, rank, nblk, copies);
}

// ------------------------------------------------------------------------------------------
extern "C" int ccjk_init2d(const DevTables *T, void *stream) {
    const int total = (T->n + 1) * T->rs;
    hipLaunchKernelGGL(k_init2d, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, *T, total);
    return (int)hipGetLastError();
}

extern "C" int ccjk_precompute_ie(const DevTables *T, void *stream) {
    const int n = T->n;
    dim3 grid((n + 255) / 256, n + 1, 1);
    hipLaunchKernelGGL(k_precompute_ie, grid, dim3(256), 0, (hipStream_t)stream, *T);
    return (int)hipGetLastError();
}

extern "C" int ccjk_diag2d(const DevTables *T, int sigma, int G, int rank, void *stream) {
    const int nint = T->n - sigma;  // intervals of the span; rank takes i = rank+1, rank+1+G, ...
    const int nb = nint > rank ? (nint - rank + G - 1) / G : 0;
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(k_diag2d, dim3(nb), dim3(256), 0, (hipStream_t)stream, *T, sigma, G, rank);
    return (int)hipGetLastError();
}

// The 2-D values of span sigma that k_diag2d writes, for the band-sharded exchange: DT_N int32 planes
// of n+1 entries (V, Vt, P, WBP, WB, WPP, WP, WMv, WMp, WM) in the tail of the level-sigma slice.
// Pack: this rank's intervals.  Unpack: every other rank's intervals (owner (i-1) % G), plus WBW.
constexpr int DT_N = XCH_DT_N;
__global__ __launch_bounds__(256) void k_dtail_pack(DevTables T, int sigma, int G, int rank, int *tail) {
    const int i = 1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int n = T.n;
    if (i + sigma > n || (i - 1) % G != rank) return;
    const int cell = sigma * T.rs + i;
    const int v[DT_N] = {T.V[cell], (int)T.Vt[cell], T.P[cell], T.WBP[cell], T.WB[cell],
                         T.WPP[cell], T.WP[cell], T.WMv[cell], T.WMp[cell], T.WM[cell]};
#pragma unroll
    for (int x = 0; x < DT_N; ++x) tail[x * (n + 1) + i] = v[x];
}
__global__ __launch_bounds__(256) void k_dtail_unpack(DevTables T, int sigma, const int16_t *recv, size_t slice, size_t off,
                                                      int G, int rank) {
    const int i = 1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int n = T.n;
    const int owner = (i - 1) % G;
    if (i + sigma > n || owner == rank) return;
    const int *tl = (const int *)(recv + (size_t)owner * slice + off);
    const int cell = sigma * T.rs + i;
    T.V[cell] = tl[0 * (n + 1) + i];
    T.Vt[cell] = (int8_t)tl[1 * (n + 1) + i];
    T.P[cell] = tl[2 * (n + 1) + i];
    T.WBP[cell] = tl[3 * (n + 1) + i];
    T.WB[cell] = tl[4 * (n + 1) + i];
    T.WPP[cell] = tl[5 * (n + 1) + i];
    T.WP[cell] = tl[6 * (n + 1) + i];
    T.WMv[cell] = tl[7 * (n + 1) + i];
    T.WMp[cell] = tl[8 * (n + 1) + i];
    T.WM[cell] = tl[9 * (n + 1) + i];
    T.WBW[cell] = make_int2(tl[3 * (n + 1) + i], tl[6 * (n + 1) + i]);
}
extern "C" int ccjk_dtail_pack(const DevTables *T, int sigma, int G, int rank, int16_t *tail, void *stream) {
    const int cnt = T->n - sigma;
    if (cnt <= 0) return 0;
    hipLaunchKernelGGL(k_dtail_pack, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, sigma, G, rank,
                       (int *)tail);
    return (int)hipGetLastError();
}
extern "C" int ccjk_dtail_unpack(const DevTables *T, int sigma, const int16_t *recv, size_t slice, size_t off, int G, int rank,
                                 void *stream) {
    const int cnt = T->n - sigma;
    if (cnt <= 0) return 0;
    hipLaunchKernelGGL(k_dtail_unpack, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, sigma, recv,
                       slice, off, G, rank);
    return (int)hipGetLastError();
}

// P terms of every span whose operands' highest level is lev (k_ppush); completes P(lev+3).
extern "C" int ccjk_ppush(const DevTables *T, int lev, int G, int rank, void *stream) {
#ifdef CCJ_ABLATE_PTERM
    return 0;
#endif
    const int n = T->n;
    const int nmax = imin(lev, n - 4 - lev) + 1;  // t2 values of part A (part B has one fewer or equal)
    if (nmax <= 0) return 0;
    const int ngrp = (n - lev - 3 + 63) / 64;
    // spans per wave = partners per reused level-T load (8; 4 and 16 measured slower) and the
    // inner-loop slice per wave (32; 16 and 64 measured the same)
    constexpr int S = PPUSH_S, hs_len = 32;
    const int nch = (nmax + S - 1) / S;
    int npairs = 0;  // (chunk, inner-loop slice) pairs, as k_ppush enumerates them
    for (int c = 0; c < nch; ++c) npairs += (imin((c + 1) * S, nmax) + hs_len - 1) / hs_len;
    const int nout = rank <= lev ? (lev - rank) / G + 1 : 0;  // this rank's outer indices r, r+G, ... <= lev
    if (nout <= 0) return 0;
    const int blocksA = (npairs * ngrp * nout + 3) / 4;
    // split steps in flight per wave: 4 (98 VGPRs) measured 42.1 us per launch standalone vs 53.8 with
    // 2 (62 VGPRs), the same bytes fetched (profiles/r5_ab.txt); CCJ_PP_STEPS=2 for the A/B
    static const int steps = getenv("CCJ_PP_STEPS") ? atoi(getenv("CCJ_PP_STEPS")) : 4;
    if (steps >= 4)
        hipLaunchKernelGGL((k_ppush<S, 4>), dim3((unsigned)(2 * blocksA)), dim3(256), 0, (hipStream_t)stream, *T, lev, ngrp,
                           npairs, hs_len, blocksA, G, rank, nout);
    else
        hipLaunchKernelGGL((k_ppush<S, 2>), dim3((unsigned)(2 * blocksA)), dim3(256), 0, (hipStream_t)stream, *T, lev, ngrp,
                           npairs, hs_len, blocksA, G, rank, nout);
    return (int)hipGetLastError();
}

extern "C" int ccjk_build_il(const DevTables *T, void *stream) {
    const int n = T->n;
    if (n < 1) return 0;
    hipLaunchKernelGGL(k_build_il, dim3(n, n + 1, 2), dim3(64), 0, (hipStream_t)stream, *T);
    return (int)hipGetLastError();
}

extern "C" int ccjk_iloop(const DevTables *T, int t, long long first_item, int nitems, int G, int rank, void *stream) {
#ifdef CCJ_ABLATE_ILOOP
    return 0;
#endif
    if (nitems <= 0) return 0;
    hipLaunchKernelGGL(k_iloop, dim3((unsigned)((nitems + IL_WPB - 1) / IL_WPB)), dim3(64 * IL_WPB), 0, (hipStream_t)stream, *T, t, first_item,
                       nitems, G, rank);
    return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Band-sharded exchange of level t, in two parts (ccj_engine.h XCH_EDGE / XCH_BULK).
// k_pack: rank r's cells of the part's blocks, all 22 matrices, into one contiguous slice
// [x][part index][M] of nmax blocks per matrix (nmax = the largest rank's count of the part at t), so
// each part is ONE all-gather of equal slices.  k_unpack: every cell of the other ranks' blocks of the
// part from the gathered slices (rank r's at recv + r * rstride) back into the level layout, plus its
// loop records and interior-loop copies (what k_level4d writes for its own cells).  The slices carry
// all 22 matrices, the record-only five included (exchange fills keep T.mat5 = 1), so the records are
// rebuilt from them.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack(DevTables T, int t, int G, int r, int part, int nmax, int16_t *send) {
    const int n = T.n, m = n - t - 2, Mt = (m * (m + 1)) >> 1;
    const long long gc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)(gc / Mt);
    if (k >= xch_pcount(t, G, r, part)) return;
    const int c = (int)(gc - (long long)k * Mt);
    const LvlDev Lt = T.ld[t];
    const int16_t *src = T.d4 + Lt.lb + (long long)shard_a(xch_own(k, part), G, r) * Mt + c;
#pragma unroll 2
    for (int x = 0; x < NMAT4; ++x) send[xch_pos(x, k, c, nmax, Mt)] = src[(long long)mslot(x) * Lt.C];
}

__global__ __launch_bounds__(256) void k_unpack(DevTables T, int t, int G, int r, int part, int nmax, const int16_t *recv,
                                                size_t rstride) {
    const int n = T.n, m = n - t - 2, Mt = (m * (m + 1)) >> 1;
    const long long gc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int a = (int)(gc / Mt);
    if (a > t) return;
    int ro, pa, k;
    xch_src(a, G, ro, pa, k);
    if (ro == r || pa != part) return;  // own cell (k_level4d wrote it with its records and copies), or the other part
    const int c = (int)(gc - (long long)a * Mt);
    const float tm = 2.0f * m + 1.0f;
    int h = (int)((tm - sqrtf(tm * tm - 8.0f * (float)c)) * 0.5f);
    h = imax(0, imin(h, m - 1));
    while (h > 0 && h * m - ((h * (h - 1)) >> 1) > c) --h;
    while (h + 1 < m && (h + 1) * m - (((h + 1) * h) >> 1) <= c) ++h;
    const int Gh = h * m - ((h * (h - 1)) >> 1);
    const int i = c - Gh + 1, b = t - a;
    const int j = i + a, kk = j + h + 2, l = kk + b;
    const LvlDev Lt = T.ld[t];
    const LvlX X = T.ldx[t];
    int16_t *dst = T.d4 + Lt.lb + (long long)a * Mt + c;
    const long long C = Lt.C;
    int v[NMAT4];
    const int16_t *sl = recv + (size_t)ro * rstride;
#pragma unroll
    for (int x = 0; x < NMAT4; ++x) {
        v[x] = sl[xch_pos(x, k, c, nmax, Mt)];
        dst[mslot(x) * C] = (int16_t)v[x];
    }
    write_records(T, Lt.lr, Lt.C, (unsigned)(a * Mt + c), v[PLmloop00], v[PMmloop00], v[POmloop00], v[PfromL], v[PfromO],
                  v[PLmloop10], v[PfromMprime], v[PK], v[PRmloop00], v[PfromR], imin(v[PL], v[PR]), v[PMmloop10],
                  v[POmloop10]);
    if (ptype(T, i, j) > 0) T.d4x[X.lbx + (long long)a * Mt + (i - 1) * m - (((i - 1) * (i - 2)) >> 1) + h] = (int16_t)v[PL];
    if (ptype(T, kk, l) > 0) {
        const int q = i + h - 1;
        T.d4x[X.lbx + Lt.C + (long long)a * Mt + ((q * (q + 1)) >> 1) + i - 1] = (int16_t)v[PR];
    }
    if (ptype(T, j, kk) > 0) T.pmx[X.pmb + ((long long)h * n + j - 1) * (t + 1) + a] = (int16_t)v[PM];
}

// The P partials of span sigma (each rank pushed only its share of the terms, k_ppush) ride in the
// tail of the level exchange: k_ptail_pack copies this rank's (value, first split) words of
// P(i, i+sigma), k_ptail_unpack takes the minimum over the ranks' tails (the same first minimum the
// atomicMin of an unsharded fill keeps) into T.Pk.
__global__ __launch_bounds__(256) void k_ptail_pack(DevTables T, int sigma, unsigned long long *tail) {
    const int i = 1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i + sigma > T.n) return;
    tail[i] = T.Pk[sigma * T.rs + i];
}
__global__ __launch_bounds__(256) void k_ptail_unpack(DevTables T, int sigma, const int16_t *recv, size_t slice, size_t off,
                                                      int G) {
    const int i = 1 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i + sigma > T.n) return;
    unsigned long long v = ~0ull;
    for (int r = 0; r < G; ++r) {
        const unsigned long long x = ((const unsigned long long *)(recv + (size_t)r * slice + off))[i];
        v = x < v ? x : v;
    }
    T.Pk[sigma * T.rs + i] = v;
}

extern "C" int ccjk_ptail_pack(const DevTables *T, int sigma, int16_t *tail, void *stream) {
    const int cnt = T->n - sigma;
    if (cnt <= 0) return 0;
    hipLaunchKernelGGL(k_ptail_pack, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, sigma,
                       (unsigned long long *)tail);
    return (int)hipGetLastError();
}

extern "C" int ccjk_ptail_unpack(const DevTables *T, int sigma, const int16_t *recv, size_t slice, size_t off, int G,
                                 void *stream) {
    const int cnt = T->n - sigma;
    if (cnt <= 0) return 0;
    hipLaunchKernelGGL(k_ptail_unpack, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, sigma, recv,
                       slice, off, G);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pack(const DevTables *T, int t, int G, int r, int part, int nmax, int16_t *send, void *stream) {
    const int m = T->n - t - 2;
    if (m <= 0) return 0;
    if (xch_pcount(t, G, r, part) > nmax) return (int)hipErrorInvalidValue;
    const long long cells = (long long)xch_pcount(t, G, r, part) * (m * (m + 1) / 2);
    if (cells <= 0) return 0;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, t, G, r, part, nmax,
                       send);
    return (int)hipGetLastError();
}

extern "C" int ccjk_unpack(const DevTables *T, int t, int G, int r, int part, int nmax, const int16_t *recv, size_t rstride,
                           void *stream) {
    const int m = T->n - t - 2;
    if (m <= 0) return 0;
    // the records of the other ranks' cells are rebuilt from the slices, which must carry all 22
    // matrices: without T.mat5 the five record-only matrices are not in d4 (k_pack would ship stale ones)
    if (!recv || !T->mat5) return (int)hipErrorInvalidValue;
    const long long cells = (long long)(t + 1) * (m * (m + 1) / 2);
    if (xch_nmax(t, G, part) > nmax) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, t, G, r, part, nmax,
                       recv, rstride);
    return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Matrix x of every level rewritten in the reference's canonical (i, j, k, l) order (l fastest):
// the input of ccj_hashes (FNV-1a over that order).  One launch per level t, one thread per cell.
// Canonical position of (i,j,k,l) = offij[i*(n+1)+j] + sum_{k'=j+2}^{k-1} (n+1-k') + (l-k).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_canon(DevTables T, int x, int t, const long long *__restrict__ offij, int16_t *out) {
    const int n = T.n, m = n - t - 2;
    if (m <= 0) return;
    const LvlDev L = T.ld[t];
    const int Mt = L.M;
    const long long cidx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (cidx >= (long long)L.C) return;
    const int a = (int)(cidx / Mt), c = (int)(cidx - (long long)a * Mt);
    const float tm = 2.0f * m + 1.0f;
    int h = (int)((tm - sqrtf(tm * tm - 8.0f * (float)c)) * 0.5f);
    h = imax(0, imin(h, m - 1));
    while (h > 0 && h * m - ((h * (h - 1)) >> 1) > c) --h;
    while (h + 1 < m && (h + 1) * m - (((h + 1) * h) >> 1) <= c) ++h;
    const int Gh = h * m - ((h * (h - 1)) >> 1);
    const int i = c - Gh + 1, j = i + a, k = j + h + 2, l = k + (t - a);
    const long long u = k - (j + 2);
    const long long pos = offij[(long long)i * (n + 1) + j] + u * (n + 1) - u * (2LL * j + 3 + u) / 2 + (l - k);
    out[pos] = (int16_t)((!T.mat5 && rec_only(x)) ? rec_get(T, x, L, cidx) : (int)T.d4[L.lb + (long long)mslot(x) * L.C + cidx]);
}

// the record-carried matrices of level t (ccj_engine.h rec_only), read back from its records into out
// (slots NMAT_ST.. of the level's host-mirror layout, mslot), for a host mirror of a context without
// them in d4
__global__ __launch_bounds__(256) void k_mat5(DevTables T, int t, int16_t *out) {
    const LvlDev L = T.ld[t];
    const long long cidx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (cidx >= (long long)L.C) return;
#pragma unroll
    for (int x = 0; x < NMAT4; ++x)
        if (rec_only(x)) out[(long long)(mslot(x) - NMAT_ST) * L.C + cidx] = (int16_t)rec_get(T, x, L, cidx);
}

extern "C" int ccjk_mat5(const DevTables *T, int t, int16_t *out, void *stream) {
    const int m = T->n - t - 2;
    if (m <= 0 || t >= T->nlev) return 0;
    const long long C = (long long)(t + 1) * (m * (m + 1) / 2);
    hipLaunchKernelGGL(k_mat5, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, t, out);
    return (int)hipGetLastError();
}

extern "C" int ccjk_canon(const DevTables *T, int x, const long long *offij, int16_t *out, void *stream) {
    const int n = T->n;
    for (int t = 0; t < T->nlev; ++t) {
        const int m = n - t - 2;
        const long long C = (long long)(t + 1) * (m * (m + 1) / 2);
        hipLaunchKernelGGL(k_canon, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *T, x, t, offij, out);
    }
    return (int)hipGetLastError();
}

// narrow levels: split each chunk's a/b loops over up to 8 waves so ~split_target waves run at once
extern "C" int ccjk_level_split(int n, int t, int nblk, int split_target) {
    const int m = n - t - 2;
    if (m <= 0 || nblk <= 0) return 1;
    const long waves = (long)nblk * ((m * (m + 1) / 2 + 63) / 64);
    int split = 1;
    while (split_target > 0 && split < 8 && waves * split * 2 <= split_target) split *= 2;
    return split;
}

extern "C" int ccjk_level4d(const DevTables *T, int t, int G, int rank, int copies, void *stream) {
    const int m = T->n - t - 2;
    if (m <= 0) return 0;
    const int Mt = m * (m + 1) / 2;
    const int wavesPerA = (Mt + 63) / 64;
    const int nblk = shard_count(t, G, rank);
    if (nblk <= 0) return 0;
    const long waves = (long)nblk * wavesPerA;
    // on the sharing levels this launch only has follower cells (short scans): never split
    const int split = (t >= T->g_lo && t < T->g_hi) ? 1 : ccjk_level_split(T->n, t, nblk, T->split_target);
    const int threads = split <= 4 ? 256 : 64 * split;
    const int cpb = threads / 64 / split;
    const long blocks = (waves + cpb - 1) / cpb;
    const size_t shmem = split > 1 ? (size_t)cpb * (split - 1) * 22 * 64 * sizeof(int) : 0;
    hipLaunchKernelGGL(k_level4d, dim3((unsigned)blocks), dim3(threads), shmem, (hipStream_t)stream, *T, t, wavesPerA, split,
                       G, rank, nblk, copies);
    return (int)hipGetLastError();
}

// the split-point-sharing leader waves of level t (no-op outside the sharing range)
extern "C" int ccjk_level4d_lead(const DevTables *T, int t, int G, int rank, void *stream) {
    if (t < T->g_lo || t >= T->g_hi) return 0;
    const int m = T->n - t - 2;
    const int Mt = m * (m + 1) / 2;
    const int wavesPerA = (Mt + 63) / 64;
    // only the rank's long-scan a-blocks (T->lord, longest first) when the list is there
    const int own = shard_count(t, G, rank);
    const int nblk = T->lord ? T->lord_off_h[t * G + rank + 1] - T->lord_off_h[t * G + rank] : own;
    if (nblk <= 0) return 0;
    const long waves = (long)nblk * wavesPerA;
    // each leader chunk's scans are split over `split` waves of one workgroup (the barriers inside
    // the leader scans need every wave of the workgroup on the same chunk)
    constexpr int lsplit = 2;  // 1 / 3 / 4 measured +1.1 / +6.5 / +9.4 ms
    // narrow late levels: as many split waves as the plain heuristic would give the rank's blocks
    const int sp = imax(lsplit, ccjk_level_split(T->n, t, own, T->split_target));
    const size_t shmem = sp > 1 ? (size_t)(sp - 1) * (LEAD_RED > 22 ? LEAD_RED : 22) * 64 * sizeof(int) : 0;
    hipLaunchKernelGGL(k_level4d_lead, dim3((unsigned)waves), dim3(64 * sp), shmem, (hipStream_t)stream, *T, t, wavesPerA,
                       sp, G, rank, nblk, 1);
    return (int)hipGetLastError();
}

#ifdef CCJ_WG_TIMELINE
// measurement build only (tools/wg_timeline.py): arm level t (clears the stamps), read them back
extern "C" int ccjk_tl_arm(int t) {
    static ulonglong4 zero[TL_CAP];
    for (int k = 0; k < TL_KINDS; ++k)
        if (hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_tl), zero, sizeof(zero), (size_t)k * sizeof(zero))) return (int)e;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_tl_level), &t, sizeof(int));
}
extern "C" int ccjk_tl_read(int kind, void *out, int cap) {
    if (kind < 0 || kind >= TL_KINDS || cap > TL_CAP) return -1;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), (size_t)cap * sizeof(ulonglong4), (size_t)kind * TL_CAP * sizeof(ulonglong4));
}
extern "C" int ccjk_tl_cap() { return TL_CAP; }
extern "C" int ccjk_tl_kinds() { return TL_KINDS; }
#endif
