// ccj_pf.hip — the CCJ partition function fill on the GPU (reference
// W_final_pf::ccj_pf, part_func.cc:152-178, and every compute_* it calls, :222-699).
//
// Same level-synchronous wavefront as the MFE fill: a 4-D cell (i,j,k,l) at level
// t = (j-i)+(l-k) reads only cells of lower levels and, inside the cell, the values the
// reference's loop order has already produced.  The reference visits (i,l) with i descending and l
// ascending and, per (i,l): V, then P, WBP, WPP, then the 4-D cells (j ascending, k descending:
// 12 mloops, PL PR PM PO, 4 Pfrom, PK), then WMv/WMp and WM (part_func.cc:154-161, 302-359).
// Every read of that order targets a finished value, so per level:
//   k_pf_pterm(s)  P(i,i+s) from the PK cells of levels <= s-3       (compute_P :383-393)
//   k_pf_diag(s)   V, VM, WBP, WPP, WMv, WMp, WM of span s            (:242-300, 361-381)
//   k_pf_level(t)  the 21 4-D recurrences of level t                  (:395-699)
// Exactness (bit-identical to part_func.cc built with -ffp-contract=off):
//   * every double sum is accumulated by one thread in the reference's term order, with the
//     reference's association, and this file is compiled without contraction;
//   * the 4-D matrices hold what Matrix4DPF keeps: the x86 int truncation of the sum (int32);
//   * P sums int products made in 32-bit int arithmetic, accumulated exactly in int64 across
//     threads and converted once; that equals the reference's serial double sum whenever the sum
//     of |terms| stays below 2^53 (always for n <= 295), which the fill checks (Pabs) and
//     otherwise reports CCJ_E_PF_RANGE instead of a result;
//   * table values (Boltzmann weights, pow(), the hairpin strstr cases) come from the host libm.
// An interior-loop term whose Boltzmann factor is exactly 0.0 (a pair that cannot pair; the
// reference skips it) adds a signed zero here: it changes no bit of a nonzero partial sum, and
// every 4-D sum ends in an int truncation, where the sign of a zero is lost.  So the iloop terms
// are added branch-free, which lets the loads of consecutive terms overlap.
// The interior-loop sums (get_PLiloop / get_PRiloop / get_PMiloop, up to 29 x 29 terms per cell)
// run before each level in k_pf_iloop, one wave per closing pair (i,j) / (k,l) / (j,k) and its
// cells, reading copies of PL / PR / PM laid out so that the 64 lanes of one candidate term read
// consecutive words; k_pf_level adds the finished sums in their place.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ccj_pf_energy.h"
#include "ccj_pf_engine.h"

using namespace ccj;

namespace {

struct PfG {  // getters with the reference's semantics
    const PfDev &D;
    __device__ __forceinline__ double d2(const double *A, int i, int j) const { return A[(j - i) * D.rs + i]; }
    // TriangleMatrix_PF::get (matrices.hh:105-108): i > j -> 0
    __device__ __forceinline__ double g2(const double *A, int i, int j) const { return i > j ? 0.0 : d2(A, i, j); }
    // get_WB / get_WP (part_func.cc:701-715)
    __device__ __forceinline__ double WB(int i, int j) const {
        if (i <= 0 || j <= 0 || i > D.n || j > D.n) return 0.0;
        if (i > j) return 1.0;
        return D.cpp[j - i + 1] + d2(D.WBP, i, j);
    }
    __device__ __forceinline__ double WP(int i, int j) const {
        if (i <= 0 || j <= 0 || i > D.n || j > D.n) return 0.0;
        if (i > j) return 1.0;
        return D.pup[j - i + 1] + d2(D.WPP, i, j);
    }
    // Matrix4DPF::get (matrices.hh:258-263): 0 outside i <= j < k-1, k <= l, else the stored int
    __device__ __forceinline__ int g4(int x, int i, int j, int k, int l) const {
        if (!(i <= j && j < k - 1 && k <= l)) return 0;
        const int a = j - i, b = l - k, t = a + b, h = k - j - 2, m = D.n - t - 2;
        const PfLvl L = D.ld[t];
        return D.d4[L.lb + (long long)x * L.C + (long long)a * L.M + h * m - ((h * (h - 1)) >> 1) + i - 1];
    }
    __device__ __forceinline__ int pt(int i, int j) const { return D.pt[(j - i) * D.rs + i]; }
};

// Wave-uniform loads of tables no kernel of the fill writes (level descriptors, expcp_pen /
// expPUP_pen): through the constant address space, so they are scalar loads with their own wait
// counter.  (As plain global loads the compiler cannot prove them unclobbered and emits vector
// loads, which a split loop then waits for in order with everything issued before them.)
__device__ __forceinline__ double ldc_f64(const double *p) {
    return *(const __attribute__((address_space(4))) double *)(unsigned long long)p;
}
struct PfLvlS { long long lb, C; int M; long long lr; };
__device__ __forceinline__ PfLvlS ldc_lvl(const PfLvl *p) {
    const auto *q = (const __attribute__((address_space(4))) PfLvl *)(unsigned long long)p;
    return PfLvlS{q->lb, q->C, q->M, q->lr};
}

// Buffer loads with a wave-uniform 32-bit byte offset (soffset) and a per-lane one (voffset) from a
// uniform base: the split loops' operands without 64-bit address arithmetic per load (as 64-bit
// indices the loop spent ~10 scalar instructions per load)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pf_rsrc(const void *p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((unsigned long long)hi << 32) | lo), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ int bld32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return (int)__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
__device__ __forceinline__ double bld64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
// a split-loop record's first three / next two or three ints (ccj_pf_engine.h PfDev::r1 .. r4)
typedef unsigned __attribute__((ext_vector_type(3))) pfu3;
typedef unsigned __attribute__((ext_vector_type(2))) pfu2;
__device__ __forceinline__ pfu3 bld96(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b96(r, voff, soff, 0);
}
__device__ __forceinline__ pfu2 bld64u(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
}

// Software-pipelined split loop over s = s0 .. s1: the loads of step s+1 are issued before step s
// is reduced, into two alternating buffers (no register copies across the back-edge, which would
// make the compiler wait for every load of the trip first).  The reduce adds each sum's terms in
// the reference's order, so the bits do not change.
template <class V, class LD, class RD>
__device__ __forceinline__ void pf_pipe(int s, int s1, LD ld, RD rd) {
    if (s > s1) return;
    V A = ld(s);
#pragma unroll 1
    for (;;) {
        if (s + 1 > s1) { rd(A); return; }
        const V B = ld(s + 1);
        rd(A);
        ++s;
        if (s + 1 > s1) { rd(B); return; }
        A = ld(s + 1);
        rd(B);
        ++s;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// P(i, i+s) (compute_P, part_func.cc:383-393): sum over j < d < k of PK(i,j,d+1,k) * PK(j+1,d,k+1,l),
// the product in int.  The sum is exact in int64 (checked through Pabs), so its order is free:
// a workgroup of 4 waves takes 64 consecutive i (lanes), one j-i (blockIdx.y) and a run of
// PT_DD values of d-i (blockIdx.z), wave w every 4th of them; each lane loops k, 4 terms per round
// in flight, and the 4 waves' partial sums meet in LDS, so each interval gets one atomic pair per
// workgroup (PT_DD (j, d) pairs) instead of one per (j, d).
// ---------------------------------------------------------------------------------------------
constexpr int PT_DD = 16;

__global__ __launch_bounds__(256) void k_pf_pterm(PfDev D, int s) {
    const int jo = blockIdx.y, dd0 = jo + 1 + (int)blockIdx.z * PT_DD;  // j = i+jo, d = i+dd
    if (dd0 > s - 2) return;  // whole workgroup
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n = D.n;
    const int i = blockIdx.x * 64 + lane + 1;
    const int ic = imin(i, n - s);  // idle lanes re-read a valid interval
    typedef const __attribute__((address_space(1))) int gint;
    long long acc = 0;
    unsigned long long aabs = 0;
    const int dd1 = imin(dd0 + PT_DD - 1, s - 2);
    for (int dd = dd0 + w; dd <= dd1; dd += 4) {
        // PK(i, j, d+1, k): level jo + (ko-dd-1), block jo, row dd-jo-1, position i;
        // PK(j+1, d, k+1, l): level (dd-jo-1) + (s-ko-1), block dd-jo-1, row ko-dd-1, position i+jo+1
        // (ko = k-i): wave-uniform level descriptors, lanes at consecutive positions
        const int a1 = jo, h1 = dd - jo - 1, a2 = dd - jo - 1;
#pragma unroll 4
        for (int ko = dd + 1; ko < s; ++ko) {
            const int h2 = ko - dd - 1, t1 = a1 + h2, t2 = a2 + (s - ko - 1);
            const int m1 = n - t1 - 2, m2 = n - t2 - 2;
            const PfLvl L1 = D.ld[t1], L2 = D.ld[t2];
            const long long U1 = L1.lb + PF_PK * L1.C + (long long)a1 * L1.M + (long long)h1 * m1 - (((long long)h1 * (h1 - 1)) >> 1) - 1;
            const long long U2 = L2.lb + PF_PK * L2.C + (long long)a2 * L2.M + (long long)h2 * m2 - (((long long)h2 * (h2 - 1)) >> 1) + jo;
            const long long x = imul_wrap(*(gint *)(D.d4 + U1 + ic), *(gint *)(D.d4 + U2 + ic));
            acc += x;
            aabs += (unsigned long long)(x < 0 ? -x : x);
        }
    }
    __shared__ long long sacc[3][64];
    __shared__ unsigned long long sabs[3][64];
    if (w > 0) {
        sacc[w - 1][lane] = acc;
        sabs[w - 1][lane] = aabs;
    }
    __syncthreads();
    if (w > 0 || i + s > n) return;
    for (int q = 0; q < 3; ++q) {
        acc += sacc[q][lane];
        aabs += sabs[q][lane];
    }
    if (acc) atomicAdd((unsigned long long *)&D.Pacc[s * D.rs + i], (unsigned long long)acc);
    if (aabs) atomicAdd(&D.Pabs[s * D.rs + i], aabs);
}

// ---------------------------------------------------------------------------------------------
// The same P terms pushed by level (the MFE engine's k_ppush scheme): k_pf_ppush(T),
// after level T, sums every term whose higher operand level is T (part A: t1 = T >= t2; part B:
// t2 = T > t1; t1 + t2 = s - 3 for P(i, i+s)).  That completes P(T+3) and adds partial sums to the
// longer spans.  The level-T operand of a term is the same cell for PF_PP_S consecutive spans, so a
// wave loads it once for PF_PP_S partners (1 + 1/PF_PP_S loads per term instead of 2), and it is
// the level just written.  The sums are exact int64 (as in k_pf_pterm), so any order is the same.
//   part A wave: (jo, 64 consecutive i, PF_PP_S consecutive t2), loop h1 = d-j-1:
//       A = level T, block jo, row h1, position i;  B = level t2, block h1, row T-jo, position i+jo+1
//   part B wave: (a2 = d-j-1, 64 consecutive l, PF_PP_S consecutive t1), loop h2 = k-d-1:
//       B = level T, block a2, row h2, position l-h2-T-2;  A = level t1, block t1-h2, row a2, position l-T-3-t1
// ---------------------------------------------------------------------------------------------

// The operands as buffer loads (the MFE k_ppush's scheme, round 5): a wave reads PK at level lev and at
// the PF_PP_S consecutive levels o0 .. o0+ns-1, each set within 4 GB of its lowest level's PK start
// (ccj_pf_create checks it), so each is one buffer resource (base = that level's PK) and an operand is
// (uniform byte offset, lane byte offset) = (soffset, voffset): no 64-bit row pointer per load (those
// took two readfirstlanes and a 64-bit address each).  Element (t, a, h, pos) of PK is
// pk_base(t) + a*M_t + G_t(h) + pos - 1, G_t(h) = h*m_t - h(h-1)/2.
__device__ __forceinline__ long long pf_pk_base(const PfDev &D, int t) {
    const PfLvlS L = ldc_lvl(D.ld + t);
    return L.lb + PF_PK * L.C;
}
__device__ __forceinline__ int pf_G(int m, int h) { return h * m - ((h * (h - 1)) >> 1); }

template <int U>
__global__ __launch_bounds__(256) void k_pf_ppush(PfDev D, int lev, int ngrp, int npairs, int hs_len, int blocksA) {
    const int n = D.n, rs = D.rs;
    const int lane = threadIdx.x & 63;
    const int partB = (int)blockIdx.x >= blocksA;
    const int item = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - (partB ? blocksA : 0)) * 4 + (int)(threadIdx.x >> 6));
    // item = (pair * nout + outer) * ngrp + g (k_ppush's enumeration, unsharded): g, 64 intervals,
    // fastest, so a workgroup's 4 waves read adjacent segments of the same rows
    const int nout = lev + 1;
    const int g = item % ngrp;
    int pr = item / ngrp;
    const int outer = pr % nout;
    pr /= nout;
    if (pr >= npairs) return;  // whole wave
    const int nmax = imin(lev, n - 4 - lev) + 1;
    int c = 0;
    for (;; ++c) {
        const int cnt = (imin((c + 1) * PF_PP_S, nmax) + hs_len - 1) / hs_len;
        if (pr < cnt) break;
        pr -= cnt;
    }
    const int hs = pr;
    const int nother = (partB ? imin(lev - 1, n - 4 - lev) : imin(lev, n - 4 - lev)) + 1;
    const int o0 = c * PF_PP_S;
    if (o0 >= nother) return;
    const int ns = imin(PF_PP_S, nother - o0);
    const int h_lo = hs * hs_len;
    const int hmax = imin(o0 + ns - 1, h_lo + hs_len - 1);
    if (h_lo > hmax) return;
    long long acc[PF_PP_S];
    unsigned long long aab[PF_PP_S];
#pragma unroll
    for (int s = 0; s < PF_PP_S; ++s) acc[s] = 0, aab[s] = 0;
    const int mT = n - lev - 2;
    const int MT = ldc_lvl(D.ld + lev).M;
    const long long baseT = pf_pk_base(D, lev), baseO = pf_pk_base(D, o0);
    const __amdgpu_buffer_rsrc_t srcT = pf_rsrc(D.d4 + baseT), srcO = pf_rsrc(D.d4 + baseO);
    auto add = [&](int s, int x, bool live) {
        const long long v = live ? (long long)x : 0;
        acc[s] += v;
        aab[s] += (unsigned long long)(v < 0 ? -v : v);
    };
    if (!partB) {
        const int jo = outer, b1 = lev - jo;
        const int i = 1 + g * 64 + lane;
        if (1 + g * 64 > n - (lev + 3 + o0)) return;  // no lane has an interval of the shortest span
        // B of span s: level t2, block h1 (soffset h1 * 4 M, per step), row b1, position
        // min(i, n - (lev+3+t2)) + jo + 1 (voffset, fixed per lane)
        int voB[PF_PP_S], Ms4[PF_PP_S];
#pragma unroll
        for (int s = 0; s < PF_PP_S; ++s) {
            const int t2 = imin(o0 + s, o0 + ns - 1);
            Ms4[s] = __builtin_amdgcn_readfirstlane(4 * ldc_lvl(D.ld + t2).M);  // uniform: a per-lane soffset would be a waterfall
            voB[s] = (int)((unsigned)(4 * (pf_pk_base(D, t2) - baseO + pf_G(n - t2 - 2, b1))) +
                           4u * (unsigned)(imin(i, n - (lev + 3 + t2)) + jo));
        }
        // U steps per iteration, all U * (PF_PP_S + 1) loads in flight together (the steps of a short
        // tail re-read the last one and are masked)
        for (int h1 = h_lo; h1 <= hmax; h1 += U) {
            int va[U], vb[U][PF_PP_S], hh[U];
#pragma unroll
            for (int u = 0; u < U; ++u) hh[u] = imin(h1 + u, hmax);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int h = hh[u];
                va[u] = bld32(srcT, 4 * (imin(i, mT - h) - 1), 4 * (jo * MT + pf_G(mT, h)));
#pragma unroll
                for (int s = 0; s < PF_PP_S; ++s) {
                    const int t2 = imin(o0 + s, o0 + ns - 1), hc = imin(h, t2);
                    vb[u][s] = bld32(srcO, voB[s], hc * Ms4[s]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool live = h1 + u <= hmax;
#pragma unroll
                for (int s = 0; s < PF_PP_S; ++s) add(s, imul_wrap(va[u], vb[u][s]), live && s < ns && hh[u] <= o0 + s);
            }
        }
#pragma unroll
        for (int s = 0; s < PF_PP_S; ++s) {
            const int sg = lev + 3 + o0 + s;
            if (s < ns && i + sg <= n) {
                if (acc[s]) atomicAdd((unsigned long long *)&D.Pacc[sg * rs + i], (unsigned long long)acc[s]);
                if (aab[s]) atomicAdd(&D.Pabs[sg * rs + i], aab[s]);
            }
        }
    } else {
        const int a2 = outer;
        const int l = lev + 4 + o0 + g * 64 + lane;
        if (lev + 4 + o0 + g * 64 > n) return;
        const int lc = imin(l, n);
        // A of span s: level t1, block t1-h2 (soffset (t1-h2) * 4 M, per step), row a2, position
        // max(1, lc - (lev+3+t1)) (voffset, fixed per lane)
        int voA[PF_PP_S], Ms4[PF_PP_S];
#pragma unroll
        for (int s = 0; s < PF_PP_S; ++s) {
            const int t1 = imin(o0 + s, o0 + ns - 1);
            Ms4[s] = __builtin_amdgcn_readfirstlane(4 * ldc_lvl(D.ld + t1).M);
            voA[s] = (int)((unsigned)(4 * (pf_pk_base(D, t1) - baseO + pf_G(n - t1 - 2, a2))) +
                           4u * (unsigned)(imax(1, lc - (lev + 3 + t1)) - 1));
        }
        for (int h2 = hmax; h2 >= h_lo; h2 -= U) {  // U steps per iteration, as in part A
            int vb[U], va[U][PF_PP_S], hh[U];
#pragma unroll
            for (int u = 0; u < U; ++u) hh[u] = imax(h2 - u, h_lo);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int h = hh[u];
                vb[u] = bld32(srcT, 4 * (imax(1, imin(lc - h - lev - 2, mT - h)) - 1), 4 * (a2 * MT + pf_G(mT, h)));
#pragma unroll
                for (int s = 0; s < PF_PP_S; ++s) {
                    const int t1 = imin(o0 + s, o0 + ns - 1), hc = imin(h, t1);
                    va[u][s] = bld32(srcO, voA[s], (t1 - hc) * Ms4[s]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool live = h2 - u >= h_lo;
#pragma unroll
                for (int s = 0; s < PF_PP_S; ++s) add(s, imul_wrap(va[u][s], vb[u]), live && s < ns && hh[u] <= o0 + s);
            }
        }
#pragma unroll
        for (int s = 0; s < PF_PP_S; ++s) {
            const int sg = lev + 3 + o0 + s;
            const int i = l - sg;
            if (s < ns && l <= n && i >= 1) {
                if (acc[s]) atomicAdd((unsigned long long *)&D.Pacc[sg * rs + i], (unsigned long long)acc[s]);
                if (aab[s]) atomicAdd(&D.Pabs[sg * rs + i], aab[s]);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// The 2-D values of span s, one wave per interval (i, j = i+s).  Every sum keeps the reference's
// term order and association: the lanes evaluate up to 64 terms at once (the products, each as
// written), then the sum adds them one after another in the reference's order (lane u's term
// read back with readlane), so the bits equal the reference's serial loop.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double rdlane(double x, int u) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, u);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), u);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// acc += term(0) + term(1) + ... + term(N-1), added in that order; term(q) evaluated by lane q % 64
template <class F>
__device__ __forceinline__ double ordered_sum(double acc, int N, int lane, F term) {
    for (int q0 = 0; q0 < N; q0 += 64) {
        const int q = q0 + lane;
        const double x = q < N ? term(q) : 0.0;
        const int cnt = imin(64, N - q0);
        for (int u = 0; u < cnt; ++u) acc += rdlane(x, u);
    }
    return acc;
}

// The same ordered sum with the terms of PF_DR rounds (PF_DR x 64 terms) evaluated first, so
// their loads are in flight together; then the serial additions in term order (identical bits).
#ifndef CCJ_PF_DR
#define CCJ_PF_DR 8
#endif
constexpr int PF_DR = CCJ_PF_DR;
template <class F>
__device__ __forceinline__ double ordered_sum_deep(double acc, int N, int lane, F term) {
    for (int q0 = 0; q0 < N; q0 += 64 * PF_DR) {
        double x[PF_DR];
#pragma unroll
        for (int r = 0; r < PF_DR; ++r) {
            const int q = q0 + r * 64 + lane;
            x[r] = q < N ? term(q) : 0.0;
        }
#pragma unroll
        for (int r = 0; r < PF_DR; ++r) {
            const int base = q0 + r * 64;
            const int cnt = imin(64, N - base);
            for (int u = 0; u < cnt; ++u) acc += rdlane(x[r], u);
        }
    }
    return acc;
}

__global__ __launch_bounds__(64) void k_pf_diag(PfDev D, int s) {
    const PfG G{D};
    const PfExp &E = *D.E;
    const int i = blockIdx.x + 1, j = i + s, n = D.n;
    if (j > n) return;  // whole wave
    const int lane = threadIdx.x;
    const int rs = D.rs;
    const int ij = s * rs + i;
    const int dang = D.dangles == 1 || D.dangles == 2;
    const short *S = D.S, *S1 = D.S1;

    // compute_energy (part_func.cc:290-300): V = hairpin + interior loops + VM
    double v_ij;
    {
        // compute_internal :222-240: k = i+1..max_k, l = j-1 down to min_l, as ONE ordered sum over
        // the flattened (k, l) terms (k-major; for k = i+1+kk there are s-1-c0-kk of them,
        // c0 = max(TURN+1, s-MAXLOOP-2)), so every term's loads go out before the serial additions
        const int max_k = imin(j - TURN - 2, i + MAXLOOP + 1);
        const int tc = G.pt(i, j);
        const int c0 = imax(TURN + 1, s - MAXLOOP - 2), nkk = imax(0, max_k - i), c1 = s - 1 - c0;
        int nterm = 0;
        for (int kk = 0; kk < nkk && c1 - kk > 0; ++kk) nterm += c1 - kk;
        const double vi = ordered_sum_deep(0.0, nterm, lane, [&](int q) {
            int kk = 0;
            while (q >= c1 - kk) { q -= c1 - kk; ++kk; }
            const int k = i + 1 + kk, l = j - 1 - q;
            double x = G.d2(D.V, k, l) *
                       exp_E_IntLoop_pf(E, k - i - 1, j - l - 1, tc, D.rtype[G.pt(k, l)], S1[i + 1], S1[j - 1], S1[k - 1], S1[l + 1]);
            x *= 1.0;  // scale[u1+u2+2]
            return x;
        });
        // compute_energy_VM :276-288, exp_Mbloop :203-212; three terms per k, in order
        const int tt = D.pair[S[j] * 8 + S[i]];
        const double mb = dang ? exp_E_MLstem_pf(E, tt, j < n ? S[j - 1] : -1, i > 1 ? S[i + 1] : -1) : exp_E_MLstem_pf(E, tt, -1, -1);
        const int nk = imax(0, j - TURN - 1 - i);  // k = i+1 .. j-TURN-1
        double vm = ordered_sum_deep(0.0, 3 * nk, lane, [&](int q) {
            const int k = i + 1 + q / 3, w = q % 3;
            const double wmp = G.g2(D.WMp, k, j - 1);
            if (w == 0) return G.g2(D.WM, i + 1, k - 1) * G.g2(D.WMv, k, j - 1) * mb * E.MLclosing;
            if (w == 1) return G.g2(D.WM, i + 1, k - 1) * wmp * mb * E.MLclosing;
            return D.mlb[k - i - 1] * wmp * mb * E.MLclosing;
        });
        vm *= 1.0;  // scale[2]
        double v = 0;
        v += D.hp[ij];
        v += vi;
        v += vm;
        if (lane == 0) {
            D.VM[ij] = vm;
            D.V[ij] = v;
        }
        v_ij = v;
    }
    // compute_pk_energies (:302-309): P (summed by k_pf_pterm), WBP, WPP
    const double p = (double)D.Pacc[ij];
    if (lane == 0) D.P[ij] = p;
    const int nd = j - i;  // d = i .. j-1, two terms each
    double wbp;
    {   // compute_WBP :361-370
        double c = ordered_sum_deep(0.0, 2 * nd, lane, [&](int q) {
            const int d = i + q / 2;
            if ((q & 1) == 0) return (d == i ? v_ij : G.d2(D.V, d, j)) * E.bp * E.PPS;
            return (d == i ? p : G.d2(D.P, d, j)) * E.PSM * E.PPS;
        });
        c += G.g2(D.WBP, i, j - 1) * D.cpp[1];
        wbp = c;
        if (lane == 0) D.WBP[ij] = c;
    }
    {   // compute_WPP :372-381 (its last term reads WBP)
        double w = ordered_sum_deep(0.0, 2 * nd, lane, [&](int q) {
            const int d = i + q / 2;
            const double wp = G.WP(i, d - 1);
            if ((q & 1) == 0) return wp * (d == i ? v_ij : G.d2(D.V, d, j)) * 1.0 * E.PPS;
            return wp * (d == i ? p : G.d2(D.P, d, j)) * E.PSP * E.PPS;
        });
        w += G.g2(D.WBP, i, j - 1) * D.pup[1];
        if (lane == 0) D.WPP[ij] = w;
    }
    (void)wbp;
    // compute_WMv_WMp (:242-256), exp_MLstem :192-201
    const int tij = G.pt(i, j);
    const double mls_ij = dang ? exp_E_MLstem_pf(E, tij, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1) : exp_E_MLstem_pf(E, tij, -1, -1);
    if (!(j - i - 1 < TURN) && lane == 0) {
        double wv = 0, wp = 0;
        wv += v_ij * mls_ij;
        wp += p * E.PSM * E.b;
        wv += G.d2(D.WMv, i, j - 1) * D.mlb[1];
        wp += G.d2(D.WMp, i, j - 1) * D.mlb[1];
        D.WMv[ij] = wv;
        D.WMp[ij] = wp;
    }
    // compute_energy_WM (:258-274): k = i .. j-TURN-1, four terms each
    if (!(j - i + 1 < 4)) {
        const int nk = j - TURN - i;
        double c = ordered_sum_deep(0.0, 4 * nk, lane, [&](int q) {
            const int k = i + q / 4, w = q % 4;
            const int tk = G.pt(k, j);
            const double mls = k == i ? mls_ij
                                      : (dang ? exp_E_MLstem_pf(E, tk, k > 1 ? S[k - 1] : -1, j < n ? S[j + 1] : -1)
                                              : exp_E_MLstem_pf(E, tk, -1, -1));
            const double q1 = (k == i ? v_ij : G.d2(D.V, k, j)) * mls;
            const double q2 = (k == i ? p : G.d2(D.P, k, j)) * E.PSM * E.b;
            const double wm = G.g2(D.WM, i, k - 1);
            if (w == 0) return D.mlb[k - i] * q1;
            if (w == 1) return D.mlb[k - i] * q2;
            if (w == 2) return wm * q1;
            return wm * q2;
        });
        c += G.d2(D.WM, i, j - 1) * D.mlb[1];
        if (lane == 0) D.WM[ij] = c;
    }
}

// ---------------------------------------------------------------------------------------------
// The 21 recurrences of one 4-D cell, in the reference's order (compute_pk_energies :315-355).
// One lane per cell of level t; blockIdx.y = a = j-i, so every loop bound and every neighbour's
// level / block is wave-uniform.  A neighbour X at (level t-dt, block a-da, row h+dh, position
// i+di) is, as in the MFE level kernel,
//     d4[ lb' + x C' + (a-da) M' + dh m' - dh(dh-1)/2 + di ]      (uniform: one scalar descriptor)
//        [ off + h (dt-dh) ]                                      (per lane; off = the cell's own offset)
// so each term costs one coalesced load on a scalar base instead of a per-lane descriptor gather.
// Each sum is still one lane's serial sum in the reference's term order and association (bits).
// The split loops run over s = d - i (or d - k):
//   X1(s) = X(i+s, j, k, l)   X2(s) = X(i, i+s, k, l)   X3(s) = X(i, j, k+s, l)   X4(s) = X(i, j, k, k+s)
// ---------------------------------------------------------------------------------------------
#ifdef CCJ_PF_LEVEL_WAVES
__attribute__((amdgpu_waves_per_eu(CCJ_PF_LEVEL_WAVES)))
#endif
__global__ __launch_bounds__(256) void k_pf_level(PfDev D, int t) {
    const PfG G{D};
    const PfExp &E = *D.E;
    const int n = D.n, a = blockIdx.y, b = t - a, m = n - t - 2, rs = D.rs;
    const PfLvl L = D.ld[t];
    const int off = blockIdx.x * 256 + threadIdx.x;
    if (off >= L.M) return;
    // row h of the a-block triangle: largest h with G(h) = h*m - h(h-1)/2 <= off
    const double bb = 2.0 * m + 1.0;
    int h = (int)((bb - sqrt(bb * bb - 8.0 * off)) * 0.5);
    if (h < 0) h = 0;
    while (h > 0 && h * m - ((h * (h - 1)) >> 1) > off) --h;
    while ((h + 1) * m - (((h + 1) * h) >> 1) <= off) ++h;
    const int i = off - (h * m - ((h * (h - 1)) >> 1)) + 1, j = i + a, k = j + h + 2, l = k + b;
    int *cell = D.d4 + L.lb + (long long)a * L.M + off;
    const long long C = L.C, off0 = (long long)a * L.M + off;  // off0: the cell in R's planes
    const double *Rt = D.R + (t & 1) * D.Rst;                   // k_pf_iloop(t)'s buffer
    auto put = [&](int x, double v) -> int {
        const int r = x86_trunc(v);
        cell[x * C] = r;
        return r;
    };
    // matrix x at (t-dt, a-da, h+dh, i+di); the caller checks that the cell exists (a-da, b-db >= 0)
    typedef const __attribute__((address_space(1))) int gint;
    auto X = [&](int x, int dt, int da, int dh, int di) -> int {
        const int tp = t - dt, mp = m + dt;
        const PfLvl Lp = D.ld[tp];
        const long long U = Lp.lb + (long long)x * Lp.C + (long long)(a - da) * Lp.M + (long long)dh * mp -
                            (((long long)dh * (dh - 1)) >> 1) + di;
        return *(gint *)(D.d4 + U + (off + h * (dt - dh)));
    };
    auto X1 = [&](int x, int s) { return X(x, s, s, 0, s); };              // X(i+s, j, k, l)
    auto X2 = [&](int x, int s) { return X(x, a - s, a - s, a - s, 0); };  // X(i, i+s, k, l)
    auto X3 = [&](int x, int s) { return X(x, s, 0, s, 0); };              // X(i, j, k+s, l)
    auto X4 = [&](int x, int s) { return X(x, b - s, 0, 0, 0); };          // X(i, j, k, k+s)
    // get_WB / get_WP (part_func.cc:701-715) of in-range intervals: expcp_pen[len] + WBP
    const double *cpp = D.cpp, *pup = D.pup, *WBP = D.WBP, *WPP = D.WPP;
    auto WBi = [&](int s) { return cpp[s] + WBP[(s - 1) * rs + i]; };                   // WB(i, i+s-1)
    auto WBj = [&](int s) { return cpp[a - s] + WBP[(a - s - 1) * rs + i + s + 1]; };   // WB(i+s+1, j)
    auto WBk = [&](int s) { return cpp[s] + WBP[(s - 1) * rs + k]; };                   // WB(k, k+s-1)
    auto WBl = [&](int s) { return cpp[b - s] + WBP[(b - s - 1) * rs + k + s + 1]; };   // WB(k+s+1, l)
    auto WPi = [&](int s) { return pup[s] + WPP[(s - 1) * rs + i]; };
    auto WPj = [&](int s) { return pup[a - s] + WPP[(a - s - 1) * rs + i + s + 1]; };
    auto WPk = [&](int s) { return pup[s] + WPP[(s - 1) * rs + k]; };
    auto WPl = [&](int s) { return pup[b - s] + WPP[(b - s - 1) * rs + k + s + 1]; };
    auto BPi = [&](int s) { return WBP[(s - 1) * rs + i]; };                            // WBP(i, i+s-1)
    auto BPj = [&](int s) { return WBP[(a - s - 1) * rs + i + s + 1]; };                // WBP(i+s+1, j)
    auto BPk = [&](int s) { return WBP[(s - 1) * rs + k]; };
    auto BPl = [&](int s) { return WBP[(b - s - 1) * rs + k + s + 1]; };
    const double bp = E.bp, ap = E.ap, cp1 = D.cpp[1], PB = E.PB;

    // The split loops of all 20 non-interior recurrences fused into one loop over the (i,j) gap
    // (s = d-i) and one over the (k,l) gap (s = d-k): each neighbour value is loaded once for every
    // sum that reads it.  Each sum is its own accumulator and receives its terms in exactly the
    // reference's order (a sum's (i,j)-gap terms all precede its (k,l)-gap terms, as in its code).
    double cLm00 = 0, cLm01 = 0, cLm10 = 0, cMm00 = 0, cMm10 = 0, cOm00 = 0, cOm10 = 0;
    double cFL = 0, cFM = 0, cFO = 0, cK = 0;
    double cRm00 = 0, cRm01 = 0, cRm10 = 0, cMm01 = 0, cOm01 = 0, cFR = 0;
    cLm00 += 0.0 * bp;  // PLmloop00 (:554-568): the seed PL(i,j,k,l) is not computed yet: 0 * beta2P
    cRm00 += 0.0 * bp;  // PRmloop00 (:592-605)
    cMm00 += 0.0 * bp;  // PMmloop00 (:628-639)
    cOm00 += 0.0 * bp;  // POmloop00 (:665-676)
    cRm01 += (b >= 1 ? X(PF_PRmloop01, 1, 0, 0, 0) : 0) * cp1;  // PRmloop01(i,j,k,l-1) * expcp_pen[1] (:608-616)
    cRm10 += (b >= 1 ? X(PF_PRmloop10, 1, 0, 1, 0) : 0) * cp1;  // PRmloop10(i,j,k+1,l) * expcp_pen[1] (:618-626)
    cMm01 += (b >= 1 ? X(PF_PMmloop01, 1, 0, 1, 0) : 0) + cp1;  // PMmloop01(i,j,k+1,l) "+ expcp_pen[1]" (:642-650)
    cMm10 += (a >= 1 ? X(PF_PMmloop10, 1, 1, 1, 0) : 0) * cp1;  // PMmloop10(i,j-1,k,l) * expcp_pen[1] (:652-663)
    // 4-D operand of a split step: matrix x at (t-dt, a-da, h+dh, i+di), descriptor by scalar load
    auto Xs = [&](const PfLvlS &Lp, int x, int dt, int da, int dh, int di) -> int {
        const int mp = m + dt;
        const long long U = Lp.lb + (long long)x * Lp.C + (long long)(a - da) * Lp.M + (long long)dh * mp -
                            (((long long)dh * (dh - 1)) >> 1) + di;
        return *(gint *)(D.d4 + U + (off + h * (dt - dh)));
    };
    // (i,j) gap, d = i+s: s = 0 (the X2 terms only), s = 1 .. a-1 pipelined, s = a (the X1 terms only)
    if (a >= 1) {  // s = 0: X2 = X(i, i, k, l), WB(i+1, j) / WBP(i+1, j)
        const double bpj = BPj(0), wbj = ldc_f64(cpp + a) + bpj;
        const int lm00 = X2(PF_PLmloop00, 0);
        cLm00 += lm00 * wbj;  // :561-562
        cLm01 += lm00 * bpj;  // :574-576
        cMm00 += X2(PF_PMmloop00, 0) * wbj;  // :632-633
    }
    // split-loop operands as buffer loads: the 2-D tables from their starts (lane offset 8i / 8k),
    // the 4-D values from the start of their level (lane offset 4(off + h*(dt-dh)))
    const __amdgpu_buffer_rsrc_t rWBP = pf_rsrc(WBP), rWPP = pf_rsrc(WPP);
    const int vi8 = 8 * i, vk8 = 8 * k, rs8 = 8 * rs;
    struct SA { double bpi, wppi, bpj, wppj; int lm1, mm1, om1, fl1, fo1, lm2, l102, mm2, fl2, fm2, k2, s; };
    auto ldA = [&](int s) {
        SA v;
        v.s = s;
        const PfLvlS L1 = ldc_lvl(D.ld + t - s), L2 = ldc_lvl(D.ld + b + s);
        const int oi = (s - 1) * rs8, oj = (a - s - 1) * rs8 + 8 * (s + 1);
        v.bpi = bld64(rWBP, vi8, oi);
        v.bpj = bld64(rWBP, vi8, oj);
        v.wppi = bld64(rWPP, vi8, oi);
        v.wppj = bld64(rWPP, vi8, oj);
        // X1 = X(i+s, j, k, l) = (t-s, a-s, h, i+s): its r1 record, record (a-s)M + s + lane (off + h s)
        const __amdgpu_buffer_rsrc_t r1 = pf_rsrc(D.r1 + PF_REC1 * L1.lr);
        const int s1 = 4 * PF_REC1 * ((a - s) * L1.M + s), v1 = 4 * PF_REC1 * (off + h * s);
        const pfu3 p1 = bld96(r1, v1, s1);
        const pfu2 q1 = bld64u(r1, v1, s1 + 12);
        v.lm1 = (int)p1.x;
        v.mm1 = (int)p1.y;
        v.om1 = (int)p1.z;
        v.fl1 = (int)q1.x;
        v.fo1 = (int)q1.y;
        // X2 = X(i, i+s, k, l) = (b+s, s, h+a-s, i): its r2 record, record s M + G(a-s) + lane off
        const __amdgpu_buffer_rsrc_t r2 = pf_rsrc(D.r2 + PF_REC2 * L2.lr);
        const int dh = a - s, s2 = 4 * PF_REC2 * (s * L2.M + dh * (m + dh) - ((dh * (dh - 1)) >> 1)), v2 = 4 * PF_REC2 * off;
        const pfu3 p2 = bld96(r2, v2, s2), q2 = bld96(r2, v2, s2 + 12);
        v.lm2 = (int)p2.x;
        v.l102 = (int)p2.y;
        v.mm2 = (int)p2.z;
        v.fl2 = (int)q2.x;
        v.fm2 = (int)q2.y;
        v.k2 = (int)q2.z;
        return v;
    };
    auto rdA = [&](const SA &v) {
        const int s = v.s;
        const double bpi = v.bpi, wbi = ldc_f64(cpp + s) + bpi;  // WB(i, i+s-1) / WBP(i, i+s-1)
        cLm00 += wbi * v.lm1;  // :558-560
        cLm10 += bpi * v.lm1;  // :582-584
        cMm10 += bpi * v.mm1;  // :656-658
        cOm00 += wbi * v.om1;  // :669-670
        cOm10 += bpi * v.om1;  // :690-692
        const double bpj = v.bpj, wbj = ldc_f64(cpp + (a - s)) + bpj;  // WB(i+s+1, j) / WBP(i+s+1, j)
        cLm00 += v.lm2 * wbj;   // :561-562
        cLm01 += v.lm2 * bpj;   // :574-576
        cLm10 += v.l102 * wbj;  // :585-587
        cMm00 += v.mm2 * wbj;   // :632-633
        // PfromL / PfromM / PfromO / PK: d = i+1 .. j-1, WP(i, d-1), WP(d+1, j)
        const double wpi = ldc_f64(pup + s) + v.wppi, wpj = ldc_f64(pup + (a - s)) + v.wppj;
        cFL += v.fl1 * wpi;  // :491-493
        cFL += v.fl2 * wpj;
        cFM += v.fm2 * wpj;  // :523-524
        cFO += v.fo1 * wpi;  // :540-541
        cK += v.k2 * wpj;    // :398-399
    };
    pf_pipe<SA>(1, a - 1, ldA, rdA);
    if (a >= 1) {  // s = a: X1 = X(j, j, k, l), WB(i, j-1) / WBP(i, j-1)
        const double bpi = BPi(a), wbi = ldc_f64(cpp + a) + bpi;
        const int lm00 = X1(PF_PLmloop00, a), mm00 = X1(PF_PMmloop00, a), om00 = X1(PF_POmloop00, a);
        cLm00 += wbi * lm00;  // :558-560
        cLm10 += bpi * lm00;  // :582-584
        cMm10 += bpi * mm00;  // :656-658
        cOm00 += wbi * om00;  // :669-670
        cOm10 += bpi * om00;  // :690-692
    }
    if (b >= 1) cOm00 = X(PF_POmloop00, 1, 0, 0, 0) * (cpp[1] + WBP[l]);  // :671-673: assigns POmloop00(i,j,k,l-1) * WB(l,l)
    // (k,l) gap, d = k+s: s = 0 (the X4 terms only), s = 1 .. b-1 pipelined, s = b (the X3 terms only)
    if (b >= 1) {  // s = 0: X4 = X(i, j, k, k), WB(k+1, l) / WBP(k+1, l)
        const double bpl = BPl(0), wbl = ldc_f64(cpp + b) + bpl;
        const int rm00 = X4(PF_PRmloop00, 0);
        cRm00 += rm00 * wbl;                   // :599-600
        cRm01 += rm00 * bpl;                   // :612-614
        cMm01 += X4(PF_PMmloop00, 0) * bpl;    // :646-648
        cOm01 += X4(PF_POmloop00, 0) * bpl;    // :682-684
    }
    struct SB { double bpk, wppk, bpl, wppl; int rm3, mm3, fr3, fm3, k3, rm4, mm4, om4, o104, fr4, fo4, s; };
    auto ldB = [&](int s) {
        SB v;
        v.s = s;
        const PfLvlS L3 = ldc_lvl(D.ld + t - s), L4 = ldc_lvl(D.ld + a + s);
        const int ok = (s - 1) * rs8, ol = (b - s - 1) * rs8 + 8 * (s + 1);
        v.bpk = bld64(rWBP, vk8, ok);
        v.bpl = bld64(rWBP, vk8, ol);
        v.wppk = bld64(rWPP, vk8, ok);
        v.wppl = bld64(rWPP, vk8, ol);
        // X3 = X(i, j, k+s, l) = (t-s, a, h+s, i): its r3 record, record a M + G(s) at m+s + lane off
        const __amdgpu_buffer_rsrc_t r3 = pf_rsrc(D.r3 + PF_REC3 * L3.lr);
        const int s3 = 4 * PF_REC3 * (a * L3.M + s * (m + s) - ((s * (s - 1)) >> 1)), v3 = 4 * PF_REC3 * off;
        const pfu3 p3 = bld96(r3, v3, s3);
        const pfu2 q3 = bld64u(r3, v3, s3 + 12);
        v.rm3 = (int)p3.x;
        v.mm3 = (int)p3.y;
        v.fr3 = (int)p3.z;
        v.fm3 = (int)q3.x;
        v.k3 = (int)q3.y;
        // X4 = X(i, j, k, k+s) = (a+s, a, h, i): its r4 record, record a M + lane (off + h (b-s))
        const __amdgpu_buffer_rsrc_t r4 = pf_rsrc(D.r4 + PF_REC4 * L4.lr);
        const int s4 = 4 * PF_REC4 * (a * L4.M), v4 = 4 * PF_REC4 * (off + h * (b - s));
        const pfu3 p4 = bld96(r4, v4, s4), q4 = bld96(r4, v4, s4 + 12);
        v.rm4 = (int)p4.x;
        v.mm4 = (int)p4.y;
        v.om4 = (int)p4.z;
        v.o104 = (int)q4.x;
        v.fr4 = (int)q4.y;
        v.fo4 = (int)q4.z;
        return v;
    };
    auto rdB = [&](const SB &v) {
        const int s = v.s;
        const double bpk = v.bpk, wbk = ldc_f64(cpp + s) + bpk;  // WB(k, k+s-1) / WBP(k, k+s-1)
        cRm00 += wbk * v.rm3;  // :596-598
        cRm10 += bpk * v.rm3;  // :622-624
        cMm00 += v.mm3 * wbk;  // :634-636
        const double bpl = v.bpl, wbl = ldc_f64(cpp + (b - s)) + bpl;  // WB(k+s+1, l) / WBP(k+s+1, l)
        cRm00 += v.rm4 * wbl;  // :599-600
        cRm01 += v.rm4 * bpl;  // :612-614
        cMm01 += v.mm4 * bpl;  // :646-648
        cOm01 += v.om4 * bpl;  // :682-684
        // d = k+1 .. l-1
        const double wpk = ldc_f64(pup + s) + v.wppk, wpl = ldc_f64(pup + (b - s)) + v.wppl;
        cMm10 += v.o104 * wbl;  // :659-661
        cOm10 += v.o104 + wbl;  // :693-695 ("+ get_WB")
        cFR += v.fr3 * wpk;     // :508-510
        cFR += v.fr4 * wpl;
        cFM += v.fm3 * wpk;     // :526-527
        cFO += v.fo4 * wpl;     // :544-545
        cK += v.k3 * wpk;       // :401-402
    };
    pf_pipe<SB>(1, b - 1, ldB, rdB);
    if (b >= 1) {  // s = b: X3 = X(i, j, l, l), WB(k, l-1) / WBP(k, l-1)
        const double bpk = BPk(b), wbk = ldc_f64(cpp + b) + bpk;
        const int rm00 = X3(PF_PRmloop00, b);
        cRm00 += wbk * rm00;                   // :596-598
        cRm10 += bpk * rm00;                   // :622-624
        cMm00 += X3(PF_PMmloop00, b) * wbk;    // :634-636
    }
    // The rest of the cell reads pair types, the level t-2 neighbours of the stack terms and
    // k_pf_iloop's sums, none of which depends on the sums above: issue every load before the first
    // store (gfx950's vmcnt counts loads and stores in order, so a load behind a store waits for it),
    // then evaluate PL, PR, PM, PO exactly as before.
    const int ptij = G.pt(i, j), ptkl = G.pt(k, l), ptjk = G.pt(j, k), ptil = G.pt(i, l);
    const PfLvlS L2 = ldc_lvl(D.ld + (t >= 2 ? t - 2 : 0));
    // PL: inner cell (i+1, j-1, k, l) = (t-2, a-2, h+1, i+1), outside the matrix (0) when a < 2
    const bool inL = a >= 2;
    const int xL = (inL && a < 6) ? Xs(L2, PF_PL, 2, 2, 1, 1) : 0;
    const int xLm10 = inL ? Xs(L2, PF_PLmloop10, 2, 2, 1, 1) : 0, xLm01 = inL ? Xs(L2, PF_PLmloop01, 2, 2, 1, 1) : 0;
    const int xFL = inL ? Xs(L2, PF_PfromL, 2, 2, 1, 1) : 0;
    const double rL = a >= 6 ? Rt[off0] : 0.0, eL = a < 6 ? D.est[a * rs + i] : 0.0;
    // PR: (i, j, k+1, l-1) = (t-2, a, h+1, i), outside when b < 2
    const bool inR = b >= 2;
    const int xR = (inR && b < 6) ? Xs(L2, PF_PR, 2, 0, 1, 0) : 0;
    const int xRm10 = inR ? Xs(L2, PF_PRmloop10, 2, 0, 1, 0) : 0, xRm01 = inR ? Xs(L2, PF_PRmloop01, 2, 0, 1, 0) : 0;
    const int xFR = inR ? Xs(L2, PF_PfromR, 2, 0, 1, 0) : 0;
    const double rR = b >= 6 ? Rt[C + off0] : 0.0, eR = b < 6 ? D.est[b * rs + k] : 0.0;
    // PM: (i, j-1, k+1, l) = (t-2, a-1, h+2, i), outside when a < 1 or b < 1
    const bool inM = a >= 1 && b >= 1, winM = a >= 2 && b >= 2;
    const int xM = (inM && !winM) ? Xs(L2, PF_PM, 2, 1, 2, 0) : 0;
    const int xMm10 = inM ? Xs(L2, PF_PMmloop10, 2, 1, 2, 0) : 0, xMm01 = inM ? Xs(L2, PF_PMmloop01, 2, 1, 2, 0) : 0;
    const int xFM = inM ? Xs(L2, PF_PfromM, 2, 1, 2, 0) : 0;
    // get_e_stP(j-1, k+1): for j == 1 or k == n the reference indexes pair[][] with S[0] (= n) or
    // S[n+1]; the factor multiplies PM(i, j-1, k+1, l), which is then outside the matrix (0), so
    // any finite value gives 0 — use 0 instead of reading past the table
    const double rM = winM ? Rt[2 * C + off0] : 0.0, eM = (!winM && j > 1 && k < n) ? D.est[(h + 4) * rs + (j - 1)] : 0.0;
    // PO: (i+1, j, k, l-1) = (t-2, a-1, h, i+1), outside when a < 1 or b < 1
    const int xO = inM ? Xs(L2, PF_PO, 2, 1, 0, 1) : 0;
    const int xOm10 = inM ? Xs(L2, PF_POmloop10, 2, 1, 0, 1) : 0, xOm01 = inM ? Xs(L2, PF_POmloop01, 2, 1, 0, 1) : 0;
    const int xFO = inM ? Xs(L2, PF_PfromO, 2, 1, 0, 1) : 0;
    const double eO = D.est[(t + h + 2) * rs + i];

    const int sLm00 = put(PF_PLmloop00, cLm00);
    put(PF_PLmloop01, cLm01);
    const int sLm10 = put(PF_PLmloop10, cLm10);
    const int sRm00 = put(PF_PRmloop00, cRm00);
    put(PF_PRmloop01, cRm01);
    put(PF_PRmloop10, cRm10);
    const int sMm00 = put(PF_PMmloop00, cMm00);
    put(PF_PMmloop01, cMm01);
    put(PF_PMmloop10, cMm10);
    const int sOm00 = put(PF_POmloop00, cOm00);
    put(PF_POmloop01, cOm01);
    const int sOm10 = put(PF_POmloop10, cOm10);

    // PL (:414-430) with get_PLiloop (:736-756) and get_PLmloop (:758-768)
    int PL = 0;
    {
        double c = 0;
        if (ptij > 0) {
            double r = 0;
            if (a >= 6) r = rL;  // k_pf_iloop: the stack term, then the window
            else r += xL * eL;   // no window (u2 <= a-u1-6)
            c += r;
            double q = 0;
            q += xLm10 * ap * bp;
            q += (double)imul_wrap(xLm01, D.ap_int) * bp;
            c += q * bp;
            if (j >= i + TURN + 1) c += xFL * 1.0;
        }
        PL = put(PF_PL, c);
        if (ptij > 0) D.cx[L.lbx + a * L.M + (i - 1) * m - (((i - 1) * (i - 2)) >> 1) + h] = PL;
    }
    // PR (:432-447), get_PRiloop (:770-790), get_PRmloop (:792-802)
    int PR = 0;
    {
        double c = 0;
        if (ptkl > 0) {
            double r = 0;
            if (b >= 6) r = rR;
            else r += xR * eR;
            c += r;
            double q = 0;
            q += xRm10 * ap * bp;
            q += xRm01 * ap * bp;
            c += q * bp;
            if (l >= k + TURN + 1) c += xFR * 1.0;
        }
        PR = put(PF_PR, c);
        const int q = i + h - 1;
        if (ptkl > 0) D.cx[L.lbx + C + a * L.M + ((q * (q + 1)) >> 1) + i - 1] = PR;
    }
    // PM (:449-467), get_PMiloop (:804-824), get_PMmloop (:826-836)
    int PM = 0;
    {
        double c = 0;
        if (ptjk > 0) {
            double r = 0;
            if (winM) r = rM;
            else r += xM * eM;
            c += r;
            double q = 0;
            q += xMm10 * ap * bp;
            q += xMm01 * ap * bp;
            c += q * bp;
            if (k >= j + TURN - 1) c += xFM * 1.0;
            if (i == j && k == l) c += 1.0;
        }
        PM = put(PF_PM, c);
        if (ptjk > 0) D.pmx[L.pmb + ((long long)h * n + j - 1) * (t + 1) + a] = PM;
    }
    // PO (:469-486), get_POiloop (:838-858: reads PO(d,j,dp,k) with dp > k, always 0), get_POmloop
    int PO = 0;
    {
        double c = 0;
        if (ptil > 0) {
            double r = 0;
            r += xO * eO;
            c += r;
            double q = 0;
            q += xOm10 * ap * bp;
            q += xOm01 * ap * bp;
            c += q * bp;
            if (l >= i + TURN + 1) c += xFO * 1.0;
        }
        PO = put(PF_PO, c);
    }
    int sFL, sFR, sFM, sFO, sK;
    {  // PfromL (:488-503): split terms above, then the same-cell P* terms
        double c = cFL;
        c += PR * 1.0 * PB;
        c += PM * 1.0 * PB;
        c += PO * 1.0 * PB;
        sFL = put(PF_PfromL, c);
    }
    {  // PfromR (:505-518)
        double c = cFR;
        c += PM * 1.0 * PB;
        c += PO * 1.0 * PB;
        sFR = put(PF_PfromR, c);
    }
    {  // PfromM (:520-535)
        double c = cFM;
        c += PL * 1.0 * PB;
        c += PR * 1.0 * PB;
        sFM = put(PF_PfromM, c);
    }
    {  // PfromO (:537-552)
        double c = cFO;
        c += PL * 1.0 * PB;
        c += PR * 1.0 * PB;
        sFO = put(PF_PfromO, c);
    }
    {  // PK (:395-412)
        double c = cK;
        c += PL * 1.0 * PB;
        c += PM * 1.0 * PB;
        c += PR * 1.0 * PB;
        c += PO * 1.0 * PB;
        sK = put(PF_PK, c);
    }
    // the cell's split-loop records (ccj_pf_engine.h PfDev::r1 .. r4), read by later levels
    const long long rc = L.lr + off0;
    int *w1 = D.r1 + PF_REC1 * rc, *w2 = D.r2 + PF_REC2 * rc, *w3 = D.r3 + PF_REC3 * rc, *w4 = D.r4 + PF_REC4 * rc;
    w1[0] = sLm00; w1[1] = sMm00; w1[2] = sOm00; w1[3] = sFL; w1[4] = sFO;
    w2[0] = sLm00; w2[1] = sLm10; w2[2] = sMm00; w2[3] = sFL; w2[4] = sFM; w2[5] = sK;
    w3[0] = sRm00; w3[1] = sMm00; w3[2] = sFR; w3[3] = sFM; w3[4] = sK;
    w4[0] = sRm00; w4[1] = sMm00; w4[2] = sOm00; w4[3] = sOm10; w4[4] = sFR; w4[5] = sFO;
}

// ---------------------------------------------------------------------------------------------
// Interior-loop sums of level t (get_PLiloop :736-756, get_PRiloop :770-790, get_PMiloop :804-824),
// one wave per work item of ccj_items.h (a closing pair and up to 64 of the cells it closes):
//   PL  pair (i, j = i+a), lanes h      PL(d, dp, k, l)  = PLx(t-dt, a-dt, h+1+u2, d)
//   PR  pair (k, l = k+b), lanes i      PR(i, j, d, dp)  = PRx(t-dt, a, h+1+u1, i)
//   PM  pair (j, k),       lanes a      PM(i, d, dp, l)  = PMx(t-dt, h+dt, d, a-1-u1)
// (dt = 2+u1+u2).  In each copy the lanes of one term read consecutive words; the weights of one
// pair's window are contiguous (ieO / ieI) and wave-uniform, so they come through scalar loads.
// r = stack term, then the window terms in the reference's (u1, u2) order; the copies hold 0 where
// the inner pair cannot pair (the 4-D value there is 0).  A term whose weight is 0.0 or whose inner
// pair cannot pair adds a zero: per-pair bit masks (mO / mI) skip those loads altogether.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t low_bits(int u) { return u < 0 ? 0u : (2u << u) - 1u; }  // bits 0..u (u <= 30)

// readlane of a 64-bit value (lane l wave-uniform)
__device__ __forceinline__ long long rdl64(long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned long long)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// r + w_k * x(u2_k) for the set bits u2_0 < u2_1 < ... of mk (the reference's u2 order), where lane
// predicate on(u2) holds.  w = the row's weights compacted to the mask's set bits (ccj_pf.cc), so a
// round's weights are one scalar load; up to 8 terms per round, their loads in flight together.
template <class LDX, class P>
__device__ __forceinline__ double window_row(double r, uint32_t mk, const double *w, LDX ldx, P on) {
    for (int k = 0; mk; k += PF_ILW) {
        int q[PF_ILW];
        bool v[PF_ILW];
        q[0] = __builtin_ctz(mk);
        v[0] = true;
        mk &= mk - 1;
#pragma unroll
        for (int e = 1; e < PF_ILW; ++e) {
            v[e] = mk != 0;
            q[e] = v[e] ? __builtin_ctz(mk) : q[0];
            mk &= mk - 1;
        }
        int x[PF_ILW];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = ldx(q[e]);
#pragma unroll
        for (int g = 4; g < PF_ILW; g += 4) {  // the round's later quarters only when they hold a term
            if (v[g]) {
#pragma unroll
                for (int e = g; e < g + 4; ++e) x[e] = ldx(q[e]);
            } else {
#pragma unroll
                for (int e = g; e < g + 4; ++e) x[e] = 0;
            }
        }
        double wv[PF_ILW];
#pragma unroll
        for (int e = 0; e < PF_ILW; ++e) wv[e] = w[k + e];
#pragma unroll
        for (int e = 0; e < PF_ILW; ++e)
            if (v[e] && on(q[e])) r += wv[e] * x[e] * 1.0;
    }
    return r;
}

// The partner of candidate (u1, u2) (dt = 2+u1+u2, source level t-dt) is one int per lane at
//   row(u1)[dt] + lane offset,
// where row(u1)[dt] (a pointer) sits in lane dt of a per-wave table: the level's block base from its
// descriptor (once per wave) plus the u1 row's terms (once per row).  A candidate then costs two
// readlanes and one vector address add; as a dependent descriptor load plus 64-bit index arithmetic
// per candidate the kernel was bound by its scalar instruction stream.
__global__ __launch_bounds__(256) void k_pf_iloop(PfDev D, int t, long long first, int nitems) {
    const int wv = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (wv >= nitems) return;
    const int lane = threadIdx.x & 63;
    const uint32_t it = (uint32_t)__builtin_amdgcn_readfirstlane((int)D.items[first + wv]);
    const int role = (int)(it >> 30), f1 = (int)((it >> 20) & 1023), f2 = (int)((it >> 10) & 1023), ch = (int)(it & 1023);
    const int n = D.n, rs = D.rs, m = n - t - 2;
    const PfLvl L = D.ld[t];
    typedef const __attribute__((address_space(1))) int gint;
    const int *cx = D.cx, *pmx = D.pmx;
    constexpr int W2 = PF_IEW * PF_IEW;
    // lane dt: level t-dt's descriptor (dt = 2 .. t; other lanes unused)
    const bool lv = lane >= 2 && lane <= t;
    const PfLvl Ll = D.ld[lv ? t - lane : t];
    auto at = [&](const int *rowp, int dt) { return (const int *)rdl64((long long)rowp, dt); };
    double r = 0;
    long long dst;  // the cell in R
    bool act;
    if (role == 0) {  // PL: lanes h <= m-i
        const int a = f1, i = f2, j = i + a, h = ch * 64 + lane;
        act = h <= m - i;
        const int hc = act ? h : m - i;
        dst = (long long)a * L.M + hc * m - ((hc * (hc - 1)) >> 1) + i - 1;
        {   // PL(i+1, j-1, k, l) = PLx(t-2, a-2, h+1, i+1)
            const PfLvl L2 = D.ld[t - 2];
            const int x = *(gint *)(cx + L2.lbx + (long long)(a - 2) * L2.M + i * (m + 2) - ((i * (i - 1)) >> 1) + hc + 1);
            r += x * D.est[a * rs + i];
        }
        // d = i+1+u1 < min(j, i+30); dp = j-1-u2 > max(d+3, j-30): u1 <= min(a,30)-2, u2 <= min(a-u1-6, 28)
        // PLx(t-dt, a-dt, h+1+u2, d) = cx[lbx + (a-dt)M + (d-1)(m+dt) - (d-1)(d-2)/2 + hc + 1 + u2]
        const long long X = Ll.lbx + (long long)(a - lane) * Ll.M + 1 + (long long)i * lane;  // + i*dt
        const size_t pr = (size_t)a * rs + i;
        const double *ew = D.ieO + pr * W2;
        const uint32_t *mw = D.mO + pr * PF_IEW;
        const int u1m = imin(a, MAXLOOP) - 2;
        for (int u1 = 0; u1 <= u1m; ++u1) {
            const int u2m = imin(a - u1 - 6, PF_IEW - 1), d1 = i + u1;
            const uint32_t mk = mw[u1] & low_bits(u2m);
            if (!mk) continue;
            // + (i+u1)m - (i+u1)(i+u1-1)/2 + u1*dt + u2, u2 = dt-2-u1
            const int *rowp = cx + (X + (long long)d1 * m - (((long long)d1 * (d1 - 1)) >> 1) + u1 * lane + (lane - 2 - u1));
            r = window_row(r, mk, ew + u1 * PF_IEW, [&](int u2) { return *(gint *)(at(rowp, 2 + u1 + u2) + hc); },
                           [](int) { return true; });
        }
    } else if (role == 1) {  // PR: q = i+h-1 fixed, lanes i <= q+1
        const int a = f1, q = f2, b = t - a, k = q + a + 3, i = ch * 64 + lane + 1;
        act = i <= q + 1;
        const int ic = act ? i : q + 1, h = q + 1 - ic;
        dst = L.C + (long long)a * L.M + h * m - ((h * (h - 1)) >> 1) + ic - 1;
        {   // PR(i, j, k+1, l-1) = PRx(t-2, a, h+1, i): row q+1
            const PfLvl L2 = D.ld[t - 2];
            const int x = *(gint *)(cx + L2.lbx + L2.C + (long long)a * L2.M + (((q + 1) * (q + 2)) >> 1) + ic - 1);
            r += x * D.est[b * rs + k];
        }
        // PRx(t-dt, a, h+1+u1, i) = cx[lbx + C + a*M + qq(qq+1)/2 + ic - 1], qq = q+1+u1
        const long long X = Ll.lbx + Ll.C + (long long)a * Ll.M - 1;
        const size_t pr = (size_t)b * rs + k;
        const double *ew = D.ieO + pr * W2;
        const uint32_t *mw = D.mO + pr * PF_IEW;
        const int u1m = imin(b, MAXLOOP) - 2;
        for (int u1 = 0; u1 <= u1m; ++u1) {
            const int u2m = imin(b - u1 - 6, PF_IEW - 1), qq = q + 1 + u1;
            const uint32_t mk = mw[u1] & low_bits(u2m);
            if (!mk) continue;
            const int *rowp = cx + (X + ((qq * (qq + 1)) >> 1));
            r = window_row(r, mk, ew + u1 * PF_IEW, [&](int u2) { return *(gint *)(at(rowp, 2 + u1 + u2) + ic); },
                           [](int) { return true; });
        }
    } else {  // PM: pair (j, k = j+h+2), lanes a in [alo, ahi]
        const int h = f1, j = f2, k = j + h + 2;
        const int alo = imax(2, t - (n - k)), ahi = imin(t - 2, j - 1);
        const int a = alo + ch * 64 + lane;
        act = a <= ahi;
        const int ac = act ? a : ahi, i = j - ac, b = t - ac;
        dst = 2 * L.C + (long long)ac * L.M + h * m - ((h * (h - 1)) >> 1) + i - 1;
        {   // PM(i, j-1, k+1, l) = PMx(t-2, h+2, j-1, a-1); a >= 2, b >= 2 so j > 1 and k < n
            const PfLvl L2 = D.ld[t - 2];
            const int x = *(gint *)(pmx + L2.pmb + ((long long)(h + 2) * n + j - 2) * (t - 1) + ac - 1);
            r += x * D.est[(h + 4) * rs + (j - 1)];
        }
        // d = j-1-u1 > max(i, j-30), dp = k+1+u2 < min(l, k+30): u1 <= min(a-2, 28), u2 <= min(b-2, 28)
        // PMx(tp, h+dt, d, min(ap, tp)) = pmx[pmb + ((h+dt)n + j-2-u1)(tp+1) + min(ap, tp)], tp = t-dt
        const long long X = Ll.pmb + ((long long)(h + lane) * n + j - 2) * (t - lane + 1);
        const size_t pr = (size_t)(h + 2) * rs + j;
        const double *ew = D.ieI + pr * W2;
        const uint32_t *mw = D.mI + pr * PF_IEW;
        const int u1m = imin(ahi - 2, PF_IEW - 1), u2m = imin(t - alo - 2, PF_IEW - 1);
        const int u2l = b - 2;  // this lane's u2 bound
        for (int u1 = 0; u1 <= u1m; ++u1) {
            const bool on1 = u1 <= ac - 2;
            const int ap = imax(ac - 1 - u1, 0);
            const int u2e = imin(u2m, t - 4 - u1);  // a lane with u1 <= a-2 has b-2 <= t-4-u1
            const uint32_t mk = u2e >= 0 ? mw[u1] & low_bits(u2e) : 0u;
            if (!mk) continue;
            const int *rowp = pmx + (X - (long long)u1 * (t - lane + 1));
            r = window_row(r, mk, ew + u1 * PF_IEW, [&](int u2) {
                const int dt = 2 + u1 + u2;
                return *(gint *)(at(rowp, dt) + imin(ap, t - dt));
            }, [&](int u2) { return on1 && u2 <= u2l; });
        }
    }
    if (act) D.R[(t & 1) * D.Rst + dst] = r;
}

// canonical-order gather of one 4-D matrix for the parity hashes: out[q] for the q-th cell of
// i = 1..n, j = i..n, k = j+2..n, l = k..n; one thread per (i, j, k) row of l.
__global__ __launch_bounds__(256) void k_pf_canon(PfDev D, int x, const long long *__restrict__ rowoff, int nrows,
                                                 int *__restrict__ out) {
    const PfG G{D};
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrows) return;
    // decode r -> (i, j, k) in canonical order by the host-built offsets (rowoff[r] = first q)
    const long long q0 = rowoff[2 * r], ijk = rowoff[2 * r + 1];
    const int i = (int)(ijk >> 40), j = (int)((ijk >> 20) & 0xfffff), k = (int)(ijk & 0xfffff);
    for (int l = k; l <= D.n; ++l) out[q0 + (l - k)] = G.g4(x, i, j, k, l);
}

extern "C" int ccjk_pf_pterm(const PfDev *D, int s, void *stream) {
#ifdef CCJ_ABLATE_PF_PTERM
    return 0;  // timing only: this PF kernel skipped (wrong results)
#endif
    const int ni = D->n - s;
    if (s < 3 || ni <= 0) return 0;
    hipLaunchKernelGGL(k_pf_pterm, dim3((unsigned)((ni + 63) / 64), (unsigned)(s - 2), (unsigned)((s - 2 + PT_DD - 1) / PT_DD)),
                       dim3(256), 0, (hipStream_t)stream, *D, s);
    return (int)hipGetLastError();
}

// P terms whose operands' highest level is lev (k_pf_ppush); completes P(lev+3).  The grid as
// ccjk_ppush's (MFE) for one rank.
extern "C" int ccjk_pf_ppush(const PfDev *D, int lev, void *stream) {
#ifdef CCJ_ABLATE_PF_PTERM
    return 0;  // timing only: this PF kernel skipped (wrong results)
#endif
    const int n = D->n;
    const int nmax = imin(lev, n - 4 - lev) + 1;
    if (nmax <= 0) return 0;
    const int ngrp = (n - lev - 3 + 63) / 64;
    constexpr int hs_len = 32;
    const int nch = (nmax + PF_PP_S - 1) / PF_PP_S;
    int npairs = 0;
    for (int c = 0; c < nch; ++c) npairs += (imin((c + 1) * PF_PP_S, nmax) + hs_len - 1) / hs_len;
    const int blocksA = (npairs * ngrp * (lev + 1) + 3) / 4;
    // split steps in flight per wave (CCJ_PF_PP_STEPS, default 4; 2 for the A/B)
    static const int steps = getenv("CCJ_PF_PP_STEPS") ? atoi(getenv("CCJ_PF_PP_STEPS")) : 4;
    if (steps >= 4)
        hipLaunchKernelGGL((k_pf_ppush<4>), dim3((unsigned)(2 * blocksA)), dim3(256), 0, (hipStream_t)stream, *D, lev, ngrp,
                           npairs, hs_len, blocksA);
    else
        hipLaunchKernelGGL((k_pf_ppush<2>), dim3((unsigned)(2 * blocksA)), dim3(256), 0, (hipStream_t)stream, *D, lev, ngrp,
                           npairs, hs_len, blocksA);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_diag(const PfDev *D, int s, void *stream) {
#ifdef CCJ_ABLATE_PF_DIAG
    return 0;  // timing only: this PF kernel skipped (wrong results)
#endif
    const int ni = D->n - s;
    if (ni <= 0) return 0;
    hipLaunchKernelGGL(k_pf_diag, dim3((unsigned)ni), dim3(64), 0, (hipStream_t)stream, *D, s);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_level(const PfDev *D, const PfLvl *Lh, int t, void *stream) {
    const int M = Lh[t].M;
    if (M <= 0) return 0;
    hipLaunchKernelGGL(k_pf_level, dim3((unsigned)((M + 255) / 256), (unsigned)(t + 1)), dim3(256), 0, (hipStream_t)stream,
                       *D, t);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_iloop(const PfDev *D, int t, long long first, int nitems, void *stream) {
#ifdef CCJ_ABLATE_PF_ILOOP
    return 0;  // timing only: this PF kernel skipped (wrong results)
#endif
    if (nitems <= 0) return 0;
    hipLaunchKernelGGL(k_pf_iloop, dim3((unsigned)((nitems + 3) / 4)), dim3(256), 0, (hipStream_t)stream, *D, t, first,
                       nitems);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_canon(const PfDev *D, int x, const long long *rowoff, int nrows, int *out, void *stream) {
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(k_pf_canon, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *D, x, rowoff,
                       nrows, out);
    return (int)hipGetLastError();
}
