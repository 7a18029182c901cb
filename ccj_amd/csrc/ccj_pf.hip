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
//   * P sums int products made in 32-bit int arithmetic; each partial sum is an integer below
//     2^53 for n <= 295, so it is accumulated exactly in int64 across threads and converted once;
//   * table values (Boltzmann weights, pow(), the hairpin strstr cases) come from the host libm.
// A term whose Boltzmann factor is exactly 0.0 adds a signed zero to a sum that is truncated to
// int (interior-loop windows): such terms are skipped.
#pragma clang fp contract(off)

// CCJ_PF_ABLATE_ILOOP (timing experiments only, wrong results): skip the interior-loop windows
#ifdef CCJ_PF_ABLATE_ILOOP
#define PF_ILOOP_ON 0
#else
#define PF_ILOOP_ON 1
#endif

#include <hip/hip_runtime.h>

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

}  // namespace

// ---------------------------------------------------------------------------------------------
// P(i, i+s) (compute_P, part_func.cc:383-393): sum over j < d < k of PK(i,j,d+1,k) * PK(j+1,d,k+1,l),
// the product in int.  Lanes take 64 consecutive i; a workgroup takes one (j-i, d-i) and loops k.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pf_pterm(PfDev D, int s) {
    const PfG G{D};
    const int jo = blockIdx.y, dd = blockIdx.z;  // j = i+jo, d = i+dd
    if (dd <= jo || dd > s - 2) return;
    const int i = blockIdx.x * 64 + threadIdx.x + 1;
    if (i + s > D.n) return;
    const int l = i + s, j = i + jo, d = i + dd;
    long long acc = 0;
    for (int k = d + 1; k < l; ++k) acc += imul_wrap(G.g4(PF_PK, i, j, d + 1, k), G.g4(PF_PK, j + 1, d, k + 1, l));
    if (acc) atomicAdd((unsigned long long *)&D.Pacc[s * D.rs + i], (unsigned long long)acc);
}

// ---------------------------------------------------------------------------------------------
// The 2-D values of span s, one thread per interval (i, j = i+s), in the reference's order.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pf_diag(PfDev D, int s) {
    const PfG G{D};
    const PfExp &E = *D.E;
    const int i = blockIdx.x * 64 + threadIdx.x + 1, j = i + s, n = D.n;
    if (j > n) return;
    const int rs = D.rs;
    const int ij = s * rs + i;
    const int dang = D.dangles == 1 || D.dangles == 2;
    const short *S = D.S, *S1 = D.S1;

    // compute_energy (part_func.cc:290-300): V = hairpin + interior loops + VM
    {
        double vi = 0;  // compute_internal :222-240
        const int max_k = imin(j - TURN - 2, i + MAXLOOP + 1);
        const int tc = G.pt(i, j);
        for (int k = i + 1; k <= max_k; ++k) {
            const int min_l = imax(k + TURN + 1 + MAXLOOP + 2, k + j - i) - MAXLOOP - 2;
            for (int l = j - 1; l >= min_l; --l) {
                double x = G.d2(D.V, k, l) *
                           exp_E_IntLoop_pf(E, k - i - 1, j - l - 1, tc, D.rtype[G.pt(k, l)], S1[i + 1], S1[j - 1], S1[k - 1], S1[l + 1]);
                x *= 1.0;  // scale[u1+u2+2]
                vi += x;
            }
        }
        // compute_energy_VM :276-288, exp_Mbloop :203-212
        const int tt = D.pair[S[j] * 8 + S[i]];
        const double mb = dang ? exp_E_MLstem_pf(E, tt, j < n ? S[j - 1] : -1, i > 1 ? S[i + 1] : -1) : exp_E_MLstem_pf(E, tt, -1, -1);
        double vm = 0;
        for (int k = i + 1; k <= j - TURN - 1; ++k) {
            const double wm = G.g2(D.WM, i + 1, k - 1), wmv = G.g2(D.WMv, k, j - 1), wmp = G.g2(D.WMp, k, j - 1);
            vm += wm * wmv * mb * E.MLclosing;
            vm += wm * wmp * mb * E.MLclosing;
            vm += D.mlb[k - i - 1] * wmp * mb * E.MLclosing;
        }
        vm *= 1.0;  // scale[2]
        D.VM[ij] = vm;
        double v = 0;
        v += D.hp[ij];
        v += vi;
        v += vm;
        D.V[ij] = v;
    }
    // compute_pk_energies (:302-309): P (summed by k_pf_pterm), WBP, WPP
    const double p = (double)D.Pacc[ij];
    D.P[ij] = p;
    {
        double c = 0;  // compute_WBP :361-370
        for (int d = i; d < j; ++d) {
            c += G.d2(D.V, d, j) * E.bp * E.PPS;
            c += (d == i ? p : G.d2(D.P, d, j)) * E.PSM * E.PPS;
        }
        c += G.g2(D.WBP, i, j - 1) * D.cpp[1];
        D.WBP[ij] = c;
        double w = 0;  // compute_WPP :372-381 (its last term reads WBP)
        for (int d = i; d < j; ++d) {
            const double wp = G.WP(i, d - 1);
            w += wp * G.d2(D.V, d, j) * 1.0 * E.PPS;
            w += wp * (d == i ? p : G.d2(D.P, d, j)) * E.PSP * E.PPS;
        }
        w += G.g2(D.WBP, i, j - 1) * D.pup[1];
        D.WPP[ij] = w;
    }
    // compute_WMv_WMp (:242-256), exp_MLstem :192-201
    const int tij = G.pt(i, j);
    const double mls_ij = dang ? exp_E_MLstem_pf(E, tij, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1) : exp_E_MLstem_pf(E, tij, -1, -1);
    if (!(j - i - 1 < TURN)) {
        double wv = 0, wp = 0;
        wv += D.V[ij] * mls_ij;
        wp += p * E.PSM * E.b;
        wv += G.d2(D.WMv, i, j - 1) * D.mlb[1];
        wp += G.d2(D.WMp, i, j - 1) * D.mlb[1];
        D.WMv[ij] = wv;
        D.WMp[ij] = wp;
    }
    // compute_energy_WM (:258-274)
    if (!(j - i + 1 < 4)) {
        double c = 0;
        for (int k = i; k < j - TURN; ++k) {
            const int tk = G.pt(k, j);
            const double mls = k == i ? mls_ij
                                      : (dang ? exp_E_MLstem_pf(E, tk, k > 1 ? S[k - 1] : -1, j < n ? S[j + 1] : -1)
                                              : exp_E_MLstem_pf(E, tk, -1, -1));
            const double q1 = (k == i ? D.V[ij] : G.d2(D.V, k, j)) * mls;
            const double q2 = (k == i ? p : G.d2(D.P, k, j)) * E.PSM * E.b;
            c += D.mlb[k - i] * q1;
            c += D.mlb[k - i] * q2;
            const double wm = G.g2(D.WM, i, k - 1);
            c += wm * q1;
            c += wm * q2;
        }
        c += G.d2(D.WM, i, j - 1) * D.mlb[1];
        D.WM[ij] = c;
    }
}

// ---------------------------------------------------------------------------------------------
// The 21 recurrences of one 4-D cell, in the reference's order (compute_pk_energies :315-355).
// One thread per cell of level t; blockIdx.y = a = j-i (every loop bound is block-uniform).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pf_level(PfDev D, int t) {
    const PfG G{D};
    const PfExp &E = *D.E;
    const int n = D.n, a = blockIdx.y, b = t - a, m = n - t - 2;
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
    const long long C = L.C;
    auto put = [&](int x, double v) -> int {
        const int r = x86_trunc(v);
        cell[x * C] = r;
        return r;
    };
    const double bp = E.bp, ap = E.ap, cp1 = D.cpp[1], PB = E.PB;

    // PLmloop00 (:554-568); the seed PL(i,j,k,l) is not computed yet: 0 * beta2P
    {
        double c = 0;
        c += 0.0 * bp;
        for (int d = i; d <= j; ++d) {
            if (d > i) c += G.WB(i, d - 1) * G.g4(PF_PLmloop00, d, j, k, l);
            if (d < j) c += G.g4(PF_PLmloop00, i, d, k, l) * G.WB(d + 1, j);
        }
        put(PF_PLmloop00, c);
    }
    {  // PLmloop01 (:570-578)
        double c = 0;
        for (int d = i; d < j; ++d) c += G.g4(PF_PLmloop00, i, d, k, l) * G.g2(D.WBP, d + 1, j);
        put(PF_PLmloop01, c);
    }
    {  // PLmloop10 (:580-590)
        double c = 0;
        for (int d = i + 1; d <= j; ++d) {
            c += G.g2(D.WBP, i, d - 1) * G.g4(PF_PLmloop00, d, j, k, l);
            if (d < j) c += G.g4(PF_PLmloop10, i, d, k, l) * G.WB(d + 1, j);
        }
        put(PF_PLmloop10, c);
    }
    {  // PRmloop00 (:592-605)
        double c = 0;
        c += 0.0 * bp;
        for (int d = k; d <= l; ++d) {
            if (d > k) c += G.WB(k, d - 1) * G.g4(PF_PRmloop00, i, j, d, l);
            if (d < l) c += G.g4(PF_PRmloop00, i, j, k, d) * G.WB(d + 1, l);
        }
        put(PF_PRmloop00, c);
    }
    {  // PRmloop01 (:608-616)
        double c = 0;
        c += G.g4(PF_PRmloop01, i, j, k, l - 1) * cp1;
        for (int d = k; d < l; ++d) c += G.g4(PF_PRmloop00, i, j, k, d) * G.g2(D.WBP, d + 1, l);
        put(PF_PRmloop01, c);
    }
    {  // PRmloop10 (:618-626)
        double c = 0;
        c += G.g4(PF_PRmloop10, i, j, k + 1, l) * cp1;
        for (int d = k + 1; d <= l; ++d) c += G.g2(D.WBP, k, d - 1) * G.g4(PF_PRmloop00, i, j, d, l);
        put(PF_PRmloop10, c);
    }
    {  // PMmloop00 (:628-639)
        double c = 0;
        c += 0.0 * bp;
        for (int d = i; d < j; ++d) c += G.g4(PF_PMmloop00, i, d, k, l) * G.WB(d + 1, j);
        for (int d = k + 1; d <= l; ++d) c += G.g4(PF_PMmloop00, i, j, d, l) * G.WB(k, d - 1);
        put(PF_PMmloop00, c);
    }
    {  // PMmloop01 (:642-650): "+ expcp_pen[1]"
        double c = 0;
        c += G.g4(PF_PMmloop01, i, j, k + 1, l) + cp1;
        for (int d = k; d < l; ++d) c += G.g4(PF_PMmloop00, i, j, k, d) * G.g2(D.WBP, d + 1, l);
        put(PF_PMmloop01, c);
    }
    {  // PMmloop10 (:652-663)
        double c = 0;
        c += G.g4(PF_PMmloop10, i, j - 1, k, l) * cp1;
        for (int d = i + 1; d <= j; ++d) c += G.g2(D.WBP, i, d - 1) * G.g4(PF_PMmloop00, d, j, k, l);
        for (int d = k + 1; d < l; ++d) c += G.g4(PF_POmloop10, i, j, k, d) * G.WB(d + 1, l);
        put(PF_PMmloop10, c);
    }
    {  // POmloop00 (:665-676): the second loop assigns, so only its last term survives
        double c = 0;
        c += 0.0 * bp;
        for (int d = i + 1; d <= j; ++d) c += G.WB(i, d - 1) * G.g4(PF_POmloop00, d, j, k, l);
        if (k < l) c = G.g4(PF_POmloop00, i, j, k, l - 1) * G.WB(l, l);
        put(PF_POmloop00, c);
    }
    {  // POmloop01 (:679-686)
        double c = 0;
        for (int d = k; d < l; ++d) c += G.g4(PF_POmloop00, i, j, k, d) * G.g2(D.WBP, d + 1, l);
        put(PF_POmloop01, c);
    }
    {  // POmloop10 (:688-699): "+ get_WB"
        double c = 0;
        for (int d = i + 1; d <= j; ++d) c += G.g2(D.WBP, i, d - 1) * G.g4(PF_POmloop00, d, j, k, l);
        for (int d = k + 1; d < l; ++d) c += G.g4(PF_POmloop10, i, j, k, d) + G.WB(d + 1, l);
        put(PF_POmloop10, c);
    }

    const int rs = D.rs;
    // PL (:414-430) with get_PLiloop (:736-756) and get_PLmloop (:758-768)
    int PL = 0;
    {
        double c = 0;
        if (G.pt(i, j) > 0) {
            double r = 0;
            r += G.g4(PF_PL, i + 1, j - 1, k, l) * D.est[a * rs + i];
            const int dmax = PF_ILOOP_ON ? imin(j, i + MAXLOOP) : 0;
            for (int d = i + 1; d < dmax; ++d) {
                const int u1 = d - i - 1;
                const int dpmin = imax(d + TURN, j - MAXLOOP);
                for (int dp = j - 1; dp > dpmin; --dp) {
                    const int u2 = j - dp - 1;
                    const double e = D.ie[((size_t)(u1 * PF_IEW + u2) * (n + 1) + a) * rs + i];
                    if (e != 0.0) r += e * G.g4(PF_PL, d, dp, k, l) * 1.0;
                }
            }
            c += r;
            double q = 0;
            q += G.g4(PF_PLmloop10, i + 1, j - 1, k, l) * ap * bp;
            q += (double)imul_wrap(G.g4(PF_PLmloop01, i + 1, j - 1, k, l), D.ap_int) * bp;
            c += q * bp;
            if (j >= i + TURN + 1) c += G.g4(PF_PfromL, i + 1, j - 1, k, l) * 1.0;
        }
        PL = put(PF_PL, c);
    }
    // PR (:432-447), get_PRiloop (:770-790), get_PRmloop (:792-802)
    int PR = 0;
    {
        double c = 0;
        if (G.pt(k, l) > 0) {
            double r = 0;
            r += G.g4(PF_PR, i, j, k + 1, l - 1) * D.est[b * rs + k];
            const int dmax = PF_ILOOP_ON ? imin(l, k + MAXLOOP) : 0;
            for (int d = k + 1; d < dmax; ++d) {
                const int u1 = d - k - 1;
                const int dpmin = imax(d + TURN, l - MAXLOOP);
                for (int dp = l - 1; dp > dpmin; --dp) {
                    const int u2 = l - dp - 1;
                    const double e = D.ie[((size_t)(u1 * PF_IEW + u2) * (n + 1) + b) * rs + k];
                    if (e != 0.0) r += e * G.g4(PF_PR, i, j, d, dp) * 1.0;
                }
            }
            c += r;
            double q = 0;
            q += G.g4(PF_PRmloop10, i, j, k + 1, l - 1) * ap * bp;
            q += G.g4(PF_PRmloop01, i, j, k + 1, l - 1) * ap * bp;
            c += q * bp;
            if (l >= k + TURN + 1) c += G.g4(PF_PfromR, i, j, k + 1, l - 1) * 1.0;
        }
        PR = put(PF_PR, c);
    }
    // PM (:449-467), get_PMiloop (:804-824), get_PMmloop (:826-836)
    int PM = 0;
    {
        double c = 0;
        if (G.pt(j, k) > 0) {
            double r = 0;
            // get_e_stP(j-1, k+1): for j == 1 or k == n the reference indexes pair[][] with S[0] (= n)
            // or S[n+1]; the factor multiplies PM(i, j-1, k+1, l), which is then outside the matrix
            // (0), so any finite value gives 0 — use 0 instead of reading past the table
            const double est_m = (j > 1 && k < n) ? D.est[(h + 4) * rs + (j - 1)] : 0.0;
            r += G.g4(PF_PM, i, j - 1, k + 1, l) * est_m;
            const int dmin = PF_ILOOP_ON ? imax(i, j - MAXLOOP) : j, dpmax = imin(l, k + MAXLOOP);
            for (int d = j - 1; d > dmin; --d) {
                const int u1 = j - d - 1;
                for (int dp = k + 1; dp < dpmax; ++dp) {
                    const int u2 = dp - k - 1;
                    const double e = D.ie[((size_t)(u1 * PF_IEW + u2) * (n + 1) + (dp - d)) * rs + d];
                    if (e != 0.0) r += e * G.g4(PF_PM, i, d, dp, l) * 1.0;
                }
            }
            c += r;
            double q = 0;
            q += G.g4(PF_PMmloop10, i, j - 1, k + 1, l) * ap * bp;
            q += G.g4(PF_PMmloop01, i, j - 1, k + 1, l) * ap * bp;
            c += q * bp;
            if (k >= j + TURN - 1) c += G.g4(PF_PfromM, i, j - 1, k + 1, l) * 1.0;
            if (i == j && k == l) c += 1.0;
        }
        PM = put(PF_PM, c);
    }
    // PO (:469-486), get_POiloop (:838-858: reads PO(d,j,dp,k) with dp > k, always 0), get_POmloop
    int PO = 0;
    {
        double c = 0;
        if (G.pt(i, l) > 0) {
            double r = 0;
            r += G.g4(PF_PO, i + 1, j, k, l - 1) * D.est[(t + h + 2) * rs + i];
            c += r;
            double q = 0;
            q += G.g4(PF_POmloop10, i + 1, j, k, l - 1) * ap * bp;
            q += G.g4(PF_POmloop01, i + 1, j, k, l - 1) * ap * bp;
            c += q * bp;
            if (l >= i + TURN + 1) c += G.g4(PF_PfromO, i + 1, j, k, l - 1) * 1.0;
        }
        PO = put(PF_PO, c);
    }
    {  // PfromL (:488-503)
        double c = 0;
        for (int d = i + 1; d < j; ++d) {
            c += G.g4(PF_PfromL, d, j, k, l) * G.WP(i, d - 1);
            c += G.g4(PF_PfromL, i, d, k, l) * G.WP(d + 1, j);
        }
        c += PR * 1.0 * PB;
        c += PM * 1.0 * PB;
        c += PO * 1.0 * PB;
        put(PF_PfromL, c);
    }
    {  // PfromR (:505-518)
        double c = 0;
        for (int d = k + 1; d < l; ++d) {
            c += G.g4(PF_PfromR, i, j, d, l) * G.WP(k, d - 1);
            c += G.g4(PF_PfromR, i, j, k, d) * G.WP(d + 1, l);
        }
        c += PM * 1.0 * PB;
        c += PO * 1.0 * PB;
        put(PF_PfromR, c);
    }
    {  // PfromM (:520-535)
        double c = 0;
        for (int d = i + 1; d < j; ++d) c += G.g4(PF_PfromM, i, d, k, l) * G.WP(d + 1, j);
        for (int d = k + 1; d < l; ++d) c += G.g4(PF_PfromM, i, j, d, l) * G.WP(k, d - 1);
        c += PL * 1.0 * PB;
        c += PR * 1.0 * PB;
        put(PF_PfromM, c);
    }
    {  // PfromO (:537-552)
        double c = 0;
        for (int d = i + 1; d < j; ++d) c += G.g4(PF_PfromO, d, j, k, l) * G.WP(i, d - 1);
        for (int d = k + 1; d < l; ++d) c += G.g4(PF_PfromO, i, j, k, d) * G.WP(d + 1, l);
        c += PL * 1.0 * PB;
        c += PR * 1.0 * PB;
        put(PF_PfromO, c);
    }
    {  // PK (:395-412)
        double c = 0;
        for (int d = i + 1; d < j; ++d) c += G.g4(PF_PK, i, d, k, l) * G.WP(d + 1, j);
        for (int d = k + 1; d < l; ++d) c += G.g4(PF_PK, i, j, d, l) * G.WP(k, d - 1);
        c += PL * 1.0 * PB;
        c += PM * 1.0 * PB;
        c += PR * 1.0 * PB;
        c += PO * 1.0 * PB;
        put(PF_PK, c);
    }
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
    const int ni = D->n - s;
    if (s < 3 || ni <= 0) return 0;
    hipLaunchKernelGGL(k_pf_pterm, dim3((unsigned)((ni + 63) / 64), (unsigned)(s - 2), (unsigned)(s - 1)), dim3(64), 0,
                       (hipStream_t)stream, *D, s);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_diag(const PfDev *D, int s, void *stream) {
    const int ni = D->n - s;
    if (ni <= 0) return 0;
    hipLaunchKernelGGL(k_pf_diag, dim3((unsigned)((ni + 63) / 64)), dim3(64), 0, (hipStream_t)stream, *D, s);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_level(const PfDev *D, const PfLvl *Lh, int t, void *stream) {
    const int M = Lh[t].M;
    if (M <= 0) return 0;
    hipLaunchKernelGGL(k_pf_level, dim3((unsigned)((M + 255) / 256), (unsigned)(t + 1)), dim3(256), 0, (hipStream_t)stream,
                       *D, t);
    return (int)hipGetLastError();
}

extern "C" int ccjk_pf_canon(const PfDev *D, int x, const long long *rowoff, int nrows, int *out, void *stream) {
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(k_pf_canon, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *D, x, rowoff,
                       nrows, out);
    return (int)hipGetLastError();
}
