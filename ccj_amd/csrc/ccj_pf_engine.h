// ccj_pf_engine.h — device-side layout of the partition-function fill (ccj_pf.hip, ccj_pf.cc).
//
// 4-D matrices: the MFE engine's level-major layout with int32 cells and the 21
// matrices of W_final_pf (part_func.hh:86-113):
//   elem(x,t,a,h,i) = lb_t + x*C_t + a*M_t + h*m_t - h(h-1)/2 + (i-1),  m_t = n-t-2,
//   M_t = m_t(m_t+1)/2, C_t = (t+1) M_t.
// 2-D matrices: doubles, span-major [w][p] with row stride rs = n+2.
// Interior-loop weights get_e_intP (part_func.cc:886-891), u1, u2 < PF_IEW, in two tables whose
// window rows (one pair, one u1) are compacted to the set bits of the pair's mask row (mO / mI, bit u2
// set = the weight is nonzero): the k-th set bit of mask row (pair, u1) -> slot k of that row (rows keep
// their PF_IEW-double stride, zero past the last set bit), PF_ILW doubles of zero tail padding after
// the last row (k_pf_iloop reads a round
// of PF_ILW slots with one scalar load).  The un-compacted window is:
//   ieO[w][p][u1][u2]: the loop closed by (p, p+w) around (p+1+u1, p+w-1-u2)   (PL, PR)
//   ieI[g][j][u1][u2]: the loop closed by (j-1-u1, j+g+1+u2) around (j, j+g)    (PM)
#pragma once
#include <stdint.h>

#include "../../include/ccj_pf.h"
#include "ccj_pf_energy.h"

namespace ccj {

enum {
    PF_PK = CCJ_PF_PK, PF_PL = CCJ_PF_PL, PF_PR = CCJ_PF_PR, PF_PM = CCJ_PF_PM, PF_PO = CCJ_PF_PO,
    PF_PfromL = CCJ_PF_PfromL, PF_PfromR = CCJ_PF_PfromR, PF_PfromM = CCJ_PF_PfromM, PF_PfromO = CCJ_PF_PfromO,
    PF_PLmloop00 = CCJ_PF_PLmloop00, PF_PLmloop01 = CCJ_PF_PLmloop01, PF_PLmloop10 = CCJ_PF_PLmloop10,
    PF_PRmloop00 = CCJ_PF_PRmloop00, PF_PRmloop01 = CCJ_PF_PRmloop01, PF_PRmloop10 = CCJ_PF_PRmloop10,
    PF_PMmloop00 = CCJ_PF_PMmloop00, PF_PMmloop01 = CCJ_PF_PMmloop01, PF_PMmloop10 = CCJ_PF_PMmloop10,
    PF_POmloop00 = CCJ_PF_POmloop00, PF_POmloop01 = CCJ_PF_POmloop01, PF_POmloop10 = CCJ_PF_POmloop10,
    PF_NMAT4 = CCJ_PF_NMAT4
};

constexpr int PF_IEW = MAXLOOP - 1;  // interior-loop window per side: u <= 28
#ifndef CCJ_PF_ILW
#define CCJ_PF_ILW 8
#endif
constexpr int PF_ILW = CCJ_PF_ILW;   // k_pf_iloop: window terms per round (multiple of 4); the compacted
                                     // weight rows carry PF_ILW doubles of tail padding
static_assert(PF_ILW % 4 == 0 && PF_ILW >= 4, "CCJ_PF_ILW: window_row reads whole groups of 4 terms");

// k_pf_ppush: spans per wave = consecutive partner levels a wave reads through one buffer resource
constexpr int PF_PP_S = 8;

struct PfLvl {
    long long lb;  // element offset of level t
    long long C;   // cells of one matrix at level t
    int M;         // cells of one a-block
    int pad;
    long long lbx; // element offset of level t in the PL/PR copies (PLx then PRx, C each)
    long long pmb; // element offset of level t in the PM copy (m * n * (t+1))
    long long lr;  // cells of the levels below t: level t's first split-loop record (PfDev::r1 .. r4)
};

struct PfDev {
    int n, rs, dangles, ap_int;  // ap_int: the int ap_penalty (get_PLmloop multiplies an int by it)
    const PfExp *E;
    const short *S, *S1;
    const int8_t *pt;     // [w][p] pair[S[p]][S[p+w]]
    const int8_t *pair;   // 8x8
    const int8_t *rtype;  // 8
    const double *hp;     // [w][p] HairpinE
    const double *est;    // [w][p] get_e_stP
    const double *ieO, *ieI;  // get_e_intP by outer / inner pair (above)
    const uint32_t *mO, *mI;  // [pair][u1]: bit u2 set when that weight is nonzero and the loop's other pair can pair
    const double *mlb, *cpp, *pup;  // expMLbase[], expcp_pen[], expPUP_pen[] (n+2)
    double *V, *VM, *WM, *WMv, *WMp, *WBP, *WPP, *P;  // [w][p]
    long long *Pacc;      // [w][p] exact integer P sums
    unsigned long long *Pabs;  // [w][p] sum of |term| (exactness check: < 2^53 => the reference's double sum is exact)
    int *d4;
    const PfLvl *ld;
    // interior-loop copies of PL / PR / PM in the MFE engine's layouts (written by
    // k_pf_level where the pair can pair), so that k_pf_iloop's lanes read consecutive words:
    //   PLx(t,a,h,i) = lbx + a*M + G(i-1) + h;  PRx = lbx + C + a*M + q(q+1)/2 + i-1, q = i+h-1;
    //   PMx = pmb + (h*n + j-1)*(t+1) + a
    int *cx, *pmx;
    const uint32_t *items;  // k_pf_iloop work items of all levels (ccj_items.h)
    double *R;              // k_pf_iloop's interior-loop sums, two level buffers (t & 1) of [role][a*M + off]
    long long Rst;          // doubles per buffer (3 * max C_t)
    // split-loop operand records, written by k_pf_level with the cell, indexed like a
    // matrix (record lr + a*M + off): the values one side of a split step reads at one neighbour,
    // contiguous, so a step costs two buffer loads per side instead of five or six int loads
    //   r1 (X1 = X(d,j,k,l), 5 ints): PLmloop00 PMmloop00 POmloop00 PfromL PfromO
    //   r2 (X2 = X(i,d,k,l), 6 ints): PLmloop00 PLmloop10 PMmloop00 PfromL PfromM PK
    //   r3 (X3 = X(i,j,d,l), 5 ints): PRmloop00 PMmloop00 PfromR PfromM PK
    //   r4 (X4 = X(i,j,k,d), 6 ints): PRmloop00 PMmloop00 POmloop00 POmloop10 PfromR PfromO
    int *r1, *r2, *r3, *r4;
};
constexpr int PF_REC1 = 5, PF_REC2 = 6, PF_REC3 = 5, PF_REC4 = 6;
constexpr int PF_RECS = PF_REC1 + PF_REC2 + PF_REC3 + PF_REC4;  // ints per cell

}  // namespace ccj

extern "C" {
int ccjk_pf_pterm(const ccj::PfDev *D, int s, void *stream);
int ccjk_pf_ppush(const ccj::PfDev *D, int lev, void *stream);
int ccjk_pf_diag(const ccj::PfDev *D, int s, void *stream);
int ccjk_pf_level(const ccj::PfDev *D, const ccj::PfLvl *Lh, int t, void *stream);
int ccjk_pf_iloop(const ccj::PfDev *D, int t, long long first, int nitems, void *stream);
int ccjk_pf_canon(const ccj::PfDev *D, int x, const long long *rowoff, int nrows, int *out, void *stream);
}
