// ccj_energy.h — Turner nearest-neighbour loop energies used by the CCJ path, callable from
// host C++ (backtrack, table precompute) and from HIP device code (fill kernels).
//
// Semantics follow the reference exactly (integer dcal/mol, type-0 rows included):
//   E_IntLoop  : src/ViennaRNA/loops/internal.h:477-569
//   E_Hairpin  : src/ViennaRNA/loops/hairpin.h:148-200   (host only: strstr on special loops)
//   E_MLstem   : src/ViennaRNA/loops/multibranch.h:225-246
//   E_ExtLoop  : src/ViennaRNA/loops/external.c:2191-2209 (== vrna_E_ext_stem :384-402)
// The only floating point in these functions is (int)(lxc*log(x/30.)) for loops longer than
// 30 nt.  It is evaluated once on the host with the same libm as the reference and passed in
// as the integer table `lx[x]`, so device math libraries never touch a result.
#pragma once
#include "ccj_params.h"

#ifdef __HIPCC__
#define CCJ_HD __host__ __device__ __forceinline__
#else
#define CCJ_HD inline
#endif

namespace ccj {

constexpr int INF = CCJ_INF;
constexpr int TURN = CCJ_TURN;
constexpr int MAXLOOP = CCJ_MAXLOOP;
constexpr int INTERN_INF = 32767;

CCJ_HD int imin(int a, int b) { return a < b ? a : b; }
CCJ_HD int imax(int a, int b) { return a > b ? a : b; }

CCJ_HD int E_IntLoop(const ccj_energy_params *P, const int *lx, int n1, int n2, int type, int type_2,
                     int si1, int sj1, int sp1, int sq1) {
    int nl, ns, energy;
    if (n1 > n2) { nl = n1; ns = n2; } else { nl = n2; ns = n1; }
    if (nl == 0) return P->stack[type][type_2];
    if (ns == 0) {
        energy = (nl <= MAXLOOP) ? P->bulge[nl] : (P->bulge[30] + lx[nl]);
        if (nl == 1) {
            energy += P->stack[type][type_2];
        } else {
            if (type > 2) energy += P->TerminalAU;
            if (type_2 > 2) energy += P->TerminalAU;
        }
        return energy;
    }
    if (ns == 1) {
        if (nl == 1) return P->int11[type][type_2][si1][sj1];
        if (nl == 2) {
            if (n1 == 1) return P->int21[type][type_2][si1][sq1][sj1];
            return P->int21[type_2][type][sq1][si1][sp1];
        }
        energy = (nl + 1 <= MAXLOOP) ? P->internal_loop[nl + 1] : (P->internal_loop[30] + lx[nl + 1]);
        energy += imin(P->max_ninio, (nl - ns) * P->ninio2);
        energy += P->mismatch1nI[type][si1][sj1] + P->mismatch1nI[type_2][sq1][sp1];
        return energy;
    }
    if (ns == 2) {
        if (nl == 2) return P->int22[type][type_2][si1][sp1][sq1][sj1];
        if (nl == 3) {
            energy = P->internal_loop[5] + P->ninio2;
            energy += P->mismatch23I[type][si1][sj1] + P->mismatch23I[type_2][sq1][sp1];
            return energy;
        }
    }
    const int u = nl + ns;
    energy = (u <= MAXLOOP) ? P->internal_loop[u] : (P->internal_loop[30] + lx[u]);
    energy += imin(P->max_ninio, (nl - ns) * P->ninio2);
    energy += P->mismatchI[type][si1][sj1] + P->mismatchI[type_2][sq1][sp1];
    return energy;
}

CCJ_HD int E_MLstem(const ccj_energy_params *P, int type, int si1, int sj1) {
    int energy = 0;
    if (si1 >= 0 && sj1 >= 0) energy += P->mismatchM[type][si1][sj1];
    else if (si1 >= 0) energy += P->dangle5[type][si1];
    else if (sj1 >= 0) energy += P->dangle3[type][sj1];
    if (type > 2) energy += P->TerminalAU;
    energy += P->MLintern[type];
    return energy;
}

CCJ_HD int E_ExtLoop(const ccj_energy_params *P, int type, int si1, int sj1) {
    int energy = 0;
    if (si1 >= 0 && sj1 >= 0) energy += P->mismatchExt[type][si1][sj1];
    else if (si1 >= 0) energy += P->dangle5[type][si1];
    else if (sj1 >= 0) energy += P->dangle3[type][sj1];
    if (type > 2) energy += P->TerminalAU;
    return energy;
}

// ViennaRNA pair table (pair_mat.h:19-31) for the ACGU(T) alphabet, energy_set == 0.
// Codes: 0 '_', 1 A, 2 C, 3 G, 4 U/T.
CCJ_HD int encode_base(char c) {
    switch (c) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 3;
        case 'U': case 'u': case 'T': case 't': return 4;
        default: return 0;
    }
}

}  // namespace ccj
