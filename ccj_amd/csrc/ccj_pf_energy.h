// ccj_pf_energy.h — Boltzmann weights of the CCJ partition function, shared by
// the host (table build, W, stochastic traceback) and the HIP fill kernels.
//
// PfExp holds the fields of ViennaRNA's vrna_exp_param_t (params/basic.h:120-173) that
// part_func.cc reads, computed on the host with the host libm exactly as get_scaled_exp_params
// (params/params.c:558-738) does at 37 C, plus the rescaled pseudoknot penalties of
// W_final_pf::rescale_pk_globals (part_func.cc:127-146).  The functions below restate
// exp_E_IntLoop (loops/internal.h:572-651), exp_E_MLstem (loops/multibranch.h:255-276) and
// vrna_exp_E_ext_stem (loops/external_pf.c:100-119) with the same operation order, so device
// and host give the reference's bits (every file that includes this is compiled without
// floating-point contraction).
//
// expinternal[] has 31 entries in the reference, but the pseudoknot interior loops (window
// u1, u2 <= 28) ask exp_E_IntLoop for loop sizes up to 56 and read past its end into
// expmismatchExt[0][0][0...] (the next member).  internal57 reproduces those reads.
#pragma once
#include "ccj_energy.h"

namespace ccj {

struct PfExp {
    double stack[8][8];
    double hairpin[31];
    double bulge[31];
    double internal57[57];  // expinternal[0..30] then expmismatchExt flat[0..25] (see above)
    double mismatchExt[8][5][5];
    double mismatchI[8][5][5];
    double mismatch23I[8][5][5];
    double mismatch1nI[8][5][5];
    double mismatchH[8][5][5];
    double mismatchM[8][5][5];
    double dangle5[8][5];
    double dangle3[8][5];
    double int11[8][8][5][5];
    double int21[8][8][5][5][5];
    double int22[8][8][5][5][5][5];
    double ninio[31];  // expninio[2][*]
    double lxc, MLbase, MLintern[8], MLclosing, TermAU, kT, pf_scale;
    double tetra[40], tri[40], hex[40];
    // rescale_pk_globals (part_func.cc:132-145)
    double PS, PSM, PSP, PB, PUP, PPS, a, b, c, ap, bp, cp;
};

// exp_E_IntLoop, loops/internal.h:572-651 (noGUclosure == 0, the model default)
CCJ_HD double exp_E_IntLoop_pf(const PfExp &P, int u1, int u2, int type, int type2, int si1, int sj1, int sp1, int sq1) {
    int ul, us;
    if (u1 > u2) {
        ul = u1;
        us = u2;
    } else {
        ul = u2;
        us = u1;
    }
    double z;
    if (ul == 0) return P.stack[type][type2];
    if (us == 0) {
        z = P.bulge[ul];
        if (ul == 1) {
            z *= P.stack[type][type2];
        } else {
            if (type > 2) z *= P.TermAU;
            if (type2 > 2) z *= P.TermAU;
        }
        return z;
    }
    if (us == 1) {
        if (ul == 1) return P.int11[type][type2][si1][sj1];
        if (ul == 2) {
            if (u1 == 1) return P.int21[type][type2][si1][sq1][sj1];
            return P.int21[type2][type][sq1][si1][sp1];
        }
        z = P.internal57[ul + us] * P.mismatch1nI[type][si1][sj1] * P.mismatch1nI[type2][sq1][sp1];
        return z * P.ninio[ul - us];
    }
    if (us == 2) {
        if (ul == 2) return P.int22[type][type2][si1][sp1][sq1][sj1];
        if (ul == 3) {
            z = P.internal57[5] * P.mismatch23I[type][si1][sj1] * P.mismatch23I[type2][sq1][sp1];
            return z * P.ninio[1];
        }
    }
    z = P.internal57[ul + us] * P.mismatchI[type][si1][sj1] * P.mismatchI[type2][sq1][sp1];
    return z * P.ninio[ul - us];
}

// exp_E_MLstem, loops/multibranch.h:255-276
CCJ_HD double exp_E_MLstem_pf(const PfExp &P, int type, int si1, int sj1) {
    double e = 1.0;
    if (si1 >= 0 && sj1 >= 0) e = P.mismatchM[type][si1][sj1];
    else if (si1 >= 0) e = P.dangle5[type][si1];
    else if (sj1 >= 0) e = P.dangle3[type][sj1];
    if (type > 2) e *= P.TermAU;
    e *= P.MLintern[type];
    return e;
}

// vrna_exp_E_ext_stem, loops/external_pf.c:100-119
CCJ_HD double exp_E_ExtLoop_pf(const PfExp &P, int type, int si1, int sj1) {
    double e = 1.0;
    if (si1 >= 0 && sj1 >= 0) e = P.mismatchExt[type][si1][sj1];
    else if (si1 >= 0) e = P.dangle5[type][si1];
    else if (sj1 >= 0) e = P.dangle3[type][sj1];
    if (type > 2) e *= P.TermAU;
    return e;
}

// Matrix4DPF::set(..., energy_t e) converts the double sum with cvttsd2si: the truncated value,
// or INT_MIN when it is out of int range or NaN (x86 "integer indefinite").
CCJ_HD int x86_trunc(double v) {
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : (int)0x80000000u;
}

// 32-bit wrapping int product (part_func.cc:388 multiplies two int getters)
CCJ_HD int imul_wrap(int a, int b) { return (int)((unsigned)a * (unsigned)b); }

}  // namespace ccj
