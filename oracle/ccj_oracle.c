/*
 * oracle/ccj_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the CCJ MFE fill.
 *
 * This is the checker the HIP engine is compared against (task ③).  It restates, in plain C
 * and in the reference's own loop order, the recurrences of:
 *   src/W_final.cc:58-79          fill driver + exterior W
 *   src/s_energy_matrix.cc:54-358 V / WM / WMv / WMp
 *   src/pseudo_loop.cc:69-850     P / WBP / WPP and the 22 four-dimensional gap matrices
 *   src/matrices.hh:14-232        storage semantics (INF domains, int16 clamp, get() guards)
 *   src/ViennaRNA/loops/{internal.h:477-569, hairpin.h:148-200, multibranch.h:225-246}
 *   src/ViennaRNA/loops/external.c:2191-2209, src/ViennaRNA/pair_mat.h:19-183
 * Energy tables come from our blob (include/ccj_params.h).
 *
 * Pinning: tests/test_oracle.py checks every matrix hash of this restatement against the real
 * reference (oracle/_ref/ref_driver, built from /root/reference by oracle/Makefile) through the
 * committed fixtures tests/golden/hashes_*.json.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The shipped engine never links it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include "ccj_params.h"
#ifdef _OPENMP
#include <omp.h>
#endif

#define INF CCJ_INF
#define TURN CCJ_TURN
#define MAXLOOP CCJ_MAXLOOP
#define INTERN_INF 32767
#define MIN2(a, b) ((a) < (b) ? (a) : (b))

enum { NMAT4 = 22 };

typedef struct oracle {
    int n, dangles;
    const ccj_energy_params *P;
    ccj_pk_penalties pen;
    char *seq;
    short *S, *S1;
    int pair[8][8];
    int rtype[8];
    /* 2-D: dense (n+2)*(n+2) */
    int *V; char *Vt; int *WM, *WMv, *WMp, *Pm, *WBP, *WPP;
    int *W;
    /* 4-D: the reference's offsets (Matrix4D::construct_index, matrices.hh:208-221), held as a
       2-D (i,j) base table plus the closed form of its inner k sum, + l-k */
    size_t *idx2;
    size_t slice;
    int16_t *M4[NMAT4];
    /* memo of get_e_intP (pseudo_loop.cc:827-840) over every pseudoknot interior-loop window:
       eint[(p*(n+2)+q)*29*29 + u1*29 + u2] = lrint(e_intP * E_IntLoop) for the outer pair (p,q)
       and the inner pair (p+1+u1, q-1-u2); the same value the reference recomputes per candidate */
    int *eint;
} oracle;

/* matrix ids, reference allocate_space order (pseudo_loop.cc:37-62) */
enum { PK, PL, PR, PM, PO, PfromL, PfromR, PfromM, PfromMprime, PfromO,
       PLmloop00, PLmloop01, PLmloop10, PRmloop00, PRmloop01, PRmloop10,
       PMmloop00, PMmloop01, PMmloop10, POmloop00, POmloop01, POmloop10 };

#define D2(o, i, j) ((size_t)(i) * (size_t)((o)->n + 2) + (size_t)(j))

/* ---- sequence encoding: pair_mat.h:47-183 (energy_set == 0) ---- */
static const int BP_pair[8][8] = {
    {0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 5, 0, 0, 5}, {0, 0, 0, 1, 0, 0, 0, 0},
    {0, 0, 2, 0, 3, 0, 0, 0}, {0, 6, 0, 4, 0, 0, 0, 6}, {0, 0, 0, 0, 0, 0, 2, 0},
    {0, 0, 0, 0, 0, 1, 0, 0}, {0, 6, 0, 0, 5, 0, 0, 0}};

static int encode_char(char c) {
    switch (c) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 3;
        case 'U': case 'u': case 'T': case 't': return 4;
        default: return 0;
    }
}

/* ---- energy primitives ---- */
static int E_IntLoop(const oracle *o, int n1, int n2, int type, int type_2, int si1, int sj1,
                     int sp1, int sq1) {
    /* ViennaRNA/loops/internal.h:477-569 */
    const ccj_energy_params *P = o->P;
    int nl, ns, u, energy;
    if (n1 > n2) { nl = n1; ns = n2; } else { nl = n2; ns = n1; }
    if (nl == 0) return P->stack[type][type_2];
    if (ns == 0) {
        energy = (nl <= MAXLOOP) ? P->bulge[nl] : (P->bulge[30] + (int)(P->lxc * log(nl / 30.)));
        if (nl == 1) energy += P->stack[type][type_2];
        else {
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
        energy = (nl + 1 <= MAXLOOP) ? P->internal_loop[nl + 1]
                                     : (P->internal_loop[30] + (int)(P->lxc * log((nl + 1) / 30.)));
        energy += MIN2(P->max_ninio, (nl - ns) * P->ninio2);
        energy += P->mismatch1nI[type][si1][sj1] + P->mismatch1nI[type_2][sq1][sp1];
        return energy;
    } else if (ns == 2) {
        if (nl == 2) return P->int22[type][type_2][si1][sp1][sq1][sj1];
        if (nl == 3) {
            energy = P->internal_loop[5] + P->ninio2;
            energy += P->mismatch23I[type][si1][sj1] + P->mismatch23I[type_2][sq1][sp1];
            return energy;
        }
    }
    u = nl + ns;
    energy = (u <= MAXLOOP) ? P->internal_loop[u] : (P->internal_loop[30] + (int)(P->lxc * log(u / 30.)));
    energy += MIN2(P->max_ninio, (nl - ns) * P->ninio2);
    energy += P->mismatchI[type][si1][sj1] + P->mismatchI[type_2][sq1][sp1];
    return energy;
}

static int E_Hairpin(const oracle *o, int size, int type, int si1, int sj1, const char *string) {
    /* ViennaRNA/loops/hairpin.h:148-200 */
    const ccj_energy_params *P = o->P;
    int energy;
    if (size <= 30) energy = P->hairpin[size];
    else energy = P->hairpin[30] + (int)(P->lxc * log(size / 30.));
    if (size < 3) return energy;
    if (string && P->special_hp) {
        if (size == 4) {
            char tl[7] = {0}; const char *ts;
            memcpy(tl, string, 6);
            if ((ts = strstr(P->Tetraloops, tl))) return P->Tetraloop_E[(ts - P->Tetraloops) / 7];
        } else if (size == 6) {
            char tl[9] = {0}; const char *ts;
            memcpy(tl, string, 8);
            if ((ts = strstr(P->Hexaloops, tl))) return P->Hexaloop_E[(ts - P->Hexaloops) / 9];
        } else if (size == 3) {
            char tl[6] = {0}; const char *ts;
            memcpy(tl, string, 5);
            if ((ts = strstr(P->Triloops, tl))) return P->Triloop_E[(ts - P->Triloops) / 6];
            return energy + (type > 2 ? P->TerminalAU : 0);
        }
    }
    energy += P->mismatchH[type][si1][sj1];
    return energy;
}

static int E_MLstem(const oracle *o, int type, int si1, int sj1) {
    /* ViennaRNA/loops/multibranch.h:225-246 */
    const ccj_energy_params *P = o->P;
    int energy = 0;
    if (si1 >= 0 && sj1 >= 0) energy += P->mismatchM[type][si1][sj1];
    else if (si1 >= 0) energy += P->dangle5[type][si1];
    else if (sj1 >= 0) energy += P->dangle3[type][sj1];
    if (type > 2) energy += P->TerminalAU;
    energy += P->MLintern[type];
    return energy;
}

static int E_ExtLoop(const oracle *o, int type, int si1, int sj1) {
    /* ViennaRNA/loops/external.c:2191-2209 (== vrna_E_ext_stem :384-402) */
    const ccj_energy_params *P = o->P;
    int energy = 0;
    if (si1 >= 0 && sj1 >= 0) energy += P->mismatchExt[type][si1][sj1];
    else if (si1 >= 0) energy += P->dangle5[type][si1];
    else if (sj1 >= 0) energy += P->dangle3[type][sj1];
    if (type > 2) energy += P->TerminalAU;
    return energy;
}

/* ---- storage semantics ---- */
static inline int getV(const oracle *o, int i, int j) { /* s_energy_matrix.hh:37 */
    if (i >= j) return INF;
    return o->V[D2(o, i, j)];
}
static inline int getWM(const oracle *o, int i, int j) { if (i >= j) return INF; return o->WM[D2(o, i, j)]; }
static inline int getWMv(const oracle *o, int i, int j) { if (i >= j) return INF; return o->WMv[D2(o, i, j)]; }
static inline int getWMp(const oracle *o, int i, int j) { if (i >= j) return INF; return o->WMp[D2(o, i, j)]; }
static inline int tri_get(const oracle *o, const int *m, int i, int j) { /* matrices.hh:38-41 */
    if (i > j) return INF;
    return m[D2(o, i, j)];
}

static inline size_t idx4(const oracle *o, int i, int j, int k, int l) { /* matrices.hh:229-231 */
    /* construct_index adds (n - k') for k' = j..k-1 (0-based) to the (i,j) base */
    size_t n = (size_t)o->n, dk = (size_t)(k - j);
    return o->idx2[(size_t)(i - 1) * n + (size_t)(j - 1)] + dk * n - dk * (size_t)(k + j - 3) / 2 + (size_t)(l - k);
}
static inline int get4(const oracle *o, int m, int i, int j, int k, int l) { /* matrices.hh:177-182 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    return o->M4[m][idx4(o, i, j, k, l)];
}
static inline void set4(oracle *o, int m, int i, int j, int k, int l, int e) { /* matrices.hh:188-191 */
    if (e >= INTERN_INF) e = INTERN_INF;
    o->M4[m][idx4(o, i, j, k, l)] = (int16_t)e;
}

static inline int get_WB(const oracle *o, int i, int j) { /* pseudo_loop.cc:647-653 */
    if (i <= 0 || j <= 0 || i > o->n || j > o->n) return INF;
    if (i > j) return 0;
    return MIN2(o->pen.cp * (j - i + 1), tri_get(o, o->WBP, i, j));
}
static inline int get_WP(const oracle *o, int i, int j) { /* pseudo_loop.cc:655-661 */
    if (i <= 0 || j <= 0 || i > o->n || j > o->n) return INF;
    if (i > j) return 0;
    return MIN2(o->pen.PUP * (j - i + 1), tri_get(o, o->WPP, i, j));
}
static inline int can_pair(const oracle *o, int i, int j) { /* pseudo_loop.hh:117-136 */
    if (j - i <= TURN) return 0;
    return o->pair[o->S[i]][o->S[j]] > 0;
}
static inline int ptype(const oracle *o, int i, int j) { return o->pair[o->S[i]][o->S[j]]; }

/* pseudo_loop.cc:822-840 */
static int compute_int(const oracle *o, int i, int j, int k, int l) {
    return E_IntLoop(o, k - i - 1, j - l - 1, ptype(o, i, j), o->rtype[ptype(o, k, l)], o->S1[i + 1],
                     o->S1[j - 1], o->S1[k - 1], o->S1[l + 1]);
}
static int get_e_stP(const oracle *o, int i, int j) {
    if (i + 1 == j - 1) return INF;
    int ss = compute_int(o, i, j, i + 1, j - 1);
    return (int)lrint(o->pen.e_stP * ss);
}
static int get_e_intP_direct(const oracle *o, int i, int ip, int jp, int j) {
    int e = compute_int(o, i, j, ip, jp);
    return (int)lrint(o->pen.e_intP * e);
}
enum { EW = MAXLOOP - 1 };  /* u1, u2 <= 28 in every iloop window of pseudo_loop.cc:682-808 */
static inline int get_e_intP(const oracle *o, int i, int ip, int jp, int j) {
    return o->eint[((size_t)i * (size_t)(o->n + 2) + (size_t)j) * EW * EW + (size_t)(ip - i - 1) * EW +
                   (size_t)(j - jp - 1)];
}

/* ---- s_energy_matrix.cc ---- */
static int E_MLStem(const oracle *o, int vij, int vi1j, int vij1, int vi1j1, int i, int j) {
    /* s_energy_matrix.cc:54-112 */
    const short *S = o->S;
    int e = INF, en;
    int type = o->pair[S[i]][S[j]];
    int n = o->n;
    en = vij;
    if (en != INF) {
        if (o->dangles == 2) {
            int mm5 = i > 1 ? S[i - 1] : -1;
            int mm3 = j < n ? S[j + 1] : -1;
            en += E_MLstem(o, type, mm5, mm3);
        } else en += E_MLstem(o, type, -1, -1);
        e = MIN2(e, en);
    }
    if (o->dangles == 1) {
        int mm5 = S[i], mm3 = S[j];
        en = (j - i - 1 > TURN) ? vi1j : INF;
        if (en != INF) { en += o->P->MLbase; type = o->pair[S[i + 1]][S[j]]; en += E_MLstem(o, type, mm5, -1); e = MIN2(e, en); }
        en = (j - 1 - i > TURN) ? vij1 : INF;
        if (en != INF) { en += o->P->MLbase; type = o->pair[S[i]][S[j - 1]]; en += E_MLstem(o, type, -1, mm3); e = MIN2(e, en); }
        en = (j - 1 - i - 1 > TURN) ? vi1j1 : INF;
        if (en != INF) { en += 2 * o->P->MLbase; type = o->pair[S[i + 1]][S[j - 1]]; en += E_MLstem(o, type, mm5, mm3); e = MIN2(e, en); }
    }
    return e;
}

static int E_MbLoop(const oracle *o, int WM2ij, int WM2ip1j, int WM2ijm1, int WM2ip1jm1, int i, int j) {
    /* s_energy_matrix.cc:122-205 */
    const short *S = o->S;
    const ccj_energy_params *P = o->P;
    int e = INF, en;
    int tt = o->pair[S[j]][S[i]];
    switch (o->dangles) {
        case 2:
            e = WM2ij;
            if (e != INF) e += E_MLstem(o, tt, S[j - 1], S[i + 1]) + P->MLclosing;
            break;
        case 1:
            e = WM2ij;
            if (e != INF) e += E_MLstem(o, tt, -1, -1) + P->MLclosing;
            en = WM2ip1j;
            if (en != INF) en += E_MLstem(o, tt, -1, S[i + 1]) + P->MLclosing + P->MLbase;
            e = MIN2(e, en);
            en = WM2ijm1;
            if (en != INF) en += E_MLstem(o, tt, S[j - 1], -1) + P->MLclosing + P->MLbase;
            e = MIN2(e, en);
            en = WM2ip1jm1;
            if (en != INF) en += E_MLstem(o, tt, S[j - 1], S[i + 1]) + P->MLclosing + 2 * P->MLbase;
            e = MIN2(e, en);
            break;
        case 0:
            e = WM2ij;
            if (e != INF) e += E_MLstem(o, tt, -1, -1) + P->MLclosing;
            break;
    }
    return e;
}

static void compute_WMv_WMp(oracle *o, int i, int j, int WMB) { /* s_energy_matrix.cc:206-217 */
    if (j - i + 1 < 4) return;
    size_t ij = D2(o, i, j), ijm1 = D2(o, i, j - 1);
    int v = E_MLStem(o, getV(o, i, j), getV(o, i + 1, j), getV(o, i, j - 1), getV(o, i + 1, j - 1), i, j);
    int p = WMB + o->pen.PSM + o->pen.b;
    int t = o->WMv[ijm1] + o->P->MLbase;
    o->WMv[ij] = MIN2(v, t);
    t = o->WMp[ijm1] + o->P->MLbase;
    o->WMp[ij] = MIN2(p, t);
}

static void compute_energy_WM(oracle *o, int i, int j) { /* s_energy_matrix.cc:219-241 */
    if (j - i + 1 < 4) return;
    int m1 = INF, m2 = INF, m3 = INF, m4 = INF, m5;
    for (int k = j - TURN - 1; k >= i; --k) {
        int wm_kj = E_MLStem(o, getV(o, k, j), getV(o, k + 1, j), getV(o, k, j - 1), getV(o, k + 1, j - 1), k, j);
        int wmb_kj = o->Pm[D2(o, k, j)] + o->pen.PSM + o->pen.b;
        int base = (k - i) * o->P->MLbase;
        m1 = MIN2(m1, base + wm_kj);
        m2 = MIN2(m2, base + wmb_kj);
        m3 = MIN2(m3, getWM(o, i, k - 1) + wm_kj);
        m4 = MIN2(m4, getWM(o, i, k - 1) + wmb_kj);
    }
    m5 = o->WM[D2(o, i, j - 1)] + o->P->MLbase;
    int r = MIN2(MIN2(m1, m2), MIN2(MIN2(m3, m4), m5));
    o->WM[D2(o, i, j)] = r;
}

static int compute_energy_VM(const oracle *o, int i, int j) { /* s_energy_matrix.cc:243-268 */
    int mn = INF, MLb = o->P->MLbase;
    for (int k = i + 1; k <= j - 3; ++k) {
        int a = getWM(o, i + 1, k - 1) + getWMv(o, k, j - 1);
        a = MIN2(a, getWM(o, i + 1, k - 1) + getWMp(o, k, j - 1));
        a = MIN2(a, (k - i - 1) * MLb + getWMp(o, k, j - 1));
        int b = getWM(o, i + 2, k - 1) + getWMv(o, k, j - 1);
        b = MIN2(b, getWM(o, i + 2, k - 1) + getWMp(o, k - 1, j - 1)); /* sic: A-Q7 */
        b = MIN2(b, (k - (i + 1) - 1) * MLb + getWMp(o, k, j - 1));
        int c = getWM(o, i + 1, k - 1) + getWMv(o, k, j - 2);
        c = MIN2(c, getWM(o, i + 1, k - 1) + getWMp(o, k, j - 2));
        c = MIN2(c, (k - i - 1) * MLb + getWMp(o, k, j - 2));
        int d = getWM(o, i + 2, k - 1) + getWMv(o, k, j - 2);
        d = MIN2(d, getWM(o, i + 2, k - 1) + getWMp(o, k, j - 2));
        d = MIN2(d, (k - (i + 1) - 1) * MLb + getWMp(o, k, j - 2));
        mn = MIN2(mn, E_MbLoop(o, a, b, c, d, i, j));
    }
    return mn;
}

static void compute_V(oracle *o, int i, int j) { /* s_energy_matrix.cc:315-358 */
    int en[3];
    int tc = ptype(o, i, j);
    /* HairpinE :275-282 */
    en[0] = (tc == 0) ? INF : E_Hairpin(o, j - i - 1, tc, o->S1[i + 1], o->S1[j - 1], o->seq + i - 1);
    /* compute_internal :287-299 */
    int v_iloop = INF;
    int max_k = MIN2(j - TURN - 2, i + MAXLOOP + 1);
    for (int k = i + 1; k <= max_k; ++k) {
        int a = k + TURN + 1 + MAXLOOP + 2, b = k + j - i;
        int min_l = (a > b ? a : b) - MAXLOOP - 2;
        for (int l = j - 1; l >= min_l; --l) {
            int e = E_IntLoop(o, k - i - 1, j - l - 1, tc, o->rtype[ptype(o, k, l)], o->S1[i + 1],
                              o->S1[j - 1], o->S1[k - 1], o->S1[l + 1]) + getV(o, k, l);
            v_iloop = MIN2(v_iloop, e);
        }
    }
    en[1] = v_iloop;
    en[2] = compute_energy_VM(o, i, j);
    int mn = INF / 2, rank = -1;
    for (int k = 0; k < 3; ++k)
        if (en[k] < mn) { mn = en[k]; rank = k; }
    char type = rank == 0 ? 'H' : rank == 1 ? 'I' : rank == 2 ? 'M' : 'N';
    if (mn < INF / 2) { o->V[D2(o, i, j)] = mn; o->Vt[D2(o, i, j)] = type; }
}

/* ---- pseudo_loop.cc 2-D ---- */
static void compute_WBP(oracle *o, int i, int l) { /* :134-148 */
    int b1 = INF, b2 = INF;
    for (int d = i; d < l; ++d) {
        int wb = get_WB(o, i, d - 1);
        b1 = MIN2(b1, wb + getV(o, d, l) + o->pen.bp + o->pen.PPS);
        b2 = MIN2(b2, wb + tri_get(o, o->Pm, d, l) + o->pen.PSM + o->pen.PPS);
    }
    int b3 = tri_get(o, o->WBP, i, l - 1) + o->pen.cp;
    int m = MIN2(MIN2(b1, b2), b3);
    if (m < INF / 2) o->WBP[D2(o, i, l)] = m;
}
static void compute_WPP(oracle *o, int i, int l) { /* :150-164 */
    int b1 = INF, b2 = INF;
    for (int d = i; d < l; ++d) {
        int wp = get_WP(o, i, d - 1);
        b1 = MIN2(b1, wp + getV(o, d, l) + 0 + o->pen.PPS);
        b2 = MIN2(b2, wp + tri_get(o, o->Pm, d, l) + o->pen.PSP + o->pen.PPS);
    }
    int b3 = tri_get(o, o->WPP, i, l - 1) + o->pen.PUP;
    int m = MIN2(MIN2(b1, b2), b3);
    if (m < INF / 2) o->WPP[D2(o, i, l)] = m;
}
static void compute_P(oracle *o, int i, int l) { /* :166-179 */
    int m = INF;
    for (int j = i; j < l; ++j)
        for (int d = j + 1; d < l; ++d)
            for (int k = d + 1; k < l; ++k) {
                int b1 = get4(o, PK, i, j, d + 1, k) + get4(o, PK, j + 1, d, k + 1, l);
                m = MIN2(m, b1);
            }
    if (m < INF / 2) o->Pm[D2(o, i, l)] = m;
}

/* ---- pseudo_loop.cc 4-D ---- */
#define SETIF(mat, e) do { if ((e) < INF / 2) set4(o, mat, i, j, k, l, (e)); } while (0)

static int get_PLiloop(const oracle *o, int i, int j, int k, int l) { /* :682-703 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (!can_pair(o, i, j)) return INF;
    int m = INF;
    if (i + TURN + 2 < j) m = get4(o, PL, i + 1, j - 1, k, l) + get_e_stP(o, i, j);
    int max_d = MIN2(j, i + MAXLOOP);
    for (int d = i + 1; d < max_d; ++d) {
        int min_dp = d + TURN > j - MAXLOOP ? d + TURN : j - MAXLOOP;
        for (int dp = j - 1; dp > min_dp; --dp) {
            if (!can_pair(o, d, dp)) continue;
            m = MIN2(m, get_e_intP(o, i, d, dp, j) + get4(o, PL, d, dp, k, l));
        }
    }
    return m;
}
static int get_PRiloop(const oracle *o, int i, int j, int k, int l) { /* :717-738 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (!can_pair(o, k, l)) return INF;
    int m = INF;
    if (k + TURN + 2 < l) m = get4(o, PR, i, j, k + 1, l - 1) + get_e_stP(o, k, l);
    int max_d = MIN2(l, k + MAXLOOP);
    for (int d = k + 1; d < max_d; ++d) {
        int min_dp = d + TURN > l - MAXLOOP ? d + TURN : l - MAXLOOP;
        for (int dp = l - 1; dp > min_dp; --dp) {
            if (!can_pair(o, d, dp)) continue;
            m = MIN2(m, get_e_intP(o, k, d, dp, l) + get4(o, PR, i, j, d, dp));
        }
    }
    return m;
}
static int get_PMiloop(const oracle *o, int i, int j, int k, int l) { /* :752-773 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (!can_pair(o, j, k)) return INF;
    int m = INF;
    if (i < j && k < l) m = get4(o, PM, i, j - 1, k + 1, l) + get_e_stP(o, j - 1, k + 1);
    int max_d = i > j - MAXLOOP ? i : j - MAXLOOP;
    for (int d = j - 1; d > max_d; --d) {
        int min_dp = MIN2(l, k + MAXLOOP);
        for (int dp = k + 1; dp < min_dp; ++dp) {
            if (!can_pair(o, d, dp)) continue;
            m = MIN2(m, get_e_intP(o, d, j, k, dp) + get4(o, PM, i, d, dp, l));
        }
    }
    return m;
}
static int get_POiloop(const oracle *o, int i, int j, int k, int l) { /* :787-808 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (!can_pair(o, i, l)) return INF;
    int m = INF;
    if (i < j && k < l) m = get4(o, PO, i + 1, j, k, l - 1) + get_e_stP(o, i, l);
    int max_d = MIN2(j, i + MAXLOOP);
    for (int d = i + 1; d < max_d; ++d) {
        int min_dp = l - MAXLOOP > k ? l - MAXLOOP : k;
        for (int dp = l - 1; dp > min_dp; --dp) {
            if (!can_pair(o, d, dp)) continue;
            m = MIN2(m, get_e_intP(o, i, d, dp, l) + get4(o, PO, d, j, dp, k));
        }
    }
    return m;
}
static int get_PfromMdoubleprime(const oracle *o, int i, int j, int k, int l) { /* :663-679 */
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (i == j && k == l) return ptype(o, i, l) == 0 ? INF : 0;
    int b1 = get4(o, PL, i, j, k, l) + o->pen.PB;
    int b2 = get4(o, PR, i, j, k, l) + o->pen.PB;
    return MIN2(b1, b2);
}

static void compute_cell(oracle *o, int i, int j, int k, int l) {
    const ccj_pk_penalties *pe = &o->pen;
    int bp = pe->bp, cp = pe->cp, ap = pe->ap, PB = pe->PB;
    int m, t;
    /* PLmloop00 :445-463 */
    m = get4(o, PL, i, j, k, l) + bp;
    for (int d = i; d <= j; ++d) {
        if (d > i) { t = get_WB(o, i, d - 1) + get4(o, PLmloop00, d, j, k, l); m = MIN2(m, t); }
        if (d < j) { t = get4(o, PLmloop00, i, d, k, l) + get_WB(o, d + 1, j); m = MIN2(m, t); }
    }
    SETIF(PLmloop00, m);
    /* PLmloop01 :465-476 */
    m = INF;
    for (int d = i; d < j; ++d) { t = get4(o, PLmloop00, i, d, k, l) + tri_get(o, o->WBP, d + 1, j); m = MIN2(m, t); }
    SETIF(PLmloop01, m);
    /* PLmloop10 :478-493 */
    m = INF;
    for (int d = i + 1; d <= j; ++d) {
        t = tri_get(o, o->WBP, i, d - 1) + get4(o, PLmloop00, d, j, k, l); m = MIN2(m, t);
        if (d < j) { t = get4(o, PLmloop10, i, d, k, l) + get_WB(o, d + 1, j); m = MIN2(m, t); }
    }
    SETIF(PLmloop10, m);
    /* PRmloop00 :495-513 */
    m = get4(o, PR, i, j, k, l) + bp;
    for (int d = k; d <= l; ++d) {
        if (d > k) { t = get_WB(o, k, d - 1) + get4(o, PRmloop00, i, j, d, l); m = MIN2(m, t); }
        if (d < l) { t = get4(o, PRmloop00, i, j, k, d) + get_WB(o, d + 1, l); m = MIN2(m, t); }
    }
    SETIF(PRmloop00, m);
    /* PRmloop01 :516-528 */
    m = get4(o, PRmloop01, i, j, k, l - 1) + cp;
    for (int d = k; d < l; ++d) { t = get4(o, PRmloop00, i, j, k, d) + tri_get(o, o->WBP, d + 1, l); m = MIN2(m, t); }
    SETIF(PRmloop01, m);
    /* PRmloop10 :530-542 */
    m = get4(o, PRmloop10, i, j, k + 1, l) + cp;
    for (int d = k + 1; d <= l; ++d) { t = tri_get(o, o->WBP, k, d - 1) + get4(o, PRmloop00, i, j, d, l); m = MIN2(m, t); }
    SETIF(PRmloop10, m);
    /* PMmloop00 :544-560 */
    m = get4(o, PM, i, j, k, l) + bp;
    for (int d = i; d < j; ++d) { t = get4(o, PMmloop00, i, d, k, l) + get_WB(o, d + 1, j); m = MIN2(m, t); }
    for (int d = k + 1; d <= l; ++d) { t = get4(o, PMmloop00, i, j, d, l) + get_WB(o, k, d - 1); m = MIN2(m, t); }
    SETIF(PMmloop00, m);
    /* PMmloop01 :563-575 */
    m = get4(o, PMmloop01, i, j, k + 1, l) + cp;
    for (int d = k; d < l; ++d) { t = get4(o, PMmloop00, i, j, k, d) + tri_get(o, o->WBP, d + 1, l); m = MIN2(m, t); }
    SETIF(PMmloop01, m);
    /* PMmloop10 :577-593 */
    m = get4(o, PMmloop10, i, j - 1, k, l) + cp;
    for (int d = i + 1; d <= j; ++d) { t = tri_get(o, o->WBP, i, d - 1) + get4(o, PMmloop00, d, j, k, l); m = MIN2(m, t); }
    for (int d = k + 1; d < l; ++d) { t = get4(o, PMmloop10, i, j, k, d) + get_WB(o, d + 1, l); m = MIN2(m, t); }
    SETIF(PMmloop10, m);
    /* POmloop00 :595-612 */
    m = get4(o, PO, i, j, k, l) + bp;
    for (int d = i + 1; d <= j; ++d) { t = get_WB(o, i, d - 1) + get4(o, POmloop00, d, j, k, l); m = MIN2(m, t); }
    for (int d = k; d < l; ++d) { t = get4(o, POmloop00, i, j, k, d) + get_WB(o, d + 1, l); m = MIN2(m, t); }
    SETIF(POmloop00, m);
    /* POmloop01 :615-627 */
    m = INF;
    for (int d = k; d < l; ++d) { t = get4(o, POmloop00, i, j, k, d) + tri_get(o, o->WBP, d + 1, l); m = MIN2(m, t); }
    SETIF(POmloop01, m);
    /* POmloop10 :629-644 */
    m = INF;
    for (int d = i + 1; d <= j; ++d) { t = tri_get(o, o->WBP, i, d - 1) + get4(o, POmloop00, d, j, k, l); m = MIN2(m, t); }
    for (int d = k + 1; d < l; ++d) { t = get4(o, POmloop10, i, j, k, d) + get_WB(o, d + 1, l); m = MIN2(m, t); }
    SETIF(POmloop10, m);

    /* PL :232-253 */
    {
        int b1 = INF, b2 = INF, b3 = INF;
        if (ptype(o, i, j) > 0) {
            b1 = get_PLiloop(o, i, j, k, l);
            int x = get4(o, PLmloop10, i + 1, j - 1, k, l) + ap + bp;  /* get_PLmloop :705-715 */
            int y = get4(o, PLmloop01, i + 1, j - 1, k, l) + ap + bp;
            b2 = MIN2(x, y) + bp;
            if (j >= i + TURN + 1) b3 = get4(o, PfromL, i + 1, j - 1, k, l);
        }
        m = MIN2(MIN2(b1, b2), b3);
        SETIF(PL, m);
    }
    /* PR :255-275 */
    {
        int b1 = INF, b2 = INF, b3 = INF;
        if (ptype(o, k, l) > 0) {
            b1 = get_PRiloop(o, i, j, k, l);
            int x = get4(o, PRmloop10, i, j, k + 1, l - 1) + ap + bp;  /* :740-750 */
            int y = get4(o, PRmloop01, i, j, k + 1, l - 1) + ap + bp;
            b2 = MIN2(x, y) + bp;
            if (l >= k + TURN + 1) b3 = get4(o, PfromR, i, j, k + 1, l - 1);
        }
        m = MIN2(MIN2(b1, b2), b3);
        SETIF(PR, m);
    }
    /* PM :277-300 */
    {
        int b1 = INF, b2 = INF, b3 = INF, b4 = INF;
        if (ptype(o, j, k) > 0) {
            b1 = get_PMiloop(o, i, j, k, l);
            int x = get4(o, PMmloop10, i, j - 1, k + 1, l) + ap + bp;  /* :775-785 */
            int y = get4(o, PMmloop01, i, j - 1, k + 1, l) + ap + bp;
            b2 = MIN2(x, y) + bp;
            if (k >= j + TURN - 1) b3 = get4(o, PfromM, i, j - 1, k + 1, l);
            if (i == j && k == l) b4 = 0;
        }
        m = MIN2(MIN2(b1, b2), MIN2(b3, b4));
        SETIF(PM, m);
    }
    /* PO :302-322 */
    {
        int b1 = INF, b2 = INF, b3 = INF;
        if (ptype(o, i, l) > 0) {
            b1 = get_POiloop(o, i, j, k, l);
            int x = get4(o, POmloop10, i + 1, j, k, l - 1) + ap + bp;  /* :810-820 */
            int y = get4(o, POmloop01, i + 1, j, k, l - 1) + ap + bp;
            b2 = MIN2(x, y) + bp;
            if (l >= i + TURN + 1) b3 = get4(o, PfromO, i + 1, j, k, l - 1);
        }
        m = MIN2(MIN2(b1, b2), b3);
        SETIF(PO, m);
    }
    /* PfromL :354-374 */
    {
        int b1 = INF, b2 = INF;
        for (int d = i + 1; d < j; ++d) {
            t = get4(o, PfromL, d, j, k, l) + get_WP(o, i, d - 1); b1 = MIN2(b1, t);
            t = get4(o, PfromL, i, d, k, l) + get_WP(o, d + 1, j); b2 = MIN2(b2, t);
        }
        int b3 = get4(o, PR, i, j, k, l) + PB;
        int b4 = get4(o, PM, i, j, k, l) + PB;
        int b5 = get4(o, PO, i, j, k, l) + PB;
        m = MIN2(MIN2(b1, b2), MIN2(MIN2(b3, b4), b5));
        SETIF(PfromL, m);
    }
    /* PfromR :376-394 */
    {
        int b1 = INF, b2 = INF;
        for (int d = k + 1; d < l; ++d) {
            t = get4(o, PfromR, i, j, d, l) + get_WP(o, k, d - 1); b1 = MIN2(b1, t);
            t = get4(o, PfromR, i, j, k, d) + get_WP(o, d + 1, l); b2 = MIN2(b2, t);
        }
        int b3 = get4(o, PM, i, j, k, l) + PB;
        int b4 = get4(o, PO, i, j, k, l) + PB;
        m = MIN2(MIN2(b1, b2), MIN2(b3, b4));
        SETIF(PfromR, m);
    }
    /* PfromM :396-407 */
    m = INF;
    for (int d = i + 1; d < j; ++d) { t = get4(o, PfromMprime, i, d, k, l) + get_WP(o, d + 1, j); m = MIN2(m, t); }
    SETIF(PfromM, m);
    /* PfromMprime :409-420 */
    m = INF;
    for (int d = k + 1; d < l; ++d) { t = get_PfromMdoubleprime(o, i, j, d, l) + get_WP(o, k, d - 1); m = MIN2(m, t); }
    SETIF(PfromMprime, m);
    /* PfromO :422-443 */
    {
        int b1 = INF, b2 = INF;
        for (int d = i + 1; d < j; ++d) { t = get4(o, PfromO, d, j, k, l) + get_WP(o, i, d - 1); b1 = MIN2(b1, t); }
        for (int d = k + 1; d < l; ++d) { t = get4(o, PfromO, i, j, k, d) + get_WP(o, d + 1, l); b2 = MIN2(b2, t); }
        int b3 = get4(o, PL, i, j, k, l) + PB;
        int b4 = get4(o, PR, i, j, k, l) + PB;
        m = MIN2(MIN2(b1, b2), MIN2(b3, b4));
        SETIF(PfromO, m);
    }
    /* PK :181-202 */
    {
        int b1 = INF, b2 = INF;
        for (int d = i + 1; d < j; ++d) { t = get4(o, PK, i, d, k, l) + get_WP(o, d + 1, j); b1 = MIN2(b1, t); }
        for (int d = k + 1; d < l; ++d) { t = get4(o, PK, i, j, d, l) + get_WP(o, k, d - 1); b2 = MIN2(b2, t); }
        int b3 = get4(o, PL, i, j, k, l) + PB;
        int b4 = get4(o, PM, i, j, k, l) + PB;
        int b5 = get4(o, PR, i, j, k, l) + PB;
        int b6 = get4(o, PO, i, j, k, l) + PB;
        m = MIN2(MIN2(MIN2(b1, b2), MIN2(b3, b4)), MIN2(b5, b6));
        SETIF(PK, m);
    }
}

static int E_ext_Stem(const oracle *o, int vij, int vi1j, int vij1, int vi1j1, int i, int j) {
    /* W_final.cc:118-173 */
    const short *S = o->S;
    int n = o->n, e = INF, en;
    int tt = o->pair[S[i]][S[j]];
    en = vij;
    if (en != INF) {
        if (o->dangles == 2) en += E_ExtLoop(o, tt, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1);
        else en += E_ExtLoop(o, tt, -1, -1);
        e = MIN2(e, en);
    }
    if (o->dangles == 1) {
        tt = o->pair[S[i + 1]][S[j]];
        en = (j - i - 1 > TURN) ? vi1j : INF;
        if (en != INF) en += E_ExtLoop(o, tt, S[i], -1);
        e = MIN2(e, en);
        tt = o->pair[S[i]][S[j - 1]];
        en = (j - 1 - i > TURN) ? vij1 : INF;
        if (en != INF) en += E_ExtLoop(o, tt, -1, S[j]);
        e = MIN2(e, en);
        tt = o->pair[S[i + 1]][S[j - 1]];
        en = (j - 1 - i - 1 > TURN) ? vi1j1 : INF;
        if (en != INF) en += E_ExtLoop(o, tt, S[i], S[j]);
        e = MIN2(e, en);
    }
    return e;
}

/* ------------------------------------------------------------------------------------------ */
/* public C API (ctypes)                                                                       */
/* ------------------------------------------------------------------------------------------ */
void ccj_oracle_free(oracle *o);

static oracle *oracle_alloc(const char *seq, const ccj_energy_params *P, int dangles, int noGU) {
    oracle *o = (oracle *)calloc(1, sizeof(oracle));
    int n = (int)strlen(seq);
    o->n = n;
    o->dangles = dangles;
    o->P = P;
    ccj_pk_penalties pen = CCJ_PK_PENALTIES_DEFAULT;
    o->pen = pen;
    o->seq = strdup(seq);
    /* make_pair_matrix, pair_mat.h:81-155 */
    int base_rtype[8] = {0, 2, 1, 4, 3, 6, 5, 7};
    memcpy(o->rtype, base_rtype, sizeof(base_rtype));
    for (int a = 0; a < 8; ++a)
        for (int b = 0; b < 8; ++b) o->pair[a][b] = BP_pair[a][b];
    if (noGU) o->pair[3][4] = o->pair[4][3] = 0;
    for (int a = 0; a < 8; ++a)
        for (int b = 0; b < 8; ++b) o->rtype[o->pair[a][b]] = o->pair[b][a];
    /* encode_sequence, pair_mat.h:159-183 */
    o->S = (short *)calloc((size_t)n + 2, sizeof(short));
    o->S1 = (short *)calloc((size_t)n + 2, sizeof(short));
    for (int i = 1; i <= n; ++i) o->S[i] = o->S1[i] = (short)encode_char(seq[i - 1]);
    o->S[n + 1] = o->S[1]; o->S[0] = (short)n;
    o->S1[n + 1] = o->S1[1]; o->S1[0] = o->S1[n];

    size_t n2 = (size_t)(n + 2) * (size_t)(n + 2);
    o->V = (int *)malloc(n2 * sizeof(int));
    o->Vt = (char *)malloc(n2);
    o->WM = (int *)malloc(n2 * sizeof(int));
    o->WMv = (int *)malloc(n2 * sizeof(int));
    o->WMp = (int *)malloc(n2 * sizeof(int));
    o->Pm = (int *)malloc(n2 * sizeof(int));
    o->WBP = (int *)malloc(n2 * sizeof(int));
    o->WPP = (int *)malloc(n2 * sizeof(int));
    for (size_t x = 0; x < n2; ++x) {
        o->V[x] = 10000; o->Vt[x] = 'N';          /* h_struct.hh:94-103 */
        o->WM[x] = o->WMv[x] = o->WMp[x] = INF + 1; /* matrices.hh:25 */
        o->Pm[x] = o->WBP[x] = o->WPP[x] = INF + 1;
    }
    o->W = (int *)calloc((size_t)n + 1, sizeof(int));

    /* Matrix4D::construct_index, matrices.hh:208-221 */
    if (n >= 1) {
        o->idx2 = (size_t *)malloc((size_t)n * n * sizeof(size_t));
        size_t idx = 0;
        for (int i = 0; i < n; ++i)
            for (int j = i; j < n; ++j) {
                o->idx2[(size_t)i * n + (size_t)j] = idx;
                for (int k = j; k < n; ++k) idx += (size_t)(n - k);
            }
        o->slice = idx;
        o->eint = (int *)malloc((size_t)(n + 2) * (size_t)(n + 2) * EW * EW * sizeof(int));
        if (!o->eint) { ccj_oracle_free(o); return NULL; }
#pragma omp parallel for schedule(dynamic, 1)
        for (int p = 1; p <= n; ++p)
            for (int q = p + 1; q <= n; ++q)
                for (int u1 = 0; u1 < EW; ++u1)
                    for (int u2 = 0; u2 < EW; ++u2) {
                        int ip = p + 1 + u1, jp = q - 1 - u2;
                        o->eint[((size_t)p * (size_t)(n + 2) + (size_t)q) * EW * EW + (size_t)u1 * EW + (size_t)u2] =
                            ip < jp ? get_e_intP_direct(o, p, ip, jp, q) : INF;
                    }
        for (int m = 0; m < NMAT4; ++m) {
            o->M4[m] = (int16_t *)malloc(o->slice * sizeof(int16_t));
            if (!o->M4[m]) { ccj_oracle_free(o); return NULL; }
#pragma omp parallel for schedule(static)
            for (size_t x = 0; x < o->slice; ++x) o->M4[m][x] = INTERN_INF;
        }
    }

    return o;
}

static void oracle_exterior(oracle *o) {
    /* exterior, W_final.cc:68-77 */
    int n = o->n;
    for (int j = TURN + 1; j <= n; ++j) {
        int m1 = o->W[j - 1], m2 = INF, m3 = INF;
        for (int k = 1; k <= j - TURN - 1; ++k) {
            int acc = (k > 1) ? o->W[k - 1] : 0;
            int e = E_ext_Stem(o, getV(o, k, j), getV(o, k + 1, j), getV(o, k, j - 1), getV(o, k + 1, j - 1), k, j);
            m2 = MIN2(m2, acc + e);
            int p1 = tri_get(o, o->Pm, k, j), p2 = tri_get(o, o->Pm, k + 1, j);
            int p3 = tri_get(o, o->Pm, k, j - 1), p4 = tri_get(o, o->Pm, k + 1, j - 1);
            int pm = MIN2(MIN2(p1, p2), MIN2(p3, p4));
            m3 = MIN2(m3, acc + pm + o->pen.PS);
        }
        o->W[j] = MIN2(MIN2(m1, m2), m3);
    }
}


oracle *ccj_oracle_fold(const char *seq, const ccj_energy_params *P, int dangles, int noGU) {
    oracle *o = oracle_alloc(seq, P, dangles, noGU);
    if (!o) return NULL;
    int n = o->n;
    /* fill, W_final.cc:60-67 and pseudo_loop.cc:69-132 */
    for (int i = n; i >= 1; --i)
        for (int l = i; l <= n; ++l) {
            compute_V(o, i, l);
            compute_P(o, i, l);
            compute_WBP(o, i, l);
            compute_WPP(o, i, l);
            for (int j = i; j < l; ++j)
                for (int k = l; k >= j + 2; --k) compute_cell(o, i, j, k, l);
            compute_WMv_WMp(o, i, l, tri_get(o, o->Pm, i, l));
            compute_energy_WM(o, i, l);
        }
    oracle_exterior(o);
    return o;
}

/*
 * Level-parallel restatement of the same fill, for the sizes the
 * sequential loop cannot reach in a test budget (config 5, n=400).  Write a cell as (i,j,k,l),
 * a = j-i, b = l-k, level t = a+b.  Every 4-D read of the reference recurrences
 * (pseudo_loop.cc:181-820) other than the same cell targets a level < t; every 2-D value a level-t
 * cell reads has span <= t-1; a 2-D interval of span s (s_energy_matrix.cc:206-358,
 * pseudo_loop.cc:134-179) reads only 4-D levels <= s-3, 2-D spans < s and, for WBP/WPP/WMv/WM, the
 * V/P of its own interval, which the reference computes first (W_final.cc:60-67).  So
 *     for t = 0..n:  all intervals of span t-1 (each in the reference's per-interval order),
 *                    then all cells of level t (each in compute_cell's in-cell order)
 * reads exactly the values the reference's i-descending / l-ascending loop reads; the intervals of
 * one span and the cells of one level are independent and run on OpenMP threads.
 * tests/test_oracle.py checks this mode against the reference's hashes and the sequential mode.
 */
static void fill_span(oracle *o, int s) {
    int n = o->n;
#pragma omp parallel for schedule(dynamic, 1)
    for (int i = n - s; i >= 1; --i) {
        int l = i + s;
        compute_V(o, i, l);
        compute_P(o, i, l);
        compute_WBP(o, i, l);
        compute_WPP(o, i, l);
        compute_WMv_WMp(o, i, l, tri_get(o, o->Pm, i, l));
        compute_energy_WM(o, i, l);
    }
}

static void fill_level(oracle *o, int t) {
    int n = o->n;
    long rows = (long)n * (t + 1);  /* (i, a) pairs */
#pragma omp parallel for schedule(dynamic, 4)
    for (long x = 0; x < rows; ++x) {
        int i = (int)(x / (t + 1)) + 1, a = (int)(x % (t + 1)), b = t - a;
        int j = i + a;
        for (int k = j + 2; k + b <= n; ++k) compute_cell(o, i, j, k, k + b);
    }
}

oracle *ccj_oracle_fold_par(const char *seq, const ccj_energy_params *P, int dangles, int noGU, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    oracle *o = oracle_alloc(seq, P, dangles, noGU);
    if (!o) return NULL;
    int n = o->n;
    int progress = getenv("CCJ_ORACLE_PROGRESS") != NULL;
    for (int t = 0; t <= n; ++t) {
        if (t >= 1) fill_span(o, t - 1);
        if (t <= n - 3) fill_level(o, t);
        if (progress && t % 10 == 0) { fprintf(stderr, "oracle level %d/%d\n", t, n); fflush(stderr); }
    }
    oracle_exterior(o);
    return o;
}

void ccj_oracle_free(oracle *o) {
    if (!o) return;
    free(o->seq); free(o->S); free(o->S1);
    free(o->V); free(o->Vt); free(o->WM); free(o->WMv); free(o->WMp);
    free(o->Pm); free(o->WBP); free(o->WPP); free(o->W); free(o->idx2); free(o->eint);
    for (int m = 0; m < NMAT4; ++m) free(o->M4[m]);
    free(o);
}

int ccj_oracle_n(const oracle *o) { return o->n; }
int ccj_oracle_W(const oracle *o, int j) { return o->W[j]; }

/* reference getter semantics (matrices.hh:177-182) */
int ccj_oracle_get4(const oracle *o, int m, int i, int j, int k, int l) { return get4(o, m, i, j, k, l); }

/* raw 2-D value for 1 <= i <= j <= n: 0 P, 1 WBP, 2 WPP, 3 V, 4 Vtype, 5 WM, 6 WMv, 7 WMp */
int ccj_oracle_get2(const oracle *o, int m, int i, int j) {
    size_t x = D2(o, i, j);
    switch (m) {
        case 0: return o->Pm[x];
        case 1: return o->WBP[x];
        case 2: return o->WPP[x];
        case 3: return o->V[x];
        case 4: return o->Vt[x];
        case 5: return o->WM[x];
        case 6: return o->WMv[x];
        case 7: return o->WMp[x];
    }
    return 0;
}

static uint64_t fnv(uint64_t h, const void *p, size_t n) {
    const unsigned char *c = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
    return h;
}

/* 22 + 8 + 1 hashes in ref_driver order: 4-D matrices, P WBP WPP V Vtype WM WMv WMp, W */
void ccj_oracle_hashes(const oracle *o, uint64_t *out) {
    int n = o->n;
#pragma omp parallel for schedule(dynamic, 1)
    for (int m = 0; m < NMAT4; ++m) {
        uint64_t h = 1469598103934665603ull;
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j)
                for (int k = j + 2; k <= n; ++k)
                    for (int l = k; l <= n; ++l) {
                        int16_t v = (int16_t)get4(o, m, i, j, k, l);
                        h = fnv(h, &v, 2);
                    }
        out[m] = h;
    }
    for (int m = 0; m < 8; ++m) {
        uint64_t h = 1469598103934665603ull;
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j) {
                int32_t v = ccj_oracle_get2(o, m, i, j);
                h = fnv(h, &v, 4);
            }
        out[NMAT4 + m] = h;
    }
    uint64_t h = 1469598103934665603ull;
    for (int j = 0; j <= n; ++j) { int32_t v = o->W[j]; h = fnv(h, &v, 4); }
    out[NMAT4 + 8] = h;
}
