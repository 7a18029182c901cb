/*
 * ccj_params.h — on-disk / in-memory energy parameter blob for the CCJ MFE engine.
 *
 * This is the MI355X engine's own table format (the "mmapped Turner/DP energy tables" of the
 * north star).  It holds exactly the temperature-scaled (37 C) fields of ViennaRNA's
 * vrna_param_t that the CCJ path reads, plus the ViennaRNA global
 * MAX_NINIO.  Field meaning follows the reference:
 *   reference: src/ViennaRNA/params/basic.h:57-115   (struct vrna_param_s)
 *              src/ViennaRNA/params/params.c:399-555 (get_scaled_params, tempf == 1.0 at 37 C)
 *              src/ViennaRNA/params/default.c:71     (MAX_NINIO global)
 * All arrays keep ViennaRNA's index order, including pair type 0 and base code 0 rows, because
 * the reference reads type-0 rows for non-canonical pairs.
 *
 * Plain C, fixed-width fields, little endian, no pointers: the same struct is mmapped on the
 * host and copied verbatim to device memory.
 */
#ifndef CCJ_PARAMS_H
#define CCJ_PARAMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCJ_PARAMS_MAGIC   0x504a4343u /* "CCJP" little endian */
#define CCJ_PARAMS_VERSION 1u

#define CCJ_NBPAIRS 7   /* reference: ViennaRNA/params/constants.h NBPAIRS */
#define CCJ_MAXLOOP 30  /* reference: ViennaRNA/params/constants.h:29 */
#define CCJ_TURN    3   /* reference: ViennaRNA/params/constants.h:27 */
#define CCJ_INF     10000000 /* reference: matrices.hh:10, params/constants.h:17 */

typedef struct ccj_energy_params {
    uint32_t magic;
    uint32_t version;
    uint32_t size_bytes;   /* sizeof(ccj_energy_params) */
    uint32_t special_hp;   /* model_details.special_hp (1 in the reference) */

    int32_t stack[8][8];
    int32_t hairpin[31];
    int32_t bulge[31];
    int32_t internal_loop[31];
    int32_t mismatchExt[8][5][5];
    int32_t mismatchI[8][5][5];
    int32_t mismatch1nI[8][5][5];
    int32_t mismatch23I[8][5][5];
    int32_t mismatchH[8][5][5];
    int32_t mismatchM[8][5][5];
    int32_t dangle5[8][5];
    int32_t dangle3[8][5];
    int32_t int11[8][8][5][5];
    int32_t int21[8][8][5][5][5];
    int32_t int22[8][8][5][5][5][5];
    int32_t ninio2;        /* vrna_param_t::ninio[2] */
    int32_t max_ninio;     /* ViennaRNA global MAX_NINIO */
    int32_t MLbase;
    int32_t MLclosing;
    int32_t TerminalAU;
    int32_t MLintern[8];
    int32_t pad0;
    double  lxc;           /* vrna_param_t::lxc */
    int32_t Tetraloop_E[200];
    int32_t Triloop_E[40];
    int32_t Hexaloop_E[40];
    char    Tetraloops[1408];  /* NUL-terminated, 7 chars per entry ("GAAAC " style) */
    char    Triloops[248];     /* 6 chars per entry */
    char    Hexaloops[1808];   /* 9 chars per entry */
} ccj_energy_params;

/* Hard-coded HotKnots-v2 / DP09 pseudoknot penalties (reference: h_globals.hh:7-25). */
typedef struct ccj_pk_penalties {
    int32_t PS, PSM, PSP, PB, PUP, PPS;
    int32_t a, b, c, ap, bp, cp;
    double  e_stP, e_intP;
} ccj_pk_penalties;

#define CCJ_PK_PENALTIES_DEFAULT \
    { -138, 1007, 1500, 246, 6, 96, 339, 3, 2, 341, 56, 12, 0.89, 0.74 }

#ifdef __cplusplus
}
#endif

#endif /* CCJ_PARAMS_H */
