/*
 * ccj_pf.h — C ABI of the CCJ partition function in libccj_hip.so.
 *
 * Replaces the reference's W_final_pf (src/part_func.hh:28-194): the constructor
 * (part_func.cc:31-93, Boltzmann tables of scale_pf_parameters() + rescale_pk_globals
 * :127-146 + exp_params_rescale :97-125), the fill ccj_pf() (part_func.cc:152-178: every
 * compute_* of :222-699 over the same 2-D / 4-D matrices) and the stochastic traceback
 * Sample_W/V/VM/WM/WMv/WMp (stoch_backtrack.cc:36-326).  The reference never compiles these
 * files into its binary (CMakeLists.txt:23,25) and never calls them (CCJ.cc:51-56,105); this ABI
 * is what a maintainer would bind to switch that path on.
 *
 * Semantics are the reference's as written, evaluated in IEEE double without contraction (the
 * oracle builds part_func.cc with -ffp-contract=off): every 4-D matrix stores the x86 int
 * truncation of its double sum (Matrix4DPF::set takes an int, matrices.hh:265-267, and get
 * returns int, :251-263), the P term multiplies those ints in 32-bit int arithmetic
 * (part_func.cc:388), expinternal[] is read past its 31 entries for pseudoknot interior loops
 * longer than 30 (part_func.cc:874 -> internal.h:645), and the recurrences keep the reference's
 * typos (POmloop00's '=' :673, PMmloop01 / POmloop10's '+' :645,695, get_WB/get_WP's '+'
 * :706,714).  DESIGN.md §10 lists them.
 *
 * Plain C types only.  Positions are 1-based like the reference.
 */
#ifndef CCJ_PF_H
#define CCJ_PF_H

#include <stdint.h>
#include "ccj.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CCJ_E_PF_SAMPLE 8 /* a Sample_* "backtracking failed" path: the reference prints and exit(0)s */
#define CCJ_E_PF_RANGE 10 /* ccj_pf_fill: some P(i,l) has sum |terms| >= 2^53, so the reference's serial
                             double sum of its int products (part_func.cc:383-393) could round
                             differently from the exact sum the GPU forms; no result is reported.
                             Only reachable for long sequences (never below n = 296). */

/* 4-D matrices of W_final_pf (part_func.hh:86-113), in canonical-hash order */
enum ccj_pf_mat4 {
    CCJ_PF_PK = 0, CCJ_PF_PL, CCJ_PF_PR, CCJ_PF_PM, CCJ_PF_PO,
    CCJ_PF_PfromL, CCJ_PF_PfromR, CCJ_PF_PfromM, CCJ_PF_PfromO,
    CCJ_PF_PLmloop00, CCJ_PF_PLmloop01, CCJ_PF_PLmloop10,
    CCJ_PF_PRmloop00, CCJ_PF_PRmloop01, CCJ_PF_PRmloop10,
    CCJ_PF_PMmloop00, CCJ_PF_PMmloop01, CCJ_PF_PMmloop10,
    CCJ_PF_POmloop00, CCJ_PF_POmloop01, CCJ_PF_POmloop10,
    CCJ_PF_NMAT4
};

/* 2-D matrices (TriangleMatrix_PF, part_func.hh:62,76-84) */
enum ccj_pf_mat2 {
    CCJ_PF_V = 0, CCJ_PF_VM, CCJ_PF_WM, CCJ_PF_WMv, CCJ_PF_WMp, CCJ_PF_WBP, CCJ_PF_WPP, CCJ_PF_P,
    CCJ_PF_NMAT2
};

typedef struct ccj_pf_ctx ccj_pf_ctx;

/* The raw 37 C tables the Boltzmann weights of the dangles and the multiloop / exterior
 * mismatches come from (ViennaRNA dangle5_37, dangle3_37, mismatchM37, mismatchExt37).  The MFE
 * blob holds them clamped to <= 0 (params.c:487-512), which loses their INF entries, while
 * get_scaled_exp_params smooths the raw values (SMOOTH(-INF) -> weight 1).  ccj_amd/params/<set>.pfraw
 * holds them for the bundled sets. */
#define CCJ_PF_RAW_MAGIC 0x52434343u /* "CCCR" */
typedef struct ccj_pf_raw {
    uint32_t magic;
    uint32_t size_bytes; /* sizeof(ccj_pf_raw) */
    int32_t dangle5[8][5];
    int32_t dangle3[8][5];
    int32_t mismatchM[8][5][5];
    int32_t mismatchExt[8][5][5];
} ccj_pf_raw;

/* W_final_pf(seq, MFE_structure, MFE_energy, dangle, num_samples, PSplot) minus the arguments the
 * reference ignores (MFE_structure and PSplot are stored only; MFE_energy only feeds a pf_scale
 * that exp_params_rescale then forces to 1, part_func.cc:101-107).  prob->params are the 37 C
 * tables; raw = their unclamped dangle / mismatch tables (NULL: the blob's values with the pair
 * type 0 rows taken as INF, which every shipped set has).  device = HIP ordinal. */
int ccj_pf_create(const ccj_problem *prob, const ccj_pf_raw *raw, int device, ccj_pf_ctx **out);
void ccj_pf_destroy(ccj_pf_ctx *ctx);
/* The device and host bytes ccj_pf_create allocates for a sequence of length n (its up-front size
 * check compares them with the device's free memory and the host's MemAvailable). */
void ccj_pf_footprint(int n, unsigned long long *device_bytes, unsigned long long *host_bytes);

/* ccj_pf(): the whole fill on the GPU, then W on the host.  *energy = to_Energy(W[n], n)
 * (part_func.cc:148-150,173). */
int ccj_pf_fill(ccj_pf_ctx *ctx, double *energy);

/* W[0..n] (n+1 doubles) after ccj_pf_fill. */
int ccj_pf_W(ccj_pf_ctx *ctx, double *W);

/* One 2-D matrix, canonical order i = 1..n, j = i..n (n(n+1)/2 doubles). */
int ccj_pf_get2(ccj_pf_ctx *ctx, int which, double *out);

/* One 4-D value with Matrix4DPF::get semantics (matrices.hh:258-263): 0 outside i <= j < k-1, k <= l. */
int ccj_pf_get4(ccj_pf_ctx *ctx, int which, int i, int j, int k, int l, int *out);

/* FNV-1a of every matrix in canonical order: h4[CCJ_PF_NMAT4] over the int32 values of the 4-D
 * matrices (i <= j < k-1, k <= l), h2[CCJ_PF_NMAT2] over the IEEE bits of the 2-D matrices. */
int ccj_pf_hashes(ccj_pf_ctx *ctx, uint64_t *h4, uint64_t *h2);

/* Hashes of the Boltzmann tables (names and order: ccj_pf_exp_names), for pinning against the
 * reference's scale_pf_parameters(). */
int ccj_pf_exp_hashes(ccj_pf_ctx *ctx, uint64_t *out, int cap);
const char *ccj_pf_exp_names(void); /* space-separated */
/* The same tables for a parameter blob without a context (no GPU needed). */
int ccj_pf_exp_hashes_params(const ccj_energy_params *params, const ccj_pf_raw *raw, const ccj_pk_penalties *pen,
                             uint64_t *out, int cap);

/* Stochastic traceback: nsamples times Sample_W(1, n) (stoch_backtrack.cc:36-85).  vrna_urn() of
 * the reference build is rand()/RAND_MAX (utils.c:262-271; its CMake defines no HAVE_ERAND48);
 * each context draws from its own glibc random_r state, which starts like a process that never
 * called srand() and is reseeded by ccj_pf_srand (= srand(seed)).  structures receives nsamples
 * NUL-terminated strings of n characters at stride n+1.  On a reference failure path (it prints
 * a line and calls exit(0)) that line is returned by ccj_pf_last_message() and the call returns
 * CCJ_E_PF_SAMPLE with *done = the samples completed before it. */
int ccj_pf_srand(ccj_pf_ctx *ctx, unsigned int seed);
int ccj_pf_sample(ccj_pf_ctx *ctx, int nsamples, char *structures, int *done);
const char *ccj_pf_last_message(ccj_pf_ctx *ctx);

/* Fill timing of the last ccj_pf_fill (ms, HIP events). */
int ccj_pf_timing(ccj_pf_ctx *ctx, float *fill_ms);
/* on != 0: the following fills record an event pair around every kernel launch (measurement only;
 * it adds the event cost to fill_ms).  ccj_pf_kernel_ms then gives the summed launch durations of
 * the last fill per family: [0] k_pf_iloop, [1] k_pf_level, [2] the P terms (k_pf_ppush; k_pf_pterm
 * with CCJ_PF_PULL=1), [3] k_pf_diag (0 when timing was off). */
int ccj_pf_set_timing(ccj_pf_ctx *ctx, int on);
int ccj_pf_kernel_ms(ccj_pf_ctx *ctx, double *ms4);
/* Algorithmic HBM bytes of one fill per kernel family (same order): the operands the
 * recurrences read and write, counted over this sequence's work items.  Host-side, no GPU work. */
int ccj_pf_work_model(ccj_pf_ctx *ctx, double *bytes4);

#ifdef __cplusplus
}
#endif

#endif /* CCJ_PF_H */
