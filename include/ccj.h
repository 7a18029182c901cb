/*
 * ccj.h — C ABI of libccj_hip.so, the MI355X-native CCJ pseudoknot MFE engine.
 *
 * Drop-in boundary.  The reference has no FFI; its seam is the fill loop of
 * W_final::ccj() (reference src/W_final.cc:60-67), which calls, per interval (i,l),
 *   s_energy_matrix::compute_energy / compute_WMv_WMp / compute_energy_WM  (s_energy_matrix.cc:206-358)
 *   pseudo_loop::compute_energies                                            (pseudo_loop.cc:69-132)
 * and afterwards W (W_final.cc:68-79), backtrack (W_final.cc:84-104, pseudo_loop.cc:861-2820)
 * and bracket emission (W_final.cc:764-819).  This ABI replaces that whole body: one
 * ccj_fill() runs every recurrence on the GPU; ccj_result() runs W + backtrack + emission on
 * the GPU by default (k_compute_W / k_backtrack over the device matrices), or, with
 * ccj_options.host_traceback = 1, on the host against a host mirror; the getters keep the
 * reference's semantics either way.
 *
 * Plain C types only (no torch / HIP types).  All positions are 1-based like the reference.
 * Not re-entrant per context; independent contexts may run on separate host threads.
 */
#ifndef CCJ_H
#define CCJ_H

#include <stdint.h>
#include "ccj_params.h"

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (SURVEY.md §8b "Errors") */
#define CCJ_OK           0
#define CCJ_E_ARG        1   /* bad argument (sequence, n, parameter blob) */
#define CCJ_E_OOM        2   /* host or device allocation failed */
#define CCJ_E_HIP        3   /* HIP runtime error */
#define CCJ_E_PARAMS     4   /* parameter set outside what the int16 tables can represent */
#define CCJ_E_BACKTRACK  5   /* reference backtrack would exit(EXIT_FAILURE); message in ccj_last_error() */
#define CCJ_E_STATE      6   /* call out of order (e.g. ccj_result before ccj_fill) */
#define CCJ_E_INTER_EXIT 7   /* reference "NOT GOOD RESTR INTER" path: it prints and exit(0) */
#define CCJ_E_COMM       9   /* band-sharded exchange failed: an RCCL error on the communicator, or no
                                progress within CCJ_COMM_TIMEOUT_S seconds (default 300; a peer rank
                                died or hung); the communicator is aborted and the context must be
                                destroyed */

/* 4-D gap matrices, reference pseudo_loop.hh:62-108 / allocation order pseudo_loop.cc:37-62 */
enum ccj_mat4 {
    CCJ_PK = 0, CCJ_PL, CCJ_PR, CCJ_PM, CCJ_PO,
    CCJ_PfromL, CCJ_PfromR, CCJ_PfromM, CCJ_PfromMprime, CCJ_PfromO,
    CCJ_PLmloop00, CCJ_PLmloop01, CCJ_PLmloop10,
    CCJ_PRmloop00, CCJ_PRmloop01, CCJ_PRmloop10,
    CCJ_PMmloop00, CCJ_PMmloop01, CCJ_PMmloop10,
    CCJ_POmloop00, CCJ_POmloop01, CCJ_POmloop10,
    CCJ_NMAT4
};

/* 2-D interval matrices (raw stored value for 1 <= i <= j <= n) */
enum ccj_mat2 {
    CCJ_M2_P = 0, CCJ_M2_WBP, CCJ_M2_WPP, CCJ_M2_V, CCJ_M2_VTYPE, CCJ_M2_WM, CCJ_M2_WMV, CCJ_M2_WMP,
    CCJ_NMAT2
};

typedef struct ccj_problem {
    const char *seq;                 /* upper-case A/C/G/U/T, length n (validated by caller like CCJ.cc:23-36) */
    int dangles;                     /* -d, reference W_final.cc:25 */
    int noGU;                        /* --noGU global, reference pair_mat.h:94-95 */
    const ccj_energy_params *params; /* scaled 37 C tables (include/ccj_params.h) */
    const ccj_pk_penalties *pen;     /* NULL -> reference h_globals.hh defaults */
} ccj_problem;

typedef struct ccj_ctx ccj_ctx;

/* Engine options for ccj_create.  device = HIP device ordinal. */
typedef struct ccj_options {
    int device;
    int overlap_d2h;     /* 1: stream finished levels to the host mirror while later levels compute */
    /* Band sharding of one sequence over shard_world processes (one per GPU):
     * this process computes the a-blocks ccj_shard_blocks() gives it and each level is all-gathered
     * over RCCL (ccj_comm_init, or ccj_comm_init_local, before the first fill).  0 or 1 = unsharded. */
    int shard_world;
    int shard_rank;
    int shard_simulate;  /* 1: run every shard's launches in this one context, no exchange (tests) */
    /* 0 (default): W and the traceback run on the GPU (no host copy of the 4-D matrices; getters
     * copy them on first use).  1: on the host over the mirror (the reference restatement). */
    int host_traceback;
    /* Level-kernel tuning (0 = default for both).
     * split_target: narrow late levels split each cell's split-point loops over up to 8 waves so
     *   about this many waves run at once (default 9216); < 0 never splits.
     * share_splits: split-point sharing between the cells of one gap column: a
     *   leader cell scans its whole split range once for itself and the next CCJ_SHARE_R-1 cells of
     *   its column; < 0 turns it off (every cell scans its own range). */
    int split_target;
    int share_splits;
} ccj_options;

/* Create a context for one sequence: copies the problem, allocates device + pinned host
 * storage (22 x C(n+1,4) int16 + 2-D tables).  Replaces W_final::W_final + space_allocation
 * (reference W_final.cc:20-56).  opts may be NULL. */
int  ccj_create(const ccj_problem *prob, const ccj_options *opts, ccj_ctx **out);

/* Rebind a context to another sequence of the same length n (same tables, dangles, noGU,
 * options): rebuilds only the sequence tables and the interior-loop work lists and reuses every
 * allocation, so a batch of equal-length sequences pays ccj_create's multi-GB allocation once.
 * The reference has no equivalent (each fold constructs a new W_final, W_final.cc:20-56).
 * Blocking: the interior-loop work-list count pass runs on the context's stream and the call
 * waits for it (the host sizes the fill's launches from the counts), so it returns only after
 * the work already queued on that stream; with CCJ_HOST_COUNT=1 the count runs on host threads.
 * CCJ_E_ARG if the length differs or the sequence has characters other than ACGUT; CCJ_E_STATE
 * while a fold is in flight. */
int  ccj_reset(ccj_ctx *ctx, const char *seq);

/* Run the whole DP fill on the GPU (replaces W_final.cc:60-67).  With host_traceback = 1 it
 * also makes the host mirror valid (ccj_sync_host is implied); by default the matrices stay on
 * the device and the getters copy them on first use. */
int  ccj_fill(ccj_ctx *ctx);

/* Device-only fill, no host mirror (for timing the kernels alone).  CCJ_E_STATE while a fold
 * is in flight (ccj_fill_async without ccj_wait). */
int  ccj_fill_device(ccj_ctx *ctx);
/* Copy the device matrices to the host mirror. */
int  ccj_sync_host(ccj_ctx *ctx);

/* W (W_final.cc:68-79), backtrack and bracket emission: on the GPU by default (k_compute_W,
 * k_backtrack; results copied back), on the host mirror with host_traceback = 1.  Both are
 * bit-identical to the reference.
 * structure: buffer of n+1 chars (NUL-terminated on return); *energy_kcal = W[n]/100.0;
 * stdout_msgs: optional buffer receiving the reference's stdout side messages
 * ("Should not be here!\n" lines, W_final.cc:715), NUL-terminated, may be NULL. */
int  ccj_result(ccj_ctx *ctx, char *structure, double *energy_kcal, char *stdout_msgs, int msgs_cap);

/* Asynchronous fold, for pipelining a batch over contexts: ccj_fill_async enqueues the fill and
 * (device traceback) W + traceback on the context's streams and returns at once; ccj_wait blocks
 * until they are done and returns exactly what ccj_fill + ccj_result would.  While one context's
 * traceback (one wave) runs, another context's fill can use the rest of the GPU.  One fold in
 * flight per context; ccj_reset / ccj_fill refuse with CCJ_E_STATE until ccj_wait. */
int  ccj_fill_async(ccj_ctx *ctx);
/* The same, but the fill starts only when `after`'s last enqueued fill has ended (not its W +
 * traceback): two contexts on one device then alternate fills back to back while each fold's
 * traceback runs beside the next fill.  after == NULL: ccj_fill_async. */
int  ccj_fill_async_after(ccj_ctx *ctx, const ccj_ctx *after);
int  ccj_wait(ccj_ctx *ctx, char *structure, double *energy_kcal, char *stdout_msgs, int msgs_cap);

/* Reference getter semantics (matrices.hh:177-182: INF outside i<=j<k-1<=l-1). */
int  ccj_get4(const ccj_ctx *ctx, int mat, int i, int j, int k, int l);
/* Raw 2-D value for 1 <= i <= j <= n (ccj_mat2). */
int  ccj_get2(const ccj_ctx *ctx, int mat, int i, int j);
/* W[j], 0 <= j <= n (valid after ccj_result). */
int  ccj_getW(const ccj_ctx *ctx, int j);
/* FNV-1a 64 hashes in canonical order: 22 4-D matrices, 8 2-D (ccj_mat2), W. out[31]. */
int  ccj_hashes(const ccj_ctx *ctx, uint64_t *out);

/* Timing of the last ccj_fill_device (ms, HIP events on the streams the kernels run on) and of
 * its kernel families: kernel_ms[0] = k_level4d, [1] = k_diag2d, [2] = precompute. */
int  ccj_last_timing(const ccj_ctx *ctx, double *fill_ms, double *kernel_ms3);
/* Sum of the k_iloop (interior-loop pass) times of the last fill (ms). */
double ccj_iloop_ms(const ccj_ctx *ctx);
/* summed k_ppush (P terms) launch times of the last fill in timing mode 2 (ms) */
double ccj_ppush_ms(const ccj_ctx *ctx);
/* Host side of the last fold (ms): out3[0] = wait for the host mirror (D2H tail), [1] = W, [2] = backtrack. */
int  ccj_host_timing(const ccj_ctx *ctx, double *out3);
/* Per-level kernel times of the last fill (ms): level_ms[t] (k_level4d, level t), diag_ms[s]
 * (k_diag2d, span s); ccj_iloop_times: iloop_ms[t] (k_iloop, level t). */
int  ccj_level_times(const ccj_ctx *ctx, double *level_ms, double *diag_ms, int cap);
/* Band-sharded contexts in timing mode 2, per level (0 elsewhere; either pointer may be NULL):
 * edge_ms[t] = the edge part's share of the level span on the level stream (from the end of the
 * level's launches to the end of its unpack: the waits for the P and span tails, pack, all-gather,
 * unpack); bulk_ms[t] = the bulk part on its side stream (from the level's end: pack, all-gather,
 * unpack), which overlaps the next level. */
int  ccj_exchange_times(const ccj_ctx *ctx, double *edge_ms, double *bulk_ms, int cap);
int  ccj_iloop_times(const ccj_ctx *ctx, double *iloop_ms, int cap);
/* ccj_ppush_times: ppush_ms[t] (k_ppush after level t), timing mode 2 */
int  ccj_ppush_times(const ccj_ctx *ctx, double *ppush_ms, int cap);
/* What the next fills time (HIP events): 0 = the fill only; 1 (default) = + per-level durations
 * (level_ms, from events the fill records anyway); 2 = + k_diag2d / k_iloop times and level spans
 * from extra marker events around every launch (they slow the fill down by a few percent). */
int  ccj_set_timing(ccj_ctx *ctx, int mode);

/* ---- band sharding (one sequence over several GPUs) ---- */
#define CCJ_COMM_ID_BYTES 128
/* A fresh RCCL unique id (call on one rank, broadcast the bytes to the others). */
int  ccj_comm_unique_id(char *id_out);
/* Join the sharded context to the RCCL communicator of shard_world ranks. */
int  ccj_comm_init(ccj_ctx *ctx, const char *id);
/* The a-blocks of level t that rank computes (host helper, no GPU): writes up to cap of them to
 * a_out, ascending, and returns how many there are (< 0: bad arguments).  Block a belongs to rank
 * (a / 4) % world on every level. */
int  ccj_shard_blocks(int n, int t, int world, int rank, int *a_out, int cap);
/* Per-matrix element count C_t of level t and the a-block size M_t (the same for every world). */
int  ccj_level_layout(int n, int t, int world, long long *C, int *M);
/* The level-t exchange is two all-gathers: part 0 ("edge") = each rank's blocks
 * a % 4 == 3, the only cells of level t another rank's level t+1 reads, then its P(t+1) partials
 * (4(n+1) elements) and span t (20(n+1) elements), on the level stream; part 1 ("bulk") = the other
 * blocks, no tail, on a side stream that overlaps level t+1.  (P(n-1)'s partials travel alone after
 * the last level.)  ccj_exchange_layout (host helper, no GPU; the geometry k_pack / k_unpack use), in
 * int16 elements: out3 = {nmax (the largest rank's block count of the part), tail offset, slice size}.
 * The body is [matrix][part index][cell] of nmax blocks per matrix. */
int  ccj_exchange_layout(int n, int t, int world, int part, long long *out3);
/* which = 0: for each body element of rank's slice of the part, the level element (x*C + a*M + c:
 * matrix-major by matrix index x of ccj_mat4; d4 keeps matrix x at its storage slot) packed there
 * (-1: padding); which = 1: for each level element, its position in the part's
 * gathered buffer (owner * slice + body position) as rank unpacks it (-1: rank's own cell or the other
 * part's).  Returns the entry count; fills out only when cap >= that count.  < 0: bad arguments. */
long long ccj_exchange_index(int n, int t, int world, int rank, int part, int which, long long *out, long long cap);
/* In-process exchange group (tests, and several ranks sharing one device): shard_world contexts,
 * each driven by its own host thread, join one group instead of an RCCL communicator. */
typedef struct ccj_group ccj_group;
int  ccj_group_create(int world, ccj_group **out);
void ccj_group_destroy(ccj_group *g);
int  ccj_comm_init_local(ccj_ctx *ctx, ccj_group *g);

/* Algorithmic work model of this sequence:
 * out[0] = bytes moved by the 4-D level kernels (2 B per int16 operand read + 44 B of writes per cell),
 * out[1] = bytes of the P terms in the 2-D kernels, out[2] = R4 (4-D operand reads), out[3] = cells. */
int  ccj_work_model(const ccj_ctx *ctx, double *out4);
/* Split of out[0] by kernel: out2[0] = bytes of k_iloop (interior-loop candidate reads),
 * out2[1] = bytes of k_level4d (split-point, stack and t-2 reads + 44 B of stores per cell). */
int  ccj_work_split(const ccj_ctx *ctx, double *out2);
/* Same model for a bare sequence (no GPU, no context). */
int  ccj_work_model_seq(const char *seq, int noGU, double *out4);

int  ccj_n(const ccj_ctx *ctx);
const char *ccj_last_error(const ccj_ctx *ctx);
void ccj_destroy(ccj_ctx *ctx);

/* Number of 4-D DP cells (unit of work): C(n+1,4). */
uint64_t ccj_num_cells(int n);

#ifdef __cplusplus
}
#endif

#endif /* CCJ_H */
