// ccj_engine.h — internal data layout shared by the HIP kernels and the host engine.
//
// HBM layout:
//   * 4-D gap matrices: level-major.  A cell (i,j,k,l) has a = j-i, g = k-j (>= 2), b = l-k,
//     level t = a+b, h = g-2.  Level t holds (t+1) blocks (one per a) of M_t = m_t(m_t+1)/2 cells,
//     m_t = n-t-2, each block a triangle of rows h = 0..m_t-1 of length m_t-h, i fastest.
//     Within a level the 22 matrices are stored one after another (SoA), so one level is one
//     contiguous span:  elem(x,t,a,h,i) = LB_t + x*C_t + a*M_t + G_t(h) + (i-1),
//     G_t(h) = h*m_t - h(h-1)/2, C_t = (t+1)*M_t.
//     Every dependency of a level-t cell lies in levels < t, and lanes of one
//     wave (same t, a) read shifted neighbours whose offsets differ by a lane-uniform amount,
//     so reads and writes are coalesced along i.
//   * 2-D interval arrays: span-major [w][p] (w = j-i, p = i), row stride n+2, so a wave
//     reading (i, i+w) for consecutive i touches consecutive words.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "ccj_params.h"

namespace ccj {

constexpr int NMAT4 = 22;
enum Mat4 {
    PK = 0, PL, PR, PM, PO, PfromL, PfromR, PfromM, PfromMprime, PfromO,
    PLmloop00, PLmloop01, PLmloop10, PRmloop00, PRmloop01, PRmloop10,
    PMmloop00, PMmloop01, PMmloop10, POmloop00, POmloop01, POmloop10
};

// The matrices the loop records carry (below), which d4 does not store unless DevTables::mat5: the 5
// no fill kernel reads back as matrices and 6 more the level kernel's stack terms read from the
// records (rec_get); d4 stores the other 11.
constexpr unsigned REC_MASK = (1u << PfromL) | (1u << PfromR) | (1u << PfromMprime) | (1u << PfromO) | (1u << PLmloop00) |
                              (1u << PLmloop10) | (1u << PRmloop00) | (1u << PMmloop00) | (1u << PMmloop10) |
                              (1u << POmloop00) | (1u << POmloop10);
__host__ __device__ constexpr bool rec_only(int x) { return (REC_MASK >> x) & 1u; }
constexpr int NMAT_REC = __builtin_popcount(REC_MASK);
constexpr int NMAT_ST = NMAT4 - NMAT_REC;
// Storage slot of matrix x inside a level of d4 and of the host mirror: the 11 stored matrices in
// enum order, then the 11 record-carried ones.  d4 holds slots [0, 11) per level, or all 22 when
// DevTables::mat5 (band-sharded exchange, a host mirror streamed during the fill); the host mirror
// always holds 22.  Matrix-major "level element" indices of the exchange API (x*C + a*M + c) are by
// matrix, not by slot.
__host__ __device__ constexpr int rec_below(int x) { return __builtin_popcount(REC_MASK & ((1u << x) - 1u)); }
__host__ __device__ constexpr int mslot(int x) { return rec_only(x) ? NMAT_ST + rec_below(x) : x - rec_below(x); }
static_assert(NMAT_REC == 11 && mslot(PK) == 0 && mslot(PO) == 4 && mslot(PfromM) == 5 && mslot(POmloop01) == NMAT_ST - 1,
              "stored slots");
static_assert(mslot(PfromL) == NMAT_ST && mslot(POmloop10) == NMAT4 - 1, "record-carried slots");

constexpr int IE_U = 29;  // u1,u2 in [0,28] for pseudoknot interior loops (pseudo_loop.cc:694-806)
#ifndef CCJ_ILB
#define CCJ_ILB 8
#endif
constexpr int IL_B = CCJ_ILB;  // interior-loop candidates per load batch (k_iloop)
constexpr int IL_CAP = (IE_U * IE_U + IL_B + 7) / 8 * 8;  // candidate-list capacity per pair (+ IL_B null tail)
constexpr int IL_SEG = 64;   // per pair: seg[dt] = first list entry of source-level distance dt

// k_ppush: spans per wave, i.e. consecutive partner levels a wave reads through one buffer resource
constexpr int PPUSH_S = 8;

struct LevelDesc {
    int16_t *base;  // first element of level t (matrix 0)
    int C;          // cells per matrix in this level
    int M;          // cells per a-block
    int m;          // n - t - 2 (rows per a-block)
    int pad;
};

struct LvlDev {     // per-level descriptor read by the level kernel (one s_load_dwordx8)
    long long lb;  // element offset of level t in the 4-D storage
    long long lr;  // record offset of level t in the AoS loop records (3 record types x C)
    int C;         // cells per matrix in level t = (t+1)*M
    int M;         // cells per a-block = m(m+1)/2, m = n-t-2
    int pad[2];
};

// AoS loop records: the operands the fused split-point loops of k_level4d read at
// one neighbour cell, int16 fields packed in one record, so each neighbour costs one dwordx4 (dwordx3)
// load instead of 5-7 int16 loads.  Three record types per level, each indexed like a matrix
// (a*M + G(h) + i-1): RA and RL (16 bytes) in T.rec, level t at ld[t].lr (RA: C records, then RL),
// RK (12 bytes) in T.rk at ld[t].lr / 2:
//   RA (a-loop, both sides): PLmloop00 PMmloop00 | POmloop00 PfromL | PfromO PLmloop10 | PfromMprime PK
//   RK (b-loop, k side):     PRmloop00 PMmloop00 | PfromR min(PL,PR) | PK -
//   RL (b-loop, l side):     PRmloop00 PMmloop00 | POmloop00 PMmloop10 | POmloop10 PfromR | PfromO -
// Values are the stored (clamped) int16 matrix values; unused slots hold 32767.
enum RecType { RA = 0, RL = 1, NREC = 2 };  // 16-byte record types in T.rec (RK lives in T.rk)
static_assert(sizeof(uint3) == 12, "RK records are 12 bytes");

// Split-point sharing (k_level4d).  The cells of one gap column — same (j,k,l)
// for the i-side split, (i,k,l) j-side, (i,j,l) k-side, (i,j,k) l-side — sit on consecutive levels
// and read the same neighbours over the same split range, shifted by one split point per level.
// A leader cell (a % SHARE_R == 0 for the a-loop, b % SHARE_R == 0 for the b-loop) scans its whole
// range once and also reduces it for the next SHARE_R-1 cells of each of its columns; those
// followers scan only the split points the leader did not see and take the rest from a partial
// record.  Partial records live in a ring of SHARE_R level slots (the level t' cells' records are
// written at levels t'-SHARE_R+1 .. t'-1 and read at t'), SHARE_NACC 16-byte records per cell:
//   AI (i side): PLmloop00 PLmloop10 | PMmloop10 POmloop00 | POmloop10 PfromL | PfromO -
//   AJ (j side): PLmloop00 PLmloop01 | PMmloop00 PLmloop10 | PfromL PfromMprime | PK -
//   AK (k side): PRmloop00 PRmloop10 | PMmloop00 PfromR | PfromM'' PK | PfromO(l side) -
//   AL (l side): PRmloop00 PRmloop01 | PMmloop01 POmloop00 | POmloop01 PMmloop10 | POmloop10 PfromR
// (AK's 7th slot carries the l side's 9th field; it is written by the l-side leader, the first six
// by the k-side leader, so the two never write the same bytes.)  Values are min-clamped at 32767
// like a store (clamp commutes with min).  The leader's W(i-r, .) / W(., j+r) operands are read
// from the span-major WBW pairs (span s-1+r, coalesced along the lanes).
#ifndef CCJ_SHARE_R
#define CCJ_SHARE_R 4
#endif
constexpr int SHARE_R = CCJ_SHARE_R;
constexpr int SHARE_NACC = 4;
// ring slots (one per target level): the leader launch of level t reads slot t (its follower
// sides) and writes slots t+1 .. t+SHARE_R-1, after level t's plain launch on the same stream
constexpr int SHARE_SLOTS = SHARE_R;
enum AccRec { AI = 0, AJ = 1, AK = 2, AL = 3 };

// Band sharding: a-block a of every level belongs to rank (a / SHARD_GRP) % world,
// the same rank on every level, so a split-sharing leader (a % SHARE_R == 0) and its followers
// (a+1 .. a+SHARE_R-1, later levels) always live on one rank.  A rank's blocks are numbered by
// their "own index" o = 0, 1, ...: a = shard_a(o) ascending.  world = 1: a = o.
constexpr int SHARD_GRP = SHARE_R;
__host__ __device__ __forceinline__ int shard_owner(int a, int G) { return (a / SHARD_GRP) % G; }
__host__ __device__ __forceinline__ int shard_a(int o, int G, int r) {
    return ((o / SHARD_GRP) * G + r) * SHARD_GRP + o % SHARD_GRP;
}
// number of a in [0, x] owned by rank r (x >= -1)
__host__ __device__ __forceinline__ int shard_count(int x, int G, int r) {
    const int nb = x + 1, qf = nb / SHARD_GRP, rem = nb % SHARD_GRP;
    const int full = qf / G + (qf % G > r ? 1 : 0);
    return full * SHARD_GRP + (qf % G == r ? rem : 0);
}
// own index of the first a >= x owned by rank r
__host__ __device__ __forceinline__ int shard_ceil(int x, int G, int r) {
    if (x < 0) x = 0;
    int q = x / SHARD_GRP, off = x % SHARD_GRP;
    if (q % G != r) {
        q += ((r - q % G) + G) % G;
        off = 0;
    }
    return (q / G) * SHARD_GRP + off;
}

// The band-sharded exchange of level t has two parts, each ONE all-gather of equal
// slices:
//   part XCH_EDGE: the rank's blocks with a % SHARD_GRP == SHARD_GRP-1 (own index o % SHARD_GRP ==
//     SHARD_GRP-1): of level t, another rank's level t+1 reads only these (its group's first block a
//     reads block a-1 at split step 1, pseudo_loop.cc:357-362); then the tail: the P tail (XCH_PTAIL:
//     this rank's partials of P(t+1), pushed after level t-2) and the span tail (XCH_DTAIL: span t,
//     which level t+1 reads).  Gathered on the level stream: the critical path.
//   part XCH_BULK: the rank's other blocks (read from level t+2 on, and by k_iloop(t+3) / k_ppush(t)),
//     no tail.  Gathered on a side stream while level t+1 runs.
// The partials of P(n-1) (pushed after level n-4; no level n-2 carries them) travel alone after the
// last level, as a slice of one P tail.
// A part's slice: body [matrix x][part index k][cell c] of nmax blocks per matrix (nmax = the largest
// rank's block count of that part at t), padded to 8 bytes, then the part's tail.  k_pack / k_unpack /
// k_?tail_* and the host's buffer sizing use these; ccj_exchange_layout / ccj_exchange_index export
// them (tests).
constexpr int XCH_EDGE = 0, XCH_BULK = 1;
constexpr int XCH_DT_N = 10;  // span tail planes: V, Vt, P, WBP, WB, WPP, WP, WMv, WMp, WM
__host__ __device__ __forceinline__ long long xch_body(int nmax, int M) { return ((long long)22 * nmax * M + 3) & ~3LL; }
__host__ __device__ __forceinline__ long long xch_ptail(int n) { return 4LL * (n + 1); }
__host__ __device__ __forceinline__ long long xch_dtail(int n) { return 2LL * XCH_DT_N * (n + 1); }
__host__ __device__ __forceinline__ long long xch_tail(int n, int part) { return part == XCH_EDGE ? xch_ptail(n) + xch_dtail(n) : 0; }
__host__ __device__ __forceinline__ long long xch_slice(int n, int nmax, int M, int part) { return xch_body(nmax, M) + xch_tail(n, part); }
// part of own index o, its index inside the part, and back
__host__ __device__ __forceinline__ int xch_part(int o) { return o % SHARD_GRP == SHARD_GRP - 1 ? XCH_EDGE : XCH_BULK; }
__host__ __device__ __forceinline__ int xch_pidx(int o) {
    return xch_part(o) == XCH_EDGE ? o / SHARD_GRP : (o / SHARD_GRP) * (SHARD_GRP - 1) + o % SHARD_GRP;
}
__host__ __device__ __forceinline__ int xch_own(int k, int part) {
    return part == XCH_EDGE ? k * SHARD_GRP + SHARD_GRP - 1 : (k / (SHARD_GRP - 1)) * SHARD_GRP + k % (SHARD_GRP - 1);
}
// rank r's blocks of the part at level t (own indices 0 .. shard_count(t)-1)
__host__ __device__ __forceinline__ int xch_pcount(int t, int G, int r, int part) {
    const int own = shard_count(t, G, r);
    return part == XCH_EDGE ? own / SHARD_GRP : own - own / SHARD_GRP;
}
// body position of matrix x, part index k, cell c
__host__ __device__ __forceinline__ long long xch_pos(int x, int k, int c, int nmax, int M) {
    return ((long long)x * nmax + k) * M + c;
}
// where block a's cells arrive: its owner's slice of the block's part, at the block's part index
__host__ __device__ __forceinline__ void xch_src(int a, int G, int &owner, int &part, int &k) {
    owner = shard_owner(a, G);
    const int o = shard_count(a - 1, G, owner);
    part = xch_part(o);
    k = xch_pidx(o);
}
// the largest rank's block count of the part at level t
__host__ __device__ __forceinline__ int xch_nmax(int t, int G, int part) {
    int nm = 0;
    for (int r = 0; r < G; ++r) nm = xch_pcount(t, G, r, part) > nm ? xch_pcount(t, G, r, part) : nm;
    return nm;
}

struct LvlX {        // per-level bases of the interior-loop copies
    long long lbx;  // element offset of level t in d4x: PLx (C_t elements) then PRx (C_t)
    long long pmb;  // element offset of level t in pmx: m_t * n * (t+1) elements
};

struct Penalties {  // integer PK penalties, h_globals.hh:7-25
    int PS, PSM, PSP, PB, PUP, PPS, a, b, c, ap, bp, cp;
};

struct DevTables {
    int n;
    int nlev;                      // levels that hold cells (t <= n-3)
    int rs;                        // 2-D row stride (n+2)
    int dangles;
    Penalties pen;
    double e_stP, e_intP;
    const ccj_energy_params *prm;  // device copy of the blob
    const int *lx;                 // (int)(lxc*log(x/30.)), x in [0, 2n+64)
    const short *S, *S1;           // encoded sequence, n+2
    const int8_t *pt;              // [w][p] pair type pair[S[p]][S[p+w]]
    const int8_t *pair;            // 8x8 pair table (after noGU)
    const int8_t *rtype;           // 8
    const int *hp;                 // [w][p] HairpinE (s_energy_matrix.cc:275-282), INF if type 0
    const int16_t *est;            // [w][p] e_stP, saturated at 32767
    int16_t *ie;                   // [w][p] e_intP of the u1 = u2 = 0 interior loop (k_precompute_ie), 32767 where skipped
    int *V; int8_t *Vt; int *WM, *WMv, *WMp, *P, *WBP, *WPP, *WB, *WP;  // [w][p]
    int2 *WBW;                     // [w][p] (WBP, WP): the two 2-D operands of a k_level4d split step, one load
    unsigned long long *Pk;        // [w][p] (P + 2^31) << 32 | first (j,d,k) split of the minimum (k_pterm)
    const LevelDesc *lv;           // per level t
    int16_t *d4;                   // 4-D storage base
    const long long *lb;           // element offset of level t in d4
    const LvlDev *ld;             // per-level descriptors
    uint4 *rec;                    // AoS loop records RA, RL: level t at ld[t].lr
    long long nrec;                // records allocated (debug bounds checks)
    uint3 *rk;                     // RK records: level t at ld[t].lr / 2 (nrec / 2 of them)
    // interior-loop copies of PL / PR / PM, laid out so that the lanes of one k_iloop wave share
    // the loop's closing pair:
    //   PLx(t,a,h,i) = lbx + a*M + G(i-1) + h               (h fastest: fixed (i,j), lanes k)
    //   PRx(t,a,h,i) = lbx + C + a*M + q(q+1)/2 + i-1       (q = i+h-1: fixed (k,l), lanes i)
    //   PMx(t,a,h,i) = pmb + (h*n + j-1)*(t+1) + a          (j = i+a: fixed (j,k), lanes a)
    int16_t *d4x, *pmx;
    long long nx, npm;             // elements of d4x / pmx (debug bounds checks)
    const LvlX *ldx;
    // interior-loop candidate lists (k_build_il): per pair [w][p], the (u1,u2) whose inner pair can
    // pair, ordered by dt = 2+u1+u2 then u1; entry .x = dt << 21 | u1 << 16 | (uint16)energy,
    // .y = 2*u1*dt (the address cross term); IL_B null entries (dt 63) follow the last one
    uint2 *il, *ilm;               // il: pair (p,p+w) closes the loop (PL, PR); ilm: pair encloses (PM)
    int16_t *dummy;                // n+64 values 32767: target of the null entries
    const uint32_t *items;         // k_iloop work items (role << 30 | f1 << 20 | f2 << 10 | chunk)
    int mat5;                      // 1: the 5 record-only matrices are stored in d4 too (22 slots per level, mslot)
    uint32_t *ilseg, *ilmseg;      // [pair][IL_SEG]
    int *err;                      // device error word
    // split-point sharing (above): levels [g_lo, g_hi) share; partial-record ring of SHARE_R
    // slots x SHARE_NACC x accC
    int split_target;              // k_level4d: narrow levels split loops so ~this many waves run (0: never)
    long long xpad;                // 32767 sentinel elements in front of every level's PLx/PRx and PMx (k_iloop's null target)
    long long xspan;               // bytes k_iloop may address from a wave's buffer base (debug check)
    int g_lo, g_hi;
    // k_level4d_lead walks only the long-scan a-blocks of a sharing level, longest scan first:
    // rank r's list lord[lord_off[t*G+r] .. lord_off[t*G+r+1]) (device), lord_off_h = the same
    // offsets on the host
    const int16_t *lord;
    const int *lord_off;
    const int *lord_off_h;
    uint4 *acc;
    long long accC;
};

// The record-carried matrices (rec_only) live only in the loop records (RA / RK / RL), unless
// DevTables::mat5: the level kernel skips their d4 stores and d4 has no slots for them.
// rec_get reads one from the records of the cell at in-level offset cell (a*M + G(h) + i-1); k_mat5
// writes a level's eleven into a scratch buffer for the host mirror.
__device__ __forceinline__ int rlo16(unsigned w) { return (int)(int16_t)(w & 0xffffu); }
__device__ __forceinline__ int rhi16(unsigned w) { return (int)(int16_t)(w >> 16); }
__device__ __forceinline__ int rec_get(const DevTables &T, int x, const LvlDev &L, long long cell) {
    const uint4 *rp = T.rec + L.lr;
    if (x == PRmloop00 || x == PfromR) {  // RK: Rm00|Mm00, fR|PLR, K|-
        const uint3 r = T.rk[(L.lr >> 1) + cell];
        return x == PRmloop00 ? rlo16(r.x) : rlo16(r.y);
    }
    if (x == PMmloop10 || x == POmloop10) {  // RL: Rm00|Mm00, Om00|Mm10, Om10|fR, fO|-
        const uint4 r = rp[(long long)L.C + cell];
        return x == PMmloop10 ? rhi16(r.y) : rlo16(r.z);
    }
    const uint4 r = rp[cell];  // RA: Lm00|Mm00, Om00|fL, fO|Lm10, fMp|K
    switch (x) {
        case PLmloop00: return rlo16(r.x);
        case PMmloop00: return rhi16(r.x);
        case POmloop00: return rlo16(r.y);
        case PfromL: return rhi16(r.y);
        case PfromO: return rlo16(r.z);
        case PLmloop10: return rhi16(r.z);
        default: return rlo16(r.w);  // PfromMprime
    }
}

// element offset of cell (a,h,i) of matrix x inside level t of the host mirror (relative to lv_offh[t])
inline int64_t cell_offset_host(const LevelDesc &L, int x, int a, int h, int i) {
    return (int64_t)mslot(x) * L.C + (int64_t)a * L.M + (int64_t)h * L.m - (int64_t)h * (h - 1) / 2 + (i - 1);
}

}  // namespace ccj

// Kernel launchers (ccj_kernels.hip); all return a hipError_t as int.
extern "C" {
int ccjk_init2d(const ccj::DevTables *T, void *stream);
int ccjk_precompute_ie(const ccj::DevTables *T, void *stream);
int ccjk_build_il(const ccj::DevTables *T, void *stream);
int ccjk_iloop(const ccj::DevTables *T, int t, long long first_item, int nitems, int G, int rank, void *stream);
int ccjk_diag2d(const ccj::DevTables *T, int sigma, int G, int rank, void *stream);
int ccjk_dtail_pack(const ccj::DevTables *T, int sigma, int G, int rank, int16_t *tail, void *stream);
int ccjk_dtail_unpack(const ccj::DevTables *T, int sigma, const int16_t *recv, size_t slice, size_t off, int G, int rank,
                      void *stream);
int ccjk_level4d(const ccj::DevTables *T, int t, int G, int rank, int copies, void *stream);
int ccjk_level_split(int n, int t, int nblk, int split_target);
int ccjk_level4d_lead(const ccj::DevTables *T, int t, int G, int rank, void *stream);
int ccjk_pack(const ccj::DevTables *T, int t, int G, int r, int part, int nmax, int16_t *send, void *stream);
int ccjk_unpack(const ccj::DevTables *T, int t, int G, int r, int part, int nmax, const int16_t *recv, size_t rstride, void *stream);
int ccjk_pterm(const ccj::DevTables *T, int sigma, void *stream);
int ccjk_ppush(const ccj::DevTables *T, int lev, int G, int rank, void *stream);
int ccjk_ptail_pack(const ccj::DevTables *T, int sigma, int16_t *tail, void *stream);
int ccjk_ptail_unpack(const ccj::DevTables *T, int sigma, const int16_t *recv, size_t slice, size_t off, int G, void *stream);
int ccjk_items(const ccj::DevTables *T, int G, int rank, int simulate, long long *counts, const long long *offs,
               uint32_t *items, int pass, void *stream);
int ccjk_canon(const ccj::DevTables *T, int x, const long long *offij, int16_t *out, void *stream);
int ccjk_mat5(const ccj::DevTables *T, int t, int16_t *out, void *stream);
}
