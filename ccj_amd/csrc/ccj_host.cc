// ccj_host.cc — host side of libccj_hip.so: context + HBM allocation, sequence tables,
// level-by-level kernel schedule on a HIP stream, overlapped D2H of finished levels into a
// pinned host mirror, the exterior W array, and the host backtrack / bracket emission.
//
// The backtrack and emission are restated from the reference so the output is bit-identical,
// including its quirks:
//   W_final::ccj (exterior W + driver)   reference src/W_final.cc:58-105
//   W_final::E_ext_Stem                   reference src/W_final.cc:118-173
//   W_final::backtrack                    reference src/W_final.cc:175-719
//   pseudo_loop::backtrack                reference src/pseudo_loop.cc:861-2820
//   W_final::fill_structure               reference src/W_final.cc:764-819
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <stack>
#include <string>
#include <thread>
#include <vector>

#include "ccj.h"
#include "ccj_energy.h"
#include "ccj_engine.h"
#include "ccj_backtrack.h"
#include "ccj_items.h"

using namespace ccj;

namespace {

const int BP_PAIR[8][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 5, 0, 0, 5}, {0, 0, 0, 1, 0, 0, 0, 0},
                           {0, 0, 2, 0, 3, 0, 0, 0}, {0, 6, 0, 4, 0, 0, 0, 6}, {0, 0, 0, 0, 0, 0, 2, 0},
                           {0, 0, 0, 0, 0, 1, 0, 0}, {0, 6, 0, 0, 5, 0, 0, 0}};

struct BacktrackExit {  // reference exit(...) inside the backtrack
    int code;
    std::string stderr_msg;
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t count = 0;
};

}  // namespace

// In-process stand-in for the RCCL communicator (tests): world contexts, one host
// thread each, exchange through device-to-device copies with a host barrier around every level.
struct ccj_group {
    int world = 1;
    std::vector<ccj_ctx *> members;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    bool broken = false;
    int busy = 0;  // members between taking the peers' send pointers and finishing their copies
    // false when a member gave up (error or 120 s without the others)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const long g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

// timing events per level (timing mode 2): [0,1] k_diag2d, [2,3] k_iloop, [4,5] the level, [6] the
// edge exchange's start (band-sharded), [7,8] k_ppush, [9,10] the bulk exchange (band-sharded, st_x)
constexpr int TEV_PER = 11;

struct ccj_ctx {
    // problem
    int n = 0;
    std::string seq;
    int dangles = 2;
    int noGU = 0;
    ccj_energy_params prm{};
    Penalties pen{};
    double e_stP = 0.89, e_intP = 0.74;
    int pair[8][8]{};
    int rtype[8]{};
    std::vector<short> S, S1;
    std::vector<int> lx;
    int rs = 0;
    int device = 0;
    bool overlap = true;
    int world = 1, rank = 0, simulate = 0;  // band sharding
    bool host_tb = false;                   // W + traceback on the host over the mirror (else on the GPU)
    int split_target = 9216;                // k_level4d split heuristic (0: never split)
    bool share = true;                      // split-point sharing
    // fill timing (ccj_set_timing, CCJ_LEVEL_TIMING): 0 = fill only; 1 = + level durations from the
    // lev_done events the fill records anyway (no extra packets); 2 = + a marker pair around every
    // kernel family launch (k_diag2d, k_iloop, the level span).  The markers of mode 2 are barrier
    // packets on the streams and cost ~3 ms per n=200 fill, so the default is 1.
    int level_timing = 1;
    ncclComm_t comm = nullptr;    // the edge all-gathers (level stream)
    ncclComm_t comm_b = nullptr;  // the bulk all-gathers (st_x), split from comm: one communicator per stream

    // layout
    std::vector<LevelDesc> lv_host;     // device pointers
    std::vector<int64_t> lv_off;        // element offset of each level in d4 (nm4 slots per level)
    std::vector<int64_t> lv_offh;       // element offset of each level in the host mirror (NMAT4 slots)
    int64_t ncell = 0;                  // cells of the 4-D state per matrix, C(n+1, 4)
    int64_t total4 = 0;                 // elements of d4: nm4 * ncell
    int nm4 = NMAT_ST;                  // matrix slots per level in d4 (NMAT4 when T.mat5; ccj_engine.h mslot)
    bool mat5 = false;                  // the record-carried matrices stored in d4 too (DevTables::mat5)
    int nlev = 0;                       // levels with cells (0..n-3)

    // device
    int16_t *d4 = nullptr;
    int16_t *d_ie = nullptr, *d_est = nullptr;
    int *d_hp = nullptr, *d_lx = nullptr, *d_err = nullptr;
    int8_t *d_pt = nullptr, *d_pair = nullptr, *d_rtype = nullptr;
    short *d_S = nullptr, *d_S1 = nullptr;
    ccj_energy_params *d_prm = nullptr;
    LevelDesc *d_lv = nullptr;
    long long *d_lb = nullptr;
    LvlDev *d_ld = nullptr;
    int16_t *d4x = nullptr, *pmx = nullptr;  // interior-loop copies of PL/PR and PM (IT_PAD into the allocations)
    int16_t *d4x_alloc = nullptr, *pmx_alloc = nullptr;
    uint4 *d_rec = nullptr;                  // AoS loop records RA, RL (16 bytes)
    uint3 *d_rk = nullptr;                   // AoS loop records RK (12 bytes)
    uint4 *d_acc = nullptr;                  // partial-record ring (split-point sharing)
    int16_t *d_lord = nullptr;               // long-scan a-blocks per sharing level, longest first
    int *d_lord_off = nullptr;
    std::vector<int> lord_off;
    int2 *d_wbw = nullptr;                   // (WBP, WP) pairs [w][p]
    long long nrec = 0;
    long long nx = 0, npm = 0, xpad = 0, xspan = 0;
    LvlX *d_ldx = nullptr;
    uint2 *d_il = nullptr, *d_ilm = nullptr;
    int16_t *d_dummy = nullptr;
    uint32_t *d_items = nullptr;          // k_iloop work items, all levels back to back
    size_t items_cap = 0;
    // band-sharded exchange, per part (XCH_EDGE, XCH_BULK): own slice, world slices
    int16_t *d_send[2] = {nullptr, nullptr}, *d_recv[2] = {nullptr, nullptr};
    std::vector<int> xnmax[2];            // per level: the largest rank's block count of the part (slice = 22 x nmax x M + tail)
    ccj_group *lgroup = nullptr;          // in-process exchange between contexts (tests), else RCCL
    long long *d_icount = nullptr, *d_ioff = nullptr;  // k_items: items per (t, r), first item
    long long *h_ioff = nullptr;          // pinned staging of it_off
    long long *h_icount = nullptr;        // pinned landing of the k_items counts (so the copy is asynchronous)
    void *h_stage = nullptr;              // pinned staging of the sequence tables
    hipEvent_t ev_stage = nullptr;        // the uploads from the staging (and h_ioff) are done
    std::vector<long long> it_off;        // first item of (level t, shard r) at t*world + r
    uint32_t *d_ilseg = nullptr, *d_ilmseg = nullptr;
    int *d2i = nullptr;       // 9 int 2-D arrays back to back: V WM WMv WMp P WBP WPP WB WP
    unsigned long long *d_pk = nullptr;  // P with its first split (k_pterm), [w][p]
    int *d_W = nullptr, *d_fpair = nullptr;  // device traceback outputs
    int *d_wterm = nullptr;                  // W's (k, j) terms [j][k] (ccjk_compute_W scratch)
    int8_t *d_ftype = nullptr;
    BtOut *d_btout = nullptr;
    std::vector<unsigned long long> h_pk;
    int8_t *d_vt = nullptr;
    hipStream_t st = nullptr, st_copy = nullptr, st_p = nullptr, st_il = nullptr, st_d = nullptr;
    hipStream_t st_x = nullptr;          // band-sharded: the bulk part of each level's exchange
    std::vector<hipEvent_t> bulk_done;   // band-sharded: level t complete on this rank (bulk part unpacked)
    // in-process group: this rank's bulk slice packed / the peers' bulk slices copied (reused every level;
    // the group's barriers order each record before the peers' waits on it)
    hipEvent_t ev_bpacked = nullptr, ev_bcopied = nullptr;
    bool join_diag = true;               // k_diag2d(t-1) after k_iloop(t) on st_il (one cross-stream wait per level)
    std::vector<hipEvent_t> p_done;  // P(sigma) reduced
    std::vector<hipEvent_t> pp_done; // band-sharded: this rank's P-term push of span sigma done (before the exchange)
    std::vector<double> lev_ms_v, diag_ms_v, il_ms_v, xch_ms_v, xbulk_ms_v, pp_ms_v;
    std::vector<hipEvent_t> il_done, dg_done;  // k_iloop(t) / k_diag2d(sigma) finished
    std::vector<hipEvent_t> lev_done;
    std::vector<hipEvent_t> tev;  // timing events (TEV_PER per level): 2 per k_level4d, k_iloop, k_diag2d and k_ppush launch
    hipEvent_t ev_start = nullptr, ev_end = nullptr, ev_pre = nullptr;
    DevTables T{};

    // host mirror
    int16_t *h4 = nullptr;
    std::vector<int> h2i;     // same 9 arrays
    std::vector<int8_t> hvt;
    std::vector<int> hpt_h;   // pair type table [w][p] host copy (int)
    bool filled = false, mirrored = false, mirrored2d = false;
    bool pending = false;                 // a fill is enqueued and not yet finished (fill_finish)
    bool res_pending = false;             // W + traceback enqueued (result_enqueue), not yet read
    hipEvent_t ev_res = nullptr;          // device traceback results copied to the pinned buffers
    int *hr_W = nullptr, *hr_fp = nullptr;  // pinned: W, f[].pair, f[].type, the exit record
    int8_t *hr_ft = nullptr;
    BtOut *hr_bo = nullptr;
    std::vector<int> W;

    double fill_ms = 0, level_ms = 0, diag_ms = 0, pre_ms = 0, il_ms = 0, pp_ms = 0;
    double sync_ms = 0, w_ms = 0, bt_ms = 0;  // host side of the last fold
    int bt_steps = 0;
    std::string err;

    // ---- host accessors (reference getter semantics) ----
    size_t a2(int i, int j) const { return (size_t)(j - i) * rs + i; }
    int hV(int i, int j) const { return h2i[0 * plane() + a2(i, j)]; }
    int plane() const { return (n + 1) * rs; }
    int raw2(int which, int i, int j) const { return h2i[(size_t)which * plane() + a2(i, j)]; }
};

namespace {

int set_err(ccj_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
    return code;
}

#define HIPCHK(ctx, x)                                                                                   \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) return set_err((ctx), CCJ_E_HIP, "%s: %s", #x, hipGetErrorString(e_));     \
    } while (0)

enum { A2_V = 0, A2_WM, A2_WMV, A2_WMP, A2_P, A2_WBP, A2_WPP, A2_WB, A2_WP, A2_N };

// --------------------------------------------------------------------------------------------
// host energy helpers
// --------------------------------------------------------------------------------------------
int E_Hairpin_host(const ccj_energy_params *P, const int *lx, int size, int type, int si1, int sj1,
                   const char *string) {
    // reference ViennaRNA/loops/hairpin.h:148-200
    int energy;
    if (size <= 30) energy = P->hairpin[size];
    else energy = P->hairpin[30] + lx[size];
    if (size < 3) return energy;
    if (string && P->special_hp) {
        if (size == 4) {
            char tl[7] = {0};
            memcpy(tl, string, 6);
            if (const char *ts = strstr(P->Tetraloops, tl)) return P->Tetraloop_E[(ts - P->Tetraloops) / 7];
        } else if (size == 6) {
            char tl[9] = {0};
            memcpy(tl, string, 8);
            if (const char *ts = strstr(P->Hexaloops, tl)) return P->Hexaloop_E[(ts - P->Hexaloops) / 9];
        } else if (size == 3) {
            char tl[6] = {0};
            memcpy(tl, string, 5);
            if (const char *ts = strstr(P->Triloops, tl)) return P->Triloop_E[(ts - P->Triloops) / 6];
            return energy + (type > 2 ? P->TerminalAU : 0);
        }
    }
    energy += P->mismatchH[type][si1][sj1];
    return energy;
}

// --------------------------------------------------------------------------------------------
// The host-side view used by W + backtrack: reference getters over the mirror.
// --------------------------------------------------------------------------------------------
struct HostView {
    ccj_ctx *c;
    int n;
    const short *S, *S1;
    const ccj_energy_params *P;
    const int *lx;

    explicit HostView(ccj_ctx *cc) : c(cc), n(cc->n), S(cc->S.data()), S1(cc->S1.data()), P(&cc->prm), lx(cc->lx.data()) {}

    int pr(int i, int j) const { return c->pair[S[i]][S[j]]; }
    // s_energy_matrix.hh:37-43
    int V(int i, int j) const { return i >= j ? INF : c->raw2(A2_V, i, j); }
    char Vtype(int i, int j) const { return (char)c->hvt[c->a2(i, j)]; }
    int WM(int i, int j) const { return i >= j ? INF : c->raw2(A2_WM, i, j); }
    int WMv(int i, int j) const { return i >= j ? INF : c->raw2(A2_WMV, i, j); }
    int WMp(int i, int j) const { return i >= j ? INF : c->raw2(A2_WMP, i, j); }
    // TriangleMatrix::get (matrices.hh:38-41)
    int Pg(int i, int j) const { return i > j ? INF : c->raw2(A2_P, i, j); }
    int WBPg(int i, int j) const { return i > j ? INF : c->raw2(A2_WBP, i, j); }
    int WPPg(int i, int j) const { return i > j ? INF : c->raw2(A2_WPP, i, j); }
    // pseudo_loop.cc:647-661
    int WB(int i, int j) const {
        if (i <= 0 || j <= 0 || i > n || j > n) return INF;
        if (i > j) return 0;
        return std::min(c->pen.cp * (j - i + 1), WBPg(i, j));
    }
    int WP(int i, int j) const {
        if (i <= 0 || j <= 0 || i > n || j > n) return INF;
        if (i > j) return 0;
        return std::min(c->pen.PUP * (j - i + 1), WPPg(i, j));
    }
    // Matrix4D::get (matrices.hh:177-182); get_uc's assert (matrices.hh:167) is live in the
    // reference build, so an in-order but out-of-range cell aborts there.
    int g4(int x, int i, int j, int k, int l) const {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (i <= 0 || l > n) throw BacktrackExit{134, "CCJ: matrices.hh:167: Assertion `!(i<=0 || l> n_)' failed.\n"};
        const int t = (j - i) + (l - k);
        const LevelDesc &L = c->lv_host[t];
        const int64_t off = c->lv_offh[t] + cell_offset_host(L, x, j - i, k - j - 2, i);
        return (int)c->h4[off];
    }
    bool can_pair(int i, int j) const {  // pseudo_loop.hh:131-135 (assert(i<=j) live in reference)
        if (j - i <= TURN) return false;
        return pr(i, j) > 0;
    }
    // pseudo_loop.cc:822-840
    int compute_int(int i, int j, int k, int l) const {
        return E_IntLoop(P, lx, k - i - 1, j - l - 1, pr(i, j), c->rtype[pr(k, l)], S1[i + 1], S1[j - 1], S1[k - 1],
                         S1[l + 1]);
    }
    int e_stP(int i, int j) const {
        if (i + 1 == j - 1) return INF;
        return (int)lrint(c->e_stP * compute_int(i, j, i + 1, j - 1));
    }
    int e_intP(int i, int ip, int jp, int j) const { return (int)lrint(c->e_intP * compute_int(i, j, ip, jp)); }
    int PfromMdoubleprime(int i, int j, int k, int l) const {  // pseudo_loop.cc:663-679
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (i == j && k == l) return pr(i, l) == 0 ? INF : 0;
        return std::min(g4(PL, i, j, k, l) + c->pen.PB, g4(PR, i, j, k, l) + c->pen.PB);
    }
};

// --------------------------------------------------------------------------------------------
// W (W_final.cc:68-79) and E_ext_Stem (W_final.cc:118-173)
// --------------------------------------------------------------------------------------------
int E_ext_Stem(const HostView &H, int dangles, int vij, int vi1j, int vij1, int vi1j1, int i, int j) {
    const short *S = H.S;
    const int n = H.n;
    int e = INF, en;
    int tt = H.pr(i, j);
    en = vij;
    if (en != INF) {
        if (dangles == 2) en += E_ExtLoop(H.P, tt, i > 1 ? S[i - 1] : -1, j < n ? S[j + 1] : -1);
        else en += E_ExtLoop(H.P, tt, -1, -1);
        e = std::min(e, en);
    }
    if (dangles == 1) {
        tt = H.pr(i + 1, j);
        en = (j - i - 1 > TURN) ? vi1j : INF;
        if (en != INF) en += E_ExtLoop(H.P, tt, S[i], -1);
        e = std::min(e, en);
        tt = H.pr(i, j - 1);
        en = (j - 1 - i > TURN) ? vij1 : INF;
        if (en != INF) en += E_ExtLoop(H.P, tt, -1, S[j]);
        e = std::min(e, en);
        tt = H.pr(i + 1, j - 1);
        en = (j - 1 - i - 1 > TURN) ? vi1j1 : INF;
        if (en != INF) en += E_ExtLoop(H.P, tt, S[i], S[j]);
        e = std::min(e, en);
    }
    return e;
}

void compute_W(ccj_ctx *c) {
    HostView H(c);
    const int n = c->n;
    c->W.assign(n + 1, 0);
    std::vector<int> &W = c->W;
    for (int j = TURN + 1; j <= n; j++) {
        int m1 = W[j - 1], m2 = INF, m3 = INF;
        for (int k = 1; k <= j - TURN - 1; ++k) {
            const int acc = (k > 1) ? W[k - 1] : 0;
            m2 = std::min(m2, acc + E_ext_Stem(H, c->dangles, H.V(k, j), H.V(k + 1, j), H.V(k, j - 1), H.V(k + 1, j - 1), k, j));
            m3 = std::min(m3, acc + std::min({H.Pg(k, j), H.Pg(k + 1, j), H.Pg(k, j - 1), H.Pg(k + 1, j - 1)}) + c->pen.PS);
        }
        W[j] = std::min({m1, m2, m3});
    }
}

// --------------------------------------------------------------------------------------------
// Backtrack
// --------------------------------------------------------------------------------------------
struct Minfold {  // h_struct.hh:9-19
    int pair = -1;
    char type = T_NONE;
};

struct Backtracker {
    const HostView &H;
    ccj_ctx *c;
    int n;
    std::vector<Interval> stk;  // LIFO; back() is the top (reference insert_node pushes on the head)
    std::vector<Minfold> f;
    std::string structure;
    std::string out;  // reference stdout side channel
    const Penalties &pe;

    Backtracker(const HostView &h, ccj_ctx *cc)
        : H(h), c(cc), n(cc->n), f(cc->n + 1), structure(cc->n + 1, '.'), pe(cc->pen) {}

    void push2(int i, int j, char type) { stk.push_back(Interval{i, j, 0, 0, type}); }
    // pseudo_loop::insert_node(i, j, k, l, type): fields i, j(=l of the region), k(=j), l(=k)
    void push4(int i, int j, int k, int l, char type) { stk.push_back(Interval{i, j, k, l, type}); }
    [[noreturn]] void die(const char *msg) { throw BacktrackExit{1, std::string(msg) + "\n"}; }

    void run() {
        // W_final.cc:84-99
        push2(1, n, FREE);
        while (!stk.empty()) {
            Interval cur = stk.back();
            stk.pop_back();
            wf_backtrack(cur);
        }
    }

    // W_final::backtrack, W_final.cc:175-719
    void wf_backtrack(const Interval &cur) {
        switch (cur.type) {
            case LOOP: bt_loop(cur); break;
            case FREE: bt_free(cur); break;
            case M_WM: bt_wm(cur); break;
            case M_WMv: bt_wmv(cur); break;
            case M_WMp: bt_wmp(cur); break;
            case P_PK: case P_PL: case P_PR: case P_PM: case P_PO: case P_PfromL: case P_PfromR: case P_PfromM:
            case P_PfromO: case P_PLiloop: case P_PLiloop5: case P_PLmloop: case P_PLmloop00: case P_PLmloop01:
            case P_PLmloop10: case P_PRiloop: case P_PRiloop5: case P_PRmloop: case P_PRmloop00: case P_PRmloop01:
            case P_PRmloop10: case P_PMiloop: case P_PMiloop5: case P_PMmloop: case P_PMmloop00: case P_PMmloop01:
            case P_PMmloop10: case P_POiloop: case P_POiloop5: case P_POmloop: case P_POmloop00: case P_POmloop01:
            case P_POmloop10: case P_WB: case P_WBP: case P_WP: case P_WPP: case P_P:
                pl_backtrack(cur);
                break;
            default:
                out += "Should not be here!\n";  // A-B1: P_PfromMprime / P_PfromMdoubleprime land here
        }
    }

    void bt_loop(const Interval &cur) {
        const int i = cur.i, j = cur.j;
        if (i >= j) return;
        f[i].pair = j;
        f[j].pair = i;
        structure[i] = '(';
        structure[j] = ')';
        const char type = H.Vtype(i, j);
        switch (type) {
            case T_HAIRP:
                f[i].type = T_HAIRP;
                f[j].type = T_HAIRP;
                break;
            case T_INTER: {
                f[i].type = T_INTER;
                f[j].type = T_INTER;
                int best_ip = j, best_jp = i;
                int mn = INF;
                const int max_ip = std::min(j - TURN - 2, i + MAXLOOP + 1);
                for (int k = i + 1; k <= max_ip; ++k) {
                    const int min_l = std::max(k + TURN + 1 + MAXLOOP + 2, k + j - i) - MAXLOOP - 2;
                    for (int l = j - 1; l >= min_l; --l) {
                        // s_energy_matrix::compute_int (:309-313): E_IntLoop + V(k,l)
                        const int tmp = E_IntLoop(H.P, H.lx, k - i - 1, j - l - 1, H.pr(i, j), c->rtype[H.pr(k, l)],
                                                  H.S1[i + 1], H.S1[j - 1], H.S1[k - 1], H.S1[l + 1]) + H.V(k, l);
                        if (tmp < mn) { mn = tmp; best_ip = k; best_jp = l; }
                    }
                }
                if (best_ip < best_jp) push2(best_ip, best_jp, LOOP);
                else {
                    char buf[160];
                    snprintf(buf, sizeof buf, "NOT GOOD RESTR INTER, i=%d, j=%d, best_ip=%d, best_jp=%d\n", i, j, best_ip, best_jp);
                    throw BacktrackExit{0, buf};
                }
            } break;
            case T_MULTI: {
                f[i].type = T_MULTI;
                f[j].type = T_MULTI;
                const short *S = H.S;
                const ccj_energy_params *P = H.P;
                const int tt = H.pr(j, i);
                int best_k = -1, best_row = -1, tmp = INF, mn = INF;
                for (int k = i + 1; k <= j - 1; k++) {
                    tmp = H.WM(i + 1, k - 1) + std::min(H.WMv(k, j - 1), H.WMp(k, j - 1)) + E_MLstem(P, tt, -1, -1) + P->MLclosing;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 1; }
                    tmp = H.WM(i + 2, k - 1) + std::min(H.WMv(k, j - 1), H.WMp(k, j - 1)) + E_MLstem(P, tt, -1, S[i + 1]) + P->MLclosing + P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 2; }
                    tmp = H.WM(i + 1, k - 1) + std::min(H.WMv(k, j - 2), H.WMp(k, j - 2)) + E_MLstem(P, tt, S[j - 1], -1) + P->MLclosing + P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 3; }
                    tmp = H.WM(i + 2, k - 1) + std::min(H.WMv(k, j - 2), H.WMp(k, j - 2)) + E_MLstem(P, tt, S[j - 1], S[i + 1]) + P->MLclosing + 2 * P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 4; }
                    tmp = (k - i - 1) * P->MLbase + H.WMp(k, j - 1) + E_MLstem(P, tt, -1, -1) + P->MLclosing;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 5; }
                    if ((k - (i + 1) - 1) >= 0) tmp = (k - (i + 1) - 1) * P->MLbase + H.WMp(k, j - 1) + E_MLstem(P, tt, -1, S[i + 1]) + P->MLclosing + P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 6; }
                    tmp = (k - i - 1) * P->MLbase + H.WMp(k, j - 2) + E_MLstem(P, tt, S[j - 1], -1) + P->MLclosing + P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 7; }
                    if ((k - (i + 1) - 1) >= 0) tmp = (k - (i + 1) - 1) * P->MLbase + H.WMp(k, j - 2) + E_MLstem(P, tt, S[j - 1], S[i + 1]) + P->MLclosing + 2 * P->MLbase;
                    if (tmp < mn) { mn = tmp; best_k = k; best_row = 8; }
                }
                switch (best_row) {
                    case 1: push2(i + 1, best_k - 1, M_WM); push2(best_k, j - 1, M_WM); break;
                    case 2: push2(i + 2, best_k - 1, M_WM); push2(best_k, j - 1, M_WM); break;
                    case 3: push2(i + 1, best_k - 1, M_WM); push2(best_k, j - 2, M_WM); break;
                    case 4: push2(i + 2, best_k - 1, M_WM); push2(best_k, j - 2, M_WM); break;
                    case 5: push2(best_k, j - 1, M_WM); break;
                    case 6: push2(best_k, j - 1, M_WM); break;
                    case 7: push2(best_k, j - 2, M_WM); break;
                    case 8: push2(best_k, j - 2, M_WM); break;
                }
            } break;
        }
    }

    void bt_free(const Interval &cur) {
        const int j = cur.j;
        if (j == 1) return;
        const short *S = H.S;
        const int dangles = c->dangles;
        int mn = INF, tmp = INF, acc = INF, eij = INF;
        int best_row = -1, best_i = -1;
        tmp = c->W[j - 1];
        if (tmp < mn) { mn = tmp; best_row = 0; }
        for (int i = 1; i <= j - 1; i++) {
            acc = (i > 1) ? c->W[i - 1] : 0;
            eij = H.V(i, j);
            if (eij < INF) {
                if (dangles == 2) {
                    const int si1 = i > 1 ? S[i - 1] : -1;
                    const int sj1 = j < n ? S[j + 1] : -1;
                    tmp = eij + E_ExtLoop(H.P, H.pr(i, j), si1, sj1) + acc;
                } else
                    tmp = eij + E_ExtLoop(H.P, H.pr(i, j), -1, -1) + acc;
                if (tmp < mn) { mn = tmp; best_i = i; best_row = 1; }
            }
            if (dangles == 1) {
                eij = H.V(i + 1, j);
                if (eij < INF) {
                    tmp = eij + E_ExtLoop(H.P, H.pr(i + 1, j), S[i], -1) + acc;
                    if (tmp < mn) { mn = tmp; best_i = i; best_row = 2; }
                }
                eij = H.V(i, j - 1);
                if (eij < INF) {
                    tmp = eij + E_ExtLoop(H.P, H.pr(i, j - 1), -1, S[j]) + acc;
                    if (tmp < mn) { mn = tmp; best_i = i; best_row = 3; }
                }
                eij = H.V(i + 1, j - 1);
                if (eij < INF) {
                    tmp = eij + E_ExtLoop(H.P, H.pr(i + 1, j - 1), S[i], S[j]) + acc;
                    if (tmp < mn) { mn = tmp; best_i = i; best_row = 4; }
                }
            }
        }
        for (int i = 1; i <= j - 1; i++) {
            acc = (i - 1 > 0) ? c->W[i - 1] : 0;
            eij = H.Pg(i, j);
            if (eij < INF) {
                tmp = eij + pe.PS + acc;
                if (tmp < mn) { mn = tmp; best_row = 5; best_i = i; }
            }
            if (dangles == 1) {
                eij = H.Pg(i + 1, j);
                if (eij < INF) {
                    tmp = eij + pe.PS + acc;
                    if (tmp < mn) { mn = tmp; best_row = 6; best_i = i; }
                }
                eij = H.Pg(i, j - 1);
                if (eij < INF) {
                    tmp = eij + pe.PS + acc;
                    if (tmp < mn) { mn = tmp; best_row = 7; best_i = i; }
                }
                eij = H.Pg(i + 1, j - 1);
                if (eij < INF) {
                    tmp = eij + pe.PS + acc;
                    if (tmp < mn) { mn = tmp; best_row = 8; best_i = i; }
                }
            }
        }
        switch (best_row) {
            case 0: push2(1, j - 1, FREE); break;
            case 1: push2(best_i, j, LOOP); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
            case 2: push2(best_i + 1, j, LOOP); if (best_i >= 1) push2(1, best_i, FREE); break;
            case 3: push2(best_i, j - 1, LOOP); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
            case 4: push2(best_i + 1, j - 1, LOOP); if (best_i >= 1) push2(1, best_i, FREE); break;
            case 5: push2(best_i, j, P_P); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
            case 6: push2(best_i + 1, j, P_P); if (best_i >= 1) push2(1, best_i, FREE); break;
            case 7: push2(best_i, j - 1, P_P); if (best_i - 1 > 1) push2(1, best_i - 1, FREE); break;
            case 8: push2(best_i + 1, j - 1, P_P); if (best_i >= 1) push2(1, best_i, FREE); break;
        }
    }

    void bt_wm(const Interval &cur) {
        const int i = cur.i, j = cur.j;
        const int MLb = H.P->MLbase;
        int mn = H.WM(i, j - 1) + MLb;
        int best_k = j, best_row = 5;
        for (int k = i; k <= j - TURN - 1; k++) {
            const int m1 = (k - i) * MLb + H.WMv(k, j);
            if (m1 < mn) { mn = m1; best_k = k; best_row = 1; }
            const int m2 = (k - i) * MLb + H.WMp(k, j);
            if (m2 < mn) { mn = m2; best_k = k; best_row = 2; }
            const int m3 = H.WM(i, k - 1) + H.WMv(k, j);
            if (m3 < mn) { mn = m3; best_k = k; best_row = 3; }
            const int m4 = H.WM(i, k - 1) + H.WMp(k, j);
            if (m4 < mn) { mn = m4; best_k = k; best_row = 4; }
        }
        switch (best_row) {
            case 1: push2(best_k, j, M_WMv); break;
            case 2: push2(best_k, j, M_WMp); break;
            case 3: push2(i, best_k - 1, M_WM); push2(best_k, j, M_WMv); break;
            case 4: push2(i, best_k - 1, M_WM); push2(best_k + 1, j, M_WMp); break;  // A-B3
            case 5: push2(i, j - 1, M_WM); break;
        }
    }

    void bt_wmv(const Interval &cur) {
        const int i = cur.i, j = cur.j;
        const short *S = H.S;
        const ccj_energy_params *P = H.P;
        const int si = S[i], sj = S[j];
        const int si1 = (i > 1) ? S[i - 1] : -1;
        const int sj1 = (j < n) ? S[j + 1] : -1;
        int tt = H.pr(i, j);
        int mn = H.V(i, j) + ((c->dangles == 2) ? E_MLstem(P, tt, si1, sj1) : E_MLstem(P, tt, -1, -1));
        int best_row = 1;
        if (c->dangles == 1) {
            tt = H.pr(i + 1, j);
            int tmp = H.V(i + 1, j) + E_MLstem(P, tt, si, -1) + P->MLbase;
            if (tmp < mn) { mn = tmp; best_row = 2; }
            tt = H.pr(i, j - 1);
            tmp = H.V(i, j - 1) + E_MLstem(P, tt, -1, sj) + P->MLbase;
            if (tmp < mn) { mn = tmp; best_row = 3; }
            tt = H.pr(i + 1, j - 1);
            tmp = H.V(i + 1, j - 1) + E_MLstem(P, tt, si, sj) + 2 * P->MLbase;
            if (tmp < mn) { mn = tmp; best_row = 4; }
        }
        const int tmp = H.WMv(i, j - 1) + P->MLbase;
        if (tmp < mn) { mn = tmp; best_row = 5; }
        switch (best_row) {
            case 1: push2(i, j, LOOP); break;
            case 2: push2(i + 1, j, LOOP); break;
            case 3: push2(i, j - 1, LOOP); break;
            case 4: push2(i + 1, j - 1, LOOP); break;
            case 5: push2(i, j - 1, M_WMv); break;
        }
    }

    void bt_wmp(const Interval &cur) {
        const int i = cur.i, j = cur.j;
        int mn = H.Pg(i, j) + pe.PSM + pe.b;
        int best_row = 1;
        const int tmp = H.WMp(i, j - 1) + H.P->MLbase;
        if (tmp < mn) { mn = tmp; best_row = 2; }
        if (best_row == 2) push2(i, j - 1, M_WMp);  // case 1 commented out in reference (A-B2)
    }

    // ---------------------------------------------------------------------------------------
    // pseudo_loop::backtrack, pseudo_loop.cc:861-2820
    // ---------------------------------------------------------------------------------------
    bool in_range4(int i, int j, int k, int l) const {
        return !(i <= 0 || j <= 0 || k <= 0 || l <= 0 || i > n || j > n || k > n || l > n);
    }

    void pl_backtrack(const Interval &cur) {
        const int PB = pe.PB, bp = pe.bp, cp = pe.cp, ap = pe.ap;
        switch (cur.type) {
            case P_P: {
                const int i = cur.i, l = cur.j;
                if (i >= l) die("border case: This should not have happened!, P_P");
                int best_d = 0, best_j = 0, best_k = 0;
                // first (j,d,k) in the reference's loop order whose sum equals the minimum P(i,l):
                // k_pterm keeps it next to the minimum (Pk)
                const int target = H.Pg(i, l);
                if (l - i >= 3 && target < INF / 2) {
                    const unsigned long long key = c->h_pk[c->a2(i, l)];
                    const unsigned sig = (unsigned)(l - i), kk = (unsigned)(key & 0xffffffffull);
                    best_j = i + (int)(kk / (sig * sig));
                    best_d = i + (int)((kk / sig) % sig);
                    best_k = i + (int)(kk % sig);
                }
                push4(i, best_k, best_j, best_d + 1, P_PK);
                push4(best_j + 1, l, best_d, best_k + 1, P_PK);
            } break;

            case P_PK: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PK");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PK");
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = i + 1; d < j; ++d) {
                    tmp = H.g4(PK, i, d, k, l) + H.WP(d + 1, j);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                }
                for (int d = k + 1; d < l; ++d) {
                    tmp = H.g4(PK, i, j, d, l) + H.WP(k, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.g4(PL, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
                tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
                tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 5; best_d = -1; }
                tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 6; best_d = -1; }
                switch (best_row) {
                    case 1: if (best_d > -1) { push4(i, l, best_d, k, P_PK); push2(best_d + 1, j, P_WP); } break;
                    case 2: if (best_d > -1) { push4(i, l, j, best_d, P_PK); push2(k, best_d - 1, P_WP); } break;
                    case 3: push4(i, l, j, k, P_PL); break;
                    case 4: push4(i, l, j, k, P_PM); break;
                    case 5: push4(i, l, j, k, P_PR); break;
                    case 6: push4(i, l, j, k, P_PO); break;
                }
            } break;

            case P_PL: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PL");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PL");
                int mn = INF, tmp, best_row = -1;
                if (H.pr(i, j) > 0) {
                    tmp = get_PLiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                    tmp = get_PXmloop(PLmloop10, PLmloop01, i + 1, j - 1, k, l, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                    if (j >= i + TURN + 1) { tmp = H.g4(PfromL, i + 1, j - 1, k, l); if (tmp < mn) { mn = tmp; best_row = 3; } }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PLiloop); break;
                    case 2: push4(i, l, j, k, P_PLmloop); break;
                    case 3:
                        push4(i + 1, l, j - 1, k, P_PfromL);
                        f[i].pair = j; f[j].pair = i; f[i].type = P_PL; f[j].type = P_PL;
                        break;
                }
            } break;

            case P_PR: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("boder cases: This should not have happened!, P_PR");
                if (i < 0 || j < 0 || k < 0 || l < 0 || i >= n || j >= n || k >= n || l >= n)  // A-B5
                    die("impossible cases: This should not have happened!, P_PR");
                int mn = INF, tmp, best_row = -1;
                if (H.pr(k, l) > 0) {
                    tmp = get_PRiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                    tmp = get_PXmloop(PRmloop10, PRmloop01, i, j, k + 1, l - 1, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                    if (l >= k + TURN + 1) { tmp = H.g4(PfromR, i, j, k + 1, l - 1); if (tmp < mn) { mn = tmp; best_row = 3; } }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PRiloop); break;
                    case 2: push4(i, l, j, k, P_PRmloop); break;
                    case 3:
                        push4(i, l - 1, j, k + 1, P_PfromR);
                        f[k].pair = l; f[l].pair = k; f[k].type = P_PR; f[l].type = P_PR;
                        break;
                }
            } break;

            case P_PM: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PM");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PM");
                if (i == j && k == l) {
                    f[j].pair = k; f[k].pair = j; f[j].type = P_PM; f[k].type = P_PM;
                    return;
                }
                int mn = INF, tmp, best_row = -1;
                if (H.pr(j, k) > 0) {
                    tmp = get_PMiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                    tmp = get_PXmloop(PMmloop10, PMmloop01, i, j - 1, k + 1, l, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                    if (k >= j + TURN - 1) { tmp = H.g4(PfromM, i, j - 1, k + 1, l); if (tmp < mn) { mn = tmp; best_row = 3; } }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PMiloop); break;
                    case 2: push4(i, l, j, k, P_PMmloop); break;
                    case 3:
                        push4(i, l, j - 1, k + 1, P_PfromM);
                        f[j].pair = k; f[k].pair = j; f[j].type = P_PM; f[k].type = P_PM;
                        break;
                }
            } break;

            case P_PO: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PO");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PO");
                int mn = INF, tmp, best_row = -1;
                if (H.pr(i, l) > 0) {
                    tmp = get_POiloop(i, j, k, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                    tmp = get_PXmloop(POmloop10, POmloop01, i + 1, j, k, l - 1, i, j, k, l) + bp; if (tmp < mn) { mn = tmp; best_row = 2; }
                    if (l >= i + TURN + 1) { tmp = H.g4(PfromO, i + 1, j, k, l - 1); if (tmp < mn) { mn = tmp; best_row = 3; } }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_POiloop); break;
                    case 2: push4(i, l, j, k, P_POmloop); break;
                    case 3:
                        push4(i + 1, l - 1, j, k, P_PfromO);
                        f[i].pair = l; f[l].pair = i; f[i].type = P_PO; f[l].type = P_PO;
                        break;
                }
            } break;

            case P_PfromL: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("This should not have happened!, P_PfromL");
                if (!in_range4(i, j, k, l)) die("This should not have happened!, P_PfromL");
                if (i == j && k == l) return;
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = i + 1; d < j; d++) {
                    tmp = H.g4(PfromL, d, j, k, l) + H.WP(i, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                    tmp = H.g4(PfromL, i, d, k, l) + H.WP(d + 1, j);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
                tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
                tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 5; best_d = -1; }
                switch (best_row) {
                    case 1: if (best_d > -1) { push4(best_d, l, j, k, P_PfromL); push2(i, best_d - 1, P_WP); } break;
                    case 2: if (best_d > -1) { push4(i, l, best_d, k, P_PfromL); push2(best_d + 1, j, P_WP); } break;
                    case 3: push4(i, l, j, k, P_PR); break;
                    case 4: push4(i, l, j, k, P_PM); break;
                    case 5: push4(i, l, j, k, P_PO); break;
                }
            } break;

            case P_PfromR: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("This should not have happened!, P_PfromR");
                if (!in_range4(i, j, k, l)) die("impossible case: This should not have happened!, P_PfromR");
                if (i == j && k == l) return;
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = k + 1; d < l; d++) {
                    tmp = H.g4(PfromR, i, j, d, l) + H.WP(k, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                    tmp = H.g4(PfromR, i, j, k, d) + H.WP(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.g4(PM, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
                tmp = H.g4(PO, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
                switch (best_row) {
                    case 1: if (best_d > -1) { push4(i, l, j, best_d, P_PfromR); push2(k, best_d - 1, P_WP); } break;
                    case 2: if (best_d > -1) { push4(i, best_d, j, k, P_PfromR); push2(best_d + 1, l, P_WP); } break;
                    case 3: push4(i, l, j, k, P_PM); break;
                    case 4: push4(i, l, j, k, P_PO); break;
                }
            } break;

            case P_PfromM: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("This should not have happened!, P_PfromM");
                if (!in_range4(i, j, k, l)) die("This should not have happened!, P_PfromM");
                if (i == j && k == l) return;
                int mn = INF, tmp, best_d = -1;
                for (int d = i + 1; d < j; d++) {
                    tmp = H.g4(PfromMprime, i, d, k, l) + H.WP(d + 1, j);
                    if (tmp < mn) { mn = tmp; best_d = d; }
                }
                if (best_d > -1) { push4(i, l, best_d, k, P_PfromMprime); push2(best_d + 1, j, P_WP); }
            } break;

            case P_PfromO: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PfromO");
                if (!in_range4(i, j, k, l)) die("impossible case: This should not have happened!, P_PfromO");
                if (i == j && k == l) return;
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = i + 1; d < j; d++) {
                    tmp = H.g4(PfromO, d, j, k, l) + H.WP(i, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                }
                for (int d = k + 1; d < l; d++) {
                    tmp = H.g4(PfromO, i, j, k, d) + H.WP(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.g4(PL, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 3; best_d = -1; }
                tmp = H.g4(PR, i, j, k, l) + PB; if (tmp < mn) { mn = tmp; best_row = 4; best_d = -1; }
                switch (best_row) {
                    case 1: if (best_d > -1) { push4(best_d, l, j, k, P_PfromO); push2(i, best_d - 1, P_WP); } break;
                    case 2: if (best_d > -1) { push4(i, best_d, j, k, P_PfromO); push2(best_d + 1, l, P_WP); } break;
                    case 3: push4(i, l, j, k, P_PL); break;
                    case 4: push4(i, l, j, k, P_PR); break;
                }
            } break;

            case P_WB: {
                const int i = cur.i, l = cur.j;
                if (i <= 0 || l <= 0 || i > n || l > n) die("impossible cases: This should not have happened!, P_WB");
                if (i > l) return;
                int mn = INF, tmp, best_row = -1;
                tmp = H.WBPg(i, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = cp * (l - i + 1); if (tmp < mn) { mn = tmp; best_row = 2; }
                if (best_row == 1) push2(i, l, P_WBP);
            } break;

            case P_WBP: {
                const int i = cur.i, l = cur.j;
                if (i > l) die("border case: This should not have happened!, P_WBP");
                if (i <= 0 || l <= 0 || i > n || l > n) die("impossible cases: This should not have happened!, P_WBP");
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = i; d < l; d++) {
                    tmp = H.WB(i, d - 1) + H.V(d, l) + bp + pe.PPS;
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                    tmp = H.WB(i, d - 1) + H.Pg(d, l) + pe.PSM + pe.PPS;
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.WBPg(i, l - 1) + cp;
                if (tmp < mn) { mn = tmp; best_row = 3; }
                switch (best_row) {
                    case 1: push2(i, best_d - 1, P_WB); push2(best_d, l, LOOP); break;
                    case 2: push2(i, best_d - 1, P_WB); push2(best_d, l, P_P); break;
                    case 3: push2(i, l - 1, P_WBP); break;
                }
            } break;

            case P_WP: {
                const int i = cur.i, l = cur.j;
                if (i <= 0 || l <= 0 || i > n || l > n) die("impossible cases: This should not have happened!, P_WP");
                if (i > l) return;
                int mn = INF, tmp, best_row = -1;
                tmp = H.WPPg(i, l); if (tmp < mn) { mn = tmp; best_row = 1; }
                tmp = pe.PUP * (l - i + 1); if (tmp < mn) { mn = tmp; best_row = 2; }
                if (best_row == 1) push2(i, l, P_WPP);
            } break;

            case P_WPP: {
                const int i = cur.i, l = cur.j;
                if (i > l) die("border case: This should not have happened!, P_WPP");
                if (i <= 0 || l <= 0 || i > n || l > n) die("impossible cases: This should not have happened!, P_WPP");
                int mn = INF, tmp, best_row = -1, best_d = -1;
                for (int d = i; d < l; d++) {
                    tmp = H.WP(i, d - 1) + H.V(d, l) + 0 + pe.PPS;
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                    tmp = H.WP(i, d - 1) + H.Pg(d, l) + pe.PSP + pe.PPS;
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                tmp = H.WPPg(i, l - 1) + pe.PUP;
                if (tmp < mn) { mn = tmp; best_row = 3; }
                switch (best_row) {
                    case 1: push2(i, best_d - 1, P_WP); push2(best_d, l, LOOP); break;
                    case 2: push2(i, best_d - 1, P_WP); push2(best_d, l, P_P); break;
                    case 3: push2(i, l - 1, P_WPP); break;
                }
            } break;

            case P_PLiloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i < j && j < k - 1 && k < l)) die("border cases: This should not have happened!, P_PLiloop");
                if (!in_range4(i, j, k, l)) die("impossbible cases: This should not have happened!, P_PLiloop");
                f[i].pair = j; f[j].pair = i; f[i].type = P_PLiloop; f[j].type = P_PLiloop;
                int mn = INF, tmp, best_row = -1, best_d = -1, best_dp = -1;
                if (H.pr(i, j) > 0) {
                    tmp = H.g4(PL, i + 1, j - 1, k, l) + H.e_stP(i, j);  // no i+TURN+2<j test here
                    if (tmp < mn) { mn = tmp; best_row = 1; }
                    const int max_d = std::min(j, i + MAXLOOP);
                    for (int d = i + 1; d < max_d; ++d) {
                        const int min_dp = std::max(d + TURN, j - MAXLOOP);
                        for (int dp = j - 1; dp > min_dp; --dp) {  // no can_pair filter here
                            tmp = H.e_intP(i, d, dp, j) + H.g4(PL, d, dp, k, l);
                            if (tmp < mn) { mn = tmp; best_d = d; best_dp = dp; best_row = 2; }
                        }
                    }
                }
                switch (best_row) {
                    case 1: push4(i + 1, l, j - 1, k, P_PL); break;
                    case 2: push4(best_d, l, best_dp, k, P_PL); break;
                }
            } break;

            case P_PLmloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PLmloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PLmloop");
                f[i].pair = j; f[j].pair = i; f[i].type = P_PLmloop; f[j].type = P_PLmloop;
                const int br1 = H.g4(PLmloop10, i + 1, j - 1, k, l) + ap + bp;
                const int br2 = H.g4(PLmloop01, i + 1, j - 1, k, l) + ap + bp;
                if (br1 < br2) push4(i + 1, l, j - 1, k, P_PLmloop10);
                else push4(i + 1, l, j - 1, k, P_PLmloop01);
            } break;

            case P_PLmloop00: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PLmloop00");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PLmloop00");
                int mn = H.g4(PL, i, j, k, l) + bp, tmp;
                int best_row = 1, best_d = -1;
                for (int d = i; d <= j; ++d) {
                    if (d > i) {
                        tmp = H.WB(i, d - 1) + H.g4(PLmloop00, d, j, k, l);
                        if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                    }
                    if (d < j) {
                        tmp = H.g4(PLmloop00, i, d, k, l) + H.WB(d + 1, j);
                        if (tmp < mn) { mn = tmp; best_row = 3; best_d = d; }
                    }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PL); break;
                    case 2: push4(best_d, l, j, k, P_PLmloop00); push2(i, best_d - 1, P_WB); break;
                    case 3: push4(i, l, best_d, k, P_PLmloop00); push2(best_d + 1, j, P_WB); break;
                }
            } break;

            case P_PLmloop01: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PLmloop01");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PLmloop01");
                int mn = INF, tmp, best_d = -1;
                for (int d = i; d < j; ++d) {
                    tmp = H.g4(PLmloop00, i, d, k, l) + H.WBPg(d + 1, j);
                    if (tmp < mn) { mn = tmp; best_d = d; }
                }
                push4(i, l, best_d, k, P_PLmloop00);
                push2(best_d + 1, j, P_WBP);
            } break;

            case P_PLmloop10: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PLmloop10");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PLmloop10");
                int mn = INF, tmp, best_d = -1, best_row = -1;
                for (int d = i + 1; d <= j; ++d) {
                    tmp = H.WBPg(i, d - 1) + H.g4(PLmloop00, d, j, k, l);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                    if (d < j) {
                        tmp = H.g4(PLmloop10, i, d, k, l) + H.WB(d + 1, j);
                        if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                    }
                }
                switch (best_row) {
                    case 1: push2(i, best_d - 1, P_WBP); push4(best_d, l, j, k, P_PLmloop00); break;
                    case 2: push4(i, l, best_d, k, P_PLmloop10); push2(best_d + 1, j, P_WB); break;
                }
            } break;

            case P_PRiloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PRiloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PRiloop");
                f[k].pair = l; f[l].pair = k; f[k].type = P_PRiloop; f[l].type = P_PRiloop;
                int mn = INF, tmp, best_row = -1, best_d = -1, best_dp = -1;
                if (H.pr(k, l) > 0) {
                    tmp = H.g4(PR, i, j, k + 1, l - 1) + H.e_stP(k, l);
                    if (tmp < mn) { mn = tmp; best_row = 1; }
                    const int max_d = std::min(l, k + MAXLOOP);
                    for (int d = k + 1; d < max_d; ++d) {
                        const int min_dp = std::max(d + TURN, l - MAXLOOP);
                        for (int dp = l - 1; dp > min_dp; --dp) {
                            tmp = H.e_intP(k, d, dp, l) + H.g4(PR, i, j, d, dp);
                            if (tmp < mn) { mn = tmp; best_d = d; best_dp = dp; best_row = 2; }
                        }
                    }
                }
                switch (best_row) {
                    case 1: push4(i, l - 1, j, k + 1, P_PR); break;
                    case 2: push4(i, best_dp, j, best_d, P_PR); break;
                }
            } break;

            case P_PRmloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PRmloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PRmloop");
                f[k].pair = l; f[l].pair = k; f[k].type = P_PRmloop; f[l].type = P_PRmloop;
                const int br1 = H.g4(PRmloop10, i, j, k + 1, l - 1) + ap + bp;
                const int br2 = H.g4(PRmloop01, i, j, k + 1, l - 1) + ap + bp;
                if (br1 < br2) push4(i, l - 1, j, k + 1, P_PRmloop10);
                else push4(i, l - 1, j, k + 1, P_PRmloop01);
            } break;

            case P_PRmloop00: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PRmloop00");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PRmloop00");
                int mn = H.g4(PR, i, j, k, l) + bp, tmp;
                int best_row = 1, best_d = -1;
                for (int d = k; d <= l; ++d) {
                    if (d > k) {
                        tmp = H.WB(k, d - 1) + H.g4(PRmloop00, i, j, d, l);
                        if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                    }
                    if (d < l) {
                        tmp = H.g4(PRmloop00, i, j, k, d) + H.WB(d + 1, l);
                        if (tmp < mn) { mn = tmp; best_row = 3; best_d = d; }
                    }
                }
                switch (best_row) {  // A-B4: (i,j,k,l) argument order
                    case 1: push4(i, j, k, l, P_PR); break;
                    case 2: push4(i, j, best_d, l, P_PRmloop00); push2(k, best_d - 1, P_WB); break;
                    case 3: push4(i, j, k, best_d, P_PRmloop00); push2(best_d + 1, l, P_WB); break;
                }
            } break;

            case P_PRmloop01: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PRmloop01");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PRmloop01");
                int mn = H.g4(PRmloop01, i, j, k, l - 1) + cp, tmp;
                int best_row = 1, best_d = -1;
                for (int d = k; d < l; d++) {
                    tmp = H.g4(PRmloop00, i, j, k, d) + H.WBPg(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l - 1, j, k, P_PRmloop01); break;
                    case 2: push2(best_d + 1, l, P_WBP); push4(i, best_d, j, k, P_PRmloop00); break;
                }
            } break;

            case P_PRmloop10: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PRmloop10");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PRmloop10");
                int mn = H.g4(PRmloop10, i, j, k + 1, l) + cp, tmp;
                int best_row = 1, best_d = -1;
                for (int d = k + 1; d <= l; ++d) {
                    tmp = H.WBPg(k, d - 1) + H.g4(PRmloop00, i, j, d, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k + 1, P_PRmloop10); break;
                    case 2: push2(k, best_d - 1, P_WBP); push4(i, l, j, best_d, P_PRmloop00); break;
                }
            } break;

            case P_PMiloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PMiloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PMiloop");
                f[j].pair = k; f[k].pair = j; f[j].type = P_PMiloop; f[k].type = P_PMiloop;
                int mn = INF, tmp, best_d = -1, best_dp = -1, best_row = -1;
                if (H.pr(j, k) > 0) {
                    tmp = H.g4(PM, i, j - 1, k + 1, l) + H.e_stP(j - 1, k + 1);
                    if (tmp < mn) { mn = tmp; best_row = 1; }
                    const int max_d = std::max(i, j - MAXLOOP);
                    for (int d = j - 1; d > max_d; --d) {
                        const int min_dp = std::min(l, k + MAXLOOP);
                        for (int dp = k + 1; dp < min_dp; ++dp) {
                            tmp = H.e_intP(d, j, k, dp) + H.g4(PM, i, d, dp, l);
                            if (tmp < mn) { mn = tmp; best_d = d; best_dp = dp; best_row = 2; }
                        }
                    }
                }
                switch (best_row) {
                    case 1: push4(i, l, j - 1, k + 1, P_PM); break;
                    case 2: push4(i, l, best_d, best_dp, P_PM); break;
                }
            } break;

            case P_PMmloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PMmloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PMmloop");
                f[j].pair = k; f[k].pair = j; f[j].type = P_PMmloop; f[k].type = P_PMmloop;
                const int br1 = H.g4(PMmloop10, i, j - 1, k + 1, l) + ap + bp;
                const int br2 = H.g4(PMmloop01, i, j - 1, k + 1, l) + ap + bp;
                if (br1 < br2) push4(i, l, j - 1, k + 1, P_PMmloop10);
                else push4(i, l, j - 1, k + 1, P_PMmloop01);
            } break;

            case P_PMmloop00: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PMmloop00");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PMmloop00");
                f[j].pair = k; f[k].pair = j; f[j].type = P_PMmloop; f[k].type = P_PMmloop;
                int tmp, mn = H.g4(PM, i, j, k, l) + bp;
                int best_row = 1, best_d = -1;
                for (int d = i; d < j; ++d) {
                    tmp = H.WB(d + 1, j) + H.g4(PMmloop00, i, d, k, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                for (int d = k + 1; d <= l; d++) {
                    tmp = H.g4(PMmloop00, i, j, d, l) + H.WB(k, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 3; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PM); break;
                    case 2: push4(i, l, best_d, k, P_PMmloop00); push2(best_d + 1, j, P_WB); break;
                    case 3: push4(i, l, j, best_d, P_PMmloop00); push2(k, best_d - 1, P_WB); break;
                }
            } break;

            case P_PMmloop01: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PMmloop01");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PMmloop01");
                int tmp, mn = H.g4(PMmloop01, i, j, k + 1, l) + cp;
                int best_row = 1, best_d = -1;
                for (int d = k + 1; d <= l; ++d) {
                    tmp = H.g4(PMmloop00, i, j, d, l) + H.WBPg(k, d - 1);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k + 1, P_PMmloop01); break;
                    case 2: push4(i, l, j, best_d, P_PMmloop00); push2(k, best_d - 1, P_WBP); break;
                }
            } break;

            case P_PMmloop10: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_PMmloop10");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_PMmloop10");
                int tmp, mn = H.g4(PMmloop10, i, j - 1, k, l) + cp;
                int best_row = 1, best_d = -1;
                for (int d = i + 1; d < j; ++d) {
                    tmp = H.WBPg(d, j) + H.g4(PMmloop00, i, d - 1, k, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l, j - 1, k, P_PMmloop10); break;
                    case 2: push4(i, l, best_d - 1, k, P_PMmloop00); push2(best_d, j, P_WBP); break;
                }
            } break;

            case P_POiloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_POiloop");
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_POiloop");
                f[i].pair = l; f[l].pair = i; f[i].type = P_POiloop; f[l].type = P_POiloop;
                int mn = INF, best_d = -1, best_dp = -1, best_row = -1;
                if (H.pr(i, l) > 0) {
                    const int tmp = H.g4(PO, i + 1, j, k, l - 1) + H.e_stP(i, l);
                    if (tmp < mn) { mn = tmp; best_row = 1; }
                    const int max_d = std::min(j, i + MAXLOOP);
                    for (int d = i + 1; d < max_d; ++d) {
                        const int min_dp = std::max(l - MAXLOOP, k);
                        for (int dp = l - 1; dp > min_dp; --dp) {
                            const int br2 = H.e_intP(i, d, dp, l) + H.g4(PO, d, j, dp, k);
                            if (br2 < mn) { mn = br2; best_row = 2; best_d = d; best_dp = dp; }
                        }
                    }
                }
                switch (best_row) {
                    case 1: push4(i + 1, l - 1, j, k, P_PO); break;
                    case 2: push4(best_d, k, j, best_dp, P_PO); break;
                }
            } break;

            case P_POmloop: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_POmloop");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_POmloop");
                f[i].pair = l; f[l].pair = i; f[i].type = P_POmloop; f[l].type = P_POmloop;
                const int br1 = H.g4(POmloop10, i + 1, j, k, l - 1) + ap + bp;
                const int br2 = H.g4(POmloop01, i + 1, j, k, l - 1) + ap + bp;
                if (br1 < br2) push4(i + 1, l - 1, j, k, P_POmloop10);
                else push4(i + 1, l - 1, j, k, P_POmloop01);
            } break;

            case P_POmloop00: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_POmloop00");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_POmloop00");
                int mn = H.g4(PO, i, j, k, l) + bp, tmp;
                int best_row = 1, best_d = -1;
                for (int d = i + 1; d <= j; ++d) {
                    tmp = H.WB(i, d - 1) + H.g4(POmloop00, d, j, k, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                for (int d = k; d < l; ++d) {
                    tmp = H.g4(POmloop00, i, j, k, d) + H.WB(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_row = 3; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(i, l, j, k, P_PO); break;
                    case 2: push4(best_d, l, j, k, P_POmloop00); push2(i, best_d - 1, P_WBP); break;  // sic
                    case 3: push4(i, best_d, j, k, P_POmloop00); push2(best_d + 1, l, P_WB); break;
                }
            } break;

            case P_POmloop01: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_POmloop01");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_POmloop01");
                int mn = INF, tmp, best_d = -1;
                for (int d = k; d < l; d++) {
                    tmp = H.g4(POmloop00, i, j, k, d) + H.WBPg(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_d = d; }
                }
                push4(i, best_d, j, k, P_POmloop00);
                push2(best_d + 1, l, P_WBP);
            } break;

            case P_POmloop10: {
                const int i = cur.i, l = cur.j, j = cur.k, k = cur.l;
                if (!(i <= j && j < k - 1 && k <= l)) die("border cases: This should not have happened!, P_POmloop10");
                if (!in_range4(i, j, k, l)) die("impossible cases: This should not have happened!, P_POmloop10");
                int mn = INF, tmp, best_d = -1, best_row = -1;
                for (int d = i + 1; d <= j; ++d) {
                    tmp = H.WBPg(i, d - 1) + H.g4(POmloop00, d, j, k, l);
                    if (tmp < mn) { mn = tmp; best_row = 1; best_d = d; }
                }
                for (int d = k + 1; d < l; ++d) {
                    tmp = H.g4(POmloop10, i, j, k, d) + H.WB(d + 1, l);
                    if (tmp < mn) { mn = tmp; best_row = 2; best_d = d; }
                }
                switch (best_row) {
                    case 1: push4(best_d, l, j, k, P_POmloop00); push2(i, best_d - 1, P_WBP); break;
                    case 2: push4(i, best_d, j, k, P_POmloop10); push2(best_d + 1, l, P_WB); break;
                }
            } break;

            default:
                break;  // P_PLiloop5 etc.: no case in pseudo_loop::backtrack
        }
    }

    // get_P?iloop (forward versions, with the can_pair filter), pseudo_loop.cc:682-808
    int get_PLiloop(int i, int j, int k, int l) {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (!H.can_pair(i, j)) return INF;
        int mn = INF;
        if (i + TURN + 2 < j) mn = H.g4(PL, i + 1, j - 1, k, l) + H.e_stP(i, j);
        const int max_d = std::min(j, i + MAXLOOP);
        for (int d = i + 1; d < max_d; ++d) {
            const int min_dp = std::max(d + TURN, j - MAXLOOP);
            for (int dp = j - 1; dp > min_dp; --dp) {
                if (!H.can_pair(d, dp)) continue;
                mn = std::min(mn, H.e_intP(i, d, dp, j) + H.g4(PL, d, dp, k, l));
            }
        }
        return mn;
    }
    int get_PRiloop(int i, int j, int k, int l) {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (!H.can_pair(k, l)) return INF;
        int mn = INF;
        if (k + TURN + 2 < l) mn = H.g4(PR, i, j, k + 1, l - 1) + H.e_stP(k, l);
        const int max_d = std::min(l, k + MAXLOOP);
        for (int d = k + 1; d < max_d; ++d) {
            const int min_dp = std::max(d + TURN, l - MAXLOOP);
            for (int dp = l - 1; dp > min_dp; --dp) {
                if (!H.can_pair(d, dp)) continue;
                mn = std::min(mn, H.e_intP(k, d, dp, l) + H.g4(PR, i, j, d, dp));
            }
        }
        return mn;
    }
    int get_PMiloop(int i, int j, int k, int l) {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (!H.can_pair(j, k)) return INF;
        int mn = INF;
        if (i < j && k < l) mn = H.g4(PM, i, j - 1, k + 1, l) + H.e_stP(j - 1, k + 1);
        const int max_d = std::max(i, j - MAXLOOP);
        for (int d = j - 1; d > max_d; --d) {
            const int min_dp = std::min(l, k + MAXLOOP);
            for (int dp = k + 1; dp < min_dp; ++dp) {
                if (!H.can_pair(d, dp)) continue;
                mn = std::min(mn, H.e_intP(d, j, k, dp) + H.g4(PM, i, d, dp, l));
            }
        }
        return mn;
    }
    int get_POiloop(int i, int j, int k, int l) {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        if (!H.can_pair(i, l)) return INF;
        int mn = INF;
        if (i < j && k < l) mn = H.g4(PO, i + 1, j, k, l - 1) + H.e_stP(i, l);
        const int max_d = std::min(j, i + MAXLOOP);
        for (int d = i + 1; d < max_d; ++d) {
            const int min_dp = std::max(l - MAXLOOP, k);
            for (int dp = l - 1; dp > min_dp; --dp) {
                if (!H.can_pair(d, dp)) continue;
                mn = std::min(mn, H.e_intP(i, d, dp, l) + H.g4(PO, d, j, dp, k));
            }
        }
        return mn;
    }
    // get_P?mloop (pseudo_loop.cc:705-820): validity of the outer cell, then min of the two
    int get_PXmloop(int m10, int m01, int i2, int j2, int k2, int l2, int i, int j, int k, int l) {
        if (!(i <= j && j < k - 1 && k <= l)) return INF;
        const int b1 = H.g4(m10, i2, j2, k2, l2) + pe.ap + pe.bp;
        const int b2 = H.g4(m01, i2, j2, k2, l2) + pe.ap + pe.bp;
        return std::min(b1, b2);
    }

    // W_final::fill_structure, W_final.cc:764-819
    void fill_structure() {
        struct Brack { char open, close; };
        struct Band { char open, close; int outer_start, outer_end, inner_start, inner_end; };
        std::stack<Brack> st;
        st.push({'<', '>'});
        st.push({'{', '}'});
        st.push({'[', ']'});
        st.push({'(', ')'});
        std::list<Band> bands;
        bands.push_back({'|', '|', 0, 0, 0, 0});
        for (int i = 1; i <= n; i++) {
            const int j = f[i].pair;
            if (j == -1) {
                structure[i] = '.';
            } else if (i < j) {
                bool inband = false;
                for (auto it = bands.begin(); it != bands.end(); ++it) {
                    if (i > it->inner_start && j < it->inner_end) {
                        it->inner_start = i;
                        it->inner_end = j;
                        structure[i] = it->open;
                        structure[j] = it->close;
                        inband = true;
                        break;
                    }
                }
                if (!inband) {
                    if (st.empty()) throw BacktrackExit{139, "CCJ: fill_structure: more than 4 crossing bands (reference pops an empty std::stack)\n"};
                    Brack e = st.top();
                    st.pop();
                    bands.push_back({e.open, e.close, i, j, i, j});
                    structure[i] = e.open;
                    structure[j] = e.close;
                }
            } else {
                for (auto it = bands.begin(); it != bands.end(); ++it) {
                    if (i == it->outer_end) {
                        st.push({it->open, it->close});
                        break;
                    }
                }
            }
        }
    }
};

uint64_t fnv(uint64_t h, const void *p, size_t nb) {
    const unsigned char *c = (const unsigned char *)p;
    for (size_t x = 0; x < nb; ++x) { h ^= c[x]; h *= 1099511628211ull; }
    return h;
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" uint64_t ccj_num_cells(int n) {
    if (n < 3) return 0;
    const uint64_t m = (uint64_t)n + 1;
    return m * (m - 1) * (m - 2) * (m - 3) / 24;
}

static thread_local std::string g_create_err;


// One part of a level's exchange through the in-process group: every member pulls each member's
// packed slice of the part into its own receive buffer (same device) on stream q, between two
// barriers, so no slice is overwritten by the part's next pack before every member has read it.
static int local_allgather(ccj_ctx *c, int part, size_t slice, hipStream_t q) {
    ccj_group *g = c->lgroup;
    HIPCHK(c, hipStreamSynchronize(q));  // own slice packed
    if (!g->barrier()) return set_err(c, CCJ_E_STATE, "local exchange: a group member failed");
    // take the peers' send buffers under the lock and hold the group busy until the copies are
    // done: ccj_destroy of a peer waits for busy == 0 before it frees anything
    std::vector<const int16_t *> src(g->world, nullptr);
    {
        std::lock_guard<std::mutex> lk(g->mu);
        for (int r = 0; r < g->world; ++r) {
            if (!g->members[r]) {
                g->broken = true;  // every other member's next barrier fails instead of waiting
                g->cv.notify_all();
                return set_err(c, CCJ_E_STATE, "local exchange: rank %d has no context", r);
            }
            src[r] = g->members[r]->d_send[part];
        }
        ++g->busy;
    }
    hipError_t e = hipSuccess;
    for (int r = 0; r < g->world && e == hipSuccess; ++r)
        e = hipMemcpyAsync(c->d_recv[part] + (size_t)r * slice, src[r], slice * sizeof(int16_t), hipMemcpyDeviceToDevice, q);
    const hipError_t e2 = hipStreamSynchronize(q);
    {
        std::lock_guard<std::mutex> lk(g->mu);
        --g->busy;
        g->cv.notify_all();
    }
    HIPCHK(c, e);
    HIPCHK(c, e2);
    if (!g->barrier()) return set_err(c, CCJ_E_STATE, "local exchange: a group member failed");
    return CCJ_OK;
}

// The bulk part of a level's exchange through the in-process group, without blocking the host: after
// one barrier (every member has recorded its ev_bpacked for this level), each member's bulk slice is
// copied on this member's side stream behind that member's ev_bpacked, and ev_bcopied marks the copies
// (a member's next bulk pack waits for every member's ev_bcopied, bulk_start).  The level chain keeps
// running meanwhile; only the edge part (local_allgather) synchronises the host with the level.
static int local_bulk_gather(ccj_ctx *c, size_t slice) {
    ccj_group *g = c->lgroup;
    if (!g->barrier()) return set_err(c, CCJ_E_STATE, "local exchange: a group member failed");
    std::lock_guard<std::mutex> lk(g->mu);
    for (int r = 0; r < g->world; ++r) {
        const ccj_ctx *p = g->members[r];
        if (!p) {
            g->broken = true;
            g->cv.notify_all();
            return set_err(c, CCJ_E_STATE, "local exchange: rank %d has no context", r);
        }
        HIPCHK(c, hipStreamWaitEvent(c->st_x, p->ev_bpacked, 0));
        HIPCHK(c, hipMemcpyAsync(c->d_recv[XCH_BULK] + (size_t)r * slice, p->d_send[XCH_BULK], slice * sizeof(int16_t),
                                 hipMemcpyDeviceToDevice, c->st_x));
    }
    HIPCHK(c, hipEventRecord(c->ev_bcopied, c->st_x));
    return CCJ_OK;
}
// before this member's next bulk pack overwrites its send slice: every member's copies of it are done
static int local_bulk_wait_copied(ccj_ctx *c) {
    ccj_group *g = c->lgroup;
    std::lock_guard<std::mutex> lk(g->mu);
    for (int r = 0; r < g->world; ++r)
        if (const ccj_ctx *p = g->members[r]) HIPCHK(c, hipStreamWaitEvent(c->st_x, p->ev_bcopied, 0));
    return CCJ_OK;
}

// Everything that depends on the sequence itself (not only on n): the encoding, the pair-type,
// hairpin and e_stP tables, and the k_iloop work items.  ccj_create runs it once, ccj_reset for
// each new sequence of the same length (the allocations are reused).
static int seq_setup(ccj_ctx *c) {
    ccj_ctx *cp = c;
    const int n = c->n;
    const bool trace = getenv("CCJ_TRACE_SETUP") != nullptr;
    auto tp0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!trace) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "seq_setup %-10s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp0).count());
        tp0 = now;
    };
    const size_t plane = (size_t)(n + 1) * c->rs;
    // pair_mat.h:159-183 encode_sequence
    c->S.assign(n + 2, 0);
    c->S1.assign(n + 2, 0);
    for (int i = 1; i <= n; ++i) c->S[i] = c->S1[i] = (short)encode_base(c->seq[i - 1]);
    c->S[n + 1] = c->S[1];
    c->S[0] = (short)n;
    c->S1[n + 1] = c->S1[1];
    c->S1[0] = c->S1[n];
    // ---- host-side sequence tables: pair types, hairpins, e_stP
    std::vector<int8_t> pt(plane, 0);
    std::vector<int> hp(plane, INF);
    std::vector<int16_t> est(plane, (int16_t)INTERN_INF);
    c->hpt_h.assign(plane, 0);
    for (int w = 0; w < n; ++w)
        for (int p = 1; p + w <= n; ++p) {
            const size_t x = (size_t)w * c->rs + p;
            const int tc = c->pair[c->S[p]][c->S[p + w]];
            pt[x] = (int8_t)tc;
            c->hpt_h[x] = tc;
        }
    // the energy tables, built on the host while the GPU counts the work items (below)
    const char *tab_err = nullptr;
    auto energy_tables = [&]() {
        for (int w = 0; w < n; ++w)
            for (int p = 1; p + w <= n; ++p) {
                const int q = p + w;
                const size_t x = (size_t)w * c->rs + p;
                const int tc = pt[x];
                // HairpinE, s_energy_matrix.cc:275-282
                hp[x] = (tc == 0) ? INF
                                  : E_Hairpin_host(&c->prm, c->lx.data(), w - 1, tc, c->S1[p + 1], c->S1[q - 1],
                                                   c->seq.c_str() + p - 1);
                // get_e_stP, pseudo_loop.cc:828-834 (saturated, see k_precompute_ie)
                if (q - p >= 2 && p + 1 != q - 1) {
                    const int t2 = c->pair[c->S[p + 1]][c->S[q - 1]];
                    const int e = E_IntLoop(&c->prm, c->lx.data(), 0, 0, tc, c->rtype[t2], c->S1[p + 1], c->S1[q - 1],
                                            c->S1[p], c->S1[q]);
                    const long v = lrint(c->e_stP * e);
                    if (v < -32768) { tab_err = "e_stP below int16 range"; return; }
                    if (tc > 0 && t2 > 0 && v >= INTERN_INF) { tab_err = "e_stP of a canonical stack >= 32767"; return; }
                    est[x] = (int16_t)(v >= INTERN_INF ? INTERN_INF : v);
                }
            }
    };
    lap("pair types");
    // the sequence tables go up asynchronously on st from pinned staging (a reset never blocks on
    // work another context has running on the GPU); the fill's launches follow on st
    const size_t stage_bytes = plane * (1 + sizeof(int) + sizeof(int16_t)) + 2 * (size_t)(n + 2) * sizeof(short);
    if (!c->h_stage) {
        HIPCHK(cp, hipHostMalloc(&c->h_stage, stage_bytes, hipHostMallocDefault));
        HIPCHK(cp, hipEventCreateWithFlags(&c->ev_stage, hipEventDisableTiming));
    } else {
        HIPCHK(cp, hipEventSynchronize(c->ev_stage));  // the previous uploads have read the staging
    }
    char *stg = (char *)c->h_stage;
    auto up = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
        memcpy(stg, src, bytes);
        const hipError_t e = hipMemcpyAsync(dst, stg, bytes, hipMemcpyHostToDevice, c->st);
        stg += bytes;
        return e;
    };
    HIPCHK(cp, up(c->d_pt, pt.data(), plane));
    // ---- k_iloop work items (one per wave), counted per (level, shard), then written by k_items
    // on the GPU at the prefix offsets.  By default the count pass runs on the GPU too (k_items
    // pass 0 on st) and the host WAITS for it (hipStreamSynchronize): the offsets are needed on
    // the host to size the k_iloop launches, so ccj_reset blocks until the context's stream has
    // run it.  CCJ_HOST_COUNT=1 counts on host threads instead (the same enumeration, ccj_items.h;
    // slower, ~1.3 ms at n=200, but no device round trip).
    if (n > 1023) return set_err(cp, CCJ_E_ARG, "sequence longer than 1023 (k_iloop item encoding)");
    {
        const int G = c->world;
        const int nb = n * G;
        const int rs = c->rs;
        struct HostPT {
            const int8_t *pt;
            int rs;
            int operator()(int i, int j) const { return pt[(size_t)(j - i) * rs + i]; }
        } hpt{pt.data(), rs};
        std::vector<long long> cnt((size_t)nb, 0), cnt2((size_t)nb * KI_SPLIT, 0);  // per (t, r) / per split
        // default: counted on the GPU by k_items (KI_SPLIT workgroups per level, then one round
        // trip); CCJ_HOST_COUNT=1: on host threads (slower, but no device round trip, so a reset
        // never waits behind another context's fill on a shared hardware queue)
        static const bool host_count = getenv("CCJ_HOST_COUNT") && atoi(getenv("CCJ_HOST_COUNT")) != 0;
        if (!host_count) {
            HIPCHK(cp, (hipError_t)ccjk_items(&c->T, G, c->rank, c->simulate, c->d_icount, nullptr, nullptr, 0, c->st));
            if (!c->h_icount) HIPCHK(cp, hipHostMalloc(&c->h_icount, cnt2.size() * sizeof(long long), hipHostMallocDefault));
            HIPCHK(cp, hipMemcpyAsync(c->h_icount, c->d_icount, cnt2.size() * sizeof(long long), hipMemcpyDeviceToHost, c->st));
            energy_tables();
            lap("tables");
            HIPCHK(cp, hipStreamSynchronize(c->st));
            memcpy(cnt2.data(), c->h_icount, cnt2.size() * sizeof(long long));
        } else {
            energy_tables();
            lap("tables");
        }
        if (tab_err) return set_err(cp, CCJ_E_PARAMS, "%s", tab_err);
        std::atomic<int> next{0};
        static const bool check = getenv("CCJ_CHECK_ITEMS") && atoi(getenv("CCJ_CHECK_ITEMS")) != 0;
        std::atomic<bool> bad{false};
        auto worker = [&]() {
            for (int b; (b = next.fetch_add(1)) < nb;) {
                const int t = b / G, r = b % G;
                if (!(c->simulate || r == c->rank) || t < 4 || t >= c->nlev) continue;
                const long long hc = count_level_items(pt.data(), rs, n, t, G, r, IL_CW);
                long long gpu = 0;
                for (int s = 0; s < KI_SPLIT; ++s) gpu += cnt2[(size_t)b * KI_SPLIT + s];
                if (!host_count && hc != gpu) bad = true;  // check mode: host and GPU counts agree
                if (host_count || check) {  // the generic enumeration per split (host mode sizes the splits with it)
                    const ItemRows R = item_rows(n, t, G, r);
                    long long sum = 0;
                    uint32_t it0;
                    for (int s = 0; s < KI_SPLIT; ++s) {
                        int lo, hi;
                        ki_split_rows(R.nPL + R.nPR + R.nPM, s, lo, hi);
                        long long cs = 0;
                        for (int x = lo; x < hi; ++x) cs += item_row(hpt, n, t, R, x, G, r, it0, IL_CW);
                        if (host_count) cnt2[(size_t)b * KI_SPLIT + s] = cs;
                        else if (cs != cnt2[(size_t)b * KI_SPLIT + s]) bad = true;
                        sum += cs;
                    }
                    if (sum != hc) bad = true;
                }
            }
        };
        if (host_count || check) {
            const int nth = std::max(1, std::min<int>(8, (int)std::thread::hardware_concurrency()));
            std::vector<std::thread> pool;
            for (int x = 1; x < nth; ++x) pool.emplace_back(worker);
            worker();
            for (auto &th : pool) th.join();
        }
        if (bad) return set_err(cp, CCJ_E_STATE, "k_iloop item count pass disagrees with the enumeration");
        for (int b = 0; b < nb; ++b)
            for (int s = 0; s < KI_SPLIT; ++s) cnt[b] += cnt2[(size_t)b * KI_SPLIT + s];
        c->it_off.assign((size_t)nb + 1, 0);
        for (int x = 0; x < nb; ++x) c->it_off[x + 1] = c->it_off[x] + cnt[x];
        const size_t total = (size_t)c->it_off[nb];
        lap("count");
        if (total > c->items_cap || !c->d_items) {  // ccj_reset: grow only
            if (c->d_items) HIPCHK(cp, hipFree(c->d_items));
            c->d_items = nullptr;
            c->items_cap = std::max<size_t>(total, 1);
            HIPCHK(cp, hipMalloc(&c->d_items, c->items_cap * sizeof(uint32_t)));
        }
        c->T.items = c->d_items;
        // the first item of every split, through pinned staging so the upload is asynchronous on st
        // (the fill's first launches follow it)
        const size_t nsp = (size_t)nb * KI_SPLIT;
        if (!c->h_ioff) HIPCHK(cp, hipHostMalloc(&c->h_ioff, nsp * sizeof(long long), hipHostMallocDefault));
        for (int b = 0; b < nb; ++b) {
            long long o = c->it_off[b];
            for (int s = 0; s < KI_SPLIT; ++s) {
                c->h_ioff[(size_t)b * KI_SPLIT + s] = o;
                o += cnt2[(size_t)b * KI_SPLIT + s];
            }
        }
        HIPCHK(cp, hipMemcpyAsync(c->d_ioff, c->h_ioff, nsp * sizeof(long long), hipMemcpyHostToDevice, c->st));
        HIPCHK(cp, (hipError_t)ccjk_items(&c->T, G, c->rank, c->simulate, c->d_icount, c->d_ioff, c->d_items, 1, c->st));
    }
    HIPCHK(cp, up(c->d_hp, hp.data(), plane * sizeof(int)));
    HIPCHK(cp, up(c->d_est, est.data(), plane * sizeof(int16_t)));
    HIPCHK(cp, up(c->d_S, c->S.data(), (n + 2) * sizeof(short)));
    HIPCHK(cp, up(c->d_S1, c->S1.data(), (n + 2) * sizeof(short)));
    HIPCHK(cp, hipEventRecord(c->ev_stage, c->st));
    lap("upload");
    c->filled = c->mirrored = c->mirrored2d = false;
    return CCJ_OK;
}

static int create_impl(const ccj_problem *prob, const ccj_options *opts, std::unique_ptr<ccj_ctx> &c, ccj_ctx **out) {
    c->seq = prob->seq;
    c->n = (int)c->seq.size();
    c->dangles = prob->dangles;
    c->noGU = prob->noGU ? 1 : 0;
    c->device = opts ? opts->device : 0;
    c->overlap = opts ? (opts->overlap_d2h != 0) : true;
    c->world = (opts && opts->shard_world > 1) ? opts->shard_world : 1;
    c->rank = (opts && c->world > 1) ? opts->shard_rank : 0;
    c->simulate = (opts && c->world > 1) ? (opts->shard_simulate != 0) : 0;
    c->host_tb = opts ? (opts->host_traceback != 0) : false;
    {
        const char *e = getenv("CCJ_SPLIT_TARGET");
        c->split_target = e ? atoi(e) : 9216;
        if (opts && opts->split_target) c->split_target = opts->split_target < 0 ? 0 : opts->split_target;
        const char *lt = getenv("CCJ_LEVEL_TIMING");
        if (lt) c->level_timing = std::max(0, std::min(2, atoi(lt)));
        // k_diag2d(t-1) behind k_iloop(t) on one side stream, so each level waits on one event
        // (fill -0.25 ms at n=200 in 3/3 alternating runs); band-sharded fills with an exchange
        // partition each span instead, and the level-t exchange carries span t
        c->join_diag = !(c->world > 1 && !c->simulate);
        const char *g = getenv("CCJ_SHARE_SPLITS");
        c->share = !(g && atoi(g) < 0) && !(opts && opts->share_splits < 0);
    }
    if (c->rank < 0 || c->rank >= c->world) return CCJ_E_ARG;
    memcpy(&c->prm, prob->params, sizeof(ccj_energy_params));
    if (c->prm.magic != CCJ_PARAMS_MAGIC || c->prm.size_bytes != sizeof(ccj_energy_params))
        return CCJ_E_ARG;
    ccj_pk_penalties pk = CCJ_PK_PENALTIES_DEFAULT;
    if (prob->pen) pk = *prob->pen;
    c->pen = Penalties{pk.PS, pk.PSM, pk.PSP, pk.PB, pk.PUP, pk.PPS, pk.a, pk.b, pk.c, pk.ap, pk.bp, pk.cp};
    c->e_stP = pk.e_stP;
    c->e_intP = pk.e_intP;
    const int n = c->n;
    if (n < 1) return CCJ_E_ARG;
    for (char ch : c->seq)
        if (!(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'U' || ch == 'T')) return CCJ_E_ARG;

    // pair_mat.h:81-155 make_pair_matrix + 159-183 encode_sequence
    const int base_rtype[8] = {0, 2, 1, 4, 3, 6, 5, 7};
    memcpy(c->rtype, base_rtype, sizeof base_rtype);
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) c->pair[x][y] = BP_PAIR[x][y];
    if (c->noGU) c->pair[3][4] = c->pair[4][3] = 0;
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) c->rtype[c->pair[x][y]] = c->pair[y][x];
    // (int)(lxc*log(x/30.)) with the host libm, as ViennaRNA computes it
    c->lx.assign(2 * n + 128, 0);
    for (size_t x = 31; x < c->lx.size(); ++x) c->lx[x] = (int)(c->prm.lxc * log((double)x / 30.));
    c->rs = n + 2;

    // level layout.  d4 stores 11 matrix slots per level, or all 22 (mat5) where the band-sharded
    // exchange packs them or a host mirror streams them during the fill (ccj_engine.h mslot); the
    // host mirror always has 22
    c->mat5 = (c->world > 1 && !c->simulate) || c->overlap || (getenv("CCJ_MAT5") && atoi(getenv("CCJ_MAT5")) != 0);
    c->nm4 = c->mat5 ? NMAT4 : NMAT_ST;
    c->lv_host.assign(std::max(n, 1), LevelDesc{nullptr, 0, 0, 0, 0});
    c->lv_off.assign(std::max(n, 1), 0);
    c->lv_offh.assign(std::max(n, 1), 0);
    int64_t off = 0, cells = 0;
    for (int t = 0; t < n; ++t) {
        const int m = n - t - 2;
        LevelDesc L{nullptr, 0, 0, m > 0 ? m : 0, 0};
        if (m > 0) {
            long long C = 0;
            ccj_level_layout(n, t, c->world, &C, &L.M);
            L.C = (int)C;
            c->nlev = t + 1;
        }
        c->lv_off[t] = off;
        c->lv_offh[t] = (int64_t)NMAT4 * cells;
        c->lv_host[t] = L;
        off += (int64_t)c->nm4 * L.C;
        cells += L.C;
    }
    c->total4 = off;
    c->ncell = cells;
    if ((uint64_t)cells != (uint64_t)ccj_num_cells(n))
        return set_err(c.get(), CCJ_E_ARG, "layout size mismatch");
    // k_ppush addresses the PK rows of PPUSH_S consecutive levels as 32-bit byte offsets from the
    // lowest one's start (one buffer resource per wave): that span must stay below 4 GB
    for (int t = 0; t < c->nlev; ++t) {
        const int tt = std::min(t + PPUSH_S - 1, c->nlev - 1);
        if (2 * (c->lv_off[tt] + (long long)c->lv_host[tt].C - c->lv_off[t]) >= (1LL << 32))
            return set_err(c.get(), CCJ_E_ARG, "n=%d: the PK rows of %d levels exceed 4 GB (k_ppush offsets)", n, PPUSH_S);
    }

    ccj_ctx *cp = c.get();
    HIPCHK(cp, hipSetDevice(c->device));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st_copy, hipStreamNonBlocking));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st_p, hipStreamNonBlocking));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st_il, hipStreamNonBlocking));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st_d, hipStreamNonBlocking));
    HIPCHK(cp, hipStreamCreateWithFlags(&c->st_x, hipStreamNonBlocking));
    // The cross-stream events only order work on this device, so they are recorded without the
    // default system-scope fence (hipEventDisableSystemFence: fill -0.65 ms at n=200).
    // ev_start / ev_end, which the host waits on, keep it.
    constexpr unsigned fence_fl = (unsigned)hipEventDisableSystemFence;
    const unsigned sync_fl = hipEventDisableTiming | fence_fl;
    c->il_done.resize(n + 1);
    for (auto &e : c->il_done) HIPCHK(cp, hipEventCreateWithFlags(&e, sync_fl));
    c->dg_done.resize(n + 1);
    for (auto &e : c->dg_done) HIPCHK(cp, hipEventCreateWithFlags(&e, sync_fl));
    HIPCHK(cp, hipEventCreate(&c->ev_start));
    HIPCHK(cp, hipEventCreate(&c->ev_end));
    HIPCHK(cp, hipEventCreate(&c->ev_pre));
    c->lev_done.resize(n + 1);
    // timed: the level durations (mode 1; recording them untimed measured the same)
    for (auto &e : c->lev_done) HIPCHK(cp, hipEventCreateWithFlags(&e, fence_fl));
    c->p_done.resize(n + 1);
    for (auto &e : c->p_done) HIPCHK(cp, hipEventCreateWithFlags(&e, sync_fl));
    c->pp_done.resize(n + 1);
    for (auto &e : c->pp_done) HIPCHK(cp, hipEventCreateWithFlags(&e, sync_fl));
    c->bulk_done.resize(n + 1);
    for (auto &e : c->bulk_done) HIPCHK(cp, hipEventCreateWithFlags(&e, sync_fl));
    HIPCHK(cp, hipEventCreateWithFlags(&c->ev_bpacked, sync_fl));
    HIPCHK(cp, hipEventCreateWithFlags(&c->ev_bcopied, sync_fl));
    c->tev.resize(TEV_PER * (size_t)n + TEV_PER);
    for (auto &e : c->tev) HIPCHK(cp, hipEventCreate(&e));

    const size_t plane = (size_t)(n + 1) * c->rs;
    const size_t ie_elems = (size_t)(n + 1) * c->rs;  // the u1 = u2 = 0 plane (k_build_il evaluates the rest)
    if (c->total4 > 0 && hipMalloc(&c->d4, (size_t)c->total4 * sizeof(int16_t)) != hipSuccess)
        return set_err(cp, CCJ_E_OOM, "device allocation of %.2f GB for 4-D matrices failed", c->total4 * 2e-9);
    // AoS loop records: NREC 16-byte records per cell (ccj_engine.h)
    c->nrec = c->ncell * NREC;
    if (c->nrec > 0 && (hipMalloc(&c->d_rec, (size_t)c->nrec * sizeof(uint4)) != hipSuccess ||
                        hipMalloc(&c->d_rk, (size_t)c->ncell * sizeof(uint3)) != hipSuccess))
        return set_err(cp, CCJ_E_OOM, "device allocation of %.2f GB for loop records failed",
                       c->nrec * 16e-9 + c->ncell * 12e-9);
    // split-point sharing: the level range it covers (every level of it runs unsplit, so each leader
    // and its followers run one cell per lane) and the partial-record ring
    int g_lo = 0, g_hi = 0;
    long long accC = 0;
    if (c->share) {
        // from the first level that runs unsplit to the last level: the narrow early levels keep
        // their split loops (short scans); on the narrow late levels k_level4d_lead splits the long
        // scans like the level heuristic would (ccjk_level4d_lead).  (Sharing on the unsplit middle
        // levels only measured 0.6 ms slower at n=200.)
        g_lo = -1;
        for (int t = 0; t < c->nlev && g_lo < 0; ++t)
            if (ccjk_level_split(n, t, t + 1, c->split_target) == 1) g_lo = t;
        if (g_lo < 0) {
            g_hi = g_lo < 0 ? 0 : g_lo;
            for (int t = std::max(g_lo, 0); g_lo >= 0 && t < c->nlev; ++t)
                if (ccjk_level_split(n, t, t + 1, c->split_target) == 1 && g_hi == t) g_hi = t + 1;
            if (g_lo < 0) g_lo = 0;
        } else {
            g_hi = c->nlev;
        }
        for (int t = g_lo; t < g_hi; ++t) accC = std::max<long long>(accC, c->lv_host[t].C);
    }
    if (g_hi > g_lo) {
        // the a-blocks k_level4d_lead runs on each sharing level (a leader or a full scan on either
        // side; the roles of level4d_body), ordered by scan cost, longest first, so the longest
        // waves do not start last.  A leader step costs about 2.5 plain steps.  One list per
        // (level t, rank r) at t*world + r: the rank's own blocks (ccj_engine.h shard_owner).
        std::vector<int16_t> lord;
        const int G = c->world;
        c->lord_off.assign((size_t)n * G + 1, 0);
        std::vector<std::pair<double, int>> blk;
        for (int tr = 0; tr < n * G; ++tr) {
            const int t = tr / G, r = tr % G;
            c->lord_off[tr] = (int)lord.size();
            if (t < g_lo || t >= g_hi) continue;
            blk.clear();
            for (int a = 0; a <= t; ++a) {
                if (shard_owner(a, G) != r) continue;
                const int b = t - a, ra = a % SHARE_R, rb = b % SHARE_R;
                const int ar = b >= SHARE_R - 1 ? (ra == 0 ? 1 : (t - ra >= g_lo ? 2 : 0)) : 0;
                const int br = a >= SHARE_R - 1 ? (rb == 0 ? 1 : (t - rb >= g_lo ? 2 : 0)) : 0;
                if (ar == 2 && br == 2) continue;
                const double cost = (ar == 1 ? 2.5 : 1.0) * (ar == 2 ? ra : a) + (br == 1 ? 2.5 : 1.0) * (br == 2 ? rb : b);
                blk.push_back({cost, a});
            }
            std::stable_sort(blk.begin(), blk.end(), [](const auto &x, const auto &y) { return x.first > y.first; });
            for (auto &e : blk) lord.push_back((int16_t)e.second);
        }
        c->lord_off[(size_t)n * G] = (int)lord.size();
        HIPCHK(cp, hipMalloc(&c->d_lord, std::max<size_t>(lord.size(), 1) * sizeof(int16_t)));
        HIPCHK(cp, hipMalloc(&c->d_lord_off, c->lord_off.size() * sizeof(int)));
        if (!lord.empty())
            HIPCHK(cp, hipMemcpy(c->d_lord, lord.data(), lord.size() * sizeof(int16_t), hipMemcpyHostToDevice));
        HIPCHK(cp, hipMemcpy(c->d_lord_off, c->lord_off.data(), c->lord_off.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    if (g_hi > g_lo) {
        if (hipMalloc(&c->d_acc, (size_t)SHARE_SLOTS * SHARE_NACC * accC * sizeof(uint4)) != hipSuccess)
            return set_err(cp, CCJ_E_OOM, "device allocation of %.2f GB for split-sharing records failed",
                           SHARE_SLOTS * SHARE_NACC * accC * 16e-9);
    }
    HIPCHK(cp, hipMalloc(&c->d_ie, ie_elems * sizeof(int16_t)));
    HIPCHK(cp, hipMalloc(&c->d_est, plane * sizeof(int16_t)));
    HIPCHK(cp, hipMalloc(&c->d_hp, plane * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_pt, plane));
    HIPCHK(cp, hipMalloc(&c->d_pair, 64));
    HIPCHK(cp, hipMalloc(&c->d_rtype, 8));
    HIPCHK(cp, hipMalloc(&c->d_lx, c->lx.size() * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_err, sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_S, (n + 2) * sizeof(short)));
    HIPCHK(cp, hipMalloc(&c->d_S1, (n + 2) * sizeof(short)));
    HIPCHK(cp, hipMalloc(&c->d_prm, sizeof(ccj_energy_params)));
    HIPCHK(cp, hipMalloc(&c->d_lv, c->lv_host.size() * sizeof(LevelDesc)));
    HIPCHK(cp, hipMalloc(&c->d_lb, c->lv_off.size() * sizeof(long long)));
    HIPCHK(cp, hipMalloc(&c->d_ld, c->lv_off.size() * sizeof(LvlDev)));
    {
        // interior-loop copies (ccj_engine.h): PLx+PRx mirror the level sizes, PMx is padded per (h, j).
        // In front of every level: xpad sentinel elements of 32767, the null target of k_iloop's
        // waves (a wave addresses its source levels as 32-bit offsets from the pad of the lowest)
        const long long xpad = n + 256;
        std::vector<LvlX> ldx(c->lv_off.size(), LvlX{0, 0});
        long long ox = 0, op = 0, span = 0;
        for (int t = 0; t < c->nlev; ++t) {
            ox += xpad;
            op += xpad;
            ldx[t] = LvlX{ox, op};
            ox += 2LL * c->lv_host[t].C;
            op += (long long)c->lv_host[t].m * n * (t + 1);
            const int tlo = std::max(0, t - (2 * MAXLOOP - 2));  // a wave of level t + 3 .. t + 58 reads down to tlo
            span = std::max({span, 2 * (ox - (ldx[tlo].lbx - xpad)), 2 * (op - (ldx[tlo].pmb - xpad))});
        }
        if (span >= (1LL << 32) - 4096)
            return set_err(cp, CCJ_E_ARG, "n=%d: the interior-loop copies of 56 levels exceed 4 GB (k_iloop offsets)", n);
        const size_t pad = 256;
        c->nx = ox;
        c->npm = op;
        c->xpad = xpad;
        c->xspan = span;
        // pad elements on both sides; everything starts as 32767 (the pads stay so: no level writes them)
        if (hipMalloc(&c->d4x_alloc, ((size_t)ox + 2 * pad) * sizeof(int16_t)) != hipSuccess ||
            hipMalloc(&c->pmx_alloc, ((size_t)op + 2 * pad) * sizeof(int16_t)) != hipSuccess)
            return set_err(cp, CCJ_E_OOM, "device allocation of %.2f GB for interior-loop copies failed", (ox + op) * 2e-9);
        HIPCHK(cp, hipMemsetD16((hipDeviceptr_t)c->d4x_alloc, (unsigned short)INTERN_INF, (size_t)ox + 2 * pad));
        HIPCHK(cp, hipMemsetD16((hipDeviceptr_t)c->pmx_alloc, (unsigned short)INTERN_INF, (size_t)op + 2 * pad));
        c->d4x = c->d4x_alloc + pad;
        c->pmx = c->pmx_alloc + pad;
        HIPCHK(cp, hipMalloc(&c->d_ldx, ldx.size() * sizeof(LvlX)));
        HIPCHK(cp, hipMemcpy(c->d_ldx, ldx.data(), ldx.size() * sizeof(LvlX), hipMemcpyHostToDevice));
        std::vector<int16_t> dummy((size_t)n + 64, (int16_t)INTERN_INF);
        HIPCHK(cp, hipMalloc(&c->d_dummy, dummy.size() * sizeof(int16_t)));
        HIPCHK(cp, hipMemcpy(c->d_dummy, dummy.data(), dummy.size() * sizeof(int16_t), hipMemcpyHostToDevice));
        {  // the k_iloop work items' candidate lists (k_build_il)
            const size_t pairs = (size_t)(n + 1) * c->rs;
            const size_t ents = pairs * IL_CAP;
            HIPCHK(cp, hipMalloc(&c->d_il, ents * sizeof(uint2)));
            HIPCHK(cp, hipMalloc(&c->d_ilm, ents * sizeof(uint2)));
            HIPCHK(cp, hipMalloc(&c->d_ilseg, pairs * IL_SEG * sizeof(uint32_t)));
            HIPCHK(cp, hipMalloc(&c->d_ilmseg, pairs * IL_SEG * sizeof(uint32_t)));
            HIPCHK(cp, hipMemset(c->d_ilseg, 0, pairs * IL_SEG * sizeof(uint32_t)));
            HIPCHK(cp, hipMemset(c->d_ilmseg, 0, pairs * IL_SEG * sizeof(uint32_t)));
        }
    }
    HIPCHK(cp, hipMalloc(&c->d2i, A2_N * plane * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_wbw, plane * sizeof(int2)));
    HIPCHK(cp, hipMalloc(&c->d_pk, plane * sizeof(unsigned long long)));
    HIPCHK(cp, hipMalloc(&c->d_W, (n + 1) * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_wterm, plane * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_fpair, (n + 1) * sizeof(int)));
    HIPCHK(cp, hipMalloc(&c->d_ftype, (n + 1)));
    HIPCHK(cp, hipMalloc(&c->d_btout, sizeof(BtOut)));
    HIPCHK(cp, hipMalloc(&c->d_vt, plane));
    // the pinned host mirror is only needed by the host traceback and the getters: allocate it up
    // front when the fill streams into it, else on first use (ccj_sync_host)
    if (c->overlap && c->total4 > 0 &&
        hipHostMalloc(&c->h4, (size_t)NMAT4 * c->ncell * sizeof(int16_t), hipHostMallocDefault) != hipSuccess)
        return set_err(cp, CCJ_E_OOM, "pinned host allocation of %.2f GB failed", NMAT4 * c->ncell * 2e-9);
    c->h2i.assign(A2_N * plane, 0);
    c->hvt.assign(plane, 0);

    for (int t = 0; t < n; ++t) c->lv_host[t].base = c->d4 ? c->d4 + c->lv_off[t] : nullptr;

    int8_t pair8[64], rt8[8];
    for (int x = 0; x < 8; ++x) {
        rt8[x] = (int8_t)c->rtype[x];
        for (int y = 0; y < 8; ++y) pair8[x * 8 + y] = (int8_t)c->pair[x][y];
    }
    HIPCHK(cp, hipMemcpy(c->d_pair, pair8, 64, hipMemcpyHostToDevice));
    HIPCHK(cp, hipMemcpy(c->d_rtype, rt8, 8, hipMemcpyHostToDevice));
    HIPCHK(cp, hipMemcpy(c->d_lx, c->lx.data(), c->lx.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(cp, hipMemcpy(c->d_prm, &c->prm, sizeof(ccj_energy_params), hipMemcpyHostToDevice));
    HIPCHK(cp, hipMemcpy(c->d_lv, c->lv_host.data(), c->lv_host.size() * sizeof(LevelDesc), hipMemcpyHostToDevice));
    {
        std::vector<long long> lb(c->lv_off.begin(), c->lv_off.end());
        HIPCHK(cp, hipMemcpy(c->d_lb, lb.data(), lb.size() * sizeof(long long), hipMemcpyHostToDevice));
        std::vector<LvlDev> ld(c->lv_off.size());
        long long lr = 0;
        for (size_t t = 0; t < ld.size(); ++t) {
            ld[t] = LvlDev{c->lv_off[t], lr, c->lv_host[t].C, c->lv_host[t].M, {0, 0}};
            lr += (long long)NREC * c->lv_host[t].C;
        }
        HIPCHK(cp, hipMemcpy(c->d_ld, ld.data(), ld.size() * sizeof(LvlDev), hipMemcpyHostToDevice));
    }

    DevTables &T = c->T;
    T.n = n;
    T.nlev = c->nlev;
    T.rs = c->rs;
    T.dangles = c->dangles;
    T.pen = c->pen;
    T.e_stP = c->e_stP;
    T.e_intP = c->e_intP;
    T.prm = c->d_prm;
    T.lx = c->d_lx;
    T.S = c->d_S;
    T.S1 = c->d_S1;
    T.pt = c->d_pt;
    T.pair = c->d_pair;
    T.rtype = c->d_rtype;
    T.hp = c->d_hp;
    T.est = c->d_est;
    T.ie = c->d_ie;
    T.V = c->d2i + A2_V * plane;
    T.WM = c->d2i + A2_WM * plane;
    T.WMv = c->d2i + A2_WMV * plane;
    T.WMp = c->d2i + A2_WMP * plane;
    T.P = c->d2i + A2_P * plane;
    T.Pk = c->d_pk;
    T.WBP = c->d2i + A2_WBP * plane;
    T.WPP = c->d2i + A2_WPP * plane;
    T.WB = c->d2i + A2_WB * plane;
    T.WP = c->d2i + A2_WP * plane;
    T.WBW = c->d_wbw;
    T.Vt = c->d_vt;
    T.lv = c->d_lv;
    T.d4 = c->d4;
    T.lb = c->d_lb;
    T.ld = c->d_ld;
    T.d4x = c->d4x;
    T.rec = c->d_rec;
    T.rk = c->d_rk;
    T.nrec = c->nrec;
    T.pmx = c->pmx;
    T.nx = c->nx;
    T.npm = c->npm;
    T.xpad = c->xpad;
    T.xspan = c->xspan;
    T.ldx = c->d_ldx;
    T.il = c->d_il;
    T.ilm = c->d_ilm;
    T.dummy = c->d_dummy;
    T.items = c->d_items;
    // the exchange packs all 22 matrices from d4, a mirror streamed during the fill copies them;
    // CCJ_MAT5=1 stores them in every fill (A/B timing)
    T.mat5 = c->mat5 ? 1 : 0;
    T.ilseg = c->d_ilseg;
    T.ilmseg = c->d_ilmseg;
    T.err = c->d_err;
    T.split_target = c->split_target;
    T.g_lo = g_lo;
    T.g_hi = g_hi;
    T.acc = c->d_acc;
    T.lord = c->d_lord;
    T.lord_off = c->d_lord_off;
    T.lord_off_h = c->lord_off.empty() ? nullptr : c->lord_off.data();
    T.accC = accC;
    {
        const int G = c->world;
        HIPCHK(cp, hipMalloc(&c->d_icount, (size_t)n * G * KI_SPLIT * sizeof(long long)));
        HIPCHK(cp, hipMalloc(&c->d_ioff, (size_t)n * G * KI_SPLIT * sizeof(long long)));
        if (G > 1 && !c->simulate) {
            // exchange slices, per part: 22 matrices x the largest rank's blocks of the
            // part x M, then the part's tail
            for (int part = 0; part < 2; ++part) {
                c->xnmax[part].assign(n, 0);
                size_t slice = 0;
                for (int t = 0; t < c->nlev; ++t) {
                    const int nm = xch_nmax(t, G, part);
                    c->xnmax[part][t] = nm;
                    slice = std::max(slice, (size_t)xch_slice(n, nm, c->lv_host[t].M, part));
                }
                if (hipMalloc(&c->d_send[part], std::max<size_t>(slice, 1) * sizeof(int16_t)) != hipSuccess ||
                    hipMalloc(&c->d_recv[part], std::max<size_t>(slice * G, 1) * sizeof(int16_t)) != hipSuccess)
                    return set_err(cp, CCJ_E_OOM, "device allocation of the exchange buffers (%.2f GB) failed",
                                   slice * (G + 1) * 2e-9);
            }
        }
    }
    if (const int rc = seq_setup(cp)) return rc;
    *out = c.release();
    return CCJ_OK;
}

extern "C" int ccj_create(const ccj_problem *prob, const ccj_options *opts, ccj_ctx **out) {
    if (!out) return CCJ_E_ARG;
    *out = nullptr;
    g_create_err.clear();
    if (!prob || !prob->seq || !prob->params) {
        g_create_err = "null problem / sequence / params";
        return CCJ_E_ARG;
    }
    std::unique_ptr<ccj_ctx> c(new ccj_ctx());
    const int rc = create_impl(prob, opts, c, out);
    if (rc != CCJ_OK) {
        g_create_err = c ? c->err : std::string("ccj_create failed");
        if (g_create_err.empty()) g_create_err = "invalid problem (sequence alphabet, length or parameter blob)";
        if (c) ccj_destroy(c.release());
    }
    return rc;
}

extern "C" int ccj_reset(ccj_ctx *c, const char *seq) {
    if (!c || !seq) return CCJ_E_ARG;
    const std::string s(seq);
    if ((int)s.size() != c->n) return set_err(c, CCJ_E_ARG, "ccj_reset: length %zu differs from the context's n=%d", s.size(), c->n);
    for (char ch : s)
        if (!(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'U' || ch == 'T'))
            return set_err(c, CCJ_E_ARG, "ccj_reset: invalid character in sequence");
    if (c->pending || c->res_pending) return set_err(c, CCJ_E_STATE, "ccj_reset: a fold is in flight (ccj_wait first)");
    HIPCHK(c, hipSetDevice(c->device));
    // no fold is in flight (checked above): ccj_wait / ccj_fill returned only after the fill and
    // the traceback completed, so the streams are idle.  Only the optional host-mirror copies can
    // still run.  (A hipStreamSynchronize here would enqueue a marker that can wait behind another
    // context's fill on a shared hardware queue.)
    if (c->overlap && c->h4) HIPCHK(c, hipStreamSynchronize(c->st_copy));
    c->seq = s;
    c->W.clear();
    return seq_setup(c);
}

// Enqueue the whole fill on the context's streams; it ends with ev_end on st, after which every
// stream's work of the fill is complete (st waits for the last span, which waits for the last P,
// and every level waited for its k_iloop / leader launches).
// The P terms that complete P(lev+3): every term whose operands' highest level is lev (k_ppush,
// DESIGN.md §4).  Band-sharded, each rank pushes its share (outer index r, r+G, ...; every share in
// simulation) and the spans are min-combined in the exchange of level lev+1.
static int pterm_launch(const ccj_ctx *c, int lev, hipStream_t s) {
    for (int r = 0; r < c->world; ++r) {
        if (!c->simulate && r != c->rank) continue;
        if (const int e = ccjk_ppush(&c->T, lev, c->world, r, s)) return e;
    }
    return 0;
}

static int fill_enqueue(ccj_ctx *c, const ccj_ctx *after = nullptr) {
    if (!c) return CCJ_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int n = c->n;
    hipStream_t st = c->st;
    // pipelining (ccj_fill_async_after): start when the other context's last enqueued fill has
    // ended (its ev_end; its W + traceback may still run beside this fill)
    if (after && after != c && after->ev_end) HIPCHK(c, hipStreamWaitEvent(st, after->ev_end, 0));
    const auto enq0 = std::chrono::steady_clock::now();
    c->filled = c->mirrored = c->mirrored2d = false;
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(int), st));
    HIPCHK(c, hipEventRecord(c->ev_start, st));
    HIPCHK(c, (hipError_t)ccjk_init2d(&c->T, st));
    HIPCHK(c, (hipError_t)ccjk_precompute_ie(&c->T, st));
    HIPCHK(c, (hipError_t)ccjk_build_il(&c->T, st));
    HIPCHK(c, hipEventRecord(c->ev_pre, st));
    // Four streams:
    //   st_d : k_diag2d(s)  needs P(s) (p_done) and spans < s (stream order)
    //   st_il: k_iloop(t)   needs 4-D levels <= t-3 (lev_done[t-3]; the dt = 2 term is in k_level4d)
    //   st   : k_level4d(t) needs level t-1 (stream order), k_iloop(t), k_diag2d(t-1)
    //   st_p : k_pterm(s)   needs PK levels <= s-3 (lev_done[s-3])
    // so k_diag2d(t) and k_iloop(t+1) overlap k_level4d(t).  Every event is recorded (enqueued)
    // before a stream waits on it.
    HIPCHK(c, hipStreamWaitEvent(c->st_d, c->ev_pre, 0));
    HIPCHK(c, hipStreamWaitEvent(c->st_il, c->ev_pre, 0));
    HIPCHK(c, hipStreamWaitEvent(c->st_p, c->ev_pre, 0));
    const bool xchg = c->world > 1 && !c->simulate;
    // level t complete on this rank: its lev_done, or, band-sharded, when the bulk part of its
    // exchange is unpacked (bulk_done[t]; lev_done[t] then only covers the rank's own cells and the
    // other ranks' edge blocks, which is all level t+1 reads of level t)
    const std::vector<hipEvent_t> &lvl_full = xchg ? c->bulk_done : c->lev_done;
    // what follows a level's completion on this rank: P terms pushed by it, the host-mirror copy
    auto after_level = [&](int s) -> int {
        if (c->overlap && c->h4) {
            // stream the finished level to the pinned host mirror while later levels run
            HIPCHK(c, hipStreamWaitEvent(c->st_copy, lvl_full[s], 0));
            const size_t bytes = (size_t)NMAT4 * c->lv_host[s].C * sizeof(int16_t);
            HIPCHK(c, hipMemcpyAsync(c->h4 + c->lv_offh[s], c->d4 + c->lv_off[s], bytes, hipMemcpyDeviceToHost, c->st_copy));
        }
        // P(s+3) only needs PK levels <= s; band-sharded, this rank's partials are combined in the
        // bulk exchange of level s+1, which then records p_done[s+3]
        if (s + 3 < n) {
            hipEvent_t *ev = &c->tev[TEV_PER * (size_t)s];
            HIPCHK(c, hipStreamWaitEvent(c->st_p, lvl_full[s], 0));
            if (c->level_timing == 2) HIPCHK(c, hipEventRecord(ev[7], c->st_p));
            HIPCHK(c, (hipError_t)pterm_launch(c, s, c->st_p));
            if (c->level_timing == 2) HIPCHK(c, hipEventRecord(ev[8], c->st_p));
            HIPCHK(c, hipEventRecord((xchg ? c->pp_done : c->p_done)[s + 3], c->st_p));
        }
        return CCJ_OK;
    };
    // Band-sharded exchange of level s, part `part` (ccj_engine.h XCH_EDGE / XCH_BULK):
    // pack the rank's blocks of the part (+ the part's tail), gather, unpack.  The edge part runs on the
    // level stream; the bulk part on st_x, split into its start (wait, pack; over RCCL also gather and
    // unpack) and, for the in-process group, its finish one level later (the host-side gather), so
    // that the host thread does not block on it before the next level is enqueued.
    auto part_slice = [&](int s, int part) { return (size_t)xch_slice(n, c->xnmax[part][s], c->lv_host[s].M, part); };
    auto part_body = [&](int s, int part) { return (size_t)xch_body(c->xnmax[part][s], c->lv_host[s].M); };
    auto gather = [&](int s, int part, hipStream_t q) -> int {
        if (c->lgroup) return local_allgather(c, part, part_slice(s, part), q);
        ncclComm_t cm = part == XCH_EDGE ? c->comm : c->comm_b;
        if (!cm) return set_err(c, CCJ_E_STATE, "sharded context without ccj_comm_init");
        if (ncclAllGather(c->d_send[part], c->d_recv[part], part_slice(s, part) * sizeof(int16_t), ncclInt8, cm, q) != ncclSuccess)
            return set_err(c, CCJ_E_COMM, "ncclAllGather (%s) failed at level %d", part == XCH_EDGE ? "edge" : "bulk", s);
        return CCJ_OK;
    };
    auto bulk_unpack = [&](int s) -> int {
        hipEvent_t *ev = &c->tev[TEV_PER * (size_t)s];
        HIPCHK(c, (hipError_t)ccjk_unpack(&c->T, s, c->world, c->rank, XCH_BULK, c->xnmax[XCH_BULK][s], c->d_recv[XCH_BULK],
                                          part_slice(s, XCH_BULK), c->st_x));
        if (c->level_timing == 2) HIPCHK(c, hipEventRecord(ev[10], c->st_x));
        HIPCHK(c, hipEventRecord(c->bulk_done[s], c->st_x));
        return CCJ_OK;
    };
    auto bulk_start = [&](int s) -> int {
        hipEvent_t *ev = &c->tev[TEV_PER * (size_t)s];
        HIPCHK(c, hipStreamWaitEvent(c->st_x, c->lev_done[s], 0));
        if (c->lgroup) {
            if (const int rc = local_bulk_wait_copied(c)) return rc;
        }
        if (c->level_timing == 2) HIPCHK(c, hipEventRecord(ev[9], c->st_x));
        HIPCHK(c, (hipError_t)ccjk_pack(&c->T, s, c->world, c->rank, XCH_BULK, c->xnmax[XCH_BULK][s], c->d_send[XCH_BULK], c->st_x));
        if (c->lgroup) {  // gathered and unpacked when the next level is enqueued (bulk_finish)
            HIPCHK(c, hipEventRecord(c->ev_bpacked, c->st_x));
            return CCJ_OK;
        }
        if (const int rc = gather(s, XCH_BULK, c->st_x)) return rc;
        return bulk_unpack(s);
    };
    // the in-process group's bulk gather of level s, then what waits for level s to be complete
    auto bulk_finish = [&](int s) -> int {
        if (c->lgroup) {
            if (const int rc = local_bulk_gather(c, part_slice(s, XCH_BULK))) return rc;
            if (const int rc = bulk_unpack(s)) return rc;
        }
        return after_level(s);
    };
    for (int s = 0; s < n; ++s) {
        hipEvent_t *ev = &c->tev[TEV_PER * (size_t)s];
        // timing markers (ev[0..10]) only when per-kernel timing is on
        auto trec = [&](int x, hipStream_t q) { return c->level_timing == 2 ? hipEventRecord(ev[x], q) : hipSuccess; };
        // k_diag2d(sigma) on st_d; or, joined (c->join_diag), on st_il right after k_iloop(sigma+1),
        // so that level sigma+1 waits on one event that covers both
        auto enqueue_diag = [&](int sg, hipStream_t q) -> int {
            hipEvent_t *evd = &c->tev[TEV_PER * (size_t)sg];
            if (sg >= 3) HIPCHK(c, hipStreamWaitEvent(q, c->p_done[sg], 0));
            // band-sharded: span sg-1 is complete on this rank only after the level-(sg-1) edge
            // exchange, which carries it
            if (xchg && sg >= 1 && sg - 1 < c->nlev) HIPCHK(c, hipStreamWaitEvent(q, c->lev_done[sg - 1], 0));
            if (c->level_timing == 2) HIPCHK(c, hipEventRecord(evd[0], q));
            if (c->simulate) {  // every rank's share of the span, in one context
                for (int r = 0; r < c->world; ++r) HIPCHK(c, (hipError_t)ccjk_diag2d(&c->T, sg, c->world, r, q));
            } else if (xchg && sg < c->nlev) {  // this rank's intervals; the exchange of level sg brings the rest
                HIPCHK(c, (hipError_t)ccjk_diag2d(&c->T, sg, c->world, c->rank, q));
            } else {  // unsharded, or the spans past the last 4-D level (no exchange left): every interval
                HIPCHK(c, (hipError_t)ccjk_diag2d(&c->T, sg, 1, 0, q));
            }
            if (c->level_timing == 2) HIPCHK(c, hipEventRecord(evd[1], q));
            HIPCHK(c, hipEventRecord(c->dg_done[sg], q));
            return CCJ_OK;
        };
        const bool joined = c->join_diag && s >= 1 && s < c->nlev;  // diag(s-1) follows iloop(s)
        if (!c->join_diag || s >= c->nlev) {
            if (c->join_diag && s == c->nlev && s >= 1 && s - 1 < c->nlev) {
                if (const int rc = enqueue_diag(s - 1, c->st_il)) return rc;  // last one behind iloop
            }
            if (const int rc = enqueue_diag(s, c->join_diag ? c->st_il : c->st_d)) return rc;
        }
        if (s < c->nlev) {
            // k_iloop(s) reads levels <= s-3 (complete: band-sharded, their bulk parts unpacked)
            if (s >= 3) HIPCHK(c, hipStreamWaitEvent(c->st_il, lvl_full[s - 3], 0));
            HIPCHK(c, trec(2, c->st_il));
            const int G = c->world;
            for (int r = 0; r < G; ++r) {  // every rank's launches in simulation, else this rank's
                if (!c->simulate && r != c->rank) continue;
                const size_t tr = (size_t)s * G + r;
                HIPCHK(c, (hipError_t)ccjk_iloop(&c->T, s, c->it_off[tr], (int)(c->it_off[tr + 1] - c->it_off[tr]), G, r,
                                                 c->st_il));
            }
            HIPCHK(c, trec(3, c->st_il));
            if (joined) {
                if (const int rc = enqueue_diag(s - 1, c->st_il)) return rc;
            }
            HIPCHK(c, hipEventRecord(c->il_done[s], c->st_il));
            HIPCHK(c, hipStreamWaitEvent(st, c->il_done[s], 0));
            if (s >= 1 && !c->join_diag) HIPCHK(c, hipStreamWaitEvent(st, c->dg_done[s - 1], 0));
            // band-sharded: level s reads the other ranks' blocks of level s-2 from its bulk part (the
            // edge part of level s-1 arrived on this stream; older levels precede s-2 on st_x)
            if (xchg && s >= 2) HIPCHK(c, hipStreamWaitEvent(st, c->bulk_done[s - 2], 0));
            HIPCHK(c, trec(4, st));
            // the level: its plain launch, then (sharing levels) the leaders on the same stream, no
            // cross-stream hop between the two launches or between levels
            for (int r = 0; r < G; ++r) {
                if (!c->simulate && r != c->rank) continue;
                HIPCHK(c, (hipError_t)ccjk_level4d(&c->T, s, G, r, 1, st));
            }
            for (int r = 0; r < G; ++r) {
                if (!c->simulate && r != c->rank) continue;
                HIPCHK(c, (hipError_t)ccjk_level4d_lead(&c->T, s, G, r, st));
            }
            if (xchg) {
                // the previous level's bulk part (in-process: its gather), the P terms it completes
                if (s >= 1) {
                    if (const int rc = bulk_finish(s - 1)) return rc;
                }
                HIPCHK(c, trec(6, st));  // timing mode 2: the edge exchange's share of the level span
                // edge part: the rank's blocks a % 4 == 3 (all 22 matrices), its partials of P(s+1)
                // (pushed after level s-2, so a level of slack) and its intervals of span s
                const size_t body = part_body(s, XCH_EDGE), dt_off = body + (size_t)xch_ptail(n);
                const int sig = s + 1;
                const bool ptail = sig >= 3 && sig <= n - 2;
                if (ptail) {
                    HIPCHK(c, hipStreamWaitEvent(st, c->pp_done[sig], 0));
                    HIPCHK(c, (hipError_t)ccjk_ptail_pack(&c->T, sig, c->d_send[XCH_EDGE] + body, st));
                }
                HIPCHK(c, hipStreamWaitEvent(st, c->dg_done[s], 0));
                HIPCHK(c, (hipError_t)ccjk_dtail_pack(&c->T, s, G, c->rank, c->d_send[XCH_EDGE] + dt_off, st));
                HIPCHK(c, (hipError_t)ccjk_pack(&c->T, s, G, c->rank, XCH_EDGE, c->xnmax[XCH_EDGE][s], c->d_send[XCH_EDGE], st));
                if (const int rc = gather(s, XCH_EDGE, st)) return rc;
                HIPCHK(c, (hipError_t)ccjk_unpack(&c->T, s, G, c->rank, XCH_EDGE, c->xnmax[XCH_EDGE][s], c->d_recv[XCH_EDGE],
                                                  part_slice(s, XCH_EDGE), st));
                HIPCHK(c, (hipError_t)ccjk_dtail_unpack(&c->T, s, c->d_recv[XCH_EDGE], part_slice(s, XCH_EDGE), dt_off, G, c->rank,
                                                        st));
                if (ptail) {
                    HIPCHK(c, (hipError_t)ccjk_ptail_unpack(&c->T, sig, c->d_recv[XCH_EDGE], part_slice(s, XCH_EDGE), body, G, st));
                    HIPCHK(c, hipEventRecord(c->p_done[sig], st));  // P(sig) final on every rank
                }
            }
            HIPCHK(c, trec(5, st));
            HIPCHK(c, hipEventRecord(c->lev_done[s], st));
            if (xchg) {
                if (const int rc = bulk_start(s)) return rc;
            } else if (const int rc = after_level(s)) {
                return rc;
            }
        } else {
            if (xchg && s == c->nlev && s >= 1) {  // the last level's bulk part
                if (const int rc = bulk_finish(s - 1)) return rc;
            }
            if (xchg && s == c->nlev && n - 1 >= 3) {
                // the partials of P(n-1) (pushed after level n-4): no level n-2 carries them, so they
                // travel alone, as a slice of one P tail in the edge buffers
                const int sig = n - 1;
                const size_t pslice = (size_t)xch_ptail(n);
                HIPCHK(c, hipStreamWaitEvent(st, c->pp_done[sig], 0));
                HIPCHK(c, (hipError_t)ccjk_ptail_pack(&c->T, sig, c->d_send[XCH_EDGE], st));
                if (c->lgroup) {
                    if (const int rc = local_allgather(c, XCH_EDGE, pslice, st)) return rc;
                } else {
                    if (!c->comm) return set_err(c, CCJ_E_STATE, "sharded context without ccj_comm_init");
                    if (ncclAllGather(c->d_send[XCH_EDGE], c->d_recv[XCH_EDGE], pslice * sizeof(int16_t), ncclInt8, c->comm, st) !=
                        ncclSuccess)
                        return set_err(c, CCJ_E_COMM, "ncclAllGather (P tail) failed");
                }
                HIPCHK(c, (hipError_t)ccjk_ptail_unpack(&c->T, sig, c->d_recv[XCH_EDGE], pslice, 0, c->world, st));
                HIPCHK(c, hipEventRecord(c->p_done[sig], st));
            }
            if (s + 3 < n && s + 3 >= 3) {
                HIPCHK(c, (hipError_t)pterm_launch(c, s, c->st_p));
                HIPCHK(c, hipEventRecord(c->p_done[s + 3], c->st_p));
            }
        }
    }
    if (getenv("CCJ_TRACE_ENQUEUE"))
        fprintf(stderr, "ccj_fill_device: enqueue %.2f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - enq0).count());
    // join: the fill ends when the last level (every rank's part of it) and the last span are done
    HIPCHK(c, hipStreamWaitEvent(st, c->dg_done[n - 1], 0));
    if (xchg && c->nlev >= 1) HIPCHK(c, hipStreamWaitEvent(st, c->bulk_done[c->nlev - 1], 0));
    HIPCHK(c, hipEventRecord(c->ev_end, st));
    c->pending = true;
    return CCJ_OK;
}

// Wait for the fill's end event.  A band-sharded fill over RCCL cannot finish if a peer rank died
// or hangs (its all-gathers never complete): the wait polls the communicator's asynchronous error
// state and a deadline (CCJ_COMM_TIMEOUT_S, default 300 s) and, on either, aborts the communicator
// (ncclCommAbort makes the pending collectives return) and fails with CCJ_E_COMM instead of hanging.
static int wait_fill_end(ccj_ctx *c) {
    if (!c->comm) {
        HIPCHK(c, hipEventSynchronize(c->ev_end));
        return CCJ_OK;
    }
    static const double limit_s = [] {
        const char *e = getenv("CCJ_COMM_TIMEOUT_S");
        return e && atof(e) > 0 ? atof(e) : 300.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(c->ev_end);
        if (q == hipSuccess) return CCJ_OK;
        if (q != hipErrorNotReady) return set_err(c, CCJ_E_HIP, "fill: %s", hipGetErrorString(q));
        ncclResult_t ae = ncclSuccess, ae2 = ncclSuccess;
        ncclResult_t qr = ncclCommGetAsyncError(c->comm, &ae);
        if (qr == ncclSuccess && ae == ncclSuccess && c->comm_b) {  // the bulk communicator too
            qr = ncclCommGetAsyncError(c->comm_b, &ae2);
            ae = ae2;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (qr != ncclSuccess || ae != ncclSuccess || el > limit_s) {
            if (c->comm_b) ncclCommAbort(c->comm_b);
            ncclCommAbort(c->comm);
            c->comm = c->comm_b = nullptr;
            if (qr != ncclSuccess || ae != ncclSuccess)
                return set_err(c, CCJ_E_COMM, "band-sharded exchange failed: %s",
                               ncclGetErrorString(qr != ncclSuccess ? qr : ae));
            return set_err(c, CCJ_E_COMM, "band-sharded exchange made no progress for %.0f s (a peer rank failed?)", limit_s);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// Wait for an enqueued fill, check the device error word and read its timings.
static int fill_finish(ccj_ctx *c) {
    if (!c || !c->pending) return c ? set_err(c, CCJ_E_STATE, "no fill in flight") : CCJ_E_ARG;
    c->pending = false;
    HIPCHK(c, hipSetDevice(c->device));
    const int n = c->n;
    if (const int rc = wait_fill_end(c)) return rc;
    int herr = 0;
    HIPCHK(c, hipMemcpy(&herr, c->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (herr & 1) return set_err(c, CCJ_E_PARAMS, "e_intP table value outside int16 range (flags %d)", herr);
    if (herr) return set_err(c, CCJ_E_HIP, "device bounds check failed (flags %d)", herr);
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_start, c->ev_end));
    c->fill_ms = ms;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_start, c->ev_pre));
    c->pre_ms = ms;
    double lsum = 0, dsum = 0, isum = 0;
    c->lev_ms_v.assign(n, 0.0);
    c->diag_ms_v.assign(n, 0.0);
    c->il_ms_v.assign(n, 0.0);
    c->xch_ms_v.assign(n, 0.0);
    c->xbulk_ms_v.assign(n, 0.0);
    c->pp_ms_v.assign(n, 0.0);
    double psum = 0;
    if (c->level_timing == 1) {
        // level s = from the end of level s-1 (ev_pre for s = 0) to its lev_done on st: the waits for
        // k_iloop(s) / k_diag2d(s-1), the plain launch and the leaders
        for (int s = 0; s < c->nlev && s < n; ++s) {
            HIPCHK(c, hipEventElapsedTime(&ms, s == 0 ? c->ev_pre : c->lev_done[s - 1], c->lev_done[s]));
            lsum += ms;
            c->lev_ms_v[s] = ms;
        }
    }
    for (int s = 0; s < n && c->level_timing == 2; ++s) {
        const hipEvent_t *ev = &c->tev[TEV_PER * (size_t)s];
        HIPCHK(c, hipEventElapsedTime(&ms, ev[0], ev[1]));
        dsum += ms;
        c->diag_ms_v[s] = ms;
        if (s < c->nlev) {
            HIPCHK(c, hipEventElapsedTime(&ms, ev[2], ev[3]));
            isum += ms;
            c->il_ms_v[s] = ms;
            // the level's span: from its first launch to its last (exchange included when sharded)
            HIPCHK(c, hipEventElapsedTime(&ms, ev[4], ev[5]));
            lsum += ms;
            c->lev_ms_v[s] = ms;
            if (s + 3 < n) {  // k_ppush(s) on st_p
                HIPCHK(c, hipEventElapsedTime(&ms, ev[7], ev[8]));
                psum += ms;
                c->pp_ms_v[s] = ms;
            }
            if (c->world > 1 && !c->simulate) {
                // the edge part on the level stream: waits for span s, packs, all-gather, unpacks
                HIPCHK(c, hipEventElapsedTime(&ms, ev[6], ev[5]));
                c->xch_ms_v[s] = ms;
                // the bulk part on st_x: from its start (after the level) to its unpack
                HIPCHK(c, hipEventElapsedTime(&ms, ev[9], ev[10]));
                c->xbulk_ms_v[s] = ms;
            }
        }
    }
    c->level_ms = lsum;
    c->diag_ms = dsum;
    c->il_ms = isum;
    c->pp_ms = psum;
    c->filled = true;
    return CCJ_OK;
}

extern "C" int ccj_fill_device(ccj_ctx *c) {
    if (!c) return CCJ_E_ARG;
    if (c->pending || c->res_pending) return set_err(c, CCJ_E_STATE, "ccj_fill_device: a fold is in flight (ccj_wait first)");
    if (const int rc = fill_enqueue(c)) return rc;
    return fill_finish(c);
}

extern "C" int ccj_sync_host(ccj_ctx *c) {
    if (!c || !c->filled) return CCJ_E_STATE;
    const auto t0 = std::chrono::steady_clock::now();
    struct Rec {
        ccj_ctx *c;
        std::chrono::steady_clock::time_point t0;
        ~Rec() { c->sync_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } rec{c, t0};
    HIPCHK(c, hipSetDevice(c->device));
    const size_t plane = (size_t)(c->n + 1) * c->rs;
    if (c->overlap && c->h4) {
        HIPCHK(c, hipStreamSynchronize(c->st_copy));
    } else if (c->total4 > 0) {
        const size_t hbytes = (size_t)NMAT4 * c->ncell * sizeof(int16_t);
        if (!c->h4 && hipHostMalloc(&c->h4, hbytes, hipHostMallocDefault) != hipSuccess)
            return set_err(c, CCJ_E_OOM, "pinned host allocation of %.2f GB failed", hbytes * 1e-9);
        if (c->mat5) {  // d4 has the mirror's layout
            HIPCHK(c, hipMemcpy(c->h4, c->d4, hbytes, hipMemcpyDeviceToHost));
        } else {  // per level: the NMAT_ST stored slots, then the record-carried ones read back from the records
            size_t cmax = 0;
            for (int t = 0; t < c->nlev; ++t) cmax = std::max(cmax, (size_t)c->lv_host[t].C);
            int16_t *scr = nullptr;
            if (hipMalloc(&scr, (size_t)NMAT_REC * cmax * sizeof(int16_t)) != hipSuccess)
                return set_err(c, CCJ_E_OOM, "ccj_sync_host: device scratch of %.2f GB", NMAT_REC * cmax * 2e-9);
            int rc = CCJ_OK;
            for (int t = 0; t < c->nlev && rc == CCJ_OK; ++t) {
                const size_t C = (size_t)c->lv_host[t].C;
                if (hipMemcpy(c->h4 + c->lv_offh[t], c->d4 + c->lv_off[t], (size_t)NMAT_ST * C * sizeof(int16_t),
                              hipMemcpyDeviceToHost) != hipSuccess ||
                    ccjk_mat5(&c->T, t, scr, c->st) != 0 || hipStreamSynchronize(c->st) != hipSuccess ||
                    hipMemcpy(c->h4 + c->lv_offh[t] + (size_t)NMAT_ST * C, scr, (size_t)NMAT_REC * C * sizeof(int16_t),
                              hipMemcpyDeviceToHost) != hipSuccess)
                    rc = set_err(c, CCJ_E_HIP, "ccj_sync_host: mirror copy of level %d failed", t);
            }
            hipFree(scr);
            if (rc != CCJ_OK) return rc;
        }
    }
    HIPCHK(c, hipMemcpy(c->h2i.data(), c->d2i, A2_N * plane * sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(c->hvt.data(), c->d_vt, plane, hipMemcpyDeviceToHost));
    c->h_pk.resize(plane);
    HIPCHK(c, hipMemcpy(c->h_pk.data(), c->d_pk, plane * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    c->mirrored = true;
    return CCJ_OK;
}

extern "C" int ccj_fill(ccj_ctx *c) {
    if (c && (c->pending || c->res_pending)) return set_err(c, CCJ_E_STATE, "ccj_fill: a fold is in flight (ccj_wait first)");
    int rc = ccj_fill_device(c);
    if (rc) return rc;
    // the device traceback needs no host mirror; getters make it on demand (ccj_sync_host)
    return c->host_tb ? ccj_sync_host(c) : CCJ_OK;
}

namespace {
int ensure_mirror(const ccj_ctx *cc) {
    ccj_ctx *c = const_cast<ccj_ctx *>(cc);
    return c->mirrored ? CCJ_OK : ccj_sync_host(c);
}

// only the 2-D arrays (no 4-D copy): what ccj_get2 needs
int ensure_mirror_2d(const ccj_ctx *cc) {
    ccj_ctx *c = const_cast<ccj_ctx *>(cc);
    if (c->mirrored || c->mirrored2d) return CCJ_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t plane = (size_t)(c->n + 1) * c->rs;
    HIPCHK(c, hipMemcpy(c->h2i.data(), c->d2i, A2_N * plane * sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(c->hvt.data(), c->d_vt, plane, hipMemcpyDeviceToHost));
    c->mirrored2d = true;
    return CCJ_OK;
}

// W + traceback on the GPU (ccj_backtrack.hip); brackets on the host
// W + traceback on the GPU (ccj_backtrack.hip), enqueued on st behind the fill; the outputs land in
// pinned host buffers, ev_res marks them complete
int result_enqueue(ccj_ctx *c) {
    const int n = c->n;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->hr_W) {
        HIPCHK(c, hipHostMalloc(&c->hr_W, (n + 1) * sizeof(int), hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc(&c->hr_fp, (n + 1) * sizeof(int), hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc(&c->hr_ft, n + 1, hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc(&c->hr_bo, sizeof(BtOut), hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_res, hipEventDisableTiming));
    }
    HIPCHK(c, (hipError_t)ccjk_compute_W(&c->T, c->d_W, c->d_wterm, c->st));
    const int cap = std::min(4 * n + 64, 3000);
    HIPCHK(c, (hipError_t)ccjk_backtrack(&c->T, c->d_W, c->d_fpair, c->d_ftype, c->d_btout, cap, c->st));
    HIPCHK(c, hipMemcpyAsync(c->hr_W, c->d_W, (n + 1) * sizeof(int), hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(c->hr_fp, c->d_fpair, (n + 1) * sizeof(int), hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(c->hr_ft, c->d_ftype, n + 1, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(c->hr_bo, c->d_btout, sizeof(BtOut), hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipEventRecord(c->ev_res, c->st));
    c->res_pending = true;
    return CCJ_OK;
}

// wait for result_enqueue's outputs; the reference's exits, then brackets on the host
int result_finish(ccj_ctx *c, std::string &structure, std::string &out, std::chrono::steady_clock::time_point t0) {
    const int n = c->n;
    if (!c->res_pending) return set_err(c, CCJ_E_STATE, "no traceback in flight");
    c->res_pending = false;
    HIPCHK(c, hipEventSynchronize(c->ev_res));
    const BtOut bo = *c->hr_bo;
    c->W.assign(c->hr_W, c->hr_W + n + 1);
    c->w_ms = 0;
    c->bt_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->bt_steps = bo.steps;
    const int cap = std::min(4 * n + 64, 3000);
    for (int x = 0; x < bo.n_snbh; ++x) out += "Should not be here!\n";
    switch (bo.status) {
        case BT_OK: break;
        case BT_DIE:
            c->err = std::string(bt_prefix(bo.prefix)) + "This should not have happened!, " + bt_case_name(bo.node) + "\n";
            return CCJ_E_BACKTRACK;
        case BT_INTER: {
            char buf[160];
            snprintf(buf, sizeof buf, "NOT GOOD RESTR INTER, i=%d, j=%d, best_ip=%d, best_jp=%d\n", bo.args[0], bo.args[1],
                     bo.args[2], bo.args[3]);
            c->err = buf;
            return CCJ_E_INTER_EXIT;
        }
        case BT_ASSERT:
            c->err = "CCJ: matrices.hh:167: Assertion `!(i<=0 || l> n_)' failed.\n";
            return CCJ_E_BACKTRACK;
        default:
            return set_err(c, CCJ_E_HIP, "device traceback stack overflow (capacity %d)", cap);
    }
    HostView H(c);
    Backtracker B(H, c);
    for (int x = 1; x <= n; ++x) {
        B.f[x].pair = c->hr_fp[x];
        B.f[x].type = (char)c->hr_ft[x];
    }
    B.fill_structure();
    structure = B.structure;
    return CCJ_OK;
}

int device_result(ccj_ctx *c, std::string &structure, std::string &out) {
    const auto t0 = std::chrono::steady_clock::now();
    if (const int rc = result_enqueue(c)) return rc;
    return result_finish(c, structure, out, t0);
}

// the reference's outputs of W_final::ccj() (W_final.cc:79-104) into the caller's buffers
int emit_result(ccj_ctx *c, int rc, const std::string &st, const std::string &out, char *structure, double *energy_kcal,
                char *msgs, int msgs_cap) {
    if (msgs && msgs_cap > 0) {
        const size_t nb = std::min((size_t)msgs_cap - 1, out.size());
        memcpy(msgs, out.data(), nb);
        msgs[nb] = 0;
    }
    if (rc != CCJ_OK) return rc;
    if (energy_kcal) *energy_kcal = c->W[c->n] / 100.0;
    if (structure) {
        memcpy(structure, st.data() + 1, c->n);
        structure[c->n] = 0;
    }
    return CCJ_OK;
}
}  // namespace

extern "C" int ccj_result(ccj_ctx *c, char *structure, double *energy_kcal, char *msgs, int msgs_cap) {
    if (!c) return CCJ_E_ARG;
    if (!c->filled) return set_err(c, CCJ_E_STATE, "ccj_result before ccj_fill");
    std::string st, out;
    int rc = CCJ_OK;
    if (!c->host_tb) {
        rc = device_result(c, st, out);
    } else {
        if (int e = ensure_mirror(c)) return e;
        const auto t0 = std::chrono::steady_clock::now();
        compute_W(c);
        const auto t1 = std::chrono::steady_clock::now();
        c->w_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        HostView H(c);
        Backtracker B(H, c);
        try {
            B.run();
            B.fill_structure();
        } catch (const BacktrackExit &e) {
            c->err = e.stderr_msg;
            rc = e.code == 0 ? CCJ_E_INTER_EXIT : e.code == 2 ? CCJ_E_HIP : CCJ_E_BACKTRACK;
        }
        c->bt_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        st = B.structure;
        out = B.out;
    }
    return emit_result(c, rc, st, out, structure, energy_kcal, msgs, msgs_cap);
}

extern "C" int ccj_fill_async_after(ccj_ctx *c, const ccj_ctx *after) {
    if (!c) return CCJ_E_ARG;
    if (c->pending || c->res_pending) return set_err(c, CCJ_E_STATE, "ccj_fill_async: a fold is already in flight");
    if (after && after->device != c->device) return set_err(c, CCJ_E_ARG, "ccj_fill_async_after: contexts on different devices");
    if (const int rc = fill_enqueue(c, after)) return rc;
    // the device traceback follows the fill on the same stream; the host traceback needs the mirror
    return c->host_tb ? CCJ_OK : result_enqueue(c);
}

extern "C" int ccj_fill_async(ccj_ctx *c) { return ccj_fill_async_after(c, nullptr); }

extern "C" int ccj_wait(ccj_ctx *c, char *structure, double *energy_kcal, char *msgs, int msgs_cap) {
    if (!c) return CCJ_E_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    if (const int rc = fill_finish(c)) {
        c->res_pending = false;
        return rc;
    }
    if (c->host_tb) {
        if (const int rc = ccj_sync_host(c)) return rc;
        return ccj_result(c, structure, energy_kcal, msgs, msgs_cap);
    }
    std::string st, out;
    const int rc = result_finish(c, st, out, t0);
    return emit_result(c, rc, st, out, structure, energy_kcal, msgs, msgs_cap);
}

extern "C" int ccj_get4(const ccj_ctx *c, int mat, int i, int j, int k, int l) {
    if (!c || !c->filled || ensure_mirror(c) || mat < 0 || mat >= NMAT4) return INF;
    if (!(i <= j && j < k - 1 && k <= l)) return INF;
    if (i < 1 || l > c->n) return INF;
    const int t = (j - i) + (l - k);
    return (int)c->h4[c->lv_offh[t] + cell_offset_host(c->lv_host[t], mat, j - i, k - j - 2, i)];
}

extern "C" int ccj_get2(const ccj_ctx *c, int mat, int i, int j) {
    if (!c || !c->filled || ensure_mirror_2d(c) || i < 1 || j > c->n || i > j) return INF;
    switch (mat) {
        case CCJ_M2_P: return c->raw2(A2_P, i, j);
        case CCJ_M2_WBP: return c->raw2(A2_WBP, i, j);
        case CCJ_M2_WPP: return c->raw2(A2_WPP, i, j);
        case CCJ_M2_V: return c->raw2(A2_V, i, j);
        case CCJ_M2_VTYPE: return c->hvt[c->a2(i, j)];
        case CCJ_M2_WM: return c->raw2(A2_WM, i, j);
        case CCJ_M2_WMV: return c->raw2(A2_WMV, i, j);
        case CCJ_M2_WMP: return c->raw2(A2_WMP, i, j);
    }
    return INF;
}

extern "C" int ccj_getW(const ccj_ctx *c, int j) {
    if (!c || j < 0 || j >= (int)c->W.size()) return INF;
    return c->W[j];
}

extern "C" int ccj_hashes(const ccj_ctx *cc, uint64_t *out) {
    if (!cc || !cc->filled || !out) return CCJ_E_STATE;
    ccj_ctx *c = const_cast<ccj_ctx *>(cc);
    const int n = c->n;
    const uint64_t H0 = 1469598103934665603ull;
    // 4-D: each matrix is rewritten in canonical (i,j,k,l) order on the GPU (k_canon), copied back,
    // and FNV-hashed on host threads (one chain per matrix)
    const size_t cells = (size_t)ccj_num_cells(n);
    if (cells > 0) {
        HIPCHK(c, hipSetDevice(c->device));
        std::vector<long long> offij((size_t)(n + 1) * (n + 1), 0);
        long long pos = 0;
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j) {
                offij[(size_t)i * (n + 1) + j] = pos;
                for (int k = j + 2; k <= n; ++k) pos += n - k + 1;
            }
        long long *d_off = nullptr;
        int16_t *d_canon = nullptr;
        HIPCHK(c, hipMalloc(&d_off, offij.size() * sizeof(long long)));
        if (hipMalloc(&d_canon, cells * sizeof(int16_t)) != hipSuccess) {
            hipFree(d_off);
            return set_err(c, CCJ_E_OOM, "ccj_hashes: device scratch of %.2f GB", cells * 2e-9);
        }
        HIPCHK(c, hipMemcpy(d_off, offij.data(), offij.size() * sizeof(long long), hipMemcpyHostToDevice));
        std::vector<std::vector<int16_t>> host(NMAT4);
        std::vector<std::thread> th;
        int rc = CCJ_OK;
        for (int m = 0; m < NMAT4 && rc == CCJ_OK; ++m) {
            host[m].resize(cells);
            if (ccjk_canon(&c->T, m, d_off, d_canon, c->st) != 0 ||
                hipMemcpyAsync(host[m].data(), d_canon, cells * sizeof(int16_t), hipMemcpyDeviceToHost, c->st) != hipSuccess ||
                hipStreamSynchronize(c->st) != hipSuccess) {
                rc = set_err(c, CCJ_E_HIP, "ccj_hashes: canonical copy of matrix %d failed", m);
                break;
            }
            th.emplace_back([&host, out, m, H0] {
                out[m] = fnv(H0, host[m].data(), host[m].size() * sizeof(int16_t));
                std::vector<int16_t>().swap(host[m]);
            });
        }
        for (auto &x : th) x.join();
        hipFree(d_off);
        hipFree(d_canon);
        if (rc != CCJ_OK) return rc;
        if (ensure_mirror_2d(c)) return CCJ_E_STATE;
    } else {
        if (ensure_mirror(c)) return CCJ_E_STATE;
        for (int m = 0; m < NMAT4; ++m) {
            uint64_t h = H0;
            for (int i = 1; i <= n; ++i)
                for (int j = i; j <= n; ++j)
                    for (int k = j + 2; k <= n; ++k)
                        for (int l = k; l <= n; ++l) {
                            const int16_t v = (int16_t)ccj_get4(c, m, i, j, k, l);
                            h = fnv(h, &v, 2);
                        }
            out[m] = h;
        }
    }
    for (int m = 0; m < CCJ_NMAT2; ++m) {
        uint64_t h = H0;
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j) {
                const int32_t v = ccj_get2(c, m, i, j);
                h = fnv(h, &v, 4);
            }
        out[NMAT4 + m] = h;
    }
    uint64_t h = H0;
    for (size_t j = 0; j < c->W.size(); ++j) {
        const int32_t v = c->W[j];
        h = fnv(h, &v, 4);
    }
    out[NMAT4 + CCJ_NMAT2] = h;
    return CCJ_OK;
}

extern "C" int ccj_last_timing(const ccj_ctx *c, double *fill_ms, double *kernel_ms3) {
    if (!c) return CCJ_E_ARG;
    if (fill_ms) *fill_ms = c->fill_ms;
    if (kernel_ms3) {
        kernel_ms3[0] = c->level_ms;
        kernel_ms3[1] = c->diag_ms;
        kernel_ms3[2] = c->pre_ms;
    }
    return CCJ_OK;
}


// Algorithmic work model: R4 = sum over cells of 14a + 16b (the linear split-point
// reads of pseudo_loop.cc:181-644) + can_pair-filtered interior-loop candidates and stack terms
// (get_P{L,R,M}iloop :682-773; PO's interior branch reads nothing, A-Q5) ; each read is one int16.
// Writes are 22 int16 per cell.  The 2-D kernel's P recurrence (:166-179) reads 2 int16 per term.
static int work_model(int n, const short *S, const int (*pairt)[8], double *out) {
    auto pr = [&](int p, int q) { return pairt[S[p]][S[q]]; };
    auto can = [&](int p, int q) { return (q - p > TURN) && pr(p, q) > 0; };
    // PL/PR window count for outer (p, p+w): u1 <= min(w,30)-2, u2 <= min(w-u1-6, 28)
    std::vector<int> cntW((size_t)(n + 1) * (n + 2), 0);
    for (int w = 0; w < n; ++w)
        for (int p = 1; p + w <= n; ++p) {
            const int q = p + w;
            int cnt = 0;
            for (int u1 = 0; u1 <= std::min(w, MAXLOOP) - 2; ++u1)
                for (int u2 = 0; u2 <= std::min(w - u1 - 6, MAXLOOP - 2); ++u2)
                    cnt += can(p + u1 + 1, q - u2 - 1);
            cntW[(size_t)w * (n + 2) + p] = cnt;
        }
    double reads = 0, cells = 0, ilreads = 0;
    std::vector<int> cum(IE_U * IE_U);
    for (int j = 1; j <= n; ++j)
        for (int g = 2; j + g <= n; ++g) {
            const int k = j + g;
            const bool pm_ok = pr(j, k) > 0 && g > TURN;
            if (pm_ok)
                for (int u1 = 0; u1 < IE_U; ++u1)
                    for (int u2 = 0; u2 < IE_U; ++u2) {
                        const int d = j - 1 - u1, dp = k + 1 + u2;
                        int v = (d >= 1 && dp <= n) ? (int)can(d, dp) : 0;
                        if (u1) v += cum[(u1 - 1) * IE_U + u2];
                        if (u2) v += cum[u1 * IE_U + u2 - 1];
                        if (u1 && u2) v -= cum[(u1 - 1) * IE_U + u2 - 1];
                        cum[u1 * IE_U + u2] = v;
                    }
            for (int a = 0; a < j; ++a) {
                const int i = j - a;
                const bool pl = pr(i, j) > 0 && a > TURN;
                const double rl = pl ? (double)((a > TURN + 2) + cntW[(size_t)a * (n + 2) + i]) : 0.0;
                const double il_l = pl ? (double)cntW[(size_t)a * (n + 2) + i] : 0.0;
                for (int b = 0; k + b <= n; ++b) {
                    const int l = k + b;
                    double r = 14.0 * a + 16.0 * b + rl;
                    double il = il_l;
                    if (b > TURN && pr(k, l) > 0) {
                        r += (b > TURN + 2) + cntW[(size_t)b * (n + 2) + k];
                        il += cntW[(size_t)b * (n + 2) + k];
                    }
                    if (pm_ok) {
                        r += (a >= 1 && b >= 1);
                        if (a >= 2 && b >= 2) {
                            const int cm = cum[std::min(a - 2, IE_U - 1) * IE_U + std::min(b - 2, IE_U - 1)];
                            r += cm;
                            il += cm;
                        }
                    }
                    ilreads += il;
                    if (a >= 1 && b >= 1 && l - i > TURN && pr(i, l) > 0) r += 1;
                    reads += r;
                }
                cells += (double)(n - k + 1);
            }
        }
    double pterms = 0;
    for (int s = 3; s < n; ++s) pterms += (double)(n - s) * ((double)s * (s - 1) * (s - 2) / 6.0);
    out[0] = 2.0 * reads + 44.0 * cells;  // bytes, 4-D level kernels
    out[1] = 4.0 * pterms;                 // bytes, P terms of the 2-D kernels
    out[2] = reads;                        // R4 (4-D part)
    out[3] = cells;
    out[4] = ilreads;                      // interior-loop candidate reads (k_iloop)
    return CCJ_OK;
}

extern "C" int ccj_work_model(const ccj_ctx *c, double *out) {
    if (!c || !out) return CCJ_E_ARG;
    double w[5];
    const int rc = work_model(c->n, c->S.data(), c->pair, w);
    for (int x = 0; x < 4; ++x) out[x] = w[x];
    return rc;
}

extern "C" int ccj_work_split(const ccj_ctx *c, double *out2) {
    if (!c || !out2) return CCJ_E_ARG;
    double w[5];
    const int rc = work_model(c->n, c->S.data(), c->pair, w);
    out2[0] = 2.0 * w[4];                    // k_iloop: candidate reads
    out2[1] = w[0] - out2[0];                // k_level4d: everything else (incl. 44 B of stores per cell)
    return rc;
}

extern "C" int ccj_work_model_seq(const char *seq, int noGU, double *out) {
    if (!seq || !out) return CCJ_E_ARG;
    const int n = (int)strlen(seq);
    int pairt[8][8];
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) pairt[x][y] = BP_PAIR[x][y];
    if (noGU) pairt[3][4] = pairt[4][3] = 0;
    std::vector<short> S(n + 2, 0);
    for (int i = 1; i <= n; ++i) S[i] = (short)encode_base(seq[i - 1]);
    double w[5];
    const int rc = work_model(n, S.data(), pairt, w);
    for (int x = 0; x < 4; ++x) out[x] = w[x];
    return rc;
}

extern "C" int ccj_host_timing(const ccj_ctx *c, double *out3) {
    if (!c || !out3) return CCJ_E_ARG;
    out3[0] = c->sync_ms;
    out3[1] = c->w_ms;
    out3[2] = c->bt_ms;
    return CCJ_OK;
}

extern "C" int ccj_level_times(const ccj_ctx *c, double *level_ms, double *diag_ms, int cap) {
    if (!c) return CCJ_E_ARG;
    for (int t = 0; t < cap && t < (int)c->lev_ms_v.size(); ++t) {
        if (level_ms) level_ms[t] = c->lev_ms_v[t];
        if (diag_ms) diag_ms[t] = c->diag_ms_v[t];
    }
    return CCJ_OK;
}

extern "C" int ccj_iloop_times(const ccj_ctx *c, double *iloop_ms, int cap) {
    if (!c || !iloop_ms) return CCJ_E_ARG;
    for (int t = 0; t < cap && t < (int)c->il_ms_v.size(); ++t) iloop_ms[t] = c->il_ms_v[t];
    return CCJ_OK;
}

extern "C" int ccj_exchange_times(const ccj_ctx *c, double *edge_ms, double *bulk_ms, int cap) {
    if (!c || (!edge_ms && !bulk_ms)) return CCJ_E_ARG;
    for (int t = 0; t < cap && t < (int)c->xch_ms_v.size(); ++t) {
        if (edge_ms) edge_ms[t] = c->xch_ms_v[t];
        if (bulk_ms) bulk_ms[t] = c->xbulk_ms_v[t];
    }
    return CCJ_OK;
}

extern "C" double ccj_iloop_ms(const ccj_ctx *c) { return c ? c->il_ms : 0.0; }
extern "C" double ccj_ppush_ms(const ccj_ctx *c) { return c ? c->pp_ms : 0.0; }
extern "C" int ccj_ppush_times(const ccj_ctx *c, double *ppush_ms, int cap) {
    if (!c || !ppush_ms) return CCJ_E_ARG;
    for (int t = 0; t < cap && t < (int)c->pp_ms_v.size(); ++t) ppush_ms[t] = c->pp_ms_v[t];
    return CCJ_OK;
}

extern "C" int ccj_set_timing(ccj_ctx *c, int mode) {
    if (!c || mode < 0 || mode > 2) return CCJ_E_ARG;
    c->level_timing = mode;
    return CCJ_OK;
}

extern "C" int ccj_shard_blocks(int n, int t, int world, int rank, int *a_out, int cap) {
    if (world < 1 || rank < 0 || rank >= world || t < 0 || (cap > 0 && !a_out)) return -CCJ_E_ARG;
    (void)n;
    const int cnt = shard_count(t, world, rank);
    for (int o = 0; o < cnt && o < cap; ++o) a_out[o] = shard_a(o, world, rank);
    return cnt;
}

extern "C" int ccj_level_layout(int n, int t, int world, long long *C, int *M) {
    if (!C || !M || world < 1 || t < 0) return CCJ_E_ARG;
    const int m = n - t - 2;
    *M = m > 0 ? m * (m + 1) / 2 : 0;
    *C = (long long)(t + 1) * *M;  // unpadded for every world (the exchange packs slices)
    return CCJ_OK;
}

// The exchange geometry k_pack / k_unpack use (ccj_engine.h xch_*), per part (0 = edge, 1 = bulk),
// for tests and integrators: {nmax, tail offset (= padded body), slice elements}.
extern "C" int ccj_exchange_layout(int n, int t, int world, int part, long long *out3) {
    if (!out3 || world < 1 || t < 0 || n < 4 || t > n - 3 || (part != XCH_EDGE && part != XCH_BULK)) return CCJ_E_ARG;
    const int m = n - t - 2, M = m * (m + 1) / 2, nmax = xch_nmax(t, world, part);
    out3[0] = nmax;
    out3[1] = xch_body(nmax, M);                // the part's tail (edge: P(t+1) partials, then span t; bulk: none)
    out3[2] = xch_slice(n, nmax, M, part);      // slice elements
    return CCJ_OK;
}

// which == 0 (pack, rank `rank`): out[k] for every body element k of the rank's slice of the part =
//   the level element (x * C + a * M + c) k_pack copies there, -1 for padding;
// which == 1 (unpack at rank `rank`): out[e] for every level element e = x * C + a * M + c = the
//   position in the part's gathered buffer (owner * slice + body position) k_unpack reads it from, -1
//   for the rank's own cells and the other part's.
// Returns the number of entries (cap: the room in out), or -CCJ_E_ARG.
extern "C" long long ccj_exchange_index(int n, int t, int world, int rank, int part, int which, long long *out, long long cap) {
    if (world < 1 || rank < 0 || rank >= world || t < 0 || n < 4 || t > n - 3 || (which != 0 && which != 1) ||
        (part != XCH_EDGE && part != XCH_BULK))
        return -CCJ_E_ARG;
    const int m = n - t - 2, M = m * (m + 1) / 2, nmax = xch_nmax(t, world, part);
    const long long C = (long long)(t + 1) * M, slice = xch_slice(n, nmax, M, part);
    const long long cnt = which == 0 ? (long long)NMAT4 * nmax * M : (long long)NMAT4 * C;
    if (cap < cnt || !out) return cnt;
    if (which == 0) {
        for (long long k = 0; k < cnt; ++k) out[k] = -1;
        const int np = xch_pcount(t, world, rank, part);
        for (int x = 0; x < NMAT4; ++x)
            for (int k = 0; k < np; ++k)
                for (int c = 0; c < M; ++c)
                    out[xch_pos(x, k, c, nmax, M)] = x * C + (long long)shard_a(xch_own(k, part), world, rank) * M + c;
    } else {
        for (int x = 0; x < NMAT4; ++x)
            for (int a = 0; a <= t; ++a) {
                int ro, pa, k;
                xch_src(a, world, ro, pa, k);
                for (int c = 0; c < M; ++c)
                    out[x * C + (long long)a * M + c] = (ro == rank || pa != part) ? -1 : ro * slice + xch_pos(x, k, c, nmax, M);
            }
    }
    return cnt;
}

extern "C" int ccj_comm_unique_id(char *id_out) {
    if (!id_out) return CCJ_E_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return CCJ_E_HIP;
    static_assert(sizeof(id) == CCJ_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id_out, &id, sizeof id);
    return CCJ_OK;
}

extern "C" int ccj_comm_init(ccj_ctx *c, const char *id_in) {
    if (!c || !id_in) return CCJ_E_ARG;
    if (c->world == 1 || c->simulate) return CCJ_OK;
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId id;
    memcpy(&id, id_in, sizeof id);
    if (c->comm_b) ncclCommDestroy(c->comm_b);
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = c->comm_b = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c->comm, c->world, id, c->rank);
    if (r != ncclSuccess) return set_err(c, CCJ_E_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    // the bulk all-gathers run on their own stream: their own communicator (same ranks, same order), so
    // the two streams' collectives never queue behind each other inside one communicator
    const ncclResult_t r2 = ncclCommSplit(c->comm, 0, c->rank, &c->comm_b, nullptr);
    if (r2 != ncclSuccess) return set_err(c, CCJ_E_HIP, "ncclCommSplit: %s", ncclGetErrorString(r2));
    return CCJ_OK;
}

extern "C" int ccj_group_create(int world, ccj_group **out) {
    if (!out || world < 1) return CCJ_E_ARG;
    *out = new ccj_group();
    (*out)->world = world;
    (*out)->members.assign(world, nullptr);
    return CCJ_OK;
}

extern "C" void ccj_group_destroy(ccj_group *g) { delete g; }

extern "C" int ccj_comm_init_local(ccj_ctx *c, ccj_group *g) {
    if (!c || !g || g->world != c->world || c->world < 2 || c->simulate) return CCJ_E_ARG;
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->members[c->rank] && g->members[c->rank] != c)
        return set_err(c, CCJ_E_STATE, "ccj_comm_init_local: rank %d of the group is already taken", c->rank);
    g->members[c->rank] = c;
    c->lgroup = g;
    return CCJ_OK;
}

extern "C" int ccj_n(const ccj_ctx *c) { return c ? c->n : 0; }
extern "C" const char *ccj_last_error(const ccj_ctx *c) { return c ? c->err.c_str() : g_create_err.c_str(); }

extern "C" void ccj_destroy(ccj_ctx *c) {
    if (!c) return;
    bool leak_send = false;
    if (c->lgroup) {  // leave the in-process group: no member may copy from this context's buffers
        ccj_group *g = c->lgroup;
        std::unique_lock<std::mutex> lk(g->mu);
        if (g->members[c->rank] == c) {  // registered (a failed ccj_comm_init_local never was)
            g->members[c->rank] = nullptr;
            g->broken = true;  // the exchange cannot complete without this rank
            g->cv.notify_all();
        }
        // peers still copying from d_send; bounded like the group's barriers (a peer stuck in a
        // GPU call must not hang this destroy): on timeout d_send is leaked instead of freed
        if (!g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->busy == 0; })) {
            fprintf(stderr, "ccj_destroy: a group member is still copying after 120 s; leaking its source buffer\n");
            leak_send = true;
        }
        // the peers' asynchronous bulk copies (local_bulk_gather) from this member's send slice
        for (ccj_ctx *p : g->members)
            if (p && p->st_x) hipStreamSynchronize(p->st_x);
        c->lgroup = nullptr;
    }
    hipSetDevice(c->device);
    if (c->st) hipStreamSynchronize(c->st);
    if (c->st_copy) hipStreamSynchronize(c->st_copy);
    if (c->st_p) hipStreamSynchronize(c->st_p);
    if (c->st_il) hipStreamSynchronize(c->st_il);
    if (c->st_d) hipStreamSynchronize(c->st_d);
    if (c->st_x) hipStreamSynchronize(c->st_x);
    hipFree(c->d4);
    hipFree(c->d_ie);
    hipFree(c->d_est);
    hipFree(c->d_hp);
    hipFree(c->d_pt);
    hipFree(c->d_pair);
    hipFree(c->d_rtype);
    hipFree(c->d_lx);
    hipFree(c->d_err);
    hipFree(c->d_S);
    hipFree(c->d_S1);
    hipFree(c->d_prm);
    hipFree(c->d_lv);
    hipFree(c->d_lb);
    hipFree(c->d_ld);
    hipFree(c->d4x_alloc);
    hipFree(c->d_icount);
    hipFree(c->d_ioff);
    hipFree(c->d_rec);
    hipFree(c->d_rk);
    hipFree(c->d_acc);
    hipFree(c->d_wterm);
    hipFree(c->d_lord);
    hipFree(c->d_lord_off);
    hipFree(c->d_wbw);
    hipFree(c->pmx_alloc);
    hipFree(c->d_ldx);
    hipFree(c->d_il);
    hipFree(c->d_ilm);
    hipFree(c->d_dummy);
    hipFree(c->d_items);
    for (int part = 0; part < 2; ++part) {
        if (!leak_send) hipFree(c->d_send[part]);
        hipFree(c->d_recv[part]);
    }
    if (c->h_stage) hipHostFree(c->h_stage);
    if (c->h_ioff) hipHostFree(c->h_ioff);
    if (c->h_icount) hipHostFree(c->h_icount);
    if (c->ev_stage) hipEventDestroy(c->ev_stage);
    if (c->hr_W) hipHostFree(c->hr_W);
    if (c->hr_fp) hipHostFree(c->hr_fp);
    if (c->hr_ft) hipHostFree(c->hr_ft);
    if (c->hr_bo) hipHostFree(c->hr_bo);
    if (c->ev_res) hipEventDestroy(c->ev_res);
    hipFree(c->d_ilseg);
    hipFree(c->d_ilmseg);
    hipFree(c->d2i);
    hipFree(c->d_pk);
    hipFree(c->d_W);
    hipFree(c->d_fpair);
    hipFree(c->d_ftype);
    hipFree(c->d_btout);
    hipFree(c->d_vt);
    if (c->h4) hipHostFree(c->h4);
    for (auto e : c->lev_done) hipEventDestroy(e);
    for (auto e : c->p_done) hipEventDestroy(e);
    for (auto e : c->pp_done) hipEventDestroy(e);
    for (auto e : c->bulk_done) hipEventDestroy(e);
    if (c->ev_bpacked) hipEventDestroy(c->ev_bpacked);
    if (c->ev_bcopied) hipEventDestroy(c->ev_bcopied);
    if (c->st_p) hipStreamDestroy(c->st_p);
    if (c->st_x) hipStreamDestroy(c->st_x);
    if (c->comm_b) ncclCommDestroy(c->comm_b);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->st_il) hipStreamDestroy(c->st_il);
    if (c->st_d) hipStreamDestroy(c->st_d);
    for (auto e : c->il_done) hipEventDestroy(e);
    for (auto e : c->dg_done) hipEventDestroy(e);
    for (auto e : c->tev) hipEventDestroy(e);
    if (c->ev_start) hipEventDestroy(c->ev_start);
    if (c->ev_end) hipEventDestroy(c->ev_end);
    if (c->ev_pre) hipEventDestroy(c->ev_pre);
    if (c->st) hipStreamDestroy(c->st);
    if (c->st_copy) hipStreamDestroy(c->st_copy);
    delete c;
}
