// ccj_pf.cc — host side of the CCJ partition function (include/ccj_pf.h).
//
// Builds the Boltzmann tables the way the reference's W_final_pf constructor gets them
// (part_func.cc:31-93: scale_pf_parameters() -> get_scaled_exp_params, params.c:558-738;
// rescale_pk_globals :127-146; exp_params_rescale :97-125), the per-sequence weight tables
// (HairpinE :214-220 with the special-hairpin strstr cases, get_e_stP / get_e_intP :877-891, which
// call pow()), drives the level-synchronous fill of ccj_pf.hip, then runs W (:163-172) and the
// stochastic traceback (stoch_backtrack.cc:36-326) on the host over the 2-D matrices.
//
// Everything here is evaluated as written, without floating-point contraction, with the host
// libm — the same exp/log/pow/sin the reference links — so the device only ever multiplies and
// adds table values and the results are bit-identical to part_func.cc (-ffp-contract=off).
//
// Raw INF entries.  get_scaled_exp_params reads the raw 37 C tables, in which some dangles /
// multiloop and exterior mismatches are INF (SMOOTH turns INF into a weight of 1).  The
// ccj_energy_params blob holds the MFE tables, where those entries are clamped to 0
// (params.c:487-512), so the raw tables come separately (ccj_pf_raw, the .pfraw files).  Without
// them the pair type 0 rows are taken as INF — true for every parameter file the reference ships;
// its other raw-INF entries (the 'N' column, pair type 7) are unreachable for A/C/G/U sequences.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ccj_pf.h"
#include "ccj_pf_energy.h"
#include "ccj_pf_engine.h"
#include "ccj_items.h"

using namespace ccj;

namespace {

constexpr double K0 = 273.15, GASCONST = 1.98717;  // params/constants.h:13-15

const int BP_PAIR_PF[8][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 5, 0, 0, 5}, {0, 0, 0, 1, 0, 0, 0, 0},
                              {0, 0, 2, 0, 3, 0, 0, 0}, {0, 6, 0, 4, 0, 0, 0, 6}, {0, 0, 0, 0, 0, 0, 2, 0},
                              {0, 0, 0, 0, 0, 1, 0, 0}, {0, 6, 0, 0, 5, 0, 0, 0}};  // pair_mat.h:20-29

uint64_t fnv_init() { return 1469598103934665603ull; }
void fnv_bytes(uint64_t &h, const void *p, size_t n) {
    const unsigned char *c = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) {
        h ^= c[i];
        h *= 1099511628211ull;
    }
}
template <class T>
uint64_t fnv_arr(const T *p, size_t cnt) {
    uint64_t h = fnv_init();
    fnv_bytes(h, p, cnt * sizeof(T));
    return h;
}

// RESCALE_BF (params.c:66-72) at 37 C: RESCALE_dG is the identity (dT == 1.0) and pf_smooth == 1
// makes TRUNC_MAYBE the identity.
double bf(double kT, int dG) { return exp(-(double)dG * 10. / kT); }
// RESCALE_BF_SMOOTH (params.c:39-45, 74-82), SCALE == 10
double bf_smooth(double kT, int dG) {
    const double X = -(double)dG;
    double s;
    if (X / 10 < -1.2283697) s = 0;
    else if (X / 10 > 0.8660254) s = X;
    else s = 10 * 0.38490018 * (sin(X / 10 - 0.34242663) + 1) * (sin(X / 10 - 0.34242663) + 1);
    return exp(s * 10. / kT);
}

void build_exp(const ccj_energy_params &p, const ccj_pf_raw *raw, const ccj_pk_penalties &k, PfExp &E) {
    memset(&E, 0, sizeof E);
    const double kT = 1. * (37. + K0) * GASCONST;  // betaScale * (temperature + K0) * GASCONST
    E.kT = kT;
    E.pf_scale = 1.;  // exp_params_rescale forces 1 (part_func.cc:107)
    E.lxc = p.lxc * 1.0;
    E.TermAU = bf(kT, p.TerminalAU);
    E.MLbase = bf(kT, p.MLbase);
    E.MLclosing = bf(kT, p.MLclosing);
    for (int i = 0; i < 31; ++i) E.hairpin[i] = bf(kT, p.hairpin[i]);
    double internal[31];
    for (int i = 0; i <= 30; ++i) {
        E.bulge[i] = bf(kT, p.bulge[i]);
        internal[i] = bf(kT, p.internal_loop[i]);
    }
    internal[2] = exp(-80 * 10. / kT);  // james_rule (params.c:609-610)
    for (int j = 0; j <= 30; ++j) {
        const double GT = (double)p.ninio2;
        E.ninio[j] = exp(-(p.max_ninio < j * GT ? (double)p.max_ninio : j * GT) * 10. / kT);
    }
    const int ntetra = (int)strnlen(p.Tetraloops, sizeof p.Tetraloops);
    for (int i = 0; i * 7 < ntetra && i < 40; ++i) E.tetra[i] = bf(kT, p.Tetraloop_E[i]);
    const int ntri = (int)strnlen(p.Triloops, sizeof p.Triloops);
    for (int i = 0; i * 5 < ntri && i < 40; ++i) E.tri[i] = bf(kT, p.Triloop_E[i]);
    const int nhex = (int)strnlen(p.Hexaloops, sizeof p.Hexaloops);
    for (int i = 0; i * 9 < nhex && i < 40; ++i) E.hex[i] = bf(kT, p.Hexaloop_E[i]);
    for (int i = 0; i < 8; ++i) E.MLintern[i] = bf(kT, p.MLintern[1]);  // one ML_intern37 for every type
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 5; ++j) {
            E.dangle5[i][j] = bf_smooth(kT, raw ? raw->dangle5[i][j] : i == 0 ? CCJ_INF : p.dangle5[i][j]);
            E.dangle3[i][j] = bf_smooth(kT, raw ? raw->dangle3[i][j] : i == 0 ? CCJ_INF : p.dangle3[i][j]);
        }
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) E.stack[i][j] = bf(kT, p.stack[i][j]);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 5; ++j)
            for (int q = 0; q < 5; ++q) {
                E.mismatchI[i][j][q] = bf(kT, p.mismatchI[i][j][q]);
                E.mismatch1nI[i][j][q] = bf(kT, p.mismatch1nI[i][j][q]);
                E.mismatchH[i][j][q] = bf(kT, p.mismatchH[i][j][q]);
                E.mismatch23I[i][j][q] = bf(kT, p.mismatch23I[i][j][q]);
                E.mismatchM[i][j][q] = bf_smooth(kT, raw ? raw->mismatchM[i][j][q] : i == 0 ? CCJ_INF : p.mismatchM[i][j][q]);
                E.mismatchExt[i][j][q] =
                    bf_smooth(kT, raw ? raw->mismatchExt[i][j][q] : i == 0 ? CCJ_INF : p.mismatchExt[i][j][q]);
            }
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j)
            for (int a = 0; a < 5; ++a)
                for (int b = 0; b < 5; ++b) {
                    E.int11[i][j][a][b] = bf(kT, p.int11[i][j][a][b]);
                    for (int c = 0; c < 5; ++c) {
                        E.int21[i][j][a][b][c] = bf(kT, p.int21[i][j][a][b][c]);
                        for (int d = 0; d < 5; ++d) E.int22[i][j][a][b][c][d] = bf(kT, p.int22[i][j][a][b][c][d]);
                    }
                }
    // expinternal[0..30] and the 26 doubles that follow it in vrna_exp_param_t (basic.h:127-128)
    for (int i = 0; i <= 30; ++i) E.internal57[i] = internal[i];
    for (int i = 31; i < 57; ++i) E.internal57[i] = (&E.mismatchExt[0][0][0])[i - 31];
    // rescale_pk_globals: RESCALE_BF(x, 3x, TT, kT) == exp(-x*10/kT) at 37 C
    E.PS = bf(kT, k.PS);
    E.PSM = bf(kT, k.PSM);
    E.PSP = bf(kT, k.PSP);
    E.PB = bf(kT, k.PB);
    E.PUP = bf(kT, k.PUP);
    E.PPS = bf(kT, k.PPS);
    E.a = bf(kT, k.a);
    E.b = bf(kT, k.b);
    E.c = bf(kT, k.c);
    E.ap = bf(kT, k.ap);
    E.bp = bf(kT, k.bp);
    E.cp = bf(kT, k.cp);
}

const char *const kExpNames =
    "expstack exphairpin expbulge expinternal expninio expmismatchI expmismatch1nI expmismatch23I expmismatchH "
    "expmismatchM expmismatchExt expdangle5 expdangle3 expint11 expint21 expint22 expMLintern scalars exptetra exptri "
    "exphex pk";
constexpr int kNExp = 22;

}  // namespace

struct ccj_pf_ctx {
    int n = 0, rs = 0, dangles = 2, device = 0;
    std::string seq;
    ccj_energy_params prm{};
    ccj_pk_penalties pen{};
    int pair[8][8]{};
    int rtype[8]{};
    std::vector<short> S, S1;
    PfExp E{};
    std::vector<double> mlb, cpp, pup, hp;
    std::vector<PfLvl> lv;
    long long cells = 0;  // cells of one 4-D matrix
    // device
    PfExp *d_E = nullptr;
    short *d_S = nullptr, *d_S1 = nullptr;
    int8_t *d_pt = nullptr, *d_pair = nullptr, *d_rtype = nullptr;
    double *d_hp = nullptr, *d_est = nullptr, *d_ieO = nullptr, *d_ieI = nullptr, *d_mlb = nullptr, *d_cpp = nullptr, *d_pup = nullptr;
    double *d_2d = nullptr;  // CCJ_PF_NMAT2 planes of (n+1)*rs
    long long *d_Pacc = nullptr;
    unsigned long long *d_Pabs = nullptr;
    int *d_d4 = nullptr;
    int *d_prec = nullptr;  // split-loop operand records (PfDev::r1 .. r4)
    int *d_cx = nullptr, *d_pmx = nullptr;  // k_pf_iloop's copies of PL / PR and PM (ccj_pf_engine.h)
    double *d_R = nullptr;                  // k_pf_iloop's sums of one level, 3 planes of max C_t
    uint32_t *d_items = nullptr, *d_mO = nullptr, *d_mI = nullptr;
    std::vector<long long> ifirst;          // k_pf_iloop items of level t: [ifirst[t], ifirst[t+1])
    std::vector<uint32_t> h_items, h_mO, h_mI;  // host copies (ccj_pf_work_model)
    PfLvl *d_ld = nullptr;
    hipStream_t st = nullptr;     // levels (k_pf_level), the memsets, the result copies
    hipStream_t st_il = nullptr;  // k_pf_iloop(t): after level t-2
    hipStream_t st_d = nullptr;   // k_pf_ppush(s-3) (P of span s), k_pf_diag(s): after level s-3
    std::vector<hipEvent_t> ev_lev, ev_il, ev_dg;  // level t done, iloop t done, span s done
    hipEvent_t ev_start = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    PfDev D{};
    // results
    bool filled = false;
    std::vector<double> h2d;  // host copies of the 2-D planes
    std::vector<double> W;
    double energy = 0;
    float fill_ms = 0;
    // per-kernel-family timing (ccj_pf_set_timing): an event pair around every launch
    bool timing = false;
    std::vector<hipEvent_t> tev;
    std::vector<int> tfam;      // family of launch q: 0 k_pf_iloop, 1 k_pf_level, 2 P terms (k_pf_ppush / k_pf_pterm), 3 k_pf_diag
    double kms[4] = {0, 0, 0, 0};
    std::string msg;
    // vrna_urn() of the reference build: rand() / RAND_MAX (utils.c:262-271, no HAVE_ERAND48), on
    // this context's own glibc random_r state (a fresh one behaves like a process that never
    // called srand, i.e. srand(1))
    struct random_data rnd {};
    char rnd_state[128]{};

    size_t plane() const { return (size_t)(n + 1) * rs; }
    double g2(int m, int i, int j) const { return i > j ? 0.0 : h2d[(size_t)m * plane() + (size_t)(j - i) * rs + i]; }
    int ptype(int i, int j) const { return pair[S[i]][S[j]]; }
};

// The allocations of ccj_pf_create for a sequence of length n, in bytes: device (every hipMalloc
// of create_impl; the work items, sequence-dependent, by their count when every pair can pair) and host (the two get_e_intP window tables, built before they are uploaded).
extern "C" void ccj_pf_footprint(int n, unsigned long long *device_bytes, unsigned long long *host_bytes) {
    if (n < 1) n = 1;
    const unsigned long long rs = (unsigned long long)n + 2, plane = (unsigned long long)(n + 1) * rs;
    const unsigned long long ie = 2ull * (PF_IEW * PF_IEW * plane + PF_ILW) * sizeof(double);  // ieO + ieI (+ tail pad)
    unsigned long long d4 = 0, cx = 0, pmx = 0, maxC = 1, rows = 0;
    for (int t = 0; t <= n - 3; ++t) {
        const unsigned long long m = (unsigned long long)(n - t - 2), C = (unsigned long long)(t + 1) * (m * (m + 1) / 2);
        d4 += (unsigned long long)PF_NMAT4 * C;
        cx += 2 * C;
        pmx += m * (unsigned long long)n * (t + 1);
        maxC = std::max(maxC, C);
        // work items: create_impl's enumeration with every pair able to pair (its upper bound), one item
        // per 64-lane chunk of each PL / PR / PM row
        const int mi = (int)m;
        for (int i = 1; i <= mi; ++i) rows += (unsigned long long)std::max(0, t - 5) * ((mi - i) / 64 + 1);  // PL, a in [6, t]
        for (int q = 0; q < mi; ++q) rows += (unsigned long long)std::max(0, t - 5) * (q / 64 + 1);         // PR, a in [0, t-6]
        for (int h = 0; h <= mi - 1; ++h)                                                                   // PM
            for (int j = 1; j + h + 2 <= n; ++j) {
                const int k = j + h + 2, alo = std::max(2, t - (n - k)), ahi = std::min(t - 2, j - 1);
                if (alo <= ahi) rows += (unsigned long long)((ahi - alo) / 64 + 1);
            }
    }
    unsigned long long dev = ie + (d4 + cx + pmx + (unsigned long long)PF_RECS * (d4 / PF_NMAT4)) * sizeof(int) +
                             2ull * 3 * maxC * sizeof(double);  // d4, copies, split-loop records, R
    dev += (unsigned long long)CCJ_PF_NMAT2 * plane * sizeof(double) + 2 * plane * sizeof(long long);  // 2-D, Pacc, Pabs
    dev += 3 * plane * sizeof(double) + plane + 2ull * plane * PF_IEW * sizeof(uint32_t);             // hp, est, cp; pt; mO, mI
    dev += rows * sizeof(uint32_t) + sizeof(PfExp) + (1u << 20);                                      // items; small tables
    if (device_bytes) *device_bytes = dev;
    if (host_bytes) *host_bytes = ie;
}

namespace {

int pf_err(ccj_pf_ctx *c, int code, const char *what, hipError_t e = hipSuccess) {
    if (c) c->msg = e == hipSuccess ? std::string(what) : std::string(what) + ": " + hipGetErrorString(e);
    return code;
}
#define PFCHK(c, x)                                                   \
    do {                                                              \
        const hipError_t e_ = (x);                                    \
        if (e_ != hipSuccess) return pf_err((c), CCJ_E_HIP, #x, e_);  \
    } while (0)

// exp_E_Hairpin (loops/hairpin.h:231-291) * scale[j-i+1] for HairpinE(i, j) (part_func.cc:214-220)
double hairpin_pf(const ccj_pf_ctx &c, int i, int j) {
    const int type = c.ptype(i, j);
    if (type == 0) return 0;
    const PfExp &P = c.E;
    const int u = j - i - 1;
    double q;
    if (u <= 30) q = P.hairpin[u];
    else q = P.hairpin[30] * exp(-(P.lxc * log(u / 30.)) * 10. / P.kT);
    if (u < 3) return q * 1.0;
    const char *str = c.seq.c_str() + (i - 1);
    if (c.prm.special_hp) {
        if (u == 4) {
            char tl[7] = {0};
            memcpy(tl, str, 6);
            if (const char *ts = strstr(c.prm.Tetraloops, tl)) {
                if (type != 7) return P.tetra[(ts - c.prm.Tetraloops) / 7] * 1.0;
                q *= P.tetra[(ts - c.prm.Tetraloops) / 7];
            }
        } else if (u == 6) {
            char tl[9] = {0};
            memcpy(tl, str, 8);
            if (const char *ts = strstr(c.prm.Hexaloops, tl)) return P.hex[(ts - c.prm.Hexaloops) / 9] * 1.0;
        } else if (u == 3) {
            char tl[6] = {0};
            memcpy(tl, str, 5);
            if (const char *ts = strstr(c.prm.Triloops, tl)) return P.tri[(ts - c.prm.Triloops) / 6] * 1.0;
            return (type > 2 ? q * P.TermAU : q) * 1.0;
        }
    }
    q *= P.mismatchH[type][c.S1[i + 1]][c.S1[j - 1]];
    return q * 1.0;
}

// compute_int (part_func.cc:872-875)
double compute_int_pf(const ccj_pf_ctx &c, int i, int j, int k, int l) {
    return exp_E_IntLoop_pf(c.E, k - i - 1, j - l - 1, c.ptype(i, j), c.rtype[c.ptype(k, l)], c.S1[i + 1], c.S1[j - 1],
                            c.S1[k - 1], c.S1[l + 1]);
}

double ext_pf(const ccj_pf_ctx &c, int i, int j) {  // exp_Extloop :180-190
    const int tt = c.ptype(i, j);
    if (c.dangles == 1 || c.dangles == 2) return exp_E_ExtLoop_pf(c.E, tt, i > 1 ? c.S[i - 1] : -1, j < c.n ? c.S[j + 1] : -1);
    return exp_E_ExtLoop_pf(c.E, tt, -1, -1);
}
double mlstem_pf(const ccj_pf_ctx &c, int i, int j) {  // exp_MLstem :192-201
    const int tt = c.ptype(i, j);
    if (c.dangles == 1 || c.dangles == 2) return exp_E_MLstem_pf(c.E, tt, i > 1 ? c.S[i - 1] : -1, j < c.n ? c.S[j + 1] : -1);
    return exp_E_MLstem_pf(c.E, tt, -1, -1);
}
double mbloop_pf(const ccj_pf_ctx &c, int i, int j) {  // exp_Mbloop :203-212
    const int tt = c.pair[c.S[j]][c.S[i]];
    if (c.dangles == 1 || c.dangles == 2) return exp_E_MLstem_pf(c.E, tt, j < c.n ? c.S[j - 1] : -1, i > 1 ? c.S[i + 1] : -1);
    return exp_E_MLstem_pf(c.E, tt, -1, -1);
}

void run_threads(int total, int nthr, const std::function<void(int, int)> &f) {
    std::vector<std::thread> th;
    const int per = (total + nthr - 1) / nthr;
    for (int t = 0; t < nthr; ++t) {
        const int lo = t * per, hi = std::min(total, lo + per);
        if (lo < hi) th.emplace_back(f, lo, hi);
    }
    for (auto &x : th) x.join();
}

void free_dev(ccj_pf_ctx *c) {
    void *ptrs[] = {c->d_E, c->d_S, c->d_S1, c->d_pt, c->d_pair, c->d_rtype, c->d_hp, c->d_est, c->d_ieO, c->d_ieI,
                    c->d_mlb, c->d_cpp, c->d_pup, c->d_2d, c->d_Pacc, c->d_Pabs, c->d_d4, c->d_cx, c->d_pmx,
                    c->d_prec, c->d_R, c->d_items, c->d_mO, c->d_mI, c->d_ld};
    for (void *p : ptrs)
        if (p) hipFree(p);
    if (c->e0) hipEventDestroy(c->e0);
    if (c->e1) hipEventDestroy(c->e1);
    for (hipEvent_t e : c->tev) hipEventDestroy(e);
    c->tev.clear();
    for (auto *v : {&c->ev_lev, &c->ev_il, &c->ev_dg}) {
        for (hipEvent_t e : *v)
            if (e) hipEventDestroy(e);
        v->clear();
    }
    if (c->ev_start) hipEventDestroy(c->ev_start);
    if (c->st_il) hipStreamDestroy(c->st_il);
    if (c->st_d) hipStreamDestroy(c->st_d);
    if (c->st) hipStreamDestroy(c->st);
}

// Algorithmic bytes of one fill per kernel family (ccj_pf_work_model): the operands each kernel's
// recurrences read from and write to HBM-resident arrays, counted from the same enumerations the
// kernels run (the small 2-D tables and weight windows, which stay in cache, are not charged).
//   k_pf_iloop: 4 B per active lane per window term it loads (masked), 4 B stack operand, 8 B R store
//   k_pf_level: 4 B per 4-D operand load of the 21 recurrences (split loops, seeds, P blocks as
//               evaluated for this sequence's pairs), 8 B per R read, 21 x 4 B stores + 4 B per copy
//   P terms (k_pf_ppush / k_pf_pterm): 2 x 4 B per PK product, the pull form's operands;  k_pf_diag: 8 B per 2-D operand of the span's sums
struct PfWork {
    double iloop = 0, level = 0, pterm = 0, diag = 0;
};

PfWork pf_work_model(const ccj_pf_ctx &c) {
    const int n = c.n, rs = c.rs;
    PfWork w;
    if (n < 3) return w;
    auto low = [](int u) { return u < 0 ? 0u : (2u << u) - 1u; };
    const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<double> il(n, 0.0), lv(n, 0.0);
    run_threads(n - 2, nthr, [&](int t0, int t1) {
        for (int t = t0; t < t1; ++t) {
            const int m = n - t - 2;
            double b_il = 0;
            for (long long q = c.ifirst[t]; q < c.ifirst[t + 1]; ++q) {
                const uint32_t it = c.h_items[q];
                const int role = (int)(it >> 30), f1 = (int)((it >> 20) & 1023), f2 = (int)((it >> 10) & 1023),
                          ch = (int)(it & 1023);
                if (role < 2) {
                    const int a = f1, b = t - a;
                    const int lanes = role == 0 ? std::min(64, m - f2 + 1 - ch * 64) : std::min(64, f2 + 1 - ch * 64);
                    const int w0 = role == 0 ? a : b, p0 = role == 0 ? f2 : f2 + a + 3;
                    const uint32_t *mw = c.h_mO.data() + ((size_t)w0 * rs + p0) * PF_IEW;
                    long long terms = 0;
                    for (int u1 = 0; u1 <= std::min(w0, MAXLOOP) - 2; ++u1)
                        terms += __builtin_popcount(mw[u1] & low(std::min(w0 - u1 - 6, PF_IEW - 1)));
                    b_il += (double)lanes * (12.0 + 4.0 * terms);
                } else {
                    const int h = f1, j = f2, k = j + h + 2;
                    const int alo = std::max(2, t - (n - k)), ahi = std::min(t - 2, j - 1);
                    const int a0 = alo + ch * 64, a1 = std::min(ahi, a0 + 63);
                    const uint32_t *mw = c.h_mI.data() + ((size_t)(h + 2) * rs + j) * PF_IEW;
                    double lt = 0;
                    for (int u1 = 0; u1 <= std::min(a1 - 2, PF_IEW - 1); ++u1) {
                        uint32_t mk = mw[u1] & low(std::min(std::min(t - a0 - 2, PF_IEW - 1), t - 4 - u1));
                        while (mk) {
                            const int u2 = __builtin_ctz(mk);
                            mk &= mk - 1;
                            lt += std::max(0, std::min(a1, t - 2 - u2) - std::max(a0, u1 + 2) + 1);
                        }
                    }
                    b_il += 12.0 * (a1 - a0 + 1) + 4.0 * lt;
                }
            }
            il[t] = b_il;
            double b_lv = 0;
            for (int a = 0; a <= t; ++a) {
                const int b = t - a;
                const double split = (a >= 1 ? 11.0 * a - 6 : 0) + (b >= 1 ? 11.0 * b - 6 : 0) + 4.0 * (b >= 1) + (a >= 1);
                for (int h = 0; h < m; ++h)
                    for (int i = 1; i + h <= m; ++i) {
                        const int j = i + a, k = j + h + 2, l = k + b;
                        double r4 = split, by = 21.0 * 4;
                        if (c.ptype(i, j) > 0) {
                            const bool in = a >= 2;
                            by += (a >= 6 ? 8 : 0) + 4;  // R or the stack operand; the copy store
                            r4 += (a < 6 && in ? 1 : 0) + (in ? 2 : 0) + (in && j >= i + TURN + 1 ? 1 : 0);
                        }
                        if (c.ptype(k, l) > 0) {
                            const bool in = b >= 2;
                            by += (b >= 6 ? 8 : 0) + 4;
                            r4 += (b < 6 && in ? 1 : 0) + (in ? 2 : 0) + (in && l >= k + TURN + 1 ? 1 : 0);
                        }
                        const bool in11 = a >= 1 && b >= 1;
                        if (c.ptype(j, k) > 0) {
                            const bool rr = a >= 2 && b >= 2;
                            by += (rr ? 8 : 0) + 4;
                            r4 += (!rr && in11 ? 1 : 0) + (in11 ? 2 : 0) + (in11 && k >= j + TURN - 1 ? 1 : 0);
                        }
                        if (c.ptype(i, l) > 0) r4 += in11 ? 3 + (l >= i + TURN + 1 ? 1 : 0) : 0;
                        b_lv += 4.0 * r4 + by;
                    }
            }
            lv[t] = b_lv;
        }
    });
    for (int t = 0; t < n; ++t) {
        w.iloop += il[t];
        w.level += lv[t];
    }
    for (int s = 3; s <= n - 1; ++s)  // C(s,3) (j, d, k) triples per i, two 4-B operands each
        w.pterm += 8.0 * (n - s) * ((double)s * (s - 1) * (s - 2) / 6.0);
    for (int s = 0; s <= n - 1; ++s)
        for (int i = 1; i + s <= n; ++i) {
            const int j = i + s;
            double ops = 0;
            for (int k = i + 1; k <= std::min(j - TURN - 2, i + MAXLOOP + 1); ++k)
                ops += std::max(0, j - (std::max(k + TURN + 1 + MAXLOOP + 2, k + j - i) - MAXLOOP - 2));
            ops += 3.0 * std::max(0, j - TURN - 1 - i) * 2 + 2.0 * s * 3 * 2 + 4.0 * std::max(0, j - TURN - i) * 3;
            w.diag += 8.0 * ops;
        }
    return w;
}

int create_impl(const ccj_problem *prob, const ccj_pf_raw *raw, int device, ccj_pf_ctx *c) {
    if (!prob || !prob->seq || !prob->params) return pf_err(c, CCJ_E_ARG, "null problem");
    if (prob->params->magic != CCJ_PARAMS_MAGIC || prob->params->size_bytes != sizeof(ccj_energy_params))
        return pf_err(c, CCJ_E_ARG, "bad parameter blob");
    c->seq = prob->seq;
    c->n = (int)c->seq.size();
    const int n = c->n;
    if (n < 1) return pf_err(c, CCJ_E_ARG, "empty sequence");
    if (n > 1023) return pf_err(c, CCJ_E_ARG, "sequence longer than 1023");
    for (char ch : c->seq)
        if (!(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'U' || ch == 'T'))
            return pf_err(c, CCJ_E_ARG, "sequence must be A/C/G/U/T");
    c->dangles = prob->dangles;
    c->device = device;
    c->prm = *prob->params;
    const ccj_pk_penalties defp = CCJ_PK_PENALTIES_DEFAULT;
    c->pen = prob->pen ? *prob->pen : defp;
    c->rs = n + 2;
    const int rs = c->rs;
    {
        // Size check before any table is built (ccj_pf_footprint: the allocations below, summed).
        // Past what the host or the GPU can hold, fail with CCJ_E_OOM up front instead of after
        // seconds of table building.  CCJ_PF_DEVMEM_LIMIT (bytes) stands in for the device's free
        // memory (tests pin the accept/reject boundary with it).
        unsigned long long dev_b = 0, host_b = 0;
        ccj_pf_footprint(n, &dev_b, &host_b);
        size_t dfree = 0, dtotal = 0;
        char msg[200];
        const char *lim = getenv("CCJ_PF_DEVMEM_LIMIT");
        if (lim && *lim) dfree = (size_t)strtoull(lim, nullptr, 10);
        else if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&dfree, &dtotal) != hipSuccess) dfree = SIZE_MAX;
        if ((double)dev_b > (double)dfree) {
            snprintf(msg, sizeof msg, "n=%d needs ~%.1f GB of device memory, %.1f GB free", n, dev_b / 1e9, dfree / 1e9);
            return pf_err(c, CCJ_E_OOM, msg);
        }
        // MemAvailable counts reclaimable page cache (sysconf(_SC_AVPHYS_PAGES) does not)
        unsigned long long avail_kb = 0;
        if (FILE *f = fopen("/proc/meminfo", "r")) {
            char line[256];
            while (fgets(line, sizeof line, f))
                if (sscanf(line, "MemAvailable: %llu kB", &avail_kb) == 1) break;
            fclose(f);
        }
        if (avail_kb > 0 && (double)host_b > (double)avail_kb * 1024.0) {
            snprintf(msg, sizeof msg, "n=%d needs ~%.1f GB of host memory for the interior-loop tables", n, host_b / 1e9);
            return pf_err(c, CCJ_E_OOM, msg);
        }
    }
    // make_pair_matrix / encode_sequence (pair_mat.h:81-183)
    const int base_rtype[8] = {0, 2, 1, 4, 3, 6, 5, 7};
    memcpy(c->rtype, base_rtype, sizeof base_rtype);
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) c->pair[x][y] = BP_PAIR_PF[x][y];
    if (prob->noGU) c->pair[3][4] = c->pair[4][3] = 0;
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) c->rtype[c->pair[x][y]] = c->pair[y][x];
    c->S.assign(n + 2, 0);
    c->S1.assign(n + 2, 0);
    for (int i = 1; i <= n; ++i) c->S[i] = c->S1[i] = (short)encode_base(c->seq[i - 1]);
    c->S[n + 1] = c->S[1];
    c->S[0] = (short)n;
    c->S1[n + 1] = c->S1[1];
    c->S1[0] = c->S1[n];

    if (raw && (raw->magic != CCJ_PF_RAW_MAGIC || raw->size_bytes != sizeof(ccj_pf_raw)))
        return pf_err(c, CCJ_E_ARG, "bad ccj_pf_raw table");
    build_exp(c->prm, raw, c->pen, c->E);
    // exp_params_rescale (part_func.cc:97-125), pf_scale == 1 so every scale[] is 1
    c->mlb.assign(n + 2, 0);
    c->cpp.assign(n + 2, 0);
    c->pup.assign(n + 2, 0);
    c->mlb[0] = 1;
    c->mlb[1] = c->E.MLbase / 1.;
    c->cpp[0] = 1;
    c->cpp[1] = c->E.cp / 1.;
    c->pup[0] = 1;
    c->pup[1] = c->E.PUP / 1.;
    for (int i = 2; i <= n; ++i) {
        c->mlb[i] = pow(c->E.MLbase, (double)i) * 1.;
        c->cpp[i] = pow(c->E.cp, (double)i) * 1.;
        c->pup[i] = pow(c->E.PUP, (double)i) * 1.;
    }

    // per-sequence tables
    const size_t plane = c->plane();
    std::vector<int8_t> pt(plane, 0);
    c->hp.assign(plane, 0);
    std::vector<double> est(plane, 0);
    for (int w = 0; w <= n - 1; ++w)
        for (int p = 1; p + w <= n; ++p) {
            const size_t ix = (size_t)w * rs + p;
            pt[ix] = (int8_t)c->ptype(p, p + w);
            c->hp[ix] = hairpin_pf(*c, p, p + w);
            // get_e_stP (part_func.cc:877-884); w == 0 is never read with a nonzero factor
            if (w >= 1 && w != 2) est[ix] = pow(compute_int_pf(*c, p, p + w, p + 1, p + w - 1), c->pen.e_stP);
        }
    // ieO / ieI: get_e_intP by outer / inner pair, each pair's 29 x 29 window contiguous
    constexpr int W2 = PF_IEW * PF_IEW;
    const size_t ie_n = (size_t)W2 * plane;
    std::vector<double> ie(ie_n, 0.0), ieI(ie_n, 0.0);
    {
        const int nthr = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        run_threads(n, nthr, [&](int w0, int w1) {
            for (int w = w0; w < w1; ++w)
                for (int p = 1; p + w <= n; ++p) {
                    const int q = p + w;
                    for (int u1 = 0; u1 < PF_IEW; ++u1)
                        for (int u2 = 0; u2 < PF_IEW; ++u2) {
                            const int ip = p + 1 + u1, jp = q - 1 - u2;
                            if (ip >= jp || (u1 == 0 && u2 == 0)) continue;  // get_e_intP's stack case is 0
                            ie[((size_t)w * rs + p) * W2 + u1 * PF_IEW + u2] =
                                pow(compute_int_pf(*c, p, q, ip, jp), c->pen.e_intP);
                        }
                }
        });
        // ieI[g][j][u1][u2] = ieO[g+2+u1+u2][j-1-u1][u1][u2] (closing (j-1-u1, j+g+1+u2))
        run_threads(n, nthr, [&](int g0, int g1) {
            for (int g = g0; g < g1; ++g)
                for (int j = 1; j + g <= n; ++j)
                    for (int u1 = 0; u1 < PF_IEW; ++u1)
                        for (int u2 = 0; u2 < PF_IEW; ++u2) {
                            const int p = j - 1 - u1, w = g + 2 + u1 + u2;
                            if (p < 1 || p + w > n) continue;
                            ieI[((size_t)g * rs + j) * W2 + u1 * PF_IEW + u2] = ie[((size_t)w * rs + p) * W2 + u1 * PF_IEW + u2];
                        }
        });
    }
    // window masks: a term adds nothing when its weight is 0.0 or the pair of the 4-D value it reads
    // cannot pair (that value is 0): mO over (p+1+u1, p+w-1-u2), mI over (j-1-u1, j+g+1+u2)
    std::vector<uint32_t> mO(plane * PF_IEW, 0u), mI(plane * PF_IEW, 0u);
    for (int w = 0; w <= n - 1; ++w)
        for (int p = 1; p + w <= n; ++p)
            for (int u1 = 0; u1 < PF_IEW; ++u1) {
                const size_t r = ((size_t)w * rs + p) * PF_IEW + u1;
                for (int u2 = 0; u2 < PF_IEW; ++u2) {
                    const size_t e = ((size_t)w * rs + p) * W2 + u1 * PF_IEW + u2;
                    {   // outer (p, p+w)
                        const int ip = p + 1 + u1, jp = p + w - 1 - u2;
                        if (ip < jp && ie[e] != 0.0 && c->ptype(ip, jp) > 0) mO[r] |= 1u << u2;
                    }
                    {   // inner (p, p+w) = (j, j+g)
                        const int d = p - 1 - u1, dp = p + w + 1 + u2;
                        if (d >= 1 && dp <= n && ieI[e] != 0.0 && c->ptype(d, dp) > 0) mI[r] |= 1u << u2;
                    }
                }
            }

    // level layout
    c->lv.assign(std::max(n - 2, 1), PfLvl{0, 0, 0, 0, 0, 0, 0});
    long long off = 0, offx = 0, offm = 0, maxC = 1;
    for (int t = 0; t <= n - 3; ++t) {
        const long long m = n - t - 2, M = m * (m + 1) / 2;
        c->lv[t] = PfLvl{off, (t + 1) * M, (int)M, 0, offx, offm, c->cells};
        off += (long long)PF_NMAT4 * (t + 1) * M;
        offx += 2 * (t + 1) * M;
        offm += m * n * (t + 1);
        maxC = std::max(maxC, (t + 1) * M);
        c->cells += (t + 1) * M;
    }
    // k_pf_ppush addresses the PK rows of PF_PP_S consecutive levels as 32-bit byte offsets from the
    // lowest one's PK start (one buffer resource per wave): that span must stay below 4 GB
    for (int t = 0; t <= n - 3; ++t) {
        const int tt = std::min(t + PF_PP_S - 1, n - 3);
        const long long lo = c->lv[t].lb + PF_PK * c->lv[t].C, hi = c->lv[tt].lb + PF_PK * c->lv[tt].C + c->lv[tt].C;
        if (4 * (hi - lo) >= (1LL << 32)) return pf_err(c, CCJ_E_ARG, "n too large: the PK rows of 8 levels exceed 4 GB (k_pf_ppush offsets)");
    }
    // k_pf_iloop work items: the cells of each pairing closing pair in 64-lane chunks, encoded as
    // ccj_items.h's (unsharded).  PL and PR rows are the MFE engine's; PM rows here start at h = 0,
    // since get_PMiloop has no hairpin bound on (j, k) (part_func.cc:804-824)
    std::vector<uint32_t> items;
    c->ifirst.assign(std::max(n - 1, 2), 0);
    {
        struct PT {
            const int8_t *p;
            int rs;
            int operator()(int i, int j) const { return p[(size_t)(j - i) * rs + i]; }
        } ptf{pt.data(), rs};
        for (int t = 0; t <= n - 3; ++t) {
            c->ifirst[t] = (long long)items.size();
            const ItemRows R = item_rows(n, t, 1, 0);
            for (int x = 0; x < R.nPL + R.nPR; ++x) {
                uint32_t it0 = 0;
                const int cnt = item_row(ptf, n, t, R, x, 1, 0, it0);
                for (int q = 0; q < cnt; ++q) items.push_back(it0 | (uint32_t)q);
            }
            for (int h = 0; h <= R.m - 1; ++h)  // PM: pair (j, k = j+h+2), lanes a in [alo, ahi]
                for (int j = 1; j + h + 2 <= n; ++j) {
                    const int k = j + h + 2, alo = std::max(2, t - (n - k)), ahi = std::min(t - 2, j - 1);
                    if (alo > ahi || ptf(j, k) <= 0) continue;
                    const uint32_t it0 = (2u << 30) | ((uint32_t)h << 20) | ((uint32_t)j << 10);
                    for (int q = 0; q <= (ahi - alo) / 64; ++q) items.push_back(it0 | (uint32_t)q);
                }
        }
        c->ifirst[std::max(n - 2, 1)] = (long long)items.size();
    }

    // device
    PFCHK(c, hipSetDevice(device));
    PFCHK(c, hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    PFCHK(c, hipStreamCreateWithFlags(&c->st_il, hipStreamNonBlocking));
    PFCHK(c, hipStreamCreateWithFlags(&c->st_d, hipStreamNonBlocking));
    PFCHK(c, hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    for (auto *v : {&c->ev_lev, &c->ev_il, &c->ev_dg}) {
        v->assign(n + 1, nullptr);
        for (hipEvent_t &e : *v) PFCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    PFCHK(c, hipEventCreate(&c->e0));
    PFCHK(c, hipEventCreate(&c->e1));
    auto up = [&](void **d, const void *h, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(d, bytes ? bytes : 8);
        if (e != hipSuccess) return e;
        return bytes ? hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) : hipSuccess;
    };
    int8_t pair8[64], rt8[8];
    for (int x = 0; x < 8; ++x) {
        rt8[x] = (int8_t)c->rtype[x];
        for (int y = 0; y < 8; ++y) pair8[x * 8 + y] = (int8_t)c->pair[x][y];
    }
    PFCHK(c, up((void **)&c->d_E, &c->E, sizeof(PfExp)));
    PFCHK(c, up((void **)&c->d_S, c->S.data(), c->S.size() * sizeof(short)));
    PFCHK(c, up((void **)&c->d_S1, c->S1.data(), c->S1.size() * sizeof(short)));
    PFCHK(c, up((void **)&c->d_pt, pt.data(), pt.size()));
    PFCHK(c, up((void **)&c->d_pair, pair8, 64));
    PFCHK(c, up((void **)&c->d_rtype, rt8, 8));
    PFCHK(c, up((void **)&c->d_hp, c->hp.data(), plane * sizeof(double)));
    PFCHK(c, up((void **)&c->d_est, est.data(), plane * sizeof(double)));
    // k_pf_iloop reads the weights of a window row only at the row's mask bits, in ascending order:
    // store them compacted (k-th set bit -> slot k), so that a round's weights are one scalar load;
    // PF_ILW zero doubles of tail padding cover the last row's round-wide reads
    auto compact = [&](std::vector<double> &v, const std::vector<uint32_t> &mk) {
        for (size_t r = 0; r < mk.size(); ++r) {
            double *row = v.data() + r * PF_IEW;
            int k = 0;
            for (int u2 = 0; u2 < PF_IEW; ++u2)
                if (mk[r] >> u2 & 1u) row[k++] = row[u2];
            for (; k < PF_IEW; ++k) row[k] = 0.0;
        }
        v.resize(v.size() + PF_ILW, 0.0);
    };
    compact(ie, mO);
    compact(ieI, mI);
    PFCHK(c, up((void **)&c->d_ieO, ie.data(), ie.size() * sizeof(double)));
    PFCHK(c, up((void **)&c->d_ieI, ieI.data(), ieI.size() * sizeof(double)));
    PFCHK(c, up((void **)&c->d_items, items.data(), items.size() * sizeof(uint32_t)));
    PFCHK(c, up((void **)&c->d_mO, mO.data(), mO.size() * sizeof(uint32_t)));
    PFCHK(c, up((void **)&c->d_mI, mI.data(), mI.size() * sizeof(uint32_t)));
    c->h_items = std::move(items);
    c->h_mO = std::move(mO);
    c->h_mI = std::move(mI);
    PFCHK(c, up((void **)&c->d_mlb, c->mlb.data(), c->mlb.size() * sizeof(double)));
    PFCHK(c, up((void **)&c->d_cpp, c->cpp.data(), c->cpp.size() * sizeof(double)));
    PFCHK(c, up((void **)&c->d_pup, c->pup.data(), c->pup.size() * sizeof(double)));
    PFCHK(c, up((void **)&c->d_ld, c->lv.data(), c->lv.size() * sizeof(PfLvl)));
    PFCHK(c, hipMalloc((void **)&c->d_2d, (size_t)CCJ_PF_NMAT2 * plane * sizeof(double)));
    PFCHK(c, hipMalloc((void **)&c->d_Pacc, plane * sizeof(long long)));
    PFCHK(c, hipMalloc((void **)&c->d_Pabs, plane * sizeof(unsigned long long)));
    PFCHK(c, hipMalloc((void **)&c->d_d4, (size_t)std::max(off, 1LL) * sizeof(int)));
    PFCHK(c, hipMalloc((void **)&c->d_prec, (size_t)PF_RECS * std::max(c->cells, 1LL) * sizeof(int)));
    // the copies stay 0 where the pair cannot pair (never written): set once per context
    PFCHK(c, hipMalloc((void **)&c->d_cx, (size_t)std::max(offx, 1LL) * sizeof(int)));
    PFCHK(c, hipMalloc((void **)&c->d_pmx, (size_t)std::max(offm, 1LL) * sizeof(int)));
    PFCHK(c, hipMemset(c->d_cx, 0, (size_t)std::max(offx, 1LL) * sizeof(int)));
    PFCHK(c, hipMemset(c->d_pmx, 0, (size_t)std::max(offm, 1LL) * sizeof(int)));
    PFCHK(c, hipMalloc((void **)&c->d_R, (size_t)2 * 3 * maxC * sizeof(double)));
    c->D.Rst = 3 * maxC;

    PfDev &D = c->D;
    D.n = n;
    D.rs = rs;
    D.dangles = c->dangles;
    D.ap_int = c->pen.ap;
    D.E = c->d_E;
    D.S = c->d_S;
    D.S1 = c->d_S1;
    D.pt = c->d_pt;
    D.pair = c->d_pair;
    D.rtype = c->d_rtype;
    D.hp = c->d_hp;
    D.est = c->d_est;
    D.ieO = c->d_ieO;
    D.ieI = c->d_ieI;
    D.mO = c->d_mO;
    D.mI = c->d_mI;
    D.mlb = c->d_mlb;
    D.cpp = c->d_cpp;
    D.pup = c->d_pup;
    double *pl[CCJ_PF_NMAT2];
    for (int m = 0; m < CCJ_PF_NMAT2; ++m) pl[m] = c->d_2d + (size_t)m * plane;
    D.V = pl[CCJ_PF_V];
    D.VM = pl[CCJ_PF_VM];
    D.WM = pl[CCJ_PF_WM];
    D.WMv = pl[CCJ_PF_WMv];
    D.WMp = pl[CCJ_PF_WMp];
    D.WBP = pl[CCJ_PF_WBP];
    D.WPP = pl[CCJ_PF_WPP];
    D.P = pl[CCJ_PF_P];
    D.Pacc = c->d_Pacc;
    D.Pabs = c->d_Pabs;
    D.d4 = c->d_d4;
    D.r1 = c->d_prec;
    D.r2 = D.r1 + (size_t)PF_REC1 * c->cells;
    D.r3 = D.r2 + (size_t)PF_REC2 * c->cells;
    D.r4 = D.r3 + (size_t)PF_REC3 * c->cells;
    D.cx = c->d_cx;
    D.pmx = c->d_pmx;
    D.items = c->d_items;
    D.R = c->d_R;
    D.ld = c->d_ld;
    return CCJ_OK;
}

int fill_impl(ccj_pf_ctx *c) {
    const int n = c->n;
    const size_t plane = c->plane();
    c->filled = false;  // a failed re-fill must not leave the previous fill's tables looking valid
    PFCHK(c, hipSetDevice(c->device));
    PFCHK(c, hipMemsetAsync(c->d_2d, 0, (size_t)CCJ_PF_NMAT2 * plane * sizeof(double), c->st));
    PFCHK(c, hipMemsetAsync(c->d_Pacc, 0, plane * sizeof(long long), c->st));
    PFCHK(c, hipMemsetAsync(c->d_Pabs, 0, plane * sizeof(unsigned long long), c->st));
    PFCHK(c, hipEventRecord(c->e0, c->st));
    // level t needs the 2-D spans <= t-1; span s needs P(s), i.e. the levels <= s-3
    // timed launches: an event pair from the context's pool around each (ccj_pf_set_timing)
    c->tfam.clear();
    auto launch = [&](int fam, hipStream_t s, auto &&go) -> hipError_t {
        const size_t q = c->tfam.size();
        if (c->timing) {
            while (c->tev.size() < 2 * q + 2) {
                hipEvent_t e;
                const hipError_t r = hipEventCreate(&e);
                if (r != hipSuccess) return r;
                c->tev.push_back(e);
            }
            c->tfam.push_back(fam);
            const hipError_t r = hipEventRecord(c->tev[2 * q], s);
            if (r != hipSuccess) return r;
        }
        const hipError_t e = (hipError_t)go();
        if (e != hipSuccess || !c->timing) return e;
        return hipEventRecord(c->tev[2 * q + 1], s);
    };
    // Three streams: level t needs k_pf_iloop(t) and the spans <= t-1; k_pf_iloop(t)
    // reads the copies of levels <= t-2 and refills the R buffer level t-2 read; P(s) needs the
    // levels <= s-3 and span s the spans < s.  So iloop(t) and the span s = t+1 (with its P terms)
    // run beside level t-1, off the level chain.  Every event is recorded before a wait on it is
    // enqueued (host order below).
    const int nl = n - 2;  // levels 0 .. n-3
    // P(s): pushed by level (k_pf_ppush(s-3) completes it, after every earlier push on this stream),
    // or pulled per span (k_pf_pterm, CCJ_PF_PULL=1)
    const bool pull = getenv("CCJ_PF_PULL") && atoi(getenv("CCJ_PF_PULL")) != 0;
    auto span = [&](int s) -> hipError_t {
        hipError_t e = launch(2, c->st_d, [&] {
            return pull ? ccjk_pf_pterm(&c->D, s, c->st_d) : s >= 3 ? ccjk_pf_ppush(&c->D, s - 3, c->st_d) : 0;
        });
        if (e == hipSuccess) e = launch(3, c->st_d, [&] { return ccjk_pf_diag(&c->D, s, c->st_d); });
        return e != hipSuccess ? e : hipEventRecord(c->ev_dg[s], c->st_d);
    };
    auto iloop = [&](int t) -> hipError_t {
        const long long f = c->ifirst[t];
        const hipError_t e = launch(0, c->st_il, [&] { return ccjk_pf_iloop(&c->D, t, f, (int)(c->ifirst[t + 1] - f), c->st_il); });
        return e != hipSuccess ? e : hipEventRecord(c->ev_il[t], c->st_il);
    };
    PFCHK(c, hipEventRecord(c->ev_start, c->st));
    PFCHK(c, hipStreamWaitEvent(c->st_d, c->ev_start, 0));
    PFCHK(c, hipStreamWaitEvent(c->st_il, c->ev_start, 0));
    for (int s = 0; s <= std::min(2, n - 1); ++s) PFCHK(c, span(s));   // no P terms below span 3
    for (int t = 0; t <= std::min(1, nl - 1); ++t) PFCHK(c, iloop(t));
    for (int t = 0; t < nl; ++t) {
        PFCHK(c, hipStreamWaitEvent(c->st, c->ev_il[t], 0));
        if (t >= 1) PFCHK(c, hipStreamWaitEvent(c->st, c->ev_dg[t - 1], 0));
        PFCHK(c, launch(1, c->st, [&] { return ccjk_pf_level(&c->D, c->lv.data(), t, c->st); }));
        PFCHK(c, hipEventRecord(c->ev_lev[t], c->st));
        if (t + 2 < nl) {
            PFCHK(c, hipStreamWaitEvent(c->st_il, c->ev_lev[t], 0));
            PFCHK(c, iloop(t + 2));
        }
        if (t + 3 <= n - 1) {
            PFCHK(c, hipStreamWaitEvent(c->st_d, c->ev_lev[t], 0));
            PFCHK(c, span(t + 3));
        }
    }
    PFCHK(c, hipStreamWaitEvent(c->st, c->ev_dg[n - 1], 0));
    PFCHK(c, hipEventRecord(c->e1, c->st));
    c->h2d.assign((size_t)CCJ_PF_NMAT2 * plane, 0.0);
    PFCHK(c, hipMemcpyAsync(c->h2d.data(), c->d_2d, c->h2d.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
    std::vector<unsigned long long> pabs(plane, 0);
    PFCHK(c, hipMemcpyAsync(pabs.data(), c->d_Pabs, plane * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->st));
    PFCHK(c, hipStreamSynchronize(c->st));
    // the exact int64 P sums equal the reference's serial double sums only while every partial sum
    // is an exactly representable integer: guaranteed by sum |term| < 2^53 (part_func.cc:383-393)
    // CCJ_PF_RANGE_LOG2 lowers the 2^53 bound (tests only: reaches this exit with short sequences)
    unsigned long long range_lim = 1ull << 53;
    if (const char *e = getenv("CCJ_PF_RANGE_LOG2")) {
        const int l2 = atoi(e);
        if (l2 >= 1 && l2 <= 53) range_lim = 1ull << l2;
    }
    for (int w = 0; w < n; ++w)
        for (int p = 1; p + w <= n; ++p)
            if (pabs[(size_t)w * c->rs + p] >= range_lim) {
                char msg[160];
                snprintf(msg, sizeof msg, "P(%d,%d): sum of |terms| >= 2^53, the reference's double sum may round", p, p + w);
                return pf_err(c, CCJ_E_PF_RANGE, msg);
            }
    PFCHK(c, hipEventElapsedTime(&c->fill_ms, c->e0, c->e1));
    for (double &k : c->kms) k = 0;
    for (size_t q = 0; q < c->tfam.size(); ++q) {
        float ms = 0;
        PFCHK(c, hipEventElapsedTime(&ms, c->tev[2 * q], c->tev[2 * q + 1]));
        c->kms[c->tfam[q]] += ms;
    }

    // W (part_func.cc:163-172)
    c->W.assign(n + 1, 1.0);  // W.resize(n+1, scale[1])
    for (int j = TURN + 1; j <= n; ++j) {
        double s = 0;
        s += c->W[j - 1] * 1.0;
        for (int k = 1; k <= j - TURN - 1; ++k) {
            const double acc = (k > 1) ? c->W[k - 1] : 1;
            s += acc * c->g2(CCJ_PF_V, k, j) * ext_pf(*c, k, j);
            s += acc * c->g2(CCJ_PF_P, k, j) * c->E.PS;
        }
        c->W[j] = s;
    }
    // to_Energy (part_func.cc:148-150)
    c->energy = (-log(c->W[n]) - n * log(c->E.pf_scale)) * c->E.kT / 1000.0;
    c->filled = true;
    return CCJ_OK;
}

// ---------------------------------------------------------------------------------------------
// Stochastic traceback (stoch_backtrack.cc).  Each failure path of the reference prints a line and
// calls exit(0); here it is reported as CCJ_E_PF_SAMPLE with that line in ccj_pf_last_message.
// ---------------------------------------------------------------------------------------------
struct Sampler {
    ccj_pf_ctx &c;
    std::string &st;
    bool failed = false;

    double urn() {  // vrna_urn (utils.c:262-271) without HAVE_ERAND48
        int32_t r = 0;
        random_r(&c.rnd, &r);
        return ((double)r) / RAND_MAX;
    }
    double V(int i, int j) const { return c.g2(CCJ_PF_V, i, j); }
    double VM(int i, int j) const { return c.g2(CCJ_PF_VM, i, j); }
    double WM(int i, int j) const { return c.g2(CCJ_PF_WM, i, j); }
    double WMv(int i, int j) const { return c.g2(CCJ_PF_WMv, i, j); }
    double WMp(int i, int j) const { return c.g2(CCJ_PF_WMp, i, j); }
    double P(int i, int j) const { return c.g2(CCJ_PF_P, i, j); }
    void fail(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c.msg = buf;
        failed = true;
    }

    // boustrophedon (stoch_backtrack.cc:17-34)
    static std::vector<int> bous(int start, int end) {
        std::vector<int> s;
        if (end >= start) {
            s.push_back(end - start + 1);
            for (int pos = 1; pos <= end - start + 1; ++pos) {
                const int count = pos - 1, adv = count / 2;
                s.push_back(start + (end - start) * (count % 2) + adv - (2 * (count % 2)) * adv);
            }
        }
        return s;
    }

    void W_(int start, int end) {  // :36-85
        if (failed) return;
        int j = end, m;
        double W_temp = 0;
        const std::vector<double> &W = c.W;
        if (end > start) {
            for (; j > start; --j) {
                W_temp = W[j - 1] * 1.0;
                const double r = urn() * W[j];
                if (r > W_temp) break;
            }
            if (j <= start + TURN) return;
            const double r = urn() * (W[j] - W_temp);
            const std::vector<int> is = bous(start, j - 1);
            const int bn = (int)is.size();
            double qt = 0;
            int k = start;
            bool pk = false;
            for (m = 1; m < bn; ++m) {
                k = is[m];
                const double acc = (k > 1) ? W[k - 1] : 1;
                double Wkl = acc * V(k, j) * ext_pf(c, k, j);
                qt += Wkl;
                if (qt > r) break;
                Wkl = acc * P(k, j) * c.E.PS;
                qt += Wkl;
                if (qt > r) {
                    pk = true;
                    break;
                }
            }
            if (k + start > j) {
                fail("backtracking failed in ext loop at %d and %d with W[j] = %f, qt:%f < r:%f\n", start, end, W[j], qt, r);
                return;
            }
            W_(start, k - 1);
            if (failed) return;
            if (!pk) V_(k, j);
            // else Sample_P (:323-326) is empty
        }
    }

    void V_(int i, int j) {  // :87-141
        if (failed) return;
        int k = i, l = j;
        st[i - 1] = '(';
        st[j - 1] = ')';
        const double qbr = V(i, j);
        const double r = urn() * qbr;
        double qbt1 = 0, V_temp = hairpin_pf(c, i, j);
        qbt1 += V_temp;
        if (qbt1 >= r) return;
        const int max_k = std::min(j - TURN - 2, i + MAXLOOP + 1);
        // stoch_backtrack.cc:112,119 read `pair` of ViennaRNA/pair_mat.h, a static array every
        // translation unit owns; only part_func.cc's copy is filled (make_pair_matrix in the
        // constructor), so here every pair type is 0 and rtype[0] is 0.
        const int tc = 0, t2 = 0;
        for (k = i + 1; k <= max_k; k++) {
            const int min_l = std::max(k + TURN + 1 + MAXLOOP + 2, k + j - i) - MAXLOOP - 2;
            for (l = j - 1; l >= min_l; --l) {
                const int u1 = k - i - 1, u2 = j - l - 1;
                V_temp = V(k, l) * exp_E_IntLoop_pf(c.E, u1, u2, tc, t2, c.S1[i + 1], c.S1[j - 1], c.S1[k - 1], c.S1[l + 1]);
                V_temp *= 1.0;
                qbt1 += V_temp;
                if (qbt1 >= r) break;
            }
            if (qbt1 >= r) break;
        }
        if (qbt1 >= r) {
            V_(k, l);
            return;
        }
        V_temp = VM(i, j);
        qbt1 += V_temp;
        if (qbt1 < r) {
            fail("Backtracking failed for pair (%d,%d)\n", i, j);
            return;
        }
        VM_(i, j);
    }

    void VM_(int i, int j) {  // :143-192
        if (failed) return;
        int k;
        double qt = 0;
        if ((i + 1) + 2 * TURN + 2 >= (j - 1)) {
            fail("backtracking impossible for VM[%d, %d]\n", i, j);
            return;
        }
        double V_temp;
        const double VM_inside = VM(i, j) / 1.0;
        const double r = urn() * VM_inside;
        bool unpaired = false, pk = false;
        const double mb = mbloop_pf(c, i, j), mc = c.E.MLclosing;
        for (k = i + 1; k <= j - TURN - 1; ++k) {
            V_temp = WM(i + 1, k - 1) * WMv(k, j - 1) * mb * mc;
            qt += V_temp;
            if (qt > r) break;
            V_temp = (WM(i + 1, k - 1) * WMp(k, j - 1) * mb * mc);
            qt += V_temp;
            if (qt > r) {
                pk = true;
                break;
            }
            V_temp = (c.mlb[k - i - 1] * WMp(k, j - 1) * mb * mc);
            qt += V_temp;
            if (qt > r) {
                unpaired = true;
                pk = true;
                break;
            }
        }
        if (k > j - TURN) {
            fail("backtracking failed for VM at i=%d and j =%d\n", i, j);
            return;
        }
        if (!unpaired) WM_(i + 1, k - 1);
        if (failed) return;
        if (!pk) WMv_(k, j - 1);
        else WMp_(k, j - 1);
    }

    void WM_(int i, int j) {  // :193-272
        if (failed) return;
        int k;
        double qt = 0, qbt1 = 0, qbt2 = 0, V_temp = 0;
        bool unpaired = false, pk = false;
        if (i + TURN >= j) {
            fail("backtracking impossible for WM[%u, %u]\n", (unsigned)i, (unsigned)j);
            return;
        }
        for (; j > i + TURN; --j) {
            const double r = urn() * (WM(i, j));
            V_temp = WM(i, j - 1) * c.mlb[1];
            qt = V_temp;
            if (r > qt) break;
        }
        if (i + TURN == j) {
            fail("backtracking failed for WM\n");
            return;
        }
        qt = 0.;
        const double qm_rem = WM(i, j) - V_temp;
        const double r = urn() * qm_rem;
        for (k = i; k < j - TURN; ++k) {
            qbt1 = V(k, j) * mlstem_pf(c, k, j);
            qbt2 = P(k, j) * c.E.PSM * c.E.b;
            V_temp = c.mlb[k - i] * qbt1;
            qt += V_temp;
            if (qt >= r) {
                unpaired = true;
                break;
            }
            V_temp = c.mlb[k - i] * qbt2;
            qt += V_temp;
            if (qt >= r) {
                unpaired = true;
                pk = true;
                break;
            }
            V_temp = WM(i, k - 1) * qbt1;
            qt += V_temp;
            if (qt >= r) break;
            V_temp = WM(i, k - 1) * qbt2;
            qt += V_temp;
            if (qt >= r) {
                pk = true;
                break;
            }
        }
        if (k > j - TURN || qt < r) {
            fail("backtracking failed for WM at i=%d and j =%d with k=%d, qt=%f and r =%f and qt<r=%d\n", i, j, k, qt, r,
                 qt < r);
            return;
        }
        if (!unpaired) WM_(i, k - 1);
        if (failed) return;
        if (!pk) V_(k, j);
    }

    void WMv_(int i, int j) {  // :273-296
        if (failed) return;
        double qt = 0, V_temp = 0;
        (void)qt;
        for (; j > i + TURN; --j) {
            const double r = urn() * WMv(i, j);
            V_temp = WMv(i, j - 1) * c.mlb[1];
            qt = V_temp;
            if (r > qt) break;
        }
        if (i + TURN == j) {
            fail("backtracking failed for WMV\n");
            return;
        }
        V_(i, j);
    }

    void WMp_(int i, int j) {  // :298-321
        if (failed) return;
        double qt = 0, V_temp = 0;
        (void)qt;
        for (; j > i + TURN; --j) {
            const double r = urn() * WMp(i, j);
            V_temp = WMp(i, j - 1) * c.mlb[1];
            qt = V_temp;
            if (r > qt) break;
        }
        if (i + TURN == j) {
            fail("backtracking failed for WMP\n");
            return;
        }
        // Sample_P(i, j) is empty (:323-326)
    }
};

int exp_hashes(const PfExp &P, const ccj_energy_params &prm, uint64_t *out);

}  // namespace

extern "C" {

int ccj_pf_create(const ccj_problem *prob, const ccj_pf_raw *raw, int device, ccj_pf_ctx **out) {
    if (!out) return CCJ_E_ARG;
    *out = nullptr;
    ccj_pf_ctx *c = new (std::nothrow) ccj_pf_ctx();
    if (!c) return CCJ_E_OOM;
    initstate_r(1, c->rnd_state, sizeof c->rnd_state, &c->rnd);
    int rc;
    try {
        rc = create_impl(prob, raw, device, c);
    } catch (const std::bad_alloc &) {  // host tables: no exception crosses the C ABI
        rc = pf_err(c, CCJ_E_OOM, "host allocation failed");
    }
    if (rc != CCJ_OK) {
        fprintf(stderr, "ccj_pf_create: %s\n", c->msg.c_str());
        free_dev(c);
        delete c;
        return rc;
    }
    *out = c;
    return CCJ_OK;
}

void ccj_pf_destroy(ccj_pf_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    free_dev(c);
    delete c;
}

int ccj_pf_fill(ccj_pf_ctx *c, double *energy) {
    if (!c) return CCJ_E_ARG;
    const int rc = fill_impl(c);
    if (rc != CCJ_OK) return rc;
    if (energy) *energy = c->energy;
    return CCJ_OK;
}

int ccj_pf_W(ccj_pf_ctx *c, double *W) {
    if (!c || !W) return CCJ_E_ARG;
    if (!c->filled) return CCJ_E_STATE;
    memcpy(W, c->W.data(), c->W.size() * sizeof(double));
    return CCJ_OK;
}

int ccj_pf_get2(ccj_pf_ctx *c, int which, double *out) {
    if (!c || !out || which < 0 || which >= CCJ_PF_NMAT2) return CCJ_E_ARG;
    if (!c->filled) return CCJ_E_STATE;
    size_t q = 0;
    for (int i = 1; i <= c->n; ++i)
        for (int j = i; j <= c->n; ++j) out[q++] = c->g2(which, i, j);
    return CCJ_OK;
}

int ccj_pf_get4(ccj_pf_ctx *c, int x, int i, int j, int k, int l, int *out) {
    if (!c || !out || x < 0 || x >= CCJ_PF_NMAT4) return CCJ_E_ARG;
    if (!c->filled) return CCJ_E_STATE;
    if (!(i <= j && j < k - 1 && k <= l)) {  // Matrix4DPF::get (matrices.hh:258-263)
        *out = 0;
        return CCJ_OK;
    }
    if (i <= 0 || l > c->n) return CCJ_E_ARG;  // the reference's get_uc assert
    const int a = j - i, b = l - k, t = a + b, h = k - j - 2, m = c->n - t - 2;
    const PfLvl &L = c->lv[t];
    const long long off = L.lb + (long long)x * L.C + (long long)a * L.M + h * m - ((h * (h - 1)) >> 1) + i - 1;
    PFCHK(c, hipSetDevice(c->device));
    PFCHK(c, hipMemcpy(out, c->d_d4 + off, sizeof(int), hipMemcpyDeviceToHost));
    return CCJ_OK;
}

int ccj_pf_hashes(ccj_pf_ctx *c, uint64_t *h4, uint64_t *h2) {
    if (!c) return CCJ_E_ARG;
    if (!c->filled) return CCJ_E_STATE;
    const int n = c->n;
    if (h2) {
        for (int m = 0; m < CCJ_PF_NMAT2; ++m) {
            uint64_t h = fnv_init();
            for (int i = 1; i <= n; ++i)
                for (int j = i; j <= n; ++j) {
                    const double v = c->g2(m, i, j);
                    fnv_bytes(h, &v, 8);
                }
            h2[m] = h;
        }
    }
    if (h4) {
        // canonical (i, j, k) rows of l, gathered on the GPU
        std::vector<long long> rows;
        long long q = 0;
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j)
                for (int k = j + 2; k <= n; ++k) {
                    rows.push_back(q);
                    rows.push_back(((long long)i << 40) | ((long long)j << 20) | k);
                    q += n - k + 1;
                }
        const int nrows = (int)(rows.size() / 2);
        long long *d_rows = nullptr;
        int *d_out = nullptr;
        PFCHK(c, hipSetDevice(c->device));
        PFCHK(c, hipMalloc((void **)&d_rows, std::max<size_t>(rows.size(), 1) * sizeof(long long)));
        hipError_t e = hipMalloc((void **)&d_out, std::max<long long>(q, 1) * sizeof(int));
        if (e != hipSuccess) {
            hipFree(d_rows);
            return pf_err(c, CCJ_E_OOM, "hash buffer", e);
        }
        std::vector<int> hbuf((size_t)std::max<long long>(q, 1));
        int rc = CCJ_OK;
        if ((e = hipMemcpy(d_rows, rows.data(), rows.size() * sizeof(long long), hipMemcpyHostToDevice)) != hipSuccess)
            rc = pf_err(c, CCJ_E_HIP, "hash rows", e);
        for (int x = 0; x < CCJ_PF_NMAT4 && rc == CCJ_OK; ++x) {
            if ((e = (hipError_t)ccjk_pf_canon(&c->D, x, d_rows, nrows, d_out, c->st)) != hipSuccess ||
                (e = hipMemcpyAsync(hbuf.data(), d_out, q * sizeof(int), hipMemcpyDeviceToHost, c->st)) != hipSuccess ||
                (e = hipStreamSynchronize(c->st)) != hipSuccess) {
                rc = pf_err(c, CCJ_E_HIP, "hash gather", e);
                break;
            }
            h4[x] = fnv_arr(hbuf.data(), (size_t)q);
        }
        hipFree(d_rows);
        hipFree(d_out);
        if (rc != CCJ_OK) return rc;
    }
    return CCJ_OK;
}

const char *ccj_pf_exp_names(void) { return kExpNames; }

int ccj_pf_exp_hashes(ccj_pf_ctx *c, uint64_t *out, int cap) {
    if (!c || !out || cap < kNExp) return CCJ_E_ARG;
    return exp_hashes(c->E, c->prm, out);
}

int ccj_pf_exp_hashes_params(const ccj_energy_params *prm, const ccj_pf_raw *raw, const ccj_pk_penalties *pen,
                             uint64_t *out, int cap) {
    if (!prm || !out || cap < kNExp || prm->magic != CCJ_PARAMS_MAGIC) return CCJ_E_ARG;
    if (raw && (raw->magic != CCJ_PF_RAW_MAGIC || raw->size_bytes != sizeof(ccj_pf_raw))) return CCJ_E_ARG;
    const ccj_pk_penalties defp = CCJ_PK_PENALTIES_DEFAULT;
    PfExp *E = new PfExp;
    build_exp(*prm, raw, pen ? *pen : defp, *E);
    const int q = exp_hashes(*E, *prm, out);
    delete E;
    return q;
}

}  // extern "C"

namespace {

int exp_hashes(const PfExp &P, const ccj_energy_params &prm, uint64_t *out) {
    int q = 0;
    out[q++] = fnv_arr(&P.stack[0][0], 64);
    out[q++] = fnv_arr(P.hairpin, 31);
    out[q++] = fnv_arr(P.bulge, 31);
    out[q++] = fnv_arr(P.internal57, 31);
    out[q++] = fnv_arr(P.ninio, 31);
    out[q++] = fnv_arr(&P.mismatchI[0][0][0], 200);
    out[q++] = fnv_arr(&P.mismatch1nI[0][0][0], 200);
    out[q++] = fnv_arr(&P.mismatch23I[0][0][0], 200);
    out[q++] = fnv_arr(&P.mismatchH[0][0][0], 200);
    out[q++] = fnv_arr(&P.mismatchM[0][0][0], 200);
    out[q++] = fnv_arr(&P.mismatchExt[0][0][0], 200);
    out[q++] = fnv_arr(&P.dangle5[0][0], 40);
    out[q++] = fnv_arr(&P.dangle3[0][0], 40);
    out[q++] = fnv_arr(&P.int11[0][0][0][0], 64 * 25);
    out[q++] = fnv_arr(&P.int21[0][0][0][0][0], 64 * 125);
    out[q++] = fnv_arr(&P.int22[0][0][0][0][0][0], 64 * 625);
    out[q++] = fnv_arr(P.MLintern, 8);
    const double sc[] = {P.TermAU, P.MLbase, P.MLclosing, P.kT, P.lxc, P.pf_scale};
    out[q++] = fnv_arr(sc, 6);
    out[q++] = fnv_arr(P.tetra, strnlen(prm.Tetraloops, sizeof prm.Tetraloops) / 7);
    out[q++] = fnv_arr(P.tri, strnlen(prm.Triloops, sizeof prm.Triloops) / 6);
    out[q++] = fnv_arr(P.hex, strnlen(prm.Hexaloops, sizeof prm.Hexaloops) / 9);
    const double pk[] = {P.PS, P.PSM, P.PSP, P.PB, P.PUP, P.PPS, P.a, P.b, P.c, P.ap, P.bp, P.cp};
    out[q++] = fnv_arr(pk, 12);
    return q;
}

}  // namespace

extern "C" {

int ccj_pf_srand(ccj_pf_ctx *c, unsigned int seed) {
    if (!c) return CCJ_E_ARG;
    return srandom_r(seed, &c->rnd) == 0 ? CCJ_OK : CCJ_E_ARG;
}

int ccj_pf_sample(ccj_pf_ctx *c, int nsamples, char *structures, int *done) {
    if (!c || nsamples < 0 || (nsamples > 0 && !structures)) return CCJ_E_ARG;
    if (done) *done = 0;
    if (!c->filled) return CCJ_E_STATE;
    const int n = c->n;
    for (int s = 0; s < nsamples; ++s) {
        std::string st(n, '.');
        Sampler S{*c, st};
        S.W_(1, n);
        if (S.failed) return CCJ_E_PF_SAMPLE;
        memcpy(structures + (size_t)s * (n + 1), st.c_str(), n + 1);
        if (done) *done = s + 1;
    }
    return CCJ_OK;
}

const char *ccj_pf_last_message(ccj_pf_ctx *c) { return c ? c->msg.c_str() : ""; }

int ccj_pf_timing(ccj_pf_ctx *c, float *fill_ms) {
    if (!c || !fill_ms) return CCJ_E_ARG;
    *fill_ms = c->fill_ms;
    return CCJ_OK;
}

int ccj_pf_set_timing(ccj_pf_ctx *c, int on) {
    if (!c) return CCJ_E_ARG;
    c->timing = on != 0;
    return CCJ_OK;
}

int ccj_pf_kernel_ms(ccj_pf_ctx *c, double *ms4) {
    if (!c || !ms4) return CCJ_E_ARG;
    for (int k = 0; k < 4; ++k) ms4[k] = c->kms[k];
    return CCJ_OK;
}

int ccj_pf_work_model(ccj_pf_ctx *c, double *bytes4) {
    if (!c || !bytes4) return CCJ_E_ARG;
    const PfWork w = pf_work_model(*c);
    bytes4[0] = w.iloop;
    bytes4[1] = w.level;
    bytes4[2] = w.pterm;
    bytes4[3] = w.diag;
    return CCJ_OK;
}

}  // extern "C"
