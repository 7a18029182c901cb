// ccj_wfinal.cc — the C++ W_final facade (include/W_final.hh) over the C ABI (include/ccj.h).
//
//   W_final::W_final  reference src/W_final.cc:20-56  (tables snapshot, sequence encoding, storage)
//   W_final::ccj      reference src/W_final.cc:58-105 (fill, W, backtrack, fill_structure)
//   vrna_params_load  reference src/ViennaRNA/params/io.c:252-276 (native reader, ccj_parfile.h)
//   vrna_params_load_DNA_Mathews2004  reference io.c:1110-1126
// The tables in force live here, as the reference keeps them in ViennaRNA's process globals:
// they start as the compiled-in Turner 2004 defaults (ccj_amd/params/default.ccjp next to the
// library) and every load overlays the current state.
#include <dlfcn.h>
#include <errno.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>
#include <stdexcept>
#include <algorithm>
#include <string>
#include <vector>

#include "W_final.hh"
#include "W_final_pf.hh"
#include "ccj.h"
#include "ccj_pf.h"
#include "ccj_parfile.h"

extern "C" {
int noGU = 0;  // ViennaRNA/model.c:54; CCJ.cc:77 sets it before constructing W_final
}

// The reference's PK penalties are globals defined by the program that includes its
// h_globals.hh (h_globals.hh:7-25, declared in h_externs.hh).  Weak references: when the program
// defines them they are read at construction time, otherwise the defaults apply.
extern int PS_penalty __attribute__((weak));
extern int PSM_penalty __attribute__((weak));
extern int PSP_penalty __attribute__((weak));
extern int PB_penalty __attribute__((weak));
extern int PUP_penalty __attribute__((weak));
extern int PPS_penalty __attribute__((weak));
extern int a_penalty __attribute__((weak));
extern int b_penalty __attribute__((weak));
extern int c_penalty __attribute__((weak));
extern int ap_penalty __attribute__((weak));
extern int bp_penalty __attribute__((weak));
extern int cp_penalty __attribute__((weak));
extern double e_stP_penalty __attribute__((weak));
extern double e_intP_penalty __attribute__((weak));

namespace {

std::mutex g_mu;
bool g_init = false;
ccj_energy_params g_tables;  // the tables in force
ccj_pf_raw g_pfraw;          // their raw dangle / mismatch tables (partition function)
bool g_pfraw_ok = false;     // false: not known (a .par file read natively), see ccj_pf.h

std::string params_dir() {
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&vrna_params_load), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t s = p.find_last_of('/');
        return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/../params/";
    }
    return "ccj_amd/params/";
}

bool read_raw(const std::string &name) {
    std::ifstream f(params_dir() + name, std::ios::binary);
    g_pfraw_ok = false;
    if (!f) return false;
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() != sizeof(ccj_pf_raw)) return false;
    memcpy(&g_pfraw, b.data(), sizeof g_pfraw);
    g_pfraw_ok = g_pfraw.magic == CCJ_PF_RAW_MAGIC;
    return g_pfraw_ok;
}

bool read_tables(const std::string &name, ccj_energy_params &out) {
    std::ifstream f(params_dir() + name, std::ios::binary);
    if (!f) return false;
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() != sizeof(ccj_energy_params)) return false;
    memcpy(&out, b.data(), sizeof out);
    return out.magic == CCJ_PARAMS_MAGIC;
}

// callers hold g_mu
void ensure_defaults() {
    if (g_init) return;
    if (!read_tables("default.ccjp", g_tables))
        throw std::runtime_error("W_final: compiled-in default tables missing (" + params_dir() + "default.ccjp)");
    read_raw("default.pfraw");
    g_init = true;
}

template <class T>
T weak_or(const T *p, T dflt) {
    return p ? *p : dflt;
}

ccj_pk_penalties program_penalties();

}  // namespace

extern "C" int vrna_params_load(const char *fname, unsigned int /*options*/) {
    std::lock_guard<std::mutex> lk(g_mu);
    ensure_defaults();
    ccj_energy_params out;
    std::vector<char> log(1 << 20);
    const int rc = ccj_params_load_par(fname, &g_tables, &out, log.data(), (int)log.size());
    fputs(log.data(), stderr);
    if (rc == CCJ_E_PARFILE) exit(EXIT_FAILURE);  // vrna_message_error, io.c
    if (rc == 1) {
        g_tables = out;
        g_pfraw_ok = false;
    }
    return rc;
}

extern "C" int vrna_params_load_DNA_Mathews2004(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    ensure_defaults();
    ccj_energy_params t;
    if (!read_tables("DNA_Mathews2004.ccjp", t)) return 0;
    g_tables = t;
    read_raw("DNA_Mathews2004.pfraw");
    // check_symmetry (io.c:1126): the built-in DNA set has two asymmetric stack-enthalpy pairs
    for (int w = 0; w < 4; ++w) fputs("WARNING: stacking enthalpies not symmetric\n", stderr);
    return 1;
}

void ccj_wfinal_use_tables(const ccj_energy_params &tables) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_tables = tables;
    g_pfraw_ok = false;
    g_init = true;
}

W_final::W_final(std::string seq, int dangle) : params_(nullptr), seq_(std::move(seq)), dangle_(dangle), noGU_(noGU) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        ensure_defaults();
        tables_ = g_tables;  // scale_parameters() snapshot, W_final.cc:23
    }
    params_ = &tables_;
    const long long n = (long long)seq_.size();
    const char *compat = getenv("CCJ_REF_COMPAT_ABORT");
    if (compat && atoi(compat) != 0) {
        // stock build: Matrix4D::init asserts slice_size_ == n*(n+1)*(n+2)*(n+3)/24 in int
        // arithmetic (matrices.hh:159-160), which overflows for n >= 214
        const long long slice = n * (n + 1) * (n + 2) * (n + 3) / 24;
        const int lhs = (int)(uint32_t)(n * (n + 1) * (n + 2) * (n + 3));
        if (slice != (long long)(lhs / 24)) {
            fflush(stdout);
            fprintf(stderr,
                    "%s: src/matrices.hh:160: void Matrix4D::init(cand_pos_t, index_offset_t&): Assertion "
                    "`slice_size_ == n*(n+1)*(n+2)*(n+3)/24' failed.\n",
                    program_invocation_short_name);
            abort();
        }
    }
    ccj_pk_penalties pen = program_penalties();
    const char *dev = getenv("CCJ_DEVICE");
    ccj_problem prob{seq_.c_str(), dangle_, noGU_, &tables_, &pen};
    ccj_options o{};
    o.device = dev ? atoi(dev) : 0;
    const int rc = ccj_create(&prob, &o, &ctx_);
    if (rc != CCJ_OK)
        throw std::runtime_error(std::string("W_final: engine error ") + std::to_string(rc) + ": " + ccj_last_error(nullptr));
}

namespace {
ccj_pk_penalties program_penalties() {
    ccj_pk_penalties pen = CCJ_PK_PENALTIES_DEFAULT;
    pen.PS = weak_or(&PS_penalty, pen.PS);
    pen.PSM = weak_or(&PSM_penalty, pen.PSM);
    pen.PSP = weak_or(&PSP_penalty, pen.PSP);
    pen.PB = weak_or(&PB_penalty, pen.PB);
    pen.PUP = weak_or(&PUP_penalty, pen.PUP);
    pen.PPS = weak_or(&PPS_penalty, pen.PPS);
    pen.a = weak_or(&a_penalty, pen.a);
    pen.b = weak_or(&b_penalty, pen.b);
    pen.c = weak_or(&c_penalty, pen.c);
    pen.ap = weak_or(&ap_penalty, pen.ap);
    pen.bp = weak_or(&bp_penalty, pen.bp);
    pen.cp = weak_or(&cp_penalty, pen.cp);
    pen.e_stP = weak_or(&e_stP_penalty, pen.e_stP);
    pen.e_intP = weak_or(&e_intP_penalty, pen.e_intP);
    return pen;
}
}  // namespace

W_final::~W_final() {
    if (ctx_) ccj_destroy(ctx_);
}

double W_final::ccj() {
    int rc = ccj_fill(ctx_);
    if (rc != CCJ_OK)
        throw std::runtime_error(std::string("W_final::ccj: engine error ") + std::to_string(rc) + ": " + ccj_last_error(ctx_));
    std::string s(seq_.size() + 1, '\0');
    std::vector<char> msgs(1 << 16);
    double energy = 0;
    rc = ccj_result(ctx_, &s[0], &energy, msgs.data(), (int)msgs.size());
    fputs(msgs.data(), stdout);  // the reference's printf side messages, in order
    if (rc == CCJ_E_BACKTRACK || rc == CCJ_E_INTER_EXIT) {
        const std::string err = ccj_last_error(ctx_);
        fflush(stdout);
        std::cout.flush();
        fputs(err.c_str(), stderr);
        fflush(stderr);
        if (rc == CCJ_E_INTER_EXIT) exit(0);
        if (err.find("Assertion") != std::string::npos) abort();
        exit(EXIT_FAILURE);
    }
    if (rc != CCJ_OK)
        throw std::runtime_error(std::string("W_final::ccj: engine error ") + std::to_string(rc) + ": " + ccj_last_error(ctx_));
    s.resize(seq_.size());
    structure = s;
    return energy;
}

// ---- W_final_pf (include/W_final_pf.hh) -------------------------------------------------------

W_final_pf::W_final_pf(std::string &seq, std::string & /*MFE_structure*/, double /*MFE_energy*/, int dangle,
                       int num_samples_, bool /*PSplot*/)
    : num_samples(num_samples_), seq_(seq) {
    ccj_energy_params tables;
    ccj_pf_raw raw;
    bool raw_ok;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        ensure_defaults();
        tables = g_tables;
        raw = g_pfraw;
        raw_ok = g_pfraw_ok;
    }
    ccj_pk_penalties pen = program_penalties();
    const char *dev = getenv("CCJ_DEVICE");
    ccj_problem prob{seq_.c_str(), dangle, noGU, &tables, &pen};
    const int rc = ccj_pf_create(&prob, raw_ok ? &raw : nullptr, dev ? atoi(dev) : 0, &ctx_);
    if (rc != CCJ_OK) throw std::runtime_error(std::string("W_final_pf: engine error ") + std::to_string(rc));
}

W_final_pf::~W_final_pf() {
    if (ctx_) ccj_pf_destroy(ctx_);
}

pf_t W_final_pf::ccj_pf() {
    double e = 0;
    const int rc = ccj_pf_fill(ctx_, &e);
    if (rc != CCJ_OK)
        throw std::runtime_error(std::string("W_final_pf::ccj_pf: engine error ") + std::to_string(rc) + ": " +
                                 ccj_pf_last_message(ctx_));
    filled_ = true;
    structure = std::string(seq_.size(), '.');
    return e;
}

void W_final_pf::srand_samples(unsigned int seed) { ccj_pf_srand(ctx_, seed); }

std::vector<std::string> W_final_pf::sample(int k) {
    if (!filled_) ccj_pf();
    const size_t n = seq_.size();
    std::vector<char> buf((size_t)std::max(k, 1) * (n + 1));
    int done = 0;
    const int rc = ccj_pf_sample(ctx_, k, buf.data(), &done);
    std::vector<std::string> out;
    for (int s = 0; s < done; ++s) out.emplace_back(buf.data() + (size_t)s * (n + 1), n);
    if (rc == CCJ_E_PF_SAMPLE) {  // the reference prints the line and exit(0)s (stoch_backtrack.cc)
        fputs(ccj_pf_last_message(ctx_), stdout);
        fflush(stdout);
        exit(0);
    }
    if (rc != CCJ_OK) throw std::runtime_error("W_final_pf::sample: engine error " + std::to_string(rc));
    return out;
}
