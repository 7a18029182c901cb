// oracle/ref_driver.cc — TEST INFRASTRUCTURE ONLY (never part of the shipped engine).
//
// A driver of our own that links the reference CCJ sources compiled where they lie under
// /root/reference/src (see oracle/Makefile; nothing is copied).  It is the "real reference"
// strengthening of the oracle (task ③):
//   fold         run W_final(seq,dangle).ccj() exactly as src/CCJ.cc:44-49,104-108 does and print
//                the same two stdout lines; optionally print FNV-1a hashes of every DP matrix in
//                the canonical (i,j,k,l) order and dump them for byte-level diffs.
//   dump-params  write the scaled vrna_param_t fields the CCJ path reads into our blob format
//                (include/ccj_params.h) — this is how tests/golden/params/*.ccjp are produced.
// Parameters can come from a .par file (-P, as the reference CLI), the DNA Mathews 2004 set
// (--dna, CCJ.cc:88-90), or one of our blobs (--blob): the blob is written back into the
// ViennaRNA 37 C globals that scale_parameters() reads, so the reference binary can run on the
// GPU box where /root/reference (and its params/ directory) does not exist.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <iostream>
#include <fstream>
#include <chrono>
#include <algorithm>
#include <stack>
#include <list>
#include <limits>
#include <cassert>
#include <cmath>
#include <array>
#include <functional>

// Reach into the reference's private members for hashing only (layout is unaffected).
#define private public
#define protected public
#include "W_final.hh"
#include "h_globals.hh"
#undef private
#undef protected

extern "C" {
#include "ViennaRNA/params/io.h"
#include "ViennaRNA/params/basic.h"
#include "ViennaRNA/model.h"
}
#include "ccj_params.h"

// ViennaRNA 37 C parameter globals (ViennaRNA/params/default.c), written by --blob.
extern "C" {
extern int stack37[NBPAIRS + 1][NBPAIRS + 1];
extern int hairpin37[31];
extern int bulge37[31];
extern int internal_loop37[31];
extern int mismatchI37[NBPAIRS + 1][5][5];
extern int mismatchH37[NBPAIRS + 1][5][5];
extern int mismatchM37[NBPAIRS + 1][5][5];
extern int mismatch1nI37[NBPAIRS + 1][5][5];
extern int mismatch23I37[NBPAIRS + 1][5][5];
extern int mismatchExt37[NBPAIRS + 1][5][5];
extern int dangle5_37[NBPAIRS + 1][5];
extern int dangle3_37[NBPAIRS + 1][5];
extern int int11_37[NBPAIRS + 1][NBPAIRS + 1][5][5];
extern int int21_37[NBPAIRS + 1][NBPAIRS + 1][5][5][5];
extern int int22_37[NBPAIRS + 1][NBPAIRS + 1][5][5][5][5];
extern int ML_BASE37, ML_closing37, ML_intern37, ninio37, TerminalAU37, MAX_NINIO;
extern double lxc37;
extern char Triloops[241];
extern int Triloop37[40];
extern char Tetraloops[281];
extern int Tetraloop37[40];
extern char Hexaloops[361];
extern int Hexaloop37[40];
}

static uint64_t fnv_init() { return 1469598103934665603ull; }
static void fnv_bytes(uint64_t &h, const void *p, size_t n) {
    const unsigned char *c = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
}

static bool read_file(const std::string &path, std::vector<char> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

static void fill_blob(ccj_energy_params &b, const vrna_param_t *p) {
    memset(&b, 0, sizeof(b));
    b.magic = CCJ_PARAMS_MAGIC;
    b.version = CCJ_PARAMS_VERSION;
    b.size_bytes = sizeof(b);
    b.special_hp = p->model_details.special_hp;
    memcpy(b.stack, p->stack, sizeof(b.stack));
    memcpy(b.hairpin, p->hairpin, sizeof(b.hairpin));
    memcpy(b.bulge, p->bulge, sizeof(b.bulge));
    memcpy(b.internal_loop, p->internal_loop, sizeof(b.internal_loop));
    memcpy(b.mismatchExt, p->mismatchExt, sizeof(b.mismatchExt));
    memcpy(b.mismatchI, p->mismatchI, sizeof(b.mismatchI));
    memcpy(b.mismatch1nI, p->mismatch1nI, sizeof(b.mismatch1nI));
    memcpy(b.mismatch23I, p->mismatch23I, sizeof(b.mismatch23I));
    memcpy(b.mismatchH, p->mismatchH, sizeof(b.mismatchH));
    memcpy(b.mismatchM, p->mismatchM, sizeof(b.mismatchM));
    memcpy(b.dangle5, p->dangle5, sizeof(b.dangle5));
    memcpy(b.dangle3, p->dangle3, sizeof(b.dangle3));
    memcpy(b.int11, p->int11, sizeof(b.int11));
    memcpy(b.int21, p->int21, sizeof(b.int21));
    memcpy(b.int22, p->int22, sizeof(b.int22));
    b.ninio2 = p->ninio[2];
    b.max_ninio = MAX_NINIO;
    b.MLbase = p->MLbase;
    b.MLclosing = p->MLclosing;
    b.TerminalAU = p->TerminalAU;
    memcpy(b.MLintern, p->MLintern, sizeof(b.MLintern));
    b.lxc = p->lxc;
    memcpy(b.Tetraloop_E, p->Tetraloop_E, sizeof(b.Tetraloop_E));
    memcpy(b.Triloop_E, p->Triloop_E, sizeof(b.Triloop_E));
    memcpy(b.Hexaloop_E, p->Hexaloop_E, sizeof(b.Hexaloop_E));
    strncpy(b.Tetraloops, p->Tetraloops, sizeof(b.Tetraloops) - 1);
    strncpy(b.Triloops, p->Triloops, sizeof(b.Triloops) - 1);
    strncpy(b.Hexaloops, p->Hexaloops, sizeof(b.Hexaloops) - 1);
}

// Write a blob back into the 37 C globals.  At 37 C tempf == 1.0 so scaling is the identity
// (params.c:60 RESCALE_dG) and the dangle/mismatch clamps (params.c:487-512) are idempotent.
static void inject_blob(const ccj_energy_params &b) {
    memcpy(stack37, b.stack, sizeof(b.stack));
    memcpy(hairpin37, b.hairpin, sizeof(b.hairpin));
    memcpy(bulge37, b.bulge, sizeof(bulge37));
    memcpy(internal_loop37, b.internal_loop, sizeof(internal_loop37));
    memcpy(mismatchExt37, b.mismatchExt, sizeof(b.mismatchExt));
    memcpy(mismatchI37, b.mismatchI, sizeof(b.mismatchI));
    memcpy(mismatch1nI37, b.mismatch1nI, sizeof(b.mismatch1nI));
    memcpy(mismatch23I37, b.mismatch23I, sizeof(b.mismatch23I));
    memcpy(mismatchH37, b.mismatchH, sizeof(b.mismatchH));
    memcpy(mismatchM37, b.mismatchM, sizeof(b.mismatchM));
    memcpy(dangle5_37, b.dangle5, sizeof(b.dangle5));
    memcpy(dangle3_37, b.dangle3, sizeof(b.dangle3));
    memcpy(int11_37, b.int11, sizeof(b.int11));
    memcpy(int21_37, b.int21, sizeof(b.int21));
    memcpy(int22_37, b.int22, sizeof(b.int22));
    ninio37 = b.ninio2;
    MAX_NINIO = b.max_ninio;
    ML_BASE37 = b.MLbase;
    ML_closing37 = b.MLclosing;
    TerminalAU37 = b.TerminalAU;
    ML_intern37 = b.MLintern[1];
    lxc37 = b.lxc;
    memset(Tetraloops, 0, sizeof(Tetraloops));
    memset(Triloops, 0, sizeof(Triloops));
    memset(Hexaloops, 0, sizeof(Hexaloops));
    strncpy(Tetraloops, b.Tetraloops, sizeof(Tetraloops) - 1);
    strncpy(Triloops, b.Triloops, sizeof(Triloops) - 1);
    strncpy(Hexaloops, b.Hexaloops, sizeof(Hexaloops) - 1);
    memcpy(Tetraloop37, b.Tetraloop_E, sizeof(Tetraloop37));
    memcpy(Triloop37, b.Triloop_E, sizeof(Triloop37));
    memcpy(Hexaloop37, b.Hexaloop_E, sizeof(Hexaloop37));
}

struct Opts {
    int dangles = 2;
    bool noGU = false;
    std::string parfile, blob, dump, out;
    bool dna = false, timing = false, hash = false;
    std::string seq;
};

static int load_params(const Opts &o) {
    if (!o.blob.empty()) {
        std::vector<char> buf;
        if (!read_file(o.blob, buf) || buf.size() != sizeof(ccj_energy_params)) {
            fprintf(stderr, "ref_driver: bad blob %s\n", o.blob.c_str());
            return 1;
        }
        ccj_energy_params b;
        memcpy(&b, buf.data(), sizeof(b));
        if (b.magic != CCJ_PARAMS_MAGIC) { fprintf(stderr, "ref_driver: bad magic\n"); return 1; }
        inject_blob(b);
    } else if (o.dna) {
        vrna_params_load_DNA_Mathews2004();
    } else if (!o.parfile.empty()) {
        if (!vrna_params_load(o.parfile.c_str(), VRNA_PARAMETER_FORMAT_DEFAULT)) {
            fprintf(stderr, "ref_driver: cannot load %s\n", o.parfile.c_str());
            return 1;
        }
    }
    return 0;
}

struct Hasher {
    std::vector<std::pair<std::string, uint64_t>> hashes;
    FILE *dump = nullptr;
    void add4(const char *name, const Matrix4D &M, int n) {
        uint64_t h = fnv_init();
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j)
                for (int k = j + 2; k <= n; ++k)
                    for (int l = k; l <= n; ++l) {
                        int16_t v = (int16_t)M.get(i, j, k, l);
                        fnv_bytes(h, &v, 2);
                        if (dump) { int32_t w = v; fwrite(&w, 4, 1, dump); }
                    }
        hashes.push_back({name, h});
    }
    template <class F> void add2(const char *name, int n, F get) {
        uint64_t h = fnv_init();
        for (int i = 1; i <= n; ++i)
            for (int j = i; j <= n; ++j) {
                int32_t v = get(i, j);
                fnv_bytes(h, &v, 4);
                if (dump) fwrite(&v, 4, 1, dump);
            }
        hashes.push_back({name, h});
    }
};

// One FNV-1a hash per DP matrix in canonical (i,j,k,l) order, printed as HASH lines.
static void hash_all(const Opts &o, W_final &wf, int n) {
    pseudo_loop *P = wf.P;
    s_energy_matrix *V = wf.V;
    Hasher H;
    if (!o.dump.empty()) H.dump = fopen(o.dump.c_str(), "wb");
    H.add4("PK", P->PK, n);
    H.add4("PL", P->PL, n);
    H.add4("PR", P->PR, n);
    H.add4("PM", P->PM, n);
    H.add4("PO", P->PO, n);
    H.add4("PfromL", P->PfromL, n);
    H.add4("PfromR", P->PfromR, n);
    H.add4("PfromM", P->PfromM, n);
    H.add4("PfromMprime", P->PfromMprime, n);
    H.add4("PfromO", P->PfromO, n);
    H.add4("PLmloop00", P->PLmloop00, n);
    H.add4("PLmloop01", P->PLmloop01, n);
    H.add4("PLmloop10", P->PLmloop10, n);
    H.add4("PRmloop00", P->PRmloop00, n);
    H.add4("PRmloop01", P->PRmloop01, n);
    H.add4("PRmloop10", P->PRmloop10, n);
    H.add4("PMmloop00", P->PMmloop00, n);
    H.add4("PMmloop01", P->PMmloop01, n);
    H.add4("PMmloop10", P->PMmloop10, n);
    H.add4("POmloop00", P->POmloop00, n);
    H.add4("POmloop01", P->POmloop01, n);
    H.add4("POmloop10", P->POmloop10, n);
    H.add2("P", n, [&](int i, int j) { return (int32_t)P->P.get(i, j); });
    H.add2("WBP", n, [&](int i, int j) { return (int32_t)P->WBP.get(i, j); });
    H.add2("WPP", n, [&](int i, int j) { return (int32_t)P->WPP.get(i, j); });
    H.add2("V", n, [&](int i, int j) { return (int32_t)V->get_node(i, j)->energy; });
    H.add2("Vtype", n, [&](int i, int j) { return (int32_t)V->get_node(i, j)->type; });
    H.add2("WM", n, [&](int i, int j) { return (int32_t)V->WM.get(i, j); });
    H.add2("WMv", n, [&](int i, int j) { return (int32_t)V->WMv.get(i, j); });
    H.add2("WMp", n, [&](int i, int j) { return (int32_t)V->WMp.get(i, j); });
    {
        uint64_t h = fnv_init();
        for (int j = 0; j <= n; ++j) {
            int32_t v = wf.W[j];
            fnv_bytes(h, &v, 4);
            if (H.dump) fwrite(&v, 4, 1, H.dump);
        }
        H.hashes.push_back({"W", h});
    }
    if (H.dump) fclose(H.dump);
    for (auto &kv : H.hashes) printf("HASH %s %016llx\n", kv.first.c_str(), (unsigned long long)kv.second);
}

static int cmd_fold(const Opts &o) {
    noGU = o.noGU ? 1 : 0;
    if (load_params(o)) return 1;
    std::string seq = o.seq;
    auto t0 = std::chrono::steady_clock::now();
    W_final wf(seq, o.dangles);
    double energy = wf.ccj();
    auto t1 = std::chrono::steady_clock::now();
    std::cout << seq << std::endl;
    std::cout << wf.structure << " (" << energy << ")" << std::endl;
    if (o.timing)
        fprintf(stderr, "TIME %.6f\n", std::chrono::duration<double>(t1 - t0).count());
    if (o.hash) {  // the matrices and W survive ccj(); hash them after the fold's own output
        fflush(stdout);
        hash_all(o, wf, (int)seq.size());
        printf("MFE %d\n", (int)wf.W[seq.size()]);
    }
    return 0;
}

// Fill only, by calling the reference's own member functions in the order of
// W_final.cc:60-77 (no backtrack, so reference backtrack exits cannot hide the matrices), then
// print one FNV-1a hash per matrix in canonical order.
static int cmd_hash(const Opts &o) {
    noGU = o.noGU ? 1 : 0;
    if (load_params(o)) return 1;
    std::string seq = o.seq;
    W_final wf(seq, o.dangles);
    int n = (int)seq.size();
    pseudo_loop *P = wf.P;
    s_energy_matrix *V = wf.V;
    for (int i = n; i >= 1; --i)
        for (int j = i; j <= n; ++j) {
            V->compute_energy(i, j);
            P->compute_energies(i, j);
            V->compute_WMv_WMp(i, j, P->get_energy(i, j));
            V->compute_energy_WM(i, j, P->P);
        }
    for (int j = TURN + 1; j <= n; j++) {
        energy_t m1 = wf.W[j - 1], m2 = INF, m3 = INF;
        for (int k = 1; k <= j - TURN - 1; ++k) {
            energy_t acc = (k > 1) ? wf.W[k - 1] : 0;
            m2 = std::min(m2, acc + wf.E_ext_Stem(V->get_energy(k, j), V->get_energy(k + 1, j), V->get_energy(k, j - 1),
                                                   V->get_energy(k + 1, j - 1), wf.S_, wf.params_, k, j, n));
            m3 = std::min(m3, acc + std::min({P->get_energy(k, j), P->get_energy(k + 1, j), P->get_energy(k, j - 1),
                                              P->get_energy(k + 1, j - 1)}) + PS_penalty);
        }
        wf.W[j] = std::min({m1, m2, m3});
    }
    hash_all(o, wf, n);
    printf("MFE %d\n", (int)wf.W[n]);
    return 0;
}

static int cmd_dump_params(const Opts &o) {
    if (load_params(o)) return 1;
    vrna_param_t *p = scale_parameters();
    ccj_energy_params b;
    fill_blob(b, p);
    free(p);
    FILE *f = fopen(o.out.c_str(), "wb");
    if (!f) { fprintf(stderr, "cannot write %s\n", o.out.c_str()); return 1; }
    fwrite(&b, sizeof(b), 1, f);
    fclose(f);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: ref_driver fold|dump-params [opts] [SEQ]\n");
        return 2;
    }
    std::string cmd = argv[1];
    Opts o;
    for (int a = 2; a < argc; ++a) {
        std::string s = argv[a];
        if (s == "-d" && a + 1 < argc) o.dangles = atoi(argv[++a]);
        else if (s == "--noGU") o.noGU = true;
        else if (s == "-P" && a + 1 < argc) o.parfile = argv[++a];
        else if (s == "--blob" && a + 1 < argc) o.blob = argv[++a];
        else if (s == "--dna") o.dna = true;
        else if (s == "--time") o.timing = true;
        else if (s == "--hash") o.hash = true;
        else if (s == "--dump" && a + 1 < argc) o.dump = argv[++a];
        else if (s == "-o" && a + 1 < argc) o.out = argv[++a];
        else o.seq = s;
    }
    if (cmd == "fold") {
        if (o.seq.empty()) std::getline(std::cin, o.seq);
        return cmd_fold(o);
    }
    if (cmd == "hash") {
        if (o.seq.empty()) std::getline(std::cin, o.seq);
        return cmd_hash(o);
    }
    if (cmd == "dump-params") return cmd_dump_params(o);
    fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 2;
}
