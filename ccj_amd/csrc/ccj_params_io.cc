// ccj_params_io.cc — native "RNAfold parameter file v2.0" reader (include/ccj_parfile.h).
//
// Behaviour follows the reference loader the CCJ binary links (ViennaRNA 2.x):
//   section loop / identifiers      src/ViennaRNA/params/io.c:454-673, gettype io.c:1701-1782
//   value lists ('*', 'x', DEF/INF/NST, C comments)   get_array1 io.c:713-762, ignore_comment io.c:1100-1120
//   N-d slices with pre/post shifts rd_*dim_slice io.c:778-1016 (dims/shifts io.c:37-76)
//   special hairpin lists           rd_Tetraloop37 / rd_Triloop37 / rd_Hexaloop37 io.c:1020-1096
//   int22 non-standard maxima       update_nst io.c:1184-1299
//   symmetry warnings               check_symmetry io.c:1126-1180
//   37 C scaling                    get_scaled_params params.c:399-555 (tempf == 1.0: every
//                                   RESCALE_dG is the identity; mismatchM/mismatchExt/dangles
//                                   are clamped to <= 0 since md.dangles == 2 at scaling time)
// Quirks kept on purpose because they change the tables a file produces:
//   * every value block starts on a fresh line; extra tokens on its last line are dropped;
//   * a special-hairpin list ends at the first line that does not scan as "SEQ dG dH" — that
//     line is consumed (so a following "# Triloops" header is swallowed) and a space is still
//     appended to the list string, and a short sequence leaves a NUL gap that hides later
//     entries from strlen();
//   * Tetra/Tri/Hexaloop_E are refreshed for i*7 / i*5 / i*9 < strlen(list) (params.c:447-454).
// Differences (undefined behaviour in the reference, documented in DESIGN.md §9):
//   * '*' inside ML_params / NINIO / Misc keeps the value in force (the reference stores an
//     uninitialised stack slot);
//   * enthalpy tables are not part of the blob: they start at zero (the compiled-in defaults are
//     symmetric — loading a dG-only file prints no symmetry warning) and only feed the
//     symmetry warnings;
//   * list indices past 40 (possible only for > 33 triloops) are not read.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <climits>
#include <cstdlib>
#include <string>
#include <vector>

#include "ccj_parfile.h"

namespace {

constexpr int kDEF = -50, kINF = 10000000, kNST = 0;  // params/constants.h
constexpr int NP = CCJ_NBPAIRS + 1;                    // pair-type extent (8)
constexpr int kLoopCap = 40;                           // entries per special-hairpin list

struct Fatal {
    std::string msg;
};

// sscanf "%Ns": skip white space, take up to `width` non-space characters.
bool scan_word(const char *&p, int width, std::string &out) {
    while (*p && isspace((unsigned char)*p)) ++p;
    if (!*p) return false;
    out.clear();
    while (*p && !isspace((unsigned char)*p) && (int)out.size() < width) out.push_back(*p++);
    return true;
}

// sscanf "%d": optional sign then at least one digit, value truncated from long like glibc.
bool scan_int(const char *&p, int &v) {
    const char *q = p;
    while (*q && isspace((unsigned char)*q)) ++q;
    const char *d = q + ((*q == '+' || *q == '-') ? 1 : 0);
    if (!isdigit((unsigned char)*d)) return false;
    char *end = nullptr;
    long x = strtol(q, &end, 10);
    v = (int)x;
    p = end;
    return true;
}

struct SpecialList {  // one of Tetraloops / Triloops / Hexaloops plus its dG column
    std::vector<char> str;  // reference char[281] / [241] / [361]
    int E[kLoopCap];
    int stride, width;
    size_t len() const { return strnlen(str.data(), str.size()); }
};

class ParReader {
  public:
    ParReader(std::vector<std::string> lines, const ccj_energy_params &base)
        : L_(std::move(lines)), base_(base), w_(base) {
        ml_intern_ = base.MLintern[1];
        init_list(tetra_, 281, 7, 6, base.Tetraloops, base.Tetraloop_E);
        init_list(tri_, 241, 6, 5, base.Triloops, base.Triloop_E);
        init_list(hexa_, 361, 9, 8, base.Hexaloops, base.Hexaloop_E);
        stackH_.assign(NP * NP, 0);
        int11H_.assign(NP * NP * 25, 0);
        int22H_.assign(NP * NP * 625, 0);
    }

    // set_parameters_from_string: 0 when there is no first line, else 1 (throws Fatal).
    int run() {
        if (L_.empty()) return 0;
        if (strncmp(L_[0].c_str(), "## RNAfold parameter file v2.0", 30) != 0)
            warn("Missing header line in file.\nMay be this file has not v2.0 format.\nUse INTERRUPT-key to stop.");
        ln_ = 1;
        while (const std::string *line = next_line()) section(*line);
        check_symmetry();
        return 1;
    }

    void finish(ccj_energy_params &out) const {
        out = w_;
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < 5; ++j) {
                for (int k = 0; k < 5; ++k) {
                    if (out.mismatchM[i][j][k] > 0) out.mismatchM[i][j][k] = 0;
                    if (out.mismatchExt[i][j][k] > 0) out.mismatchExt[i][j][k] = 0;
                }
                if (out.dangle5[i][j] > 0) out.dangle5[i][j] = 0;
                if (out.dangle3[i][j] > 0) out.dangle3[i][j] = 0;
            }
        for (int i = 0; i < NP; ++i) out.MLintern[i] = ml_intern_;
        emit_list(tetra_, 7, out.Tetraloops, sizeof out.Tetraloops, out.Tetraloop_E, 200);
        emit_list(tri_, 5, out.Triloops, sizeof out.Triloops, out.Triloop_E, 40);
        emit_list(hexa_, 9, out.Hexaloops, sizeof out.Hexaloops, out.Hexaloop_E, 40);
    }

    std::string messages;

  private:
    std::vector<std::string> L_;
    size_t ln_ = 0;
    const ccj_energy_params &base_;
    ccj_energy_params w_;  // raw 37 C tables in blob layout
    int ml_intern_;
    SpecialList tetra_, tri_, hexa_;
    std::vector<int> stackH_, int11H_, int22H_, scratch_;
    int ml_dH_[3] = {0, 0, 0}, ninio_dH_ = 0, misc_dH_[2] = {0, 0}, duplex_init_ = 0;

    void warn(const std::string &m) { messages += "WARNING: " + m + "\n"; }

    // content[line_no++]; the reference's array is NULL-terminated.
    const std::string *next_line() {
        size_t k = ln_++;
        return k < L_.size() ? &L_[k] : nullptr;
    }

    static void init_list(SpecialList &s, size_t cap, int stride, int width, const char *src, const int32_t *E) {
        s.str.assign(cap, 0);
        memcpy(s.str.data(), src, strnlen(src, cap - 1));
        s.stride = stride;
        s.width = width;
        for (int i = 0; i < kLoopCap; ++i) s.E[i] = E[i];
    }

    static void emit_list(const SpecialList &s, int step, char *dst, size_t dcap, int32_t *E, int ecap) {
        memset(dst, 0, dcap);
        size_t n = s.len();
        memcpy(dst, s.str.data(), n < dcap - 1 ? n : dcap - 1);
        for (int i = 0; i < ecap; ++i) E[i] = 0;
        for (int i = 0; i < kLoopCap && i < ecap && (size_t)(i * step) < n; ++i) E[i] = s.E[i];
    }

    // io.c:1100 — cut the first "/* ... */" out of the line.
    static void strip_comment(std::string &s) {
        size_t a = s.find("/*");
        if (a == std::string::npos) return;
        size_t b = s.find("*/", a);  // searched from the "/*" itself, as strstr(cp1, "*/")
        if (b == std::string::npos) throw Fatal{"unclosed comment in parameter file"};
        s.erase(a, b + 2 - a);
    }

    // io.c:713 get_array1 — `size` values from fresh lines into arr[0..size).
    void values(int *arr, int size) {
        int i = 0, last = 0;
        while (i < size) {
            const std::string *src = next_line();
            if (!src) throw Fatal{"unexpected end of file in get_array1"};
            std::string line = *src;
            strip_comment(line);
            const char *p = line.c_str();
            std::string tok;
            while (i < size && scan_word(p, 15, tok)) {
                int v;
                if (tok[0] == '*') {
                    ++i;
                    continue;
                } else if (tok[0] == 'x') {
                    if (i == 0) throw Fatal{"can't extrapolate first value"};
                    double g = 0.5 + base_.lxc * log((double)i / (double)last);
                    // last == 0 gives +inf; x86 cvttsd2si turns that into INT_MIN
                    int inc = (g >= 2147483648.0 || g != g) ? INT_MIN : (int)g;
                    v = (int)((unsigned)arr[last] + (unsigned)inc);
                } else if (tok == "DEF") {
                    v = kDEF;
                } else if (tok == "INF") {
                    v = kINF;
                } else if (tok == "NST") {
                    v = kNST;
                } else {
                    const char *t = tok.c_str();
                    if (!scan_int(t, v)) throw Fatal{std::string("\nrd_1dim: ") + p};
                    last = i;
                }
                arr[i++] = v;
            }
        }
    }

    // io.c:778-1016 rd_Ndim_slice, generic over the dimension count.
    void block(int *a, const int *dim, const int *pre, const int *post, int nd) {
        if (nd == 1) {
            values(a + pre[0], dim[0] - pre[0] - post[0]);
            return;
        }
        int shifted = 0, total = 1;
        for (int d = 0; d < nd; ++d) shifted += pre[d] + post[d], total *= dim[d];
        if (shifted == 0) {
            values(a, total);
            return;
        }
        int stride = total / dim[0];
        for (int i = pre[0]; i < dim[0] - post[0]; ++i) block(a + i * stride, dim + 1, pre + 1, post + 1, nd - 1);
    }

    int *scratch(size_t n) {
        scratch_.assign(n, 0);
        return scratch_.data();
    }

    // sscanf(line, "%Ws %d %d", &list[stride*i], &E[i], &dH) — assignments made before a
    // failure stick; returns the conversion count or -1 at end of input.
    static int scan_entry(const std::string &line, SpecialList &s, int i) {
        const char *p = line.c_str();
        std::string word;
        if (!scan_word(p, s.width, word)) return -1;
        size_t at = (size_t)s.stride * i;
        if (at + word.size() < s.str.size()) {
            memcpy(&s.str[at], word.data(), word.size());
            s.str[at + word.size()] = 0;
        }
        int v;
        if (!scan_int(p, v)) return 1;
        s.E[i] = v;
        if (!scan_int(p, v)) return 2;
        return 3;
    }

    // io.c:1020-1096
    void special(SpecialList &s) {
        std::fill(s.str.begin(), s.str.end(), 0);
        for (int i = 0; i < kLoopCap; ++i) s.E[i] = 0;
        int i = 0, r;
        do {
            const std::string *line = next_line();
            if (!line) break;
            r = scan_entry(*line, s, i);
            size_t n = s.len();
            if (n + 1 < s.str.size()) s.str[n] = ' ', s.str[n + 1] = 0;
            ++i;
        } while (r == 3 && i < kLoopCap);
    }

    void section(const std::string &line) {
        if (line.empty() || line[0] != '#') return;
        const char *p = line.c_str() + 1;
        std::string id;
        if (!scan_word(p, 255, id)) return;  // "# %255s" did not convert

        static const int d_stack[2] = {NP, NP}, s_stack[2] = {1, 1}, z2[2] = {0, 0};
        static const int d_mm[3] = {NP, 5, 5}, s_mm[3] = {1, 0, 0}, z3[3] = {0, 0, 0};
        static const int d_11[4] = {NP, NP, 5, 5}, s_11[4] = {1, 1, 0, 0}, z4[4] = {0, 0, 0, 0};
        static const int d_21[5] = {NP, NP, 5, 5, 5}, s_21[5] = {1, 1, 0, 0, 0}, z5[5] = {0, 0, 0, 0, 0};
        static const int d_22[6] = {NP, NP, 5, 5, 5, 5}, s_22[6] = {1, 1, 1, 1, 1, 1}, p_22[6] = {1, 1, 0, 0, 0, 0};
        static const int d_dg[2] = {NP, 5}, s_dg[2] = {1, 0};
        const int z1[1] = {0}, d31[1] = {31};

        auto is = [&](const char *name) { return id == name; };
        auto mm = [&](int *a) { block(a, d_mm, s_mm, z3, 3); };
        if (is("stack")) block(&w_.stack[0][0], d_stack, s_stack, z2, 2);
        else if (is("stack_enthalpies")) block(stackH_.data(), d_stack, s_stack, z2, 2);
        else if (is("hairpin")) block(w_.hairpin, d31, z1, z1, 1);
        else if (is("bulge")) block(w_.bulge, d31, z1, z1, 1);
        else if (is("interior")) block(w_.internal_loop, d31, z1, z1, 1);
        else if (is("hairpin_enthalpies") || is("bulge_enthalpies") || is("interior_enthalpies"))
            block(scratch(31), d31, z1, z1, 1);
        else if (is("mismatch_exterior")) mm(&w_.mismatchExt[0][0][0]);
        else if (is("mismatch_hairpin")) mm(&w_.mismatchH[0][0][0]);
        else if (is("mismatch_interior")) mm(&w_.mismatchI[0][0][0]);
        else if (is("mismatch_interior_1n")) mm(&w_.mismatch1nI[0][0][0]);
        else if (is("mismatch_interior_23")) mm(&w_.mismatch23I[0][0][0]);
        else if (is("mismatch_multi")) mm(&w_.mismatchM[0][0][0]);
        else if (is("mismatch_exterior_enthalpies") || is("mismatch_hairpin_enthalpies") ||
                 is("mismatch_interior_enthalpies") || is("mismatch_interior_1n_enthalpies") ||
                 is("mismatch_interior_23_enthalpies") || is("mismatch_multi_enthalpies"))
            mm(scratch(NP * 25));
        else if (is("int11")) block(&w_.int11[0][0][0][0], d_11, s_11, z4, 4);
        else if (is("int11_enthalpies")) block(int11H_.data(), d_11, s_11, z4, 4);
        else if (is("int21")) block(&w_.int21[0][0][0][0][0], d_21, s_21, z5, 5);
        else if (is("int21_enthalpies")) block(scratch(NP * NP * 125), d_21, s_21, z5, 5);
        else if (is("int22")) {
            block(&w_.int22[0][0][0][0][0][0], d_22, s_22, p_22, 6);
            update_nst(&w_.int22[0][0][0][0][0][0]);
        } else if (is("int22_enthalpies")) {
            block(int22H_.data(), d_22, s_22, p_22, 6);
            update_nst(int22H_.data());
        } else if (is("dangle5")) block(&w_.dangle5[0][0], d_dg, s_dg, z2, 2);
        else if (is("dangle3")) block(&w_.dangle3[0][0], d_dg, s_dg, z2, 2);
        else if (is("dangle5_enthalpies") || is("dangle3_enthalpies")) block(scratch(NP * 5), d_dg, s_dg, z2, 2);
        else if (is("ML_params")) {
            int v[6] = {w_.MLbase, ml_dH_[0], w_.MLclosing, ml_dH_[1], ml_intern_, ml_dH_[2]};
            values(v, 6);
            w_.MLbase = v[0], ml_dH_[0] = v[1], w_.MLclosing = v[2], ml_dH_[1] = v[3], ml_intern_ = v[4],
            ml_dH_[2] = v[5];
        } else if (is("NINIO")) {
            int v[3] = {w_.ninio2, ninio_dH_, w_.max_ninio};
            values(v, 3);
            w_.ninio2 = v[0], ninio_dH_ = v[1], w_.max_ninio = v[2];
        } else if (is("Misc")) {
            int v[4] = {duplex_init_, misc_dH_[0], w_.TerminalAU, misc_dH_[1]};
            values(v, 4);
            duplex_init_ = v[0], misc_dH_[0] = v[1], w_.TerminalAU = v[2], misc_dH_[1] = v[3];
        } else if (is("Tetraloops")) special(tetra_);
        else if (is("Triloops")) special(tri_);
        else if (is("Hexaloops")) special(hexa_);
        else if (is("END")) {
        } else warn("read_epars: Unknown field identifier in `" + line + "'");
    }

    // io.c:1184 — maxima over {C,G,A,U} for the non-standard (index 0 / NBPAIRS) slots.
    static void update_nst(int *a) {
        auto A = [a](int i, int j, int k, int l, int m, int n) -> int & {
            return a[((((i * NP + j) * 5 + k) * 5 + l) * 5 + m) * 5 + n];
        };
        const int P = CCJ_NBPAIRS;
        auto mx = [](int x, int y) { return x > y ? x : y; };
        for (int i = 1; i < P; ++i)
            for (int j = 1; j < P; ++j) {
                for (int k = 1; k < 5; ++k)
                    for (int l = 1; l < 5; ++l)
                        for (int m = 1; m < 5; ++m) {
                            int m1 = -kINF, m2 = -kINF, m3 = -kINF, m4 = -kINF;
                            for (int n = 1; n < 5; ++n) {
                                m1 = mx(m1, A(i, j, k, l, m, n));
                                m2 = mx(m2, A(i, j, k, l, n, m));
                                m3 = mx(m3, A(i, j, k, n, l, m));
                                m4 = mx(m4, A(i, j, n, k, l, m));
                            }
                            A(i, j, k, l, m, 0) = m1;
                            A(i, j, k, l, 0, m) = m2;
                            A(i, j, k, 0, l, m) = m3;
                            A(i, j, 0, k, l, m) = m4;
                        }
            }
        for (int i = 1; i < P; ++i)
            for (int j = 1; j < P; ++j)
                for (int k = 1; k < 5; ++k)
                    for (int l = 1; l < 5; ++l) {
                        int m1 = -kINF, m2 = -kINF, m3 = -kINF, m4 = -kINF, m5 = -kINF, m6 = -kINF;
                        for (int m = 1; m < 5; ++m) {
                            m1 = mx(m1, A(i, j, k, l, m, 0));
                            m2 = mx(m2, A(i, j, k, m, 0, l));
                            m3 = mx(m3, A(i, j, m, 0, k, l));
                            m4 = mx(m4, A(i, j, 0, k, l, m));
                            m5 = mx(m5, A(i, j, 0, k, m, l));
                            m6 = mx(m6, A(i, j, k, 0, l, m));
                        }
                        A(i, j, k, l, 0, 0) = m1;
                        A(i, j, k, 0, 0, l) = m2;
                        A(i, j, 0, 0, k, l) = m3;
                        A(i, j, k, 0, l, 0) = m6;
                        A(i, j, 0, k, 0, l) = m5;
                        A(i, j, 0, k, l, 0) = m4;
                    }
        for (int i = 1; i < P; ++i)
            for (int j = 1; j < P; ++j)
                for (int k = 1; k < 5; ++k) {
                    int m1 = -kINF, m2 = -kINF, m3 = -kINF, m4 = -kINF;
                    for (int l = 1; l < 5; ++l) {
                        m1 = mx(m1, A(i, j, k, l, 0, 0));
                        m2 = mx(m2, A(i, j, 0, k, l, 0));
                        m3 = mx(m3, A(i, j, 0, 0, k, l));
                        m4 = mx(m4, A(i, j, 0, 0, l, k));
                    }
                    A(i, j, k, 0, 0, 0) = m1;
                    A(i, j, 0, k, 0, 0) = m2;
                    A(i, j, 0, 0, k, 0) = m3;
                    A(i, j, 0, 0, 0, k) = m4;
                }
        for (int i = 1; i < P; ++i)
            for (int j = 1; j < P; ++j) {
                int m1 = -kINF;
                for (int k = 1; k < 5; ++k) m1 = mx(m1, A(i, j, k, 0, 0, 0));
                A(i, j, 0, 0, 0, 0) = m1;
            }
        // non-standard pairs: one, then both
        for (int i = 1; i < P; ++i)
            for (int k = 0; k < 5; ++k)
                for (int l = 0; l < 5; ++l)
                    for (int m = 0; m < 5; ++m)
                        for (int n = 0; n < 5; ++n) {
                            int m1 = -kINF, m2 = -kINF;
                            for (int j = 1; j < P; ++j) {
                                m1 = mx(m1, A(i, j, k, l, m, n));
                                m2 = mx(m2, A(j, i, k, l, m, n));
                            }
                            A(i, P, k, l, m, n) = m1;
                            A(P, i, k, l, m, n) = m2;
                        }
        for (int k = 0; k < 5; ++k)
            for (int l = 0; l < 5; ++l)
                for (int m = 0; m < 5; ++m)
                    for (int n = 0; n < 5; ++n) {
                        int m1 = -kINF;
                        for (int j = 1; j < P; ++j) m1 = mx(m1, A(P, j, k, l, m, n));
                        A(P, P, k, l, m, n) = m1;
                    }
    }

    // io.c:1126 — one warning per asymmetric element, in the reference's order.
    void check_symmetry() {
        auto S = [](const int *s, int i, int j) { return s[i * NP + j]; };
        const int *st = &w_.stack[0][0];
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                if (S(st, i, j) != S(st, j, i)) warn("stacking energies not symmetric");
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                if (S(stackH_.data(), i, j) != S(stackH_.data(), j, i)) warn("stacking enthalpies not symmetric");
        auto I11 = [](const int *a, int i, int j, int k, int l) { return a[((i * NP + j) * 5 + k) * 5 + l]; };
        const int *e11 = &w_.int11[0][0][0][0];
        char buf[160];
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                for (int k = 0; k < 5; ++k)
                    for (int l = 0; l < 5; ++l)
                        if (I11(e11, i, j, k, l) != I11(e11, j, i, l, k)) {
                            snprintf(buf, sizeof buf, "int11 energies not symmetric (%d,%d,%d,%d) (%d vs. %d)", i, j, k,
                                     l, I11(e11, i, j, k, l), I11(e11, j, i, l, k));
                            warn(buf);
                        }
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                for (int k = 0; k < 5; ++k)
                    for (int l = 0; l < 5; ++l)
                        if (I11(int11H_.data(), i, j, k, l) != I11(int11H_.data(), j, i, l, k))
                            warn("int11 enthalpies not symmetric");
        auto I22 = [](const int *a, int i, int j, int k, int l, int m, int n) {
            return a[((((i * NP + j) * 5 + k) * 5 + l) * 5 + m) * 5 + n];
        };
        const int *e22 = &w_.int22[0][0][0][0][0][0];
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                for (int k = 0; k < 5; ++k)
                    for (int l = 0; l < 5; ++l)
                        for (int m = 0; m < 5; ++m)
                            for (int n = 0; n < 5; ++n)
                                if (I22(e22, i, j, k, l, m, n) != I22(e22, j, i, m, n, k, l))
                                    warn("int22 energies not symmetric");
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < NP; ++j)
                for (int k = 0; k < 5; ++k)
                    for (int l = 0; l < 5; ++l)
                        for (int m = 0; m < 5; ++m)
                            for (int n = 0; n < 5; ++n)
                                if (I22(int22H_.data(), i, j, k, l, m, n) != I22(int22H_.data(), j, i, m, n, k, l)) {
                                    snprintf(buf, sizeof buf, "int22 enthalpies not symmetric: %d %d %d %d %d %d", i, j,
                                             k, l, m, n);
                                    warn(buf);
                                }
    }
};

void put_log(const std::string &s, char *log, int cap) {
    if (!log || cap <= 0) return;
    size_t n = s.size() < (size_t)(cap - 1) ? s.size() : (size_t)(cap - 1);
    memcpy(log, s.data(), n);
    log[n] = 0;
}

bool base_ok(const ccj_energy_params *b) {
    return b && b->magic == CCJ_PARAMS_MAGIC && b->size_bytes == sizeof(ccj_energy_params);
}

int apply(std::vector<std::string> lines, const ccj_energy_params *base, ccj_energy_params *out, char *log, int cap) {
    ParReader r(std::move(lines), *base);
    int rc;
    try {
        rc = r.run();
    } catch (const Fatal &f) {
        put_log(r.messages + "ERROR: " + f.msg + "\n", log, cap);
        return CCJ_E_PARFILE;
    }
    if (rc == 1) r.finish(*out);
    else *out = *base;
    put_log(r.messages, log, cap);
    return rc;
}

}  // namespace

extern "C" int ccj_params_load_par(const char *path, const ccj_energy_params *base, ccj_energy_params *out, char *log,
                                   int log_cap) {
    if (!path || !out || !base_ok(base)) return -1;
    FILE *f = fopen(path, "r");
    if (!f) {
        *out = *base;
        put_log(std::string("WARNING: read_parameter_file():Can't open file ") + path + "\n\n", log, log_cap);
        return 0;
    }
    // vrna_read_line (io_utils.c:79): lines of any length, '\n' removed, no trailing empty line
    std::vector<std::string> lines;
    std::string cur;
    bool open_line = false;
    for (int c; (c = fgetc(f)) != EOF;) {
        if (c == '\n') {
            lines.push_back(cur.c_str());  // a NUL byte ends what strlen() sees
            cur.clear();
            open_line = false;
        } else {
            cur.push_back((char)c);
            open_line = true;
        }
    }
    if (open_line) lines.push_back(cur.c_str());
    fclose(f);
    return apply(std::move(lines), base, out, log, log_cap);
}

extern "C" int ccj_params_load_par_string(const char *text, const ccj_energy_params *base, ccj_energy_params *out,
                                          char *log, int log_cap) {
    if (!out || !base_ok(base)) return -1;
    if (!text) {
        *out = *base;
        put_log("", log, log_cap);
        return 0;
    }
    std::vector<std::string> lines;  // strtok_r(.., "\n"): empty lines vanish
    for (const char *p = text; *p;) {
        const char *e = strchr(p, '\n');
        size_t n = e ? (size_t)(e - p) : strlen(p);
        if (n) lines.emplace_back(p, n);
        p += n + (e ? 1 : 0);
    }
    return apply(std::move(lines), base, out, log, log_cap);
}
