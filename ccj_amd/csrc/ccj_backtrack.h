// ccj_backtrack.h — backtrack node types and the exit records shared by the host traceback
// (ccj_host.cc, over the host mirror) and the device traceback (ccj_backtrack.hip).
#pragma once
#include <stdint.h>

namespace ccj {

// backtrack interval types, reference constants.hh:21-73
constexpr char T_NONE = 'N', T_HAIRP = 'H', T_INTER = 'I', T_MULTI = 'M';
constexpr char M_WM = 'B', M_WMv = 'v', M_WMp = 'p', FREE = 'W', LOOP = 'V';
constexpr char P_P = 'P', P_PK = 'k', P_PL = 'l', P_PR = 'r', P_PM = 'm', P_PO = 'o';
constexpr char P_PfromL = 'f', P_PfromR = 'g', P_PfromM = 'h', P_PfromMprime = '[', P_PfromMdoubleprime = ']',
               P_PfromO = 'i';
constexpr char P_PLiloop = 'j', P_PLiloop5 = 'b', P_PLmloop = 'c', P_PLmloop10 = 'e', P_PLmloop01 = 'n',
               P_PLmloop00 = 'a';
constexpr char P_PRiloop = 'q', P_PRiloop5 = 's', P_PRmloop = 't', P_PRmloop10 = 'u', P_PRmloop01 = '&',
               P_PRmloop00 = '9';
constexpr char P_PMiloop = 'w', P_PMiloop5 = 'x', P_PMmloop = 'y', P_PMmloop10 = '0', P_PMmloop01 = '1',
               P_PMmloop00 = '8';
constexpr char P_POiloop = 'z', P_POiloop5 = '5', P_POmloop = '+', P_POmloop10 = '-', P_POmloop01 = '=',
               P_POmloop00 = '_';
constexpr char P_WB = '*', P_WBP = '^', P_WP = '#', P_WPP = '@';

struct Interval {  // reference h_struct.hh:65-92 (seq_interval)
    int i, j, k, l;
    int type;  // one of the chars above
};

// How a traceback ended (device record; the host turns it into the reference's exit).
enum BtStatus : int {
    BT_OK = 0,
    BT_DIE = 1,        // exit(EXIT_FAILURE) after "<prefix>This should not have happened!, <case>"
    BT_INTER = 2,      // "NOT GOOD RESTR INTER, ..." then exit(0) (W_final.cc:224-225)
    BT_ASSERT = 3,     // Matrix4D::get_uc assert (matrices.hh:167), exit 134
    BT_OVERFLOW = 4,   // device stack capacity exceeded (engine limit, not a reference exit)
};
// message prefixes of the reference's "This should not have happened!" exits
constexpr int BT_NPREFIX = 7;
inline const char *bt_prefix(int p) {
    static const char *tab[BT_NPREFIX] = {"", "border case: ", "border cases: ", "boder cases: ", "impossible cases: ",
                                          "impossible case: ", "impossbible cases: "};
    return (p >= 0 && p < BT_NPREFIX) ? tab[p] : "";
}

struct BtOut {
    int status;      // BtStatus
    int prefix;      // BT_DIE: message prefix id
    int node;        // BT_DIE: node type (case name)
    int args[4];     // BT_INTER: i, j, best_ip, best_jp
    int n_snbh;      // "Should not be here!" lines (A-B1)
    int steps;       // nodes processed
    int pad;
};

inline const char *bt_case_name(int type) {
    switch (type) {
        case P_P: return "P_P";
        case P_PK: return "P_PK";
        case P_PL: return "P_PL";
        case P_PR: return "P_PR";
        case P_PM: return "P_PM";
        case P_PO: return "P_PO";
        case P_PfromL: return "P_PfromL";
        case P_PfromR: return "P_PfromR";
        case P_PfromM: return "P_PfromM";
        case P_PfromO: return "P_PfromO";
        case P_WB: return "P_WB";
        case P_WBP: return "P_WBP";
        case P_WP: return "P_WP";
        case P_WPP: return "P_WPP";
        case P_PLiloop: return "P_PLiloop";
        case P_PLmloop: return "P_PLmloop";
        case P_PLmloop00: return "P_PLmloop00";
        case P_PLmloop01: return "P_PLmloop01";
        case P_PLmloop10: return "P_PLmloop10";
        case P_PRiloop: return "P_PRiloop";
        case P_PRmloop: return "P_PRmloop";
        case P_PRmloop00: return "P_PRmloop00";
        case P_PRmloop01: return "P_PRmloop01";
        case P_PRmloop10: return "P_PRmloop10";
        case P_PMiloop: return "P_PMiloop";
        case P_PMmloop: return "P_PMmloop";
        case P_PMmloop00: return "P_PMmloop00";
        case P_PMmloop01: return "P_PMmloop01";
        case P_PMmloop10: return "P_PMmloop10";
        case P_POiloop: return "P_POiloop";
        case P_POmloop: return "P_POmloop";
        case P_POmloop00: return "P_POmloop00";
        case P_POmloop01: return "P_POmloop01";
        case P_POmloop10: return "P_POmloop10";
    }
    return "?";
}

}  // namespace ccj

extern "C" {
// One-workgroup kernels (ccj_backtrack.hip): W (W_final.cc:68-79) into W[0..n], then the whole
// traceback into f_pair/f_type (h_struct.hh:9-19) and *out.  stack_cap = device stack entries.
int ccjk_compute_W(const void *T, int *W, int *S, void *stream);  // S: (n+1)*rs ints of scratch
int ccjk_backtrack(const void *T, const int *W, int *f_pair, int8_t *f_type, ccj::BtOut *out, int stack_cap,
                   void *stream);
}
