// ccj_cli.cc — the `CCJ` command line on top of libccj_hip.so (drop-in for reference src/CCJ.cc).
//
//   CCJ [-i FILE] [-d N] [-P paramfile] [--noConv] [--noGU] [sequence]
//
// Mirrors reference CCJ.cc:58-115 and ccj.ggo:13-31: sequence from argv[0] or the first stdin
// line (not read at all when -i is given), toupper, T->U unless --noConv, validation messages on
// stdout + exit 1, "Not a valid parameter file!" on stderr + exit 1, DNA Mathews 2004 + noGU when
// a 'T' survives, output "SEQ\nSTRUCT (E)\n" with std::cout's default double formatting, and the
// reference's backtrack exits (stderr text + exit code).
// Parameter files: -P takes one of our table blobs (*.ccjp) or the name of a reference parameter
// file (rna_Turner04.par, ...), resolved to the blob dumped from it (ccj_amd/params/).
// Without -P the DirksPierce09 tables are used (the reference reads params/rna_DirksPierce09.par
// relative to the CWD and fails elsewhere).
#include <getopt.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "ccj.h"

static bool exists(const std::string &p) {
    struct stat b;
    return stat(p.c_str(), &b) == 0;
}

static std::string exe_dir() {
    char buf[4096];
    ssize_t r = readlink("/proc/self/exe", buf, sizeof buf - 1);
    if (r <= 0) return ".";
    buf[r] = 0;
    std::string s(buf);
    return s.substr(0, s.find_last_of('/'));
}

static std::string blob_for(const std::string &arg) {
    if (arg.size() > 5 && arg.substr(arg.size() - 5) == ".ccjp") return arg;
    std::string base = arg.substr(arg.find_last_of('/') + 1);
    if (base.size() > 4 && base.substr(base.size() - 4) == ".par") base = base.substr(0, base.size() - 4);
    static const char *map[][2] = {{"rna_Turner04", "Turner04"},           {"rna_DirksPierce09", "DirksPierce09"},
                                   {"rna_DirksPierce03", "DirksPierce03"}, {"rna_CaoChen06", "CaoChen06"},
                                   {"rna_CaoChen09", "CaoChen09"},         {"dna_Matthews04", "Matthews04"}};
    for (auto &m : map)
        if (base == m[0] || base == m[1]) return exe_dir() + "/../params/" + m[1] + ".ccjp";
    return "";
}

static bool read_blob(const std::string &path, std::vector<char> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return out.size() == sizeof(ccj_energy_params);
}

int main(int argc, char *argv[]) {
    int dangles = 2, noConv = 0, noGU_flag = 0, input_given = 0, device = 0;
    std::string param_file;
    static option opts[] = {{"input-file", required_argument, nullptr, 'i'}, {"dangles", required_argument, nullptr, 'd'},
                            {"paramFile", required_argument, nullptr, 'P'},  {"noConv", no_argument, nullptr, 1},
                            {"noGU", no_argument, nullptr, 2},               {"device", required_argument, nullptr, 3},
                            {"help", no_argument, nullptr, 'h'},             {"version", no_argument, nullptr, 'V'},
                            {nullptr, 0, nullptr, 0}};
    int ch;
    while ((ch = getopt_long(argc, argv, "i:d:P:hV", opts, nullptr)) != -1) {
        switch (ch) {
            case 'i': input_given = 1; break;
            case 'd': dangles = atoi(optarg); break;
            case 'P': param_file = optarg; break;
            case 1: noConv = 1; break;
            case 2: noGU_flag = 1; break;
            case 3: device = atoi(optarg); break;
            case 'h':
                std::cout << "Usage: CCJ [options] [sequence]\n  -i, --input-file=STRING\n  -d, --dangles=INT (default=`2')\n"
                             "  -P, --paramFile=STRING\n      --noConv\n      --noGU\n";
                return 0;
            case 'V': std::cout << "CCJ 1.0 (MI355X engine)\n"; return 0;
            default: return 1;
        }
    }
    std::string seq;
    if (optind < argc) seq = argv[optind];
    else if (!input_given) std::getline(std::cin, seq);
    std::transform(seq.begin(), seq.end(), seq.begin(), ::toupper);
    if (!noConv)
        for (char &c : seq)
            if (c == 'T') c = 'U';
    int noGU = noGU_flag;
    if (seq.empty()) {
        std::cout << "sequence is missing" << std::endl;
        return EXIT_FAILURE;
    }
    for (char c : seq)
        if (!(c == 'G' || c == 'C' || c == 'A' || c == 'U' || c == 'T')) {
            std::cout << "Sequence contains character " << c << " that is not G,C,A,U, or T." << std::endl;
            return EXIT_FAILURE;
        }
    std::string blob_path;
    if (!param_file.empty()) {
        if (!exists(param_file)) {
            std::cerr << "Not a valid parameter file!" << std::endl;
            return EXIT_FAILURE;
        }
        blob_path = blob_for(param_file);
    } else if (seq.find('T') != std::string::npos) {
        noGU = 1;
        blob_path = exe_dir() + "/../params/DNA_Mathews2004.ccjp";
    } else {
        blob_path = exe_dir() + "/../params/DirksPierce09.ccjp";
    }
    std::vector<char> blob;
    if (blob_path.empty() || !read_blob(blob_path, blob)) {
        std::cerr << "Not a valid parameter file!" << std::endl;
        return EXIT_FAILURE;
    }
    ccj_problem prob{seq.c_str(), dangles, noGU, reinterpret_cast<const ccj_energy_params *>(blob.data()), nullptr};
    ccj_options o{device, 0, 0, 0, 0, 0};  // fill + traceback on the GPU
    ccj_ctx *ctx = nullptr;
    int rc = ccj_create(&prob, &o, &ctx);
    if (rc != CCJ_OK) {
        std::cerr << "CCJ: engine error " << rc << ": " << ccj_last_error(ctx) << std::endl;
        return 2;
    }
    rc = ccj_fill(ctx);
    if (rc != CCJ_OK) {
        std::cerr << "CCJ: engine error " << rc << ": " << ccj_last_error(ctx) << std::endl;
        ccj_destroy(ctx);
        return 2;
    }
    std::string structure(seq.size() + 1, '\0');
    std::vector<char> msgs(1 << 16);
    double energy = 0;
    rc = ccj_result(ctx, &structure[0], &energy, msgs.data(), (int)msgs.size());
    std::cout << msgs.data();
    if (rc == CCJ_E_BACKTRACK || rc == CCJ_E_INTER_EXIT) {
        std::string err = ccj_last_error(ctx);
        std::cout.flush();
        std::cerr << err;
        ccj_destroy(ctx);
        return rc == CCJ_E_INTER_EXIT ? 0 : (err.find("Assertion") != std::string::npos ? 134 : EXIT_FAILURE);
    }
    structure.resize(seq.size());
    std::cout << seq << std::endl;
    std::cout << structure << " (" << energy << ")" << std::endl;
    ccj_destroy(ctx);
    return 0;
}
