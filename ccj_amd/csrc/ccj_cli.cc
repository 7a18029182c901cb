// ccj_cli.cc — the `CCJ` command line on top of libccj_hip.so (drop-in for reference src/CCJ.cc).
//
//   CCJ [-h] [-V] [-i FILE] [-d N] [-P paramfile] [--noConv] [--noGU] [sequence]
//
// Option handling follows the gengetopt parser the reference is built with (src/ccj.ggo:1-33,
// src/cmdline.cc:505-640, update_arg cmdline.cc:375-470): the same getopt_long table (so the
// same prefix matching, permutation and glibc messages with argv[0]), -h / -V print and exit 0
// as soon as they are seen, a repeated option is "`--x' (`-c') option given more than once",
// -d goes through strtol(base 0) and rejects trailing characters with "invalid numeric value".
// Main body follows reference CCJ.cc:58-115: sequence from the first non-option argument or the
// first stdin line (not read at all when -i is given), toupper, T->U unless --noConv, validation
// messages on stdout + exit 1, "Not a valid parameter file!" on stderr + exit 1 for a -P path that
// does not exist, DNA Mathews 2004 + noGU when a 'T' survives, output "SEQ\nSTRUCT (E)\n" with
// std::cout's default double formatting, and the reference's backtrack exits.
// Parameter files: -P reads any ViennaRNA v2.0 .par file natively (ccj_parfile.h) on top of the
// compiled-in defaults, printing the reference loader's warnings/errors; a *.ccjp path is taken as
// one of our table blobs.  Without -P the reference loads params/rna_DirksPierce09.par relative
// to the CWD: that file is read when present, otherwise the bundled DirksPierce09 tables are used
// (the reference would print "Not a valid parameter file!" there).
// Device: $CCJ_DEVICE (default 0) — the reference has no device option, so none is added.
#include <getopt.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "ccj.h"
#include "ccj_parfile.h"

static const char kHelp[] =
    "Usage: CCJ [options] [sequence]\n"
    "Pseudoknotted minimum free energy folding of RNAs\n"
    "\n"
    "Read RNA sequence from stdin or cmdline; predict minimum\n"
    "free energy and optimum structure\n"
    "\n"
    "  -h, --help               Print help and exit\n"
    "  -V, --version            Print version and exit\n"
    "  -i, --input-file=STRING  Give a path to an input file containing the sequence\n"
    "                             (and input structure if known)\n"
    "  -d, --dangles=INT        Specify the dangle model to be used (base is 2)\n"
    "                             (default=`2')\n"
    "  -P, --paramFile=STRING   Read energy parameters from paramfile, instead of\n"
    "                             using the default parameter set.\n"
    "      --noConv             Do not convert DNA into RNA. This will use the\n"
    "                             Matthews 2004 parameters for DNA  (default=off)\n"
    "      --noGU               Turn off G-U and U-G (and G-T and T-G) base pairing\n"
    "                             (default=off)\n"
    "\n"
    "The input sequence is read from standard input, unless it is\n"
    "given on the command line.\n"
    "\n";

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

static bool read_blob(const std::string &path, std::vector<char> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return out.size() == sizeof(ccj_energy_params);
}

static std::string bundled(const char *name) { return exe_dir() + "/../params/" + name + ".ccjp"; }

// vrna_params_load on top of the compiled-in defaults; 0 ok, 1 = reference would exit(1).
static int load_par_file(const std::string &path, std::vector<char> &blob) {
    std::vector<char> base;
    if (!read_blob(bundled("default"), base)) {
        std::cerr << "CCJ: missing " << bundled("default") << std::endl;
        return 1;
    }
    blob.assign(sizeof(ccj_energy_params), 0);
    std::vector<char> log(1 << 22);
    int rc = ccj_params_load_par(path.c_str(), reinterpret_cast<const ccj_energy_params *>(base.data()),
                                 reinterpret_cast<ccj_energy_params *>(blob.data()), log.data(), (int)log.size());
    std::cerr << log.data();
    if (rc == CCJ_E_PARFILE) return 1;
    return 0;
}

struct Args {
    int dangles = 2;
    bool input_given = false, noConv = false, noGU = false, paramFile_given = false;
    std::string paramFile;
    std::vector<std::string> inputs;
};

// gengetopt's cmdline_parser: 0 ok, 1 failure (message printed), -1 help/version printed.
static int parse(int argc, char *argv[], Args &a) {
    static option table[] = {{"help", no_argument, nullptr, 'h'},          {"version", no_argument, nullptr, 'V'},
                             {"input-file", required_argument, nullptr, 'i'}, {"dangles", required_argument, nullptr, 'd'},
                             {"paramFile", required_argument, nullptr, 'P'},  {"noConv", no_argument, nullptr, 0},
                             {"noGU", no_argument, nullptr, 0},               {nullptr, 0, nullptr, 0}};
    const char *prog = argv[0];
    int given_i = 0, given_d = 0, given_P = 0, given_conv = 0, given_gu = 0;
    auto twice = [&](int &g, const char *lng, char sht) {
        if (g++ == 0) return false;
        if (sht) fprintf(stderr, "%s: `--%s' (`-%c') option given more than once\n", prog, lng, sht);
        else fprintf(stderr, "%s: `--%s' option given more than once\n", prog, lng);
        return true;
    };
    opterr = 1;
    for (;;) {
        int idx = 0;
        int c = getopt_long(argc, argv, "hVi:d:P:", table, &idx);
        if (c == -1) break;
        switch (c) {
            case 'h': fputs(kHelp, stdout); return -1;
            case 'V': fputs("CCJ 1.0\n", stdout); return -1;
            case 'i':
                if (twice(given_i, "input-file", 'i')) return 1;
                a.input_given = true;
                break;
            case 'd': {
                if (twice(given_d, "dangles", 'd')) return 1;
                char *stop = nullptr;
                a.dangles = (int)strtol(optarg, &stop, 0);
                if (!(stop && *stop == '\0')) {
                    fprintf(stderr, "%s: invalid numeric value: %s\n", prog, optarg);
                    return 1;
                }
                break;
            }
            case 'P':
                if (twice(given_P, "paramFile", 'P')) return 1;
                a.paramFile_given = true;
                a.paramFile = optarg;
                break;
            case 0:
                if (!strcmp(table[idx].name, "noConv")) {
                    if (twice(given_conv, "noConv", 0)) return 1;
                    a.noConv = true;
                } else {
                    if (twice(given_gu, "noGU", 0)) return 1;
                    a.noGU = true;
                }
                break;
            default: return 1;  // getopt_long already printed the message
        }
    }
    for (int k = optind; k < argc; ++k) a.inputs.push_back(argv[k]);
    return 0;
}

int main(int argc, char *argv[]) {
    Args a;
    int pr = parse(argc, argv, a);
    if (pr < 0) return EXIT_SUCCESS;
    if (pr > 0) return 1;
    const char *dev_env = getenv("CCJ_DEVICE");
    int device = dev_env ? atoi(dev_env) : 0;

    std::string seq;
    if (!a.inputs.empty()) seq = a.inputs[0];
    else if (!a.input_given) std::getline(std::cin, seq);
    std::transform(seq.begin(), seq.end(), seq.begin(), ::toupper);
    if (!a.noConv)
        for (char &c : seq)
            if (c == 'T') c = 'U';
    int noGU = a.noGU;
    if (seq.empty()) {
        std::cout << "sequence is missing" << std::endl;
        return EXIT_FAILURE;
    }
    for (char c : seq)
        if (!(c == 'G' || c == 'C' || c == 'A' || c == 'U' || c == 'T')) {
            std::cout << "Sequence contains character " << c << " that is not G,C,A,U, or T." << std::endl;
            return EXIT_FAILURE;
        }
    std::vector<char> blob;
    if (a.paramFile_given) {
        if (!exists(a.paramFile)) {
            std::cerr << "Not a valid parameter file!" << std::endl;
            return EXIT_FAILURE;
        }
        size_t L = a.paramFile.size();
        if (L > 5 && a.paramFile.compare(L - 5, 5, ".ccjp") == 0) {
            if (!read_blob(a.paramFile, blob)) {
                std::cerr << "Not a valid parameter file!" << std::endl;
                return EXIT_FAILURE;
            }
        } else if (load_par_file(a.paramFile, blob)) {
            return EXIT_FAILURE;
        }
    } else if (seq.find('T') != std::string::npos) {
        noGU = 1;
        read_blob(bundled("DNA_Mathews2004"), blob);
        // vrna_params_load_DNA_Mathews2004 ends in check_symmetry (io.c:1126); the built-in DNA
        // set has two asymmetric stack-enthalpy pairs, so the reference always prints this
        for (int w = 0; w < 4; ++w) std::cerr << "WARNING: stacking enthalpies not symmetric" << std::endl;
    } else if (exists("params/rna_DirksPierce09.par")) {
        if (load_par_file("params/rna_DirksPierce09.par", blob)) return EXIT_FAILURE;
    } else {
        read_blob(bundled("DirksPierce09"), blob);
    }
    if (blob.size() != sizeof(ccj_energy_params)) {
        std::cerr << "CCJ: bundled parameter tables missing next to " << exe_dir() << std::endl;
        return 2;
    }
    ccj_problem prob{seq.c_str(), a.dangles, noGU, reinterpret_cast<const ccj_energy_params *>(blob.data()), nullptr};
    ccj_options o{device, 0, 0, 0, 0, 0, 0, 0};  // fill + traceback on the GPU
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
