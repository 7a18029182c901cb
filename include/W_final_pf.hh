/*
 * W_final_pf.hh — C++ drop-in for the reference's partition-function class, over ccj_pf.h.
 *
 * Mirrors reference src/part_func.hh:28-62 (the public surface a caller uses):
 *     W_final_pf(std::string &seq, std::string &MFE_structure, double MFE_energy, int dangle,
 *                int num_samples, bool PSplot);   ~W_final_pf();   pf_t ccj_pf();
 *     std::string structure;   int num_samples;   std::unordered_map<std::string, int> structures;
 * The constructor snapshots the parameter tables in force (vrna_params_load & co. of W_final.hh;
 * scale_pf_parameters() in part_func.cc:32) and the PK penalty globals; ccj_pf() runs the fill on
 * the GPU ($CCJ_DEVICE, default 0) and returns the ensemble free energy, bit-identical to
 * part_func.cc built without floating-point contraction; like the reference it sets `structure`
 * to n dots (part_func.cc:175).
 * Extension: sample(k) draws k structures with the reference's stochastic traceback
 * (Sample_W(1, n), stoch_backtrack.cc) from this object's rand() stream (srand_samples reseeds
 * it); on the reference's "backtracking failed" paths it prints the same line and exit(0)s.
 */
#ifndef CCJ_W_FINAL_PF_HH
#define CCJ_W_FINAL_PF_HH
#ifndef PART_FUNC
#define PART_FUNC
#endif

#include <string>
#include <unordered_map>
#include <vector>

#include "W_final.hh"

struct ccj_pf_ctx;
typedef double pf_t;

class W_final_pf {
   public:
    std::string structure;
    int num_samples;
    std::unordered_map<std::string, int> structures;

    W_final_pf(std::string &seq, std::string &MFE_structure, double MFE_energy, int dangle, int num_samples, bool PSplot);
    ~W_final_pf();
    W_final_pf(const W_final_pf &) = delete;
    W_final_pf &operator=(const W_final_pf &) = delete;

    pf_t ccj_pf();

    // extensions
    std::vector<std::string> sample(int k);
    void srand_samples(unsigned int seed);

   private:
    std::string seq_;
    ccj_pf_ctx *ctx_ = nullptr;
    bool filled_ = false;
};

#endif /* CCJ_W_FINAL_PF_HH */
