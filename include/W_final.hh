/*
 * W_final.hh — C++ drop-in for the reference's fold class, over the C ABI in ccj.h.
 *
 * Mirrors reference src/W_final.hh:18-30 (the public surface a caller uses):
 *     W_final(std::string seq, int dangle);   ~W_final();   double ccj();
 *     vrna_param_t *params_;                   std::string structure;
 * plus the parameter-loading globals the reference's CCJ.cc reaches through ViennaRNA
 * (ViennaRNA/params/io.h vrna_params_load / vrna_params_load_DNA_Mathews2004, the `noGU` global of
 * ViennaRNA/model.c), so the reference's own driver src/CCJ.cc compiles and links unchanged against
 * this header and libccj_hip.so (tests/test_wfinal_facade.py does exactly that).
 *
 * Behaviour follows the reference:
 *   - the constructor snapshots the parameter tables in force (scale_parameters() in
 *     W_final.cc:23) and the `noGU` global; ccj() returns W[n]/100 and fills `structure`;
 *   - the reference's stdout side messages ("Should not be here!", W_final.cc:715) go to stdout,
 *     and where its backtrack calls exit()/abort() (pseudo_loop.cc:873-875 passim) this does too,
 *     with the same stderr text and status;
 *   - the PK penalties are the program's `PS_penalty` ... `cp_penalty` globals when it defines
 *     them (the reference's h_globals.hh does), else the reference defaults;
 *   - the stock build's n >= 214 assert abort (matrices.hh:160) is reproduced only when
 *     CCJ_REF_COMPAT_ABORT=1; by default every n that fits in HBM folds.
 * Engine failures the reference cannot have (no GPU, out of device memory) throw
 * std::runtime_error.  The GPU is $CCJ_DEVICE (default 0).
 */
#ifndef CCJ_W_FINAL_HH
#define CCJ_W_FINAL_HH
/* the reference header's guard too, so a translation unit that still finds the reference's own
 * W_final.hh on its include path (e.g. next to an unmodified CCJ.cc) gets this one, not both */
#ifndef W_FINAL_H_
#define W_FINAL_H_
#endif

#include <string>

#include "ccj_params.h"

extern "C" {
/* the scaled 37 C tables; field names follow ViennaRNA's vrna_param_t (params/basic.h:57-115) */
typedef ccj_energy_params vrna_param_t;
#ifndef VRNA_PARAMETER_FORMAT_DEFAULT
#define VRNA_PARAMETER_FORMAT_DEFAULT 0
#endif
/* reference ViennaRNA/params/io.c:252: overlay a v2.0 .par file on the tables in force; 1 applied,
 * 0 not (unreadable/empty file); a syntax error prints the reference's ERROR text and exit(1)s */
int vrna_params_load(const char *fname, unsigned int options);
/* reference io.c:1110: the built-in DNA Mathews 2004 set (prints its 4 symmetry warnings) */
int vrna_params_load_DNA_Mathews2004(void);
/* reference ViennaRNA/model.c:54 */
extern int noGU;
}

struct ccj_ctx;

/* Extension (no reference counterpart): make `tables` the tables in force (e.g. a .ccjp blob). */
void ccj_wfinal_use_tables(const ccj_energy_params &tables);

class W_final {
   public:
    W_final(std::string seq, int dangle);
    ~W_final();
    W_final(const W_final &) = delete;
    W_final &operator=(const W_final &) = delete;

    double ccj();

    vrna_param_t *params_;
    std::string structure;  // MFE structure (dot-bracket, length n) after ccj()

   private:
    std::string seq_;
    int dangle_;
    int noGU_;
    vrna_param_t tables_;
    ccj_ctx *ctx_ = nullptr;
};

#endif /* CCJ_W_FINAL_HH */
