/*
 * ccj_parfile.h — native reader for ViennaRNA "RNAfold parameter file v2.0" (.par) files,
 * producing the engine's scaled 37 C table blob (ccj_params.h).  Part of libccj_hip.so.
 *
 * Replaces, for the CCJ path, the reference's
 *   vrna_params_load()              src/ViennaRNA/params/io.c:252-276
 *   vrna_params_load_from_string()  src/ViennaRNA/params/io.c:287-335
 *   set_parameters_from_string()    src/ViennaRNA/params/io.c:454-673
 * followed by get_scaled_params() at 37 C (src/ViennaRNA/params/params.c:399-555), which is what
 * W_final's constructor ends up reading.  The reference mutates process-global tables, so a
 * load always lands on top of whatever was in force: `base` is that state (ccj_amd/params/
 * default.ccjp = the compiled-in Turner 2004 defaults, as at reference CCJ.cc start-up).
 *
 * Return value (vrna_params_load's):  1 = file parsed and applied, 0 = nothing applied (file
 * could not be opened or was empty; *out = *base).  CCJ_E_PARFILE = the reference would have
 * called vrna_message_error() and exit(1) mid-file; *out is then undefined.
 * `log` receives exactly what the reference prints on stderr while loading ("WARNING: ..." /
 * "ERROR: ..." lines, non-tty form), NUL-terminated and truncated to log_cap bytes.
 */
#ifndef CCJ_PARFILE_H
#define CCJ_PARFILE_H

#include "ccj_params.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CCJ_E_PARFILE 8 /* .par syntax error: reference prints "ERROR: ..." and exits 1 */

/* reference: vrna_params_load (io.c:252) + get_scaled_params (params.c:399) */
int ccj_params_load_par(const char *path, const ccj_energy_params *base, ccj_energy_params *out, char *log,
                        int log_cap);

/* reference: vrna_params_load_from_string (io.c:287) + get_scaled_params; empty lines are
 * dropped (strtok on "\n"), unlike the file reader. */
int ccj_params_load_par_string(const char *text, const ccj_energy_params *base, ccj_energy_params *out, char *log,
                               int log_cap);

#ifdef __cplusplus
}
#endif

#endif /* CCJ_PARFILE_H */
