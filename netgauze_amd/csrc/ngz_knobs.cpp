// Experiment knobs and diagnostics: the only place the library reads its environment.
//
// The product library takes no tuning from the environment: every knob below returns its
// default, so a collector's environment cannot change which kernels run or how the columns
// are laid out.  Behaviour a host may choose is an option of the C ABI instead
// (ngz_ctx_set_option, ngz_agg_set_option).  A build with -DNGZ_EXPERIMENTS
// (tools/build_experiments.sh: netgauze_amd/libngz_exp.so, never the product library) reads
// NGZ_<name> for the A/B measurements DESIGN.md reports.  Diagnostics stay environment-driven
// in every build: NGZ_DEBUG prints host-side traces to stderr and changes nothing else.
#include <cstdlib>

#include "ngz_internal.h"

static const char *knob_env(const char *name) {
#ifdef NGZ_EXPERIMENTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

int64_t ngz_knob(const char *name, int64_t dflt) {
    const char *e = knob_env(name);
    return e && *e ? atoll(e) : dflt;
}

const char *ngz_knob_str(const char *name, const char *dflt) {
    const char *e = knob_env(name);
    return e && *e ? e : dflt;
}

bool ngz_debug() {
    static const bool on = getenv("NGZ_DEBUG") != nullptr;
    return on;
}

extern "C" int ngz_experiments_build() {
#ifdef NGZ_EXPERIMENTS
    return 1;
#else
    return 0;
#endif
}
