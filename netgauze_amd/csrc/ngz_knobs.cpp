// Experiment knobs and diagnostics: the only place the library reads its environment.
//
// The product library takes no tuning from the environment: every knob below returns its
// default, so a collector's environment cannot change which kernels run or how the columns
// are laid out.  Behaviour a host may choose is an option of the C ABI instead
// (ngz_ctx_set_option, ngz_agg_set_option).  A build with -DNGZ_EXPERIMENTS
// (tools/build_experiments.sh: tools/exp/libngz_exp.so, never the product library) reads
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

// NGZ_DEBUG set: host-side traces (level 1); NGZ_DEBUG=2 also dumps the generated source of every
// template kernel compile (many templates flood stderr, so it is not part of level 1)
int ngz_debug_level() {
    static const int lvl = [] {
        const char *e = getenv("NGZ_DEBUG");
        if (e == nullptr) return 0;
        return atoi(e) >= 2 ? 2 : 1;
    }();
    return lvl;
}

bool ngz_debug() { return ngz_debug_level() > 0; }

extern "C" int ngz_experiments_build() {
#ifdef NGZ_EXPERIMENTS
    return 1;
#else
    return 0;
#endif
}
