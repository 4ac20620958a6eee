// mof_knobs.cpp -- the only place libmofhip reads its environment (mof_knobs.h).
#include "mof_knobs.h"

#include <algorithm>
#include <cstdlib>

namespace mof {

namespace {
const char *const kNames[(int)Knob::Count] = {
    "MOF_IO_THREADS", "MOF_RCCL_LIB", "MOF_VERBOSE",   "MOF_STAGE_MB",
    "MOF_SYM_READS",  "MOF_AMG_SMOOTH", "MOF_AMG_OMEGA", "MOF_AMG_BSW",
};

const char *env(const char *name) {
    const char *v = std::getenv(name);
    return v && *v ? v : nullptr;
}
}  // namespace

const char *knob(Knob k) { return env(kNames[(int)k]); }

int knob_int(Knob k, int dflt) {
    const char *v = knob(k);
    return v ? std::atoi(v) : dflt;
}

int32_t knob_threads(int32_t cap) {
    for (const char *v : {knob(Knob::IoThreads), env("OMP_NUM_THREADS")})
        if (v && std::atoi(v) > 0) return std::min<int32_t>(std::atoi(v), cap);
    return 0;
}

}  // namespace mof
