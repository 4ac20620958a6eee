// mof_knobs.h -- the library's environment switches, read in one place
// (mof_knobs.cpp; INTEGRATION.md §5 lists them with their defaults). Every
// other behaviour is decided per mesh by the library itself; the A/B switches
// of rounds 1-5 whose alternative lost are gone with their alternatives.
#pragma once

#include <cstdint>

namespace mof {

enum class Knob : int {
    IoThreads,  // MOF_IO_THREADS: host threads of the CSV files and the staging copies
    RcclLib,    // MOF_RCCL_LIB: path of librccl (mof_dd_create_rank)
    Verbose,    // MOF_VERBOSE: solve, multigrid and host-staging diagnostics on stderr
    StageMB,    // MOF_STAGE_MB: largest pinned ring chunk of host-pointer solves (MiB)
    SymReads,   // MOF_SYM_READS=0/1: plain / symmetric operator reads (changes V bits)
    AmgSmooth,  // MOF_AMG_SMOOTH=0/1: tentative / smoothed level-0 prolongator (V bits)
    AmgOmega,   // MOF_AMG_OMEGA=w0[,w1]: fine [, coarse] smoother damping (V bits)
    AmgBsw,     // MOF_AMG_BSW=k: boundary-row sweeps per side on open surfaces (V bits)
    Count
};

// the switch's value, nullptr when unset or empty
const char *knob(Knob k);
// integer value, dflt when unset
int knob_int(Knob k, int dflt);
// MOF_IO_THREADS, else OMP_NUM_THREADS (the process's CPU share on shared
// hosts) when > 0, capped at cap; else 0
int32_t knob_threads(int32_t cap);

}  // namespace mof
