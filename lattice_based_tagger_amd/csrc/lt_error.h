// lt_error.h -- the library's thread-local error message (lt_last_error).
#pragma once
#include "../../include/lattice_decode.h"

namespace lt {
// Records the message for lt_last_error() and returns st.
lt_status set_error(lt_status st, const char* fmt, ...);
// Host worker threads: OMP_NUM_THREADS when set (the job's CPU share on a
// shared machine, where hardware_concurrency reports every core), else the
// hardware concurrency.
int host_threads();
}  // namespace lt
