// lt_error.h -- the library's thread-local error message (lt_last_error).
#pragma once
#include "../../include/lattice_decode.h"

namespace lt {
// Records the message for lt_last_error() and returns st.
lt_status set_error(lt_status st, const char* fmt, ...);
}  // namespace lt
