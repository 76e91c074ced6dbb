// Thread-local error message behind nr_last_error() (C ABI).
#include "common.h"

static thread_local char g_err[512] = "";

void nr_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

NR_API const char* nr_last_error(void) { return g_err; }
