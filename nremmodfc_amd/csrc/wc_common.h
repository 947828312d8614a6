// wc_common.h -- shared helpers of the libwcsde translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../include/wcsde.h"

// one thread-local message buffer for the whole library (inline: a single
// instance across translation units), read back by wc_last_error()
inline char* wc_errbuf() {
    static thread_local char buf[512];
    return buf;
}
inline int wc_set_err(int code, const char* msg) {
    snprintf(wc_errbuf(), 512, "%s", msg);
    return code;
}
inline void wc_clear_err() { wc_errbuf()[0] = 0; }
inline int wc_hip_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(wc_errbuf(), 512, "%s: %s", what, hipGetErrorString(e));
        return WC_EHIP;
    }
    return WC_OK;
}
