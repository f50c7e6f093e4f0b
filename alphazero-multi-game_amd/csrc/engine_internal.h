// engine_internal.h -- pieces of the host runtime shared by the C-ABI translation units
// (engine.hip, dataset.hip): the engine handle, the thread-local error report and the
// allocation / HIP-status helpers.  Not part of the public boundary (include/az_engine.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <mutex>

#include "../../include/az_engine.h"

struct az_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipDeviceProp_t prop{};
    std::mutex mu;
};

// Sets the az_last_error() message; returns code.
int az_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIPCHK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return az_fail(AZ_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

template <class T>
inline int dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return az_fail(AZ_ERR_OOM, "hipMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
    return 0;
}
#define DALLOC(p, n) do { int r_ = dalloc(&(p), (n)); if (r_) return r_; } while (0)
