// engine_internal.h -- pieces of the host runtime shared by the C-ABI translation units
// (engine.hip, dataset.hip): the engine handle, the thread-local error report and the
// allocation / HIP-status helpers.  Not part of the public boundary (include/az_engine.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <mutex>
#include <utility>
#include <vector>

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

// While set (a net's first weight load, WeightRegistry), every dalloc is recorded here: the list of
// device buffers that hold a net's weights, in allocation order (az_net_broadcast_weights).
inline thread_local std::vector<std::pair<void*, size_t>>* g_dalloc_reg = nullptr;
struct WeightRegistry {
    explicit WeightRegistry(std::vector<std::pair<void*, size_t>>* r) { g_dalloc_reg = r; }
    ~WeightRegistry() { g_dalloc_reg = nullptr; }
};

template <class T>
inline int dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return az_fail(AZ_ERR_OOM, "hipMalloc(%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
    if (g_dalloc_reg) g_dalloc_reg->emplace_back((void*)*p, n * sizeof(T));
    return 0;
}

// Net internals for the multi-GPU collectives (dist.hip, az_net_broadcast_weights):
// the device buffers of the net's loaded weights (every packed piece set), allocating them with a
// load of zero weights if the net was never loaded; the canonical blob on the host.
struct az_net;
int net_weight_buffers(az_net* n, std::vector<std::pair<void*, size_t>>& out);
const std::vector<float>& net_host_blob(az_net* n);
size_t net_param_count(az_net* n);
az_engine* net_engine(az_net* n);
std::mutex& net_mutex(az_net* n);
// after a broadcast filled the device buffers: the host copy of the canonical blob, loaded = true
void net_adopt_blob(az_net* n, const float* blob);
#define DALLOC(p, n) do { int r_ = dalloc(&(p), (n)); if (r_) return r_; } while (0)
