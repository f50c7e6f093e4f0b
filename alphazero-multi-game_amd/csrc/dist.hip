// dist.hip -- the multi-GPU collectives of the self-play path, native over
// RCCL: one process per GPU, games sharded by contiguous global id ranges with no data-path
// collective, and RCCL only to (1) broadcast rank 0's weights into every rank's device weight
// buffers and (2) reduce the throughput counters / the max elapsed time of a timed region.
//
// The reference scales self-play by process (python/scripts/orchestrate_selfplay.py:303-311,
// 741-749 spawns one self_play binary per GPU, each loading the model file itself); here the
// weights travel GPU to GPU over xGMI (ncclBroadcast straight into the packed device buffers of the
// net -- every piece set, fp32 / bf16 / fp16 hi+lo -- plus the canonical fp32 blob), no host hop.
//
// Every collective runs on the engine's stream (so a barrier also drains the engine's queued
// work) and is awaited with a deadline: a rank that died leaves the others in the collective, and
// they fail with AZ_ERR_STATE after the communicator's timeout (ncclCommAbort) instead of hanging.
#include <rccl/rccl.h>

#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>

#include "engine_internal.h"

struct az_dist {
    az_engine* e = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    int timeout_ms = 600000;
    bool broken = false;              // aborted after a timeout / async error: every later call fails
    double* dbuf = nullptr;           // counters staging [AZ_DIST_MAX_COUNTERS]
    float* blob = nullptr;            // canonical weight blob staging
    size_t blob_cap = 0;
    std::mutex mu;
};

namespace {

constexpr int AZ_DIST_MAX_COUNTERS = 64;

int nccl_fail(ncclResult_t r, const char* what) {
    return az_fail(AZ_ERR_HIP, "%s: %s", what, ncclGetErrorString(r));
}
#define NCCLCHK(x)                                        \
    do {                                                  \
        ncclResult_t r_ = (x);                            \
        if (r_ != ncclSuccess) return nccl_fail(r_, #x);  \
    } while (0)

// The collectives queued on the engine stream, done -- or the communicator aborted at the deadline
// (or on an asynchronous RCCL error) and AZ_ERR_STATE returned.
int wait_done(az_dist* d, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(d->e->stream);
        if (q == hipSuccess) return 0;
        if (q != hipErrorNotReady) return az_fail(AZ_ERR_HIP, "%s: %s", what, hipGetErrorString(q));
        ncclResult_t ar = ncclSuccess;
        if (ncclCommGetAsyncError(d->comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress) {
            ncclCommAbort(d->comm);
            d->comm = nullptr;
            d->broken = true;
            return az_fail(AZ_ERR_STATE, "%s: RCCL error %s (communicator aborted)", what, ncclGetErrorString(ar));
        }
        const long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > d->timeout_ms) {
            ncclCommAbort(d->comm);
            d->comm = nullptr;
            d->broken = true;
            return az_fail(AZ_ERR_STATE, "%s: collective not complete after %d ms (a rank died or never joined); "
                                         "communicator aborted", what, d->timeout_ms);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

int usable(az_dist* d) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dist");
    if (d->broken || !d->comm) return az_fail(AZ_ERR_STATE, "the communicator was aborted by an earlier failure");
    return 0;
}

// in[count] (host) -> out[count] (host), reduced over the ranks with op
int allreduce_host(az_dist* d, const double* in, double* out, int count, ncclRedOp_t op, const char* what) {
    hipStream_t st = d->e->stream;
    HIPCHK(hipMemcpyAsync(d->dbuf, in, (size_t)count * 8, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclAllReduce(d->dbuf, d->dbuf, count, ncclFloat64, op, d->comm, st));
    HIPCHK(hipMemcpyAsync(out, d->dbuf, (size_t)count * 8, hipMemcpyDeviceToHost, st));
    return wait_done(d, what);
}

}  // namespace

extern "C" {

int az_dist_unique_id(unsigned char* id) {
    if (!id) return az_fail(AZ_ERR_ARG, "null id");
    static_assert(sizeof(ncclUniqueId) == AZ_DIST_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, AZ_DIST_ID_BYTES);
    return 0;
}

int az_dist_init(az_engine* e, int rank, int world, const unsigned char* id, int timeout_ms, az_dist** out) {
    if (!e || !id || !out || world < 1 || rank < 0 || rank >= world) return az_fail(AZ_ERR_ARG, "bad argument");
    *out = nullptr;
    HIPCHK(hipSetDevice(e->device));
    auto* d = new az_dist();
    d->e = e;
    d->rank = rank;
    d->world = world;
    if (timeout_ms > 0) d->timeout_ms = timeout_ms;
    if (int r = dalloc(&d->dbuf, AZ_DIST_MAX_COUNTERS)) { delete d; return r; }
    ncclUniqueId u;
    std::memcpy(&u, id, AZ_DIST_ID_BYTES);
    // ncclCommInitRank blocks until every rank joined: it runs on a helper thread, awaited with the
    // communicator's deadline (a rank that never starts fails the others instead of hanging them;
    // on a timeout the helper is left behind, blocked in RCCL, and the process is expected to exit)
    struct Init {
        ncclComm_t comm = nullptr;
        ncclResult_t r = ncclInternalError;
        std::atomic<bool> done{false};
    };
    auto job = std::make_shared<Init>();
    const int dev = e->device;
    std::thread([job, world, u, rank, dev] {
        pthread_setname_np(pthread_self(), "az-rccl-init");
        if (hipSetDevice(dev) == hipSuccess) job->r = ncclCommInitRank(&job->comm, world, u, rank);
        job->done = true;
    }).detach();
    const auto t0 = std::chrono::steady_clock::now();
    while (!job->done) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(d->timeout_ms)) {
            (void)hipFree(d->dbuf);
            delete d;
            return az_fail(AZ_ERR_STATE, "ncclCommInitRank: not every rank joined within %d ms", timeout_ms > 0 ? timeout_ms : 600000);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (job->r != ncclSuccess) {
        (void)hipFree(d->dbuf);
        delete d;
        return nccl_fail(job->r, "ncclCommInitRank");
    }
    d->comm = job->comm;
    *out = d;
    return 0;
}

void az_dist_destroy(az_dist* d) {
    if (!d) return;
    (void)hipSetDevice(d->e->device);
    if (d->comm) {
        if (hipStreamSynchronize(d->e->stream) == hipSuccess) ncclCommDestroy(d->comm);
        else ncclCommAbort(d->comm);
    }
    if (d->dbuf) (void)hipFree(d->dbuf);
    if (d->blob) (void)hipFree(d->blob);
    delete d;
}

int az_dist_info(az_dist* d, int* rank, int* world) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dist");
    if (rank) *rank = d->rank;
    if (world) *world = d->world;
    return 0;
}

int az_dist_barrier(az_dist* d) {
    if (int r = usable(d)) return r;
    std::lock_guard<std::mutex> lk(d->mu);
    HIPCHK(hipSetDevice(d->e->device));
    const double one = 1.0;
    double n = 0.0;
    if (int r = allreduce_host(d, &one, &n, 1, ncclSum, "az_dist_barrier")) return r;
    if ((int)n != d->world) return az_fail(AZ_ERR_STATE, "az_dist_barrier: %d ranks answered, %d expected", (int)n, d->world);
    return 0;
}

int az_counters_allreduce(az_dist* d, const double* in, double* out, int count, int op) {
    if (int r = usable(d)) return r;
    if (!in || !out || count < 1 || count > AZ_DIST_MAX_COUNTERS || (op != AZ_DIST_SUM && op != AZ_DIST_MAX))
        return az_fail(AZ_ERR_ARG, "az_counters_allreduce: 1..%d counters, AZ_DIST_SUM or AZ_DIST_MAX", AZ_DIST_MAX_COUNTERS);
    std::lock_guard<std::mutex> lk(d->mu);
    HIPCHK(hipSetDevice(d->e->device));
    return allreduce_host(d, in, out, count, op == AZ_DIST_SUM ? ncclSum : ncclMax, "az_counters_allreduce");
}

int az_net_broadcast_weights(az_dist* d, az_net* n, int root) {
    if (int r = usable(d)) return r;
    if (!n || root < 0 || root >= d->world) return az_fail(AZ_ERR_ARG, "bad argument");
    if (net_engine(n)->device != d->e->device) return az_fail(AZ_ERR_ARG, "net and communicator on different devices");
    std::lock_guard<std::mutex> lk(d->mu);
    std::lock_guard<std::mutex> ln(net_mutex(n));
    HIPCHK(hipSetDevice(d->e->device));
    hipStream_t st = d->e->stream;
    const size_t np = net_param_count(n);
    if (d->rank == root && net_host_blob(n).size() != np) return az_fail(AZ_ERR_STATE, "root net has no weights loaded");
    std::vector<std::pair<void*, size_t>> bufs;
    if (int r = net_weight_buffers(n, bufs)) return r;
    // every rank must hold the same layout: (buffer count, total bytes, parameters) min == max
    double shape[3] = {(double)bufs.size(), 0.0, (double)np};
    for (auto& b : bufs) shape[1] += (double)b.second;
    double lo[3], hi[3];
    const double neg[3] = {-shape[0], -shape[1], -shape[2]};
    if (int r = allreduce_host(d, shape, hi, 3, ncclMax, "az_net_broadcast_weights")) return r;
    if (int r = allreduce_host(d, neg, lo, 3, ncclMax, "az_net_broadcast_weights")) return r;
    for (int i = 0; i < 3; ++i)
        if (hi[i] != -lo[i])
            return az_fail(AZ_ERR_ARG, "az_net_broadcast_weights: the ranks' nets differ (buffers / bytes / parameters)");
    if (d->blob_cap < np) {
        if (d->blob) (void)hipFree(d->blob);
        d->blob = nullptr;
        d->blob_cap = 0;
        if (int r = dalloc(&d->blob, np)) return r;
        d->blob_cap = np;
    }
    if (d->rank == root) HIPCHK(hipMemcpyAsync(d->blob, net_host_blob(n).data(), np * 4, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclBroadcast(d->blob, d->blob, np, ncclFloat32, root, d->comm, st));
    // the packed buffers (~550 for a 20-block net) in groups of 64 broadcasts: one fused launch
    // per group, well inside RCCL's per-group work limits
    constexpr size_t GROUP = 64;
    for (size_t g0 = 0; g0 < bufs.size(); g0 += GROUP) {
        NCCLCHK(ncclGroupStart());
        ncclResult_t gr = ncclSuccess;
        for (size_t i = g0; gr == ncclSuccess && i < std::min(bufs.size(), g0 + GROUP); ++i)
            gr = ncclBroadcast(bufs[i].first, bufs[i].first, bufs[i].second, ncclUint8, root, d->comm, st);
        const ncclResult_t ge = ncclGroupEnd();
        if (gr != ncclSuccess) return nccl_fail(gr, "ncclBroadcast");
        if (ge != ncclSuccess) return nccl_fail(ge, "ncclGroupEnd");
    }
    std::vector<float> host;
    if (d->rank != root) {
        host.resize(np);
        HIPCHK(hipMemcpyAsync(host.data(), d->blob, np * 4, hipMemcpyDeviceToHost, st));
    }
    if (int r = wait_done(d, "az_net_broadcast_weights")) return r;
    if (d->rank != root) net_adopt_blob(n, host.data());
    return 0;
}

// Diagnostic (tests/test_gpu_dist.py): what a broadcast does to a non-root rank's net, on one device --
// src's weight buffers copied into dst's (dst allocated by a zero load if never loaded) and the
// canonical blob adopted.  A dst net that then computes exactly what src computes, in every
// precision, shows the recorded buffer list covers every weight a forward reads.
int az_diag_net_copy_weights(az_net* dst, az_net* src) {
    if (!dst || !src || net_engine(dst)->device != net_engine(src)->device) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> la(net_mutex(dst));
    std::lock_guard<std::mutex> lb(net_mutex(src));
    HIPCHK(hipSetDevice(net_engine(src)->device));
    if (net_host_blob(src).size() != net_param_count(src)) return az_fail(AZ_ERR_STATE, "src has no weights loaded");
    std::vector<std::pair<void*, size_t>> a, b;
    if (int r = net_weight_buffers(dst, a)) return r;
    if (int r = net_weight_buffers(src, b)) return r;
    if (a.size() != b.size() || net_param_count(dst) != net_param_count(src))
        return az_fail(AZ_ERR_ARG, "the nets differ");
    for (size_t i = 0; i < a.size(); ++i) {
        if (a[i].second != b[i].second) return az_fail(AZ_ERR_ARG, "the nets differ (buffer %zu)", i);
        HIPCHK(hipMemcpy(a[i].first, b[i].first, a[i].second, hipMemcpyDeviceToDevice));
    }
    const std::vector<float> blob = net_host_blob(src);
    net_adopt_blob(dst, blob.data());
    return 0;
}

}  // extern "C"
