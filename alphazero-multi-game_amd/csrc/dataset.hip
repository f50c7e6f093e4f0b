// dataset.hip -- host side of the device-resident training-example store (include/az_engine.h
// az_dataset_*): alphazero::selfplay::Dataset (src/selfplay/dataset.cpp).
//
// Records are validated on the host (every index the kernel dereferences), uploaded once, and
// k_dataset_extract (tree_kernels.hip) replays every game on device and writes each position's
// examples -- the original and, with augmentation, the 7 symmetries -- straight into their
// shuffled slots.  getBatch / getRandomSubset / shuffle are device gathers (k_dataset_gather).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <numeric>
#include <random>
#include <vector>

#include "engine_internal.h"
#include "tree.h"

__global__ void k_dataset_extract(DatasetDev d, TreeDev t);
__global__ void k_dataset_gather(const float* states, const float* policy, const int* plen, const float* value, int row,
                                 int NA, const long long* idx, int n, float* ostates, float* opolicy, int* oplen,
                                 float* ovalue);

struct az_dataset {
    az_engine* e = nullptr;
    int game = 0, bs = 0, A = 0, NA = 0, C = 0;
    int64_t E = 0, cap = 0;
    float* states = nullptr; float* policy = nullptr; int* plen = nullptr; float* value = nullptr;
    uint64_t* zzero = nullptr;             // Go capture code updates a hash: zero keys (planes need none)
    std::vector<void*> scratch;            // per-call uploads
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0, last_bytes = 0.0;
    std::mt19937 rng{std::random_device{}()};   // Dataset::rng_ (dataset.cpp:57)
    std::mutex mu;
};

namespace {

// Example rows of one storage set.
struct Rows {
    float* states = nullptr; float* policy = nullptr; int* plen = nullptr; float* value = nullptr;
    int64_t cap = 0;
    void release() {
        for (void* p : {(void*)states, (void*)policy, (void*)plen, (void*)value}) if (p) (void)hipFree(p);
        *this = Rows{};
    }
};

int rows_alloc(Rows& r, int64_t n, int C, int A, int NA) {
    DALLOC(r.states, (size_t)n * C * A);
    DALLOC(r.policy, (size_t)n * NA);
    DALLOC(r.plen, (size_t)n);
    DALLOC(r.value, (size_t)n);
    r.cap = n;
    return 0;
}

Rows rows_of(az_dataset* d) { Rows r; r.states = d->states; r.policy = d->policy; r.plen = d->plen; r.value = d->value; r.cap = d->cap; return r; }
void set_rows(az_dataset* d, const Rows& r) { d->states = r.states; d->policy = r.policy; d->plen = r.plen; d->value = r.value; d->cap = r.cap; }

void free_scratch(az_dataset* d) {
    for (void* p : d->scratch) (void)hipFree(p);
    d->scratch.clear();
}

template <class T>
int upload(az_dataset* d, const T* host, size_t n, T** dev) {
    int r = dalloc(dev, n);
    if (r) return r;
    d->scratch.push_back(*dev);
    if (n && host) HIPCHK(hipMemcpyAsync(*dev, host, n * sizeof(T), hipMemcpyHostToDevice, d->e->stream));
    return 0;
}

// storage for n rows (grow-only; contents are not preserved)
int reserve(az_dataset* d, int64_t n) {
    if (n <= d->cap) return 0;
    Rows r = rows_of(d);
    r.release();
    set_rows(d, r);
    Rows nr;
    int rc = rows_alloc(nr, n, d->C, d->A, d->NA);
    if (rc) { nr.release(); return rc; }
    set_rows(d, nr);
    return 0;
}

int check_perm(const int64_t* order, int64_t n) {
    std::vector<uint8_t> seen((size_t)n, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (order[i] < 0 || order[i] >= n || seen[(size_t)order[i]])
            return az_fail(AZ_ERR_ARG, "order is not a permutation of 0..%lld", (long long)n - 1);
        seen[(size_t)order[i]] = 1;
    }
    return 0;
}

// rows idx[0..n) of d into `out` (device), on the engine stream
int gather_rows(az_dataset* d, const long long* idx_dev, int64_t n, Rows& out) {
    const int row = d->C * d->A;
    for (int64_t b = 0; b < n; b += 1 << 30) {
        const int cnt = (int)std::min<int64_t>(n - b, 1 << 30);
        hipLaunchKernelGGL(k_dataset_gather, dim3(cnt), dim3(256), 0, d->e->stream, d->states, d->policy, d->plen,
                           d->value, row, d->NA, idx_dev + b, cnt, out.states + b * row, out.policy + b * d->NA,
                           out.plen + b, out.value + b);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int az_dataset_create(az_engine* e, int game_type, int board_size, az_dataset** out) {
    if (!e || !out) return az_fail(AZ_ERR_ARG, "null argument");
    if (game_type != AZ_GAME_GOMOKU && game_type != AZ_GAME_GO)
        return az_fail(AZ_ERR_ARG, "dataset: game type %d has no device rules (Gomoku and Go only)", game_type);
    if (board_size < 2 || board_size * board_size > AZ_MAXA)
        return az_fail(AZ_ERR_ARG, "dataset: board size %d out of range", board_size);
    HIPCHK(hipSetDevice(e->device));
    auto* d = new az_dataset();
    d->e = e;
    d->game = game_type == AZ_GAME_GO ? GAME_GO : GAME_GOMOKU;
    d->bs = board_size;
    d->A = board_size * board_size;
    d->NA = d->game == GAME_GO ? d->A + 1 : d->A;
    d->C = d->game == GAME_GO ? 8 : 11;
    int r = dalloc(&d->zzero, (size_t)2 * d->A);
    hipError_t he = hipSuccess;
    if (!r) he = hipMemset(d->zzero, 0, (size_t)2 * d->A * 8);
    if (!r && he == hipSuccess) he = hipEventCreate(&d->ev0);
    if (!r && he == hipSuccess) he = hipEventCreate(&d->ev1);
    if (!r && he != hipSuccess) r = az_fail(AZ_ERR_HIP, "dataset init: %s", hipGetErrorString(he));
    if (r) { az_dataset_destroy(d); return r; }
    *out = d;
    return 0;
}

void az_dataset_destroy(az_dataset* d) {
    if (!d) return;
    (void)hipSetDevice(d->e->device);
    free_scratch(d);
    Rows r = rows_of(d);
    r.release();
    if (d->zzero) (void)hipFree(d->zzero);
    if (d->ev0) (void)hipEventDestroy(d->ev0);
    if (d->ev1) (void)hipEventDestroy(d->ev1);
    delete d;
}

int az_dataset_extract(az_dataset* d, int n_games, const int* n_moves, const int* actions, const int* n_children,
                       const float* policies, const int* results, int augment, const int64_t* order,
                       int64_t* n_examples) {
    if (!d || n_games < 0 || (n_games && (!n_moves || !results))) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(d->mu);
    std::vector<int> move_off((size_t)n_games + 1, 0);
    for (int g = 0; g < n_games; ++g) {
        if (n_moves[g] < 0) return az_fail(AZ_ERR_ARG, "game %d: negative move count", g);
        if (results[g] < 0 || results[g] > 3) return az_fail(AZ_ERR_ARG, "game %d: bad GameResult %d", g, results[g]);
        if ((int64_t)move_off[g] + n_moves[g] > (int64_t)INT32_MAX / 8) return az_fail(AZ_ERR_ARG, "too many moves");
        move_off[g + 1] = move_off[g] + n_moves[g];
    }
    const int M = move_off[n_games];
    if (M && (!actions || !n_children || !policies)) return az_fail(AZ_ERR_ARG, "null move arrays");
    std::vector<long long> pol_off((size_t)M + 1, 0);
    const int amin = d->game == GAME_GO ? -1 : 0;
    for (int g = 0; g < n_games; ++g) {
        std::vector<uint8_t> occ((size_t)d->A, 0);
        for (int m = move_off[g]; m < move_off[g + 1]; ++m) {
            const int a = actions[m];
            const int mv = m - move_off[g];
            if (a < amin || a >= d->A) return az_fail(AZ_ERR_ARG, "game %d move %d: action %d out of range", g, mv, a);
            if (d->game == GAME_GOMOKU) {   // Go cells are freed by captures; Gomoku cells never are
                if (occ[(size_t)a]) return az_fail(AZ_ERR_ARG, "game %d move %d: cell %d occupied", g, mv, a);
                occ[(size_t)a] = 1;
            }
            if (n_children[m] < 0 || n_children[m] > d->NA)
                return az_fail(AZ_ERR_ARG, "game %d move %d: policy length %d > %d", g, mv, n_children[m], d->NA);
            pol_off[(size_t)m + 1] = pol_off[(size_t)m] + n_children[m];
        }
    }
    const int K = augment ? 8 : 1;
    const int64_t E = (int64_t)M * K;
    std::vector<long long> dst;
    if (order) {
        int r = check_perm(order, E);
        if (r) return r;
        dst.resize((size_t)E);
        for (int64_t i = 0; i < E; ++i) dst[(size_t)order[i]] = i;
    }
    HIPCHK(hipSetDevice(d->e->device));
    int r = reserve(d, E);
    if (r) return r;
    d->E = E;
    if (n_examples) *n_examples = E;
    d->last_ms = 0.0;
    d->last_bytes = 0.0;
    if (M == 0) return 0;
    int* mo = nullptr; int* ac = nullptr; long long* po = nullptr; int* nc = nullptr; float* pp = nullptr;
    int* rs = nullptr; long long* ds = nullptr;
    r = upload(d, move_off.data(), move_off.size(), &mo);
    if (!r) r = upload(d, actions, (size_t)M, &ac);
    if (!r) r = upload(d, pol_off.data(), (size_t)M, &po);
    if (!r) r = upload(d, n_children, (size_t)M, &nc);
    if (!r) r = upload(d, policies, (size_t)pol_off[(size_t)M], &pp);
    if (!r) r = upload(d, results, (size_t)n_games, &rs);
    if (!r && order) r = upload(d, dst.data(), dst.size(), &ds);
    if (r) { (void)hipStreamSynchronize(d->e->stream); free_scratch(d); return r; }
    DatasetDev dv{};
    dv.game = d->game; dv.bs = d->bs; dv.A = d->A; dv.NA = d->NA; dv.C = d->C; dv.K = K; dv.n_games = n_games;
    dv.move_off = mo; dv.actions = ac; dv.pol_off = po; dv.n_children = nc; dv.policies = pp; dv.results = rs;
    dv.dst = ds;
    dv.states = d->states; dv.policy = d->policy; dv.plen = d->plen; dv.value = d->value;
    TreeDev t{};
    t.bs = d->bs; t.A = d->A; t.NA = d->NA; t.game = d->game; t.zpiece = d->zzero;
    hipError_t he = hipEventRecord(d->ev0, d->e->stream);
    if (he == hipSuccess) {
        hipLaunchKernelGGL(k_dataset_extract, dim3(n_games), dim3(AZ_DS_THREADS), 0, d->e->stream, dv, t);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipEventRecord(d->ev1, d->e->stream);
    hipError_t se = hipStreamSynchronize(d->e->stream);
    free_scratch(d);
    if (he == hipSuccess) he = se;
    if (he != hipSuccess) return az_fail(AZ_ERR_HIP, "k_dataset_extract: %s", hipGetErrorString(he));
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, d->ev0, d->ev1));
    d->last_ms = ms;
    // algorithmic bytes: every example written once (states, padded policy, length, value), the
    // records read once (action, offsets and policy floats per move), the slot table
    d->last_bytes = (double)E * (4.0 * d->C * d->A + 4.0 * d->NA + 8.0) + (double)M * 16.0 +
                    4.0 * (double)pol_off[(size_t)M] + (order ? 8.0 * (double)E : 0.0);
    return 0;
}

int az_dataset_info(az_dataset* d, int64_t* n_examples, int* planes, int* board_size, int* policy_stride) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dataset");
    if (n_examples) *n_examples = d->E;
    if (planes) *planes = d->C;
    if (board_size) *board_size = d->bs;
    if (policy_stride) *policy_stride = d->NA;
    return 0;
}

int az_dataset_seed(az_dataset* d, uint32_t seed) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dataset");
    std::lock_guard<std::mutex> lk(d->mu);
    d->rng.seed(seed);
    return 0;
}

int az_dataset_shuffle_order(az_dataset* d, int64_t n, int64_t* order) {
    if (!d || n < 0 || (n && !order)) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(d->mu);
    std::vector<long long> idx((size_t)n);   // element type does not change std::shuffle's swaps
    std::iota(idx.begin(), idx.end(), 0LL);
    std::shuffle(idx.begin(), idx.end(), d->rng);
    std::copy(idx.begin(), idx.end(), order);
    return 0;
}

int az_dataset_upload(az_dataset* d, int64_t n, const float* states, const float* policy, const int* policy_len,
                      const float* value) {
    if (!d || n < 0 || (n && (!states || !policy || !policy_len || !value))) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(d->mu);
    for (int64_t i = 0; i < n; ++i)
        if (policy_len[i] < 0 || policy_len[i] > d->NA)
            return az_fail(AZ_ERR_ARG, "example %lld: policy length %d > %d", (long long)i, policy_len[i], d->NA);
    HIPCHK(hipSetDevice(d->e->device));
    int r = reserve(d, n);
    if (r) return r;
    d->E = n;
    if (n == 0) return 0;
    const size_t row = (size_t)d->C * d->A;
    HIPCHK(hipMemcpy(d->states, states, (size_t)n * row * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->policy, policy, (size_t)n * d->NA * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->plen, policy_len, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->value, value, (size_t)n * 4, hipMemcpyHostToDevice));
    return 0;
}

int az_dataset_permute(az_dataset* d, const int64_t* order) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dataset");
    std::lock_guard<std::mutex> lk(d->mu);
    if (d->E == 0) return 0;
    if (!order) return az_fail(AZ_ERR_ARG, "null order");
    int r = check_perm(order, d->E);
    if (r) return r;
    HIPCHK(hipSetDevice(d->e->device));
    Rows nr;
    long long* idx = nullptr;
    r = rows_alloc(nr, d->E, d->C, d->A, d->NA);
    if (!r) r = upload(d, (const long long*)order, (size_t)d->E, &idx);
    if (!r) r = gather_rows(d, idx, d->E, nr);
    hipError_t se = hipStreamSynchronize(d->e->stream);
    free_scratch(d);
    if (!r && se != hipSuccess) r = az_fail(AZ_ERR_HIP, "dataset permute: %s", hipGetErrorString(se));
    if (r) { nr.release(); return r; }
    Rows old = rows_of(d);
    old.release();
    set_rows(d, nr);
    return 0;
}

int az_dataset_gather(az_dataset* d, const int64_t* idx, int n, float* states, float* policy, int* policy_len,
                      float* value) {
    if (!d || n < 0 || (n && (!idx || !states || !policy || !policy_len || !value))) return az_fail(AZ_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(d->mu);
    for (int i = 0; i < n; ++i)
        if (idx[i] < 0 || idx[i] >= d->E)
            return az_fail(AZ_ERR_ARG, "index %lld out of range (%lld examples)", (long long)idx[i], (long long)d->E);
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(d->e->device));
    Rows t;
    long long* di = nullptr;
    int r = rows_alloc(t, n, d->C, d->A, d->NA);
    if (!r) r = upload(d, (const long long*)idx, (size_t)n, &di);
    if (!r) r = gather_rows(d, di, n, t);
    hipError_t he = hipSuccess;
    if (!r) {
        const size_t row = (size_t)d->C * d->A;
        he = hipMemcpyAsync(states, t.states, (size_t)n * row * 4, hipMemcpyDeviceToHost, d->e->stream);
        if (he == hipSuccess) he = hipMemcpyAsync(policy, t.policy, (size_t)n * d->NA * 4, hipMemcpyDeviceToHost, d->e->stream);
        if (he == hipSuccess) he = hipMemcpyAsync(policy_len, t.plen, (size_t)n * 4, hipMemcpyDeviceToHost, d->e->stream);
        if (he == hipSuccess) he = hipMemcpyAsync(value, t.value, (size_t)n * 4, hipMemcpyDeviceToHost, d->e->stream);
    }
    hipError_t se = hipStreamSynchronize(d->e->stream);
    if (he == hipSuccess) he = se;
    if (!r && he != hipSuccess) r = az_fail(AZ_ERR_HIP, "dataset gather: %s", hipGetErrorString(he));
    free_scratch(d);
    t.release();
    return r;
}

int az_dataset_profile_read(az_dataset* d, double* extract_ms, double* bytes) {
    if (!d) return az_fail(AZ_ERR_ARG, "null dataset");
    if (extract_ms) *extract_ms = d->last_ms;
    if (bytes) *bytes = d->last_bytes;
    return 0;
}

}  // extern "C"
