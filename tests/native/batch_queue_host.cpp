// CPU test of alphazero::nn::BatchQueue (cpp/include/alphazero/nn/batch_queue.h) on the
// MockNeuralNetwork pattern of the reference's tests/nn/batch_queue_test.cpp:11-52: a host-only
// network whose outputs are a function of the state's hash, so every answer can be checked
// against a direct predictBatch.  Prints "OK" and exits 0 when every check holds.
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/nn/batch_queue.h"
#ifdef AZ_BQ_GPU
#include "alphazero/nn/hip_neural_network.h"
#endif

using namespace alphazero;

#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                   \
        }                                                                   \
    } while (0)

class MockNeuralNetwork : public nn::NeuralNetwork {
 public:
    std::mutex mu;
    std::condition_variable cv;
    bool gate_open = true;            // predictBatch blocks while closed
    bool fail = false;                // predictBatch throws
    std::vector<int> batch_sizes;
    std::vector<uint64_t> order;      // hashes in evaluation order
    std::atomic<int> inside{0};

    static std::pair<std::vector<float>, float> out(const core::IGameState& s) {
        const uint64_t h = s.getHash();
        std::vector<float> p(s.getActionSpaceSize());
        for (size_t i = 0; i < p.size(); ++i) p[i] = (float)((h >> (i % 48)) & 1023) / 1024.0f;
        return {p, (float)(h % 1000) / 1000.0f - 0.5f};
    }
    std::pair<std::vector<float>, float> predict(const core::IGameState& s) override { return out(s); }
    void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                      std::vector<std::vector<float>>& policies, std::vector<float>& values) override {
        inside++;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return gate_open; });
            batch_sizes.push_back((int)states.size());
            for (auto& s : states) order.push_back(s.get().getHash());
        }
        if (fail) throw std::runtime_error("mock failure");
        policies.clear();
        values.clear();
        for (auto& s : states) {
            auto o = out(s.get());
            policies.push_back(o.first);
            values.push_back(o.second);
        }
    }
    std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& s) override {
        std::promise<std::pair<std::vector<float>, float>> p;
        p.set_value(out(s));
        return p.get_future();
    }
    bool isGpuAvailable() const override { return false; }
    std::string getDeviceInfo() const override { return "Mock"; }
    float getInferenceTimeMs() const override { return 0.1f; }
    int getBatchSize() const override { return 8; }
    std::string getModelInfo() const override { return "Mock"; }
    size_t getModelSizeBytes() const override { return 0; }
    void benchmark(int, int) override {}
    void enableDebugMode(bool) override {}
    void printModelSummary() const override {}
    void close_gate() { std::lock_guard<std::mutex> lk(mu); gate_open = false; }
    void open_gate() {
        { std::lock_guard<std::mutex> lk(mu); gate_open = true; }
        cv.notify_all();
    }
};

static std::unique_ptr<gomoku::GomokuState> position(int k) {
    auto s = std::make_unique<gomoku::GomokuState>(9, false);
    for (int i = 0; i < k % 20; ++i) s->makeMove((k * 7 + i * 13) % 81 == 40 ? 41 : ((k * 7 + i * 13) % 81));
    return s;
}

static bool same(const std::pair<std::vector<float>, float>& a, const std::pair<std::vector<float>, float>& b) {
    return a.first == b.first && a.second == b.second;
}

#ifdef AZ_BQ_GPU
// The queue in front of the device net: every answer bitwise equal to the net's own predictBatch
// of that state alone (a board's output does not depend on its batch, test_gpu_net.py).
static int gpu_main() {
    nn::NetShape sh;
    sh.boardSize = 9; sh.actionSize = 81; sh.channels = 32; sh.blocks = 2; sh.maxBatch = 16;
    sh.precision = AZ_PREC_F32;
    nn::HipNeuralNetwork net(sh);
    net.initRandom(3);
    nn::BatchQueueConfig cfg;
    cfg.batchSize = 8;
    cfg.timeoutMs = 20;
    cfg.numWorkerThreads = 2;
    nn::BatchQueue q(&net, cfg);
    std::vector<std::future<nn::BatchQueue::Result>> fut(48);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            for (int k = t; k < 48; k += 4) fut[k] = q.enqueue(*position(k));
        });
    for (auto& x : th) x.join();
    for (int k = 0; k < 48; ++k) {
        auto s = position(k);
        std::vector<std::reference_wrapper<const core::IGameState>> one{std::cref(*s)};
        std::vector<std::vector<float>> pol;
        std::vector<float> val;
        net.predictBatch(one, pol, val);
        CHECK(same(fut[k].get(), {pol[0], val[0]}));
    }
    CHECK(q.getStats().totalRequests == 48 && q.getStats().droppedRequests == 0);
    std::printf("OK gpu batches=%zu\n", (size_t)q.getStats().totalBatches);
    return 0;
}
#endif

int main(int argc, char** argv) {
#ifdef AZ_BQ_GPU
    if (argc > 1 && std::string(argv[1]) == "gpu") return gpu_main();
#endif
    (void)argc; (void)argv;
    // reference tests/nn/batch_queue_test.cpp: SetBatchSize, SetTimeout
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.batchSize = 4;
        cfg.timeoutMs = 20;
        cfg.numWorkerThreads = 1;
        nn::BatchQueue q(&net, cfg);
        q.setBatchSize(8);
        CHECK(q.getBatchSize() == 8);
        bool threw = false;
        try { q.setBatchSize(0); } catch (const std::invalid_argument&) { threw = true; }
        CHECK(threw && q.getBatchSize() == 8);
        q.setTimeout(50);
        CHECK(q.getTimeout() == 50);
    }
    // answers equal a direct evaluation; requests from 4 threads; the caller's state may die at once
    // (the queue evaluates its own clone); batches never exceed the target
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.batchSize = 4;
        cfg.timeoutMs = 50;
        cfg.useAdaptiveBatching = false;
        nn::BatchQueue q(&net, cfg);
        std::vector<std::future<nn::BatchQueue::Result>> fut(64);
        std::vector<std::thread> th;
        for (int t = 0; t < 4; ++t)
            th.emplace_back([&, t] {
                for (int k = t; k < 64; k += 4) {
                    auto s = position(k);
                    fut[k] = q.enqueue(*s);
                }   // s destroyed here, before its batch runs
            });
        for (auto& x : th) x.join();
        for (int k = 0; k < 64; ++k) CHECK(same(fut[k].get(), MockNeuralNetwork::out(*position(k))));
        int total = 0;
        for (int b : net.batch_sizes) { CHECK(b >= 1 && b <= 4); total += b; }
        CHECK(total == 64);
        CHECK(q.getStats().totalRequests == 64 && q.getStats().totalBatches == net.batch_sizes.size());
        CHECK(q.getStats().avgBatchSize == 64 && q.getPendingRequests() == 0);
        CHECK(q.getStats().toString().find("Total requests: 64") != std::string::npos);
    }
    // priorities: with the worker held inside a batch, later requests queue; the highest priority
    // is served first, FIFO within a priority
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.batchSize = 1;
        cfg.timeoutMs = 5;
        cfg.useAdaptiveBatching = false;
        nn::BatchQueue q(&net, cfg);
        net.close_gate();
        auto f0 = q.enqueue(*position(1));
        while (net.inside.load() < 1) std::this_thread::yield();   // worker blocked on request 1
        auto lo1 = q.enqueue(*position(2), 0);
        auto lo2 = q.enqueue(*position(3), 0);
        auto hi = q.enqueue(*position(4), 5);
        CHECK(q.getPendingRequests() == 3);
        net.open_gate();
        f0.get(); lo1.get(); lo2.get(); hi.get();
        CHECK(net.order.size() == 4);
        CHECK(net.order[1] == position(4)->getHash() && net.order[2] == position(2)->getHash() &&
              net.order[3] == position(3)->getHash());
    }
    // a full queue answers uniformly at once and counts the drop; no network -> uniform
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.batchSize = 1;
        cfg.maxQueueSize = 2;
        cfg.useAdaptiveBatching = false;
        nn::BatchQueue q(&net, cfg);
        net.close_gate();
        auto f0 = q.enqueue(*position(5));
        while (net.inside.load() < 1) std::this_thread::yield();
        auto f1 = q.enqueue(*position(6));
        auto f2 = q.enqueue(*position(7));
        auto f3 = q.enqueue(*position(8));       // queue holds 2: dropped
        CHECK(f3.wait_for(std::chrono::seconds(0)) == std::future_status::ready);
        auto r3 = f3.get();
        CHECK(r3.first.size() == 81 && r3.first[0] == 1.0f / 81 && r3.second == 0.0f);
        CHECK(q.getStats().droppedRequests == 1);
        net.open_gate();
        CHECK(same(f1.get(), MockNeuralNetwork::out(*position(6))) && same(f2.get(), MockNeuralNetwork::out(*position(7))));
        f0.get();
        nn::BatchQueue none(nullptr, 4, 10);
        auto u = none.enqueue(*position(9)).get();
        CHECK(u.first.size() == 81 && u.first[80] == 1.0f / 81 && u.second == 0.0f);
    }
    // a failing network answers its batch uniformly
    {
        MockNeuralNetwork net;
        net.fail = true;
        nn::BatchQueue q(&net, 4, 10);
        auto r = q.enqueue(*position(10)).get();
        CHECK(r.first.size() == 81 && r.first[3] == 1.0f / 81 && r.second == 0.0f);
    }
    // adaptive batching moves the target toward the queue pressure, within its bounds
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.batchSize = 4;
        cfg.timeoutMs = 2;
        cfg.adaptiveBatchInterval = 0;              // adapt before every batch (timing-independent)
        cfg.maxAdaptiveBatchSize = 12;
        nn::BatchQueue q(&net, cfg);
        net.close_gate();
        std::vector<std::future<nn::BatchQueue::Result>> fut;
        fut.push_back(q.enqueue(*position(11)));
        while (net.inside.load() < 1) std::this_thread::yield();
        for (int k = 0; k < 60; ++k) fut.push_back(q.enqueue(*position(12 + k)));
        net.open_gate();
        for (auto& f : fut) f.get();
        int mx = 0;
        for (int b : net.batch_sizes) mx = std::max(mx, b);
        CHECK(mx > 4 && mx <= 12 && q.getCurrentBatchSize() <= 12 && q.getCurrentBatchSize() >= 1);
    }
    // setConfig with another worker count restarts the workers; requests keep flowing
    {
        MockNeuralNetwork net;
        nn::BatchQueue q(&net, 2, 5);
        nn::BatchQueueConfig cfg;
        cfg.numWorkerThreads = 3;
        cfg.batchSize = 3;
        q.setConfig(cfg);
        CHECK(q.getConfig().numWorkerThreads == 3 && q.getBatchSize() == 3);
        std::vector<std::future<nn::BatchQueue::Result>> fut;
        for (int k = 0; k < 30; ++k) fut.push_back(q.enqueue(*position(k)));
        for (int k = 0; k < 30; ++k) CHECK(same(fut[k].get(), MockNeuralNetwork::out(*position(k))));
    }
    // latency (batch_queue.cpp:219-265): a lone caller's request runs as soon as the queue is
    // drained -- it never waits timeoutMs for the batch to fill; below minBatchSize a batch waits
    // timeoutMs / 4 for company and then runs anyway (a timed-out batch)
    {
        MockNeuralNetwork net;
        nn::BatchQueueConfig cfg;
        cfg.timeoutMs = 200;
        nn::BatchQueue q(&net, cfg);
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 20; ++k) CHECK(same(q.enqueue(*position(k)).get(), MockNeuralNetwork::out(*position(k))));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        CHECK(ms < 20 * 100.0);                       // a fill-wait would cost 20 x 200 ms (generous bound: loaded CI hosts)
        CHECK(q.getStats().totalTimedOutBatches == 0);
        cfg.minBatchSize = 3;
        nn::BatchQueue q3(&net, cfg);
        const auto t1 = std::chrono::steady_clock::now();
        CHECK(same(q3.enqueue(*position(3)).get(), MockNeuralNetwork::out(*position(3))));
        const double ms3 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        CHECK(ms3 >= 40.0 && ms3 < 1000.0);           // waits timeoutMs / 4 = 50 ms (the lower bound is the behaviour;
                                                      // the upper one only excludes a 5 x timeoutMs hang)
        CHECK(q3.getStats().totalTimedOutBatches == 1);
    }
    // the network may be swapped while workers run (the next batch uses the new one)
    {
        MockNeuralNetwork a, b;
        nn::BatchQueue q(&a, 2, 2);
        std::atomic<bool> done{false};
        std::thread sw([&] {
            for (int k = 0; !done.load(); ++k) {
                q.setNeuralNetwork(k % 2 ? &a : &b);
                std::this_thread::yield();
            }
        });
        for (int k = 0; k < 40; ++k) CHECK(same(q.enqueue(*position(k)).get(), MockNeuralNetwork::out(*position(k))));
        done = true;
        sw.join();
        CHECK(q.getNeuralNetwork() == &a || q.getNeuralNetwork() == &b);
    }
    // destruction with requests still queued returns (their futures report a broken promise)
    {
        MockNeuralNetwork net;
        std::future<nn::BatchQueue::Result> late;
        std::thread opener;
        {
            nn::BatchQueue q(&net, 1, 5);
            net.close_gate();
            auto f0 = q.enqueue(*position(1));
            while (net.inside.load() < 1) std::this_thread::yield();
            late = q.enqueue(*position(2));
            opener = std::thread([&] { std::this_thread::sleep_for(std::chrono::milliseconds(50)); net.open_gate(); });
        }
        opener.join();
        bool broken = false;
        try { late.get(); } catch (const std::future_error&) { broken = true; }
        CHECK(broken);
    }
    std::printf("OK\n");
    return 0;
}
