// alphazero/nn/batch_queue.h -- the reference's inference request queue
// (include/alphazero/nn/batch_queue.h:28-266, src/nn/batch_queue.cpp:61-363) on the host API.
//
// Callers enqueue single game states and get a std::future of (policy, value); worker threads
// coalesce queued requests into batches for NeuralNetwork::predictBatch.  Same configuration,
// statistics and error behaviour as the reference:
//   * no network, a full queue (maxQueueSize; counted in droppedRequests) or a failing clone:
//     the future holds the uniform policy and value 0 at once;
//   * a predictBatch that throws answers every request of the batch with the uniform policy;
//   * setBatchSize(<= 0) throws std::invalid_argument;
//   * adaptive batching (useAdaptiveBatching): every adaptiveBatchInterval ms the batch target
//     moves toward an estimate from the queue pressure (up by at most 2, down by 1, clamped to
//     [minBatchSize, maxAdaptiveBatchSize]).
// Differences, both fixes of reference defects that change no result:
//   * a request owns its state's clone until its batch has been evaluated (the reference pops the
//     request -- destroying the clone -- while the batch still holds a reference to it);
//   * requests of equal priority are served first-in first-out (std::priority_queue gives no order).
// The device self-play path (SelfPlayManager / az_selfplay_run) needs no queue: every game of a
// handle advances one simulation per step and all their leaves form one batch on the device.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "alphazero/core/igamestate.h"
#include "alphazero/nn/neural_network.h"

namespace alphazero {
namespace nn {

struct BatchQueueConfig {
    int batchSize = 16;                // target batch size
    int timeoutMs = 10;                // how long a partial batch may wait for more requests
    int maxQueueSize = 1024;           // requests beyond this are answered uniformly (dropped)
    int numWorkerThreads = 1;
    bool prioritizeBatchSize = true;   // kept for the API; unused, as in the reference (batch_queue.cpp never reads it)
    int minBatchSize = 1;
    bool useAdaptiveBatching = true;
    int adaptiveBatchInterval = 100;   // ms
    int maxAdaptiveBatchSize = 64;
};

struct BatchQueueStats {
    std::atomic<size_t> totalRequests{0};
    std::atomic<size_t> totalBatches{0};
    std::atomic<size_t> totalTimedOutBatches{0};
    std::atomic<size_t> avgBatchSize{0};          // sum of batch sizes (toString divides by totalBatches)
    std::atomic<size_t> maxQueueSize{0};
    std::atomic<size_t> avgQueueWaitTimeMs{0};    // sum over requests (divided by totalRequests)
    std::atomic<size_t> avgProcessingTimeMs{0};   // sum over batches (divided by totalBatches)
    std::atomic<size_t> droppedRequests{0};

    void reset();
    std::string toString() const;
};

class BatchQueue {
 public:
    using Result = std::pair<std::vector<float>, float>;

    BatchQueue(NeuralNetwork* neuralNetwork, const BatchQueueConfig& config = BatchQueueConfig());
    BatchQueue(NeuralNetwork* neuralNetwork, int batchSize, int timeoutMs = 10);
    ~BatchQueue();
    BatchQueue(const BatchQueue&) = delete;
    BatchQueue& operator=(const BatchQueue&) = delete;

    std::future<Result> enqueue(const core::IGameState& state, int priority = 0);

    const BatchQueueConfig& getConfig() const { return config_; }
    void setConfig(const BatchQueueConfig& config);
    void setBatchSize(int batchSize);
    void setTimeout(int timeoutMs);
    int getBatchSize() const;
    int getTimeout() const;
    int getPendingRequests() const;
    const BatchQueueStats& getStats() const { return stats_; }
    void resetStats() { stats_.reset(); }
    NeuralNetwork* getNeuralNetwork() const { return neuralNetwork_.load(); }
    // takes effect from the next batch a worker evaluates (workers read the pointer once per batch)
    void setNeuralNetwork(NeuralNetwork* neuralNetwork) { neuralNetwork_.store(neuralNetwork); }
    // batch target of the adaptive batching (== getBatchSize() without it)
    int getCurrentBatchSize() const;

 private:
    struct Request {
        std::unique_ptr<core::IGameState> state;
        std::promise<Result> promise;
        std::chrono::steady_clock::time_point enqueued;
    };
    using Clock = std::chrono::steady_clock;

    void startWorkers(int n);
    void stopWorkers(std::unique_lock<std::mutex>& lk);
    void worker();
    std::vector<Request> takeBatch(std::unique_lock<std::mutex>& lk, bool& timedOut);
    void evaluate(std::vector<Request>& batch);
    void adapt();
    static Result uniform(const core::IGameState& s);

    std::atomic<NeuralNetwork*> neuralNetwork_;
    BatchQueueConfig config_;
    std::map<int, std::deque<Request>, std::greater<int>> queue_;   // by priority, highest first; FIFO inside
    size_t size_ = 0;
    mutable std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    int current_;                                  // adaptive batch target
    Clock::time_point lastAdapt_;
    std::vector<std::thread> workers_;
    BatchQueueStats stats_;
};

}  // namespace nn
}  // namespace alphazero
