// batch_queue.cpp -- alphazero::nn::BatchQueue (see the header; reference behaviour from
// src/nn/batch_queue.cpp:61-363).
#include "alphazero/nn/batch_queue.h"

#include <algorithm>
#include <stdexcept>

namespace alphazero {
namespace nn {

void BatchQueueStats::reset() {
    totalRequests = 0;
    totalBatches = 0;
    totalTimedOutBatches = 0;
    avgBatchSize = 0;
    maxQueueSize = 0;
    avgQueueWaitTimeMs = 0;
    avgProcessingTimeMs = 0;
    droppedRequests = 0;
}

// the reference's report (batch_queue.h:61-77): averages are sums divided by their counts
std::string BatchQueueStats::toString() const {
    const size_t b = totalBatches, r = totalRequests;
    std::stringstream ss;
    ss << "Batch Queue Stats:\n"
       << "  Total requests: " << r << "\n"
       << "  Total batches: " << b << "\n"
       << "  Timed out batches: " << totalTimedOutBatches << "\n"
       << "  Avg batch size: " << (b ? avgBatchSize.load() / b : 0) << "\n"
       << "  Max queue size: " << maxQueueSize << "\n"
       << "  Avg queue wait time: " << (r ? avgQueueWaitTimeMs.load() / r : 0) << " ms\n"
       << "  Avg processing time: " << (b ? avgProcessingTimeMs.load() / b : 0) << " ms\n"
       << "  Dropped requests: " << droppedRequests << "\n";
    return ss.str();
}

BatchQueue::BatchQueue(NeuralNetwork* neuralNetwork, const BatchQueueConfig& config)
    : neuralNetwork_(neuralNetwork), config_(config), current_(config.batchSize), lastAdapt_(Clock::now()) {
    startWorkers(config_.numWorkerThreads);
}

BatchQueue::BatchQueue(NeuralNetwork* neuralNetwork, int batchSize, int timeoutMs)
    : neuralNetwork_(neuralNetwork), current_(batchSize), lastAdapt_(Clock::now()) {
    config_.batchSize = batchSize;
    config_.timeoutMs = timeoutMs;
    startWorkers(1);
}

BatchQueue::~BatchQueue() {
    std::unique_lock<std::mutex> lk(mu_);
    stopWorkers(lk);
    // requests still queued are dropped with their promises (their futures report broken_promise),
    // as the reference's destructor clears its queue
    queue_.clear();
    size_ = 0;
}

void BatchQueue::startWorkers(int n) {
    stop_ = false;
    for (int i = 0; i < std::max(1, n); ++i) workers_.emplace_back(&BatchQueue::worker, this);
}

void BatchQueue::stopWorkers(std::unique_lock<std::mutex>& lk) {
    stop_ = true;
    cv_.notify_all();
    std::vector<std::thread> w;
    w.swap(workers_);
    lk.unlock();
    for (auto& t : w)
        if (t.joinable()) t.join();
    lk.lock();
}

BatchQueue::Result BatchQueue::uniform(const core::IGameState& s) {
    const int A = s.getActionSpaceSize();
    return {std::vector<float>(A, 1.0f / (float)A), 0.0f};
}

std::future<BatchQueue::Result> BatchQueue::enqueue(const core::IGameState& state, int priority) {
    auto answered = [&](Result r) {
        std::promise<Result> p;
        p.set_value(std::move(r));
        return p.get_future();
    };
    if (!neuralNetwork_) return answered(uniform(state));
    Request rq;
    try {
        rq.state = state.clone();
    } catch (const std::exception&) {
        return answered(uniform(state));
    }
    rq.enqueued = Clock::now();
    std::future<Result> f = rq.promise.get_future();
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (size_ >= (size_t)config_.maxQueueSize) {
            stats_.droppedRequests.fetch_add(1, std::memory_order_relaxed);
            return answered(uniform(state));
        }
        if (size_ > stats_.maxQueueSize.load(std::memory_order_relaxed))
            stats_.maxQueueSize.store(size_, std::memory_order_relaxed);
        queue_[priority].push_back(std::move(rq));
        ++size_;
        stats_.totalRequests.fetch_add(1, std::memory_order_relaxed);
    }
    cv_.notify_one();
    return f;
}

void BatchQueue::setConfig(const BatchQueueConfig& config) {
    std::unique_lock<std::mutex> lk(mu_);
    const bool restart = (int)workers_.size() != std::max(1, config.numWorkerThreads);
    config_ = config;
    current_ = config.batchSize;
    if (restart) {
        stopWorkers(lk);
        startWorkers(config_.numWorkerThreads);
    }
}

void BatchQueue::setBatchSize(int batchSize) {
    if (batchSize <= 0) throw std::invalid_argument("Batch size must be positive");
    std::lock_guard<std::mutex> lk(mu_);
    config_.batchSize = batchSize;
    current_ = batchSize;
}

// the configuration is read by the workers under the queue lock, so the setters / getters take it too
void BatchQueue::setTimeout(int timeoutMs) {
    std::lock_guard<std::mutex> lk(mu_);
    config_.timeoutMs = timeoutMs;
}

int BatchQueue::getBatchSize() const {
    std::lock_guard<std::mutex> lk(mu_);
    return config_.batchSize;
}

int BatchQueue::getTimeout() const {
    std::lock_guard<std::mutex> lk(mu_);
    return config_.timeoutMs;
}

int BatchQueue::getPendingRequests() const {
    std::lock_guard<std::mutex> lk(mu_);
    return (int)size_;
}

int BatchQueue::getCurrentBatchSize() const {
    std::lock_guard<std::mutex> lk(mu_);
    return current_;
}

// batch_queue.cpp:327-363: move the target toward an estimate from the queue pressure
void BatchQueue::adapt() {
    const int q = (int)size_;
    int opt;
    if (q <= config_.minBatchSize) opt = config_.minBatchSize;
    else if (q > 2 * current_) opt = std::min(q / 2, config_.maxAdaptiveBatchSize);
    else if (NeuralNetwork* nn = neuralNetwork_.load(); nn && nn->isGpuAvailable()) opt = std::min(config_.batchSize * 2, config_.maxAdaptiveBatchSize);
    else opt = config_.batchSize;
    if (opt > current_) current_ = std::min(opt, current_ + 2);
    else if (opt < current_) current_ = std::max(opt, current_ - 1);
    current_ = std::max(config_.minBatchSize, std::min(current_, config_.maxAdaptiveBatchSize));
}

// batch_queue.cpp:219-265: up to the batch target from the highest priority down.  The batch
// runs as soon as the queue is drained and it holds at least minBatchSize requests (the reference
// never reads prioritizeBatchSize); below minBatchSize it waits timeoutMs / 4 for more and then
// runs with what it has.  Past timeoutMs of collecting, a batch of at least minBatchSize stops
// taking requests.  Either early stop counts as a timed-out batch.
std::vector<BatchQueue::Request> BatchQueue::takeBatch(std::unique_lock<std::mutex>& lk, bool& timedOut) {
    std::vector<Request> batch;
    const auto start = Clock::now();
    const auto limit = std::chrono::milliseconds(config_.timeoutMs);
    const size_t target = (size_t)std::max(1, current_);
    const size_t minB = (size_t)std::max(0, config_.minBatchSize);
    while (batch.size() < target && size_ > 0) {
        if (Clock::now() - start >= limit && batch.size() >= minB) {
            timedOut = true;
            break;
        }
        auto it = queue_.begin();
        batch.push_back(std::move(it->second.front()));
        it->second.pop_front();
        if (it->second.empty()) queue_.erase(it);
        --size_;
        if (size_ == 0 && batch.size() < minB) {
            const bool more = cv_.wait_for(lk, std::chrono::milliseconds(std::max(1, config_.timeoutMs / 4)),
                                           [&] { return size_ > 0 || stop_; });
            if (stop_) break;
            if (!more && !batch.empty()) {
                timedOut = true;
                break;
            }
        }
    }
    return batch;
}

void BatchQueue::worker() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
        if (config_.useAdaptiveBatching) {
            const auto now = Clock::now();
            if (now - lastAdapt_ >= std::chrono::milliseconds(config_.adaptiveBatchInterval)) {
                adapt();
                lastAdapt_ = now;
            }
        }
        if (size_ == 0) {
            cv_.wait_for(lk, std::chrono::milliseconds(std::max(1, config_.timeoutMs)), [&] { return size_ > 0 || stop_; });
            continue;
        }
        bool timedOut = false;
        std::vector<Request> batch = takeBatch(lk, timedOut);
        if (batch.empty()) continue;
        lk.unlock();
        if (timedOut) stats_.totalTimedOutBatches.fetch_add(1, std::memory_order_relaxed);
        evaluate(batch);
        lk.lock();
    }
}

// One predictBatch over the batch's own state clones (alive until every promise is set).  The
// statistics are recorded before the promises are fulfilled, so a caller that has its answer sees
// its batch counted.
void BatchQueue::evaluate(std::vector<Request>& batch) {
    const auto t0 = Clock::now();
    size_t waited = 0;
    for (const Request& r : batch)
        waited += (size_t)std::chrono::duration_cast<std::chrono::milliseconds>(t0 - r.enqueued).count();
    std::vector<std::reference_wrapper<const core::IGameState>> states;
    states.reserve(batch.size());
    for (const Request& r : batch) states.push_back(std::cref(*r.state));
    std::vector<std::vector<float>> policies;
    std::vector<float> values;
    NeuralNetwork* nn = neuralNetwork_.load();
    bool ok = true;
    try {
        if (!nn) throw std::runtime_error("BatchQueue: no network");
        nn->predictBatch(states, policies, values);
    } catch (const std::exception&) {
        ok = false;
    }
    const size_t ms = (size_t)std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count();
    stats_.totalBatches.fetch_add(1, std::memory_order_relaxed);
    stats_.avgBatchSize.fetch_add(batch.size(), std::memory_order_relaxed);
    stats_.avgProcessingTimeMs.fetch_add(ms, std::memory_order_relaxed);
    stats_.avgQueueWaitTimeMs.fetch_add(waited, std::memory_order_relaxed);
    for (size_t i = 0; i < batch.size(); ++i) {
        Request& r = batch[i];
        if (!ok) r.promise.set_value(uniform(*r.state));                   // batch_queue.cpp:288-309
        else if (i < policies.size() && i < values.size()) r.promise.set_value({std::move(policies[i]), values[i]});
        else   // the network answered fewer states (batch_queue.cpp:282-286)
            r.promise.set_value({std::vector<float>(r.state->getActionSpaceSize(), 0.0f), 0.0f});
    }
}

}  // namespace nn
}  // namespace alphazero
