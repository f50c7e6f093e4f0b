// alphazero/mcts/transposition_table.h -- TranspositionTable of the host API.  The table
// itself lives on the device, one direct-mapped 2^k-slot table per game (TranspositionTable
// semantics, transposition_table.cpp:44-191, 405-439); this object carries the size a
// ParallelMCTS should use and collects the device's lookup / hit counters.
#pragma once
#include <cstddef>
#include <cstdint>

namespace alphazero {
namespace mcts {

class TranspositionTable {
 public:
    explicit TranspositionTable(size_t size = 1048576, size_t numShards = 1024);
    size_t getSize() const { return size_; }
    int log2Size() const;
    float getHitRate() const { return lookups_ ? (float)hits_ / (float)lookups_ : 0.0f; }
    size_t getLookups() const { return lookups_; }
    size_t getHits() const { return hits_; }
    size_t getEntryCount() const { return entries_; }
    size_t getMemoryUsageBytes() const { return size_ * 24; }   // device bytes per slot
    void clear() { lookups_ = hits_ = entries_ = 0; }
    void resize(size_t size);
    // device counters of the owning search (ParallelMCTS calls this after every search)
    void record(uint64_t lookups, uint64_t hits, uint64_t entries) { lookups_ = lookups; hits_ = hits; entries_ = entries; }

 private:
    size_t size_;
    size_t shards_;
    uint64_t lookups_ = 0, hits_ = 0, entries_ = 0;
};

}  // namespace mcts
}  // namespace alphazero
