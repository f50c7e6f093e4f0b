// alphazero/mcts/search_group.h -- several ParallelMCTS objects on ONE device search handle.
//
// The reference's usage is one ParallelMCTS object per game (examples/test_mcts_nn.cpp;
// SelfPlayManager's worker threads each own one, self_play_manager.cpp:69-89).  On the device a
// single-game handle runs every simulation step at batch 1.  A SearchGroup owns one az_search
// handle with `capacity` game slots; each member object (ParallelMCTS(root, group)) plays in its
// own slot, and the search() calls of members that arrive together -- typically from several
// threads, one per game, as the reference's thread pool calls them -- run as ONE masked device
// search over all their slots (one leaf batch per simulation step).  Every other member call
// (selectAction, updateWithMove, noise, releaseMemory, root statistics) touches only the member's
// slot.  Results are bit-identical to a standalone object's: each slot is its own game with its
// own tree, table and rng_, seeded as a single-game handle's game (stream id 0).
//
// Members share the group's evaluator and search parameters; a member whose setter changes them
// (setNeuralNetwork, setNumSimulations, setConfig with other device parameters, ...) leaves the
// group: it gets a handle of its own and its history is replayed, as a standalone object
// rebuilds.  Host-callback evaluators (a NeuralNetwork subclass other than HipNeuralNetwork /
// RandomPolicyNetwork) are not grouped.  The group must outlive its members.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "alphazero/core/igamestate.h"
#include "alphazero/mcts/transposition_table.h"
#include "alphazero/nn/neural_network.h"
#include "az_engine.h"

namespace alphazero {
namespace mcts {

struct MCTSConfig;
class ParallelMCTS;

// The device configuration of a search for `config` on games like `state` (board, game type),
// evaluated by nn, with a table of tt's size (or config.transpositionTableSize), nGames slots.
az_search_cfg makeSearchConfig(const MCTSConfig& config, const core::IGameState& state, nn::NeuralNetwork* nn,
                               const TranspositionTable* tt, int nGames);

class SearchGroup {
 public:
    SearchGroup(nn::NeuralNetwork* nn, const MCTSConfig& config, const core::IGameState& prototype, int capacity,
                const TranspositionTable* tt = nullptr);
    ~SearchGroup();
    SearchGroup(const SearchGroup&) = delete;
    SearchGroup& operator=(const SearchGroup&) = delete;

    int capacity() const { return capacity_; }
    int members() const;
    size_t searches() const;       // member search() calls served
    size_t deviceRuns() const;     // masked device searches that served them
    // A search() that finds no run in progress gathers the other live members' requests before it
    // starts: until every live member has one in, or no new one has arrived for this long (a sliding
    // window, at most 64 windows in all).  Default 2000 us: one thread per member issues its next
    // search a few host calls (selectAction, updateWithMove, noise: each a short device call on the
    // shared handle) after the last run; a single-threaded caller pays one window per search.
    // 0: requests that arrive during a run are batched into the next one only.
    void setGatherMicros(int us);

 private:
    friend class ParallelMCTS;
    int acquire(const core::IGameState& root);   // a fresh game in a free slot, the root's history replayed
    void release(int slot);
    void search(int slot);                       // blocks until a device search covering `slot` has finished
    az_search* handle() const { return s_; }
    const az_search_cfg& deviceConfig() const { return cfg_; }
    nn::NeuralNetwork* network() const { return nn_; }

    nn::NeuralNetwork* nn_;
    az_search_cfg cfg_{};
    int capacity_;
    az_search* s_ = nullptr;
    mutable std::mutex mu_;
    std::condition_variable cv_;
    std::vector<char> used_;
    std::set<int> pending_, inflight_;
    std::map<int, std::string> errors_;
    bool running_ = false;
    int gatherUs_ = 2000;
    size_t searches_ = 0, runs_ = 0;
};

}  // namespace mcts
}  // namespace alphazero
