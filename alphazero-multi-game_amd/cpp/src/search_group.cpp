// search_group.cpp -- mcts::SearchGroup (alphazero/mcts/search_group.h).
#include "alphazero/mcts/search_group.h"

#include <algorithm>
#include <chrono>
#include <stdexcept>

#include "alphazero/games/go/go_state.h"
#include "alphazero/mcts/parallel_mcts.h"

namespace alphazero {
namespace mcts {

static void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + az_last_error());
}

SearchGroup::SearchGroup(nn::NeuralNetwork* nn, const MCTSConfig& config, const core::IGameState& prototype,
                         int capacity, const TranspositionTable* tt)
    : nn_(nn), capacity_(capacity), used_(capacity > 0 ? capacity : 0, 0) {
    if (capacity < 1) throw std::invalid_argument("SearchGroup: capacity >= 1");
    const bool go = prototype.getGameType() == core::GameType::GO;
    if (!go && prototype.getGameType() != core::GameType::GOMOKU) throw std::invalid_argument("SearchGroup: Gomoku or Go");
    if (go) {
        auto* g = dynamic_cast<const go::GoState*>(&prototype);
        if (!g || g->getKomi() != 7.5f || !g->isChineseRules() || !g->isEnforcingSuperko())
            throw std::invalid_argument("SearchGroup: the device Go rules are komi 7.5, Chinese rules, superko");
    }
    const DeviceEvaluator ev = deviceEvaluator(nn);
    if (ev.kind == AZ_EVAL_CALLBACK)
        throw std::invalid_argument("SearchGroup: host-callback evaluators are not grouped (HipNeuralNetwork, "
                                    "RandomPolicyNetwork or no network)");
    cfg_ = makeSearchConfig(config, prototype, nn, tt, capacity);
    check(az_search_create(ev.engine, ev.net, &cfg_, &s_), "az_search_create");
}

SearchGroup::~SearchGroup() {
    if (s_) az_search_destroy(s_);
}

int SearchGroup::members() const {
    std::lock_guard<std::mutex> lk(mu_);
    int n = 0;
    for (char u : used_) n += u != 0;
    return n;
}

size_t SearchGroup::searches() const {
    std::lock_guard<std::mutex> lk(mu_);
    return searches_;
}

size_t SearchGroup::deviceRuns() const {
    std::lock_guard<std::mutex> lk(mu_);
    return runs_;
}

void SearchGroup::setGatherMicros(int us) {
    std::lock_guard<std::mutex> lk(mu_);
    gatherUs_ = us > 0 ? us : 0;
}

// A fresh game in a free slot, seeded as a single-game handle's game (stream id 0: the same
// evaluator and noise streams as a standalone ParallelMCTS), then the root's history replayed
// (each move a fresh root, as a standalone object's rebuild does).
int SearchGroup::acquire(const core::IGameState& root) {
    int slot = -1;
    {
        std::lock_guard<std::mutex> lk(mu_);
        for (int i = 0; i < capacity_ && slot < 0; ++i)
            if (!used_[i]) slot = i;
        if (slot < 0) throw std::runtime_error("SearchGroup: every slot is taken");
        used_[slot] = 1;
    }
    try {
        const int id = 0;
        check(az_search_new_games_ids(s_, &slot, &id, 1), "az_search_new_games_ids");
        std::vector<int> acts(capacity_, AZ_ACTION_NONE), t(capacity_), r(capacity_);
        for (int a : root.getMoveHistory()) {
            acts[slot] = a;
            check(az_search_apply(s_, acts.data(), t.data(), r.data()), "az_search_apply");
        }
    } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        used_[slot] = 0;
        throw;
    }
    return slot;
}

void SearchGroup::release(int slot) {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot >= 0 && slot < capacity_) used_[slot] = 0;
}

// The search() of a member: its slot joins the pending set.  The first caller that finds no run
// in progress leads: (after the gather window) it takes every pending slot and runs ONE masked
// device search over them; callers whose slots were taken wait for that run, the others lead or
// join the next one.  Errors reach every member of the failed run.
void SearchGroup::search(int slot) {
    std::unique_lock<std::mutex> lk(mu_);
    pending_.insert(slot);
    searches_ += 1;
    cv_.notify_all();
    while (pending_.count(slot)) {
        if (running_) {
            cv_.wait(lk);
            continue;
        }
        running_ = true;
        if (gatherUs_ > 0) {
            // sliding window: every new request extends it by gatherUs_, up to 64 windows in all
            using clk = std::chrono::steady_clock;
            const auto win = std::chrono::microseconds(gatherUs_);
            const auto cap = clk::now() + 64 * win;
            auto until = clk::now() + win;
            size_t seen = pending_.size();
            int live = 0;
            for (char u : used_) live += u != 0;
            while ((int)pending_.size() < live) {
                const auto t = clk::now();
                if (t >= until || t >= cap) break;
                cv_.wait_until(lk, std::min(until, cap));
                if (pending_.size() != seen) {
                    seen = pending_.size();
                    until = clk::now() + win;
                }
            }
        }
        std::vector<uint8_t> mask(capacity_, 0);
        for (int g : pending_) mask[g] = 1;
        inflight_ = pending_;
        pending_.clear();
        runs_ += 1;
        lk.unlock();
        const int rc = az_search_run_masked(s_, mask.data());
        const std::string err = rc ? az_last_error() : "";
        lk.lock();
        for (int g : inflight_)
            if (rc) errors_[g] = err;
        inflight_.clear();
        running_ = false;
        cv_.notify_all();
    }
    cv_.wait(lk, [&] { return !inflight_.count(slot); });
    auto e = errors_.find(slot);
    if (e != errors_.end()) {
        const std::string m = e->second;
        errors_.erase(e);
        throw std::runtime_error("az_search_run_masked: " + m);
    }
}

}  // namespace mcts
}  // namespace alphazero
