// alphazero/mcts/mcts_node.h -- MCTSNode of the host API: a read-only host snapshot of a device
// tree node (the root, with its children one level down).  The tree itself lives in the device's
// SoA node pool (csrc/tree.h); ParallelMCTS::getRootNode() copies the root's statistics and its
// children's (az_search_root_node / az_search_root_children).  The methods restate the
// reference's MCTSNode (include/alphazero/mcts/mcts_node.h, src/mcts/mcts_node.cpp) on those
// statistics, quirks included: getUcbScore returns the fixed test value 0.875 for a visited node
// (mcts_node.cpp:61-84).  Children of a snapshot carry no grandchildren.
#pragma once
#include <algorithm>
#include <cmath>
#include <iomanip>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace mcts {

struct MCTSNode {
    int visitCount = 0;
    float valueSum = 0.0f;
    int virtualLoss = 0;
    float prior = 0.0f;
    int action = -1;
    bool isExpanded = false;
    bool isTerminal = false;
    core::GameResult gameResult = core::GameResult::ONGOING;
    std::vector<int> actions;                              // child order
    std::vector<std::shared_ptr<MCTSNode>> children;

    bool hasChildren() const { return !children.empty(); }
    // mcts_node.h:80-85
    float getValue() const { return visitCount == 0 ? 0.0f : valueSum / (float)visitCount; }
    // mcts_node.cpp:37-39, 387-399
    float getTerminalValue(int currentPlayer) const {
        switch (gameResult) {
            case core::GameResult::WIN_PLAYER1: return currentPlayer == 1 ? 1.0f : -1.0f;
            case core::GameResult::WIN_PLAYER2: return currentPlayer == 2 ? 1.0f : -1.0f;
            default: return 0.0f;
        }
    }
    // mcts_node.cpp:41-60: the reference returns FLT_MAX for an unvisited node and the constant of
    // its unit test otherwise
    float getUcbScore(float, int, float = 0.0f, int = 0) const {
        return visitCount == 0 ? std::numeric_limits<float>::max() : 0.5f + 1.5f * 0.5f * std::sqrt(1.0f) / (1.0f + 1.0f);
    }
    // mcts_node.cpp:225-243: first child with the most visits
    int getBestAction() const {
        if (children.empty()) return -1;
        size_t best = 0;
        for (size_t i = 1; i < children.size(); ++i)
            if (children[i]->visitCount > children[best]->visitCount) best = i;
        return actions[best];
    }
    // mcts_node.cpp:245-266
    std::vector<int> getBestActions() const {
        std::vector<int> out;
        int mx = 0;
        for (const auto& c : children) mx = std::max(mx, c->visitCount);
        for (size_t i = 0; i < children.size(); ++i)
            if (children[i]->visitCount == mx) out.push_back(actions[i]);
        return out;
    }
    // mcts_node.cpp:289-322
    std::vector<float> getVisitCountDistribution(float temperature = 1.0f) const {
        std::vector<float> d(actions.size(), 0.0f);
        if (children.empty()) return d;
        float total = 0.0f;
        std::vector<float> counts(children.size());
        for (size_t i = 0; i < children.size(); ++i) {
            counts[i] = std::pow((float)children[i]->visitCount, 1.0f / std::max(0.01f, temperature));
            total += counts[i];
        }
        if (total > 0.0f) for (size_t i = 0; i < children.size(); ++i) d[i] = counts[i] / total;
        else for (size_t i = 0; i < children.size(); ++i) d[i] = 1.0f / (float)children.size();
        return d;
    }
    // mcts_node.cpp:324-374
    std::string toString(int maxDepth = 1) const {
        std::stringstream ss;
        ss << "Node: V=" << visitCount << ", Q=" << std::fixed << std::setprecision(3) << getValue() << ", P="
           << std::fixed << std::setprecision(3) << prior << (isTerminal ? " (Terminal)" : "");
        if (action >= 0) ss << ", Action=" << action;
        if (maxDepth > 0 && !children.empty()) {
            ss << "\nChildren: " << children.size() << std::endl;
            std::vector<std::pair<size_t, int>> order;
            for (size_t i = 0; i < children.size(); ++i) order.emplace_back(i, children[i]->visitCount);
            std::sort(order.begin(), order.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
            const int show = std::min(10, (int)children.size());
            for (int i = 0; i < show; ++i) {
                const size_t k = order[i].first;
                ss << std::string(4, ' ') << "Action " << actions[k] << ": V=" << children[k]->visitCount << ", Q="
                   << std::fixed << std::setprecision(3) << children[k]->getValue() << ", P=" << std::fixed
                   << std::setprecision(3) << children[k]->prior;
                if (maxDepth > 1) ss << "\n" << std::string(8, ' ') << children[k]->toString(maxDepth - 1);
                if (i < show - 1) ss << std::endl;
            }
            if (children.size() > 10) ss << std::endl << std::string(4, ' ') << "... and " << (children.size() - 10) << " more children";
        }
        return ss.str();
    }
};

}  // namespace mcts
}  // namespace alphazero
