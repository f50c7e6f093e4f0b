// alphazero/selfplay/distributed.h -- one rank of a per-GPU self-play job on the engine's RCCL
// communicator (include/az_engine.h az_dist_*).  The reference shards self-play by process: its
// orchestrator starts one self_play binary per GPU, each with its own games and output
// (python/scripts/orchestrate_selfplay.py:303-311,741-749, flags src/selfplay/selfplay_main.cpp:
// 166-189).  Here the ranks also share rank 0's weights over xGMI (ncclBroadcast into the device
// weight buffers) and reduce the job's counters; games stay sharded with no data-path collective.
#pragma once
#include <array>
#include <string>
#include <vector>

#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/selfplay/self_play_manager.h"
#include "az_engine.h"

namespace alphazero {
namespace selfplay {

using DistId = std::array<unsigned char, AZ_DIST_ID_BYTES>;

// rank's GameShard (self_play_manager.h) of totalGames global game ids
GameShard shardGames(int rank, int world, int totalGames, unsigned noiseSeed = 42);

class Distributed {
 public:
    static DistId uniqueId();
    // rank 0 writes the id file (atomically: temp file + rename); the others wait for it
    static void writeIdFile(const std::string& path, const DistId& id);
    static DistId readIdFile(const std::string& path, int timeoutMs = 600000);

    // device < 0: the rank's engine is engineForDevice(-1) (LOCAL_RANK or 0); timeoutMs <= 0: 600 s
    Distributed(int rank, int world, const DistId& id, int device = -1, int timeoutMs = 0);
    ~Distributed();
    Distributed(const Distributed&) = delete;
    Distributed& operator=(const Distributed&) = delete;

    int rank() const { return rank_; }
    int world() const { return world_; }
    az_dist* handle() const { return d_; }

    void barrier();
    std::vector<double> allreduceSum(const std::vector<double>& v);
    std::vector<double> allreduceMax(const std::vector<double>& v);
    // rank root's weights into `net` on every rank (device to device), host copy refreshed
    void broadcastWeights(nn::HipNeuralNetwork& net, int root = 0);

 private:
    az_dist* d_ = nullptr;
    int rank_ = 0, world_ = 1;
};

}  // namespace selfplay
}  // namespace alphazero
