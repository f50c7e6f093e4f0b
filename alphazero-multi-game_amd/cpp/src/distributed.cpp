// Distributed: the engine's RCCL communicator for the C++ host API (see distributed.h).
#include "alphazero/selfplay/distributed.h"

#include <chrono>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <thread>

namespace alphazero {
namespace selfplay {

namespace {
void check(int rc, const char* what) {
    if (rc != AZ_OK) throw std::runtime_error(std::string(what) + ": " + az_last_error());
}
}  // namespace

GameShard shardGames(int rank, int world, int totalGames, unsigned noiseSeed) {
    if (world < 1 || rank < 0 || rank >= world || totalGames < 0) throw std::invalid_argument("shardGames: bad rank / world");
    const int base = totalGames / world, extra = totalGames % world;
    GameShard s;
    s.firstGame = rank * base + std::min(rank, extra);
    s.numGames = base + (rank < extra ? 1 : 0);
    s.noiseSeed = noiseSeed + (unsigned)s.firstGame;
    return s;
}

DistId Distributed::uniqueId() {
    DistId id{};
    check(az_dist_unique_id(id.data()), "az_dist_unique_id");
    return id;
}

void Distributed::writeIdFile(const std::string& path, const DistId& id) {
    const std::string tmp = path + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
        if (!f) throw std::runtime_error("cannot write " + tmp);
        f.write(reinterpret_cast<const char*>(id.data()), (std::streamsize)id.size());
        if (!f) throw std::runtime_error("cannot write " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp + " to " + path);
}

DistId Distributed::readIdFile(const std::string& path, int timeoutMs) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        std::ifstream f(path, std::ios::binary);
        if (f) {
            DistId id{};
            f.read(reinterpret_cast<char*>(id.data()), (std::streamsize)id.size());
            if (f.gcount() == (std::streamsize)id.size()) return id;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs))
            throw std::runtime_error("no communicator id in " + path + " (rank 0 writes it)");
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

Distributed::Distributed(int rank, int world, const DistId& id, int device, int timeoutMs) : rank_(rank), world_(world) {
    check(az_dist_init(nn::engineForDevice(device), rank, world, id.data(), timeoutMs, &d_), "az_dist_init");
}

Distributed::~Distributed() {
    if (d_) az_dist_destroy(d_);
}

void Distributed::barrier() { check(az_dist_barrier(d_), "az_dist_barrier"); }

std::vector<double> Distributed::allreduceSum(const std::vector<double>& v) {
    std::vector<double> out(v.size());
    check(az_counters_allreduce(d_, v.data(), out.data(), (int)v.size(), AZ_DIST_SUM), "az_counters_allreduce");
    return out;
}

std::vector<double> Distributed::allreduceMax(const std::vector<double>& v) {
    std::vector<double> out(v.size());
    check(az_counters_allreduce(d_, v.data(), out.data(), (int)v.size(), AZ_DIST_MAX), "az_counters_allreduce");
    return out;
}

void Distributed::broadcastWeights(nn::HipNeuralNetwork& net, int root) {
    check(az_net_broadcast_weights(d_, net.handle(), root), "az_net_broadcast_weights");
    net.refreshHostWeights();
}

}  // namespace selfplay
}  // namespace alphazero
