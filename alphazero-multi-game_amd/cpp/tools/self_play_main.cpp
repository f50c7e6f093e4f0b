// self_play -- the reference's self-play entry point (src/selfplay/selfplay_main.cpp:156-392: the
// binary its orchestrator starts once per GPU, python/scripts/orchestrate_selfplay.py:394-400) on
// the MI355X engine: the same flags and defaults, the same record files (<dir>/<id>_<ts>.json) and
// run metadata file (<dir>/metadata_<ticks>.json), with every game of the run on the device.
//
// Engine extensions:
//   --rank R --world W --dist-id-file PATH   one rank of a per-GPU job: rank 0 writes the RCCL
//                      communicator id to PATH, the others read it; rank 0 loads (or initialises)
//                      the net and broadcasts its shape and weights over xGMI; the --num-games
//                      global game ids are sharded contiguously; the job's counters are reduced
//   --device D         the HIP device (default: LOCAL_RANK, else 0)
//   --net-blocks B --net-channels F --seed S   without --model: a random-init residual net of that
//                      shape (the BASELINE architecture, e.g. 20 x 256) instead of RandomPolicyNetwork
//   --precision P      trunk precision of a device net: fp16 | f16x3 | bf16x3 | f32 (--fp16 = fp16;
//                      default: the fp32-faithful f16x3 where its kernels exist)
//   --concurrent-games N   device game slots, at most --batch-size (the reference's batch: one leaf
//                      per game slot per simulation step)
//   --max-moves N      cut games at N moves
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <map>
#include <memory>
#include <string>
#include <thread>

#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/nn/random_policy_network.h"
#include "alphazero/selfplay/distributed.h"
#include "alphazero/selfplay/run_metadata.h"
#include "alphazero/selfplay/self_play_manager.h"

using namespace alphazero;

namespace {

struct Args {
    std::map<std::string, std::string> kv;
    bool has(const std::string& k) const { return kv.count(k) != 0; }
    std::string get(const std::string& k, const std::string& d) const { return has(k) ? kv.at(k) : d; }
    int getInt(const std::string& k, int d) const { return has(k) ? std::stoi(kv.at(k)) : d; }
    float getFloat(const std::string& k, float d) const { return has(k) ? std::stof(kv.at(k)) : d; }
};

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        if (k.rfind("--", 0) != 0) continue;
        if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) a.kv[k] = argv[++i];
        else a.kv[k] = "";
    }
    return a;
}

void usage() {
    std::cout << "Usage: self_play [options]\n"
                 "  --model PATH            model file (.pt TorchScript of the reference's ResNet, or .azw)\n"
                 "  --game TYPE             gomoku | go (default gomoku)\n"
                 "  --size N                board size (default 15 gomoku, 19 go)\n"
                 "  --num-games N           games to generate (default 100; over all ranks)\n"
                 "  --simulations N         MCTS simulations per move (default 800)\n"
                 "  --threads N             recorded only: concurrency is the device slot count\n"
                 "  --output-dir DIR        game records + metadata (default data/games)\n"
                 "  --temperature T         initial temperature (default 1.0)\n"
                 "  --temp-drop N           move where the temperature drops (default 30)\n"
                 "  --final-temp T          final temperature (default 0.0)\n"
                 "  --dirichlet-alpha A     (default 0.03)\n"
                 "  --dirichlet-epsilon E   (default 0.25)\n"
                 "  --batch-size N          network batch = device game slots per step (default 8)\n"
                 "  --batch-timeout MS      recorded (default 10)\n"
                 "  --fp16                  fp16 trunk (the reference's useFp16)\n"
                 "  --c-puct C              (default 1.5)\n"
                 "  --fpu-reduction F       (default 0.1)\n"
                 "  --virtual-loss N        (default 3)\n"
                 "  --no-tt                 recorded (the device search keeps its per-game table)\n"
                 "  --rank R --world W --dist-id-file PATH   one rank of a per-GPU job (RCCL)\n"
                 "  --device D              HIP device (default LOCAL_RANK, else 0)\n"
                 "  --net-blocks B --net-channels F --seed S   random-init residual net without --model\n"
                 "  --precision P           fp16 | f16x3 | bf16x3 | f32\n"
                 "  --concurrent-games N    device game slots, at most --batch-size\n"
                 "  --max-moves N           cut games at N moves\n";
}

core::GameType gameTypeOf(const std::string& s) {
    if (s == "gomoku") return core::GameType::GOMOKU;
    if (s == "go") return core::GameType::GO;
    if (s == "chess") throw std::invalid_argument("chess: the reference's Chess rules recurse without bound (DESIGN.md); "
                                                  "self-play runs gomoku and go");
    throw std::invalid_argument("unknown game " + s);
}

int precisionOf(const std::string& s) {
    if (s == "fp16") return AZ_PREC_FP16;
    if (s == "f16x3") return AZ_PREC_F16X3;
    if (s == "bf16x3") return AZ_PREC_BF16X3;
    if (s == "f32") return AZ_PREC_F32;
    throw std::invalid_argument("unknown precision " + s);
}

const char* precisionName(int p) {
    switch (p) {
        case AZ_PREC_FP16: return "fp16";
        case AZ_PREC_F16X3: return "f16x3";
        case AZ_PREC_BF16X3: return "bf16x3";
        case AZ_PREC_BF16: return "bf16";
        default: return "f32";
    }
}

int run(int argc, char** argv) {
    const Args args = parse(argc, argv);
    if (args.has("--help")) { usage(); return 0; }
    const std::string modelPath = args.get("--model", "");
    const std::string gameStr = args.get("--game", "gomoku");
    const core::GameType type = gameTypeOf(gameStr);
    int boardSize = args.getInt("--size", 0);
    if (boardSize <= 0) boardSize = type == core::GameType::GO ? 19 : 15;
    const int numGames = args.getInt("--num-games", 100);
    const int numSimulations = args.getInt("--simulations", 800);
    int numThreads = args.getInt("--threads", 0);
    if (numThreads <= 0) numThreads = std::max(1, (int)(std::thread::hardware_concurrency() * 0.75));
    const std::string outputDir = args.get("--output-dir", "data/games");
    const float temperature = args.getFloat("--temperature", 1.0f);
    const int tempDrop = args.getInt("--temp-drop", 30);
    const float finalTemp = args.getFloat("--final-temp", 0.0f);
    const float alpha = args.getFloat("--dirichlet-alpha", 0.03f);
    const float eps = args.getFloat("--dirichlet-epsilon", 0.25f);
    const bool variant = args.has("--variant");
    const int batchSize = args.getInt("--batch-size", 8);
    const int batchTimeout = args.getInt("--batch-timeout", 10);
    if (args.has("--no-gpu")) throw std::invalid_argument("--no-gpu: the engine has no CPU path");
    const bool fp16 = args.has("--fp16");
    const float cPuct = args.getFloat("--c-puct", 1.5f);
    const float fpu = args.getFloat("--fpu-reduction", 0.1f);
    const int vloss = args.getInt("--virtual-loss", 3);
    const bool useTT = !args.has("--no-tt");
    const bool pw = args.has("--progressive-widening");
    const int rank = args.getInt("--rank", 0), world = args.getInt("--world", 1);
    const int device = args.getInt("--device", -1);
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("--rank / --world");

    std::unique_ptr<selfplay::Distributed> dist;
    if (world > 1 || args.has("--dist-id-file")) {     // (a world of 1 with an id file: the same path on one GPU)
        if (!args.has("--dist-id-file")) throw std::invalid_argument("--world > 1 needs --dist-id-file");
        const std::string idf = args.get("--dist-id-file", "");
        selfplay::DistId id{};
        if (rank == 0) {
            id = selfplay::Distributed::uniqueId();
            selfplay::Distributed::writeIdFile(idf, id);
        } else {
            id = selfplay::Distributed::readIdFile(idf);
        }
        dist = std::make_unique<selfplay::Distributed>(rank, world, id, device);
    }

    // the network: rank 0 loads / initialises it; the other ranks get its shape and weights
    std::unique_ptr<nn::NeuralNetwork> net;
    nn::HipNeuralNetwork* hip = nullptr;
    const int netBlocks = args.getInt("--net-blocks", 0), netChannels = args.getInt("--net-channels", 0);
    const bool deviceNet = !modelPath.empty() || (netBlocks > 0 && netChannels > 0);
    if (deviceNet) {
        std::vector<double> shape(12, 0.0);
        if (rank == 0) {
            if (!modelPath.empty()) {
                net = nn::NeuralNetwork::create(modelPath, type, boardSize, true);
            } else {
                nn::NetShape s;
                s.boardSize = boardSize;
                s.inPlanes = type == core::GameType::GO ? 8 : 11;
                s.actionSize = boardSize * boardSize + (type == core::GameType::GO ? 1 : 0);
                s.channels = netChannels;
                s.blocks = netBlocks;
                s.precision = AZ_PREC_F32;
                s.maxBatch = std::max(batchSize, args.getInt("--concurrent-games", batchSize));
                auto h = std::make_unique<nn::HipNeuralNetwork>(s, device);
                h->initRandom((uint64_t)args.getInt("--seed", 1234));
                net = std::move(h);
            }
            hip = dynamic_cast<nn::HipNeuralNetwork*>(net.get());
            if (hip) {
                const nn::NetShape& s = hip->shape();
                shape = {(double)s.boardSize, (double)s.inPlanes, (double)s.channels, (double)s.blocks,
                         (double)s.actionSize, (double)s.headChannels, (double)s.pool, (double)s.fcHidden,
                         (double)s.residual, (double)s.convBias, (double)s.precision, (double)s.maxBatch};
            }
        }
        if (dist) {
            shape = dist->allreduceSum(shape);   // rank 0's shape (the others add zeros)
            if (rank != 0 && shape[0] > 0) {
                nn::NetShape s;
                int* f[12] = {&s.boardSize, &s.inPlanes, &s.channels, &s.blocks, &s.actionSize, &s.headChannels,
                              &s.pool, &s.fcHidden, &s.residual, &s.convBias, &s.precision, &s.maxBatch};
                for (int i = 0; i < 12; ++i) *f[i] = (int)shape[i];
                auto h = std::make_unique<nn::HipNeuralNetwork>(s, device);
                hip = h.get();
                net = std::move(h);
            }
            if (hip) dist->broadcastWeights(*hip, 0);
        }
        if (hip) {
            const bool x3 = hip->shape().channels % 128 == 0 || (hip->shape().channels == 64 && boardSize == 15);
            int prec = fp16 ? AZ_PREC_FP16 : x3 ? AZ_PREC_F16X3 : AZ_PREC_BF16X3;
            if (args.has("--precision")) prec = precisionOf(args.get("--precision", ""));
            if (!modelPath.empty() && !fp16 && !args.has("--precision")) prec = hip->shape().precision;   // as loaded
            hip->setPrecision(prec);
        }
    } else {
        net = std::make_unique<nn::RandomPolicyNetwork>(type, boardSize);
    }
    if (rank == 0) std::cout << "Network: " << net->getDeviceInfo() << " -- " << net->getModelInfo() << std::endl;

    const selfplay::GameShard shard = selfplay::shardGames(rank, world, numGames, 42);
    selfplay::SelfPlayManager mgr(net.get(), numGames, numSimulations, numThreads);
    mgr.setShard(shard);
    mgr.setExplorationParams(alpha, eps, temperature, tempDrop, finalTemp);
    mgr.setBatchConfig(batchSize, batchTimeout);
    if (args.has("--concurrent-games")) mgr.setConcurrentGames(args.getInt("--concurrent-games", batchSize));
    if (args.has("--max-moves")) mgr.setMaxMoves(args.getInt("--max-moves", 0));
    mgr.setSaveGames(true, outputDir);
    mcts::MCTSConfig mc;
    mc.numThreads = numThreads;
    mc.numSimulations = numSimulations;
    mc.cPuct = cPuct;
    mc.fpuReduction = fpu;
    mc.virtualLoss = vloss;
    mc.useDirichletNoise = true;    // as the reference's main: root noise on every search as well
    mc.dirichletAlpha = alpha;
    mc.dirichletEpsilon = eps;
    mc.useBatchInference = true;
    mc.useBatchedMCTS = !args.has("--no-batched-search");
    mc.batchSize = batchSize;
    mc.batchTimeoutMs = batchTimeout;
    mc.useProgressiveWidening = pw;
    mc.useFmapCache = useTT;
    mgr.setMctsConfig(mc);
    if (dist) mgr.setDistributed(dist.get());
    auto last = std::chrono::steady_clock::now();
    mgr.setProgressCallback([&](int gameId, int move, int totalGames, int totalMoves) {
        const auto now = std::chrono::steady_clock::now();
        if (std::chrono::duration<double>(now - last).count() >= 10.0) {
            last = now;
            std::cout << "[rank " << rank << "] game " << gameId + shard.firstGame << " move " << move << ", "
                      << totalMoves << " moves of " << totalGames << " games" << std::endl;
        }
    });

    if (rank == 0) {
        std::cout << "Starting self-play generation...\n"
                  << "Game: " << gameStr << ", board " << boardSize << "x" << boardSize << ", " << numGames
                  << " games over " << world << " rank(s), " << numSimulations << " simulations per move\n"
                  << "Output directory: " << outputDir << std::endl;
    }
    const auto t0 = std::chrono::high_resolution_clock::now();
    const auto records = mgr.generateGames(type, boardSize, variant);
    const long long duration =
        std::chrono::duration_cast<std::chrono::seconds>(std::chrono::high_resolution_clock::now() - t0).count();
    const int totalMoves = mgr.getTotalMovesCount();

    selfplay::RunMetadata md;
    md.game = gameStr;
    md.boardSize = boardSize;
    md.numGamesRequested = shard.numGames;
    md.numGamesCompleted = (int)records.size();
    md.simulations = numSimulations;
    md.threads = numThreads;
    md.temperature = temperature;
    md.tempDrop = tempDrop;
    md.finalTemp = finalTemp;
    md.dirichletAlpha = alpha;
    md.dirichletEpsilon = eps;
    md.variant = variant;
    md.modelPath = modelPath;
    md.totalMoves = totalMoves;
    md.avgMovesPerGame = records.empty() ? 0.0f : (float)totalMoves / (float)records.size();
    md.totalTimeSeconds = duration;
    md.avgMovesPerSecond = duration > 0 ? (float)totalMoves / (float)duration : 0.0f;
    md.useGpu = true;
    md.batchSize = batchSize;
    md.batchTimeout = batchTimeout;
    md.fp16Used = hip && hip->shape().precision == AZ_PREC_FP16;
    md.cPuct = cPuct;
    md.fpuReduction = fpu;
    md.virtualLoss = vloss;
    md.useTranspositionTable = useTT;
    md.progressiveWidening = pw;
    md.rank = rank;
    md.world = world;
    md.firstGameId = shard.firstGame;
    md.precision = hip ? precisionName(hip->shape().precision) : "";
    md.device = net->getDeviceInfo();
    if (dist) {
        const selfplay::JobStats& j = mgr.getJobStats();
        md.jobGamesCompleted = j.gamesCompleted;
        md.jobTotalMoves = j.totalMoves;
        md.jobSeconds = j.seconds;
        md.jobMovesPerSecond = j.seconds > 0 ? (double)j.totalMoves / j.seconds : 0.0;
    }
    const std::string path = selfplay::writeRunMetadata(md, outputDir);
    std::cout << "[rank " << rank << "] Generated " << records.size() << " games (" << totalMoves << " moves) in "
              << duration << " seconds" << std::endl;
    if (rank == 0 && dist)
        std::cout << "Job: " << md.jobGamesCompleted << " games, " << md.jobTotalMoves << " moves in " << std::fixed
                  << std::setprecision(1) << md.jobSeconds << " s = " << md.jobMovesPerSecond << " moves/s over "
                  << world << " GPU(s)" << std::endl;
    if (!path.empty()) std::cout << "Metadata saved to " << path << std::endl;
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return run(argc, argv);
    } catch (const std::exception& e) {
        std::cerr << "self_play: " << e.what() << std::endl;
        return 1;
    }
}
