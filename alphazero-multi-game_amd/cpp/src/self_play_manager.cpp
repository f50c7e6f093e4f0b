// SelfPlayManager of the host API: generateGames = az_selfplay_run over device game slots.
#include "alphazero/selfplay/self_play_manager.h"

#include <chrono>
#include <cstdio>
#include <ctime>
#include <filesystem>
#include <iomanip>
#include <iostream>
#include <sstream>

#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/selfplay/distributed.h"

namespace alphazero {
namespace selfplay {

SelfPlayManager::SelfPlayManager(nn::NeuralNetwork* nn, int numGames, int numSimulations, int numThreads)
    : nn_(nn), numGames_(numGames), numSimulations_(numSimulations), numThreads_(numThreads) {}

SelfPlayManager::~SelfPlayManager() { abort_ = 1; }

void SelfPlayManager::setExplorationParams(float a, float e, float ti, int drop, float tf) {
    alpha_ = a; eps_ = e; tInit_ = ti; tempDrop_ = drop; tFinal_ = tf;
}

void SelfPlayManager::setSaveGames(bool s, const std::string& dir) { save_ = s; outDir_ = dir; }

void SelfPlayManager::setMctsConfig(const mcts::MCTSConfig& c) {
    mcts_ = c;
    if (c.useBatchedMCTS) { batchSize_ = c.batchSize; batchTimeoutMs_ = c.batchTimeoutMs; }
}

namespace {
struct RunCtx {
    SelfPlayManager* self;
    int firstGame;                  // global id of local game 0 (setShard)
    std::vector<std::string> files; // record files written by this attempt
    std::vector<GameRecord>* records;
    core::GameType type;
    bool variant;
    bool save;
    std::string dir;
    std::function<void(int, int, int, int)>* progress;
    std::atomic<int>* completed;
    std::atomic<int>* totalMoves;
    std::vector<char>* done;
};

void sink(void* user, int gid, int bs, int n, const az_move_rec* moves, int result) {
    auto* c = static_cast<RunCtx*>(user);
    GameRecord rec(c->type, bs, c->variant);
    for (int i = 0; i < n; ++i)
        rec.addMove(moves[i].action, std::vector<float>(moves[i].policy, moves[i].policy + moves[i].n_children),
                    moves[i].value, moves[i].thinking_time_ms);
    rec.setResult((core::GameResult)result);
    if (c->save) {   // <dir>/<id:03>_<YYYYmmdd_HHMMSS>.json (self_play_manager.cpp:220-229)
        const std::time_t t = std::time(nullptr);
        std::tm tm{};
        localtime_r(&t, &tm);
        std::ostringstream f;
        f << c->dir << "/" << std::setfill('0') << std::setw(3) << gid + c->firstGame << "_"
          << std::put_time(&tm, "%Y%m%d_%H%M%S") << ".json";
        if (rec.saveToFile(f.str())) c->files.push_back(f.str());
    }
    (*c->records)[gid] = std::move(rec);
    (*c->done)[gid] = 1;
    c->completed->fetch_add(1);
}

// AZ_EVAL_CALLBACK (a NeuralNetwork subclass without a device implementation): every leaf is the
// initial state of the game type plus the moves the engine reports; predictBatch evaluates them all
// (a throwing evaluator gets the reference's uniform / 0 fallback, parallel_mcts.cpp:903-916)
struct EvalCtx {
    nn::NeuralNetwork* nn;
    core::GameType type;
    int bs;
};

int host_eval(void* user, int n, const int* /*games*/, const int* len, const int* moves, int maxPath,
              const float* /*planes*/, int /*nPlanes*/, float* policy, float* value) {
    auto* c = static_cast<EvalCtx*>(user);
    std::vector<std::unique_ptr<core::IGameState>> leaves;
    for (int i = 0; i < n; ++i) {
        auto st = core::createGameState(c->type, c->bs, false);
        for (int k = 0; k < len[i]; ++k) st->makeMove(moves[(size_t)i * maxPath + k]);
        leaves.push_back(std::move(st));
    }
    const int A = leaves.empty() ? 0 : leaves[0]->getActionSpaceSize();
    std::vector<std::reference_wrapper<const core::IGameState>> refs;
    for (auto& l : leaves) refs.emplace_back(*l);
    std::vector<std::vector<float>> ps;
    std::vector<float> vs;
    bool ok = true;
    try { c->nn->predictBatch(refs, ps, vs); } catch (const std::exception&) { ok = false; }
    for (int i = 0; i < n; ++i) {
        const bool have = ok && i < (int)ps.size() && i < (int)vs.size();
        for (int a = 0; a < A; ++a)
            policy[(size_t)i * A + a] = have ? (a < (int)ps[i].size() ? ps[i][a] : 0.0f) : 1.0f / (float)A;
        value[i] = have ? vs[i] : 0.0f;
    }
    return 0;
}

void progress(void* user, int gid, int move, int total_games, int64_t /*total_moves*/) {
    auto* c = static_cast<RunCtx*>(user);
    const int tm = c->totalMoves->fetch_add(1);
    if (*c->progress) (*c->progress)(gid, move, total_games, tm);
}
}  // namespace

// One az_selfplay_run over numGames_ games: the records of the finished games, the record files
// written; returns the engine's status.
int SelfPlayManager::runGames(core::GameType type, int bs, bool variant, std::vector<GameRecord>& records,
                              std::vector<char>& done, std::vector<std::string>& written) {
    const bool go = type == core::GameType::GO;
    const mcts::DeviceEvaluator ev = mcts::deviceEvaluator(nn_);
    az_search_cfg c{};
    c.game = go ? AZ_GAME_GO : AZ_GAME_GOMOKU;
    c.n_games = slots_ > 0 ? slots_ : std::min(std::max(numGames_, 1), 2048);
    if (batchSet_ && batchSize_ > 0) c.n_games = std::min(c.n_games, batchSize_);   // network batch per step
    c.board_size = bs;
    c.num_simulations = numSimulations_;
    c.c_puct = mcts_.cPuct > 0.0f ? mcts_.cPuct : 1.5f;       // :177-178
    c.fpu_reduction = mcts_.fpuReduction >= 0.0f ? mcts_.fpuReduction : 0.1f;
    c.virtual_loss = mcts_.virtualLoss;
    c.eval_kind = ev.kind;
    c.eval_seed = ev.seed + (uint32_t)firstGame_;           // per-game evaluator streams by global id
    c.zobrist_seed = 12345u;
    c.noise_seed = noiseSeed_;
    c.noise_seed_stride = noiseStride_;
    c.use_dirichlet_each_search = mcts_.useDirichletNoise ? 1 : 0;
    c.dirichlet_alpha = alpha_;
    c.dirichlet_eps = eps_;
    c.tt_log2 = 20;                                            // TranspositionTable tt(1048576), :159
    az_search* s = nullptr;
    if (az_search_create(ev.engine, ev.net, &c, &s)) throw std::runtime_error(az_last_error());
    EvalCtx ectx{nn_, type, bs};
    if (ev.kind == AZ_EVAL_CALLBACK && az_search_set_evaluator(s, host_eval, &ectx)) {
        az_search_destroy(s);
        throw std::runtime_error(az_last_error());
    }
    log_ = EvalLog{};
    if (logSlot_ >= 0 && az_search_enable_eval_log(s, logSlot_, logCap_)) {
        az_search_destroy(s);
        throw std::runtime_error(az_last_error());
    }
    az_selfplay_cfg sc{tempDrop_, tInit_, tFinal_, 0};
    RunCtx ctx{this, firstGame_, {}, &records, type, variant, save_, outDir_, &progress_, &completed_, &totalMoves_,
               &done};
    int rc = az_selfplay_run(s, &sc, numGames_, maxMoves_, sink, progress, &ctx, &abort_);
    written = ctx.files;
    if (!rc && logSlot_ >= 0) {
        EvalLog& L = log_;
        L.policySize = go ? bs * bs + 1 : bs * bs;
        L.planes = go ? 8 : 11;
        L.cells = bs * bs;
        L.policy.resize((size_t)logCap_ * L.policySize);
        L.value.resize(logCap_);
        L.features.resize((size_t)logCap_ * L.planes * L.cells);
        rc = az_search_read_eval_log(s, L.policy.data(), L.value.data(), L.features.data(), &L.count);
        L.policy.resize((size_t)L.count * L.policySize);
        L.value.resize(L.count);
        L.features.resize((size_t)L.count * L.planes * L.cells);
    }
    az_search_destroy(s);
    return rc;
}

std::vector<GameRecord> SelfPlayManager::generateGames(core::GameType type, int boardSize, bool variant) {
    const bool go = type == core::GameType::GO;
    if (!go && type != core::GameType::GOMOKU) throw std::invalid_argument("generateGames: Gomoku or Go (no Chess rules)");
    if (variant) throw std::invalid_argument("generateGames: variant rules are not supported");
    running_ = true;
    abort_ = 0;
    const int bs = boardSize > 0 ? boardSize : go ? 19 : 15;
    if (save_) std::filesystem::create_directories(outDir_);
    std::vector<GameRecord> records;
    std::vector<char> done;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        // a load-time-chosen F16X3 net whose activations leave the fp16 range (AZ_ERR_RANGE) switches
        // to BF16X3 and the whole run repeats (its record files removed), as predictBatch does for a batch
        for (int attempt = 0;; ++attempt) {
            records.assign(numGames_, GameRecord(type, bs, variant));
            done.assign(numGames_, 0);
            completed_ = 0;
            totalMoves_ = 0;
            std::vector<std::string> written;
            const int rc = runGames(type, bs, variant, records, done, written);
            auto* hip = dynamic_cast<nn::HipNeuralNetwork*>(nn_);
            if (rc == AZ_ERR_RANGE && attempt == 0 && hip && hip->fallbackToFp32Range()) {
                for (const std::string& f : written) std::remove(f.c_str());
                continue;
            }
            if (rc) throw std::runtime_error(az_last_error());
            break;
        }
    } catch (...) {
        running_ = false;
        throw;
    }
    running_ = false;
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    job_ = JobStats{completed_.load(), totalMoves_.load(), secs};
    if (dist_) {   // the job's counters over the ranks (every rank reaches this point)
        const std::vector<double> sum = dist_->allreduceSum({(double)job_.gamesCompleted, (double)job_.totalMoves});
        job_.gamesCompleted = (long long)sum[0];
        job_.totalMoves = (long long)sum[1];
        job_.seconds = dist_->allreduceMax({secs})[0];
    }
    std::vector<GameRecord> out;   // finished games in game-id order (all of them unless aborted)
    for (int g = 0; g < numGames_; ++g)
        if (done[g]) out.push_back(std::move(records[g]));
    return out;
}

}  // namespace selfplay
}  // namespace alphazero
