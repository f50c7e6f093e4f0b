// _alphazero_cpp: the reference's Python module surface (src/pybind/python_bindings.cpp:26-458)
// over the MI355X host API.  The GIL is released around search / generateGames / predict /
// predictBatch / benchmark and re-acquired for the progress callback, as in the reference.
// Not bound: the LibTorch module classes (DDWRandWire, SEBlock, ...).
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "alphazero/nn/torchscript_reader.h"
#include "alphazero/games/go/go_state.h"
#include "alphazero/games/gomoku/gomoku_state.h"
#include "alphazero/mcts/parallel_mcts.h"
#include "alphazero/nn/hip_neural_network.h"
#include "alphazero/nn/random_policy_network.h"
#include "alphazero/selfplay/dataset.h"
#include "alphazero/selfplay/game_record.h"
#include "alphazero/selfplay/distributed.h"
#include "alphazero/selfplay/run_metadata.h"
#include "alphazero/selfplay/self_play_manager.h"

namespace py = pybind11;
using namespace alphazero;

static std::vector<std::reference_wrapper<const core::IGameState>> stateRefs(const py::list& states) {
    std::vector<std::reference_wrapper<const core::IGameState>> v;
    for (auto h : states) v.push_back(std::cref(h.cast<const core::IGameState&>()));
    return v;
}

// Python subclasses of NeuralNetwork (a user evaluator written in Python): ParallelMCTS reaches them
// through the AZ_EVAL_CALLBACK host evaluator.  predict / predictBatch take the GIL; predictBatch
// may be overridden as predictBatch(states) -> (policies, values).
class PyNeuralNetwork : public nn::NeuralNetwork {
 public:
    using nn::NeuralNetwork::NeuralNetwork;
    std::pair<std::vector<float>, float> predict(const core::IGameState& s) override {
        py::gil_scoped_acquire gil;
        py::function f = py::get_override(static_cast<const nn::NeuralNetwork*>(this), "predict");
        if (!f) throw std::runtime_error("NeuralNetwork subclass without predict");
        py::object r = f(py::cast(s, py::return_value_policy::reference));
        auto t = r.cast<py::tuple>();
        return {t[0].cast<std::vector<float>>(), t[1].cast<float>()};
    }
    void predictBatch(const std::vector<std::reference_wrapper<const core::IGameState>>& states,
                      std::vector<std::vector<float>>& policies, std::vector<float>& values) override {
        py::gil_scoped_acquire gil;
        py::function f = py::get_override(static_cast<const nn::NeuralNetwork*>(this), "predictBatch");
        policies.clear();
        values.clear();
        if (!f) {
            for (auto& r : states) {
                auto pv = predict(r.get());
                policies.push_back(pv.first);
                values.push_back(pv.second);
            }
            return;
        }
        py::list l;
        for (auto& r : states) l.append(py::cast(r.get(), py::return_value_policy::reference));
        auto t = f(l).cast<py::tuple>();
        policies = t[0].cast<std::vector<std::vector<float>>>();
        values = t[1].cast<std::vector<float>>();
    }
    std::future<std::pair<std::vector<float>, float>> predictAsync(const core::IGameState& s) override {
        std::promise<std::pair<std::vector<float>, float>> p;
        p.set_value(predict(s));
        return p.get_future();
    }
    bool isGpuAvailable() const override { return false; }
    std::string getDeviceInfo() const override { return "python"; }
    float getInferenceTimeMs() const override { return 0.0f; }
    int getBatchSize() const override { return 1; }
    std::string getModelInfo() const override { return "Python NeuralNetwork subclass"; }
    size_t getModelSizeBytes() const override { return 0; }
    void benchmark(int, int) override {}
    void enableDebugMode(bool) override {}
    void printModelSummary() const override {}
};

PYBIND11_MODULE(_alphazero_cpp, m) {
    m.doc() = "AlphaZero multi-game engine, MI355X (HIP) backend";

    py::enum_<core::GameType>(m, "GameType")
        .value("GOMOKU", core::GameType::GOMOKU).value("CHESS", core::GameType::CHESS).value("GO", core::GameType::GO)
        .export_values();
    py::enum_<core::GameResult>(m, "GameResult")
        .value("ONGOING", core::GameResult::ONGOING).value("DRAW", core::GameResult::DRAW)
        .value("WIN_PLAYER1", core::GameResult::WIN_PLAYER1).value("WIN_PLAYER2", core::GameResult::WIN_PLAYER2)
        .export_values();
    py::enum_<mcts::MCTSNodeSelection>(m, "MCTSNodeSelection")
        .value("UCB", mcts::MCTSNodeSelection::UCB).value("PUCT", mcts::MCTSNodeSelection::PUCT)
        .value("PROGRESSIVE_BIAS", mcts::MCTSNodeSelection::PROGRESSIVE_BIAS).value("RAVE", mcts::MCTSNodeSelection::RAVE)
        .export_values();
    py::enum_<mcts::MCTSSearchMode>(m, "MCTSSearchMode")
        .value("SERIAL", mcts::MCTSSearchMode::SERIAL).value("PARALLEL", mcts::MCTSSearchMode::PARALLEL)
        .value("BATCHED", mcts::MCTSSearchMode::BATCHED)
        .export_values();

    py::class_<core::IGameState>(m, "IGameState")
        .def("getLegalMoves", &core::IGameState::getLegalMoves)
        .def("isLegalMove", &core::IGameState::isLegalMove)
        .def("makeMove", &core::IGameState::makeMove)
        .def("undoMove", &core::IGameState::undoMove)
        .def("isTerminal", &core::IGameState::isTerminal)
        .def("getGameResult", &core::IGameState::getGameResult)
        .def("getCurrentPlayer", &core::IGameState::getCurrentPlayer)
        .def("getBoardSize", &core::IGameState::getBoardSize)
        .def("getActionSpaceSize", &core::IGameState::getActionSpaceSize)
        .def("getTensorRepresentation", &core::IGameState::getTensorRepresentation)
        .def("getEnhancedTensorRepresentation", &core::IGameState::getEnhancedTensorRepresentation)
        .def("getHash", &core::IGameState::getHash)
        .def("actionToString", &core::IGameState::actionToString)
        .def("stringToAction", &core::IGameState::stringToAction)
        .def("toString", &core::IGameState::toString)
        .def("getMoveHistory", &core::IGameState::getMoveHistory)
        .def("getGameType", &core::IGameState::getGameType)
        .def("clone", [](const core::IGameState& s) { return s.clone(); });

    py::class_<gomoku::GomokuState, core::IGameState>(m, "GomokuState")
        .def(py::init<int, bool, bool, int, bool>(), py::arg("board_size") = 15, py::arg("use_renju") = false,
             py::arg("use_omok") = false, py::arg("seed") = 0, py::arg("use_pro_long_opening") = false)
        .def("is_occupied", &gomoku::GomokuState::is_occupied)
        .def("get_board", &gomoku::GomokuState::get_board);

    // not in the reference module (its GoState is C++-only); bound for the device Go path
    py::class_<go::GoState, core::IGameState>(m, "GoState")
        .def(py::init<int, float, bool, bool>(), py::arg("board_size") = 19, py::arg("komi") = 7.5f,
             py::arg("chinese_rules") = true, py::arg("enforce_superko") = true)
        .def("getStone", py::overload_cast<int>(&go::GoState::getStone, py::const_))
        .def("getCapturedStones", &go::GoState::getCapturedStones)
        .def("getKoPoint", &go::GoState::getKoPoint)
        .def("getKomi", &go::GoState::getKomi)
        .def("calculateScore", &go::GoState::calculateScore);

    m.def("createGameState", &core::createGameState, py::arg("type"), py::arg("boardSize") = 0,
          py::arg("variantRules") = false);

    py::class_<nn::NeuralNetwork, PyNeuralNetwork>(m, "NeuralNetwork")
        .def(py::init<>())
        .def("predict", [](nn::NeuralNetwork& self, const core::IGameState& s) {
            py::gil_scoped_release release;
            return self.predict(s);
        })
        .def("predictBatch", [](nn::NeuralNetwork& self, const py::list& states) {
            auto refs = stateRefs(states);
            std::vector<std::vector<float>> p;
            std::vector<float> v;
            {
                py::gil_scoped_release release;
                self.predictBatch(refs, p, v);
            }
            return py::make_tuple(p, v);
        })
        .def("predictBatch", [](nn::NeuralNetwork& self, const py::list& states, py::list policies, py::list values) {
            // reference signature: output lists filled in place
            auto refs = stateRefs(states);
            std::vector<std::vector<float>> p;
            std::vector<float> v;
            {
                py::gil_scoped_release release;
                self.predictBatch(refs, p, v);
            }
            policies.attr("clear")();
            values.attr("clear")();
            for (auto& x : p) policies.append(py::cast(x));
            for (float x : v) values.append(x);
        })
        .def("isGpuAvailable", &nn::NeuralNetwork::isGpuAvailable)
        .def("getDeviceInfo", &nn::NeuralNetwork::getDeviceInfo)
        .def("getInferenceTimeMs", &nn::NeuralNetwork::getInferenceTimeMs)
        .def("getBatchSize", &nn::NeuralNetwork::getBatchSize)
        .def("getModelInfo", &nn::NeuralNetwork::getModelInfo)
        .def("getModelSizeBytes", &nn::NeuralNetwork::getModelSizeBytes)
        .def("benchmark", [](nn::NeuralNetwork& self, int n, int b) {
            py::gil_scoped_release release;
            self.benchmark(n, b);
        }, py::arg("numIterations") = 100, py::arg("batchSize") = 16)
        .def("enableDebugMode", &nn::NeuralNetwork::enableDebugMode)
        .def("is_gil_safe", [](nn::NeuralNetwork&) { return true; });

    py::class_<nn::HipNeuralNetwork, nn::NeuralNetwork>(m, "HipNeuralNetwork")
        .def(py::init([](int boardSize, int channels, int blocks, int inPlanes, int precision, int maxBatch,
                         int residual, int convBias, int device) {
                 nn::NetShape s;
                 s.boardSize = boardSize; s.channels = channels; s.blocks = blocks; s.inPlanes = inPlanes;
                 s.actionSize = boardSize * boardSize; s.precision = precision; s.maxBatch = maxBatch;
                 s.residual = residual; s.convBias = convBias;
                 return std::make_unique<nn::HipNeuralNetwork>(s, device);
             }),
             py::arg("boardSize") = 15, py::arg("channels") = 256, py::arg("blocks") = 20, py::arg("inPlanes") = 11,
             py::arg("precision") = (int)AZ_PREC_FP16, py::arg("maxBatch") = 2048, py::arg("residual") = 1,
             py::arg("convBias") = 0, py::arg("device") = -1)
        .def("loadWeights", [](nn::HipNeuralNetwork& self, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
            std::vector<float> blob(a.data(), a.data() + a.size());
            self.loadWeights(blob);
        })
        .def("initRandom", &nn::HipNeuralNetwork::initRandom)
        .def("setPrecision", &nn::HipNeuralNetwork::setPrecision)
        .def("save", &nn::HipNeuralNetwork::save)
        .def_static("load", &nn::HipNeuralNetwork::load, py::arg("path"), py::arg("device") = -1)
        .def_static("loadTorchScript", &nn::HipNeuralNetwork::loadTorchScript, py::arg("path"), py::arg("gameType"),
                    py::arg("boardSize") = 0, py::arg("precision") = -1, py::arg("maxBatch") = 2048,
                    py::arg("device") = -1);
    // host-only reader of a TorchScript archive's tensors (no code executed): [(name, array)] in
    // state_dict order, and the plain-ResNet shape + canonical blob the engine loads
    m.def("readTorchScript", [](const std::string& path) {
        py::list out;
        for (auto& t : nn::readTorchScript(path)) {
            std::vector<py::ssize_t> shape(t.shape.begin(), t.shape.end());
            py::array_t<float> a(shape);
            std::copy(t.data.begin(), t.data.end(), a.mutable_data());
            out.append(py::make_tuple(t.name, a));
        }
        return out;
    }, py::arg("path"));
    m.def("torchScriptResNet", [](const std::string& path, core::GameType type, int boardSize) {
        nn::NetShape s;
        std::vector<float> blob = nn::torchScriptResNet(path, type, boardSize, s);
        py::dict d;
        d["board"] = s.boardSize; d["in_planes"] = s.inPlanes; d["channels"] = s.channels; d["blocks"] = s.blocks;
        d["action_size"] = s.actionSize; d["head_channels"] = s.headChannels; d["pool"] = s.pool;
        d["fc_hidden"] = s.fcHidden; d["residual"] = s.residual; d["conv_bias"] = s.convBias;
        py::array_t<float> a((py::ssize_t)blob.size());
        std::copy(blob.begin(), blob.end(), a.mutable_data());
        return py::make_tuple(d, a);
    }, py::arg("path"), py::arg("gameType"), py::arg("boardSize") = 0);
    // TorchNeuralNetwork::createDDWRandWireResNet / DDWRandWireResNetCpp(input_channels, output_size,
    // channels=128, num_blocks=20) (reference python_bindings.cpp:168-173) on the device engine
    m.def("createDDWRandWireResNet",
          [](int input_channels, int output_size, int channels, int num_blocks, int board_size, int max_batch,
             int device) {
              return nn::HipNeuralNetwork::createDDWRandWireResNet(input_channels, output_size, channels, num_blocks,
                                                                   board_size, max_batch, device);
          },
          py::arg("input_channels"), py::arg("output_size"), py::arg("channels") = 128, py::arg("num_blocks") = 20,
          py::arg("board_size") = 15, py::arg("max_batch") = 256, py::arg("device") = -1);

    py::class_<nn::RandomPolicyNetwork, nn::NeuralNetwork>(m, "RandomPolicyNetwork")
        .def(py::init<core::GameType, int, unsigned int>(), py::arg("gameType"), py::arg("boardSize") = 0,
             py::arg("seed") = 0);

    m.def("createNeuralNetwork", &nn::NeuralNetwork::create, py::arg("modelPath"), py::arg("gameType"),
          py::arg("boardSize") = 0, py::arg("useGpu") = true);

    py::class_<mcts::MCTSConfig>(m, "MCTSConfig")
        .def(py::init<>())
        .def_readwrite("numThreads", &mcts::MCTSConfig::numThreads)
        .def_readwrite("numSimulations", &mcts::MCTSConfig::numSimulations)
        .def_readwrite("cPuct", &mcts::MCTSConfig::cPuct)
        .def_readwrite("fpuReduction", &mcts::MCTSConfig::fpuReduction)
        .def_readwrite("virtualLoss", &mcts::MCTSConfig::virtualLoss)
        .def_readwrite("maxSearchDepth", &mcts::MCTSConfig::maxSearchDepth)
        .def_readwrite("useDirichletNoise", &mcts::MCTSConfig::useDirichletNoise)
        .def_readwrite("dirichletAlpha", &mcts::MCTSConfig::dirichletAlpha)
        .def_readwrite("dirichletEpsilon", &mcts::MCTSConfig::dirichletEpsilon)
        .def_readwrite("useBatchInference", &mcts::MCTSConfig::useBatchInference)
        .def_readwrite("useTemporalDifference", &mcts::MCTSConfig::useTemporalDifference)
        .def_readwrite("tdLambda", &mcts::MCTSConfig::tdLambda)
        .def_readwrite("useProgressiveWidening", &mcts::MCTSConfig::useProgressiveWidening)
        .def_readwrite("minVisitsForWidening", &mcts::MCTSConfig::minVisitsForWidening)
        .def_readwrite("progressiveWideningBase", &mcts::MCTSConfig::progressiveWideningBase)
        .def_readwrite("progressiveWideningExponent", &mcts::MCTSConfig::progressiveWideningExponent)
        .def_readwrite("selectionStrategy", &mcts::MCTSConfig::selectionStrategy)
        .def_readwrite("batchSize", &mcts::MCTSConfig::batchSize)
        .def_readwrite("useBatchedMCTS", &mcts::MCTSConfig::useBatchedMCTS)
        .def_readwrite("batchTimeoutMs", &mcts::MCTSConfig::batchTimeoutMs)
        .def_readwrite("searchMode", &mcts::MCTSConfig::searchMode)
        .def_readwrite("transpositionTableSize", &mcts::MCTSConfig::transpositionTableSize);

    py::class_<mcts::MCTSStats>(m, "MCTSStats")
        .def_property_readonly("nodesCreated", [](const mcts::MCTSStats& s) { return s.nodesCreated.load(); })
        .def_property_readonly("nodesExpanded", [](const mcts::MCTSStats& s) { return s.nodesExpanded.load(); })
        .def_property_readonly("nodesTotalVisits", [](const mcts::MCTSStats& s) { return s.nodesTotalVisits.load(); })
        .def_property_readonly("simulationCount", [](const mcts::MCTSStats& s) { return s.simulationCount.load(); })
        .def_property_readonly("evaluationCalls", [](const mcts::MCTSStats& s) { return s.evaluationCalls.load(); })
        .def_property_readonly("cacheHits", [](const mcts::MCTSStats& s) { return s.cacheHits.load(); })
        .def_property_readonly("cacheMisses", [](const mcts::MCTSStats& s) { return s.cacheMisses.load(); })
        .def_property_readonly("batchedEvaluations", [](const mcts::MCTSStats& s) { return s.batchedEvaluations.load(); })
        .def_property_readonly("totalBatches", [](const mcts::MCTSStats& s) { return s.totalBatches.load(); });

    py::class_<mcts::TranspositionTable>(m, "TranspositionTable")
        .def(py::init<size_t, size_t>(), py::arg("size") = 1048576, py::arg("numShards") = 1024)
        .def("getSize", &mcts::TranspositionTable::getSize)
        .def("getHitRate", &mcts::TranspositionTable::getHitRate)
        .def("getLookups", &mcts::TranspositionTable::getLookups)
        .def("getHits", &mcts::TranspositionTable::getHits)
        .def("getEntryCount", &mcts::TranspositionTable::getEntryCount)
        .def("getMemoryUsageBytes", &mcts::TranspositionTable::getMemoryUsageBytes)
        .def("clear", &mcts::TranspositionTable::clear)
        .def("resize", &mcts::TranspositionTable::resize);

    // python_bindings.cpp:245-253 of the reference; here a host snapshot (ParallelMCTS.getRootNode)
    py::class_<mcts::MCTSNode, std::shared_ptr<mcts::MCTSNode>>(m, "MCTSNode")
        .def("getUcbScore", &mcts::MCTSNode::getUcbScore, py::arg("cPuct"), py::arg("currentPlayer"),
             py::arg("fpuReduction") = 0.0f, py::arg("parentVisits") = 0)
        .def("getTerminalValue", &mcts::MCTSNode::getTerminalValue)
        .def("getValue", &mcts::MCTSNode::getValue)
        .def("getBestAction", &mcts::MCTSNode::getBestAction)
        .def("getBestActions", &mcts::MCTSNode::getBestActions)
        .def("getVisitCountDistribution", &mcts::MCTSNode::getVisitCountDistribution, py::arg("temperature") = 1.0f)
        .def("toString", &mcts::MCTSNode::toString, py::arg("maxDepth") = 1)
        .def("hasChildren", &mcts::MCTSNode::hasChildren)
        .def_readonly("visitCount", &mcts::MCTSNode::visitCount)
        .def_readonly("valueSum", &mcts::MCTSNode::valueSum)
        .def_readonly("virtualLoss", &mcts::MCTSNode::virtualLoss)
        .def_readonly("prior", &mcts::MCTSNode::prior)
        .def_readonly("action", &mcts::MCTSNode::action)
        .def_readonly("isExpanded", &mcts::MCTSNode::isExpanded)
        .def_readonly("isTerminal", &mcts::MCTSNode::isTerminal)
        .def_readonly("actions", &mcts::MCTSNode::actions)
        .def_readonly("children", &mcts::MCTSNode::children);

    py::class_<mcts::SearchGroup>(m, "SearchGroup")
        .def(py::init<nn::NeuralNetwork*, const mcts::MCTSConfig&, const core::IGameState&, int,
                      const mcts::TranspositionTable*>(),
             py::arg("nn"), py::arg("config"), py::arg("prototype"), py::arg("capacity"), py::arg("tt") = nullptr,
             py::keep_alive<1, 2>())
        .def("capacity", &mcts::SearchGroup::capacity)
        .def("members", &mcts::SearchGroup::members)
        .def("searches", &mcts::SearchGroup::searches)
        .def("deviceRuns", &mcts::SearchGroup::deviceRuns)
        .def("setGatherMicros", &mcts::SearchGroup::setGatherMicros);

    py::class_<mcts::ParallelMCTS>(m, "ParallelMCTS")
        .def(py::init<const core::IGameState&, nn::NeuralNetwork*, mcts::TranspositionTable*, int, int, float, float, int>(),
             py::arg("rootState"), py::arg("nn") = nullptr, py::arg("tt") = nullptr, py::arg("numThreads") = 1,
             py::arg("numSimulations") = 800, py::arg("cPuct") = 1.5f, py::arg("fpuReduction") = 0.0f,
             py::arg("virtualLoss") = 3, py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
        .def(py::init<const core::IGameState&, const mcts::MCTSConfig&, nn::NeuralNetwork*, mcts::TranspositionTable*>(),
             py::arg("rootState"), py::arg("config"), py::arg("nn") = nullptr, py::arg("tt") = nullptr,
             py::keep_alive<1, 4>(), py::keep_alive<1, 5>())
        .def(py::init<const core::IGameState&, mcts::SearchGroup&>(), py::arg("rootState"), py::arg("group"),
             py::keep_alive<1, 3>())
        .def("inGroup", &mcts::ParallelMCTS::inGroup)
        .def("slot", &mcts::ParallelMCTS::slot)
        .def("search", [](mcts::ParallelMCTS& self) {
            py::gil_scoped_release release;
            self.search();
        })
        .def("runSingleSimulation", [](mcts::ParallelMCTS& self) {
            py::gil_scoped_release release;
            self.runSingleSimulation();
        })
        .def("runBatchedSearch", [](mcts::ParallelMCTS& self) {
            py::gil_scoped_release release;
            self.runBatchedSearch();
        })
        .def("releaseMemory", &mcts::ParallelMCTS::releaseMemory, py::arg("visitThreshold") = 10)
        .def("getRootNode", &mcts::ParallelMCTS::getRootNode)
        .def("selectAction", &mcts::ParallelMCTS::selectAction, py::arg("isTraining") = false, py::arg("temperature") = 1.0f)
        .def("getActionProbabilities", &mcts::ParallelMCTS::getActionProbabilities, py::arg("temperature") = 1.0f)
        .def("getChildActions", &mcts::ParallelMCTS::getChildActions)
        .def("getRootValue", &mcts::ParallelMCTS::getRootValue)
        .def("updateWithMove", &mcts::ParallelMCTS::updateWithMove)
        .def("addDirichletNoise", &mcts::ParallelMCTS::addDirichletNoise, py::arg("alpha") = 0.03f,
             py::arg("epsilon") = 0.25f)
        .def("setNumThreads", &mcts::ParallelMCTS::setNumThreads)
        .def("setNumSimulations", &mcts::ParallelMCTS::setNumSimulations)
        .def("setCPuct", &mcts::ParallelMCTS::setCPuct)
        .def("setFpuReduction", &mcts::ParallelMCTS::setFpuReduction)
        .def("setVirtualLoss", &mcts::ParallelMCTS::setVirtualLoss)
        .def("setNeuralNetwork", &mcts::ParallelMCTS::setNeuralNetwork, py::keep_alive<1, 2>())
        .def("setTranspositionTable", &mcts::ParallelMCTS::setTranspositionTable, py::keep_alive<1, 2>())
        .def("setSelectionStrategy", &mcts::ParallelMCTS::setSelectionStrategy)
        .def("setConfig", &mcts::ParallelMCTS::setConfig)
        .def("enableBatchedMCTS", &mcts::ParallelMCTS::enableBatchedMCTS)
        .def("setBatchSize", &mcts::ParallelMCTS::setBatchSize)
        .def("setBatchTimeout", &mcts::ParallelMCTS::setBatchTimeout)
        .def("setDeterministicMode", &mcts::ParallelMCTS::setDeterministicMode)
        .def("setDebugMode", &mcts::ParallelMCTS::setDebugMode)
        .def("printSearchStats", &mcts::ParallelMCTS::printSearchStats)
        .def("getSearchInfo", &mcts::ParallelMCTS::getSearchInfo)
        .def("printSearchPath", &mcts::ParallelMCTS::printSearchPath)
        .def("getMemoryUsage", &mcts::ParallelMCTS::getMemoryUsage)
        .def("analyzePosition", &mcts::ParallelMCTS::analyzePosition, py::arg("topN") = 10)
        .def("getStats", &mcts::ParallelMCTS::getStats, py::return_value_policy::reference_internal);

    py::class_<selfplay::MoveData>(m, "MoveData")
        .def(py::init<>())
        .def_readwrite("action", &selfplay::MoveData::action)
        .def_readwrite("policy", &selfplay::MoveData::policy)
        .def_readwrite("value", &selfplay::MoveData::value)
        .def_readwrite("thinking_time_ms", &selfplay::MoveData::thinking_time_ms)
        .def("toJson", &selfplay::MoveData::toJson)
        .def_static("fromJson", &selfplay::MoveData::fromJson);

    py::class_<selfplay::GameRecord>(m, "GameRecord")
        .def(py::init<core::GameType, int, bool>(), py::arg("gameType"), py::arg("boardSize"),
             py::arg("useVariantRules") = false)
        .def("addMove", &selfplay::GameRecord::addMove)
        .def("setResult", &selfplay::GameRecord::setResult)
        .def("getMetadata", &selfplay::GameRecord::getMetadata)
        .def("getMoves", &selfplay::GameRecord::getMoves)
        .def("getResult", &selfplay::GameRecord::getResult)
        .def("toJson", &selfplay::GameRecord::toJson)
        .def("saveToFile", &selfplay::GameRecord::saveToFile)
        .def("setTimestamp", [](selfplay::GameRecord& r, int64_t unix_seconds) {
            r.setTimestamp(std::chrono::system_clock::from_time_t((std::time_t)unix_seconds));
        })
        .def_static("fromJson", &selfplay::GameRecord::fromJson)
        .def_static("loadFromFile", &selfplay::GameRecord::loadFromFile);
    m.def("jsonNumber", &selfplay::jsonNumber);

    // python_bindings.cpp:339-358
    py::class_<selfplay::TrainingExample>(m, "TrainingExample")
        .def(py::init<>())
        .def_readwrite("state", &selfplay::TrainingExample::state)
        .def_readwrite("policy", &selfplay::TrainingExample::policy)
        .def_readwrite("value", &selfplay::TrainingExample::value)
        .def("toJson", &selfplay::TrainingExample::toJson)
        .def_static("fromJson", &selfplay::TrainingExample::fromJson);

    py::class_<selfplay::Dataset>(m, "Dataset")
        .def(py::init<>())
        .def(py::init<int>(), py::arg("device"))
        .def("addGameRecord", &selfplay::Dataset::addGameRecord, py::arg("record"),
             py::arg("useEnhancedFeatures") = true)
        .def("extractExamples", [](selfplay::Dataset& self, bool aug) {
            py::gil_scoped_release release;
            self.extractExamples(aug);
        }, py::arg("includeAugmentations") = true)
        .def("size", &selfplay::Dataset::size)
        .def("getBatch", &selfplay::Dataset::getBatch)
        .def("shuffle", &selfplay::Dataset::shuffle)
        .def("saveToFile", &selfplay::Dataset::saveToFile)
        .def("loadFromFile", &selfplay::Dataset::loadFromFile)
        .def("getRandomSubset", &selfplay::Dataset::getRandomSubset)
        .def("setSeed", &selfplay::Dataset::setSeed)
        .def("getExamples", &selfplay::Dataset::getExamples)
        .def("lastExtractMs", &selfplay::Dataset::lastExtractMs);

    py::class_<selfplay::RunMetadata>(m, "RunMetadata")
        .def(py::init<>())
        .def_readwrite("game", &selfplay::RunMetadata::game)
        .def_readwrite("boardSize", &selfplay::RunMetadata::boardSize)
        .def_readwrite("numGamesRequested", &selfplay::RunMetadata::numGamesRequested)
        .def_readwrite("numGamesCompleted", &selfplay::RunMetadata::numGamesCompleted)
        .def_readwrite("simulations", &selfplay::RunMetadata::simulations)
        .def_readwrite("threads", &selfplay::RunMetadata::threads)
        .def_readwrite("temperature", &selfplay::RunMetadata::temperature)
        .def_readwrite("tempDrop", &selfplay::RunMetadata::tempDrop)
        .def_readwrite("finalTemp", &selfplay::RunMetadata::finalTemp)
        .def_readwrite("dirichletAlpha", &selfplay::RunMetadata::dirichletAlpha)
        .def_readwrite("dirichletEpsilon", &selfplay::RunMetadata::dirichletEpsilon)
        .def_readwrite("variant", &selfplay::RunMetadata::variant)
        .def_readwrite("modelPath", &selfplay::RunMetadata::modelPath)
        .def_readwrite("totalMoves", &selfplay::RunMetadata::totalMoves)
        .def_readwrite("avgMovesPerGame", &selfplay::RunMetadata::avgMovesPerGame)
        .def_readwrite("totalTimeSeconds", &selfplay::RunMetadata::totalTimeSeconds)
        .def_readwrite("avgMovesPerSecond", &selfplay::RunMetadata::avgMovesPerSecond)
        .def_readwrite("useGpu", &selfplay::RunMetadata::useGpu)
        .def_readwrite("batchSize", &selfplay::RunMetadata::batchSize)
        .def_readwrite("batchTimeout", &selfplay::RunMetadata::batchTimeout)
        .def_readwrite("fp16Used", &selfplay::RunMetadata::fp16Used)
        .def_readwrite("cPuct", &selfplay::RunMetadata::cPuct)
        .def_readwrite("fpuReduction", &selfplay::RunMetadata::fpuReduction)
        .def_readwrite("virtualLoss", &selfplay::RunMetadata::virtualLoss)
        .def_readwrite("useTranspositionTable", &selfplay::RunMetadata::useTranspositionTable)
        .def_readwrite("progressiveWidening", &selfplay::RunMetadata::progressiveWidening)
        .def_readwrite("rank", &selfplay::RunMetadata::rank)
        .def_readwrite("world", &selfplay::RunMetadata::world)
        .def_readwrite("firstGameId", &selfplay::RunMetadata::firstGameId)
        .def_readwrite("precision", &selfplay::RunMetadata::precision)
        .def_readwrite("device", &selfplay::RunMetadata::device)
        .def_readwrite("jobGamesCompleted", &selfplay::RunMetadata::jobGamesCompleted)
        .def_readwrite("jobTotalMoves", &selfplay::RunMetadata::jobTotalMoves)
        .def_readwrite("jobSeconds", &selfplay::RunMetadata::jobSeconds)
        .def_readwrite("jobMovesPerSecond", &selfplay::RunMetadata::jobMovesPerSecond);
    m.def("runMetadataJson", &selfplay::runMetadataJson);
    m.def("writeRunMetadata", &selfplay::writeRunMetadata, py::arg("metadata"), py::arg("outputDir"));
    py::class_<selfplay::GameShard>(m, "GameShard")
        .def(py::init<>())
        .def_readwrite("firstGame", &selfplay::GameShard::firstGame)
        .def_readwrite("numGames", &selfplay::GameShard::numGames)
        .def_readwrite("noiseSeed", &selfplay::GameShard::noiseSeed);
    m.def("shardGames", &selfplay::shardGames, py::arg("rank"), py::arg("world"), py::arg("totalGames"),
          py::arg("noiseSeed") = 42u);

    py::class_<selfplay::SelfPlayManager>(m, "SelfPlayManager")
        .def(py::init<nn::NeuralNetwork*, int, int, int>(), py::arg("neuralNetwork"), py::arg("numGames") = 100,
             py::arg("numSimulations") = 800, py::arg("numThreads") = 4, py::keep_alive<1, 2>())
        .def("generateGames", [](selfplay::SelfPlayManager& self, core::GameType t, int bs, bool variant) {
            py::gil_scoped_release release;
            return self.generateGames(t, bs, variant);
        }, py::arg("gameType"), py::arg("boardSize") = 0, py::arg("useVariantRules") = false)
        .def("setExplorationParams", &selfplay::SelfPlayManager::setExplorationParams,
             py::arg("dirichletAlpha") = 0.03f, py::arg("dirichletEpsilon") = 0.25f,
             py::arg("initialTemperature") = 1.0f, py::arg("temperatureDropMove") = 30,
             py::arg("finalTemperature") = 0.0f)
        .def("setProgressCallback", [](selfplay::SelfPlayManager& self, std::function<void(int, int, int, int)> cb) {
            self.setProgressCallback([cb](int g, int mv, int tg, int tm) {
                py::gil_scoped_acquire acquire;
                cb(g, mv, tg, tm);
            });
        })
        .def("setBatchConfig", &selfplay::SelfPlayManager::setBatchConfig)
        .def("setSaveGames", &selfplay::SelfPlayManager::setSaveGames, py::arg("saveGames"),
             py::arg("outputDir") = "games")
        .def("setAbort", &selfplay::SelfPlayManager::setAbort)
        .def("isRunning", &selfplay::SelfPlayManager::isRunning)
        .def("setMctsConfig", &selfplay::SelfPlayManager::setMctsConfig)
        .def("getCompletedGamesCount", &selfplay::SelfPlayManager::getCompletedGamesCount)
        .def("getTotalMovesCount", &selfplay::SelfPlayManager::getTotalMovesCount)
        .def("setConcurrentGames", &selfplay::SelfPlayManager::setConcurrentGames)
        .def("setMaxMoves", &selfplay::SelfPlayManager::setMaxMoves)
        .def("setSeeds", &selfplay::SelfPlayManager::setSeeds)
        .def("setShard", &selfplay::SelfPlayManager::setShard)
        .def("getFirstGameId", &selfplay::SelfPlayManager::getFirstGameId)
        .def("setEvalLog", &selfplay::SelfPlayManager::setEvalLog, py::arg("slot"), py::arg("capacity"))
        .def("getEvalLog", [](const selfplay::SelfPlayManager& self) {
            // (policy [n][NA], value [n], planes [n][C][bs][bs]) as numpy arrays
            const auto& L = self.getEvalLog();
            const int bs = (int)std::lround(std::sqrt((double)L.cells));
            py::array_t<float> pol({(py::ssize_t)L.count, (py::ssize_t)L.policySize});
            py::array_t<float> val((py::ssize_t)L.count);
            py::array_t<float> pl({(py::ssize_t)L.count, (py::ssize_t)L.planes, (py::ssize_t)bs, (py::ssize_t)bs});
            std::copy(L.policy.begin(), L.policy.end(), pol.mutable_data());
            std::copy(L.value.begin(), L.value.end(), val.mutable_data());
            std::copy(L.features.begin(), L.features.end(), pl.mutable_data());
            return py::make_tuple(pol, val, pl);
        });
}
