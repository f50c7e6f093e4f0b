// alphazero/selfplay/run_metadata.h -- the run metadata file a self-play run leaves next to its
// games: the reference's metadata_<ticks>.json (src/selfplay/selfplay_main.cpp:353-389), same keys
// in the same order and the same text (ostream defaults: "temperature": 1, "dirichlet_alpha": 0.03),
// followed by the engine's extension keys (rank / world of a sharded run, the job-wide counters
// reduced over RCCL, the trunk precision, the device).  SURVEY.md row f1.
#pragma once
#include <string>

namespace alphazero {
namespace selfplay {

struct RunMetadata {
    // the reference's fields, in its order
    std::string game = "gomoku";
    int boardSize = 15;
    int numGamesRequested = 100;
    int numGamesCompleted = 0;
    int simulations = 800;
    int threads = 0;
    float temperature = 1.0f;
    int tempDrop = 30;
    float finalTemp = 0.0f;
    float dirichletAlpha = 0.03f;
    float dirichletEpsilon = 0.25f;
    bool variant = false;
    std::string modelPath;
    int totalMoves = 0;
    float avgMovesPerGame = 0.0f;
    long long totalTimeSeconds = 0;      // whole seconds (duration_cast<seconds>, as the reference)
    float avgMovesPerSecond = 0.0f;      // totalMoves / totalTimeSeconds (0 when under a second)
    bool useGpu = true;
    int batchSize = 8;
    int batchTimeout = 10;
    bool fp16Used = false;
    float cPuct = 1.5f;
    float fpuReduction = 0.1f;
    int virtualLoss = 3;
    bool useTranspositionTable = true;
    bool progressiveWidening = false;
    // engine extensions (written after the reference's keys)
    int rank = 0, world = 1;
    int firstGameId = 0;                 // this rank's global game ids start here
    std::string precision;               // trunk precision the net ran (fp16 / f16x3 / bf16x3 / f32)
    std::string device;
    long long jobGamesCompleted = -1;    // summed over the ranks (world > 1); -1: not reduced
    long long jobTotalMoves = -1;
    double jobSeconds = -1.0;            // the slowest rank's generateGames time
    double jobMovesPerSecond = -1.0;
};

// The file's text.
std::string runMetadataJson(const RunMetadata& m);
// Writes <outputDir>/metadata_<system_clock ticks>.json (the reference's name); returns the path,
// "" when the file cannot be opened (the reference then skips it silently).
std::string writeRunMetadata(const RunMetadata& m, const std::string& outputDir);

}  // namespace selfplay
}  // namespace alphazero
