// The self-play run metadata file (run_metadata.h; the reference's selfplay_main.cpp:353-389).
#include "alphazero/selfplay/run_metadata.h"

#include <chrono>
#include <fstream>
#include <sstream>

namespace alphazero {
namespace selfplay {

namespace {
// the reference writes its strings raw; quotes and backslashes are escaped here so that a path
// holding one still gives valid JSON (identical text for every other string)
std::string quoted(const std::string& s) {
    std::string o = "\"";
    for (char c : s) {
        if (c == '"' || c == '\\') o += '\\';
        o += c;
    }
    return o + "\"";
}
const char* tf(bool b) { return b ? "true" : "false"; }
}  // namespace

std::string runMetadataJson(const RunMetadata& m) {
    std::ostringstream f;   // default float formatting, as the reference's fresh std::ofstream
    f << "{\n";
    f << "  \"game\": " << quoted(m.game) << ",\n";
    f << "  \"board_size\": " << m.boardSize << ",\n";
    f << "  \"num_games_requested\": " << m.numGamesRequested << ",\n";
    f << "  \"num_games_completed\": " << m.numGamesCompleted << ",\n";
    f << "  \"simulations\": " << m.simulations << ",\n";
    f << "  \"threads\": " << m.threads << ",\n";
    f << "  \"temperature\": " << m.temperature << ",\n";
    f << "  \"temp_drop\": " << m.tempDrop << ",\n";
    f << "  \"final_temp\": " << m.finalTemp << ",\n";
    f << "  \"dirichlet_alpha\": " << m.dirichletAlpha << ",\n";
    f << "  \"dirichlet_epsilon\": " << m.dirichletEpsilon << ",\n";
    f << "  \"variant\": " << tf(m.variant) << ",\n";
    f << "  \"model_path\": " << quoted(m.modelPath) << ",\n";
    f << "  \"total_moves\": " << m.totalMoves << ",\n";
    f << "  \"avg_moves_per_game\": " << m.avgMovesPerGame << ",\n";
    f << "  \"total_time_seconds\": " << m.totalTimeSeconds << ",\n";
    f << "  \"avg_moves_per_second\": " << m.avgMovesPerSecond << ",\n";
    f << "  \"use_gpu\": " << tf(m.useGpu) << ",\n";
    f << "  \"batch_size\": " << m.batchSize << ",\n";
    f << "  \"batch_timeout\": " << m.batchTimeout << ",\n";
    f << "  \"fp16_used\": " << tf(m.fp16Used) << ",\n";
    f << "  \"c_puct\": " << m.cPuct << ",\n";
    f << "  \"fpu_reduction\": " << m.fpuReduction << ",\n";
    f << "  \"virtual_loss\": " << m.virtualLoss << ",\n";
    f << "  \"use_transposition_table\": " << tf(m.useTranspositionTable) << ",\n";
    f << "  \"progressive_widening\": " << tf(m.progressiveWidening) << ",\n";
    // engine extensions
    f << "  \"rank\": " << m.rank << ",\n";
    f << "  \"world\": " << m.world << ",\n";
    f << "  \"first_game_id\": " << m.firstGameId << ",\n";
    f << "  \"precision\": " << quoted(m.precision) << ",\n";
    f << "  \"device\": " << quoted(m.device) << ",\n";
    f << "  \"job_games_completed\": " << m.jobGamesCompleted << ",\n";
    f << "  \"job_total_moves\": " << m.jobTotalMoves << ",\n";
    f << "  \"job_seconds\": " << m.jobSeconds << ",\n";
    f << "  \"job_moves_per_second\": " << m.jobMovesPerSecond << "\n";
    f << "}\n";
    return f.str();
}

std::string writeRunMetadata(const RunMetadata& m, const std::string& outputDir) {
    const std::string path = outputDir + "/metadata_" +
                             std::to_string(std::chrono::system_clock::now().time_since_epoch().count()) + ".json";
    std::ofstream f(path);
    if (!f.is_open()) return "";
    f << runMetadataJson(m);
    return f ? path : "";
}

}  // namespace selfplay
}  // namespace alphazero
