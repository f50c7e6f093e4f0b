// oracle/chess_probe.cpp -- TEST INFRASTRUCTURE ONLY (probe, not an oracle).
// Constructs the reference's ChessState and asks for its legal moves; built by
// oracle/chess_probe.sh against a patched temp copy of the reference chess sources.
#include <cstdio>

#include "alphazero/games/chess/chess_state.h"

int main() {
    alphazero::chess::ChessState s;
    std::fprintf(stderr, "ChessState constructed, hash %llu\n", (unsigned long long)s.getHash());
    std::vector<int> m = s.getLegalMoves();   // chess_state.cpp:498 -> chess_rules.cpp:38
    std::fprintf(stderr, "legal moves: %zu\n", m.size());
    return 0;
}
