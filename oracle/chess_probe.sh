#!/usr/bin/env bash
# oracle/chess_probe.sh -- TEST INFRASTRUCTURE ONLY: shows that the reference's ChessState cannot
# generate a move, so there is no reference chess behaviour to reproduce.
#
# Copies the reference chess sources to a temp dir OUTSIDE the repository, applies two patches that
# only make them compile (no arithmetic change), builds oracle/chess_probe.cpp against them, runs it:
#   P7 chess_rules.cpp:2   include chess_state.h before chess_rules.h (chess_rules.h:165 uses
#                          PieceColor::WHITE of an incomplete enum)
#   P8 chess_state.cpp:30  zobrist_(GameType::CHESS, 8, 12) -> zobrist_(8, 12, 2, 12345u) (as P2)
# Expected: the constructor returns, getLegalMoves() never does -- ChessState::makeMove calls
# isLegalMove (chess_state.cpp:977), which calls ChessRules::moveExposesKing (chess_rules.cpp:116),
# which calls cloneWithMove (chess_rules.cpp:747) -> makeMove again: unbounded recursion, stack
# overflow (SIGSEGV, exit 139).
set -uo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
[ -d "$REF/src/games/chess" ] || { echo "chess_probe.sh: $REF not present" >&2; exit 0; }
TMP=$(mktemp -d /tmp/az_chessprobe.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
cp -r "$REF/include" "$TMP/include"
mkdir -p "$TMP/src"
cp "$REF"/src/games/chess/{chess_state,chess_rules,chess960}.cpp "$REF"/src/core/zobrist_hash.cpp "$TMP/src/"
chmod -R u+w "$TMP"
sed -i '2d' "$TMP/src/chess_rules.cpp"
sed -i 's|^#include "alphazero/games/chess/chess_state.h"|&\n#include "alphazero/games/chess/chess_rules.h"|' "$TMP/src/chess_rules.cpp"
sed -i '30s/zobrist_(core::GameType::CHESS, 8, 12)/zobrist_(8, 12, 2, 12345u)/' "$TMP/src/chess_state.cpp"
grep -q 'zobrist_(8, 12, 2, 12345u)' "$TMP/src/chess_state.cpp" || exit 1
g++ -std=c++17 -O0 -DLIBTORCH_OFF -I"$TMP/include" -w "$TMP"/src/*.cpp "$HERE/chess_probe.cpp" -o "$TMP/probe" || exit 1
(ulimit -s 8192; timeout 60 "$TMP/probe")
rc=$?
echo "chess probe exit status: $rc (139 = SIGSEGV: the move-generation recursion overflowed the stack)"
