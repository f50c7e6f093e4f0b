#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds the minimally patched REFERENCE search into oracle/_ref/ref_harness, the
# golden-vector generator for tests/golden/ (SURVEY.md §8(c), Appendix B).
#
# The reference snapshot does not compile unmodified and its search
# self-deadlocks (F3).  The recipe copies ONLY the hot-path translation units into a
# throw-away temp directory OUTSIDE the repository, applies three patches that do not
# touch any arithmetic, compiles them with g++ (no -march, no FMA contraction: the
# reference's own flags), links oracle/ref_harness.cpp, and deletes the temp copy.
# Nothing from /root/reference is ever written into this repository; only the binary
# lands in oracle/_ref/ (git-ignored).
#
#   P1 parallel_mcts.cpp:1557  lambda capture [this, i, &completed...] += numThreads  (compile error)
#   P2 gomoku_state.cpp:32     zobrist_(GameType,bs,2) -> zobrist_(bs, 2, 2, 12345u)  (ctor no longer
#                              exists; fixed seed => deterministic Zobrist keys)
#   P5 mcts_node.h:64 + parallel_mcts.cpp  std::mutex expansionMutex -> std::recursive_mutex
#                              (removes the F3 self-deadlock; no arithmetic change)
#   P6 go_state.cpp:21         zobrist_(GameType::GO,bs,2) -> zobrist_(bs, 2, 2, 12345u)  (as P2, for GoState)
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF/src/mcts" ]; then
  echo "build_ref.sh: $REF not present; skipping reference oracle build" >&2
  exit 0
fi
mkdir -p "$OUT"
TMP=$(mktemp -d /tmp/az_refbuild.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/src/mcts" "$TMP/src/nn" "$TMP/src/games/gomoku" "$TMP/src/games/go" "$TMP/src/core"
cp -r "$REF/include" "$TMP/include"
cp "$REF"/src/mcts/{parallel_mcts,mcts_node,transposition_table,thread_pool}.cpp "$TMP/src/mcts/"
cp "$REF"/src/nn/{batch_queue,random_policy_network}.cpp "$TMP/src/nn/"
cp "$REF"/src/games/gomoku/{gomoku_state,gomoku_rules}.cpp "$TMP/src/games/gomoku/"
cp "$REF"/src/games/go/{go_state,go_rules}.cpp "$TMP/src/games/go/"
cp "$REF"/src/core/zobrist_hash.cpp "$TMP/src/core/"
chmod -R u+w "$TMP"

# P1
sed -i '1557s/\[this, i, &completedSimulations\]/[this, i, numThreads, \&completedSimulations]/' "$TMP/src/mcts/parallel_mcts.cpp"
grep -q 'this, i, numThreads, &completedSimulations' "$TMP/src/mcts/parallel_mcts.cpp"
# P2
sed -i '32s/zobrist_(core::GameType::GOMOKU, board_size, 2)/zobrist_(board_size, 2, 2, 12345u)/' "$TMP/src/games/gomoku/gomoku_state.cpp"
grep -q 'zobrist_(board_size, 2, 2, 12345u)' "$TMP/src/games/gomoku/gomoku_state.cpp"
# P6
sed -i '21s/zobrist_(core::GameType::GO, board_size, 2)/zobrist_(board_size, 2, 2, 12345u)/' "$TMP/src/games/go/go_state.cpp"
grep -q 'zobrist_(board_size, 2, 2, 12345u)' "$TMP/src/games/go/go_state.cpp"
# P5
sed -i '64s/std::mutex expansionMutex;/std::recursive_mutex expansionMutex;/' "$TMP/include/alphazero/mcts/mcts_node.h"
grep -q 'std::recursive_mutex expansionMutex;' "$TMP/include/alphazero/mcts/mcts_node.h"
sed -i 's/std::lock_guard<std::mutex> lock(\(rootNode_\|node\)->expansionMutex)/std::lock_guard<std::recursive_mutex> lock(\1->expansionMutex)/' "$TMP/src/mcts/parallel_mcts.cpp"
test "$(grep -c 'lock_guard<std::recursive_mutex> lock(.*expansionMutex)' "$TMP/src/mcts/parallel_mcts.cpp")" = 6

CXXFLAGS="-std=c++17 -O2 -pthread -DLIBTORCH_OFF -I$TMP/include"
OBJS=()
for f in "$TMP"/src/mcts/*.cpp "$TMP"/src/nn/*.cpp "$TMP"/src/games/gomoku/*.cpp "$TMP"/src/games/go/*.cpp "$TMP"/src/core/*.cpp; do
  o="$TMP/$(basename "$f" .cpp).o"
  g++ $CXXFLAGS -w -c "$f" -o "$o" &
  OBJS+=("$o")
done
wait
g++ $CXXFLAGS -c "$HERE/ref_harness.cpp" -o "$TMP/ref_harness.o"
g++ -pthread "$TMP/ref_harness.o" "${OBJS[@]}" -o "$OUT/ref_harness"
echo "built $OUT/ref_harness"
