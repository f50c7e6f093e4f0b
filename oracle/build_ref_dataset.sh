#!/usr/bin/env bash
# oracle/build_ref_dataset.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds the REFERENCE training-example code (src/selfplay/dataset.cpp: extractExamples,
# augmentExample, getBatch, getRandomSubset, shuffle) into oracle/_ref/ref_dataset, the generator
# of tests/golden/ref_dataset.npz.  As build_ref.sh: only the needed translation
# units are copied into a throw-away temp directory OUTSIDE the repository, patched there, compiled
# with g++ and linked with oracle/ref_dataset.cpp (ours); only the binary lands in oracle/_ref/.
#
# dataset.cpp and game_record.cpp include <nlohmann/json.hpp>, which this image lacks.  Their JSON
# functions are the only code that uses it, and none of them is on the path under test, so the
# temp copies drop exactly those functions (no stand-in header is written):
#   P11 dataset.cpp      drop the nlohmann include, `using json`, TrainingExample::toJson/fromJson
#                        (:7, :13, :15-55) and Dataset::saveToFile/loadFromFile (:151-226)
#   P12 game_record.cpp  drop the nlohmann include, `using json`, MoveData::toJson/fromJson
#                        (:8, :13, :15-32) and GameRecord::toJson/fromJson/saveToFile/loadFromFile (:64-end)
#   P3  registry.cpp     add #include <mutex>
#   P2  gomoku_state.cpp fixed Zobrist seed (as build_ref.sh; the hash is not used by the dataset)
# The game factory is the reference's own (core/game_factory.cpp createGameState -> GameRegistry ->
# gomoku_state_plugin.cpp's REGISTER_GAME); Go is not registered there, so the reference's
# extractExamples handles Gomoku only.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/src/selfplay/dataset.cpp" ]; then
  echo "build_ref_dataset.sh: $REF not present; skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
TMP=$(mktemp -d /tmp/az_refds.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/src"
cp -r "$REF/include" "$TMP/include"
cp "$REF"/src/selfplay/{dataset,game_record}.cpp "$REF"/src/core/{game_factory,registry,gomoku_state_plugin,zobrist_hash}.cpp \
   "$REF"/src/games/gomoku/{gomoku_state,gomoku_rules}.cpp "$TMP/src/"
chmod -R u+w "$TMP"
D="$TMP/src/dataset.cpp"
G="$TMP/src/game_record.cpp"
# P11: check the dropped ranges are what we think they are, then delete them (highest first)
sed -n '7p' "$D" | grep -q 'nlohmann/json.hpp'
sed -n '13p' "$D" | grep -q 'using json = nlohmann::json;'
sed -n '15p' "$D" | grep -q 'TrainingExample::toJson'
sed -n '57p' "$D" | grep -q 'Dataset::Dataset()'
sed -n '151p' "$D" | grep -q 'Dataset::saveToFile'
sed -n '228p' "$D" | grep -q 'Dataset::getRandomSubset'
sed -i '151,226d;15,55d;13d;7d' "$D"
! grep -q 'json' "$D"
# P12
sed -n '8p' "$G" | grep -q 'nlohmann/json.hpp'
sed -n '13p' "$G" | grep -q 'using json = nlohmann::json;'
sed -n '15p' "$G" | grep -q 'MoveData::toJson'
sed -n '34p' "$G" | grep -q 'GameRecord::GameRecord'
sed -n '64p' "$G" | grep -q 'GameRecord::toJson'
N=$(awk "END{print NR}" "$G")
sed -i "64,$((N - 3))d;15,32d;13d;8d" "$G"
! grep -q 'json\|Json' "$G"
# P3
sed -i '2a #include <mutex>' "$TMP/src/registry.cpp"
# P2
sed -i '32s/zobrist_(core::GameType::GOMOKU, board_size, 2)/zobrist_(board_size, 2, 2, 12345u)/' "$TMP/src/gomoku_state.cpp"
grep -q 'zobrist_(board_size, 2, 2, 12345u)' "$TMP/src/gomoku_state.cpp"

CXXFLAGS="-std=c++17 -O2 -pthread -DLIBTORCH_OFF -I$TMP/include -I$TMP/include/alphazero/games/gomoku -I$TMP/include/alphazero/core"
OBJS=()
for f in "$TMP"/src/*.cpp; do
  o="$TMP/$(basename "$f" .cpp).o"
  g++ $CXXFLAGS -w -c "$f" -o "$o" &
  OBJS+=("$o")
done
wait
g++ $CXXFLAGS -c "$HERE/ref_dataset.cpp" -o "$TMP/ref_dataset.o"
g++ -pthread "$TMP/ref_dataset.o" "${OBJS[@]}" -o "$OUT/ref_dataset"
echo "built $OUT/ref_dataset"
