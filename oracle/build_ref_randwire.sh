#!/usr/bin/env bash
# oracle/build_ref_randwire.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds oracle/_ref/ref_randwire: the REFERENCE's DDW-RandWire translation unit
# (src/nn/ddw_randwire_resnet.cpp + include/) linked with oracle/ref_randwire.cpp against the
# LibTorch shipped inside the image's PyTorch wheel (headers + libtorch_cpu).  The TU is copied
# into a throw-away temp directory outside the repository with ONE patch that touches no
# arithmetic:
#   P9  ddw_randwire_resnet.cpp  drop `#include <spdlog/spdlog.h>` and the single-line
#       spdlog::info/warn/error log statements (spdlog is not in the image; they only log in
#       save / load / export_to_torchscript, which the harness never calls)
#   P10 ddw_randwire_resnet.cpp:301-302  the rewiring loop's duplicate-edge test compares
#       DG.successors(u).end() with std::find over the begin/end of two OTHER temporaries
#       (successors() returns by value): undefined behaviour that in practice is always "true",
#       so the first rewired edge spins forever -- unpatched, RandWireBlock(16, 32, 0.75, 0)
#       never returns (probe: oracle/_ref/ref_randwire_unpatched, `graphs 1` under a timeout).
#       The patch evaluates the test as written, on ONE successors() copy per lookup:
#       has_edge(a, b) = b in DG.successors(a).  No arithmetic changes.
# Nothing from /root/reference is written into the repository; the binary lands in oracle/_ref/.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/src/nn/ddw_randwire_resnet.cpp" ]; then
  echo "build_ref_randwire.sh: $REF not present; skipping" >&2
  exit 0
fi
TP=$(python3 -c 'import os, torch; print(os.path.dirname(torch.__file__))')
mkdir -p "$OUT"
TMP=$(mktemp -d /tmp/az_rwbuild.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
cp -r "$REF/include" "$TMP/include"
cp "$REF/src/nn/ddw_randwire_resnet.cpp" "$TMP/"
chmod -R u+w "$TMP"
cp "$TMP/ddw_randwire_resnet.cpp" "$TMP/ddw_unpatched.cpp"
# P10
grep -q 'while (w == u || w == v || (u < w && DG.successors(u).end() != std::find' "$TMP/ddw_randwire_resnet.cpp"
sed -i '301,302c\            auto has_edge_p10 = [\&DG](int a, int b) { const auto s = DG.successors(a); return std::find(s.begin(), s.end(), b) != s.end(); };\n            while (w == u || w == v || (u < w \&\& has_edge_p10(u, w)) || (w < u \&\& has_edge_p10(w, u))) {' "$TMP/ddw_randwire_resnet.cpp"
grep -q 'has_edge_p10(w, u))) {' "$TMP/ddw_randwire_resnet.cpp"
# P9 (both copies)
for f in "$TMP/ddw_randwire_resnet.cpp" "$TMP/ddw_unpatched.cpp"; do
  sed -i '/#include <spdlog\/spdlog.h>/d; /^[[:space:]]*spdlog::[a-z]*(.*);[[:space:]]*$/d' "$f"
  ! grep -q spdlog "$f"
done
FLAGS="-std=c++17 -O2 -D_GLIBCXX_USE_CXX11_ABI=1 -I$TMP/include -I$TP/include -I$TP/include/torch/csrc/api/include"
g++ $FLAGS -w -c "$TMP/ddw_randwire_resnet.cpp" -o "$TMP/ddw.o" &
g++ $FLAGS -w -c "$TMP/ddw_unpatched.cpp" -o "$TMP/ddw_unpatched.o" &
g++ $FLAGS -w -c "$HERE/ref_randwire.cpp" -o "$TMP/harness.o" &
wait
g++ "$TMP/harness.o" "$TMP/ddw_unpatched.o" -L"$TP/lib" -Wl,-rpath,"$TP/lib" -ltorch -ltorch_cpu -lc10 -pthread -o "$OUT/ref_randwire_unpatched"
g++ "$TMP/harness.o" "$TMP/ddw.o" -L"$TP/lib" -Wl,-rpath,"$TP/lib" -ltorch -ltorch_cpu -lc10 -pthread -o "$OUT/ref_randwire"
echo "built $OUT/ref_randwire"
