// oracle/ref_dataset.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Drives the REFERENCE alphazero::selfplay::Dataset (src/selfplay/dataset.cpp, built by
// oracle/build_ref_dataset.sh with only its nlohmann-json functions removed) on game records given
// on stdin, and writes what it produced to the binary file argv[1]:
//   extractExamples(augment) -- dataset.cpp:64-114 (augmentExample :245-434, shuffle :147-149)
//   then, with `ops`, getBatch(37) (:120-145), getRandomSubset(5) (:228-243) and shuffle().
// The Dataset's rng_ is seeded by std::random_device (:57); to make the output reproducible the
// harness seeds it explicitly (private member access in THIS translation unit only: the reference
// source is not modified for it).
//
// stdin (text): seed augment ops n_games, then per game: board result n_moves, then per move:
//   action policy_len policy_bits... (IEEE-754 bit patterns as unsigned integers: NaN entries exact).
// argv[1] (binary, little endian): a store record for examples_ after extractExamples
//   int64 E; int32 C, H, W, PMAX; float32 state[E][C][H][W]; int32 plen[E]; float32 policy[E][PMAX];
//   float32 value[E]
// and with ops: the same record for getBatch(37) (values as one list), getRandomSubset(5), and
// examples_ after shuffle().
#include <algorithm>
#include <any>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <optional>
#include <random>
#include <shared_mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <variant>
#include <vector>

#define private public
#include "alphazero/selfplay/dataset.h"
#undef private
#include "alphazero/selfplay/game_record.h"

using namespace alphazero;
using Ex = selfplay::TrainingExample;

static void put(std::ofstream& f, const void* p, size_t n) { f.write(reinterpret_cast<const char*>(p), (std::streamsize)n); }

static void dump(std::ofstream& f, const std::vector<std::vector<std::vector<std::vector<float>>>>& states,
                 const std::vector<std::vector<float>>& pols, const std::vector<float>& vals) {
    const int64_t E = (int64_t)states.size();
    int32_t C = 0, H = 0, W = 0, PMAX = 0;
    if (E) { C = (int32_t)states[0].size(); H = (int32_t)states[0][0].size(); W = (int32_t)states[0][0][0].size(); }
    for (const auto& p : pols) PMAX = std::max(PMAX, (int32_t)p.size());
    put(f, &E, 8);
    int32_t hdr[4] = {C, H, W, PMAX};
    put(f, hdr, 16);
    for (const auto& s : states) {
        if ((int32_t)s.size() != C) throw std::runtime_error("ragged planes");
        for (const auto& pl : s)
            for (const auto& row : pl) put(f, row.data(), row.size() * 4);
    }
    for (const auto& p : pols) { int32_t n = (int32_t)p.size(); put(f, &n, 4); }
    for (const auto& p : pols) {
        std::vector<float> row(PMAX, 0.0f);
        std::copy(p.begin(), p.end(), row.begin());
        put(f, row.data(), row.size() * 4);
    }
    put(f, vals.data(), vals.size() * 4);
}

static void dump_examples(std::ofstream& f, const std::vector<Ex>& ex) {
    std::vector<std::vector<std::vector<std::vector<float>>>> st;
    std::vector<std::vector<float>> po;
    std::vector<float> va;
    for (const Ex& e : ex) { st.push_back(e.state); po.push_back(e.policy); va.push_back(e.value); }
    dump(f, st, po, va);
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_dataset OUT < records\n"); return 2; }
    unsigned seed;
    int augment, ops, n_games;
    if (!(std::cin >> seed >> augment >> ops >> n_games)) return 2;
    selfplay::Dataset ds;
    ds.rng_.seed(seed);
    for (int g = 0; g < n_games; ++g) {
        int bs, result, n;
        std::cin >> bs >> result >> n;
        selfplay::GameRecord rec(core::GameType::GOMOKU, bs, false);
        for (int m = 0; m < n; ++m) {
            int action, plen;
            std::cin >> action >> plen;
            std::vector<float> p(plen);
            for (int k = 0; k < plen; ++k) {
                uint32_t b;
                std::cin >> b;
                std::memcpy(&p[k], &b, 4);
            }
            rec.addMove(action, p, 0.0f, 0);
        }
        rec.setResult(static_cast<core::GameResult>(result));
        ds.addGameRecord(rec);
    }
    if (!std::cin) { std::fprintf(stderr, "bad input\n"); return 2; }
    ds.extractExamples(augment != 0);
    std::ofstream f(argv[1], std::ios::binary);
    dump_examples(f, ds.examples_);
    if (ops) {
        auto [bst, bpo, bva] = ds.getBatch(37);
        dump(f, bst, bpo, bva);
        dump_examples(f, ds.getRandomSubset(5));
        ds.shuffle();
        dump_examples(f, ds.examples_);
    }
    std::printf("examples %zu\n", ds.size());
    return 0;
}
