// GameRecord / MoveData JSON (row f1): the text nlohmann::json::dump produces for the
// reference's objects (src/selfplay/game_record.cpp:17-145), written and parsed without a
// JSON library.
#include "alphazero/selfplay/game_record.h"

#include "json_internal.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <ctime>
#include <fstream>
#include <iomanip>
#include <map>
#include <memory>
#include <sstream>

namespace alphazero {
namespace selfplay {

using json_internal::Parser;
using json_internal::Value;

std::string jsonNumber(double v) {
    if (!std::isfinite(v)) return "null";
    if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);   // shortest digits
    std::string sci(buf, r.ptr);
    std::string out;
    if (sci[0] == '-') { out = "-"; sci.erase(0, 1); }
    const size_t epos = sci.find('e');
    std::string digits = sci.substr(0, epos);
    const int e10 = std::atoi(sci.c_str() + epos + 1);
    digits.erase(std::remove(digits.begin(), digits.end(), '.'), digits.end());
    const int k = (int)digits.size();
    const int n = e10 + 1;           // value = 0.d1d2..dk * 10^n
    if (k <= n && n <= 15) {         // integral: digits, zeros, ".0"
        out += digits + std::string(n - k, '0') + ".0";
    } else if (0 < n && n <= 15) {   // dd.ddd
        out += digits.substr(0, n) + "." + digits.substr(n);
    } else if (-4 < n && n <= 0) {   // 0.000ddd
        out += "0." + std::string(-n, '0') + digits;
    } else {                         // d.ddde+XX
        out += digits.substr(0, 1);
        if (k > 1) out += "." + digits.substr(1);
        const int ex = n - 1;
        char eb[16];
        std::snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
        out += eb;
    }
    return out;
}

// ---------------------------------------------------------------- writer
namespace {

struct W {
    std::ostringstream o;
    int indent;   // -1: compact
    void nl(int level) {
        if (indent < 0) return;
        o << '\n' << std::string((size_t)indent * level, ' ');
    }
    const char* sep() const { return indent < 0 ? ":" : ": "; }
};

void writeFloats(W& w, const std::vector<float>& v, int level) {
    if (v.empty()) { w.o << "[]"; return; }
    w.o << '[';
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) w.o << ',';
        w.nl(level + 1);
        w.o << jsonNumber((double)v[i]);
    }
    w.nl(level);
    w.o << ']';
}

void writeMove(W& w, const MoveData& m, int level) {
    w.o << '{';
    w.nl(level + 1); w.o << "\"action\"" << w.sep() << m.action << ',';
    w.nl(level + 1); w.o << "\"policy\"" << w.sep(); writeFloats(w, m.policy, level + 1); w.o << ',';
    w.nl(level + 1); w.o << "\"thinking_time_ms\"" << w.sep() << m.thinking_time_ms << ',';
    w.nl(level + 1); w.o << "\"value\"" << w.sep() << jsonNumber((double)m.value);
    w.nl(level);
    w.o << '}';
}

float toFloat(const Value& v) { return v.kind == Value::NUM ? (float)v.num : NAN; }   // null (NaN) -> NaN

MoveData moveFrom(const Value& m) {
    MoveData d;
    d.action = (int)m.at("action").num;
    for (const Value& p : m.at("policy").arr) d.policy.push_back(toFloat(p));
    d.value = toFloat(m.at("value"));
    d.thinking_time_ms = (int64_t)m.at("thinking_time_ms").num;
    return d;
}

}  // namespace

std::string MoveData::toJson() const {
    W w{{}, -1};
    writeMove(w, *this, 0);
    return w.o.str();
}

MoveData MoveData::fromJson(const std::string& json) {
    Parser p{json};
    return moveFrom(p.parse());
}

GameRecord::GameRecord(core::GameType gameType, int boardSize, bool useVariantRules)
    : gameType_(gameType), boardSize_(boardSize), useVariantRules_(useVariantRules),
      timestamp_(std::chrono::system_clock::now()) {}

void GameRecord::addMove(int action, const std::vector<float>& policy, float value, int64_t ms) {
    moves_.push_back(MoveData{action, policy, value, ms});
}

std::string GameRecord::toJson() const {
    W w{{}, 4};
    const std::time_t t = std::chrono::system_clock::to_time_t(timestamp_);
    std::tm tm{};
    gmtime_r(&t, &tm);
    char ts[32];
    std::strftime(ts, sizeof ts, "%FT%TZ", &tm);
    w.o << '{';
    w.nl(1); w.o << "\"board_size\": " << boardSize_ << ',';
    w.nl(1); w.o << "\"game_type\": " << (int)gameType_ << ',';
    w.nl(1); w.o << "\"moves\": ";
    if (moves_.empty()) {
        w.o << "[]";
    } else {
        w.o << '[';
        for (size_t i = 0; i < moves_.size(); ++i) {
            if (i) w.o << ',';
            w.nl(2);
            writeMove(w, moves_[i], 2);
        }
        w.nl(1);
        w.o << ']';
    }
    w.o << ',';
    w.nl(1); w.o << "\"result\": " << (int)result_ << ',';
    w.nl(1); w.o << "\"timestamp\": \"" << ts << "\",";
    w.nl(1); w.o << "\"use_variant_rules\": " << (useVariantRules_ ? "true" : "false");
    w.nl(0);
    w.o << '}';
    return w.o.str();
}

GameRecord GameRecord::fromJson(const std::string& json) {
    try {
        Parser p{json};
        const Value v = p.parse();
        GameRecord r((core::GameType)(int)v.at("game_type").num, (int)v.at("board_size").num,
                     v.at("use_variant_rules").b);
        r.result_ = (core::GameResult)(int)v.at("result").num;
        for (const Value& m : v.at("moves").arr) r.moves_.push_back(moveFrom(m));
        const std::string ts = v.obj.count("timestamp") ? v.at("timestamp").str : "";
        std::tm tm{};
        if (!ts.empty() && strptime(ts.c_str(), "%Y-%m-%dT%H:%M:%SZ", &tm))
            r.timestamp_ = std::chrono::system_clock::from_time_t(timegm(&tm));
        return r;
    } catch (const std::exception& e) {
        throw std::runtime_error(std::string("Failed to parse JSON: ") + e.what());
    }
}

bool GameRecord::saveToFile(const std::string& filename) const {
    std::ofstream f(filename);
    if (!f) return false;
    f << toJson();
    return (bool)f;
}

GameRecord GameRecord::loadFromFile(const std::string& filename) {
    std::ifstream f(filename);
    if (!f) throw std::runtime_error("Failed to load game record: Could not open file: " + filename);
    std::stringstream b;
    b << f.rdbuf();
    return fromJson(b.str());
}

}  // namespace selfplay
}  // namespace alphazero
