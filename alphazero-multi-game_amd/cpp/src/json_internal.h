// json_internal.h -- the minimal JSON reader shared by the host API's record / dataset parsers
// (GameRecord::fromJson, TrainingExample::fromJson, Dataset::loadFromFile).  Internal.
#pragma once
#include <cctype>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace alphazero {
namespace selfplay {
namespace json_internal {

struct Value {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    double num = 0.0;
    bool b = false;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;
    const Value& at(const std::string& k) const {
        auto it = obj.find(k);
        if (it == obj.end()) throw std::runtime_error("missing key " + k);
        return it->second;
    }
};

struct Parser {
    const std::string& s;
    size_t i = 0;
    void ws() { while (i < s.size() && std::isspace((unsigned char)s[i])) ++i; }
    [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("JSON: ") + m + " at " + std::to_string(i)); }
    Value parse() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        Value v;
        const char c = s[i];
        if (c == '{') {
            v.kind = Value::OBJ; ++i; ws();
            if (s[i] == '}') { ++i; return v; }
            for (;;) {
                ws();
                Value k = parse();
                if (k.kind != Value::STR) fail("key");
                ws();
                if (s[i++] != ':') fail("colon");
                v.obj[k.str] = parse();
                ws();
                if (s[i] == ',') { ++i; continue; }
                if (s[i] == '}') { ++i; return v; }
                fail("object");
            }
        }
        if (c == '[') {
            v.kind = Value::ARR; ++i; ws();
            if (s[i] == ']') { ++i; return v; }
            for (;;) {
                v.arr.push_back(parse());
                ws();
                if (s[i] == ',') { ++i; continue; }
                if (s[i] == ']') { ++i; return v; }
                fail("array");
            }
        }
        if (c == '"') {
            v.kind = Value::STR; ++i;
            while (i < s.size() && s[i] != '"') {
                if (s[i] == '\\' && i + 1 < s.size()) ++i;
                v.str += s[i++];
            }
            ++i;
            return v;
        }
        if (s.compare(i, 4, "null") == 0) { i += 4; return v; }
        if (s.compare(i, 4, "true") == 0) { i += 4; v.kind = Value::BOOL; v.b = true; return v; }
        if (s.compare(i, 5, "false") == 0) { i += 5; v.kind = Value::BOOL; return v; }
        char* end = nullptr;
        v.num = std::strtod(s.c_str() + i, &end);
        if (end == s.c_str() + i) fail("value");
        i = (size_t)(end - s.c_str());
        v.kind = Value::NUM;
        return v;
    }
};

}  // namespace json_internal
}  // namespace selfplay
}  // namespace alphazero
