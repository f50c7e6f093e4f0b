// torchscript_reader.cpp -- see alphazero/nn/torchscript_reader.h.
#include "alphazero/nn/torchscript_reader.h"

#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>

#include "alphazero/nn/hip_neural_network.h"

namespace alphazero {
namespace nn {
namespace {

[[noreturn]] void fail(const std::string& m) { throw std::invalid_argument("TorchScript archive: " + m); }

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t* p) { return (uint32_t)rd16(p) | ((uint32_t)rd16(p + 2) << 16); }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

// ---------------------------------------------------------------- zip directory (stored entries)
struct Zip {
    std::vector<uint8_t> buf;
    std::map<std::string, std::pair<size_t, size_t>> entries;   // name -> (data offset, size), stored only

    explicit Zip(const std::string& path) {
        std::ifstream f(path, std::ios::binary);
        if (!f) fail("cannot open " + path);
        buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
        const size_t n = buf.size();
        if (n < 22) fail("not a zip file");
        size_t eocd = std::string::npos;
        for (size_t i = n - 22 + 1; i-- > (n > 65557 ? n - 65557 : 0);)
            if (rd32(&buf[i]) == 0x06054b50u) { eocd = i; break; }
        if (eocd == std::string::npos) fail("no zip end-of-directory record");
        uint64_t count = rd16(&buf[eocd + 10]), cd = rd32(&buf[eocd + 16]);
        if (count == 0xffff || cd == 0xffffffffu) {            // zip64 end of central directory
            if (eocd < 20 || rd32(&buf[eocd - 20]) != 0x07064b50u) fail("zip64 locator missing");
            const uint64_t z = rd64(&buf[eocd - 20 + 8]);
            if (z > n || n - z < 56 || rd32(&buf[z]) != 0x06064b50u) fail("zip64 record missing");
            count = rd64(&buf[z + 32]);
            cd = rd64(&buf[z + 48]);
        }
        if (cd > n) fail("central directory outside the file");
        size_t p = cd;
        for (uint64_t e = 0; e < count; ++e) {
            if (n - p < 46 || rd32(&buf[p]) != 0x02014b50u) fail("bad central directory");
            const uint16_t method = rd16(&buf[p + 10]);
            uint64_t csize = rd32(&buf[p + 20]), usize = rd32(&buf[p + 24]);
            const uint16_t nl = rd16(&buf[p + 28]), xl = rd16(&buf[p + 30]), cl = rd16(&buf[p + 32]);
            uint64_t loc = rd32(&buf[p + 42]);
            if (n - p - 46 < (size_t)nl + xl + cl) fail("central directory entry past the end of the file");
            const std::string name(reinterpret_cast<const char*>(&buf[p + 46]), nl);
            // zip64 extra: the fields that overflowed, in the order usize, csize, offset
            const size_t xend = p + 46 + nl + xl;
            for (size_t x = p + 46 + nl; x + 4 <= xend;) {
                const uint16_t id = rd16(&buf[x]), len = rd16(&buf[x + 2]);
                if (xend - x - 4 < len) fail("zip extra field past its record");
                if (id == 0x0001) {
                    size_t q = x + 4;
                    const size_t qend = x + 4 + len;
                    auto take = [&](uint64_t& f) {
                        if (qend - q < 8) fail("short zip64 extra field");
                        f = rd64(&buf[q]);
                        q += 8;
                    };
                    if (usize == 0xffffffffu) take(usize);
                    if (csize == 0xffffffffu) take(csize);
                    if (loc == 0xffffffffu) take(loc);
                }
                x += 4 + len;
            }
            if (loc > n || n - loc < 30 || rd32(&buf[loc]) != 0x04034b50u) fail("bad local header of " + name);
            const uint64_t hdr = 30 + (uint64_t)rd16(&buf[loc + 26]) + rd16(&buf[loc + 28]);
            if (n - loc < hdr) fail("truncated local header of " + name);
            const size_t data = loc + hdr;
            if (method == 0) {
                if (usize > n - data) fail("truncated entry " + name);
                entries[name] = {data, (size_t)usize};
            }
            p += 46 + nl + xl + cl;
        }
    }
    const std::pair<size_t, size_t>& get(const std::string& name) const {
        auto it = entries.find(name);
        if (it == entries.end()) fail("missing (or compressed) entry " + name);
        return it->second;
    }
};

// ---------------------------------------------------------------- restricted pickle machine
struct Val;
using VP = std::shared_ptr<Val>;
struct Val {
    enum Kind { NONE, BOOL, INT, FLOAT, STR, TUPLE, LIST, DICT, GLOBAL, OBJECT, STORAGE, TENSOR, MARK } k = NONE;
    int64_t i = 0;
    double f = 0;
    std::string s;                                  // STR, GLOBAL ("module name"), OBJECT class
    std::vector<VP> items;                          // TUPLE, LIST
    std::vector<std::pair<VP, VP>> dict;            // DICT, OBJECT state
    // STORAGE: s = dtype name, i = numel, key; TENSOR: storage, offset, size, stride
    std::string key;
    VP storage;
    int64_t offset = 0;
    std::vector<int64_t> size, stride;
};
VP mk(Val::Kind k) { auto v = std::make_shared<Val>(); v->k = k; return v; }

VP unpickle(const uint8_t* p, size_t n) {
    std::vector<VP> st;
    std::vector<size_t> marks;
    std::map<uint64_t, VP> memo;
    size_t i = 0;
    auto need = [&](size_t k) { if (i + k > n) fail("truncated data.pkl"); };
    auto pop = [&]() {
        if (st.empty()) fail("pickle stack underflow");
        VP v = st.back();
        st.pop_back();
        if (!v) fail("null pickle value");
        return v;
    };
    auto pop_mark = [&]() {
        if (marks.empty()) fail("pickle mark underflow");
        const size_t m = marks.back();
        marks.pop_back();
        std::vector<VP> out(st.begin() + m, st.end());
        st.resize(m);
        return out;
    };
    auto str = [&](size_t len) { need(len); std::string s(reinterpret_cast<const char*>(p + i), len); i += len; return s; };
    auto line = [&]() {
        size_t j = i;
        while (j < n && p[j] != '\n') ++j;
        if (j >= n) fail("unterminated GLOBAL");
        std::string s(reinterpret_cast<const char*>(p + i), j - i);
        i = j + 1;
        return s;
    };
    auto setitems = [&](VP d, const std::vector<VP>& kv) {
        if (d->k != Val::DICT) fail("SETITEMS on a non-dict");
        if (kv.size() % 2) fail("odd SETITEMS");
        for (size_t q = 0; q < kv.size(); q += 2) d->dict.push_back({kv[q], kv[q + 1]});
    };
    auto tuple = [&](std::vector<VP> v) { VP t = mk(Val::TUPLE); t->items = std::move(v); return t; };
    auto as_ints = [&](const VP& t) {
        if (t->k != Val::TUPLE) fail("expected a tuple of ints");
        std::vector<int64_t> out;
        for (auto& x : t->items) {
            if (x->k != Val::INT) fail("expected a tuple of ints");
            out.push_back(x->i);
        }
        return out;
    };
    for (;;) {
        need(1);
        const uint8_t op = p[i++];
        switch (op) {
            case 0x80: need(1); i += 1; break;                                  // PROTO
            case '(': marks.push_back(st.size()); break;                        // MARK
            case '.': if (st.size() != 1) fail("bad stack at STOP"); return st.back();
            case 'N': st.push_back(mk(Val::NONE)); break;
            case 0x88: case 0x89: { VP b = mk(Val::BOOL); b->i = op == 0x88; st.push_back(b); break; }
            case 'K': { need(1); VP v = mk(Val::INT); v->i = p[i]; i += 1; st.push_back(v); break; }
            case 'M': { need(2); VP v = mk(Val::INT); v->i = rd16(p + i); i += 2; st.push_back(v); break; }
            case 'J': { need(4); VP v = mk(Val::INT); v->i = (int32_t)rd32(p + i); i += 4; st.push_back(v); break; }
            case 0x8a: {                                                        // LONG1
                need(1);
                const size_t len = p[i++];
                need(len);
                if (len > 8) fail("LONG1 wider than 64 bits");
                int64_t v = 0;
                for (size_t b = 0; b < len; ++b) v |= (int64_t)p[i + b] << (8 * b);
                if (len && len < 8 && (p[i + len - 1] & 0x80)) v -= (int64_t)1 << (8 * len);
                i += len;
                VP x = mk(Val::INT); x->i = v; st.push_back(x);
                break;
            }
            case 'G': {                                                         // BINFLOAT (big-endian)
                need(8);
                uint64_t u = 0;
                for (int b = 0; b < 8; ++b) u = (u << 8) | p[i + b];
                i += 8;
                VP x = mk(Val::FLOAT); std::memcpy(&x->f, &u, 8); st.push_back(x);
                break;
            }
            case 'X': { need(4); const uint32_t len = rd32(p + i); i += 4; VP x = mk(Val::STR); x->s = str(len); st.push_back(x); break; }
            case 0x8c: { need(1); const size_t len = p[i++]; VP x = mk(Val::STR); x->s = str(len); st.push_back(x); break; }
            case 'U': { need(1); const size_t len = p[i++]; VP x = mk(Val::STR); x->s = str(len); st.push_back(x); break; }
            case 'T': { need(4); const uint32_t len = rd32(p + i); i += 4; VP x = mk(Val::STR); x->s = str(len); st.push_back(x); break; }
            case ')': st.push_back(tuple({})); break;
            case 't': st.push_back(tuple(pop_mark())); break;
            case 0x85: { VP a = pop(); st.push_back(tuple({a})); break; }
            case 0x86: { VP b = pop(), a = pop(); st.push_back(tuple({a, b})); break; }
            case 0x87: { VP c = pop(), b = pop(), a = pop(); st.push_back(tuple({a, b, c})); break; }
            case ']': st.push_back(mk(Val::LIST)); break;
            case 'l': { VP l = mk(Val::LIST); l->items = pop_mark(); st.push_back(l); break; }
            case 'a': { VP v = pop(); if (st.empty() || st.back()->k != Val::LIST) fail("APPEND"); st.back()->items.push_back(v); break; }
            case 'e': {
                std::vector<VP> v = pop_mark();
                if (st.empty() || st.back()->k != Val::LIST) fail("APPENDS");
                for (auto& x : v) st.back()->items.push_back(x);
                break;
            }
            case '}': st.push_back(mk(Val::DICT)); break;
            case 'd': { VP d = mk(Val::DICT); setitems(d, pop_mark()); st.push_back(d); break; }
            case 's': { VP v = pop(), k = pop(); if (st.empty()) fail("SETITEM"); setitems(st.back(), {k, v}); break; }
            case 'u': { std::vector<VP> kv = pop_mark(); if (st.empty()) fail("SETITEMS"); setitems(st.back(), kv); break; }
            case 'q': { need(1); if (st.empty()) fail("BINPUT on an empty stack"); memo[p[i]] = st.back(); i += 1; break; }
            case 'r': { need(4); if (st.empty()) fail("LONG_BINPUT on an empty stack"); memo[rd32(p + i)] = st.back(); i += 4; break; }
            case 'h': { need(1); auto it = memo.find(p[i]); if (it == memo.end()) fail("BINGET of an unset memo"); st.push_back(it->second); i += 1; break; }
            case 'j': { need(4); auto it = memo.find(rd32(p + i)); if (it == memo.end()) fail("LONG_BINGET of an unset memo"); st.push_back(it->second); i += 4; break; }
            case 'c': {                                                         // GLOBAL: the allow-list
                const std::string mod = line(), name = line();
                const bool ok = mod.rfind("__torch__", 0) == 0 ||
                                (mod == "torch._utils" && (name == "_rebuild_tensor_v2" || name == "_rebuild_parameter")) ||
                                (mod == "torch" && name.size() > 7 && name.compare(name.size() - 7, 7, "Storage") == 0) ||
                                (mod == "collections" && name == "OrderedDict");
                if (!ok) fail("refusing global " + mod + "." + name);
                VP g = mk(Val::GLOBAL); g->s = mod + " " + name; st.push_back(g);
                break;
            }
            case 0x81: {                                                        // NEWOBJ: a module object
                VP args = pop(), cls = pop();
                if (cls->k != Val::GLOBAL || cls->s.rfind("__torch__", 0) != 0) fail("NEWOBJ of a non-module class");
                VP o = mk(Val::OBJECT); o->s = cls->s; st.push_back(o);
                break;
            }
            case 'b': {                                                         // BUILD: the object's attributes
                VP state = pop();
                if (st.empty() || st.back()->k != Val::OBJECT || state->k != Val::DICT) fail("BUILD");
                st.back()->dict = state->dict;
                break;
            }
            case 'Q': {                                                         // BINPERSID: a storage record
                VP pid = pop();
                if (pid->k != Val::TUPLE || pid->items.size() < 5 || pid->items[0]->k != Val::STR ||
                    pid->items[0]->s != "storage" || pid->items[1]->k != Val::GLOBAL || pid->items[2]->k != Val::STR ||
                    pid->items[4]->k != Val::INT)
                    fail("unknown persistent id");
                VP s = mk(Val::STORAGE);
                s->s = pid->items[1]->s.substr(pid->items[1]->s.find(' ') + 1);
                s->key = pid->items[2]->s;
                s->i = pid->items[4]->i;
                st.push_back(s);
                break;
            }
            case 'R': {                                                         // REDUCE on an allowed callable
                VP args = pop(), fn = pop();
                if (fn->k != Val::GLOBAL || args->k != Val::TUPLE) fail("REDUCE");
                if (fn->s == "collections OrderedDict") { st.push_back(mk(Val::DICT)); break; }
                if (fn->s == "torch._utils _rebuild_parameter") {
                    if (args->items.empty() || args->items[0]->k != Val::TENSOR) fail("_rebuild_parameter");
                    st.push_back(args->items[0]);
                    break;
                }
                if (fn->s == "torch._utils _rebuild_tensor_v2") {
                    if (args->items.size() < 4 || args->items[0]->k != Val::STORAGE || args->items[1]->k != Val::INT)
                        fail("_rebuild_tensor_v2 arguments");
                    VP t = mk(Val::TENSOR);
                    t->storage = args->items[0];
                    t->offset = args->items[1]->i;
                    t->size = as_ints(args->items[2]);
                    t->stride = as_ints(args->items[3]);
                    st.push_back(t);
                    break;
                }
                fail("refusing to call " + fn->s);
            }
            default: {
                char b[64];
                std::snprintf(b, sizeof b, "unsupported pickle opcode 0x%02x at %zu", op, i - 1);
                fail(b);
            }
        }
    }
}

float half_to_f(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023;
    float f;
    if (e == 0) f = std::ldexp((float)m, -24);
    else if (e == 31) f = m ? NAN : INFINITY;
    else f = std::ldexp((float)(m | 1024), (int)e - 25);
    return s ? -f : f;
}

}  // namespace

bool isZipArchive(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    uint8_t m[4] = {0, 0, 0, 0};
    f.read(reinterpret_cast<char*>(m), 4);
    return f.gcount() == 4 && rd32(m) == 0x04034b50u;
}

std::vector<NamedTensor> readTorchScript(const std::string& path) {
    Zip z(path);
    std::string prefix;
    for (auto& e : z.entries) {
        const std::string& nm = e.first;
        if (nm.size() >= 8 && nm.compare(nm.size() - 8, 8, "data.pkl") == 0 &&
            (nm.size() == 8 || nm[nm.size() - 9] == '/') && nm.find('/') == nm.size() - 9) {
            prefix = nm.substr(0, nm.size() - 8);
            break;
        }
    }
    if (prefix.empty() && !z.entries.count("data.pkl")) fail("no data.pkl (not a torch archive)");
    const auto& d = z.get(prefix + "data.pkl");
    VP root = unpickle(z.buf.data() + d.first, d.second);
    std::vector<NamedTensor> out;
    // module nesting is shallow in any real archive; a BUILD state that reaches its own object
    // through the memo would otherwise recurse without bound
    constexpr int MAX_DEPTH = 64;
    std::function<void(const VP&, const std::string&, int)> walk = [&](const VP& v, const std::string& pre, int depth) {
        if (depth > MAX_DEPTH) fail("module nesting deeper than 64 (cyclic BUILD state?)");
        for (auto& kv : v->dict) {
            if (!kv.first || !kv.second) fail("null dictionary entry");
            if (kv.first->k != Val::STR) continue;
            const std::string name = pre + kv.first->s;
            const VP& x = kv.second;
            if (x->k == Val::OBJECT) {
                walk(x, name + ".", depth + 1);
            } else if (x->k == Val::TENSOR) {
                NamedTensor t;
                t.name = name;
                t.shape = x->size;
                if (!x->storage || x->size.size() != x->stride.size()) fail("tensor " + name + ": size / stride mismatch");
                for (size_t a = 0; a < x->size.size(); ++a)
                    if (x->size[a] < 0 || x->stride[a] < -((int64_t)1 << 40) || x->stride[a] > ((int64_t)1 << 40))
                        fail("tensor " + name + ": size / stride out of range");
                if (x->offset < 0 || x->offset > ((int64_t)1 << 40)) fail("tensor " + name + ": storage offset out of range");
                const std::string& ty = x->storage->s;
                const size_t es = ty == "DoubleStorage" || ty == "LongStorage" ? 8 : ty == "FloatStorage" || ty == "IntStorage" ? 4
                                  : ty == "HalfStorage" || ty == "BFloat16Storage" ? 2 : 0;
                if (!es) fail("unsupported storage type " + ty + " of " + name);
                const auto& e = z.get(prefix + "data/" + x->storage->key);
                const uint8_t* base = z.buf.data() + e.first;
                int64_t numel = 1;
                for (int64_t s : x->size) {
                    if (s && numel > ((int64_t)1 << 40) / s) fail("tensor " + name + " too large");
                    numel *= s;
                }
                t.data.resize((size_t)numel);
                const size_t nd = x->size.size();
                for (int64_t lin = 0; lin < numel; ++lin) {
                    int64_t rem = lin, off = x->offset;
                    for (size_t a = nd; a-- > 0;) {
                        off += (rem % x->size[a]) * x->stride[a];
                        rem /= x->size[a];
                    }
                    if ((uint64_t)(off + 1) * es > e.second || off < 0) fail("tensor " + name + " exceeds its storage");
                    const uint8_t* q = base + (size_t)off * es;
                    float f;
                    if (ty == "FloatStorage") std::memcpy(&f, q, 4);
                    else if (ty == "DoubleStorage") { double g; std::memcpy(&g, q, 8); f = (float)g; }
                    else if (ty == "HalfStorage") f = half_to_f(rd16(q));
                    else if (ty == "BFloat16Storage") { const uint32_t u = (uint32_t)rd16(q) << 16; std::memcpy(&f, &u, 4); }
                    else if (ty == "LongStorage") f = (float)(int64_t)rd64(q);
                    else f = (float)(int32_t)rd32(q);
                    t.data[(size_t)lin] = f;
                }
                out.push_back(std::move(t));
            }
        }
    };
    if (root && (root->k == Val::OBJECT || root->k == Val::DICT)) walk(root, "", 0);
    else fail("data.pkl does not hold a module or a state dict");
    return out;
}

std::vector<float> torchScriptResNet(const std::string& path, core::GameType type, int boardSize, NetShape& shape) {
    std::vector<NamedTensor> ts = readTorchScript(path);
    std::vector<const NamedTensor*> t;
    for (const auto& x : ts)
        if (x.name.size() < 19 || x.name.compare(x.name.size() - 19, 19, "num_batches_tracked") != 0) t.push_back(&x);
    auto has = [&](const std::string& s) {
        for (auto* x : t) if (x->name.find(s) != std::string::npos) return true;
        return false;
    };
    int residual;
    if (has("res_blocks.")) residual = 1;                 // python/simple_export.py SimplifiedModel
    else if (has("middle_layers.")) residual = 0;         // python/scripts/simple_export.py exporter fallback
    else fail("unrecognised module layout (expected res_blocks.* or middle_layers.*: the reference's plain ResNet)");
    std::vector<const NamedTensor*> conv3, conv1, lin;
    for (auto* x : t) {
        if (x->shape.size() == 4 && x->shape[2] == 3 && x->shape[3] == 3) conv3.push_back(x);
        else if (x->shape.size() == 4 && x->shape[2] == 1 && x->shape[3] == 1) conv1.push_back(x);
        else if (x->shape.size() == 2) lin.push_back(x);
    }
    if (conv3.empty() || conv3.size() % 2 == 0 || conv1.size() != 2 || lin.size() != 3) fail("not a plain ResNet of the reference's shape");
    NetShape s;
    s.channels = (int)conv3[0]->shape[0];
    s.inPlanes = (int)conv3[0]->shape[1];
    s.blocks = (int)(conv3.size() - 1) / 2;
    s.headChannels = (int)conv1[0]->shape[0];
    s.actionSize = (int)lin[0]->shape[0];
    s.fcHidden = (int)lin[1]->shape[0];
    const int pp = (int)lin[0]->shape[1] / std::max(1, s.headChannels);
    s.pool = (int)std::lround(std::sqrt((double)pp));
    s.residual = residual;
    s.convBias = has(conv3[0]->name.substr(0, conv3[0]->name.size() - 6) + "bias") ? 1 : 0;
    if (boardSize <= 0) {
        const int A = s.actionSize - (type == core::GameType::GO ? 1 : 0);
        boardSize = (int)std::lround(std::sqrt((double)A));
        if (boardSize * boardSize != A) fail("cannot infer the board size from the policy size");
    }
    s.boardSize = boardSize;
    if (s.pool * s.pool != pp || lin[2]->shape[0] != 1 || lin[1]->shape[1] != lin[0]->shape[1])
        fail("head shapes do not match the reference's ResNet heads");
    s.precision = shape.precision;
    s.maxBatch = shape.maxBatch;
    std::vector<float> blob;
    for (auto* x : t) blob.insert(blob.end(), x->data.begin(), x->data.end());
    shape = s;
    return blob;
}

}  // namespace nn
}  // namespace alphazero
