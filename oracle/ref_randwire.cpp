// oracle/ref_randwire.cpp -- TEST INFRASTRUCTURE ONLY (golden-vector generator for row f4).
//
// Links the REFERENCE's own DDW-RandWire translation unit (src/nn/ddw_randwire_resnet.cpp,
// compiled by oracle/build_ref_randwire.sh against the LibTorch that ships with the image's
// PyTorch) and dumps what the device rebuild must reproduce:
//
//   ref_randwire graphs NB
//       per rand-wire block i < NB (RandWireBlock(C, 32, 0.75, seed = i), ddw_randwire_resnet.cpp:399):
//       nodes() order, input / output nodes, predecessors per node (router concat order),
//       topological order, the edge list in DiGraph::edges() order -- one JSON object per line
//   ref_randwire forward IN A C NB H B blob.f32 planes.f32 out.f32
//       DDWRandWireResNet(IN, A, C, NB) (ddw_randwire_resnet.cpp:387-427) in eval() mode, every
//       parameter / buffer overwritten from blob.f32 in torch state_dict order (modules in
//       pre-order, each module's parameters then buffers; num_batches_tracked skipped), forward
//       (:429-468) of planes [B][IN][H][W]; writes logits [B][A] then value [B] (fp32).  The
//       state entry names and shapes go to stdout as JSON lines.
//
// The RandWireBlock graph members are private in the reference header; the harness reads them
// through the usual `#define private public` test idiom (no arithmetic involved).
#include <torch/torch.h>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <memory>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>
#define private public
#include "alphazero/nn/ddw_randwire_resnet.h"
#undef private

using alphazero::nn::DDWRandWireResNet;
using alphazero::nn::RandWireBlock;

static void json_list(std::ostream& o, const std::vector<int>& v) {
    o << "[";
    for (size_t i = 0; i < v.size(); ++i) o << (i ? "," : "") << v[i];
    o << "]";
}

static std::vector<float> read_f32(const char* path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(2); }
    const size_t n = (size_t)f.tellg() / 4;
    std::vector<float> v(n);
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * 4));
    return v;
}

static int graphs(int nb) {
    for (int i = 0; i < nb; ++i) {
        RandWireBlock blk(16, 32, 0.75, i);
        const auto& g = blk.graph_;
        std::cout << "{\"block\":" << i << ",\"nodes\":";
        json_list(std::cout, g.nodes());
        std::cout << ",\"input_nodes\":";
        json_list(std::cout, blk.input_nodes_);
        std::cout << ",\"output_nodes\":";
        json_list(std::cout, blk.output_nodes_);
        std::cout << ",\"topo\":";
        json_list(std::cout, g.topological_sort());
        std::cout << ",\"preds\":{";
        bool first = true;
        for (int v : g.nodes()) {
            std::cout << (first ? "" : ",") << "\"" << v << "\":";
            json_list(std::cout, g.predecessors(v));
            first = false;
        }
        std::cout << "},\"edges\":[";
        const auto e = g.edges();
        for (size_t k = 0; k < e.size(); ++k) std::cout << (k ? "," : "") << "[" << e[k].from << "," << e[k].to << "]";
        std::cout << "]}\n";
    }
    return 0;
}

static int forward(int argc, char** argv) {
    if (argc != 11) { std::fprintf(stderr, "forward IN A C NB H B blob planes out\n"); return 2; }
    const int IN = atoi(argv[2]), A = atoi(argv[3]), C = atoi(argv[4]), NB = atoi(argv[5]);
    const int H = atoi(argv[6]), B = atoi(argv[7]);
    torch::manual_seed(0);
    auto model = std::make_shared<DDWRandWireResNet>(IN, A, C, NB);
    model->eval();
    const std::vector<float> blob = read_f32(argv[8]);
    size_t off = 0;
    torch::NoGradGuard ng;
    for (const auto& m : model->named_modules()) {
        auto fill = [&](const std::string& name, torch::Tensor& t) {
            if (name.size() >= 19 && name.compare(name.size() - 19, 19, "num_batches_tracked") == 0) return;
            const size_t n = (size_t)t.numel();
            std::cout << "{\"name\":\"" << (m.key().empty() ? "" : m.key() + ".") << name << "\",\"shape\":";
            std::vector<int> sh(t.sizes().begin(), t.sizes().end());
            json_list(std::cout, sh);
            std::cout << "}\n";
            if (off + n > blob.size()) { std::fprintf(stderr, "blob too short\n"); std::exit(3); }
            auto src = torch::from_blob(const_cast<float*>(blob.data() + off), t.sizes(), torch::kFloat32);
            t.copy_(src);
            off += n;
        };
        for (auto& p : m.value()->named_parameters(false)) fill(p.key(), p.value());
        for (auto& b : m.value()->named_buffers(false)) fill(b.key(), b.value());
    }
    if (off != blob.size()) { std::fprintf(stderr, "blob size %zu, model takes %zu\n", blob.size(), off); return 3; }
    const std::vector<float> planes = read_f32(argv[9]);
    if (planes.size() != (size_t)B * IN * H * H) { std::fprintf(stderr, "planes size\n"); return 3; }
    auto x = torch::from_blob(const_cast<float*>(planes.data()), {B, IN, H, H}, torch::kFloat32).clone();
    auto [pol, val] = model->forward(x);
    pol = pol.contiguous();
    val = val.reshape({B}).contiguous();
    std::ofstream o(argv[10], std::ios::binary);
    o.write(reinterpret_cast<const char*>(pol.data_ptr<float>()), (std::streamsize)B * A * 4);
    o.write(reinterpret_cast<const char*>(val.data_ptr<float>()), (std::streamsize)B * 4);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 3 && std::string(argv[1]) == "graphs") return graphs(atoi(argv[2]));
    if (argc >= 2 && std::string(argv[1]) == "forward") return forward(argc, argv);
    std::fprintf(stderr, "usage: ref_randwire graphs NB | forward IN A C NB H B blob planes out\n");
    return 2;
}
