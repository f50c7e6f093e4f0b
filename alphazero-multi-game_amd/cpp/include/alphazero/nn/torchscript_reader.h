// alphazero/nn/torchscript_reader.h -- the parameters and buffers of a TorchScript archive
// (torch.jit.save: the reference's model files, exported by python/scripts/self_play.py:139-193 and
// loaded by TorchNeuralNetwork through torch::jit::load, torch_neural_network.cpp:90), read WITHOUT
// executing anything from the file: a zip directory reader (the tensor records are stored
// uncompressed) and a restricted pickle machine for data.pkl that knows only the opcodes torch's
// pickler emits and resolves only these globals -- the archive's own module classes
// (__torch__.*, kept as plain attribute dictionaries), torch._utils._rebuild_tensor_v2 /
// _rebuild_parameter, torch.<T>Storage and collections.OrderedDict.  Anything else throws.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "alphazero/core/igamestate.h"

namespace alphazero {
namespace nn {

struct NamedTensor {
    std::string name;                 // state_dict key ("input_conv.weight", "res_blocks.0.1.running_var", ...)
    std::vector<int64_t> shape;
    std::vector<float> data;          // converted to fp32 (float / double / half / bfloat16 / int64 / int32 storages)
};

// Every tensor of the module tree in state_dict order (a module's attributes in the order the
// archive lists them: parameters, buffers, then submodules).
std::vector<NamedTensor> readTorchScript(const std::string& path);

// true when the file starts with a zip local header (a TorchScript / torch.save archive)
bool isZipArchive(const std::string& path);

struct NetShape;

// The reference's plain ResNet family as a TorchScript archive -> the engine's net shape and
// canonical weight blob (state_dict order, num_batches_tracked dropped).  Recognised layouts:
// python/simple_export.py SimplifiedModel (res_blocks.*: residual blocks, conv biases) and the
// exporter fallback of python/scripts/simple_export.py (middle_layers.*: a plain conv stack,
// adaptive 8x8 pool).  boardSize <= 0: from the policy size (A = bs^2, Go A = bs^2 + 1).
// Throws std::invalid_argument for any other module layout (e.g. the rand-wire net).
std::vector<float> torchScriptResNet(const std::string& path, core::GameType type, int boardSize, NetShape& shape);

}  // namespace nn
}  // namespace alphazero
