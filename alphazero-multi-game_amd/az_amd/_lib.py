"""ctypes binding of include/az_engine.h (libaz_hip.so, built in-tree).

Loading fails loudly if the library is missing; there is no CPU fallback."""
import ctypes
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG, "build", "libaz_hip.so")
# Measurement tools (tools/ab_builds.sh) may load an in-tree diagnostic build of the same library,
# named by AZ_DIAG_HIP_LIB; only PKG/build*/libaz_hip.so is accepted (never another library).
_diag = os.environ.get("AZ_DIAG_HIP_LIB")
if _diag:
    _d = os.path.realpath(_diag)
    if not (os.path.basename(_d) == "libaz_hip.so" and os.path.dirname(os.path.dirname(_d)) == os.path.realpath(PKG)
            and os.path.basename(os.path.dirname(_d)).startswith("build")):
        raise RuntimeError(f"AZ_DIAG_HIP_LIB={_diag}: only an in-tree build (build*/libaz_hip.so) may be loaded")
    LIB_PATH = _d

c_int, c_float, c_size_t, c_uint32, c_uint64, c_int64 = (ctypes.c_int, ctypes.c_float, ctypes.c_size_t,
                                                          ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64)
P = ctypes.POINTER
vp = ctypes.c_void_p

AZ_PREC_F32, AZ_PREC_BF16X3, AZ_PREC_BF16, AZ_PREC_FP16, AZ_PREC_F16X3 = 0, 1, 2, 3, 4
AZ_EVAL_NET, AZ_EVAL_HASH, AZ_EVAL_RANDOM, AZ_EVAL_UNIFORM, AZ_EVAL_CALLBACK = 0, 1, 2, 3, 4


class NetDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("board_size", "in_planes", "channels", "blocks", "action_size", "head_channels",
                                     "pool", "fc_hidden", "residual", "conv_bias", "precision", "max_batch")]


class SearchCfg(ctypes.Structure):
    _fields_ = [("n_games", c_int), ("board_size", c_int), ("num_simulations", c_int), ("c_puct", c_float),
                ("fpu_reduction", c_float), ("virtual_loss", c_int), ("eval_kind", c_int), ("eval_seed", c_uint32),
                ("zobrist_seed", c_uint32), ("noise_seed", c_uint32), ("noise_seed_stride", c_int),
                ("use_dirichlet_each_search", c_int), ("dirichlet_alpha", c_float), ("dirichlet_eps", c_float),
                ("tt_log2", c_int), ("node_capacity", c_int), ("prior_ring", c_int), ("game", c_int)]


class SelfPlayCfg(ctypes.Structure):
    _fields_ = [("temp_drop_move", c_int), ("t_init", c_float), ("t_final", c_float), ("restart_finished", c_int)]


class MoveRec(ctypes.Structure):
    _fields_ = [("action", c_int), ("value", c_float), ("n_children", c_int), ("policy", P(c_float)),
                ("child_actions", P(c_int)), ("thinking_time_ms", c_int64)]


EVAL_FN = ctypes.CFUNCTYPE(c_int, vp, c_int, P(c_int), P(c_int), P(c_int), c_int, P(c_float), c_int, P(c_float),
                           P(c_float))
GAME_SINK = ctypes.CFUNCTYPE(None, vp, c_int, c_int, c_int, P(MoveRec), c_int)
PROGRESS_FN = ctypes.CFUNCTYPE(None, vp, c_int, c_int, c_int, c_int64)

EXPORTS = {
    "az_last_error": (ctypes.c_char_p, []),
    "az_engine_create": (c_int, [c_int, P(vp)]),
    "az_engine_destroy": (None, [vp]),
    "az_engine_device_name": (c_int, [vp, ctypes.c_char_p, c_int]),
    "az_net_create": (c_int, [vp, P(NetDesc), P(vp)]),
    "az_net_create_randwire": (c_int, [vp, P(NetDesc), P(vp)]),
    "az_net_create_randwire_graphs": (c_int, [vp, P(NetDesc), P(c_int), c_size_t, P(vp)]),
    "az_randwire_graph": (c_int, [c_int, P(c_int), P(c_int), P(c_int), P(c_int), P(c_int), P(c_int), P(c_int), P(c_int),
                                  c_int]),
    "az_net_destroy": (None, [vp]),
    "az_net_num_params": (c_int, [vp, P(c_size_t)]),
    "az_net_load_weights": (c_int, [vp, P(c_float), c_size_t]),
    "az_net_init_random": (c_int, [vp, c_uint64]),
    "az_net_get_weights": (c_int, [vp, P(c_float), c_size_t]),
    "az_net_set_precision": (c_int, [vp, c_int]),
    "az_net_forward": (c_int, [vp, P(c_float), c_int, P(c_float), P(c_float)]),
    "az_net_predict_batch": (c_int, [vp, P(c_float), c_int, P(c_float), P(c_float)]),
    "az_net_profile": (c_int, [vp, c_int]),
    "az_net_profile_read": (c_int, [vp, P(ctypes.c_double), P(c_int64), P(c_int64)]),
    "az_net_trunk_kernel": (c_int, [vp, ctypes.c_char_p, c_int]),
    "az_search_create": (c_int, [vp, vp, P(SearchCfg), P(vp)]),
    "az_search_destroy": (None, [vp]),
    "az_search_new_games": (c_int, [vp, P(c_int), c_int]),
    "az_search_add_noise": (c_int, [vp, c_float, c_float]),
    "az_search_add_noise_masked": (c_int, [vp, c_float, c_float, P(ctypes.c_uint8)]),
    "az_search_run": (c_int, [vp]),
    "az_search_simulate": (c_int, [vp, c_int]),
    "az_search_release": (c_int, [vp, c_int, P(c_int64)]),
    "az_search_select_action": (c_int, [vp, c_int, c_int, c_float, c_int, P(c_int), c_int, P(c_int)]),
    "az_search_select": (c_int, [vp, c_int, c_float, P(c_int), P(c_float), P(c_float), P(c_int), P(c_int)]),
    "az_search_apply": (c_int, [vp, P(c_int), P(c_int), P(c_int)]),
    "az_search_root_children": (c_int, [vp, c_int, P(c_int), P(c_int), P(c_int), P(c_float), P(c_float), P(c_int)]),
    "az_search_root_flags": (c_int, [vp, c_int, P(c_int)]),
    "az_search_seed": (c_int, [vp, c_int, c_uint32]),
    "az_search_get_rng": (c_int, [vp, c_int, vp]),
    "az_search_set_net": (c_int, [vp, vp]),
    "az_search_run_masked": (c_int, [vp, vp]),
    "az_search_simulate_masked": (c_int, [vp, c_int, vp]),
    "az_search_release_masked": (c_int, [vp, c_int, vp, vp]),
    "az_search_new_games_ids": (c_int, [vp, vp, vp, c_int]),
    "az_search_clear_tt": (c_int, [vp]),
    "az_search_set_rng": (c_int, [vp, c_int, vp]),
    "az_search_set_evaluator": (c_int, [vp, EVAL_FN, vp]),
    "az_search_set_params": (c_int, [vp, P(SearchCfg)]),
    "az_search_root_node": (c_int, [vp, c_int, P(c_int), P(c_int), P(c_float)]),
    "az_search_counters": (c_int, [vp, c_int, P(c_int64)]),
    "az_search_profile": (c_int, [vp, c_int]),
    "az_search_profile_read": (c_int, [vp, P(ctypes.c_double), P(ctypes.c_double), P(c_int64), P(c_int64), P(c_int64)]),
    "az_search_profile_read_fused": (c_int, [vp, P(ctypes.c_double), P(c_int64)]),
    "az_search_enable_eval_log": (c_int, [vp, c_int, c_int]),
    "az_search_read_eval_log": (c_int, [vp, P(c_float), P(c_float), P(c_float), P(c_int)]),
    "az_selfplay_step": (c_int, [vp, P(SelfPlayCfg), P(c_int64), P(c_int64)]),
    "az_selfplay_step_moves": (c_int, [vp, P(P(MoveRec)), P(P(c_int)), P(c_int)]),
    "az_selfplay_run": (c_int, [vp, P(SelfPlayCfg), c_int, c_int, GAME_SINK, PROGRESS_FN, vp, P(c_int)]),
    "az_dataset_create": (c_int, [vp, c_int, c_int, P(vp)]),
    "az_dataset_destroy": (None, [vp]),
    "az_dataset_extract": (c_int, [vp, c_int, P(c_int), P(c_int), P(c_int), P(c_float), P(c_int), c_int, P(c_int64),
                                   P(c_int64)]),
    "az_dataset_info": (c_int, [vp, P(c_int64), P(c_int), P(c_int), P(c_int)]),
    "az_dataset_seed": (c_int, [vp, c_uint32]),
    "az_dataset_shuffle_order": (c_int, [vp, c_int64, P(c_int64)]),
    "az_dataset_upload": (c_int, [vp, c_int64, P(c_float), P(c_float), P(c_int), P(c_float)]),
    "az_dataset_permute": (c_int, [vp, P(c_int64)]),
    "az_dataset_gather": (c_int, [vp, P(c_int64), c_int, P(c_float), P(c_float), P(c_int), P(c_float)]),
    "az_dataset_profile_read": (c_int, [vp, P(ctypes.c_double), P(ctypes.c_double)]),
    "az_dist_unique_id": (c_int, [P(ctypes.c_ubyte)]),
    "az_dist_init": (c_int, [vp, c_int, c_int, P(ctypes.c_ubyte), c_int, P(vp)]),
    "az_dist_destroy": (None, [vp]),
    "az_dist_info": (c_int, [vp, P(c_int), P(c_int)]),
    "az_dist_barrier": (c_int, [vp]),
    "az_counters_allreduce": (c_int, [vp, P(ctypes.c_double), P(ctypes.c_double), c_int, c_int]),
    "az_net_broadcast_weights": (c_int, [vp, vp, c_int]),
}
AZ_DIST_ID_BYTES = 128
AZ_DIST_SUM, AZ_DIST_MAX = 0, 1

_lib = None


def lib():
    """Load libaz_hip.so and bind every entry point declared in include/az_engine.h."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libaz_hip.so not built ({LIB_PATH}); run __graft_entry__.build() / make -C "
                               f"alphazero-multi-game_amd")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


AZ_ERR_ARG, AZ_ERR_HIP, AZ_ERR_OOM, AZ_ERR_CAPACITY, AZ_ERR_STATE, AZ_ERR_RANGE = -1, -2, -3, -4, -5, -6


class AzError(RuntimeError):
    def __init__(self, msg, code=0):
        super().__init__(msg)
        self.code = code


def check(rc):
    if rc != 0:
        raise AzError(f"az error {rc}: {lib().az_last_error().decode()}", rc)
    return rc
