"""ctypes binding of libmzgo.so (include/mzgo.h).

torch is imported first on purpose: its bundled HIP runtime (soname
libamdhip64.so.7) is then the one libmzgo.so binds to, so device pointers and
streams are shared with torch in one HIP context.

There is no CPU fallback anywhere in ``mzgo``: if the library is missing this
module raises at import time.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede loading libmzgo.so)

LIB_PATH = os.environ.get("MZGO_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmzgo.so")

MZGO_OK, MZGO_EINVAL, MZGO_EHIP, MZGO_ENOWEIGHTS, MZGO_EASSERT = 0, -1, -2, -3, -4


class Config(ctypes.Structure):
    """``mzgo_config`` (field order and types must match include/mzgo.h)."""

    _fields_ = [
        ("board_size", ctypes.c_int),
        ("latent_dim", ctypes.c_int),
        ("num_games", ctypes.c_int),
        ("num_simulations", ctypes.c_int),
        ("max_moves", ctypes.c_int),
        ("compat", ctypes.c_int),
        ("temperature_moves", ctypes.c_int),
        ("search_variant", ctypes.c_int),
        ("c_puct", ctypes.c_double),
        ("discount", ctypes.c_double),
        ("dirichlet_alpha", ctypes.c_double),
        ("dirichlet_epsilon", ctypes.c_double),
        ("pass_epsilon", ctypes.c_double),
        ("temperature", ctypes.c_double),
        ("komi", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("game_base", ctypes.c_int),
        ("device", ctypes.c_int),
        ("direct_dynamics", ctypes.c_int),
        ("tower", ctypes.c_int),
        ("res_blocks", ctypes.c_int),
    ]


# name -> (restype, argtypes); every symbol include/mzgo.h declares
_P = ctypes.c_void_p
_I = ctypes.c_int
SIGNATURES = {
    "mzgo_default_config": (None, [ctypes.POINTER(Config), _I]),
    "mzgo_engine_create": (_I, [ctypes.POINTER(Config), ctypes.POINTER(_P)]),
    "mzgo_engine_destroy": (None, [_P]),
    "mzgo_last_error": (ctypes.c_char_p, []),
    "mzgo_engine_device_bytes": (ctypes.c_int64, [_P]),
    "mzgo_set_weights": (_I, [_P, ctypes.c_char_p, _P, ctypes.POINTER(ctypes.c_int64), _I]),
    "mzgo_weights_ready": (_I, [_P]),
    "mzgo_initial_inference": (_I, [_P, _P, _I, _P, _P, _P, _P]),
    "mzgo_recurrent_inference": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P]),
    "mzgo_check_inference_errors": (_I, [_P, _P]),
    "mzgo_search": (_I, [_P, _P, _P, _I, _I, _P, _P, _P]),
    "mzgo_tree_export": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mzgo_board_reset": (_I, [_P, _P]),
    "mzgo_board_step": (_I, [_P, _P, _P, _P, _P]),
    "mzgo_board_planes": (_I, [_P, _P, _P]),
    "mzgo_board_set": (_I, [_P, _I, _P, _P, _P, _P]),
    "mzgo_selfplay_reset": (_I, [_P, _I, _P]),
    "mzgo_selfplay_move": (_I, [_P, _P]),
    "mzgo_selfplay_moves": (_I, [_P, _I, _P]),
    "mzgo_arena_move": (_I, [_P, _P, _P]),
    "mzgo_arena_moves": (_I, [_P, _P, _I, _P]),
    "mzgo_selfplay_counters": (_I, [_P, _P, _P]),
    "mzgo_selfplay_set_timing": (_I, [_P, _I]),
    "mzgo_selfplay_launch_times": (_I, [_P, _P, _P, _I, _P]),
    "mzgo_stream_wait_started": (_I, [_P, ctypes.c_uint64, _P]),
    "mzgo_tower_timing": (_I, [_P, _I, _P, _P]),
    "mzgo_selfplay_inject_noise": (_I, [_P, _P]),
    "mzgo_selfplay_record_noise": (_I, [_P, _P]),
    "mzgo_tower_record_nodes": (_I, [_P, _P]),
    "mzgo_records_export": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mzgo_records_pack": (_I, [_P, _P, ctypes.c_int64, _P, _P]),
    "mzgo_dyn_conv_backward_workspace": (_I, [_I, _I, ctypes.POINTER(ctypes.c_int64)]),
    "mzgo_dyn_conv_backward": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P, ctypes.c_int64, _P]),
    "mzgo_conv3x3_relu_forward": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "mzgo_conv3x3_backward_workspace": (_I, [_I, _I, _I, ctypes.POINTER(ctypes.c_int64)]),
    "mzgo_conv3x3_backward": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, ctypes.c_int64, _P]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()' from the repo root)")
    lib = ctypes.CDLL(LIB_PATH)
    # (an older library loaded for an A/B, MZGO_LIB, may lack newer entry
    # points: they stay unbound there; the product library has every one)
    tolerant = "MZGO_LIB" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if tolerant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class MzgoError(RuntimeError):
    pass


def check(rc):
    """Raise on a non-zero mzgo status; GymGo's assertions stay AssertionError."""
    if rc == MZGO_OK:
        return
    msg = lib.mzgo_last_error().decode(errors="replace")
    if rc == MZGO_EASSERT:
        raise AssertionError(msg)
    if rc == MZGO_EINVAL and "index out of range" in msg:
        raise IndexError(msg)
    raise MzgoError(f"mzgo error {rc}: {msg}")


def ptr(t):
    """Device (or host) address of a contiguous torch tensor / numpy array."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        assert t.is_contiguous()
        return ctypes.c_void_p(t.data_ptr())
    return t.ctypes.data_as(ctypes.c_void_p)


def stream_of(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
