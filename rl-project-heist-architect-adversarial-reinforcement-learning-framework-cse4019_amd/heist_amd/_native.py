"""ctypes binding of libheist_hip.so (include/heist.h).

torch is imported first on purpose: the library is linked against the HIP runtime
that torch ships (same soname), so torch tensors' device pointers and streams are
valid inside it.  There is no CPU fallback: if the library or the GPU is missing,
the calls raise.
"""
import ctypes
import os
import re

import torch

from . import _build

_lib = None

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_d = ctypes.c_double
_f = ctypes.c_float

# name -> (restype, argtypes); pointers are passed as c_void_p (device addresses).
SIGNATURES = {
    "heist_abi_version": (_i, []),
    "heist_last_error": (ctypes.c_char_p, []),
    "heist_create": (_i, [_i, _i, _i, _i, _i, _i, _i, ctypes.POINTER(_d), _i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "heist_destroy": (_i, [_vp]),
    "heist_set_layout": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "heist_reset": (_i, [_vp, _vp, _vp, _vp]),
    "heist_step": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp]),
    "heist_step_multi": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp]),
    "heist_export": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "heist_count_samples": (_i, [_vp, _vp]),
    "heist_count_redo": (_i, [_vp, _vp]),
    "heist_set_ray_mode": (_i, [_vp, _i]),
    "heist_set_guard_cones": (_i, [_vp, _i]),
    "heist_step_waves": (_i, [_vp]),
    "heist_get_config": (_i, [_vp, _vp, _i]),
    "heist_step_stamps": (_i, [_vp, _vp, _i64]),
    "heist_stamp_words": (_i64, [_vp, _i]),
    "heist_bfs_valid": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "heist_cones": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "heist_cones_mode": (_i, [_i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp]),
    "heist_cone_order": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "heist_fast_dir": (_i, [_vp, _i64, _vp, _vp, _vp]),
    "heist_architect_decode": (_i, [_vp, _i, _i, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp]),
    "heist_sincos": (_i, [_vp, _i64, _vp, _vp, _vp]),
    "heist_arch_update_workspace_bytes": (_i64, []),
    "heist_arch_update_supported": (_i, [_i, _i]),
    "heist_arch_update_sequence": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _i, _i,
                                        _vp, _i, _vp, _d, _d, _d, _d, _d, _vp, _vp, _vp]),
    "heist_arch_update_timed_out": (_i, [_vp, ctypes.POINTER(_i), _vp]),
    "heist_arch_update_status": (_i, [_vp, ctypes.POINTER(_i), _vp]),
    "heist_bias_relu_nhwc": (_i, [_vp, _vp, _i64, _i, _vp]),
    "heist_bias_relu_pool_nhwc": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "heist_pool_relu_bwd_nhwc": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "heist_relu_bwd_nhwc": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "heist_arch_update_stamps": (_i, [_vp]),
    "heist_gae": (_i, [_vp, _vp, _vp, _vp, _i, _i, _d, _d, _vp, _vp, _vp]),
    "heist_lstm_cell": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "heist_rollout_tally": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "heist_adv_moments": (_i, [_vp, _i64, _i, _vp, _vp]),
    "heist_adv_apply": (_i, [_vp, _i64, _vp, _f, _vp]),
    "heist_adv_normalize": (_i, [_vp, _i64, _vp, _f, _vp]),
    "heist_ppo_loss": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _d, _d, _d, _vp, _vp, _vp, _vp, _vp]),
    "heist_solver_packed_bytes": (_i, []),
    "heist_solver_pack": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "heist_solver_features": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp]),
    "heist_solver_stamps": (_i, [_vp]),
    "heist_solver_head_packed_bytes": (_i, []),
    "heist_solver_head_pack": (_i, [_vp] * 14 + [_i, _vp, _vp]),
    "heist_solver_head": (_i, [_vp, _vp, _vp, _i, _vp, _i, ctypes.c_uint64, ctypes.c_uint64] + [_vp] * 7),
    "heist_train_conv_supported": (_i, [_i, _i]),
    "heist_train_conv_frag_floats": (_i, [_i, _i]),
    "heist_train_conv_pack": (_i, [_i, _i, _vp, _vp, _vp]),
    "heist_train_conv": (_i, [_i, _i, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "heist_train_conv_partial_floats": (_i64, [_i, _i, _i, _i]),
    "heist_train_conv_wgrad": (_i, [_i, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "heist_train_obs_nhwc4": (_i, [_vp, _i, _i, _i, _i64, _i64, _i64, _i64, _vp, _vp]),
    "heist_train_pool": (_i, [_vp, _i, _i, _i, _vp, _vp]),
    "heist_train_pool_bwd": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
}


class HeistError(RuntimeError):
    pass


def header_functions():
    """Function names declared in include/heist.h (the ABI contract)."""
    with open(os.path.join(_build.INCLUDE, "heist.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(heist_\w+)\s*\(", txt, re.M)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_build.LIB_PATH):
            raise HeistError("libheist_hip.so is not built (%s); run __graft_entry__.build()" % _build.LIB_PATH)
        L = ctypes.CDLL(_build.LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().heist_last_error()
        raise HeistError("%s failed (code %d): %s" % (what, rc, msg.decode() if msg else ""))


def ptr(t):
    """Device address of a tensor (None -> NULL).  Tensors must be contiguous."""
    if t is None:
        return None
    if not t.is_cuda:
        raise HeistError("expected a device tensor, got %s" % t.device)
    if not t.is_contiguous():
        raise HeistError("expected a contiguous tensor")
    return _vp(t.data_ptr())


def ptr_nhwc(t):
    """Device address of a 4-D tensor laid out channels-last (NHWC), dense."""
    if not t.is_cuda:
        raise HeistError("expected a device tensor, got %s" % t.device)
    if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last):
        raise HeistError("expected a dense channels-last [N, C, H, W] tensor")
    return _vp(t.data_ptr())


def stream(device=None):
    return _vp(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(device=None):
    if not torch.cuda.is_available():
        raise HeistError("no HIP device: heist_amd has no CPU fallback")
    d = torch.device(device) if device is not None else torch.device("cuda")
    if d.type != "cuda":
        raise HeistError("heist_amd runs on HIP devices, got %s" % d)
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())
