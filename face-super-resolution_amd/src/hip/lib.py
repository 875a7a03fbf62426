"""ctypes binding of libfen_hip.so (include/fen.h) -- the only way the package reaches the GPU.

The shared library is built in-tree (`face-super-resolution_amd/csrc/Makefile`, or
`__graft_entry__.build()`).  There is no fallback: if the library is missing every HIP
op raises, loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_float, c_int, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FEN_HIP_LIB", os.path.join(_HERE, "libfen_hip.so"))

F32, BF16, F16 = 0, 1, 2

EPI_BIAS = 1
EPI_PRELU = 2
EPI_SHUFFLE = 4
EPI_PRELU_BWD = 8
EPI_UNSHUFFLE = 16
EPI_POOL = 32
EPI_LAST = 64
EPI_DOT = 128
EPI_RELU_BWD = 4096


class AdamwJob(Structure):
    _fields_ = [("p", c_void_p), ("g", c_void_p), ("m", c_void_p), ("v", c_void_p), ("step", c_void_p),
                ("n", c_size_t)]


class ConvDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("Cin", c_int), ("Cout", c_int),
        ("x", c_void_p), ("w", c_void_p), ("bias", c_void_p), ("epi", c_int), ("alpha", c_void_p),
        ("y", c_void_p), ("y_pre", c_void_p), ("res", c_void_p * 3), ("pre_in", c_void_p),
        ("part", c_void_p), ("lr", c_void_p), ("scale", c_int), ("clamp", c_int), ("hr", c_void_p),
        ("dout", c_void_p), ("l1_scale", c_float), ("loss_part", c_void_p), ("debug", c_int),
        ("s2d_in", c_int), ("s2d_out", c_int),
        ("pre_elide", c_int), ("post_in", c_void_p), ("y_pool", c_void_p), ("y_images", c_int),
    ]


class ColsumJob(Structure):
    _fields_ = [("part", c_void_p), ("out", c_void_p), ("rows", c_int), ("cols", c_int), ("scale", c_float),
                ("accumulate", c_int)]


class PackJob(Structure):
    _fields_ = [("w", c_void_p), ("out", c_void_p), ("mode", c_int), ("Cout", c_int), ("Cin", c_int)]


class RcabDeferredDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("Cr", c_int),
        ("x", c_void_p), ("tp", c_void_p), ("pp", c_void_p), ("pfc1", c_void_p), ("pfc2", c_void_p),
        ("res_scale", c_float), ("inv_hw", c_float), ("ps", c_void_p), ("pmean", c_void_p), ("phid", c_void_p),
        ("xo", c_void_p), ("w1", c_void_p), ("b1", c_void_p), ("alpha", c_void_p), ("w2", c_void_p),
        ("b2", c_void_p), ("t", c_void_p), ("part", c_void_p), ("z1", c_void_p), ("a1", c_void_p),
        ("stamps", c_void_p),
    ]


class RcabBwdDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int),
        ("dt", c_void_p), ("w2t", c_void_p), ("z1", c_void_p), ("alpha", c_void_p), ("w1t", c_void_p),
        ("dy", c_void_p), ("dz1", c_void_p), ("dalpha_part", c_void_p), ("dx", c_void_p),
        ("dot_t", c_void_p), ("dot_part", c_void_p),
        ("se_part", c_void_p), ("se_s", c_void_p), ("se_mean", c_void_p), ("se_hid", c_void_p),
        ("se_w1", c_void_p), ("se_w2", c_void_p), ("se_dw1p", c_void_p), ("se_dw2p", c_void_p),
        ("se_res_scale", c_float), ("se_Cr", c_int), ("dres", c_void_p),
    ]


GS_MAXNB = 20   # FEN_GS_MAXNB


class GroupStripDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("Cr", c_int), ("nb", c_int),
        ("res_scale", c_float), ("x", c_void_p), ("y", c_void_p),
        ("w1", c_void_p * GS_MAXNB), ("b1", c_void_p * GS_MAXNB), ("alpha", c_void_p * GS_MAXNB),
        ("w2", c_void_p * GS_MAXNB), ("b2", c_void_p * GS_MAXNB), ("fc1", c_void_p * GS_MAXNB),
        ("fc2", c_void_p * GS_MAXNB), ("s_out", c_void_p * GS_MAXNB),
        ("wg", c_void_p), ("bg", c_void_p), ("work", c_void_p), ("work_bytes", c_size_t),
        ("save", c_int), ("sv_x", c_void_p * GS_MAXNB), ("sv_z1", c_void_p * GS_MAXNB),
        ("sv_a1", c_void_p * GS_MAXNB), ("sv_t", c_void_p * GS_MAXNB), ("sv_mean", c_void_p * GS_MAXNB),
        ("sv_hid", c_void_p * GS_MAXNB), ("x_last", c_void_p), ("status", c_void_p), ("fault", c_int),
        ("pre_elide", c_int),
    ]


class GroupStripChainTail(Structure):    # fen_group_strip_chain_tail: conv_after_body in the chain
    _fields_ = [("w", c_void_p), ("bias", c_void_p), ("skip", c_void_p), ("y", c_void_p)]


class GroupStripBwdDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("Cr", c_int), ("nb", c_int),
        ("res_scale", c_float), ("dy", c_void_p), ("dx", c_void_p), ("dres", c_void_p), ("wgt", c_void_p),
        ("w1t", c_void_p * GS_MAXNB), ("w2t", c_void_p * GS_MAXNB), ("alpha", c_void_p * GS_MAXNB),
        ("fc1", c_void_p * GS_MAXNB), ("fc2", c_void_p * GS_MAXNB), ("z1", c_void_p * GS_MAXNB),
        ("t", c_void_p * GS_MAXNB), ("s", c_void_p * GS_MAXNB), ("mean", c_void_p * GS_MAXNB),
        ("hid", c_void_p * GS_MAXNB), ("dt", c_void_p * GS_MAXNB), ("dz1", c_void_p * GS_MAXNB),
        ("dalpha_part", c_void_p * GS_MAXNB), ("dw1p", c_void_p * GS_MAXNB), ("dw2p", c_void_p * GS_MAXNB),
        ("work", c_void_p), ("work_bytes", c_size_t), ("status", c_void_p), ("fault", c_int),
        ("a1", c_void_p * GS_MAXNB),
    ]


class RcabC128Desc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("Cr", c_int), ("mode", c_int),
        ("res_scale", c_float), ("x", c_void_p), ("tp", c_void_p), ("pp", c_void_p), ("pfc1", c_void_p),
        ("pfc2", c_void_p), ("ps", c_void_p), ("xo", c_void_p), ("w", c_void_p), ("bias", c_void_p),
        ("alpha", c_void_p), ("res", c_void_p), ("y", c_void_p), ("z1", c_void_p), ("part", c_void_p),
    ]


class WgradDesc(Structure):
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("Cin", c_int), ("Cout", c_int),
        ("cout_valid", c_int), ("x", c_void_p), ("dy", c_void_p), ("dw", c_void_p), ("db", c_void_p),
        ("accumulate", c_int), ("work", c_void_p),
    ]


_SIGS = {
    "fen_conv3x3": (c_int, [POINTER(ConvDesc), c_void_p]),
    "fen_wgrad_work_floats": (c_size_t, [POINTER(WgradDesc)]),
    "fen_wgrad3x3": (c_int, [POINTER(WgradDesc), c_void_p]),
    "fen_wgrad_multi_work_floats": (c_size_t, [c_int, c_void_p]),
    "fen_wgrad3x3_multi": (c_int, [c_int, c_void_p, c_void_p]),
    "fen_rcab_deferred_supported": (c_int, [c_int] * 6),
    "fen_rcab_bwd_se_supported": (c_int, [c_int] * 6),
    "fen_rcab_deferred": (c_int, [POINTER(RcabDeferredDesc), c_void_p]),
    "fen_rcab_bwd": (c_int, [POINTER(RcabBwdDesc), c_void_p]),
    "fen_rcab_group_end": (c_int, [POINTER(RcabDeferredDesc)] + [c_void_p] * 5),
    "fen_group_strip_supported": (c_int, [c_int] * 7),
    "fen_group_strip_work_bytes": (c_size_t, [c_int, c_int]),
    "fen_group_strip": (c_int, [POINTER(GroupStripDesc), c_void_p]),
    "fen_group_strip_chain_work_bytes": (c_size_t, [c_int, c_int, c_int]),
    "fen_group_strip_chain_prepare": (c_int, [POINTER(GroupStripDesc), c_int, POINTER(GroupStripChainTail),
                                              c_void_p]),
    "fen_group_strip_chain": (c_int, [POINTER(GroupStripDesc), c_int, POINTER(GroupStripChainTail), c_void_p]),
    "fen_group_strip_bwd_supported": (c_int, [c_int] * 7),
    "fen_group_strip_bwd_work_bytes": (c_size_t, [c_int, c_int]),
    "fen_group_strip_bwd_dal_rows": (c_int, [c_int, c_int]),
    "fen_group_strip_bwd": (c_int, [POINTER(GroupStripBwdDesc), c_void_p]),
    "fen_rcab_c128_supported": (c_int, [c_int] * 6),
    "fen_rcab_c128_tiles": (c_int, [c_int] * 2),
    "fen_rcab_c128": (c_int, [POINTER(RcabC128Desc), c_void_p]),
    "fen_conv_first_fwd": (c_int, [c_int] * 6 + [c_void_p] * 4 + [c_void_p]),
    "fen_conv_first_fwd_ex": (c_int, [c_int] * 6 + [c_void_p] * 5 + [c_float, c_void_p, c_void_p]),
    "fen_conv_first_work_floats": (c_size_t, [c_int] * 5),
    "fen_conv_first_wgrad": (c_int, [c_int] * 6 + [c_void_p] * 4 + [c_int, c_void_p, c_void_p]),
    "fen_conv_last_dgrad_part_rows": (c_size_t, [c_int] * 3),
    "fen_conv_last_bwd_supported": (c_int, [c_int] * 6),
    "fen_conv_last_bwd": (c_int, [c_int] * 6 + [c_void_p] * 9 + [c_void_p]),
    "fen_conv_last_dgrad": (c_int, [c_int] * 6 + [c_void_p] * 7 + [c_void_p]),
    "fen_se_fwd": (c_int, [c_int, c_int, c_int, c_int, c_float] + [c_void_p] * 6 + [c_void_p]),
    "fen_se_fused": (c_int, [c_int] * 6 + [c_float] + [c_void_p] * 7 + [c_float, c_void_p, c_void_p, c_void_p]),
    "fen_se_apply": (c_int, [c_int] * 4 + [c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p]),
    "fen_pool_parts": (c_size_t, [c_int]),
    "fen_pool_dot": (c_int, [c_int] * 4 + [c_void_p] * 3 + [c_void_p]),
    "fen_se_bwd": (c_int, [c_int] * 4 + [c_float, c_float] + [c_void_p] * 9 + [c_void_p]),
    "fen_se_bwd_fused": (c_int, [c_int] * 6 + [c_float, c_float] + [c_void_p] * 11 + [c_void_p]),
    "fen_se_bwd_apply": (c_int, [c_int] * 4 + [c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p]),
    "fen_bicubic_down4": (c_int, [c_int] * 4 + [c_void_p, c_void_p, c_void_p]),
    "fen_colsum": (c_int, [c_int, c_int, c_void_p, c_float, c_void_p, c_int, c_void_p]),
    "fen_colsum_multi": (c_int, [c_int, c_void_p, c_void_p]),
    "fen_pack_conv_w": (c_int, [c_int] * 4 + [c_void_p, c_void_p, c_void_p]),
    "fen_pack_table_bytes": (c_size_t, [c_int]),
    "fen_pack_table": (c_int, [c_int, c_int, c_void_p, c_void_p, POINTER(c_size_t)]),
    "fen_pack_multi": (c_int, [c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "fen_packed_elems": (c_size_t, [c_int] * 3),
    "fen_nchw_to_nhwc": (c_int, [c_int] * 6 + [c_void_p, c_void_p, c_void_p]),
    "fen_prelu_bwd_unshuffle": (c_int, [c_int] * 5 + [c_void_p] * 5 + [c_void_p]),
    "fen_nhwc_to_nchw": (c_int, [c_int] * 5 + [c_void_p, c_void_p, c_void_p]),
    "fen_sumsq_parts": (c_int, [c_size_t]),
    "fen_sumsq": (c_int, [c_size_t, c_void_p, c_void_p, c_void_p]),
    "fen_optim_prepare": (c_int, [c_int, c_void_p, c_float, c_float, c_float, c_float, c_void_p, c_void_p]),
    "fen_adamw": (c_int, [c_size_t] + [c_void_p] * 5 + [c_float, c_float, c_float, c_void_p]),
    "fen_scale": (c_int, [c_size_t, c_void_p, c_float, c_void_p]),
    "fen_maxpool2": (c_int, [c_int] * 5 + [c_void_p] * 3),
    "fen_maxpool2_bwd_relu": (c_int, [c_int] * 5 + [c_void_p] * 4),
    "fen_feat_loss_parts": (c_int, []),
    "fen_feat_loss": (c_int, [c_int, c_size_t, c_void_p, c_int, c_float, c_void_p, c_int, c_void_p, c_void_p]),
    "fen_ssim_parts": (c_size_t, [c_int] * 4),
    "fen_ssim_work_floats": (c_size_t, [c_int] * 4),
    "fen_ssim_ex": (c_int, [c_int] * 5 + [c_void_p] * 3 + [c_int, c_float, c_float, c_void_p, c_void_p, c_float, c_int,
                                                          c_void_p, c_void_p]),
    "fen_ssim": (c_int, [c_int] * 5 + [c_void_p] * 3 + [c_int, c_float, c_float, c_void_p, c_void_p, c_float, c_int,
                                                        c_void_p]),
    "fen_augment_u8": (c_int, [c_int, c_int] + [c_void_p] * 5),
    "fen_bn_work_floats": (c_size_t, [c_int]),
    "fen_bn_stats": (c_int, [c_int, c_size_t, c_int, c_void_p, c_float, c_float] + [c_void_p] * 5),
    "fen_bn_apply": (c_int, [c_int, c_size_t, c_int] + [c_void_p] * 5 + [c_float, c_void_p, c_void_p]),
    "fen_bn_bwd": (c_int, [c_int, c_size_t, c_int] + [c_void_p] * 5 + [c_float] + [c_void_p] * 3 +
                   [c_int, c_void_p, c_void_p]),
    "fen_bn_stats_n": (c_int, [c_int, c_int, c_size_t, c_int, c_void_p, c_float, c_float] + [c_void_p] * 5),
    "fen_bn_apply_n": (c_int, [c_int, c_int, c_size_t, c_int] + [c_void_p] * 3 + [c_int] + [c_void_p] * 2 +
                       [c_float, c_void_p, c_void_p]),
    "fen_bn_bwd_n": (c_int, [c_int, c_int, c_size_t, c_int] + [c_void_p] * 5 + [c_float] + [c_void_p] * 3 +
                     [c_int, c_void_p, c_void_p]),
    "fen_subsample2": (c_int, [c_int] * 5 + [c_void_p] * 3),
    "fen_s2d2": (c_int, [c_int] * 5 + [c_void_p] * 2 + [c_int, c_void_p]),
    "fen_s2d_filter": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "fen_zero_insert2": (c_int, [c_int] * 5 + [c_void_p] * 3),
    "fen_adamw_multi": (c_int, [c_int, c_void_p] + [c_float] * 7 + [c_void_p]),
    "fen_l1_loss": (c_int, [c_size_t] + [c_void_p] * 3 + [c_float] + [c_void_p] * 3),
    "fen_gan_loss": (c_int, [c_int, c_int, c_void_p, c_float, c_void_p, c_void_p]),
    "fen_gan_loss_bwd": (c_int, [c_int, c_int, c_void_p, c_float, c_void_p, c_void_p, c_void_p]),
    "fen_dhead_work_floats": (c_size_t, [c_int] * 3),
    "fen_dhead_fwd": (c_int, [c_int] * 3 + [c_void_p] * 5 + [c_float, c_int] + [c_void_p] * 4),
    "fen_dhead_bwd": (c_int, [c_int] * 3 + [c_void_p] * 6 + [c_float, c_int] + [c_void_p] * 7),
    "fen_status_word": (c_int, [POINTER(c_void_p), POINTER(c_void_p)]),
    "fen_status_take": (c_int, [c_void_p]),
    "fen_rccl_unique_id": (c_int, [c_void_p]),
    "fen_rccl_init": (c_int, [POINTER(c_void_p), c_void_p, c_int, c_int, c_int]),
    "fen_rccl_allreduce_bucket": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "fen_rccl_check": (c_int, [c_void_p]),
    "fen_rccl_destroy": (c_int, [c_void_p]),
    "fen_last_rccl_error": (ctypes.c_char_p, []),
    "fen_rccl_library": (ctypes.c_char_p, []),
    "fen_status_string": (ctypes.c_char_p, [c_int]),
    "fen_last_hip_error": (ctypes.c_char_p, []),
    "fen_build_info": (ctypes.c_char_p, []),
}

EXPORTED = tuple(_SIGS)

_lib = None


class FenError(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes handle; raises FenError if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FenError(
            f"libfen_hip.so not found at {LIB_PATH}: build it with `make -C face-super-resolution_amd/csrc` "
            "or __graft_entry__.build(); the HIP backend has no fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(code: int, what: str = "") -> None:
    if code != 0:
        msg = load().fen_status_string(code).decode()
        if code == -3:
            msg += f" [{load().fen_last_hip_error().decode()}]"
        elif code == -4:
            msg += f" [{load().fen_last_rccl_error().decode()}]"
        raise FenError(f"{what}: {msg} (status {code})")


STATUS_GS_FWD, STATUS_GS_BWD, STATUS_GS_TABLE = 1, 2, 4   # FEN_STATUS_GS_*

_status = {}


def strip_status_ptr(device) -> int:
    """Device address of this process's status word for `device` (fen_status_word: one int in
    host-mapped coherent pinned memory): every fen_group_strip / fen_group_strip_bwd launch
    reports a timed-out hand-off wait there (include/fen.h).  The host reads the word without
    synchronising (`check_strip_status`), so a replayed hipGraph needs no extra node and the
    fault-free path costs nothing."""
    import torch
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ent = _status.get(key)
    if ent is None:
        hp, dp = c_void_p(), c_void_p()
        with torch.cuda.device(key):
            check(load().fen_status_word(ctypes.byref(hp), ctypes.byref(dp)), "status_word")
        # the host reads it through ctypes: no torch op (and no sync) per check
        ent = _status[key] = (int(dp.value), int(hp.value))
    return ent[0]


def check_strip_status() -> None:
    """Raise FenError if a strip launch enqueued earlier reported a timed-out wait (its outputs,
    and everything computed from them, are invalid), and clear the word.  A launch still in
    flight is seen by a later check."""
    for key, (_, host) in _status.items():
        v = load().fen_status_take(host)     # read + clear in one atomic exchange
        if v:
            if v & STATUS_GS_TABLE:
                raise FenError(f"fen_group_strip_chain on cuda:{key}: the launch found no parameter table prepared "
                               "for its descriptors in its workspace (fen_group_strip_chain_prepare after every "
                               "(re)allocation); it computed nothing")
            kinds = [n for b, n in ((STATUS_GS_FWD, "fen_group_strip"), (STATUS_GS_BWD, "fen_group_strip_bwd"))
                     if v & b]
            raise FenError(f"{' / '.join(kinds) or 'strip kernel'} on cuda:{key}: a hand-off wait between "
                           "strips timed out (another kernel held the CUs); that launch's outputs were invalid")


def dtype_code(torch_dtype) -> int:
    import torch
    if torch_dtype == torch.float32:
        return F32
    if torch_dtype == torch.bfloat16:
        return BF16
    if torch_dtype == torch.float16:
        return F16
    raise FenError(f"unsupported compute dtype {torch_dtype}")
