"""The C-ABI library loads on CPU and exports every entry point include/fen.h declares."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "fen.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fen_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from src.hip import lib as L
    lib = L.load()
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(L.EXPORTED), set(names) ^ set(L.EXPORTED)


def test_status_strings_and_pure_queries():
    from src.hip import lib as L
    lib = L.load()
    assert lib.fen_status_string(-2).startswith(b"FEN_EUNSUPPORTED")
    assert b"gfx950" in lib.fen_build_info()
    assert lib.fen_packed_elems(0, 3, 64) == 9 * 16 * 64
    assert lib.fen_packed_elems(2, 256, 64) == 9 * 64 * 256
    assert lib.fen_pool_parts(4096) == 64
    assert lib.fen_sumsq_parts(5115651) == 1024


def test_bad_args_rejected_without_gpu():
    """Argument validation happens before any launch, so it is testable on CPU."""
    from src.hip import lib as L
    lib = L.load()
    d = L.ConvDesc()
    assert lib.fen_conv3x3(None, None) == L.load().fen_conv3x3(None, None) == -1
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = 1, 1, 8, 8, 36, 64  # 72-B pixel rows: not whole 16-B chunks
    d.x = d.w = d.y = 16
    assert lib.fen_conv3x3(d, None) == -2
    with pytest.raises(L.FenError):
        L.check(-2, "conv")


def test_rcab_deferred_validation_without_gpu():
    from src.hip import lib as L
    lib = L.load()
    assert lib.fen_rcab_deferred(None, None) == -1
    assert lib.fen_rcab_deferred_supported(L.BF16, 32, 64, 64, 64, 16) == 1
    assert lib.fen_rcab_deferred_supported(L.F16, 32, 64, 64, 64, 16) == 1
    assert lib.fen_rcab_deferred_supported(L.F32, 32, 64, 64, 64, 16) == 0      # 16-bit only
    assert lib.fen_rcab_deferred_supported(L.BF16, 32, 64, 60, 64, 16) == 0     # W % 16
    assert lib.fen_rcab_deferred_supported(L.BF16, 32, 64, 64, 128, 32) == 0    # C = 64 only
    d = L.RcabDeferredDesc()
    d.dtype, d.B, d.H, d.W, d.C, d.Cr = L.BF16, 2, 32, 32, 64, 16
    d.x = d.w1 = d.w2 = d.b1 = d.b2 = d.alpha = d.t = d.part = 16
    d.tp = 16                       # deferred input without part_{j-1} / fc weights / x_j out
    assert lib.fen_rcab_deferred(d, None) == -1
    d.tp, d.z1 = 0, 16              # z1 without a1
    assert lib.fen_rcab_deferred(d, None) == -1


def test_wgrad_multi_validation_without_gpu():
    """fen_wgrad3x3_multi: job count bounds, one shape per launch, workspace size (n jobs of
    the persistent kernel share the ~256 slabs of one job)."""
    import ctypes
    from src.hip import lib as L
    lib = L.load()
    arr = (L.WgradDesc * 33)()                                    # FEN_WGRAD_MAXJOBS + 1
    for d in arr:
        d.dtype, d.B, d.H, d.W, d.Cin, d.Cout, d.cout_valid = L.BF16, 32, 64, 64, 64, 64, 64
        d.x = d.dy = d.dw = d.work = 16
    p = ctypes.cast(arr, ctypes.c_void_p)
    assert lib.fen_wgrad3x3_multi(0, p, None) == -1
    assert lib.fen_wgrad3x3_multi(33, p, None) == -1
    assert lib.fen_wgrad_multi_work_floats(33, p) == 0
    one = lib.fen_wgrad_work_floats(ctypes.byref(arr[0]))
    assert one == 256 * (64 * 64 * 9 + 64)
    assert lib.fen_wgrad_multi_work_floats(4, p) == one          # 4 jobs x 64 chunks
    arr[2].H = 32                                                 # shapes differ
    assert lib.fen_wgrad3x3_multi(4, p, None) == -1
    arr[2].H = 64
    arr[3].x = None
    assert lib.fen_wgrad3x3_multi(4, p, None) == -1
    arr[3].x = 16
    # njobs x (Cout/64) x (Cin/64) > 256 even at one chunk per job: the launch geometry must
    # terminate (one chunk per job, more than one wave of blocks) rather than spin on the host
    for n, c in ((5, 512), (17, 256)):
        for d in arr:
            d.Cin = d.Cout = d.cout_valid = c
        assert lib.fen_wgrad_multi_work_floats(n, p) == n * (c * c * 9 + c)


def test_conv_dot_epilogue_validation_without_gpu():
    """FEN_EPI_DOT needs pre_in (the dotted tensor) and part, and is one partial-sum stream:
    not combinable with POOL / PRELU_BWD, SHUFFLE / UNSHUFFLE or LAST."""
    from src.hip import lib as L
    lib = L.load()
    d = L.ConvDesc()
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = L.BF16, 1, 16, 16, 64, 64
    d.x = d.w = d.y = 16
    d.epi = L.EPI_DOT
    assert lib.fen_conv3x3(d, None) == -1            # no pre_in / part
    d.pre_in = d.part = 16
    d.epi = L.EPI_DOT | L.EPI_POOL
    assert lib.fen_conv3x3(d, None) == -2
    d.epi = L.EPI_DOT | L.EPI_UNSHUFFLE
    assert lib.fen_conv3x3(d, None) == -2


def test_conv_relu_bwd_and_pool_validation_without_gpu():
    """FEN_EPI_RELU_BWD needs pre_in and excludes the other pre_in modes; y_images needs y_pool;
    y_pool needs the PReLU epilogue and even H, W (all refused before any launch)."""
    from src.hip import lib as L
    lib = L.load()
    d = L.ConvDesc()
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = L.BF16, 2, 16, 16, 64, 64
    d.x = d.w = d.y = 16
    d.epi = L.EPI_RELU_BWD
    assert lib.fen_conv3x3(d, None) == -1            # no pre_in
    d.pre_in = d.part = d.alpha = 16
    d.epi = L.EPI_RELU_BWD | L.EPI_PRELU_BWD
    assert lib.fen_conv3x3(d, None) == -2
    d.epi = L.EPI_RELU_BWD | L.EPI_SHUFFLE
    assert lib.fen_conv3x3(d, None) == -2
    d.epi = 1 << 20
    assert lib.fen_conv3x3(d, None) == -1            # unknown flag
    d.epi, d.y_images = L.EPI_PRELU, 1
    assert lib.fen_conv3x3(d, None) == -1            # y_images without y_pool
    d.y_pool, d.y_images = 16, 3
    assert lib.fen_conv3x3(d, None) == -1            # y_images > B
    d.epi, d.y_images = 0, 0
    assert lib.fen_conv3x3(d, None) == -2            # y_pool without PReLU
    d.epi, d.H = L.EPI_PRELU, 15
    assert lib.fen_conv3x3(d, None) == -2            # odd H


def test_group_strip_chain_validation_without_gpu():
    """fen_group_strip_chain's host checks run before any copy or launch: a broken chain, too many
    step tags and a tail aliasing the body's buffers are refused on CPU (a launch without a
    matching prepared table is refused on the GPU, by the kernel: test_gpu_group_chain.py)."""
    from src.hip import lib as L
    lib = L.load()
    B, H, nb, G = 2, 64, 2, 3
    nbytes = lib.fen_group_strip_chain_work_bytes(B, H, G)
    assert nbytes > lib.fen_group_strip_work_bytes(B, H)
    assert lib.fen_group_strip_chain_work_bytes(B, 12, G) == 0          # H not a multiple of 8
    ds = (L.GroupStripDesc * G)()
    for g in range(G):
        d = ds[g]
        d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.nb, d.res_scale = 1, B, H, 64, 64, 16, nb, 0.2
        d.x, d.y = 0x10000 * (g + 1), 0x10000 * (g + 2)                  # group g's output = g+1's input
        for j in range(nb):
            d.w1[j] = d.b1[j] = d.alpha[j] = d.w2[j] = d.b2[j] = d.fc1[j] = d.fc2[j] = 0x1000
        d.wg = d.bg = 0x1000
        d.work, d.work_bytes = 0x100000, nbytes
    # not a chain: group 1's input is not group 0's output
    ds[1].x = 0x90000
    assert lib.fen_group_strip_chain(ds, G, None, None) == -1
    assert lib.fen_group_strip_chain_prepare(ds, G, None, None) == -1
    ds[1].x = ds[0].y
    # the conv_after_body step may not write the body's output or its skip
    t = L.GroupStripChainTail()
    t.w = t.bias = 0x1000
    t.skip, t.y = ds[0].x, ds[G - 1].y
    assert lib.fen_group_strip_chain_prepare(ds, G, t, None) == -1
    # more steps than the 8-bit step tags hold: (nb + 1) * groups > 254
    big = (L.GroupStripDesc * 13)()
    for g in range(13):
        big[g] = ds[0]
        big[g].nb = 19
        big[g].x, big[g].y = 0x10000 * (g + 1), 0x10000 * (g + 2)
    assert lib.fen_group_strip_chain_prepare(big, 13, None, None) == -2


def test_rccl_and_status_entry_points_without_gpu():
    """fen_rccl_* validate their arguments before touching RCCL; fen_status_take reads and
    clears a word in one atomic exchange (here on plain host memory)."""
    import ctypes
    from src.hip import lib as L
    lib = L.load()
    assert lib.fen_status_string(-4).startswith(b"FEN_ERCCL")
    assert lib.fen_rccl_allreduce_bucket(None, None, 16, None) == -1
    assert lib.fen_rccl_init(None, None, 1, 0, 0) == -1
    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * 128)()
    assert lib.fen_rccl_init(ctypes.byref(h), uid, 2, 2, 0) == -1       # rank outside nranks
    assert lib.fen_rccl_check(None) == -1
    assert lib.fen_rccl_destroy(None) == 0
    w = ctypes.c_int32(3)
    assert lib.fen_status_take(ctypes.addressof(w)) == 3 and w.value == 0
    assert lib.fen_status_take(ctypes.addressof(w)) == 0
    assert lib.fen_status_take(None) == 0
