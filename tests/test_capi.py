"""C ABI checks that need no GPU: the library loads, exports exactly what
include/dro_amd.h declares, and rejects bad arguments before launching."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dro_amd.h")
LIB = os.path.join(ROOT, "dro-sfm_amd", "libdro_amd.so")


def declared():
    txt = open(HEADER).read()
    return set(re.findall(r"\b(dro_[a-z0-9_]+)\s*\(", txt))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libdro_amd.so not built: run `make -C dro-sfm_amd/csrc`")
    import torch  # noqa: F401  (HIP runtime of torch first, as the product does)
    from dro_sfm_amd.hip import _lib
    return _lib.load()


def test_header_matches_exports(lib):
    from dro_sfm_amd.hip import _lib
    names = declared()
    assert names == set(_lib.EXPORTED)
    for n in names:
        assert hasattr(lib, n), n


def test_abi_version(lib):
    assert lib.dro_abi_version() == 10


def test_null_arguments_rejected(lib):
    NULL = None
    st = lib.dro_warp_cost_forward(NULL, NULL, NULL, 0, 0.0, 0.0, NULL, NULL, 0.125, NULL, 0,
                                   1, 1, 1, 2, 2, 1, 0, NULL, NULL)
    assert st == -1
    assert b"NULL" in lib.dro_last_error()
    st = lib.dro_photometric_forward(NULL, NULL, NULL, NULL, NULL, NULL, 0, 1, 1, 1, 8, 8, 0.85,
                                     1e-4, 9e-4, 1e-3, 1, 1, 0.0, NULL, NULL, NULL)
    assert st == -1
    st = lib.dro_convex_upsample_forward(NULL, NULL, 1, 2, 2, 8, 0.0, 1.0, NULL, NULL)
    assert st == -1


def test_bad_sizes_and_modes_rejected(lib):
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    # h = 1 is out of range (normalisation divides by h-1)
    assert lib.dro_warp_cost_forward(p, p, p, 0, 0.0, 0.0, p, p, 0.125, p, 0, 1, 1, 1, 1, 4, 1, 0,
                                     p, None) == -2
    # unknown pose mode
    assert lib.dro_warp_cost_forward(p, p, p, 0, 0.0, 0.0, p, p, 0.125, p, 7, 1, 1, 1, 2, 2, 1, 0,
                                     p, None) == -3
    # unknown reference layout
    assert lib.dro_warp_cost_forward(p, p, p, 0, 0.0, 0.0, p, p, 0.125, p, 0, 1, 1, 1, 2, 2, 1, 2,
                                     p, None) == -3
    # automask needs the min reduction
    assert lib.dro_photometric_forward(p, p, p, p, p, p, 0, 1, 1, 1, 8, 8, 0.85, 1e-4, 9e-4, 1e-3,
                                       1, 0, 0.0, p, p, None) == -3
    # clip_loss NaN
    assert lib.dro_photometric_forward(p, p, p, p, p, p, 0, 1, 1, 1, 8, 8, 0.85, 1e-4, 9e-4, 1e-3,
                                       1, 1, float("nan"), p, p, None) == -3
    assert lib.dro_convex_upsample_forward(p, p, 1, 2, 2, 9, 0.0, 1.0, p, None) == -2


def test_workspace_sizes(lib):
    assert lib.dro_warp_cost_workspace_bytes(2, 2, 24, 80) >= 2 * 2 * 24 * 80 * 2 * 4
    assert lib.dro_photometric_workspace_bytes(2, 2, 9, 192, 640, 0.0) >= 9 * 2 * 192 * 640
    # clip_loss > 0 keeps the N*n warped maps between the two forward passes
    assert (lib.dro_photometric_workspace_bytes(2, 2, 9, 192, 640, 0.5)
            >= lib.dro_photometric_workspace_bytes(2, 2, 9, 192, 640, 0.0) + 4 * 2 * 9 * 2 * 192 * 640)
    pm, thr = (lib.dro_photometric_clip_offset(2, 2, 9, 192, 640, w) for w in (0, 1))
    assert pm + 4 * 2 * 9 * 2 * 192 * 640 <= thr and pm % 4 == 0 and thr % 4 == 0
    assert thr + 4 * (2 * 9 + 2) <= lib.dro_photometric_workspace_bytes(2, 2, 9, 192, 640, 0.5)
    # conv: at least the pre-activation gradient and the weight-gradient partials
    P = 2 * 24 * 80
    assert lib.dro_conv2d_workspace_bytes(2, 24, 80, 320, 256, 1, 5) >= 256 * P * 4 + 256 * 320 * 5 * 4
    assert lib.dro_conv2d_workspace_bytes(0, 24, 80, 320, 256, 1, 5) == 0


def test_no_cpu_fallback():
    """Product ops refuse CPU tensors (there is no CPU path)."""
    import torch
    import dro_sfm_amd.hip as H
    x = torch.zeros(1, 4, 2, 2)
    with pytest.raises(RuntimeError):
        H.warp_cost(x, x.unsqueeze(0), torch.ones(1, 1, 2, 2), torch.zeros(1, 6), torch.eye(3).unsqueeze(0))
    with pytest.raises(RuntimeError):
        H.convex_upsample(torch.zeros(1, 1, 2, 2), torch.zeros(1, 576, 2, 2))


# every conv shape of the update blocks / heads / GRU (hd 64 and 128) and the
# parity tests, forward (rows=Cout, kch=Cin) and data gradient (rows=Cin, kch=Cout)
CONV_SHAPES = [  # (Cin, Cout, KH, KW)
    (160, 128, 1, 5), (160, 64, 1, 5), (160, 128, 5, 1), (160, 64, 5, 1),
    (320, 256, 1, 5), (320, 128, 1, 5), (320, 256, 5, 1), (320, 128, 5, 1),
    (128, 64, 1, 1), (64, 64, 3, 3), (1, 64, 7, 7), (6, 64, 7, 7), (128, 63, 3, 3), (128, 58, 3, 3),
    (64, 192, 3, 3), (64, 1, 3, 3), (128, 576, 1, 1), (64, 6, 3, 3), (128, 128, 3, 3), (128, 1, 3, 3),
    (256, 128, 3, 3), (128, 6, 3, 3), (128, 256, 3, 3), (256, 576, 1, 1), (48, 45, 5, 3), (128, 128, 3, 3),
    (1, 128, 7, 7), (6, 128, 7, 7),
]
IMAGES = [(2, 24, 80), (4, 24, 80), (2, 24, 40), (3, 7, 13), (1, 8, 12), (8, 30, 40), (16, 30, 40)]


def test_conv_plans_within_kernel_limits(lib):
    """Host-side launch plans respect the limits the kernels are written for
    (per-thread staging registers, LDS budget, K-half reduction buffer)."""
    import ctypes
    info = (ctypes.c_longlong * 16)()
    for Cin, Cout, KH, KW in CONV_SHAPES:
        for B, H, W in IMAGES:
            for rows, kch in ((Cout, Cin), (Cin, Cout)):
                assert lib.dro_conv2d_plan(rows, kch, KH, KW, B, H, W, info) == 0
                halo, bm, rt, pt, ks, cps, TH, TW, HWd, HPAD, tx, timg, CK, lds, part, kin = list(info)
                assert bm in (32, 64) and rt * bm >= rows and ks >= 1 and cps >= 1
                assert kin in (1, 2, 4) and (halo or kin == 1)
                assert bool(halo) == ((KH, KW) in ((1, 5), (5, 1), (3, 3), (1, 1)))
                if not halo:
                    continue
                T = KH * KW
                assert TH * TW == 64 and HWd == TW + KW - 1
                halo_n = (TH + KH - 1) * HWd
                assert halo_n <= 256 and HPAD >= halo_n and HPAD % 64 == 32
                assert (bm, CK) in ((32, 16), (32, 8), (64, 8), (64, 4), (32, 32), (64, 16))
                assert (bm * CK * T + 255) // 256 <= 16            # weight slots per thread
                odd = lambda n: n | 1
                stage = max(bm * odd(CK * T), CK * odd(bm * T)) + CK * HPAD
                assert lds == max(2 * stage * 4, 2 * 16 * 64 * 4) <= 64 * 1024
                # kin wave groups: one LDS region each (<= 160 KiB per block), and
                # room for the cross-group reduction (4 waves x 16 x 64 floats)
                assert lds * kin <= 160 * 1024 and (kin == 1 or lds >= 4 * 16 * 64 * 4)
                assert tx == -(-W // TW) and timg == -(-H // TH) * tx and pt == B * timg
                nck = -(-kch // CK)
                assert cps * ks >= nck and cps * (ks - 1) < nck
                if ks > 1:
                    assert part >= ks * rows * B * H * W * 4


def test_bn_fusion_arguments_rejected(lib):
    """ABI 10 (BN inside the 3x3 convs): argument checks before any launch."""
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert lib.dro_bn_state_bytes(2, 8, 8, 16) > 0
    assert lib.dro_bn_state_bytes(2, 8, 8, 5000) == 0                       # C >= 4096
    # NULL x / weight / out
    assert lib.dro_conv2d_bn_forward(None, 2, 8, 8, 4, p, 4, None, None, None, None, None, None, None, 0,
                                     None) == -1
    # in_state without in_y; skip without in_state
    assert lib.dro_conv2d_bn_forward(p, 2, 8, 8, 4, p, 4, p, None, None, None, None, p, p, 1 << 20, None) == -1
    assert lib.dro_conv2d_bn_forward(p, 2, 8, 8, 4, p, 4, None, p, None, None, None, p, p, 1 << 20, None) == -1
    assert lib.dro_conv2d_bn_forward(p, 0, 8, 8, 4, p, 4, None, None, None, None, None, p, p, 1 << 20, None) == -2
    # g with accumulation, and both gin_state and src_bn in one call
    gp = (ctypes.c_void_p * 7)(p.value, p.value, None, p.value, p.value, None, None)
    assert lib.dro_conv2d_bn_backward_data(p, 2, 8, 8, 4, 4, p, None, None, None, gp, p, p, 1, p, 1 << 20,
                                           None) == -3
    assert lib.dro_conv2d_bn_backward_data(p, 2, 8, 8, 4, 4, p, p, p, p, gp, p, p, 0, p, 1 << 20, None) == -3
    assert lib.dro_bn_apply(None, None, 1, 2, 4, 8, 8, p, p, None) == -1
    assert lib.dro_bn_apply(p, None, 2, 2, 4, 8, 8, p, p, None) == -3          # relu must be 0 / 1
    assert lib.dro_bn_backward_apply(p, None, 2, 4, 8, 8, p, p, None) == -1
