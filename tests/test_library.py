"""torch.library registration of the hot-path ops (SURVEY.md §8(b) "Native op
ABI"): every kernel entry point the drop-in modules
use is torch.ops.dro.<name> with a schema, a fake (meta) kernel and, where
differentiable, a registered autograd formula over a registered backward op.

CPU tests: the schemas, the fake kernels' shapes (FakeTensorMode, no device
needed) and the refusal of CPU tensors (no CPU fallback).  GPU tests:
torch.library.opcheck on real launches.
"""
import pytest
import torch

import dro_sfm_amd.hip  # noqa: F401  (registers the ops)

SCHEMAS = {
    "warp_cost": "dro::warp_cost(Tensor fmap, Tensor fmap_ref, Tensor depth, Tensor pose, Tensor K, Tensor ref_K, "
                 "SymInt depth_mode, float min_disp, float max_disp, float scale, SymInt pose_mode, bool reduce_mean, "
                 "Tensor? cells) -> Tensor",
    "view_synthesis": "dro::view_synthesis(Tensor ref_image, Tensor depth, Tensor pose, Tensor K, Tensor ref_K, "
                      "SymInt depth_mode, float min_disp, float max_disp, float scale, SymInt pose_mode, "
                      "Tensor? cells) -> Tensor",
    "plane_sweep": "dro::plane_sweep(Tensor fmap, Tensor fmap_ref, Tensor disp, Tensor pose, Tensor K, Tensor ref_K, "
                   "float min_disp, float max_disp, float scale, SymInt pose_mode) -> Tensor",
    "photometric_loss": "dro::photometric_loss(Tensor image, Tensor context, Tensor inv_depths, Tensor pose, "
                        "Tensor K, Tensor ref_K, SymInt pose_mode, float ssim_w, float C1, float C2, float smooth_w, "
                        "bool automask, bool reduce_min, float clip_loss, Tensor? cells, Tensor? l1_signs) -> "
                        "(Tensor, Tensor, Tensor)",
    "supervised_loss": "dro::supervised_loss(Tensor gt_inv, Tensor inv_depths, Tensor pose, Tensor gt_pose, Tensor K, "
                       "Tensor ref_K, SymInt pose_mode, float min_depth, float max_depth) -> (Tensor, Tensor)",
    "convex_upsample": "dro::convex_upsample(Tensor inv, Tensor mask, SymInt ratio, float add, float mul) -> Tensor",
    "convex_upsample_many": "dro::convex_upsample_many(Tensor[] invs, Tensor[] masks, SymInt ratio, float add, "
                            "float mul) -> Tensor",
    "conv2d": "dro::conv2d(Tensor[] srcs, Tensor weight, Tensor? bias, SymInt act, float alpha, Tensor[] params, "
              "SymInt nweight) -> Tensor",
    "conv2d_strided": "dro::conv2d_strided(Tensor x, Tensor weight, Tensor? bias, SymInt stride, SymInt pad, "
                      "SymInt act) -> Tensor",
    "sepconvgru_half": "dro::sepconvgru_half(Tensor h, Tensor wz, Tensor bz, Tensor wr, Tensor br, Tensor wq, "
                       "Tensor bq, Tensor[] xs, Tensor? wzr, Tensor? bzr) -> (Tensor, Tensor, Tensor, Tensor)",
    "pose_mean": "dro::pose_mean(Tensor y, Tensor? pose, float rot_scale) -> Tensor",
    "maxpool3x3s2": "dro::maxpool3x3s2(Tensor x) -> (Tensor, Tensor)",
    "bilinear_upsample2x": "dro::bilinear_upsample2x(Tensor x) -> Tensor",
}
BACKWARD_OPS = ["warp_cost_backward", "view_synthesis_backward", "photometric_loss_backward",
                "supervised_loss_backward", "convex_upsample_backward", "convex_upsample_many_backward",
                "conv2d_backward", "conv2d_strided_backward", "gru_backward_elem", "convgru_candidate_backward", "convgru_gates_backward",
                "pose_mean_backward",
                "maxpool3x3s2_backward", "bilinear_upsample2x_backward"]


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_schema(name):
    assert str(getattr(torch.ops.dro, name).default._schema) == SCHEMAS[name]


@pytest.mark.parametrize("name", BACKWARD_OPS)
def test_backward_op_registered(name):
    schema = str(getattr(torch.ops.dro, name).default._schema)
    assert schema.startswith(f"dro::{name}(")


def test_backward_ops_mutate_only_declared_buffers():
    """In-place gradient sinks and the cell test hook are declared mutations
    (Tensor(a!)) in the backward schemas; the forward ops mutate nothing."""
    bw = str(torch.ops.dro.warp_cost_backward.default._schema)
    assert "Tensor(a17!)? grad_fmap_out" in bw and "Tensor(a18!)? grad_fmap_ref_out" in bw and "!)? cells" in bw
    for name in SCHEMAS:
        assert "!" not in str(getattr(torch.ops.dro, name).default._schema), name


def test_fake_kernels_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        B, C, h, w, N = 2, 128, 24, 80, 2
        f, r = torch.empty(B, C, h, w), torch.empty(N, B, C, h, w)
        d, p, K = torch.empty(B, 1, h, w), torch.empty(N, B, 6), torch.empty(B, 3, 3)
        assert torch.ops.dro.warp_cost(f, r, d, p, K, K, 2, 0.0, 1.0, 0.125, 0, True, None).shape == (B, C, h, w)
        assert torch.ops.dro.warp_cost(f, r, d, p, K, K, 2, 0.0, 1.0, 0.125, 0, False, None).shape == (N, B, C, h, w)
        disp = torch.empty(64)
        assert torch.ops.dro.plane_sweep(f, f, disp, p[0], K, K, 0.0, 1.0, 0.125, 0).shape == (B, 64, C, h, w)
        img = torch.empty(N, B, 3, 192, 640)
        assert torch.ops.dro.view_synthesis(img, torch.empty(B, 1, 192, 640), p, K, K, 1, 0.0, 0.0, 1.0, 0,
                                            None).shape == img.shape
        inv, mask = torch.empty(B, 1, h, w), torch.empty(B, 576, h, w)
        assert torch.ops.dro.convex_upsample(inv, mask, 8, 0.0, 1.0).shape == (B, 1, 192, 640)
        assert torch.ops.dro.convex_upsample_many([inv] * 3, [mask] * 3, 8, 0.0, 1.0).shape == (3, B, 1, 192, 640)
        x, wgt = torch.empty(B, 160, h, w), torch.empty(128, 160, 1, 5)
        assert torch.ops.dro.conv2d([x], wgt, None, 0, 1.0, [], 0).shape == (B, 128, h, w)
        xs = torch.empty(B, 64, 96, 320)
        assert torch.ops.dro.conv2d_strided(xs, torch.empty(128, 64, 3, 3), None, 2, 1, 0).shape == (B, 128, 48, 160)
        hh = torch.empty(B, 64, h, w)
        outs = torch.ops.dro.sepconvgru_half(hh, *(torch.empty(64, 160, 1, 5), torch.empty(64)) * 3,
                                             [torch.empty(B, 96, h, w)], None, None)
        assert [o.shape[1] for o in outs] == [64, 128, 64, 64]
        assert torch.ops.dro.pose_mean(torch.empty(B, 6, h, w), None, 0.01).shape == (B, 6)
        y, arg = torch.ops.dro.maxpool3x3s2(torch.empty(B, 64, 96, 320))
        assert y.shape == (B, 64, 48, 160) and arg.dtype == torch.uint8
        assert torch.ops.dro.bilinear_upsample2x(torch.empty(B, 64, 6, 20)).shape == (B, 64, 12, 40)


def test_cpu_tensors_raise():
    """No CPU kernel: the ops refuse host tensors before anything launches."""
    B, C, h, w = 1, 8, 4, 6
    with pytest.raises(RuntimeError, match="ROCm device"):
        torch.ops.dro.warp_cost(torch.zeros(B, C, h, w), torch.zeros(1, B, C, h, w), torch.ones(B, 1, h, w),
                                torch.zeros(1, B, 6), torch.eye(3).expand(B, 3, 3), torch.eye(3).expand(B, 3, 3),
                                0, 0.0, 0.0, 0.125, 0, True, None)
    with pytest.raises(RuntimeError, match="ROCm device"):
        torch.ops.dro.conv2d([torch.zeros(B, C, h, w)], torch.zeros(4, C, 3, 3), None, 0, 1.0, [], 0)


@pytest.mark.gpu
def test_opcheck_on_device():
    """torch.library.opcheck (schema, fake tensor and autograd-registration
    tests) on real launches of the functional ops."""
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    B, C, h, w, N = 2, 16, 12, 20, 2
    K = torch.tensor([[40.0, 0, 9.5], [0, 40.0, 5.5], [0, 0, 1]]).repeat(B, 1, 1).to(dev)
    mk = lambda *s: torch.rand(*s, generator=g).to(dev)
    pose = (0.02 * torch.randn(N, B, 6, generator=g)).to(dev)
    tests = ("test_schema", "test_faketensor", "test_autograd_registration")
    torch.library.opcheck(torch.ops.dro.warp_cost.default,
                          (mk(B, C, h, w).requires_grad_(), mk(N, B, C, h, w).requires_grad_(),
                           (0.2 + mk(B, 1, h, w)).requires_grad_(), pose.clone().requires_grad_(), K, K,
                           1, 0.0, 0.0, 1.0, 0, True, None), test_utils=tests)
    torch.library.opcheck(torch.ops.dro.view_synthesis.default,
                          (mk(N, B, 3, 8 * h, 8 * w), (0.2 + mk(B, 1, 8 * h, 8 * w)).requires_grad_(),
                           pose.clone().requires_grad_(), K, K, 1, 0.0, 0.0, 1.0, 0, None), test_utils=tests)
    torch.library.opcheck(torch.ops.dro.convex_upsample.default,
                          (mk(B, 1, h, w).requires_grad_(), mk(B, 576, h, w).requires_grad_(), 8, 0.0, 1.0),
                          test_utils=tests)
    torch.library.opcheck(torch.ops.dro.pose_mean.default, (mk(B, 6, h, w).requires_grad_(), None, 0.01),
                          test_utils=tests)
    torch.library.opcheck(torch.ops.dro.plane_sweep.default,
                          (mk(B, C, h, w), mk(B, C, h, w), torch.linspace(0, 1, 8).to(dev), pose[0], K, K,
                           1 / 80, 2.0, 0.125, 0), test_utils=("test_schema", "test_faketensor"))
