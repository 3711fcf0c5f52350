"""One ResNet encoder (fnet's configuration) forward + backward with random
input and output gradient: MIOpen stride-2 convs vs the native ones vs fp64
PyTorch on the CPU (same module, training-mode BN) -- per-parameter max-rel
errors and the input-gradient error.  Localises a native-path difference to
the encoder (or clears it).  usage: python tools/diag_encoder_ab.py"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dro_sfm_amd.networks.optim.extractor as ex  # noqa: E402


def _up2(x, _orig=ex.hip.bilinear_upsample2x):
    if x.is_cuda:
        return _orig(x)
    return torch.nn.functional.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def main():
    ex.hip.bilinear_upsample2x = _up2
    torch.manual_seed(0)
    enc = ex.ResNetEncoder(out_chs=128, stride=8)
    for B, H, W, cin in ((5, 64, 96, 3), (4, 64, 96, 6), (2, 192, 640, 3)):
        e0 = ex.ResNetEncoder(num_input_images=cin // 3, out_chs=128, stride=8)
        e0.load_state_dict({k: v for k, v in enc.state_dict().items() if not k.startswith("conv1.")}, strict=False)
        g = torch.Generator().manual_seed(B * H)
        x = torch.randn(B, cin, H, W, generator=g)
        ref_mod = copy.deepcopy(e0).double().train()
        xr = x.double().requires_grad_()
        yr = ref_mod(xr)
        G = torch.randn(yr.shape, generator=g)
        (yr * G.double()).sum().backward()
        refs = {k: p.grad for k, p in ref_mod.named_parameters()}
        for native in (False, True):
            ex.set_native_strided_convs(native)
            m = copy.deepcopy(e0).cuda().train()
            xd = x.cuda().requires_grad_()
            y = m(xd)
            (y * G.cuda()).sum().backward()
            torch.cuda.synchronize()
            ey = float((y.double().cpu() - yr.detach()).abs().max() / yr.detach().abs().max())
            ex_ = float((xd.grad.double().cpu() - xr.grad).abs().max() / xr.grad.abs().max())
            errs = sorted(((float((p.grad.double().cpu() - refs[k]).abs().max() / refs[k].abs().max()), k)
                           for k, p in m.named_parameters()), reverse=True)
            print(f"{(B, cin, H, W)} {'native' if native else 'miopen'}: y {ey:.2e} dx {ex_:.2e} worst "
                  + ", ".join(f"{k} {e:.2e}" for e, k in errs[:4]), flush=True)


if __name__ == "__main__":
    main()
