"""fp32 accuracy of MIOpen conv / batchnorm vs fp64 CPU at the hot-path shapes."""
import torch, torch.nn.functional as F


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def conv_case(B, cin, cout, h, w, k, pad, stride=1):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, *k, generator=g) / (cin * k[0] * k[1]) ** 0.5
    bias = torch.randn(cout, generator=g)
    G = torch.randn(B, cout, (h + 2 * pad[0] - k[0]) // stride + 1, (w + 2 * pad[1] - k[1]) // stride + 1, generator=g)
    out = {}
    for dev, dt in (("cpu", torch.float64), ("cuda", torch.float32)):
        xx, ww, bb = (t.to(dev, dt).requires_grad_(True) for t in (x, wt, bias))
        y = F.conv2d(xx, ww, bb, stride=stride, padding=pad)
        (y * G.to(dev, dt)).sum().backward()
        out[dev] = (y, xx.grad, ww.grad, bb.grad)
    e = [rel(a, b) for a, b in zip(out["cuda"], out["cpu"])]
    print(f"conv B{B} {cin}->{cout} {h}x{w} k{k} s{stride}: y {e[0]:.1e} dx {e[1]:.1e} dw {e[2]:.1e} db {e[3]:.1e}", flush=True)


def bn_case(B, c, h, w, mean=3.0):
    g = torch.Generator().manual_seed(1)
    x = mean + torch.randn(B, c, h, w, generator=g)
    G = torch.randn(B, c, h, w, generator=g)
    wt, bias = 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    out = {}
    for dev, dt in (("cpu", torch.float64), ("cuda", torch.float32)):
        xx, ww, bb = (t.to(dev, dt).requires_grad_(True) for t in (x, wt, bias))
        y = F.batch_norm(xx, torch.zeros(c, device=dev, dtype=dt), torch.ones(c, device=dev, dtype=dt), ww, bb, training=True)
        (y * G.to(dev, dt)).sum().backward()
        out[dev] = (y, xx.grad, ww.grad, bb.grad)
    e = [rel(a, b) for a, b in zip(out["cuda"], out["cpu"])]
    print(f"bn B{B} c{c} {h}x{w} mean{mean}: y {e[0]:.1e} dx {e[1]:.1e} dw {e[2]:.1e} db {e[3]:.1e}", flush=True)


for case in [(2, 64, 64, 24, 80, (3, 3), (1, 1)), (2, 160, 128, 24, 80, (1, 5), (0, 2)), (4, 160, 64, 24, 80, (5, 1), (2, 0)),
             (2, 128, 576, 24, 80, (1, 1), (0, 0)), (6, 64, 64, 48, 160, (3, 3), (1, 1)), (2, 1, 64, 24, 80, (7, 7), (3, 3)),
             (6, 256, 128, 24, 80, (3, 3), (1, 1))]:
    conv_case(*case)
conv_case(6, 3, 64, 192, 640, (7, 7), (3, 3), 2)
conv_case(6, 64, 128, 48, 160, (3, 3), (1, 1), 2)
for c in [(6, 64, 96, 320, 0.5), (6, 128, 24, 80, 3.0), (2, 256, 12, 40, 10.0)]:
    bn_case(*c)
print("cudnn(miopen) enabled", torch.backends.cudnn.enabled)
torch.backends.cudnn.enabled = False
print("--- native (MIOpen disabled) ---")
conv_case(2, 64, 64, 24, 80, (3, 3), (1, 1))
conv_case(2, 160, 128, 24, 80, (1, 5), (0, 2))
bn_case(6, 128, 24, 80, 3.0)
