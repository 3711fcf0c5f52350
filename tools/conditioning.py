"""How well-conditioned is a full-size training step of the reference algorithm
(oracle/dro_oracle.py) on the parity tests' weights?  The fp32 oracle against
the fp64 oracle on the SAME branch (the fp64 run's bilinear cells forced in the
fp32 run) -- what any fp32 implementation can reach.  With `damp` the weights
first go through tests/golden/common.condition_params (the documented damping
of the update heads' output convolutions the full-size parity tests use).
CPU only (test infrastructure).

usage: python tools/conditioning.py kitti|sup_view3|selfsup_view5 [damp ...]
       python tools/conditioning.py golden it8|it12h [flip]     (the reference fixtures' inputs)
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import common as C  # noqa: E402
import test_hip_parity as T  # noqa: E402
from oracle import dro_oracle as O  # noqa: E402

T.DEV = "cpu"


def run(params, version, kind, mind, maxd, batch, dt, book, forced=None, flip=False):
    p = {k: (v.to(dt).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dt) if v.is_floating_point() else v)) for k, v in params.items()}
    b = {k: (v.clone().to(dt) if torch.is_tensor(v) and v.is_floating_point() else
             ([t.to(dt) for t in v] if isinstance(v, list) else v)) for k, v in batch.items()}
    out = O.train_step_loss(p, version, mind, maxd, b, kind=kind, cells=book, forced_selection=forced, flip=flip)
    out["loss"].sum().backward()
    return out, {k: v.grad for k, v in p.items() if getattr(v, "grad", None) is not None}


def main():
    case = sys.argv[1]
    flip = False
    if case == "golden":
        import grad_floor
        tag = sys.argv[2]
        flip = "flip" in sys.argv[3:]
        tag, version, kind, mind, maxd, batch = grad_floor.golden_case(
            tag, "it8-seq4-inter-out" if tag == "it8" else "it12-h-out", "selfsup" if tag == "it8" else "sup")
        batch = {k: (v.cpu().clone() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in batch.items()}
        damps = [1.0]
        case = f"golden {tag}{' flip' if flip else ''}"
    else:
        damps = [float(x) for x in sys.argv[2:]] or [1.0]
        tag, version, kind, mind, maxd, batch = T.full_size_case(case)
    spec = T.load_spec(os.path.join(T.G, f"depthposenet_{tag}_keys.json"))
    for damp in damps:
        params = C.condition_params(C.params_from_spec(spec), damp)
        t0 = time.time()
        rec = O.Cells(record=True)
        O.LAST_SELECTION.clear()
        o64, g64 = run(params, version, kind, mind, maxd, batch, torch.float64, rec, flip=flip)
        # the fp64 run's whole branch: cells, ReLU masks, pooling argmax, min-selection
        sel = torch.stack(list(O.LAST_SELECTION)) if kind == "selfsup" else None
        for k_ in list(O.PIN_STATS):
            O.PIN_STATS[k_] = 0
        o32, g32 = run(params, version, kind, mind, maxd, batch, torch.float32, O.Cells(forced=rec.as_forced()), sel,
                       flip=flip)
        per, l2 = T._grad_check_vs(g32, g64)
        worst = sorted(per.items(), key=lambda kv: -kv[1])[:3]
        print(f"{case} damp {damp:g}: loss {float(o64['loss']):.6f} rel {T.rel(o32['loss'], o64['loss']):.2e}  "
              f"gradient L2 {l2:.3e}  worst " + ", ".join(f"{k} {e:.2e}" for k, e in worst)
              + f"  pinned {dict(O.PIN_STATS)}  ({time.time() - t0:.0f} s)", flush=True)
        den = sum(float(g64[k].double().pow(2).sum()) for k in per)
        share = sorted(((float((g32[k].double() - g64[k].double()).pow(2).sum()) / den, k) for k in per), reverse=True)[:4]
        print("    L2^2 shares: " + ", ".join(f"{k} {v ** 0.5:.1e}" for v, k in share), flush=True)


if __name__ == "__main__":
    main()
