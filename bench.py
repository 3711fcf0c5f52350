#!/usr/bin/env python
"""Training-throughput benchmark: KITTI 192x640 multi-frame self-supervised.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Workload (BASELINE.json configs[1]): SelfSupModelMF +
DepthPoseNet('it8-seq4-inter-out', min_depth 0.5, max_depth 80), Adam lr 2e-4,
B=2 target frames per GPU, 2 context frames, 192x640, photometric loss with
automask + min reduction, flip_lr_prob 0.5 (the default).  Synthetic data of
that shape (smooth random textures, shifted context frames), random init.
A step = zero_grad -> forward -> loss -> backward -> RCCL all-reduce -> Adam.

Prints ONE JSON line on rank 0; `value` = images/s over all ranks (weak
scaling: per-GPU batch fixed).  Also reports the roofline of the dominant
kernel (HIP events) and the CPU-oracle baseline on this host's cores.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "training images/sec (KITTI 192x640 mf self-sup)"
KITTI_K = [[371.8, 0.0, 314.1], [0.0, 369.4, 88.5], [0.0, 0.0, 1.0]]
SCANNET_K = [[289.0, 0.0, 160.0], [0.0, 290.0, 120.0], [0.0, 0.0, 1.0]]
# BASELINE.json configs; `kitti_selfsup` (configs[1]) is the metric's workload and
# the default.  The others are single-GPU runs of configs[2] / the per-GPU shard of
# configs[4], reported with --workload.
WORKLOADS = {
    "kitti_selfsup": dict(name="KITTI 192x640 mf self-sup (configs[1])", kind="selfsup",
                          version="it8-seq4-inter-out", H=192, W=640, nref=2, batch=2, min_d=0.5,
                          max_d=80.0, K=KITTI_K,
                          metric="training images/sec (KITTI 192x640 mf self-sup)"),
    "scannet_sup": dict(name="ScanNet 240x320 view3 supervised (configs[2])", kind="sup",
                        version="it12-h-out", H=240, W=320, nref=2, batch=8, min_d=0.2, max_d=10.0,
                        K=SCANNET_K, metric="training images/sec (ScanNet 240x320 view3 sup)"),
    "scannet_selfsup5": dict(name="ScanNet 240x320 view5 self-sup, one rank of configs[4]",
                             kind="selfsup", version="it12-h-out", H=240, W=320, nref=4, batch=4,
                             min_d=0.2, max_d=10.0, K=SCANNET_K,
                             metric="training images/sec (ScanNet 240x320 view5 self-sup)"),
}
WL = dict(WORKLOADS["kitti_selfsup"])
VERSION = WL["version"]
H, W, NREF, MIN_D, MAX_D = WL["H"], WL["W"], WL["nref"], WL["min_d"], WL["max_d"]


def set_workload(name):
    global WL, VERSION, H, W, NREF, MIN_D, MAX_D
    WL = dict(WORKLOADS[name])
    VERSION = WL["version"]
    H, W, NREF, MIN_D, MAX_D = WL["H"], WL["W"], WL["nref"], WL["min_d"], WL["max_d"]


def loss_kw():
    return dict(ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4, C2=9e-4,
                photometric_reduce_op="min", disp_norm=True, clip_loss=0.0, progressive_scaling=0.0,
                padding_mode="zeros", automask_loss=True, num_scales=4, rotation_mode="euler",
                upsample_depth_maps=True, min_depth=MIN_D, max_depth=MAX_D,
                supervised_method="sparse-l1", supervised_num_scales=4)


HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def smooth_images(n, gen, device):
    lo = torch.rand(n, 3, H // 8, W // 8, generator=gen, device=device)
    up = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
    return (up + 0.1 * torch.rand(n, 3, H, W, generator=gen, device=device)).clamp(0, 1)


def _vec_to_mat(vec):
    """[B,6] (t, euler xyz) -> [B,4,4] (geometry/pose_utils.py:40-85)."""
    from dro_sfm_amd.geometry.pose import euler2mat
    T = torch.eye(4, device=vec.device).repeat(vec.shape[0], 1, 1)
    T[:, :3, :3] = euler2mat(vec[:, 3:])
    T[:, :3, 3] = vec[:, :3]
    return T


def make_batch(B, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    img = smooth_images(B, g, device)
    refs = []
    for j in range(NREF):
        shift = (-1) ** j * (2 + j)
        refs.append((0.97 * torch.roll(img, shift, 3) + 0.03 * smooth_images(B, g, device)).clamp(0, 1))
    K = torch.tensor(WL["K"], device=device).unsqueeze(0).repeat(B, 1, 1)
    batch = {"rgb": img, "rgb_context": refs, "rgb_original": img, "rgb_context_original": refs,
             "intrinsics": K, "_K0": K.clone()}
    if WL["kind"] == "sup":
        # dense GT depth U[min, max/4*1.2] (ScanNet-like) and GT context poses
        batch["depth"] = MIN_D + (MAX_D / 4 * 1.2 - MIN_D) * torch.rand(B, 1, H, W, generator=g,
                                                                         device=device)
        vec = torch.cat([0.1 * torch.randn(B, 3, generator=g, device=device),
                         0.01 * torch.randn(B, 3, generator=g, device=device)], 1)
        batch["pose_context"] = [_vec_to_mat((-1) ** j * vec) for j in range(NREF)]
    return batch


def raw_host_batch(batch, raw=(375, 1242)):
    """The synthetic batch as the data loader would hand it over before the
    GPU pipeline (datasets/gpu_loader.collate_decoded): decoded uint8 HWC
    frames at the KITTI raw size in pinned host memory, raw intrinsics."""
    def to_raw(t):
        up = torch.nn.functional.interpolate(t, size=raw, mode="bilinear", align_corners=False)
        u8 = (up.clamp(0, 1) * 255).round().to(torch.uint8).permute(0, 2, 3, 1).contiguous().cpu()
        return [f.pin_memory() for f in u8]
    K = batch["_K0"].detach().cpu().clone()
    K[:, 0] *= raw[1] / W
    K[:, 1] *= raw[0] / H
    return {"rgb": to_raw(batch["rgb"]), "rgb_context": [to_raw(c) for c in batch["rgb_context"]],
            "intrinsics": K}


def build_model(device, flip_prob):
    from dro_sfm_amd.networks.depth_pose.DepthPoseNet import DepthPoseNet
    if WL["kind"] == "sup":
        from dro_sfm_amd.models.SupModelMF import SupModelMF as Model
    else:
        from dro_sfm_amd.models.SelfSupModelMF import SelfSupModelMF as Model
    model = Model(flip_lr_prob=flip_prob, **loss_kw())
    model.add_depth_net(DepthPoseNet(version=VERSION, min_depth=MIN_D, max_depth=MAX_D))
    return model.to(device)


# ----------------------------------------------------------------------------- roofline
def roofline_photometric(B, device, iters=20):
    """Dominant custom kernel pair: the fused photometric loss (forward + backward)
    at the metric shape.  Algorithmic bytes per forward+backward launch pair (each
    input read once, each output written once):
      fwd: image 12 + context 12N + inv 4n + sel n   bytes/px
      bwd: image 12 + context 12N + inv 4n + sel n + grad_inv 4n bytes/px."""
    import dro_sfm_amd.hip as hip
    n = 9 if VERSION.startswith("it8") else 4
    g = torch.Generator(device=device)
    g.manual_seed(5)
    img = smooth_images(B, g, device)
    ctx = torch.stack([smooth_images(B, g, device) for _ in range(NREF)])
    # inverse depths as the net produces them: smooth fields upsampled from 1/8
    # resolution (per-pixel noise would scatter every warp's gathers)
    low = 0.02 + 0.3 * torch.rand(n * B, 1, H // 8, W // 8, generator=g, device=device)
    invs = torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear", align_corners=False)
    invs = invs.view(n, B, 1, H, W).contiguous().requires_grad_(True)
    pose = torch.cat([0.1 * torch.randn(NREF, n, B, 3, generator=g, device=device),
                      0.02 * torch.randn(NREF, n, B, 3, generator=g, device=device)], 3).requires_grad_(True)
    K = torch.tensor(WL["K"], device=device).unsqueeze(0).repeat(B, 1, 1)
    for _ in range(3):
        loss, _ = hip.photometric_loss(img, ctx, invs, pose, K)
        loss.backward()
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    fwd_ms = bwd_ms = 0.0
    for _ in range(iters):
        e0.record()
        loss, _ = hip.photometric_loss(img, ctx, invs, pose, K)
        e1.record()
        loss.backward()
        e2.record()
        torch.cuda.synchronize()
        fwd_ms += e0.elapsed_time(e1)
        bwd_ms += e1.elapsed_time(e2)
    fwd_ms, bwd_ms = fwd_ms / iters, bwd_ms / iters
    HW = H * W
    fwd_bytes = HW * B * (12 + 12 * NREF) + HW * B * n * 5
    bwd_bytes = HW * B * (12 + 12 * NREF) + HW * B * n * 9
    total_bytes = fwd_bytes + bwd_bytes
    achieved = total_bytes / ((fwd_ms + bwd_ms) * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "photometric fwd+bwd (photo_fwd_kernel + photo_bwd_kernel)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "note": "gather/latency-bound, not HBM-bound (profiles/r2_photometric_counters.json); the "
                    "backward's time depends on the min-selection (a ref unselected in a tile is skipped)",
            "algorithmic_bytes": int(total_bytes), "fwd_ms": round(fwd_ms, 4), "bwd_ms": round(bwd_ms, 4)}


def _event_loop(fn, iters, device):
    """Average ms of fn() over iters launches, HIP events on the launch stream."""
    stream = torch.cuda.current_stream(device)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def roofline_plane_sweep(device, D=64, B=2, C=128, iters=20):
    """D = 64 depth-hypothesis stress of configs[1]: one
    plane_sweep_lds_kernel launch (plane_sweep_wide_kernel for shapes the LDS
    kernel's 4-pixel vectors do not tile) builds the cost volume [B, D, C, h, w] of D
    fronto-parallel planes (disp = linspace(0, 1, D) through disp_to_depth) at
    the feature resolution.  Algorithmic bytes per launch: fmap + fmap_ref read
    once (2 * 4 * B*C*P) + the volume written once (4 * B*D*C*P)."""
    import dro_sfm_amd.hip as hip
    h, w = H // 8, W // 8
    g = torch.Generator(device=device)
    g.manual_seed(17)
    fmap = torch.randn(B, C, h, w, generator=g, device=device)
    fref = torch.randn(B, C, h, w, generator=g, device=device)
    disp = torch.linspace(0, 1, D, device=device)
    pose = torch.cat([0.1 * torch.randn(B, 3, generator=g, device=device),
                      0.01 * torch.randn(B, 3, generator=g, device=device)], 1)
    K = torch.tensor(WL["K"], device=device).unsqueeze(0).repeat(B, 1, 1)
    ms = _event_loop(lambda: hip.plane_sweep_cost(fmap, fref, disp, pose, K, min_depth=MIN_D,
                                                  max_depth=MAX_D), iters, device)
    P = h * w
    nbytes = 2 * 4 * B * C * P + 4 * B * D * C * P
    achieved = nbytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": f"plane_sweep_lds_kernel (D={D}, B={B}, C={C}, {h}x{w})",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "algorithmic_bytes": int(nbytes), "avg_launch_us": round(ms * 1e3, 2), "launches": iters}


def roofline_supervised(B, device, n=4, iters=20):
    """Fused supervised loss (csrc/supervised.hip) forward + backward at the
    workload shape.  Algorithmic bytes: fwd gt_inv + n inv maps read (4 + 4n per
    px), bwd the same plus n gradient maps written (4 + 8n per px)."""
    import dro_sfm_amd.hip as hip
    g = torch.Generator(device=device)
    g.manual_seed(19)
    gt = MIN_D + (MAX_D / 4 - MIN_D) * torch.rand(B, 1, H, W, generator=g, device=device)
    gt_inv = 1.0 / gt
    invs = (gt_inv.unsqueeze(0) + 0.02 * torch.randn(n, B, 1, H, W, generator=g, device=device))
    invs.requires_grad_(True)
    vec = torch.cat([0.1 * torch.randn(NREF, n, B, 3, generator=g, device=device),
                     0.01 * torch.randn(NREF, n, B, 3, generator=g, device=device)], 3)
    vec.requires_grad_(True)
    gtp = torch.stack([_vec_to_mat(vec[j, 0].detach() + 0.01) for j in range(NREF)])
    K = torch.tensor(WL["K"], device=device).unsqueeze(0).repeat(B, 1, 1)

    def fb():
        loss, _ = hip.supervised_loss(gt_inv, invs, vec, gtp, K, min_depth=MIN_D, max_depth=MAX_D)
        loss.backward()
    ms = _event_loop(fb, iters, device)
    HW = H * W
    nbytes = B * HW * ((4 + 4 * n) + (4 + 8 * n))
    achieved = nbytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "sup_loss_kernel fwd+bwd (+ finalize kernels)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "algorithmic_bytes": int(nbytes), "fwd_bwd_ms": round(ms, 4)}


# HBM bytes per launch of the roofline kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
# passes (tools/pmc_traffic.py; FETCH_SIZE doubled per MI355X_MICROARCH.md); used only
# when the file was measured on the same kernel(s) this build launches
def _latest_traffic_file():
    import glob
    import re
    files = glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                   "r*_roofline_traffic.json"))
    rnd = lambda f: int(re.search(r"r(\d+)_roofline", os.path.basename(f)).group(1))
    return max(files, key=rnd) if files else None


TRAFFIC_FILE = _latest_traffic_file()
# the roofline conv: the weight gradient of the feature encoder's layer1 3x3
# convolution at the KITTI metric shape (6 frames of 48x160, 64 -> 64)
RF_B, RF_C, RF_H, RF_W = 6, 64, 192 // 4, 640 // 4
MFMA_F32_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: dense f32 MFMA (v_mfma_f32_32x32x2_f32)


def roofline_kernels():
    """Names of the kernels one roofline call launches: the weight-gradient
    kernel and its split-sum finish (rocprof name prefixes)."""
    return ["wgrad2_kernel<3, 3, 0, true, 1>", "wgrad2_finish_kernel<"], None, None


def roofline_conv(device, iters=50, traffic_file=None):
    """Dominant kernel of the step: the conv engine's weight gradient
    (csrc/conv.hip wgrad2_kernel; the largest kernel class of the step,
    profiles/r3_bench_steady_state.txt), measured at its heaviest shape: the
    fnet layer1 3x3 conv (reference extractor.py:7-107 / torchvision
    BasicBlock) over the 6 frames of a KITTI metric batch (B=2 targets + 4
    refs, 48x160, 64 -> 64 channels), through the same entry point the
    trainer's in-place path uses (dro_conv2d_weight_grad_multi, one use):
    wgrad2_kernel<3,3,0,true,1> over 240 pixel splits + wgrad2_finish_kernel
    (fixed-order split sum into the weight gradient).  HIP events bracket both
    launches on the launch stream.  Algorithmic flops per call:
    2 * Cout * Cin * 9 * B*H*W."""
    import ctypes
    from dro_sfm_amd.hip import _lib
    from dro_sfm_amd.hip.conv import DroWgradUse, _slices
    lib = _lib.load()
    B, C, Hh, Ww = RF_B, RF_C, RF_H, RF_W
    kernels, _, _ = roofline_kernels()
    g = torch.Generator(device=device)
    g.manual_seed(11)
    x = torch.randn(B, C, Hh, Ww, generator=g, device=device)
    gout = torch.randn(B, C, Hh, Ww, generator=g, device=device)
    gw = torch.empty(C, C, 3, 3, device=device)
    sl = _slices([x])
    use = (DroWgradUse * 1)()
    use[0].srcs = ctypes.cast(sl, ctypes.c_void_p)
    use[0].dout = gout.data_ptr()
    use[0].y = None
    nb = int(lib.dro_conv2d_weight_grad_multi_workspace_bytes(1, B, Hh, Ww, C, C, 3, 3))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device)
    st = ctypes.c_void_p(stream.cuda_stream)

    def launch():
        _lib.check(lib.dro_conv2d_weight_grad_multi(use, 1, 1, B, Hh, Ww, C, 3, 3, 0, ctypes.c_float(1.0),
                                                    _lib.ptr(gw), None, 0, _lib.ptr(ws), nb, st),
                   "dro_conv2d_weight_grad_multi")
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    flops = 2.0 * C * C * 9 * B * Hh * Ww
    achieved = flops / (us * 1e-6) / 1e12
    traffic = None
    if traffic_file and os.path.exists(traffic_file):
        with open(traffic_file) as f:
            tf = json.load(f)
        if tf.get("kernels") == kernels:       # measured on this very launch sequence
            traffic = tf.get("hbm_bytes_per_launch")
    return {"bound": "mfma", "kernel": kernels[0] + " + " + kernels[1].rstrip("<") +
            " (fnet layer1 3x3 weight gradient, B=6 48x160, 64 -> 64)", "achieved": round(achieved, 2), "peak": MFMA_F32_PEAK_TFS,
            "unit": "TFLOP/s", "frac": round(achieved / MFMA_F32_PEAK_TFS, 4), "traffic": traffic,
            "flops_per_launch": int(flops), "avg_launch_us": round(us, 2), "launches": iters,
            "algorithmic_bytes_per_launch": int(4 * (x.numel() + gout.numel() + gw.numel()))}


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(model, budget_s=12.0, max_steps=40):
    """Reference algorithm on the host cores: the CPU oracle (a restatement of the
    reference's PyTorch path, pinned to its golden vectors) running the same
    training step -- forward, loss, backward, Adam -- on the same weights."""
    from oracle import dro_oracle as O
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    params = {k: v.detach().cpu().clone() for k, v in model.depth_net.state_dict().items()}
    leaves = []
    for k, v in params.items():
        if v.is_floating_point() and "running" not in k:
            v.requires_grad_(True)
            leaves.append(v)
    opt = torch.optim.Adam(leaves, lr=2e-4)
    B = WL["batch"]
    batch = make_batch(B, 1234, "cpu")
    times = []
    s = 0
    while s == 0 or (sum(times) < budget_s and len(times) < max_steps) or len(times) < 2:
        t0 = time.perf_counter()
        opt.zero_grad()
        out = O.train_step_loss(params, VERSION, MIN_D, MAX_D, batch, kind=WL["kind"], loss_kw={})
        out["loss"].sum().backward()
        opt.step()
        if s > 0:
            times.append(time.perf_counter() - t0)
        s += 1
    steps = len(times)
    sec = sum(times) / len(times)
    return {"value": round(B / sec, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{steps} timed steps (+1 warmup; ~{budget_s:.0f} s budget) of the full training "
                      f"step, B={B}, {H}x{W}, "
                      f"N={NREF}, {VERSION}, CPU oracle oracle/dro_oracle.py, torch {torch.__version__}",
            "sec_per_step": round(sec, 3), "sec_per_step_min_max": [round(min(times), 3), round(max(times), 3)],
            "cpu_model": _cpu_model(), "cpu_capability": torch.backends.cpu.get_cpu_capability(),
            "host_cpus": os.cpu_count(),
            "cores_note": f"cores = the CPUs in this process's affinity mask ({threads}; OMP_NUM_THREADS "
                          f"{os.environ.get('OMP_NUM_THREADS', 'unset')}), which the GPU box sets; the host "
                          f"has {os.cpu_count()}"}


def _cpu_model():
    """The host CPU's model name (/proc/cpuinfo, as lscpu prints it)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ----------------------------------------------------------------------------- launcher
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(argv, gpus, port):
    """The torch.distributed.run command that starts `gpus` ranks of this script
    (one process per GPU; each rank pins cuda:LOCAL_RANK)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def maybe_launch_ranks(argv, gpus):
    """`python bench.py --gpus N` without torchrun's env starts N ranks itself
    (the reference's `mpirun -np NGPUS`, run.sh:4; its dormant DP at
    horovod_trainer.py:66-69, model_wrapper.py:818-822).  Runs BEFORE anything
    touches the GPU in this process: the ranks are children (no exec), and this
    process exits with their launcher's status.  Returns None when this process
    is itself a rank (or N == 1)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != gpus:
            print(f"[bench] --gpus {gpus} but WORLD_SIZE={env_world}", file=sys.stderr, flush=True)
            return 2
        return None
    if gpus <= 1:
        return None
    import subprocess
    cmd = launch_command(argv, gpus, _free_port())
    print(f"[bench] launching {gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ))


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="kitti_selfsup",
                    help="BASELINE.json config (default: the metric's, configs[1])")
    ap.add_argument("--batch", type=int, default=None, help="target frames per GPU (default: the workload's)")
    ap.add_argument("--flip-prob", type=float, default=0.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--pipeline", choices=("resident", "gpu"), default="resident",
                    help="resident: float batches already in HBM (the metric's contract); gpu: every step "
                         "starts from decoded uint8 KITTI raw frames (375x1242) in pinned host memory and "
                         "runs the data pipeline (H2D, resize, colour jitter, to_tensor) on the GPU "
                         "(datasets/gpu_loader.py) inside the timed region")
    ap.add_argument("--miopen-strided-convs", action="store_true",
                    help="A/B: the encoders' stride-2 convs on MIOpen instead of the HIP engine")
    ap.add_argument("--miopen-encoder-convs", action="store_true",
                    help="A/B: the encoders' stride-1 3x3 convolutions on MIOpen instead of the HIP engine")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the roofline kernel loop (for rocprofv3 --stats / --pmc runs)")
    ap.add_argument("--roofline-iters", type=int, default=50)
    args = ap.parse_args()
    rc = maybe_launch_ranks(sys.argv[1:], args.gpus)
    if rc is not None:
        sys.exit(rc)
    set_workload(args.workload)
    if args.batch is None:
        args.batch = WL["batch"]
    if args.roofline_only:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        print(json.dumps({"roofline": roofline_conv(dev, args.roofline_iters, TRAFFIC_FILE)}), flush=True)
        return
    from dro_sfm_amd.networks.optim import extractor as _extractor
    _extractor.set_native_convs(not args.miopen_encoder_convs)
    _extractor.set_native_strided_convs(not args.miopen_strided_convs)

    from dro_sfm_amd.trainers.dp_trainer import (DataParallelTrainer, GraphedTrainStep,
                                                  init_distributed)
    # DRO_BENCH_DEVICE: every rank on this device (an N > 1 rehearsal on a
    # one-GPU box with DRO_DIST_BACKEND=gloo; never set by the driver)
    local = int(os.environ.get("DRO_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    rank, world, _ = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the process group has {world} ranks")
    torch.manual_seed(42)
    model = build_model(device, args.flip_prob)
    model.seed(42 + rank)
    trainer = DataParallelTrainer(model, lr=2e-4, bucket_mb=25.0, capturable=not args.eager)
    batches = [make_batch(args.batch, 1000 * rank + i, device) for i in range(4)]
    mode, stepper = "eager", None
    if not args.eager:
        try:
            stepper = GraphedTrainStep(trainer, batches[0], warmup=max(args.warmup, 2))
            mode = "hipgraph"
        except Exception as exc:  # keep measuring, but say so
            print(f"[bench] graph capture failed ({type(exc).__name__}: {exc}); running eager",
                  file=sys.stderr, flush=True)

    pipe, host_batches = None, None
    if args.pipeline == "gpu":
        from dro_sfm_amd.datasets.gpu_loader import GPUTrainPipeline
        pipe = GPUTrainPipeline((H, W), (0.2, 0.2, 0.2, 0.05), device=device,
                                generator=torch.Generator().manual_seed(7 + rank))
        host_batches = [raw_host_batch(b) for b in batches]

    def run(step_i):
        b = batches[step_i % len(batches)]
        if pipe is not None:
            b = pipe(host_batches[step_i % len(host_batches)])
        if stepper is not None:
            return stepper.step(b)
        if "_K0" in b:                       # the data loader hands a fresh K every step
            b["intrinsics"].copy_(b["_K0"])
        return trainer.step(b)

    for i in range(args.warmup):
        loss, _ = run(i)
    if not torch.isfinite(loss).all():
        raise RuntimeError(f"non-finite loss in warmup: {loss}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss, _ = run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    images = world * args.batch * args.steps
    result = {
        "metric": WL["metric"], "value": round(images / elapsed, 3), "unit": "images/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic" if args.pipeline == "resident" else
                "synthetic decoded uint8 375x1242 frames, GPU data pipeline in the timed region",
        "config": {"workload": WL["name"], "model": f"DepthPoseNet {VERSION}",
                   "global_batch": world * args.batch, "per_gpu_batch": args.batch, "ref_frames": NREF,
                   "image": [H, W], "parallelism": f"dp{world}", "flip_lr_prob": args.flip_prob,
                   "optimizer": "Adam lr 2e-4", "execution": mode,
                   "update_blocks": "depth block + pose block (side stream, with both context encoders)",
                   "encoder_3x3_s1": "miopen" if args.miopen_encoder_convs else "hip",
                   "encoder_strided": "miopen" if args.miopen_strided_convs else "hip",
                   "exchange": ("none (world 1)" if world == 1 else
                                "bucketed all-reduce in the step graph, overlapping backward"
                                if getattr(stepper, "in_graph", False) else
                                "all-reduce after each graph replay" if stepper is not None else
                                "bucketed all-reduce from backward hooks (eager)")},
        "final_loss": round(float(loss), 6),
    }
    if rank == 0 and not args.no_roofline:
        result["roofline"] = roofline_conv(device, args.roofline_iters, TRAFFIC_FILE)
        if WL["kind"] == "selfsup":
            result["roofline_photometric"] = roofline_photometric(args.batch, device)
        else:
            result["roofline_supervised"] = roofline_supervised(args.batch, device)
        if args.workload == "kitti_selfsup":
            result["roofline_plane_sweep"] = roofline_plane_sweep(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(model)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
