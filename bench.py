"""Throughput of the drop-in render_rays path on MI355X.

Default workload (``--config cfg2``, BASELINE.json configs[1]): one step = one
NeRFSystem.training_step of the reference (train.py:103-117) on synthetic
Blender-lego 400x400 rays: B=4096 rays per rank generated on the device from
the 100 camera poses of an orbit (nr_gen_rays; an epoch-shuffled permutation of
all 16M pixels, like the reference's shuffled DataLoader over its ray buffer,
with the target colours gathered in the same pass) -> render_rays (64 coarse +
128 fine, perturb=1, noise_std=1: opt.py defaults) -> MSE(coarse)+MSE(fine) ->
backward -> [RCCL all-reduce of the 4.77 MB gradient when N>1] -> Adam(lr=5e-4,
eps=1e-8) as one fused launch.  The backward of the split arithmetics runs over
the samples whose output gradient is nonzero (nr_active_samples, DESIGN.md 10:
the other samples add exact zeros, so the gradients are the every-sample
backward's up to the order of the split-K sums); the line's
``backward_samples`` reports the share listed per pass, and the rooflines of
the backward kernels count only those samples' work.

The other BASELINE.json configs are selectable (``--config``; the driver's
default run is cfg2):

* ``cfg3``: LLFF fern 504x378, forward-facing NDC rays (get_ndc_rays), 64 + 64
  samples, batch 4096, training step as above (train.py with llff, 20 poses);
* ``cfg4``: Blender lego 800x800, 64 + 128, batch 4096 per rank -- cfg2 at 800^2
  (the 8-GPU data-parallel config);
* ``cfg5``: shadow-mapping step of train_efficient_sm.py:143-199 at 128x128:
  sigma-only render of 512 camera rays (64 + 64, noise 0, with gradients), the
  whole 128x128 light image re-rendered every step (64 + 64 light importance,
  no_grad: sample_light_depth_every=1), efficient_sm (shadow_method_2), MSE,
  backward, Adam; camera batches in dataset order (its DataLoader has
  shuffle=False), light image replicated on every rank;
* ``eval``: eval.py's render of one 400x400 test view of cfg2's model
  (test_time=True, perturb=0, noise_std=0, chunks of 32768 rays).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).  ``value`` = rays/s over all ranks (camera rays
for cfg5).  The ``roofline`` object is for the dominant kernel, timed with HIP
events around each of its launches inside the timed region; ``cpu_baseline``
times the CPU oracle (the reference algorithm restated in PyTorch-CPU, pinned
to the reference by tests/golden) on a bounded sample of the same workload on
this host's cores.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# at least 8 HIP hardware queues, before the first HIP call (the GPU boxes
# export HIP's default of 4; nerf_pl_amd/__init__.py and DESIGN.md 15: with 4,
# RCCL's streams and the training step's three share queues and serialise)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP32_MFMA_PEAK_TF = 157.3          # MI355X_MICROARCH.md: fp32 matrix (= vector) peak
BF16_MFMA_PEAK_TF = 16 * FP32_MFMA_PEAK_TF   # dense bf16 MFMA (1/16 ratio, same guide)
# split-operand arithmetics: every fp32 product costs six bf16 (bf16x6) or three
# fp16 (f16x3; dense fp16 = dense bf16 rate) MFMA products -> fp32-equivalent ceiling
SPLIT_PRODUCTS = {"bf16x6": 6, "f16x3": 3, "bf16": 1}
HBM_PEAK_GBS = 8000.0
# algorithmic FLOP per sample: forward, data-grad, weight-grad
FLOP_FWD = 1_186_816
FLOP_FWD_SIGMA = 982_528
FLOP_DGRAD = 1_115_392
# the reference algorithm's weight-gradient FLOPs per sample (autograd's
# sum dz x^T of every layer) ...
FLOP_WGRAD_REF = 1_186_816
# ... and what the kernels execute: xyz_encoding_final's per-sample term
# (2 * 256 * 256, its input feat is not saved) is replaced by the per-launch
# products of nr_wgrad_dir_feat (G W_final^T and W_dir^T G, 2 x 2*128*256*256,
# plus W_dir^T db: DIRFEAT_FLOP), whose launches the rooflines time with it
FLOP_WGRAD = FLOP_WGRAD_REF - 2 * 256 * 256                     # 1,055,744
DIRFEAT_FLOP = 2 * (2 * 128 * 256 * 256) + 2 * 256 * 128       # 33,619,968 per launch
FLOP_TRAIN = FLOP_FWD + FLOP_DGRAD + FLOP_WGRAD_REF   # 3,489,024 (reference algorithm)
# sigma-only graph trained (cfg5): forward + weight-grad of the sigma-only
# layers, data-grad without the two PE inputs (layer 1 and layer 5's skip)
FLOP_TRAIN_SIGMA = 2 * FLOP_FWD_SIGMA + 2 * (FLOP_FWD_SIGMA // 2 - 2 * 63 * 256)
# weight gradient: algorithmic HBM bytes per sample (every saved segment read
# once).  The forward saves 2272 activation values per sample (PE 64, h1..h8,
# hdir 128, dir PE 32: xyz_encoding_final's output is not saved, the dir
# layer's feat columns come from h8), the backward 2180 gradient values
# (dz1..dz8, dz_dir, head 4: d feat is not saved either -- xyz_encoding_final's
# weight gradient is W_dir[:, :256]^T G with G = dz_dir^T h8, wgrad.hip task 10)
SAVED_VALUES = 2272
GRAD_VALUES = 2180
BYTES_WGRAD = 4 * (SAVED_VALUES + GRAD_VALUES)              # 17,808
# bf16 variant: every segment stored in bf16 except the 4-float head gradient
# (itself bf16 too: 8 B/sample) -> 2 * (2272 + 2180) = 8,904
BYTES_WGRAD_BF16 = 2 * (SAVED_VALUES + GRAD_VALUES)
# the sigma-only graph trained on its own kernels (rendering_shadows.py:167):
# data gradient without layer 1 and layer 5's PE columns; weight gradient of
# xyz_encoding_1..8 + sigma, reading PE, h1..h8, dz1..dz8 and the head once
FLOP_DGRAD_SIGMA = FLOP_FWD_SIGMA - 2 * 2 * 63 * 256             # 918,016
BYTES_WGRAD_SIGMA = 4 * (64 + 8 * 256 + 8 * 256 + 4)             # 16,656
KERNEL_FLOP = {"mlp_fwd": FLOP_FWD, "mlp_fwd_sigma": FLOP_FWD_SIGMA,
               "mlp_fwd_sigma_train": FLOP_FWD_SIGMA,
               # the deferred save's re-run over the listed samples (functions.DEFER_SAVE)
               "mlp_fwd_listed": FLOP_FWD, "mlp_fwd_sigma_listed": FLOP_FWD_SIGMA,
               "mlp_bwd_dgrad": FLOP_DGRAD, "mlp_bwd_dgrad_sigma": FLOP_DGRAD_SIGMA,
               "mlp_wgrad": FLOP_WGRAD, "mlp_wgrad_sigma": FLOP_FWD_SIGMA}
CONFIGS = ("cfg2", "cfg3", "cfg4", "cfg5", "eval")


def kernel_roofline(k, events, math_, traffic_json, extra=None):
    """Roofline of one MLP kernel from its largest (fine-pass) launches, timed
    with HIP events on the stream it runs on.  The weight gradient streams every
    saved segment once at 60 FLOP/B: HBM-bound (algorithmic bytes); the fused
    forward and data-gradient chains are MFMA-bound (algorithmic FLOPs of the
    fp32 products).  ``extra`` = (ms, FLOP) of a follow-up launch that belongs
    to each launch of this kernel (the weight gradient's nr_wgrad_dir_feat):
    its time and work are added to the launch's."""
    big = [(ev[0].elapsed_time(ev[1]), ev[2], active_samples(ev)) for ev in events]
    nmax = max(n for _, n, _ in big)
    durs = [t for t, n, _ in big if n == nmax]
    avg = sum(durs) / len(durs) + (extra[0] if extra else 0.0)
    # samples the fine-pass launches actually worked on (the backward skips
    # the blocks whose output gradient is exactly zero)
    nwork = sum(w for _, n, w in big if n == nmax) / len(durs)
    flops = KERNEL_FLOP[k]
    tflops = (flops * nwork + (extra[1] if extra else 0)) / (avg * 1e-3) / 1e12
    traffic, tsrc = None, None
    t = traffic_json.get(f"{math_}/{k}") or traffic_json.get(k)
    if t and int(t["samples"]) == nmax and t.get("arithmetic", math_) == math_:
        traffic = round(t["hbm_bytes"] / 1e9, 3)
        tsrc = f"{t.get('file', '?')} ({t['method']})"
    common = dict(kernel=k, traffic=traffic, traffic_unit="GB per launch", traffic_source=tsrc,
                  samples_per_launch=nmax, avg_launch_ms=round(avg, 4))
    if nwork != nmax:
        common["active_samples_per_launch"] = round(nwork, 1)
        common["active_basis"] = ("achieved counts the samples the backward worked on "
                                  "(nr_active_samples: those with a nonzero output gradient)")
    np_ = SPLIT_PRODUCTS.get(math_)
    peak = BF16_MFMA_PEAK_TF / np_ if np_ else FP32_MFMA_PEAK_TF
    # the weight gradient streams every saved segment once at 60 FLOP/B: below
    # the ridge (peak FLOP/s / 8 TB/s) of the split arithmetics, HBM-bound;
    # above the fp32 MFMA ridge (19.7 FLOP/B), MFMA-bound
    bps = BYTES_WGRAD_SIGMA if k == "mlp_wgrad_sigma" else BYTES_WGRAD
    if math_ == "bf16":
        bps //= 2
    if k.startswith("mlp_wgrad") and flops / bps < peak * 1e12 / (HBM_PEAK_GBS * 1e9):
        ach = bps * nwork / (avg * 1e-3) / 1e9
        return dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / HBM_PEAK_GBS, 4), bytes_per_sample=bps,
                    bytes_basis=(f"every saved activation ({SAVED_VALUES} values/sample) and gradient "
                                 f"({GRAD_VALUES} values/sample) segment read once, " if k == "mlp_wgrad"
                                 else "the sigma-only graph's saved PE, h1..h8, dz1..dz8 and "
                                      "head (4164 values/sample) read once, ")
                                + ("bf16" if math_ == "bf16" else "fp32"),
                    tflops_fp32_equiv=round(tflops, 2), **common)
    basis = {
        "bf16x6": "bf16x6: fp32 FLOPs on v_mfma_f32_16x16x32_bf16, six bf16 products per "
                  f"fp32 product -> ceiling = dense bf16 peak {BF16_MFMA_PEAK_TF:.0f} / 6",
        "f16x3": "f16x3: fp32 FLOPs on v_mfma_f32_16x16x32_f16, three fp16 products per "
                 f"fp32 product -> ceiling = dense fp16 peak {BF16_MFMA_PEAK_TF:.0f} / 3",
        "bf16": "bf16: one v_mfma_f32_16x16x32_bf16 product per product -> ceiling = dense "
                f"bf16 peak {BF16_MFMA_PEAK_TF:.0f}",
    }.get(math_, "fp32: v_mfma_f32_32x32x2_f32 dense peak")
    return dict(bound="mfma", achieved=round(tflops, 2), peak=round(peak, 1), unit="TFLOP/s",
                frac=round(tflops / peak, 4), flop_per_sample=flops, peak_basis=basis,
                **{("frac_of_fp32_mfma_peak" if math_ == "fp32" else "speed_vs_fp32_mfma_peak"):
                   round(tflops / FP32_MFMA_PEAK_TF, 4)}, **common)


def _math():
    from nerf_pl_amd import ops
    return ops.MATH


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=CONFIGS, default="cfg2",
                    help="BASELINE.json workload (cfg2 = the headline metric)")
    ap.add_argument("--batch", type=int, default=None, help="rays per rank per step")
    ap.add_argument("--img", type=int, default=None, help="image side (Blender configs)")
    ap.add_argument("--poses", type=int, default=100)
    ap.add_argument("--n-samples", type=int, default=None)
    ap.add_argument("--n-importance", type=int, default=None)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="budget of the CPU oracle sample (0 disables)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--light-shard", action="store_true",
                    help="cfg5 with N>1: render the light image sharded over the ranks and "
                         "all-gather the maps (SURVEY 8e phase 2) instead of on every rank")
    ap.add_argument("--grad-on-light", action="store_true",
                    help="cfg5: train_efficient_sm.py --grad_on_light (the mode 60 of the "
                         "reference's 63 launchers use): the light image rendered under "
                         "autograd every step, the shadow loss back-propagated into it")
    ap.add_argument("--light-importance", type=int, default=None,
                    help="cfg5: Light_N_importance (default 64; -1 = a random choice of "
                         "{0, 8, 16, 32} per step, train_efficient_sm.py:153-154, drawn from a "
                         "generator seeded alike on every rank)")
    ap.add_argument("--fp32-leg-steps", type=int, default=None,
                    help="after the timed region, time this many steps (after --warmup "
                         "untimed ones) with the exact fp32 MLP arithmetic "
                         "(v_mfma_f32_32x32x2_f32) for the fp32-MFMA roofline; default: "
                         "--steps; 0 disables")
    # the hot-path hyperparameters of opt.py:18-37 (same names, same meaning); None
    # keeps the workload's own default (cfg2-4: the opt.py defaults; cfg5: the
    # noise_std=0 of every train_efficient_sm launcher; eval: eval.py's 0/0)
    ap.add_argument("--perturb", type=float, default=None,
                    help="opt.py --perturb: factor to perturb depth sampling points")
    ap.add_argument("--noise-std", type=float, default=None,
                    help="opt.py --noise_std: std dev of the noise added to sigma")
    ap.add_argument("--lr", type=float, default=5e-4, help="opt.py --lr (Adam)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="one optimizer step after the whole backward (no coarse/fine "
                         "step pipelining, nerf_pl_amd/pipeline.py; env NR_BENCH_PIPELINE=0)")
    ap.set_defaults(pipeline=os.environ.get("NR_BENCH_PIPELINE", "1") != "0")
    ap.add_argument("--chunk", type=int, default=32 * 1024,
                    help="opt.py --chunk: the batch is rendered in chunks of this many rays "
                         "(NeRFSystem.forward, train.py:49-71), one render_rays call each")
    ap.add_argument("--use-disp", action="store_true",
                    help="opt.py --use_disp: sample linearly in inverse depth")
    ap.add_argument("--white-back", action="store_true",
                    help="the dataset's white_back (blender.py:21 sets it False; "
                         "blender_efficient_sm.py:22 True)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: --batch rays per rank (the driver's default); strong: --batch "
                         "rays per step in total, split over the ranks (SURVEY 8e)")
    ap.add_argument("--math", choices=("f16x3", "bf16x6", "fp32", "bf16"), default=None,
                    help="MLP arithmetic (default: $NERF_PL_AMD_MATH or f16x3); bf16 is "
                         "BASELINE configs[1]'s reduced-precision variant")
    a = ap.parse_args()
    if a.math:                      # read by nerf_pl_amd.ops at import
        os.environ["NERF_PL_AMD_MATH"] = a.math
    d = {"cfg2": (4096, 400, 64, 128), "cfg3": (4096, 504, 64, 64), "cfg4": (4096, 800, 64, 128),
         "cfg5": (512, 128, 64, 64), "eval": (32768, 400, 64, 128)}[a.config]
    a.batch = a.batch or d[0]
    a.img = a.img or d[1]
    a.n_samples = a.n_samples or d[2]
    a.n_importance = a.n_importance if a.n_importance is not None else d[3]
    if a.light_importance is None:
        a.light_importance = a.n_importance
    if a.fp32_leg_steps is None:
        a.fp32_leg_steps = a.steps
    if a.chunk <= 0:
        ap.error("--chunk must be positive")
    dflt = {"cfg5": (1.0, 0.0), "eval": (0.0, 0.0)}.get(a.config, (1.0, 1.0))
    a.perturb = dflt[0] if a.perturb is None else a.perturb
    a.noise_std = dflt[1] if a.noise_std is None else a.noise_std
    return a


def hyper(a):
    """the opt.py hyperparameters a workload line states"""
    return (f"perturb={a.perturb:g}, noise_std={a.noise_std:g}"
            + (", use_disp" if a.use_disp else "") + (", white_back" if a.white_back else "")
            + (f", chunk={a.chunk}" if a.chunk != 32 * 1024 else ""))


def render_chunked(render, models, emb, rays, a, S, I, test_time=False, **kw):
    """NeRFSystem.forward (train.py:49-71): render the batch in chunks of
    ``a.chunk`` rays, one render_rays call each, and concatenate the results."""
    B = rays.shape[0]
    if B <= a.chunk:
        return render(models, emb, rays, S, a.use_disp, a.perturb, a.noise_std, I, a.chunk,
                      a.white_back, test_time, **kw)
    parts = [render(models, emb, rays[i:i + a.chunk], S, a.use_disp, a.perturb, a.noise_std, I,
                    a.chunk, a.white_back, test_time, **kw) for i in range(0, B, a.chunk)]
    return {k: torch.cat([p[k] for p in parts], 0) for k in parts[0]}


class KernelTimer:
    """HIP events around every launch of the instrumented kernels (on the
    stream they are launched on: torch's current stream)."""

    def __init__(self):
        self.events = {}
        self.enabled = False

    def summary(self):
        out = {}
        for tag, lst in self.events.items():
            ms = [s.elapsed_time(e) for s, e, *_ in lst]
            out[tag] = dict(launches=len(lst), total_ms=sum(ms), avg_ms=sum(ms) / len(ms),
                            samples=sum(ev[2] for ev in lst) / len(lst))
            if any(ev[3] is not None for ev in lst):
                # the zero-gradient-block backward: samples of the listed blocks
                out[tag]["active_samples"] = sum(active_samples(ev) for ev in lst) / len(lst)
        return out


def active_samples(ev):
    """samples a launch worked on: all n, or for a *_active backward entry the
    samples nr_active_samples listed (read after the timed region)"""
    n, act = ev[2], ev[3]
    if act is None:
        return n
    sl, i = act
    return min(n, int(sl[i].item()))


def install_timers(timer):
    from nerf_pl_amd import _lib, ops

    def call_tag(name, *a):
        base = name[:-3] if name[-3:] in ("_x3", "_h3", "_b1") else name
        base = base[:-7] if base.endswith(("_active", "_listed")) else base
        if name.startswith("nr_mlp_fwd_listed"):   # a[5]: sigma_only
            return ("mlp_fwd_sigma_listed" if a[5] else "mlp_fwd_listed"), int(a[3])
        if base == "nr_mlp_fwd":
            if a[7]:     # sigma_only: inference, or the sigma-only training forward (save)
                return ("mlp_fwd_sigma_train" if a[9] else "mlp_fwd_sigma"), int(a[3])
            return "mlp_fwd", int(a[3])
        if base == "nr_mlp_bwd":
            return "mlp_bwd_dgrad", int(a[5])
        if base == "nr_mlp_bwd_sigma":
            return "mlp_bwd_dgrad_sigma", int(a[5])
        if base == "nr_wgrad":
            return "mlp_wgrad", int(a[2])
        if base == "nr_wgrad_sigma":
            return "mlp_wgrad_sigma", int(a[2])
        if name == "nr_adam_step":
            return "adam", 0
        return name[3:], 0

    orig_call = _lib.call
    import nerf_pl_amd.functions as F
    F.ACTIVE_LOG = []

    def timed_call(name, *a):
        if not timer.enabled:
            return orig_call(name, *a)
        tag, n = call_tag(name, *a)
        # a *_active backward entry: the block list functions.py just built
        act = F.ACTIVE_LOG[-1] if ("_active" in name or "_listed" in name) and F.ACTIVE_LOG \
            else None
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        orig_call(name, *a)
        e.record()
        timer.events.setdefault(tag, []).append((s, e, n, act))

    _lib.call = timed_call
    ops.call = timed_call
    import nerf_pl_amd.efficient_shadow_mapping as SM
    import nerf_pl_amd.functions as F
    import nerf_pl_amd.optim as OP
    import nerf_pl_amd.rays as R
    for m in (F, OP, SM, R):
        m.call = timed_call


# ---------------------------------------------------------------------------
# CPU baselines: the oracle (reference algorithm, PyTorch CPU) on a bounded
# sample of the same workload, on this host's cores
# ---------------------------------------------------------------------------
_CPU_THREADS = None      # set for the single-thread row


def host_cpus():
    """CPUs this process may run on: os.cpu_count() (the machine), the
    affinity mask, and the cgroup CPU quota (cpu.max) -- on the GPU boxes
    os.cpu_count() reports the whole machine (256) while the container is
    granted 16 CPUs of time, so 256 torch threads would only be throttled."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(total, aff, quota or total)
    return dict(os_cpu_count=total, affinity=aff, cgroup_quota=quota, usable=usable)


def _cpu_threads():
    t = _CPU_THREADS or host_cpus()["usable"]
    torch.set_num_threads(t)
    return t


def _timed_loop(fn, budget_s, min_iters=2):
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s and n >= min_iters:
            return n, el


def cpu_train(args, budget_s, rays_all, label):
    """Oracle training steps (render_rays fwd + bwd + Adam) on the workload's own
    batch (args.batch rays: 4096 at cfg2), at least 2 steps; the single-thread
    row times 256-ray batches (one 4096-ray step would take ~40 s
    on one core)."""
    from oracle import nerf_oracle as O
    threads = _cpu_threads()
    torch.manual_seed(0)
    b = 256 if threads == 1 else args.batch
    params = [{k: v.requires_grad_(True) for k, v in O.make_params(s).items()} for s in (1, 2)]
    opt = torch.optim.Adam([p for d in params for p in d.values()], lr=args.lr)

    def step():
        idx = torch.randint(0, rays_all.shape[0], (b,))
        res = render_chunked(lambda m, e, *r: O.render_rays(m, *r), params, None, rays_all[idx],
                             args, args.n_samples, args.n_importance)
        loss = O.mse_loss(res, torch.rand(b, 3))
        opt.zero_grad()
        loss.backward()
        opt.step()
    n, el = _timed_loop(step, budget_s)
    return dict(value=n * b / el, unit="rays/s", cores=threads, kind="port",
                host=host_cpus(),
                sample=f"{n} oracle training steps x {b} rays ({label}, {args.n_samples}+"
                       f"{args.n_importance} samples, perturb {args.perturb}, noise_std "
                       f"{args.noise_std}, fwd+bwd+Adam) in {el:.1f} s, torch CPU "
                       f"{threads} threads")


def cpu_eval(args, budget_s, rays_all):
    from oracle import nerf_oracle as O
    threads = _cpu_threads()
    b = 1024
    params = [O.make_params(s) for s in (1, 2)]
    pos = [0]

    def step():
        rays = rays_all[pos[0]:pos[0] + b]
        pos[0] = (pos[0] + b) % (rays_all.shape[0] - b)
        with torch.no_grad():
            render_chunked(lambda m, e, *r: O.render_rays(m, *r), params, None, rays, args,
                           args.n_samples, args.n_importance, True)
    n, el = _timed_loop(step, budget_s)
    return dict(value=n * b / el, unit="rays/s", cores=threads, kind="port",
                sample=f"{n} oracle test_time renders x {b} rays ({args.n_samples}+"
                       f"{args.n_importance}) in {el:.1f} s, torch CPU {threads} threads")


def cpu_shadow(args, budget_s, scene):
    """cfg5 on the CPU oracle, timed in two parts on bounded samples -- the
    camera part (sigma-only render of b rays + efficient_sm against a light
    map + MSE backward + Adam) and the light render (per ray: no_grad, or with
    autograd and its backward under --grad-on-light) -- then combined into the
    step rate of the full workload (512 camera rays + the whole light image per
    step)."""
    from oracle import nerf_oracle as O
    from oracle import shadow_oracle as SO
    threads = _cpu_threads()
    torch.manual_seed(0)
    params = [{k: v.requires_grad_(True) for k, v in O.make_params(s).items()} for s in (1, 2)]
    opt = torch.optim.Adam([p for d in params for p in d.values()], lr=args.lr)
    S, I, wh = args.n_samples, args.n_importance, args.img
    lrays = scene["light_rays"].cpu()
    lpix = scene["light_pixels"].cpu()
    leye, lcam = scene["light_eye"].cpu(), scene["light_cam"].cpu()
    bl = 256
    light_map = {"depth_coarse": torch.full((wh * wh,), 4.0), "depth_fine": torch.full((wh * wh,), 4.0)}

    LI = max(args.light_importance, 0) if args.light_importance != -1 else 16

    def light_part():
        # --grad_on_light: the light render under autograd and its backward
        with torch.set_grad_enabled(args.grad_on_light):
            res = SO.render_rays(params, lrays[:bl], S, args.use_disp, args.perturb,
                                 args.noise_std, LI, args.chunk, args.white_back)
        if args.grad_on_light:
            opt.zero_grad()
            sum(v.sum() for k, v in res.items() if k.startswith("depth")).backward()
    b = 64

    def cam_part():
        sel = torch.arange(b)
        rays = scene["rays_all"][sel].cpu()
        ppc = {"eye_pos": scene["eyes"][0].cpu().expand(b, 3),
               "camera": scene["mats"][0].cpu().expand(b, 3, 3)}
        res = SO.render_rays(params, rays, S, args.use_disp, args.perturb, args.noise_std, I,
                             args.chunk, args.white_back)
        out = SO.efficient_sm(scene["pixels"][sel].cpu(), lpix, res, light_map, ppc, leye, lcam,
                              (wh, wh), I > 0, LI > 0, "shadow_method_2")
        tgt = torch.rand(b, 3)
        loss = torch.mean((out["rgb_coarse"] - tgt) ** 2) + torch.mean((out["rgb_fine"] - tgt) ** 2)
        opt.zero_grad()
        loss.backward()
        opt.step()
    nc, elc = _timed_loop(cam_part, budget_s / 2)
    nl, ell = _timed_loop(light_part, budget_s / 2)
    t_cam, t_light = elc / (nc * b), ell / (nl * bl)
    t_step = args.batch * t_cam + wh * wh * t_light
    return dict(value=args.batch / t_step, unit="camera rays/s", cores=threads, kind="port",
                host=host_cpus(),
                sample=f"camera part {nc} x {b} rays in {elc:.1f} s, light render "
                       f"{'with autograd + backward ' if args.grad_on_light else ''}{nl} x {bl} "
                       f"rays in {ell:.1f} s (oracle, torch CPU {threads} threads), combined per "
                       f"step as {args.batch} camera rays + {wh * wh} light rays")


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
def _models(dev):
    from nerf_pl_amd import Embedding, NeRF
    torch.manual_seed(0)                      # identical initial weights on every rank
    models = [NeRF().to(dev), NeRF().to(dev)]
    return models, [Embedding(3, 10), Embedding(3, 4)]


def wl_nerf_train(args, dev, rank, ndc):
    """cfg2 / cfg4 (Blender) and cfg3 (LLFF NDC) training steps."""
    from nerf_pl_amd import render_rays
    from nerf_pl_amd.losses import MSELoss
    from nerf_pl_amd.rays import RaySampler, blender_focal, pose_spherical
    if ndc:
        W, H, focal, near, far = 504, 378, 407.0, 0.0, 1.0
        poses = []
        for k in range(20):                   # forward-facing: small translations, no rotation
            ang = 2 * math.pi * k / 20
            c2w = torch.eye(4)[:3].clone()
            c2w[:, 3] = torch.tensor([0.1 * math.cos(ang), 0.1 * math.sin(ang), 0.0])
            poses.append(c2w)
        poses = torch.stack(poses).to(dev)
    else:
        W = H = args.img
        focal, near, far = blender_focal(W), 1.0, 200.0   # datasets/blender.py:40-41
        poses = torch.stack([pose_spherical(-180.0 + 360.0 * k / args.poses, -30.0, 4.0)
                             for k in range(args.poses)]).to(dev)
    torch.manual_seed(1234)                   # the same target colours on every rank
    pool_rgb = torch.rand(poses.shape[0] * H * W, 3, device=dev)
    # one permutation per epoch shared by the ranks, rank r taking perm[r::world]
    # (DistributedSampler under Lightning DDP, train.py:89-94)
    world = dist.get_world_size() if dist.is_initialized() else 1
    sampler = RaySampler(poses, H, W, focal, near, far, rgb_pool=pool_rgb, ndc=ndc,
                         seed=99, rank=rank, world=world)
    models, emb = _models(dev)
    torch.manual_seed(4321 + rank)            # per-rank seeds of the in-kernel Philox draws
    S, I = args.n_samples, args.n_importance
    loss_fn = MSELoss()                       # losses.py:4-14 (train.py:107), one launch each way

    def step():
        rays, rgbs = sampler.next(args.batch)
        res = render_chunked(render_rays, models, emb, rays, args, S, I)
        return loss_fn(res, rgbs)

    hp = hyper(args)
    if ndc:
        name = "cfg3"
        metric = f"rays/sec ({S}c+{I}f) LLFF fern 504x378 NDC training step"
        work = (f"cfg3: LLFF fern 504x378 (20 forward-facing poses, focal 407), NDC rays "
                f"(near/far 0/1), {S} coarse + {I} fine, batch {args.batch} rays/rank, "
                f"{hp}, MSE coarse+fine, Adam lr {args.lr:g}")
        data = "synthetic (forward-facing NDC rays generated on device per batch, random target colours)"
    else:
        name = "cfg2" if args.img == 400 else f"cfg4" if args.img == 800 else f"blender{args.img}"
        metric = f"rays/sec ({S}c+{I}f) Blender-lego {W}^2 training step"
        work = (f"{name}: Blender lego {W}x{W}, {S} coarse + {I} fine, batch {args.batch} "
                f"rays/rank, {hp}, MSE coarse+fine, Adam lr {args.lr:g}")
        data = (f"synthetic (Blender-lego {W}x{W}, {args.poses}-pose camera orbit, rays generated "
                "on device per batch, random target colours, seeded default-init NeRF coarse+fine)")

    def cpu(budget):
        if ndc:
            from nerf_pl_amd.rays import llff_ndc_rays
            rays_all = llff_ndc_rays(504, 378, 4, 407.0)
        else:
            from nerf_pl_amd.rays import blender_rays
            rays_all = blender_rays(W, 1)
        return cpu_train(args, budget, rays_all, name)

    return dict(name=name, metric=metric, workload=work, data=data, step=step, train=True,
                pipeline_ok=I > 0, models=models, rays_per_step=args.batch, samples_per_ray=S + I,
                flop_per_ray=S * FLOP_TRAIN + (S + I) * FLOP_TRAIN, cpu=cpu)


def wl_eval(args, dev, rank):
    """eval.py:58-86 -- one test view rendered in chunks (test_time=True)."""
    from nerf_pl_amd import render_rays
    from nerf_pl_amd.rays import blender_focal, generate_rays, pose_spherical
    W = args.img
    models, emb = _models(dev)
    for m in models:
        m.requires_grad_(False)
    S, I = args.n_samples, args.n_importance
    poses = torch.stack([pose_spherical(-180.0 + 360.0 * k / 8, -30.0, 4.0) for k in range(8)]).to(dev)
    views = [generate_rays(poses[k:k + 1], W, W, blender_focal(W), 1.0, 200.0)
             for k in range(poses.shape[0])]
    it = [rank]

    def step():
        rays = views[it[0] % len(views)]
        it[0] += 1
        with torch.no_grad():
            for i in range(0, rays.shape[0], args.batch):
                render_chunked(render_rays, models, emb, rays[i:i + args.batch], args, S, I,
                               True)
        return None

    def cpu(budget):
        from nerf_pl_amd.rays import blender_rays
        return cpu_eval(args, budget, blender_rays(W, 1))

    return dict(name="eval", metric=f"rays/sec ({S}c+{I}f) Blender-lego {W}^2 test-view render",
                workload=f"eval: eval.py render of one {W}x{W} Blender-lego test view per step "
                         f"({W * W} rays, test_time=True: sigma-only coarse {S}, full fine "
                         f"{S + I}; {hyper(args)}, chunks of {args.batch} rays)",
                data="synthetic (Blender-lego camera orbit, seeded default-init NeRF coarse+fine)",
                step=step, train=False, models=models, rays_per_step=W * W,
                samples_per_ray=S + I, flop_per_ray=S * FLOP_FWD_SIGMA + (S + I) * FLOP_FWD,
                cpu=cpu)


def shadow_scene(wh, n_poses, dev):
    """datasets/blender_efficient_sm.py-style scene (as tests/golden/make_golden_shadow.py):
    a light camera on the sphere, n_poses camera poses, [i+.5, j+.5, 1] pixels."""
    from nerf_pl_amd.camera import Camera
    from nerf_pl_amd.rays import LEGO_CAMERA_ANGLE_X, blender_focal, generate_rays, pose_spherical
    focal = blender_focal(wh)
    hfov = LEGO_CAMERA_ANGLE_X * 180. / math.pi
    l2w = pose_spherical(35.0, -55.0, 4.0)
    light = Camera(hfov, (wh, wh))
    light.set_pose_using_blender_matrix(l2w, False)
    jj, ii = torch.meshgrid(torch.arange(wh), torch.arange(wh), indexing="ij")
    pixels = torch.stack([ii + 0.5, jj + 0.5, torch.ones_like(ii, dtype=torch.float32)], -1)
    pixels = pixels.reshape(-1, 3).float().to(dev)
    c2ws, eyes, mats = [], [], []
    for k in range(n_poses):
        c2w = pose_spherical(-180.0 + 360.0 * k / n_poses, -30.0, 4.0)
        cam = Camera(hfov, (wh, wh))
        cam.set_pose_using_blender_matrix(c2w, False)
        c2ws.append(c2w)
        eyes.append(cam.eye_pos)
        mats.append(cam.camera)
    c2ws = torch.stack(c2ws).to(dev)
    return dict(light_rays=generate_rays(l2w.reshape(1, 3, 4).to(dev), wh, wh, focal, 1.0, 200.0),
                light_pixels=pixels, light_eye=light.eye_pos.float(), light_cam=light.camera.float(),
                light=light, c2ws=c2ws, eyes=torch.stack(eyes).float().to(dev),
                mats=torch.stack(mats).float().to(dev), pixels=pixels, focal=focal,
                rays_all=generate_rays(c2ws[:1], wh, wh, focal, 1.0, 200.0))


def wl_shadow(args, dev, rank):
    """cfg5: train_efficient_sm.py:139-208 (sample_light_depth_every=1)."""
    import numpy as np
    from nerf_pl_amd import rendering_shadows as RS
    from nerf_pl_amd.losses import MSELoss
    from nerf_pl_amd.rays import generate_rays
    wh, S, I, B = args.img, args.n_samples, args.n_importance, args.batch
    LI = args.light_importance
    scene = shadow_scene(wh, args.poses, dev)
    models, emb = _models(dev)
    torch.manual_seed(4321 + rank)
    hw = wh * wh
    total = args.poses * hw
    pos = [(rank * B) % total]
    tgt_pool = torch.rand(total, 3, device=dev)
    light_ppc = {"eye_pos": scene["light_eye"], "camera": scene["light_cam"]}
    loss_fn = MSELoss()                       # train_efficient_sm.py's loss_dict['mse']
    from nerf_pl_amd.losses import OpactiyLoss
    opacity_fn = OpactiyLoss()                # :43, evaluated (logged, not trained) at :191
    # Light_N_importance == -1: np.random.choice([0, 8, 16, 32]) per light render
    # (:153-154); one generator seeded alike on every rank keeps the ranks'
    # light renders the same shape (the sharded render gathers them)
    li_rng = np.random.RandomState(2024)
    shard = args.light_shard and dist.is_initialized() and dist.get_world_size() > 1

    def step():
        # dataset order (shuffle=False): B consecutive pixels of one view
        sel = torch.arange(pos[0], pos[0] + B, device=dev)
        pos[0] = (pos[0] + B * max(1, dist.get_world_size() if dist.is_initialized() else 1)) % total
        rays = generate_rays(scene["c2ws"], wh, wh, scene["focal"], 1.0, 200.0, sel)
        pose = sel // hw
        ppc = {"eye_pos": scene["eyes"][pose], "camera": scene["mats"][pose]}
        cam = render_chunked(RS.render_rays, models, emb, rays, args, S, I)
        li = int(li_rng.choice([0, 8, 16, 32])) if LI == -1 else LI
        # --grad_on_light renders the light under autograd (:158-162), else no_grad (:164-168)
        with torch.set_grad_enabled(args.grad_on_light):
            if shard:
                light = RS.render_rays_sharded(models, emb, scene["light_rays"], S,
                                               args.use_disp, args.perturb, args.noise_std, li,
                                               args.chunk, args.white_back)
            else:
                light = render_chunked(RS.render_rays, models, emb, scene["light_rays"], args, S,
                                       li, were_gradients_computed=False)
        out = RS.efficient_sm(scene["pixels"][sel % hw], scene["light_pixels"], cam, light, ppc,
                              light_ppc, (wh, wh), I > 0, li > 0, "shadow_method_2")
        tgt = tgt_pool[sel]
        with torch.no_grad():                 # log['train/train_opactiy'] (:191-195)
            opacity_fn(light, tgt)
        return loss_fn(out, tgt)

    lname = "random {0,8,16,32}" if LI == -1 else str(LI)
    # light samples per light ray: coarse S, plus S + li fine when li > 0
    lis = [0, 8, 16, 32] if LI == -1 else [LI]
    light_samples = S + sum((S + li) if li > 0 else 0 for li in lis) / len(lis)
    gol = args.grad_on_light
    return dict(name="cfg5",
                metric=f"camera rays/sec shadow-mapping step ({S}c+{I}f, {wh}^2 light image "
                       f"re-rendered per step{', --grad_on_light' if gol else ''})",
                workload=f"cfg5: train_efficient_sm.py step at {wh}x{wh}: sigma-only render of "
                         f"{B} camera rays/rank ({S}+{I}, {hyper(args)}, with gradients) + "
                         f"{'autograd' if gol else 'no_grad'} render of the {hw}-ray light image "
                         f"({S}+{lname}"
                         f"{', sharded over the ranks + all-gather' if args.light_shard else ''}) + efficient_sm "
                         "(shadow_method_2, per-pose runs) + MSE + backward"
                         " + the logged OpactiyLoss"
                         f"{' (through the light render too)' if gol else ''} + Adam lr "
                         f"{args.lr:g}",
                data=f"synthetic ({args.poses}-pose camera orbit + one light camera, rays "
                     "generated on device, random targets, seeded default-init NeRF pair)",
                step=step, train=True, models=models, rays_per_step=B,
                samples_per_ray=S + I,
                flop_per_ray=(S + (S + I)) * FLOP_TRAIN_SIGMA
                + hw / B * light_samples * (FLOP_TRAIN_SIGMA if gol else FLOP_FWD_SIGMA),
                cpu=lambda budget: cpu_shadow(args, budget, scene))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters when rehearsing N ranks on
    # fewer GPUs (NR_BENCH_DIST_BACKEND=gloo: RCCL refuses two ranks on one GPU)
    local %= max(1, torch.cuda.device_count())
    backend = os.environ.get("NR_BENCH_DIST_BACKEND", "nccl")
    # NR_BENCH_FORCE_DIST=1: the distributed path (process group, hook-launched
    # gradient all-reduce, barriers, max-over-ranks timing) at one rank too --
    # a real-RCCL rehearsal of the driver's N-GPU run on a one-GPU box
    use_dist = world > 1 or os.environ.get("NR_BENCH_FORCE_DIST") == "1"
    t_start = time.perf_counter()

    def progress(msg):
        """one short line per phase on stderr from every rank of a distributed
        run (the JSON line stays rank 0's only stdout): a multi-rank run is
        never silent for long, and a hang names its phase and rank"""
        if use_dist:
            print(f"[bench rank {rank}/{world} +{time.perf_counter() - t_start:.1f}s] {msg}",
                  file=sys.stderr, flush=True)

    if use_dist and os.environ.get("NR_BENCH_WATCHDOG"):
        # NR_BENCH_WATCHDOG=<s>: every rank dumps all its threads' Python stacks
        # to stderr every <s> seconds (a hung multi-rank run names where it waits)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["NR_BENCH_WATCHDOG"]), repeat=True,
                                          file=sys.stderr)
    if use_dist:
        torch.cuda.set_device(local)
        progress(f"init_process_group({backend})")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        progress("process group up")
    if args.scaling == "strong":
        if args.batch % world:
            raise SystemExit(f"--scaling strong: batch {args.batch} not divisible by {world} ranks")
        args.batch //= world
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from nerf_pl_amd.optim import FusedAdam

    timer = KernelTimer()
    F_ = None
    if not args.no_kernel_timing:
        install_timers(timer)
        import nerf_pl_amd.functions as F_

    if args.config == "eval":
        wl = wl_eval(args, dev, rank)
    elif args.config == "cfg5":
        wl = wl_shadow(args, dev, rank)
    else:
        wl = wl_nerf_train(args, dev, rank, ndc=args.config == "cfg3")

    opt, reducer, pstep = None, None, None
    if wl["train"]:
        params = [p for m in wl["models"] for p in m.parameters()]
        if not (args.pipeline and wl.get("pipeline_ok")):
            opt = FusedAdam(params, lr=args.lr, eps=1e-8)
        if use_dist:
            from nerf_pl_amd.distributed import GradAllReducer
            # one bucket per model: the fine model's all-reduce overlaps the
            # coarse model's backward
            # collectives issued after the backward is enqueued (hook_launch=False):
            # one issued from a gradient hook held autograd's thread until its
            # input was computed, serialising the two backward chains
            reducer = GradAllReducer(params, buckets=[list(m.parameters()) for m in wl["models"]],
                                     hook_launch=False)
            # first collective on the main thread: the communicator is set up
            # here, not inside the first gradient hook (autograd's thread)
            dist.barrier()
            progress("first collective done")
        if opt is None:
            # the coarse model's Adam and the next step's coarse pass beside
            # the fine model's backward tail (nerf_pl_amd/pipeline.py)
            from nerf_pl_amd.pipeline import PipelinedStep
            pstep = PipelinedStep(wl["models"], lr=args.lr, eps=1e-8, reducer=reducer)

    first = [use_dist]

    def step():
        from nerf_pl_amd import rendering as _r
        if pstep is not None and _r.FINE_STREAM:
            loss = pstep(wl["step"])
            if first[0]:
                torch.cuda.synchronize()
                progress("first step (pipelined) done")
            first[0] = False
            return loss
        loss = wl["step"]()
        if first[0]:
            torch.cuda.synchronize()
            progress("first step: forward done")
        if pstep is not None:    # the serialised pass: the same optimizers, one stream
            pstep.opt_c.zero_grad(set_to_none=True)
            pstep.opt_f.zero_grad(set_to_none=True)
            loss.backward()
            if reducer is not None:
                reducer()
            pstep.opt_c.step()
            pstep.opt_f.step()
        elif opt is not None:
            opt.zero_grad(set_to_none=True)
            loss.backward()
            if first[0]:
                torch.cuda.synchronize()
                progress("first step: backward done")
            if reducer is not None:
                reducer()            # waits for the RCCL all-reduces of the 4.77 MB gradient
            if first[0]:
                progress("first step: gradient all-reduce done")
            opt.step()
        first[0] = False
        return loss

    def run(steps, warmup, what="main"):
        """warmup untimed steps, then `steps` timed ones between barriers;
        (seconds = max over ranks, last loss)."""
        loss = None
        for i in range(warmup):
            step()
            if i == 0:
                torch.cuda.synchronize()
                progress(f"{what}: first warmup step done")
        if pstep is not None:
            pstep.flush()        # a deferred fine update (distributed path)
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        progress(f"{what}: {warmup} warmup steps done, timing {steps}")
        timer.events = {}
        if F_ is not None:
            F_.ACTIVE_LOG = []
        # the timed region's time origin on the device: every kernel event's
        # offset from it places launches of both streams on one clock (the
        # MLP stage's busy time is the union of its launches' intervals)
        timer.ref = torch.cuda.Event(enable_timing=True)
        timer.ref.record()
        timer.enabled = True
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step()
        if pstep is not None:
            pstep.flush()        # the last step's deferred fine update is part of it
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        timer.enabled = False
        if use_dist:
            t = torch.tensor([el], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        progress(f"{what}: timed region done ({el / max(steps, 1) * 1e3:.2f} ms/step)")
        return el, loss

    def rooflines(math_, ms, steps):
        fp32_key = "frac_of_fp32_mfma_peak" if math_ == "fp32" else "speed_vs_fp32_mfma_peak"
        ks = timer.summary()
        roof, roofs, stage = None, {}, None
        if ks:
            tj = {}
            for rel in ("profiles/r06/traffic.json", "profiles/r05/late/traffic.json",
                        "profiles/r05/traffic.json"):
                tf = os.path.join(REPO, rel)
                if os.path.exists(tf):
                    tj = {k: dict(v, file=rel) for k, v in json.load(open(tf)).items()
                          if isinstance(v, dict)}
                    break
            # nr_wgrad_dir_feat finishes every full-graph weight gradient (one
            # launch each): its average launch is part of mlp_wgrad's
            df = ks.get("wgrad_dir_feat")
            for k in KERNEL_FLOP:
                if k in ks:
                    roofs[k] = kernel_roofline(k, timer.events[k], math_, tj,
                                               extra=(df["avg_ms"], DIRFEAT_FLOP)
                                               if k == "mlp_wgrad" and df else None)
                    if k == "mlp_wgrad" and df:
                        roofs[k]["includes"] = "nr_wgrad_dir_feat (one launch per weight gradient)"
            if roofs:
                dom = max(roofs, key=lambda k: ks[k]["total_ms"])
                roof = roofs[dom]
                ks[dom]["share_of_step"] = ks[dom]["total_ms"] / (ms * steps)
                # the MLP stage (every fused MLP launch: forward, data and weight
                # gradients) against the fp32 MFMA peak -- the north star's ratio
                fl = sum(KERNEL_FLOP[k] * active_samples(ev) for k in roofs for ev in timer.events[k])
                t = sum(ks[k]["total_ms"] for k in roofs)
                if df and "mlp_wgrad" in roofs:
                    fl += DIRFEAT_FLOP * df["launches"]
                    t += df["total_ms"]
                # the fine pass's backward runs on its own stream beside the
                # coarse pass's (rendering.FINE_STREAM): the stage's time is the
                # union of its launches' intervals on the device clock, not the
                # sum of their (overlapping) durations
                iv = sorted((timer.ref.elapsed_time(ev[0]), timer.ref.elapsed_time(ev[1]))
                            for k in list(roofs) + (["wgrad_dir_feat"] if df else [])
                            for ev in timer.events[k])
                busy, cur = 0.0, None
                for a0, a1 in iv:
                    if cur is None or a0 > cur[1]:
                        if cur is not None:
                            busy += cur[1] - cur[0]
                        cur = [a0, a1]
                    else:
                        cur[1] = max(cur[1], a1)
                if cur is not None:
                    busy += cur[1] - cur[0]
                t_sum, t = t, busy
                tf_ = fl / (t * 1e-3) / 1e12
                stage = dict(kernels=sorted(roofs) + (["wgrad_dir_feat"] if df else []),
                             flop_per_step=int(fl / steps), ms_per_step=round(t / steps, 4),
                             launch_ms_sum_per_step=round(t_sum / steps, 4),
                             time_basis="union of the launches' intervals (HIP events, one clock; "
                                        "the two passes' backward launches overlap)",
                             share_of_step=round(t / (ms * steps), 4),
                             tflops_fp32_equiv=round(tf_, 2),
                             fp32_mfma_peak=FP32_MFMA_PEAK_TF,
                             **{fp32_key: round(tf_ / FP32_MFMA_PEAK_TF, 4)})
        return ks, roof, roofs, stage

    el, loss = run(args.steps, args.warmup)
    ms = el / args.steps * 1e3
    rays_per_s = wl["rays_per_step"] * world * args.steps / el
    math_main = _math()
    ks, roof, roofs, stage = rooflines(math_main, ms, args.steps)

    # the split arithmetics' backward skips the samples whose output gradient
    # is exactly zero (nr_active_samples): the share it worked on, per launch
    # size (coarse / fine pass), over the timed steps
    from nerf_pl_amd import functions as _functions
    backward_blocks = dict(skip_zero_gradient_samples=bool(_functions.ACTIVE_SAMPLES
                                                           and math_main in _functions.ACTIVE_ARITHS),
                           deferred_save=_functions.DEFER_SAVE,
                           deferred_save_threshold=_functions.DEFER_AUTO)
    for k in ("mlp_bwd_dgrad", "mlp_bwd_dgrad_sigma"):
        evs = timer.events.get(k, [])
        if evs and any(ev[3] is not None for ev in evs):
            by_n = {}
            for ev in evs:
                by_n.setdefault(ev[2], []).append(active_samples(ev) / ev[2])
            backward_blocks[k] = {f"samples_{n}": round(sum(v) / len(v), 4)
                                  for n, v in sorted(by_n.items())}
    # per-kernel rooflines with the two passes serialised: in the timed region
    # the fine pass's backward launches share the GPU with the coarse pass's
    # (rendering.FINE_STREAM), so their HIP-event durations there are wall
    # times under contention ("rooflines_concurrent"); a short pass on one
    # stream gives each kernel's own launch time ("rooflines")
    roofs_conc, roofs_iso = roofs, None
    from nerf_pl_amd import rendering as _rendering
    if wl["train"] and ks and _rendering.FINE_STREAM:
        _rendering.FINE_STREAM = False
        try:
            el_i, _ = run(10, 3, "serialised kernels")
        finally:
            _rendering.FINE_STREAM = True
        _, roof_i, roofs_iso, _ = rooflines(math_main, el_i / 10 * 1e3, 10)
        # the dominant kernel by its own launch time; a backward kernel (it
        # overlaps the other pass's backward in the timed region, where its
        # HIP-event duration includes waiting for CUs) is reported from the
        # serialised pass, a forward kernel (never overlapped) from the timed
        # region as before
        if roof_i is not None:
            dk = roof_i.get("kernel")
            if dk in roofs and not dk.startswith("mlp_bwd") and dk != "mlp_wgrad" and "wgrad" not in dk:
                roof = roofs[dk]
            else:
                roof = dict(roof_i, basis="serialised pass (in the timed region this backward kernel "
                                          "shares the GPU with the other pass's backward)")
    # exact-fp32 leg: the same workload on v_mfma_f32_32x32x2_f32 (fp32
    # products, no operand splitting) -- its own roofline against the fp32
    # MFMA peak, next to the default arithmetic's
    fp32_leg = None
    if args.fp32_leg_steps > 0 and math_main != "fp32":
        from nerf_pl_amd import ops as _ops
        _ops.MATH = "fp32"
        try:
            el32, _ = run(args.fp32_leg_steps, args.warmup, "fp32 leg")
        finally:
            _ops.MATH = math_main
        ms32 = el32 / args.fp32_leg_steps * 1e3
        ks32, roof32, roofs32, stage32 = rooflines("fp32", ms32, args.fp32_leg_steps)
        fp32_leg = dict(dtype="fp32", mlp_arithmetic="fp32 (v_mfma_f32_32x32x2_f32: exact fp32 "
                        "products, fp32 accumulation)", steps=args.fp32_leg_steps, warmup=args.warmup,
                        value=round(wl["rays_per_step"] * world * args.fp32_leg_steps / el32, 1),
                        unit="rays/s", ms_per_step=round(ms32, 3), roofline=roof32,
                        rooflines=roofs32, mlp_stage=stage32,
                        kernels={k: {kk: round(vv, 4) if isinstance(vv, float) else vv
                                     for kk, vv in v.items()} for k, v in ks32.items()})

    cpu = None
    cpu1 = None
    progress("done")
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0:
        cpu = wl["cpu"](args.cpu_baseline_seconds)
        # "... and a 1-thread row too" (a third of the budget)
        global _CPU_THREADS
        _CPU_THREADS = 1
        try:
            cpu1 = wl["cpu"](args.cpu_baseline_seconds / 3)
        finally:
            _CPU_THREADS = None
            _cpu_threads()

    if rank == 0:
        line = {
            "metric": wl["metric"],
            "value": round(rays_per_s, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            # the arithmetic the MLP computes in: f16x3 = fp32 operands
            # split into two fp16 pieces on fp16 matrix cores (not plain fp32)
            "dtype": math_main,
            "mlp_arithmetic": {
                "bf16x6": "bf16x6 (fp32 operands split exactly into 3 bf16 pieces, 6 piece "
                          "products accumulated in fp32; fp32-level accuracy, parity-tested "
                          "against the reference at 1e-4)",
                "f16x3": "f16x3 (fp32 operands split into 2 fp16 pieces, hi*hi + hi*lo + lo*hi "
                         "accumulated in fp32 with power-of-two range scaling: the 3xTF32 "
                         "scheme; fp32 inputs/outputs, parity-tested against the reference "
                         "at 1e-4)",
                "bf16": "bf16 (the reduced-precision variant of BASELINE configs[1]: matrix-core "
                        "operands rounded once to bf16, one product, fp32 accumulation; fp32 "
                        "activations, gradients and optimiser; judged on PSNR, not on the 1e-4 "
                        "parity bound)",
            }.get(_math(), "fp32"),
            "data": wl["data"],
            "config": {"workload": wl["workload"] + (" (bf16 MLP variant)" if _math() == "bf16" else ""),
                       "global_batch": wl["rays_per_step"] * world,
                       "samples_per_ray": wl["samples_per_ray"],
                       "parallelism": f"dp{world}" if wl["train"] else f"replicas{world}"},
            # the MLP work the kernels executed (every launch, the samples the
            # backward listed) per second of the whole step -- mlp_stage's FLOPs
            # over the step time -- and the reference algorithm's nominal count
            # (every sample through forward and both gradients), which the
            # zero-gradient skip never does
            "model_tflops": (round(stage["flop_per_step"] / (ms * 1e-3) / 1e12, 2)
                             if stage else None),
            "model_tflops_nominal": round(rays_per_s * wl["flop_per_ray"] / 1e12, 2),
            "model_tflops_basis": ("model_tflops: mlp_stage.flop_per_step (the MLP FLOPs executed, "
                                   "fp32-equivalent) / ms_per_step; model_tflops_nominal: the "
                                   "reference algorithm's FLOPs per ray (forward + data + weight "
                                   "gradient of every sample) x rays/s"),
            "roofline": roof,
            "rooflines": roofs_iso or roofs,
            "rooflines_basis": ("per-kernel launch times from 10 extra steps with both passes on "
                                "one stream (the timed region overlaps the two backward chains); "
                                "'roofline' is the kernel with the largest launch time there "
                                "(fine-pass launches): a forward kernel (the fine forward never "
                                "overlaps other work) is taken from the timed region itself, a "
                                "backward kernel from this serialised pass"
                                if roofs_iso else "the timed region"),
            "rooflines_concurrent": roofs_conc if roofs_iso else None,
            "mlp_stage": stage,
            "fp32_leg": fp32_leg,
            "backward_samples": backward_blocks,
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv
                            for kk, vv in v.items()} for k, v in ks.items()},
            "final_loss": round(loss.item(), 5) if loss is not None else None,
        }
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
