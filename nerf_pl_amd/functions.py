"""Autograd functions binding the HIP forward/backward kernels.

``_FusedMLP``: fused PE + MLP forward (saving activations when any parameter
needs a gradient); backward = fused data-gradient chain (``nr_mlp_bwd``) then
the grouped split-K weight-gradient GEMM (``nr_wgrad``), returning one gradient
per ``NeRF`` parameter (views into one flat buffer, named_parameters order).

``_Composite``: volume compositing forward/backward (``nr_composite_*``).
"""
from __future__ import annotations

import collections
import functools
import os
import threading
import weakref

import torch

from . import ops, packing
from ._lib import call, stream_of


@functools.lru_cache(maxsize=4)
def _wgrad_workspace(device_index: int, stream: int = 0) -> torch.Tensor:
    """Split-K slab workspace of the weight gradient, one per (device, stream):
    backward passes enqueued on different streams never share slabs.  The
    size is the library's bound over every launch shape (~1.2 GB; the slabs a
    launch uses depend only on the task list, not on n).  At most 4 are kept
    (least recently used evicted): a workspace is allocated while its stream is
    current, so once evicted the caching allocator hands its memory only to
    later work on that same stream, which runs after the kernels still using
    it -- code that creates side streams per iteration cannot pin unbounded
    device memory."""
    from ._lib import lib
    nbytes = int(lib().nr_wgrad_workspace_bytes(0))
    return torch.empty(nbytes // 4, dtype=torch.float32, device=torch.device("cuda", device_index))


# sigma-only graphs train on the sigma-only kernels (NERF_PL_AMD_SIGMA_TRAIN=0:
# on the full kernels with a zero rgb gradient -- the A/B reference of the tests)
SIGMA_TRAIN_KERNELS = os.environ.get("NERF_PL_AMD_SIGMA_TRAIN", "1") != "0"

# the backward works on the samples with a nonzero output
# gradient only (nr_active_samples; exact: the others add zeros to every sum),
# packed densely.  NERF_PL_AMD_ACTIVE_SAMPLES=0: every sample (the A/B reference)
ACTIVE_SAMPLES = os.environ.get("NERF_PL_AMD_ACTIVE_SAMPLES", "1") != "0"
# the arithmetics with *_active entry points (the bf16 variant keeps its
# sample-major 16x16 bf16 chunks whole: no gather)
ACTIVE_ARITHS = ("f16x3", "bf16x6", "fp32")
# Deferred save: a training forward whose backward will list
# few samples runs without saving activations (the inference kernel), and the
# backward re-evaluates the listed samples only, saving them by position
# (nr_mlp_fwd_listed*) -- exact: the recomputed layers are the forward's layers
# bit for bit, so every step's results are the same whichever way it goes.
# "sigma": the sigma-only graphs of the shadow path (rendering_shadows.py:167),
# whose backward lists ~0.1% of a light image's samples and ~20% of the camera
# rays'; "all": every training forward; "none": none; "auto" (default): the
# sigma-only graphs, and a full graph whenever its model's last backward listed
# fewer than DEFER_AUTO of the samples (a trained NeRF leaves most samples in
# empty space; at the bench's random init ~half are listed, where saving at
# forward time is faster)
DEFER_SAVE = os.environ.get("NERF_PL_AMD_DEFER_SAVE", "auto")
if DEFER_SAVE not in ("sigma", "all", "none", "auto"):
    raise ValueError(f"NERF_PL_AMD_DEFER_SAVE must be auto, sigma, all or none, got {DEFER_SAVE!r}")
DEFER_AUTO = float(os.environ.get("NERF_PL_AMD_DEFER_AUTO", "0.3"))


# Per-model statistics of the deferred-save policy: model -> {sigma_only:
# _ListedStats}.  Kept outside the module (a WeakKeyDictionary: an entry dies
# with its model) so a NeRF stays deep-copyable and picklable after training
# steps -- the entries hold CUDA events, which cannot be pickled.
_LISTED = weakref.WeakKeyDictionary()
_LISTED_LOCK = threading.Lock()


class _ListedStats:
    """the latest completed list fraction and the copies still in flight"""
    __slots__ = ("frac", "pending")

    def __init__(self):
        self.frac = None
        self.pending = collections.deque()     # (pinned host count, event, n), oldest first


def _listed_fraction(model, sigma_only):
    """the fraction of samples the model's latest completed backward of this
    graph kind listed, or None when none has completed yet.  Each backward
    queues a device -> pinned host copy of its list length behind an event
    (_note_listed); this reads the copies whose events have completed, oldest
    first (one stream: they complete in order) -- no synchronisation, and a
    host running several steps ahead of the GPU still sees the newest finished
    count.  All trimming happens here, under the lock, and an entry is popped
    only after its own event was seen complete (a backward on
    another thread can append concurrently)."""
    with _LISTED_LOCK:
        e = _LISTED.get(model, {}).get(sigma_only)
        if e is None:
            return None
        while e.pending and e.pending[0][1].query():
            host, _, n = e.pending.popleft()
            e.frac = int(host[0]) / max(n, 1)
        # a host far ahead of the GPU: keep the newest 16 copies in flight
        while len(e.pending) > 16:
            e.pending.popleft()
        return e.frac


def _note_listed(model, sigma_only, count_dev, n):
    """queue the copy of a backward's sample-list length for _listed_fraction"""
    host = torch.empty(1, dtype=torch.int32, pin_memory=True)
    host.copy_(count_dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    with _LISTED_LOCK:
        per_model = _LISTED.get(model)
        if per_model is None:
            per_model = _LISTED[model] = {}
        per_model.setdefault(sigma_only, _ListedStats()).pending.append((host, ev, n))


# bench.py's kernel timer: a list every backward appends its (sample list
# buffer, index of its length) to, so the rooflines count the samples worked on
ACTIVE_LOG = None

# NERF_PL_AMD_DEBUG=1 keeps the last backward's buffers here (dev/ scripts;
# tests set it to {} for one call) and every training forward's save buffer
_DEBUG = {} if os.environ.get("NERF_PL_AMD_DEBUG") == "1" else None

_SHAPES = list(packing.param_shapes().items())
# parameters the sigma-only graph does not reach (reference autograd leaves them None)
_SIGMA_ONLY_UNUSED = {"xyz_encoding_final.weight", "xyz_encoding_final.bias",
                      "dir_encoding.0.weight", "dir_encoding.0.bias",
                      "rgb.0.weight", "rgb.0.bias"}


class _FusedMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, rays, z, spr, x, sigma_only, *params):
        train = any(ctx.needs_input_grad[6:])
        if train and sigma_only and x is not None:
            raise NotImplementedError("nerf_pl_amd: training NeRF.forward(x, sigma_only=True) on "
                                      "pre-embedded input is not supported; use render_rays")
        packed_f, packed_b = model.packed(backward=train)
        # a sigma-only graph (rendering_shadows.py:167) trains through the
        # sigma-only training kernels (layers 1-8 and the sigma head: no
        # xyz_encoding_final / dir / rgb work), in every arithmetic
        so_train = train and sigma_only and SIGMA_TRAIN_KERNELS and x is None
        kern_sigma_only = sigma_only and (not train or so_train)
        defer = False
        if train and x is None and ACTIVE_SAMPLES and ops.arith_of(packed_b) in ACTIVE_ARITHS:
            if DEFER_SAVE == "all" or (DEFER_SAVE in ("sigma", "auto") and so_train):
                defer = True
            elif DEFER_SAVE == "auto":
                frac = _listed_fraction(model, sigma_only)
                defer = frac is not None and frac < DEFER_AUTO
        model.__dict__["_nr_defer_last"] = defer
        if x is None:
            # the tensors the kernels read (contiguous copies of strided views):
            # the deferred backward re-reads exactly these
            rays = ops._dev(rays, "rays", 8)
            z = ops._dev(z, "z")
        out, save = ops.mlp_forward(packed_f, rays=rays, z=z, samples_per_ray=spr, x=x,
                                    sigma_only=kern_sigma_only, save=train and not defer)
        if _DEBUG is not None and save is not None:
            # the training forward's saved activations, in call order (tests
            # read the ReLU masks the kernels chose: tests/grad64.py mlp_flips)
            _DEBUG.setdefault("fwd_saves", []).append((save, out.shape[0], ops.MATH))
        if train:
            # the flat parameters the forward ran with (the dir layer's
            # feat-column weight gradient reads W_final, b_final and W_dir
            # there: nr_wgrad_dir_feat), and the parameters themselves, so that
            # autograd's version check raises if one changes in place between
            # this forward and its backward, as it would for the reference's
            # nn.Linear graph (a parameter's storage is a view of
            # flat, but its version counter is its own)
            flat = model.flat_params()
            if defer:     # the backward recomputes the listed samples' activations
                ctx.save_for_backward(out, rays, z, packed_f, packed_b, flat, *params)
                ctx.spr = spr
            else:
                ctx.save_for_backward(out, save, packed_f, packed_b, flat, *params)
            ctx.defer = defer
            ctx.sigma_only = sigma_only
            ctx.model = model if DEFER_SAVE == "auto" else None
            ctx.so_kernels = so_train
        if sigma_only and train and out.shape[1] == 4:
            out = out[:, 3:4].contiguous()
        return out

    @staticmethod
    def backward(ctx, g_out):
        if ctx.defer:
            return _FusedMLP._backward_deferred(ctx, g_out)
        out, save, packed_f, packed_b, flat = ctx.saved_tensors[:5]
        n = out.shape[0]
        dev = out.device
        if ctx.sigma_only:
            g4 = torch.zeros(n, 4, device=dev)
            g4[:, 3:4] = g_out
            g_out = g4
        grad_ws = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
        g_out = g_out.contiguous()
        sfx = "_sigma" if ctx.so_kernels else ""
        st = stream_of(dev)
        active = ()
        if ACTIVE_SAMPLES and ops.arith_of(packed_b) in ACTIVE_ARITHS:
            # the samples with a nonzero output gradient, ascending (int32 [0, n)),
            # their count ([n]) and the compaction's scratch
            sl = torch.empty(n + 1 + 2 * ((n + 31) // 32), dtype=torch.int32, device=dev)
            call("nr_active_samples", g_out.data_ptr(), n, sl.data_ptr(), sl.data_ptr() + 4 * n,
                 sl.data_ptr() + 4 * (n + 1), st)
            active = (sl.data_ptr(), sl.data_ptr() + 4 * n)
            if ACTIVE_LOG is not None:
                ACTIVE_LOG.append((sl, n))
            if ctx.model is not None:
                _note_listed(ctx.model, ctx.sigma_only, sl[n:n + 1], n)
            sfx += "_active"
        call(ops.entry("nr_mlp_bwd" + sfx, packed_b), packed_b.data_ptr(), ops.head_ptr(packed_f),
             out.data_ptr(), g_out.data_ptr(), save.data_ptr(), n, grad_ws.data_ptr(), *active, st)
        gflat = torch.empty(packing.N_PARAMS, device=dev)
        ws = _wgrad_workspace(dev.index, int(st))
        call(ops.entry("nr_wgrad" + sfx, packed_b), save.data_ptr(), grad_ws.data_ptr(), n,
             ws.data_ptr(), gflat.data_ptr(), *active, st)
        if not ctx.so_kernels:
            _dir_feat(flat, gflat, st)
        if _DEBUG is not None:
            _DEBUG.update(save=save, grad_ws=grad_ws, g_out=g_out, gflat=gflat, n=n)
            _DEBUG.setdefault("g_outs", []).append(g_out)
        return (None,) * 6 + _param_grads(gflat, ctx.sigma_only)

    @staticmethod
    def _backward_deferred(ctx, g_out):
        """The deferred save's backward: the sample list of g_out, the training
        forward re-run over the listed samples (activations saved by position),
        then the data and weight gradients over those positions."""
        out, rays, z, packed_f, packed_b, flat = ctx.saved_tensors[:6]
        n = z.numel()
        dev = z.device
        if g_out.shape[1] == 1:            # a sigma-only graph's d sigma
            g4 = torch.zeros(n, 4, device=dev)
            g4[:, 3:4] = g_out
            g_out = g4
        g_out = g_out.contiguous()
        if out.shape[1] != 4:              # the rgb rows only feed the rgb head's backward
            out = g_out
        st = stream_of(dev)
        sl = torch.empty(n + 1 + 2 * ((n + 31) // 32), dtype=torch.int32, device=dev)
        call("nr_active_samples", g_out.data_ptr(), n, sl.data_ptr(), sl.data_ptr() + 4 * n,
             sl.data_ptr() + 4 * (n + 1), st)
        lst = (sl.data_ptr(), sl.data_ptr() + 4 * n)
        if ACTIVE_LOG is not None:
            ACTIVE_LOG.append((sl, n))
        if ctx.model is not None:
            _note_listed(ctx.model, ctx.sigma_only, sl[n:n + 1], n)
        so = ctx.so_kernels
        save = torch.empty(ops.save_floats(n), device=dev)
        call(ops.entry("nr_mlp_fwd_listed", packed_f), packed_f.data_ptr(), rays.data_ptr(),
             z.data_ptr(), n, int(ctx.spr), int(so), save.data_ptr(), *lst, st)
        grad_ws = torch.empty(ops.n_blocks(n) * ops.GRAD_PER_BLOCK, device=dev)
        sfx = "_sigma_listed" if so else "_listed"
        call(ops.entry("nr_mlp_bwd" + sfx, packed_b), packed_b.data_ptr(), ops.head_ptr(packed_f),
             out.data_ptr(), g_out.data_ptr(), save.data_ptr(), n, grad_ws.data_ptr(), *lst, st)
        gflat = torch.empty(packing.N_PARAMS, device=dev)
        ws = _wgrad_workspace(dev.index, int(st))
        call(ops.entry("nr_wgrad" + sfx, packed_b), save.data_ptr(), grad_ws.data_ptr(), n,
             ws.data_ptr(), gflat.data_ptr(), *lst, st)
        if not so:
            _dir_feat(flat, gflat, st)
        return (None,) * 6 + _param_grads(gflat, ctx.sigma_only)


def _dir_feat(flat, gflat, st):
    """dir_encoding.0.weight's feat columns: the weight-gradient launch leaves
    G = sum dz_dir h8^T there (feat is not saved); G W_final^T + db b_final^T"""
    call("nr_wgrad_dir_feat", flat.data_ptr(), gflat.data_ptr(), st)


def _param_grads(gflat, sigma_only):
    """one view of the flat gradient per NeRF parameter (named_parameters
    order); None for the parameters a sigma-only graph does not reach"""
    grads, off = [], 0
    for name, shp in _SHAPES:
        k = 1
        for d in shp:
            k *= d
        g = gflat[off:off + k].view(shp)
        off += k
        grads.append(None if (sigma_only and name in _SIGMA_ONLY_UNUSED) else g)
    return tuple(grads)


def mlp_apply(model, *, rays=None, z=None, spr=0, x=None, sigma_only=False):
    """Run ``model`` (a nerf_pl_amd.NeRF) on rays+depths or on embedded x."""
    if x is not None and x.requires_grad:
        raise NotImplementedError("nerf_pl_amd: gradients w.r.t. the embedded input are not "
                                  "produced (the reference never needs them)")
    params = model.ordered_params()
    if z is not None:
        z = z.reshape(-1)
    if not any(p.requires_grad for p in params) or not torch.is_grad_enabled():
        packed_f, _ = model.packed()
        out, _ = ops.mlp_forward(packed_f, rays=rays, z=z, samples_per_ray=spr, x=x,
                                 sigma_only=sigma_only)
        return out
    return _FusedMLP.apply(model, rays, z, spr, x, sigma_only, *params)


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z, rays, noise, noise_std, seed, stream, white_back):
        rgb, depth, opac, w = ops.composite_forward(raw, z, rays, noise, noise_std, seed, stream,
                                                    white_back)
        ctx.save_for_backward(raw, z, rays, noise if noise is not None else torch.empty(0))
        ctx.cfg = (noise is not None, noise_std, seed, stream, white_back)
        ctx.mark_non_differentiable(w)
        # unused outputs (depth, opacity in the training loss) reach backward as
        # None -- the kernel treats a null gradient as zero -- instead of as
        # zero tensors autograd would fill with one launch each
        ctx.set_materialize_grads(False)
        return rgb, depth, opac, w

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_opac, g_w):   # noqa: ARG004 -- weights not differentiable
        raw, z, rays, noise = ctx.saved_tensors
        has_noise, noise_std, seed, stream, white_back = ctx.cfg
        g_raw = ops.composite_backward(raw, z, rays, noise if has_noise else None, noise_std, seed,
                                       stream, white_back, g_rgb, g_depth, g_opac)
        return g_raw, None, None, None, None, None, None, None


def composite_apply(raw, z, rays, noise, noise_std, seed, stream, white_back):
    if torch.is_grad_enabled() and raw.requires_grad:
        return _Composite.apply(raw, z, rays, noise, noise_std, seed, stream, white_back)
    return ops.composite_forward(raw, z, rays, noise, noise_std, seed, stream, white_back)
