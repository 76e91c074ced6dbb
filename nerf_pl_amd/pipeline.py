"""The training step of a coarse/fine NeRF pair with the coarse model's
optimizer step -- and so the next step's coarse pass -- running beside the
fine model's backward tail (train.py:103-117: render, MSE, backward, Adam;
SURVEY.md 8f row 3, training glue).

``render_rays`` runs the fine pass on a side stream, so autograd runs the
fine model's backward there, beside the coarse model's on the caller's
stream (rendering.py).  At the end of ``loss.backward()``
autograd makes the caller's stream wait for every stream the backward used,
so with ONE optimizer step after it the next step's first kernel waits for
the fine model's weight gradient, which ends every step alone on the GPU
(~1.8 ms of ~8 ms at cfg2).  But the next step's coarse pass (ray
generation, coarse MLP, compositing, sample_pdf) reads only the coarse
model, and the two models' gradients and Adam updates are independent
(Adam is elementwise; sample_pdf's output is detached, rendering.py:253-255).

``PipelinedStep`` therefore
  * records an event when the coarse model's last gradient is accumulated
    (a post-accumulate-grad hook: before autograd's final stream join);
  * alternates the caller-side ("main") stream between two streams, so the
    next step's main stream waits only for that event -- not for the join;
  * runs the coarse model's Adam on the next main stream and the fine
    model's on the side stream, after its backward (stream order), where the
    next step's fine pass will run after it.
Every kernel reads exactly what it reads in the sequential schedule: the
parameters after a step are bit-identical (tests/test_gpu_pipeline.py).
With a ``GradAllReducer`` of one bucket per model (coarse first), each
bucket's all-reduce is issued after the backward has been enqueued, on the
stream of its model's Adam; the fine model's all-reduce and Adam are deferred
to just before the next step's fine pass (``rendering.BEFORE_FINE``), because
issuing an RCCL collective waits on the host for its input, and issued at the
end of the step it would hold back the next step's coarse pass.  ``flush()``
applies a deferred update (``__call__`` returns with one pending).
"""
from __future__ import annotations

import os

import torch

from .optim import FusedAdam

__all__ = ["PipelinedStep"]


class PipelinedStep:
    def __init__(self, models, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 reducer=None):
        from . import rendering
        if len(models) != 2:
            raise ValueError("PipelinedStep: a (coarse, fine) model pair")
        self.models = models
        kw = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.opt_c = FusedAdam([p for p in models[0].parameters() if p.requires_grad], **kw)
        self.opt_f = FusedAdam([p for p in models[1].parameters() if p.requires_grad], **kw)
        self.reducer = reducer
        if reducer is not None:
            if len(reducer.buckets) != 2:
                raise ValueError("PipelinedStep: the reducer needs one bucket per model, coarse first")
            # collectives issued after the backward is enqueued, each model's
            # on the stream of its Adam (GradAllReducer.hook_launch)
            reducer.hook_launch = False
        dev = next(models[0].parameters()).device
        self.device = dev
        # NERF_PL_AMD_MAIN_PRIORITY (A/B knob, e.g. -1): both main streams
        # created with that HIP priority instead of the caller's stream + one
        pr = os.environ.get("NERF_PL_AMD_MAIN_PRIORITY")
        if pr is None:
            self.mains = [torch.cuda.current_stream(dev), torch.cuda.Stream(device=dev)]
        else:
            self.mains = [torch.cuda.Stream(device=dev, priority=int(pr)) for _ in range(2)]
        self.side = rendering._side_stream(dev.index)
        self.k = 0
        self._coarse = [p for p in models[0].parameters() if p.requires_grad]
        self._n = 0
        self._ev = None
        self._pending = None      # the deferred fine update (distributed path)
        self._hooks = [p.register_post_accumulate_grad_hook(self._accumulated) for p in self._coarse]

    def _accumulated(self, p):
        # runs inside autograd's AccumulateGrad node, with the current stream
        # set to the one that produced the gradient (the coarse chain's); a
        # parameter accumulated more than once (a model used twice) records
        # the event again, so the last accumulation is the one waited for
        self._n += 1
        if self._n >= len(self._coarse):
            self._ev = torch.cuda.Event()
            self._ev.record()

    @property
    def stream(self):
        """the main stream the next step runs on"""
        return self.mains[self.k & 1]

    def __call__(self, loss_fn):
        """one step: ``loss_fn()`` renders and returns the loss (on the current
        stream, which this sets); returns the loss"""
        from . import rendering
        if not rendering.FINE_STREAM:
            raise RuntimeError("PipelinedStep needs rendering.FINE_STREAM (the fine pass on its "
                               "own stream)")
        cur, nxt = self.mains[self.k & 1], self.mains[(self.k + 1) & 1]
        if self._pending is not None:
            rendering.BEFORE_FINE.append(self.flush)
        with torch.cuda.stream(cur):
            loss = loss_fn()
        if self._pending is not None:      # loss_fn ran no fine pass
            if self.flush in rendering.BEFORE_FINE:
                rendering.BEFORE_FINE.remove(self.flush)
            self.flush()
        with torch.cuda.stream(cur):
            self.opt_c.zero_grad(set_to_none=True)
            self.opt_f.zero_grad(set_to_none=True)
            self._n, self._ev = 0, None
            loss.backward()
        if self._ev is None:
            raise RuntimeError("PipelinedStep: the coarse model received no gradient")
        nxt.wait_event(self._ev)
        # (the coarse gradients were allocated on cur: keep their blocks from
        # cur's later allocations until the Adam on nxt has read them)
        for p in self._coarse:
            if p.grad is not None:
                p.grad.record_stream(nxt)
        with torch.cuda.stream(nxt):
            if self.reducer is not None:
                self.reducer.finish(0)
            self.opt_c.step()
        if self.reducer is None:
            with torch.cuda.stream(self.side):
                self.opt_f.step()
        else:
            self._pending = True
        self.k += 1
        return loss

    def flush(self):
        """the deferred fine update: its all-reduce and Adam on the side stream"""
        if self._pending is None:
            return
        self._pending = None
        with torch.cuda.stream(self.side):
            self.reducer.finish(1)
            self.opt_f.step()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
