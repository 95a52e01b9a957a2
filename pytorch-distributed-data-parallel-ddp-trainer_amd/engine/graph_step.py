"""Whole-step hipGraph capture for the module path (forward, backward with the DDP
bucket all-reduces, optimizer) - the MI355X replacement for a tracing compiler.

ResNet-18 at batch 32 issues ~200 kernels per step; eager, the Python autograd engine
and the launch path leave ~10 % of the step idle between kernels (profiles/r1_resnet).
One captured graph replays the same kernels back to back.  Everything in the step must
be capturable: our HIP ops launch on the current stream, FlatSpace gradients are
zeroed with a memset, the native reducer's comm stream forks / joins the capture
through hipEvents, and BatchNorm's num_batches_tracked is bumped inside bn_finalize.

Usage::

    step = GraphedStep(lambda x, y: train_step(x, y), (x0, y0), warmup=3)
    for x, y in batches:
        loss = step(x, y)      # copies into the static inputs, replays the graph
"""
from __future__ import annotations

import torch


class GraphedStep:
    def __init__(self, step_fn, example_inputs, warmup: int = 3):
        """``step_fn(*static_inputs) -> tensor`` runs one full training step.  The
        ``warmup`` eager calls (on a side stream, as capture requires) are real steps:
        they allocate optimizer state and the kernels' workspaces before capture."""
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.static = [t.clone() for t in example_inputs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self.warmup_out = step_fn(*self.static)  # the last warm-up step's result
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = step_fn(*self.static)
        self.replays = 0

    def __call__(self, *inputs):
        for dst, src in zip(self.static, inputs):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        return self.out
