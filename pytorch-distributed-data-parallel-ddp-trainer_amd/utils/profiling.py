"""Tracing / timing helpers (SURVEY.md §5.1 - the reference has none).

* :func:`trace_range` - a roctx range (``torch.cuda.nvtx`` is backed by roctx on
  ROCm builds) that shows up in ``rocprofv3 --marker-trace`` timelines; no-op on CPU.
* :class:`StepTimer` - hipEvent-based device timing of named regions on a stream
  (no host sync until :meth:`summary`), with mean / p50 / p90 per region.
* :func:`images_per_sec` - the headline metric.
"""
from __future__ import annotations

import contextlib
import statistics
import time

import torch


@contextlib.contextmanager
def trace_range(name: str):
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    """Accumulates device time per region.  Usage::

        t = StepTimer(stream)
        with t("fwd"): ...
        print(t.summary())
    """

    def __init__(self, stream=None, enabled: bool = True):
        self.stream = stream
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: list[tuple[str, object, object]] = []
        self._host: dict[str, list[float]] = {}
        self.times: dict[str, list[float]] = {}

    @contextlib.contextmanager
    def __call__(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            yield
            self._host.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
            return
        s = self.stream or torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        try:
            with trace_range(name):
                yield
        finally:
            b.record(s)
            self._pending.append((name, a, b))

    def _collect(self):
        for name, a, b in self._pending:
            b.synchronize()
            self.times.setdefault(name, []).append(a.elapsed_time(b))
        self._pending.clear()
        for k, v in self._host.items():
            self.times.setdefault(k, []).extend(v)
        self._host.clear()

    def summary(self) -> dict:
        """{region: {"n", "mean_ms", "p50_ms", "p90_ms", "total_ms"}}"""
        self._collect()
        out = {}
        for k, v in self.times.items():
            sv = sorted(v)
            out[k] = {"n": len(v), "mean_ms": statistics.fmean(v), "p50_ms": sv[len(sv) // 2],
                      "p90_ms": sv[min(len(sv) - 1, int(0.9 * len(sv)))], "total_ms": sum(v)}
        return out


def images_per_sec(images: int, seconds: float) -> float:
    return images / seconds if seconds > 0 else float("nan")
