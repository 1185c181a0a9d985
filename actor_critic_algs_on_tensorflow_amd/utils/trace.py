"""Phase timers and ROCTx ranges (the reference has no tracing at all).

``PhaseTimer.phase(name)`` brackets a region with a ROCTx range (``torch.cuda.nvtx`` is backed by roctx on ROCm
builds, so a rocprofv3 marker trace shows the rollout / returns / learn / update phases next to the kernels) and two
timing events on the current stream. The events are read only when :meth:`summary` is called (the trainer's log
cadence), so timing adds no host synchronisation to the training loop. On the CPU the wall clock is used.
"""
from __future__ import annotations

import contextlib
import time

import torch


class PhaseTimer:
    def __init__(self, device, enabled=False, markers=True):
        self.device = torch.device(device)
        self.enabled = bool(enabled)
        self.markers = markers and self.device.type == "cuda"
        self.suspended = False          # set while a hipGraph is being captured (no timing events inside a capture)
        self._pending = []
        self._acc = {}

    @contextlib.contextmanager
    def phase(self, name):
        if not self.enabled or self.suspended:
            yield
            return
        cuda = self.device.type == "cuda"
        if self.markers:
            torch.cuda.nvtx.range_push(name)
        if cuda:
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record()
        else:
            t0 = time.perf_counter()
        try:
            yield
        finally:
            if cuda:
                end.record()
                self._pending.append((name, start, end))
            else:
                self._add(name, (time.perf_counter() - t0) * 1e3)
            if self.markers:
                torch.cuda.nvtx.range_pop()

    def _add(self, name, ms):
        tot, n = self._acc.get(name, (0.0, 0))
        self._acc[name] = (tot + ms, n + 1)

    def summary(self, reset=True):
        """-> {phase: mean ms per occurrence} since the last summary (synchronises on the recorded events)."""
        for name, s, e in self._pending:
            e.synchronize()
            self._add(name, s.elapsed_time(e))
        self._pending = []
        out = {k: round(tot / max(n, 1), 4) for k, (tot, n) in self._acc.items()}
        if reset:
            self._acc = {}
        return out
