"""Batch sharding across GPUs: problems are independent, so a batch of B
problems splits into contiguous row ranges, one per device, with no collective.

Two launch styles:
  * one process per GPU (torch.distributed.run; bench.py): each rank takes
    ``shard_range(B, rank, world)`` of the global batch;
  * one process, many GPUs: :class:`ShardedSQP` runs one host thread per device (ctypes drops
    the GIL inside the library call, so the devices work concurrently) and concatenates.
"""
from __future__ import annotations

import threading
from typing import List, Sequence, Tuple

import numpy as np


def shard_range(B: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of a B-row batch owned by ``rank`` of ``world`` (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(B, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_ranges(B: int, world: int) -> List[Tuple[int, int]]:
    return [shard_range(B, r, world) for r in range(world)]


class ShardedSQP:
    """Full SQP solves of a (B, .) batch split over several GPUs of this process.

    ``qp_mode`` defaults like ``OSQPSolver`` and ``batch_sqp``: "admm" (OSQP's iteration, the
    reference's numbers) with each problem's OSQP state carried in its device's handle from call to
    call — so a problem must come back to the same shard: keep B (hence the contiguous ranges) fixed
    across calls, as the reference's batch axis does (src/gato_mpc_batch.py:38-52).  "direct" is
    the exact KKT solve."""

    def __init__(self, model, devices: Sequence[int], N=32, max_batch_per_device=4096, qp_mode="admm", admm=None,
                 **cost_kw):
        from . import _lib

        if qp_mode not in ("direct", "admm"):
            raise ValueError("qp_mode must be 'direct' or 'admm'")
        mode = _lib.QP_ADMM if qp_mode == "admm" else _lib.QP_DIRECT
        self.devices = list(devices)
        self.handles = [_lib.Handle(model, N=N, max_batch=max_batch_per_device, device_id=d, qp_mode=mode, admm=admm,
                                    **cost_kw) for d in self.devices]
        self.N = N
        self.qp_mode = qp_mode
        self._B = None  # the batch size whose ranges own the carried OSQP state (ADMM mode)

    def solve(self, xcur, goals, XU):
        XU = np.ascontiguousarray(XU, dtype=float)
        B = XU.shape[0]
        if self.qp_mode == "admm" and self._B is not None and B != self._B:
            raise ValueError(f"ADMM mode carries each problem's OSQP state on its shard: batch {B} after {self._B} "
                             "would move problems between devices; call reset() first")
        self._B = B
        ranges = shard_ranges(B, len(self.handles))
        outs = [None] * len(self.handles)
        errs = []

        def work(i, lo, hi):
            try:
                if hi > lo:
                    outs[i] = self.handles[i].solve(xcur[lo:hi], goals[lo:hi], XU[lo:hi])
            except Exception as e:  # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=work, args=(i, lo, hi)) for i, (lo, hi) in enumerate(ranges)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        parts = [o for o in outs if o is not None]
        if not parts:  # B = 0: empty results, as Handle.solve / i7m_solve give
            from ._lib import STATS_DTYPE
            return np.empty((0, XU.shape[1] if XU.ndim == 2 else 18 * self.N - 6)), np.zeros(0, dtype=STATS_DTYPE)
        return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])

    def reset(self):
        """A fresh solver on every device (i7m_reset: ADMM mode's OSQP state from scratch)."""
        for h in self.handles:
            h.reset()
        self._B = None

    def admm_state(self, B):
        """The carried OSQP state of problems [0, B) (x, z, y, q, rho), gathered from the shards."""
        parts = [h.admm_state(hi - lo) for h, (lo, hi) in zip(self.handles, shard_ranges(B, len(self.handles)))
                 if hi > lo]
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(5))
