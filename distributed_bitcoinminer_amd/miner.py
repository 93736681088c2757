"""Miner-side mirror of ``evalRoutine`` (cmu440/bitcoin/miner/miner.go:36-68).

``Miner.eval_request`` is one iteration of the reference's loop body
(miner.go:44-62): unmarshal the Request (errors ignored, :45), scan
``[Lower, Upper]`` for the min hash and marshal ``NewResult(hash, nonce)``.
The scan itself -- the reference's hot loop, miner.go:46-59 -- runs on the
GPU through ``hm_scan``.  The reference's ``upper := Upper+1`` (:52) is a
uint64 add, so ``Upper == 2^64-1`` scans nothing and yields
``(MaxUint64, 0)``; that quirk (SURVEY A-inv-5) is reproduced here, in the
caller, exactly as the Go shim in go/src/hipminer does it.

This adapter is GPU-only: if the GPU path fails, ``HipMinerError``
propagates.  The miner processes (hm_miner, Go gpuminer) instead fall back to
the host scan hm_scan_cpu (``_lib.scan_cpu``) so that a Result is always
written; ``eval_range`` gives the range either one scans.
"""
from __future__ import annotations

from . import _lib
from .bitcoin import MAXU64, NewResult, marshal, unmarshal


def eval_range(lower: int, upper: int):
    """The scan range miner.go:50-53 actually visits, or None if empty."""
    up = (upper + 1) & MAXU64  # miner.go:52, uint64 wrap
    if not lower < up:
        return None
    return lower, up - 1


class Miner:
    """GPU-backed miner: evalRoutine's Request -> Result step."""

    def __init__(self, ctx: _lib.Context | None = None, devices=None):
        self.ctx = ctx if ctx is not None else _lib.Context(devices)

    def scan(self, data, lower: int, upper: int) -> tuple[int, int]:
        """(result, index) of miner.go:46-59 for Request{data, lower, upper}."""
        rng = eval_range(lower, upper)
        if rng is None:
            return MAXU64, 0  # miner.go:48-49 initial values, loop never runs
        return self.ctx.scan(data, rng[0], rng[1])

    def eval_request(self, payload: bytes) -> bytes:
        """One evalRoutine step: Request payload in, Result payload out."""
        req, _err = unmarshal(payload)  # error ignored, miner.go:45
        h, n = self.scan(req.Data, req.Lower, req.Upper)
        return marshal(NewResult(h, n))

    def close(self):
        self.ctx.close()
