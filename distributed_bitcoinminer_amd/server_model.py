"""Model of the unchanged reference server's split and merge (SURVEY A-inv-7).

The server (cmu440/bitcoin/server/server.go) is out of scope and stays as it
is; this model gives exact end-to-end expectations for GPU miners driven by it:

* ``load_balance`` restates server.go:165-205: ``upper += 1`` (:169, uint64),
  ``totalLoad = upper - lower``, equal chunks with the remainder added to
  chunk 0, each sent as Request(data, start, end) that the miner then scans
  INCLUSIVELY (so neighbouring chunks overlap by one nonce); more miners than
  nonces gives ``totalLoad`` chunks of 1.
* ``merge_in_arrival_order`` restates server.go:140-141 (seed
  (MaxUint64, MaxUint64)) and :273-276 (strict ``<`` in arrival order).
* ``expected_client_result`` combines both with the miner semantics
  (miner.go:46-59 incl. the Upper+1 wrap) for a given scan function.
* ``ServerSim`` is the whole event loop of the server (server.go:207-400) as a
  deterministic state machine: FIFO of client requests, miner joins, results,
  and the drop / reassign paths for miners and clients.  Driving real GPU
  miners with it gives exact expectations when miners fail.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

from . import bitcoin

MAXU64 = (1 << 64) - 1


def load_balance(lower: int, upper: int, n_miners: int) -> list[tuple[int, int]]:
    """Requests (Lower, Upper) the server sends, in miner order."""
    upper = (upper + 1) & MAXU64                     # :169
    total = (upper - lower) & MAXU64                 # :170
    num = n_miners
    individual = total // num                        # :171
    leftover = total - individual * num              # :172
    if individual == 0:                              # :173-177
        individual, leftover, num = 1, 0, total
    chunks = []
    start = lower
    for i in range(num):                             # :181-204
        end = (start + individual) & MAXU64
        if i == 0:
            end = (end + leftover) & MAXU64
        chunks.append((start, end))
        start = end
    return chunks


def merge_in_arrival_order(results) -> tuple[int, int]:
    min_hash, min_nonce = MAXU64, MAXU64             # :140-141
    for h, n in results:
        if h < min_hash:                             # :273-276
            min_hash, min_nonce = h, n
    return min_hash, min_nonce


def expected_client_result(data, lower: int, upper: int, n_miners: int,
                           miner_scan: Callable, order=None):
    """What the client prints for Request(data, lower, upper) with n miners.

    ``miner_scan(data, Lower, Upper)`` must implement the miner's step
    (e.g. ``Miner.scan``).  Returns None when the request never completes
    (no chunk assigned: lower == 0 and upper == MaxUint64)."""
    chunks = load_balance(lower, upper, n_miners)
    if not chunks:
        return None
    results = [miner_scan(data, lo, hi) for lo, hi in chunks]
    if order is not None:
        results = [results[i] for i in order]
    return merge_in_arrival_order(results)


# ---------------------------------------------------------------------------
# Event-driven server model (server.go:207-400)
# ---------------------------------------------------------------------------

class ServerPanic(RuntimeError):
    """A state in which the Go server would panic (nil dereference)."""


@dataclass
class _Job:
    """clientRequest (server.go:32-42)."""
    conn_id: int
    data: object
    lower: int
    upper: int
    responsible: list = field(default_factory=list)  # miner ids, one per chunk sent
    min_hash: int = MAXU64                            # :140
    min_nonce: int = MAXU64                           # :141
    responses: int = 0
    dropped: bool = False


@dataclass
class _MinerSlot:
    """miner (server.go:50-57): its current chunk and whether it is idle."""
    miner_id: int
    data: object = b""
    lower: int = 0
    upper: int = 0
    available: bool = True


class ServerSim:
    """The reference server's mainRoutine as a deterministic state machine.

    Each event method returns the LSP writes the server makes, as a list of
    ``(conn_id, bitcoin.Message)`` in order.  Events mirror the server's
    channels: ``client_request`` (a Request read, :131-145 -> :211-219),
    ``miner_join`` (:146-152 -> :222-254), ``miner_result`` (:153-159 ->
    :257-325) and ``drop`` (a Read error, :122-125 -> :326-400).

    Quirks kept on purpose: Requests use the A-inv-7 chunks; a result from a
    miner that is no longer registered or responsible is ignored; a dropped
    miner's chunk goes to the first idle miner, else waits for the next result
    or join; a dropped client's request stays current until every responsible
    miner has answered (and forever if one of them was dropped meanwhile)."""

    def __init__(self):
        self.waiting: list[_Job] = []
        self.curr: _Job | None = None
        self.miners: list[_MinerSlot] = []
        self.dropped: list[_MinerSlot] = []

    # -- helpers -------------------------------------------------------------
    def _find(self, mid):
        for m in self.miners:
            if m.miner_id == mid:
                return m
        return None

    def _assign(self, m: _MinerSlot, data, lo: int, hi: int, out: list):
        m.data, m.lower, m.upper, m.available = data, lo, hi, False
        out.append((m.miner_id, bitcoin.NewRequest(data, lo, hi)))

    def _take_over(self, m: _MinerSlot, gone: _MinerSlot, out: list):
        """m inherits the chunk of the dropped miner `gone` (:227-242, :286-302, :352-369)."""
        self._assign(m, gone.data, gone.lower, gone.upper, out)
        if self.curr is None:
            raise ServerPanic("reassignment with no current request")
        self.curr.responsible = [m.miner_id if r == gone.miner_id else r
                                 for r in self.curr.responsible]

    def _load_balance(self, job: _Job, out: list):
        """server.go:165-205 over every registered miner, in join order."""
        self.curr = job
        for m, (lo, hi) in zip(self.miners, load_balance(job.lower, job.upper, len(self.miners))):
            self._assign(m, job.data, lo, hi, out)
            job.responsible.append(m.miner_id)

    # -- events --------------------------------------------------------------
    def client_request(self, conn_id: int, data, lower: int, upper: int) -> list:
        out = []
        job = _Job(conn_id, data, lower, upper)
        if not self.waiting and self.curr is None and self.miners:   # :212
            self._load_balance(job, out)
        else:
            self.waiting.append(job)
        return out

    def miner_join(self, miner_id: int) -> list:
        out = []
        m = _MinerSlot(miner_id)
        if self.dropped:                                               # :224-244
            self._take_over(m, self.dropped[0], out)
            self.dropped.pop(0)
        self.miners.append(m)
        if self.curr is None and self.waiting:                         # :246-253
            self._load_balance(self.waiting.pop(0), out)
        return out

    def miner_result(self, miner_id: int, hash_: int, nonce: int) -> list:
        out = []
        job = self.curr
        if job is None:                                                # :259-261
            return out
        if miner_id not in job.responsible or self._find(miner_id) is None:
            return out                                                 # :269-271
        if hash_ < job.min_hash:                                       # :273-276
            job.min_hash, job.min_nonce = hash_, nonce
        job.responses += 1
        m = self._find(miner_id)
        m.available = True
        if self.dropped:                                               # :285-304
            self._take_over(m, self.dropped[0], out)
            self.dropped.pop(0)
        if job.responses == len(job.responsible):                      # :309-325
            if not job.dropped:
                out.append((job.conn_id, bitcoin.NewResult(job.min_hash, job.min_nonce)))
            self.curr = None
            if self.waiting:
                self._load_balance(self.waiting.pop(0), out)
        return out

    def drop(self, conn_id: int) -> list:
        out = []
        gone = self._find(conn_id)
        if gone is not None:                                           # a miner, :327-376
            self.miners.remove(gone)
            job = self.curr
            if job is None or job.dropped:
                return out
            idle = next((m for m in self.miners if m.available), None)
            if idle is not None:
                self._take_over(idle, gone, out)
            else:
                self.dropped.append(gone)
            return out
        # a client, :377-400
        if self.curr is not None and self.curr.conn_id == conn_id:
            self.curr.dropped = True
            for m in self.miners:
                m.available = True
            self.dropped = []
        self.waiting = [j for j in self.waiting if j.conn_id != conn_id]
        return out
