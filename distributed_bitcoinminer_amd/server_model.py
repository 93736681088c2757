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
  (miner.go:63-76 incl. the Upper+1 wrap) for a given scan function.
"""
from __future__ import annotations

from typing import Callable

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
