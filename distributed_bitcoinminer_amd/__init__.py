"""MI355X-native miner backend for alexsun705/distributed_bitcoinMiner's min-hash scan.

The hot path is the miner's scan (cmu440/bitcoin/miner/miner.go:46-59 calling
bitcoin.Hash, cmu440/bitcoin/hash.go:13-17).  It runs as hand-written gfx950
HIP kernels behind the C ABI in include/hipminer.h (libhipminer.so); this
package mirrors the reference's Go interface on top of that ABI:

  bitcoin   -- Message / NewRequest / NewResult / NewJoin / Hash (message.go, hash.go)
  miner     -- Miner.eval_request: evalRoutine's Request -> Result step (miner.go)
  parallel  -- sharding over GPUs/ranks and the RCCL all-gather merge
  server_model -- the unchanged server's chunking + merge (server.go), for
                  end-to-end expectations
"""
from ._lib import Context, HipMinerError, host_hash  # noqa: F401

__all__ = ["Context", "HipMinerError", "host_hash"]
