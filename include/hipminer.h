/*
 * hipminer.h -- C ABI of the MI355X (gfx950) miner backend.
 *
 * Drop-in boundary for ONE hot path of alexsun705/distributed_bitcoinMiner:
 * the miner's min-hash scan.  Reference interfaces replaced (paths relative to
 * the reference root, cmu440/ = p1/src/github.com/cmu440/):
 *
 *   hm_hash  replaces  bitcoin.Hash(msg string, nonce uint64) uint64
 *                      cmu440/bitcoin/hash.go:13-17
 *   hm_scan  replaces  the scan loop of evalRoutine,
 *                      cmu440/bitcoin/miner/miner.go:46-59
 *                      (result = maxUint; index = 0; for i := lower; i < upper;
 *                       i++ { hash := bitcoin.Hash(data, i); if hash < result ...})
 *                      fed by bitcoin.Message{Data, Lower, Upper}
 *                      (cmu440/bitcoin/message.go:18-23) and producing the
 *                      values of bitcoin.NewResult(hash, nonce) (:38-44).
 *
 * The cgo binding a maintainer adds to the Go miner is in INTEGRATION.md.
 *
 * Semantics (bit-exact with the reference):
 *   - bytes hashed per nonce: msg[0..len) ‖ 0x20 ‖ decimal(nonce)   (hash.go:15)
 *   - key: first 8 bytes of SHA-256, big-endian                      (hash.go:16)
 *   - hm_scan: lexicographic min of (key, nonce) over the INCLUSIVE range
 *     [lo, hi], seeded with (UINT64_MAX, 0).  This equals the reference's
 *     ascending strict-< loop, ties to the lowest nonce.  lo > hi gives
 *     (UINT64_MAX, 0).  hi may be UINT64_MAX: the reference miner's
 *     `upper := Upper+1` wrap (miner.go:52) is NOT applied here; callers that
 *     mirror evalRoutine apply it (see distributed_bitcoinminer_amd/miner.py).
 *
 * Ownership: msg is borrowed for the call only (never retained), so a cgo
 * caller may pass Go memory.  `out` is written only when the call returns
 * HM_OK.  The context owns its device buffers and streams.
 *
 * Threading: calls on one context are serialised by an internal mutex; every
 * call re-binds its device (hipSetDevice), so Go may call from any OS thread.
 * hm_close must not race other calls on the same context (the caller owns
 * the context's lifetime, as with any C handle).
 *
 * Errors: 0 = HM_OK; negative codes below; hm_strerror() describes them.
 * Nothing aborts the process, and a failed GPU scan is reported, never
 * silently replaced.  With HM_OPT_DEADLINE_MS a scan that the GPU does not
 * finish in time returns HM_ERR_TIMEOUT instead of blocking (ABI 1.8).  hm_scan_cpu (ABI 1.7) is the host scan a caller may
 * choose when hm_open or hm_scan fails, so that a Result is still written
 * (SURVEY §8(b)); the GPU entry points never call it.
 */
#ifndef HIPMINER_H
#define HIPMINER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 16 bytes: the (hash, nonce) candidate; also the RCCL all-gather element. */
typedef struct hm_result {
    uint64_t hash;
    uint64_t nonce;
} hm_result;

typedef struct hm_ctx hm_ctx;

/* Timing and work accounting of the most recent hm_scan on a context. */
typedef struct hm_stats {
    double wall_ms;          /* host wall time of the hm_scan call              */
    double kernel_ms;        /* time during which some scan kernel ran: union of
                                the launches' HIP-event intervals, summed over
                                devices                                          */
    double dom_kernel_ms;    /* summed duration of the dominant scan kernel's
                                launches (dominant = most nonces; one kernel
                                instantiation may serve several segments)       */
    uint64_t nonces;         /* nonces covered by the call                       */
    uint64_t dom_nonces;     /* nonces covered by the dominant kernel            */
    uint64_t dom_compressions; /* SHA-256 compressions per nonce after the host
                                  midstate in the dominant kernel's segments (C
                                  of SURVEY §8d; algorithmic, before hoisting)  */
    int32_t launches;        /* scan-kernel launches issued                      */
    int32_t dom_kind;        /* HM_KIND_* of the dominant kernel                 */
    int32_t ndev;            /* devices used                                      */
    int32_t dom_grid;        /* workgroups of the dominant kernel's largest launch */
    int32_t dom_launches;    /* launches of the dominant kernel                  */
    int32_t merge;           /* HM_MERGE_*: how the per-device 16-B results were
                                merged (ABI 1.4; was reserved)                   */
    char dom_kernel[64];     /* its name as rocprofv3 lists it (without args)   */
    double dom_compressions_eff; /* SHA-256 compressions per nonce the dominant
                                  kernel executes (ABI 1.4): dom_compressions
                                  minus the work hoisted out of the per-nonce
                                  loop.  Tiled: 1 (+1 with a constant trailer
                                  block); chained: 1 + 1/tch, the per-lane block
                                  0 amortised over tch loop values (f <= 4
                                  final-block digits: tch = min(10^f, 1000);
                                  f >= 5: tch = min(10^fe, 100), fe the table
                                  digits) (counted exactly per launch since ABI
                                  1.5: one block-0 compression per task and
                                  lane, guided-split pieces included); generic:
                                  dom_compressions.  Mean over the dominant
                                  kernel's nonces (one instantiation may serve
                                  several segments). */
    double enqueue_ms;       /* host time the call spent enqueuing GPU work on
                                its devices (planning, K+W table allocation,
                                launches) before waiting for results, summed
                                over its chunks of <= 64 requests (ABI 1.6)     */
    int32_t mid_call_syncs;  /* host waits on GPU work issued while the call was
                                still enqueuing work for some device (ABI 1.6;
                                0: every device's work is queued before the
                                host waits on any, so devices overlap)          */
    int32_t table_grows;     /* chained K+W tables enlarged by the call; an old
                                table may still be read by queued work, so it
                                is kept (< 1/9 of the new one) until
                                hm_close, as hipFree would wait for the whole
                                device (1.7 freed it at the end of the call):
                                growth never waits on the device mid-enqueue
                                (ABI 1.6)                                       */
    double deadline_ms;      /* the deadline the call ran under (ABI 1.8;
                                HM_OPT_DEADLINE_MS; 0 = none)                    */
} hm_stats;

/* sizeof(hm_stats) by ABI version.  The struct only grows at its end. */
#define HM_STATS_SIZE_1_0 136 /* ABI 1.0 .. 1.3                                 */
#define HM_STATS_SIZE_1_4 144 /* ABI 1.4, 1.5: + dom_compressions_eff          */
#define HM_STATS_SIZE_1_6 160 /* ABI 1.6, 1.7: + enqueue_ms, mid_call_syncs,
                                 table_grows                                     */
#define HM_STATS_SIZE_1_8 168 /* ABI 1.8+: + deadline_ms                         */

#define HM_MERGE_NONE 0 /* one device: its result is read back directly      */
#define HM_MERGE_HOST 1 /* several devices: 16-B results merged on the host  */
#define HM_MERGE_RCCL 2 /* RCCL ncclAllGather of the 16-B results on the
                           devices, then a device-side lexicographic fold
                           (HM_OPT_MERGE_RCCL; any device count, incl. 1)    */

#define HM_OK 0
#define HM_ERR_INVALID (-1)   /* bad argument                                   */
#define HM_ERR_NO_DEVICE (-2) /* no usable HIP device / runtime                  */
#define HM_ERR_HIP (-3)       /* a HIP runtime call failed                       */
#define HM_ERR_NOMEM (-4)     /* device or host allocation failed                */
#define HM_ERR_RCCL (-5)      /* an RCCL call failed                              */
#define HM_ERR_INTERNAL (-6)  /* planner invariant violated                      */
#define HM_ERR_TIMEOUT (-7)   /* ABI 1.8: the call passed its HM_OPT_DEADLINE_MS
                                 deadline before the GPU finished.  The context
                                 is ABANDONED: its queued work may still run, so
                                 every later call on it returns HM_ERR_TIMEOUT
                                 without touching a device, and hm_close frees
                                 only host memory (device buffers and streams
                                 are left to the process exit).  `out` is not
                                 written: the caller answers from hm_scan_cpu or
                                 a new context.                                  */

#define HM_KIND_NONE 0
#define HM_KIND_GENERIC 1  /* one nonce per lane, generic tail builder          */
#define HM_KIND_TILED 2    /* tile-planned final block (lane + loop digits)      */
#define HM_KIND_CHAINED 3  /* two-block tail: per-lane block 0, table-driven final block */
#define HM_KIND_FUSED 4    /* every segment of a small request in one launch, each
                              with its own layout's task body (ABI 1.7)          */

/* Options for hm_set_option. */
#define HM_OPT_FORCE_GENERIC 1 /* 1: route every segment to the generic kernel  */
#define HM_OPT_MERGE_RCCL 2    /* 1: merge the per-device candidates with one RCCL
                                  all-gather (also with one device: a 1-rank
                                  communicator); needs distinct device ordinals:
                                  hm_set_option returns HM_ERR_INVALID for a
                                  context that names a device twice (ABI 1.5)  */
#define HM_OPT_GRID_PER_CU 3   /* workgroups per CU for scan launches (0 = auto) */
#define HM_OPT_STREAMS 4       /* HIP streams per device for segment launches
                                  (1..4, default 4): the dominant kernel's
                                  segments on a high-priority stream, the
                                  others on low-priority streams that fill
                                  its last launch's tail; 1 = strictly serial.
                                  Since ABI 1.8 hm_open makes stream 0 only and
                                  a call makes streams 1.. when it first
                                  enqueues onto them: every HIP stream holds a
                                  hardware queue until the process exits, so a
                                  process sharing its GPU sets 1 or 2        */
#define HM_OPT_TABLE_DIGITS 7  /* test hook (-1..7, 0 = default 7): the final-
                                  block digits one K+W table of the chained
                                  kernel covers; the remaining high final-block
                                  digits run as epochs (one table each).  Smaller
                                  values exercise the epochs on small ranges;
                                  -1 keeps final blocks of >= 5 digits on the
                                  tiled kernel (ABI 1.5)                        */
#define HM_OPT_TABLE_ROWS_CAP 8 /* test hook (>= 0, 0 = off): a K+W table may not
                                  grow beyond this many rows, as if the device
                                  were out of memory; the chained layout then
                                  falls back to smaller tables and more epochs
                                  (the HM_ERR_NOMEM path of table growth; ABI
                                  1.6)                                          */
#define HM_OPT_TEST_MID_SYNC 9  /* test hook (0/1): the call waits on the host for
                                  each device's first queued work while still
                                  enqueuing, which hm_stats.mid_call_syncs must
                                  count (ABI 1.7)                               */
#define HM_OPT_FUSED 10         /* 1 (default): a request (per device shard) of at
                                  most 2^27 nonces whose segments all fit the
                                  fused launch runs as ONE planner + ONE scan
                                  launch (HM_KIND_FUSED); 0: one launch per
                                  digit segment (ABI 1.7)                       */
#define HM_OPT_FUSED_FLAGS 11   /* experiment hook (0..31): how the fused launch's
                                  waves get tasks -- bit 0: first task = the
                                  wave's slot (no opening burst of queue
                                  atomics); bit 1: dequeue the next task while
                                  the current one runs; bit 2: no queue, wave
                                  slots strided over the task ids; bit 3:
                                  dequeue through the workgroup's LDS
                                  dispenser (ABI 1.7); bit 4: a wave's priority
                                  falls with the tasks it ran (ABI 1.8)         */
#define HM_OPT_FUSED_PARTS 12   /* experiment hook (1, 2, 5, 10; default 1): a
                                  tiled task of the fused launch covers 10 /
                                  parts steps of its units loop (ABI 1.7)       */
#define HM_OPT_DEADLINE_MS 13   /* ABI 1.8 (SURVEY §8(b) liveness): 0 (default) =
                                  a call blocks until its GPU work is done; > 0 =
                                  a call returns HM_ERR_TIMEOUT (and abandons the
                                  context) once this many ms have passed since it
                                  began; -1 = auto: 2 s + 8 x the call's modelled
                                  kernel time (the layouts' measured cost, the
                                  model hm_partition balances with).  The host
                                  then polls the GPU instead of blocking on it.
                                  A miner whose LSP thread keeps heartbeating
                                  would otherwise hold its chunk forever: the
                                  server reassigns only dropped miners
                                  (server.go:326-376)                           */
#define HM_OPT_FUSED_TAIL 14    /* 1, 2, 5 or 10 (default 2; ABI 1.8): the tasks
                                  of a fused launch's last, partial wave-round
                                  (tasks mod waves; the cheapest layouts, queued
                                  last) run as up to this many pieces each --
                                  as many as still fit one round of the grid --
                                  so the launch does not end on a round of
                                  whole tasks with most waves idle; 1 = no
                                  split                                        */
#define HM_OPT_TAIL_FUSED 15    /* 1 (default; ABI 1.8): the segments of a large
                                  request that its dominant kernel does not run
                                  (bradfitz [0, 2^32): d <= 8) go into ONE fused
                                  launch on a low-priority stream, in the
                                  dominant launch's tail, when they fit one; 0:
                                  one launch per segment on the tail streams */
#define HM_OPT_HOST_RESULT 16   /* experiment hook (0/1, default 0; ABI 1.8): 1 =
                                  the call's last fold kernel stores the 16-B
                                  results into pinned host memory (system-scope
                                  stores) instead of a hipMemcpyAsync readback;
                                  measured no faster                            */
#define HM_OPT_QUEUE_BATCH 17   /* experiment hook (0, 4, 8, 16, 32; ABI 1.8):
                                  tasks a workgroup fetches per work-queue
                                  atomic in the per-segment kernels; 0 (default)
                                  = 4, and 16 for launches of >= 10^11 nonces */
#define HM_OPT_FUSED_TRACE 18   /* diagnostics (0/1; ABI 1.8): fused launches on
                                  device 0 record each wave's timeline
                                  (tools/fused_trace.py)                        */

/* bitcoin.Hash (hash.go:13-17) evaluated on the host.  Not the hot path: used
 * to verify single results and for planning; needs no GPU. */
uint64_t hm_hash(const uint8_t *msg, size_t len, uint64_t nonce);

/* Open a context on `ndev` HIP devices (`devices` lists ordinals); ndev == 0
 * uses every visible device.  Returns HM_ERR_NO_DEVICE without a GPU. */
int hm_open(const int *devices, int ndev, hm_ctx **out);

/* Min-hash scan of the inclusive range [lo, hi] (see semantics above).  With
 * several devices the range is sharded contiguously and the per-device 16-B
 * candidates are merged (RCCL all-gather when HM_OPT_MERGE_RCCL is set); the
 * shards are those of hm_partition (cost-weighted). */
int hm_scan(hm_ctx *ctx, const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi,
            hm_result *out);

/* One request of a batch: the same meaning as hm_scan's arguments. */
typedef struct hm_request {
    const uint8_t *msg; /* borrowed for the call; may be NULL when len == 0 */
    size_t len;
    uint64_t lo, hi;    /* inclusive */
} hm_request;

/* Batch form of hm_scan: outs[i] = hm_scan(reqs[i]) for i < n.  All requests'
 * GPU work is enqueued before one host synchronisation (SURVEY §8(f) rank 4:
 * the server's FIFO (cmu440/bitcoin/server/server.go:211-219, 318-324) hands a
 * miner one small chunk at a time; a miner or a future GPU-side server can
 * batch them here).  outs is written only when the call returns HM_OK. */
int hm_scan_many(hm_ctx *ctx, const hm_request *reqs, int n, hm_result *outs);

/* Checked scan: hm_scan's result plus a coverage checksum computed on the GPU
 * by the checked variants of the same kernels (same planner, tiles, lane and
 * loop layout, guided task split and multi-device shards):
 *   *sum   = sum over n in [lo, hi] of Hash(msg, n), mod 2^64
 *   *count = number of nonces hashed (must be hi - lo + 1, mod 2^64)
 * A nonce skipped, hashed twice or hashed with wrong bytes changes the pair,
 * so it checks coverage at sizes no CPU can rescan; the sums of disjoint
 * sub-ranges add up to the sum of their union.  A verification entry point,
 * not the hot path: it runs slower than hm_scan. */
int hm_scan_checked(hm_ctx *ctx, const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi,
                    hm_result *out, uint64_t *sum, uint64_t *count);

/* Split the inclusive range [lo, hi] into n contiguous, ascending shards of
 * near-equal modelled GPU cost for msg (digit segments whose kernels cost more
 * per nonce get fewer nonces).  bounds[2i], bounds[2i+1] = shard
 * i's inclusive [lo, hi]; an empty shard is written as [1, 0].  The shards
 * cover [lo, hi] exactly, so per-shard hm_scan results merged by (hash, nonce)
 * minimum equal hm_scan over [lo, hi].  Host-only; needs no GPU.  This is how
 * hm_scan shards one request across a multi-device context, and what a
 * process-per-GPU caller (torch.distributed ranks, one Go miner per GPU) uses
 * to cut its range. */
int hm_partition(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int n,
                 uint64_t *bounds);

/* Stats of the last successful hm_scan / hm_scan_many on ctx: the FIRST
 * HM_STATS_SIZE_1_4 BYTES ONLY (through dom_compressions_eff), the size the
 * ABI 1.4/1.5 headers promised.  Frozen since ABI 1.7, so a binary built
 * against any header from 1.4 on never gets more bytes than its struct
 * holds (ABI 1.6 wrote 160 bytes here, past a 1.5 caller's struct).  The
 * fields after dom_compressions_eff come only from hm_scan_stats_sized.
 * A caller built against the 1.6 header that reads enqueue_ms,
 * mid_call_syncs or table_grows MUST switch to hm_scan_stats_sized (pass
 * sizeof(hm_stats)): through this export those fields are no longer
 * written and hold whatever the caller's struct held. */
int hm_scan_stats(const hm_ctx *ctx, hm_stats *out);

/* hm_scan_stats writing at most `size` bytes (pass sizeof(hm_stats) as the
 * caller compiled it; >= HM_STATS_SIZE_1_0): the prefix of the current
 * layout that fits.  ABI 1.5.  The call to use for every field. */
int hm_scan_stats_sized(const hm_ctx *ctx, hm_stats *out, size_t size);

/* The same scan as hm_scan -- lexicographic min of (Hash(msg, n), n) over
 * the INCLUSIVE [lo, hi], seeded (UINT64_MAX, 0), bit-identical -- on the
 * host's cores, without a GPU (ABI 1.7; SURVEY §8(b)'s liveness path).
 * `threads` <= 0 uses one thread per CPU this process may run on (its
 * affinity mask, at most 1024); the range is split into that many
 * contiguous chunks (ranges below 4096 nonces per thread use fewer).
 * x86 SHA extensions when the CPU has them (HM_CPU_NO_SHA=1 forces portable
 * C).  Orders of magnitude slower than hm_scan: for callers whose GPU is
 * missing or failed (hm_miner, the Go gpuminer), so a Result is still
 * written; never called by the GPU entry points.  `out` is written only on
 * HM_OK. */
int hm_scan_cpu(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                hm_result *out);

int hm_set_option(hm_ctx *ctx, int opt, int64_t value);

const char *hm_strerror(int rc);

void hm_close(hm_ctx *ctx);

/* ABI version: (major << 16) | minor. */
int hm_version(void);

/* Build identity (ABI 1.6): 16 hex digits of sha256 over the sources the
 * library was built from (distributed_bitcoinminer_amd/build_id.py: csrc/ and
 * this header, by path and content).  A caller holding the source tree can
 * check that the loaded library is that tree's build.  Static storage. */
const char *hm_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* HIPMINER_H */
