/*
 * libpatrolhip — MI355X (gfx950) bucket-state engine for Patrol.
 *
 * A C ABI (plain pointers and sizes, no C++ types, no exceptions) that a Go
 * maintainer binds with cgo to replace Patrol's in-memory bucket map and its
 * two hot loops (INTEGRATION.md shows the binding):
 *
 *   Patrol seam (reference file:line)                 replaced by
 *   ------------------------------------------------  ------------------------------
 *   Repo interface              repo.go:15-18          phip_open / phip_get / batched calls
 *   NewLocalRepo(clock, bs...)  repo.go:179-185        phip_open + phip_seed
 *   LocalRepo.GetBucket         repo.go:189-211        device table find-or-create (inside every batch)
 *   LocalRepo.UpsertBucket      repo.go:215-235        phip_upsert_soa
 *   ReplicatedRepo.Receive loop repo.go:54-92,108-120  phip_receive_datagrams / phip_receive_soa
 *   Bucket.UnmarshalBinary      bucket.go:71-91        device decode inside phip_receive_datagrams
 *   Bucket.MarshalBinary        bucket.go:51-68        phip_marshal (host; unicast/broadcast egress)
 *   Bucket.Merge                bucket.go:240-263      device merge inside receive/upsert/apply
 *   Bucket.Take                 bucket.go:186-225      phip_take / phip_apply_mixed
 *   Bucket.IsZero               bucket.go:165-170      receive status (merge vs incast)
 *   ParseRate                   bucket.go:102-123      phip_parse_rate (host)
 *   API.takeBucket              api.go:51-86           phip_api_take (host handler logic over phip_take)
 *
 * Semantics are the Go reference's, op for op, in batch index order ("seq"):
 * a batch gives exactly the results of running the Go code on its elements
 * one after another (DESIGN.md §3 explains how the parallel kernels keep that
 * guarantee).  Buckets are identified by their full name (the FNV-1a hash is
 * only the table's probe key; names are always compared).
 *
 * Conventions
 *  - Return 0 (PHIP_OK) or a negative phip_err; never abort.  Details in
 *    phip_last_error().
 *  - Input buffers are caller-owned and only read during the call; output
 *    buffers are caller-owned.  Host pointers are staged into the library's
 *    own device buffers.  With PHIP_DEVICE_PTRS every pointer of that call
 *    (inputs and outputs) is device memory of the handle's GPU; the call then
 *    runs without host copies (the form bench.py times).
 *  - Times are int64 nanoseconds since the Unix epoch (the `clock()` reading
 *    Patrol passes around); durations are int64 ns (time.Duration).
 *  - float64 values cross the ABI as IEEE-754 bit patterns (uint64) so NaN
 *    payloads and -0.0 survive bit-exactly.
 *  - One handle per GPU; calls on a handle are serialised by an internal
 *    mutex and every entry point sets its device (cgo goroutines migrate
 *    between OS threads).
 */
#ifndef PATROLHIP_H
#define PATROLHIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PHIP_ABI_VERSION 3

/* bucket.go:36-44 */
#define PHIP_BUCKET_FIXED_SIZE 25
#define PHIP_BUCKET_PACKET_SIZE 256
/* Names are 0..PHIP_MAX_NAME_LEN bytes (bucket.go:44-48).  Host batches are
 * checked (PHIP_ERR_NAME_TOO_LARGE); a batch passed by device pointers is
 * not read on the host, so its producer guarantees the bound.  (A datagram
 * carries its name length in one byte: phip_receive_datagrams takes names
 * of up to 255 bytes, as UnmarshalBinary does, bucket.go:72-91.) */
#define PHIP_MAX_NAME_LEN 231

typedef struct phip_handle phip_handle;

typedef enum phip_err {
  PHIP_OK = 0,
  PHIP_ERR_INVALID = -1,        /* bad argument */
  PHIP_ERR_HIP = -2,            /* HIP runtime error */
  PHIP_ERR_FULL = -3,           /* table load factor limit reached */
  PHIP_ERR_ARENA = -4,          /* long-name arena exhausted */
  PHIP_ERR_SHORT_BUFFER = -5,   /* io.ErrShortBuffer from a datagram (bucket.go:72,84) */
  PHIP_ERR_NAME_TOO_LARGE = -6, /* ErrNameTooLarge (bucket.go:48) */
  PHIP_ERR_NO_DEVICE = -7,
  PHIP_ERR_IO = -8,             /* socket error (phip_udp_*; errno holds the cause) */
  PHIP_ERR_BUSY = -9,           /* ring slot not available (phip_ring_*) */
  PHIP_ERR_RCCL = -10           /* RCCL call failed (phip_group_*) */
} phip_err;

/* Per-op status codes (one uint8 per op). */
enum {
  PHIP_ST_MERGED = 1,          /* non-zero remote merged: repo.go:78-79                 */
  PHIP_ST_INCAST_REPLY = 2,    /* zero remote, existed && !local.IsZero(): repo.go:86-90 */
  PHIP_ST_INCAST_NOREPLY = 3,  /* zero remote otherwise                                  */
  PHIP_ST_SHORT = 4,           /* datagram failed UnmarshalBinary: Receive returns      */
  PHIP_ST_NOT_PROCESSED = 5,   /* after a PHIP_ST_SHORT (the Go loop has exited)        */
  PHIP_ST_TAKE_OK = 6,         /* Take returned ok=true                                 */
  PHIP_ST_TAKE_DENIED = 7,     /* Take returned ok=false (HTTP 429)                     */
  PHIP_ST_UPSERT_INSERTED = 8, /* UpsertBucket inserted the state as-is (repo.go:225-230) */
  PHIP_ST_CREATED = 0x80       /* flag: this op's GetBucket created the bucket          */
};

/* Op kinds for phip_apply_mixed. */
enum {
  PHIP_OP_TAKE = 0,     /* GetBucket + Take(now, Rate{freq, per}, count) (api.go:67-74)   */
  PHIP_OP_RECEIVE = 1,  /* received replica state (repo.go:78-90)                         */
  PHIP_OP_UPSERT = 2    /* LocalRepo.UpsertBucket of a distinct state (repo.go:215-235)   */
};

/* Call flags. */
#define PHIP_DEVICE_PTRS 0x1u   /* all pointers of the call are device memory */
#define PHIP_ROUTE_COMBINE 0x2u /* phip_route_pack: combine hot names at the sender */
#define PHIP_GROUP_RCCL_SELF 0x4u /* phip_group_receive (testing): a member's own segment also
                                     travels through RCCL (ncclSend/ncclRecv to itself) instead
                                     of a device copy, and a world-1 group exchanges through
                                     RCCL instead of merging its send buffers in place, so the
                                     per-peer RCCL exchange runs on a single GPU */
#define PHIP_GROUP_SMALL_CHUNKS 0x8u /* phip_group_receive (testing): pipeline the exchange in
                                        chunks of 4096 messages instead of 2^24, so that small
                                        batches run many pack / exchange rounds */
#define PHIP_RECV_ASYNC 0x20u /* phip_receive_soa with PHIP_DEVICE_PTRS, >= 2^16 messages: the
                                 call queues the batch and returns; the batch is finished
                                 (misses created, its dirty buckets through the ordered path,
                                 outputs final) by the handle's next call or phip_flush,
                                 which also returns its error (phip_len and phip_capacity
                                 finish it too, and leave its error to the handle's next
                                 call that returns a status).  Inputs and outputs must stay
                                 untouched until then.  A receive call queues its batch's
                                 classification and hot directory behind the batch before
                                 it, so the host's read-back of that batch overlaps them. */

/* phip_config.flags */
#define PHIP_CFG_NO_GROW 0x1u   /* refuse (PHIP_ERR_FULL / PHIP_ERR_ARENA) instead of growing */
#define PHIP_CFG_NO_SMALL 0x2u  /* ordered batches of <= 1024 host ops also take the large,
                                   multi-launch path (by default they run as one launch) */
#define PHIP_CFG_FIXED_SEED 0x4u /* place buckets with hash_seed as given (0: the unseeded
                                    placement) instead of a random per-handle seed */
#define PHIP_CFG_ISOLATE 0x8u   /* set every Receive batch's dirty buckets apart (phip_receive_soa
                                   "Order"); by default a handle does so from the first batch
                                   after one that held an incast or -0.0 field until 256
                                   clean batches in a row (a clean batch pays ~30 us for it) */

typedef struct phip_config {
  int32_t device;        /* HIP device ordinal                                          */
  uint32_t log2_slots;   /* initial table capacity = 2^log2_slots slots (4..31)         */
  uint64_t arena_bytes;  /* initial device arena for names longer than 22 bytes         */
  uint32_t max_load_pct; /* load factor that triggers growth (default 90, at most 95)  */
  uint32_t debug_tag_bits; /* 0 in production; 1..63 truncates the name hash so tests can
                              force tag collisions (names are always compared)          */
  uint32_t flags;        /* PHIP_CFG_*                                                   */
  uint32_t reserved;
  uint64_t hash_seed;    /* only with PHIP_CFG_FIXED_SEED (see "Placement" below)        */
} phip_config;
/*
 * Placement.  A bucket's tag is FNV-1a 64 of its name (also the shard map's
 * key, phip_group_*); its home slot is the top log2_slots bits of a 64-bit
 * mix of (tag ^ seed), with a seed drawn from the OS for every handle.  Go's
 * map, which the reference keeps its buckets in (repo.go:175), hashes with a
 * per-process random seed too: names chosen to collide under one placement
 * do not pile up on one probe chain under another.  Names are always
 * compared, so the seed never changes results, only where records lie.
 */
/*
 * Capacity.  Go's map never refuses a bucket (repo.go:204-207,225-227), so by
 * default the table and the long-name arena grow: before a batch creates
 * buckets, the engine reserves room for all of them (an upper bound: the
 * batch's distinct missing names) and rehashes into a table of 2x the slots
 * (k_rehash) or a larger arena whenever the reservation would pass
 * max_load_pct or the arena's end.  PHIP_ERR_FULL / PHIP_ERR_ARENA are then
 * only returned when growth is impossible (2^31 slots, device memory) or
 * disabled (PHIP_CFG_NO_GROW).  Such a refusal comes before any bucket of
 * the insert step is claimed: no bucket of the refused names is created, and
 * the table holds exactly what it held plus the merges the call's per-op
 * statuses report as applied (merges into existing buckets commute, so
 * re-submitting the other ops later is exact).
 */

/* Bucket state as Patrol holds it (bucket.go:20-32, name excluded). */
typedef struct phip_state {
  uint64_t added;    /* float64 bits */
  uint64_t taken;    /* float64 bits */
  int64_t elapsed;   /* time.Duration ns */
  int64_t created;   /* local creation time, ns since the Unix epoch */
} phip_state;

/*
 * Decoded replica states (the fields UnmarshalBinary fills, bucket.go:78-87).
 * Name i is names[name_offs[i] .. name_offs[i+1]).  With PHIP_DEVICE_PTRS the
 * names blob must stay readable 8 bytes past name_offs[n].
 *
 * names_len (the field was `reserved` before; same layout): the names blob's
 * length in bytes, or 0.  Host batches are checked on the host either way.
 * A device batch with names_len != 0 is checked on the device: every entry
 * must have name_offs[i] <= name_offs[i+1] <= names_len and at most
 * PHIP_MAX_NAME_LEN bytes.  No kernel then reads the blob at a malformed
 * entry's offsets, and the call returns PHIP_ERR_INVALID:
 *   - phip_receive_soa: the batch stops at the first malformed message k, as
 *     the Go loop stops at a short datagram (repo.go:70-74): messages before
 *     k are received as usual, k gets PHIP_ST_SHORT and every later one
 *     PHIP_ST_NOT_PROCESSED (a queued batch reports it from the call that
 *     finishes it);
 *   - phip_upsert_soa / phip_apply_mixed (phip_ops.names_len): nothing of the
 *     batch is applied.
 * With names_len == 0 a device batch's offsets are trusted: a wild offset is
 * a read of device memory the kernels do not own.  A queued batch's input
 * columns must stay untouched until it is finished (PHIP_RECV_ASYNC): a
 * column reused early reads as corrupted offsets.
 */
typedef struct phip_msgs {
  uint32_t n;
  uint32_t names_len;
  const uint8_t* names;
  const uint32_t* name_offs; /* n+1 entries */
  const uint64_t* added;     /* float64 bits */
  const uint64_t* taken;     /* float64 bits */
  const int64_t* elapsed;
} phip_msgs;

/* A mixed ordered stream (one entry per op, applied in index order). */
typedef struct phip_ops {
  uint32_t n;
  uint32_t names_len;        /* the names blob's length, or 0 (see phip_msgs)   */
  const uint8_t* kind;       /* PHIP_OP_*                                       */
  const uint8_t* names;
  const uint32_t* name_offs; /* n+1 entries                                     */
  const int64_t* now;        /* clock() reading of each op (also `created`)     */
  const int64_t* freq;       /* Rate.Freq   (TAKE)                              */
  const int64_t* per;        /* Rate.Per ns (TAKE)                              */
  const uint64_t* count;     /* n tokens    (TAKE)                              */
  const uint64_t* added;     /* float64 bits (RECEIVE/UPSERT)                   */
  const uint64_t* taken;     /* float64 bits (RECEIVE/UPSERT)                   */
  const int64_t* elapsed;    /* (RECEIVE/UPSERT)                                */
} phip_ops;

/* Per-op results (any pointer may be NULL). */
typedef struct phip_results {
  uint8_t* status;           /* PHIP_ST_* (| PHIP_ST_CREATED)                   */
  uint64_t* remaining;       /* TAKE: uint64(remaining) as Go returns it        */
  uint64_t* have;            /* TAKE: float64 bits of the value truncated       */
  phip_state* reply;         /* the bucket's state right after the op, for:
                                  TAKE: what UpsertBucket broadcasts after the take
                                        (api.go:74, repo.go:123-127);
                                  UPSERT: the upserted bucket (repo.go:123-127);
                                  RECEIVE of a zero state (incast): the local state,
                                        unchanged by it: the unicast payload of an
                                        INCAST_REPLY (repo.go:86-90), and what
                                        GetBucket found or created (repo.go:189-211).
                                  A merged replica (PHIP_ST_MERGED of a RECEIVE op)
                                  has no reply state: its entry is all zeros.       */
} phip_results;

/* ---- lifecycle ---- */
int phip_abi_version(void);
/* 16 hex digits naming the library's sources (a hash of csrc/, this header
 * and the Makefile taken when the library was built): counter profiles and
 * bench lines record it, so a measurement can be tied to the code that ran. */
const char* phip_build_id(void);
int phip_open(const phip_config* cfg, phip_handle** out);
void phip_close(phip_handle* h);
const char* phip_last_error(const phip_handle* h);
int phip_flush(phip_handle* h);                    /* hipStreamSynchronize */
/* Run every later call of this handle on `stream` (a hipStream_t of the
 * handle's device, e.g. the producer's stream of PHIP_DEVICE_PTRS inputs, so
 * that no cross-stream synchronisation is needed); NULL restores the
 * handle's own stream.  Work queued earlier is finished first. */
int phip_set_stream(phip_handle* h, void* stream);
uint64_t phip_len(phip_handle* h);                 /* number of buckets */
uint64_t phip_capacity(phip_handle* h);            /* number of slots */

/* ---- repo ---- */
/* NewLocalRepo(clock, bs...): insert (or overwrite) buckets as given. */
int phip_seed(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
              const phip_state* states, uint32_t flags);
/* Lookup without creating.  Returns 1 found, 0 absent, <0 error. */
int phip_get(phip_handle* h, const uint8_t* name, uint32_t len, phip_state* out);
/* Dump every bucket (unordered).  Call with names==NULL to size: *n_out and
 * *names_bytes_out are filled.  name_offs has n+1 entries. */
/* Snapshot / restore (the reference has none and recovers a
 * restarted node through incast, repo.go:96-106).  phip_snapshot writes
 * phip_snapshot_bytes(h) bytes into a host buffer: a 64-byte header (magic
 * "PHIPSNP1", ABI version, log2_slots, bucket count, arena bytes), the 2^L
 * slot records as they lie in HBM (64 B each), then the used long-name arena.
 * phip_restore loads such an image into a handle opened with the same
 * log2_slots (and an arena at least as large): the table is reproduced
 * exactly, with no rehash.  phip_dump + phip_seed is the portable route
 * between different table sizes. */
uint64_t phip_snapshot_bytes(phip_handle* h);
int phip_snapshot(phip_handle* h, uint8_t* out, uint64_t cap);
int phip_restore(phip_handle* h, const uint8_t* in, uint64_t len);

/* Egress batching (replaces the per-peer, per-take marshal of
 * repo.go:129-158 broadcast and :160-169 unicast): the current state of each
 * named bucket as its byte-identical MarshalBinary datagram (bucket.go:51-68).
 * Datagram i is out[25*i + (name_offs[i] - name_offs[0])], 25 + len_i bytes
 * long, so `out` holds 25*n + name bytes and the datagrams are back to back
 * in the order given (ready for one sendmmsg).  found[i] = 1 when the bucket
 * exists; an absent bucket's datagram bytes are zero.  Host or device
 * pointers (PHIP_DEVICE_PTRS). */
int phip_export_datagrams(phip_handle* h, const uint8_t* names, const uint32_t* name_offs,
                          uint32_t n, uint8_t* out, uint8_t* found, uint32_t flags);
int phip_dump(phip_handle* h, uint8_t* names, uint64_t names_cap, uint64_t* name_offs,
              phip_state* states, uint64_t max_n, uint64_t* n_out, uint64_t* names_bytes_out);

/* ---- hot path ---- */
/* ReplicatedRepo.Receive over n raw datagrams (byte-identical wire format,
 * bucket.go:59-64): bytes[offs[i] .. offs[i+1]).  `now` is the clock reading
 * used for buckets created by this batch.  Stops at the first malformed
 * datagram like the Go loop (repo.go:72-73): *stop_index receives its index
 * (or n) and the call returns PHIP_ERR_SHORT_BUFFER when one was found.
 * With PHIP_DEVICE_PTRS, `bytes` must be 8-byte aligned and readable up to
 * the next 8-byte boundary past offs[n] (the fast path reads the datagrams
 * in place as aligned words). */
int phip_receive_datagrams(phip_handle* h, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                           int64_t now, const phip_results* res, uint32_t* stop_index,
                           uint32_t flags);
/* The same loop over pre-decoded states.
 * Order: a message's result depends only on the earlier messages naming its
 * bucket (repo.go:77-106), and only incasts (a zero state) and -0.0 fields
 * make that order visible.  A batch with at most 4096 such "dirty" messages,
 * each named in at most 14 bytes, has its other buckets merged in one
 * order-free pass and only its dirty buckets' sequences (each dirty message,
 * and one merge of the clean messages between two of them) applied in order
 * afterwards (phip_kernels.hpp "Dirty buckets"; phip_receive_datagrams
 * alike).  Larger dirty sets apply everything from the first dirty message
 * on in order.  The results are the Go loop's either way. */
int phip_receive_soa(phip_handle* h, const phip_msgs* m, int64_t now, const phip_results* res,
                     uint32_t flags);
/* LocalRepo.UpsertBucket for each state, in order. */
int phip_upsert_soa(phip_handle* h, const phip_msgs* m, int64_t now, const phip_results* res,
                    uint32_t flags);
/* Ordered mixed stream of TAKE / RECEIVE / UPSERT ops. */
int phip_apply_mixed(phip_handle* h, const phip_ops* ops, const phip_results* res, uint32_t flags);
/* All-TAKE convenience form of phip_apply_mixed. */
int phip_take(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
              const int64_t* now, const int64_t* freq, const int64_t* per, const uint64_t* count,
              uint64_t* remaining_out, uint8_t* ok_out, uint32_t flags);

/* ---- host helpers (no device work) ---- */
/* ParseRate: returns 0 or <0 on error; freq and per receive the values Go
 * returns beside the error (api.go:61 uses them). */
int phip_parse_rate(const char* s, uint32_t len, int64_t* freq, int64_t* per);
/* MarshalBinary: writes 25+len bytes to out (>= 256 bytes), returns the size
 * or PHIP_ERR_NAME_TOO_LARGE. */
int phip_marshal(const uint8_t* name, uint32_t len, const phip_state* s, uint8_t* out);
/* API.takeBucket (api.go:51-86) over this engine: returns the HTTP status
 * code (200/429/400) and writes the response body (<= 64 bytes). */
int phip_api_take(phip_handle* h, const uint8_t* name, uint32_t len, const char* rate,
                  uint32_t rate_len, const char* count, uint32_t count_len, int64_t now,
                  char* body, uint32_t* body_len);

/* ---- request-coalescing Take batcher ----
 * Replaces the per-request GetBucket -> Take -> UpsertBucket of the HTTP
 * handler (api.go:67-74; Bucket.Take bucket.go:186-225) for callers that
 * serve one request per thread (a Go goroutine per HTTP request calling
 * through cgo).  Each call enqueues one Take and blocks until its batch ran:
 * a dispatcher thread closes a batch window_us after the batch's first
 * request arrived, or at max_batch requests, and runs it with
 * phip_apply_mixed (arrival order = op order, so each bucket sees its Takes
 * in the order they were enqueued).  Requests arriving while a batch runs
 * form the next one.  Thread-safe; the handle must not be closed before the
 * batcher. */
typedef struct phip_batcher phip_batcher;
typedef struct phip_batcher_config {
  uint32_t window_us;   /* batch window after its first request (0: dispatch at once)  */
  uint32_t max_batch;   /* requests per batch at most (0: 65536)                       */
} phip_batcher_config;
int phip_batcher_open(phip_handle* h, const phip_batcher_config* cfg, phip_batcher** out);
/* Runs the requests already queued, then stops the dispatcher. */
void phip_batcher_close(phip_batcher* b);
/* GetBucket + Take(now, Rate{freq, per}, count): *remaining and *ok as Go's
 * Take returns them (ok = 1 means HTTP 200, 0 means 429).  *seq (optional)
 * receives the request's arrival number: the requests of a batcher took
 * effect exactly as Go running them one by one in seq order. */
int phip_batcher_take(phip_batcher* b, const uint8_t* name, uint32_t len, int64_t now,
                      int64_t freq, int64_t per, uint64_t count, uint64_t* remaining,
                      uint8_t* ok, uint64_t* seq);
/* API.takeBucket (api.go:51-86) through the batcher: phip_api_take's
 * contract (HTTP status 200/429/400, body <= 64 bytes). */
int phip_batcher_api_take(phip_batcher* b, const uint8_t* name, uint32_t len, const char* rate,
                          uint32_t rate_len, const char* count, uint32_t count_len, int64_t now,
                          char* body, uint32_t* body_len);
/* out[0] batches run, out[1] requests served, out[2] largest batch,
 * out[3] ns spent in phip_apply_mixed, out[4] batches that failed.
 * Returns the number written (<= 5). */
int phip_batcher_stats(phip_batcher* b, uint64_t* out, int max);
/* Everything the reference handler does after GetBucket -> Take ->
 * UpsertBucket (api.go:67-74), from the same batched launch: whether the
 * Take's GetBucket created the bucket (ReplicatedRepo.GetBucket then sends
 * its zero-state incast request, repo.go:96-106: datagram bytes [24, len)
 * with 24 zero bytes in front) and the MarshalBinary datagram of the state
 * right after the Take, which UpsertBucket broadcasts (repo.go:123-158). */
typedef struct phip_take_reply {
  uint64_t remaining;      /* uint64(remaining) as Take returns it (the HTTP body)          */
  uint8_t ok;              /* 1: HTTP 200, 0: 429                                            */
  uint8_t created;         /* this request's GetBucket created the bucket                    */
  uint16_t datagram_len;   /* 25 + len(name); 0 when nothing was taken (HTTP 400)           */
  uint32_t reserved;
  uint64_t seq;            /* arrival number (phip_batcher_take)                             */
  phip_state state;        /* the bucket right after the Take                                */
  uint8_t datagram[PHIP_BUCKET_PACKET_SIZE]; /* MarshalBinary(state) (bucket.go:51-68)       */
} phip_take_reply;
int phip_batcher_take_reply(phip_batcher* b, const uint8_t* name, uint32_t len, int64_t now,
                            int64_t freq, int64_t per, uint64_t count, phip_take_reply* out);
/* API.takeBucket (api.go:51-86) through the batcher, as phip_batcher_api_take,
 * plus *out for the replication it triggers (out->datagram_len = 0 on 400). */
int phip_batcher_api_take_reply(phip_batcher* b, const uint8_t* name, uint32_t len,
                                const char* rate, uint32_t rate_len, const char* count,
                                uint32_t count_len, int64_t now, char* body, uint32_t* body_len,
                                phip_take_reply* out);

/* ---- batched UDP ingest (command.go's replicator) ----
 * The reference's Receive goroutine reads ONE datagram per iteration into a
 * 256-byte buffer under a 3 s deadline (repo.go:54-73,108-120) and answers
 * each incast with its own WriteTo (repo.go:86-90,160-169).  The batched
 * pipeline is:
 *
 *   phip_ring_acquire      a free pinned host slot (bytes + offs arrays)
 *   phip_udp_recv_batch    recvmmsg straight into that slot
 *   phip_ring_submit       hipMemcpyAsync of the slot on the ring's copy
 *                          stream (returns at once; the next slot can be
 *                          filled while this one is copied and merged)
 *   phip_ring_receive      the handle's stream waits for the copy, then
 *                          phip_receive_datagrams over the device copy;
 *                          results land in host buffers; the slot is freed
 *   phip_incast_replies +  MarshalBinary of the batch's INCAST_REPLY states
 *   phip_udp_send_batch    and one sendmmsg back to their peers
 *
 * Peers are sockaddr_storage records (PHIP_PEER_BYTES each). */
#define PHIP_PEER_BYTES 128

typedef struct phip_ring phip_ring;
/* nslots pinned slots of max_msgs datagrams / max_bytes bytes each (max_bytes
 * >= 256 * max_msgs lets phip_udp_recv_batch fill a slot to max_msgs). */
int phip_ring_open(phip_handle* h, uint32_t nslots, uint32_t max_msgs, uint64_t max_bytes,
                   phip_ring** out);
void phip_ring_close(phip_ring* r);
/* The next slot in ring order, if it is free (PHIP_ERR_BUSY: that slot is
 * still submitted and not yet received).  *bytes / *offs are pinned host
 * arrays of max_bytes and max_msgs + 1 entries; the caller writes datagram i
 * to bytes[offs[i] .. offs[i+1]) with offs[0] = 0. */
int phip_ring_acquire(phip_ring* r, uint32_t* slot, uint8_t** bytes, uint64_t** offs);
/* Start the host->device copy of the slot's first n datagrams. */
int phip_ring_submit(phip_ring* r, uint32_t slot, uint32_t n);
/* ReplicatedRepo.Receive over a submitted slot (phip_receive_datagrams
 * semantics; res holds host pointers) and release the slot.  Slots must be
 * received in the order they were submitted. */
int phip_ring_receive(phip_ring* r, uint32_t slot, int64_t now, const phip_results* res,
                      uint32_t* stop_index);

/* recvmmsg up to max_msgs datagrams from fd: waits up to timeout_ms for the
 * first (a timeout returns PHIP_OK with *n_out = 0, as the Go loop continues
 * on a Timeout error), then takes what is queued without waiting.  Each
 * datagram is cut at PHIP_BUCKET_PACKET_SIZE bytes (Go's read buffer) and
 * packed back to back: datagram i is bytes[offs[i] .. offs[i+1]), offs[0] = 0.
 * peers (optional) receives each sender's address. */
int phip_udp_recv_batch(int fd, uint8_t* bytes, uint64_t cap, uint64_t* offs, uint32_t max_msgs,
                        uint8_t* peers, int timeout_ms, uint32_t* n_out);
/* MarshalBinary (bucket.go:51-68) of reply[i] under datagram i's name for
 * every message whose status is PHIP_ST_INCAST_REPLY, in batch order, packed
 * into out / out_offs (as phip_udp_recv_batch packs); out_peers (optional)
 * receives the matching peers[i]. */
int phip_incast_replies(const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                        const uint8_t* status, const phip_state* reply, const uint8_t* peers,
                        uint8_t* out, uint64_t cap, uint64_t* out_offs, uint8_t* out_peers,
                        uint32_t* n_out);
/* sendmmsg datagrams bytes[offs[i] .. offs[i+1]) for i < n, datagram i to
 * peers + i * peer_stride (stride 0: every datagram to one peer, e.g. an
 * egress batch from phip_export_datagrams; peers NULL: a connected socket). */
int phip_udp_send_batch(int fd, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                        const uint8_t* peers, uint32_t peer_stride, uint32_t* sent_out);

/* ---- shard layer ---- */
/* FNV-1a 64 of each name (the table's probe key; also the shard map:
 * owner = ((hash >> 32) * world) >> 32).  Host pointers need no GPU (h may be
 * NULL); with PHIP_DEVICE_PTRS the hashes are computed on h's GPU. */
int phip_hash_names(phip_handle* h, const uint8_t* names, const uint32_t* name_offs, uint32_t n,
                    uint64_t* out, uint32_t flags);

/* Owner routing, the exchange step of a sharded merge: the n
 * decoded messages of m are stable-partitioned by owner = ((FNV-1a(name) >>
 * 32) * world) >> 32 into owner-major send buffers (send_* have n entries,
 * send_names holds every name byte; names are packed back to back, so
 * send_lens carries their lengths).  counts[o] / name_bytes[o] (world
 * entries, device memory) receive each owner's message and byte counts: the
 * splits of the all-to-all that moves the segments to their owners.  Device
 * pointers only; world <= 64.
 *
 * With PHIP_ROUTE_COMBINE (SURVEY §8e "sender-side combine"), a batch of
 * >= 2^20 messages with no incast and no -0.0 field has the messages of its
 * hottest names (a sampled directory of <= 512 short names) max-combined
 * per workgroup: each workgroup sends one message per hot name it saw,
 * carrying the field-wise maxima (NaN for a float field no message of the
 * group raised), after its other messages.  Merging that message equals
 * merging the ones it replaces (merges commute in that domain); messages
 * whose three fields are all <= 0 or NaN are never combined, so a combined
 * message is never an incast.  counts / name_bytes then describe the
 * combined buffers (never more than without the flag).  A dirty or smaller
 * batch is packed exactly as without the flag. */
int phip_route_pack(phip_handle* h, const phip_msgs* m, uint32_t world, uint8_t* send_names,
                    uint32_t* send_lens, uint64_t* send_added, uint64_t* send_taken,
                    int64_t* send_elapsed, uint64_t* counts, uint64_t* name_bytes,
                    uint32_t flags);

/* Anti-entropy over simulated replicas (BASELINE configs[4]).  `replicas`
 * holds nrep replicas of nbuckets buckets, each as three int64 planes
 * [r][0..2][i]: E codes (the order-preserving key of the engine, mirrored by
 * patrol_amd.shard.e_encode) of added and taken, then elapsed ns.  Device
 * pointers only (flags must include PHIP_DEVICE_PTRS).
 * phip_ae_local_max writes out[3][nbuckets], the field-wise join of the local
 * replicas in signed form (E ^ 2^63 for the float planes; a NaN replica value
 * never wins, as Go's `<` never adopts one), ready for an RCCL all-reduce(MAX)
 * across GPUs.  phip_ae_apply then sets every local replica to
 * max(own, joined): Bucket.Merge (bucket.go:240-263) of every replica into
 * every other one, a replica's own NaN sticking. */
int phip_ae_local_max(phip_handle* h, const int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                      int64_t* out, uint32_t flags);
int phip_ae_apply(phip_handle* h, int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                  const int64_t* joined, uint32_t flags);
/* The join of one GPU's replicas with no exchange: phip_ae_local_max then
 * phip_ae_apply in one pass (each field read once, written only where the
 * join raises it).  What phip_group_anti_entropy runs in a world of one. */
int phip_ae_join(phip_handle* h, int64_t* replicas, uint32_t nrep, uint64_t nbuckets,
                 uint32_t flags);

/* ---- shard group: owner routing and anti-entropy over RCCL ----
 * A group is the set of GPUs the buckets are hash-sharded over (owner =
 * ((FNV-1a(name) >> 32) * world) >> 32), each GPU one table (a phip_handle)
 * and one rank of an RCCL communicator (xGMI between the GPUs of a node).
 * It replaces the single-table Receive loop (repo.go:54-92) of one node by a
 * sharded one, with no Python or torch on the path:
 *   - phip_group_open_all: one process driving n GPUs (ncclCommInitAll); the
 *     group opens and owns a handle per GPU (cfg->device is ignored).  A
 *     device listed more than once (all entries the same device) gives n
 *     shards on that one GPU, which exchange by device copies instead of
 *     RCCL (RCCL takes one rank per device): the same packing, segments and
 *     merge order, to rehearse an n-GPU group on one;
 *   - phip_group_open_rank: one process per GPU (ncclCommInitRank) around the
 *     caller's handle; rank 0 makes the id with phip_group_unique_id and the
 *     caller hands it to every rank by its own means.
 * Calls taking one argument per local member (index i = local member i) run
 * the members concurrently, one host thread each. */
#define PHIP_GROUP_ID_BYTES 128
typedef struct phip_group phip_group;
int phip_group_unique_id(uint8_t* id /* PHIP_GROUP_ID_BYTES */);
int phip_group_open_all(const phip_config* cfg, const int32_t* devices, uint32_t n,
                        phip_group** out);
int phip_group_open_rank(phip_handle* h, const uint8_t* id, uint32_t nranks, uint32_t rank,
                         phip_group** out);
/* Destroys the communicators, and the handles phip_group_open_all opened. */
void phip_group_close(phip_group* g);
const char* phip_group_last_error(const phip_group* g);
uint32_t phip_group_world(const phip_group* g);
uint32_t phip_group_local(const phip_group* g);          /* local members */
phip_handle* phip_group_handle(phip_group* g, uint32_t i);
/* Owner-routed Receive (the C4 step): batches[i] (device pointers on member
 * i's GPU, as phip_receive_soa takes them) are the messages that arrived at
 * member i, addressed to buckets of every shard.  Each member packs its batch
 * by owner (phip_route_pack; PHIP_ROUTE_COMBINE max-combines a clean batch's
 * hot names at the sender), the members exchange the packed segments (one
 * all-to-all of the split sizes, then grouped send/recv per column), and
 * every owner merges what it received (phip_receive_soa, `now` for buckets
 * it creates).  The pack, the exchange and the merge are pipelined by chunks
 * of 2^24 messages (while chunk k travels, the pack of chunk k+1 and the
 * owner's merge of chunk k-1 run); an owner merges chunk by chunk (one
 * phip_receive_soa each), sources in rank order within a chunk, every
 * source's messages in their order (as peers' datagrams interleave in
 * Patrol: per-bucket order from one source is kept).  Every member runs the
 * longest batch's number of rounds (a shorter batch sends empty chunks).  sent[i] /
 * merged[i] (optional) receive the messages member i sent after the combine
 * and merged.  A world of one (without PHIP_GROUP_RCCL_SELF) has nothing to
 * route: the batch is merged as it came, PHIP_ROUTE_COMBINE is ignored (the
 * fast path's hot directory does what the combine would) and sent / merged
 * are the batch's raw message count. */
int phip_group_receive(phip_group* g, const phip_msgs* batches, int64_t now, uint64_t* sent,
                       uint64_t* merged, uint32_t flags);
/* Anti-entropy round over simulated replicas (BASELINE configs[4]):
 * replicas[i] holds member i's nrep replicas in phip_ae_local_max's layout
 * (device memory).  Local join (phip_ae_local_max), RCCL all-reduce(MAX) of
 * the [3, nbuckets] join across the group, phip_ae_apply: afterwards every
 * replica of every member is the CvRDT join of all of them. */
int phip_group_anti_entropy(phip_group* g, int64_t* const* replicas, uint32_t nrep,
                            uint64_t nbuckets, uint32_t flags);
/* Stage timing of the group's calls (off by default): with it on, every
 * later phip_group_receive / phip_group_anti_entropy records HIP events
 * around each chunk's work on the stream it runs on, and
 * phip_group_stage_ms reads member i's busy time of the last call per stage
 * (the sum over its chunks): ms[0] pack (phip_route_pack; the local join of
 * an anti-entropy round), ms[1] exchange (split sizes and segments over RCCL
 * or device copies; the all-reduce), ms[2] the owner's merges (the apply).
 * The stages overlap, so their sum can exceed the call.  The read
 * synchronises on the events. */
int phip_group_set_timing(phip_group* g, int on);
int phip_group_stage_ms(phip_group* g, uint32_t i, float* ms /* [3] */);
/* The RCCL member i's communicator runs on: ncclGetVersion, ncclCommCount
 * (must equal the world; 0 for a shared-device group, which has none) and
 * the path of the librccl the library's RCCL symbols resolved to (dladdr).
 * A process that loaded another librccl first (torch's, same soname
 * librccl.so.1) shares that one copy. */
int phip_group_rccl_info(phip_group* g, uint32_t i, int32_t* version, int32_t* comm_count,
                         char* lib_path, uint32_t path_cap);

/* ---- diagnostics ---- */
/* Per-kernel timing of the last hot-path call (every call since
 * phip_set_timing(h, 2) in that mode), measured with HIP events on the
 * handle's stream: writes up to max entries of (name, ms) and returns the
 * count. */
int phip_last_timings(phip_handle* h, const char** names, float* ms, int max);
/* Enable (1) or disable (0) event timing (off by default); 2 keeps the
 * timings of every later call until the next phip_set_timing, so a timed
 * loop can read them once, after it ends (the reads synchronise). */
void phip_set_timing(phip_handle* h, int on);
/* Counters of the last fast-path Receive batch: out[0] hot-directory
 * entries, out[1] messages folded through the directory, out[2] messages
 * that missed the table (inserted); out[3] table growths (rehashes) since
 * phip_open; out[4] messages of the batch that went through the ordered path
 * (the dirty buckets' sub-batch, or the suffix from the first dirty
 * message: phip_receive_soa).  Returns the number written (<= 5). */
int phip_last_stats(phip_handle* h, uint64_t* out, int max);
/* Placement quality of the table (one scan of the slots): out[0] buckets,
 * out[1] slots, out[2] the longest probe distance of a bucket from its home
 * slot, out[3] the sum of those distances.  Returns the number written
 * (<= 4) or < 0. */
int phip_table_stats(phip_handle* h, uint64_t* out, int max);

#ifdef __cplusplus
}
#endif
#endif /* PATROLHIP_H */
