/*
 * rl_hip.h — C ABI of the MI355X-native fixed-window rate-limit backend.
 *
 * This is the drop-in boundary for the reference's hot path. It replaces
 *   limiter.RateLimitCache.DoLimit / Flush         src/limiter/cache.go:15-33
 * as implemented by the Redis backend
 *   fixedRateLimitCacheImpl.DoLimit                src/redis/fixed_cache_impl.go:31-123
 *   redis.Client.PipeAppend / PipeDo (INCRBY+EXPIRE pipeline)
 *                                                  src/redis/driver.go:13-47, fixed_cache_impl.go:26-29
 * A Go `src/hip` package binds these entry points over cgo; the C++
 * mirror of the Go interface lives in api-ratelimit_amd/csrc/rl_cache.hpp.
 *
 * Plain C types only; no exceptions cross the ABI. Every call returns 0 on success or a
 * negative RL_E* code; rl_last_error() then holds a message (the Go side turns a
 * non-zero return into panic(redis.RedisError(msg)), src/redis/driver.go:6-10, so the
 * service maps it to the redis_error stat exactly as for Redis, service/ratelimit.go:276-281).
 * All calls on one engine must come from one thread (the batch submitter).
 */
#ifndef RL_HIP_H
#define RL_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 7u

/* rule id of a descriptor whose limit is nil ("don't check", src/limiter/cache.go:19-22) */
#define RL_NIL_RULE 0xFFFFFFFFu

/* pb.RateLimitResponse_RateLimit_Unit (go-control-plane v0.9.7) */
enum { RL_UNIT_UNKNOWN = 0, RL_UNIT_SECOND = 1, RL_UNIT_MINUTE = 2, RL_UNIT_HOUR = 3, RL_UNIT_DAY = 4 };
/* pb.RateLimitResponse_Code */
enum { RL_CODE_UNKNOWN = 0, RL_CODE_OK = 1, RL_CODE_OVER_LIMIT = 2 };
/* rl_status.code_flags bits 8.. */
enum {
  RL_FLAG_HAS_LIMIT = 1u,       /* DescriptorStatus.CurrentLimit != nil and DurationUntilReset set */
  RL_FLAG_LOCAL_CACHE_HIT = 2u, /* over limit via the local cache: add over_limit_delta to
                                   OverLimitWithLocalCache too (base_limiter.go:76-81) */
  RL_FLAG_SHADOW = 4u           /* extension (rule with RL_RULE_SHADOW): the descriptor was over its limit
                                   and is reported OK; add 1 to Stats.ShadowMode. Counters, local cache,
                                   limit_remaining and the over/near deltas are those of the OVER_LIMIT decision */
};

/* error codes */
enum {
  RL_OK = 0,
  RL_EINVAL = -1,    /* bad argument / malformed batch */
  RL_EHIP = -2,      /* HIP runtime error */
  RL_ENOSPC = -3,    /* a counter-table region would pass its load limit: the batch was refused before
                        any counter changed (raise log2_slots / max_load_permille) */
  RL_ECAPACITY = -4, /* batch larger than the engine was created for */
  RL_ESTATE = -5,    /* call out of order (e.g. rl_wait without rl_submit) */
  RL_EDEVICE = -6,   /* device-side fault detected (bounded spin expired) */
  RL_EPEER = -7,     /* rl_router_step: another shard failed this step (its code in rl_router_stats) */
  RL_ECOMM = -8,     /* rl_router: RCCL error */
  RL_ELATE = -9      /* rl_router: this shard's origin batch starts more than 3 s behind the step clock; none of
                        its descriptors was applied (the other shards' steps went ahead: a clock-skew signal,
                        counted in rl_router_stats.late_steps) */
};

typedef struct rl_engine rl_engine;

/* Engine configuration (REDIS_* settings analogues, src/settings/settings.go:10-48). */
typedef struct rl_config {
  uint32_t struct_size;        /* = sizeof(rl_config) */
  int32_t device;              /* HIP device ordinal (HIP_DEVICES) */
  uint32_t log2_slots[4];      /* table slots per window generation of the key strings whose home unit is
                                  SECOND/MINUTE/HOUR/DAY (HIP_TABLE_SLOTS) */
  float near_limit_ratio;      /* NEAR_LIMIT_RATIO, default 0.8 (settings.go:44) */
  uint32_t local_cache;        /* 1 = local over-limit cache on (LOCAL_CACHE_SIZE_IN_BYTES > 0, settings.go:45) */
  uint32_t per_second_split;   /* REDIS_PERSECOND (settings.go:35): SECOND keys count in their own store; else
                                  one store holds every unit and same-string keys share a counter */
  uint32_t max_batch_desc;     /* capacity: descriptors per batch (HIP_BATCH_LIMIT) */
  uint32_t max_batch_req;      /* capacity: requests per batch */
  uint32_t max_blob_bytes;     /* capacity: key-prefix bytes per batch */
  uint32_t sort_bits;          /* LSD pipeline: fingerprint bits radix-sorted per batch (8..64, multiple of 8; 0 = 48) */
  uint32_t flags;              /* RL_CFG_* */
  uint64_t hash_seed;          /* fingerprint seed: one value for every engine of a deployment (multi-GPU
                                  owners must agree), secret against hash flooding */
  uint32_t max_load_permille;  /* load limit per table region, 100..950 (0 = 750): a batch that could push a
                                  region past it is refused with RL_ENOSPC before anything changes */
  uint32_t reserved;           /* 0 */
} rl_config;

/* rl_config.flags */
enum {
  RL_CFG_LSD_ONLY = 1u,  /* always use the LSD radix-sort pipeline (default: v4 pipeline, LSD as fallback) */
  RL_CFG_LAG_WINDOW = 2u /* keep a SECOND key string findable for requests up to 3 s behind the newest time the
                            table has seen, at up to twice the SECOND regions' live slots against the same load
                            limit. rl_router_create turns it on for its engines (origins' clocks differ); a lone
                            engine fed in enqueue order does not need it */
};

/* One rate-limit rule: config.RateLimit.Limit (src/config/config.go:26-32). */
typedef struct rl_rule {
  uint32_t requests_per_unit;
  uint32_t unit; /* RL_UNIT_SECOND..RL_UNIT_DAY, optionally | RL_RULE_SHADOW; anything else is RL_EINVAL
                    (utilities.go:31 panics) */
} rl_rule;
/* Shadow mode (BASELINE config 4; an extension: this fork has none, config_impl.go:49-59 rejects a
 * shadow_mode key). A rule whose unit carries this bit never answers OVER_LIMIT: such a decision
 * is reported as RL_CODE_OK with RL_FLAG_SHADOW, everything else unchanged (envoyproxy/ratelimit's
 * later `shadow_mode`: counters still increment, the local cache still freezes the key, over/near
 * stats still count). Parity unpinned by a reference fixture. */
#define RL_RULE_SHADOW 0x100u

/* A batch of requests in serial (enqueue) order. Descriptor i belongs to request req_of[i]
 * (non-decreasing). Its cache-key prefix is the exact byte string
 *   domain '_' key1 '_' value1 '_' ... keyN '_' valueN '_'
 * of GenerateCacheKey (src/limiter/cache_key.go:57-65) without the window timestamp, which
 * the device appends (cache_key.go:66-68): bytes prefix_blob[prefix_off[i] .. prefix_off[i+1]).
 * The same struct carries host pointers (rl_submit) or device pointers (rl_submit_device).
 * A device prefix_blob must be readable (not meaningful) for RL_BLOB_SLACK bytes past
 * blob_bytes, non-null even when every prefix is empty: the device reads prefixes in 16-B
 * words. Host batches need no slack (rl_submit stages them with it). A batch with
 * descriptors has at least one request. */
#define RL_BLOB_SLACK 32
typedef struct rl_batch {
  uint32_t n_desc;
  uint32_t n_req;
  uint32_t blob_bytes;
  uint32_t reserved;
  const uint8_t* prefix_blob;
  const uint32_t* prefix_off;  /* n_desc + 1 entries */
  const uint32_t* rule_id;     /* n_desc, RL_NIL_RULE for a nil limit */
  const uint32_t* req_of;      /* n_desc */
  const int64_t* now;          /* n_req: unix seconds, one per request (TimeSource.UnixNow) */
  const uint32_t* hits_addend; /* n_req: RateLimitRequest.HitsAddend (0 means 1, fixed_cache_impl.go:39) */
  const uint16_t* ttl_jitter;  /* n_desc or NULL (= all 0): seconds added to the EXPIRE of the descriptor's
                                  INCRBY, JitterRand.Int63n(EXPIRATION_JITTER_MAX_SECONDS) drawn by the host in
                                  serial order (fixed_cache_impl.go:69-72); the key lives until its last INCRBY's
                                  now + divider + jitter. Ignored for nil limits and local-cache hits.
                                  Draw order: the reference draws no jitter for a local-cache hit
                                  (fixed_cache_impl.go:60-72); the device cache's hits are known only
                                  after the batch, so a host drawing one per descriptor with a limit
                                  matches the reference's sequence of draws only with the local cache
                                  off or with HIP_LOCAL_CACHE=freecache (its hits are found on the
                                  host, before the draws). Each INCRBY's jitter is still one
                                  independent draw (tests/test_jitter.py pins the current behaviour) */
} rl_batch;

/* One DescriptorStatus plus its stat increments (20 B). */
typedef struct rl_status {
  uint32_t code_flags;       /* RL_CODE_* | RL_FLAG_* << 8 */
  uint32_t limit_remaining;  /* DescriptorStatus.LimitRemaining */
  uint32_t reset_s;          /* DescriptorStatus.DurationUntilReset.Seconds (0 if no limit) */
  uint32_t over_limit_delta; /* add to Stats.OverLimit (and OverLimitWithLocalCache if LOCAL_CACHE_HIT) */
  uint32_t near_limit_delta; /* add to Stats.NearLimit */
} rl_status;
/* Stats.TotalHits is incremented by max(1, HitsAddend) for every non-nil limit on the host
 * (base_limiter.go:49-51); it needs no device round trip. */

typedef struct rl_engine_stats {
  uint64_t batches;           /* batches completed */
  uint64_t descriptors;       /* descriptors decided */
  uint64_t resorts;           /* batches re-sorted on the full fingerprint after a sort-prefix collision */
  uint64_t inserted_keys;     /* table slots claimed since creation (one per key string and window) */
  uint64_t lsd_fallbacks;     /* batches the bucketed pipeline handed to the LSD pipeline */
  uint64_t hot_keys;          /* size of the hot-key set used by the last batch */
  uint64_t live_keys;         /* slots of the current window generations, all regions (after the last batch) */
  uint64_t host_batches;      /* batches submitted from host memory (rl_submit) */
} rl_engine_stats;

/* Occupancy of the 8 table regions (home unit x window parity) after the last completed batch. */
typedef struct rl_occupancy {
  uint32_t gen[8];    /* window generation the count belongs to (home window index + 1; 0 = unused) */
  uint32_t live[8];   /* slots claimed for that generation */
  uint32_t limit[8];  /* load limit (slots) */
  uint32_t slots[8];  /* region size */
} rl_occupancy;

int rl_create(const rl_config* cfg, rl_engine** out);
void rl_destroy(rl_engine* e);
/* The engine's last error message; with e == NULL, the calling thread's last rl_create
 * failure (which HIP call failed and why). */
const char* rl_last_error(const rl_engine* e);
uint32_t rl_abi_version(void);

/* Load the rule table; rule ids index it. While batches are in flight the new table must keep
 * every loaded rule at its id and may only append (RL_ESTATE otherwise): in-flight batches read
 * rules by id, and the appended entries are written to slots none of them reads. A micro-batcher
 * whose rule registry only grows (new (L, unit) pairs from a config reload or a descriptor.Limit
 * override, src/config/config_impl.go:281-289) can therefore load at any time. Replacing or
 * dropping rules needs nothing in flight. */
int rl_load_rules(rl_engine* e, const rl_rule* rules, uint32_t n);

/* Batches that may be in flight at once (rl_submit, rl_submit_pipelined). */
#define RL_MAX_IN_FLIGHT 3

/* ---- Host-memory batches (the Go micro-batcher's path) ---------------------------------
 * Up to RL_MAX_IN_FLIGHT host batches are in flight: each has its own pinned staging slot,
 * its H2D copies run on a copy stream while the previous batch's kernels run, and its D2H
 * copies on another while the next batch's run.
 *
 * rl_host_acquire returns the next free staging slot: pinned host arrays (C memory, so a cgo
 * caller fills them through unsafe slices without passing Go pointers) with their
 * capacities. rl_submit takes a batch whose arrays are that slot's (no copy) or any host
 * memory (copied into the slot before rl_submit returns: the caller's arrays are free again).
 * out[n_desc] / req_throttle_ms[n_req] (DoLimitResponse.ThrottleMillis, base_limiter.go:163-165)
 * may be NULL: the results then stay in the engine until rl_wait_into copies them out
 * (the cgo-safe form: Go memory is only touched during that call); non-NULL C memory is
 * filled by rl_wait and must stay valid until then. Completion is in submission order. */
typedef struct rl_host_batch {
  uint8_t* prefix_blob;
  uint32_t* prefix_off;
  uint32_t* rule_id;
  uint32_t* req_of;
  int64_t* now;
  uint32_t* hits_addend;
  uint16_t* ttl_jitter;  /* the slot's jitter array: pass it as rl_batch.ttl_jitter to use it */
  uint32_t max_desc, max_req, max_blob, reserved;
} rl_host_batch;
int rl_host_acquire(rl_engine* e, rl_host_batch* out);
int rl_submit(rl_engine* e, const rl_batch* batch, rl_status* out, uint32_t* req_throttle_ms);
/* Complete the oldest batch in flight (any submit form). */
int rl_wait(rl_engine* e);
/* Non-blocking: 1 if the oldest batch in flight is done on the device (rl_wait would not block on
 * it, barring a rerun the device asked for), 0 if not yet, RL_ESTATE with nothing in flight. A
 * batcher gathering its next batch polls it to answer the callers of the batch in flight as soon
 * as they can be answered (no counterpart in the reference: radix's pipelining answers each
 * command as its reply arrives, src/redis/driver_impl.go:84-89). */
int rl_query(rl_engine* e);
/* Complete the oldest batch in flight, copying its results into out[n_desc] and
 * req_throttle_ms[n_req] (a host batch's, or NULL to discard). */
int rl_wait_into(rl_engine* e, rl_status* out, uint32_t* req_throttle_ms);
/* Complete the oldest batch in flight, a host batch (rl_submit) whose outputs were NULL, and
 * hand out its results where they landed: its staging slot's pinned arrays (C memory; a cgo
 * caller reads them through unsafe slices, no copy). *out holds n_desc statuses and
 * *req_throttle_ms n_req words. They stay valid until the slot is reused: until the batch
 * submitted RL_MAX_IN_FLIGHT places after this one is submitted (a caller that keeps two
 * batches in flight and collects one after each submit may read them until its next submit
 * after this call returns). A device batch, or a host batch submitted with output pointers,
 * gives RL_ESTATE (nothing completed).
 * Replaces the copy of rl_wait_into for a batcher that answers its callers straight from the
 * slot (DoLimit's []*DescriptorStatus, src/redis/fixed_cache_impl.go:108-123). */
int rl_wait_view(rl_engine* e, const rl_status** out, const uint32_t** req_throttle_ms);

/* ---- Compact host batches (the PCIe wire format of a Go batcher) ------------------------
 * The same batch as rl_batch in fewer bytes: per descriptor the prefix bytes plus ONE word
 *   desc_word[i] = prefix_len (bits 0-15) | rule_id (bits 16-31; RL_NIL_RULE16 = nil limit)
 * (prefixes lie back to back in prefix_blob, so their offsets are implicit), per request ONE word
 *   req_word[r]  = hits_addend (bits 0-23; 0 means 1) | (now - now_base) (bits 24-31)
 * and the request index of each descriptor only when requests hold several descriptors
 * (req_of; NULL with RL_BC_ONE_PER_REQ: descriptor i belongs to request i). At one descriptor
 * per request that is len(prefix) + 8 bytes per descriptor against len(prefix) + 24 for
 * rl_batch. A batch whose rule ids reach 0xFFFF, whose prefixes pass 65535 bytes, whose
 * hits_addend pass 2^24 - 1 or whose request times span more than 255 s goes through rl_submit.
 * The device expands the words into the rl_batch arrays (a kernel on the copy stream) and runs
 * the pipeline unchanged.
 * Results come back as raw replies, 8 B per descriptor: the INCRBY post-value each descriptor
 * saw, or its local-cache hit, or nil — what Redis answers the reference's DoLimit
 * (fixed_cache_impl.go:91-102) plus the local-cache verdict (base_limiter.go:57-66). The status
 * is then made on the host by the unchanged BaseRateLimiter logic (GetResponseDescriptorStatus,
 * base_limiter.go:70-195): rl_decide_raw in C, or the Go service's own BaseRateLimiter. */
#define RL_NIL_RULE16 0xFFFFu
#define RL_RAW_NIL 2u /* rl_raw_reply.flags: a nil-limit descriptor (no INCRBY) */
enum { RL_BC_ONE_PER_REQ = 1u /* req_of is implicit: descriptor i belongs to request i (n_desc == n_req) */ };
typedef struct rl_batch_c {
  uint32_t n_desc;
  uint32_t n_req;
  uint32_t blob_bytes;          /* = sum of the prefix lengths */
  uint32_t flags;               /* RL_BC_* */
  int64_t now_base;             /* request r's time = now_base + (req_word[r] >> 24) */
  const uint8_t* prefix_blob;
  const uint32_t* desc_word;    /* n_desc */
  const uint32_t* req_word;     /* n_req */
  const uint32_t* req_of;       /* n_desc, or NULL with RL_BC_ONE_PER_REQ */
  const uint16_t* ttl_jitter;   /* n_desc or NULL: rl_batch.ttl_jitter */
} rl_batch_c;
typedef struct rl_host_batch_c {
  uint8_t* prefix_blob;
  uint32_t* desc_word;
  uint32_t* req_word;
  uint32_t* req_of;
  uint16_t* ttl_jitter;
  uint32_t max_desc, max_req, max_blob, reserved;
} rl_host_batch_c;
/* The next free staging slot, compact layout (the rl_host_acquire contract). */
int rl_host_acquire_c(rl_engine* e, rl_host_batch_c* out);
/* Submit a compact host batch (arrays in the acquired slot, or any host memory: copied before
 * the call returns). Complete it with rl_wait_raw_view / rl_wait_raw_into. */
int rl_submit_c(rl_engine* e, const rl_batch_c* batch);
typedef struct rl_raw_reply rl_raw_reply;
/* Complete the oldest batch in flight, a compact host batch, and hand out its n_desc raw replies
 * in the slot's pinned memory (valid as rl_wait_view's results are). */
int rl_wait_raw_view(rl_engine* e, const rl_raw_reply** out);
/* The same, copying the replies into out[n_desc] (NULL discards). */
int rl_wait_raw_into(rl_engine* e, rl_raw_reply* out);
/* Host side of the compact form: GetResponseDescriptorStatus + the near/over checks + the
 * ThrottleMillis max (base_limiter.go:70-195) for descriptors [d0, d1) of a compact batch from
 * its raw replies (indexed like the batch), with the engine's loaded rules. out / req_throttle_ms
 * are indexed by descriptor / request; a request's ThrottleMillis is written once every one of
 * its descriptors is in [d0, d1) (so a caller may split the range over threads at request
 * boundaries). Bit-exact with the statuses rl_submit returns. Thread-safe against itself; not
 * against rl_load_rules. */
int rl_decide_raw(rl_engine* e, const rl_batch_c* batch, const rl_raw_reply* raw, uint32_t d0, uint32_t d1,
                  rl_status* out, uint32_t* req_throttle_ms);

/* Device-memory batch (inputs already resident in HBM; outputs stay in HBM), with nothing
 * else in flight. Ordered on the engine's stream; rl_wait() completes it. Used by the
 * multi-GPU router and by the benchmark. */
int rl_submit_device(rl_engine* e, const rl_batch* device_batch, rl_status* d_out, uint32_t* d_req_throttle_ms);

/* Device-memory batch whose inputs are complete when the call is made, submitted behind at
 * most RL_MAX_IN_FLIGHT - 1 batches still in flight (the micro-batcher's multi-buffering:
 * batch k+1, k+2 are handed over before rl_wait returns batch k). The engine fingerprints and
 * tile-sorts batch k+2 on a second stream as soon as batch k is done on the GPU, while batch
 * k+1 is decided, and decides batches strictly in submission order, so the results equal
 * serial rl_submit_device/rl_wait rounds. rl_wait completes the oldest batch. Batches in
 * flight together need distinct d_out / d_req_throttle_ms buffers. More than one batch in
 * flight needs the default (v4) pipeline; otherwise RL_ESTATE. Replaces nothing in the
 * reference: it is how the batcher overlaps the radix-style implicit pipelining of
 * src/redis/driver_impl.go:84-89 across batches. */
int rl_submit_pipelined(rl_engine* e, const rl_batch* device_batch, rl_status* d_out, uint32_t* d_req_throttle_ms);

/* The engine's HIP stream (hipStream_t), for ordering external work against it. */
void* rl_stream(rl_engine* e);

/* Run the engine's work on an external stream (e.g. the stream RCCL collectives run on), so
 * that device-side ordering needs no host synchronisation; NULL restores the engine's own
 * stream. The stream must outlive its use. Not while a batch is in flight. */
int rl_set_stream(rl_engine* e, void* hip_stream);

/* ---- Multi-GPU router -------------------------------------------------
 * One engine per GPU; GPU s owns the keys whose prefix fingerprint maps to s (every window
 * of a key lands on the same GPU, like a Redis cluster slot for the reference's INCRBY
 * pipeline, src/redis/fixed_cache_impl.go:66-80, driver_impl.go:56-90). All shards must use
 * the same hash_seed and rule table. One routed step:
 *   origin: rl_route_pack       batch -> records grouped by owner, per-owner counts
 *   RCCL:   all-to-all of counts, then of records (send_counts / received counts)
 *   owner:  rl_submit_routed    records received from every origin (origin-major) -> replies
 *   RCCL:   all-to-all of replies (reverse splits)
 *   origin: rl_route_unpack     replies -> rl_status[n_desc], ThrottleMillis[n_req]
 * An owner decides records in origin-major order, i.e. as if the origins' batches had been
 * submitted to one engine one after another. */
#define RL_ROUTE_RECORD_BYTES 32u
#define RL_ROUTE_REPLY_BYTES 24u
#define RL_ROUTE_MAX_SHARDS 16u
#define RL_ROUTE_MAX_REQ (1u << 27) /* requests per origin batch */
#define RL_ROUTE_LOCAL 0xFFFFFFFFu  /* perm[] value of a nil-limit descriptor (decided at the origin) */

/* Device batch -> d_send[n_desc routed records, grouped by owner 0..n_shards-1, serial order
 * inside each group], d_perm[n_desc] (record position, or RL_ROUTE_LOCAL), per-owner record
 * counts in d_send_counts[n_shards] and h_send_counts[n_shards]. Validates the batch
 * (unknown rule / request index, time outside [0, 2^32)) and synchronises the stream. */
int rl_route_pack(rl_engine* e, const rl_batch* device_batch, uint32_t origin, uint32_t n_shards, void* d_send,
                  uint32_t* d_send_counts, uint32_t* d_perm, uint32_t* h_send_counts);

/* rl_route_pack without the host round trip: the same records and d_perm, and for the count
 * exchange d_x[2 j] = records for owner j, d_x[2 j + 1] = 0 or RL_EINVAL when the device found
 * the batch malformed (an unknown rule / request index, a time outside the range) — the pair
 * each origin sends to owner j in the all-to-all of counts (router.py). Ordered on the engine
 * stream, nothing synchronised; argument errors are returned at once. */
int rl_route_pack_async(rl_engine* e, const rl_batch* device_batch, uint32_t origin, uint32_t n_shards, void* d_send,
                        uint32_t* d_x, uint32_t* d_perm);

/* rl_route_pack_async into a strided send buffer, in one kernel: owner j's records at
 * d_send[j * stride ...] (d_send holds n_shards * stride records), d_perm[i] = j * stride +
 * position, pairs in d_x as above (status RL_EDEVICE if the device's look-back spin expired).
 * For transports that take per-peer displacements (ncclAllToAllv; rl_router_step uses it):
 * no temporary records, no separate scan. n_desc must be <= stride <= 2^27. */
int rl_route_pack_strided(rl_engine* e, const rl_batch* device_batch, uint32_t origin, uint32_t n_shards,
                          uint32_t stride, void* d_send, uint32_t* d_x, uint32_t* d_perm);

/* Owner side: decide n routed records (device memory, RL_ROUTE_RECORD_BYTES each) and write
 * one reply per record (RL_ROUTE_REPLY_BYTES each: rl_status + ThrottleMillis) into d_reply.
 * Asynchronous like rl_submit_device; rl_wait() completes it. */
int rl_submit_routed(rl_engine* e, const void* d_records, uint32_t n, void* d_reply);

/* Owner side, asynchronous and pipelined: like rl_submit_routed, but with RL_ROUTED_RAW the
 * owner writes one raw reply per record (rl_raw_reply, 8 B: the INCRBY post-value the record
 * saw, or a local-cache hit) and the origin makes the decisions (rl_route_unpack_raw); the call
 * may be made while up to RL_MAX_IN_FLIGHT - 1 batches are in flight (distinct reply buffers),
 * and the pipeline waits on the device for ready_event (a hipEvent_t recorded after the records
 * arrived, e.g. on the stream of the exchange; NULL: ordered on the engine stream). flags = 0 is
 * rl_submit_routed (ready_event must be NULL). rl_wait completes the oldest batch. */
#define RL_ROUTED_RAW 1u
struct rl_raw_reply {
  uint32_t after; /* INCRBY post-value (uint32, as fixed_cache_impl.go:51 decodes it); 0 for a hit */
  uint32_t flags; /* RL_RAW_LOCAL_HIT: the key was in the local over-limit cache, no INCRBY;
                     RL_RAW_NIL: nil limit */
};
#define RL_RAW_LOCAL_HIT 1u
int rl_submit_routed_async(rl_engine* e, const void* d_records, uint32_t n, void* d_reply, uint32_t flags,
                           void* ready_event);

/* Origin side: replies (in d_send order) -> d_out[n_desc] and d_req_throttle_ms[n_req].
 * Ordered on the engine stream; no host synchronisation. */
int rl_route_unpack(rl_engine* e, const rl_batch* device_batch, const uint32_t* d_perm, const void* d_reply,
                    rl_status* d_out, uint32_t* d_req_throttle_ms);

/* ---- Router object: the routed step above behind one call ------------------------------
 * Owns the exchange buffers and the transport, so a non-Python host (the Go service over cgo)
 * can route without torch.distributed:
 *   RCCL transport  (rccl_id != NULL): one process per GPU, engines[0] = this rank's engine;
 *                   counts, records and replies move by ncclAllToAll / ncclAllToAllv over the
 *                   communicator the router owns (xGMI between GPUs of a node). rank 0 makes the
 *                   id with rl_router_unique_id and hands it to the others out of band.
 *   local transport (rccl_id == NULL): n_shards engines in this process (logical shards, one
 *                   device or several); the exchanges are device-to-device copies.
 * One step: each origin packs its batch by owner into a strided send buffer —
 * one record per descriptor, except that descriptors of a hot prefix (the router's route hot
 * set) are combined into one record carrying their sum of hits_addend (exact: one request time,
 * one rule, local cache off; otherwise the batch is packed without combining); counts, then
 * records move by all-to-all; each owner decides its records in origin order and answers each
 * with its raw INCRBY post-value (rl_raw_reply); the replies return by the reverse all-to-all
 * and the origin makes every descriptor's decision.
 * Every shard finishes every exchange of a step even when one fails, then all of them return
 * the failure: the failing shard its own code, the others RL_EPEER. The counts exchange
 * carries each origin's pack status, the reply exchange each owner's decide status (and any
 * local HIP failure after the counts), so a bad batch or a fault on one GPU cannot leave its
 * peers blocked in a collective. An RCCL failure aborts the communicator (ncclCommAbort) and
 * every later call returns RL_ECOMM. A refused owner batch (RL_ENOSPC, RL_ECAPACITY) leaves that
 * owner's table unchanged; other owners of the step have applied theirs (per-shard atomicity,
 * as a Redis cluster pipeline gives per-node): rl_router_stats.status says which, and after a
 * failure at an owner (decide or later) the outputs still hold every decision the healthy
 * owners made, the descriptors of a failed owner coming out with code RL_CODE_UNKNOWN (not
 * known to be applied) — the caller can answer those requests and fail only the others. After
 * a pack failure (any origin) nothing was applied anywhere and the statuses are untouched; the
 * ThrottleMillis words of origins whose pack ran may have been zeroed (the pack starts them at 0).
 * Request times: every origin's batch-time range travels with its counts. An owner decides its
 * records origin by origin in engine batches whose times span at most one second, so origins
 * whose clocks or batch cuts differ by seconds are exact. An origin whose batch starts more than
 * 3 s behind the newest request time before it (the step clock: earlier steps and the origins
 * before it in rank order) is left out of the step alone: its shard returns RL_ELATE with none of
 * its descriptors applied, every other shard's step goes ahead (the late shard still decides the
 * records it owns), and the clock does not move for it. */
#define RL_ROUTER_ID_BYTES 128u
typedef struct rl_router rl_router;

typedef struct rl_router_config {
  uint32_t struct_size;   /* sizeof(rl_router_config) */
  uint32_t n_shards;      /* 1..RL_ROUTE_MAX_SHARDS */
  uint32_t rank;          /* RCCL transport: this process's shard; local transport: 0 */
  uint32_t max_desc;      /* descriptors per origin batch (an owner can receive n_shards x this) */
  const uint8_t* rccl_id; /* RL_ROUTER_ID_BYTES from rl_router_unique_id, or NULL: local transport */
  uint32_t flags;         /* RL_ROUTER_* */
  uint32_t max_blob_bytes; /* host staging (RL_ROUTER_HOST): key-prefix bytes per origin batch (0 = 64 x max_desc) */
} rl_router_config;
enum {
  RL_ROUTER_NO_COMBINE = 1u, /* one record per descriptor (no hot-prefix combining) */
  RL_ROUTER_HOST = 2u,       /* allocate pinned host staging: rl_router_host_acquire / _submit_host / _wait_into */
  RL_ROUTER_EMULATED = 4u,   /* rccl_id is an rl_router_emu_world id: the collective transport's code path with
                                the collectives emulated in process (one thread per rank; tests) */
  RL_ROUTER_HOST_XCHG = 8u   /* the collectives through the host exchange registered by rl_router_use_host_xchg
                                (one process per rank where RCCL cannot run them; tests). rccl_id unused */
};

typedef struct rl_router_stats {
  uint64_t steps;
  uint32_t n_shards;
  int32_t status[RL_ROUTE_MAX_SHARDS]; /* last step: each shard's status (0 = ok, RL_EPEER = a peer failed) */
  uint32_t recv[RL_ROUTE_MAX_SHARDS];  /* last step: records each owner decided (RCCL: this rank's only) */
  uint32_t sent[RL_ROUTE_MAX_SHARDS];  /* last step: records origin 0 (RCCL: this rank) sent each owner */
  double pack_us, exchange_us, decide_us, decide_max_us, reply_us, unpack_us, step_us; /* last step, host clock */
  uint32_t hot_groups;     /* last step: route hot set size of origin 0 (RCCL: this rank) */
  uint32_t combined;       /* last step: combined records origin 0 (RCCL: this rank) sent (one per hot group) */
  uint64_t repacks;        /* steps packed again without combining (a hot group not one key string) */
  uint64_t combined_steps; /* steps whose origin 0 combined */
  uint32_t owner_batches;  /* last step: engine batches owner 0 (collective: this rank) decided its records in
                              (origins whose request times differ by 2 s or more go to separate batches) */
  uint32_t step_clock;     /* the newest request time of every step applied so far (unix seconds) */
  uint64_t late_steps;     /* steps in which this rank's origin batch (local transport: any shard's) was refused
                              with RL_ELATE */
} rl_router_stats;

/* A fresh RCCL unique id (ncclGetUniqueId), RL_ROUTER_ID_BYTES bytes. */
int rl_router_unique_id(uint8_t* id_out);
/* An in-process world of n_ranks emulated ranks (RL_ROUTER_EMULATED): the id to pass as
 * rccl_id to each rank's rl_router_create, every rank driven by its own thread. The collective
 * transport runs unchanged; ncclAllToAll / ncclAllToAllv / ncclAllGather become device copies
 * driven by the same count and displacement vectors, each rank's receive counts checked against
 * its peers' send counts. The world is freed when the last of its n_ranks routers is destroyed. */
int rl_router_emu_world(uint32_t n_ranks, uint8_t* id_out);
/* A host exchange (RL_ROUTER_HOST_XCHG; tests): an all-to-all-v of host bytes among the ranks of
 * a process group the caller runs (e.g. torch.distributed over gloo). Rank j's bytes for this
 * rank arrive at recv + recv_displs[j]; n_ranks counts and displacements each way. 0 = success.
 * The collective transport then runs its code path unchanged with one process per rank on any
 * number of GPUs — RCCL refuses two ranks on one device, so a one-GPU box cannot run it across
 * processes otherwise. Every collective stages through host memory: not for performance. The
 * registration holds for this thread's next rl_router_create with the flag. */
typedef int (*rl_host_xchg_fn)(void* ctx, const void* send, const size_t* send_counts, const size_t* send_displs,
                               void* recv, const size_t* recv_counts, const size_t* recv_displs);
int rl_router_use_host_xchg(rl_host_xchg_fn fn, void* ctx);
/* engines: n_shards engines (local transport) or 1 (RCCL transport). The router does not own
 * them; they must outlive it and be used by nothing else while a step runs. All engines share
 * hash_seed and the rule table. */
int rl_router_create(const rl_router_config* cfg, rl_engine* const* engines, rl_router** out);
/* One routed step, synchronous: rl_router_submit + rl_router_wait. batches / d_out /
 * d_req_throttle_ms: one per engine passed at create (device pointers; the same layouts as
 * rl_submit_device). Decisions equal one engine deciding the origins' batches one after
 * another in shard order. */
int rl_router_step(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_req_throttle_ms);
/* Pipelined steps: up to three in flight. rl_router_submit packs, exchanges counts, exchanges
 * the replies of the older steps in flight, exchanges records and hands the owner its records
 * (returns once they are queued); rl_router_wait completes the oldest step (its origin's
 * decisions) and returns its status. With two in flight, step k+1's pack overlaps step k's
 * decide on the device. Every
 * shard must make the same sequence of submit / wait calls (the collectives follow it). Inputs
 * and outputs of a step stay untouched by the caller until its wait returns. */
int rl_router_submit(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_req_throttle_ms);
int rl_router_wait(rl_router* r);
/* Host-memory steps (RL_ROUTER_HOST): a Go service on a multi-GPU node stages its batch in the
 * router's pinned memory — rl_router_host_acquire hands out the next step's slot of a shard
 * (RCCL: shard 0), C memory a cgo caller fills through unsafe slices — or passes any host
 * arrays (copied before rl_router_submit_host returns). rl_router_wait_into completes the oldest
 * step and copies each shard's statuses / ThrottleMillis into host memory during the call
 * (NULL entries discard). No caller memory is retained. */
int rl_router_host_acquire(rl_router* r, uint32_t shard, rl_host_batch* out);
int rl_router_submit_host(rl_router* r, const rl_batch* host_batches);
int rl_router_wait_into(rl_router* r, rl_status* const* out, uint32_t* const* req_throttle_ms);
/* A small collective over the router's transport (collective transports only): every rank
 * contributes n_bytes (<= RL_ROUTER_AG_MAX, the same on every rank) of host memory `in`, and out
 * receives n_shards * n_bytes in rank order. Synchronous. Every rank must make the same sequence
 * of router calls (steps and these), e.g. with no step in flight at the same step number: a
 * multi-GPU batcher uses it to agree new rules and a stop at the same step on every rank (rule
 * ids must mean the same limit on every owner). */
#define RL_ROUTER_AG_MAX 8192u
int rl_router_allgather_host(rl_router* r, const void* in, uint32_t n_bytes, void* out);
int rl_router_get_stats(const rl_router* r, rl_router_stats* out);
const char* rl_router_last_error(const rl_router* r);
void rl_router_destroy(rl_router* r);

/* Clear the counter table and local-cache state (FLUSHALL analogue; tests and restarts). */
int rl_reset(rl_engine* e);

int rl_get_stats(rl_engine* e, rl_engine_stats* s);
/* Table occupancy (synchronises the engine's stream; not while a batch is in flight). */
int rl_get_occupancy(rl_engine* e, rl_occupancy* o);

/* Per-kernel timing with HIP events on the engine stream (off by default). When on, each
 * pipeline kernel is bracketed by an event pair; rl_kernel_times() returns the accumulated
 * milliseconds and launch counts for up to `cap` kernels, their names in names[] (static strings). */
int rl_set_timing(rl_engine* e, int on);
int rl_kernel_times(rl_engine* e, const char** names, double* total_ms, uint64_t* launches, uint32_t cap,
                    uint32_t* n_out);

/* Algorithmic-byte accounting for the last completed batch: unique keys U
 * (segments), descriptors, requests and prefix bytes, read back from the device. */
int rl_last_batch_info(rl_engine* e, uint64_t* unique_keys, uint64_t* n_desc, uint64_t* n_req,
                       uint64_t* blob_bytes);

/* ---- Descriptor-tree resolution (GetLimit) ------------------------
 * Replaces rateLimitConfigImpl.GetLimit (src/config/config_impl.go:274-323) per descriptor,
 * batched on the device: it yields the rule id each descriptor of an rl_batch carries.
 * The tree is the loaded YAML config (loadDescriptors, config_impl.go:115-165) flattened:
 * node i has a parent (a node before it, or RL_TREE_ROOT for a domain), its map key in
 * `names` (the domain name, or finalKey = key["_" value], config_impl.go:126-129) and the
 * rule id of its limit (RL_NIL_RULE = no rate_limit). Stats keys (FullKey) stay on the host. */
#define RL_TREE_ROOT 0xFFFFFFFFu
typedef struct rl_tree_node {
  uint32_t parent;
  uint32_t name_off;
  uint32_t name_len;
  uint32_t rule;
} rl_tree_node;

/* Replace the tree. RL_EINVAL on a forward parent, an empty key, or a duplicate (parent,
 * name) — the reference's "duplicate descriptor composite key" / "duplicate domain" panics.
 * Not while a batch is in flight. */
int rl_load_tree(rl_engine* e, const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names,
                 uint32_t names_len);

/* One resolution batch. Strings are (offset, length) ranges of `bytes`. override_rule (may
 * be NULL) holds, per descriptor, the rule id the host registered for descriptor.Limit
 * (config_impl.go:286-296; RL_NIL_RULE = no override): it applies when the domain exists. */
typedef struct rl_resolve_batch {
  uint32_t n_desc;
  uint32_t n_entries;
  uint32_t bytes_len;
  uint32_t reserved;            /* 0 */
  const uint8_t* bytes;
  const uint32_t* domain;       /* [2 n_desc]: domain (off, len) per descriptor */
  const uint32_t* entry_first;  /* [n_desc + 1]: entries of descriptor i are [entry_first[i], entry_first[i+1]) */
  const uint32_t* entry;        /* [4 n_entries]: key off, key len, value off, value len */
  const uint32_t* override_rule;
} rl_resolve_batch;

/* Host memory in and out; synchronous. rule_out[n_desc]. */
int rl_resolve(rl_engine* e, const rl_resolve_batch* batch, uint32_t* rule_out);
/* Device memory in and out, asynchronous: ordered before the engine's next submit (run on the
 * stream that submit's first kernel uses, so with batches in flight it runs beside their
 * decisions, as the next batch's fingerprint pass does). It is NOT ordered after batches
 * already in flight: d_rule_out must not be the rule_id array of a batch still in flight
 * (give each batch in flight its own, as rl_batch inputs are). Two kernels: a level-pipelined
 * walk, then the exact walk for the descriptors it leaves (rl_resolve.hip). */
int rl_resolve_device(rl_engine* e, const rl_resolve_batch* device_batch, uint32_t* d_rule_out);

#ifdef __cplusplus
}
#endif
#endif /* RL_HIP_H */
