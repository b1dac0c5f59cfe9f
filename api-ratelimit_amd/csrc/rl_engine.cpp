// rl_engine.cpp — host runtime behind the C ABI in include/rl_hip.h.
//
// Owns the HBM counter table, the per-batch scratch, the HIP streams, the pinned host
// staging and the launch sequence of the decision pipelines (rl_kernels_v4.hip, default;
// rl_kernels.hip, LSD fallback). The host path mirrors what fixedRateLimitCacheImpl.DoLimit
// does around redis PipeDo (src/redis/fixed_cache_impl.go:91-102): ship the batch, run it,
// bring the per-descriptor outcomes back — except that the decisions themselves are also
// computed on the device, and up to RL_MAX_IN_FLIGHT batches overlap (copies in, kernels,
// copies out), as radix's implicit pipelining overlaps round trips (driver_impl.go:84-89).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rl_common.h"
#include "rl_hip.h"
#include "rl_internal.h"
#include "rl_resolve.h"

namespace rlhip {
void launch_fingerprint(hipStream_t, const rl_batch&, const DevRule*, uint32_t, uint64_t, uint64_t*, ItemRec*,
                        rl_status*, uint32_t*, uint32_t*, EngineCtl*);
void launch_histogram(hipStream_t, const uint64_t*, uint32_t, int, int, uint32_t*, const uint32_t*, uint32_t*);
void launch_hist_scan(hipStream_t, const uint32_t*, uint32_t, uint32_t*, int, const uint32_t*, const RegionOcc*,
                      EngineCtl*, uint32_t);
uint32_t hist_blocks(uint32_t n);
uint32_t hist_sub_words();
void launch_fallback_lo_keys(hipStream_t, const ItemRec*, const uint64_t*, uint32_t, uint64_t*, uint32_t*);
void launch_gather_keys(hipStream_t, const uint64_t*, const uint32_t*, uint32_t, uint64_t*);
uint32_t sort_tiles(uint32_t n);
uint32_t scan_tiles(uint32_t n);
void launch_sort_pass(hipStream_t, const uint64_t*, const uint32_t*, uint64_t*, uint32_t*, uint32_t, int,
                      const uint32_t*, uint32_t*, uint32_t*, EngineCtl*);
void launch_scan(hipStream_t, const uint64_t*, const uint32_t*, const ItemRec*, uint32_t, int, int, SortedRec*,
                 uint64_t*, uint64_t*, uint32_t*, uint32_t*, EngineCtl*);
void launch_leader(hipStream_t, const uint64_t*, SortedRec*, const ItemRec*, const DevRule*, uint32_t,
                   const TableDesc&, SegInfo*, const uint32_t*, uint32_t, HotCand*, EngineCtl*);
void launch_decide(hipStream_t, const SortedRec*, const SegInfo*, const DevRule*, uint32_t, rl_status*, uint32_t*, int,
                   EngineCtl*);
void launch_occ_update(hipStream_t, RegionOcc*, EngineCtl*, uint32_t);
void launch_cand_state(hipStream_t, const rl_batch&, const DevRule*, uint64_t, HotCand*, EngineCtl*);
uint32_t route_bcnt_words(uint32_t n);
void launch_route_pack_strided(hipStream_t, const rl_batch&, const DevRule*, uint32_t, uint64_t, uint32_t, uint32_t,
                               uint32_t, RRec*, uint32_t*, uint32_t*, uint32_t*);
void launch_route_pack(hipStream_t, const rl_batch&, const DevRule*, uint32_t, uint64_t, uint32_t, uint32_t, RRec*,
                       uint8_t*, uint32_t*, RRec*, uint32_t*, uint32_t*, EngineCtl*, uint32_t*);
void launch_route_reply(hipStream_t, uint32_t, const rl_status*, const uint32_t*, RReply*);
hipError_t route_set_spin_limit(uint32_t v);
void launch_route_unpack(hipStream_t, uint32_t, const uint32_t*, const uint32_t*, const RReply*, rl_status*,
                         uint32_t*);
uint32_t compact_chunks(uint32_t n);
void launch_compact_expand(hipStream_t, uint32_t, uint32_t, int64_t, const uint32_t*, const uint32_t*, const uint32_t*,
                           uint32_t*, uint32_t*, uint32_t*, uint32_t*, int64_t*, uint32_t*);
uint32_t v4_tiles(uint32_t n);
uint32_t v4_group_blocks(uint32_t n);
uint32_t v4_scan_blocks();
size_t v4_scratch_bytes();
void launch_v4_hist(hipStream_t, const rl_batch&, const DevRule*, uint32_t, uint64_t, const HotEntry*, uint32_t*,
                    uint32_t*, uint16_t*, unsigned long long*, MRec*, rl_status*, EngineCtl*);
void launch_v4_scan(hipStream_t st, uint32_t n, const uint16_t* tstart, const unsigned long long* thsum,
                    unsigned long long* hoff, const uint32_t* fpart, const HotEntry* hot_list, HotBucket* hb,
                    const TableDesc& tab, HotCand* cand, uint32_t* heads_out, uint32_t* ins_out, void* scratch,
                    const uint32_t* poison, const RegionOcc* occ, EngineCtl* ctl);
void launch_v4_place(hipStream_t st, const rl_batch& b, const MRec* srec, const uint16_t* tstart,
                     void* scratch, const DevRule* rules, uint32_t n_rules, const unsigned long long* hoff, HotBucket* hb,
                     int local_cache, rl_status* out, uint32_t* req_thr, Deferred* dfr, int routed,
                     uint32_t* poison, EngineCtl* ctl);
void launch_v4_group(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, const TableDesc& tab,
                     rl_status* out, uint32_t* req_thr, const HotBucket* hb, const Deferred* dfr, HotCand* cand,
                     int cand_on, uint64_t seed, void* scratch, uint32_t* wg_heads, uint32_t* wg_ins,
                     const uint32_t* scan_heads, const uint32_t* scan_ins, int routed, RegionOcc* occ, EngineCtl* ctl,
                     EngineCtl* next_ctl, EngineCtl* hctl, HotCand* hcand, const MRec* srec,
                     const uint16_t* tstart);
}  // namespace rlhip

using namespace rlhip;

namespace {

enum KernelId {
  KT_FINGERPRINT, KT_HISTOGRAM, KT_HIST_SCAN, KT_SORT_PASS, KT_SCAN, KT_LEADER, KT_DECIDE, KT_FALLBACK, KT_MEMSET,
  KT_CAND, KT_V4_HIST, KT_V4_SCAN, KT_V4_PLACE, KT_V4_GROUP, KT_RESOLVE, KT_COUNT
};
const char* const kKernelNames[KT_COUNT] = {"k_fingerprint", "k_histogram", "k_hist_scan", "k_sort_pass", "k_scan",
                                            "k_leader",      "k_decide",    "fallback",    "memset",      "k_cand_state",
                                            "k4_hist",       "k4_scan",     "k4_place",    "k4_group",
                                            "k_resolve"};

enum Mode { MODE_LSD = 1, MODE_LSD_FULL = 2, MODE_V4 = 4 };

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Wait for an event by polling. A blocking wait wakes the submitter thread ≈20 µs after the
// GPU signals, and with two batches in flight that delay lands directly on the next batch's
// k4_hist (it is submitted after this wait returns). The submitter thread is dedicated to its
// device (rl_hip.h threading rule), so spinning costs no other work; after a bounded spin (a
// batch far longer than any steady-state one) it falls back to blocking.
hipError_t wait_event_polling(hipEvent_t ev) {
  for (int k = 0; k < (1 << 18); ++k) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
  }
  return hipEventSynchronize(ev);
}

}  // namespace

// Host slots: one per batch in flight (pinned staging, control-block and candidate copies,
// completion events, hot-table versions). v4 device buffers of k4_hist have two slots,
// because k4_hist of batch k waits for batch k-2 to finish on the GPU.
constexpr int HSLOTS = RL_MAX_IN_FLIGHT;

struct rl_engine {
  rl_config cfg{};
  int lo_bit = 16, npasses = 6;
  hipStream_t stream = nullptr;      // the stream all kernels are ordered on (own_stream or rl_set_stream's)
  hipStream_t own_stream = nullptr;
  hipStream_t front = nullptr;       // k4_hist of a batch submitted behind one in flight
  hipStream_t xin = nullptr;         // host path: H2D copies
  hipStream_t xout = nullptr;        // host path: D2H copies
  std::string err;

  // counter table
  Slot* table = nullptr;
  size_t table_slots = 0;
  TableDesc tab{};
  RegionOcc* d_occ = nullptr;        // per-region occupancy (device, updated by the last kernel of a batch)
  RegionOcc occ[8] = {};             // host mirror (same update from the control-block copy)

  // rules
  DevRule* d_rules = nullptr;
  uint32_t n_rules = 0, rules_cap = 0;
  std::vector<DevRule> h_rules;      // what d_rules[0, n_rules) holds

  // host staging (rl_submit): per host slot one pinned input region with the device layout,
  // its device twin, device outputs and pinned outputs
  struct Stage {
    uint8_t* h_in = nullptr;
    uint8_t* d_in = nullptr;
    rl_status* d_out = nullptr;
    uint32_t* d_thr = nullptr;
    rl_status* h_out = nullptr;
    uint32_t* h_thr = nullptr;
    uint8_t* d_cin = nullptr;   // compact batches: device copies of the desc / req words and req_of
    uint32_t* d_csum = nullptr; // compact batches: per-chunk prefix-length sums
  };
  Stage stage[HSLOTS];
  size_t in_bytes = 0, o_off = 0, o_rule = 0, o_req = 0, o_now = 0, o_hits = 0, o_jit = 0;
  size_t c_pitch = 0;  // compact layout: rows desc_word | req_word | req_of at this pitch from o_off (host), 0 (device)

  // LSD pipeline scratch
  uint64_t *keys_orig = nullptr, *keys_a = nullptr, *keys_b = nullptr;
  uint32_t *vals_a = nullptr, *vals_b = nullptr;
  ItemRec* recs = nullptr;
  SortedRec* srec = nullptr;
  SegInfo* seg = nullptr;
  uint32_t* offs = nullptr;
  uint32_t* hist_part = nullptr;  // per-block partial digit histograms
  uint32_t* fp_part = nullptr;    // per-block fingerprint partials
  uint32_t* fp_part2 = nullptr;   // the same folded per histogram block
  uint32_t* tile_heads = nullptr; // per-scan-tile segment-head counts
  uint8_t* zero_block = nullptr;  // ctl | look-backs (zeroed per LSD batch)
  size_t zero_cap = 0;

  // hot set (both pipelines)
  HotEntry* d_hot = nullptr;                  // device hot-key table: tag words (HOT_SLOTS units) + list by hot index (HOT_MAX)
  HotEntry* d_hot_buf[HSLOTS] = {};           // d_hot = d_hot_buf[hot_ver]; one per batch in flight
  int hot_ver = 0;
  HotEntry* h_hot_stage = nullptr;            // pinned upload staging
  HotCand* d_cand = nullptr;                  // hot-set candidates (CAND_MAX)
  HotCand* h_cand = nullptr;                  // pinned copy (current host slot)
  HotCand* h_cand_s[HSLOTS] = {};
  std::vector<HotKey> hot;                    // current hot-key set (index = hot idx)
  bool hot_dirty = true;
  std::vector<HotCand> cand_stash;
  bool cand_pending = false;
  bool want_cand = true;                      // copy the candidates back after the next batch

  // v4 pipeline
  uint16_t* v4_tcount[2] = {};                // [tile][V4_ROW16] bucket starts
  unsigned long long* v4_thsum[2] = {};       // [tile][HOT_BUCKETS] hot h sums
  MRec* v4_srt[2] = {};                       // tile-sorted records
  uint32_t* v4_fpart[2] = {};                 // per-tile fingerprint partials
  unsigned long long* v4_hoff = nullptr;      // [tile][HOT_BUCKETS] exclusive h prefix over tiles
  Deferred* v4_dfr = nullptr;                 // deferred hot descriptors
  HotBucket* v4_hb = nullptr;                 // per hot bucket batch state
  void* v4_scratch = nullptr;                 // k4_group global scratch + k4_scan ranges
  uint32_t* v4_heads = nullptr;               // per-block unique-key counts (k4_group, then k4_scan)
  uint32_t* v4_ins = nullptr;                 // per-block new slots per region, 16-bit pairs (k4_group, then k4_scan)
  EngineCtl* v4_ctl[3] = {};                  // control blocks rotate over three (k4_group clears batch k+2's)
  uint32_t* d_poison = nullptr;               // set by k4_place of a refused batch, read by k4_scan

  // per host slot: pinned control block, completion events
  EngineCtl* h_ctl = nullptr;
  EngineCtl* h_ctl_s[HSLOTS] = {};
  hipEvent_t ev_done[HSLOTS] = {};            // the slot's batch complete (outputs copied, for host batches)
  hipEvent_t ev_dd[HSLOTS] = {};              // device batch complete: device-scope release only (no
                                              // system-scope cache write-back between batches)
  hipEvent_t done_ev[HSLOTS] = {};            // the completion event recorded for the slot's batch
  hipEvent_t ev_in[HSLOTS] = {};              // host path: the slot's inputs copied in
  hipEvent_t ev_kern[HSLOTS] = {};            // host path: the slot's kernels done (D2H may start)
  hipEvent_t ev_front[2] = {};                // k4_hist of the device slot done (on front)
  hipEvent_t ev_ready = nullptr;              // inputs of a non-pipelined submit ready (on stream)
  hipEvent_t ev_resolve = nullptr;            // an rl_resolve_device launched on the front stream
  bool resolve_pending = false;               // ... not yet ordered before a submit
  hipEvent_t ev_hot = nullptr;                // hot-set upload copy done (staging reusable)
  uint64_t sub_seq = 0;                       // batches submitted (host slot = seq % HSLOTS, device slot = seq & 1)
  int acquired = -1;                          // host slot handed out by rl_host_acquire

  // descriptor tree (rl_load_tree / rl_resolve)
  TreeNodeDev* d_tree_nodes = nullptr;
  uint64_t* d_tree_slots = nullptr;
  uint8_t* d_tree_names = nullptr;
  FastNode* d_tree_fnodes = nullptr;  // the first pass's copy (build_fast_tree)
  uint64_t* d_tree_fslots = nullptr;
  TreeDesc2 tree{};
  bool has_tree = false;
  uint8_t* d_res = nullptr;  // rl_resolve staging (grown on demand)
  size_t res_cap = 0;
  // k_resolve's per-block flags (grown on demand): RES_FLAG_SLOTS sets, one per call in turn, so
  // a resolve on the front stream never shares its flags with one still running on the engine
  // stream (a call finds at most RL_MAX_IN_FLIGHT batches, with their resolves, ahead of it)
  static constexpr uint32_t RES_FLAG_SLOTS = RL_MAX_IN_FLIGHT + 1;
  uint32_t* d_res_flags = nullptr;
  uint32_t res_flag_cap = 0;  // words per set
  uint64_t res_seq = 0;

  // multi-GPU router scratch (allocated on first use)
  RRec* r_tmp = nullptr;           // origin: routed records in descriptor order
  uint8_t* r_own = nullptr;        // origin: owner per descriptor
  uint32_t* r_bcnt = nullptr;      // origin: per (block, owner) counts -> send offsets
  EngineCtl* r_ctl = nullptr;      // origin: error word of rl_route_pack
  uint32_t* h_route = nullptr;     // pinned: [0] err, [1..16] send counts
  uint32_t* r_thr = nullptr;       // owner: ThrottleMillis per routed record
  rl_status* r_out = nullptr;      // owner: statuses per routed record

  // batches in flight, oldest first
  struct Flight {
    rl_batch b{};                  // device pointers
    rl_status* out = nullptr;      // device outputs
    uint32_t* thr = nullptr;
    RReply* reply = nullptr;       // routed batch: reply destination
    uint32_t slot = 0;             // host slot
    bool want_cand = false;
    bool settled = false;          // reruns done
    bool fell_back = false;
    bool host = false;             // host batch: results D2H into the slot's pinned outputs
    bool raw = false;              // raw replies (compact host batch): RawReply per descriptor, no ThrottleMillis
    uint32_t errs = 0;
    rl_status* user_out = nullptr; // host batch: rl_wait copies here (may be null)
    uint32_t* user_thr = nullptr;
    bool poll = false;             // completion = k4_group's done word behind h_ctl (no event)
  };
  Flight fl[HSLOTS];
  // A device v4 batch completes on the word k4_group's last block writes behind the slot's pinned
  // control block after everything else (rl_kernels_v4.hip), not on a completion event: the
  // event's marker packet cost ≈5 µs between k4_group of batch k and k4_scan of k+1, and the
  // host sees the word as soon as it lands (profiles/r05_ab_poll_done.txt).
  volatile uint32_t* done_word(uint32_t slot) {
    return reinterpret_cast<volatile uint32_t*>(h_ctl_s[slot] + 1);
  }
  // A wait longer than 5 ms (a batch takes ~0.1 ms) asks the stream too, every 5 ms: a fault in
  // a kernel before the word shows there (the word would stay 0), and a stream that drained
  // without the word (k4_group writes it last) ends the spin as the old bound's stream
  // synchronize did. Normal waits never call into the runtime: a hipStreamQuery every 2^14 reads
  // fell inside ordinary waits and cost 8-18 % of the config-3 step.
  hipError_t poll_done(const Flight& f) {
    volatile uint32_t* w = done_word(f.slot);
    auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(5);
    for (uint64_t k = 0;; ++k) {
      if (*w) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        return hipSuccess;
      }
      if ((k & 0x3FFu) != 0x3FFu || std::chrono::steady_clock::now() < next) continue;
      const hipError_t q = hipStreamQuery(stream);
      if (q != hipErrorNotReady) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        return q;
      }
      next = std::chrono::steady_clock::now() + std::chrono::milliseconds(5);
    }
  }
  int n_fl = 0;

  // timing
  bool timing = false;
  struct Mark { int kid; hipEvent_t a, b; };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double kt_ms[KT_COUNT] = {};
  uint64_t kt_n[KT_COUNT] = {};

  // stats
  rl_engine_stats st{};
  uint64_t last_unique = 0, last_n = 0, last_req = 0, last_blob = 0;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) { return fail(RL_EHIP, "%s: %s", what, hipGetErrorString(e)); }

  hipEvent_t next_event() {
    if (ev_used == ev_pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
  }
  template <class F>
  void timed(int kid, F f) {
    if (!timing) { f(); return; }
    hipEvent_t a = next_event(), b = next_event();
    hipEventRecord(a, stream);
    f();
    hipEventRecord(b, stream);
    marks.push_back({kid, a, b});
  }

  // Layout of the LSD per-batch zero block for n descriptors.
  struct ZLayout { size_t ctl, lb_sort, lb_sum, lb_head, total; };
  ZLayout zlayout(uint32_t n, int passes) const {
    ZLayout z;
    z.ctl = 0;
    z.lb_sort = align_up(sizeof(EngineCtl), 256);
    z.lb_sum = z.lb_sort + align_up((size_t)passes * sort_tiles(n > 0 ? n : 1) * RADIX * 4, 256);
    z.lb_head = z.lb_sum + align_up((size_t)scan_tiles(n > 0 ? n : 1) * 8, 256);
    z.total = z.lb_head + align_up((size_t)scan_tiles(n > 0 ? n : 1) * 8, 256);
    return z;
  }

  // k4_hist of the next v4 batch runs on the front stream (while the batch in flight is decided),
  // otherwise (nothing in flight, kernels timed, or the LSD pipeline) on the engine stream
  bool split_hist() const {
    static const bool no_split = getenv("RL_DIAG_NO_SPLIT") != nullptr;  // diagnostics
    return !timing && n_fl > 0 && !no_split;
  }
  int default_mode() const {
    if (cfg.flags & RL_CFG_LSD_ONLY) return MODE_LSD;
    if (n_rules > V4_MAX_RULES) return MODE_LSD;  // MRec packs the rule id in 15 bits
    return MODE_V4;
  }
  int run_pipeline(const rl_batch& b, rl_status* out, uint32_t* thr, int mode, hipEvent_t in_ev, bool inputs_ready);
  int upload_hot(hipStream_t us);
  void update_hot(const HotCand* cand, uint32_t n_cand);
  int settle(Flight& f);
  int finish(rl_status* out, uint32_t* thr, bool into);
  int enqueue_d2h(const Flight& f, hipStream_t s);
  int check_batch(const rl_batch* b, bool host);
  int submit_common(const rl_batch& d, rl_status* out, uint32_t* thr, RReply* reply, hipEvent_t in_ev,
                    bool inputs_ready, bool host, rl_status* user_out, uint32_t* user_thr, bool raw = false);
  void occ_host_update(const EngineCtl* c) {
    for (int r = 0; r < 8; ++r) occ_advance(occ[r], lazy_region(tab.lag, (uint32_t)r), c->gen_max[r], c->ins[r]);
  }
  uint64_t live_total() const {
    uint64_t s = 0;
    for (int r = 0; r < 8; ++r) s += occ[r].live;
    return s;
  }
  int reset_occ() {
    for (int r = 0; r < 8; ++r) {
      occ[r].gen = 0;
      occ[r].live = 0;
      occ[r].prev = 0;
    }
    hipError_t e = hipMemcpy(d_occ, occ, sizeof occ, hipMemcpyHostToDevice);
    return e == hipSuccess ? 0 : hip_fail(e, "reset occupancy");
  }
};

int rl_engine::run_pipeline(const rl_batch& b, rl_status* out, uint32_t* thr, int mode, hipEvent_t in_ev,
                            bool inputs_ready) {
  if (resolve_pending) {  // rl_resolve_device ran on the front stream: a batch not starting there waits for it
    if (!(mode == MODE_V4 && split_hist())) hipStreamWaitEvent(stream, ev_resolve, 0);
    resolve_pending = false;
  }
  const uint32_t n = b.n_desc;
  const bool full = mode == MODE_LSD_FULL;
  const int passes = full ? 16 : npasses;
  const ZLayout z = zlayout(n, passes);
  EngineCtl* ctl = reinterpret_cast<EngineCtl*>(zero_block + z.ctl);
  uint32_t* hist = hist_part;
  uint32_t* lb_sort = reinterpret_cast<uint32_t*>(zero_block + z.lb_sort);
  uint64_t* lb_sum = reinterpret_cast<uint64_t*>(zero_block + z.lb_sum);
  uint64_t* lb_head = reinterpret_cast<uint64_t*>(zero_block + z.lb_head);
  const size_t lb_pass_stride = (size_t)sort_tiles(n > 0 ? n : 1) * RADIX;  // per-digit look-back words
  // how decisions are written (rl_common.h OUT_*): statuses, routed statuses, raw replies
  const int routed = (b.reserved & RL_BATCH_RAW) ? OUT_RAW : (b.reserved & RL_BATCH_ROUTED) ? OUT_ROUTED : OUT_STATUS;
  hipError_t e;
  if (mode == MODE_V4) {
    const uint32_t sl = (uint32_t)(sub_seq & 1u);
    EngineCtl* c4 = v4_ctl[sub_seq % 3];
    EngineCtl* c4n = v4_ctl[(sub_seq + 2) % 3];  // batch seq+2's control block (k4_group clears it)
    // k4_hist runs on the front stream while the previous batch is still being decided (a
    // submit behind a batch in flight); otherwise, or when kernels are timed, on the engine stream
    const bool split = split_hist();
    hipStream_t fs = split ? front : stream;
    if (split) {
      // slot buffers and control block free: batch seq-2 done
      if (n_fl >= 2 && fl[n_fl - 2].poll && !fl[n_fl - 2].settled) {
        // three in flight: batch seq-2 has no event to wait for on the device; the host waits
        hipError_t pe = poll_done(fl[n_fl - 2]);
        if (pe != hipSuccess) return hip_fail(pe, "poll");
      } else if (n_fl >= 2) {
        hipStreamWaitEvent(front, done_ev[(sub_seq + HSLOTS - 2) % HSLOTS], 0);
      }
      // (with one batch in flight, batch seq-2 has completed through rl_wait: nothing to wait
      // for, and no API call between rl_wait and this k4_hist launch)
      if (in_ev) {
        hipStreamWaitEvent(front, in_ev, 0);
      } else if (!inputs_ready) {  // inputs come from work queued on the stream
        hipEventRecord(ev_ready, stream);
        hipStreamWaitEvent(front, ev_ready, 0);
      }
    } else if (in_ev) {
      hipStreamWaitEvent(stream, in_ev, 0);
    }
    if (n == 0) {
      if (thr && b.n_req) hipMemsetAsync(thr, 0, (size_t)b.n_req * 4, stream);
      hipMemsetAsync(c4, 0, sizeof(EngineCtl), stream);
      hipMemsetAsync(c4n, 0, sizeof(EngineCtl), stream);
      e = hipMemcpyAsync(h_ctl, c4, sizeof(EngineCtl), hipMemcpyDeviceToHost, stream);
      return e == hipSuccess ? 0 : hip_fail(e, "hipMemcpyAsync(ctl)");
    }
    if (hot_dirty) {
      int rc = upload_hot(fs);
      if (rc) return rc;
    }
    const HotEntry* hot_t = d_hot;
    const int lc = cfg.local_cache ? 1 : 0;
    const uint32_t ng = v4_group_blocks(n);
    MRec* srt = v4_srt[sl];
    timed(KT_V4_HIST, [&] {
      launch_v4_hist(fs, b, d_rules, n_rules, cfg.hash_seed, hot_t, thr, v4_fpart[sl], v4_tcount[sl], v4_thsum[sl],
                     srt, out, c4);
    });
    if (split) {
      hipEventRecord(ev_front[sl], front);
      hipStreamWaitEvent(stream, ev_front[sl], 0);
    }
    timed(KT_V4_SCAN, [&] {
      launch_v4_scan(stream, n, v4_tcount[sl], v4_thsum[sl], v4_hoff, v4_fpart[sl], hot_t + HOT_SLOTS, v4_hb, tab,
                     want_cand ? d_cand : nullptr, v4_heads + ng, v4_ins + (size_t)ng * 4, v4_scratch, d_poison,
                     d_occ, c4);
    });
    timed(KT_V4_PLACE, [&] {
      launch_v4_place(stream, b, srt, v4_tcount[sl], v4_scratch, d_rules, n_rules, v4_hoff, v4_hb, lc, out,
                      thr, v4_dfr, routed, d_poison, c4);
    });
    timed(KT_V4_GROUP, [&] {
      launch_v4_group(stream, b, d_rules, n_rules, tab, out, thr, v4_hb, v4_dfr, d_cand, want_cand ? 1 : 0,
                      cfg.hash_seed, v4_scratch, v4_heads, v4_ins, v4_heads + ng, v4_ins + (size_t)ng * 4, routed,
                      d_occ, c4, c4n, h_ctl, want_cand ? h_cand : nullptr, srt, v4_tcount[sl]);
    });
    // k4_group's last block writes the summary into h_ctl / h_cand (pinned host memory)
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    return 0;
  }
  if (in_ev) hipStreamWaitEvent(stream, in_ev, 0);
  timed(KT_MEMSET, [&] {
    hipMemsetAsync(zero_block, 0, z.total, stream);
    // request throttles are zeroed by k_fingerprint; only an empty batch needs a memset
    if (thr && b.n_req && n == 0) hipMemsetAsync(thr, 0, (size_t)b.n_req * 4, stream);
  });
  if (n == 0) {
    e = hipMemcpyAsync(h_ctl, ctl, sizeof(EngineCtl), hipMemcpyDeviceToHost, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "hipMemcpyAsync(ctl)");
  }
  const uint64_t* skeys;
  const uint32_t* svals;
  if (!full) {
    timed(KT_FINGERPRINT, [&] {
      launch_fingerprint(stream, b, d_rules, n_rules, cfg.hash_seed, keys_orig, recs, out, thr, fp_part, ctl);
    });
    timed(KT_HISTOGRAM, [&] { launch_histogram(stream, keys_orig, n, lo_bit, npasses, hist, fp_part, fp_part2); });
    timed(KT_HIST_SCAN, [&] { launch_hist_scan(stream, hist, n, offs, npasses, fp_part2, d_occ, ctl, tab.lag); });
    const uint64_t* kin = keys_orig;
    const uint32_t* vin = nullptr;
    for (int p = 0; p < npasses; ++p) {
      uint64_t* kout = (p & 1) ? keys_b : keys_a;
      uint32_t* vout = (p & 1) ? vals_b : vals_a;
      timed(KT_SORT_PASS, [&] {
        launch_sort_pass(stream, kin, vin, kout, vout, n, lo_bit + 8 * p, offs + p * hist_sub_words(),
                         lb_sort + p * lb_pass_stride, &ctl->tile_ctr[p][0], ctl);
      });
      kin = kout;
      vin = vout;
    }
    skeys = kin;
    svals = vin;
  } else {
    // Full-fingerprint order: stable sort by fp_lo, then by the 64-bit sort key.
    timed(KT_FALLBACK, [&] {
      launch_fingerprint(stream, b, d_rules, n_rules, cfg.hash_seed, keys_orig, recs, out, thr, fp_part, ctl);
      launch_fallback_lo_keys(stream, recs, keys_orig, n, keys_a, vals_a);
      launch_histogram(stream, keys_a, n, 0, 8, hist, fp_part, fp_part2);
      launch_hist_scan(stream, hist, n, offs, 8, fp_part2, d_occ, ctl, tab.lag);
    });
    const uint64_t* kin = keys_a;
    const uint32_t* vin = vals_a;
    for (int p = 0; p < 8; ++p) {
      uint64_t* kout = (p & 1) ? keys_a : keys_b;
      uint32_t* vout = (p & 1) ? vals_a : vals_b;
      timed(KT_SORT_PASS, [&] {
        launch_sort_pass(stream, kin, vin, kout, vout, n, 8 * p, offs + p * hist_sub_words(), lb_sort + p * lb_pass_stride,
                         &ctl->tile_ctr[p][0], ctl);
      });
      kin = kout;
      vin = vout;
    }
    // after 8 passes the result is in keys_a/vals_a; gather the sort keys in that order
    timed(KT_FALLBACK, [&] {
      launch_gather_keys(stream, keys_orig, vals_a, n, keys_b);
      launch_histogram(stream, keys_b, n, 0, 8, hist, nullptr, nullptr);
      launch_hist_scan(stream, hist, n, offs + 8 * hist_sub_words(), 8, nullptr, nullptr, ctl, tab.lag);
    });
    kin = keys_b;
    vin = vals_a;
    for (int p = 0; p < 8; ++p) {
      uint64_t* kout = (p & 1) ? keys_b : keys_a;
      uint32_t* vout = (p & 1) ? vals_a : vals_b;
      timed(KT_SORT_PASS, [&] {
        launch_sort_pass(stream, kin, vin, kout, vout, n, 8 * p, offs + (8 + p) * hist_sub_words(),
                         lb_sort + (8 + p) * lb_pass_stride, &ctl->tile_ctr[8 + p][0], ctl);
      });
      kin = kout;
      vin = vout;
    }
    skeys = kin;
    svals = vin;
  }
  timed(KT_SCAN, [&] {
    launch_scan(stream, skeys, svals, recs, n, full ? 0 : lo_bit, full ? 0 : 1, srec, lb_sum, lb_head,
                &ctl->tile_ctr[31][0], tile_heads, ctl);
  });
  timed(KT_LEADER, [&] {
    launch_leader(stream, skeys, srec, recs, d_rules, n, tab, seg, tile_heads, scan_tiles(n), d_cand, ctl);
  });
  timed(KT_DECIDE, [&] {
    launch_decide(stream, srec, seg, d_rules, n, out, thr, routed, ctl);
    launch_occ_update(stream, d_occ, ctl, tab.lag);
  });
  timed(KT_CAND, [&] { launch_cand_state(stream, b, d_rules, cfg.hash_seed, d_cand, ctl); });
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  e = hipMemcpyAsync(h_ctl, ctl, sizeof(EngineCtl), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h_cand, d_cand, sizeof(HotCand) * CAND_MAX, hipMemcpyDeviceToHost, stream);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(ctl)");
  return 0;
}

// Upload the hot-key set: open-addressed tag words (rl_common.h HOT_TAGS; home = hot_home(a),
// word = hot_tag(a) | index + 1) followed by the entries in hot-index order.
int rl_engine::upload_hot(hipStream_t us) {
  std::vector<HotEntry> t;
  build_hot_table(hot, t);
  // Into the version no in-flight batch reads, through a pinned staging buffer whose last
  // copy is done.
  hipError_t e = hipEventSynchronize(ev_hot);
  if (e == hipSuccess) {
    memcpy(h_hot_stage, t.data(), sizeof(HotEntry) * t.size());
    e = hipMemcpyAsync(d_hot_buf[(hot_ver + 1) % HSLOTS], h_hot_stage, sizeof(HotEntry) * t.size(),
                       hipMemcpyHostToDevice, us);
  }
  if (e == hipSuccess) e = hipEventRecord(ev_hot, us);
  if (e != hipSuccess) return hip_fail(e, "upload hot set");
  hot_ver = (hot_ver + 1) % HSLOTS;
  d_hot = d_hot_buf[hot_ver];
  hot_dirty = false;
  st.hot_keys = hot.size();
  return 0;
}

// Maintain the hot-key set from this batch's long segments (candidates with their prefix
// state). Keys are prefix states; the two windows of one prefix merge; a prefix seen under
// two rules (two units included) is not bucketable. Hysteresis keeps the set (and its upload)
// stable on a steady skewed stream: a hot key stays while it has >= HOT_CAND_MIN descriptors
// per batch, a new key joins with >= HOT_MIN_SEG while there is room.
void rl_engine::update_hot(const HotCand* cand, uint32_t n_cand) {
  n_cand = n_cand < (uint32_t)CAND_MAX ? n_cand : (uint32_t)CAND_MAX;
  auto ident_less = [](const HotKey& x, const HotKey& y) { return x.a != y.a ? x.a < y.a : x.b < y.b; };
  auto same_ident = [](const HotKey& x, const HotKey& y) { return x.a == y.a && x.b == y.b; };
  std::vector<HotKey> agg;
  agg.reserve(n_cand);
  for (uint32_t i = 0; i < n_cand; ++i) {
    const HotCand& c = cand[i];
    agg.push_back(HotKey{c.a, c.b, c.unit, c.rule, c.count});
  }
  std::sort(agg.begin(), agg.end(), ident_less);
  std::vector<HotKey> merged;  // count 0 marks a rule conflict
  for (const HotKey& x : agg) {
    if (!merged.empty() && same_ident(merged.back(), x)) {
      HotKey& m = merged.back();
      if (m.rule != x.rule) m.count = 0, m.rule = 0xFFFFFFFFu;
      else if (m.rule != 0xFFFFFFFFu) m.count += x.count;
    } else {
      merged.push_back(x);
    }
  }
  auto find = [&](const HotKey& k) -> const HotKey* {
    auto it = std::lower_bound(merged.begin(), merged.end(), k, ident_less);
    return (it != merged.end() && same_ident(*it, k)) ? &*it : nullptr;
  };
  std::vector<HotKey> next;
  bool changed = false;
  for (const HotKey& x : hot) {
    const HotKey* m = find(x);
    if (m && m->rule == x.rule && m->count >= HOT_CAND_MIN) next.push_back(*m);
    else changed = true;
  }
  if (next.size() < (size_t)HOT_MAX) {
    std::vector<HotKey> cur(hot);
    std::sort(cur.begin(), cur.end(), ident_less);
    std::vector<HotKey> fresh;
    for (const HotKey& m : merged) {
      if (m.count < HOT_MIN_SEG || m.rule == 0xFFFFFFFFu) continue;
      auto it = std::lower_bound(cur.begin(), cur.end(), m, ident_less);
      if (it == cur.end() || !same_ident(*it, m)) fresh.push_back(m);
    }
    std::sort(fresh.begin(), fresh.end(), [](const HotKey& x, const HotKey& y) { return x.count > y.count; });
    for (const HotKey& m : fresh) {
      if (next.size() >= (size_t)HOT_MAX) break;
      next.push_back(m);
      changed = true;
    }
  }
  if (changed) {
    hot = std::move(next);
    hot_dirty = true;
  }
}

int rl_engine::enqueue_d2h(const Flight& f, hipStream_t s) {
  hipError_t e;
  const Stage& g = stage[f.slot];
  if (f.raw) {  // 8-B raw replies, no ThrottleMillis
    e = f.b.n_desc ? hipMemcpyAsync(g.h_out, f.out, (size_t)f.b.n_desc * sizeof(RawReply), hipMemcpyDeviceToHost, s)
                   : hipSuccess;
    return e == hipSuccess ? 0 : hip_fail(e, "hipMemcpyAsync(D2H raw)");
  }
  if (f.b.n_desc) {
    e = hipMemcpyAsync(g.h_out, f.out, (size_t)f.b.n_desc * sizeof(rl_status), hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(D2H out)");
  }
  if (f.b.n_req) {
    e = hipMemcpyAsync(g.h_thr, f.thr, (size_t)f.b.n_req * 4, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(D2H thr)");
  }
  return 0;
}

// Wait for an in-flight batch and rerun it if the device refused it: on the LSD pipeline
// when the bucketed pipeline could not take it, on the full fingerprint order when a sort-
// prefix run held two fingerprints. Reruns are synchronous, so they are on the table before
// anything submitted later.
int rl_engine::settle(Flight& f) {
  h_ctl = h_ctl_s[f.slot];
  h_cand = h_cand_s[f.slot];
  hipError_t e = timing ? hipStreamSynchronize(stream) : f.poll ? poll_done(f) : wait_event_polling(done_ev[f.slot]);
  if (e == hipSuccess && timing && f.host) e = hipStreamSynchronize(xout);
  if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
  uint32_t errs = h_ctl->err;
  if ((errs & ERR_FALLBACK) && !(errs & (ERR_BAD_INPUT | ERR_BAD_TIME))) {
    // The bucketed pipeline refused the batch before touching the table (oversized bucket, a
    // hot prefix with a second rule, an expiry inside a hot key's batch, or the batch before
    // it was refused): run it on the LSD pipeline.
    ++st.lsd_fallbacks;
    f.fell_back = true;
    // slots the refused attempt's hot keys claimed (k4_group counted them into the device's
    // occupancy): the same into the host mirror
    occ_host_update(h_ctl);
    st.inserted_keys += h_ctl->n_inserted;
    int rc = run_pipeline(f.b, f.out, f.thr, MODE_LSD, nullptr, true);
    if (rc) return rc;
    if (f.reply) launch_route_reply(stream, f.b.n_desc, f.out, f.thr, f.reply);
    if (f.host && (rc = enqueue_d2h(f, stream)) != 0) return rc;
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    errs = h_ctl->err;
  }
  if (errs & ERR_NEED_RESORT) {
    // A sort-prefix run held two fingerprints: nothing touched the table (k_leader and
    // k_decide return early), so re-run the batch on the full fingerprint order.
    ++st.resorts;
    int rc = run_pipeline(f.b, f.out, f.thr, MODE_LSD_FULL, nullptr, true);
    if (rc) return rc;
    if (f.reply) launch_route_reply(stream, f.b.n_desc, f.out, f.thr, f.reply);
    if (f.host && (rc = enqueue_d2h(f, stream)) != 0) return rc;
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    errs = h_ctl->err;
  }
  f.errs = errs;
  f.settled = true;
  return 0;
}

// Complete the oldest in-flight batch: reruns (settle), then errors, hot-set maintenance,
// stats and the host-path copy. A refused batch poisons the batch behind it (k4_place ->
// k4_scan), so that one is settled here too, before anything else can be submitted.
int rl_engine::finish(rl_status* out_into, uint32_t* thr_into, bool into) {
  Flight f = fl[0];
  for (int q = 1; q < n_fl; ++q) fl[q - 1] = fl[q];
  --n_fl;
  const bool settled_here = !f.settled;  // else the previous batch's finish reran this one
  if (settled_here) {
    int rc = settle(f);
    if (rc) return rc;
  }
  if (settled_here && f.fell_back) {
    hipError_t e = hipMemsetAsync(d_poison, 0, 4, stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(poison)");
    for (int q = 0; q < n_fl && !fl[q].settled; ++q) {  // refused in turn (poison chain)
      int rc = settle(fl[q]);
      if (rc) return rc;
      if (!fl[q].fell_back) break;
      hipError_t e2 = hipMemsetAsync(d_poison, 0, 4, stream);
      if (e2 != hipSuccess) return hip_fail(e2, "hipMemsetAsync(poison)");
    }
  }
  h_ctl = h_ctl_s[f.slot];
  h_cand = h_cand_s[f.slot];
  const uint32_t errs = f.errs;
  if (timing) {
    hipError_t e = hipStreamSynchronize(stream);  // the next batch's marks too
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    for (auto& m : marks) {
      float ms = 0;
      hipEventElapsedTime(&ms, m.a, m.b);
      kt_ms[m.kid] += ms;
      kt_n[m.kid] += 1;
    }
    marks.clear();
    ev_used = 0;
  }
  if (errs & ERR_BAD_INPUT)
    return fail(RL_EINVAL, "batch references an unknown rule id or request index, or malformed prefix offsets / "
                           "request order");
  if (errs & ERR_BAD_TIME) return fail(RL_EINVAL, "request time outside [0, 0xFFFD0000] unix seconds");
  if (errs & ERR_WINDOW_SPAN)
    return fail(RL_EINVAL, "batch spans more than two windows of one unit; split it at window boundaries");
  if (errs & ERR_TABLE_FULL)
    return fail(RL_ENOSPC, "counter table region would pass its load limit; batch refused before any update "
                           "(raise log2_slots or max_load_permille)");
  if (errs & ERR_SPIN) return fail(RL_EDEVICE, "device spin limit exceeded or range invariant violated");
  if (errs & ERR_NEED_RESORT) return fail(RL_EDEVICE, "full-fingerprint re-sort still found a mixed run");
  // Hot-set maintenance costs host time between batches: every batch while the set is
  // empty or after a fallback, else every 8th batch (a skewed stream's head moves slowly).
  if (!(cfg.flags & RL_CFG_LSD_ONLY) && (f.want_cand || f.fell_back)) {
    const uint32_t nc = std::min(h_ctl->tile_ctr[CAND_CTR][0], (uint32_t)CAND_MAX);
    if (f.fell_back) {  // rare: take the set now
      update_hot(h_cand, nc);
    } else {
      cand_stash.assign(h_cand, h_cand + nc);
      cand_pending = true;
    }
  }
  occ_host_update(h_ctl);
  last_unique = h_ctl->n_segments;
  last_n = f.b.n_desc;
  last_req = f.b.n_req;
  last_blob = f.b.blob_bytes;
  st.batches += 1;
  st.descriptors += f.b.n_desc;
  st.inserted_keys += h_ctl->n_inserted;
  st.live_keys = live_total();
  want_cand = hot.empty() || (st.batches & 7) == 0;
  if (f.host && f.raw) {
    if (into && out_into && f.b.n_desc) memcpy(out_into, stage[f.slot].h_out, (size_t)f.b.n_desc * sizeof(RawReply));
  } else if (f.host) {
    rl_status* o = into ? out_into : f.user_out;
    uint32_t* t = into ? thr_into : f.user_thr;
    const Stage& g = stage[f.slot];
    if (o && f.b.n_desc) memcpy(o, g.h_out, (size_t)f.b.n_desc * sizeof(rl_status));
    if (t && f.b.n_req) memcpy(t, g.h_thr, (size_t)f.b.n_req * 4);
  }
  return 0;
}

int rl_engine::check_batch(const rl_batch* b, bool host) {
  if (b->n_desc > cfg.max_batch_desc || b->n_req > cfg.max_batch_req || (host && b->blob_bytes > cfg.max_blob_bytes))
    return fail(RL_ECAPACITY, "batch exceeds engine capacity (%u desc, %u req, %u blob bytes)", cfg.max_batch_desc,
                cfg.max_batch_req, cfg.max_blob_bytes);
  if (b->reserved) return fail(RL_EINVAL, "rl_batch.reserved must be 0");
  if (b->n_desc && (!b->prefix_off || !b->rule_id || !b->req_of)) return fail(RL_EINVAL, "null descriptor array");
  if (b->n_req && (!b->now || !b->hits_addend)) return fail(RL_EINVAL, "null request array");
  if (b->n_desc && !b->n_req) return fail(RL_EINVAL, "descriptors without requests");
  if (b->n_desc && !b->prefix_blob && (!host || b->blob_bytes))
    return fail(RL_EINVAL, "null prefix_blob (a device blob must be readable even when empty)");
  if (!d_rules) {
    int rc = rl_load_rules(this, nullptr, 0);
    if (rc) return rc;
  }
  return 0;
}

// Common tail of every submit form: run the pipeline behind what is in flight, record the
// completion point, queue the flight.
int rl_engine::submit_common(const rl_batch& d, rl_status* out, uint32_t* thr, RReply* reply, hipEvent_t in_ev,
                             bool inputs_ready, bool host, rl_status* user_out, uint32_t* user_thr, bool raw) {
  const uint32_t s = (uint32_t)(sub_seq % HSLOTS);
  h_ctl = h_ctl_s[s];
  h_cand = h_cand_s[s];
  *done_word(s) = 0;  // (the slot's previous batch is complete)
  const bool want = want_cand;
  int rc = run_pipeline(d, out, thr, default_mode(), in_ev, inputs_ready);
  if (rc) return rc;
  if (reply) launch_route_reply(stream, d.n_desc, out, thr, reply);
  Flight f;
  f.b = d;
  f.out = out;
  f.thr = thr;
  f.reply = reply;
  f.slot = s;
  f.want_cand = want;
  f.host = host;
  f.user_out = user_out;
  f.user_thr = user_thr;
  f.raw = raw;
  hipError_t e;
  if (host) {
    // outputs leave on the copy-out stream while the next batch's kernels run
    e = hipEventRecord(ev_kern[s], stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(xout, ev_kern[s], 0);
    if (e != hipSuccess) return hip_fail(e, "host path events");
    if ((rc = enqueue_d2h(f, xout)) != 0) return rc;
    e = hipEventRecord(ev_done[s], xout);
    done_ev[s] = ev_done[s];
  } else {
    // outputs stay in device memory; the host summary was written with a system-scope
    // release by k4_group (or copied by the LSD path's own D2H copy, ordered before this)
    const bool dev_only = default_mode() == MODE_V4 && !reply && d.n_desc;
    if (dev_only && !timing) {
      f.poll = true;  // k4_group writes the done word (cleared at this submit's start)
      e = hipSuccess;
    } else {
      done_ev[s] = dev_only ? ev_dd[s] : ev_done[s];
      e = hipEventRecord(done_ev[s], stream);
    }
  }
  if (e != hipSuccess) return hip_fail(e, "hipEventRecord(done)");
  fl[n_fl++] = f;
  ++sub_seq;
  if (cand_pending) {
    // Hot-set maintenance from a completed batch's candidates runs after the next submit has
    // enqueued its kernels, not between rl_wait and that submit, where it would delay the
    // next batch's k4_hist; the set it yields applies one batch later. Decisions do not
    // depend on the hot set, only speed does.
    cand_pending = false;
    update_hot(cand_stash.data(), (uint32_t)cand_stash.size());
  }
  return 0;
}

namespace rlhip {
int rlx_engine_view(rl_engine* e, EngineView* v) {
  if (!e || !v) return RL_EINVAL;
  if (!e->d_rules) {
    int rc = rl_load_rules(e, nullptr, 0);
    if (rc) return rc;
  }
  v->rules = e->d_rules;
  v->n_rules = e->n_rules;
  v->seed = e->cfg.hash_seed;
  v->local_cache = e->cfg.local_cache ? 1 : 0;
  v->device = e->cfg.device;
  v->max_batch_desc = e->cfg.max_batch_desc;
  return 0;
}
void rlx_engine_hot(rl_engine* e, std::vector<HotKey>& out) { out = e->hot; }
int rlx_engine_set_lag(rl_engine* e, bool dry) {
  if (e->tab.lag) return 0;
  // An engine that already decided batches kept its SECOND regions' occupancy under the
  // one-generation rule (RegionOcc.prev stays 0 there), so lag mode's capacity check would
  // under-count live slots: such an engine needs RL_CFG_LAG_WINDOW from rl_create.
  if (e->st.batches > 0 || e->n_fl) return RL_ESTATE;
  if (!dry) {
    e->tab.lag = 1u;
    e->cfg.flags |= RL_CFG_LAG_WINDOW;
  }
  return 0;
}
}  // namespace rlhip

extern "C" {

uint32_t rl_abi_version(void) { return RL_ABI_VERSION; }

// rl_create's failures have no engine to hold their message: rl_last_error(NULL) returns the
// calling thread's last one.
static thread_local std::string t_create_err = "no rl_create failure on this thread";
const char* rl_last_error(const rl_engine* e) { return e ? e->err.c_str() : t_create_err.c_str(); }

int rl_create(const rl_config* cfg_in, rl_engine** out) {
  if (!cfg_in || !out) return RL_EINVAL;
  *out = nullptr;
  if (cfg_in->struct_size != sizeof(rl_config)) return RL_EINVAL;
  auto* e = new rl_engine();
  e->cfg = *cfg_in;
  rl_config& c = e->cfg;
  for (int u = 0; u < 4; ++u) {
    if (c.log2_slots[u] == 0) c.log2_slots[u] = 20;
    if (c.log2_slots[u] < 4 || c.log2_slots[u] > 31) {
      delete e;
      return RL_EINVAL;
    }
  }
  if (c.max_load_permille == 0) c.max_load_permille = 750;
  if (c.max_load_permille < 100 || c.max_load_permille > 950 || c.reserved) { delete e; return RL_EINVAL; }
  if (c.max_batch_desc == 0) c.max_batch_desc = 1u << 20;
  if (c.max_batch_req == 0) c.max_batch_req = c.max_batch_desc;
  if (c.max_blob_bytes == 0) c.max_blob_bytes = c.max_batch_desc * 64u;
  if (c.max_batch_desc > (1u << 28) || c.max_blob_bytes > (1u << 31)) { delete e; return RL_EINVAL; }
  if (c.sort_bits == 0) c.sort_bits = 48;
  if (c.sort_bits % 8 || c.sort_bits < 8 || c.sort_bits > 64) { delete e; return RL_EINVAL; }
  e->npasses = (int)c.sort_bits / 8;
  e->lo_bit = 64 - (int)c.sort_bits;
  hipError_t he = hipSetDevice(c.device);
  if (he != hipSuccess) {
    t_create_err = std::string("rl_create: hipSetDevice: ") + hipGetErrorString(he);
    delete e;
    return RL_EHIP;
  }
  const char* where = "";
  auto chk_at = [&](hipError_t x, const char* what) {
    if (x != hipSuccess && he == hipSuccess) he = x, where = what;
  };
#define chk(x) chk_at((x), #x)
  chk(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
  chk(hipStreamCreateWithFlags(&e->front, hipStreamNonBlocking));
  chk(hipStreamCreateWithFlags(&e->xin, hipStreamNonBlocking));
  chk(hipStreamCreateWithFlags(&e->xout, hipStreamNonBlocking));
  e->stream = e->own_stream;
  // counter table: 8 regions (home unit x window parity)
  size_t off = 0;
  for (int r = 0; r < 8; ++r) {
    const uint32_t lg = c.log2_slots[r / 2];
    e->tab.region_base[r] = off;
    e->tab.region_log2[r] = lg;
    e->occ[r].gen = 0;
    e->occ[r].live = 0;
    e->occ[r].limit = (uint32_t)(((uint64_t)1 << lg) * c.max_load_permille / 1000);
    e->occ[r].prev = 0;
    off += (size_t)1 << lg;
  }
  e->tab.split = c.per_second_split ? 1u : 0u;
  e->tab.local_cache = c.local_cache ? 1u : 0u;
  e->tab.lag = (c.flags & RL_CFG_LAG_WINDOW) ? 1u : 0u;
  e->table_slots = off;
  chk(hipMalloc(&e->table, off * sizeof(Slot)));
  if (he == hipSuccess) chk(hipMemset(e->table, 0, off * sizeof(Slot)));
  e->tab.slots = e->table;
  chk(hipMalloc(&e->d_occ, sizeof e->occ));
  if (he == hipSuccess) chk(hipMemcpy(e->d_occ, e->occ, sizeof e->occ, hipMemcpyHostToDevice));
  const size_t N = c.max_batch_desc, R = c.max_batch_req, B = c.max_blob_bytes;
  // host staging: blob | off | rule | req | now | hits (same layout on host and device)
  e->o_off = align_up(B + RL_BLOB_SLACK, 256);
  // prefix_off, rule_id and req_of at one pitch: their H2D copies go as one 2-D copy
  e->o_rule = e->o_off + align_up((N + 1) * 4, 256);
  e->o_req = e->o_rule + align_up((N + 1) * 4, 256);
  e->o_now = e->o_req + align_up((N + 1) * 4, 256);
  e->o_hits = e->o_now + align_up(R * 8, 256);
  e->in_bytes = e->o_hits + align_up(R * 4, 256);
  // compact layout (rl_batch_c): blob, then three rows (desc words, req words, req_of)
  e->c_pitch = align_up((std::max(N, R) + 1) * 4, 256);
  e->in_bytes = std::max(e->in_bytes, e->o_off + 3 * e->c_pitch);
  // both layouts: the EXPIRE jitter per descriptor (rl_batch.ttl_jitter) after everything else
  e->o_jit = align_up(e->in_bytes, 256);
  e->in_bytes = e->o_jit + align_up(N * 2, 256);
  for (auto& g : e->stage) {
    chk(hipMalloc(&g.d_cin, 3 * e->c_pitch));
    chk(hipMalloc(&g.d_csum, (size_t)compact_chunks((uint32_t)N) * 4 + 64));
    chk(hipMalloc(&g.d_in, e->in_bytes));
    chk(hipHostMalloc(&g.h_in, e->in_bytes, hipHostMallocDefault));
    chk(hipMalloc(&g.d_out, N * sizeof(rl_status) + 64));
    chk(hipMalloc(&g.d_thr, R * 4 + 64));
    chk(hipHostMalloc(&g.h_out, N * sizeof(rl_status) + 64, hipHostMallocDefault));
    chk(hipHostMalloc(&g.h_thr, R * 4 + 64, hipHostMallocDefault));
  }
  // LSD pipeline
  chk(hipMalloc(&e->keys_orig, N * 8));
  chk(hipMalloc(&e->keys_a, N * 8));
  chk(hipMalloc(&e->keys_b, N * 8));
  chk(hipMalloc(&e->vals_a, N * 4));
  chk(hipMalloc(&e->vals_b, N * 4));
  chk(hipMalloc(&e->recs, N * sizeof(ItemRec)));
  chk(hipMalloc(&e->srec, N * sizeof(SortedRec)));
  chk(hipMalloc(&e->seg, N * sizeof(SegInfo)));
  chk(hipMalloc(&e->offs, (size_t)MAX_PASSES * hist_sub_words() * 4));
  chk(hipMalloc(&e->hist_part, (size_t)hist_blocks((uint32_t)N) * MAX_PASSES * RADIX * 4));
  chk(hipMalloc(&e->fp_part2, (size_t)hist_blocks((uint32_t)N) * FP_PART_WORDS * 4 + 64));
  chk(hipMalloc(&e->fp_part, ((N + 255) / 256) * FP_PART_WORDS * 4 + 64));
  chk(hipMalloc(&e->tile_heads, (size_t)scan_tiles((uint32_t)N) * 4 + 64));
  e->zero_cap = e->zlayout((uint32_t)N, MAX_PASSES).total;
  chk(hipMalloc(&e->zero_block, e->zero_cap));
  // hot set
  for (int k = 0; k < HSLOTS; ++k) chk(hipMalloc(&e->d_hot_buf[k], sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX)));
  e->d_hot = e->d_hot_buf[0];
  chk(hipHostMalloc(&e->h_hot_stage, sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX), hipHostMallocDefault));
  chk(hipMalloc(&e->d_cand, sizeof(HotCand) * CAND_MAX));
  for (int k = 0; k < HSLOTS; ++k) {
    chk(hipHostMalloc(&e->h_cand_s[k], sizeof(HotCand) * CAND_MAX, hipHostMallocDefault));
    chk(hipHostMalloc(&e->h_ctl_s[k], sizeof(EngineCtl) + 64, hipHostMallocDefault));  // + k4_group's done word
  }
  e->h_cand = e->h_cand_s[0];
  e->h_ctl = e->h_ctl_s[0];
  // v4 pipeline
  {
    const size_t T4 = v4_tiles((uint32_t)N);
    for (int k = 0; k < 2; ++k) {
      chk(hipMalloc(&e->v4_tcount[k], T4 * V4_ROW16 * 2));
      chk(hipMalloc(&e->v4_thsum[k], T4 * HOT_BUCKETS * 8));
      chk(hipMalloc(&e->v4_srt[k], N * sizeof(MRec) + 64));
      chk(hipMalloc(&e->v4_fpart[k], T4 * FP_PART_WORDS * 4 + 64));
    }
    chk(hipMalloc(&e->v4_hoff, T4 * HOT_BUCKETS * 8));
    chk(hipMalloc(&e->v4_dfr, N * sizeof(Deferred) + 64));
    // the buckets, then per bucket the freezing request's last INCRBY (index, jitter): hot_exp()
    chk(hipMalloc(&e->v4_hb, HOT_BUCKETS * (sizeof(HotBucket) + 8)));
    const size_t nb = (size_t)v4_group_blocks((uint32_t)N) + v4_scan_blocks();
    chk(hipMalloc(&e->v4_heads, nb * 4 + 64));
    chk(hipMalloc(&e->v4_ins, nb * 4 * 4 + 64));
    chk(hipMalloc(&e->v4_scratch, v4_scratch_bytes()));
    for (int k = 0; k < 3; ++k) {
      chk(hipMalloc(&e->v4_ctl[k], sizeof(EngineCtl)));
      if (he == hipSuccess) chk(hipMemset(e->v4_ctl[k], 0, sizeof(EngineCtl)));
    }
    chk(hipMalloc(&e->d_poison, 64));
    if (he == hipSuccess) chk(hipMemset(e->d_poison, 0, 64));
  }
  std::vector<hipEvent_t*> evs = {&e->ev_front[0], &e->ev_front[1], &e->ev_ready, &e->ev_hot, &e->ev_resolve};
  for (int k = 0; k < HSLOTS; ++k) {
    evs.push_back(&e->ev_done[k]);
    evs.push_back(&e->ev_in[k]);
    evs.push_back(&e->ev_kern[k]);
  }
  for (hipEvent_t* ev : evs) {
    chk(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    if (he == hipSuccess) chk(hipEventRecord(*ev, e->stream));
  }
  for (int k = 0; k < HSLOTS; ++k) {
    chk(hipEventCreateWithFlags(&e->ev_dd[k], hipEventDisableTiming | hipEventReleaseToDevice));
    e->done_ev[k] = e->ev_done[k];
  }
  if (he == hipSuccess) chk(hipMemset(e->zero_block, 0, e->zero_cap));
  // the route packs' look-back bound: the default, or a diagnostic value (tests of the
  // RL_EDEVICE path set it tiny)
  if (he == hipSuccess) {
    const char* sl = getenv("RL_DIAG_LB_SPIN_LIMIT");
    chk(route_set_spin_limit(sl ? (uint32_t)strtoul(sl, nullptr, 10) : (1u << 22)));
  }
  if (he == hipSuccess) chk(hipDeviceSynchronize());
#undef chk
  if (he != hipSuccess) {
    t_create_err = std::string("rl_create: ") + where + ": " + hipGetErrorString(he);
    rl_destroy(e);
    return RL_EHIP;
  }
  *out = e;
  return 0;
}

void rl_destroy(rl_engine* e) {
  if (!e) return;
  for (hipStream_t s : {e->stream, e->front, e->xin, e->xout})
    if (s) hipStreamSynchronize(s);
  for (auto ev : e->ev_pool) hipEventDestroy(ev);
  for (hipEvent_t ev : {e->ev_front[0], e->ev_front[1], e->ev_ready, e->ev_hot})
    if (ev) hipEventDestroy(ev);
  for (int k = 0; k < HSLOTS; ++k) {
    for (hipEvent_t ev : {e->ev_done[k], e->ev_dd[k], e->ev_in[k], e->ev_kern[k]})
      if (ev) hipEventDestroy(ev);
    hipFree(e->d_hot_buf[k]);
    hipHostFree(e->h_cand_s[k]);
    hipHostFree(e->h_ctl_s[k]);
  }
  for (auto& g : e->stage) {
    hipFree(g.d_cin);
    hipFree(g.d_csum);
    hipFree(g.d_in);
    hipHostFree(g.h_in);
    hipFree(g.d_out);
    hipFree(g.d_thr);
    hipHostFree(g.h_out);
    hipHostFree(g.h_thr);
  }
  for (int k = 0; k < 2; ++k) {
    hipFree(e->v4_tcount[k]);
    hipFree(e->v4_thsum[k]);
    hipFree(e->v4_srt[k]);
    hipFree(e->v4_fpart[k]);
  }
  for (int k = 0; k < 3; ++k) hipFree(e->v4_ctl[k]);
  for (void* p : {(void*)e->v4_hoff, (void*)e->v4_dfr, (void*)e->v4_hb,
                  (void*)e->v4_heads, (void*)e->v4_ins, e->v4_scratch, (void*)e->d_poison, (void*)e->d_tree_nodes,
                  (void*)e->d_tree_slots, (void*)e->d_tree_names, (void*)e->d_tree_fnodes, (void*)e->d_tree_fslots, (void*)e->d_res, (void*)e->d_res_flags, (void*)e->table, (void*)e->d_occ,
                  (void*)e->d_rules, (void*)e->keys_orig, (void*)e->keys_a, (void*)e->keys_b, (void*)e->vals_a,
                  (void*)e->vals_b, (void*)e->recs, (void*)e->srec, (void*)e->seg, (void*)e->offs,
                  (void*)e->hist_part, (void*)e->fp_part, (void*)e->fp_part2, (void*)e->tile_heads,
                  (void*)e->zero_block, (void*)e->d_cand, (void*)e->r_tmp, (void*)e->r_own, (void*)e->r_bcnt,
                  (void*)e->r_ctl, (void*)e->r_thr, (void*)e->r_out})
    hipFree(p);
  hipHostFree(e->h_hot_stage);
  hipHostFree(e->h_route);
  for (hipStream_t s : {e->front, e->xin, e->xout, e->own_stream})
    if (s) hipStreamDestroy(s);
  delete e;
}

int rl_load_rules(rl_engine* e, const rl_rule* rules, uint32_t n) {
  if (!e) return RL_EINVAL;
  if (n && !rules) return e->fail(RL_EINVAL, "null rule array");
  std::vector<DevRule> h(n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t u = rules[i].unit & ~RL_RULE_SHADOW;
    if (u < RL_UNIT_SECOND || u > RL_UNIT_DAY)
      return e->fail(RL_EINVAL, "rule %u: unit %u is not SECOND/MINUTE/HOUR/DAY (utilities.go:31 panics)", i,
                     rules[i].unit);
    h[i] = DevRule{};
    h[i].shadow = (rules[i].unit & RL_RULE_SHADOW) ? 1u : 0u;
    h[i].L = rules[i].requests_per_unit;
    // nearLimitThreshold = uint32(math.Floor(float64(float32(L) * nearLimitRatio)))  base_limiter.go:86
    const float p = (float)rules[i].requests_per_unit * e->cfg.near_limit_ratio;
    h[i].near = (uint32_t)std::floor((double)p);
    h[i].div = unit_div(u);
    h[i].unit = u;
  }
  // Rule ids never change meaning while batches are in flight: a batch reads rules by id (its
  // launch validated ids against the n_rules of that moment), so a table that keeps the loaded
  // prefix and appends rules can be loaded at any time — the micro-batcher registers the
  // (L, unit) of a new config.RateLimit, e.g. a descriptor.Limit override
  // (config_impl.go:281-289), while earlier batches are still being decided. Only the appended
  // entries are copied, into slots no in-flight batch reads, with a blocking copy that is
  // complete before any later launch. A table that changes or drops a loaded rule, or that
  // must grow the device allocation, needs nothing in flight.
  const uint32_t n_old = e->n_rules;
  if (e->n_fl) {
    bool prefix = n >= n_old;
    for (uint32_t i = 0; prefix && i < n_old; ++i) prefix = memcmp(&h[i], &e->h_rules[i], sizeof(DevRule)) == 0;
    if (!prefix)
      return e->fail(RL_ESTATE, "rl_load_rules while a batch is in flight may only append rules (ids keep their meaning)");
    if (n > e->rules_cap || (n > V4_MAX_RULES) != (n_old > V4_MAX_RULES))
      return e->fail(RL_ESTATE, "rl_load_rules: %u rules need a larger table; call rl_wait until nothing is in flight", n);
  }
  const uint32_t first = e->n_fl ? n_old : 0u;  // entries to copy
  if (n > e->rules_cap || !e->d_rules) {
    hipFree(e->d_rules);
    e->d_rules = nullptr;
    // room for the v4 pipeline's whole rule-id space, so appends never reallocate
    const uint32_t cap = n < V4_MAX_RULES ? V4_MAX_RULES : n;
    hipError_t he = hipMalloc(&e->d_rules, (size_t)cap * sizeof(DevRule));
    if (he != hipSuccess) {
      e->rules_cap = 0;
      e->n_rules = 0;
      e->h_rules.clear();
      return e->hip_fail(he, "hipMalloc(rules)");
    }
    e->rules_cap = cap;
  }
  if (n > first) {
    hipError_t he = hipMemcpy(e->d_rules + first, h.data() + first, (size_t)(n - first) * sizeof(DevRule),
                              hipMemcpyHostToDevice);
    if (he != hipSuccess) return e->hip_fail(he, "hipMemcpy(rules)");
  }
  e->h_rules = std::move(h);
  e->n_rules = n;
  return 0;
}

int rl_host_acquire(rl_engine* e, rl_host_batch* out) {
  if (!e || !out) return RL_EINVAL;
  if (e->n_fl >= HSLOTS) return e->fail(RL_ESTATE, "rl_host_acquire with %d batches in flight (call rl_wait)", HSLOTS);
  const int s = (int)(e->sub_seq % HSLOTS);
  uint8_t* h = e->stage[s].h_in;
  out->prefix_blob = h;
  out->prefix_off = reinterpret_cast<uint32_t*>(h + e->o_off);
  out->rule_id = reinterpret_cast<uint32_t*>(h + e->o_rule);
  out->req_of = reinterpret_cast<uint32_t*>(h + e->o_req);
  out->now = reinterpret_cast<int64_t*>(h + e->o_now);
  out->hits_addend = reinterpret_cast<uint32_t*>(h + e->o_hits);
  out->ttl_jitter = reinterpret_cast<uint16_t*>(h + e->o_jit);
  out->max_desc = e->cfg.max_batch_desc;
  out->max_req = e->cfg.max_batch_req;
  out->max_blob = e->cfg.max_blob_bytes;
  out->reserved = 0;
  e->acquired = s;
  return 0;
}

int rl_submit(rl_engine* e, const rl_batch* b, rl_status* out, uint32_t* req_throttle_ms) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl >= HSLOTS) return e->fail(RL_ESTATE, "rl_submit with %d batches in flight (call rl_wait)", HSLOTS);
  int rc = e->check_batch(b, true);
  if (rc) return rc;
  if (e->n_fl && e->default_mode() != MODE_V4)
    return e->fail(RL_ESTATE, "a second batch in flight needs the v4 pipeline (call rl_wait)");
  const uint32_t s = (uint32_t)(e->sub_seq % HSLOTS);
  rl_engine::Stage& g = e->stage[s];
  uint8_t* h = g.h_in;
  // Stage into the slot's pinned memory unless the caller built the batch there
  // (rl_host_acquire); the slot's previous batch is complete (batches complete in order and
  // fewer than HSLOTS are in flight).
  struct Arr { const void* src; size_t o, n; } arrs[] = {
      {b->prefix_blob, 0, b->blob_bytes}, {b->prefix_off, e->o_off, b->n_desc ? ((size_t)b->n_desc + 1) * 4 : 0},
      {b->rule_id, e->o_rule, (size_t)b->n_desc * 4}, {b->req_of, e->o_req, (size_t)b->n_desc * 4},
      {b->now, e->o_now, (size_t)b->n_req * 8}, {b->hits_addend, e->o_hits, (size_t)b->n_req * 4},
      {b->ttl_jitter, e->o_jit, b->ttl_jitter ? (size_t)b->n_desc * 2 : 0}};
  for (auto& a : arrs)
    if (a.n && a.src != h + a.o) memcpy(h + a.o, a.src, a.n);
  memset(h + b->blob_bytes, 0, RL_BLOB_SLACK);  // the device reads prefixes in 16-B words
  e->acquired = -1;
  hipError_t he = hipSuccess;
  // Copy only the used extents of each array, on the copy-in stream: the previous batch's
  // kernels keep running meanwhile. prefix_off / rule_id / req_of (one pitch apart) move as one
  // 2-D copy: four copies per batch instead of six (each costs 10-20 us of copy-engine gap).
  const size_t ext[] = {(size_t)b->blob_bytes + RL_BLOB_SLACK, arrs[1].n, arrs[2].n, arrs[3].n, arrs[4].n, arrs[5].n};
  if (ext[0]) he = hipMemcpyAsync(g.d_in, h, ext[0], hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess && b->n_desc) {
    const size_t pitch = e->o_rule - e->o_off;
    he = hipMemcpy2DAsync(g.d_in + e->o_off, pitch, h + e->o_off, pitch, ext[1], 3, hipMemcpyHostToDevice, e->xin);
  }
  for (int k = 4; k < 6 && he == hipSuccess; ++k)
    if (ext[k]) he = hipMemcpyAsync(g.d_in + arrs[k].o, h + arrs[k].o, ext[k], hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess && arrs[6].n)
    he = hipMemcpyAsync(g.d_in + e->o_jit, h + e->o_jit, arrs[6].n, hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess) he = hipEventRecord(e->ev_in[s], e->xin);
  if (he != hipSuccess) return e->hip_fail(he, "hipMemcpyAsync(H2D)");
  rl_batch d = *b;
  d.prefix_blob = g.d_in;
  d.prefix_off = reinterpret_cast<const uint32_t*>(g.d_in + e->o_off);
  d.rule_id = reinterpret_cast<const uint32_t*>(g.d_in + e->o_rule);
  d.req_of = reinterpret_cast<const uint32_t*>(g.d_in + e->o_req);
  d.now = reinterpret_cast<const int64_t*>(g.d_in + e->o_now);
  d.hits_addend = reinterpret_cast<const uint32_t*>(g.d_in + e->o_hits);
  d.ttl_jitter = b->ttl_jitter ? reinterpret_cast<const uint16_t*>(g.d_in + e->o_jit) : nullptr;
  e->st.host_batches += 1;
  return e->submit_common(d, g.d_out, g.d_thr, nullptr, e->ev_in[s], false, true, out, req_throttle_ms);
}

int rl_wait(rl_engine* e) {
  if (!e) return RL_EINVAL;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_wait without a batch in flight");
  return e->finish(nullptr, nullptr, false);
}

int rl_query(rl_engine* e) {
  if (!e) return RL_EINVAL;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_query without a batch in flight");
  const rl_engine::Flight& f = e->fl[0];
  if (f.settled) return 1;
  if (f.poll) {
    if (*e->done_word(f.slot)) return 1;
    // not done: a fault on the stream shows in its query (the word would never be written)
    const hipError_t q = hipStreamQuery(e->stream);
    if (q == hipSuccess) return 1;  // (the stream drained: the batch is complete)
    if (q == hipErrorNotReady) return 0;
    return e->hip_fail(q, "hipStreamQuery");
  }
  const hipError_t q = hipEventQuery(e->done_ev[f.slot]);
  if (q == hipSuccess) return 1;
  if (q == hipErrorNotReady) return 0;
  return e->hip_fail(q, "hipEventQuery");
}

int rl_wait_into(rl_engine* e, rl_status* out, uint32_t* req_throttle_ms) {
  if (!e) return RL_EINVAL;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_wait_into without a batch in flight");
  if (e->fl[0].raw) return e->fail(RL_ESTATE, "rl_wait_into: the oldest batch is compact (rl_wait_raw_into)");
  return e->finish(out, req_throttle_ms, true);
}

int rl_wait_view(rl_engine* e, const rl_status** out, const uint32_t** req_throttle_ms) {
  if (!e || !out || !req_throttle_ms) return RL_EINVAL;
  *out = nullptr;
  *req_throttle_ms = nullptr;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_wait_view without a batch in flight");
  const rl_engine::Flight& f = e->fl[0];
  if (!f.host || f.raw || f.user_out || f.user_thr)
    return e->fail(RL_ESTATE, "rl_wait_view: the oldest batch is not a host batch submitted without output pointers");
  const uint32_t s = f.slot;
  int rc = e->finish(nullptr, nullptr, true);  // (into, with no targets: no copy)
  if (rc) return rc;
  *out = e->stage[s].h_out;
  *req_throttle_ms = e->stage[s].h_thr;
  return 0;
}

// ---- compact host batches (rl_batch_c) ----------------------------------------------------

int rl_host_acquire_c(rl_engine* e, rl_host_batch_c* out) {
  if (!e || !out) return RL_EINVAL;
  if (e->n_fl >= HSLOTS) return e->fail(RL_ESTATE, "rl_host_acquire_c with %d batches in flight (call rl_wait)", HSLOTS);
  const int s = (int)(e->sub_seq % HSLOTS);
  uint8_t* h = e->stage[s].h_in;
  out->prefix_blob = h;
  out->desc_word = reinterpret_cast<uint32_t*>(h + e->o_off);
  out->req_word = reinterpret_cast<uint32_t*>(h + e->o_off + e->c_pitch);
  out->req_of = reinterpret_cast<uint32_t*>(h + e->o_off + 2 * e->c_pitch);
  out->ttl_jitter = reinterpret_cast<uint16_t*>(h + e->o_jit);
  out->max_desc = e->cfg.max_batch_desc;
  out->max_req = e->cfg.max_batch_req;
  out->max_blob = e->cfg.max_blob_bytes;
  out->reserved = 0;
  e->acquired = s;
  return 0;
}

int rl_submit_c(rl_engine* e, const rl_batch_c* b) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl >= HSLOTS) return e->fail(RL_ESTATE, "rl_submit_c with %d batches in flight (call rl_wait)", HSLOTS);
  if (b->n_desc > e->cfg.max_batch_desc || b->n_req > e->cfg.max_batch_req || b->blob_bytes > e->cfg.max_blob_bytes)
    return e->fail(RL_ECAPACITY, "batch exceeds engine capacity (%u desc, %u req, %u blob bytes)",
                   e->cfg.max_batch_desc, e->cfg.max_batch_req, e->cfg.max_blob_bytes);
  if (b->flags & ~(uint32_t)RL_BC_ONE_PER_REQ) return e->fail(RL_EINVAL, "unknown rl_batch_c flags 0x%x", b->flags);
  const bool one = (b->flags & RL_BC_ONE_PER_REQ) != 0;
  if (one && b->n_desc != b->n_req) return e->fail(RL_EINVAL, "RL_BC_ONE_PER_REQ needs n_desc == n_req");
  if (b->n_desc && (!b->desc_word || (!one && !b->req_of))) return e->fail(RL_EINVAL, "null descriptor array");
  if (b->n_req && !b->req_word) return e->fail(RL_EINVAL, "null request array");
  if (b->n_desc && !b->n_req) return e->fail(RL_EINVAL, "descriptors without requests");
  if (b->blob_bytes && !b->prefix_blob) return e->fail(RL_EINVAL, "null prefix_blob");
  if (b->now_base < 0 || b->now_base > MAX_NOW) return e->fail(RL_EINVAL, "now_base outside [0, 0xFFFD0000]");
  if (e->n_fl && e->default_mode() != MODE_V4)
    return e->fail(RL_ESTATE, "a second batch in flight needs the v4 pipeline (call rl_wait)");
  if (!e->d_rules) {
    int rc = rl_load_rules(e, nullptr, 0);
    if (rc) return rc;
  }
  const uint32_t s = (uint32_t)(e->sub_seq % HSLOTS);
  rl_engine::Stage& g = e->stage[s];
  uint8_t* h = g.h_in;
  const size_t P = e->c_pitch;
  struct Arr { const void* src; size_t o, n; } arrs[] = {
      {b->prefix_blob, 0, b->blob_bytes}, {b->desc_word, e->o_off, (size_t)b->n_desc * 4},
      {b->req_word, e->o_off + P, (size_t)b->n_req * 4}, {one ? nullptr : b->req_of, e->o_off + 2 * P, one ? 0 : (size_t)b->n_desc * 4},
      {b->ttl_jitter, e->o_jit, b->ttl_jitter ? (size_t)b->n_desc * 2 : 0}};
  for (auto& a : arrs)
    if (a.n && a.src != h + a.o) memcpy(h + a.o, a.src, a.n);
  memset(h + b->blob_bytes, 0, RL_BLOB_SLACK);  // the device reads prefixes in 16-B words
  e->acquired = -1;
  // Two copies at one descriptor per request: the blob, and the desc and req words as one
  // 2-D copy (rows P apart); req_of, when present, is a third.
  hipError_t he = hipMemcpyAsync(g.d_in, h, (size_t)b->blob_bytes + RL_BLOB_SLACK, hipMemcpyHostToDevice, e->xin);
  const size_t w = (size_t)std::max(b->n_desc, b->n_req) * 4;
  if (he == hipSuccess && w) he = hipMemcpy2DAsync(g.d_cin, P, h + e->o_off, P, w, 2, hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess && arrs[3].n)
    he = hipMemcpyAsync(g.d_cin + 2 * P, h + e->o_off + 2 * P, arrs[3].n, hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess && arrs[4].n)  // (used in place by the pipeline: no expansion)
    he = hipMemcpyAsync(g.d_in + e->o_jit, h + e->o_jit, arrs[4].n, hipMemcpyHostToDevice, e->xin);
  if (he == hipSuccess) he = hipEventRecord(e->ev_in[s], e->xin);
  if (he != hipSuccess) return e->hip_fail(he, "hipMemcpyAsync(H2D compact)");
  // The rl_batch arrays, expanded on the device behind the copies, on the stream k4_hist runs on
  // (the copy stream carries copies only: a kernel there would hold the next batch's H2D copies
  // behind the CUs the batches in flight occupy).
  const bool v4 = e->default_mode() == MODE_V4;
  hipStream_t ks = v4 && e->split_hist() ? e->front : e->stream;
  he = hipStreamWaitEvent(ks, e->ev_in[s], 0);
  if (he != hipSuccess) return e->hip_fail(he, "hipStreamWaitEvent(compact)");
  uint32_t* d_off = reinterpret_cast<uint32_t*>(g.d_in + e->o_off);
  uint32_t* d_rule = reinterpret_cast<uint32_t*>(g.d_in + e->o_rule);
  uint32_t* d_req = reinterpret_cast<uint32_t*>(g.d_in + e->o_req);
  int64_t* d_now = reinterpret_cast<int64_t*>(g.d_in + e->o_now);
  uint32_t* d_hits = reinterpret_cast<uint32_t*>(g.d_in + e->o_hits);
  if (b->n_desc || b->n_req)
    launch_compact_expand(ks, b->n_desc, b->n_req, b->now_base, reinterpret_cast<const uint32_t*>(g.d_cin),
                          reinterpret_cast<const uint32_t*>(g.d_cin + P),
                          one ? nullptr : reinterpret_cast<const uint32_t*>(g.d_cin + 2 * P), g.d_csum, d_off, d_rule,
                          d_req, d_now, d_hits);
  he = hipGetLastError();
  if (he != hipSuccess) return e->hip_fail(he, "compact expand");
  rl_batch d{};
  d.n_desc = b->n_desc;
  d.n_req = b->n_req;
  d.blob_bytes = b->blob_bytes;
  d.reserved = RL_BATCH_RAW;
  d.prefix_blob = g.d_in;
  d.prefix_off = d_off;
  d.rule_id = d_rule;
  d.req_of = d_req;
  d.now = d_now;
  d.hits_addend = d_hits;
  d.ttl_jitter = b->ttl_jitter ? reinterpret_cast<const uint16_t*>(g.d_in + e->o_jit) : nullptr;
  e->st.host_batches += 1;
  // raw replies land in the slot's device output array (8 B of its 20 per descriptor)
  // inputs_ready: the expansion is queued ahead of k4_hist on its stream
  return e->submit_common(d, g.d_out, nullptr, nullptr, nullptr, true, true, nullptr, nullptr, true);
}

int rl_wait_raw_view(rl_engine* e, const rl_raw_reply** out) {
  if (!e || !out) return RL_EINVAL;
  *out = nullptr;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_wait_raw_view without a batch in flight");
  if (!e->fl[0].raw) return e->fail(RL_ESTATE, "rl_wait_raw_view: the oldest batch is not a compact host batch");
  const uint32_t s = e->fl[0].slot;
  int rc = e->finish(nullptr, nullptr, true);
  if (rc) return rc;
  *out = reinterpret_cast<const rl_raw_reply*>(e->stage[s].h_out);
  return 0;
}

int rl_wait_raw_into(rl_engine* e, rl_raw_reply* out) {
  if (!e) return RL_EINVAL;
  if (!e->n_fl) return e->fail(RL_ESTATE, "rl_wait_raw_into without a batch in flight");
  if (!e->fl[0].raw) return e->fail(RL_ESTATE, "rl_wait_raw_into: the oldest batch is not a compact host batch");
  return e->finish(reinterpret_cast<rl_status*>(out), nullptr, true);
}

// GetResponseDescriptorStatus per descriptor from its INCRBY reply (base_limiter.go:70-195),
// with the rules the device decided with (their near thresholds computed as Go does) and the
// decision code the device runs (decide_status, rl_common.h).
int rl_decide_raw(rl_engine* e, const rl_batch_c* b, const rl_raw_reply* raw, uint32_t d0, uint32_t d1,
                  rl_status* out, uint32_t* thr) {
  if (!e || !b || d0 > d1 || d1 > b->n_desc) return RL_EINVAL;
  if (d0 == d1) return 0;
  if (!raw || !out || !thr || !b->desc_word || !b->req_word) return RL_EINVAL;
  const bool one = (b->flags & RL_BC_ONE_PER_REQ) != 0;
  if (!one && !b->req_of) return RL_EINVAL;
  const DevRule* rules = e->h_rules.data();
  const uint32_t n_rules = e->n_rules;
  static_assert(sizeof(rl_raw_reply) == sizeof(RawReply), "raw reply layout");
  // Requests are written once all their descriptors lie in [d0, d1): a request that begins
  // before d0 or ends at or past d1 is left to the call that holds its other descriptors.
  // Requests without descriptors get 0 (the device zeroes every request's ThrottleMillis).
  auto req_at = [&](uint32_t i) { return one ? i : b->req_of[i]; };
  // The caller's arrays are sized by n_req: every request index of the range must fall inside
  // it and never decrease (the device takes nil-limit descriptors without looking at theirs)
  // before anything is written.
  if (one ? d1 > b->n_req : false)
    return e->fail(RL_EINVAL, "rl_decide_raw: %u descriptors, one per request, but %u requests", d1, b->n_req);
  if (!one)
    for (uint32_t i = d0, prev = 0; i < d1; ++i) {
      const uint32_t r = b->req_of[i];
      if (r >= b->n_req || (i > d0 && r < prev))
        return e->fail(RL_EINVAL, "rl_decide_raw: descriptor %u has request index %u (n_req %u, previous %u)", i, r,
                       b->n_req, prev);
      prev = r;
    }
  const uint32_t r_first = req_at(d0), r_last = req_at(d1 - 1);
  const bool first_whole = d0 == 0 || req_at(d0 - 1) != r_first;
  const bool last_whole = d1 == b->n_desc || req_at(d1) != r_last;
  if (d0 == 0)
    for (uint32_t q = 0; q < r_first; ++q) thr[q] = 0;
  if (d1 == b->n_desc)
    for (uint32_t q = r_last + 1; q < b->n_req; ++q) thr[q] = 0;
  uint32_t cur_req = r_first, cur_thr = 0;
  auto flush = [&](uint32_t next) {
    if ((cur_req != r_first || first_whole) && (cur_req != r_last || last_whole)) thr[cur_req] = cur_thr;
    for (uint32_t q = cur_req + 1; q < next; ++q) thr[q] = 0;  // requests without descriptors
  };
  for (uint32_t i = d0; i < d1; ++i) {
    const uint32_t r = req_at(i);
    if (r != cur_req) {
      flush(r);
      cur_req = r;
      cur_thr = 0;
    }
    const uint32_t rw = b->req_word[r];
    const uint32_t rule = b->desc_word[i] >> 16;
    rl_status& st = out[i];
    if (rule == RL_NIL_RULE16 || (raw[i].flags & RL_RAW_NIL)) {  // base_limiter.go:72-75
      st.code_flags = RL_CODE_OK;
      st.limit_remaining = st.reset_s = st.over_limit_delta = st.near_limit_delta = 0;
      continue;
    }
    if (rule >= n_rules) return e->fail(RL_EINVAL, "rl_decide_raw: descriptor %u has rule %u of %u", i, rule, n_rules);
    const DevRule& R = rules[rule];
    const uint64_t now = (uint64_t)(b->now_base + (int64_t)(rw >> 24));
    const uint32_t hh = rw & 0xFFFFFFu;
    const uint32_t h = hh > 1u ? hh : 1u;  // utils.Max(1, HitsAddend)  fixed_cache_impl.go:39
    const uint32_t now_mod = (uint32_t)(now % R.div);
    const uint32_t t = decide_status(raw[i].after, (raw[i].flags & RL_RAW_LOCAL_HIT) != 0u, h, now_mod, R, st);
    cur_thr = t > cur_thr ? t : cur_thr;  // response.ThrottleMillis = max  base_limiter.go:163-165
  }
  flush(cur_req + 1);
  return 0;
}

int rl_submit_device(rl_engine* e, const rl_batch* b, rl_status* d_out, uint32_t* d_req_throttle_ms) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_submit_device while a batch is in flight (call rl_wait)");
  int rc = e->check_batch(b, false);
  if (rc) return rc;
  return e->submit_common(*b, d_out, d_req_throttle_ms, nullptr, nullptr, false, false, nullptr, nullptr);
}

int rl_submit_pipelined(rl_engine* e, const rl_batch* b, rl_status* d_out, uint32_t* d_req_throttle_ms) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl >= HSLOTS)
    return e->fail(RL_ESTATE, "rl_submit_pipelined with %d batches in flight (call rl_wait)", HSLOTS);
  int rc = e->check_batch(b, false);
  if (rc) return rc;
  if (e->n_fl && e->default_mode() != MODE_V4)
    return e->fail(RL_ESTATE, "a second batch in flight needs the v4 pipeline (call rl_wait)");
  for (int q = 0; q < e->n_fl; ++q)
    if (e->fl[q].out == d_out || e->fl[q].thr == d_req_throttle_ms)
      return e->fail(RL_EINVAL, "batches in flight together need distinct output buffers");
  return e->submit_common(*b, d_out, d_req_throttle_ms, nullptr, nullptr, true, false, nullptr, nullptr);
}

void* rl_stream(rl_engine* e) { return e ? (void*)e->stream : nullptr; }

int rl_set_stream(rl_engine* e, void* hip_stream) {
  if (!e) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_set_stream while a batch is in flight");
  hipError_t he = hipStreamSynchronize(e->stream);  // work already queued finishes first
  if (he != hipSuccess) return e->hip_fail(he, "hipStreamSynchronize");
  e->stream = hip_stream ? (hipStream_t)hip_stream : e->own_stream;
  return 0;
}

// The checks and launches shared by rl_route_pack and rl_route_pack_async (d_x: the async
// form's (count, status) pairs; d_send_counts: the synchronous form's counts).
static int route_pack_launch(rl_engine* e, const rl_batch* b, uint32_t origin, uint32_t n_shards, void* d_send,
                             uint32_t* d_send_counts, uint32_t* d_perm, uint32_t* d_x) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_route_pack while a batch is in flight (call rl_wait)");
  if (n_shards == 0 || n_shards > ROUTE_MAX_SHARDS || origin >= ROUTE_MAX_SHARDS)
    return e->fail(RL_EINVAL, "n_shards must be 1..%u and origin < %u", ROUTE_MAX_SHARDS, ROUTE_MAX_SHARDS);
  if (b->n_desc > e->cfg.max_batch_desc) return e->fail(RL_ECAPACITY, "batch exceeds engine capacity");
  if (b->n_req > RL_ROUTE_MAX_REQ) return e->fail(RL_EINVAL, "routed batch holds more than 2^27 requests");
  if (b->reserved) return e->fail(RL_EINVAL, "rl_batch.reserved must be 0");
  if ((!d_send_counts && !d_x) || (b->n_desc && (!d_send || !d_perm))) return e->fail(RL_EINVAL, "null routing buffer");
  if (!e->d_rules) rl_load_rules(e, nullptr, 0);
  hipError_t he = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && he == hipSuccess) he = x; };
  const size_t N = e->cfg.max_batch_desc ? e->cfg.max_batch_desc : 1;
  if (!e->r_tmp) {
    chk(hipMalloc(&e->r_tmp, N * sizeof(RRec)));
    chk(hipMalloc(&e->r_own, N));
    if (!e->r_bcnt) chk(hipMalloc(&e->r_bcnt, (size_t)route_bcnt_words((uint32_t)N) * 4));  // (strided pack)
    chk(hipMalloc(&e->r_ctl, sizeof(EngineCtl)));
    chk(hipHostMalloc(&e->h_route, 64 * 4, hipHostMallocDefault));
    if (he != hipSuccess) return e->hip_fail(he, "router scratch allocation");
  }
  // k_route_scan writes the error word and the owner totals into r_ctl's first words (and
  // the pairs into d_x)
  launch_route_pack(e->stream, *b, e->d_rules, e->n_rules, e->cfg.hash_seed, origin, n_shards, e->r_tmp, e->r_own,
                    e->r_bcnt, reinterpret_cast<RRec*>(d_send), d_send_counts, d_perm, e->r_ctl, d_x);
  chk(hipGetLastError());
  if (he != hipSuccess) return e->hip_fail(he, "rl_route_pack");
  return 0;
}

int rl_route_pack(rl_engine* e, const rl_batch* b, uint32_t origin, uint32_t n_shards, void* d_send,
                  uint32_t* d_send_counts, uint32_t* d_perm, uint32_t* h_send_counts) {
  if (!d_send_counts || !h_send_counts) return e ? e->fail(RL_EINVAL, "null routing buffer") : RL_EINVAL;
  if (int rc = route_pack_launch(e, b, origin, n_shards, d_send, d_send_counts, d_perm, nullptr)) return rc;
  hipError_t he = hipMemcpyAsync(e->h_route, e->r_ctl, (1 + n_shards) * 4, hipMemcpyDeviceToHost, e->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
  if (he != hipSuccess) return e->hip_fail(he, "rl_route_pack");
  const uint32_t errs = e->h_route[0];
  if (errs & ERR_BAD_INPUT)
    return e->fail(RL_EINVAL, "batch references an unknown rule id or request index, or malformed prefix offsets");
  if (errs & ERR_BAD_TIME) return e->fail(RL_EINVAL, "request time outside [0, 0xFFFD0000] unix seconds");
  memcpy(h_send_counts, e->h_route + 1, n_shards * 4);
  return 0;
}

int rl_route_pack_async(rl_engine* e, const rl_batch* b, uint32_t origin, uint32_t n_shards, void* d_send,
                        uint32_t* d_x, uint32_t* d_perm) {
  if (!d_x) return e ? e->fail(RL_EINVAL, "null routing buffer") : RL_EINVAL;
  return route_pack_launch(e, b, origin, n_shards, d_send, nullptr, d_perm, d_x);
}

int rl_route_pack_strided(rl_engine* e, const rl_batch* b, uint32_t origin, uint32_t n_shards, uint32_t stride,
                          void* d_send, uint32_t* d_x, uint32_t* d_perm) {
  if (!d_x) return e ? e->fail(RL_EINVAL, "null routing buffer") : RL_EINVAL;
  if (!e || !b) return RL_EINVAL;
  if (b->n_desc > stride) return e->fail(RL_ECAPACITY, "batch of %u descriptors exceeds the owner stride %u", b->n_desc, stride);
  if (stride > RL_ROUTE_MAX_REQ) return e->fail(RL_EINVAL, "owner stride above 2^27 records");
  // the same checks and scratch as the three-kernel pack; its launches are replaced below
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_route_pack while a batch is in flight (call rl_wait)");
  if (n_shards == 0 || n_shards > ROUTE_MAX_SHARDS || origin >= ROUTE_MAX_SHARDS)
    return e->fail(RL_EINVAL, "n_shards must be 1..%u and origin < %u", ROUTE_MAX_SHARDS, ROUTE_MAX_SHARDS);
  if (b->n_desc > e->cfg.max_batch_desc) return e->fail(RL_ECAPACITY, "batch exceeds engine capacity");
  if (b->n_req > RL_ROUTE_MAX_REQ) return e->fail(RL_EINVAL, "routed batch holds more than 2^27 requests");
  if (b->reserved) return e->fail(RL_EINVAL, "rl_batch.reserved must be 0");
  if (b->n_desc && (!d_send || !d_perm)) return e->fail(RL_EINVAL, "null routing buffer");
  if (!e->d_rules) rl_load_rules(e, nullptr, 0);
  const size_t N = e->cfg.max_batch_desc ? e->cfg.max_batch_desc : 1;
  hipError_t he = hipSuccess;
  if (!e->r_bcnt) he = hipMalloc(&e->r_bcnt, (size_t)route_bcnt_words((uint32_t)N) * 4);
  if (he == hipSuccess) he = hipMemsetAsync(e->r_bcnt, 0, (size_t)route_bcnt_words(b->n_desc) * 4, e->stream);
  if (he == hipSuccess) {
    launch_route_pack_strided(e->stream, *b, e->d_rules, e->n_rules, e->cfg.hash_seed, origin, n_shards, stride,
                              reinterpret_cast<RRec*>(d_send), d_perm, e->r_bcnt, d_x);
    he = hipGetLastError();
  }
  return he == hipSuccess ? 0 : e->hip_fail(he, "rl_route_pack_strided");
}

int rl_submit_routed(rl_engine* e, const void* d_records, uint32_t n, void* d_reply) {
  if (!e) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_submit_routed while a batch is in flight (call rl_wait)");
  if (n > e->cfg.max_batch_desc)
    return e->fail(RL_ECAPACITY, "routed batch of %u records exceeds engine capacity (%u desc)", n,
                   e->cfg.max_batch_desc);
  if (n && (!d_records || !d_reply)) return e->fail(RL_EINVAL, "null routed buffer");
  if (!e->d_rules) rl_load_rules(e, nullptr, 0);
  if (!e->r_thr) {
    const size_t N = e->cfg.max_batch_desc ? e->cfg.max_batch_desc : 1;
    hipError_t he = hipMalloc(&e->r_thr, N * 4 + 64);
    if (he == hipSuccess) he = hipMalloc(&e->r_out, N * sizeof(rl_status) + 64);
    if (he != hipSuccess) return e->hip_fail(he, "router scratch allocation");
  }
  rl_batch b{};
  b.n_desc = n;
  b.n_req = n;  // every record has its own ThrottleMillis slot
  b.reserved = RL_BATCH_ROUTED;
  b.prefix_blob = reinterpret_cast<const uint8_t*>(d_records);
  return e->submit_common(b, e->r_out, e->r_thr, reinterpret_cast<RReply*>(d_reply), nullptr, false, false, nullptr,
                          nullptr);
}

int rl_submit_routed_async(rl_engine* e, const void* d_records, uint32_t n, void* d_reply, uint32_t flags,
                           void* ready_event) {
  if (!e) return RL_EINVAL;
  if (flags & ~RL_ROUTED_RAW) return e->fail(RL_EINVAL, "unknown rl_submit_routed_async flags 0x%x", flags);
  if (!(flags & RL_ROUTED_RAW)) {
    if (ready_event) return e->fail(RL_EINVAL, "rl_submit_routed_async: status replies need ready_event == NULL");
    return rl_submit_routed(e, d_records, n, d_reply);
  }
  if (e->n_fl >= HSLOTS)
    return e->fail(RL_ESTATE, "rl_submit_routed_async with %d batches in flight (call rl_wait)", HSLOTS);
  if (e->n_fl && e->default_mode() != MODE_V4)
    return e->fail(RL_ESTATE, "a second batch in flight needs the v4 pipeline (call rl_wait)");
  if (n > e->cfg.max_batch_desc)
    return e->fail(RL_ECAPACITY, "routed batch of %u records exceeds engine capacity (%u desc)", n,
                   e->cfg.max_batch_desc);
  if (n && (!d_records || !d_reply)) return e->fail(RL_EINVAL, "null routed buffer");
  for (int q = 0; q < e->n_fl; ++q)
    if (e->fl[q].out == reinterpret_cast<rl_status*>(d_reply))
      return e->fail(RL_EINVAL, "batches in flight together need distinct reply buffers");
  if (!e->d_rules) rl_load_rules(e, nullptr, 0);
  rl_batch b{};
  b.n_desc = n;
  b.n_req = n;
  b.reserved = RL_BATCH_ROUTED | RL_BATCH_RAW;
  b.prefix_blob = reinterpret_cast<const uint8_t*>(d_records);
  // the replies are the pipeline's output array (RawReply per record); no ThrottleMillis slots
  return e->submit_common(b, reinterpret_cast<rl_status*>(d_reply), nullptr, nullptr,
                          reinterpret_cast<hipEvent_t>(ready_event), false, false, nullptr, nullptr);
}

int rl_route_unpack(rl_engine* e, const rl_batch* b, const uint32_t* d_perm, const void* d_reply, rl_status* d_out,
                    uint32_t* d_req_throttle_ms) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_route_unpack while a batch is in flight (call rl_wait)");
  if (b->n_desc && (!d_perm || !d_out || !b->req_of)) return e->fail(RL_EINVAL, "null routing buffer");
  if (b->n_req && !d_req_throttle_ms) return e->fail(RL_EINVAL, "null throttle buffer");
  hipError_t he = hipSuccess;
  if (b->n_req) he = hipMemsetAsync(d_req_throttle_ms, 0, (size_t)b->n_req * 4, e->stream);
  if (he == hipSuccess) {
    launch_route_unpack(e->stream, b->n_desc, b->req_of, d_perm, reinterpret_cast<const RReply*>(d_reply), d_out,
                        d_req_throttle_ms);
    he = hipGetLastError();
  }
  return he == hipSuccess ? 0 : e->hip_fail(he, "rl_route_unpack");
}

int rl_reset(rl_engine* e) {
  if (!e) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_reset while a batch is in flight");
  e->hot.clear();
  e->hot_dirty = true;
  e->cand_pending = false;
  e->cand_stash.clear();
  hipError_t he = hipMemsetAsync(e->table, 0, e->table_slots * sizeof(Slot), e->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
  if (he != hipSuccess) return e->hip_fail(he, "rl_reset");
  e->st.live_keys = 0;
  return e->reset_occ();
}

int rl_get_stats(rl_engine* e, rl_engine_stats* s) {
  if (!e || !s) return RL_EINVAL;
  *s = e->st;
  return 0;
}

int rl_get_occupancy(rl_engine* e, rl_occupancy* o) {
  if (!e || !o) return RL_EINVAL;
  for (int r = 0; r < 8; ++r) {
    o->gen[r] = e->occ[r].gen;
    o->live[r] = e->occ[r].live;
    o->limit[r] = e->occ[r].limit;
    o->slots[r] = 1u << e->tab.region_log2[r];
  }
  return 0;
}

int rl_set_timing(rl_engine* e, int on) {
  if (!e) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_set_timing while a batch is in flight");
  e->timing = on != 0;
  for (int k = 0; k < KT_COUNT; ++k) { e->kt_ms[k] = 0; e->kt_n[k] = 0; }
  return 0;
}

int rl_kernel_times(rl_engine* e, const char** names, double* total_ms, uint64_t* launches, uint32_t cap,
                    uint32_t* n_out) {
  if (!e) return RL_EINVAL;
  uint32_t n = 0;
  for (int k = 0; k < KT_COUNT && n < cap; ++k, ++n) {
    if (names) names[n] = kKernelNames[k];
    if (total_ms) total_ms[n] = e->kt_ms[k];
    if (launches) launches[n] = e->kt_n[k];
  }
  if (n_out) *n_out = n;
  return 0;
}

int rl_last_batch_info(rl_engine* e, uint64_t* unique_keys, uint64_t* n_desc, uint64_t* n_req, uint64_t* blob_bytes) {
  if (!e) return RL_EINVAL;
  if (unique_keys) *unique_keys = e->last_unique;
  if (n_desc) *n_desc = e->last_n;
  if (n_req) *n_req = e->last_req;
  if (blob_bytes) *blob_bytes = e->last_blob;
  return 0;
}

int rl_load_tree(rl_engine* e, const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names, uint32_t names_len) {
  if (!e) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_load_tree while a batch is in flight");
  if ((n_nodes && !nodes) || (names_len && !names)) return e->fail(RL_EINVAL, "null tree array");
  std::vector<TreeNodeDev> hn;
  std::vector<uint64_t> hs;
  std::string err;
  uint32_t mask = 0;
  int rc = build_tree(nodes, n_nodes, names, names_len, hn, hs, mask, err);
  if (rc) return e->fail(rc, "%s", err.c_str());
  std::vector<FastNode> fn;
  std::vector<uint64_t> fs;
  uint32_t fmask = 0;
  build_fast_tree(hn, names, fn, fs, fmask);
  hipError_t he = hipStreamSynchronize(e->stream);  // resolutions queued on the old tree finish first
  hipFree(e->d_tree_nodes);
  hipFree(e->d_tree_slots);
  hipFree(e->d_tree_names);
  hipFree(e->d_tree_fnodes);
  hipFree(e->d_tree_fslots);
  e->d_tree_nodes = nullptr;
  e->d_tree_slots = nullptr;
  e->d_tree_names = nullptr;
  e->d_tree_fnodes = nullptr;
  e->d_tree_fslots = nullptr;
  e->has_tree = false;
  if (he == hipSuccess) he = hipMalloc(&e->d_tree_nodes, std::max<size_t>(1, hn.size()) * sizeof(TreeNodeDev));
  if (he == hipSuccess) he = hipMalloc(&e->d_tree_slots, hs.size() * 8);
  if (he == hipSuccess) he = hipMalloc(&e->d_tree_names, std::max<size_t>(16, names_len));
  if (he == hipSuccess && !hn.empty())
    he = hipMemcpy(e->d_tree_nodes, hn.data(), hn.size() * sizeof(TreeNodeDev), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemcpy(e->d_tree_slots, hs.data(), hs.size() * 8, hipMemcpyHostToDevice);
  if (he == hipSuccess && names_len) he = hipMemcpy(e->d_tree_names, names, names_len, hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMalloc(&e->d_tree_fnodes, std::max<size_t>(1, fn.size()) * sizeof(FastNode));
  if (he == hipSuccess) he = hipMalloc(&e->d_tree_fslots, fs.size() * 8);
  if (he == hipSuccess && !fn.empty())
    he = hipMemcpy(e->d_tree_fnodes, fn.data(), fn.size() * sizeof(FastNode), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemcpy(e->d_tree_fslots, fs.data(), fs.size() * 8, hipMemcpyHostToDevice);
  if (he != hipSuccess) return e->hip_fail(he, "rl_load_tree");
  e->tree.nodes = e->d_tree_nodes;
  e->tree.slots = e->d_tree_slots;
  e->tree.names = e->d_tree_names;
  e->tree.mask = mask;
  e->tree.fnodes = e->d_tree_fnodes;
  e->tree.fslots = e->d_tree_fslots;
  e->tree.fmask = fmask;
  e->tree.n_fnodes = (uint32_t)fn.size();
  e->has_tree = true;
  return 0;
}

static ResolveIn resolve_in(const rl_resolve_batch* b) {
  ResolveIn in;
  in.n_desc = b->n_desc;
  in.n_entries = b->n_entries;
  in.bytes_len = b->bytes_len;
  in.bytes = b->bytes;
  in.domain = b->domain;
  in.entry_first = b->entry_first;
  in.entry = b->entry;
  in.override_rule = b->override_rule;
  return in;
}

int rl_resolve_device(rl_engine* e, const rl_resolve_batch* b, uint32_t* d_rule_out) {
  if (!e || !b) return RL_EINVAL;
  if (!e->has_tree) return e->fail(RL_ESTATE, "rl_resolve without a tree (rl_load_tree)");
  if (b->reserved) return e->fail(RL_EINVAL, "rl_resolve_batch.reserved must be 0");
  if (!b->n_desc) return 0;
  if (!b->domain || !b->entry_first || !d_rule_out || (b->n_entries && (!b->entry || !b->bytes)))
    return e->fail(RL_EINVAL, "null resolve array");
  // On the stream the next submit's first kernel runs on: the front stream while batches are in
  // flight (k4_hist of the next batch runs there, beside the decisions of the one before), else
  // the engine stream — so resolving the next batch never waits for the batch in flight.
  const bool front = e->default_mode() == MODE_V4 && e->split_hist();
  // (kernel timing runs everything on the engine stream: split_hist() is off then)
  const uint32_t nf = resolve_flag_words(b->n_desc);
  if (nf > e->res_flag_cap) {  // the first batch of a size (then sized for the engine's batches)
    const uint32_t cap = std::max(nf, resolve_flag_words(e->cfg.max_batch_desc));
    hipError_t fe = hipDeviceSynchronize();  // older resolves may still read them
    if (fe == hipSuccess) {
      hipFree(e->d_res_flags);
      e->d_res_flags = nullptr;
      e->res_flag_cap = 0;
      fe = hipMalloc(&e->d_res_flags, (size_t)cap * 4 * rl_engine::RES_FLAG_SLOTS);
      if (fe == hipSuccess) fe = hipMemset(e->d_res_flags, 0, (size_t)cap * 4 * rl_engine::RES_FLAG_SLOTS);
    }
    if (fe != hipSuccess) return e->hip_fail(fe, "rl_resolve flags");
    e->res_flag_cap = cap;
  }
  uint32_t* flags = e->d_res_flags + (size_t)(e->res_seq++ % rl_engine::RES_FLAG_SLOTS) * e->res_flag_cap;
  const uint32_t seq = (uint32_t)(e->res_seq % 0xFFFFFFFFull) + 1u;  // non-zero, differs from the slot's last
  e->timed(KT_RESOLVE, [&] {
    launch_resolve(front ? e->front : e->stream, resolve_in(b), e->tree, d_rule_out, flags, seq);
  });
  hipError_t he = hipGetLastError();
  if (he == hipSuccess && front) {
    // a next submit that does not start on the front stream waits for it (run_pipeline)
    he = hipEventRecord(e->ev_resolve, e->front);
    e->resolve_pending = he == hipSuccess;
  }
  return he == hipSuccess ? 0 : e->hip_fail(he, "k_resolve launch");
}

int rl_resolve(rl_engine* e, const rl_resolve_batch* b, uint32_t* rule_out) {
  if (!e || !b) return RL_EINVAL;
  if (e->n_fl) return e->fail(RL_ESTATE, "rl_resolve while a batch is in flight");
  if (!e->has_tree) return e->fail(RL_ESTATE, "rl_resolve without a tree (rl_load_tree)");
  if (b->reserved) return e->fail(RL_EINVAL, "rl_resolve_batch.reserved must be 0");
  const uint32_t n = b->n_desc, ne = b->n_entries;
  if (!n) return 0;
  if (!b->domain || !b->entry_first || !rule_out || (ne && (!b->entry || !b->bytes)))
    return e->fail(RL_EINVAL, "null resolve array");
  // Host-side bounds checks: every string inside bytes, entry ranges monotone and inside n_entries.
  if (b->entry_first[0] != 0 || b->entry_first[n] != ne) return e->fail(RL_EINVAL, "entry_first must span [0, n_entries]");
  for (uint32_t i = 0; i < n; ++i) {
    if (b->entry_first[i + 1] < b->entry_first[i]) return e->fail(RL_EINVAL, "entry_first not monotone at %u", i);
    if ((uint64_t)b->domain[2 * i] + b->domain[2 * i + 1] > b->bytes_len)
      return e->fail(RL_EINVAL, "domain string outside bytes at %u", i);
  }
  for (uint32_t k = 0; k < ne; ++k)
    if ((uint64_t)b->entry[4 * k] + b->entry[4 * k + 1] > b->bytes_len ||
        (uint64_t)b->entry[4 * k + 2] + b->entry[4 * k + 3] > b->bytes_len)
      return e->fail(RL_EINVAL, "entry string outside bytes at %u", k);
  const size_t o_dom = align_up(b->bytes_len + 16, 256), o_ef = o_dom + align_up((size_t)n * 8, 256),
               o_ent = o_ef + align_up(((size_t)n + 1) * 4, 256), o_ov = o_ent + align_up((size_t)ne * 16, 256),
               o_out = o_ov + align_up((size_t)n * 4, 256), total = o_out + align_up((size_t)n * 4, 256);
  hipError_t he = hipSuccess;
  if (total > e->res_cap) {
    hipFree(e->d_res);
    e->d_res = nullptr;
    he = hipMalloc(&e->d_res, total);
    if (he != hipSuccess) { e->res_cap = 0; return e->hip_fail(he, "rl_resolve staging"); }
    e->res_cap = total;
  }
  uint8_t* d = e->d_res;
  struct Cp { size_t o; const void* src; size_t n; } cps[] = {
      {0, b->bytes, b->bytes_len}, {o_dom, b->domain, (size_t)n * 8}, {o_ef, b->entry_first, ((size_t)n + 1) * 4},
      {o_ent, b->entry, (size_t)ne * 16}, {o_ov, b->override_rule, b->override_rule ? (size_t)n * 4 : 0}};
  for (auto& c : cps)
    if (c.n && he == hipSuccess) he = hipMemcpyAsync(d + c.o, c.src, c.n, hipMemcpyHostToDevice, e->stream);
  if (he != hipSuccess) return e->hip_fail(he, "rl_resolve H2D");
  rl_resolve_batch db = *b;
  db.bytes = d;
  db.domain = reinterpret_cast<const uint32_t*>(d + o_dom);
  db.entry_first = reinterpret_cast<const uint32_t*>(d + o_ef);
  db.entry = reinterpret_cast<const uint32_t*>(d + o_ent);
  db.override_rule = b->override_rule ? reinterpret_cast<const uint32_t*>(d + o_ov) : nullptr;
  int rc = rl_resolve_device(e, &db, reinterpret_cast<uint32_t*>(d + o_out));
  if (rc) return rc;
  he = hipMemcpyAsync(rule_out, d + o_out, (size_t)n * 4, hipMemcpyDeviceToHost, e->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
  return he == hipSuccess ? 0 : e->hip_fail(he, "rl_resolve D2H");
}

}  // extern "C"
