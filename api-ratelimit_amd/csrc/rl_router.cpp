// rl_router.cpp — the routed DoLimit step behind the C ABI (include/rl_hip.h
// "Router object").
//
// The reference sends each key's INCRBY to the Redis server that holds it and pipelines the
// commands of a request (src/redis/fixed_cache_impl.go:66-80, src/redis/driver_impl.go:84-110).
// Here GPU s owns the keys whose prefix fingerprint maps to s (route_owner). One step:
//   origin   pack its batch by owner into a strided send buffer: one record per descriptor,
//            except hot prefixes (the shard's route hot set), whose descriptors travel as ONE
//            combined record per prefix carrying their sum of hits_addend (rl_route.hip)
//   exchange per-owner (count, status) pairs, then the records (all-to-all)
//   owner    decide the records received from every origin, in origin order, answering each
//            with its raw INCRBY post-value (rl_submit_routed_async, RL_ROUTED_RAW)
//   exchange the owners' statuses and the raw replies (reverse all-to-all)
//   origin   every descriptor's post-value from its record's reply (and, inside a combined
//            record, its prefix of hits_addend), then its decision (k_route_unpack_raw)
//
// Transports: collective (one rank per GPU: RCCL's ncclAllToAll / ncclAllToAllv / ncclAllGather
// on a stream the router owns, or the same code path over an in-process emulation of those three
// collectives for G ranks driven by G threads of one process — device copies driven by the very
// count and displacement vectors RCCL would get, every rank's counts checked against its peers',
// so the N > 1 exchange runs and is tested on one GPU) or local (n_shards engines in one process,
// device copies). Status words ride in the counts exchange (pack) and the reply exchange
// (decide, and any local HIP failure after the counts), so every shard completes every
// collective of a step and all of them fail together.
//
// Time: each origin's (count, status) word pair to an owner carries its batch's
// request-time range. An owner decides its records origin by origin in runs whose times span at
// most one second (the engine's window rule), so origins whose clocks or batch cuts differ by
// seconds never make a step fail; the table keeps a SECOND key string findable for a request up
// to 3 s behind the newest time it has seen (rl_common.h slot_free_for, RL_CFG_LAG_WINDOW); an
// origin further behind the node's step clock is left out of the step alone (RL_ELATE on its
// shard; every other shard's step goes ahead).
//
// Two steps may be in flight (rl_router_submit / rl_router_wait): step k+1's pack, counts and
// record exchange run on the origin and exchange streams while step k's owner batch is decided
// on the engine's streams (the engine pipelines routed batches like rl_submit_pipelined).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "rl_common.h"
#include "rl_hip.h"
#include "rl_internal.h"

using namespace rlhip;

namespace {

constexpr uint32_t REC = sizeof(RRec);
constexpr uint32_t RAWB = sizeof(RawReply);
constexpr uint32_t MAXS = RL_ROUTE_MAX_SHARDS;
constexpr int NSLOT = 3;                   // steps in flight
constexpr uint64_t ROUTE_HOT_EVERY = 8;    // route hot set refresh period (steps)
constexpr uint32_t ROUTE_HOT_KEEP = 64;    // a group stays while its origin sends it >= this sum of hits per step
static_assert(REC == RL_ROUTE_RECORD_BYTES && RAWB == sizeof(rl_raw_reply), "record layouts");
// d_x / h_x words per step: [XS G] (count, status, tmin, tmax) sent to each owner | [XS G] received
// from each origin | [G] decide statuses sent | [G] received; the pinned mirror then holds the hot
// scan's group sums and control words at HX_HOT
constexpr uint32_t XS = 4;
constexpr uint32_t HX_HOT = (2 * XS + 2) * MAXS;
constexpr uint32_t MAX_LAG_S = 3;          // a request may come this many seconds behind the step clock

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Fault injection for the tests (RL_ROUTER_FAULT="phase:shard", read at create, fires once):
// the shard behaves as if a HIP call of that phase failed.
// "comm": the shard's communicator fails at the counts exchange (the transport aborts; every rank
// is broken from then on).
// "stall": the shard's exchange stream stalls before the counts exchange (a device kernel that
// waits for the router's abort, at most 20 s), as if a peer never reached the collective.
enum Phase { PH_NONE = 0, PH_PACK, PH_RECORDS, PH_DECIDE, PH_REPLIES, PH_UNPACK, PH_STATUS, PH_COMM, PH_STALL };
const char* const kPhaseNames[] = {"", "pack", "records", "decide", "replies", "unpack", "status", "comm", "stall"};

// ---- collective transports ----------------------------------------------------------------
// The three collectives a routed step uses, in bytes, on the router's exchange stream.
struct Xport {
  virtual ~Xport() = default;
  virtual ncclResult_t a2av(const void* s, const size_t* sc, const size_t* sd, void* r, const size_t* rc,
                            const size_t* rd, hipStream_t st) = 0;
  virtual ncclResult_t a2a(const void* s, void* r, size_t n, hipStream_t st) = 0;
  virtual ncclResult_t allgather(const void* s, void* r, size_t n, hipStream_t st) = 0;
  virtual ncclResult_t group_start() { return ncclSuccess; }
  virtual ncclResult_t group_end() { return ncclSuccess; }
  virtual void abort() = 0;
  // an asynchronous failure of the communicator (a peer's, or the network's), polled while the
  // host waits for work behind a collective
  virtual ncclResult_t async_error() = 0;
  virtual std::string why(ncclResult_t r) { return ncclGetErrorString(r); }
};

struct RcclXport : Xport {
  ncclComm_t comm = nullptr;
  ~RcclXport() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  ncclResult_t a2av(const void* s, const size_t* sc, const size_t* sd, void* r, const size_t* rc, const size_t* rd,
                    hipStream_t st) override {
    return ncclAllToAllv(s, sc, sd, r, rc, rd, ncclUint8, comm, st);
  }
  ncclResult_t a2a(const void* s, void* r, size_t n, hipStream_t st) override {
    return ncclAllToAll(s, r, n, ncclUint8, comm, st);
  }
  ncclResult_t allgather(const void* s, void* r, size_t n, hipStream_t st) override {
    return ncclAllGather(s, r, n, ncclUint8, comm, st);
  }
  ncclResult_t group_start() override { return ncclGroupStart(); }
  ncclResult_t group_end() override { return ncclGroupEnd(); }
  void abort() override {
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
  }
  ncclResult_t async_error() override {
    ncclResult_t r = ncclSuccess;
    if (comm && ncclCommGetAsyncError(comm, &r) != ncclSuccess) return ncclSystemError;
    return r;
  }
};

// In-process emulation of the collectives for G ranks (one thread each, one or more devices of
// this process): every rank posts its buffers, count and displacement vectors and an event
// recorded on its exchange stream; after a host barrier each rank copies what its peers send it
// (device-to-device on its own stream, behind their events), checking that each peer's send
// count equals its own receive count (RCCL would silently corrupt: here the world aborts with
// the mismatch); a second barrier orders every peer's copies before a rank's stream moves on
// (its send buffer may be rewritten then), as the completion of an RCCL collective does.
struct EmuWorld {
  uint32_t G = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint32_t arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  int refs = 0;
  std::string why;
  struct Post {
    const uint8_t* s;
    uint8_t* r;
    size_t sc[MAXS], sd[MAXS];
    hipEvent_t ev;
  };
  Post post[MAXS];
  hipEvent_t done[MAXS];
  int64_t timeout_ms = 120000;  // the routers' RL_ROUTER_TIMEOUT_MS
  // all G ranks arrive, or the world aborts (a rank failed, or one never came within the timeout)
  bool barrier() {
    std::unique_lock<std::mutex> l(mu);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == G) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(l, std::chrono::milliseconds(timeout_ms), [&] { return gen != g || aborted; });
    if (aborted) return false;
    if (!ok) {
      aborted = true;
      why = "a rank did not arrive at a collective within " + std::to_string(timeout_ms) + " ms";
      cv.notify_all();
      return false;
    }
    return true;
  }
  void abort(const std::string& w) {
    std::lock_guard<std::mutex> l(mu);
    if (!aborted && why.empty()) why = w;
    aborted = true;
    cv.notify_all();
  }
};
constexpr uint64_t EMU_MAGIC = 0x444c524f57554d45ull;  // "EMUWORLD"

// Host exchange (RL_ROUTER_HOST_XCHG, tests): each collective drains the stream, copies the send
// sections to host memory (compact), calls the caller's all-to-all-v of host bytes, and copies
// the received sections to their device displacements. The collective transport's code runs
// unchanged with one process per rank.
struct HostXchgXport : Xport {
  rl_host_xchg_fn fn = nullptr;
  void* ctx = nullptr;
  uint32_t G = 0;
  bool failed = false;
  std::vector<uint8_t> hs, hr;
  ncclResult_t a2av(const void* s, const size_t* sc, const size_t* sd, void* r, const size_t* rc, const size_t* rd,
                    hipStream_t st) override {
    if (failed) return ncclRemoteError;
    size_t cs[MAXS], ds[MAXS], cr[MAXS], dr[MAXS], ns = 0, nr = 0;
    for (uint32_t j = 0; j < G; ++j) {
      cs[j] = sc[j], ds[j] = ns, ns += sc[j];
      cr[j] = rc[j], dr[j] = nr, nr += rc[j];
    }
    hs.resize(std::max<size_t>(ns, 1));
    hr.resize(std::max<size_t>(nr, 1));
    hipError_t he = hipStreamSynchronize(st);
    for (uint32_t j = 0; j < G && he == hipSuccess; ++j)
      if (cs[j]) he = hipMemcpy(hs.data() + ds[j], static_cast<const uint8_t*>(s) + sd[j], cs[j], hipMemcpyDeviceToHost);
    if (he != hipSuccess || fn(ctx, hs.data(), cs, ds, hr.data(), cr, dr) != 0) {
      failed = true;
      return he != hipSuccess ? ncclUnhandledCudaError : ncclRemoteError;
    }
    for (uint32_t j = 0; j < G && he == hipSuccess; ++j)
      if (cr[j]) he = hipMemcpyAsync(static_cast<uint8_t*>(r) + rd[j], hr.data() + dr[j], cr[j], hipMemcpyHostToDevice, st);
    if (he == hipSuccess) he = hipStreamSynchronize(st);  // (hr is reused by the next collective)
    if (he != hipSuccess) {
      failed = true;
      return ncclUnhandledCudaError;
    }
    return ncclSuccess;
  }
  ncclResult_t a2a(const void* s, void* r, size_t n, hipStream_t st) override {
    size_t c[MAXS], d[MAXS];
    for (uint32_t j = 0; j < G; ++j) c[j] = n, d[j] = j * n;
    return a2av(s, c, d, r, c, d, st);
  }
  ncclResult_t allgather(const void* s, void* r, size_t n, hipStream_t st) override {
    size_t c[MAXS], z[MAXS], d[MAXS];
    for (uint32_t j = 0; j < G; ++j) c[j] = n, z[j] = 0, d[j] = j * n;
    return a2av(s, c, z, r, c, d, st);
  }
  void abort() override { failed = true; }
  ncclResult_t async_error() override { return failed ? ncclRemoteError : ncclSuccess; }
  std::string why(ncclResult_t r) override { return std::string("host exchange: ") + ncclGetErrorString(r); }
};
thread_local rl_host_xchg_fn t_xchg_fn = nullptr;
thread_local void* t_xchg_ctx = nullptr;

struct EmuXport : Xport {
  EmuWorld* w = nullptr;
  uint32_t me = 0;
  hipEvent_t ev_pre = nullptr, ev_post = nullptr;
  ~EmuXport() override {
    for (hipEvent_t e : {ev_pre, ev_post})
      if (e) (void)hipEventDestroy(e);
    if (w) {
      bool last;
      {
        std::lock_guard<std::mutex> l(w->mu);
        last = --w->refs == 0;
      }
      if (last) delete w;
    }
  }
  ncclResult_t a2av(const void* s, const size_t* sc, const size_t* sd, void* r, const size_t* rc, const size_t* rd,
                    hipStream_t st) override {
    const uint32_t G = w->G;
    if (hipEventRecord(ev_pre, st) != hipSuccess) {
      w->abort("rank " + std::to_string(me) + ": hipEventRecord");
      return ncclUnhandledCudaError;
    }
    {
      std::lock_guard<std::mutex> l(w->mu);
      EmuWorld::Post& p = w->post[me];
      p.s = static_cast<const uint8_t*>(s);
      p.r = static_cast<uint8_t*>(r);
      for (uint32_t j = 0; j < G; ++j) p.sc[j] = sc[j], p.sd[j] = sd[j];
      p.ev = ev_pre;
    }
    if (!w->barrier()) return ncclRemoteError;
    hipError_t he = hipSuccess;
    for (uint32_t i = 0; i < G; ++i) {
      const EmuWorld::Post& p = w->post[i];
      if (p.sc[me] != rc[i]) {
        w->abort("rank " + std::to_string(me) + " expects " + std::to_string(rc[i]) + " bytes from rank " +
                 std::to_string(i) + ", which sends " + std::to_string(p.sc[me]));
        return ncclInvalidUsage;
      }
      if (he == hipSuccess) he = hipStreamWaitEvent(st, p.ev, 0);
      if (he == hipSuccess && rc[i])
        he = hipMemcpyAsync(static_cast<uint8_t*>(r) + rd[i], p.s + p.sd[me], rc[i], hipMemcpyDeviceToDevice, st);
    }
    if (he == hipSuccess) he = hipEventRecord(ev_post, st);
    if (he != hipSuccess) {
      w->abort("rank " + std::to_string(me) + ": " + hipGetErrorString(he));
      return ncclUnhandledCudaError;
    }
    {
      std::lock_guard<std::mutex> l(w->mu);
      w->done[me] = ev_post;
    }
    if (!w->barrier()) return ncclRemoteError;
    for (uint32_t i = 0; i < G; ++i)
      if (hipStreamWaitEvent(st, w->done[i], 0) != hipSuccess) {
        w->abort("rank " + std::to_string(me) + ": hipStreamWaitEvent");
        return ncclUnhandledCudaError;
      }
    return ncclSuccess;
  }
  ncclResult_t a2a(const void* s, void* r, size_t n, hipStream_t st) override {
    size_t c[MAXS], d[MAXS];
    for (uint32_t j = 0; j < w->G; ++j) c[j] = n, d[j] = j * n;
    return a2av(s, c, d, r, c, d, st);
  }
  ncclResult_t allgather(const void* s, void* r, size_t n, hipStream_t st) override {
    size_t c[MAXS], z[MAXS], d[MAXS];
    for (uint32_t j = 0; j < w->G; ++j) c[j] = n, z[j] = 0, d[j] = j * n;
    return a2av(s, c, z, r, c, d, st);
  }
  void abort() override { w->abort("rank " + std::to_string(me) + " aborted the communicator"); }
  ncclResult_t async_error() override {
    std::lock_guard<std::mutex> l(w->mu);
    return w->aborted ? ncclRemoteError : ncclSuccess;
  }
  std::string why(ncclResult_t r) override {
    std::lock_guard<std::mutex> l(w->mu);
    return std::string(ncclGetErrorString(r)) + (w->why.empty() ? "" : " (" + w->why + ")");
  }
};

// One owner run: consecutive origins' records (compact by origin) whose times fit one engine batch.
struct Run {
  uint32_t off, n;
};
// Split an owner's records at origin boundaries into runs whose request times span at most one
// second (rl_submit's window rule: a batch may straddle one window boundary of a unit). rcv[i]:
// records from origin i; [tmin[i], tmax[i]]: its batch's times.
void owner_runs(const uint32_t* rcv, const uint32_t* tmin, const uint32_t* tmax, uint32_t G, std::vector<Run>& runs) {
  runs.clear();
  uint32_t off = 0, lo = 0, hi = 0;
  bool open = false;
  Run cur{0, 0};
  for (uint32_t i = 0; i < G; off += rcv[i], ++i) {
    if (!rcv[i]) continue;
    const uint32_t a = std::min(tmin[i], tmax[i]), b = tmax[i];
    if (open && std::max(hi, b) - std::min(lo, a) <= 1u) {
      cur.n += rcv[i];
      lo = std::min(lo, a);
      hi = std::max(hi, b);
      continue;
    }
    if (open) runs.push_back(cur);
    cur = Run{off, rcv[i]};
    lo = a;
    hi = b;
    open = true;
  }
  if (open) runs.push_back(cur);
}

// One hot-set entry as exchanged between ranks (32 B): an owner's hot prefix.
struct AgEntry {
  uint64_t a, b;
  uint32_t unit, rule, count, pad;
};
static_assert(sizeof(AgEntry) == 32, "allgather entry");

// Pinned + device staging of one shard's host batch (RL_ROUTER_HOST), the engine's layout.
struct HostStage {
  uint8_t* h_in = nullptr;
  uint8_t* d_in = nullptr;
  rl_status* d_out = nullptr;
  rl_status* h_out = nullptr;
  uint32_t* d_thr = nullptr;
  uint32_t* h_thr = nullptr;
};

// One shard's part of one step in flight.
struct ShardStep {
  RoutePackBufs pb{};
  uint8_t* zero = nullptr;    // look-back areas + control words: clear before every pack
  size_t zero_bytes = 0;
  bool zeroed = true;         // the unpack cleared them (else the next pack memsets first)
  RRec* recv = nullptr;       // owner: records from every origin
  RawReply* reply = nullptr;  // owner: one raw reply per received record
  RawReply* back = nullptr;   // origin: replies to its records, strided like send
  int32_t* d_x = nullptr;     // step words (XS layout above)
  int32_t* h_x = nullptr;     // pinned mirror; at HX_HOT the hot sums, then the control words
  HostStage hs;
  rl_batch b{};               // the origin batch (device pointers)
  rl_status* out = nullptr;
  uint32_t* thr = nullptr;
  uint32_t cnt[MAXS] = {};    // records this origin sends each owner
  uint32_t rcv[MAXS] = {};    // records this owner receives from each origin
  uint32_t tmin[MAXS] = {}, tmax[MAXS] = {};  // each origin's request-time range
  uint32_t n_in = 0;
  uint32_t n_sub = 0;         // owner batches (runs) handed to the engine and not yet completed
  uint32_t n_runs = 0;        // owner batches of the step
  int rc_pack = 0, rc_dec = 0, rc_local = 0;
  std::string msg;
  const char* phase = "";     // where msg comes from: pack, records, decide, replies, unpack, status
  bool combined = false;
  bool late = false;          // origin batch refused (RL_ELATE): nothing sent, nothing unpacked
};

struct Shard {
  rl_engine* e = nullptr;
  EngineView v{};
  hipStream_t os = nullptr;   // origin work: staging copies, pack, hot scan, unpack
  hipEvent_t ev = nullptr;    // os -> exchange stream
  ShardStep st[NSLOT];
  // route hot set (this shard as origin)
  std::vector<HotKey> hot;
  HotEntry* d_hot = nullptr;
  HotEntry* h_hot = nullptr;
  hipEvent_t ev_hot = nullptr;
  uint32_t last_tot[HOT_MAX] = {};  // sums of hits per group, last step that combined
  bool last_valid = false;
  bool repacked = false;            // since the last refresh
};

struct StepSlot {
  bool busy = false;
  bool host = false;
  bool counts_failed = false;  // every shard left after the counts exchange
  bool replied = false;        // collective: the reply exchange is enqueued
  bool unpacked = false;       // ... and the unpack behind it
  bool end_rec = false;        // ... and ev_end recorded behind them
  hipError_t rep_he = hipSuccess;
  hipEvent_t ev_end = nullptr; // the reply exchange (rs) and the unpack (os) of the step
  hipEvent_t ev_rec = nullptr; // collective: the step's record exchange (its owner batches wait for it)
  bool rec_rec = false;        // ... recorded
  double t0 = 0;
  int32_t status[MAXS] = {};   // per shard (collective: as received from every origin / owner)
  bool late[MAXS] = {};        // per origin: refused for starting too far behind the step clock
};

// A routed step's configuration words, compared across ranks at create (the owners' combining
// and local-cache semantics must agree, rl_hip.h "Router object").
struct CfgWord {
  uint64_t magic, seed;
  uint32_t local_cache, n_shards, max_desc, flags;
};
static_assert(sizeof(CfgWord) == 32, "config word");

}  // namespace

struct rl_router {
  rl_router_config cfg{};
  bool coll = false, broken = false;  // coll: RCCL or emulated collectives (one rank per router)
  std::unique_ptr<Xport> xp;
  hipStream_t rs = nullptr;  // exchanges (collective transports: the origin stream itself)
  bool rs_own = true;        // rs is the router's own stream (local transport)
  hipEvent_t ev_rs = nullptr;
  hipEvent_t ev_cnt = nullptr;  // the counts' host copy
  std::vector<Shard> sh;
  StepSlot slot[NSLOT];
  uint64_t seq = 0, done = 0;
  uint32_t tclock = 0;       // the step clock: the newest request time of every step applied so far
  double t_pack0 = 0;        // start of the current submit's packs (host clock)
  size_t in_bytes = 0, o_off = 0, o_rule = 0, o_req = 0, o_now = 0, o_hits = 0, o_jit = 0;  // host staging layout
  AgEntry* d_ag = nullptr;   // collective hot-set allgather: [HOT_MAX] send | [G * HOT_MAX] receive
  int32_t* d_ok = nullptr;   // [MAXS] zero words: the decide status sent when the decide succeeded
  AgEntry* h_ag = nullptr;
  int fault_phase = PH_NONE;
  uint32_t fault_shard = 0;
  uint64_t fault_step = 0;   // fires in a submit of step >= fault_step (or a wait after it)
  uint32_t* h_stall = nullptr;  // "stall" fault: the stalled kernel's release word (pinned)
  int64_t timeout_ms = 60000;   // bound of every host wait behind a collective (RL_ROUTER_TIMEOUT_MS)
  rl_router_stats st{};
  std::string err;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  // collective failure: abort the communicator (its peers' collectives return), every later call fails
  int nccl_fail(ncclResult_t nr, const char* what) {
    const std::string w = xp ? xp->why(nr) : ncclGetErrorString(nr);
    abort_comm();
    return fail(RL_ECOMM, "%s: %s (communicator aborted)", what, w.c_str());
  }
  void abort_comm() {
    // (a stalled test kernel ends first: ncclCommAbort waits for the work queued behind it)
    if (h_stall) __atomic_store_n(h_stall, 1u, __ATOMIC_RELEASE);
    if (xp) xp->abort();
    broken = true;
  }
  // Collective transports: the host's wait for work queued behind a collective (an event, or the
  // stream when ev is null). A peer that never reaches the collective (a rank that diverged or
  // stopped without its launcher ending the job) would hold that work, and so this rank, forever:
  // the wait polls the communicator's asynchronous error and ends after timeout_ms, and either
  // aborts the communicator (which ends its pending kernels, here and at every peer) and returns
  // RL_ECOMM; every later call of the router fails with it. The reference's analog: a Redis
  // failure becomes a RedisError panic, not a stall (src/redis/driver_impl.go:50-54). Returns 0
  // with *he the wait's own HIP result otherwise.
  int wait_bounded(hipEvent_t ev, hipStream_t q, const char* what, hipError_t* he) {
    const double t_end = now_us() + 1e3 * (double)timeout_ms;
    for (uint64_t k = 0;; ++k) {
      const hipError_t r = ev ? hipEventQuery(ev) : hipStreamQuery(q);
      if (r != hipErrorNotReady) {
        if (he) *he = r;
        return 0;
      }
      if ((k & 255u) != 255u) continue;
      const ncclResult_t ar = xp ? xp->async_error() : ncclSuccess;
      if (ar != ncclSuccess && ar != ncclInProgress) return nccl_fail(ar, what);
      if (now_us() > t_end) {
        abort_comm();
        return fail(RL_ECOMM, "%s: no progress within %lld ms (RL_ROUTER_TIMEOUT_MS): a peer did not reach the "
                              "collective (communicator aborted)", what, (long long)timeout_ms);
      }
      if (k > (1u << 16)) std::this_thread::sleep_for(std::chrono::microseconds(20));  // a long wait: yield the core
    }
  }
  bool fault(int phase, uint32_t s) {
    if (fault_phase != phase || fault_shard != s || (fault_step && seq <= fault_step)) return false;
    fault_phase = PH_NONE;
    return true;
  }
  uint32_t n_local() const { return (uint32_t)sh.size(); }
  uint32_t shard_id(uint32_t s) const { return coll ? cfg.rank : s; }

  int alloc_shard(Shard& s);
  void free_all();
  int validate(const rl_batch& b) const;
  int stage_host(uint32_t s, uint32_t k, const rl_batch& hb, rl_batch& db);
  void pack(uint32_t s, uint32_t k);
  void note_combine(uint32_t s, uint32_t k);
  void refresh_hot();
  int check_config();
  bool step_clock(uint32_t k, const uint32_t* tmin, const uint32_t* tmax, uint32_t* late);
  int submit_owner(uint32_t s, uint32_t k, const Run& u, void* ready);
  void drain(Shard& S, ShardStep& x);
  int submit(const rl_batch* batches, rl_status* const* out, uint32_t* const* thr, bool host);
  int wait(rl_status* const* out, uint32_t* const* thr, bool into);
  int submit_coll(uint32_t k);
  int submit_local(uint32_t k);
  void reply_coll(uint32_t k);
  void unpack_coll(uint32_t k);
  void wait_coll(uint32_t k);
  void wait_local(uint32_t k);
  int step_result(uint32_t k);
};

void rl_router::free_all() {
  for (Shard& s : sh) {
    for (ShardStep& t : s.st) {
      for (void* p : {(void*)t.pb.send, (void*)t.pb.perm, (void*)t.pb.bhs, (void*)t.pb.bstat, (void*)t.zero,
                      (void*)t.pb.hot_pos, (void*)t.recv, (void*)t.reply, (void*)t.back, (void*)t.d_x,
                      (void*)t.hs.d_in, (void*)t.hs.d_out, (void*)t.hs.d_thr})
        if (p) (void)hipFree(p);
      for (void* p : {(void*)t.h_x, (void*)t.hs.h_in, (void*)t.hs.h_out, (void*)t.hs.h_thr})
        if (p) (void)hipHostFree(p);
    }
    if (s.d_hot) (void)hipFree(s.d_hot);
    if (s.h_hot) (void)hipHostFree(s.h_hot);
    if (s.ev_hot) (void)hipEventDestroy(s.ev_hot);
    if (s.ev) (void)hipEventDestroy(s.ev);
    if (s.os) (void)hipStreamDestroy(s.os);
  }
  sh.clear();
  if (d_ag) (void)hipFree(d_ag);
  if (d_ok) (void)hipFree(d_ok);
  if (h_ag) (void)hipHostFree(h_ag);
  xp.reset();
  for (StepSlot& q : slot) {
    for (hipEvent_t e : {q.ev_end, q.ev_rec})
      if (e) (void)hipEventDestroy(e);
    q.ev_end = q.ev_rec = nullptr;
  }
  if (h_stall) (void)hipHostFree(h_stall);
  h_stall = nullptr;
  for (hipEvent_t e : {ev_rs, ev_cnt})
    if (e) (void)hipEventDestroy(e);
  if (rs && rs_own) (void)hipStreamDestroy(rs);
  d_ag = nullptr;
  d_ok = nullptr;
  h_ag = nullptr;
  ev_rs = ev_cnt = nullptr;
  rs = nullptr;
}

int rl_router::alloc_shard(Shard& s) {
  const uint32_t G = cfg.n_shards;
  const size_t D = cfg.max_desc;
  hipError_t he = hipSuccess;
  auto chk = [&](hipError_t x) { if (x != hipSuccess && he == hipSuccess) he = x; };
  chk(hipStreamCreateWithFlags(&s.os, hipStreamNonBlocking));
  chk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  chk(hipEventCreateWithFlags(&s.ev_hot, hipEventDisableTiming));
  chk(hipMalloc(&s.d_hot, sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX)));
  chk(hipHostMalloc(&s.h_hot, sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX), hipHostMallocDefault));
  if (he == hipSuccess) chk(hipEventRecord(s.ev_hot, s.os));
  const size_t lbw = route2_lb_words((uint32_t)D);
  // words after rctl: [16] step words, the hot scan's look-back words, its u64 sums, then (on a
  // 256-B line) the pack's 8 x 64 time-range words
  const size_t tr_off = (16 + route2_hot_lb_words() + 2 * (size_t)HOT_MAX + 63) / 64 * 64;
  for (ShardStep& t : s.st) {
    chk(hipMalloc(&t.pb.send, D * G * REC));
    chk(hipMalloc(&t.pb.perm, D * 4 + 64));
    chk(hipMalloc(&t.pb.bhs, route2_bhs_words((uint32_t)D) * 4 + 64));
    chk(hipMalloc(&t.pb.bstat, (size_t)route2_blocks((uint32_t)D) * 16 + 64));
    chk(hipMalloc(&t.pb.hot_pos, (size_t)HOT_MAX * 8));  // hot_pos | hot_tot
    t.pb.hot_tot = t.pb.hot_pos + HOT_MAX;
    // zeroed per step: two look-back areas, the control words, the hot scan's words, the time words
    t.zero_bytes = (2 * lbw + tr_off + 8 * 64) * 4;
    chk(hipMalloc(&t.zero, t.zero_bytes + 64));
    t.pb.lb = reinterpret_cast<uint32_t*>(t.zero);
    t.pb.rctl = t.pb.lb + 2 * lbw;
    t.pb.tr = t.pb.rctl + tr_off;
    t.pb.xs = XS;
    t.pb.zero_words = (uint32_t)(t.zero_bytes / 4);
    if (he == hipSuccess) chk(hipMemset(t.zero, 0, t.zero_bytes));
    t.zeroed = true;
    chk(hipMalloc(&t.recv, D * G * REC));
    chk(hipMalloc(&t.reply, D * G * RAWB));
    chk(hipMalloc(&t.back, D * G * RAWB));
    chk(hipMalloc(&t.d_x, HX_HOT * 4));
    chk(hipHostMalloc(&t.h_x, (HX_HOT + HOT_MAX + 16) * 4, hipHostMallocDefault));
    t.pb.x = reinterpret_cast<uint32_t*>(t.d_x);
    t.pb.h_hot = reinterpret_cast<uint32_t*>(t.h_x + HX_HOT);
    if (cfg.flags & RL_ROUTER_HOST) {
      chk(hipMalloc(&t.hs.d_in, in_bytes));
      chk(hipHostMalloc(&t.hs.h_in, in_bytes, hipHostMallocDefault));
      chk(hipMalloc(&t.hs.d_out, D * sizeof(rl_status) + 64));
      chk(hipHostMalloc(&t.hs.h_out, D * sizeof(rl_status) + 64, hipHostMallocDefault));
      chk(hipMalloc(&t.hs.d_thr, D * 4 + 64));
      chk(hipHostMalloc(&t.hs.h_thr, D * 4 + 64, hipHostMallocDefault));
    }
  }
  return he == hipSuccess ? 0 : fail(RL_EHIP, "router allocation: %s", hipGetErrorString(he));
}

int rl_router::validate(const rl_batch& b) const {
  if (b.n_desc > cfg.max_desc) return RL_ECAPACITY;
  if (b.reserved || b.n_req > RL_ROUTE_MAX_REQ || (b.n_desc && !b.n_req)) return RL_EINVAL;
  if (b.n_desc && (!b.prefix_blob || !b.prefix_off || !b.rule_id || !b.req_of)) return RL_EINVAL;
  if (b.n_req && (!b.now || !b.hits_addend)) return RL_EINVAL;
  return 0;
}

// Host batch -> the slot's pinned staging (unless the caller built it there) -> device, on the
// shard's origin stream ahead of its pack.
int rl_router::stage_host(uint32_t s, uint32_t k, const rl_batch& b, rl_batch& d) {
  ShardStep& t = sh[s].st[k];
  uint8_t* h = t.hs.h_in;
  if ((size_t)b.blob_bytes + RL_BLOB_SLACK > o_off || b.n_desc > cfg.max_desc || b.n_req > cfg.max_desc)
    return RL_ECAPACITY;
  struct Arr { const void* src; size_t o, n; } arrs[] = {
      {b.prefix_blob, 0, b.blob_bytes}, {b.prefix_off, o_off, b.n_desc ? ((size_t)b.n_desc + 1) * 4 : 0},
      {b.rule_id, o_rule, (size_t)b.n_desc * 4}, {b.req_of, o_req, (size_t)b.n_desc * 4},
      {b.now, o_now, (size_t)b.n_req * 8}, {b.hits_addend, o_hits, (size_t)b.n_req * 4},
      {b.ttl_jitter, o_jit, b.ttl_jitter ? (size_t)b.n_desc * 2 : 0}};
  for (auto& a : arrs)
    if (a.n && a.src != h + a.o) memcpy(h + a.o, a.src, a.n);
  memset(h + b.blob_bytes, 0, RL_BLOB_SLACK);  // the device reads prefixes in 16-B words
  const size_t ext[] = {(size_t)b.blob_bytes + RL_BLOB_SLACK, arrs[1].n, arrs[2].n, arrs[3].n, arrs[4].n, arrs[5].n,
                        arrs[6].n};
  hipError_t he = hipSuccess;
  for (int q = 0; q < 7 && he == hipSuccess; ++q)
    if (ext[q]) he = hipMemcpyAsync(t.hs.d_in + arrs[q].o, h + arrs[q].o, ext[q], hipMemcpyHostToDevice, sh[s].os);
  if (he != hipSuccess) return RL_EHIP;
  d = b;
  d.prefix_blob = t.hs.d_in;
  d.prefix_off = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_off);
  d.rule_id = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_rule);
  d.req_of = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_req);
  d.now = reinterpret_cast<const int64_t*>(t.hs.d_in + o_now);
  d.hits_addend = reinterpret_cast<const uint32_t*>(t.hs.d_in + o_hits);
  d.ttl_jitter = b.ttl_jitter ? reinterpret_cast<const uint16_t*>(t.hs.d_in + o_jit) : nullptr;
  return 0;
}

// Origin pack of shard s for slot k on its origin stream: the (count, status, tmin, tmax) words
// land in d_x[0, XS G) and, with combining, the groups' sums and the control words in the
// pinned mirror.
void rl_router::pack(uint32_t s, uint32_t k) {
  Shard& S = sh[s];
  ShardStep& t = S.st[k];
  const uint32_t G = cfg.n_shards;
  t.combined = false;
  auto send_status = [&](int32_t rc) {  // (0, rc, no times) to every owner; the decide statuses' failure words
    for (uint32_t j = 0; j < G; ++j) {
      t.h_x[XS * j] = 0;
      t.h_x[XS * j + 1] = rc;
      t.h_x[XS * j + 2] = (int32_t)0xFFFFFFFFu;
      t.h_x[XS * j + 3] = 0;
      t.h_x[2 * XS * G + j] = RL_EHIP;
    }
    (void)hipMemcpyAsync(t.d_x, t.h_x, 4 * XS * G, hipMemcpyHostToDevice, S.os);
    (void)hipMemcpyAsync(t.d_x + 2 * XS * G, t.h_x + 2 * XS * G, 4 * G, hipMemcpyHostToDevice, S.os);
  };
  if (t.rc_pack || !t.b.n_desc) {
    if (!t.rc_pack && t.b.n_req && t.thr) (void)hipMemsetAsync(t.thr, 0, (size_t)t.b.n_req * 4, S.os);
    send_status(t.rc_pack);
    return;
  }
  // (no combining with EXPIRE jitter: a combined record's EXPIRE would need the group's last
  // descriptor's jitter)
  const bool combine = !(cfg.flags & RL_ROUTER_NO_COMBINE) && !S.v.local_cache && !S.hot.empty() && !t.b.ttl_jitter;
  if (!t.zeroed) (void)hipMemsetAsync(t.zero, 0, t.zero_bytes, S.os);  // (the slot's last step had no unpack)
  t.pb.thr = t.thr;  // zeroed by the pack
  // the hot scan writes the group sums and its verdict straight into the pinned mirror
  launch_route_pack2(S.os, t.b, S.v.rules, S.v.n_rules, S.v.seed, shard_id(s), G, cfg.max_desc,
                     combine ? S.d_hot : nullptr, t.pb);
  t.zeroed = false;
  t.combined = combine;
  const hipError_t he = hipGetLastError();
  if (he != hipSuccess || fault(PH_PACK, s)) {  // the pack cannot be trusted: fail the step everywhere
    t.rc_pack = RL_EHIP;
    t.msg = he != hipSuccess ? std::string("route pack: ") + hipGetErrorString(he) : "injected fault (pack)";
    t.phase = "pack";
    t.combined = false;
    send_status(RL_EHIP);
  }
}

// After the counts: did shard s's pack combine (its groups' sums keep the route hot set), or
// did its batch need the repack (a hot group was not one key string)?
void rl_router::note_combine(uint32_t s, uint32_t k) {
  ShardStep& t = sh[s].st[k];
  if (!t.combined) return;
  const uint32_t* ctl = reinterpret_cast<const uint32_t*>(t.h_x + HX_HOT + HOT_MAX);  // k_route_hot_scan
  if (ctl[0] || !ctl[1]) {
    if (s == 0) ++st.repacks;
    sh[s].repacked = true;
    t.combined = false;
  } else {
    memcpy(sh[s].last_tot, t.h_x + HX_HOT, sizeof sh[s].last_tot);
    sh[s].last_valid = true;
    if (s == 0) ++st.combined_steps;
  }
}

// Route hot set refresh (every ROUTE_HOT_EVERY steps, at the same step on every shard): keep the
// groups this origin still sends with >= ROUTE_HOT_KEEP hits per step, add the owners' hot keys
// (each engine's own hot set: prefixes that reach it with many records per batch; over the
// collective transport gathered from every rank), up to HOT_MAX. A shard that had to repack
// starts over.
void rl_router::refresh_hot() {
  std::vector<HotKey> cand;
  if (coll) {
    std::vector<HotKey> mine;
    rlx_engine_hot(sh[0].e, mine);
    for (uint32_t i = 0; i < HOT_MAX; ++i) {
      AgEntry& a = h_ag[i];
      memset(&a, 0, sizeof a);
      if (i < mine.size()) a = AgEntry{mine[i].a, mine[i].b, mine[i].unit, mine[i].rule, std::max(1u, mine[i].count), 0};
    }
    const size_t n = HOT_MAX * sizeof(AgEntry);
    hipError_t he = hipMemcpyAsync(d_ag, h_ag, n, hipMemcpyHostToDevice, rs);
    const ncclResult_t nr = xp->allgather(d_ag, d_ag + HOT_MAX, n, rs);
    if (nr != ncclSuccess) {
      nccl_fail(nr, "allgather(hot sets)");
      return;
    }
    if (he == hipSuccess) he = hipMemcpyAsync(h_ag + HOT_MAX, d_ag + HOT_MAX, n * cfg.n_shards, hipMemcpyDeviceToHost, rs);
    if (he == hipSuccess && wait_bounded(nullptr, rs, "allgather(hot sets)", &he)) return;
    if (he != hipSuccess) return;  // keep the current sets (decisions do not depend on them)
    for (uint32_t i = 0; i < HOT_MAX * cfg.n_shards; ++i) {
      const AgEntry& a = h_ag[HOT_MAX + i];
      if (a.count) cand.push_back(HotKey{a.a, a.b, a.unit, a.rule, a.count});
    }
  } else {
    for (Shard& s : sh) {
      std::vector<HotKey> h;
      rlx_engine_hot(s.e, h);
      cand.insert(cand.end(), h.begin(), h.end());
    }
  }
  std::stable_sort(cand.begin(), cand.end(), [](const HotKey& x, const HotKey& y) { return x.count > y.count; });
  for (Shard& s : sh) {
    std::vector<HotKey> next;
    std::unordered_set<uint64_t> seen;
    if (!s.repacked && s.last_valid)
      for (size_t i = 0; i < s.hot.size(); ++i)
        if (s.last_tot[i] >= ROUTE_HOT_KEEP) {
          HotKey k = s.hot[i];
          k.count = s.last_tot[i];
          seen.insert(k.a);
          next.push_back(k);
        }
    for (const HotKey& c : cand) {
      if (next.size() >= (size_t)HOT_MAX) break;
      if (!seen.insert(c.a).second) continue;  // (a prefix seen with a second rule: the pack repacks)
      next.push_back(c);
    }
    s.repacked = false;
    bool same = next.size() == s.hot.size();
    for (size_t i = 0; same && i < next.size(); ++i)
      same = next[i].a == s.hot[i].a && next[i].b == s.hot[i].b && next[i].rule == s.hot[i].rule;
    if (same) continue;
    std::vector<HotEntry> t;
    build_hot_table(next, t);
    // the staging's previous copy is done; the next pack is ordered behind this copy on os
    // (collective transports: os carries the exchanges, so the wait is bounded)
    hipError_t hw = hipSuccess;
    if (coll) {
      if (wait_bounded(s.ev_hot, nullptr, "hot set staging", &hw)) return;
    } else {
      hw = hipEventSynchronize(s.ev_hot);
    }
    if (hw != hipSuccess) continue;
    memcpy(s.h_hot, t.data(), sizeof(HotEntry) * t.size());
    if (hipMemcpyAsync(s.d_hot, s.h_hot, sizeof(HotEntry) * t.size(), hipMemcpyHostToDevice, s.os) != hipSuccess)
      continue;
    (void)hipEventRecord(s.ev_hot, s.os);
    s.hot = std::move(next);
    s.last_valid = false;
  }
}

// At create: every rank's configuration words (collective transports) or every engine's (local)
// must agree — one hash seed (owners), one local-cache setting (combining is exact only when no
// owner freezes a key inside a combined group). A mismatch fails create on every rank alike.
int rl_router::check_config() {
  auto word = [&](const EngineView& v) {
    return CfgWord{0x52544346474f5752ull, v.seed, (uint32_t)v.local_cache, cfg.n_shards, cfg.max_desc,
                   cfg.flags & (RL_ROUTER_NO_COMBINE | RL_ROUTER_HOST)};
  };
  std::vector<CfgWord> all;
  if (coll) {
    CfgWord* hw = reinterpret_cast<CfgWord*>(h_ag);
    CfgWord* dw = reinterpret_cast<CfgWord*>(d_ag);
    hw[0] = word(sh[0].v);
    hipError_t he = hipMemcpyAsync(dw, hw, sizeof(CfgWord), hipMemcpyHostToDevice, rs);
    const ncclResult_t nr = xp->allgather(dw, dw + 1, sizeof(CfgWord), rs);
    if (nr != ncclSuccess) return nccl_fail(nr, "allgather(router configuration)");
    if (he == hipSuccess)
      he = hipMemcpyAsync(hw + 1, dw + 1, sizeof(CfgWord) * cfg.n_shards, hipMemcpyDeviceToHost, rs);
    if (he == hipSuccess)
      if (int rc = wait_bounded(nullptr, rs, "allgather(router configuration)", &he)) return rc;
    if (he != hipSuccess) return fail(RL_EHIP, "router configuration exchange: %s", hipGetErrorString(he));
    all.assign(hw + 1, hw + 1 + cfg.n_shards);
  } else {
    for (Shard& s : sh) all.push_back(word(s.v));
  }
  for (uint32_t j = 1; j < all.size(); ++j)
    if (memcmp(&all[j], &all[0], sizeof(CfgWord)) != 0)
      return fail(RL_EINVAL, "shard %u's configuration differs from shard 0's (hash_seed, local_cache, n_shards, "
                             "max_desc and flags must agree on every shard)", j);
  return 0;
}

// The step clock after the counts: origin i's batch may start at most MAX_LAG_S seconds behind
// the newest request time of everything before it in rank order (earlier steps included) — the
// table keeps a SECOND key string findable that far back. Every rank computes the same verdict
// from the same exchanged ranges; late[i] = 1 for an origin behind it. A late origin is left out
// of the step (its records are neither sent nor decided) and does not move the clock; the rest of
// the step goes ahead, so one slow host fails only its own callers (a Redis cluster would decide
// its late INCRBYs on their own; this table cannot place them exactly any more).
bool rl_router::step_clock(uint32_t k, const uint32_t* tmin, const uint32_t* tmax, uint32_t* late) {
  uint32_t c = tclock;
  bool any = false;
  for (uint32_t i = 0; i < cfg.n_shards; ++i) {
    late[i] = 0;
    slot[k].late[i] = false;
    if (tmin[i] > tmax[i]) continue;  // no routed descriptors
    if (c > tmin[i] + MAX_LAG_S) {
      late[i] = 1;
      slot[k].late[i] = true;
      any = true;
      continue;
    }
    c = std::max(c, tmax[i]);
  }
  tclock = c;
  return any;
}

// Complete the oldest owner batch of the engine: x's (the older step's first, FIFO).
void rl_router::drain(Shard& S, ShardStep& x) {
  if (coll && !broken) {
    // the step's owner batches run behind its record exchange: a bounded wait for that first
    // (on expiry the communicator is aborted, which ends the exchange, and the engine drains)
    const StepSlot& q = slot[&x - S.st];
    if (q.rec_rec) (void)wait_bounded(q.ev_rec, nullptr, "all-to-all-v(records)", nullptr);
  }
  const int rp = rl_wait(S.e);
  if (rp && !x.rc_dec) {
    x.rc_dec = rp;
    x.msg = rl_last_error(S.e);
    x.phase = "decide";
  }
  --x.n_sub;
}

// One owner run to the engine; an engine that cannot take another batch now (in flight at its
// limit, or an LSD engine that cannot pipeline) completes its oldest ones first.
int rl_router::submit_owner(uint32_t s, uint32_t k, const Run& u, void* ready) {
  Shard& S = sh[s];
  ShardStep& t = S.st[k];
  for (;;) {
    const int rc = rl_submit_routed_async(S.e, t.recv + u.off, u.n, t.reply + u.off, RL_ROUTED_RAW, ready);
    if (rc != RL_ESTATE) {
      if (!rc) ++t.n_sub;
      return rc;
    }
    ShardStep* old = nullptr;  // the oldest step in flight (this one included) with owner batches
    for (uint64_t q = done; q < seq && !old; ++q)
      if (S.st[q % NSLOT].n_sub) old = &S.st[q % NSLOT];
    if (!old) return rc;
    drain(S, *old);
  }
}

// Collective transport: counts (+ pack statuses and time ranges), then records; the owner's runs
// are handed to the engine.
int rl_router::submit_coll(uint32_t k) {
  const uint32_t G = cfg.n_shards, me = cfg.rank;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  const double t0 = t_pack0;
  hipError_t he = hipSuccess;
  if (rs != S.os) {
    he = hipEventRecord(S.ev, S.os);
    if (he == hipSuccess) he = hipStreamWaitEvent(rs, S.ev, 0);
  }
  // (the decide statuses this rank sends in the reply exchange start as a failure word, written
  // by the pack or with the host's status words: only a successful upload of its real status
  // replaces it (reply_coll), so a failed upload cannot hand peers a stale status of an earlier step)
  if (fault(PH_COMM, 0)) return nccl_fail(ncclInternalError, "all-to-all(counts): injected fault (comm)");
  if (h_stall && fault(PH_STALL, 0)) launch_router_stall(rs, h_stall);
  ncclResult_t nr = xp->a2a(t.d_x, t.d_x + XS * G, 4 * XS, rs);
  if (nr != ncclSuccess) return nccl_fail(nr, "all-to-all(counts)");
  if (he == hipSuccess) he = hipMemcpyAsync(t.h_x, t.d_x, 8 * XS * G, hipMemcpyDeviceToHost, rs);
  if (he == hipSuccess) he = hipEventRecord(ev_cnt, rs);
  if (he == hipSuccess)
    if (int rc = wait_bounded(ev_cnt, nullptr, "all-to-all(counts)", &he)) return rc;
  if (he != hipSuccess) {  // the counts are unknown: nobody can take part in the record exchange
    abort_comm();
    return fail(RL_ECOMM, "counts exchange: %s (communicator aborted)", hipGetErrorString(he));
  }
  const int32_t* hs = t.h_x;
  const int32_t* hr = t.h_x + XS * G;
  if (!t.rc_pack && hs[1]) {  // the device refused the pack (one status in every owner's words)
    t.rc_pack = hs[1];
    t.msg = t.rc_pack == RL_EDEVICE ? "route pack: the device's look-back spin limit expired (device fault)"
                                    : "route pack: batch references an unknown rule id or request index, malformed "
                                      "prefix offsets, or a time outside [0, 0xFFFD0000]";
    t.phase = "pack";
  }
  st.pack_us = now_us() - t0;
  bool any = false;
  for (uint32_t j = 0; j < G; ++j) {
    t.cnt[j] = t.rc_pack ? 0u : (uint32_t)hs[XS * j];
    t.rcv[j] = (uint32_t)hr[XS * j];
    t.tmin[j] = (uint32_t)hr[XS * j + 2];
    t.tmax[j] = (uint32_t)hr[XS * j + 3];
    slot[k].status[j] = hr[XS * j + 1];
    any |= hr[XS * j + 1] != 0;
  }
  if (!any) {  // every rank sees the same ranges: the same verdict everywhere
    uint32_t late[MAXS];
    if (step_clock(k, t.tmin, t.tmax, late)) {
      for (uint32_t j = 0; j < G; ++j)
        if (late[j]) t.rcv[j] = 0;  // (every rank drops the same origins: the exchanges still pair up)
      if (late[me]) {
        for (uint32_t j = 0; j < G; ++j) t.cnt[j] = 0;
        t.late = true;
        ++st.late_steps;
        t.msg = "the batch's request times start more than 3 s behind the step clock (the newest time of the "
                "origins before it); the table cannot keep SECOND keys that long";
        t.phase = "pack";
      }
    }
  }
  if (any) {  // every rank saw the same status words: all leave after this exchange
    slot[k].counts_failed = true;
    return 0;
  }
  note_combine(0, k);
  // The reply exchanges of the steps before this one go first: their decides were handed to the
  // engine one submit earlier (behind this rank's pack, so done or nearly), the caller's wait for
  // them then returns while this step's records and decide are on their way, and its next pack
  // runs beside this decide. (Every rank submits and waits in the same order, so every rank
  // issues these collectives in the same order.)
  // Their unpacks follow this step's records on the origin stream, so the decide of this step
  // starts as early as it can.
  // The older steps' replies and this step's records form ONE collective group: one launch, and
  // no host gap between the two exchanges on the origin stream (RL_ROUTER_SPLIT_GROUPS: two).
#ifdef RL_ROUTER_SPLIT_GROUPS
  constexpr bool fused = false;
#else
  constexpr bool fused = true;
#endif
  if (fused) {
    const ncclResult_t gr = xp->group_start();
    if (gr != ncclSuccess) return nccl_fail(gr, "group(replies, records)");
  }
  for (uint64_t q = done; q + 1 < seq; ++q) {
    const uint32_t kq = (uint32_t)(q % NSLOT);
    if (slot[kq].busy && !slot[kq].counts_failed && !slot[kq].replied) {
      reply_coll(kq);
      if (broken) {
        if (fused) (void)xp->group_end();
        return RL_ECOMM;
      }
#ifdef RL_ROUTER_UNPACK_FIRST
      unpack_coll(kq);
#endif
    }
  }
  // records: to owner j this origin's section j (stride D); from origin j its count, compact
  const size_t D = cfg.max_desc;
  size_t sc[MAXS], sd[MAXS], rc[MAXS], rd[MAXS];
  uint64_t ro = 0;
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)t.cnt[j] * REC;
    sd[j] = j * D * REC;
    rc[j] = (size_t)t.rcv[j] * REC;
    rd[j] = ro;
    ro += rc[j];
    st.sent[j] = t.cnt[j];
  }
  t.n_in = (uint32_t)(ro / REC);
  for (uint32_t j = 0; j < G; ++j) st.recv[j] = j == me ? t.n_in : 0;
  nr = xp->a2av(t.pb.send, sc, sd, t.recv, rc, rd, rs);
  if (fused) {
    const ncclResult_t ge = xp->group_end();  // (ends the group on a failed a2av too)
    if (nr == ncclSuccess) nr = ge;
  }
  if (nr != ncclSuccess) return nccl_fail(nr, "all-to-all-v(records)");
  const double t1 = now_us();
  he = hipEventRecord(slot[k].ev_rec, rs);
  slot[k].rec_rec = he == hipSuccess;
#ifndef RL_ROUTER_OWNER_FIRST
  // The older steps' unpacks go out before this step's owner batch: they follow the records on
  // the origin stream, which carries the step's critical chain (pack, exchanges, unpack), while
  // the owner's kernels wait for the records on the engine's streams anyway; launching the owner
  // batch first held the unpack back by its launch calls (~10 us of host time).
  for (uint64_t q = done; q + 1 < seq; ++q) {
    const uint32_t kq = (uint32_t)(q % NSLOT);
    if (slot[kq].replied && !slot[kq].unpacked) unpack_coll(kq);
  }
#endif
  if (fault(PH_RECORDS, 0)) he = hipErrorUnknown;
  if (he != hipSuccess) {  // keep going: the failure travels in the reply exchange
    t.rc_local = RL_EHIP;
    t.msg = std::string("record exchange: ") + (he == hipErrorUnknown ? "injected fault (records)" : hipGetErrorString(he));
    t.phase = "records";
  } else if (t.n_in) {
    std::vector<Run> runs;
    owner_runs(t.rcv, t.tmin, t.tmax, G, runs);
    t.n_runs = (uint32_t)runs.size();
    for (const Run& u : runs) {
      const int rc2 = submit_owner(0, k, u, slot[k].ev_rec);
      if (rc2) {
        if (!t.rc_dec) {
          t.rc_dec = rc2;
          t.msg = rl_last_error(S.e);
          t.phase = "decide";
        }
        break;  // (runs after a refused one are not applied, like the rest of a refused batch)
      }
    }
  }
#ifdef RL_ROUTER_OWNER_FIRST
  for (uint64_t q = done; q + 1 < seq; ++q) {
    const uint32_t kq = (uint32_t)(q % NSLOT);
    if (slot[kq].replied && !slot[kq].unpacked) unpack_coll(kq);
  }
#endif
  st.exchange_us = now_us() - t1;
  return 0;
}

// Local transport: every shard's counts on the host, records by device copies; the owners
// decide one after another, each timed alone (each models one GPU: decide_max_us is the step's
// critical path on G real GPUs).
int rl_router::submit_local(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  const double t0 = t_pack0;
  uint32_t tmin[MAXS], tmax[MAXS];
  for (uint32_t s = 0; s < G; ++s) {
    ShardStep& t = sh[s].st[k];
    hipError_t he = hipMemcpyAsync(t.h_x, t.d_x, 4 * XS * G, hipMemcpyDeviceToHost, sh[s].os);
    if (he == hipSuccess) he = hipStreamSynchronize(sh[s].os);
    if (he != hipSuccess && !t.rc_pack) {
      t.rc_pack = RL_EHIP;
      t.msg = std::string("counts: ") + hipGetErrorString(he);
      t.phase = "pack";
    }
    if (!t.rc_pack && t.h_x[1]) {
      t.rc_pack = t.h_x[1];
      t.msg = t.rc_pack == RL_EDEVICE ? "route pack: the device's look-back spin limit expired (device fault)"
                                      : "route pack: batch references an unknown rule id or request index, malformed "
                                        "prefix offsets, or a time outside [0, 0xFFFD0000]";
      t.phase = "pack";
    }
    slot[k].status[s] = t.rc_pack;
    tmin[s] = t.rc_pack ? 0xFFFFFFFFu : (uint32_t)t.h_x[2];
    tmax[s] = t.rc_pack ? 0u : (uint32_t)t.h_x[3];
  }
  st.pack_us = now_us() - t0;
  bool any = false;
  for (uint32_t s = 0; s < G; ++s) any |= sh[s].st[k].rc_pack != 0;
  if (any) {
    slot[k].counts_failed = true;
    return 0;
  }
  uint32_t late[MAXS];
  if (step_clock(k, tmin, tmax, late)) {
    ++st.late_steps;
    for (uint32_t s = 0; s < G; ++s)
      if (late[s]) {
        ShardStep& t = sh[s].st[k];
        t.late = true;
        t.msg = "the batch's request times start more than 3 s behind the step clock (the newest time of the "
                "origins before it); the table cannot keep SECOND keys that long";
        t.phase = "pack";
      }
  }
  for (uint32_t s = 0; s < G; ++s) {
    ShardStep& t = sh[s].st[k];
    for (uint32_t j = 0; j < G; ++j) t.cnt[j] = t.late ? 0u : (uint32_t)t.h_x[XS * j];
    note_combine(s, k);
  }
  for (uint32_t j = 0; j < G; ++j) st.sent[j] = sh[0].st[k].cnt[j];
  const size_t D = cfg.max_desc;
  hipError_t he = hipSuccess;
  for (uint32_t j = 0; j < G; ++j) {  // owner j: origin 0's section j, then origin 1's, ...
    uint64_t o = 0;
    for (uint32_t i = 0; i < G; ++i) {
      const uint32_t c = sh[i].st[k].cnt[j];
      ShardStep& tj = sh[j].st[k];
      tj.rcv[i] = c;
      tj.tmin[i] = tmin[i];
      tj.tmax[i] = tmax[i];
      if (c && he == hipSuccess)
        he = hipMemcpyAsync(tj.recv + o, sh[i].st[k].pb.send + j * D, (size_t)c * REC, hipMemcpyDeviceToDevice, rs);
      o += c;
    }
    sh[j].st[k].n_in = (uint32_t)o;
    st.recv[j] = (uint32_t)o;
  }
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  const double t1 = now_us();
  st.exchange_us = t1 - t0 - st.pack_us;
  st.decide_max_us = 0;
  std::vector<Run> runs;
  for (uint32_t j = 0; j < G; ++j) {
    ShardStep& t = sh[j].st[k];
    if (he != hipSuccess || fault(PH_RECORDS, j)) {
      t.rc_local = RL_EHIP;
      t.msg = he != hipSuccess ? std::string("record exchange: ") + hipGetErrorString(he) : "injected fault (records)";
      t.phase = "records";
      continue;
    }
    const double a = now_us();
    if (t.n_in) {
      owner_runs(t.rcv, t.tmin, t.tmax, G, runs);
      t.n_runs = (uint32_t)runs.size();
      for (const Run& u : runs) {
        int rc = rl_submit_routed_async(sh[j].e, t.recv + u.off, u.n, t.reply + u.off, RL_ROUTED_RAW, nullptr);
        if (!rc) rc = rl_wait(sh[j].e);
        if (rc) {
          t.rc_dec = rc;
          t.msg = rl_last_error(sh[j].e);
          t.phase = "decide";
          break;
        }
      }
    }
    st.decide_max_us = std::max(st.decide_max_us, now_us() - a);
  }
  st.decide_us = now_us() - t1;
  return 0;
}

int rl_router::submit(const rl_batch* batches, rl_status* const* out, uint32_t* const* thr, bool host) {
  if (broken) return fail(RL_ECOMM, "the router's communicator was aborted after a transport failure");
  const uint32_t k = (uint32_t)(seq % NSLOT);
  if (slot[k].busy) return fail(RL_ESTATE, "%d routed steps in flight: call rl_router_wait", NSLOT);
  if (host && !(cfg.flags & RL_ROUTER_HOST)) return fail(RL_EINVAL, "router created without RL_ROUTER_HOST");
  const uint32_t G = cfg.n_shards, nl = n_local();
  if (!coll)  // the local transport refuses a bad batch before anything moves (collective: in the counts exchange)
    for (uint32_t s = 0; s < G; ++s)
      if (batches[s].n_desc > cfg.max_desc)
        return fail(RL_ECAPACITY, "shard %u: batch of %u descriptors exceeds the router's max_desc %u", s,
                    batches[s].n_desc, cfg.max_desc);
  for (uint32_t j = 0; j < MAXS; ++j) st.recv[j] = 0, st.sent[j] = 0, slot[k].status[j] = 0, slot[k].late[j] = false;
  slot[k].t0 = now_us();
  t_pack0 = slot[k].t0;
  slot[k].host = host;
  slot[k].counts_failed = false;
  slot[k].replied = slot[k].unpacked = slot[k].end_rec = false;
  if (seq % ROUTE_HOT_EVERY == 0) {
    refresh_hot();
    if (broken) return RL_ECOMM;
  }
  for (uint32_t s = 0; s < nl; ++s) {
    Shard& S = sh[s];
    ShardStep& t = S.st[k];
    t.rc_pack = t.rc_dec = t.rc_local = 0;
    t.late = false;
    t.msg.clear();
    t.phase = "";
    t.n_sub = t.n_runs = 0;
    t.n_in = 0;
    t.rc_pack = validate(batches[s]);
    if (t.rc_pack) {
      t.msg = "bad origin batch (capacity, reserved, request count or null arrays)";
      t.phase = "pack";
    }
    if (host) {
      t.out = t.hs.d_out;
      t.thr = t.hs.d_thr;
      if (!t.rc_pack) {
        t.rc_pack = stage_host(s, k, batches[s], t.b);
        if (t.rc_pack) {
          t.msg = "host staging (capacity)";
          t.phase = "pack";
        }
      }
      if (t.rc_pack) t.b = rl_batch{};
    } else {
      t.b = batches[s];
      t.out = out[s];
      t.thr = thr[s];
      if (t.rc_pack) t.b = rl_batch{};
    }
    const int rc = rlx_engine_view(S.e, &S.v);  // (rules may have been appended since)
    if (rc && !t.rc_pack) {
      t.rc_pack = rc;
      t.msg = rl_last_error(S.e);
      t.phase = "pack";
    }
    pack(s, k);
    // local transport (logical shards on one device): one origin's pack at a time, so
    // pack_us / G is one origin's pack (as on G GPUs)
    if (!coll) (void)hipStreamSynchronize(S.os);
  }
  slot[k].busy = true;
  ++seq;
  return coll ? submit_coll(k) : submit_local(k);
}

// The step's outcome from each shard's status: the first failing shard's code on that shard
// (local transport: returned), RL_EPEER on the others.
int rl_router::step_result(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  for (uint32_t j = 0; j < MAXS; ++j) st.status[j] = j < G ? slot[k].status[j] : 0;
  int bad = -1;
  for (uint32_t j = 0; j < G && bad < 0; ++j)
    if (st.status[j]) bad = (int)j;
  if (bad < 0) {  // every owner decided: only late origins fail, each alone
    int late = -1;
    for (uint32_t j = 0; j < G; ++j)
      if (slot[k].late[j]) {
        st.status[j] = RL_ELATE;
        if (late < 0 && (!coll || j == cfg.rank)) late = (int)j;
      }
    if (late < 0) return 0;
    const ShardStep& t = sh[coll ? 0 : late].st[k];
    return fail(RL_ELATE, "shard %d (%s): %s", late, t.phase, t.msg.c_str());
  }
  const int code = st.status[bad];
  for (uint32_t j = 0; j < G; ++j)
    if (st.status[j] == 0) st.status[j] = RL_EPEER;
  if (coll && (uint32_t)bad != cfg.rank) {
    const int32_t own = st.status[cfg.rank];
    const ShardStep& t = sh[0].st[k];
    if (own != RL_EPEER) return fail(own, "shard %u (%s): %s", cfg.rank, t.phase, t.msg.c_str());
    return fail(RL_EPEER, "shard %d failed this step with %d (see rl_router_stats.status)", bad, code);
  }
  const ShardStep& t = sh[coll ? 0 : bad].st[k];
  return fail(code, "shard %d (%s): %s", bad, t.phase, t.msg.c_str());
}

// The owner's decide of step k completed, its status and replies exchanged.
void rl_router::reply_coll(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  slot[k].replied = true;
  const double t0 = now_us();
  while (t.n_sub) drain(S, t);
  if (broken) return;  // a record exchange that never completed (drain's bounded wait aborted)
  if (!t.rc_dec && !t.rc_local && fault(PH_DECIDE, 0)) {
    t.rc_dec = RL_EHIP;
    t.msg = "injected fault (decide)";
    t.phase = "decide";
  }
  st.decide_us = st.decide_max_us = now_us() - t0;
  const double t1 = now_us();
  int32_t* hs = t.h_x + 2 * XS * G;  // statuses sent | received
  int32_t mine = t.rc_dec ? t.rc_dec : t.rc_local;
  if (!mine && fault(PH_REPLIES, 0)) {
    mine = t.rc_local = RL_EHIP;
    t.msg = "injected fault (replies)";
    t.phase = "replies";
  }
  for (uint32_t j = 0; j < G; ++j) hs[j] = mine;
  // this rank's status words: a success sends the constant zero words (no upload on the step's
  // chain); a failure is uploaded over the failure words the pack wrote, and a failed upload
  // leaves those (so it never hands peers a stale status of an earlier step)
  const int32_t* sw = t.d_x + 2 * XS * G;
  hipError_t hu = hipSuccess;
  if (fault(PH_STATUS, 0)) hu = hipErrorUnknown;
  else if (mine) hu = hipMemcpyAsync(t.d_x + 2 * XS * G, hs, 4 * G, hipMemcpyHostToDevice, rs);
  else sw = d_ok;
  if (hu != hipSuccess) {
    if (!t.rc_dec && !t.rc_local) {
      t.rc_local = RL_EHIP;
      t.msg = std::string("decide status upload: ") +
              (hu == hipErrorUnknown ? "injected fault (status)" : hipGetErrorString(hu));
      t.phase = "status";
    }
  }
  // replies: to origin j the replies to its records (compact), into its back buffer at my section
  const size_t D = cfg.max_desc;
  size_t sc[MAXS], sd[MAXS], rc[MAXS], rd[MAXS];
  uint64_t so = 0;
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)t.rcv[j] * RAWB;
    sd[j] = so;
    so += sc[j];
    rc[j] = (size_t)t.cnt[j] * RAWB;
    rd[j] = j * D * RAWB;  // perm = owner * D + position
  }
  ncclResult_t nr = xp->group_start();
  if (nr == ncclSuccess) nr = xp->a2a(sw, t.d_x + 2 * XS * G + G, 4, rs);
  if (nr == ncclSuccess) nr = xp->a2av(t.reply, sc, sd, t.back, rc, rd, rs);
  const ncclResult_t ne = xp->group_end();
  if (nr != ncclSuccess || ne != ncclSuccess) {
    nccl_fail(nr != ncclSuccess ? nr : ne, "all-to-all(replies)");
    return;
  }
  hipError_t he = hipSuccess;
  if (rs != S.os) he = hipEventRecord(ev_rs, rs);
  if (he == hipSuccess && rs != S.os) he = hipStreamWaitEvent(S.os, ev_rs, 0);
  slot[k].rep_he = he;
  st.reply_us = now_us() - t1;
}

// The origin's unpack of step k (and the host copies) behind its reply exchange; slot[k].ev_end
// marks their end.
void rl_router::unpack_coll(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  slot[k].unpacked = true;
  hipError_t he = slot[k].rep_he;
  const double t2 = now_us();
  // (the owners' statuses arrived with the replies; thr zeroed by the pack); the unpack copies
  // the statuses into the pinned step words, else a copy does
  int32_t* hst = t.h_x + 2 * XS * G + G;
  bool copied = false;
  if (he == hipSuccess && t.b.n_desc && !t.late) {
    launch_route_unpack_raw(S.os, t.b, S.v.rules, t.pb, t.back, t.d_x + 2 * XS * G + G, cfg.max_desc, t.out, t.thr,
                            hst, G);
    he = hipGetLastError();
    t.zeroed = copied = he == hipSuccess;
  }
  if (!copied) {
    const hipError_t hc = hipMemcpyAsync(hst, t.d_x + 2 * XS * G + G, 4 * G, hipMemcpyDeviceToHost, S.os);
    if (he == hipSuccess) he = hc;
  }
  if (he == hipSuccess && slot[k].host && !t.late) {
    if (t.b.n_desc)
      he = hipMemcpyAsync(t.hs.h_out, t.out, (size_t)t.b.n_desc * sizeof(rl_status), hipMemcpyDeviceToHost, S.os);
    if (he == hipSuccess && t.b.n_req) he = hipMemcpyAsync(t.hs.h_thr, t.thr, (size_t)t.b.n_req * 4, hipMemcpyDeviceToHost, S.os);
  }
  // the unpack waited for the reply exchange (ev_rs), so one event on os covers both streams
  slot[k].rep_he = he;
  slot[k].end_rec = he == hipSuccess && hipEventRecord(slot[k].ev_end, S.os) == hipSuccess;
  st.unpack_us = now_us() - t2;
}

void rl_router::wait_coll(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  Shard& S = sh[0];
  ShardStep& t = S.st[k];
  if (!slot[k].replied) {
    reply_coll(k);
    if (broken) return;
  }
  if (!slot[k].unpacked) unpack_coll(k);
  const double t2 = now_us();
  hipError_t he = slot[k].rep_he;
  // after a failure to enqueue, drain both streams
  hipError_t h2 = hipSuccess;
  if (slot[k].end_rec) {
    if (wait_bounded(slot[k].ev_end, nullptr, "all-to-all(replies)", &h2)) return;
    he = h2;
  } else {
    if (wait_bounded(nullptr, rs, "all-to-all(replies)", &h2)) return;
    if (he == hipSuccess) he = h2;
    if (he == hipSuccess && wait_bounded(nullptr, S.os, "all-to-all(replies)", &he)) return;
  }
  if (he == hipSuccess && fault(PH_UNPACK, 0)) he = hipErrorUnknown;
  st.unpack_us += now_us() - t2;
  for (uint32_t j = 0; j < G; ++j) slot[k].status[j] = h2 == hipSuccess ? t.h_x[2 * XS * G + G + j] : RL_EHIP;
  if (he != hipSuccess) {  // after the last collective: only this shard's results are lost
    slot[k].status[cfg.rank] = RL_EHIP;
    t.msg = std::string("reply exchange / unpack: ") +
            (he == hipErrorUnknown ? "injected fault (unpack)" : hipGetErrorString(he));
    t.phase = "unpack";
  }
}

void rl_router::wait_local(uint32_t k) {
  const uint32_t G = cfg.n_shards;
  const size_t D = cfg.max_desc;
  const double t0 = now_us();
  for (uint32_t j = 0; j < G; ++j) {
    ShardStep& t = sh[j].st[k];
    if (!t.rc_dec && !t.rc_local && fault(PH_DECIDE, j)) {
      t.rc_dec = RL_EHIP;
      t.msg = "injected fault (decide)";
      t.phase = "decide";
    }
    if (!t.rc_dec && !t.rc_local && (fault(PH_REPLIES, j) || fault(PH_STATUS, j))) {
      t.rc_local = RL_EHIP;
      t.msg = "injected fault (replies)";
      t.phase = "replies";
    }
    slot[k].status[j] = t.rc_dec ? t.rc_dec : t.rc_local;
  }
  hipError_t he = hipSuccess;
  for (uint32_t j = 0; j < G; ++j) {  // owner j's replies, origin-major, into each origin's section j
    uint64_t o = 0;
    for (uint32_t i = 0; i < G; ++i) {
      const uint32_t c = sh[j].st[k].rcv[i];
      if (c && he == hipSuccess)
        he = hipMemcpyAsync(sh[i].st[k].back + j * D, sh[j].st[k].reply + o, (size_t)c * RAWB, hipMemcpyDeviceToDevice,
                            rs);
      o += c;
    }
  }
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  st.reply_us = now_us() - t0;
  const double t1 = now_us();
  for (uint32_t i = 0; i < G; ++i) {
    Shard& S = sh[i];
    ShardStep& t = S.st[k];
    hipError_t hu = he;
    // every owner's decide status into this origin's device words (as the collective reply
    // exchange delivers them)
    int32_t* srecv = t.h_x + 2 * XS * G + G;
    for (uint32_t j = 0; j < G; ++j) srecv[j] = slot[k].status[j];
    if (hu == hipSuccess) hu = hipMemcpyAsync(t.d_x + 2 * XS * G + G, srecv, 4 * G, hipMemcpyHostToDevice, S.os);
    if (hu == hipSuccess && !t.late) {  // (thr zeroed by the pack)
      launch_route_unpack_raw(S.os, t.b, S.v.rules, t.pb, t.back, t.d_x + 2 * XS * G + G, cfg.max_desc, t.out, t.thr);
      hu = hipGetLastError();
      t.zeroed = hu == hipSuccess && t.b.n_desc;
    }
    if (hu == hipSuccess && slot[k].host && !t.late) {
      if (t.b.n_desc)
        hu = hipMemcpyAsync(t.hs.h_out, t.out, (size_t)t.b.n_desc * sizeof(rl_status), hipMemcpyDeviceToHost, S.os);
      if (hu == hipSuccess && t.b.n_req)
        hu = hipMemcpyAsync(t.hs.h_thr, t.thr, (size_t)t.b.n_req * 4, hipMemcpyDeviceToHost, S.os);
    }
    if (hu == hipSuccess) hu = hipStreamSynchronize(S.os);
    if (hu == hipSuccess && fault(PH_UNPACK, i)) hu = hipErrorUnknown;
    if (hu != hipSuccess && !slot[k].status[i]) {
      slot[k].status[i] = RL_EHIP;
      t.msg = std::string("reply exchange / unpack: ") +
              (hu == hipErrorUnknown ? "injected fault (unpack)" : hipGetErrorString(hu));
      t.phase = "unpack";
    }
  }
  st.unpack_us = now_us() - t1;
}

int rl_router::wait(rl_status* const* out, uint32_t* const* thr, bool into) {
  if (broken) return fail(RL_ECOMM, "the router's communicator was aborted after a transport failure");
  const uint32_t k = (uint32_t)(done % NSLOT);
  if (!slot[k].busy) return fail(RL_ESTATE, "rl_router_wait without a routed step in flight");
  if (!slot[k].counts_failed) {
    if (coll) wait_coll(k);
    else wait_local(k);
  }
  slot[k].busy = false;
  ++done;
  if (broken) return RL_ECOMM;
  const int rc = step_result(k);
  const ShardStep& t0s = sh[0].st[k];
  st.hot_groups = (uint32_t)sh[0].hot.size();
  st.combined = 0;
  st.owner_batches = t0s.n_runs;
  st.step_clock = tclock;
  if (t0s.combined)
    for (uint32_t i = 0; i < HOT_MAX; ++i) st.combined += t0s.h_x[HX_HOT + i] != 0 ? 1u : 0u;
  if (into && !rc && slot[k].host)
    for (uint32_t s = 0; s < n_local(); ++s) {
      const ShardStep& t = sh[s].st[k];
      if (out && out[s] && t.b.n_desc) memcpy(out[s], t.hs.h_out, (size_t)t.b.n_desc * sizeof(rl_status));
      if (thr && thr[s] && t.b.n_req) memcpy(thr[s], t.hs.h_thr, (size_t)t.b.n_req * 4);
    }
  st.step_us = now_us() - slot[k].t0;
  ++st.steps;
  return rc;
}

extern "C" {

int rl_router_unique_id(uint8_t* id_out) {
  if (!id_out) return RL_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RL_ECOMM;
  memcpy(id_out, &id, RL_ROUTER_ID_BYTES);
  return 0;
}

int rl_router_emu_world(uint32_t n_ranks, uint8_t* id_out) {
  if (!id_out || n_ranks == 0 || n_ranks > MAXS) return RL_EINVAL;
  EmuWorld* w = new EmuWorld();
  w->G = n_ranks;
  w->refs = (int)n_ranks;
  memset(id_out, 0, RL_ROUTER_ID_BYTES);
  const uint64_t words[3] = {EMU_MAGIC, (uint64_t)(uintptr_t)w, n_ranks};
  memcpy(id_out, words, sizeof words);
  return 0;
}

int rl_router_use_host_xchg(rl_host_xchg_fn fn, void* ctx) {
  t_xchg_fn = fn;
  t_xchg_ctx = ctx;
  return 0;
}

int rl_router_create(const rl_router_config* cfg, rl_engine* const* engines, rl_router** out) {
  if (!cfg || !engines || !out) return RL_EINVAL;
  *out = nullptr;
  if (cfg->struct_size != sizeof(rl_router_config)) return RL_EINVAL;
  const uint32_t G = cfg->n_shards;
  if (G == 0 || G > MAXS || cfg->max_desc == 0 || cfg->max_desc > (1u << 27)) return RL_EINVAL;
  if (cfg->flags & ~(uint32_t)(RL_ROUTER_NO_COMBINE | RL_ROUTER_HOST | RL_ROUTER_EMULATED | RL_ROUTER_HOST_XCHG))
    return RL_EINVAL;
  const bool emu = (cfg->flags & RL_ROUTER_EMULATED) != 0;
  const bool hx = (cfg->flags & RL_ROUTER_HOST_XCHG) != 0;
  const bool coll = cfg->rccl_id != nullptr || hx;
  if (emu && (!cfg->rccl_id || hx)) return RL_EINVAL;
  if (hx && !t_xchg_fn) return RL_EINVAL;
  if (coll && cfg->rank >= G) return RL_EINVAL;
  EmuWorld* world = nullptr;
  if (emu) {
    uint64_t words[3];
    memcpy(words, cfg->rccl_id, sizeof words);
    world = reinterpret_cast<EmuWorld*>((uintptr_t)words[1]);
    if (words[0] != EMU_MAGIC || !world || words[2] != G) return RL_EINVAL;
  }
  const uint32_t n_eng = coll ? 1u : G;
  for (uint32_t s = 0; s < n_eng; ++s)
    if (!engines[s]) return RL_EINVAL;
  rl_router* r = new rl_router();
  r->cfg = *cfg;
  r->cfg.rccl_id = nullptr;
  r->coll = coll;
  r->st.n_shards = G;
  if (emu) {  // attached now: the world lives until every rank's router is destroyed
    auto* ex = new EmuXport();
    ex->w = world;
    ex->me = cfg->rank;
    r->xp.reset(ex);
  }
  {
    const size_t N = cfg->max_desc, B = cfg->max_blob_bytes ? cfg->max_blob_bytes : (size_t)cfg->max_desc * 64;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    r->o_off = al(B + RL_BLOB_SLACK);
    r->o_rule = r->o_off + al((N + 1) * 4);
    r->o_req = r->o_rule + al(N * 4);
    r->o_now = r->o_req + al(N * 4);
    r->o_hits = r->o_now + al(N * 8);
    r->o_jit = r->o_hits + al(N * 4);
    r->in_bytes = r->o_jit + al(N * 2);
  }
  if (const char* t = getenv("RL_ROUTER_TIMEOUT_MS")) {
    const long long v = atoll(t);
    if (v > 0) r->timeout_ms = v;
  }
  if (emu) {
    std::lock_guard<std::mutex> l(world->mu);
    world->timeout_ms = r->timeout_ms;
  }
  if (const char* f = getenv("RL_ROUTER_FAULT")) {  // tests: "phase:shard[:step]"
    char ph[32] = {0};
    unsigned s = 0, k = 0;
    if (sscanf(f, "%31[a-z]:%u:%u", ph, &s, &k) >= 2) {
      r->fault_step = k;
      for (int p = 1; p <= PH_STALL; ++p)
        if (!strcmp(ph, kPhaseNames[p])) {
          r->fault_phase = p;
          r->fault_shard = coll ? (s == cfg->rank ? 0u : 0xFFFFFFFFu) : s;
        }
    }
  }
  auto bail = [&](int code) {
    if (emu && r->xp) r->xp->abort();  // peers blocked in create's exchange return
    r->free_all();
    delete r;
    return code;
  };
  if (hipStreamCreateWithFlags(&r->rs, hipStreamNonBlocking) != hipSuccess) return bail(RL_EHIP);
  if (hipEventCreateWithFlags(&r->ev_rs, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&r->ev_cnt, hipEventDisableTiming) != hipSuccess ||
      std::any_of(std::begin(r->slot), std::end(r->slot), [](StepSlot& q) {
        return hipEventCreateWithFlags(&q.ev_end, hipEventDisableTiming) != hipSuccess ||
               hipEventCreateWithFlags(&q.ev_rec, hipEventDisableTiming) != hipSuccess;
      }))
    return bail(RL_EHIP);
  if (r->fault_phase == PH_STALL) {
    if (hipHostMalloc(&r->h_stall, 64, hipHostMallocDefault) != hipSuccess) return bail(RL_EHIP);
    *r->h_stall = 0;
  }
  if (emu) {
    auto* ex = static_cast<EmuXport*>(r->xp.get());
    if (hipEventCreateWithFlags(&ex->ev_pre, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ex->ev_post, hipEventDisableTiming) != hipSuccess)
      return bail(RL_EHIP);
  }
  r->sh.resize(n_eng);
  for (uint32_t s = 0; s < n_eng; ++s) {
    r->sh[s].e = engines[s];
    if (rlx_engine_view(engines[s], &r->sh[s].v)) return bail(RL_EINVAL);
    if (rlx_engine_set_lag(engines[s], true)) {
      r->err = "an engine that already decided batches needs RL_CFG_LAG_WINDOW at rl_create to serve a router";
      return bail(RL_ESTATE);
    }
    if (r->alloc_shard(r->sh[s])) return bail(RL_EHIP);
  }
#ifndef RL_ROUTER_TWO_STREAMS
  if (coll) {
    // One rank, one origin: its pack, exchanges and unpack on one stream. They form one chain
    // anyway, and every hand-over between two streams costs ~10-15 us on the critical path
    // (pack -> counts, replies -> unpack), more than their overlap with each other can win.
    (void)hipStreamDestroy(r->rs);
    r->rs = r->sh[0].os;
    r->rs_own = false;
  }
#endif
  if (coll) {
    if (hipMalloc(&r->d_ag, sizeof(AgEntry) * HOT_MAX * (G + 1)) != hipSuccess ||
        hipHostMalloc(&r->h_ag, sizeof(AgEntry) * HOT_MAX * (G + 1), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&r->d_ok, 4 * MAXS) != hipSuccess || hipMemset(r->d_ok, 0, 4 * MAXS) != hipSuccess)
      return bail(RL_EHIP);
    if (hx) {
      auto* xx = new HostXchgXport();
      xx->fn = t_xchg_fn;
      xx->ctx = t_xchg_ctx;
      xx->G = G;
      r->xp.reset(xx);
    } else if (!emu) {
      auto* rx = new RcclXport();
      r->xp.reset(rx);
      ncclUniqueId id;
      memcpy(&id, cfg->rccl_id, RL_ROUTER_ID_BYTES);
      if (ncclCommInitRank(&rx->comm, (int)G, id, (int)cfg->rank) != ncclSuccess) {
        rx->comm = nullptr;
        return bail(RL_ECOMM);
      }
    }
  }
  if (int rc = r->check_config()) return bail(rc);
  for (uint32_t s = 0; s < n_eng; ++s) (void)rlx_engine_set_lag(engines[s], false);  // (checked above)
  *out = r;
  return 0;
}

int rl_router_submit(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_thr) {
  if (!r || !batches || !d_out || !d_thr) return RL_EINVAL;
  return r->submit(batches, d_out, d_thr, false);
}

int rl_router_wait(rl_router* r) {
  if (!r) return RL_EINVAL;
  return r->wait(nullptr, nullptr, false);
}

int rl_router_step(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_thr) {
  const int rc = rl_router_submit(r, batches, d_out, d_thr);
  if (rc) return rc;
  return rl_router_wait(r);
}

int rl_router_host_acquire(rl_router* r, uint32_t shard, rl_host_batch* out) {
  if (!r || !out) return RL_EINVAL;
  if (!(r->cfg.flags & RL_ROUTER_HOST)) return r->fail(RL_EINVAL, "router created without RL_ROUTER_HOST");
  if (shard >= r->n_local()) return r->fail(RL_EINVAL, "shard %u out of range", shard);
  const uint32_t k = (uint32_t)(r->seq % NSLOT);
  if (r->slot[k].busy) return r->fail(RL_ESTATE, "%d routed steps in flight: call rl_router_wait_into", NSLOT);
  uint8_t* h = r->sh[shard].st[k].hs.h_in;
  out->prefix_blob = h;
  out->prefix_off = reinterpret_cast<uint32_t*>(h + r->o_off);
  out->rule_id = reinterpret_cast<uint32_t*>(h + r->o_rule);
  out->req_of = reinterpret_cast<uint32_t*>(h + r->o_req);
  out->now = reinterpret_cast<int64_t*>(h + r->o_now);
  out->hits_addend = reinterpret_cast<uint32_t*>(h + r->o_hits);
  out->ttl_jitter = reinterpret_cast<uint16_t*>(h + r->o_jit);
  out->max_desc = r->cfg.max_desc;
  out->max_req = r->cfg.max_desc;
  out->max_blob = (uint32_t)(r->o_off - RL_BLOB_SLACK);
  out->reserved = 0;
  return 0;
}

int rl_router_submit_host(rl_router* r, const rl_batch* host_batches) {
  if (!r || !host_batches) return RL_EINVAL;
  return r->submit(host_batches, nullptr, nullptr, true);
}

int rl_router_wait_into(rl_router* r, rl_status* const* out, uint32_t* const* thr) {
  if (!r) return RL_EINVAL;
  return r->wait(out, thr, true);
}

int rl_router_allgather_host(rl_router* r, const void* in, uint32_t n_bytes, void* out) {
  if (!r || (n_bytes && (!in || !out))) return RL_EINVAL;
  if (!r->coll) return r->fail(RL_ESTATE, "rl_router_allgather_host needs the collective transport");
  if (n_bytes > RL_ROUTER_AG_MAX) return r->fail(RL_EINVAL, "rl_router_allgather_host: %u bytes > %u", n_bytes,
                                                 RL_ROUTER_AG_MAX);
  if (r->broken) return r->fail(RL_ECOMM, "the router's communicator was aborted after a transport failure");
  const uint32_t G = r->cfg.n_shards;
  uint8_t* hs = reinterpret_cast<uint8_t*>(r->h_ag);
  uint8_t* ds = reinterpret_cast<uint8_t*>(r->d_ag);
  static_assert(RL_ROUTER_AG_MAX <= sizeof(AgEntry) * HOT_MAX, "allgather staging");
  if (n_bytes) memcpy(hs, in, n_bytes);
  hipError_t he = n_bytes ? hipMemcpyAsync(ds, hs, n_bytes, hipMemcpyHostToDevice, r->rs) : hipSuccess;
  const ncclResult_t nr = r->xp->allgather(ds, ds + RL_ROUTER_AG_MAX, n_bytes, r->rs);
  if (nr != ncclSuccess) return r->nccl_fail(nr, "allgather(host words)");
  if (he == hipSuccess && n_bytes)
    he = hipMemcpyAsync(hs + RL_ROUTER_AG_MAX, ds + RL_ROUTER_AG_MAX, (size_t)n_bytes * G, hipMemcpyDeviceToHost, r->rs);
  if (he == hipSuccess)
    if (int rc = r->wait_bounded(nullptr, r->rs, "allgather(host words)", &he)) return rc;
  if (he != hipSuccess) {  // the peers have their words; this rank cannot tell what it received
    r->abort_comm();
    return r->fail(RL_ECOMM, "allgather(host words): %s (communicator aborted)", hipGetErrorString(he));
  }
  if (n_bytes) memcpy(out, hs + RL_ROUTER_AG_MAX, (size_t)n_bytes * G);
  return 0;
}

int rl_router_get_stats(const rl_router* r, rl_router_stats* out) {
  if (!r || !out) return RL_EINVAL;
  *out = r->st;
  return 0;
}

const char* rl_router_last_error(const rl_router* r) { return r ? r->err.c_str() : "null router"; }

void rl_router_destroy(rl_router* r) {
  if (!r) return;
  // steps still in flight: complete them (every rank issued their collectives)
  while (!r->broken && r->done < r->seq) (void)r->wait(nullptr, nullptr, false);
  // A broken router leaves steps unwaited: their owner batches are still queued in the engine,
  // which outlives the router, and read and write buffers free_all releases. Complete them
  // oldest step first (the engine's FIFO order), every slot.
  for (Shard& s : r->sh) {
    for (uint64_t q = r->done; q < r->seq; ++q) {
      ShardStep& x = s.st[q % NSLOT];
      while (x.n_sub) r->drain(s, x);
    }
    for (ShardStep& x : s.st)
      while (x.n_sub) r->drain(s, x);
    (void)hipStreamSynchronize(s.os);
  }
  if (r->rs) (void)hipStreamSynchronize(r->rs);
  r->free_all();
  delete r;
}

}  // extern "C"
