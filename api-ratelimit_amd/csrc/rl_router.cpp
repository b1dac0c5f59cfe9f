// rl_router.cpp — the routed DoLimit step behind one C call (include/rl_hip.h
// "Router object").
//
// The reference sends each key's INCRBY to the Redis server that holds it and pipelines the
// commands of a request (src/redis/fixed_cache_impl.go:66-80, src/redis/driver_impl.go:84-110).
// Here GPU s owns the keys whose prefix fingerprint maps to s (route_owner); one step of a
// shard packs its origin batch by owner (rl_route_pack), exchanges per-owner counts and then
// the 32-B records, decides what it received as owner (rl_submit_routed, origin-major), sends
// the 24-B replies back and unpacks them (rl_route_unpack).
//
// Transports: RCCL (one process per GPU, ncclAllToAll / ncclAllToAllv on a stream the router
// owns) or local (n_shards engines in one process, device-to-device copies). Both carry a
// status word per shard through each exchange, so every shard completes every collective of
// a step and then all of them fail together.
//
// Local transport: host-synchronous between phases. RCCL transport: three host waits per
// step (counts, the owner's decide, the end), the two streams ordered by events otherwise.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rl_hip.h"

namespace {

constexpr uint32_t REC = RL_ROUTE_RECORD_BYTES;
constexpr uint32_t REP = RL_ROUTE_REPLY_BYTES;
constexpr uint32_t MAXS = RL_ROUTE_MAX_SHARDS;

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-shard exchange buffers (device): an origin's records by owner and its reply area, an
// owner's received records and replies.
struct ShardBufs {
  rl_engine* e = nullptr;
  void* send = nullptr;       // max_desc records, grouped by owner
  uint32_t* d_cnt = nullptr;  // per-owner counts (rl_route_pack)
  uint32_t* perm = nullptr;   // max_desc
  void* recv = nullptr;       // n_shards * max_desc records
  void* reply = nullptr;      // n_shards * max_desc replies
  void* back = nullptr;       // max_desc replies (origin side)
  uint32_t cnt[MAXS] = {};    // records this origin sends each owner
};

}  // namespace

struct rl_router {
  rl_router_config cfg{};
  bool rccl = false;
  ncclComm_t comm = nullptr;
  hipStream_t rs = nullptr;  // exchanges
  std::vector<ShardBufs> sh;
  int32_t* d_x = nullptr;    // RCCL: [2G] send + [2G] receive status/count words
  int32_t* h_x = nullptr;    // pinned mirror of d_x + [G] owner statuses
  hipEvent_t ev = nullptr;   // orders the router and engine streams
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
  int hip(hipError_t he, const char* what) {
    return he == hipSuccess ? 0 : fail(RL_EHIP, "%s: %s", what, hipGetErrorString(he));
  }
  int nccl(ncclResult_t nr, const char* what) {
    return nr == ncclSuccess ? 0 : fail(RL_ECOMM, "%s: %s", what, ncclGetErrorString(nr));
  }
  int step_local(const rl_batch* b, rl_status* const* out, uint32_t* const* thr);
  int step_rccl(const rl_batch* b, rl_status* out, uint32_t* thr);
  void free_all();
};

void rl_router::free_all() {
  for (ShardBufs& s : sh) {
    for (void* p : {s.send, (void*)s.d_cnt, (void*)s.perm, s.recv, s.reply, s.back})
      if (p) (void)hipFree(p);
  }
  sh.clear();
  if (d_x) (void)hipFree(d_x);
  if (h_x) (void)hipHostFree(h_x);
  if (comm) (void)ncclCommDestroy(comm);
  if (rs) (void)hipStreamDestroy(rs);
  if (ev) (void)hipEventDestroy(ev);
  ev = nullptr;
  d_x = nullptr;
  h_x = nullptr;
  comm = nullptr;
  rs = nullptr;
}

// Local transport: every shard's batch, all exchanges by copies on the router stream.
int rl_router::step_local(const rl_batch* b, rl_status* const* out, uint32_t* const* thr) {
  const uint32_t G = cfg.n_shards;
  const double t0 = now_us();
  int first_err = 0;
  for (uint32_t s = 0; s < G; ++s) {
    const int rc = rl_route_pack(sh[s].e, &b[s], s, G, sh[s].send, sh[s].d_cnt, sh[s].perm, sh[s].cnt);
    st.status[s] = rc;
    if (rc && !first_err) {
      first_err = rc;
      fail(rc, "shard %u (pack): %s", s, rl_last_error(sh[s].e));
    }
  }
  const double t1 = now_us();
  st.pack_us = t1 - t0;
  if (first_err) return first_err;
  for (uint32_t j = 0; j < G; ++j) st.sent[j] = sh[0].cnt[j];
  // records: owner j receives origin 0's group j, then origin 1's, ...
  std::vector<uint64_t> sdis(G * G), rdis(G * G);  // [i*G+j]: record offset of (origin i, owner j)
  for (uint32_t i = 0; i < G; ++i) {
    uint64_t o = 0;
    for (uint32_t j = 0; j < G; ++j) {
      sdis[i * G + j] = o;
      o += sh[i].cnt[j];
    }
  }
  for (uint32_t j = 0; j < G; ++j) {
    uint64_t o = 0;
    for (uint32_t i = 0; i < G; ++i) {
      rdis[i * G + j] = o;
      o += sh[i].cnt[j];
    }
    st.recv[j] = (uint32_t)o;
  }
  hipError_t he = hipSuccess;
  for (uint32_t i = 0; i < G && he == hipSuccess; ++i)
    for (uint32_t j = 0; j < G && he == hipSuccess; ++j)
      if (sh[i].cnt[j])
        he = hipMemcpyAsync(static_cast<uint8_t*>(sh[j].recv) + rdis[i * G + j] * REC,
                            static_cast<const uint8_t*>(sh[i].send) + sdis[i * G + j] * REC, (size_t)sh[i].cnt[j] * REC,
                            hipMemcpyDeviceToDevice, rs);
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  if (int rc = hip(he, "record exchange")) return rc;
  const double t2 = now_us();
  st.exchange_us = t2 - t1;
  // owners decide one after another (logical shards share the device; each alone is the
  // model of one GPU, so decide_max_us is the step's critical path on G real GPUs)
  st.decide_max_us = 0;
  for (uint32_t j = 0; j < G; ++j) {
    const double a = now_us();
    int rc = 0;
    if (st.recv[j]) {
      rc = rl_submit_routed(sh[j].e, sh[j].recv, st.recv[j], sh[j].reply);
      if (!rc) rc = rl_wait(sh[j].e);
    }
    const double d = now_us() - a;
    st.decide_max_us = d > st.decide_max_us ? d : st.decide_max_us;
    st.status[j] = rc;
    if (rc && !first_err) {
      first_err = rc;
      fail(rc, "shard %u (decide): %s", j, rl_last_error(sh[j].e));
    }
  }
  const double t3 = now_us();
  st.decide_us = t3 - t2;
  if (first_err) return first_err;
  for (uint32_t i = 0; i < G && he == hipSuccess; ++i)
    for (uint32_t j = 0; j < G && he == hipSuccess; ++j)
      if (sh[i].cnt[j])
        he = hipMemcpyAsync(static_cast<uint8_t*>(sh[i].back) + sdis[i * G + j] * REP,
                            static_cast<const uint8_t*>(sh[j].reply) + rdis[i * G + j] * REP,
                            (size_t)sh[i].cnt[j] * REP, hipMemcpyDeviceToDevice, rs);
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  if (int rc = hip(he, "reply exchange")) return rc;
  const double t4 = now_us();
  st.reply_us = t4 - t3;
  for (uint32_t i = 0; i < G; ++i) {
    int rc = rl_route_unpack(sh[i].e, &b[i], sh[i].perm, sh[i].back, out[i], thr[i]);
    if (!rc) rc = hip(hipStreamSynchronize((hipStream_t)rl_stream(sh[i].e)), "unpack");
    else fail(rc, "shard %u (unpack): %s", i, rl_last_error(sh[i].e));
    if (rc) return rc;
  }
  st.unpack_us = now_us() - t4;
  return 0;
}

// RCCL transport: this rank's batch; counts + status, records, replies + status over the
// communicator. Every rank runs all three exchanges whatever its own status.
//
// Three host waits per step: the counts (the record exchange's split sizes), the owner's
// decide (its status), and the end of the step. rl_route_pack_async writes the (count, status)
// pairs on the device, so the pack needs no wait of its own; the router stream and the engine
// stream are ordered by events around the record exchange and the unpack. The unpack runs
// before the owners' statuses are read: when a step fails, out and thr hold garbage.
int rl_router::step_rccl(const rl_batch* b, rl_status* out, uint32_t* thr) {
  const uint32_t G = cfg.n_shards, me = cfg.rank;
  ShardBufs& s = sh[0];
  hipStream_t es = (hipStream_t)rl_stream(s.e);
  const double t0 = now_us();
  int rc_pack = RL_ECAPACITY;
  std::string pack_msg = "batch exceeds the router's max_desc";
  if (b->n_desc <= cfg.max_desc) {
    rc_pack = rl_route_pack_strided(s.e, b, me, G, cfg.max_desc, s.send, reinterpret_cast<uint32_t*>(d_x), s.perm);
    pack_msg = rc_pack ? rl_last_error(s.e) : "";
  }
  int32_t* hs = h_x;           // [2G] sent
  int32_t* hr = h_x + 2 * G;   // [2G] received
  hipError_t he;
  if (rc_pack) {  // found on the host: no pairs on the device, send (0, rc_pack) to every owner
    for (uint32_t j = 0; j < G; ++j) {
      hs[2 * j] = 0;
      hs[2 * j + 1] = rc_pack;
    }
    he = hipMemcpyAsync(d_x, hs, 8 * G, hipMemcpyHostToDevice, rs);
  } else {
    he = hipEventRecord(ev, es);
    if (he == hipSuccess) he = hipStreamWaitEvent(rs, ev, 0);
  }
  if (int rc = hip(he, "counts upload")) return rc;
  if (int rc = nccl(ncclAllToAll(d_x, d_x + 2 * G, 2, ncclInt32, comm, rs), "ncclAllToAll(counts)")) return rc;
  he = hipMemcpyAsync(h_x, d_x, 16 * G, hipMemcpyDeviceToHost, rs);  // sent and received pairs
  if (he == hipSuccess) he = hipStreamSynchronize(rs);
  if (int rc = hip(he, "counts exchange")) return rc;
  if (!rc_pack && hs[1]) {  // the device found the batch malformed (rl_route_pack's checks)
    rc_pack = hs[1];
    pack_msg = "rl_route_pack_async: batch references an unknown rule id or request index, malformed prefix "
               "offsets, or a time outside [0, 0xFFFD0000]";
  }
  const double t1 = now_us();
  st.pack_us = t1 - t0;
  int first_err = 0;
  for (uint32_t j = 0; j < G; ++j) {
    s.cnt[j] = rc_pack ? 0u : (uint32_t)hs[2 * j];
    st.status[j] = hr[2 * j + 1];
    if (hr[2 * j + 1] && !first_err) first_err = j == me ? hr[2 * j + 1] : RL_EPEER;
  }
  if (first_err) {  // every rank saw the same status words: all leave here together
    if (rc_pack) return fail(rc_pack, "shard %u (pack): %s", me, pack_msg.c_str());
    return fail(RL_EPEER, "a peer shard failed to pack its batch (see rl_router_stats.status)");
  }
  std::vector<size_t> sc(G), sd(G), rc_(G), rd(G);
  uint64_t so = 0, ro = 0;
  const size_t D = cfg.max_desc;  // owner stride of the send and back buffers (rl_route_pack_strided)
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)s.cnt[j] * REC;
    sd[j] = j * D * REC;
    rc_[j] = (size_t)(uint32_t)hr[2 * j] * REC;
    rd[j] = ro;
    ro += rc_[j];
    st.sent[j] = s.cnt[j];
  }
  const uint32_t n_in = (uint32_t)(ro / REC);
  for (uint32_t j = 0; j < G; ++j) st.recv[j] = j == me ? n_in : 0;
  if (int rc = nccl(ncclAllToAllv(s.send, sc.data(), sd.data(), s.recv, rc_.data(), rd.data(), ncclUint8, comm, rs),
                    "ncclAllToAllv(records)"))
    return rc;
  he = hipEventRecord(ev, rs);  // the owner's decide reads the received records
  if (he == hipSuccess) he = hipStreamWaitEvent(es, ev, 0);
  if (int rc = hip(he, "record exchange")) return rc;
  const double t2 = now_us();
  st.exchange_us = t2 - t1;  // enqueue only: the exchange's time is inside decide_us
  int rc_dec = 0;
  if (n_in) {
    rc_dec = rl_submit_routed(s.e, s.recv, n_in, s.reply);
    if (!rc_dec) rc_dec = rl_wait(s.e);
  }
  std::string dec_msg = rc_dec ? rl_last_error(s.e) : "";
  if (!n_in) {  // nothing decided: the exchange still has to be complete before the replies
    if (int rc = hip(hipStreamSynchronize(es), "record exchange")) return rc;
  }
  const double t3 = now_us();
  st.decide_us = st.decide_max_us = t3 - t2;
  for (uint32_t j = 0; j < G; ++j) hs[j] = rc_dec;
  he = hipMemcpyAsync(d_x, hs, 4 * G, hipMemcpyHostToDevice, rs);
  if (int rc = hip(he, "status upload")) return rc;
  // replies go back with the reverse splits; the status words ride in the same group
  for (uint32_t j = 0; j < G; ++j) {
    sc[j] = (size_t)(uint32_t)hr[2 * j] * REP;  // to origin j: the replies to its records
    rc_[j] = (size_t)s.cnt[j] * REP;
  }
  so = 0;
  for (uint32_t j = 0; j < G; ++j) {
    sd[j] = so;
    so += sc[j];
    rd[j] = j * D * REP;  // perm[i] = owner * D + position
  }
  ncclResult_t nr = ncclGroupStart();
  if (nr == ncclSuccess) nr = ncclAllToAll(d_x, d_x + 2 * G, 1, ncclInt32, comm, rs);
  if (nr == ncclSuccess)
    nr = ncclAllToAllv(s.reply, sc.data(), sd.data(), s.back, rc_.data(), rd.data(), ncclUint8, comm, rs);
  const ncclResult_t ne = ncclGroupEnd();
  if (int rc = nccl(nr != ncclSuccess ? nr : ne, "ncclAllToAll(replies)")) return rc;
  int32_t* hst = h_x + 4 * G;  // the owners' statuses (own pinned words: hs is still being uploaded)
  he = hipMemcpyAsync(hst, d_x + 2 * G, 4 * G, hipMemcpyDeviceToHost, rs);
  if (he == hipSuccess) he = hipEventRecord(ev, rs);
  if (he == hipSuccess) he = hipStreamWaitEvent(es, ev, 0);
  if (int rc = hip(he, "reply exchange")) return rc;
  int rc = rl_route_unpack(s.e, b, s.perm, s.back, out, thr);
  if (rc) {
    (void)hipStreamSynchronize(rs);  // the exchange is complete before the error returns
    return fail(rc, "shard %u (unpack): %s", me, rl_last_error(s.e));
  }
  if ((rc = hip(hipStreamSynchronize(es), "reply exchange and unpack"))) return rc;
  st.reply_us = now_us() - t3;
  st.unpack_us = 0;  // inside reply_us
  for (uint32_t j = 0; j < G; ++j) {
    st.status[j] = hst[j];
    if (hst[j] && !first_err) first_err = j == me ? hst[j] : RL_EPEER;
  }
  if (first_err) {
    if (rc_dec) return fail(rc_dec, "shard %u (decide): %s", me, dec_msg.c_str());
    return fail(RL_EPEER, "a peer shard failed to decide its records (see rl_router_stats.status)");
  }
  return 0;
}

extern "C" {

int rl_router_unique_id(uint8_t* id_out) {
  if (!id_out) return RL_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RL_ECOMM;
  memcpy(id_out, &id, RL_ROUTER_ID_BYTES);
  return 0;
}

int rl_router_create(const rl_router_config* cfg, rl_engine* const* engines, rl_router** out) {
  if (!cfg || !engines || !out) return RL_EINVAL;
  if (cfg->struct_size != sizeof(rl_router_config)) return RL_EINVAL;
  const uint32_t G = cfg->n_shards;
  if (G == 0 || G > MAXS || cfg->max_desc == 0 || cfg->max_desc > (1u << 27)) return RL_EINVAL;
  const bool rccl = cfg->rccl_id != nullptr;
  if (rccl && cfg->rank >= G) return RL_EINVAL;
  const uint32_t n_eng = rccl ? 1u : G;
  for (uint32_t s = 0; s < n_eng; ++s)
    if (!engines[s]) return RL_EINVAL;
  rl_router* r = new rl_router();
  r->cfg = *cfg;
  r->cfg.rccl_id = nullptr;
  r->rccl = rccl;
  r->st.n_shards = G;
  auto bail = [&](hipError_t he) {
    r->free_all();
    delete r;
    return he == hipSuccess ? RL_ECOMM : RL_EHIP;
  };
  hipError_t he = hipStreamCreateWithFlags(&r->rs, hipStreamNonBlocking);
  if (he != hipSuccess) return bail(he);
  const size_t D = cfg->max_desc;
  r->sh.resize(n_eng);
  for (uint32_t s = 0; s < n_eng && he == hipSuccess; ++s) {
    ShardBufs& b = r->sh[s];
    b.e = engines[s];
    // RCCL transport: owner-strided send / back buffers (rl_route_pack_strided); local: compact
    he = hipMalloc(&b.send, D * (rccl ? G : 1) * REC);
    if (he == hipSuccess) he = hipMalloc(&b.d_cnt, MAXS * 4);
    if (he == hipSuccess) he = hipMalloc(&b.perm, D * 4);
    if (he == hipSuccess) he = hipMalloc(&b.recv, D * G * REC);
    if (he == hipSuccess) he = hipMalloc(&b.reply, D * G * REP);
    if (he == hipSuccess) he = hipMalloc(&b.back, D * (rccl ? G : 1) * REP);
  }
  if (he == hipSuccess && rccl) {
    he = hipMalloc(&r->d_x, 4 * G * 4);
    if (he == hipSuccess) he = hipHostMalloc(&r->h_x, 5 * G * 4, hipHostMallocDefault);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
  }
  if (he != hipSuccess) return bail(he);
  if (rccl) {
    ncclUniqueId id;
    memcpy(&id, cfg->rccl_id, RL_ROUTER_ID_BYTES);
    if (ncclCommInitRank(&r->comm, (int)G, id, (int)cfg->rank) != ncclSuccess) {
      r->comm = nullptr;
      return bail(hipSuccess);
    }
  }
  *out = r;
  return 0;
}

int rl_router_step(rl_router* r, const rl_batch* batches, rl_status* const* d_out, uint32_t* const* d_thr) {
  if (!r || !batches || !d_out || !d_thr) return RL_EINVAL;
  if (!r->rccl)  // (the RCCL transport reports an oversized batch through the counts exchange)
    for (uint32_t s = 0; s < r->cfg.n_shards; ++s)
      if (batches[s].n_desc > r->cfg.max_desc)
        return r->fail(RL_ECAPACITY, "shard %u: batch of %u descriptors exceeds the router's max_desc %u", s,
                       batches[s].n_desc, r->cfg.max_desc);
  for (uint32_t j = 0; j < MAXS; ++j) r->st.status[j] = 0, r->st.recv[j] = 0, r->st.sent[j] = 0;
  const double t0 = now_us();
  const int rc = r->rccl ? r->step_rccl(batches, d_out[0], d_thr[0]) : r->step_local(batches, d_out, d_thr);
  r->st.step_us = now_us() - t0;
  ++r->st.steps;
  return rc;
}

int rl_router_get_stats(const rl_router* r, rl_router_stats* out) {
  if (!r || !out) return RL_EINVAL;
  *out = r->st;
  return 0;
}

const char* rl_router_last_error(const rl_router* r) { return r ? r->err.c_str() : "null router"; }

void rl_router_destroy(rl_router* r) {
  if (!r) return;
  r->free_all();
  delete r;
}

}  // extern "C"
