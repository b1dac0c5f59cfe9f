// rl_route.hip — multi-GPU key routing.
//
// The reference scales DoLimit out by pointing every ratelimit replica at one Redis (or a
// Redis cluster that shards keys by slot); the decision for a key is made where its
// counter lives (src/redis/fixed_cache_impl.go:66-80 pipelines INCRBY to the key's
// server). Here each GPU owns the counter table of the keys that route_owner() assigns to
// it. An origin GPU turns its batch into 32-B routed records grouped by owner (stable, so
// every owner sees an origin's descriptors in serial order), the records travel with one
// RCCL all-to-all, each owner decides them with the ordinary pipeline, and the 24-B
// replies travel back with the reverse all-to-all into the origin's descriptor order.
//
//   k_route_hash    descriptor -> RRec (prefix lanes hashed once, at the origin) + owner
//   k_route_scan    per (block, owner) counts -> stable send offsets, per-owner totals
//   k_route_scatter RRec -> send buffer position, perm[i] = position (or RL_ROUTE_LOCAL)
//   k_route_reply   owner: (out, thr) of the routed batch -> RReply records
//   k_route_unpack  origin: replies -> out[i], max into ThrottleMillis of req_of[i]
#include "rl_common.h"
#include "rl_decide.h"
#include "rl_device.h"
#include "rl_internal.h"

namespace rlhip {
namespace route {

constexpr int NT = 256;       // descriptors per block (one per thread)
constexpr int NS = ROUTE_MAX_SHARDS;
constexpr int SCAN_NT = 1024;

__global__ __launch_bounds__(NT) void k_route_hash(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                                    uint64_t seed, uint32_t origin, uint32_t n_shards,
                                                    RRec* __restrict__ tmp, uint8_t* __restrict__ own,
                                                    uint32_t* __restrict__ bcnt, EngineCtl* ctl) {
  __shared__ uint32_t s_cnt[NS];
  __shared__ uint32_t s_err;
  const uint32_t tid = threadIdx.x, i = blockIdx.x * NT + tid;
  if (tid < NS) s_cnt[tid] = 0;
  if (tid == 0) s_err = 0;
  __syncthreads();
  if (i < in.n_desc) {
    // two levels of loads, each issued together (clamped indices; the blob is readable
    // RL_BLOB_SLACK bytes past its end): (rule, request, prefix offsets), then (now, hits, the
    // prefix's first 32 bytes)
    const uint32_t rule = in.rule[i], q = in.req_of[i], qp = in.req_of[i ? i - 1u : 0u];
    const uint32_t o0 = in.off[i], o1 = in.off[i + 1];
    uint32_t err = 0, o = ROUTE_LOCAL;
    if (o1 < o0 || o1 > in.blob_bytes || qp > q) err |= ERR_BAD_INPUT;
    const bool nil = rule == RL_NIL_RULE;
    if (!nil && !err && (rule >= n_rules || rule >= RREC_MAX_RULE || q >= in.n_req)) err |= ERR_BAD_INPUT;
    const uint32_t qc = q < in.n_req ? q : 0u;
    const uint32_t oc = err ? 0u : o0;
    const int64_t now = in.now[qc];
    const uint32_t ha = in.hits[qc];
    const u32x4* pw = reinterpret_cast<const u32x4*>(in.blob + (oc & ~3u));
    const u32x4 w0 = pw[0];
    const u32x4 w1 = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint32_t*>(pw) + 4);
    if (!nil && !err) {
      if (now < 0 || now > MAX_NOW) {
        err |= ERR_BAD_TIME;
      } else {
        const FpState s = prefix_state_pre(w0, w1, in.blob, o0, o1 - o0, seed);
        RRec r;
        r.a = s.a;
        r.b = s.b;
        r.now = (uint32_t)now;
        r.rule = rule | (desc_jit(in, i) << 16);  // the EXPIRE jitter travels with the record
        r.h = ha > 1u ? ha : 1u;  // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
        r.greq = (origin << ROUTE_REQ_BITS) | q;
        tmp[i] = r;
        o = route_owner(s.a, s.b, n_shards);
        atomicAdd(&s_cnt[o], 1u);
      }
    }
    own[i] = (uint8_t)o;
    if (err) atomicOr(&s_err, err);
  }
  __syncthreads();
  if (tid < NS) bcnt[blockIdx.x * NS + tid] = s_cnt[tid];
  // the block's error flags after every block's counts (k_route_scan folds them: no atomic,
  // no memset of the error word before the launch)
  if (tid == 0) bcnt[gridDim.x * NS + blockIdx.x] = s_err;
}

// One block: wave w < n_shards scans column w over the blocks (exclusive, in place), in
// chunks of 64 x RPL blocks: lane l holds RPL consecutive blocks' counts in registers (all
// loads in flight together, clamped), one DPP scan of the lanes' sums, then the lane writes
// its run's prefixes. Owner totals are scanned into owner offsets in between (a second
// read of the column is cheap: it is in the L2). The blocks' error flags are folded into
// ctl->err; ctl words 1..n_shards get the owner totals too, so the host reads both in one copy.
constexpr int RPL = 32;
__global__ __launch_bounds__(SCAN_NT) void k_route_scan(uint32_t* __restrict__ bcnt, uint32_t nb, uint32_t n_shards,
                                                        uint32_t* __restrict__ send_counts, EngineCtl* ctl,
                                                        uint32_t* __restrict__ x) {
  __shared__ uint32_t s_tot[NS], s_off[NS], s_err;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  static_assert(SCAN_NT / 64 >= NS, "one wave per shard column");
  if (tid == 0) s_err = 0;
  __syncthreads();
  constexpr uint32_t CH = 64u * RPL;  // blocks per chunk
  // pass 1: column totals
  if (w < n_shards) {  // wave-uniform
    uint32_t tot = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += CH) {
      uint32_t v[RPL];
#pragma unroll
      for (int u = 0; u < RPL; ++u) v[u] = bcnt[(size_t)min(c0 + lane * RPL + u, nb - 1u) * NS + w];
      uint32_t sum = 0;
#pragma unroll
      for (int u = 0; u < RPL; ++u) sum += c0 + lane * RPL + u < nb ? v[u] : 0u;
      tot += wave_sum_u32(sum);
    }
    if (lane == 0) s_tot[w] = tot;
  }
  uint32_t err = 0;
  for (uint32_t b = tid; b < nb; b += SCAN_NT) err |= bcnt[(size_t)nb * NS + b];
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    uint32_t* cw = reinterpret_cast<uint32_t*>(ctl);
    for (uint32_t s2 = 0; s2 < n_shards; ++s2) {
      s_off[s2] = acc;
      if (send_counts) send_counts[s2] = s_tot[s2];
      cw[1 + s2] = s_tot[s2];
      if (x) {  // rl_route_pack_async: (count, status) per owner for the all-to-all of counts
        x[2 * s2] = s_tot[s2];
        x[2 * s2 + 1] = s_err & (ERR_BAD_INPUT | ERR_BAD_TIME) ? (uint32_t)RL_EINVAL : 0u;
      }
      acc += s_tot[s2];
    }
    cw[0] = s_err;
  }
  __syncthreads();
  // pass 2: exclusive prefixes + the owner's offset
  if (w < n_shards) {
    uint32_t carry = s_off[w];
    for (uint32_t c0 = 0; c0 < nb; c0 += CH) {
      uint32_t v[RPL];
#pragma unroll
      for (int u = 0; u < RPL; ++u) v[u] = bcnt[(size_t)min(c0 + lane * RPL + u, nb - 1u) * NS + w];
      uint32_t sum = 0;
#pragma unroll
      for (int u = 0; u < RPL; ++u) {
        v[u] = c0 + lane * RPL + u < nb ? v[u] : 0u;
        sum += v[u];
      }
      const uint32_t incl = wave_incl_scan_u32(sum);
      uint32_t run = carry + incl - sum;
#pragma unroll
      for (int u = 0; u < RPL; ++u) {
        const uint32_t b = c0 + lane * RPL + u;
        if (b < nb) bcnt[(size_t)b * NS + w] = run;
        run += v[u];
      }
      carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
  }
}

// Stable scatter: rank inside the block by (wave, lane) order among descriptors of the same
// owner (5 ballots match the owner byte, ROUTE_LOCAL included).
__global__ __launch_bounds__(NT) void k_route_scatter(uint32_t n, const RRec* __restrict__ tmp,
                                                       const uint8_t* __restrict__ own,
                                                       const uint32_t* __restrict__ boff, RRec* __restrict__ send,
                                                       uint32_t* __restrict__ perm) {
  constexpr int W = NT / 64;
  __shared__ uint32_t s_wc[W][NS + 1];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = blockIdx.x * NT + tid;
  for (uint32_t k = tid; k < W * (NS + 1); k += NT) (&s_wc[0][0])[k] = 0;
  __syncthreads();
  const uint32_t o = i < n ? own[i] : ROUTE_LOCAL;
  const uint32_t d = o == ROUTE_LOCAL ? (uint32_t)NS : o;  // 0..16
  uint64_t m = ~0ull;
#pragma unroll
  for (int bt = 0; bt < 5; ++bt) {
    const bool bit = (d >> bt) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
  if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_wc[w][d] = (uint32_t)__popcll(m);
  __syncthreads();
  if (i >= n) return;
  if (d == (uint32_t)NS) {
    perm[i] = RL_ROUTE_LOCAL;
    return;
  }
  uint32_t before = 0;
#pragma unroll
  for (int k = 0; k < W; ++k) before += (uint32_t)k < w ? s_wc[k][d] : 0u;
  const uint32_t pos = boff[blockIdx.x * NS + d] + before + rank;
  send[pos] = tmp[i];
  perm[i] = pos;
}

// One-pass pack into a strided send buffer (owner j's records at [j * stride, j * stride +
// count_j)): hash and owner as k_route_hash, ranks inside the block as k_route_scatter, and
// each block's offset per owner from a decoupled look-back over the blocks before it, so the
// records are written once, straight to their place (no tmp records, no scan launch). lb
// holds one word per (block, owner), block-major: each block's words in a line of their own
// (owner-major, 32 blocks share a line and their publishing stores from every XCD contend
// for it: 66 us per 10^6 descriptors against 32): flag in the top two bits (A = the block's own count, P =
// inclusive prefix), zeroed before the launch together with gerr. Workgroups are dispatched
// in blockIdx order, so every block looked at is resident or done; the spin is bounded all
// the same (ERR_SPIN -> RL_EDEVICE in the pairs). The last block writes the (count, status)
// pair of every owner. Every block ORs its error flags into gerr before it publishes, and the
// look-back acquires what the blocks before it released, so the last block's read of gerr
// sees every block's flags. The look-back words are self-contained (flag and value in one
// word), so they are read and written relaxed at agent scope: acquire loads and release
// stores would invalidate / write back the XCD's L2 on every block (738 us per 10^6
// descriptors measured with them, against the three-kernel pack's 42). The look-back is wave-wide (64 blocks per read): one lane walking
// back one block at a time took 2 ms per 10^6 descriptors.
constexpr uint32_t LB_A = 1u << 30, LB_P = 2u << 30, LB_V = (1u << 30) - 1u;
constexpr uint32_t LB_SPIN_LIMIT = 1u << 22;
// The look-back's bound (tests lower it: RL_DIAG_LB_SPIN_LIMIT, read by rl_create).
__device__ uint32_t g_lb_spin_limit = LB_SPIN_LIMIT;
constexpr int LB_U = 1;  // look-back words per lane per read (4: 52 us, every extra word a line)
// (Round 4: the words owner-major instead, lb[j * nb + k], so a read of 64 blocks is 256
// contiguous bytes, read one or four windows at a time: k_route_pack2 +7 / +17 us per 10^6
// descriptors — 32 blocks then publish into one line.)
__global__ __launch_bounds__(NT) void k_route_pack1(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                                     uint64_t seed, uint32_t origin, uint32_t n_shards, uint32_t stride,
                                                     RRec* __restrict__ send, uint32_t* __restrict__ perm,
                                                     uint32_t* lb, uint32_t* gerr, uint32_t* __restrict__ x) {
  constexpr int W = NT / 64;
  __shared__ uint32_t s_wc[W][NS + 1];
  __shared__ uint32_t s_base[NS];
  __shared__ uint32_t s_err;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = blockIdx.x * NT + tid;
  for (uint32_t k = tid; k < W * (NS + 1); k += NT) (&s_wc[0][0])[k] = 0;
  if (tid == 0) s_err = 0;
  __syncthreads();
  RRec r{};
  uint32_t o = ROUTE_LOCAL, err = 0;
  if (i < in.n_desc) {
    const uint32_t rule = in.rule[i], q = in.req_of[i], qp = in.req_of[i ? i - 1u : 0u];
    const uint32_t o0 = in.off[i], o1 = in.off[i + 1];
    if (o1 < o0 || o1 > in.blob_bytes || qp > q) err |= ERR_BAD_INPUT;
    const bool nil = rule == RL_NIL_RULE;
    if (!nil && !err && (rule >= n_rules || rule >= RREC_MAX_RULE || q >= in.n_req)) err |= ERR_BAD_INPUT;
    const uint32_t qc = q < in.n_req ? q : 0u;
    const uint32_t oc = err ? 0u : o0;
    const int64_t now = in.now[qc];
    const uint32_t ha = in.hits[qc];
    const u32x4* pw = reinterpret_cast<const u32x4*>(in.blob + (oc & ~3u));
    const u32x4 w0 = pw[0];
    const u32x4 w1 = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint32_t*>(pw) + 4);
    if (!nil && !err) {
      if (now < 0 || now > MAX_NOW) {
        err |= ERR_BAD_TIME;
      } else {
        const FpState fs = prefix_state_pre(w0, w1, in.blob, o0, o1 - o0, seed);
        r.a = fs.a;
        r.b = fs.b;
        r.now = (uint32_t)now;
        r.rule = rule | (desc_jit(in, i) << 16);  // the EXPIRE jitter travels with the record
        r.h = ha > 1u ? ha : 1u;  // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
        r.greq = (origin << ROUTE_REQ_BITS) | q;
        o = route_owner(fs.a, fs.b, n_shards);
      }
    }
  }
  const uint32_t d = o == ROUTE_LOCAL ? (uint32_t)NS : o;  // 0..16
  uint64_t m = ~0ull;
#pragma unroll
  for (int bt = 0; bt < 5; ++bt) {
    const bool bit = (d >> bt) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
  if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_wc[w][d] = (uint32_t)__popcll(m);
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  if (tid == 0 && s_err) {  // before any owner's word of this block is published
    atomicOr(gerr, s_err);
    __threadfence();
  }
  __syncthreads();
  // wave w publishes and looks back for owners w, w + W, ...: the wave reads the 64 blocks
  // before the window's end at once (LB_U per lane), stops at the nearest P (summing the A's before it) or
  // moves 64 blocks back when all are A; it waits only for blocks nearer than that P
  const uint32_t bi = blockIdx.x;
  for (uint32_t j = w; j < n_shards; j += W) {  // wave-uniform
    uint32_t agg = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) agg += s_wc[k][j];
    if (lane == 0)
      __hip_atomic_store(&lb[(size_t)bi * NS + j], (bi ? LB_A : LB_P) | agg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t excl = 0;
    if (bi) {
      int32_t end = (int32_t)bi - 1;
      uint32_t spun = 0;
      for (;;) {
        // lane l reads blocks end - LB_U l - u: distance t = LB_U l + u
        uint32_t v[LB_U];
#pragma unroll
        for (int u = 0; u < LB_U; ++u) {
          const int32_t k = end - (int32_t)(lane * LB_U + u);
          v[u] = k >= 0 ? __hip_atomic_load(&lb[(size_t)k * NS + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : LB_P;  // before block 0: an inclusive prefix of 0
        }
        uint32_t up = LB_U, un = LB_U;  // the lane's first P and first unpublished word
#pragma unroll
        for (int u = LB_U - 1; u >= 0; --u) {
          if ((v[u] >> 30) == 2u) up = u;
          if ((v[u] >> 30) == 0u) un = u;
        }
        const uint64_t pm = __ballot(up < LB_U);
        const uint32_t lp = pm ? (uint32_t)__ffsll((unsigned long long)pm) - 1u : 64u;  // lane of the first P
        // waiting: an unpublished word nearer than the first P
        const bool wait = lane < lp ? un < LB_U : lane == lp ? un < up : false;
        if (__ballot(wait)) {
          if (++spun > g_lb_spin_limit) {
            if (lane == 0) {
              atomicOr(gerr, (uint32_t)ERR_SPIN);
              __threadfence();  // the flag is visible before the (wrong) prefix below is published
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint32_t part = 0;
#pragma unroll
        for (int u = 0; u < LB_U; ++u)
          part += lane < lp || (lane == lp && (uint32_t)u <= up) ? v[u] & LB_V : 0u;
        excl += wave_sum_u32(part);
        if (pm) break;
        end -= 64 * LB_U;
      }
      if (lane == 0)
        __hip_atomic_store(&lb[(size_t)bi * NS + j], LB_P | ((excl + agg) & LB_V), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_base[j] = excl;
      if (bi == gridDim.x - 1u) x[2 * j] = excl + agg;  // the last block: every owner's total
    }
  }
  __syncthreads();
  // The last block writes the batch's status into every owner's pair, from ONE read of gerr
  // after all of its look-backs: every rank then receives the same status from this origin and
  // all of them take the same exit (rl_router.cpp). Every block ORed its flags (and a timed-out
  // look-back its ERR_SPIN) into gerr before publishing the words this block has read.
  if (bi == gridDim.x - 1u && tid == 0) {
    __threadfence();
    const uint32_t e = __hip_atomic_load(gerr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t status = e & ERR_SPIN ? (uint32_t)RL_EDEVICE
                            : e & (ERR_BAD_INPUT | ERR_BAD_TIME) ? (uint32_t)RL_EINVAL : 0u;
    for (uint32_t j = 0; j < n_shards; ++j) x[2 * j + 1] = status;
  }
  if (i >= in.n_desc) return;
  if (d == (uint32_t)NS) {
    perm[i] = RL_ROUTE_LOCAL;
    return;
  }
  uint32_t before = 0;
#pragma unroll
  for (int k = 0; k < W; ++k) before += (uint32_t)k < w ? s_wc[k][d] : 0u;
  const uint32_t pos = d * stride + s_base[d] + before + rank;
  send[pos] = r;
  perm[i] = pos;
}

__global__ __launch_bounds__(NT) void k_route_reply(uint32_t n, const rl_status* __restrict__ out,
                                                     const uint32_t* __restrict__ thr, RReply* __restrict__ reply) {
  const uint32_t i = blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  RReply r;
  r.st = out[i];
  r.thr = thr[i];
  reply[i] = r;
}

__global__ __launch_bounds__(NT) void k_route_unpack(uint32_t n, const uint32_t* __restrict__ req_of,
                                                      const uint32_t* __restrict__ perm,
                                                      const RReply* __restrict__ reply, rl_status* __restrict__ out,
                                                      uint32_t* __restrict__ req_thr) {
  const uint32_t i = blockIdx.x * NT + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = perm[i];
  if (p == RL_ROUTE_LOCAL) {
    // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
    rl_status st;
    st.code_flags = RL_CODE_OK;
    st.limit_remaining = 0;
    st.reset_s = 0;
    st.over_limit_delta = 0;
    st.near_limit_delta = 0;
    out[i] = st;
    return;
  }
  const RReply r = reply[p];
  out[i] = r.st;
  // DoLimitResponse.ThrottleMillis = max over the request's descriptors  base_limiter.go:163-165
  if (r.thr) atomicMax(&req_thr[req_of[i]], r.thr);
}


// ---------------------------------------------------------------------------------------------
// Combining router (rl_router.cpp). Under a skewed key distribution the hottest
// keys arrive from every origin at their one owner (Zipf 1.1: the top 256 prefixes are about
// half of all descriptors), so per-descriptor records overload that owner. An origin combines
// its descriptors of a hot prefix into ONE record carrying their sum of hits_addend: a run of
// INCRBYs of one key string at one request time is one INCRBY of the sum (no EXPIRE can fall
// between them, and the local cache is off when combining is on). The owner answers every
// record with its raw INCRBY post-value (rl_raw_reply); the origin rebuilds each descriptor's
// post-value as (record post-value - record sum + the descriptor's inclusive prefix of h inside
// its group, in arrival order) and makes the decisions itself.
//
//   k_route_pack2     hash, owner, hot-set lookup (tags in LDS); cold descriptors ranked
//                     stably per owner (block ranks + decoupled look-back, as k_route_pack1)
//                     and written once to the strided send buffer; hot descriptors: per-block
//                     h sums per group and each descriptor's exclusive prefix inside its block
//   k_route_hot_scan  per group: exclusive prefix of the block sums over blocks, the group's
//                     total; the last block checks the batch (one request time over all hot
//                     descriptors, every hot descriptor with its entry's rule, sums in range)
//                     and appends one combined record per group to its owner's section, or
//                     asks for a repack without combining
//   k_route_pack2<repack>  the pack again without combining, only when asked (else it returns)
//   k_route_unpack_raw     origin: raw replies -> each descriptor's post-value -> decision
// ---------------------------------------------------------------------------------------------
constexpr int PR = 4;                   // descriptors per thread
constexpr int PBLK = NT * PR;           // per block
constexpr int PW = NT / 64;             // waves per block
constexpr int PV = PR * PW;             // virtual waves per block, (round, wave) in arrival order
static_assert(PBLK == (int)ROUTE2_BLOCK, "pack block");
constexpr uint32_t RF_MISMATCH = 1u, RF_OVERFLOW = 2u, RF_HOT = 4u;
constexpr uint32_t CAT_LOCAL = NS, CAT_HOT = NS + 1;
constexpr uint32_t HOT_PRE_MAX = (1u << PERM_HOT_PRE_BITS) - 1u;
constexpr uint32_t HOT_H_MAX = 4095u;   // a combined descriptor's h: 1024 x 4095 < 2^22
static_assert(HOT_MAX <= 256, "hot group index in 8 perm bits");

RL_DEV uint32_t route_hot_lookup(const uint32_t* s_tags, const HotEntry* __restrict__ ent, uint64_t a, uint64_t b,
                                 uint32_t& rule) {
  const uint32_t t = hot_tag(a);
  uint32_t s = hot_home(a);
  for (int probe = 0; probe < HOT_TAGS; ++probe) {
    const uint32_t w = s_tags[s];
    if (w == 0u) return 0xFFFFFFFFu;
    if ((w & HOT_TAG_MASK) == t) {
      const HotEntry e = ent[(w & ~HOT_TAG_MASK) - 1u];
      if (e.a == a && e.b == b) {
        rule = e.rule;
        return e.idx;
      }
    }
    s = (s + 1) & (HOT_TAGS - 1);
  }
  return 0xFFFFFFFFu;
}

// Decoupled look-back of one owner's count over the blocks before this one (k_route_pack1's,
// run by one wave): returns the exclusive prefix and publishes the inclusive one.
RL_DEV uint32_t lookback_owner(uint32_t* lb, uint32_t* gerr, uint32_t bi, uint32_t j, uint32_t agg) {
  const uint32_t lane = threadIdx.x & 63;
  if (lane == 0)
    __hip_atomic_store(&lb[(size_t)bi * NS + j], (bi ? LB_A : LB_P) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t excl = 0;
  if (bi) {
    int32_t end = (int32_t)bi - 1;
    uint32_t spun = 0;
    for (;;) {
      const int32_t k = end - (int32_t)lane;
      const uint32_t v = k >= 0 ? __hip_atomic_load(&lb[(size_t)k * NS + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : LB_P;
      const uint64_t pm = __ballot((v >> 30) == 2u);
      const uint32_t lp = pm ? (uint32_t)__ffsll((unsigned long long)pm) - 1u : 64u;
      const bool wait = lane <= lp && lane < 64u && (v >> 30) == 0u;
      if (__ballot(wait)) {
        if (++spun > g_lb_spin_limit) {
          if (lane == 0) {
            atomicOr(gerr, (uint32_t)ERR_SPIN);
            __threadfence();
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += wave_sum_u32(lane <= lp ? v & LB_V : 0u);
      if (pm) break;
      end -= 64;
    }
    if (lane == 0)
      __hip_atomic_store(&lb[(size_t)bi * NS + j], LB_P | ((excl + agg) & LB_V), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  return excl;
}

template <bool COMBINE, bool REPACK>
__global__ __launch_bounds__(NT) void k_route_pack2(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                                     uint64_t seed, uint32_t origin, uint32_t n_shards, uint32_t stride,
                                                     const HotEntry* __restrict__ hot, RRec* __restrict__ send,
                                                     uint32_t* __restrict__ perm, uint32_t* lb, uint32_t* gerr,
                                                     uint32_t* __restrict__ x, uint32_t* __restrict__ bhs,
                                                     uint32_t* __restrict__ bstat, const uint32_t* __restrict__ rctl,
                                                     uint32_t* __restrict__ req_thr, uint32_t xs, uint32_t* tr) {
  __shared__ uint32_t s_wc[PR][PW][NS + 2];
  __shared__ uint32_t s_tot[NS], s_base[NS];
  __shared__ uint32_t s_err;
  __shared__ uint32_t s_tags[COMBINE ? HOT_TAGS : 1];
  __shared__ uint32_t s_hw[COMBINE ? PV : 1][COMBINE ? HOT_MAX : 1];
  __shared__ uint32_t s_st[3];  // the block's hot descriptors: ~min now, max now, RF_* flags
  __shared__ uint32_t s_tr[2];  // the block's routed descriptors: ~min now, max now + 1 (0: none)
  if (REPACK && rctl[0] == 0u) return;  // combining was accepted: nothing to redo
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, bi = blockIdx.x;
  if (!REPACK && req_thr)  // ThrottleMillis starts at 0 (k_route_unpack_raw takes the max per request)
    for (uint32_t q = bi * NT + tid; q < in.n_req; q += gridDim.x * NT) req_thr[q] = 0u;
  for (uint32_t k = tid; k < PR * PW * (NS + 2); k += NT) (&s_wc[0][0][0])[k] = 0;
  if constexpr (COMBINE) {
    const uint32_t* tg = reinterpret_cast<const uint32_t*>(hot);
    for (uint32_t k = tid; k < (uint32_t)HOT_TAGS; k += NT) s_tags[k] = tg[k];
    for (uint32_t k = tid; k < (uint32_t)(PV * HOT_MAX); k += NT) (&s_hw[0][0])[k] = 0;
  }
  if (tid == 0) s_err = 0;
  if (tid < 3) s_st[tid] = 0;
  if (tid < 2) s_tr[tid] = 0;
  __syncthreads();
  const uint32_t i0 = bi * PBLK, last = in.n_desc - 1u;  // n_desc >= 1, n_req >= 1 (host-checked)
  // two levels of loads, each issued together at clamped indices (k_route_pack1)
  uint32_t rl[PR], q[PR], qp[PR], oa[PR], ob[PR], jv[PR];
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    const uint32_t i = min(i0 + r * NT + tid, last);
    rl[r] = in.rule[i];
    q[r] = in.req_of[i];
    qp[r] = in.req_of[i ? i - 1u : 0u];
    oa[r] = in.off[i];
    ob[r] = in.off[i + 1u];
    jv[r] = desc_jit(in, i);  // (kernel-uniform test: no load without jitter; combining is off with it)
  }
  bool okv[PR];
  int64_t nowv[PR];
  uint32_t hav[PR];
  u32x4 w0[PR], w1[PR];
  uint32_t err = 0;
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    const bool v = i0 + r * NT + tid < in.n_desc;
    const bool lay = oa[r] <= ob[r] && ob[r] <= in.blob_bytes && qp[r] <= q[r];
    const bool nil = rl[r] == RL_NIL_RULE, q_ok = q[r] < in.n_req;
    const bool rule_ok = rl[r] < n_rules && rl[r] < RREC_MAX_RULE;  // (the record's rule word carries the jitter)
    if (v && (!lay || (!nil && (!rule_ok || !q_ok)))) err |= ERR_BAD_INPUT;
    okv[r] = v && !nil && lay && rule_ok && q_ok;
    const uint32_t qc = q_ok ? q[r] : 0u;
    nowv[r] = in.now[qc];
    hav[r] = in.hits[qc];
    const u32x4* pw = reinterpret_cast<const u32x4*>(in.blob + ((okv[r] ? oa[r] : 0u) & ~3u));
    w0[r] = pw[0];
    w1[r] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint32_t*>(pw) + 4);
  }
  RRec rec[PR];
  uint32_t cat[PR], hix[PR], stf = 0;
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    cat[r] = CAT_LOCAL;
    hix[r] = 0;
    rec[r].a = rec[r].b = 0;
    rec[r].now = rec[r].rule = rec[r].h = rec[r].greq = 0;
    if (!okv[r]) continue;
    if (nowv[r] < 0 || nowv[r] > MAX_NOW) {
      err |= ERR_BAD_TIME;
      continue;
    }
    const FpState fs = prefix_state_pre(w0[r], w1[r], in.blob, oa[r], ob[r] - oa[r], seed);
    rec[r].a = fs.a;
    rec[r].b = fs.b;
    rec[r].now = (uint32_t)nowv[r];
    rec[r].rule = rl[r] | (jv[r] << 16);
    rec[r].h = hav[r] > 1u ? hav[r] : 1u;  // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
    rec[r].greq = (origin << ROUTE_REQ_BITS) | q[r];
    cat[r] = route_owner(fs.a, fs.b, n_shards);
    if constexpr (COMBINE) {
      uint32_t hr = 0;
      const uint32_t hx = route_hot_lookup(s_tags, hot + HOT_SLOTS, fs.a, fs.b, hr);
      if (hx != 0xFFFFFFFFu) {
        cat[r] = CAT_HOT;
        hix[r] = hx;
        // the group is one key string only if every descriptor has the entry's rule
        if (hr != rl[r]) stf |= RF_MISMATCH;
        if (rec[r].h > HOT_H_MAX) stf |= RF_OVERFLOW;
      }
    }
  }
  // stable ranks per owner: (round, wave, lane) is arrival order inside the block
  const uint64_t lt = lanemask_lt();
  uint32_t rank[PR];
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int bt = 0; bt < 5; ++bt) {
      const bool bit = (cat[r] >> bt) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    rank[r] = (uint32_t)__popcll(m & lt);
    if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_wc[r][w][cat[r]] = (uint32_t)__popcll(m);
  }
  uint32_t hex[PR];  // hot: exclusive prefix of h among the wave's descriptors of the same group
#pragma unroll
  for (int r = 0; r < PR; ++r) hex[r] = 0;
  if constexpr (COMBINE) {
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
#pragma unroll
    for (int r = 0; r < PR; ++r) {
      const bool ht = cat[r] == CAT_HOT;
      uint64_t todo = __ballot(ht);
      if (todo && __ballot(ht && rec[r].h != 1u) == 0ull) {
        // every hot h of the wave's round is 1 (hits_addend 0 or 1, the common case): a lane's
        // exclusive prefix is the number of its group's lanes below it. The group's lanes by
        // a match on the 8 group-index bits, no loop over the wave's groups.
        uint64_t m = todo;
#pragma unroll
        for (int bt = 0; bt < 8; ++bt) {
          const bool bit = (hix[r] >> bt) & 1u;
          const uint64_t bal = __ballot(bit);
          m &= bit ? bal : ~bal;
        }
        if (ht) {
          hex[r] = (uint32_t)__popcll(m & lt);
          if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_hw[r * PW + w][hix[r]] = (uint32_t)__popcll(m);
        }
        todo = 0;
      }
      while (todo) {  // one group of the wave per iteration (wave-uniform)
        const uint32_t ld = (uint32_t)__ffsll((unsigned long long)todo) - 1u;
        const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)hix[r], (int)ld);
        const bool mine = cat[r] == CAT_HOT && hix[r] == hl;
        const uint64_t m = __ballot(mine);
        const uint32_t v = mine ? rec[r].h : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        if (mine) hex[r] = incl - v;
        if (lane == ld) s_hw[r * PW + w][hl] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        todo &= ~m;
      }
      if (cat[r] == CAT_HOT) {
        mn = min(mn, rec[r].now);
        mx = max(mx, rec[r].now);
      }
    }
    if (__ballot(mx != 0u || mn != 0xFFFFFFFFu)) {  // the wave has hot descriptors (wave-uniform)
      mn = wave_min_u32(mn);
      mx = wave_max_u32(mx);
      if (lane == 0) {
        atomicMax(&s_st[0], ~mn);
        atomicMax(&s_st[1], mx);
        atomicOr(&s_st[2], RF_HOT);
      }
    }
    if (stf) atomicOr(&s_st[2], stf);
  }
  if (err) atomicOr(&s_err, err);
  if (!REPACK) {  // the batch's request-time range (every owner learns it in the counts exchange)
    uint32_t tmn = 0xFFFFFFFFu, tmx = 0;
#pragma unroll
    for (int r = 0; r < PR; ++r)
      if (cat[r] != CAT_LOCAL) {
        tmn = min(tmn, rec[r].now);
        tmx = max(tmx, rec[r].now);
      }
    tmn = wave_min_u32(tmn);
    tmx = wave_max_u32(tmx);
    if (lane == 0 && tmn <= tmx) {
      atomicMax(&s_tr[0], ~tmn);
      atomicMax(&s_tr[1], tmx + 1u);
    }
  }
  __syncthreads();
  if (tid < NS) {  // per owner: exclusive offsets of the (round, wave) runs, block total
    uint32_t run = 0;
#pragma unroll
    for (int r = 0; r < PR; ++r)
#pragma unroll
      for (int v = 0; v < PW; ++v) {
        const uint32_t c = s_wc[r][v][tid];
        s_wc[r][v][tid] = run;
        run += c;
      }
    s_tot[tid] = run;
  }
  if constexpr (COMBINE) {
    for (uint32_t hl = tid; hl < (uint32_t)HOT_MAX; hl += NT) {
      uint32_t t = 0;
#pragma unroll
      for (int v = 0; v < PV; ++v) t += s_hw[v][hl];
      bhs[(size_t)bi * HOT_MAX + hl] = t;
      if (t > HOT_PRE_MAX) atomicOr(&s_st[2], RF_OVERFLOW);
    }
  }
  __syncthreads();
  if (tid == 0 && s_err) {  // before any owner's word of this block is published
    atomicOr(gerr, s_err);
    __threadfence();
  }
  if (!REPACK && tid == 0 && s_tr[0]) {
    // into one of 8 lines (fewer same-line atomics in a row); returning atomics, their values
    // consumed: performed before this thread publishes owner 0's look-back word below, so the
    // last block, whose look-back transitively saw every block's word, reads every block's range
    uint32_t* tw = tr + (size_t)(bi & 7u) * 64u;
    const uint32_t pa = __hip_atomic_fetch_max(&tw[0], s_tr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t pb = __hip_atomic_fetch_max(&tw[1], s_tr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::"v"(pa), "v"(pb));
  }
  if (COMBINE && tid < 3) bstat[(size_t)bi * 4 + tid] = s_st[tid];
  __syncthreads();
  for (uint32_t j = w; j < n_shards; j += PW) {  // wave-uniform
    const uint32_t excl = lookback_owner(lb, gerr, bi, j, s_tot[j]);
    if (lane == 0) {
      s_base[j] = excl;
      if (bi == gridDim.x - 1u) x[xs * j] = excl + s_tot[j];  // the last block: every owner's cold total
    }
  }
  __syncthreads();
  if (bi == gridDim.x - 1u && tid == 0) {  // one status for every owner (k_route_pack1)
    __threadfence();
    const uint32_t e = __hip_atomic_load(gerr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t status = e & ERR_SPIN ? (uint32_t)RL_EDEVICE
                            : e & (ERR_BAD_INPUT | ERR_BAD_TIME) ? (uint32_t)RL_EINVAL : 0u;
    for (uint32_t j = 0; j < n_shards; ++j) x[xs * j + 1] = status;
    // the decide statuses this rank will send in the reply exchange start as a failure word
    // (after the counts words sent and received: rl_router.cpp's step words)
    if (!REPACK)
      for (uint32_t j = 0; j < n_shards; ++j) x[2u * xs * n_shards + j] = (uint32_t)RL_EHIP;
    if (!REPACK && xs >= 4u) {  // (tmin, tmax) of the batch's routed descriptors to every owner
      uint32_t mn = 0, mx = 0;
      for (uint32_t l = 0; l < 8u; ++l) {
        mn = max(mn, __hip_atomic_fetch_or(&tr[l * 64u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        mx = max(mx, __hip_atomic_fetch_or(&tr[l * 64u + 1u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      for (uint32_t j = 0; j < n_shards; ++j) {
        x[xs * j + 2] = mn ? ~mn : 0xFFFFFFFFu;
        x[xs * j + 3] = mx ? mx - 1u : 0u;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    const uint32_t i = i0 + r * NT + tid;
    if (i >= in.n_desc) continue;
    if (cat[r] == CAT_LOCAL) {
      perm[i] = RL_ROUTE_LOCAL;
    } else if (COMBINE && cat[r] == CAT_HOT) {
      uint32_t pre = hex[r];
      const uint32_t v0 = (uint32_t)(r * PW) + w;
      for (uint32_t v = 0; v < v0; ++v) pre += s_hw[v][hix[r]];
      perm[i] = PERM_HOT | (hix[r] << PERM_HOT_PRE_BITS) | (pre & HOT_PRE_MAX);
    } else {
      const uint32_t d = cat[r];
      const uint32_t pos = d * stride + s_base[d] + s_wc[r][w][d] + rank[r];
      send[pos] = rec[r];
      perm[i] = pos;
    }
  }
}

// Hot scan: the per-(block, group) sums of k_route_pack2 -> exclusive prefixes over blocks (in
// place) and each group's total; then the last block's verdict and the combined records.
// Grid: HS_CC column chunks of 64 groups (lane = group) x HS_RCH row chunks (the pack blocks,
// split in 16); each wave loads up to HS_Q rows of its chunk into registers (one coalesced
// 256-B row segment per load), the chunk's column sums go out through a decoupled look-back
// over the row chunks before it (64-bit words, flag in bit 63), and the prefixes are written
// from the registers. At 1024 threads x 16 columns the kernel spilled 76 VGPRs and took 32 us
// per 10^6 descriptors; at 256 x 16 (two passes over the rows) 14.8 us.
constexpr int HS_NT = 256, HS_W = HS_NT / 64, HS_CC = HOT_MAX / 64, HS_RCH = 16, HS_Q = 16;
static_assert(HOT_MAX % 64 == 0 && HS_NT == HOT_MAX, "hot scan geometry: one last-block thread per group");
constexpr unsigned long long HLB_FLAG = 1ull << 63;
// h_out (pinned host words, written through): [0, HOT_MAX) each group's sum of h this step
// (0 for a group without descriptors), [HOT_MAX] 1 = the batch needs the repack, [HOT_MAX + 1]
// 1 = combining applied — read by the host after the step's counts, with no copy.
// hlb: [HS_RCH][HOT_MAX] look-back words, zero before the launch.
__global__ __launch_bounds__(HS_NT) void k_route_hot_scan(uint32_t nb, uint32_t n_shards, uint32_t origin,
                                                           uint32_t stride, const HotEntry* __restrict__ hot,
                                                           uint32_t* __restrict__ bhs, const uint32_t* bstat,
                                                           RRec* __restrict__ send, uint32_t* x, uint32_t* rctl,
                                                           uint32_t* __restrict__ hot_pos,
                                                           uint32_t* __restrict__ hot_tot,
                                                           unsigned long long* tot64, uint32_t* gerr,
                                                           uint32_t* h_out, unsigned long long* hlb, uint32_t xs) {
  __shared__ unsigned long long s_w[HS_W][64];
  __shared__ uint32_t s_last, s_mn, s_mx, s_fl, s_bad;
  __shared__ uint32_t s_oc[4][NS + 1];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t cc = blockIdx.x % HS_CC, rc = blockIdx.x / HS_CC;
  const uint32_t col = cc * 64 + lane;
  const uint32_t R = (nb + HS_RCH - 1) / HS_RCH;             // rows per chunk
  const uint32_t RW = (R + HS_W - 1) / HS_W;                 // rows per wave
  const uint32_t r0 = min(nb, rc * R + wv * RW), r1 = min(min(nb, rc * R + R), r0 + RW);
  const bool in_regs = RW <= (uint32_t)HS_Q;                 // grid-uniform
  uint32_t v[HS_Q];
  unsigned long long sum = 0;
  if (in_regs) {
#pragma unroll
    for (int u = 0; u < HS_Q; ++u) v[u] = r0 + u < r1 ? bhs[(size_t)(r0 + u) * HOT_MAX + col] : 0u;
#pragma unroll
    for (int u = 0; u < HS_Q; ++u) sum += v[u];
  } else {
#pragma unroll 1
    for (uint32_t rr = r0; rr < r1; rr += HS_Q) {
#pragma unroll
      for (int u = 0; u < HS_Q; ++u) v[u] = bhs[(size_t)min(rr + u, r1 - 1u) * HOT_MAX + col];
#pragma unroll
      for (int u = 0; u < HS_Q; ++u) sum += rr + u < r1 ? v[u] : 0u;
    }
  }
  s_w[wv][lane] = sum;
  __syncthreads();
  if (wv == 0) {  // the chunk's column sums: publish, then look back over the chunks before it
    unsigned long long agg = 0;
#pragma unroll
    for (int k = 0; k < HS_W; ++k) agg += s_w[k][lane];
    __hip_atomic_store(&hlb[(size_t)rc * HOT_MAX + col], HLB_FLAG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every earlier chunk's word loaded at once (one memory round trip per poll, not one per
    // chunk: the chunks publish their sums right away, so the first poll usually finds them all)
    unsigned long long ex = 0;
    uint32_t spun = 0;
    uint32_t pending = (1u << rc) - 1u;  // rc < HS_RCH <= 16
    while (pending) {
      unsigned long long wv[HS_RCH];
#pragma unroll
      for (int k = 0; k < HS_RCH; ++k)
        wv[k] = __hip_atomic_load(&hlb[(size_t)min((uint32_t)k, rc) * HOT_MAX + col], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < HS_RCH; ++k)
        if (((pending >> k) & 1u) && (wv[k] & HLB_FLAG)) {
          ex += wv[k] & ~HLB_FLAG;
          pending &= ~(1u << k);
        }
      if (__ballot(pending != 0u) == 0ull) break;
      if (++spun > g_lb_spin_limit) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (__ballot(spun > g_lb_spin_limit) && lane == 0) {
      atomicOr(gerr, (uint32_t)ERR_SPIN);
      __threadfence();
    }
    if (rc == HS_RCH - 1u) tot64[col] = ex + agg;
    unsigned long long run = ex;  // (wave 0 alone reads and rewrites s_w; the others wait below)
#pragma unroll
    for (int k = 0; k < HS_W; ++k) {  // each wave's first row: the chunks before + the waves before
      const unsigned long long y = s_w[k][lane];
      s_w[k][lane] = run;
      run += y;
    }
  }
  __syncthreads();
  {
    unsigned long long run = s_w[wv][lane];
    if (in_regs) {
#pragma unroll
      for (int u = 0; u < HS_Q; ++u)
        if (r0 + u < r1) {
          bhs[(size_t)(r0 + u) * HOT_MAX + col] = (uint32_t)run;
          run += v[u];
        }
    } else {
#pragma unroll 1
      for (uint32_t rr = r0; rr < r1; rr += HS_Q) {  // the same rows again (L2)
#pragma unroll
        for (int u = 0; u < HS_Q; ++u) v[u] = bhs[(size_t)min(rr + u, r1 - 1u) * HOT_MAX + col];
#pragma unroll
        for (int u = 0; u < HS_Q; ++u)
          if (rr + u < r1) {
            bhs[(size_t)(rr + u) * HOT_MAX + col] = (uint32_t)run;
            run += v[u];
          }
      }
    }
  }
  // hand-off to the last block (MI355X_MICROARCH.md, inter-workgroup visibility): every storing
  // wave drains, barrier, one lane's release + counter; the last arriver's lane acquires
  drain_vmem();
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    s_last = atomicAdd(&rctl[2], 1u) == gridDim.x - 1u;
    if (s_last) __threadfence();
  }
  __syncthreads();
  if (!s_last) return;
  // the last block: the batch's verdict, then one combined record per group
  if (tid == 0) {
    s_mn = 0;
    s_mx = 0;
    s_fl = 0;
    s_bad = 0;
  }
  if (tid < 4 * (NS + 1)) (&s_oc[0][0])[tid] = 0;
  __syncthreads();
  {
    uint32_t mn = 0, mx = 0, fl = 0;
    for (uint32_t b = tid; b < nb; b += HS_NT) {
      mn = max(mn, bstat[(size_t)b * 4]);
      mx = max(mx, bstat[(size_t)b * 4 + 1]);
      fl |= bstat[(size_t)b * 4 + 2];
    }
    mn = wave_max_u32(mn);
    mx = wave_max_u32(mx);
    fl = wave_or_u32(fl);
    if ((tid & 63) == 0) {
      atomicMax(&s_mn, mn);
      atomicMax(&s_mx, mx);
      atomicOr(&s_fl, fl);
    }
  }
  unsigned long long t = 0;
  HotEntry e{};
  if (tid < (uint32_t)HOT_MAX) {
    t = tot64[tid];
    e = hot[HOT_SLOTS + tid];
    if (t >= (1ull << 32)) atomicOr(&s_bad, 1u);
  }
  __syncthreads();
  const uint32_t fl = s_fl, now_min = ~s_mn, now_max = s_mx;
  const uint32_t ge = __hip_atomic_load(gerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool refused = ge != 0u;  // the batch is refused: nothing to add
  if (refused && tid < n_shards)  // (the pack's status, or this kernel's look-back spin expiry)
    x[xs * tid + 1] = ge & ERR_SPIN ? (uint32_t)RL_EDEVICE : (uint32_t)RL_EINVAL;
  const bool ok = !s_bad && !(fl & (RF_MISMATCH | RF_OVERFLOW)) && (!(fl & RF_HOT) || now_min == now_max);
  h_out[tid] = ok && !refused ? (uint32_t)t : 0u;
  if (tid == 0) {
    h_out[HOT_MAX] = !refused && !ok ? 1u : 0u;
    h_out[HOT_MAX + 1] = !refused && ok ? 1u : 0u;
  }
  if (refused || !ok) {
    if (tid == 0 && !refused) rctl[0] = 1u;  // k_route_pack2<repack> redoes the batch without combining
    __threadfence_system();
    return;
  }
  // rank of each non-empty group among its owner's groups (index order), per wave then over waves
  const uint32_t w = wv;
  const bool act = tid < (uint32_t)HOT_MAX && t > 0;
  const uint32_t o = act ? route_owner(e.a, e.b, n_shards) : (uint32_t)NS;
  uint32_t rank = 0;
  if (tid < (uint32_t)HOT_MAX) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int bt = 0; bt < 5; ++bt) {
      const bool bit = (o >> bt) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    rank = (uint32_t)__popcll(m & lanemask_lt());
    if (lane == (uint32_t)__ffsll((unsigned long long)m) - 1u) s_oc[w][o] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  uint32_t before = 0, cnt = 0;
  if (act) {
    for (uint32_t k = 0; k < 4; ++k) before += k < w ? s_oc[k][o] : 0u;
    const uint32_t pos = o * stride + x[xs * o] + before + rank;
    RRec r;
    r.a = e.a;
    r.b = e.b;
    r.now = now_min;
    r.rule = e.rule;
    r.h = (uint32_t)t;
    r.greq = origin << ROUTE_REQ_BITS;
    send[pos] = r;
    hot_pos[tid] = pos;
    hot_tot[tid] = (uint32_t)t;
  }
  if (tid < NS) {
    for (uint32_t k = 0; k < 4; ++k) cnt += s_oc[k][tid];
  }
  __syncthreads();  // every group read x[] above
  if (tid < n_shards) x[xs * tid] += cnt;
  if (tid == 0) rctl[1] = 1u;  // combining applied
  __threadfence_system();
}

// Origin: every descriptor's decision from its owner's raw reply.
// owner_status[j] != 0: owner j refused its records (nothing applied for them): their
// descriptors get code RL_CODE_UNKNOWN, so a caller can answer every other descriptor.
__global__ __launch_bounds__(NT) void k_route_unpack_raw(DevBatch in, const DevRule* __restrict__ rules,
                                                          const uint32_t* __restrict__ perm,
                                                          const RawReply* __restrict__ back,
                                                          const uint32_t* __restrict__ boff,
                                                          const uint32_t* __restrict__ hot_pos,
                                                          const uint32_t* __restrict__ hot_tot,
                                                          const int32_t* __restrict__ owner_status, uint32_t stride,
                                                          rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                                          uint32_t* __restrict__ zero, uint32_t zero_words,
                                                          int32_t* h_status, uint32_t n_shards) {
  const uint32_t i = blockIdx.x * NT + threadIdx.x;
  if (h_status && i < n_shards) {  // every owner's decide status into the pinned step words (no copy)
    h_status[i] = owner_status[i];
    __threadfence_system();
  }
  // the slot's look-back words and step words, cleared for its next step (the pack of step
  // k + 2 runs behind this kernel on the same stream): no memset between steps
  for (uint32_t k = i; k < zero_words; k += gridDim.x * NT) zero[k] = 0u;
  const bool valid = i < in.n_desc;
  uint32_t thr = 0, q = 0xFFFFFFFFu;
  if (valid) {
    rl_status st;
    st.limit_remaining = 0;
    st.reset_s = 0;
    st.over_limit_delta = 0;
    st.near_limit_delta = 0;
    const uint32_t p = perm[i];
    q = in.req_of[i];
    if (p == RL_ROUTE_LOCAL) {
      st.code_flags = RL_CODE_OK;  // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
    } else {
      const uint32_t rule = in.rule[i];
      const int64_t now = in.now[q];
      const uint32_t ha = in.hits[q];
      const uint32_t h = ha > 1u ? ha : 1u;  // utils.Max(1, request.HitsAddend)  fixed_cache_impl.go:39
      const DevRule R = rules[rule];
      const uint32_t hl = (p >> PERM_HOT_PRE_BITS) & (uint32_t)(HOT_MAX - 1);
      const uint32_t pos = (p & PERM_HOT) ? hot_pos[hl] : p;
      if (owner_status[pos / stride] != 0) {  // refused by its owner: undecided
        st.code_flags = RL_CODE_UNKNOWN;
      } else {
        const RawReply rr = back[pos];
        uint32_t after = rr.after;
        if (p & PERM_HOT) {
          // post-value of this descriptor's INCRBY inside its combined group: the group's reply
          // minus the group's sum plus the inclusive prefix of h up to this descriptor (arrival order)
          const uint32_t P = boff[(size_t)(i / PBLK) * HOT_MAX + hl] + (p & HOT_PRE_MAX) + h;
          after = after - hot_tot[hl] + P;
        }
        const uint32_t now_mod = (uint32_t)now % R.div;  // now - (now / div) * div
        thr = decide_status(after, (rr.flags & RAW_LOCAL_HIT) != 0u, h, now_mod, R, st);
      }
    }
    out[i] = st;
  }
  // DoLimitResponse.ThrottleMillis = max over the request's descriptors  base_limiter.go:163-165.
  // A request's descriptors are consecutive (req_of nondecreasing, checked by the pack): a
  // segmented max over the wave, then one store per request — a plain store when the request
  // lies inside the wave, an atomicMax on the pack's zero when it crosses the wave's edge.
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t qo = (uint32_t)__shfl_up((int)q, d, 64);
    const uint32_t to = (uint32_t)__shfl_up((int)thr, d, 64);
    if (lane >= (uint32_t)d && qo == q) thr = max(thr, to);
  }
  const uint32_t qn = (uint32_t)__shfl_down((int)q, 1, 64);
  const uint32_t q0 = (uint32_t)__shfl((int)q, 0, 64);
  const bool seg_end = lane == 63u || qn != q;
  if (valid && seg_end && thr) {
    if (lane < 63u && q != q0) req_thr[q] = thr;  // every descriptor of the request is in this wave
    else atomicMax(&req_thr[q], thr);
  }
}

}  // namespace route

static uint32_t route_blocks(uint32_t n) { return n ? (n + route::NT - 1) / route::NT : 1; }
uint32_t route_bcnt_words(uint32_t n) { return route_blocks(n) * (route::NS + 1); }  // counts, then errors

// RL_ROUTER_FAULT=stall (tests): one wave holds the stream until the router raises the release
// word on abort, or 20 s of the 100-MHz real-time clock pass (every launch ends).
__global__ __launch_bounds__(64) void k_router_stall(const uint32_t* release) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
         __builtin_amdgcn_s_memrealtime() - t0 < 2000000000ull)
    __builtin_amdgcn_s_sleep(127);
}
void launch_router_stall(hipStream_t st, const uint32_t* release) {
  hipLaunchKernelGGL(k_router_stall, dim3(1), dim3(64), 0, st, release);
}

void launch_route_pack(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                       uint32_t origin, uint32_t n_shards, RRec* tmp, uint8_t* own, uint32_t* bcnt, RRec* send,
                       uint32_t* send_counts, uint32_t* perm, EngineCtl* ctl, uint32_t* x) {
  const uint32_t nb = route_blocks(b.n_desc);
  hipLaunchKernelGGL(route::k_route_hash, dim3(nb), dim3(route::NT), 0, st, make_dev_batch(b), rules, n_rules, seed,
                     origin, n_shards, tmp, own, bcnt, ctl);
  hipLaunchKernelGGL(route::k_route_scan, dim3(1), dim3(route::SCAN_NT), 0, st, bcnt, nb, n_shards, send_counts, ctl,
                     x);
  hipLaunchKernelGGL(route::k_route_scatter, dim3(nb), dim3(route::NT), 0, st, b.n_desc, tmp, own, bcnt, send,
                     perm);
}

void launch_route_pack_strided(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules,
                               uint64_t seed, uint32_t origin, uint32_t n_shards, uint32_t stride, RRec* send,
                               uint32_t* perm, uint32_t* lb, uint32_t* x) {
  const uint32_t nb = route_blocks(b.n_desc);  // lb: nb * NS look-back words + the error word, zeroed
  hipLaunchKernelGGL(route::k_route_pack1, dim3(nb), dim3(route::NT), 0, st, make_dev_batch(b), rules, n_rules, seed,
                     origin, n_shards, stride, send, perm, lb, lb + (size_t)nb * route::NS, x);
}

uint32_t route2_blocks(uint32_t n) { return n ? (n + ROUTE2_BLOCK - 1) / ROUTE2_BLOCK : 1; }
size_t route2_hot_lb_words() { return (size_t)route::HS_RCH * HOT_MAX * 2; }
size_t route2_lb_words(uint32_t n) { return ((size_t)route2_blocks(n) * route::NS + 1 + 63) / 64 * 64; }
size_t route2_bhs_words(uint32_t n) { return (size_t)route2_blocks(n) * HOT_MAX; }

void launch_route_pack2(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                        uint32_t origin, uint32_t n_shards, uint32_t stride, const HotEntry* hot,
                        const RoutePackBufs& o) {
  const uint32_t nb = route2_blocks(b.n_desc);
  const DevBatch in = make_dev_batch(b);
  const size_t area = route2_lb_words(b.n_desc);
  uint32_t* lb1 = o.lb;
  uint32_t* lb2 = o.lb + area;
  const size_t gw = (size_t)nb * route::NS;  // the error word follows the look-back words
  if (!hot) {
    hipLaunchKernelGGL((route::k_route_pack2<false, false>), dim3(nb), dim3(route::NT), 0, st, in, rules, n_rules, seed,
                       origin, n_shards, stride, hot, o.send, o.perm, lb1, lb1 + gw, o.x, o.bhs, o.bstat, o.rctl, o.thr,
                       o.xs, o.tr);
    return;
  }
  hipLaunchKernelGGL((route::k_route_pack2<true, false>), dim3(nb), dim3(route::NT), 0, st, in, rules, n_rules, seed,
                     origin, n_shards, stride, hot, o.send, o.perm, lb1, lb1 + gw, o.x, o.bhs, o.bstat, o.rctl, o.thr,
                     o.xs, o.tr);
  unsigned long long* hlb = reinterpret_cast<unsigned long long*>(o.rctl + 16);  // zeroed with the look-back areas
  hipLaunchKernelGGL(route::k_route_hot_scan, dim3(route::HS_CC * route::HS_RCH), dim3(route::HS_NT), 0, st, nb,
                     n_shards, origin, stride, hot, o.bhs, o.bstat, o.send, o.x, o.rctl, o.hot_pos, o.hot_tot,
                     hlb + (size_t)route::HS_RCH * HOT_MAX, lb1 + gw, o.h_hot, hlb, o.xs);
  hipLaunchKernelGGL((route::k_route_pack2<false, true>), dim3(nb), dim3(route::NT), 0, st, in, rules, n_rules, seed,
                     origin, n_shards, stride, hot, o.send, o.perm, lb2, lb2 + gw, o.x, o.bhs, o.bstat, o.rctl, nullptr,
                     o.xs, o.tr);
}

void launch_route_unpack_raw(hipStream_t st, const rl_batch& b, const DevRule* rules, const RoutePackBufs& o,
                             const RawReply* back, const int32_t* owner_status, uint32_t stride, rl_status* out,
                             uint32_t* thr, int32_t* h_status, uint32_t n_shards) {
  if (!b.n_desc) return;
  hipLaunchKernelGGL(route::k_route_unpack_raw, dim3(route_blocks(b.n_desc)), dim3(route::NT), 0, st, make_dev_batch(b),
                     rules, o.perm, back, o.bhs, o.hot_pos, o.hot_tot, owner_status, stride, out, thr, o.lb,
                     o.zero_words, h_status, n_shards);
}

hipError_t route_set_spin_limit(uint32_t v) {
  return hipMemcpyToSymbol(HIP_SYMBOL(route::g_lb_spin_limit), &v, sizeof v);
}

void launch_route_reply(hipStream_t st, uint32_t n, const rl_status* out, const uint32_t* thr, RReply* reply) {
  if (!n) return;
  hipLaunchKernelGGL(route::k_route_reply, dim3(route_blocks(n)), dim3(route::NT), 0, st, n, out, thr, reply);
}

void launch_route_unpack(hipStream_t st, uint32_t n, const uint32_t* req_of, const uint32_t* perm,
                         const RReply* reply, rl_status* out, uint32_t* req_thr) {
  if (!n) return;
  hipLaunchKernelGGL(route::k_route_unpack, dim3(route_blocks(n)), dim3(route::NT), 0, st, n, req_of, perm, reply,
                     out, req_thr);
}

}  // namespace rlhip
