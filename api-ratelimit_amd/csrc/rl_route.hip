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
#include "rl_device.h"

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
    if (!nil && !err && (rule >= n_rules || q >= in.n_req)) err |= ERR_BAD_INPUT;
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
        r.rule = rule;
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
constexpr int LB_U = 1;  // look-back words per lane per read (4: 52 us, every extra word a line)
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
    if (!nil && !err && (rule >= n_rules || q >= in.n_req)) err |= ERR_BAD_INPUT;
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
        r.rule = rule;
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
          if (++spun > LB_SPIN_LIMIT) {
            if (lane == 0) atomicOr(gerr, (uint32_t)ERR_SPIN);
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
      if (bi == gridDim.x - 1u) {  // the last block: every owner's total and the batch's status
        const uint32_t e = __hip_atomic_load(gerr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        x[2 * j] = excl + agg;
        x[2 * j + 1] = e & ERR_SPIN ? (uint32_t)RL_EDEVICE
                       : e & (ERR_BAD_INPUT | ERR_BAD_TIME) ? (uint32_t)RL_EINVAL : 0u;
      }
    }
  }
  __syncthreads();
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

}  // namespace route

static uint32_t route_blocks(uint32_t n) { return n ? (n + route::NT - 1) / route::NT : 1; }
uint32_t route_bcnt_words(uint32_t n) { return route_blocks(n) * (route::NS + 1); }  // counts, then errors

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
