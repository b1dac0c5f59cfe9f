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
