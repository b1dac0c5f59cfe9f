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
  const uint32_t tid = threadIdx.x, i = blockIdx.x * NT + tid;
  if (tid < NS) s_cnt[tid] = 0;
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
    if (err) atomicOr(&ctl->err, err);
  }
  __syncthreads();
  if (tid < NS) bcnt[blockIdx.x * NS + tid] = s_cnt[tid];
}

// One block: wave w < n_shards scans column w over the blocks (exclusive, in place), then
// owner totals are scanned into owner offsets and added to every entry.
__global__ __launch_bounds__(SCAN_NT) void k_route_scan(uint32_t* __restrict__ bcnt, uint32_t nb, uint32_t n_shards,
                                                        uint32_t* __restrict__ send_counts) {
  __shared__ uint32_t s_tot[NS], s_off[NS];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (w < n_shards) {
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
      const uint32_t b = b0 + lane;
      const uint32_t v = b < nb ? bcnt[b * NS + w] : 0u;
      uint32_t x = v;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t y = __shfl_up(x, s, 64);
        if (lane >= (uint32_t)s) x += y;
      }
      if (b < nb) bcnt[b * NS + w] = carry + x - v;
      carry += __shfl(x, 63, 64);
    }
    if (lane == 0) s_tot[w] = carry;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t s = 0; s < n_shards; ++s) {
      s_off[s] = acc;
      send_counts[s] = s_tot[s];
      acc += s_tot[s];
    }
  }
  __syncthreads();
  for (uint32_t k = tid; k < nb * NS; k += SCAN_NT) {
    const uint32_t s = k % NS;
    if (s < n_shards) bcnt[k] += s_off[s];
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
uint32_t route_bcnt_words(uint32_t n) { return route_blocks(n) * route::NS; }

void launch_route_pack(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                       uint32_t origin, uint32_t n_shards, RRec* tmp, uint8_t* own, uint32_t* bcnt, RRec* send,
                       uint32_t* send_counts, uint32_t* perm, EngineCtl* ctl) {
  const uint32_t nb = route_blocks(b.n_desc);
  hipLaunchKernelGGL(route::k_route_hash, dim3(nb), dim3(route::NT), 0, st, make_dev_batch(b), rules, n_rules, seed,
                     origin, n_shards, tmp, own, bcnt, ctl);
  hipLaunchKernelGGL(route::k_route_scan, dim3(1), dim3(route::SCAN_NT), 0, st, bcnt, nb, n_shards, send_counts);
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
