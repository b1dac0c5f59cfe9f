// rl_compact.hip — device side of the compact host wire format (rl_hip.h rl_batch_c).
//
// A compact batch crosses PCIe as the prefix bytes plus one word per descriptor (prefix
// length | rule id) and one per request (hits_addend | time delta); the request index of each
// descriptor only when requests hold several. These two kernels turn it into the rl_batch
// arrays every pipeline reads (prefix_off, rule_id, req_of, now, hits_addend), in HBM, on the
// copy-in stream right behind the H2D copies, so k4_hist sees an ordinary device batch.
//
//   k_c_sums    per 4096-descriptor chunk: the sum of its prefix lengths
//   k_c_expand  per chunk: its base offset (the sums of the chunks before it), an LDS scan of
//               its lengths -> prefix_off, rule ids widened (0xFFFF -> RL_NIL_RULE), req_of;
//               per request: now = now_base + delta, hits_addend = low 24 bits
//
// Both are streaming passes (≈ 12 B read + 24 B written per descriptor at one descriptor per
// request), hidden under the PCIe copies of the next batch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_device.h"

namespace rlhip {
namespace compact {

constexpr int NT = 256;
constexpr int PER = 16;            // descriptors per thread
constexpr int CHUNK = NT * PER;    // descriptors per block

struct CArgs {
  uint32_t n_desc, n_req, flags, pad;
  int64_t now_base;
  const uint32_t* dw;   // desc words
  const uint32_t* rw;   // req words
  const uint32_t* rq;   // req_of (or null)
  uint32_t* csum;       // per-chunk length sums
  uint32_t* off;        // n_desc + 1
  uint32_t* rule;
  uint32_t* req_of;
  int64_t* now;
  uint32_t* hits;
};

__global__ __launch_bounds__(NT) void k_c_sums(CArgs a) {
  const uint32_t c = blockIdx.x, tid = threadIdx.x;
  const uint32_t i0 = c * CHUNK;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = i0 + k * NT + tid;  // coalesced
    if (i < a.n_desc) s += a.dw[i] & 0xFFFFu;
  }
  s = wave_sum_u32(s);
  __shared__ uint32_t sh[NT / 64];
  if ((tid & 63) == 0) sh[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += sh[w];
    a.csum[c] = t;
  }
}

__global__ __launch_bounds__(NT) void k_c_expand(CArgs a) {
  const uint32_t c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ uint32_t sh_w[NT / 64];
  __shared__ uint32_t sh_base;
  // base offset of the chunk: the length sums of the chunks before it (blocks past the last
  // chunk only expand requests)
  const uint32_t nc = (a.n_desc + CHUNK - 1) / CHUNK;
  uint32_t b = 0;
  for (uint32_t k = tid; k < c && k < nc; k += NT) b += a.csum[k];
  b = wave_sum_u32(b);
  if (lane == 0) sh_w[wave] = b;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += sh_w[w];
    sh_base = t;
  }
  __syncthreads();
  // this thread's PER consecutive descriptors (a blocked layout for the scan; the loads of a
  // wave touch 64 x 64 B = 4 KB contiguous)
  const uint32_t i0 = c * CHUNK + tid * PER;
  uint32_t w[PER], len[PER], s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = i0 + k;
    w[k] = i < a.n_desc ? a.dw[i] : 0u;
    len[k] = w[k] & 0xFFFFu;
    s += len[k];
  }
  const uint32_t incl = wave_incl_scan_u32(s);
  __syncthreads();  // (sh_w reused)
  if (lane == 63) sh_w[wave] = incl;
  __syncthreads();
  uint32_t run = sh_base + incl - s;
#pragma unroll
  for (int w2 = 0; w2 < NT / 64; ++w2) run += (uint32_t)w2 < wave ? sh_w[w2] : 0u;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = i0 + k;
    if (i < a.n_desc) {
      a.off[i] = run;
      const uint32_t r16 = w[k] >> 16;
      a.rule[i] = r16 == 0xFFFFu ? RL_NIL_RULE : r16;
      a.req_of[i] = a.rq ? a.rq[i] : i;
      if (i + 1 == a.n_desc) a.off[i + 1] = run + len[k];
    }
    run += len[k];
  }
  // requests: a grid-stride pass (coalesced)
  for (uint32_t r = c * NT + tid; r < a.n_req; r += gridDim.x * NT) {
    const uint32_t x = a.rw[r];
    a.now[r] = a.now_base + (int64_t)(x >> 24);
    a.hits[r] = x & 0xFFFFFFu;
  }
}

}  // namespace compact

uint32_t compact_chunks(uint32_t n) { return (n + compact::CHUNK - 1) / compact::CHUNK; }

// Expand a compact batch (device copies of its words) into rl_batch arrays; csum holds
// compact_chunks(n_desc) words. An empty batch of requests still gets its now / hits.
void launch_compact_expand(hipStream_t st, uint32_t n_desc, uint32_t n_req, int64_t now_base, const uint32_t* dw,
                           const uint32_t* rw, const uint32_t* rq, uint32_t* csum, uint32_t* off, uint32_t* rule,
                           uint32_t* req_of, int64_t* now, uint32_t* hits) {
  compact::CArgs a;
  a.n_desc = n_desc;
  a.n_req = n_req;
  a.flags = 0;
  a.pad = 0;
  a.now_base = now_base;
  a.dw = dw;
  a.rw = rw;
  a.rq = rq;
  a.csum = csum;
  a.off = off;
  a.rule = rule;
  a.req_of = req_of;
  a.now = now;
  a.hits = hits;
  const uint32_t nc = compact_chunks(n_desc);
  const uint32_t nr = (n_req + compact::NT - 1) / compact::NT;
  const uint32_t grid = nc > nr ? nc : (nr > 0 ? nr : 1u);
  if (nc) hipLaunchKernelGGL(compact::k_c_sums, dim3(nc), dim3(compact::NT), 0, st, a);
  hipLaunchKernelGGL(compact::k_c_expand, dim3(grid), dim3(compact::NT), 0, st, a);
}

}  // namespace rlhip
