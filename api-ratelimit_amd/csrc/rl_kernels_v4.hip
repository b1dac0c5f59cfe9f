// rl_kernels_v4.hip — the default decision pipeline: four launches per batch.
//
// Same contract and outputs as the LSD pipeline (rl_kernels.hip). Each tile writes its
// descriptors ONCE, already sorted by bucket, with a row of bucket starts per tile; k4_group
// gathers each range of MSD buckets straight from those tile-sorted runs (one run per tile),
// so MSD records are written once and read once. k4_hist needs nothing from the table, so
// with two batches in flight it runs for batch k+1 on a second stream while batch k is
// decided (rl_engine.cpp, rl_submit_pipelined).
//
//   k4_hist    per 2048-descriptor tile: fingerprint (fixed_cache_impl.go:43-53 via
//              cache_key.go:57-68), hot-set lookup, bucket; stable LDS sort of the tile by
//              bucket and a segmented scan; the tile's records in bucket order (32-B MRec; a
//              hot record carries its in-tile INCRBY prefix), the row of bucket starts, the
//              hot buckets' h sums; nil-limit descriptors decided (base_limiter.go:72-75)
//   k4_scan    per hot bucket: exclusive scan of the h sums over tiles, table claim and the
//              counter before the batch; per MSD bucket the batch total (size check), and
//              per group of 64 MSD buckets the k4_group ranges
//              (whole buckets packed up to the LDS stage) — all before any table write, so a
//              refused batch leaves the table untouched
//   k4_place   per tile: hot descriptors decided in place (post-value = base + tile prefix +
//              in-tile prefix; local-cache freezes of requests that straddle tiles deferred)
//   k4_group   per MSD range: records gathered into LDS from every tile's run (tile order =
//              arrival order inside a key),
//              grouped by full fingerprint, segmented INCRBY prefix, one leader per key
//              (table probe/claim, serial-order INCRBY, local-cache freeze), decisions. The
//              last block to finish decides the deferred hot descriptors, counts U, fills
//              hot-set candidates and clears the control block of batch k+2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"
#include "rl_decide.h"
#include "rl_device.h"
#include "rl_tile.h"

namespace rlhip {
namespace v4 {

using tile::D3;
using tile::NT;
using tile::R;
using tile::SegEl;
using tile::T;
using tile::W;
using tile::BKT_NONE;

constexpr int ROW = V4_ROW16;  // u16 bucket starts per tile (entries [0, NBUCKETS] used)
// k4_hist's per-(tile, hot bucket) word: h sum (<= 2048 x (2^32 - 1) < 2^52) | count << 52
constexpr int HS_CNT_SHIFT = 52;
constexpr unsigned long long HS_SUM_MASK = (1ull << HS_CNT_SHIFT) - 1ull;
static_assert((unsigned long long)V4_TILE * 0xFFFFFFFFull <= HS_SUM_MASK && V4_TILE < (1 << 12), "hot word fields");
static_assert(ROW >= NBUCKETS + 1, "row holds every bucket start and the end");
#ifndef RL_G_CAP
// 896 records (two average config-3 buckets) per LDS stage at 3 blocks per CU (50 KB LDS,
// 152 VGPRs, no spills) measured 114.5 us/step against 118.5 for 640 x 4 blocks (spilling at
// 128 VGPRs) and 134.6 for 1024 x 2 (tools/build_variants.sh, bench --lib, one box)
#define RL_G_CAP 896
#define RL_G_HASH 1024
#define RL_G_OCC 3
#endif
constexpr int GBLOCKS = 256 * RL_G_OCC;    // k4_group blocks: RL_G_OCC per CU, one round
constexpr int MSD_GROUPS = MSD_BUCKETS / 64;  // k4_scan blocks of MSD buckets (one range list each)
constexpr uint32_t RPG = GBLOCKS / MSD_GROUPS;  // k4_group blocks per MSD group
static_assert(GBLOCKS % MSD_GROUPS == 0, "blocks per MSD group");
constexpr int RANGE_MAX = 128;             // ranges per MSD group (two per bucket at most)
// k4_scan -> k4_place / k4_group, one array of words: [0, MSD_GROUPS) ranges per group;
// R_START: per group RANGE_MAX + 1 range entries (bucket << 1 | half inside the group, last = 128);
// R_BPRE / R_GTOT: unused (reserved words of the layout).
constexpr int R_START = MSD_GROUPS;
constexpr int R_BPRE = R_START + MSD_GROUPS * (RANGE_MAX + 1);
constexpr int R_GTOT = R_BPRE + MSD_BUCKETS;
constexpr int R_BTOT = R_GTOT + MSD_GROUPS;  // per MSD bucket its batch total (k4_scan block pair hand-off)
constexpr int RANGE_WORDS = R_BTOT + MSD_BUCKETS;
constexpr int DONE_CTR = 27;               // EngineCtl::tile_ctr[DONE_CTR][0]: k4_group blocks done
#ifndef RL_G_NT
#define RL_G_NT 256
#endif
constexpr int G_NT = RL_G_NT;
constexpr int G_W = G_NT / 64;
constexpr int G_CAP = RL_G_CAP;    // records grouped in LDS (a larger pair runs bucket by bucket)
constexpr int G_HASH = RL_G_HASH;  // LDS hash slots (power of two > G_CAP)
constexpr int G_IPT = (G_CAP + G_NT - 1) / G_NT;  // positions per thread in registers (table read-ahead)
constexpr int GS_HASH = 2048;   // global-scratch hash slots (> BUCKET_CAP)
constexpr uint32_t G_EMPTY = 0xFFFFFFFFu;
static_assert(G_CAP <= G_NT * G_IPT && G_HASH > G_CAP && GS_HASH > BUCKET_CAP, "k4_group geometry");
static_assert(DONE_CTR != DFR_CTR && DONE_CTR != CAND_CTR &&
                  (DONE_CTR < INS_CTR0 || DONE_CTR >= INS_CTR0 + INS_LINES),
              "control-block rows");

using tile::rule_of;

#ifdef RL_STAMPS
// Diagnostic build only (tools/stamps_view.py): per-block phase timestamps (s_memrealtime,
// 100 MHz) of wave 0 of k4_group blocks. g_st4 is defined in rl_tile.h.
#define ST4(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_st4[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define ST4V(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_st4[blockIdx.x][k] = (v); } while (0)
// k4_group per-block facts of the batch in rows 3072 + block: [0] records grouped, [1] keys led,
// [2] ranges, [3] split ranges
#define ST4X(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_st4[3072 + blockIdx.x][k] += (v); } while (0)
// k4_scan blocks stamp rows 2048 + block (thread 0).
#define ST5(k) do { if (threadIdx.x == 0) g_st4[2048 + blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
// the last k4_group block's epilogue: row 4000
#define STL(k) do { if (threadIdx.x == 0) g_st4[4000][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
// k4_hist tiles: rows 1024 + tile
#ifdef RL_HIST_FINE  // load_descs stamps its two load levels into columns 2 and 3 (rl_tile.h)
#define STH(k) do { if ((k) < 2 || (k) > 5 || (k) == 2 || (k) == 3) { constexpr int c_ = (k) == 2 ? 4 : (k) == 3 ? 5 : (k); \
  if (threadIdx.x == 0 && blockIdx.x < 1024) g_st4[1024 + blockIdx.x][c_] = __builtin_amdgcn_s_memrealtime(); } } while (0)
#else
#define STH(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_st4[1024 + blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#endif
#else
#define STH(k) do { } while (0)
#define STL(k) do { } while (0)
#define ST5(k) do { } while (0)
#define ST4(k) do { } while (0)
#define ST4V(k, v) do { } while (0)
#define ST4X(k, v) do { } while (0)
#endif

// Stores handed to the last k4_group block bypass the L2 of the storing XCD (sc1, written
// through), and the last block reads them with sc1 loads: no agent-scope fences
// (MI355X_MICROARCH.md, hand-off table row 1).
RL_DEV void st_sc1_32B(void* p, const void* v) {
  const uint64_t* s = reinterpret_cast<const uint64_t*>(v);
  uint64_t* d = reinterpret_cast<uint64_t*>(p);
#pragma unroll
  for (int k = 0; k < 4; ++k) st_relaxed64(d + k, s[k]);
}
RL_DEV void ld_sc1_32B(void* v, const void* p) {
  const uint64_t* s = reinterpret_cast<const uint64_t*>(p);
  uint64_t* d = reinterpret_cast<uint64_t*>(v);
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = ld_relaxed64(s + k);
}
RL_DEV void emit_cand_sc1(EngineCtl* ctl, HotCand* __restrict__ cand, uint32_t rule, uint32_t count,
                          uint32_t first_idx, uint64_t a = 0, uint64_t b = 0, uint32_t unit = 0) {
  const uint32_t c = atomicAdd(&ctl->tile_ctr[CAND_CTR][0], 1u);
  if (c < (uint32_t)CAND_MAX) {
    HotCand hc;
    hc.a = a;
    hc.b = b;
    hc.unit = unit;
    hc.rule = rule;
    hc.count = count;
    hc.first_idx = first_idx;
    st_sc1_32B(&cand[c], &hc);
  }
}
static_assert(sizeof(HotCand) == 32 && sizeof(Deferred) == 32, "32-B hand-off records");
static_assert(sizeof(HotBucket) == 64, "HotBucket is one 64-B line");
// The counter a hot key's INCRBYs go to: the main store's, or the per-second store's.
RL_DEV uint32_t* hot_counter(const HotBucket& x) {
  Slot* s = reinterpret_cast<Slot*>(x.slot);
  return (x.flags & HB_PS) ? &s->pcount : &s->count;
}
constexpr int SHARD_CTR0 = 0;  // EngineCtl::tile_ctr[0..7][0]: k4_group blocks done, by blockIdx & 7

// ---------------------------------------------------------------------------
// k4_hist
// ---------------------------------------------------------------------------
template <bool ROUTED>
__global__ __launch_bounds__(NT) void k4_hist(DevBatch in, const DevRule* __restrict__ rules, uint32_t n_rules,
                                              uint64_t seed, const HotEntry* __restrict__ hot,
                                              uint32_t* __restrict__ req_thr, uint32_t* __restrict__ fpart,
                                              uint16_t* __restrict__ tstart, unsigned long long* __restrict__ thsum,
                                              MRec* __restrict__ srec, rl_status* __restrict__ out, EngineCtl* ctl) {
#ifndef RL_HIST_GLOBAL_HOT
  // sh_hot (the hot table: tag words, then the entries, rl_common.h) and s_res (hot in-tile
  // prefixes) share one pool: once every thread holds its descriptors' prefixes, the pool
  // stages half a tile of records at a time for coalesced, whole-line stores.
  constexpr size_t HOT_LDS = sizeof(HotEntry) * (HOT_SLOTS + HOT_MAX);
  __shared__ __attribute__((aligned(32))) uint8_t s_pool[HOT_LDS + sizeof(unsigned long long) * T];
  HotEntry* const sh_hot = reinterpret_cast<HotEntry*>(s_pool);
#else
  // Measured and not kept (round 4, A/B on one box): the hot table read where it lies (16 KB,
  // L1/L2-resident) instead of copied into LDS, so a block needs ≈48 KB of LDS instead of ≈64
  // and the pool stages a quarter tile per pass. k4_hist alone 42 -> 45 µs and the pipelined
  // step 106 -> 122 µs: more of the next batch's tiles then sit beside k4_group and both slow
  // down (with the VGPR budget cut to 96 as well, so that one tile fits beside two k4_group
  // blocks, no better).
  constexpr size_t HOT_LDS = 0;
  __shared__ __attribute__((aligned(32))) uint8_t s_pool[sizeof(unsigned long long) * T];
  const HotEntry* const sh_hot = hot;
#endif
  unsigned long long* const s_res = reinterpret_cast<unsigned long long*>(s_pool + HOT_LDS);
  MRec* const s_stage = reinterpret_cast<MRec*>(s_pool);
  constexpr uint32_t STAGE = (uint32_t)(sizeof(s_pool) / sizeof(MRec));  // records per staging pass
  static_assert(HOT_LDS % 16 == 0 && STAGE >= (uint32_t)T / 4 && T % STAGE == 0, "record staging");
  __shared__ uint16_t sh_cnt[ROW];
  __shared__ unsigned long long sh_hs[HOT_BUCKETS];
  __shared__ uint16_t s_d[T];
  __shared__ uint16_t s_pa[T], s_pb[T];
  __shared__ uint32_t s_h[T];
  __shared__ uint32_t s_cnt[W][64];
  __shared__ uint32_t sh_w[W];
  __shared__ SegEl s_agg[W];
  __shared__ uint32_t sh_f[FP_PART_WORDS];
  __shared__ uint32_t sh_err;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tile = blockIdx.x, ntiles = gridDim.x;
  const uint32_t t0 = tile * T;
  STH(0);
#ifndef RL_HIST_GLOBAL_HOT
  tile::load_hot_table(hot, sh_hot);
#endif
  for (int b = tid; b < ROW / 2; b += NT) reinterpret_cast<uint32_t*>(sh_cnt)[b] = 0;
  for (int b = tid; b < HOT_BUCKETS; b += NT) sh_hs[b] = 0;
  if (tid < FP_PART_WORDS) sh_f[tid] = 0;
  if (tid == 0) sh_err = 0;
  // DoLimitResponse.ThrottleMillis starts at 0 for every request (base_limiter.go:163-165)
  {
    const uint32_t per = (in.n_req + ntiles - 1) / ntiles;
    const uint32_t r0 = tile * per, r1 = min(in.n_req, r0 + per);
    if (req_thr)  // (raw replies: no ThrottleMillis slots)
      for (uint32_t q = r0 + tid; q < r1; q += NT) req_thr[q] = 0;
  }
  __syncthreads();
  STH(1);
  D3 d[R];
  uint32_t err = 0;
  if (ROUTED)
    tile::load_routed(in, rules, n_rules, sh_hot, t0, d, err);
  else
    tile::load_descs(in, rules, n_rules, seed, sh_hot, t0, d, err);
  STH(2);
  uint32_t nil = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t o = r * NT + tid;
    const uint32_t b = d[r].bucket;
    s_d[o] = (uint16_t)b;
    s_h[o] = d[r].h;
    s_pa[o] = (uint16_t)o;
    nil += b == NIL_BUCKET;
  }
  // Per-region generation range and descriptor count; per (unit, parity) the unit window of
  // hot descriptors. Reductions run only for regions / windows present in the wave.
#pragma unroll
  for (int rg = 0; rg < 8; ++rg) {
    uint32_t mn = 0xFFFFFFFFu, mx = 0, c = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool m = d[r].bucket < NIL_BUCKET && key_region(d[r].key) == (uint32_t)rg;
      c += (uint32_t)__popcll(__ballot(m));
      if (m) {
        mn = d[r].gen < mn ? d[r].gen : mn;
        mx = d[r].gen > mx ? d[r].gen : mx;
      }
    }
    if (c) {  // wave-uniform
      mn = wave_min_u32(mn);
      mx = wave_max_u32(mx);
      if (lane == 0) {
        atomicMax(&sh_f[FP_GMIN + rg], ~mn);
        atomicMax(&sh_f[FP_GMAX + rg], mx);
        atomicAdd(&sh_f[FP_CNT + rg], c);
      }
    }
    uint32_t um = 0;
    uint64_t any = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool m = d[r].bucket < (uint32_t)HOT_BUCKETS && d[r].uw == (uint32_t)rg;
      any |= __ballot(m);
      if (m) um = d[r].uwv > um ? d[r].uwv : um;
    }
    if (any) {
      um = wave_max_u32(um);
      if (lane == 0) atomicMax(&sh_f[FP_UW + rg], um);
    }
  }
  nil = tile::wave_sum(nil);
  if (lane == 0 && nil) atomicAdd(&sh_f[FP_NIL], nil);
  if (err) atomicOr(&sh_err, err);
  // Stable sort of the tile by bucket, then a segmented scan in sorted order:
  // hot -> inclusive prefix of h inside (tile, bucket); each bucket's last descriptor ->
  // the bucket's count (and h sum) in this tile.
  STH(3);
  tile::tile_digit_pass(s_d, s_pa, s_pb, 0, s_cnt, sh_w);  // includes barriers
  STH(4);
  tile::tile_digit_pass(s_d, s_pb, s_pa, 6, s_cnt, sh_w);
  STH(5);
  {
    const uint32_t s0 = tid * R;
    uint32_t od[R], dd[R], fl[R];
    unsigned long long hv[R];
    uint32_t prev_d = s0 == 0 ? 0xFFFFFFFFu : s_d[s_pa[s0 - 1]];
    const uint32_t next_d = s0 + R < (uint32_t)T ? s_d[s_pa[s0 + R]] : 0xFFFFFFFFu;
    SegEl t{0, 0, 0};
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const uint32_t o = s_pa[s0 + q];
      const uint32_t dv = s_d[o];
      od[q] = o;
      dd[q] = dv;
      fl[q] = dv != prev_d;
      hv[q] = s_h[o];
      prev_d = dv;
      t = tile::seg_op(t, SegEl{fl[q], s0 + q, hv[q]});
    }
    SegEl incl = t;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      SegEl y;
      y.f = __shfl_up(incl.f, s, 64);
      y.hp = __shfl_up(incl.hp, s, 64);
      y.s = __shfl_up(incl.s, s, 64);
      if (lane >= (uint32_t)s) incl = tile::seg_op(y, incl);
    }
    if (lane == 63) s_agg[wave] = incl;
    SegEl wex;
    wex.f = __shfl_up(incl.f, 1, 64);
    wex.hp = __shfl_up(incl.hp, 1, 64);
    wex.s = __shfl_up(incl.s, 1, 64);
    if (lane == 0) wex = SegEl{0, 0, 0};
    __syncthreads();
    SegEl run{0, 0, 0};
#pragma unroll
    for (int w = 0; w < W - 1; ++w) {
      const SegEl a = s_agg[w];  // wave-uniform LDS read
      if ((uint32_t)w < wave) run = tile::seg_op(run, a);
    }
    run = tile::seg_op(run, wex);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      run = tile::seg_op(run, SegEl{fl[q], s0 + q, hv[q]});
      const uint32_t b = dd[q];
      if (b < (uint32_t)HOT_BUCKETS) s_res[od[q]] = run.s;
      s_pb[od[q]] = (uint16_t)(s0 + q);  // sorted position of descriptor od[q]
      const uint32_t nd = q + 1 < R ? dd[q + 1] : next_d;
      if (b < NIL_BUCKET && nd != b) {  // the bucket's last descriptor of the tile
        sh_cnt[b] = (uint16_t)(s0 + q + 1u - run.hp);
        if (b < (uint32_t)HOT_BUCKETS) sh_hs[b] = run.s;
      }
    }
  }
  __syncthreads();
  // Bucket starts of the tile: exclusive scan of the counts (entries [0, ROW), 6 per thread).
  {
    constexpr int PER = (ROW + NT - 1) / NT;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t e = tid * PER + k;
      v[k] = e < (uint32_t)ROW ? sh_cnt[e] : 0u;
      sum += v[k];
    }
    uint32_t total;
    uint32_t run = tile::block_excl_scan<NT>(sum, sh_w, total);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t e = tid * PER + k;
      if (e < (uint32_t)ROW) sh_cnt[e] = (uint16_t)run;
      run += v[k];
    }
  }
  STH(6);
  // Records in bucket order. A hot record carries its in-tile INCRBY prefix and its bucket;
  // an MSD record its sort key and fp_lo; a nil-limit descriptor is decided here. Each record
  // goes to its sorted position in the LDS stage (half a tile per pass), and the stage leaves
  // in 16-B stores, consecutive across the block: whole 128-B lines, where scattered 32-B
  // stores left partly written lines for the L2 to evict (≈14 MB of extra writes per batch).
  uint32_t spos[R];
  unsigned long long sres[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t o = r * NT + tid;
    spos[r] = s_pb[o];
    sres[r] = d[r].bucket < (uint32_t)HOT_BUCKETS ? s_res[o] : 0ull;
  }
  const uint32_t nvalid = min((uint32_t)T, in.n_desc > t0 ? in.n_desc - t0 : 0u);  // the tile's records
  for (uint32_t h0 = 0; h0 < (uint32_t)T; h0 += STAGE) {
    __syncthreads();  // (h0 = 0: every thread has read s_res; else: the previous pass's copy is done)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t o = r * NT + tid;
      const uint32_t i = t0 + o;
      const D3& x = d[r];
      if (x.bucket == BKT_NONE || spos[r] - h0 >= STAGE) continue;
      if (x.bucket == NIL_BUCKET) {
        if (in.raw) {  // raw replies (a routed batch never carries a nil limit)
          emit_raw(out, i, 0u, RAW_NIL);
          continue;
        }
        // GetResponseDescriptorStatus("" key) -> {OK, nil limit, 0}  base_limiter.go:72-75
        rl_status st;
        st.code_flags = RL_CODE_OK;
        st.limit_remaining = 0;
        st.reset_s = 0;
        st.over_limit_delta = 0;
        st.near_limit_delta = 0;
        out[i] = st;
        continue;
      }
      const bool hotb = x.bucket < (uint32_t)HOT_BUCKETS;
      MRec m;
      m.key = hotb ? (uint64_t)sres[r] : x.key;
      // EXPIRE jitter: a routed record's rides in x.lo's high half (load_routed); an unrouted
      // descriptor's is read here (kernel-uniform test: no load without jitter), not carried
      // through the tile
      const uint32_t jt = in.recs ? (uint32_t)(x.lo >> 32) : desc_jit(in, i);
      m.fp_lo = (hotb ? (uint64_t)x.bucket : (uint64_t)(uint32_t)x.lo) | ((uint64_t)jt << 32);
      m.idx = i;
      m.req = x.req;
      m.h = x.h;
      m.rn = rule_of(x.rule) | (x.now_mod << V4_RULE_BITS);
      s_stage[spos[r] - h0] = m;
    }
    __syncthreads();
    // the pass's records (positions past the tile's valid ones hold nil / past-the-end
    // descriptors: never read, and not stored past the batch)
    const uint32_t np = nvalid > h0 ? min(STAGE, nvalid - h0) : 0u;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));  // 16-B aligned: one dwordx4 each
    const v4u* sv = reinterpret_cast<const v4u*>(s_stage);
    v4u* dv = reinterpret_cast<v4u*>(srec + t0 + h0);
    for (uint32_t c = tid; c < np * (uint32_t)(sizeof(MRec) / 16); c += NT) dv[c] = sv[c];
  }
  __syncthreads();
  uint32_t* trow = reinterpret_cast<uint32_t*>(tstart + (size_t)tile * ROW);
  for (int b = tid; b < ROW / 2; b += NT) trow[b] = reinterpret_cast<const uint32_t*>(sh_cnt)[b];
  // per hot bucket one word: its h sum in the tile | its descriptor count << HS_CNT_SHIFT (k4_scan
  // reads one word per (tile, hot bucket), not two u16 row entries and the sum)
  unsigned long long* hrow = thsum + (size_t)tile * HOT_BUCKETS;
  for (int b = tid; b < HOT_BUCKETS; b += NT)
    hrow[b] = sh_hs[b] | ((unsigned long long)(sh_cnt[b + 1] - sh_cnt[b]) << HS_CNT_SHIFT);
  // word-major ([word][tile]): k4_scan's hot blocks read each word of every tile coalesced
  if (tid < FP_PART_WORDS) fpart[(size_t)tid * ntiles + tile] = sh_f[tid];
  if (tid == 0 && sh_err) atomicOr(&ctl->err, sh_err);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STH(7);
}

// ---------------------------------------------------------------------------
// k4_scan — 64 buckets per block (one per lane); the 16 waves split the tiles.
// ---------------------------------------------------------------------------
constexpr int SCAN_NT = 1024;
constexpr int SCAN_W = SCAN_NT / 64;
constexpr int SCAN_U = 16;  // column loads in flight per lane (columns longer than SCAN_Q)
// One MSD block per group of 64 buckets (lane = bucket, wave = tile slice, up to SCAN_Q tiles
// per lane in registers): the block holds the group's 64 bucket totals itself and packs the
// group's k4_group ranges right away (a pair of 32-bucket blocks needed a hand-off through
// global memory and a pair counter: three more round trips on k4_scan's critical path).
constexpr int MSD_PER_BLOCK = 64;
constexpr int MSD_SCAN_BLOCKS = MSD_GROUPS;
constexpr int SCAN_Q = 32;  // MSD column entries per lane kept in registers (16 slices x 32 = 512 tiles)
// Hot blocks take 16 buckets each over 64 tile slices (lane = slice % 4 * 16 + bucket, wave =
// slice / 4): 32 blocks instead of 8, so the hot columns (u16 starts + u64 h sums of every
// tile) are pulled by 32 CUs, 8 tiles per lane at config 3.
#ifndef RL_HOT_PER_BLOCK
#define RL_HOT_PER_BLOCK 16
#endif
constexpr int HOT_PER_BLOCK = RL_HOT_PER_BLOCK;
static_assert(HOT_PER_BLOCK >= 4 && HOT_PER_BLOCK <= 16 && (HOT_PER_BLOCK & (HOT_PER_BLOCK - 1)) == 0, "hot buckets per block");
constexpr int HOT_SCAN_BLOCKS = HOT_BUCKETS / HOT_PER_BLOCK;
constexpr int HOT_Q = 16;   // hot column entries per lane kept in registers
static_assert(HOT_BUCKETS % 64 == 0 && MSD_BUCKETS % 64 == 0, "bucket blocks");
static_assert(T < 65536 && MSD_GROUPS <= 64, "k4_scan geometry");

// Records of the group's bucket b0 + lane in tiles [tb, te) ∩ [tb, tb + SCAN_Q): one dword of
// the tile's row per lane and tile, so each bucket start is loaded once. Lane l reads dword
// (l + 1) / 2 of the group's row segment: an even lane holds its bucket's start and end, an
// odd lane its bucket's end and the next one's (its start is the even lane below's high
// half; lane 63 reads entry 64 of the segment). Sums of the low and high halves over the
// tiles first, then one shuffle.
static_assert(ROW % 2 == 0 && HOT_BUCKETS % 2 == 0 && NBUCKETS + 1 <= ROW, "dword-aligned row segments");
RL_DEV uint32_t column_total(const uint16_t* __restrict__ tstart, uint32_t b0, uint32_t tb, uint32_t te) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t di = (lane + 1u) >> 1;
  uint32_t d[SCAN_Q];
#pragma unroll
  for (int u = 0; u < SCAN_Q; ++u) {  // clamped tiles: all loads in flight together
    const uint32_t* row = reinterpret_cast<const uint32_t*>(tstart + (size_t)min(tb + u, te - 1u) * ROW + b0);
    d[u] = row[di];
  }
  uint32_t slo = 0, shi = 0;
#pragma unroll
  for (int u = 0; u < SCAN_Q; ++u) {
    const uint32_t x = tb + u < te ? d[u] : 0u;
    slo += x & 0xFFFFu;
    shi += x >> 16;
  }
  const uint32_t shi_prev = __shfl_up(shi, 1, 64);
  return (lane & 1u) ? slo - shi_prev : shi - slo;
}

__global__ __launch_bounds__(SCAN_NT) void k4_scan(const uint16_t* __restrict__ tstart,
                                                   const unsigned long long* __restrict__ thsum, uint32_t ntiles,
                                                   uint32_t n_desc,
                                                   unsigned long long* __restrict__ hoff,
                                                   const uint32_t* __restrict__ fpart,
                                                   const HotEntry* __restrict__ hot_list, HotBucket* __restrict__ hb,
                                                   TableDesc tab, HotCand* __restrict__ cand,
                                                   uint32_t* __restrict__ heads_out, uint32_t* __restrict__ ins_out,
                                                   uint32_t* __restrict__ ranges,
                                                   const uint32_t* __restrict__ poison,
                                                   const RegionOcc* __restrict__ occ, EngineCtl* ctl) {
  const uint32_t local_cache = tab.local_cache;
  __shared__ uint32_t s_f[FP_PART_WORDS];
  __shared__ uint32_t s_pc[SCAN_W][64];
  __shared__ unsigned long long s_ph[SCAN_W][64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // A batch submitted behind a refused one (two batches in flight) is refused too, before
  // anything touches the table: the engine reruns both, in order (rl_engine::settle).
  if (*poison) {
    if (blockIdx.x == 0 && tid == 0) atomicOr(&ctl->err, ERR_FALLBACK);
    return;
  }
  ST5(0);
  const bool hotb = blockIdx.x < (uint32_t)HOT_SCAN_BLOCKS;  // block-uniform
  const uint32_t errs = ctl->err;
  const HotEntry he = hot_list[((blockIdx.x % (uint32_t)HOT_SCAN_BLOCKS) * HOT_PER_BLOCK + (lane & (HOT_PER_BLOCK - 1u))) >> 1];
  RegionOcc oc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) oc[r] = occ[r];
  // Hot blocks fold the per-tile partials (generation range per region, nil count; the hot
  // claims need the generations, block 0 publishes them). The partials' loads are issued
  // here and reduced after the column pass, so the two latencies overlap; MSD blocks need
  // none of it.
  // Partials: wave v folds words v, v + 16, v + 32 over the tiles (lane = tile mod 64, FPT
  // tiles a lane in registers, loaded here at clamped indices, all in flight together), one
  // wave reduction per word instead of one per word in every wave.
  constexpr int FPW = (FP_PART_WORDS + SCAN_W - 1) / SCAN_W;
  constexpr int FPT = 8;
  uint32_t fl[FPW][FPT];
  if (hotb) {
#pragma unroll
    for (int q = 0; q < FPW; ++q)
#pragma unroll
      for (int u = 0; u < FPT; ++u) {
        const uint32_t w = min(wave + (uint32_t)q * SCAN_W, (uint32_t)FP_PART_WORDS - 1u);
        const uint32_t t = min(lane + (uint32_t)u * 64u, ntiles - 1u);
        fl[q][u] = fpart[(size_t)w * ntiles + t];
      }
  }

  // Column pass. MSD blocks: bucket b = lane, tiles [wave*Q, wave*Q + Q). Hot blocks: bucket
  // b = lane % 16 of the block's 16, tile slice wave * 4 + lane / 16.
  const uint32_t m = blockIdx.x - HOT_SCAN_BLOCKS;  // MSD block: group m
  const uint32_t bpb = hotb ? HOT_PER_BLOCK : MSD_PER_BLOCK;  // buckets per block
  const uint32_t bb = lane & (bpb - 1u);
  const uint32_t nsl = SCAN_NT / bpb;  // tile slices
  const uint32_t slice = wave * (64 / bpb) + lane / bpb;
  const uint32_t mb0 = HOT_BUCKETS + m * 64;  // MSD: first bucket of the block
  const uint32_t b = hotb ? blockIdx.x * HOT_PER_BLOCK + bb : mb0 + bb;
  const uint32_t Q = (ntiles + nsl - 1) / nsl;
  const uint32_t tb = min(ntiles, slice * Q), te = min(ntiles, tb + Q);
  uint32_t c = 0;
  unsigned long long hs = 0;
  // Columns up to SCAN_Q (MSD) / HOT_Q (hot) tiles per lane are loaded once, all loads in
  // flight together, and kept in registers for the prefix pass below.
  const bool in_regs = Q <= (uint32_t)(hotb ? HOT_Q : SCAN_Q);  // block-uniform
  unsigned long long hq[HOT_Q];  // hot: h sums
  if (in_regs && hotb) {
    // every load at a clamped tile, so all of them are in flight together (a load behind a
    // per-lane condition waits for the one before it)
#pragma unroll
    for (int u = 0; u < HOT_Q; ++u) {
      const uint32_t t = min(tb + u, ntiles - 1u);
      hq[u] = thsum[(size_t)t * HOT_BUCKETS + b];  // h sum | count << HS_CNT_SHIFT
    }
#pragma unroll
    for (int u = 0; u < HOT_Q; ++u) {
      const bool v = tb + u < te;
      c += v ? (uint32_t)(hq[u] >> HS_CNT_SHIFT) : 0u;
      hq[u] = v ? hq[u] & HS_SUM_MASK : 0ull;
      hs += hq[u];
    }
  } else if (in_regs) {
    c = column_total(tstart, mb0, tb, te);
  } else {
    for (uint32_t t = tb; t < te; t += SCAN_U) {
      uint32_t cv[SCAN_U];
      unsigned long long hv[SCAN_U];
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) {
        const uint16_t* row = tstart + (size_t)(t + u) * ROW + b;
        const unsigned long long w = (hotb && t + u < te) ? thsum[(size_t)(t + u) * HOT_BUCKETS + b] : 0ull;
        cv[u] = t + u >= te ? 0u : hotb ? (uint32_t)(w >> HS_CNT_SHIFT) : (uint32_t)row[1] - (uint32_t)row[0];
        hv[u] = w & HS_SUM_MASK;
      }
#pragma unroll
      for (int u = 0; u < SCAN_U; ++u) {
        c += cv[u];
        hs += hv[u];
      }
    }
  }
  s_pc[wave][lane] = c;
  bool span = false, cap_ok = true;
  if (hotb) {
    s_ph[wave][lane] = hs;
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const uint32_t w = wave + (uint32_t)q * SCAN_W;
      if (w >= (uint32_t)FP_PART_WORDS) break;  // wave-uniform
      const bool mx = fp_is_max((int)w);
      uint32_t v = 0;
#pragma unroll
      for (int u = 0; u < FPT; ++u) {
        const uint32_t x = lane + (uint32_t)u * 64u < ntiles ? fl[q][u] : 0u;
        v = mx ? max(v, x) : v + x;
      }
      for (uint32_t t = 64u * FPT + lane; t < ntiles + lane; t += 64u) {  // more than 64 x FPT tiles
        const uint32_t x = t < ntiles ? fpart[(size_t)w * ntiles + t] : 0u;
        v = mx ? max(v, x) : v + x;
      }
      v = mx ? wave_max_u32(v) : tile::wave_sum(v);
      if (lane == 0) s_f[w] = v;
    }
  }
  __syncthreads();
  ST5(2);
  if (hotb) {
    // Two window generations of one region in one batch must be adjacent;
    // a region's generations share its parity, so a valid batch has ONE generation per region.
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
      const uint32_t mx = s_f[FP_GMAX + rg], mn = ~s_f[FP_GMIN + rg];
      span |= mx != 0 && mx - mn > 1u;
    }
    // Capacity (before any table write): every hot block computes the same verdict and
    // claims nothing when it fails; block 0 refuses the batch.
    cap_ok = capacity_ok(oc, &s_f[FP_GMAX], &s_f[FP_CNT], tab.lag);
    if (blockIdx.x == 0) {
      if (tid < 8) ctl->gen_min[tid] = ~s_f[FP_GMIN + tid];
      else if (tid < 16) ctl->gen_max[tid - 8] = s_f[FP_GMAX + tid - 8];
      else if (tid == 16) ctl->n_nil = s_f[FP_NIL];
      if (tid == 0 && span) atomicOr(&ctl->err, ERR_WINDOW_SPAN);
      if (tid == 0 && !cap_ok) atomicOr(&ctl->err, ERR_TABLE_FULL);
    }
  }
  uint32_t ctot = 0;
  unsigned long long hrun = 0, htot = 0;
  if (hotb) {  // bucket totals over the 64 slices; h sums of the slices before this lane's
#pragma unroll
    for (int w = 0; w < SCAN_W; ++w) {
#pragma unroll
      for (int q = 0; q < 64 / HOT_PER_BLOCK; ++q) {
        const uint32_t sl = (uint32_t)(w * (64 / HOT_PER_BLOCK) + q);
        const uint32_t x = s_pc[w][q * HOT_PER_BLOCK + bb];
        const unsigned long long y = s_ph[w][q * HOT_PER_BLOCK + bb];
        ctot += x;
        htot += y;
        hrun += sl < slice ? y : 0ull;
      }
    }
  } else {  // bucket totals over the 16 slices
#pragma unroll
    for (int w = 0; w < SCAN_W; ++w) ctot += s_pc[w][bb];
  }
  if (!hotb) {
    // (no per-tile offsets: k4_group gathers a range's records from each tile's run. A bucket
    // over BUCKET_CAP records sends the batch to the LSD pipeline before the table is touched.)
    if (wave != 0) return;
    ST5(3);
    if (lane == 0) heads_out[blockIdx.x] = 0;
    if (ctot > (uint32_t)BUCKET_CAP) atomicOr(&ctl->err, ERR_FALLBACK);
    const uint32_t g = m;
    // Pack the group's 64 buckets into k4_group ranges of whole buckets, at most G_CAP records
    // each (a single larger bucket: two half ranges of its own), balanced over the group's RPG
    // blocks (a k4_group block's time grows with its range's records, and the kernel lasts as
    // long as its largest range). Entries are marked in two masks: bit k of ev = entry 2k (a
    // range starts at bucket k), of od = entry 2k | 1 (the second half of oversized bucket k);
    // the lanes then store the entries in order in one step.
    //   Common case, in parallel: bucket k joins range floor((E_k + c_k / 2) / t), E_k its
    // exclusive prefix, t = ceil(total / RPG): a range closes before a bucket whose midpoint
    // passes the next multiple of the even share. Taken when no bucket is oversized and every
    // range fits the stage; otherwise a sequential walk (a range closes before a bucket whose
    // midpoint would pass the even share of what is left), ~5 us of scalar code per group.
    uint32_t* rb = ranges + R_START + g * (RANGE_MAX + 1);
    uint64_t ev = 0, od = 0;
    const uint32_t rem0 = tile::wave_sum(ctot);
    const uint32_t excl = wave_incl_scan_u32(ctot) - ctot;
    const uint32_t t_share = max(rem0 / RPG + (rem0 % RPG != 0u ? 1u : 0u), 1u);
    const uint32_t rid = min((excl + ctot / 2u) / t_share, RPG - 1u);
    const uint32_t rid_prev = __shfl_up(rid, 1, 64);
    const bool starts = lane == 0 || rid != rid_prev;
    const uint64_t smask = __ballot(starts);
    const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    const uint32_t nxt = (smask & above) ? (uint32_t)__ffsll((unsigned long long)(smask & above)) - 1u : 64u;
    const uint32_t e_next = __shfl(excl, nxt & 63u, 64);
    const uint32_t rsize = (nxt < 64u ? e_next : rem0) - excl;
    const bool fits = __ballot(ctot > (uint32_t)G_CAP || (starts && rsize > (uint32_t)G_CAP)) == 0ull;
    if (fits) {
      ev = smask & ~1ull;
    } else {
      uint32_t cur = 0, last = 0;  // last = the latest entry
      uint32_t rem = rem0, left = RPG;  // records not in closed ranges; ranges to form
#pragma unroll 1
      for (int k = 0; k < 64; ++k) {
        const uint32_t cb = (uint32_t)__builtin_amdgcn_readlane((int)ctot, k);
        const uint32_t ek = (uint32_t)k << 1;
        if (cb > (uint32_t)G_CAP) {
          // Oversized bucket (<= BUCKET_CAP): two ranges of its own, one per fingerprint half
          // (entries ek and ek | 1), grouped by two blocks; the next bucket starts a range.
          if (last != ek) {
            ev |= 1ull << k;
            rem -= cur;
            left = left > 1u ? left - 1u : 1u;
          }
          od |= 1ull << k;
          last = ek | 1u;
          left = left > 1u ? left - 1u : 1u;
          cur = cb;
          continue;
        }
        if (cur && (cur + cb > (uint32_t)G_CAP || (2u * cur + cb) * left > 2u * rem)) {
          ev |= 1ull << k;
          last = ek;
          rem -= cur;
          left = left > 1u ? left - 1u : 1u;
          cur = 0;
        }
        cur += cb;
      }
    }
    {
      const uint64_t below = lanemask_lt();
      const uint32_t has_ev = (uint32_t)(ev >> lane) & 1u, has_od = (uint32_t)(od >> lane) & 1u;
      const uint32_t p_ev = 1u + (uint32_t)__popcll(ev & below) + (uint32_t)__popcll(od & below);
      if (has_ev) rb[p_ev] = lane << 1;
      if (has_od) rb[p_ev + has_ev] = (lane << 1) | 1u;
      const uint32_t nr = (uint32_t)__popcll(ev) + (uint32_t)__popcll(od) + 1u;
      if (lane == 0) {
        rb[0] = 0;
        rb[nr] = 64u << 1;
        ranges[g] = nr;
      }
    }
    ST5(4);
    return;
  }
  if (in_regs) {
#pragma unroll
    for (int u = 0; u < HOT_Q; ++u) {
      if (tb + u < te) hoff[(size_t)(tb + u) * HOT_BUCKETS + b] = hrun;
      hrun += hq[u];
    }
  }
  for (uint32_t t = in_regs ? te : tb; t < te; t += SCAN_U) {
    unsigned long long hv[SCAN_U];
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u) hv[u] = t + u < te ? thsum[(size_t)(t + u) * HOT_BUCKETS + b] & HS_SUM_MASK : 0ull;
#pragma unroll
    for (int u = 0; u < SCAN_U; ++u) {
      if (t + u < te) hoff[(size_t)(t + u) * HOT_BUCKETS + b] = hrun;
      hrun += hv[u];
    }
  }
  const bool lead = wave == 0 && lane < (uint32_t)HOT_PER_BLOCK && ctot && !span && cap_ok &&
                    !(errs & (ERR_BAD_INPUT | ERR_BAD_TIME | ERR_FALLBACK));
  // (cand = nullptr: no candidates wanted for this batch, the engine samples every 8th)
  const uint64_t cmask = __ballot(lead && ctot >= HOT_CAND_MIN && cand != nullptr);
  uint32_t cbase = 0;  // lane 0: the first reserved slot (read where it is used)
  if (wave == 0 && lane == 0 && cmask) cbase = atomicAdd(&ctl->tile_ctr[CAND_CTR][0], (uint32_t)__popcll(cmask));
  if (wave == 0) {
    ST5(3);
    // Hot key leader: find or claim the key's slot and read the counter before this batch. A
    // claimed slot starts at count 0, which is invisible if the batch is later rejected.
    HotBucket x;
    x.key = x.fp_lo = x.base = x.slot = x.total = 0;
    x.rule = 0;
    x.flags = 0;
    x.rstar = 0xFFFFFFFFu;
    x.ws = x.t_all = x.t_rstar = 0;
    uint32_t heads = 0;
    uint32_t ins_region = 8;  // region of a newly claimed slot
    // lanes 0..15 of wave 0 (slice 0) lead the block's 16 hot buckets
    if (lane < (uint32_t)HOT_PER_BLOCK && ctot && !span && cap_ok &&
        !(errs & (ERR_BAD_INPUT | ERR_BAD_TIME | ERR_FALLBACK))) {
      // the key string's window: the hot prefix's unit window of this parity
      const uint32_t uwv = s_f[FP_UW + (he.unit - 1u) * 2u + (b & 1u)];
      const uint32_t div = unit_div(he.unit);
      const uint32_t ws = (uwv - 1u) * div;
      const Place pl = place_of(ws);
      uint64_t hi, lo;
      fp_final(FpState{he.a, he.b}, ws, hi, lo);
      x.key = make_sort_key(pl.region, hi);
      x.fp_lo = lo;
      x.rule = he.rule;
      x.total = htot;
      x.ws = ws;
      Slot* slot = nullptr;
      bool existed = false;
      KeyState ks{0, 0, 0, 0};
      if (!table_claim(tab, x.key, lo, pl.gen, slot, existed, ks)) {
        atomicOr(&ctl->err, ERR_TABLE_FULL);  // unreachable below the load limit
      } else {
        if (!existed) {
          slot_reset(slot, x.key);
          ins_region = pl.region;
        }
        const bool ps = per_second_store(tab, he.unit);
        bool frozen_pre = false;
        if (!fast_state(ks, ps, local_cache != 0, ws, div, x.base, frozen_pre)) {
          // an expiry falls among this batch's touches of a shared string: exact path
          atomicOr(&ctl->err, ERR_FALLBACK);
        } else {
          // an expired main counter restarts at 0 before the atomicMax updates of k4_place
          if (!ps && ks.exp <= ws && ks.count) slot->count = 0;
          x.flags = (frozen_pre ? HB_FROZEN_PRE : 0u) | (ps ? HB_PS : 0u);
        }
        x.slot = (uint64_t)(uintptr_t)slot;
        // The local-cache freeze point is found from a monotone INCRBY sequence; a batch whose
        // counter would pass 2^32 goes to the LSD pipeline (uint32 wraparound, R10).
        if (local_cache && !(x.flags & HB_FROZEN_PRE) && x.base + htot >= (1ull << 32))
          atomicOr(&ctl->err, ERR_FALLBACK);
        heads = 1;
      }
      if (cand && ctot >= HOT_CAND_MIN) {
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cbase, 0) + (uint32_t)__popcll(cmask & lanemask_lt());
        if (c < (uint32_t)CAND_MAX) {
          HotCand hc;
          hc.a = he.a; hc.b = he.b; hc.unit = he.unit; hc.rule = he.rule; hc.count = ctot; hc.first_idx = 0xFFFFFFFFu;
          cand[c] = hc;
        }
      }
    }
    // new slots per region of this block, two 16-bit counts a word (the last k4_group block
    // adds them to RegionOcc)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const uint32_t lo_n = (uint32_t)__popcll(__ballot(ins_region == (uint32_t)(2 * x)));
      const uint32_t hi_n = (uint32_t)__popcll(__ballot(ins_region == (uint32_t)(2 * x + 1)));
      if (lane == 0) ins_out[blockIdx.x * 4 + x] = lo_n | (hi_n << 16);
    }
    if (lane < (uint32_t)HOT_PER_BLOCK) {
      hb[b] = x;
      if (local_cache) hot_exp(hb)[b] = 0;  // the freezing request's last INCRBY: (index, jitter), k4_place / k4_group
    }
    heads = tile::wave_sum(heads);
    if (lane == 0) heads_out[blockIdx.x] = heads;
    ST5(4);
  }
}

// ---------------------------------------------------------------------------
// k4_group
// ---------------------------------------------------------------------------
// Storage of one grouped range: LDS arrays (G_CAP records) or a block's global scratch.
struct GS {
  MRec* rec;       // staged records by position; a leader overwrites its own key with the
                   // counter before the batch and its fp_lo with the freeze
  uint64_t* P;     // INCRBY prefix by position
  uint16_t* list;  // positions grouped by key, each key's in position (= arrival) order
  uint16_t* grp;   // position -> hash slot
  uint32_t* slot;  // hash slot -> first position inserted with the key (G_EMPTY = free)
  uint32_t* cnt;   // hash slot -> records of the key
  uint16_t* end;   // hash slot -> end of the key's list (start = end - cnt)
  uint32_t* cursor;
  uint32_t hs;     // hash slots (power of two)
};

// Barrier between phases. The LDS path exchanges data through LDS only, so it waits for
// LDS traffic alone and leaves the table read-ahead loads in flight across the barrier.
template <bool LDS>
RL_DEV void gbar() {
  if constexpr (LDS) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __threadfence_block();
    __syncthreads();
  }
}

// Hash slot counts: records of the key in the low 16 bits; CNT_MIXED when a record's rule
// differs from the first record's, CNT_MIXED_UNIT when its unit does too (found here, in
// parallel, instead of by a walk of the key's list).
constexpr uint32_t CNT_MASK = 0xFFFFu, CNT_MIXED = 0x10000u, CNT_MIXED_UNIT = 0x20000u;
RL_DEV bool g_insert(const GS& g, uint32_t k, const DevRule* __restrict__ rules) {
  // identity: the sort key and the tag (fp_lo's low half; its high half is the record's jitter)
  const uint64_t key = g.rec[k].key;
  const uint32_t lo = (uint32_t)g.rec[k].fp_lo;
  const uint32_t hmask = g.hs - 1u;
  uint32_t s = (uint32_t)key & hmask;
  uint32_t v;
#ifdef RL_PROBE_STATS  // diagnostics: probes and inserts per k4_group block (stamp rows 3072 + block)
  uint32_t probes = 0;
#endif
  for (;;) {
    v = atomicCAS(&g.slot[s], G_EMPTY, k);
#ifdef RL_PROBE_STATS
    ++probes;
#endif
    if (v == G_EMPTY || (g.rec[v].key == key && (uint32_t)g.rec[v].fp_lo == lo)) break;
    s = (s + 1) & hmask;
  }
#ifdef RL_PROBE_STATS
  if (blockIdx.x < 1024) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&g_st4[3072 + blockIdx.x][4]), (unsigned long long)probes);
    atomicAdd(reinterpret_cast<unsigned long long*>(&g_st4[3072 + blockIdx.x][5]), 1ull);
    if (v == G_EMPTY) atomicAdd(reinterpret_cast<unsigned long long*>(&g_st4[3072 + blockIdx.x][6]), 1ull);
  }
#endif
  g.grp[k] = (uint16_t)s;
  uint32_t inc = 1u;
  if (v != G_EMPTY) {
    const uint32_t r0 = rule_of(g.rec[v].rn), r1 = rule_of(g.rec[k].rn);
    if (r0 != r1) inc |= rules[r0].unit != rules[r1].unit ? (CNT_MIXED | CNT_MIXED_UNIT) : CNT_MIXED;
  }
  if (inc == 1u) atomicAdd(&g.cnt[s], 1u);
  else atomicOr(&g.cnt[s], inc & ~1u), atomicAdd(&g.cnt[s], 1u);
  return v == G_EMPTY;  // this position claimed the hash slot: it leads the key
}

// One wave: each key's list in position order (positions [0, m), 64 at a time).
RL_DEV void g_layout(const GS& g, uint32_t m) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lt = lanemask_lt();
  for (uint32_t c = 0; c < m; c += 64) {
    const uint32_t k = c + lane;
    const bool valid = k < m;
    const uint32_t s = valid ? g.grp[k] : 0u;
    uint64_t mm = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      if ((g.hs >> b) <= 1u) break;  // wave-uniform
      const bool bit = (s >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      mm &= bit ? bal : ~bal;
    }
    uint32_t before = 0;
    if (valid) before = g.end[s];
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      if (lane == (uint32_t)__ffsll((unsigned long long)mm) - 1u) g.end[s] = (uint16_t)(before + (uint32_t)__popcll(mm));
      g.list[before + (uint32_t)__popcll(mm & lt)] = (uint16_t)k;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

struct LSeg {
  uint32_t f;
  unsigned long long s;
};
RL_DEV LSeg lseg_op(const LSeg& a, const LSeg& b) { return b.f ? b : LSeg{a.f, a.s + b.s}; }

// Segmented inclusive scan of h over the lists (list positions [0, m) in chunks of
// G_NT * G_IPT, blocked G_IPT per thread): g.P[position] = INCRBY prefix of its key.
template <bool LDS>
RL_DEV void g_scan(const GS& g, uint32_t m, LSeg* s_agg, LSeg* s_carry) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) *s_carry = LSeg{0, 0};
  gbar<LDS>();
  for (uint32_t c0 = 0; c0 < m; c0 += G_NT * G_IPT) {
    uint32_t pos[G_IPT], hd[G_IPT];
    unsigned long long hv[G_IPT];
    LSeg t{0, 0};
#pragma unroll
    for (int q = 0; q < G_IPT; ++q) {
      const uint32_t e = c0 + tid * G_IPT + q;
      pos[q] = 0xFFFFFFFFu;
      hd[q] = 0;
      hv[q] = 0;
      if (e < m) {
        const uint32_t k = g.list[e];
        const uint32_t s = g.grp[k];
        pos[q] = k;
        hd[q] = e == (uint32_t)g.end[s] - (g.cnt[s] & CNT_MASK);
        hv[q] = g.rec[k].h;
        t = lseg_op(t, LSeg{hd[q], hv[q]});
      }
    }
    LSeg incl = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      LSeg y;
      y.f = __shfl_up(incl.f, d, 64);
      y.s = __shfl_up(incl.s, d, 64);
      if (lane >= (uint32_t)d) incl = lseg_op(y, incl);
    }
    if (lane == 63) s_agg[wave] = incl;
    LSeg wex;
    wex.f = __shfl_up(incl.f, 1, 64);
    wex.s = __shfl_up(incl.s, 1, 64);
    if (lane == 0) wex = LSeg{0, 0};
    gbar<LDS>();
    LSeg run = *s_carry;
    for (uint32_t w = 0; w < wave; ++w) run = lseg_op(run, s_agg[w]);
    run = lseg_op(run, wex);
#pragma unroll
    for (int q = 0; q < G_IPT; ++q) {
      if (pos[q] == 0xFFFFFFFFu) continue;
      run = lseg_op(run, LSeg{hd[q], hv[q]});
      g.P[pos[q]] = run.s;
    }
    gbar<LDS>();
    if (tid == G_NT - 1) {  // carry = the whole chunk, folded onto the previous carry
      LSeg all = *s_carry;
      for (int w = 0; w < G_W; ++w) all = lseg_op(all, s_agg[w]);
      *s_carry = all;
    }
    gbar<LDS>();
  }
}

RL_DEV uint32_t g_tail(const GS& g, uint32_t k) { return g.list[g.end[g.grp[k]] - 1u]; }

// The exact sequential path of a key (rare: a string shared by units of different sizes
// whose expiry falls inside the batch), run by its leader in a pass after the leaders' so
// its registers are not live across the fast path's. rec[k].key holds the key's slot.
constexpr uint32_t SEG_EXOTIC_PENDING = 0xFFFFFFFCu;
RL_DEV void g_lead_exotic(const GS& g, uint32_t k, const DevRule* __restrict__ rules, const TableDesc& tab,
                          EngineCtl* ctl) {
  Slot* slot = reinterpret_cast<Slot*>(g.rec[k].key);
  const uint32_t s = g.grp[k];
  const uint32_t n = g.cnt[s] & CNT_MASK, e0 = g.end[s] - n;
  const uint32_t region = key_region(slot->key);
  const uint32_t ws = region_ws(region, ctl->gen_max[region]);
  KeyState ks = read_state(slot);
  exotic_sequence(
      ks, tab, rules, n,
      [&](uint32_t q) {
        const MRec& m = g.rec[g.list[e0 + q]];
        return SeqItem{m.req, ws + (m.rn >> V4_RULE_BITS), m.h, rule_of(m.rn), mrec_jit(m.fp_lo)};
      },
      [&](uint32_t q, uint64_t v) { g.P[g.list[e0 + q]] = v; });
  write_state(slot, ks);
  g.rec[k].key = 0;
  g.rec[k].fp_lo = SEG_EXOTIC;
}

// Run by the key's last record: table probe/claim, INCRBY of the key's whole sequence in
// serial order, EXPIRE, local-cache freeze (fixed_cache_impl.go:55-123, base_limiter.go:88-106).
// Leaves the counter before the batch in rec[k].key and the freeze in rec[k].fp_lo; an exotic
// key (a string shared by units of different sizes whose expiry falls inside the batch)
// leaves per-position replies in P (SEG_EXOTIC). New slots are counted per region in ins[].
RL_DEV void g_lead(const GS& g, uint32_t k, const DevRule* __restrict__ rules, const TableDesc& tab, HotCand* cand,
                   EngineCtl* ctl, const uint32_t* s_gen, bool has_pre, const SlotView& pre, int cand_on,
                   uint32_t& heads, uint64_t& ins) {
  // k: the position that claimed the key's hash slot (any record of the key); the key's
  // results go to its last record (tail), where the decisions read them
  const uint64_t key = g.rec[k].key, lo = g.rec[k].fp_lo;
  const uint32_t rule = rule_of(g.rec[k].rn);
  const uint32_t s = g.grp[k];
  const uint32_t cw = g.cnt[s];
  const uint32_t n = cw & CNT_MASK, e1 = g.end[s], e0 = e1 - n;
  const uint32_t tail = g.list[e1 - 1];
  const bool mixed = (cw & CNT_MIXED) != 0, mixed_unit = (cw & CNT_MIXED_UNIT) != 0;
  const uint64_t Pk = g.P[tail];
  const DevRule R0 = rules[rule];
  heads += 1;
  if (cand_on && n >= HOT_MIN_SEG && !mixed) emit_cand_sc1(ctl, cand, rule, n, g.rec[g.list[e0]].idx);
  const uint32_t region = key_region(key);
  const uint32_t gen = s_gen[region];  // the region's one generation (k4_scan; staged in LDS)
  const uint32_t ws = region_ws(region, gen);
  Slot* slot = nullptr;
  bool existed = false;
  KeyState ks{0, 0, 0, 0};
  const bool claimed = has_pre ? table_claim_pre(tab, key, lo, gen, pre, slot, existed, ks)
                               : table_claim(tab, key, lo, gen, slot, existed, ks);
  if (!claimed) {
    atomicOr(&ctl->err, ERR_TABLE_FULL);  // unreachable below the load limit
    g.rec[tail].key = 0;
    g.rec[tail].fp_lo = SEG_NO_FREEZE;
    return;
  }
  if (!existed) {
    slot_reset(slot, key);
    heads += 1u << 16;
    ins += 1ull << (8 * region);  // per-region new-slot counts, 8 bits each (reduced per block)
  }
  const bool ps = per_second_store(tab, R0.unit);
  uint64_t base = 0;
  bool frozen_pre = false;
  if (mixed_unit || !fast_state(ks, ps, tab.local_cache != 0, ws, R0.div, base, frozen_pre)) {
    // exact sequential path, in a pass of its own after the leaders (g_lead_exotic); the tail
    // record keeps its jitter in fp_lo's high half
    g.rec[tail].key = (uint64_t)(uintptr_t)slot;
    g.rec[tail].fp_lo = (g.rec[tail].fp_lo & ~0xFFFFFFFFull) | SEG_EXOTIC_PENDING;
    return;
  }
  uint32_t freeze = SEG_NO_FREEZE;
  uint64_t final_count = base + Pk;
  uint32_t last = tail;  // the key's last record whose INCRBY happens
  if (frozen_pre) {
    freeze = SEG_FROZEN_BEFORE;  // every descriptor is a local-cache hit: no INCRBY
  } else if (tab.local_cache) {
    // the first record (arrival order) whose INCRBY reply exceeds its limit freezes the key;
    // the INCRBYs of its own request still happen (all lookups precede the Sets)
    uint32_t estar = e1;
    if (!mixed && base + Pk < (1ull << 32)) {
      // one limit, no wrap: after = base + P rises along the list, binary search
      if (base + Pk > (uint64_t)R0.L) {
        uint32_t a = e0, b = e1 - 1;
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (base + g.P[g.list[mid]] > (uint64_t)R0.L) b = mid; else a = mid + 1;
        }
        estar = a;
      }
    } else {
      for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t j = g.list[e];
        if ((uint32_t)(base + g.P[j]) > rules[rule_of(g.rec[j].rn)].L) { estar = e; break; }
      }
    }
    if (estar < e1) {
      const uint32_t rstar = g.rec[g.list[estar]].req;
      uint32_t f = estar;
      while (f + 1 < e1 && g.rec[g.list[f + 1]].req == rstar) ++f;
      last = g.list[f];
      freeze = rstar;
      final_count = base + g.P[last];
    }
  }
  if (freeze != SEG_FROZEN_BEFORE) {
    const uint32_t t_last = ws + (g.rec[last].rn >> V4_RULE_BITS);
    if (ps) {
      ks.pcount = (uint32_t)final_count;
    } else {
      ks.count = (uint32_t)final_count;
      // EXPIRE key div + jitter of the last INCRBY (fixed_cache_impl.go:69-72)
      ks.exp = t_last + R0.div + mrec_jit(g.rec[last].fp_lo);
    }
    if (freeze != SEG_NO_FREEZE) ks.frz = t_last + R0.div;  // freecache TTL (base_limiter.go:102)
    write_state(slot, ks);
  }
  g.rec[tail].key = base;
  g.rec[tail].fp_lo = freeze;
}

// All phases of one staged range of m records (whole keys). Returns the keys led (low 16
// bits) and the new table slots claimed (high 16 bits) by this thread.
template <bool LDS>
RL_DEV uint32_t group_range(const GS& g, uint32_t m, const DevRule* __restrict__ rules, const TableDesc& tab,
                            rl_status* __restrict__ out, uint32_t* __restrict__ req_thr, HotCand* cand, int cand_on,
                            int routed, LSeg* s_agg, LSeg* s_carry, uint32_t* sh_w, uint64_t& ins, EngineCtl* ctl,
                            const uint32_t* s_gen) {
  const uint32_t tid = threadIdx.x, wave = tid >> 6;
  uint32_t heads = 0;
  // Insert every position into the LDS hash; the position that claims a key's hash slot leads
  // the key and reads its first table slot right away, so the leader's probe overlaps the
  // grouping (one table read-ahead per key, not per record).
  constexpr int KPT = (BUCKET_CAP + G_NT - 1) / G_NT;  // positions per thread (global path)
  static_assert(KPT <= 8 && G_IPT <= KPT, "owner bits");
  uint32_t own = 0;  // bit j: position tid + j * G_NT leads its key
  SlotView pre[G_IPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t k = tid + j * G_NT;
    if (k < m && g_insert(g, k, rules)) own |= 1u << j;
  }
  if constexpr (LDS) {
    // every thread issues G_IPT slot loads at once, a position that leads no key reading the
    // table's first slot instead (no branch around a load: a load under a condition made the
    // compiler wait for it at the merge point, one table round trip per position)
#pragma unroll
    for (int j = 0; j < G_IPT; ++j) {
      const uint32_t k = min(tid + (uint32_t)j * G_NT, (uint32_t)G_CAP - 1u);
      const Slot* a = ((own >> j) & 1u) ? slot_first(tab, g.rec[k].key) : tab.slots;
      pre[j] = load_slot(a);
    }
  }
  gbar<LDS>();
  ST4(1);
  // each key's list start: exclusive prefix of the per-slot counts (hash-slot order)
  {
    const uint32_t spt = g.hs / G_NT, s0 = tid * spt;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < spt; ++q) sum += g.cnt[s0 + q] & CNT_MASK;
    uint32_t tot;
    uint32_t run = tile::block_excl_scan<G_NT>(sum, sh_w, tot);
    for (uint32_t q = 0; q < spt; ++q) {
      g.end[s0 + q] = (uint16_t)run;
      run += g.cnt[s0 + q] & CNT_MASK;
    }
  }
  gbar<LDS>();
  ST4(6);
  if (wave == 0) g_layout(g, m);
  gbar<LDS>();
  ST4(7);
  g_scan<LDS>(g, m, s_agg, s_carry);
  gbar<LDS>();
  ST4(3);
  if constexpr (LDS) {
#pragma unroll
    for (int j = 0; j < G_IPT; ++j)
      if ((own >> j) & 1u) g_lead(g, tid + j * G_NT, rules, tab, cand, ctl, s_gen, true, pre[j], cand_on, heads, ins);
  } else {
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if ((own >> j) & 1u)
        g_lead(g, tid + j * G_NT, rules, tab, cand, ctl, s_gen, false, SlotView{}, cand_on, heads, ins);
  }
  __threadfence_block();
  __syncthreads();
  // exotic keys (rare): their leaders' sequential pass
  for (uint32_t k = tid; k < m; k += G_NT)
    if ((uint32_t)g.rec[k].fp_lo == SEG_EXOTIC_PENDING && g_tail(g, k) == k) g_lead_exotic(g, k, rules, tab, ctl);
  __threadfence_block();
  __syncthreads();
  ST4(4);
  for (uint32_t k = tid; k < m; k += G_NT) {
    const MRec x = g.rec[k];
    const uint32_t t = g_tail(g, k);
    const MRec& lt = g.rec[t];
    tile::decide_at(x.idx, x.req, rule_of(x.rn), x.h, x.rn >> V4_RULE_BITS, lt.key, g.P[k], (uint32_t)lt.fp_lo, rules,
                  out, req_thr, routed);
  }
  return heads;
}

// ---------------------------------------------------------------------------
// k4_place — per tile (tile-sorted records): hot descriptors decided in place. MSD records
// stay where k4_hist wrote them; k4_group gathers its ranges from the tile runs.
// ---------------------------------------------------------------------------
// LR: the rule table (n_rules <= LDS_RULES) is staged in LDS (every hot descriptor's decision
// reads its rule).
constexpr uint32_t LDS_RULES = 32;
template <bool LR>
__global__ __launch_bounds__(NT) void k4_place(DevBatch in, const MRec* __restrict__ srec,
                                               const uint16_t* __restrict__ tstart,
                                               const uint32_t* __restrict__ ranges,
                                               const DevRule* __restrict__ rules_g, uint32_t n_rules,
                                               const unsigned long long* __restrict__ hoff,
                                               HotBucket* __restrict__ hb, int local_cache,
                                               rl_status* __restrict__ out,
                                               uint32_t* __restrict__ req_thr, Deferred* __restrict__ dfr, int routed,
                                               uint32_t* __restrict__ poison, EngineCtl* ctl) {
  __shared__ __attribute__((aligned(16))) uint16_t s_row[HOT_BUCKETS + 8];
  __shared__ uint32_t s_rstar[HOT_BUCKETS];
  __shared__ uint32_t s_err;
  __shared__ DevRule s_rules[LR ? LDS_RULES : 1];
  const DevRule* __restrict__ rules = LR ? s_rules : rules_g;
  const uint32_t tid = threadIdx.x;
  const uint32_t t = blockIdx.x, t0 = t * T;
  if (tid == 0) s_err = ctl->err;
  if (LR && tid >= 64 && tid < 64 + n_rules) s_rules[tid - 64] = rules_g[tid - 64];
  {  // the hot part of the tile's row of bucket starts (MSD records stay where k4_hist put
     // them: k4_group gathers its ranges from the tile-sorted records)
    const uint32_t* rsrc = reinterpret_cast<const uint32_t*>(tstart + (size_t)t * ROW);
    for (int k = tid; k < (HOT_BUCKETS + 8) / 2; k += NT) reinterpret_cast<uint32_t*>(s_row)[k] = rsrc[k];
  }
  if (local_cache)
    for (int b = tid; b < HOT_BUCKETS; b += NT) s_rstar[b] = 0xFFFFFFFFu;
  __syncthreads();
  // A batch the engine will rerun on the LSD pipeline poisons the next batch's k4_scan.
  if (t == 0 && tid == 0 && (s_err & ERR_FALLBACK) && !(s_err & (ERR_BAD_INPUT | ERR_BAD_TIME))) *poison = 1u;
  // Nothing is decided and nothing touches the table unless the whole batch is valid.
  if (s_err) return;
  // Hot keys without a freeze in this batch: the final counter is base + total (spread over
  // the blocks, about one bucket each, so no block carries the whole loop).
  for (uint32_t b = t + tid * gridDim.x; b < (uint32_t)HOT_BUCKETS; b += NT * gridDim.x) {
    const HotBucket x = hb[b];
    if (!x.slot || (x.flags & HB_FROZEN_PRE)) continue;
    if (!local_cache || x.base + x.total <= (uint64_t)rules[x.rule].L) *hot_counter(x) = (uint32_t)(x.base + x.total);
  }
  const uint32_t nhot = s_row[HOT_BUCKETS];
  const MRec* src = srec + t0;
  const unsigned long long* hrow = hoff + (size_t)t * HOT_BUCKETS;
  if (nhot == 0) return;  // block-uniform
  if (local_cache) {
    // The descriptor whose INCRBY reply first exceeds the limit freezes the key
    // (base_limiter.go:94-106). The post-value is monotone (k4_scan), so it is the unique
    // descriptor with after > L >= before, or the key's first descriptor of the batch.
    for (uint32_t p = tid; p < nhot; p += NT) {
      const MRec a = src[p];
      const uint32_t b = (uint32_t)a.fp_lo;
      const HotBucket& x = hb[b];
      if (x.flags & HB_FROZEN_PRE) continue;
      const uint64_t P = hrow[b] + a.key;
      const uint64_t after = x.base + P;
      const uint32_t L = rules[rule_of(a.rn)].L;
      if (after > L && (after - a.h <= L || P == a.h)) {
        s_rstar[b] = a.req;
        hb[b].rstar = a.req;
        hb[b].t_rstar = x.ws + (a.rn >> V4_RULE_BITS);  // the freecache Set's time (k4_group finalises)
      }
    }
    __syncthreads();
  }
  const uint32_t q0 = in.recs ? in.recs[t0].greq : in.req_of[t0];  // request of the tile's first descriptor
  for (uint32_t p = tid; p < nhot; p += NT) {
    const MRec a = src[p];
    const uint32_t b = (uint32_t)a.fp_lo;
    const uint32_t rule = rule_of(a.rn), now_mod = a.rn >> V4_RULE_BITS;
    const uint32_t i = a.idx;
    const unsigned long long P = hrow[b] + a.key;
    const HotBucket& hx = hb[b];
    const DevRule& rl = rules[rule];
    if (hx.flags & HB_FROZEN_PRE) {
      tile::emit_local_hit(out, i, a.h, rl.div - now_mod, rl.shadow, routed);  // every descriptor is a local-cache hit
      continue;
    }
    const uint64_t after = hx.base + P;
    if (!local_cache || after <= rl.L) {
      tile::decide_at(i, a.req, rule, a.h, now_mod, hx.base, P, SEG_NO_FREEZE, rules, out, req_thr, routed);
      // the key's last INCRBY: EXPIRE at its time + div + its jitter
      if (P == hx.total) hb[b].t_all = hx.ws + now_mod + mrec_jit(a.fp_lo);
      continue;
    }
    const uint32_t rs = s_rstar[b];
    if (rs != 0xFFFFFFFFu) {  // the freezing descriptor is in this tile, at or before this one
      if (a.req > rs) {
        tile::emit_local_hit(out, i, a.h, rl.div - now_mod, rl.shadow, routed);
      } else {  // same request as the freezing descriptor: its INCRBY still happens
        tile::decide_at(i, a.req, rule, a.h, now_mod, hx.base, P, SEG_NO_FREEZE, rules, out, req_thr, routed);
        atomicMax(hot_counter(hx), (uint32_t)after);
        atomicMax(&hot_exp(hb)[b], ((unsigned long long)i << 32) | mrec_jit(a.fp_lo));  // the last of them sets EXPIRE
      }
    } else if (a.req > q0) {  // froze in an earlier tile, in a request <= q0
      tile::emit_local_hit(out, i, a.h, rl.div - now_mod, rl.shadow, routed);
    } else {  // a request that began in an earlier tile: decided by k4_group
      const uint32_t e = atomicAdd(&ctl->tile_ctr[DFR_CTR][0], 1u);
      Deferred df;
      df.P = P;
      df.idx = i;
      df.bucket = b | (mrec_jit(a.fp_lo) << 16);
      df.req = a.req;
      df.h = a.h;
      df.rule = rule;
      df.now_mod = now_mod;
      dfr[e] = df;
    }
  }
}

// ---------------------------------------------------------------------------
// k4_group — one block per range of whole MSD buckets (k4_scan packs them to fit LDS; a
// bucket larger than the stage is gathered into the block's global scratch and grouped there
// by fingerprint half). Every block also
// decides a share of the deferred hot descriptors; the last block to finish counts U, fills
// the hot-set candidates and clears the next batch's control block.
// ---------------------------------------------------------------------------
struct GScratch4 {
  MRec* rec;       // [GBLOCKS][BUCKET_CAP] an oversized bucket's records, gathered
  uint64_t* P;     // [GBLOCKS][BUCKET_CAP]
  uint16_t* list;  // [GBLOCKS][BUCKET_CAP]
  uint16_t* grp;   // [GBLOCKS][BUCKET_CAP]
  uint32_t* slot;  // [GBLOCKS][GS_HASH]
  uint32_t* cnt;   // [GBLOCKS][GS_HASH]
  uint16_t* end;   // [GBLOCKS][GS_HASH]
  uint32_t* cursor;  // [GBLOCKS]
};

// The records of MSD buckets [B0, B1) in arrival order, gathered straight from the
// tile-sorted records k4_hist wrote: inside a tile the range is one contiguous run, and runs
// taken tile by tile keep every key's records in arrival order (a key lives in one bucket).
// dst[0, m): the LDS stage or a block's global scratch. GATHER_T tiles per chunk: their run
// starts and exclusive prefix in LDS, then every output position finds its tile by binary
// search and all of a thread's record loads are in flight together.
constexpr int GATHER_T = 512;
constexpr int GATHER_TPT = GATHER_T / G_NT;
template <int PPT, int CAP>  // output positions per thread; dst holds CAP <= PPT * G_NT records
RL_DEV uint32_t gather_runs(const MRec* __restrict__ srec, const uint16_t* __restrict__ tstart, uint32_t ntiles,
                            uint32_t B0, uint32_t B1, MRec* dst, uint16_t* s_ra, uint16_t* s_pre, uint32_t* sh_w) {
  const uint32_t tid = threadIdx.x;
  uint32_t done = 0;
  for (uint32_t c0 = 0; c0 < ntiles; c0 += GATHER_T) {
    const uint32_t nt = min((uint32_t)GATHER_T, ntiles - c0);
    uint32_t a[GATHER_TPT], l[GATHER_TPT], sum = 0;
#pragma unroll
    for (int q = 0; q < GATHER_TPT; ++q) {  // clamped tiles: the loads go out together
      const uint32_t t = tid * GATHER_TPT + q;
      const uint16_t* row = tstart + (size_t)(c0 + min(t, nt - 1u)) * ROW;
      const uint32_t x0 = row[B0], x1 = row[B1];
      a[q] = x0;
      l[q] = t < nt ? x1 - x0 : 0u;
      sum += l[q];
    }
    uint32_t tot;
    uint32_t run = tile::block_excl_scan<G_NT>(sum, sh_w, tot);
#pragma unroll
    for (int q = 0; q < GATHER_TPT; ++q) {
      s_ra[tid * GATHER_TPT + q] = (uint16_t)a[q];
      s_pre[tid * GATHER_TPT + q] = (uint16_t)run;
      run += l[q];
    }
    __syncthreads();
    if (tot) {  // block-uniform
      // the last tile whose prefix is <= p holds p (zero-length runs share a prefix with the
      // next tile); all PPT searches step together, one LDS read each per halving
      uint32_t p[PPT], lo[PPT];
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        p[u] = min(tid + u * G_NT, tot - 1u);
        lo[u] = 0;
      }
#pragma unroll
      for (uint32_t step = GATHER_T / 2; step >= 1; step >>= 1)
#pragma unroll
        for (int u = 0; u < PPT; ++u) lo[u] = s_pre[lo[u] + step] <= p[u] ? lo[u] + step : lo[u];
      MRec v[PPT];
#pragma unroll
      for (int u = 0; u < PPT; ++u) v[u] = srec[(size_t)(c0 + lo[u]) * T + s_ra[lo[u]] + (p[u] - s_pre[lo[u]])];
#pragma unroll
      for (int u = 0; u < PPT; ++u)
        if (tid + u * G_NT < tot && done + p[u] < (uint32_t)CAP) dst[done + p[u]] = v[u];
    }
    done += tot;
    __syncthreads();  // s_ra / s_pre of the next chunk
  }
  return done;
}

// LR: the rule table (n_rules <= LDS_RULES) is staged in LDS; the leaders and the decisions
// read a rule per key / per record.
template <bool LR>
__global__ __launch_bounds__(G_NT, RL_G_OCC) void k4_group(DevBatch in,
                                                 const DevRule* __restrict__ rules_g, TableDesc tab,
                                                 rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                                                 const HotBucket* __restrict__ hb, const Deferred* __restrict__ dfr,
                                                 HotCand* __restrict__ cand, int cand_on, uint64_t seed,
                                                 GScratch4 gs, uint32_t* __restrict__ wg_heads,
                                                 uint32_t* __restrict__ wg_ins,
                                                 const uint32_t* __restrict__ scan_heads,
                                                 const uint32_t* __restrict__ scan_ins, uint32_t n_scan_heads,
                                                 const uint32_t* __restrict__ ranges, int routed,
                                                 RegionOcc* __restrict__ occ, EngineCtl* ctl, EngineCtl* next_ctl,
                                                 EngineCtl* hctl, HotCand* hcand,
                                                 const MRec* __restrict__ srec, const uint16_t* __restrict__ tstart,
                                                 uint32_t ntiles, uint32_t n_rules) {
  __shared__ DevRule s_rules[LR ? LDS_RULES : 1];
  const DevRule* __restrict__ rules = LR ? s_rules : rules_g;
  __shared__ MRec s_rec[G_CAP];
  __shared__ uint64_t s_P[G_CAP];
  static_assert(sizeof(uint64_t) * G_CAP >= 4 * GATHER_T, "the gather's run tables alias s_P");
  uint16_t* const s_ra = reinterpret_cast<uint16_t*>(s_P);  // only while a range is gathered
  uint16_t* const s_pre = s_ra + GATHER_T;
  __shared__ uint16_t s_list[G_CAP];
  __shared__ uint16_t s_grp[G_CAP];
  __shared__ uint32_t s_slot[G_HASH];
  __shared__ uint32_t s_cnt[G_HASH];
  __shared__ uint16_t s_end[G_HASH];
  __shared__ LSeg s_agg[G_W];
  __shared__ LSeg s_carry;
  __shared__ uint32_t s_cursor, s_heads, s_last, s_err;
  __shared__ uint32_t s_rq[6];  // this block's group: range count, entries of its first two ranges; deferred count
  __shared__ uint32_t sh_w[G_W];
  __shared__ uint32_t s_ins[8];
  __shared__ uint32_t s_gen[8];  // per region the batch's window generation (k4_scan)
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t j = blockIdx.x;
  uint32_t heads = 0;
  uint64_t ins = 0;  // new slots per region, 8 bits each
  if (tid < 8) s_ins[tid] = 0;
  // Block j takes ranges q = j / MSD_GROUPS, + RPG, ... of MSD group g = j % MSD_GROUPS (no
  // prefix over the groups first): the group's range count and the entries of the block's
  // first two ranges are loaded together with the error word and the deferred count.
  const uint32_t g = j % MSD_GROUPS, q0 = j / MSD_GROUPS;
  const uint32_t* rb = ranges + R_START + g * (RANGE_MAX + 1);
  if (tid < 6) {
    const uint32_t i2 = min(q0 + RPG, (uint32_t)RANGE_MAX - 1u);
    s_rq[tid] = tid == 0 ? ranges[g] : tid == 1 ? rb[q0] : tid == 2 ? rb[q0 + 1] : tid == 3 ? rb[i2]
              : tid == 4 ? rb[i2 + 1] : ctl->tile_ctr[DFR_CTR][0];
  }
  if (tid == 0) {
    s_heads = 0;
    s_err = ld_relaxed(&ctl->err);
  }
  if (tid >= 8 && tid < 16) s_gen[tid - 8] = ctl->gen_max[tid - 8];
  if (LR && tid >= 32 && tid < 32 + n_rules) s_rules[tid - 32] = rules_g[tid - 32];
  __syncthreads();
  ST4(0);
#ifdef RL_STAMPS
  if (tid == 0 && j < 1024) for (int k = 0; k < 8; ++k) g_st4[3072 + j][k] = 0;  // this batch's facts only
#endif
  if (s_err == 0 && j < (uint32_t)(HOT_BUCKETS / G_NT)) {
    // Hot keys (decided by k4_place) that no request froze: EXPIRE from the time and jitter of
    // the last INCRBY (fixed_cache_impl.go:69-72). A key frozen in this batch gets its EXPIRE and
    // freecache TTLs in the last block, once the deferred hot descriptors below have recorded
    // which INCRBY of the freezing request came last.
    const HotBucket x = hb[j * G_NT + tid];
    if (x.slot && !(x.flags & (HB_FROZEN_PRE | HB_PS)) && x.rstar == 0xFFFFFFFFu) {
      Slot* sl = reinterpret_cast<Slot*>(x.slot);
      sl->exp = x.t_all + rules[x.rule].div;
    }
  }
  if (s_err == 0) {
    // Hot descriptors of a request that began before the tile where their key froze
    // (k4_place, a previous launch, recorded them and the freezing requests).
    const uint32_t nd = s_rq[5];
    for (uint32_t e = j * G_NT + tid; e < nd; e += gridDim.x * G_NT) {
      const Deferred df = dfr[e];
      const uint32_t bk = df.bucket & 0xFFFFu;
      const HotBucket& x = hb[bk];
      if (df.req > x.rstar) {
        tile::emit_local_hit(out, df.idx, df.h, rules[df.rule].div - df.now_mod, rules[df.rule].shadow, routed);
      } else {
        tile::decide_at(df.idx, df.req, df.rule, df.h, df.now_mod, x.base, df.P, SEG_NO_FREEZE, rules, out, req_thr,
                      routed);
        atomicMax(hot_counter(x), (uint32_t)(x.base + df.P));
        atomicMax(&hot_exp(hb)[bk], ((unsigned long long)df.idx << 32) | (df.bucket >> 16));
      }
    }
    const uint32_t nq = s_rq[0];  // ranges of group g
    for (uint32_t q = q0, it = 0; q < nq; q += RPG, ++it) {
      // Range entries are bucket << 1 | half (see k4_scan): [e0, e1) is whole buckets, or one
      // fingerprint half of an oversized bucket (e0 odd: half 1; e1 == e0 | 1: half 0).
      const uint32_t e0 = it == 0 ? s_rq[1] : it == 1 ? s_rq[3] : rb[q];
      const uint32_t e1 = it == 0 ? s_rq[2] : it == 1 ? s_rq[4] : rb[q + 1];
      const int split_half = (e0 & 1u) ? 1 : (e1 == (e0 | 1u) ? 0 : -1);
      const uint32_t k0 = e0 >> 1, k1 = split_half >= 0 ? k0 + 1u : e1 >> 1;
      const uint32_t B0 = HOT_BUCKETS + g * 64u + k0, B1 = HOT_BUCKETS + g * 64u + k1;
      __syncthreads();  // the previous range is done with LDS
      if (split_half < 0) {  // whole buckets: at most G_CAP records (k4_scan's packing)
        for (uint32_t s = tid; s < (uint32_t)G_HASH; s += G_NT) {
          s_slot[s] = G_EMPTY;
          s_cnt[s] = 0;
        }
        if (tid == 0) s_cursor = 0;
        const uint32_t m = gather_runs<G_IPT, G_CAP>(srec, tstart, ntiles, B0, B1, s_rec, s_ra, s_pre, sh_w);
        if (m == 0) continue;  // block-uniform
        if (m > (uint32_t)G_CAP) {  // unreachable: k4_scan packs whole buckets up to G_CAP
          if (tid == 0) atomicOr(&ctl->err, ERR_SPIN);
          continue;
        }
        __syncthreads();
        ST4(2);
        const GS gl{s_rec, s_P, s_list, s_grp, s_slot, s_cnt, s_end, &s_cursor, G_HASH};
        {
          const uint32_t hh = group_range<true>(gl, m, rules, tab, out, req_thr, cand, cand_on, routed, s_agg,
                                                &s_carry, sh_w, ins, ctl, s_gen);
          heads += hh;
          ST4X(0, m);
          ST4X(1, hh & 0xFFFFu);
          ST4X(2, 1);
        }
        continue;
      }
      // One bucket larger than the LDS stage. Its keys split by the fingerprint bit below the
      // bucket bits into two halves of whole keys; each half that fits is grouped in LDS.
      ST4X(3, 1);
      constexpr int SPLIT_BIT = 64 - 3 - MSD_BITS - 1;
      constexpr int SU = BUCKET_CAP / G_NT;
      MRec* const src = gs.rec + (size_t)j * BUCKET_CAP;  // the bucket, gathered (<= BUCKET_CAP records)
      const uint32_t m = gather_runs<BUCKET_CAP / G_NT, BUCKET_CAP>(srec, tstart, ntiles, B0, B1, src, s_ra, s_pre, sh_w);
      ST4X(0, m);
      __threadfence_block();
      __syncthreads();
      auto half_of = [&](uint32_t k) -> uint32_t {
        return k < m ? (uint32_t)(__builtin_nontemporal_load(&src[k].key) >> SPLIT_BIT) & 1u : 2u;
      };
      uint32_t n0 = 0;
      for (int u = 0; u < SU; ++u) n0 += half_of(tid + u * G_NT) == 0u;
      uint32_t tot0;
      tile::block_excl_scan<G_NT>(n0, sh_w, tot0);
      if (tot0 <= (uint32_t)G_CAP && m - tot0 <= (uint32_t)G_CAP) {
        // a split range takes its own half (the other half is another block's range)
        for (uint32_t part = split_half == 1 ? 1u : 0u; part < (split_half == 0 ? 1u : 2u); ++part) {
          __syncthreads();  // the previous half is done with LDS
          for (uint32_t s = tid; s < (uint32_t)G_HASH; s += G_NT) {
            s_slot[s] = G_EMPTY;
            s_cnt[s] = 0;
          }
          // compact the half's records in position (= arrival) order: one block scan per
          // 256-position chunk
          uint32_t mp = 0;
          for (int u = 0; u < SU; ++u) {
            const uint32_t k = tid + u * G_NT;
            const bool mine = half_of(k) == part;
            uint32_t ct;
            const uint32_t pos = mp + tile::block_excl_scan<G_NT>(mine ? 1u : 0u, sh_w, ct);
            if (mine) s_rec[pos] = src[k];
            mp += ct;
          }
          if (tid == 0) s_cursor = 0;
          __syncthreads();
          if (mp == 0) continue;
          const GS gl{s_rec, s_P, s_list, s_grp, s_slot, s_cnt, s_end, &s_cursor, G_HASH};
          heads += group_range<true>(gl, mp, rules, tab, out, req_thr, cand, cand_on, routed, s_agg, &s_carry,
                                     sh_w, ins, ctl, s_gen);
        }
      } else if (split_half != 1) {
        // grouped in place in bucket order (global scratch); for a split bucket by its half-0
        // range's block (the half-1 block has nothing to do)
        const GS gg{src,                              gs.P + (size_t)j * BUCKET_CAP,
                    gs.list + (size_t)j * BUCKET_CAP,  gs.grp + (size_t)j * BUCKET_CAP,
                    gs.slot + (size_t)j * GS_HASH,     gs.cnt + (size_t)j * GS_HASH,
                    gs.end + (size_t)j * GS_HASH,      gs.cursor + j,
                    GS_HASH};
        for (uint32_t s = tid; s < (uint32_t)GS_HASH; s += G_NT) {
          gg.slot[s] = G_EMPTY;
          gg.cnt[s] = 0;
        }
        if (tid == 0) *gg.cursor = 0;
        __threadfence_block();
        __syncthreads();
        heads += group_range<false>(gg, m, rules, tab, out, req_thr, cand, cand_on, routed, s_agg, &s_carry,
                                    sh_w, ins, ctl, s_gen);
      }
    }
  }
  heads = tile::wave_sum(heads);
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t c = tile::wave_sum((uint32_t)(ins >> (8 * r)) & 0xFFu);
    if (lane == 0 && c) atomicAdd(&s_ins[r], c);
  }
  __syncthreads();
  if (lane == 0 && heads) atomicAdd(&s_heads, heads);
  __syncthreads();
  ST4(5);
  // The last block to finish: U, hot-set candidates, next control block. Hand-off without
  // fences: every wave waits for its own stores (the sc1 ones the last block reads among
  // them), then one lane adds to the block's shard counter (blockIdx & 7); the last block of a
  // shard adds to the global counter; the last of those is the last block.
  if (tid == 0) st_relaxed(&wg_heads[j], s_heads);
  if (tid < 4) st_relaxed(&wg_ins[j * 4 + tid], s_ins[2 * tid] | (s_ins[2 * tid + 1] << 16));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t shard = j & 7u;
    const uint32_t per = (gridDim.x - shard + 7u) / 8u;  // blocks of this shard
    bool last = atomicAdd(&ctl->tile_ctr[SHARD_CTR0 + shard][0], 1u) == per - 1u;
    if (last) {
      const uint32_t shards = gridDim.x < 8u ? gridDim.x : 8u;
      last = atomicAdd(&ctl->tile_ctr[DONE_CTR][0], 1u) == shards - 1u;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  STL(0);
  // U = Σ per-block unique-key counts (this kernel and k4_scan's hot leaders); new slots per
  // region into the occupancy counts (only for a batch that was applied); the hot-set
  // candidates' prefix states. Every load the epilogue needs goes out first, in three
  // dependent levels: (block words, candidates, occupancy) -> (candidates' prefix offsets or
  // routed records) -> (prefix bytes).
  if (tid == 0) s_heads = 0;
  if (tid < 8) s_ins[tid] = 0;
  constexpr int EPI = (GBLOCKS + HOT_SCAN_BLOCKS + G_NT - 1) / G_NT;
  constexpr int CPT = CAND_MAX / G_NT;  // candidate entries per thread
  static_assert(CAND_MAX % G_NT == 0, "candidates per thread");
  const uint32_t nb = gridDim.x + n_scan_heads;
  uint32_t hv[EPI], w[EPI][4];
  HotCand cc[CPT];
  // k4_scan's hot blocks wrote their words right behind this kernel's (the engine passes
  // scan_heads = wg_heads + gridDim.x, scan_ins = wg_ins + 4 * gridDim.x): every thread loads
  // all of its blocks' five words at once (clamped indices), then DPP sums per wave
#pragma unroll
  for (int e = 0; e < EPI; ++e) {
    const uint32_t k = min(tid + e * G_NT, nb - 1u);
    hv[e] = ld_relaxed(&wg_heads[k]);
#pragma unroll
    for (int x = 0; x < 4; ++x) w[e][x] = ld_relaxed(&wg_ins[k * 4 + x]);
  }
  // candidates only for a batch whose candidates the host wants (hcand set: every 8th batch)
  const bool do_cand = hcand != nullptr;  // kernel-uniform
  if (do_cand) {
#pragma unroll
    for (int e = 0; e < CPT; ++e) ld_sc1_32B(&cc[e], &cand[tid + e * G_NT]);  // unused entries: stale
  }
  const uint32_t nc = min((uint32_t)CAND_MAX, ld_relaxed(&ctl->tile_ctr[CAND_CTR][0]));
  const uint32_t gm = ctl->gen_max[tid & 7u];
  RegionOcc ro = occ[tid & 7u];
  // the control block's header words for the host's copy (k4_scan's and the blocks' words are
  // final: every block's stores completed before it counted itself done)
  const uint32_t hdr = ld_relaxed(reinterpret_cast<const uint32_t*>(ctl) + (tid & 63u));
  __syncthreads();  // s_heads / s_ins cleared
  {
    uint32_t u = 0, cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < EPI; ++e) {
      if (tid + e * G_NT >= nb) continue;
      u += hv[e] & 0xFFFFu;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        cs[2 * x] += w[e][x] & 0xFFFFu;
        cs[2 * x + 1] += w[e][x] >> 16;
      }
    }
    u = tile::wave_sum(u);
    if (lane == 0 && u) atomicAdd(&s_heads, u);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t c = tile::wave_sum(cs[r]);
      if (lane == 0 && c) atomicAdd(&s_ins[r], c);
    }
  }
  // candidates found by k4_group leaders carry their first descriptor: its prefix offsets (or
  // the routed record's prefix state), all loads in flight together
  uint32_t po[CPT] = {}, pl[CPT] = {};
  uint64_t ra[CPT] = {}, rbv[CPT] = {};
  const bool any_cand = do_cand && nc > 0 && in.n_desc > 0;  // block-uniform
#pragma unroll
  for (int e = 0; e < CPT && any_cand; ++e) {
    const uint32_t i = tid + e * G_NT;
    const uint32_t d = i < nc && cc[e].first_idx != 0xFFFFFFFFu ? min(cc[e].first_idx, in.n_desc - 1u) : 0u;
    if (in.recs) {  // routed batch (kernel-uniform)
      ra[e] = in.recs[d].a;
      rbv[e] = in.recs[d].b;
      po[e] = pl[e] = 0;
    } else {
      po[e] = in.off[d];
      pl[e] = in.off[d + 1u] - po[e];
      ra[e] = rbv[e] = 0;
    }
  }
  __syncthreads();
  if (tid < 8) {
    // one thread per region; also for a refused batch: its hot keys may have claimed slots in
    // k4_scan before the refusal (they hold the empty state; the rerun finds them)
    const uint32_t r = tid;
    ctl->ins[r] = s_ins[r];
    if (gm) {
      occ_advance(ro, lazy_region(tab.lag, r), gm, s_ins[r]);
      occ[r] = ro;
    }
  }
  if (tid == 8) {
    ctl->n_segments = s_heads;
    uint32_t n = 0;
    for (int r = 0; r < 8; ++r) n += s_ins[r];
    ctl->n_inserted = n;
  }
  STL(1);
  if (any_cand && !in.recs) {
    u32x4 b0[CPT], b1[CPT];
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      const u32x4* q = reinterpret_cast<const u32x4*>(in.blob + (po[e] & ~3u));
      b0[e] = q[0];
      b1[e] = q[1];
    }
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      const FpState st = prefix_state_pre(b0[e], b1[e], in.blob, po[e], pl[e], seed);
      ra[e] = st.a;
      rbv[e] = st.b;
    }
  }
#pragma unroll
  for (int e = 0; e < CPT && do_cand; ++e) {
    const uint32_t i = tid + e * G_NT;
    if (i >= nc) continue;
    HotCand c = cc[e];
    if (c.first_idx != 0xFFFFFFFFu) {  // a hot key's candidate already carries its state
      c.a = ra[e];
      c.b = rbv[e];
      c.unit = rules[c.rule].unit;
      cand[i] = c;
    }
    if (hcand) hcand[i] = c;
  }
  // The batch's summary straight into the host's pinned control block (header words and the
  // candidate count): no device-to-host copy between this batch and the next one's kernels.
  __syncthreads();  // ins / n_segments / n_inserted written above by threads 0..8
  if (hctl) {
    constexpr uint32_t HEAD = offsetof(EngineCtl, tile_ctr) / 4;
    static_assert(HEAD == 64 && offsetof(EngineCtl, n_segments) == 8 && offsetof(EngineCtl, n_inserted) == 12,
                  "header words");
    constexpr uint32_t INS0 = offsetof(EngineCtl, ins) / 4;
    uint32_t* hw = reinterpret_cast<uint32_t*>(hctl);
    if (tid < HEAD) {
      uint32_t v = hdr;
      if (tid == 2) v = s_heads;
      if (tid == 3) {
        v = 0;
        for (int r = 0; r < 8; ++r) v += s_ins[r];
      }
      if (tid >= INS0 && tid < INS0 + 8) v = s_ins[tid - INS0];
      hw[tid] = v;
    }
    if (tid == HEAD) hctl->tile_ctr[CAND_CTR][0] = nc;
    __threadfence_system();
  }
  // (here, where the epilogue's candidate registers are dead)
  if (tab.local_cache && s_err == 0) {
    // Hot keys a request froze in this batch (base_limiter.go:94-106): freecache TTL from the
    // freezing request's time, EXPIRE from the time and jitter of that request's last INCRBY of
    // the key (every block's k4_place / deferred atomicMax is done; read at the memory side)
    for (uint32_t b = tid; b < (uint32_t)HOT_BUCKETS; b += G_NT) {
      // field loads, not a copy of the 64-B bucket (which leaves a private-segment frame)
      const uint64_t slot = hb[b].slot;
      const uint32_t flags = hb[b].flags, rstar = hb[b].rstar;
      if (!slot || (flags & HB_FROZEN_PRE) || rstar == 0xFFFFFFFFu) continue;
      Slot* sl = reinterpret_cast<Slot*>(slot);
      const uint32_t t = hb[b].t_rstar + rules[hb[b].rule].div;
      const unsigned long long w = __hip_atomic_load(&hot_exp(hb)[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(flags & HB_PS)) sl->exp = t + (uint32_t)w;
      sl->frz = t;
    }
  }
  uint32_t* z = reinterpret_cast<uint32_t*>(next_ctl);
  constexpr uint32_t words = sizeof(EngineCtl) / 4;
  STL(2);
  for (uint32_t w = tid; w < words; w += G_NT) z[w] = 0;
  STL(3);
  if (hctl) {
    // The batch is complete: the host's done word behind its pinned control block, which
    // rl_wait polls in place of a completion event. Last, after the frozen keys and the clear
    // of batch k+2's control block, which batch k+2's k4_hist (launched once the host sees this
    // word) uses.
    __threadfence();
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(reinterpret_cast<uint32_t*>(hctl + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace v4

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
uint32_t v4_tiles(uint32_t n) { return n ? (n + V4_TILE - 1) / V4_TILE : 1; }
uint32_t v4_group_blocks(uint32_t) { return v4::GBLOCKS; }
uint32_t v4_scan_blocks() { return v4::HOT_SCAN_BLOCKS + v4::MSD_SCAN_BLOCKS; }
size_t v4_scratch_bytes() {
  using namespace v4;
  return (size_t)GBLOCKS * BUCKET_CAP * (sizeof(MRec) + 8 + 2 + 2) + (size_t)GBLOCKS * GS_HASH * (4 + 4 + 2) +
         (size_t)GBLOCKS * 4 + RANGE_WORDS * 4 + 1024;
}
static uint32_t* v4_ranges(void* scratch) {  // the last RANGE_WORDS words (+ slack) of the scratch
  return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(scratch) + v4_scratch_bytes() - 1024 -
                                     v4::RANGE_WORDS * 4);
}

void launch_v4_hist(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, uint64_t seed,
                    const HotEntry* hot, uint32_t* req_thr, uint32_t* fpart, uint16_t* tstart,
                    unsigned long long* thsum, MRec* srec, rl_status* out, EngineCtl* ctl) {
  const DevBatch in = make_dev_batch(b);
  if (in.recs)
    hipLaunchKernelGGL(v4::k4_hist<true>, dim3(v4_tiles(b.n_desc)), dim3(V4_THREADS), 0, st, in, rules, n_rules, seed,
                       hot, req_thr, fpart, tstart, thsum, srec, out, ctl);
  else
    hipLaunchKernelGGL(v4::k4_hist<false>, dim3(v4_tiles(b.n_desc)), dim3(V4_THREADS), 0, st, in, rules, n_rules,
                       seed, hot, req_thr, fpart, tstart, thsum, srec, out, ctl);
}
void launch_v4_scan(hipStream_t st, uint32_t n, const uint16_t* tstart, const unsigned long long* thsum,
                    unsigned long long* hoff, const uint32_t* fpart, const HotEntry* hot_list, HotBucket* hb,
                    const TableDesc& tab, HotCand* cand, uint32_t* heads_out, uint32_t* ins_out, void* scratch,
                    const uint32_t* poison, const RegionOcc* occ, EngineCtl* ctl) {
  hipLaunchKernelGGL(v4::k4_scan, dim3(v4_scan_blocks()), dim3(v4::SCAN_NT), 0, st, tstart, thsum, v4_tiles(n), n, hoff,
                     fpart, hot_list, hb, tab, cand, heads_out, ins_out, v4_ranges(scratch), poison, occ, ctl);
}
void launch_v4_place(hipStream_t st, const rl_batch& b, const MRec* srec, const uint16_t* tstart,
                     void* scratch, const DevRule* rules, uint32_t n_rules, const unsigned long long* hoff,
                     HotBucket* hb, int local_cache, rl_status* out, uint32_t* req_thr, Deferred* dfr, int routed,
                     uint32_t* poison, EngineCtl* ctl) {
  if (n_rules <= v4::LDS_RULES)
    hipLaunchKernelGGL(v4::k4_place<true>, dim3(v4_tiles(b.n_desc)), dim3(V4_THREADS), 0, st, make_dev_batch(b), srec,
                       tstart, v4_ranges(scratch), rules, n_rules, hoff, hb, local_cache, out, req_thr, dfr, routed,
                       poison, ctl);
  else
    hipLaunchKernelGGL(v4::k4_place<false>, dim3(v4_tiles(b.n_desc)), dim3(V4_THREADS), 0, st, make_dev_batch(b), srec,
                       tstart, v4_ranges(scratch), rules, n_rules, hoff, hb, local_cache, out, req_thr, dfr, routed,
                       poison, ctl);
}
void launch_v4_group(hipStream_t st, const rl_batch& b, const DevRule* rules, uint32_t n_rules, const TableDesc& tab,
                     rl_status* out, uint32_t* req_thr, const HotBucket* hb, const Deferred* dfr, HotCand* cand,
                     int cand_on, uint64_t seed, void* scratch, uint32_t* wg_heads, uint32_t* wg_ins,
                     const uint32_t* scan_heads, const uint32_t* scan_ins, int routed, RegionOcc* occ, EngineCtl* ctl,
                     EngineCtl* next_ctl, EngineCtl* hctl, HotCand* hcand, const MRec* srec,
                     const uint16_t* tstart) {
  using namespace v4;
  uint8_t* p = reinterpret_cast<uint8_t*>(scratch);
  GScratch4 gs;
  gs.rec = reinterpret_cast<MRec*>(p);
  p += (size_t)GBLOCKS * BUCKET_CAP * sizeof(MRec);
  gs.P = reinterpret_cast<uint64_t*>(p);
  p += (size_t)GBLOCKS * BUCKET_CAP * 8;
  gs.slot = reinterpret_cast<uint32_t*>(p);
  p += (size_t)GBLOCKS * GS_HASH * 4;
  gs.cnt = reinterpret_cast<uint32_t*>(p);
  p += (size_t)GBLOCKS * GS_HASH * 4;
  gs.cursor = reinterpret_cast<uint32_t*>(p);
  p += (size_t)GBLOCKS * 4;
  gs.list = reinterpret_cast<uint16_t*>(p);
  p += (size_t)GBLOCKS * BUCKET_CAP * 2;
  gs.grp = reinterpret_cast<uint16_t*>(p);
  p += (size_t)GBLOCKS * BUCKET_CAP * 2;
  gs.end = reinterpret_cast<uint16_t*>(p);
  if (n_rules <= LDS_RULES)
    hipLaunchKernelGGL(k4_group<true>, dim3(GBLOCKS), dim3(G_NT), 0, st, make_dev_batch(b), rules, tab, out, req_thr,
                       hb, dfr, cand, cand_on, seed, gs, wg_heads, wg_ins, scan_heads, scan_ins,
                       (uint32_t)HOT_SCAN_BLOCKS, v4_ranges(scratch), routed, occ, ctl, next_ctl, hctl, hcand, srec,
                       tstart, v4_tiles(b.n_desc), n_rules);
  else
    hipLaunchKernelGGL(k4_group<false>, dim3(GBLOCKS), dim3(G_NT), 0, st, make_dev_batch(b), rules, tab, out, req_thr,
                       hb, dfr, cand, cand_on, seed, gs, wg_heads, wg_ins, scan_heads, scan_ins,
                       (uint32_t)HOT_SCAN_BLOCKS, v4_ranges(scratch), routed, occ, ctl, next_ctl, hctl, hcand, srec,
                       tstart, v4_tiles(b.n_desc), n_rules);
}

}  // namespace rlhip

#ifdef RL_STAMPS
extern "C" int rl_debug_st4(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlhip::g_st4), sizeof(uint64_t) * 4096 * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
