// rl_device.h — device helpers shared by the LSD and v4 pipelines.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_common.h"

namespace rlhip {

#define RL_DEV __device__ __forceinline__

RL_DEV uint32_t ld_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
RL_DEV uint64_t ld_relaxed64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
RL_DEV void st_relaxed(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
RL_DEV void st_relaxed64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

RL_DEV uint64_t lanemask_lt() {
  const uint32_t lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

constexpr uint32_t SPIN_LIMIT = 1u << 24;

// ---------------------------------------------------------------------------
// k_fingerprint
// ---------------------------------------------------------------------------
struct DevBatch {
  uint32_t n_desc, n_req, blob_bytes;
  uint32_t raw;  // 1: decisions leave as raw replies (RawReply per descriptor), no ThrottleMillis
  const uint8_t* blob;
  const uint32_t* off;
  const uint32_t* rule;
  const uint32_t* req_of;
  const int64_t* now;
  const uint32_t* hits;
  const RRec* recs;  // routed batch (multi-GPU owner side): records instead of prefix bytes
  const uint16_t* jit;  // rl_batch.ttl_jitter (NULL: none); a routed record carries its own (rrec_jit)
};
inline DevBatch make_dev_batch(const rl_batch& b) {
  DevBatch d;
  d.n_desc = b.n_desc;
  d.n_req = b.n_req;
  d.blob_bytes = b.blob_bytes;
  d.raw = (b.reserved & RL_BATCH_RAW) ? 1u : 0u;
  d.blob = b.prefix_blob;
  d.off = b.prefix_off;
  d.rule = b.rule_id;
  d.req_of = b.req_of;
  d.now = b.now;
  d.hits = b.hits_addend;
  d.recs = (b.reserved & RL_BATCH_ROUTED) ? reinterpret_cast<const RRec*>(b.prefix_blob) : nullptr;
  d.jit = d.recs ? nullptr : b.ttl_jitter;
  return d;
}
// EXPIRE jitter of an unrouted descriptor (rl_batch.ttl_jitter, fixed_cache_impl.go:69-72).
RL_DEV uint32_t desc_jit(const DevBatch& in, uint32_t i) { return in.jit ? (uint32_t)in.jit[i] : 0u; }

// Unaligned little-endian 8-byte words of a byte string, read as aligned dwords and
// funnel-shifted (v_alignbyte_b32). The blob has >= 16 bytes of slack past its end.
RL_DEV void hash_prefix(const uint8_t* blob, uint32_t off, uint32_t len, FpState& s) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(blob + (off & ~3u));
  const uint32_t sh = (off & 3u) * 8u;
  uint32_t d0 = p[0];
  uint32_t rem = len;
  for (uint32_t k = 0; rem > 0; ++k) {
    const uint32_t d1 = p[2 * k + 1];
    const uint32_t d2 = p[2 * k + 2];
    uint32_t lo = sh ? __builtin_amdgcn_alignbyte(d1, d0, sh / 8) : d0;
    uint32_t hi = sh ? __builtin_amdgcn_alignbyte(d2, d1, sh / 8) : d1;
    uint64_t w = ((uint64_t)hi << 32) | lo;
    if (rem < 8) w &= (~0ull) >> (64 - 8 * rem);
    fp_word(s, w);
    d0 = d2;
    rem = rem > 8 ? rem - 8 : 0;
  }
}

// Prefix hashing from a preload of the prefix's first 32 bytes (two 16-B loads from the dword
// at off & ~3, issued with the descriptor's other loads): prefixes up to 24 B hash inline.
constexpr int PREFIX_PRE_DW = 8;
static_assert(PREFIX_PRE_DW % 4 == 0, "the preload is whole 16-B loads");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));

// Words of a prefix beyond the preloaded dwords, 32 bytes (three words) per pair of 16-B
// loads. p = dword holding the next word's first byte; the blob is readable 32 B past its end.
RL_DEV void hash_tail32(const uint32_t* p, uint32_t sh, uint32_t rem, FpState& s) {
  while (rem > 0) {
    const u32x4 x0 = *reinterpret_cast<const u32x4*>(p), x1 = *reinterpret_cast<const u32x4*>(p + 4);
    const uint32_t dw[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (rem > 0) {
        const uint32_t lo = __builtin_amdgcn_alignbyte(dw[2 * k + 1], dw[2 * k], sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(dw[2 * k + 2], dw[2 * k + 1], sh);
        uint64_t w = ((uint64_t)hi << 32) | lo;
        if (rem < 8) w &= (~0ull) >> (64 - 8 * rem);
        fp_word(s, w);
        rem = rem > 8 ? rem - 8 : 0;
      }
    }
    p += 6;
  }
}

// Prefix state of blob[o0, o0 + len) whose first 32 bytes from the dword at o0 & ~3 are
// already loaded (w0, w1); longer prefixes read the rest 32 bytes a step (the blob is
// readable 32 bytes past its end).
RL_DEV FpState prefix_state_pre(const u32x4 w0, const u32x4 w1, const uint8_t* blob, uint32_t o0, uint32_t len,
                                uint64_t seed) {
  const uint32_t dw[PREFIX_PRE_DW + 1] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, 0u};
  const uint32_t sh = o0 & 3u;
  FpState s = fp_init(len, seed);
  uint32_t rem = len;
#pragma unroll
  for (int k = 0; k < (PREFIX_PRE_DW - 1) / 2; ++k) {
    if (rem > 0) {
      const uint32_t lo = __builtin_amdgcn_alignbyte(dw[2 * k + 1], dw[2 * k], sh);
      const uint32_t hi = __builtin_amdgcn_alignbyte(dw[2 * k + 2], dw[2 * k + 1], sh);
      uint64_t w = ((uint64_t)hi << 32) | lo;
      if (rem < 8) w &= (~0ull) >> (64 - 8 * rem);
      fp_word(s, w);
      rem = rem > 8 ? rem - 8 : 0;
    }
  }
  constexpr int DONE_DW = 2 * ((PREFIX_PRE_DW - 1) / 2);  // dword holding the next word's first byte
  if (rem) hash_tail32(reinterpret_cast<const uint32_t*>(blob + (o0 & ~3u)) + DONE_DW, sh, rem, s);
  return s;
}

RL_DEV int64_t div_const(int64_t now, uint32_t unit) {
  switch (unit) {
    case RL_UNIT_SECOND: return now;
    case RL_UNIT_MINUTE: return now / 60;
    case RL_UNIT_HOUR: return now / 3600;
    default: return now / 86400;
  }
}

// Whole-wave reductions and scans with DPP lane moves (VALU, no LDS round trip per step):
// quad swaps, row_shr 4 / 8 (bound_ctrl: out-of-row lanes read 0), then row_bcast 15 / 31 over
// the rows; the result is in lane 63. All 64 lanes must be active.
template <int CTRL, int ROWM = 0xF, bool BOUND0 = true>
RL_DEV uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, 0xF, BOUND0);
}
RL_DEV uint32_t wave_max_u32(uint32_t v) {
  v = max(v, dpp_mov<0xB1>(v));  // quad_perm [1,0,3,2]
  v = max(v, dpp_mov<0x4E>(v));  // quad_perm [2,3,0,1]
  v = max(v, dpp_mov<0x114>(v));  // row_shr:4
  v = max(v, dpp_mov<0x118>(v));  // row_shr:8
  v = max(v, dpp_mov<0x142, 0xA, false>(v));  // row_bcast:15 into rows 1, 3
  v = max(v, dpp_mov<0x143, 0xC, false>(v));  // row_bcast:31 into rows 2, 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
RL_DEV uint32_t wave_min_u32(uint32_t v) { return ~wave_max_u32(~v); }
RL_DEV uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x114>(v);
  v += dpp_mov<0x118>(v);
  v += dpp_mov<0x142, 0xA, false>(v);
  v += dpp_mov<0x143, 0xC, false>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
RL_DEV uint32_t wave_or_u32(uint32_t v) {
  v |= dpp_mov<0xB1>(v);
  v |= dpp_mov<0x4E>(v);
  v |= dpp_mov<0x114>(v);
  v |= dpp_mov<0x118>(v);
  v |= dpp_mov<0x142, 0xA, false>(v);
  v |= dpp_mov<0x143, 0xC, false>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// Inclusive scan: row_shr 1, 2, 4, 8 inside each row of 16, then the row carries.
RL_DEV uint32_t wave_incl_scan_u32(uint32_t v) {
  v += dpp_mov<0x111>(v);
  v += dpp_mov<0x112>(v);
  v += dpp_mov<0x114>(v);
  v += dpp_mov<0x118>(v);
  v += dpp_mov<0x142, 0xA, false>(v);
  v += dpp_mov<0x143, 0xC, false>(v);
  return v;
}

RL_DEV void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace rlhip
