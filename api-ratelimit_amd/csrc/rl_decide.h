// rl_decide.h — per-key table update and per-descriptor decision, shared by the LSD
// pipeline (k_leader / k_decide) and the bucketed pipeline (k_bscan / k_bgroup).
#pragma once
#include "rl_device.h"

namespace rlhip {

constexpr uint32_t MAX_PROBE = 4096;

// Find the slot of (key, fp_lo) for window generation G in its region, or claim an empty one
// (a slot whose generation is older than G is empty for this window: window expiry).
// Returns false when MAX_PROBE slots are all taken.
RL_DEV bool table_claim(const TableDesc& tab, uint64_t key, uint64_t fp_lo, uint32_t G, Slot*& slot_out,
                        bool& existed_out) {
  const uint32_t region = key_region(key);
  const uint32_t lg = tab.region_log2[region];
  const uint64_t mask = (1ull << lg) - 1ull;
  Slot* rbase = tab.slots + tab.region_base[region];
  uint64_t pos = (key << 3) >> (64 - lg);  // top lg bits below the region bits
  const uint32_t tag = (uint32_t)fp_lo;
  const uint32_t lohi = (uint32_t)(fp_lo >> 32);
  Slot* slot = nullptr;
  bool existed = false;
  for (uint32_t probe = 0; probe < MAX_PROBE;) {
    Slot* s = rbase + (pos & mask);
    // ctrl by an L1-bypassing atomic load (it may be CASed concurrently); the identity
    // words in the same load burst (written by earlier batches, or by a concurrent
    // claimer of a different key, which can never match).
    const uint64_t c = ld_relaxed64(&s->ctrl);
    const uint64_t skey = s->key;
    const uint32_t slohi = s->fp_lo_hi;
    const uint32_t g = (uint32_t)c;
    if (g == G && (uint32_t)(c >> 32) == tag && skey == key && slohi == lohi) {
      slot = s;
      existed = true;
      break;
    }
    if (g < G) {
      // empty for this window generation: claim it
      const unsigned long long want = ((unsigned long long)tag << 32) | G;
      const unsigned long long old = atomicCAS((unsigned long long*)&s->ctrl, (unsigned long long)c, want);
      if (old == c) {
        slot = s;
        break;
      }
      continue;  // lost the race: re-examine this slot
    }
    ++pos;
    ++probe;
  }
  slot_out = slot;
  existed_out = existed;
  return slot != nullptr;
}

// First probe slot of a key in its region.
RL_DEV Slot* slot_first(const TableDesc& tab, uint64_t key) {
  const uint32_t region = key_region(key);
  const uint32_t lg = tab.region_log2[region];
  return tab.slots + tab.region_base[region] + (((key << 3) >> (64 - lg)) & ((1ull << lg) - 1ull));
}

// A whole 32-B slot, read ahead of its use with two 16-B loads (table_claim_pre).
struct SlotView {
  uint64_t ctrl, key;
  uint32_t lohi, flags;
  uint64_t count;
};
RL_DEV SlotView load_slot(const Slot* s) {
  const uint4 a = reinterpret_cast<const uint4*>(s)[0];
  const uint4 b = reinterpret_cast<const uint4*>(s)[1];
  SlotView v;
  v.ctrl = (uint64_t)a.x | ((uint64_t)a.y << 32);
  v.key = (uint64_t)a.z | ((uint64_t)a.w << 32);
  v.lohi = b.x;
  v.flags = b.y;
  v.count = (uint64_t)b.z | ((uint64_t)b.w << 32);
  return v;
}

// table_claim with the first probe slot already read (pre). The read-ahead may predate a
// concurrent claim of that slot by another key: a claim is permanent for the window
// generation, so a stale "taken by another key" stays true, a stale "free" makes the CAS
// fail and the slot is re-read. A key's own slot is only claimed by its own leader, and
// count/flags are only written by that leader, so the read-ahead values of the key's slot
// are current. Also returns the counter and flags of an existing slot.
RL_DEV bool table_claim_pre(const TableDesc& tab, uint64_t key, uint64_t fp_lo, uint32_t G, const SlotView pre,
                            Slot*& slot_out, bool& existed_out, uint64_t& count_out, uint32_t& flags_out) {
  const uint32_t region = key_region(key);
  const uint32_t lg = tab.region_log2[region];
  const uint64_t mask = (1ull << lg) - 1ull;
  Slot* rbase = tab.slots + tab.region_base[region];
  uint64_t pos = (key << 3) >> (64 - lg);
  const uint32_t tag = (uint32_t)fp_lo;
  const uint32_t lohi = (uint32_t)(fp_lo >> 32);
  bool use_pre = true;
  slot_out = nullptr;
  existed_out = false;
  count_out = 0;
  flags_out = 0;
  for (uint32_t probe = 0; probe < MAX_PROBE;) {
    Slot* s = rbase + (pos & mask);
    uint64_t c, skey;
    uint32_t slohi;
    if (use_pre) {
      c = pre.ctrl;
      skey = pre.key;
      slohi = pre.lohi;
    } else {
      c = ld_relaxed64(&s->ctrl);
      skey = s->key;
      slohi = s->fp_lo_hi;
    }
    const uint32_t g = (uint32_t)c;
    if (g == G && (uint32_t)(c >> 32) == tag && skey == key && slohi == lohi) {
      slot_out = s;
      existed_out = true;
      count_out = use_pre ? pre.count : s->count;
      flags_out = use_pre ? pre.flags : s->flags;
      return true;
    }
    if (g < G) {  // empty for this window generation: claim it
      const unsigned long long want = ((unsigned long long)tag << 32) | G;
      const unsigned long long old = atomicCAS((unsigned long long*)&s->ctrl, (unsigned long long)c, want);
      if (old == c) {
        slot_out = s;
        return true;
      }
      use_pre = false;
      continue;  // lost the race (or a stale read-ahead): re-examine this slot
    }
    use_pre = false;
    ++pos;
    ++probe;
  }
  return false;
}

// Report a long segment as a hot-set candidate for the next batch (bucketed pipeline).
RL_DEV void emit_candidate(EngineCtl* ctl, HotCand* __restrict__ cand, uint32_t rule, uint32_t count,
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
    cand[c] = hc;
  }
}

// New-key count for the engine stats: one atomic per wave, spread over INS_LINES lines.
RL_DEV void count_inserts(bool inserted, EngineCtl* ctl) {
  const uint64_t ins = __ballot(inserted);
  if (ins && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1))
    atomicAdd(&ctl->tile_ctr[INS_CTR0 + ((blockIdx.x * 4 + (threadIdx.x >> 6)) & (INS_LINES - 1))][0],
              (uint32_t)__popcll(ins));
}

// Table update for the segment [hp, j] of the sorted order (one unique key): INCRBY of the
// whole segment in serial order, local-cache freeze (fixed_cache_impl.go:55-123,
// base_limiter.go:88-106). Writes the key's SegInfo at seg[hp].
RL_DEV void leader_segment(uint32_t hp, uint32_t j, const SortedRec& tail, bool mixed_rule,
                           const uint64_t* __restrict__ skeys, const SortedRec* __restrict__ srec,
                           const ItemRec* __restrict__ recs, const DevRule* __restrict__ rules, const TableDesc& tab,
                           int local_cache, SegInfo* __restrict__ seg, EngineCtl* ctl) {
  const uint64_t key = skeys[j];
  const ItemRec rec = recs[tail.idx];
  const uint32_t region = key_region(key);
  // Two window generations of one region in one batch must be adjacent (a batch may
  // straddle one window boundary); otherwise the older would read as empty.
  if (ctl->gen_max[region] - ctl->gen_min[region] > 1u) {
    atomicOr(&ctl->err, ERR_WINDOW_SPAN);
    return;
  }
  Slot* slot = nullptr;
  bool existed = false;
  if (!table_claim(tab, key, rec.fp_lo, rec.gen, slot, existed)) {
    atomicOr(&ctl->err, ERR_TABLE_FULL);
    return;
  }
  uint64_t base = 0;
  bool frozen_pre = false;
  if (existed) {
    base = slot->count;
    frozen_pre = (slot->flags & SLOT_FROZEN) != 0;
  } else {
    slot->key = key;
    slot->fp_lo_hi = (uint32_t)(rec.fp_lo >> 32);
  }
  count_inserts(!existed, ctl);

  uint32_t freeze = SEG_NO_FREEZE;
  uint64_t final_count = base + tail.P;
  if (frozen_pre) {
    // every descriptor is a local-cache hit: no INCRBY (fixed_cache_impl.go:61-65)
    freeze = SEG_FROZEN_BEFORE;
    final_count = base;
  } else if (local_cache) {
    // first descriptor whose INCRBY reply exceeds its limit (base_limiter.go:88,94-106);
    // all later requests of this key are local-cache hits.
    uint32_t jstar = 0xFFFFFFFFu;
    const uint32_t L0 = rules[tail.rule].L;
    if (!mixed_rule && base + tail.P < (1ull << 32)) {
      // after = base + P is strictly increasing in the segment: binary search.
      if ((uint64_t)(uint32_t)(base + tail.P) > L0) {
        uint32_t lo_i = hp, hi_i = j;
        while (lo_i < hi_i) {
          const uint32_t mid = lo_i + (hi_i - lo_i) / 2;
          if (base + srec[mid].P > (uint64_t)L0) hi_i = mid; else lo_i = mid + 1;
        }
        jstar = lo_i;
      }
    } else {
      for (uint32_t k = hp; k <= j; ++k) {
        const SortedRec r = srec[k];
        if ((uint32_t)(base + r.P) > rules[r.rule].L) { jstar = k; break; }
      }
    }
    if (jstar != 0xFFFFFFFFu) {
      const uint32_t rstar = srec[jstar].req;
      uint32_t last = jstar;
      while (last < j && srec[last + 1].req == rstar) ++last;
      freeze = rstar;
      final_count = base + srec[last].P;
    }
  }
  slot->count = final_count;
  if (freeze != SEG_NO_FREEZE && freeze != SEG_FROZEN_BEFORE) slot->flags = slot->flags | SLOT_FROZEN;
  if (!existed && freeze == SEG_NO_FREEZE) slot->flags = 0;
  if (!existed && freeze != SEG_NO_FREEZE && freeze != SEG_FROZEN_BEFORE) slot->flags = SLOT_FROZEN;
  SegInfo si;
  si.base = base;
  si.freeze = freeze;
  si.pad = 0;
  seg[hp] = si;
}

// GetResponseDescriptorStatus + checkOverLimitThreshold + checkNearLimitThreshold +
// CalculateReset (base_limiter.go:70-195, utilities.go:34-38) for one descriptor.
// thr_idx: the ThrottleMillis slot (the request index; a routed record's own position).
RL_DEV void decide_one(const SortedRec& r, const SegInfo& si, const DevRule& R, rl_status* __restrict__ out,
                       uint32_t* __restrict__ req_thr, uint32_t thr_idx) {
  const uint32_t h = r.h;
  const uint32_t reset = R.div - (uint32_t)r.now_mod;  // div - now % div
  rl_status st;
  st.reset_s = reset;
  st.over_limit_delta = 0;
  st.near_limit_delta = 0;
  const bool local_hit = si.freeze == SEG_FROZEN_BEFORE || (si.freeze != SEG_NO_FREEZE && r.req > si.freeze);
  uint32_t throttle = 0;
  if (local_hit) {
    st.code_flags = RL_CODE_OVER_LIMIT | ((RL_FLAG_HAS_LIMIT | RL_FLAG_LOCAL_CACHE_HIT) << 8);
    st.limit_remaining = 0;
    st.over_limit_delta = h;
  } else {
    const uint32_t after = (uint32_t)(si.base + r.P);
    const uint32_t before = after - h;
    const uint32_t L = R.L, near = R.near;
    if (after > L) {
      st.code_flags = RL_CODE_OVER_LIMIT | (RL_FLAG_HAS_LIMIT << 8);
      st.limit_remaining = 0;
      if (before >= L) {
        st.over_limit_delta = h;
      } else {
        st.over_limit_delta = after - L;
        st.near_limit_delta = L - (near > before ? near : before);
      }
    } else {
      st.code_flags = RL_CODE_OK | (RL_FLAG_HAS_LIMIT << 8);
      st.limit_remaining = L - after;
      if (after > near) {
        const uint32_t millis = reset * 1000u;  // uint32(end - now) * 1000
        const uint32_t calls = (L - after) > 1u ? (L - after) : 1u;
        throttle = millis / calls;
        st.near_limit_delta = before >= near ? h : after - near;
      }
    }
  }
  out[r.idx] = st;
  if (throttle) atomicMax(&req_thr[thr_idx], throttle);
}

RL_DEV void decide_pos(uint32_t j, const SortedRec* __restrict__ srec, const SegInfo* __restrict__ seg,
                       const DevRule* __restrict__ rules, rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                       int routed) {
  const SortedRec r = srec[j];
  decide_one(r, seg[r.head & ~HEAD_MIXED_RULE], rules[r.rule], out, req_thr, routed ? r.idx : r.req);
}

}  // namespace rlhip
