// rl_decide.h — per-key table update and per-descriptor decision, shared by the LSD
// pipeline (k_leader / k_decide) and the v4 pipeline (k4_scan / k4_place / k4_group).
#pragma once
#include "rl_device.h"

namespace rlhip {

// First probe slot of a key in its region.
// A region's first slot offset and log2 size by a select chain over constant indices: the
// kernel argument words stay in scalar registers. A dynamic index into the by-value TableDesc
// compiled to vector loads from the argument segment whose waits (vmcnt) also drained every
// table read-ahead issued before them.
RL_DEV void region_geom(const TableDesc& tab, uint32_t region, uint64_t& rb, uint32_t& lg) {
  rb = tab.region_base[0];
  lg = tab.region_log2[0];
#pragma unroll
  for (int r = 1; r < 8; ++r) {
    rb = region == (uint32_t)r ? tab.region_base[r] : rb;
    lg = region == (uint32_t)r ? tab.region_log2[r] : lg;
  }
}
RL_DEV Slot* slot_first(const TableDesc& tab, uint64_t key) {
  uint64_t rb;
  uint32_t lg;
  region_geom(tab, key_region(key), rb, lg);
  return tab.slots + rb + (((key << 3) >> (64 - lg)) & ((1ull << lg) - 1ull));
}

// The per-key state of a slot: both stores' counters, the main counter's expiry and the
// local-cache entry's expiry (rl_common.h Slot).
struct KeyState {
  uint32_t count, exp, pcount, frz;
};

// A whole 32-B slot, read ahead of its use with two 16-B loads (table_claim_pre).
struct SlotView {
  uint64_t ctrl, key;
  KeyState st;
};
RL_DEV SlotView load_slot(const Slot* s) {
  const uint4 a = reinterpret_cast<const uint4*>(s)[0];
  const uint4 b = reinterpret_cast<const uint4*>(s)[1];
  SlotView v;
  v.ctrl = (uint64_t)a.x | ((uint64_t)a.y << 32);
  v.key = (uint64_t)a.z | ((uint64_t)a.w << 32);
  v.st = KeyState{b.x, b.y, b.z, b.w};
  return v;
}
RL_DEV KeyState read_state(const Slot* s) {
  const uint4 b = reinterpret_cast<const uint4*>(s)[1];
  return KeyState{b.x, b.y, b.z, b.w};
}
RL_DEV void write_state(Slot* s, const KeyState& k) {
  uint4 v;
  v.x = k.count;
  v.y = k.exp;
  v.z = k.pcount;
  v.w = k.frz;
  reinterpret_cast<uint4*>(s)[1] = v;
}
// A freshly claimed slot: the string is absent from both stores and from the local cache.
RL_DEV void slot_reset(Slot* s, uint64_t key) {
  s->key = key;
  write_state(s, KeyState{0, 0, 0, 0});
}

// Find the slot of (key, fp_lo) for window generation G in its region, or claim an empty one
// (a slot of an older generation is empty for this window: window expiry, slot_free_for). The
// capacity check (RegionOcc, before any table write) keeps every region below its load
// limit, so a free slot always exists within the region: the probe is bounded by its size.
// A claimed slot is reset by the caller (slot_reset) before anything reads it: a key's slot
// is only ever looked up by the key's one leader of the batch.
// table_claim_pre: with the first probe slot already read (pre). The read-ahead may predate a
// concurrent claim of that slot by another key: a claim is permanent for the window
// generation, so a stale "taken by another key" stays true, a stale "free" makes the CAS
// fail and the slot is re-read. A key's own slot is only claimed by its own leader, and
// its state is only written by that leader, so the read-ahead state of the key's slot is
// current. Returns the state of an existing slot (zeros for a claimed one).
RL_DEV bool table_claim_pre(const TableDesc& tab, uint64_t key, uint64_t fp_lo, uint32_t G, const SlotView pre,
                            Slot*& slot_out, bool& existed_out, KeyState& st_out) {
  uint64_t rb;
  uint32_t lg;
  region_geom(tab, key_region(key), rb, lg);
  const uint64_t mask = (1ull << lg) - 1ull;
  Slot* rbase = tab.slots + rb;
  uint64_t pos = (key << 3) >> (64 - lg);
  const uint32_t tag = (uint32_t)fp_lo;
  slot_out = nullptr;
  existed_out = false;
  st_out = KeyState{0, 0, 0, 0};
  SlotView cur = pre;
  for (uint64_t probe = 0; probe <= mask;) {
    Slot* s = rbase + (pos & mask);
    const uint32_t g = (uint32_t)cur.ctrl;
    if (g == G && (uint32_t)(cur.ctrl >> 32) == tag && cur.key == key) {
      slot_out = s;
      existed_out = true;
      st_out = cur.st;
      return true;
    }
    if (slot_free_for(g, G, lazy_region(tab.lag, key_region(key)))) {  // empty for this window generation: claim it
      const unsigned long long want = ((unsigned long long)tag << 32) | G;
      const unsigned long long old = atomicCAS((unsigned long long*)&s->ctrl, (unsigned long long)cur.ctrl, want);
      if (old == cur.ctrl) {
        slot_out = s;
        return true;
      }
      // lost the race, or the read was stale: the CAS returned the slot's claim word, which
      // now belongs to another key of this generation (a key is claimed only by its own
      // leader) or is still older; re-examine the slot with it
      cur.ctrl = old;
      continue;
    }
    ++pos;
    ++probe;
    cur = load_slot(rbase + (pos & mask));  // the whole next slot in one round trip
  }
  return false;
}
// table_claim from the key's first slot, read here; returns the state of an existing slot.
RL_DEV bool table_claim(const TableDesc& tab, uint64_t key, uint64_t fp_lo, uint32_t G, Slot*& slot_out,
                        bool& existed_out, KeyState& st_out) {
  return table_claim_pre(tab, key, fp_lo, G, load_slot(slot_first(tab, key)), slot_out, existed_out, st_out);
}

// Fast-path state of a key all of whose descriptors in the batch have one unit (one store),
// touched inside its window [ws, ws + div): the counter before the batch and whether the
// local cache holds the key for the whole batch. False when an expiry can fall among the
// batch's touches (a string shared by units of different sizes): the key then
// takes the exact sequential path (exotic_sequence).
//   EXPIRE key div + jitter (fixed_cache_impl.go:69-72): alive while now < exp;
//   freecache Set(key, TTL = div) (base_limiter.go:102): hit while now < frz.
RL_DEV bool fast_state(const KeyState& s, bool ps, bool local_cache, uint32_t ws, uint32_t div, uint64_t& base,
                       bool& frozen_pre) {
  if (ps) base = s.pcount;
  else if (s.exp <= ws) base = 0;
  else if (s.exp >= ws + div) base = s.count;
  else return false;
  if (!local_cache || s.frz <= ws) frozen_pre = false;
  else if (s.frz >= ws + div) frozen_pre = true;
  else return false;
  return true;
}

// One descriptor of a key's batch sequence, for the sequential path.
struct SeqItem {
  uint32_t req, t, h, rule, jit;  // jit: EXPIRE jitter (seconds) of the descriptor's INCRBY
};

// Exact serial DoLimit of one key's descriptors (positions 0..n-1 in arrival order), for keys
// the fast path cannot take. Per request: every descriptor of the key sees the local-cache
// lookup made before the request's INCRBYs (fixed_cache_impl.go:55-86); each INCRBY goes to
// its store (main or per-second, :74-85), a main counter past its EXPIRE restarts at 0; then
// every descriptor whose reply exceeds its limit Sets the local cache with TTL = its unit's
// divider (base_limiter.go:94-106), the last Set winning. put(q, reply | P_LOCAL_HIT).
template <class Get, class Put>
RL_DEV void exotic_sequence(KeyState& s, const TableDesc& tab, const DevRule* __restrict__ rules, uint32_t n, Get get,
                            Put put) {
  uint32_t e = 0;
  while (e < n) {
    const SeqItem d0 = get(e);
    const bool hit = tab.local_cache && d0.t < s.frz;
    uint32_t f = e;
    bool set = false;
    uint32_t nf = 0;
    for (; f < n; ++f) {
      const SeqItem d = f == e ? d0 : get(f);
      if (d.req != d0.req) break;
      if (hit) {
        put(f, P_LOCAL_HIT);
        continue;
      }
      const DevRule R = rules[d.rule];
      uint32_t after;
      if (per_second_store(tab, R.unit)) {
        s.pcount += d.h;
        after = s.pcount;
      } else {
        if (d.t >= s.exp) s.count = 0;  // expired (or absent): INCRBY starts from 0
        s.count += d.h;
        s.exp = d.t + R.div + d.jit;  // EXPIRE key div + JitterRand.Int63n(max)
        after = s.count;
      }
      put(f, (uint64_t)after);
      if (tab.local_cache && after > R.L) {
        set = true;
        nf = d.t + R.div;
      }
    }
    if (set) s.frz = nf;
    e = f;
  }
}

// Capacity check, before any table write: every region the batch touches must
// stay within its load limit even if each of its descriptors in that region claimed a new
// slot. Counts are per window generation: a newer generation finds the region empty (its
// older slots are free for it). gmax / cnt: the batch's generation and descriptor count per
// region (0 = untouched).
RL_DEV bool capacity_ok(const RegionOcc (&o)[8], const uint32_t* gmax, const uint32_t* cnt, uint32_t lag) {
  bool ok = true;
#pragma unroll
  for (int r = 0; r < 8; ++r)
    ok &= !cnt[r] || (uint64_t)region_live(o[r], lazy_region(lag, (uint32_t)r), gmax[r]) + cnt[r] <= (uint64_t)o[r].limit;
  return ok;
}
RL_DEV bool capacity_ok(const RegionOcc* __restrict__ occ, const uint32_t* gmax, const uint32_t* cnt, uint32_t lag) {
  RegionOcc o[8];  // all eight loads in flight together (no load behind a branch)
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = occ[r];
  return capacity_ok(o, gmax, cnt, lag);
}
// After the batch: add its new slots (one thread).
RL_DEV void occ_update(RegionOcc* __restrict__ occ, const uint32_t* gmax, const uint32_t* ins, uint32_t lag) {
  for (int r = 0; r < 8; ++r) {
    if (!gmax[r]) continue;  // region untouched
    RegionOcc o = occ[r];
    occ_advance(o, lazy_region(lag, (uint32_t)r), gmax[r], ins[r]);
    occ[r] = o;
  }
}

// Report a long segment as a hot-set candidate for the next batch.
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

// New-slot count per region (LSD leader): one atomic per wave and region on the region's line.
RL_DEV void count_inserts(bool inserted, uint32_t region, EngineCtl* ctl) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t r = 0; r < 8; ++r) {
    const uint64_t m = __ballot(inserted && region == r);
    if (m && lane == (uint32_t)(__ffsll((unsigned long long)m) - 1))
      atomicAdd(&ctl->tile_ctr[INS_CTR0 + r][0], (uint32_t)__popcll(m));
  }
}

// Table update for the segment [hp, j] of the sorted order (one unique key): INCRBY of the
// whole segment in serial order, EXPIRE, local-cache freeze (fixed_cache_impl.go:55-123,
// base_limiter.go:88-106). Writes the key's SegInfo at seg[hp]; an exotic key (fast_state
// false, or units mixed in the segment) gets per-descriptor replies in srec[k].P.
RL_DEV void leader_segment(uint32_t hp, uint32_t j, const SortedRec& tail, bool mixed_rule,
                           const uint64_t* __restrict__ skeys, SortedRec* __restrict__ srec,
                           const ItemRec* __restrict__ recs, const DevRule* __restrict__ rules, const TableDesc& tab,
                           SegInfo* __restrict__ seg, EngineCtl* ctl) {
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
  KeyState ks{0, 0, 0, 0};
  if (!table_claim(tab, key, rec.fp_lo, rec.gen, slot, existed, ks)) {
    atomicOr(&ctl->err, ERR_TABLE_FULL);  // unreachable below the load limit
    return;
  }
  if (!existed) slot_reset(slot, key);
  count_inserts(!existed, region, ctl);
  const uint32_t ws = region_ws(region, rec.gen);
  const DevRule R0 = rules[tail.rule];
  bool exotic = false;
  if (mixed_rule)
    for (uint32_t k = hp; k <= j; ++k) exotic |= rules[srec[k].rule].unit != R0.unit;
  const bool ps = per_second_store(tab, R0.unit);
  uint64_t base = 0;
  bool frozen_pre = false;
  if (!exotic) exotic = !fast_state(ks, ps, tab.local_cache != 0, ws, R0.div, base, frozen_pre);
  SegInfo si;
  si.pad = 0;
  if (exotic) {
    exotic_sequence(
        ks, tab, rules, j - hp + 1,
        [&](uint32_t q) {
          const SortedRec r = srec[hp + q];
          return SeqItem{r.req, ws + (uint32_t)r.now_mod, r.h, r.rule, recs[r.idx].jit};
        },
        [&](uint32_t q, uint64_t v) { srec[hp + q].P = v; });
    write_state(slot, ks);
    si.base = 0;
    si.freeze = SEG_EXOTIC;
    seg[hp] = si;
    return;
  }
  uint32_t freeze = SEG_NO_FREEZE;
  uint32_t last = j;  // the last descriptor whose INCRBY happens
  uint64_t final_count = base + tail.P;
  if (frozen_pre) {
    // every descriptor is a local-cache hit: no INCRBY (fixed_cache_impl.go:61-65)
    freeze = SEG_FROZEN_BEFORE;
  } else if (tab.local_cache) {
    // first descriptor whose INCRBY reply exceeds its limit (base_limiter.go:88,94-106);
    // all later requests of this key are local-cache hits.
    uint32_t jstar = 0xFFFFFFFFu;
    if (!mixed_rule && base + tail.P < (1ull << 32)) {
      // after = base + P is strictly increasing in the segment: binary search.
      if ((uint64_t)(uint32_t)(base + tail.P) > R0.L) {
        uint32_t lo_i = hp, hi_i = j;
        while (lo_i < hi_i) {
          const uint32_t mid = lo_i + (hi_i - lo_i) / 2;
          if (base + srec[mid].P > (uint64_t)R0.L) hi_i = mid; else lo_i = mid + 1;
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
      last = jstar;
      while (last < j && srec[last + 1].req == rstar) ++last;
      freeze = rstar;
      final_count = base + srec[last].P;
    }
  }
  if (freeze != SEG_FROZEN_BEFORE) {
    const uint32_t t_last = ws + (uint32_t)srec[last].now_mod;
    if (ps) {
      ks.pcount = (uint32_t)final_count;
    } else {
      ks.count = (uint32_t)final_count;
      ks.exp = t_last + R0.div + recs[srec[last].idx].jit;  // EXPIRE of the last INCRBY, with its jitter
    }
    if (freeze != SEG_NO_FREEZE) ks.frz = t_last + R0.div;
    write_state(slot, ks);
  }
  si.base = base;
  si.freeze = freeze;
  seg[hp] = si;
}

// GetResponseDescriptorStatus + checkOverLimitThreshold + checkNearLimitThreshold +
// CalculateReset (base_limiter.go:70-195, utilities.go:34-38) for one descriptor.
// thr_idx: the ThrottleMillis slot (the request index; a routed record's own position).
// A raw reply (OUT_RAW): the post-value or the local-cache hit, for the origin to decide.
RL_DEV void emit_raw(rl_status* __restrict__ out, uint32_t idx, uint32_t after, uint32_t flags) {
  RawReply r;
  r.after = after;
  r.flags = flags;
  reinterpret_cast<RawReply*>(out)[idx] = r;
}

// decide_status (rl_common.h): the decision from the INCRBY reply, on the device and the host.

// One descriptor of a segment: its post-value from the segment's state, then the decision
// (or the raw reply). thr_idx: the ThrottleMillis slot (the request; a routed record's own
// position).
RL_DEV void decide_one(const SortedRec& r, const SegInfo& si, const DevRule& R, rl_status* __restrict__ out,
                       uint32_t* __restrict__ req_thr, uint32_t thr_idx, int mode) {
  bool local_hit;
  uint32_t after;
  if (si.freeze == SEG_EXOTIC) {
    local_hit = (r.P & P_LOCAL_HIT) != 0;
    after = (uint32_t)r.P;
  } else {
    local_hit = si.freeze == SEG_FROZEN_BEFORE || (si.freeze != SEG_NO_FREEZE && r.req > si.freeze);
    after = (uint32_t)(si.base + r.P);
  }
  if (mode == OUT_RAW) {
    emit_raw(out, r.idx, local_hit ? 0u : after, local_hit ? RAW_LOCAL_HIT : 0u);
    return;
  }
  rl_status st;
  const uint32_t throttle = decide_status(after, local_hit, r.h, (uint32_t)r.now_mod, R, st);
  out[r.idx] = st;
  if (throttle) atomicMax(&req_thr[thr_idx], throttle);
}

RL_DEV void decide_pos(uint32_t j, const SortedRec* __restrict__ srec, const SegInfo* __restrict__ seg,
                       const DevRule* __restrict__ rules, rl_status* __restrict__ out, uint32_t* __restrict__ req_thr,
                       int mode) {
  const SortedRec r = srec[j];
  decide_one(r, seg[r.head & ~HEAD_MIXED_RULE], rules[r.rule], out, req_thr, mode != OUT_STATUS ? r.idx : r.req, mode);
}

}  // namespace rlhip
