// rl_resolve.hip — descriptor-tree resolution (GetLimit) as a batched device pass.
//
// The step before the decision path: for each descriptor of a batch, walk the domain's
// descriptor tree exactly like rateLimitConfigImpl.GetLimit (src/config/config_impl.go:274-323)
// and return the rule id of the limit it resolves to (RL_NIL_RULE = nil limit), which is
// what rl_submit consumes per descriptor.
//
//   * unknown domain -> nil (:279-284); a descriptor limit override -> the override's rule,
//     before any tree walk (:286-296);
//   * per entry i: node = map[key "_" value], else map[key] (:300-309); the node's limit
//     counts only at the last entry (:311-318); descend while the node has children, else
//     stop (:320-325).
//
// Device layout: the tree's nodes (64 B each: parent, name length, rule, child count, name
// hash and the name's first 32 bytes) and an open-addressing table over (parent, name) edges
// (hash << 32 | node id, load <= 1/8), both small enough to stay in L2. Names are compared
// byte-exactly after the hash matches, so ("a_b") and ("a", "b") resolve exactly as the
// reference's string maps do. One thread per descriptor. A level of the walk loads the key and
// the value as whole dwords into registers (one round trip), folds them, reads both edges'
// first probe rounds (key_value and key) together, then both first candidates' nodes, whose
// inline names compare against the register strings: three round trips per level where the
// first version (byte loads in data-dependent loops) needed one per byte. Names longer than
// 32 bytes take that byte path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "rl_common.h"
#include "rl_resolve.h"

namespace rlhip {

namespace {

#define RL_HD __host__ __device__
constexpr int RS_NT = 256;        // descriptors per block, one per thread
constexpr int SW = 8;             // dwords of a string held in registers
constexpr uint32_t SB = 4 * SW;   // bytes: names up to 32 bytes take the register path

// ---- the byte path (long names, strings at the blob's edges, an unaligned blob) ----
// A byte from the aligned dword that holds it (never past that byte's page; no sub-dword
// loads that the compiler could merge into misaligned wider ones). The byte path is written
// out explicitly (no lookup template taking a compare lambda, no struct copies): its first
// forms were bit-exact on the host and at -O1 but returned wrong lookups at -O3 on the device;
// this form is checked there by tests/test_gpu_resolve.py and tools/diag_resolve.py (blobs
// shifted by 1-3 bytes send every lookup down this path). Out of line it is also right, but
// the kernel then needs a stack and took 118 us instead of 94 on config 4.
RL_HD inline uint32_t ld_u8(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return (*reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3) >> (8u * (uint32_t)(a & 3u))) & 0xFFu;
}
// Fold of the query name A["_" B] of length len (byte loads; the register path folds words).
RL_HD uint32_t fold_query_bytes(const uint8_t* bytes, uint32_t a, uint32_t al, uint32_t b, uint32_t len) {
  uint32_t h = TREE_FOLD0;
  for (uint32_t k = 0; k < len; k += 4) {
    uint32_t w = 0;
    for (uint32_t j = 0; j < 4 && k + j < len; ++j) {
      const uint32_t q = k + j;
      const uint32_t c = q < al ? ld_u8(bytes + a + q) : q == al ? (uint32_t)'_' : ld_u8(bytes + b + (q - al - 1u));
      w |= c << (8u * j);
    }
    h = tree_fold_word(h, w);
  }
  return h;
}
// The queried name: A (wb false), or A "_" B (finalKey, config_impl.go:126-129 and :300), of
// total length len, against the node's name in the names blob.
RL_HD bool name_eq_bytes(const uint8_t* names, uint32_t noff, uint32_t len, const uint8_t* bytes, uint32_t a,
                         uint32_t al, uint32_t b) {
  uint32_t diff = 0;
  for (uint32_t k = 0; k < len; ++k) {
    const uint32_t c = k < al ? ld_u8(bytes + a + k) : k == al ? (uint32_t)'_' : ld_u8(bytes + b + (k - al - 1u));
    diff |= ld_u8(names + noff + k) ^ c;
  }
  return diff == 0;
}

// The byte path's probe: (parent, name A["_" B]) with hash h, names compared in the blob.
RL_HD uint32_t find_bytes(const TreeDesc2& t, uint32_t parent, uint32_t h, const uint8_t* bytes, uint32_t a,
                          uint32_t al, uint32_t b, uint32_t len, uint32_t& rule, uint32_t& nch) {
  uint32_t s = h & t.mask;
  for (uint32_t probes = 0; probes <= t.mask; ++probes, s = (s + 1) & t.mask) {
    const uint64_t w = t.slots[s];
    if ((uint32_t)w == TREE_EMPTY) break;
    if ((uint32_t)(w >> 32) != h) continue;
    const uint32_t id = (uint32_t)w;
    const uint32_t np = t.nodes[id].parent, nl = t.nodes[id].name_len, no = t.nodes[id].name_off;
    if (np != parent || nl != len || !name_eq_bytes(t.names, no, len, bytes, a, al, b)) continue;
    rule = t.nodes[id].rule;
    nch = t.nodes[id].n_children;
    return id;
  }
  return TREE_NONE;
}

// ---- the register path ----
// bytes sh.. of the pair hi:lo (v_alignbyte_b32)
RL_HD inline uint32_t align_byte(uint32_t hi, uint32_t lo, uint32_t sh) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbyte(hi, lo, sh);  // one VALU op (the host form below is the same value)
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
#endif
}
// s[k] = bytes 4k..4k+3 of the string at bytes + off (little-endian), zero past len (<= SB).
// The blob is 4-B aligned and the string's last dword lies inside it (checked by the caller):
// whole-dword loads at clamped indices, all in flight together.
RL_HD void load_str(const uint8_t* bytes, uint32_t off, uint32_t len, uint32_t (&s)[SW]) {
  if (len == 0) {
#pragma unroll
    for (int k = 0; k < SW; ++k) s[k] = 0u;
    return;
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(bytes) + (off >> 2);
  const uint32_t sh = off & 3u, nd = (sh + len + 3u) >> 2;  // dwords that hold the string (>= 1 if len)
  const uint32_t last = nd ? nd - 1u : 0u;
  uint32_t d[SW + 1];
#pragma unroll
  for (int k = 0; k <= SW; ++k) d[k] = w[min((uint32_t)k, last)];
#pragma unroll
  for (int k = 0; k < SW; ++k) {
    const uint32_t v = align_byte(d[k + 1], d[k], sh);
    const uint32_t b0 = 4u * (uint32_t)k;
    s[k] = b0 >= len ? 0u : b0 + 4u <= len ? v : v & ((1u << (8u * (len - b0))) - 1u);
  }
}
RL_HD uint32_t fold_reg(const uint32_t (&s)[SW], uint32_t len) {
  uint32_t h = TREE_FOLD0;
  const uint32_t nw = (len + 3u) >> 2;
#pragma unroll
  for (int k = 0; k < SW; ++k)
    if ((uint32_t)k < nw) h = tree_fold_word(h, s[k]);
  return h;
}
// r = x moved n bytes up (byte j of r = byte j - n of x; zero below n), n < SB.
RL_HD void shl_bytes(const uint32_t (&x)[SW], uint32_t n, uint32_t (&r)[SW]) {
  uint32_t a[SW];
#pragma unroll
  for (int k = 0; k < SW; ++k) a[k] = x[k];
#pragma unroll
  for (int st = 4; st >= 1; st >>= 1) {  // whole dwords: a log shifter on n >> 2
    const bool on = ((n >> 2) & (uint32_t)st) != 0;
#pragma unroll
    for (int k = SW - 1; k >= 0; --k) a[k] = on ? (k >= st ? a[k - st] : 0u) : a[k];
  }
  const uint32_t b = n & 3u;
#pragma unroll
  for (int k = SW - 1; k >= 0; --k) {
    const uint32_t lo = k ? a[k - 1] : 0u;
    r[k] = b ? align_byte(a[k], lo, 4u - b) : a[k];
  }
}
// A node's header and inline name as four 16-B loads (fields read from the words: no copy of
// the 64-B aligned struct, whose byte-path form the compiler got wrong).
struct NodeView {
  uint32_t parent, len, rule, nch, name[SW];
};
RL_HD NodeView load_node(const TreeDesc2& t, uint32_t id) {
  const uint4* p = reinterpret_cast<const uint4*>(t.nodes + id);
  const uint4 h = p[0], n0 = p[2], n1 = p[3];
  NodeView v;
  v.parent = h.x;
  v.len = h.y;
  v.rule = h.z;
  v.nch = h.w;
  v.name[0] = n0.x; v.name[1] = n0.y; v.name[2] = n0.z; v.name[3] = n0.w;
  v.name[4] = n1.x; v.name[5] = n1.y; v.name[6] = n1.z; v.name[7] = n1.w;
  return v;
}
RL_HD bool same(const NodeView& nd, uint32_t parent, uint32_t len, const uint32_t (&q)[SW]) {
  uint32_t diff = (nd.parent ^ parent) | (nd.len ^ len);
#pragma unroll
  for (int k = 0; k < SW; ++k) diff |= nd.name[k] ^ q[k];
  return diff == 0;
}
// The register path's full probe (a hash collision in the first round, or a longer chain).
RL_HD uint32_t find_reg(const TreeDesc2& t, uint32_t parent, uint32_t h, uint32_t len, const uint32_t (&q)[SW],
                        uint32_t& rule, uint32_t& nch) {
  uint32_t s = h & t.mask;
  for (uint32_t probes = 0; probes <= t.mask; ++probes, s = (s + 1) & t.mask) {
    const uint64_t w = t.slots[s];
    if ((uint32_t)w == TREE_EMPTY) break;
    if ((uint32_t)(w >> 32) != h) continue;
    const NodeView v = load_node(t, (uint32_t)w);
    if (!same(v, parent, len, q)) continue;
    rule = v.rule;
    nch = v.nch;
    return (uint32_t)w;
  }
  return TREE_NONE;
}
// First slot of the probe round (4 words from h's home) whose hash is h: its node id, or
// TREE_NONE; done = the round settles it (an empty slot before any match).
RL_HD uint32_t first_match(const uint64_t (&w)[TREE_PROBE], uint32_t h, bool& done) {
  done = false;
#pragma unroll
  for (int j = 0; j < TREE_PROBE; ++j) {
    if ((uint32_t)w[j] == TREE_EMPTY) {
      done = true;
      return TREE_NONE;
    }
    if ((uint32_t)(w[j] >> 32) == h) return (uint32_t)w[j];
  }
  return TREE_NONE;
}
RL_HD void probe_round(const TreeDesc2& t, uint32_t h, uint64_t (&w)[TREE_PROBE]) {
  const uint64_t* p = t.slots + (h & t.mask);  // (one address, the slots at immediate offsets)
#pragma unroll
  for (int j = 0; j < TREE_PROBE; ++j) w[j] = p[j];
}

// rateLimitConfigImpl.GetLimit (config_impl.go:274-323) for one descriptor: unknown domain ->
// nil (:279-284); a descriptor limit override -> its rule before any walk (:286-296); per
// entry the node of key_value, else of key (:300-309); the node's limit counts only at the
// last entry (:311-318); descend while the node has children (:320-325).
RL_HD uint32_t resolve_one(const ResolveIn& in, const TreeDesc2& t, uint32_t i) {
  const uint32_t doff = in.domain[2 * i], dlen = in.domain[2 * i + 1];
  const uint32_t e0 = in.entry_first[i], e1 = in.entry_first[i + 1];
  const uint32_t ov = in.override_rule ? in.override_rule[i] : RL_NIL_RULE;
  const uint64_t blen = in.bytes_len;
  // a string outside bytes, or entries outside the entry array: nil (rl_resolve, the host
  // form, refuses such a batch)
  auto inside = [&](uint32_t o, uint32_t l) { return (uint64_t)o + l <= blen; };
  // the register path: a 4-B aligned blob, the string's last dword inside it, <= SB bytes
  const bool aligned = (reinterpret_cast<uintptr_t>(in.bytes) & 3u) == 0;
  const uint64_t bwords = blen & ~3ull;
  auto reg_ok = [&](uint32_t o, uint32_t l) { return aligned && l <= SB && (((uint64_t)o + l + 3u) & ~3ull) <= bwords; };
  uint32_t rule = RL_NIL_RULE;
  if (!(e0 <= e1 && e1 <= in.n_entries) || !inside(doff, dlen)) return rule;
  uint32_t xr = RL_NIL_RULE, xn = 0;
  uint32_t dom;
  if (reg_ok(doff, dlen)) {
    uint32_t D[SW];
    load_str(in.bytes, doff, dlen, D);
    dom = find_reg(t, RL_TREE_ROOT, tree_hash(RL_TREE_ROOT, fold_reg(D, dlen), dlen), dlen, D, xr, xn);
  } else {
    dom = find_bytes(t, RL_TREE_ROOT, tree_hash(RL_TREE_ROOT, fold_query_bytes(in.bytes, doff, dlen, 0, dlen), dlen),
                     in.bytes, doff, dlen, 0, dlen, xr, xn);
  }
  if (dom == TREE_NONE) return rule;
  if (ov != RL_NIL_RULE) return ov;  // descriptor.GetLimit() != nil (config_impl.go:286-296)
  uint32_t parent = dom;
  for (uint32_t e = e0; e < e1; ++e) {
    const uint4 E = make_uint4(in.entry[4 * e], in.entry[4 * e + 1], in.entry[4 * e + 2], in.entry[4 * e + 3]);
    const uint32_t ko = E.x, kl = E.y, vo = E.z, vl = E.w;
    if (!inside(ko, kl) || !inside(vo, vl)) {
      rule = RL_NIL_RULE;
      break;
    }
    const uint32_t lv = kl + 1u + vl;  // key "_" value
    uint32_t nd = TREE_NONE;
    if (reg_ok(ko, kl) && reg_ok(vo, vl) && lv <= SB) {
      uint32_t K[SW], V[SW], Q[SW];
      load_str(in.bytes, ko, kl, K);
      load_str(in.bytes, vo, vl, V);
      shl_bytes(V, kl + 1u, Q);  // Q = K "_" V
#pragma unroll
      for (int k = 0; k < SW; ++k) {
        const uint32_t us = (uint32_t)k == (kl >> 2) ? (uint32_t)'_' << (8u * (kl & 3u)) : 0u;
        Q[k] |= K[k] | us;
      }
      const uint32_t hv = tree_hash(parent, fold_reg(Q, lv), lv), hk = tree_hash(parent, fold_reg(K, kl), kl);
      // both edges' first probe rounds, then both first candidates' nodes, in two round trips
      uint64_t wv[TREE_PROBE], wk[TREE_PROBE];
      probe_round(t, hv, wv);
      probe_round(t, hk, wk);
      bool dv, dk;
      const uint32_t cv = first_match(wv, hv, dv), ck = first_match(wk, hk, dk);
      NodeView nv{}, nk{};
      if (cv != TREE_NONE) nv = load_node(t, cv);
      if (ck != TREE_NONE) nk = load_node(t, ck);
      if (cv != TREE_NONE && same(nv, parent, lv, Q)) {
        nd = cv;
        xr = nv.rule;
        xn = nv.nch;
      } else if (!dv) {  // a hash collision in the round, or a longer probe chain: the full probe
        nd = find_reg(t, parent, hv, lv, Q, xr, xn);
      }
      if (nd == TREE_NONE) {
        if (ck != TREE_NONE && same(nk, parent, kl, K)) {
          nd = ck;
          xr = nk.rule;
          xn = nk.nch;
        } else if (!dk) {
          nd = find_reg(t, parent, hk, kl, K, xr, xn);
        }
      }
    } else {
      nd = find_bytes(t, parent, tree_hash(parent, fold_query_bytes(in.bytes, ko, kl, vo, lv), lv), in.bytes, ko, kl, vo,
                      lv, xr, xn);
      if (nd == TREE_NONE)
        nd = find_bytes(t, parent, tree_hash(parent, fold_query_bytes(in.bytes, ko, kl, 0, kl), kl), in.bytes, ko, kl, 0,
                        kl, xr, xn);
    }
    if (nd == TREE_NONE) break;
    if (xr != RL_NIL_RULE && e == e1 - 1) rule = xr;
    if (xn == 0) break;
    parent = nd;
  }
  return rule;
}

// ---- the level-pipelined walk (k_resolve's first pass) ----
// resolve_one spends about four dependent round trips per level: the entry's words, its two
// strings, the edge probe rounds, the candidate nodes. None of the first two depend on the
// walk, and a node is needed only to confirm a hash match (its rule matters only at the last
// entry). So this pass loads each level's entry words two levels ahead and its strings one
// level ahead, hashes both names from registers and looks them up among the children hashes
// of the node it is standing on (FastNode: the node's own 64-B load both confirms it and holds
// its children's hashes), taking the match unconfirmed until the next level loads that node:
// one round trip per level, plus one for the last node.
//   * A miss is exact (equal names hash equally; siblings with equal hashes, and nodes with
//     more than FAST_CHILDREN children, keep their children in the fast edge table, read by
//     probe rounds). A match whose node carries another name, and any string the register path
//     cannot hold (over 16 bytes, an unaligned blob, a load window past the blob's end) leave
//     the descriptor to the exact walk (k_resolve_exact).
//   * The usual batch lays each entry out as key "_" value inside the descriptor's own bytes
//     (the cache key's prefix): one load window then holds the whole name. Other layouts load
//     the value's window too and join the two in registers.
//   * No child count check: the reference stops at a node without children (config_impl.go
//     :320-325); this walk goes on and looks the next entry up among no children, misses and
//     stops there with the same (nil) result.
constexpr uint32_t RS_EXACT = 0xFFFFFFFEu;  // first pass: left to the exact walk
// (Measured and not kept, config 4, one box, interleaved: the string windows two levels ahead
// instead of one, entries three ahead, 76 VGPRs: k_resolve 55.6-56.1 us against 53.8-55.1; never
// reading value windows (other layouts to the exact walk) saves about 2 us more.)
#ifndef RL_RESOLVE_FW
#define RL_RESOLVE_FW 4
#endif
// Names the first pass holds in registers: FW dwords (16 bytes; config 4's longest key "_" value
// is 9). Longer ones go to the exact walk: every dword held here costs the pass occupancy.
constexpr int FW = RL_RESOLVE_FW;
constexpr uint32_t FB = 4 * FW;
static_assert(FW == 4, "first-pass names: one 16-B node name load");
constexpr uint32_t FWB = 4 * (FW + 1);  // bytes of a string's load window (from its aligned start)

// Raw buffer loads: a load wholly past the buffer's end returns zeros (the hardware's range
// check; the host form does the same), so the loads a level does not need are sent past the end
// (RS_OOB) rather than put behind a condition: a load behind a condition — even a wave-uniform
// one — made the wave wait for every load before it (141 us for this pass against 96 for the
// old walk). Buffers are capped below RS_OOB, and the walk never uses a load that is partly past
// the end (windows are checked against the capped length).
constexpr uint32_t RS_OOB = 0x80000000u;
constexpr uint32_t RS_BUF_MAX = RS_OOB - 64u;
struct Buf {
#ifdef __HIP_DEVICE_COMPILE__
  __amdgpu_buffer_rsrc_t r;
#else
  const uint8_t* p;
  uint32_t n;
#endif
};
RL_HD inline Buf make_buf(const void* p, uint64_t n) {
  const uint32_t m = (uint32_t)(p ? (n < RS_BUF_MAX ? n : RS_BUF_MAX) : 0);
  Buf b;
#ifdef __HIP_DEVICE_COMPILE__
  b.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)m, 0x00020000);
#else
  b.p = static_cast<const uint8_t*>(p);
  b.n = m;
#endif
  return b;
}
RL_HD inline uint4 bld4(const Buf& b, uint32_t off) {
#ifdef __HIP_DEVICE_COMPILE__
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(b.r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
#else
  uint4 v = make_uint4(0, 0, 0, 0);
  if ((uint64_t)off + 16 <= b.n) memcpy(&v, b.p + off, 16);
  return v;
#endif
}
RL_HD inline uint2 bld2(const Buf& b, uint32_t off) {
#ifdef __HIP_DEVICE_COMPILE__
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(b.r, (int)off, 0, 0);
  return make_uint2(v[0], v[1]);
#else
  uint2 v = make_uint2(0, 0);
  if ((uint64_t)off + 8 <= b.n) memcpy(&v, b.p + off, 8);
  return v;
#endif
}
RL_HD inline uint32_t bld1(const Buf& b, uint32_t off) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_raw_buffer_load_b32(b.r, (int)off, 0, 0);
#else
  uint32_t v = 0;
  if ((uint64_t)off + 4 <= b.n) memcpy(&v, b.p + off, 4);
  return v;
#endif
}
struct FastBufs {
  Buf bytes, dom, efirst, ent, ovr, fnodes, fslots;
};
RL_HD inline FastBufs fast_bufs(const ResolveIn& in, const TreeDesc2& t) {
  FastBufs B;
  B.bytes = make_buf(in.bytes, in.bytes_len);
  B.dom = make_buf(in.domain, (uint64_t)in.n_desc * 8);
  B.efirst = make_buf(in.entry_first, ((uint64_t)in.n_desc + 1) * 4);
  B.ent = make_buf(in.entry, (uint64_t)in.n_entries * 16);
  B.ovr = make_buf(in.override_rule, (uint64_t)in.n_desc * 4);
  B.fnodes = make_buf(t.fnodes, (uint64_t)t.n_fnodes * sizeof(FastNode));
  B.fslots = make_buf(t.fslots, ((uint64_t)t.fmask + TREE_PROBE) * 8);
  return B;
}

// A string's load window: the FW + 1 dwords from its aligned start (RS_OOB: zeros).
RL_HD inline void load_win(const Buf& b, uint32_t off, uint32_t (&d)[FW + 1]) {
  const uint4 a = bld4(b, off);
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  d[4] = bld1(b, off + 16u);
}
// s[k] = bytes 4k..4k+3 of the window from byte sh of its first dword (not masked)
RL_HD inline void win_words(const uint32_t (&d)[FW + 1], uint32_t sh, uint32_t (&s)[FW]) {
#pragma unroll
  for (int k = 0; k < FW; ++k) s[k] = align_byte(d[k + 1], d[k], sh);
}
// m[k] = the bytes of word k that lie below len (len <= FB)
RL_HD inline void len_masks(uint32_t len, uint32_t (&m)[FW]) {
#pragma unroll
  for (int k = 0; k < FW; ++k) {
    const uint32_t b = min(max((int32_t)(8u * len) - 32 * k, 0), 32);  // bits of word k in the name
    m[k] = b >= 32u ? 0xFFFFFFFFu : (1u << b) - 1u;
  }
}
RL_HD inline bool any_lane(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
  return __any(p);
#else
  return p;
#endif
}
// = fold_reg for len <= FB; a word no lane of the wave needs is skipped (config 4's keys are one
// word, its key "_" value names three)
RL_HD uint32_t fold_w(const uint32_t (&s)[FW], uint32_t len) {
  uint32_t h = tree_fold_word(TREE_FOLD0, s[0]);
  h = len ? h : TREE_FOLD0;
  const uint32_t nw = (len + 3u) >> 2;
#pragma unroll
  for (int k = 1; k < FW; ++k)
    if (any_lane((uint32_t)k < nw)) h = (uint32_t)k < nw ? tree_fold_word(h, s[k]) : h;
  return h;
}
// r = K "_" V (finalKey, config_impl.go:300): V moved kl + 1 bytes up (kl + 1 <= FB), then K and
// the underscore
RL_HD void key_value_w(const uint32_t (&K)[FW], const uint32_t (&V)[FW], uint32_t kl, uint32_t (&r)[FW]) {
  const uint32_t n = kl + 1u;
  uint32_t a[FW];
#pragma unroll
  for (int k = 0; k < FW; ++k) a[k] = V[k];
#pragma unroll
  for (int st = 4; st >= 1; st >>= 1) {  // whole dwords: a log shifter on n >> 2
    const bool on = ((n >> 2) & (uint32_t)st) != 0;
#pragma unroll
    for (int k = FW - 1; k >= 0; --k) a[k] = on ? (k >= st ? a[k - st] : 0u) : a[k];
  }
  const uint32_t b = n & 3u;
#pragma unroll
  for (int k = FW - 1; k >= 0; --k) {
    const uint32_t lo = k ? a[k - 1] : 0u;
    const uint32_t us = (uint32_t)k == (kl >> 2) ? (uint32_t)'_' << (8u * (kl & 3u)) : 0u;
    r[k] = (b ? align_byte(a[k], lo, 4u - b) : a[k]) | K[k] | us;
  }
}
// A fast node: header, first 16 name bytes and the children's hashes (four 16-B loads).
struct NodeF {
  uint32_t parent, len_flags, rule, first, name[FW], ch[FAST_CHILDREN];
};
RL_HD inline NodeF load_fnode(const Buf& b, uint32_t id) {
  const uint32_t o = id * (uint32_t)sizeof(FastNode);
  const uint4 h = bld4(b, o), n0 = bld4(b, o + 16u), c0 = bld4(b, o + 32u), c1 = bld4(b, o + 48u);
  NodeF v;
  v.parent = h.x; v.len_flags = h.y; v.rule = h.z; v.first = h.w;
  v.name[0] = n0.x; v.name[1] = n0.y; v.name[2] = n0.z; v.name[3] = n0.w;
  v.ch[0] = c0.x; v.ch[1] = c0.y; v.ch[2] = c0.z; v.ch[3] = c0.w;
  v.ch[4] = c1.x; v.ch[5] = c1.y; v.ch[6] = c1.z; v.ch[7] = c1.w;
  return v;
}
// the node against (parent, len, q): q is zero past len (<= FB), as the node's inline name is
RL_HD inline bool confirm_f(const NodeF& nd, uint32_t parent, uint32_t len, const uint32_t (&q)[FW]) {
  uint32_t diff = (nd.parent ^ parent) | ((nd.len_flags & 0xFFFFFFu) ^ len);
#pragma unroll
  for (int k = 0; k < FW; ++k) diff |= nd.name[k] ^ q[k];
  return diff == 0;
}
// the child whose hash is h (fast id), or TREE_NONE (at most one: build_fast_tree)
RL_HD inline uint32_t child_of(const NodeF& nd, uint32_t h) {
  uint32_t k = TREE_NONE;
#pragma unroll
  for (int j = FAST_CHILDREN - 1; j >= 0; --j) k = nd.ch[j] == h ? (uint32_t)j : k;
  return k == TREE_NONE ? TREE_NONE : nd.first + k;
}
// the fast edge table: a probe round (4 slots from h's home), then the chain slot by slot when
// the round neither matches nor ends (rare at load <= 1/8)
RL_HD inline void probe_round_f(const Buf& b, uint32_t h, uint32_t mask, uint64_t (&w)[TREE_PROBE]) {
  const uint32_t o = (h & mask) * 8u;
  const uint4 a = bld4(b, o), c = bld4(b, o + 16u);
  w[0] = (uint64_t)a.y << 32 | a.x; w[1] = (uint64_t)a.w << 32 | a.z;
  w[2] = (uint64_t)c.y << 32 | c.x; w[3] = (uint64_t)c.w << 32 | c.z;
}
RL_HD uint32_t match_chain_f(const Buf& b, uint32_t mask, uint32_t h, const uint64_t (&w)[TREE_PROBE]) {
  bool done;
  const uint32_t c = first_match(w, h, done);
  if (c != TREE_NONE || done) return c;
  uint32_t s = (h + TREE_PROBE) & mask;
  for (uint32_t probes = TREE_PROBE; probes <= mask; ++probes, s = (s + 1) & mask) {
    const uint2 x = bld2(b, s * 8u);
    if (x.x == TREE_EMPTY) break;
    if (x.y == h) return x.x;
  }
  return TREE_NONE;
}

// rule id of descriptor i (exact), or RS_EXACT: the exact walk (resolve_one) decides it.
RL_HD uint32_t resolve_fast(const ResolveIn& in, const TreeDesc2& t, const FastBufs& B, uint32_t i) {
  const uint2 dm = bld2(B.dom, 8u * i), ef = bld2(B.efirst, 4u * i);
  const uint32_t ov = in.override_rule ? bld1(B.ovr, 4u * i) : RL_NIL_RULE;
  const uint32_t doff = dm.x, dlen = dm.y, e0 = ef.x, e1 = ef.y;
  const uint32_t blen = in.bytes_len;
  // (32-bit bounds: o + l <= blen without the sum overflowing)
  auto inside = [&](uint32_t o, uint32_t l) { return o <= blen && l <= blen - o; };
  if (!(e0 <= e1 && e1 <= in.n_entries) || !inside(doff, dlen)) return RL_NIL_RULE;  // as resolve_one
  const bool aligned = (reinterpret_cast<uintptr_t>(in.bytes) & 3u) == 0;
  const uint32_t wlim = (blen < RS_BUF_MAX ? blen : RS_BUF_MAX);
  const uint32_t wmax = wlim >= FWB ? wlim - FWB : 0u;  // the last aligned start whose window lies inside
  const bool wany = wlim >= FWB;
  auto win_ok = [&](uint32_t o) { return wany && (o & ~3u) <= wmax; };
  if (!aligned || dlen > FB || !win_ok(doff)) return RS_EXACT;
  const uint32_t n = e1 - e0;
  // an entry's windows: key "_" value from the key's window when the value follows the key's
  // separator, else the value's window too
  auto joined_at = [](const uint4& x) { return x.z == x.x + x.y + 1u; };
  auto load_strings = [&](const uint4& x, bool ld, uint32_t (&W)[FW + 1], uint32_t (&Vw)[FW + 1]) {
    load_win(B.bytes, ld ? x.x & ~3u : RS_OOB, W);
    load_win(B.bytes, ld && !joined_at(x) ? x.z & ~3u : RS_OOB, Vw);
  };
  // round trip 1: the domain's window and the first two entries' words
  uint32_t Q[FW];  // the name to confirm, zero past its length: the domain, then a level's name
  {
    uint32_t D[FW + 1], M[FW];
    load_win(B.bytes, doff & ~3u, D);
    len_masks(dlen, M);
    win_words(D, doff & 3u, Q);
#pragma unroll
    for (int k = 0; k < FW; ++k) Q[k] &= M[k];
  }
  uint4 E = bld4(B.ent, n > 0 ? 16u * e0 : RS_OOB);
  uint4 En = bld4(B.ent, n > 1 ? 16u * (e0 + 1u) : RS_OOB);
  const uint32_t hd = fast_hash(RL_TREE_ROOT, fold_w(Q, dlen), dlen);
  // round trip 2: the domain's probe round and level 0's windows
  uint64_t w[TREE_PROBE];
  probe_round_f(B.fslots, hd, t.fmask, w);
  uint32_t W[FW + 1], Vw[FW + 1];
  load_strings(E, n > 0, W, Vw);
  uint32_t pend = match_chain_f(B.fslots, t.fmask, hd, w);  // the node to confirm (parent pp, name Q, length pl)
  if (pend == TREE_NONE) return RL_NIL_RULE;  // unknown domain (:279-284)
  uint32_t pp = RL_TREE_ROOT, pl = dlen;
  if (ov != RL_NIL_RULE || n == 0) {  // override (:286-296), or no entries: the domain alone decides
    if (!confirm_f(load_fnode(B.fnodes, pend), pp, pl, Q)) return RS_EXACT;
    return ov;
  }
  for (uint32_t l = 0; l < n; ++l) {
    // level l: W / Vw hold entry l's windows, E its words, En entry l+1's
    const uint32_t ko = E.x, kl = E.y, vo = E.z, vl = E.w;
    if (!inside(ko, kl) || !inside(vo, vl)) return RL_NIL_RULE;  // as resolve_one: the walk ends nil
    const uint32_t lv = kl + 1u + vl;
    const bool jn = joined_at(E);
    if (kl > FB || vl > FB || lv > FB || !win_ok(ko) || (!jn && !win_ok(vo))) return RS_EXACT;
    // Qn = key "_" value and K = key, zero past their lengths (joined: both from the key's window)
    uint32_t S[FW], Mk[FW], Qn[FW], K[FW];
    win_words(W, ko & 3u, S);
    len_masks(kl, Mk);
#pragma unroll
    for (int k = 0; k < FW; ++k) K[k] = S[k] & Mk[k];
    if (jn) {
      uint32_t Mv[FW], sep = 0;
      len_masks(lv, Mv);
#pragma unroll
      for (int k = 0; k < FW; ++k) {
        Qn[k] = S[k] & Mv[k];
        sep = (uint32_t)k == (kl >> 2) ? S[k] : sep;
      }
      if (((sep >> (8u * (kl & 3u))) & 0xFFu) != (uint32_t)'_') return RS_EXACT;  // (its value window was not read)
    } else {
      uint32_t V[FW], Mv[FW];
      win_words(Vw, vo & 3u, V);
      len_masks(vl, Mv);
#pragma unroll
      for (int k = 0; k < FW; ++k) V[k] &= Mv[k];
      key_value_w(K, V, kl, Qn);
    }
    const uint32_t hv = fast_hash(pend, fold_w(Qn, lv), lv), hk = fast_hash(pend, fold_w(K, kl), kl);
    // one round trip: the pending node (its children's hashes), level l+1's windows, entry l+2's words
    const NodeF nf = load_fnode(B.fnodes, pend);
    load_strings(En, l + 1 < n, W, Vw);
    const uint4 Enn = bld4(B.ent, l + 2 < n ? 16u * (e0 + l + 2u) : RS_OOB);
    if (!confirm_f(nf, pp, pl, Q)) return RS_EXACT;
    uint32_t cv, ck;
    if (!(nf.len_flags & FAST_OVERFLOW)) {
      cv = child_of(nf, hv);
      ck = child_of(nf, hk);
    } else {  // children in the fast edge table
      uint64_t wv[TREE_PROBE], wk[TREE_PROBE];
      probe_round_f(B.fslots, hv, t.fmask, wv);
      probe_round_f(B.fslots, hk, t.fmask, wk);
      cv = match_chain_f(B.fslots, t.fmask, hv, wv);
      ck = match_chain_f(B.fslots, t.fmask, hk, wk);
    }
    if (cv == TREE_NONE && ck == TREE_NONE) return RL_NIL_RULE;  // neither edge: the walk stops (:309), nil
    const bool byv = cv != TREE_NONE;  // key "_" value first (:300-309)
    pl = byv ? lv : kl;
#pragma unroll
    for (int k = 0; k < FW; ++k) Q[k] = byv ? Qn[k] : K[k];
    pp = pend;
    pend = byv ? cv : ck;
    E = En;
    En = Enn;
  }
  // the last entry's node: confirmed, and its limit (:311-318)
  const NodeF v = load_fnode(B.fnodes, pend);
  if (!confirm_f(v, pp, pl, Q)) return RS_EXACT;
  return v.rule;
}

// First pass: one thread per descriptor; a block with a descriptor left to the exact walk raises
// its flag (every block writes its flag, so nothing needs clearing between batches). 6 waves per
// SIMD: 79 VGPRs and no spill (5 waves at the compiler's own 84; 7 or 8 spill). Measured and not
// kept (config 4, one box): a persistent grid of 1024 / 512 blocks striding over the chunks, so
// the pass leaves CUs to the engine stream's kernels: k_resolve 90 -> 95 / 113 us, the step
// slower; the engine stream at a higher priority than the front stream: no change.
// flags[gridDim.x] = seq when any block raised its flag (this launch's number: no clearing).
#ifndef RL_RESOLVE_WAVES
#define RL_RESOLVE_WAVES 6
#endif
__global__ __launch_bounds__(RS_NT) __attribute__((amdgpu_waves_per_eu(RL_RESOLVE_WAVES, RL_RESOLVE_WAVES))) void k_resolve(
    ResolveIn in, TreeDesc2 t, uint32_t* __restrict__ rule_out, uint32_t* __restrict__ flags, uint32_t seq) {
  const uint32_t i = blockIdx.x * RS_NT + threadIdx.x;
  const uint32_t r = i >= in.n_desc ? 0u : resolve_fast(in, t, fast_bufs(in, t), i);
  if (i < in.n_desc) rule_out[i] = r;
  const int any = __syncthreads_or(r == RS_EXACT);
  if (threadIdx.x == 0) {
    flags[blockIdx.x] = (uint32_t)any;
    if (any) flags[gridDim.x] = seq;
  }
}
// Second pass: blocks stride over the first pass's flags; a flagged block's descriptors left
// to the exact walk take it.
constexpr uint32_t RS_EXACT_BLOCKS = 2048;  // (a tree of long names leaves every descriptor here)
__global__ __launch_bounds__(RS_NT) void k_resolve_exact(ResolveIn in, TreeDesc2 t, uint32_t* __restrict__ rule_out,
                                                        const uint32_t* __restrict__ flags, uint32_t nblk, uint32_t seq) {
  if (flags[nblk] != seq) return;  // no block raised its flag (one load: the common case)
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    if (!flags[b]) continue;  // block-uniform
    const uint32_t i = b * RS_NT + threadIdx.x;
    if (i < in.n_desc && rule_out[i] == RS_EXACT) rule_out[i] = resolve_one(in, t, i);
  }
}

}  // namespace

// The same walk on the host, over host copies of the tree and the batch (tests/cshim: the
// device code path checked against the config oracle without a GPU): the first pass, then the
// exact walk for what it leaves. *exact (optional) tells which pass decided.
uint32_t resolve_one_host(const ResolveIn& in, const TreeDesc2& t, uint32_t i, bool* exact) {
  const uint32_t r = resolve_fast(in, t, fast_bufs(in, t), i);
  if (exact) *exact = r == RS_EXACT;
  return r == RS_EXACT ? resolve_one(in, t, i) : r;
}
uint32_t resolve_exact_host(const ResolveIn& in, const TreeDesc2& t, uint32_t i) { return resolve_one(in, t, i); }
uint32_t resolve_flag_words(uint32_t n_desc) { return (n_desc + RS_NT - 1) / RS_NT + 1u; }  // + the "any" word

int build_tree(const rl_tree_node* nodes, uint32_t n, const uint8_t* names, uint32_t names_len,
               std::vector<TreeNodeDev>& out_nodes, std::vector<uint64_t>& out_slots, uint32_t& mask,
               std::string& err) {
  out_nodes.assign(n, TreeNodeDev{});
  uint32_t cap = 16;
  while (cap < 8u * n) cap <<= 1;  // load <= 1/8: a probe chain rarely passes its first round
  out_slots.assign(cap + TREE_PROBE - 1, ~0ull);
  mask = cap - 1;
  for (uint32_t i = 0; i < n; ++i) {
    const rl_tree_node& x = nodes[i];
    if (x.parent != RL_TREE_ROOT && x.parent >= i) {
      err = "tree node " + std::to_string(i) + ": parent must precede its children";
      return RL_EINVAL;
    }
    if ((uint64_t)x.name_off + x.name_len > names_len || (x.parent != RL_TREE_ROOT && x.name_len == 0)) {
      err = "tree node " + std::to_string(i) + ": name outside the names blob or empty";
      return RL_EINVAL;
    }
    TreeNodeDev& d = out_nodes[i];
    d.parent = x.parent;
    d.name_off = x.name_off;
    d.name_len = x.name_len;
    d.rule = x.rule;
    d.n_children = 0;
    uint32_t f = TREE_FOLD0, w = 0;
    for (uint32_t k = 0; k < x.name_len; ++k) {
      const uint32_t c = names[x.name_off + k];
      w |= c << (8 * (k & 3));
      if ((k & 3) == 3 || k + 1 == x.name_len) {
        f = tree_fold_word(f, w);
        w = 0;
      }
      if (k < (uint32_t)TREE_INLINE) d.name[k >> 2] |= c << (8 * (k & 3));
    }
    const uint32_t h = d.hash = tree_hash(x.parent, f, x.name_len);
    if (x.parent != RL_TREE_ROOT) out_nodes[x.parent].n_children += 1;
    uint32_t s = h & mask;
    for (;; s = (s + 1) & mask) {
      const uint64_t o = out_slots[s];
      if ((uint32_t)o == TREE_EMPTY) break;
      const TreeNodeDev& y = out_nodes[(uint32_t)o];
      if (y.hash == h && y.parent == x.parent && y.name_len == x.name_len &&
          std::equal(names + y.name_off, names + y.name_off + y.name_len, names + x.name_off)) {
        // loadDescriptors (config_impl.go:131-135) / loadConfig (:239-242)
        err = std::string(x.parent == RL_TREE_ROOT ? "duplicate domain '" : "duplicate descriptor key '") +
              std::string(reinterpret_cast<const char*>(names + x.name_off), x.name_len) + "'";
        return RL_EINVAL;
      }
    }
    out_slots[s] = (uint64_t)h << 32 | i;
  }
  for (int j = 0; j < TREE_PROBE - 1; ++j) out_slots[cap + j] = out_slots[j];  // probe rounds never wrap
  return 0;
}

static uint32_t name_fold(const uint8_t* names, uint32_t off, uint32_t len) {
  uint32_t f = TREE_FOLD0, w = 0;
  for (uint32_t k = 0; k < len; ++k) {
    w |= (uint32_t)names[off + k] << (8 * (k & 3));
    if ((k & 3) == 3 || k + 1 == len) {
      f = tree_fold_word(f, w);
      w = 0;
    }
  }
  return f;
}

// Breadth-first ids (the domains first, then each node's children together, in id order), the
// children's hashes inline, overflow children and the domains in the fast edge table.
void build_fast_tree(const std::vector<TreeNodeDev>& nodes, const uint8_t* names, std::vector<FastNode>& out_nodes,
                     std::vector<uint64_t>& out_slots, uint32_t& mask, std::vector<uint32_t>* fast_id) {
  const uint32_t n = (uint32_t)nodes.size();
  std::vector<std::vector<uint32_t>> kids(n);
  std::vector<uint32_t> order, fid(n, TREE_NONE);
  for (uint32_t i = 0; i < n; ++i) {
    if (nodes[i].parent == RL_TREE_ROOT) order.push_back(i);
    else kids[nodes[i].parent].push_back(i);  // (build_tree: parents precede their children)
  }
  for (size_t q = 0; q < order.size(); ++q)
    for (uint32_t c : kids[order[q]]) order.push_back(c);
  for (uint32_t f = 0; f < n; ++f) fid[order[f]] = f;
  out_nodes.assign(n, FastNode{});
  std::vector<std::pair<uint32_t, uint32_t>> edges;  // (fast hash, fast id) for the edge table
  for (uint32_t f = 0; f < n; ++f) {
    const TreeNodeDev& d = nodes[order[f]];
    FastNode& x = out_nodes[f];
    x.parent = d.parent == RL_TREE_ROOT ? RL_TREE_ROOT : fid[d.parent];
    x.len_flags = std::min<uint32_t>(d.name_len, 0xFFFFFFu);
    x.rule = d.rule;
    for (int k = 0; k < 4; ++k) x.name[k] = d.name[k];
    for (int k = 0; k < FAST_CHILDREN; ++k) x.chash[k] = FAST_NO_CHILD;
    const std::vector<uint32_t>& ks = kids[order[f]];
    x.first_child = ks.empty() ? 0u : fid[ks[0]];
    std::vector<uint32_t> hs;
    for (uint32_t c : ks) hs.push_back(fast_hash(f, name_fold(names, nodes[c].name_off, nodes[c].name_len), nodes[c].name_len));
    bool over = ks.size() > (size_t)FAST_CHILDREN;
    for (size_t a = 0; a < hs.size() && !over; ++a)
      for (size_t b = a + 1; b < hs.size(); ++b) over |= hs[a] == hs[b];
    if (over) {
      x.len_flags |= FAST_OVERFLOW;
      for (size_t k = 0; k < ks.size(); ++k) edges.emplace_back(hs[k], fid[ks[k]]);
    } else {
      for (size_t k = 0; k < ks.size(); ++k) x.chash[k] = hs[k];
    }
    if (d.parent == RL_TREE_ROOT)
      edges.emplace_back(fast_hash(RL_TREE_ROOT, name_fold(names, d.name_off, d.name_len), d.name_len), f);
  }
  uint32_t cap = 16;
  while (cap < 8u * (uint32_t)edges.size()) cap <<= 1;  // load <= 1/8, as the exact walk's table
  out_slots.assign(cap + TREE_PROBE - 1, ~0ull);
  mask = cap - 1;
  for (const auto& e : edges) {
    uint32_t s = e.first & mask;
    while ((uint32_t)out_slots[s] != TREE_EMPTY) s = (s + 1) & mask;
    out_slots[s] = (uint64_t)e.first << 32 | e.second;
  }
  for (int j = 0; j < TREE_PROBE - 1; ++j) out_slots[cap + j] = out_slots[j];  // probe rounds never wrap
  if (fast_id) *fast_id = fid;
}

void launch_resolve(hipStream_t st, const ResolveIn& in, const TreeDesc2& t, uint32_t* rule_out, uint32_t* flags,
                    uint32_t seq) {
  if (!in.n_desc) return;
  const uint32_t nblk = resolve_flag_words(in.n_desc) - 1u;
  hipLaunchKernelGGL(k_resolve, dim3(nblk), dim3(RS_NT), 0, st, in, t, rule_out, flags, seq);
  hipLaunchKernelGGL(k_resolve_exact, dim3(std::min(nblk, RS_EXACT_BLOCKS)), dim3(RS_NT), 0, st, in, t, rule_out, flags,
                     nblk, seq);
}

}  // namespace rlhip
