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
// Device layout: the tree's nodes (32 B each: parent, name, rule, child count, name hash) and
// an open-addressing table over (parent, name) edges (u32 node ids, load <= 1/2), both small
// enough to stay in L2. Names are compared byte-exactly after the hash matches, so
// ("a_b") and ("a", "b") resolve exactly as the reference's string maps do. One thread per
// descriptor; the work is a few dependent L2 lookups per entry.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "rl_common.h"
#include "rl_resolve.h"

namespace rlhip {

namespace {

__device__ __forceinline__ uint32_t ld_byte(const uint8_t* p, uint32_t i) { return p[i]; }

// name = A, or A "_" B (finalKey, config_impl.go:126-129 and :300)
__device__ uint32_t lookup(const TreeDesc2& t, uint32_t parent, const uint8_t* bytes, uint32_t a_off, uint32_t a_len,
                           bool with_b, uint32_t b_off, uint32_t b_len) {
  uint32_t h = tree_hash_init(parent);
  for (uint32_t k = 0; k < a_len; ++k) h = tree_hash_step(h, ld_byte(bytes, a_off + k));
  uint32_t len = a_len;
  if (with_b) {
    h = tree_hash_step(h, '_');
    for (uint32_t k = 0; k < b_len; ++k) h = tree_hash_step(h, ld_byte(bytes, b_off + k));
    len += 1 + b_len;
  }
  h = tree_hash_final(h);
  for (uint32_t s = h & t.mask, probes = 0; probes <= t.mask; s = (s + 1) & t.mask, ++probes) {
    const uint32_t id = t.slots[s];
    if (id == TREE_EMPTY) return TREE_NONE;
    const TreeNodeDev nd = t.nodes[id];
    if (nd.hash != h || nd.parent != parent || nd.name_len != len) continue;
    bool eq = true;
    for (uint32_t k = 0; eq && k < a_len; ++k) eq = t.names[nd.name_off + k] == ld_byte(bytes, a_off + k);
    if (with_b) {
      eq = eq && t.names[nd.name_off + a_len] == '_';
      for (uint32_t k = 0; eq && k < b_len; ++k) eq = t.names[nd.name_off + a_len + 1 + k] == ld_byte(bytes, b_off + k);
    }
    if (eq) return id;
  }
  return TREE_NONE;
}

__global__ __launch_bounds__(256) void k_resolve(ResolveIn in, TreeDesc2 t, uint32_t* __restrict__ rule_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= in.n_desc) return;
  uint32_t rule = RL_NIL_RULE;
  const uint32_t dom = lookup(t, RL_TREE_ROOT, in.bytes, in.domain[2 * i], in.domain[2 * i + 1], false, 0, 0);
  if (dom != TREE_NONE) {
    const uint32_t ov = in.override_rule ? in.override_rule[i] : RL_NIL_RULE;
    if (ov != RL_NIL_RULE) {
      rule = ov;  // descriptor.GetLimit() != nil (config_impl.go:286-296)
    } else {
      const uint32_t e0 = in.entry_first[i], e1 = in.entry_first[i + 1];
      uint32_t parent = dom;
      for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t ko = in.entry[4 * e], kl = in.entry[4 * e + 1], vo = in.entry[4 * e + 2],
                       vl = in.entry[4 * e + 3];
        uint32_t nd = lookup(t, parent, in.bytes, ko, kl, true, vo, vl);  // key "_" value
        if (nd == TREE_NONE) nd = lookup(t, parent, in.bytes, ko, kl, false, 0, 0);  // key (default)
        if (nd == TREE_NONE) break;
        const TreeNodeDev x = t.nodes[nd];
        if (x.rule != RL_NIL_RULE && e == e1 - 1) rule = x.rule;
        if (x.n_children == 0) break;
        parent = nd;
      }
    }
  }
  rule_out[i] = rule;
}

}  // namespace

int build_tree(const rl_tree_node* nodes, uint32_t n, const uint8_t* names, uint32_t names_len,
               std::vector<TreeNodeDev>& out_nodes, std::vector<uint32_t>& out_slots, std::string& err) {
  out_nodes.assign(n, TreeNodeDev{});
  uint32_t cap = 16;
  while (cap < 2u * n) cap <<= 1;
  out_slots.assign(cap, TREE_EMPTY);
  const uint32_t mask = cap - 1;
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
    uint32_t h = tree_hash_init(x.parent);
    for (uint32_t k = 0; k < x.name_len; ++k) h = tree_hash_step(h, names[x.name_off + k]);
    d.hash = h = tree_hash_final(h);
    if (x.parent != RL_TREE_ROOT) out_nodes[x.parent].n_children += 1;
    uint32_t s = h & mask;
    for (;; s = (s + 1) & mask) {
      const uint32_t o = out_slots[s];
      if (o == TREE_EMPTY) break;
      const TreeNodeDev& y = out_nodes[o];
      if (y.hash == h && y.parent == x.parent && y.name_len == x.name_len &&
          std::equal(names + y.name_off, names + y.name_off + y.name_len, names + x.name_off)) {
        // loadDescriptors (config_impl.go:131-135) / loadConfig (:239-242)
        err = std::string(x.parent == RL_TREE_ROOT ? "duplicate domain '" : "duplicate descriptor key '") +
              std::string(reinterpret_cast<const char*>(names + x.name_off), x.name_len) + "'";
        return RL_EINVAL;
      }
    }
    out_slots[s] = i;
  }
  return 0;
}

void launch_resolve(hipStream_t st, const ResolveIn& in, const TreeDesc2& t, uint32_t* rule_out) {
  if (!in.n_desc) return;
  hipLaunchKernelGGL(k_resolve, dim3((in.n_desc + 255) / 256), dim3(256), 0, st, in, t, rule_out);
}

}  // namespace rlhip
