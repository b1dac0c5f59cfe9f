// Test shim: the device resolve walk (rl_resolve.hip, resolve_one) run on the host over host
// copies of the tree and the batch, so tests check the kernel's own code path against the
// config oracle without a GPU (tests/test_resolve_host.py). Test infrastructure only.
#include <string>
#include <vector>

#include "rl_resolve.h"

// exact_out (may be NULL): per descriptor 1 when k_resolve's first pass left it to the exact
// walk (k_resolve_exact), 0 when the level-pipelined walk decided it. mode 1: the exact walk
// alone (resolve_one), for comparison.
extern "C" int rls_resolve2(const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names, uint32_t names_len,
                            const rl_resolve_batch* b, uint32_t* rule_out, uint8_t* exact_out, int mode) {
  std::vector<rlhip::TreeNodeDev> hn;
  std::vector<uint64_t> hs;
  uint32_t mask = 0;
  std::string err;
  const int rc = rlhip::build_tree(nodes, n_nodes, names, names_len, hn, hs, mask, err);
  if (rc) return rc;
  std::vector<rlhip::FastNode> fn;
  std::vector<uint64_t> fs;
  uint32_t fmask = 0;
  rlhip::build_fast_tree(hn, names, fn, fs, fmask);
  const rlhip::TreeDesc2 t{hn.data(), hs.data(), names, mask, fn.data(), fs.data(), fmask, (uint32_t)fn.size()};
  const rlhip::ResolveIn in{b->n_desc, b->n_entries, b->bytes_len, b->bytes, b->domain,
                            b->entry_first, b->entry, b->override_rule};
  for (uint32_t i = 0; i < b->n_desc; ++i) {
    bool ex = true;
    rule_out[i] = mode == 1 ? rlhip::resolve_exact_host(in, t, i) : rlhip::resolve_one_host(in, t, i, &ex);
    if (exact_out) exact_out[i] = ex ? 1 : 0;
  }
  return 0;
}
extern "C" int rls_resolve(const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names, uint32_t names_len,
                           const rl_resolve_batch* b, uint32_t* rule_out) {
  return rls_resolve2(nodes, n_nodes, names, names_len, b, rule_out, nullptr, 0);
}
// tree_hash(parent, fold(name), len) as the device computes it (tests build colliding names)
extern "C" uint32_t rls_tree_hash(uint32_t parent, const uint8_t* name, uint32_t len) {
  uint32_t f = rlhip::TREE_FOLD0, w = 0;
  for (uint32_t k = 0; k < len; ++k) {
    w |= (uint32_t)name[k] << (8 * (k & 3));
    if ((k & 3) == 3 || k + 1 == len) {
      f = rlhip::tree_fold_word(f, w);
      w = 0;
    }
  }
  return rlhip::tree_hash(parent, f, len);
}
// fast_hash(parent, fold(name), len): the first pass's edge hash (parent = a fast id)
extern "C" uint32_t rls_fast_hash(uint32_t parent, const uint8_t* name, uint32_t len) {
  return rls_tree_hash(parent, name, len) & ~1u;
}
// The first pass's (breadth-first) id of tree node `id`, or 0xFFFFFFFF on a bad tree.
extern "C" uint32_t rls_fast_id(const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names, uint32_t names_len,
                                uint32_t id) {
  std::vector<rlhip::TreeNodeDev> hn;
  std::vector<uint64_t> hs;
  uint32_t mask = 0;
  std::string err;
  if (rlhip::build_tree(nodes, n_nodes, names, names_len, hn, hs, mask, err) || id >= n_nodes) return 0xFFFFFFFFu;
  std::vector<rlhip::FastNode> fn;
  std::vector<uint64_t> fs;
  std::vector<uint32_t> fid;
  uint32_t fmask = 0;
  rlhip::build_fast_tree(hn, names, fn, fs, fmask, &fid);
  return fid[id];
}
