// Test shim: the device resolve walk (rl_resolve.hip, resolve_one) run on the host over host
// copies of the tree and the batch, so tests check the kernel's own code path against the
// config oracle without a GPU (tests/test_resolve_host.py). Test infrastructure only.
#include <string>
#include <vector>

#include "rl_resolve.h"

extern "C" int rls_resolve(const rl_tree_node* nodes, uint32_t n_nodes, const uint8_t* names, uint32_t names_len,
                           const rl_resolve_batch* b, uint32_t* rule_out) {
  std::vector<rlhip::TreeNodeDev> hn;
  std::vector<uint64_t> hs;
  uint32_t mask = 0;
  std::string err;
  const int rc = rlhip::build_tree(nodes, n_nodes, names, names_len, hn, hs, mask, err);
  if (rc) return rc;
  const rlhip::TreeDesc2 t{hn.data(), hs.data(), names, mask};
  const rlhip::ResolveIn in{b->n_desc, b->n_entries, b->bytes_len, b->bytes, b->domain,
                            b->entry_first, b->entry, b->override_rule};
  for (uint32_t i = 0; i < b->n_desc; ++i) rule_out[i] = rlhip::resolve_one_host(in, t, i);
  return 0;
}
