// lmm_cc_kernels.hpp — connected components of the variable-constraint graph on gfx950 (included by
// lmm_hip.hip).
//
// The reference finds a component by a recursive walk from a modified constraint through its enabled
// variables' other constraints (System::update_modified_set_rec, maxmin.cpp:898-922).  Spreading a system's
// components over GPUs needs every component at once, so here the whole bipartite graph is
// labelled in two passes, lock-free union-find in the style of ECL-CC:
//   nodes    variable v -> v, constraint c -> nV + c; parent[] with parent[x] <= x at all times;
//   cc_hook  one thread per variable: for each element (v, c) the roots of v and nV + c are united by
//            hooking the larger root under the smaller one with a compare-and-swap (a failed CAS restarts
//            from the value it found, which is an ancestor); finds halve the path as they go (plain
//            stores of an ancestor: any interleaving keeps parent[x] <= x and the same trees);
//   cc_root  after the hooks (kernel boundary), each node's root — the SMALLEST node of its component, since a
//            root only ever goes under a smaller one: the labelling is deterministic, whatever the order in
//            which the CASes landed; root flags -> exclusive scan -> compact component ids in root order.
// Memory traffic: the CSR once (4 B per element + 4 B per row offset) plus the parent gathers, which
// collapse to the root after the first few hooks of a component; HBM / latency bound, no MFMA.
#pragma once
#include "lmm_dev.hpp"

namespace lmmdev {

__global__ void __launch_bounds__(kBlock) cc_init(int32_t* par, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    par[i] = int32_t(i);
}

// Root of x with path halving (ECL-CC's intermediate pointer jumping).  Loads are relaxed agent-scope
// atomics: other threads rewrite parent[] meanwhile.
__device__ __forceinline__ int32_t cc_rep(int32_t* par, int32_t x) {
  int32_t cur = ld_rlx(&par[x]);
  if (cur != x) {
    int32_t prev = x, next;
    while (cur > (next = ld_rlx(&par[cur]))) {
      st_rlx(&par[prev], next);
      prev = cur;
      cur = next;
    }
  }
  return cur;
}

__global__ void __launch_bounds__(kBlock) cc_hook(Dev s, int32_t* par) {
  for (int64_t v = int64_t(blockIdx.x) * kBlock + threadIdx.x; v < s.nV; v += int64_t(gridDim.x) * kBlock) {
    const uint32_t b = s.var_ptr[v], e = s.var_ptr[v + 1];
    int32_t a = cc_rep(par, int32_t(v));
    for (uint32_t j = b; j < e; j++) {
      int32_t o = cc_rep(par, s.nV + s.csr_c[j]);
      while (a != o) {  // hook the larger root under the smaller one
        if (a < o) {
          const int32_t r = atomicCAS(&par[o], o, a);
          if (r == o)
            break;
          o = r;  // o had been hooked meanwhile: continue from its new parent (an ancestor)
        } else {
          const int32_t r = atomicCAS(&par[a], a, o);
          if (r == a) {
            a = o;
            break;
          }
          a = r;
        }
      }
      a = cc_rep(par, a);
    }
  }
}

// Final roots (all hooks done) and root flags for the scan.
__global__ void __launch_bounds__(kBlock) cc_root(int32_t* par, int64_t n, int64_t* is_root) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    int32_t r = par[i];
    while (true) {
      const int32_t q = par[r];
      if (q == r)
        break;
      r = q;
    }
    par[i] = r;  // (only this thread writes par[i] now; readers of par[i] see an ancestor either way)
    is_root[i] = r == i;
  }
}

// Compact labels: component id = number of roots before the node's root.
__global__ void __launch_bounds__(kBlock) cc_label(const int32_t* par, const int64_t* rank, int64_t nv, int64_t n,
                                                   int32_t* var_label, int32_t* cnst_label) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t l = int32_t(rank[par[i]]);
    if (i < nv)
      var_label[i] = l;
    else
      cnst_label[i - nv] = l;
  }
}

}  // namespace lmmdev
