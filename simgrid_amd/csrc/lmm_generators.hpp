// Synthetic LMM system generators (input generation only — no solver arithmetic here).
//
// Both generators drive a System-like "builder" through the reference's own mutation API
// (constraint_new / set_concurrency_limit / variable_new / set_concurrency_share / expand /
// expand_add), so the same call sequence can be replayed against the product System and the
// oracle and yields identical systems.
//
//  * maxmin_bench(): the exact generator of teshsuite/surf/maxmin_bench/maxmin_bench.cpp:21-108
//    (Park-Miller RNG, same consumption order, float rate_no_limit comparison), used for the
//    golden-pinned configs C1 ("small") and C3 ("medium").
//  * synthetic(): the scaled "maxmin_bench-style" generator of SURVEY.md §8(d) C2.  The reference
//    RNG yields only 1000 distinct values, so constraint indices come from splitmix64 instead;
//    bounds and weights keep maxmin_bench's quantised distributions.
#pragma once

#include <cstdint>
#include <vector>

namespace lmm_gen {

// ---- maxmin_bench.cpp:18-35 ----
struct ParkMiller {
  int64_t seedx = 0;
  int myrand() {
    seedx = seedx * 16807 % 2147483647;
    return static_cast<int32_t>(seedx % 1000);
  }
  double float_random(double max) { return (max * myrand()) / (1000.0 + 1.0); }
  unsigned int_random(int max) { return static_cast<uint32_t>(float_random(max)); }
};

struct BenchClass {  // maxmin_bench.cpp:110-116
  int nb_cnst, nb_var, pw_base, pw_max;
};
static constexpr BenchClass kBenchClasses[4] = {
    {10, 10, 1, 2}, {100, 100, 3, 6}, {2000, 2000, 5, 8}, {20000, 20000, 7, 10}};

inline int bench_nb_elem(const BenchClass& k) { return (1 << k.pw_base) + (1 << (8 * k.pw_max / 10)); }

// One run of maxmin_bench's test() (maxmin_bench.cpp:37-83), run index `run` (seed = run + 1).
// Returns the two RNG check values the tesh pins ("Starting i: (x)", "Starting to solve(y)").
template <class B>
void maxmin_bench(B& b, const BenchClass& k, int run, int* check_start, int* check_solve,
                  std::vector<typename B::Cnst>* cnst_out, std::vector<typename B::Var>* var_out) {
  const float rate_no_limit = 0.2f;  // maxmin_bench.cpp:122 (a float!)
  const int max_share = 2;           // maxmin_bench.cpp:169
  const int nb_elem = bench_nb_elem(k);
  ParkMiller r;
  r.seedx = run + 1;
  *check_start = r.myrand() % 1000;

  std::vector<typename B::Cnst> cnst(k.nb_cnst);
  std::vector<int> used(k.nb_cnst);
  for (int i = 0; i < k.nb_cnst; i++) {
    cnst[i] = b.constraint_new(r.float_random(10.0));
    int l;
    if (rate_no_limit > r.float_random(1.0))
      l = -1;
    else
      l = (1 << k.pw_base) + (1 << r.int_random(k.pw_max));
    b.set_concurrency_limit(cnst[i], l);
  }
  std::vector<typename B::Var> var(k.nb_var);
  for (int i = 0; i < k.nb_var; i++) {
    var[i] = b.variable_new(1.0, -1.0, nb_elem);
    int share = 1 + r.int_random(max_share);
    b.set_concurrency_share(var[i], share);
    for (int j = 0; j < k.nb_cnst; j++)
      used[j] = 0;
    for (int j = 0; j < nb_elem; j++) {
      int c = r.int_random(k.nb_cnst);
      if (used[c] >= share) {
        j--;
        continue;
      }
      b.expand(cnst[c], var[i], r.float_random(1.5));
      b.expand_add(cnst[c], var[i], r.float_random(1.5));
      used[c]++;
    }
  }
  *check_solve = r.myrand() % 1000;
  if (cnst_out)
    *cnst_out = std::move(cnst);
  if (var_out)
    *var_out = std::move(var);
}

// ---- scaled generator (SURVEY.md §8(d) C2 and its stress variant) ----
struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  unsigned u1000() { return unsigned(next() % 1000); }
};

struct SynthParams {
  int64_t nb_cnst = 1000000;
  int64_t nb_var = 10000000;
  int elems_per_var = 8;
  uint64_t seed = 1;
  int max_share = 2;         // concurrency share drawn in [1, max_share] (duplicates allowed)
  int penalty_mix = 0;       // 0: all penalties 1; 1: penalties drawn from {1, 2, 4}
  int bounded_permille = 0;  // variables with a finite bound, per mille
  int fatpipe_permille = 0;  // FATPIPE constraints, per mille
  int cnst_offset = 0;       // (batched systems) unused by the generator itself
};

template <class B>
void synthetic(B& b, const SynthParams& p, std::vector<typename B::Cnst>* cnst_out,
               std::vector<typename B::Var>* var_out) {
  SplitMix64 r{p.seed * 0x2545F4914F6CDD1Dull + 1};
  std::vector<typename B::Cnst> cnst(p.nb_cnst);
  for (int64_t i = 0; i < p.nb_cnst; i++) {
    cnst[i] = b.constraint_new(10.0 * r.u1000() / 1001.0);
    if (p.fatpipe_permille && (int)r.u1000() < p.fatpipe_permille)
      b.unshare(cnst[i]);
  }
  std::vector<typename B::Var> var;
  if (var_out)
    var.resize(p.nb_var);
  const double pen_tab[3] = {1.0, 2.0, 4.0};
  std::vector<int64_t> used_c;
  std::vector<int> used_n;
  for (int64_t i = 0; i < p.nb_var; i++) {
    double pen = p.penalty_mix ? pen_tab[r.next() % 3] : 1.0;
    double bound = -1.0;
    if (p.bounded_permille && (int)r.u1000() < p.bounded_permille)
      bound = 0.01 + 2.0 * r.u1000() / 1001.0;
    auto v = b.variable_new(pen, bound, p.elems_per_var);
    int share = 1 + int(r.next() % unsigned(p.max_share));
    b.set_concurrency_share(v, share);
    used_c.clear();
    used_n.clear();
    for (int j = 0; j < p.elems_per_var; j++) {
      int64_t c = int64_t(r.next() % uint64_t(p.nb_cnst));
      size_t s = 0;
      while (s < used_c.size() && used_c[s] != c)
        s++;
      if (s < used_c.size() && used_n[s] >= share) {
        j--;
        continue;
      }
      b.expand(cnst[c], v, 1.5 * r.u1000() / 1001.0);
      b.expand_add(cnst[c], v, 1.5 * r.u1000() / 1001.0);
      if (s == used_c.size()) {
        used_c.push_back(c);
        used_n.push_back(1);
      } else {
        used_n[s]++;
      }
    }
    if (var_out)
      var[i] = v;
  }
  if (cnst_out)
    *cnst_out = std::move(cnst);
  if (var_out)
    *var_out = std::move(var);
}

}  // namespace lmm_gen
