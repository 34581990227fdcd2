// Host-side data-pipeline primitives: the integer work of
// the atomic-file pipeline at 20 M interactions — grouping rows by user for the
// ratio split / leave-one-out (recbole/data/dataset.py:1249-1337), the per-phase
// used-id sets of the sampler (recbole/sampler/sampler.py:206-227) — as O(n)
// counting passes instead of comparison sorts. CPU code in the same library as
// the kernels (no GPU needed); plain pointers to host memory.
#include "common.h"

#include <algorithm>
#include <thread>
#include <vector>

using namespace mirec;

// order = the stable sort permutation of keys (keys in [0, key_space)):
// counting sort, one histogram pass and one scatter pass.
extern "C" int mirec_host_counting_order(const int64_t* keys, int64_t n, int64_t key_space,
                                         int64_t* order) {
  if (n < 0 || key_space <= 0 || (n > 0 && (!keys || !order))) {
    set_error("mirec_host_counting_order: bad arguments");
    return -1;
  }
  std::vector<int64_t> start((size_t)key_space + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = keys[i];
    if (k < 0 || k >= key_space) {
      set_error("mirec_host_counting_order: key %lld at %lld outside [0, %lld)", (long long)k,
                (long long)i, (long long)key_space);
      return -1;
    }
    ++start[(size_t)k + 1];
  }
  for (int64_t k = 0; k < key_space; ++k) start[(size_t)k + 1] += start[(size_t)k];
  for (int64_t i = 0; i < n; ++i) order[start[(size_t)keys[i]]++] = i;
  return 0;
}

// CSR of the DISTINCT (key, value) pairs, each row's values ascending:
// ptr[n_keys + 1], cols[<= n] (the caller sizes cols for n). Returns the number of
// distinct pairs (ptr[n_keys]) or < 0. Values must lie in [0, 2^31).
extern "C" int64_t mirec_host_csr_build(const int64_t* keys, const int64_t* vals, int64_t n,
                                        int64_t n_keys, int64_t* ptr, int32_t* cols) {
  if (n < 0 || n_keys < 0 || !ptr || (n > 0 && (!keys || !vals || !cols))) {
    set_error("mirec_host_csr_build: bad arguments");
    return -1;
  }
  std::fill(ptr, ptr + n_keys + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = keys[i], v = vals[i];
    if (k < 0 || k >= n_keys || v < 0 || v > INT32_MAX) {
      set_error("mirec_host_csr_build: pair (%lld, %lld) out of range", (long long)k,
                (long long)v);
      return -1;
    }
    ++ptr[k + 1];
  }
  for (int64_t k = 0; k < n_keys; ++k) ptr[k + 1] += ptr[k];
  std::vector<int64_t> fill(ptr, ptr + n_keys);
  for (int64_t i = 0; i < n; ++i) cols[fill[(size_t)keys[i]]++] = (int32_t)vals[i];
  // sort + dedupe each row in place (rows split over threads by element count),
  // then compact the rows to the front
  std::vector<int64_t> len((size_t)n_keys);
  auto sort_rows = [&](int64_t k0, int64_t k1) {
    for (int64_t k = k0; k < k1; ++k) {
      int32_t* b = cols + ptr[k];
      int32_t* e = cols + ptr[k + 1];
      std::sort(b, e);
      len[(size_t)k] = std::unique(b, e) - b;
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(
      std::min<unsigned>(std::thread::hardware_concurrency(), 16u), n / (1 << 16)));
  if (nt <= 1) {
    sort_rows(0, n_keys);
  } else {
    std::vector<std::thread> th;
    int64_t k0 = 0;
    for (int t = 0; t < nt && k0 < n_keys; ++t) {
      const int64_t target = n * (t + 1) / nt;          // balanced by elements
      const int64_t k1 = t == nt - 1 ? n_keys
                                     : std::upper_bound(ptr, ptr + n_keys + 1, target) - ptr - 1;
      const int64_t hi = std::max(k0 + 1, std::min(k1, n_keys));
      th.emplace_back(sort_rows, k0, hi);
      k0 = hi;
    }
    for (auto& x : th) x.join();
  }
  int64_t w = 0;
  for (int64_t k = 0; k < n_keys; ++k) {
    const int64_t b = ptr[k];
    ptr[k] = w;
    if (w != b) std::copy(cols + b, cols + b + len[(size_t)k], cols + w);
    w += len[(size_t)k];
  }
  ptr[n_keys] = w;
  return w;
}
