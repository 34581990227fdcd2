/*
 * oracle/walk.c — TEST INFRASTRUCTURE ONLY (parity checker / CPU baseline).
 * Never linked into, called by, or shipped with the product path
 * (recbole_amd/*); only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Plain-C restatement of RecBole's negative sampler walk:
 *   AbstractSampler.random_num        recbole/sampler/sampler.py:82-101
 *   AbstractSampler.sample_by_key_ids recbole/sampler/sampler.py:103-154
 *     (multi-key branch :144-153; the single-key branch :120-143 computes the
 *      same thing with np.isin — rejected slots are refilled, in ascending slot
 *      order, with consecutive values of the walk until none is used)
 *   Sampler.get_used_ids              recbole/sampler/sampler.py:206-227
 *
 * Parity pinning: the reference's own tests pin only the id RANGE of sampled
 * negatives (tests/data/test_dataloader.py:76-84, 101-113); the values are
 * pinned here against the algorithm as written in sampler.py (see
 * tests/test_oracle.py, which also cross-checks this C code against a
 * line-by-line numpy restatement of both reference branches).
 */
#include <stdint.h>
#include <stdlib.h>

static int contains(const int32_t* cols, int64_t lo, int64_t hi, int32_t key) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (cols[mid] == key) return 1;
    if (cols[mid] < key) lo = mid + 1; else hi = mid;
  }
  return 0;
}

/* returns 0, -2 on an out-of-range key (reference: ValueError), or -3 when the
 * rejection rounds exceed 4L+1024 (the reference would loop forever) */
int oracle_sample_walk(const int32_t* rl, int64_t L, int64_t* pr_io, const int64_t* keys,
                       int64_t K, int64_t num, const int64_t* used_ptr,
                       const int32_t* used_cols, int64_t key_space, int reject, int64_t* out) {
  int64_t total = K * num;
  int64_t pr = *pr_io % L;
  int64_t* check = (int64_t*)malloc(sizeof(int64_t) * (total > 0 ? total : 1));
  int64_t n_check = 0;
  for (int64_t k = 0; k < K; ++k)
    if (keys[k] < 0 || keys[k] >= key_space) { free(check); return -2; }
  /* value_ids = random_num(total) */
  for (int64_t t = 0; t < total; ++t) {
    out[t] = rl[(pr + t) % L];
  }
  pr = (pr + total) % L;
  if (reject) {
    for (int64_t t = 0; t < total; ++t) {
      int64_t key = keys[t % K];
      if (contains(used_cols, used_ptr[key], used_ptr[key + 1], (int32_t)out[t]))
        check[n_check++] = t;
    }
    int64_t rounds = 0;
    while (n_check > 0) {
      if (++rounds > 4 * L + 1024) { free(check); *pr_io = pr; return -3; }  /* livelock */
      /* value_ids[check_list] = random_num(len(check_list)) */
      for (int64_t i = 0; i < n_check; ++i) out[check[i]] = rl[(pr + i) % L];
      pr = (pr + n_check) % L;
      int64_t m = 0;
      for (int64_t i = 0; i < n_check; ++i) {
        int64_t t = check[i];
        int64_t key = keys[t % K];
        if (contains(used_cols, used_ptr[key], used_ptr[key + 1], (int32_t)out[t]))
          check[m++] = t;
      }
      n_check = m;
    }
  }
  *pr_io = pr;
  free(check);
  return 0;
}
