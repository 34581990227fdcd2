// K4 — bit-exact negative sampler: cyclic walk over the shuffled random_list
// with rejection of "used" items, refilled in ascending slot order.
//
// Restates AbstractSampler.random_num + sample_by_key_ids
// (recbole/sampler/sampler.py:82-101, 103-154):
//   random_num(num): value[t] = random_list[(random_pr + t) mod L], random_pr += num
//   round 0:  value[0..K*num) = random_num(K*num); key of slot t = keys[t mod K]
//   round i:  check = [t in check (ascending) if value[t] in used[key(t)]]
//             value[check] = random_num(len(check))
// Both branches of sample_by_key_ids (single key / many keys) have exactly this
// semantics. The walk is inherently sequential in `random_pr`, so one
// workgroup walks the batches in order; the membership tests of a round run in
// parallel over 1024 lanes and the refill order is a block prefix sum.
// The sampler only depends on the data pipeline (never on model state), so the
// trainer runs it ahead of the model step on a side stream.
#include "common.h"

namespace mirec {

constexpr int kSampThreads = 1024;

__global__ __launch_bounds__(kSampThreads) void sample_walk_kernel(
    const int32_t* __restrict__ rl, int64_t L, int64_t* __restrict__ pr_dev,
    const int64_t* __restrict__ keys, int64_t n_keys, int64_t batch_keys, int64_t n_batches,
    int64_t num, const int64_t* __restrict__ used_ptr, const int32_t* __restrict__ used_cols,
    int64_t key_space, int reject, int64_t* __restrict__ out, int64_t out_stride,
    int32_t* __restrict__ status,
    int32_t* __restrict__ rejA, int32_t* __restrict__ rejB) {
  __shared__ int scan_lds[kSampThreads / 64 + 1];
  int64_t pr = pr_dev[0] % L;
  int bad_key = 0;

  for (int64_t b = 0; b < n_batches; ++b) {
    const int64_t k0 = b * batch_keys;
    const int64_t Kb = min(batch_keys, n_keys - k0);
    if (Kb <= 0) break;
    const int64_t total = Kb * num;
    const int64_t* __restrict__ bkeys = keys + k0;
    int64_t* __restrict__ bout = out + b * out_stride;

    // ---- round 0: fill every slot, collect rejected slots in ascending order
    int32_t nrej = 0;
    for (int64_t base = 0; base < total; base += kSampThreads) {
      const int64_t t = base + threadIdx.x;
      int rej = 0;
      if (t < total) {
        int64_t pos = pr + t;
        if (pos >= L) pos %= L;
        const int32_t v = rl[pos];
        bout[t] = v;
        if (reject) {
          const int64_t key = bkeys[t % Kb];
          if (key < 0 || key >= key_space) {
            bad_key = 1;
          } else {
            rej = sorted_contains(used_cols, used_ptr[key], used_ptr[key + 1], v) ? 1 : 0;
          }
        }
      }
      int tot;
      const int excl = block_exclusive_scan(rej, scan_lds, &tot);
      if (rej) rejA[nrej + excl] = (int32_t)t;
      nrej += tot;
    }
    pr = (pr + total) % L;
    __syncthreads();

    // ---- refill rounds: the i-th rejected slot takes the i-th next walk value.
    // The reference loops until no slot is rejected; on adversarial inputs
    // (a user whose free items all sit outside the walk positions its slots
    // can reach) that never ends. Give up after a bound and report -3.
    int32_t* cur = rejA;
    int32_t* nxt = rejB;
    int64_t rounds = 0;
    const int64_t max_rounds = 4 * L + 1024;
    while (nrej > 0) {
      if (++rounds > max_rounds) {
        if (threadIdx.x == 0) atomicExch(status, -3);
        break;
      }
      int32_t nnew = 0;
      for (int32_t base = 0; base < nrej; base += kSampThreads) {
        const int32_t i = base + threadIdx.x;
        int rej = 0;
        int32_t t = 0;
        if (i < nrej) {
          t = cur[i];
          int64_t pos = pr + i;
          if (pos >= L) pos %= L;
          const int32_t v = rl[pos];
          bout[t] = v;
          const int64_t key = bkeys[t % Kb];
          rej = sorted_contains(used_cols, used_ptr[key], used_ptr[key + 1], v) ? 1 : 0;
        }
        int tot;
        const int excl = block_exclusive_scan(rej, scan_lds, &tot);
        if (rej) nxt[nnew + excl] = t;
        nnew += tot;
      }
      pr = (pr + nrej) % L;
      int32_t* tmp = cur; cur = nxt; nxt = tmp;
      nrej = nnew;
      __syncthreads();
    }
  }
  if (bad_key) atomicExch(status, -2);
  __syncthreads();
  if (threadIdx.x == 0) pr_dev[0] = pr;
}

}  // namespace mirec

using namespace mirec;

extern "C" size_t mirec_sample_walk_workspace_size(int64_t batch_keys, int64_t num) {
  if (batch_keys <= 0 || num <= 0) return 256;
  return (size_t)(2 * batch_keys * num) * sizeof(int32_t) + 256;
}

extern "C" int mirec_sample_walk(const int32_t* random_list, int64_t L, int64_t* pr_dev,
                                 const int64_t* keys, int64_t n_keys, int64_t batch_keys,
                                 int64_t n_batches, int64_t num, const int64_t* used_ptr,
                                 const int32_t* used_cols, int64_t n_key_space, int reject,
                                 int64_t* out, int64_t out_stride, int32_t* status_dev, void* ws,
                                 size_t ws_bytes,
                                 void* stream) {
  if (L <= 0 || !random_list || !pr_dev || !out || !status_dev || n_keys < 0 || num < 0 ||
      batch_keys <= 0 || n_batches < 0) {
    set_error("mirec_sample_walk: bad arguments (L=%lld)", (long long)L);
    return -1;
  }
  if (n_keys == 0 || num == 0 || n_batches == 0) return 0;
  if (reject && (!used_ptr || !used_cols)) {
    set_error("mirec_sample_walk: reject=1 needs the used-id CSR");
    return -1;
  }
  if (batch_keys * num > INT32_MAX) {
    set_error("mirec_sample_walk: batch_keys*num exceeds int32");
    return -1;
  }
  const size_t need = mirec_sample_walk_workspace_size(batch_keys, num);
  if (!ws || ws_bytes < need) {
    set_error("mirec_sample_walk: workspace %zu < %zu", ws_bytes, need);
    return -1;
  }
  if (out_stride == 0) out_stride = batch_keys * num;
  int32_t* rejA = (int32_t*)ws;
  int32_t* rejB = rejA + batch_keys * num;
  hipLaunchKernelGGL(sample_walk_kernel, dim3(1), dim3(kSampThreads), 0, (hipStream_t)stream,
                     random_list, L, pr_dev, keys, n_keys, batch_keys, n_batches, num, used_ptr,
                     used_cols, n_key_space, reject, out, out_stride, status_dev, rejA, rejB);
  return launch_status("mirec_sample_walk");
}
