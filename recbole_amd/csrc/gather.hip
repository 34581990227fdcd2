// K1 — row gather out[i,:] = table[idx[i],:] for any row width.
// Replaces nn.Embedding forward (torch embedding = index_select of rows,
// bpr.py:58-72) and the column gathers of Interaction slicing / shuffle
// (recbole/data/interaction.py:260-276). Vectorised to 16 B per lane whenever
// the row width and both base pointers allow it, so one wave moves 1 KiB per
// instruction; consecutive lanes walk one row, so each row is read as whole
// 64-B segments.
#include "common.h"
#include <algorithm>

namespace mirec {

template <typename V, typename I>
__global__ __launch_bounds__(256) void gather_kernel(const V* __restrict__ table, int64_t n_rows,
                                                     int64_t vpr, const I* __restrict__ idx,
                                                     int64_t n, V* __restrict__ out) {
  const int64_t total = n * vpr;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / vpr;
    const int64_t c = e - i * vpr;
    int64_t r = (int64_t)idx[i];
    // out-of-range ids are a caller bug; clamp so the kernel never faults
    r = r < 0 ? 0 : (r >= n_rows ? n_rows - 1 : r);
    out[e] = table[r * vpr + c];
  }
}

template <typename I>
static int gather_impl(const void* table, int64_t n_rows, int64_t row_bytes, const I* idx,
                       int64_t n, void* out, hipStream_t st) {
  if (n == 0) return 0;
  if (!table || !idx || !out || n < 0 || row_bytes <= 0 || n_rows <= 0) {
    set_error("mirec_gather_rows: bad arguments");
    return -1;
  }
  const uintptr_t al = (uintptr_t)table | (uintptr_t)out | (uintptr_t)row_bytes;
  int64_t total;
  auto grid = [&](int64_t tot) {
    int64_t g = (tot + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return dim3((unsigned)g);
  };
  if ((al & 15) == 0) {
    const int64_t vpr = row_bytes / 16;
    total = n * vpr;
    hipLaunchKernelGGL((gather_kernel<int4, I>), grid(total), dim3(256), 0, st,
                       (const int4*)table, n_rows, vpr, idx, n, (int4*)out);
  } else if ((al & 7) == 0) {
    const int64_t vpr = row_bytes / 8;
    total = n * vpr;
    hipLaunchKernelGGL((gather_kernel<int2, I>), grid(total), dim3(256), 0, st,
                       (const int2*)table, n_rows, vpr, idx, n, (int2*)out);
  } else if ((al & 3) == 0) {
    const int64_t vpr = row_bytes / 4;
    total = n * vpr;
    hipLaunchKernelGGL((gather_kernel<int, I>), grid(total), dim3(256), 0, st,
                       (const int*)table, n_rows, vpr, idx, n, (int*)out);
  } else {
    const int64_t vpr = row_bytes;
    total = n * vpr;
    hipLaunchKernelGGL((gather_kernel<char, I>), grid(total), dim3(256), 0, st,
                       (const char*)table, n_rows, vpr, idx, n, (char*)out);
  }
  return launch_status("mirec_gather_rows");
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_gather_rows(const void* table, int64_t n_rows, int64_t row_bytes,
                                 const int64_t* idx, int64_t n, void* out, void* stream) {
  return gather_impl<int64_t>(table, n_rows, row_bytes, idx, n, out, (hipStream_t)stream);
}

extern "C" int mirec_gather_rows_i32idx(const void* table, int64_t n_rows, int64_t row_bytes,
                                        const int32_t* idx, int64_t n, void* out, void* stream) {
  return gather_impl<int32_t>(table, n_rows, row_bytes, idx, n, out, (hipStream_t)stream);
}

// Sliding-window gather for the sequential loaders (SequentialDataLoader.augmentation,
// recbole/data/dataloader/sequential_dataloader.py:95-127, computed on the device):
// out[i, t] = col[start[i] + t] for t < len[i], else 0; elements of 4 or 8 bytes.
namespace mirec {

template <typename T>
__global__ __launch_bounds__(256) void window_gather_kernel(const T* __restrict__ col,
                                                            const int64_t* __restrict__ start,
                                                            const int64_t* __restrict__ len,
                                                            int64_t n, int L, T* __restrict__ out) {
  const int64_t total = n * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / L;
    const int t = (int)(e - i * L);
    out[e] = t < len[i] ? col[start[i] + t] : T(0);
  }
}

}  // namespace mirec

extern "C" int mirec_window_gather(const void* col, int32_t elem_bytes, const int64_t* start,
                                   const int64_t* len, int64_t n, int32_t L, void* out,
                                   void* stream) {
  if (n == 0) return 0;
  if (!col || !start || !len || !out || n < 0 || L <= 0 || (elem_bytes != 4 && elem_bytes != 8)) {
    set_error("mirec_window_gather: bad arguments");
    return -1;
  }
  int64_t g = (n * L + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  hipStream_t st = (hipStream_t)stream;
  if (elem_bytes == 8)
    hipLaunchKernelGGL(window_gather_kernel<int64_t>, dim3((unsigned)g), dim3(256), 0, st,
                       (const int64_t*)col, start, len, n, L, (int64_t*)out);
  else
    hipLaunchKernelGGL(window_gather_kernel<int32_t>, dim3((unsigned)g), dim3(256), 0, st,
                       (const int32_t*)col, start, len, n, L, (int32_t*)out);
  return launch_status("mirec_window_gather");
}

// ---- chunk preparation (include/mirec.h mirec_chunk_prep)
namespace mirec {

int sort_chunk_pair(const int64_t* ukeys, int64_t nU_keys, int64_t Bu, int64_t u_space,
                    int32_t* u_perm, int32_t* u_uniq, int32_t* u_seg, int32_t* u_nu,
                    const int64_t* ikeys, int64_t nI_keys, int64_t Bi, int64_t i_space,
                    int32_t* i_perm, int32_t* i_uniq, int32_t* i_seg, int32_t* i_nu,
                    int64_t n_batches, int32_t* u_ahead, int32_t* u_nah, int32_t* i_ahead,
                    int32_t* i_nah, void* ws, size_t ws_bytes, hipStream_t st);

__global__ __launch_bounds__(256) void chunk_keys_kernel(const int64_t* __restrict__ users,
                                                         const int64_t* __restrict__ items,
                                                         int64_t s0, int64_t n, int64_t Bc,
                                                         int64_t KI, int64_t* __restrict__ ukeys,
                                                         int64_t* __restrict__ ikeys) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    ukeys[i] = users[s0 + i];
    ikeys[(i / Bc) * KI + i % Bc] = items[s0 + i];
  }
}

}  // namespace mirec

static bool prep_ok(const mirec_chunk_prep* p) {
  if (!p || !p->users || !p->items || !p->user_keys || !p->item_keys || p->n_batches <= 0 ||
      p->Bc <= 0 || p->T <= 0 || p->s0 < 0) {
    mirec::set_error("mirec_prepare_chunk: bad arguments");
    return false;
  }
  return true;
}

extern "C" int mirec_prepare_chunk_walk(const mirec_chunk_prep* p, void* stream) {
  if (!prep_ok(p)) return -1;
  const int64_t n = p->n_batches * p->Bc, KI = (1 + p->T) * p->Bc;
  if (p->spec_ws && !p->alias_thr)        // K4s: walk + key rows, no keys launch
    return mirec_sample_walk_spec(p->random_list, p->L, p->pr_dev, p->users + p->s0,
                                  p->items + p->s0, p->n_batches, p->Bc, p->T, p->used_ptr,
                                  p->used_cols, p->used_bits, p->n_bits, p->n_users, p->reject,
                                  p->r_mean, p->r_sd, p->item_keys + p->Bc, KI, p->user_keys,
                                  p->item_keys, KI, p->status, p->spec_ws, p->spec_ws_bytes,
                                  stream);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(mirec::chunk_keys_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     p->users, p->items, p->s0, n, p->Bc, KI, p->user_keys, p->item_keys);
  int rc = mirec::launch_status("mirec_prepare_chunk: keys");
  if (rc) return rc;
  if (p->alias_thr)
    return mirec_sample_alias(p->alias_thr, p->alias_idx, p->n_alias, p->alias_seed,
                              p->alias_counter, p->user_keys, n, p->Bc, p->T, p->used_ptr,
                              p->used_cols, p->used_bits, p->n_bits, p->n_users, p->reject,
                              p->item_keys + p->Bc, KI, p->status, stream);
  return mirec_sample_walk(p->random_list, p->L, p->pr_dev, p->user_keys, n, p->Bc,
                           p->n_batches, p->T, p->used_ptr, p->used_cols, p->used_bits,
                           p->n_bits, p->n_users, p->reject, p->item_keys + p->Bc, KI,
                           p->status, p->walk_ws, p->walk_ws_bytes, stream);
}

extern "C" int mirec_prepare_chunk_group(const mirec_chunk_prep* p, void* stream) {
  if (!prep_ok(p)) return -1;
  const int64_t n = p->n_batches * p->Bc, KI = (1 + p->T) * p->Bc;
  // K36: grouping + records + look-ahead lists in one launch where the shapes allow
  const int g = mirec_chunk_group(p->user_keys, p->item_keys, p->n_batches, p->Bc,
                                  (int32_t)p->T, p->n_users, p->n_items, p->u_perm, p->u_uniq,
                                  p->u_seg, p->u_nu, p->i_perm, p->i_uniq, p->i_seg, p->i_nu,
                                  p->u_rec, p->u_crec, p->i_rec, p->i_crec, p->u_ahead,
                                  p->u_ahead ? p->u_nah : nullptr, p->i_ahead,
                                  p->i_ahead ? p->i_nah : nullptr, stream);
  if (g != 0) return g < 0 ? g : 0;
  // with K35 records the look-ahead lists come from the records launch (one launch
  // after the sort instead of two)
  const bool rec = p->u_rec != nullptr;
  const int rc = mirec::sort_chunk_pair(p->user_keys, n, p->Bc, p->n_users, p->u_perm,
                                        p->u_uniq, p->u_seg, p->u_nu, p->item_keys,
                                        p->n_batches * KI, KI, p->n_items, p->i_perm, p->i_uniq,
                                        p->i_seg, p->i_nu, p->n_batches,
                                        rec ? nullptr : p->u_ahead, p->u_nah,
                                        rec ? nullptr : p->i_ahead, p->i_nah, p->sort_ws,
                                        p->sort_ws_bytes, (hipStream_t)stream);
  if (rc || !rec) return rc;
  return mirec_step_records(p->user_keys, p->item_keys, p->n_batches, p->Bc, (int32_t)p->T,
                            p->n_users, p->n_items, p->u_perm, p->u_uniq, p->u_seg, p->u_nu,
                            p->i_perm, p->i_uniq, p->i_seg, p->i_nu, p->u_rec, p->u_crec,
                            p->i_rec, p->i_crec, p->u_ahead, p->u_ahead ? p->u_nah : nullptr,
                            p->i_ahead, p->i_ahead ? p->i_nah : nullptr, stream);
}

extern "C" int mirec_prepare_chunk(const mirec_chunk_prep* p, void* stream) {
  const int rc = mirec_prepare_chunk_walk(p, stream);
  return rc ? rc : mirec_prepare_chunk_group(p, stream);
}
