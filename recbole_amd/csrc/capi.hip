// Error state, version and the small reduction kernels of the trainer loop.
#include <stdarg.h>
#include "common.h"
#include <algorithm>

namespace mirec {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Fixed-order sum: 1024 threads, thread t sums x[t], x[t+1024], ... in order,
// then a fixed binary tree over the 1024 partials. Independent of timing.
__device__ __forceinline__ float block_fixed_sum(const float* __restrict__ x, int64_t n,
                                                 float* lds /*1024*/) {
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) acc += x[i];
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) lds[threadIdx.x] += lds[threadIdx.x + s];
    __syncthreads();
  }
  return lds[0];
}

__global__ __launch_bounds__(1024) void sum_kernel(const float* __restrict__ x, int64_t n,
                                                   float* __restrict__ out) {
  __shared__ float lds[1024];
  float s = block_fixed_sum(x, n, lds);
  if (threadIdx.x == 0) out[0] = s;
}

__global__ __launch_bounds__(1024) void step_finish_kernel(const float* __restrict__ loss_k,
                                                           int64_t n, float denom,
                                                           float* __restrict__ loss_hist,
                                                           int32_t* __restrict__ step_idx) {
  __shared__ float lds[1024];
  float s = block_fixed_sum(loss_k, n, lds);
  if (threadIdx.x == 0) {
    int32_t st = step_idx[0];
    if (loss_hist) loss_hist[st] = s / denom;
    step_idx[0] = st + 1;
  }
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_abi_version(void) { return MIREC_ABI_VERSION; }
extern "C" const char* mirec_last_error(void) { return mirec::g_err; }

extern "C" int mirec_sum_f32(const float* x, int64_t n, float* out, void* stream) {
  if (!out || n < 0 || (n > 0 && !x)) { set_error("mirec_sum_f32: bad arguments"); return -1; }
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, n, out);
  return launch_status("mirec_sum_f32");
}

extern "C" int mirec_step_finish(const float* loss_k, int64_t n, float denom, float* loss_hist,
                                 int32_t* step_idx_dev, void* stream) {
  if (!step_idx_dev || n < 0 || (n > 0 && !loss_k)) {
    set_error("mirec_step_finish: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(step_finish_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, loss_k, n,
                     denom, loss_hist, step_idx_dev);
  return launch_status("mirec_step_finish");
}

// Per-chunk version: n_steps losses at loss_k[c*stride .. +n), each reduced in
// exactly step_finish's order, written to loss_hist[step_base + c]; then
// step_base += n_steps. One workgroup per step (the reductions run side by
// side); the workgroup that takes the last ticket — every workgroup has read
// step_base before taking one — advances the counter and resets the ticket.
__global__ __launch_bounds__(1024) void chunk_finish_kernel(const float* __restrict__ loss_k,
                                                            int64_t n, int64_t stride,
                                                            int32_t n_steps, float denom,
                                                            float* __restrict__ loss_hist,
                                                            int32_t* __restrict__ step_base,
                                                            int32_t* __restrict__ ticket) {
  __shared__ float lds[1024];
  const int c = blockIdx.x;
  float s = block_fixed_sum(loss_k + (int64_t)c * stride, n, lds);
  if (threadIdx.x == 0) {
    const int32_t st = __hip_atomic_load(step_base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (loss_hist) loss_hist[st + c] = s / denom;
    const int32_t t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == n_steps - 1) {
      __hip_atomic_store(step_base, st + n_steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

extern "C" int mirec_chunk_finish(const float* loss_k, int64_t n, int64_t stride,
                                  int32_t n_steps, float denom, float* loss_hist,
                                  int32_t* step_base_dev, int32_t* ticket_dev, void* stream) {
  if (!step_base_dev || !ticket_dev || n < 0 || n_steps < 0 || stride < n ||
      (n > 0 && n_steps > 0 && !loss_k)) {
    set_error("mirec_chunk_finish: bad arguments");
    return -1;
  }
  if (n_steps == 0) return 0;
  hipLaunchKernelGGL(chunk_finish_kernel, dim3(n_steps), dim3(1024), 0, (hipStream_t)stream,
                     loss_k, n, stride, n_steps, denom, loss_hist, step_base_dev, ticket_dev);
  return launch_status("mirec_chunk_finish");
}


// ---- small host -> device writes that a graph capture records by value
namespace mirec {
constexpr int kPayloadWords = 992;     // 3,968 B of kernel arguments per launch (< 4 KiB)
struct Payload { uint32_t w[kPayloadWords]; };

__global__ __launch_bounds__(256) void write_bytes_kernel(uint32_t* __restrict__ dst, Payload p,
                                                          int n_words) {
  for (int i = threadIdx.x; i < n_words; i += blockDim.x) dst[i] = p.w[i];
}
}  // namespace mirec

// Many device-to-device copies in one launch (the per-step copy of a batch's columns
// into a captured graph's static inputs): up to kCopyDescs (src, dst, bytes) per
// launch, passed by value; block b copies slice b % per of copy b / per ... with
// 16-B vectors when src, dst and the size allow, bytes otherwise.
constexpr int kCopyDescs = 96;
struct CopyDescs {
  const char* src[kCopyDescs];
  char* dst[kCopyDescs];
  int64_t bytes[kCopyDescs];
};

__global__ __launch_bounds__(256) void copy_many_kernel(CopyDescs d, int n, int blocks_per) {
  const int c = blockIdx.x / blocks_per;
  if (c >= n) return;
  const int64_t nb = d.bytes[c];
  const char* __restrict__ src = d.src[c];
  char* __restrict__ dst = d.dst[c];
  const int64_t t0 = (int64_t)(blockIdx.x % blocks_per) * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)blocks_per * blockDim.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t nv = nb / 16;
    const int4* __restrict__ s4 = reinterpret_cast<const int4*>(src);
    int4* __restrict__ d4 = reinterpret_cast<int4*>(dst);
    for (int64_t i = t0; i < nv; i += stride) d4[i] = s4[i];
    for (int64_t i = nv * 16 + t0; i < nb; i += stride) dst[i] = src[i];
  } else {
    for (int64_t i = t0; i < nb; i += stride) dst[i] = src[i];
  }
}

extern "C" int mirec_copy_many(const void* const* src, void* const* dst, const int64_t* bytes,
                               int n, void* stream) {
  if (n < 0 || (n > 0 && (!src || !dst || !bytes))) {
    set_error("mirec_copy_many: bad arguments");
    return -1;
  }
  for (int off = 0; off < n; off += kCopyDescs) {
    const int m = std::min(kCopyDescs, n - off);
    CopyDescs d;
    int64_t mx = 0;
    for (int i = 0; i < m; ++i) {
      if (bytes[off + i] < 0 || (bytes[off + i] && (!src[off + i] || !dst[off + i]))) {
        set_error("mirec_copy_many: bad descriptor %d", off + i);
        return -1;
      }
      d.src[i] = (const char*)src[off + i];
      d.dst[i] = (char*)dst[off + i];
      d.bytes[i] = bytes[off + i];
      mx = std::max(mx, bytes[off + i]);
    }
    // blocks per copy: enough 16-B lanes for the largest copy, at most 64
    const int per = (int)std::max<int64_t>(1, std::min<int64_t>(64, (mx / 16 + 255) / 256));
    hipLaunchKernelGGL(copy_many_kernel, dim3((unsigned)(m * per)), dim3(256), 0,
                       (hipStream_t)stream, d, m, per);
  }
  return launch_status("mirec_copy_many");
}

extern "C" int mirec_write_bytes(void* dst_dev, const void* src_host, size_t n_bytes,
                                 void* stream) {
  if ((n_bytes && (!dst_dev || !src_host)) || (n_bytes & 3) || ((uintptr_t)dst_dev & 3)) {
    set_error("mirec_write_bytes: bad arguments (n_bytes %zu)", n_bytes);
    return -1;
  }
  const uint32_t* src = (const uint32_t*)src_host;
  uint32_t* dst = (uint32_t*)dst_dev;
  for (size_t off = 0; off < n_bytes / 4; off += kPayloadWords) {
    const int n = (int)std::min<size_t>(kPayloadWords, n_bytes / 4 - off);
    Payload p;
    memcpy(p.w, src + off, (size_t)n * 4);
    hipLaunchKernelGGL(write_bytes_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, dst + off,
                       p, n);
  }
  return launch_status("mirec_write_bytes");
}
