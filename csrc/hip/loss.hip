// Fused softmax cross-entropy + top-1/top-5 + gradient, G packed configs
// (SURVEY.md K11, K12).
//
// One 256-thread block per (sample b, config g) row of N logits.  A single
// pass over the row (kept in registers) gives max, log-sum-exp, the label's
// rank (-> top-1/top-5 hit, ties broken by index like a stable top-k),
// the per-config mean loss, the metric accumulators (atomics into acc[g][4] =
// {loss_sum, top1, top5, count}) and, when requested, dlogits =
// (softmax - onehot) / B written in the compute dtype for the backward pass.
#include "common.h"

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }

constexpr int CE_THREADS = 256;
constexpr int CE_MAXPER = 8;  // N <= 2048

template <typename T, typename TD>
__global__ __launch_bounds__(CE_THREADS) void softmax_ce_kernel(
    const T* __restrict__ logits, const int* __restrict__ labels, float* __restrict__ acc,
    float* __restrict__ loss_out, TD* __restrict__ dlogits, int B, int G, int N,
    float* __restrict__ dbias = nullptr, int64_t dbias_stride = 0) {
  __shared__ float smem[16];
  const int b = blockIdx.x, g = blockIdx.y;
  const int64_t base = (int64_t)b * G * N + (int64_t)g * N;
  const int lab = labels[g * B + b];
  float z[CE_MAXPER];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < CE_MAXPER; ++k) {
    int j = threadIdx.x + k * CE_THREADS;
    z[k] = (j < N) ? ld<T>(logits, base + j) : -INFINITY;
    mx = fmaxf(mx, z[k]);
  }
  mx = block_max(mx, smem);
  float zl = ld<T>(logits, base + lab);
  float se = 0.f, cnt = 0.f;
#pragma unroll
  for (int k = 0; k < CE_MAXPER; ++k) {
    int j = threadIdx.x + k * CE_THREADS;
    if (j < N) {
      se += __expf(z[k] - mx);
      cnt += (z[k] > zl || (z[k] == zl && j < lab)) ? 1.f : 0.f;
    }
  }
  se = block_sum(se, smem);
  cnt = block_sum(cnt, smem);
  const float lse = mx + __logf(se);
  if (dlogits) {
    const float inv_b = 1.f / (float)B, inv_se = 1.f / se;
#pragma unroll
    for (int k = 0; k < CE_MAXPER; ++k) {
      int j = threadIdx.x + k * CE_THREADS;
      if (j < N) {
        float p = __expf(z[k] - mx) * inv_se;
        const float d = (p - (j == lab ? 1.f : 0.f)) * inv_b;
        st1(dlogits + base + j, d);
        // the head linear's bias gradient (sum over the batch of dlogits),
        // accumulated into the zeroed gradient arena (cer_softmax_ce_f32_head)
        if (dbias) atomicAdd(dbias + (int64_t)g * dbias_stride + j, d);
      }
    }
  }
  if (threadIdx.x == 0) {
    const float nll = lse - zl;
    atomicAdd(&acc[g * 4 + 0], nll);
    atomicAdd(&acc[g * 4 + 1], cnt < 1.f ? 1.f : 0.f);
    atomicAdd(&acc[g * 4 + 2], (N > 2) ? (cnt < 5.f ? 1.f : 0.f) : 1.f);
    atomicAdd(&acc[g * 4 + 3], 1.f);
    if (loss_out) atomicAdd(&loss_out[g], nll / (float)B);
  }
}

CER_API int cer_softmax_ce(const void* logits, int logits_bf16, const int* labels, float* acc,
                           float* loss_out, bf16_t* dlogits, int B, int G, int N,
                           hipStream_t stream) {
  if (N > CE_THREADS * CE_MAXPER) return (int)hipErrorInvalidValue;
  if (loss_out) cer_zero_async(loss_out, sizeof(float) * G, stream);
  dim3 grid(B, G);
  if (logits_bf16)
    softmax_ce_kernel<bf16_t, bf16_t><<<grid, CE_THREADS, 0, stream>>>(
        (const bf16_t*)logits, labels, acc, loss_out, dlogits, B, G, N);
  else
    softmax_ce_kernel<float, bf16_t><<<grid, CE_THREADS, 0, stream>>>(
        (const float*)logits, labels, acc, loss_out, dlogits, B, G, N);
  return (int)hipGetLastError();
}

// reference-precision mode: fp32 logits in, fp32 dlogits out
CER_API int cer_softmax_ce_f32(const float* logits, const int* labels, float* acc,
                               float* loss_out, float* dlogits, int B, int G, int N,
                               hipStream_t stream) {
  if (N > CE_THREADS * CE_MAXPER) return (int)hipErrorInvalidValue;
  if (loss_out) cer_zero_async(loss_out, sizeof(float) * G, stream);
  softmax_ce_kernel<float, float><<<dim3(B, G), CE_THREADS, 0, stream>>>(logits, labels, acc,
                                                                          loss_out, dlogits, B, G,
                                                                          N);
  return (int)hipGetLastError();
}

// training step form: no per-config loss output (the engine reads the
// metric accumulators; the backward seeds a unit gradient), and the bias
// gradient of the head linear that produced the logits (an act-free Dense:
// d bias = sum_b dlogits) added into ``dbias`` (config stride dbias_stride,
// zeroed: the optimizer clears the gradient it consumes), so the linear's
// backward needs no bias pass
CER_API int cer_softmax_ce_f32_head(const float* logits, const int* labels, float* acc,
                                    float* dlogits, float* dbias, int64_t dbias_stride, int B,
                                    int G, int N, hipStream_t stream) {
  if (N > CE_THREADS * CE_MAXPER) return (int)hipErrorInvalidValue;
  softmax_ce_kernel<float, float><<<dim3(B, G), CE_THREADS, 0, stream>>>(
      logits, labels, acc, nullptr, dlogits, B, G, N, dbias, dbias_stride);
  return (int)hipGetLastError();
}
