// Fused multi-configuration Adam over the flat arena.
//
// One launch updates all G configs: grid.y = config row, each thread owns 8
// consecutive parameters (two 16-B loads per operand).  Per-row lr / lambda
// and the step counter live on device, so the update is HIP-graph
// capturable.  Semantics = torch.optim.Adam(lr, weight_decay=lambda):
//   g += wd * p;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// and the bf16 compute shadow of p is written in the same pass.
// Bytes/param: read p,m,v,g (16) + write p,m,v (12) + bf16 shadow (2).
// zero_grad: the consumed gradient is cleared in the same pass (+4 B), so the
// next backward's split-K weight-gradient kernels can accumulate into it
// without a memset per layer.
#include "common.h"

#include <stdlib.h>

// streamed-once operands: non-temporal loads / stores (NT) keep them from
// evicting the L2 / MALL lines the next forward reads (CER_ADAM_NT)
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
  if (NT) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(float4* p, float4 v) {
  if (NT) {
    const f4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
  } else {
    *p = v;
  }
}

__global__ void adam_inc_step(float* state, int64_t row_stride, int64_t off_step, int G) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < G) state[g * row_stride + off_step] += 1.0f;
}

// 8 fp32 -> the split image chunk [8 x bf16 hi | 8 x bf16 lo] (conv.hip
// cer_conv_set_wsplit): hi = bf16(v), lo = bf16(v - hi)
__device__ __forceinline__ void store_split8(uint32_t* dst, const float* v) {
  uint4 h, l;
  uint32_t* hw = reinterpret_cast<uint32_t*>(&h);
  uint32_t* lw = reinterpret_cast<uint32_t*>(&l);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t hp = pack_bf2(v[2 * k], v[2 * k + 1]);
    hw[k] = hp;
    lw[k] = pack_bf2(v[2 * k] - __uint_as_float(hp << 16),
                     v[2 * k + 1] - __uint_as_float(hp & 0xffff0000u));
  }
  reinterpret_cast<uint4*>(dst)[0] = h;
  reinterpret_cast<uint4*>(dst)[1] = l;
}

// work modes: 0 none (fp32 compute reads the params), 1 bf16 shadow,
// 2 split image of the params (fp32 compute with pre-split weights)
template <bool WRITE_BF16, bool NT = false, bool SPLIT = false>
__global__ __launch_bounds__(256) void adam_kernel(
    float* __restrict__ state, int64_t row_stride, int64_t n_train, int64_t off_m,
    int64_t off_v, int64_t off_step, float* __restrict__ grad, int64_t grad_stride, int zero_grad,
    bf16_t* __restrict__ work, int64_t work_stride, const float* __restrict__ lr,
    const float* __restrict__ wd, float b1, float b2, float eps, int l2) {
  const int g = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n_train) return;
  float* row = state + g * row_stride;
  const float t = row[off_step];
  const float bc1 = 1.f - __powf(b1, t);
  const float bc2 = 1.f - __powf(b2, t);
  const float step_size = lr[g] / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  const float lam = l2 ? wd[g] : 0.f;

  float4* pp = reinterpret_cast<float4*>(row + i);
  float4* mp = reinterpret_cast<float4*>(row + off_m + i);
  float4* vp = reinterpret_cast<float4*>(row + off_v + i);
  float4* gp = reinterpret_cast<float4*>(grad + g * grad_stride + i);
  float4 p[2] = {ld4<NT>(pp), ld4<NT>(pp + 1)}, m[2] = {ld4<NT>(mp), ld4<NT>(mp + 1)},
         v[2] = {ld4<NT>(vp), ld4<NT>(vp + 1)};
  const float4 gr[2] = {ld4<NT>(gp), ld4<NT>(gp + 1)};
  if (zero_grad) {
    st4<NT>(gp, make_float4(0.f, 0.f, 0.f, 0.f));
    st4<NT>(gp + 1, make_float4(0.f, 0.f, 0.f, 0.f));
  }
  float* pf = reinterpret_cast<float*>(p);
  float* mf = reinterpret_cast<float*>(m);
  float* vf = reinterpret_cast<float*>(v);
  const float* gf = reinterpret_cast<const float*>(gr);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float gk = gf[k] + lam * pf[k];
    mf[k] = b1 * mf[k] + (1.f - b1) * gk;
    vf[k] = b2 * vf[k] + (1.f - b2) * gk * gk;
    float denom = sqrtf(vf[k]) * inv_sqrt_bc2 + eps;
    pf[k] -= step_size * mf[k] / denom;
  }
  st4<NT>(pp, p[0]); st4<NT>(pp + 1, p[1]);
  st4<NT>(mp, m[0]); st4<NT>(mp + 1, m[1]);
  st4<NT>(vp, v[0]); st4<NT>(vp + 1, v[1]);
  if (SPLIT) {
    store_split8(reinterpret_cast<uint32_t*>(work) + g * work_stride + i, pf);
  } else if (WRITE_BF16) {
    uint4 o;
    o.x = pack_bf2(pf[0], pf[1]);
    o.y = pack_bf2(pf[2], pf[3]);
    o.z = pack_bf2(pf[4], pf[5]);
    o.w = pack_bf2(pf[6], pf[7]);
    *reinterpret_cast<uint4*>(work + g * work_stride + i) = o;
  }
}

// Adam that also writes the split image of the updated params: ``split`` =
// [G][n_train] 32-bit slots, ``split_stride`` in slots
CER_API int cer_adam_step_split(float* state, int64_t row_stride, int64_t n_train, int64_t off_m,
                                int64_t off_v, int64_t off_step, float* grad,
                                int64_t grad_stride, int zero_grad, void* split,
                                int64_t split_stride, const float* lr, const float* wd, int G,
                                float b1, float b2, float eps, int l2, hipStream_t stream) {
  if (n_train % 8 != 0) return (int)hipErrorInvalidValue;
  adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G);
  dim3 grid(cer_blocks(n_train / 8, 256), G);
  adam_kernel<false, false, true><<<grid, 256, 0, stream>>>(
      state, row_stride, n_train, off_m, off_v, off_step, grad, grad_stride, zero_grad,
      reinterpret_cast<bf16_t*>(split), split_stride, lr, wd, b1, b2, eps, l2);
  return (int)hipGetLastError();
}

// split image of fp32 params (after init / load / hop): [G][n] -> [G][n] slots
__global__ void split_image_kernel(const float* __restrict__ src, int64_t src_stride,
                                   uint32_t* __restrict__ dst, int64_t dst_stride, int64_t n) {
  const int g = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  float v[8];
  const float4* sp = reinterpret_cast<const float4*>(src + g * src_stride + i);
  const float4 a = sp[0], b = sp[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  store_split8(dst + g * dst_stride + i, v);
}

CER_API int cer_split_image(const float* src, int64_t src_stride, void* dst, int64_t dst_stride,
                            int64_t n, int G, hipStream_t stream) {
  if (n % 8 != 0) return (int)hipErrorInvalidValue;
  dim3 grid(cer_blocks(n / 8, 256), G);
  split_image_kernel<<<grid, 256, 0, stream>>>(src, src_stride,
                                               reinterpret_cast<uint32_t*>(dst), dst_stride, n);
  return (int)hipGetLastError();
}

CER_API int cer_adam_step(float* state, int64_t row_stride, int64_t n_train, int64_t off_m,
                          int64_t off_v, int64_t off_step, float* grad, int64_t grad_stride,
                          int zero_grad, bf16_t* work, int64_t work_stride, const float* lr,
                          const float* wd, int G, float b1, float b2, float eps, int l2,
                          hipStream_t stream) {
  if (n_train % 8 != 0) return (int)hipErrorInvalidValue;
  adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G);
  dim3 grid(cer_blocks(n_train / 8, 256), G);
  static int nt = -1;
  if (nt < 0) {
    const char* e = getenv("CER_ADAM_NT");
    nt = (e && e[0] == '1') ? 1 : 0;
  }
  if (work && nt)
    adam_kernel<true, true><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_v,
                                                       off_step, grad, grad_stride, zero_grad,
                                                       work, work_stride, lr, wd, b1, b2, eps,
                                                       l2);
  else if (work)
    adam_kernel<true><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_v,
                                                 off_step, grad, grad_stride, zero_grad, work,
                                                 work_stride,
                                                 lr, wd, b1, b2, eps, l2);
  else
    adam_kernel<false><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_v,
                                                  off_step, grad, grad_stride, zero_grad, nullptr,
                                                  0, lr,
                                                  wd, b1, b2, eps, l2);
  return (int)hipGetLastError();
}

// Adam over the parameter range [lo, hi) of every row (an update split
// across streams: the range whose gradients are final early runs on a side
// stream while backward finishes the rest).  inc_step: also advance the step
// counters (exactly once per step, before any range reads them); fp32
// compute only (no shadow / split image).
CER_API int cer_adam_step_range(float* state, int64_t row_stride, int64_t lo, int64_t hi,
                                int64_t off_m, int64_t off_v, int64_t off_step, float* grad,
                                int64_t grad_stride, int zero_grad, const float* lr,
                                const float* wd, int G, float b1, float b2, float eps, int l2,
                                int inc_step, hipStream_t stream) {
  if (lo % 8 || hi % 8 || hi < lo) return (int)hipErrorInvalidValue;
  if (inc_step)
    adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G);
  if (hi == lo) return (int)hipGetLastError();
  dim3 grid(cer_blocks((hi - lo) / 8, 256), G);
  adam_kernel<false><<<grid, 256, 0, stream>>>(state + lo, row_stride, hi - lo, off_m, off_v,
                                                off_step - lo, grad + lo, grad_stride, zero_grad,
                                                nullptr, 0, lr, wd, b1, b2, eps, l2);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// SGD with momentum, torch.optim.SGD semantics (dampening 0, no Nesterov):
//   g += wd * p;  buf = mu * buf + g;  p -= lr * buf
// (buf = the arena's first-moment slot; first step buf = g as in torch).
// ---------------------------------------------------------------------------
template <bool WRITE_BF16>
__global__ __launch_bounds__(256) void sgd_kernel(
    float* __restrict__ state, int64_t row_stride, int64_t n_train, int64_t off_m,
    int64_t off_step, float* __restrict__ grad, int64_t grad_stride, int zero_grad,
    bf16_t* __restrict__ work, int64_t work_stride, const float* __restrict__ lr,
    const float* __restrict__ wd, float mu, int l2) {
  const int g = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n_train) return;
  float* row = state + g * row_stride;
  const bool first = row[off_step] <= 1.0f;
  const float rate = lr[g];
  const float lam = l2 ? wd[g] : 0.f;
  float4* pp = reinterpret_cast<float4*>(row + i);
  float4* mp = reinterpret_cast<float4*>(row + off_m + i);
  float4* gp = reinterpret_cast<float4*>(grad + g * grad_stride + i);
  float4 p[2] = {pp[0], pp[1]}, m[2] = {mp[0], mp[1]};
  const float4 gr[2] = {gp[0], gp[1]};
  if (zero_grad) {
    gp[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    gp[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float* pf = reinterpret_cast<float*>(p);
  float* mf = reinterpret_cast<float*>(m);
  const float* gf = reinterpret_cast<const float*>(gr);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float gk = gf[k] + lam * pf[k];
    mf[k] = (mu == 0.f) ? gk : (first ? gk : mu * mf[k] + gk);
    pf[k] -= rate * mf[k];
  }
  pp[0] = p[0]; pp[1] = p[1];
  mp[0] = m[0]; mp[1] = m[1];
  if (WRITE_BF16) {
    uint4 o;
    o.x = pack_bf2(pf[0], pf[1]);
    o.y = pack_bf2(pf[2], pf[3]);
    o.z = pack_bf2(pf[4], pf[5]);
    o.w = pack_bf2(pf[6], pf[7]);
    *reinterpret_cast<uint4*>(work + g * work_stride + i) = o;
  }
}

CER_API int cer_sgd_step(float* state, int64_t row_stride, int64_t n_train, int64_t off_m,
                         int64_t off_step, float* grad, int64_t grad_stride, int zero_grad,
                         bf16_t* work, int64_t work_stride, const float* lr, const float* wd,
                         int G, float momentum, int l2, hipStream_t stream) {
  if (n_train % 8 != 0) return (int)hipErrorInvalidValue;
  adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G);
  dim3 grid(cer_blocks(n_train / 8, 256), G);
  if (work)
    sgd_kernel<true><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_step, grad,
                                               grad_stride, zero_grad, work, work_stride, lr, wd,
                                               momentum, l2);
  else
    sgd_kernel<false><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_step,
                                                grad, grad_stride, zero_grad, nullptr, 0, lr, wd,
                                                momentum, l2);
  return (int)hipGetLastError();
}
