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

// + the group's data cursor (the next step's batch, runtime/group.py), so the
// step's tail is one small launch instead of two
__global__ void adam_inc_step(float* state, int64_t row_stride, int64_t off_step, int G,
                              int* cursor) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < G) state[g * row_stride + off_step] += 1.0f;
  if (cursor && g == 0) cursor[0] += 1;
}

// Side jobs of the NEXT optimizer launch (cer_adam_set_aux; cleared by it):
// the data cursor to advance, and a buffer to zero -- the BN statistics
// arena of the step (ops/_hip.py _StatsArena), zeroed here at the end of a
// step for the next one instead of by a fill kernel at its start.
static int* g_aux_cursor = nullptr;
static float* g_aux_zero = nullptr;
static int64_t g_aux_zero_n = 0;
CER_API void cer_adam_set_aux(int* cursor, float* zero, int64_t zero_n) {
  g_aux_cursor = cursor;
  g_aux_zero = zero;
  g_aux_zero_n = zero ? zero_n : 0;
}

// HL image of the params (fp32 mode; runtime/arena.py Arena.whl) the NEXT
// optimizer launch writes next to them: every 8 updated params as [8 x bf16
// hi | 8 x bf16 lo] (common.h st8_hl), the operand format the fp32 conv
// kernels read without splitting (conv.hip cer_conv_set_whl).  Cleared by
// that launch.
static float* g_hl_img = nullptr;
static int64_t g_hl_stride = 0;
CER_API void cer_adam_set_hl(float* img, int64_t stride) {
  g_hl_img = img;
  g_hl_stride = img ? stride : 0;
}

// the HL image of rows of an fp32 tensor: dst[g][i..] = HL(src[g][i..]),
// n % 8 == 0 (Arena.sync_work after host / hop writes of the params)
__global__ __launch_bounds__(256) void hl_image_kernel(const float* __restrict__ src,
                                                       int64_t src_stride, float* __restrict__ dst,
                                                       int64_t dst_stride, int64_t n) {
  const int g = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  float v[8];
  ld8(src + g * src_stride + i, v);
  st8_hl(dst + g * dst_stride + i, v);
}

CER_API int cer_hl_image(const float* src, int64_t src_stride, float* dst, int64_t dst_stride,
                         int64_t n, int G, hipStream_t stream) {
  if (n % 8 != 0 || G <= 0) return (int)hipErrorInvalidValue;
  dim3 grid(cer_blocks(n / 8, 256), G);
  hl_image_kernel<<<grid, 256, 0, stream>>>(src, src_stride, dst, dst_stride, n);
  return (int)hipGetLastError();
}

// grid-stride share of blocks (x, 0) in zeroing n floats (n % 4 == 0)
__device__ __forceinline__ void aux_zero(float* z, int64_t n) {
  if (!z || blockIdx.y != 0) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; k < n; k += stride)
    *reinterpret_cast<float4*>(z + k) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// WRITE_BF16: also write the bf16 compute shadow of the params (bf16 mode);
// fp32 compute reads the params themselves
template <bool WRITE_BF16>
__global__ __launch_bounds__(256) void adam_kernel(
    float* __restrict__ state, int64_t row_stride, int64_t n_train, int64_t off_m,
    int64_t off_v, int64_t off_step, float* __restrict__ grad, int64_t grad_stride, int zero_grad,
    bf16_t* __restrict__ work, int64_t work_stride, const float* __restrict__ lr,
    const float* __restrict__ wd, float b1, float b2, float eps, int l2, float* zero,
    int64_t zero_n, float* __restrict__ hl, int64_t hl_stride) {
  aux_zero(zero, zero_n);
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
  float4 p[2] = {pp[0], pp[1]}, m[2] = {mp[0], mp[1]}, v[2] = {vp[0], vp[1]};
  const float4 gr[2] = {gp[0], gp[1]};
  if (zero_grad) {
    gp[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    gp[1] = make_float4(0.f, 0.f, 0.f, 0.f);
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
  pp[0] = p[0]; pp[1] = p[1];
  mp[0] = m[0]; mp[1] = m[1];
  vp[0] = v[0]; vp[1] = v[1];
  if (hl) st8_hl(hl + g * hl_stride + i, pf);
  if (WRITE_BF16) {
    uint4 o;
    o.x = pack_bf2(pf[0], pf[1]);
    o.y = pack_bf2(pf[2], pf[3]);
    o.z = pack_bf2(pf[4], pf[5]);
    o.w = pack_bf2(pf[6], pf[7]);
    *reinterpret_cast<uint4*>(work + g * work_stride + i) = o;
  }
}

CER_API int cer_adam_step(float* state, int64_t row_stride, int64_t n_train, int64_t off_m,
                          int64_t off_v, int64_t off_step, float* grad, int64_t grad_stride,
                          int zero_grad, bf16_t* work, int64_t work_stride, const float* lr,
                          const float* wd, int G, float b1, float b2, float eps, int l2,
                          hipStream_t stream) {
  if (n_train % 8 != 0 || g_aux_zero_n % 4 != 0) {
    cer_adam_set_aux(nullptr, nullptr, 0);   // a refused launch consumes its side jobs too
    cer_adam_set_hl(nullptr, 0);
    return (int)hipErrorInvalidValue;
  }
  adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G,
                                                      g_aux_cursor);
  dim3 grid(cer_blocks(n_train / 8, 256), G);
  if (work)
    adam_kernel<true><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_v,
                                                 off_step, grad, grad_stride, zero_grad, work,
                                                 work_stride, lr, wd, b1, b2, eps, l2, g_aux_zero,
                                                 g_aux_zero_n, g_hl_img, g_hl_stride);
  else
    adam_kernel<false><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_v,
                                                  off_step, grad, grad_stride, zero_grad, nullptr,
                                                  0, lr, wd, b1, b2, eps, l2, g_aux_zero,
                                                  g_aux_zero_n, g_hl_img, g_hl_stride);
  cer_adam_set_aux(nullptr, nullptr, 0);
  cer_adam_set_hl(nullptr, 0);
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
    const float* __restrict__ wd, float mu, int l2, float* zero, int64_t zero_n,
    float* __restrict__ hl, int64_t hl_stride) {
  aux_zero(zero, zero_n);
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
  if (hl) st8_hl(hl + g * hl_stride + i, pf);
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
  if (n_train % 8 != 0 || g_aux_zero_n % 4 != 0) {
    cer_adam_set_aux(nullptr, nullptr, 0);
    cer_adam_set_hl(nullptr, 0);
    return (int)hipErrorInvalidValue;
  }
  adam_inc_step<<<cer_blocks(G, 64), 64, 0, stream>>>(state, row_stride, off_step, G,
                                                      g_aux_cursor);
  dim3 grid(cer_blocks(n_train / 8, 256), G);
  if (work)
    sgd_kernel<true><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_step, grad,
                                               grad_stride, zero_grad, work, work_stride, lr, wd,
                                               momentum, l2, g_aux_zero, g_aux_zero_n, g_hl_img,
                                               g_hl_stride);
  else
    sgd_kernel<false><<<grid, 256, 0, stream>>>(state, row_stride, n_train, off_m, off_step,
                                                grad, grad_stride, zero_grad, nullptr, 0, lr, wd,
                                                momentum, l2, g_aux_zero, g_aux_zero_n, g_hl_img,
                                                g_hl_stride);
  cer_adam_set_aux(nullptr, nullptr, 0);
  cer_adam_set_hl(nullptr, 0);
  return (int)hipGetLastError();
}
