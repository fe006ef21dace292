// Depthwise k x k convolution over packed NHWC channels (MobileNet V1/V2;
// SURVEY.md §2.2 B1).  Channel (g, c) of the packed tensor has its own k x k
// filter at w + g*w_gstride + c*k*k (Keras depthwise_kernel, per-config).
// Purely bandwidth-bound, so every kernel moves 8 channels (16 B) per
// thread; the weights for those 8 channels stay in registers.
//
//  fwd   : one thread = 8 channels x 4 consecutive output columns
//  dgrad : one thread = 8 channels x 1 input pixel (gathers the dy taps that
//          reach it; stride 2 handled by divisibility)
//  wgrad : block = 8 channels x 256 row lanes; each lane accumulates the
//          k*k*8 products over its pixels, LDS tree, fp32 atomics into the
//          gradient arena (which the optimizer keeps zeroed)
#include "common.h"

namespace {

constexpr int DW_V = 8;     // channels per thread
constexpr int DW_X = 4;     // output columns per fwd thread

__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void st8(bf16_t* p, const float* v) {
  uint4 u;
  u.x = pack_bf2(v[0], v[1]);
  u.y = pack_bf2(v[2], v[3]);
  u.z = pack_bf2(v[4], v[5]);
  u.w = pack_bf2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

struct DWGeom {
  int B, H, W, C, G, Ho, Wo, k, st, pad;
  int64_t w_gstride;
};

template <int K>
__device__ __forceinline__ void load_w(const bf16_t* w, const DWGeom& d, int gc0,
                                       float (&wr)[K * K][DW_V]) {
  const int g = gc0 / d.C, c0 = gc0 - g * d.C;
  const bf16_t* base = w + g * d.w_gstride + (int64_t)c0 * K * K;
#pragma unroll
  for (int i = 0; i < DW_V; ++i)
#pragma unroll
    for (int t = 0; t < K * K; ++t) wr[t][i] = bf2f(base[i * K * K + t]);
}

template <int K>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w,
                                                     bf16_t* __restrict__ y, DWGeom d) {
  const int GC = d.G * d.C, CV = GC / DW_V;
  const int xgroups = (d.Wo + DW_X - 1) / DW_X;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)d.B * d.Ho * xgroups * CV;
  if (idx >= total) return;
  const int cv = (int)(idx % CV);
  int64_t t = idx / CV;
  const int xg = (int)(t % xgroups);
  t /= xgroups;
  const int ho = (int)(t % d.Ho);
  const int b = (int)(t / d.Ho);
  const int gc0 = cv * DW_V;
  float wr[K * K][DW_V];
  load_w<K>(w, d, gc0, wr);
  for (int xi = 0; xi < DW_X; ++xi) {
    const int wo = xg * DW_X + xi;
    if (wo >= d.Wo) break;
    float acc[DW_V] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int hi = ho * d.st - d.pad + r;
      if (hi < 0 || hi >= d.H) continue;
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int wi = wo * d.st - d.pad + s;
        if (wi < 0 || wi >= d.W) continue;
        float v[DW_V];
        ld8(x + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, v);
#pragma unroll
        for (int i = 0; i < DW_V; ++i) acc[i] += v[i] * wr[r * K + s][i];
      }
    }
    st8(y + (((int64_t)b * d.Ho + ho) * d.Wo + wo) * GC + gc0, acc);
  }
}

template <int K>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ dx, DWGeom d) {
  const int GC = d.G * d.C, CV = GC / DW_V;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)d.B * d.H * d.W * CV;
  if (idx >= total) return;
  const int cv = (int)(idx % CV);
  int64_t t = idx / CV;
  const int wi = (int)(t % d.W);
  t /= d.W;
  const int hi = (int)(t % d.H);
  const int b = (int)(t / d.H);
  const int gc0 = cv * DW_V;
  float wr[K * K][DW_V];
  load_w<K>(w, d, gc0, wr);
  float acc[DW_V] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < K; ++r) {
    const int hn = hi + d.pad - r;
    if (hn < 0 || hn % d.st) continue;
    const int ho = hn / d.st;
    if (ho >= d.Ho) continue;
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const int wn = wi + d.pad - s;
      if (wn < 0 || wn % d.st) continue;
      const int wo = wn / d.st;
      if (wo >= d.Wo) continue;
      float v[DW_V];
      ld8(dy + (((int64_t)b * d.Ho + ho) * d.Wo + wo) * GC + gc0, v);
#pragma unroll
      for (int i = 0; i < DW_V; ++i) acc[i] += v[i] * wr[r * K + s][i];
    }
  }
  st8(dx + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, acc);
}

// grid (GC / 8, row slabs); 256 lanes stride over the slab's output pixels
template <int K>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ dy,
                                                       float* __restrict__ dw,
                                                       int64_t dw_gstride, DWGeom d,
                                                       int64_t pix_per_slab) {
  __shared__ float red[K * K * DW_V][4];
  const int GC = d.G * d.C;
  const int gc0 = blockIdx.x * DW_V;
  constexpr int kk = K * K;
  const int64_t P = (int64_t)d.B * d.Ho * d.Wo;
  const int64_t p0 = (int64_t)blockIdx.y * pix_per_slab;
  const int64_t p1 = min(P, p0 + pix_per_slab);
  float acc[kk][DW_V];
#pragma unroll
  for (int t = 0; t < kk; ++t)
#pragma unroll
    for (int i = 0; i < DW_V; ++i) acc[t][i] = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const int wo = (int)(p % d.Wo);
    const int64_t q = p / d.Wo;
    const int ho = (int)(q % d.Ho);
    const int b = (int)(q / d.Ho);
    float g[DW_V];
    ld8(dy + p * GC + gc0, g);
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int hi = ho * d.st - d.pad + r;
      if (hi < 0 || hi >= d.H) continue;
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int wi = wo * d.st - d.pad + s;
        if (wi < 0 || wi >= d.W) continue;
        float v[DW_V];
        ld8(x + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, v);
#pragma unroll
        for (int i = 0; i < DW_V; ++i) acc[r * K + s][i] += v[i] * g[i];
      }
    }
  }
  // wave reduction, then 4 waves -> LDS -> one atomic per (tap, channel)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < kk; ++t)
#pragma unroll
    for (int i = 0; i < DW_V; ++i) {
      const float v = warp_sum(acc[t][i]);
      if (lane == 0) red[t * DW_V + i][wid] = v;
    }
  __syncthreads();
  for (int e = threadIdx.x; e < kk * DW_V; e += 256) {
    const float v = red[e][0] + red[e][1] + red[e][2] + red[e][3];
    const int t = e / DW_V, i = e - t * DW_V;
    const int gc = gc0 + i, g = gc / d.C, c = gc - g * d.C;
    atomicAdd(dw + g * dw_gstride + (int64_t)c * kk + t, v);
  }
}

DWGeom make_dw(int B, int H, int W, int C, int G, int k, int st, int pad, int64_t ws) {
  DWGeom d;
  d.B = B;
  d.H = H;
  d.W = W;
  d.C = C;
  d.G = G;
  d.k = k;  // dispatch picks the K template
  d.st = st;
  d.pad = pad;
  d.Ho = (H + 2 * pad - k) / st + 1;
  d.Wo = (W + 2 * pad - k) / st + 1;
  d.w_gstride = ws;
  return d;
}

}  // namespace

CER_API int cer_dwconv_fwd(const bf16_t* x, int B, int H, int W, int C, int G, const bf16_t* w,
                           int64_t w_gstride, int k, int st, int pad, bf16_t* y,
                           hipStream_t stream) {
  if (C % DW_V || (k != 3 && k != 5)) return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, k, st, pad, w_gstride);
  const int64_t n = (int64_t)B * d.Ho * ((d.Wo + DW_X - 1) / DW_X) * (G * C / DW_V);
  if (k == 3)
    dw_fwd_kernel<3><<<cer_blocks(n, 256), 256, 0, stream>>>(x, w, y, d);
  else
    dw_fwd_kernel<5><<<cer_blocks(n, 256), 256, 0, stream>>>(x, w, y, d);
  return (int)hipGetLastError();
}

// dw must be zero on entry (accumulated with atomics); dx may be null
CER_API int cer_dwconv_bwd(const bf16_t* dy, const bf16_t* x, int B, int H, int W, int C, int G,
                           const bf16_t* w, int64_t w_gstride, float* dw, int64_t dw_gstride,
                           int k, int st, int pad, bf16_t* dx, hipStream_t stream) {
  if (C % DW_V || (k != 3 && k != 5)) return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, k, st, pad, w_gstride);
  if (dx) {
    const int64_t n = (int64_t)B * H * W * (G * C / DW_V);
    if (k == 3)
      dw_dgrad_kernel<3><<<cer_blocks(n, 256), 256, 0, stream>>>(dy, w, dx, d);
    else
      dw_dgrad_kernel<5><<<cer_blocks(n, 256), 256, 0, stream>>>(dy, w, dx, d);
  }
  const int64_t P = (int64_t)B * d.Ho * d.Wo;
  const int cblocks = G * C / DW_V;
  int64_t slabs = (2048 + cblocks - 1) / cblocks;
  int64_t per = (P + slabs - 1) / slabs;
  if (per < 256) per = 256;
  slabs = (P + per - 1) / per;
  dim3 grid(cblocks, (unsigned)slabs);
  if (k == 3)
    dw_wgrad_kernel<3><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, per);
  else
    dw_wgrad_kernel<5><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, per);
  return (int)hipGetLastError();
}
