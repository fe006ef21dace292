// Depthwise k x k convolution over packed NHWC channels (MobileNet V1/V2,
// NASNet-Mobile separable convs).  Channel (g, c) of the
// packed tensor has its own k x k filter at w + g*w_gstride + c*k*k (Keras
// depthwise_kernel, per-config).  k in {3, 5, 7}, stride 1 or 2; padding may
// be asymmetric (Keras stride-2 "correct_pad": top/left = k/2 - 1 on even
// inputs): the caller passes the top/left pad and the output size, and the
// bottom/right pad is implied by the bounds checks.
//
// Bandwidth-bound, so every kernel moves 8 channels (16 B) per thread (1 for
// channel counts that are not multiples of 8); only
// one filter row (k x 8 fp32) is register-resident at a time, so k = 7 does
// not spill.
//
//  fwd   : one thread = 8 channels x 4 consecutive output columns; per filter
//          row the (4-1)*stride + k input pixels are loaded once (sliding
//          window) instead of 4k times
//  dgrad : one thread = 8 channels x 1 input pixel (gathers the dy taps that
//          reach it; stride 2 handled by divisibility)
//  wgrad : block = 8 channels x 256 row lanes x a band of filter rows; each
//          lane accumulates the band's taps over its pixels, wave reduction,
//          LDS across waves, fp32 atomics into the gradient arena (which the
//          optimizer keeps zeroed)
#include "common.h"

namespace {

constexpr int DW_V = 8;     // channels per thread
constexpr int DW_X = 4;     // output columns per fwd thread

struct DWGeom {
  int B, H, W, C, G, Ho, Wo, pt, pl;
  int64_t w_gstride;
};

// filter row r of the V channels starting at packed channel gc0 (V = 8: one
// config holds all 8, as C % 8 == 0)
template <int K, int V, typename T>
__device__ __forceinline__ void load_wrow(const T* w, const DWGeom& d, int gc0, int r,
                                          float (&wr)[K][V]) {
  const int g = gc0 / d.C, c0 = gc0 - g * d.C;
  const T* base = w + g * d.w_gstride + (int64_t)c0 * K * K + r * K;
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int s = 0; s < K; ++s) wr[s][i] = ld1(base + i * K * K + s);
}

template <int K, int ST, int V, typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ x,
                                                     const T* __restrict__ w,
                                                     T* __restrict__ y, DWGeom d) {
  constexpr int NWIN = (DW_X - 1) * ST + K;
  const int GC = d.G * d.C, CV = GC / V;
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
  const int gc0 = cv * V;
  const int wo0 = xg * DW_X;
  const int wi0 = wo0 * ST - d.pl;
  float acc[DW_X][V];
#pragma unroll
  for (int xi = 0; xi < DW_X; ++xi)
#pragma unroll
    for (int i = 0; i < V; ++i) acc[xi][i] = 0.f;
  for (int r = 0; r < K; ++r) {
    const int hi = ho * ST - d.pt + r;
    if (hi < 0 || hi >= d.H) continue;
    float wr[K][V];
    load_wrow<K, V, T>(w, d, gc0, r, wr);
    const T* xrow = x + ((int64_t)b * d.H + hi) * d.W * GC + gc0;
    float win[NWIN][V];
#pragma unroll
    for (int j = 0; j < NWIN; ++j) {
      const int wi = wi0 + j;
      if (wi >= 0 && wi < d.W) {
        ldv<V>(xrow + (int64_t)wi * GC, win[j]);
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) win[j][i] = 0.f;
      }
    }
#pragma unroll
    for (int xi = 0; xi < DW_X; ++xi)
#pragma unroll
      for (int s = 0; s < K; ++s)
#pragma unroll
        for (int i = 0; i < V; ++i) acc[xi][i] += win[xi * ST + s][i] * wr[s][i];
  }
#pragma unroll
  for (int xi = 0; xi < DW_X; ++xi) {
    const int wo = wo0 + xi;
    if (wo < d.Wo) stv<V>(y + (((int64_t)b * d.Ho + ho) * d.Wo + wo) * GC + gc0, acc[xi]);
  }
}

template <int K, int ST, int V, typename T>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const T* __restrict__ dy,
                                                       const T* __restrict__ w,
                                                       T* __restrict__ dx, DWGeom d) {
  const int GC = d.G * d.C, CV = GC / V;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)d.B * d.H * d.W * CV;
  if (idx >= total) return;
  const int cv = (int)(idx % CV);
  int64_t t = idx / CV;
  const int wi = (int)(t % d.W);
  t /= d.W;
  const int hi = (int)(t % d.H);
  const int b = (int)(t / d.H);
  const int gc0 = cv * V;
  float acc[V] = {};
  for (int r = 0; r < K; ++r) {
    const int hn = hi + d.pt - r;
    if (hn < 0 || hn % ST) continue;
    const int ho = hn / ST;
    if (ho >= d.Ho) continue;
    float wr[K][V];
    load_wrow<K, V, T>(w, d, gc0, r, wr);
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const int wn = wi + d.pl - s;
      if (wn < 0 || wn % ST) continue;
      const int wo = wn / ST;
      if (wo >= d.Wo) continue;
      float v[V];
      ldv<V>(dy + (((int64_t)b * d.Ho + ho) * d.Wo + wo) * GC + gc0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += v[i] * wr[s][i];
    }
  }
  stv<V>(dx + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, acc);
}

// grid (GC / 8, row slabs, K / RB filter-row bands); 256 lanes stride over the
// slab's output pixels, each accumulating RB x K taps x 8 channels
template <int K, int RB, int V, typename T>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ dy,
                                                       float* __restrict__ dw,
                                                       int64_t dw_gstride, DWGeom d, int st,
                                                       int64_t pix_per_slab) {
  constexpr int NT = RB * K;
  __shared__ float red[NT * V][4];
  const int GC = d.G * d.C;
  const int gc0 = blockIdx.x * V;
  const int r0 = blockIdx.z * RB;
  const int64_t P = (int64_t)d.B * d.Ho * d.Wo;
  const int64_t p0 = (int64_t)blockIdx.y * pix_per_slab;
  const int64_t p1 = min(P, p0 + pix_per_slab);
  float acc[NT][V];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < V; ++i) acc[t][i] = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const int wo = (int)(p % d.Wo);
    const int64_t q = p / d.Wo;
    const int ho = (int)(q % d.Ho);
    const int b = (int)(q / d.Ho);
    float g[V];
    ldv<V>(dy + p * GC + gc0, g);
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      const int hi = ho * st - d.pt + r0 + rr;
      if (hi < 0 || hi >= d.H) continue;
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int wi = wo * st - d.pl + s;
        if (wi < 0 || wi >= d.W) continue;
        float v[V];
        ldv<V>(x + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, v);
#pragma unroll
        for (int i = 0; i < V; ++i) acc[rr * K + s][i] += v[i] * g[i];
      }
    }
  }
  // wave reduction, then 4 waves -> LDS -> one atomic per (tap, channel)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float v = warp_sum(acc[t][i]);
      if (lane == 0) red[t * V + i][wid] = v;
    }
  __syncthreads();
  for (int e = threadIdx.x; e < NT * V; e += 256) {
    const float v = red[e][0] + red[e][1] + red[e][2] + red[e][3];
    const int t = e / V, i = e - t * V;
    const int gc = gc0 + i, g = gc / d.C, c = gc - g * d.C;
    atomicAdd(dw + g * dw_gstride + (int64_t)c * K * K + r0 * K + t, v);
  }
}

DWGeom make_dw(int B, int H, int W, int C, int G, int pt, int pl, int Ho, int Wo, int64_t ws) {
  DWGeom d;
  d.B = B;
  d.H = H;
  d.W = W;
  d.C = C;
  d.G = G;
  d.pt = pt;
  d.pl = pl;
  d.Ho = Ho;
  d.Wo = Wo;
  d.w_gstride = ws;
  return d;
}

bool dw_shape_ok(int C, int k, int st, int pt, int pl, int Ho, int Wo) {
  return C > 0 && (k == 3 || k == 5 || k == 7) && (st == 1 || st == 2) && pt >= 0 &&
         pl >= 0 && pt < k && pl < k && Ho > 0 && Wo > 0;
}

// V = 8 channels per thread when every config's channel count is a multiple
// of 8, else 1 (ragged widths, e.g. NASNet-Mobile's 11 / 22 / 44)
template <int K, int V, typename T>
void launch_fwd_v(const T* x, const T* w, T* y, const DWGeom& d, int st,
                  hipStream_t stream) {
  const int64_t n = (int64_t)d.B * d.Ho * ((d.Wo + DW_X - 1) / DW_X) * (d.G * d.C / V);
  if (st == 1)
    dw_fwd_kernel<K, 1, V, T><<<cer_blocks(n, 256), 256, 0, stream>>>(x, w, y, d);
  else
    dw_fwd_kernel<K, 2, V, T><<<cer_blocks(n, 256), 256, 0, stream>>>(x, w, y, d);
}

template <int K, typename T>
void launch_fwd(const T* x, const T* w, T* y, const DWGeom& d, int st, hipStream_t stream) {
  if (d.C % DW_V == 0)
    launch_fwd_v<K, DW_V, T>(x, w, y, d, st, stream);
  else
    launch_fwd_v<K, 1, T>(x, w, y, d, st, stream);
}

template <int K, int V, typename T>
void launch_dgrad_v(const T* dy, const T* w, T* dx, const DWGeom& d, int st,
                    hipStream_t stream) {
  const int64_t n = (int64_t)d.B * d.H * d.W * (d.G * d.C / V);
  if (st == 1)
    dw_dgrad_kernel<K, 1, V, T><<<cer_blocks(n, 256), 256, 0, stream>>>(dy, w, dx, d);
  else
    dw_dgrad_kernel<K, 2, V, T><<<cer_blocks(n, 256), 256, 0, stream>>>(dy, w, dx, d);
}

template <int K, typename T>
void launch_dgrad(const T* dy, const T* w, T* dx, const DWGeom& d, int st, hipStream_t stream) {
  if (d.C % DW_V == 0)
    launch_dgrad_v<K, DW_V, T>(dy, w, dx, d, st, stream);
  else
    launch_dgrad_v<K, 1, T>(dy, w, dx, d, st, stream);
}

template <int V, typename T>
void launch_wgrad(const T* x, const T* dy, float* dw, int64_t dw_gstride, const DWGeom& d, int k,
                  int st, hipStream_t stream) {
  const int64_t P = (int64_t)d.B * d.Ho * d.Wo;
  const int cblocks = d.G * d.C / V;
  const int bands = (k == 7) ? 7 : 1;      // k = 7: one filter row per block (56 accumulators)
  int64_t slabs = (2048 + (int64_t)cblocks * bands - 1) / ((int64_t)cblocks * bands);
  int64_t per = (P + slabs - 1) / slabs;
  if (per < 256) per = 256;
  slabs = (P + per - 1) / per;
  dim3 grid(cblocks, (unsigned)slabs, bands);
  if (k == 3)
    dw_wgrad_kernel<3, 3, V, T><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, st, per);
  else if (k == 5)
    dw_wgrad_kernel<5, 5, V, T><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, st, per);
  else
    dw_wgrad_kernel<7, 1, V, T><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, st, per);
}

}  // namespace

// pt / pl: top / left zero padding; Ho / Wo: output size (fixes bottom/right)
template <typename T>
static int dwconv_fwd_t(const T* x, int B, int H, int W, int C, int G, const T* w,
                           int64_t w_gstride, int k, int st, int pt, int pl, int Ho, int Wo,
                           T* y, hipStream_t stream) {
  if (!dw_shape_ok(C, k, st, pt, pl, Ho, Wo)) return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, pt, pl, Ho, Wo, w_gstride);
  if (k == 3)
    launch_fwd<3, T>(x, w, y, d, st, stream);
  else if (k == 5)
    launch_fwd<5, T>(x, w, y, d, st, stream);
  else
    launch_fwd<7, T>(x, w, y, d, st, stream);
  return (int)hipGetLastError();
}

// dw must be zero on entry (accumulated with atomics); dx may be null
template <typename T>
static int dwconv_bwd_t(const T* dy, const T* x, int B, int H, int W, int C, int G,
                           const T* w, int64_t w_gstride, float* dw, int64_t dw_gstride,
                           int k, int st, int pt, int pl, int Ho, int Wo, T* dx,
                           hipStream_t stream) {
  if (!dw_shape_ok(C, k, st, pt, pl, Ho, Wo)) return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, pt, pl, Ho, Wo, w_gstride);
  if (dx) {
    if (k == 3)
      launch_dgrad<3, T>(dy, w, dx, d, st, stream);
    else if (k == 5)
      launch_dgrad<5, T>(dy, w, dx, d, st, stream);
    else
      launch_dgrad<7, T>(dy, w, dx, d, st, stream);
  }
  if (C % DW_V == 0)
    launch_wgrad<DW_V, T>(x, dy, dw, dw_gstride, d, k, st, stream);
  else
    launch_wgrad<1, T>(x, dy, dw, dw_gstride, d, k, st, stream);
  return (int)hipGetLastError();
}

#define CER_DW_ENTRY_POINTS(T, SFX)                                                              \
  CER_API int cer_dwconv_fwd##SFX(const T* x, int B, int H, int W, int C, int G, const T* w,    \
                                  int64_t w_gstride, int k, int st, int pt, int pl, int Ho,     \
                                  int Wo, T* y, hipStream_t stream) {                           \
    return dwconv_fwd_t<T>(x, B, H, W, C, G, w, w_gstride, k, st, pt, pl, Ho, Wo, y, stream);   \
  }                                                                                              \
  CER_API int cer_dwconv_bwd##SFX(const T* dy, const T* x, int B, int H, int W, int C, int G,   \
                                  const T* w, int64_t w_gstride, float* dw, int64_t dw_gstride, \
                                  int k, int st, int pt, int pl, int Ho, int Wo, T* dx,         \
                                  hipStream_t stream) {                                         \
    return dwconv_bwd_t<T>(dy, x, B, H, W, C, G, w, w_gstride, dw, dw_gstride, k, st, pt, pl,   \
                           Ho, Wo, dx, stream);                                                 \
  }

CER_DW_ENTRY_POINTS(bf16_t, )
CER_DW_ENTRY_POINTS(float, _f32)
