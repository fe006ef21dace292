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
//  dgrad : one thread = 8 channels x 4 consecutive input columns (gathers
//          the dy taps that reach them; a sliding dy window at stride 1,
//          divisibility checks at stride 2)
//  wgrad : block = up to 64 channel groups x 256/CB position lanes x a band
//          of filter rows; channel-contiguous lanes (coalesced), 4 output
//          columns per position with a sliding input window, shuffle + LDS
//          reduction, fp32 atomics into the gradient arena (which the
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

// one thread = V channels x DW_X consecutive input columns: each filter row's
// weights are loaded once per 4 pixels, and at stride 1 the row's
// DW_X + K - 1 dy pixels once (sliding window) instead of 4K times
template <int K, int ST, int V, typename T>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const T* __restrict__ dy,
                                                       const T* __restrict__ w,
                                                       T* __restrict__ dx, DWGeom d) {
  const int GC = d.G * d.C, CV = GC / V;
  const int xgroups = (d.W + DW_X - 1) / DW_X;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)d.B * d.H * xgroups * CV;
  if (idx >= total) return;
  const int cv = (int)(idx % CV);
  int64_t t = idx / CV;
  const int xg = (int)(t % xgroups);
  t /= xgroups;
  const int hi = (int)(t % d.H);
  const int b = (int)(t / d.H);
  const int gc0 = cv * V;
  const int wi0 = xg * DW_X;
  float acc[DW_X][V];
#pragma unroll
  for (int xi = 0; xi < DW_X; ++xi)
#pragma unroll
    for (int i = 0; i < V; ++i) acc[xi][i] = 0.f;
  for (int r = 0; r < K; ++r) {
    const int hn = hi + d.pt - r;
    if (hn < 0 || hn % ST) continue;
    const int ho = hn / ST;
    if (ho >= d.Ho) continue;
    float wr[K][V];
    load_wrow<K, V, T>(w, d, gc0, r, wr);
    const T* dyrow = dy + ((int64_t)b * d.Ho + ho) * d.Wo * GC + gc0;
    if constexpr (ST == 1) {
      // window j <-> output column wi0 + pl - (K - 1) + j
      constexpr int NWIN = DW_X + K - 1;
      const int wo_lo = wi0 + d.pl - (K - 1);
      float win[NWIN][V];
#pragma unroll
      for (int j = 0; j < NWIN; ++j) {
        const int wo = wo_lo + j;
        if (wo >= 0 && wo < d.Wo) {
          ldv<V>(dyrow + (int64_t)wo * GC, win[j]);
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
          for (int i = 0; i < V; ++i) acc[xi][i] += win[xi + K - 1 - s][i] * wr[s][i];
    } else {
#pragma unroll
      for (int xi = 0; xi < DW_X; ++xi)
#pragma unroll
        for (int s = 0; s < K; ++s) {
          const int wn = wi0 + xi + d.pl - s;
          if (wn < 0 || wn % ST) continue;
          const int wo = wn / ST;
          if (wo >= d.Wo) continue;
          float v[V];
          ldv<V>(dyrow + (int64_t)wo * GC, v);
#pragma unroll
          for (int i = 0; i < V; ++i) acc[xi][i] += v[i] * wr[s][i];
        }
    }
  }
#pragma unroll
  for (int xi = 0; xi < DW_X; ++xi) {
    const int wi = wi0 + xi;
    if (wi < d.W) stv<V>(dx + (((int64_t)b * d.H + hi) * d.W + wi) * GC + gc0, acc[xi]);
  }
}

// grid (ceil(CV / CB), position slabs, K / RB filter-row bands), CV = GC / V
// channel groups.  Thread t = (position lane t >> lcb, channel group t & (CB-1)):
// adjacent lanes read adjacent channel groups of ONE pixel, so a wave's load
// covers 64 / CB pixels with CB * V contiguous channels each (the earlier
// lane-per-pixel layout touched 64 cache lines per load and was bound by the
// vector-cache line rate).  A position is X consecutive output columns of one
// row: dy is loaded once per position, and per filter row the (X-1)*ST + K
// input pixels once (sliding window), instead of X * (1 + RB * K) loads.
// Position lanes of a channel group reduce by shuffles, the 4 waves by LDS
// atomics, then one fp32 atomic per (channel, tap) into the gradient arena.
template <int K, int RB, int ST, int X, int V, typename T>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ dy,
                                                       float* __restrict__ dw,
                                                       int64_t dw_gstride, DWGeom d, int lcb,
                                                       int pos_per_slab) {
  constexpr int NT = RB * K;
  constexpr int NWIN = (X - 1) * ST + K;
  __shared__ float red[64 * NT * V];
  const int CB = 1 << lcb;
  const int GC = d.G * d.C, CV = GC / V;
  const int c = threadIdx.x & (CB - 1), pr = threadIdx.x >> lcb, PR = 256 >> lcb;
  const int cv = blockIdx.x * CB + c;
  const bool active = cv < CV;
  const int gc0 = cv * V;
  const int r0 = blockIdx.z * RB;
  const int xgroups = (d.Wo + X - 1) / X;
  // positions fit in 32 bits (checked on the host): 32-bit division per step
  const int Pn = d.B * d.Ho * xgroups;
  const int q0 = blockIdx.y * pos_per_slab;
  const int q1 = min(Pn, q0 + pos_per_slab);
  float acc[NT][V];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < V; ++i) acc[t][i] = 0.f;
  if (active) {
    for (int q = q0 + pr; q < q1; q += PR) {
      const unsigned u = (unsigned)q / (unsigned)xgroups;
      const int xg = q - (int)u * xgroups;
      const unsigned bq = u / (unsigned)d.Ho;
      const int ho = (int)u - (int)bq * d.Ho;
      const int b = (int)bq;
      const int wo0 = xg * X;
      float g[X][V];
#pragma unroll
      for (int xi = 0; xi < X; ++xi) {
        if (wo0 + xi < d.Wo) {
          ldv<V>(dy + (((int64_t)b * d.Ho + ho) * d.Wo + wo0 + xi) * GC + gc0, g[xi]);
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) g[xi][i] = 0.f;
        }
      }
      const int wi0 = wo0 * ST - d.pl;
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const int hi = ho * ST - d.pt + r0 + rr;
        if (hi < 0 || hi >= d.H) continue;
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
        for (int xi = 0; xi < X; ++xi)
#pragma unroll
          for (int s = 0; s < K; ++s)
#pragma unroll
            for (int i = 0; i < V; ++i) acc[rr * K + s][i] += win[xi * ST + s][i] * g[xi][i];
      }
    }
  }
  // position lanes of a wave (lane ^ CB, ^ 2CB, ...) -> lanes 0..CB-1
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float v = acc[t][i];
      for (int o = CB; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[t][i] = v;
    }
  const int n = CB * NT * V;
  for (int e = threadIdx.x; e < n; e += 256) red[e] = 0.f;
  __syncthreads();
  if ((threadIdx.x & 63) < CB && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < V; ++i) atomicAdd(&red[(c * NT + t) * V + i], acc[t][i]);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += 256) {
    const int ce = e / (NT * V), rem = e - ce * (NT * V);
    const int t = rem / V, i = rem - t * V;
    const int cve = blockIdx.x * CB + ce;
    if (cve >= CV) continue;
    const int gc = cve * V + i, g = gc / d.C, ch = gc - g * d.C;
    atomicAdd(dw + g * dw_gstride + (int64_t)ch * K * K + r0 * K + t, red[e]);
  }
}

// 3x3 forward + the BN (sum, sum^2) partials of its output for the BN that
// consumes it (ops.nn.dwconv2d stats=True), so that BN skips its statistics
// pass.  Layout as dw_wgrad_kernel: grid (ceil(CV / CB), position slabs),
// thread = (position lane, channel group of 8); the whole 3x3 x 8 filter stays
// in registers for the slab; per position the fwd sliding window.  Position
// lanes reduce by shuffles, the 4 waves through LDS in a fixed order, then
// fp64 atomics into slab (blockIdx.y % nsl) of the [nsl][2][GC] buffer in the
// conv epilogue's SLAB_F64 format (conv.hip stat_store), which bn.hip's
// fold-finalize apply reads.
template <int ST, typename T>
__global__ __launch_bounds__(256) void dw_fwd_stats_kernel(const T* __restrict__ x,
                                                           const T* __restrict__ w,
                                                           T* __restrict__ y, DWGeom d, int lcb,
                                                           int pos_per_slab,
                                                           float* __restrict__ part, int nsl) {
  constexpr int K = 3, V = DW_V, X = DW_X;
  constexpr int NWIN = (X - 1) * ST + K;
  __shared__ float red[4][64][2 * V];
  const int CB = 1 << lcb;
  const int GC = d.G * d.C, CV = GC / V;
  const int c = threadIdx.x & (CB - 1), pr = threadIdx.x >> lcb, PR = 256 >> lcb;
  const int cv = blockIdx.x * CB + c;
  const bool active = cv < CV;
  const int gc0 = cv * V;
  const int xgroups = (d.Wo + X - 1) / X;
  const int Pn = d.B * d.Ho * xgroups;
  const int q0 = blockIdx.y * pos_per_slab;
  const int q1 = min(Pn, q0 + pos_per_slab);
  float sm[V], sq[V];
#pragma unroll
  for (int i = 0; i < V; ++i) sm[i] = sq[i] = 0.f;
  if (active) {
    float wk[K][K][V];
#pragma unroll
    for (int r = 0; r < K; ++r) load_wrow<K, V, T>(w, d, gc0, r, wk[r]);
    for (int q = q0 + pr; q < q1; q += PR) {
      const unsigned u = (unsigned)q / (unsigned)xgroups;
      const int xg = q - (int)u * xgroups;
      const unsigned bq = u / (unsigned)d.Ho;
      const int ho = (int)u - (int)bq * d.Ho;
      const int b = (int)bq;
      const int wo0 = xg * X;
      const int wi0 = wo0 * ST - d.pl;
      float acc[X][V];
#pragma unroll
      for (int xi = 0; xi < X; ++xi)
#pragma unroll
        for (int i = 0; i < V; ++i) acc[xi][i] = 0.f;
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int hi = ho * ST - d.pt + r;
        if (hi < 0 || hi >= d.H) continue;
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
        for (int xi = 0; xi < X; ++xi)
#pragma unroll
          for (int s = 0; s < K; ++s)
#pragma unroll
            for (int i = 0; i < V; ++i) acc[xi][i] += win[xi * ST + s][i] * wk[r][s][i];
      }
#pragma unroll
      for (int xi = 0; xi < X; ++xi) {
        if (wo0 + xi >= d.Wo) continue;
        T* yp = y + (((int64_t)b * d.Ho + ho) * d.Wo + wo0 + xi) * GC + gc0;
        stv<V>(yp, acc[xi]);
        // statistics of the STORED values (bf16 output: rounded as BN reads them)
#pragma unroll
        for (int i = 0; i < V; ++i) {
          float v = acc[xi][i];
          if constexpr (!std::is_same<T, float>::value) v = bf2f(f2bf(v));
          sm[i] += v;
          sq[i] += v * v;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i)
    for (int o = CB; o < 64; o <<= 1) {
      sm[i] += __shfl_xor(sm[i], o, 64);
      sq[i] += __shfl_xor(sq[i], o, 64);
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < CB) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      red[wid][lane][i] = sm[i];
      red[wid][lane][V + i] = sq[i];
    }
  }
  __syncthreads();
  double* slab = reinterpret_cast<double*>(part) + (int64_t)(blockIdx.y % nsl) * 2 * GC;
  for (int e = threadIdx.x; e < CB * 2 * V; e += 256) {
    const int ce = e / (2 * V), rem = e - ce * (2 * V);
    const int cve = blockIdx.x * CB + ce;
    if (cve >= CV) continue;
    const float v = red[0][ce][rem] + red[1][ce][rem] + red[2][ce][rem] + red[3][ce][rem];
    const int row = rem / V, i = rem - row * V;
    atomicAdd(slab + (int64_t)row * GC + cve * V + i, (double)v);
  }
}

// 3x3 input gradient + the backward partials of the BN that PRODUCED the
// depthwise input (BN link, ops.nn.BNLink: MobileNetV2's expansion BN), so
// that BN skips its own pass over (dy, z, y).  dx is that BN's output
// gradient d; with its output y (= this conv's input) and input z:
//   dz = act'(y) d,  partials (sum dz, sum dz (z - mean) invstd)
// -- the conv dgrad epilogue's YM_Y arithmetic (conv.hip epi32 bnbwd), over
// the STORED d.  Layout and reduction as dw_fwd_stats_kernel (positions are
// 4 input columns); fp64 atomics into slab (blockIdx.y % nsl).
template <int ST, typename T>
__global__ __launch_bounds__(256) void dw_dgrad_bn_kernel(
    const T* __restrict__ dy, const T* __restrict__ w, T* __restrict__ dx, DWGeom d, int lcb,
    int pos_per_slab, const T* __restrict__ ybn, const T* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ invstd, int act,
    float* __restrict__ part, int nsl) {
  constexpr int K = 3, V = DW_V, X = DW_X;
  __shared__ float red[4][64][2 * V];
  const int CB = 1 << lcb;
  const int GC = d.G * d.C, CV = GC / V;
  const int c = threadIdx.x & (CB - 1), pr = threadIdx.x >> lcb, PR = 256 >> lcb;
  const int cv = blockIdx.x * CB + c;
  const bool active = cv < CV;
  const int gc0 = cv * V;
  const int xgroups = (d.W + X - 1) / X;
  const int Pn = d.B * d.H * xgroups;
  const int q0 = blockIdx.y * pos_per_slab;
  const int q1 = min(Pn, q0 + pos_per_slab);
  float sm[V], sq[V];
#pragma unroll
  for (int i = 0; i < V; ++i) sm[i] = sq[i] = 0.f;
  if (active) {
    float wk[K][K][V], mu[V], is[V];
#pragma unroll
    for (int r = 0; r < K; ++r) load_wrow<K, V, T>(w, d, gc0, r, wk[r]);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      mu[i] = mean[gc0 + i];
      is[i] = invstd[gc0 + i];
    }
    for (int q = q0 + pr; q < q1; q += PR) {
      const unsigned u = (unsigned)q / (unsigned)xgroups;
      const int xg = q - (int)u * xgroups;
      const unsigned bq = u / (unsigned)d.H;
      const int hi = (int)u - (int)bq * d.H;
      const int b = (int)bq;
      const int wi0 = xg * X;
      float acc[X][V];
#pragma unroll
      for (int xi = 0; xi < X; ++xi)
#pragma unroll
        for (int i = 0; i < V; ++i) acc[xi][i] = 0.f;
#pragma unroll
      for (int r = 0; r < K; ++r) {
        const int hn = hi + d.pt - r;
        if (hn < 0 || hn % ST) continue;
        const int ho = hn / ST;
        if (ho >= d.Ho) continue;
        const T* dyrow = dy + ((int64_t)b * d.Ho + ho) * d.Wo * GC + gc0;
        if constexpr (ST == 1) {
          constexpr int NWIN = X + K - 1;
          const int wo_lo = wi0 + d.pl - (K - 1);
          float win[NWIN][V];
#pragma unroll
          for (int j = 0; j < NWIN; ++j) {
            const int wo = wo_lo + j;
            if (wo >= 0 && wo < d.Wo) {
              ldv<V>(dyrow + (int64_t)wo * GC, win[j]);
            } else {
#pragma unroll
              for (int i = 0; i < V; ++i) win[j][i] = 0.f;
            }
          }
#pragma unroll
          for (int xi = 0; xi < X; ++xi)
#pragma unroll
            for (int s = 0; s < K; ++s)
#pragma unroll
              for (int i = 0; i < V; ++i) acc[xi][i] += win[xi + K - 1 - s][i] * wk[r][s][i];
        } else {
#pragma unroll
          for (int xi = 0; xi < X; ++xi)
#pragma unroll
            for (int s = 0; s < K; ++s) {
              const int wn = wi0 + xi + d.pl - s;
              if (wn < 0 || wn % ST) continue;
              const int wo = wn / ST;
              if (wo >= d.Wo) continue;
              float v[V];
              ldv<V>(dyrow + (int64_t)wo * GC, v);
#pragma unroll
              for (int i = 0; i < V; ++i) acc[xi][i] += v[i] * wk[r][s][i];
            }
        }
      }
#pragma unroll
      for (int xi = 0; xi < X; ++xi) {
        if (wi0 + xi >= d.W) continue;
        const int64_t off = (((int64_t)b * d.H + hi) * d.W + wi0 + xi) * GC + gc0;
        stv<V>(dx + off, acc[xi]);
        float yv[V], zv[V];
        ldv<V>(ybn + off, yv);
        ldv<V>(z + off, zv);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          float dd = acc[xi][i];
          if constexpr (!std::is_same<T, float>::value) dd = bf2f(f2bf(dd));
          const bool pass = act == 6 ? (yv[i] > 0.f && yv[i] < 6.f) : act == 1 ? yv[i] > 0.f : true;
          const float dz = pass ? dd : 0.f;
          sm[i] += dz;
          sq[i] += dz * (zv[i] - mu[i]) * is[i];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i)
    for (int o = CB; o < 64; o <<= 1) {
      sm[i] += __shfl_xor(sm[i], o, 64);
      sq[i] += __shfl_xor(sq[i], o, 64);
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < CB) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      red[wid][lane][i] = sm[i];
      red[wid][lane][V + i] = sq[i];
    }
  }
  __syncthreads();
  double* slab = reinterpret_cast<double*>(part) + (int64_t)(blockIdx.y % nsl) * 2 * GC;
  for (int e = threadIdx.x; e < CB * 2 * V; e += 256) {
    const int ce = e / (2 * V), rem = e - ce * (2 * V);
    const int cve = blockIdx.x * CB + ce;
    if (cve >= CV) continue;
    const float v = red[0][ce][rem] + red[1][ce][rem] + red[2][ce][rem] + red[3][ce][rem];
    const int row = rem / V, i = rem - row * V;
    atomicAdd(slab + (int64_t)row * GC + cve * V + i, (double)v);
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
  const int64_t n = (int64_t)d.B * d.H * ((d.W + DW_X - 1) / DW_X) * (d.G * d.C / V);
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

// channel groups per block: the widest power of two <= 64 that leaves at most
// 1/8 of the block's channel lanes idle
inline int wgrad_lcb(int CV) {
  int l = 6;
  while (l > 0) {
    const int cb = 1 << l;
    const int64_t n = (int64_t)(CV + cb - 1) / cb * cb;
    if ((n - CV) * 8 <= CV) break;
    --l;
  }
  return l;
}

// target block counts of the slab-loop grids: wgrad (CER_DWW_BLOCKS) and the
// fwd / dgrad kernels with BN statistics (CER_DW_BN_BLOCKS).  Fewer, longer
// slabs won on MobileNetV2 at 8 configs (wgrad 1024 -> 256 blocks: +3.3 %,
// one config neutral; profiles/r3_secondary_published.md)
inline int64_t env_blocks(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  const long v = e ? atol(e) : 0;
  return v > 0 ? (int64_t)v : dflt;
}
inline int64_t dww_blocks() {
  static const int64_t n = env_blocks("CER_DWW_BLOCKS", 256);
  return n;
}
inline int64_t dwbn_blocks() {
  static const int64_t n = env_blocks("CER_DW_BN_BLOCKS", 1024);
  return n;
}

#ifndef CER_DWW_X
#define CER_DWW_X 4   // output columns per wgrad position (A/B twins: -DCER_DWW_X=2)
#endif

template <int K, int RB, int V, typename T>
void launch_wgrad_k(const T* x, const T* dy, float* dw, int64_t dw_gstride, const DWGeom& d,
                    int st, hipStream_t stream) {
  constexpr int X = CER_DWW_X;
  const int CV = d.G * d.C / V;
  const int lcb = wgrad_lcb(CV), CB = 1 << lcb, PR = 256 >> lcb;
  const int cblocks = (CV + CB - 1) / CB;
  constexpr int bands = K / RB;
  const int64_t Pn = (int64_t)d.B * d.Ho * ((d.Wo + X - 1) / X);
  // ~dww_blocks() blocks; every position lane at least 2 positions (bounds the atomics)
  const int64_t target = dww_blocks();
  int64_t slabs = (target + (int64_t)cblocks * bands - 1) / ((int64_t)cblocks * bands);
  int64_t per = (Pn + slabs - 1) / slabs;
  if (per < 2 * PR) per = 2 * PR;
  slabs = (Pn + per - 1) / per;
  dim3 grid(cblocks, (unsigned)slabs, bands);
  if (st == 1)
    dw_wgrad_kernel<K, RB, 1, X, V, T><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, lcb,
                                                                 (int)per);
  else
    dw_wgrad_kernel<K, RB, 2, X, V, T><<<grid, 256, 0, stream>>>(x, dy, dw, dw_gstride, d, lcb,
                                                                 (int)per);
}

template <int V, typename T>
void launch_wgrad(const T* x, const T* dy, float* dw, int64_t dw_gstride, const DWGeom& d, int k,
                  int st, hipStream_t stream) {
  // k = 3: the whole filter per block (72 accumulators at V = 8); k = 5 / 7:
  // one filter row per block
  if (k == 3)
    launch_wgrad_k<3, 3, V, T>(x, dy, dw, dw_gstride, d, st, stream);
  else if (k == 5)
    launch_wgrad_k<5, 1, V, T>(x, dy, dw, dw_gstride, d, st, stream);
  else
    launch_wgrad_k<7, 1, V, T>(x, dy, dw, dw_gstride, d, st, stream);
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
  if ((int64_t)B * Ho * Wo > INT32_MAX) return (int)hipErrorInvalidValue;
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

// 3x3, every config's C % 8 == 0; ``part`` zeroed [nsl][2][G*C] doubles
template <typename T>
static int dwconv_fwd_stats_t(const T* x, int B, int H, int W, int C, int G, const T* w,
                              int64_t w_gstride, int k, int st, int pt, int pl, int Ho, int Wo,
                              T* y, float* part, int nsl, hipStream_t stream) {
  if (!dw_shape_ok(C, k, st, pt, pl, Ho, Wo) || k != 3 || C % DW_V || nsl <= 0)
    return (int)hipErrorInvalidValue;
  if ((int64_t)B * Ho * Wo > INT32_MAX) return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, pt, pl, Ho, Wo, w_gstride);
  const int CV = G * C / DW_V;
  const int lcb = wgrad_lcb(CV), CB = 1 << lcb, PR = 256 >> lcb;
  const int cblocks = (CV + CB - 1) / CB;
  const int64_t Pn = (int64_t)B * Ho * ((Wo + DW_X - 1) / DW_X);
  int64_t slabs = (dwbn_blocks() + cblocks - 1) / cblocks;
  int64_t per = (Pn + slabs - 1) / slabs;
  if (per < 2 * PR) per = 2 * PR;
  slabs = (Pn + per - 1) / per;
  dim3 grid(cblocks, (unsigned)slabs);
  if (st == 1)
    dw_fwd_stats_kernel<1, T><<<grid, 256, 0, stream>>>(x, w, y, d, lcb, (int)per, part, nsl);
  else
    dw_fwd_stats_kernel<2, T><<<grid, 256, 0, stream>>>(x, w, y, d, lcb, (int)per, part, nsl);
  return (int)hipGetLastError();
}

// backward with the producing BN's backward partials (dw_dgrad_bn_kernel):
// 3x3, C % 8 == 0, act in {0, 1 (ReLU), 6 (ReLU6)}; ``part`` zeroed
// [nsl][2][G*C] doubles; dw zero on entry
template <typename T>
static int dwconv_bwd_bn_t(const T* dy, const T* x, const T* z, const float* mean,
                           const float* invstd, int act, int B, int H, int W, int C, int G,
                           const T* w, int64_t w_gstride, float* dw, int64_t dw_gstride, int k,
                           int st, int pt, int pl, int Ho, int Wo, T* dx, float* part, int nsl,
                           hipStream_t stream) {
  if (!dw_shape_ok(C, k, st, pt, pl, Ho, Wo) || k != 3 || C % DW_V || nsl <= 0 || !dx ||
      (act != 0 && act != 1 && act != 6))
    return (int)hipErrorInvalidValue;
  if ((int64_t)B * H * W > INT32_MAX || (int64_t)B * Ho * Wo > INT32_MAX)
    return (int)hipErrorInvalidValue;
  const DWGeom d = make_dw(B, H, W, C, G, pt, pl, Ho, Wo, w_gstride);
  const int CV = G * C / DW_V;
  const int lcb = wgrad_lcb(CV), CB = 1 << lcb, PR = 256 >> lcb;
  const int cblocks = (CV + CB - 1) / CB;
  const int64_t Pn = (int64_t)B * H * ((W + DW_X - 1) / DW_X);
  int64_t slabs = (dwbn_blocks() + cblocks - 1) / cblocks;
  int64_t per = (Pn + slabs - 1) / slabs;
  if (per < 2 * PR) per = 2 * PR;
  slabs = (Pn + per - 1) / per;
  dim3 grid(cblocks, (unsigned)slabs);
  if (st == 1)
    dw_dgrad_bn_kernel<1, T><<<grid, 256, 0, stream>>>(dy, w, dx, d, lcb, (int)per, x, z, mean,
                                                       invstd, act, part, nsl);
  else
    dw_dgrad_bn_kernel<2, T><<<grid, 256, 0, stream>>>(dy, w, dx, d, lcb, (int)per, x, z, mean,
                                                       invstd, act, part, nsl);
  launch_wgrad<DW_V, T>(x, dy, dw, dw_gstride, d, k, st, stream);
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
  }                                                                                              \
  CER_API int cer_dwconv_fwd_stats##SFX(const T* x, int B, int H, int W, int C, int G,          \
                                        const T* w, int64_t w_gstride, int k, int st, int pt,   \
                                        int pl, int Ho, int Wo, T* y, float* part, int nsl,     \
                                        hipStream_t stream) {                                   \
    return dwconv_fwd_stats_t<T>(x, B, H, W, C, G, w, w_gstride, k, st, pt, pl, Ho, Wo, y,     \
                                 part, nsl, stream);                                            \
  }                                                                                              \
  CER_API int cer_dwconv_bwd_bn##SFX(const T* dy, const T* x, const T* z, const float* mean,    \
                                     const float* invstd, int act, int B, int H, int W, int C,  \
                                     int G, const T* w, int64_t w_gstride, float* dw,           \
                                     int64_t dw_gstride, int k, int st, int pt, int pl, int Ho, \
                                     int Wo, T* dx, float* part, int nsl, hipStream_t stream) { \
    return dwconv_bwd_bn_t<T>(dy, x, z, mean, invstd, act, B, H, W, C, G, w, w_gstride, dw,    \
                              dw_gstride, k, st, pt, pl, Ho, Wo, dx, part, nsl, stream);        \
  }

CER_DW_ENTRY_POINTS(bf16_t, )
CER_DW_ENTRY_POINTS(float, _f32)
