// BatchNorm (+ residual add) (+ ReLU / ReLU6) over packed NHWC channels
// (SURVEY.md K7).  Activations x [M, C] bf16 with C = G*Cper packed channels
// (M = B*H*W); per-channel parameters live in the arena with a per-config
// stride: channel (g, c) -> ptr + g*stride + c.
//
// Thread mapping (all kernels): a 256-thread block covers CBd = 8*TCd
// channels x TRd row lanes, TCd = min(32, C/8), TRd = 256/TCd; a thread owns
// one 8-channel vector (16-B loads/stores) and strides over rows by TRd, so
// every thread of every block is busy even for narrow layers (C = 64).
//
// Forward (training): partials (per row slab, deterministic, no atomics) ->
// finalize (mean, invstd, running stats) -> apply y = act(xhat*g + b + res).
// Backward: partials (sum dz, sum dz*xhat) -> finalize (dgamma, dbeta into the
// fp32 gradient arena) -> apply dx = g*invstd*(dz - mean dz - xhat mean(dz xhat)),
// dres = dz.  dz = act'(.) * dy takes the activation mask from (YM):
//   YM_NONE  no activation: y is never read,
//   YM_Y     y (ReLU6, or a residual join: y = act(xhat*g + b + res)),
//   YM_Z     a plain ReLU without residual: mask = (x*sc + sh > 0), recomputed
//            from the BN input with the forward's exact scale/shift, so the
//            backward reads two tensors per pass (dy, x) instead of three.
#include "common.h"

#include <stdlib.h>

constexpr int BN_T = 256;
constexpr int VEC = 8;  // channels per thread

struct Strided {
  const void* p;
  int64_t stride;  // elements between configs
};

__device__ __forceinline__ float act_fwd(float z, int code) {
  if (code == 6) return fminf(fmaxf(z, 0.f), 6.f);
  if (code) return fmaxf(z, 0.f);
  return z;
}

__device__ __forceinline__ float act_bwd(float dy, float y, int code) {
  if (code == 6) return (y > 0.f && y < 6.f) ? dy : 0.f;
  if (code) return y > 0.f ? dy : 0.f;
  return dy;
}

struct Map {
  int tc_n, tr_n, cb;  // threads along channels, row lanes, channels per block
};

// V channels per thread (VEC, or 1 for ragged channel counts).  tc_n need
// not divide BN_T: the BN_T % tc_n surplus threads (tr == tr_n) are idle in
// every kernel
static Map make_map(int C, int V = VEC) {
  const int cap = V == 1 ? 64 : 32;
  int tc = (C / V) < cap ? (C / V) : cap;
  if (tc < 1) tc = 1;
  return Map{tc, BN_T / tc, tc * V};
}

// grid (channel blocks, row slabs) with ~`target` blocks and >= min_rows rows per slab
static void make_grid(int64_t M, int C, const Map& mp, int target, int min_rows, dim3* grid,
                      int* rows) {
  const int cblocks = (C + mp.cb - 1) / mp.cb;
  int64_t want = (target + cblocks - 1) / cblocks;
  int64_t r = (M + want - 1) / want;
  if (r < min_rows) r = min_rows;
  *rows = (int)r;
  *grid = dim3(cblocks, (unsigned)((M + r - 1) / r));
}

// ---------------------------------------------------------------------------
// plain / agent-scope element access (SC: a value handed between blocks of
// one kernel, across the non-coherent per-XCD L2s, moves by agent-scope
// atomic stores / loads; every launch path here hands off between kernels)
template <bool SC>
__device__ __forceinline__ float ldf(const float* p) {
  if (SC) return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

template <bool SC>
__device__ __forceinline__ void stf(float* p, float v) {
  if (SC)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

// ---------------------------------------------------------------------------
// stage 1: per-slab partial sums -> part[slab][2][C]
// ---------------------------------------------------------------------------
constexpr int YM_NONE = 0, YM_Y = 1, YM_Z = 2, YM_M = 3;

// YM_M: the activation mask of a residual join as one bit per element,
// written by the forward apply (mask_out [M][C / 8] bytes, bit i = channel
// 8j + i active: act_bwd(1, y) != 0) and read in backward instead of the
// fp32 output y -- 1/32 of y's bytes, bit-identical decisions (8-aligned
// widths only).  The backward kernels take the mask through their y pointer.
__device__ __forceinline__ uint32_t act_bits8(const float* o, int act) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) m |= (o[i] > 0.f && (act != 6 || o[i] < 6.f)) ? (1u << i) : 0u;
  return m;
}

// 8 mask bits -> y-like values (1 active / 0 not) for the YM_Y arithmetic
__device__ __forceinline__ void mask_to_y8(const uint8_t* mrow, int c0, float* yv) {
  const uint32_t m = mrow[c0 >> 3];
#pragma unroll
  for (int i = 0; i < 8; ++i) yv[i] = (m >> i) & 1u ? 1.f : 0.f;
}

// forward scale / shift of 8 channels (bitwise the apply_fwd_tile values)
template <typename T, int V = VEC>
__device__ __forceinline__ void bn_scale_shift(const Strided& gamma, const Strided& beta, int g,
                                               int cc, const float* mu, const float* is,
                                               float* sc, float* sh) {
  float ga[VEC], be[VEC];
  ldv<V>((const T*)gamma.p + g * gamma.stride + cc, ga);
  ldv<V>((const T*)beta.p + g * beta.stride + cc, be);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    sc[i] = is[i] * ga[i];
    sh[i] = be[i] - mu[i] * sc[i];
  }
}

// activation gradient of one element under mask mode YM
template <int YM>
__device__ __forceinline__ float dz_of(float d, float yv, float xv, float sc, float sh, int act) {
  if (YM == YM_NONE) return d;
  if (YM == YM_Z) return (xv * sc + sh + 0.f) > 0.f ? d : 0.f;
  if (YM == YM_M) return yv > 0.f ? d : 0.f;
  return act_bwd(d, yv, act);
}

// one (channel block cbk, row slab) tile; `red` = 2*BN_T*VEC floats of LDS
template <typename T, int MODE, bool SC, int YM = YM_Y, int V = VEC>  // MODE 0: (sum x, sum x^2)   1: (sum dz, sum dz*xhat)
__device__ __forceinline__ void partials_tile(
    const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ part,
    int64_t M, int C, int rows_per_slab, int act, const Map& mp, int cbk, int slab, float* red,
    const Strided& gamma = Strided{nullptr, 0}, const Strided& beta = Strided{nullptr, 0},
    int Cper = 1, int f64 = 0) {
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = cbk * mp.cb + tc * V;
  const bool cok = c0 < C && tr < mp.tr_n;
  float s[VEC] = {0, 0, 0, 0, 0, 0, 0, 0}, q[VEC] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[VEC], is[VEC], sc[VEC], sh[VEC];
  if (MODE == 1 && cok) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      mu[i] = mean[c0 + i];
      is[i] = invstd[c0 + i];
    }
    if (YM == YM_Z) {
      const int g = c0 / Cper;
      bn_scale_shift<T, V>(gamma, beta, g, c0 - g * Cper, mu, is, sc, sh);
    }
  }
  const int64_t r0 = (int64_t)slab * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  // PU rows in flight per thread: loads of all rows issue before any use
  // (narrow layers / small batches leave few waves per CU to hide latency)
  constexpr int PU = 4;
  if (cok) {
    for (int64_t r = r0 + tr; r < r1; r += PU * mp.tr_n) {
      float v[PU][VEC], d[PU][VEC], yv[PU][VEC];
      bool ok[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t rr = r + (int64_t)u * mp.tr_n;
        ok[u] = rr < r1;
        if (ok[u]) {
          ldv<V>(x + rr * C + c0, v[u]);
          if (MODE == 1) {
            ldv<V>(dy + rr * C + c0, d[u]);
            if (YM == YM_Y) ldv<V>(y + rr * C + c0, yv[u]);
            if constexpr (YM == YM_M)
              mask_to_y8(reinterpret_cast<const uint8_t*>(y) + rr * (C / 8), c0, yv[u]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (!ok[u]) continue;
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < V; ++i) {
            s[i] += v[u][i];
            q[i] += v[u][i] * v[u][i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const float dz = dz_of<YM>(d[u][i], yv[u][i], v[u][i], sc[i], sh[i], act);
            s[i] += dz;
            q[i] += dz * (v[u][i] - mu[i]) * is[i];
          }
        }
      }
    }
  }
  float* rs = red;
  float* rq = red + BN_T * VEC;
  if (tr < mp.tr_n) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      rs[tr * mp.cb + tc * V + i] = s[i];
      rq[tr * mp.cb + tc * V + i] = q[i];
    }
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < mp.cb; cl += BN_T) {
    const int c = cbk * mp.cb + cl;
    if (c >= C) continue;
    float a = 0.f, b = 0.f;
    for (int k = 0; k < mp.tr_n; ++k) {
      a += rs[k * mp.cb + cl];
      b += rq[k * mp.cb + cl];
    }
    if (f64) {        // fp64 atomics into slab (row slab % f64) of a zeroed buffer
      double* dd = reinterpret_cast<double*>(part) + (int64_t)(slab % f64) * 2 * C;
      atomicAdd(dd + c, (double)a);
      atomicAdd(dd + C + c, (double)b);
      continue;
    }
    float* dst = part + (int64_t)slab * 2 * C;
    stf<SC>(dst + c, a);
    stf<SC>(dst + C + c, b);
  }
  __syncthreads();  // `red` is reused by the next tile of a cooperative block
}

template <typename T, int MODE, int YM = YM_Y, int V = VEC>
__global__ __launch_bounds__(BN_T) void bn_partials(
    const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ part,
    int64_t M, int C, int rows_per_slab, int act, Map mp, Strided gamma = Strided{nullptr, 0},
    Strided beta = Strided{nullptr, 0}, int Cper = 1, int f64 = 0) {
  __shared__ float red[2 * BN_T * VEC];
  partials_tile<T, MODE, false, YM, V>(x, dy, y, mean, invstd, part, M, C, rows_per_slab, act, mp,
                                 blockIdx.x, blockIdx.y, red, gamma, beta, Cper, f64);
}

// ---------------------------------------------------------------------------
// stage 2: finalize
// ---------------------------------------------------------------------------
// one task = 8 channels x 32 slab lanes; each lane keeps 8 slab loads in
// flight (the partials were just written by other CUs: every round trip is an
// L2/MALL miss, so the reduction is latency-bound), LDS tree
constexpr int FIN_C = 8, FIN_L = 32, FIN_U = 8;

template <bool SC>
__device__ __forceinline__ void sum_slabs(const float* __restrict__ part, int slabs, int C,
                                          int task, float* a_out, float* b_out) {
  __shared__ float sa[FIN_L][FIN_C], sb[FIN_L][FIN_C];
  const int cl = threadIdx.x % FIN_C, ln = threadIdx.x / FIN_C;
  const int c = task * FIN_C + cl;
  float a = 0.f, b = 0.f;
  if (c < C) {
    float au[FIN_U], bu[FIN_U];
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) au[u] = bu[u] = 0.f;
    int k = ln;
    for (; k + (FIN_U - 1) * FIN_L < slabs; k += FIN_U * FIN_L) {
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        au[u] += ldf<SC>(part + (int64_t)(k + u * FIN_L) * 2 * C + c);
        bu[u] += ldf<SC>(part + (int64_t)(k + u * FIN_L) * 2 * C + C + c);
      }
    }
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) {
      const int kk = k + u * FIN_L;
      if (kk < slabs) {
        au[u] += ldf<SC>(part + (int64_t)kk * 2 * C + c);
        bu[u] += ldf<SC>(part + (int64_t)kk * 2 * C + C + c);
      }
    }
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) {
      a += au[u];
      b += bu[u];
    }
  }
  sa[ln][cl] = a;
  sb[ln][cl] = b;
  __syncthreads();
  if (ln == 0) {
#pragma unroll
    for (int k = 1; k < FIN_L; ++k) {
      a += sa[k][cl];
      b += sb[k][cl];
    }
  }
  __syncthreads();  // sa/sb are reused by the next task of a cooperative block
  *a_out = a;
  *b_out = b;
}

// partials from an earlier kernel (plain loads); ws written for the apply
// stage (SC: read by other blocks of the same kernel)
template <bool SC>
__device__ __forceinline__ void finalize_fwd_task(
    const float* __restrict__ part, int slabs, float* __restrict__ ws, float* mean_out,
    float* invstd_out, float* rmean, float* rvar, int64_t rstat_stride, int64_t M, int C,
    int Cper, float eps, float momentum, int task) {
  float a, b;
  sum_slabs<false>(part, slabs, C, task, &a, &b);
  const int c = task * FIN_C + threadIdx.x;
  if (threadIdx.x >= FIN_C || c >= C) return;
  const float inv_m = 1.f / (float)M;
  const float mu = a * inv_m;
  const float var = fmaxf(b * inv_m - mu * mu, 0.f);
  const float is = rsqrtf(var + eps);
  stf<SC>(ws + c, mu);
  stf<SC>(ws + C + c, is);
  mean_out[c] = mu;
  invstd_out[c] = is;
  const int g = c / Cper, cc = c - g * Cper;
  float* rm = rmean + g * rstat_stride + cc;
  float* rv = rvar + g * rstat_stride + cc;
  const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
  *rm = (1.f - momentum) * *rm + momentum * mu;
  *rv = (1.f - momentum) * *rv + momentum * unb;
}

template <bool SC>
__device__ __forceinline__ void finalize_bwd_task(const float* __restrict__ part, int slabs,
                                                  float* __restrict__ ws, float* dgamma,
                                                  float* dbeta, int64_t gstride, int C, int Cper,
                                                  int task) {
  float a, b;
  sum_slabs<SC>(part, slabs, C, task, &a, &b);
  const int c = task * FIN_C + threadIdx.x;
  if (threadIdx.x >= FIN_C || c >= C) return;
  stf<SC>(ws + c, a);
  stf<SC>(ws + C + c, b);
  const int g = c / Cper, cc = c - g * Cper;
  dgamma[g * gstride + cc] = b;
  dbeta[g * gstride + cc] = a;
}

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_finalize_fwd(
    const float* __restrict__ part, int slabs, float* __restrict__ ws, float* mean_out,
    float* invstd_out, float* rmean, float* rvar, int64_t rstat_stride, int64_t M, int C,
    int Cper, float eps, float momentum) {
  finalize_fwd_task<false>(part, slabs, ws, mean_out, invstd_out, rmean, rvar, rstat_stride, M,
                           C, Cper, eps, momentum, blockIdx.x);
}

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_finalize_bwd(
    const float* __restrict__ part, int slabs, float* __restrict__ ws, float* dgamma,
    float* dbeta, int64_t gstride, int C, int Cper) {
  finalize_bwd_task<false>(part, slabs, ws, dgamma, dbeta, gstride, C, Cper, blockIdx.x);
}

// ---------------------------------------------------------------------------
// stage 3: elementwise apply (scale/shift per channel computed once per thread)
// ---------------------------------------------------------------------------
// MODE 0: train fwd, ws = (mean, invstd); MODE 1: eval fwd from running stats
template <typename T, int MODE, bool SC, int AU = 2, int V = VEC>   // AU: rows in flight per thread
__device__ __forceinline__ void apply_fwd_tile(
    const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
    const float* __restrict__ ws, const float* __restrict__ rmean,
    const float* __restrict__ rvar, int64_t rstat_stride, float eps, const Strided& gamma,
    const Strided& beta, int64_t M, int C, int Cper, int rows_per_slab, int act, const Map& mp,
    int cbk, int slab, uint8_t* __restrict__ mask_out = nullptr) {
  const bool hl = (act >> 8) & 1;          // HL-format output (cer_bn_set_hl_out)
  act &= 0xff;
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = cbk * mp.cb + tc * V;
  if (c0 >= C || tr >= mp.tr_n) return;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  float mu[VEC], is[VEC], sc[VEC], sh[VEC];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    if (MODE == 0) {
      mu[i] = ldf<SC>(ws + c0 + i);
      is[i] = ldf<SC>(ws + C + c0 + i);
    } else {
      mu[i] = rmean[g * rstat_stride + cc + i];
      is[i] = rsqrtf(rvar[g * rstat_stride + cc + i] + eps);
    }
  }
  bn_scale_shift<T, V>(gamma, beta, g, cc, mu, is, sc, sh);
  const int64_t r0 = (int64_t)slab * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float v[AU][VEC], rv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        ldv<V>(x + rr * C + c0, v[u]);
        if (res) ldv<V>(res + rr * C + c0, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr >= r1) continue;
      float o[VEC];
#pragma unroll
      for (int i = 0; i < V; ++i)
        o[i] = act_fwd(v[u][i] * sc[i] + sh[i] + (res ? rv[u][i] : 0.f), act);
      if constexpr (V == VEC) {
        if (hl)
          st8_hl(y + rr * C + c0, o);
        else
          st8(y + rr * C + c0, o);
        if (mask_out) mask_out[rr * (C / VEC) + (c0 >> 3)] = (uint8_t)act_bits8(o, act);
      } else {
        stv<V>(y + rr * C + c0, o);       // ragged widths: never HL / mask (host-gated)
      }
    }
  }
}

template <typename T, int MODE, int AU = 2, int V = VEC>
__global__ __launch_bounds__(BN_T) void bn_apply_fwd(
    const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
    const float* __restrict__ ws, const float* __restrict__ rmean,
    const float* __restrict__ rvar, int64_t rstat_stride, float eps, Strided gamma,
    Strided beta, int64_t M, int C, int Cper, int rows_per_slab, int act, Map mp,
    uint8_t* __restrict__ mask_out = nullptr) {
  apply_fwd_tile<T, MODE, false, AU, V>(x, res, y, ws, rmean, rvar, rstat_stride, eps, gamma, beta, M, C,
                              Cper, rows_per_slab, act, mp, blockIdx.x, blockIdx.y, mask_out);
}

template <typename T, bool SC, int YM = YM_Y, int AU = 2, int V = VEC>
__device__ __forceinline__ void apply_bwd_tile(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ ws,
    const Strided& gamma, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C,
    int Cper, int rows_per_slab, int act, const Map& mp, int cbk, int slab,
    const Strided& beta = Strided{nullptr, 0}) {
  const bool hl = (act >> 8) & 1;          // HL-format output (cer_bn_set_hl_out)
  act &= 0xff;
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = cbk * mp.cb + tc * V;
  if (c0 >= C || tr >= mp.tr_n) return;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  float ga[VEC], mu[VEC], is[VEC], k1[VEC], k2[VEC], sdz[VEC], sc[VEC], sh[VEC];
  ldv<V>((const T*)gamma.p + g * gamma.stride + cc, ga);
  const float inv_m = 1.f / (float)M;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    mu[i] = mean[c0 + i];
    is[i] = invstd[c0 + i];
    k1[i] = ga[i] * is[i];
    k2[i] = ldf<SC>(ws + C + c0 + i) * inv_m;
    sdz[i] = ldf<SC>(ws + c0 + i) * inv_m;
  }
  if (YM == YM_Z) bn_scale_shift<T, V>(gamma, beta, g, cc, mu, is, sc, sh);
  const int64_t r0 = (int64_t)slab * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float d[AU][VEC], xv[AU][VEC], yv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        ldv<V>(dy + rr * C + c0, d[u]);
        ldv<V>(x + rr * C + c0, xv[u]);
        if (YM == YM_Y) ldv<V>(y + rr * C + c0, yv[u]);
        if constexpr (YM == YM_M)
          mask_to_y8(reinterpret_cast<const uint8_t*>(y) + rr * (C / 8), c0, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr >= r1) continue;
      float o[VEC], dz[VEC];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        dz[i] = dz_of<YM>(d[u][i], yv[u][i], xv[u][i], sc[i], sh[i], act);
        const float xh = (xv[u][i] - mu[i]) * is[i];
        o[i] = k1[i] * (dz[i] - sdz[i] - xh * k2[i]);
      }
      if constexpr (V == VEC) {
        if (hl)
          st8_hl(dx + rr * C + c0, o);
        else
          st8(dx + rr * C + c0, o);
      } else {
        stv<V>(dx + rr * C + c0, o);      // ragged widths: never HL (host-gated)
      }
      if (dres) stv<V>(dres + rr * C + c0, dz);
    }
  }
}

template <typename T, int YM, int AU = 2, int V = VEC>
__global__ __launch_bounds__(BN_T) void bn_apply_bwd(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ ws,
    Strided gamma, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C,
    int Cper, int rows_per_slab, int act, Map mp, Strided beta) {
  apply_bwd_tile<T, false, YM, AU, V>(dy, x, y, mean, invstd, ws, gamma, dx, dres, M, C, Cper,
                            rows_per_slab, act, mp, blockIdx.x, blockIdx.y, beta);
}

// ---------------------------------------------------------------------------
// finalize folded into the apply (few slabs)
// ---------------------------------------------------------------------------
// When a layer has at most g_fold_max row slabs of partials (the small late
// stages of a one-config step), every apply block reduces the partials of its
// own channel block itself instead of waiting for a separate finalize launch:
// one launch per layer and direction fewer, at the price of re-reading
// nslab x 2 x (channels of the block) floats per block from L2.  All blocks
// sum in the same order, so they agree bit for bit (the order differs from
// bn_finalize_*; results match it to fp32 rounding).  Returns the block's
// (a, b) sums for this thread's 8 channels.
__device__ __forceinline__ void fold_partials(const float* __restrict__ part, int nslab, int C,
                                              const Map& mp, int cbk, float* red, float* a8,
                                              float* b8) {
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = cbk * mp.cb + tc * VEC;
  float a[VEC] = {0, 0, 0, 0, 0, 0, 0, 0}, b[VEC] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < C && tr < mp.tr_n) {
    // FU slabs' loads issued before any add (the partials were just written
    // by other CUs: each load is an L2/MALL round trip)
    constexpr int FU = 4;
    for (int sl0 = tr; sl0 < nslab; sl0 += FU * mp.tr_n) {
      float4 a0[FU], a1[FU], b0[FU], b1[FU];
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        const int sl = sl0 + u * mp.tr_n;
        if (sl < nslab) {
          const float4* pa = reinterpret_cast<const float4*>(part + (int64_t)sl * 2 * C + c0);
          const float4* pb = reinterpret_cast<const float4*>(part + (int64_t)sl * 2 * C + C + c0);
          a0[u] = pa[0]; a1[u] = pa[1]; b0[u] = pb[0]; b1[u] = pb[1];
        } else {
          a0[u] = a1[u] = b0[u] = b1[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int u = 0; u < FU; ++u) {
        a[0] += a0[u].x; a[1] += a0[u].y; a[2] += a0[u].z; a[3] += a0[u].w;
        a[4] += a1[u].x; a[5] += a1[u].y; a[6] += a1[u].z; a[7] += a1[u].w;
        b[0] += b0[u].x; b[1] += b0[u].y; b[2] += b0[u].z; b[3] += b0[u].w;
        b[4] += b1[u].x; b[5] += b1[u].y; b[6] += b1[u].z; b[7] += b1[u].w;
      }
    }
  }
  float* rs = red;
  float* rq = red + BN_T * VEC;
  if (tr < mp.tr_n) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      rs[tr * mp.cb + tc * VEC + i] = a[i];
      rq[tr * mp.cb + tc * VEC + i] = b[i];
    }
  }
  __syncthreads();
  float* fin = red + 2 * BN_T * VEC;          // [2][cb]
  for (int cl = threadIdx.x; cl < mp.cb; cl += BN_T) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < mp.tr_n; ++k) {
      sa += rs[k * mp.cb + cl];
      sb += rq[k * mp.cb + cl];
    }
    fin[cl] = sa;
    fin[mp.cb + cl] = sb;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    a8[i] = fin[tc * VEC + i];
    b8[i] = fin[mp.cb + tc * VEC + i];
  }
}

// fp64 slabs (conv.hip SLAB_F64: a few atomic-accumulated slabs [n][2][C]
// of doubles, exact sums): every block sums its channels' n slabs in fp64,
// one lane row per channel vector, and rounds once
constexpr int SLAB_F64 = 1 << 24;

__device__ __forceinline__ void fold_partials_f64(const double* __restrict__ part, int nslab, int C,
                                                  const Map& mp, int cbk, float* red, float* a8,
                                                  float* b8) {
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = cbk * mp.cb + tc * VEC;
  float* fin = red;                              // [2][cb]
  if (tr == 0 && c0 < C) {
    double a[VEC], b[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) a[i] = b[i] = 0.0;
    for (int sl = 0; sl < nslab; ++sl) {
      const double* pa = part + (int64_t)sl * 2 * C + c0;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        a[i] += pa[i];
        b[i] += pa[C + i];
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      fin[tc * VEC + i] = (float)a[i];
      fin[mp.cb + tc * VEC + i] = (float)b[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    a8[i] = fin[tc * VEC + i];
    b8[i] = fin[mp.cb + tc * VEC + i];
  }
}

// either slab format (nslab carries SLAB_F64 for the fp64 one)
__device__ __forceinline__ void fold_any(const float* __restrict__ part, int nslab, int C,
                                         const Map& mp, int cbk, float* red, float* a8, float* b8) {
  if (nslab & SLAB_F64)
    fold_partials_f64(reinterpret_cast<const double*>(part), nslab & (SLAB_F64 - 1), C, mp, cbk,
                      red, a8, b8);
  else
    fold_partials(part, nslab, C, mp, cbk, red, a8, b8);
}

constexpr int FOLD_LDS = 2 * BN_T * VEC + 2 * 32 * VEC;   // partial tree + [2][cb], cb <= 256

template <typename T>
__global__ __launch_bounds__(BN_T) void bn_apply_fwd_fold(
    const float* __restrict__ part, int nslab, float* mean_out, float* invstd_out, float* rmean,
    float* rvar, int64_t rstat_stride, float eps, float momentum, const T* __restrict__ x,
    const T* __restrict__ res, T* __restrict__ y, Strided gamma, Strided beta,
    int64_t M, int C, int Cper, int rows_per_slab, int act, Map mp,
    uint8_t* __restrict__ mask_out) {
  const bool hl = (act >> 8) & 1;          // HL-format output (cer_bn_set_hl_out)
  act &= 0xff;
  __shared__ float red[FOLD_LDS];
  float a[VEC], b[VEC];
  fold_any(part, nslab, C, mp, blockIdx.x, red, a, b);
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = blockIdx.x * mp.cb + tc * VEC;
  if (c0 >= C || tr >= mp.tr_n) return;
  const float inv_m = 1.f / (float)M;
  float mu[VEC], is[VEC], var[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    mu[i] = a[i] * inv_m;
    var[i] = fmaxf(b[i] * inv_m - mu[i] * mu[i], 0.f);
    is[i] = rsqrtf(var[i] + eps);
  }
  const int g = c0 / Cper, cc = c0 - g * Cper;
  if (blockIdx.y == 0 && tr == 0) {          // one writer per channel
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      mean_out[c0 + i] = mu[i];
      invstd_out[c0 + i] = is[i];
      float* rm = rmean + g * rstat_stride + cc + i;
      float* rv = rvar + g * rstat_stride + cc + i;
      const float unb = M > 1 ? var[i] * (float)M / (float)(M - 1) : var[i];
      *rm = (1.f - momentum) * *rm + momentum * mu[i];
      *rv = (1.f - momentum) * *rv + momentum * unb;
    }
  }
  float sc[VEC], sh[VEC];
  bn_scale_shift<T>(gamma, beta, g, cc, mu, is, sc, sh);
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  constexpr int AU = 2;
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float v[AU][VEC], rv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        ld8(x + rr * C + c0, v[u]);
        if (res) ld8(res + rr * C + c0, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr >= r1) continue;
      float o[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i)
        o[i] = act_fwd(v[u][i] * sc[i] + sh[i] + (res ? rv[u][i] : 0.f), act);
      if (hl)
        st8_hl(y + rr * C + c0, o);
      else
        st8(y + rr * C + c0, o);
      if (mask_out) mask_out[rr * (C / VEC) + (c0 >> 3)] = (uint8_t)act_bits8(o, act);
    }
  }
}

template <typename T, int YM>
__global__ __launch_bounds__(BN_T) void bn_apply_bwd_fold(
    const float* __restrict__ part, int nslab, float* dgamma, float* dbeta, int64_t gstride,
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, Strided gamma,
    Strided beta, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C, int Cper,
    int rows_per_slab, int act, Map mp) {
  const bool hl = (act >> 8) & 1;          // HL-format output (cer_bn_set_hl_out)
  act &= 0xff;
  __shared__ float red[FOLD_LDS];
  float a[VEC], b[VEC];
  fold_any(part, nslab, C, mp, blockIdx.x, red, a, b);
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = blockIdx.x * mp.cb + tc * VEC;
  if (c0 >= C || tr >= mp.tr_n) return;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  if (blockIdx.y == 0 && tr == 0) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      dgamma[g * gstride + cc + i] = b[i];
      dbeta[g * gstride + cc + i] = a[i];
    }
  }
  float ga[VEC], mu[VEC], is[VEC], k1[VEC], k2[VEC], sdz[VEC], sc[VEC], sh[VEC];
  ld8((const T*)gamma.p + g * gamma.stride + cc, ga);
  const float inv_m = 1.f / (float)M;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    mu[i] = mean[c0 + i];
    is[i] = invstd[c0 + i];
    k1[i] = ga[i] * is[i];
    k2[i] = b[i] * inv_m;
    sdz[i] = a[i] * inv_m;
  }
  if (YM == YM_Z) bn_scale_shift<T>(gamma, beta, g, cc, mu, is, sc, sh);
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  constexpr int AU = 2;
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float d[AU][VEC], xv[AU][VEC], yv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        ld8(dy + rr * C + c0, d[u]);
        ld8(x + rr * C + c0, xv[u]);
        if (YM == YM_Y) ld8(y + rr * C + c0, yv[u]);
        if constexpr (YM == YM_M)
          mask_to_y8(reinterpret_cast<const uint8_t*>(y) + rr * (C / 8), c0, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr >= r1) continue;
      float o[VEC], dz[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        dz[i] = dz_of<YM>(d[u][i], yv[u][i], xv[u][i], sc[i], sh[i], act);
        const float xh = (xv[u][i] - mu[i]) * is[i];
        o[i] = k1[i] * (dz[i] - sdz[i] - xh * k2[i]);
      }
      if (hl)
        st8_hl(dx + rr * C + c0, o);
      else
        st8(dx + rr * C + c0, o);
      if (dres) st8(dres + rr * C + c0, dz);
    }
  }
}

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
constexpr int RED_TARGET = 512, RED_MIN_ROWS = 64;
constexpr int APPLY_TARGET = 2048, APPLY_MIN_ROWS = 16;

// finalize folded into the apply when a layer has at most this many slabs
// (CER_BN_FOLD, default 64; 0 = always launch the finalize kernel)
static int g_fold_max = -1;
static int fold_max() {
  if (g_fold_max < 0) {
    const char* e = getenv("CER_BN_FOLD");
    g_fold_max = e ? atoi(e) : 64;
  }
  return g_fold_max;
}
CER_API void cer_bn_set_fold(int max_slabs) { g_fold_max = max_slabs; }

// minimum rows per block of a folded apply: the plain apply grid's 16 (fatter
// blocks re-read the partials less but measured flat: r2_ab_kernel_knobs.md;
// so did 4 instead of 2 rows in flight per thread, the apply kernels' AU)
constexpr int FOLD_ROWS = 16;

// ReLU mask recomputed from the BN input in backward (YM_Z); 0 = always read y
static int g_zmask = 1;
CER_API void cer_bn_set_zmask(int on) { g_zmask = on; }

// HL-format output of the NEXT training-mode apply launches (fwd y / bwd dx,
// fp32 only; st8_hl): the value's only consumers are fp32 3-pass conv
// operand loads (conv.hip take_hi_lo), which read the pre-split pair instead
// of splitting the fp32 value -- bit-identical operands, no split VALU
static int g_bn_hl = 0;
CER_API void cer_bn_set_hl_out(int on) { g_bn_hl = on ? 1 : 0; }

// mask source of a BN backward (also used by the dgrad-epilogue statistics)
// residual-join activation masks as bits (YM_M): the NEXT training-mode
// forward apply also writes its mask to ``mask`` ([M][C / 8] bytes; null
// = off); cer_bn_set_mask_in(1): backward launches whose mode would be YM_Y
// read such a mask through their y argument instead
static uint8_t* g_mask_out = nullptr;
static int g_mask_in = 0;
CER_API void cer_bn_set_mask_out(void* mask) { g_mask_out = reinterpret_cast<uint8_t*>(mask); }
CER_API void cer_bn_set_mask_in(int on) { g_mask_in = on ? 1 : 0; }

// the NEXT backward launches of a residual-join BN leave dres unwritten
// (cer_bn_set_dres_skip; ops.nn.MaskedGrad: the consumer of the residual's
// gradient recomputes dres = mask * dy in its dgrad epilogue instead of
// reading a stored copy); aligned widths only
static int g_dres_skip = 0;
CER_API void cer_bn_set_dres_skip(int on) { g_dres_skip = on ? 1 : 0; }

// The NEXT backward launches that compute their own partials (no dgrad-epilogue
// link) may accumulate them by fp64 atomics into n slabs of their part buffer
// (zeroed by the caller, n * 2 * C doubles), so the apply folds the finalize
// for any layer size -- the conv epilogues' slab format (SLAB_F64) -- instead
// of a separate finalize launch for layers with more than fold_max() row
// slabs.  0 = off (one fp32 slab per row slab).
static int g_bwd_f64 = 0;
CER_API void cer_bn_set_bwd_f64(int nslabs) { g_bwd_f64 = nslabs > 0 ? nslabs : 0; }

// floats of zeroed buffer a backward launch of this size would accumulate its
// partials in with ``nslabs`` fp64 slabs (cer_bn_set_bwd_f64), or 0 when it
// keeps the fp32 slab format (few row slabs, unaligned widths)
CER_API int64_t cer_bn_bwd_f64_floats(int64_t M, int C, int Cper, int nslabs) {
  if (nslabs <= 0 || C % VEC || Cper % VEC) return 0;
  const Map mp = make_map(C);
  dim3 rg;
  int rrows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
  if ((int)rg.y <= fold_max()) return 0;
  return (int64_t)nslabs * 2 * C * 2;
}

int bn_mask_mode(int act, int has_res) {
  if (act == 0) return YM_NONE;
  if (act == 1 && !has_res && g_zmask) return YM_Z;
  return g_mask_in ? YM_M : YM_Y;
}

// floats of scratch the partials need (part[slabs][2][C])
CER_API int64_t cer_bn_part_floats(int64_t M, int C) {
  int64_t n = 0;
  for (int V : {VEC, 1}) {            // aligned and ragged (V = 1) grids
    const Map mp = make_map(C, V);
    dim3 g;
    int rows;
    make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &g, &rows);
    n = n > (int64_t)g.y * 2 * C ? n : (int64_t)g.y * 2 * C;
  }
  return n;
}

// ---- ragged channel counts (C or Cper not a multiple of 8): one channel per
// thread (V = 1), statistics by partials -> finalize -> apply, no fold, no
// HL output (NASNet-Mobile's 11 / 22 / 44-filter layers; ops.nn gates HL on
// 8-aligned widths only)
template <typename T>
static int bn_fwd_train_ragged(const T* x, const T* res, T* y, const T* gamma,
                               int64_t gamma_stride, const T* beta, int64_t beta_stride,
                               float* rmean, float* rvar, int64_t rstat_stride, float* mean_out,
                               float* invstd_out, float* ws, float* part, int64_t M, int C,
                               int Cper, float eps, float momentum, int act, hipStream_t stream) {
  if ((act >> 8) || g_mask_out) return (int)hipErrorInvalidValue;  // HL / bit masks: aligned only
  const Map mp = make_map(C, 1);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  bn_partials<T, 0, YM_Y, 1><<<rg, BN_T, 0, stream>>>(x, nullptr, nullptr, nullptr, nullptr,
                                                      part, M, C, rrows, 0, mp);
  bn_finalize_fwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(
      part, (int)rg.y, ws, mean_out, invstd_out, rmean, rvar, rstat_stride, M, C, Cper, eps,
      momentum);
  bn_apply_fwd<T, 0, 2, 1><<<ag, BN_T, 0, stream>>>(x, res, y, ws, nullptr, nullptr, 0, 0.f,
                                                    Strided{gamma, gamma_stride},
                                                    Strided{beta, beta_stride}, M, C, Cper,
                                                    arows, act, mp);
  return (int)hipGetLastError();
}

template <typename T>
static int bn_bwd_ragged(const T* dy, const T* x, const T* y, const float* mean,
                         const float* invstd, const T* gamma, int64_t gamma_stride,
                         const T* beta, int64_t beta_stride, float* dgamma, float* dbeta,
                         int64_t grad_stride, T* dx, T* dres, float* ws, float* part, int64_t M,
                         int C, int Cper, int act, hipStream_t stream) {
  if (act >> 8 || g_dres_skip) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C, 1);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  const int ym = bn_mask_mode(act, dres != nullptr);
  if (ym == YM_M) return (int)hipErrorInvalidValue;     // bit masks: 8-aligned widths only
  const Strided gs{gamma, gamma_stride}, bs{beta, beta_stride};
  if (ym == YM_NONE)
    bn_partials<T, 1, YM_NONE, 1><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C,
                                                          rrows, act, mp, gs, bs, Cper);
  else if (ym == YM_Z)
    bn_partials<T, 1, YM_Z, 1><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C,
                                                       rrows, act, mp, gs, bs, Cper);
  else
    bn_partials<T, 1, YM_Y, 1><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C,
                                                       rrows, act, mp, gs, bs, Cper);
  bn_finalize_bwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(part, (int)rg.y, ws, dgamma,
                                                                    dbeta, grad_stride, C, Cper);
  if (ym == YM_NONE)
    bn_apply_bwd<T, YM_NONE, 2, 1><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx,
                                                           dres, M, C, Cper, arows, act, mp, bs);
  else if (ym == YM_Z)
    bn_apply_bwd<T, YM_Z, 2, 1><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres,
                                                        M, C, Cper, arows, act, mp, bs);
  else
    bn_apply_bwd<T, YM_Y, 2, 1><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres,
                                                        M, C, Cper, arows, act, mp, bs);
  return (int)hipGetLastError();
}

template <typename T>
static int bn_fwd_train_impl(const T* x, const T* res, T* y, const T* gamma,
                             int64_t gamma_stride, const T* beta, int64_t beta_stride,
                             float* rmean, float* rvar, int64_t rstat_stride, float* mean_out,
                             float* invstd_out, float* ws, float* part, int nslab, int64_t M,
                             int C, int Cper, float eps, float momentum, int act,
                             hipStream_t stream) {
  const int act_k = act | (sizeof(T) == 4 ? g_bn_hl << 8 : 0);   // + HL output bit
  if (C % VEC || Cper % VEC) {
    if (nslab > 0) return (int)hipErrorInvalidValue;    // conv-epilogue partials: aligned only
    return bn_fwd_train_ragged(x, res, y, gamma, gamma_stride, beta, beta_stride, rmean, rvar,
                               rstat_stride, mean_out, invstd_out, ws, part, M, C, Cper, eps,
                               momentum, act_k, stream);
  }
  const Map mp = make_map(C);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  if (nslab <= 0) {  // statistics not produced upstream: reduce x here
    make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
    bn_partials<T, 0><<<rg, BN_T, 0, stream>>>(x, nullptr, nullptr, nullptr, nullptr, part, M, C,
                                            rrows, 0, mp);
    nslab = (int)rg.y;
  }
  if ((nslab & SLAB_F64) || nslab <= fold_max()) {     // fp64 slabs: always few
    dim3 fg;
    int frows;
    make_grid(M, C, mp, APPLY_TARGET, FOLD_ROWS, &fg, &frows);
    bn_apply_fwd_fold<T><<<fg, BN_T, 0, stream>>>(part, nslab, mean_out, invstd_out, rmean, rvar,
                                               rstat_stride, eps, momentum, x, res, y,
                                               Strided{gamma, gamma_stride},
                                               Strided{beta, beta_stride}, M, C, Cper, frows, act_k,
                                               mp, g_mask_out);
    return (int)hipGetLastError();
  }
  bn_finalize_fwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(part, nslab, ws, mean_out,
                                                          invstd_out, rmean, rvar, rstat_stride,
                                                          M, C, Cper, eps, momentum);
  bn_apply_fwd<T, 0><<<ag, BN_T, 0, stream>>>(x, res, y, ws, nullptr, nullptr, 0, 0.f,
                                           Strided{gamma, gamma_stride},
                                           Strided{beta, beta_stride}, M, C, Cper, arows, act_k,
                                           mp, g_mask_out);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_bn_fwd_train_t(const T* x, const T* res, T* y, const T* gamma,
                             int64_t gamma_stride, const T* beta, int64_t beta_stride,
                             float* rmean, float* rvar, int64_t rstat_stride, float* mean_out,
                             float* invstd_out, float* ws, float* part, int64_t M, int C,
                             int Cper, float eps, float momentum, int act, hipStream_t stream) {
  return bn_fwd_train_impl(x, res, y, gamma, gamma_stride, beta, beta_stride, rmean, rvar,
                           rstat_stride, mean_out, invstd_out, ws, part, 0, M, C, Cper, eps,
                           momentum, act, stream);
}

// same, with the per-slab (sum, sum^2) partials already produced by the
// producing convolution's epilogue (cer_conv_fwd_stats)
template <typename T>
static int cer_bn_fwd_train_part_t(const T* x, const T* res, T* y,
                                  const T* gamma, int64_t gamma_stride, const T* beta,
                                  int64_t beta_stride, float* rmean, float* rvar,
                                  int64_t rstat_stride, float* mean_out, float* invstd_out,
                                  float* ws, float* part, int nslab, int64_t M, int C, int Cper,
                                  float eps, float momentum, int act, hipStream_t stream) {
  if (nslab <= 0) return (int)hipErrorInvalidValue;
  return bn_fwd_train_impl(x, res, y, gamma, gamma_stride, beta, beta_stride, rmean, rvar,
                           rstat_stride, mean_out, invstd_out, ws, part, nslab, M, C, Cper, eps,
                           momentum, act, stream);
}

// apply only: y = act(xhat * gamma + beta (+ res)) with ws = (mean, invstd)
// already produced (conv-fused statistics, cer_conv_fwd_bnstat)
template <typename T>
static int cer_bn_apply_fwd_t(const T* x, const T* res, T* y, const float* ws,
                             const T* gamma, int64_t gamma_stride, const T* beta,
                             int64_t beta_stride, int64_t M, int C, int Cper, int act,
                             hipStream_t stream) {
  const int act_k = act | (sizeof(T) == 4 ? g_bn_hl << 8 : 0);   // + HL output bit
  if (C % VEC || Cper % VEC) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C);
  dim3 ag;
  int arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  bn_apply_fwd<T, 0><<<ag, BN_T, 0, stream>>>(x, res, y, ws, nullptr, nullptr, 0, 0.f,
                                           Strided{gamma, gamma_stride},
                                           Strided{beta, beta_stride}, M, C, Cper, arows, act_k,
                                           mp);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_bn_fwd_eval_t(const T* x, const T* res, T* y, const T* gamma,
                            int64_t gamma_stride, const T* beta, int64_t beta_stride,
                            const float* rmean, const float* rvar, int64_t rstat_stride,
                            int64_t M, int C, int Cper, float eps, int act, hipStream_t stream) {
  const bool rag = (C % VEC) || (Cper % VEC);
  const Map mp = make_map(C, rag ? 1 : VEC);
  dim3 ag;
  int arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  if (rag)
    bn_apply_fwd<T, 1, 2, 1><<<ag, BN_T, 0, stream>>>(x, res, y, nullptr, rmean, rvar,
                                                      rstat_stride, eps,
                                                      Strided{gamma, gamma_stride},
                                                      Strided{beta, beta_stride}, M, C, Cper,
                                                      arows, act, mp);
  else
    bn_apply_fwd<T, 1><<<ag, BN_T, 0, stream>>>(x, res, y, nullptr, rmean, rvar, rstat_stride,
                                             eps, Strided{gamma, gamma_stride},
                                             Strided{beta, beta_stride}, M, C, Cper, arows, act,
                                             mp);
  return (int)hipGetLastError();
}

// pre_nslab > 0: part already holds pre_nslab partials (computed in the
// epilogue of the dgrad that produced dy): skip the partials pass
template <typename T>
static int bn_bwd_impl(const T* dy, const T* x, const T* y, const float* mean,
                       const float* invstd, const T* gamma, int64_t gamma_stride,
                       const T* beta, int64_t beta_stride, float* dgamma, float* dbeta,
                       int64_t grad_stride, T* dx, T* dres, float* ws, float* part,
                       int pre_nslab, int64_t M, int C, int Cper, int act, hipStream_t stream) {
  const int act_k = act | (sizeof(T) == 4 ? g_bn_hl << 8 : 0);   // + HL output bit
  if (C % VEC || Cper % VEC) {
    if (pre_nslab > 0) return (int)hipErrorInvalidValue;  // dgrad-epilogue partials: aligned only
    return bn_bwd_ragged(dy, x, y, mean, invstd, gamma, gamma_stride, beta, beta_stride, dgamma,
                         dbeta, grad_stride, dx, dres, ws, part, M, C, Cper, act_k, stream);
  }
  const Map mp = make_map(C);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  // mask source: none / y / recomputed from x (see the header); a residual
  // join's mask depends on the residual, so it needs y
  const int ym = bn_mask_mode(act, dres != nullptr || g_dres_skip);
  if (g_dres_skip) dres = nullptr;
  const Strided gs{gamma, gamma_stride}, bs{beta, beta_stride};
  const int f64 = pre_nslab <= 0 && (int)rg.y > fold_max() ? g_bwd_f64 : 0;
  const int nslab = pre_nslab > 0 ? pre_nslab
                                  : f64 ? ((int)rg.y < f64 ? (int)rg.y : f64) | SLAB_F64
                                        : (int)rg.y;
  if (pre_nslab <= 0) {
    if (ym == YM_NONE)
      bn_partials<T, 1, YM_NONE><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C,
                                                       rrows, act, mp, gs, bs, Cper, f64);
    else if (ym == YM_Z)
      bn_partials<T, 1, YM_Z><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C, rrows,
                                                    act, mp, gs, bs, Cper, f64);
    else if (ym == YM_M)
      bn_partials<T, 1, YM_M><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C, rrows,
                                                    act, mp, gs, bs, Cper, f64);
    else
      bn_partials<T, 1, YM_Y><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C, rrows,
                                                    act, mp, gs, bs, Cper, f64);
  }
  if ((nslab & SLAB_F64) || nslab <= fold_max()) {
    dim3 fg;
    int frows;
    make_grid(M, C, mp, APPLY_TARGET, FOLD_ROWS, &fg, &frows);
    if (ym == YM_NONE)
      bn_apply_bwd_fold<T, YM_NONE><<<fg, BN_T, 0, stream>>>(part, nslab, dgamma, dbeta,
                                                          grad_stride, dy, x, y, mean, invstd, gs,
                                                          bs, dx, dres, M, C, Cper, frows, act_k,
                                                          mp);
    else if (ym == YM_Z)
      bn_apply_bwd_fold<T, YM_Z><<<fg, BN_T, 0, stream>>>(part, nslab, dgamma, dbeta,
                                                       grad_stride, dy, x, y, mean, invstd, gs, bs,
                                                       dx, dres, M, C, Cper, frows, act_k, mp);
    else if (ym == YM_M)
      bn_apply_bwd_fold<T, YM_M><<<fg, BN_T, 0, stream>>>(part, nslab, dgamma, dbeta,
                                                       grad_stride, dy, x, y, mean, invstd, gs, bs,
                                                       dx, dres, M, C, Cper, frows, act_k, mp);
    else
      bn_apply_bwd_fold<T, YM_Y><<<fg, BN_T, 0, stream>>>(part, nslab, dgamma, dbeta,
                                                       grad_stride, dy, x, y, mean, invstd, gs, bs,
                                                       dx, dres, M, C, Cper, frows, act_k, mp);
    return (int)hipGetLastError();
  }
  bn_finalize_bwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(part, nslab, ws, dgamma, dbeta,
                                                          grad_stride, C, Cper);
  if (ym == YM_NONE) {
    bn_apply_bwd<T, YM_NONE><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres, M,
                                                   C, Cper, arows, act_k, mp, bs);
  } else if (ym == YM_Z) {
    bn_apply_bwd<T, YM_Z><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres, M, C,
                                                Cper, arows, act_k, mp, bs);
  } else if (ym == YM_M) {
    bn_apply_bwd<T, YM_M><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres, M, C,
                                                Cper, arows, act_k, mp, bs);
  } else {
    bn_apply_bwd<T, YM_Y><<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws, gs, dx, dres, M, C,
                                                Cper, arows, act_k, mp, bs);
  }
  return (int)hipGetLastError();
}

template <typename T>
static int cer_bn_bwd_t(const T* dy, const T* x, const T* y, const float* mean,
                       const float* invstd, const T* gamma, int64_t gamma_stride,
                       const T* beta, int64_t beta_stride, float* dgamma, float* dbeta,
                       int64_t grad_stride, T* dx, T* dres, float* ws, float* part,
                       int64_t M, int C, int Cper, int act, hipStream_t stream) {
  return bn_bwd_impl(dy, x, y, mean, invstd, gamma, gamma_stride, beta, beta_stride, dgamma,
                     dbeta, grad_stride, dx, dres, ws, part, 0, M, C, Cper, act, stream);
}

// same, with the nslab (sum dz, sum dz*xhat) partials already in `part`
// (cer_conv_dgrad_bnbwd)
template <typename T>
static int cer_bn_bwd_part_t(const T* dy, const T* x, const T* y,
                            const float* mean, const float* invstd, const T* gamma,
                            int64_t gamma_stride, const T* beta, int64_t beta_stride,
                            float* dgamma, float* dbeta, int64_t grad_stride, T* dx,
                            T* dres, float* ws, float* part, int nslab, int64_t M, int C,
                            int Cper, int act, hipStream_t stream) {
  if (nslab <= 0) return (int)hipErrorInvalidValue;
  return bn_bwd_impl(dy, x, y, mean, invstd, gamma, gamma_stride, beta, beta_stride, dgamma,
                     dbeta, grad_stride, dx, dres, ws, part, nslab, M, C, Cper, act, stream);
}

// C entry points: bf16 (compute mode) and _f32 (reference-precision mode)
// twins of every BatchNorm op, same arguments
#define CER_BN_ENTRY_POINTS(T, SFX)                                                              \
  CER_API int cer_bn_fwd_train##SFX(                                                             \
      const T* x, const T* res, T* y, const T* gamma, int64_t gs, const T* beta, int64_t bs,    \
      float* rmean, float* rvar, int64_t rstride, float* mean_out, float* invstd_out, float* ws, \
      float* part, int64_t M, int C, int Cper, float eps, float momentum, int act,                \
      hipStream_t stream) {                                                                      \
    return cer_bn_fwd_train_t<T>(x, res, y, gamma, gs, beta, bs, rmean, rvar, rstride, mean_out, \
                                 invstd_out, ws, part, M, C, Cper, eps, momentum, act, stream);  \
  }                                                                                              \
  CER_API int cer_bn_fwd_train_part##SFX(                                                        \
      const T* x, const T* res, T* y, const T* gamma, int64_t gs, const T* beta, int64_t bs,    \
      float* rmean, float* rvar, int64_t rstride, float* mean_out, float* invstd_out, float* ws, \
      float* part, int nslab, int64_t M, int C, int Cper, float eps, float momentum, int act,    \
      hipStream_t stream) {                                                                      \
    return cer_bn_fwd_train_part_t<T>(x, res, y, gamma, gs, beta, bs, rmean, rvar, rstride,     \
                                      mean_out, invstd_out, ws, part, nslab, M, C, Cper, eps,    \
                                      momentum, act, stream);                                    \
  }                                                                                              \
  CER_API int cer_bn_apply_fwd##SFX(const T* x, const T* res, T* y, const float* ws,            \
                                    const T* gamma, int64_t gs, const T* beta, int64_t bs,      \
                                    int64_t M, int C, int Cper, int act, hipStream_t stream) {   \
    return cer_bn_apply_fwd_t<T>(x, res, y, ws, gamma, gs, beta, bs, M, C, Cper, act, stream);   \
  }                                                                                              \
  CER_API int cer_bn_fwd_eval##SFX(const T* x, const T* res, T* y, const T* gamma, int64_t gs,  \
                                   const T* beta, int64_t bs, const float* rmean,               \
                                   const float* rvar, int64_t rstride, int64_t M, int C,         \
                                   int Cper, float eps, int act, hipStream_t stream) {          \
    return cer_bn_fwd_eval_t<T>(x, res, y, gamma, gs, beta, bs, rmean, rvar, rstride, M, C,      \
                                Cper, eps, act, stream);                                         \
  }                                                                                              \
  CER_API int cer_bn_bwd##SFX(const T* dy, const T* x, const T* y, const float* mean,           \
                              const float* invstd, const T* gamma, int64_t gs, const T* beta,    \
                              int64_t bs, float* dgamma, float* dbeta, int64_t grad_stride,      \
                              T* dx, T* dres, float* ws, float* part, int64_t M, int C,          \
                              int Cper, int act, hipStream_t stream) {                          \
    return cer_bn_bwd_t<T>(dy, x, y, mean, invstd, gamma, gs, beta, bs, dgamma, dbeta,           \
                           grad_stride, dx, dres, ws, part, M, C, Cper, act, stream);            \
  }                                                                                              \
  CER_API int cer_bn_bwd_part##SFX(const T* dy, const T* x, const T* y, const float* mean,      \
                                   const float* invstd, const T* gamma, int64_t gs,             \
                                   const T* beta, int64_t bs, float* dgamma, float* dbeta,       \
                                   int64_t grad_stride, T* dx, T* dres, float* ws, float* part,  \
                                   int nslab, int64_t M, int C, int Cper, int act,               \
                                   hipStream_t stream) {                                         \
    return cer_bn_bwd_part_t<T>(dy, x, y, mean, invstd, gamma, gs, beta, bs, dgamma, dbeta,      \
                                grad_stride, dx, dres, ws, part, nslab, M, C, Cper, act, stream);\
  }

CER_BN_ENTRY_POINTS(bf16_t, )
CER_BN_ENTRY_POINTS(float, _f32)
