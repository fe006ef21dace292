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
// dres = dz.
#include "common.h"

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

__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
  uint4 u;
  u.x = pack_bf2(v[0], v[1]);
  u.y = pack_bf2(v[2], v[3]);
  u.z = pack_bf2(v[4], v[5]);
  u.w = pack_bf2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

struct Map {
  int tc_n, tr_n, cb;  // threads along channels, row lanes, channels per block
};

static Map make_map(int C) {
  int tc = (C / VEC) < 32 ? (C / VEC) : 32;
  if (tc < 1) tc = 1;
  return Map{tc, BN_T / tc, tc * VEC};
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
// stage 1: per-slab partial sums -> part[slab][2][C]
// ---------------------------------------------------------------------------
template <int MODE>  // 0: (sum x, sum x^2)   1: (sum dz, sum dz*xhat)
__global__ __launch_bounds__(BN_T) void bn_partials(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ part,
    int64_t M, int C, int rows_per_slab, int act, Map mp) {
  __shared__ float red[2 * BN_T * VEC];
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = blockIdx.x * mp.cb + tc * VEC;
  const bool cok = c0 < C;
  float s[VEC] = {0, 0, 0, 0, 0, 0, 0, 0}, q[VEC] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[VEC], is[VEC];
  if (MODE == 1 && cok) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      mu[i] = mean[c0 + i];
      is[i] = invstd[c0 + i];
    }
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
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
          load8(x + rr * C + c0, v[u]);
          if (MODE == 1) {
            load8(dy + rr * C + c0, d[u]);
            load8(y + rr * C + c0, yv[u]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (!ok[u]) continue;
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            s[i] += v[u][i];
            q[i] += v[u][i] * v[u][i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            const float dz = act_bwd(d[u][i], yv[u][i], act);
            s[i] += dz;
            q[i] += dz * (v[u][i] - mu[i]) * is[i];
          }
        }
      }
    }
  }
  float* rs = red;
  float* rq = red + BN_T * VEC;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    rs[tr * mp.cb + tc * VEC + i] = s[i];
    rq[tr * mp.cb + tc * VEC + i] = q[i];
  }
  __syncthreads();
  for (int cl = threadIdx.x; cl < mp.cb; cl += BN_T) {
    const int c = blockIdx.x * mp.cb + cl;
    if (c >= C) continue;
    float a = 0.f, b = 0.f;
    for (int k = 0; k < mp.tr_n; ++k) {
      a += rs[k * mp.cb + cl];
      b += rq[k * mp.cb + cl];
    }
    float* dst = part + (int64_t)blockIdx.y * 2 * C;
    dst[c] = a;
    dst[C + c] = b;
  }
}

// ---------------------------------------------------------------------------
// stage 2: finalize
// ---------------------------------------------------------------------------
// one block = 8 channels x 32 slab lanes; each lane keeps 8 slab loads in
// flight (the partials were just written by other CUs: every round trip is an
// L2/MALL miss, so the reduction is latency-bound), LDS tree
constexpr int FIN_C = 8, FIN_L = 32, FIN_U = 8;

__device__ __forceinline__ void sum_slabs(const float* __restrict__ part, int slabs, int C,
                                          float* a_out, float* b_out) {
  __shared__ float sa[FIN_L][FIN_C], sb[FIN_L][FIN_C];
  const int cl = threadIdx.x % FIN_C, ln = threadIdx.x / FIN_C;
  const int c = blockIdx.x * FIN_C + cl;
  float a = 0.f, b = 0.f;
  if (c < C) {
    float au[FIN_U], bu[FIN_U];
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) au[u] = bu[u] = 0.f;
    int k = ln;
    for (; k + (FIN_U - 1) * FIN_L < slabs; k += FIN_U * FIN_L) {
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) {
        au[u] += part[(int64_t)(k + u * FIN_L) * 2 * C + c];
        bu[u] += part[(int64_t)(k + u * FIN_L) * 2 * C + C + c];
      }
    }
#pragma unroll
    for (int u = 0; u < FIN_U; ++u) {
      const int kk = k + u * FIN_L;
      if (kk < slabs) {
        au[u] += part[(int64_t)kk * 2 * C + c];
        bu[u] += part[(int64_t)kk * 2 * C + C + c];
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
  *a_out = a;
  *b_out = b;
}

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_finalize_fwd(
    const float* __restrict__ part, int slabs, float* __restrict__ ws, float* mean_out,
    float* invstd_out, float* rmean, float* rvar, int64_t rstat_stride, int64_t M, int C,
    int Cper, float eps, float momentum) {
  float a, b;
  sum_slabs(part, slabs, C, &a, &b);
  const int c = blockIdx.x * FIN_C + threadIdx.x;
  if (threadIdx.x >= FIN_C || c >= C) return;
  const float inv_m = 1.f / (float)M;
  const float mu = a * inv_m;
  const float var = fmaxf(b * inv_m - mu * mu, 0.f);
  const float is = rsqrtf(var + eps);
  ws[c] = mu;
  ws[C + c] = is;
  mean_out[c] = mu;
  invstd_out[c] = is;
  const int g = c / Cper, cc = c - g * Cper;
  float* rm = rmean + g * rstat_stride + cc;
  float* rv = rvar + g * rstat_stride + cc;
  const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
  *rm = (1.f - momentum) * *rm + momentum * mu;
  *rv = (1.f - momentum) * *rv + momentum * unb;
}

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_finalize_bwd(
    const float* __restrict__ part, int slabs, float* __restrict__ ws, float* dgamma,
    float* dbeta, int64_t gstride, int C, int Cper) {
  float a, b;
  sum_slabs(part, slabs, C, &a, &b);
  const int c = blockIdx.x * FIN_C + threadIdx.x;
  if (threadIdx.x >= FIN_C || c >= C) return;
  ws[c] = a;
  ws[C + c] = b;
  const int g = c / Cper, cc = c - g * Cper;
  dgamma[g * gstride + cc] = b;
  dbeta[g * gstride + cc] = a;
}

// ---------------------------------------------------------------------------
// stage 3: elementwise apply (scale/shift per channel computed once per thread)
// ---------------------------------------------------------------------------
// MODE 0: train fwd, ws = (mean, invstd); MODE 1: eval fwd from running stats
template <int MODE>
__global__ __launch_bounds__(BN_T) void bn_apply_fwd(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
    const float* __restrict__ ws, const float* __restrict__ rmean,
    const float* __restrict__ rvar, int64_t rstat_stride, float eps, Strided gamma,
    Strided beta, int64_t M, int C, int Cper, int rows_per_slab, int act, Map mp) {
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = blockIdx.x * mp.cb + tc * VEC;
  if (c0 >= C) return;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  float ga[VEC], be[VEC], sc[VEC], sh[VEC];
  load8((const bf16_t*)gamma.p + g * gamma.stride + cc, ga);
  load8((const bf16_t*)beta.p + g * beta.stride + cc, be);
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    float mu, is;
    if (MODE == 0) {
      mu = ws[c0 + i];
      is = ws[C + c0 + i];
    } else {
      mu = rmean[g * rstat_stride + cc + i];
      is = rsqrtf(rvar[g * rstat_stride + cc + i] + eps);
    }
    sc[i] = is * ga[i];
    sh[i] = be[i] - mu * sc[i];
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  constexpr int AU = 2;     // rows in flight per thread
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float v[AU][VEC], rv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        load8(x + rr * C + c0, v[u]);
        if (res) load8(res + rr * C + c0, rv[u]);
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
      store8(y + rr * C + c0, o);
    }
  }
}

__global__ __launch_bounds__(BN_T) void bn_apply_bwd(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ ws,
    Strided gamma, bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, int64_t M, int C,
    int Cper, int rows_per_slab, int act, Map mp) {
  const int tc = threadIdx.x % mp.tc_n, tr = threadIdx.x / mp.tc_n;
  const int c0 = blockIdx.x * mp.cb + tc * VEC;
  if (c0 >= C) return;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  float ga[VEC], mu[VEC], is[VEC], k1[VEC], k2[VEC], sdz[VEC];
  load8((const bf16_t*)gamma.p + g * gamma.stride + cc, ga);
  const float inv_m = 1.f / (float)M;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    mu[i] = mean[c0 + i];
    is[i] = invstd[c0 + i];
    k1[i] = ga[i] * is[i];
    k2[i] = ws[C + c0 + i] * inv_m;
    sdz[i] = ws[c0 + i] * inv_m;
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  const int64_t r1 = min(M, r0 + rows_per_slab);
  constexpr int AU = 2;     // rows in flight per thread
  for (int64_t r = r0 + tr; r < r1; r += AU * mp.tr_n) {
    float d[AU][VEC], xv[AU][VEC], yv[AU][VEC];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr < r1) {
        load8(dy + rr * C + c0, d[u]);
        load8(x + rr * C + c0, xv[u]);
        load8(y + rr * C + c0, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t rr = r + (int64_t)u * mp.tr_n;
      if (rr >= r1) continue;
      float o[VEC], dz[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        dz[i] = act_bwd(d[u][i], yv[u][i], act);
        const float xh = (xv[u][i] - mu[i]) * is[i];
        o[i] = k1[i] * (dz[i] - sdz[i] - xh * k2[i]);
      }
      store8(dx + rr * C + c0, o);
      if (dres) store8(dres + rr * C + c0, dz);
    }
  }
}

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
constexpr int RED_TARGET = 512, RED_MIN_ROWS = 64;
constexpr int APPLY_TARGET = 2048, APPLY_MIN_ROWS = 16;

// floats of scratch the partials need (part[slabs][2][C])
CER_API int64_t cer_bn_part_floats(int64_t M, int C) {
  Map mp = make_map(C);
  dim3 g;
  int rows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &g, &rows);
  return (int64_t)g.y * 2 * C;
}

static int bn_fwd_train_impl(const bf16_t* x, const bf16_t* res, bf16_t* y, const bf16_t* gamma,
                             int64_t gamma_stride, const bf16_t* beta, int64_t beta_stride,
                             float* rmean, float* rvar, int64_t rstat_stride, float* mean_out,
                             float* invstd_out, float* ws, float* part, int nslab, int64_t M,
                             int C, int Cper, float eps, float momentum, int act,
                             hipStream_t stream) {
  if (C % VEC || Cper % VEC) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  if (nslab <= 0) {  // statistics not produced upstream: reduce x here
    make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
    bn_partials<0><<<rg, BN_T, 0, stream>>>(x, nullptr, nullptr, nullptr, nullptr, part, M, C,
                                            rrows, 0, mp);
    nslab = (int)rg.y;
  }
  bn_finalize_fwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(part, nslab, ws, mean_out,
                                                          invstd_out, rmean, rvar, rstat_stride,
                                                          M, C, Cper, eps, momentum);
  bn_apply_fwd<0><<<ag, BN_T, 0, stream>>>(x, res, y, ws, nullptr, nullptr, 0, 0.f,
                                           Strided{gamma, gamma_stride},
                                           Strided{beta, beta_stride}, M, C, Cper, arows, act, mp);
  return (int)hipGetLastError();
}

CER_API int cer_bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, const bf16_t* gamma,
                             int64_t gamma_stride, const bf16_t* beta, int64_t beta_stride,
                             float* rmean, float* rvar, int64_t rstat_stride, float* mean_out,
                             float* invstd_out, float* ws, float* part, int64_t M, int C,
                             int Cper, float eps, float momentum, int act, hipStream_t stream) {
  return bn_fwd_train_impl(x, res, y, gamma, gamma_stride, beta, beta_stride, rmean, rvar,
                           rstat_stride, mean_out, invstd_out, ws, part, 0, M, C, Cper, eps,
                           momentum, act, stream);
}

// same, with the per-slab (sum, sum^2) partials already produced by the
// producing convolution's epilogue (cer_conv_fwd_stats)
CER_API int cer_bn_fwd_train_part(const bf16_t* x, const bf16_t* res, bf16_t* y,
                                  const bf16_t* gamma, int64_t gamma_stride, const bf16_t* beta,
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
CER_API int cer_bn_apply_fwd(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* ws,
                             const bf16_t* gamma, int64_t gamma_stride, const bf16_t* beta,
                             int64_t beta_stride, int64_t M, int C, int Cper, int act,
                             hipStream_t stream) {
  if (C % VEC || Cper % VEC) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C);
  dim3 ag;
  int arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  bn_apply_fwd<0><<<ag, BN_T, 0, stream>>>(x, res, y, ws, nullptr, nullptr, 0, 0.f,
                                           Strided{gamma, gamma_stride},
                                           Strided{beta, beta_stride}, M, C, Cper, arows, act, mp);
  return (int)hipGetLastError();
}

CER_API int cer_bn_fwd_eval(const bf16_t* x, const bf16_t* res, bf16_t* y, const bf16_t* gamma,
                            int64_t gamma_stride, const bf16_t* beta, int64_t beta_stride,
                            const float* rmean, const float* rvar, int64_t rstat_stride,
                            int64_t M, int C, int Cper, float eps, int act, hipStream_t stream) {
  if (C % VEC || Cper % VEC) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C);
  dim3 ag;
  int arows;
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  bn_apply_fwd<1><<<ag, BN_T, 0, stream>>>(x, res, y, nullptr, rmean, rvar, rstat_stride, eps,
                                           Strided{gamma, gamma_stride},
                                           Strided{beta, beta_stride}, M, C, Cper, arows, act, mp);
  return (int)hipGetLastError();
}

CER_API int cer_bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* mean,
                       const float* invstd, const bf16_t* gamma, int64_t gamma_stride,
                       float* dgamma, float* dbeta, int64_t grad_stride, bf16_t* dx,
                       bf16_t* dres, float* ws, float* part, int64_t M, int C, int Cper, int act,
                       hipStream_t stream) {
  if (C % VEC || Cper % VEC) return (int)hipErrorInvalidValue;
  const Map mp = make_map(C);
  dim3 rg, ag;
  int rrows, arows;
  make_grid(M, C, mp, RED_TARGET, RED_MIN_ROWS, &rg, &rrows);
  make_grid(M, C, mp, APPLY_TARGET, APPLY_MIN_ROWS, &ag, &arows);
  bn_partials<1><<<rg, BN_T, 0, stream>>>(x, dy, y, mean, invstd, part, M, C, rrows, act, mp);
  bn_finalize_bwd<<<cer_blocks(C, FIN_C), FIN_C * FIN_L, 0, stream>>>(part, (int)rg.y, ws, dgamma, dbeta,
                                                          grad_stride, C, Cper);
  bn_apply_bwd<<<ag, BN_T, 0, stream>>>(dy, x, y, mean, invstd, ws,
                                        Strided{gamma, gamma_stride}, dx, dres, M, C, Cper, arows,
                                        act, mp);
  return (int)hipGetLastError();
}
