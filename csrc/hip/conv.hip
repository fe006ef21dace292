// Grouped implicit-GEMM convolution / linear on MFMA for packed NHWC
// (SURVEY.md K4-K6, K8).  G configs are trained at once: blockIdx.z = config
// g, whose activations are channel block g of the packed tensor and whose
// weights sit at w + g*w_gstride in the arena.
//
//  fwd   : y[m, n]  = sum_k im2col(x)[m, k] * W[n, k]          (NT kernel)
//          m = (b, ho, wo), n = cout, k = (r, s, cin)
//  dgrad : dx[m, c] = sum_k col2im(dy)[m, k] * Wt[c, k]          (NT kernel)
//          m = (b, h, w),  k = (r, s, cout), Wt = per-config transpose of W
//  wgrad : dW[n, k] = sum_m dy[m, n] * im2col(x)[m, k]           (TN kernel)
//          reduction over m split across blocks, fp32 atomics into the
//          gradient arena
// A linear layer is the 1x1 conv on a 1x1 image.
//
// Tiles: BM x BN x 32, 256 threads = 2x2 waves, each wave (BM/2)x(BN/2) of
// v_mfma_f32_16x16x32_bf16.  Operands are register-staged global -> LDS with
// a double-buffered LDS ring (one barrier per K-step: the next tile's global
// loads are issued before the MFMAs of the current one).
//  * NT tiles are K-contiguous [rows][32] (64-B rows), read with
//    ds_read_b128; the 16-B chunk is XOR-swizzled by row so that every
//    ds_read_b128 lane group hits 16 distinct bank slots.
//  * TN tiles are [32 (reduction)][cols]; MFMA fragments come out of
//    ds_read_b64_tr_b16 (hardware transpose), with an 8-B-chunk XOR swizzle
//    that keeps each 32-lane half conflict-free.
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 32;
constexpr int NTHREADS = 256;

// ---------------------------------------------------------------------------
// parameters
// ---------------------------------------------------------------------------
struct GatherGeom {
  const bf16_t* src;  // gathered activation tensor (packed NHWC)
  int Ctot;           // pixel stride (G * Cg)
  int Cg;             // channels per config of the gathered tensor
  int Hs, Ws;         // gathered tensor spatial dims
  int Hm, Wm;         // GEMM row grid (pixels of the GEMM's M dimension)
  int kh, kw, st, pad;
};

struct NTParams {
  GatherGeom a;
  int dgrad;              // 0: hi = y*st - pad + r ; 1: (y + pad - r) / st if divisible
  const bf16_t* w;        // [N][K] per config
  int64_t w_gstride;
  bf16_t* out;            // [M][ldc] with config block at g*N
  int ldc;
  int M, N, K;
  const bf16_t* bias;     // optional fused epilogue: out = act(acc + bias[g][n])
  int64_t bias_gstride;
  int act;                // 0 none, 1 relu, 6 relu6
};

struct WGParams {
  GatherGeom x;           // im2col source (Hm, Wm = output grid Ho, Wo)
  const bf16_t* dy;       // [Mred][ldy], config block g*N
  int ldy;
  float* dw;              // [N][K] per config (fp32 grad arena)
  int64_t dw_gstride;
  int Mred, N, K;
  int m_per_split;
};

// ---------------------------------------------------------------------------
// gather helpers
// ---------------------------------------------------------------------------
struct RowPos {
  int b, y, x;
  bool ok;
};

__device__ __forceinline__ RowPos decode_row(int m, int M, int Hm, int Wm) {
  RowPos p;
  p.ok = m < M;
  int mm = p.ok ? m : 0;
  p.x = mm % Wm;
  int t = mm / Wm;
  p.y = t % Hm;
  p.b = t / Hm;
  return p;
}

// source pixel offset (elements, without channel) or -1 when the tap is padding
__device__ __forceinline__ int64_t src_pixel(const GatherGeom& g, const RowPos& p, int r, int s,
                                             int dgrad) {
  int hi, wi;
  if (!dgrad) {
    hi = p.y * g.st - g.pad + r;
    wi = p.x * g.st - g.pad + s;
  } else {
    int hn = p.y + g.pad - r, wn = p.x + g.pad - s;
    if (hn < 0 || wn < 0) return -1;
    if (g.st > 1) {
      if ((hn % g.st) | (wn % g.st)) return -1;
      hn /= g.st;
      wn /= g.st;
    }
    hi = hn;
    wi = wn;
  }
  if (!p.ok || hi < 0 || wi < 0 || hi >= g.Hs || wi >= g.Ws) return -1;
  return (((int64_t)p.b * g.Hs + hi) * g.Ws + wi) * g.Ctot;
}

template <bool ALIGNED>
__device__ __forceinline__ uint4 gather_chunk(const GatherGeom& g, int cfg, const RowPos& p,
                                              int k0, int K, int dgrad) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (ALIGNED) {
    if (k0 >= K) return v;
    const int tap = k0 / g.Cg, c = k0 - tap * g.Cg;
    const int r = tap / g.kw, s = tap - r * g.kw;
    const int64_t off = src_pixel(g, p, r, s, dgrad);
    if (off >= 0) v = *reinterpret_cast<const uint4*>(g.src + off + (int64_t)cfg * g.Cg + c);
  } else {
    uint16_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      e[i] = 0;
      const int k = k0 + i;
      if (k < K) {
        const int tap = k / g.Cg, c = k - tap * g.Cg;
        const int r = tap / g.kw, s = tap - r * g.kw;
        const int64_t off = src_pixel(g, p, r, s, dgrad);
        if (off >= 0) e[i] = g.src[off + (int64_t)cfg * g.Cg + c];
      }
    }
    v.x = e[0] | ((uint32_t)e[1] << 16);
    v.y = e[2] | ((uint32_t)e[3] << 16);
    v.z = e[4] | ((uint32_t)e[5] << 16);
    v.w = e[6] | ((uint32_t)e[7] << 16);
  }
  return v;
}

template <bool ALIGNED>
__device__ __forceinline__ uint4 weight_chunk(const bf16_t* w, int n, int k0, int N, int K) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (n >= N || k0 >= K) return v;
  const bf16_t* p = w + (int64_t)n * K + k0;
  if (ALIGNED) return *reinterpret_cast<const uint4*>(p);
  uint16_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = (k0 + i < K) ? p[i] : 0;
  v.x = e[0] | ((uint32_t)e[1] << 16);
  v.y = e[2] | ((uint32_t)e[3] << 16);
  v.z = e[4] | ((uint32_t)e[5] << 16);
  v.w = e[6] | ((uint32_t)e[7] << 16);
  return v;
}

// ---------------------------------------------------------------------------
// NT LDS tile: [rows][32] bf16, 64-B rows, 16-B chunk XOR swizzle
//   chunk' = chunk ^ f((row >> 2) & 3), f = {0, 2, 3, 1}
// makes every ds_read_b128 lane group of the MFMA fragment read
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) hit 16 distinct 16-B slots.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nt_off(int row, int chunk) {
  const int f = (0x1320 >> (4 * ((row >> 2) & 3))) & 3;
  return row * BK + 8 * (chunk ^ f);
}

template <int BM, int BN, bool ALIGNED>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_nt(NTParams p) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = BM * 4 / NTHREADS, B_CH = BN * 4 / NTHREADS;
  constexpr int TILE_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + 8);
  constexpr int LDS_ELEMS = TILE_ELEMS > EPI_ELEMS ? TILE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
  // ring buffers: A[buf] at buf*BM*BK, B[buf] at 2*BM*BK + buf*BN*BK
#define SA(buf) (lds + (buf) * (BM * BK))
#define SB(buf) (lds + 2 * BM * BK + (buf) * (BN * BK))

  const int cfg = blockIdx.z;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const bf16_t* wbase = p.w + (int64_t)cfg * p.w_gstride;

  RowPos rows[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int row = (tid + NTHREADS * i) >> 2;
    rows[i] = decode_row(m0 + row, p.M, p.a.Hm, p.a.Wm);
  }
  const int my_chunk = tid & 3;
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + 8 * my_chunk;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) ra[i] = gather_chunk<ALIGNED>(p.a, cfg, rows[i], k0, p.K, p.dgrad);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = (tid + NTHREADS * i) >> 2;
      rb[i] = weight_chunk<ALIGNED>(wbase, n0 + row, k0, p.N, p.K);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid + NTHREADS * i) >> 2;
      *reinterpret_cast<uint4*>(SA(buf) + nt_off(row, my_chunk)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = (tid + NTHREADS * i) >> 2;
      *reinterpret_cast<uint4*>(SB(buf) + nt_off(row, my_chunk)) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = (p.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fc = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tiles(kt + 1);
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(SA(cur) + nt_off(wm * TM + 16 * i + fr, fc));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(SB(cur) + nt_off(wn * TN + 16 * j + fr, fc));
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < KT) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // epilogue: (bias + act in fp32, one rounding), stage the bf16 tile in
  // LDS, then 16-B coalesced stores
  constexpr int LDE = BN + 8;
  float bcol[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + 16 * j + fr;
    bcol[j] = (p.bias && n < p.N) ? bf2f(p.bias[(int64_t)cfg * p.bias_gstride + n]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = wm * TM + 16 * i + 4 * fc + e;
        const int c = wn * TN + 16 * j + fr;
        float v = acc[i][j][e] + bcol[j];
        v = p.act == 6 ? fminf(fmaxf(v, 0.f), 6.f) : (p.act ? fmaxf(v, 0.f) : v);
        lds[r * LDE + c] = f2bf(v);
      }
  __syncthreads();
  constexpr int CPR = BN / 8;
  bf16_t* obase = p.out + (int64_t)cfg * p.N;
  for (int idx = tid; idx < BM * CPR; idx += NTHREADS) {
    const int r = idx / CPR, cc = idx - r * CPR;
    const int m = m0 + r, n = n0 + 8 * cc;
    if (m >= p.M || n >= p.N) continue;
    bf16_t* dst = obase + (int64_t)m * p.ldc + n;
    const bf16_t* src = lds + r * LDE + 8 * cc;
    if (n + 8 <= p.N && ((p.N | p.ldc) & 7) == 0) {
      *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    } else {
      for (int e = 0; e < 8 && n + e < p.N; ++e) dst[e] = src[e];
    }
  }
}

// ---------------------------------------------------------------------------
// TN (wgrad) LDS tile: [32 reduction rows][COLS] bf16; 8-B chunk swizzle
// ---------------------------------------------------------------------------
template <int COLS>
__device__ __forceinline__ int tn_off(int row, int col) {  // col multiple of 4
  int sw;
  if (COLS == 128)
    sw = (row & 3) | (((row >> 3) & 1) << 2);
  else
    sw = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return row * COLS + 4 * ((col >> 2) ^ (4 * sw));
}

template <int COLS>
__device__ __forceinline__ bf16x8 tn_frag(const bf16_t* tile, int col_base, int lane) {
  // lane l: elements e = 0..7 of reduction rows 8*(l>>4)+e at column col_base + (l&15)
  const int h = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const bf16_t* p0 = tile + tn_off<COLS>(8 * h + q, col_base + 4 * pp);
  const bf16_t* p1 = tile + tn_off<COLS>(8 * h + 4 + q, col_base + 4 * pp);
  s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  s16x8 t = __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, t);
}

template <int BM, int BN, bool ALIGNED>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_wgrad(WGParams p) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;           // 16-B chunks per tile row
  constexpr int A_CH = BK * A_CPR / NTHREADS, B_CH = BK * B_CPR / NTHREADS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (BM + BN) * BK];

  const int cfg = blockIdx.z;
  const int tiles_k = (p.K + BN - 1) / BN;
  const int tn_ = blockIdx.x / tiles_k, tk = blockIdx.x % tiles_k;
  const int n0 = tn_ * BM, k0 = tk * BN;
  const int ms = blockIdx.y * p.m_per_split;
  const int me = min(p.Mred, ms + p.m_per_split);
  if (ms >= me) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wa = wid >> 1, wb = wid & 1;

  // A (dy) chunk coordinates: row = idx / A_CPR, chunk = idx % A_CPR (fixed per thread)
  // B (x) chunk coordinates: row = idx / B_CPR, k chunk fixed -> tap decode once
  int b_r[B_CH], b_s[B_CH], b_c[B_CH];
  bool b_kok[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int idx = tid + NTHREADS * i;
    const int kk = k0 + 8 * (idx % B_CPR);
    b_kok[i] = kk < p.K;
    const int tap = kk / p.x.Cg;
    b_c[i] = kk - tap * p.x.Cg;
    b_r[i] = tap / p.x.kw;
    b_s[i] = tap - b_r[i] * p.x.kw;
  }
  uint4 ra[A_CH], rb[B_CH];
  const bf16_t* dyb = p.dy + (int64_t)cfg * p.N;

  auto load_tiles = [&](int mt) {
    const int mbase = ms + mt * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int idx = tid + NTHREADS * i;
      const int row = idx / A_CPR, n = n0 + 8 * (idx % A_CPR);
      const int m = mbase + row;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m < me && n < p.N) {
        const bf16_t* src = dyb + (int64_t)m * p.ldy + n;
        if (ALIGNED && n + 8 <= p.N) {
          v = *reinterpret_cast<const uint4*>(src);
        } else {
          uint16_t e[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (n + t < p.N) ? src[t] : 0;
          v.x = e[0] | ((uint32_t)e[1] << 16);
          v.y = e[2] | ((uint32_t)e[3] << 16);
          v.z = e[4] | ((uint32_t)e[5] << 16);
          v.w = e[6] | ((uint32_t)e[7] << 16);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int idx = tid + NTHREADS * i;
      const int row = idx / B_CPR;
      const int m = mbase + row;
      RowPos pos = decode_row(m, me, p.x.Hm, p.x.Wm);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b_kok[i] && pos.ok) {
        if (ALIGNED) {
          const int64_t off = src_pixel(p.x, pos, b_r[i], b_s[i], 0);
          if (off >= 0)
            v = *reinterpret_cast<const uint4*>(p.x.src + off + (int64_t)cfg * p.x.Cg + b_c[i]);
        } else {
          v = gather_chunk<false>(p.x, cfg, pos, k0 + 8 * (idx % B_CPR), p.K, 0);
        }
      }
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int idx = tid + NTHREADS * i;
      const int row = idx / A_CPR, col = 8 * (idx % A_CPR);
      *reinterpret_cast<uint4*>(SA(buf) + tn_off<BM>(row, col)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int idx = tid + NTHREADS * i;
      const int row = idx / B_CPR, col = 8 * (idx % B_CPR);
      *reinterpret_cast<uint4*>(SB(buf) + tn_off<BN>(row, col)) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int MT = (me - ms + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int mt = 0; mt < MT; ++mt) {
    const int cur = mt & 1;
    if (mt + 1 < MT) load_tiles(mt + 1);
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = tn_frag<BM>(SA(cur), wa * TM + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = tn_frag<BN>(SB(cur), wb * TN + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (mt + 1 < MT) store_tiles(cur ^ 1);
    __syncthreads();
  }

  float* dwb = p.dw + (int64_t)cfg * p.dw_gstride;
  const int fr = lane & 15, fc = lane >> 4;
  const bool split = gridDim.y > 1;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wa * TM + 16 * i + 4 * fc + e;
        const int k = k0 + wb * TN + 16 * j + fr;
        if (n < p.N && k < p.K) {
          float* d = dwb + (int64_t)n * p.K + k;
          if (split)
            atomicAdd(d, acc[i][j][e]);
          else
            *d = acc[i][j][e];
        }
      }
}

#undef SA
#undef SB

// ---------------------------------------------------------------------------
// per-config weight transpose for dgrad: W[N][T][C] -> Wt[C][T][N]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void transpose_w_kernel(const bf16_t* __restrict__ w,
                                                          int64_t w_gstride,
                                                          bf16_t* __restrict__ wt, int N,
                                                          int T, int C) {
  __shared__ bf16_t tile[32][33];
  const int cfg = blockIdx.z;
  const int t = blockIdx.y;
  const int tiles_c = (C + 31) / 32;
  const int tn = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const bf16_t* src = w + (int64_t)cfg * w_gstride;
  bf16_t* dst = wt + (int64_t)cfg * N * T * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int yy = ty; yy < 32; yy += 8) {
    const int n = tn * 32 + yy, c = tc * 32 + tx;
    tile[yy][tx] = (n < N && c < C) ? src[((int64_t)n * T + t) * C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int c = tc * 32 + yy, n = tn * 32 + tx;
    if (c < C && n < N) dst[((int64_t)c * T + t) * N + n] = tile[tx][yy];
  }
}

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
template <int BM, int BN>
static int launch_nt(const NTParams& p, int G, bool aligned, hipStream_t stream) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, 1, G);
  if (aligned)
    igemm_nt<BM, BN, true><<<grid, NTHREADS, 0, stream>>>(p);
  else
    igemm_nt<BM, BN, false><<<grid, NTHREADS, 0, stream>>>(p);
  return (int)hipGetLastError();
}

static int run_nt(const NTParams& p, int G, hipStream_t stream) {
  const bool aligned = (p.a.Cg % 8 == 0) && (p.a.Ctot % 8 == 0) && (p.K % 8 == 0);
  const long big = (long)((p.M + 127) / 128) * ((p.N + 127) / 128) * G;
  if (big >= 512) return launch_nt<128, 128>(p, G, aligned, stream);
  return launch_nt<64, 64>(p, G, aligned, stream);
}

CER_API int cer_conv_fwd(const bf16_t* x, int B, int H, int W, int Cin, int G, const bf16_t* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         bf16_t* y, int Ho, int Wo, const bf16_t* bias, int64_t bias_gstride,
                         int act, hipStream_t stream) {
  NTParams p;
  p.bias = bias;
  p.bias_gstride = bias_gstride;
  p.act = act;
  p.a = GatherGeom{x, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad};
  p.dgrad = 0;
  p.w = w;
  p.w_gstride = w_gstride;
  p.out = y;
  p.ldc = G * Cout;
  p.M = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  return run_nt(p, G, stream);
}

// wt: scratch of G * Cout*kh*kw*Cin elements (per-config transposed weights)
CER_API int cer_conv_dgrad(const bf16_t* dy, int B, int Ho, int Wo, int Cout, int G,
                           const bf16_t* w, int64_t w_gstride, bf16_t* wt, int Cin, int kh,
                           int kw, int st, int pad, bf16_t* dx, int H, int W,
                           hipStream_t stream) {
  const int T = kh * kw;
  dim3 tg(((Cout + 31) / 32) * ((Cin + 31) / 32), T, G);
  transpose_w_kernel<<<tg, 256, 0, stream>>>(w, w_gstride, wt, Cout, T, Cin);
  NTParams p;
  p.bias = nullptr;
  p.bias_gstride = 0;
  p.act = 0;
  p.a = GatherGeom{dy, G * Cout, Cout, Ho, Wo, H, W, kh, kw, st, pad};
  p.dgrad = 1;
  p.w = wt;
  p.w_gstride = (int64_t)Cout * T * Cin;
  p.out = dx;
  p.ldc = G * Cin;
  p.M = B * H * W;
  p.N = Cin;
  p.K = T * Cout;
  return run_nt(p, G, stream);
}

template <int BM, int BN>
static int launch_wg(WGParams p, int G, bool aligned, int splits, hipStream_t stream) {
  const int tiles = ((p.N + BM - 1) / BM) * ((p.K + BN - 1) / BN);
  p.m_per_split = ((p.Mred + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
  dim3 grid(tiles, splits, G);
  if (aligned)
    igemm_wgrad<BM, BN, true><<<grid, NTHREADS, 0, stream>>>(p);
  else
    igemm_wgrad<BM, BN, false><<<grid, NTHREADS, 0, stream>>>(p);
  return (int)hipGetLastError();
}

// dw must be zeroed by the caller when more than one split is used (splits > 1)
CER_API int cer_conv_wgrad(const bf16_t* x, int B, int H, int W, int Cin, int G,
                           const bf16_t* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                           int pad, float* dw, int64_t dw_gstride, int splits,
                           hipStream_t stream) {
  WGParams p;
  p.x = GatherGeom{x, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad};
  p.dy = dy;
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  const bool aligned = (Cin % 8 == 0) && (Cout % 8 == 0);
  const bool big = ((long)((p.N + 127) / 128) * ((p.K + 127) / 128) * G) >= 256;
  if (big) return launch_wg<128, 128>(p, G, aligned, splits, stream);
  return launch_wg<64, 64>(p, G, aligned, splits, stream);
}

// the split count the host should use (and whether dw needs zeroing)
CER_API int cer_wgrad_splits(int Mred, int N, int K, int G) {
  const bool big = ((long)((N + 127) / 128) * ((K + 127) / 128) * G) >= 256;
  const int bm = big ? 128 : 64;
  const long tiles = (long)((N + bm - 1) / bm) * ((K + bm - 1) / bm) * G;
  long want = (1024 + tiles - 1) / tiles;          // aim for ~1024 blocks
  long maxs = (Mred + 255) / 256;                  // >= 256 rows per split
  long s = want < maxs ? want : maxs;
  return (int)(s < 1 ? 1 : s);
}
