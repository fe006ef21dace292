// Grouped implicit-GEMM convolution / linear on MFMA for packed NHWC
// (SURVEY.md K4-K6, K8).  G configs are trained at once: blockIdx.z = config
// g, whose activations are channel block g of the packed tensor and whose
// weights sit at w + g*w_gstride in the arena.
//
//  fwd   : y[m, n]  = act(sum_k im2col(x)[m, k] * W[n, k] + b[n])   (NT kernel)
//          m = (b, ho, wo), n = cout, k = (r, s, cin)
//  dgrad : dx[m, c] = sum_k col2im(dy)[m, k] * W[(k), c]            (NN kernel)
//          m = (b, h, w),  k = (r, s, cout); W rows read in place through the
//          LDS transpose read; strided 1x1 convs only compute nonzero rows
//  wgrad : dW[n, k] = sum_m dy[m, n] * im2col(x)[m, k]                (TN kernel)
//          reduction over m split across blocks, fp32 atomics into the
//          gradient arena when split
// A linear layer is the 1x1 conv on a 1x1 image.
//
// Tiles: BM x BN x 64, 256 threads = 2x2 waves, each wave (BM/2)x(BN/2) of
// v_mfma_f32_16x16x32_bf16 (two k-substeps per tile).  Operands are
// register-staged global -> LDS through a double-buffered LDS ring with ONE
// barrier per 64-deep K-step; the next tile's global loads are issued before
// the current tile's MFMAs so HBM latency hides under them.
//  * NT tiles are K-contiguous [rows][64] (128-B rows) read with
//    ds_read_b128; 16-B chunk swizzle chunk ^ ((row >> 1) & 7) makes each of
//    the four ds_read_b128 lane groups hit 16 distinct bank slots.
//  * TN tiles are [64 (reduction)][cols]; MFMA fragments come out of
//    ds_read_b64_tr_b16 (hardware transpose), 8-B-chunk XOR swizzle keeps
//    each 32-lane half conflict-free.
//  * im2col addressing is incremental (no integer division in the K loop);
//    row decode uses magic-number division.
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 64;
constexpr int NTHREADS = 256;

// ---------------------------------------------------------------------------
// n / d for 0 <= n < 2^31 by multiply-high (Granlund-Montgomery)
// ---------------------------------------------------------------------------
struct FastDiv {
  uint32_t d, m, s;
};

static FastDiv make_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

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
  FastDiv dWm, dHm, dCg, dkw;
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
  int o_st, o_H, o_W;     // o_st > 1: GEMM row (b,y,x) stores to output pixel (b, y*o_st, x*o_st)
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

static GatherGeom make_geom(const bf16_t* src, int Ctot, int Cg, int Hs, int Ws, int Hm, int Wm,
                            int kh, int kw, int st, int pad) {
  GatherGeom g{src, Ctot, Cg, Hs, Ws, Hm, Wm, kh, kw, st, pad, {}, {}, {}, {}};
  g.dWm = make_div((uint32_t)Wm);
  g.dHm = make_div((uint32_t)Hm);
  g.dCg = make_div((uint32_t)Cg);
  g.dkw = make_div((uint32_t)kw);
  return g;
}

// ---------------------------------------------------------------------------
// gather helpers
// ---------------------------------------------------------------------------
struct RowPos {
  int b, y, x;
  bool ok;
};

__device__ __forceinline__ RowPos decode_row(int m, int M, const GatherGeom& g) {
  RowPos p;
  p.ok = m < M;
  const uint32_t mm = p.ok ? (uint32_t)m : 0u;
  const uint32_t t = fdiv(mm, g.dWm);
  p.x = (int)(mm - t * (uint32_t)g.Wm);
  const uint32_t b = fdiv(t, g.dHm);
  p.y = (int)(t - b * (uint32_t)g.Hm);
  p.b = (int)b;
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

__device__ __forceinline__ uint4 pack8(const uint16_t* e) {
  uint4 v;
  v.x = e[0] | ((uint32_t)e[1] << 16);
  v.y = e[2] | ((uint32_t)e[3] << 16);
  v.z = e[4] | ((uint32_t)e[5] << 16);
  v.w = e[6] | ((uint32_t)e[7] << 16);
  return v;
}

// generic per-element gather (channel counts not multiple of 8, e.g. the stem)
__device__ __forceinline__ uint4 gather_chunk_slow(const GatherGeom& g, int cfg, const RowPos& p,
                                                   int k0, int K, int dgrad) {
  uint16_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    e[i] = 0;
    const int k = k0 + i;
    if (k < K) {
      const int tap = (int)fdiv((uint32_t)k, g.dCg), c = k - tap * g.Cg;
      const int r = (int)fdiv((uint32_t)tap, g.dkw), s = tap - r * g.kw;
      const int64_t off = src_pixel(g, p, r, s, dgrad);
      if (off >= 0) e[i] = g.src[off + (int64_t)cfg * g.Cg + c];
    }
  }
  return pack8(e);
}

// running im2col position of a thread's fixed 8-wide k-chunk within the BK window
struct KPos {
  int c, r, s;  // channel offset, tap row, tap col
};

__device__ __forceinline__ KPos kpos_init(const GatherGeom& g, int k) {
  const int tap = (int)fdiv((uint32_t)k, g.dCg);
  const int r = (int)fdiv((uint32_t)tap, g.dkw);
  return KPos{k - tap * g.Cg, r, tap - r * g.kw};
}

__device__ __forceinline__ void kpos_advance(const GatherGeom& g, KPos& kp) {
  kp.c += BK;
  while (kp.c >= g.Cg) {
    kp.c -= g.Cg;
    if (++kp.s == g.kw) {
      kp.s = 0;
      ++kp.r;
    }
  }
}

// ---------------------------------------------------------------------------
// NT LDS tile: [rows][64] bf16, 128-B rows, 16-B chunk c stored at
// c ^ ((row >> 1) & 7)  (conflict-free for the MFMA ds_read_b128 pattern)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nt_off(int row, int chunk) {
  return row * BK + 8 * (chunk ^ ((row >> 1) & 7));
}

// epilogue store of a staged [BM][BN] bf16 tile (shared by the NT and NN kernels)
template <int BM, int BN>
__device__ __forceinline__ void store_tile(const NTParams& p, const bf16_t* lds, int LDE, int cfg,
                                           int m0, int n0, int tid) {
  constexpr int OCPR = BN / 8;
  bf16_t* obase = p.out + (int64_t)cfg * p.N;
  const bool vec_ok = ((p.N | p.ldc) & 7) == 0;
  for (int idx = tid; idx < BM * OCPR; idx += NTHREADS) {
    const int r = idx / OCPR, cc = idx - r * OCPR;
    const int m = m0 + r, n = n0 + 8 * cc;
    if (m >= p.M || n >= p.N) continue;
    int64_t orow = m;
    if (p.o_st > 1) {
      const RowPos q = decode_row(m, p.M, p.a);
      orow = ((int64_t)q.b * p.o_H + (int64_t)q.y * p.o_st) * p.o_W + (int64_t)q.x * p.o_st;
    }
    bf16_t* dst = obase + orow * p.ldc + n;
    const bf16_t* src = lds + r * LDE + 8 * cc;
    if (vec_ok && n + 8 <= p.N) {
      *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    } else {
      for (int e = 0; e < 8 && n + e < p.N; ++e) dst[e] = src[e];
    }
  }
}

template <int BM, int BN, bool ALIGNED>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_nt(NTParams p) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int CPR = BK / 8;                                  // 16-B chunks per row
  constexpr int A_CH = BM * CPR / NTHREADS, B_CH = BN * CPR / NTHREADS;
  constexpr int TILE_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + 8);
  constexpr int LDS_ELEMS = TILE_ELEMS > EPI_ELEMS ? TILE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
#define SA(buf) (lds + (buf) * (BM * BK))
#define SB(buf) (lds + 2 * BM * BK + (buf) * (BN * BK))

  const int cfg = blockIdx.z;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);                        // same for every i below
  const bf16_t* wbase = p.w + (int64_t)cfg * p.w_gstride;
  const bf16_t* abase = p.a.src + (int64_t)cfg * p.a.Cg;

  RowPos rows[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) rows[i] = decode_row(m0 + (tid + NTHREADS * i) / CPR, p.M, p.a);
  KPos kp = kpos_init(p.a, 8 * my_chunk);
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + 8 * my_chunk;
    if (ALIGNED) {
      const bool kok = k0 < p.K;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kok) {
          const int64_t off = src_pixel(p.a, rows[i], kp.r, kp.s, p.dgrad);
          if (off >= 0) v = *reinterpret_cast<const uint4*>(abase + off + kp.c);
        }
        ra[i] = v;
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid + NTHREADS * i) / CPR;
        rb[i] = (kok && n < p.N) ? *reinterpret_cast<const uint4*>(wbase + (int64_t)n * p.K + k0)
                                 : make_uint4(0, 0, 0, 0);
      }
      kpos_advance(p.a, kp);
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) ra[i] = gather_chunk_slow(p.a, cfg, rows[i], k0, p.K, p.dgrad);
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid + NTHREADS * i) / CPR;
        uint16_t e[8];
        const bf16_t* src = wbase + (int64_t)n * p.K + k0;
#pragma unroll
        for (int t = 0; t < 8; ++t) e[t] = (n < p.N && k0 + t < p.K) ? src[t] : 0;
        rb[i] = pack8(e);
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<uint4*>(SA(buf) + nt_off((tid + NTHREADS * i) / CPR, my_chunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      *reinterpret_cast<uint4*>(SB(buf) + nt_off((tid + NTHREADS * i) / CPR, my_chunk)) = rb[i];
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
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(SA(cur) + nt_off(wm * TM + 16 * i + fr, fc + 4 * kk));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(SB(cur) + nt_off(wn * TN + 16 * j + fr, fc + 4 * kk));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
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
  store_tile<BM, BN>(p, lds, LDE, cfg, m0, n0, tid);
}


// ---------------------------------------------------------------------------
// TN (wgrad) LDS tile: [64 reduction rows][COLS] bf16; 8-B chunk swizzle
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
__device__ __forceinline__ bf16x8 tn_frag(const bf16_t* tile, int row0, int col_base, int lane) {
  // lane l: elements e = 0..7 of reduction rows row0 + 8*(l>>4) + e at column col_base + (l&15)
  const int h = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const bf16_t* p0 = tile + tn_off<COLS>(row0 + 8 * h + q, col_base + 4 * pp);
  const bf16_t* p1 = tile + tn_off<COLS>(row0 + 8 * h + 4 + q, col_base + 4 * pp);
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
  constexpr int A_RSTEP = NTHREADS / A_CPR, B_RSTEP = NTHREADS / B_CPR;
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

  // each thread's chunk column is fixed; its rows step by 256 / chunks-per-row
  const int a_col = 8 * (tid % A_CPR), b_col = 8 * (tid % B_CPR);
  const int a_row0 = tid / A_CPR, b_row0 = tid / B_CPR;
  const int kk0 = k0 + b_col;
  const bool b_kok = kk0 < p.K;
  KPos bk{0, 0, 0};
  if (b_kok) bk = kpos_init(p.x, kk0);
  uint4 ra[A_CH], rb[B_CH];
  const bf16_t* dyb = p.dy + (int64_t)cfg * p.N;
  const bf16_t* xb = p.x.src + (int64_t)cfg * p.x.Cg;

  auto load_tiles = [&](int mt) {
    const int mbase = ms + mt * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = mbase + a_row0 + A_RSTEP * i, n = n0 + a_col;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m < me && n < p.N) {
        const bf16_t* src = dyb + (int64_t)m * p.ldy + n;
        if (ALIGNED && n + 8 <= p.N) {
          v = *reinterpret_cast<const uint4*>(src);
        } else {
          uint16_t e[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (n + t < p.N) ? src[t] : 0;
          v = pack8(e);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int m = mbase + b_row0 + B_RSTEP * i;
      const RowPos pos = decode_row(m, me, p.x);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b_kok && pos.ok) {
        if (ALIGNED) {
          const int64_t off = src_pixel(p.x, pos, bk.r, bk.s, 0);
          if (off >= 0) v = *reinterpret_cast<const uint4*>(xb + off + bk.c);
        } else {
          v = gather_chunk_slow(p.x, cfg, pos, kk0, p.K, 0);
        }
      }
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
    bf16_t* sa = lds + buf * (BK * BM);
    bf16_t* sb = lds + 2 * BK * BM + buf * (BK * BN);
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<uint4*>(sa + tn_off<BM>(a_row0 + A_RSTEP * i, a_col)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      *reinterpret_cast<uint4*>(sb + tn_off<BN>(b_row0 + B_RSTEP * i, b_col)) = rb[i];
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
    const bf16_t* sa = lds + cur * (BK * BM);
    const bf16_t* sb = lds + 2 * BK * BM + cur * (BK * BN);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = tn_frag<BM>(sa, 32 * kk, wa * TM + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = tn_frag<BN>(sb, 32 * kk, wb * TN + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
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


// ---------------------------------------------------------------------------
// NN (dgrad) kernel: A = col2im(dy) K-contiguous (NT-style LDS, ds_read_b128),
// B = W read as [k = (tap, cout)] x [cin] rows straight from the arena (TN-
// style LDS, ds_read_b64_tr_b16) -> no per-step weight transpose.
//   dx[m, c] = sum_{tap, n} dy~[m, (tap, n)] * W[n][tap][c]
// ---------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_nn_dgrad(NTParams p, int T, FastDiv dCout) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int CPR = BK / 8;
  constexpr int A_CH = BM * CPR / NTHREADS;
  constexpr int B_CPR = BN / 8, B_CH = BK * B_CPR / NTHREADS, B_RSTEP = NTHREADS / B_CPR;
  constexpr int TILE_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + 8);
  constexpr int LDS_ELEMS = TILE_ELEMS > EPI_ELEMS ? TILE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];

  const int cfg = blockIdx.z;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);
  const int Cout = p.a.Cg;          // reduction channels (k = tap*Cout + n)
  const int Cin = p.N;              // output channels
  const bf16_t* wbase = p.w + (int64_t)cfg * p.w_gstride;
  const bf16_t* abase = p.a.src + (int64_t)cfg * p.a.Cg;
  const int b_col = 8 * (tid % B_CPR), b_row0 = tid / B_CPR;

  RowPos rows[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) rows[i] = decode_row(m0 + (tid + NTHREADS * i) / CPR, p.M, p.a);
  KPos kp = kpos_init(p.a, 8 * my_chunk);
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + 8 * my_chunk;
    const bool kok = k0 < p.K;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kok) {
        const int64_t off = src_pixel(p.a, rows[i], kp.r, kp.s, p.dgrad);
        if (off >= 0) v = *reinterpret_cast<const uint4*>(abase + off + kp.c);
      }
      ra[i] = v;
    }
    kpos_advance(p.a, kp);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int k = kt * BK + b_row0 + B_RSTEP * i;
      const int c = n0 + b_col;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < p.K && c < Cin) {
        const int tap = (int)fdiv((uint32_t)k, dCout);
        const int n = k - tap * Cout;
        v = *reinterpret_cast<const uint4*>(wbase + ((int64_t)n * T + tap) * Cin + c);
      }
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
    bf16_t* sa = lds + buf * (BM * BK);
    bf16_t* sb = lds + 2 * BM * BK + buf * (BK * BN);
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<uint4*>(sa + nt_off((tid + NTHREADS * i) / CPR, my_chunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      *reinterpret_cast<uint4*>(sb + tn_off<BN>(b_row0 + B_RSTEP * i, b_col)) = rb[i];
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
    const bf16_t* sa = lds + cur * (BM * BK);
    const bf16_t* sb = lds + 2 * BM * BK + cur * (BK * BN);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc + 4 * kk));
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = tn_frag<BN>(sb, 32 * kk, wn * TN + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_tiles(cur ^ 1);
    __syncthreads();
  }
  constexpr int LDE = BN + 8;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        lds[(wm * TM + 16 * i + 4 * fc + e) * LDE + wn * TN + 16 * j + fr] = f2bf(acc[i][j][e]);
  __syncthreads();
  store_tile<BM, BN>(p, lds, LDE, cfg, m0, n0, tid);
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
  p.a = make_geom(x, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad);
  p.dgrad = 0;
  p.w = w;
  p.w_gstride = w_gstride;
  p.out = y;
  p.ldc = G * Cout;
  p.M = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  p.bias = bias;
  p.bias_gstride = bias_gstride;
  p.act = act;
  p.o_st = 1;
  p.o_H = Ho;
  p.o_W = Wo;
  return run_nt(p, G, stream);
}

template <int BM, int BN>
static int launch_nn(const NTParams& p, int G, int T, hipStream_t stream) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, 1, G);
  igemm_nn_dgrad<BM, BN><<<grid, NTHREADS, 0, stream>>>(p, T, make_div((uint32_t)p.a.Cg));
  return (int)hipGetLastError();
}

// dx = dgrad(dy, W).  Aligned channels: NN kernel (weights read in place, no
// transpose); a strided 1x1 conv only computes the B*Ho*Wo rows that receive
// gradient (the rest of dx is zero-filled).  Otherwise the transpose + NT path.
// wt: scratch of G * Cout*kh*kw*Cin elements (used by the fallback only)
CER_API int cer_conv_dgrad(const bf16_t* dy, int B, int Ho, int Wo, int Cout, int G,
                           const bf16_t* w, int64_t w_gstride, bf16_t* wt, int Cin, int kh,
                           int kw, int st, int pad, bf16_t* dx, int H, int W,
                           hipStream_t stream) {
  const int T = kh * kw;
  NTParams p;
  p.bias = nullptr;
  p.bias_gstride = 0;
  p.act = 0;
  p.o_st = 1;
  p.o_H = H;
  p.o_W = W;
  p.out = dx;
  p.ldc = G * Cin;
  p.N = Cin;
  p.K = T * Cout;
  const bool aligned = (Cout % 8 == 0) && (Cin % 8 == 0);
  if (aligned) {
    p.w = w;
    p.w_gstride = w_gstride;
    if (kh == 1 && kw == 1 && pad == 0 && st > 1) {
      // rows (b, ho, wo) of dy map to dx pixels (b, ho*st, wo*st); others get 0
      hipMemsetAsync(dx, 0, sizeof(bf16_t) * (size_t)B * H * W * G * Cin, stream);
      p.a = make_geom(dy, G * Cout, Cout, Ho, Wo, Ho, Wo, 1, 1, 1, 0);
      p.dgrad = 0;
      p.M = B * Ho * Wo;
      p.o_st = st;
    } else {
      p.a = make_geom(dy, G * Cout, Cout, Ho, Wo, H, W, kh, kw, st, pad);
      p.dgrad = 1;
      p.M = B * H * W;
    }
    const long big = (long)((p.M + 127) / 128) * ((p.N + 127) / 128) * G;
    if (big >= 512) return launch_nn<128, 128>(p, G, T, stream);
    return launch_nn<64, 64>(p, G, T, stream);
  }
  dim3 tg(((Cout + 31) / 32) * ((Cin + 31) / 32), T, G);
  transpose_w_kernel<<<tg, 256, 0, stream>>>(w, w_gstride, wt, Cout, T, Cin);
  p.a = make_geom(dy, G * Cout, Cout, Ho, Wo, H, W, kh, kw, st, pad);
  p.dgrad = 1;
  p.w = wt;
  p.w_gstride = (int64_t)Cout * T * Cin;
  p.M = B * H * W;
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

static bool wgrad_big(int N, int K, int G) {
  return ((long)((N + 127) / 128) * ((K + 127) / 128) * G) >= 256;
}

// dw must be zeroed by the caller when more than one split is used (splits > 1)
CER_API int cer_conv_wgrad(const bf16_t* x, int B, int H, int W, int Cin, int G,
                           const bf16_t* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                           int pad, float* dw, int64_t dw_gstride, int splits,
                           hipStream_t stream) {
  WGParams p;
  p.x = make_geom(x, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad);
  p.dy = dy;
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  const bool aligned = (Cin % 8 == 0) && (Cout % 8 == 0);
  if (wgrad_big(p.N, p.K, G)) return launch_wg<128, 128>(p, G, aligned, splits, stream);
  return launch_wg<64, 64>(p, G, aligned, splits, stream);
}

// the split count the host should use (and whether dw needs zeroing)
CER_API int cer_wgrad_splits(int Mred, int N, int K, int G) {
  const int bm = wgrad_big(N, K, G) ? 128 : 64;
  const long tiles = (long)((N + bm - 1) / bm) * ((K + bm - 1) / bm) * G;
  long want = (1024 + tiles - 1) / tiles;          // aim for ~1024 blocks
  long maxs = (Mred + 511) / 512;                  // >= 512 rows per split
  long s = want < maxs ? want : maxs;
  return (int)(s < 1 ? 1 : s);
}
