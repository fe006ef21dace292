// Grouped implicit-GEMM convolution / linear on MFMA for packed NHWC
// (SURVEY.md K4-K6, K8).  G configs are trained at once: work item -> config
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

#include <stdlib.h>

#include <type_traits>
#include <utility>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 64;
constexpr int NTHREADS = 256;
// bf16 elements after the staged C tile for the BN-statistics exchange
// ([2 waves][2][BN] floats, reused as [2][NTHREADS] floats by the fused
// finalize, and as [2][lanes][BN] = 4096 floats by the BN-backward
// statistics of a dgrad epilogue) and the last-arriver flag.  Every kernel's
// operand staging area is at least this big, so it costs no LDS.
constexpr int STAT_XCH = 2 * 4096 + 8;

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
  int kh, kw, st, pad;  // stride / padding along H (and W unless overridden below)
  uint32_t bytes;     // size of src in bytes (buffer-load range); 0 = too big for 32-bit offsets
  FastDiv dWm, dHm, dCg, dkw, dst;
  int st_w, pad_w;    // stride / padding along W
  int64_t cfg_off;    // elements between configs (Cg for the packed layout)
};

// BN-backward statistics in a dgrad epilogue: the dgrad output is the input
// gradient dy of a BatchNorm layer (whose output the conv consumed), so the
// epilogue also produces that BN's per-(M tile, channel) partials
// (sum dz, sum dz * xhat), dz = act'(.) dy, exactly what bn_partials<1>
// would compute from the stored bf16 dy -> the BN backward skips its
// partials pass over (dy, x[, y]).  part == nullptr: off.
struct BNBwdEpi {
  float* part;                  // [M tiles][2][ldc]
  const bf16_t* z;              // BN input, [M][ldc]
  const bf16_t* y;              // BN output (mask mode YM_Y)
  const float* mean;            // [ldc]
  const float* invstd;
  const bf16_t* gamma;          // per-config parameters (mask mode YM_Z)
  int64_t gstride;
  const bf16_t* beta;
  int64_t bstride;
  int ym, act;                  // mask mode (bn.hip YM_*) and activation code
};

struct NTParams {
  GatherGeom a;
  int dgrad;              // generic path only: 0: hi = y*st - pad + r ; 1: (y + pad - r) / st
  const bf16_t* w;        // [N][K] per config
  int64_t w_gstride;
  bf16_t* out;            // [M][ldc] with config block at g*N
  int ldc;
  int M, N, K;
  const bf16_t* bias;     // optional fused epilogue: out = act(acc + bias[g][n])
  int64_t bias_gstride;
  int act;                // 0 none, 1 relu, 6 relu6
  int o_st, o_H, o_W;     // o_st > 1: GEMM row (b,y,x) stores to output pixel (b, y*o_st, x*o_st)
  float* stats;           // optional BN partials part[slab][2][ldc] (sum, sum^2) of the
                          // bf16 outputs; slab = M tile (fused BN forward)
  int splits = 1;         // split-K: K-tile ranges per output tile (fwd / dgrad, small grids)
  float* skws = nullptr;  // split-K fp32 partial slots [tile][split][acc regs x threads]
  unsigned* skcnt = nullptr;  // split-K per-tile arrival counters (zero; last arriver re-zeroes)
  const bf16_t* addend = nullptr;  // optional: out += addend (same layout as out), rounded once
                                   // (dgrad of a tensor with two consumers: the other one's
                                   // input gradient joins here instead of in an add kernel)
  const uint8_t* addend_mask = nullptr;  // fp32: the addend counts only where this bit mask
                                         // ([M][ldc / 8] bytes) is set (a residual join's
                                         // dres = mask * dy, never stored: ops.nn.MaskedGrad)
  BNBwdEpi bb = BNBwdEpi{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0,
                         0, 0};
  int stat_slabs = 0;     // BN partials: 0 = one slab per M tile (plain stores); n > 0 = n
                          // slabs, tile t atomically adds into slab t % n (zeroed by the caller)
  int a_hl = 0;           // fp32 kernels: the A operand is in HL format (take_hi_lo)
  int w_hl = 0;           // fp32 GM_GEMM / GM_TAP kernels: w is the HL image of the weights
                          // (cer_conv_set_whl: written by the optimizer, no split in the K loop)
};

// Slab count for the BN partials of the next conv launches (cer_conv_set_stat_slabs):
// with n > 0 every M tile adds its fp32 (sum, sum^2) / (sum dz, sum dz*xhat)
// into slab (tile % n) of an fp64 buffer [n][2][ldc] by fp64 atomics, so the
// BN apply that consumes them reduces n slabs, not one per tile, and folds
// the finalize (one BN launch per layer and direction instead of two).
// fp64 makes the slab sums near-deterministic (~1e-16 relative; a large layer
// adds ~200 mixed-sign tile partials per slab, so the order can still round
// in the last fp64 bit): fp32 atomics here made two identical steps differ by 5 % in the
// gradients of a fresh ResNet-50 (50 BN layers amplify 1e-7 statistic noise;
// scripts/debug/slab_determinism.py).  The caller hands zeroed buffers; the
// slab count it gets back carries SLAB_F64 (bn.hip reads the fp64 format).
static int g_stat_slabs = 0;
CER_API void cer_conv_set_stat_slabs(int n) { g_stat_slabs = n > 0 ? n : 0; }

// HL operand format (take_hi_lo) of the NEXT fp32 launches until reset:
// x_hl -- the activation (fwd A operand, wgrad B operand) is HL; dy_hl -- the
// output gradient (dgrad / wgrad A operand) is HL.  Only the aligned gathers
// read HL: a launch that would take a generic (per-element) gather or a
// grouped per-config launch returns hipErrorInvalidValue instead.
static int g_hl_x = 0, g_hl_dy = 0;
CER_API void cer_conv_set_hl(int x_hl, int dy_hl) {
  g_hl_x = x_hl ? 1 : 0;
  g_hl_dy = dy_hl ? 1 : 0;
}
constexpr int SLAB_F64 = 1 << 24;

// one partial into the statistics buffer: plain fp32 store (one slab per
// tile) or an fp64 atomic add (``slabs`` > 0; ``dst`` then addresses the
// float buffer as doubles at the same element index)
__device__ __forceinline__ void stat_store(float* base, int64_t idx, float v, int slabs) {
  if (slabs)
    atomicAdd(reinterpret_cast<double*>(base) + idx, (double)v);
  else
    base[idx] = v;
}

// element offset of (slab of M tile ``tile``, config, stat row 0)
__device__ __forceinline__ int64_t stat_base(int tile, int slabs, int ldc, int cfg, int N) {
  return (slabs ? tile % slabs : tile) * 2 * (int64_t)ldc + (int64_t)cfg * N;
}

static int stat_nslab(int tiles_m, int slabs) {
  return slabs ? (tiles_m > slabs ? slabs : tiles_m) | SLAB_F64 : tiles_m;
}

// BNBwdEpi mode YM_BIAS ("bias-act link", cer_conv_dgrad_babwd): the dgrad
// output is the output gradient of a conv + bias + activation layer whose
// activation y = act(conv + b) this conv consumed (VGG's conv -> conv).  The
// epilogue applies the activation derivative itself -- dz = act'(y) * dx is
// what it writes -- and adds the tile's per-channel sum of dz into the bias
// gradient (fp32 atomics; the optimizer clears the gradient it consumes), so
// the layer's separate bias_act_bwd pass over (dy, y, dz) disappears.
// Fields: part = the bias gradient, z = y (fp32 [M][ldc]), gstride = the
// bias-gradient stride per config, act = 1 (ReLU) / 6 (ReLU6).
constexpr int YM_BIAS = 4;

__device__ __forceinline__ bool act_pass(int act, float y) {
  return act == 6 ? (y > 0.f && y < 6.f) : (act ? y > 0.f : true);
}

// the addend-mask bits of element el (of [M][ldc]) and the next 3 (el % 4 ==
// 0 on the vector paths: one byte); all set without a mask
__device__ __forceinline__ uint32_t addend_bits(const NTParams& p, int64_t el) {
  if (!p.addend_mask) return 0xfu;
  return (uint32_t)p.addend_mask[el >> 3] >> (uint32_t)(el & 7);
}

// the block's per-channel sums (xch rows 0 and 2: the two M-direction waves)
// into the bias gradient
template <int BN>
__device__ __forceinline__ void bias_link_store(const BNBwdEpi& bb, const float* xch, int cfg,
                                                int n0, int N, int tid) {
  for (int nl = tid; nl < BN; nl += NTHREADS) {
    const int n = n0 + nl;
    if (n < N) atomicAdd(bb.part + (int64_t)cfg * bb.gstride + n, xch[nl] + xch[2 * BN + nl]);
  }
}


struct WGParams {
  GatherGeom x;           // im2col source (Hm, Wm = output grid Ho, Wo)
  const bf16_t* dy;       // [Mred][ldy], config block g*N
  int ldy;
  float* dw;              // [N][K] per config (fp32 grad arena)
  int64_t dw_gstride;
  int Mred, N, K;
  int m_per_split;
  int splits;
  int x_hl = 0, dy_hl = 0;  // HL-format operands (take_hi_lo)
  int gemm = 0;             // fp32: 1 = 1x1 / stride 1 / pad 0 (GM_GEMM body), 2 = k x k,
                            // stride 1, same-size output (GM_TAP body); 0 = im2col body
};

// es: element size of the gathered tensor (2 = bf16, 4 = fp32)
static GatherGeom make_geom(const void* src, int B, int Ctot, int Cg, int Hs, int Ws, int Hm,
                            int Wm, int kh, int kw, int st, int pad, int es = 2) {
  GatherGeom g{reinterpret_cast<const bf16_t*>(src), Ctot, Cg, Hs, Ws, Hm, Wm, kh, kw, st, pad,
               0u, {}, {}, {}, {}, {}, st, pad, Cg};
  const uint64_t bytes = (uint64_t)B * Hs * Ws * Ctot * (uint64_t)es;
  g.bytes = bytes < (1ull << 31) ? (uint32_t)bytes : 0u;
  g.dWm = make_div((uint32_t)Wm);
  g.dHm = make_div((uint32_t)Hm);
  g.dCg = make_div((uint32_t)Cg);
  g.dkw = make_div((uint32_t)kw);
  g.dst = make_div((uint32_t)st);
  return g;
}

// ---------------------------------------------------------------------------
// gather helpers
// ---------------------------------------------------------------------------
// Gather modes.  The fast modes (8-channel aligned operands) are branch-free:
// every 16-B chunk is one buffer_load whose byte offset is set past the
// descriptor's range for padding taps / out-of-range rows, so the hardware
// returns zeros.
enum { GM_SLOW = 0, GM_FWD = 1, GM_DG1 = 2, GM_DGS = 3, GM_GEMM = 4, GM_TAP = 5 };
//  GM_FWD : hi = y*st - pad + r                (forward, wgrad, strided-1x1 dgrad)
//  GM_DG1 : hi = y + pad - r                   (stride-1 dgrad)
//  GM_DGS : hi = (y + pad - r) / st if exact   (strided k x k dgrad)
// fp32 kernels only, "uniform K" modes: a 32-deep K step
// lies inside ONE tap, so the step's tap / channel offset is wave-uniform
// (scalar registers) and each thread keeps a per-row base offset computed
// once -- the K loop does one add and one select per 16-B chunk pair instead
// of the per-chunk im2col decode (FastDiv, bounds, the per-thread tap walk):
//  GM_GEMM: 1x1 pad-0 convs and linear layers (fwd, any stride; dgrad on
//           the 1x1 geometry, the strided one included; wgrad at stride 1):
//           the operand rows are the GEMM rows, K walked as channels
//  GM_TAP : k x k convs with Cg % 32 == 0 (fwd; stride-1 dgrad): a per-row
//           bit mask of the in-range taps replaces the per-chunk bounds test
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  // inputs made provably wave-uniform so the descriptor lives in SGPRs
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

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

// per-row state of the fast gather: tap-(0,0) coordinates and pixel index
struct RowA {
  int hy, wx, pix;
};

template <int GM>
__device__ __forceinline__ RowA row_init(const GatherGeom& g, int m, int M) {
  const RowPos p = decode_row(m, M, g);
  RowA a;
  if (GM == GM_FWD) {
    a.hy = p.y * g.st - g.pad;
    a.wx = p.x * g.st_w - g.pad_w;
  } else {
    a.hy = p.y + g.pad;
    a.wx = p.x + g.pad_w;
  }
  a.pix = (GM == GM_DGS) ? p.b * g.Hs : (p.b * g.Hs + a.hy) * g.Ws + a.wx;
  if (!p.ok) a.hy = -(1 << 29);  // every tap out of range
  return a;
}

// byte offset of channel c of tap (r, s) for a row, or OOB (-> zeros);
// ES = element size in bytes (2 bf16, 4 fp32)
template <int GM, int ES = 2>
__device__ __forceinline__ uint32_t a_off(const GatherGeom& g, const RowA& a, int r, int s, int c) {
  int hi, wi;
  uint32_t pix;
  if (GM == GM_FWD) {
    hi = a.hy + r;
    wi = a.wx + s;
    pix = (uint32_t)a.pix + (uint32_t)(r * g.Ws + s);
  } else if (GM == GM_DG1) {
    hi = a.hy - r;
    wi = a.wx - s;
    pix = (uint32_t)a.pix - (uint32_t)(r * g.Ws + s);
  } else {
    const int hn = a.hy - r, wn = a.wx - s;
    const uint32_t hq = fdiv((uint32_t)max(hn, 0), g.dst), wq = fdiv((uint32_t)max(wn, 0), g.dst);
    const bool exact = (hn >= 0) & (wn >= 0) & ((int)hq * g.st == hn) & ((int)wq * g.st == wn);
    hi = exact ? (int)hq : -1;
    wi = (int)wq;
    pix = ((uint32_t)a.pix + hq) * (uint32_t)g.Ws + wq;
  }
  const bool ok = ((unsigned)hi < (unsigned)g.Hs) & ((unsigned)wi < (unsigned)g.Ws);
  return ok ? (pix * (uint32_t)g.Ctot + (uint32_t)c) * (uint32_t)ES : OOB;
}

// --- generic (unaligned) path ------------------------------------------------
// source pixel offset (elements, without channel) or -1 when the tap is padding
__device__ __forceinline__ int64_t src_pixel(const GatherGeom& g, const RowPos& p, int r, int s,
                                             int dgrad) {
  int hi, wi;
  if (!dgrad) {
    hi = p.y * g.st - g.pad + r;
    wi = p.x * g.st_w - g.pad_w + s;
  } else {
    int hn = p.y + g.pad - r, wn = p.x + g.pad_w - s;
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

// per-element gather (channel counts not multiple of 8, e.g. the stem)
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
      if (off >= 0) e[i] = g.src[off + (int64_t)cfg * g.cfg_off + c];
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

template <int STEP = BK>
__device__ __forceinline__ void kpos_advance(const GatherGeom& g, KPos& kp) {
  kp.c += STEP;
  while (kp.c >= g.Cg) {
    kp.c -= g.Cg;
    if (++kp.s == g.kw) {
      kp.s = 0;
      ++kp.r;
    }
  }
}

// XCD-aware work order: the dispatcher deals consecutive block ids round-robin
// to the 8 XCDs (each with a private L2); remap so every XCD walks one
// contiguous range of (config, tile) work -> a config's weights and input
// rows stay in one L2.  Bijective for any grid size.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// ---------------------------------------------------------------------------
// NT LDS tile: [rows][64] bf16, 128-B rows, 16-B chunk c stored at
// c ^ ((row >> 1) & 7)  (conflict-free for the MFMA ds_read_b128 pattern)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int nt_off(int row, int chunk) {
  return row * BK + 8 * (chunk ^ ((row >> 1) & 7));
}

// epilogue store of a staged [BM][BN] bf16 tile (shared by the NT and NN kernels)
// EXT (the NN dgrad kernels): addend + BN-backward statistics, loads of
// PF rows issued together; otherwise (NT kernels) a plain store loop that
// still honours an addend (the unaligned dgrad fallback runs on NT).
template <int BM, int BN, bool EXT = false>
__device__ __forceinline__ void store_tile(const NTParams& p, const bf16_t* lds, int LDE, int cfg,
                                           int m0, int n0, int tid) {
  constexpr int OCPR = BN / 8;
  constexpr int LANES = NTHREADS / OCPR;    // rows in flight; a thread keeps one column chunk
  constexpr int NIT = BM * OCPR / NTHREADS;
  constexpr int PF = NIT > 4 ? 4 : NIT;     // rows per prefetch group (bounds the VGPRs)
  static_assert(NTHREADS % OCPR == 0 && NIT * NTHREADS == BM * OCPR && NIT % PF == 0,
                "store_tile mapping");
  bf16_t* obase = p.out + (int64_t)cfg * p.N;
  const bool vec_ok = ((p.N | p.ldc) & 7) == 0;
  const int cc = tid % OCPR, lane = tid / OCPR;
  const int ncol = n0 + 8 * cc;
  if (!EXT || !vec_ok) {  // (BN statistics need aligned channels: host-gated)
    for (int it = 0; it < NIT; ++it) {
      const int r = lane + it * LANES, m = m0 + r;
      if (m >= p.M || ncol >= p.N) continue;
      int64_t orow = m;
      if (p.o_st > 1) {
        const RowPos q = decode_row(m, p.M, p.a);
        orow = ((int64_t)q.b * p.o_H + (int64_t)q.y * p.o_st) * p.o_W + (int64_t)q.x * p.o_st;
      }
      bf16_t* dst = obase + orow * p.ldc + ncol;
      const bf16_t* src = lds + r * LDE + 8 * cc;
      if (vec_ok && !p.addend) {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
        continue;
      }
      for (int e = 0; e < 8 && ncol + e < p.N; ++e)
        dst[e] = p.addend ? f2bf(bf2f(src[e]) + bf2f(p.addend[(int64_t)cfg * p.N + orow * p.ldc +
                                                             ncol + e]))
                          : src[e];
    }
    return;
  }
  const BNBwdEpi& bb = p.bb;
  const bool bstat = bb.part != nullptr;
  float s8[8], q8[8], mu8[8], is8[8], sc8[8], sh8[8];
  if (bstat) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s8[e] = q8[e] = 0.f;
      const int n = min(ncol + e, p.N - 1);
      const int64_t c = (int64_t)cfg * p.N + n;
      mu8[e] = bb.mean[c];
      is8[e] = bb.invstd[c];
      if (bb.ym == 2) {                     // YM_Z: the forward's scale / shift
        const float ga = bf2f(bb.gamma[cfg * bb.gstride + n]);
        const float be = bf2f(bb.beta[cfg * bb.bstride + n]);
        sc8[e] = is8[e] * ga;
        sh8[e] = be - mu8[e] * sc8[e];
      }
    }
  }
  // per group of PF rows: issue the group's global loads (addend, BN input /
  // output) together, then store and accumulate
#pragma unroll
  for (int g0 = 0; g0 < NIT; g0 += PF) {
  int64_t orow[PF];
  bool ok[PF];
  uint4 ad[PF], zu[PF], yu[PF];
#pragma unroll
  for (int it = 0; it < PF; ++it) {
    const int m = m0 + lane + (g0 + it) * LANES;
    ok[it] = m < p.M && ncol < p.N;
    orow[it] = m;
    if (ok[it] && p.o_st > 1) {
      const RowPos q = decode_row(m, p.M, p.a);
      orow[it] = ((int64_t)q.b * p.o_H + (int64_t)q.y * p.o_st) * p.o_W + (int64_t)q.x * p.o_st;
    }
    const int64_t go = (int64_t)cfg * p.N + orow[it] * p.ldc + ncol;
    if (ok[it] && p.addend) ad[it] = *reinterpret_cast<const uint4*>(p.addend + go);
    if (ok[it] && bstat) {
      zu[it] = *reinterpret_cast<const uint4*>(bb.z + go);
      if (bb.ym == 1) yu[it] = *reinterpret_cast<const uint4*>(bb.y + go);
    }
  }
#pragma unroll
  for (int it = 0; it < PF; ++it) {
    if (!ok[it]) continue;
    const int r = lane + (g0 + it) * LANES;
    uint4 u = *reinterpret_cast<const uint4*>(lds + r * LDE + 8 * cc);
    if (p.addend) {
      // bf16(acc) + addend in fp32, one rounding: the same value an add
      // kernel over the two bf16 tensors would produce
      const uint32_t us[4] = {u.x, u.y, u.z, u.w},
                     ws[4] = {ad[it].x, ad[it].y, ad[it].z, ad[it].w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = __uint_as_float(us[k] << 16) + __uint_as_float(ws[k] << 16);
        const float hi =
            __uint_as_float(us[k] & 0xffff0000u) + __uint_as_float(ws[k] & 0xffff0000u);
        o[k] = pack_bf2(lo, hi);
      }
      u = make_uint4(o[0], o[1], o[2], o[3]);
    }
    *reinterpret_cast<uint4*>(obase + orow[it] * p.ldc + ncol) = u;
    if (bstat) {
      const uint32_t dw[4] = {u.x, u.y, u.z, u.w},
                     zw[4] = {zu[it].x, zu[it].y, zu[it].z, zu[it].w};
      uint32_t yw[4] = {0u, 0u, 0u, 0u};
      if (bb.ym == 1) {
        yw[0] = yu[it].x; yw[1] = yu[it].y; yw[2] = yu[it].z; yw[3] = yu[it].w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t shf = (e & 1) ? 0u : 16u, mk = 0xffff0000u;
        const float d = __uint_as_float((dw[e >> 1] << shf) & mk);
        const float zv = __uint_as_float((zw[e >> 1] << shf) & mk);
        float dz = d;
        if (bb.ym == 2) {
          dz = (zv * sc8[e] + sh8[e] + 0.f) > 0.f ? d : 0.f;
        } else if (bb.ym == 1) {
          const float yv = __uint_as_float((yw[e >> 1] << shf) & mk);
          dz = bb.act == 6 ? ((yv > 0.f && yv < 6.f) ? d : 0.f) : (yv > 0.f ? d : 0.f);
        }
        s8[e] += dz;
        q8[e] += dz * (zv - mu8[e]) * is8[e];
      }
    }
  }
  }
  if (!bstat) return;
  // rows of the tile -> one deterministic partial per (M tile, channel)
  float* xs = reinterpret_cast<float*>(const_cast<bf16_t*>(lds) + BM * LDE);  // [2][LANES][BN]
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    xs[lane * BN + 8 * cc + e] = s8[e];
    xs[(LANES + lane) * BN + 8 * cc + e] = q8[e];
  }
  __syncthreads();
  const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
  for (int t = tid; t < 2 * BN; t += NTHREADS) {
    const int q = t / BN, nl = t - q * BN, n = n0 + nl;
    if (n >= p.N) continue;
    float v = 0.f;
    for (int l = 0; l < LANES; ++l) v += xs[(q * LANES + l) * BN + nl];
    stat_store(bb.part, sb + (int64_t)q * p.ldc + n, v, p.stat_slabs);
  }
}

// In-launch hand-off (agent-scope release/acquire, cdna_hip_programming.md
// Guideline 16 recipe): every block of a group publishes its slab, then
// takes a ticket; returns true in the block that arrives last, after which
// all its threads may read the other blocks' slabs.  The last arriver
// re-zeroes the counter, so a persistent counter serves every replay.
// The published slabs are written with sc1 (write-through) stores and read
// back with sc1 loads, so no agent-scope release fence (= an L2 writeback,
// buffer_wbl2) is needed: every wave drains its stores, then one relaxed
// agent-scope ticket.
__device__ __forceinline__ bool last_arriver(unsigned* cnt, unsigned expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == expected - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// K-tile range [kt0, kt1) of this block's split
struct KRange {
  int kt0, kt1;
};

template <int STEP = BK>
__device__ __forceinline__ KRange split_range(const NTParams& p, int split) {
  const int KT = (p.K + STEP - 1) / STEP;
  const int per = (KT + p.splits - 1) / p.splits;
  const int kt0 = split * per;
  return KRange{kt0, min(KT, kt0 + per)};
}

// Split-K seam (fwd / dgrad GEMMs whose tile count cannot fill 256 CUs, e.g.
// the 4x4 / 7x7 stages of a one-config step): every split publishes its fp32
// accumulators to its own slot with write-through stores (thread-private
// layout, coalesced across the block); the last-arriving split of the tile
// re-reads all slots in split order (deterministic sum) and runs the normal
// epilogue.  Returns false in the blocks that must exit.
template <int BM, int BN>
__device__ __forceinline__ bool splitk_reduce(const NTParams& p, f32x4 (&acc)[BM / 32][BN / 32],
                                              int tile_id, int split, int tid) {
  constexpr int FI = BM / 32, FJ = BN / 32, NA = FI * FJ * 4;
  __shared__ int sk_flag;
  float* base = p.skws + (int64_t)tile_id * p.splits * (NA * NTHREADS);
  float* mine = base + (int64_t)split * (NA * NTHREADS);
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) st_sc1(mine + ((i * FJ + j) * 4 + e) * NTHREADS + tid, acc[i][j][e]);
  if (!last_arriver(p.skcnt + tile_id, (unsigned)p.splits, &sk_flag)) return false;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < p.splits; ++sp) {
    const float* src = base + (int64_t)sp * (NA * NTHREADS);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] += ld_sc1(src + ((i * FJ + j) * 4 + e) * NTHREADS + tid);
  }
  return true;
}

// sum over each 16-lane row of the wave (DPP butterfly, no LDS traffic)
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1,
                                                             0xF, 0xF, false));  // quad [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E,
                                                             0xF, 0xF, false));  // quad [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141,
                                                             0xF, 0xF, false));  // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140,
                                                             0xF, 0xF, false));  // row_mirror
  return v;
}

// Epilogue staging for the NT / NN kernels.  Their MFMAs take the weight
// fragment as the FIRST operand, so a lane's accumulator holds 4 consecutive
// output channels of one output row, C[16i + fr][16j + 4fc + e]: bias + act
// in fp32, one rounding, one 8-B LDS write per fragment.
template <int BM, int BN>
__device__ __forceinline__ void stage_c(const NTParams& p, bf16_t* lds,
                                        const f32x4 (&acc)[BM / 32][BN / 32], int cfg, int m0,
                                        int n0, int wm, int wn, int lane) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16, LDE = BN + 8;
  const int fr = lane & 15, fc = lane >> 4;
  float bc[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + wn * TN + 16 * j + 4 * fc + e;
      bc[j][e] = (p.bias && n < p.N) ? bf2f(p.bias[(int64_t)cfg * p.bias_gstride + n]) : 0.f;
    }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bc[j][e];
        v[e] = p.act == 6 ? fminf(fmaxf(v[e], 0.f), 6.f) : (p.act ? fmaxf(v[e], 0.f) : v[e]);
      }
      uint2 pk;
      pk.x = pack_bf2(v[0], v[1]);
      pk.y = pack_bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(lds + (wm * TM + 16 * i + fr) * LDE + wn * TN + 16 * j + 4 * fc) = pk;
    }
  if (p.stats) {
    // per-channel (sum, sum^2) of the ROUNDED outputs: in-lane over the i
    // fragments, DPP butterfly across the 16 lanes of equal fc, then the
    // two M-direction waves meet in LDS (stats_finish) -> one deterministic
    // partial per (M tile, channel).  Rows past M are zero (BN convs carry
    // no bias) and add nothing.
    float* xch = reinterpret_cast<float*>(lds + BM * LDE);  // [2 wm][2][BN]
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sm = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const float r = bf2f(f2bf(acc[i][j][e]));
          sm += r;
          sq += r * r;
        }
        sm = row16_sum(sm);
        sq = row16_sum(sq);
        if (fr == 0) {
          const int nl = wn * TN + 16 * j + 4 * fc + e;
          xch[(wm * 2) * BN + nl] = sm;
          xch[(wm * 2 + 1) * BN + nl] = sq;
        }
      }
  }
}

// second half of the fused BN statistics (after the epilogue barrier)
template <int BM, int BN>
__device__ __forceinline__ void stats_finish(const NTParams& p, const bf16_t* lds, int cfg, int m0,
                                             int n0, int tid) {
  if (!p.stats) return;
  constexpr int LDE = BN + 8;
  const float* xch = reinterpret_cast<const float*>(lds + BM * LDE);
  const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
  for (int t = tid; t < 2 * BN; t += NTHREADS) {
    const int q = t / BN, nl = t - q * BN, n = n0 + nl;
    if (n < p.N)
      stat_store(p.stats, sb + (int64_t)q * p.ldc + n, xch[q * BN + nl] + xch[(2 + q) * BN + nl],
                 p.stat_slabs);
  }
}

template <int BM, int BN, int GM>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_nt(NTParams p) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int CPR = BK / 8;                                  // 16-B chunks per row
  constexpr int A_CH = BM * CPR / NTHREADS, B_CH = BN * CPR / NTHREADS;
  constexpr int TILE_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + 8) + STAT_XCH;   // C tile + BN-stat exchange
  constexpr int LDS_ELEMS = TILE_ELEMS > EPI_ELEMS ? TILE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
#define SA(buf) (lds + (buf) * (BM * BK))
#define SB(buf) (lds + 2 * BM * BK + (buf) * (BN * BK))

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;       // splits of one tile: adjacent ids, one XCD
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KRange kr = split_range(p, split);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);                        // same for every i below
  const bf16_t* wbase = p.w + (int64_t)cfg * p.w_gstride;
  const bf16_t* abase = p.a.src + (int64_t)cfg * p.a.cfg_off;

  RowPos rows[A_CH];
  RowA rowa[A_CH];
  __amdgpu_buffer_rsrc_t rA, rB;
  if constexpr (GM != GM_SLOW) {
    rA = make_rsrc(abase, p.a.bytes);
    rB = make_rsrc(wbase, (uint32_t)p.N * (uint32_t)p.K * 2u);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) rowa[i] = row_init<GM>(p.a, m0 + (tid + NTHREADS * i) / CPR, p.M);
  } else {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) rows[i] = decode_row(m0 + (tid + NTHREADS * i) / CPR, p.M, p.a);
  }
  KPos kp = kpos_init(p.a, kr.kt0 * BK + 8 * my_chunk);
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + 8 * my_chunk;
    if constexpr (GM != GM_SLOW) {
      const bool kok = k0 < p.K;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const uint32_t off = a_off<GM>(p.a, rowa[i], kp.r, kp.s, kp.c);
        ra[i] = bload(rA, kok ? off : OOB);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid + NTHREADS * i) / CPR;
        rb[i] = bload(rB, (kok && n < p.N) ? (uint32_t)(n * p.K + k0) * 2u : OOB);
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

  load_tiles(kr.kt0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fc = lane >> 4;
  for (int kt = kr.kt0; kt < kr.kt1; ++kt) {
    const int cur = (kt - kr.kt0) & 1;
    if (kt + 1 < kr.kt1) load_tiles(kt + 1);
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kr.kt1) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // epilogue: stage the bf16 tile in LDS, then 16-B coalesced stores
  if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
  constexpr int LDE = BN + 8;
  stage_c<BM, BN>(p, lds, acc, cfg, m0, n0, wm, wn, lane);
  __syncthreads();
  stats_finish<BM, BN>(p, lds, cfg, m0, n0, tid);
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

// register-staged wgrad tile body; `work` = this block's (config, split, tile)
// index, `lds` = 2 * (BM + BN) * BK bf16
template <int BM, int BN, int GM>
__device__ __forceinline__ void wgrad_reg_body(const WGParams& p, int work, bf16_t* lds) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;           // 16-B chunks per tile row
  constexpr int A_CH = BK * A_CPR / NTHREADS, B_CH = BK * B_CPR / NTHREADS;
  constexpr int A_RSTEP = NTHREADS / A_CPR, B_RSTEP = NTHREADS / B_CPR;

  const int tiles_k = (p.K + BN - 1) / BN;
  const int tiles = ((p.N + BM - 1) / BM) * tiles_k;
  const int cfg = work / (tiles * p.splits);
  const int rem = work - cfg * tiles * p.splits;
  const int split = rem / tiles, tile = rem - split * tiles;
  const int tn_ = tile / tiles_k, tk = tile - tn_ * tiles_k;
  const int n0 = tn_ * BM, k0 = tk * BN;
  const int ms = split * p.m_per_split;
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
  const bf16_t* xb = p.x.src + (int64_t)cfg * p.x.cfg_off;
  __amdgpu_buffer_rsrc_t rDY, rX;
  if constexpr (GM != GM_SLOW) {
    rDY = make_rsrc(dyb, (uint32_t)p.Mred * (uint32_t)p.ldy * 2u);
    rX = make_rsrc(xb, p.x.bytes);
  }

  auto load_tiles = [&](int mt) {
    const int mbase = ms + mt * BK;
    if constexpr (GM != GM_SLOW) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int m = mbase + a_row0 + A_RSTEP * i, n = n0 + a_col;
        ra[i] = bload(rDY, (m < me && n < p.N) ? (uint32_t)(m * p.ldy + n) * 2u : OOB);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const RowA ra_ = row_init<GM_FWD>(p.x, mbase + b_row0 + B_RSTEP * i, me);
        const uint32_t off = a_off<GM_FWD>(p.x, ra_, bk.r, bk.s, bk.c);
        rb[i] = bload(rX, b_kok ? off : OOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int m = mbase + a_row0 + A_RSTEP * i, n = n0 + a_col;
        uint16_t e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (m < me && n < p.N) {
          const bf16_t* src = dyb + (int64_t)m * p.ldy + n;
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (n + t < p.N) ? src[t] : 0;
        }
        ra[i] = pack8(e);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int m = mbase + b_row0 + B_RSTEP * i;
        const RowPos pos = decode_row(m, me, p.x);
        rb[i] = (b_kok && pos.ok) ? gather_chunk_slow(p.x, cfg, pos, kk0, p.K, 0)
                                  : make_uint4(0, 0, 0, 0);
      }
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
  const bool split_k = p.splits > 1;
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
          if (split_k)
            atomicAdd(d, acc[i][j][e]);
          else
            *d = acc[i][j][e];
        }
      }
}

template <int BM, int BN, int GM>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_wgrad(WGParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (BM + BN) * BK];
  wgrad_reg_body<BM, BN, GM>(p, xcd_remap(blockIdx.x, gridDim.x), lds);
}


// ---------------------------------------------------------------------------
// NN (dgrad) kernel: A = col2im(dy) K-contiguous (NT-style LDS, ds_read_b128),
// B = W read as [k = (tap, cout)] x [cin] rows straight from the arena (TN-
// style LDS, ds_read_b64_tr_b16) -> no per-step weight transpose.
//   dx[m, c] = sum_{tap, n} dy~[m, (tap, n)] * W[n][tap][c]
// GM_DG1 (stride 1, and the strided-1x1 case on the dy grid) or GM_DGS.
// ---------------------------------------------------------------------------
template <int BM, int BN, int GM>
__global__ __launch_bounds__(NTHREADS, 2) void igemm_nn_dgrad(NTParams p, int T, FastDiv dCout) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int CPR = BK / 8;
  constexpr int A_CH = BM * CPR / NTHREADS;
  constexpr int B_CPR = BN / 8, B_CH = BK * B_CPR / NTHREADS, B_RSTEP = NTHREADS / B_CPR;
  constexpr int TILE_ELEMS = 2 * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + 8) + STAT_XCH;   // C tile + BN-stat exchange
  constexpr int LDS_ELEMS = TILE_ELEMS > EPI_ELEMS ? TILE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;       // splits of one tile: adjacent ids, one XCD
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KRange kr = split_range(p, split);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);
  const int Cout = p.a.Cg;          // reduction channels (k = tap*Cout + n)
  const int Cin = p.N;              // output channels
  const bf16_t* wbase = p.w + (int64_t)cfg * p.w_gstride;
  const bf16_t* abase = p.a.src + (int64_t)cfg * p.a.cfg_off;
  const int b_col = 8 * (tid % B_CPR), b_row0 = tid / B_CPR;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(abase, p.a.bytes);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(wbase, (uint32_t)Cout * (uint32_t)T * (uint32_t)Cin * 2u);

  RowA rowa[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) rowa[i] = row_init<GM>(p.a, m0 + (tid + NTHREADS * i) / CPR, p.M);
  KPos kp = kpos_init(p.a, kr.kt0 * BK + 8 * my_chunk);
  uint4 ra[A_CH], rb[B_CH];

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + 8 * my_chunk;
    const bool kok = k0 < p.K;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const uint32_t off = a_off<GM>(p.a, rowa[i], kp.r, kp.s, kp.c);
      ra[i] = bload(rA, kok ? off : OOB);
    }
    kpos_advance(p.a, kp);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int k = kt * BK + b_row0 + B_RSTEP * i;
      const int c = n0 + b_col;
      const int tap = (int)fdiv((uint32_t)k, dCout);
      const int n = k - tap * Cout;
      rb[i] = bload(rW, (k < p.K && c < Cin) ? (uint32_t)((n * T + tap) * Cin + c) * 2u : OOB);
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

  load_tiles(kr.kt0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fc = lane >> 4;
  for (int kt = kr.kt0; kt < kr.kt1; ++kt) {
    const int cur = (kt - kr.kt0) & 1;
    if (kt + 1 < kr.kt1) load_tiles(kt + 1);
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kr.kt1) store_tiles(cur ^ 1);
    __syncthreads();
  }
  if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
  constexpr int LDE = BN + 8;
  stage_c<BM, BN>(p, lds, acc, cfg, m0, n0, wm, wn, lane);
  __syncthreads();
  stats_finish<BM, BN>(p, lds, cfg, m0, n0, tid);
  store_tile<BM, BN, true>(p, lds, LDE, cfg, m0, n0, tid);
}

#undef SA
#undef SB

// ===========================================================================
// Pipelined kernels (8/64-channel aligned operands): operand tiles go
// global -> LDS by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction,
// padding / out-of-range chunks zero-filled by the descriptor range check)
// into an S-stage LDS ring.  One raw barrier per 64-deep K-step, a counted
// vmcnt keeps the next stage's DMA in flight across it (S = 3: two K-steps of
// loads overlap each K-step's MFMAs), no VGPR staging, no ds_write pass.
// The LDS images are the same swizzled layouts as above; the swizzle is
// applied to the per-lane SOURCE address because a DMA piece lands
// lane-linearly in LDS.
// ===========================================================================
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, bf16_t* dst, uint32_t voff,
                                       uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// 16-B column index (global) of LDS slot col16 of a TN tile row (tn_off swizzle)
template <int COLS>
__device__ __forceinline__ int tn_col16(int row, int col16) {
  int sw;
  if (COLS == 128)
    sw = (row & 3) | (((row >> 3) & 1) << 2);
  else
    sw = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return col16 ^ (2 * sw);
}

// NT-image MFMA step over one 64-deep stage: A [BM][64], B [BN][64]
template <int BM, int BN>
__device__ __forceinline__ void mma_nt(const bf16_t* sa, const bf16_t* sb, int wm, int wn, int lane,
                                       f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc + 4 * kk));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(sb + nt_off(wn * TN + 16 * j + fr, fc + 4 * kk));
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
}

// A as NT image, B as TN image (dgrad)
template <int BM, int BN>
__device__ __forceinline__ void mma_nn(const bf16_t* sa, const bf16_t* sb, int wm, int wn, int lane,
                                       f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
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
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
}

// both TN images (wgrad)
template <int BM, int BN>
__device__ __forceinline__ void mma_tn(const bf16_t* sa, const bf16_t* sb, int wm, int wn, int lane,
                                       f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = tn_frag<BM>(sa, 32 * kk, wm * TM + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = tn_frag<BN>(sb, 32 * kk, wn * TN + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
}

// S-stage ring driver: issue(t, stage) queues tile t's DMA pieces (LPW per
// wave), mma(stage) consumes one stage.
template <int S, int LPW, typename Issue, typename Mma>
__device__ __forceinline__ void ring_loop(int KT, Issue&& issue, Mma&& mma) {
  issue(0, 0);
  if (S > 2 && KT > 1) issue(1, 1);
  int st = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if (S > 2 && kt + 1 < KT)
      wait_vm<LPW>();          // tile kt landed; tile kt+1 stays in flight
    else
      wait_vm<0>();
    lds_barrier();             // tile kt visible to all waves; stage (kt-1) % S free
    const int nxt = kt + S - 1;
    if (nxt < KT) issue(nxt, (st + S - 1) % S);
    mma(st);
    st = (st + 1 == S) ? 0 : st + 1;
  }
  lds_barrier();               // every wave done reading before LDS is reused
}

template <int BM, int BN>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[BM / 32][BN / 32]) {
#pragma unroll
  for (int i = 0; i < BM / 32; ++i)
#pragma unroll
    for (int j = 0; j < BN / 32; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// forward: y = act(im2col(x) W^T + b); requires Cg % 64 == 0
template <int BM, int BN, int S>
__global__ __launch_bounds__(NTHREADS, 2) void pipe_nt(NTParams p) {
  constexpr int AJ = BM / 32, BJ = BN / 32, LPW = AJ + BJ;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int EPI = BM * (BN + 8) + STAT_XCH;   // C tile + BN-stat exchange
  constexpr int LDS_ELEMS = S * STAGE > EPI ? S * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;       // splits of one tile: adjacent ids, one XCD
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KRange kr = split_range(p, split);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const auto rA = make_rsrc(p.a.src + (int64_t)cfg * p.a.cfg_off, p.a.bytes);
  const auto rB = make_rsrc(p.w + (int64_t)cfg * p.w_gstride, (uint32_t)p.N * (uint32_t)p.K * 2u);

  RowA arow[AJ];
  int achan[AJ];
  uint32_t boff[BJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int row = (wid * AJ + j) * 8 + (lane >> 3);
    achan[j] = 8 * ((lane & 7) ^ ((row >> 1) & 7));
    arow[j] = row_init<GM_FWD>(p.a, m0 + row, p.M);
  }
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int row = (wid * BJ + j) * 8 + (lane >> 3);
    const int n = n0 + row;
    boff[j] = n < p.N ? (uint32_t)(n * p.K + 8 * ((lane & 7) ^ ((row >> 1) & 7))) * 2u : OOB;
  }
  // tap / channel of the next K tile to issue (uniform; Cg % 64 == 0: a K tile
  // never straddles taps)
  int tc = (kr.kt0 * BK) % p.a.Cg, tr = (kr.kt0 * BK) / p.a.Cg;
  int ts = tr % p.a.kw;
  tr /= p.a.kw;
  auto issue = [&](int kt, int st) {
    bf16_t* sa = lds + st * STAGE;
    bf16_t* sb = sa + BM * BK;
#pragma unroll
    for (int j = 0; j < AJ; ++j)
      glds16(rA, sa + (wid * AJ + j) * 512, a_off<GM_FWD>(p.a, arow[j], tr, ts, tc + achan[j]), 0);
#pragma unroll
    for (int j = 0; j < BJ; ++j) glds16(rB, sb + (wid * BJ + j) * 512, boff[j], (uint32_t)kt * (BK * 2));
    tc += BK;
    if (tc == p.a.Cg) {
      tc = 0;
      if (++ts == p.a.kw) {
        ts = 0;
        ++tr;
      }
    }
  };
  f32x4 acc[BM / 32][BN / 32];
  zero_acc<BM, BN>(acc);
  ring_loop<S, LPW>(kr.kt1 - kr.kt0, [&](int t, int st) { issue(kr.kt0 + t, st); }, [&](int st) {
    mma_nt<BM, BN>(lds + st * STAGE, lds + st * STAGE + BM * BK, wm, wn, lane, acc);
  });

  if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
  constexpr int LDE = BN + 8;
  stage_c<BM, BN>(p, lds, acc, cfg, m0, n0, wm, wn, lane);
  __syncthreads();
  stats_finish<BM, BN>(p, lds, cfg, m0, n0, tid);
  store_tile<BM, BN>(p, lds, LDE, cfg, m0, n0, tid);
}

// dgrad: dx = col2im(dy) * W; requires Cout % 64 == 0, Cin % 8 == 0
template <int BM, int BN, int S, int GM>
__global__ __launch_bounds__(NTHREADS, 2) void pipe_nn(NTParams p, int T) {
  constexpr int AJ = BM / 32, BJ = BN / 32, LPW = AJ + BJ;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int EPI = BM * (BN + 8) + STAT_XCH;   // C tile + BN-stat exchange
  constexpr int LDS_ELEMS = S * STAGE > EPI ? S * STAGE : EPI;
  constexpr int BROWS = 512 / BN, BC16 = BN / 8;   // rows / 16-B columns per B piece
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;       // splits of one tile: adjacent ids, one XCD
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KRange kr = split_range(p, split);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int Cout = p.a.Cg, Cin = p.N;
  const auto rA = make_rsrc(p.a.src + (int64_t)cfg * p.a.cfg_off, p.a.bytes);
  const auto rW = make_rsrc(p.w + (int64_t)cfg * p.w_gstride,
                            (uint32_t)Cout * (uint32_t)T * (uint32_t)Cin * 2u);

  RowA arow[AJ];
  int achan[AJ];
  uint32_t boff[BJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int row = (wid * AJ + j) * 8 + (lane >> 3);
    achan[j] = 8 * ((lane & 7) ^ ((row >> 1) & 7));
    arow[j] = row_init<GM>(p.a, m0 + row, p.M);
  }
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int row = (wid * BJ + j) * BROWS + lane / BC16;
    const int c = n0 + 8 * tn_col16<BN>(row, lane % BC16);
    boff[j] = c < Cin ? (uint32_t)(row * T * Cin + c) * 2u : OOB;
  }
  int tc = (kr.kt0 * BK) % Cout, tr = (kr.kt0 * BK) / Cout;
  int ts = tr % p.a.kw;
  tr /= p.a.kw;
  auto issue = [&](int kt, int st) {
    bf16_t* sa = lds + st * STAGE;
    bf16_t* sb = sa + BM * BK;
#pragma unroll
    for (int j = 0; j < AJ; ++j)
      glds16(rA, sa + (wid * AJ + j) * 512, a_off<GM>(p.a, arow[j], tr, ts, tc + achan[j]), 0);
    const uint32_t wso = (uint32_t)(tc * T + tr * p.a.kw + ts) * (uint32_t)Cin * 2u;
#pragma unroll
    for (int j = 0; j < BJ; ++j) glds16(rW, sb + (wid * BJ + j) * 512, boff[j], wso);
    tc += BK;
    if (tc == Cout) {
      tc = 0;
      if (++ts == p.a.kw) {
        ts = 0;
        ++tr;
      }
    }
  };
  f32x4 acc[BM / 32][BN / 32];
  zero_acc<BM, BN>(acc);
  ring_loop<S, LPW>(kr.kt1 - kr.kt0, [&](int t, int st) { issue(kr.kt0 + t, st); }, [&](int st) {
    mma_nn<BM, BN>(lds + st * STAGE, lds + st * STAGE + BM * BK, wm, wn, lane, acc);
  });

  if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
  constexpr int LDE = BN + 8;
  stage_c<BM, BN>(p, lds, acc, cfg, m0, n0, wm, wn, lane);
  __syncthreads();
  stats_finish<BM, BN>(p, lds, cfg, m0, n0, tid);
  store_tile<BM, BN, true>(p, lds, LDE, cfg, m0, n0, tid);
}

// wgrad: dW[n, k] = sum_m dy[m, n] im2col(x)[m, k]; requires Cin % 8 == 0, Cout % 8 == 0
// LDS-DMA ring wgrad tile body; `lds` = S * (BM + BN) * BK bf16
template <int BM, int BN, int S>
__device__ __forceinline__ void wgrad_pipe_body(const WGParams& p, int work, bf16_t* lds) {
  constexpr int AJ = BM / 32, BJ = BN / 32, LPW = AJ + BJ;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int AROWS = 512 / BM, AC16 = BM / 8, BROWS = 512 / BN, BC16 = BN / 8;

  const int tiles_k = (p.K + BN - 1) / BN;
  const int tiles = ((p.N + BM - 1) / BM) * tiles_k;
  const int cfg = work / (tiles * p.splits);
  const int rem = work - cfg * tiles * p.splits;
  const int split = rem / tiles, tile = rem - split * tiles;
  const int tn_ = tile / tiles_k, tk = tile - tn_ * tiles_k;
  const int n0 = tn_ * BM, k0 = tk * BN;
  const int ms = split * p.m_per_split;
  const int me = min(p.Mred, ms + p.m_per_split);
  if (ms >= me) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const auto rDY = make_rsrc(p.dy + (int64_t)cfg * p.N, (uint32_t)p.Mred * (uint32_t)p.ldy * 2u);
  const auto rX = make_rsrc(p.x.src + (int64_t)cfg * p.x.cfg_off, p.x.bytes);

  int arow[AJ];
  uint32_t aoff[AJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    arow[j] = (wid * AJ + j) * AROWS + lane / AC16;
    const int n = n0 + 8 * tn_col16<BM>(arow[j], lane % AC16);
    aoff[j] = n < p.N ? (uint32_t)(arow[j] * p.ldy + n) * 2u : OOB;
  }
  int brow[BJ];
  KPos bk[BJ];
  bool bok[BJ];
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    brow[j] = (wid * BJ + j) * BROWS + lane / BC16;
    const int k = k0 + 8 * tn_col16<BN>(brow[j], lane % BC16);
    bok[j] = k < p.K;
    bk[j] = kpos_init(p.x, bok[j] ? k : 0);
  }
  auto issue = [&](int mt, int st) {
    bf16_t* sa = lds + st * STAGE;
    bf16_t* sb = sa + BM * BK;
    const int mbase = ms + mt * BK, lim = me - mbase;
    const uint32_t so = (uint32_t)mbase * (uint32_t)p.ldy * 2u;
#pragma unroll
    for (int j = 0; j < AJ; ++j) glds16(rDY, sa + (wid * AJ + j) * 512, arow[j] < lim ? aoff[j] : OOB, so);
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const RowA ra = row_init<GM_FWD>(p.x, mbase + brow[j], me);
      const uint32_t off = a_off<GM_FWD>(p.x, ra, bk[j].r, bk[j].s, bk[j].c);
      glds16(rX, sb + (wid * BJ + j) * 512, bok[j] ? off : OOB, 0);
    }
  };
  f32x4 acc[BM / 32][BN / 32];
  zero_acc<BM, BN>(acc);
  ring_loop<S, LPW>((me - ms + BK - 1) / BK, issue, [&](int st) {
    mma_tn<BM, BN>(lds + st * STAGE, lds + st * STAGE + BM * BK, wm, wn, lane, acc);
  });

  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  float* dwb = p.dw + (int64_t)cfg * p.dw_gstride;
  const int fr = lane & 15, fc = lane >> 4;
  const bool split_k = p.splits > 1;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wm * TM + 16 * i + 4 * fc + e;
        const int k = k0 + wn * TN + 16 * j + fr;
        if (n < p.N && k < p.K) {
          float* d = dwb + (int64_t)n * p.K + k;
          if (split_k)
            atomicAdd(d, acc[i][j][e]);
          else
            *d = acc[i][j][e];
        }
      }
}

template <int BM, int BN, int S>
__global__ __launch_bounds__(NTHREADS, 2) void pipe_wg(WGParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[S * (BM + BN) * BK];
  wgrad_pipe_body<BM, BN, S>(p, xcd_remap(blockIdx.x, gridDim.x), lds);
}

// ---------------------------------------------------------------------------
// Batched weight gradients: the wgrads of up to WGB_MAX conv layers in ONE
// launch.  Each layer's wgrad only feeds the optimizer, so the engine defers
// them during backward (ops.streams) and flushes them together: one launch
// instead of one per layer, and the small late-stage layers of a one-config
// step (a few dozen tiles each) share the chip instead of running alone.
// Block b (XCD-remapped) belongs to the layer whose [start, start + blocks)
// range holds it; every layer splits its reduction into chunks of at most
// `rows` GEMM rows so all blocks carry similar work.
// ---------------------------------------------------------------------------
constexpr int WGB_MAX = 20;
struct WGBatch {
  int n;
  int start[WGB_MAX + 1];
  WGParams p[WGB_MAX];
};
static_assert(sizeof(WGBatch) <= 4096, "WGBatch must fit the 4 KB kernel-argument segment");

template <int BM, int BN, int KIND>  // KIND 0: register-staged, 1: LDS-DMA ring (2 stages)
__global__ __launch_bounds__(NTHREADS, 2) void wgrad_batch(WGBatch b) {
  constexpr int LDSE = 2 * (BM + BN) * BK;   // both bodies use two stages
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDSE];
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  int i = 0;
  while (i + 1 < b.n && work >= b.start[i + 1]) ++i;
  const WGParams p = b.p[i];
  if (KIND == 0)
    wgrad_reg_body<BM, BN, GM_FWD>(p, work - b.start[i], lds);
  else
    wgrad_pipe_body<BM, BN, 2>(p, work - b.start[i], lds);
}

// ===========================================================================
// fp32 (reference-precision) path: 3-pass split-bf16 MFMA
// ===========================================================================
// The reference trains in fp32 (TF 1.14 / PyTorch 1.4 defaults).  In this
// mode every operand and output stays fp32 in HBM; gfx950 has no xf32, and
// its fp32 MFMA runs at 1/16 of the bf16 rate, so products go through the
// bf16 matrix cores in three passes instead:
//   v = hi + lo,  hi = bf16(v),  lo = bf16(v - hi)     (v - hi is exact)
//   a * b ~= ah*bh + ah*bl + al*bh                      (al*bl ~ 2^-16 |ab| dropped)
// with fp32 accumulation: per-product relative error <= ~2^-15, fp32 level
// for training (tests: relative L2 error vs an fp64 reference <= 1e-4).
// Operands are register-staged (global fp32 -> split -> LDS).  A stage
// covers KS = 32 reduction elements and lands in the SAME LDS images as the
// bf16 kernels: for K-contiguous (NT) rows hi sits in chunks 0-3 and lo in
// chunks 4-7; for TN tiles hi fills reduction rows 0-31 and lo rows 32-63.
// The bf16 fragment reads of substep kk = 0 / 1 thus return the hi / lo
// fragments of the same 32 k, and each fragment pair takes three MFMAs.
// Epilogues write fp32 straight from the accumulators (a lane holds 4
// consecutive output channels of one row: one 16-B store).
constexpr int KS = 32;

// 8 fp32 (two 16-B loads) -> 8 bf16 hi + 8 bf16 lo
// CER_TIMING_NOSPLIT / CER_TIMING_1PASS: timing-only A/B builds (wrong
// numerics): no hi/lo split VALU, or one MFMA per fragment pair instead of
// three -- what the split and the extra passes cost (tools.conv_one)
#ifndef CER_TIMING_NOSPLIT
#define CER_TIMING_NOSPLIT 0
#endif
#ifndef CER_TIMING_NOAW
#define CER_TIMING_NOAW 0       // timing only: no LDS stores of the A operand (loads kept)
#endif
#ifndef CER_TIMING_1PASS
#define CER_TIMING_1PASS 0
#endif
__device__ __forceinline__ void split_hi_lo(const uint4& a, const uint4& b, uint4& hi, uint4& lo) {
  if (CER_TIMING_NOSPLIT) {
    hi = a;
    lo = b;
    return;
  }
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = __uint_as_float(w[2 * i]), x1 = __uint_as_float(w[2 * i + 1]);
    const uint32_t hp = cvt_pk_bf16(x0, x1);
    h[i] = hp;
    l[i] = cvt_pk_bf16(x0 - __uint_as_float(hp << 16), x1 - __uint_as_float(hp & 0xffff0000u));
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

// HL operand format (conv-only activations and BN-backward gradients, see
// cer_conv_set_hl): every 8 channels are stored as [8 x bf16 hi | 8 x bf16
// lo] of the fp32 values, split exactly as split_hi_lo does -- the same 32
// bytes at the same offsets as 8 fp32, so the gathers are unchanged and the
// 3-pass MFMAs see bit-identical operands.  An HL chunk IS the (hi, lo) pair.
// timing builds: keep a loaded value (and its load) without using it
__device__ __forceinline__ void keep_alive(const uint4& v) {
  asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
}

__device__ __forceinline__ void take_hi_lo(bool hl, const uint4& a, const uint4& b, uint4& hi,
                                           uint4& lo) {
  if (hl) {
    hi = a;
    lo = b;
  } else {
    split_hi_lo(a, b, hi, lo);
  }
}

__device__ __forceinline__ uint4 f4_bits(const float* e) {
  return make_uint4(__float_as_uint(e[0]), __float_as_uint(e[1]), __float_as_uint(e[2]),
                    __float_as_uint(e[3]));
}

// per-element fp32 im2col gather of an 8-wide k chunk (unaligned operands)
__device__ __forceinline__ void gather_chunk_slow32(const GatherGeom& g, int cfg, const RowPos& p,
                                                    int k0, int K, int dgrad, uint4& c0,
                                                    uint4& c1) {
  const float* src = reinterpret_cast<const float*>(g.src);
  float e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    e[i] = 0.f;
    const int k = k0 + i;
    if (k < K) {
      const int tap = (int)fdiv((uint32_t)k, g.dCg), c = k - tap * g.Cg;
      const int r = (int)fdiv((uint32_t)tap, g.dkw), s = tap - r * g.kw;
      const int64_t off = src_pixel(g, p, r, s, dgrad);
      if (off >= 0) e[i] = src[off + (int64_t)cfg * g.cfg_off + c];
    }
  }
  c0 = f4_bits(e);
  c1 = f4_bits(e + 4);
}

// 8 consecutive fp32 of a row (bounds per element), as two uint4
__device__ __forceinline__ void load_row8_slow32(const float* src, int valid, uint4& c0,
                                                 uint4& c1) {
  float e[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) e[t] = t < valid ? src[t] : 0.f;
  c0 = f4_bits(e);
  c1 = f4_bits(e + 4);
}

// three MFMAs per fragment pair: (first operand, second operand) = (x, y)
__device__ __forceinline__ f32x4 mfma3(const bf16x8& xh, const bf16x8& xl, const bf16x8& yh,
                                       const bf16x8& yl, f32x4 acc) {
  if (CER_TIMING_1PASS) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, yh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl, yh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, yl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh, yh, acc, 0, 0, 0);
}

// fp32 K loop: register-staged operands through a double-buffered LDS
// image, ONE barrier per KS-deep step.  With CER_FP32_PF = 2 two register
// sets alternate, so the global loads of step k+2 are issued before the
// MFMAs of step k and land in LDS only at the end of step k+1: two steps of
// MFMA work (2 x 768 cycles per wave at 128x128) cover the L2 / HBM latency
// instead of one.  ``load(k, S)`` / ``store(buf, S)`` take the register set
// as a std::integral_constant so every index stays compile-time (no
// scratch); ``mma(buf)`` consumes LDS buffer ``buf`` (0 / 1 by step parity).
// 128x128 tiles stay at one set: the second one (+32 VGPRs) would push them
// past the 256-VGPR budget of 2 workgroups per CU (spills).
#ifndef CER_FP32_PF
#define CER_FP32_PF 2
#endif
#ifndef CER_FP32_PF_SMALL
#define CER_FP32_PF_SMALL CER_FP32_PF
#endif
#ifndef CER_FP32_PF_BIG
#define CER_FP32_PF_BIG 1
#endif
// The wide (32x32x16) 128x128 forward holds ~45 fewer VGPRs than the
// 16x16x32 one (169 vs 215 at one set), but a second set still spills (256
// VGPRs + 28-204 B scratch), so it stays at one (knob kept for A/B builds).
#ifndef CER_FP32W_PF_BIG
#define CER_FP32W_PF_BIG 1
#endif
// workgroups per CU the big (128x128) fp32 tiles are compiled for (the
// launch bound: 2 = 256 registers per lane; 1 = 512, room for a second
// prefetch set at half the waves -- an A/B build knob)
#ifndef CER_BIG_OCC
#define CER_BIG_OCC 2
#endif
template <int BM, int BN>
constexpr int fp32_occ() {
  return BM * BN > 128 * 64 ? CER_BIG_OCC : 2;
}
template <int BM, int BN, bool WIDE = false>
constexpr int fp32_sets() {
  return BM * BN > 128 * 64 ? (WIDE ? CER_FP32W_PF_BIG : CER_FP32_PF_BIG)
                            : BM * BN > 64 * 64 ? CER_FP32_PF : CER_FP32_PF_SMALL;
}
// the weight-gradient body holds ~45-85 fewer registers than the NT / NN
// kernels at one set (170 at 128x128): its big tiles may take two
// (CER_WG_PF_BIG; A/B build knob)
#ifndef CER_WG_PF_BIG
#define CER_WG_PF_BIG CER_FP32_PF_BIG
#endif
template <int BM, int BN>
constexpr int wgrad_sets() {
  return BM * BN > 128 * 64 ? CER_WG_PF_BIG : fp32_sets<BM, BN>();
}
using RS0 = std::integral_constant<int, 0>;

template <int SETS, typename Load, typename Store, typename Mma>
__device__ __forceinline__ void kloop32(int k0, int k1, Load&& load, Store&& store, Mma&& mma) {
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, (1 % SETS)>;
  using I2 = std::integral_constant<int, (2 % SETS)>;
  using I3 = std::integral_constant<int, (3 % SETS)>;
  load(k0, I0{});
  store(0, I0{});
  if constexpr (SETS > 1) {
    // register ring of SETS sets: the loads of step k + SETS are issued (into
    // the set step k just emptied) before the MFMAs of step k and land in LDS
    // at the end of step k + SETS - 1, so SETS steps of MFMA work cover the
    // load latency.  Loads past k1 are issued anyway (out-of-range offsets,
    // the buffer loads return zeros): no branch around a load, so the
    // compiler keeps counted vmcnt waits instead of draining at every join;
    // the breaks below are loop exits only.
    load(k0 + 1, I1{});
    if constexpr (SETS > 2) load(k0 + 2, I2{});
    if constexpr (SETS > 3) load(k0 + 3, I3{});
    __syncthreads();
    auto step = [&](int k, auto U, auto U1) {
      load(k + SETS, U);
      const int buf = (k - k0) & 1;
      mma(buf);
      store(buf ^ 1, U1);
      __syncthreads();
    };
    for (int kt = k0; kt < k1; kt += SETS) {
      step(kt, I0{}, I1{});
      if (kt + 1 >= k1) break;
      if constexpr (SETS == 2) {
        step(kt + 1, I1{}, I0{});
      } else {
        step(kt + 1, I1{}, I2{});
        if (kt + 2 >= k1) break;
        if constexpr (SETS == 3) {
          step(kt + 2, I2{}, I0{});
        } else {
          step(kt + 2, I2{}, I3{});
          if (kt + 3 >= k1) break;
          step(kt + 3, I3{}, I0{});
        }
      }
    }
  } else {
    __syncthreads();
    for (int kt = k0; kt < k1; ++kt) {
      const int cur = (kt - k0) & 1;
      if (kt + 1 < k1) load(kt + 1, I0{});
      mma(cur);
      if (kt + 1 < k1) store(cur ^ 1, I0{});
      __syncthreads();
    }
  }
}

// A: NT image, B: NT image (forward)
template <int BM, int BN>
__device__ __forceinline__ void mma3_nt(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                        int lane, f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
  bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    ah[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc));
    al[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc + 4));
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    bh[j] = *reinterpret_cast<const bf16x8*>(sb + nt_off(wn * TN + 16 * j + fr, fc));
    bl[j] = *reinterpret_cast<const bf16x8*>(sb + nt_off(wn * TN + 16 * j + fr, fc + 4));
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = mfma3(bh[j], bl[j], ah[i], al[i], acc[i][j]);
}

// A: NT image, B: TN image (dgrad)
template <int BM, int BN>
__device__ __forceinline__ void mma3_nn(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                        int lane, f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
  bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    ah[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc));
    al[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 16 * i + fr, fc + 4));
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    bh[j] = tn_frag<BN>(sb, 0, wn * TN + 16 * j, lane);
    bl[j] = tn_frag<BN>(sb, KS, wn * TN + 16 * j, lane);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = mfma3(bh[j], bl[j], ah[i], al[i], acc[i][j]);
}

// both TN images (wgrad)
template <int BM, int BN>
__device__ __forceinline__ void mma3_tn(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                        int lane, f32x4 (&acc)[BM / 32][BN / 32]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    ah[i] = tn_frag<BM>(sa, 0, wm * TM + 16 * i, lane);
    al[i] = tn_frag<BM>(sa, KS, wm * TM + 16 * i, lane);
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    bh[j] = tn_frag<BN>(sb, 0, wn * TN + 16 * j, lane);
    bl[j] = tn_frag<BN>(sb, KS, wn * TN + 16 * j, lane);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = mfma3(ah[i], al[i], bh[j], bl[j], acc[i][j]);
}

// fp32 epilogue of the NT / NN kernels, straight from the accumulators
// (reference form; epi32 below is the prefetching one):
// lane (fr, fc) of wave (wm, wn) owns rows wm*TM + 16i + fr and channels
// wn*TN + 16j + 4fc .. +3.  out = act(acc + bias) (+ addend), one 16-B
// store per fragment; optional per-(M tile, channel) statistics partials:
// forward BN (sum, sum^2) of the outputs (p.stats) or the BN-backward
// (sum dz, sum dz*xhat) of a dgrad output (p.bb.part, BNBwdEpi).  xch: LDS
// scratch of 4*BN floats.
template <int BM, int BN>
__device__ __forceinline__ void epi32_ref(const NTParams& p, const f32x4 (&acc)[BM / 32][BN / 32],
                                      float* xch, int cfg, int m0, int n0, int wm, int wn,
                                      int lane, int tid) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
  float* obase = reinterpret_cast<float*>(p.out) + (int64_t)cfg * p.N;
  const float* adb =
      p.addend ? reinterpret_cast<const float*>(p.addend) + (int64_t)cfg * p.N : nullptr;
  const BNBwdEpi& bb = p.bb;
  const bool fstat = p.stats != nullptr;
  const bool bstat = bb.part != nullptr;
  const bool vec = ((p.N | p.ldc) & 3) == 0;
  const float* zb = bstat ? reinterpret_cast<const float*>(bb.z) + (int64_t)cfg * p.N : nullptr;
  const float* yb = bstat && bb.ym == 1 ? reinterpret_cast<const float*>(bb.y) + (int64_t)cfg * p.N
                                       : nullptr;
  // ym 3 (bn.hip YM_M): the activation mask as bits, [M][ldc / 8] bytes
  const uint8_t* mb = bstat && bb.ym == 3 ? reinterpret_cast<const uint8_t*>(bb.y) : nullptr;
  float bc[FN][4], mu[FN][4], is[FN][4], sc[FN][4], sh[FN][4], s[FN][4], q[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + wn * TN + 16 * j + 4 * fc + e;
      const int nn = n < p.N ? n : p.N - 1;
      bc[j][e] = p.bias ? reinterpret_cast<const float*>(p.bias)[(int64_t)cfg * p.bias_gstride + nn]
                        : 0.f;
      s[j][e] = q[j][e] = 0.f;
      mu[j][e] = is[j][e] = sc[j][e] = sh[j][e] = 0.f;
      if (bstat && bb.ym != YM_BIAS) {
        const int64_t c = (int64_t)cfg * p.N + nn;
        mu[j][e] = bb.mean[c];
        is[j][e] = bb.invstd[c];
        if (bb.ym == 2) {                   // YM_Z: the forward's scale / shift
          const float ga = reinterpret_cast<const float*>(bb.gamma)[cfg * bb.gstride + nn];
          const float be = reinterpret_cast<const float*>(bb.beta)[cfg * bb.bstride + nn];
          sc[j][e] = is[j][e] * ga;
          sh[j][e] = be - mu[j][e] * sc[j][e];
        }
      }
    }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + 16 * i + fr;
    if (m >= p.M) continue;
    int64_t orow = m;
    if (p.o_st > 1) {
      const RowPos r = decode_row(m, p.M, p.a);
      orow = ((int64_t)r.b * p.o_H + (int64_t)r.y * p.o_st) * p.o_W + (int64_t)r.x * p.o_st;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + 16 * j + 4 * fc;
      if (n >= p.N) continue;
      const int64_t go = orow * p.ldc + n;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bc[j][e];
        v[e] = p.act == 6 ? fminf(fmaxf(v[e], 0.f), 6.f) : (p.act ? fmaxf(v[e], 0.f) : v[e]);
      }
      if (vec) {
        if (adb) {
          const float4 a = *reinterpret_cast<const float4*>(adb + go);
          const uint32_t am = addend_bits(p, go + (int64_t)cfg * p.N);
          v[0] += am & 1u ? a.x : 0.f;
          v[1] += am & 2u ? a.y : 0.f;
          v[2] += am & 4u ? a.z : 0.f;
          v[3] += am & 8u ? a.w : 0.f;
        }
        if (bstat && bb.ym == YM_BIAS) {
          const float4 y4 = *reinterpret_cast<const float4*>(zb + go);
          const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = act_pass(bb.act, yv[e]) ? v[e] : 0.f;
            s[j][e] += v[e];
          }
        }
        *reinterpret_cast<float4*>(obase + go) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < p.N) {
            if (adb && (addend_bits(p, go + e + (int64_t)cfg * p.N) & 1u)) v[e] += adb[go + e];
            if (bstat && bb.ym == YM_BIAS) {
              v[e] = act_pass(bb.act, zb[go + e]) ? v[e] : 0.f;
              s[j][e] += v[e];
            }
            obase[go + e] = v[e];
          }
      }
      if (fstat) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[j][e] += v[e];
          q[j][e] += v[e] * v[e];
        }
      } else if (bstat && bb.ym != YM_BIAS) {      // host-gated: vec
        const float4 z4 = *reinterpret_cast<const float4*>(zb + go);
        const float zv[4] = {z4.x, z4.y, z4.z, z4.w};
        float yv[4] = {0.f, 0.f, 0.f, 0.f};
        if (yb) {
          const float4 y4 = *reinterpret_cast<const float4*>(yb + go);
          yv[0] = y4.x; yv[1] = y4.y; yv[2] = y4.z; yv[3] = y4.w;
        } else if (mb) {
          const int64_t bi = go + (int64_t)cfg * p.N;     // element index in [M][ldc]
          const uint32_t m = (uint32_t)mb[bi >> 3] >> (bi & 7);
#pragma unroll
          for (int e = 0; e < 4; ++e) yv[e] = (m >> e) & 1u ? 1.f : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float dz = v[e];
          if (bb.ym == 2)
            dz = (zv[e] * sc[j][e] + sh[j][e] + 0.f) > 0.f ? dz : 0.f;
          else if (bb.ym == 1 || bb.ym == 3)
            dz = bb.act == 6 ? ((yv[e] > 0.f && yv[e] < 6.f) ? dz : 0.f) : (yv[e] > 0.f ? dz : 0.f);
          s[j][e] += dz;
          q[j][e] += dz * (zv[e] - mu[j][e]) * is[j][e];
        }
      }
    }
  }
  if (!fstat && !bstat) return;
  // rows -> one deterministic partial per (M tile, channel): DPP over the 16
  // lanes of equal fc, then the two M-direction waves meet in LDS
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sm = row16_sum(s[j][e]);
      const float sq = row16_sum(q[j][e]);
      if (fr == 0) {
        const int nl = wn * TN + 16 * j + 4 * fc + e;
        xch[(wm * 2) * BN + nl] = sm;
        xch[(wm * 2 + 1) * BN + nl] = sq;
      }
    }
  __syncthreads();
  if (bstat && bb.ym == YM_BIAS) {
    bias_link_store<BN>(bb, xch, cfg, n0, p.N, tid);
    return;
  }
  float* dst = fstat ? p.stats : bb.part;
  const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
  for (int t = tid; t < 2 * BN; t += NTHREADS) {
    const int qd = t / BN, nl = t - qd * BN, n = n0 + nl;
    if (n < p.N)
      stat_store(dst, sb + (int64_t)qd * p.ldc + n, xch[qd * BN + nl] + xch[(2 + qd) * BN + nl],
                 p.stat_slabs);
  }
}

// Epilogue operands as buffer descriptors: a null or unused source gets a
// 0-byte descriptor, so its loads return zeros with no branch around them.
// A load under a branch makes hipcc's vmcnt bookkeeping path-dependent and
// it then drains (vmcnt(0)) at the next use: the reference epilogue, whose
// per-channel parameters and per-fragment addend / BN-input loads sit in
// such branches between stores, paid ~20 dependent memory round trips per
// tile, which dominated the small-K (K = 64) dgrad / forward kernels.
constexpr uint32_t EPI_BIG = 0x7ffffff0u;
constexpr int EPI_FULL = 0, EPI_FWD = 1, EPI_ZLINK = 2, EPI_JOIN = 3, EPI_ADD = 4,
              EPI_BLINK = 5;   // epi32 MODE
__device__ __forceinline__ float bload_f32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ uint32_t bload_u8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)off, 0, 0);
}

// true when every epilogue tensor offset of this launch fits the 31-bit
// buffer offsets (output rows of a strided dgrad: at most (st + 1)^2 per row)
__device__ __forceinline__ bool epi_fits(const NTParams& p) {
  const int64_t rows = p.o_st > 1 ? (int64_t)p.M * (p.o_st + 1) * (p.o_st + 1) : (int64_t)p.M;
  return rows * p.ldc * 4 < (int64_t)EPI_BIG;
}

// fp32 epilogue of the NT / NN kernels, straight from the accumulators:
// lane (fr, fc) of wave (wm, wn) owns rows wm*TM + 16i + fr and channels
// wn*TN + 16j + 4fc .. +3.  Same outputs as epi32_ref, with every load of
// the epilogue issued before its first use: the per-channel parameters
// (bias, BN mean / invstd / gamma / beta) and the first row group's addend
// and BN-input / mask operands together (one row group of <= 4 fragments:
// every 64x64 tile; larger tiles walk 2-4 groups, one round trip each: a
// second, double-buffered group spills the 128x128 kernels and costs the
// 128x64 ones a wave per SIMD).
// Unaligned channels, the y-form BN link (ym 1) and > 2 GB tensors take
// epi32_ref.  xch: LDS scratch of 4*BN floats.  MODE (compile time) drops
// the operands a launch class never has -- through empty descriptors their
// loads still cost instructions and registers in every tile:
//   EPI_FULL  everything above (run-time flags);
//   EPI_FWD   the uniform-K forward kernels: bias + activation + forward
//             statistics only;
//   EPI_ZLINK a uniform-K dgrad whose only extra is a BN link with the mask
//             recomputed from z (ym 2): no bias, addend, addend mask or
//             stored mask;
//   EPI_JOIN  a uniform-K dgrad into a residual join: BN link with the
//             stored activation bits (ym 3), any addend / addend mask, no
//             bias, no scale / shift;
//   EPI_ADD   a uniform-K dgrad with no BN link (its input is not a BN
//             output, e.g. the max pool's): any addend / addend mask only;
//   EPI_BLINK a uniform-K dgrad with the bias-act link (ym YM_BIAS, VGG's
//             conv -> conv) and nothing else.
template <int BM, int BN, int MODE = EPI_FULL>
__device__ __forceinline__ void epi32(const NTParams& p, const f32x4 (&acc)[BM / 32][BN / 32],
                                      float* xch, int cfg, int m0, int n0, int wm, int wn,
                                      int lane, int tid) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  constexpr int CH = FM * FN <= 4 ? FM : (4 / FN > 0 ? 4 / FN : 1);   // rows per group
  constexpr int NG = (FM + CH - 1) / CH;
  const BNBwdEpi& bb = p.bb;
  const bool fstat = p.stats != nullptr;
  const bool bstat = MODE != EPI_ADD && bb.part != nullptr;   // EPI_ADD: host-gated none
  const bool vec = ((p.N | p.ldc) & 3) == 0;
  if (!vec || (bstat && bb.ym == 1) || !epi_fits(p)) {
    epi32_ref<BM, BN>(p, acc, xch, cfg, m0, n0, wm, wn, lane, tid);
    return;
  }
  const int fr = lane & 15, fc = lane >> 4;
  float* obase = reinterpret_cast<float*>(p.out) + (int64_t)cfg * p.N;
  if constexpr (MODE == EPI_FWD) {
    // the bias loads only when there is a bias (a uniform branch: nothing
    // else is in flight here, so its vmcnt drain costs nothing, while 16
    // loads through an empty descriptor would still be issued and waited on)
    float bl[FN][4], sl[FN][4], ql[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) bl[j][e] = sl[j][e] = ql[j][e] = 0.f;
    if (p.bias) {
      const auto rB = make_rsrc(p.bias, EPI_BIG);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0 + wn * TN + 16 * j + 4 * fc + e;
          const uint32_t nn = (uint32_t)(n < p.N ? n : p.N - 1);
          bl[j][e] = bload_f32(rB, ((uint32_t)cfg * (uint32_t)p.bias_gstride + nn) * 4u);
        }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + 16 * i + fr;
      if (m >= p.M) continue;
      int64_t orow = m;
      if (p.o_st > 1) {
        const RowPos r = decode_row(m, p.M, p.a);
        orow = ((int64_t)r.b * p.o_H + (int64_t)r.y * p.o_st) * p.o_W + (int64_t)r.x * p.o_st;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + 4 * fc;
        if (n >= p.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] + bl[j][e];
          v[e] = p.act == 6 ? fminf(fmaxf(v[e], 0.f), 6.f) : (p.act ? fmaxf(v[e], 0.f) : v[e]);
          sl[j][e] += v[e];
          ql[j][e] += v[e] * v[e];
        }
        *reinterpret_cast<float4*>(obase + orow * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    if (!fstat) return;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sm = row16_sum(sl[j][e]);
        const float sq = row16_sum(ql[j][e]);
        if (fr == 0) {
          const int nl = wn * TN + 16 * j + 4 * fc + e;
          xch[(wm * 2) * BN + nl] = sm;
          xch[(wm * 2 + 1) * BN + nl] = sq;
        }
      }
    __syncthreads();
    const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
    for (int t = tid; t < 2 * BN; t += NTHREADS) {
      const int qd = t / BN, nl = t - qd * BN, n = n0 + nl;
      if (n < p.N)
        stat_store(p.stats, sb + (int64_t)qd * p.ldc + n, xch[qd * BN + nl] + xch[(2 + qd) * BN + nl],
                   p.stat_slabs);
    }
    return;
  }
  constexpr bool ZL = MODE == EPI_ZLINK;       // host-gated: bstat, ym 2, nothing else
  constexpr bool JN = MODE == EPI_JOIN;        // host-gated: bstat, ym 3, no bias
  constexpr bool AD = MODE == EPI_ADD;        // host-gated: no BN link, no bias
  constexpr bool BL = MODE == EPI_BLINK;      // host-gated: bias link, nothing else
  constexpr bool NOBIAS = ZL || JN || AD || BL;
  const bool ymz = ZL || (!JN && !BL && bstat && bb.ym == 2);
  const bool ymm = JN || (!ZL && !BL && bstat && bb.ym == 3);
  const bool ymb = BL || (!ZL && !JN && bstat && bb.ym == YM_BIAS);
  const auto rBias = make_rsrc(p.bias, !NOBIAS && p.bias ? EPI_BIG : 0u);
  const auto rMean = make_rsrc(bb.mean, bstat && !ymb ? EPI_BIG : 0u);
  const auto rInv = make_rsrc(bb.invstd, bstat && !ymb ? EPI_BIG : 0u);
  const auto rGa = make_rsrc(bb.gamma, ymz ? EPI_BIG : 0u);
  const auto rBe = make_rsrc(bb.beta, ymz ? EPI_BIG : 0u);
  const auto rAd = make_rsrc(p.addend, p.addend ? EPI_BIG : 0u);
  const bool amask = p.addend_mask != nullptr;
  const auto rAm = make_rsrc(p.addend_mask, amask ? EPI_BIG : 0u);
  const auto rZ = make_rsrc(bb.z, bstat ? EPI_BIG : 0u);
  const auto rMk = make_rsrc(bb.y, ymm ? EPI_BIG : 0u);
  float bc[FN][4], mu[FN][4], is[FN][4], ga[FN][4], be[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + wn * TN + 16 * j + 4 * fc + e;
      const uint32_t nn = (uint32_t)(n < p.N ? n : p.N - 1);
      const uint32_t c = (uint32_t)cfg * (uint32_t)p.N + nn;
      bc[j][e] = NOBIAS ? 0.f : bload_f32(rBias, ((uint32_t)cfg * (uint32_t)p.bias_gstride + nn) * 4u);
      mu[j][e] = AD || BL ? 0.f : bload_f32(rMean, c * 4u);
      is[j][e] = AD || BL ? 0.f : bload_f32(rInv, c * 4u);
      ga[j][e] = JN || AD || BL ? 0.f : bload_f32(rGa, ((uint32_t)cfg * (uint32_t)bb.gstride + nn) * 4u);
      be[j][e] = JN || AD || BL ? 0.f : bload_f32(rBe, ((uint32_t)cfg * (uint32_t)bb.bstride + nn) * 4u);
    }
  // one row group's operands: [row in group][j]
  uint4 ad[CH][FN], zz[CH][FN];
  uint32_t mk[CH][FN], amk[CH][FN];
  int64_t orow[FM];
  bool rok[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + 16 * i + fr;
    rok[i] = m < p.M;
    orow[i] = m;
    if (p.o_st > 1 && rok[i]) {
      const RowPos r = decode_row(m, p.M, p.a);
      orow[i] = ((int64_t)r.b * p.o_H + (int64_t)r.y * p.o_st) * p.o_W + (int64_t)r.x * p.o_st;
    }
  }
  auto fetch = [&](int g) {
#pragma unroll
    for (int ii = 0; ii < CH; ++ii) {
      const int i = g * CH + ii;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + 4 * fc;
        const bool ok = i < FM && rok[i < FM ? i : 0] && n < p.N;
        const int64_t el = orow[i < FM ? i : 0] * p.ldc + (int64_t)cfg * p.N + n;
        const uint32_t off = ok ? (uint32_t)el * 4u : OOB;
        zz[ii][j] = AD ? make_uint4(0u, 0u, 0u, 0u) : bload(rZ, off);
        if constexpr (AD) {
          ad[ii][j] = bload(rAd, off);
          amk[ii][j] = bload_u8(rAm, ok ? (uint32_t)(el >> 3) : OOB) >> (uint32_t)(el & 7);
          mk[ii][j] = 0u;
        } else if constexpr (BL) {
          ad[ii][j] = make_uint4(0u, 0u, 0u, 0u);
          mk[ii][j] = amk[ii][j] = 0u;
        } else if constexpr (!ZL) {
          ad[ii][j] = bload(rAd, off);
          mk[ii][j] = bload_u8(rMk, ok ? (uint32_t)(el >> 3) : OOB) >> (uint32_t)(el & 7);
          amk[ii][j] = bload_u8(rAm, ok ? (uint32_t)(el >> 3) : OOB) >> (uint32_t)(el & 7);
        } else {
          ad[ii][j] = make_uint4(0u, 0u, 0u, 0u);
          mk[ii][j] = amk[ii][j] = 0u;
        }
      }
    }
  };
  fetch(0);
  float sc[FN][4], sh[FN][4], s[FN][4], q[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[j][e] = is[j][e] * ga[j][e];
      sh[j][e] = be[j][e] - mu[j][e] * sc[j][e];
      s[j][e] = q[j][e] = 0.f;
    }
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (g > 0) fetch(g);
#pragma unroll
    for (int ii = 0; ii < CH; ++ii) {
      const int i = g * CH + ii;
      if (i >= FM || !rok[i]) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + 4 * fc;
        if (n >= p.N) continue;
        const float av[4] = {__uint_as_float(ad[ii][j].x), __uint_as_float(ad[ii][j].y),
                             __uint_as_float(ad[ii][j].z), __uint_as_float(ad[ii][j].w)};
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] + bc[j][e];
          v[e] = p.act == 6 ? fminf(fmaxf(v[e], 0.f), 6.f) : (p.act ? fmaxf(v[e], 0.f) : v[e]);
          if constexpr (!ZL && !BL) v[e] += !amask || ((amk[ii][j] >> e) & 1u) ? av[e] : 0.f;
        }
        if (ymb) {                   // bias-act link: dz = act'(y) * dx, written
          const float yv[4] = {__uint_as_float(zz[ii][j].x), __uint_as_float(zz[ii][j].y),
                               __uint_as_float(zz[ii][j].z), __uint_as_float(zz[ii][j].w)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = act_pass(bb.act, yv[e]) ? v[e] : 0.f;
            s[j][e] += v[e];
          }
        }
        *reinterpret_cast<float4*>(obase + orow[i] * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
        if (fstat) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s[j][e] += v[e];
            q[j][e] += v[e] * v[e];
          }
        } else if (bstat && !ymb) {
          const float zv[4] = {__uint_as_float(zz[ii][j].x), __uint_as_float(zz[ii][j].y),
                               __uint_as_float(zz[ii][j].z), __uint_as_float(zz[ii][j].w)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float dz = v[e];
            if (ymz)
              dz = (zv[e] * sc[j][e] + sh[j][e] + 0.f) > 0.f ? dz : 0.f;
            else if (ymm) {
              const float yv = (mk[ii][j] >> e) & 1u ? 1.f : 0.f;
              dz = bb.act == 6 ? ((yv > 0.f && yv < 6.f) ? dz : 0.f) : (yv > 0.f ? dz : 0.f);
            }
            s[j][e] += dz;
            q[j][e] += dz * (zv[e] - mu[j][e]) * is[j][e];
          }
        }
      }
    }
  }
  if (!fstat && !bstat) return;
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sm = row16_sum(s[j][e]);
      const float sq = row16_sum(q[j][e]);
      if (fr == 0) {
        const int nl = wn * TN + 16 * j + 4 * fc + e;
        xch[(wm * 2) * BN + nl] = sm;
        xch[(wm * 2 + 1) * BN + nl] = sq;
      }
    }
  __syncthreads();
  if (bstat && bb.ym == YM_BIAS) {
    bias_link_store<BN>(bb, xch, cfg, n0, p.N, tid);
    return;
  }
  float* dst = fstat ? p.stats : bb.part;
  const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
  for (int t = tid; t < 2 * BN; t += NTHREADS) {
    const int qd = t / BN, nl = t - qd * BN, n = n0 + nl;
    if (n < p.N)
      stat_store(dst, sb + (int64_t)qd * p.ldc + n, xch[qd * BN + nl] + xch[(2 + qd) * BN + nl],
                 p.stat_slabs);
  }
}

// ---- wide-MFMA form of the fp32 forward (v_mfma_f32_32x32x16_bf16) --------
// Same staging, LDS images and K loop as the 16x16x32 kernels; only the
// fragment reads, the accumulator layout and the epilogue differ.  Why: the
// fp32 kernels are bound by the VALU work of the hi/lo split, which can only
// issue in the cycles an MFMA leaves the SIMD's vector port free -- 8 of the
// 16 cycles of a 16x16x32 but 24 of the 32 of a 32x32x16 (MI355X_MICROARCH
// "vector-instruction ISSUE cost").  Per stage the same FLOPs therefore leave
// 1.5x the VALU slack for the split (e.g. 128x128: 2304 vs 1536 cycles per
// wave-step against ~1700 of split work).
// Operand maps (32x32x16): lane l (r = l & 31, h = l >> 5) holds
// X[row r][k = 8h + j]; the weight fragment goes FIRST, so D[n][m] comes out
// with the output row m = r on the lane and channels 8q + 4h + e (q = reg >> 2,
// e = reg & 3) in the registers: one 16-B store per register quad.
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BM, int BN, bool WIDE>
struct AccT {
  using type = f32x4[BM / 32][BN / 32];
};
template <int BM, int BN>
struct AccT<BM, BN, true> {
  using type = f32x16[BM / 64][BN / 64];
};

template <int BM, int BN>
__device__ __forceinline__ void zero_accw(f32x16 (&acc)[BM / 64][BN / 64]) {
#pragma unroll
  for (int i = 0; i < BM / 64; ++i)
#pragma unroll
    for (int j = 0; j < BN / 64; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
}

__device__ __forceinline__ f32x16 mfma3w(const bf16x8& xh, const bf16x8& xl, const bf16x8& yh,
                                         const bf16x8& yl, f32x16 acc) {
  if (CER_TIMING_1PASS) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, yh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl, yh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, yl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, yh, acc, 0, 0, 0);
}

// NT x NT images (hi in chunks 0-3, lo in 4-7): two 16-deep substeps
template <int BM, int BN>
__device__ __forceinline__ void mma3w_nt(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                         int lane, f32x16 (&acc)[BM / 64][BN / 64]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 32 * i + r, 2 * s + h));
      al[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 32 * i + r, 4 + 2 * s + h));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(sb + nt_off(wn * TN + 32 * j + r, 2 * s + h));
      bl[j] = *reinterpret_cast<const bf16x8*>(sb + nt_off(wn * TN + 32 * j + r, 4 + 2 * s + h));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma3w(bh[j], bl[j], ah[i], al[i], acc[i][j]);
  }
}

// fp32 ring images (32 fp32 per row as 8 swizzled 16-B chunks): the k of
// substep s, half h are fp32 16s + 8h .. +7 = chunks 4s + 2h, 4s + 2h + 1
template <int BM, int BN>
__device__ __forceinline__ void mma3w_ring_nt(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                              int lane, f32x16 (&acc)[BM / 64][BN / 64],
                                              bool ahl, bool bhl = false) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * TN + 32 * j + r;
      const uint4 x0 = *reinterpret_cast<const uint4*>(sb + nt_off(row, 4 * s + 2 * h));
      const uint4 x1 = *reinterpret_cast<const uint4*>(sb + nt_off(row, 4 * s + 2 * h + 1));
      uint4 hh, ll;
      take_hi_lo(bhl, x0, x1, hh, ll);
      bh[j] = __builtin_bit_cast(bf16x8, hh);
      bl[j] = __builtin_bit_cast(bf16x8, ll);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * TM + 32 * i + r;
      const uint4 x0 = *reinterpret_cast<const uint4*>(sa + nt_off(row, 4 * s + 2 * h));
      const uint4 x1 = *reinterpret_cast<const uint4*>(sa + nt_off(row, 4 * s + 2 * h + 1));
      uint4 hh, ll;
      take_hi_lo(ahl, x0, x1, hh, ll);
      ah[i] = __builtin_bit_cast(bf16x8, hh);
      al[i] = __builtin_bit_cast(bf16x8, ll);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma3w(bh[j], bl[j], ah[i], al[i], acc[i][j]);
  }
}

// TN image of the wide kernels: [reduction rows][COLS] bf16, 8-B column
// chunks XOR-swizzled per row so that the 32x32x16 transposed fragment read
// (tn_frag32: per 32-lane half, rows q = 0..3 x 8 consecutive 8-B chunks) hits
// 64 distinct banks; the XOR is even, so the 16-B staging stores stay whole.
//   COLS 128 (256-B rows, all rows on the same banks): chunk ^ 8 (row & 3)
//   COLS  64 (128-B rows, odd rows on the other half): chunk ^ 8 ((row >> 1) & 1)
template <int COLS>
__device__ __forceinline__ int tn_off_w(int row, int col) {  // col multiple of 4
  const int sw = COLS == 128 ? 8 * (row & 3) : 8 * ((row >> 1) & 1);
  return row * COLS + 4 * ((col >> 2) ^ sw);
}

// B-operand map of the 32x32x16 MFMA from a TN image: lane l (r = l & 31,
// h = l >> 5) gets element j = 0..7 of reduction row row0 + 8h + j at column
// col_base + r.  ds_read_b64_tr_b16 transposes a 4-row x 16-column block
// across 16 lanes (lane i supplies row i >> 2, columns 4 (i & 3) .. +3 and
// receives column i), so each 16-lane group g = (l >> 4) & 1 reads columns
// col_base + 16g .. +15, rows +0..3 then +4..7.
template <int COLS>
__device__ __forceinline__ bf16x8 tn_frag32(const bf16_t* tile, int row0, int col_base, int lane) {
  const int h = lane >> 5, g = (lane >> 4) & 1, i = lane & 15, q = i >> 2, pp = i & 3;
  const int col = col_base + 16 * g + 4 * pp;
  const bf16_t* p0 = tile + tn_off_w<COLS>(row0 + 8 * h + q, col);
  const bf16_t* p1 = tile + tn_off_w<COLS>(row0 + 8 * h + 4 + q, col);
  s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  s16x8 t = __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, t);
}

// A: NT image, B: TN image (tn_off_w; hi rows 0-31, lo rows 32-63) -- dgrad
template <int BM, int BN>
__device__ __forceinline__ void mma3w_nn(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                         int lane, f32x16 (&acc)[BM / 64][BN / 64]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 32 * i + r, 2 * s + h));
      al[i] = *reinterpret_cast<const bf16x8*>(sa + nt_off(wm * TM + 32 * i + r, 4 + 2 * s + h));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = tn_frag32<BN>(sb, 16 * s, wn * TN + 32 * j, lane);
      bl[j] = tn_frag32<BN>(sb, KS + 16 * s, wn * TN + 32 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma3w(bh[j], bl[j], ah[i], al[i], acc[i][j]);
  }
}

// both TN images (tn_off_w) -- wgrad: D[n][k], k on the lane
template <int BM, int BN>
__device__ __forceinline__ void mma3w_tn(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                         int lane, f32x16 (&acc)[BM / 64][BN / 64]) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      ah[i] = tn_frag32<BM>(sa, 16 * s, wm * TM + 32 * i, lane);
      al[i] = tn_frag32<BM>(sa, KS + 16 * s, wm * TM + 32 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = tn_frag32<BN>(sb, 16 * s, wn * TN + 32 * j, lane);
      bl[j] = tn_frag32<BN>(sb, KS + 16 * s, wn * TN + 32 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma3w(ah[i], al[i], bh[j], bl[j], acc[i][j]);
  }
}

// split-K seam of the wide kernels (splitk_reduce with the 32x32 accumulators)
template <int BM, int BN>
__device__ __forceinline__ bool splitk_reduce_w(const NTParams& p,
                                                f32x16 (&acc)[BM / 64][BN / 64], int tile_id,
                                                int split, int tid) {
  constexpr int FI = BM / 64, FJ = BN / 64, NA = FI * FJ * 16;
  __shared__ int sk_flag;
  float* base = p.skws + (int64_t)tile_id * p.splits * (NA * NTHREADS);
  float* mine = base + (int64_t)split * (NA * NTHREADS);
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        st_sc1(mine + ((i * FJ + j) * 16 + e) * NTHREADS + tid, acc[i][j][e]);
  if (!last_arriver(p.skcnt + tile_id, (unsigned)p.splits, &sk_flag)) return false;
  zero_accw<BM, BN>(acc);
  for (int sp = 0; sp < p.splits; ++sp) {
    const float* src = base + (int64_t)sp * (NA * NTHREADS);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          acc[i][j][e] += ld_sc1(src + ((i * FJ + j) * 16 + e) * NTHREADS + tid);
  }
  return true;
}

// fp32 epilogue of the wide NT / NN kernels (epi32 with the 32x32 layout):
// out = act(acc + bias) (+ addend), and optionally the forward BN partials
// (sum, sum^2) or a dgrad output's BN-backward partials (sum dz, sum dz*xhat,
// BNBwdEpi) per (M tile, channel).  Walks one 32-channel block j at a time so
// only 16 channels of per-channel state are live next to the accumulators.
// xch: LDS scratch of 4*BN floats.
template <int BM, int BN, bool BSTAT = false>
__device__ __forceinline__ void epi32w(const NTParams& p, const f32x16 (&acc)[BM / 64][BN / 64],
                                       float* xch, int cfg, int m0, int n0, int wm, int wn,
                                       int lane, int tid) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
  const int r = lane & 31, h = lane >> 5;
  float* obase = reinterpret_cast<float*>(p.out) + (int64_t)cfg * p.N;
  const float* adb =
      p.addend ? reinterpret_cast<const float*>(p.addend) + (int64_t)cfg * p.N : nullptr;
  const BNBwdEpi& bb = p.bb;
  const bool fstat = p.stats != nullptr;
  const bool bstat = BSTAT && bb.part != nullptr;   // compile-time off in the forward kernels
  const bool vec = ((p.N | p.ldc) & 3) == 0;
  const float* zb = bstat ? reinterpret_cast<const float*>(bb.z) + (int64_t)cfg * p.N : nullptr;
  const float* yb = bstat && bb.ym == 1 ? reinterpret_cast<const float*>(bb.y) + (int64_t)cfg * p.N
                                       : nullptr;
  // ym 3 (bn.hip YM_M): the activation mask as bits, [M][ldc / 8] bytes
  const uint8_t* mb = bstat && bb.ym == 3 ? reinterpret_cast<const uint8_t*>(bb.y) : nullptr;
  int64_t orow[FM];
  bool rok[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + 32 * i + r;
    rok[i] = m < p.M;
    orow[i] = m;
    if (p.o_st > 1 && rok[i]) {
      const RowPos rp = decode_row(m, p.M, p.a);
      orow[i] = ((int64_t)rp.b * p.o_H + (int64_t)rp.y * p.o_st) * p.o_W + (int64_t)rp.x * p.o_st;
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nb = n0 + wn * TN + 32 * j + 4 * h;       // + 8q + e
    float bc[4][4], s[4][4], q[4][4], mu[4][4], is[4][4], sc[4][4], sh[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = nb + 8 * g + e;
        const int nn = n < p.N ? n : p.N - 1;
        bc[g][e] = p.bias
                       ? reinterpret_cast<const float*>(p.bias)[(int64_t)cfg * p.bias_gstride + nn]
                       : 0.f;
        s[g][e] = q[g][e] = 0.f;
        mu[g][e] = is[g][e] = sc[g][e] = sh[g][e] = 0.f;
        if (bstat && bb.ym != YM_BIAS) {
          const int64_t c = (int64_t)cfg * p.N + nn;
          mu[g][e] = bb.mean[c];
          is[g][e] = bb.invstd[c];
          if (bb.ym == 2) {                   // YM_Z: the forward's scale / shift
            const float ga = reinterpret_cast<const float*>(bb.gamma)[cfg * bb.gstride + nn];
            const float be = reinterpret_cast<const float*>(bb.beta)[cfg * bb.bstride + nn];
            sc[g][e] = is[g][e] * ga;
            sh[g][e] = be - mu[g][e] * sc[g][e];
          }
        }
      }
    // bias-act link: this block's y operands, all loads in flight before the
    // first use (one memory round trip per 32-channel block, as in epi32)
    float4 ypre[FM][4];
    if (bstat && bb.ym == YM_BIAS && vec) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = nb + 8 * g;
          ypre[i][g] = rok[i] && n < p.N
                           ? *reinterpret_cast<const float4*>(zb + orow[i] * p.ldc + n)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (!rok[i]) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = nb + 8 * g;
        if (n >= p.N) continue;
        const int64_t go = orow[i] * p.ldc + n;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][4 * g + e] + bc[g][e];
          v[e] = p.act == 6 ? fminf(fmaxf(v[e], 0.f), 6.f) : (p.act ? fmaxf(v[e], 0.f) : v[e]);
        }
        if (vec) {
          if (adb) {
            const float4 a = *reinterpret_cast<const float4*>(adb + go);
            const uint32_t am = addend_bits(p, go + (int64_t)cfg * p.N);
            v[0] += am & 1u ? a.x : 0.f;
            v[1] += am & 2u ? a.y : 0.f;
            v[2] += am & 4u ? a.z : 0.f;
            v[3] += am & 8u ? a.w : 0.f;
          }
          if (bstat && bb.ym == YM_BIAS) {
            const float yv[4] = {ypre[i][g].x, ypre[i][g].y, ypre[i][g].z, ypre[i][g].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = act_pass(bb.act, yv[e]) ? v[e] : 0.f;
              s[g][e] += v[e];
            }
          }
          *reinterpret_cast<float4*>(obase + go) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) {
              if (adb && (addend_bits(p, go + e + (int64_t)cfg * p.N) & 1u)) v[e] += adb[go + e];
              if (bstat && bb.ym == YM_BIAS) {
                v[e] = act_pass(bb.act, zb[go + e]) ? v[e] : 0.f;
                s[g][e] += v[e];
              }
              obase[go + e] = v[e];
            }
        }
        if (fstat) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s[g][e] += v[e];
            q[g][e] += v[e] * v[e];
          }
        } else if (bstat && bb.ym != YM_BIAS) {      // host-gated: vec
          const float4 z4 = *reinterpret_cast<const float4*>(zb + go);
          const float zv[4] = {z4.x, z4.y, z4.z, z4.w};
          float yv[4] = {0.f, 0.f, 0.f, 0.f};
          if (yb) {
            const float4 y4 = *reinterpret_cast<const float4*>(yb + go);
            yv[0] = y4.x; yv[1] = y4.y; yv[2] = y4.z; yv[3] = y4.w;
          } else if (mb) {
            const int64_t bi = go + (int64_t)cfg * p.N;     // element index in [M][ldc]
            const uint32_t m = (uint32_t)mb[bi >> 3] >> (bi & 7);
#pragma unroll
            for (int e = 0; e < 4; ++e) yv[e] = (m >> e) & 1u ? 1.f : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float dz = v[e];
            if (bb.ym == 2)
              dz = (zv[e] * sc[g][e] + sh[g][e] + 0.f) > 0.f ? dz : 0.f;
            else if (bb.ym == 1 || bb.ym == 3)
              dz = bb.act == 6 ? ((yv[e] > 0.f && yv[e] < 6.f) ? dz : 0.f) : (yv[e] > 0.f ? dz : 0.f);
            s[g][e] += dz;
            q[g][e] += dz * (zv[e] - mu[g][e]) * is[g][e];
          }
        }
      }
    }
    if (fstat || bstat) {
      // rows live on the 32 lanes of equal h: DPP sum over 16, then xor 16
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sm = row16_sum(s[g][e]);
          float sq = row16_sum(q[g][e]);
          sm += __shfl_xor(sm, 16, 64);
          sq += __shfl_xor(sq, 16, 64);
          if (r == 0) {
            const int nl = wn * TN + 32 * j + 8 * g + 4 * h + e;
            xch[(wm * 2) * BN + nl] = sm;
            xch[(wm * 2 + 1) * BN + nl] = sq;
          }
        }
    }
  }
  if (!fstat && !bstat) return;
  __syncthreads();
  if (bstat && bb.ym == YM_BIAS) {
    bias_link_store<BN>(bb, xch, cfg, n0, p.N, tid);
    return;
  }
  float* dst = fstat ? p.stats : bb.part;
  const int64_t sb = stat_base(m0 / BM, p.stat_slabs, p.ldc, cfg, p.N);
  for (int t = tid; t < 2 * BN; t += NTHREADS) {
    const int qd = t / BN, nl = t - qd * BN, n = n0 + nl;
    if (n < p.N)
      stat_store(dst, sb + (int64_t)qd * p.ldc + n, xch[qd * BN + nl] + xch[(2 + qd) * BN + nl],
                 p.stat_slabs);
  }
}

// Intra-block K split (WG = 2 wave groups of 256 threads, 512-thread
// blocks): group g runs the unchanged 4-wave tile loop over its half of the
// block's K range in its own LDS region, then group 1 hands its accumulators
// to group 0 through LDS and exits; group 0 adds them and runs the epilogue
// (barriers after the exit count the surviving waves only).  Doubles the
// waves in flight per tile without split-K's workspace round trip: for the
// latency-bound small-grid GEMMs of a one-config step (4x4 / 7x7 stages)
// where 1-2 waves per SIMD cannot hide the load latency.  Both groups run the
// same step count (the last group's surplus steps load zeros: every k at or
// past ``klim`` is masked), so the block-wide barriers stay matched.
struct KSplitRange {
  int kt0, kt1, klim;
};
template <int WG>
__device__ __forceinline__ KSplitRange group_range(const KRange& kr, int grp, int K) {
  if constexpr (WG == 1) {
    return KSplitRange{kr.kt0, kr.kt1, K};
  } else {
    const int h = (kr.kt1 - kr.kt0 + WG - 1) / WG;
    const int g0 = kr.kt0 + grp * h;
    return KSplitRange{g0, g0 + h, min(K, kr.kt1 * KS)};
  }
}

// groups 1..WG-1 -> group 0 accumulator hand-off, each through its own LDS
// region (``regions`` = the block's LDS, ``stride`` floats per group);
// false in the groups that must exit
template <int WG, int BM, int BN>
__device__ __forceinline__ bool group_reduce(f32x4 (&acc)[BM / 32][BN / 32], float* regions,
                                             int stride, int grp, int tid) {
  if constexpr (WG == 1) {
    return true;
  } else {
    constexpr int FI = BM / 32, FJ = BN / 32;
    __syncthreads();
    if (grp > 0) {
      float* red = regions + grp * stride;
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[((i * FJ + j) * 4 + e) * NTHREADS + tid] = acc[i][j][e];
    }
    __syncthreads();
    if (grp > 0) return false;
#pragma unroll
    for (int g = 1; g < WG; ++g) {
      const float* red = regions + g * stride;
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] += red[((i * FJ + j) * 4 + e) * NTHREADS + tid];
    }
    return true;
  }
}

// forward (and the unaligned-dgrad fallback through transposed weights):
// y = act(im2col(x) W^T + b), fp32 in / out.  WIDE: 32x32x16 MFMAs (above).
template <int BM, int BN, int GM, bool WIDE = false, int WG = 1>
__global__ __launch_bounds__(NTHREADS * WG, WG == 1 ? (fp32_occ<BM, BN>()) : 1)
void igemm_nt32(NTParams p) {
  static_assert(WG == 1 || !WIDE, "intra-block K split: 16x16x16 kernels only");
  constexpr int NST = 2;                                       // LDS stages
  constexpr int CPR = KS / 8;                                  // 8-float chunks per row
  constexpr int A_CH = BM * CPR / NTHREADS, B_CH = BN * CPR / NTHREADS;
  constexpr int TILE_ELEMS = NST * (BM + BN) * BK;
  constexpr int LDS_ELEMS = TILE_ELEMS > 8 * BN ? TILE_ELEMS : 8 * BN;
  static_assert(WG == 1 || LDS_ELEMS * 2 >= (BM / 32) * (BN / 32) * 16 * NTHREADS,
                "group hand-off must fit one group's LDS region");
  __shared__ __attribute__((aligned(16))) bf16_t lds_all[LDS_ELEMS * WG];
  const int grp = WG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x / NTHREADS);
  bf16_t* const lds = lds_all + grp * LDS_ELEMS;
#define SA(buf) (lds + (buf) * (BM * BK))
#define SB(buf) (lds + NST * BM * BK + (buf) * (BN * BK))

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KSplitRange kr = group_range<WG>(split_range<KS>(p, split), grp, p.K);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x & (NTHREADS - 1), lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);
  const float* wbase = reinterpret_cast<const float*>(p.w) + (int64_t)cfg * p.w_gstride;
  const float* abase = reinterpret_cast<const float*>(p.a.src) + (int64_t)cfg * p.a.cfg_off;

  constexpr bool UK = GM == GM_GEMM || GM == GM_TAP;           // uniform-K modes
  RowPos rows[A_CH];
  RowA rowa[A_CH];
  uint32_t abo[A_CH], amask[A_CH], bbo[B_CH];   // UK: per-row byte bases, tap masks
  __amdgpu_buffer_rsrc_t rA, rB;
  if constexpr (GM != GM_SLOW) {
    rA = make_rsrc(abase, p.a.bytes);
    rB = make_rsrc(wbase, (uint32_t)p.N * (uint32_t)p.K * 4u);
  }
  if constexpr (UK) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = m0 + (tid + NTHREADS * i) / CPR;
      const RowA ra_ = row_init<GM_FWD>(p.a, m, p.M);
      // tap (0, 0)'s pixel may lie in the padding (negative): the uint32
      // arithmetic wraps and a valid tap's offset wraps back into range
      abo[i] = ((uint32_t)ra_.pix * (uint32_t)p.a.Ctot + (uint32_t)(8 * my_chunk)) * 4u;
      uint32_t mk = 0;
      if constexpr (GM == GM_TAP) {
        for (int r = 0; r < p.a.kh; ++r)
          for (int s2 = 0; s2 < p.a.kw; ++s2)
            if (((unsigned)(ra_.hy + r) < (unsigned)p.a.Hs) &
                ((unsigned)(ra_.wx + s2) < (unsigned)p.a.Ws))
              mk |= 1u << (r * p.a.kw + s2);
      } else {
        if (m < p.M) mk = 1u;
      }
      amask[i] = mk;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = n0 + (tid + NTHREADS * i) / CPR;
      bbo[i] = n < p.N ? (uint32_t)(n * p.K + 8 * my_chunk) * 4u : OOB;
    }
  } else if constexpr (GM != GM_SLOW) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) rowa[i] = row_init<GM>(p.a, m0 + (tid + NTHREADS * i) / CPR, p.M);
  } else {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) rows[i] = decode_row(m0 + (tid + NTHREADS * i) / CPR, p.M, p.a);
  }
  KPos kp{0, 0, 0};
  if constexpr (!UK) kp = kpos_init(p.a, kr.kt0 * KS + 8 * my_chunk);
  // UK: tap (index, row, col) and channel offset of the next K step to load
  // (wave-uniform: SGPRs); a step of KS channels never straddles a tap
  int u_c = 0, u_t = 0, u_r = 0, u_s = 0;
  if constexpr (GM == GM_TAP) {
    u_t = (kr.kt0 * KS) / p.a.Cg;
    u_c = kr.kt0 * KS - u_t * p.a.Cg;
    u_r = u_t / p.a.kw;
    u_s = u_t - u_r * p.a.kw;
  }
  constexpr int SETS = fp32_sets<BM, BN, WIDE>();
  uint4 ra[SETS][2 * A_CH], rb[SETS][2 * B_CH];

  auto load_tiles = [&](int kt, auto S) {
    constexpr int s = decltype(S)::value;
    const int k0 = kt * KS + 8 * my_chunk;
    if constexpr (UK) {
      const bool kok = kt * KS < kr.klim;
      const uint32_t kb = (uint32_t)(kt * KS) * 4u;
      uint32_t ko = kb;
      if constexpr (GM == GM_TAP)
        ko = ((uint32_t)(u_r * p.a.Ws + u_s) * (uint32_t)p.a.Ctot + (uint32_t)u_c) * 4u;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const uint32_t bit = GM == GM_TAP ? (amask[i] >> (u_t & 31)) & 1u : amask[i];
        const uint32_t o = (kok && bit) ? abo[i] + ko : OOB;
        ra[s][2 * i] = bload(rA, o);
        ra[s][2 * i + 1] = bload(rA, o + 16u);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const uint32_t o = kok ? bbo[i] + kb : OOB;
        rb[s][2 * i] = bload(rB, o);
        rb[s][2 * i + 1] = bload(rB, o + 16u);
      }
      if constexpr (GM == GM_TAP) {
        u_c += KS;
        if (u_c == p.a.Cg) {
          u_c = 0;
          ++u_t;
          if (++u_s == p.a.kw) {
            u_s = 0;
            ++u_r;
          }
        }
      }
    } else if constexpr (GM != GM_SLOW) {
      const bool kok = k0 < kr.klim;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const uint32_t off = a_off<GM, 4>(p.a, rowa[i], kp.r, kp.s, kp.c);
        const uint32_t o = kok ? off : OOB;
        ra[s][2 * i] = bload(rA, o);
        ra[s][2 * i + 1] = bload(rA, o + 16u);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid + NTHREADS * i) / CPR;
        const uint32_t o = (kok && n < p.N) ? (uint32_t)(n * p.K + k0) * 4u : OOB;
        rb[s][2 * i] = bload(rB, o);
        rb[s][2 * i + 1] = bload(rB, o + 16u);
      }
      kpos_advance<KS>(p.a, kp);
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i)
        gather_chunk_slow32(p.a, cfg, rows[i], k0, kr.klim, p.dgrad, ra[s][2 * i], ra[s][2 * i + 1]);
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid + NTHREADS * i) / CPR;
        load_row8_slow32(wbase + (int64_t)n * p.K + k0, n < p.N ? max(kr.klim - k0, 0) : 0, rb[s][2 * i],
                         rb[s][2 * i + 1]);
      }
    }
  };
  auto store_tiles = [&](int buf, auto S) {
    constexpr int s = decltype(S)::value;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid + NTHREADS * i) / CPR;
      if constexpr (CER_TIMING_NOAW) {
        keep_alive(ra[s][2 * i]);
        keep_alive(ra[s][2 * i + 1]);
        continue;
      }
      uint4 h, l;
      take_hi_lo(p.a_hl != 0, ra[s][2 * i], ra[s][2 * i + 1], h, l);
      *reinterpret_cast<uint4*>(SA(buf) + nt_off(row, my_chunk)) = h;
      *reinterpret_cast<uint4*>(SA(buf) + nt_off(row, my_chunk + 4)) = l;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = (tid + NTHREADS * i) / CPR;
      uint4 h, l;
      take_hi_lo(UK && p.w_hl != 0, rb[s][2 * i], rb[s][2 * i + 1], h, l);
      *reinterpret_cast<uint4*>(SB(buf) + nt_off(row, my_chunk)) = h;
      *reinterpret_cast<uint4*>(SB(buf) + nt_off(row, my_chunk + 4)) = l;
    }
  };

  typename AccT<BM, BN, WIDE>::type acc;
  if constexpr (WIDE) {
    zero_accw<BM, BN>(acc);
    auto mma = [&](int cur) { mma3w_nt<BM, BN>(SA(cur), SB(cur), wm, wn, lane, acc); };
    kloop32<SETS>(kr.kt0, kr.kt1, load_tiles, store_tiles, mma);
    if (p.splits > 1 && !splitk_reduce_w<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    epi32w<BM, BN>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  } else {
    zero_acc<BM, BN>(acc);
    kloop32<SETS>(kr.kt0, kr.kt1, load_tiles, store_tiles,
                  [&](int cur) { mma3_nt<BM, BN>(SA(cur), SB(cur), wm, wn, lane, acc); });
    if (!group_reduce<WG, BM, BN>(acc, reinterpret_cast<float*>(lds_all), LDS_ELEMS / 2, grp,
                                  tid))
      return;
    if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    epi32<BM, BN, (UK || GM == GM_FWD) ? EPI_FWD : EPI_FULL>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  }
#undef SA
#undef SB
}

// ---- fp32 LDS-DMA ring (forward): operand tiles go global -> LDS as fp32
// by buffer_load ... lds (no VGPR staging, no ds_write pass) into an S-stage
// ring; each wave splits its fragments into (hi, lo) bf16 right after the
// ds_read.  A 32-deep fp32 stage has the byte geometry of a 64-deep bf16
// stage (rows of 8 swizzled 16-B chunks), so the DMA addressing and the
// ring driver are the bf16 pipe_nt's.  The split moves from the staging
// pass (once per element) to the fragment reads (once per element per wave
// reading it: 2x the cvt work) in exchange for the LDS write traffic, which
// costs 2.5x a read per byte on the VGPR -> LDS path.  Requires Cg % 32 == 0.
template <int BM, int BN>
__device__ __forceinline__ void mma3_ring_nt(const bf16_t* sa, const bf16_t* sb, int wm, int wn,
                                             int lane, f32x4 (&acc)[BM / 32][BN / 32], bool ahl,
                                             bool bhl = false) {
  constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
  const int fr = lane & 15, fc = lane >> 4;
  bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int row = wn * TN + 16 * j + fr;
    const uint4 x0 = *reinterpret_cast<const uint4*>(sb + nt_off(row, 2 * fc));
    const uint4 x1 = *reinterpret_cast<const uint4*>(sb + nt_off(row, 2 * fc + 1));
    uint4 h, l;
    take_hi_lo(bhl, x0, x1, h, l);
    bh[j] = __builtin_bit_cast(bf16x8, h);
    bl[j] = __builtin_bit_cast(bf16x8, l);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wm * TM + 16 * i + fr;
    const uint4 x0 = *reinterpret_cast<const uint4*>(sa + nt_off(row, 2 * fc));
    const uint4 x1 = *reinterpret_cast<const uint4*>(sa + nt_off(row, 2 * fc + 1));
    uint4 h, l;
    take_hi_lo(ahl, x0, x1, h, l);
    ah[i] = __builtin_bit_cast(bf16x8, h);
    al[i] = __builtin_bit_cast(bf16x8, l);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = mfma3(bh[j], bl[j], ah[i], al[i], acc[i][j]);
}

template <int BM, int BN, int S, bool WIDE = false>
__global__ __launch_bounds__(NTHREADS, 2) void pipe_nt32(NTParams p) {
  constexpr int AJ = BM / 32, BJ = BN / 32, LPW = AJ + BJ;
  constexpr int STAGE = (BM + BN) * BK;             // bf16 units = (BM + BN) x 32 fp32
  constexpr int EPI = 8 * BN;
  constexpr int LDS_ELEMS = S * STAGE > EPI ? S * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KRange kr = split_range<KS>(p, split);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const float* abase = reinterpret_cast<const float*>(p.a.src) + (int64_t)cfg * p.a.cfg_off;
  const float* wbase = reinterpret_cast<const float*>(p.w) + (int64_t)cfg * p.w_gstride;
  const auto rA = make_rsrc(abase, p.a.bytes);
  const auto rB = make_rsrc(wbase, (uint32_t)p.N * (uint32_t)p.K * 4u);

  RowA arow[AJ];
  int achan[AJ];
  uint32_t boff[BJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const int row = (wid * AJ + j) * 8 + (lane >> 3);
    achan[j] = 4 * ((lane & 7) ^ ((row >> 1) & 7));
    arow[j] = row_init<GM_FWD>(p.a, m0 + row, p.M);
  }
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    const int row = (wid * BJ + j) * 8 + (lane >> 3);
    const int n = n0 + row;
    boff[j] = n < p.N ? (uint32_t)(n * p.K + 4 * ((lane & 7) ^ ((row >> 1) & 7))) * 4u : OOB;
  }
  // tap / channel of the next K tile to issue (Cg % 32 == 0: a 32-deep tile
  // never straddles taps)
  int tc = (kr.kt0 * KS) % p.a.Cg, tr = (kr.kt0 * KS) / p.a.Cg;
  int ts = tr % p.a.kw;
  tr /= p.a.kw;
  auto issue = [&](int kt, int st) {
    bf16_t* sa = lds + st * STAGE;
    bf16_t* sb = sa + BM * BK;
#pragma unroll
    for (int j = 0; j < AJ; ++j)
      glds16(rA, sa + (wid * AJ + j) * 512, a_off<GM_FWD, 4>(p.a, arow[j], tr, ts, tc + achan[j]),
             0);
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      glds16(rB, sb + (wid * BJ + j) * 512, boff[j], (uint32_t)kt * (KS * 4));
    tc += KS;
    if (tc == p.a.Cg) {
      tc = 0;
      if (++ts == p.a.kw) {
        ts = 0;
        ++tr;
      }
    }
  };
  typename AccT<BM, BN, WIDE>::type acc;
  if constexpr (WIDE) {
    zero_accw<BM, BN>(acc);
    ring_loop<S, LPW>(kr.kt1 - kr.kt0, [&](int t, int st) { issue(kr.kt0 + t, st); }, [&](int st) {
      mma3w_ring_nt<BM, BN>(lds + st * STAGE, lds + st * STAGE + BM * BK, wm, wn, lane, acc,
                            p.a_hl != 0, p.w_hl != 0);
    });
    if (p.splits > 1 && !splitk_reduce_w<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    epi32w<BM, BN>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  } else {
    zero_acc<BM, BN>(acc);
    ring_loop<S, LPW>(kr.kt1 - kr.kt0, [&](int t, int st) { issue(kr.kt0 + t, st); }, [&](int st) {
      mma3_ring_nt<BM, BN>(lds + st * STAGE, lds + st * STAGE + BM * BK, wm, wn, lane, acc,
                           p.a_hl != 0, p.w_hl != 0);
    });
    if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    // host-gated (run_nt32): ring launches are plain forwards
    epi32<BM, BN, EPI_FWD>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  }
}

// dgrad: dx = col2im(dy) * W with W read in place ([k = (tap, cout)] x [cin]
// rows, TN image), fp32 in / out; Cout % 8 == 0, Cin % 8 == 0
template <int BM, int BN, int GM, bool WIDE = false, int WG = 1, int EPI = EPI_FULL>
__global__ __launch_bounds__(NTHREADS * WG, WG == 1 ? (fp32_occ<BM, BN>()) : 1)
void igemm_nn32(NTParams p, int T, FastDiv dCout) {
  static_assert(WG == 1 || !WIDE, "intra-block K split: 16x16x16 kernels only");
  constexpr int NST = 2;
  constexpr int CPR = KS / 8;
  constexpr int A_CH = BM * CPR / NTHREADS;
  constexpr int B_CPR = BN / 8, B_CH = KS * B_CPR / NTHREADS, B_RSTEP = NTHREADS / B_CPR;
  constexpr int TILE_ELEMS = NST * (BM + BN) * BK;
  constexpr int LDS_ELEMS = TILE_ELEMS > 8 * BN ? TILE_ELEMS : 8 * BN;
  static_assert(WG == 1 || LDS_ELEMS * 2 >= (BM / 32) * (BN / 32) * 16 * NTHREADS,
                "group hand-off must fit one group's LDS region");
  __shared__ __attribute__((aligned(16))) bf16_t lds_all[LDS_ELEMS * WG];
  const int grp = WG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x / NTHREADS);
  bf16_t* const lds = lds_all + grp * LDS_ELEMS;

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tiles_n;
  int work = xcd_remap(blockIdx.x, gridDim.x);
  const int split = work % p.splits;
  work /= p.splits;
  const int cfg = work / tiles, tile = work - cfg * tiles;
  const KSplitRange kr = group_range<WG>(split_range<KS>(p, split), grp, p.K);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x & (NTHREADS - 1), lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int my_chunk = tid & (CPR - 1);
  const int Cout = p.a.Cg, Cin = p.N;
  const float* wbase = reinterpret_cast<const float*>(p.w) + (int64_t)cfg * p.w_gstride;
  const float* abase = reinterpret_cast<const float*>(p.a.src) + (int64_t)cfg * p.a.cfg_off;
  const int b_col = 8 * (tid % B_CPR), b_row0 = tid / B_CPR;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(abase, p.a.bytes);
  const __amdgpu_buffer_rsrc_t rW =
      make_rsrc(wbase, (uint32_t)Cout * (uint32_t)T * (uint32_t)Cin * 4u);

  // uniform-K modes (GM_GEMM: the 1x1 geometry, dy rows = GEMM rows; GM_TAP:
  // stride-1 k x k, Cout % 32 == 0): per-row dy bases + tap masks, and per
  // thread weight-row bases; a K step (32 output channels of one tap) adds
  // a wave-uniform offset to each
  constexpr bool UK = GM == GM_GEMM || GM == GM_TAP;
  RowA rowa[A_CH];
  uint32_t abo[A_CH], amask[A_CH], bbo[B_CH];
  if constexpr (UK) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = m0 + (tid + NTHREADS * i) / CPR;
      const RowA ra_ = row_init<GM_DG1>(p.a, m, p.M);
      abo[i] = ((uint32_t)ra_.pix * (uint32_t)p.a.Ctot + (uint32_t)(8 * my_chunk)) * 4u;
      uint32_t mk = 0;
      if constexpr (GM == GM_TAP) {
        for (int r = 0; r < p.a.kh; ++r)
          for (int s2 = 0; s2 < p.a.kw; ++s2)
            if (((unsigned)(ra_.hy - r) < (unsigned)p.a.Hs) &
                ((unsigned)(ra_.wx - s2) < (unsigned)p.a.Ws))
              mk |= 1u << (r * p.a.kw + s2);
      } else {
        if (m < p.M) mk = 1u;
      }
      amask[i] = mk;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int c = n0 + b_col;
      bbo[i] = c < Cin ? (uint32_t)((b_row0 + B_RSTEP * i) * T * Cin + c) * 4u : OOB;
    }
  } else {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) rowa[i] = row_init<GM>(p.a, m0 + (tid + NTHREADS * i) / CPR, p.M);
  }
  KPos kp{0, 0, 0};
  if constexpr (!UK) kp = kpos_init(p.a, kr.kt0 * KS + 8 * my_chunk);
  int u_c = 0, u_t = 0, u_r = 0, u_s = 0;     // UK: the next step's (channel, tap), uniform
  if constexpr (GM == GM_TAP) {
    u_t = (kr.kt0 * KS) / Cout;
    u_c = kr.kt0 * KS - u_t * Cout;
    u_r = u_t / p.a.kw;
    u_s = u_t - u_r * p.a.kw;
  }
  constexpr int SETS = fp32_sets<BM, BN>();
  uint4 ra[SETS][2 * A_CH], rb[SETS][2 * B_CH];

  auto load_tiles = [&](int kt, auto S) {
    constexpr int s = decltype(S)::value;
    const int k0 = kt * KS + 8 * my_chunk;
    const bool kok = k0 < kr.klim;
    if constexpr (UK) {
      const bool kup = kt * KS < kr.klim;
      uint32_t ko, wo;
      if constexpr (GM == GM_TAP) {
        ko = ((uint32_t)u_c - (uint32_t)(u_r * p.a.Ws + u_s) * (uint32_t)p.a.Ctot) * 4u;
        wo = (uint32_t)((u_c * T + u_t) * Cin) * 4u;
      } else {
        ko = (uint32_t)(kt * KS) * 4u;
        wo = (uint32_t)(kt * KS * Cin) * 4u;
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const uint32_t bit = GM == GM_TAP ? (amask[i] >> (u_t & 31)) & 1u : amask[i];
        const uint32_t o = (kup && bit) ? abo[i] + ko : OOB;
        ra[s][2 * i] = bload(rA, o);
        ra[s][2 * i + 1] = bload(rA, o + 16u);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const uint32_t o = kup ? bbo[i] + wo : OOB;
        rb[s][2 * i] = bload(rW, o);
        rb[s][2 * i + 1] = bload(rW, o + 16u);
      }
      if constexpr (GM == GM_TAP) {
        u_c += KS;
        if (u_c == Cout) {
          u_c = 0;
          ++u_t;
          if (++u_s == p.a.kw) {
            u_s = 0;
            ++u_r;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const uint32_t off = a_off<GM, 4>(p.a, rowa[i], kp.r, kp.s, kp.c);
      const uint32_t o = kok ? off : OOB;
      ra[s][2 * i] = bload(rA, o);
      ra[s][2 * i + 1] = bload(rA, o + 16u);
    }
    kpos_advance<KS>(p.a, kp);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int k = kt * KS + b_row0 + B_RSTEP * i;
      const int c = n0 + b_col;
      const int tap = (int)fdiv((uint32_t)k, dCout);
      const int n = k - tap * Cout;
      const uint32_t o = (k < kr.klim && c < Cin) ? (uint32_t)((n * T + tap) * Cin + c) * 4u : OOB;
      rb[s][2 * i] = bload(rW, o);
      rb[s][2 * i + 1] = bload(rW, o + 16u);
    }
  };
  auto store_tiles = [&](int buf, auto S) {
    constexpr int s = decltype(S)::value;
    bf16_t* sa = lds + buf * (BM * BK);
    bf16_t* sb = lds + NST * BM * BK + buf * (BK * BN);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid + NTHREADS * i) / CPR;
      if constexpr (CER_TIMING_NOAW) {
        keep_alive(ra[s][2 * i]);
        keep_alive(ra[s][2 * i + 1]);
        continue;
      }
      uint4 h, l;
      take_hi_lo(p.a_hl != 0, ra[s][2 * i], ra[s][2 * i + 1], h, l);
      *reinterpret_cast<uint4*>(sa + nt_off(row, my_chunk)) = h;
      *reinterpret_cast<uint4*>(sa + nt_off(row, my_chunk + 4)) = l;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = b_row0 + B_RSTEP * i;
      uint4 h, l;
      take_hi_lo(UK && p.w_hl != 0, rb[s][2 * i], rb[s][2 * i + 1], h, l);
      if constexpr (WIDE) {
        *reinterpret_cast<uint4*>(sb + tn_off_w<BN>(row, b_col)) = h;
        *reinterpret_cast<uint4*>(sb + tn_off_w<BN>(row + KS, b_col)) = l;
      } else {
        *reinterpret_cast<uint4*>(sb + tn_off<BN>(row, b_col)) = h;
        *reinterpret_cast<uint4*>(sb + tn_off<BN>(row + KS, b_col)) = l;
      }
    }
  };

  typename AccT<BM, BN, WIDE>::type acc;
  if constexpr (WIDE) {
    zero_accw<BM, BN>(acc);
    auto mma = [&](int cur) {
      mma3w_nn<BM, BN>(lds + cur * (BM * BK), lds + NST * BM * BK + cur * (BK * BN), wm, wn, lane,
                       acc);
    };
    kloop32<SETS>(kr.kt0, kr.kt1, load_tiles, store_tiles, mma);
    if (p.splits > 1 && !splitk_reduce_w<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    epi32w<BM, BN, true>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  } else {
    zero_acc<BM, BN>(acc);
    kloop32<SETS>(kr.kt0, kr.kt1, load_tiles, store_tiles, [&](int cur) {
      mma3_nn<BM, BN>(lds + cur * (BM * BK), lds + 2 * BM * BK + cur * (BK * BN), wm, wn, lane,
                      acc);
    });
    if (!group_reduce<WG, BM, BN>(acc, reinterpret_cast<float*>(lds_all), LDS_ELEMS / 2, grp,
                                  tid))
      return;
    if (p.splits > 1 && !splitk_reduce<BM, BN>(p, acc, cfg * tiles + tile, split, tid)) return;
    epi32<BM, BN, EPI>(p, acc, reinterpret_cast<float*>(lds), cfg, m0, n0, wm, wn, lane, tid);
  }
}

// wgrad tile body (fp32 operands): dW[n, k] = sum_m dy[m, n] im2col(x)[m, k]
template <int BM, int BN, int GM, bool WIDE = false>
__device__ __forceinline__ void wgrad_reg_body32(const WGParams& p, int work, bf16_t* lds) {
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;
  constexpr int A_CH = KS * A_CPR / NTHREADS, B_CH = KS * B_CPR / NTHREADS;
  constexpr int A_RSTEP = NTHREADS / A_CPR, B_RSTEP = NTHREADS / B_CPR;

  const int tiles_k = (p.K + BN - 1) / BN;
  const int tiles = ((p.N + BM - 1) / BM) * tiles_k;
  const int cfg = work / (tiles * p.splits);
  const int rem = work - cfg * tiles * p.splits;
  const int split = rem / tiles, tile = rem - split * tiles;
  const int tn_ = tile / tiles_k, tk = tile - tn_ * tiles_k;
  const int n0 = tn_ * BM, k0 = tk * BN;
  const int ms = split * p.m_per_split;
  const int me = min(p.Mred, ms + p.m_per_split);
  if (ms >= me) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wa = wid >> 1, wb = wid & 1;
  const int a_col = 8 * (tid % A_CPR), b_col = 8 * (tid % B_CPR);
  const int a_row0 = tid / A_CPR, b_row0 = tid / B_CPR;
  const int kk0 = k0 + b_col;
  const bool b_kok = kk0 < p.K;
  KPos bk{0, 0, 0};
  if (GM != GM_GEMM && b_kok) bk = kpos_init(p.x, kk0);
  // GM_TAP (k x k, stride 1, same-size output): a thread's x column (tap r,
  // s and channel c) is fixed for the whole block, so its x row address is
  // the dy row's pixel shifted by the tap -- a per-row base plus the
  // uniform step offset; only the tap's bounds test needs the row's pixel
  // (y, x), advanced by KS rows per step without a division
  int ty[B_CH], tx[B_CH];
  int dxs = 0, dys = 0, ry = 0, rx = 0;
  constexpr int SETS = wgrad_sets<BM, BN>();
  uint4 ra[SETS][2 * A_CH], rb[SETS][2 * B_CH];
  const float* dyb = reinterpret_cast<const float*>(p.dy) + (int64_t)cfg * p.N;
  const float* xb = reinterpret_cast<const float*>(p.x.src) + (int64_t)cfg * p.x.cfg_off;
  __amdgpu_buffer_rsrc_t rDY, rX;
  if constexpr (GM != GM_SLOW) {
    rDY = make_rsrc(dyb, (uint32_t)p.Mred * (uint32_t)p.ldy * 4u);
    rX = make_rsrc(xb, p.x.bytes);
  }
  // GM_GEMM (1x1, stride 1, pad 0: x rows = dy rows = the reduction index):
  // per-thread row / column byte bases; a step adds the uniform row offset
  uint32_t abo[A_CH], bbo[B_CH];
  if constexpr (GM == GM_GEMM || GM == GM_TAP) {
    const int n = n0 + a_col;
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      abo[i] = n < p.N ? (uint32_t)((a_row0 + A_RSTEP * i) * p.ldy + n) * 4u : OOB;
    if constexpr (GM == GM_GEMM) {
#pragma unroll
      for (int i = 0; i < B_CH; ++i)
        bbo[i] = b_kok ? (uint32_t)((b_row0 + B_RSTEP * i) * p.x.Ctot + kk0) * 4u : OOB;
    } else {
      ry = bk.r - p.x.pad;
      rx = bk.s - p.x.pad_w;
      const int dpix = ry * p.x.Ws + rx;
      dxs = KS % p.x.Wm;
      dys = (KS / p.x.Wm) % p.x.Hm;
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int m = ms + b_row0 + B_RSTEP * i;
        const RowPos q = decode_row(m, p.Mred, p.x);
        ty[i] = q.y;
        tx[i] = q.x;
        // offsets relative to the split's first row (ms): the step adds
        // (mbase - ms) rows; the uint32 arithmetic wraps for taps left of /
        // above the pixel, and a valid tap's offset wraps back into range
        bbo[i] = b_kok ? (uint32_t)((b_row0 + B_RSTEP * i + dpix) * p.x.Ctot + bk.c) * 4u +
                             (uint32_t)(ms * p.x.Ctot) * 4u
                       : OOB;
      }
    }
  }

  auto load_tiles = [&](int mt, auto S) {
    constexpr int s = decltype(S)::value;
    const int mbase = ms + mt * KS;
    if constexpr (GM == GM_GEMM || GM == GM_TAP) {
      const int left = me - mbase;                 // rows of this step inside the split
      const uint32_t ao = (uint32_t)(mbase * p.ldy) * 4u;
      const uint32_t xo = (uint32_t)((GM == GM_TAP ? mbase - ms : mbase) * p.x.Ctot) * 4u;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const uint32_t o = a_row0 + A_RSTEP * i < left ? abo[i] + ao : OOB;
        ra[s][2 * i] = bload(rDY, o);
        ra[s][2 * i + 1] = bload(rDY, o + 16u);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        bool ok = b_row0 + B_RSTEP * i < left;
        if constexpr (GM == GM_TAP) {
          ok = ok && ((unsigned)(ty[i] + ry) < (unsigned)p.x.Hs) &&
               ((unsigned)(tx[i] + rx) < (unsigned)p.x.Ws);
          // the next step's row pixel: KS rows on, within the image grid
          int xn = tx[i] + dxs;
          const int carry = xn >= p.x.Wm ? 1 : 0;
          xn -= carry ? p.x.Wm : 0;
          int yn = ty[i] + dys + carry;
          yn -= yn >= p.x.Hm ? p.x.Hm : 0;
          tx[i] = xn;
          ty[i] = yn;
        }
        const uint32_t o = ok ? bbo[i] + xo : OOB;
        rb[s][2 * i] = bload(rX, o);
        rb[s][2 * i + 1] = bload(rX, o + 16u);
      }
    } else if constexpr (GM != GM_SLOW) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int m = mbase + a_row0 + A_RSTEP * i, n = n0 + a_col;
        const uint32_t o = (m < me && n < p.N) ? (uint32_t)(m * p.ldy + n) * 4u : OOB;
        ra[s][2 * i] = bload(rDY, o);
        ra[s][2 * i + 1] = bload(rDY, o + 16u);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const RowA rr = row_init<GM_FWD>(p.x, mbase + b_row0 + B_RSTEP * i, me);
        const uint32_t off = a_off<GM_FWD, 4>(p.x, rr, bk.r, bk.s, bk.c);
        const uint32_t o = b_kok ? off : OOB;
        rb[s][2 * i] = bload(rX, o);
        rb[s][2 * i + 1] = bload(rX, o + 16u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int m = mbase + a_row0 + A_RSTEP * i, n = n0 + a_col;
        load_row8_slow32(dyb + (int64_t)m * p.ldy + n, (m < me && n < p.N) ? p.N - n : 0,
                         ra[s][2 * i], ra[s][2 * i + 1]);
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int m = mbase + b_row0 + B_RSTEP * i;
        const RowPos pos = decode_row(m, me, p.x);
        if (b_kok && pos.ok) {
          gather_chunk_slow32(p.x, cfg, pos, kk0, p.K, 0, rb[s][2 * i], rb[s][2 * i + 1]);
        } else {
          rb[s][2 * i] = make_uint4(0, 0, 0, 0);
          rb[s][2 * i + 1] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };
  auto store_tiles = [&](int buf, auto S) {
    constexpr int s = decltype(S)::value;
    bf16_t* sa = lds + buf * (BK * BM);
    bf16_t* sb = lds + 2 * BK * BM + buf * (BK * BN);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = a_row0 + A_RSTEP * i;
      uint4 h, l;
      take_hi_lo(p.dy_hl != 0, ra[s][2 * i], ra[s][2 * i + 1], h, l);
      if constexpr (WIDE) {
        *reinterpret_cast<uint4*>(sa + tn_off_w<BM>(row, a_col)) = h;
        *reinterpret_cast<uint4*>(sa + tn_off_w<BM>(row + KS, a_col)) = l;
      } else {
        *reinterpret_cast<uint4*>(sa + tn_off<BM>(row, a_col)) = h;
        *reinterpret_cast<uint4*>(sa + tn_off<BM>(row + KS, a_col)) = l;
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = b_row0 + B_RSTEP * i;
      uint4 h, l;
      take_hi_lo(p.x_hl != 0, rb[s][2 * i], rb[s][2 * i + 1], h, l);
      if constexpr (WIDE) {
        *reinterpret_cast<uint4*>(sb + tn_off_w<BN>(row, b_col)) = h;
        *reinterpret_cast<uint4*>(sb + tn_off_w<BN>(row + KS, b_col)) = l;
      } else {
        *reinterpret_cast<uint4*>(sb + tn_off<BN>(row, b_col)) = h;
        *reinterpret_cast<uint4*>(sb + tn_off<BN>(row + KS, b_col)) = l;
      }
    }
  };

  const int MT = (me - ms + KS - 1) / KS;
  float* dwb = p.dw + (int64_t)cfg * p.dw_gstride;
  const bool split_k = p.splits > 1;
  if constexpr (WIDE) {
    f32x16 acc[BM / 64][BN / 64];
    zero_accw<BM, BN>(acc);
    kloop32<SETS>(0, MT, load_tiles, store_tiles, [&](int cur) {
      mma3w_tn<BM, BN>(lds + cur * (BK * BM), lds + 2 * BK * BM + cur * (BK * BN), wa, wb, lane,
                       acc);
    });
    // D[n][k]: k = lane & 31 (32 consecutive k per register: 128-B stores)
    constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 32, FN = TN / 32;
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = n0 + wa * TM + 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
          const int k = k0 + wb * TN + 32 * j + r;
          if (n < p.N && k < p.K) {
            float* d = dwb + (int64_t)n * p.K + k;
            if (split_k)
              atomicAdd(d, acc[i][j][e]);
            else
              *d = acc[i][j][e];
          }
        }
  } else {
    f32x4 acc[BM / 32][BN / 32];
    zero_acc<BM, BN>(acc);
    kloop32<SETS>(0, MT, load_tiles, store_tiles, [&](int cur) {
      mma3_tn<BM, BN>(lds + cur * (BK * BM), lds + 2 * BK * BM + cur * (BK * BN), wa, wb, lane,
                      acc);
    });
    constexpr int TM = BM / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;
    const int fr = lane & 15, fc = lane >> 4;
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
            if (split_k)
              atomicAdd(d, acc[i][j][e]);
            else
              *d = acc[i][j][e];
          }
        }
  }
}

template <int BM, int BN, int GM, bool WIDE = false>
__global__ __launch_bounds__(NTHREADS, (fp32_occ<BM, BN>())) void igemm_wgrad32(WGParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (BM + BN) * BK];
  wgrad_reg_body32<BM, BN, GM, WIDE>(p, xcd_remap(blockIdx.x, gridDim.x), lds);
}

// batched fp32 weight gradients (see wgrad_batch)
template <int BM, int BN, bool WIDE = false>
// A grid smaller than the batch's work items (cer_wgrad_batch_set_grid: a
// side-stream batch that should leave most CUs to the dgrad chain) walks the
// items persistently, block-strided; the full grid takes one item per block
// in XCD-aware order.
__global__ __launch_bounds__(NTHREADS, (fp32_occ<BM, BN>())) void wgrad_batch32(WGBatch b) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (BM + BN) * BK];
  const int total = b.start[b.n];
  const int nwg = (int)gridDim.x;
  for (int w = blockIdx.x; w < total; w += nwg) {
    const int work = nwg >= total ? xcd_remap(w, nwg) : w;
    int i = 0;
    while (i + 1 < b.n && work >= b.start[i + 1]) ++i;
    const WGParams p = b.p[i];
    if (p.gemm == 1)
      wgrad_reg_body32<BM, BN, GM_GEMM, WIDE>(p, work - b.start[i], lds);
    else if (p.gemm == 2)
      wgrad_reg_body32<BM, BN, GM_TAP, WIDE>(p, work - b.start[i], lds);
    else
      wgrad_reg_body32<BM, BN, GM_FWD, WIDE>(p, work - b.start[i], lds);
    if (w + nwg < total) __syncthreads();     // the next item restages the LDS images
  }
}

// ---------------------------------------------------------------------------
// per-config weight transpose for dgrad: W[N][T][C] -> Wt[C][T][N]
// ---------------------------------------------------------------------------
template <typename E>
__global__ __launch_bounds__(256) void transpose_w_kernel(const E* __restrict__ w,
                                                          int64_t w_gstride,
                                                          E* __restrict__ wt, int N,
                                                          int T, int C) {
  __shared__ E tile[32][33];
  const int cfg = blockIdx.z;
  const int t = blockIdx.y;
  const int tiles_c = (C + 31) / 32;
  const int tn = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const E* src = w + (int64_t)cfg * w_gstride;
  E* dst = wt + (int64_t)cfg * N * T * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int yy = ty; yy < 32; yy += 8) {
    const int n = tn * 32 + yy, c = tc * 32 + tx;
    tile[yy][tx] = (n < N && c < C) ? src[((int64_t)n * T + t) * C + c] : (E)0;
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
// Kernel variants: (staging kind) x (tile).  kind 0 = register-staged
// double buffer, 1 = LDS-DMA ring; tile 0 = 64x64, 1 = 128x128, 2 = 128x64
// (BM x BN; for wgrad BM tiles Cout, BN tiles K).  v = 3 * kind + tile.
// fp32 only: 12-23 = the 32x32x16-MFMA twins of 0-11; 24-35 = the
// intra-block K-split (512-thread, 2 wave groups) twins of the
// register-staged fwd / dgrad kernels (ring ids map to their register twin;
// 128x128 has none).  Four groups (1024 threads, 64x64) measured neutral at
// G = 1 (profiles/r3_ksplit.md) and are not instantiated.
// cer_conv_set_variant(op, v) pins a variant per op (0 fwd, 1 dgrad, 2 wgrad)
// for tuning; -1 = the built-in choice.
static int g_variant[3] = {-1, -1, -1};

CER_API void cer_conv_set_variant(int op, int v) {
  if (op >= 0 && op < 3) g_variant[op] = v;
}

// uniform-K fp32 kernels (GM_GEMM / GM_TAP: conv fwd, dgrad and the 1x1
// wgrad).  CER_UK=0 (or cer_conv_set_uk(0)) keeps the
// per-chunk im2col addressing for A/B runs.
static int g_uk = -1;
static bool uk_on() {
  if (g_uk < 0) {
    const char* e = getenv("CER_UK");
    g_uk = e ? atoi(e) : 1;
  }
  return g_uk > 0;
}
CER_API void cer_conv_set_uk(int on) { g_uk = on ? 1 : 0; }

// HL image of the weights for the NEXT fp32 fwd / dgrad launch (same layout
// and per-config stride as w; the optimizer writes it, runtime/arena.py
// Arena.whl); used by the uniform-K kernels only, null = split in the K loop
static const void* g_whl = nullptr;
static int64_t g_whl_gstride = 0;
CER_API void cer_conv_set_whl(const void* whl, int64_t gstride) {
  g_whl = whl;
  g_whl_gstride = whl ? gstride : 0;
}

// split-K workspace (persistent; registered by the host before launches)
struct SplitKWs {
  float* ws = nullptr;
  int64_t floats = 0;
  unsigned* cnt = nullptr;
  int ncnt = 0;
};
static SplitKWs g_sk;

CER_API void cer_conv_set_splitk(float* ws, int64_t floats, unsigned* cnt, int ncnt) {
  g_sk.ws = ws;
  g_sk.floats = floats;
  g_sk.cnt = cnt;
  g_sk.ncnt = ncnt;
}

static long ntiles(long M, long N, int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

// built-in choice (from the per-shape sweep of tools/bench_conv --sweep)
static int choose(int op, long M, long N, long K, int G, bool pipe_ok) {
  if (g_variant[op] >= 0) {
    int v = g_variant[op];
    // fp32 twins: 12-23 wide, 24-35 intra-block K split
    int wide = v >= 24 ? 24 : v >= 12 ? 12 : 0;
    v -= wide;
    if (op == 2 && wide >= 24) wide = 0;            // wgrad: no K-split twins here
    if (op == 2 && v >= 6) v -= 6;                  // wgrad has its own split-K
    v += wide;
    if (((v / 3) & 1) && !pipe_ok) v -= 3;
    return v;
  }
  if (op != 2 && ntiles(M, N, 64, 64) * G < 128 && K / BK >= 16)
    return 6;                                       // too few tiles to fill the chip
  int tile;
  if (op == 2) {
    tile = ntiles(N, K, 128, 128) * G >= 256 ? 1 : 0;
  } else if (N <= 64) {
    tile = ntiles(M, N, 128, 64) * G >= 512 ? 2 : 0;
  } else {
    tile = ntiles(M, N, 128, 128) * G >= 512 ? 1 : 0;
  }
  return tile;
}

static void tile_dims(int v, int& bm, int& bn) {
  const int t = v % 3;
  bm = t == 0 ? 64 : 128;
  bn = t == 1 ? 128 : 64;
}

// split count for a fwd / dgrad GEMM: enough blocks for ~1.5 waves of 256 CUs
// (SK_TARGET), at most SK_MAX splits, >= 4 K tiles per split, within the
// registered workspace (more, shorter splits lose at one config: each pays
// the prologue, the partial-slot round trip and the last-arriver reduction;
// r2_ab_kernel_knobs.md)
constexpr int SK_TARGET = 384, SK_MAX = 8;

static int nt_splits(const NTParams& p, int G, int bm, int bn, int ks) {
  const long tiles = ntiles(p.M, p.N, bm, bn) * G;
  const int KT = (p.K + ks - 1) / ks;
  const int target = SK_TARGET;
  const int smax = SK_MAX;
  int s = (int)((target + tiles - 1) / tiles);
  if (s > smax) s = smax;
  if (s > KT / 4) s = KT / 4;
  if (s < 2 || !g_sk.ws || tiles > g_sk.ncnt) return 1;
  const int per = (KT + s - 1) / s;
  s = (KT + per - 1) / per;
  if ((int64_t)tiles * s * bm * bn > g_sk.floats) return 1;
  return s;
}

static void set_splits(NTParams& p, int G, int v, int ks = BK) {
  int bm, bn;
  tile_dims(v, bm, bn);
  p.splits = (v / 3) >= 2 ? nt_splits(p, G, bm, bn, ks) : 1;
  p.skws = g_sk.ws;
  p.skcnt = g_sk.cnt;
}

template <int BM, int BN>
static void launch_nt_t(const NTParams& p, int G, int kind, bool fast, hipStream_t stream) {
  dim3 grid((unsigned)(ntiles(p.M, p.N, BM, BN) * G * p.splits));
  if (kind == 1) {
    if (p.K / BK >= 3)
      pipe_nt<BM, BN, 3><<<grid, NTHREADS, 0, stream>>>(p);
    else
      pipe_nt<BM, BN, 2><<<grid, NTHREADS, 0, stream>>>(p);
  } else if (fast) {
    igemm_nt<BM, BN, GM_FWD><<<grid, NTHREADS, 0, stream>>>(p);
  } else {
    igemm_nt<BM, BN, GM_SLOW><<<grid, NTHREADS, 0, stream>>>(p);
  }
}

// fast = 8-channel aligned operands addressed by 32-bit buffer offsets
static bool nt_fast(const NTParams& p) {
  return p.dgrad == 0 && (p.a.Cg % 8 == 0) && (p.a.Ctot % 8 == 0) && (p.K % 8 == 0) &&
         p.a.bytes != 0 && (uint64_t)p.N * p.K * 2 < (1ull << 31);
}

static int run_nt(NTParams p, int G, hipStream_t stream, int* nslab = nullptr) {
  p.stat_slabs = p.stats ? g_stat_slabs : 0;
  const bool fast = nt_fast(p);
  const bool pipe_ok = fast && p.a.Cg % 64 == 0;
  int v = choose(0, p.M, p.N, p.K, G, pipe_ok);
  v %= 12;                                          // wide / K-split ids: fp32 kernels only
  if (!fast) v = (v >= 6 ? 6 : 0) + v % 3;         // generic gather: register-staged only
  set_splits(p, G, v);
  const int kind = (v / 3) & 1;
  if (nslab) {
    int bm, bn;
    tile_dims(v, bm, bn);
    *nslab = stat_nslab((int)((p.M + bm - 1) / bm), p.stat_slabs);
  }
  switch (v % 3) {
    case 0: launch_nt_t<64, 64>(p, G, kind, fast, stream); break;
    case 1: launch_nt_t<128, 128>(p, G, kind, fast, stream); break;
    default: launch_nt_t<128, 64>(p, G, kind, fast, stream); break;
  }
  return (int)hipGetLastError();
}

// ---- fp32 (3-pass split-bf16) launches: register-staged variants only; an
// LDS-DMA variant id maps to its register-staged twin (v - 3)
// register-staged fp32 forward kernel of addressing mode gm (GM_FWD /
// GM_GEMM / GM_TAP; GM_SLOW for unaligned operands)
template <int BM, int BN, bool WIDE, int WG>
static void nt32_go(int gm, dim3 grid, const NTParams& p, hipStream_t stream) {
  const unsigned th = NTHREADS * WG;
  switch (gm) {
    case GM_GEMM: igemm_nt32<BM, BN, GM_GEMM, WIDE, WG><<<grid, th, 0, stream>>>(p); break;
    case GM_TAP: igemm_nt32<BM, BN, GM_TAP, WIDE, WG><<<grid, th, 0, stream>>>(p); break;
    case GM_SLOW: igemm_nt32<BM, BN, GM_SLOW, WIDE, WG><<<grid, th, 0, stream>>>(p); break;
    default: igemm_nt32<BM, BN, GM_FWD, WIDE, WG><<<grid, th, 0, stream>>>(p); break;
  }
}

template <int BM, int BN>
static void launch_nt32_t(const NTParams& p, int G, bool fast, int kind, hipStream_t stream,
                          bool wide = false, int wg = 1, int gm = GM_FWD) {
  dim3 grid((unsigned)(ntiles(p.M, p.N, BM, BN) * G * p.splits));
  if (!fast) gm = GM_SLOW;
  if constexpr (BM * BN <= 128 * 64) {
    if (wg > 1 && fast && kind == 0 && !wide) {    // intra-block K split, 512 threads
      nt32_go<BM, BN, false, 2>(gm, grid, p, stream);
      return;
    }
  }
  if (wide) {                      // 32x32x16 MFMA twins
    if (kind == 1) {
      if constexpr (BM * BN <= 128 * 64)
        if (p.K / KS >= 3) {
          pipe_nt32<BM, BN, 3, true><<<grid, NTHREADS, 0, stream>>>(p);
          return;
        }
      pipe_nt32<BM, BN, 2, true><<<grid, NTHREADS, 0, stream>>>(p);
    } else {
      nt32_go<BM, BN, true, 1>(gm, grid, p, stream);
    }
    return;
  }
  if (kind == 1) {
    // 128x128: two stages keep 2 workgroups per CU (3 x 32 KiB would not)
    if constexpr (BM * BN <= 128 * 64)
      if (p.K / KS >= 3) {
        pipe_nt32<BM, BN, 3><<<grid, NTHREADS, 0, stream>>>(p);
        return;
      }
    pipe_nt32<BM, BN, 2><<<grid, NTHREADS, 0, stream>>>(p);
  } else {
    nt32_go<BM, BN, false, 1>(gm, grid, p, stream);
  }
}

// uniform-K addressing mode of an fp32 forward GEMM (0 = none)
static int nt_uk_mode(const NTParams& p, bool fast) {
  const GatherGeom& g = p.a;
  if (!fast || !uk_on() || p.dgrad || g.Cg % KS || p.K % KS) return 0;
  if (g.kh == 1 && g.kw == 1 && g.pad == 0 && g.pad_w == 0) return GM_GEMM;
  return g.kh * g.kw <= 32 ? GM_TAP : 0;
}

static bool nt_fast32(const NTParams& p) {
  return p.dgrad == 0 && (p.a.Cg % 8 == 0) && (p.a.Ctot % 8 == 0) && (p.K % 8 == 0) &&
         p.a.bytes != 0 && (uint64_t)p.N * p.K * 4 < (1ull << 31);
}

static int fp32_variant(int v) { return (v >= 6 ? 6 : 0) + v % 3; }

// fp32 forward variants: 0-2 register-staged, 3-5 LDS-DMA ring (pipe_nt32),
// 6-8 register-staged split-K, 9-11 ring split-K (v % 3 = tile shape);
// 12-23: the same twelve on the 32x32x16 MFMA (wide) kernels
static int run_nt32(NTParams p, int G, hipStream_t stream, int* nslab = nullptr) {
  p.stat_slabs = p.stats ? g_stat_slabs : 0;
  const bool fast = nt_fast32(p);
  if (p.a_hl && !fast) return (int)hipErrorInvalidValue;
  const bool ring_ok = fast && p.a.Cg % KS == 0;
  int v = choose(0, p.M, p.N, p.K, G, ring_ok);
  bool wide = false;
  int wg = 1;
  if (v >= 24) {
    wg = 2;
    v -= 24;
    if ((v / 3) & 1) v -= 3;                       // register-staged kernels only
  } else if (v >= 12) {
    v -= 12;
    // BN-backward statistics (the unaligned-dgrad fallback) only in the NN
    // kernels' wide epilogue
    wide = p.bb.part == nullptr;
    if (((v / 3) & 1) && !ring_ok) v -= 3;
  }
  if (!fast) v = fp32_variant(v);
  // a launch carrying an addend or BN-backward operands (the unaligned dgrad
  // fallback) never reaches the uniform-K or ring kernels, whose epilogue is
  // the lean forward one (epi32 EPI_FWD)
  const bool epi_plain = p.addend == nullptr && p.addend_mask == nullptr && p.bb.part == nullptr;
  if (((v / 3) & 1) && !epi_plain) v -= 3;
  const int kind = (v / 3) & 1;
  set_splits(p, G, v, KS);
  if (nslab) {
    int bm, bn;
    tile_dims(v, bm, bn);
    *nslab = stat_nslab((int)((p.M + bm - 1) / bm), p.stat_slabs);
  }
  // register-staged kernels: uniform-K addressing; with it, and in the
  // LDS-DMA ring kernels (their own addressing), the HL weight image
  const int gm = kind == 0 && epi_plain ? nt_uk_mode(p, fast) : 0;
  // the aligned gather (GM_FWD) kernels carry the lean forward epilogue too:
  // an addend / BN-backward launch only ever comes through the unaligned
  // dgrad fallback (p.dgrad = 1, GM_SLOW); refuse anything else loudly
  if (fast && !epi_plain) return (int)hipErrorInvalidValue;
  if ((gm || kind == 1) && p.w_hl) {   // the caller allowed the HL image (not grouped)
    p.w = reinterpret_cast<const bf16_t*>(g_whl);
    p.w_gstride = g_whl_gstride;
  } else {
    p.w_hl = 0;
  }
  switch (v % 3) {
    case 0: launch_nt32_t<64, 64>(p, G, fast, kind, stream, wide, wg, gm ? gm : GM_FWD); break;
    case 1: launch_nt32_t<128, 128>(p, G, fast, kind, stream, wide, 1, gm ? gm : GM_FWD); break;
    default: launch_nt32_t<128, 64>(p, G, fast, kind, stream, wide, wg, gm ? gm : GM_FWD); break;
  }
  return (int)hipGetLastError();
}

static int conv_fwd_impl(const void* x, int B, int H, int W, int Cin, int G, const void* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         void* y, int Ho, int Wo, const void* bias, int64_t bias_gstride,
                         int act, float* stats, int* nslab, bool f32, hipStream_t stream,
                         int ctot = 0, int ldc = 0, uint32_t shift = 0);


CER_API int cer_conv_fwd(const bf16_t* x, int B, int H, int W, int Cin, int G, const bf16_t* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         bf16_t* y, int Ho, int Wo, const bf16_t* bias, int64_t bias_gstride,
                         int act, hipStream_t stream) {
  return conv_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo, bias,
                       bias_gstride, act, nullptr, nullptr, false, stream);
}

CER_API int cer_conv_fwd_f32(const float* x, int B, int H, int W, int Cin, int G, const float* w,
                             int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                             float* y, int Ho, int Wo, const float* bias, int64_t bias_gstride,
                             int act, hipStream_t stream) {
  return conv_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo, bias,
                       bias_gstride, act, nullptr, nullptr, true, stream);
}

// forward + BN statistics partials (bias-free, no activation): part holds
// cer_conv_stats_floats(M, C) floats; *nslab receives the slab count to hand
// to the BN finalize
CER_API int cer_conv_fwd_stats(const bf16_t* x, int B, int H, int W, int Cin, int G,
                               const bf16_t* w, int64_t w_gstride, int Cout, int kh, int kw,
                               int st, int pad, bf16_t* y, int Ho, int Wo, float* part,
                               int* nslab, hipStream_t stream) {
  return conv_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo,
                       nullptr, 0, 0, part, nslab, false, stream);
}

CER_API int cer_conv_fwd_stats_f32(const float* x, int B, int H, int W, int Cin, int G,
                                   const float* w, int64_t w_gstride, int Cout, int kh, int kw,
                                   int st, int pad, float* y, int Ho, int Wo, float* part,
                                   int* nslab, hipStream_t stream) {
  return conv_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo,
                       nullptr, 0, 0, part, nslab, true, stream);
}

// upper bound over tile choices: one slab per 64-row M tile
CER_API int64_t cer_conv_stats_floats(int64_t M, int C) {
  return ((M + 63) / 64) * 2 * (int64_t)C;
}

static int conv_fwd_impl(const void* x, int B, int H, int W, int Cin, int G, const void* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         void* y, int Ho, int Wo, const void* bias, int64_t bias_gstride,
                         int act, float* stats, int* nslab, bool f32, hipStream_t stream,
                         int ctot, int ldc, uint32_t shift) {
  // ctot / ldc: channel pitch of x / y when they hold more than these G
  // packed blocks (grouped convs launch per config on shifted pointers;
  // ``shift`` = bytes x was advanced by, taken off the buffer-load range)
  NTParams p;
  p.a = make_geom(x, B, ctot ? ctot : G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad, f32 ? 4 : 2);
  if (p.a.bytes) p.a.bytes -= shift;
  p.dgrad = 0;
  p.w = reinterpret_cast<const bf16_t*>(w);
  p.w_gstride = w_gstride;
  p.out = reinterpret_cast<bf16_t*>(y);
  p.ldc = ldc ? ldc : G * Cout;
  p.M = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  p.bias = reinterpret_cast<const bf16_t*>(bias);
  p.bias_gstride = bias_gstride;
  p.act = act;
  p.o_st = 1;
  p.o_H = Ho;
  p.o_W = Wo;
  p.stats = stats;
  if (f32) {
    p.a_hl = g_hl_x;
    if (p.a_hl && (ctot || ldc)) return (int)hipErrorInvalidValue;   // grouped: no HL
    p.w_hl = g_whl && !ctot && !ldc ? 1 : 0;    // run_nt32 decides whether to read it
  }
  return f32 ? run_nt32(p, G, stream, nslab) : run_nt(p, G, stream, nslab);
}

template <int BM, int BN>
static void launch_nn_t(const NTParams& p, int G, int T, int kind, bool strided,
                        hipStream_t stream) {
  dim3 grid((unsigned)(ntiles(p.M, p.N, BM, BN) * G * p.splits));
  if (kind == 1) {
    const bool s3 = p.K / BK >= 3;
    if (strided) {
      if (s3)
        pipe_nn<BM, BN, 3, GM_DGS><<<grid, NTHREADS, 0, stream>>>(p, T);
      else
        pipe_nn<BM, BN, 2, GM_DGS><<<grid, NTHREADS, 0, stream>>>(p, T);
    } else {
      if (s3)
        pipe_nn<BM, BN, 3, GM_DG1><<<grid, NTHREADS, 0, stream>>>(p, T);
      else
        pipe_nn<BM, BN, 2, GM_DG1><<<grid, NTHREADS, 0, stream>>>(p, T);
    }
    return;
  }
  const FastDiv dc = make_div((uint32_t)p.a.Cg);
  if (strided)
    igemm_nn_dgrad<BM, BN, GM_DGS><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
  else
    igemm_nn_dgrad<BM, BN, GM_DG1><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
}

// dx = dgrad(dy, W).  Aligned channels: NN kernel (weights read in place, no
// transpose); a strided 1x1 conv only computes the B*Ho*Wo rows that receive
// gradient (the rest of dx is zero-filled).  Otherwise the transpose + NT path.
// wt: scratch of G * Cout*kh*kw*Cin elements (used by the fallback only)
// BN-backward statistics for the NEXT cer_conv_dgrad calls (until cleared
// with part == nullptr): see BNBwdEpi.  *nslab_out receives the partial count
// (M tiles of the variant that ran).  bn_mask_mode is bn.hip's YM rule.
int bn_mask_mode(int act, int has_res);
static BNBwdEpi g_bb = BNBwdEpi{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr,
                                0, 0, 0};
static int* g_bb_nslab = nullptr;

// the next strided-1x1 dgrads' addend is zero off their stride grid (st; 0:
// unknown): a ResNet stage transition, where c1 and the projection shortcut
// are both strided 1x1 convs of one BN output, so the first one's parked dx
// holds zeros wherever the second one writes nothing.  Every nonzero dx pixel
// then comes out of the second one's epilogue, which can compute the BN-link
// statistics (the zero pixels add nothing to sum dz and sum dz * xhat).
static int g_addend_grid = 0;
CER_API void cer_conv_set_addend_grid(int st) { g_addend_grid = st; }

// the next fp32 cer_conv_dgrad calls' addend is masked by these bits
// ([M][ldc / 8] bytes, NTParams::addend_mask; nullptr: off).  Only the
// aligned, non-strided NN path applies it: the others return an error
// instead of adding the unmasked addend.
static const uint8_t* g_addend_mask = nullptr;
CER_API void cer_conv_set_addend_mask(const void* m) {
  g_addend_mask = reinterpret_cast<const uint8_t*>(m);
}

// z, y, gamma, beta: bf16 for cer_conv_dgrad, fp32 for cer_conv_dgrad_f32
CER_API void cer_conv_dgrad_bnbwd(float* part, const void* z, const void* y,
                                  const float* mean, const float* invstd, const void* gamma,
                                  int64_t gstride, const void* beta, int64_t bstride, int act,
                                  int has_res, int* nslab_out) {
  g_bb = BNBwdEpi{part, reinterpret_cast<const bf16_t*>(z), reinterpret_cast<const bf16_t*>(y),
                  mean, invstd, reinterpret_cast<const bf16_t*>(gamma), gstride,
                  reinterpret_cast<const bf16_t*>(beta), bstride, bn_mask_mode(act, has_res), act};
  g_bb_nslab = part ? nslab_out : nullptr;
}

// bias-act link (YM_BIAS) for the NEXT fp32 cer_conv_dgrad calls, until
// cleared with dbias == nullptr: dbias = the linked layer's bias gradient
// (fp32, config stride dbstride), y = its fp32 output act(conv + b), act =
// its activation code.  *done_out is set non-zero by a launch that applied it
// (aligned NN path, stride 1, no addend); zero means the caller runs the
// layer's own bias_act_bwd.
CER_API void cer_conv_dgrad_babwd(float* dbias, int64_t dbstride, const void* y, int act,
                                  int* done_out) {
  g_bb = BNBwdEpi{dbias, reinterpret_cast<const bf16_t*>(y), nullptr, nullptr, nullptr, nullptr,
                  dbstride, nullptr, 0, YM_BIAS, act};
  g_bb_nslab = dbias ? done_out : nullptr;
  if (!dbias) g_bb.ym = 0;
}

template <int BM, int BN>
static void launch_nn32_t(const NTParams& p, int G, int T, bool strided, hipStream_t stream,
                          bool wide = false, int wg = 1, int gm = 0) {
  dim3 grid((unsigned)(ntiles(p.M, p.N, BM, BN) * G * p.splits));
  const FastDiv dc = make_div((uint32_t)p.a.Cg);
  if (gm) {                        // uniform-K addressing (GM_GEMM / GM_TAP)
    // a BN link with the mask from z and nothing else (the c2 / c3 dgrads of
    // a bottleneck) takes the lean epilogue (epi32 EPI_ZLINK)
    const bool zl = p.bb.part != nullptr && p.bb.ym == 2 && p.addend == nullptr &&
                    p.addend_mask == nullptr && p.bias == nullptr;
    // a residual join's BN link (stored activation bits), any addend
    const bool jn = p.bb.part != nullptr && p.bb.ym == 3 && p.bias == nullptr;
    // no BN link at all (the input is not a BN output), addend only
    const bool ad = p.bb.part == nullptr && p.bias == nullptr && p.stats == nullptr;
    // the bias-act link (VGG's conv -> conv) and nothing else
    const bool bl = p.bb.part != nullptr && p.bb.ym == YM_BIAS && p.addend == nullptr &&
                    p.addend_mask == nullptr && p.bias == nullptr;
    if constexpr (BM * BN <= 128 * 64) {
      if (wg > 1 && !wide) {
        if (gm == GM_GEMM) {
          if (zl)
            igemm_nn32<BM, BN, GM_GEMM, false, 2, EPI_ZLINK><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
          else if (jn)
            igemm_nn32<BM, BN, GM_GEMM, false, 2, EPI_JOIN><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
          else if (ad)
            igemm_nn32<BM, BN, GM_GEMM, false, 2, EPI_ADD><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
          else
            igemm_nn32<BM, BN, GM_GEMM, false, 2><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
        } else {
          if (zl)
            igemm_nn32<BM, BN, GM_TAP, false, 2, EPI_ZLINK><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
          else
            igemm_nn32<BM, BN, GM_TAP, false, 2><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
        }
        return;
      }
    }
    if (wide) {
      if (gm == GM_GEMM)
        igemm_nn32<BM, BN, GM_GEMM, true><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else
        igemm_nn32<BM, BN, GM_TAP, true><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
    } else if (gm == GM_GEMM) {
      if (zl)
        igemm_nn32<BM, BN, GM_GEMM, false, 1, EPI_ZLINK><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else if (jn)
        igemm_nn32<BM, BN, GM_GEMM, false, 1, EPI_JOIN><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else if (ad)
        igemm_nn32<BM, BN, GM_GEMM, false, 1, EPI_ADD><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else if (bl)
        igemm_nn32<BM, BN, GM_GEMM, false, 1, EPI_BLINK><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else
        igemm_nn32<BM, BN, GM_GEMM><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
    } else {
      if (zl)
        igemm_nn32<BM, BN, GM_TAP, false, 1, EPI_ZLINK><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else if (bl)
        igemm_nn32<BM, BN, GM_TAP, false, 1, EPI_BLINK><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
      else
        igemm_nn32<BM, BN, GM_TAP><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
    }
    return;
  }
  if constexpr (BM * BN <= 128 * 64) {
    if (wg > 1 && !wide) {                         // intra-block K split, 512 threads
      if (strided)
        igemm_nn32<BM, BN, GM_DGS, false, 2><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
      else
        igemm_nn32<BM, BN, GM_DG1, false, 2><<<grid, 2 * NTHREADS, 0, stream>>>(p, T, dc);
      return;
    }
  }
  if (wide) {                      // 32x32x16 MFMA twins
    if (strided)
      igemm_nn32<BM, BN, GM_DGS, true><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
    else
      igemm_nn32<BM, BN, GM_DG1, true><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
    return;
  }
  if (strided)
    igemm_nn32<BM, BN, GM_DGS><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
  else
    igemm_nn32<BM, BN, GM_DG1><<<grid, NTHREADS, 0, stream>>>(p, T, dc);
}

static int conv_dgrad_impl(const void* dy, int B, int Ho, int Wo, int Cout, int G, const void* w,
                           int64_t w_gstride, void* wt, int Cin, int kh, int kw, int st, int pad,
                           void* dx, int H, int W, const void* addend, bool f32,
                           hipStream_t stream, int cout_tot = 0, int cin_tot = 0,
                           uint32_t shift = 0) {
  // cout_tot / cin_tot: channel pitch of dy / dx (grouped convs, per-config
  // launches on shifted pointers; ``shift`` = bytes dy was advanced by)
  const int T = kh * kw;
  const int es = f32 ? 4 : 2;
  const int ctot_dy = cout_tot ? cout_tot : G * Cout;
  NTParams p;
  p.addend = reinterpret_cast<const bf16_t*>(addend);  // dx = dgrad + addend (null: dx = dgrad)
  if (g_addend_mask) {
    const bool strided1 = kh == 1 && kw == 1 && pad == 0 && st > 1;
    if (!f32 || !addend || strided1 || Cout % 8 || Cin % 8 || cout_tot || cin_tot)
      return (int)hipErrorInvalidValue;
    p.addend_mask = g_addend_mask;
  }
  p.stats = nullptr;
  p.bias = nullptr;
  p.bias_gstride = 0;
  p.act = 0;
  p.o_st = 1;
  p.o_H = H;
  p.o_W = W;
  p.out = reinterpret_cast<bf16_t*>(dx);
  p.ldc = cin_tot ? cin_tot : G * Cin;
  p.N = Cin;
  p.K = T * Cout;
  const bool aligned = (Cout % 8 == 0) && (Cin % 8 == 0) &&
                       (uint64_t)B * Ho * Wo * ctot_dy * es < (1ull << 31) &&
                       (uint64_t)Cout * T * Cin * es < (1ull << 31);
  if (f32) {
    p.a_hl = g_hl_dy;
    if (p.a_hl && (cout_tot || cin_tot)) return (int)hipErrorInvalidValue;   // grouped: no HL
  }
  if (p.addend_mask && !aligned) return (int)hipErrorInvalidValue;
  if (aligned) {
    p.w = reinterpret_cast<const bf16_t*>(w);
    p.w_gstride = w_gstride;
    bool strided = false;
    if (kh == 1 && kw == 1 && pad == 0 && st > 1) {
      if (cin_tot) return (int)hipErrorInvalidValue;   // grouped: not a strided 1x1
      // rows (b, ho, wo) of dy map to dx pixels (b, ho*st, wo*st); others get 0
      // (or the addend, which the kernel adds on the written pixels)
      const size_t bytes = (size_t)es * B * H * W * G * Cin;
      if (addend) {
        if (addend != dx) cer_copy_async(dx, addend, bytes, stream);   // in place: nothing to copy
      } else {
        cer_zero_async(dx, bytes, stream);
      }
      p.a = make_geom(dy, B, G * Cout, Cout, Ho, Wo, Ho, Wo, 1, 1, 1, 0, es);
      p.dgrad = 0;
      p.M = B * Ho * Wo;
      p.o_st = st;
    } else {
      p.a = make_geom(dy, B, ctot_dy, Cout, Ho, Wo, H, W, kh, kw, st, pad, es);
      if (p.a.bytes) p.a.bytes -= shift;
      p.dgrad = 1;
      p.M = B * H * W;
      strided = st > 1;
    }
    int v = choose(1, p.M, p.N, p.K, G, !f32 && Cout % 64 == 0);
    bool wide = false;
    int wg = 1;
    if (v >= 24) {                        // fp32 intra-block K-split twins
      wg = f32 ? 2 : 1;
      v -= 24;
    } else if (v >= 12) {                 // fp32 32x32x16-MFMA twins of 0-11
      v -= 12;
      wide = f32;
    }
    if (f32) v = fp32_variant(v);
    set_splits(p, G, v, f32 ? KS : BK);
    const int kind = (v / 3) & 1;
    // BN-backward statistics: every nonzero dx pixel must come out of the
    // epilogue (a strided 1x1 dgrad leaves pixels at zero: fine without an
    // addend, or with one that is zero off the same grid)
    const bool bb_ok = g_bb.ym == YM_BIAS ? f32 && p.o_st == 1 && !addend
                                          : p.o_st == 1 || !addend || g_addend_grid == p.o_st;
    if (g_bb.part && bb_ok) {
      p.bb = g_bb;
      p.stat_slabs = g_stat_slabs;
      int bm, bn;
      tile_dims(v, bm, bn);
      if (g_bb_nslab) *g_bb_nslab = stat_nslab((p.M + bm - 1) / bm, g_stat_slabs);
    } else if (g_bb_nslab) {
      *g_bb_nslab = 0;                    // not produced: the BN runs its own partials
    }
    if (f32) {
      // uniform-K addressing: the 1x1 geometry (stride-1 1x1 and the
      // strided 1x1's dy rows) and stride-1 k x k, a K step (32 output
      // channels) inside one tap; with it the HL weight image (not grouped)
      int gm = 0;
      if (uk_on() && Cout % KS == 0) {
        if (p.a.kh == 1 && p.a.kw == 1 && p.a.pad == 0 && p.a.Hm == p.a.Hs && p.a.Wm == p.a.Ws)
          gm = GM_GEMM;
        else if (!strided && T <= 32)
          gm = GM_TAP;
      }
      if (gm && g_whl && !cout_tot && !cin_tot) {
        p.w = reinterpret_cast<const bf16_t*>(g_whl);
        p.w_gstride = g_whl_gstride;
        p.w_hl = 1;
      }
      switch (v % 3) {
        case 0: launch_nn32_t<64, 64>(p, G, T, strided, stream, wide, wg, gm); break;
        case 1: launch_nn32_t<128, 128>(p, G, T, strided, stream, wide, 1, gm); break;
        default: launch_nn32_t<128, 64>(p, G, T, strided, stream, wide, wg, gm); break;
      }
      return (int)hipGetLastError();
    }
    switch (v % 3) {
      case 0: launch_nn_t<64, 64>(p, G, T, kind, strided, stream); break;
      case 1: launch_nn_t<128, 128>(p, G, T, kind, strided, stream); break;
      default: launch_nn_t<128, 64>(p, G, T, kind, strided, stream); break;
    }
    return (int)hipGetLastError();
  }
  if (g_bb_nslab) *g_bb_nslab = 0;       // fallback path: no BN statistics
  dim3 tg(((Cout + 31) / 32) * ((Cin + 31) / 32), T, G);
  if (f32)
    transpose_w_kernel<float><<<tg, 256, 0, stream>>>(reinterpret_cast<const float*>(w),
                                                      w_gstride, reinterpret_cast<float*>(wt),
                                                      Cout, T, Cin);
  else
    transpose_w_kernel<bf16_t><<<tg, 256, 0, stream>>>(reinterpret_cast<const bf16_t*>(w),
                                                       w_gstride, reinterpret_cast<bf16_t*>(wt),
                                                       Cout, T, Cin);
  p.a = make_geom(dy, B, ctot_dy, Cout, Ho, Wo, H, W, kh, kw, st, pad, es);
  if (p.a.bytes) p.a.bytes -= shift;
  p.dgrad = 1;
  p.w = reinterpret_cast<const bf16_t*>(wt);
  p.w_gstride = (int64_t)Cout * T * Cin;
  p.M = B * H * W;
  return f32 ? run_nt32(p, G, stream) : run_nt(p, G, stream);
}

CER_API int cer_conv_dgrad(const bf16_t* dy, int B, int Ho, int Wo, int Cout, int G,
                           const bf16_t* w, int64_t w_gstride, bf16_t* wt, int Cin, int kh,
                           int kw, int st, int pad, bf16_t* dx, int H, int W,
                           const bf16_t* addend, hipStream_t stream) {
  return conv_dgrad_impl(dy, B, Ho, Wo, Cout, G, w, w_gstride, wt, Cin, kh, kw, st, pad, dx, H, W,
                         addend, false, stream);
}

CER_API int cer_conv_dgrad_f32(const float* dy, int B, int Ho, int Wo, int Cout, int G,
                               const float* w, int64_t w_gstride, float* wt, int Cin, int kh,
                               int kw, int st, int pad, float* dx, int H, int W,
                               const float* addend, hipStream_t stream) {
  return conv_dgrad_impl(dy, B, Ho, Wo, Cout, G, w, w_gstride, wt, Cin, kh, kw, st, pad, dx, H, W,
                         addend, true, stream);
}

static int wg_variant(int N, int K, int G, bool fast) {
  int v = choose(2, 0, N, K, G, fast);
  if (v >= 12) v -= 12;                             // same tile as its wide twin
  return fast ? v : v % 3;
}

static int wg_splits(int Mred, int N, int K, int G, int v) {
  int bm, bn;
  tile_dims(v, bm, bn);
  const long tiles = ntiles(N, K, bm, bn) * G;
  long want = (1024 + tiles - 1) / tiles;          // aim for ~1024 blocks
  long maxs = (Mred + 511) / 512;                  // >= 512 rows per split
  long s = want < maxs ? want : maxs;
  return (int)(s < 1 ? 1 : s);
}

template <int BM, int BN>
static void launch_wg_t(WGParams p, int G, int kind, bool fast, int splits, hipStream_t stream) {
  p.m_per_split = ((p.Mred + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
  p.splits = splits;
  dim3 grid((unsigned)(ntiles(p.N, p.K, BM, BN) * splits * G));
  if (kind == 1) {
    if (p.m_per_split / BK >= 3)
      pipe_wg<BM, BN, 3><<<grid, NTHREADS, 0, stream>>>(p);
    else
      pipe_wg<BM, BN, 2><<<grid, NTHREADS, 0, stream>>>(p);
  } else if (fast) {
    igemm_wgrad<BM, BN, GM_FWD><<<grid, NTHREADS, 0, stream>>>(p);
  } else {
    igemm_wgrad<BM, BN, GM_SLOW><<<grid, NTHREADS, 0, stream>>>(p);
  }
}

static bool wg_fast(int Cin, int Cout, const WGParams& p) {
  return (Cin % 8 == 0) && (Cout % 8 == 0) && p.x.bytes != 0 &&
         (uint64_t)p.Mred * p.ldy * 2 < (1ull << 31);
}

// dw must be zeroed by the caller when more than one split is used (splits > 1)
CER_API int cer_conv_wgrad(const bf16_t* x, int B, int H, int W, int Cin, int G,
                           const bf16_t* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                           int pad, float* dw, int64_t dw_gstride, int splits,
                           hipStream_t stream) {
  WGParams p;
  p.x = make_geom(x, B, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad);
  p.dy = dy;
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  const bool fast = wg_fast(Cin, Cout, p);
  const int v = wg_variant(p.N, p.K, G, fast);
  const int kind = v / 3;
  switch (v % 3) {
    case 0: launch_wg_t<64, 64>(p, G, kind, fast, splits, stream); break;
    case 1: launch_wg_t<128, 128>(p, G, kind, fast, splits, stream); break;
    default: launch_wg_t<128, 64>(p, G, kind, fast, splits, stream); break;
  }
  return (int)hipGetLastError();
}

// ---- fp32 weight gradients (register-staged 3-pass kernels) ----------------
template <int BM, int BN>
static void launch_wg32_t(WGParams p, int G, bool fast, int splits, hipStream_t stream,
                          bool wide = false) {
  p.m_per_split = ((p.Mred + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
  p.splits = splits;
  dim3 grid((unsigned)(ntiles(p.N, p.K, BM, BN) * splits * G));
  if (wide)   // 32x32x16-MFMA twins
    if (fast && p.gemm == 1)
      igemm_wgrad32<BM, BN, GM_GEMM, true><<<grid, NTHREADS, 0, stream>>>(p);
    else if (fast && p.gemm == 2)
      igemm_wgrad32<BM, BN, GM_TAP, true><<<grid, NTHREADS, 0, stream>>>(p);
    else if (fast)
      igemm_wgrad32<BM, BN, GM_FWD, true><<<grid, NTHREADS, 0, stream>>>(p);
    else
      igemm_wgrad32<BM, BN, GM_SLOW, true><<<grid, NTHREADS, 0, stream>>>(p);
  else if (fast && p.gemm == 1)
    igemm_wgrad32<BM, BN, GM_GEMM><<<grid, NTHREADS, 0, stream>>>(p);
  else if (fast && p.gemm == 2)
    igemm_wgrad32<BM, BN, GM_TAP><<<grid, NTHREADS, 0, stream>>>(p);
  else if (fast)
    igemm_wgrad32<BM, BN, GM_FWD><<<grid, NTHREADS, 0, stream>>>(p);
  else
    igemm_wgrad32<BM, BN, GM_SLOW><<<grid, NTHREADS, 0, stream>>>(p);
}

// the weight gradient of a 1x1 / stride-1 / pad-0 conv is a plain GEMM over
// rows shared by x and dy (1: GM_GEMM body); a stride-1 k x k conv with a
// same-size output reads x at the dy row's pixel shifted by the tap (2:
// GM_TAP body); others keep the im2col body (0)
static int wg_gemm(const WGParams& p) {
  const GatherGeom& g = p.x;
  if (!uk_on() || g.st != 1 || g.st_w != 1 || g.Hm != g.Hs || g.Wm != g.Ws) return 0;
  if (g.kh == 1 && g.kw == 1) return g.pad == 0 && g.pad_w == 0 ? 1 : 0;
  return 2;
}

static bool wg_fast32(int Cin, int Cout, const WGParams& p) {
  return (Cin % 8 == 0) && (Cout % 8 == 0) && p.x.bytes != 0 &&
         (uint64_t)p.Mred * p.ldy * 4 < (1ull << 31);
}

static void run_wg32(WGParams p, int G, int splits, bool fast, hipStream_t stream) {
  const int vv = choose(2, 0, p.N, p.K, G, false);
  const bool wide = vv >= 12;
  switch (vv % 3) {
    case 0: launch_wg32_t<64, 64>(p, G, fast, splits, stream, wide); break;
    case 1: launch_wg32_t<128, 128>(p, G, fast, splits, stream, wide); break;
    default: launch_wg32_t<128, 64>(p, G, fast, splits, stream, wide); break;
  }
}

CER_API int cer_conv_wgrad_f32(const float* x, int B, int H, int W, int Cin, int G,
                               const float* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                               int pad, float* dw, int64_t dw_gstride, int splits,
                               hipStream_t stream) {
  WGParams p;
  p.x = make_geom(x, B, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad, 4);
  p.dy = reinterpret_cast<const bf16_t*>(dy);
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  p.x_hl = g_hl_x;
  p.dy_hl = g_hl_dy;
  if ((p.x_hl || p.dy_hl) && !wg_fast32(Cin, Cout, p)) return (int)hipErrorInvalidValue;
  p.gemm = wg_gemm(p);
  run_wg32(p, G, splits, wg_fast32(Cin, Cout, p), stream);
  return (int)hipGetLastError();
}

// ---- grouped convolutions (ResNeXt cardinality) ----------------------------
// A conv with ``groups`` channel groups inside each of the G packed configs
// is, per config g, a packed conv of ``groups`` sub-configs: input channels
// [g*Cin + j*Cin/groups, ...), output channels [g*Cout + j*Cout/groups, ...),
// weights (per config [Cout][kh][kw][Cin/groups]) of group j at
// w + g*w_gstride + j*(Cout/groups)*kh*kw*(Cin/groups).  The entry points
// below launch the ordinary kernels once per config on shifted pointers with
// the full tensors' channel pitch (G launches; ResNeXt packs are small).
// Strided 1x1 grouped convs are refused (ResNeXt's grouped convs are 3x3).
static bool grouped_ok(int Cin, int Cout, int groups) {
  return groups >= 1 && Cin % groups == 0 && Cout % groups == 0;
}

template <typename E>
static int grouped_fwd(const E* x, int B, int H, int W, int Cin, int G, int groups, const E* w,
                       int64_t w_gstride, int Cout, int kh, int kw, int st, int pad, E* y, int Ho,
                       int Wo, hipStream_t stream) {
  if (!grouped_ok(Cin, Cout, groups)) return (int)hipErrorInvalidValue;
  const int ci = Cin / groups, co = Cout / groups;
  const int64_t wsub = (int64_t)co * kh * kw * ci;
  const bool f32 = sizeof(E) == 4;
  for (int g = 0; g < G; ++g) {
    const int rc = conv_fwd_impl(x + (int64_t)g * Cin, B, H, W, ci, groups, w + g * w_gstride, wsub,
                                 co, kh, kw, st, pad, y + (int64_t)g * Cout, Ho, Wo, nullptr, 0, 0,
                                 nullptr, nullptr, f32, stream, G * Cin, G * Cout,
                                 (uint32_t)((size_t)g * Cin * sizeof(E)));
    if (rc) return rc;
  }
  return (int)hipGetLastError();
}

template <typename E>
static int grouped_dgrad(const E* dy, int B, int Ho, int Wo, int Cout, int G, int groups,
                         const E* w, int64_t w_gstride, E* wt, int Cin, int kh, int kw, int st,
                         int pad, E* dx, int H, int W, hipStream_t stream) {
  if (!grouped_ok(Cin, Cout, groups) || (kh == 1 && kw == 1 && pad == 0 && st > 1))
    return (int)hipErrorInvalidValue;
  const int ci = Cin / groups, co = Cout / groups;
  const int64_t wsub = (int64_t)co * kh * kw * ci;
  const bool f32 = sizeof(E) == 4;
  for (int g = 0; g < G; ++g) {
    const int rc = conv_dgrad_impl(dy + (int64_t)g * Cout, B, Ho, Wo, co, groups,
                                   w + g * w_gstride, wsub, wt, ci, kh, kw, st, pad,
                                   dx + (int64_t)g * Cin, H, W, nullptr, f32, stream, G * Cout,
                                   G * Cin, (uint32_t)((size_t)g * Cout * sizeof(E)));
    if (rc) return rc;
  }
  return (int)hipGetLastError();
}

// WGParams of config g of a grouped conv (sub-configs = its groups)
template <typename E>
static WGParams grouped_wg_params(const E* x, int B, int H, int W, int Cin, int G, int groups,
                                  const E* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                                  int pad, float* dw, int64_t dw_gstride, int g) {
  const int ci = Cin / groups, co = Cout / groups;
  WGParams p;
  p.x = make_geom(x + (int64_t)g * Cin, B, G * Cin, ci, H, W, Ho, Wo, kh, kw, st, pad,
                  (int)sizeof(E));
  if (p.x.bytes) p.x.bytes -= (uint32_t)((size_t)g * Cin * sizeof(E));
  p.dy = reinterpret_cast<const bf16_t*>(dy + (int64_t)g * Cout);
  p.ldy = G * Cout;
  p.dw = dw + g * dw_gstride;
  p.dw_gstride = (int64_t)co * kh * kw * ci;
  p.Mred = B * Ho * Wo;
  p.N = co;
  p.K = kh * kw * ci;
  return p;
}

CER_API int cer_conv_grouped_fwd(const bf16_t* x, int B, int H, int W, int Cin, int G,
                                 int groups, const bf16_t* w, int64_t w_gstride, int Cout,
                                 int kh, int kw, int st, int pad, bf16_t* y, int Ho, int Wo,
                                 hipStream_t stream) {
  return grouped_fwd(x, B, H, W, Cin, G, groups, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo,
                     stream);
}

CER_API int cer_conv_grouped_fwd_f32(const float* x, int B, int H, int W, int Cin, int G,
                                     int groups, const float* w, int64_t w_gstride, int Cout,
                                     int kh, int kw, int st, int pad, float* y, int Ho, int Wo,
                                     hipStream_t stream) {
  return grouped_fwd(x, B, H, W, Cin, G, groups, w, w_gstride, Cout, kh, kw, st, pad, y, Ho, Wo,
                     stream);
}

// wt: scratch of G * Cout * kh * kw * Cin / groups elements (unaligned fallback)
CER_API int cer_conv_grouped_dgrad(const bf16_t* dy, int B, int Ho, int Wo, int Cout, int G,
                                   int groups, const bf16_t* w, int64_t w_gstride, bf16_t* wt,
                                   int Cin, int kh, int kw, int st, int pad, bf16_t* dx, int H,
                                   int W, hipStream_t stream) {
  return grouped_dgrad(dy, B, Ho, Wo, Cout, G, groups, w, w_gstride, wt, Cin, kh, kw, st, pad, dx,
                       H, W, stream);
}

CER_API int cer_conv_grouped_dgrad_f32(const float* dy, int B, int Ho, int Wo, int Cout, int G,
                                       int groups, const float* w, int64_t w_gstride, float* wt,
                                       int Cin, int kh, int kw, int st, int pad, float* dx, int H,
                                       int W, hipStream_t stream) {
  return grouped_dgrad(dy, B, Ho, Wo, Cout, G, groups, w, w_gstride, wt, Cin, kh, kw, st, pad, dx,
                       H, W, stream);
}

// dw must be zeroed by the caller when more than one split is used
CER_API int cer_conv_grouped_wgrad(const bf16_t* x, int B, int H, int W, int Cin, int G,
                                   int groups, const bf16_t* dy, int Ho, int Wo, int Cout, int kh,
                                   int kw, int st, int pad, float* dw, int64_t dw_gstride,
                                   int splits, hipStream_t stream) {
  if (!grouped_ok(Cin, Cout, groups)) return (int)hipErrorInvalidValue;
  for (int g = 0; g < G; ++g) {
    WGParams p = grouped_wg_params(x, B, H, W, Cin, G, groups, dy, Ho, Wo, Cout, kh, kw, st, pad,
                                   dw, dw_gstride, g);
    const bool fast = wg_fast(Cin / groups, Cout / groups, p);
    const int v = wg_variant(p.N, p.K, groups, fast);
    switch (v % 3) {
      case 0: launch_wg_t<64, 64>(p, groups, v / 3, fast, splits, stream); break;
      case 1: launch_wg_t<128, 128>(p, groups, v / 3, fast, splits, stream); break;
      default: launch_wg_t<128, 64>(p, groups, v / 3, fast, splits, stream); break;
    }
  }
  return (int)hipGetLastError();
}

CER_API int cer_conv_grouped_wgrad_f32(const float* x, int B, int H, int W, int Cin, int G,
                                       int groups, const float* dy, int Ho, int Wo, int Cout,
                                       int kh, int kw, int st, int pad, float* dw,
                                       int64_t dw_gstride, int splits, hipStream_t stream) {
  if (!grouped_ok(Cin, Cout, groups) || g_hl_x || g_hl_dy) return (int)hipErrorInvalidValue;
  for (int g = 0; g < G; ++g) {
    WGParams p = grouped_wg_params(x, B, H, W, Cin, G, groups, dy, Ho, Wo, Cout, kh, kw, st, pad,
                                   dw, dw_gstride, g);
    run_wg32(p, groups, splits, wg_fast32(Cin / groups, Cout / groups, p), stream);
  }
  return (int)hipGetLastError();
}

// ---- batched (deferred) weight gradients ----------------------------------
// one queue per dtype; a flush launches both
static WGParams g_wgq[4096];
static int g_wgq_G[4096];
static int g_wgq_n = 0;
static WGParams g_wgq32[4096];
static int g_wgq32_G[4096];
static int g_wgq32_n = 0;
static int g_wgb_rows = 0;

// rows per split of the next queued wgrads (0: CER_WGB_ROWS / 1024); the
// runtime sets it per packed step (more rows for wider packs, A/B in profiles/)
CER_API void cer_wgrad_batch_set_rows(int rows) {
  g_wgb_rows = rows > 0 ? (rows < BK ? BK : rows / BK * BK) : 0;
}

static int wgb_rows() {
  if (!g_wgb_rows) {
    const char* e = getenv("CER_WGB_ROWS");
    g_wgb_rows = e ? atoi(e) : 1024;
    if (g_wgb_rows < BK) g_wgb_rows = BK;
    g_wgb_rows = g_wgb_rows / BK * BK;
  }
  return g_wgb_rows;
}

// Queue one layer's wgrad for cer_wgrad_batch_flush.  Returns the split count
// the batch will use (> 1: dw must be zero before the flush) or 0 when the
// layer is not eligible (unaligned channels / >2 GB operands / queue full):
// the caller then launches it on its own (cer_conv_wgrad).
CER_API int cer_wgrad_batch_add(const bf16_t* x, int B, int H, int W, int Cin, int G,
                                const bf16_t* dy, int Ho, int Wo, int Cout, int kh, int kw,
                                int st, int pad, float* dw, int64_t dw_gstride) {
  if (g_wgq_n >= 4096) return 0;
  WGParams p;
  p.x = make_geom(x, B, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad);
  p.dy = dy;
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  if (!wg_fast(Cin, Cout, p)) return 0;
  const int rows = wgb_rows();
  p.m_per_split = p.Mred < rows ? (p.Mred + BK - 1) / BK * BK : rows;
  p.splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
  g_wgq_G[g_wgq_n] = G;     // folded into the block count at flush time
  g_wgq[g_wgq_n++] = p;
  return p.splits;
}

CER_API int cer_wgrad_batch_add_f32(const float* x, int B, int H, int W, int Cin, int G,
                                    const float* dy, int Ho, int Wo, int Cout, int kh, int kw,
                                    int st, int pad, float* dw, int64_t dw_gstride) {
  if (g_wgq32_n >= 4096) return 0;
  WGParams p;
  p.x = make_geom(x, B, G * Cin, Cin, H, W, Ho, Wo, kh, kw, st, pad, 4);
  p.dy = reinterpret_cast<const bf16_t*>(dy);
  p.ldy = G * Cout;
  p.dw = dw;
  p.dw_gstride = dw_gstride;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kw * Cin;
  p.x_hl = g_hl_x;
  p.dy_hl = g_hl_dy;
  if (!wg_fast32(Cin, Cout, p)) return 0;     // HL operands: the direct launch refuses
  p.gemm = wg_gemm(p);
  const int rows = wgb_rows();
  p.m_per_split = p.Mred < rows ? (p.Mred + BK - 1) / BK * BK : rows;
  p.splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
  g_wgq32_G[g_wgq32_n] = G;
  g_wgq32[g_wgq32_n++] = p;
  return p.splits;
}

// queue a grouped conv's wgrad: one batch entry per config (sub-configs =
// its groups); returns the split count or 0 (not eligible: launch directly)
template <typename E>
static int grouped_batch_add(const E* x, int B, int H, int W, int Cin, int G, int groups,
                             const E* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                             int pad, float* dw, int64_t dw_gstride) {
  const bool f32 = sizeof(E) == 4;
  int& n = f32 ? g_wgq32_n : g_wgq_n;
  if (!grouped_ok(Cin, Cout, groups) || n + G > 4096 || g_hl_x || g_hl_dy) return 0;
  int splits = 0;
  for (int g = 0; g < G; ++g) {
    WGParams p = grouped_wg_params(x, B, H, W, Cin, G, groups, dy, Ho, Wo, Cout, kh, kw, st, pad,
                                   dw, dw_gstride, g);
    if (!(f32 ? wg_fast32(Cin / groups, Cout / groups, p) : wg_fast(Cin / groups, Cout / groups, p)))
      return g == 0 ? 0 : -1;               // configs differ only by offsets: all or none
    const int rows = wgb_rows();
    p.m_per_split = p.Mred < rows ? (p.Mred + BK - 1) / BK * BK : rows;
    p.splits = (p.Mred + p.m_per_split - 1) / p.m_per_split;
    splits = p.splits;
    if (f32) {
      g_wgq32_G[g_wgq32_n] = groups;
      g_wgq32[g_wgq32_n++] = p;
    } else {
      g_wgq_G[g_wgq_n] = groups;
      g_wgq[g_wgq_n++] = p;
    }
  }
  return splits;
}

CER_API int cer_wgrad_batch_add_grouped(const bf16_t* x, int B, int H, int W, int Cin, int G,
                                        int groups, const bf16_t* dy, int Ho, int Wo, int Cout,
                                        int kh, int kw, int st, int pad, float* dw,
                                        int64_t dw_gstride) {
  return grouped_batch_add(x, B, H, W, Cin, G, groups, dy, Ho, Wo, Cout, kh, kw, st, pad, dw,
                           dw_gstride);
}

CER_API int cer_wgrad_batch_add_grouped_f32(const float* x, int B, int H, int W, int Cin, int G,
                                            int groups, const float* dy, int Ho, int Wo, int Cout,
                                            int kh, int kw, int st, int pad, float* dw,
                                            int64_t dw_gstride) {
  return grouped_batch_add(x, B, H, W, Cin, G, groups, dy, Ho, Wo, Cout, kh, kw, st, pad, dw,
                           dw_gstride);
}

// grid cap of the next fp32 batch flushes (0 = one block per work item)
static int g_wgb_grid = 0;
CER_API void cer_wgrad_batch_set_grid(int blocks) { g_wgb_grid = blocks > 0 ? blocks : 0; }

template <int BM, int BN, bool WIDE = false>
static void wgb32_launch_sel(hipStream_t stream, const int* idx, int n) {
  for (int b0 = 0; b0 < n; b0 += WGB_MAX) {
    WGBatch bt;
    bt.n = n - b0 < WGB_MAX ? n - b0 : WGB_MAX;
    int tot = 0;
    for (int i = 0; i < bt.n; ++i) {
      const int k = idx[b0 + i];
      bt.p[i] = g_wgq32[k];
      bt.start[i] = tot;
      tot += (int)(ntiles(bt.p[i].N, bt.p[i].K, BM, BN) * bt.p[i].splits * g_wgq32_G[k]);
    }
    bt.start[bt.n] = tot;
    const int grid = g_wgb_grid > 0 && g_wgb_grid < tot ? g_wgb_grid : tot;
    if (tot <= 0) continue;
    wgrad_batch32<BM, BN, WIDE><<<grid, NTHREADS, 0, stream>>>(bt);
  }
}

// Items whose output-channel count N (tile rows) is at most 64 would leave
// half of every 128x128 tile empty (VGG block 1, ResNet stage 2): they go to
// their own launch with 64x128 tiles (CER_WGB_NARROW=2, default: all their
// rows, twice a 64x64 tile's columns; round 6: +0.4 % at 8 configs, -0.8 %
// one-config step time vs 64x64), 1: 64x64 tiles, 0: one launch.
static int g_wgb_narrow = -1;
static bool wgb_narrow() {
  if (g_wgb_narrow < 0) {
    const char* e = getenv("CER_WGB_NARROW");
    g_wgb_narrow = e ? atoi(e) : 2;
  }
  return g_wgb_narrow > 0;
}
// 0 = no split, 1 = 64x64 tiles, 2 = 64x128 tiles for the narrow items
CER_API void cer_wgrad_batch_set_narrow(int on) { g_wgb_narrow = on > 0 ? on : 0; }

template <int BM, int BN>
static void wgb32_launch_one(hipStream_t stream, bool wide, const int* idx, int n) {
  if (n <= 0) return;
  if (wide)
    wgb32_launch_sel<BM, BN, true>(stream, idx, n);
  else
    wgb32_launch_sel<BM, BN>(stream, idx, n);
}

template <int BM, int BN>
static int wgb32_launch(hipStream_t stream, bool wide = false) {
  // 128x128 batches: items with N <= 64 output channels take 64x64 tiles;
  // the rest stay on the batch's tile.  (Routing K <= 64 items to 128x64
  // tiles as well measured neutral-to-slower on ResNet-50: profiles/r5_final.md)
  static int idx[4096], narn[4096];
  int n = 0, nn = 0;
  const bool split = BM == 128 && BN == 128 && wgb_narrow();
  for (int k = 0; k < g_wgq32_n; ++k) {
    if (split && g_wgq32[k].N <= 64)
      narn[nn++] = k;
    else
      idx[n++] = k;
  }
  if (g_wgb_narrow == 2)             // 64x128: all <= 64 rows, twice the columns
    wgb32_launch_one<64, 128>(stream, wide, narn, nn);
  else
    wgb32_launch_one<64, 64>(stream, wide, narn, nn);
  wgb32_launch_one<BM, BN>(stream, wide, idx, n);
  return (int)hipGetLastError();
}

template <int BM, int BN, int KIND>
static int wgb_launch(hipStream_t stream) {
  for (int b0 = 0; b0 < g_wgq_n; b0 += WGB_MAX) {
    WGBatch bt;
    bt.n = g_wgq_n - b0 < WGB_MAX ? g_wgq_n - b0 : WGB_MAX;
    int tot = 0;
    for (int i = 0; i < bt.n; ++i) {
      bt.p[i] = g_wgq[b0 + i];
      bt.start[i] = tot;
      tot += (int)(ntiles(bt.p[i].N, bt.p[i].K, BM, BN) * bt.p[i].splits * g_wgq_G[b0 + i]);
    }
    bt.start[bt.n] = tot;
    if (tot > 0) wgrad_batch<BM, BN, KIND><<<tot, NTHREADS, 0, stream>>>(bt);
  }
  return (int)hipGetLastError();
}

// Launch every queued wgrad (WGB_MAX layers per launch) with tile variant v
// (0 reg 64x64, 1 reg 128x128, 2 reg 128x64, 3-5 the LDS-DMA ring twins) and
// clear the queue.  `discard` != 0 only clears it.
CER_API int cer_wgrad_batch_flush(int v, int discard, hipStream_t stream) {
  int rc = 0;
  if (!discard && g_wgq_n > 0) {
    switch (v >= 12 ? v % 3 : v) {
      case 1: rc = wgb_launch<128, 128, 0>(stream); break;
      case 2: rc = wgb_launch<128, 64, 0>(stream); break;
      case 3: rc = wgb_launch<64, 64, 1>(stream); break;
      case 4: rc = wgb_launch<128, 128, 1>(stream); break;
      case 5: rc = wgb_launch<128, 64, 1>(stream); break;
      default: rc = wgb_launch<64, 64, 0>(stream); break;
    }
  }
  if (!discard && g_wgq32_n > 0 && rc == 0) {
    const bool wide = v >= 12;   // fp32: 12-14 = 32x32x16-MFMA tiles
    switch (v % 3) {         // fp32: the register-staged tile of the same shape
      case 1: rc = wgb32_launch<128, 128>(stream, wide); break;
      case 2: rc = wgb32_launch<128, 64>(stream, wide); break;
      default: rc = wgb32_launch<64, 64>(stream, wide); break;
    }
  }
  g_wgq_n = 0;
  g_wgq32_n = 0;
  return rc;
}

CER_API int cer_wgrad_batch_pending() { return g_wgq_n + g_wgq32_n; }

// the split count the host should use (and whether dw needs zeroing); the
// variant is re-derived exactly as cer_conv_wgrad will (fast path assumed
// when channels are 8-aligned)
CER_API int cer_wgrad_splits(int Mred, int N, int K, int G) {
  return wg_splits(Mred, N, K, G, wg_variant(N, K, G, true));
}

// ---------------------------------------------------------------------------
// Narrow-input stem (Cin <= 4, stride 2, odd padding, even width: ResNet's
// 7x7/2 and MobileNetV2's 3x3/2 first layers).  With 3 channels an im2col
// row has no aligned 16-B chunks, so the generic path gathers element by
// element.  Instead the image is repacked per config as [B][H][W][4]
// (channel 3 = 0) and read as PIXEL PAIRS: [B][H][W/2][8].  The stride-2
// conv over W becomes a stride-1 conv over pairs with kw' = kw/2 + 1 taps:
// original tap s = 2*sp + px - 1 (px = pixel within the pair), so every
// 16-B chunk is one (row tap, pair tap) and the aligned MFMA path applies.
// Weights are re-laid [N][kh][kw'][8] per step (zeros on padded taps /
// channels); the wgrad runs on the same geometry and is folded back.
// STEM_PAD8 (Cin < 8, stride 1: VGG's 3x3/1 block1_conv1): no pixel pairs;
// the image is repacked per config as [B][H][W][8] (channels Cin..7 = 0) and
// the weights as [N][kh][kw][8], so every tap is one aligned 8-channel chunk
// (K = kh*kw*8) at the price of 8/Cin x the MFMA work on a tiny layer.
// ---------------------------------------------------------------------------
enum { STEM_NONE = 0, STEM_PAD8 = 1, STEM_PAIR = 2 };
// element i of the input repack: (pixel, config) -> [G][P][CP], channels >= C zero
template <typename E>
__device__ __forceinline__ void stem_repack_one(const E* __restrict__ x, E* __restrict__ x4,
                                                int64_t i, int64_t P, int G, int C, int CP) {
  if (i >= P * G) return;
  const int64_t p = i / G;
  const int g = (int)(i - p * G);
  const E* src = x + p * G * C + (int64_t)g * C;
  E* dst = x4 + ((int64_t)g * P + p) * CP;
  for (int c = 0; c < CP; ++c) dst[c] = c < C ? src[c] : (E)0;
}

// element i of the weight re-layout [G][N][kh][kwp][8]
template <typename E>
__device__ __forceinline__ void stem_pack_w_one(const E* __restrict__ w, int64_t w_gstride,
                                                E* __restrict__ wp, int64_t i, int N, int kh,
                                                int kw, int C, int kwp, int G, int pad8) {
  const int64_t per = (int64_t)N * kh * kwp * 8;
  if (i >= per * G) return;
  const int g = (int)(i / per);
  int64_t t = i - g * per;
  const int q = (int)(t % 8);
  t /= 8;
  const int sp = (int)(t % kwp);
  t /= kwp;
  const int r = (int)(t % kh);
  const int n = (int)(t / kh);
  // pad8 (STEM_PAD8): tap sp, channel q; else pixel pairs
  const int px = pad8 ? 0 : q >> 2, c = pad8 ? q : q & 3, s = pad8 ? sp : 2 * sp + px - 1;
  E v = 0;
  if (s >= 0 && s < kw && c < C) v = w[g * w_gstride + (((int64_t)n * kh + r) * kw + s) * C + c];
  wp[i] = v;
}

// The stem's per-step preparation in ONE launch: blocks [0, nbx) repack the
// input, the next nbw blocks re-lay the weights, the rest zero the stem
// wgrad's split-K scratch of this step (cer_stem_set_wgrad_scratch; nzero
// floats, a multiple of 4) -- three small dependent launches became one
template <typename E>
__global__ __launch_bounds__(256) void stem_prep_kernel(
    const E* __restrict__ x, E* __restrict__ x4, int64_t P, int G, int C, int CP, int nbx,
    const E* __restrict__ w, int64_t w_gstride, E* __restrict__ wp, int N, int kh, int kw,
    int kwp, int pad8, int nbw, float* __restrict__ zero, int64_t nzero) {
  int b = blockIdx.x;
  if (b < nbx) {
    stem_repack_one(x, x4, (int64_t)b * 256 + threadIdx.x, P, G, C, CP);
    return;
  }
  b -= nbx;
  if (b < nbw) {
    stem_pack_w_one(w, w_gstride, wp, (int64_t)b * 256 + threadIdx.x, N, kh, kw, C, kwp, G, pad8);
    return;
  }
  b -= nbw;
  const int64_t k = ((int64_t)b * 256 + threadIdx.x) * 4;
  if (k < nzero) *reinterpret_cast<float4*>(zero + k) = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void stem_fold_grad_kernel(const float* __restrict__ dwp,
                                                             float* __restrict__ dw,
                                                             int64_t dw_gstride, int N, int kh,
                                                             int kw, int C, int kwp, int G,
                                                             int pad8) {
  const int64_t per = (int64_t)N * kh * kw * C;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= per * G) return;
  const int g = (int)(i / per);
  int64_t t = i - g * per;
  const int c = (int)(t % C);
  t /= C;
  const int s = (int)(t % kw);
  t /= kw;
  const int r = (int)(t % kh);
  const int n = (int)(t / kh);
  if (pad8) {                                          // STEM_PAD8
    dw[g * dw_gstride + (((int64_t)n * kh + r) * kw + s) * C + c] =
        dwp[((((int64_t)g * N + n) * kh + r) * kw + s) * 8 + c];
    return;
  }
  const int sp = (s + 1) >> 1, px = (s + 1) & 1;
  dw[g * dw_gstride + (((int64_t)n * kh + r) * kw + s) * C + c] =
      dwp[((((int64_t)g * N + n) * kh + r) * kwp + sp) * 8 + px * 4 + c];
}

// the stem geometry of a first layer (STEM_*): pixel pairs for Cin <= 4,
// stride 2, odd padding, even width; channel padding to 8 for Cin < 8 at
// stride 1; none otherwise
// (CER_STEM_PAD8=0: stride-1 narrow first layers take the generic gather, A/B)
static const int g_stem_pad8 = [] {
  const char* e = getenv("CER_STEM_PAD8");
  return e ? atoi(e) : 1;
}();
CER_API int cer_stem_ok(int Cin, int W, int kw, int st, int pad) {
  if (Cin <= 4 && st == 2 && (pad & 1) && (W % 2) == 0 && kw >= 2) return STEM_PAIR;
  if (Cin < 8 && st == 1 && g_stem_pad8) return STEM_PAD8;
  return STEM_NONE;
}

static int stem_kwp(int kw, int mode) { return mode == STEM_PAD8 ? kw : kw / 2 + 1; }
// channels per pixel of the repacked input
static int stem_cp(int mode) { return mode == STEM_PAD8 ? 8 : 4; }

// scratch sizes (elements): x4 = G*B*H*W*cer_stem_cp, wpk = G*Cout*kh*kwp*8
CER_API int64_t cer_stem_wpk_elems(int G, int Cout, int kh, int kw, int mode) {
  return (int64_t)G * Cout * kh * stem_kwp(kw, mode) * 8;
}
CER_API int cer_stem_cp(int mode) { return stem_cp(mode); }

static GatherGeom stem_geom(const void* x4, int B, int H, int W, int Ho, int Wo, int kh,
                            int kw, int pad, int mode) {
  if (mode == STEM_PAD8) {
    GatherGeom g = make_geom(x4, B, 8, 8, H, W, Ho, Wo, kh, kw, 1, pad);
    g.cfg_off = (int64_t)B * H * W * 8;
    return g;
  }
  const int kwp = stem_kwp(kw, mode);
  GatherGeom g = make_geom(x4, B, 8, 8, H, W / 2, Ho, Wo, kh, kwp, 2, pad);
  g.st_w = 1;
  g.pad_w = (pad + 1) / 2;
  g.cfg_off = (int64_t)B * H * (W / 2) * 8;
  return g;
}

// the NEXT stem forward also zeroes this step's stem-wgrad scratch (fp32,
// cer_stem_wpk_elems floats), and the NEXT stem wgrad takes its scratch as
// already zeroed (cer_stem_set_wgrad_zeroed): ops._hip stem paths
static float* g_stem_zero = nullptr;
static int g_stem_zeroed = 0;
CER_API void cer_stem_set_wgrad_scratch(float* dwp) { g_stem_zero = dwp; }
CER_API void cer_stem_set_wgrad_zeroed(int on) { g_stem_zeroed = on ? 1 : 0; }

static int stem_fwd_impl(const void* x, int B, int H, int W, int Cin, int G, const void* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         void* x4, void* wpk, void* y, int Ho, int Wo, float* part,
                         int* nslab, const void* bias, int64_t bias_gstride, int act, bool f32,
                         hipStream_t stream) {
  const int mode = cer_stem_ok(Cin, W, kw, st, pad);
  float* zero = g_stem_zero;
  g_stem_zero = nullptr;
  if (mode == STEM_NONE) return (int)hipErrorInvalidValue;
  const int64_t P = (int64_t)B * H * W;
  const int kwp = stem_kwp(kw, mode), cp = stem_cp(mode);
  const int64_t nw = (int64_t)G * Cout * kh * kwp * 8;       // (also the scratch's floats)
  const int nbx = (int)cer_blocks(P * G, 256), nbw = (int)cer_blocks(nw, 256);
  const int nbz = zero ? (int)cer_blocks(nw / 4, 256) : 0;   // nw % 8 == 0
  const dim3 grid(nbx + nbw + nbz);
  if (f32)
    stem_prep_kernel<float><<<grid, 256, 0, stream>>>(
        reinterpret_cast<const float*>(x), reinterpret_cast<float*>(x4), P, G, Cin, cp, nbx,
        reinterpret_cast<const float*>(w), w_gstride, reinterpret_cast<float*>(wpk), Cout, kh, kw,
        kwp, mode == STEM_PAD8, nbw, zero, zero ? nw : 0);
  else
    stem_prep_kernel<bf16_t><<<grid, 256, 0, stream>>>(
        reinterpret_cast<const bf16_t*>(x), reinterpret_cast<bf16_t*>(x4), P, G, Cin, cp, nbx,
        reinterpret_cast<const bf16_t*>(w), w_gstride, reinterpret_cast<bf16_t*>(wpk), Cout, kh,
        kw, kwp, mode == STEM_PAD8, nbw, zero, zero ? nw : 0);
  NTParams p;
  p.a = stem_geom(x4, B, H, W, Ho, Wo, kh, kw, pad, mode);
  // the whole [G][B][H][W][cp] buffer is the buffer-load range
  const uint64_t bytes = (uint64_t)G * P * cp * (f32 ? 4 : 2);
  p.a.bytes = bytes < (1ull << 31) ? (uint32_t)bytes : 0u;
  p.dgrad = 0;
  p.w = reinterpret_cast<const bf16_t*>(wpk);
  p.w_gstride = (int64_t)Cout * kh * kwp * 8;
  p.out = reinterpret_cast<bf16_t*>(y);
  p.ldc = G * Cout;
  p.M = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kwp * 8;
  p.bias = reinterpret_cast<const bf16_t*>(bias);
  p.bias_gstride = bias ? bias_gstride : 0;
  p.act = act;
  p.o_st = 1;
  p.o_H = Ho;
  p.o_W = Wo;
  p.stats = part;
  return f32 ? run_nt32(p, G, stream, nslab) : run_nt(p, G, stream, nslab);
}

// repack + weight re-layout + forward conv (+ BN partials when part != null;
// + bias and activation in the epilogue when bias != null / act != 0)
CER_API int cer_stem_fwd(const bf16_t* x, int B, int H, int W, int Cin, int G, const bf16_t* w,
                         int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                         bf16_t* x4, bf16_t* wpk, bf16_t* y, int Ho, int Wo, float* part,
                         int* nslab, const bf16_t* bias, int64_t bias_gstride, int act,
                         hipStream_t stream) {
  return stem_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, x4, wpk, y, Ho,
                       Wo, part, nslab, bias, bias_gstride, act, false, stream);
}

// fp32 twin: x4 / wpk / y fp32 (same element counts)
CER_API int cer_stem_fwd_f32(const float* x, int B, int H, int W, int Cin, int G, const float* w,
                             int64_t w_gstride, int Cout, int kh, int kw, int st, int pad,
                             float* x4, float* wpk, float* y, int Ho, int Wo, float* part,
                             int* nslab, const float* bias, int64_t bias_gstride, int act,
                             hipStream_t stream) {
  return stem_fwd_impl(x, B, H, W, Cin, G, w, w_gstride, Cout, kh, kw, st, pad, x4, wpk, y, Ho,
                       Wo, part, nslab, bias, bias_gstride, act, true, stream);
}

// dW of the stem from the repacked input; dwp: fp32 scratch of
// cer_stem_wpk_elems floats (zeroed here when the reduction is split)
static int stem_wgrad_impl(const void* x4, int B, int H, int W, int Cin, int G, const void* dy,
                           int Ho, int Wo, int Cout, int kh, int kw, int st, int pad, float* dwp,
                           float* dw, int64_t dw_gstride, bool f32, hipStream_t stream) {
  const int mode = cer_stem_ok(Cin, W, kw, st, pad);
  if (mode == STEM_NONE) return (int)hipErrorInvalidValue;
  const int kwp = stem_kwp(kw, mode);
  WGParams p;
  p.x = stem_geom(x4, B, H, W, Ho, Wo, kh, kw, pad, mode);
  const uint64_t bytes = (uint64_t)G * B * H * W * stem_cp(mode) * (f32 ? 4 : 2);
  p.x.bytes = bytes < (1ull << 31) ? (uint32_t)bytes : 0u;
  p.dy = reinterpret_cast<const bf16_t*>(dy);
  p.ldy = G * Cout;
  p.dw = dwp;
  p.dw_gstride = (int64_t)Cout * kh * kwp * 8;
  p.Mred = B * Ho * Wo;
  p.N = Cout;
  p.K = kh * kwp * 8;
  const bool fast = f32 ? wg_fast32(8, Cout, p) : wg_fast(8, Cout, p);
  const int v = wg_variant(p.N, p.K, G, fast && !f32);
  const int splits = wg_splits(p.Mred, p.N, p.K, G, v);
  const int zeroed = g_stem_zeroed;
  g_stem_zeroed = 0;
  if (splits > 1 && !zeroed)
    cer_zero_async(dwp, sizeof(float) * (size_t)G * p.dw_gstride, stream);
  if (f32) {
    run_wg32(p, G, splits, fast, stream);
  } else {
    const int kind = v / 3;
    switch (v % 3) {
      case 0: launch_wg_t<64, 64>(p, G, kind, fast, splits, stream); break;
      case 1: launch_wg_t<128, 128>(p, G, kind, fast, splits, stream); break;
      default: launch_wg_t<128, 64>(p, G, kind, fast, splits, stream); break;
    }
  }
  const int64_t n = (int64_t)G * Cout * kh * kw * Cin;
  stem_fold_grad_kernel<<<cer_blocks(n, 256), 256, 0, stream>>>(dwp, dw, dw_gstride, Cout, kh, kw,
                                                                Cin, kwp, G, mode == STEM_PAD8);
  return (int)hipGetLastError();
}

CER_API int cer_stem_wgrad(const bf16_t* x4, int B, int H, int W, int Cin, int G,
                           const bf16_t* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                           int pad, float* dwp, float* dw, int64_t dw_gstride,
                           hipStream_t stream) {
  return stem_wgrad_impl(x4, B, H, W, Cin, G, dy, Ho, Wo, Cout, kh, kw, st, pad, dwp, dw,
                         dw_gstride, false, stream);
}

CER_API int cer_stem_wgrad_f32(const float* x4, int B, int H, int W, int Cin, int G,
                               const float* dy, int Ho, int Wo, int Cout, int kh, int kw, int st,
                               int pad, float* dwp, float* dw, int64_t dw_gstride,
                               hipStream_t stream) {
  return stem_wgrad_impl(x4, B, H, W, Cin, G, dy, Ho, Wo, Cout, kh, kw, st, pad, dwp, dw,
                         dw_gstride, true, stream);
}
