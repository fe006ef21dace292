// Pooling + bias/activation elementwise kernels on packed NHWC (SURVEY.md
// K10, K15).  All kernels move 8 channels per thread (16 B in bf16, 32 B in fp32),
// or 1 when the channel count is not a multiple of 8 (ragged widths, e.g.
// NASNet-Mobile's); every op has a bf16 and an _f32 entry point.
//
// maxpool fwd stores the argmax window offset (uint8) per output element;
// maxpool bwd is a deterministic *gather* (each input pixel sums the
// gradients of the <= ceil(k/s)^2 windows whose argmax is it) — no atomics.
#include "common.h"

constexpr int PT = 256;

template <typename T, int V>
__global__ __launch_bounds__(PT) void maxpool_fwd_kernel(const T* __restrict__ x,
                                                         T* __restrict__ y,
                                                         uint8_t* __restrict__ arg, int B, int H,
                                                         int W, int C, int Ho, int Wo, int k,
                                                         int s, int pad, int relu_bit) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  const int64_t total = (int64_t)B * Ho * Wo * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * V;
  int64_t pix = t / cv;
  const int wo = (int)(pix % Wo);
  pix /= Wo;
  const int ho = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  float best[V];
  uint8_t bi[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    best[i] = -INFINITY;
    bi[i] = 0;
  }
  for (int r = 0; r < k; ++r) {
    const int h = ho * s - pad + r;
    if (h < 0 || h >= H) continue;
    for (int q = 0; q < k; ++q) {
      const int w = wo * s - pad + q;
      if (w < 0 || w >= W) continue;
      float v[V];
      ldv<V>(x + (((int64_t)b * H + h) * W + w) * C + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i)
        if (v[i] > best[i]) {
          best[i] = v[i];
          bi[i] = (uint8_t)(r * k + q);
        }
    }
  }
  const int64_t o = (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
  stv<V>(y + o, best);
  if (relu_bit) {                 // the window max is > 0: its ReLU was active (k*k <= 128)
#pragma unroll
    for (int i = 0; i < V; ++i) bi[i] |= best[i] > 0.f ? 0x80 : 0;
  }
  if constexpr (V == 8) {
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + o) = packed;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) arg[o + i] = bi[i];
  }
}

template <typename T, int V>
__global__ __launch_bounds__(PT) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                         const uint8_t* __restrict__ arg,
                                                         T* __restrict__ dx, int B, int H,
                                                         int W, int C, int Ho, int Wo, int k,
                                                         int s, int pad) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  const int64_t total = (int64_t)B * H * W * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * V;
  int64_t pix = t / cv;
  const int w = (int)(pix % W);
  pix /= W;
  const int h = (int)(pix % H);
  const int b = (int)(pix / H);
  float acc[V] = {};
  // windows containing h: ho*s - pad <= h <= ho*s - pad + k - 1
  int ho0 = (h + pad - k + 1 + s - 1) / s;
  if (h + pad - k + 1 < 0) ho0 = 0;
  const int ho1 = min(Ho - 1, (h + pad) / s);
  int wo0 = (w + pad - k + 1 + s - 1) / s;
  if (w + pad - k + 1 < 0) wo0 = 0;
  const int wo1 = min(Wo - 1, (w + pad) / s);
  for (int ho = ho0; ho <= ho1; ++ho) {
    for (int wo = wo0; wo <= wo1; ++wo) {
      const uint8_t want = (uint8_t)((h + pad - ho * s) * k + (w + pad - wo * s));
      const int64_t o = (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
      float g[V];
      ldv<V>(dy + o, g);
      if constexpr (V == 8) {
        uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          uint32_t word = i < 4 ? packed.x : packed.y;
          uint8_t a = (uint8_t)(word >> (8 * (i & 3)));
          if (a == want) acc[i] += g[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i)
          if (arg[o + i] == want) acc[i] += g[i];
      }
    }
  }
  stv<V>(dx + (((int64_t)b * H + h) * W + w) * C + c0, acc);
}

// Max-pool backward fused with the backward of the conv + bias + ReLU layer
// that produced the pool's input (VGG's last conv of a block; ops.nn
// BiasActLink): the forward stored bit 7 of each argmax byte = "the window
// max is > 0" (relu_bit), so the input gradient of the pool IS the ReLU'ed
// dz -- dz(p) = dy(window) where p is the window's argmax and its value was
// > 0 -- and the same pass sums dz per channel into the layer's bias
// gradient (fp32 atomics, one per channel and block; the optimizer clears
// the gradient it consumes).  Replaces maxpool_bwd + bias_act_bwd, which
// read and wrote the full-resolution tensor three more times.
// Block = cw channel groups (8 channels each) x lanes pixel rows; blockIdx.y
// walks pixel chunks of ppb pixels.
template <typename T>
__global__ __launch_bounds__(PT) void maxpool_bwd_relu_bias_kernel(
    const T* __restrict__ dy, const uint8_t* __restrict__ arg, T* __restrict__ dx,
    float* __restrict__ dbias, int64_t gstride, int Cper, int B, int H, int W, int C, int Ho,
    int Wo, int k, int s, int pad, int64_t ppb) {
  constexpr int V = 8;
  __shared__ float red[PT * V];
  const int cv = C / V;
  const int cw = cv < PT ? cv : PT;
  const int lanes = PT / cw;
  const int j = threadIdx.x % cw, l = threadIdx.x / cw;
  const int cg = blockIdx.x * cw + j;
  const bool on = l < lanes && cg < cv;
  const int c0 = cg * V;
  const int64_t P = (int64_t)B * H * W;
  const int64_t p0 = (int64_t)blockIdx.y * ppb;
  const int64_t p1 = p0 + ppb < P ? p0 + ppb : P;
  float sum[V] = {};
  if (on) {
    for (int64_t pix = p0 + l; pix < p1; pix += lanes) {
      const int w = (int)(pix % W);
      const int64_t bh = pix / W;
      const int h = (int)(bh % H);
      const int b = (int)(bh / H);
      float acc[V] = {};
      int ho0 = (h + pad - k + 1 + s - 1) / s;
      if (h + pad - k + 1 < 0) ho0 = 0;
      const int ho1 = min(Ho - 1, (h + pad) / s);
      int wo0 = (w + pad - k + 1 + s - 1) / s;
      if (w + pad - k + 1 < 0) wo0 = 0;
      const int wo1 = min(Wo - 1, (w + pad) / s);
      for (int ho = ho0; ho <= ho1; ++ho) {
        for (int wo = wo0; wo <= wo1; ++wo) {
          const uint32_t want = 0x80u | (uint32_t)((h + pad - ho * s) * k + (w + pad - wo * s));
          const int64_t o = (((int64_t)b * Ho + ho) * Wo + wo) * C + c0;
          float g[V];
          ldv<V>(dy + o, g);
          const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const uint32_t word = i < 4 ? packed.x : packed.y;
            if (((word >> (8 * (i & 3))) & 0xffu) == want) acc[i] += g[i];
          }
        }
      }
      stv<V>(dx + pix * C + c0, acc);
#pragma unroll
      for (int i = 0; i < V; ++i) sum[i] += acc[i];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) red[threadIdx.x * V + i] = sum[i];
  __syncthreads();
  if (on && l == 0) {
    for (int ll = 1; ll < lanes; ++ll)
#pragma unroll
      for (int i = 0; i < V; ++i) sum[i] += red[(ll * cw + j) * V + i];
    const int g = c0 / Cper, cc = c0 - g * Cper;
#pragma unroll
    for (int i = 0; i < V; ++i) atomicAdd(dbias + (int64_t)g * gstride + cc + i, sum[i]);
  }
}

// The same for a tiling pool (k == s, no padding, H % k == W % k == 0:
// VGG's 2x2/2): one thread per (pooled pixel, 8 channels) reads dy and the
// argmax bytes ONCE and writes its whole k x k window (dz at the argmax if
// its ReLU was active, zeros elsewhere), four pooled pixels' loads in flight
// per thread.  Few blocks (~512 per launch): every block adds one partial
// per channel into the bias gradient, and thousands of same-address fp32
// atomics per channel serialise in L2 (the first version, 8192 blocks, ran at
// 0.9 TB/s; profiles/r5_vgg.md).
template <typename T>
__global__ __launch_bounds__(PT) void maxpool_bwd_relu_bias_tiled_kernel(
    const T* __restrict__ dy, const uint8_t* __restrict__ arg, T* __restrict__ dx,
    float* __restrict__ dbias, int64_t gstride, int Cper, int B, int H, int W, int C, int Ho,
    int Wo, int k, int64_t qpb) {
  constexpr int V = 8, U = 4;
  __shared__ float red[PT * V];
  const int cv = C / V;
  const int cw = cv < PT ? cv : PT;
  const int lanes = PT / cw;
  const int j = threadIdx.x % cw, l = threadIdx.x / cw;
  const int cg = blockIdx.x * cw + j;
  const bool on = l < lanes && cg < cv;
  const int c0 = cg * V;
  const int64_t Q = (int64_t)B * Ho * Wo;
  const int64_t q0 = (int64_t)blockIdx.y * qpb;
  const int64_t q1 = q0 + qpb < Q ? q0 + qpb : Q;
  float sum[V] = {};
  if (on) {
    for (int64_t qb = q0 + l; qb < q1; qb += U * lanes) {
      float g[U][V];
      uint2 pk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {            // all loads first
        const int64_t q = qb + (int64_t)u * lanes;
        if (q < q1) {
          ldv<V>(dy + q * C + c0, g[u]);
          pk[u] = *reinterpret_cast<const uint2*>(arg + q * C + c0);
        } else {
          pk[u] = make_uint2(0u, 0u);
#pragma unroll
          for (int i = 0; i < V; ++i) g[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = qb + (int64_t)u * lanes;
        if (q >= q1) break;
        uint32_t a[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
          a[i] = ((i < 4 ? pk[u].x : pk[u].y) >> (8 * (i & 3))) & 0xffu;
          if (a[i] & 0x80u) sum[i] += g[u][i];
        }
        const int wo = (int)(q % Wo);
        const int64_t bho = q / Wo;
        const int ho = (int)(bho % Ho);
        const int b = (int)(bho / Ho);
        for (int r = 0; r < k; ++r)
          for (int t = 0; t < k; ++t) {
            const uint32_t want = 0x80u | (uint32_t)(r * k + t);
            float o[V];
#pragma unroll
            for (int i = 0; i < V; ++i) o[i] = a[i] == want ? g[u][i] : 0.f;
            stv<V>(dx + (((int64_t)b * H + ho * k + r) * W + wo * k + t) * C + c0, o);
          }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) red[threadIdx.x * V + i] = sum[i];
  __syncthreads();
  if (on && l == 0) {
    for (int ll = 1; ll < lanes; ++ll)
#pragma unroll
      for (int i = 0; i < V; ++i) sum[i] += red[(ll * cw + j) * V + i];
    const int g = c0 / Cper, cc = c0 - g * Cper;
#pragma unroll
    for (int i = 0; i < V; ++i) atomicAdd(dbias + (int64_t)g * gstride + cc + i, sum[i]);
  }
}

// global average pool: x [B, HW, C] -> y [B, C]
template <typename T, int V>
__global__ __launch_bounds__(PT) void gavg_fwd_kernel(const T* __restrict__ x,
                                                      T* __restrict__ y, int B, int HW,
                                                      int C) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  if (t >= (int64_t)B * cv) return;
  const int c0 = (int)(t % cv) * V;
  const int b = (int)(t / cv);
  float acc[V] = {};
  for (int i = 0; i < HW; ++i) {
    float v[V];
    ldv<V>(x + ((int64_t)b * HW + i) * C + c0, v);
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] += v[j];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] *= inv;
  stv<V>(y + (int64_t)b * C + c0, acc);
}

template <typename T, int V>
__global__ __launch_bounds__(PT) void gavg_bwd_kernel(const T* __restrict__ dy,
                                                      T* __restrict__ dx, int B, int HW,
                                                      int C) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  const int64_t total = (int64_t)B * HW * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * V;
  const int64_t pix = t / cv;
  const int b = (int)(pix / HW);
  float g[V];
  ldv<V>(dy + (int64_t)b * C + c0, g);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < V; ++j) g[j] *= inv;
  stv<V>(dx + pix * C + c0, g);
}

// bias + activation: y = act(x + bias[g][c]) over [M, C] packed channels
template <typename T>
__global__ __launch_bounds__(PT) void bias_act_fwd_kernel(const T* __restrict__ x,
                                                          const T* __restrict__ bias,
                                                          int64_t bstride, T* __restrict__ y,
                                                          int64_t M, int C, int Cper, int act) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / 8;
  if (t >= M * cv) return;
  const int c0 = (int)(t % cv) * 8;
  const int g = c0 / Cper, cc = c0 - g * Cper;
  float v[8], b[8];
  ld8(x + t * 8, v);
  ld8(bias + g * bstride + cc, b);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float z = v[i] + b[i];
    v[i] = act == 6 ? fminf(fmaxf(z, 0.f), 6.f) : (act ? fmaxf(z, 0.f) : z);
  }
  st8(y + t * 8, v);
}

// dz = act'(y) * dy  (written to dx) and per-channel partial sums of dz
template <typename T>
__global__ __launch_bounds__(PT) void bias_act_bwd_kernel(const T* __restrict__ dy,
                                                          const T* __restrict__ y,
                                                          T* __restrict__ dx, float* ws,
                                                          int64_t M, int C, int rows, int act) {
  const int c0 = (blockIdx.x * PT + threadIdx.x) * 8;
  if (c0 >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = min(M, r0 + rows);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = r0; r < r1; ++r) {
    float d[8], yv[8];
    ld8(dy + r * C + c0, d);
    ld8(y + r * C + c0, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float z = act == 6 ? ((yv[i] > 0.f && yv[i] < 6.f) ? d[i] : 0.f)
                         : (act ? (yv[i] > 0.f ? d[i] : 0.f) : d[i]);
      d[i] = z;
      s[i] += z;
    }
    st8(dx + r * C + c0, d);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) atomicAdd(&ws[c0 + i], s[i]);
}

__global__ void bias_grad_scatter(const float* ws, float* dbias, int64_t gstride, int C,
                                  int Cper) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int g = c / Cper;
  dbias[g * gstride + (c - g * Cper)] = ws[c];
}

// scalar fallbacks for channel counts that are not multiples of 8 (N = 500, 10, 2 heads)
template <typename T>
__global__ __launch_bounds__(PT) void bias_act_fwd_scalar(const T* __restrict__ x,
                                                          const T* __restrict__ bias,
                                                          int64_t bstride, T* __restrict__ y,
                                                          int64_t M, int C, int Cper, int act) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  if (t >= M * C) return;
  const int c = (int)(t % C);
  const int g = c / Cper;
  float z = ld1(x + t) + ld1(bias + g * bstride + (c - g * Cper));
  z = act == 6 ? fminf(fmaxf(z, 0.f), 6.f) : (act ? fmaxf(z, 0.f) : z);
  st1(y + t, z);
}

template <typename T>
__global__ __launch_bounds__(PT) void bias_act_bwd_scalar(const T* __restrict__ dy,
                                                          const T* __restrict__ y,
                                                          T* __restrict__ dx, float* ws,
                                                          int64_t M, int C, int rows, int act) {
  const int c = blockIdx.x * PT + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = min(M, r0 + rows);
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    const float d = ld1(dy + r * C + c), yv = ld1(y + r * C + c);
    const float z = act == 6 ? ((yv > 0.f && yv < 6.f) ? d : 0.f) : (act ? (yv > 0.f ? d : 0.f) : d);
    st1(dx + r * C + c, z);
    s += z;
  }
  atomicAdd(&ws[c], s);
}

template <typename T>
static int cer_maxpool_fwd_t(const T* x, T* y, uint8_t* arg, int B, int H, int W, int C,
                            int Ho, int Wo, int k, int s, int pad, int relu_bit,
                            hipStream_t stream) {
  if (k * k > 255 || (relu_bit && (k * k > 128 || C % 8))) return (int)hipErrorInvalidValue;
  // 8 channels per thread when C % 8 == 0, else 1 (ragged widths)
  if (C % 8 == 0)
    maxpool_fwd_kernel<T, 8><<<cer_blocks((int64_t)B * Ho * Wo * (C / 8), PT), PT, 0, stream>>>(
        x, y, arg, B, H, W, C, Ho, Wo, k, s, pad, relu_bit);
  else
    maxpool_fwd_kernel<T, 1><<<cer_blocks((int64_t)B * Ho * Wo * C, PT), PT, 0, stream>>>(
        x, y, arg, B, H, W, C, Ho, Wo, k, s, pad, 0);
  return (int)hipGetLastError();
}

// dz of the pooled conv + bias + ReLU layer and its bias gradient (see
// maxpool_bwd_relu_bias_kernel); the forward ran with relu_bit = 1
template <typename T>
static int cer_maxpool_bwd_relu_bias_t(const T* dy, const uint8_t* arg, T* dx, float* dbias,
                                      int64_t gstride, int Cper, int B, int H, int W, int C,
                                      int Ho, int Wo, int k, int s, int pad, hipStream_t stream) {
  if (C % 8 || Cper % 8 || k * k > 128) return (int)hipErrorInvalidValue;
  const int cv = C / 8;
  const int cw = cv < PT ? cv : PT;
  const int gx = (cv + cw - 1) / cw;
  const int64_t P = (int64_t)B * H * W;
  const int lanes = PT / cw;
  if (k == s && pad == 0 && H == Ho * k && W == Wo * k) {
    // tiling pool: thread per pooled pixel; ~512 blocks (bias atomics per
    // channel), >= 4 pooled pixels per lane
    const int64_t Q = (int64_t)B * Ho * Wo;
    int64_t gy = (512 + gx - 1) / gx;
    int64_t qpb = (Q + gy - 1) / gy;
    if (qpb < 4 * lanes) qpb = 4 * lanes;
    gy = (Q + qpb - 1) / qpb;
    maxpool_bwd_relu_bias_tiled_kernel<T><<<dim3((unsigned)gx, (unsigned)gy), PT, 0, stream>>>(
        dy, arg, dx, dbias, gstride, Cper, B, H, W, C, Ho, Wo, k, qpb);
    return (int)hipGetLastError();
  }
  // ~512 blocks (bias atomics per channel), at least 4 pixels per lane
  int64_t gy = (512 + gx - 1) / gx;
  int64_t ppb = (P + gy - 1) / gy;
  if (ppb < 4 * lanes) ppb = 4 * lanes;
  gy = (P + ppb - 1) / ppb;
  maxpool_bwd_relu_bias_kernel<T><<<dim3((unsigned)gx, (unsigned)gy), PT, 0, stream>>>(
      dy, arg, dx, dbias, gstride, Cper, B, H, W, C, Ho, Wo, k, s, pad, ppb);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_maxpool_bwd_t(const T* dy, const uint8_t* arg, T* dx, int B, int H,
                            int W, int C, int Ho, int Wo, int k, int s, int pad,
                            hipStream_t stream) {
  if (C % 8 == 0)
    maxpool_bwd_kernel<T, 8><<<cer_blocks((int64_t)B * H * W * (C / 8), PT), PT, 0, stream>>>(
        dy, arg, dx, B, H, W, C, Ho, Wo, k, s, pad);
  else
    maxpool_bwd_kernel<T, 1><<<cer_blocks((int64_t)B * H * W * C, PT), PT, 0, stream>>>(
        dy, arg, dx, B, H, W, C, Ho, Wo, k, s, pad);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_gavgpool_fwd_t(const T* x, T* y, int B, int HW, int C,
                             hipStream_t stream) {
  if (C % 8 == 0)
    gavg_fwd_kernel<T, 8><<<cer_blocks((int64_t)B * (C / 8), PT), PT, 0, stream>>>(x, y, B, HW, C);
  else
    gavg_fwd_kernel<T, 1><<<cer_blocks((int64_t)B * C, PT), PT, 0, stream>>>(x, y, B, HW, C);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_gavgpool_bwd_t(const T* dy, T* dx, int B, int HW, int C,
                             hipStream_t stream) {
  if (C % 8 == 0)
    gavg_bwd_kernel<T, 8><<<cer_blocks((int64_t)B * HW * (C / 8), PT), PT, 0, stream>>>(dy, dx, B,
                                                                                      HW, C);
  else
    gavg_bwd_kernel<T, 1><<<cer_blocks((int64_t)B * HW * C, PT), PT, 0, stream>>>(dy, dx, B, HW, C);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_bias_act_fwd_t(const T* x, const T* bias, int64_t bstride, T* y,
                             int64_t M, int C, int Cper, int act, hipStream_t stream) {
  if (C % 8 || Cper % 8) {
    bias_act_fwd_scalar<T><<<cer_blocks(M * C, PT), PT, 0, stream>>>(x, bias, bstride, y, M, C,
                                                                  Cper, act);
    return (int)hipGetLastError();
  }
  bias_act_fwd_kernel<T><<<cer_blocks(M * (C / 8), PT), PT, 0, stream>>>(x, bias, bstride, y, M, C,
                                                                      Cper, act);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_bias_act_bwd_t(const T* dy, const T* y, T* dx, float* dbias,
                             int64_t gstride, float* ws, int64_t M, int C, int Cper, int act,
                             hipStream_t stream) {
  if (C % 8 || Cper % 8) {
    const int cb = cer_blocks(C, PT);
    int64_t want = (1024 + cb - 1) / cb;
    int64_t rows = (M + want - 1) / want;
    if (rows < 16) rows = 16;
    dim3 grid(cb, (unsigned)((M + rows - 1) / rows));
    cer_zero_async(ws, sizeof(float) * C, stream);
    bias_act_bwd_scalar<T><<<grid, PT, 0, stream>>>(dy, y, dx, ws, M, C, (int)rows, act);
    bias_grad_scatter<<<cer_blocks(C, 256), 256, 0, stream>>>(ws, dbias, gstride, C, Cper);
    return (int)hipGetLastError();
  }
  int cblocks = cer_blocks(C / 8, PT);
  int64_t want = (2048 + cblocks - 1) / cblocks;
  int64_t rows = (M + want - 1) / want;
  if (rows < 16) rows = 16;
  dim3 grid(cblocks, (unsigned)((M + rows - 1) / rows));
  cer_zero_async(ws, sizeof(float) * C, stream);
  bias_act_bwd_kernel<T><<<grid, PT, 0, stream>>>(dy, y, dx, ws, M, C, (int)rows, act);
  bias_grad_scatter<<<cer_blocks(C, 256), 256, 0, stream>>>(ws, dbias, gstride, C, Cper);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// k x k average pooling, stride s, top/left zero padding (pt, pl); the output
// size fixes the bottom/right padding.  count_pad: divide by k*k, else by the
// number of in-bounds taps (TF/Keras 'same', torch count_include_pad=False).
// DenseNet transitions (2x2/2) and NASNet cells (3x3/1 same, 3x3/2 valid).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float avg_div(int ho, int wo, int H, int W, int k, int s, int pt,
                                         int pl, int count_pad) {
  if (count_pad) return 1.f / (float)(k * k);
  const int h0 = max(ho * s - pt, 0), h1 = min(ho * s - pt + k, H);
  const int w0 = max(wo * s - pl, 0), w1 = min(wo * s - pl + k, W);
  const int n = max(h1 - h0, 0) * max(w1 - w0, 0);
  return n > 0 ? 1.f / (float)n : 0.f;
}

template <typename T, int V>
__global__ __launch_bounds__(PT) void avgpool_fwd_kernel(const T* __restrict__ x,
                                                         T* __restrict__ y, int B, int H,
                                                         int W, int C, int Ho, int Wo, int k,
                                                         int s, int pt, int pl, int count_pad) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  const int64_t total = (int64_t)B * Ho * Wo * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * V;
  int64_t pix = t / cv;
  const int wo = (int)(pix % Wo);
  pix /= Wo;
  const int ho = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  float acc[V] = {};
  for (int r = 0; r < k; ++r) {
    const int h = ho * s - pt + r;
    if (h < 0 || h >= H) continue;
    for (int q = 0; q < k; ++q) {
      const int w = wo * s - pl + q;
      if (w < 0 || w >= W) continue;
      float v[V];
      ldv<V>(x + (((int64_t)b * H + h) * W + w) * C + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += v[i];
    }
  }
  const float inv = avg_div(ho, wo, H, W, k, s, pt, pl, count_pad);
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] *= inv;
  stv<V>(y + (((int64_t)b * Ho + ho) * Wo + wo) * C + c0, acc);
}

// deterministic gather: each input pixel sums dy / divisor over the windows covering it
template <typename T, int V>
__global__ __launch_bounds__(PT) void avgpool_bwd_kernel(const T* __restrict__ dy,
                                                         T* __restrict__ dx, int B, int H,
                                                         int W, int C, int Ho, int Wo, int k,
                                                         int s, int pt, int pl, int count_pad) {
  const int64_t t = (int64_t)blockIdx.x * PT + threadIdx.x;
  const int cv = C / V;
  const int64_t total = (int64_t)B * H * W * cv;
  if (t >= total) return;
  const int c0 = (int)(t % cv) * V;
  int64_t pix = t / cv;
  const int w = (int)(pix % W);
  pix /= W;
  const int h = (int)(pix % H);
  const int b = (int)(pix / H);
  // windows containing h: ho*s - pt <= h <= ho*s - pt + k - 1
  const int hl = h + pt - k + 1, wl = w + pl - k + 1;
  const int ho0 = hl <= 0 ? 0 : (hl + s - 1) / s;
  const int wo0 = wl <= 0 ? 0 : (wl + s - 1) / s;
  const int ho1 = min(Ho - 1, (h + pt) / s);
  const int wo1 = min(Wo - 1, (w + pl) / s);
  float acc[V] = {};
  for (int ho = ho0; ho <= ho1; ++ho) {
    for (int wo = wo0; wo <= wo1; ++wo) {
      float g[V];
      ldv<V>(dy + (((int64_t)b * Ho + ho) * Wo + wo) * C + c0, g);
      const float inv = avg_div(ho, wo, H, W, k, s, pt, pl, count_pad);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += g[i] * inv;
    }
  }
  stv<V>(dx + (((int64_t)b * H + h) * W + w) * C + c0, acc);
}

template <typename T>
static int cer_avgpool_fwd_t(const T* x, T* y, int B, int H, int W, int C, int Ho,
                            int Wo, int k, int s, int pt, int pl, int count_pad,
                            hipStream_t stream) {
  if (k < 1 || s < 1 || pt < 0 || pl < 0 || pt >= k || pl >= k)
    return (int)hipErrorInvalidValue;
  if (C % 8 == 0)
    avgpool_fwd_kernel<T, 8><<<cer_blocks((int64_t)B * Ho * Wo * (C / 8), PT), PT, 0, stream>>>(
        x, y, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad);
  else
    avgpool_fwd_kernel<T, 1><<<cer_blocks((int64_t)B * Ho * Wo * C, PT), PT, 0, stream>>>(
        x, y, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad);
  return (int)hipGetLastError();
}

template <typename T>
static int cer_avgpool_bwd_t(const T* dy, T* dx, int B, int H, int W, int C, int Ho,
                            int Wo, int k, int s, int pt, int pl, int count_pad,
                            hipStream_t stream) {
  if (k < 1 || s < 1 || pt < 0 || pl < 0 || pt >= k || pl >= k)
    return (int)hipErrorInvalidValue;
  if (C % 8 == 0)
    avgpool_bwd_kernel<T, 8><<<cer_blocks((int64_t)B * H * W * (C / 8), PT), PT, 0, stream>>>(
        dy, dx, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad);
  else
    avgpool_bwd_kernel<T, 1><<<cer_blocks((int64_t)B * H * W * C, PT), PT, 0, stream>>>(
        dy, dx, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad);
  return (int)hipGetLastError();
}

#define CER_POOL_ENTRY_POINTS(T, SFX)                                                            \
  CER_API int cer_maxpool_fwd##SFX(const T* x, T* y, uint8_t* arg, int B, int H, int W, int C,  \
                                   int Ho, int Wo, int k, int s, int pad, int relu_bit,          \
                                   hipStream_t st) {                                             \
    return cer_maxpool_fwd_t<T>(x, y, arg, B, H, W, C, Ho, Wo, k, s, pad, relu_bit, st);         \
  }                                                                                              \
  CER_API int cer_maxpool_bwd_relu_bias##SFX(const T* dy, const uint8_t* arg, T* dx,            \
                                             float* dbias, int64_t gstride, int Cper, int B,     \
                                             int H, int W, int C, int Ho, int Wo, int k, int s,  \
                                             int pad, hipStream_t st) {                          \
    return cer_maxpool_bwd_relu_bias_t<T>(dy, arg, dx, dbias, gstride, Cper, B, H, W, C, Ho, Wo, \
                                          k, s, pad, st);                                        \
  }                                                                                              \
  CER_API int cer_maxpool_bwd##SFX(const T* dy, const uint8_t* arg, T* dx, int B, int H, int W, \
                                   int C, int Ho, int Wo, int k, int s, int pad,                 \
                                   hipStream_t st) {                                             \
    return cer_maxpool_bwd_t<T>(dy, arg, dx, B, H, W, C, Ho, Wo, k, s, pad, st);                 \
  }                                                                                              \
  CER_API int cer_gavgpool_fwd##SFX(const T* x, T* y, int B, int HW, int C, hipStream_t st) {   \
    return cer_gavgpool_fwd_t<T>(x, y, B, HW, C, st);                                            \
  }                                                                                              \
  CER_API int cer_gavgpool_bwd##SFX(const T* dy, T* dx, int B, int HW, int C, hipStream_t st) { \
    return cer_gavgpool_bwd_t<T>(dy, dx, B, HW, C, st);                                          \
  }                                                                                              \
  CER_API int cer_bias_act_fwd##SFX(const T* x, const T* bias, int64_t bstride, T* y,           \
                                    int64_t M, int C, int Cper, int act, hipStream_t st) {       \
    return cer_bias_act_fwd_t<T>(x, bias, bstride, y, M, C, Cper, act, st);                      \
  }                                                                                              \
  CER_API int cer_bias_act_bwd##SFX(const T* dy, const T* y, T* dx, float* dbias,               \
                                    int64_t gstride, float* ws, int64_t M, int C, int Cper,      \
                                    int act, hipStream_t st) {                                   \
    return cer_bias_act_bwd_t<T>(dy, y, dx, dbias, gstride, ws, M, C, Cper, act, st);            \
  }                                                                                              \
  CER_API int cer_avgpool_fwd##SFX(const T* x, T* y, int B, int H, int W, int C, int Ho, int Wo,\
                                   int k, int s, int pt, int pl, int count_pad,                  \
                                   hipStream_t st) {                                             \
    return cer_avgpool_fwd_t<T>(x, y, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad, st);          \
  }                                                                                              \
  CER_API int cer_avgpool_bwd##SFX(const T* dy, T* dx, int B, int H, int W, int C, int Ho,      \
                                   int Wo, int k, int s, int pt, int pl, int count_pad,          \
                                   hipStream_t st) {                                             \
    return cer_avgpool_bwd_t<T>(dy, dx, B, H, W, C, Ho, Wo, k, s, pt, pl, count_pad, st);        \
  }

CER_POOL_ENTRY_POINTS(bf16_t, )
CER_POOL_ENTRY_POINTS(float, _f32)
