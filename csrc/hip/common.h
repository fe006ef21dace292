// Shared helpers for the CDNA4 (gfx950) kernels of cerebro_ds_kpgi_amd.
//
// Every entry point is `extern "C"`, takes raw device pointers + a
// hipStream_t, launches on that stream (so HIP-graph capture by the caller
// works) and returns the hipError_t of the launch.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define CER_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;  // raw bf16 bits (round-to-nearest-even conversions below)

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// pack two floats into one dword of bf16 (lo = a, hi = b)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// ---------------------------------------------------------------------------
// Storage-dtype generic element access.  Every activation / parameter kernel
// is a template over its storage type T (bf16_t: the bf16 compute mode,
// float: the reference-precision fp32 mode); arithmetic is always fp32.
// 8 consecutive elements = one 16-B (bf16) or two 16-B (fp32) accesses.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ void st8(bf16_t* p, const float* v) {
  uint4 u;
  u.x = pack_bf2(v[0], v[1]);
  u.y = pack_bf2(v[2], v[3]);
  u.z = pack_bf2(v[4], v[5]);
  u.w = pack_bf2(v[6], v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

__device__ __forceinline__ void st8(float* p, const float* v) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  // gfx950 v_cvt_pk_bf16_f32 (round to nearest even, NaN preserving)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}

// 8 fp32 -> HL format: [8 x bf16 hi | 8 x bf16 lo], hi = RNE(x), lo =
// RNE(x - hi) -- exactly the operand split of the fp32 3-pass conv kernels
// (conv.hip split_hi_lo / take_hi_lo), in the 32 bytes of the 8 fp32
__device__ __forceinline__ void st8_hl(float* p, const float* v) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t hp = cvt_pk_bf16(v[2 * i], v[2 * i + 1]);
    h[i] = hp;
    l[i] = cvt_pk_bf16(v[2 * i] - __uint_as_float(hp << 16),
                       v[2 * i + 1] - __uint_as_float(hp & 0xffff0000u));
  }
  reinterpret_cast<uint4*>(p)[0] = make_uint4(h[0], h[1], h[2], h[3]);
  reinterpret_cast<uint4*>(p)[1] = make_uint4(l[0], l[1], l[2], l[3]);
}
__device__ __forceinline__ void st8_hl(bf16_t* p, const float* v) { st8(p, v); }  // bf16: unused

__device__ __forceinline__ float ld1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }

// V consecutive elements (V = 8: ld8 / st8; V = 1: one element) -- the
// vector width of the per-channel kernels (BN, pooling, depthwise conv):
// 8 when every config's channel count is a multiple of 8, else 1 (ragged
// widths such as NASNet-Mobile's 11 / 22 / 44 filters)
template <int V, typename T>
__device__ __forceinline__ void ldv(const T* p, float* v) {
  if constexpr (V == 8) {
    ld8(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = ld1(p + i);
  }
}

template <int V, typename T>
__device__ __forceinline__ void stv(T* p, const float* v) {
  if constexpr (V == 8) {
    st8(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) st1(p + i, v[i]);
  }
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide reduction for blockDim.x <= 1024 (wave64). `smem` >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = warp_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < (unsigned)nw) ? smem[threadIdx.x] : 0.f;
  if (wid == 0) r = warp_sum(r);
  if (threadIdx.x == 0) smem[0] = r;
  __syncthreads();
  r = smem[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_max(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = warp_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < (unsigned)nw) ? smem[threadIdx.x] : -INFINITY;
  if (wid == 0) r = warp_max(r);
  if (threadIdx.x == 0) smem[0] = r;
  __syncthreads();
  r = smem[0];
  __syncthreads();
  return r;
}

static inline int cer_blocks(int64_t n, int per_block) {
  return (int)((n + per_block - 1) / per_block);
}

// ---------------------------------------------------------------------------
// Device fill / copy as KERNELS.  Never hipMemsetAsync / hipMemcpyAsync on a
// launch path: captured into a HIP graph, a small hipMemsetAsync node does not
// re-execute correctly from the second replay on (ROCm 7.x; 4 KB fill ->
// garbage, scripts/debug/graph_memset_repro.py).  That was the root cause of
// the round-1 graph-replay corruption (non-finite weights from replay 2).
// A kernel node replays like every other kernel.
// ---------------------------------------------------------------------------
static __global__ __launch_bounds__(256) void cer_fill_kernel(uint8_t* __restrict__ dst,
                                                              const uint8_t* __restrict__ src,
                                                              size_t bytes, int vec) {
  // src == nullptr: zero fill; vec: 16-B body (both pointers 16-B aligned) + byte tail
  const size_t n16 = vec ? bytes / 16 : 0;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t k = i; k < n16; k += stride)
    reinterpret_cast<uint4*>(dst)[k] = src ? reinterpret_cast<const uint4*>(src)[k]
                                           : make_uint4(0u, 0u, 0u, 0u);
  for (size_t k = n16 * 16 + i; k < bytes; k += stride) dst[k] = src ? src[k] : (uint8_t)0;
}

static inline void cer_launch_fill(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (!bytes) return;
  const int vec = ((uintptr_t)dst % 16 == 0) && ((uintptr_t)src % 16 == 0);
  int blocks = cer_blocks((int64_t)(vec ? (bytes + 15) / 16 : bytes), 256);
  if (blocks > 4096) blocks = 4096;
  cer_fill_kernel<<<blocks, 256, 0, stream>>>((uint8_t*)dst, (const uint8_t*)src, bytes, vec);
}

static inline void cer_zero_async(void* dst, size_t bytes, hipStream_t stream) {
  cer_launch_fill(dst, nullptr, bytes, stream);
}

static inline void cer_copy_async(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  cer_launch_fill(dst, src, bytes, stream);
}
