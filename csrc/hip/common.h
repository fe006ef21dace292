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
