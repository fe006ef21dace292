// Device-side batch gather + normalisation from the HBM partition store
// (replaces the reference's per-sample Python generators).
//
// X     uint8 [P, n, H, W, 3]   partitions pinned in HBM
// perm  int32 [P, n]            this epoch's shuffle of every partition
// part  int32 [G]               partition trained by config row g
// cursor int32 [1]              batch index (device scalar -> graph capturable)
// out   bf16 / fp32 [B, H, W, G*3]  packed NHWC input of the G configs
// yout  int32 [G, B]
// One thread per output pixel-config (3 channels).  Reads are 3-byte
// gathers of random images; writes of a pixel's G*3 channels are contiguous.
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void gather_images_kernel(
    const uint8_t* __restrict__ X, const int* __restrict__ Y, const int* __restrict__ perm,
    const int* __restrict__ part, const int* __restrict__ cursor, T* __restrict__ out,
    int* __restrict__ yout, int n, int HW, int G, int B, float m0, float m1, float m2,
    float s0, float s1, float s2) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * HW * G;
  if (tid >= total) return;
  const int g = (int)(tid % G);
  const int64_t pix = tid / G;  // b * HW + hw
  const int b = (int)(pix / HW);
  const int hw = (int)(pix % HW);
  const int p = part[g];
  const int row = perm[(int64_t)p * n + (int64_t)cursor[0] * B + b];
  const uint8_t* src = X + (((int64_t)p * n + row) * HW + hw) * 3;
  T* dst = out + pix * (G * 3) + g * 3;
  st1(dst + 0, ((float)src[0] - m0) * s0);
  st1(dst + 1, ((float)src[1] - m1) * s1);
  st1(dst + 2, ((float)src[2] - m2) * s2);
  if (hw == 0) yout[g * B + b] = Y[(int64_t)p * n + row];
}

template <typename T>
static int gather_images_t(const uint8_t* X, const int* Y, const int* perm, const int* part,
                           const int* cursor, T* out, int* yout, int n, int HW, int G, int B,
                           const float* mean255, const float* inv_std255, hipStream_t stream) {
  int64_t total = (int64_t)B * HW * G;
  gather_images_kernel<T><<<cer_blocks(total, 256), 256, 0, stream>>>(
      X, Y, perm, part, cursor, out, yout, n, HW, G, B, mean255[0], mean255[1], mean255[2],
      inv_std255[0], inv_std255[1], inv_std255[2]);
  return (int)hipGetLastError();
}

// out: bf16 (compute mode) / fp32 (_f32, reference-precision mode)
CER_API int cer_gather_images(const uint8_t* X, const int* Y, const int* perm, const int* part,
                              const int* cursor, bf16_t* out, int* yout, int n, int HW, int G,
                              int B, const float* mean255, const float* inv_std255,
                              hipStream_t stream) {
  return gather_images_t(X, Y, perm, part, cursor, out, yout, n, HW, G, B, mean255, inv_std255,
                         stream);
}

CER_API int cer_gather_images_f32(const uint8_t* X, const int* Y, const int* perm, const int* part,
                                  const int* cursor, float* out, int* yout, int n, int HW, int G,
                                  int B, const float* mean255, const float* inv_std255,
                                  hipStream_t stream) {
  return gather_images_t(X, Y, perm, part, cursor, out, yout, n, HW, G, B, mean255, inv_std255,
                         stream);
}
