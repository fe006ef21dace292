// Embedding-bag first layer of the Criteo MLP: a one-hot
// input row with <= nnz active columns times a dense [K, N] kernel is the sum
// of nnz kernel rows.  idx [G, B, nnz] int32 (-1 = padding), W_g [K, N] bf16
// at w + g*w_gstride, bias_g [N].
//   fwd : y[b, g*N + n] = act(bias_g[n] + sum_j W_g[idx[g,b,j], n])
//   bwd : dz = act'(y) * dy ; dW_g[idx, :] += dz (fp32 atomics into the
//         gradient arena, which the optimizer keeps zeroed) ; db_g += sum_b dz
// One block per (b, g); a thread owns 8 consecutive n (16-B row loads).
#include "common.h"

namespace {

constexpr int EB_V = 8;

__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__global__ __launch_bounds__(128) void embbag_fwd_kernel(
    const int32_t* __restrict__ idx, int B, int nnz, const bf16_t* __restrict__ w,
    int64_t w_gstride, const bf16_t* __restrict__ bias, int64_t b_gstride, int N, int act,
    bf16_t* __restrict__ y) {
  const int b = blockIdx.x, g = blockIdx.y;
  const int G = gridDim.y;
  const int32_t* ids = idx + ((int64_t)g * B + b) * nnz;
  const bf16_t* wg = w + g * w_gstride;
  for (int n0 = threadIdx.x * EB_V; n0 < N; n0 += blockDim.x * EB_V) {
    float acc[EB_V];
    ld8(bias + g * b_gstride + n0, acc);
    for (int j = 0; j < nnz; ++j) {
      const int id = ids[j];
      if (id < 0) continue;
      float v[EB_V];
      ld8(wg + (int64_t)id * N + n0, v);
#pragma unroll
      for (int i = 0; i < EB_V; ++i) acc[i] += v[i];
    }
    uint4 o;
    uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int i = 0; i < EB_V / 2; ++i) {
      float a0 = acc[2 * i], a1 = acc[2 * i + 1];
      if (act) {
        a0 = fmaxf(a0, 0.f);
        a1 = fmaxf(a1, 0.f);
      }
      ow[i] = pack_bf2(a0, a1);
    }
    *reinterpret_cast<uint4*>(y + (int64_t)b * G * N + (int64_t)g * N + n0) = o;
  }
}

__global__ __launch_bounds__(128) void embbag_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const int32_t* __restrict__ idx,
    int B, int nnz, float* __restrict__ dw, int64_t dw_gstride, float* __restrict__ db,
    int64_t db_gstride, int N, int act) {
  const int b = blockIdx.x, g = blockIdx.y;
  const int G = gridDim.y;
  const int32_t* ids = idx + ((int64_t)g * B + b) * nnz;
  float* dwg = dw + g * dw_gstride;
  for (int n0 = threadIdx.x * EB_V; n0 < N; n0 += blockDim.x * EB_V) {
    const int64_t off = (int64_t)b * G * N + (int64_t)g * N + n0;
    float d[EB_V], yv[EB_V];
    ld8(dy + off, d);
    if (act) {
      ld8(y + off, yv);
#pragma unroll
      for (int i = 0; i < EB_V; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < EB_V; ++i) atomicAdd(db + g * db_gstride + n0 + i, d[i]);
    for (int j = 0; j < nnz; ++j) {
      const int id = ids[j];
      if (id < 0) continue;
      float* row = dwg + (int64_t)id * N + n0;
#pragma unroll
      for (int i = 0; i < EB_V; ++i) atomicAdd(row + i, d[i]);
    }
  }
}

}  // namespace

CER_API int cer_embbag_fwd(const int32_t* idx, int G, int B, int nnz, const bf16_t* w,
                           int64_t w_gstride, const bf16_t* bias, int64_t b_gstride, int N,
                           int act, bf16_t* y, hipStream_t stream) {
  if (N % EB_V) return (int)hipErrorInvalidValue;
  embbag_fwd_kernel<<<dim3(B, G), 128, 0, stream>>>(idx, B, nnz, w, w_gstride, bias, b_gstride,
                                                    N, act, y);
  return (int)hipGetLastError();
}

// dw / db must be zero on entry
CER_API int cer_embbag_bwd(const bf16_t* dy, const bf16_t* y, const int32_t* idx, int G, int B,
                           int nnz, float* dw, int64_t dw_gstride, float* db, int64_t db_gstride,
                           int N, int act, hipStream_t stream) {
  if (N % EB_V) return (int)hipErrorInvalidValue;
  embbag_bwd_kernel<<<dim3(B, G), 128, 0, stream>>>(dy, y, idx, B, nnz, dw, dw_gstride, db,
                                                    db_gstride, N, act);
  return (int)hipGetLastError();
}
