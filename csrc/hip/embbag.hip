// Embedding-bag first layer of the Criteo MLP: a one-hot
// input row with <= nnz active columns times a dense [K, N] kernel is the sum
// of nnz kernel rows.  idx [G, B, nnz] int32 (-1 = padding), W_g [K, N] bf16 / fp32
// at w + g*w_gstride, bias_g [N].
//   fwd : y[b, g*N + n] = act(bias_g[n] + sum_j W_g[idx[g,b,j], n])
//   bwd : dz = act'(y) * dy ; dW_g[idx, :] += dz (fp32 atomics into the
//         gradient arena, which the optimizer keeps zeroed) ; db_g += sum_b dz
// One block per (b, g); a thread owns 8 consecutive n (16-B row loads).
#include "common.h"

namespace {

constexpr int EB_V = 8;

template <typename T>
__global__ __launch_bounds__(128) void embbag_fwd_kernel(
    const int32_t* __restrict__ idx, int B, int nnz, const T* __restrict__ w,
    int64_t w_gstride, const T* __restrict__ bias, int64_t b_gstride, int N, int act,
    T* __restrict__ y) {
  const int b = blockIdx.x, g = blockIdx.y;
  const int G = gridDim.y;
  const int32_t* ids = idx + ((int64_t)g * B + b) * nnz;
  const T* wg = w + g * w_gstride;
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
    if (act) {
#pragma unroll
      for (int i = 0; i < EB_V; ++i) acc[i] = fmaxf(acc[i], 0.f);
    }
    st8(y + (int64_t)b * G * N + (int64_t)g * N + n0, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(128) void embbag_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ y, const int32_t* __restrict__ idx,
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

template <typename T>
static int embbag_fwd_t(const int32_t* idx, int G, int B, int nnz, const T* w,
                           int64_t w_gstride, const T* bias, int64_t b_gstride, int N,
                           int act, T* y, hipStream_t stream) {
  if (N % EB_V) return (int)hipErrorInvalidValue;
  embbag_fwd_kernel<T><<<dim3(B, G), 128, 0, stream>>>(idx, B, nnz, w, w_gstride, bias, b_gstride,
                                                    N, act, y);
  return (int)hipGetLastError();
}

// dw / db must be zero on entry
template <typename T>
static int embbag_bwd_t(const T* dy, const T* y, const int32_t* idx, int G, int B,
                           int nnz, float* dw, int64_t dw_gstride, float* db, int64_t db_gstride,
                           int N, int act, hipStream_t stream) {
  if (N % EB_V) return (int)hipErrorInvalidValue;
  embbag_bwd_kernel<T><<<dim3(B, G), 128, 0, stream>>>(dy, y, idx, B, nnz, dw, dw_gstride, db,
                                                    db_gstride, N, act);
  return (int)hipGetLastError();
}

#define CER_EMBBAG_ENTRY_POINTS(T, SFX)                                                          \
  CER_API int cer_embbag_fwd##SFX(const int32_t* idx, int G, int B, int nnz, const T* w,        \
                                  int64_t w_gstride, const T* bias, int64_t b_gstride, int N,   \
                                  int act, T* y, hipStream_t stream) {                          \
    return embbag_fwd_t<T>(idx, G, B, nnz, w, w_gstride, bias, b_gstride, N, act, y, stream);   \
  }                                                                                              \
  CER_API int cer_embbag_bwd##SFX(const T* dy, const T* y, const int32_t* idx, int G, int B,    \
                                  int nnz, float* dw, int64_t dw_gstride, float* db,            \
                                  int64_t db_gstride, int N, int act, hipStream_t stream) {     \
    return embbag_bwd_t<T>(dy, y, idx, G, B, nnz, dw, dw_gstride, db, db_gstride, N, act,       \
                           stream);                                                              \
  }

CER_EMBBAG_ENTRY_POINTS(bf16_t, )
CER_EMBBAG_ENTRY_POINTS(float, _f32)
