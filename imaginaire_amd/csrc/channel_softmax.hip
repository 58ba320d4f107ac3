// k15: softmax over the channels of an NHWC (channels-last) activation, forward and backward.
//
// Few-shot vid2vid's reference encoder (reference generators/fs_vid2vid.py:780-788,
// ``mul_ref_label``) normalises every encoded reference-label map with softmax(dim=1) before
// pooling the image features with it. On a channels-last tensor dim 1 is the innermost,
// contiguous one, but PyTorch treats dim=1 softmax as a "spatial" softmax and walks it with a
// strided per-channel kernel (cunn_SpatialSoftMaxForward: 25 ms per 5 recipe iterations,
// profiles/recipe_fsvid2vid512_kernels_mi355x.txt). Here every pixel's C channels are one
// contiguous row: a group of G lanes (G = min(64, C / 8)) owns a row, each lane loads 16-byte
// bf16 chunks, the max / sum reductions stay inside the group (__shfl_xor over G lanes), and
// the row is written back with 16-byte stores — one read and one write of the tensor, fp32
// arithmetic.
//   forward : y = exp(x - max) / sum
//   backward: dx = y * (dy - sum(dy * y))
#include "common.h"

namespace iamd {
namespace {

constexpr int kT = 256;

template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// G lanes per row, NC = C / (8 G) 16-byte chunks per lane (compile-time: registers)
template <int G, int NC>
__global__ void __launch_bounds__(kT) csm_fwd(const __hip_bfloat16* __restrict__ x,
                                              __hip_bfloat16* __restrict__ y, int64_t rows,
                                              int C) {
  constexpr int kRowsPerBlock = kT / G;
  const int gl = threadIdx.x % G;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / G;
  if (row >= rows) return;
  const __hip_bfloat16* xr = x + row * C;
  float v[NC][8];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    load_vec<__hip_bfloat16, 8>(xr + (c * G + gl) * 8, v[c]);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, v[c][k]);
  }
  m = group_max<G>(m);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[c][k] = __expf(v[c][k] - m);
      s += v[c][k];
    }
  const float inv = 1.f / group_sum<G>(s);
  __hip_bfloat16* yr = y + row * C;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[c][k] *= inv;
    store_vec<__hip_bfloat16, 8>(yr + (c * G + gl) * 8, v[c]);
  }
}

template <int G, int NC>
__global__ void __launch_bounds__(kT) csm_bwd(const __hip_bfloat16* __restrict__ y,
                                              const __hip_bfloat16* __restrict__ dy,
                                              __hip_bfloat16* __restrict__ dx, int64_t rows,
                                              int C) {
  constexpr int kRowsPerBlock = kT / G;
  const int gl = threadIdx.x % G;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / G;
  if (row >= rows) return;
  float yv[NC][8], gv[NC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    load_vec<__hip_bfloat16, 8>(y + row * C + (c * G + gl) * 8, yv[c]);
    load_vec<__hip_bfloat16, 8>(dy + row * C + (c * G + gl) * 8, gv[c]);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += yv[c][k] * gv[c][k];
  }
  s = group_sum<G>(s);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[c][k] = yv[c][k] * (gv[c][k] - s);
    store_vec<__hip_bfloat16, 8>(dx + row * C + (c * G + gl) * 8, gv[c]);
  }
}

void check_csm(const at::Tensor& t, const char* what) {
  IAMD_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 &&
                 t.is_contiguous(at::MemoryFormat::ChannelsLast),
             what, ": packed channels-last bf16 4-D tensor expected");
  const int64_t C = t.size(1);
  IAMD_CHECK(C >= 16 && C <= 4096 && (C & (C - 1)) == 0,
             what, ": channel count must be a power of two in [16, 4096], got ", C);
}

// launch for C = 8 * G * NC: G = min(64, C / 8) lanes per row, NC <= 8 chunks per lane
template <typename F>
void dispatch_c(int C, F&& f) {
  switch (C) {
    case 16: f(std::integral_constant<int, 2>(), std::integral_constant<int, 1>()); break;
    case 32: f(std::integral_constant<int, 4>(), std::integral_constant<int, 1>()); break;
    case 64: f(std::integral_constant<int, 8>(), std::integral_constant<int, 1>()); break;
    case 128: f(std::integral_constant<int, 16>(), std::integral_constant<int, 1>()); break;
    case 256: f(std::integral_constant<int, 32>(), std::integral_constant<int, 1>()); break;
    case 512: f(std::integral_constant<int, 64>(), std::integral_constant<int, 1>()); break;
    case 1024: f(std::integral_constant<int, 64>(), std::integral_constant<int, 2>()); break;
    case 2048: f(std::integral_constant<int, 64>(), std::integral_constant<int, 4>()); break;
    default: f(std::integral_constant<int, 64>(), std::integral_constant<int, 8>()); break;
  }
}

}  // namespace

at::Tensor channel_softmax_fwd(const at::Tensor& x) {
  check_csm(x, "channel_softmax_fwd");
  auto y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int C = (int)x.size(1);
  const int64_t rows = x.numel() / C;
  if (rows == 0) return y;
  dispatch_c(C, [&](auto gv, auto ncv) {
    constexpr int G = decltype(gv)::value, NC = decltype(ncv)::value;
    const int64_t blocks = (rows + kT / G - 1) / (kT / G);
    hipLaunchKernelGGL((csm_fwd<G, NC>), dim3((unsigned)blocks), dim3(kT), 0, stream(),
                       reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(y.data_ptr()), rows, C);
  });
  IAMD_LAUNCH_CHECK();
  return y;
}

at::Tensor channel_softmax_bwd(const at::Tensor& y, const at::Tensor& dy) {
  check_csm(y, "channel_softmax_bwd");
  check_csm(dy, "channel_softmax_bwd");
  IAMD_CHECK(y.sizes() == dy.sizes(), "channel_softmax_bwd: shape mismatch");
  auto dx = at::empty_like(y, y.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int C = (int)y.size(1);
  const int64_t rows = y.numel() / C;
  if (rows == 0) return dx;
  dispatch_c(C, [&](auto gv, auto ncv) {
    constexpr int G = decltype(gv)::value, NC = decltype(ncv)::value;
    const int64_t blocks = (rows + kT / G - 1) / (kT / G);
    hipLaunchKernelGGL((csm_bwd<G, NC>), dim3((unsigned)blocks), dim3(kT), 0, stream(),
                       reinterpret_cast<const __hip_bfloat16*>(y.data_ptr()),
                       reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(dx.data_ptr()), rows, C);
  });
  IAMD_LAUNCH_CHECK();
  return dx;
}

}  // namespace iamd
