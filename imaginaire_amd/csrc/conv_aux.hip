// Conv-path helper kernels around k10 / k11 (gfx950).
//
// * conv_weight_flip_t — the stride-1 data gradient of a conv is the forward conv of dy with the
//   spatially flipped, in/out-transposed weight: wt[ci][kh][kw][co] = w[co][KH-1-kh][KW-1-kw][ci]
//   (both channels-last). One pass, a 64 x 64 (co, ci) tile per workgroup and tap staged
//   through LDS: 16-byte coalesced loads along ci, 16-byte coalesced stores along co. Replaces
//   PyTorch's index-based flip kernel followed by a strided channels-last copy (two passes,
//   ~2 ms of a SPADE step on MI355X, profiles/spade_step_op_shapes_mi355x.txt).
// * wgrad_finalize — the k11 weight gradient's epilogue: sums the S fp32 split-K slabs
//   [S][Cout_p][KK][Cin_p], crops the zero-padded channels (odd label counts, RGB) and writes
//   the parameter's dtype in its channels-last layout [Cout][KK][Cin] in the same pass, instead
//   of sum -> slice copy -> dtype-cast copy.
//
// Reference: the reference gets both from cuDNN inside nn.Conv2d's autograd
// (layers/conv.py:59-91); these kernels have no reference counterpart.
#include "common.h"

namespace iamd {
namespace {

constexpr int kT = 256;
constexpr int kTile = 64;
constexpr int kLdsStride = kTile + 2;  // bf16 elements per LDS row (+4 B: conflict-free column reads)

// grid (ceil(Cin/64), ceil(Cout/64), Jy*Jx), block 256. Output tap (jy, jx) of the
// [Cin][Jy][Jx][Cout] result reads source tap (qy + s (Jy-1-jy), qx + s (Jx-1-jx)) of the
// [Cout][KH][KW][Cin] weight (s = 1, q = 0: the plain flip).
__global__ void __launch_bounds__(kT)
flip_t_kernel(const __hip_bfloat16* __restrict__ w, __hip_bfloat16* __restrict__ wt, int Cout,
              int Cin, int KH, int KW, int Jy, int Jx, int s, int qy, int qx) {
  __shared__ __hip_bfloat16 tile[kTile * kLdsStride];
  const int ci0 = blockIdx.x * kTile, co0 = blockIdx.y * kTile, tap = blockIdx.z;
  const int jy = tap / Jx, jx = tap - jy * Jx;
  const int ftap = (qy + s * (Jy - 1 - jy)) * KW + (qx + s * (Jx - 1 - jx));
  const int KK = KH * KW, JJ = Jy * Jx;
  const int tid = threadIdx.x;
  // load: 64 co rows x 8 chunks of 8 ci
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int e = tid + r * kT;
    const int row = e >> 3, ch = e & 7;
    const int co = co0 + row, ci = ci0 + ch * 8;
    Pack<__hip_bfloat16, 8> v;
    if (co < Cout && ci < Cin) {
      v = *reinterpret_cast<const Pack<__hip_bfloat16, 8>*>(
          w + ((int64_t)co * KK + ftap) * Cin + ci);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v.v[k] = __float2bfloat16(0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[row * kLdsStride + ch * 8 + k] = v.v[k];
  }
  __syncthreads();
  // store: 64 ci rows x 8 chunks of 8 co
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int e = tid + r * kT;
    const int row = e >> 3, ch = e & 7;
    const int ci = ci0 + row, co = co0 + ch * 8;
    if (ci >= Cin || co >= Cout) continue;
    Pack<__hip_bfloat16, 8> v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v.v[k] = tile[(ch * 8 + k) * kLdsStride + row];
    *reinterpret_cast<Pack<__hip_bfloat16, 8>*>(wt + ((int64_t)ci * JJ + tap) * Cout + co) = v;
  }
}

// out[co][t][ci] = sum_s part[s][co][t][ci] for co < Cout, ci < Cin (padded slabs: Cop, Cip).
template <typename T, bool VEC>
__global__ void __launch_bounds__(kT)
wgrad_finalize_kernel(const float* __restrict__ part, T* __restrict__ out, int S, int Cop, int Cip,
                      int Cout, int Cin, int KK) {
  const int per = VEC ? Cin / 4 : Cin;
  const int64_t n = (int64_t)Cout * KK * per;
  const int64_t slab = (int64_t)Cop * KK * Cip;
  for (int64_t i = blockIdx.x * (int64_t)kT + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kT) {
    const int c = (int)(i % per);
    const int64_t rt = i / per;  // co * KK + t
    const int t = (int)(rt % KK);
    const int co = (int)(rt / KK);
    const int64_t src = ((int64_t)co * KK + t) * Cip + (VEC ? c * 4 : c);
    if constexpr (VEC) {
      float4 acc = *reinterpret_cast<const float4*>(part + src);
      for (int s = 1; s < S; ++s) {
        const float4 v = *reinterpret_cast<const float4*>(part + s * slab + src);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      const float a[4] = {acc.x, acc.y, acc.z, acc.w};
      T* o = out + rt * Cin + c * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = from_f<T>(a[k]);
    } else {
      float acc = part[src];
      for (int s = 1; s < S; ++s) acc += part[s * slab + src];
      out[rt * Cin + c] = from_f<T>(acc);
    }
  }
}

}  // namespace

// w: [Cout, Cin, KH, KW] bf16 channels-last -> [Cin, Cout, Jy, Jx] bf16 channels-last with
// wt[ci][jy][jx][co] = w[co][qy + s (Jy-1-jy)][qx + s (Jx-1-jx)][ci], Jy = ceil((KH-qy)/s)
// (s = 1, q = 0: the spatially flipped, in/out-transposed weight of the stride-1 dgrad).
at::Tensor conv_weight_flip_t(const at::Tensor& w, int64_t s, int64_t qy, int64_t qx) {
  IAMD_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kBFloat16,
             "conv_weight_flip_t: 4-D bf16 CUDA weight expected");
  IAMD_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv_weight_flip_t: packed channels-last weight expected");
  const int Cout = (int)w.size(0), Cin = (int)w.size(1), KH = (int)w.size(2), KW = (int)w.size(3);
  IAMD_CHECK(Cout % 8 == 0 && Cin % 8 == 0, "conv_weight_flip_t: channels must be multiples of 8");
  IAMD_CHECK(s >= 1 && qy >= 0 && qx >= 0 && qy < KH && qx < KW, "conv_weight_flip_t: bad phase");
  const int Jy = (int)((KH - qy + s - 1) / s), Jx = (int)((KW - qx + s - 1) / s);
  auto wt = at::empty({Cin, Cout, Jy, Jx}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (wt.numel() == 0) return wt;
  const dim3 grid(ceil_div(Cin, kTile), ceil_div(Cout, kTile), Jy * Jx);
  hipLaunchKernelGGL(flip_t_kernel, grid, dim3(kT), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(w.data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(wt.data_ptr()), Cout, Cin, KH, KW, Jy, Jx,
                     (int)s, (int)qy, (int)qx);
  IAMD_LAUNCH_CHECK();
  return wt;
}

// part: fp32 [S * Cop * KK * Cip] -> [Cout, Cin, KH, KW] channels-last in `dtype`.
at::Tensor wgrad_finalize(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                          int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                          at::ScalarType dtype) {
  IAMD_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous(),
             "wgrad_finalize: contiguous fp32 slabs expected");
  IAMD_CHECK(part.numel() >= S * Cop * KH * KW * Cip && Cout <= Cop && Cin <= Cip,
             "wgrad_finalize: slab shape");
  auto out = at::empty({Cout, Cin, KH, KW},
                       part.options().dtype(dtype).memory_format(at::MemoryFormat::ChannelsLast));
  const int KK = (int)(KH * KW);
  const bool vec = Cin % 4 == 0 && Cip % 4 == 0;
  const int64_t n = Cout * KK * (vec ? Cin / 4 : Cin);
  if (n == 0) return out;
  const int blocks = (int)std::min<int64_t>((n + kT - 1) / kT, 8192);
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    if (vec)
      hipLaunchKernelGGL((wgrad_finalize_kernel<T, true>), dim3(blocks), dim3(kT), 0, stream(),
                         part.data_ptr<float>(), reinterpret_cast<T*>(out.data_ptr()), (int)S,
                         (int)Cop, (int)Cip, (int)Cout, (int)Cin, KK);
    else
      hipLaunchKernelGGL((wgrad_finalize_kernel<T, false>), dim3(blocks), dim3(kT), 0, stream(),
                         part.data_ptr<float>(), reinterpret_cast<T*>(out.data_ptr()), (int)S,
                         (int)Cop, (int)Cip, (int)Cout, (int)Cin, KK);
  };
  if (dtype == at::kBFloat16) launch(__hip_bfloat16());
  else if (dtype == at::kFloat) launch(float());
  else IAMD_CHECK(false, "wgrad_finalize: bf16 or fp32 output expected");
  IAMD_LAUNCH_CHECK();
  return out;
}

}  // namespace iamd
