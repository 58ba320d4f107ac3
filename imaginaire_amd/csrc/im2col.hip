// Tap-packed operands for thin-input convolutions (Cin <= 16: RGB / RGB+mask / flow inputs).
//
// A 7x7 stem on a 3-channel image run as an implicit GEMM pads every filter tap's 3 channels
// to a 64-deep k-chunk: 49 k-steps of which 95% are zeros (MUNIT / FUNIT / pix2pixHD stems,
// ~0.5 ms per call at 256x256 x 16, profiles/recipe_munit256_conv_log_mi355x.txt). Packing the
// taps instead makes K = KH * KW * Cin (147 -> 192 padded: 3 k-steps): im2col_pack writes the
// [M][Kp] operand once (k = (ky * KW + kx) * Cin + ci, zeros for padding pixels and k >= K),
// the conv is then a 1x1 k10 GEMM and its weight gradient a 1x1 k11 GEMM on the same operand.
// (The packing's adjoint — a [M][Kp] dcol GEMM gathered back per input pixel — ran at ~12 TF/s
// on its 2-byte gathers, so the data gradient stays on the k10 dgrad: ops/conv.py.) The same
// packing of an output gradient serves the thin-OUTPUT convs (RGB heads, Cout <= 16): dx and dW
// both as 1x1 GEMMs of the packed dy (ops/conv.py _thin_output_grads).
// Reference: the convolutions of /root/reference/imaginaire/layers/conv.py:59-91.
#include "common.h"

namespace iamd {
namespace {

struct PackGeom {
  int B, Cin, H, W, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, K, Kp;
  int64_t sb, sc, sy, sx;  // element strides of x / dx (any layout)
};

// one thread per (output pixel, 8-wide k chunk): 16-byte stores, gathered loads (the thin input
// is small and L2-resident)
template <typename T>
__global__ void __launch_bounds__(256) im2col_pack_kernel(const T* __restrict__ x,
                                                          __hip_bfloat16* __restrict__ col,
                                                          PackGeom g) {
  const int nch = g.Kp / 8;
  const int64_t total = (int64_t)g.B * g.Ho * g.Wo * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % nch);
    const int64_t m = i / nch;
    const int ow = (int)(m % g.Wo);
    const int64_t t = m / g.Wo;
    const int oh = (int)(t % g.Ho), b = (int)(t / g.Ho);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = c * 8 + e;
      v[e] = 0.f;
      if (k < g.K) {
        const int tap = k / g.Cin, ci = k - tap * g.Cin;
        const int ky = tap / g.KW, kx = tap - ky * g.KW;
        const int ih = oh * g.sh - g.ph + ky * g.dh, iw = ow * g.sw - g.pw + kx * g.dw;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          v[e] = to_f<T>(x[b * g.sb + ci * g.sc + ih * g.sy + iw * g.sx]);
      }
    }
    store_vec<__hip_bfloat16, 8>(col + m * g.Kp + c * 8, v);
  }
}

PackGeom make_geom(int B, int Cin, int H, int W, int64_t KH, int64_t KW, int64_t sh, int64_t sw,
                   int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t Kp) {
  PackGeom g;
  g.B = B; g.Cin = Cin; g.H = H; g.W = W;
  g.KH = (int)KH; g.KW = (int)KW; g.sh = (int)sh; g.sw = (int)sw;
  g.ph = (int)ph; g.pw = (int)pw; g.dh = (int)dh; g.dw = (int)dw;
  g.Ho = (int)((H + 2 * ph - dh * (KH - 1) - 1) / sh + 1);
  g.Wo = (int)((W + 2 * pw - dw * (KW - 1) - 1) / sw + 1);
  g.K = (int)(KH * KW * Cin);
  g.Kp = (int)Kp;
  return g;
}

int grid_for(int64_t total) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 65536));
}

}  // namespace

// x [B, Cin, H, W] (fp32 / bf16, any layout), Cin <= 16 -> col [B, Kp, Ho, Wo] channels-last
// bf16 with col[m][(ky * KW + kx) * Cin + ci] = x[b, ci, oh*sh - ph + ky*dh, ow*sw - pw + kx*dw]
at::Tensor im2col_pack(const at::Tensor& x, int64_t KH, int64_t KW, int64_t sh, int64_t sw,
                       int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t Kp) {
  IAMD_CHECK(x.is_cuda() && x.dim() == 4, "im2col_pack: 4-D CUDA tensor expected");
  IAMD_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16,
             "im2col_pack: fp32 / bf16 input");
  const int B = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  IAMD_CHECK(Cin >= 1 && Cin <= 16, "im2col_pack: Cin must be 1..16");
  IAMD_CHECK(Kp % 64 == 0 && Kp >= KH * KW * Cin && sh >= 1 && sw >= 1 && dh >= 1 && dw >= 1,
             "im2col_pack: bad geometry");
  PackGeom g = make_geom(B, Cin, H, W, KH, KW, sh, sw, ph, pw, dh, dw, Kp);
  IAMD_CHECK(g.Ho > 0 && g.Wo > 0, "im2col_pack: empty output");
  g.sb = x.stride(0); g.sc = x.stride(1); g.sy = x.stride(2); g.sx = x.stride(3);
  auto col = at::empty({B, Kp, g.Ho, g.Wo},
                       x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = (int64_t)B * g.Ho * g.Wo * (Kp / 8);
  if (x.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(im2col_pack_kernel<float>, dim3(grid_for(total)), dim3(256), 0, stream(),
                       x.data_ptr<float>(), reinterpret_cast<__hip_bfloat16*>(col.data_ptr()), g);
  else
    hipLaunchKernelGGL(im2col_pack_kernel<__hip_bfloat16>, dim3(grid_for(total)), dim3(256), 0,
                       stream(), reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(col.data_ptr()), g);
  IAMD_LAUNCH_CHECK();
  return col;
}

}  // namespace iamd
