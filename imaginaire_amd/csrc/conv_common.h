// Shared pieces of the k10 implicit-GEMM convolution kernels (conv_mfma.hip: v1-v5 tiles,
// conv_rw.hip: the generalised row-window tile): operand types, the launch argument block,
// the bias / activation / residual epilogue store and the split-K reduction.
#pragma once

#include "common.h"

namespace iamd {

struct ConvArgs {
  const __hip_bfloat16* x;
  const __hip_bfloat16* w;
  const float* bias;
  __hip_bfloat16* y;
  int xbytes, wbytes;
  int H, W, Cin, Ho, Wo, Cout;
  int KH, KW, sh, sw, ph, pw, dh, dw;
  int M, nk, cpt, nNt;
  int kps;          // k-steps per split (split-K: blockIdx.y = split)
  float* part;      // split-K fp32 partial slabs [S][M][Cout] (nullptr: direct epilogue)
  float slope;
  // output-pixel mapping (phase-decomposed stride-2 data gradient): GEMM row m = (b, oh, ow)
  // is stored at pixel (b, oh * osy + ory, ow * osx + orx) of a [B, oH, oW, Cout] tensor.
  // omode 0: identity (row m is pixel m)
  int omode, oH, oW, osy, osx, ory, orx;
  // batch of independent convs (per-sample weights: the fs-vid2vid hyper convolutions), one per
  // blockIdx.z: operand / output / bias strides in elements between samples (v1 kernel only)
  int64_t xbs, wbs, ybs;
  int bbs, nz;
  // channels stored per output pixel = row stride of y (<= Cout, a multiple of 8): the padded
  // output channels of a Cout % 64 != 0 conv are never written, so no crop copy follows
  int ldy;
  // residual added after the activation, same layout as y (nullptr: none): the shortcut of a
  // residual block whose branch ends in this conv (reference layers/residual.py:150
  // ``x_shortcut + dx``) lands in the epilogue instead of a separate full-tensor add
  const __hip_bfloat16* res;
  // spectrally normalised weight (layers/spectral_norm.py): the operand w is bf16(W) and the
  // epilogue scales the accumulator by 1 / *ascale (sigma, a device scalar written by the power
  // iteration in the same graph) before the bias: conv(x, W / sigma) without a W / sigma copy.
  // nullptr: no scale.
  const float* ascale = nullptr;
  // row-window tile geometry (conv_rw.hip): GEMM rows are "virtual" output pixels — segments of
  // SW consecutive pixels of one output row (nct segments per row, the last one masked past
  // Wo); nseg = B * Ho * nct segments; P = LDS window rows per segment, Ph = rows of the
  // even-column half of a stride-2 window
  int SW = 0, nct = 1, nseg = 0, P = 0, Ph = 0;
};

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) bf16x4* lds_bf16x4_t;

constexpr int kBK = 64;
constexpr int kRowBytes = kBK * 2;  // 128 B per staged row
constexpr int kEpiStride = 272;     // epilogue LDS row stride in bytes (BN<=128 bf16 + 16 pad)

// buffer-resource word 3 for raw (unformatted, stride-0) buffers on gfx9-family parts
constexpr int kBufCfg = 0x00020000;
// a byte offset past every tensor this kernel accepts (< 2^31 bytes): the buffer unit
// returns zeros for it
constexpr int kOobOffset = 0x7ffffff0;


__device__ __forceinline__ float ascale_of(const ConvArgs& a) {
  return a.ascale ? 1.f / a.ascale[0] : 1.f;
}

// y[off .. off + 8) = v (+ res[off .. off + 8) when the conv carries a residual), one 16-byte
// store. The residual is added to the bf16-rounded conv output and rounded again: the same
// two roundings as the unfused bf16 conv followed by a bf16 add.
__device__ __forceinline__ void store_chunk(const ConvArgs& a, __hip_bfloat16* y, size_t off,
                                            uint4 v) {
  if (a.res) {
    const uint4 r = *reinterpret_cast<const uint4*>(a.res + off);
    const uint32_t* pv = reinterpret_cast<const uint32_t*>(&v);
    const uint32_t* pr = reinterpret_cast<const uint32_t*>(&r);
    uint4 o;
    uint32_t* po = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(pv[k] << 16) + __uint_as_float(pr[k] << 16);
      const float hi = __uint_as_float(pv[k] & 0xffff0000u) + __uint_as_float(pr[k] & 0xffff0000u);
      const __hip_bfloat16 blo = __float2bfloat16(lo), bhi = __float2bfloat16(hi);
      po[k] = (uint32_t)(*reinterpret_cast<const uint16_t*>(&blo)) |
              ((uint32_t)(*reinterpret_cast<const uint16_t*>(&bhi)) << 16);
    }
    v = o;
  }
  *reinterpret_cast<uint4*>(y + off) = v;
}

// destination pixel (row of the NHWC output) of GEMM row m
__device__ __forceinline__ size_t out_row(const ConvArgs& a, int m) {
  if (!a.omode) return (size_t)m;
  const int HoWo = a.Ho * a.Wo;
  const int b = m / HoWo, r = m - b * HoWo;
  const int oh = r / a.Wo, ow = r - oh * a.Wo;
  return ((size_t)b * a.oH + oh * a.osy + a.ory) * a.oW + ow * a.osx + a.orx;
}

// y = act(sum_s part[s] + bias) in bf16, 8 channels per thread.
__global__ void __launch_bounds__(256)
conv_splitk_reduce(const float* __restrict__ part, const float* __restrict__ bias,
                   __hip_bfloat16* __restrict__ y, int S, int64_t MC, int C, float slope,
                   ConvArgs map) {
  const float asc = ascale_of(map);
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < MC / 8;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;
    float acc[8];
    const float4* p = reinterpret_cast<const float4*>(part + e);
    float4 lo = p[0], hi = p[1];
    acc[0] = lo.x; acc[1] = lo.y; acc[2] = lo.z; acc[3] = lo.w;
    acc[4] = hi.x; acc[5] = hi.y; acc[6] = hi.z; acc[7] = hi.w;
    for (int s = 1; s < S; ++s) {
      const float4* q = reinterpret_cast<const float4*>(part + (int64_t)s * MC + e);
      lo = q[0]; hi = q[1];
      acc[0] += lo.x; acc[1] += lo.y; acc[2] += lo.z; acc[3] += lo.w;
      acc[4] += hi.x; acc[5] += hi.y; acc[6] += hi.z; acc[7] += hi.w;
    }
    const int c = (int)(e % C);
    if (c >= map.ldy) continue;  // padded output channels are not stored
    const int zb = (int)(e / ((int64_t)map.M * C));  // sample of a batched launch
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = fmaf(acc[k], asc, bias ? bias[zb * map.bbs + c + k] : 0.f);
      acc[k] = t > 0.f ? t : t * slope;
    }
    const int64_t m = e / C - (int64_t)zb * map.M;
    const size_t off = (size_t)zb * map.ybs + out_row(map, (int)m) * map.ldy + c;
    if (map.res) {  // (bf16 conv output + residual, as store_chunk)
      float r[8];
      load_vec<__hip_bfloat16, 8>(map.res + off, r);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __bfloat162float(__float2bfloat16(acc[k])) + r[k];
    }
    store_vec<__hip_bfloat16, 8>(y + off, acc);
  }
}

}  // namespace

// Row-window k10 for the shapes the v4 / v5 tiles do not take (stride 2, 1x1 / 4x4 / 7x7
// filters, Cout = 64, Cin = 32, output rows of any width): conv_rw.hip. Launches and returns
// true when the shape is eligible (IMAGINAIRE_AMD_CONV_RW != 0), else launches nothing.
bool run_rw(ConvArgs& a, const at::Tensor& x, bool forced);
bool rw_eligible(const ConvArgs& a);
// the narrow row-window variant is switched on for this shape (IMAGINAIRE_AMD_CONV_RW_SMALL=1)
bool rw_small_pref(const ConvArgs& a);
}  // namespace iamd
