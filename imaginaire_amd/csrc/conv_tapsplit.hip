// Tap-split convolution for narrow-output heads (gfx950).
//
// The image heads of the generators — SPADE conv_img (256 -> 3, 5x5 at 256x512,
// reference generators/spade.py:240-262), pix2pixHD / vid2vid 7x7 -> 3 — have Cout <= 8.
// As an implicit GEMM their N dimension is 3: a 64-wide MFMA tile wastes 95% of its columns
// and, worse, streams the whole KH*KW*Cin im2col A operand for 3 outputs per pixel (k10 ran
// conv_img at 267 "padded" TF/s = 25 real TF/s, profiles/spade_step_conv_log_mi355x.txt).
//
// Re-associated instead:
//     Z[p, t*Cout + c] = sum_ci x[p, ci] * W[c, ci, t]          (1x1 conv: k10 MFMA GEMM,
//                                                               N = KH*KW*Cout padded to 64)
//     y[o, c]          = bias[c] + sum_t Z[o + off(t), t*Cout + c]   (conv_tap_sum, here)
// so every input element is read once by an MFMA tile of useful width, and the spatial taps
// become a cheap gather-sum over a [pixels, KH*KW*Cout] bf16 tensor.
// Backward:  dZ[q, t*Cout + c] = dy[q - off(t), c]  (conv_tap_gather, here), then
//     dx = dZ (1x1 conv) W_z^T  (k10),   dW_z = dZ^T x  (k11 1x1 weight gradient).
// Stride 1, any padding / dilation. NHWC bf16 everywhere; fp32 accumulation.
#include "common.h"

namespace iamd {
namespace {

constexpr int kT = 256;
constexpr int kMaxCout = 8;

// Workgroup = a tile of R output rows x kTW output columns of one image. Filter row kh only
// touches the KW*Cout partial channels [kh*KW*Cout, (kh+1)*KW*Cout) of input row
// ho - ph + kh*dh, so for each kh the tile stages exactly those channel segments of R input
// rows x (kTW + (KW-1)*dw) columns in LDS (lane-contiguous 2-byte reads along each pixel's
// segment) and then sums the KW taps out of LDS: every partial is fetched from memory once
// (plus the column halo), instead of one 128-byte line per 6 useful bytes.
constexpr int kTW = 64;

__global__ void __launch_bounds__(kT)
tap_sum_kernel(const __hip_bfloat16* __restrict__ z, const float* __restrict__ bias,
               __hip_bfloat16* __restrict__ y, int H, int W, int Cz, int Ho, int Wo, int Cout,
               int KH, int KW, int ph, int pw, int dh, int dw, int R) {
  extern __shared__ __hip_bfloat16 seg_lds[];
  const int seg = KW * Cout, ncols = kTW + (KW - 1) * dw;
  const int wo0 = blockIdx.x * kTW, ho0 = blockIdx.y * R, b = blockIdx.z;
  const int tid = threadIdx.x;
  const int nout = R * kTW;          // <= 2 * kT (host guarantees R <= 8)
  float acc[2][kMaxCout];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int c = 0; c < kMaxCout; ++c) acc[o][c] = 0.f;
  const __hip_bfloat16* zb = z + (int64_t)b * H * W * Cz;
  const int nld = R * ncols * seg;
  for (int kh = 0; kh < KH; ++kh) {
    __syncthreads();
    for (int e = tid; e < nld; e += kT) {
      const int r = e / (ncols * seg);
      const int rem = e - r * ncols * seg;
      const int col = rem / seg, ch = rem - col * seg;
      const int hi = ho0 + r - ph + kh * dh, wi = wo0 - pw + col;
      __hip_bfloat16 v = __float2bfloat16(0.f);
      if (hi >= 0 && hi < H && wi >= 0 && wi < W)
        v = zb[((int64_t)hi * W + wi) * Cz + kh * seg + ch];
      seg_lds[e] = v;
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const int idx = tid + o * kT;
      if (idx >= nout) continue;
      const int r = idx / kTW, col = idx - r * kTW;
      const __hip_bfloat16* row = seg_lds + (r * ncols + col) * seg;
      for (int kw = 0; kw < KW; ++kw) {
        const __hip_bfloat16* p = row + kw * dw * seg + kw * Cout;
#pragma unroll
        for (int c = 0; c < kMaxCout; ++c)
          if (c < Cout) acc[o][c] += __bfloat162float(p[c]);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int idx = tid + o * kT;
    if (idx >= nout) continue;
    const int r = idx / kTW, col = idx - r * kTW;
    const int ho = ho0 + r, wo = wo0 + col;
    if (ho >= Ho || wo >= Wo) continue;
    __hip_bfloat16* yp = y + (((int64_t)b * Ho + ho) * Wo + wo) * Cout;
#pragma unroll
    for (int c = 0; c < kMaxCout; ++c)
      if (c < Cout) yp[c] = __float2bfloat16(acc[o][c] + (bias != nullptr ? bias[c] : 0.f));
  }
}

// one thread per (input pixel, 8-channel chunk of Z): dZ[q, t*Cout + c] = dy[q - off(t), c],
// zero for padded channels and for taps whose output pixel falls outside the output. The
// per-channel (row offset, column offset, output channel) table is built once per workgroup
// in LDS (no integer divisions in the element loop); consecutive lanes write consecutive
// 16-byte chunks of a pixel's dZ row.
constexpr int kMaxCz = 512;

__global__ void __launch_bounds__(kT)
tap_gather_kernel(const __hip_bfloat16* __restrict__ dy, __hip_bfloat16* __restrict__ dz, int B,
                  int H, int W, int Cz, int Ho, int Wo, int Cout, int KH, int KW, int ph, int pw,
                  int dh, int dw) {
  __shared__ int tab[kMaxCz][3];
  const int real = KH * KW * Cout;
  for (int j = threadIdx.x; j < Cz; j += kT) {
    if (j < real) {
      const int t = j / Cout, c = j - t * Cout;
      const int kh = t / KW, kw = t - kh * KW;
      tab[j][0] = ph - kh * dh;
      tab[j][1] = pw - kw * dw;
      tab[j][2] = c;
    } else {
      tab[j][0] = 0; tab[j][1] = 0; tab[j][2] = -1;
    }
  }
  __syncthreads();
  const int chunks = Cz / 8;
  const int64_t total = (int64_t)B * H * W * chunks;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kT) {
    const int ch = (int)(i % chunks);
    const int64_t q = i / chunks;  // input pixel (b, hi, wi)
    const int wi = (int)(q % W);
    const int64_t r = q / W;
    const int hi = (int)(r % H), b = (int)(r / H);
    const __hip_bfloat16* dyb = dy + (int64_t)b * Ho * Wo * Cout;
    Pack<__hip_bfloat16, 8> v;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = ch * 8 + k;
      const int ho = hi + tab[j][0], wo = wi + tab[j][1], c = tab[j][2];
      __hip_bfloat16 val = __float2bfloat16(0.f);
      if (c >= 0 && ho >= 0 && ho < Ho && wo >= 0 && wo < Wo)
        val = dyb[((int64_t)ho * Wo + wo) * Cout + c];
      v.v[k] = val;
    }
    *reinterpret_cast<Pack<__hip_bfloat16, 8>*>(dz + q * Cz + ch * 8) = v;
  }
}

int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + kT - 1) / kT, 16384));
}

void check_geometry(int H, int W, int Ho, int Wo, int KH, int KW, int ph, int pw, int dh, int dw) {
  IAMD_CHECK(Ho == H + 2 * ph - dh * (KH - 1) && Wo == W + 2 * pw - dw * (KW - 1),
             "tap-split conv: output size does not match a stride-1 conv");
}

}  // namespace

// z [B, Cz, H, W] channels-last bf16 (Cz >= KH*KW*Cout) -> y [B, Cout, Ho, Wo] channels-last bf16
at::Tensor conv_tap_sum(const at::Tensor& z, const c10::optional<at::Tensor>& bias, int64_t Cout,
                        int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  IAMD_CHECK(z.is_cuda() && z.scalar_type() == at::kBFloat16 && z.dim() == 4 &&
                 z.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv_tap_sum: packed channels-last bf16 partials expected");
  IAMD_CHECK(Cout >= 1 && Cout <= kMaxCout && KH * KW * Cout <= z.size(1),
             "conv_tap_sum: Cout must be 1..8 and KH*KW*Cout <= Cz");
  const int B = (int)z.size(0), Cz = (int)z.size(1), H = (int)z.size(2), W = (int)z.size(3);
  const int Ho = (int)(H + 2 * ph - dh * (KH - 1)), Wo = (int)(W + 2 * pw - dw * (KW - 1));
  IAMD_CHECK(Ho > 0 && Wo > 0, "conv_tap_sum: empty output");
  auto y = at::empty({B, Cout, Ho, Wo}, z.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor bf;
  if (bias.has_value() && bias->defined()) {
    IAMD_CHECK(bias->numel() == Cout, "conv_tap_sum: bias size");
    bf = bias->to(at::kFloat).contiguous();
  }
  // R output rows per tile: <= 8 (two outputs per thread), LDS segment buffer <= 48 KB
  const int64_t row_bytes = (int64_t)(kTW + (KW - 1) * dw) * KW * Cout * 2;
  const int R = (int)std::max<int64_t>(1, std::min<int64_t>(8, (48 << 10) / row_bytes));
  IAMD_CHECK(R * row_bytes <= (64 << 10), "conv_tap_sum: filter too wide for the LDS tile");
  IAMD_CHECK(B <= 65535, "conv_tap_sum: batch too large");
  dim3 grid((Wo + kTW - 1) / kTW, (Ho + R - 1) / R, B);
  hipLaunchKernelGGL(tap_sum_kernel, grid, dim3(kT), (size_t)(R * row_bytes), stream(),
                     reinterpret_cast<const __hip_bfloat16*>(z.data_ptr()),
                     bf.defined() ? bf.data_ptr<float>() : nullptr,
                     reinterpret_cast<__hip_bfloat16*>(y.data_ptr()), H, W, Cz, Ho, Wo,
                     (int)Cout, (int)KH, (int)KW, (int)ph, (int)pw, (int)dh, (int)dw, R);
  IAMD_LAUNCH_CHECK();
  return y;
}

// dy [B, Cout, Ho, Wo] bf16 -> dZ [B, Cz, H, W] channels-last bf16 (Cz % 8 == 0)
at::Tensor conv_tap_gather(const at::Tensor& dy, int64_t Cz, int64_t KH, int64_t KW, int64_t ph,
                           int64_t pw, int64_t dh, int64_t dw, int64_t H, int64_t W) {
  IAMD_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4,
             "conv_tap_gather: 4-D bf16 gradient expected");
  const int B = (int)dy.size(0), Cout = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  IAMD_CHECK(Cz % 8 == 0 && Cz <= kMaxCz && KH * KW * Cout <= Cz, "conv_tap_gather: Cz");
  check_geometry((int)H, (int)W, Ho, Wo, (int)KH, (int)KW, (int)ph, (int)pw, (int)dh, (int)dw);
  auto g = dy.contiguous(at::MemoryFormat::ChannelsLast);
  auto dz = at::empty({B, Cz, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  hipLaunchKernelGGL(tap_gather_kernel, dim3(grid_for((int64_t)B * H * W * (Cz / 8))), dim3(kT), 0,
                     stream(), reinterpret_cast<const __hip_bfloat16*>(g.data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(dz.data_ptr()), B, (int)H, (int)W, (int)Cz,
                     Ho, Wo, Cout, (int)KH, (int)KW, (int)ph, (int)pw, (int)dh, (int)dw);
  IAMD_LAUNCH_CHECK();
  return dz;
}

}  // namespace iamd
