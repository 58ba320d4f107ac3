// k6 FlowNet cost-volume correlation and k8 channel-norm, gfx950.
//
// Semantics follow reference third_party/correlation/src/correlation_cuda_kernel.cu:73-334
// (zero-padded inputs, output channel tc = (tj+R)*(2R+1) + (ti+R), value averaged over
// kernel_size^2 * C) and third_party/channelnorm/src/channelnorm_kernel.cu:19-96
// (L2 norm over channels, grad = g*x/(norm+1e-9)).
//
// MI355X design:
//   * Inputs are NHWC (channels-last), the layout every conv in the framework produces,
//     so a pixel's feature vector is one contiguous, 16-byte-vectorisable run.
//   * The kernel_size==1 forward (the only configuration FlowNet2 uses: pad 20,
//     max_disp 20, stride2 2 -> 21x21 = 441 displacements) is LDS-tiled: one workgroup
//     owns 32 output pixels of one output row and one displacement row tj. It stages the
//     32 first-image feature vectors and the (31*s1 + 2R*s2 + 1)-wide second-image strip
//     through LDS in 32-channel chunks (rows padded to 33 floats -> conflict-free), and
//     each lane accumulates up to 3 displacements for its pixel in fp32 registers.
//     Every input element is read from HBM once per displacement row instead of once
//     per displacement (21x fewer global reads than the per-pixel reference kernel).
//   * bf16 inputs with C % 32 == 0 (FlowNetC's 256-channel conv3 features) take the MFMA
//     forward corr_fwd_mfma: a parity-split banded 16x48 v_mfma_f32_16x16x32_bf16 product per
//     (row, displacement row, 16*stride2 pixels), fragments loaded straight from NHWC rows.
//   * Backward is gather-form, no atomics, deterministic. kernel_size 1 / stride1 1 (FlowNetC):
//     corr_bwd_k1 stages, per (image row, displacement row), the two strips and grad_out rows the
//     row's input gradients read in LDS and accumulates from there; other configurations use
//     the per-element corr_bwd (one lane per (pixel, channel), 441-displacement loop).
//   * Output is written channels-last [N, oH, oW, D*D] so the FlowNetC concat +
//     conv3_1 that consume it stay NHWC.
#include "common.h"

#include <cstdlib>

namespace iamd {
namespace {

constexpr int kTX = 32;       // output pixels per workgroup (one row segment)
constexpr int kCC = 32;       // channel chunk staged through LDS
constexpr int kLdsPad = kCC + 1;
constexpr int kCorrThreads = 256;
constexpr int kMaxDispPerLane = 3;  // ceil(D / (256/32)) for D <= 24

template <typename T>
__device__ __forceinline__ float ld_pad(const T* __restrict__ x, int n, int y, int xx, int c,
                                        int H, int W, int C) {
  if (y < 0 || y >= H || xx < 0 || xx >= W) return 0.f;
  return to_f<T>(x[(((int64_t)n * H + y) * W + xx) * C + c]);
}

// Tiled forward for kernel_size == 1. grid = (ceil(oW/32), oH, N*D), block = 256.
template <typename T>
__global__ __launch_bounds__(kCorrThreads) void corr_fwd_k1(
    const T* __restrict__ in1, const T* __restrict__ in2, T* __restrict__ out, int H, int W,
    int C, int oH, int oW, int pad, int md, int s1, int s2, int R, int D) {
  __shared__ float sA[kTX * kLdsPad];
  extern __shared__ float sB[];  // [span][kLdsPad]
  const int ox0 = blockIdx.x * kTX;
  const int oy = blockIdx.y;
  const int n = blockIdx.z / D;
  const int tjr = blockIdx.z % D;  // tj + R
  const int tid = threadIdx.x;
  const int px = tid % kTX;
  const int grp = tid / kTX;  // 8 groups of 32 lanes
  const int ngrp = kCorrThreads / kTX;
  const int span = (kTX - 1) * s1 + 2 * R * s2 + 1;
  // padded-frame centre of the first output pixel of the tile
  const int y1 = oy * s1 + md;
  const int x1_0 = ox0 * s1 + md;
  const int y2 = y1 + (tjr - R) * s2;
  const int bx0 = x1_0 - R * s2;  // first second-image column (padded frame)

  float acc[kMaxDispPerLane];
#pragma unroll
  for (int k = 0; k < kMaxDispPerLane; ++k) acc[k] = 0.f;

  for (int c0 = 0; c0 < C; c0 += kCC) {
    const int cc = min(kCC, C - c0);
    __syncthreads();
    for (int e = tid; e < kTX * kCC; e += kCorrThreads) {
      int p = e / kCC, c = e % kCC;
      float v = 0.f;
      if (c < cc && ox0 + p < oW)
        v = ld_pad(in1, n, y1 - pad, x1_0 + p * s1 - pad, c0 + c, H, W, C);
      sA[p * kLdsPad + c] = v;
    }
    for (int e = tid; e < span * kCC; e += kCorrThreads) {
      int p = e / kCC, c = e % kCC;
      float v = 0.f;
      if (c < cc) v = ld_pad(in2, n, y2 - pad, bx0 + p - pad, c0 + c, H, W, C);
      sB[p * kLdsPad + c] = v;
    }
    __syncthreads();
    for (int c = 0; c < cc; ++c) {
      const float a = sA[px * kLdsPad + c];
#pragma unroll
      for (int k = 0; k < kMaxDispPerLane; ++k) {
        const int tir = grp + k * ngrp;
        if (tir < D) acc[k] += a * sB[(px * s1 + tir * s2) * kLdsPad + c];
      }
    }
  }
  const int ox = ox0 + px;
  if (ox >= oW) return;
  const float inv = 1.f / (float)C;
  T* o = out + (((int64_t)n * oH + oy) * oW + ox) * (D * D);
#pragma unroll
  for (int k = 0; k < kMaxDispPerLane; ++k) {
    const int tir = grp + k * ngrp;
    if (tir < D) o[tjr * D + tir] = from_f<T>(acc[k] * inv);
  }
}

// MFMA forward for kernel_size == 1, stride1 == 1, stride2 in {1, 2}, bf16, C % 32 == 0 (the
// FlowNetC configuration: pad 20, max_disp 20, stride2 2 on 256-channel conv3 features).
// For one output row, one displacement row tj and TX = 16*S2 output pixels, split the pixels
// by parity r = x mod S2: pixel x = S2*a + r needs strip pixel S2*(a + t) + r for t in [0, D),
// so G_r[a][j] = sum_c A[S2*a + r][c] * B[S2*j + r][c] is a 16 x 48 MFMA product
// (v_mfma_f32_16x16x32_bf16, three 16-column fragments) and out[x][t] = G_r[a][a + t] is its
// band. Fragments are 16-byte NHWC channel runs loaded straight from global/L2 (each lane
// holds 8 channels of one pixel, the MFMA operand layout), so the kernel needs no LDS; the
// strip row of image 2 is shared by the D blocks of neighbouring output rows through L2.
template <int S2>
__global__ __launch_bounds__(64) void corr_fwd_mfma(
    const __hip_bfloat16* __restrict__ in1, const __hip_bfloat16* __restrict__ in2,
    __hip_bfloat16* __restrict__ out, int H, int W, int C, int oH, int oW, int pad, int md,
    int R, int D) {
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
  typedef __attribute__((ext_vector_type(4))) float f32x4;
  constexpr int TX = 16 * S2;
  const int ox0 = blockIdx.x * TX, oy = blockIdx.y;
  const int n = blockIdx.z / D, tjr = blockIdx.z - (blockIdx.z / D) * D;
  const int lane = threadIdx.x;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int y1 = oy + md - pad;
  const int y2 = y1 + (tjr - R) * S2;
  const bool row1 = (unsigned)y1 < (unsigned)H, row2 = (unsigned)y2 < (unsigned)H;
  const int xa0 = ox0 + md - pad;   // image column of tile pixel 0
  const int xb0 = xa0 - R * S2;     // image column of strip pixel 0
  const __hip_bfloat16* r1 = in1 + ((int64_t)n * H + (row1 ? y1 : 0)) * W * C;
  const __hip_bfloat16* r2 = in2 + ((int64_t)n * H + (row2 ? y2 : 0)) * W * C;
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  int aoff[S2], boff[S2][3];
  bool aok[S2], bok[S2][3];
#pragma unroll
  for (int r = 0; r < S2; ++r) {
    const int xa = xa0 + S2 * fr + r;
    aok[r] = row1 && (unsigned)xa < (unsigned)W && ox0 + S2 * fr + r < oW;
    aoff[r] = aok[r] ? xa * C + fk : 0;
#pragma unroll
    for (int cf = 0; cf < 3; ++cf) {
      const int xb = xb0 + S2 * (cf * 16 + fr) + r;
      bok[r][cf] = row2 && (unsigned)xb < (unsigned)W;
      boff[r][cf] = bok[r][cf] ? xb * C + fk : 0;
    }
  }
  f32x4 acc[S2][3];
#pragma unroll
  for (int r = 0; r < S2; ++r)
#pragma unroll
    for (int cf = 0; cf < 3; ++cf) acc[r][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < C; c0 += 32) {
#pragma unroll
    for (int r = 0; r < S2; ++r) {
      const bf16x8 af = aok[r] ? *reinterpret_cast<const bf16x8*>(r1 + aoff[r] + c0) : zero;
#pragma unroll
      for (int cf = 0; cf < 3; ++cf) {
        const bf16x8 bfr =
            bok[r][cf] ? *reinterpret_cast<const bf16x8*>(r2 + boff[r][cf] + c0) : zero;
        acc[r][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[r][cf], 0, 0, 0);
      }
    }
  }
  const float inv = 1.f / (float)C;
  const int DD = D * D;
#pragma unroll
  for (int r = 0; r < S2; ++r)
#pragma unroll
    for (int cf = 0; cf < 3; ++cf)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int a = (lane >> 4) * 4 + e;
        const int t = cf * 16 + fr - a;
        const int ox = ox0 + S2 * a + r;
        if (t >= 0 && t < D && ox < oW)
          out[(((int64_t)n * oH + oy) * oW + ox) * DD + tjr * D + t] =
              __float2bfloat16(acc[r][cf][e] * inv);
      }
}

// The same banded MFMA product, organised along the image-2 row (multi-wave): every (output row
// oy, displacement row tj) pair with oy + (tj - R) S2 = const reads the SAME image-2 strip, so a
// block owns one image-2 row y2 and one TX-pixel segment, stages that strip (TX + 2 R S2 pixels x
// all C channels) in LDS once, and its 4 waves run the D pairs of the diagonal (wave w: tj = w,
// w + 4, ...), each reading its image-1 fragments from global / L2 and the strip fragments from
// LDS. Per pair that is ~18 KB of L2 traffic instead of ~64 KB (the strip was re-read by each of
// the D blocks sharing it). LDS rows are padded by 16 B so the 16 fragment rows of a read (S2
// strip pixels apart) fall in different banks.
template <int S2>
__global__ __launch_bounds__(256) void corr_fwd_mfma_diag(
    const __hip_bfloat16* __restrict__ in1, const __hip_bfloat16* __restrict__ in2,
    __hip_bfloat16* __restrict__ out, int H, int W, int C, int oH, int oW, int pad, int md,
    int R, int D) {
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
  typedef __attribute__((ext_vector_type(4))) float f32x4;
  constexpr int TX = 16 * S2;
  constexpr int NP = 48 * S2;                   // strip pixels staged (3 x 16 per parity)
  extern __shared__ __attribute__((aligned(16))) char strip[];
  const int rowb = C * 2 + 16;                  // LDS bytes per strip pixel (padded)
  const int ox0 = blockIdx.x * TX;
  const int n = blockIdx.z;
  const int y2 = (md - pad - R * S2) + (int)blockIdx.y;  // image-2 row of this diagonal
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int xa0 = ox0 + md - pad;   // image column of tile pixel 0
  const int xb0 = xa0 - R * S2;     // image column of strip pixel 0
  const bool row2 = (unsigned)y2 < (unsigned)H;
  // ---- stage the strip: NP pixels x C channels, 16-byte chunks, zeros outside the image ------
  const int cpp = C / 8;  // chunks per pixel
  const __hip_bfloat16* r2 = in2 + ((int64_t)n * H + (row2 ? y2 : 0)) * W * C;
  for (int e = tid; e < NP * cpp; e += 256) {
    const int pxl = e / cpp, ch = e - pxl * cpp;
    const int xb = xb0 + pxl;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (row2 && (unsigned)xb < (unsigned)W)
      v = *reinterpret_cast<const uint4*>(r2 + (int64_t)xb * C + ch * 8);
    *reinterpret_cast<uint4*>(strip + pxl * rowb + ch * 16) = v;
  }
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const float inv = 1.f / (float)C;
  const int DD = D * D;
  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int tj = wid; tj < D; tj += 4) {
    const int y1 = y2 - (tj - R) * S2;          // image-1 row of this pair
    const int oy = y1 - md + pad;
    if ((unsigned)oy >= (unsigned)oH) continue;
    const bool row1 = row2 && (unsigned)y1 < (unsigned)H;
    const __hip_bfloat16* r1 = in1 + ((int64_t)n * H + (row1 ? y1 : 0)) * W * C;
    int aoff[S2];
    bool aok[S2];
#pragma unroll
    for (int r = 0; r < S2; ++r) {
      const int xa = xa0 + S2 * fr + r;
      aok[r] = row1 && (unsigned)xa < (unsigned)W && ox0 + S2 * fr + r < oW;
      aoff[r] = aok[r] ? xa * C + fk : 0;
    }
    f32x4 acc[S2][3];
#pragma unroll
    for (int r = 0; r < S2; ++r)
#pragma unroll
      for (int cf = 0; cf < 3; ++cf) acc[r][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (row1) {
      for (int c0 = 0; c0 < C; c0 += 32) {
#pragma unroll
        for (int r = 0; r < S2; ++r) {
          const bf16x8 af = aok[r] ? *reinterpret_cast<const bf16x8*>(r1 + aoff[r] + c0) : zero;
#pragma unroll
          for (int cf = 0; cf < 3; ++cf) {
            const int pxl = S2 * (cf * 16 + fr) + r;
            const bf16x8 bfr =
                *reinterpret_cast<const bf16x8*>(strip + pxl * rowb + (c0 + fk) * 2);
            acc[r][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[r][cf], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < S2; ++r)
#pragma unroll
      for (int cf = 0; cf < 3; ++cf)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int a = (lane >> 4) * 4 + e;
          const int t = cf * 16 + fr - a;
          const int ox = ox0 + S2 * a + r;
          if (t >= 0 && t < D && ox < oW)
            out[(((int64_t)n * oH + oy) * oW + ox) * DD + tj * D + t] =
                __float2bfloat16(acc[r][cf][e] * inv);
        }
  }
}

// Generic forward (any kernel_size): one workgroup (one wave) per output pixel.
template <typename T>
__global__ __launch_bounds__(kWave) void corr_fwd_generic(
    const T* __restrict__ in1, const T* __restrict__ in2, T* __restrict__ out, int H, int W,
    int C, int oH, int oW, int pad, int ks, int md, int s1, int s2, int R, int D) {
  const int ox = blockIdx.x, oy = blockIdx.y, n = blockIdx.z;
  const int kr = (ks - 1) / 2;
  const int y1 = oy * s1 + md, x1 = ox * s1 + md;
  const float inv = 1.f / (float)(ks * ks * C);
  T* o = out + (((int64_t)n * oH + oy) * oW + ox) * (D * D);
  for (int tj = -R; tj <= R; ++tj) {
    for (int ti = -R; ti <= R; ++ti) {
      const int y2 = y1 + tj * s2, x2 = x1 + ti * s2;
      float acc = 0.f;
      for (int j = -kr; j <= kr; ++j)
        for (int i = -kr; i <= kr; ++i)
          for (int c = threadIdx.x; c < C; c += kWave)
            acc += ld_pad(in1, n, y1 + j - pad, x1 + i - pad, c, H, W, C) *
                   ld_pad(in2, n, y2 + j - pad, x2 + i - pad, c, H, W, C);
      acc = wave_sum(acc);
      if (threadIdx.x == 0) o[(tj + R) * D + (ti + R)] = from_f<T>(acc * inv);
    }
  }
}

// Backward w.r.t. both inputs, gather form. One lane per (n, y, x, c) of the
// *unpadded* inputs; grad_out is channels-last [N, oH, oW, D*D] fp32.
template <typename T>
__global__ __launch_bounds__(256) void corr_bwd(
    const T* __restrict__ in1, const T* __restrict__ in2, const float* __restrict__ gout,
    float* __restrict__ g1, float* __restrict__ g2, int N, int H, int W, int C, int oH, int oW,
    int pad, int ks, int md, int s1, int s2, int R, int D) {
  const int64_t total = (int64_t)N * H * W * C;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = idx % C;
  int64_t r = idx / C;
  const int x = r % W;
  r /= W;
  const int y = r % H;
  const int n = r / H;
  const int kr = (ks - 1) / 2;
  const int py = y + pad, px = x + pad;  // padded frame
  const int DD = D * D;
  const float inv = 1.f / (float)(ks * ks * C);
  float a1 = 0.f, a2 = 0.f;
  for (int j = -kr; j <= kr; ++j) {
    for (int i = -kr; i <= kr; ++i) {
      // grad_in1: this element is in1 at window offset (j,i) of centre (py-j, px-i)
      {
        const int cy = py - j, cx = px - i;
        const int ty = cy - md, tx = cx - md;
        if (ty >= 0 && tx >= 0 && ty % s1 == 0 && tx % s1 == 0) {
          const int oy = ty / s1, ox = tx / s1;
          if (oy < oH && ox < oW) {
            const float* go = gout + (((int64_t)n * oH + oy) * oW + ox) * DD;
            for (int tj = -R; tj <= R; ++tj)
              for (int ti = -R; ti <= R; ++ti)
                a1 += go[(tj + R) * D + ti + R] *
                      ld_pad(in2, n, cy + tj * s2 + j - pad, cx + ti * s2 + i - pad, c, H, W, C);
          }
        }
      }
      // grad_in2: this element is in2 at window offset (j,i) of displaced centre
      for (int tj = -R; tj <= R; ++tj) {
        const int cy = py - tj * s2 - j;
        const int ty = cy - md;
        if (ty < 0 || ty % s1 != 0 || ty / s1 >= oH) continue;
        const int oy = ty / s1;
        for (int ti = -R; ti <= R; ++ti) {
          const int cx = px - ti * s2 - i;
          const int tx = cx - md;
          if (tx < 0 || tx % s1 != 0 || tx / s1 >= oW) continue;
          const int ox = tx / s1;
          a2 += gout[(((int64_t)n * oH + oy) * oW + ox) * DD + (tj + R) * D + ti + R] *
                ld_pad(in1, n, cy + j - pad, cx + i - pad, c, H, W, C);
        }
      }
    }
  }
  g1[idx] = a1 * inv;
  g2[idx] = a2 * inv;
}

// Tiled backward for kernel_size == 1, stride1 == 1 (the FlowNetC configuration), gather form.
// One workgroup owns 32 consecutive pixels of one image row and CC channels; per displacement
// row tj it stages, in LDS, the two (32 + 2 R s2)-pixel strips the row's gradients read — the
// second-image strip for d(in1), the first-image strip for d(in2) — plus the grad_out rows they
// pair with, then each lane (pixel, CC/8 channels) accumulates its D displacements of this tj
// from LDS. Every input / grad_out element is read from L2 once per (row, tj) instead of once
// per (element, displacement) as in corr_bwd; deterministic, no atomics.
constexpr int kBX = 32;       // pixels per workgroup
constexpr int kBCC = 64;      // channels per workgroup (8 per lane)
template <typename T>
__global__ __launch_bounds__(256) void corr_bwd_k1(
    const T* __restrict__ in1, const T* __restrict__ in2, const float* __restrict__ gout,
    float* __restrict__ g1, float* __restrict__ g2, int H, int W, int C, int oH, int oW, int off,
    int s2, int R, int D) {
  extern __shared__ float smem[];
  const int span = kBX + 2 * R * s2;
  float* G1 = smem;                       // [kBX][D]
  float* G2 = G1 + kBX * D;               // [span][D]
  float* S2 = G2 + (span * D + 3) / 4 * 4;  // in2 strip [span][kBCC] (16-byte aligned)
  float* S1 = S2 + span * kBCC;           // in1 strip [span][kBCC]
  const int x0 = blockIdx.x * kBX, y = blockIdx.y;
  const int nc = C / kBCC;
  const int n = blockIdx.z / nc, c0 = (blockIdx.z - n * nc) * kBCC;
  const int tid = threadIdx.x, px = tid >> 3, cl = (tid & 7) * 8;
  const int DD = D * D;
  const int ws = x0 - R * s2;             // image column of strip pixel 0
  float a1[8], a2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a1[k] = a2[k] = 0.f;
  const int oy1 = y - off;                // output row paired with d(in1) of row y
  for (int tj = 0; tj < D; ++tj) {
    const int dy = (tj - R) * s2;
    const int y2 = y + dy;                // in2 row read by d(in1)
    const int yb = y - dy;                // in1 row (and output row yb - off) for d(in2)
    const int oy2 = yb - off;
    __syncthreads();
    for (int e = tid; e < kBX * D; e += 256) {
      const int p = e / D, ti = e - p * D;
      const int ox = x0 + p - off;
      float v = 0.f;
      if ((unsigned)oy1 < (unsigned)oH && (unsigned)ox < (unsigned)oW)
        v = gout[(((int64_t)n * oH + oy1) * oW + ox) * DD + tj * D + ti];
      G1[e] = v;
    }
    for (int e = tid; e < span * D; e += 256) {
      const int p = e / D, ti = e - p * D;
      const int ox = ws + p - off;
      float v = 0.f;
      if ((unsigned)oy2 < (unsigned)oH && (unsigned)ox < (unsigned)oW)
        v = gout[(((int64_t)n * oH + oy2) * oW + ox) * DD + tj * D + ti];
      G2[e] = v;
    }
    for (int e = tid; e < span * (kBCC / 8); e += 256) {
      const int p = e / (kBCC / 8), c8 = (e - p * (kBCC / 8)) * 8;
      const int x = ws + p;
      float v2[8], v1[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v2[k] = v1[k] = 0.f;
      if ((unsigned)x < (unsigned)W) {
        if ((unsigned)y2 < (unsigned)H)
          load_vec<T, 8>(in2 + (((int64_t)n * H + y2) * W + x) * C + c0 + c8, v2);
        if ((unsigned)yb < (unsigned)H)
          load_vec<T, 8>(in1 + (((int64_t)n * H + yb) * W + x) * C + c0 + c8, v1);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        S2[p * kBCC + c8 + k] = v2[k];
        S1[p * kBCC + c8 + k] = v1[k];
      }
    }
    __syncthreads();
    for (int ti = 0; ti < D; ++ti) {
      const float w1 = G1[px * D + ti];
      const int i1 = px + ti * s2;                 // strip index of x + (ti - R) s2
      const int i2 = px + (2 * R - ti) * s2;       // strip index of x - (ti - R) s2
      const float w2 = G2[i2 * D + ti];
      const float4* r2 = reinterpret_cast<const float4*>(S2 + i1 * kBCC + cl);
      const float4* r1 = reinterpret_cast<const float4*>(S1 + i2 * kBCC + cl);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 b = r2[q], a = r1[q];
        a1[4 * q + 0] += w1 * b.x; a1[4 * q + 1] += w1 * b.y;
        a1[4 * q + 2] += w1 * b.z; a1[4 * q + 3] += w1 * b.w;
        a2[4 * q + 0] += w2 * a.x; a2[4 * q + 1] += w2 * a.y;
        a2[4 * q + 2] += w2 * a.z; a2[4 * q + 3] += w2 * a.w;
      }
    }
  }
  const int x = x0 + px;
  if (x >= W) return;
  const float inv = 1.f / (float)C;
  const int64_t o = (((int64_t)n * H + y) * W + x) * C + c0 + cl;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    reinterpret_cast<float4*>(g1 + o)[q] =
        make_float4(a1[4 * q] * inv, a1[4 * q + 1] * inv, a1[4 * q + 2] * inv, a1[4 * q + 3] * inv);
    reinterpret_cast<float4*>(g2 + o)[q] =
        make_float4(a2[4 * q] * inv, a2[4 * q + 1] * inv, a2[4 * q + 2] * inv, a2[4 * q + 3] * inv);
  }
}

// Register-blocked variant of corr_bwd_k1 (opt-in, for s2 in {1, 2} and 16-bit inputs): 96
// pixels x 64 channels per workgroup, each lane owns kRPX = 3 pixels of one parity class (s2
// apart) x 8 channels. Pixel m at displacement ti reads strip row (m + ti) s2 for d(in1) and
// (m + 2R - ti) s2 for d(in2), so stepping ti slides a 3-row register window by one row: one
// 16-byte (bf16) LDS read per window and ti feeds 24 FMAs, against 8 FMAs per 32-byte read in
// corr_bwd_k1, which is bound by LDS bandwidth. Strips are kept in the input dtype (half the LDS
// bytes of fp32), so the FlowNetC shape needs 54 KB.
constexpr int kRPX = 3;            // pixels per lane
constexpr int kRBX = 32 * kRPX;    // pixels per workgroup
template <typename T>
__global__ __launch_bounds__(256) void corr_bwd_k1r(
    const T* __restrict__ in1, const T* __restrict__ in2, const float* __restrict__ gout,
    float* __restrict__ g1, float* __restrict__ g2, int H, int W, int C, int oH, int oW, int off,
    int s2, int R, int D) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int span = kRBX + 2 * R * s2;
  float* G1 = smem;                            // [kRBX][D]
  float* G2 = G1 + kRBX * D;                   // [span][D]
  T* S2 = reinterpret_cast<T*>(G2 + (span * D + 3) / 4 * 4);  // in2 strip [span][kBCC]
  T* S1 = S2 + span * kBCC;                    // in1 strip [span][kBCC]
  const int x0 = blockIdx.x * kRBX, y = blockIdx.y;
  const int nc = C / kBCC;
  const int n = blockIdx.z / nc, c0 = (blockIdx.z - n * nc) * kBCC;
  const int tid = threadIdx.x, pl = tid >> 3, cl = (tid & 7) * 8;
  // this lane's pixels: base + m s2, m < kRPX (strip / tile index)
  const int base = s2 == 1 ? pl * kRPX : (pl >> 1) * (2 * kRPX) + (pl & 1);
  const int DD = D * D;
  const int ws = x0 - R * s2;
  float a1[kRPX][8], a2[kRPX][8];
#pragma unroll
  for (int m = 0; m < kRPX; ++m)
#pragma unroll
    for (int k = 0; k < 8; ++k) a1[m][k] = a2[m][k] = 0.f;
  const int oy1 = y - off;
  for (int tj = 0; tj < D; ++tj) {
    const int dy = (tj - R) * s2;
    const int y2 = y + dy, yb = y - dy, oy2 = yb - off;
    __syncthreads();
    for (int e = tid; e < kRBX * D; e += 256) {
      const int p = e / D, ti = e - p * D;
      const int ox = x0 + p - off;
      float v = 0.f;
      if ((unsigned)oy1 < (unsigned)oH && (unsigned)ox < (unsigned)oW)
        v = gout[(((int64_t)n * oH + oy1) * oW + ox) * DD + tj * D + ti];
      G1[e] = v;
    }
    for (int e = tid; e < span * D; e += 256) {
      const int p = e / D, ti = e - p * D;
      const int ox = ws + p - off;
      float v = 0.f;
      if ((unsigned)oy2 < (unsigned)oH && (unsigned)ox < (unsigned)oW)
        v = gout[(((int64_t)n * oH + oy2) * oW + ox) * DD + tj * D + ti];
      G2[e] = v;
    }
    for (int e = tid; e < span * (kBCC / 8); e += 256) {
      const int p = e / (kBCC / 8), c8 = (e - p * (kBCC / 8)) * 8;
      const int x = ws + p;
      float v2[8], v1[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v2[k] = v1[k] = 0.f;
      if ((unsigned)x < (unsigned)W) {
        if ((unsigned)y2 < (unsigned)H)
          load_vec<T, 8>(in2 + (((int64_t)n * H + y2) * W + x) * C + c0 + c8, v2);
        if ((unsigned)yb < (unsigned)H)
          load_vec<T, 8>(in1 + (((int64_t)n * H + yb) * W + x) * C + c0 + c8, v1);
      }
      store_vec<T, 8>(S2 + p * kBCC + c8, v2);
      store_vec<T, 8>(S1 + p * kBCC + c8, v1);
    }
    __syncthreads();
    // windows (kRPX rows): r2[m] = S2 row base + (ti + m) s2, r1[m] = S1 row base + (m + 2R - ti) s2
    float r2[kRPX][8], r1[kRPX][8];
#pragma unroll
    for (int m = 0; m < kRPX; ++m) {
      load_vec<T, 8>(S2 + (base + m * s2) * kBCC + cl, r2[m]);
      load_vec<T, 8>(S1 + (base + (m + 2 * R) * s2) * kBCC + cl, r1[m]);
    }
    for (int ti = 0; ti < D; ++ti) {
      float w1[kRPX], w2[kRPX];
#pragma unroll
      for (int m = 0; m < kRPX; ++m) {
        w1[m] = G1[(base + m * s2) * D + ti];
        w2[m] = G2[(base + (m + 2 * R - ti) * s2) * D + ti];
      }
#pragma unroll
      for (int m = 0; m < kRPX; ++m)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a1[m][k] = fmaf(w1[m], r2[m][k], a1[m][k]);
          a2[m][k] = fmaf(w2[m], r1[m][k], a2[m][k]);
        }
      if (ti + 1 < D) {
#pragma unroll
        for (int m = 0; m < kRPX - 1; ++m)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            r2[m][k] = r2[m + 1][k];
            r1[kRPX - 1 - m][k] = r1[kRPX - 2 - m][k];
          }
        load_vec<T, 8>(S2 + (base + (ti + kRPX) * s2) * kBCC + cl, r2[kRPX - 1]);
        load_vec<T, 8>(S1 + (base + (2 * R - ti - 1) * s2) * kBCC + cl, r1[0]);
      }
    }
  }
  const float inv = 1.f / (float)C;
#pragma unroll
  for (int m = 0; m < kRPX; ++m) {
    const int x = x0 + base + m * s2;
    if (x >= W) continue;
    const int64_t o = (((int64_t)n * H + y) * W + x) * C + c0 + cl;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      reinterpret_cast<float4*>(g1 + o)[q] = make_float4(a1[m][4 * q] * inv, a1[m][4 * q + 1] * inv,
                                                         a1[m][4 * q + 2] * inv, a1[m][4 * q + 3] * inv);
      reinterpret_cast<float4*>(g2 + o)[q] = make_float4(a2[m][4 * q] * inv, a2[m][4 * q + 1] * inv,
                                                         a2[m][4 * q + 2] * inv, a2[m][4 * q + 3] * inv);
    }
  }
}

// ---- k8 channel norm (generic 4-D strides, fp32 accumulate) -------------------
template <typename T>
__global__ void chnorm_fwd(const T* __restrict__ x, T* __restrict__ out, int N, int C, int H,
                           int W, int64_t sn, int64_t sc, int64_t sh, int64_t sw) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * H * W) return;
  const int xx = idx % W;
  const int y = (idx / W) % H;
  const int n = idx / ((int64_t)H * W);
  const T* p = x + n * sn + y * sh + xx * sw;
  float acc = 0.f;
  for (int c = 0; c < C; ++c) {
    float v = to_f<T>(p[c * sc]);
    acc += v * v;
  }
  out[idx] = from_f<T>(sqrtf(acc));
}

template <typename T>
__global__ void chnorm_bwd(const T* __restrict__ x, const T* __restrict__ nrm,
                           const T* __restrict__ g, T* __restrict__ dx, int N, int C, int H,
                           int W, int64_t sn, int64_t sc, int64_t sh, int64_t sw) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * H * W) return;
  const int xx = idx % W;
  const int y = (idx / W) % H;
  const int n = idx / ((int64_t)H * W);
  const int64_t off = n * sn + y * sh + xx * sw;
  const float k = to_f<T>(g[idx]) / (to_f<T>(nrm[idx]) + 1e-9f);
  for (int c = 0; c < C; ++c) dx[off + c * sc] = from_f<T>(to_f<T>(x[off + c * sc]) * k);
}

inline int corr_out_size(int in, int pad, int ks, int md, int s1) {
  const int border = (ks - 1) / 2 + md;
  const int padded = in + 2 * pad;
  return (int)std::ceil((double)(padded - 2 * border) / (double)s1);
}

}  // namespace

// in1, in2: [N, C, H, W] (any memory format; made channels-last internally)
// returns [N, D*D, oH, oW] in channels-last memory format, dtype of the inputs.
at::Tensor correlation_forward(const at::Tensor& input1, const at::Tensor& input2, int64_t pad,
                               int64_t ks, int64_t md, int64_t s1, int64_t s2) {
  IAMD_CHECK(input1.dim() == 4 && input1.sizes() == input2.sizes(), "correlation: shapes");
  IAMD_CHECK(ks >= 1 && ks % 2 == 1 && s1 >= 1 && s2 >= 1, "correlation: bad params");
  auto a = input1.contiguous(at::MemoryFormat::ChannelsLast);
  auto b = input2.to(a.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  const int N = a.size(0), C = a.size(1), H = a.size(2), W = a.size(3);
  const int R = md / s2, D = 2 * R + 1;
  const int oH = corr_out_size(H, pad, ks, md, s1), oW = corr_out_size(W, pad, ks, md, s1);
  IAMD_CHECK(oH > 0 && oW > 0, "correlation: empty output");
  auto out = at::empty({N, D * D, oH, oW},
                       a.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int ngrp = kCorrThreads / kTX;
  const char* mf = std::getenv("IMAGINAIRE_AMD_CORR_MFMA");
  if ((mf == nullptr || mf[0] != '0') && a.scalar_type() == at::kBFloat16 && ks == 1 && s1 == 1 &&
      (s2 == 1 || s2 == 2) &&
      C % 32 == 0 && D <= 33 && (int64_t)H * W * C < (1ll << 31)) {
    auto pa = reinterpret_cast<const __hip_bfloat16*>(a.data_ptr());
    auto pb = reinterpret_cast<const __hip_bfloat16*>(b.data_ptr());
    auto po = reinterpret_cast<__hip_bfloat16*>(out.data_ptr());
    // the diagonal multi-wave kernel (strip staged once per image-2 row) when the strip fits in
    // LDS; IMAGINAIRE_AMD_CORR_DIAG=0 keeps the one-wave-per-(row, tj) kernel
    const char* dg = std::getenv("IMAGINAIRE_AMD_CORR_DIAG");
    const size_t strip_bytes = (size_t)48 * s2 * (C * 2 + 16);
    const bool diag = (dg == nullptr || dg[0] != '0') && strip_bytes <= 64 * 1024;
    const dim3 gdiag((unsigned)ceil_div(oW, 16 * (int)s2), (unsigned)(oH + 2 * R * (int)s2),
                     (unsigned)N);
    if (diag && s2 == 2)
      hipLaunchKernelGGL((corr_fwd_mfma_diag<2>), gdiag, dim3(256), strip_bytes, stream(), pa, pb,
                         po, H, W, C, oH, oW, (int)pad, (int)md, R, D);
    else if (diag)
      hipLaunchKernelGGL((corr_fwd_mfma_diag<1>), gdiag, dim3(256), strip_bytes, stream(), pa, pb,
                         po, H, W, C, oH, oW, (int)pad, (int)md, R, D);
    else if (s2 == 2)
      hipLaunchKernelGGL((corr_fwd_mfma<2>), dim3(ceil_div(oW, 32), oH, N * D), dim3(64), 0,
                         stream(), pa, pb, po, H, W, C, oH, oW, (int)pad, (int)md, R, D);
    else
      hipLaunchKernelGGL((corr_fwd_mfma<1>), dim3(ceil_div(oW, 16), oH, N * D), dim3(64), 0,
                         stream(), pa, pb, po, H, W, C, oH, oW, (int)pad, (int)md, R, D);
    IAMD_LAUNCH_CHECK();
    return out;
  }
  IAMD_DISPATCH_FLOAT_TYPES(a.scalar_type(), "correlation_fwd", [&] {
    auto pa = reinterpret_cast<const scalar_t*>(a.data_ptr());
    auto pb = reinterpret_cast<const scalar_t*>(b.data_ptr());
    auto po = reinterpret_cast<scalar_t*>(out.data_ptr());
    const int span = (kTX - 1) * s1 + 2 * R * s2 + 1;
    const size_t lds = (size_t)span * kLdsPad * sizeof(float);
    if (ks == 1 && D <= ngrp * kMaxDispPerLane && lds <= 96 * 1024) {
      dim3 grid(ceil_div(oW, kTX), oH, N * D);
      hipLaunchKernelGGL((corr_fwd_k1<scalar_t>), grid, dim3(kCorrThreads), lds, stream(), pa,
                         pb, po, H, W, C, oH, oW, (int)pad, (int)md, (int)s1, (int)s2, R, D);
    } else {
      dim3 grid(oW, oH, N);
      hipLaunchKernelGGL((corr_fwd_generic<scalar_t>), grid, dim3(kWave), 0, stream(), pa, pb,
                         po, H, W, C, oH, oW, (int)pad, (int)ks, (int)md, (int)s1, (int)s2, R,
                         D);
    }
  });
  IAMD_LAUNCH_CHECK();
  return out;
}

// returns {grad_input1, grad_input2} fp32, channels-last [N, C, H, W]
std::vector<at::Tensor> correlation_backward(const at::Tensor& input1, const at::Tensor& input2,
                                             const at::Tensor& grad_out, int64_t pad,
                                             int64_t ks, int64_t md, int64_t s1, int64_t s2) {
  auto a = input1.contiguous(at::MemoryFormat::ChannelsLast);
  auto b = input2.to(a.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  auto g = grad_out.to(at::kFloat).contiguous(at::MemoryFormat::ChannelsLast);
  const int N = a.size(0), C = a.size(1), H = a.size(2), W = a.size(3);
  const int R = md / s2, D = 2 * R + 1;
  const int oH = corr_out_size(H, pad, ks, md, s1), oW = corr_out_size(W, pad, ks, md, s1);
  IAMD_CHECK(g.size(0) == N && g.size(1) == D * D && g.size(2) == oH && g.size(3) == oW,
             "correlation_backward: grad_out shape");
  auto fopt = a.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast);
  auto g1 = at::empty({N, C, H, W}, fopt);
  auto g2 = at::empty({N, C, H, W}, fopt);
  const int64_t total = (int64_t)N * H * W * C;
  if (total == 0) return {g1, g2};
  const size_t span = (size_t)(kBX + 2 * R * s2);
  const size_t lds = ((size_t)kBX * D + (span * D + 3) / 4 * 4 + 2 * span * kBCC) * sizeof(float);
  const char* tb = std::getenv("IMAGINAIRE_AMD_CORR_BWD_TILED");
  // register-blocked tiled kernel (IMAGINAIRE_AMD_CORR_BWD_TILED=2): measured 0.69-0.86x
  // corr_bwd_k1 at the FlowNetC shapes (profiles/corr_bwd_probe_mi355x.txt), so not the default
  const size_t rspan = (size_t)(kRBX + 2 * R * s2);
  const size_t rlds = ((size_t)kRBX * D + (rspan * D + 3) / 4 * 4) * sizeof(float) +
                      2 * rspan * kBCC * a.element_size();
  if (tb != nullptr && tb[0] == '2' && ks == 1 && s1 == 1 && (s2 == 1 || s2 == 2) &&
      a.element_size() == 2 && C % kBCC == 0 && rlds <= 64 * 1024) {
    IAMD_DISPATCH_FLOAT_TYPES(a.scalar_type(), "correlation_bwd_k1r", [&] {
      dim3 grid(ceil_div(W, kRBX), H, N * (C / kBCC));
      hipLaunchKernelGGL((corr_bwd_k1r<scalar_t>), grid, dim3(256), rlds, stream(),
                         reinterpret_cast<const scalar_t*>(a.data_ptr()),
                         reinterpret_cast<const scalar_t*>(b.data_ptr()), g.data_ptr<float>(),
                         g1.data_ptr<float>(), g2.data_ptr<float>(), H, W, C, oH, oW,
                         (int)(md - pad), (int)s2, R, D);
    });
    IAMD_LAUNCH_CHECK();
    return {g1, g2};
  }
  if ((tb == nullptr || tb[0] != '0') && ks == 1 && s1 == 1 && C % kBCC == 0 &&
      lds <= 96 * 1024) {
    IAMD_DISPATCH_FLOAT_TYPES(a.scalar_type(), "correlation_bwd_k1", [&] {
      dim3 grid(ceil_div(W, kBX), H, N * (C / kBCC));
      hipLaunchKernelGGL((corr_bwd_k1<scalar_t>), grid, dim3(256), lds, stream(),
                         reinterpret_cast<const scalar_t*>(a.data_ptr()),
                         reinterpret_cast<const scalar_t*>(b.data_ptr()), g.data_ptr<float>(),
                         g1.data_ptr<float>(), g2.data_ptr<float>(), H, W, C, oH, oW,
                         (int)(md - pad), (int)s2, R, D);
    });
    IAMD_LAUNCH_CHECK();
    return {g1, g2};
  }
  IAMD_DISPATCH_FLOAT_TYPES(a.scalar_type(), "correlation_bwd", [&] {
    hipLaunchKernelGGL((corr_bwd<scalar_t>), dim3(ceil_div(total, 256)), dim3(256), 0, stream(),
                       reinterpret_cast<const scalar_t*>(a.data_ptr()),
                       reinterpret_cast<const scalar_t*>(b.data_ptr()), g.data_ptr<float>(),
                       g1.data_ptr<float>(), g2.data_ptr<float>(), N, H, W, C, oH, oW, (int)pad,
                       (int)ks, (int)md, (int)s1, (int)s2, R, D);
  });
  IAMD_LAUNCH_CHECK();
  return {g1, g2};
}

// x: [N, C, H, W] any strides -> [N, 1, H, W]
at::Tensor channelnorm_forward(const at::Tensor& x) {
  IAMD_CHECK(x.dim() == 4, "channelnorm: 4-D input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto out = at::empty({N, 1, H, W}, x.options());
  const int64_t total = (int64_t)N * H * W;
  if (total == 0) return out;
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "channelnorm_fwd", [&] {
    hipLaunchKernelGGL((chnorm_fwd<scalar_t>), dim3(ceil_div(total, 256)), dim3(256), 0, stream(),
                       reinterpret_cast<const scalar_t*>(x.data_ptr()),
                       reinterpret_cast<scalar_t*>(out.data_ptr()), N, C, H, W, x.stride(0),
                       x.stride(1), x.stride(2), x.stride(3));
  });
  IAMD_LAUNCH_CHECK();
  return out;
}

at::Tensor channelnorm_backward(const at::Tensor& x, const at::Tensor& out,
                                const at::Tensor& grad_out) {
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto nrm = out.to(x.scalar_type()).contiguous();
  auto g = grad_out.to(x.scalar_type()).contiguous();
  auto dx = at::empty_strided(x.sizes(), x.strides(), x.options());
  const int64_t total = (int64_t)N * H * W;
  if (total == 0) return dx;
  IAMD_CHECK(x.is_non_overlapping_and_dense(), "channelnorm_backward: dense input");
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "channelnorm_bwd", [&] {
    hipLaunchKernelGGL((chnorm_bwd<scalar_t>), dim3(ceil_div(total, 256)), dim3(256), 0, stream(),
                       reinterpret_cast<const scalar_t*>(x.data_ptr()),
                       reinterpret_cast<const scalar_t*>(nrm.data_ptr()),
                       reinterpret_cast<const scalar_t*>(g.data_ptr()),
                       reinterpret_cast<scalar_t*>(dx.data_ptr()), N, C, H, W, x.stride(0),
                       x.stride(1), x.stride(2), x.stride(3));
  });
  IAMD_LAUNCH_CHECK();
  return dx;
}

}  // namespace iamd
