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
// * pad_nhwc — reflect / replicate padding of NHWC activations (the UNIT / MUNIT / FUNIT conv
//   blocks, reference layers/conv.py:59-91 padding_mode='reflect'): a 16-byte gather forward and a
//   GATHER backward (each input pixel sums the <= 4 padded pixels that copied it per axis pair).
//   PyTorch's reflection_pad2d backward ran at ~1/50 of HBM bandwidth on channels-last bf16
//   activations — a quarter of a MUNIT iteration (profiles/recipe_munit256_kernels_mi355x.txt).
//
// Reference: the reference gets the first two from cuDNN inside nn.Conv2d's autograd
// (layers/conv.py:59-91); these kernels have no reference counterpart.
#include "common.h"

#include <array>
#include <mutex>
#include <unordered_map>

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
  const int KK = KH * KW, JJ = Jy * Jx;
  const int ci0 = blockIdx.x * kTile, co0 = blockIdx.y * kTile;
  const int nbz = blockIdx.z / JJ, tap = blockIdx.z - nbz * JJ;  // (sample, output tap)
  w += (size_t)nbz * Cout * KK * Cin;
  wt += (size_t)nbz * Cin * JJ * Cout;
  const int jy = tap / Jx, jx = tap - jy * Jx;
  const int ftap = (qy + s * (Jy - 1 - jy)) * KW + (qx + s * (Jx - 1 - jx));
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
// A block sums OPB = 256 / G outputs (4 channels each when VEC) with G thread groups splitting
// the S slabs (s = g, g + G, ...), then adds the G partials in a fixed order (deterministic):
// a one-tile weight gradient (1x1 conv, 64 x 64) is split over up to 1024 pixel ranges, and a
// single thread per output walking all slabs was latency-bound at ~0.3 ms.
template <typename T, bool VEC>
__global__ void __launch_bounds__(kT)
wgrad_finalize_kernel(const float* __restrict__ part, T* __restrict__ out, int S, int Cop, int Cip,
                      int Cout, int Cin, int KK, int G) {
  __shared__ float4 red[kT];
  const int opb = kT / G;
  const int tid = threadIdx.x, o = tid % opb, g = tid / opb;
  const int per = VEC ? Cin / 4 : Cin;
  const int64_t n = (int64_t)Cout * KK * per;
  const int64_t slab = (int64_t)Cop * KK * Cip;
  for (int64_t i0 = (int64_t)blockIdx.x * opb; i0 < n; i0 += (int64_t)gridDim.x * opb) {
    const int64_t i = i0 + o;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t rt = 0, src = 0;
    int c = 0;
    if (i < n) {
      c = (int)(i % per);
      rt = i / per;  // co * KK + t
      const int t = (int)(rt % KK);
      const int co = (int)(rt / KK);
      src = ((int64_t)co * KK + t) * Cip + (VEC ? c * 4 : c);
      for (int sl = g; sl < S; sl += G) {
        if constexpr (VEC) {
          const float4 v = *reinterpret_cast<const float4*>(part + sl * slab + src);
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        } else {
          acc.x += part[sl * slab + src];
        }
      }
    }
    red[tid] = acc;
    __syncthreads();
    if (g == 0 && i < n) {
      for (int k = 1; k < G; ++k) {
        const float4 v = red[k * opb + o];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      if constexpr (VEC) {
        const float a[4] = {acc.x, acc.y, acc.z, acc.w};
        T* dst = out + rt * Cin + c * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = from_f<T>(a[k]);
      } else {
        out[rt * Cin + c] = from_f<T>(acc.x);
      }
    }
    __syncthreads();
  }
}

// As wgrad_finalize_kernel (fp32 out, real dims), with the spectral-norm backward applied:
//   dW[co][t][ci] = G / sigma - (<G, W> / sigma^2) u[co] v[ci * KK + t]
// where <G, W> = sum of the k11 blocks' partials dotp[0 .. ndot) (every block sums them itself,
// in a fixed order) and v is in the reference's logical column order (ci, kh, kw).
template <bool VEC>
__global__ void __launch_bounds__(kT)
wgrad_finalize_sn_kernel(const float* __restrict__ part, float* __restrict__ out, int S, int Cop,
                         int Cip, int Cout, int Cin, int KK, int G,
                         const float* __restrict__ dotp, int ndot, const float* __restrict__ u,
                         const float* __restrict__ v, const float* __restrict__ sigma) {
  __shared__ float4 red[kT];
  __shared__ float dsh[kT / 64];
  const int opb = kT / G;
  const int tid = threadIdx.x, o = tid % opb, g = tid / opb;
  float dd = 0.f;
  for (int k = tid; k < ndot; k += kT) dd += dotp[k];
  dd = wave_sum(dd);
  if ((tid & 63) == 0) dsh[tid >> 6] = dd;
  __syncthreads();
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < kT / 64; ++k) dot += dsh[k];
  const float inv = 1.f / sigma[0];
  const float cf = dot * inv * inv;  // <G, W> / sigma^2
  const int per = VEC ? Cin / 4 : Cin;
  const int64_t n = (int64_t)Cout * KK * per;
  const int64_t slab = (int64_t)Cop * KK * Cip;
  for (int64_t i0 = (int64_t)blockIdx.x * opb; i0 < n; i0 += (int64_t)gridDim.x * opb) {
    const int64_t i = i0 + o;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t rt = 0, src = 0;
    int c = 0, t = 0, co = 0;
    if (i < n) {
      c = (int)(i % per);
      rt = i / per;  // co * KK + t
      t = (int)(rt % KK);
      co = (int)(rt / KK);
      src = ((int64_t)co * KK + t) * Cip + (VEC ? c * 4 : c);
      for (int sl = g; sl < S; sl += G) {
        if constexpr (VEC) {
          const float4 w4 = *reinterpret_cast<const float4*>(part + sl * slab + src);
          acc.x += w4.x; acc.y += w4.y; acc.z += w4.z; acc.w += w4.w;
        } else {
          acc.x += part[sl * slab + src];
        }
      }
    }
    red[tid] = acc;
    __syncthreads();
    if (g == 0 && i < n) {
      for (int k = 1; k < G; ++k) {
        const float4 w4 = red[k * opb + o];
        acc.x += w4.x; acc.y += w4.y; acc.z += w4.z; acc.w += w4.w;
      }
      const float cu = cf * u[co];
      if constexpr (VEC) {
        const float* vv = v + (int64_t)c * 4 * KK + t;
        *reinterpret_cast<float4*>(out + rt * Cin + c * 4) =
            make_float4(fmaf(acc.x, inv, -cu * vv[0]), fmaf(acc.y, inv, -cu * vv[KK]),
                        fmaf(acc.z, inv, -cu * vv[2 * KK]), fmaf(acc.w, inv, -cu * vv[3 * KK]));
      } else {
        out[rt * Cin + c] = fmaf(acc.x, inv, -cu * v[(int64_t)c * KK + t]);
      }
    }
    __syncthreads();
  }
}

// padded index o -> source index along one axis (mode 0 reflect, 1 replicate)
__device__ __forceinline__ int pad_src(int o, int p, int n, int mode) {
  int i = o - p;
  if (mode == 0) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * (n - 1) - i;
  } else {
    i = min(max(i, 0), n - 1);
  }
  return i;
}

constexpr int kPadMax = 16;  // padded indices that may copy one source index (per axis)

__device__ __forceinline__ int pad_list(int i, int p0, int p1, int n, int mode,
                                        int (&idx)[kPadMax]) {
  // candidates: the direct copy, its reflections across both edges, or (replicate) the whole
  // edge band
  int cnt = 0;
  const int no = n + p0 + p1;
  int lo = i + p0, hi = i + p0;
  if (mode == 1) {
    if (i == 0) lo = 0;
    if (i == n - 1) hi = no - 1;
    for (int o = lo; o <= hi && cnt < kPadMax; ++o) idx[cnt++] = o;
    return cnt;
  }
  idx[cnt++] = i + p0;
  const int a = p0 - i;                      // reflection across the leading edge
  if (i > 0 && a >= 0) idx[cnt++] = a;
  const int b = 2 * (n - 1) - i + p0;        // reflection across the trailing edge
  if (i < n - 1 && b < no && b != i + p0) idx[cnt++] = b;
  return cnt;
}

// grid (ceil(Wo*C/V / kT), B*Ho): one block row per output image row, 32-bit in-row indices
// (the flat int64 index with three 64-bit div/mods per 16-byte copy made these kernels
// ALU-bound at ~1/10 of HBM bandwidth). V channels per thread: 8 (16-byte copies) when
// C % 8 == 0, else the widest of 4 / 2 / 1 dividing C (RGB inputs, 1-channel masks).
template <typename T, int V>
__global__ void __launch_bounds__(kT)
pad_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int C, int H, int W, int Ho,
               int Wo, int pt, int pl, int mode) {
  const int cv = C / V;
  const int e = blockIdx.x * kT + threadIdx.x;
  if (e >= Wo * cv) return;
  const int ox = e / cv, c8 = e - ox * cv;
  const int sx = pad_src(ox, pl, W, mode);
  for (int row = blockIdx.y; row < B * Ho; row += gridDim.y) {  // row = b * Ho + oy
    const int b = row / Ho, oy = row - b * Ho;
    const int64_t src = (((int64_t)b * H + pad_src(oy, pt, H, mode)) * W + sx) * C + c8 * V;
    *reinterpret_cast<Pack<T, V>*>(y + ((int64_t)row * Wo + ox) * C + c8 * V) =
        *reinterpret_cast<const Pack<T, V>*>(x + src);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(kT)
pad_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int B, int C, int H, int W, int Ho,
               int Wo, int pt, int pb, int pl, int pr, int mode) {
  // grid (ceil(W*C/V / kT), B*H): one block row per input image row (see pad_fwd_kernel); a
  // gather over the (at most kPadMax^2) padded positions that copy this input pixel — no
  // atomics (PyTorch's reflection_pad2d backward scatters with atomics)
  const int cv = C / V;
  const int e = blockIdx.x * kT + threadIdx.x;
  if (e >= W * cv) return;
  const int ix = e / cv, c8 = e - ix * cv;
  int xs[kPadMax];
  const int nx = pad_list(ix, pl, pr, W, mode, xs);
  for (int row = blockIdx.y; row < B * H; row += gridDim.y) {  // row = b * H + iy
    const int b = row / H, iy = row - b * H;
    const int64_t t = (int64_t)row * W * cv + e;
    int ys[kPadMax];
    const int ny = pad_list(iy, pt, pb, H, mode, ys);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    const T* base = dy + (int64_t)b * Ho * Wo * C + c8 * V;
    for (int u = 0; u < ny; ++u)
      for (int v = 0; v < nx; ++v) {
        float g[V];
        load_vec<T, V>(base + ((int64_t)ys[u] * Wo + xs[v]) * C, g);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += g[k];
      }
    store_vec<T, V>(dx + t * V, acc);
  }
}

// Phase scatter of the strided-conv data gradient: dx[b, s*q + ry, s*q2 + rx, c] =
// src[b, i0 + q, j0 + q2, c] for q < Qy, q2 < Qx (both NHWC, C % 8 == 0). The s*s phase
// convolutions (k10) each fill one parity sub-grid of dx; 16-byte loads and stores along C.
__global__ void __launch_bounds__(kT)
phase_scatter_kernel(const __hip_bfloat16* __restrict__ src, __hip_bfloat16* __restrict__ dst,
                     int B, int C, int Hs, int Ws, int H, int W, int s, int ry, int rx, int i0,
                     int j0, int Qy, int Qx) {
  const int cv = C / 8;
  const int64_t total = (int64_t)B * Qy * Qx * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int q2 = (int)(p % Qx);
    p /= Qx;
    const int q = (int)(p % Qy);
    const int b = (int)(p / Qy);
    const uint4 v = *reinterpret_cast<const uint4*>(
        src + (((int64_t)b * Hs + i0 + q) * Ws + j0 + q2) * C + c8 * 8);
    *reinterpret_cast<uint4*>(dst + (((int64_t)b * H + s * q + ry) * W + s * q2 + rx) * C +
                              c8 * 8) = v;
  }
}

// Zero-padded channel copy with dtype cast: y[b, h, w, c] = c < C ? x[b, c, h, w] : 0 for
// c < Cp, y channels-last in TO, x in TI with arbitrary strides (NHWC activations, NCHW image
// batches). One thread per 8 output channels of a pixel: one 16-byte (bf16) / two (fp32)
// stores, instead of a strided zero-fill of the tail plus a strided copy plus a cast pass.
template <typename TI, typename TO>
__global__ void __launch_bounds__(kT)
pad_cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int B, int C, int H, int W, int Cp,
                int64_t sb, int64_t sc, int64_t sh, int64_t sw) {
  const int cv = Cp / 8;
  const int64_t total = (int64_t)B * H * W * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int b = (int)(p / H);
    const TI* xp = x + b * sb + h * sh + w * sw;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 * 8 + k;
      v[k] = c < C ? to_f<TI>(xp[c * sc]) : 0.f;
    }
    store_vec<TO, 8>(y + t * 8, v);
  }
}

// (in-row blocks, rows): rows beyond the grid's y limit are walked by a grid-stride loop
dim3 pad_rows_grid(int64_t per_row, int64_t rows) {
  IAMD_CHECK(per_row < (1ll << 30) && rows < (1ll << 31), "pad_nhwc: tensor too large");
  return dim3((unsigned)((per_row + kT - 1) / kT), (unsigned)std::min<int64_t>(rows, 65535));
}

int pad_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kT - 1) / kT, 65536)); }

}  // namespace

// x [B, C, H, W] channels-last (C % 8 == 0, bf16 / fp32) -> padded [B, C, H+pt+pb, W+pl+pr];
// mode 0 reflect, 1 replicate.
namespace {
// out[p, 0:ca] = a[p], out[p, ca:ca+cb] = b[p], out[p, ca+cb:cp] = 0 for every pixel p of NHWC
// tensors: one 8-channel output group per lane, 16-byte (bf16) stores; the sources' odd channel
// counts (the 185-channel COCO-Stuff label) are gathered element-wise, coalesced across lanes.
template <typename T>
__global__ void __launch_bounds__(256) nhwc_concat_kernel(const T* __restrict__ a,
                                                         const T* __restrict__ b,
                                                         T* __restrict__ out, int64_t P, int ca,
                                                         int cb, int cp) {
  const int G = cp / 8;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= P * G) return;
  const int64_t p = idx / G;
  const int c0 = (int)(idx - p * G) * 8;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    v[k] = c < ca ? to_f<T>(a[p * ca + c])
                  : (c < ca + cb ? to_f<T>(b[p * cb + (c - ca)]) : 0.f);
  }
  store_vec<T, 8>(out + p * cp + c0, v);
}
}  // namespace

// Write cat(a, b, zeros) along channels into ``out`` (all NHWC-dense: [N, C, H, W] with
// channels-last strides, same N/H/W; out has cp >= ca + cb channels, cp % 8 == 0): the
// discriminator input ``cat(label, image)`` in one pass (the strided slice copies ran on
// PyTorch's generic element-offset copy kernel).
void nhwc_concat_into(at::Tensor& out, const at::Tensor& a, const at::Tensor& b) {
  auto cl = at::MemoryFormat::ChannelsLast;
  IAMD_CHECK(out.dim() == 4 && a.dim() == 4 && b.dim() == 4 && out.is_cuda(),
             "nhwc_concat_into: 4-D CUDA tensors expected");
  IAMD_CHECK(out.is_contiguous(cl) && a.is_contiguous(cl) && b.is_contiguous(cl),
             "nhwc_concat_into: channels-last dense tensors expected");
  IAMD_CHECK(a.scalar_type() == out.scalar_type() && b.scalar_type() == out.scalar_type(),
             "nhwc_concat_into: one dtype expected");
  const int64_t N = out.size(0), H = out.size(2), W = out.size(3);
  IAMD_CHECK(a.size(0) == N && b.size(0) == N && a.size(2) == H && b.size(2) == H &&
                 a.size(3) == W && b.size(3) == W,
             "nhwc_concat_into: batch / spatial sizes differ");
  const int ca = (int)a.size(1), cb = (int)b.size(1), cp = (int)out.size(1);
  IAMD_CHECK(cp % 8 == 0 && ca + cb <= cp, "nhwc_concat_into: channel counts");
  const int64_t P = N * H * W;
  if (P == 0) return;
  IAMD_DISPATCH_FLOAT_TYPES(out.scalar_type(), "nhwc_concat_into", [&] {
    hipLaunchKernelGGL((nhwc_concat_kernel<scalar_t>), dim3(ceil_div(P * (cp / 8), 256)),
                       dim3(256), 0, stream(), reinterpret_cast<const scalar_t*>(a.data_ptr()),
                       reinterpret_cast<const scalar_t*>(b.data_ptr()),
                       reinterpret_cast<scalar_t*>(out.data_ptr()), P, ca, cb, cp);
  });
  IAMD_LAUNCH_CHECK();
}

namespace {
int pad_vec(int C) { return C % 8 == 0 ? 8 : C % 4 == 0 ? 4 : C % 2 == 0 ? 2 : 1; }

template <typename F>
void by_pad_vec(at::ScalarType st, int V, F&& f) {
  auto by_v = [&](auto tv) {
    switch (V) {
      case 8: f(tv, std::integral_constant<int, 8>()); break;
      case 4: f(tv, std::integral_constant<int, 4>()); break;
      case 2: f(tv, std::integral_constant<int, 2>()); break;
      default: f(tv, std::integral_constant<int, 1>()); break;
    }
  };
  if (st == at::kBFloat16) by_v(__hip_bfloat16());
  else by_v(float());
}
}  // namespace

at::Tensor pad_nhwc_fwd(const at::Tensor& x, int64_t pl, int64_t pr, int64_t pt, int64_t pb,
                        int64_t mode) {
  IAMD_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
             "pad_nhwc_fwd: packed channels-last bf16/fp32 tensor expected");
  const int B = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  IAMD_CHECK(pl >= 0 && pr >= 0 && pt >= 0 && pb >= 0 && (mode == 1 ||
             (pl < W && pr < W && pt < H && pb < H)), "pad_nhwc_fwd: bad padding");
  const int Ho = (int)(H + pt + pb), Wo = (int)(W + pl + pr);
  auto y = at::empty({B, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if ((int64_t)B * Ho * Wo * C == 0) return y;
  const int V = pad_vec(C);
  auto launch = [&](auto tv, auto vv) {
    using T = decltype(tv);
    constexpr int VV = decltype(vv)::value;
    hipLaunchKernelGGL((pad_fwd_kernel<T, VV>), pad_rows_grid(Wo * (C / VV), B * Ho), dim3(kT), 0,
                       stream(), reinterpret_cast<const T*>(x.data_ptr()),
                       reinterpret_cast<T*>(y.data_ptr()), B, C, H, W, Ho, Wo, (int)pt, (int)pl,
                       (int)mode);
  };
  by_pad_vec(x.scalar_type(), V, launch);
  IAMD_LAUNCH_CHECK();
  return y;
}

at::Tensor pad_nhwc_bwd(const at::Tensor& dy, int64_t H, int64_t W, int64_t pl, int64_t pr,
                        int64_t pt, int64_t pb, int64_t mode) {
  IAMD_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat) &&
                 dy.size(2) == H + pt + pb && dy.size(3) == W + pl + pr,
             "pad_nhwc_bwd: gradient shape / layout");
  IAMD_CHECK(mode == 0 || (pt + 1 <= kPadMax && pb + 1 <= kPadMax && pl + 1 <= kPadMax &&
                           pr + 1 <= kPadMax), "pad_nhwc_bwd: replicate padding above 15");
  const int B = (int)dy.size(0), C = (int)dy.size(1);
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  if ((int64_t)B * H * W * C == 0) return dx;
  const int V = pad_vec(C);
  auto launch = [&](auto tv, auto vv) {
    using T = decltype(tv);
    constexpr int VV = decltype(vv)::value;
    hipLaunchKernelGGL((pad_bwd_kernel<T, VV>), pad_rows_grid((int)W * (C / VV), B * (int)H),
                       dim3(kT), 0, stream(), reinterpret_cast<const T*>(dy.data_ptr()),
                       reinterpret_cast<T*>(dx.data_ptr()), B, C, (int)H, (int)W,
                       (int)dy.size(2), (int)dy.size(3), (int)pt, (int)pb, (int)pl, (int)pr,
                       (int)mode);
  };
  by_pad_vec(dy.scalar_type(), V, launch);
  IAMD_LAUNCH_CHECK();
  return dx;
}

// w: [Cout, Cin, KH, KW] bf16 channels-last -> [Cin, Cout, Jy, Jx] bf16 channels-last with
// wt[ci][jy][jx][co] = w[co][qy + s (Jy-1-jy)][qx + s (Jx-1-jx)][ci], Jy = ceil((KH-qy)/s)
// (s = 1, q = 0: the spatially flipped, in/out-transposed weight of the stride-1 dgrad).
// nb > 1: w holds nb per-sample weights [nb * Cout, ...] -> [nb * Cin, Cout, Jy, Jx].
at::Tensor conv_weight_flip_t(const at::Tensor& w, int64_t s, int64_t qy, int64_t qx,
                              int64_t nb) {
  IAMD_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kBFloat16,
             "conv_weight_flip_t: 4-D bf16 CUDA weight expected");
  IAMD_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv_weight_flip_t: packed channels-last weight expected");
  IAMD_CHECK(nb >= 1 && w.size(0) % nb == 0, "conv_weight_flip_t: rows not divisible by nb");
  const int Cout = (int)(w.size(0) / nb), Cin = (int)w.size(1), KH = (int)w.size(2),
            KW = (int)w.size(3);
  IAMD_CHECK(Cout % 8 == 0 && Cin % 8 == 0, "conv_weight_flip_t: channels must be multiples of 8");
  IAMD_CHECK(s >= 1 && qy >= 0 && qx >= 0 && qy < KH && qx < KW, "conv_weight_flip_t: bad phase");
  const int Jy = (int)((KH - qy + s - 1) / s), Jx = (int)((KW - qx + s - 1) / s);
  auto wt = at::empty({nb * Cin, Cout, Jy, Jx},
                      w.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (wt.numel() == 0) return wt;
  const dim3 grid(ceil_div(Cin, kTile), ceil_div(Cout, kTile), (unsigned)(nb * Jy * Jx));
  hipLaunchKernelGGL(flip_t_kernel, grid, dim3(kT), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(w.data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(wt.data_ptr()), Cout, Cin, KH, KW, Jy, Jx,
                     (int)s, (int)qy, (int)qx);
  IAMD_LAUNCH_CHECK();
  return wt;
}

// Every phase sub-kernel of a stride-s conv weight in ONE launch (the strided data gradient's
// s*s phase convolutions, conv_mfma.hip conv2d_dgrad_strided): original tap (ky, kx) belongs to
// phase (ky mod s, kx mod s) at in-phase position ((ky - qy) / s, (kx - qx) / s), stored flipped
// into that phase's [Cin][Jy][Jx][Cout] block of one flat buffer (block offsets poff[phase]).
// Replaces s*s flip_t launches per strided conv (~85 small launches per SPADE step).
namespace {
struct PhaseOffsets {
  int64_t off[16];
};

__global__ void __launch_bounds__(kT)
phase_flip_kernel(const __hip_bfloat16* __restrict__ w, __hip_bfloat16* __restrict__ out,
                  int Cout, int Cin, int KH, int KW, int s, PhaseOffsets po) {
  __shared__ __hip_bfloat16 tile[kTile * kLdsStride];
  const int ci0 = blockIdx.x * kTile, co0 = blockIdx.y * kTile;
  const int ky = blockIdx.z / KW, kx = blockIdx.z - (blockIdx.z / KW) * KW;
  const int qy = ky % s, qx = kx % s;
  const int Jy = (KH - qy + s - 1) / s, Jx = (KW - qx + s - 1) / s;
  const int jy = Jy - 1 - (ky - qy) / s, jx = Jx - 1 - (kx - qx) / s;
  const int JJ = Jy * Jx, tap = jy * Jx + jx;
  __hip_bfloat16* wt = out + po.off[qy * s + qx];
  const int tid = threadIdx.x;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int e = tid + r * kT;
    const int row = e >> 3, ch = e & 7;
    const int co = co0 + row, ci = ci0 + ch * 8;
    Pack<__hip_bfloat16, 8> v;
    if (co < Cout && ci < Cin) {
      v = *reinterpret_cast<const Pack<__hip_bfloat16, 8>*>(
          w + ((int64_t)co * KH * KW + blockIdx.z) * Cin + ci);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v.v[k] = __float2bfloat16(0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[row * kLdsStride + ch * 8 + k] = v.v[k];
  }
  __syncthreads();
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
}  // namespace

// w [Cout, Cin, KH, KW] bf16 channels-last, stride s (2..4) -> the s*s phase weights
// conv_weight_flip_t(w, s, qy, qx) for (qy, qx) in row-major phase order, as channels-last views
// of one buffer (an empty view for a phase without taps).
std::vector<at::Tensor> conv_weight_phase_flip(const at::Tensor& w, int64_t s) {
  IAMD_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kBFloat16 &&
                 w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv_weight_phase_flip: packed channels-last 4-D bf16 CUDA weight expected");
  IAMD_CHECK(s >= 1 && s <= 4, "conv_weight_phase_flip: stride must be 1..4");
  const int Cout = (int)w.size(0), Cin = (int)w.size(1), KH = (int)w.size(2), KW = (int)w.size(3);
  IAMD_CHECK(Cout % 8 == 0 && Cin % 8 == 0,
             "conv_weight_phase_flip: channels must be multiples of 8");
  PhaseOffsets po;
  std::vector<std::array<int64_t, 3>> shp;  // (Jy, Jx, offset)
  int64_t off = 0;
  for (int qy = 0; qy < s; ++qy)
    for (int qx = 0; qx < s; ++qx) {
      const int64_t Jy = qy < KH ? (KH - qy + s - 1) / s : 0;
      const int64_t Jx = qx < KW ? (KW - qx + s - 1) / s : 0;
      po.off[qy * s + qx] = off;
      shp.push_back({Jy, Jx, off});
      off += (int64_t)Cin * Cout * Jy * Jx;
    }
  auto flat = at::empty({std::max<int64_t>(off, 1)}, w.options());
  std::vector<at::Tensor> out;
  for (auto& e : shp)
    out.push_back(flat.as_strided({Cin, Cout, e[0], e[1]},
                                  {e[0] * e[1] * Cout, 1, e[1] * Cout, Cout}, e[2]));
  if (off == 0) return out;
  const dim3 grid(ceil_div(Cin, kTile), ceil_div(Cout, kTile), (unsigned)(KH * KW));
  hipLaunchKernelGGL(phase_flip_kernel, grid, dim3(kT), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(w.data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(flat.data_ptr()), Cout, Cin, KH, KW, (int)s,
                     po);
  IAMD_LAUNCH_CHECK();
  return out;
}

namespace {

// ---- multi-tensor plain flip (s = 1): every stride-1 conv weight of a network in one launch --
// The data gradient of each stride-1 conv needs its flipped, transposed weight. Flipping in the
// conv's backward costs one small launch per layer (~220 per SPADE step, 1.26 ms,
// profiles/spade_step_latest_mi355x.txt); the spectral-norm group that produces every layer's
// bf16 W / sigma in one launch (sn_power.hip k5c) flips them all right after it, in one more.
struct FlipEntry {
  int64_t src;  // element offset of the source weight from the base pointer (may be < 0)
  int64_t dst;  // element offset in the flat output
  int Cout, Cin, KH, KW, nci, nco;
};

__global__ void __launch_bounds__(kT)
mt_flip_kernel(const FlipEntry* __restrict__ ents, const int* __restrict__ blocks,
               const __hip_bfloat16* __restrict__ base, __hip_bfloat16* __restrict__ out) {
  __shared__ __hip_bfloat16 tile[kTile * kLdsStride];
  const FlipEntry e = ents[blocks[2 * blockIdx.x]];
  int b = blocks[2 * blockIdx.x + 1];
  const int KK = e.KH * e.KW;
  const int tap = b % KK;
  b /= KK;
  const int cit = b % e.nci, cot = b / e.nci;
  const int ci0 = cit * kTile, co0 = cot * kTile;
  const int jy = tap / e.KW, jx = tap - jy * e.KW;
  const int ftap = (e.KH - 1 - jy) * e.KW + (e.KW - 1 - jx);
  const __hip_bfloat16* w = base + e.src;
  __hip_bfloat16* wt = out + e.dst;
  const int tid = threadIdx.x;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = tid + r * kT;
    const int row = q >> 3, ch = q & 7;
    const int co = co0 + row, ci = ci0 + ch * 8;
    Pack<__hip_bfloat16, 8> v;
    if (co < e.Cout && ci < e.Cin) {
      v = *reinterpret_cast<const Pack<__hip_bfloat16, 8>*>(
          w + ((int64_t)co * KK + ftap) * e.Cin + ci);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v.v[k] = __float2bfloat16(0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[row * kLdsStride + ch * 8 + k] = v.v[k];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = tid + r * kT;
    const int row = q >> 3, ch = q & 7;
    const int ci = ci0 + row, co = co0 + ch * 8;
    if (ci >= e.Cin || co >= e.Cout) continue;
    Pack<__hip_bfloat16, 8> v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v.v[k] = tile[(ch * 8 + k) * kLdsStride + row];
    *reinterpret_cast<Pack<__hip_bfloat16, 8>*>(wt + ((int64_t)ci * KK + tap) * e.Cout + co) = v;
  }
}

struct FlipPlan {
  at::Tensor ents, blocks;
  int nblocks;
  int64_t total;
  std::vector<int64_t> offs;
};
std::mutex g_flip_mu;
std::unordered_map<uint64_t, FlipPlan> g_flip_cache;

}  // namespace

// Plain flips wt[ci][kh][kw][co] = w[co][KH-1-kh][KW-1-kw][ci] of every weight in ``ws`` (bf16,
// channels-last, channels multiples of 8) into ONE flat buffer, one launch. The launch plan is
// cached on the weights' shapes and their offsets from ws[0] (the views of one flat buffer
// keep them from call to call).
std::vector<at::Tensor> mt_conv_weight_flip_t(const std::vector<at::Tensor>& ws) {
  IAMD_CHECK(!ws.empty(), "mt_conv_weight_flip_t: empty list");
  const char* base = reinterpret_cast<const char*>(ws[0].data_ptr());
  uint64_t h = 0x9E3779B97F4A7C15ULL;
  for (auto& w : ws) {
    IAMD_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kBFloat16 &&
                   w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(0) % 8 == 0 &&
                   w.size(1) % 8 == 0 && w.device() == ws[0].device(),
               "mt_conv_weight_flip_t: channels-last bf16 weights with channels % 8 == 0");
    const int64_t rel = reinterpret_cast<const char*>(w.data_ptr()) - base;
    IAMD_CHECK(rel % 2 == 0, "mt_conv_weight_flip_t: misaligned weight");
    for (int64_t v : {rel, w.size(0), w.size(1), w.size(2), w.size(3)})
      h ^= (uint64_t)v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  }
  FlipPlan* pp;
  {
    std::lock_guard<std::mutex> lk(g_flip_mu);
    auto it = g_flip_cache.find(h);
    if (it == g_flip_cache.end()) {
      FlipPlan p;
      std::vector<FlipEntry> ents;
      std::vector<int32_t> bm;
      int64_t off = 0;
      for (size_t i = 0; i < ws.size(); ++i) {
        const auto& w = ws[i];
        FlipEntry e;
        e.src = (reinterpret_cast<const char*>(w.data_ptr()) - base) / 2;
        e.dst = off;
        e.Cout = (int)w.size(0); e.Cin = (int)w.size(1); e.KH = (int)w.size(2);
        e.KW = (int)w.size(3);
        e.nci = ceil_div(e.Cin, kTile);
        e.nco = ceil_div(e.Cout, kTile);
        ents.push_back(e);
        p.offs.push_back(off);
        const int nb = e.nci * e.nco * e.KH * e.KW;
        for (int b = 0; b < nb; ++b) {
          bm.push_back((int32_t)i);
          bm.push_back(b);
        }
        off += (w.numel() + 7) / 8 * 8;
      }
      p.total = off;
      p.ents = stage_to_device(ents.data(), ents.size() * sizeof(FlipEntry), ws[0].device());
      p.blocks = stage_to_device(bm.data(), bm.size() * sizeof(int32_t), ws[0].device())
                     .view(at::kInt);
      p.nblocks = (int)(bm.size() / 2);
      if (g_flip_cache.size() > 64) g_flip_cache.clear();
      it = g_flip_cache.emplace(h, std::move(p)).first;
    }
    pp = &it->second;
    keep_for_graph(pp->ents);
    keep_for_graph(pp->blocks);
  }
  auto flat = at::empty({pp->total}, ws[0].options());
  hipLaunchKernelGGL(mt_flip_kernel, dim3(pp->nblocks), dim3(kT), 0, stream(),
                     reinterpret_cast<const FlipEntry*>(pp->ents.data_ptr()),
                     pp->blocks.data_ptr<int>(),
                     reinterpret_cast<const __hip_bfloat16*>(ws[0].data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(flat.data_ptr()));
  IAMD_LAUNCH_CHECK();
  std::vector<at::Tensor> out;
  for (size_t i = 0; i < ws.size(); ++i) {
    const auto& w = ws[i];
    const int64_t co = w.size(0), ci = w.size(1), kh = w.size(2), kw = w.size(3);
    // [Cin, Cout, KH, KW] channels-last: strides (KH*KW*Cout, 1, KW*Cout, Cout)
    out.push_back(flat.as_strided({ci, co, kh, kw}, {kh * kw * co, 1, kw * co, co}, pp->offs[i]));
  }
  return out;
}

// part: fp32 [S * Cop * KK * Cip] -> [Cout, Cin, KH, KW] channels-last in `dtype`.
// dst_opt: write into this tensor instead (the DDP bucket slice of the parameter's gradient:
// [Cout, Cin, KH, KW] channels-last in `dtype`), so no copy into the bucket follows.
static at::Tensor finalize_out(const at::Tensor& part, int64_t Cout, int64_t Cin, int64_t KH,
                               int64_t KW, at::ScalarType dtype,
                               const c10::optional<at::Tensor>& dst_opt) {
  if (dst_opt.has_value() && dst_opt->defined()) {
    const at::Tensor& d = *dst_opt;
    IAMD_CHECK(d.is_cuda() && d.scalar_type() == dtype && d.dim() == 4 && d.size(0) == Cout &&
                   d.size(1) == Cin && d.size(2) == KH && d.size(3) == KW &&
                   d.is_contiguous(at::MemoryFormat::ChannelsLast),
               "wgrad_finalize: the destination must be a channels-last [Cout, Cin, KH, KW] "
               "tensor of the gradient dtype");
    return d;
  }
  return at::empty({Cout, Cin, KH, KW},
                   part.options().dtype(dtype).memory_format(at::MemoryFormat::ChannelsLast));
}

at::Tensor wgrad_finalize(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                          int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                          at::ScalarType dtype, const c10::optional<at::Tensor>& dst) {
  IAMD_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous(),
             "wgrad_finalize: contiguous fp32 slabs expected");
  IAMD_CHECK(part.numel() >= S * Cop * KH * KW * Cip && Cout <= Cop && Cin <= Cip,
             "wgrad_finalize: slab shape");
  auto out = finalize_out(part, Cout, Cin, KH, KW, dtype, dst);
  const int KK = (int)(KH * KW);
  const bool vec = Cin % 4 == 0 && Cip % 4 == 0;
  const int64_t n = Cout * KK * (vec ? Cin / 4 : Cin);
  if (n == 0) return out;
  int G = 1;  // slab groups per output: more of them when there are many slabs, few outputs
  while (G < 16 && G < S && (n * G * 2 <= (int64_t)256 * 4096 || G * 8 < S)) G *= 2;
  const int opb = kT / G;
  const int blocks = (int)std::min<int64_t>((n + opb - 1) / opb, 8192);
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    if (vec)
      hipLaunchKernelGGL((wgrad_finalize_kernel<T, true>), dim3(blocks), dim3(kT), 0, stream(),
                         part.data_ptr<float>(), reinterpret_cast<T*>(out.data_ptr()), (int)S,
                         (int)Cop, (int)Cip, (int)Cout, (int)Cin, KK, G);
    else
      hipLaunchKernelGGL((wgrad_finalize_kernel<T, false>), dim3(blocks), dim3(kT), 0, stream(),
                         part.data_ptr<float>(), reinterpret_cast<T*>(out.data_ptr()), (int)S,
                         (int)Cop, (int)Cip, (int)Cout, (int)Cin, KK, G);
  };
  if (dtype == at::kBFloat16) launch(__hip_bfloat16());
  else if (dtype == at::kFloat) launch(float());
  else IAMD_CHECK(false, "wgrad_finalize: bf16 or fp32 output expected");
  IAMD_LAUNCH_CHECK();
  return out;
}

at::Tensor wgrad_finalize_sn(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                             int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                             const at::Tensor& dotp, const at::Tensor& u, const at::Tensor& v,
                             const at::Tensor& sigma, const c10::optional<at::Tensor>& dst) {
  IAMD_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                 part.numel() >= S * Cop * KH * KW * Cip && Cout <= Cop && Cin <= Cip,
             "wgrad_finalize_sn: slab shape");
  IAMD_CHECK(dotp.scalar_type() == at::kFloat && u.scalar_type() == at::kFloat &&
                 v.scalar_type() == at::kFloat && sigma.scalar_type() == at::kFloat &&
                 u.numel() == Cout && v.numel() == Cin * KH * KW && sigma.numel() == 1 &&
                 u.is_contiguous() && v.is_contiguous() && dotp.is_contiguous(),
             "wgrad_finalize_sn: u / v / sigma / partials");
  auto out = finalize_out(part, Cout, Cin, KH, KW, at::kFloat, dst);
  const int KK = (int)(KH * KW);
  const bool vec = Cin % 4 == 0 && Cip % 4 == 0;
  const int64_t n = Cout * KK * (vec ? Cin / 4 : Cin);
  if (n == 0) return out;
  int G = 1;
  while (G < 16 && G < S && (n * G * 2 <= (int64_t)256 * 4096 || G * 8 < S)) G *= 2;
  const int opb = kT / G;
  const int blocks = (int)std::min<int64_t>((n + opb - 1) / opb, 8192);
  if (vec)
    hipLaunchKernelGGL((wgrad_finalize_sn_kernel<true>), dim3(blocks), dim3(kT), 0, stream(),
                       part.data_ptr<float>(), out.data_ptr<float>(), (int)S, (int)Cop, (int)Cip,
                       (int)Cout, (int)Cin, KK, G, dotp.data_ptr<float>(), (int)dotp.numel(),
                       u.data_ptr<float>(), v.data_ptr<float>(), sigma.data_ptr<float>());
  else
    hipLaunchKernelGGL((wgrad_finalize_sn_kernel<false>), dim3(blocks), dim3(kT), 0, stream(),
                       part.data_ptr<float>(), out.data_ptr<float>(), (int)S, (int)Cop, (int)Cip,
                       (int)Cout, (int)Cin, KK, G, dotp.data_ptr<float>(), (int)dotp.numel(),
                       u.data_ptr<float>(), v.data_ptr<float>(), sigma.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  return out;
}

namespace {
// scale * sum over pixels p and channels c < C of a[p * Ca + c] * b[p * Cb + c] (bf16, packed
// channels-last, C % 8 == 0): one fp32 partial per block, fixed grid and order (deterministic)
constexpr int kDotBlocks = 512;
__global__ void __launch_bounds__(kT)
sn_dot_kernel(const __hip_bfloat16* __restrict__ a, const __hip_bfloat16* __restrict__ b,
              int64_t P, int Ca, int Cb, int C, const float* __restrict__ scale,
              float* __restrict__ part) {
  const int cv = C / 8;
  const int64_t n = P * cv;
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    const int64_t p = i / cv;
    const int c = (int)(i - p * cv) * 8;
    float x[8], y[8];
    load_vec<__hip_bfloat16, 8>(a + p * Ca + c, x);
    load_vec<__hip_bfloat16, 8>(b + p * Cb + c, y);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = fmaf(x[k], y[k], acc);
  }
  __shared__ float red[kT / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kT / 64; ++k) t += red[k];
    part[blockIdx.x] = t * (scale ? scale[0] : 1.f);
  }
}
}  // namespace

// <G, W> of a spectrally normalised conv from its data gradient: for y = conv(x, W) / sigma,
// <G, W> = sum_m dy_m . conv(x, W)_m = <conv^T(dy, W), x> = sigma * <dx, x> (the adjoint
// identity; any stride / padding / dilation). dx [B, Ca, H, W] is the k10 data gradient
// (1 / sigma applied), x [B, Cb, H, W] the conv's bf16 input; channels >= min(Ca, Cb) are zero
// in whichever operand has them. Returns kDotBlocks partials whose sum is <G, W> — the dotp of
// wgrad_finalize_sn, replacing the k11 epilogue's per-block W reads where the activation is
// smaller than the weight (deep, low-resolution layers).
at::Tensor sn_dot_partials(const at::Tensor& dx, const at::Tensor& x, const at::Tensor& sigma) {
  IAMD_CHECK(dx.is_cuda() && x.is_cuda() && dx.scalar_type() == at::kBFloat16 &&
                 x.scalar_type() == at::kBFloat16 && dx.dim() == 4 && x.dim() == 4 &&
                 dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 x.is_contiguous(at::MemoryFormat::ChannelsLast) && dx.size(0) == x.size(0) &&
                 dx.size(2) == x.size(2) && dx.size(3) == x.size(3),
             "sn_dot_partials: packed channels-last bf16 [B, C, H, W] operands of one shape");
  IAMD_CHECK(sigma.scalar_type() == at::kFloat && sigma.numel() == 1, "sn_dot_partials: sigma");
  const int Ca = (int)dx.size(1), Cb = (int)x.size(1), C = std::min(Ca, Cb);
  IAMD_CHECK(C % 8 == 0 && Ca % 8 == 0 && Cb % 8 == 0, "sn_dot_partials: channels % 8");
  auto part = at::empty({kDotBlocks}, x.options().dtype(at::kFloat));
  const int64_t P = x.size(0) * x.size(2) * x.size(3);
  hipLaunchKernelGGL(sn_dot_kernel, dim3(kDotBlocks), dim3(kT), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(dx.data_ptr()),
                     reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()), P, Ca, Cb, C,
                     sigma.data_ptr<float>(), part.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  return part;
}

// src [B, C, Hs, Ws] -> the (ry, rx) parity sub-grid of dst [B, C, H, W] (both channels-last bf16)
void conv_phase_scatter(const at::Tensor& src, at::Tensor& dst, int64_t s, int64_t ry, int64_t rx,
                        int64_t i0, int64_t j0, int64_t Qy, int64_t Qx) {
  IAMD_CHECK(src.is_cuda() && dst.is_cuda() && src.scalar_type() == at::kBFloat16 &&
                 dst.scalar_type() == at::kBFloat16 && src.dim() == 4 && dst.dim() == 4 &&
                 src.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 dst.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv_phase_scatter: packed channels-last bf16 tensors expected");
  const int B = (int)src.size(0), C = (int)src.size(1), Hs = (int)src.size(2), Ws = (int)src.size(3);
  const int H = (int)dst.size(2), W = (int)dst.size(3);
  IAMD_CHECK(dst.size(0) == B && dst.size(1) == C && C % 8 == 0, "conv_phase_scatter: shapes");
  IAMD_CHECK(Qy >= 0 && Qx >= 0 && i0 >= 0 && j0 >= 0 && i0 + Qy <= Hs && j0 + Qx <= Ws &&
                 ry >= 0 && rx >= 0 && ry < s && rx < s && s * (Qy - 1) + ry < H + (Qy == 0) * s &&
                 s * (Qx - 1) + rx < W + (Qx == 0) * s,
             "conv_phase_scatter: phase window out of range");
  const int64_t total = (int64_t)B * Qy * Qx * (C / 8);
  if (total == 0) return;
  hipLaunchKernelGGL(phase_scatter_kernel, dim3(pad_grid(total)), dim3(kT), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(src.data_ptr()),
                     reinterpret_cast<__hip_bfloat16*>(dst.data_ptr()), B, C, Hs, Ws, H, W, (int)s,
                     (int)ry, (int)rx, (int)i0, (int)j0, (int)Qy, (int)Qx);
  IAMD_LAUNCH_CHECK();
}

// x [B, C, H, W] (bf16 / fp32, any strides) -> channels-last [B, Cp, H, W] in `dtype`, channels
// C..Cp-1 zero (Cp % 8 == 0, Cp >= C)
at::Tensor pad_channels_cast(const at::Tensor& x, int64_t Cp, at::ScalarType dtype) {
  IAMD_CHECK(x.is_cuda() && x.dim() == 4, "pad_channels_cast: 4-D CUDA tensor expected");
  IAMD_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
             "pad_channels_cast: bf16 / fp32 input");
  IAMD_CHECK(dtype == at::kBFloat16 || dtype == at::kFloat, "pad_channels_cast: bf16 / fp32 out");
  const int B = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  IAMD_CHECK(Cp % 8 == 0 && Cp >= C, "pad_channels_cast: Cp must be a multiple of 8 >= C");
  auto y = at::empty({B, Cp, H, W}, x.options().dtype(dtype).memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = (int64_t)B * H * W * (Cp / 8);
  if (total == 0) return y;
  auto launch = [&](auto ti, auto to) {
    using TI = decltype(ti);
    using TO = decltype(to);
    hipLaunchKernelGGL((pad_cast_kernel<TI, TO>), dim3(pad_grid(total)), dim3(kT), 0, stream(),
                       reinterpret_cast<const TI*>(x.data_ptr()), reinterpret_cast<TO*>(y.data_ptr()),
                       B, C, H, W, (int)Cp, x.stride(0), x.stride(1), x.stride(2), x.stride(3));
  };
  const bool ib = x.scalar_type() == at::kBFloat16, ob = dtype == at::kBFloat16;
  if (ib && ob) launch(__hip_bfloat16(), __hip_bfloat16());
  else if (ib) launch(__hip_bfloat16(), float());
  else if (ob) launch(float(), __hip_bfloat16());
  else launch(float(), float());
  IAMD_LAUNCH_CHECK();
  return y;
}


// ---- test support: fill the LDS of every CU with a NaN bit pattern ---------------------------
// LDS is not cleared between workgroups, so a kernel that reads LDS it never wrote picks up
// whatever the previous workgroup on that CU left there — in a hipGraph replay a different
// predecessor than in an eager run. Running this right before a kernel under test turns such a
// read into NaN outputs (tests/test_kernels_gpu.py).
namespace {
constexpr int kPoisonBytes = 160 * 1024;
__global__ void __launch_bounds__(256) lds_poison_kernel(int iters) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[kPoisonBytes / 4];
  volatile uint32_t* vb = buf;  // volatile: the stores have no reader and must not be dropped
  for (int it = 0; it < iters; ++it)
    for (int i = threadIdx.x; i < kPoisonBytes / 4; i += 256) vb[i] = 0xffffffffu;
}
}  // namespace

void lds_poison(int64_t blocks) {
  hipLaunchKernelGGL(lds_poison_kernel, dim3((unsigned)std::max<int64_t>(1, blocks)), dim3(256),
                     0, stream(), 1);
  IAMD_LAUNCH_CHECK();
}

}  // namespace iamd
