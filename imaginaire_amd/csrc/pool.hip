// k14: NHWC average pooling (bf16 / fp32, any kernel / stride / padding, count_include_pad
// either way) with a GATHER backward.
//
// The discriminators downsample with average pools: the ResDiscriminator of MUNIT / UNIT
// (reference discriminators/residual.py:66, AvgPool2d(2)), the SPADE / FPSE label pyramids
// (discriminators/spade.py, fpse.py:119-122), pix2pixHD's and vid2vid's 3x3 stride-2
// downsamplers (generators/pix2pixHD.py, vid2vid.py). PyTorch's channels-last avg_pool2d
// backward ran at a small fraction of HBM bandwidth (~4.6% of a MUNIT iteration,
// profiles/recipe_munit256_kernels_mi355x.txt). Here:
//   * forward: one thread per (output pixel, 8 channels): k*k 16-byte loads, one 16-byte store;
//   * backward: one thread per (input pixel, 8 channels) sums dy / count over exactly the
//     output windows that cover it — no atomics, deterministic, one 16-byte store.
#include "common.h"

#include <cmath>

namespace iamd {
namespace {

constexpr int kT = 256;

struct PoolGeom {
  int B, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw;
  bool include_pad;
};

__device__ __forceinline__ float window_count(const PoolGeom& g, int oy, int ox) {
  const int y0 = oy * g.sh - g.ph, x0 = ox * g.sw - g.pw;
  if (g.include_pad) {
    // PyTorch: the window clipped to the PADDED extent
    const int y1 = min(y0 + g.kh, g.H + g.ph), x1 = min(x0 + g.kw, g.W + g.pw);
    return (float)((y1 - y0) * (x1 - x0));
  }
  const int ya = max(y0, 0), xa = max(x0, 0);
  const int yb = min(y0 + g.kh, g.H), xb = min(x0 + g.kw, g.W);
  return (float)((yb - ya) * (xb - xa));
}

// V channels per thread: 8 (16-byte accesses) when C % 8 == 0, else 1 (the 185-channel COCO
// label maps the FPSE discriminator pools)
template <typename T, int V>
__global__ void __launch_bounds__(kT)
avgpool_fwd(const T* __restrict__ x, T* __restrict__ y, PoolGeom g) {
  const int cv = g.C / V;
  const int64_t total = (int64_t)g.B * g.Ho * g.Wo * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ox = (int)(p % g.Wo);
    p /= g.Wo;
    const int oy = (int)(p % g.Ho);
    const int b = (int)(p / g.Ho);
    const int y0 = oy * g.sh - g.ph, x0 = ox * g.sw - g.pw;
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int dy = 0; dy < g.kh; ++dy) {
      const int iy = y0 + dy;
      if (iy < 0 || iy >= g.H) continue;
      for (int dx = 0; dx < g.kw; ++dx) {
        const int ix = x0 + dx;
        if (ix < 0 || ix >= g.W) continue;
        float v[V];
        load_vec<T, V>(x + (((int64_t)b * g.H + iy) * g.W + ix) * g.C + c8 * V, v);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += v[k];
      }
    }
    const float inv = 1.f / window_count(g, oy, ox);
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] *= inv;
    store_vec<T, V>(y + t * V, acc);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(kT)
avgpool_bwd(const T* __restrict__ dy, T* __restrict__ dx, PoolGeom g) {
  const int cv = g.C / V;
  const int64_t total = (int64_t)g.B * g.H * g.W * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ix = (int)(p % g.W);
    p /= g.W;
    const int iy = (int)(p % g.H);
    const int b = (int)(p / g.H);
    // output rows whose window [oy*sh - ph, oy*sh - ph + kh) contains iy
    const int oy_lo = max(0, (iy + g.ph - g.kh + g.sh) / g.sh);
    const int oy_hi = min(g.Ho - 1, (iy + g.ph) / g.sh);
    const int ox_lo = max(0, (ix + g.pw - g.kw + g.sw) / g.sw);
    const int ox_hi = min(g.Wo - 1, (ix + g.pw) / g.sw);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      if (iy < oy * g.sh - g.ph || iy >= oy * g.sh - g.ph + g.kh) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        if (ix < ox * g.sw - g.pw || ix >= ox * g.sw - g.pw + g.kw) continue;
        float v[V];
        load_vec<T, V>(dy + (((int64_t)b * g.Ho + oy) * g.Wo + ox) * g.C + c8 * V, v);
        const float inv = 1.f / window_count(g, oy, ox);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += v[k] * inv;
      }
    }
    store_vec<T, V>(dx + t * V, acc);
  }
}

// NHWC max pooling, non-overlapping windows (kernel == stride, no padding: VGG-19's 2x2 pools in
// the perceptual losses). Forward: one thread per (output pixel, V channels). Backward: one thread
// per (output window, V channels) recomputes the window's argmax from the saved input — the first
// maximum in scan order, the last NaN winning as in PyTorch's kernels — and writes the whole window of dx (dy at
// the argmax, zeros elsewhere): no int64 index tensor, no atomics, every dx element written once.
template <typename T, int V>
__global__ void __launch_bounds__(kT)
maxpool_fwd(const T* __restrict__ x, T* __restrict__ y, PoolGeom g) {
  const int cv = g.C / V;
  const int64_t total = (int64_t)g.B * g.Ho * g.Wo * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ox = (int)(p % g.Wo);
    p /= g.Wo;
    const int oy = (int)(p % g.Ho);
    const int b = (int)(p / g.Ho);
    float m[V];
#pragma unroll
    for (int k = 0; k < V; ++k) m[k] = -INFINITY;
    for (int dy = 0; dy < g.kh; ++dy)
      for (int dx = 0; dx < g.kw; ++dx) {
        float v[V];
        load_vec<T, V>(x + (((int64_t)b * g.H + oy * g.sh + dy) * g.W + ox * g.sw + dx) * g.C +
                           c8 * V, v);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (v[k] > m[k] || isnan(v[k])) m[k] = v[k];
      }
    store_vec<T, V>(y + t * V, m);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(kT)
maxpool_bwd(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx, PoolGeom g) {
  const int cv = g.C / V;
  const int64_t total = (int64_t)g.B * g.Ho * g.Wo * cv;
  for (int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kT) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ox = (int)(p % g.Wo);
    p /= g.Wo;
    const int oy = (int)(p % g.Ho);
    const int b = (int)(p / g.Ho);
    float m[V];
    int arg[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      m[k] = -INFINITY;
      arg[k] = 0;
    }
    for (int i = 0; i < g.kh * g.kw; ++i) {
      const int ddy = i / g.kw, ddx = i - ddy * g.kw;
      float v[V];
      load_vec<T, V>(x + (((int64_t)b * g.H + oy * g.sh + ddy) * g.W + ox * g.sw + ddx) * g.C +
                         c8 * V, v);
#pragma unroll
      for (int k = 0; k < V; ++k)
        if (v[k] > m[k] || isnan(v[k])) {
          m[k] = v[k];
          arg[k] = i;
        }
    }
    float gv[V];
    load_vec<T, V>(dy + t * V, gv);
    for (int i = 0; i < g.kh * g.kw; ++i) {
      const int ddy = i / g.kw, ddx = i - ddy * g.kw;
      float o[V];
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = arg[k] == i ? gv[k] : 0.f;
      store_vec<T, V>(dx + (((int64_t)b * g.H + oy * g.sh + ddy) * g.W + ox * g.sw + ddx) * g.C +
                          c8 * V, o);
    }
  }
}

int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + kT - 1) / kT, 65536));
}

PoolGeom geom(const at::Tensor& x, int64_t Ho, int64_t Wo, int64_t kh, int64_t kw, int64_t sh,
              int64_t sw, int64_t ph, int64_t pw, bool include_pad) {
  PoolGeom g;
  g.B = (int)x.size(0); g.C = (int)x.size(1); g.H = (int)x.size(2); g.W = (int)x.size(3);
  g.Ho = (int)Ho; g.Wo = (int)Wo; g.kh = (int)kh; g.kw = (int)kw; g.sh = (int)sh; g.sw = (int)sw;
  g.ph = (int)ph; g.pw = (int)pw; g.include_pad = include_pad;
  IAMD_CHECK(kh >= 1 && kw >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && 2 * ph <= kh &&
                 2 * pw <= kw && Ho >= 1 && Wo >= 1,
             "avg_pool_nhwc: bad geometry");
  // every window must hold at least one real pixel (PyTorch's output-size rule guarantees it)
  IAMD_CHECK((Ho - 1) * sh - ph < g.H && (Wo - 1) * sw - pw < g.W,
             "avg_pool_nhwc: output window outside the input");
  return g;
}

}  // namespace

at::Tensor avg_pool_nhwc_fwd(const at::Tensor& x, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                             int64_t ph, int64_t pw, bool include_pad) {
  IAMD_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
             "avg_pool_nhwc_fwd: packed channels-last bf16 / fp32 tensor expected");
  const int64_t Ho = (x.size(2) + 2 * ph - kh) / sh + 1, Wo = (x.size(3) + 2 * pw - kw) / sw + 1;
  const PoolGeom g = geom(x, Ho, Wo, kh, kw, sh, sw, ph, pw, include_pad);
  auto y = at::empty({g.B, g.C, g.Ho, g.Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool v8 = g.C % 8 == 0;
  const int64_t n = (int64_t)g.B * g.Ho * g.Wo * (v8 ? g.C / 8 : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "avg_pool_nhwc_fwd", [&] {
    if (v8)
      hipLaunchKernelGGL((avgpool_fwd<scalar_t, 8>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<scalar_t*>(y.data_ptr()), g);
    else
      hipLaunchKernelGGL((avgpool_fwd<scalar_t, 1>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<scalar_t*>(y.data_ptr()), g);
  });
  IAMD_LAUNCH_CHECK();
  return y;
}

at::Tensor avg_pool_nhwc_bwd(const at::Tensor& dy, int64_t H, int64_t W, int64_t kh, int64_t kw,
                             int64_t sh, int64_t sw, int64_t ph, int64_t pw, bool include_pad) {
  IAMD_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat),
             "avg_pool_nhwc_bwd: packed channels-last bf16 / fp32 gradient expected");
  auto dx = at::empty({dy.size(0), dy.size(1), H, W},
                      dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  IAMD_CHECK(dy.size(2) == (H + 2 * ph - kh) / sh + 1 && dy.size(3) == (W + 2 * pw - kw) / sw + 1,
             "avg_pool_nhwc_bwd: gradient size does not match the pooled input");
  const PoolGeom g = geom(dx, dy.size(2), dy.size(3), kh, kw, sh, sw, ph, pw, include_pad);
  const bool v8 = g.C % 8 == 0;
  const int64_t n = (int64_t)g.B * g.H * g.W * (v8 ? g.C / 8 : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(dy.scalar_type(), "avg_pool_nhwc_bwd", [&] {
    if (v8)
      hipLaunchKernelGGL((avgpool_bwd<scalar_t, 8>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(dy.data_ptr()),
                         reinterpret_cast<scalar_t*>(dx.data_ptr()), g);
    else
      hipLaunchKernelGGL((avgpool_bwd<scalar_t, 1>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(dy.data_ptr()),
                         reinterpret_cast<scalar_t*>(dx.data_ptr()), g);
  });
  IAMD_LAUNCH_CHECK();
  return dx;
}

// (kernel == stride, no padding; rows / columns past the last whole window get no window)
at::Tensor max_pool_nhwc_fwd(const at::Tensor& x, int64_t kh, int64_t kw) {
  IAMD_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) &&
                 x.size(2) >= kh && x.size(3) >= kw && kh >= 1 && kw >= 1,
             "max_pool_nhwc_fwd: packed channels-last bf16 / fp32 tensor, window within it");
  const PoolGeom g = geom(x, x.size(2) / kh, x.size(3) / kw, kh, kw, kh, kw, 0, 0, true);
  auto y = at::empty({g.B, g.C, g.Ho, g.Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool v8 = g.C % 8 == 0;
  const int64_t n = (int64_t)g.B * g.Ho * g.Wo * (v8 ? g.C / 8 : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "max_pool_nhwc_fwd", [&] {
    if (v8)
      hipLaunchKernelGGL((maxpool_fwd<scalar_t, 8>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<scalar_t*>(y.data_ptr()), g);
    else
      hipLaunchKernelGGL((maxpool_fwd<scalar_t, 1>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<scalar_t*>(y.data_ptr()), g);
  });
  IAMD_LAUNCH_CHECK();
  return y;
}

at::Tensor max_pool_nhwc_bwd(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw) {
  IAMD_CHECK(x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4 &&
                 x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 x.scalar_type() == dy.scalar_type() &&
                 (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) &&
                 dy.size(0) == x.size(0) && dy.size(1) == x.size(1) &&
                 dy.size(2) == x.size(2) / kh && dy.size(3) == x.size(3) / kw,
             "max_pool_nhwc_bwd: input / gradient shapes");
  const PoolGeom g = geom(x, dy.size(2), dy.size(3), kh, kw, kh, kw, 0, 0, true);
  // pixels past the last whole window get no gradient: zero-fill only when there are any
  const bool tail = x.size(2) % kh != 0 || x.size(3) % kw != 0;
  auto dx = tail ? at::zeros_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast))
                 : at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool v8 = g.C % 8 == 0;
  const int64_t n = (int64_t)g.B * g.Ho * g.Wo * (v8 ? g.C / 8 : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "max_pool_nhwc_bwd", [&] {
    if (v8)
      hipLaunchKernelGGL((maxpool_bwd<scalar_t, 8>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<const scalar_t*>(dy.data_ptr()),
                         reinterpret_cast<scalar_t*>(dx.data_ptr()), g);
    else
      hipLaunchKernelGGL((maxpool_bwd<scalar_t, 1>), dim3(grid_for(n)), dim3(kT), 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()),
                         reinterpret_cast<const scalar_t*>(dy.data_ptr()),
                         reinterpret_cast<scalar_t*>(dx.data_ptr()), g);
  });
  IAMD_LAUNCH_CHECK();
  return dx;
}

}  // namespace iamd
