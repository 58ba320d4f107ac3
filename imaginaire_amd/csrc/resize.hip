// k12: bilinear and nearest resizes of NHWC (channels-last) activations, bf16 / fp32 I/O.
//
// Replaces the two bilinear resizes of the SPADE discriminator (reference
// discriminators/spade.py:86-88: the 0.5x input pyramid, align_corners=True;
// discriminators/fpse.py:74: the 2x top-down upsampling, align_corners=False). Under bf16
// autocast PyTorch runs them in fp32 (cast + fp32 resize + fp32 tensor) and their backward is
// an atomic scatter; here
//   * the forward reads 4 taps x 8 channels per thread with 16-byte loads, optionally adds a
//     residual in the same pass (FPSE: up(top) + lateral), and writes the input dtype;
//   * the backward is a GATHER: every input pixel collects the (at most a few) output pixels
//     whose taps touch it — no atomics, deterministic, one 16-byte store per 8 channels.
// Nearest (the SPADE generator's 2x upsampling between blocks and the per-resolution label
// maps; reference generators/spade.py:237-399 uses nn.Upsample / F.interpolate) is a 16-byte
// gather in the input dtype with a gather backward (PyTorch's NHWC nearest kernels ran at ~1/5
// of HBM bandwidth on MI355X, profiles/spade_step_op_shapes_mi355x.txt).
// The source-coordinate rule is PyTorch's area_pixel_compute_source_index (align_corners:
// src = scale * dst; otherwise src = max(scale * (dst + 0.5) - 0.5, 0)) with the caller's
// scale, so results match F.interpolate bit-for-bit up to the output rounding.
#include "common.h"

namespace iamd {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxTaps = 8;  // output rows (cols) a single input row (col) can feed

struct Axis {
  int in, out;
  float scale;
  bool ac;
};

__device__ __forceinline__ float src_index(const Axis& a, int dst) {
  if (a.ac) return a.scale * (float)dst;
  const float s = a.scale * ((float)dst + 0.5f) - 0.5f;
  return s < 0.f ? 0.f : s;
}

// taps of output index `dst` along one axis: (i0, i1, lambda)
__device__ __forceinline__ void taps(const Axis& a, int dst, int& i0, int& i1, float& l) {
  const float s = src_index(a, dst);
  i0 = min((int)s, a.in - 1);
  i1 = min(i0 + 1, a.in - 1);
  l = s - (float)i0;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
resize_fwd(const T* __restrict__ x, const T* __restrict__ add, T* __restrict__ y, int B, int C,
           Axis ay, Axis ax) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * ay.out * ax.out * cv;
  for (int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * kThreads) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ox = (int)(p % ax.out);
    p /= ax.out;
    const int oy = (int)(p % ay.out);
    const int b = (int)(p / ay.out);
    int y0, y1, x0, x1;
    float ly, lx;
    taps(ay, oy, y0, y1, ly);
    taps(ax, ox, x0, x1, lx);
    const T* base = x + (int64_t)b * ay.in * ax.in * C + c8 * 8;
    float v00[8], v01[8], v10[8], v11[8], o[8];
    load_vec<T, 8>(base + ((int64_t)y0 * ax.in + x0) * C, v00);
    load_vec<T, 8>(base + ((int64_t)y0 * ax.in + x1) * C, v01);
    load_vec<T, 8>(base + ((int64_t)y1 * ax.in + x0) * C, v10);
    load_vec<T, 8>(base + ((int64_t)y1 * ax.in + x1) * C, v11);
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx;
    const float w10 = ly * (1.f - lx), w11 = ly * lx;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = w00 * v00[k] + w01 * v01[k] + w10 * v10[k] + w11 * v11[k];
    const int64_t off = (((int64_t)b * ay.out + oy) * ax.out + ox) * C + c8 * 8;
    if (add) {
      float r[8];
      load_vec<T, 8>(add + off, r);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] += r[k];
    }
    store_vec<T, 8>(y + off, o);
  }
}

// outputs along one axis that read input index `i`, with their weights
__device__ __forceinline__ int gather_list(const Axis& a, int i, int (&idx)[kMaxTaps],
                                          float (&w)[kMaxTaps]) {
  // an output o reads i only if src(o) lies in [i - 1, i + 1] (i0 or i1 == i); scan a
  // conservative window around the preimage of that interval
  const float inv = a.scale > 0.f ? 1.f / a.scale : 0.f;
  int lo, hi;
  if (a.scale > 0.f) {
    const float c0 = a.ac ? ((float)i - 1.f) * inv : ((float)i - 1.f + 0.5f) * inv - 0.5f;
    const float c1 = a.ac ? ((float)i + 1.f) * inv : ((float)i + 1.f + 0.5f) * inv - 0.5f;
    lo = max(0, (int)floorf(c0) - 1);
    hi = min(a.out - 1, (int)ceilf(c1) + 1);
  } else {  // single-pixel input axis: every output reads index 0
    lo = 0;
    hi = a.out - 1;
  }
  int n = 0;
  for (int o = lo; o <= hi && n < kMaxTaps; ++o) {
    int i0, i1;
    float l;
    taps(a, o, i0, i1, l);
    float ww = 0.f;
    if (i0 == i) ww += 1.f - l;
    if (i1 == i) ww += l;
    if (ww != 0.f) {
      idx[n] = o;
      w[n] = ww;
      ++n;
    }
  }
  return n;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
resize_bwd(const T* __restrict__ dy, T* __restrict__ dx, int B, int C, Axis ay, Axis ax) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * ay.in * ax.in * cv;
  for (int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * kThreads) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ix = (int)(p % ax.in);
    p /= ax.in;
    const int iy = (int)(p % ay.in);
    const int b = (int)(p / ay.in);
    int oys[kMaxTaps], oxs[kMaxTaps];
    float wys[kMaxTaps], wxs[kMaxTaps];
    const int ny = gather_list(ay, iy, oys, wys);
    const int nx = gather_list(ax, ix, oxs, wxs);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    const T* base = dy + (int64_t)b * ay.out * ax.out * C + c8 * 8;
    for (int a = 0; a < ny; ++a) {
      const T* row = base + (int64_t)oys[a] * ax.out * C;
      for (int c = 0; c < nx; ++c) {
        float g[8];
        load_vec<T, 8>(row + (int64_t)oxs[c] * C, g);
        const float w = wys[a] * wxs[c];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(w, g[k], acc[k]);
      }
    }
    store_vec<T, 8>(dx + (((int64_t)b * ay.in + iy) * ax.in + ix) * C + c8 * 8, acc);
  }
}

// ---- nearest (PyTorch's nearest_idx: exact 2x -> o >> 1, same size -> o, otherwise
// min(floor(o * scale), in - 1) in float) --------------------------------------------------
__device__ __forceinline__ int nearest_src(const Axis& a, int o) {
  if (a.out == a.in) return o;
  if (a.out == 2 * a.in) return o >> 1;
  return min((int)floorf((float)o * a.scale), a.in - 1);
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
nearest_fwd(const T* __restrict__ x, T* __restrict__ y, int B, int C, Axis ay, Axis ax) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * ay.out * ax.out * cv;
  for (int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * kThreads) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ox = (int)(p % ax.out);
    p /= ax.out;
    const int oy = (int)(p % ay.out);
    const int b = (int)(p / ay.out);
    const int64_t src = (((int64_t)b * ay.in + nearest_src(ay, oy)) * ax.in +
                         nearest_src(ax, ox)) * C + c8 * 8;
    *reinterpret_cast<Pack<T, 8>*>(y + t * 8) = *reinterpret_cast<const Pack<T, 8>*>(x + src);
  }
}

// outputs along one axis whose nearest source is input index i
__device__ __forceinline__ int nearest_list(const Axis& a, int i, int (&idx)[kMaxTaps]) {
  int lo = 0, hi = a.out - 1;
  if (a.out == a.in) {
    lo = hi = i;
  } else if (a.out == 2 * a.in) {
    lo = 2 * i;
    hi = 2 * i + 1;
  } else if (a.scale > 0.f) {
    lo = max(0, (int)floorf((float)i / a.scale) - 1);
    hi = min(a.out - 1, (int)ceilf((float)(i + 1) / a.scale) + 1);
  }
  int n = 0;
  for (int o = lo; o <= hi && n < kMaxTaps; ++o)
    if (nearest_src(a, o) == i) idx[n++] = o;
  return n;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
nearest_bwd(const T* __restrict__ dy, T* __restrict__ dx, int B, int C, Axis ay, Axis ax) {
  const int cv = C / 8;
  const int64_t n = (int64_t)B * ay.in * ax.in * cv;
  for (int64_t t = blockIdx.x * (int64_t)kThreads + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * kThreads) {
    const int c8 = (int)(t % cv);
    int64_t p = t / cv;
    const int ix = (int)(p % ax.in);
    p /= ax.in;
    const int iy = (int)(p % ay.in);
    const int b = (int)(p / ay.in);
    int oys[kMaxTaps], oxs[kMaxTaps];
    const int ny = nearest_list(ay, iy, oys);
    const int nx = nearest_list(ax, ix, oxs);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    const T* base = dy + (int64_t)b * ay.out * ax.out * C + c8 * 8;
    for (int a = 0; a < ny; ++a)
      for (int c = 0; c < nx; ++c) {
        float g[8];
        load_vec<T, 8>(base + ((int64_t)oys[a] * ax.out + oxs[c]) * C, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += g[k];
      }
    store_vec<T, 8>(dx + t * 8, acc);
  }
}

Axis make_axis(int64_t in, int64_t out, double scale, bool ac) {
  Axis a;
  a.in = (int)in;
  a.out = (int)out;
  a.scale = (float)scale;
  a.ac = ac;
  return a;
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + kThreads - 1) / kThreads, 65536); }

void check_nhwc(const at::Tensor& t, const char* what) {
  IAMD_CHECK(t.is_cuda() && t.dim() == 4, what, ": 4-D CUDA tensor expected");
  IAMD_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what,
             ": packed channels-last tensor expected");
  IAMD_CHECK(t.size(1) % 8 == 0, what, ": channels must be a multiple of 8");
  IAMD_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, what,
             ": bf16 or fp32 expected");
}

}  // namespace

// y[B, C, Ho, Wo] (channels-last) = bilinear(x) (+ add); scale_* = PyTorch's source scale
at::Tensor resize_bilinear_fwd(const at::Tensor& x, int64_t Ho, int64_t Wo, double scale_h,
                               double scale_w, bool align_corners,
                               const c10::optional<at::Tensor>& add) {
  check_nhwc(x, "resize_bilinear_fwd");
  const int B = (int)x.size(0), C = (int)x.size(1);
  auto y = at::empty({B, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const void* ap = nullptr;
  if (add.has_value() && add->defined()) {
    IAMD_CHECK(add->sizes() == y.sizes() && add->scalar_type() == x.scalar_type() &&
                   add->is_contiguous(at::MemoryFormat::ChannelsLast),
               "resize_bilinear_fwd: residual must match the output (channels-last)");
    ap = add->data_ptr();
  }
  const Axis ay = make_axis(x.size(2), Ho, scale_h, align_corners);
  const Axis ax = make_axis(x.size(3), Wo, scale_w, align_corners);
  const int64_t n = (int64_t)B * Ho * Wo * (C / 8);
  if (n == 0) return y;
  if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((resize_fwd<__hip_bfloat16>), dim3(grid_for(n)), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                       reinterpret_cast<const __hip_bfloat16*>(ap),
                       reinterpret_cast<__hip_bfloat16*>(y.data_ptr()), B, C, ay, ax);
  else
    hipLaunchKernelGGL((resize_fwd<float>), dim3(grid_for(n)), dim3(kThreads), 0, stream(),
                       x.data_ptr<float>(), reinterpret_cast<const float*>(ap),
                       y.data_ptr<float>(), B, C, ay, ax);
  IAMD_LAUNCH_CHECK();
  return y;
}

// dx[B, C, H, W] from dy[B, C, Ho, Wo] (gather form, deterministic)
at::Tensor resize_bilinear_bwd(const at::Tensor& dy, int64_t H, int64_t W, double scale_h,
                               double scale_w, bool align_corners) {
  check_nhwc(dy, "resize_bilinear_bwd");
  const int B = (int)dy.size(0), C = (int)dy.size(1);
  const Axis ay = make_axis(H, dy.size(2), scale_h, align_corners);
  const Axis ax = make_axis(W, dy.size(3), scale_w, align_corners);
  // an input index feeds at most 2 / scale + 2 outputs per axis (kMaxTaps bounds the list)
  IAMD_CHECK((scale_h <= 0.0 || 2.0 / scale_h + 2.0 <= kMaxTaps) &&
                 (scale_w <= 0.0 || 2.0 / scale_w + 2.0 <= kMaxTaps),
             "resize_bilinear_bwd: upsampling factor above 3 unsupported");
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t n = (int64_t)B * H * W * (C / 8);
  if (n == 0) return dx;
  if (dy.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((resize_bwd<__hip_bfloat16>), dim3(grid_for(n)), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(dx.data_ptr()), B, C, ay, ax);
  else
    hipLaunchKernelGGL((resize_bwd<float>), dim3(grid_for(n)), dim3(kThreads), 0, stream(),
                       dy.data_ptr<float>(), dx.data_ptr<float>(), B, C, ay, ax);
  IAMD_LAUNCH_CHECK();
  return dx;
}

// y[B, C, Ho, Wo] (channels-last) = nearest(x); scale_* = PyTorch's source scale (in / out or
// 1 / scale_factor). A pure gather of 16-byte channel chunks in the input dtype.
at::Tensor resize_nearest_fwd(const at::Tensor& x, int64_t Ho, int64_t Wo, double scale_h,
                              double scale_w) {
  check_nhwc(x, "resize_nearest_fwd");
  const int B = (int)x.size(0), C = (int)x.size(1);
  auto y = at::empty({B, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const Axis ay = make_axis(x.size(2), Ho, scale_h, false);
  const Axis ax = make_axis(x.size(3), Wo, scale_w, false);
  const int64_t n = (int64_t)B * Ho * Wo * (C / 8);
  if (n == 0) return y;
  if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((nearest_fwd<__hip_bfloat16>), dim3(grid_for(n)), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(y.data_ptr()), B, C, ay, ax);
  else
    hipLaunchKernelGGL((nearest_fwd<float>), dim3(grid_for(n)), dim3(kThreads), 0, stream(),
                       reinterpret_cast<const float*>(x.data_ptr()),
                       reinterpret_cast<float*>(y.data_ptr()), B, C, ay, ax);
  IAMD_LAUNCH_CHECK();
  return y;
}

// dx[B, C, H, W] = sum of dy over the outputs that copied each input pixel (gather form)
at::Tensor resize_nearest_bwd(const at::Tensor& dy, int64_t H, int64_t W, double scale_h,
                              double scale_w) {
  check_nhwc(dy, "resize_nearest_bwd");
  const int B = (int)dy.size(0), C = (int)dy.size(1);
  const Axis ay = make_axis(H, dy.size(2), scale_h, false);
  const Axis ax = make_axis(W, dy.size(3), scale_w, false);
  IAMD_CHECK((ay.out <= 2 * ay.in || (scale_h > 0.0 && 1.0 / scale_h + 3.0 <= kMaxTaps)) &&
                 (ax.out <= 2 * ax.in || (scale_w > 0.0 && 1.0 / scale_w + 3.0 <= kMaxTaps)),
             "resize_nearest_bwd: upsampling factor above 5 unsupported");
  auto dx = at::empty({B, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t n = (int64_t)B * H * W * (C / 8);
  if (n == 0) return dx;
  if (dy.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((nearest_bwd<__hip_bfloat16>), dim3(grid_for(n)), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr()),
                       reinterpret_cast<__hip_bfloat16*>(dx.data_ptr()), B, C, ay, ax);
  else
    hipLaunchKernelGGL((nearest_bwd<float>), dim3(grid_for(n)), dim3(kThreads), 0, stream(),
                       dy.data_ptr<float>(), dx.data_ptr<float>(), B, C, ay, ax);
  IAMD_LAUNCH_CHECK();
  return dx;
}

}  // namespace iamd
