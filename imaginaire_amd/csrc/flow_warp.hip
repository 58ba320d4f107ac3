// k9: optical-flow warp (bilinear, border padding, align_corners=True) and
// k7: FlowNet2 Resample2d (bilinear warp with edge clamping, kernel_size window).
//
// k9 reproduces model_utils/fs_vid2vid.py:14-38 (F.grid_sample on a pixel grid
// shifted by the flow): out[b,c,y,x] = bilinear(img[b,c], x + fx, y + fy) with
// the sample position clamped to the image (border padding; zero gradient
// w.r.t. the flow where clamped). One thread per output pixel loops over
// channels so the 4 tap weights / addresses are computed once and reused.
// Backward: d(image) by fp32 atomics (4 taps per pixel, contention-free across
// waves), d(flow) = Σ_c dout · ∂sample/∂(x,y) with no atomics. When the image needs no
// gradient (the detached previous frame of vid2vid) the scatter is skipped entirely, and
// ops/flow_warp.py replaces it by a sort-based deterministic scatter in deterministic mode.
//
// k7 reproduces third_party/resample2d/src/resample2d_kernel.cu:15-203
// semantics (edge-clamped taps, kernel_size² window average), written for
// NCHW fp32/bf16 with one thread per output element.
#include "common.h"

namespace iamd {
namespace {

constexpr int kThreads = 256;

struct Taps {
  int x0, x1, y0, y1;
  float wx, wy;       // fractional weights toward x1 / y1
  bool cx, cy;        // coordinate clamped (no flow gradient)
};

__device__ __forceinline__ Taps make_taps(float sx, float sy, int H, int W) {
  Taps t;
  t.cx = sx <= 0.f || sx >= (float)(W - 1);
  t.cy = sy <= 0.f || sy >= (float)(H - 1);
  sx = fminf(fmaxf(sx, 0.f), (float)(W - 1));
  sy = fminf(fmaxf(sy, 0.f), (float)(H - 1));
  const float fx = floorf(sx), fy = floorf(sy);
  t.x0 = (int)fx; t.y0 = (int)fy;
  t.x1 = min(t.x0 + 1, W - 1);
  t.y1 = min(t.y0 + 1, H - 1);
  t.wx = sx - fx; t.wy = sy - fy;
  return t;
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
warp_fwd(const T* __restrict__ img, const T* __restrict__ flow, T* __restrict__ out, int B, int C,
         int H, int W, int64_t isb, int64_t isc, int64_t isy, int64_t isx, int64_t fsb,
         int64_t fsc, int64_t fsy, int64_t fsx, int64_t osb, int64_t osc, int64_t osy,
         int64_t osx) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(i % W), y = (int)((i / W) % H), b = (int)(i / ((int64_t)H * W));
    const T* fp = flow + b * fsb + y * fsy + x * fsx;
    const float fx = to_f<T>(fp[0]), fy = to_f<T>(fp[fsc]);
    const Taps t = make_taps(x + fx, y + fy, H, W);
    const float w00 = (1.f - t.wx) * (1.f - t.wy), w01 = t.wx * (1.f - t.wy);
    const float w10 = (1.f - t.wx) * t.wy, w11 = t.wx * t.wy;
    const T* ib = img + b * isb;
    T* ob = out + b * osb + y * osy + x * osx;
    const int64_t o00 = t.y0 * isy + t.x0 * isx, o01 = t.y0 * isy + t.x1 * isx;
    const int64_t o10 = t.y1 * isy + t.x0 * isx, o11 = t.y1 * isy + t.x1 * isx;
    for (int c = 0; c < C; ++c) {
      const T* ic = ib + c * isc;
      const float v = w00 * to_f<T>(ic[o00]) + w01 * to_f<T>(ic[o01]) + w10 * to_f<T>(ic[o10]) +
                      w11 * to_f<T>(ic[o11]);
      ob[c * osc] = from_f<T>(v);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
warp_bwd(const T* __restrict__ img, const T* __restrict__ flow, const T* __restrict__ dout,
         float* __restrict__ dimg, float* __restrict__ dflow, int B, int C, int H, int W,
         int64_t isb, int64_t isc, int64_t isy, int64_t isx, int64_t fsb, int64_t fsc,
         int64_t fsy, int64_t fsx, int64_t dsb, int64_t dsc, int64_t dsy, int64_t dsx) {
  // dimg: contiguous fp32 [B, C, H, W]; dflow: contiguous fp32 [B, 2, H, W]
  const int64_t total = (int64_t)B * H * W;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(i % W), y = (int)((i / W) % H), b = (int)(i / ((int64_t)H * W));
    const T* fp = flow + b * fsb + y * fsy + x * fsx;
    const float fx = to_f<T>(fp[0]), fy = to_f<T>(fp[fsc]);
    const Taps t = make_taps(x + fx, y + fy, H, W);
    const float w00 = (1.f - t.wx) * (1.f - t.wy), w01 = t.wx * (1.f - t.wy);
    const float w10 = (1.f - t.wx) * t.wy, w11 = t.wx * t.wy;
    const T* ib = img + b * isb;
    const T* db = dout + b * dsb + y * dsy + x * dsx;
    float* gb = dimg != nullptr ? dimg + (int64_t)b * C * H * W : nullptr;
    const int64_t HW = (int64_t)H * W;
    float gx = 0.f, gy = 0.f;
    for (int c = 0; c < C; ++c) {
      const float g = to_f<T>(db[c * dsc]);
      const T* ic = ib + c * isc;
      const float v00 = to_f<T>(ic[t.y0 * isy + t.x0 * isx]);
      const float v01 = to_f<T>(ic[t.y0 * isy + t.x1 * isx]);
      const float v10 = to_f<T>(ic[t.y1 * isy + t.x0 * isx]);
      const float v11 = to_f<T>(ic[t.y1 * isy + t.x1 * isx]);
      gx += g * ((v01 - v00) * (1.f - t.wy) + (v11 - v10) * t.wy);
      gy += g * ((v10 - v00) * (1.f - t.wx) + (v11 - v01) * t.wx);
      if (dimg != nullptr) {
        float* gc = gb + c * HW;
        atomicAdd(gc + t.y0 * W + t.x0, g * w00);
        atomicAdd(gc + t.y0 * W + t.x1, g * w01);
        atomicAdd(gc + t.y1 * W + t.x0, g * w10);
        atomicAdd(gc + t.y1 * W + t.x1, g * w11);
      }
    }
    float* dfp = dflow + (int64_t)b * 2 * HW + (int64_t)y * W + x;
    dfp[0] = t.cx ? 0.f : gx;
    dfp[HW] = t.cy ? 0.f : gy;
  }
}

// ---------------- k7: Resample2d (FlowNet2) -------------------------------
// Edge-clamped bilinear taps at (x + fx, y + fy); for kernel_size > 1 the
// reference averages a kernel_size² window of taps around the sample point.
template <typename T>
__global__ void __launch_bounds__(kThreads)
resample2d_fwd(const T* __restrict__ in1, const T* __restrict__ flow, T* __restrict__ out, int B,
               int C, int H, int W, int ks) {
  const int64_t total = (int64_t)B * C * H * W;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(i % W), y = (int)((i / W) % H);
    const int c = (int)((i / ((int64_t)H * W)) % C), b = (int)(i / ((int64_t)C * H * W));
    const int64_t HW = (int64_t)H * W;
    const float dx = to_f<T>(flow[(int64_t)b * 2 * HW + (int64_t)y * W + x]);
    const float dy = to_f<T>(flow[(int64_t)b * 2 * HW + HW + (int64_t)y * W + x]);
    const float xf = (float)x + dx, yf = (float)y + dy;
    const float alpha = xf - floorf(xf), beta = yf - floorf(yf);
    const int xL = max(min((int)floorf(xf), W - 1), 0), xR = max(min((int)floorf(xf) + 1, W - 1), 0);
    const int yT = max(min((int)floorf(yf), H - 1), 0), yB = max(min((int)floorf(yf) + 1, H - 1), 0);
    const T* ic = in1 + ((int64_t)b * C + c) * HW;
    float v = 0.f;
    for (int fy = 0; fy < ks; ++fy) {
      for (int fx = 0; fx < ks; ++fx) {
        const int yt = max(min(yT + fy, H - 1), 0), yb = max(min(yB + fy, H - 1), 0);
        const int xl = max(min(xL + fx, W - 1), 0), xr = max(min(xR + fx, W - 1), 0);
        v += (1.f - alpha) * (1.f - beta) * to_f<T>(ic[(int64_t)yt * W + xl]);
        v += alpha * (1.f - beta) * to_f<T>(ic[(int64_t)yt * W + xr]);
        v += (1.f - alpha) * beta * to_f<T>(ic[(int64_t)yb * W + xl]);
        v += alpha * beta * to_f<T>(ic[(int64_t)yb * W + xr]);
      }
    }
    out[i] = from_f<T>(v);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
resample2d_bwd(const T* __restrict__ in1, const T* __restrict__ flow, const T* __restrict__ dout,
               float* __restrict__ din1, float* __restrict__ dflow, int B, int C, int H, int W,
               int ks) {
  // one thread per (b, y, x): loops channels, accumulates dflow without atomics
  const int64_t total = (int64_t)B * H * W;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(i % W), y = (int)((i / W) % H), b = (int)(i / ((int64_t)H * W));
    const int64_t HW = (int64_t)H * W;
    const float dx = to_f<T>(flow[(int64_t)b * 2 * HW + (int64_t)y * W + x]);
    const float dy = to_f<T>(flow[(int64_t)b * 2 * HW + HW + (int64_t)y * W + x]);
    const float xf = (float)x + dx, yf = (float)y + dy;
    const float alpha = xf - floorf(xf), beta = yf - floorf(yf);
    const int xL = max(min((int)floorf(xf), W - 1), 0), xR = max(min((int)floorf(xf) + 1, W - 1), 0);
    const int yT = max(min((int)floorf(yf), H - 1), 0), yB = max(min((int)floorf(yf) + 1, H - 1), 0);
    float gx = 0.f, gy = 0.f;
    for (int c = 0; c < C; ++c) {
      const int64_t base = ((int64_t)b * C + c) * HW;
      const float g = to_f<T>(dout[base + (int64_t)y * W + x]);
      const T* ic = in1 + base;
      float* dc = din1 + base;
      for (int fy = 0; fy < ks; ++fy) {
        for (int fx = 0; fx < ks; ++fx) {
          const int yt = max(min(yT + fy, H - 1), 0), yb = max(min(yB + fy, H - 1), 0);
          const int xl = max(min(xL + fx, W - 1), 0), xr = max(min(xR + fx, W - 1), 0);
          const float tl = to_f<T>(ic[(int64_t)yt * W + xl]), tr = to_f<T>(ic[(int64_t)yt * W + xr]);
          const float bl = to_f<T>(ic[(int64_t)yb * W + xl]), br = to_f<T>(ic[(int64_t)yb * W + xr]);
          gx += g * ((1.f - beta) * (tr - tl) + beta * (br - bl));
          gy += g * ((1.f - alpha) * (bl - tl) + alpha * (br - tr));
          atomicAdd(dc + (int64_t)yt * W + xl, g * (1.f - alpha) * (1.f - beta));
          atomicAdd(dc + (int64_t)yt * W + xr, g * alpha * (1.f - beta));
          atomicAdd(dc + (int64_t)yb * W + xl, g * (1.f - alpha) * beta);
          atomicAdd(dc + (int64_t)yb * W + xr, g * alpha * beta);
        }
      }
    }
    dflow[(int64_t)b * 2 * HW + (int64_t)y * W + x] = gx;
    dflow[(int64_t)b * 2 * HW + HW + (int64_t)y * W + x] = gy;
  }
}

int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, 8192));
}

}  // namespace

at::Tensor flow_warp_fwd(const at::Tensor& img, const at::Tensor& flow) {
  IAMD_CHECK(img.dim() == 4 && flow.dim() == 4 && flow.size(1) == 2, "flow_warp: shapes");
  IAMD_CHECK(img.size(0) == flow.size(0) && img.size(2) == flow.size(2) &&
                 img.size(3) == flow.size(3), "flow_warp: image/flow size mismatch");
  at::Tensor fl = flow.scalar_type() == img.scalar_type() ? flow : flow.to(img.scalar_type());
  const int B = img.size(0), C = img.size(1), H = img.size(2), W = img.size(3);
  auto out = at::empty_like(img);
  IAMD_DISPATCH_FLOAT_TYPES(img.scalar_type(), "flow_warp_fwd", [&] {
    hipLaunchKernelGGL((warp_fwd<scalar_t>), dim3(grid_for((int64_t)B * H * W)), dim3(kThreads),
                       0, stream(), reinterpret_cast<const scalar_t*>(img.data_ptr()),
                       reinterpret_cast<const scalar_t*>(fl.data_ptr()),
                       reinterpret_cast<scalar_t*>(out.data_ptr()), B, C, H, W, img.stride(0),
                       img.stride(1), img.stride(2), img.stride(3), fl.stride(0), fl.stride(1),
                       fl.stride(2), fl.stride(3), out.stride(0), out.stride(1), out.stride(2),
                       out.stride(3));
  });
  IAMD_LAUNCH_CHECK();
  return out;
}

std::vector<at::Tensor> flow_warp_bwd(const at::Tensor& img, const at::Tensor& flow,
                                      const at::Tensor& dout, bool need_dimg) {
  at::Tensor fl = flow.scalar_type() == img.scalar_type() ? flow : flow.to(img.scalar_type());
  at::Tensor g = dout.scalar_type() == img.scalar_type() ? dout : dout.to(img.scalar_type());
  const int B = img.size(0), C = img.size(1), H = img.size(2), W = img.size(3);
  auto fopt = img.options().dtype(at::kFloat);
  auto dimg = need_dimg ? at::zeros({B, C, H, W}, fopt) : at::Tensor();
  auto dflow = at::empty({B, 2, H, W}, fopt);
  IAMD_DISPATCH_FLOAT_TYPES(img.scalar_type(), "flow_warp_bwd", [&] {
    hipLaunchKernelGGL((warp_bwd<scalar_t>), dim3(grid_for((int64_t)B * H * W)), dim3(kThreads),
                       0, stream(), reinterpret_cast<const scalar_t*>(img.data_ptr()),
                       reinterpret_cast<const scalar_t*>(fl.data_ptr()),
                       reinterpret_cast<const scalar_t*>(g.data_ptr()),
                       need_dimg ? dimg.data_ptr<float>() : nullptr,
                       dflow.data_ptr<float>(), B, C, H, W, img.stride(0), img.stride(1),
                       img.stride(2), img.stride(3), fl.stride(0), fl.stride(1), fl.stride(2),
                       fl.stride(3), g.stride(0), g.stride(1), g.stride(2), g.stride(3));
  });
  IAMD_LAUNCH_CHECK();
  return {dimg, dflow};
}

at::Tensor resample2d_forward(const at::Tensor& in1, const at::Tensor& flow, int64_t ks) {
  auto x = in1.contiguous();
  auto f = flow.contiguous().to(x.scalar_type());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  IAMD_CHECK(f.size(0) == B && f.size(1) == 2 && f.size(2) == H && f.size(3) == W,
             "resample2d: flow shape");
  auto out = at::empty_like(x);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "resample2d_fwd", [&] {
    hipLaunchKernelGGL((resample2d_fwd<scalar_t>), dim3(grid_for(x.numel())), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const scalar_t*>(x.data_ptr()),
                       reinterpret_cast<const scalar_t*>(f.data_ptr()),
                       reinterpret_cast<scalar_t*>(out.data_ptr()), B, C, H, W, (int)ks);
  });
  IAMD_LAUNCH_CHECK();
  return out;
}

std::vector<at::Tensor> resample2d_backward(const at::Tensor& in1, const at::Tensor& flow,
                                            const at::Tensor& dout, int64_t ks) {
  auto x = in1.contiguous();
  auto f = flow.contiguous().to(x.scalar_type());
  auto g = dout.contiguous().to(x.scalar_type());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto fopt = x.options().dtype(at::kFloat);
  auto d1 = at::zeros({B, C, H, W}, fopt);
  auto d2 = at::empty({B, 2, H, W}, fopt);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "resample2d_bwd", [&] {
    hipLaunchKernelGGL((resample2d_bwd<scalar_t>), dim3(grid_for((int64_t)B * H * W)),
                       dim3(kThreads), 0, stream(),
                       reinterpret_cast<const scalar_t*>(x.data_ptr()),
                       reinterpret_cast<const scalar_t*>(f.data_ptr()),
                       reinterpret_cast<const scalar_t*>(g.data_ptr()), d1.data_ptr<float>(),
                       d2.data_ptr<float>(), B, C, H, W, (int)ks);
  });
  IAMD_LAUNCH_CHECK();
  return {d1, d2};
}

}  // namespace iamd
