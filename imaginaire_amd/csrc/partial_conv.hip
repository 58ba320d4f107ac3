// k3: partial-convolution mask update + re-normalisation.
//
// Reference semantics (layers/conv.py:956-1009):
//   s      = conv(mask, ones)                       (window sum of the mask)
//   update = clamp(s, 0, 1);  ratio = winsize / (s + eps) * update
//   out    = ((raw - b) * ratio + b) * update       (raw = conv(x*mask) + b)
// Here the convolution runs bias-free on MIOpen, so out = (raw_nb*ratio + b)*update.
// Kernel 1 computes (ratio, update) once per output pixel (shared by all output
// channels; the reference recomputes a full conv for it), kernel 2 applies the
// re-normalisation to the MIOpen output in one vectorised pass.
#include "common.h"

namespace iamd {
namespace {

constexpr int kThreads = 256;

template <typename M>
__global__ void mask_window_kernel(const M* __restrict__ mask, int Nm, int Cm, int H, int W,
                                   int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw,
                                   int dh, int dw, float winsize, float eps,
                                   float* __restrict__ ratio, float* __restrict__ update,
                                   int64_t mcs, int64_t mns, int64_t mhs, int64_t mws) {
  const int64_t total = (int64_t)Nm * Ho * Wo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(i % Wo);
    const int oy = (int)((i / Wo) % Ho);
    const int n = (int)(i / ((int64_t)Ho * Wo));
    float s = 0.f;
    for (int c = 0; c < Cm; ++c) {
      const M* mp = mask + n * mns + c * mcs;
      for (int ky = 0; ky < kh; ++ky) {
        const int iy = oy * sh - ph + ky * dh;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < kw; ++kx) {
          const int ix = ox * sw - pw + kx * dw;
          if (ix < 0 || ix >= W) continue;
          s += to_f<M>(mp[iy * mhs + ix * mws]);
        }
      }
    }
    const float u = fminf(fmaxf(s, 0.f), 1.f);
    update[i] = u;
    ratio[i] = winsize / (s + eps) * u;
  }
}

template <typename T, bool CL>
__global__ void renorm_kernel(const T* __restrict__ raw, T* __restrict__ out,
                              const float* __restrict__ ratio, const float* __restrict__ update,
                              const float* __restrict__ bias, int N, int C, int HWo, int mask_n) {
  const int64_t total = (int64_t)N * C * HWo;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int n, c, p;
    if (CL) {
      c = (int)(e % C);
      p = (int)((e / C) % HWo);
      n = (int)(e / ((int64_t)C * HWo));
    } else {
      p = (int)(e % HWo);
      c = (int)((e / HWo) % C);
      n = (int)(e / ((int64_t)C * HWo));
    }
    const int64_t mi = (int64_t)(mask_n > 1 ? n : 0) * HWo + p;
    const float b = bias ? bias[c] : 0.f;
    out[e] = from_f<T>((to_f<T>(raw[e]) * ratio[mi] + b) * update[mi]);
  }
}

}  // namespace

// raw: bias-free conv output [N, C, Ho, Wo]; mask: [Nm, Cm, H, W].
// Returns (out, ratio[Nm,1,Ho,Wo] fp32, update[Nm,1,Ho,Wo] fp32).
std::vector<at::Tensor> partial_conv_renorm(const at::Tensor& raw, const at::Tensor& mask,
                                            const c10::optional<at::Tensor>& bias, int64_t kh,
                                            int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                                            int64_t pw, int64_t dh, int64_t dw, double winsize,
                                            double eps) {
  IAMD_CHECK(raw.dim() == 4 && mask.dim() == 4, "partial_conv_renorm: 4-D tensors expected");
  const int N = (int)raw.size(0), C = (int)raw.size(1), Ho = (int)raw.size(2), Wo = (int)raw.size(3);
  const int Nm = (int)mask.size(0), Cm = (int)mask.size(1), H = (int)mask.size(2), W = (int)mask.size(3);
  IAMD_CHECK(Nm == 1 || Nm == N, "mask batch must be 1 or N");
  auto fopt = raw.options().dtype(at::kFloat);
  auto ratio = at::empty({Nm, 1, Ho, Wo}, fopt);
  auto update = at::empty({Nm, 1, Ho, Wo}, fopt);
  const int64_t tot_m = (int64_t)Nm * Ho * Wo;
  const int gm = (int)std::min<int64_t>((tot_m + kThreads - 1) / kThreads, 4096);
  IAMD_DISPATCH_FLOAT_TYPES(mask.scalar_type(), "mask_window", [&] {
    hipLaunchKernelGGL((mask_window_kernel<scalar_t>), dim3(std::max(gm, 1)), dim3(kThreads), 0,
                       stream(), reinterpret_cast<const scalar_t*>(mask.data_ptr()), Nm, Cm, H, W,
                       Ho, Wo, (int)kh, (int)kw, (int)sh, (int)sw, (int)ph, (int)pw, (int)dh,
                       (int)dw, (float)winsize, (float)eps, ratio.data_ptr<float>(),
                       update.data_ptr<float>(), mask.stride(1), mask.stride(0), mask.stride(2),
                       mask.stride(3));
  });
  IAMD_LAUNCH_CHECK();
  const bool cl = raw.is_contiguous(at::MemoryFormat::ChannelsLast) && !raw.is_contiguous();
  at::Tensor rawc = cl ? raw : raw.contiguous();
  auto out = at::empty_like(rawc);
  at::Tensor bf;
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) { bf = bias->to(at::kFloat).contiguous(); bp = bf.data_ptr<float>(); }
  const int64_t tot = rawc.numel();
  const int g = (int)std::min<int64_t>((tot + kThreads - 1) / kThreads, 8192);
  IAMD_DISPATCH_FLOAT_TYPES(raw.scalar_type(), "partial_renorm", [&] {
    auto rp = reinterpret_cast<const scalar_t*>(rawc.data_ptr());
    auto op = reinterpret_cast<scalar_t*>(out.data_ptr());
    if (cl)
      hipLaunchKernelGGL((renorm_kernel<scalar_t, true>), dim3(std::max(g, 1)), dim3(kThreads), 0,
                         stream(), rp, op, ratio.data_ptr<float>(), update.data_ptr<float>(), bp,
                         N, C, Ho * Wo, Nm);
    else
      hipLaunchKernelGGL((renorm_kernel<scalar_t, false>), dim3(std::max(g, 1)), dim3(kThreads), 0,
                         stream(), rp, op, ratio.data_ptr<float>(), update.data_ptr<float>(), bp,
                         N, C, Ho * Wo, Nm);
  });
  IAMD_LAUNCH_CHECK();
  return {out, ratio, update};
}

}  // namespace iamd
