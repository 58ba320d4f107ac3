// k13: multi-tensor weighted L1 loss  L = sum_t w_t * mean(|a_t - b_t|)  and its gradient.
//
// The perceptual loss (reference losses/perceptual.py:139-180: 5 VGG-19 layers) and the
// discriminator feature-matching loss (losses/feature_matching.py:19-38: every feature of
// every D scale) are sums of per-layer L1 distances between bf16 NHWC feature maps. Under
// autocast PyTorch promotes each l1_loss to fp32: two fp32 copies of every feature map, an
// fp32 |a-b|, a mean per layer, and an fp32 sign * scale backward cast back to bf16 — ~25
// launches and ~1 GB of extra traffic per SPADE step. Here:
//   * forward: ONE launch reads every (a_t, b_t) pair once (16-byte bf16 loads, fp32 |a-b|
//     accumulation) and writes one weighted partial per block; a one-block kernel sums the
//     partials in a fixed order (deterministic, no atomics);
//   * backward: ONE launch writes every dL/da_t = w_t / n_t * sign(a_t - b_t) * dL in the
//     feature dtype.
// The targets b may be fp32 where the inputs a are bf16 (the fp32 real frames of the vid2vid /
// MUNIT reconstruction L1s): the difference is then taken in fp32 on the unrounded target, as
// autocast's fp32 l1_loss does.
// Up to kMaxT pairs per launch travel in the kernel arguments (no device table).
//
// k13b: multi-tensor GAN loss  L = sum_t w_t * mean(phi_t(x_t))  over every discriminator
// output of a pass (reference losses/gan.py:12-132: per-output min/mean/neg kernels, averaged
// over the multi-scale list), one forward + one fixed-order reduce launch and one backward
// launch for all outputs:
//   kind 0  phi = relu(a + b x)               hinge, D update (a = 1, b = -1 real / +1 fake)
//   kind 1  phi = b x                         hinge G update / wasserstein (b = -1 / +1)
//   kind 2  phi = bce_with_logits(x, y = a)   non_saturated
//   kind 3  phi = 0.5 (x - a)^2               least_square
#include "common.h"

namespace iamd {
namespace {

constexpr int kMaxT = 16;
constexpr int kThreads = 256;
constexpr int64_t kChunk = 256 * 8 * 8;  // elements per block (8 x 16-byte loads per thread)

template <typename T, typename TB = T>
struct L1Args {
  const T* a[kMaxT];
  const TB* b[kMaxT];
  T* g[kMaxT];
  int64_t n[kMaxT];
  float scale[kMaxT];   // w_t / n_t
  int start[kMaxT + 1];  // prefix sums of blocks per tensor
  int nt;
};

template <typename P>
__device__ __forceinline__ int find_tensor(const P& p, int bid) {
  int t = 0;
#pragma unroll
  for (int k = 1; k < kMaxT; ++k)
    if (k < p.nt && bid >= p.start[k]) t = k;
  return t;
}

template <typename T, typename TB>
__global__ void __launch_bounds__(kThreads) l1_partials(const L1Args<T, TB> p, float* __restrict__ part) {
  __shared__ float sh[kThreads / 64];
  const int bid = blockIdx.x;
  const int t = find_tensor(p, bid);
  const int64_t c0 = (int64_t)(bid - p.start[t]) * kChunk;
  const int64_t c1 = min(p.n[t], c0 + kChunk);
  const T* __restrict__ a = p.a[t];
  const TB* __restrict__ b = p.b[t];
  float acc = 0.f;
  const bool vec = (((uintptr_t)a | (uintptr_t)b) % 16 == 0);
  if (vec) {
    int64_t i = c0 + threadIdx.x * 8;
    for (; i + 7 < c1; i += kThreads * 8) {
      float va[8], vb[8];
      load_vec<T, 8>(a + i, va);
      load_vec<TB, 8>(b + i, vb);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += fabsf(va[k] - vb[k]);
    }
    // tail of a tensor whose size is not a multiple of 8
    const int64_t tail = c0 + ((c1 - c0) / 8) * 8;
    for (int64_t j = tail + threadIdx.x; j < c1; j += kThreads) acc += fabsf(to_f<T>(a[j]) - to_f<TB>(b[j]));
  } else {
    for (int64_t j = c0 + threadIdx.x; j < c1; j += kThreads) acc += fabsf(to_f<T>(a[j]) - to_f<TB>(b[j]));
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) s += sh[k];
    part[bid] = s * p.scale[t];
  }
}

// out[0] = sum of part[0 .. n) in a fixed order (one block)
__global__ void __launch_bounds__(1024) sum_fixed(const float* __restrict__ part, int n,
                                                  float* __restrict__ out) {
  __shared__ float sh[1024 / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) acc += part[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 1024 / 64; ++k) s += sh[k];
    out[0] = s;
  }
}

template <typename T, typename TB>
__global__ void __launch_bounds__(kThreads) l1_grad(const L1Args<T, TB> p, const float* __restrict__ gout) {
  const int bid = blockIdx.x;
  const int t = find_tensor(p, bid);
  const int64_t c0 = (int64_t)(bid - p.start[t]) * kChunk;
  const int64_t c1 = min(p.n[t], c0 + kChunk);
  const T* __restrict__ a = p.a[t];
  const TB* __restrict__ b = p.b[t];
  T* __restrict__ g = p.g[t];
  const float s = p.scale[t] * gout[0];
  auto sgn = [](float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); };
  const bool vec = (((uintptr_t)a | (uintptr_t)b | (uintptr_t)g) % 16 == 0);
  int64_t j0 = c0;
  if (vec) {
    for (int64_t i = c0 + threadIdx.x * 8; i + 7 < c1; i += kThreads * 8) {
      float va[8], vb[8], o[8];
      load_vec<T, 8>(a + i, va);
      load_vec<TB, 8>(b + i, vb);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = s * sgn(va[k] - vb[k]);
      store_vec<T, 8>(g + i, o);
    }
    j0 = c0 + ((c1 - c0) / 8) * 8;
  }
  for (int64_t j = j0 + threadIdx.x; j < c1; j += kThreads)
    g[j] = from_f<T>(s * sgn(to_f<T>(a[j]) - to_f<TB>(b[j])));
}

template <typename T>
struct GanArgs {
  const T* x[kMaxT];
  T* g[kMaxT];
  int64_t n[kMaxT];
  float scale[kMaxT];  // w_t / n_t
  float pa[kMaxT], pb[kMaxT];
  int kind[kMaxT];
  int start[kMaxT + 1];
  int nt;
};

__device__ __forceinline__ float gan_phi(int kind, float a, float b, float x) {
  switch (kind) {
    case 0: return fmaxf(a + b * x, 0.f);
    case 1: return b * x;
    case 2: return fmaxf(x, 0.f) - x * a + log1pf(expf(-fabsf(x)));
    default: { const float d = x - a; return 0.5f * d * d; }
  }
}

__device__ __forceinline__ float gan_dphi(int kind, float a, float b, float x) {
  switch (kind) {
    case 0: return (a + b * x) > 0.f ? b : 0.f;
    case 1: return b;
    case 2: return 1.f / (1.f + expf(-x)) - a;
    default: return x - a;
  }
}

template <typename T>
__device__ __forceinline__ int find_gan_tensor(const GanArgs<T>& p, int bid) {
  int t = 0;
#pragma unroll
  for (int k = 1; k < kMaxT; ++k)
    if (k < p.nt && bid >= p.start[k]) t = k;
  return t;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) gan_partials(const GanArgs<T> p, float* __restrict__ part) {
  __shared__ float sh[kThreads / 64];
  const int bid = blockIdx.x;
  const int t = find_gan_tensor(p, bid);
  const int64_t c0 = (int64_t)(bid - p.start[t]) * kChunk;
  const int64_t c1 = min(p.n[t], c0 + kChunk);
  const T* __restrict__ x = p.x[t];
  const int kind = p.kind[t];
  const float a = p.pa[t], b = p.pb[t];
  float acc = 0.f;
  for (int64_t j = c0 + threadIdx.x; j < c1; j += kThreads) acc += gan_phi(kind, a, b, to_f<T>(x[j]));
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) s += sh[k];
    part[bid] = s * p.scale[t];
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) gan_grad(const GanArgs<T> p, const float* __restrict__ gout) {
  const int bid = blockIdx.x;
  const int t = find_gan_tensor(p, bid);
  const int64_t c0 = (int64_t)(bid - p.start[t]) * kChunk;
  const int64_t c1 = min(p.n[t], c0 + kChunk);
  const T* __restrict__ x = p.x[t];
  T* __restrict__ g = p.g[t];
  const int kind = p.kind[t];
  const float a = p.pa[t], b = p.pb[t], s = p.scale[t] * gout[0];
  for (int64_t j = c0 + threadIdx.x; j < c1; j += kThreads)
    g[j] = from_f<T>(s * gan_dphi(kind, a, b, to_f<T>(x[j])));
}

template <typename T>
GanArgs<T> make_gan_args(const std::vector<at::Tensor>& xs, const std::vector<int64_t>& kinds,
                         const std::vector<double>& pa, const std::vector<double>& pb,
                         const std::vector<double>& w, int& nblocks) {
  GanArgs<T> p;
  p.nt = (int)xs.size();
  int blocks = 0;
  for (int t = 0; t < kMaxT; ++t) {
    p.start[t] = blocks;
    p.g[t] = nullptr;
    if (t < p.nt) {
      p.x[t] = reinterpret_cast<const T*>(xs[t].data_ptr());
      p.n[t] = xs[t].numel();
      p.scale[t] = (float)(w[t] / (double)std::max<int64_t>(1, xs[t].numel()));
      p.kind[t] = (int)kinds[t];
      p.pa[t] = (float)pa[t];
      p.pb[t] = (float)pb[t];
      blocks += (int)((p.n[t] + kChunk - 1) / kChunk);
    } else {
      p.x[t] = nullptr;
      p.n[t] = 0;
      p.scale[t] = p.pa[t] = p.pb[t] = 0.f;
      p.kind[t] = 1;
    }
  }
  p.start[kMaxT] = blocks;
  nblocks = blocks;
  return p;
}

void check_gan(const std::vector<at::Tensor>& xs, const std::vector<int64_t>& kinds,
               const std::vector<double>& pa, const std::vector<double>& pb,
               const std::vector<double>& w) {
  IAMD_CHECK(!xs.empty() && (int)xs.size() <= kMaxT, "mt_gan_loss: 1..", kMaxT, " tensors");
  IAMD_CHECK(kinds.size() == xs.size() && pa.size() == xs.size() && pb.size() == xs.size() &&
                 w.size() == xs.size(), "mt_gan_loss: list sizes differ");
  const auto dt = xs[0].scalar_type();
  IAMD_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "mt_gan_loss: bf16 or fp32 tensors");
  for (size_t t = 0; t < xs.size(); ++t) {
    IAMD_CHECK(xs[t].is_cuda() && xs[t].scalar_type() == dt && xs[t].is_non_overlapping_and_dense(),
               "mt_gan_loss: dense CUDA tensors of one dtype expected");
    IAMD_CHECK(kinds[t] >= 0 && kinds[t] <= 3, "mt_gan_loss: kind must be 0..3");
  }
}

template <typename T, typename TB>
L1Args<T, TB> make_args(const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                        const std::vector<double>& w, int& nblocks) {
  L1Args<T, TB> p;
  p.nt = (int)a.size();
  int blocks = 0;
  for (int t = 0; t < kMaxT; ++t) {
    p.start[t] = blocks;
    if (t < p.nt) {
      p.a[t] = reinterpret_cast<const T*>(a[t].data_ptr());
      p.b[t] = reinterpret_cast<const TB*>(b[t].data_ptr());
      p.g[t] = nullptr;
      p.n[t] = a[t].numel();
      p.scale[t] = (float)(w[t] / (double)std::max<int64_t>(1, a[t].numel()));
      blocks += (int)((p.n[t] + kChunk - 1) / kChunk);
    } else {
      p.a[t] = nullptr;
      p.b[t] = nullptr;
      p.g[t] = nullptr;
      p.n[t] = 0;
      p.scale[t] = 0.f;
    }
  }
  p.start[kMaxT] = blocks;
  nblocks = blocks;
  return p;
}

void check_pairs(const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                 const std::vector<double>& w) {
  IAMD_CHECK(!a.empty() && a.size() == b.size() && a.size() == w.size(),
             "mt_l1_loss: list sizes differ");
  IAMD_CHECK((int)a.size() <= kMaxT, "mt_l1_loss: at most ", kMaxT, " pairs per call");
  const auto dt = a[0].scalar_type(), dtb = b[0].scalar_type();
  IAMD_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "mt_l1_loss: bf16 or fp32 tensors");
  IAMD_CHECK(dtb == dt || dtb == at::kFloat, "mt_l1_loss: targets of the inputs' dtype or fp32");
  for (size_t t = 0; t < a.size(); ++t) {
    IAMD_CHECK(a[t].is_cuda() && b[t].is_cuda() && a[t].scalar_type() == dt &&
                   b[t].scalar_type() == dtb,
               "mt_l1_loss: CUDA tensors, one input dtype and one target dtype expected");
    IAMD_CHECK(a[t].sizes() == b[t].sizes() && a[t].strides() == b[t].strides() &&
                   a[t].is_non_overlapping_and_dense(),
               "mt_l1_loss: pair ", t, " must be dense tensors of identical layout");
  }
}

}  // namespace

at::Tensor mt_l1_loss(const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                      const std::vector<double>& w) {
  check_pairs(a, b, w);
  auto out = at::empty({}, a[0].options().dtype(at::kFloat));
  int nb = 0;
  auto launch = [&](auto tag, auto tagb) {
    using T = decltype(tag);
    using TB = decltype(tagb);
    auto p = make_args<T, TB>(a, b, w, nb);
    auto part = at::empty({std::max(nb, 1)}, a[0].options().dtype(at::kFloat));
    if (nb > 0)
      hipLaunchKernelGGL((l1_partials<T, TB>), dim3(nb), dim3(kThreads), 0, stream(), p,
                         part.data_ptr<float>());
    hipLaunchKernelGGL(sum_fixed, dim3(1), dim3(1024), 0, stream(), part.data_ptr<float>(), nb,
                       out.data_ptr<float>());
  };
  if (a[0].scalar_type() == at::kFloat) launch(float(), float());
  else if (b[0].scalar_type() == at::kFloat) launch(__hip_bfloat16(), float());
  else launch(__hip_bfloat16(), __hip_bfloat16());
  IAMD_LAUNCH_CHECK();
  return out;
}

std::vector<at::Tensor> mt_l1_loss_backward(const std::vector<at::Tensor>& a,
                                            const std::vector<at::Tensor>& b,
                                            const std::vector<double>& w, const at::Tensor& gout) {
  check_pairs(a, b, w);
  IAMD_CHECK(gout.is_cuda() && gout.numel() == 1, "mt_l1_loss_backward: scalar grad expected");
  auto g32 = gout.to(at::kFloat).contiguous();
  std::vector<at::Tensor> grads;
  for (auto& t : a) grads.push_back(at::empty_like(t));
  int nb = 0;
  auto launch = [&](auto tag, auto tagb) {
    using T = decltype(tag);
    using TB = decltype(tagb);
    auto p = make_args<T, TB>(a, b, w, nb);
    for (size_t t = 0; t < a.size(); ++t) p.g[t] = reinterpret_cast<T*>(grads[t].data_ptr());
    if (nb > 0)
      hipLaunchKernelGGL((l1_grad<T, TB>), dim3(nb), dim3(kThreads), 0, stream(), p,
                         g32.data_ptr<float>());
  };
  if (a[0].scalar_type() == at::kFloat) launch(float(), float());
  else if (b[0].scalar_type() == at::kFloat) launch(__hip_bfloat16(), float());
  else launch(__hip_bfloat16(), __hip_bfloat16());
  IAMD_LAUNCH_CHECK();
  return grads;
}

at::Tensor mt_gan_loss(const std::vector<at::Tensor>& xs, const std::vector<int64_t>& kinds,
                       const std::vector<double>& pa, const std::vector<double>& pb,
                       const std::vector<double>& w) {
  check_gan(xs, kinds, pa, pb, w);
  auto out = at::empty({}, xs[0].options().dtype(at::kFloat));
  int nb = 0;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    auto p = make_gan_args<T>(xs, kinds, pa, pb, w, nb);
    auto part = at::empty({std::max(nb, 1)}, xs[0].options().dtype(at::kFloat));
    if (nb > 0)
      hipLaunchKernelGGL((gan_partials<T>), dim3(nb), dim3(kThreads), 0, stream(), p,
                         part.data_ptr<float>());
    hipLaunchKernelGGL(sum_fixed, dim3(1), dim3(1024), 0, stream(), part.data_ptr<float>(), nb,
                       out.data_ptr<float>());
  };
  if (xs[0].scalar_type() == at::kBFloat16) launch(__hip_bfloat16()); else launch(float());
  IAMD_LAUNCH_CHECK();
  return out;
}

std::vector<at::Tensor> mt_gan_loss_backward(const std::vector<at::Tensor>& xs,
                                             const std::vector<int64_t>& kinds,
                                             const std::vector<double>& pa,
                                             const std::vector<double>& pb,
                                             const std::vector<double>& w, const at::Tensor& gout) {
  check_gan(xs, kinds, pa, pb, w);
  IAMD_CHECK(gout.is_cuda() && gout.numel() == 1, "mt_gan_loss_backward: scalar grad expected");
  auto g32 = gout.to(at::kFloat).contiguous();
  std::vector<at::Tensor> grads;
  for (auto& t : xs) grads.push_back(at::empty_like(t));
  int nb = 0;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    auto p = make_gan_args<T>(xs, kinds, pa, pb, w, nb);
    for (size_t t = 0; t < xs.size(); ++t) p.g[t] = reinterpret_cast<T*>(grads[t].data_ptr());
    if (nb > 0)
      hipLaunchKernelGGL((gan_grad<T>), dim3(nb), dim3(kThreads), 0, stream(), p,
                         g32.data_ptr<float>());
  };
  if (xs[0].scalar_type() == at::kBFloat16) launch(__hip_bfloat16()); else launch(float());
  IAMD_LAUNCH_CHECK();
  return grads;
}

}  // namespace iamd
