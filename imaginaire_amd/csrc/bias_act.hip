// k2: fused bias + activation epilogue for conv / linear outputs.
//
// Replaces the reference's conv(bias) -> separate LeakyReLU/ReLU kernel pair
// ('CNA' / 'CA' orders with no norm, layers/conv.py:59-91): the convolution runs
// without bias on MIOpen and this kernel adds the bias and applies the
// activation in one 16-byte-vectorised pass (in place when allowed).
// Backward computes dx = dy * act'(out) and the bias gradient Σ dx per channel
// in the same pass (per-block channel partials + one tiny sum kernel).
#include "common.h"

#include <cstdlib>

namespace iamd {
namespace {

constexpr int kThreads = 256;

template <typename T, bool CL, int VEC, bool HAS_BIAS>
__global__ void __launch_bounds__(kThreads)
bias_act_fwd_kernel(const T* __restrict__ x, T* __restrict__ out, const float* __restrict__ bias,
                    int64_t total_vec, int C, int HW, float slope) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total_vec;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i * VEC;
    float v[VEC];
    load_vec<T, VEC>(x + e, v);
    if (CL) {
      const int c = (int)(e % C);
#pragma unroll
      for (int k = 0; k < VEC; ++k) v[k] = act_fwd(HAS_BIAS ? v[k] + bias[c + k] : v[k], slope);
    } else {
      const int c = (int)((e / HW) % C);
      const float b = HAS_BIAS ? bias[c] : 0.f;
#pragma unroll
      for (int k = 0; k < VEC; ++k) v[k] = act_fwd(v[k] + b, slope);
    }
    store_vec<T, VEC>(out + e, v);
  }
}

// dx = dy * act'(out); per-block channel partial sums of dx (CL layout: rows x C).
// ACT = false (identity activation): only the bias gradient is needed, dx IS dy, so the
// kernel reads dy alone and writes no dx (a third of the bytes).
// U rows per trip with all their loads issued first (more loads in flight per lane for the
// bias-only pass, which reads dy alone)
template <typename T, int VEC, bool ACT, int U>
__global__ void __launch_bounds__(kThreads)
bias_act_bwd_cl(const T* __restrict__ out, const T* __restrict__ dy, T* __restrict__ dx,
                int64_t rows, int C, int64_t rows_per_block, int tpr, float slope,
                float* __restrict__ partial) {
  __shared__ float sh[kThreads][VEC];
  const int tid = threadIdx.x;
  const int rpb = kThreads / tpr;
  const int tc = tid % tpr, r = tid / tpr;
  const int c0 = (blockIdx.y * tpr + tc) * VEC;
  const bool active = r < rpb && c0 < C;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
  if (active) {
    for (int64_t row = r0 + r; row < r1; row += (int64_t)rpb * U) {
      float o[U][VEC], g[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = row + (int64_t)u * rpb;
        if (rr < r1) {
          load_vec<T, VEC>(dy + rr * C + c0, g[u]);
          if constexpr (ACT) load_vec<T, VEC>(out + rr * C + c0, o[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = row + (int64_t)u * rpb;
        if (rr < r1) {
          if constexpr (ACT) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) g[u][k] *= act_grad(o[u][k], slope);
            store_vec<T, VEC>(dx + rr * C + c0, g[u]);
          }
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc[k] += g[u][k];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < VEC; ++k) sh[tid][k] = acc[k];
  __syncthreads();
  if (active && r == 0) {
    for (int rr = 1; rr < rpb; ++rr)
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += sh[tid + rr * tpr][k];
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      if (c0 + k < C) partial[(int64_t)blockIdx.x * C + c0 + k] = acc[k];
  }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(kThreads)
bias_act_bwd_nchw(const T* __restrict__ out, const T* __restrict__ dy, T* __restrict__ dx, int N,
                  int C, int HW, float slope, float* __restrict__ partial) {
  // grid: (N, C); one block reduces one (n, c) plane
  __shared__ float sh[kThreads / 64];
  const int n = blockIdx.x, c = blockIdx.y;
  const int64_t base = ((int64_t)n * C + c) * HW;
  float acc = 0.f;
  for (int p = threadIdx.x * VEC; p < HW; p += kThreads * VEC) {
    float o[VEC], g[VEC];
    load_vec<T, VEC>(out + base + p, o);
    load_vec<T, VEC>(dy + base + p, g);
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      g[k] *= act_grad(o[k], slope);
      acc += g[k];
    }
    store_vec<T, VEC>(dx + base + p, g);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) t += sh[i];
    partial[(int64_t)n * C + c] = t;
  }
}

// Column sums of a [P, C] fp32 matrix: block = 64 columns x 8 row-groups
// (coalesced along C), row-groups combined through LDS.
constexpr int kColRows = 16;
__global__ void __launch_bounds__(64 * kColRows)
col_sum(const float* __restrict__ partial, int P, int C, float* __restrict__ out) {
  __shared__ float sh[kColRows][64];
  const int lane = threadIdx.x, row = threadIdx.y;
  const int c = blockIdx.x * 64 + lane;
  float t = 0.f;
  if (c < C) {
    // four independent loads in flight per thread: the column walk is latency-bound
    float t1 = 0.f, t2 = 0.f, t3 = 0.f;
    int p = row;
    for (; p + 3 * kColRows < P; p += 4 * kColRows) {
      t += partial[(int64_t)p * C + c];
      t1 += partial[(int64_t)(p + kColRows) * C + c];
      t2 += partial[(int64_t)(p + 2 * kColRows) * C + c];
      t3 += partial[(int64_t)(p + 3 * kColRows) * C + c];
    }
    for (; p < P; p += kColRows) t += partial[(int64_t)p * C + c];
    t += t1 + t2 + t3;
  }
  sh[row][lane] = t;
  __syncthreads();
  if (row == 0 && c < C) {
    for (int k = 1; k < kColRows; ++k) t += sh[k][lane];
    out[c] = t;
  }
}

bool is_cl(const at::Tensor& x) {
  return x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && !x.is_contiguous();
}

}  // namespace

// x: [N, C, ...] (NCHW / channels_last / [N, C] for linear). Returns out (may alias x).
at::Tensor bias_act_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& bias, double slope,
                        bool inplace) {
  const bool cl = is_cl(x);
  IAMD_CHECK(cl || x.is_contiguous(), "bias_act: x must be contiguous or channels_last");
  const int C = (int)x.size(1);
  const int64_t HW = x.numel() / std::max<int64_t>(1, x.size(0) * C);
  at::Tensor out = inplace ? x : at::empty_like(x);
  at::Tensor bf;
  const bool hb = bias.has_value() && bias->defined();
  if (hb) bf = bias->to(at::kFloat).contiguous();
  const bool lin = x.dim() == 2;  // [N, C]: channel is fastest like CL
  const bool chan_fast = cl || lin;
  int vec = 16 / (int)x.element_size();
  while (vec > 1 && ((chan_fast ? C : HW) % vec)) vec >>= 1;
  const int64_t total_vec = x.numel() / vec;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total_vec + kThreads - 1) / kThreads, 4096));
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "bias_act_fwd", [&] {
    auto xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    auto op = reinterpret_cast<scalar_t*>(out.data_ptr());
    const float* bp = hb ? bf.data_ptr<float>() : nullptr;
    auto launch = [&](auto vt, auto clt, auto bt) {
      constexpr int V = decltype(vt)::value;
      constexpr bool CLv = decltype(clt)::value;
      constexpr bool B = decltype(bt)::value;
      hipLaunchKernelGGL((bias_act_fwd_kernel<scalar_t, CLv, V, B>), dim3(grid), dim3(kThreads), 0,
                         stream(), xp, op, bp, total_vec, C, (int)HW, (float)slope);
    };
    auto by_b = [&](auto vt, auto clt) {
      if (hb) launch(vt, clt, std::true_type()); else launch(vt, clt, std::false_type());
    };
    auto by_cl = [&](auto vt) {
      if (chan_fast) by_b(vt, std::true_type()); else by_b(vt, std::false_type());
    };
    switch (vec) {
      case 8: by_cl(std::integral_constant<int, 8>()); break;
      case 4: by_cl(std::integral_constant<int, 4>()); break;
      case 2: by_cl(std::integral_constant<int, 2>()); break;
      default: by_cl(std::integral_constant<int, 1>()); break;
    }
  });
  IAMD_LAUNCH_CHECK();
  return out;
}

// Returns (dx, dbias[C] fp32).
std::vector<at::Tensor> bias_act_bwd(const at::Tensor& out, const at::Tensor& dy_in, double slope) {
  const bool cl = is_cl(out);
  const bool lin = out.dim() == 2;
  at::Tensor dy = cl ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  if (dy.scalar_type() != out.scalar_type()) dy = dy.to(out.scalar_type());
  const int N = (int)out.size(0), C = (int)out.size(1);
  const int64_t HW = out.numel() / std::max<int64_t>(1, (int64_t)N * C);
  // identity activation on the channels-fast path: the kernel writes no dx, dx is dy itself
  auto dx = ((cl || lin) && slope == 1.0) ? dy : at::empty_like(out);
  auto fopt = out.options().dtype(at::kFloat);
  // one allocation for the partials and db (db is its tail): the partials live as long as db,
  // so no later allocation of the (graph) pool can reuse their block while the column sum
  // might still read them
  at::Tensor buf, partial;
  int P;
  IAMD_DISPATCH_FLOAT_TYPES(out.scalar_type(), "bias_act_bwd", [&] {
    auto op = reinterpret_cast<const scalar_t*>(out.data_ptr());
    auto gp = reinterpret_cast<const scalar_t*>(dy.data_ptr());
    auto dp = reinterpret_cast<scalar_t*>(dx.data_ptr());
    if (cl || lin) {
      int vec = 16 / (int)out.element_size();
      while (vec > 1 && (C % vec)) vec >>= 1;
      const int tpr = std::max(1, std::min(C / vec, kThreads));
      const int nzc = ceil_div(C, (int64_t)tpr * vec);
      const int64_t rows = (int64_t)N * HW;
      const int rpb = kThreads / tpr;
      int64_t rows_per_block = std::max<int64_t>(rpb * 4, (rows + 511) / 512);
      P = (int)((rows + rows_per_block - 1) / rows_per_block);
      buf = at::empty({(int64_t)P * C + C}, fopt);
      partial = buf.narrow(0, 0, (int64_t)P * C);
      const bool act = slope != 1.0;
      // IMAGINAIRE_AMD_BIASACT_UNROLL (read per call, A/B): rows per trip, 4 or 1. Default: 4 for
      // the bias-only pass (1.00-1.17x), 1 with an activation (already 4.7-5.7 TB/s; 0.97-1.00x
      // unrolled): profiles/bias_act_bwd_unroll_ab_r6_mi355x.txt
      const char* ue = std::getenv("IMAGINAIRE_AMD_BIASACT_UNROLL");
      const bool unroll = ue == nullptr ? !act : std::atoi(ue) != 1;
      auto launch = [&](auto vt) {
        constexpr int V = decltype(vt)::value;
        auto go = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(P, nzc), dim3(kThreads), 0, stream(), op, gp, dp, rows, C,
                             rows_per_block, tpr, (float)slope, partial.data_ptr<float>());
        };
        if (act && unroll) go(bias_act_bwd_cl<scalar_t, V, true, 4>);
        else if (act) go(bias_act_bwd_cl<scalar_t, V, true, 1>);
        else if (unroll) go(bias_act_bwd_cl<scalar_t, V, false, 4>);
        else go(bias_act_bwd_cl<scalar_t, V, false, 1>);
      };
      switch (vec) {
        case 8: launch(std::integral_constant<int, 8>()); break;
        case 4: launch(std::integral_constant<int, 4>()); break;
        case 2: launch(std::integral_constant<int, 2>()); break;
        default: launch(std::integral_constant<int, 1>()); break;
      }
    } else {
      int vec = 16 / (int)out.element_size();
      while (vec > 1 && (HW % vec)) vec >>= 1;
      P = N;
      buf = at::empty({(int64_t)N * C + C}, fopt);
      partial = buf.narrow(0, 0, (int64_t)N * C);
      auto launch = [&](auto vt) {
        constexpr int V = decltype(vt)::value;
        hipLaunchKernelGGL((bias_act_bwd_nchw<scalar_t, V>), dim3(N, C), dim3(kThreads), 0,
                           stream(), op, gp, dp, N, C, (int)HW, (float)slope,
                           partial.data_ptr<float>());
      };
      switch (vec) {
        case 8: launch(std::integral_constant<int, 8>()); break;
        case 4: launch(std::integral_constant<int, 4>()); break;
        case 2: launch(std::integral_constant<int, 2>()); break;
        default: launch(std::integral_constant<int, 1>()); break;
      }
    }
  });
  IAMD_LAUNCH_CHECK();
  auto db = buf.narrow(0, (int64_t)P * C, C);
  hipLaunchKernelGGL(col_sum, dim3(ceil_div(C, 64)), dim3(64, kColRows), 0, stream(),
                     partial.data_ptr<float>(), P, C, db.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  return {dx, db};
}

}  // namespace iamd
