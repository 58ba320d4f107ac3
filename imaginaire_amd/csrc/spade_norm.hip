// k1: fused normalisation + spatially-adaptive modulation + activation.
//
// Covers the reference's hot normalisation paths in one kernel family:
//   SpatiallyAdaptiveNorm (layers/activation_norm.py:211-234):
//       out = act( (norm(x)*a + b) * (1 + gamma) + beta )
//   AdaptiveNorm / AdaIN (activation_norm.py:79-106): per-(n,c) scale/shift
//   plain BatchNorm / SyncBatchNorm / InstanceNorm + activation ('NA' orders)
// with the activation of the following 'A' in the block order (leaky-relu 0.2
// for SPADE's 'NACNAC'), expressed as a slope (1 = identity, 0 = relu).
//
// Three passes, each a single streaming read of the activation:
//   stats   : per-(n, pixel-chunk, c) shifted (count, mean, M2) partials, merged
//             with Chan's formula -> robust fp32 statistics;
//   finalize: merge partials over chunks (and over n for batch statistics) and
//             fold affine weight/bias into per-(g,c) scale/shift;
//   apply   : 16-byte vectorised elementwise modulation + activation.
// Backward mirrors it: reduce (writes dgamma/dbeta, accumulates Σg, Σg·x̂),
// then apply (dx). For SyncBN the per-rank partial statistics are exchanged by
// the Python layer with one RCCL collective between the passes.
//
// Layouts: channels-last (NHWC, CL=true, vector runs along C) and NCHW (vector
// runs along HW). gamma/beta/dgamma/dbeta are strided views so the gamma/beta
// halves of one fused conv output ([.., 2C]) are consumed without a copy.
#include "common.h"

namespace iamd {
namespace {

constexpr int kThreads = 256;

struct ModView {
  const void* ptr;
  int64_t sn, sc, sp;  // element strides for batch, channel, pixel
};

// ------------------------------------------------------------------------
// stats partials
// ------------------------------------------------------------------------
template <typename T, int VEC>
__global__ void __launch_bounds__(kThreads)
stats_partial_cl(const T* __restrict__ x, int C, int HW, int P, int chunk, int tpr,
                 float* __restrict__ pcnt, float* __restrict__ pmean, float* __restrict__ pm2) {
  __shared__ float sh_n[kThreads];
  __shared__ float sh_mean[kThreads][VEC];
  __shared__ float sh_m2[kThreads][VEC];
  const int tid = threadIdx.x;
  const int rpb = kThreads / tpr;
  const int tc = tid % tpr, r = tid / tpr;
  const int p = blockIdx.x, n = blockIdx.y;
  const int c0 = (blockIdx.z * tpr + tc) * VEC;
  const bool active = (r < rpb) && (c0 < C);
  const int pix0 = p * chunk, pix1 = min(HW, pix0 + chunk);

  float K[VEC], s1[VEC], s2[VEC];
  float cnt = 0.f;
#pragma unroll
  for (int v = 0; v < VEC; ++v) { K[v] = 0.f; s1[v] = 0.f; s2[v] = 0.f; }
  if (active) {
    const T* base = x + (int64_t)n * HW * C + c0;
    int pix = pix0 + r;
    if (pix < pix1) {
      float xv[VEC];
      load_vec<T, VEC>(base + (int64_t)pix * C, xv);
#pragma unroll
      for (int v = 0; v < VEC; ++v) K[v] = xv[v];
    }
    for (; pix < pix1; pix += rpb) {
      float xv[VEC];
      load_vec<T, VEC>(base + (int64_t)pix * C, xv);
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float d = xv[v] - K[v];
        s1[v] += d;
        s2[v] = fmaf(d, d, s2[v]);
      }
      cnt += 1.f;
    }
  }
  // shifted sums -> (count, mean, M2)
  sh_n[tid] = cnt;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    float m = cnt > 0.f ? s1[v] / cnt : 0.f;
    sh_mean[tid][v] = K[v] + m;
    sh_m2[tid][v] = cnt > 0.f ? fmaxf(s2[v] - s1[v] * m, 0.f) : 0.f;
  }
  __syncthreads();
  int s = 1;
  while (s < rpb) s <<= 1;
  for (s >>= 1; s > 0; s >>= 1) {
    if (active && r < s && r + s < rpb) {
      const int o = tid + s * tpr;
      float na = sh_n[tid];
      float nb = sh_n[o];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float n_a = na, mean_a = sh_mean[tid][v], m2_a = sh_m2[tid][v];
        chan_merge(n_a, mean_a, m2_a, nb, sh_mean[o][v], sh_m2[o][v]);
        sh_mean[tid][v] = mean_a;
        sh_m2[tid][v] = m2_a;
      }
      sh_n[tid] = na + nb;
    }
    __syncthreads();
  }
  if (active && r == 0) {
    const int64_t o = ((int64_t)n * P + p) * C + c0;
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      if (c0 + v < C) {
        pcnt[o + v] = sh_n[tid];
        pmean[o + v] = sh_mean[tid][v];
        pm2[o + v] = sh_m2[tid][v];
      }
    }
  }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(kThreads)
stats_partial_nchw(const T* __restrict__ x, int C, int HW, int P, int chunk,
                   float* __restrict__ pcnt, float* __restrict__ pmean, float* __restrict__ pm2) {
  __shared__ float sh_n[kThreads], sh_mean[kThreads], sh_m2[kThreads];
  const int tid = threadIdx.x;
  const int p = blockIdx.x, n = blockIdx.y, c = blockIdx.z;
  const int pix0 = p * chunk, pix1 = min(HW, pix0 + chunk);
  const T* base = x + ((int64_t)n * C + c) * HW;
  float K = 0.f, s1 = 0.f, s2 = 0.f, cnt = 0.f;
  int pix = pix0 + tid * VEC;
  if (pix < pix1) K = to_f<T>(base[pix]);
  for (; pix < pix1; pix += kThreads * VEC) {
    float xv[VEC];
    load_vec<T, VEC>(base + pix, xv);
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float d = xv[v] - K;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
    cnt += (float)VEC;
  }
  float m = cnt > 0.f ? s1 / cnt : 0.f;
  sh_n[tid] = cnt;
  sh_mean[tid] = K + m;
  sh_m2[tid] = cnt > 0.f ? fmaxf(s2 - s1 * m, 0.f) : 0.f;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (tid < s) {
      float na = sh_n[tid], mean_a = sh_mean[tid], m2_a = sh_m2[tid];
      chan_merge(na, mean_a, m2_a, sh_n[tid + s], sh_mean[tid + s], sh_m2[tid + s]);
      sh_n[tid] = na; sh_mean[tid] = mean_a; sh_m2[tid] = m2_a;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int64_t o = ((int64_t)n * P + p) * C + c;
    pcnt[o] = sh_n[0];
    pmean[o] = sh_mean[0];
    pm2[o] = sh_m2[0];
  }
}

// Merge partials [N][P][C] -> per-group (count, mean, var) and fold the
// per-channel affine (a, b) into scale/shift. G = N (instance) or 1 (batch).
// Parallel merge: block = 64 channels (one wave across channels -> coalesced
// partial reads) x kFinRows row-groups, each row-group Chan-merges a strided
// subset of the N*P partial rows, then the row-groups merge through LDS.
// Grid = (ceil(C/64), G). Replaces a one-thread-per-channel serial merge.
constexpr int kFinRows = 8;
// Stage 1 of the partial merge (latency hiding): grid (ceil(C/64), G, RS); each
// block Chan-merges its slice of the N*P partial rows of group g into one
// (count, mean, M2) row of tmp [G][RS][C]. Stage 2 (stats_finalize) merges RS.
__global__ void __launch_bounds__(64 * kFinRows)
stats_merge_rows(const float* __restrict__ pcnt, const float* __restrict__ pmean,
                 const float* __restrict__ pm2, int N, int P, int C, int per_instance, int RS,
                 float* __restrict__ tcnt, float* __restrict__ tmean, float* __restrict__ tm2) {
  __shared__ float sh_n[kFinRows][64], sh_mean[kFinRows][64], sh_m2[kFinRows][64];
  const int lane = threadIdx.x, row = threadIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const int g = blockIdx.y, rs = blockIdx.z;
  const int n_lo = per_instance ? g : 0, n_hi = per_instance ? g + 1 : N;
  const int rows = (n_hi - n_lo) * P;
  const int per = (rows + RS - 1) / RS;
  const int r0 = rs * per, r1 = min(rows, r0 + per);
  float n_a = 0.f, mean_a = 0.f, m2_a = 0.f;
  if (c < C) {
    for (int r = r0 + row; r < r1; r += kFinRows) {
      const int64_t o = ((int64_t)(n_lo * P + r)) * C + c;
      chan_merge(n_a, mean_a, m2_a, pcnt[o], pmean[o], pm2[o]);
    }
  }
  sh_n[row][lane] = n_a;
  sh_mean[row][lane] = mean_a;
  sh_m2[row][lane] = m2_a;
  __syncthreads();
  if (row != 0 || c >= C) return;
  for (int k = 1; k < kFinRows; ++k)
    chan_merge(n_a, mean_a, m2_a, sh_n[k][lane], sh_mean[k][lane], sh_m2[k][lane]);
  const int64_t o = ((int64_t)g * RS + rs) * C + c;
  tcnt[o] = n_a;
  tmean[o] = mean_a;
  tm2[o] = m2_a;
}

__global__ void __launch_bounds__(64 * kFinRows)
stats_finalize(const float* __restrict__ pcnt, const float* __restrict__ pmean,
               const float* __restrict__ pm2, int N, int P, int C, int per_instance,
               float eps, const float* __restrict__ weight,
               const float* __restrict__ bias, float* __restrict__ out_cnt,
               float* __restrict__ out_mean, float* __restrict__ out_var,
               float* __restrict__ out_scale, float* __restrict__ out_shift,
               float* __restrict__ out_rstd, float* __restrict__ run_mean,
               float* __restrict__ run_var, int64_t* __restrict__ num_batches, float factor) {
  __shared__ float sh_n[kFinRows][64], sh_mean[kFinRows][64], sh_m2[kFinRows][64];
  const int lane = threadIdx.x, row = threadIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const int g = blockIdx.y;
  const int n_lo = per_instance ? g : 0, n_hi = per_instance ? g + 1 : N;
  const int rows = (n_hi - n_lo) * P;
  float n_a = 0.f, mean_a = 0.f, m2_a = 0.f;
  if (c < C) {
    for (int r = row; r < rows; r += kFinRows) {
      const int64_t o = ((int64_t)(n_lo * P + r)) * C + c;
      chan_merge(n_a, mean_a, m2_a, pcnt[o], pmean[o], pm2[o]);
    }
  }
  sh_n[row][lane] = n_a;
  sh_mean[row][lane] = mean_a;
  sh_m2[row][lane] = m2_a;
  __syncthreads();
  if (row != 0 || c >= C) return;
  for (int k = 1; k < kFinRows; ++k)
    chan_merge(n_a, mean_a, m2_a, sh_n[k][lane], sh_mean[k][lane], sh_m2[k][lane]);
  const int idx = g * C + c;
  const float var = n_a > 0.f ? m2_a / n_a : 0.f;
  out_cnt[idx] = n_a;
  out_mean[idx] = mean_a;
  out_var[idx] = var;
  const float rstd = rsqrtf(var + eps);
  if (out_rstd != nullptr) out_rstd[idx] = rstd;
  if (out_scale != nullptr) {
    const float a = weight ? weight[c] : 1.f;
    const float b = bias ? bias[c] : 0.f;
    out_scale[idx] = rstd * a;
    out_shift[idx] = b - mean_a * rstd * a;
  }
  // running statistics (one group: batch norm), unbiased variance as torch's BatchNorm:
  // r <- (1 - f) r + f x, in place — replaces ~9 one-element-per-channel PyTorch launches
  if (run_mean != nullptr) {
    const float unb = var * n_a / fmaxf(n_a - 1.f, 1.f);
    run_mean[c] = (1.f - factor) * run_mean[c] + factor * mean_a;
    run_var[c] = (1.f - factor) * run_var[c] + factor * unb;
  }
  if (num_batches != nullptr && idx == 0) num_batches[0] += 1;
}

// Sync-BN: merge the all-gathered per-rank (count, mean, var) rows allst [W][3][C] (Chan) and
// finish like stats_finalize — global (count, mean, var), rstd, the affine scale / shift, and the
// running statistics + batch counter in place — in ONE launch (PyTorch: ~25 one-element-per-
// channel launches per sync-BN layer: the merge, rsqrt, scale / shift and the running update).
__global__ void __launch_bounds__(256)
sync_stats_merge_kernel(const float* __restrict__ allst, int W, int C, float eps,
                        const float* __restrict__ weight, const float* __restrict__ bias,
                        float* __restrict__ out_cnt, float* __restrict__ out_mean,
                        float* __restrict__ out_var, float* __restrict__ out_rstd,
                        float* __restrict__ out_scale, float* __restrict__ out_shift,
                        float* __restrict__ run_mean, float* __restrict__ run_var,
                        int64_t* __restrict__ num_batches, float factor) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float n_a = 0.f, mean_a = 0.f, m2_a = 0.f;
  for (int w = 0; w < W; ++w) {
    const float* r = allst + (int64_t)w * 3 * C;
    const float n = r[c];
    chan_merge(n_a, mean_a, m2_a, n, r[C + c], r[2 * C + c] * n);
  }
  const float var = n_a > 0.f ? m2_a / n_a : 0.f;
  const float rstd = rsqrtf(var + eps);
  out_cnt[c] = n_a;
  out_mean[c] = mean_a;
  out_var[c] = var;
  out_rstd[c] = rstd;
  const float a = weight ? weight[c] : 1.f;
  const float b = bias ? bias[c] : 0.f;
  out_scale[c] = rstd * a;
  out_shift[c] = b - mean_a * rstd * a;
  if (run_mean != nullptr) {
    const float unb = var * n_a / fmaxf(n_a - 1.f, 1.f);
    run_mean[c] = (1.f - factor) * run_mean[c] + factor * mean_a;
    run_var[c] = (1.f - factor) * run_var[c] + factor * unb;
  }
  if (num_batches != nullptr && c == 0) num_batches[0] += 1;
}

// Backward coefficients of the k1 data gradient from the per-sample sums S1 = Σ g', S2 =
// Σ g'·x̂ ([N, C] each) in one launch (PyTorch: 2 column sums, a stack, a multiply and two
// divides with their copies per norm layer). Batch norm (per_instance 0): k1 = rstd·w, k2 =
// ΣS1·invM, k3 = ΣS2·invM ([1, C]); instance norm: k1 = rstd·w, k2 = S1·invM, k3 = S2·invM
// ([N, C], invM = 1/HW). dw = ΣS2, db = ΣS1 over the batch (affine gradients).
__global__ void __launch_bounds__(256)
norm_bwd_coeffs_kernel(const float* __restrict__ S1, const float* __restrict__ S2,
                       const float* __restrict__ rstd, const float* __restrict__ w, int N, int C,
                       int per_instance, float invM, float* __restrict__ k1,
                       float* __restrict__ k2, float* __restrict__ k3, float* __restrict__ dw,
                       float* __restrict__ db) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float a = w ? w[c] : 1.f;
  float s1 = 0.f, s2 = 0.f;
  for (int n = 0; n < N; ++n) {
    const float x1 = S1[(int64_t)n * C + c], x2 = S2[(int64_t)n * C + c];
    s1 += x1;
    s2 += x2;
    if (per_instance) {
      const int64_t o = (int64_t)n * C + c;
      k1[o] = rstd[o] * a;
      k2[o] = x1 * invM;
      k3[o] = x2 * invM;
    }
  }
  if (!per_instance) {
    k1[c] = rstd[c] * a;
    k2[c] = s1 * invM;
    k3[c] = s2 * invM;
  }
  if (dw != nullptr) dw[c] = s2;
  if (db != nullptr) db[c] = s1;
}

// ------------------------------------------------------------------------
// forward apply
// ------------------------------------------------------------------------
template <typename T, bool CL, int VEC, bool MOD>
__global__ void __launch_bounds__(kThreads)
apply_fwd(const T* __restrict__ x, T* __restrict__ out, int N, int C, int HW,
          const float* __restrict__ scale, const float* __restrict__ shift, int per_n,
          ModView gam, ModView bet, float slope) {
  const int64_t total = (int64_t)N * C * HW / VEC;
  const T* __restrict__ gp = reinterpret_cast<const T*>(gam.ptr);
  const T* __restrict__ bp = reinterpret_cast<const T*>(bet.ptr);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i * VEC;
    int n, c, p;
    if (CL) {
      c = (int)(e % C);
      const int64_t np = e / C;
      p = (int)(np % HW);
      n = (int)(np / HW);
    } else {
      p = (int)(e % HW);
      const int64_t nc = e / HW;
      c = (int)(nc % C);
      n = (int)(nc / C);
    }
    float xv[VEC], o[VEC];
    load_vec<T, VEC>(x + e, xv);
    const int64_t sidx = (int64_t)(per_n ? n : 0) * C + c;
    float gv[VEC], bv[VEC];
    if (MOD) {
      load_vec<T, VEC>(gp + n * gam.sn + (int64_t)c * gam.sc + (int64_t)p * gam.sp, gv);
      load_vec<T, VEC>(bp + n * bet.sn + (int64_t)c * bet.sc + (int64_t)p * bet.sp, bv);
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int64_t si = CL ? sidx + v : sidx;
      float y = fmaf(xv[v], scale[si], shift[si]);
      if (MOD) y = fmaf(y, 1.f + gv[v], bv[v]);
      o[v] = act_fwd(y, slope);
    }
    store_vec<T, VEC>(out + e, o);
  }
}

// ------------------------------------------------------------------------
// backward reduce: writes dgamma / dbeta, accumulates S1 = Σ g, S2 = Σ g·x̂
// per (n, pixel-chunk, c) where g = d(norm-affine output).
// ------------------------------------------------------------------------
template <typename T, bool CL, int VEC, bool MOD, bool BCAST>
__global__ void __launch_bounds__(kThreads)
bwd_reduce(const T* __restrict__ x, const T* __restrict__ dout, int N, int C, int HW, int P,
           int chunk, int tpr, const float* __restrict__ scale, const float* __restrict__ shift,
           const float* __restrict__ mean, const float* __restrict__ rstd, int per_n_aff,
           int per_n_stat, ModView gam, ModView bet, ModView dgam, ModView dbet, float slope,
           float* __restrict__ ps1, float* __restrict__ ps2, float* __restrict__ ps3,
           float* __restrict__ ps4) {
  // BCAST: gamma/beta are per-(n,c) (pixel stride 0, AdaIN / CBN); their
  // gradients are pixel reductions (S3 = Σ dy·nrm, S4 = Σ dy) instead of maps.
  __shared__ float sh1[kThreads][CL ? VEC : 1];
  __shared__ float sh2[kThreads][CL ? VEC : 1];
  __shared__ float sh3[BCAST ? kThreads : 1][CL ? VEC : 1];
  __shared__ float sh4[BCAST ? kThreads : 1][CL ? VEC : 1];
  const T* __restrict__ gp = reinterpret_cast<const T*>(gam.ptr);
  const T* __restrict__ bp = reinterpret_cast<const T*>(bet.ptr);
  T* __restrict__ dgp = reinterpret_cast<T*>(const_cast<void*>(dgam.ptr));
  T* __restrict__ dbp = reinterpret_cast<T*>(const_cast<void*>(dbet.ptr));
  const int tid = threadIdx.x;
  const int p = blockIdx.x, n = blockIdx.y;
  const int pix0 = p * chunk, pix1 = min(HW, pix0 + chunk);
  if (CL) {
    const int rpb = kThreads / tpr;
    const int tc = tid % tpr, r = tid / tpr;
    const int c0 = (blockIdx.z * tpr + tc) * VEC;
    const bool active = (r < rpb) && (c0 < C);
    float a1[VEC], a2[VEC], a3[VEC], a4[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) { a1[v] = 0.f; a2[v] = 0.f; a3[v] = 0.f; a4[v] = 0.f; }
    if (active) {
      float sc[VEC], sh[VEC], mu[VEC], rs[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int64_t ai = (int64_t)(per_n_aff ? n : 0) * C + c0 + v;
        const int64_t si = (int64_t)(per_n_stat ? n : 0) * C + c0 + v;
        sc[v] = scale[ai]; sh[v] = shift[ai]; mu[v] = mean[si]; rs[v] = rstd[si];
      }
      for (int pix = pix0 + r; pix < pix1; pix += rpb) {
        const int64_t e = ((int64_t)n * HW + pix) * C + c0;
        float xv[VEC], dv[VEC], gv[VEC], bv[VEC], dg[VEC], db[VEC];
        load_vec<T, VEC>(x + e, xv);
        load_vec<T, VEC>(dout + e, dv);
        const int64_t go = n * gam.sn + (int64_t)c0 * gam.sc + (int64_t)pix * gam.sp;
        const int64_t bo = n * bet.sn + (int64_t)c0 * bet.sc + (int64_t)pix * bet.sp;
        if (MOD) {
          load_vec<T, VEC>(gp + go, gv);
          load_vec<T, VEC>(bp + bo, bv);
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float nrm = fmaf(xv[v], sc[v], sh[v]);
          float y = nrm, g;
          if (MOD) y = fmaf(nrm, 1.f + gv[v], bv[v]);
          const float dy = dv[v] * act_grad(y, slope);
          if (MOD) {
            dg[v] = dy * nrm;
            db[v] = dy;
            g = dy * (1.f + gv[v]);
          } else {
            g = dy;
          }
          const float xh = (xv[v] - mu[v]) * rs[v];
          a1[v] += g;
          a2[v] = fmaf(g, xh, a2[v]);
          if (BCAST) { a3[v] += dg[v]; a4[v] += db[v]; }
        }
        if (MOD && !BCAST) {
          store_vec<T, VEC>(dgp + n * dgam.sn + (int64_t)c0 * dgam.sc + (int64_t)pix * dgam.sp, dg);
          store_vec<T, VEC>(dbp + n * dbet.sn + (int64_t)c0 * dbet.sc + (int64_t)pix * dbet.sp, db);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      sh1[tid][v] = a1[v]; sh2[tid][v] = a2[v];
      if (BCAST) { sh3[tid][v] = a3[v]; sh4[tid][v] = a4[v]; }
    }
    __syncthreads();
    int s = 1;
    while (s < rpb) s <<= 1;
    for (s >>= 1; s > 0; s >>= 1) {
      if (active && r < s && r + s < rpb) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          sh1[tid][v] += sh1[tid + s * tpr][v];
          sh2[tid][v] += sh2[tid + s * tpr][v];
          if (BCAST) {
            sh3[tid][v] += sh3[tid + s * tpr][v];
            sh4[tid][v] += sh4[tid + s * tpr][v];
          }
        }
      }
      __syncthreads();
    }
    if (active && r == 0) {
      const int64_t o = ((int64_t)n * P + p) * C + c0;
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        if (c0 + v < C) {
          ps1[o + v] = sh1[tid][v]; ps2[o + v] = sh2[tid][v];
          if (BCAST) { ps3[o + v] = sh3[tid][v]; ps4[o + v] = sh4[tid][v]; }
        }
    }
  } else {
    const int c = blockIdx.z;
    const int64_t ai = (int64_t)(per_n_aff ? n : 0) * C + c;
    const int64_t si = (int64_t)(per_n_stat ? n : 0) * C + c;
    const float sc = scale[ai], sh = shift[ai], mu = mean[si], rs = rstd[si];
    float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
    const int64_t base = ((int64_t)n * C + c) * HW;
    for (int pix = pix0 + tid * VEC; pix < pix1; pix += kThreads * VEC) {
      float xv[VEC], dv[VEC], gv[VEC], bv[VEC], dg[VEC], db[VEC];
      load_vec<T, VEC>(x + base + pix, xv);
      load_vec<T, VEC>(dout + base + pix, dv);
      if (MOD) {
        load_vec<T, VEC>(gp + n * gam.sn + (int64_t)c * gam.sc + pix * gam.sp, gv);
        load_vec<T, VEC>(bp + n * bet.sn + (int64_t)c * bet.sc + pix * bet.sp, bv);
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float nrm = fmaf(xv[v], sc, sh);
        float y = nrm, g;
        if (MOD) y = fmaf(nrm, 1.f + gv[v], bv[v]);
        const float dy = dv[v] * act_grad(y, slope);
        if (MOD) {
          dg[v] = dy * nrm; db[v] = dy; g = dy * (1.f + gv[v]);
        } else {
          g = dy;
        }
        a1 += g;
        a2 = fmaf(g, (xv[v] - mu) * rs, a2);
        if (BCAST) { a3 += dg[v]; a4 += db[v]; }
      }
      if (MOD && !BCAST) {
        store_vec<T, VEC>(dgp + n * dgam.sn + (int64_t)c * dgam.sc + pix * dgam.sp, dg);
        store_vec<T, VEC>(dbp + n * dbet.sn + (int64_t)c * dbet.sc + pix * dbet.sp, db);
      }
    }
    a1 = wave_sum(a1);
    a2 = wave_sum(a2);
    if (BCAST) { a3 = wave_sum(a3); a4 = wave_sum(a4); }
    const int lane = tid & 63, w = tid >> 6;
    if (lane == 0) {
      sh1[w][0] = a1; sh2[w][0] = a2;
      if (BCAST) { sh3[w][0] = a3; sh4[w][0] = a4; }
    }
    __syncthreads();
    if (tid == 0) {
      float t1 = 0.f, t2 = 0.f, t3 = 0.f, t4 = 0.f;
      for (int i = 0; i < kThreads / 64; ++i) {
        t1 += sh1[i][0]; t2 += sh2[i][0];
        if (BCAST) { t3 += sh3[i][0]; t4 += sh4[i][0]; }
      }
      const int64_t o = ((int64_t)n * P + p) * C + c;
      ps1[o] = t1;
      ps2[o] = t2;
      if (BCAST) { ps3[o] = t3; ps4[o] = t4; }
    }
  }
}

// Sum partials over the chunk axis: [N][P][C] -> [N][C].
// ps: Q planes of [N][P][C] (plane stride qstride) -> out: Q planes of [N][C].
// Block = 64 channels x kFinRows partial-row groups; grid = (ceil(C/64), N, Q).
__global__ void __launch_bounds__(64 * kFinRows)
sum_partials(const float* __restrict__ ps, int Q, int64_t qstride, int N, int P, int C, int RS,
             float* __restrict__ out) {
  // grid (ceil(C/64), N, Q*RS): RS row-splits per (n, q) accumulate into a zeroed out
  __shared__ float sh[kFinRows][64];
  const int lane = threadIdx.x, row = threadIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const int n = blockIdx.y, q = blockIdx.z / RS, rs = blockIdx.z % RS;
  const int per = (P + RS - 1) / RS;
  const int p0 = rs * per, p1 = min(P, p0 + per);
  float t = 0.f;
  if (c < C)
    for (int p = p0 + row; p < p1; p += kFinRows)
      t += ps[q * qstride + ((int64_t)n * P + p) * C + c];
  sh[row][lane] = t;
  __syncthreads();
  if (row == 0 && c < C) {
    for (int k = 1; k < kFinRows; ++k) t += sh[k][lane];
    float* o = out + (int64_t)q * N * C + (int64_t)n * C + c;
    if (RS == 1) *o = t; else atomicAdd(o, t);
  }
}

// ------------------------------------------------------------------------
// backward apply: dx = k1 * (g - k2 - x̂ * k3)   (per-(group, c) coefficients)
// ------------------------------------------------------------------------
template <typename T, bool CL, int VEC, bool MOD>
__global__ void __launch_bounds__(kThreads)
bwd_apply(const T* __restrict__ x, const T* __restrict__ dout, T* __restrict__ dx, int N, int C,
          int HW, const float* __restrict__ scale, const float* __restrict__ shift, int per_n_aff,
          const float* __restrict__ mean, const float* __restrict__ rstd,
          const float* __restrict__ k1, const float* __restrict__ k2, const float* __restrict__ k3,
          int per_n_stat, ModView gam, ModView bet, float slope) {
  const int64_t total = (int64_t)N * C * HW / VEC;
  const T* __restrict__ gp = reinterpret_cast<const T*>(gam.ptr);
  const T* __restrict__ bp = reinterpret_cast<const T*>(bet.ptr);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i * VEC;
    int n, c, p;
    if (CL) {
      c = (int)(e % C);
      const int64_t np = e / C;
      p = (int)(np % HW);
      n = (int)(np / HW);
    } else {
      p = (int)(e % HW);
      const int64_t nc = e / HW;
      c = (int)(nc % C);
      n = (int)(nc / C);
    }
    float xv[VEC], dv[VEC], gv[VEC], bv[VEC], o[VEC];
    load_vec<T, VEC>(x + e, xv);
    load_vec<T, VEC>(dout + e, dv);
    if (MOD) {
      load_vec<T, VEC>(gp + n * gam.sn + (int64_t)c * gam.sc + (int64_t)p * gam.sp, gv);
      load_vec<T, VEC>(bp + n * bet.sn + (int64_t)c * bet.sc + (int64_t)p * bet.sp, bv);
    }
    const int64_t ai = (int64_t)(per_n_aff ? n : 0) * C + c;
    const int64_t si = (int64_t)(per_n_stat ? n : 0) * C + c;
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int64_t av = CL ? ai + v : ai, sv = CL ? si + v : si;
      const float nrm = fmaf(xv[v], scale[av], shift[av]);
      float y = nrm;
      if (MOD) y = fmaf(nrm, 1.f + gv[v], bv[v]);
      float g = dv[v] * act_grad(y, slope);
      if (MOD) g *= (1.f + gv[v]);
      const float xh = (xv[v] - mean[sv]) * rstd[sv];
      o[v] = k1[sv] * (g - k2[sv] - xh * k3[sv]);
    }
    store_vec<T, VEC>(dx + e, o);
  }
}

// ------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------
struct Geom {
  int N, C, HW;
  bool cl;
};

Geom geom_of(const at::Tensor& x) {
  IAMD_CHECK(x.dim() == 4, "expected NCHW-shaped 4-D tensor");
  Geom g{(int)x.size(0), (int)x.size(1), (int)(x.size(2) * x.size(3)), false};
  if (x.is_contiguous(at::MemoryFormat::ChannelsLast) && !x.is_contiguous()) {
    g.cl = true;
  } else if (x.is_contiguous()) {
    g.cl = false;
  } else if (x.is_contiguous(at::MemoryFormat::ChannelsLast)) {
    g.cl = true;
  } else {
    IAMD_CHECK(false, "tensor must be NCHW- or channels_last-contiguous");
  }
  // 1x1 spatial tensors are both; treat as NCHW.
  return g;
}

ModView view_of(const c10::optional<at::Tensor>& t, const Geom& g) {
  if (!t.has_value() || !t->defined()) return ModView{nullptr, 0, 0, 0};
  const auto& a = *t;
  IAMD_CHECK(a.dim() == 4 && a.size(0) == g.N && a.size(1) == g.C &&
                 a.size(2) * a.size(3) == g.HW,
             "modulation tensor shape mismatch");
  // pixel stride: along W (H stride must equal W*pixel stride for flat pixel indexing)
  const int64_t sp = a.stride(3);
  IAMD_CHECK(a.size(2) == 1 || a.stride(2) == a.size(3) * sp, "modulation tensor pixel layout");
  return ModView{a.data_ptr(), a.stride(0), a.stride(1), sp};
}

int pick_vec(const Geom& g, int elem_size, const std::vector<ModView>& mods) {
  int vec = 16 / elem_size;
  auto ok = [&](int v) {
    if (g.cl) {
      if (g.C % v) return false;
      for (auto& m : mods)
        if (m.ptr && (m.sc != 1 || (m.sp % v) || (m.sn % v) ||
                      (reinterpret_cast<uintptr_t>(m.ptr) % (v * elem_size))))
          return false;
    } else {
      if (g.HW % v) return false;
      for (auto& m : mods)
        if (m.ptr && (m.sp != 1 || (m.sc % v) || (m.sn % v) ||
                      (reinterpret_cast<uintptr_t>(m.ptr) % (v * elem_size))))
          return false;
    }
    return true;
  };
  while (vec > 1 && !ok(vec)) vec >>= 1;
  return vec;
}

// chunking of the pixel axis for reductions: aim for >= ~1024 blocks.
void reduce_plan(const Geom& g, int vec, int& P, int& chunk, int& tpr, int& nzc) {
  if (g.cl) {
    tpr = std::min(g.C / vec, kThreads);
    if (tpr < 1) tpr = 1;
    nzc = ceil_div(g.C, (int64_t)tpr * vec);
    const int rpb = kThreads / tpr;
    const int target_blocks = 1024;
    int per_n = std::max(1, target_blocks / std::max(1, g.N * nzc));
    chunk = std::max(rpb * 4, ceil_div(g.HW, per_n));
    P = ceil_div(g.HW, chunk);
  } else {
    tpr = 0;
    nzc = g.C;
    const int target_blocks = 1024;
    int per_nc = std::max(1, target_blocks / std::max(1, g.N * g.C));
    chunk = std::max(kThreads * vec, ceil_div(g.HW, per_nc));
    chunk = ((chunk + vec - 1) / vec) * vec;
    P = ceil_div(g.HW, chunk);
  }
}

int apply_grid(int64_t total_vec) {
  int64_t blocks = (total_vec + kThreads - 1) / kThreads;
  return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 256 * 16));
}

}  // namespace

// Returns (count[G,C], mean[G,C], var[G,C], scale[G,C], shift[G,C]); scale/shift
// include the per-channel affine (weight/bias may be undefined).
// running_mean / running_var (fp32 [C], batch statistics only) are updated in place with
// factor `momentum`, num_batches (int64 [1]) incremented; the 6th output is rstd [G, C].
std::vector<at::Tensor> norm_stats(const at::Tensor& x, bool per_instance, double eps,
                                   const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, bool partial_only,
                                   const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var,
                                   const c10::optional<at::Tensor>& num_batches,
                                   double momentum) {
  IAMD_CHECK(x.is_cuda(), "norm_stats: x must be on the GPU");
  Geom g = geom_of(x);
  const int vec = pick_vec(g, x.element_size(), {});
  int P, chunk, tpr, nzc;
  reduce_plan(g, vec, P, chunk, tpr, nzc);
  auto fopt = x.options().dtype(at::kFloat);
  auto pcnt = at::empty({g.N, P, g.C}, fopt);
  auto pmean = at::empty({g.N, P, g.C}, fopt);
  auto pm2 = at::empty({g.N, P, g.C}, fopt);
  dim3 grid(P, g.N, g.cl ? nzc : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "norm_stats", [&] {
    const scalar_t* xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    auto launch = [&](auto vtag) {
      constexpr int V = decltype(vtag)::value;
      if (g.cl)
        hipLaunchKernelGGL((stats_partial_cl<scalar_t, V>), grid, dim3(kThreads), 0, stream(), xp,
                           g.C, g.HW, P, chunk, tpr, pcnt.data_ptr<float>(),
                           pmean.data_ptr<float>(), pm2.data_ptr<float>());
      else
        hipLaunchKernelGGL((stats_partial_nchw<scalar_t, V>), grid, dim3(kThreads), 0, stream(),
                           xp, g.C, g.HW, P, chunk, pcnt.data_ptr<float>(),
                           pmean.data_ptr<float>(), pm2.data_ptr<float>());
    };
    switch (vec) {
      case 8: launch(std::integral_constant<int, 8>()); break;
      case 4: launch(std::integral_constant<int, 4>()); break;
      case 2: launch(std::integral_constant<int, 2>()); break;
      default: launch(std::integral_constant<int, 1>()); break;
    }
  });
  IAMD_LAUNCH_CHECK();
  const int G = per_instance ? g.N : 1;
  // count / mean / var as rows of ONE [3, G, C] buffer: sync-BN hands it to its all-gather
  // as is (ops/norm.py _stats_rows), no stack copy
  auto stats3 = at::empty({3, G, g.C}, fopt);
  auto cnt = stats3[0], mean = stats3[1], var = stats3[2];
  at::Tensor scale, shift;
  auto rstd = at::empty({G, g.C}, fopt);
  if (!partial_only) {
    scale = at::empty({G, g.C}, fopt);
    shift = at::empty({G, g.C}, fopt);
  }
  float* rmp = nullptr;
  float* rvp = nullptr;
  int64_t* nbp = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    IAMD_CHECK(!per_instance && running_var.has_value() && running_var->defined() &&
                   running_mean->scalar_type() == at::kFloat &&
                   running_var->scalar_type() == at::kFloat && running_mean->is_contiguous() &&
                   running_var->is_contiguous() && running_mean->numel() == g.C &&
                   running_var->numel() == g.C,
               "norm_stats: running statistics must be contiguous fp32 [C] (batch norm)");
    rmp = running_mean->data_ptr<float>();
    rvp = running_var->data_ptr<float>();
  }
  if (num_batches.has_value() && num_batches->defined()) {
    IAMD_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
               "norm_stats: num_batches must be one int64");
    nbp = num_batches->data_ptr<int64_t>();
  }
  const float* wp = nullptr;
  const float* bp = nullptr;
  at::Tensor wf, bf;
  if (weight.has_value() && weight->defined()) { wf = weight->contiguous().to(at::kFloat); wp = wf.data_ptr<float>(); }
  if (bias.has_value() && bias->defined()) { bf = bias->contiguous().to(at::kFloat); bp = bf.data_ptr<float>(); }
  // two-stage merge: RS row-splits per group keep many CUs busy on the N*P partial rows
  const int rows = (per_instance ? 1 : g.N) * P;
  const int RS = std::max(1, std::min(32, rows / 16));
  const float* mc = pcnt.data_ptr<float>();
  const float* mm = pmean.data_ptr<float>();
  const float* m2p = pm2.data_ptr<float>();
  int fN = g.N, fP = P;
  at::Tensor tc, tmn, tm2;
  if (RS > 1) {
    tc = at::empty({G, RS, g.C}, fopt);
    tmn = at::empty({G, RS, g.C}, fopt);
    tm2 = at::empty({G, RS, g.C}, fopt);
    hipLaunchKernelGGL(stats_merge_rows, dim3(ceil_div(g.C, 64), G, RS), dim3(64, kFinRows), 0,
                       stream(), mc, mm, m2p, g.N, P, g.C, per_instance ? 1 : 0, RS,
                       tc.data_ptr<float>(), tmn.data_ptr<float>(), tm2.data_ptr<float>());
    mc = tc.data_ptr<float>();
    mm = tmn.data_ptr<float>();
    m2p = tm2.data_ptr<float>();
    fN = G;
    fP = RS;
  }
  hipLaunchKernelGGL(stats_finalize, dim3(ceil_div(g.C, 64), G), dim3(64, kFinRows), 0,
                     stream(), mc, mm, m2p, fN, fP, g.C, (per_instance || RS > 1) ? 1 : 0,
                     (float)eps, wp, bp, cnt.data_ptr<float>(), mean.data_ptr<float>(),
                     var.data_ptr<float>(), partial_only ? nullptr : scale.data_ptr<float>(),
                     partial_only ? nullptr : shift.data_ptr<float>(), rstd.data_ptr<float>(),
                     rmp, rvp, nbp, (float)momentum);
  IAMD_LAUNCH_CHECK();
  return {cnt, mean, var, scale, shift, rstd};
}

// Sync-BN merge of the gathered [W, 3, C] (count, mean, var) rows: returns (count, mean, var,
// rstd, scale, shift), each [1, C] fp32; running_mean / running_var (fp32 [C]) and num_batches
// (int64 [1]) are updated in place when given.
std::vector<at::Tensor> sync_stats_merge(const at::Tensor& allst, double eps,
                                         const c10::optional<at::Tensor>& weight,
                                         const c10::optional<at::Tensor>& bias,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         const c10::optional<at::Tensor>& num_batches,
                                         double momentum) {
  IAMD_CHECK(allst.is_cuda() && allst.scalar_type() == at::kFloat && allst.dim() == 3 &&
                 allst.size(1) == 3 && allst.is_contiguous(),
             "sync_stats_merge: contiguous fp32 [W, 3, C] rows expected");
  const int W = (int)allst.size(0), C = (int)allst.size(2);
  auto fopt = allst.options();
  auto cnt = at::empty({1, C}, fopt), mean = at::empty({1, C}, fopt), var = at::empty({1, C}, fopt);
  auto rstd = at::empty({1, C}, fopt), scale = at::empty({1, C}, fopt),
       shift = at::empty({1, C}, fopt);
  at::Tensor wf, bf;
  if (weight.has_value() && weight->defined()) wf = weight->contiguous().to(at::kFloat);
  if (bias.has_value() && bias->defined()) bf = bias->contiguous().to(at::kFloat);
  float *rmp = nullptr, *rvp = nullptr;
  int64_t* nbp = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    IAMD_CHECK(running_var.has_value() && running_var->defined() &&
                   running_mean->scalar_type() == at::kFloat &&
                   running_var->scalar_type() == at::kFloat && running_mean->is_contiguous() &&
                   running_var->is_contiguous() && running_mean->numel() == C &&
                   running_var->numel() == C,
               "sync_stats_merge: fp32 contiguous running statistics expected");
    rmp = running_mean->data_ptr<float>();
    rvp = running_var->data_ptr<float>();
  }
  if (num_batches.has_value() && num_batches->defined()) {
    IAMD_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1,
               "sync_stats_merge: int64 batch counter expected");
    nbp = num_batches->data_ptr<int64_t>();
  }
  hipLaunchKernelGGL(sync_stats_merge_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, stream(),
                     allst.data_ptr<float>(), W, C, (float)eps,
                     wf.defined() ? wf.data_ptr<float>() : nullptr,
                     bf.defined() ? bf.data_ptr<float>() : nullptr, cnt.data_ptr<float>(),
                     mean.data_ptr<float>(), var.data_ptr<float>(), rstd.data_ptr<float>(),
                     scale.data_ptr<float>(), shift.data_ptr<float>(), rmp, rvp, nbp,
                     (float)momentum);
  IAMD_LAUNCH_CHECK();
  return {cnt, mean, var, rstd, scale, shift};
}

// (k1, k2, k3, dweight, dbias) of the k1 backward from the per-sample sums (see kernel)
std::vector<at::Tensor> norm_bwd_coeffs(const at::Tensor& S1, const at::Tensor& S2,
                                        const at::Tensor& rstd,
                                        const c10::optional<at::Tensor>& weight,
                                        bool per_instance, double invM, bool need_dw,
                                        bool need_db) {
  IAMD_CHECK(S1.dim() == 2 && S1.sizes() == S2.sizes() && S1.scalar_type() == at::kFloat &&
                 S2.scalar_type() == at::kFloat && S1.is_contiguous() && S2.is_contiguous() &&
                 rstd.scalar_type() == at::kFloat && rstd.is_contiguous(),
             "norm_bwd_coeffs: fp32 contiguous [N, C] sums and rstd expected");
  const int N = (int)S1.size(0), C = (int)S1.size(1);
  IAMD_CHECK(rstd.numel() == (per_instance ? (int64_t)N * C : (int64_t)C),
             "norm_bwd_coeffs: rstd shape");
  auto fopt = S1.options();
  const int64_t R = per_instance ? N : 1;
  auto k1 = at::empty({R, C}, fopt), k2 = at::empty({R, C}, fopt), k3 = at::empty({R, C}, fopt);
  at::Tensor wf, dw, db;
  if (weight.has_value() && weight->defined()) wf = weight->contiguous().to(at::kFloat);
  if (need_dw) dw = at::empty({C}, fopt);
  if (need_db) db = at::empty({C}, fopt);
  hipLaunchKernelGGL(norm_bwd_coeffs_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, stream(),
                     S1.data_ptr<float>(), S2.data_ptr<float>(), rstd.data_ptr<float>(),
                     wf.defined() ? wf.data_ptr<float>() : nullptr, N, C, per_instance ? 1 : 0,
                     (float)invM, k1.data_ptr<float>(), k2.data_ptr<float>(), k3.data_ptr<float>(),
                     need_dw ? dw.data_ptr<float>() : nullptr,
                     need_db ? db.data_ptr<float>() : nullptr);
  IAMD_LAUNCH_CHECK();
  return {k1, k2, k3, dw, db};
}

at::Tensor norm_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                      const c10::optional<at::Tensor>& gamma,
                      const c10::optional<at::Tensor>& beta, double slope) {
  Geom g = geom_of(x);
  IAMD_CHECK(scale.is_contiguous() && shift.is_contiguous() && scale.scalar_type() == at::kFloat,
             "scale/shift must be contiguous fp32");
  const int per_n = scale.size(0) == g.N && g.N > 1 ? 1 : 0;
  ModView gm = view_of(gamma, g), bt = view_of(beta, g);
  const bool mod = gm.ptr != nullptr;
  IAMD_CHECK(mod == (bt.ptr != nullptr), "gamma and beta must be given together");
  if (mod) IAMD_CHECK(gamma->scalar_type() == x.scalar_type() && beta->scalar_type() == x.scalar_type(),
                      "gamma/beta dtype must match x");
  auto out = at::empty_like(x);
  const int vec = pick_vec(g, x.element_size(), {gm, bt});
  const int64_t total_vec = (int64_t)g.N * g.C * g.HW / vec;
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "norm_apply", [&] {
    const scalar_t* xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    scalar_t* op = reinterpret_cast<scalar_t*>(out.data_ptr());
    auto launch = [&](auto vtag, auto cltag, auto modtag) {
      constexpr int V = decltype(vtag)::value;
      constexpr bool CLv = decltype(cltag)::value;
      constexpr bool M = decltype(modtag)::value;
      hipLaunchKernelGGL((apply_fwd<scalar_t, CLv, V, M>), dim3(apply_grid(total_vec)),
                         dim3(kThreads), 0, stream(), xp, op, g.N, g.C, g.HW,
                         scale.data_ptr<float>(), shift.data_ptr<float>(), per_n, gm, bt,
                         (float)slope);
    };
    auto by_mod = [&](auto vtag, auto cltag) {
      if (mod) launch(vtag, cltag, std::true_type());
      else launch(vtag, cltag, std::false_type());
    };
    auto by_cl = [&](auto vtag) {
      if (g.cl) by_mod(vtag, std::true_type());
      else by_mod(vtag, std::false_type());
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

// Backward reduce: returns (S1[N,C], S2[N,C]) and fills dgamma/dbeta (if given).
std::vector<at::Tensor> norm_bwd_reduce(const at::Tensor& x, const at::Tensor& dout,
                                        const at::Tensor& scale, const at::Tensor& shift,
                                        const at::Tensor& mean, const at::Tensor& rstd,
                                        const c10::optional<at::Tensor>& gamma,
                                        const c10::optional<at::Tensor>& beta,
                                        const c10::optional<at::Tensor>& dgamma,
                                        const c10::optional<at::Tensor>& dbeta, double slope) {
  Geom g = geom_of(x);
  Geom gd = geom_of(dout);
  IAMD_CHECK(gd.cl == g.cl || g.HW == 1, "dout layout must match x");
  const int per_n_aff = scale.size(0) == g.N && g.N > 1 ? 1 : 0;
  const int per_n_stat = mean.size(0) == g.N && g.N > 1 ? 1 : 0;
  ModView gm = view_of(gamma, g), bt = view_of(beta, g), dgm = view_of(dgamma, g),
          dbt = view_of(dbeta, g);
  const bool mod = gm.ptr != nullptr;
  // broadcast modulation (per-(n,c) gamma/beta): pixel stride 0
  const bool bcast = mod && gm.sp == 0 && bt.sp == 0 && g.HW > 1;
  IAMD_CHECK(!mod || bcast || (dgm.ptr != nullptr && dbt.ptr != nullptr),
             "norm_bwd_reduce: spatial modulation needs dgamma/dbeta outputs (gamma strides n/c/p=",
             gm.sn, "/", gm.sc, "/", gm.sp, " beta p=", bt.sp, " HW=", g.HW, " dg=",
             dgm.ptr != nullptr, " db=", dbt.ptr != nullptr, ")");
  const int vec = pick_vec(g, x.element_size(), {gm, bt, dgm, dbt});
  int P, chunk, tpr, nzc;
  reduce_plan(g, vec, P, chunk, tpr, nzc);
  auto fopt = x.options().dtype(at::kFloat);
  const int Q = bcast ? 4 : 2;
  auto ps = at::empty({Q, g.N, P, g.C}, fopt);
  const int64_t qs = (int64_t)g.N * P * g.C;
  float* ps1 = ps.data_ptr<float>();
  float* ps2 = ps1 + qs;
  float* ps3 = bcast ? ps1 + 2 * qs : nullptr;
  float* ps4 = bcast ? ps1 + 3 * qs : nullptr;
  dim3 grid(P, g.N, g.cl ? nzc : g.C);
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "norm_bwd_reduce", [&] {
    const scalar_t* xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    const scalar_t* dp = reinterpret_cast<const scalar_t*>(dout.data_ptr());
    auto launch = [&](auto vtag, auto cltag, auto modtag, auto bctag) {
      constexpr int V = decltype(vtag)::value;
      constexpr bool CLv = decltype(cltag)::value;
      constexpr bool M = decltype(modtag)::value;
      constexpr bool B = decltype(bctag)::value;
      hipLaunchKernelGGL((bwd_reduce<scalar_t, CLv, V, M, B>), grid, dim3(kThreads), 0, stream(),
                         xp, dp, g.N, g.C, g.HW, P, chunk, tpr, scale.data_ptr<float>(),
                         shift.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                         per_n_aff, per_n_stat, gm, bt, dgm, dbt, (float)slope, ps1, ps2, ps3,
                         ps4);
    };
    auto by_mod = [&](auto vtag, auto cltag) {
      if (bcast) launch(vtag, cltag, std::true_type(), std::true_type());
      else if (mod) launch(vtag, cltag, std::true_type(), std::false_type());
      else launch(vtag, cltag, std::false_type(), std::false_type());
    };
    auto by_cl = [&](auto vtag) {
      if (g.cl) by_mod(vtag, std::true_type());
      else by_mod(vtag, std::false_type());
    };
    switch (vec) {
      case 8: by_cl(std::integral_constant<int, 8>()); break;
      case 4: by_cl(std::integral_constant<int, 4>()); break;
      case 2: by_cl(std::integral_constant<int, 2>()); break;
      default: by_cl(std::integral_constant<int, 1>()); break;
    }
  });
  IAMD_LAUNCH_CHECK();
  // atomics across row-splits reorder fp32 sums: single split in deterministic mode
  const int RSs = at::globalContext().deterministicAlgorithms()
                      ? 1 : std::max(1, std::min(16, P / 16));
  auto sums = RSs > 1 ? at::zeros({Q, g.N, g.C}, fopt) : at::empty({Q, g.N, g.C}, fopt);
  hipLaunchKernelGGL(sum_partials, dim3(ceil_div(g.C, 64), g.N, Q * RSs), dim3(64, kFinRows), 0,
                     stream(), ps1, Q, qs, g.N, P, g.C, RSs, sums.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  // (S1, S2[, S3 = dgamma, S4 = dbeta for broadcast modulation]), each [N, C]
  std::vector<at::Tensor> out;
  for (int q = 0; q < Q; ++q) out.push_back(sums[q]);
  return out;
}

at::Tensor norm_bwd_apply(const at::Tensor& x, const at::Tensor& dout, const at::Tensor& scale,
                          const at::Tensor& shift, const at::Tensor& mean, const at::Tensor& rstd,
                          const at::Tensor& k1, const at::Tensor& k2, const at::Tensor& k3,
                          const c10::optional<at::Tensor>& gamma,
                          const c10::optional<at::Tensor>& beta, double slope) {
  Geom g = geom_of(x);
  const int per_n_aff = scale.size(0) == g.N && g.N > 1 ? 1 : 0;
  const int per_n_stat = mean.size(0) == g.N && g.N > 1 ? 1 : 0;
  IAMD_CHECK(k1.size(0) == mean.size(0), "k coefficients must match stat groups");
  ModView gm = view_of(gamma, g), bt = view_of(beta, g);
  const bool mod = gm.ptr != nullptr;
  auto dx = at::empty_like(x);
  const int vec = pick_vec(g, x.element_size(), {gm, bt});
  const int64_t total_vec = (int64_t)g.N * g.C * g.HW / vec;
  IAMD_DISPATCH_FLOAT_TYPES(x.scalar_type(), "norm_bwd_apply", [&] {
    const scalar_t* xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    const scalar_t* dp = reinterpret_cast<const scalar_t*>(dout.data_ptr());
    scalar_t* op = reinterpret_cast<scalar_t*>(dx.data_ptr());
    auto launch = [&](auto vtag, auto cltag, auto modtag) {
      constexpr int V = decltype(vtag)::value;
      constexpr bool CLv = decltype(cltag)::value;
      constexpr bool M = decltype(modtag)::value;
      hipLaunchKernelGGL((bwd_apply<scalar_t, CLv, V, M>), dim3(apply_grid(total_vec)),
                         dim3(kThreads), 0, stream(), xp, dp, op, g.N, g.C, g.HW,
                         scale.data_ptr<float>(), shift.data_ptr<float>(), per_n_aff,
                         mean.data_ptr<float>(), rstd.data_ptr<float>(), k1.data_ptr<float>(),
                         k2.data_ptr<float>(), k3.data_ptr<float>(), per_n_stat, gm, bt,
                         (float)slope);
    };
    auto by_mod = [&](auto vtag, auto cltag) {
      if (mod) launch(vtag, cltag, std::true_type());
      else launch(vtag, cltag, std::false_type());
    };
    auto by_cl = [&](auto vtag) {
      if (g.cl) by_mod(vtag, std::true_type());
      else by_mod(vtag, std::false_type());
    };
    switch (vec) {
      case 8: by_cl(std::integral_constant<int, 8>()); break;
      case 4: by_cl(std::integral_constant<int, 4>()); break;
      case 2: by_cl(std::integral_constant<int, 2>()); break;
      default: by_cl(std::integral_constant<int, 1>()); break;
    }
  });
  IAMD_LAUNCH_CHECK();
  return dx;
}

}  // namespace iamd
