// k5b: batched spectral-norm power iteration for every SN layer of a network.
//
// PyTorch's spectral_norm runs, per layer and per forward, two GEMVs + two
// normalisations + a dot (plus a weight reshape copy for channels-last
// convs) — ~10 tiny launches per layer, ~4000 per SPADE forward, and under
// autocast the GEMVs go through bf16 hipBLASLt with a host-side heuristic
// query each call. Here ONE set of 4 launches covers all L layers, in fp32:
//
//   K1 colsum : t_l  = W_l^T u_l                 (column-parallel, coalesced; one fp32 partial
//               slab per 64-row split, summed in split order by K1b tsum — no float
//               atomics, so the iteration is bitwise reproducible run to run)
//   K2 tnorm  : |t_l|^2                           (one block per layer)
//   K3 rows   : s_l  = W_l (t_l / max(|t_l|,eps)) (one wave per row)
//   K4 final  : u_l <- s_l / max(|s_l|,eps), v_l <- t_l / max(|t_l|,eps),
//               sigma_l = u_l . s_l               (one block per layer)
//
// With update=false (eval) K1/K2 are skipped and K3 uses v_l directly:
// sigma_l = u_l . (W_l v_l), u/v untouched — exactly torch's semantics.
// Weights may be channels-last: memory column (kh,kw,ci) maps to logical
// column (ci,kh,kw) so u/v keep the reference (logical) order.
#include "common.h"

#include <mutex>
#include <unordered_map>

namespace iamd {
namespace {

constexpr int kT = 256;
constexpr int kColTile = 4 * kT;  // columns per K1 block (4 per thread)
constexpr int kRowsPerSplit = 64; // rows per K1 block
constexpr int kRowsPerBlock = 4;  // rows (waves) per K3 block

struct SnEntry {
  const float* W;
  const __hip_bfloat16* Wb;  // bf16 copy of W (the optimizer's shadow): read instead when set
  float* u;
  float* v;
  float* t;  // workspace [w]
  float* s;  // workspace [h]
  float* tp; // workspace [nsplit][w]: K1 partials per row split
  int64_t nsplit;
  int64_t h, w;
  int64_t cl_cin, cl_khw;  // channels-last mapping (0 = none)
  int64_t vec;             // w % 4 == 0 and W 16-byte aligned: 16-B row loads
};

// memory column -> logical column (32-bit: every SN weight row is < 2^31 elements).
// Only the u/v state vectors are kept in logical (reference checkpoint) order; the per-call
// workspaces t/s stay in memory order so the hot GEMV loops never divide.
__device__ __forceinline__ int64_t logical_col(const SnEntry& e, int64_t c) {
  if (!e.cl_cin) return c;
  const uint32_t cc = (uint32_t)c, cin = (uint32_t)e.cl_cin;
  const uint32_t q = cc / cin;
  return (int64_t)(cc - q * cin) * e.cl_khw + q;
}

__device__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < kT / 64; ++k) s += sh[k];
  __syncthreads();
  if (threadIdx.x == 0) sh[0] = s;
  __syncthreads();
  s = sh[0];
  __syncthreads();
  return s;
}

// blocks: {layer, col_tile, row_split}. Each thread owns 4 adjacent columns (16-B loads when
// the row length is a multiple of 4) and keeps 8 rows of loads in flight: the plain
// one-column-per-thread walk ran at ~1.5 TB/s (profiles/spade_step_latest_mi355x.txt).
__global__ void __launch_bounds__(kT) sn_colsum(const SnEntry* __restrict__ ents,
                                                 const int* __restrict__ blocks) {
  const int* bm = blocks + 3 * blockIdx.x;
  const SnEntry e = ents[bm[0]];
  const int64_t c = (int64_t)bm[1] * kColTile + threadIdx.x * 4;
  if (c >= e.w) return;
  const int64_t r0 = (int64_t)bm[2] * kRowsPerSplit;
  const int64_t r1 = min(e.h, r0 + kRowsPerSplit);
  const bool vec = e.vec;  // then c + 3 < w as well
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (e.Wb && vec) {
    // bf16 shadow rows: 8-byte loads, so 16 rows in flight per thread (8 left the pass
    // latency-bound at ~1.6 TB/s)
    for (int64_t r = r0; r < r1; r += 16) {
      float wv[16][4], uv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t rr = r + i;
        const bool ok = rr < r1;
        uv[i] = ok ? e.u[rr] : 0.f;
        load_vec<__hip_bfloat16, 4>(e.Wb + (ok ? rr : r0) * e.w + c, wv[i]);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = fmaf(wv[i][k], uv[i], acc[k]);
    }
    *reinterpret_cast<float4*>(e.tp + bm[2] * e.w + c) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    return;
  }
  for (int64_t r = r0; r < r1; r += 8) {
    float wv[8][4], uv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t rr = r + i;
      const bool ok = rr < r1;
      uv[i] = ok ? e.u[rr] : 0.f;
      const int64_t off = (ok ? rr : r0) * e.w + c;
      if (e.Wb) {
        if (vec) {
          load_vec<__hip_bfloat16, 4>(e.Wb + off, wv[i]);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) wv[i][k] = c + k < e.w ? __bfloat162float(e.Wb[off + k]) : 0.f;
        }
      } else {
        const float* src = e.W + off;
        if (vec) {
          const float4 v4 = *reinterpret_cast<const float4*>(src);
          wv[i][0] = v4.x; wv[i][1] = v4.y; wv[i][2] = v4.z; wv[i][3] = v4.w;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) wv[i][k] = c + k < e.w ? src[k] : 0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = fmaf(wv[i][k], uv[i], acc[k]);
  }
  float* o = e.tp + bm[2] * e.w + c;  // memory order, this row split's slab
  if (vec) {
    *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < e.w) o[k] = acc[k];
  }
}

// blocks: {layer, col_tile}: t[c] = sum over row splits of the K1 slabs, in split order
__global__ void __launch_bounds__(kT) sn_tsum(const SnEntry* __restrict__ ents,
                                               const int* __restrict__ blocks) {
  const int* bm = blocks + 2 * blockIdx.x;
  const SnEntry e = ents[bm[0]];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t c = (int64_t)bm[1] * kColTile + q * kT + threadIdx.x;
    if (c >= e.w) return;
    float acc = 0.f;
    for (int64_t k = 0; k < e.nsplit; ++k) acc += e.tp[k * e.w + c];
    e.t[c] = acc;
  }
}

// one block per layer: sums of squares of t -> scal[l*4 + 0]
__global__ void __launch_bounds__(kT) sn_tnorm(const SnEntry* __restrict__ ents,
                                                float* __restrict__ scal) {
  __shared__ float sh[kT / 64];
  const SnEntry e = ents[blockIdx.x];
  float acc = 0.f;
  for (int64_t c = threadIdx.x; c < e.w; c += kT) acc = fmaf(e.t[c], e.t[c], acc);
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) scal[4 * blockIdx.x] = acc;
}

// blocks: {layer, first_row}; one wave per row. Input vector: t/|t| (update) or v.
__global__ void __launch_bounds__(64 * kRowsPerBlock) sn_rows(const SnEntry* __restrict__ ents,
                                                               const int* __restrict__ blocks,
                                                               const float* __restrict__ scal,
                                                               int update, float eps) {
  const int* bm = blocks + 2 * blockIdx.x;
  const SnEntry e = ents[bm[0]];
  const int64_t r = (int64_t)bm[1] + (threadIdx.x >> 6);
  if (r >= e.h) return;
  const int lane = threadIdx.x & 63;
  const float k = update ? 1.f / fmaxf(sqrtf(scal[4 * bm[0]]), eps) : 1.f;
  const float* row = e.W + r * e.w;
  float acc = 0.f;
  if (update && e.Wb) {  // bf16 copy of W: 8 elements per lane and trip
    const __hip_bfloat16* rb = e.Wb + r * e.w;
    const float* x = e.t;
    if (e.vec && e.w % 8 == 0) {
      // two 16-byte row loads per lane and trip in flight
      for (int64_t c = lane * 8; c < e.w; c += 64 * 16) {
        const int64_t c2 = c + 64 * 8;
        const bool two = c2 < e.w;
        float a[2][8], b[2][8];
        load_vec<__hip_bfloat16, 8>(rb + c, a[0]);
        load_vec<float, 4>(x + c, *reinterpret_cast<float(*)[4]>(b[0]));
        load_vec<float, 4>(x + c + 4, *reinterpret_cast<float(*)[4]>(b[0] + 4));
        if (two) {
          load_vec<__hip_bfloat16, 8>(rb + c2, a[1]);
          load_vec<float, 4>(x + c2, *reinterpret_cast<float(*)[4]>(b[1]));
          load_vec<float, 4>(x + c2 + 4, *reinterpret_cast<float(*)[4]>(b[1] + 4));
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) a[1][k] = b[1][k] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = fmaf(a[0][k], b[0][k], acc);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = fmaf(a[1][k], b[1][k], acc);
      }
    } else {
      for (int64_t c = lane; c < e.w; c += 64) acc = fmaf(__bfloat162float(rb[c]), x[c], acc);
    }
  } else if (update) {  // t is in memory order: straight dot, 16-B loads, 4 per lane in flight
    const float* x = e.t;
    if (e.vec) {
      const float4* r4 = reinterpret_cast<const float4*>(row);
      const float4* x4 = reinterpret_cast<const float4*>(x);
      const int64_t w4 = e.w / 4;
      for (int64_t c = lane; c < w4; c += 4 * 64) {
        float4 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = c + i * 64 < w4;
          a[i] = ok ? r4[c + i * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
          b[i] = ok ? x4[c + i * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc = fmaf(a[i].x, b[i].x, fmaf(a[i].y, b[i].y, fmaf(a[i].z, b[i].z,
                                                               fmaf(a[i].w, b[i].w, acc))));
      }
    } else {
      for (int64_t c = lane; c < e.w; c += 64) acc = fmaf(row[c], x[c], acc);
    }
  } else if (e.Wb) {
    const __hip_bfloat16* rb = e.Wb + r * e.w;
    for (int64_t c = lane; c < e.w; c += 64)
      acc = fmaf(__bfloat162float(rb[c]), e.v[logical_col(e, c)], acc);
  } else {
    for (int64_t c = lane; c < e.w; c += 64) acc = fmaf(row[c], e.v[logical_col(e, c)], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) e.s[r] = acc * k;
}

// one block per layer: finalize u, v, sigma
__global__ void __launch_bounds__(kT) sn_final(const SnEntry* __restrict__ ents,
                                                float* __restrict__ scal,
                                                float* __restrict__ sigma, int update,
                                                float eps) {
  __shared__ float sh[kT / 64];
  const SnEntry e = ents[blockIdx.x];
  if (update) {
    float acc = 0.f;
    for (int64_t r = threadIdx.x; r < e.h; r += kT) acc = fmaf(e.s[r], e.s[r], acc);
    const float ss = block_sum(acc, sh);
    const float inv_s = 1.f / fmaxf(sqrtf(ss), eps);
    const float inv_t = 1.f / fmaxf(sqrtf(scal[4 * blockIdx.x]), eps);
    for (int64_t r = threadIdx.x; r < e.h; r += kT) e.u[r] = e.s[r] * inv_s;
    for (int64_t c = threadIdx.x; c < e.w; c += kT) e.v[logical_col(e, c)] = e.t[c] * inv_t;
    if (threadIdx.x == 0) {
      scal[4 * blockIdx.x + 1] = ss;
      sigma[blockIdx.x] = ss * inv_s;  // u . s = |s|^2 / max(|s|, eps)
    }
  } else {
    float acc = 0.f;
    for (int64_t r = threadIdx.x; r < e.h; r += kT) acc = fmaf(e.u[r], e.s[r], acc);
    const float d = block_sum(acc, sh);
    if (threadIdx.x == 0) sigma[blockIdx.x] = d;
  }
}

struct SnPlan {
  at::Tensor ents;         // device SnEntry[L]
  at::Tensor col_blocks;   // device int3
  at::Tensor sum_blocks;   // device int2
  at::Tensor row_blocks;   // device int2
  at::Tensor t_ws, s_ws, tp_ws;   // fp32 workspaces (flat)
  int n_col_blocks, n_sum_blocks, n_row_blocks, L;
};

std::mutex g_sn_mu;
std::unordered_map<uint64_t, SnPlan> g_sn_cache;

void keep_plan(const SnPlan& p) {
  for (const at::Tensor* t : {&p.ents, &p.col_blocks, &p.sum_blocks, &p.row_blocks, &p.t_ws,
                              &p.s_ws, &p.tp_ws})
    keep_for_graph(*t);
}

SnPlan& get_plan(const std::vector<at::Tensor>& W, const std::vector<at::Tensor>& U,
                 const std::vector<at::Tensor>& V, const std::vector<at::Tensor>& WB) {
  uint64_t hsh = 0x51ed270b0b6e3a6dULL;
  for (size_t i = 0; i < WB.size(); ++i)
    hsh ^= reinterpret_cast<uint64_t>(WB[i].data_ptr()) * 0x2545F4914F6CDD1DULL + (hsh << 5);
  for (size_t i = 0; i < W.size(); ++i) {
    hsh ^= reinterpret_cast<uint64_t>(W[i].data_ptr()) + 0x9e3779b97f4a7c15ULL + (hsh << 6);
    hsh ^= reinterpret_cast<uint64_t>(U[i].data_ptr()) + (hsh >> 2);
    hsh ^= reinterpret_cast<uint64_t>(V[i].data_ptr()) * 31 + (uint64_t)W[i].numel();
    hsh ^= (uint64_t)W[i].size(0) * 0x100000001b3ULL + (uint64_t)W[i].is_contiguous() + (hsh << 3);
  }
  std::lock_guard<std::mutex> lk(g_sn_mu);
  auto it = g_sn_cache.find(hsh);
  if (it != g_sn_cache.end()) {
    keep_plan(it->second);
    return it->second;
  }
  const int L = (int)W.size();
  int64_t tot_w = 0, tot_h = 0, tot_p = 0;
  for (int i = 0; i < L; ++i) {
    tot_h += W[i].size(0);
    tot_w += (W[i].numel() / W[i].size(0) + 3) / 4 * 4;
    tot_p += ((W[i].size(0) + kRowsPerSplit - 1) / kRowsPerSplit * (W[i].numel() / W[i].size(0)) +
              3) / 4 * 4;
  }
  SnPlan p;
  auto fopt = W[0].options().dtype(at::kFloat);
  p.t_ws = at::zeros({tot_w}, fopt);
  p.s_ws = at::zeros({tot_h}, fopt);
  p.tp_ws = at::empty({tot_p}, fopt);
  std::vector<SnEntry> ents(L);
  std::vector<int32_t> cb, sb, rb;
  int64_t ow = 0, oh = 0, op = 0;
  for (int i = 0; i < L; ++i) {
    const at::Tensor& w = W[i];
    IAMD_CHECK(w.scalar_type() == at::kFloat && w.is_non_overlapping_and_dense(),
               "mt_sn_power: weights must be dense fp32");
    IAMD_CHECK(U[i].is_contiguous() && V[i].is_contiguous(), "mt_sn_power: u/v contiguous");
    SnEntry& e = ents[i];
    e.W = w.data_ptr<float>();
    e.Wb = nullptr;
    if (!WB.empty()) {
      IAMD_CHECK(WB[i].scalar_type() == at::kBFloat16 && WB[i].sizes() == w.sizes() &&
                     WB[i].strides() == w.strides() &&
                     (reinterpret_cast<uintptr_t>(WB[i].data_ptr()) & 15) == 0,
                 "mt_sn_power: a bf16 copy must be laid out like its weight, 16-B aligned");
      e.Wb = reinterpret_cast<const __hip_bfloat16*>(WB[i].data_ptr());
    }
    e.u = U[i].data_ptr<float>();
    e.v = V[i].data_ptr<float>();
    e.h = w.size(0);
    e.w = w.numel() / e.h;
    IAMD_CHECK(U[i].numel() == e.h && V[i].numel() == e.w, "mt_sn_power: u/v sizes");
    const bool cl = w.dim() == 4 && !w.is_contiguous() &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast);
    IAMD_CHECK(cl || w.is_contiguous(), "mt_sn_power: weight must be contiguous or CL");
    e.cl_cin = cl ? w.size(1) : 0;
    e.cl_khw = cl ? w.size(2) * w.size(3) : 0;
    e.t = p.t_ws.data_ptr<float>() + ow;
    // (workspace slices start at multiples of 4 floats: 16-B aligned)
    e.vec = (e.w % 4 == 0) && (reinterpret_cast<uintptr_t>(e.W) & 15) == 0;
    e.s = p.s_ws.data_ptr<float>() + oh;
    const int ntile = (int)((e.w + kColTile - 1) / kColTile);
    const int nsplit = (int)((e.h + kRowsPerSplit - 1) / kRowsPerSplit);
    e.tp = p.tp_ws.data_ptr<float>() + op;
    e.nsplit = nsplit;
    ow += (e.w + 3) / 4 * 4;
    oh += e.h;
    op += ((int64_t)nsplit * e.w + 3) / 4 * 4;
    for (int a = 0; a < ntile; ++a) {
      for (int b = 0; b < nsplit; ++b) {
        cb.push_back(i);
        cb.push_back(a);
        cb.push_back(b);
      }
      sb.push_back(i);
      sb.push_back(a);
    }
    for (int64_t r = 0; r < e.h; r += kRowsPerBlock) {
      rb.push_back(i);
      rb.push_back((int32_t)r);
    }
  }
  auto dev = W[0].device();
  auto stage = [&](const void* src, size_t bytes) { return stage_to_device(src, bytes, dev); };
  p.ents = stage(ents.data(), ents.size() * sizeof(SnEntry));
  p.col_blocks = stage(cb.data(), cb.size() * sizeof(int32_t)).view(at::kInt);
  p.sum_blocks = stage(sb.data(), sb.size() * sizeof(int32_t)).view(at::kInt);
  p.n_sum_blocks = (int)(sb.size() / 2);
  p.row_blocks = stage(rb.data(), rb.size() * sizeof(int32_t)).view(at::kInt);
  p.n_col_blocks = (int)(cb.size() / 3);
  p.n_row_blocks = (int)(rb.size() / 2);
  p.L = L;
  keep_plan(p);
  if (g_sn_cache.size() > 64) g_sn_cache.clear();
  return g_sn_cache.emplace(hsh, std::move(p)).first->second;
}

}  // namespace

// Returns sigma [L] (fp32). update=true runs one power iteration (u, v updated in place).
// shadows (optional, parallel to weights): bf16 copies of W (written by the optimizer step) that
// the GEMV passes read instead of the fp32 weights (half the bytes).
at::Tensor mt_sn_power(const std::vector<at::Tensor>& weights, const std::vector<at::Tensor>& us,
                       const std::vector<at::Tensor>& vs, bool update, double eps,
                       const std::vector<at::Tensor>& shadows) {
  IAMD_CHECK(!weights.empty() && weights.size() == us.size() && us.size() == vs.size(),
             "mt_sn_power: list sizes");
  IAMD_CHECK(shadows.empty() || shadows.size() == weights.size(), "mt_sn_power: shadow list size");
  SnPlan& p = get_plan(weights, us, vs, shadows);
  auto fopt = weights[0].options().dtype(at::kFloat);
  auto sigma = at::empty({p.L}, fopt);
  auto scal = at::empty({p.L, 4}, fopt);
  const auto* ents = reinterpret_cast<const SnEntry*>(p.ents.data_ptr());
  hipStream_t st = stream();
  if (update) {
    hipLaunchKernelGGL(sn_colsum, dim3(p.n_col_blocks), dim3(kT), 0, st, ents,
                       p.col_blocks.data_ptr<int>());
    hipLaunchKernelGGL(sn_tsum, dim3(p.n_sum_blocks), dim3(kT), 0, st, ents,
                       p.sum_blocks.data_ptr<int>());
    hipLaunchKernelGGL(sn_tnorm, dim3(p.L), dim3(kT), 0, st, ents, scal.data_ptr<float>());
  }
  hipLaunchKernelGGL(sn_rows, dim3(p.n_row_blocks), dim3(64 * kRowsPerBlock), 0, st, ents,
                     p.row_blocks.data_ptr<int>(), scal.data_ptr<float>(), update ? 1 : 0,
                     (float)eps);
  hipLaunchKernelGGL(sn_final, dim3(p.L), dim3(kT), 0, st, ents, scal.data_ptr<float>(),
                     sigma.data_ptr<float>(), update ? 1 : 0, (float)eps);
  IAMD_LAUNCH_CHECK();
  return sigma;
}

}  // namespace iamd

// ---------------------------------------------------------------------------
// k5c: W_l / sigma_l for every SN layer, written straight into ONE flat bf16
// buffer (the autocast compute dtype). Replaces a per-layer fp32 divide plus
// autocast's per-layer fp32->bf16 cast (two launches and two fp32 passes per
// layer per forward) with one launch. Layer l's output is a view at offset
// off_l with W_l's strides (channels-last stays channels-last).
// ---------------------------------------------------------------------------
namespace iamd {
namespace {

constexpr int kScChunk = 256 * 8 * 8;

struct ScEntry {
  const float* W;
  const __hip_bfloat16* Wb;  // read this bf16 copy of W instead (shadow), or
  __hip_bfloat16* Ws;        // write bf16(W) here too (refresh the shadow)
  int64_t numel;
  int64_t off;
  int64_t vec;  // W 16-byte aligned: vector path
};

__global__ void __launch_bounds__(kT) sn_scale_cast(const ScEntry* __restrict__ ents,
                                                     const int* __restrict__ blocks,
                                                     const float* __restrict__ sigma,
                                                     __hip_bfloat16* __restrict__ out) {
  const int t = blocks[2 * blockIdx.x], chunk = blocks[2 * blockIdx.x + 1];
  const ScEntry e = ents[t];
  const float inv = 1.f / sigma[t];
  const int64_t start = (int64_t)chunk * kScChunk;
  const int64_t end = min(e.numel, start + (int64_t)kScChunk);
  __hip_bfloat16* o = out + e.off;  // 16-B aligned (offsets are multiples of 8 elements)
  auto wat = [&](int64_t i) { return e.Wb ? __bfloat162float(e.Wb[i]) : e.W[i]; };
  if (e.vec && e.Wb) {  // shadow reads: 4 x 16-B loads per lane in flight, then the stores
    const int64_t vend = start + ((end - start) & ~(int64_t)7);
    for (int64_t i0 = start + threadIdx.x * 8; i0 < vend; i0 += kT * 8 * 4) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + (int64_t)u * kT * 8;
        if (i < vend) load_vec<__hip_bfloat16, 8>(e.Wb + i, v[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + (int64_t)u * kT * 8;
        if (i >= vend) continue;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[u][k] *= inv;
        store_vec<__hip_bfloat16, 8>(o + i, v[u]);
      }
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += kT) o[i] = __float2bfloat16(wat(i) * inv);
  } else if (e.vec) {  // 8 elements per lane per trip: two 16-B fp32 loads, 16-B stores
    const int64_t vend = start + ((end - start) & ~(int64_t)7);
    for (int64_t i = start + threadIdx.x * 8; i < vend; i += kT * 8) {
      float v[8];
      if (e.Wb) {
        load_vec<__hip_bfloat16, 8>(e.Wb + i, v);
      } else {
        load_vec<float, 4>(e.W + i, *reinterpret_cast<float(*)[4]>(v));
        load_vec<float, 4>(e.W + i + 4, *reinterpret_cast<float(*)[4]>(v + 4));
        if (e.Ws) store_vec<__hip_bfloat16, 8>(e.Ws + i, v);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= inv;
      store_vec<__hip_bfloat16, 8>(o + i, v);
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += kT) {
      const float w = wat(i);
      if (e.Ws) e.Ws[i] = __float2bfloat16(w);
      o[i] = __float2bfloat16(w * inv);
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += kT) {
      const float w = wat(i);
      if (e.Ws) e.Ws[i] = __float2bfloat16(w);
      o[i] = __float2bfloat16(w * inv);
    }
  }
}

struct ScPlan {
  at::Tensor ents, blocks;
  int nblocks;
  int64_t total;
  std::vector<int64_t> offs;
};
std::mutex g_sc_mu;
std::unordered_map<uint64_t, ScPlan> g_sc_cache;

// mode 0: read fp32 W; 1: read the bf16 shadows; 2: read fp32 W and write the shadows too
ScPlan& get_sc_plan(const std::vector<at::Tensor>& W, const std::vector<at::Tensor>& S, int mode) {
  uint64_t h = 0x2545F4914F6CDD1DULL ^ (uint64_t)(mode * 0x9E3779B1);
  for (auto& w : W) h ^= reinterpret_cast<uint64_t>(w.data_ptr()) + 0x9e3779b97f4a7c15ULL +
                        (h << 6) + (h >> 2) + (uint64_t)w.numel();
  for (auto& t : S) h ^= reinterpret_cast<uint64_t>(t.data_ptr()) * 0x100000001b3ULL + (h << 7);
  std::lock_guard<std::mutex> lk(g_sc_mu);
  auto it = g_sc_cache.find(h);
  if (it != g_sc_cache.end()) {
    keep_for_graph(it->second.ents);
    keep_for_graph(it->second.blocks);
    return it->second;
  }
  ScPlan p;
  std::vector<ScEntry> ents;
  std::vector<int32_t> bm;
  int64_t off = 0;
  for (size_t i = 0; i < W.size(); ++i) {
    IAMD_CHECK(W[i].scalar_type() == at::kFloat && W[i].is_non_overlapping_and_dense(),
               "mt_sn_scale_cast: weights must be dense fp32");
    const __hip_bfloat16* wb = nullptr;
    __hip_bfloat16* ws = nullptr;
    if (mode) {
      IAMD_CHECK(S[i].scalar_type() == at::kBFloat16 && S[i].sizes() == W[i].sizes() &&
                     S[i].strides() == W[i].strides() &&
                     (reinterpret_cast<uintptr_t>(S[i].data_ptr()) & 15) == 0,
                 "mt_sn_scale_cast: a shadow must be laid out like its weight, 16-B aligned");
      if (mode == 1) wb = reinterpret_cast<const __hip_bfloat16*>(S[i].data_ptr());
      else ws = reinterpret_cast<__hip_bfloat16*>(S[i].data_ptr());
    }
    ents.push_back({W[i].data_ptr<float>(), wb, ws, W[i].numel(), off,
                    (int64_t)((reinterpret_cast<uintptr_t>(W[i].data_ptr()) & 15) == 0)});
    p.offs.push_back(off);
    const int64_t nch = (W[i].numel() + kScChunk - 1) / kScChunk;
    for (int64_t c = 0; c < nch; ++c) {
      bm.push_back((int32_t)i);
      bm.push_back((int32_t)c);
    }
    off += (W[i].numel() + 7) / 8 * 8;  // 16-byte aligned views
  }
  p.total = off;
  auto dev = W[0].device();
  p.ents = stage_to_device(ents.data(), ents.size() * sizeof(ScEntry), dev);
  p.blocks = stage_to_device(bm.data(), bm.size() * sizeof(int32_t), dev).view(at::kInt);
  p.nblocks = (int)(bm.size() / 2);
  if (g_sc_cache.size() > 64) g_sc_cache.clear();
  return g_sc_cache.emplace(h, std::move(p)).first->second;
}

}  // namespace

// shadows (optional): bf16 copies of the weights; shadow_mode 1 reads them instead of the fp32
// weights, 2 writes them (bf16(W)) in the same pass.
std::vector<at::Tensor> mt_sn_scale_cast(const std::vector<at::Tensor>& weights,
                                         const at::Tensor& sigma,
                                         const std::vector<at::Tensor>& shadows,
                                         int64_t shadow_mode) {
  IAMD_CHECK(!weights.empty() && sigma.numel() == (int64_t)weights.size() &&
                 sigma.scalar_type() == at::kFloat,
             "mt_sn_scale_cast: sigma must be fp32 [L]");
  IAMD_CHECK(shadow_mode == 0 || shadows.size() == weights.size(),
             "mt_sn_scale_cast: shadow list size");
  ScPlan& p = get_sc_plan(weights, shadows, shadow_mode == 0 ? 0 : (int)shadow_mode);
  auto flat = at::empty({p.total}, weights[0].options().dtype(at::kBFloat16));
  hipLaunchKernelGGL(sn_scale_cast, dim3(p.nblocks), dim3(kT), 0, stream(),
                     reinterpret_cast<const ScEntry*>(p.ents.data_ptr()),
                     p.blocks.data_ptr<int>(), sigma.data_ptr<float>(),
                     reinterpret_cast<__hip_bfloat16*>(flat.data_ptr()));
  IAMD_LAUNCH_CHECK();
  std::vector<at::Tensor> out;
  out.reserve(weights.size());
  for (size_t i = 0; i < weights.size(); ++i)
    out.push_back(flat.as_strided(weights[i].sizes(), weights[i].strides(), p.offs[i]));
  return out;
}

}  // namespace iamd

namespace iamd {

// ---- k5d: spectral-norm scale backward -------------------------------------------------
//   dW = G/σ − (⟨G, W⟩/σ²) u vᵀ      (W/σ with u, v, σ held constant; reference semantics of
//                                    torch.nn.utils.spectral_norm's weight = W_orig / σ)
// Two launches per layer instead of ~7 full-weight PyTorch passes (fp32 cast of G, G·W, sum,
// outer(u, v), scale, divide, subtract): K1 partial ⟨G, W⟩ per block + v permuted into the
// weight's memory column order; K2 sums the partials (same order in every block:
// deterministic) and writes dW row by row with coalesced v reads.
namespace {

constexpr int kSnbT = 256;

__device__ __forceinline__ void load_w8(const float* p, float (&v)[8]) {
  load_vec<float, 4>(p, *reinterpret_cast<float(*)[4]>(v));
  load_vec<float, 4>(p + 4, *reinterpret_cast<float(*)[4]>(v + 4));
}
__device__ __forceinline__ void load_w8(const __hip_bfloat16* p, float (&v)[8]) {
  load_vec<__hip_bfloat16, 8>(p, v);
}

template <typename G, typename WT>
__global__ void __launch_bounds__(kSnbT)
snb_reduce(const G* __restrict__ g, const WT* __restrict__ W, int64_t n,
           const float* __restrict__ v, float* __restrict__ vm, int64_t w, int64_t cl_cin,
           int64_t cl_khw, float* __restrict__ partial) {
  __shared__ float sh[kSnbT / 64];
  const int64_t gtid = (int64_t)blockIdx.x * kSnbT + threadIdx.x;
  const int64_t gsz = (int64_t)gridDim.x * kSnbT;
  for (int64_t c = gtid; c < w; c += gsz) {
    int64_t lc = c;
    if (cl_cin) {
      const uint32_t q = (uint32_t)c / (uint32_t)cl_cin;
      lc = (int64_t)((uint32_t)c - q * (uint32_t)cl_cin) * cl_khw + q;
    }
    vm[c] = v[lc];
  }
  float acc = 0.f;
  if ((n & 7) == 0) {  // 8 elements per lane per trip, two trips in flight
    for (int64_t i = gtid * 8; i < n; i += gsz * 16) {
      const int64_t j = i + gsz * 8;
      const bool two = j < n;
      float gv[2][8], wv[2][8];
      load_vec<G, 8>(g + i, gv[0]);
      load_w8(W + i, wv[0]);
      if (two) {
        load_vec<G, 8>(g + j, gv[1]);
        load_w8(W + j, wv[1]);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) gv[1][k] = wv[1][k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = fmaf(gv[0][k], wv[0][k], acc);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = fmaf(gv[1][k], wv[1][k], acc);
    }
  } else {
    for (int64_t i = gtid; i < n; i += gsz) acc = fmaf(to_f<G>(g[i]), to_f<WT>(W[i]), acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < kSnbT / 64; ++k) s += sh[k];
    // a bf16 W read is the shadow bf16(W), already the weight itself: no rescale needed
    partial[blockIdx.x] = s;
  }
}

template <typename G>
__global__ void __launch_bounds__(kSnbT)
snb_apply(const G* __restrict__ g, const float* __restrict__ u, const float* __restrict__ vm,
          const float* __restrict__ sigma, const float* __restrict__ partial, int P,
          float* __restrict__ dw, int64_t h, int64_t w) {
  __shared__ float sh[kSnbT / 64];
  float d = 0.f;
  for (int k = threadIdx.x; k < P; k += kSnbT) d += partial[k];
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = d;
  __syncthreads();
  float dot = 0.f;
  for (int k = 0; k < kSnbT / 64; ++k) dot += sh[k];
  const float s = sigma[0];
  const float inv = 1.f / s;
  const float coef = dot / (s * s);
  const int64_t n = h * w;
  if ((w & 7) == 0) {  // flat walk, 8 columns of one row per lane: 16-B loads and stores
    const int64_t step = (int64_t)gridDim.x * kSnbT * 8;
    // two trips' loads in flight per lane
    for (int64_t i0 = ((int64_t)blockIdx.x * kSnbT + threadIdx.x) * 8; i0 < n; i0 += 2 * step) {
      float gv[2][8], vv[2][8], cu[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int64_t i = i0 + h2 * step;
        if (i >= n) continue;
        const uint32_t r = (uint32_t)i / (uint32_t)w;  // n < 2^31 (checked on the host)
        const int64_t c = i - (int64_t)r * w;
        cu[h2] = coef * u[r];
        load_vec<G, 8>(g + i, gv[h2]);
        load_vec<float, 4>(vm + c, *reinterpret_cast<float(*)[4]>(vv[h2]));
        load_vec<float, 4>(vm + c + 4, *reinterpret_cast<float(*)[4]>(vv[h2] + 4));
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int64_t i = i0 + h2 * step;
        if (i >= n) continue;
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf(gv[h2][k], inv, -cu[h2] * vv[h2][k]);
        store_vec<float, 4>(dw + i, *reinterpret_cast<float(*)[4]>(o));
        store_vec<float, 4>(dw + i + 4, *reinterpret_cast<float(*)[4]>(o + 4));
      }
    }
    return;
  }
  for (int64_t r = blockIdx.x; r < h; r += gridDim.x) {
    const float cu = coef * u[r];
    const G* gr = g + r * w;
    float* dr = dw + r * w;
    for (int64_t c = threadIdx.x; c < w; c += kSnbT)
      dr[c] = fmaf(to_f<G>(gr[c]), inv, -cu * vm[c]);
  }
}

}  // namespace

// shadow (optional, may be undefined / empty): bf16(W) laid out like W, read instead of the fp32
// weight for the <G, W> reduction (half the bytes of that pass)
at::Tensor sn_scale_backward(const at::Tensor& grad_in, const at::Tensor& weight,
                             const at::Tensor& u, const at::Tensor& v, const at::Tensor& sigma,
                             const c10::optional<at::Tensor>& shadow,
                             const c10::optional<at::Tensor>& dst) {
  IAMD_CHECK(weight.is_cuda() && weight.scalar_type() == at::kFloat, "sn_scale_backward: fp32 W");
  IAMD_CHECK(u.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat &&
                 sigma.scalar_type() == at::kFloat && sigma.numel() >= 1,
             "sn_scale_backward: fp32 u, v, sigma");
  const bool cl = weight.dim() == 4 && !weight.is_contiguous() &&
                  weight.is_contiguous(at::MemoryFormat::ChannelsLast);
  IAMD_CHECK(cl || weight.is_contiguous(), "sn_scale_backward: W contiguous or channels-last");
  const auto fmt = cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  at::Tensor grad = grad_in.contiguous(fmt);
  const int64_t n = weight.numel(), h = weight.size(0), w = n / std::max<int64_t>(1, h);
  IAMD_CHECK(u.numel() == h && v.numel() == w, "sn_scale_backward: u/v sizes");
  IAMD_CHECK(w < (1ll << 31), "sn_scale_backward: row too long");
  const int64_t cl_cin = cl ? weight.size(1) : 0, cl_khw = cl ? weight.size(2) * weight.size(3) : 0;
  // dst: the parameter's DDP bucket slice (parallel/ddp.py): dW lands there, no copy after
  const bool has_dst = dst.has_value() && dst->defined();
  if (has_dst)
    IAMD_CHECK(dst->is_cuda() && dst->scalar_type() == at::kFloat && dst->numel() == n &&
                   dst->sizes() == weight.sizes() && dst->strides() == weight.strides(),
               "sn_scale_backward: dst must be fp32 and laid out like W");
  auto dw = has_dst ? *dst : at::empty_like(weight, fmt);
  IAMD_CHECK(n < (1ll << 31), "sn_scale_backward: weight too large");
  const int P = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 4095) / 4096));
  const int P4 = (P + 3) & ~3;  // keeps vm 16-byte aligned for the vector loads
  auto ws = at::empty({P4 + w}, weight.options());
  float* partial = ws.data_ptr<float>();
  float* vm = partial + P4;
  const int ablocks = (w & 7) == 0
                          ? (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 2047) / 2048))
                          : (int)std::max<int64_t>(1, std::min<int64_t>(h, 1024));
  hipStream_t st = stream();
  const bool use_shadow = shadow.has_value() && shadow->defined() && shadow->numel() == n;
  if (use_shadow)
    IAMD_CHECK(shadow->scalar_type() == at::kBFloat16 && shadow->strides() == weight.strides() &&
                   (reinterpret_cast<uintptr_t>(shadow->data_ptr()) & 15) == 0,
               "sn_scale_backward: the shadow must be bf16, laid out like W, 16-B aligned");
  auto run = [&](auto* gp) {
    using G = std::remove_const_t<std::remove_pointer_t<decltype(gp)>>;
    if (use_shadow)
      hipLaunchKernelGGL((snb_reduce<G, __hip_bfloat16>), dim3(P), dim3(kSnbT), 0, st, gp,
                         reinterpret_cast<const __hip_bfloat16*>(shadow->data_ptr()), n,
                         v.data_ptr<float>(), vm, w, cl_cin, cl_khw, partial);
    else
      hipLaunchKernelGGL((snb_reduce<G, float>), dim3(P), dim3(kSnbT), 0, st, gp,
                         weight.data_ptr<float>(), n, v.data_ptr<float>(), vm, w, cl_cin, cl_khw,
                         partial);
    hipLaunchKernelGGL((snb_apply<G>), dim3(ablocks), dim3(kSnbT), 0, st, gp,
                       u.data_ptr<float>(), vm, sigma.data_ptr<float>(), partial, P,
                       dw.data_ptr<float>(), h, w);
  };
  if (grad.scalar_type() == at::kBFloat16)
    run(reinterpret_cast<const __hip_bfloat16*>(grad.data_ptr()));
  else if (grad.scalar_type() == at::kFloat)
    run(grad.data_ptr<float>());
  else
    IAMD_CHECK(false, "sn_scale_backward: grad must be bf16 or fp32");
  IAMD_LAUNCH_CHECK();
  return dw;
}

}  // namespace iamd
