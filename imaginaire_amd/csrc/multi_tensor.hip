// k4 / k5: multi-tensor optimizer and model-averaging kernels.
//
// One launch covers every parameter tensor of a network: the host builds a
// device-resident table {pointers, numel} plus a block map (tensor id, chunk
// offset) once per distinct tensor list (cached by pointer signature, so the
// steady state costs no host work beyond a hash and is hipGraph-capturable),
// and each workgroup streams one 16-byte-vectorised chunk.
//
//   mt_adam     : Adam / AdamW (reference FusedAdam, utils/trainer.py:271-281)
//                 fp32 master params, fp32 or bf16 grads, optional bf16 shadow
//                 copy of the updated weights written in the same pass.
//   mt_sn_sigma : σ_i = u_iᵀ W_i v_i for every spectral-normalised weight
//                 (reference ModelAverage.sn_compute_weight, model_average.py:183-197)
//   mt_ema      : t = β·t + (1-β)·s·scale_i  (model_average.py:87-131; scale_i = 1/σ_i
//                 absorbs spectral norm into the averaged model)
//   mt_scale    : x *= s (gradient clipping / unscale)
//   mt_sqnorm   : Σ x² per list (gradient-norm for clipping)
#include "common.h"

#include <cstdlib>
#include <type_traits>
#include <mutex>
#include <unordered_map>
#include <unordered_set>

namespace iamd {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 256 * 4 * 16;  // elements per workgroup (fp32: 64 KiB per operand)

struct TensorEntry {
  void* p[5];
  int64_t numel;
  int64_t cols;  // numel / size(0): row length when viewed as a matrix (spectral norm)
  // channels-last 4-D weights: memory column (kh, kw, ci) -> logical column (ci, kh, kw)
  int64_t cl_cin;  // 0 = memory order == logical order
  int64_t cl_khw;
};

struct Table {
  at::Tensor entries;  // device: TensorEntry[T]
  at::Tensor blocks;   // device: int2 {tensor, chunk} per workgroup
  int nblocks;
};

std::mutex g_mu;
std::unordered_map<uint64_t, Table> g_cache;

}  // namespace

// ---- host -> device table staging that is safe under hipGraph capture -----------------------
// Outside a capture: pinned staging + async copy on the current stream (never blocks the
// host). During a capture no copy may be enqueued (a pageable/pinned H2D node would re-read a
// host buffer that is gone by replay time), so the device buffer is allocated (from the
// graph's private pool) and the upload is DEFERRED: flush_deferred_uploads() copies it
// synchronously after the capture has ended, before the first replay. Buffers created during
// a capture are also kept alive for the life of the process, so a later cache eviction can
// never free memory a graph still reads.
namespace {
struct Deferred {
  at::Tensor dst;
  std::vector<uint8_t> bytes;
};
std::mutex g_def_mu;
std::vector<Deferred> g_deferred;
std::vector<at::Tensor> g_graph_keep;
// Tables made during a capture are carved from a persistent arena allocated OUTSIDE any
// capture (regular caching-allocator memory): graph-pool memory allocated inside a capture
// belongs to the graph's own allocation nodes and need not hold host-written bytes at
// replay time.
constexpr int64_t kArenaBytes = 64ll << 20;
std::unordered_map<int, std::pair<at::Tensor, int64_t>> g_arena;

void ensure_arena(const at::Device& dev) {
  auto& a = g_arena[dev.index()];
  if (!a.first.defined())
    a = {at::empty({kArenaBytes}, at::TensorOptions().dtype(at::kByte).device(dev)), 0};
}
}  // namespace

bool stream_capturing() {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  IAMD_HIP_CHECK(hipStreamIsCapturing(stream(), &st));
  return st != hipStreamCaptureStatusNone;
}

at::Tensor stage_to_device(const void* src, size_t bytes, const at::Device& dev) {
  const int64_t n = (int64_t)std::max<size_t>(bytes, 1);
  if (stream_capturing()) {
    std::lock_guard<std::mutex> lk(g_def_mu);
    auto it = g_arena.find(dev.index());
    IAMD_CHECK(it != g_arena.end() && it->second.first.defined(),
               "no table arena: run the step once eagerly before capturing it");
    const int64_t off = (it->second.second + 255) / 256 * 256;
    IAMD_CHECK(off + n <= kArenaBytes, "capture table arena exhausted");
    auto d = it->second.first.narrow(0, off, n);
    it->second.second = off + n;
    Deferred df;
    df.dst = d;
    df.bytes.assign(reinterpret_cast<const uint8_t*>(src),
                    reinterpret_cast<const uint8_t*>(src) + bytes);
    g_deferred.push_back(std::move(df));
    g_graph_keep.push_back(d);
    return d;
  }
  {
    std::lock_guard<std::mutex> lk(g_def_mu);
    ensure_arena(dev);  // reserved at the first eager use, ready for a later capture
  }
  auto pin = at::TensorOptions().dtype(at::kByte).pinned_memory(true);
  auto h = at::empty({n}, pin);
  if (bytes) memcpy(h.data_ptr(), src, bytes);
  return h.to(dev, /*non_blocking=*/true);
}

void keep_for_graph(const at::Tensor& t) {
  if (!t.defined() || !stream_capturing()) return;
  static std::unordered_set<const void*> kept;
  std::lock_guard<std::mutex> lk(g_def_mu);
  const void* key = t.storage().unsafeGetStorageImpl();
  if (kept.insert(key).second) g_graph_keep.push_back(t);
}

int64_t flush_deferred_uploads() {
  std::lock_guard<std::mutex> lk(g_def_mu);
  const int64_t n = (int64_t)g_deferred.size();
  for (auto& d : g_deferred)
    if (!d.bytes.empty())
      IAMD_HIP_CHECK(hipMemcpy(d.dst.data_ptr(), d.bytes.data(), d.bytes.size(),
                               hipMemcpyHostToDevice));
  g_deferred.clear();
  return n;
}

namespace {

uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  return h;
}

// Build (or fetch from cache) the device table for up to 5 parallel tensor lists.
Table& get_table(const std::vector<std::vector<at::Tensor>>& lists, const at::Device& dev) {
  const size_t T = lists[0].size();
  uint64_t h = 1469598103934665603ULL ^ (uint64_t)lists.size();
  // the key covers everything an entry records: pointers, sizes and the memory layout (a
  // freed tensor's address reused by one of another shape must not hit a stale entry)
  for (size_t i = 0; i < T; ++i) {
    for (auto& l : lists) {
      // (an empty tensor stands for "no operand": the optional bf16 shadow of a parameter)
      h = mix(h, l[i].numel() ? reinterpret_cast<uint64_t>(l[i].data_ptr()) : 0);
      h = mix(h, (uint64_t)l[i].numel());
    }
    const at::Tensor& t0 = lists[0][i];
    h = mix(h, t0.dim() > 0 ? (uint64_t)t0.size(0) : 0);
    h = mix(h, t0.dim() == 4 ? (uint64_t)(t0.size(1) * 31 + t0.size(2) * 7 + t0.size(3)) : 1);
    h = mix(h, (uint64_t)t0.is_contiguous());
  }
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cache.find(h);
  if (it != g_cache.end()) {
    keep_for_graph(it->second.entries);
    keep_for_graph(it->second.blocks);
    return it->second;
  }
  std::vector<TensorEntry> ents(T);
  std::vector<int32_t> bm;
  for (size_t i = 0; i < T; ++i) {
    for (size_t k = 0; k < 5; ++k)
      ents[i].p[k] = (k < lists.size() && lists[k][i].numel()) ? lists[k][i].data_ptr() : nullptr;
    ents[i].numel = lists[0][i].numel();
    ents[i].cols = lists[0][i].dim() > 0 && lists[0][i].size(0) > 0
                       ? ents[i].numel / lists[0][i].size(0) : 1;
    const at::Tensor& t0 = lists[0][i];
    const bool cl = t0.dim() == 4 && !t0.is_contiguous() &&
                    t0.is_contiguous(at::MemoryFormat::ChannelsLast);
    ents[i].cl_cin = cl ? t0.size(1) : 0;
    ents[i].cl_khw = cl ? t0.size(2) * t0.size(3) : 0;
    // every parallel operand of the same rank must share the layout of list 0
    for (size_t k = 1; k < lists.size(); ++k)
      if (lists[k][i].dim() == t0.dim())
        IAMD_CHECK(lists[k][i].strides() == t0.strides(),
                   "multi-tensor: operand layouts differ (strides must match)");
    const int64_t nch = (ents[i].numel + kChunk - 1) / kChunk;
    for (int64_t c = 0; c < nch; ++c) {
      bm.push_back((int32_t)i);
      bm.push_back((int32_t)c);
    }
  }
  // pinned staging + async copy on the current stream (deferred under graph capture)
  Table t;
  t.entries = stage_to_device(ents.data(), T * sizeof(TensorEntry), dev);
  t.blocks = stage_to_device(bm.data(), bm.size() * sizeof(int32_t), dev).view(at::kInt);
  t.nblocks = (int)(bm.size() / 2);
  if (g_cache.size() > 256) g_cache.clear();
  auto res = g_cache.emplace(h, std::move(t));
  return res.first->second;
}

// Device-resident Adam hyper-parameters [lr, step, step_size, rsqrt(bc2)] (capturable
// optimizer step: the step count and the bias corrections live on the device, so a replayed
// hipGraph advances them instead of baking the capture-time values).
__global__ void adam_hyper_step(float* __restrict__ hyper, float beta1, float beta2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float step = hyper[1] + 1.f;
    hyper[1] = step;
    const float bc1 = 1.f - powf(beta1, step);
    const float bc2 = 1.f - powf(beta2, step);
    hyper[2] = hyper[0] / bc1;
    hyper[3] = rsqrtf(bc2);
  }
}

// Streaming (non-temporal) 16-B fp32 load / store: Adam touches every byte once per step, so
// its traffic need not displace L2 lines. 2.44 -> 2.39 ms for the 415M-parameter SPADE set
// (5.1 -> 5.2 TB/s, profiles/adam_nt_ab_r6_mi355x.txt); IMAGINAIRE_AMD_ADAM_NT=0 switches back.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void ld4(const float* __restrict__ p, float (&o)[4]) {
  f32x4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p))
               : *reinterpret_cast<const f32x4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <bool NT>
__device__ __forceinline__ void st4(float* __restrict__ p, const float (&i)[4]) {
  f32x4 v = {i[0], i[1], i[2], i[3]};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  else *reinterpret_cast<f32x4*>(p) = v;
}

template <typename G, bool NT>
__global__ void __launch_bounds__(kThreads)
adam_kernel(const TensorEntry* __restrict__ ents, const int* __restrict__ blocks, float lr,
            float beta1, float beta2, float eps, float bc1, float bc2, float wd, int adamw,
            float grad_scale, const float* __restrict__ hyper) {
  const int b = blockIdx.x;
  const int t = blocks[2 * b], chunk = blocks[2 * b + 1];
  const TensorEntry e = ents[t];
  float* __restrict__ p = reinterpret_cast<float*>(e.p[0]);
  const G* __restrict__ g = reinterpret_cast<const G*>(e.p[1]);
  float* __restrict__ m = reinterpret_cast<float*>(e.p[2]);
  float* __restrict__ v = reinterpret_cast<float*>(e.p[3]);
  __hip_bfloat16* __restrict__ shadow = reinterpret_cast<__hip_bfloat16*>(e.p[4]);
  const int64_t start = (int64_t)chunk * kChunk;
  const int64_t end = min(e.numel, start + (int64_t)kChunk);
  float step_size, rbc2;
  if (hyper) {
    lr = hyper[0];
    step_size = hyper[2];
    rbc2 = hyper[3];
  } else {
    step_size = lr / bc1;
    rbc2 = rsqrtf(bc2);
  }
  const bool vec_ok = (((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) % 16 == 0) &&
                      ((uintptr_t)g % (4 * sizeof(G)) == 0) && (start % 4 == 0);
  if (vec_ok) {
    // U groups of 4 elements per lane per trip, all loads issued before any math: 4 x U 16-B
    // loads in flight per lane (one group at a time left the kernel latency-bound at ~1.5 TB/s)
    constexpr int U = 4;
    for (int64_t base = start + threadIdx.x * 4; base < end; base += kThreads * 4 * U) {
      float pv[U][4], gv[U][4], mv[U][4], vv[U][4];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kThreads * 4;
        ok[u] = i + 3 < end;
        if (ok[u]) {
          ld4<NT>(p + i, pv[u]);
          load_vec<G, 4>(g + i, gv[u]);
          ld4<NT>(m + i, mv[u]);
          ld4<NT>(v + i, vv[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const int64_t i = base + (int64_t)u * kThreads * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float gr = gv[u][k] * grad_scale;
          if (!adamw && wd != 0.f) gr = fmaf(wd, pv[u][k], gr);
          mv[u][k] = fmaf(beta1, mv[u][k], (1.f - beta1) * gr);
          vv[u][k] = fmaf(beta2, vv[u][k], (1.f - beta2) * gr * gr);
          const float denom = sqrtf(vv[u][k]) * rbc2 + eps;
          if (adamw && wd != 0.f) pv[u][k] *= (1.f - lr * wd);
          pv[u][k] -= step_size * mv[u][k] / denom;
        }
        st4<NT>(p + i, pv[u]);
        st4<NT>(m + i, mv[u]);
        st4<NT>(v + i, vv[u]);
        if (shadow) store_vec<__hip_bfloat16, 4>(shadow + i, pv[u]);
      }
    }
    // tail (numel not multiple of 4)
    const int64_t tail0 = start + ((end - start) / 4) * 4;
    for (int64_t i = tail0 + threadIdx.x; i < end; i += kThreads) {
      float gr = to_f<G>(g[i]) * grad_scale;
      float pv = p[i];
      if (!adamw && wd != 0.f) gr = fmaf(wd, pv, gr);
      float mv = fmaf(beta1, m[i], (1.f - beta1) * gr);
      float vv = fmaf(beta2, v[i], (1.f - beta2) * gr * gr);
      if (adamw && wd != 0.f) pv *= (1.f - lr * wd);
      pv -= step_size * mv / (sqrtf(vv) * rbc2 + eps);
      p[i] = pv; m[i] = mv; v[i] = vv;
      if (shadow) shadow[i] = __float2bfloat16(pv);
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
      float gr = to_f<G>(g[i]) * grad_scale;
      float pv = p[i];
      if (!adamw && wd != 0.f) gr = fmaf(wd, pv, gr);
      float mv = fmaf(beta1, m[i], (1.f - beta1) * gr);
      float vv = fmaf(beta2, v[i], (1.f - beta2) * gr * gr);
      if (adamw && wd != 0.f) pv *= (1.f - lr * wd);
      pv -= step_size * mv / (sqrtf(vv) * rbc2 + eps);
      p[i] = pv; m[i] = mv; v[i] = vv;
      if (shadow) shadow[i] = __float2bfloat16(pv);
    }
  }
}

// σ_i = Σ_{r,c} u[r] W[r,c] v[c]  (W viewed as [rows, numel/rows]); one partial per chunk.
// entry: p0 = W (fp32), p1 = u, p2 = v; rows carried in the sigma-rows array.
__global__ void __launch_bounds__(kThreads)
sn_sigma_kernel(const TensorEntry* __restrict__ ents, const int* __restrict__ blocks,
                float* __restrict__ part) {
  __shared__ float sh[kThreads / 64];
  const int b = blockIdx.x;
  const int t = blocks[2 * b], chunk = blocks[2 * b + 1];
  const TensorEntry e = ents[t];
  const float* __restrict__ W = reinterpret_cast<const float*>(e.p[0]);
  const float* __restrict__ u = reinterpret_cast<const float*>(e.p[1]);
  // p[3]: v permuted to the weight's MEMORY column order by sn_vperm (coalesced reads; the
  // logical-order v of a channels-last conv weight would be a stride-KH*KW gather)
  const float* __restrict__ v = reinterpret_cast<const float*>(e.p[3]);
  const int64_t ncol = e.cols;
  const int64_t start = (int64_t)chunk * kChunk;
  const int64_t end = min(e.numel, start + (int64_t)kChunk);
  float acc = 0.f;
  if ((ncol & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(v) & 15) == 0) {
    // 4 consecutive elements (one row: ncol % 4 == 0) per lane and trip, 16-B loads of W and v;
    // chunk starts are multiples of 4 (kChunk % 4 == 0)
    const int64_t i0 = start + threadIdx.x * 4;
    int64_t r = i0 / ncol;
    int64_t c = i0 - r * ncol;
    for (int64_t i = i0; i < end; i += kThreads * 4) {
      const float4 w4 = *reinterpret_cast<const float4*>(W + i);
      const float4 v4 = *reinterpret_cast<const float4*>(v + c);
      acc = fmaf(u[r], fmaf(w4.x, v4.x, fmaf(w4.y, v4.y, fmaf(w4.z, v4.z, w4.w * v4.w))), acc);
      c += kThreads * 4;
      while (c >= ncol) { c -= ncol; ++r; }
    }
  } else {
    // (row, column) walked incrementally: no 64-bit division per element
    const int64_t i0 = start + threadIdx.x;
    int64_t r = i0 / ncol;
    int64_t c = i0 - r * ncol;
    for (int64_t i = i0; i < end; i += kThreads) {
      acc = fmaf(u[r] * W[i], v[c], acc);
      c += kThreads;
      while (c >= ncol) { c -= ncol; ++r; }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < kThreads / 64; ++k) s += sh[k];
    part[b] = s;  // per-workgroup partial; reduce_block_partials sums them in a fixed order
  }
}

// out[t] = Σ_{b : blocks[b].tensor == t} part[b], one workgroup per tensor (T = 1 with
// all_blocks: every partial). Fixed per-thread strides + a fixed tree: bitwise reproducible,
// unlike one float atomic per workgroup (whose arrival order varies run to run).
__global__ void __launch_bounds__(kThreads)
reduce_block_partials(const float* __restrict__ part, const int* __restrict__ blocks, int nblocks,
                      bool all_blocks, float* __restrict__ out) {
  __shared__ float sh[kThreads / 64];
  const int t = blockIdx.x;
  float acc = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += kThreads)
    if (all_blocks || blocks[2 * b] == t) acc += part[b];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < kThreads / 64; ++k) s += sh[k];
    out[t] = s;
  }
}

// one block per tensor: vm[c] = v[logical(c)] for every memory column c
__global__ void __launch_bounds__(kThreads)
sn_vperm(const TensorEntry* __restrict__ ents) {
  const TensorEntry e = ents[blockIdx.x];
  const float* __restrict__ v = reinterpret_cast<const float*>(e.p[2]);
  float* __restrict__ vm = reinterpret_cast<float*>(e.p[3]);
  const uint32_t cin = (uint32_t)e.cl_cin;
  for (int64_t c = threadIdx.x; c < e.cols; c += kThreads) {
    int64_t lc = c;
    if (cin) {
      const uint32_t q = (uint32_t)c / cin;
      lc = (int64_t)((uint32_t)c - q * cin) * e.cl_khw + q;
    }
    vm[c] = v[lc];
  }
}

// t = beta*t + (1-beta)*s*scale[t_idx]; p0 = target, p1 = source (same dtype: fp32).
// NT: the average itself is streamed (non-temporal fp32 load / store: nothing else in the step
// reads it): 0.962 -> 0.928 ms for 415M parameters (profiles/ema_nt_ab_r6_mi355x.txt);
// IMAGINAIRE_AMD_EMA_NT=0 switches back to plain accesses.
template <typename T, bool NT>
__global__ void __launch_bounds__(kThreads)
ema_kernel(const TensorEntry* __restrict__ ents, const int* __restrict__ blocks, float beta,
           const float* __restrict__ inv_scale, const int64_t* __restrict__ count,
           int64_t warm_until) {
  const int b = blockIdx.x;
  const int t = blocks[2 * b], chunk = blocks[2 * b + 1];
  const TensorEntry e = ents[t];
  // device-side warm-up switch (model_average.py: beta = 0 until start_iteration), so a
  // replayed hipGraph turns the average on at the right iteration
  if (count && *count <= warm_until) beta = 0.f;
  T* __restrict__ dst = reinterpret_cast<T*>(e.p[0]);
  const T* __restrict__ src = reinterpret_cast<const T*>(e.p[1]);
  const float sc = inv_scale ? 1.f / inv_scale[t] : 1.f;
  const float a = 1.f - beta;
  const int64_t start = (int64_t)chunk * kChunk;
  const int64_t end = min(e.numel, start + (int64_t)kChunk);
  const float as = a * sc;
  if (sizeof(T) == 4 && (((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    // 16-B accesses, U groups per lane per trip with every load issued first
    constexpr int U = 4;
    const int64_t vend = start + ((end - start) & ~(int64_t)3);
    for (int64_t base = start + threadIdx.x * 4; base < vend; base += kThreads * 4 * U) {
      float dv[U][4], sv[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kThreads * 4;
        if (i < vend) {
          if constexpr (std::is_same<T, float>::value) ld4<NT>(dst + i, dv[u]);
          else load_vec<T, 4>(dst + i, dv[u]);
          load_vec<T, 4>(src + i, sv[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * kThreads * 4;
        if (i >= vend) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) dv[u][k] = fmaf(beta, dv[u][k], as * sv[u][k]);
        if constexpr (std::is_same<T, float>::value) st4<NT>(dst + i, dv[u]);
        else store_vec<T, 4>(dst + i, dv[u]);
      }
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += kThreads)
      dst[i] = from_f<T>(fmaf(beta, to_f<T>(dst[i]), as * to_f<T>(src[i])));
    return;
  }
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads)
    dst[i] = from_f<T>(fmaf(beta, to_f<T>(dst[i]), as * to_f<T>(src[i])));
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
scale_kernel(const TensorEntry* __restrict__ ents, const int* __restrict__ blocks,
             const float* __restrict__ s) {
  const int b = blockIdx.x;
  const int t = blocks[2 * b], chunk = blocks[2 * b + 1];
  const TensorEntry e = ents[t];
  T* __restrict__ x = reinterpret_cast<T*>(e.p[0]);
  const float f = *s;
  const int64_t start = (int64_t)chunk * kChunk;
  const int64_t end = min(e.numel, start + (int64_t)kChunk);
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) x[i] = from_f<T>(to_f<T>(x[i]) * f);
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
sqnorm_kernel(const TensorEntry* __restrict__ ents, const int* __restrict__ blocks,
              float* __restrict__ part) {
  __shared__ float sh[kThreads / 64];
  const int b = blockIdx.x;
  const int t = blocks[2 * b], chunk = blocks[2 * b + 1];
  const TensorEntry e = ents[t];
  const T* __restrict__ x = reinterpret_cast<const T*>(e.p[0]);
  const int64_t start = (int64_t)chunk * kChunk;
  const int64_t end = min(e.numel, start + (int64_t)kChunk);
  float acc = 0.f;
  for (int64_t i = start + threadIdx.x; i < end; i += kThreads) {
    const float v = to_f<T>(x[i]);
    acc = fmaf(v, v, acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < kThreads / 64; ++k) s += sh[k];
    part[b] = s;
  }
}

void check_same_dtype(const std::vector<at::Tensor>& l, at::ScalarType st, const char* what) {
  for (auto& t : l) {
    IAMD_CHECK(t.scalar_type() == st, what, ": dtype mismatch");
    IAMD_CHECK(t.is_non_overlapping_and_dense(), what, ": tensors must be dense");
  }
}

}  // namespace

void mt_adam(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
             const std::vector<at::Tensor>& exp_avgs, const std::vector<at::Tensor>& exp_avg_sqs,
             const std::vector<at::Tensor>& shadows, double lr, double beta1, double beta2,
             double eps, int64_t step, double weight_decay, bool adamw, double grad_scale,
             const c10::optional<at::Tensor>& hyper) {
  if (params.empty()) return;
  float* hp = nullptr;
  if (hyper.has_value() && hyper->defined()) {
    IAMD_CHECK(hyper->is_cuda() && hyper->scalar_type() == at::kFloat && hyper->numel() == 4 &&
                   hyper->is_contiguous(),
               "mt_adam: hyper must be a contiguous fp32 device tensor [lr, step, ., .]");
    hp = hyper->data_ptr<float>();
  }
  IAMD_CHECK(params.size() == grads.size() && params.size() == exp_avgs.size() &&
                 params.size() == exp_avg_sqs.size(),
             "mt_adam: list sizes differ");
  check_same_dtype(params, at::kFloat, "mt_adam params");
  check_same_dtype(exp_avgs, at::kFloat, "mt_adam exp_avg");
  check_same_dtype(exp_avg_sqs, at::kFloat, "mt_adam exp_avg_sq");
  const auto gdt = grads[0].scalar_type();
  check_same_dtype(grads, gdt, "mt_adam grads");
  std::vector<std::vector<at::Tensor>> lists{params, grads, exp_avgs, exp_avg_sqs};
  if (!shadows.empty()) {
    // optional per parameter: an empty tensor = no shadow for that parameter
    IAMD_CHECK(shadows.size() == params.size(), "mt_adam: shadow list size");
    for (size_t i = 0; i < shadows.size(); ++i) {
      if (shadows[i].numel() == 0) continue;
      IAMD_CHECK(shadows[i].scalar_type() == at::kBFloat16 && shadows[i].is_cuda() &&
                     shadows[i].sizes() == params[i].sizes() &&
                     shadows[i].strides() == params[i].strides(),
                 "mt_adam: a shadow must be a bf16 tensor laid out like its parameter");
    }
    lists.push_back(shadows);
  }
  Table& tb = get_table(lists, params[0].device());
  const float bc1 = 1.f - (float)std::pow(beta1, (double)step);
  const float bc2 = 1.f - (float)std::pow(beta2, (double)step);
  auto ents = reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr());
  auto blks = tb.blocks.data_ptr<int>();
  if (hp)
    hipLaunchKernelGGL(adam_hyper_step, dim3(1), dim3(64), 0, stream(), hp, (float)beta1,
                       (float)beta2);
  static const bool nt = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_ADAM_NT");
    return !(e && e[0] == '0');
  }();
#define IAMD_ADAM_LAUNCH(G, NT)                                                              \
  hipLaunchKernelGGL((adam_kernel<G, NT>), dim3(tb.nblocks), dim3(kThreads), 0, stream(), ents, \
                     blks, (float)lr, (float)beta1, (float)beta2, (float)eps, bc1, bc2,        \
                     (float)weight_decay, adamw ? 1 : 0, (float)grad_scale, hp)
  if (gdt == at::kFloat) {
    if (nt) IAMD_ADAM_LAUNCH(float, true);
    else IAMD_ADAM_LAUNCH(float, false);
  } else if (gdt == at::kBFloat16) {
    if (nt) IAMD_ADAM_LAUNCH(__hip_bfloat16, true);
    else IAMD_ADAM_LAUNCH(__hip_bfloat16, false);
  }
#undef IAMD_ADAM_LAUNCH
  else
    IAMD_CHECK(false, "mt_adam: grads must be fp32 or bf16");
  IAMD_LAUNCH_CHECK();
}

at::Tensor mt_sn_sigma(const std::vector<at::Tensor>& weights, const std::vector<at::Tensor>& us,
                       const std::vector<at::Tensor>& vs) {
  IAMD_CHECK(!weights.empty(), "mt_sn_sigma: empty list");
  check_same_dtype(weights, at::kFloat, "mt_sn_sigma W");
  check_same_dtype(us, at::kFloat, "mt_sn_sigma u");
  check_same_dtype(vs, at::kFloat, "mt_sn_sigma v");
  // persistent per-device workspace for the memory-order v copies: stable pointers keep the
  // cached device table valid across calls
  static std::mutex ws_mu;
  static std::unordered_map<int, at::Tensor> ws_map;
  int64_t total = 0;
  for (auto& w : weights) total += w.numel() / std::max<int64_t>(1, w.size(0));
  std::vector<at::Tensor> vms;
  {
    std::lock_guard<std::mutex> lk(ws_mu);
    const int dev = weights[0].get_device();
    at::Tensor& ws = ws_map[dev];
    if (!ws.defined() || ws.numel() < total) {
      // an old workspace that a captured graph names is never freed (kept by keep_for_graph);
      // one only ever used eagerly is released with its last reference
      ws = at::empty({total}, weights[0].options());
    }
    keep_for_graph(ws);  // (no-op outside a capture)
    int64_t off = 0;
    for (auto& w : weights) {
      const int64_t cols = w.numel() / std::max<int64_t>(1, w.size(0));
      vms.push_back(ws.narrow(0, off, cols));
      off += cols;
    }
  }
  Table& tb = get_table({weights, us, vs, vms}, weights[0].device());
  auto sigma = at::empty({(int64_t)weights.size()}, weights[0].options());
  auto part = at::empty({(int64_t)tb.nblocks}, weights[0].options());
  hipLaunchKernelGGL(sn_vperm, dim3((unsigned)weights.size()), dim3(kThreads), 0, stream(),
                     reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr()));
  hipLaunchKernelGGL(sn_sigma_kernel, dim3(tb.nblocks), dim3(kThreads), 0, stream(),
                     reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr()),
                     tb.blocks.data_ptr<int>(), part.data_ptr<float>());
  hipLaunchKernelGGL(reduce_block_partials, dim3((unsigned)weights.size()), dim3(kThreads), 0,
                     stream(), part.data_ptr<float>(), tb.blocks.data_ptr<int>(), tb.nblocks,
                     false, sigma.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  return sigma;
}

void mt_ema(const std::vector<at::Tensor>& targets, const std::vector<at::Tensor>& sources,
            double beta, const c10::optional<at::Tensor>& sigma,
            const c10::optional<at::Tensor>& count, int64_t start) {
  if (targets.empty()) return;
  const int64_t* cp = nullptr;
  if (count.has_value() && count->defined()) {
    IAMD_CHECK(count->is_cuda() && count->scalar_type() == at::kLong && count->numel() == 1,
               "mt_ema: count must be a 1-element int64 device tensor");
    cp = count->data_ptr<int64_t>();
  }
  const auto dt = targets[0].scalar_type();
  check_same_dtype(targets, dt, "mt_ema targets");
  check_same_dtype(sources, dt, "mt_ema sources");
  Table& tb = get_table({targets, sources}, targets[0].device());
  const float* sp = nullptr;
  if (sigma.has_value() && sigma->defined()) {
    IAMD_CHECK(sigma->numel() == (int64_t)targets.size() && sigma->scalar_type() == at::kFloat,
               "mt_ema: sigma must be fp32 [T]");
    sp = sigma->data_ptr<float>();
  }
  static const bool nt = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_EMA_NT");
    return !(e && e[0] == '0');
  }();
  IAMD_DISPATCH_FLOAT_TYPES(dt, "mt_ema", [&] {
    auto ents = reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr());
    if (nt)
      hipLaunchKernelGGL((ema_kernel<scalar_t, true>), dim3(tb.nblocks), dim3(kThreads), 0,
                         stream(), ents, tb.blocks.data_ptr<int>(), (float)beta, sp, cp, start);
    else
      hipLaunchKernelGGL((ema_kernel<scalar_t, false>), dim3(tb.nblocks), dim3(kThreads), 0,
                         stream(), ents, tb.blocks.data_ptr<int>(), (float)beta, sp, cp, start);
  });
  IAMD_LAUNCH_CHECK();
}

void mt_scale(const std::vector<at::Tensor>& xs, const at::Tensor& s) {
  if (xs.empty()) return;
  const auto dt = xs[0].scalar_type();
  check_same_dtype(xs, dt, "mt_scale");
  Table& tb = get_table({xs}, xs[0].device());
  auto sf = s.to(at::kFloat).contiguous();
  IAMD_DISPATCH_FLOAT_TYPES(dt, "mt_scale", [&] {
    hipLaunchKernelGGL((scale_kernel<scalar_t>), dim3(tb.nblocks), dim3(kThreads), 0, stream(),
                       reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr()),
                       tb.blocks.data_ptr<int>(), sf.data_ptr<float>());
  });
  IAMD_LAUNCH_CHECK();
}

at::Tensor mt_sqnorm(const std::vector<at::Tensor>& xs) {
  IAMD_CHECK(!xs.empty(), "mt_sqnorm: empty");
  const auto dt = xs[0].scalar_type();
  check_same_dtype(xs, dt, "mt_sqnorm");
  Table& tb = get_table({xs}, xs[0].device());
  auto out = at::empty({1}, xs[0].options().dtype(at::kFloat));
  auto part = at::empty({(int64_t)tb.nblocks}, xs[0].options().dtype(at::kFloat));
  IAMD_DISPATCH_FLOAT_TYPES(dt, "mt_sqnorm", [&] {
    hipLaunchKernelGGL((sqnorm_kernel<scalar_t>), dim3(tb.nblocks), dim3(kThreads), 0, stream(),
                       reinterpret_cast<const TensorEntry*>(tb.entries.data_ptr()),
                       tb.blocks.data_ptr<int>(), part.data_ptr<float>());
  });
  hipLaunchKernelGGL(reduce_block_partials, dim3(1), dim3(kThreads), 0, stream(),
                     part.data_ptr<float>(), tb.blocks.data_ptr<int>(), tb.nblocks, true,
                     out.data_ptr<float>());
  IAMD_LAUNCH_CHECK();
  return out;
}

}  // namespace iamd
