// Shared helpers for the imaginaire_amd gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: all cross-lane reductions assume 64 lanes (__shfl_xor width 64);
//   * 16-byte vector global accesses (8 x bf16/fp16 or 4 x fp32 per lane);
//   * fp32 accumulation for every reduction, whatever the I/O dtype;
//   * kernels are launched on the current PyTorch HIP stream so they compose
//     with MIOpen / hipBLASLt work and with hipGraph capture.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdint>

namespace iamd {

constexpr int kWave = 64;

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// True while the current stream is being captured into a hipGraph.
bool stream_capturing();
// Host bytes -> new device byte tensor: async pinned copy normally; under hipGraph capture
// the copy is deferred to flush_deferred_uploads() (multi_tensor.hip).
at::Tensor stage_to_device(const void* src, size_t bytes, const at::Device& dev);
int64_t flush_deferred_uploads();
// Under hipGraph capture: keep ``t``'s storage alive for the life of the process. Every cached
// device object (multi-tensor table, spectral-norm plan, flip plan, workspace) a capture USES
// goes through this — including ones made eagerly before the capture and merely hit by it: a
// later cache eviction would otherwise free memory the graph still reads, and the caching
// allocator would hand it to the next eager allocation (a replay then reads garbage tables).
// No-op outside a capture.
void keep_for_graph(const at::Tensor& t);

#define IAMD_CHECK(cond, ...) TORCH_CHECK(cond, "imaginaire_amd: ", __VA_ARGS__)
#define IAMD_HIP_CHECK(expr)                                                     \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " at ", \
                __FILE__, ":", __LINE__);                                        \
  } while (0)
#define IAMD_LAUNCH_CHECK() IAMD_HIP_CHECK(hipGetLastError())

// ---- scalar conversion --------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<__hip_bfloat16>(__hip_bfloat16 v) {
  return __bfloat162float(v);
}
template <> __device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}
template <> __device__ __forceinline__ __half from_f<__half>(float v) { return __float2half(v); }

// ---- 16-byte vectors ----------------------------------------------------
template <typename T> struct VecN { static constexpr int N = 16 / sizeof(T); };

template <typename T, int N>
struct alignas(sizeof(T) * N >= 16 ? 16 : sizeof(T) * N) Pack {
  T v[N];
};

template <typename T, int N>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&out)[N]) {
  Pack<T, N> pk = *reinterpret_cast<const Pack<T, N>*>(p);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = to_f<T>(pk.v[i]);
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float (&in)[N]) {
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) pk.v[i] = from_f<T>(in[i]);
  *reinterpret_cast<Pack<T, N>*>(p) = pk;
}

// ---- wave / block reductions (wave64) -------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Chan et al. parallel merge of (count, mean, M2) triples.
__device__ __forceinline__ void chan_merge(float& n_a, float& mean_a, float& m2_a, float n_b,
                                           float mean_b, float m2_b) {
  float n = n_a + n_b;
  if (n_b == 0.f) return;
  if (n_a == 0.f) {
    n_a = n_b; mean_a = mean_b; m2_a = m2_b;
    return;
  }
  float delta = mean_b - mean_a;
  float fb = n_b / n;
  mean_a = mean_a + delta * fb;
  m2_a = m2_a + m2_b + delta * delta * n_a * fb;
  n_a = n;
}

__device__ __forceinline__ float act_fwd(float y, float slope) { return y > 0.f ? y : y * slope; }
__device__ __forceinline__ float act_grad(float y, float slope) { return y > 0.f ? 1.f : slope; }

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

// XCD-aware remap of a 1-D block index (MI355X: 8 XCDs, round-robin dispatch).
// Gives each XCD a contiguous range of logical blocks so neighbouring tiles share
// an L2. Bijective for any grid size (cdna_hip_programming.md §5 "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  constexpr int kXcd = 8;
  if (nwg <= kXcd) return bid;
  int q = nwg / kXcd, r = nwg % kXcd;
  int xcd = bid % kXcd, local = bid / kXcd;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

}  // namespace iamd

#define IAMD_DISPATCH_FLOAT_TYPES(SCALAR, NAME, ...)                              \
  [&] {                                                                          \
    switch (SCALAR) {                                                            \
      case at::ScalarType::Float: {                                              \
        using scalar_t = float;                                                  \
        return __VA_ARGS__();                                                    \
      }                                                                          \
      case at::ScalarType::BFloat16: {                                           \
        using scalar_t = __hip_bfloat16;                                         \
        return __VA_ARGS__();                                                    \
      }                                                                          \
      case at::ScalarType::Half: {                                               \
        using scalar_t = __half;                                                 \
        return __VA_ARGS__();                                                    \
      }                                                                          \
      default:                                                                   \
        TORCH_CHECK(false, NAME, ": unsupported dtype ", SCALAR);                \
    }                                                                            \
  }()
