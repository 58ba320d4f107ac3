// k16: fused few-shot attention  O = softmax_keys(scale * Q K^T) V   (bf16 in / out, fp32 inside)
//
// The fs_vid2vid reference-frame attention (reference generators/fs_vid2vid.py:944-951: energy
// = bmm(key^T, query), softmax over the K*HW reference positions, bmm with the features) without
// the B x KHW x HW energy / attention matrices in HBM: one forward kernel with an online softmax
// (flash-attention style) that also writes the per-query log-sum-exp, and two backward kernels
// that recompute the probabilities from it (one owns key blocks and accumulates dK, dV; one owns
// query blocks and accumulates dQ — no atomics, deterministic).
//
// MFMA v_mfma_f32_16x16x32_bf16 throughout, 64-wide waves, 16 queries (or keys) per wave, 4 or 8
// waves per workgroup sharing LDS tiles. Layout trick: scores are computed TRANSPOSED where the next
// product needs the probabilities as its B operand — the C layout of one 16x16 tile (lane l holds
// rows 4*(l/16)+e, column l%16) then feeds the B operand of the next MFMA directly (column l%16,
// k = 8*(l/16)+t) once the 32-long k dimension is taken in the order {tile 0: rows 4g..4g+3,
// tile 1: rows 4g..4g+3}; the A operand of that MFMA reads its LDS tile in the same order (two
// 8-byte reads). Per-query softmax statistics stay per lane (the query is the lane's column);
// only the running max needs a 4-lane reduction (xor 16, 32).
//
// Shapes: q [B, Lq, D], k [B, Lk, D], v [B, Lk, DV] contiguous bf16; D in {32, 64, 128}, DV a
// multiple of 32 up to 256, or 288 (the few-shot recipe's 128 + 128 + K value channels in one
// pass; the caller zero-pads: zero columns change no dot product), Lq and Lk multiples of 64.
// Every kernel's static LDS stays under 64 KB at D = 128, DV = 288. Scores in the log2 domain:
// p = exp2(s * scale * log2(e) - lse2). Measured: profiles/fs_attention_k16_probe_mi355x.txt.
#include "common.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace iamd {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;


constexpr float kNegBig = -1.0e30f;

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 join4(const bf16x4& lo, const bf16x4& hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__device__ __forceinline__ bf16x8 pack8(const float (&lo)[4], const float (&hi)[4]) {
  bf16x8 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    r[t] = (__bf16)lo[t];
    r[4 + t] = (__bf16)hi[t];
  }
  return r;
}

// A operand of a 32-deep product whose k index runs over two 16-row tiles (rows 4g..4g+3 of
// each): two 8-byte LDS reads from a row-major [row][k] tile (row = the lane's A row).
__device__ __forceinline__ bf16x8 read_a_split(const __bf16* row, int g) {
  return join4(*reinterpret_cast<const bf16x4*>(row + g * 4),
               *reinterpret_cast<const bf16x4*>(row + 16 + g * 4));
}

// Register-staged tile copy global -> LDS in two halves: load() issues the 16-byte global loads
// of the NEXT block into registers before the current block's MFMAs, store() writes them to
// LDS after the barrier — the global latency of block k + 1 overlaps the compute of block k
// (the synchronous load -> LDS -> barrier -> compute loop waited a full L2 / HBM round trip per
// block: ~0.2 us of MFMAs per step against ~1-2 us of latency). ROWS x COLS bf16 tile, source
// row stride ``stride`` elements, LDS row pitch LDP elements, NT threads.
template <int ROWS, int COLS, int LDP, int NT>
struct TileStage {
  static constexpr int T = ROWS * COLS / 8;    // 16-byte chunks
  static constexpr int I = (T + NT - 1) / NT;  // chunks per thread
  bf16x8 r[I];
  __device__ __forceinline__ void load(const __bf16* base, int64_t stride, int tid) {
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int e = tid + i * NT;
      if (T % NT == 0 || e < T) {
        const int rr = e / (COLS / 8), cc = (e - rr * (COLS / 8)) * 8;
        r[i] = *reinterpret_cast<const bf16x8*>(base + (int64_t)rr * stride + cc);
      }
    }
  }
  __device__ __forceinline__ void store(__bf16* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int e = tid + i * NT;
      if (T % NT == 0 || e < T) {
        const int rr = e / (COLS / 8), cc = (e - rr * (COLS / 8)) * 8;
        *reinterpret_cast<bf16x8*>(lds + rr * LDP + cc) = r[i];
      }
    }
  }
};

// ---- forward -----------------------------------------------------------------------------
// workgroup: 64 queries (wave w: queries 16w..16w+15) x all keys in blocks of 64 staged in LDS
// (K row-major, V^T from a host-transposed copy: 16-byte copies, no LDS transposition). Per block and wave: S^T (4 key tiles x D/32 MFMAs), the online
// softmax, O^T += V^T P^T (DV/16 tiles x 2 MFMAs).
// Split over keys (grid.y = split, keys [split * klen, +klen)) when the query tiles alone cannot
// fill the chip: each split then writes its unnormalised fp32 output with its running max and
// sum (opart / mpart / lpart), merged by attn_fwd_combine.
template <int D, int DV, int NW>
__global__ __launch_bounds__(NW * 64) void attn_fwd_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ vt,
    __bf16* __restrict__ o, float* __restrict__ lse2, int Lq, int Lk, float sl2, int klen,
    float* __restrict__ opart, float* __restrict__ mpart, float* __restrict__ lpart) {
  constexpr int KB = 64, KP = D + 8, VP = KB + 8;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[KB * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Vt[DV * VP];
  const int b = blockIdx.z, sp = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int qi = blockIdx.x * (NW * 16) + wid * 16 + l16;  // this lane's query (B/C column)
  const __bf16* kb = k + (int64_t)b * Lk * D;
  const __bf16* vtb = vt + (int64_t)b * DV * Lk;  // V^T [DV][Lk], transposed once on the host
  bf16x8 qf[D / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8*>(q + ((int64_t)b * Lq + qi) * D + ks * 32 + g * 8);
  f32x4 acc[DV / 16];
#pragma unroll
  for (int i = 0; i < DV / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, lsum = 0.f;
  const int kbeg = sp * klen, kend = min(Lk, kbeg + klen);
  TileStage<KB, D, KP, NW * 64> sK;
  TileStage<DV, KB, VP, NW * 64> sV;  // 16-byte rows of V^T
  if (kbeg < kend) {
    sK.load(kb + (int64_t)kbeg * D, D, tid);
    sV.load(vtb + kbeg, Lk, tid);
  }
  for (int k0 = kbeg; k0 < kend; k0 += KB) {
    __syncthreads();
    sK.store(Ks, tid);
    sV.store(Vt, tid);
    __syncthreads();
    if (k0 + KB < kend) {  // the next block's loads fly during this block's MFMAs
      sK.load(kb + (int64_t)(k0 + KB) * D, D, tid);
      sV.load(vtb + k0 + KB, Lk, tid);
    }
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks)
        s[kt] = mfma16(*reinterpret_cast<const bf16x8*>(&Ks[(kt * 16 + l16) * KP + ks * 32 + g * 8]),
                       qf[ks], s[kt]);
    }
    // s[kt][e] = score of query qi and key k0 + 16 kt + 4 g + e
    float mx = m;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, s[kt][e] * sl2);
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float alpha = exp2f(m - mx);
    m = mx;
    float p[4][4];
    float ps = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        p[kt][e] = exp2f(fmaf(s[kt][e], sl2, -mx));
        ps += p[kt][e];
      }
    lsum = fmaf(lsum, alpha, ps);
#pragma unroll
    for (int i = 0; i < DV / 16; ++i) acc[i] *= alpha;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16x8 pb = pack8(p[2 * h], p[2 * h + 1]);
#pragma unroll
      for (int i = 0; i < DV / 16; ++i)
        acc[i] = mfma16(read_a_split(&Vt[(i * 16 + l16) * VP + h * 32], g), pb, acc[i]);
    }
  }
  lsum += __shfl_xor(lsum, 16);
  lsum += __shfl_xor(lsum, 32);
  if (opart) {  // split: unnormalised partial output + (max, sum) of this key range
    const int64_t row = ((int64_t)sp * gridDim.z + b) * Lq + qi;
    float* prow = opart + row * DV;
#pragma unroll
    for (int i = 0; i < DV / 16; ++i)
      *reinterpret_cast<f32x4*>(prow + i * 16 + g * 4) = acc[i];
    if (g == 0) {
      mpart[row] = m;
      lpart[row] = lsum;
    }
    return;
  }
  const float inv = 1.f / lsum;
  __bf16* orow = o + ((int64_t)b * Lq + qi) * DV;
#pragma unroll
  for (int i = 0; i < DV / 16; ++i) {
    bf16x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (__bf16)(acc[i][e] * inv);
    *reinterpret_cast<bf16x4*>(orow + i * 16 + g * 4) = w;
  }
  if (g == 0) lse2[(int64_t)b * Lq + qi] = m + log2f(lsum);
}

// merge NS key splits: M = max m_s, L = sum l_s 2^(m_s - M), O = sum O_s 2^(m_s - M) / L;
// one wave per query row
__global__ __launch_bounds__(256) void attn_fwd_combine(
    const float* __restrict__ opart, const float* __restrict__ mpart,
    const float* __restrict__ lpart, __bf16* __restrict__ o, float* __restrict__ lse2, int NS,
    int64_t rows, int DV) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float M = kNegBig;
  for (int s = 0; s < NS; ++s) M = fmaxf(M, mpart[s * rows + row]);
  float L = 0.f;
  for (int s = 0; s < NS; ++s) L += lpart[s * rows + row] * exp2f(mpart[s * rows + row] - M);
  const float inv = 1.f / L;
  for (int c = lane; c < DV; c += 64) {
    float acc = 0.f;
    for (int s = 0; s < NS; ++s)
      acc += opart[(s * rows + row) * DV + c] * exp2f(mpart[s * rows + row] - M);
    o[row * DV + c] = (__bf16)(acc * inv);
  }
  if (lane == 0) lse2[row] = M + log2f(L);
}

// out[i] = bf16(sum_s part[s * n + i]) (the split backward's fp32 partial gradients)
__global__ __launch_bounds__(256) void attn_sum_splits(const float* __restrict__ part,
                                                       __bf16* __restrict__ out, int NS,
                                                       int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  for (int s = 0; s < NS; ++s) acc += part[s * n + i];
  out[i] = (__bf16)acc;
}

// ---- backward: dK, dV ----------------------------------------------------------------------
// workgroup: 64 keys (wave w: keys 16w..16w+15, held in registers as B operands) x all queries
// in blocks of 32 staged in LDS both row-major (A operands of S, dP) and transposed (A operands
// of dV^T, dK^T). S = Q K^T and dP = dO V^T put the key in the lane's column, so P and dS feed
// dV^T += dO^T P and dK^T += Q^T dS as B operands.
// WDS: dS^T [B][Lk][Lq] bf16 is written to dst as well (a variant of its own: the stores cost
// registers the other path should not pay for), and dQ = dS K is then one GEMM
// instead of the dQ kernel (which recomputes S and dP): 288 GB of HBM holds the B x Lq x Lk
// matrix at the few-shot shapes (3.2 GB at 3 x 16384 x 32768).
// PFO: the dO / dO^T tiles are prefetched too (else loaded after the barrier, as the Q tiles
// used to be): at D = 128, DV = 288 with 8 waves the full prefetch exceeds 256 VGPRs
template <int D, int DV, int NW, bool PFO, bool WDS>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dkv_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v,
    const __bf16* __restrict__ dout, const __bf16* __restrict__ qt,
    const __bf16* __restrict__ dott, const float* __restrict__ lse2,
    const float* __restrict__ dsum, __bf16* __restrict__ dk, __bf16* __restrict__ dv, int Lq,
    int Lk, float sl2, float scale, int qlen, float* __restrict__ dkpart,
    float* __restrict__ dvpart, __bf16* __restrict__ dst) {
  constexpr int QB = 32, QP = D + 8, OP = DV + 8, TP = QB + 8;
  __shared__ __attribute__((aligned(16))) __bf16 Qs[QB * QP];
  __shared__ __attribute__((aligned(16))) __bf16 Qt[D * TP];
  __shared__ __attribute__((aligned(16))) __bf16 Os[QB * OP];
  __shared__ __attribute__((aligned(16))) __bf16 Ot[DV * TP];
  __shared__ __attribute__((aligned(16))) float Ls[QB];
  __shared__ __attribute__((aligned(16))) float Ds[QB];
  const int b = blockIdx.z, sp = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int ki = blockIdx.x * (NW * 16) + wid * 16 + l16;  // this lane's key (B/C column)
  const __bf16* qb = q + (int64_t)b * Lq * D;
  const __bf16* ob = dout + (int64_t)b * Lq * DV;
  const __bf16* qtb = qt + (int64_t)b * D * Lq;
  const __bf16* otb = dott + (int64_t)b * DV * Lq;
  bf16x8 kf[D / 32], vf[DV / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
    kf[ks] = *reinterpret_cast<const bf16x8*>(k + ((int64_t)b * Lk + ki) * D + ks * 32 + g * 8);
#pragma unroll
  for (int ks = 0; ks < DV / 32; ++ks)
    vf[ks] = *reinterpret_cast<const bf16x8*>(v + ((int64_t)b * Lk + ki) * DV + ks * 32 + g * 8);
  f32x4 dkt[D / 16], dvt[DV / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) dkt[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < DV / 16; ++i) dvt[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qbeg = sp * qlen, qend = min(Lq, (sp + 1) * qlen);
  TileStage<QB, D, QP, NW * 64> sQ;
  TileStage<D, QB, TP, NW * 64> sQt;   // Q^T rows (host-transposed copy)
  TileStage<QB, DV, OP, NW * 64> sO;
  TileStage<DV, QB, TP, NW * 64> sOt;  // dO^T rows
  float lsv = 0.f, dsv = 0.f;
  auto prefetch = [&](int q0) {
    sQ.load(qb + (int64_t)q0 * D, D, tid);
    sQt.load(qtb + q0, Lq, tid);
    if constexpr (PFO) {
      sO.load(ob + (int64_t)q0 * DV, DV, tid);
      sOt.load(otb + q0, Lq, tid);
    }
    if (tid < QB) {
      lsv = lse2[(int64_t)b * Lq + q0 + tid];
      dsv = dsum[(int64_t)b * Lq + q0 + tid];
    }
  };
  if (qbeg < qend) prefetch(qbeg);
  for (int q0 = qbeg; q0 < qend; q0 += QB) {
    __syncthreads();
    sQ.store(Qs, tid);
    sQt.store(Qt, tid);
    if constexpr (!PFO) {
      sO.load(ob + (int64_t)q0 * DV, DV, tid);
      sOt.load(otb + q0, Lq, tid);
    }
    sO.store(Os, tid);
    sOt.store(Ot, tid);
    if (tid < QB) {
      Ls[tid] = lsv;
      Ds[tid] = dsv;
    }
    __syncthreads();
    if (q0 + QB < qend) prefetch(q0 + QB);  // in flight during this block's MFMAs
    float p[2][4], ds[2][4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks)
        s = mfma16(*reinterpret_cast<const bf16x8*>(&Qs[(qt * 16 + l16) * QP + ks * 32 + g * 8]),
                   kf[ks], s);
#pragma unroll
      for (int ks = 0; ks < DV / 32; ++ks)
        dp = mfma16(*reinterpret_cast<const bf16x8*>(&Os[(qt * 16 + l16) * OP + ks * 32 + g * 8]),
                    vf[ks], dp);
      // s[e], dp[e]: query q0 + 16 qt + 4 g + e, key ki
      const f32x4 lq = *reinterpret_cast<const f32x4*>(&Ls[qt * 16 + g * 4]);
      const f32x4 dq = *reinterpret_cast<const f32x4*>(&Ds[qt * 16 + g * 4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        p[qt][e] = exp2f(fmaf(s[e], sl2, -lq[e]));
        ds[qt][e] = p[qt][e] * (dp[e] - dq[e]) * scale;
      }
    }
    const bf16x8 pb = pack8(p[0], p[1]), dsb = pack8(ds[0], ds[1]);
    if constexpr (WDS) {  // dS^T row of this lane's key: queries q0 + 4g + e, q0 + 16 + 4g + e
      __bf16* row = dst + ((int64_t)b * Lk + ki) * Lq + q0 + g * 4;
      bf16x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lo[e] = dsb[e];
        hi[e] = dsb[4 + e];
      }
      *reinterpret_cast<bf16x4*>(row) = lo;
      *reinterpret_cast<bf16x4*>(row + 16) = hi;
    }
#pragma unroll
    for (int i = 0; i < DV / 16; ++i)
      dvt[i] = mfma16(read_a_split(&Ot[(i * 16 + l16) * TP], g), pb, dvt[i]);
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      dkt[i] = mfma16(read_a_split(&Qt[(i * 16 + l16) * TP], g), dsb, dkt[i]);
  }
  if (dkpart) {  // query split: fp32 partial gradients, summed by attn_sum_splits
    const int64_t row = ((int64_t)sp * gridDim.z + b) * Lk + ki;
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      *reinterpret_cast<f32x4*>(dkpart + row * D + i * 16 + g * 4) = dkt[i];
#pragma unroll
    for (int i = 0; i < DV / 16; ++i)
      *reinterpret_cast<f32x4*>(dvpart + row * DV + i * 16 + g * 4) = dvt[i];
    return;
  }
  __bf16* dkr = dk + ((int64_t)b * Lk + ki) * D;
  __bf16* dvr = dv + ((int64_t)b * Lk + ki) * DV;
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    bf16x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (__bf16)dkt[i][e];
    *reinterpret_cast<bf16x4*>(dkr + i * 16 + g * 4) = w;
  }
#pragma unroll
  for (int i = 0; i < DV / 16; ++i) {
    bf16x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (__bf16)dvt[i][e];
    *reinterpret_cast<bf16x4*>(dvr + i * 16 + g * 4) = w;
  }
}

// ---- backward: dQ --------------------------------------------------------------------------
// workgroup: 64 queries (registers: Q and dO rows as B operands) x all keys in blocks of 32
// (K row-major and transposed, V row-major in LDS). S^T = K Q^T and dP^T = V dO^T put the query
// in the lane's column; dQ^T += K^T dS^T.
template <int D, int DV, int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dq_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v,
    const __bf16* __restrict__ dout, const __bf16* __restrict__ kt,
    const float* __restrict__ lse2, const float* __restrict__ dsum, __bf16* __restrict__ dq,
    int Lq, int Lk, float sl2,
    float scale, int klen, float* __restrict__ dqpart) {
  constexpr int KB = 32, KP = D + 8, VP = DV + 8, TP = KB + 8;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[KB * KP];
  __shared__ __attribute__((aligned(16))) __bf16 Kt[D * TP];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[KB * VP];
  const int b = blockIdx.z, sp = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int qi = blockIdx.x * (NW * 16) + wid * 16 + l16;
  const __bf16* kb = k + (int64_t)b * Lk * D;
  const __bf16* vb = v + (int64_t)b * Lk * DV;
  const __bf16* ktb = kt + (int64_t)b * D * Lk;
  bf16x8 qf[D / 32], of[DV / 32];
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8*>(q + ((int64_t)b * Lq + qi) * D + ks * 32 + g * 8);
#pragma unroll
  for (int ks = 0; ks < DV / 32; ++ks)
    of[ks] = *reinterpret_cast<const bf16x8*>(dout + ((int64_t)b * Lq + qi) * DV + ks * 32 + g * 8);
  const float lq = lse2[(int64_t)b * Lq + qi], dq0 = dsum[(int64_t)b * Lq + qi];
  f32x4 acc[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kbeg = sp * klen, kend = min(Lk, (sp + 1) * klen);
  TileStage<KB, D, KP, NW * 64> sK;
  TileStage<D, KB, TP, NW * 64> sKt;  // K^T rows (host-transposed copy)
  TileStage<KB, DV, VP, NW * 64> sV;
  auto prefetch = [&](int k0) {
    sK.load(kb + (int64_t)k0 * D, D, tid);
    sKt.load(ktb + k0, Lk, tid);
    sV.load(vb + (int64_t)k0 * DV, DV, tid);
  };
  if (kbeg < kend) prefetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += KB) {
    __syncthreads();
    sK.store(Ks, tid);
    sKt.store(Kt, tid);
    sV.store(Vs, tid);
    __syncthreads();
    if (k0 + KB < kend) prefetch(k0 + KB);  // in flight during this block's MFMAs
    float ds[2][4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks)
        s = mfma16(*reinterpret_cast<const bf16x8*>(&Ks[(kt * 16 + l16) * KP + ks * 32 + g * 8]),
                   qf[ks], s);
#pragma unroll
      for (int ks = 0; ks < DV / 32; ++ks)
        dp = mfma16(*reinterpret_cast<const bf16x8*>(&Vs[(kt * 16 + l16) * VP + ks * 32 + g * 8]),
                    of[ks], dp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pe = exp2f(fmaf(s[e], sl2, -lq));
        ds[kt][e] = pe * (dp[e] - dq0) * scale;
      }
    }
    const bf16x8 dsb = pack8(ds[0], ds[1]);
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      acc[i] = mfma16(read_a_split(&Kt[(i * 16 + l16) * TP], g), dsb, acc[i]);
  }
  if (dqpart) {  // key split: fp32 partial dQ, summed by attn_sum_splits
    const int64_t row = ((int64_t)sp * gridDim.z + b) * Lq + qi;
#pragma unroll
    for (int i = 0; i < D / 16; ++i)
      *reinterpret_cast<f32x4*>(dqpart + row * D + i * 16 + g * 4) = acc[i];
    return;
  }
  __bf16* dqr = dq + ((int64_t)b * Lq + qi) * D;
#pragma unroll
  for (int i = 0; i < D / 16; ++i) {
    bf16x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = (__bf16)acc[i][e];
    *reinterpret_cast<bf16x4*>(dqr + i * 16 + g * 4) = w;
  }
}

void check_attn(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  IAMD_CHECK(q.is_cuda() && q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 &&
                 v.scalar_type() == at::kBFloat16,
             "fused_attention: bf16 CUDA tensors expected");
  IAMD_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3 && q.is_contiguous() &&
                 k.is_contiguous() && v.is_contiguous(),
             "fused_attention: contiguous [B, L, D] tensors expected");
  IAMD_CHECK(q.size(0) == k.size(0) && k.size(0) == v.size(0) && q.size(2) == k.size(2) &&
                 k.size(1) == v.size(1),
             "fused_attention: shape mismatch");
  const int64_t d = q.size(2), dvv = v.size(2);
  IAMD_CHECK(d == 32 || d == 64 || d == 128, "fused_attention: head dim must be 32, 64 or 128");
  IAMD_CHECK(dvv % 32 == 0 && dvv >= 32 && dvv <= 288 && dvv != 224,
             "fused_attention: value dim must be 32..256 in steps of 32 (not 224), or 288");
  IAMD_CHECK(q.size(1) % 64 == 0 && k.size(1) % 64 == 0 && q.size(1) > 0 && k.size(1) > 0,
             "fused_attention: sequence lengths must be multiples of 64");
  IAMD_CHECK(q.size(0) < 65536, "fused_attention: batch too large");
  IAMD_CHECK(q.size(0) * q.size(1) * std::max<int64_t>(v.size(2), q.size(2)) * 32 < (1ll << 40),
             "fused_attention: too large");
}

// (D, DV) dispatch onto the launcher template FN<D, DV>(args...)
#define IAMD_ATTN_CASES(FN, DD, ...)                              \
  switch (dvv) {                                                  \
    case 32: FN<DD, 32>(__VA_ARGS__); break;                      \
    case 64: FN<DD, 64>(__VA_ARGS__); break;                      \
    case 96: FN<DD, 96>(__VA_ARGS__); break;                      \
    case 128: FN<DD, 128>(__VA_ARGS__); break;                    \
    case 160: FN<DD, 160>(__VA_ARGS__); break;                    \
    case 192: FN<DD, 192>(__VA_ARGS__); break;                    \
    case 256: FN<DD, 256>(__VA_ARGS__); break;                    \
    case 288: FN<DD, 288>(__VA_ARGS__); break;                    \
    default: IAMD_CHECK(false, "fused_attention: value dim");     \
  }
#define IAMD_ATTN_DISPATCH(FN, ...)            \
  if (d == 32) {                               \
    IAMD_ATTN_CASES(FN, 32, __VA_ARGS__)       \
  } else if (d == 64) {                        \
    IAMD_ATTN_CASES(FN, 64, __VA_ARGS__)       \
  } else {                                     \
    IAMD_ATTN_CASES(FN, 128, __VA_ARGS__)      \
  }

inline const __bf16* bp(const at::Tensor& t) {
  return reinterpret_cast<const __bf16*>(t.data_ptr());
}
inline __bf16* bpm(at::Tensor& t) { return reinterpret_cast<__bf16*>(t.data_ptr()); }

// key / query splits so a launch has >= ~2 workgroups per CU: NS divides the sequence into
// chunks of whole 64-row blocks
// dsum[r] = sum_j dout[r, j] * out[r, j] in fp32: one wave per row, four rows per block
__global__ __launch_bounds__(256) void attn_dsum_kernel(const __hip_bfloat16* __restrict__ dout,
                                                        const __hip_bfloat16* __restrict__ out,
                                                        float* __restrict__ dsum, int64_t rows,
                                                        int dv) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const __hip_bfloat16* a = dout + r * dv;
  const __hip_bfloat16* b = out + r * dv;
  float acc = 0.f;
  for (int j = lane; j < dv; j += 64) acc += __bfloat162float(a[j]) * __bfloat162float(b[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) dsum[r] = acc;
}

inline int pick_splits(int64_t tiles, int64_t len) {
  const int64_t want = (512 + tiles - 1) / tiles;
  const int64_t maxs = len / 64;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, std::min<int64_t>(maxs, 32)));
}
inline int split_len(int64_t len, int ns) { return (int)((len / 64 + ns - 1) / ns * 64); }

// 8 waves per workgroup (128 rows sharing each staged tile: half the LDS staging per MFMA)
// when the rows tile by 128 and that still leaves >= 256 workgroups, else 4 (at the few-shot
// recipe shape the 384-workgroup 8-wave forward is 1.38x the 768-workgroup 4-wave one:
// scripts/probe/attn_wave_ab.py)
inline int pick_waves(int64_t rows, int64_t other) {
  // IMAGINAIRE_AMD_ATTN_MIN_WG: the smallest 8-wave grid taken (read per call, A/B)
  const char* e = std::getenv("IMAGINAIRE_AMD_ATTN_MIN_WG");
  const int64_t min_wg = e ? std::atoll(e) : 256;
  return (rows % 128 == 0 && other * (rows / 128) >= min_wg) ? 8 : 4;
}
// per-kernel override of that threshold for the backward passes (read per call, A/B):
// IMAGINAIRE_AMD_ATTN_DKV_MIN_WG / IMAGINAIRE_AMD_ATTN_DQ_MIN_WG
inline int pick_waves_bwd(int64_t rows, int64_t other, const char* var) {
  const char* e = std::getenv(var);
  if (e == nullptr) return pick_waves(rows, other);
  return (rows % 128 == 0 && other * (rows / 128) >= std::atoll(e)) ? 8 : 4;
}

template <int D, int DV>
void launch_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out,
                at::Tensor& lse, float sl2) {
  const int64_t B = q.size(0), Lq = q.size(1), Lk = k.size(1);
  const int nw = pick_waves(Lq, B);
  int ns = pick_splits(B * (Lq / (nw * 16)), Lk);
  const int klen = split_len(Lk, ns);
  ns = (int)((Lk + klen - 1) / klen);
  at::Tensor opart, mpart, lpart;
  float *op = nullptr, *mp = nullptr, *lp = nullptr;
  if (ns > 1) {
    auto fo = q.options().dtype(at::kFloat);
    opart = at::empty({ns, B, Lq, (int64_t)DV}, fo);
    mpart = at::empty({ns, B, Lq}, fo);
    lpart = at::empty({ns, B, Lq}, fo);
    op = opart.data_ptr<float>();
    mp = mpart.data_ptr<float>();
    lp = lpart.data_ptr<float>();
  }
  const at::Tensor vt = v.transpose(1, 2).contiguous();  // [B, DV, Lk]
  const dim3 grid((unsigned)(Lq / (nw * 16)), (unsigned)ns, (unsigned)B);
  if (nw == 8)
    hipLaunchKernelGGL((attn_fwd_kernel<D, DV, 8>), grid, dim3(512), 0, stream(), bp(q), bp(k),
                       bp(vt), bpm(out), lse.data_ptr<float>(), (int)Lq, (int)Lk, sl2, klen, op,
                       mp, lp);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<D, DV, 4>), grid, dim3(256), 0, stream(), bp(q), bp(k),
                       bp(vt), bpm(out), lse.data_ptr<float>(), (int)Lq, (int)Lk, sl2, klen, op,
                       mp, lp);
  if (ns > 1)
    hipLaunchKernelGGL(attn_fwd_combine, dim3((unsigned)((B * Lq + 3) / 4)), dim3(256), 0,
                       stream(), op, mp, lp, bpm(out), lse.data_ptr<float>(), ns, B * Lq, DV);
}

template <int D, int DV>
void launch_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                const at::Tensor& dout, const at::Tensor& lse, const at::Tensor& dsum,
                at::Tensor& dq, at::Tensor& dk, at::Tensor& dv, float sl2, float sc) {
  const int64_t B = q.size(0), Lq = q.size(1), Lk = k.size(1);
  auto fo = q.options().dtype(at::kFloat);
  // dK / dV: key tiles x query splits
  const int nwk = pick_waves_bwd(Lk, B, "IMAGINAIRE_AMD_ATTN_DKV_MIN_WG");
  int nq = pick_splits(B * (Lk / (nwk * 16)), Lq);
  const int qlen = split_len(Lq, nq);
  nq = (int)((Lq + qlen - 1) / qlen);
  at::Tensor dkp, dvp;
  if (nq > 1) {
    dkp = at::empty({nq, B, Lk, (int64_t)D}, fo);
    dvp = at::empty({nq, B, Lk, (int64_t)DV}, fo);
  }
  const at::Tensor qt = q.transpose(1, 2).contiguous(), dott = dout.transpose(1, 2).contiguous();
  // IMAGINAIRE_AMD_ATTN_DQ_GEMM: dQ from a stored dS^T by one GEMM (1, default) or by the dQ
  // kernel (0); IMAGINAIRE_AMD_ATTN_DS_MAX_GB caps the dS^T workspace (default 16 GB)
  const char* dq_gemm_var = std::getenv("IMAGINAIRE_AMD_ATTN_DQ_GEMM");  // read per call (A/B)
  const bool dq_gemm_env = dq_gemm_var == nullptr || std::atoi(dq_gemm_var) != 0;
  static const double ds_max_gb = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_ATTN_DS_MAX_GB");
    return e == nullptr ? 16.0 : std::atof(e);
  }();
  const bool dq_gemm = dq_gemm_env && (double)B * Lq * Lk * 2 <= ds_max_gb * 1e9;
  at::Tensor dsT;
  if (dq_gemm) dsT = at::empty({B, Lk, Lq}, q.options());
  __bf16* dstp = dq_gemm ? bpm(dsT) : nullptr;
  {
    const dim3 grid((unsigned)(Lk / (nwk * 16)), (unsigned)nq, (unsigned)B);
    float* dkpp = nq > 1 ? dkp.data_ptr<float>() : nullptr;
    float* dvpp = nq > 1 ? dvp.data_ptr<float>() : nullptr;
    // IMAGINAIRE_AMD_ATTN_PF_O: prefetch the dO tiles of the 8-wave dK / dV kernel too
    // (1) or not (0; default for the widest heads, where it would spill)
    static const int pfo_env = [] {
      const char* e = std::getenv("IMAGINAIRE_AMD_ATTN_PF_O");
      return e == nullptr ? -1 : std::atoi(e);
    }();
    const bool pfo = pfo_env < 0 ? !(D == 128 && DV > 256) : pfo_env != 0;
    auto launch = [&](auto wds) {
      constexpr bool W = decltype(wds)::value;
      if (nwk == 8 && pfo)
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, DV, 8, true, W>), grid, dim3(512), 0, stream(),
                           bp(q), bp(k), bp(v), bp(dout), bp(qt), bp(dott), lse.data_ptr<float>(),
                           dsum.data_ptr<float>(), bpm(dk), bpm(dv), (int)Lq, (int)Lk, sl2, sc,
                           qlen, dkpp, dvpp, dstp);
      else if (nwk == 8)
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, DV, 8, false, W>), grid, dim3(512), 0, stream(),
                           bp(q), bp(k), bp(v), bp(dout), bp(qt), bp(dott), lse.data_ptr<float>(),
                           dsum.data_ptr<float>(), bpm(dk), bpm(dv), (int)Lq, (int)Lk, sl2, sc,
                           qlen, dkpp, dvpp, dstp);
      else
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, DV, 4, true, W>), grid, dim3(256), 0, stream(),
                           bp(q), bp(k), bp(v), bp(dout), bp(qt), bp(dott), lse.data_ptr<float>(),
                           dsum.data_ptr<float>(), bpm(dk), bpm(dv), (int)Lq, (int)Lk, sl2, sc,
                           qlen, dkpp, dvpp, dstp);
    };
    if (dq_gemm)
      launch(std::true_type{});
    else
      launch(std::false_type{});
  }
  if (nq > 1) {
    const int64_t nk = B * Lk * D, nv = B * Lk * DV;
    hipLaunchKernelGGL(attn_sum_splits, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0,
                       stream(), dkp.data_ptr<float>(), bpm(dk), nq, nk);
    hipLaunchKernelGGL(attn_sum_splits, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0,
                       stream(), dvp.data_ptr<float>(), bpm(dv), nq, nv);
  }
  if (dq_gemm) {  // dQ = dS K = (dS^T)^T K, fp32 accumulation in the GEMM
    at::bmm_out(dq, dsT.transpose(1, 2), k);
    return;
  }
  // dQ: query tiles x key splits
  const int nwq = pick_waves_bwd(Lq, B, "IMAGINAIRE_AMD_ATTN_DQ_MIN_WG");
  int nk2 = pick_splits(B * (Lq / (nwq * 16)), Lk);
  const int klen = split_len(Lk, nk2);
  nk2 = (int)((Lk + klen - 1) / klen);
  at::Tensor dqp;
  if (nk2 > 1) dqp = at::empty({nk2, B, Lq, (int64_t)D}, fo);
  const at::Tensor kt = k.transpose(1, 2).contiguous();
  {
    const dim3 grid((unsigned)(Lq / (nwq * 16)), (unsigned)nk2, (unsigned)B);
    float* dqpp = nk2 > 1 ? dqp.data_ptr<float>() : nullptr;
    if (nwq == 8)
      hipLaunchKernelGGL((attn_bwd_dq_kernel<D, DV, 8>), grid, dim3(512), 0, stream(), bp(q),
                         bp(k), bp(v), bp(dout), bp(kt), lse.data_ptr<float>(),
                         dsum.data_ptr<float>(), bpm(dq), (int)Lq, (int)Lk, sl2, sc, klen, dqpp);
    else
      hipLaunchKernelGGL((attn_bwd_dq_kernel<D, DV, 4>), grid, dim3(256), 0, stream(), bp(q),
                         bp(k), bp(v), bp(dout), bp(kt), lse.data_ptr<float>(),
                         dsum.data_ptr<float>(), bpm(dq), (int)Lq, (int)Lk, sl2, sc, klen, dqpp);
  }
  if (nk2 > 1) {
    const int64_t n = B * Lq * D;
    hipLaunchKernelGGL(attn_sum_splits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       stream(), dqp.data_ptr<float>(), bpm(dq), nk2, n);
  }
}

}  // namespace

// returns (out [B, Lq, DV] bf16, lse2 [B, Lq] fp32: log2-domain log-sum-exp of the scaled scores)
std::vector<at::Tensor> attention_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                      double scale) {
  check_attn(q, k, v);
  const int64_t B = q.size(0), Lq = q.size(1);
  auto out = at::empty({B, Lq, v.size(2)}, q.options());
  auto lse = at::empty({B, Lq}, q.options().dtype(at::kFloat));
  const float sl2 = (float)(scale * 1.4426950408889634);
  const int64_t d = q.size(2), dvv = v.size(2);
  IAMD_ATTN_DISPATCH(launch_fwd, q, k, v, out, lse, sl2)
  IAMD_LAUNCH_CHECK();
  return {out, lse};
}

// returns (dq, dk, dv), bf16; dsum = rowsum(dout * out) in fp32 is computed here
std::vector<at::Tensor> attention_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                      const at::Tensor& out, const at::Tensor& lse,
                                      const at::Tensor& dout_in, double scale) {
  check_attn(q, k, v);
  const int64_t B = q.size(0), Lq = q.size(1);
  const at::Tensor dout = dout_in.to(at::kBFloat16).contiguous();
  IAMD_CHECK(dout.sizes() == out.sizes() && lse.scalar_type() == at::kFloat &&
                 lse.numel() == B * Lq && lse.is_contiguous(),
             "attention_bwd: out / dout / lse shapes");
  IAMD_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous(),
             "attention_bwd: out must be contiguous bf16");
  const int64_t rows = B * Lq;
  const int dvv0 = (int)out.size(2);
  auto dsum = at::empty({B, Lq}, q.options().dtype(at::kFloat));
  hipLaunchKernelGGL(attn_dsum_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(dout.data_ptr()),
                     reinterpret_cast<const __hip_bfloat16*>(out.data_ptr()),
                     dsum.data_ptr<float>(), rows, dvv0);
  auto dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  const float sl2 = (float)(scale * 1.4426950408889634), sc = (float)scale;
  const int64_t d = q.size(2), dvv = v.size(2);
  IAMD_ATTN_DISPATCH(launch_bwd, q, k, v, dout, lse, dsum, dq, dk, dv, sl2, sc)
  IAMD_LAUNCH_CHECK();
  return {dq, dk, dv};
}

}  // namespace iamd
