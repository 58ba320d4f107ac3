// k10: implicit-GEMM convolution on the gfx950 matrix cores (NHWC, bf16 in, fp32 accumulate).
//
// Replaces the MIOpen forward (and, through a flipped/transposed weight, the stride-1 data
// gradient) of the convolutions that dominate a SPADE/pix2pixHD/vid2vid step: 3x3 / 5x5 /
// 4x4-stride-2 convs with 64..4096 channels at up to 256x512 (reference layers/conv.py:59-91
// runs these through cuDNN; the reference has no hand-written conv).
//
// GEMM view: rows m = output pixels (b, oh, ow), columns n = output channels,
// k = (ky, kx, ci) with ci fastest. Both operands are K-contiguous in memory:
//   A[m][k] = x[b][oh*sh - ph + ky*dh][ow*sw - pw + kx*dw][ci]   (NHWC activation)
//   B[n][k] = w[n][ky][kx][ci]                                    (OHWI = channels-last weight)
// so a 64-deep k-step is one filter tap and 64 consecutive input channels (Cin % 64 == 0;
// the Python wrapper zero-pads odd channel counts such as 185-channel label maps).
//
// Block tile BM (128 / 256 pixels) x BN (64 / 128 channels) x 64 (k), BM/32 wave64s in a
// (BM/64) x 2 grid, each wave owning a 64 x BN/2 sub-tile of v_mfma_f32_16x16x32_bf16
// accumulators.
// Staging: global -> LDS with buffer_load_dwordx4 ... lds (no VGPR round trip), two LDS buffers,
// one barrier per k-step; the load of step k+1 is in flight while step k runs on the MFMAs.
// Padding pixels (outside the image) and the pixel tail get an out-of-range buffer offset and
// the buffer unit returns zeros (no branch, no zero page); per-row tap-validity bit masks and
// SGPR-resident tap/k-step offsets keep the per-load VALU work to a select and an add.
// LDS rows are 128 B; the 16-B chunk index is XOR-swizzled with (row & 7) on the global side (the LDS write of a DMA is lane-linear), which makes the ds_read_b128 fragment
// reads bank-conflict free. Epilogue: + bias, leaky/relu slope, bf16, staged through LDS so
// every global store is a 16-byte row segment. Block ids are XCD-remapped so the BN-tiles
// that share one pixel tile run on the same XCD (shared L2 for the activation halo).
#include "conv_common.h"

#include <cstdlib>

namespace iamd {
namespace {

// BM = 128 (4 waves, 2 blocks/CU) or 256 (8 waves, 1 block/CU: the B tile is shared by twice
// the pixels, 25% fewer L2->LDS bytes per MFMA); waves form a (BM/64) x 2 grid.
// VAR (main-loop schedule experiment, IMAGINAIRE_AMD_CONV_VAR): 0 = per-32-k fragment reads
// then MFMAs; 1 = same with s_setprio(1) around the MFMA cluster; 2 = all 64-k fragments read
// up front, then 32 back-to-back MFMAs under s_setprio(1).
// The v1 body: tile bid (already XCD-remapped) of split `split` of sample zb (of nz).
template <int BM, int BN, bool HAS_BIAS, int VAR>
__device__ __forceinline__ void conv_v1_impl(const ConvArgs& a, int bid, int split, int zb,
                                             int nz) {
  // The buffer-resource builtins have no host form; the host pass only needs the launch stub.
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int kThreads = BM * 2;
  constexpr int NI = BN / 32;                 // 16-wide n-fragments per wave
  constexpr int kAbytes = BM * kRowBytes;     // 16 / 32 KB
  constexpr int kBbytes = BN * kRowBytes;     // 8 / 16 KB
  constexpr int kStage = kAbytes + kBbytes;
  constexpr int RS = kThreads / 8;            // staged rows per DMA round
  constexpr int kLoadBytes = kThreads * 16;   // LDS bytes per DMA round
  constexpr int kBLoads = BN / RS;            // DMA rounds for the B tile
  __shared__ __attribute__((aligned(16))) char smem[2 * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: the DMA's LDS base (M0)
  const int wm = wid >> 1, wn = wid & 1;
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;

  // ---- per-thread DMA sources: rows lrow + RS i, chunk csw (swizzled) -------------------
  // Buffer-resource loads straight into LDS: the per-lane 32-bit byte offset selects the
  // pixel row, the wave-uniform parts (tap, channel block, k-step) ride in SGPRs, and an
  // out-of-range offset (padding pixels, M tail) returns zeros from the buffer unit itself.
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x + (size_t)zb * a.xbs), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w + (size_t)zb * a.wbs), 0, a.wbytes, kBufCfg);
  const int lrow = tid >> 3;
  const int csw = (tid & 7) ^ (lrow & 7);
  const int HoWo = a.Ho * a.Wo;
  int a_off[4];
  uint64_t a_tmask[4];  // bit (ky * KW + kx) set when that filter tap reads inside the image
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + lrow + RS * i;
    a_off[i] = 0;
    a_tmask[i] = 0;
    if (m < a.M) {
      const int b = m / HoWo, r = m - b * HoWo;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
      a_off[i] = (((b * a.H + ih0) * a.W + iw0) * a.Cin + csw * 8) * 2;
      for (int ky = 0; ky < a.KH; ++ky) {
        if ((unsigned)(ih0 + ky * a.dh) >= (unsigned)a.H) continue;
        for (int kx = 0; kx < a.KW; ++kx)
          if ((unsigned)(iw0 + kx * a.dw) < (unsigned)a.W)
            a_tmask[i] |= 1ull << (ky * a.KW + kx);
      }
    }
  }
  const int wrow_bytes = a.nk * kBK * 2;  // = KH*KW*Cin*2
  int b_off[kBLoads];
#pragma unroll
  for (int i = 0; i < kBLoads; ++i) b_off[i] = (n0 + lrow + RS * i) * wrow_bytes + csw * 16;

  // scalar (tap, channel block) cursor of the next k-step to stage, advanced incrementally
  // (a division per k-step costs ~2 SALU per MFMA: profiles/pmc_conv_r2_mi355x.txt)
  const int ks0 = split * a.kps;
  const int ks1 = min(a.nk, ks0 + a.kps);
  int cky, ckx, cc, ctap;
  {
    ctap = ks0 / a.cpt;
    cc = (ks0 - ctap * a.cpt) * kBK;
    cky = ctap / a.KW;
    ckx = ctap - cky * a.KW;
  }
  const int row_step = a.dh * a.W * a.Cin * 2, col_step = a.dw * a.Cin * 2;
  int ctoff = cky * row_step + ckx * col_step + cc * 2;
  auto issue = [&](int ks, int buf) {
    char* As = smem + buf * kStage;
    char* Bs = As + kAbytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (a_tmask[i] >> ctap) & 1u;
      const int voff = ok ? a_off[i] + ctoff : kOobOffset;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(As + i * kLoadBytes + wid * 1024),
                                               16, voff, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kBLoads; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(Bs + i * kLoadBytes + wid * 1024),
                                               16, b_off[i], ks * kBK * 2, 0, 0);
    cc += kBK;
    ctoff += kBK * 2;
    if (cc == a.Cin) {
      cc = 0;
      ++ctap;
      if (++ckx == a.KW) {
        ckx = 0;
        ++cky;
      }
      ctoff = cky * row_step + ckx * col_step;
    }
  };

  f32x4 acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (row & 7 == lane & 7 for every fragment row of this lane)
  const int frow = lane & 15, fsw = lane & 7, fk = lane >> 4;
  // unrolled over the two LDS buffers (b = 0, 1): the fragment addresses are loop-invariant
  // registers plus immediate offsets
  auto kstep = [&](int ks, int b) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ks + 1 < ks1) issue(ks + 1, b ^ 1);
    const char* As = smem + b * kStage;
    const char* Bs = As + kAbytes;
    if constexpr (VAR == 2) {
      bf16x8 af[2][4], bfr[2][NI];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[kk][i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + frow) * kRowBytes + coff);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          bfr[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * (BN / 2) + j * 16 + frow) * kRowBytes + coff);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int coff = ((kk * 4 + fk) ^ fsw) << 4;
        bf16x8 af[4], bfr[NI];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + frow) * kRowBytes + coff);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * (BN / 2) + j * 16 + frow) * kRowBytes + coff);
        if constexpr (VAR == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (VAR == 1) __builtin_amdgcn_s_setprio(0);
      }
    }
  };
  issue(ks0, 0);
  for (int ks = ks0; ks < ks1; ks += 2) {
    kstep(ks, 0);
    if (ks + 1 < ks1) kstep(ks + 1, 1);
  }

  if (a.part) {  // split-K: raw fp32 partials [S][nz][M][Cout], bias/act/bf16 in the reduce
    float* o = a.part + ((size_t)split * nz + zb) * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          if (m < a.M) o[(size_t)m * a.Cout + n0 + wn * (BN / 2) + j * 16 + (lane & 15)] = acc[i][j][r];
        }
    return;
  }

  // ---- epilogue: bias + activation -> bf16 tile in LDS -> 16-byte row stores --------------
  __syncthreads();
  char* E = smem;
  const float asc = ascale_of(a);
  __hip_bfloat16* yz = a.y + (size_t)zb * a.ybs;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int cl = wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = HAS_BIAS ? a.bias[zb * a.bbs + n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        float v = fmaf(acc[i][j][r], asc, bv);
        v = v > 0.f ? v : v * a.slope;
        *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpiStride + cl * 2) = __float2bfloat16(v);
      }
    }
  }
  __syncthreads();
  constexpr int kChunks = BN / 8;              // 16-B chunks per output row
  constexpr int kRowsPerPass = kThreads / kChunks;
  const int ch = tid % kChunks, rr = tid / kChunks;
#pragma unroll
  for (int p = 0; p < BM / kRowsPerPass; ++p) {
    const int rl = p * kRowsPerPass + rr;
    const int m = m0 + rl;
    if (m < a.M && n0 + ch * 8 < a.ldy) {
      const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpiStride + ch * 16);
      store_chunk(a, yz, out_row(a, m) * a.ldy + n0 + ch * 8, v);
    }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

template <int BM, int BN, bool HAS_BIAS, int VAR>
__global__ __launch_bounds__(BM * 2, BM == 128 ? 2 : 1) void conv_fwd_mfma(ConvArgs a) {
  conv_v1_impl<BM, BN, HAS_BIAS, VAR>(a, xcd_remap(blockIdx.x, gridDim.x), blockIdx.y,
                                      blockIdx.z, gridDim.z);
}

// Up to four independent convs in one launch (blockIdx.z = conv): the s*s phase convolutions
// of a strided data gradient, each storing straight into its parity sub-grid of dx (omode).
struct ConvPhases {
  ConvArgs a[4];
  int tiles[4];
};

template <int BM, int BN>
__global__ __launch_bounds__(BM * 2, BM == 128 ? 2 : 1) void conv_fwd_mfma_phases(ConvPhases p) {
  const int z = blockIdx.z;
  const int tiles = p.tiles[z];
  if ((int)blockIdx.x >= tiles) return;
  conv_v1_impl<BM, BN, false, 2>(p.a[z], xcd_remap(blockIdx.x, tiles), 0, 0, 1);
}

// ---- k10 v2: 256 x 128 tile, 8 waves, 3-stage LDS ring with one stage in flight across
// the barrier ------------------------------------------------------------------------------
//
// The v1 loop above drains every DMA (vmcnt(0) + __syncthreads) once per 64-deep k-step, so
// each step waits a full L2/HBM round trip that one k-step of MFMAs (512 cycles per wave)
// cannot cover; v1 hides it only with a second co-resident block. v2 keeps the NEXT stage's
// DMA in flight across the barrier instead (cdna_hip_programming.md "Pipelining across
// barriers"): three 48 KB stages (144 KB LDS, 1 block / CU), a counted `s_waitcnt vmcnt(6)`
// (6 = buffer_load...lds per thread per stage) and a raw s_barrier, so the loads of stage
// k+2 are issued while stage k computes and stage k+1 is still landing. 8 waves as 4 (M) x 2
// (N), each owning a 64 x 64 accumulator tile (16 x v_mfma_f32_16x16x32_bf16 per 32-k).
// The (tap, channel block) cursor of the k loop is advanced in scalar registers (no
// division per step), and each A row's validity for every filter tap is a precomputed
// 32-bit tap mask (KH * KW <= 32), so staging a row costs a bit test, a select and an add.
// Epilogue identical to v1 (bias + leaky, bf16 through LDS, 16-byte row stores) or fp32
// split-K partials.
template <bool HAS_BIAS>
__global__ __launch_bounds__(512, 1) void conv_fwd_mfma_v2(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = 256, BN = 128, kThreads = 512, NST = 3;
  constexpr int NI = 4;                       // 16-wide n-fragments per wave (64 columns)
  constexpr int kAbytes = BM * kRowBytes;     // 32 KB
  constexpr int kBbytes = BN * kRowBytes;     // 16 KB
  constexpr int kStage = kAbytes + kBbytes;   // 48 KB
  constexpr int kRound = kThreads * 16;       // LDS bytes per DMA round (64 rows)
  constexpr int kLoads = (BM + BN) / 64;      // DMA rounds (= glds per thread) per stage: 6
  __shared__ __attribute__((aligned(16))) char smem[NST * kStage];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w), 0, a.wbytes, kBufCfg);
  const int lrow = tid >> 3;                 // 0..63
  const int csw = (tid & 7) ^ (lrow & 7);    // swizzled source chunk (row & 7 == lrow & 7)
  const int HoWo = a.Ho * a.Wo;
  int a_off[4];
  uint32_t a_tmask[4];  // bit (ky * KW + kx) set when that filter tap reads inside the image
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + lrow + 64 * i;
    a_off[i] = 0;
    a_tmask[i] = 0;
    if (m < a.M) {
      const int b = m / HoWo, r = m - b * HoWo;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
      a_off[i] = (((b * a.H + ih0) * a.W + iw0) * a.Cin + csw * 8) * 2;
      for (int ky = 0; ky < a.KH; ++ky) {
        if ((unsigned)(ih0 + ky * a.dh) >= (unsigned)a.H) continue;
        for (int kx = 0; kx < a.KW; ++kx)
          if ((unsigned)(iw0 + kx * a.dw) < (unsigned)a.W) a_tmask[i] |= 1u << (ky * a.KW + kx);
      }
    }
  }
  const int wrow_bytes = a.nk * kBK * 2;  // = KH*KW*Cin*2
  int b_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) b_off[i] = (n0 + lrow + 64 * i) * wrow_bytes + csw * 16;

  // scalar k cursor of the NEXT stage to issue
  const int ks0 = blockIdx.y * a.kps;
  const int ks1 = min(a.nk, ks0 + a.kps);
  int ctap = ks0 / a.cpt;
  int cc = (ks0 - ctap * a.cpt) * kBK;         // channel offset within the tap
  int cky = ctap / a.KW, ckx = ctap - cky * a.KW;
  const int row_step = a.dh * a.W * a.Cin * 2;  // byte step of one filter row
  const int col_step = a.dw * a.Cin * 2;        // byte step of one filter column
  int ctoff = cky * row_step + ckx * col_step + cc * 2;
  int cks = ks0;

  auto issue = [&](int buf) {
    char* As = smem + buf * kStage;
    char* Bs = As + kAbytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (a_tmask[i] >> ctap) & 1u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(As + i * kRound + wid * 1024), 16, ok ? a_off[i] + ctoff : kOobOffset,
          0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(Bs + i * kRound + wid * 1024),
                                               16, b_off[i], cks * (kBK * 2), 0, 0);
    // advance the cursor: next channel block, else next tap
    ++cks;
    cc += kBK;
    ctoff += kBK * 2;
    if (cc == a.Cin) {
      cc = 0;
      ++ctap;
      if (++ckx == a.KW) {
        ckx = 0;
        ++cky;
      }
      ctoff = cky * row_step + ckx * col_step;
    }
  };

  f32x4 acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fsw = lane & 7, fk = lane >> 4;
  const int nks = ks1 - ks0;
  issue(0);
  if (nks > 1) issue(1);
  int rb = 0;  // ring slot of the stage being computed
  for (int it = 0; it < nks; ++it) {
    // this wave's DMA of stage `it` has landed; 6 newer glds (stage it+1) may still fly
    if (it + 1 < nks)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's stage-it DMA landed; slot (it-1)%3 is free
    if (it + 2 < nks) issue(rb == 0 ? 2 : rb - 1);
    const char* As = smem + rb * kStage;
    const char* Bs = As + kAbytes;
    bf16x8 af[2][4], bfr[2][NI];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[kk][i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + frow) * kRowBytes + coff);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + frow) * kRowBytes + coff);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    rb = rb == 2 ? 0 : rb + 1;
  }

  if (a.part) {  // split-K: raw fp32 partials, bias/act/bf16 in conv_splitk_reduce
    float* o = a.part + (size_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          if (m < a.M) o[(size_t)m * a.Cout + n0 + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
        }
    return;
  }

  __syncthreads();  // every wave is done reading the ring: reuse it for the epilogue tile
  char* E = smem;
  const float asc = ascale_of(a);
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int cl = wn * 64 + j * 16 + (lane & 15);
    const float bv = HAS_BIAS ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        float v = fmaf(acc[i][j][r], asc, bv);
        v = v > 0.f ? v : v * a.slope;
        *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpiStride + cl * 2) = __float2bfloat16(v);
      }
    }
  }
  __syncthreads();
  constexpr int kChunks = BN / 8;                 // 16
  constexpr int kRowsPerPass = kThreads / kChunks;  // 32
  const int ch = tid % kChunks, rr = tid / kChunks;
#pragma unroll
  for (int p = 0; p < BM / kRowsPerPass; ++p) {
    const int rl = p * kRowsPerPass + rr;
    const int m = m0 + rl;
    if (m < a.M && n0 + ch * 8 < a.ldy) {
      const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpiStride + ch * 16);
      store_chunk(a, a.y, out_row(a, m) * a.ldy + n0 + ch * 8, v);
    }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

// ---- k10 v3: 256 x 256 (or 512 x 128) tile, 8 waves of 128 x 64, 8-phase half-tile schedule -
//
// Structure after the 256x256 "8-phase" GEMM of cdna_hip_programming.md §5 (T1-T5), adapted to
// the implicit-GEMM A operand. Each wave (2 (M) x 4 (N) grid) owns a 128 x 64 accumulator
// tile = 4 quadrants of 64 x 32; one K-tile (64 deep) is computed in 4 phases, one quadrant
// (16 v_mfma_f32_16x16x32_bf16) per phase, in the order (0,0) (0,1) (1,1) (1,0) so that each
// phase changes only the A or only the B half of the operands. Per phase, behind ONE barrier:
//   * one HALF-tile of the next K-tile (128 rows x 64 k = 2 buffer_load ... lds per thread) is
//     issued into the other LDS buffer — four half-tiles per K-tile, each issued 2-3 phases
//     before its first read, retired by a counted `s_waitcnt vmcnt(2|4)` (never 0 in the loop);
//   * the fragments the NEXT phase needs are read from LDS into a second register set while
//     this phase's 16 MFMAs run on the set read one phase earlier (so the MFMAs never wait on
//     a ds_read issued in their own phase);
//   * the fragment register sets rotate with a period of two K-tiles, so the loop body holds
//     8 phases (2 K-tiles) with every register index static.
// K-steps past the end of the (split-K) range are issued as out-of-range (zero) loads, so the
// schedule never branches; an odd K-step count costs one zero tile.
template <int BM, int BN, bool HAS_BIAS>
__global__ __launch_bounds__(512, 1) void conv_fwd_mfma_v3(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert((BM / 128) * (BN / 64) == 8, "8 waves of 128 x 64");
  constexpr int WN = BN / 64;                        // waves along N
  constexpr int LA = BM / 128, LB = BN / 128;        // glds per thread per A / B half-tile
  constexpr int kAbytes = BM * kRowBytes;
  constexpr int kBuf = (BM + BN) * kRowBytes;        // 64 / 80 KB per K-tile buffer
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (SGPR)
  const int wm = wid / WN, wn = wid % WN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w), 0, a.wbytes, kBufCfg);

  // ---- staging geometry: glds (half h, round i) of wave w moves 8 tile rows -----------------
  //   A rows  i*128 + h*64 + w*8 + lr          (A half h = rows with (row >> 6) & 1 == h)
  //   B rows  (2i + (w >> 2))*64 + h*32 + (w & 3)*8 + lr   (B half h = (row >> 5) & 1 == h)
  // (Cout % BN == 0: every B row exists; the B rows of one thread differ by wave-uniform
  // multiples of the weight row, carried in the scalar offset)
  const int lr = lane >> 3;
  const int csw = (lane & 7) ^ lr;  // every row group starts at a multiple of 8: row & 7 == lr
  const int HoWo = a.Ho * a.Wo;
  int a_off[2][LA];
  uint32_t a_tm[2][LA];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int m = m0 + i * 128 + h * 64 + wid * 8 + lr;
      a_off[h][i] = 0;
      a_tm[h][i] = 0;
      if (m < a.M) {
        const int b = m / HoWo, r = m - b * HoWo;
        const int oh = r / a.Wo, ow = r - oh * a.Wo;
        const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
        a_off[h][i] = (((b * a.H + ih0) * a.W + iw0) * a.Cin + csw * 8) * 2;
        for (int ky = 0; ky < a.KH; ++ky) {
          if ((unsigned)(ih0 + ky * a.dh) >= (unsigned)a.H) continue;
          for (int kx = 0; kx < a.KW; ++kx)
            if ((unsigned)(iw0 + kx * a.dw) < (unsigned)a.W) a_tm[h][i] |= 1u << (ky * a.KW + kx);
        }
      }
    }
  const int wrow_bytes = a.nk * kBK * 2;
  const int b_base = (n0 + (wid >> 2) * 64 + (wid & 3) * 8 + lr) * wrow_bytes + csw * 16;

  // ---- scalar cursor of the K-step being staged. Past the end of the split's range the
  // tap index becomes 31 (no row has that bit: KH*KW <= 31) and the weight offset runs out
  // of range, so those stages load zeros without a branch.
  const int ks0 = blockIdx.y * a.kps;
  const int ks1 = min(a.nk, ks0 + a.kps);
  int ctap = ks0 / a.cpt;
  int cc = (ks0 - ctap * a.cpt) * kBK;
  int cky = ctap / a.KW, ckx = ctap - cky * a.KW;
  const int row_step = a.dh * a.W * a.Cin * 2;
  const int col_step = a.dw * a.Cin * 2;
  int ctoff = cky * row_step + ckx * col_step + cc * 2;
  int cks = ks0;
  int mtap = ctap, csoff = cks * (kBK * 2);

  auto issueA = [&](int buf, int h) {
    const uint32_t bit = 1u << mtap;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(smem + buf * kBuf + (i * 128 + h * 64 + wid * 8) * kRowBytes), 16,
          (a_tm[h][i] & bit) ? a_off[h][i] + ctoff : kOobOffset, 0, 0, 0);
  };
  auto issueB = [&](int buf, int h) {
#pragma unroll
    for (int i = 0; i < LB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs,
          (lds_ptr_t)(smem + buf * kBuf + kAbytes +
                      ((2 * i + (wid >> 2)) * 64 + h * 32 + (wid & 3) * 8) * kRowBytes),
          16, b_base, csoff + (i * 128 + h * 32) * wrow_bytes, 0, 0);
  };
  auto advance = [&]() {
    ++cks;
    cc += kBK;
    ctoff += kBK * 2;
    if (cc == a.Cin) {
      cc = 0;
      ++ctap;
      if (++ckx == a.KW) {
        ckx = 0;
        ++cky;
      }
      ctoff = cky * row_step + ckx * col_step;
    }
    const bool kv = cks < ks1;
    mtap = kv ? ctap : 31;
    csoff = kv ? cks * (kBK * 2) : kOobOffset;
  };

  // ---- fragments ------------------------------------------------------------------------
  const int frow = lane & 15, fsw = lane & 7, fk = lane >> 4;
  auto readA = [&](int buf, int mq, bf16x8 (&f)[2][4]) {
    const char* As = smem + buf * kBuf;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f[kk][i] = *reinterpret_cast<const bf16x8*>(
            As + (wm * 128 + mq * 64 + i * 16 + frow) * kRowBytes + coff);
    }
  };
  auto readB = [&](int buf, int nq, bf16x8 (&f)[2][2]) {
    const char* Bs = smem + buf * kBuf + kAbytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        f[kk][j] = *reinterpret_cast<const bf16x8*>(
            Bs + (wn * 64 + nq * 32 + j * 16 + frow) * kRowBytes + coff);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define IAMD_V3_MFMA(AF, BF, MQ, NQ)                                                        \
  do {                                                                                      \
    __builtin_amdgcn_s_setprio(1);                                                          \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                        \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                           \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                           \
      acc[(MQ) * 4 + i][(NQ) * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(             \
          AF[kk][i], BF[kk][j], acc[(MQ) * 4 + i][(NQ) * 2 + j], 0, 0, 0);                  \
    __builtin_amdgcn_s_setprio(0);                                                          \
  } while (0)
#define IAMD_V3_SYNC(N)                                          \
  do {                                                           \
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");     \
    __builtin_amdgcn_s_barrier();                                \
  } while (0)
  // counted waits (glds per thread still allowed in flight) at each phase of a K-tile:
  // ph1 needs B0, B1 (A1 may fly), ph2 needs A1 (A0' may fly), ph3 needs nothing new (A0', B0'
  // may fly), ph4 needs A0' (B0', B1' may fly); prologue needs A0 (B0, B1, A1 may fly)
  constexpr int W1 = LA, W2 = LA, W3 = LA + LB, W4 = 2 * LB, W0 = 2 * LB + LA;

  // Register budget (2 waves / SIMD -> 256 VGPRs): 128 accumulators + at most 80 operand
  // registers live. At a K-tile boundary only the A half is read one phase ahead; the first
  // phase of a K-tile reads its B halves itself (4 + 4 ds_read_b128 it waits on, covered by
  // the partner wave's MFMAs).
  bf16x8 a0[2][4], a1[2][4], bX[2][2], bY[2][2];
  const int nks = ks1 - ks0;
  const int nt2 = (nks + 1) & ~1;  // K-tiles rounded up to the 2-tile loop body
  // prologue: stage K-tile 0 into buffer 0 in first-use order, read its A0 half
  issueA(0, 0);
  issueB(0, 0);
  issueB(0, 1);
  issueA(0, 1);
  advance();
  IAMD_V3_SYNC(W0);
  readA(0, 0, a0);
  for (int t = 0; t < nt2; t += 2) {
    // K-tile t in buffer 0, staging K-tile t+1 into buffer 1
    IAMD_V3_SYNC(W1); issueA(1, 0); readB(0, 0, bX); readB(0, 1, bY); IAMD_V3_MFMA(a0, bX, 0, 0);
    IAMD_V3_SYNC(W2); issueB(1, 0); readA(0, 1, a1); IAMD_V3_MFMA(a0, bY, 0, 1);
    IAMD_V3_SYNC(W3); issueB(1, 1); readB(0, 0, bX); IAMD_V3_MFMA(a1, bY, 1, 1);
    IAMD_V3_SYNC(W4); issueA(1, 1); advance(); readA(1, 0, a0); IAMD_V3_MFMA(a1, bX, 1, 0);
    // K-tile t+1 in buffer 1, staging K-tile t+2 into buffer 0
    IAMD_V3_SYNC(W1); issueA(0, 0); readB(1, 0, bX); readB(1, 1, bY); IAMD_V3_MFMA(a0, bX, 0, 0);
    IAMD_V3_SYNC(W2); issueB(0, 0); readA(1, 1, a1); IAMD_V3_MFMA(a0, bY, 0, 1);
    IAMD_V3_SYNC(W3); issueB(0, 1); readB(1, 0, bX); IAMD_V3_MFMA(a1, bY, 1, 1);
    IAMD_V3_SYNC(W4); issueA(0, 1); advance(); readA(0, 0, a0); IAMD_V3_MFMA(a1, bX, 1, 0);
  }
#undef IAMD_V3_MFMA
#undef IAMD_V3_SYNC
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the trailing (zero) prefetches and reads are done: smem is free

  if (a.part) {  // split-K: raw fp32 partials
    float* o = a.part + (size_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * 64 + j * 16 + (lane & 15);
          if (m < a.M) o[(size_t)m * a.Cout + n] = acc[i][j][r];
        }
    return;
  }

  // ---- epilogue: 128-column slices through LDS, 16-byte row stores ------------------------
  char* E = smem;
  const float asc = ascale_of(a);
#pragma unroll
  for (int half = 0; half < BN / 128; ++half) {
    if ((wn >> 1) == half) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = (wn & 1) * 64 + j * 16 + (lane & 15);
        const int n = n0 + half * 128 + cl;
        const float bv = HAS_BIAS ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rl = wm * 128 + i * 16 + (lane >> 4) * 4 + r;
            float v = fmaf(acc[i][j][r], asc, bv);
            v = v > 0.f ? v : v * a.slope;
            *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpiStride + cl * 2) = __float2bfloat16(v);
          }
      }
    }
    __syncthreads();
    const int ch = tid & 15, rr = tid >> 4;  // 16 chunks per row, 32 rows per pass
#pragma unroll
    for (int p = 0; p < BM / 32; ++p) {
      const int rl = p * 32 + rr;
      const int m = m0 + rl;
      if (m < a.M && n0 + half * 128 + ch * 8 < a.ldy) {
        const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpiStride + ch * 16);
        store_chunk(a, a.y, out_row(a, m) * a.ldy + n0 + half * 128 + ch * 8, v);
      }
    }
    __syncthreads();
  }
#endif  // __HIP_DEVICE_COMPILE__
}

// ---- k10 v4: row-window implicit GEMM (stride 1), 256 x 128 tile, KW-tap input windows ----
//
// In v1 / v3 every filter tap re-stages its A tile (BM shifted input pixels x 64 channels) from
// L2, so an input byte crosses the L2 -> LDS path KH * KW times. Here the 256 output pixels of a
// block are R = 256 / SW output-row segments of SW pixels (SW = 256, or the whole row when
// Wo divides 256), and for one filter row ky and 64-channel block the block stages ONE input
// window per segment — SW + KW - 1 consecutive pixels — then runs the KW taps of that filter row
// from it, tap kx reading the window rows shifted by kx (the 16-B chunk swizzle is keyed on the
// LDS row, so a shifted 16-row fragment read stays conflict free). Only the weight tile (128
// output channels x 64) is staged per tap. Per tap step: 16 KB of weights + 1/KW of a 40 KB
// window, against 256 x 128 x 64 MACs: ~2.9x fewer L2 -> LDS bytes per MFMA than the v1 tile.
//   8 waves as 4 (M) x 2 (N), 64 x 64 accumulators each; LDS: two window buffers (the next
//   (ky, channel block)'s window is staged during the first tap of the current one) and a
//   KW-slot weight ring (tap kx in slot kx, staged two tap steps ahead), 160 KB for KW = 5.
//   DMA is buffer_load ... lds (zeros for padding pixels and past the k range); waits are
//   counted vmcnt (2 or 7 glds per thread still in flight, never 0 in the loop) + raw s_barrier.
// The data gradient of a stride-1 conv runs here too (flipped / transposed weight, as v1).
// BT (data gradient without a flipped weight copy): a.w is the FORWARD weight [K][KH][KW][N]
// (K = a.Cin = dy channels, N = a.Cout = dx channels) and tap (ky, kx) reads forward tap
// (KH-1-ky, KW-1-kx). Its weight tile is staged k-major (64 rows of 128 n-channels, 256 B,
// 16-byte chunks swizzled per row) and the B fragments are read with the transposing
// ds_read_b64_tr_b16 (two 4-row reads per 8-deep fragment, as the k11 weight gradient does).
// PF (fragment prefetch across the tap barrier): a tap step's second k-half fragments (kk = 1)
// are read during the step and consumed by the NEXT step's first MFMAs, which issue right after
// its barrier while that step's kk = 0 fragments are still in flight — without it every tap
// step began with all 8 waves waiting on LDS reads (MFMA pipe busy 54-63%,
// profiles/pmc_conv_v4_r3_mi355x.txt).
template <int KW, bool HAS_BIAS, bool BT, bool PF>
__global__ __launch_bounds__(512, 1) void conv_fwd_mfma_v4(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = 256, BN = 128;
  constexpr int kArows = 320;                     // window rows per buffer: 5 DMA rounds of 64
  constexpr int kAbytes = kArows * kRowBytes;     // 40 KB
  constexpr int kBbytes = BN * kRowBytes;         // 16 KB per tap slot
  constexpr int kBoff = 2 * kAbytes;              // weight ring after the two windows
  __shared__ __attribute__((aligned(16))) char smem[2 * kAbytes + KW * kBbytes];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HoWo = a.Ho * a.Wo;
  const int SW = a.Wo >= BM ? BM : a.Wo;          // pixels per output-row segment
  const int L = SW + KW - 1;                      // window rows per segment
  const int R = BM / SW;

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w), 0, a.wbytes, kBufCfg);

  // ---- window DMA: round r of wave w moves rows 64 r + 8 w + (lane >> 3), 16-B chunk
  // (lane & 7) ^ (row & 7) of the source (the LDS write is lane-linear) -------------------
  const int dr = lane >> 3;
  const int csw = (lane & 7) ^ dr;                // row & 7 == dr for every staged row
  const int rowbytes = a.W * a.Cin * 2;           // input row stride (bytes)
  int a_off[5];
  uint32_t a_km[5];                               // bit ky: this window row reads inside
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const int row = r * 64 + wid * 8 + dr;
    const int s = row / L, j = row - s * L;
    a_off[r] = 0;
    a_km[r] = 0;
    if (s < R) {
      const int m = m0 + s * SW;                  // first output pixel of segment s
      const int b = m / HoWo, rr = m - b * HoWo;
      const int oh = rr / a.Wo, ow0 = rr - oh * a.Wo;
      const int ih0 = oh - a.ph, iw = ow0 - a.pw + j;
      if ((unsigned)iw < (unsigned)a.W) {
        a_off[r] = (b * a.H + ih0) * rowbytes + (iw * a.Cin + csw * 8) * 2;
        for (int ky = 0; ky < a.KH; ++ky)
          a_km[r] |= (uint32_t)((unsigned)(ih0 + ky) < (unsigned)a.H) << ky;
      }
    }
  }
  // weight DMA: rows 64 i + 8 w + (lane >> 3) of the 128-row tap tile (BT: k-rows
  // 32 i + 4 w + (lane >> 4) of 256 B, source chunk (lane & 15) ^ swz(row))
  const int wrow_bytes = a.nk * kBK * 2;
  const int KK = a.KH * KW;
  int b_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (BT) {
      const int row = i * 32 + wid * 4 + (lane >> 4);
      const int sch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      b_off[i] = (row * KK * a.Cout + n0 + sch * 8) * 2;
    } else {
      b_off[i] = (n0 + i * 64 + wid * 8 + dr) * wrow_bytes + csw * 16;
    }
  }

  // ---- k range of this split in outer steps o = (ky, channel block) ------------------------
  const int o0 = blockIdx.y * a.kps;
  const int o1 = min(a.nk / KW, o0 + a.kps);      // nk = KH * KW * cpt: KH * cpt outer steps
  // scalar cursors (filter row, channel offset) of outer step o (being computed) and o + 1,
  // advanced once per outer step (no division in the loop)
  int cky = o0 / a.cpt, ccc = (o0 - (o0 / a.cpt) * a.cpt) * kBK;
  int nky = cky, ncc = ccc + kBK;
  if (ncc == a.Cin) { ncc = 0; ++nky; }
  auto issueA = [&](int o, int ky, int cc, int buf) {  // window of outer step o into buf
    const bool live = o < o1;
    const int koff = ky * rowbytes + cc * 2;
    char* As = smem + buf * kAbytes;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const bool ok = live && ((a_km[r] >> (ky & 31)) & 1u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(As + r * 8192 + wid * 1024), 16, ok ? a_off[r] + koff : kOobOffset,
          0, 0, 0);
    }
  };
  auto issueB = [&](int o, int ky, int cc, int kx, int slot) {  // weight tap (ky, kx), block cc
    int soff;
    if constexpr (BT)  // forward tap (KH-1-ky, KW-1-kx), k rows cc.. of [K][KK][N]
      soff = o < o1 ? ((cc * KK + (a.KH - 1 - ky) * KW + (KW - 1 - kx)) * a.Cout) * 2
                    : kOobOffset;
    else
      soff = o < o1 ? ((ky * KW + kx) * a.Cin + cc) * 2 : kOobOffset;
    char* Bs = smem + kBoff + slot * kBbytes;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(Bs + i * 8192 + wid * 1024), 16,
                                               b_off[i], soff, 0, 0);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment rows: A = window row of output pixel wm*64 + i*16 + frow (+ kx), B = channel row
  const int frow = lane & 15, fsw = lane & 7, fk = lane >> 4;
  int wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = wm * 64 + i * 16 + frow;
    const int s = p / SW;
    wrow[i] = s * L + (p - s * SW);
  }
  // fragments of k-half kk of tap kx (window buffer abuf)
  auto load_frags = [&](int abuf, int kx, int kk, bf16x8 (&af)[4], bf16x8 (&bf)[4]) {
    const char* As = smem + abuf * kAbytes;
    const char* Bs = smem + kBoff + kx * kBbytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wrow[i] + kx;
      af[i] = *reinterpret_cast<const bf16x8*>(
          As + row * kRowBytes + (((kk * 4 + fk) ^ (row & 7)) << 4));
    }
    if constexpr (BT) {
      // lane (g, q, p): rows kk*32 + 8g + q (+4), 8-byte quarter p of a 16-column block
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      const int r0 = kk * 32 + g * 8 + q;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cb = (wn * 64 + j * 16) >> 3;
        auto baddr = [&](int row) {
          return row * 256 + (((cb + (p >> 1)) ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4) +
                 ((p & 1) << 3);
        };
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(Bs + baddr(r0)));
        const bf16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(Bs + baddr(r0 + 4)));
        bf[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    } else {
      const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + frow) * kRowBytes +
                                                 coff);
    }
  };
  auto mma = [&](const bf16x8 (&af)[4], const bf16x8 (&bf)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // PF: the previous tap step's kk = 1 fragments (zero before the first step: +0 MFMAs)
  bf16x8 pa[4], pb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pa[i] = bf16x8{};
    pb[i] = bf16x8{};
  }
  auto tapstep = [&](int abuf, int kx) {
    if constexpr (PF) {
      bf16x8 a0[4], b0[4];
      load_frags(abuf, kx, 0, a0, b0);
      mma(pa, pb);                      // previous step, kk = 1: no LDS wait after the barrier
      load_frags(abuf, kx, 1, pa, pb);  // this step's kk = 1, consumed by the next step
      mma(a0, b0);
    } else {
      const char* As = smem + abuf * kAbytes;
      const char* Bs = smem + kBoff + kx * kBbytes;
      bf16x8 af[2][4], bfr[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wrow[i] + kx;
          af[kk][i] = *reinterpret_cast<const bf16x8*>(
              As + row * kRowBytes + (((kk * 4 + fk) ^ (row & 7)) << 4));
        }
        if constexpr (BT) {
          // lane (g, q, p): rows kk*32 + 8g + q (+4), 8-byte quarter p of a 16-column block
          const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
          const int r0 = kk * 32 + g * 8 + q;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cb = (wn * 64 + j * 16) >> 3;
            auto baddr = [&](int row) {
              return row * 256 + (((cb + (p >> 1)) ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4) +
                     ((p & 1) << 3);
            };
            const bf16x4 lo =
                __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(Bs + baddr(r0)));
            const bf16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(Bs + baddr(r0 + 4)));
            bfr[kk][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        } else {
          const int coff = ((kk * 4 + fk) ^ fsw) << 4;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bfr[kk][j] = *reinterpret_cast<const bf16x8*>(
                Bs + (wn * 64 + j * 16 + frow) * kRowBytes + coff);
        }
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j],
                                                                0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  // one outer step (window buffer abuf static): KW tap steps; tap step q stages the weights of
  // tap step q + 2 into its ring slot and, at kx == 0, the next outer step's window
  auto outer = [&](int o, int abuf) {
#pragma unroll
    for (int kx = 0; kx < KW; ++kx) {
      // (lgkmcnt(0): this wave's fragment reads of the previous step are in registers before
      // any wave's DMA may overwrite their LDS slot / window)
      if (kx == 1)
        asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");  // younger: window 5 + weights 2
      else
        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");  // younger: the next weights 2
      __builtin_amdgcn_s_barrier();
      if (kx == 0) issueA(o + 1, nky, ncc, abuf ^ 1);
      if (kx + 2 < KW) issueB(o, cky, ccc, kx + 2, kx + 2);
      else issueB(o + 1, nky, ncc, kx + 2 - KW, kx + 2 - KW);
      tapstep(abuf, kx);
    }
    cky = nky;
    ccc = ncc;
    ncc += kBK;
    if (ncc == a.Cin) { ncc = 0; ++nky; }
  };
  // prologue: window of o0, weights of its taps 0 and 1
  issueA(o0, cky, ccc, 0);
  issueB(o0, cky, ccc, 0, 0);
  issueB(o0, cky, ccc, 1, 1);
  for (int o = o0; o < o1; o += 2) {
    outer(o, 0);
    if (o + 1 < o1) outer(o + 1, 1);
  }
  if constexpr (PF) mma(pa, pb);  // the last tap step's kk = 1
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // trailing (zero) prefetches landed and every wave is done reading

  if (a.part) {  // split-K: raw fp32 partials, bias/act/bf16 in conv_splitk_reduce
    float* o = a.part + (size_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          if (m < a.M) o[(size_t)m * a.Cout + n0 + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
        }
    return;
  }
  char* E = smem;
  const float asc = ascale_of(a);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn * 64 + j * 16 + (lane & 15);
    const float bv = HAS_BIAS ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        float v = fmaf(acc[i][j][r], asc, bv);
        v = v > 0.f ? v : v * a.slope;
        *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpiStride + cl * 2) = __float2bfloat16(v);
      }
  }
  __syncthreads();
  const int ch = tid & 15, rr = tid >> 4;  // 16 chunks per row, 32 rows per pass
#pragma unroll
  for (int p = 0; p < BM / 32; ++p) {
    const int rl = p * 32 + rr;
    const int m = m0 + rl;
    if (m < a.M && n0 + ch * 8 < a.ldy) {
      const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpiStride + ch * 16);
      store_chunk(a, a.y, out_row(a, m) * a.ldy + n0 + ch * 8, v);
    }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

// ---- k10 v5: row-window implicit GEMM, 256 x 256 tile, 8 waves of 128 x 64 -----------------
//
// v4's 64 x 64 wave tile reads 512 LDS bytes per MFMA (A and B fragments) and, with the DMA
// writes, keeps the LDS array ~80% busy against the MFMA pipe (MFMA busy 54-63%,
// profiles/pmc_conv_v4_r3_mi355x.txt). Here each of the 8 waves (2 (M) x 4 (N)) owns a
// 128 x 64 sub-tile of a 256-pixel x 256-channel block: 384 B per MFMA, and the window staged
// per (filter row, channel block) is shared by twice the output channels.
// LDS (144 KB): two 32 KB weight slots (tap t+1 staged during tap t: the 256-row tile is too
// large for v4's KW-slot ring) at offset 0, then two 40 KB window buffers.
// Window rows of output-row segment s start at row s * (SW + 8) (pitch padded to a multiple of
// 8 rows), so a fragment row's swizzle key (row & 7) is (lane + kx) & 7 for every fragment:
// per tap step two VGPR fragment bases, everything else is an ds_read immediate (FULLROW, one
// 256-pixel segment per block) or one add per fragment (SW = 32..128).
// DMA order per tap step: weights of the next tap, then (first tap of a filter row) the next
// window, so the wait at tap 1 (vmcnt(5)) retires only the weights; other taps vmcnt(0).
template <int KW, bool HAS_BIAS, bool FULLROW>
__global__ __launch_bounds__(512, 1) void conv_fwd_mfma_v5(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = 256, BN = 256;
  constexpr int kArows = 320;                     // window rows per buffer: 5 DMA rounds of 64
  constexpr int kAbytes = kArows * kRowBytes;     // 40 KB
  constexpr int kBbytes = BN * kRowBytes;         // 32 KB per weight slot
  constexpr int kAoff = 2 * kBbytes;              // windows after the two weight slots
  constexpr int kEpi = BN * 2 + 16;               // epilogue row stride (bytes)
  constexpr int kSmem = kAoff + 2 * kAbytes;
  static_assert(BM * kEpi <= kSmem, "v5 epilogue staging exceeds LDS");
  __shared__ __attribute__((aligned(16))) char smem[kSmem];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HoWo = a.Ho * a.Wo;
  const int SW = FULLROW ? BM : a.Wo;             // pixels per output-row segment
  const int P = SW + 8;                           // LDS row pitch of a segment's window
  const int R = BM / SW;

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w), 0, a.wbytes, kBufCfg);

  // ---- window DMA sources: round r of wave w moves LDS rows 64 r + 8 w + (lane >> 3) -------
  // Rows outside the image columns or past a segment's SW + KW - 1 window rows get an offset
  // past the tensor (any koff added keeps it past: koff < xbytes < 2^31), so the buffer unit
  // returns zeros; the filter-row validity is a per-row bit mask (FULLROW: one output row per
  // block, so the mask is wave-uniform and lives in an SGPR).
  const int dr = lane >> 3;
  const int csw = (lane & 7) ^ dr;                // row & 7 == dr for every staged row
  const int rowbytes = a.W * a.Cin * 2;
  int a_off[5];
  uint32_t a_km[FULLROW ? 1 : 5];
  if constexpr (FULLROW) {
    const int b = m0 / HoWo, rr = m0 - b * HoWo;
    const int oh = rr / a.Wo, ow0 = rr - oh * a.Wo;
    const int ih0 = oh - a.ph;
    uint32_t km = 0;
    for (int ky = 0; ky < a.KH; ++ky) km |= (uint32_t)((unsigned)(ih0 + ky) < (unsigned)a.H) << ky;
    a_km[0] = __builtin_amdgcn_readfirstlane(km);
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int j = r * 64 + wid * 8 + dr;
      const int iw = ow0 - a.pw + j;
      a_off[r] = (j < SW + KW - 1 && (unsigned)iw < (unsigned)a.W)
                     ? (b * a.H + ih0) * rowbytes + (iw * a.Cin + csw * 8) * 2
                     : kOobOffset;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int row = r * 64 + wid * 8 + dr;
      const int s = row / P, j = row - s * P;
      a_off[r] = kOobOffset;
      a_km[r] = 0;
      if (s < R && j < SW + KW - 1) {
        const int m = m0 + s * SW;
        const int b = m / HoWo, rr = m - b * HoWo;
        const int oh = rr / a.Wo, ow0 = rr - oh * a.Wo;
        const int ih0 = oh - a.ph, iw = ow0 - a.pw + j;
        if ((unsigned)iw < (unsigned)a.W) {
          a_off[r] = (b * a.H + ih0) * rowbytes + (iw * a.Cin + csw * 8) * 2;
          for (int ky = 0; ky < a.KH; ++ky)
            a_km[r] |= (uint32_t)((unsigned)(ih0 + ky) < (unsigned)a.H) << ky;
        }
      }
    }
  }
  const int wrow_bytes = a.nk * kBK * 2;
  int b_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) b_off[i] = (n0 + i * 64 + wid * 8 + dr) * wrow_bytes + csw * 16;

  const int o0 = blockIdx.y * a.kps;
  const int o1 = min(a.nk / KW, o0 + a.kps);
  // (filter row, channel offset) of the outer step being computed and of the next one
  int cky = o0 / a.cpt, ccc = (o0 - (o0 / a.cpt) * a.cpt) * kBK;
  int nky = cky, ncc = ccc + kBK;
  if (ncc == a.Cin) { ncc = 0; ++nky; }
  auto issueA = [&](int o, int ky, int cc, int buf) {
    const uint32_t live = o < o1;
    const int koff = ky * rowbytes + cc * 2;
    char* As = smem + kAoff + buf * kAbytes;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const uint32_t ok = live & (a_km[FULLROW ? 0 : r] >> (ky & 31));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(As + r * 8192 + wid * 1024), 16,
          (ok & 1u) ? a_off[r] + koff : kOobOffset, 0, 0, 0);
    }
  };
  auto issueB = [&](int o, int ky, int cc, int kx, int slot) {
    const int soff = o < o1 ? ((ky * KW + kx) * a.Cin + cc) * 2 : kOobOffset;
    char* Bs = smem + slot * kBbytes;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(Bs + i * 8192 + wid * 1024), 16,
                                               b_off[i], soff, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragment i of this wave: output pixels p = wm*128 + i*16 + frow, window row p + 8 s(p)
  // (16 | SW: a fragment never straddles two segments). Wave-uniform: SGPRs.
  int arow[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pb = wm * 128 + i * 16;
    arow[i] = FULLROW ? 0 : 8 * (pb / SW) * kRowBytes;
  }

  auto tapstep = [&](int abuf, int kx, int slot) {
    // The fragment addresses are recomputed per tap step from an opaque copy of the lane id:
    // hoisted out of the loop they are 2 * KW * (8 + 1) loop-invariant registers, which spill
    // (and a scratch reload's vmcnt wait drains the in-flight DMA).
    int l = lane;
    asm volatile("" : "+v"(l));
    const int frow = l & 15, fk = l >> 4;
    const int key = (frow + kx) & 7;
    const int rb = (wm * 128 + frow) * kRowBytes;
    const int ab0 = kAoff + rb + (((0 * 4 + fk) ^ key) << 4);
    const int ab1 = kAoff + rb + (((1 * 4 + fk) ^ key) << 4);
    const int brb = (wn * 64 + frow) * kRowBytes;
    const int bb0 = brb + (((0 * 4 + fk) ^ (frow & 7)) << 4);
    const int bb1 = brb + (((1 * 4 + fk) ^ (frow & 7)) << 4);
    // (per k-half: 12 fragments = 48 VGPRs beside the 128 accumulator registers; hoisting
    // both halves' reads spills at the 256-register budget of two waves per SIMD)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[8], bfr[4];
      const int ab = kk ? ab1 : ab0;
      const int bb = kk ? bb1 : bb0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(smem + bb + slot * kBbytes +
                                                  j * 16 * kRowBytes);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(
            smem + ab + arow[i] + abuf * kAbytes + (i * 16 + kx) * kRowBytes);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  // one outer step: KW tap steps; tap step kx stages the weights of the next tap (or of the
  // next outer step's tap 0) into the other slot and, at kx == 0, the next outer step's window.
  // ol = parity of (o - o0): slot of tap step (o, kx) = ((o - o0) * KW + kx) & 1
  auto outer = [&](int o, int abuf, int ol) {
#pragma unroll
    for (int kx = 0; kx < KW; ++kx) {
      if (kx == 1)
        asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");  // younger: the window
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int slot = (ol * KW + kx) & 1;
      if (kx + 1 < KW) issueB(o, cky, ccc, kx + 1, slot ^ 1);
      else issueB(o + 1, nky, ncc, 0, slot ^ 1);
      if (kx == 0) issueA(o + 1, nky, ncc, abuf ^ 1);
      tapstep(abuf, kx, slot);
    }
    cky = nky;
    ccc = ncc;
    ncc += kBK;
    if (ncc == a.Cin) { ncc = 0; ++nky; }
  };
  issueB(o0, cky, ccc, 0, 0);
  issueA(o0, cky, ccc, 0);
  for (int o = o0; o < o1; o += 2) {
    outer(o, 0, 0);
    if (o + 1 < o1) outer(o + 1, 1, 1);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // trailing (zero) prefetches landed and every wave is done reading

  if (a.part) {
    float* op = a.part + (size_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          if (m < a.M)
            op[(size_t)m * a.Cout + n0 + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
        }
    return;
  }
  char* E = smem;
  const float asc = ascale_of(a);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn * 64 + j * 16 + (lane & 15);
    const float bv = HAS_BIAS ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 128 + i * 16 + (lane >> 4) * 4 + r;
        float v = fmaf(acc[i][j][r], asc, bv);
        v = v > 0.f ? v : v * a.slope;
        *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpi + cl * 2) = __float2bfloat16(v);
      }
  }
  __syncthreads();
  const int ch = tid & 31, rr = tid >> 5;  // 32 chunks per row, 16 rows per pass
#pragma unroll 4
  for (int p = 0; p < BM / 16; ++p) {
    const int rl = p * 16 + rr;
    const int m = m0 + rl;
    if (m < a.M && n0 + ch * 8 < a.ldy) {
      const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpi + ch * 16);
      store_chunk(a, a.y, out_row(a, m) * a.ldy + n0 + ch * 8, v);
    }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

}  // namespace

namespace {

// v4 (row-window, 256 x 128): stride 1, undilated, KW 3..5, whole 256-pixel tiles made of
// output-row segments (Wo a multiple of 256, or 16..128 dividing 256)
bool v4_eligible(const ConvArgs& a) {
  static const bool off = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_CONV_V4");  // 0: A/B switch back to v1 / v3
    return e != nullptr && e[0] == '0';
  }();
  // (Cin = 32 runs on the row-window tile only: v4 / v5 step 64-channel k-chunks)
  return !off && a.Cin % kBK == 0 && a.nz == 1 && a.omode == 0 && a.sh == 1 && a.sw == 1 &&
         a.dh == 1 && a.dw == 1 &&
         (a.KW >= 3 && a.KW <= 5) && a.KH <= 31 && a.Cout % 128 == 0 &&
         (a.Wo % 256 == 0 || (a.Wo >= 16 && a.Wo <= 128 && 256 % a.Wo == 0)) &&
         ((int64_t)a.Ho * a.Wo) % 256 == 0;
}

void run_v4(ConvArgs& a, const at::Tensor& x, bool bt) {
  const int Cout = a.Cout, KW = a.KW;
  a.nNt = Cout / 128;
  const int64_t tiles4 = (int64_t)(a.M / 256) * a.nNt;
  const int nout = a.nk / KW;  // (filter row, channel block) outer steps
  int S4 = 1;
  if (tiles4 < 256 && nout >= 8) S4 = (int)std::min<int64_t>((256 + tiles4 - 1) / tiles4, nout / 4);
  if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_SPLITK")) S4 = std::max(1, std::atoi(e));
  S4 = std::max(1, std::min(S4, nout));
  a.kps = ceil_div(nout, S4);
  S4 = ceil_div(nout, a.kps);
  at::Tensor part4;
  a.part = nullptr;
  if (S4 > 1) {
    part4 = at::empty({(int64_t)S4 * a.M * Cout}, x.options().dtype(at::kFloat));
    a.part = part4.data_ptr<float>();
  }
  const dim3 grid4((unsigned)tiles4, (unsigned)S4, 1);
  // IMAGINAIRE_AMD_V4_PF = 0: A/B switch back to the un-prefetched tap step
  const char* pfe = std::getenv("IMAGINAIRE_AMD_V4_PF");
  const bool pf = !(pfe != nullptr && pfe[0] == '0');
  auto launch = [&](auto kv, auto hbv, auto btv) {
    constexpr int K = decltype(kv)::value;
    constexpr bool HB = decltype(hbv)::value, BTV = decltype(btv)::value;
    if (pf && !BTV)  // (the BT kernels have no registers left for a second fragment set)
      hipLaunchKernelGGL((conv_fwd_mfma_v4<K, HB, BTV, !BTV>), grid4, dim3(512), 0, stream(), a);
    else
      hipLaunchKernelGGL((conv_fwd_mfma_v4<K, HB, BTV, false>), grid4, dim3(512), 0, stream(), a);
  };
  auto by_bt = [&](auto kv, auto hbv) {
    if (bt) launch(kv, hbv, std::true_type());
    else launch(kv, hbv, std::false_type());
  };
  auto by_bias = [&](auto kv) {
    if (a.bias) by_bt(kv, std::true_type());
    else by_bt(kv, std::false_type());
  };
  if (KW == 5) by_bias(std::integral_constant<int, 5>());
  else if (KW == 4) by_bias(std::integral_constant<int, 4>());
  else by_bias(std::integral_constant<int, 3>());
  if (S4 > 1) {
    IAMD_LAUNCH_CHECK();
    const int64_t MC = (int64_t)a.M * Cout;
    const int blocks = (int)std::min<int64_t>((MC / 8 + 255) / 256, 8192);
    hipLaunchKernelGGL(conv_splitk_reduce, dim3(blocks), dim3(256), 0, stream(), a.part, a.bias,
                       a.y, S4, MC, Cout, a.slope, a);
  }
  IAMD_LAUNCH_CHECK();
}

// v5 (row-window, 256 x 256): v4's geometry with Cout % 256 == 0, KW 3 or 5, and output rows
// of >= 32 pixels (the padded segment pitch of 16-pixel rows does not fit the window buffer)
bool v5_shape_ok(const ConvArgs& a) {
  return v4_eligible(a) && a.Cout % 256 == 0 && (a.KW == 3 || a.KW == 5) &&
         (a.Wo % 256 == 0 || a.Wo >= 32);
}

bool v5_eligible(const ConvArgs& a) {
  static const int mode = [] {
    // 0: A/B switch back to v4; 2: every eligible shape, whatever its grid
    const char* e = std::getenv("IMAGINAIRE_AMD_CONV_V5");
    return e == nullptr ? 1 : std::atoi(e);
  }();
  if (mode == 0 || !v5_shape_ok(a)) return false;
  // grids below one 256 x 256 tile per CU split K and reduce; v4's 256 x 128 grid of the same
  // conv is twice as wide: v5 measured 0.57-0.93x v4 on those (G up0 1024 @ 32x64, VGG 256 @
  // 64x128) and 1.06-1.16x on every grid of >= 256 tiles (profiles/conv_v5_probe_mi355x.txt)
  return mode == 2 || (int64_t)(a.M / 256) * (a.Cout / 256) >= 256;
}

void run_v5(ConvArgs& a, const at::Tensor& x) {
  const int Cout = a.Cout, KW = a.KW;
  a.nNt = Cout / 256;
  const int64_t tiles = (int64_t)(a.M / 256) * a.nNt;
  const int nout = a.nk / KW;
  int S = 1;
  if (tiles < 256 && nout >= 8) S = (int)std::min<int64_t>((256 + tiles - 1) / tiles, nout / 4);
  if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_SPLITK")) S = std::max(1, std::atoi(e));
  S = std::max(1, std::min(S, nout));
  a.kps = ceil_div(nout, S);
  S = ceil_div(nout, a.kps);
  at::Tensor part;
  a.part = nullptr;
  if (S > 1) {
    part = at::empty({(int64_t)S * a.M * Cout}, x.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  const dim3 grid((unsigned)tiles, (unsigned)S, 1);
  const bool full = a.Wo % 256 == 0;
  auto launch = [&](auto kv, auto hbv, auto fv) {
    constexpr int K = decltype(kv)::value;
    constexpr bool HB = decltype(hbv)::value, FR = decltype(fv)::value;
    hipLaunchKernelGGL((conv_fwd_mfma_v5<K, HB, FR>), grid, dim3(512), 0, stream(), a);
  };
  auto by_full = [&](auto kv, auto hbv) {
    if (full) launch(kv, hbv, std::true_type());
    else launch(kv, hbv, std::false_type());
  };
  auto by_bias = [&](auto kv) {
    if (a.bias) by_full(kv, std::true_type());
    else by_full(kv, std::false_type());
  };
  if (KW == 5) by_bias(std::integral_constant<int, 5>());
  else by_bias(std::integral_constant<int, 3>());
  if (S > 1) {
    IAMD_LAUNCH_CHECK();
    const int64_t MC = (int64_t)a.M * Cout;
    const int blocks = (int)std::min<int64_t>((MC / 8 + 255) / 256, 8192);
    hipLaunchKernelGGL(conv_splitk_reduce, dim3(blocks), dim3(256), 0, stream(), a.part, a.bias,
                       a.y, S, MC, Cout, a.slope, a);
  }
  IAMD_LAUNCH_CHECK();
}

}  // namespace

// The k10 tile of the most recent conv2d_mfma launch on this host thread (1 = v1, 2, 3, 4, 5,
// 6 = row-window): read by the per-call conv log (ops/conv.py) and the tests.
thread_local int g_last_conv_variant = 0;
int64_t conv_last_variant() { return g_last_conv_variant; }

namespace {

// Kernel choice, split-K and launch for a filled-in ConvArgs (x supplies the tensor options of
// the split-K slabs).
void run_conv(ConvArgs& a, const at::Tensor& x) {
  const int Cout = a.Cout, KH = a.KH, KW = a.KW;
  const bool bn128 = Cout % 128 == 0;
  // Kernel choice (IMAGINAIRE_AMD_CONV_V = 0 auto | 1 | 2 | 3 forces one):
  //  v3 — 8-phase 256 x 256 (Cout % 256 == 0) or 512 x 128 (Cout % 128 == 0) tile, one block
  //       per CU; 1.12-1.22x v1 when every block runs >= 40 K-steps, slower on short K loops
  //       (profiles/conv_v3_probe_mi355x.txt);
  //  v1 — 128 x 128 / 64 tile, two blocks per CU: everything else;
  //  v2 — 256 x 128 3-stage ring: 0.83-0.95x v1 everywhere (profiles/conv_v2_probe_mi355x.txt),
  //       kept for probing only.
  int ver = 0;
  if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_V")) ver = std::atoi(e);
  if (a.nz > 1) ver = 1;  // batched (per-sample weight) launches: v1 only
  const bool v3_ok = bn128 && KH * KW <= 31;
  const int v3_bn = Cout % 256 == 0 ? 256 : 128;
  const int v3_bm = v3_bn == 256 ? 256 : 512;
  // split factor for a grid of `tiles` blocks at `slots` resident blocks
  auto split_for = [&](int64_t tiles, int64_t slots) {
    int S = 1;
    if (tiles < slots && a.nk >= 16) S = (int)std::min<int64_t>((slots + tiles - 1) / tiles, a.nk / 8);
    if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_SPLITK")) S = std::max(1, std::atoi(e));
    S = std::max(1, std::min(S, a.nk));
    return ceil_div(a.nk, ceil_div(a.nk, S));
  };
  if ((ver == 0 && v5_eligible(a)) || (ver == 5 && v5_shape_ok(a))) {
    g_last_conv_variant = 5;
    run_v5(a, x);
    return;
  }
  if ((ver == 4 || ver == 0) && v4_eligible(a)) {
    // default: every eligible conv (1.02-1.52x v1 and 1.0-1.08x v3 on the SPADE-step shapes,
    // the N = 128 data gradients 1.36-1.52x: profiles/conv_v4_probe_mi355x.txt)
    g_last_conv_variant = 4;
    run_v4(a, x, false);
    return;
  }
  // the generalised row-window tile (conv_rw.hip): stride 2, 1x1 / 4x4 / 7x7, Cout = 64,
  // Cin = 32, any output width
  // Default routing (ver 0): the row-window tile where it measured faster than v1 — long
  // filter rows (K = KH*KW*Cin >= 2048 at stride 1: 1.09-1.20x on the 7x7 / 5x5 64-128-channel
  // stems and decoders; >= 6144 at stride 2: 1.18x on the 512-channel PatchGAN layers) — and
  // Cin = 32, which v1 cannot take. Short filters stay on v1: its two co-resident 128-pixel
  // blocks overlap one tile's loads with the other's epilogue, and those convs are latency /
  // bandwidth bound (0.55-0.86x, profiles/conv_rw_probe_mi355x.txt).
  const int64_t kfull = (int64_t)KH * KW * a.Cin;
  const bool rw_pref = a.Cin == 32 || rw_small_pref(a) ||
                       (a.KW >= 3 && ((a.sh == 1 && kfull >= 2048) || (a.sh == 2 && kfull >= 6144)));
  if ((ver == 6 || (ver == 0 && rw_pref)) && run_rw(a, x, ver == 6 || a.Cin == 32)) {
    g_last_conv_variant = 6;
    return;
  }
  IAMD_CHECK(a.Cin % kBK == 0, "conv2d_mfma: Cin = ", a.Cin, " runs on the row-window tile "
             "only, which does not take this shape");
  bool v3 = false, v2 = false;
  if (ver == 3) {
    v3 = v3_ok;
  } else if (ver == 2) {
    v2 = bn128 && KH * KW <= 32;
  } else if (ver == 0 && v3_ok && v3_bn == 256) {
    // (the 512 x 128 variant measured 0.88-0.98x v1 on the 128-channel SPADE / dgrad shapes:
    // selectable with IMAGINAIRE_AMD_CONV_V=3 only)
    // only grids that fill the chip without split-K: with the incremental-cursor v1 the split
    // v3 grids measured 0.87-0.96x v1 (G head 2048 @ 16x32, up0 1024 @ 32x64), the unsplit
    // ones 1.06-1.13x (profiles/conv_v1_cursor_probe_mi355x.txt)
    const int64_t t3 = (int64_t)ceil_div(a.M, v3_bm) * (Cout / v3_bn);
    v3 = split_for(t3, 256) == 1 && a.nk >= 40;
  }
  g_last_conv_variant = v3 ? 3 : v2 ? 2 : 1;
  int bm = 128;
  if (v3) {
    bm = v3_bm;
    a.nNt = Cout / v3_bn;
  } else if (v2) {
    bm = 256;
    a.nNt = Cout / 128;
  } else {
    a.nNt = Cout / (bn128 ? 128 : 64);
    if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_BM")) {
      const int v = std::atoi(e);
      if (v == 128 || v == 256) bm = v;
    }
  }
  if (a.nz > 1) bm = 128;
  const int64_t tiles = (int64_t)ceil_div(a.M, bm) * a.nNt;
  IAMD_CHECK(tiles < (1ll << 31), "conv2d_mfma: grid too large");
  // split-K over (tap, channel-block) k-steps when the tile grid cannot fill the chip (v1: 2
  // blocks per CU, v2 / v3: 1) — the wide-K / narrow-N data gradients of the SPADE gamma/beta
  // convs at 16x32 .. 64x128 and the 2048-channel head convs
  int S = split_for(tiles * a.nz, (v2 || v3) ? 256 : 512);
  a.kps = ceil_div(a.nk, S);
  S = ceil_div(a.nk, a.kps);
  at::Tensor part;
  a.part = nullptr;
  if (S > 1) {
    part = at::empty({(int64_t)S * a.nz * a.M * Cout}, x.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  const dim3 grid((unsigned)tiles, (unsigned)S, (unsigned)a.nz);
  // main-loop schedule: VAR 2 (fragments up front + setprio) measured +1-5% over 0 / 1
  // (scripts/probe/conv_var_probe.py, profiles/conv_var_probe_mi355x.txt)
  int var = 2;
  if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_VAR")) var = std::atoi(e);
  auto launch = [&](auto bmv, auto bnv, auto hbv) {
    constexpr int BM = decltype(bmv)::value;
    constexpr int BN = decltype(bnv)::value;
    constexpr bool HB = decltype(hbv)::value;
    if constexpr (BM == 128) {
      if (var == 1)
        hipLaunchKernelGGL((conv_fwd_mfma<BM, BN, HB, 1>), grid, dim3(BM * 2), 0, stream(), a);
      else if (var == 2)
        hipLaunchKernelGGL((conv_fwd_mfma<BM, BN, HB, 2>), grid, dim3(BM * 2), 0, stream(), a);
      else
        hipLaunchKernelGGL((conv_fwd_mfma<BM, BN, HB, 0>), grid, dim3(BM * 2), 0, stream(), a);
    } else {
      hipLaunchKernelGGL((conv_fwd_mfma<BM, BN, HB, 0>), grid, dim3(BM * 2), 0, stream(), a);
    }
  };
  auto by_bn = [&](auto bmv, auto hbv) {
    if (bn128) launch(bmv, std::integral_constant<int, 128>(), hbv);
    else launch(bmv, std::integral_constant<int, 64>(), hbv);
  };
  auto by_bias = [&](auto bmv) {
    if (a.bias) by_bn(bmv, std::true_type());
    else by_bn(bmv, std::false_type());
  };
  if (v3) {
    if (v3_bn == 256) {
      if (a.bias) hipLaunchKernelGGL((conv_fwd_mfma_v3<256, 256, true>), grid, dim3(512), 0, stream(), a);
      else hipLaunchKernelGGL((conv_fwd_mfma_v3<256, 256, false>), grid, dim3(512), 0, stream(), a);
    } else {
      if (a.bias) hipLaunchKernelGGL((conv_fwd_mfma_v3<512, 128, true>), grid, dim3(512), 0, stream(), a);
      else hipLaunchKernelGGL((conv_fwd_mfma_v3<512, 128, false>), grid, dim3(512), 0, stream(), a);
    }
  } else if (v2) {
    if (a.bias) hipLaunchKernelGGL((conv_fwd_mfma_v2<true>), grid, dim3(512), 0, stream(), a);
    else hipLaunchKernelGGL((conv_fwd_mfma_v2<false>), grid, dim3(512), 0, stream(), a);
  } else if (bm == 256) {
    by_bias(std::integral_constant<int, 256>());
  } else {
    by_bias(std::integral_constant<int, 128>());
  }
  if (S > 1) {
    IAMD_LAUNCH_CHECK();
    const int64_t MC = (int64_t)a.nz * a.M * Cout;
    const int blocks = (int)std::min<int64_t>((MC / 8 + 255) / 256, 8192);
    hipLaunchKernelGGL(conv_splitk_reduce, dim3(blocks), dim3(256), 0, stream(), a.part, a.bias,
                       a.y, S, MC, Cout, a.slope, a);
  }
  IAMD_LAUNCH_CHECK();
}

}  // namespace

// The optional epilogue scale operand: a 1-element fp32 CUDA tensor (sigma) or nothing.
static const float* ascale_ptr(const c10::optional<at::Tensor>& t, const char* who) {
  if (!t.has_value() || !t->defined()) return nullptr;
  IAMD_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == 1, who,
             ": ascale must be a 1-element fp32 CUDA tensor");
  return t->data_ptr<float>();
}

// y[B, Cout, Ho, Wo] (channels-last) = act(conv2d(x, w) + bias), x/w channels-last bf16.
// nb > 1: a batch of nb independent convs with per-sample weights, w [nb * Cout, Cin, KH, KW]
// (sample-major), bias [nb * Cout]: y[b] = act(conv2d(x[b], w[b]) + bias[b]).
at::Tensor conv2d_mfma(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                       int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                       double slope, int64_t nb, int64_t ncv,
                       const c10::optional<at::Tensor>& residual,
                       const c10::optional<at::Tensor>& ascale) {
  IAMD_CHECK(x.is_cuda() && w.is_cuda(), "conv2d_mfma: CUDA tensors expected");
  IAMD_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
             "conv2d_mfma: bf16 operands expected");
  IAMD_CHECK(x.dim() == 4 && w.dim() == 4, "conv2d_mfma: 4-D tensors expected");
  IAMD_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv2d_mfma: packed channels-last operands expected");
  const int B = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  IAMD_CHECK(nb >= 1 && (nb == 1 || B == nb) && w.size(0) % nb == 0,
             "conv2d_mfma: per-sample weights need x batch == nb and w rows % nb == 0");
  const int Cout = (int)(w.size(0) / nb), KH = (int)w.size(2), KW = (int)w.size(3);
  IAMD_CHECK(w.size(1) == Cin, "conv2d_mfma: channel mismatch ", w.size(1), " vs ", Cin);
  IAMD_CHECK(Cin % kBK == 0 || Cin == 32,
             "conv2d_mfma: Cin must be a multiple of 64 (or 32: row-window tile), got ", Cin);
  IAMD_CHECK(Cout % 64 == 0, "conv2d_mfma: Cout must be a multiple of 64, got ", Cout);
  IAMD_CHECK(sh >= 1 && sw >= 1 && dh >= 1 && dw >= 1 && ph >= 0 && pw >= 0, "conv2d_mfma: bad geometry");
  const int Ho = (int)((H + 2 * ph - dh * (KH - 1) - 1) / sh + 1);
  const int Wo = (int)((W + 2 * pw - dw * (KW - 1) - 1) / sw + 1);
  IAMD_CHECK(Ho > 0 && Wo > 0, "conv2d_mfma: empty output");
  IAMD_CHECK((int64_t)B * H * W * Cin * 2 < kOobOffset && w.numel() * 2 < kOobOffset &&
                 (int64_t)B * Ho * Wo * Cout < (1ll << 31),
             "conv2d_mfma: tensor too large for 32-bit buffer offsets");
  IAMD_CHECK(KH * KW <= 64, "conv2d_mfma: filters with more than 64 taps are not supported");
  if (ncv < 0) ncv = Cout;
  IAMD_CHECK(ncv == Cout || (nb == 1 && ncv > 0 && ncv < Cout && ncv % 8 == 0),
             "conv2d_mfma: stored channels must be Cout, or a multiple of 8 below it (nb == 1)");
  auto y = at::empty({B, ncv, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor bf;
  if (bias.has_value() && bias->defined()) {
    IAMD_CHECK(bias->numel() == Cout * nb, "conv2d_mfma: bias size");
    bf = bias->to(at::kFloat).contiguous();
  }
  ConvArgs a;
  a.x = reinterpret_cast<const __hip_bfloat16*>(x.data_ptr());
  a.w = reinterpret_cast<const __hip_bfloat16*>(w.data_ptr());
  a.bias = bf.defined() ? bf.data_ptr<float>() : nullptr;
  a.y = reinterpret_cast<__hip_bfloat16*>(y.data_ptr());
  a.xbytes = (int)(x.numel() / nb * 2);
  a.wbytes = (int)(w.numel() / nb * 2);
  a.nz = (int)nb;
  a.xbs = nb > 1 ? (int64_t)H * W * Cin : 0;
  a.wbs = nb > 1 ? (int64_t)Cout * KH * KW * Cin : 0;
  a.ybs = nb > 1 ? (int64_t)Ho * Wo * Cout : 0;
  a.ldy = (int)ncv;
  a.bbs = nb > 1 ? Cout : 0;
  a.KH = KH;
  a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.KW = KW; a.sh = (int)sh; a.sw = (int)sw; a.ph = (int)ph; a.pw = (int)pw; a.dh = (int)dh; a.dw = (int)dw;
  a.M = (B / (int)nb) * Ho * Wo;
  a.cpt = Cin / kBK;
  a.nk = KH * KW * a.cpt;
  a.slope = (float)slope;
  a.omode = 0;
  a.oH = Ho; a.oW = Wo; a.osy = 1; a.osx = 1; a.ory = 0; a.orx = 0;
  a.res = nullptr;
  if (residual.has_value() && residual->defined()) {
    const at::Tensor& r = *residual;
    IAMD_CHECK(nb == 1 && r.is_cuda() && r.scalar_type() == at::kBFloat16 && r.dim() == 4 &&
                   r.size(0) == B && r.size(1) == ncv && r.size(2) == Ho && r.size(3) == Wo &&
                   r.is_contiguous(at::MemoryFormat::ChannelsLast),
               "conv2d_mfma: the residual must be a packed channels-last bf16 tensor shaped "
               "like the output (single-weight convs only)");
    a.res = reinterpret_cast<const __hip_bfloat16*>(r.data_ptr());
  }
  a.ascale = ascale_ptr(ascale, "conv2d_mfma");
  IAMD_CHECK(a.ascale == nullptr || nb == 1, "conv2d_mfma: ascale is for single-weight convs");
  run_conv(a, x);
  return y;
}


at::Tensor conv_weight_flip_t(const at::Tensor& w, int64_t s, int64_t qy, int64_t qx, int64_t nb);
std::vector<at::Tensor> conv_weight_phase_flip(const at::Tensor& w, int64_t s);

// The transposed-weight (BT) v4 data gradient saves the flipped weight copy (one small
// flip_t pass per backward) but runs 10-35% slower than v4 on the flipped copy: its
// k-major B tile is read with two ds_read_b64_tr_b16 per fragment and the KW = 5 build
// spills (profiles/spade_step_conv_log_mi355x.txt vs the flipped route). Off by default;
// IMAGINAIRE_AMD_DGRAD_BT=1 turns it on.
static bool dgrad_bt_enabled() {
  const char* e = std::getenv("IMAGINAIRE_AMD_DGRAD_BT");
  return e != nullptr && e[0] == '1';
}

// Data gradient of a stride-1, undilated conv with forward weight w [Cout, Cin, KH, KW]
// (channels-last): dx [B, Cin, H, W] = conv(dy, flip_t(w), padding (KH-1-ph, KW-1-pw)). On the v4
// path the forward weight is read directly (tap-flipped, k-major, transposing LDS reads): no
// flipped copy of the weight per backward; other shapes flip once and run the k10 routing.
at::Tensor conv2d_dgrad_mfma(const at::Tensor& dy, const at::Tensor& w, int64_t ph, int64_t pw,
                             int64_t ncv, const c10::optional<at::Tensor>& ascale) {
  IAMD_CHECK(dy.is_cuda() && w.is_cuda() && dy.scalar_type() == at::kBFloat16 &&
                 w.scalar_type() == at::kBFloat16 && dy.dim() == 4 && w.dim() == 4,
             "conv2d_dgrad_mfma: 4-D bf16 CUDA tensors expected");
  IAMD_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv2d_dgrad_mfma: packed channels-last operands expected");
  const int KH = (int)w.size(2), KW = (int)w.size(3);
  IAMD_CHECK(dy.size(1) == w.size(0), "conv2d_dgrad_mfma: dy channels != weight rows");
  IAMD_CHECK(ph <= KH - 1 && pw <= KW - 1 && ph >= 0 && pw >= 0,
             "conv2d_dgrad_mfma: padding outside the filter");
  const int64_t tph = KH - 1 - ph, tpw = KW - 1 - pw;
  const int B = (int)dy.size(0), K = (int)dy.size(1), H = (int)dy.size(2), W = (int)dy.size(3);
  const int N = (int)w.size(1);
  ConvArgs a;
  a.H = H; a.W = W; a.Cin = K; a.Cout = N; a.KH = KH; a.KW = KW;
  a.sh = a.sw = a.dh = a.dw = 1; a.ph = (int)tph; a.pw = (int)tpw;
  a.Ho = H + 2 * (int)tph - (KH - 1);
  a.Wo = W + 2 * (int)tpw - (KW - 1);
  a.nz = 1; a.omode = 0;
  const bool ok = K % kBK == 0 && a.Ho > 0 && a.Wo > 0 && v4_eligible(a) &&
                  (int64_t)B * H * W * K * 2 < kOobOffset && w.numel() * 2 < kOobOffset &&
                  (int64_t)B * a.Ho * a.Wo * N < (1ll << 31) && dgrad_bt_enabled();
  if (!ok) {
    const at::Tensor wt = conv_weight_flip_t(w, 1, 0, 0, 1);
    return conv2d_mfma(dy, wt, c10::nullopt, 1, 1, tph, tpw, 1, 1, 1.0, 1, ncv, c10::nullopt,
                       ascale);
  }
  if (ncv < 0) ncv = N;
  IAMD_CHECK(ncv == N || (ncv > 0 && ncv < N && ncv % 8 == 0),
             "conv2d_dgrad_mfma: stored channels must be Cin or a multiple of 8 below it");
  auto y = at::empty({B, ncv, a.Ho, a.Wo}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  a.x = reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr());
  a.w = reinterpret_cast<const __hip_bfloat16*>(w.data_ptr());
  a.bias = nullptr;
  a.y = reinterpret_cast<__hip_bfloat16*>(y.data_ptr());
  a.xbytes = (int)(dy.numel() * 2);
  a.wbytes = (int)(w.numel() * 2);
  a.xbs = a.wbs = a.ybs = 0;
  a.bbs = 0;
  a.ldy = (int)ncv;
  a.M = B * a.Ho * a.Wo;
  a.cpt = K / kBK;
  a.nk = KH * KW * a.cpt;
  a.slope = 1.f;
  a.oH = a.Ho; a.oW = a.Wo; a.osy = 1; a.osx = 1; a.ory = 0; a.orx = 0;
  a.res = nullptr;
  a.ascale = ascale_ptr(ascale, "conv2d_dgrad_mfma");
  run_v4(a, dy, true);
  return y;
}


// Data gradient of a stride-s conv (s = 2..4, undilated; w [Cout, Cin, KH, KW] channels-last
// bf16) as its s*s phase convolutions in ONE k10 launch (blockIdx.z = phase), each phase
// storing straight into its parity sub-grid of dx: input row i = s q + r receives
// sum_j dy[q + c - j] w[k0 + s j] (k0 = (r + p) mod s, c = (r + p - k0) / s), i.e. a J-tap
// correlation of dy with the flipped phase sub-kernel at padding J - 1 - c (negative where the
// phase starts inside dy). Replaces per phase one launch + one scatter pass
// (ops/conv.py _strided_dgrad). ncv: channels of dx stored (<= Cin, multiple of 8).
at::Tensor conv2d_dgrad_strided(const at::Tensor& dy, const at::Tensor& w, int64_t s, int64_t ph,
                                int64_t pw, int64_t H, int64_t W, int64_t ncv,
                                const c10::optional<at::Tensor>& ascale) {
  IAMD_CHECK(dy.is_cuda() && w.is_cuda() && dy.scalar_type() == at::kBFloat16 &&
                 w.scalar_type() == at::kBFloat16 && dy.dim() == 4 && w.dim() == 4,
             "conv2d_dgrad_strided: 4-D bf16 CUDA tensors expected");
  IAMD_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 w.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv2d_dgrad_strided: packed channels-last operands expected");
  const int B = (int)dy.size(0), K = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  const int N = (int)w.size(1), KH = (int)w.size(2), KW = (int)w.size(3);
  IAMD_CHECK(w.size(0) == K, "conv2d_dgrad_strided: dy channels != weight rows");
  IAMD_CHECK(s >= 2 && s <= 4 && K % kBK == 0 && N % 64 == 0 && ph >= 0 && pw >= 0 &&
                 ph < KH && pw < KW,
             "conv2d_dgrad_strided: unsupported geometry");
  IAMD_CHECK(Ho == (H + 2 * ph - KH) / s + 1 && Wo == (W + 2 * pw - KW) / s + 1,
             "conv2d_dgrad_strided: dy size does not match the conv geometry");
  IAMD_CHECK((int64_t)B * Ho * Wo * K * 2 < kOobOffset && (int64_t)B * H * W * N < (1ll << 31),
             "conv2d_dgrad_strided: tensors too large for 32-bit offsets");
  if (ncv < 0) ncv = N;
  IAMD_CHECK(ncv == N || (ncv > 0 && ncv < N && ncv % 8 == 0),
             "conv2d_dgrad_strided: stored channels must be Cin or a multiple of 8 below it");
  auto dx = at::empty({B, ncv, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  std::vector<ConvArgs> phases;
  // every phase's flipped sub-kernel in one launch (views of one buffer, freed on this stream
  // after the kernels below)
  const std::vector<at::Tensor> pw_all = conv_weight_phase_flip(w, s);
  bool zero_fill = false;
  const bool bn128 = N % 128 == 0;
  const int BN = bn128 ? 128 : 64;
  for (int ry = 0; ry < s; ++ry) {
    for (int rx = 0; rx < s; ++rx) {
      const int ky0 = (int)((ry + ph) % s), kx0 = (int)((rx + pw) % s);
      const int jy = (int)((KH - ky0 + s - 1) / s), jx = (int)((KW - kx0 + s - 1) / s);
      const int qy = (int)((H - ry + s - 1) / s), qx = (int)((W - rx + s - 1) / s);
      if (jy <= 0 || jx <= 0 || qy <= 0 || qx <= 0) {
        zero_fill = zero_fill || (qy > 0 && qx > 0);
        continue;
      }
      const int cy = (int)((ry + ph - ky0) / s), cx = (int)((rx + pw - kx0) / s);
      const at::Tensor& wt = pw_all[ky0 * s + kx0];  // [N, K, jy, jx]
      ConvArgs a;
      a.x = reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr());
      a.w = reinterpret_cast<const __hip_bfloat16*>(wt.data_ptr());
      a.bias = nullptr;
      a.y = reinterpret_cast<__hip_bfloat16*>(dx.data_ptr());
      a.res = nullptr;
      a.xbytes = (int)(dy.numel() * 2);
      a.wbytes = (int)(wt.numel() * 2);
      a.H = Ho; a.W = Wo; a.Cin = K; a.Cout = N;
      a.KH = jy; a.KW = jx; a.sh = a.sw = a.dh = a.dw = 1;
      a.ph = jy - 1 - cy; a.pw = jx - 1 - cx;  // (may be negative: the phase starts inside dy)
      a.Ho = qy; a.Wo = qx;
      a.M = B * qy * qx;
      a.cpt = K / kBK;
      a.nk = jy * jx * a.cpt;
      a.kps = a.nk;
      a.nNt = N / BN;
      a.part = nullptr;
      a.slope = 1.f;
      a.omode = 1; a.oH = (int)H; a.oW = (int)W; a.osy = (int)s; a.osx = (int)s;
      a.ory = ry; a.orx = rx;
      a.xbs = a.wbs = a.ybs = 0; a.bbs = 0; a.nz = 1;
      a.ldy = (int)ncv;
      a.ascale = ascale_ptr(ascale, "conv2d_dgrad_strided");
      phases.push_back(a);
    }
  }
  if (zero_fill) dx.zero_();
  g_last_conv_variant = 7;  // (v1 phase tiles)
  // up to four phases per launch (the ConvPhases kernel argument; s = 3, 4 take several)
  for (size_t p0 = 0; p0 < phases.size(); p0 += 4) {
    ConvPhases P;
    int np = 0, maxtiles = 0;
    for (size_t i = p0; i < phases.size() && np < 4; ++i, ++np) {
      P.a[np] = phases[i];
      P.tiles[np] = ceil_div(P.a[np].M, 128) * P.a[np].nNt;
      maxtiles = std::max(maxtiles, P.tiles[np]);
    }
    for (int i = np; i < 4; ++i) {
      P.a[i] = phases[p0];
      P.tiles[i] = 0;
    }
    const dim3 grid((unsigned)maxtiles, 1, (unsigned)np);
    if (bn128)
      hipLaunchKernelGGL((conv_fwd_mfma_phases<128, 128>), grid, dim3(256), 0, stream(), P);
    else
      hipLaunchKernelGGL((conv_fwd_mfma_phases<128, 64>), grid, dim3(256), 0, stream(), P);
    IAMD_LAUNCH_CHECK();
  }
  return dx;  // (the phase weights are freed on this stream, after the kernel)
}

}  // namespace iamd
