// k11: weight gradient of the k10 convolution on the gfx950 matrix cores.
//
//   dW[n][ky][kx][ci] = sum_m dy[m][n] * x[b][oh*sh - ph + ky*dh][ow*sw - pw + kx*dw][ci]
//
// over all output pixels m = (b, oh, ow). As a GEMM the reduction dimension (pixels) is the
// OUTER, strided dimension of both NHWC operands, so both MFMA fragments are read with the
// gfx950 transposing LDS read ds_read_b64_tr_b16: each 16-lane group fetches a 4-pixel x
// 16-channel block and every lane receives one channel's 4 pixels (cdna_hip_programming.md
// T10). Two such reads make the 8-deep k-fragment of v_mfma_f32_16x16x32_bf16.
//
// Block: one filter tap x BNO output channels x BC input channels, reducing over a
// contiguous range of 64-pixel k-steps (split-K over pixels so small-tap-count layers still
// fill 256 CUs). Both 64-pixel tiles are staged global -> LDS with global_load_lds_dwordx4
// into two buffers (the stage of step k+1 overlaps the MFMAs of step k). The LDS images are
// [pixel][channel] rows whose 16-byte chunks are XOR-swizzled per row (on the global side:
// the DMA write is lane-linear) so that the 8 rows a 32-lane half of a transposed read
// touches fall into 8 different 32-byte bank windows: conflict-free. The DMA is
// buffer_load ... lds: out-of-image input pixels (padding) and the pixel tail get an
// out-of-range offset and read as zeros; when Wo % 64 == 0 a k-step is one output-row
// segment and its pixel coordinates are wave-uniform scalars. Partial sums per split are
// written as fp32 slabs [S][Cout][taps][Cin] and summed by a second, bandwidth-bound kernel
// that also crops padded channels and casts to the parameter dtype (conv_aux.hip
// wgrad_finalize); one fp32 uncropped slab (S == 1) is written straight into dW.
//
// Reference: the reference's weight gradients come from cuDNN through nn.Conv2d autograd
// (layers/conv.py:59-91); there is no hand-written conv in the reference.
#include "common.h"

namespace iamd {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) bf16x4* lds_bf16x4_t;

constexpr int kBP = 64;  // pixels per k-step
constexpr int kThreads = 256;

// buffer-resource word 3 for raw (unformatted, stride-0) buffers on gfx9-family parts
constexpr int kBufCfg = 0x00020000;
// a byte offset past every tensor this kernel accepts: the buffer unit returns zeros for it
constexpr int kOobOffset = 0x7ffffff0;

struct WgradArgs {
  const __hip_bfloat16* dy;  // [M][Cout]
  const __hip_bfloat16* x;   // [B][H][W][Cin]
  float* out;                // [S][Cout][KK][Cin]
  int dybytes, xbytes;
  int Bn, H, W, Cin, Ho, Wo, Cout, KW, KK;
  int sh, sw, ph, pw, dh, dw;
  int M, nks, kps, nNt, nCt;
  // batch of independent weight gradients (per-sample weights), one per blockIdx.y: operand
  // strides in elements between samples; slabs are [S][nz][Cout][KK][Cin]
  int64_t dybs, xbs;
  // spectrally normalised weight (layers/spectral_norm.py): the epilogue also sums G * W over
  // the block's outputs (W = the bf16 shadow, real dims [wsn_cout][KK][wsn_cin]) into
  // dotp[blockIdx.x]; their total is <G, W> for the SN backward, folded into wgrad_finalize_sn
  const __hip_bfloat16* wsn = nullptr;
  float* dotp = nullptr;
  int wsn_cout = 0, wsn_cin = 0;
};

// one output's share of <G, W> (outputs in the zero-padded channel tail contribute nothing).
// Branch-free: the load always runs (clamped into the real weight in the tail) so the compiler can issue
// every load of the epilogue back to back; a load under a per-element branch got its own
// vmcnt(0) wait, serialising ~100 round trips per thread.
__device__ __forceinline__ float sn_term(const WgradArgs& a, int n, int tap, int ci, float gv) {
  const int nn = min(n, a.wsn_cout - 1), cc = min(ci, a.wsn_cin - 1);
  const float w = __bfloat162float(a.wsn[(nn * a.KK + tap) * a.wsn_cin + cc]);
  return (n < a.wsn_cout && ci < a.wsn_cin) ? gv * w : 0.f;
}

// block total of the per-thread <G, W> shares -> dotp[blockIdx.x] (fixed order: deterministic).
// The epilogues sum their shares BEFORE writing the slab: with the slab stores interleaved, every
// W load's wait would also wait for the stores issued before it (vmcnt counts both on CDNA).
__device__ void sn_dot_store(const WgradArgs& a, float d) {
  __shared__ float red[kThreads / 64];
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) t += red[k];
    a.dotp[blockIdx.x] = t;
  }
}

// 16-byte chunk swizzle of a [64 pixel rows][RB bytes] image: the 8 rows read by one 32-lane
// half of a transposed fragment read land in distinct 32-byte bank windows.
template <int RB>
__device__ __forceinline__ int swz(int row) {
  if constexpr (RB == 256) {
    return ((row & 3) << 2) | ((row >> 2) & 3);
  } else {
    return ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1);
  }
}

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)p);
}

template <int BNO, int BC, bool ROWS, int NST>
__global__ __launch_bounds__(kThreads, 2) void conv_wgrad_mfma(WgradArgs a) {
  // The buffer-resource builtins have no host form; the host pass only needs the launch stub.
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int RA = BNO * 2, RX = BC * 2;        // image row bytes
  constexpr int kAbytes = kBP * RA, kXbytes = kBP * RX;
  constexpr int kStage = kAbytes + kXbytes;
  constexpr int MI = BNO / 32, NI = BC / 32;      // 16-wide fragments per wave
  constexpr int CPA = RA / 16, CPX = RX / 16;     // chunks per image row
  constexpr int LA = kBP * CPA / kThreads;        // glds per thread (dy tile)
  constexpr int LX = kBP * CPX / kThreads;        // glds per thread (x tile)
  constexpr int RSA = kThreads / CPA, RSX = kThreads / CPX;  // rows per glds round
  __shared__ __attribute__((aligned(16))) char smem[NST * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = a.KK * a.nNt * a.nCt;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int tap = tile / (a.nNt * a.nCt);
  const int r2 = tile - tap * a.nNt * a.nCt;
  const int nt = r2 / a.nCt, ct = r2 - nt * a.nCt;
  const int n0 = nt * BNO, c0 = ct * BC;
  const int ky = tap / a.KW, kx = tap - ky * a.KW;
  const int ks0 = split * a.kps;
  const int ks1 = min(a.nks, ks0 + a.kps);

  // ---- DMA bookkeeping ------------------------------------------------------------------
  // buffer_load ... lds: per-lane 32-bit byte offsets, wave-uniform parts in SGPRs, and an
  // out-of-range offset (padding pixels, pixel tail) reads as zeros.
  const int zb = blockIdx.y;  // sample of a batched (per-sample weight) launch
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.dy + (size_t)zb * a.dybs), 0, a.dybytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x + (size_t)zb * a.xbs), 0, a.xbytes, kBufCfg);
  const int arow0 = tid / CPA, apos = tid % CPA;
  const int xrow0 = tid / CPX, xpos = tid % CPX;
  const int dyc = n0 + ((apos ^ swz<RA>(arow0)) << 3);  // rows arow0 + i*RSA share row&15
  const int xc = c0 + ((xpos ^ swz<RX>(xrow0)) << 3);
  int dy_off[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) dy_off[i] = ((arow0 + i * RSA) * a.Cout + dyc) * 2;
  const int dy_step = kBP * a.Cout * 2;
  const int HoWo = a.Ho * a.Wo;
  // ROWS (Wo % 64 == 0): a k-step is 64 consecutive pixels of ONE output row, so (b, oh, ow0)
  // are wave-uniform scalars advanced by 64 per step; otherwise each lane tracks its pixels.
  int sb = 0, soh = 0, sow = 0;
  int xb[LX], xoh[LX], xow[LX];
  if constexpr (ROWS) {
    const int m = ks0 * kBP;
    sb = m / HoWo;
    const int r = m - sb * HoWo;
    soh = r / a.Wo;
    sow = r - soh * a.Wo;
  } else {
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int m = ks0 * kBP + xrow0 + i * RSX;
      const int b = m / HoWo, r = m - b * HoWo;
      xb[i] = b;
      xoh[i] = r / a.Wo;
      xow[i] = r - xoh[i] * a.Wo;
    }
  }

  auto issue = [&](int ks, int buf) {
    char* As = smem + buf * kStage;
    char* Xs = As + kAbytes;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (lds_ptr_t)(As + i * 4096 + wid * 1024), 16,
                                               dy_off[i], ks * dy_step, 0, 0);
    if constexpr (ROWS) {
      const int ih = soh * a.sh - a.ph + ky * a.dh;
      const bool rowok = sb < a.Bn && (unsigned)ih < (unsigned)a.H;
      const int soff = rowok ? (sb * a.H + ih) * a.W * a.Cin * 2 : 0;
#pragma unroll
      for (int i = 0; i < LX; ++i) {
        const int iw = (sow + xrow0 + i * RSX) * a.sw - a.pw + kx * a.dw;
        const bool ok = rowok && (unsigned)iw < (unsigned)a.W;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(Xs + i * 4096 + wid * 1024), 16,
                                                 ok ? (iw * a.Cin + xc) * 2 : kOobOffset, soff,
                                                 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < LX; ++i) {
        const int ih = xoh[i] * a.sh - a.ph + ky * a.dh;
        const int iw = xow[i] * a.sw - a.pw + kx * a.dw;
        const bool ok = xb[i] < a.Bn && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xrs, (lds_ptr_t)(Xs + i * 4096 + wid * 1024), 16,
            ok ? (((xb[i] * a.H + ih) * a.W + iw) * a.Cin + xc) * 2 : kOobOffset, 0, 0, 0);
      }
    }
  };
  auto advance = [&]() {
    if constexpr (ROWS) {
      sow += kBP;
      if (sow >= a.Wo) {
        sow = 0;
        if (++soh >= a.Ho) { soh = 0; ++sb; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LX; ++i) {
        xow[i] += kBP;
        while (xow[i] >= a.Wo) { xow[i] -= a.Wo; ++xoh[i]; }
        while (xoh[i] >= a.Ho) { xoh[i] -= a.Ho; ++xb[i]; }
      }
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: group g reads pixel rows 8g + q (and + 4), lane p's
  // 8-byte quarter of the group's 16-channel (32-byte) column block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto a_addr = [&](int row, int colblk) {  // colblk: first channel / 8 of the 16-ch block
    return row * RA + ((((colblk + (p >> 1)) ^ swz<RA>(row))) << 4) + ((p & 1) << 3);
  };
  auto x_addr = [&](int row, int colblk) {
    return row * RX + ((((colblk + (p >> 1)) ^ swz<RX>(row))) << 4) + ((p & 1) << 3);
  };

  // both 32-pixel halves of the k-step read up front, then the MFMAs (see conv_wgrad_mfma_mt)
  auto compute = [&](int buf) {
    const char* As = smem + buf * kStage;
    const char* Xs = As + kAbytes;
    bf16x8 af[2][MI], xf[2][NI];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = kk * 32 + g * 8 + q;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int cb = (wm * (BNO / 2) + i * 16) >> 3;
        const bf16x4 lo = tr_read(As + a_addr(r0, cb));
        const bf16x4 hi = tr_read(As + a_addr(r0 + 4, cb));
        af[kk][i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int cb = (wn * (BC / 2) + j * 16) >> 3;
        const bf16x4 lo = tr_read(Xs + x_addr(r0, cb));
        const bf16x4 hi = tr_read(Xs + x_addr(r0 + 4, cb));
        xf[kk][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], xf[kk][j], acc[i][j],
                                                              0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (NST == 2) {
    // unrolled over the two buffers: fragment addresses = invariant register + immediate
    auto step = [&](int ks, int b) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (ks + 1 < ks1) {
        advance();
        issue(ks + 1, b ^ 1);
      }
      compute(b);
    };
    issue(ks0, 0);
    for (int ks = ks0; ks < ks1; ks += 2) {
      step(ks, 0);
      if (ks + 1 < ks1) step(ks + 1, 1);
    }
  } else {
    // three-stage ring, counted vmcnt (LA + LX glds per thread per stage), raw barrier: see
    // conv_wgrad_mfma_mt
    const int nks = ks1 - ks0;
    issue(ks0, 0);
    if (nks > 1) {
      advance();
      issue(ks0 + 1, 1);
    }
    int rb = 0;
    for (int it = 0; it < nks; ++it) {
      if (it + 1 < nks)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LA + LX) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (it + 2 < nks) {
        advance();
        issue(ks0 + it + 2, rb == 0 ? 2 : rb - 1);
      }
      compute(rb);
      rb = rb == 2 ? 0 : rb + 1;
    }
  }

  // ---- fp32 partial slab: row n (4 per lane), column ci (16 lanes contiguous) -------------
  float* o = a.out + ((size_t)split * gridDim.y + zb) * a.Cout * a.KK * a.Cin;
  if (a.wsn) {  // <G, W> share first (see sn_dot_store)
    float sd = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sd += sn_term(a, n0 + wm * (BNO / 2) + i * 16 + g * 4 + r, tap,
                        c0 + wn * (BC / 2) + j * 16 + (lane & 15), acc[i][j][r]);
    sn_dot_store(a, sd);
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * (BNO / 2) + i * 16 + g * 4 + r;
        const int ci = c0 + wn * (BC / 2) + j * 16 + (lane & 15);
        o[((size_t)n * a.KK + tap) * a.Cin + ci] = acc[i][j][r];
      }
#endif  // __HIP_DEVICE_COMPILE__
}

// ---- k11 multi-tap: one block computes ALL KW taps of one filter row ------------------------
//
// For a stride-1 conv whose output rows are whole 64-pixel k-steps (Wo % 64 == 0), the KW taps
// (ky, 0..KW-1) of one filter row read the SAME dy tile and the same input row shifted by kx
// pixels. The block stages the dy tile (64 px x BNO) and ONE input-row window of 64 + KW - 1
// pixels x BC once per k-step and runs the KW tap products from LDS (the x fragment of tap kx is
// the window read kx rows further down), so every staged byte feeds KW times the MFMAs of the
// one-tap kernel: 3x / 5x fewer L2 -> LDS bytes per FLOP on the 3x3 / 5x5 SPADE convs, and the dy
// fragments are read from LDS once for all taps. Accumulators: KW x (BNO/2 x BC/2) per wave
// (tiles: 3 taps 128 x 64, 5 / 7 taps 64 x 64 — the 256-VGPR budget of 2 waves / SIMD, no
// spills).
template <int BNO, int BC, int NT, int NST>
__global__ __launch_bounds__(kThreads, (NT == 5 && BNO == 64) ? 3 : 2) void conv_wgrad_mfma_mt(
    WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int RA = BNO * 2, RX = BC * 2;        // image row bytes
  constexpr int kAbytes = kBP * RA;
  constexpr int kXrows = kBP + 1024 / RX;           // window + one extra wave-DMA of halo rows
  static_assert(NT - 1 <= 1024 / RX, "halo rows must fit one extra wave DMA");
  constexpr int kXbytes = kXrows * RX;
  constexpr int kStage = kAbytes + kXbytes;
  constexpr int MI = BNO / 32, NI = BC / 32;
  constexpr int CPA = RA / 16, CPX = RX / 16;
  constexpr int LA = kBP * CPA / kThreads;
  constexpr int LX = kBP * CPX / kThreads;
  constexpr int RSA = kThreads / CPA, RSX = kThreads / CPX;
  __shared__ __attribute__((aligned(16))) char smem[NST * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = a.KK / a.KW * a.nNt * a.nCt;    // (ky, n-tile, c-tile)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int ky = tile / (a.nNt * a.nCt);
  const int r2 = tile - ky * a.nNt * a.nCt;
  const int nt = r2 / a.nCt, ct = r2 - nt * a.nCt;
  const int n0 = nt * BNO, c0 = ct * BC;
  const int ks0 = split * a.kps;
  const int ks1 = min(a.nks, ks0 + a.kps);

  const int zb = blockIdx.y;  // sample of a batched (per-sample weight) launch
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.dy + (size_t)zb * a.dybs), 0, a.dybytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x + (size_t)zb * a.xbs), 0, a.xbytes, kBufCfg);
  const int arow0 = tid / CPA, apos = tid % CPA;
  const int xrow0 = tid / CPX, xpos = tid % CPX;
  const int dyc = n0 + ((apos ^ swz<RA>(arow0)) << 3);
  const int xc = c0 + ((xpos ^ swz<RX>(xrow0)) << 3);
  int dy_off[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) dy_off[i] = ((arow0 + i * RSA) * a.Cout + dyc) * 2;
  const int dy_step = kBP * a.Cout * 2;
  // halo rows 64.. of the window: wave 0 only, one lane-linear 1 KB DMA
  const int hrow = kBP + lane / CPX;
  const int hxc = c0 + (((lane % CPX) ^ swz<RX>(hrow)) << 3);
  const int HoWo = a.Ho * a.Wo;
  int sb, soh, sow;
  {
    const int m = ks0 * kBP;
    sb = m / HoWo;
    const int r = m - sb * HoWo;
    soh = r / a.Wo;
    sow = r - soh * a.Wo;
  }

  auto issue = [&](int ks, int buf) {
    char* As = smem + buf * kStage;
    char* Xs = As + kAbytes;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (lds_ptr_t)(As + i * 4096 + wid * 1024), 16,
                                               dy_off[i], ks * dy_step, 0, 0);
    const int ih = soh * a.sh - a.ph + ky * a.dh;
    const bool rowok = sb < a.Bn && (unsigned)ih < (unsigned)a.H;
    const int soff = rowok ? (sb * a.H + ih) * a.W * a.Cin * 2 : 0;
    const int iw0 = sow - a.pw;  // input column of window row 0 (stride 1)
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int iw = iw0 + xrow0 + i * RSX;
      const bool ok = rowok && (unsigned)iw < (unsigned)a.W;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(Xs + i * 4096 + wid * 1024), 16,
                                               ok ? (iw * a.Cin + xc) * 2 : kOobOffset, soff, 0,
                                               0);
    }
    if (wid == 0) {
      const int iw = iw0 + hrow;
      const bool ok = rowok && (unsigned)iw < (unsigned)a.W;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(Xs + kBP * RX), 16,
                                               ok ? (iw * a.Cin + hxc) * 2 : kOobOffset, soff, 0,
                                               0);
    }
  };
  auto advance = [&]() {
    sow += kBP;
    if (sow >= a.Wo) {
      sow = 0;
      if (++soh >= a.Ho) { soh = 0; ++sb; }
    }
  };

  f32x4 acc[NT][MI][NI];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto a_addr = [&](int row, int colblk) {
    return row * RA + ((((colblk + (p >> 1)) ^ swz<RA>(row))) << 4) + ((p & 1) << 3);
  };
  auto x_addr = [&](int row, int colblk) {
    return row * RX + ((((colblk + (p >> 1)) ^ swz<RX>(row))) << 4) + ((p & 1) << 3);
  };

  // one k-step of MFMAs on the staged LDS buffer ``buf``. Every fragment of the k-step (both
  // 32-pixel halves: MI dy + NT x NI x fragments each) is read into registers BEFORE the first
  // MFMA, so the LDS latency is paid once per k-step and overlaps the first half's MFMAs,
  // instead of a read -> lgkmcnt(0) -> 4 MFMAs stall per tap (what the compiler emits when the
  // tap fragments share one register set: profiles/wgrad_sched_probe_mi355x.txt).
  // 5 taps: one half at a time (48 fragment registers instead of 96: 168 VGPRs, three blocks
  // per CU — the 5x5 shapes whose tile grid needs no split-K fill 768 block slots in one round)
  constexpr int NH = NT >= 5 ? 1 : 2;  // 32-pixel halves whose fragments are read together
  // 128 x 64 tile with 5 taps: 160 accumulator registers leave no room for all 10 x fragments
  // of a half, so the x fragments of tap t + 1 are read while tap t's MFMAs run (two buffers)
  constexpr bool kTapPipe = BNO == 128 && NT == 5;
  auto compute_tap_pipe = [&](int buf, int h) {
    const char* As = smem + buf * kStage;
    const char* Xs = As + kAbytes;
    // the lane geometry is re-derived from an opaque copy of the lane id on every call, so the
    // compiler recomputes the fragment addresses (a few VALU) instead of keeping all of them
    // live across the k loop (which spilled)
    int l = lane;
    asm volatile("" : "+v"(l));
    const int lg = l >> 4, lq = (l >> 2) & 3, lp = l & 3;
    auto a_addr = [&](int row, int colblk) {
      return row * RA + ((((colblk + (lp >> 1)) ^ swz<RA>(row))) << 4) + ((lp & 1) << 3);
    };
    auto x_addr = [&](int row, int colblk) {
      return row * RX + ((((colblk + (lp >> 1)) ^ swz<RX>(row))) << 4) + ((lp & 1) << 3);
    };
    const int r0 = h * 32 + lg * 8 + lq;
    bf16x8 af[MI], xf[2][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int cb = (wm * (BNO / 2) + i * 16) >> 3;
      const bf16x4 lo = tr_read(As + a_addr(r0, cb));
      const bf16x4 hi = tr_read(As + a_addr(r0 + 4, cb));
      af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    auto read_x = [&](int t, bf16x8 (&dst)[NI]) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int cb = (wn * (BC / 2) + j * 16) >> 3;
        const bf16x4 lo = tr_read(Xs + x_addr(r0 + t, cb));
        const bf16x4 hi = tr_read(Xs + x_addr(r0 + t + 4, cb));
        dst[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    read_x(0, xf[0]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t + 1 < NT) read_x(t + 1, xf[(t + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], xf[t & 1][j],
                                                                 acc[t][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  auto compute_halves = [&](int buf, int h0) {
    const char* As = smem + buf * kStage;
    const char* Xs = As + kAbytes;
    bf16x8 af[NH][MI], xf[NH][NT][NI];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      const int r0 = (h0 + hh) * 32 + g * 8 + q;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int cb = (wm * (BNO / 2) + i * 16) >> 3;
        const bf16x4 lo = tr_read(As + a_addr(r0, cb));
        const bf16x4 hi = tr_read(As + a_addr(r0 + 4, cb));
        af[hh][i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cb = (wn * (BC / 2) + j * 16) >> 3;
          const bf16x4 lo = tr_read(Xs + x_addr(r0 + t, cb));
          const bf16x4 hi = tr_read(Xs + x_addr(r0 + t + 4, cb));
          xf[hh][t][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[hh][i], xf[hh][t][j],
                                                                   acc[t][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto compute = [&](int buf) {
    if constexpr (kTapPipe) {
      compute_tap_pipe(buf, 0);
      compute_tap_pipe(buf, 1);
    } else {
#pragma unroll
      for (int h0 = 0; h0 < 2; h0 += NH) compute_halves(buf, h0);
    }
  };

  if constexpr (NST == 2) {
    // two LDS buffers: every k-step drains its DMA (vmcnt(0) + barrier) before the MFMAs;
    // the second co-resident block hides the wait. The loop is unrolled over the two buffers
    // so every fragment address is a loop-invariant register plus an immediate offset (no
    // per-read address VALU).
    auto step = [&](int ks, int b) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (ks + 1 < ks1) {
        advance();
        issue(ks + 1, b ^ 1);
      }
      compute(b);
    };
    issue(ks0, 0);
    for (int ks = ks0; ks < ks1; ks += 2) {
      step(ks, 0);
      if (ks + 1 < ks1) step(ks + 1, 1);
    }
  } else {
    // three-stage ring (cdna_hip_programming.md "Pipelining across barriers"): the DMA of
    // k-step it+1 stays in flight across the barrier of k-step it, retired by a counted
    // vmcnt (this wave's glds per stage: LA + LX, plus the halo piece on wave 0) — never 0
    // inside the loop — and a raw s_barrier (a __syncthreads fence would drain it). The
    // barrier of k-step it also tells every wave that buffer (it+2) % 3 = (it-1) % 3 has been
    // read, so the DMA of k-step it+2 is issued right after it.
    const int nks = ks1 - ks0;
    issue(ks0, 0);
    if (nks > 1) {
      advance();
      issue(ks0 + 1, 1);
    }
    int rb = 0;
    for (int it = 0; it < nks; ++it) {
      if (it + 1 < nks) {
        if (wid == 0)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LA + LX + 1) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LA + LX) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (it + 2 < nks) {
        advance();
        issue(ks0 + it + 2, rb == 0 ? 2 : rb - 1);
      }
      compute(rb);
      rb = rb == 2 ? 0 : rb + 1;
    }
  }

  float* o = a.out + ((size_t)split * gridDim.y + zb) * a.Cout * a.KK * a.Cin;
  if (a.wsn) {  // <G, W> share first (see sn_dot_store)
    float sd = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sd += sn_term(a, n0 + wm * (BNO / 2) + i * 16 + g * 4 + r, ky * a.KW + t,
                          c0 + wn * (BC / 2) + j * 16 + (lane & 15), acc[t][i][j][r]);
    sn_dot_store(a, sd);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = ky * a.KW + t;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wm * (BNO / 2) + i * 16 + g * 4 + r;
          const int ci = c0 + wn * (BC / 2) + j * 16 + (lane & 15);
          o[((size_t)n * a.KK + tap) * a.Cin + ci] = acc[t][i][j][r];
        }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

// ---- k11 v2: 128 x 128 x KW-tap tile, one wave per SIMD ----------------------------------
//
// The multi-tap kernel above keeps two blocks (8 waves) per CU, which caps a wave at 256 VGPRs
// and its tile at 32 x 32 per tap (5 taps): every MFMA then needs ~0.6 KB of LDS fragment
// reads, close to the CU's 1 KB-per-16x16x32-MFMA LDS budget once the DMA writes are added.
// This kernel runs ONE 256-thread block per CU (one wave per SIMD, up to 512 VGPR/AGPR) with
// a 64 (Cout) x 64 (Cin) x KW-tap accumulator per wave (KW = 5: 320 accumulators), so a
// 32-pixel k-fragment of dy (4 fragments) is read once for all KW taps and every x fragment
// feeds 4 MFMAs: ~0.3 KB of LDS reads per MFMA. The block owns 128 output x 128 input
// channels of one filter row ky and stages, per 64-pixel k-step, the dy tile (64 px x 128 ch)
// and ONE input window per output-row segment — R = 64 / WSEG segments of WSEG output pixels,
// each needing WSEG + KW - 1 input pixels (rows padded to L: the k-fragment offsets stay
// multiples of 16 rows, where the 16-B chunk swizzle repeats) — so each staged x byte feeds KW
// taps. Output rows shorter than 64 pixels (16 x 32 / 32 x 64 maps, WSEG = 16 / 32) are
// covered too: a 32-pixel k-fragment never straddles a segment. Staging is buffer_load ...
// lds (zeros for padding pixels) into an NST-deep ring, drained by a counted vmcnt (never 0
// in the loop) and a raw s_barrier, so the next k-steps' DMA stays in flight while this one
// computes; the single wave per SIMD relies on that depth instead of a co-resident block.
template <int NT, int BC, int WSEG, int NST>
__global__ __launch_bounds__(kThreads, 1) void conv_wgrad_mfma_w4(WgradArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int RB = 256;                                   // dy row bytes (128 channels)
  constexpr int RX = BC * 2;                                // x row bytes
  constexpr int NJ = BC / 32;                               // 16-channel x fragments per wave
  constexpr int R = kBP / WSEG;                             // window segments per k-step
  constexpr int L = WSEG == 64 ? 64 + NT - 1 : (WSEG + NT - 1 + 15) / 16 * 16;
  constexpr int XRPR = 1024 / (BC * 2);                     // x rows per wave DMA instruction
  constexpr int XROWS = (R * L + 4 * XRPR - 1) / (4 * XRPR) * (4 * XRPR);  // whole DMA rounds
  constexpr int KKOFF = WSEG == 64 ? 32 : (WSEG == 32 ? L : 2 * L);  // rows of k-fragment 1
  static_assert(KKOFF % 16 == 0, "k-fragment offset must keep the swizzle phase");
  constexpr int kAbytes = kBP * RB;                         // 16 KB
  constexpr int kXbytes = XROWS * RX;
  constexpr int kStage = kAbytes + kXbytes;
  constexpr int LA = kBP / 16;                              // glds per thread: dy (4)
  constexpr int LX = XROWS / (4 * XRPR);                    // glds per thread: x window
  static_assert(XROWS % (4 * XRPR) == 0, "window rows must fill whole DMA rounds");
  __shared__ __attribute__((aligned(16))) char smem[NST * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles = (a.KK / a.KW) * a.nNt * a.nCt;          // (ky, n-tile, c-tile)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int ky = tile / (a.nNt * a.nCt);
  const int r2 = tile - ky * a.nNt * a.nCt;
  const int nt = r2 / a.nCt, ct = r2 - nt * a.nCt;
  const int n0 = nt * 128, c0 = ct * BC;
  const int ks0 = split * a.kps;
  const int ks1 = min(a.nks, ks0 + a.kps);

  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.dy), 0, a.dybytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);

  // ---- DMA geometry: glds round i of wave w covers rows 16 i + 4 w + (lane >> 4), 16-B
  // chunk (lane & 15) (lane-linear 1 KB per wave instruction = 4 rows of 256 B) ----------
  const int drow = lane >> 4, dchunk = lane & 15;
  int dy_off[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = i * 16 + wid * 4 + drow;
    dy_off[i] = (row * a.Cout + n0 + ((dchunk ^ swz<RB>(row)) << 3)) * 2;
  }
  const int dy_step = kBP * a.Cout * 2;
  // window rows: segment s = row / L (>= R: padding row), column j = row % L
  int xseg[LX], xcol[LX], xch[LX];
  {
    const int xr = lane / (RX / 16), xc = lane % (RX / 16);
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int row = i * 4 * XRPR + wid * XRPR + xr;
      xseg[i] = row / L;
      xcol[i] = row - xseg[i] * L;
      xch[i] = (c0 + ((xc ^ swz<RX>(row)) << 3)) * 2;
    }
  }
  // scalar pixel cursor of the next k-step to stage: image sb, output row soh, column sow
  const int HoWo = a.Ho * a.Wo;
  int sb, soh, sow;
  {
    const int m = ks0 * kBP;
    sb = m / HoWo;
    const int r = m - sb * HoWo;
    soh = r / a.Wo;
    sow = r - soh * a.Wo;
  }
  const int rowbytes = a.W * a.Cin * 2;

  auto issue = [&](int ks, int buf) {
    char* As = smem + buf * kStage;
    char* Xs = As + kAbytes;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (lds_ptr_t)(As + i * 4096 + wid * 1024), 16,
                                               dy_off[i], ks * dy_step, 0, 0);
    const int imgoff = sb * a.H * rowbytes;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int ih = soh + xseg[i] - a.ph + ky * a.dh;        // segment s = output row soh + s
      const int iw = sow + xcol[i] - a.pw;
      const bool ok = xseg[i] < R && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(Xs + i * 4096 + wid * 1024), 16,
          ok ? imgoff + ih * rowbytes + iw * a.Cin * 2 + xch[i] : kOobOffset, 0, 0, 0);
    }
  };
  auto advance = [&]() {
    sow += kBP;
    if (sow >= a.Wo) {  // WSEG < 64: a k-step covers R whole output rows
      soh += WSEG == 64 ? 1 : R;
      sow = 0;
      if (soh >= a.Ho) { soh = 0; ++sb; }
    }
  };

  f32x4 acc[NT][4][NJ];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry (see conv_wgrad_mfma): group g reads pixel rows 8g + q and
  // 8g + q + 4 of a 32-pixel k-fragment, lane p's 8-byte quarter of a 16-channel block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto addr = [&](int row, int colblk) {
    return row * RB + ((((colblk + (p >> 1)) ^ swz<RB>(row))) << 4) + ((p & 1) << 3);
  };
  auto xaddr = [&](int row, int colblk) {
    return row * RX + ((((colblk + (p >> 1)) ^ swz<RX>(row))) << 4) + ((p & 1) << 3);
  };
  // window row of k-fragment 0, pixel 8g + q (+4), tap 0
  const int px0 = g * 8 + q;
  const int wrow0 = (px0 / WSEG) * L + (px0 % WSEG);
  const int wrow1 = ((px0 + 4) / WSEG) * L + ((px0 + 4) % WSEG);

  // per 32-pixel half: its fragments are read while the previous half's MFMAs run
  auto readkk = [&](const char* As, const char* Xs, int kk, bf16x8 (&af)[4],
                    bf16x8 (&xf)[NT][NJ]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cb = (wm * 64 + i * 16) >> 3;
      const bf16x4 lo = tr_read(As + kk * 32 * RB + addr(px0, cb));
      const bf16x4 hi = tr_read(As + kk * 32 * RB + addr(px0 + 4, cb));
      af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cb = (wn * (BC / 2) + j * 16) >> 3;
        const bf16x4 lo = tr_read(Xs + kk * KKOFF * RX + xaddr(wrow0 + t, cb));
        const bf16x4 hi = tr_read(Xs + kk * KKOFF * RX + xaddr(wrow1 + t, cb));
        xf[t][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
  };
  auto mfmas = [&](const bf16x8 (&af)[4], const bf16x8 (&xf)[NT][NJ]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], xf[t][j], acc[t][i][j],
                                                                 0, 0, 0);
  };
  auto compute = [&](int buf) {
    const char* As = smem + buf * kStage;
    const char* Xs = As + kAbytes;
    bf16x8 af0[4], xf0[NT][NJ], af1[4], xf1[NT][NJ];
    readkk(As, Xs, 0, af0, xf0);
    readkk(As, Xs, 1, af1, xf1);
    mfmas(af0, xf0);
    mfmas(af1, xf1);
  };

  // NST-deep ring: k-step it lives in slot it % NST; its DMA (LA + LX glds per thread) is
  // retired by a counted vmcnt that leaves the NST - 2 younger stages in flight, and the
  // barrier after it also tells every wave that slot (it - 1) % NST has been read, so the
  // DMA of k-step it + NST - 1 goes there right away.
  const int nks = ks1 - ks0;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    if (s < nks) {
      if (s > 0) advance();
      issue(ks0 + s, s);
    }
  }
  auto body = [&](int it, int slot) {
    const int ahead = min(NST - 2, nks - 1 - it);  // younger stages issued before this wait
    if (ahead >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LA + LX)) : "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LA + LX) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it + NST - 1 < nks) {
      advance();
      issue(ks0 + it + NST - 1, (slot + NST - 1) % NST);
    }
    compute(slot);
  };
  // unrolled over the ring slots: fragment addresses are invariant registers + immediates
  for (int it = 0; it < nks; it += NST) {
#pragma unroll
    for (int s = 0; s < NST; ++s)
      if (it + s < nks) body(it + s, s);
  }

  // ---- fp32 partial slab [S][Cout][KK][Cin]: row n (4 per lane), column ci (16 lanes) ------
  float* o = a.out + (size_t)split * a.Cout * a.KK * a.Cin;
  if (a.wsn) {  // <G, W> share first (see sn_dot_store)
    float sd = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sd += sn_term(a, n0 + wm * 64 + i * 16 + g * 4 + r, ky * a.KW + t,
                          c0 + wn * (BC / 2) + j * 16 + (lane & 15), acc[t][i][j][r]);
    sn_dot_store(a, sd);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = ky * a.KW + t;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wm * 64 + i * 16 + g * 4 + r;
          const int ci = c0 + wn * (BC / 2) + j * 16 + (lane & 15);
          o[((size_t)n * a.KK + tap) * a.Cin + ci] = acc[t][i][j][r];
        }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

}  // namespace

// conv_aux.hip: split-K sum + channel crop + dtype cast of the slabs
at::Tensor wgrad_finalize(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                          int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                          at::ScalarType dtype, const c10::optional<at::Tensor>& dst);
at::Tensor wgrad_finalize_sn(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                             int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                             const at::Tensor& dotp, const at::Tensor& u, const at::Tensor& v,
                             const at::Tensor& sigma, const c10::optional<at::Tensor>& dst);

// dW [out_cout, out_cin, KH, KW] (channels-last memory = [Cout][KH][KW][Cin]) in fp32, or bf16
// when out_bf16; out_cout / out_cin < 0 keep the (padded) channel counts of dy / x. Cropping
// and casting ride in the split-K reduction (wgrad_finalize) instead of separate copies.
// nb > 1: nb independent weight gradients (per-sample weights) -> [nb * Cout, Cin, KH, KW].
// k11 v2 eligibility (shape rules only; the default routing additionally prefers it for 3 taps
// on <= 32-pixel output rows, and ops/conv.py times both per shape under autotuning)
static bool wgrad_v2_shape_ok(int Cout, int Ho, int Wo, int64_t KW, int64_t sh, int64_t sw,
                              int64_t dh, int64_t dw, int64_t nb) {
  const int wseg = Wo % 64 == 0 ? 64 : (Wo == 32 || Wo == 16) ? Wo : 0;
  return nb == 1 && sh == 1 && sw == 1 && dh == 1 && dw == 1 && (KW == 3 || KW == 5) &&
         Cout % 128 == 0 && wseg > 0 && (Ho * Wo) % 64 == 0;
}

bool conv2d_wgrad_v2_eligible(const at::Tensor& dy, const at::Tensor& x, int64_t KH, int64_t KW,
                              int64_t sh, int64_t sw, int64_t dh, int64_t dw, int64_t nb) {
  return x.size(1) % 64 == 0 &&
         wgrad_v2_shape_ok((int)dy.size(1), (int)dy.size(2), (int)dy.size(3), KW, sh, sw, dh, dw,
                           nb);
}

// variant: 0 = default routing, 1 = never v2, 2 = v2 whenever eligible
at::Tensor conv2d_wgrad_mfma(const at::Tensor& dy, const at::Tensor& x, int64_t KH, int64_t KW,
                             int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                             int64_t dw, int64_t out_cout, int64_t out_cin, bool out_bf16,
                             int64_t nb, int64_t variant,
                             const c10::optional<std::vector<at::Tensor>>& sn,
                             const c10::optional<at::Tensor>& dst) {
  IAMD_CHECK(dy.is_cuda() && x.is_cuda(), "conv2d_wgrad_mfma: CUDA tensors expected");
  IAMD_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16,
             "conv2d_wgrad_mfma: bf16 operands expected");
  IAMD_CHECK(dy.dim() == 4 && x.dim() == 4, "conv2d_wgrad_mfma: 4-D tensors expected");
  IAMD_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                 x.is_contiguous(at::MemoryFormat::ChannelsLast),
             "conv2d_wgrad_mfma: packed channels-last operands expected");
  const int B = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  IAMD_CHECK(dy.size(0) == B, "conv2d_wgrad_mfma: batch mismatch");
  IAMD_CHECK(nb >= 1 && (nb == 1 || B == nb), "conv2d_wgrad_mfma: nb must be 1 or the batch");
  IAMD_CHECK(nb == 1 || (out_cout < 0 && out_cin < 0),
             "conv2d_wgrad_mfma: no channel crop for per-sample gradients");
  IAMD_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "conv2d_wgrad_mfma: channels must be multiples of 64");
  IAMD_CHECK(Ho == (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1 &&
                 Wo == (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1,
             "conv2d_wgrad_mfma: dy spatial size does not match the conv geometry");
  IAMD_CHECK(x.numel() * 2 < (1ll << 30) && (dy.numel() + 64ll * Cout) * 2 < (1ll << 30),
             "conv2d_wgrad_mfma: tensors too large for 32-bit buffer offsets");
  const int KK = (int)(KH * KW);
  const bool bno128 = Cout % 128 == 0, bc128 = Cin % 128 == 0;
  WgradArgs a;
  a.dy = reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr());
  a.x = reinterpret_cast<const __hip_bfloat16*>(x.data_ptr());
  a.dybytes = (int)(dy.numel() / nb * 2);
  a.xbytes = (int)(x.numel() / nb * 2);
  a.dybs = nb > 1 ? dy.numel() / nb : 0;
  a.xbs = nb > 1 ? x.numel() / nb : 0;
  a.Bn = (int)(B / nb); a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.KW = (int)KW; a.KK = KK;
  a.sh = (int)sh; a.sw = (int)sw; a.ph = (int)ph; a.pw = (int)pw; a.dh = (int)dh; a.dw = (int)dw;
  a.M = a.Bn * Ho * Wo;
  a.nks = ceil_div(a.M, kBP);
  a.nNt = Cout / (bno128 ? 128 : 64);
  a.nCt = Cin / (bc128 ? 128 : 64);
  // multi-tap kernel: stride-1, undilated, whole-row k-steps, KW in {3, 5, 7}
  const char* mt_env = std::getenv("IMAGINAIRE_AMD_WGRAD_MT");
  // v2 (one wave per SIMD, 128 x 128 x KW tile): stride 1, undilated, KW in {3, 5}, both
  // channel counts multiples of 128, output rows of 16 / 32 pixels or multiples of 64 with
  // whole k-steps per image (IMAGINAIRE_AMD_WGRAD_V2=0 disables it)
  const char* v2_env = std::getenv("IMAGINAIRE_AMD_WGRAD_V2");
  const int wseg = Wo % kBP == 0 ? 64 : (Wo == 32 || Wo == 16) ? Wo : 0;
  // default: 3 taps on <= 32-pixel output rows only (1.09-1.39x there, 0.70-0.89x elsewhere:
  // profiles/wgrad_v2_probe_mi355x.txt); IMAGINAIRE_AMD_WGRAD_V2=force / variant 2 take every
  // eligible shape, IMAGINAIRE_AMD_WGRAD_V2=0 / variant 1 none
  const bool v2_force = variant == 2 || (v2_env != nullptr && v2_env[0] == 'f');
  const bool v2_off = variant == 1 || (v2_env != nullptr && v2_env[0] == '0');
  const bool v2 = !v2_off && (v2_force || (KW == 3 && Wo <= 32)) &&
                  wgrad_v2_shape_ok(Cout, Ho, Wo, KW, sh, sw, dh, dw, nb);
  const bool mt = !v2 && (mt_env == nullptr || mt_env[0] != '0') && Wo % kBP == 0 && sw == 1 &&
                  dw == 1 && (KW == 3 || KW == 5 || KW == 7);
  // x tile: 128 input channels for 3 taps (192 accumulators per wave), 64 for 5 taps (160) or
  // when Cin % 128 != 0 — the 256 accumulation registers of a wave
  const int v2_bc = (KW == 3 && bc128) ? 128 : 64;
  if (v2) {
    a.nNt = Cout / 128;
    a.nCt = Cin / v2_bc;
  }
  // IMAGINAIRE_AMD_WGRAD_MT5=128: the 5-tap multi-tap kernel on a 128 x 64 tile (2 blocks / CU,
  // 0.35 KB of LDS fragment reads per MFMA instead of 0.6) — A/B switch
  const char* mt5_env = std::getenv("IMAGINAIRE_AMD_WGRAD_MT5");
  const bool mt5_wide = mt && KW == 5 && bno128 && mt5_env != nullptr && std::atoi(mt5_env) == 128;
  if (mt) {  // tiles sized to the 256-VGPR budget of 2 waves / SIMD without spills:
    // 3 taps 128 x 64 (or 64 x 64), 5 / 7 taps 64 x 64
    a.nNt = Cout / (((KW == 3 && bno128) || mt5_wide) ? 128 : 64);
    a.nCt = Cin / 64;
  }
  const int tiles = ((mt || v2) ? (int)KH : KK) * a.nNt * a.nCt;
  // split-K factor: fill the chip in whole rounds of co-resident blocks (2 / 3 / 5 blocks
  // per CU for the 64 / 48 / 32 KB LDS variants): a 2.3-round grid leaves the last round a
  // third full (measured: 1200 blocks ran at 28% MFMA issue vs 44% for k10,
  // profiles/pmc_conv_mi355x.txt)
  // (multi-tap: 2 blocks per CU, 3 for the 5-tap kernel's 168-VGPR build)
  const int slots = v2 ? 256 : (mt ? ((KW == 5 && !mt5_wide) ? 768 : 512)
                                   : 256 * ((bno128 && bc128) ? 2 : (bno128 || bc128) ? 3 : 5)) /
                    (int)nb;
  int S = 1;
  if (v2) {
    // one block per CU: the split count that fills whole rounds of 256 best, with at least
    // 8 k-steps per block (the ring's prologue / epilogue amortised)
    const int smax = std::max(1, std::min(1024, a.nks / 8));
    double best = -1.0;
    for (int s = 1; s <= smax; ++s) {
      const int blocks = tiles * s;
      const double eff = (double)blocks / ((double)ceil_div(blocks, slots) * slots);
      if (eff > best + 0.02) { best = eff; S = s; }
      if (blocks >= 4 * slots) break;
    }
  } else if (tiles < slots) {
    // up to 1024 splits: a 1x1 conv's gradient is ONE 64 x 64 tile reduced over ~10^6 pixels
    const int smax = std::max(1, std::min(1024, a.nks / 4));
    double best = -1.0;
    for (int s = 1; s <= smax; ++s) {
      const int blocks = tiles * s;
      if (blocks < slots * 9 / 10 && s != smax) continue;
      const double eff = (double)blocks / ((double)ceil_div(blocks, slots) * slots);
      if (eff > best + 1e-3) { best = eff; S = s; }
      if (blocks >= 2 * slots) break;
    }
  }
  a.kps = ceil_div(a.nks, S);
  S = ceil_div(a.nks, a.kps);  // no empty split
  const int64_t oc = out_cout < 0 ? Cout : out_cout, oi = out_cin < 0 ? Cin : out_cin;
  IAMD_CHECK(oc <= Cout && oi <= Cin, "conv2d_wgrad_mfma: crop larger than the operands");
  // sn = {shadow bf16 [oc, oi, KH, KW] channels-last, u [oc], v [oi * KH * KW], sigma [1]}: the
  // weight is spectrally normalised and dW is the gradient w.r.t. the fp32 parameter W of
  // W / sigma (reference torch.nn.utils.spectral_norm, u / v constant):
  //   dW = G / sigma - (<G, W> / sigma^2) u v^T,  G = the k11 gradient w.r.t. W / sigma,
  // with <G, W> summed in the k11 epilogue (one partial per block) and the rest applied by
  // wgrad_finalize_sn in the pass that sums the split-K slabs: no bf16 G round trip and no
  // separate <G, W> / apply passes (layers/spectral_norm.py _SNScale.backward)
  // a fifth element: <G, W> already known as partial sums (sn_dot_partials, from the data
  // gradient) — the epilogue then reads no W
  const bool use_sn = sn.has_value() && !sn->empty();
  at::Tensor dotp;
  if (use_sn) {
    IAMD_CHECK(nb == 1 && (sn->size() == 4 || sn->size() == 5),
               "conv2d_wgrad_mfma: sn = [shadow, u, v, sigma(, <G, W> partials)]");
    const at::Tensor& shw = (*sn)[0];
    IAMD_CHECK(shw.is_cuda() && shw.scalar_type() == at::kBFloat16 && shw.dim() == 4 &&
                   shw.size(0) == oc && shw.size(1) == oi && shw.size(2) == KH &&
                   shw.size(3) == KW && shw.is_contiguous(at::MemoryFormat::ChannelsLast),
               "conv2d_wgrad_mfma: the SN shadow must be the bf16 weight [out_cout, out_cin, KH, "
               "KW] channels-last");
    IAMD_CHECK((*sn)[1].numel() == oc && (*sn)[2].numel() == oi * KH * KW &&
                   (*sn)[3].numel() == 1 && (*sn)[1].scalar_type() == at::kFloat &&
                   (*sn)[2].scalar_type() == at::kFloat && (*sn)[3].scalar_type() == at::kFloat,
               "conv2d_wgrad_mfma: SN u / v / sigma sizes");
    if (sn->size() == 5) {
      dotp = (*sn)[4];
      IAMD_CHECK(dotp.is_cuda() && dotp.scalar_type() == at::kFloat && dotp.is_contiguous(),
                 "conv2d_wgrad_mfma: <G, W> partials must be a contiguous fp32 tensor");
    } else {
      a.wsn = reinterpret_cast<const __hip_bfloat16*>(shw.data_ptr());
      a.wsn_cout = (int)oc;
      a.wsn_cin = (int)oi;
      dotp = at::empty({(int64_t)tiles * S}, x.options().dtype(at::kFloat));
      a.dotp = dotp.data_ptr<float>();
    }
  }
  const bool direct = !use_sn && S == 1 && !out_bf16 && oc == Cout && oi == Cin;
  at::Tensor dW, part;
  // dst: the caller's destination for dW (a DDP bucket slice, ops/conv.py): the split-K sum
  // (or the single slab itself) lands there, no copy into the bucket follows
  const bool has_dst = dst.has_value() && dst->defined();
  IAMD_CHECK(!has_dst || nb == 1, "conv2d_wgrad_mfma: a destination needs nb == 1");
  if (direct) {
    if (has_dst) {
      IAMD_CHECK(dst->is_cuda() && dst->scalar_type() == at::kFloat && dst->dim() == 4 &&
                     dst->size(0) == Cout && dst->size(1) == Cin && dst->size(2) == KH &&
                     dst->size(3) == KW && dst->is_contiguous(at::MemoryFormat::ChannelsLast),
                 "conv2d_wgrad_mfma: the destination must be a channels-last fp32 "
                 "[Cout, Cin, KH, KW] tensor");
      dW = *dst;
    } else {
      dW = at::empty({nb * Cout, Cin, KH, KW},
                     x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
    }
    a.out = dW.data_ptr<float>();
  } else {
    part = at::empty({(int64_t)S * nb * Cout * KK * Cin}, x.options().dtype(at::kFloat));
    a.out = part.data_ptr<float>();
  }
  const int64_t gx = (int64_t)tiles * S;
  IAMD_CHECK(gx < (1ll << 31), "conv2d_wgrad_mfma: grid too large");
  const dim3 grid((unsigned)gx, (unsigned)nb);
  const bool rows = Wo % kBP == 0;
  // pipeline depth (IMAGINAIRE_AMD_WGRAD_STAGES = 2 | 3). Default 2: the 3-stage ring with
  // counted vmcnt measured 0.98-1.01x the 2-stage loop on every SPADE-step shape
  // (scripts/probe/wgrad_stages_probe.py, profiles/wgrad_stages_probe_mi355x.txt) — two
  // co-resident blocks per CU already hide the DMA wait, so the extra LDS buys nothing.
  int nst = 2;
  if (const char* e = std::getenv("IMAGINAIRE_AMD_WGRAD_STAGES")) nst = std::atoi(e) == 3 ? 3 : 2;
  auto launch = [&](auto bv, auto cv) {
    constexpr int BNO = decltype(bv)::value;
    constexpr int BC = decltype(cv)::value;
    // three stages only while two blocks still fit a CU's 160 KB of LDS (the 128 x 128 tile's
    // 96 KB ring would halve the resident blocks)
    constexpr bool fits3 = 2 * 3 * kBP * (BNO + BC) * 2 <= 160 * 1024;
    if (nst == 3 && fits3) {
      if (rows)
        hipLaunchKernelGGL((conv_wgrad_mfma<BNO, BC, true, 3>), grid, dim3(kThreads), 0,
                           stream(), a);
      else
        hipLaunchKernelGGL((conv_wgrad_mfma<BNO, BC, false, 3>), grid, dim3(kThreads), 0,
                           stream(), a);
    } else {
      if (rows)
        hipLaunchKernelGGL((conv_wgrad_mfma<BNO, BC, true, 2>), grid, dim3(kThreads), 0,
                           stream(), a);
      else
        hipLaunchKernelGGL((conv_wgrad_mfma<BNO, BC, false, 2>), grid, dim3(kThreads), 0,
                           stream(), a);
    }
  };
  using I64 = std::integral_constant<int, 64>;
  using I128 = std::integral_constant<int, 128>;
  auto launch_mt = [&](auto bv, auto cv, auto tv) {
    constexpr int BNO = decltype(bv)::value;
    constexpr int BC = decltype(cv)::value;
    constexpr int NT = decltype(tv)::value;
    if (nst == 3)
      hipLaunchKernelGGL((conv_wgrad_mfma_mt<BNO, BC, NT, 3>), grid, dim3(kThreads), 0,
                         stream(), a);
    else
      hipLaunchKernelGGL((conv_wgrad_mfma_mt<BNO, BC, NT, 2>), grid, dim3(kThreads), 0,
                         stream(), a);
  };
  if (v2) {
    auto lv2 = [&](auto tv, auto sv) {
      constexpr int NT = decltype(tv)::value;
      constexpr int WS = decltype(sv)::value;
      if constexpr (NT == 3) {
        if (v2_bc == 128) {
          hipLaunchKernelGGL((conv_wgrad_mfma_w4<NT, 128, WS, 3>), grid, dim3(kThreads), 0,
                             stream(), a);
          return;
        }
      }
      hipLaunchKernelGGL((conv_wgrad_mfma_w4<NT, 64, WS, 3>), grid, dim3(kThreads), 0,
                         stream(), a);
    };
    using S64 = std::integral_constant<int, 64>;
    using S32 = std::integral_constant<int, 32>;
    using S16 = std::integral_constant<int, 16>;
    auto by_seg = [&](auto tv) {
      if (wseg == 64) lv2(tv, S64());
      else if (wseg == 32) lv2(tv, S32());
      else lv2(tv, S16());
    };
    if (KW == 3) by_seg(std::integral_constant<int, 3>());
    else by_seg(std::integral_constant<int, 5>());
  } else if (mt) {
    using T3 = std::integral_constant<int, 3>;
    using T5 = std::integral_constant<int, 5>;
    if (KW == 3) {
      if (bno128) launch_mt(I128(), I64(), T3());
      else launch_mt(I64(), I64(), T3());
    } else if (KW == 5) {
      if (mt5_wide) launch_mt(I128(), I64(), T5());
      else launch_mt(I64(), I64(), T5());
    } else {
      launch_mt(I64(), I64(), std::integral_constant<int, 7>());
    }
  } else if (bno128 && bc128) launch(I128(), I128());
  else if (bno128) launch(I128(), I64());
  else if (bc128) launch(I64(), I128());
  else launch(I64(), I64());
  IAMD_LAUNCH_CHECK();
  if (direct) return dW;
  if (use_sn)
    return wgrad_finalize_sn(part, S, Cout, Cin, oc, oi, KH, KW, dotp, (*sn)[1].contiguous(),
                             (*sn)[2].contiguous(), (*sn)[3], dst);
  if (nb > 1)  // slabs [S][nb][Cout][KK][Cin]: one [nb * Cout] output, no crop
    return wgrad_finalize(part, S, nb * Cout, Cin, nb * Cout, Cin, KH, KW,
                          out_bf16 ? at::kBFloat16 : at::kFloat, c10::nullopt);
  return wgrad_finalize(part, S, Cout, Cin, oc, oi, KH, KW, out_bf16 ? at::kBFloat16 : at::kFloat,
                        dst);
}

}  // namespace iamd
