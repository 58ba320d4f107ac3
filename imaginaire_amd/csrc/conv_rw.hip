// k10 rw: the generalised row-window implicit GEMM (NHWC, bf16 in, fp32 accumulate).
//
// The v4 / v5 tiles (conv_mfma.hip) stage ONE input window per (filter row, 64-channel block)
// and run all KW taps of that filter row from it, but only for stride-1 3x3..5x5 convs with
// Cout % 128 == 0 and output rows that tile 256 pixels exactly. Everything else — the 4x4
// stride-2 PatchGAN / encoder stacks, 7x7 stems and heads, 1x1 projections, Cout = 64 layers,
// the 32-channel full-resolution layers of the video models and odd output widths (63, 127) —
// fell to the v1 tile, which re-stages its im2col A tile from L2 for every filter tap (15-31% of
// the kernel time of the MUNIT / FUNIT / pix2pixHD / vid2vid recipes). This tile
// takes all of them:
//
//   * GEMM rows are VIRTUAL output pixels: R = floor(BM / SW) segments of SW (16..BM)
//     consecutive pixels of one output row, nct = ceil(Wo / SW) segments per row, the pixels
//     past Wo and the block's rows past R * SW masked (zero window rows in, no store out). SW is
//     a power of two where one wastes <= 10% of the rows, else any width that wastes least
//     (a 66-wide data gradient of a reflect-padded 3x3 conv: 3 x 22-pixel segments per row,
//     11 per block, 94.5% of the rows live, against <= 82% for every power of two); the window
//     row of each lane's fragment row is computed per lane, so a fragment may straddle segments.
//   * Per segment the block stages the input pixels every tap of one filter row reads, once per
//     (filter row, channel block) "outer step", with buffer_load ... lds (out-of-image pixels
//     and dead segments load zeros from the buffer unit). Window layouts (LDS rows of 128 B):
//       stride 1:          row j = input column S*ow0 - pw + j; tap kx reads row p + kx;
//       stride 2 (DEINT):  the even columns first (rows [0, Ph)), then the odd ones, so tap kx
//                          reads the CONSECUTIVE rows (kx & 1) * Ph + (kx >> 1) + p;
//       Cin = 32 (PAIR):   a 64-deep k-chunk is TWO adjacent filter taps: row j holds input
//                          pixels (c, c + 1), c = S*ow0 - pw + S*j, each lane's 16-byte chunk
//                          from its own pixel; virtual tap t (filter taps 2t, 2t+1) reads row
//                          p + 2t (stride 1) or p + t (stride 2). An odd KW's last virtual tap
//                          loads the missing half of its weight tile as zeros, so 32-channel
//                          layers run without the 64-channel zero-padding pass.
//   * The 16-byte chunk index of every staged row is XOR-swizzled with (row & 7) on the global
//     side, so the shifted 16-row fragment reads stay bank-conflict free (as v4).
//   * Weights: a 3-slot ring of BN x 64 tap tiles, tap step q + 2 staged during step q; counted
//     `s_waitcnt vmcnt` (never 0 in the loop) + raw s_barrier, one barrier per tap step. The
//     second k-half's fragments of a tap step are read during it and consumed first by the next
//     step (v4's PF schedule: no MFMA waits on a read issued after the barrier).
//   * 8 waves as 4 (M) x 2 (N); BM = 256 pixels at stride 1, 128 at stride 2 (its window is
//     twice as wide), BN = 64 or 128 output channels: wave tiles 64 x 64 .. 32 x 32 of
//     v_mfma_f32_16x16x32_bf16 accumulators. (16x16x32 rather than 32x32x16: at a fixed wave
//     tile both read the same LDS bytes per FLOP, and the 16x16 loop ran 1.12-1.15x the FLOP/s
//     of the 32x32 one on random data, MI355X_MICROARCH.md "MFMA shape";
//     profiles/mfma_shape_probe_mi355x.txt.)
//   * Epilogue as v4 (1 / sigma, bias, leaky slope, residual, bf16 through LDS, 16-byte row
//     stores) with the virtual -> real pixel map and the phase-interleaved output map (omode) of
//     the strided data gradient; split-K writes fp32 slabs for conv_splitk_reduce.
// Reference: the convolutions of /root/reference/imaginaire/layers/conv.py:59-91 (cuDNN there).
#include "conv_common.h"

#include <cstdlib>

namespace iamd {
namespace {

constexpr int kNR = 5;  // window DMA rounds (64 rows each) per buffer: <= 320 rows

template <int S, bool PAIR>
__device__ __forceinline__ int rw_tapoff(int kx, int Ph) {
  if constexpr (S == 2 && !PAIR) return (kx & 1) * Ph + (kx >> 1);
  else if constexpr (S == 1 && PAIR) return 2 * kx;
  else return kx;
}

// S: stride (1 | 2). KW: filter taps per row (PAIR: virtual taps = ceil(real KW / 2)).
// BN: output channels per block (64 | 128). PAIR: Cin == 32.
// BMT / NR: block rows (256 | 128) and window DMA rounds (5 | 3). The narrow variant (stride 1,
// BN 64, BMT 128, NR 3: 72 KB of LDS) runs two blocks per CU, so one block's loads overlap the
// other's epilogue on the short-K convs (3x3 over 64 channels: 9 tap steps per block).
template <int S, int KW, int BN, bool PAIR, int BMT, int NR>
__global__ __launch_bounds__(512, (BMT == 128 && S == 1) ? 2 : 1) void conv_fwd_rw(ConvArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int BM = BMT;
  constexpr int MI = BM / 64;                   // 16-row fragments per wave (BM / 4 rows)
  constexpr int NI = BN / 32;                   // 16-column fragments per wave (BN / 2 cols)
  constexpr bool DEINT = S == 2 && !PAIR;
  constexpr int kAbytes = NR * 64 * kRowBytes;  // 40 / 24 KB per window buffer
  constexpr int kBbytes = BN * kRowBytes;        // 8 / 16 KB per weight slot
  constexpr int WB = BN / 64;                    // weight glds per thread per tap step
  constexpr int kBoff = 2 * kAbytes;
  constexpr int kSmem = kBoff + 3 * kBbytes;
  static_assert(BM * kEpiStride <= kSmem, "rw epilogue staging exceeds the LDS ring");
  __shared__ __attribute__((aligned(16))) char smem[kSmem];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / a.nNt, nt = bid - mt * a.nNt;
  const int n0 = nt * BN;
  const int SW = a.SW, P = a.P, Ph = a.Ph;
  const int R = BM / SW;  // (segment decodes below divide once per lane, outside the loop)
  const int g0 = mt * R;  // first segment of this block

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.x), 0, a.xbytes, kBufCfg);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__hip_bfloat16*>(a.w), 0, a.wbytes, kBufCfg);

  // ---- window DMA sources: round r of wave w moves LDS rows 64 r + 8 w + (lane >> 3) ------
  const int dr = lane >> 3;
  const int csw = (lane & 7) ^ dr;  // source chunk of this lane (row & 7 == dr)
  const int rowbytes = a.W * a.Cin * 2;
  // (P is a multiple of 8, so the 8 rows a wave moves per round lie in ONE segment: the
  // segment decode and the filter-row mask are wave-uniform scalar work, once per round)
  uint32_t a_off[NR];
  uint32_t a_km[NR];  // bit ky: filter row ky of this round's rows reads inside the image
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int rbase = r * 64 + wid * 8;  // wave-uniform
    const int s = rbase / P;
    const int j = rbase - s * P + dr;
    const int g = g0 + s;
    a_off[r] = kOobOffset;
    a_km[r] = 0;
    if (s < R && g < a.nseg) {
      const int ct = g % a.nct, t = g / a.nct;
      const int oh = t % a.Ho, b = t / a.Ho;
      const int c0 = S * ct * SW - a.pw;
      const int ih0 = oh * S - a.ph;
      uint32_t km = 0;
      for (int ky = 0; ky < a.KH; ++ky) km |= (uint32_t)((unsigned)(ih0 + ky) < (unsigned)a.H) << ky;
      a_km[r] = km;
      int iw;
      if constexpr (DEINT) {
        const int odd = j >= Ph ? 1 : 0;
        iw = c0 + 2 * (j - odd * Ph) + odd;
      } else if constexpr (PAIR) {
        iw = c0 + S * j + (csw >> 2);
      } else {
        iw = c0 + j;
      }
      if ((unsigned)iw < (unsigned)a.W)
        a_off[r] = (uint32_t)(((b * a.H + ih0) * a.W + iw) * a.Cin * 2 +
                              (PAIR ? (csw & 3) : csw) * 16);
    }
  }
  // weight DMA: rows n0 + 64 i + 8 w + (lane >> 3) of the BN-row tap tile; PAIR: the weight is
  // [Cout][KH][KWr][32] (KWr = a.KW real taps), virtual tap t = real taps 2t, 2t + 1 (128 B);
  // for an odd KWr the lanes of the missing tap (chunks 4..7) of the last virtual tap load zeros
  const int cinv = PAIR ? 32 : a.Cin;
  const int wrow_bytes = a.KH * a.KW * cinv * 2;
  int b_off[WB];
#pragma unroll
  for (int i = 0; i < WB; ++i) b_off[i] = (n0 + i * 64 + wid * 8 + dr) * wrow_bytes + csw * 16;
  const bool hi_lane = PAIR && csw >= 4;
  const bool odd_kw = PAIR && (a.KW & 1);

  // ---- outer steps o = (filter row ky, channel block) of this split ------------------------
  const int nout = a.KH * a.cpt;
  const int o0 = blockIdx.y * a.kps;
  const int o1 = min(nout, o0 + a.kps);
  // (ky, channel offset) cursors of outer steps o, o + 1, o + 2 (no division in the loop)
  int ky0 = o0 / a.cpt, cc0 = (o0 - (o0 / a.cpt) * a.cpt) * kBK;
  auto adv = [&](int& ky, int& cc) {
    cc += kBK;
    if (cc >= (PAIR ? kBK : a.Cin)) { cc = 0; ++ky; }
  };
  int ky1 = ky0, cc1 = cc0;
  adv(ky1, cc1);
  int ky2 = ky1, cc2 = cc1;
  adv(ky2, cc2);

  auto issueA = [&](int o, int ky, int cc, int buf) {
    const bool live = o < o1;
    const int koff = ky * rowbytes + (PAIR ? 0 : cc * 2);
    char* As = smem + buf * kAbytes;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const bool ok = live && ((a_km[r] >> (ky & 31)) & 1u);
      // (an out-of-image column keeps its out-of-range offset: kOobOffset + koff < 2^32)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xrs, (lds_ptr_t)(As + r * 8192 + wid * 1024), 16,
          ok ? (int)(a_off[r] + (uint32_t)koff) : kOobOffset, 0, 0, 0);
    }
  };
  auto issueB = [&](int o, int ky, int cc, int kx, int slot) {
    int soff;
    if constexpr (PAIR)
      soff = o < o1 ? (ky * a.KW + 2 * kx) * (cinv * 2) : kOobOffset;
    else
      soff = o < o1 ? ((ky * KW + kx) * a.Cin + cc) * 2 : kOobOffset;
    const bool zero_hi = hi_lane && odd_kw && kx == KW - 1;
    char* Bs = smem + kBoff + slot * kBbytes;
#pragma unroll
    for (int i = 0; i < WB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(Bs + i * 8192 + wid * 1024), 16,
                                               zero_hi ? kOobOffset : b_off[i], soff, 0, 0);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A fragment i of this wave: virtual pixels wm * BM/4 + 16 i + frow, window row s * P + pl
  const int frow = lane & 15, fk = lane >> 4;
  int wrow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int p = wm * (BM / 4) + i * 16 + frow;
    const int s = p / SW;
    wrow[i] = s * P + (p - s * SW);
  }
  auto load_frags = [&](int abuf, int kx, int slot, int kk, bf16x8 (&af)[MI], bf16x8 (&bf)[NI]) {
    const char* As = smem + abuf * kAbytes;
    const char* Bs = smem + kBoff + slot * kBbytes;
    const int toff = rw_tapoff<S, PAIR>(kx, Ph);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wrow[i] + toff;
      af[i] = *reinterpret_cast<const bf16x8*>(As + row * kRowBytes +
                                               (((kk * 4 + fk) ^ (row & 7)) << 4));
    }
    const int coff = ((kk * 4 + fk) ^ (frow & 7)) << 4;
#pragma unroll
    for (int j = 0; j < NI; ++j)
      bf[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * (BN / 2) + j * 16 + frow) * kRowBytes +
                                               coff);
  };
  auto mma = [&](const bf16x8 (&af)[MI], const bf16x8 (&bf)[NI]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // the previous tap step's second k-half fragments (zero before the first step: +0 MFMAs)
  bf16x8 pa[MI], pb[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i) pa[i] = bf16x8{};
#pragma unroll
  for (int j = 0; j < NI; ++j) pb[j] = bf16x8{};

  int slot = 0;  // weight slot of the tap step being computed (tap step q: slot q % 3)
  // one outer step: KW tap steps; tap step q stages (first tap) the next outer step's window,
  // then the weights of tap step q + 2
  auto outer = [&](int o, int abuf) {
#pragma unroll
    for (int kx = 0; kx < KW; ++kx) {
      // this step's weights (issued two steps ago) and window landed; younger loads may fly:
      // the weights of step q + 1 and, at kx == 1, the next window issued before them
      if (KW > 1 && kx == 1)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WB + NR) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WB) : "memory");
      __builtin_amdgcn_s_barrier();
      if (kx == 0) issueA(o + 1, ky1, cc1, abuf ^ 1);
      const int ws = slot == 0 ? 2 : slot - 1;  // (q + 2) % 3
      if (kx + 2 < KW) issueB(o, ky0, cc0, kx + 2, ws);
      else if (kx + 2 - KW < KW) issueB(o + 1, ky1, cc1, kx + 2 - KW, ws);
      else issueB(o + 2, ky2, cc2, kx + 2 - 2 * KW, ws);
      bf16x8 a0[MI], b0[NI];
      load_frags(abuf, kx, slot, 0, a0, b0);
      mma(pa, pb);                            // previous step, second k-half
      load_frags(abuf, kx, slot, 1, pa, pb);  // this step's second k-half, used next step
      mma(a0, b0);
      slot = slot == 2 ? 0 : slot + 1;
    }
    ky0 = ky1; cc0 = cc1;
    ky1 = ky2; cc1 = cc2;
    adv(ky2, cc2);
  };
  // prologue: the first window, then the weights of tap steps 0 and 1
  issueA(o0, ky0, cc0, 0);
  if (KW >= 2) {
    issueB(o0, ky0, cc0, 0, 0);
    issueB(o0, ky0, cc0, 1, 1);
  } else {
    issueB(o0, ky0, cc0, 0, 0);
    issueB(o0 + 1, ky1, cc1, 0, 1);
  }
  for (int o = o0; o < o1; o += 2) {
    outer(o, 0);
    if (o + 1 < o1) outer(o + 1, 1);
  }
  mma(pa, pb);  // the last tap step's second k-half
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // trailing (zero) prefetches landed and every wave is done reading

  // virtual row rl of this block -> real output pixel (b * Ho + oh) * Wo + ow, or -1 (masked)
  auto real_row = [&](int rl) -> int {
    const int s = rl / SW, j = rl - s * SW;
    const int g = g0 + s;
    if (s >= R || g >= a.nseg) return -1;  // (rows past R * SW: a non-power-of-two SW)
    const int ct = g % a.nct, t = g / a.nct;
    const int ow = ct * SW + j;
    return ow < a.Wo ? t * a.Wo + ow : -1;
  };
  if (a.part) {  // split-K: raw fp32 partials [S][M][Cout] (bias / act / map in the reduce)
    float* op = a.part + (size_t)blockIdx.y * a.M * a.Cout;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = real_row(wm * (BM / 4) + i * 16 + (lane >> 4) * 4 + r);
        if (m < 0) continue;
#pragma unroll
        for (int j = 0; j < NI; ++j)
          op[(size_t)m * a.Cout + n0 + wn * (BN / 2) + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    return;
  }
  char* E = smem;
  const float asc = ascale_of(a);
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int cl = wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = a.bias ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * (BM / 4) + i * 16 + (lane >> 4) * 4 + r;
        float v = fmaf(acc[i][j][r], asc, bv);
        v = v > 0.f ? v : v * a.slope;
        *reinterpret_cast<__hip_bfloat16*>(E + rl * kEpiStride + cl * 2) = __float2bfloat16(v);
      }
  }
  __syncthreads();
  constexpr int kChunks = BN / 8;                // 16-byte chunks per output row
  constexpr int kRowsPerPass = 512 / kChunks;
  const int ch = tid % kChunks, rr = tid / kChunks;
#pragma unroll
  for (int p = 0; p < BM / kRowsPerPass; ++p) {
    const int rl = p * kRowsPerPass + rr;
    const int m = real_row(rl);
    if (m >= 0 && n0 + ch * 8 < a.ldy) {
      const uint4 v = *reinterpret_cast<const uint4*>(E + rl * kEpiStride + ch * 16);
      store_chunk(a, a.y, out_row(a, m) * a.ldy + n0 + ch * 8, v);
    }
  }
#endif  // __HIP_DEVICE_COMPILE__
}

bool rw_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_CONV_RW");  // 0: A/B switch back to v1
    return e != nullptr && e[0] == '0';
  }();
  return off;
}

// IMAGINAIRE_AMD_CONV_RW_POW2=1: power-of-two segment widths only (A/B switch)
bool rw_pow2_only() {
  static const bool on = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_CONV_RW_POW2");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

int pow2ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Fill in the row-window geometry; false if the shape does not fit the tile. The segment width
// SW is the largest power of two whose masked tail wastes at most 10% of the virtual pixels
// (else the least wasteful one); with min_eff > 0 a shape wasting more than 1 - min_eff of its
// pixels is refused (default routing: a 66- or 262-wide output on 128 / 256-pixel segments ran
// at half the useful rate of the v1 tile).
bool rw_plan(ConvArgs& a, double min_eff = 0.0, int bm = 0, int nr = kNR, bool any_sw = true) {
  if (a.nz != 1 || a.dh != 1 || a.dw != 1 || a.sh != a.sw || (a.sh != 1 && a.sh != 2))
    return false;
  if (a.Cout % 64 != 0 || a.KH > 31 || a.KH < 1 || a.KW < 1) return false;
  const bool pair = a.Cin == 32;
  if (!pair && a.Cin % kBK != 0) return false;
  const int S = a.sh;
  const int kwv = pair ? (a.KW + 1) / 2 : a.KW;  // (virtual) taps per filter row
  if (pair ? (kwv > 4) : (a.KW != 1 && a.KW != 3 && a.KW != 4 && a.KW != 5 && a.KW != 7))
    return false;
  const int BM = bm > 0 ? bm : (S == 1 ? 256 : 128);
  int SW = 0;
  double best = -1.0;
  for (int sw = BM; sw >= (S == 1 ? 32 : 16); sw >>= 1) {
    const double eff = (double)a.Wo / ((double)ceil_div(a.Wo, sw) * sw);
    if (eff >= 0.9 - 1e-9) {
      SW = sw;
      best = eff;
      break;
    }
    if (eff > best + 1e-9) {
      best = eff;
      SW = sw;
    }
  }
  int P, Ph = 0;
  if (any_sw && best < 0.9 - 1e-9 && S == 1 && !pair && a.omode == 0 && !rw_pow2_only()) {
    // any segment width: live rows = (Wo / (nct SW)) (R SW / BM), the window P = SW + KW - 1
    // rounded up to 8 rows (R P <= the 320-row window buffer)
    for (int sw = BM; sw >= 16; --sw) {
      const int r = BM / sw, p = (sw + a.KW - 1 + 7) / 8 * 8;
      if (r * p > nr * 64) continue;
      const double eff = (double)a.Wo / ((double)ceil_div(a.Wo, sw) * sw) *
                         ((double)(r * sw) / BM);
      if (eff > best + 1e-3) {
        best = eff;
        SW = sw;
      }
    }
  }
  if (best < min_eff) return false;
  if (S == 2 && !pair) {
    Ph = SW + 4;  // >= SW + (KW - 1) / 2 even columns
    P = 2 * Ph;
  } else if ((SW & (SW - 1)) == 0) {
    P = SW + 8;   // >= the rows the taps read: SW + KW - 1 | SW + 2 kwv - 2 | SW + kwv - 1
  } else {
    P = (SW + a.KW - 1 + 7) / 8 * 8;
  }
  const int R = BM / SW;
  if (R * P > nr * 64) return false;
  a.SW = SW;
  a.P = P;
  a.Ph = Ph;
  a.nct = ceil_div(a.Wo, SW);
  const int64_t nseg = (int64_t)(a.M / (a.Ho * a.Wo)) * a.Ho * a.nct;
  if (nseg >= (1ll << 30)) return false;
  a.nseg = (int)nseg;
  a.cpt = pair ? 1 : a.Cin / kBK;
  return true;
}

template <int S, int KW, int BN, bool PAIR, int BMT = (S == 1 ? 256 : 128), int NR = kNR>
void rw_launch(const ConvArgs& a, dim3 grid) {
  hipLaunchKernelGGL((conv_fwd_rw<S, KW, BN, PAIR, BMT, NR>), grid, dim3(512), 0, stream(), a);
}

template <int S, int BN, bool PAIR>
void rw_by_kw(const ConvArgs& a, dim3 grid, int kwv) {
  if constexpr (PAIR) {
    switch (kwv) {
      case 1: rw_launch<S, 1, BN, true>(a, grid); break;
      case 2: rw_launch<S, 2, BN, true>(a, grid); break;
      case 3: rw_launch<S, 3, BN, true>(a, grid); break;
      default: rw_launch<S, 4, BN, true>(a, grid); break;
    }
  } else {
    switch (kwv) {
      case 1: rw_launch<S, 1, BN, false>(a, grid); break;
      case 3: rw_launch<S, 3, BN, false>(a, grid); break;
      case 4: rw_launch<S, 4, BN, false>(a, grid); break;
      case 5: rw_launch<S, 5, BN, false>(a, grid); break;
      default: rw_launch<S, 7, BN, false>(a, grid); break;
    }
  }
}

// the narrow two-blocks-per-CU variant: stride 1, BN 64, no PAIR
void rw_small_by_kw(const ConvArgs& a, dim3 grid) {
  switch (a.KW) {
    case 1: rw_launch<1, 1, 64, false, 128, 3>(a, grid); break;
    case 3: rw_launch<1, 3, 64, false, 128, 3>(a, grid); break;
    case 4: rw_launch<1, 4, 64, false, 128, 3>(a, grid); break;
    case 5: rw_launch<1, 5, 64, false, 128, 3>(a, grid); break;
    default: rw_launch<1, 7, 64, false, 128, 3>(a, grid); break;
  }
}

void rw_dispatch(const ConvArgs& a, dim3 grid, int BN, bool small) {
  if (small) {
    rw_small_by_kw(a, grid);
    return;
  }
  const bool pair = a.Cin == 32;
  const int kwv = pair ? (a.KW + 1) / 2 : a.KW;
  auto by_pair = [&](auto sv, auto bnv) {
    constexpr int S = decltype(sv)::value, B = decltype(bnv)::value;
    if (pair) rw_by_kw<S, B, true>(a, grid, kwv);
    else rw_by_kw<S, B, false>(a, grid, kwv);
  };
  auto by_bn = [&](auto sv) {
    if (BN == 128) by_pair(sv, std::integral_constant<int, 128>());
    else by_pair(sv, std::integral_constant<int, 64>());
  };
  if (a.sh == 2) by_bn(std::integral_constant<int, 2>());
  else by_bn(std::integral_constant<int, 1>());
}

}  // namespace

bool rw_eligible(const ConvArgs& a) {
  if (rw_disabled()) return false;
  ConvArgs t = a;
  return rw_plan(t);
}

// IMAGINAIRE_AMD_CONV_RW_SMALL: the narrow two-blocks-per-CU variant for stride-1 convs with
// Cout % 128 != 0 (BN 64). 2 (default): where the filter row holds >= 1152 MACs per output
// channel (K = KH * KW * Cin: 3x3 over >= 128 channels, 5x5 / 7x7 over 64): 1.10-1.24x v1 and
// 1.07-1.16x the 256-row variant there, 0.97-1.01x v1 at K = 576
// (profiles/conv_rw_small_probe_r6_mi355x.txt); 1: every such conv; 0: off.
int rw_small_mode() {
  static const int mode = [] {
    const char* e = std::getenv("IMAGINAIRE_AMD_CONV_RW_SMALL");
    return e == nullptr ? 2 : std::atoi(e);
  }();
  return mode;
}

bool rw_small_shape(const ConvArgs& a) {
  return a.sh == 1 && a.sw == 1 && a.Cin % kBK == 0 && a.Cout % 128 != 0 && a.Cout % 64 == 0 &&
         a.nz == 1 && a.dh == 1 && a.dw == 1;
}

bool rw_small_pick(const ConvArgs& a) {
  const int mode = rw_small_mode();
  if (mode == 0 || !rw_small_shape(a)) return false;
  return mode == 1 || (int64_t)a.KH * a.KW * a.Cin >= 1152;
}

bool rw_small_pref(const ConvArgs& a) { return !rw_disabled() && rw_small_pick(a); }

bool run_rw(ConvArgs& a, const at::Tensor& x, bool forced) {
  if (rw_disabled()) return false;
  // (segment widths other than powers of two only where the row-window tile is forced — Cin 32,
  // IMAGINAIRE_AMD_CONV_V=6: on the 66 / 34 / 18-wide reflect-pad data gradients they ran at
  // 0.92-0.93x v1, profiles/conv_rw_small_probe_r6_mi355x.txt)
  bool small = rw_small_pick(a) && rw_plan(a, forced ? 0.0 : 0.85, 128, 3, forced);
  if (!small && !rw_plan(a, forced ? 0.0 : 0.85, 0, kNR, forced)) return false;
  const int BM = small ? 128 : (a.sh == 1 ? 256 : 128);
  const int R = BM / a.SW;
  const int BN = a.Cout % 128 == 0 ? 128 : 64;
  a.nNt = a.Cout / BN;
  const int64_t tiles = (int64_t)ceil_div(a.nseg, R) * a.nNt;
  IAMD_CHECK(tiles < (1ll << 31), "conv rw: grid too large");
  const int nout = a.KH * a.cpt;
  int S = 1;
  if (tiles < 256 && nout >= 4) S = (int)std::min<int64_t>((256 + tiles - 1) / tiles, nout / 2);
  if (const char* e = std::getenv("IMAGINAIRE_AMD_CONV_SPLITK")) S = std::max(1, std::atoi(e));
  S = std::max(1, std::min(S, nout));
  a.kps = ceil_div(nout, S);
  S = ceil_div(nout, a.kps);
  at::Tensor part;
  a.part = nullptr;
  if (S > 1) {
    part = at::empty({(int64_t)S * a.M * a.Cout}, x.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  rw_dispatch(a, dim3((unsigned)tiles, (unsigned)S, 1), BN, small);
  if (S > 1) {
    IAMD_LAUNCH_CHECK();
    const int64_t MC = (int64_t)a.M * a.Cout;
    const int blocks = (int)std::min<int64_t>((MC / 8 + 255) / 256, 8192);
    hipLaunchKernelGGL(conv_splitk_reduce, dim3(blocks), dim3(256), 0, stream(), a.part, a.bias,
                       a.y, S, MC, a.Cout, a.slope, a);
  }
  IAMD_LAUNCH_CHECK();
  return true;
}

}  // namespace iamd
