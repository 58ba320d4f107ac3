// MFMA shape probe: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 on the same wave tile
// (64 x 64 outputs per wave, k = 32 per step), operands in registers (random bits), every CU
// busy (1024 blocks x 4 waves). Reports TFLOP/s per shape. At a fixed wave tile both shapes
// read the same LDS bytes per FLOP; this measures the issue / clock side.
//   hipcc --offload-arch=gfx950 -O3 mfma_shape_probe.hip -o mfma_shape_probe && ./mfma_shape_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ bf16x8 rnd8(unsigned& s) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s = s * 1664525u + 1013904223u;
    unsigned short b = (unsigned short)(0x3c00 | (s >> 23));  // random bf16 in [1/128, 1)
    v[i] = __builtin_bit_cast(__bf16, b);
  }
  return v;
}

// 64x64 wave tile of 16x16 fragments: 4 x 4 accumulators, 16 MFMAs per 32-deep k step
__global__ __launch_bounds__(256) void mfma16(float* out, int iters) {
  unsigned s = threadIdx.x * 7919u + blockIdx.x;
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i) { a[i] = rnd8(s); b[i] = rnd8(s); }
  f32x4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    asm volatile("" : "+v"(a[0]), "+v"(b[0]));
  }
  float t = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

// the same 64x64 wave tile of 32x32 fragments: 2 x 2 accumulators, k = 16 per MFMA, so two
// k-halves (8 MFMAs of twice the FLOPs) per 32-deep k step
__global__ __launch_bounds__(256) void mfma32(float* out, int iters) {
  unsigned s = threadIdx.x * 7919u + blockIdx.x;
  bf16x8 a[2][2], b[2][2];
  for (int h = 0; h < 2; ++h)
    for (int i = 0; i < 2; ++i) { a[h][i] = rnd8(s); b[h][i] = rnd8(s); }
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[h][i], b[h][j], acc[i][j], 0, 0, 0);
    asm volatile("" : "+v"(a[0][0]), "+v"(b[0][0]));
  }
  float t = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) t += acc[i][j][0] + acc[i][j][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const int blocks = 1024, threads = 256;  // 4 waves per block, 4 blocks per CU
  float* out;
  hipMalloc(&out, blocks * threads * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // FLOPs per wave per iteration: 64 x 64 outputs x 32 deep x 2
  const double flop = (double)blocks * (threads / 64) * iters * 64.0 * 64.0 * 32.0 * 2.0;
  for (int rep = 0; rep < 3; ++rep) {
    for (int shape = 0; shape < 2; ++shape) {
      hipEventRecord(e0);
      if (shape == 0) hipLaunchKernelGGL(mfma16, dim3(blocks), dim3(threads), 0, 0, out, iters);
      else hipLaunchKernelGGL(mfma32, dim3(blocks), dim3(threads), 0, 0, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("rep %d  %-22s %8.3f ms  %7.1f TFLOP/s\n", rep,
             shape == 0 ? "16x16x32 (4x4 acc)" : "32x32x16 (2x2 acc)", ms, flop / ms / 1e9);
    }
  }
  hipFree(out);
  return 0;
}
