// L2 -> CU load-path probe (diagnostic, not product code): how fast can a block stream an L2-resident weight set
// (the chain kernels' 352 KiB split-bf16x3 SDF weights) into LDS or registers?  Every block loops over the same
// buffer in 32 KiB k-steps (the chain16 ring step) with one barrier per step, like the chain kernels' weight ring.
//   mode 0: LDS-DMA (global_load_lds_dwordx4), 2-slot ring, wait + barrier per step
//   mode 1: global_load_dwordx4 to VGPRs, then ds_write_b128 to the ring, barrier per step
//   mode 2: global_load_dwordx4 to VGPRs only (xor-folded), no LDS, no barrier
//   mode 3: as 0, 4 KiB per step per wave issued as 4 LDS-DMAs but only every other step (half the bytes)
//   mode 4: as 0 with every block on the same step at the same time (no per-block offset: the chain kernels' pattern)
//   mode 5: as 4 plus the chain16 step's work on the data: every wave reads 34 fragments of the slot and issues 48
//           16x16x32 bf16 MFMAs per step (with EXTRA=0: the same without the DMA)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/l2_probe scripts/l2_probe.hip
// Run:   scripts/l2_probe <mode> <blocks> <waves per block> <steps per block>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void lds_dma16(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}

constexpr int kStepBytes = 32768;
constexpr int kBufSteps = 11;   // 352 KiB

template <int MODE>
__global__ __launch_bounds__(512) void probe(const f32x4* __restrict__ buf, int steps, float* __restrict__ sink, int dma) {
  __shared__ __attribute__((aligned(1024))) f32x4 ring[2][kStepBytes / 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int per = kStepBytes / 1024 / nw;   // 1 KiB chunks per wave per step
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < steps; ++s) {
    const int bs = (MODE >= 4 ? s : s + blockIdx.x) % kBufSteps;
    const f32x4* src = buf + (size_t)bs * (kStepBytes / 16);
    if constexpr (MODE == 5) {
      if (dma) {
        for (int i = 0; i < per; ++i) {
          const int c = wave + nw * i;
          lds_dma16(src + c * 64 + lane, __builtin_amdgcn_readfirstlane(
                                            (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&ring[(s + 1) & 1][c * 64])));
        }
      }
      const bf16x8* sl = reinterpret_cast<const bf16x8*>(&ring[s & 1][0]);
      bf16x8 b = __builtin_bit_cast(bf16x8, acc);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const bf16x8 ah = sl[t * 64 + lane], al = sl[(16 + t) * 64 + lane];
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, acc, 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if constexpr (MODE == 0 || MODE == 3 || MODE == 4) {
      if (MODE != 3 || (s & 1)) {
        for (int i = 0; i < per; ++i) {
          const int c = wave + nw * i;
          lds_dma16(src + c * 64 + lane, __builtin_amdgcn_readfirstlane(
                                            (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&ring[s & 1][c * 64])));
        }
      }
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      acc += ring[s & 1][threadIdx.x];
    } else if constexpr (MODE == 1) {
      f32x4 v[8];
      for (int i = 0; i < per; ++i) v[i] = src[(wave + nw * i) * 64 + lane];
      for (int i = 0; i < per; ++i) ring[s & 1][(wave + nw * i) * 64 + lane] = v[i];
      __syncthreads();
      acc += ring[s & 1][threadIdx.x];
    } else {
      for (int i = 0; i < per; ++i) acc += src[(wave + nw * i) * 64 + lane];
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) sink[blockIdx.x] = acc[0];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int blocks = argc > 2 ? atoi(argv[2]) : 2048;
  const int waves = argc > 3 ? atoi(argv[3]) : 8;
  const int steps = argc > 4 ? atoi(argv[4]) : 64;
  f32x4* buf;
  float* sink;
  hipMalloc(&buf, (size_t)kBufSteps * kStepBytes);
  hipMalloc(&sink, blocks * sizeof(float));
  hipMemset(buf, 0, (size_t)kBufSteps * kStepBytes);
  const int dma = argc > 5 ? atoi(argv[5]) : 1;
  auto launch = [&]() {
    const dim3 gr(blocks), bl(64 * waves);
    if (mode == 0) hipLaunchKernelGGL(probe<0>, gr, bl, 0, 0, buf, steps, sink, dma);
    if (mode == 1) hipLaunchKernelGGL(probe<1>, gr, bl, 0, 0, buf, steps, sink, dma);
    if (mode == 2) hipLaunchKernelGGL(probe<2>, gr, bl, 0, 0, buf, steps, sink, dma);
    if (mode == 3) hipLaunchKernelGGL(probe<3>, gr, bl, 0, 0, buf, steps, sink, dma);
    if (mode == 4) hipLaunchKernelGGL(probe<4>, gr, bl, 0, 0, buf, steps, sink, dma);
    if (mode == 5) hipLaunchKernelGGL(probe<5>, gr, bl, 0, 0, buf, steps, sink, dma);
  };
  for (int i = 0; i < 3; ++i) launch();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps;
  const double bytes = (double)blocks * steps * kStepBytes * (mode == 3 ? 0.5 : 1.0);
  printf("mode %d dma %d blocks %d waves %d steps %d: %.1f us, %.2f TB/s, %.1f B/clk/CU at 2.1 GHz, %.0f cycles/step\n",
         mode, dma, blocks, waves, steps, us, bytes / us / 1e6, bytes / (us * 1e-6) / 256 / 2.1e9,
         us * 1e-6 * 2.1e9 / ((double)blocks / 256 * steps));
  return 0;
}
