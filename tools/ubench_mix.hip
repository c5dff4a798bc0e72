// tools/ubench_mix.hip — does a scalar (SALU) instruction cost a SIMD issue slot when the other wave
// of the SIMD has vector work?  Each wave runs kIter iterations of NV independent v_fma_f32 (8
// chains) followed by NS dependent s_add_u32, at 1 and 2 waves per SIMD; the program prints
// s_memtime cycles per iteration per SIMD (= per-wave cycles / waves per SIMD).  If scalar
// instructions issue beside the other wave's vector ones, NS > 0 adds nothing at 2 waves.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/ubench_mix tools/ubench_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

constexpr int kIter = 256;

template <int NV, int NS, bool kF64, int SOP = 0>
__global__ void __launch_bounds__(256) mix(uint64_t* out, float seed) {
  float f[8];
  double d[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    f[c] = seed + c;
    d[c] = f[c];
  }
  const float a = seed * 0.5f + 0.25f;
  const double da = a;
  uint32_t sv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sv[k] = blockIdx.x + k;
  __syncthreads();
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int i = 0; i < kIter; ++i) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if constexpr (kF64) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(d[v & 7]) : "v"(da));
      else asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(f[v & 7]) : "v"(a));
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {  // independent scalar ops
      if constexpr (SOP == 0) asm volatile("s_mul_i32 %0, %0, 3" : "+s"(sv[k & 7]));
      if constexpr (SOP == 1) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sv[k & 7]) : : "scc");
      if constexpr (SOP == 2) asm volatile("s_mov_b32 %0, %1" : "=s"(sv[k & 7]) : "s"(sv[(k + 1) & 7]));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc ^= sv[k];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc ^= __float_as_uint(f[c]) ^ static_cast<uint32_t>(__double_as_longlong(d[c]));
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = t1 - t0;
    out[2 * wave + 1] = acc;
  }
}

template <int NV, int NS, bool kF64, int SOP = 0>
void row(uint64_t* dout, int cus) {
  double r[2];
  for (int k = 0; k < 2; ++k) {
    const int blocks = cus * (k + 1);
    hipLaunchKernelGGL((mix<NV, NS, kF64, SOP>), dim3(blocks), dim3(256), 0, 0, dout, 1.0f);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const int waves = blocks * 4;
    std::vector<uint64_t> h(2 * waves);
    CK(hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (int w = 0; w < waves; ++w) s += static_cast<double>(h[2 * w]);
    r[k] = s / waves / kIter / (k + 1);  // cycles per iteration per SIMD
  }
  static const char* sop[] = {"s_mul_i32", "s_add_u32", "s_mov_b32"};
  std::printf("%s x%-2d + %s x%-2d: cycles per iteration per SIMD: 1 wave %7.2f  2 waves %7.2f\n",
              kF64 ? "v_fma_f64" : "v_fma_f32", NV, sop[SOP], NS, r[0], r[1]);
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t* dout;
  CK(hipMalloc(&dout, static_cast<size_t>(cus) * 8 * 2 * 8));
  row<8, 0, false>(dout, cus);  // warm up
  row<8, 0, false>(dout, cus);
  row<8, 4, false>(dout, cus);
  row<8, 8, false>(dout, cus);
  row<0, 8, false>(dout, cus);
  row<16, 0, false>(dout, cus);
  row<16, 8, false>(dout, cus);
  row<8, 0, true>(dout, cus);
  row<8, 8, true>(dout, cus);
  row<8, 8, false, 1>(dout, cus);
  row<0, 8, false, 1>(dout, cus);
  row<16, 8, false, 1>(dout, cus);
  row<8, 8, false, 2>(dout, cus);
  row<0, 8, false, 2>(dout, cus);
  row<16, 4, false, 1>(dout, cus);
  CK(hipFree(dout));
  return 0;
}
