// tools/ubench_valu.hip — issue cost and dependent latency of the VALU
// instructions the ex_game steady kernel is made of, on gfx950, at 1, 2 and 4
// waves per SIMD (one 256-thread block = 4 waves per CU, one per SIMD).
//
// Each wave runs kIter iterations of C independent chains of one instruction
// (inline asm, so nothing is folded) and stamps s_memtime around the loop;
// the program prints cycles per instruction per wave and per SIMD
// (= per-wave cycles / waves per SIMD).  C = 8: issue cost; C = 1: latency.
// OP 7 (v_cndmask with a vcc clobber) is inflated by the s_nop 0 the compiler puts
// before each instance (the clobber reads as a VALU write of vcc): use OP 19-20.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int kIter = 512;

template <int OP>
__device__ __forceinline__ void op1(float& f, double& d, uint32_t& u, uint64_t& q, float a, double da, uint32_t ua) {
  if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f) : "v"(a), "v"(a));
  if constexpr (OP == 1) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d) : "v"(da), "v"(da));
  if constexpr (OP == 2) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"(da));
  if constexpr (OP == 3) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f) : "v"(d));
  if constexpr (OP == 4) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(f));
  if constexpr (OP == 5) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(u) : "v"(d));
  if constexpr (OP == 6) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(u) : "v"(ua), "v"(ua));
  if constexpr (OP == 7) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(u) : "v"(ua) : "vcc");
  if constexpr (OP == 8) asm volatile("v_sqrt_f32 %0, %0" : "+v"(f));
  if constexpr (OP == 9) asm volatile("v_rcp_f32 %0, %0" : "+v"(f));
  if constexpr (OP == 10) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(q) : "v"(q));
  if constexpr (OP == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u) : "v"(ua));
  if constexpr (OP == 12) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u) : "v"(ua));
  if constexpr (OP == 13) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(q) : "v"(q));
  if constexpr (OP == 14) asm volatile("v_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(u));
  if constexpr (OP == 15) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(da));
  if constexpr (OP == 16) asm volatile("v_cmp_gt_f32 vcc, %0, %1" ::"v"(f), "v"(a) : "vcc");
  if constexpr (OP == 17) asm volatile("v_div_fmas_f32 %0, %0, %1, %1" : "+v"(f) : "v"(a) : "vcc");
  if constexpr (OP == 18) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d) : "v"(u));
  // selects without the vcc clobber of OP 7 (which makes the compiler put an s_nop before each one):
  // a loop-invariant SGPR-pair mask, a cmp + select pair as the kernels emit it, and a bit select
  if constexpr (OP == 19) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u) : "v"(ua), "s"(static_cast<uint64_t>(ua) * 0x9E3779B97F4A7C15ull));
  if constexpr (OP == 20) asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, %1\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(u) : "v"(ua) : "s40", "s41");
  if constexpr (OP == 21) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(u) : "v"(ua), "v"(ua));
  if constexpr (OP == 22) asm volatile("s_nop 0" : "+v"(u));
  if constexpr (OP == 23) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f) : "v"(a), "v"(a));
  if constexpr (OP == 24) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f) : "v"(a));
  if constexpr (OP == 25) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f) : "v"(a));
  if constexpr (OP == 26) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f) : "v"(a));
  if constexpr (OP == 27) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u) : "v"(ua));
  if constexpr (OP == 28) asm volatile("v_mov_b32 %0, %1" : "=v"(u) : "v"(ua));
  if constexpr (OP == 29) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(q) : "v"(q));
  if constexpr (OP == 30) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(u) : "v"(ua));
  if constexpr (OP == 31) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(u) : "v"(ua));
  if constexpr (OP == 32) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f) : "v"(a), "s"(a));
  if constexpr (OP == 33) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u));
  if constexpr (OP == 34) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u) : "s"(ua));
  if constexpr (OP == 35) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d) : "v"(da), "s"(da));
  if constexpr (OP == 36) asm volatile("v_cvt_f32_f64 %0, %1\n\tv_fma_f32 %2, %3, %3, %2" : "=v"(f), "+v"(d), "+v"(u) : "v"(a));
  if constexpr (OP == 37) asm volatile("v_fma_f64 %0, %2, %2, %0\n\tv_fma_f32 %1, %3, %3, %1" : "+v"(d), "+v"(f) : "v"(da), "v"(a));
  if constexpr (OP == 38) asm volatile("s_add_u32 s40, s40, 1\n\tv_fma_f32 %0, %1, %1, %0" : "+v"(f) : "v"(a) : "s40");
}
static const char* kNames[] = {"v_fma_f32",     "v_fma_f64",      "v_mul_f64",     "v_cvt_f32_f64",  "v_cvt_f64_f32",
                               "v_cvt_i32_f64", "v_dot4_u32_u8",  "v_cndmask_b32", "v_sqrt_f32",     "v_rcp_f32",
                               "v_pk_fma_f32",  "v_add_u32",      "v_mul_hi_u32",  "v_lshl_add_u64", "v_add_u32_dpp",
                               "v_add_f64",     "v_cmp_gt_f32",   "v_div_fmas_f32", "v_cvt_f64_i32",
                               "cndmask_sgpr",  "cmp+nop1+cndmask", "v_bfi_b32",    "s_nop 0",        "v_med3_f32",
                               "v_max_f32",     "v_mul_f32",      "v_add_f32",     "v_and_b32",      "v_mov_b32",
                               "v_pk_mul_f32",  "v_mad_u32_u24",  "v_perm_b32",    "v_fma_f32 sgpr", "v_lshlrev_b32",
                               "v_add_u32 sgpr", "v_fma_f64 sgpr", "cvt_f32_f64+fma_f32", "fma_f64+fma_f32", "s_add+fma_f32"};
constexpr int kOps = 39;

template <int OP, int C>
__global__ void __launch_bounds__(256) ubench(uint64_t* out, float seed) {
  float f[C];
  double d[C];
  uint32_t u[C];
  uint64_t q[C];
  const float a = seed * 0.5f + 0.25f;
  const double da = static_cast<double>(a);
  const uint32_t ua = __float_as_uint(seed) | 1u;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    f[c] = seed + c;
    d[c] = f[c];
    u[c] = threadIdx.x + c;
    q[c] = (static_cast<uint64_t>(u[c]) << 32) | __float_as_uint(f[c]);
  }
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIter; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c) op1<OP>(f[c], d[c], u[c], q[c], a, da, ua);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) acc ^= __float_as_uint(f[c]) ^ static_cast<uint32_t>(__double_as_longlong(d[c])) ^ u[c] ^
                                      static_cast<uint32_t>(q[c]);
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if ((threadIdx.x & 63) == 0) {
    out[2 * wave] = t1 - t0;
    out[2 * wave + 1] = acc;
  }
}

template <int OP, int C>
double run(uint64_t* dout, int blocks) {
  hipLaunchKernelGGL((ubench<OP, C>), dim3(blocks), dim3(256), 0, 0, dout, 1.0f);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const int waves = blocks * 4;
  std::vector<uint64_t> h(2 * waves);
  CK(hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost));
  double s = 0;
  for (int w = 0; w < waves; ++w) s += static_cast<double>(h[2 * w]);
  return s / waves / (static_cast<double>(kIter) * 4 * C);  // cycles per instruction per wave
}

template <int OP>
void row(uint64_t* dout, int cus) {
  const double lat = run<OP, 1>(dout, cus);
  double tp[3];
  const int wps[3] = {1, 2, 4};
  for (int k = 0; k < 3; ++k) tp[k] = run<OP, 8>(dout, cus * wps[k]) / wps[k];
  std::printf("%-16s latency %6.2f   issue per SIMD: 1 wave %6.2f  2 waves %6.2f  4 waves %6.2f  (cycles/instr)\n",
              kNames[OP], lat, tp[0], tp[1], tp[2]);
  if constexpr (OP + 1 < kOps) row<OP + 1>(dout, cus);
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t* dout;
  CK(hipMalloc(&dout, static_cast<size_t>(cus) * 4 * 4 * 2 * 8));
  run<0, 8>(dout, cus);  // warm up
  std::printf("%s, %d CUs; s_memtime cycles\n", prop.gcnArchName, cus);
  row<0>(dout, cus);
  CK(hipFree(dout));
  return 0;
}
