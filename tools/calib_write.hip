// tools/calib_write.hip — WRITE_SIZE calibration for the brawler's snapshot
// stores (VERDICT r01 "What's weak" #4): a store-only kernel with a known byte
// count in exactly the SaveGameState pattern of steady_kernel<Brawler<P>,7>
// (kernels.hpp store_words<32>: one lane per entity group, 8 u32x4 planes, each
// plane contiguous over lanes -> 16 B per lane, fully coalesced), over the same
// 4 GiB ring (65,536 sessions x 64 lanes x 32 words x 8 slots).
//
// Each dispatch stores 7 slots (the 7 saves of one tick): 7 x 512 MiB.  The
// program prints the HIP-event bandwidth; run it under
//   rocprofv3 --pmc WRITE_SIZE -- ./tools/build/calib_write
// and compare WRITE_SIZE (KiB) per dispatch with the known 3,758,096,384 B.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int kNW = 32;  // words per lane (Brawler NWL)

__global__ void __launch_bounds__(256) save_slots(uint32_t* __restrict__ snap, unsigned Gpad, int slot0, int nslots,
                                                  uint32_t salt) {
  const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= Gpad) return;
  const unsigned slot_words = kNW * Gpad;
  for (int k = 0; k < nslots; ++k) {
    uint32_t* base = snap + static_cast<size_t>((slot0 + k) % 8) * slot_words;
#pragma unroll
    for (int j = 0; j < kNW / 4; ++j) {
      const uint32_t v = salt ^ (g * 2654435761u) ^ static_cast<uint32_t>(j * 97 + k);
      reinterpret_cast<uint4*>(base + static_cast<size_t>(j) * 4 * Gpad)[g] = make_uint4(v, v + 1, v + 2, v + 3);
    }
  }
}

int main() {
  const unsigned S = 65536, L = 64, Gpad = S * L;
  const size_t ring = static_cast<size_t>(8) * kNW * Gpad * 4;  // 4 GiB
  uint32_t* snap = nullptr;
  CK(hipMalloc(&snap, ring));
  CK(hipMemset(snap, 0, ring));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20, nslots = 7;
  const size_t bytes = static_cast<size_t>(nslots) * kNW * Gpad * 4;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(save_slots, dim3(Gpad / 256), dim3(256), 0, 0, snap, Gpad, w, nslots, 7u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(save_slots, dim3(Gpad / 256), dim3(256), 0, 0, snap, Gpad, i, nslots, static_cast<uint32_t>(i));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double per = ms / 1e3 / iters;
  std::printf("{\"kernel\": \"save_slots\", \"bytes_per_dispatch\": %zu, \"avg_us\": %.2f, \"write_GBps\": %.1f}\n",
              bytes, per * 1e6, bytes / per / 1e9);
  CK(hipFree(snap));
  return 0;
}
