// tools/calib_fetch.hip — FETCH_SIZE / WRITE_SIZE calibration per access width (VERDICT r05
// "next" 4): MI355X_MICROARCH.md documents FETCH_SIZE = half the bytes for 16 B/lane streaming
// reads and WRITE_SIZE exact for 16 B/lane stores; the P2P bookkeeping rows are 4 B/lane (and the
// input rings 1 B/lane, the ex_game checksums 2 B/lane), which nobody had calibrated.
//
// Dispatch order (each over a 4 GiB buffer, far past the 256 MiB Infinity Cache, fully coalesced:
// lane i of the grid touches element i, the grid strides over the buffer):
//   read<16>, read<8>, read<4>, read<2>, read<1>   (known bytes: 4 GiB each)
//   write<16>, write<4>, write<2>                  (known bytes: 4 GiB each)
// each REPS times.  Run it under
//   rocprofv3 --pmc FETCH_SIZE -- ./tools/build/calib_fetch
//   rocprofv3 --pmc WRITE_SIZE -- ./tools/build/calib_fetch
// and divide the counter (KiB) per dispatch by the known byte count (tools/calib_fetch.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

template <int B>
struct Elem;
template <>
struct Elem<16> {
  using T = uint4;
  __device__ static uint32_t fold(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
  __device__ static T make(uint32_t v) { return make_uint4(v, v + 1, v + 2, v + 3); }
};
template <>
struct Elem<8> {
  using T = uint2;
  __device__ static uint32_t fold(T v) { return v.x ^ v.y; }
  __device__ static T make(uint32_t v) { return make_uint2(v, v + 1); }
};
template <>
struct Elem<4> {
  using T = uint32_t;
  __device__ static uint32_t fold(T v) { return v; }
  __device__ static T make(uint32_t v) { return v; }
};
template <>
struct Elem<2> {
  using T = uint16_t;
  __device__ static uint32_t fold(T v) { return v; }
  __device__ static T make(uint32_t v) { return static_cast<T>(v); }
};
template <>
struct Elem<1> {
  using T = uint8_t;
  __device__ static uint32_t fold(T v) { return v; }
  __device__ static T make(uint32_t v) { return static_cast<T>(v); }
};

template <int B>
__global__ void __launch_bounds__(256) read_kernel(const void* __restrict__ buf, size_t n, uint32_t* __restrict__ out) {
  using T = typename Elem<B>::T;
  const T* p = static_cast<const T*>(buf);
  uint32_t acc = 0;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) acc += Elem<B>::fold(p[i]);
  if (acc == 0x9E3779B9u) out[threadIdx.x] = acc;  // never true for the zeroed buffer: keeps the loads
}

template <int B>
__global__ void __launch_bounds__(256) write_kernel(void* __restrict__ buf, size_t n, uint32_t salt) {
  using T = typename Elem<B>::T;
  T* p = static_cast<T*>(buf);
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    p[i] = Elem<B>::make(salt ^ static_cast<uint32_t>(i));
}

int main(int argc, char** argv) {
  const size_t bytes = size_t{4} << 30;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 1024));
  CK(hipMemset(buf, 0, bytes));
  const dim3 grid(256 * 64), block(256);  // 64 workgroups per CU
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char* what, auto launch) {
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("{\"kernel\": \"%s\", \"rep\": %d, \"known_bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", what, r, bytes,
                  ms, bytes / (ms * 1e-3) / 1e9);
    }
  };
  timed("read16", [&] { hipLaunchKernelGGL(read_kernel<16>, grid, block, 0, 0, buf, bytes / 16, out); });
  timed("read8", [&] { hipLaunchKernelGGL(read_kernel<8>, grid, block, 0, 0, buf, bytes / 8, out); });
  timed("read4", [&] { hipLaunchKernelGGL(read_kernel<4>, grid, block, 0, 0, buf, bytes / 4, out); });
  timed("read2", [&] { hipLaunchKernelGGL(read_kernel<2>, grid, block, 0, 0, buf, bytes / 2, out); });
  timed("read1", [&] { hipLaunchKernelGGL(read_kernel<1>, grid, block, 0, 0, buf, bytes, out); });
  timed("write16", [&] { hipLaunchKernelGGL(write_kernel<16>, grid, block, 0, 0, buf, bytes / 16, 1u); });
  timed("write4", [&] { hipLaunchKernelGGL(write_kernel<4>, grid, block, 0, 0, buf, bytes / 4, 2u); });
  timed("write2", [&] { hipLaunchKernelGGL(write_kernel<2>, grid, block, 0, 0, buf, bytes / 2, 3u); });
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
