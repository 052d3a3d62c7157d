// FETCH_SIZE calibration (measurement tool, not product code): three read
// kernels over a 1 GiB buffer (far above the 8 x 4 MB of L2, so every line is
// an L2 miss), each reading every byte exactly once with the access width our
// kernels use -- 4 B per lane (scratch_load_dword spill reloads), 8 B per lane
// (task record, inputs, model gathers) -- and the 16 B per lane the microarch
// guide's correction was calibrated on.  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and compare each dispatch's FETCH_SIZE (KiB) with the bytes printed here
// (tools/fetch_calib.py does both and writes profiles/<tag>_fetch_calib.json).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

template <class T>
__global__ void __launch_bounds__(256) read_all(const T* __restrict__ p, size_t n, double* __restrict__ sink) {
  double acc = 0;
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const T v = p[i];
    if constexpr (sizeof(T) == 16) acc += double(v.x) + double(v.y) + double(v.z) + double(v.w);
    else acc += double(v);
  }
  // one store per block (negligible beside the reads), and only when the sum is
  // exactly this impossible value: the reads cannot be optimised away
  if (acc == -1.2345e300) sink[blockIdx.x] = acc;
}

int main() {
  const size_t bytes = size_t(1) << 30;
  char* buf = nullptr;
  double* sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 8 * 4, block = 256;
  // order: 4 B, 8 B, 16 B per lane (rocprofv3 dispatch order)
  hipLaunchKernelGGL(read_all<float>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const float*>(buf),
                     bytes / 4, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(read_all<double>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const double*>(buf),
                     bytes / 8, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(read_all<int4>, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const int4*>(buf), bytes / 16,
                     sink);
  CK(hipDeviceSynchronize());
  std::printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"read_all<float>\", \"read_all<double>\", \"read_all<int4>\"]}\n",
              bytes);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
