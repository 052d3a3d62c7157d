// TEST INFRASTRUCTURE ONLY (tests/test_gpu_narrow.py): the task kernel's
// narrow-phase device code -- GJK and the wave form of EPA (epa_run_wave,
// the same function task_stage.hpp calls) -- on one wavefront per shape
// pair, so the wave EPA can be checked pair by pair against the lane-serial
// form and the oracle.  Built by build.sh into tests/_narrow_gpu.so.
#include <hip/hip_runtime.h>

#include "../dyros_robot_controller_amd/csrc/qpik_device.hpp"

using namespace drc_amd;

// in: per pair 32 doubles (type, T[12], prm[3]) x 2; out: d, pA, pB, intersect
__global__ void __launch_bounds__(64) narrow_kernel(const double* __restrict__ in, int n, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  EpaPoly* E = reinterpret_cast<EpaPoly*>(lds);
  const int i = blockIdx.x, l = threadIdx.x;
  if (i >= n) return;
  const double* p = in + 32 * i;
  const Shape A{int(p[0]), p + 1, p[13], p[14], p[15]};
  const Shape B{int(p[16]), p + 17, p[29], p[30], p[31]};
  const GjkDist g = gjk(A, B);
  double d = g.dist;
  V3 pA = g.pA, pB = g.pB;
  if (g.intersect) {  // wave-uniform
    d = epa_run_wave(A, B, E, 0);
    pA = ld3(E->out);
    pB = ld3(E->out + 3);
  }
  if (l == 0) {
    double* o = out + 8 * i;
    o[0] = d;
    o[1] = pA.x; o[2] = pA.y; o[3] = pA.z;
    o[4] = pB.x; o[5] = pB.y; o[6] = pB.z;
    o[7] = g.intersect;
  }
}

extern "C" int drc_test_narrow(const double* h_in, int n, double* h_out) {
  double *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, sizeof(double) * 32 * n) != hipSuccess) return 1;
  if (hipMalloc(&dout, sizeof(double) * 8 * n) != hipSuccess) return 1;
  (void)hipMemcpy(din, h_in, sizeof(double) * 32 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(narrow_kernel, dim3(n), dim3(64), sizeof(EpaPoly), 0, din, n, dout);
  int rc = hipGetLastError() != hipSuccess;
  rc |= hipMemcpy(h_out, dout, sizeof(double) * 8 * n, hipMemcpyDeviceToHost) != hipSuccess;
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}
