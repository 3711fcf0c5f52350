// Error plumbing of the C ABI (include/dro_amd.h).
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

static thread_local const char* g_last_error = "";

void set_error(const char* msg) { g_last_error = msg; }

// After a launch: surface a launch-configuration failure as a positive
// hipError_t (never synchronises, so it stays graph-capturable).
int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = what;
    return (int)e;
  }
  return DRO_OK;
}

// Zero a float buffer with a kernel launch.  Deliberately NOT hipMemsetAsync:
// a memset issued from this library onto a capturing stream is not recorded in
// the hipGraph on ROCm 7 (observed: it runs once at capture time and is absent
// from replays), whereas kernel launches are captured.
__global__ __launch_bounds__(256) void zero_fill_kernel(float4* __restrict__ p4, float* __restrict__ tail,
                                                        size_t n4, size_t ntail) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntail; i += stride)
    tail[i] = 0.f;
}

int launch_zero(float* p, size_t n, hipStream_t s) {
  if (n == 0) return DRO_OK;
  // float4 body needs 16-B alignment; handle a misaligned head by treating it as tail
  const uintptr_t addr = (uintptr_t)p;
  if (addr % 16 != 0) {
    const size_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(zero_fill_kernel, dim3(blocks < 4096 ? blocks : 4096), dim3(256), 0, s,
                       (float4*)nullptr, p, (size_t)0, n);
    return launch_status("zero_fill_kernel launch failed");
  }
  const size_t n4 = n / 4, ntail = n % 4;
  size_t blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(zero_fill_kernel, dim3(blocks), dim3(256), 0, s, (float4*)p, p + 4 * n4, n4,
                     ntail);
  return launch_status("zero_fill_kernel launch failed");
}

// In-graph step timeline (tools/step_timeline.py): one thread records the
// device's constant-rate real-time counter (wall_clock64, 100 MHz, common to
// all XCDs) into slot `slot` when the stream reaches this launch.
__global__ void timestamp_kernel(unsigned long long* __restrict__ buf, int slot) {
  if (threadIdx.x == 0) buf[slot] = wall_clock64();
}

}  // namespace dro

extern "C" int dro_timestamp(unsigned long long* buf, int slot, void* stream) {
  if (!buf || slot < 0) {
    dro::set_error("timestamp: NULL buffer or negative slot");
    return DRO_E_NULL;
  }
  hipLaunchKernelGGL(dro::timestamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, buf, slot);
  return dro::launch_status("timestamp_kernel launch failed");
}

extern "C" int dro_wall_clock_hz(long long* hz) {
  if (!hz) {
    dro::set_error("wall_clock_hz: NULL");
    return DRO_E_NULL;
  }
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) {
    dro::set_error("wall_clock_hz: hipDeviceGetAttribute failed");
    return DRO_E_MODE;
  }
  *hz = (long long)khz * 1000;
  return DRO_OK;
}

extern "C" const char* dro_last_error(void) { return dro::g_last_error; }

extern "C" int dro_abi_version(void) { return 10; }
