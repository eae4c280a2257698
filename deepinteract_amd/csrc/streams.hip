// Streams of the overlapped schedule (include/deepinteract_amd.h, ABI 8).
//
// The pair stream is ONE persistent launch whose waves wait on the device for signals that launches
// of the producer (GeoT) stream raise (pair_tensor.hip, pair_queue.h). That only overlaps when the
// two streams reach the GPU through different hardware queues: HIP multiplexes every stream of a
// process onto at most GPU_MAX_HW_QUEUES in-order queues per priority (the least-used queue once the
// pool is full), and two streams on one queue run one after the other -- the persistent consumer then
// sits in front of the launch that would signal it and each of its waves waits out its patience.
// Which queue a stream gets depends on every stream the process created before it (torch's stream
// pool, an RCCL communicator's internal streams), so the schedule cannot rely on it:
//   di_stream_create_dedicated: a stream with a CU mask covering every CU. The runtime gives each
//     CU-masked stream a hardware queue of its own (never pooled, never handed to another stream), so
//     two such streams always run concurrently, whatever else the process created.
//   di_streams_concurrent: the property itself, measured: a one-wave kernel on stream a waits
//     (bounded) for a word that a kernel on stream b, issued after it, raises.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <vector>
#include "common.h"
#include "../../include/deepinteract_amd.h"

namespace di {

// work[0]: the flag, work[1]: the waiter's verdict (1 saw the flag, 2 timed out)
__global__ void k_probe_wait(uint32_t* w, uint64_t patience) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen = 0;
  while (!(seen = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > patience) break;
  }
  __hip_atomic_store(w + 1, seen ? 1u : 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_probe_set(uint32_t* w) {
  if (threadIdx.x == 0) __hip_atomic_store(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace di

using namespace di;

extern "C" int di_stream_create_dedicated(void** stream) {
  if (!stream) return DI_EINVAL;
  const int cus = device_cus();
  if (cus <= 0) return DI_EINVAL;
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) mask[(size_t)c >> 5] |= 1u << (c & 31);
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) return (int)e;
  *stream = (void*)s;
  return DI_OK;
}

extern "C" int di_stream_destroy(void* stream) {
  if (!stream) return DI_EINVAL;
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? DI_OK : (int)e;
}

extern "C" int di_streams_concurrent(void* a, void* b, void* work, float patience_ms, int32_t* concurrent) {
  if (!work || !concurrent || !(patience_ms > 0.f) || patience_ms > 10000.f || a == b) return DI_EINVAL;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0)
    khz = 100000;
  const uint64_t ticks = (uint64_t)((double)patience_ms * khz);
  hipStream_t sa = (hipStream_t)a, sb = (hipStream_t)b;
  uint32_t* w = (uint32_t*)work;
  hipError_t e = hipMemsetAsync(w, 0, 256, sa);
  if (e != hipSuccess) return (int)e;
  // b's signal must not be able to run before the memset on a (b may be a different queue)
  if ((e = hipStreamSynchronize(sa)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_probe_wait, dim3(1), dim3(64), 0, sa, w, ticks);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_probe_set, dim3(1), dim3(64), 0, sb, w);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(sa)) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(sb)) != hipSuccess) return (int)e;
  uint32_t verdict = 0;
  if ((e = hipMemcpy(&verdict, w + 1, 4, hipMemcpyDeviceToHost)) != hipSuccess) return (int)e;
  *concurrent = verdict == 1 ? 1 : 0;
  return verdict == 1 || verdict == 2 ? DI_OK : DI_EINVAL;
}
