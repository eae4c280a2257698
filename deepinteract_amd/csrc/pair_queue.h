// Layout of the pair-tensor queue (include/deepinteract_amd.h, di_pair_queue_bytes) and its producer
// signal, shared by the queue kernels (pair_tensor.hip) and the GeoT launches that carry the signal
// (geot_kernels.hip: the node embedding / fused embedding + InitEdge of the next micro-batch).
// Words (uint32): READY at 0 (jobs signalled, monotonic), ERROR at 32 (bit 0: a help completion wait
// timed out, bit 1: a stream wave read a non-increasing ticket), GAVE_UP at 33, stream / help bytes (u64) at 40 / 42; job k's record at 64 + 64 k words
// (256 B): TICKET at +0, DONE at +32 (on its own 128-B line).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace di {

constexpr int PQ_READY = 0, PQ_ERROR = 32, PQ_GAVE_UP = 33, PQ_SBYTES = 40, PQ_HBYTES = 42;
constexpr int PQ_HEAD_WORDS = 64, PQ_JOB_WORDS = 64;
__device__ __forceinline__ uint32_t* pq_ticket(uint32_t* q, int k) { return q + PQ_HEAD_WORDS + PQ_JOB_WORDS * k; }
__device__ __forceinline__ uint32_t* pq_done(uint32_t* q, int k) { return pq_ticket(q, k) + 32; }

// Stream-ordered signal piggybacked on a launch: raised by one thread at the START of a launch that
// the producer's stream orders after the launch that wrote job `job`'s hT. The kernel boundary between
// them has released those stores to the agent (end-of-kernel cache write-back), so no fence is needed
// here and no launch of its own: the consumer polls READY and acquires (pair_tensor.hip).
__device__ __forceinline__ void pq_signal_at_start(uint32_t* q, int job) {
  if (q != nullptr && job >= 0 && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_fetch_max(q + PQ_READY, (uint32_t)job + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace di
