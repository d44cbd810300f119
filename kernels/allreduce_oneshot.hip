// allreduce_oneshot.hip — K3 small-message fast path: a one-shot
// all-reduce over the peer-visible buffers of N ranks on one node (xGMI point-to-point).
//
// Why: a ring all-reduce of a KB-sized message is 2(N-1) latency-bound hops; over a full xGMI
// mesh every GPU can read every peer's buffer directly, so the whole reduction is ONE kernel:
//   entry barrier  -> every rank's input is published (release) and every peer has arrived,
//   reduce         -> block b sums slice b of all N inputs (16-byte loads, fp32 accumulation in
//                     rank order 0..N-1, so every rank produces bit-identical output),
//   exit barrier   -> no rank returns (and lets its caller overwrite its input) while a peer may
//                     still be reading it.
// Each barrier is per block pair: block b of rank r stores its epoch into flags[p][phase][r][b]
// of every peer p (system-scope atomic), then polls its own flags[r][phase][p][b] for every p.
// Epochs are per call (caller passes 1, 2, 3, ...; never 0); flags are zeroed once at allocation.
// Every spin is bounded by a wall-clock deadline (s_memrealtime, 100 MHz; default 5 s, settable with
// kfamd_allreduce_oneshot_set_timeout_ms): a peer that never arrives sets *timeout and the kernel
// drains, so the GPU never hangs. A timed-out call must never look like a result: every output
// element of a block whose entry barrier timed out is written as a quiet NaN (the peer's staging
// buffer may hold a stale epoch), the exit barrier is skipped, and the flag stays set until the
// caller resets it — the flag protocol is out of step after a timeout, so callers treat it as fatal
// for the communicator (parallel/oneshot.py raises and refuses further calls).
//
// Ranks may be separate devices (peer access / IPC-opened buffers: the readiness op, DP) or, for
// tests on one GPU, several ranks simulated in ONE launch (gridDim.y = ranks in this launch,
// rank = rank0 + blockIdx.y): all blocks of a small grid are co-resident, so the same barrier
// protocol is exercised end to end.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kfamd_kernels.h"

namespace {

constexpr int kMaxRanks = 8;
constexpr int kThreads = 256;
constexpr uint64_t kTicksPerMs = 100000;  // s_memrealtime runs at a constant 100 MHz

struct Peers {
  const void* in[kMaxRanks];
  void* out[kMaxRanks];
  uint32_t* flags[kMaxRanks];
};

__device__ __forceinline__ void store_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t load_flag(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block-pair barrier: thread t < nranks signals peer t, then waits for peer t's signal.
// Returns true (in every thread of the block) when some peer missed the deadline.
__device__ __forceinline__ bool barrier(const Peers& P, int me, int nranks, int phase, uint32_t epoch,
                                        uint64_t timeout_ticks, unsigned* timeout) {
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  __shared__ int missed;
  if (t == 0) missed = 0;
  __syncthreads();  // every thread's reads / writes of this phase are done before anyone signals
  if (t < nranks) {
    // release: this rank's input (written by earlier work on its stream) and, at the exit
    // barrier, this block's reads are complete before the peer can observe the flag
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    store_flag(P.flags[t] + ((size_t)phase * nranks + me) * nb + b, epoch);
    uint32_t* mine = P.flags[me] + ((size_t)phase * nranks + t) * nb + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (load_flag(mine) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        missed = 1;
        break;
      }
    }
    // acquire: drop any stale cached copy of the peers' buffers before reading them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return missed != 0;
}

template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int kElems = 4;
  __device__ static void acc(float (&s)[8], const uint4& v) {
    s[0] += __uint_as_float(v.x);
    s[1] += __uint_as_float(v.y);
    s[2] += __uint_as_float(v.z);
    s[3] += __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float (&s)[8]) {
    return uint4{__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
  }
  __device__ static float load1(const void* p, long long i) { return static_cast<const float*>(p)[i]; }
  __device__ static void store1(void* p, long long i, float v) { static_cast<float*>(p)[i] = v; }
};
template <>
struct Vec<__bf16> {
  static constexpr int kElems = 8;
  __device__ static float lo(uint32_t w) { return __uint_as_float(w << 16); }
  __device__ static float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
  __device__ static void acc(float (&s)[8], const uint4& v) {
    s[0] += lo(v.x); s[1] += hi(v.x);
    s[2] += lo(v.y); s[3] += hi(v.y);
    s[4] += lo(v.z); s[5] += hi(v.z);
    s[6] += lo(v.w); s[7] += hi(v.w);
  }
  __device__ static uint32_t pk(float a, float b) {
    const __bf16 x = (__bf16)a, y = (__bf16)b;  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
  }
  __device__ static uint4 pack(const float (&s)[8]) {
    return uint4{pk(s[0], s[1]), pk(s[2], s[3]), pk(s[4], s[5]), pk(s[6], s[7])};
  }
  __device__ static float load1(const void* p, long long i) { return (float)static_cast<const __bf16*>(p)[i]; }
  __device__ static void store1(void* p, long long i, float v) { static_cast<__bf16*>(p)[i] = (__bf16)v; }
};

// NaN into this block's vector indices i = blockIdx.x*kThreads + t (+ k*stride) < nvec, and block 0's
// scalar tail [nvec*kElems, n): the write set of the block in the reduce loops below.
template <typename V>
__device__ void poison(void* out, long long n, long long nvec, long long stride) {
  float nan8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) nan8[k] = __builtin_nanf("");
  const uint4 nv = V::pack(nan8);
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += stride)
    static_cast<uint4*>(out)[i] = nv;
  if (blockIdx.x == 0)
    for (long long i = nvec * V::kElems + threadIdx.x; i < n; i += kThreads) V::store1(out, i, __builtin_nanf(""));
}

template <typename T>
__global__ __launch_bounds__(kThreads) void allreduce_oneshot(Peers P, long long n, int nranks, int rank0,
                                                              uint32_t epoch, uint64_t timeout_ticks,
                                                              unsigned* timeout) {
  using V = Vec<T>;
  const int me = rank0 + blockIdx.y;
  const long long nvec = n / V::kElems;
  const long long stride = (long long)gridDim.x * kThreads;
  if (barrier(P, me, nranks, 0, epoch, timeout_ticks, timeout)) {
    // a peer's input may be stale: poison exactly the share this block would have written (the same
    // vector indices as the reduce loop below, plus block 0's tail), skip the exit barrier. Blocks
    // that passed the barrier keep their (correct) sums; nothing here touches their indices.
    poison<V>(P.out[me], n, nvec, stride);
    return;
  }
  // 16-byte vectors; rank r's vector i lives at in[r] + 16 i
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += stride) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 v[kMaxRanks];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)  // issue every peer's load before the first add
      if (r < nranks) v[r] = static_cast<const uint4*>(P.in[r])[i];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < nranks) V::acc(s, v[r]);
    static_cast<uint4*>(P.out[me])[i] = V::pack(s);
  }
  // tail (n not a multiple of the vector width): block 0 only
  if (blockIdx.x == 0) {
    for (long long i = nvec * V::kElems + threadIdx.x; i < n; i += kThreads) {
      float s = 0.f;
      for (int r = 0; r < nranks; ++r) s += V::load1(P.in[r], i);
      V::store1(P.out[me], i, s);
    }
  }
  barrier(P, me, nranks, 1, epoch, timeout_ticks, timeout);
}

// ---- two-shot (reduce-scatter + all-gather) over the same peer-visible buffers -------------------
// For mid-size messages: the one-shot makes every rank read all N inputs in full
// ((N-1) x n bytes over xGMI per rank); the two-shot reads 2 (N-1)/N x n, and every rank pulls from
// all N-1 peers at once, so all 7 links of an 8-GPU hive carry traffic (a ring uses one).
//   entry barrier (phase 0) -> inputs published
//   phase A: rank r owns vector slice r; block b sums its portion of slice r over all N inputs and
//            writes it to in[r] (in place: only rank r ever reads in[r]'s slice r, and it has) and to
//            out[r]
//   mid barrier (phase 1)   -> block b of every rank has finished its portion of its slice
//   phase B: block b copies its portion of every other slice s from in[s] (peer) into out[r]
//   exit barrier (phase 2)  -> no rank reuses in[] while a peer may still read it
// Block b of every rank owns the same index pattern in every slice, so the per-block-pair barriers
// order exactly the writes and reads that meet. The scalar tail (n % vector width) is summed
// directly by block 0 of every rank. Outputs need not be peer-visible (only in[] is read remotely).
// Timeout handling as for the one-shot: the block poisons its whole write set and stops.
template <typename T>
__global__ __launch_bounds__(kThreads) void allreduce_twoshot(Peers P, long long n, int nranks, int rank0,
                                                              uint32_t epoch, uint64_t timeout_ticks,
                                                              unsigned* timeout) {
  using V = Vec<T>;
  const int me = rank0 + blockIdx.y;
  const long long nvec = n / V::kElems;
  const long long per = (nvec + nranks - 1) / nranks;  // vectors per rank slice
  const long long stride = (long long)gridDim.x * kThreads;
  const long long first = (long long)blockIdx.x * kThreads + threadIdx.x;
  auto poison_all = [&]() {  // this block's write set: its portion of every slice, and block 0's tail
    float nan8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) nan8[k] = __builtin_nanf("");
    const uint4 nv = V::pack(nan8);
    for (int sl = 0; sl < nranks; ++sl) {
      const long long s0 = (long long)sl * per, s1 = min(nvec, s0 + per);
      for (long long i = s0 + first; i < s1; i += stride) static_cast<uint4*>(P.out[me])[i] = nv;
    }
    if (blockIdx.x == 0)
      for (long long i = nvec * V::kElems + threadIdx.x; i < n; i += kThreads) V::store1(P.out[me], i, __builtin_nanf(""));
  };
  if (barrier(P, me, nranks, 0, epoch, timeout_ticks, timeout)) {
    poison_all();
    return;
  }
  {
    const long long s0 = (long long)me * per, s1 = min(nvec, s0 + per);
    for (long long i = s0 + first; i < s1; i += stride) {
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      uint4 v[kMaxRanks];
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r)
        if (r < nranks) v[r] = static_cast<const uint4*>(P.in[r])[i];
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r)
        if (r < nranks) V::acc(s, v[r]);
      const uint4 o = V::pack(s);
      static_cast<uint4*>(const_cast<void*>(P.in[me]))[i] = o;
      static_cast<uint4*>(P.out[me])[i] = o;
    }
    if (blockIdx.x == 0) {
      for (long long i = nvec * V::kElems + threadIdx.x; i < n; i += kThreads) {
        float s = 0.f;
        for (int r = 0; r < nranks; ++r) s += V::load1(P.in[r], i);
        V::store1(P.out[me], i, s);
      }
    }
  }
  if (barrier(P, me, nranks, 1, epoch, timeout_ticks, timeout)) {
    poison_all();
    return;
  }
  for (int k = 1; k < nranks; ++k) {  // start at the next rank so the peers' reads spread over links
    const int src = (me + k) % nranks;
    const long long s0 = (long long)src * per, s1 = min(nvec, s0 + per);
    for (long long i = s0 + first; i < s1; i += stride)
      static_cast<uint4*>(P.out[me])[i] = static_cast<const uint4*>(P.in[src])[i];
  }
  barrier(P, me, nranks, 2, epoch, timeout_ticks, timeout);
}

uint64_t g_timeout_ticks = 5000 * kTicksPerMs;

}  // namespace

extern "C" void kfamd_allreduce_oneshot_set_timeout_ms(int ms) {
  g_timeout_ticks = (uint64_t)(ms < 1 ? 1 : ms) * kTicksPerMs;
}

// Flag arrays are shared by the one-shot (phases 0-1) and the two-shot (phases 0-2): epochs
// increase per call whichever kernel runs, and every wait compares for equality with its own call's
// epoch, so a stale flag of an earlier call of either kind never releases a barrier.
extern "C" long long kfamd_allreduce_oneshot_flag_bytes(int nranks, int nblocks) {
  return (long long)3 * nranks * nblocks * (long long)sizeof(uint32_t);
}

extern "C" int kfamd_allreduce_twoshot_blocks(long long n, int dtype, int nranks) {
  const long long vec = dtype == KFAMD_DTYPE_BF16 ? 8 : 4;
  const long long per = ((n + vec - 1) / vec + nranks - 1) / (nranks < 1 ? 1 : nranks);
  long long b = (per + kThreads * 2 - 1) / (kThreads * 2);  // ~2 vectors per thread per slice
  return (int)(b < 1 ? 1 : (b > 64 ? 64 : b));
}

extern "C" int kfamd_allreduce_oneshot_blocks(long long n, int dtype) {
  const long long vec = dtype == KFAMD_DTYPE_BF16 ? 8 : 4;
  const long long nvec = (n + vec - 1) / vec;
  long long b = (nvec + kThreads * 4 - 1) / (kThreads * 4);  // ~4 vectors per thread
  return (int)(b < 1 ? 1 : (b > 64 ? 64 : b));
}

extern "C" int kfamd_allreduce_oneshot(const void* const* inputs, void* const* outputs, uint32_t* const* flags,
                                       int nranks, int rank0, int launch_ranks, long long n, int dtype,
                                       unsigned epoch, int nblocks, unsigned* timeout, void* stream) {
  if (nranks < 1 || nranks > kMaxRanks || launch_ranks < 1 || rank0 < 0 || rank0 + launch_ranks > nranks ||
      n < 0 || epoch == 0 || nblocks < 1 || !timeout || (dtype != KFAMD_DTYPE_F32 && dtype != KFAMD_DTYPE_BF16))
    return KFAMD_EINVAL;
  Peers P{};
  for (int r = 0; r < nranks; ++r) {
    if (!inputs[r] || !flags[r]) return KFAMD_EINVAL;
    if (reinterpret_cast<uintptr_t>(inputs[r]) & 15) return KFAMD_EALIGN;
    P.in[r] = inputs[r];
    P.flags[r] = flags[r];
  }
  for (int r = rank0; r < rank0 + launch_ranks; ++r) {
    if (!outputs[r]) return KFAMD_EINVAL;
    if (reinterpret_cast<uintptr_t>(outputs[r]) & 15) return KFAMD_EALIGN;
    P.out[r] = outputs[r];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(nblocks, launch_ranks), block(kThreads);
  if (dtype == KFAMD_DTYPE_BF16)
    hipLaunchKernelGGL(allreduce_oneshot<__bf16>, grid, block, 0, s, P, n, nranks, rank0, (uint32_t)epoch,
                       g_timeout_ticks, timeout);
  else
    hipLaunchKernelGGL(allreduce_oneshot<float>, grid, block, 0, s, P, n, nranks, rank0, (uint32_t)epoch,
                       g_timeout_ticks, timeout);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// Two-shot: inputs are peer-visible and are overwritten in place (slice r of rank r's input ends up
// holding the reduced slice); outputs are per rank, need not be peer-visible and receive the full sum.
extern "C" int kfamd_allreduce_twoshot(void* const* inputs, void* const* outputs, uint32_t* const* flags, int nranks,
                                       int rank0, int launch_ranks, long long n, int dtype, unsigned epoch,
                                       int nblocks, unsigned* timeout, void* stream) {
  if (nranks < 1 || nranks > kMaxRanks || launch_ranks < 1 || rank0 < 0 || rank0 + launch_ranks > nranks ||
      n < 0 || epoch == 0 || nblocks < 1 || !timeout || (dtype != KFAMD_DTYPE_F32 && dtype != KFAMD_DTYPE_BF16))
    return KFAMD_EINVAL;
  Peers P{};
  for (int r = 0; r < nranks; ++r) {
    if (!inputs[r] || !flags[r]) return KFAMD_EINVAL;
    if (reinterpret_cast<uintptr_t>(inputs[r]) & 15) return KFAMD_EALIGN;
    P.in[r] = inputs[r];
    P.flags[r] = flags[r];
  }
  for (int r = rank0; r < rank0 + launch_ranks; ++r) {
    if (!outputs[r]) return KFAMD_EINVAL;
    if (reinterpret_cast<uintptr_t>(outputs[r]) & 15) return KFAMD_EALIGN;
    P.out[r] = outputs[r];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(nblocks, launch_ranks), block(kThreads);
  if (dtype == KFAMD_DTYPE_BF16)
    hipLaunchKernelGGL(allreduce_twoshot<__bf16>, grid, block, 0, s, P, n, nranks, rank0, (uint32_t)epoch,
                       g_timeout_ticks, timeout);
  else
    hipLaunchKernelGGL(allreduce_twoshot<float>, grid, block, 0, s, P, n, nranks, rank0, (uint32_t)epoch,
                       g_timeout_ticks, timeout);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// ---- cross-process registration (one process per GPU, torch.distributed) ---------------------------
// Buffers the peers map through HIP IPC (dmabuf on this platform: HSA_ENABLE_IPC_MODE_LEGACY=0).
// Flags prefer uncached memory (a peer's atomic store is then seen without a cache flush); if the
// driver cannot export such an allocation, plain device memory + the system-scope atomics/fences of
// the kernel are used. The allocation is zeroed (flags must start at epoch 0).
extern "C" int kfamd_ipc_alloc(long long bytes, int uncached, void** ptr, void* handle64) {
  if (bytes <= 0 || !ptr || !handle64) return KFAMD_EINVAL;
  *ptr = nullptr;
  hipError_t e = hipErrorUnknown;
  if (uncached) {
    e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
    if (e == hipSuccess && hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle64), *ptr) != hipSuccess) {
      (void)hipFree(*ptr);
      *ptr = nullptr;
      e = hipErrorUnknown;
    }
  }
  if (e != hipSuccess) {
    e = hipMalloc(ptr, (size_t)bytes);
    if (e != hipSuccess) return static_cast<int>(e);
    e = hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle64), *ptr);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  e = hipMemset(*ptr, 0, (size_t)bytes);
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_ipc_open(const void* handle64, void** ptr) {
  if (!handle64 || !ptr) return KFAMD_EINVAL;
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle64, sizeof h);
  const hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_ipc_close(void* ptr) {
  const hipError_t e = hipIpcCloseMemHandle(ptr);
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

extern "C" int kfamd_ipc_free(void* ptr) {
  const hipError_t e = hipFree(ptr);
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}

// Stream-ordered device-to-device copy into a registered buffer (the one-shot's input staging).
extern "C" int kfamd_copy_async(void* dst, const void* src, long long bytes, void* stream) {
  const hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice,
                                      reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? KFAMD_OK : static_cast<int>(e);
}
