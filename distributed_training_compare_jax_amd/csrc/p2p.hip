// Peer-to-peer all-reduce over xGMI for the latency-bound tensor-parallel messages
// (4 all-reduces of the [tokens, d_model] fp32 residual per layer).
//
// Every rank allocates one uncached device buffer, exports it with hipIpcGetMemHandle and maps
// every peer's buffer (hipIpcOpenMemHandle), so a kernel on rank r can load any peer's memory
// directly over the point-to-point xGMI links — all 7 links of an 8-GPU node at once, instead
// of the one outgoing link a ring step uses.  The all-reduce is two-shot:
//
//   copy   x -> own buffer half (h = call parity)
//   barrier
//   reduce-scatter: rank r sums slice r of every peer's half h, in rank order, into its own half
//   barrier
//   all-gather: out[slice q] = peer q's reduced slice (own slice local)
//
// so each rank moves 2(W-1)/W of the message over xGMI, and every rank computes the SAME sum in
// the SAME order (bitwise identical replicas).  Alternating halves makes a third barrier
// unnecessary: call k+2 rewrites half h only after passing call k+1's barriers, which every rank
// reaches only after finishing call k.
//
// Barriers: rank r stores the epoch into flags[r] of every peer (system-scope release) and spins
// on its own flags[p] >= epoch (system-scope acquire).  The epoch is a device counter, so the
// whole sequence is plain stream-ordered kernels that hipGraph capture records like any other
// kernel (no graph cut, unlike an eager RCCL call).  Every spin is bounded: after ~10 s it sets
// an error word and exits, so a missing peer shows up as an error, never as a hung GPU.
#include "common.h"
#include <algorithm>
#include <cstring>

namespace {

constexpr int P2P_MAX = 8;
constexpr int FLAG_BYTES = 4096;  // flag area at the start of each buffer (epoch per source rank)

struct PeerTable {
  unsigned char* base[P2P_MAX];  // buffer base of every rank (own included), as mapped here
};

__device__ __forceinline__ uint64_t wall_clock() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// inc: 1 per barrier of the two-shot call (2 barriers), 2 for the one-shot call's single barrier, so
// every call advances the epoch by 2 and the buffer half stays (epoch >> 1) & 1 at the call's start
__global__ void p2p_barrier_kernel(PeerTable t, int rank, int world, uint32_t* __restrict__ epoch,
                                   int* __restrict__ err, int inc) {
  const int p = threadIdx.x;
  DTC_ASSERT(world >= 1 && world <= P2P_MAX && rank >= 0 && rank < world && (inc == 1 || inc == 2));
  const uint32_t e = epoch[0] + inc;
  __threadfence_system();  // this rank's prior writes (its buffer half) before the signal
  if (p < world && p != rank) {
    uint32_t* peer_flag = (uint32_t*)t.base[p] + rank;
    __hip_atomic_store(peer_flag, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = (const uint32_t*)t.base[rank] + p;
    const uint64_t t0 = wall_clock();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock() - t0 > 1000000000ull) {  // ~10 s at 100 MHz
        atomicExch(err, 1000 + p);
        break;
      }
    }
  }
  __syncthreads();
  if (p == 0) epoch[0] = e;
}

// copy x into own half h (h read from the epoch counter parity: 2 barriers per call)
__global__ void p2p_stage_kernel(const f32x4* __restrict__ x, PeerTable t, int rank, long n4, long half_bytes,
                                 const uint32_t* __restrict__ epoch) {
  const int h = (epoch[0] >> 1) & 1;
  DTC_ASSERT(16 * n4 <= half_bytes && rank >= 0);
  f32x4* dst = (f32x4*)(t.base[rank] + FLAG_BYTES + h * half_bytes);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) dst[i] = x[i];
}

__global__ void p2p_reduce_scatter_kernel(PeerTable t, int rank, int world, long n4, long half_bytes,
                                          const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 1) >> 1) & 1;  // one barrier has passed since the stage
  const long chunk = (n4 + world - 1) / world;
  const long lo = rank * chunk, hi = min(n4, lo + chunk);
  const long off = FLAG_BYTES + h * half_bytes;
  DTC_ASSERT(16 * n4 <= half_bytes && rank < world);
  for (long i = lo + (long)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (long)gridDim.x * blockDim.x) {
    f32x4 s = ((const f32x4*)(t.base[0] + off))[i];
    for (int p = 1; p < world; ++p) s += ((const f32x4*)(t.base[p] + off))[i];
    ((f32x4*)(t.base[rank] + off))[i] = s;
  }
}

__global__ void p2p_all_gather_kernel(PeerTable t, int world, long n4, long half_bytes, f32x4* __restrict__ out,
                                      const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long chunk = (n4 + world - 1) / world;
  const long off = FLAG_BYTES + h * half_bytes;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i / chunk);
    DTC_ASSERT(q < world);
    out[i] = ((const f32x4*)(t.base[q] + off))[i];
  }
}

// one-shot (small messages): after the single barrier every rank sums ALL ranks' halves itself, in
// rank order (identical result on every rank); (W-1) n bytes over xGMI instead of 2 (W-1)/W n, but
// one barrier and two fewer launches: the latency path for the CE row statistics, label logits and
// the grad-norm scalar
__global__ void p2p_oneshot_kernel(PeerTable t, int world, long n4, long half_bytes, f32x4* __restrict__ out,
                                   const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long off = FLAG_BYTES + h * half_bytes;
  DTC_ASSERT(16 * n4 <= half_bytes && world >= 1);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 s = ((const f32x4*)(t.base[0] + off))[i];
    for (int p = 1; p < world; ++p) s += ((const f32x4*)(t.base[p] + off))[i];
    out[i] = s;
  }
}

// ---------------------------------------------------------------- bf16 payload (tp_comm_dtype: bf16)
// Row-parallel partials travel as bf16 (half the xGMI bytes of the fp32 residual), are summed in fp32
// in rank order, and the LAST kernel adds the fp32 residual and the bias:
//   out[i] = resid[i] + bias[i % ncols] + sum_p partial_p[i]
// so the residual stream itself is never rounded (only the layer's delta is, once, to bf16).  The
// two-shot reduce-scatter stores its reduced slice in bf16 (the all-gather reads half the bytes).
__global__ void p2p_stage_bf16_kernel(const bf16x8* __restrict__ x, PeerTable t, int rank, long n8, long half_bytes,
                                      const uint32_t* __restrict__ epoch) {
  const int h = (epoch[0] >> 1) & 1;
  DTC_ASSERT(16 * n8 <= half_bytes && rank >= 0);
  bf16x8* dst = (bf16x8*)(t.base[rank] + FLAG_BYTES + h * half_bytes);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) dst[i] = x[i];
}

__device__ __forceinline__ void add8(float (&a)[8], const bf16x8& v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] += (float)v[e];
}

// out (fp32) = resid + bias + the 8 values a, for elements 8i .. 8i+7
__device__ __forceinline__ void finish8(float (&a)[8], long i, float* __restrict__ out, const float* __restrict__ resid,
                                        const float* __restrict__ bias, int ncols) {
  if (resid) {
    const f32x4 r0 = ((const f32x4*)resid)[2 * i], r1 = ((const f32x4*)resid)[2 * i + 1];
#pragma unroll
    for (int e = 0; e < 4; ++e) { a[e] += r0[e]; a[e + 4] += r1[e]; }
  }
  if (bias) {
    const int c0 = (int)((8 * i) % ncols);  // ncols % 8 == 0: the 8 columns share a row
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += bias[c0 + e];
  }
  ((f32x4*)out)[2 * i] = f32x4{a[0], a[1], a[2], a[3]};
  ((f32x4*)out)[2 * i + 1] = f32x4{a[4], a[5], a[6], a[7]};
}

__global__ void p2p_oneshot_bf16_kernel(PeerTable t, int world, long n8, long half_bytes, float* __restrict__ out,
                                        const float* __restrict__ resid, const float* __restrict__ bias, int ncols,
                                        const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long off = FLAG_BYTES + h * half_bytes;
  DTC_ASSERT(16 * n8 <= half_bytes && world >= 1 && ncols % 8 == 0);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) add8(a, ((const bf16x8*)(t.base[p] + off))[i]);
    finish8(a, i, out, resid, bias, ncols);
  }
}

__global__ void p2p_reduce_scatter_bf16_kernel(PeerTable t, int rank, int world, long n8, long half_bytes,
                                               const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 1) >> 1) & 1;
  const long chunk = (n8 + world - 1) / world;
  const long lo = rank * chunk, hi = min(n8, lo + chunk);
  const long off = FLAG_BYTES + h * half_bytes;
  DTC_ASSERT(16 * n8 <= half_bytes && rank < world);
  for (long i = lo + (long)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (long)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) add8(a, ((const bf16x8*)(t.base[p] + off))[i]);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(a[e]);
    ((bf16x8*)(t.base[rank] + off))[i] = o;
  }
}

__global__ void p2p_all_gather_bf16_kernel(PeerTable t, int world, long n8, long half_bytes, float* __restrict__ out,
                                           const float* __restrict__ resid, const float* __restrict__ bias, int ncols,
                                           const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long chunk = (n8 + world - 1) / world;
  const long off = FLAG_BYTES + h * half_bytes;
  DTC_ASSERT(16 * n8 <= half_bytes && world >= 1 && ncols % 8 == 0);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    add8(a, ((const bf16x8*)(t.base[(int)(i / chunk)] + off))[i]);
    finish8(a, i, out, resid, bias, ncols);
  }
}

// ---------------------------------------------------------------- sequence parallelism (tp_sequence_parallel)
// The residual stream is split by rows over the TP ranks, so the row-parallel GEMMs' partial sums are
// REDUCE-SCATTERED (each rank only needs its own rows) and the LayerNorm outputs / residual gradients
// that feed the column-parallel GEMMs are ALL-GATHERED.  Both are one barrier each: the payload (the
// whole [rows, cols] partial, or this rank's slice at its row offset) is in every rank's buffer half
// before the barrier; afterwards rank r reads what it needs straight from the peers' halves.
//
// reduce-scatter: out[i] (fp32, this rank's n_loc elements) = resid[i] + bias[col] + sum_p partial_p[lo + i],
// summed in rank order (the same order on every rank: a row's value does not depend on who owns it)
template <bool BF16>
__global__ void p2p_rs_kernel(PeerTable t, int rank, int world, long n8_loc, long half_bytes, float* __restrict__ out,
                              const float* __restrict__ resid, const float* __restrict__ bias, int ncols,
                              const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long off = FLAG_BYTES + h * half_bytes;
  const long lo8 = (long)rank * n8_loc;
  DTC_ASSERT(rank < world && (BF16 ? 16 : 32) * n8_loc * world <= half_bytes && (!bias || ncols % 8 == 0));
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8_loc; i += (long)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      if constexpr (BF16) {
        add8(a, ((const bf16x8*)(t.base[p] + off))[lo8 + i]);
      } else {
        const f32x4* src = (const f32x4*)(t.base[p] + off) + 2 * (lo8 + i);
        const f32x4 v0 = src[0], v1 = src[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) { a[e] += v0[e]; a[e + 4] += v1[e]; }
      }
    }
    finish8(a, i, out, resid, bias, ncols);  // i indexes this rank's rows: column = (8 i) % ncols
  }
}

// stage n16 16-byte pieces of x into own half at piece offset `at` (the all-gather's slot / a full partial)
__global__ void p2p_stage16_kernel(const u32x4* __restrict__ x, PeerTable t, int rank, long at, long n16,
                                   long half_bytes, const uint32_t* __restrict__ epoch) {
  const int h = (epoch[0] >> 1) & 1;
  DTC_ASSERT(16 * (at + n16) <= half_bytes && rank >= 0);
  u32x4* dst = (u32x4*)(t.base[rank] + FLAG_BYTES + h * half_bytes) + at;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) dst[i] = x[i];
}

// all-gather: out[q * n16_loc + i] = rank q's slot (16-byte pieces, any element type); own slot local
__global__ void p2p_ag_kernel(PeerTable t, int world, long n16_loc, long half_bytes, u32x4* __restrict__ out,
                              const uint32_t* __restrict__ epoch) {
  const int h = ((epoch[0] - 2) >> 1) & 1;
  const long off = FLAG_BYTES + h * half_bytes;
  const long n = n16_loc * world;
  DTC_ASSERT(16 * n <= half_bytes && world >= 1);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = ((const u32x4*)(t.base[(int)(i / n16_loc)] + off))[i];
}

// ---------------------------------------------------------------- intra-device stream flags
// Cross-stream dependencies between two separately captured hipGraphs (main / side) on the SAME
// device: a producer stream bumps flags[k] to its replay epoch (agent-scope release, after all of
// its prior kernels completed in queue order); the consumer spins until flags[k] >= its own
// epoch (agent-scope acquire).  Each graph bumps its epoch once per replay, so the two stay in
// lock step without host involvement.  Spins are bounded (~10 s -> error word, then proceed).
__global__ void epoch_inc_kernel(uint32_t* __restrict__ epoch) {
  if (threadIdx.x == 0) epoch[0] += 1;
}

__global__ void flag_set_kernel(uint32_t* __restrict__ flags, int k, const uint32_t* __restrict__ epoch) {
  if (threadIdx.x == 0) {
    __threadfence();
    __hip_atomic_store(flags + k, epoch[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void flag_wait_kernel(const uint32_t* __restrict__ flags, int k, const uint32_t* __restrict__ epoch,
                                 int* __restrict__ err) {
  if (threadIdx.x == 0) {
    const uint32_t e = epoch[0];
    const uint64_t t0 = wall_clock();
    while (__hip_atomic_load(flags + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock() - t0 > 1000000000ull) {
        atomicExch(err, 2000 + k);
        break;
      }
    }
  }
  __syncthreads();
}

// CU-occupancy probe (benchmarks/cu_steal_proxy.py): `blocks` workgroups, each requesting (nearly) a whole CU's
// LDS so no other LDS-using workgroup fits next to it, idle for `ticks` of the 100 MHz wall clock -- a stand-in
// for the CUs an RCCL collective holds while the step's kernels run on the rest.  Bounded: every wave exits.
__global__ void cu_hog_kernel(uint64_t ticks, int* __restrict__ sink) {
  extern __shared__ int hog_lds[];
  // sink[1] (host-mapped): workgroups resident so far -- the host starts timing once all are
  if (threadIdx.x == 0) __hip_atomic_fetch_add(sink + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock();
  while (wall_clock() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
  hog_lds[threadIdx.x] = (int)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && hog_lds[1] == 12345) sink[0] = 1;  // never true: keeps the LDS allocation live
}

}  // namespace

extern "C" {

int dtc_epoch_inc(uint32_t* epoch, hipStream_t st) {
  hipLaunchKernelGGL(epoch_inc_kernel, dim3(1), dim3(64), 0, st, epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_flag_set(uint32_t* flags, int k, const uint32_t* epoch, hipStream_t st) {
  hipLaunchKernelGGL(flag_set_kernel, dim3(1), dim3(64), 0, st, flags, k, epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_flag_wait(const uint32_t* flags, int k, const uint32_t* epoch, int* err, hipStream_t st) {
  hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, st, flags, k, epoch, err);
  DTC_CHECK_LAUNCH();
  return 0;
}

long dtc_p2p_flag_bytes() { return FLAG_BYTES; }

// uncached device buffer (flags + 2 data halves) and its IPC handle (64 bytes)
int dtc_p2p_alloc(long bytes, void** ptr, char* handle) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, FLAG_BYTES);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, *ptr);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "handle size");
  memcpy(handle, &h, sizeof(h));
  return 0;
}

int dtc_p2p_open(const char* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int dtc_p2p_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// Topology checks at P2P init (parallel/p2p.py): the PCI bus id identifies a GPU across processes
// (device ordinals depend on each process's visible set); can-access-peer says whether a kernel on
// `dev` can load `peer`'s memory directly (xGMI).
int dtc_device_pci_bus_id(int dev, char* buf, int len) { return (int)hipDeviceGetPCIBusId(buf, len, dev); }
int dtc_device_count(int* n) { return (int)hipGetDeviceCount(n); }
int dtc_can_access_peer(int dev, int peer, int* ok) { return (int)hipDeviceCanAccessPeer(ok, dev, peer); }
int dtc_p2p_free(void* ptr) { return (int)hipFree(ptr); }
// Node count of a captured (not yet instantiated) hipGraph: parallel/program.py drops segments that
// captured nothing (e.g. between a collective and its wait) instead of replaying empty graphs.
int dtc_graph_num_nodes(void* graph, size_t* n) { return (int)hipGraphGetNodes((hipGraph_t)graph, nullptr, n); }

// out = sum over ranks of x (fp32, n % 4 == 0, n*4 <= half_bytes).  x and out may alias.
// mode: 0 auto, 1 two-shot, 2 one-shot.  Per link, one-shot moves n bytes (each rank reads every peer
// once over that peer's link) and two-shot 2n/W, for one barrier fewer: at W = 2 the bytes are equal
// and one-shot always wins; at W = 4 / 8 it wins up to ~1 MB / 512 KB (a barrier round trip is a few
// us, a link ~150 GB/s).  Measured with 2 ranks on one device (benchmarks/p2p_bench.py): one-shot
// 6.5 / 7.5 / 11.9 / 16.9 us vs two-shot 11.2 (512 KB) / 12.3 / 18.5 / 22.8 us at 64 KB / 1 / 4 / 8 MB.
constexpr long P2P_ONESHOT_BYTES = 512 * 1024;
inline bool oneshot_auto(long bytes, int world) {
  return world <= 2 || bytes <= P2P_ONESHOT_BYTES * (world <= 4 ? 2 : 1);
}
int dtc_p2p_allreduce(const float* x, float* out, long n, void* const* bases, int rank, int world, long half_bytes,
                      uint32_t* epoch, int* err, int mode, hipStream_t st) {
  if (world < 1 || world > P2P_MAX || n % 4 || n * 4 > half_bytes) return 4001;
  PeerTable t;
  for (int p = 0; p < P2P_MAX; ++p) t.base[p] = (unsigned char*)(p < world ? bases[p] : nullptr);
  const long n4 = n / 4;
  const int blocks = (int)std::min(1024L, std::max(1L, (n4 + 255) / 256));
  const bool one = mode == 2 || (mode == 0 && oneshot_auto(n * 4, world));
  hipLaunchKernelGGL(p2p_stage_kernel, dim3(blocks), dim3(256), 0, st, (const f32x4*)x, t, rank, n4, half_bytes, epoch);
  DTC_CHECK_LAUNCH();
  if (one) {
    hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 2);
    DTC_CHECK_LAUNCH();
    hipLaunchKernelGGL(p2p_oneshot_kernel, dim3(blocks), dim3(256), 0, st, t, world, n4, half_bytes, (f32x4*)out,
                       epoch);
    DTC_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 1);
  DTC_CHECK_LAUNCH();
  const int rs_blocks = (int)std::min(1024L, std::max(1L, (n4 / world + 255) / 256));
  hipLaunchKernelGGL(p2p_reduce_scatter_kernel, dim3(rs_blocks), dim3(256), 0, st, t, rank, world, n4, half_bytes,
                     epoch);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 1);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(p2p_all_gather_kernel, dim3(blocks), dim3(256), 0, st, t, world, n4, half_bytes, (f32x4*)out,
                     epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

// out (fp32) = resid + bias + sum over ranks of x (bf16, n % 8 == 0, n * 2 <= half_bytes); resid / bias
// optional (null), bias indexed by column (ncols % 8 == 0).  mode as dtc_p2p_allreduce; x may not alias out.
// x == nullptr: the partial is already in this rank's buffer half of the call (the row-parallel GEMM wrote
// it there, parallel/p2p.py staged_out): no stage launch -- barrier + one-shot (2 launches) or barrier +
// reduce-scatter + barrier + all-gather (4).
int dtc_p2p_allreduce_bf16(const bf16* x, float* out, long n, void* const* bases, int rank, int world, long half_bytes,
                           uint32_t* epoch, int* err, int mode, const float* resid, const float* bias, int ncols,
                           hipStream_t st) {
  if (world < 1 || world > P2P_MAX || n % 8 || n * 2 > half_bytes || (bias && (ncols <= 0 || ncols % 8))) return 4001;
  PeerTable t;
  for (int p = 0; p < P2P_MAX; ++p) t.base[p] = (unsigned char*)(p < world ? bases[p] : nullptr);
  const long n8 = n / 8;
  const int blocks = (int)std::min(1024L, std::max(1L, (n8 + 255) / 256));
  const bool one = mode == 2 || (mode == 0 && oneshot_auto(n * 2, world));
  if (x) {
    hipLaunchKernelGGL(p2p_stage_bf16_kernel, dim3(blocks), dim3(256), 0, st, (const bf16x8*)x, t, rank, n8,
                       half_bytes, epoch);
    DTC_CHECK_LAUNCH();
  }
  if (one) {
    hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 2);
    DTC_CHECK_LAUNCH();
    hipLaunchKernelGGL(p2p_oneshot_bf16_kernel, dim3(blocks), dim3(256), 0, st, t, world, n8, half_bytes, out, resid,
                       bias, ncols, epoch);
    DTC_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 1);
  DTC_CHECK_LAUNCH();
  const int rs_blocks = (int)std::min(1024L, std::max(1L, (n8 / world + 255) / 256));
  hipLaunchKernelGGL(p2p_reduce_scatter_bf16_kernel, dim3(rs_blocks), dim3(256), 0, st, t, rank, world, n8, half_bytes,
                     epoch);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 1);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(p2p_all_gather_bf16_kernel, dim3(blocks), dim3(256), 0, st, t, world, n8, half_bytes, out, resid,
                     bias, ncols, epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

// ---- sequence-parallel collectives (one barrier each, epoch + 2 per call like the one-shot all-reduce)
// reduce-scatter of a [W * n_loc] partial (bf16 if bf16 else fp32) into this rank's n_loc fp32 elements:
// out = resid + bias + sum_ranks partial[rank * n_loc .. +n_loc].  x == nullptr: the producer wrote the
// partial into this call's buffer half (staged_out).  n_loc % 8 == 0; bias by column (ncols % 8 == 0,
// n_loc % ncols == 0: whole rows per rank).
int dtc_p2p_reduce_scatter(const void* x, int bf16, float* out, long n_loc, void* const* bases, int rank, int world,
                           long half_bytes, uint32_t* epoch, int* err, const float* resid, const float* bias,
                           int ncols, hipStream_t st) {
  const long esz = bf16 ? 2 : 4;
  if (world < 1 || world > P2P_MAX || n_loc % 8 || n_loc * world * esz > half_bytes ||
      (bias && (ncols <= 0 || ncols % 8 || n_loc % ncols)))
    return 4001;
  PeerTable t;
  for (int p = 0; p < P2P_MAX; ++p) t.base[p] = (unsigned char*)(p < world ? bases[p] : nullptr);
  if (x) {
    const long n16 = n_loc * world * esz / 16;
    const int sb = (int)std::min(1024L, std::max(1L, (n16 + 255) / 256));
    hipLaunchKernelGGL(p2p_stage16_kernel, dim3(sb), dim3(256), 0, st, (const u32x4*)x, t, rank, 0L, n16, half_bytes,
                       epoch);
    DTC_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 2);
  DTC_CHECK_LAUNCH();
  const long n8 = n_loc / 8;
  const int blocks = (int)std::min(1024L, std::max(1L, (n8 + 255) / 256));
  if (bf16)
    hipLaunchKernelGGL(p2p_rs_kernel<true>, dim3(blocks), dim3(256), 0, st, t, rank, world, n8, half_bytes, out, resid,
                       bias, ncols, epoch);
  else
    hipLaunchKernelGGL(p2p_rs_kernel<false>, dim3(blocks), dim3(256), 0, st, t, rank, world, n8, half_bytes, out,
                       resid, bias, ncols, epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

// all-gather of this rank's loc_bytes (x, a multiple of 16) into out [W * loc_bytes], rank-major.
// x == nullptr: the producer already wrote the slot (staged_out at offset rank * loc_bytes).
int dtc_p2p_all_gather(const void* x, void* out, long loc_bytes, void* const* bases, int rank, int world,
                       long half_bytes, uint32_t* epoch, int* err, hipStream_t st) {
  if (world < 1 || world > P2P_MAX || loc_bytes % 16 || loc_bytes * world > half_bytes) return 4001;
  PeerTable t;
  for (int p = 0; p < P2P_MAX; ++p) t.base[p] = (unsigned char*)(p < world ? bases[p] : nullptr);
  const long n16 = loc_bytes / 16;
  if (x) {
    const int sb = (int)std::min(1024L, std::max(1L, (n16 + 255) / 256));
    hipLaunchKernelGGL(p2p_stage16_kernel, dim3(sb), dim3(256), 0, st, (const u32x4*)x, t, rank, rank * n16, n16,
                       half_bytes, epoch);
    DTC_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 2);
  DTC_CHECK_LAUNCH();
  const int blocks = (int)std::min(1024L, std::max(1L, (n16 * world + 255) / 256));
  hipLaunchKernelGGL(p2p_ag_kernel, dim3(blocks), dim3(256), 0, st, t, world, n16, half_bytes, (u32x4*)out, epoch);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_cu_hog(int blocks, long ticks, int lds_bytes, int* sink, hipStream_t st) {
  if (blocks <= 0) return 0;
  if (ticks <= 0 || ticks > 200000000L || lds_bytes < 1024) return 4001;  // at most 2 s
  hipError_t e = hipFuncSetAttribute((const void*)cu_hog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(cu_hog_kernel, dim3(blocks), dim3(256), lds_bytes, st, (uint64_t)ticks, sink);
  DTC_CHECK_LAUNCH();
  return 0;
}

// A call with no payload (one barrier round, epoch + 2): keeps the number of calls per step even, so the
// buffer half of every call site -- which the host hands to a producer GEMM (staged_out) -- is the same
// on every replay of a captured step.
int dtc_p2p_barrier_round(void* const* bases, int rank, int world, uint32_t* epoch, int* err, hipStream_t st) {
  if (world < 1 || world > P2P_MAX) return 4001;
  PeerTable t;
  for (int p = 0; p < P2P_MAX; ++p) t.base[p] = (unsigned char*)(p < world ? bases[p] : nullptr);
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, t, rank, world, epoch, err, 2);
  DTC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
