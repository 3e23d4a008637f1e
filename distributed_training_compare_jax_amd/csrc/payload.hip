// Communication-payload kernels: bf16 transport with fp32 accumulation for the DP gradient exchange
// and the PP activation / gradient messages (parallel/dp.py, parallel/pp.py).
//
// DP bf16 bucket exchange (one bucket of n fp32 grads over dp ranks, shard s = n / dp):
//   cast grads -> bf16 [dp][s];  all_to_all: rank r receives shard r of every rank;
//   shard_sum: out[i] = bf16( sum_j in[j][i] ) in fp32, j ascending (every rank sums its shard in the
//   same order -> replicas stay identical);  all_gather the bf16 shards;  cast back to fp32.
// Per rank that moves (dp-1)/dp * n * 2 bytes each way over xGMI -- half an fp32 ring all-reduce -- and
// the all-to-all drives every point-to-point link of the node at once instead of one ring neighbour.
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) shard_sum_bf16_kernel(const bf16* __restrict__ in, int nshards, long s8,
                                                             bf16* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < s8; i += (long)gridDim.x * blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    DTC_ASSERT(nshards >= 1);
    for (int j = 0; j < nshards; ++j) {
      const bf16x8 v = ((const bf16x8*)in)[(long)j * s8 + i];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    ((bf16x8*)out)[i] = o;
  }
}

__global__ void __launch_bounds__(256) cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = ((const bf16x8*)x)[i];
    f32x4 a, b;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = (float)v[e];
      b[e] = (float)v[e + 4];
    }
    ((f32x4*)y)[2 * i] = a;
    ((f32x4*)y)[2 * i + 1] = b;
  }
}

inline int grid_for(long n) { return (int)std::min(4096L, std::max(1L, (n + 255) / 256)); }

}  // namespace

extern "C" {

// out[i] = bf16(sum_{j < nshards} in[j*s + i]) for i < s; s % 8 == 0, 16-B aligned buffers
int dtc_shard_sum_bf16(const bf16* in, int nshards, long s, bf16* out, hipStream_t st) {
  DTC_HOST_CHECK(in && out && nshards >= 1 && s >= 0 && s % 8 == 0);
  DTC_HOST_CHECK((unsigned long)in % 16 == 0 && (unsigned long)out % 16 == 0);
  if (s == 0) return 0;
  hipLaunchKernelGGL(shard_sum_bf16_kernel, dim3(grid_for(s / 8)), dim3(256), 0, st, in, nshards, s / 8, out);
  DTC_CHECK_LAUNCH();
  return 0;
}

// y[i] = float(x[i]); n % 8 == 0, 16-B aligned buffers
int dtc_cast_bf16_f32(const bf16* x, float* y, long n, hipStream_t st) {
  DTC_HOST_CHECK(x && y && n >= 0 && n % 8 == 0 && (unsigned long)x % 16 == 0 && (unsigned long)y % 16 == 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, x, y, n / 8);
  DTC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
