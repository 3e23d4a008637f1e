// Main-loop probe for the 256x256 lm_head GEMM: the shipped 2-buffer BK=64 loop vs an LDS-DMA
// ring of BK=32 stages (NST slots, NST-1 K-steps in flight, counted vmcnt + raw s_barrier).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm256_ring_probe.hip -o /tmp/p && /tmp/p
// MODE 0: full loop, 1: MFMA + LDS reads only (no DMA after the prologue), 2: DMA + barriers only.
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// K-major 32-k image [256 rows][32 k] (64-B rows): 16-B chunk c of row r at c ^ f((r >> 2) & 3),
// f = {0, 2, 3, 1}: conflict-free for the ds_read_b128 lane groups of a 16x32 fragment.
__device__ __forceinline__ int k32_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <bool KMAJ>
__device__ __forceinline__ void dma32(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, bf16* img,
                                      int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = q * 8 + wave;  // 16 x 1-KB pieces per image
    const bf16* src;
    if (KMAJ) {                    // 16 rows x 64 B
      const int row = blk * 16 + (lane >> 2);
      const int c = (lane & 3) ^ k32_swz(row);
      src = X + (long)min(r0 + row, rmax - 1) * ldx + k0 + c * 8;
    } else {                       // 2 k-rows x 512 B
      const int kr = blk * 2 + (lane >> 5);
      const int c = (lane & 31) ^ mn_swz(kr);
      src = X + (long)(k0 + kr) * ldx + min(r0 + c * 8, rmax - 8);
    }
    __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(img + blk * 512), 16, 0, 0);
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag32(const bf16* img, int t, int lane) {
  if (KMAJ) {
    const int g = lane >> 4, row = t * 16 + (lane & 15);
    return *(const bf16x8*)(img + row * 32 + ((g ^ k32_swz(row)) << 3));
  }
  return big_frag<false>(img, t, 0, lane);
}

constexpr int IMG32 = 256 * 32;

template <bool AK, bool BKM, int NST, int MODE>
__global__ void __launch_bounds__(NT2, 1)
ring256(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K, int tiles_m,
        int tiles_n, int gm, float* out) {
  constexpr int TM = 8, TN = 4, STAGE = 2 * IMG32, G = 4;
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int m0 = (grp * gm + in_g % gm_eff) * 256, n0 = (in_g / gm_eff) * 256;
  const int nk = K / 32;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) {
      dma32<AK>(A, lda, m0, M, s * 32, smem + s * STAGE, wave, lane);
      dma32<BKM>(B, ldb, n0, N, s * 32, smem + s * STAGE + IMG32, wave, lane);
    }
  for (int kt = 0; kt < nk; ++kt) {
    if (MODE == 1 && kt >= NST - 1) {
      wait_vmcnt<0>();
    } else {
      wait_tiles<G, 3>(min(NST - 2, nk - 1 - kt));
    }
    raw_barrier();
    const int nt = kt + NST - 1;
    if (nt < nk && MODE != 1) {
      bf16* sl = smem + (nt % NST) * STAGE;
      dma32<AK>(A, lda, m0, M, nt * 32, sl, wave, lane);
      dma32<BKM>(B, ldb, n0, N, nt * 32, sl + IMG32, wave, lane);
    }
    if (MODE == 2) continue;
    const bf16* sA = smem + (kt % NST) * STAGE;
    const bf16* sB = sA + IMG32;
    bf16x8 fa[TM], fb[TN];
#pragma unroll
    for (int j = 0; j < TM; ++j) fa[j] = frag32<AK>(sA, wm * 8 + j, lane);
#pragma unroll
    for (int i = 0; i < TN; ++i) fb[i] = frag32<BKM>(sB, wn * 4 + i, lane);
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  if (s == 12345.f) out[blockIdx.x] = s;  // keep the accumulators live
}

// copy-only probe: the same operand bytes per K-step moved global -> VGPR -> LDS (register
// staging, 2 x 16 B per lane per image, loads for step k+1 in flight while step k is written)
template <bool KMAJ>
__device__ __forceinline__ void rs_load(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, int tid,
                                        u32x4 (&v)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = q * 8 + (tid >> 6), lane = tid & 63;
    const int row = blk * 16 + (lane >> 2), c = lane & 3;
    v[q] = *(const u32x4*)(X + (long)min(r0 + row, rmax - 1) * ldx + k0 + c * 8);
  }
}
__global__ void __launch_bounds__(NT2, 1)
copy256(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K, int tiles_m,
        int tiles_n, int gm, float* out) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * IMG32];
  const int tid = threadIdx.x;
  const int ntiles = tiles_m * tiles_n;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int m0 = (grp * gm + in_g % gm_eff) * 256, n0 = (in_g / gm_eff) * 256;
  const int nk = K / 32;
  u32x4 va[2], vb[2];
  rs_load<true>(A, lda, m0, M, 0, tid, va);
  rs_load<true>(B, ldb, n0, N, 0, tid, vb);
  for (int kt = 0; kt < nk; ++kt) {
    bf16* st = smem + (kt & 1) * 2 * IMG32;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *(u32x4*)(st + (q * 512 + tid) * 8) = va[q];
      *(u32x4*)(st + IMG32 + (q * 512 + tid) * 8) = vb[q];
    }
    if (kt + 1 < nk) {
      rs_load<true>(A, lda, m0, M, (kt + 1) * 32, tid, va);
      rs_load<true>(B, ldb, n0, N, (kt + 1) * 32, tid, vb);
    }
    __syncthreads();
  }
  if (tid == 0 && smem[tid * 8] == bf16(123.f)) out[blockIdx.x] = 1.f;
}

// checks one output tile of the ring kernel against a host dot product (MODE 0 only)
template <bool AK, bool BKM, int NST>
__global__ void __launch_bounds__(NT2, 1)
ring256_check(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
              float* out) {
  constexpr int TM = 8, TN = 4, STAGE = 2 * IMG32, G = 4;
  __shared__ __attribute__((aligned(16))) bf16 smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = 0, n0 = 0, nk = K / 32;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) {
      dma32<AK>(A, lda, m0, M, s * 32, smem + s * STAGE, wave, lane);
      dma32<BKM>(B, ldb, n0, N, s * 32, smem + s * STAGE + IMG32, wave, lane);
    }
  for (int kt = 0; kt < nk; ++kt) {
    wait_tiles<G, 3>(min(NST - 2, nk - 1 - kt));
    raw_barrier();
    const int nt = kt + NST - 1;
    if (nt < nk) {
      bf16* sl = smem + (nt % NST) * STAGE;
      dma32<AK>(A, lda, m0, M, nt * 32, sl, wave, lane);
      dma32<BKM>(B, ldb, n0, N, nt * 32, sl + IMG32, wave, lane);
    }
    const bf16* sA = smem + (kt % NST) * STAGE;
    const bf16* sB = sA + IMG32;
    bf16x8 fa[TM], fb[TN];
#pragma unroll
    for (int j = 0; j < TM; ++j) fa[j] = frag32<AK>(sA, wm * 8 + j, lane);
#pragma unroll
    for (int i = 0; i < TN; ++i) fb[i] = frag32<BKM>(sB, wn * 4 + i, lane);
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
  }
  const int g4 = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = wm * 128 + j * 16 + (lane & 15), n = wn * 64 + i * 16 + g4;
      *(f32x4*)(out + m * 256 + n) = acc[i][j];
    }
}

template <bool AK, bool BKM, int NST, int MODE>
float time_ring(const bf16* A, long lda, const bf16* B, long ldb, int M, int N, int K, float* out, int reps,
                int gm = 0) {
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
  if (gm <= 0) gm = tiles_m;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto go = [&] {
    hipLaunchKernelGGL((ring256<AK, BKM, NST, MODE>), dim3(tiles_m * tiles_n), dim3(NT2), 0, 0, A, lda, B, ldb, M, N, K,
                       tiles_m, tiles_n, gm, out);
  };
  for (int i = 0; i < 3; ++i) go();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) go();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

static float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
  const int M = 4096, N = 50304, KMAX = 4096;
  std::vector<uint16_t> h((size_t)N * KMAX);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 65536.f - 0.5f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B; float* out;
  CK(hipMalloc(&A, (size_t)M * KMAX * 2)); CK(hipMalloc(&B, (size_t)N * KMAX * 2));
  CK(hipMalloc(&out, (size_t)256 * 256 * 4));
  CK(hipMemcpy(A, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data() + 7, (size_t)N * KMAX * 2, hipMemcpyHostToDevice));
  // correctness of the ring images: tile (0,0), K = 512, both layout pairings used by the lm_head
  {
    const int K = 512;
    std::vector<float> got(256 * 256);
    hipLaunchKernelGGL((ring256_check<true, true, 4>), dim3(1), dim3(NT2), 0, 0, A, (long)KMAX, B, (long)KMAX, M, N, K, out);
    CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
    double maxerr = 0;
    for (int m = 0; m < 256; m += 7)
      for (int n = 0; n < 256; n += 5) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += (double)bf2f(h[(size_t)m * KMAX + k]) * bf2f(h[7 + (size_t)n * KMAX + k]);
        maxerr = std::max(maxerr, std::fabs(s - got[m * 256 + n]));
      }
    printf("check K-major x K-major: max abs err %.3e\n", maxerr);
    // MN-major A: A^T stored [K][M] (lda = M) -- reuse B's buffer as a [K][N] matrix, take its first 256 cols
    hipLaunchKernelGGL((ring256_check<false, true, 4>), dim3(1), dim3(NT2), 0, 0, B, (long)N, A, (long)KMAX, 256, M, K, out);
    CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
    maxerr = 0;
    for (int m = 0; m < 256; m += 7)
      for (int n = 0; n < 256; n += 5) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += (double)bf2f(h[7 + (size_t)k * N + m]) * bf2f(h[(size_t)n * KMAX + k]);
        maxerr = std::max(maxerr, std::fabs(s - got[m * 256 + n]));
      }
    printf("check MN-major x K-major: max abs err %.3e\n", maxerr);
  }
  for (int K : {512, 4096}) {
    const double fl = 2.0 * M * N * K;
    float t40 = time_ring<true, true, 4, 0>(A, KMAX, B, KMAX, M, N, K, out, 10);
    float t50 = time_ring<true, true, 5, 0>(A, KMAX, B, KMAX, M, N, K, out, 10);
    float t41 = time_ring<true, true, 4, 1>(A, KMAX, B, KMAX, M, N, K, out, 10);
    float t42 = time_ring<true, true, 4, 2>(A, KMAX, B, KMAX, M, N, K, out, 10);
    float t30 = time_ring<true, true, 3, 0>(A, KMAX, B, KMAX, M, N, K, out, 10);
    printf("K=%4d ring NST=3 %7.1f us (%6.1f TF/s) | NST=4 %7.1f (%6.1f) | NST=5 %7.1f (%6.1f) | NST=4 no-DMA %7.1f "
           "(%6.1f) | NST=4 DMA-only %7.1f\n",
           K, t30, fl / t30 * 1e-6, t40, fl / t40 * 1e-6, t50, fl / t50 * 1e-6, t41, fl / t41 * 1e-6, t42);
  }
  {
    const int K = 4096, tiles_m = 16, tiles_n = (N + 255) / 256;
    auto go = [&] {
      hipLaunchKernelGGL(copy256, dim3(tiles_m * tiles_n), dim3(NT2), 0, 0, A, (long)KMAX, B, (long)KMAX, M, N, K,
                         tiles_m, tiles_n, tiles_m, out);
    };
    for (int i = 0; i < 3; ++i) go();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 5; ++i) go();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("K=4096 register-staged copy-only %7.1f us\n", ms * 1e3f / 5);
  }
  for (int gm : {16, 4}) {
    const int K = 4096;
    const double fl = 2.0 * M * N * K;
    float t0 = time_ring<true, true, 3, 0>(A, KMAX, B, KMAX, M, N, K, out, 5, gm);
    float t2 = time_ring<true, true, 3, 2>(A, KMAX, B, KMAX, M, N, K, out, 5, gm);
    printf("K=4096 gm=%2d NST=3 full %7.1f us (%6.1f TF/s) | DMA-only %7.1f us\n", gm, t0, fl / t0 * 1e-6, t2);
  }
  return 0;
}
