// Probe: an 8-wave (2 waves per SIMD) DMA-ring layer GEMM vs the production kernels, main loop only
// (EPI_NONE) and with a plain bf16 store, at the forward layer shapes.  Built and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm_dma8_micro.hip -o /tmp/d8 && /tmp/d8
// Question: does a deeper global->LDS ring with 8 waves per block lift the per-CU fill rate that
// bounds the 128^2 register-staged kernel (~45 GB/s per CU) at these 1-2 tiles-per-CU grids?
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int R, bool KMAJ, int NW>
struct DImgW {
  using Base = DImg<R, KMAJ>;
  static constexpr int ELEMS = Base::ELEMS;
  static constexpr int NI = ELEMS * 2 / 1024 / NW;
  static_assert(NI >= 1, "image too small for the wave count");
  __device__ __forceinline__ static void dma(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, bf16* img,
                                             int wave, int lane) {
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int blk = q * NW + wave;
      const bf16* src;
      if (KMAJ) {
        const int row = blk * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        src = X + (long)min(r0 + row, rmax - 1) * ldx + k0 + c * 8;
      } else {
        constexpr int LPR = R / 8;
        const int kr = blk * (64 / LPR) + lane / LPR;
        const int c = (lane % LPR) ^ dimg_mn_swz<R>(kr);
        src = X + (long)(k0 + kr) * ldx + min(r0 + c * 8, rmax - 8);
      }
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(img + blk * 512), 16, 0, 0);
    }
  }
};

template <int BM, int BN, int NSTAGE, int WGM, int WGN, bool AK, bool BKM, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN, 1)
gemm_dmaw_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
                 int tiles_m, int tiles_n, int gm, bf16* __restrict__ C, long ldc) {
  constexpr int NW = WGM * WGN;
  using IA = DImgW<BM, AK, NW>;
  using IB = DImgW<BN, BKM, NW>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  constexpr int G = IA::NI + IB::NI;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lid % ntiles, z = lid / ntiles;  // split-K slice z: k range [z*K, (z+1)*K)
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int m0 = (grp * gm + in_g % gm_eff) * BM, n0 = (in_g / gm_eff) * BN;
  const int nk = K / 64;
  A += AK ? (long)z * K : (long)z * K * lda;  // K-major: column offset; MN-major: row offset
  B += BKM ? (long)z * K : (long)z * K * ldb;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) {
      IA::dma(A, lda, m0, M, s * 64, smem + s * STAGE, wave, lane);
      IB::dma(B, ldb, n0, N, s * 64, smem + s * STAGE + IA::ELEMS, wave, lane);
    }
  for (int kt = 0; kt < nk; ++kt) {
    wait_tiles<G, NSTAGE - 2>(min(NSTAGE - 2, nk - 1 - kt));
    raw_barrier();
    const int nt = kt + NSTAGE - 1;
    if (nt < nk) {
      bf16* sl = smem + (nt % NSTAGE) * STAGE;
      IA::dma(A, lda, m0, M, nt * 64, sl, wave, lane);
      IB::dma(B, ldb, n0, N, nt * 64, sl + IA::ELEMS, wave, lane);
    }
    const bf16* sA = smem + (kt % NSTAGE) * STAGE;
    const bf16* sB = sA + IA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = DImg<BM, AK>::frag(sA, wm * TM + j, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = DImg<BN, BKM>::frag(sB, wn * TN + i, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
  }
  if constexpr (EPI == EPI_NONE) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  const int g4 = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + (lane & 15), n = n0 + wn * WN + i * 16 + g4;
      if (m < M && n + 4 <= N)
        *(bf16x4*)(C + (long)m * ldc + n) = bf16x4{f2bf(acc[i][j][0]), f2bf(acc[i][j][1]), f2bf(acc[i][j][2]), f2bf(acc[i][j][3])};
    }
}

static float timeit(const std::function<void()>& f, int reps = 40) {
  for (int i = 0; i < 3; ++i) f();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> r;
  for (int round = 0; round < 5; ++round) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    r.push_back(ms * 1e3f / reps);
  }
  std::sort(r.begin(), r.end());
  return r[2];
}

template <int BM, int BN, int NSTAGE, int WGM, int WGN, bool AK, bool BKM, int EPI>
float run_w(int M, int N, int K, const bf16* A, long lda, const bf16* B, long ldb, bf16* C, int split = 1) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN, nt = tm * tn;
  const int gm = tn <= 16 ? std::max(1, std::min(tm, (nt / 8 + tn - 1) / tn)) : tm;
  const int kk = K / split;  // split-K: each block's K range (slab epilogue not modelled: main loop only)
  return timeit([&] {
    hipLaunchKernelGGL((gemm_dmaw_kernel<BM, BN, NSTAGE, WGM, WGN, AK, BKM, EPI>), dim3(nt * split), dim3(64 * WGM * WGN), 0,
                       0, A, lda, B, ldb, M, N, kk, tm, tn, gm, C, (long)N);
  });
}

template <bool AK, bool BKM>
void sweep(const char* name, int M, int N, int K, const bf16* A, const bf16* B, bf16* C, int split) {
  const long lda = AK ? K : M, ldb = BKM ? K : N;
  printf("%-10s [%5d x %5d x %5d] split %d:", name, M, N, K, split);
  printf(" 256x128(4x2)s2 %6.2f", run_w<256, 128, 2, 4, 2, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" s3 %6.2f", run_w<256, 128, 3, 4, 2, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 256x128(2x4)s2 %6.2f", run_w<256, 128, 2, 2, 4, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 128x256(2x4)s2 %6.2f", run_w<128, 256, 2, 2, 4, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 128x128(4x2)s4 %6.2f", run_w<128, 128, 4, 4, 2, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 128x64(4x2)s4 %6.2f", run_w<128, 64, 4, 4, 2, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 128x64(2x4)s4 %6.2f", run_w<128, 64, 4, 2, 4, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  printf(" | 64x128(2x4)s4 %6.2f\n", run_w<64, 128, 4, 2, 4, AK, BKM, EPI_NONE>(M, N, K, A, lda, B, ldb, C, split));
  fflush(stdout);
}

int main() {
  const int M = 4096, KMAX = 4096, NMAX = 2048;
  std::vector<uint16_t> h((size_t)M * KMAX);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 65536.f - 0.5f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * KMAX * 2)); CK(hipMalloc(&B, (size_t)NMAX * KMAX * 2)); CK(hipMalloc(&C, (size_t)M * NMAX * 2));
  CK(hipMemcpy(A, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)NMAX * 2048 * 2, hipMemcpyHostToDevice));
  // production reference: the register-staged 128^2 kernel, main loop only
  {
    GemmArgs a{};
    a.layout = 0; a.M = M; a.N = 2048; a.K = 512; a.A = A; a.lda = 512; a.B = B; a.ldb = 512; a.C = C; a.ldc = 2048; a.alpha = 1.f;
    Plan p128{128, 128, 64, 1};
    printf("reg128 fc1 fwd main loop %6.2f us\n", timeit([&] { launch_t<128, 128, true, true, EPI_NONE, false>(a, p128, 0); }));
  }
  // wgrad (both MN-major), K = tokens
  sweep<false, false>("wgrad qkv", 1536, 512, 4096, A, B, C, 2);
  sweep<false, false>("wgrad qkv", 1536, 512, 4096, A, B, C, 4);
  sweep<false, false>("wgrad out", 512, 512, 4096, A, B, C, 4);
  sweep<false, false>("wgrad out", 512, 512, 4096, A, B, C, 8);
  sweep<false, false>("wgrad fc1", 2048, 512, 4096, A, B, C, 2);
  sweep<false, false>("wgrad fc1", 2048, 512, 4096, A, B, C, 4);
  sweep<false, false>("wgrad fc2", 512, 2048, 4096, A, B, C, 2);
  sweep<false, false>("wgrad fc2", 512, 2048, 4096, A, B, C, 4);
  return 0;
}
