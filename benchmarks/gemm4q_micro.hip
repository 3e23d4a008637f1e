// 4-wave 256^2 GEMM main loop ("gemm4q"): one wave per SIMD, 128 x 128 output per wave (256 accumulator
// registers, the MFMA accumulators in AGPRs), k32 sub-steps through a 5-slot LDS-DMA ring (5 x 32 KB = 160 KB).
// Yardstick: hipBLASLt's own MT256x256x64 kernel runs 256-thread workgroups (rocprofv3 names,
// benchmarks/hipblaslt_kernel_names.py) and beats our 8-wave ping-pong gemm8p by 20 % per K-step at 4096^3.
// Per K-step of 64 a wave reads 32 fragments for 128 MFMAs (gemm8p: 24 for 64).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm4q_micro.hip -o benchmarks/bin/gemm4q_micro
#include "../distributed_training_compare_jax_amd/csrc/common.h"
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace {

constexpr int BIG = 256;
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;
__device__ __forceinline__ int mn8_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }
__device__ __forceinline__ s16x4 ds_tr16_asm(const bf16* p) {
  s16x4 r;
  const unsigned a = (unsigned)(unsigned long)(DTC_LDS void*)(p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
#define P8_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
template <int N>
__device__ __forceinline__ void vmcnt_c() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

constexpr int Q4_IMG = BIG * 32;       // one operand's image of a k32 sub-step (16 KB)
constexpr int Q4_SLOT = 2 * Q4_IMG;    // A image | B image
#ifndef Q4_NS
#define Q4_NS 5
#endif
#ifndef Q4_EARLY
#define Q4_EARLY 0
#endif

// K-major image [256 rows][32 k], 64-B rows; 16-B piece p of row r holds k-piece p ^ q4_swz(r):
// conflict-free ds_read_b128 fragment reads (each 16-lane group covers the 4 pieces of 4 row residues)
__device__ __forceinline__ int q4_swz(int r) { return (-(r >> 2)) & 3; }

// per-lane DMA source of instruction i (0..3) of one operand at k0 = 0; instruction blk = 4 i + wave
// fills image bytes [1 KB blk, 1 KB (blk + 1)).  K-major: rows 16 blk..; MN-major: chunk blk >> 2
// ([32 k][64 cols], 128-B k-rows, 16-B piece c of k-row r at c ^ mn8_swz(r)), k-rows 8 (blk & 3)..
template <bool KMAJ>
__device__ __forceinline__ const bf16* q4_src(const bf16* __restrict__ X, long ldx, int r0, int rmax, int i, int wave,
                                              int lane) {
  const int blk = 4 * i + wave;
  if (KMAJ) {
    const int row = blk * 16 + (lane >> 2);
    const int c = (lane & 3) ^ q4_swz(row);
    return X + (long)min(r0 + row, rmax - 1) * ldx + c * 8;
  }
  const int q = blk >> 2, kr = 8 * (blk & 3) + (lane >> 3);
  const int pc = (lane & 7) ^ mn8_swz(kr);
  return X + (long)kr * ldx + min(r0 + 64 * q + 8 * pc, rmax - 8);
}

// fragment of 16-row group t (0..15) of a k32 image, natural k order (lane group g holds k 8g..8g+7)
template <bool KMAJ>
__device__ __forceinline__ bf16x8 q4_frag(const bf16* img, int t, int lane) {
  const int g = lane >> 4, li = lane & 15;
  if (KMAJ) {
    const int row = t * 16 + li;
    return *(const bf16x8*)(img + row * 32 + ((g ^ q4_swz(row)) << 3));
  }
  const int q = li >> 2, pp = li & 3;
  const bf16* base = img + (t >> 2) * 2048;
  const int k0 = 8 * g + q, k1 = k0 + 4;
  const int pc = 2 * (t & 3) + (pp >> 1), w = (pp & 1) * 4;
  const s16x4 lo = ds_tr16_asm(base + k0 * 64 + ((pc ^ mn8_swz(k0)) << 3) + w);
  const s16x4 hi = ds_tr16_asm(base + k1 * 64 + ((pc ^ mn8_swz(k1)) << 3) + w);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int N>
__device__ __forceinline__ void lgkm_c() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

// every fragment register of the set is tied to the wait, so no MFMA consumer moves above it
__device__ __forceinline__ void q4_tie(bf16x8 (&f)[8]) {
  asm volatile("" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]));
}

template <bool AK, bool BKM, int EPI>
__global__ void __launch_bounds__(256, 1)
gemm4q_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
              int tiles_m, int tiles_n, int gm, bf16* __restrict__ C, long ldc) {
  __shared__ __attribute__((aligned(16))) bf16 smem[Q4_NS * Q4_SLOT];
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles);
  const int grp = lid / (gm * tiles_n), in_g = lid % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int tm_idx = grp * gm + in_g % gm_eff, tn_idx = in_g / gm_eff;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = tm_idx * BIG, n0 = tn_idx * BIG;
  const int ns = K / 32;  // >= Q4_NS - 1 (host check)

  const bf16* sa[4];
  const bf16* sb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sa[i] = q4_src<AK>(A, lda, m0, M, i, wave, lane);
    sb[i] = q4_src<BKM>(B, ldb, n0, N, i, wave, lane);
  }
  const long stA = AK ? 32 : 32 * lda, stB = BKM ? 32 : 32 * ldb;
  // the 8 DMA instructions of the next sub-step in source order into ring slot `slot`; sources advance one
  // sub-step (past the last one they stay on it: the extra copies land in free slots, never read)
  int issued = 0;
  auto dma = [&](bf16* slot, int i) {
    bf16* img = slot + (i >= 4 ? Q4_IMG : 0) + ((i & 3) * 4 + wave) * 512;
    __builtin_amdgcn_global_load_lds((glb_vptr)(i < 4 ? sa[i] : sb[i - 4]), (lds_vptr)img, 16, 0, 0);
  };
  auto advance = [&] {
    if (++issued < ns) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { sa[i] += stA; sb[i] += stB; }
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: sub-steps 0 .. NS-2 in flight; sub-steps 0 and 1 landed before the loop
#pragma unroll
  for (int s = 0; s < Q4_NS - 1; ++s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dma(smem + s * Q4_SLOT, i);
    advance();
  }
  vmcnt_c<8 * (Q4_NS - 3)>();
  __builtin_amdgcn_s_barrier();
  bf16x8 fa[2][8], fb[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) fa[0][j] = q4_frag<AK>(smem, 8 * wr + j, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) fb[0][i] = q4_frag<BKM>(smem + Q4_IMG, 8 * wc + i, lane);
  lgkm_c<0>();
  q4_tie(fa[0]);
  q4_tie(fb[0]);

  // ring slots: rd = sub-step s + 1 (fragment reads), wrs = sub-step s + NS - 1 (DMA target)
  bf16* rd = smem + 1 * Q4_SLOT;
  bf16* wrs = smem + (Q4_NS - 1) * Q4_SLOT;
  bf16* const last = smem + (Q4_NS - 1) * Q4_SLOT;
  auto sub = [&](auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
#if Q4_EARLY  // all 16 reads in the first 4 groups: the end-of-sub-step lgkmcnt(0) finds them landed
      if (g < 4) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          fa[nxt][2 * g + u] = q4_frag<AK>(rd, 8 * wr + 2 * g + u, lane);
          fb[nxt][2 * g + u] = q4_frag<BKM>(rd + Q4_IMG, 8 * wc + 2 * g + u, lane);
        }
      }
#else
      fa[nxt][g] = q4_frag<AK>(rd, 8 * wr + g, lane);
      fb[nxt][g] = q4_frag<BKM>(rd + Q4_IMG, 8 * wc + g, lane);
#endif
      dma(wrs, g);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][g], fa[cur][j], acc[g][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    advance();
    lgkm_c<0>();
    q4_tie(fa[nxt]);
    q4_tie(fb[nxt]);
    vmcnt_c<8 * (Q4_NS - 3)>();  // sub-step s + 2 landed (s + 3 .. s + NS - 1 younger)
    __builtin_amdgcn_s_barrier();
    rd = rd == last ? smem : rd + Q4_SLOT;
    wrs = wrs == last ? smem : wrs + Q4_SLOT;
  };
  // one sub-step per trip, the prefetched fragments copied down at the end: unrolling two sub-steps (static
  // buffer parity) made the register allocator rotate ~90 accumulator registers through VGPRs every trip
  for (int s = 0; s < ns; ++s) {
    sub(std::integral_constant<int, 0>{});
#pragma unroll
    for (int g = 0; g < 8; ++g) { fa[0][g] = fa[1][g]; fb[0][g] = fb[1][g]; }
  }
  P8_VMCNT(0);
  if (EPI == EPI_NONE) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  const int g4 = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wr * 128 + j * 16 + (lane & 15), n = n0 + wc * 128 + i * 16 + g4;
      if (m < M && n < N) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        *(bf16x4*)(C + (long)m * ldc + n) = o;
      }
    }
}

// fp32 reference: C[m][n] = sum_k A(m, k) B(n, k), layout 0 (A[m][k], B[n][k]) or 2 (A[k][m], B[k][n])
__global__ void ref_kernel(const bf16* A, const bf16* B, float* C, int S, int layout) {
  const int m = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  float s = 0.f;
  for (int k = 0; k < S; ++k) {
    const float a = layout == 0 ? (float)A[(long)m * S + k] : (float)A[(long)k * S + m];
    const float b = layout == 0 ? (float)B[(long)n * S + k] : (float)B[(long)k * S + n];
    s += a * b;
  }
  C[(long)m * S + n] = s;
}

struct Args { const bf16* A; const bf16* B; bf16* C; int S; };

template <bool AK, bool BKM, int EPI>
float run4(const Args& a, int reps) {
  const int tiles = a.S / BIG;  // gemm8p's launch_big tile order: groups of gm M-tiles sweep the N-tiles
  const int gm = tiles <= 16 ? std::max(1, std::min(tiles, 32 / tiles)) : 3;
  auto go = [&] {
    hipLaunchKernelGGL((gemm4q_kernel<AK, BKM, EPI>), dim3(tiles * tiles), dim3(256), 0, 0, a.A, (long)a.S, a.B,
                       (long)a.S, a.S, a.S, a.S, tiles, tiles, gm, a.C, (long)a.S);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) go();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) go();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

}  // namespace

int main() {
  const long MAXE = 8192L * 8192;
  std::vector<uint16_t> h(MAXE), hb(MAXE);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 32768.f - 1.f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  for (auto& v : hb) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 32768.f - 1.f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, MAXE * 2)); CK(hipMalloc(&B, MAXE * 2)); CK(hipMalloc(&C, MAXE * 2)); CK(hipMalloc(&R, 4096L * 4096 * 4));
  CK(hipMemcpy(A, h.data(), MAXE * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), MAXE * 2, hipMemcpyHostToDevice));
  std::vector<uint16_t> o4(4096L * 4096);
  std::vector<float> ro(4096L * 4096);
  for (int S : {4096, 8192}) {
    const Args a{A, B, C, S};
    const double fl = 2.0 * S * S * S;
    const int reps = S == 4096 ? 20 : 5;
    for (int lay : {0, 2}) {
      float tm, ts;
      CK(hipMemset(C, 0, MAXE * 2));
      if (lay == 0) { tm = run4<true, true, EPI_NONE>(a, reps); ts = run4<true, true, EPI_STORE>(a, reps); }
      else { tm = run4<false, false, EPI_NONE>(a, reps); ts = run4<false, false, EPI_STORE>(a, reps); }
      CK(hipDeviceSynchronize());
      char chk[160] = "";
      if (S == 4096) {
        hipLaunchKernelGGL(ref_kernel, dim3(S / 256, S), dim3(256), 0, 0, (const bf16*)A, (const bf16*)B, R, S, lay);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(o4.data(), C, (long)S * S * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ro.data(), R, (long)S * S * 4, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        long bad = 0;
        for (long i = 0; i < (long)S * S; ++i) {
          const double d = fabs((double)bf2f(o4[i]) - ro[i]), r = fabs((double)ro[i]);
          md = std::max(md, d); mx = std::max(mx, r);
          if (d > 0.01 * r + 0.05) ++bad;
        }
        snprintf(chk, sizeof chk, " | vs fp32 ref: max|diff| %.4f (max|C| %.1f), %ld bad", md, mx, bad);
      }
      printf("gemm4q %d^3 %s  main %.1f us %.0f TF/s | +bf16 store %.1f us %.0f TF/s%s\n", S, lay == 0 ? "NT" : "TN", tm,
             fl / tm / 1e6, ts, fl / ts / 1e6, chk);
      fflush(stdout);
    }
  }
  return 0;
}
