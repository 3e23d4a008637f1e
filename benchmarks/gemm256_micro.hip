// Microbenchmark of the large-tile GEMM kernels (built and run on the GPU box):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm256_micro.hip -o /tmp/g256 && /tmp/g256
// Times main loop only (EPI_NONE), plain bf16 store and the fused lm_head epilogue at the
// lm_head shape, plus a K sweep of the main loop (per-K-tile cost vs fixed prologue/epilogue).
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int EPI, bool F32, bool AK = true, bool BKM = true>
float run(const GemmArgs& a, int reps, int split = 1) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) { int rc = launch_big<AK, BKM, EPI, F32>(a, split, 0); CK((hipError_t)rc); }
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch_big<AK, BKM, EPI, F32>(a, split, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  const int M = 4096, N = 50304, KMAX = 4096;
  std::vector<uint16_t> h((size_t)N * KMAX);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 65536.f - 0.5f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C; float *bias, *part, *lab; int* labels;
  CK(hipMalloc(&A, (size_t)M * KMAX * 2)); CK(hipMalloc(&B, (size_t)N * KMAX * 2)); CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&part, (size_t)M * 1024 * 8)); CK(hipMalloc(&lab, M * 4)); CK(hipMalloc(&labels, M * 4));
  CK(hipMemcpy(A, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, N * 4)); CK(hipMemset(labels, 0, M * 4));
  GemmArgs a{};
  a.layout = 0; a.M = M; a.N = N; a.K = 512; a.A = A; a.lda = KMAX; a.B = B; a.ldb = KMAX; a.C = C; a.ldc = N;
  a.alpha = 1.f; a.bias = bias; a.labels = labels; a.vocab_start = 0; a.n_valid = 50258; a.part = part; a.label_out = lab;
  const double fl = 2.0 * M * N * 512;
  float t0 = run<EPI_NONE, false>(a, 20), t1 = run<EPI_STORE, false>(a, 20), t2 = run<EPI_LMHEAD, false>(a, 20);
  printf("K=512  main-loop-only %7.1f us (%6.1f TF/s) | +bf16 store %7.1f us | +lm_head CE %7.1f us\n", t0, fl / t0 * 1e-6, t1, t2);
  for (int K : {64, 128, 256, 512, 1024, 2048, 4096}) {
    a.K = K;
    float t = run<EPI_NONE, false>(a, 10);
    printf("main loop K=%5d  %8.1f us  %6.1f TF/s\n", K, t, 2.0 * M * N * K / t * 1e-6);
  }
  // lm_head wgrad: dW[V x D] = dlogits^T[V x T] . h[T x D]  (both operands MN-major)
  float* W32; CK(hipMalloc(&W32, (size_t)N * 512 * 4));
  GemmArgs w{};
  w.layout = 2; w.M = N; w.N = 512; w.K = M; w.A = B; w.lda = N; w.B = A; w.ldb = 512; w.C = W32; w.ldc = 512;
  w.c_f32 = 1; w.alpha = 1.f;
  float tw = run<EPI_STORE, true, false, false>(w, 10);
  printf("wgrad [%d x 512 x %d] %7.1f us (%6.1f TF/s)\n", N, M, tw, 2.0 * N * 512 * M / tw * 1e-6);
  // lm_head dgrad: dH[T x D] = dlogits[T x V] . W[V x D]  (A K-major, B MN-major), split-K
  float* ws; CK(hipMalloc(&ws, (size_t)64 << 20));
  bf16* Wb; CK(hipMalloc(&Wb, (size_t)N * 512 * 2));
  CK(hipMemcpy(Wb, h.data(), (size_t)N * 512 * 2, hipMemcpyHostToDevice));
  GemmArgs d{};
  d.layout = 1; d.M = M; d.N = 512; d.K = N; d.A = B; d.lda = N; d.B = Wb; d.ldb = 512; d.C = W32; d.ldc = 512;
  d.c_f32 = 1; d.alpha = 1.f; d.workspace = ws; d.ws_bytes = (long)64 << 20;
  const int sp = big_split(1, M, 512, N);
  float td = run<EPI_STORE, true, true, false>(d, 10, sp);
  printf("dgrad [%d x 512 x %d] split %d %7.1f us (%6.1f TF/s)\n", M, N, sp, td, 2.0 * N * 512 * M / td * 1e-6);
  return 0;
}
