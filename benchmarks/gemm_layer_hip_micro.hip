// Where a layer GEMM's time goes (built and run on the GPU box):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm_layer_hip_micro.hip -o /tmp/gl && /tmp/gl
// For the fc1 forward shape [4096 x 2048 x 512] and the out_proj forward [4096 x 512 x 512]: main loop
// only (EPI_NONE) vs bf16 store vs the production epilogue, a K sweep of the main loop (fixed cost
// vs per-K-step cost) and an empty-kernel launch in the same stream.
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel() {}

float timeit(const std::function<void()>& f, int reps = 50) {
  for (int i = 0; i < 5; ++i) f();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  const int M = 4096, KMAX = 4096, NMAX = 2048;
  std::vector<uint16_t> h((size_t)M * KMAX);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 65536.f - 0.5f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C, *C2; float *bias, *R;
  CK(hipMalloc(&A, (size_t)M * KMAX * 2)); CK(hipMalloc(&B, (size_t)NMAX * KMAX * 2));
  CK(hipMalloc(&C, (size_t)M * NMAX * 2)); CK(hipMalloc(&C2, (size_t)M * NMAX * 2));
  CK(hipMalloc(&bias, NMAX * 4)); CK(hipMalloc(&R, (size_t)M * NMAX * 4));
  CK(hipMemcpy(A, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)NMAX * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, NMAX * 4)); CK(hipMemset(R, 0, (size_t)M * NMAX * 4));
  printf("empty kernel (back to back): %6.2f us\n", timeit([] { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, 0); }));
  auto args = [&](int N, int K) {
    GemmArgs a{};
    a.layout = 0; a.M = M; a.N = N; a.K = K; a.A = A; a.lda = KMAX; a.B = B; a.ldb = KMAX; a.C = C; a.ldc = N;
    a.alpha = 1.f; a.bias = bias; a.aux_out = C2;
    return a;
  };
  for (int N : {2048, 512}) {
    const int K = 512;
    const double fl = 2.0 * M * N * K;
    GemmArgs a = args(N, K);
    for (int bm : {128, 64}) {
      Plan p{bm, bm, 64, 1};
      float t0 = timeit([&] { launch_sz<true, true, EPI_NONE, false>(a, p, 0); });
      float t1 = timeit([&] { launch_sz<true, true, EPI_STORE, false>(a, p, 0); });
      GemmArgs an = a; an.bias = nullptr;
      float t1n = timeit([&] { launch_sz<true, true, EPI_STORE, false>(an, p, 0); });
      GemmArgs af = a; af.C = R; af.c_f32 = 1;
      float t1f = timeit([&] { launch_sz<true, true, EPI_STORE, true>(af, p, 0); });
      float t2 = N == 2048 ? timeit([&] { launch_sz<true, true, EPI_GELU, false>(a, p, 0); }) : 0.f;
      GemmArgs ar = a; ar.C = R; ar.c_f32 = 1; ar.aux = R; ar.ldaux = N;  // residual read from the output buffer
      float t3 = N == 512 ? timeit([&] { launch_sz<true, true, EPI_RESID, true>(ar, p, 0); }) : 0.f;
      printf("[%d x %d x %d] %3d^2: main loop %6.2f us (%5.1f TF/s) | +bf16 store %6.2f (no bias %6.2f) | +f32 store %6.2f | "
             "+gelu %6.2f | +resid f32 %6.2f\n", M, N, K, bm, t0, fl / t0 * 1e-6, t1, t1n, t1f, t2, t3);
      for (int k : {64, 512}) {
        GemmArgs ak = args(N, k);
        float t = timeit([&] { launch_sz<true, true, EPI_NONE, false>(ak, p, 0); });
        printf("    K=%5d main loop %6.2f us (%5.1f TF/s)\n", k, t, 2.0 * M * N * k / t * 1e-6);
      }
    }
  }
  return 0;
}
