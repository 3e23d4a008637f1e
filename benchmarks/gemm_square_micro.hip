// Main-loop efficiency of the 256^2 phase-interleaved kernel (gemm8p_kernel) on large square problems,
// random uniform bf16 operands (cdna_hip_programming.md §5.4 rule 25: quote random-data numbers):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/gemm_square_micro.hip -o benchmarks/bin/gemm_square_micro
// NT = both operands K-major (forward layout), TN = both MN-major (weight-gradient layout).
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <bool AK, bool BKM, int EPI>
float run(const GemmArgs& a, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) { int rc = launch_big<AK, BKM, EPI, false>(a, 1, 0); if (rc) { printf("rc %d\n", rc); exit(1); } }
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch_big<AK, BKM, EPI, false>(a, 1, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  const long MAXE = 8192L * 8192;
  std::vector<uint16_t> h(MAXE);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 32768.f - 1.f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C;
  CK(hipMalloc(&A, MAXE * 2)); CK(hipMalloc(&B, MAXE * 2)); CK(hipMalloc(&C, MAXE * 2));
  CK(hipMemcpy(A, h.data(), MAXE * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), MAXE * 2, hipMemcpyHostToDevice));
  for (int S : {4096, 8192}) {
    GemmArgs a{};
    a.M = S; a.N = S; a.K = S; a.A = A; a.lda = S; a.B = B; a.ldb = S; a.C = C; a.ldc = S; a.alpha = 1.f;
    const double fl = 2.0 * S * S * S;
    const int reps = S == 4096 ? 20 : 5;
    a.layout = 0;
    float t0 = run<true, true, EPI_NONE>(a, reps), t1 = run<true, true, EPI_STORE>(a, reps);
    a.layout = 2;
    float t2 = run<false, false, EPI_NONE>(a, reps), t3 = run<false, false, EPI_STORE>(a, reps);
    printf("%d^3  NT main %.1f us %.0f TF/s | NT store %.1f us %.0f TF/s | TN main %.1f us %.0f TF/s | TN store %.1f us %.0f TF/s\n",
           S, t0, fl / t0 / 1e6, t1, fl / t1 / 1e6, t2, fl / t2 / 1e6, t3, fl / t3 / 1e6);
  }
  return 0;
}
