// Sanitizer harness for the native host runtime (csrc/host_data.cpp), built by
// tests/test_native_sanitizers_cpu.py with -fsanitize=address,undefined (host code only: the GPU
// kernels are checked by the numerics tests on the device).  Exercises dtc_synth_tokens the way
// data/synthetic.py drives it — a Zipf-like cdf with a guide table, rank -> id and bigram-successor
// maps — over overlapping windows and edge arguments; any out-of-bounds access, overflow or UB
// aborts the run.  Invariants: every token is a valid id, a window's tokens do not depend on where
// the window starts (pure function of the global position), bad arguments are rejected.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

extern "C" int dtc_synth_tokens(uint64_t key1, uint64_t key2, const double* cdf, int vocab, const int32_t* guide,
                                int gbits, const int64_t* rank_to_id, const int64_t* succ, double p_bigram,
                                int64_t start, int64_t count, int32_t* out);

static int fail(const char* what) {
  std::fprintf(stderr, "host_data_check: %s\n", what);
  return 1;
}

int main() {
  const int vocab = 50258, gbits = 16;
  std::vector<double> cdf(vocab);
  double acc = 0.0;
  for (int r = 0; r < vocab; ++r) acc += 1.0 / std::pow(r + 2.7, 1.07);
  double run = 0.0;
  for (int r = 0; r < vocab; ++r) {
    run += 1.0 / std::pow(r + 2.7, 1.07) / acc;
    cdf[r] = run;
  }
  cdf[vocab - 1] = 1.0;
  const int nb = 1 << gbits;
  std::vector<int32_t> guide(nb + 1);
  for (int b = 0; b <= nb; ++b) {  // searchsorted_right(cdf, b / 2^gbits)
    const double u = static_cast<double>(b) / nb;
    int lo = 0, hi = vocab;
    while (lo < hi) {
      const int mid = (lo + hi) / 2;
      if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
    }
    guide[b] = lo;
  }
  std::vector<int64_t> rank_to_id(vocab), succ(vocab);
  for (int r = 0; r < vocab; ++r) {
    rank_to_id[r] = (static_cast<int64_t>(r) * 7919) % (vocab - 1);  // never the pad id 50257
    succ[r] = (static_cast<int64_t>(r) * 104729 + 13) % (vocab - 1);
  }
  const uint64_t k1 = 0x1234567887654321ull, k2 = 0x0badc0ffee0ddf00ull;
  const int64_t n = 64 * 513;
  std::vector<int32_t> a(n), b(n);
  if (dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), gbits, rank_to_id.data(), succ.data(), 0.35, 1000, n,
                       a.data()))
    return fail("window A rejected");
  for (int64_t i = 0; i < n; ++i)
    if (a[i] < 0 || a[i] >= vocab - 1) return fail("token out of range");
  const int64_t off = 12345;
  if (dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), gbits, rank_to_id.data(), succ.data(), 0.35,
                       1000 + off, n - off, b.data()))
    return fail("window B rejected");
  for (int64_t i = 0; i < n - off; ++i)
    if (b[i] != a[off + i]) return fail("token depends on the window start");
  // position 0 reads z(-1) for the bigram predecessor; an empty window writes nothing
  if (dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), gbits, rank_to_id.data(), succ.data(), 1.0, 0, 1,
                       b.data()))
    return fail("window at position 0 rejected");
  if (dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), gbits, rank_to_id.data(), succ.data(), 0.5, 7, 0,
                       nullptr))
    return fail("empty window rejected");
  if (!dtc_synth_tokens(k1, k2, cdf.data(), 0, guide.data(), gbits, rank_to_id.data(), succ.data(), 0.5, 0, 1,
                        b.data()) ||
      !dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), 25, rank_to_id.data(), succ.data(), 0.5, 0, 1,
                        b.data()) ||
      !dtc_synth_tokens(k1, k2, cdf.data(), vocab, guide.data(), gbits, rank_to_id.data(), succ.data(), 0.5, 0, -1,
                        b.data()))
    return fail("bad arguments accepted");
  std::printf("host_data_check: ok (%lld tokens)\n", static_cast<long long>(n));
  return 0;
}
