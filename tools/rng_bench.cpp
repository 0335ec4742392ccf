// Host micro-benchmark of the TransE draw protocol (kp_rng.cpp) on a batch shaped like
// the bench's transe-fb15k237-necessary step (289 calls, ~34k rows, 65 epochs, ratio 5):
// the three chains timed apart (torch-stream walk, numpy shuffles, randint fills) and the
// whole kp_rng_transe_calls + kp_rng_wait.  Not a test: timing only.
//   g++ -O3 -std=c++17 -mavx2 -mfma -ffp-contract=off -pthread -Iinclude tools/rng_bench.cpp -o variants/rng_bench
#include "../kelpie_amd/csrc/kp_rng.cpp"

#include <chrono>
#include <random>

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int parts_main();
int main(int argc, char** argv) {
  if (argc > 2) return parts_main();
  const int n = 289, epochs = 65, ratio = 5, d = 200, D = 200;
  const uint32_t nent = 14541;
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937 g(7);
  std::vector<int32_t> rb(n), rp(n);
  int64_t rows = 0;
  for (int i = 0; i < n; ++i) {
    // degree-like: most calls ~60-150 rows, a tail to 400; the base post-training once per prediction
    const int r = 20 + (int)(std::exponential_distribution<double>(1.0 / 90.0)(g));
    rp[i] = std::min(r, 420);
    rb[i] = (i % 18 == 0) ? rp[i] + 1 : -1;
    rows += rp[i] + std::max(rb[i], 0);
  }
  std::vector<uint8_t> ts(24 + kN * 8 + 64, 0);
  {
    TorchMt mt;
    for (int i = 0; i < kN; ++i) mt.s[i] = g();
    mt.left = 1;
    mt.next = 0;
    mt.store(ts.data());
  }
  std::vector<uint32_t> key(kN);
  for (auto& k : key) k = g();
  int32_t pos = kN;
  size_t words = 0;
  for (int i = 0; i < n; ++i) words += (size_t)epochs * 3 * (rp[i] + std::max(rb[i], 0));
  std::vector<int32_t> out(words);
  std::vector<float> xb((size_t)n * d), xp((size_t)n * d);
  std::printf("calls %d rows %lld words out %zu torch words %.1f M\n", n, (long long)rows, words,
              (double)rows * epochs * 2 * ratio / 1e6);
  for (int rep = 0; rep < reps; ++rep) {
    // (1) the whole protocol, synchronous walk + wait
    double t0 = now_ms();
    int rc = kp_rng_transe_calls(ts.data(), ts.size(), key.data(), &pos, 1, D, d, 0.1f, n, rb.data(), rp.data(),
                                 nullptr, epochs, ratio, nent, xb.data(), xp.data(), out.data());
    double t1 = now_ms();
    rc |= kp_rng_wait();
    double t2 = now_ms();
    // (2) numpy shuffles alone, sequential
    NumpyMt np;
    std::vector<int32_t> idx;
    double t3 = now_ms();
    int32_t* o = out.data();
    for (int i = 0; i < n; ++i) {
      if (rb[i] >= 0) {
        te_draws(key.data(), &pos, rb[i], epochs, o, (size_t)3 * rb[i], np);
        o += (size_t)epochs * 3 * rb[i];
      }
      te_draws(key.data(), &pos, rp[i], epochs, o, (size_t)3 * rp[i], np);
      o += (size_t)epochs * 3 * rp[i];
    }
    double t4 = now_ms();
    o = out.data();
    for (int i = 0; i < n; ++i) {
      if (rb[i] >= 0) {
        te_perms(rb[i], epochs, o, (size_t)3 * rb[i], o, idx);
        o += (size_t)epochs * 3 * rb[i];
      }
      te_perms(rp[i], epochs, o, (size_t)3 * rp[i], o, idx);
      o += (size_t)epochs * 3 * rp[i];
    }
    double t4b = now_ms();
    for (int i = 0; i < n; ++i) {
      if (rb[i] >= 0) te_draws(key.data(), &pos, rb[i], epochs, nullptr, 0, np);
      te_draws(key.data(), &pos, rp[i], epochs, nullptr, 0, np);
    }
    std::printf("  draws without stores %.2f ms\n", now_ms() - t4b);
    t4b = now_ms();
    // (3) torch walk alone: skip past every slot's randints
    TorchMt mt;
    mt.load(ts.data());
    double t5 = now_ms();
    for (int i = 0; i < n; ++i) {
      mt.skip(D);
      for (int k = 0; k < 2; ++k) {
        int R = k ? rp[i] : rb[i];
        if (R >= 0) mt.skip((uint64_t)epochs * 2 * ratio * R);
      }
    }
    double t6 = now_ms();
    // (4) randint fills alone, one thread
    std::vector<uint32_t> draw;
    mt.load(ts.data());
    double t7 = now_ms();
    o = out.data();
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < 2; ++k) {
        int R = k ? rp[i] : rb[i];
        if (R < 0) continue;
        TorchMt m = mt;
        te_randints(m, R, epochs, ratio, nent, o, draw);
        o += (size_t)epochs * 3 * R;
      }
    double t8 = now_ms();
    std::printf("rc %d  whole: walk %.2f + wait %.2f = %.2f ms | numpy draws %.2f perms %.2f | torch walk %.2f | randint fills %.2f ms\n",
                rc, t1 - t0, t2 - t1, t2 - t0, t4 - t3, t4b - t4, t6 - t5, t8 - t7);
  }
  return 0;
}
// (appended) component timing of te_shuffles' parts on the same batch
int parts_main() {
  const int epochs = 65;
  std::mt19937 g(7);
  std::vector<uint32_t> key(kN);
  for (auto& k : key) k = g();
  NumpyMt np;
  int32_t pos = kN;
  np.load(key.data(), &pos);
  const size_t W = 2900000;
  double t0 = now_ms();
  std::vector<uint32_t> words(W);
  for (size_t k = 0; k < W; ++k) words[k] = np.next32();
  double t1 = now_ms();
  // draw loop over the pre-tempered words, R = 110 per shuffle
  std::vector<int32_t> jv(512), perm(512);
  size_t k = 0;
  long long draws = 0;
  const int R = 110;
  double t2 = now_ms();
  while (k + 1000 < W) {
    uint32_t ui = R - 1, mask = 0xFFFFFFFFu >> __builtin_clz(ui);
    for (; ui >= 1; ++k) {
      const uint32_t v = words[k] & mask;
      jv[ui] = (int32_t)v;
      const uint32_t m1 = (ui - 1 > (mask >> 1)) ? mask : (mask >> 1);
      const bool acc = v <= ui;
      mask = acc ? m1 : mask;
      ui -= acc;
    }
    draws += R - 1;
  }
  double t3 = now_ms();
  for (int i = 0; i < R; ++i) perm[i] = i;
  double t4 = now_ms();
  for (long long e = 0; e < draws / (R - 1); ++e)
    for (int t = R - 1; t >= 1; --t) std::swap(perm[t], perm[jv[t]]);
  double t5 = now_ms();
  std::printf("parts: twist+temper+next32 %zu words %.2f ms | draw loop %lld draws %.2f ms | swaps %.2f ms (%d)\n", W,
              t1 - t0, draws, t3 - t2, t5 - t4, perm[3]);
  (void)epochs;
  return 0;
}
