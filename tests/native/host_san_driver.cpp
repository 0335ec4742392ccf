// Host-side sanitizer driver for the library's host C++ (kp_rng.cpp: the RNG
// protocol with its worker threads and per-batch arenas; kp_graph.cpp: the prefilter
// graphs).  `make asan` / `make tsan` link this driver with those two sources under
// -fsanitize=address,undefined or -fsanitize=thread (tests/test_host_sanitizers.py
// runs them in the CPU suite).  The driver replays a fixed sequence of calls on
// inputs the test writes (a torch generator state, a numpy MT19937 state, a graph)
// and writes every output back to back, so the test also checks that the
// sanitized build computes exactly what the production library computes.
//
//   host_san_driver <in_dir> <out_file>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kelpie_hip.h"

namespace {

std::vector<uint8_t> slurp(const char* dir, const char* name) {
  char path[4096];
  std::snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path);
    std::exit(2);
  }
  std::vector<uint8_t> v;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

FILE* g_out = nullptr;
void put(const void* p, size_t n) {
  if (n && std::fwrite(p, 1, n, g_out) != n) {
    std::fprintf(stderr, "short write\n");
    std::exit(2);
  }
}
template <class T>
void put(const std::vector<T>& v) {
  put(v.data(), v.size() * sizeof(T));
}

void ok(int rc, const char* what) {
  if (rc != 0) {
    std::fprintf(stderr, "%s failed: %d\n", what, rc);
    std::exit(3);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s <in_dir> <out_file>\n", argv[0]);
    return 2;
  }
  std::vector<uint8_t> ts = slurp(argv[1], "torch_state.bin");
  std::vector<uint8_t> nps = slurp(argv[1], "np_state.bin");  // key[624] uint32, pos int32
  std::vector<uint8_t> tri = slurp(argv[1], "triples.bin");   // int32 [n][3]
  std::vector<uint8_t> cls = slurp(argv[1], "classes.bin");   // int64 off[n_ent + 1], int32 cls[]
  if (nps.size() != 625 * 4) return 2;
  std::vector<uint32_t> key(624);
  std::memcpy(key.data(), nps.data(), 624 * 4);
  int32_t pos;
  std::memcpy(&pos, nps.data() + 624 * 4, 4);
  g_out = std::fopen(argv[2], "wb");
  if (!g_out) return 2;

  // 1. discard, normal, bernoulli
  ok(kp_mt19937_discard(ts.data(), ts.size(), 12345), "discard");
  put(ts);
  std::vector<float> nrm(200);
  ok(kp_rng_normal(ts.data(), ts.size(), 200, 0.f, 0.1f, 1, nrm.data()), "normal");
  put(nrm);
  std::vector<uint32_t> bits((1000 + 31) / 32);
  ok(kp_rng_bernoulli_bits(ts.data(), ts.size(), 1000, 0.8, bits.data()), "bernoulli");
  put(bits);
  // 2. one TransE post-training's draws, synchronous
  std::vector<int32_t> te(5 * 3 * 37);
  ok(kp_rng_transe_epochs(ts.data(), ts.size(), key.data(), &pos, 37, 5, 5, 14542, te.data()), "transe_epochs");
  put(te);
  // 3. deferred: many slots on the worker threads, ConvE masks interleaved, one arena
  const int n_slots = 48;
  std::vector<size_t> off(n_slots + 1, 0);
  std::vector<int32_t> mask_rows = {7, 7, 3, 12};
  const int32_t seg_elems = 200;  // one dropout of 200 units per pair, keep 0.8
  const double seg_keep = 0.8;
  size_t mask_words = 0;
  for (int r : mask_rows) mask_words += ((size_t)r * 200 + 31) / 32;
  for (int i = 0; i < n_slots; ++i) off[i + 1] = off[i] + (size_t)3 * 3 * (10 + i) + (i % 4 == 3 ? mask_words : 0);
  std::vector<int32_t> arena(off[n_slots]);
  for (int i = 0; i < n_slots; ++i) {
    ok(kp_rng_transe_enqueue(ts.data(), ts.size(), key.data(), &pos, 10 + i, 3, 5, 14542, arena.data() + off[i]),
       "transe_enqueue");
    if (i % 4 == 3)
      ok(kp_rng_conve_masks_enqueue(ts.data(), ts.size(), (int)mask_rows.size(), mask_rows.data(), 1, &seg_elems, &seg_keep,
                                    reinterpret_cast<uint32_t*>(arena.data() + off[i] + (size_t)3 * 3 * (10 + i))),
         "conve_masks_enqueue");
  }
  ok(kp_rng_wait(), "wait");
  put(arena);
  put(ts);
  put(key);
  put(&pos, 4);
  // 4. fused TransE calls (deferred epoch draws), then a synchronous ConvE mask draw
  const int n_calls = 6;
  std::vector<int32_t> rb = {12, -1, -1, 30, -1, -1}, rp = {11, 40, 9, -1, 25, 17};
  size_t tot = 0;
  for (int i = 0; i < n_calls; ++i) tot += (size_t)4 * 3 * ((rb[i] > 0 ? rb[i] : 0) + (rp[i] > 0 ? rp[i] : 0));
  std::vector<int32_t> calls(tot + 1);
  std::vector<float> xb((size_t)n_calls * 32), xp((size_t)n_calls * 32);
  ok(kp_rng_transe_calls(ts.data(), ts.size(), key.data(), &pos, 1, 32, 32, 0.2425f, n_calls, rb.data(), rp.data(),
                         nullptr, 4, 5, 14542, xb.data(), xp.data(), calls.data()),
     "transe_calls");
  ok(kp_rng_wait(), "wait");
  calls.resize(tot);
  put(calls);
  put(xb);
  put(xp);
  // the same shape with some post-trainings unwanted (another rank's): advance only
  std::vector<uint8_t> want = {1, 2, 0, 3, 0, 2};
  size_t tot2 = 0;
  for (int i = 0; i < n_calls; ++i)
    tot2 += (size_t)4 * 3 * ((want[i] & 1 && rb[i] > 0 ? rb[i] : 0) + (want[i] & 2 && rp[i] > 0 ? rp[i] : 0));
  std::vector<int32_t> calls2(tot2 + 1);
  ok(kp_rng_transe_calls(ts.data(), ts.size(), key.data(), &pos, 1, 32, 32, 0.2425f, n_calls, rb.data(), rp.data(),
                         want.data(), 4, 5, 14542, xb.data(), xp.data(), calls2.data()),
     "transe_calls(want)");
  ok(kp_rng_wait(), "wait");
  calls2.resize(tot2);
  put(calls2);
  put(xb);
  put(xp);
  std::vector<uint32_t> masks(mask_words);
  ok(kp_rng_conve_masks(ts.data(), ts.size(), (int)mask_rows.size(), mask_rows.data(), 1, &seg_elems, &seg_keep, masks.data()),
     "conve_masks");
  put(masks);
  put(ts);
  put(key);
  put(&pos, 4);

  // 5. prefilter graph: BFS and Jaccard-weighted Dijkstra
  const int64_t n_tri = (int64_t)(tri.size() / 12);
  std::vector<int32_t> t3(n_tri * 3);
  std::memcpy(t3.data(), tri.data(), tri.size());
  int32_t n_ent = 0;  // entities are columns 0 and 2 (column 1 holds relation ids)
  for (int64_t i = 0; i < n_tri; ++i) {
    n_ent = t3[3 * i] + 1 > n_ent ? t3[3 * i] + 1 : n_ent;
    n_ent = t3[3 * i + 2] + 1 > n_ent ? t3[3 * i + 2] + 1 : n_ent;
  }
  kp_graph* g = nullptr;
  ok(kp_graph_create(n_ent, n_tri, t3.data(), &g), "graph_create");
  std::vector<int32_t> src = {0, 1, 2, 3, 5, 8, 13, 21};
  std::vector<int32_t> dist(src.size() * (size_t)n_ent);
  ok(kp_graph_bfs(g, (int32_t)src.size(), src.data(), dist.data()), "bfs");
  put(dist);
  std::vector<int64_t> coff((size_t)n_ent + 1);
  std::memcpy(coff.data(), cls.data(), 8 * ((size_t)n_ent + 1));
  std::vector<int32_t> cl((cls.size() - 8 * ((size_t)n_ent + 1)) / 4);
  std::memcpy(cl.data(), cls.data() + 8 * ((size_t)n_ent + 1), 4 * cl.size());
  if (cl.empty()) cl.push_back(0);
  ok(kp_graph_set_classes(g, coff.data(), cl.data()), "set_classes");
  std::vector<int32_t> ds, dd;
  for (int i = 0; i < 64; ++i) {
    ds.push_back((i * 37) % n_ent);
    dd.push_back((i * 101 + 7) % n_ent);
  }
  std::vector<double> w(ds.size());
  ok(kp_graph_dijkstra_pairs(g, (int32_t)ds.size(), ds.data(), dd.data(), w.data()), "dijkstra");
  put(w);
  kp_graph_destroy(g);

  // 6. the asynchronous torch walk (kp_rng_transe_calls_async, two chained calls, then
  //    kp_rng_wait + kp_rng_torch_take) against the synchronous call on copies of the same
  //    generator states: identical draws, rows and end states (checked here, nothing written)
  {
    std::vector<uint8_t> tsA = ts, tsB = ts, dummy(ts.size(), 0);
    std::vector<uint32_t> keyA = key, keyB = key;
    int32_t posA = pos, posB = pos;
    std::vector<int32_t> oA(tot + 1), oB(tot + 1);
    std::vector<float> xbA(xb.size()), xpA(xp.size()), xbB(xb.size()), xpB(xp.size());
    ok(kp_rng_transe_calls(tsA.data(), tsA.size(), keyA.data(), &posA, 1, 32, 32, 0.2425f, n_calls, rb.data(),
                           rp.data(), nullptr, 4, 5, 14542, xbA.data(), xpA.data(), oA.data()),
       "transe_calls (sync reference)");
    ok(kp_rng_wait(), "wait");
    const int h = n_calls / 2;
    size_t off1 = 0;
    for (int i = 0; i < h; ++i) off1 += (size_t)4 * 3 * ((rb[i] > 0 ? rb[i] : 0) + (rp[i] > 0 ? rp[i] : 0));
    ok(kp_rng_transe_calls_async(tsB.data(), tsB.size(), keyB.data(), &posB, 1, 32, 32, 0.2425f, h, rb.data(),
                                 rp.data(), nullptr, 4, 5, 14542, xbB.data(), xpB.data(), oB.data()),
       "transe_calls_async 1");
    ok(kp_rng_transe_calls_async(dummy.data(), dummy.size(), keyB.data(), &posB, 1, 32, 32, 0.2425f, n_calls - h,
                                 rb.data() + h, rp.data() + h, nullptr, 4, 5, 14542, xbB.data() + (size_t)h * 32,
                                 xpB.data() + (size_t)h * 32, oB.data() + off1),
       "transe_calls_async 2");
    ok(kp_rng_wait(), "wait");
    int32_t taken = 0;
    ok(kp_rng_torch_take(tsB.data(), tsB.size(), &taken), "torch_take");
    if (!taken || tsA != tsB || keyA != keyB || posA != posB || oA != oB || xbA != xbB || xpA != xpB) {
      std::fprintf(stderr, "asynchronous walk differs from the synchronous one\n");
      return 1;
    }
  }
  std::fclose(g_out);
  return 0;
}
