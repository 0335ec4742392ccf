// kp_graph.cpp -- host C++ for the candidate prefilters upstream of the relevance
// engine:
//   TopologyPreFilter          src/prefilters/topology_prefilter.py:9-37
//   WeightedTopologyPreFilter  src/prefilters/weighted_topology_prefilter.py:13-56
// The reference builds a networkx MultiGraph with one undirected edge per
// training triple and, per candidate triple, asks networkx for the shortest-path
// length from the candidate's other endpoint to the prediction's object.
//
// Topology: hop distances are symmetric integers, so ONE breadth-first search
// from the object answers every candidate of a prediction (the reference runs
// one search per candidate).  Sources are processed in parallel threads.
//
// Weighted: edge cost 1 - Jaccard(classes(u), classes(v)) (utils/utils.py:11-14)
// in float64.  Float sums depend on the path order, so each (source, target)
// query replays networkx's _dijkstra_multisource exactly: neighbours in the
// MultiGraph's insertion order, a heap ordered by (distance, push counter),
// first pop finalises, stop at the target.  Distances therefore match the
// reference bit for bit, ties included.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <queue>
#include <thread>
#include <unordered_set>
#include <vector>

#include "kelpie_hip.h"

struct kp_graph {
  int32_t n = 0;
  std::vector<int64_t> off;   // CSR over neighbours, networkx insertion order
  std::vector<int32_t> adj;
  std::vector<double> cost;   // per CSR slot, set by kp_graph_set_classes
  bool weighted = false;
};

namespace {

thread_local char g_err[256] = "";

int fail(int code, const char* msg) {
  std::snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int n_workers(int64_t jobs) {
  unsigned hw = std::thread::hardware_concurrency();
  if (hw == 0) hw = 4;
  return (int)std::max<int64_t>(1, std::min<int64_t>({jobs, (int64_t)hw, 16}));
}

template <class F>
void parallel_for(int64_t n, F&& f) {
  const int T = n_workers(n);
  if (T <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int w = 0; w < T; ++w)
    th.emplace_back([&, w] {
      for (int64_t i = w; i < n; i += T) f(i);
    });
  for (auto& t : th) t.join();
}

}  // namespace

extern "C" {

const char* kp_graph_last_error(void) { return g_err; }

int kp_graph_create(int32_t n_ent, int64_t n_triples, const int32_t* triples, kp_graph** out) {
  if (!out || n_ent <= 0 || n_triples < 0 || (n_triples > 0 && !triples))
    return fail(KP_EINVAL, "kp_graph_create: bad arguments");
  *out = nullptr;
  try {
    // neighbour lists in first-edge order (MultiGraph.add_edges_from: _adj[u][v] is
    // created by the first (u, v) edge; a self loop appears once)
    std::vector<std::vector<int32_t>> nb(n_ent);
    std::vector<std::unordered_set<int32_t>> seen(n_ent);
    for (int64_t i = 0; i < n_triples; ++i) {
      const int32_t h = triples[3 * i], t = triples[3 * i + 2];
      if (h < 0 || h >= n_ent || t < 0 || t >= n_ent) return fail(KP_EINVAL, "kp_graph_create: entity id out of range");
      if (seen[h].insert(t).second) nb[h].push_back(t);
      if (h != t && seen[t].insert(h).second) nb[t].push_back(h);
    }
    kp_graph* g = new kp_graph();
    g->n = n_ent;
    g->off.assign((size_t)n_ent + 1, 0);
    for (int32_t v = 0; v < n_ent; ++v) g->off[v + 1] = g->off[v] + (int64_t)nb[v].size();
    g->adj.resize((size_t)g->off[n_ent]);
    for (int32_t v = 0; v < n_ent; ++v) std::copy(nb[v].begin(), nb[v].end(), g->adj.begin() + g->off[v]);
    *out = g;
    return KP_OK;
  } catch (const std::bad_alloc&) {
    return fail(KP_ENOMEM, "kp_graph_create: out of memory");
  }
}

void kp_graph_destroy(kp_graph* g) { delete g; }

int kp_graph_bfs(const kp_graph* g, int32_t n_src, const int32_t* src, int32_t* dist) {
  if (!g || n_src < 0 || (n_src > 0 && (!src || !dist))) return fail(KP_EINVAL, "kp_graph_bfs: bad arguments");
  for (int32_t i = 0; i < n_src; ++i)
    if (src[i] < 0 || src[i] >= g->n) return fail(KP_EINVAL, "kp_graph_bfs: source out of range");
  const int32_t n = g->n;
  parallel_for(n_src, [&](int64_t i) {
    int32_t* d = dist + (size_t)i * n;
    std::fill(d, d + n, -1);
    std::vector<int32_t> frontier{src[i]}, next;
    d[src[i]] = 0;
    int32_t level = 0;
    while (!frontier.empty()) {
      ++level;
      next.clear();
      for (int32_t u : frontier)
        for (int64_t k = g->off[u]; k < g->off[u + 1]; ++k) {
          const int32_t w = g->adj[k];
          if (d[w] < 0) {
            d[w] = level;
            next.push_back(w);
          }
        }
      frontier.swap(next);
    }
  });
  return KP_OK;
}

int kp_graph_set_classes(kp_graph* g, const int64_t* cls_off, const int32_t* cls) {
  if (!g || !cls_off || (cls_off[g->n] > 0 && !cls)) return fail(KP_EINVAL, "kp_graph_set_classes: bad arguments");
  const int32_t n = g->n;
  // per entity: sorted unique class ids
  std::vector<std::vector<int32_t>> sets(n);
  for (int32_t v = 0; v < n; ++v) {
    sets[v].assign(cls + cls_off[v], cls + cls_off[v + 1]);
    std::sort(sets[v].begin(), sets[v].end());
    sets[v].erase(std::unique(sets[v].begin(), sets[v].end()), sets[v].end());
  }
  g->cost.assign(g->adj.size(), 0.0);
  parallel_for(n, [&](int64_t v) {
    const auto& a = sets[v];
    for (int64_t k = g->off[v]; k < g->off[v + 1]; ++k) {
      const auto& b = sets[g->adj[k]];
      double jac = 0.0;  // jaccard_similarity: 0 when either set is empty
      if (!a.empty() && !b.empty()) {
        size_t i = 0, j = 0, inter = 0;
        while (i < a.size() && j < b.size()) {
          if (a[i] < b[j]) ++i;
          else if (b[j] < a[i]) ++j;
          else { ++inter; ++i; ++j; }
        }
        const size_t uni = a.size() + b.size() - inter;
        jac = (double)inter / (double)uni;  // python int / int -> float64
      }
      g->cost[k] = 1.0 - jac;
    }
  });
  g->weighted = true;
  return KP_OK;
}

int kp_graph_dijkstra_pairs(const kp_graph* g, int32_t n, const int32_t* src, const int32_t* dst, double* out) {
  if (!g || n < 0 || (n > 0 && (!src || !dst || !out))) return fail(KP_EINVAL, "kp_graph_dijkstra_pairs: bad arguments");
  if (!g->weighted) return fail(KP_EINVAL, "kp_graph_dijkstra_pairs: call kp_graph_set_classes first");
  for (int32_t i = 0; i < n; ++i)
    if (src[i] < 0 || src[i] >= g->n || dst[i] < 0 || dst[i] >= g->n)
      return fail(KP_EINVAL, "kp_graph_dijkstra_pairs: node out of range");
  struct Item {
    double d;
    uint64_t c;
    int32_t v;
    bool operator>(const Item& o) const { return d > o.d || (d == o.d && c > o.c); }
  };
  parallel_for(n, [&](int64_t q) {
    const int32_t s = src[q], t = dst[q];
    std::vector<double> dist(g->n, -1.0), seen(g->n, -1.0);  // -1: absent (costs are >= 0)
    std::priority_queue<Item, std::vector<Item>, std::greater<Item>> fringe;
    uint64_t counter = 0;
    seen[s] = 0.0;
    fringe.push({0.0, counter++, s});
    double res = INFINITY;
    while (!fringe.empty()) {
      const Item it = fringe.top();
      fringe.pop();
      if (dist[it.v] >= 0.0) continue;
      dist[it.v] = it.d;
      if (it.v == t) {
        res = it.d;
        break;
      }
      for (int64_t k = g->off[it.v]; k < g->off[it.v + 1]; ++k) {
        const int32_t u = g->adj[k];
        const double vu = dist[it.v] + g->cost[k];
        if (dist[u] >= 0.0) continue;
        if (seen[u] < 0.0 || vu < seen[u]) {
          seen[u] = vu;
          fringe.push({vu, counter++, u});
        }
      }
    }
    out[q] = res;
  });
  return KP_OK;
}

}  // extern "C"
