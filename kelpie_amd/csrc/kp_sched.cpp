// kp_sched.cpp -- host C++ for the per-call slot assembly of a post-training batch
// (SURVEY.md §8 a6/a7): the kelpie dataset edits and the rank filter lists that
// kelpie_amd/data.py:KelpieView computes per call in Python, for a whole batch of calls
// in one library call, and the batch's row / filter arrays packed straight into the
// buffers of kp_posttrain_rank.
//
// Reference semantics (src/data/kelpie_dataset.py):
//   rows: the kelpie entity's training triples (the original entity replaced by the kelpie
//     id, in the Python view's order) followed by their inverses (o, p + |R|, s)
//     (pairwise_ranking_optimizer.py:64-65);
//   remove_training_triples (:130-158): every removed triple must be a kelpie training
//     triple (KeyError otherwise), and the to_filter multiset of every key it touches must
//     still hold its entity (list.remove: ValueError); rows drop each removed triple once;
//   add_training_triples (:92-128): rows gain the added triples in order;
//   the rank filter of (kelpie, p) (kelpie_dataset.py:145-149 / 113-118): the multiset of
//     training + validation + test objects of that key after the edit, in first-insertion
//     order, the edit's new entities last (KelpieView.filter_for).
#include <cstdint>
#include <cstring>
#include <new>
#include <unordered_map>
#include <utility>
#include <vector>

#include "kelpie_hip.h"

namespace {

struct TripleKey {
  int32_t h, r, t;
  bool operator==(const TripleKey& o) const { return h == o.h && r == o.r && t == o.t; }
};
struct TripleHash {
  size_t operator()(const TripleKey& k) const {
    uint64_t x = (uint64_t)(uint32_t)k.h * 0x9E3779B97F4A7C15ull;
    x ^= (uint64_t)(uint32_t)k.r + 0x632BE59BD9B4E019ull + (x << 6) + (x >> 2);
    x ^= (uint64_t)(uint32_t)k.t * 0xC2B2AE3D27D4EB4Full + (x << 6) + (x >> 2);
    return (size_t)x;
  }
};

// insertion-ordered multiset of entities (a Python Counter)
struct OrderedCount {
  std::vector<std::pair<int32_t, int32_t>> items;  // (entity, count) in first-insertion order
  std::unordered_map<int32_t, int32_t> pos;
  void add(int32_t e, int32_t n) {
    auto it = pos.find(e);
    if (it == pos.end()) {
      pos.emplace(e, (int32_t)items.size());
      items.emplace_back(e, n);
    } else {
      items[it->second].second += n;
    }
  }
  int32_t get(int32_t e) const {
    auto it = pos.find(e);
    return it == pos.end() ? 0 : items[it->second].second;
  }
};

}  // namespace

struct kp_view {
  int32_t kelpie = 0, n_rel = 0, original = 0;
  std::vector<int32_t> base;  // [n][3]
  std::unordered_map<TripleKey, int32_t, TripleHash> index;
  std::unordered_map<int32_t, OrderedCount> filter;  // rank key (kelpie, p) -> objects
};

namespace {

// one edit's filter delta on one rank key: insertion-ordered (entity, +-count)
using Delta = OrderedCount;

void edit_delta(const kp_view& v, const std::vector<TripleKey>& conv, int sign, std::unordered_map<int32_t, Delta>& d) {
  for (const auto& t : conv) {
    if (t.h == v.kelpie) d[t.r].add(t.t, sign);
    if (t.t == v.kelpie) d[t.r + v.n_rel].add(t.h, sign);
  }
}

struct SlotRec {
  const kp_view* v = nullptr;
  int32_t rel = 0;       // rank key of the ranked triple (kelpie, rel, ·)
  int kind = 0;          // 0 base rows, 1 removal, 2 addition
  std::vector<int32_t> removed;       // removal: base indices, one per distinct triple
  std::vector<TripleKey> added;       // addition: converted triples, in order
  std::vector<int32_t> filt;          // the rank filter after the edit
};

void filter_after(const kp_view& v, int32_t rel, const std::unordered_map<int32_t, Delta>* delta,
                  std::vector<int32_t>& out) {
  out.clear();
  const auto bit = v.filter.find(rel);
  const Delta* dl = nullptr;
  if (delta) {
    auto it = delta->find(rel);
    if (it != delta->end() && !it->second.items.empty()) dl = &it->second;
  }
  if (bit != v.filter.end())
    for (const auto& [e, n] : bit->second.items)
      if (n + (dl ? dl->get(e) : 0) > 0) out.push_back(e);
  if (dl)
    for (const auto& [e, n] : dl->items)
      if ((bit == v.filter.end() || !bit->second.pos.count(e)) && n > 0) out.push_back(e);
}

}  // namespace

struct kp_sched_batch {
  std::vector<SlotRec> slots;
};

extern "C" {

int kp_view_create(int32_t kelpie, int32_t n_rel, int32_t original, const int32_t* base, int32_t n,
                   const int32_t* extra, int32_t m, kp_view** out) {
  if (!out || n < 0 || m < 0 || n_rel <= 0 || (n > 0 && !base) || (m > 0 && !extra)) return KP_EINVAL;
  *out = nullptr;
  try {
    auto* v = new kp_view();
    v->kelpie = kelpie;
    v->n_rel = n_rel;
    v->original = original;
    v->base.assign(base, base + 3 * (size_t)n);
    v->index.reserve((size_t)n * 2);
    for (int32_t i = 0; i < n; ++i) v->index[TripleKey{base[3 * i], base[3 * i + 1], base[3 * i + 2]}] = i;
    auto add = [&](const int32_t* t) {
      if (t[0] == kelpie) v->filter[t[1]].add(t[2], 1);
      if (t[2] == kelpie) v->filter[t[1] + n_rel].add(t[0], 1);
    };
    for (int32_t i = 0; i < n; ++i) add(base + 3 * i);
    for (int32_t i = 0; i < m; ++i) add(extra + 3 * i);
    *out = v;
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

void kp_view_destroy(kp_view* v) { delete v; }

int kp_sched_batch_create(kp_sched_batch** out) {
  if (!out) return KP_EINVAL;
  *out = new (std::nothrow) kp_sched_batch();
  return *out ? KP_OK : KP_ENOMEM;
}

void kp_sched_batch_destroy(kp_sched_batch* b) { delete b; }

int kp_sched_add_calls(kp_sched_batch* b, int32_t n, kp_view* const* views, const int32_t* rel, const uint8_t* flags,
                       const int32_t* cand_off, const int32_t* cands, int32_t* slot_idx, int32_t* n_rows,
                       int32_t* n_filt, int32_t* fail) {
  if (!b || n < 0 || (n > 0 && (!views || !rel || !flags || !cand_off || !slot_idx || !n_rows || !n_filt)) ||
      !fail)
    return KP_EINVAL;
  fail[0] = -1;
  fail[1] = 0;
  fail[2] = -1;
  try {
    std::vector<TripleKey> conv;
    std::unordered_map<int32_t, Delta> delta;
    for (int32_t c = 0; c < n; ++c) {
      const kp_view* v = views[c];
      if (!v) return KP_EINVAL;
      const uint8_t f = flags[c];
      const bool need_base = f & 1, own_base = f & 2, own_pt = f & 4, sufficient = f & 8;
      slot_idx[2 * c] = slot_idx[2 * c + 1] = -1;
      n_rows[2 * c] = n_rows[2 * c + 1] = 0;
      n_filt[2 * c] = n_filt[2 * c + 1] = 0;
      const int32_t nb = (int32_t)(v->base.size() / 3);
      if (need_base) {
        n_rows[2 * c] = 2 * nb;
        if (own_base) {
          SlotRec s;
          s.v = v;
          s.rel = rel[c];
          s.kind = 0;
          filter_after(*v, s.rel, nullptr, s.filt);
          n_filt[2 * c] = (int32_t)s.filt.size();
          slot_idx[2 * c] = (int32_t)b->slots.size();
          b->slots.push_back(std::move(s));
        }
      }
      // the edit (KelpieView.removed / added): checks in the reference's order
      const int32_t k0 = cand_off[c], k1 = cand_off[c + 1];
      conv.clear();
      for (int32_t k = k0; k < k1; ++k) {
        const int32_t* t = cands + 3 * (size_t)k;
        if (t[0] != v->original && t[2] != v->original) {  // the assert in removed / added
          fail[0] = c;
          fail[1] = 1;
          fail[2] = k - k0;
          return KP_OK;
        }
        conv.push_back(TripleKey{t[0] == v->original ? v->kelpie : t[0], t[1], t[2] == v->original ? v->kelpie : t[2]});
      }
      SlotRec s;
      s.v = v;
      s.rel = rel[c];
      delta.clear();
      if (!sufficient) {
        std::vector<int32_t> idx;
        for (size_t k = 0; k < conv.size(); ++k) {
          auto it = v->index.find(conv[k]);
          if (it == v->index.end()) {  // KeyError
            fail[0] = c;
            fail[1] = 2;
            fail[2] = (int32_t)k;
            return KP_OK;
          }
          idx.push_back(it->second);
        }
        edit_delta(*v, conv, -1, delta);
        for (const auto& [r, cnt] : delta) {
          auto fit = v->filter.find(r);
          for (const auto& [e, m] : cnt.items)
            if ((fit == v->filter.end() ? 0 : fit->second.get(e)) + m < 0) {  // list.remove: ValueError
              fail[0] = c;
              fail[1] = 3;
              fail[2] = -1;
              return KP_OK;
            }
        }
        std::vector<char> gone((size_t)nb, 0);
        for (int32_t i : idx)
          if (!gone[i]) {
            gone[i] = 1;
            s.removed.push_back(i);
          }
        s.kind = 1;
        n_rows[2 * c + 1] = 2 * (nb - (int32_t)s.removed.size());
      } else {
        edit_delta(*v, conv, +1, delta);
        s.kind = 2;
        s.added = conv;
        n_rows[2 * c + 1] = 2 * (nb + (int32_t)conv.size());
      }
      if (own_pt) {
        filter_after(*v, s.rel, &delta, s.filt);
        n_filt[2 * c + 1] = (int32_t)s.filt.size();
        slot_idx[2 * c + 1] = (int32_t)b->slots.size();
        b->slots.push_back(std::move(s));
      }
    }
  } catch (...) {
    return KP_ENOMEM;
  }
  return KP_OK;
}

int kp_sched_pack(const kp_sched_batch* b, int32_t n, const int32_t* idx, int32_t* rows, int64_t rows_cap,
                  int32_t* filt, int64_t filt_cap) {
  if (!b || n < 0 || (n > 0 && !idx) || rows_cap < 0 || filt_cap < 0) return KP_EINVAL;
  int64_t ro = 0, fo = 0;
  std::vector<char> gone;
  for (int32_t j = 0; j < n; ++j) {
    if (idx[j] < 0 || idx[j] >= (int32_t)b->slots.size()) return KP_EINVAL;
    const SlotRec& s = b->slots[idx[j]];
    const kp_view& v = *s.v;
    const int32_t nb = (int32_t)(v.base.size() / 3);
    const int32_t nr = s.kind == 0 ? nb : s.kind == 1 ? nb - (int32_t)s.removed.size() : nb + (int32_t)s.added.size();
    if (ro + 6 * (int64_t)nr > rows_cap || fo + (int64_t)s.filt.size() > filt_cap) return KP_EINVAL;
    int32_t* fwd = rows + ro;
    int32_t* inv = rows + ro + 3 * (int64_t)nr;
    int32_t w = 0;
    auto put = [&](int32_t h, int32_t r, int32_t t) {
      fwd[3 * w] = h;
      fwd[3 * w + 1] = r;
      fwd[3 * w + 2] = t;
      inv[3 * w] = t;
      inv[3 * w + 1] = r + v.n_rel;
      inv[3 * w + 2] = h;
      ++w;
    };
    if (s.kind == 1) {
      gone.assign((size_t)nb, 0);
      for (int32_t i : s.removed) gone[i] = 1;
    }
    for (int32_t i = 0; i < nb; ++i)
      if (s.kind != 1 || !gone[i]) put(v.base[3 * i], v.base[3 * i + 1], v.base[3 * i + 2]);
    if (s.kind == 2)
      for (const auto& t : s.added) put(t.h, t.r, t.t);
    ro += 6 * (int64_t)nr;
    if (!s.filt.empty()) std::memcpy(filt + fo, s.filt.data(), sizeof(int32_t) * s.filt.size());
    fo += (int64_t)s.filt.size();
  }
  return KP_OK;
}

int kp_gather_i32(int32_t n, const uint64_t* ptrs, const int64_t* counts, int32_t* out, int64_t cap) {
  if (n < 0 || (n > 0 && (!ptrs || !counts)) || cap < 0) return KP_EINVAL;
  int64_t o = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (counts[i] < 0 || o + counts[i] > cap || (counts[i] > 0 && !ptrs[i])) return KP_EINVAL;
    if (counts[i]) std::memcpy(out + o, reinterpret_cast<const int32_t*>(ptrs[i]), sizeof(int32_t) * counts[i]);
    o += counts[i];
  }
  return KP_OK;
}

}  // extern "C"
