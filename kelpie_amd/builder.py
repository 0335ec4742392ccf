"""Stochastic explanation builder driving the batched engine.

Same algorithm, output and RNG use as the reference
``src/explanation_builders/stochastic_builder.py:13-192`` (without
summarisation), restructured for a batched engine:

* all singleton rules of a prediction are evaluated in ONE engine batch
  (the reference's hot loop A, ``:110-124``);
* compound rules are evaluated in speculative windows of rules in prescore
  order (hot loop B, ``:126-175``).  The accept / early-return /
  ``random.random()`` termination logic is then replayed sequentially over the
  window's relevances; if the search stops inside the window, the torch /
  numpy generators are rewound to the state right after the last rule the
  reference would have evaluated, so every later draw is unchanged.

With ``pipelined`` the next window is scheduled while the current one runs on the device
(its draws follow the current window's, on this thread; its slots are packed on its batch
thread), but it is held: its device work starts only once the replay of the current
window has gone through without a stop (``engine.submit_batch(hold=True)``,
``release_batch``).  A stop inside the current window cancels it with no device work and
rewinds the generators past both, so only host work is ever thrown away.  Off by default:
the look-ahead's size is chosen before the current window's relevances are known, so its
windows run past more stops (273 against 245 evaluations for the same 224 relevances), and
that costs more device time than overlapping the host schedule saves (the schedule is 11 %
of the builder's time, the library call 85 %): headline builder leg, alternating on one
box, 439.8 / 456.9 relevances/s held look-ahead against 485.1 / 480.8 sequential
(profiles/r06/r06y/r06y7_*).  A first form started the look-ahead at once on the second
context: 392.5 / 394.7 against 452.3 / 453.1 (profiles/r06/r06i/).

Window sizes: a fixed ``window``, or ``window="auto"``: the rules before index 10
of a length (the sliding window's size: no stochastic stop can happen there, only
the early exit on ``xsi``) go as one window, and after that each window holds about
as many rules as the search is expected to run before it stops, from the stop
probability the replay has reached (1 - average / best of the sliding window),
between ``AUTO_MIN`` and ``AUTO_MAX`` rules.  Either way the results, the draws and
``#relevances`` are those of the sequential reference; only the device work spent
past a stop (``stats["wasted"]``) and the number of engine batches change.
"""
from __future__ import annotations

import itertools
import random
import time


class StochasticBuilder:
    AUTO_MIN, AUTO_MAX = 4, 32

    def __init__(self, xsi, engine, summarization: str = None, max_explanation_length: int = 4, window=32,
                 pipelined=False):
        if summarization is not None:
            raise NotImplementedError("summarisation (simulation / bisimulation) is out of scope")
        self.xsi = xsi
        self.engine = engine
        self.dataset = engine.dataset
        self.length_cap = max_explanation_length
        self.window_size = 10  # the reference's sliding window (stochastic_builder.py:24)
        self.auto = window == "auto"
        self.pipelined = bool(pipelined) and hasattr(engine, "submit_batch")
        self.spec_window = self.AUTO_MAX if self.auto else max(1, int(window))
        self.summarization = None
        self.stats = {"batches": 0, "evaluated": 0, "wasted": 0, "batch_s": 0.0, "schedule_s": 0.0, "pack_s": 0.0,
                      "lib_s": 0.0}

    def _account(self, t0):
        """Wall time of one engine batch and the engine's host / library split of it."""
        self.stats["batch_s"] += time.perf_counter() - t0
        bs = getattr(self.engine, "last_batch_stats", None)
        if isinstance(bs, dict):
            for k in ("schedule_s", "pack_s", "lib_s"):
                self.stats[k] += float(bs.get(k, 0.0) or 0.0)

    def build_explanations(self, pred, candidate_triples: list, k: int = 10):
        start = time.time()
        candidate_triples = [tuple(int(v) for v in t) for t in candidate_triples]
        triple_to_rel = self.explore_singleton_rules(pred, candidate_triples)
        srt = sorted(triple_to_rel.items(), key=lambda x: x[1], reverse=True)
        rule_to_rel = [((t,), rel) for (t, rel) in srt]
        triples_number = len(triple_to_rel)
        rels_num = triples_number
        _, best = rule_to_rel[0]
        if not best > self.xsi:
            for rule_length in range(2, min(triples_number, self.length_cap) + 1):
                cur, cur_n = self.explore_compound_rules(pred, candidate_triples, rule_length, triple_to_rel)
                rels_num += cur_n
                cur = sorted(cur.items(), key=lambda x: x[1], reverse=True)
                rule_to_rel += cur
                _, current_best = cur[0]
                if current_best > best:
                    best = current_best
                if best > self.xsi:
                    break
        rule_to_rel = sorted(rule_to_rel, key=lambda x: (x[1], 1 / len(x[0])), reverse=True)[:k]
        mapped = [(self.dataset.labels_triples(rule), rel) for rule, rel in rule_to_rel]
        return {"triple": self.dataset.labels_triple(tuple(pred)), "rule_to_relevance": mapped,
                "#relevances": rels_num, "execution_time": time.time() - start}

    def explore_singleton_rules(self, pred, triples: list):
        # one engine batch for every singleton; a duplicated candidate is evaluated
        # once per occurrence and the last value wins, like the dict of :113-123
        t0 = time.perf_counter()
        rels = self.engine.compute_relevance_batch(pred, [[t] for t in triples])
        self._account(t0)
        self.stats["batches"] += 1
        self.stats["evaluated"] += len(triples)
        out = {}
        for t, r in zip(triples, rels):
            out[t] = r
        return out

    def explore_compound_rules(self, pred, triples, length, triple_to_relevance):
        rules = itertools.combinations(triples, length)
        rules = [(r, sum(triple_to_relevance[t] for t in r)) for r in rules]
        rules = sorted(rules, key=lambda x: x[1], reverse=True)
        terminate = False
        best = -1e6
        window = [None] * self.window_size
        rule_to_relevance = {}
        computed = 0
        i = 0
        eng = self.engine
        ahead = None  # the next window, scheduled and started speculatively: (rules, checkpoints, batch)

        def submit(at, hold=False):
            chunk = [r for r, _ in rules[at:at + self._window(at, window, best)]]
            cps = []
            if self.pipelined:
                return chunk, cps, eng.submit_batch(pred, [list(r) for r in chunk], checkpoints=cps, hold=hold)
            return chunk, cps, None

        prev_cps = None
        while i < len(rules) and not terminate:
            if ahead is not None:
                chunk, cps, batch = ahead
                ahead = None
                if len(chunk) > self._window(i, window, best):
                    # sized before the previous window's relevances were known and larger than
                    # the window the sequential search now takes here: cancel it (no device
                    # work), rewind to its start and schedule the sequential one
                    eng.finish_batch(batch, discard=True)
                    self.stats["lookahead_resized"] = self.stats.get("lookahead_resized", 0) + 1
                    prev_cps[-1].restore()
                    chunk, cps, batch = submit(i)
                else:
                    eng.release_batch(batch)  # the previous window ran through: start its device work
            else:
                chunk, cps, batch = submit(i)
            prev_cps = cps
            if self.pipelined:
                t0 = time.perf_counter()
                if i + len(chunk) < len(rules):
                    # scheduled and packed while `batch` runs on the device, held until the
                    # replay below has gone through `batch` without a stop
                    ahead = submit(i + len(chunk), hold=True)
                try:
                    rels = eng.finish_batch(batch)
                except BaseException:
                    if ahead is not None:
                        eng.finish_batch(ahead[2], discard=True)  # cancelled: no device work
                    raise
                self._account(t0)
            else:
                t0 = time.perf_counter()
                rels = eng.compute_relevance_batch(pred, [list(r) for r in chunk], checkpoints=cps)
                self._account(t0)
            self.stats["batches"] += 1
            self.stats["evaluated"] += len(chunk)
            stop_at = None
            for j, rel in enumerate(rels):
                ii = i + j
                rule = chunk[j]
                rule_to_relevance[rule] = rel
                computed += 1
                window[ii % self.window_size] = rel
                if rel > self.xsi:
                    stop_at, terminate = j, True
                    break
                elif rel >= best:
                    best = rel
                elif ii >= self.window_size:
                    avg = sum(window) / self.window_size
                    thr = avg / best
                    if random.random() > thr:
                        stop_at, terminate = j, True
                        break
            if stop_at is not None:
                if ahead is not None:
                    # the held next window: cancelled before any device work (its host
                    # schedule is all that is lost); rewind past it and this window's later rules
                    eng.finish_batch(ahead[2], discard=True)
                    self.stats["lookahead_cancelled"] = self.stats.get("lookahead_cancelled", 0) + 1
                    ahead = None
                    cps[stop_at].restore()
                elif stop_at + 1 < len(chunk):
                    cps[stop_at].restore()  # rewind the speculative draws
                self.stats["wasted"] += len(chunk) - stop_at - 1
            i += len(chunk)
        return rule_to_relevance, computed

    def _window(self, i, window, best):
        """Rules in the next speculative window (see the module docstring)."""
        if not self.auto:
            return self.spec_window
        if i < self.window_size:
            return self.window_size - i
        if any(v is None for v in window) or best == 0:
            # a window scheduled before the replay has filled the sliding window (the
            # pipelined builder's look-ahead), or a best of zero: no estimate
            return 2 * self.AUTO_MIN
        if best == 0:
            return self.AUTO_MIN
        thr = (sum(window) / self.window_size) / best
        p_stop = min(1.0, max(0.0, 1.0 - thr))  # P(random.random() > thr) per rule below the best
        if p_stop <= 1.0 / self.AUTO_MAX:
            return self.AUTO_MAX
        return int(min(self.AUTO_MAX, max(self.AUTO_MIN, round(1.0 / p_stop))))
