"""Host sanitizers over the library's host C++.

``make asan`` / ``make tsan`` link ``kp_rng.cpp`` (the RNG protocol: worker threads
that run the deferred numpy shuffles and randint fills into per-batch arenas) and
``kp_graph.cpp`` (prefilter BFS / Dijkstra) into ``tests/native/host_san_driver.cpp``
under ``-fsanitize=address,undefined`` and ``-fsanitize=thread``.  The driver replays
a fixed call sequence; this test runs both builds, requires a clean exit with no
sanitizer report, and requires their output to equal the production library's output
for the same sequence (called here through ctypes)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _inputs(d):
    import torch
    g = torch.Generator()
    g.manual_seed(7)
    ts = g.get_state().numpy().copy()
    ts.tofile(os.path.join(d, "torch_state.bin"))
    _, key, pos, _, _ = np.random.RandomState(11).get_state()
    np.concatenate([key.astype(np.uint32).view(np.uint8), np.array([pos], np.int32).view(np.uint8)]).tofile(
        os.path.join(d, "np_state.bin"))
    rng = np.random.default_rng(0)
    n_ent, n_tri = 400, 2500
    tri = np.stack([rng.integers(0, n_ent, n_tri), rng.integers(0, 20, n_tri), rng.integers(0, n_ent, n_tri)], 1)
    tri[0] = [n_ent - 1, 0, 0]  # every entity id appears
    tri = tri.astype(np.int32)
    tri.tofile(os.path.join(d, "triples.bin"))
    counts = rng.integers(0, 4, n_ent)
    off = np.zeros(n_ent + 1, np.int64)
    off[1:] = np.cumsum(counts)
    cls = np.concatenate([np.sort(rng.choice(12, c, replace=False)) for c in counts]).astype(np.int32)
    with open(os.path.join(d, "classes.bin"), "wb") as f:
        f.write(off.tobytes())
        f.write(cls.tobytes())
    return ts, key.astype(np.uint32), np.int32(pos), tri, n_ent, off, cls


def _expected(ts, key, pos, tri, n_ent, off, cls):
    """The driver's call sequence on the production library."""
    from kelpie_amd import _lib
    out = []
    st = ts.copy()
    key = key.copy()
    posa = np.array([pos], np.int32)
    _lib.mt19937_discard(st, 12345)
    out.append(st.tobytes())
    out.append(_lib.rng_normal(st, 200, 0.0, 0.1, cap=1).tobytes())
    out.append(_lib.bernoulli_bits(st, 1000, 0.8).tobytes())
    out.append(_lib.transe_epochs(st, key, posa, 37, 5, 5, 14542).tobytes())
    rows = np.array([7, 7, 3, 12], np.int32)
    mw = _lib.mask_words(rows, 200)
    n_slots = 48
    offs = [0]
    for i in range(n_slots):
        offs.append(offs[-1] + 9 * (10 + i) + (mw if i % 4 == 3 else 0))
    arena = np.zeros(offs[-1], np.int32)
    ka, pa = key.ctypes.data, posa.ctypes.data
    for i in range(n_slots):
        n = 9 * (10 + i)
        _lib.transe_enqueue(st, ka, pa, 10 + i, 3, 5, 14542, out=arena[offs[i]:offs[i] + n])
        if i % 4 == 3:
            _lib.conve_masks_enqueue(st, rows, [(200, 0.8)], arena[offs[i] + n:offs[i] + n + mw])
    _lib.rng_wait()
    out += [arena.tobytes(), st.tobytes(), key.tobytes(), posa.tobytes()]
    rb = np.array([12, -1, -1, 30, -1, -1], np.int32)
    rp = np.array([11, 40, 9, -1, 25, 17], np.int32)
    tot = int(sum(4 * 3 * (max(a, 0) + max(b, 0)) for a, b in zip(rb, rp)))
    calls = np.zeros(tot + 1, np.int32)
    xb, xp = _lib.transe_calls(st, ka, pa, 1, 32, 32, float(np.float32(0.2425)), rb, rp, 4, 5, 14542, calls)
    _lib.rng_wait()
    out += [calls[:tot].tobytes(), xb.tobytes(), xp.tobytes()]
    want = np.array([1, 2, 0, 3, 0, 2], np.uint8)
    tot2 = int(sum(4 * 3 * ((max(a, 0) if w & 1 else 0) + (max(b, 0) if w & 2 else 0)) for a, b, w in zip(rb, rp, want)))
    calls2 = np.zeros(tot2 + 1, np.int32)
    xb, xp = _lib.transe_calls(st, ka, pa, 1, 32, 32, float(np.float32(0.2425)), rb, rp, 4, 5, 14542, calls2, want)
    _lib.rng_wait()
    out += [calls2[:tot2].tobytes(), xb.tobytes(), xp.tobytes()]
    out.append(_lib.conve_masks(st, rows, [(200, 0.8)]).tobytes())
    out += [st.tobytes(), key.tobytes(), posa.tobytes()]
    g = _lib.Graph(n_ent, tri)
    out.append(g.bfs(np.array([0, 1, 2, 3, 5, 8, 13, 21])).tobytes())
    g.set_classes(off, cls)
    src = np.array([(i * 37) % n_ent for i in range(64)])
    dst = np.array([(i * 101 + 7) % n_ent for i in range(64)])
    out.append(g.dijkstra_pairs(src, dst).tobytes())
    return b"".join(out)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_sanitizer_build(kind, tmp_path):
    r = subprocess.run(["make", "-C", ROOT, kind], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    inputs = _inputs(str(tmp_path))
    out = tmp_path / "out.bin"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    p = subprocess.run([os.path.join(ROOT, "build", "san", f"host_{kind}"), str(tmp_path), str(out)],
                       capture_output=True, text=True, env=env, timeout=600)
    report = p.stderr
    assert p.returncode == 0, report[-4000:]
    for marker in ("AddressSanitizer", "LeakSanitizer", "ThreadSanitizer", "runtime error"):
        assert marker not in report, report[-4000:]
    assert out.read_bytes() == _expected(*inputs)
