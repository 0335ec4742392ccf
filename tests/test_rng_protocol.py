"""The host RNG protocol's shortcuts consume exactly what the reference's calls consume."""
import json
import os

import numpy as np
import pytest
import torch

from kelpie_amd import _lib
from kelpie_amd.rng import ReferenceRNG


def _state():
    return torch.get_rng_state().numpy().copy()


def test_discard_matches_randperm():
    for n in (1, 2, 7, 72, 600):
        torch.manual_seed(3)
        s0 = _state()
        torch.randperm(n)
        ref = _state()
        _lib.mt19937_discard(s0, max(n - 1, 0))
        assert np.array_equal(s0, ref), n


def test_discard_matches_conve_construction():
    for hidden, dim in ((1216, 60), (9728, 200)):
        torch.manual_seed(5)
        torch.rand(3)
        s0 = _state()
        torch.nn.Conv2d(1, 32, (3, 3), 1, 0, bias=True)
        torch.nn.Linear(hidden, dim)
        ref = _state()
        torch.set_rng_state(torch.from_numpy(s0))
        ReferenceRNG().conve_construction(hidden, dim)
        assert np.array_equal(_state(), ref)


def test_bernoulli_bits_match_torch():
    for shape, p in (((3, 5), 0.8), ((20, 200), 0.8), ((7, 60), 0.5)):
        torch.manual_seed(11)
        s0 = _state()
        m = torch.empty(*shape).bernoulli_(p).numpy().reshape(-1)
        ref = _state()
        bits = _lib.bernoulli_bits(s0, m.size, p)
        got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:m.size]
        assert np.array_equal(got, m.astype(np.uint8))
        assert np.array_equal(s0, ref)


def test_complex_epochs_skip_is_equivalent():
    rng = ReferenceRNG()
    torch.manual_seed(9)
    rng.complex_epochs(40, 43, 512)  # skipped values
    a = torch.rand(4)
    torch.manual_seed(9)
    for _ in range(43):
        torch.randperm(40)
    b = torch.rand(4)
    assert torch.equal(a, b)


@pytest.mark.parametrize("R,E", [(9, 5), (150, 7), (700, 4)])
def test_transe_epochs_match_reference_calls(R, E):
    """R >= 16 runs the numpy shuffles on the helper thread; 700 rows cross numpy
    regenerations inside one epoch's shuffle."""
    ratio, N = 5, 301
    torch.manual_seed(2)
    np.random.seed(2)
    blob = ReferenceRNG().transe_epochs(R, E, ratio, N).reshape(E, 3, R)
    after = torch.rand(2)
    np_after = np.random.randint(0, 1 << 30, 8)
    torch.manual_seed(2)
    np.random.seed(2)
    rows = np.arange(R * 3).reshape(R, 3)
    for e in range(E):
        np.random.shuffle(rows)
        ents = torch.randint(high=N, size=(ratio * R,))
        hot = torch.randint(high=2, size=(ratio * R,))
        assert np.array_equal(rows[:, 0] // 3, blob[e, 0])
        assert np.array_equal(ents[:R].numpy(), blob[e, 1])
        assert np.array_equal(hot[:R].numpy(), blob[e, 2])
    assert torch.equal(torch.rand(2), after)
    assert np.array_equal(np.random.randint(0, 1 << 30, 8), np_after)


def test_conve_masks_match_torch_dropout_sequence():
    rng = ReferenceRNG()
    steps = [3, 7, 1]
    torch.manual_seed(21)
    words = rng.conve_masks(steps, [(20, 0.2)])
    after = torch.rand(2)
    torch.manual_seed(21)
    off = 0
    for b in steps:
        m = torch.empty(b, 20).bernoulli_(0.8).numpy().reshape(-1).astype(np.uint8)
        nw = (b * 20 + 31) // 32
        got = np.unpackbits(words[off:off + nw].view(np.uint32).view(np.uint8), bitorder="little")[:b * 20]
        assert np.array_equal(got, m)
        off += nw
    assert torch.equal(torch.rand(2), after)


def test_numpy_state_address_layout():
    """The in-place numpy path relies on mt19937_state = {uint32 key[624]; int pos}."""
    import ctypes
    from kelpie_amd.rng import _np_mt_state_address
    np.random.seed(7)
    np.random.random(5)
    _, key, pos, _, _ = np.random.get_state()
    addr = _np_mt_state_address()
    k = np.ctypeslib.as_array((ctypes.c_uint32 * 624).from_address(addr))
    p = ctypes.c_int.from_address(addr + 4 * 624).value
    assert np.array_equal(k, np.asarray(key, np.uint32)) and p == pos


def test_deferred_transe_draws_match_reference_calls():
    """ReferenceRNG.deferred(): the slots' shuffles and randints are queued to the
    library's workers (kp_rng_transe_enqueue) while other torch draws interleave on
    the calling thread; after the block every array and both generator states equal
    the reference's sequential calls.  Includes empty slots (R = 0, epochs = 0), a
    single-row slot and rows that cross numpy regenerations."""
    ratio, N, E = 5, 301, 6
    Rs = [9, 0, 150, 1, 700, 33, 16]
    torch.manual_seed(5)
    np.random.seed(5)
    rng = ReferenceRNG()
    blobs, inits = [], []
    with rng.deferred():
        for i, R in enumerate(Rs):
            inits.append(rng.rand_init(8))
            blobs.append(rng.transe_epochs(R, 0 if i == 3 else E, ratio, N))
    # the arrays of one block lie back to back in one arena
    live = [b for b in blobs if b.size]
    assert all(b.base is live[0].base for b in live)
    after = torch.rand(2)
    np_after = np.random.randint(0, 1 << 30, 8)
    torch.manual_seed(5)
    np.random.seed(5)
    for i, R in enumerate(Rs):
        assert np.array_equal(torch.rand(1, 8).numpy()[0], inits[i])
        epochs = 0 if i == 3 else E
        assert blobs[i].size == epochs * 3 * R
        blob = blobs[i].reshape(epochs, 3, R)
        rows = np.arange(R * 3).reshape(R, 3)
        for e in range(epochs):
            np.random.shuffle(rows)
            ents = torch.randint(high=N, size=(ratio * R,))
            hot = torch.randint(high=2, size=(ratio * R,))
            assert np.array_equal(rows[:, 0] // 3, blob[e, 0])
            assert np.array_equal(ents[:R].numpy(), blob[e, 1])
            assert np.array_equal(hot[:R].numpy(), blob[e, 2])
    assert torch.equal(torch.rand(2), after)
    assert np.array_equal(np.random.randint(0, 1 << 30, 8), np_after)


def _unpack(words, off, n):
    nw = (n + 31) // 32
    return np.unpackbits(words[off:off + nw].view(np.uint32).view(np.uint8), bitorder="little")[:n], off + nw


@pytest.mark.parametrize("deferred", [False, True])
def test_conve_three_dropouts_match_torch_forward_sequence(deferred):
    """The three ConvE dropouts of each step in the forward's order (conve.py:142,147,151):
    input (b x 40 x h), feature-map Dropout2d (b x 32), hidden (b x d); a rate-1 dropout
    ships zero words and draws nothing (ATen _dropout_impl), a rate-0 one is absent."""
    rng = ReferenceRNG()
    steps = [3, 5, 1]
    d = 60
    for rates in ((0.2, 0.3, 0.1), (0.2, 0.0, 0.1), (0.0, 1.0, 0.25), (0.5, 0.3, 0.0)):
        segs = [(2 * d, rates[0]), (32, rates[1]), (d, rates[2])]
        torch.manual_seed(31)
        if deferred:
            with rng.deferred():
                words = rng.conve_masks(steps, segs)
        else:
            words = rng.conve_masks(steps, segs)
        after = torch.rand(2)
        torch.manual_seed(31)
        off = 0
        for b in steps:
            for n, p in segs:
                if p == 0:
                    continue
                if p == 1:
                    got, off = _unpack(words, off, b * n)
                    assert not got.any()
                    continue
                m = torch.empty(b, n).bernoulli_(1 - p).numpy().reshape(-1).astype(np.uint8)
                got, off = _unpack(words, off, b * n)
                assert np.array_equal(got, m), (rates, b, n)
        assert off == words.size
        assert torch.equal(torch.rand(2), after), rates


def test_deferred_conve_masks_match_torch_dropout_sequence():
    """Deferred masks (kp_rng_conve_masks_enqueue) interleaved with other torch draws
    and a discard, as in a ConvE batch schedule: same bits, same final state."""
    rng = ReferenceRNG()
    plans = [[3, 7, 1], [0, 2], [], [40, 40, 13]]
    torch.manual_seed(23)
    got, inits = [], []
    with rng.deferred():
        for steps in plans:
            inits.append(rng.rand_init(6))
            rng.conve_construction(4, 20)
            got.append(rng.conve_masks(steps, [(20, 0.2)]))
    after = torch.rand(2)
    torch.manual_seed(23)
    for steps, words, init in zip(plans, got, inits):
        assert np.array_equal(torch.rand(1, 6).numpy()[0], init)
        torch.empty(32 * 9 + 32 + 4 * 20 + 20).uniform_()  # the construction's draws, one output each
        off = 0
        for b in steps:
            m = torch.empty(b, 20).bernoulli_(0.8).numpy().reshape(-1).astype(np.uint8)
            nw = (b * 20 + 31) // 32
            bits = np.unpackbits(words[off:off + nw].view(np.uint32).view(np.uint8), bitorder="little")[:b * 20]
            assert np.array_equal(bits, m)
            off += nw
        assert off == words.size
    assert torch.equal(torch.rand(2), after)


_NORMAL_CHECK = r"""
import math, random, sys
import numpy as np, torch
from kelpie_amd import _lib
cap = _lib.normal_cap()
bad = 0
for trial in range(int(sys.argv[1])):
    rr = random.Random(trial)
    torch.manual_seed(trial)
    torch.rand(rr.randint(0, 1500))
    st = torch.get_rng_state().numpy().copy()
    d = rr.choice([16, 17, 33, 50, 100, 200, 256, 400])
    std = math.sqrt(2.0 / (d + 1))
    ref = torch.empty(1, d).normal_(0.0, std).numpy()[0]
    out = _lib.rng_normal(st, d, 0.0, std, cap)
    bad += int((out != ref).sum()) + int(not np.array_equal(st, torch.get_rng_state().numpy()))
print(cap, bad)
"""


@pytest.mark.parametrize("capability", [None, "default"])
def test_normal_matches_torch_bit_for_bit(capability):
    """kp_rng_normal equals torch's normal_ value for value and leaves the same generator
    state, for the CPU kernel this torch runs (AVX2 / AVX512: avx_mathfun with FMA
    contraction) and, in a child process with ATEN_CPU_CAPABILITY=default, for the
    scalar kernel (libm)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    if capability:
        env["ATEN_CPU_CAPABILITY"] = capability
    out = subprocess.run([sys.executable, "-c", _NORMAL_CHECK, "400"], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    cap, bad = out.stdout.split()
    if capability == "default":
        assert cap == "0"
    assert bad == "0", out.stdout


def test_fused_transe_calls_match_reference_sequence():
    """ReferenceRNG.transe_calls (one library call for several compute_relevance calls)
    equals the reference's sequence per call, rand(1, D) -> xavier_normal_ -> base epochs
    -> xavier_normal_ -> pt epochs, inside and outside deferred(), with and without the
    base slot, and leaves both generators where the sequence does."""
    import math
    ratio, N, E, d = 5, 301, 4, 40
    batches = [[(12, 7), (-1, 30)], [(0, 5)], [(33, -1), (-1, 0), (-1, 9)]]
    torch.manual_seed(11)
    np.random.seed(11)
    rng = ReferenceRNG()
    got = []
    with rng.deferred():
        for b in batches[:2]:
            got.append(rng.transe_calls(d, d, [x[0] for x in b], [x[1] for x in b], E, ratio, N))
    got.append(rng.transe_calls(d, d, [x[0] for x in batches[2]], [x[1] for x in batches[2]], E, ratio, N))
    after = (torch.rand(3), np.random.randint(0, 1 << 30, 4))
    torch.manual_seed(11)
    np.random.seed(11)
    std = math.sqrt(2.0 / (d + 1))

    def epochs(R):
        out = []
        rows = np.arange(R * 3).reshape(R, 3)
        for _ in range(E):
            np.random.shuffle(rows)
            ents = torch.randint(high=N, size=(ratio * R,))
            hot = torch.randint(high=2, size=(ratio * R,))
            out.append(np.stack([rows[:, 0] // 3, ents[:R].numpy(), hot[:R].numpy()]))
        return np.concatenate(out).reshape(-1) if R > 0 else np.zeros(0, np.int64)

    for b, (xb, xp, draws) in zip(batches, got):
        for i, (Rb, Rp) in enumerate(b):
            torch.rand(1, d)
            assert np.array_equal(torch.empty(1, d).normal_(0.0, std).numpy()[0], xb[i])
            if Rb >= 0:
                assert np.array_equal(epochs(Rb), draws[i][0])
            assert np.array_equal(torch.empty(1, d).normal_(0.0, std).numpy()[0], xp[i])
            if Rp >= 0:
                assert np.array_equal(epochs(Rp), draws[i][1])
    assert torch.equal(torch.rand(3), after[0])
    assert np.array_equal(np.random.randint(0, 1 << 30, 4), after[1])


_JUMP_SCRIPT = r"""
import hashlib, json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
from kelpie_amd import _lib
torch.manual_seed(321)
base = torch.get_rng_state().numpy().copy()
out = {}
for pre in (0, 1, 300, 623):
    st = base.copy()
    if pre:
        _lib.mt19937_discard(st, pre)
    for n in (1, 623, 624, 625, 1248, 4369, 123457, 1946040, 30000001):
        s2 = st.copy()
        _lib.mt19937_discard(s2, n)
        out[f"{pre}_{n}"] = hashlib.sha1(s2.tobytes()).hexdigest()
st = base.copy()
_lib.mt19937_discard(st, 30000001)
torch.set_rng_state(torch.from_numpy(st))
out["draw"] = torch.rand(8).tolist()
print(json.dumps(out))
"""


def test_mt19937_jump_ahead_equals_the_walk():
    """kp_mt19937_discard by MT19937 jump-ahead (GF(2) characteristic polynomial,
    x^D mod P, Horner) leaves the torch generator exactly where the twist-by-twist walk
    does, across block boundaries and from every in-block position; torch then draws
    the same values.  KP_MT_JUMP_MIN=1 forces the jump for every skip past the block."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for jmin in ("0", "1"):
        env = dict(os.environ, KP_MT_JUMP_MIN=jmin)
        r = subprocess.run([sys.executable, "-c", _JUMP_SCRIPT, root], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[0] == outs[1]


def test_failed_background_draw_poisons_the_stream(monkeypatch):
    """A failed background walk leaves the generators at a state the reference never
    reaches: every later draw raises until the caller reseeds and clears the poison, or
    restores a checkpoint."""
    from kelpie_amd import rng as krng
    cp = krng.StateCheckpoint()
    r = ReferenceRNG()

    def boom():
        raise RuntimeError("walk failed")

    monkeypatch.setattr(krng._lib, "rng_wait", boom)
    monkeypatch.setattr(krng, "_outstanding", True)
    with pytest.raises(RuntimeError, match="walk failed"):
        krng.sync()
    monkeypatch.undo()
    with pytest.raises(RuntimeError, match="stream lost"):
        r.rand_init(8)
    with pytest.raises(RuntimeError, match="stream lost"):
        r.discard(3)
    cp.restore()  # a restored checkpoint is a known state again
    assert r.rand_init(8).shape == (8,)
    krng._poisoned = "x"
    krng.clear_poison()
    r.discard(2)
    krng.sync()
