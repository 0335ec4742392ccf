"""ctypes binding of ``libkelpie_hip.so`` (C ABI: ``include/kelpie_hip.h``).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) for gfx950.
There is no CPU fallback: if the library is missing every engine call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KELPIE_HIP_LIB", os.path.join(_HERE, "libkelpie_hip.so"))

KP_MODEL = {"TransE": 0, "ComplEx": 1, "ConvE": 2}
KP_INLINE = 1  # kp_rng_transe_calls_async walked inline (include/kelpie_hip.h)
KP_OPT = {"Adagrad": 0, "Adam": 1, "SGD": 2}

# symbols declared by include/kelpie_hip.h
EXPORTS = ["kp_ctx_create", "kp_ctx_destroy", "kp_last_error", "kp_posttrain_rank", "kp_all_scores",
           "kp_convertible", "kp_mt19937_discard", "kp_last_timing", "kp_version", "kp_rng_bernoulli_bits",
           "kp_rng_transe_epochs", "kp_rng_transe_enqueue", "kp_rng_wait", "kp_rng_batch_close", "kp_rng_batch_wait", "kp_rng_conve_masks", "kp_rng_conve_masks_enqueue", "kp_graph_create", "kp_graph_destroy",
           "kp_graph_last_error", "kp_graph_bfs", "kp_graph_set_classes", "kp_graph_dijkstra_pairs",
           "kp_predict_tails", "kp_dp_relevance", "kp_criage_relevance", "kp_hot_intervals", "kp_rng_normal",
           "kp_rng_transe_calls", "kp_train_epoch", "kp_read_tables", "kp_view_create", "kp_view_destroy",
           "kp_sched_batch_create", "kp_sched_batch_destroy", "kp_sched_add_calls", "kp_sched_pack",
           "kp_gather_i32", "kp_rng_transe_calls_async", "kp_rng_torch_take", "kp_conve_train_begin",
           "kp_conve_train_step", "kp_conve_train_read", "kp_host_alloc", "kp_host_free"]


class ModelDesc(C.Structure):
    _fields_ = [("model", C.c_int32), ("n_ent", C.c_int32), ("n_rel2", C.c_int32), ("dim", C.c_int32),
                ("entity", C.c_void_p), ("relation", C.c_void_p), ("conv_w", C.c_void_p), ("conv_b", C.c_void_p),
                ("fc_w", C.c_void_p), ("fc_b", C.c_void_p), ("bn_alpha", C.c_void_p), ("bn_beta", C.c_void_p),
                ("norm_p", C.c_int32)]


class HP(C.Structure):
    _fields_ = [("optimizer", C.c_int32), ("epochs", C.c_int32), ("batch_size", C.c_int32), ("lr", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("reg_weight", C.c_float),
                ("margin", C.c_float), ("neg_ratio", C.c_int32), ("label_smoothing", C.c_float),
                ("hidden_dropout", C.c_float), ("input_dropout", C.c_float), ("fmap_dropout", C.c_float),
                ("reg_kind", C.c_int32)]


KP_REG = {"N3": 0, "N2": 1}


class Batch(C.Structure):
    _fields_ = [("n_slots", C.c_int32), ("x0", C.c_void_p), ("row_off", C.c_void_p), ("rows", C.c_void_p),
                ("rng_off", C.c_void_p), ("rng", C.c_void_p), ("pred", C.c_void_p), ("filt_off", C.c_void_p),
                ("filt", C.c_void_p), ("out_x", C.c_void_p), ("out_score", C.c_void_p), ("out_rank", C.c_void_p)]


class KelpieHipError(RuntimeError):
    pass


_LIB = None


def lib():
    """Load the HIP library (raises if it is absent: no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise KelpieHipError(f"{LIB_PATH} not found: build it with `make` (hipcc --offload-arch=gfx950)")
        L = C.CDLL(LIB_PATH)
        L.kp_ctx_create.argtypes = [C.c_int, C.POINTER(ModelDesc), C.POINTER(C.c_void_p)]
        L.kp_ctx_destroy.argtypes = [C.c_void_p]
        L.kp_last_error.argtypes = [C.c_void_p]
        L.kp_last_error.restype = C.c_char_p
        L.kp_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
        L.kp_host_free.argtypes = [C.c_void_p]
        L.kp_posttrain_rank.argtypes = [C.c_void_p, C.POINTER(HP), C.POINTER(Batch)]
        L.kp_all_scores.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_convertible.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                     C.c_void_p, C.c_void_p]
        L.kp_mt19937_discard.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.kp_predict_tails.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p]
        L.kp_dp_relevance.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_float, C.c_float, C.c_int32, C.c_int32,
                                       C.c_void_p]
        L.kp_criage_relevance.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_graph_create.argtypes = [C.c_int32, C.c_int64, C.c_void_p, C.POINTER(C.c_void_p)]
        L.kp_graph_destroy.argtypes = [C.c_void_p]
        L.kp_graph_destroy.restype = None
        L.kp_graph_last_error.restype = C.c_char_p
        L.kp_graph_bfs.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.kp_graph_set_classes.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_graph_dijkstra_pairs.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_rng_bernoulli_bits.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_double, C.c_void_p]
        L.kp_rng_transe_epochs.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                           C.c_int32, C.c_int64, C.c_void_p]
        L.kp_rng_transe_enqueue.argtypes = L.kp_rng_transe_epochs.argtypes
        L.kp_rng_wait.argtypes = []
        L.kp_rng_batch_close.argtypes = [C.POINTER(C.c_int64)]
        L.kp_rng_batch_wait.argtypes = [C.c_int64]
        L.kp_train_epoch.argtypes = [C.c_void_p, C.POINTER(HP), C.c_int32, C.c_void_p, C.c_void_p, C.c_int32]
        L.kp_read_tables.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_rng_normal.argtypes = [C.c_void_p, C.c_size_t, C.c_int64, C.c_float, C.c_float, C.c_int32, C.c_void_p]
        L.kp_rng_transe_calls.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_float, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_rng_conve_masks.argtypes = [C.c_void_p, C.c_size_t, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
        L.kp_rng_conve_masks_enqueue.argtypes = L.kp_rng_conve_masks.argtypes
        L.kp_last_timing.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_int64), C.POINTER(C.c_double)]
        L.kp_hot_intervals.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(C.c_int64)]
        L.kp_version.restype = C.c_char_p
        L.kp_view_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                                     C.POINTER(C.c_void_p)]
        L.kp_view_destroy.argtypes = [C.c_void_p]
        L.kp_view_destroy.restype = None
        L.kp_sched_batch_create.argtypes = [C.POINTER(C.c_void_p)]
        L.kp_sched_batch_destroy.argtypes = [C.c_void_p]
        L.kp_sched_batch_destroy.restype = None
        L.kp_sched_add_calls.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.kp_sched_pack.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                    C.c_int64]
        L.kp_gather_i32.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.kp_rng_transe_calls_async.argtypes = L.kp_rng_transe_calls.argtypes
        L.kp_rng_torch_take.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.kp_conve_train_begin.argtypes = [C.c_void_p] * 5
        L.kp_conve_train_step.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_float, C.c_float,
                                                                                      C.c_int32]
        L.kp_conve_train_read.argtypes = [C.c_void_p] * 9
        _LIB = L
    return _LIB


def source_sha16() -> str:
    """sha256 (16 hex digits) over the library's sources -- every file of kelpie_amd/csrc
    and include/kelpie_hip.h, in name order.  tools/prof_summary.py stamps each committed
    counter pass with it, and bench.py cites a pass only when it matches the tree it
    runs (a pass older than the kernels it describes is never reported)."""
    import hashlib
    h = hashlib.sha256()
    src = os.path.join(_HERE, "csrc")
    paths = sorted(os.path.join(src, f) for f in os.listdir(src))
    paths.append(os.path.join(os.path.dirname(_HERE), "include", "kelpie_hip.h"))
    for path in paths:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def attention_contraction():
    """The ComplEx / ConvE attention kernel a new Context uses (kp_api.hip reads the same
    variable): "bf16x3" (kp_attn3, default) or "f32" (kp_attn, KP_ATTN=f32)."""
    return "f32" if os.environ.get("KP_ATTN") == "f32" else "bf16x3"


def _ptr(a):
    """Raw data address of a C-contiguous numpy array.  ``a.ctypes.data_as`` costs
    15-40 us per call once torch is imported (most of the per-slot host time of
    the TransE draws); the caller keeps ``a`` alive across the C call."""
    return None if a is None else C.c_void_p(a.__array_interface__["data"][0])


def check(rc, ctx=None):
    if rc != 0:
        msg = lib().kp_last_error(ctx).decode(errors="replace")
        raise KelpieHipError(f"libkelpie_hip error {rc}: {msg}")


def mt19937_discard(state: np.ndarray, n: int):
    """Advance a torch CPU-generator state blob (uint8[5056]) by n 32-bit draws, in place."""
    assert state.dtype == np.uint8 and state.flags.c_contiguous
    check(lib().kp_mt19937_discard(_ptr(state), state.size, int(n)))


def bernoulli_bits(state: np.ndarray, n: int, p: float) -> np.ndarray:
    """Keep-mask of ``torch.empty(n).bernoulli_(p)`` as packed little-endian bits
    (uint32 words), advancing the state blob in place like torch does."""
    words = np.zeros((n + 31) // 32, dtype=np.uint32)
    check(lib().kp_rng_bernoulli_bits(_ptr(state), state.size, int(n), float(p), _ptr(words)))
    return words


def transe_epochs(torch_state: np.ndarray, np_key, np_pos, R: int, epochs: int,
                  ratio: int, n_entities: int) -> np.ndarray:
    """``np_key`` / ``np_pos``: numpy arrays, or raw addresses (int) of a live
    MT19937 ``key[624]`` / ``pos`` pair, which are then advanced in place."""
    out = np.empty(max(1, epochs * 3 * R), np.int32)  # every element is written
    key = C.c_void_p(np_key) if isinstance(np_key, int) else _ptr(np_key)
    pos = C.c_void_p(np_pos) if isinstance(np_pos, int) else _ptr(np_pos)
    check(lib().kp_rng_transe_epochs(_ptr(torch_state), torch_state.size, key, pos, int(R),
                                     int(epochs), int(ratio), int(n_entities), _ptr(out)))
    return out[:epochs * 3 * R]


def transe_enqueue(torch_state: np.ndarray, np_key: int, np_pos: int, R: int, epochs: int,
                   ratio: int, n_entities: int, out: np.ndarray | None = None) -> np.ndarray:
    """Deferred :func:`transe_epochs` on the live numpy state at the raw addresses
    ``np_key`` / ``np_pos``: advances ``torch_state`` now and returns the output
    array (``out``, int32 C-contiguous of ``epochs*3*R`` elements, if given), which
    is complete only after :func:`rng_wait`."""
    if out is None:
        out = np.empty(max(1, epochs * 3 * R), np.int32)
    assert out.dtype == np.int32 and out.flags.c_contiguous and out.size >= epochs * 3 * R
    check(lib().kp_rng_transe_enqueue(_ptr(torch_state), torch_state.size, C.c_void_p(np_key), C.c_void_p(np_pos),
                                      int(R), int(epochs), int(ratio), int(n_entities), _ptr(out)))
    return out[:epochs * 3 * R]


def normal_cap() -> int:
    """Which ATen normal_ kernel this torch runs: 1 for its AVX2 / AVX512 builds, 0 for
    the scalar default one (kp_rng_normal's ``cap``)."""
    import torch
    return 0 if torch.backends.cpu.get_cpu_capability() == "DEFAULT" else 1


def rng_normal(state: np.ndarray, n: int, mean: float, std: float, cap: int | None = None) -> np.ndarray:
    """``torch.empty(n).normal_(mean, std)`` values (n >= 16) from the state blob, advanced in place."""
    assert state.dtype == np.uint8 and state.flags.c_contiguous
    out = np.empty(n, np.float32)
    check(lib().kp_rng_normal(_ptr(state), state.size, int(n), float(mean), float(std),
                              normal_cap() if cap is None else int(cap), _ptr(out)))
    return out


def transe_calls(state: np.ndarray, np_key: int, np_pos: int, cap: int, D: int, d: int, std: float,
                 R_base: np.ndarray, R_pt: np.ndarray, epochs: int, ratio: int, n_entities: int,
                 out: np.ndarray | None, want: np.ndarray | None = None):
    """kp_rng_transe_calls for len(R_base) calls: returns (x_base [n][d], x_pt [n][d]); the
    epoch draws land in ``out`` back to back (complete after :func:`rng_wait`).  ``want``
    (uint8 per call, bit 0 base / bit 1 pt; None = all): unwanted post-trainings only
    advance the generators."""
    n = len(R_base)
    rb = np.ascontiguousarray(R_base, dtype=np.int32)
    rp = np.ascontiguousarray(R_pt, dtype=np.int32)
    w = None if want is None else np.ascontiguousarray(want, dtype=np.uint8)
    xb = np.empty((n, d), np.float32)
    xp = np.empty((n, d), np.float32)
    check(lib().kp_rng_transe_calls(_ptr(state), state.size, C.c_void_p(np_key), C.c_void_p(np_pos), int(cap),
                                    int(D), int(d), float(std), n, _ptr(rb), _ptr(rp), _ptr(w), int(epochs),
                                    int(ratio), int(n_entities), _ptr(xb), _ptr(xp), _ptr(out)))
    return xb, xp


def transe_calls_async(state: np.ndarray, np_key: int, np_pos: int, cap: int, D: int, d: int, std: float,
                       R_base, R_pt, epochs: int, ratio: int, n_entities: int, out: np.ndarray | None,
                       want: np.ndarray | None = None):
    """kp_rng_transe_calls_async: :func:`transe_calls` with the torch-stream walk on the
    library's walker thread, starting from ``state`` unless a walk already carries the
    stream.  Everything (x_base, x_pt, ``out``) is complete after :func:`rng_wait`; the
    stream comes back with :func:`torch_take`.  Returns ``(x_base, x_pt, queued)``:
    ``queued`` False when no walker thread could start and the walk ran inline (``state``
    then holds the advanced stream and no walk carries it)."""
    n = len(R_base)
    rb = np.ascontiguousarray(R_base, dtype=np.int32)
    rp = np.ascontiguousarray(R_pt, dtype=np.int32)
    w = None if want is None else np.ascontiguousarray(want, dtype=np.uint8)
    xb = np.empty((n, d), np.float32)
    xp = np.empty((n, d), np.float32)
    rc = lib().kp_rng_transe_calls_async(_ptr(state), state.size, C.c_void_p(np_key), C.c_void_p(np_pos), int(cap),
                                         int(D), int(d), float(std), n, _ptr(rb), _ptr(rp), _ptr(w), int(epochs),
                                         int(ratio), int(n_entities), _ptr(xb), _ptr(xp), _ptr(out))
    if rc != KP_INLINE:
        check(rc)
    return xb, xp, rc != KP_INLINE


def torch_take(state: np.ndarray) -> bool:
    """Wait for the asynchronous walks and write the torch stream they carry into ``state``
    (True), or leave ``state`` alone when none carries it (False)."""
    taken = np.zeros(1, np.int32)
    check(lib().kp_rng_torch_take(_ptr(state), state.size, _ptr(taken)))
    return bool(taken[0])


def rng_wait():
    check(lib().kp_rng_wait())


def rng_batch_close() -> int:
    """Close the open batch of deferred draws; returns its id (kp_rng_batch_close)."""
    v = C.c_int64(0)
    check(lib().kp_rng_batch_close(C.byref(v)))
    return int(v.value)


def rng_batch_wait(batch_id: int):
    """Wait for every deferred draw of the batches <= batch_id (kp_rng_batch_wait)."""
    check(lib().kp_rng_batch_wait(int(batch_id)))


def _segments(segs):
    """[(elements per pair, keep probability)] -> (int32 elems, float64 keeps)."""
    e = np.ascontiguousarray([int(n) for n, _ in segs], dtype=np.int32)
    k = np.ascontiguousarray([float(p) for _, p in segs], dtype=np.float64)
    return e, k


def mask_words(rows_per_step, seg_elems) -> int:
    """uint32 words of the per-step packed dropout masks: per step, one word-aligned run
    of keep bits per segment (``seg_elems``: elements per pair, an int or a list)."""
    rows = np.asarray(rows_per_step, dtype=np.int64)
    elems = [seg_elems] if np.isscalar(seg_elems) else list(seg_elems)
    return int(sum(((rows * int(n) + 31) // 32).sum() for n in elems))


def conve_masks_enqueue(torch_state: np.ndarray, rows_per_step, segs, out: np.ndarray):
    """Deferred :func:`conve_masks` into ``out`` (int32 / uint32, :func:`mask_words`
    elements): advances ``torch_state`` now; ``out`` is complete after :func:`rng_wait`."""
    rows = np.ascontiguousarray(rows_per_step, dtype=np.int32)
    e, k = _segments(segs)
    assert out.dtype.itemsize == 4 and out.flags.c_contiguous and out.size >= mask_words(rows, e)
    check(lib().kp_rng_conve_masks_enqueue(_ptr(torch_state), torch_state.size, len(rows), _ptr(rows), len(e),
                                           _ptr(e), _ptr(k), _ptr(out)))
    return out


def conve_masks(torch_state: np.ndarray, rows_per_step, segs) -> np.ndarray:
    """ConvE dropout keep bits (kp_rng_conve_masks): ``segs`` = [(elements per pair,
    keep probability)] in the forward's draw order."""
    rows = np.ascontiguousarray(rows_per_step, dtype=np.int32)
    e, k = _segments(segs)
    words = mask_words(rows, e)
    out = np.zeros(max(1, words), np.uint32)
    check(lib().kp_rng_conve_masks(_ptr(torch_state), torch_state.size, len(rows), _ptr(rows), len(e), _ptr(e),
                                   _ptr(k), _ptr(out)))
    return out[:words]


class Context:
    """One device context holding the frozen model tables (kp_ctx)."""

    def __init__(self, model_name, entity, relation, conve=None, device=0, norm_p=0):
        L = lib()
        self._keep = []
        E = np.ascontiguousarray(entity, dtype=np.float32)
        R = np.ascontiguousarray(relation, dtype=np.float32)
        d = ModelDesc(KP_MODEL[model_name], E.shape[0], R.shape[0], E.shape[1], _ptr(E), _ptr(R))
        d.norm_p = int(norm_p)
        self._keep += [E, R]
        if conve is not None:
            for k in ("conv_w", "conv_b", "fc_w", "fc_b", "bn_alpha", "bn_beta"):
                a = np.ascontiguousarray(conve[k], dtype=np.float32)
                self._keep.append(a)
                setattr(d, k, _ptr(a))
        h = C.c_void_p()
        rc = L.kp_ctx_create(int(device), C.byref(d), C.byref(h))
        if rc != 0:
            raise KelpieHipError(f"kp_ctx_create failed ({rc}): {L.kp_last_error(None).decode()}")
        self.h = h
        self.n_ent, self.dim = E.shape
        self._keep = []  # tables are copied to the device

    def close(self):
        if getattr(self, "h", None):
            lib().kp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def posttrain_rank(self, hp: HP, x0, row_off, rows, rng_off, rng, pred, filt_off, filt, want_x=False):
        n = len(row_off) - 1
        x0 = np.ascontiguousarray(x0, dtype=np.float32)
        row_off = np.ascontiguousarray(row_off, dtype=np.int32)
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        rng_off = np.ascontiguousarray(rng_off, dtype=np.int64)
        rng = np.ascontiguousarray(rng, dtype=np.int32)
        pred = np.ascontiguousarray(pred, dtype=np.int32)
        filt_off = np.ascontiguousarray(filt_off, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32)
        out_x = np.zeros((n, self.dim), np.float32) if want_x else None
        out_s = np.zeros(n, np.float32)
        out_r = np.zeros(n, np.int64)
        b = Batch(n, _ptr(x0), _ptr(row_off), _ptr(rows), _ptr(rng_off), _ptr(rng), _ptr(pred), _ptr(filt_off),
                  _ptr(filt), _ptr(out_x), _ptr(out_s), _ptr(out_r))
        check(lib().kp_posttrain_rank(self.h, C.byref(hp), C.byref(b)), self.h)
        return out_s, out_r, out_x

    def all_scores(self, heads, rels):
        heads = np.ascontiguousarray(heads, dtype=np.int32)
        rels = np.ascontiguousarray(rels, dtype=np.int32)
        out = np.zeros((len(heads), self.n_ent), np.float32)
        check(lib().kp_all_scores(self.h, len(heads), _ptr(heads), _ptr(rels), _ptr(out)), self.h)
        return out

    def convertible(self, heads, rel, obj, filt_off, filt):
        heads = np.ascontiguousarray(heads, dtype=np.int32)
        filt_off = np.ascontiguousarray(filt_off, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32)
        keep = np.zeros(len(heads), np.uint8)
        check(lib().kp_convertible(self.h, len(heads), _ptr(heads), int(rel), int(obj), _ptr(filt_off),
                                   _ptr(filt), _ptr(keep)), self.h)
        return keep

    def predict_tails(self, triples, filt_off, filt):
        """kp_predict_tails: (target scores float32, filtered ranks int64) per triple."""
        t = np.ascontiguousarray(np.asarray(triples, dtype=np.int32).reshape(-1, 3))
        filt_off = np.ascontiguousarray(filt_off, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32) if len(filt) else np.zeros(1, np.int32)
        score = np.zeros(len(t), np.float32)
        rank = np.zeros(len(t), np.int64)
        check(lib().kp_predict_tails(self.h, len(t), _ptr(t), _ptr(filt_off), _ptr(filt), _ptr(score), _ptr(rank)),
              self.h)
        return score, rank

    def train_epoch(self, hp: HP, triples, aux, epoch: int):
        """kp_train_epoch: one optimizer epoch on this context's own tables (ComplEx: aux =
        the epoch's permutation; TransE: triples / aux = positive / corrupted rows)."""
        t = np.ascontiguousarray(np.asarray(triples, dtype=np.int32).reshape(-1, 3))
        pm = np.ascontiguousarray(aux, dtype=np.int32)
        assert len(pm) == len(t)
        check(lib().kp_train_epoch(self.h, C.byref(hp), len(t), _ptr(t), _ptr(pm), int(epoch)), self.h)

    def conve_train_begin(self, bn_w, bn_b, bn_m, bn_v):
        """kp_conve_train_begin: batch-norm parameters and running statistics (1 + 32 + dim each)."""
        a = [np.ascontiguousarray(v, dtype=np.float32).reshape(-1) for v in (bn_w, bn_b, bn_m, bn_v)]
        assert all(len(v) == 33 + self.dim for v in a)
        check(lib().kp_conve_train_begin(self.h, *[_ptr(v) for v in a]), self.h)

    def conve_train_step(self, pairs, tail_off, tails, in_noise, fm_noise, hid_noise, lr, label_smoothing,
                         bn_train):
        """kp_conve_train_step: one BCEOptimizer step on the batch ``pairs`` [B][2]."""
        pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
        to = np.ascontiguousarray(tail_off, dtype=np.int32)
        tl = np.ascontiguousarray(tails, dtype=np.int32) if len(tails) else np.zeros(1, np.int32)
        nz = [None if v is None else np.ascontiguousarray(v, dtype=np.float32) for v in (in_noise, fm_noise, hid_noise)]
        check(lib().kp_conve_train_step(self.h, len(pr), _ptr(pr), _ptr(to), _ptr(tl), *[_ptr(v) for v in nz],
                                        float(lr), float(label_smoothing), int(bool(bn_train))), self.h)

    def conve_train_read(self):
        """kp_conve_train_read: the trained layers (the tables: :meth:`read_tables`)."""
        d = self.dim
        hid = 32 * 38 * (d // 20 - 2)
        out = {"conv_w": np.zeros((32, 9), np.float32), "conv_b": np.zeros(32, np.float32),
               "fc_w": np.zeros((d, hid), np.float32), "fc_b": np.zeros(d, np.float32)}
        for k in ("bn_w", "bn_b", "bn_m", "bn_v"):
            out[k] = np.zeros(33 + d, np.float32)
        check(lib().kp_conve_train_read(self.h, *[_ptr(out[k]) for k in ("conv_w", "conv_b", "fc_w", "fc_b", "bn_w",
                                                                        "bn_b", "bn_m", "bn_v")]), self.h)
        return out

    def read_tables(self, n_rel2: int):
        """kp_read_tables: (entity [n_ent][dim], relation [n_rel2][dim]) float32."""
        E = np.zeros((self.n_ent, self.dim), np.float32)
        R = np.zeros((n_rel2, self.dim), np.float32)
        check(lib().kp_read_tables(self.h, _ptr(E), _ptr(R)), self.h)
        return E, R

    def dp_relevance(self, items, epsilon, lambd, step_sign, rel_sign):
        """kp_dp_relevance: items int [n, 7] -> float32 [n]."""
        it = np.ascontiguousarray(np.asarray(items, dtype=np.int32).reshape(-1, 7))
        out = np.zeros(len(it), np.float32)
        check(lib().kp_dp_relevance(self.h, len(it), _ptr(it), float(epsilon), float(lambd), int(step_sign),
                                    int(rel_sign), _ptr(out)), self.h)
        return out

    def criage_relevance(self, items, ent_ids, tails_off, tails):
        """kp_criage_relevance: items int [n, 5] -> (float64 [n], status int32 [n])."""
        it = np.ascontiguousarray(np.asarray(items, dtype=np.int32).reshape(-1, 5))
        ents = np.ascontiguousarray(ent_ids, dtype=np.int32)
        off = np.ascontiguousarray(tails_off, dtype=np.int32)
        tl = np.ascontiguousarray(np.asarray(tails, dtype=np.int32).reshape(-1, 2)) if len(tails) \
            else np.zeros((1, 2), np.int32)
        out = np.zeros(len(it), np.float64)
        status = np.zeros(len(it), np.int32)
        check(lib().kp_criage_relevance(self.h, len(it), _ptr(it), len(ents), _ptr(ents), _ptr(off), _ptr(tl),
                                        _ptr(out), _ptr(status)), self.h)
        return out, status

    def hot_intervals(self) -> np.ndarray:
        """[start, end] seconds of each dominant-kernel launch of the last batch (kp_hot_intervals)."""
        n = C.c_int64()
        check(lib().kp_hot_intervals(self.h, 0, None, C.byref(n)), self.h)
        out = np.zeros((max(1, n.value), 2), np.float64)
        check(lib().kp_hot_intervals(self.h, n.value, _ptr(out), C.byref(n)), self.h)
        return out[:n.value]

    def last_timing(self):
        a, b, n, w = C.c_double(), C.c_double(), C.c_int64(), C.c_double()
        check(lib().kp_last_timing(self.h, C.byref(a), C.byref(b), C.byref(n), C.byref(w)), self.h)
        return {"device_s": a.value, "hot_s": b.value, "hot_launches": n.value, "hot_work": w.value}


class Graph:
    """Prefilter graph (kp_graph_*): undirected multigraph of the training triples."""

    def __init__(self, n_ent: int, triples):
        t = np.ascontiguousarray(np.asarray(triples, dtype=np.int32).reshape(-1, 3))
        h = C.c_void_p()
        self._lib = lib()
        self._check(self._lib.kp_graph_create(int(n_ent), len(t), _ptr(t), C.byref(h)))
        self._h = h
        self.n_ent = int(n_ent)

    def _check(self, rc):
        if rc != 0:
            raise KelpieHipError(f"libkelpie_hip error {rc}: {self._lib.kp_graph_last_error().decode()}")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.kp_graph_destroy(h)
            self._h = None

    def bfs(self, sources) -> np.ndarray:
        src = np.ascontiguousarray(sources, dtype=np.int32).reshape(-1)
        out = np.empty((len(src), self.n_ent), np.int32)
        self._check(self._lib.kp_graph_bfs(self._h, len(src), _ptr(src), _ptr(out)))
        return out

    def set_classes(self, cls_off, cls):
        off = np.ascontiguousarray(cls_off, dtype=np.int64)
        c = np.ascontiguousarray(cls, dtype=np.int32) if len(cls) else np.zeros(1, np.int32)
        assert len(off) == self.n_ent + 1
        self._check(self._lib.kp_graph_set_classes(self._h, _ptr(off), _ptr(c)))

    def dijkstra_pairs(self, src, dst) -> np.ndarray:
        s = np.ascontiguousarray(src, dtype=np.int32).reshape(-1)
        d = np.ascontiguousarray(dst, dtype=np.int32).reshape(-1)
        assert len(s) == len(d)
        out = np.empty(len(s), np.float64)
        self._check(self._lib.kp_graph_dijkstra_pairs(self._h, len(s), _ptr(s), _ptr(d), _ptr(out)))
        return out


class NativeView:
    """A kelpie view in the library's host scheduler (kp_view_create, csrc/kp_sched.cpp):
    the kelpie entity's training triples ``base`` [n][3] (original entity already replaced,
    in the Python view's order) and its validation / test triples ``extra`` (filters only)."""

    def __init__(self, kelpie: int, n_rel: int, original: int, base: np.ndarray, extra: np.ndarray):
        b = np.ascontiguousarray(base, dtype=np.int32).reshape(-1, 3)
        e = np.ascontiguousarray(extra, dtype=np.int32).reshape(-1, 3)
        h = C.c_void_p()
        self._lib = lib()
        check(self._lib.kp_view_create(int(kelpie), int(n_rel), int(original), _ptr(b), len(b), _ptr(e), len(e),
                                       C.byref(h)))
        self.h = h.value

    def __del__(self):
        h = getattr(self, "h", None)
        if h and C is not None:  # not at interpreter shutdown (module globals cleared)
            self._lib.kp_view_destroy(C.c_void_p(h))
            self.h = None


class SchedBatch:
    """One engine batch's natively assembled slots (kp_sched_*): ``add_calls`` edits the
    views and builds the rank filters of a run of calls, ``pack`` writes the rows and
    filters of any of its slots into the kp_posttrain_rank arrays."""

    def __init__(self):
        h = C.c_void_p()
        self._lib = lib()
        check(self._lib.kp_sched_batch_create(C.byref(h)))
        self.h = h.value
        self.views = []  # the NativeViews its slots point into (kept alive with the batch)
        # the engine's TransE fast path (kelpie_amd/engine.py _flush_fused / _pack_native):
        # slots created so far, one record per flush, the per-slot arrays built from them
        self.n_slots = 0
        self.recs = []
        self.packed = None
        self.dim = 0

    def __del__(self):
        h = getattr(self, "h", None)
        if h and C is not None:  # not at interpreter shutdown (module globals cleared)
            self._lib.kp_sched_batch_destroy(C.c_void_p(h))
            self.h = None

    def add_calls(self, views, rels, flags, cand_off, cands):
        """Per call (flags: bit 0 base needed, 1 base owned, 2 pt owned, 3 sufficient):
        returns (slot index [n][2], rows [n][2], filter lengths [n][2], fail (call, code,
        triple)); code 1 assertion, 2 KeyError, 3 ValueError; -1 entries: no slot."""
        n = len(views)
        v = np.array(views, dtype=np.uint64)
        r = np.ascontiguousarray(rels, dtype=np.int32)
        f = np.ascontiguousarray(flags, dtype=np.uint8)
        co = np.ascontiguousarray(cand_off, dtype=np.int32)
        ct = np.ascontiguousarray(cands, dtype=np.int32).reshape(-1, 3) if len(cands) else np.zeros((1, 3), np.int32)
        idx = np.empty((n, 2), np.int32)
        rows = np.empty((n, 2), np.int32)
        nf = np.empty((n, 2), np.int32)
        fail = np.empty(3, np.int32)
        check(self._lib.kp_sched_add_calls(C.c_void_p(self.h), n, _ptr(v), _ptr(r), _ptr(f), _ptr(co), _ptr(ct),
                                           _ptr(idx), _ptr(rows), _ptr(nf), _ptr(fail)))
        return idx, rows, nf, (int(fail[0]), int(fail[1]), int(fail[2]))

    def pack(self, idx, rows: np.ndarray, filt: np.ndarray):
        i = np.ascontiguousarray(idx, dtype=np.int32)
        assert rows.dtype == np.int32 and rows.flags.c_contiguous and filt.dtype == np.int32
        check(self._lib.kp_sched_pack(C.c_void_p(self.h), len(i), _ptr(i), _ptr(rows), rows.size, _ptr(filt),
                                      filt.size))


# Page-locked int32 arenas (kp_host_alloc), pooled for the life of the process: the
# deferred-draw arenas of kelpie_amd.rng come from here when a GPU is present, so a
# batch's draws reach the device by DMA straight from where the RNG workers wrote them.
# Page-locked memory is committed and locked, so the pool is small (KP_PINNED_ARENAS).
_PINNED = []       # the pool's arrays
_PINNED_IDLE = []  # per pool array: no lease of it is alive
_PINNED_MAX = int(os.environ.get("KP_PINNED_ARENAS", "6"))
_PINNED_OK = None


class ArenaLease(np.ndarray):
    """A pooled arena handed to one batch.  Every view taken of it is an ArenaLease whose
    ``base`` chain leads back to it (numpy does not collapse the chain through a
    subclass), so the lease -- and with it the arena -- stays busy while any of the
    batch's draw arrays is alive; when the last one is gone a weakref finalizer returns
    the arena to the pool.  No reference counting of the pool's own arrays."""


def _lease(i: int) -> ArenaLease:
    _PINNED_IDLE[i] = False
    lease = _PINNED[i].view(ArenaLease)
    weakref.finalize(lease, _PINNED_IDLE.__setitem__, i, True)
    return lease


def pinned_i32(n: int):
    """A lease on an idle pooled page-locked int32 array of at least ``n`` words, or None
    (pool full and busy, or no usable GPU: then the caller takes pageable memory)."""
    global _PINNED_OK
    for i, a in enumerate(_PINNED):
        if _PINNED_IDLE[i] and a.size >= n:
            return _lease(i)
    if _PINNED_OK is False or len(_PINNED) >= _PINNED_MAX:
        return None
    p = C.c_void_p()
    if lib().kp_host_alloc(4 * int(n), C.byref(p)) != 0 or not p.value:
        _PINNED_OK = False
        return None
    _PINNED_OK = True
    _PINNED.append(np.ctypeslib.as_array((C.c_int32 * int(n)).from_address(p.value)))
    _PINNED_IDLE.append(True)
    return _lease(len(_PINNED) - 1)


def arena_of(a: np.ndarray):
    """The lease ``a`` is (a view of), or None when it is not a pooled arena's."""
    x = a
    while isinstance(x, ArenaLease):
        b = x.base
        if any(b is p for p in _PINNED):
            return x
        x = b
    return None


def is_pinned(a: np.ndarray) -> bool:
    """``a`` is (a view of) a pooled page-locked arena."""
    return arena_of(a) is not None


def gather_i32(arrays, out: np.ndarray) -> np.ndarray:
    """``out[:total]`` = the int32 arrays back to back, copied by the library (kp_gather_i32:
    the interpreter lock is released for the copy)."""
    ptrs = np.array([a.__array_interface__["data"][0] for a in arrays], dtype=np.uint64)
    cnt = np.array([a.size for a in arrays], dtype=np.int64)
    assert out.dtype == np.int32 and out.flags.c_contiguous
    assert all(a.dtype.itemsize == 4 and (a.size == 0 or a.flags.c_contiguous) for a in arrays)
    check(lib().kp_gather_i32(len(arrays), _ptr(ptrs), _ptr(cnt), _ptr(out), out.size))
    return out[:int(cnt.sum())]
