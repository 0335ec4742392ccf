"""Host layer of the product engine vs the reference golden vectors, on CPU.

The HIP context is replaced by the oracle-backed stand-in (tests/cpu_backend.py),
so these tests pin everything the product does on the host -- kelpie views and
filters, the RNG protocol (draw order, skipped draws), slot assembly, relevance
formulas, batching and the builder's speculative windows with RNG rewind.
"""
import pytest

from engine_cases import check_builder, check_necessary, check_pipeline, check_pipeline_explain, check_sufficient
from golden_io import CASES

FAST = ["transe_tiny", "complex_tiny", "complex_adam_tiny", "conve60_tiny", "conve60_drop_tiny", "complex_n3_tiny",
        "complex_n2_tiny", "transe_l1_tiny"]


@pytest.mark.parametrize("name", FAST)
@pytest.mark.parametrize("batched", [False, True])
def test_necessary_host_protocol(name, batched):
    check_necessary(name, "cpu", batched)


@pytest.mark.parametrize("name", FAST)
def test_sufficient_host_protocol(name):
    check_sufficient(name, "cpu", batched=True)


@pytest.mark.parametrize("name", ["transe_tiny", "complex_tiny", "conve60_tiny", "conve60_drop_tiny"])
@pytest.mark.parametrize("window", [1, 4, 32, "auto"])
def test_builder_speculative_windows(name, window):
    check_builder(name, "cpu", window=window)


@pytest.mark.parametrize("name", ["complex_tiny", "transe_tiny", "conve60_tiny"])
@pytest.mark.parametrize("window", [4, "auto"])
def test_builder_pipelined_windows(name, window):
    """The look-ahead window (scheduled before the current one is replayed and held; on a
    stop cancelled and rewound) gives the sequential reference's explanations too, and a
    cancelled look-ahead makes no library call: one call per evaluated engine batch."""
    for calls, st in check_builder(name, "cpu", window=window, pipelined=True):
        assert calls == st["batches"], (calls, st)


@pytest.mark.parametrize("name", ["complex_tiny", "transe_tiny"])
def test_pipeline_host_protocol(name):
    check_pipeline(name, "cpu")


@pytest.mark.parametrize("name", ["complex_tiny", "transe_tiny"])
def test_pipeline_two_contexts(name):
    """Two batches in flight on two contexts (batch b on context b mod 2) return the
    reference's sequential results, in order."""
    check_pipeline(name, "cpu", two_contexts=True)


@pytest.mark.parametrize("name", ["complex_tiny", "transe_tiny"])
@pytest.mark.parametrize("lookahead,workers,detach", [("1", "1", "1"), ("0", "0", "1"), ("1", "0", "0")])
def test_pipeline_switches(name, lookahead, workers, detach, monkeypatch):
    """The pipeline's A/B switches (KELPIE_PIPELINE_LOOKAHEAD: batches scheduled ahead of
    the contexts; KELPIE_PIPELINE_WORKERS=0: a thread per batch; KELPIE_PIPELINE_DETACH=0:
    the scheduling thread waits for each batch's draws) keep the reference's sequential
    results, in order, with two batches in flight."""
    monkeypatch.setenv("KELPIE_PIPELINE_LOOKAHEAD", lookahead)
    monkeypatch.setenv("KELPIE_PIPELINE_WORKERS", workers)
    monkeypatch.setenv("KELPIE_PIPELINE_DETACH", detach)
    check_pipeline(name, "cpu", two_contexts=True)


@pytest.mark.parametrize("name", ["complex_tiny", "transe_tiny"])
def test_explain_pipeline_and_output_json(name, tmp_path):
    check_pipeline_explain(name, "cpu", str(tmp_path))
