"""Multi-rank path on CPU (gloo, world_size 2): sharding and the one result gather."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from kelpie_amd import distributed as kd
    r, w, _ = kd.init_from_env(backend="gloo")
    items = list(range(11))
    mine = kd.shard(items, r, w)
    recs = np.array([[float(i), i * 2.0, 0, 0, 0] for i in mine]).reshape(-1, kd.RECORD)
    allr = kd.gather_records(recs, device="cpu")
    mx = kd.max_over_ranks(float(r + 1), device="cpu")
    kd.barrier()
    q.put((r, mine, allr[:, 0].tolist(), mx))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_shard_and_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    assert out[0][1] + out[1][1] == list(range(11))  # disjoint, complete shards
    for r, mine, gathered, mx in out:
        assert gathered == [float(i) for i in range(11)]  # rank order, padded counts trimmed
        assert mx == 2.0


def test_shard_single_rank():
    from kelpie_amd import distributed as kd
    assert kd.shard([1, 2, 3], 0, 1) == [1, 2, 3]
    recs = np.zeros((2, kd.RECORD))
    assert kd.gather_records(recs).shape == (2, kd.RECORD)


# ---------------------------------------------------------------------------
# engine-level sharding: world-2 results == world-1 results, bit for bit
# ---------------------------------------------------------------------------
ENGINE_CASES = ["complex_tiny", "transe_tiny", "conve60_tiny"]


def _engine_run(name, sharding, backend="cpu"):
    """necessary batches (every golden block), sufficient with select_entities_to_convert,
    the two-context batch pipeline and the builder pipeline, on the CPU stand-in engine."""
    import sys
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from engine_cases import build_product
    from golden_io import seed_all
    import kelpie_amd as ka
    from kelpie_amd.pipeline import build_pipeline, explain_preds
    rec, ds, model = build_product(name, backend)
    out = {}
    seed_all(rec["seed"])
    eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
    eng.sharding = sharding
    out["necessary"] = []
    for block in rec["necessary"]:
        eng.set_cache()
        rules = [[tuple(t) for t in c["rule"]] for c in block["calls"]]
        out["necessary"].append(eng.compute_relevance_batch(tuple(block["pred"]), rules))
    items = [(tuple(b["pred"]), [[tuple(t) for t in c["rule"]] for c in b["calls"][:4]]) for b in rec["necessary"]]
    out["pipeline"] = eng.compute_relevance_pipeline([[it] for it in items], depth=2)
    seed_all(rec["seed"])
    seng = ka.SufficientPostTrainingEngine(model, ds, rec["hp"])
    seng.sharding = sharding
    blk = rec["sufficient"][0]
    out["entities"] = seng.select_entities_to_convert(tuple(blk["pred"]), 3, 200)
    out["sufficient"] = seng.compute_relevance_batch(tuple(blk["pred"]),
                                                     [[tuple(t) for t in c["rule"]] for c in blk["calls"]])
    b = rec.get("builder")
    if b:
        seed_all(rec["seed"])
        pipe = build_pipeline(model, ds, rec["hp"], "necessary", xsi=b["xsi"], window=4)
        pipe.engine.sharding = sharding
        with tempfile.TemporaryDirectory() as tmp:
            preds = [list(ds.labels_triple(tuple(b["pred"])))]
            res = explain_preds(pipe, ds, preds, prefilter_k=len(b["candidates"]))
        out["builder"] = [(r["rule_to_relevance"], r["#relevances"]) for r in res]
    out["gathers"] = sharding.gathers if sharding is not None else 0
    if sharding is not None:
        # one collective per gather: every rank's block size is known from the claims
        assert sharding.collectives == sharding.gathers, (sharding.collectives, sharding.gathers)
    if sharding is not None and sharding.world > 1:
        # the last batch: this rank scheduled in full only the slots it claimed
        eng.set_cache()
        with eng.rng.deferred():
            slots, _, _ = eng._schedule_all(items[:1], None)
        own = [s for s in slots if s.own]
        assert 0 < len(own) < len(slots) and all(s.filt is None and (s.rng is None or s.rng.size == 0) for s in slots if not s.own)
    return out


def _engine_worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from kelpie_amd import distributed as kd
    kd.init_from_env(backend="gloo")
    try:
        res = {name: _engine_run(name, kd.SlotSharding(device="cpu")) for name in ENGINE_CASES}
        q.put((rank, res))
    except BaseException as e:  # report instead of hanging the other rank's gather
        q.put((rank, repr(e)))
        raise
    finally:
        import torch.distributed as dist
        dist.destroy_process_group()


def test_engine_sharding_world2_equals_world1():
    """Every rank schedules every batch (the one global random stream stays in lockstep)
    and post-trains its share of the slots; the gathered relevances, conversion entities
    and builder explanations equal the single-process run bit for bit (CPU stand-in for
    the HIP context)."""
    single = {name: _engine_run(name, None) for name in ENGINE_CASES}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out:
        assert not isinstance(res, str), res
        for name in ENGINE_CASES:
            got, exp = dict(res[name]), dict(single[name])
            assert got.pop("gathers") > 0
            exp.pop("gathers")
            assert got == exp, (rank, name)


def _engine_worker_gpu(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from kelpie_amd import distributed as kd
    kd.init_from_env(backend="gloo")  # two ranks share the box's one GPU
    try:
        res = {name: _engine_run(name, kd.SlotSharding(device="cpu"), backend="gpu") for name in ENGINE_CASES}
        q.put((rank, res))
    except BaseException as e:
        q.put((rank, repr(e)))
        raise
    finally:
        import torch.distributed as dist
        dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_sharding_world2_gpu():
    """The same on the MI355X: two ranks (one GPU, gloo) each post-train their share of
    every batch through the HIP library; results equal the single-process run.  The
    goldens here are well conditioned, so ranks and relevances match exactly."""
    single = {name: _engine_run(name, None, backend="gpu") for name in ENGINE_CASES}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker_gpu, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out:
        assert not isinstance(res, str), res
        for name in ENGINE_CASES:
            got, exp = dict(res[name]), dict(single[name])
            got.pop("gathers"), exp.pop("gathers")
            assert got == exp, (rank, name)


def _nccl_world1_worker(port, q, backend="nccl"):
    """One rank, one RCCL (`nccl` backend) group on the GPU, the gathers forced through
    the collective: every slot record goes out as a device tensor through
    all_gather_into_tensor over RCCL and comes back (backend "gloo": the same on the
    CPU stand-in)."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0", "WORLD_SIZE": "1",
                       "LOCAL_RANK": "0"})
    import torch
    import torch.distributed as dist
    from kelpie_amd import distributed as kd
    kd.init_from_env(backend=backend, force=True)
    try:
        dev = torch.device("cuda", 0) if backend == "nccl" else "cpu"
        sh = kd.SlotSharding(device=dev, force_collective=True)
        res = {name: _engine_run(name, sh, backend="gpu" if backend == "nccl" else "cpu") for name in ENGINE_CASES}
        q.put((dist.get_backend(), sh.collectives, res))
    except BaseException as e:
        q.put(("error", 0, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_gather_over_rccl_world1():
    """The RCCL branch of the slot gather on the MI355X: a world-1 `nccl` process group
    with the gathers forced through `all_gather_into_tensor` on device tensors
    (SlotSharding.force_collective); results equal the run without a process group."""
    single = {name: _engine_run(name, None, backend="gpu") for name in ENGINE_CASES}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), q))
    p.start()
    backend, collectives, res = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0 and backend == "nccl", (backend, res)
    assert collectives > 0
    for name in ENGINE_CASES:
        got, exp = dict(res[name]), dict(single[name])
        assert got.pop("gathers") > 0
        exp.pop("gathers")
        assert got == exp, name


def test_engine_gather_forced_collective_world1_cpu():
    """The forced-collective path of the RCCL test on the CPU stand-in: a world-1 gloo
    group, every gather through the process group; results equal the plain run."""
    single = {name: _engine_run(name, None) for name in ENGINE_CASES}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), q, "gloo"))
    p.start()
    backend, collectives, res = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0 and backend == "gloo", (backend, res)
    assert collectives > 0
    for name in ENGINE_CASES:
        got, exp = dict(res[name]), dict(single[name])
        assert got.pop("gathers") > 0
        exp.pop("gathers")
        assert got == exp, name


def _failing_worker(rank, world, port, q):
    """Rank 1's device work fails in the second batch: both ranks must raise (rank 1 its
    own error, rank 0 the gathered failure) instead of rank 0 waiting in the gather."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from engine_cases import build_product
    from golden_io import seed_all
    import kelpie_amd as ka
    from kelpie_amd import distributed as kd
    from kelpie_amd._lib import KelpieHipError
    kd.init_from_env(backend="gloo")
    try:
        rec, ds, model = build_product("complex_tiny", "cpu")
        seed_all(rec["seed"])
        eng = ka.NecessaryPostTrainingEngine(model, ds, rec["hp"])
        eng.sharding = kd.SlotSharding(device="cpu")
        block = rec["necessary"][0]
        rules = [[tuple(t) for t in c["rule"]] for c in block["calls"]]
        eng.compute_relevance_batch(tuple(block["pred"]), rules)
        if rank == 1:
            def boom(*a, **k):
                raise KelpieHipError("injected device failure")
            model.ctx.posttrain_rank = boom
        eng.set_cache()
        try:
            eng.compute_relevance_batch(tuple(block["pred"]), rules)
            q.put((rank, "no error"))
        except Exception as e:  # noqa: BLE001
            q.put((rank, type(e).__name__ + ": " + str(e)))
    finally:
        import torch.distributed as dist
        dist.barrier()  # both ranks have read the gather before the connection closes
        dist.destroy_process_group()


def test_engine_sharding_failure_raises_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert out[1].startswith("KelpieHipError: injected device failure"), out
    assert out[0].startswith("RuntimeError: slot sharding: the device work of rank(s) [1] failed"), out
