"""Per-phase issue-cycle breakdown of kp_attn (diagnostic build, `make stamps`).

    KELPIE_HIP_LIB=kelpie_amd/libkelpie_hip_stamps.so python tools/attn_stamps.py [workload]

Runs two engine batches of a bench workload and prints, summed over waves, the
s_memtime cycles each wave spent issuing the S phase (+ next-tile DMA), the
softmax, the O phase and the tile end (DMA wait + barrier), per tile.
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
os.environ.setdefault("KELPIE_HIP_LIB", os.path.join(HERE, "kelpie_amd", "libkelpie_hip_stamps.so"))

import bench  # noqa: E402
from kelpie_amd import NecessaryPostTrainingEngine, _lib  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "complex-fb15k237-necessary"
wl = bench.WORKLOADS[name]
ds, model, _ = bench.build(wl, 0, 0)
eng = NecessaryPostTrainingEngine(model, ds, wl["hp"])
preds = bench.pick_preds(ds, 2 * wl["preds_per_step"], seed=1234)
bench.seed_all(42)
L = _lib.lib()
fn = L.kp_debug_attn_stamps_conve if wl["model"] == "ConvE" else L.kp_debug_attn_stamps
fn.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
k = wl["preds_per_step"]
for i in range(2):
    eng.set_cache()
    eng.compute_relevance_multi([(p, [[c] for c in bench.candidates_of(ds, p, wl["candidates"])])
                                 for p in preds[i * k:(i + 1) * k]])
    fn(buf, 1)
    tiles = max(1, buf[4])
    names = ["S+DMA issue", "softmax", "O phase", "tile end"]
    tot = sum(buf[j] for j in range(4))
    print(f"batch {i}: wave-tiles {tiles}", ", ".join(f"{n} {buf[j] / tiles:.0f} cyc ({100 * buf[j] / tot:.1f}%)"
                                                      for j, n in enumerate(names)), flush=True)
