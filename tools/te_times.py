"""Per-slot timeline of kp_te_posttrain (diagnostic build, `make stamps`).

    KELPIE_HIP_LIB=kelpie_amd/libkelpie_hip_stamps.so python tools/te_times.py [KELPIE_TE_NT]

Runs two engine batches of the TransE bench workload and prints, per slot, its
row count R, start / end offsets from the launch's first workgroup start and the
time per epoch (wall_clock64, 100 MHz), plus a summary by R bucket.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
os.environ.setdefault("KELPIE_HIP_LIB", os.path.join(HERE, "kelpie_amd", "libkelpie_hip_stamps.so"))

import bench  # noqa: E402
from kelpie_amd import NecessaryPostTrainingEngine, _lib  # noqa: E402

wl = bench.WORKLOADS["transe-fb15k237-necessary"]
ds, model, _ = bench.build(wl, 0, 0)
eng = NecessaryPostTrainingEngine(model, ds, wl["hp"])
k = wl["preds_per_step"]
preds = bench.pick_preds(ds, 2 * k, seed=1234)
bench.seed_all(42)
L = _lib.lib()
L.kp_debug_te_times.argtypes = [C.c_void_p, C.c_int]
ep = wl["hp"]["epochs"]
for i in range(2):
    eng.set_cache()
    eng.compute_relevance_multi([(p, [[c] for c in bench.candidates_of(ds, p, wl["candidates"])])
                                 for p in preds[i * k:(i + 1) * k]])
    n = eng.last_batch_stats["slots"]
    buf = np.zeros(8 * n, np.int64)
    L.kp_debug_te_times(buf.ctypes.data, n)
    t = buf.reshape(n, 8)
    t0 = t[:, 2].min()
    dur = (t[:, 3] - t[:, 2]) / 100.0  # us
    print(f"batch {i}: {n} slots, launch span {(t[:, 3].max() - t0) / 100:.0f} us, "
          f"hot {eng.last_batch_stats['hot_s'] * 1e6:.0f} us", flush=True)
    R = t[:, 1]
    for lo, hi in ((0, 40), (40, 100), (100, 200), (200, 400), (400, 10 ** 9)):
        sel = (R >= lo) & (R < hi)
        if sel.any():
            print(f"  R in [{lo},{hi}): {sel.sum():4d} slots, dur mean {dur[sel].mean():7.0f} us max {dur[sel].max():7.0f}"
                  f", per epoch {dur[sel].mean() / ep:6.2f} us, start max {(t[sel, 2].max() - t0) / 100:6.0f} us")
            print(f"     cycles per epoch: wave 0 fetch+wait {np.mean(t[sel, 4]) / ep:7.0f}, wave 0 compute "
                  f"{np.mean(t[sel, 5]) / ep:7.0f}, slowest wave's item loop {np.mean(t[sel, 7]) / ep:7.0f}, "
                  f"whole step {np.mean(t[sel, 6]) / ep:7.0f}")
