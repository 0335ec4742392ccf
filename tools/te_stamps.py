"""Phase breakdown of kp_te_posttrain (diagnostic build, `make stamps`).

    KELPIE_HIP_LIB=kelpie_amd/libkelpie_hip_stamps.so python tools/te_stamps.py
"""
import ctypes as C
import os
import sys

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
L.kp_debug_te_stamps.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
for i in range(2):
    eng.set_cache()
    eng.compute_relevance_multi([(p, [[c] for c in bench.candidates_of(ds, p, wl["candidates"])])
                                 for p in preds[i * k:(i + 1) * k]])
    st = eng.last_batch_stats
    L.kp_debug_te_stamps(buf, 1)
    wgs, rows = max(1, buf[4]), buf[5]
    rounds = max(1, buf[3])
    print(f"batch {i}: slots {wgs} mean R {rows / wgs:.1f} max R {buf[7]} kernel {st['hot_s'] * 1e3:.2f} ms; "
          f"staging {buf[0] / wgs / wl['hp']['epochs']:.0f} ticks/slot-epoch, pair loop {buf[1] / rounds:.0f} "
          f"ticks/round of which load wait {buf[2] / rounds:.0f}; rounds {rounds}", flush=True)
