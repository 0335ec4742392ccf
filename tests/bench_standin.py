"""bench.py on the CPU stand-in for the HIP context (TEST INFRASTRUCTURE).

Runs ``bench.main()`` with every frozen model's device context replaced by the
oracle-backed stand-in (tests/cpu_backend.py), so the launcher and the multi-rank
protocol of ``bench.py --gpus N`` (gloo on the CPU) are exercised without a GPU.
The product bench never imports this file; ``bench.launch_local_ranks`` re-runs
whatever script was started, so the ranks it spawns come back here.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def _install_standin():
    import kelpie_amd as ka
    from cpu_backend import OracleBackedContext
    for cls in (ka.models.TransE, ka.models.ComplEx, ka.models.ConvE):
        orig = cls.__init__

        def init(self, *a, _orig=orig, **k):
            _orig(self, *a, **k)
            self._ctx = OracleBackedContext(self)

        cls.__init__ = init


if __name__ == "__main__":
    import bench
    _install_standin()
    bench.main()
