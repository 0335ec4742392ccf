"""Run bench.py against another copy of the kelpie_amd package (A/B of host-side changes
on one box): ``python tools/ab_pkg.py <dir holding kelpie_amd/> [bench.py args...]``.
bench.py imports kelpie_amd inside main(), so the directory put first on sys.path after
importing bench decides which package runs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = os.path.abspath(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

sys.path.insert(0, pkg)
import kelpie_amd  # noqa: E402

assert os.path.dirname(os.path.dirname(os.path.abspath(kelpie_amd.__file__))) == pkg, kelpie_amd.__file__
print(f"[ab_pkg] kelpie_amd from {kelpie_amd.__file__}", file=sys.stderr)
bench.main()
