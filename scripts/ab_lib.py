"""A/B: run bench.py against another build of libmcmc355 (same box, same
process layout).  python scripts/ab_lib.py LIB.so [bench.py args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib_path = os.path.abspath(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
from mlx_mcmc_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path
import bench  # noqa: E402

bench.main()
