"""A/B: run bench.py (or another script) against another build of libmcmc355
(same box, same process layout).
    python scripts/ab_lib.py LIB.so [bench.py args...]
    python scripts/ab_lib.py LIB.so scripts/bench_configs.py [args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib_path = os.path.abspath(sys.argv[1])
rest = sys.argv[2:]
script = os.path.join(ROOT, "bench.py")
if rest and rest[0].endswith(".py"):
    script, rest = os.path.abspath(rest[0]), rest[1:]
sys.argv = [script] + rest
import __graft_entry__ as ge  # noqa: E402

ge._ensure_pkg()
from mlx_mcmc_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path
runpy.run_path(script, run_name="__main__")
