"""bench.py's own rank launch (VERDICT r5 "Next round" 1): the
driver's command shape `python bench.py --gpus N ...` runs N rank processes,
one per GPU, and the parent never touches torch or the device.

On CPU the rank command is replaced by a probe that joins a real gloo
rendezvous from the environment bench.py gives it (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_*); the GPU side (the real bench under gloo on the one-GPU
box) is tests/test_gpu_multirank.py::test_bench_spawns_ranks_itself.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one spawned rank: rendezvous over gloo, sum the ranks, rank 0 prints a line
PROBE = r"""
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print(json.dumps({"world": dist.get_world_size(), "sum": float(t.item()),
                      "local": os.environ["LOCAL_RANK"], "addr": os.environ["MASTER_ADDR"],
                      "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
"""

# the parent: bench.main() with the probe as the rank command; torch must
# stay unimported in this process, before and after the ranks ran
PARENT = r"""
import json, sys
sys.path.insert(0, {root!r})
import bench
bench.rank_command = lambda argv: [sys.executable, "-c", {probe!r}] + list(argv)
sys.argv = ["bench.py"] + {argv!r}
code = 0
try:
    bench.main()
except SystemExit as e:
    code = e.code
print(json.dumps({{"code": code, "torch_imported": "torch" in sys.modules}}), flush=True)
"""


def _parent(argv, probe=PROBE, env=None):
    src = PARENT.format(root=ROOT, probe=probe, argv=argv)
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=240,
                       env=e, cwd=ROOT)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


def test_gpus_n_spawns_n_ranks_without_touching_torch():
    r, lines = _parent(["--gpus", "3", "--steps", "4", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 2, r.stdout        # rank 0's line, then the parent's report
    rank0, parent = lines
    assert rank0["world"] == 3 and rank0["sum"] == 6.0
    assert rank0["local"] == "0" and rank0["addr"] == "127.0.0.1"
    assert rank0["argv"] == ["--gpus", "3", "--steps", "4", "--no-cpu-baseline"]
    assert parent == {"code": 0, "torch_imported": False}


def test_failed_rank_stops_the_others_and_fails_the_launch():
    # rank 1 fails at once; rank 0 would wait in the rendezvous forever
    probe = ("import os, sys, time\n"
             "if os.environ['RANK'] == '1': sys.exit(5)\n"
             "time.sleep(600)\n")
    r, lines = _parent(["--gpus", "2"], probe=probe)
    assert lines and lines[-1] == {"code": 5, "torch_imported": False}, (r.stdout, r.stderr)
    assert "rank 1 exited with status 5" in r.stderr


def test_world_size_mismatch_exits_non_zero():
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "2"], capture_output=True, text=True, timeout=120, env=env,
                       cwd=ROOT)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_matching_world_size_runs_in_process():
    """Under a launcher (WORLD_SIZE == --gpus) bench.py spawns nothing."""
    import bench

    class A:
        gpus = 2

    old = os.environ.get("WORLD_SIZE")
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.resolve_world(A()) is None
        A.gpus = 0
        assert bench.resolve_world(A()) == 2
    finally:
        if old is None:
            os.environ.pop("WORLD_SIZE")
        else:
            os.environ["WORLD_SIZE"] = old
