"""bench.py's own rank launcher (`python bench.py --gpus N` without torchrun):
N fresh child processes, each with its RANK / LOCAL_RANK / WORLD_SIZE and a
127.0.0.1 rendezvous; the parent waits and returns the first failing exit
code.  CPU only: the children here are a probe script, not the GPU bench."""
import json
import subprocess
import sys
from pathlib import Path

import bench

PROBE = """
import json, os, sys
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
out = {k: os.environ.get(k) for k in keys}
out["argv"] = sys.argv[1:]
open(os.path.join(sys.argv[1], "rank%s.json" % os.environ["RANK"]), "w").write(json.dumps(out))
sys.exit(int(os.environ.get("PROBE_FAIL_RANK", "-1")) == int(os.environ["RANK"]) and 3 or 0)
"""


def _probe(tmp_path):
    p = tmp_path / "probe.py"
    p.write_text(PROBE)
    return p


def test_two_children_see_world_size_two(tmp_path):
    rc = bench.launch_ranks(2, [str(tmp_path), "--gpus", "2"], script=_probe(tmp_path), poll_s=0.05)
    assert rc == 0
    seen = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(2)]
    assert [s["RANK"] for s in seen] == ["0", "1"]
    assert [s["LOCAL_RANK"] for s in seen] == ["0", "1"]
    assert all(s["WORLD_SIZE"] == "2" and s["LOCAL_WORLD_SIZE"] == "2" for s in seen)
    assert all(s["MASTER_ADDR"] == "127.0.0.1" for s in seen)
    assert seen[0]["MASTER_PORT"] == seen[1]["MASTER_PORT"]
    assert all(s["argv"] == [str(tmp_path), "--gpus", "2"] for s in seen)


def test_failing_rank_fails_the_job(tmp_path, monkeypatch):
    monkeypatch.setenv("PROBE_FAIL_RANK", "1")
    rc = bench.launch_ranks(2, [str(tmp_path)], script=_probe(tmp_path), poll_s=0.05)
    assert rc == 3


def test_requested_gpus_parse():
    assert bench._requested_gpus(["--gpus", "4", "--steps", "3"]) == 4
    assert bench._requested_gpus(["--steps", "3"]) == 1


def test_bench_entry_spawns_ranks_before_torch(tmp_path):
    """`python bench.py --gpus 2` in a process without WORLD_SIZE re-runs
    bench.py as 2 ranks; with WORLD_SIZE set (the driver's torchrun) it does
    not.  Checked without a GPU: the children run with --help, which parses
    and exits before anything touches a device."""
    root = Path(bench.__file__).resolve().parent
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--help"], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    # each of the two children printed the usage once
    assert r.stdout.count("usage:") == 2, r.stdout
