"""bench.py --gpus N without a launcher starts N rank processes itself (bench.launch_ranks), the
way torch.distributed.run would: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT per
child, the first failing rank's status returned and the other ranks stopped; N above the visible
devices is refused. CPU only: the rank script here is a stand-in that records its environment."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

RANK_SCRIPT = """
import json, os, sys, time
out = sys.argv[1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]},
          open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w"))
if len(sys.argv) > 2 and os.environ["RANK"] == sys.argv[2]:
    sys.exit(3)              # this rank fails
if len(sys.argv) > 2:
    time.sleep(60)           # the others would wait forever in a collective
"""


def _script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launch_ranks_environment(tmp_path):
    rc = bench.launch_ranks(3, [str(tmp_path)], device_count=4, script=_script(tmp_path))
    assert rc == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "3", "3")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["argv"] == [str(tmp_path)]


def test_launch_ranks_failure_stops_the_others(tmp_path):
    t0 = time.time()
    rc = bench.launch_ranks(3, [str(tmp_path), "1"], device_count=3, script=_script(tmp_path))
    assert rc == 3
    assert time.time() - t0 < 30  # ranks 0 and 2 were terminated, not waited for


def test_launch_ranks_refuses_more_than_visible(tmp_path):
    with pytest.raises(SystemExit, match="only 2 GPU"):
        bench.launch_ranks(4, [], device_count=2, script=_script(tmp_path))


def test_bench_gpus_flag_is_honoured_without_gpus():
    """No GPU in this container: `bench.py --gpus 2` must refuse (not silently run one rank)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "--gpus 2 but only" in r.stderr


def test_bench_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
