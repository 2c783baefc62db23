"""bench.py's multi-GPU launch contract on the CPU (gloo): `--gpus N` without
an external launcher starts N ranks itself (torch.distributed.run, one process
per GPU on the box), the line reports the ranks that actually ran and carries
the config-5 exchange, and a launcher/flag mismatch fails instead of silently
running one rank."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
BENCH = os.path.join(os.path.dirname(HERE), "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


import pytest


@pytest.mark.parametrize("world", [2, 4])
def test_self_launch_dry_run(world):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--dry-run", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["dry_run"] is True and line["value"] is None
    assert line["exchange"]["assembled_ok"] is True and line["exchange"]["documents"] == 8 * world
    # both exchange modes (--exchange-mode both, the default): the all-to-all by
    # owner and north_star's all-gather each assemble exactly the rank's documents
    modes = line["exchange"]["modes"]
    assert set(modes) == {"all_to_all", "all_gather"}
    for md, v in modes.items():
        assert v["mode"] == md and v["assembled_ok"] is True, (md, v)
    # the all-gather receives every rank's whole (padded) log: more bytes than the all-to-all
    assert modes["all_gather"]["recv_bytes_per_rank"] > modes["all_to_all"]["recv_bytes_per_rank"]


def test_rank_count_mismatch_fails():
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2 and "rank(s) were launched" in p.stderr
